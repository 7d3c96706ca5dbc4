// ofdis_tvrb.hip -- the latency mode of the variational refinement (option sor_mode = 1): a level's whole inner
// loop -- compute_smoothness, the system (compute_data, sub_laplacian, the SOR matrix), the red-black SOR -- for
// every inner iteration, then the flow update uu = wx + du, in ONE launch: one workgroup per frame, everything a
// phase shares in LDS, every pixel's SOR coefficients in its owner thread's registers.
//
// Reference: refine_variational.cpp:185-231 (RefLevelOF / RefLevelDE: the inner loop and the final flow),
// FDF1.0.1/opticalflow_aux.c:138-187 (compute_smoothness), :194-223 (sub_laplacian), :408-747 (compute_data /
// compute_data_DE), FDF1.0.1/solver.c:83-433 and :439-471 (the per-pixel SOR update, here in red-black order as
// SURVEY §7 4(ii) proposes).  The same device functions as the two-launch path (ofdis_tv_dev.inc: smooth_compute,
// sys_compute, rb_update), so every system is the reference's bits; the SOR order is not.
//
// Why: a drop-in CLI call (one pair) or a config-D shard (32 pairs per GPU) cannot fill the
// chip.  There the exact-order SOR pays ~1,900 dependent wavefront steps per 1080p pair and the two-launch inner
// iteration 36 small launches.  Red-black order runs 2 * solverit fully parallel half-sweeps per inner iteration,
// and with the system in the same launch an inner iteration costs 1 + 2 * solverit workgroup barriers and no
// launch.  It is a different iteration from the reference's lexicographic SOR: bit-exact against the oracle's
// red-black restatement (ofo_sor_rb_of / _de) and EPE-gated against the exact path (tests/test_gpu_redblack.py).
//
// Layout (TvArgs::lat, written by k_tv_prepd): pixel p = y w + x of colour c = (x + y) & 1 is entry e = p >> 1 of
// colour c, stored at c E + e (E = ceil(w h / 2): w even has w / 2 pixels of each colour per row, w odd has colour
// = p & 1).  Every 4-neighbour of a colour-c pixel is the colour-(1 - c) entry (p -+ 1) >> 1 or (p -+ w) >> 1, so a
// wave's consecutive entries have consecutive neighbour entries: every LDS access of a phase is a contiguous run
// (conflict-free) and the derivative planes are read coalesced.  Thread t owns entries t + T k (k < CPT) of both
// colours for the whole launch.  LDS: (du, dv), (wx, wy) and s of every pixel, 20 B per pixel for optical flow
// (8192 pixels fill the 160 KB), 12 B for depth.  A missing neighbour reads the pixel's own entry: the clamped
// neighbourhood of compute_smoothness, and a value the system and the update select away.
#include "ofdis_internal.h"
#include "ofdis_math.h"

#pragma clang fp contract(off)

namespace ofdis {
namespace {

#include "ofdis_tv_dev.inc"

constexpr int kLvT = 1024, kLvCpt = 4;
constexpr int kLvPix = 2 * kLvT * kLvCpt;  // 8192 pixels per level

template <int NOP>
struct LvV {
  using T = float;
};
template <>
struct LvV<2> {
  using T = float2;
};
__device__ __forceinline__ float lv_x(float v) { return v; }
__device__ __forceinline__ float lv_x(float2 v) { return v.x; }
__device__ __forceinline__ float lv_y(float) { return 0.0f; }
__device__ __forceinline__ float lv_y(float2 v) { return v.y; }

__host__ __device__ __forceinline__ size_t lv_lds(int nop, int w, int h) {
  return (size_t)2 * lat_entries(w, h) * (nop == 2 ? 20 : 12);
}

// Pixel of entry e of colour c: p = 2 e + (the colour-c member of the pair (2 e, 2 e + 1)); -1 when outside.
__device__ __forceinline__ int lv_pixel(int e, int c, int w, int wh, int E) {
  if (e >= E) return -1;
  const int y0 = (2 * e) / w;
  const int p = 2 * e + ((w & 1) ? c : ((y0 ^ c) & 1));
  return p < wh ? p : -1;
}

// The owned pixel's packed coordinate, opaque to the optimiser: everything derived from it (neighbour indices,
// plane offsets) is recomputed in each phase (a few VALU) instead of being hoisted out of the inner-iteration loop
// and held live in registers for all 2 CPT pixels at once (which spilled under the 128-VGPR budget of 1024 threads).
__device__ __forceinline__ int lv_fresh(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// LDS indices of the centre and its left, right, upper, lower neighbours (a missing one: the centre)
struct LvNb {
  int i[5];
};
__device__ __forceinline__ LvNb lv_nb(int x, int y, int c, int w, int h, int E) {
  const int p = y * w + x, ob = (1 - c) * E, own = c * E + (p >> 1);
  LvNb n;
  n.i[0] = own;
  n.i[1] = x > 0 ? ob + ((p - 1) >> 1) : own;
  n.i[2] = x < w - 1 ? ob + ((p + 1) >> 1) : own;
  n.i[3] = y > 0 ? ob + ((p - w) >> 1) : own;
  n.i[4] = y < h - 1 ? ob + ((p + w) >> 1) : own;
  return n;
}

// The same where a missing neighbour may be any entry (the system's and the update's uses of it are selected away):
// (p -+ 1) >> 1 and (p -+ w) >> 1 need no border test, right = left + 1 and down = up + w whatever the row, and only
// the two indices that can leave the arrays are clamped -- a colour-1 pixel's upper neighbour in row 0 (below entry
// 0), a colour-0 pixel's lower one in the last row (past 2 E: the s array ends there).  c is a compile-time colour.
__device__ __forceinline__ LvNb lv_nb_any(int x, int y, int c, int w, int E) {
  const int p = y * w + x, ob = (1 - c) * E;
  LvNb n;
  n.i[0] = c * E + (p >> 1);
  n.i[1] = ob + ((p - 1) >> 1);
  n.i[2] = n.i[1] + 1;
  const int u = ob + ((p - w) >> 1);
  n.i[3] = c ? max(u, 0) : u;
  n.i[4] = c ? u + w : min(u + w, 2 * E - 1);
  return n;
}

// rb_update's optical-flow update on (u, v) pairs: v_pk_mul_f32 / v_pk_add_f32 round each half like the scalar
// instruction and the operations are rb_update's, in its order (sor_rhs's operand selects per component), so the
// same bits in about half the VALU issue.
__device__ __forceinline__ f2v rb_update_of_pk(const RbPix &d, bool hasl, bool hasr, bool border, bool notop,
                                               float omega, f2v l, f2v r, f2v t, f2v b, f2v o) {
  const f2v R = hasr ? r : f2v{0.0f, 0.0f};
  const f2v X = f2v{d.hr, d.hr} * R, Y = f2v{d.vt, d.vt} * t, Z = f2v{d.vb, d.vb} * b;
  const f2v Bv = f2v{d.b1, d.b2};
  const f2v lft = X + (border ? Bv : Y);
  const f2v rgt = (border ? f2v{-0.0f, -0.0f} : Bv) + (border ? (notop ? Z : Y) : Z);
  const f2v s = lft + rgt;
  const f2v B = hasl ? f2v{d.hl, d.hl} * l + s : s;
  const f2v m = f2v{d.i11, d.i12} * f2v{B.x, B.x} + f2v{d.i12, d.i22} * f2v{B.y, B.y};
  return o + f2v{omega, omega} * (m - o);
}
__device__ __forceinline__ f2v lv_f2(float2 v) { return f2v{v.x, v.y}; }

// The eight derivative values of one owned pixel (per channel), read from the colour-split planes
template <int NOC>
struct LvDeriv {
  float Ix[NOC], Iy[NOC], Iz[NOC], Ixx[NOC], Ixy[NOC], Iyy[NOC], Ixz[NOC], Iyz[NOC];
};
template <int NOC>
__device__ __forceinline__ void lv_load_deriv(const TvArgs &a, int f, unsigned idx, LvDeriv<NOC> &D) {
#pragma unroll
  for (int ch = 0; ch < NOC; ++ch) {  // wave-uniform plane base + 32-bit offset (ldu)
    const long pb = ((long)f * NOC + ch) * a.sp;
    D.Ix[ch] = ldu(a.Ix + pb, idx); D.Iy[ch] = ldu(a.Iy + pb, idx); D.Iz[ch] = ldu(a.Iz + pb, idx);
    D.Ixx[ch] = ldu(a.Ixx + pb, idx); D.Ixy[ch] = ldu(a.Ixy + pb, idx); D.Iyy[ch] = ldu(a.Iyy + pb, idx);
    D.Ixz[ch] = ldu(a.Ixz + pb, idx); D.Iyz[ch] = ldu(a.Iyz + pb, idx);
  }
}

template <int NOP, int NOC, int CPT>
__global__ __launch_bounds__(kLvT) void k_tv_level_rb(TvArgs a, int n_inner) {
  using V = typename LvV<NOP>::T;
  constexpr int MODE = NOP == 2 ? 0 : 2;
  // CPT 4 (2,049..8,192 pixels): the four diffusivities of each update (hl, hr, vt, vb) are re-derived from s in LDS
  // (still the iteration's s during the half-sweeps) instead of being held for all eight pixels -- the registers the
  // 1024-thread budget lacks; the same sums as sys_finish's
  constexpr bool SLDS = CPT >= 4 || (NOC == 3 && CPT >= 2);
  constexpr bool PF = NOC == 1;  // colour images: 24 derivative values per pixel, no register room for a second buffer
  extern __shared__ float4 lv_raw[];
  const int w = a.w, h = a.h, wh = w * h, E = lat_entries(w, h), T = blockDim.x, f = blockIdx.x;
  V *UV = reinterpret_cast<V *>(lv_raw);               // [2 E] (du, dv)
  V *WXY = UV + 2 * E;                                 // [2 E] (wx, wy)
  float *S = reinterpret_cast<float *>(WXY + 2 * E);   // [2 E] s
  const long fo = (long)f * a.sp;

  int xy[2][CPT];  // x | y << 16 of the owned pixels, -1: none
  RbPix d[2][CPT];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int e = threadIdx.x + T * k;
      const int p = lv_pixel(e, c, w, wh, E);
      xy[c][k] = -1;
      if (p < 0) continue;
      const int y = p / w, x = p - y * w;
      xy[c][k] = x | (y << 16);
      const int idx = c * E + e;
      if constexpr (NOP == 2) {
        WXY[idx] = make_float2(a.wxs[fo + idx], a.wys[fo + idx]);
        UV[idx] = make_float2(0.0f, 0.0f);
      } else {
        WXY[idx] = a.wxs[fo + idx];
        UV[idx] = 0.0f;
      }
    }
  __syncthreads();

  // the derivative planes of an owned pixel are read one pixel ahead of its system (two buffers, compile-time
  // indexed; the first pixel's during the smoothness phase): the L2 round trip overlaps the previous system
  // instead of opening each one.  Pixel j = c CPT + k is entry c E + threadIdx.x + T k (a missing one reads entry 0).
  auto deriv_idx = [&](int j) -> unsigned {
    const int c = j / CPT, k = j % CPT, e = threadIdx.x + T * k;
    return (unsigned)lv_fresh(xy[c][k] < 0 ? 0 : c * E + e);
  };
  LvDeriv<NOC> dbuf[2];
#pragma unroll 1
  for (int it = 0; it < n_inner; ++it) {
    const bool first = it == 0;
    if (PF) lv_load_deriv<NOC>(a, f, deriv_idx(0), dbuf[0]);
    // ---- compute_smoothness (opticalflow_aux.c:138-160) on uu = wx + du over the clamped neighbourhood
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        if (xy[c][k] < 0) continue;
        const int q = lv_fresh(xy[c][k]), x = q & 0xffff, y = q >> 16;
        const LvNb nb = lv_nb(x, y, c, w, h, E);
        float wx5[5], du5[5], wy5[5], dv5[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const V wv = WXY[nb.i[i]], uv = UV[nb.i[i]];
          wx5[i] = lv_x(wv);
          du5[i] = lv_x(uv);
          wy5[i] = lv_y(wv);
          dv5[i] = lv_y(uv);
        }
        S[nb.i[0]] = smooth_compute<NOP>(a, first, wx5, du5, wy5, dv5);
        __builtin_amdgcn_sched_barrier(0);  // one pixel's temporaries at a time (register budget of 1024 threads)
      }
    __syncthreads();
    // ---- the system of every owned pixel into registers (tv_system_px's gather, sys_compute).  No barrier before
    // the first half-sweep: the system reads only its own (du, dv), which only its own thread writes.
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        const int j = c * CPT + k;
        // the next pixel's derivatives are requested whether or not this thread owns pixel j
        if (PF && j + 1 < 2 * CPT) lv_load_deriv<NOC>(a, f, deriv_idx(j + 1), dbuf[(j + 1) & 1]);
        if (xy[c][k] < 0) continue;
        const int q = lv_fresh(xy[c][k]), x = q & 0xffff, y = q >> 16;
        const LvNb nb = lv_nb_any(x, y, c, w, E);
        const int idx = nb.i[0];
        if (!PF) lv_load_deriv<NOC>(a, f, deriv_idx(j), dbuf[0]);
        const LvDeriv<NOC> &D = dbuf[PF ? j & 1 : 0];
        float S5[5], X5[5], Y5[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const V wv = WXY[nb.i[i]];
          S5[i] = S[nb.i[i]];
          X5[i] = lv_x(wv);
          Y5[i] = lv_y(wv);
        }
        const V uv = UV[idx];
        const float m = warp_mask(x, y, X5[0], Y5[0], w, h);
        float4 c0, c1;
        sys_compute<NOP, NOC>(a, x, y, S5, X5, Y5, m, lv_x(uv), lv_y(uv), D.Ix, D.Iy, D.Iz, D.Ixx, D.Ixy, D.Iyy,
                              D.Ixz, D.Iyz, c0, c1);
        RbPix &r = d[c][k];
        if (NOP == 2) {
          r.i11 = c0.x; r.i12 = c0.y; r.i22 = c0.w; r.b1 = c1.x; r.b2 = c1.y;
          if (!SLDS) { r.hr = c1.z; r.vb = c1.w; }
        } else {
          r.i11 = c0.x; r.i12 = 0.0f; r.i22 = 0.0f; r.b1 = c0.y; r.b2 = 0.0f;
          if (!SLDS) { r.hr = c0.z; r.vb = c0.w; }
        }
        // sh of the left pixel (s[x-1] + s[x]) and sv of the upper one (s[y-1] + s[y]): rb_load's hl / vt
        if (!SLDS) {
          r.hl = x > 0 ? S5[1] + S5[0] : 0.0f;
          r.vt = y > 0 ? S5[3] + S5[0] : 0.0f;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    // ---- red-black SOR: colour 0 (x + y even), then colour 1, solverit times; a half-sweep reads the other
    // colour's entries only and writes its own thread's
#pragma unroll 1
    for (int sw = 0; sw < a.solverit; ++sw) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          if (xy[c][k] < 0) continue;
          const int q = lv_fresh(xy[c][k]), x = q & 0xffff, y = q >> 16;
          const LvNb nb = lv_nb_any(x, y, c, w, E);
          const V o = UV[nb.i[0]], l = UV[nb.i[1]], r = UV[nb.i[2]], t = UV[nb.i[3]], b = UV[nb.i[4]];
          if (SLDS) {
            const float sc = S[nb.i[0]], sl = S[nb.i[1]], sr = S[nb.i[2]], su = S[nb.i[3]], sd = S[nb.i[4]];
            d[c][k].hl = x > 0 ? sl + sc : 0.0f;
            d[c][k].vt = y > 0 ? su + sc : 0.0f;
            d[c][k].hr = x < w - 1 ? sc + sr : 0.0f;
            d[c][k].vb = y < h - 1 ? sc + sd : 0.0f;
          }
          if constexpr (NOP == 2) {
            const f2v n = rb_update_of_pk(d[c][k], x > 0, x < w - 1, y == 0 || y >= h - 1, y == 0, a.omega, lv_f2(l),
                                          lv_f2(r), lv_f2(t), lv_f2(b), lv_f2(o));
            UV[nb.i[0]] = make_float2(n.x, n.y);
          } else {
            float u = o, v = 0.0f;
            rb_update<MODE>(d[c][k], x, y, w, h, a.omega, l, r, t, b, 0.0f, 0.0f, 0.0f, 0.0f, u, v);
            UV[nb.i[0]] = u;
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
      }
    }
  }

  // ---- the level's flow: uu = wx + du, vv = wy + dv (DE: clamped to the camera side) -- k_tv_final's values
  float *WX = a.flow + (long)f * a.nop * wh;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      if (xy[c][k] < 0) continue;
      const int x = xy[c][k] & 0xffff, y = xy[c][k] >> 16, p = y * w + x;
      const int idx = c * E + (p >> 1);
      const V wv = WXY[idx], uv = UV[idx];
      if constexpr (NOP == 2) {
        WX[p] = wv.x + uv.x;
        WX[wh + p] = wv.y + uv.y;
      } else {
        const float s = wv + uv;
        WX[p] = a.camlr == 0 ? ssemin(s, 0.0f) : ssemax(s, 0.0f);
      }
    }
}

template <int NOP, int NOC>
void launch_level_rb_n(const TvArgs &a, int n_inner, hipStream_t s) {
  const int E = lat_entries(a.w, a.h);
  const size_t lds = lv_lds(NOP, a.w, a.h);
  auto threads = [](int per) { return (per + 63) / 64 * 64; };
  if (E <= kLvT) k_tv_level_rb<NOP, NOC, 1><<<a.n, threads(E), lds, s>>>(a, n_inner);
  else if (E <= 2 * kLvT) k_tv_level_rb<NOP, NOC, 2><<<a.n, threads((E + 1) / 2), lds, s>>>(a, n_inner);
  else k_tv_level_rb<NOP, NOC, 4><<<a.n, threads((E + 3) / 4), lds, s>>>(a, n_inner);
}

}  // namespace

__global__ void k_warm_tvrb(int *p) {  // code-object warm-up of this unit (warm_kernels_module)
  if (p) *p = 0;
}
void warm_tvrb_module(hipStream_t s) { k_warm_tvrb<<<1, 64, 0, s>>>(nullptr); }

// The fused level launch: red-black order (sor_mode = 1), the block SOR (not the OpenMP build's point SOR, not
// levels under 2 x 2, which run solver.c's point form), levels of at most kLvPix pixels, the prep + derivatives
// launch writing the colour-split layout.
bool tv_level_rb_ok(const TvArgs &a) {
  return a.sor_redblack && !a.sor_point && a.w >= 2 && a.h >= 2 && (long)a.w * a.h <= kLvPix &&
         tv_prepd_ok(a) && lv_lds(a.nop, a.w, a.h) <= 160 * 1024 && (a.noc == 1 || a.noc == 3);
}

void launch_tv_level_rb(const TvArgs &a, int n_inner, hipStream_t s) {
  if (a.nop == 2) {
    if (a.noc == 1) launch_level_rb_n<2, 1>(a, n_inner, s);
    else launch_level_rb_n<2, 3>(a, n_inner, s);
  } else {
    if (a.noc == 1) launch_level_rb_n<1, 1>(a, n_inner, s);
    else launch_level_rb_n<1, 3>(a, n_inner, s);
  }
}

}  // namespace ofdis
