// ofdis_tvsysor.hip -- one TV inner iteration of a level of at most 128 rows as ONE launch: the system
// (compute_smoothness, compute_data, sub_laplacian and the 2x2 inverse of sor_coupled's first sweep) is produced
// four anti-diagonals ahead of the exact-order SOR wavefront, inside the SOR's own barrier steps, and handed to the
// sweeps through LDS -- no coefficient round trip through HBM, no separate system launch.
//
// Reference: refine_variational.cpp:192-222 (the inner iteration), FDF1.0.1/opticalflow_aux.c:138-187
// (compute_smoothness), :194-223 (sub_laplacian), :408-594 (compute_data, intensity images), FDF1.0.1/solver.c:83-433
// (sor_coupled).  The same device functions as the two-launch path (ofdis_tv_dev.inc: smooth_compute, the two halves
// of data_of, sys_finish) and the same SOR update as k_tv_sor_lanes, so the same bits.
//
// Why: the two-launch form writes 32 B of coefficients per pixel and inner iteration and reads
// them back, and costs one extra launch per inner iteration -- 18 of them in the drop-in CLI's single 1080p pair.
// The dataflow forms of round 4 (progress-counter polls instead of barriers) lost to the barrier they replaced; here
// every hand-over is ordered by the one s_barrier per step the exact-order SOR pays anyway.
//
// One workgroup per frame; lane = row y of a row group g (G = ceil(h / 64) <= 2), every wave joins every barrier:
//   S x G sweep waves, wave (g, s) = sweep s of rows 64 g .. 64 g + 63 (k_tv_sor_lanes' schedule: pixel (x, y) of
//     sweep s at step t = x + y + 2 s; interval t >= 0 is SOR step t);
//   4 x G producer waves, wave (g, j) = the system of the diagonals d = j (mod 4), spread over four intervals:
//     A at d - 4: writes row d + 3 into the row ring (loaded at its previous A), the pixel's own values, the mask and
//       the colour half of the data term, issues the loads of row d + 7 and of diagonal d + 4's derivatives;
//     B at d - 3: s(d + 2) into the s ring;
//     C at d - 2: the gradient half of the data term;
//     D at d - 1: sub_laplacian from the s and wx / wy rings, the inverse (sys_finish), the coefficient ring write.
//   Row r is written at interval r - 7 and read until r (sweep 0 takes the old (du, dv) from the row ring), s(e) lives
//   from e - 5 to e, the coefficients of d from d - 1 to d + 2 (S - 1): eight slots each.
// LDS rings are lane-major -- [entry y][slot], slot = diagonal mod 8, strides padded to an odd number of 16-byte
// (or 4-byte) units, so a wave's ds_read_b128 / b64 / b32 of one slot is conflict-free; every SOR slot offset is an
// immediate of the 8-step unrolled block.  Entries exist for rows 0 .. h - 1 (lanes beyond h read row h - 1: their
// values are never used) and the (u, v) rings keep a dump entry h + 1 for them.
#include "ofdis_internal.h"
#include "ofdis_math.h"

#include <algorithm>

#pragma clang fp contract(off)

namespace ofdis {
namespace {

#include "ofdis_tv_dev.inc"

constexpr int kYS = 8;                       // s / coefficient ring slots (power of 2)
constexpr int kRS = kYS;                     // row ring slots (the sweeps index it with the coefficient slot)
constexpr int kRowStride = 16 * (kRS + 1);   // bytes per row-ring entry: 8 float4 slots + 1 pad
constexpr int kPh = 4;                       // producer phases = producer waves per row group
constexpr int kSStride = 4 * (kYS + 1);      // s ring: 8 floats + 1 pad
constexpr int kCStride = 32 * kYS + 16;      // coefficient ring: 8 x (c0, c1) + 1 float4 pad
constexpr int kUVSlots = 4;                  // (u, v) ring depth (steps t, t-1, t-2; a power of 2)
constexpr int kUVStride = 8 * (kUVSlots + 1);  // bytes per (u, v) ring entry
constexpr int kSU = 8;                       // SOR steps per unrolled block (a multiple of kYS and kUVSlots)

__host__ __device__ __forceinline__ size_t sysor_lds(int S, int h) {
  const size_t uv = (size_t)S * (h + 2) * kUVStride;
  return (uv + 15) / 16 * 16 + (size_t)h * (kCStride + kRowStride + kSStride);
}

// Skewed plane row of diagonal d (clamped into the plane; folded modulo w when h <= w): see sor_row2.
__device__ __forceinline__ int plane_row(int d, int lim, int rmax) {
  const int dd = max(d, 0);
  return min(dd >= lim ? dd - lim : dd, rmax);
}

struct SysSorLds {
  char *uv, *coef, *rows, *sr;
  __device__ SysSorLds(char *lds, int S, int h) {
    uv = lds;
    coef = lds + ((size_t)S * (h + 2) * kUVStride + 15) / 16 * 16;
    rows = coef + (size_t)h * kCStride;
    sr = rows + (size_t)h * kRowStride;
  }
};

// Register pins: the values are "redefined" here, so no computation that uses them can move above this point and
// none that produces them below it.  Around each barrier they keep a phase's arithmetic inside its interval (the
// barrier orders memory only: the compiler otherwise hoisted phase B's register-only work into phase A).
__device__ __forceinline__ void pin(float &x) { asm volatile("" : "+v"(x)); }
template <class... T>
__device__ __forceinline__ void pins(T &...x) {
  (pin(x), ...);
}

// ------------------------------------------------------------------------------------------------ producer
struct Producer {
  TvArgs a;  // a copy: its fields live in scalar registers
  int y, w, h, lim, rmax;
  bool yin;
  unsigned o_ye, o_yu, o_yd;  // lane entry offsets of rows min(y, h-1), and of the rows above / below (clamped)
  char *rows, *sr, *coef;
  const float *pw[4];          // wx, wy, du, dv planes of the frame
  const float *pd[8];          // Ix, Iy, Iz, Ixx, Ixy, Iyy, Ixz, Iyz planes of the frame
  float4 rowv;                 // the row loaded at the previous phase A (wx, wy, du, dv)
  float dq[8];                 // the derivatives of the next diagonal of this wave
  // carried from A to C
  float u, v, m, wxc, wyc, A11, A12, A22, B1, B2;
  bool first;

  __device__ __forceinline__ float4 &row_at(int r, unsigned oe) const {
    return *reinterpret_cast<float4 *>(rows + oe * kRowStride + (unsigned)(r & (kRS - 1)) * 16u);
  }
  __device__ __forceinline__ float &s_at(int e, unsigned oe) const {
    return *reinterpret_cast<float *>(sr + oe * kSStride + (unsigned)(e & (kYS - 1)) * 4u);
  }
  __device__ __forceinline__ unsigned goff(int r) const { return (unsigned)(plane_row(r, lim, rmax) * h) + o_ye; }
  __device__ __forceinline__ void load_row(int r) {
    const unsigned o = goff(r);
    rowv = make_float4(ldu(pw[0], o), ldu(pw[1], o), ldu(pw[2], o), ldu(pw[3], o));
  }
  __device__ __forceinline__ void load_deriv(int d) {
    const unsigned o = goff(d);
#pragma unroll
    for (int k = 0; k < 8; ++k) dq[k] = ldu(pd[k], o);
  }
  // s of diagonal e at this lane's row (compute_smoothness, replicate border by operand selection): rows e - 1 .. e + 1
  __device__ __forceinline__ void smooth(int e) {
    const int x = e - y;
    const float4 q0 = row_at(e, o_ye), ql = row_at(e - 1, o_ye), qr = row_at(e + 1, o_ye);
    const float4 qu = row_at(e - 1, o_yu), qd = row_at(e + 1, o_yd);
    const float4 q1 = x > 0 ? ql : q0, q2 = x < w - 1 ? qr : q0, q3 = y > 0 ? qu : q0, q4 = y < h - 1 ? qd : q0;
    const float wx5[5] = {q0.x, q1.x, q2.x, q3.x, q4.x}, du5[5] = {q0.z, q1.z, q2.z, q3.z, q4.z};
    const float wy5[5] = {q0.y, q1.y, q2.y, q3.y, q4.y}, dv5[5] = {q0.w, q1.w, q2.w, q3.w, q4.w};
    const float sv = smooth_compute<2>(a, first, wx5, du5, wy5, dv5);
    if (yin) s_at(e, o_ye) = (unsigned)x < (unsigned)w ? sv : 0.0f;
  }
  // A (interval d - 4): the row loaded four intervals ago into the ring (row d + 3), the pixel's own values, image_warp's
  // mask, the colour half of the data term; the loads of row d + 7 and of diagonal d + 4's derivatives (this wave's
  // next diagonal)
  __device__ __forceinline__ void phase_a(int d) {
    if (yin) row_at(d + 3, o_ye) = rowv;
#pragma unroll
    for (int k = 0; k < 8; ++k) cur[k] = dq[k];
    const float4 own = row_at(d, o_ye);
    wxc = own.x;
    wyc = own.y;
    u = own.z;
    v = own.w;
    m = warp_mask(d - y, y, wxc, wyc, w, h);
    data_of_gray_colour(u, v, m, cur[0], cur[1], cur[2], a.hdo3, A11, A12, A22, B1, B2);
    load_row(d + 7);
    load_deriv(d + 4);
  }
  // B (d - 3): s(d + 2) into the s ring (rows d + 1 .. d + 3)
  __device__ __forceinline__ void phase_b(int d) { smooth(d + 2); }
  float cur[8];
  __device__ __forceinline__ void pin_ab() {
    pins(u, v, m, wxc, wyc, A11, A12, A22, B1, B2, cur[3], cur[4], cur[5], cur[6], cur[7]);
  }
  __device__ __forceinline__ void pin_bc() { pin_ab(); }
  __device__ __forceinline__ void pin_cd() { pins(wxc, wyc, A11, A12, A22, B1, B2); }
  // C (d - 2): the gradient half
  __device__ __forceinline__ void phase_c() {
    data_of_gray_gradient(u, v, m, cur[3], cur[4], cur[5], cur[6], cur[7], a.hgo3, A11, A12, A22, B1, B2);
  }
  // D (d - 1): sub_laplacian, the inverse, the coefficient ring write
  __device__ __forceinline__ void phase_d(int d) {
    const int x = d - y;
    const float S5[5] = {s_at(d, o_ye), s_at(d - 1, o_ye), s_at(d + 1, o_ye), s_at(d - 1, o_yu), s_at(d + 1, o_yd)};
    const float4 ql = row_at(d - 1, o_ye), qr = row_at(d + 1, o_ye), qu = row_at(d - 1, o_yu), qd = row_at(d + 1, o_yd);
    const float X5[5] = {wxc, ql.x, qr.x, qu.x, qd.x}, Y5[5] = {wyc, ql.y, qr.y, qu.y, qd.y};
    float4 c0, c1;
    sys_finish<2>(a, x, y, S5, X5, Y5, A11, A12, A22, B1, B2, c0, c1);
    if (yin) {
      float4 *C = reinterpret_cast<float4 *>(coef + o_ye * kCStride + (unsigned)(d & (kYS - 1)) * 32u);
      C[0] = c0;
      C[1] = c1;
    }
  }
};

// ------------------------------------------------------------------------------------------------ sweeps
// Sweep SI of one row group, k_tv_sor_lanes' step (sor_coupled, solver.c:83-433) with every operand from LDS: the
// coefficients from the producers' ring, sweep 0's old (du, dv) from the row ring.
template <int S, int SI>
struct Sweep {
  static constexpr bool FIRST = SI == 0, LAST = SI == S - 1;
  f2v pp, prv;
  float phr, pvv;
  bool top_lds, border, notop;
  int y, w, h, lim, rmax;
  const char *crow, *rrow, *rrow1;  // lane entry of the coefficient ring (row ye), the row ring (ye, ye1)
  const char *ctop;                  // the coefficient ring entry of row y - 1 (top_lds lanes)
  f2v *ring_s, *ring_s_top;          // this sweep's (u, v) ring: own entry, the entry of row y - 1
  const f2v *ring_p, *ring_pb;       // previous sweep's: own entry, the entry of row y + 1
  float *du, *dv;
  float omega;

  template <int Q>
  __device__ __forceinline__ void step(const int t) {
    constexpr int cs = ((Q - 2 * SI) % kYS + kYS) % kYS, cs1 = (cs + 1) % kYS, ct = (cs + kYS - 1) % kYS;
    constexpr int m0 = Q % kUVSlots, m1 = (Q + kUVSlots - 1) % kUVSlots;
    const int d = t - 2 * SI;
    const int xp = d - y;
    const bool hasl = xp > 0, hasr = xp < w - 1;
    f2v o, rgt, bt;
    if (FIRST) {  // (du, dv) = (.z, .w) of the row-ring float4
      o = *reinterpret_cast<const f2v *>(rrow + cs * 16 + 8);
      rgt = *reinterpret_cast<const f2v *>(rrow + cs1 * 16 + 8);
      bt = *reinterpret_cast<const f2v *>(rrow1 + cs1 * 16 + 8);
    } else {  // own value after the previous sweep (step t-2) = the right neighbour read at step t-1
      o = prv;
      rgt = ring_p[m1];
      bt = ring_pb[m1];
      prv = rgt;
    }
    const float4 c0 = *reinterpret_cast<const float4 *>(crow + cs * 32);
    const float4 c1 = *reinterpret_cast<const float4 *>(crow + cs * 32 + 16);
    f2v tp = f2v{dpp_from_prev_lane(pp.x), dpp_from_prev_lane(pp.y)};
    float tsv = dpp_from_prev_lane(pvv);
    if (top_lds) {
      tp = ring_s_top[m1];
      tsv = reinterpret_cast<const float4 *>(ctop + ct * 32 + 16)->w;
    }
    const float hr = c1.z, vv = c1.w;
    const f2v bb = f2v{c1.x, c1.y};
    const f2v rr = hasr ? rgt : f2v{0.0f, 0.0f};
    const f2v X = hr * rr, Y = tsv * tp, Z = vv * bt;
    // solver.c's three border expression trees (sor_rhs), lane-constant operand selects
    const f2v l = X + (border ? bb : Y);
    const f2v rg = (border ? f2v{-0.0f, -0.0f} : bb) + (border ? (notop ? Z : Y) : Z);
    const f2v srr = l + rg;
    const f2v Bv = hasl ? phr * pp + srr : srr;
    const f2v m_1 = f2v{c0.x, c0.y} * Bv.x, m_2 = f2v{c0.z, c0.w} * Bv.y;  // (i11,i12), (i12,i22)
    const f2v nw = o + omega * ((m_1 + m_2) - o);
    ring_s[m0] = nw;
    if (LAST && (unsigned)xp < (unsigned)w && y < h) {
      const unsigned r0 = (unsigned)plane_row(d, lim, rmax) * (unsigned)h + (unsigned)y;
      du[r0] = nw.x;
      dv[r0] = nw.y;
    }
    pp = nw;
    pvv = vv;
    phr = hr;
    __syncthreads();
  }
  template <int J>
  __device__ __forceinline__ void block(const int t) {
    step<J>(t + J);
    if constexpr (J + 1 < kSU) block<J + 1>(t);
  }
  // Steps [0, T), T a multiple of kSU; the wave's rows y0 .. ymax are inside the frame for t - 2 SI in
  // [y0, ymax + w - 1]: blocks wholly outside only join the barriers.
  __device__ __forceinline__ void run(int T, int y0, int ymax) {
    pp = f2v{0.0f, 0.0f};
    phr = 0.0f;
    pvv = 0.0f;
    const int ta = max(0, (y0 + 2 * SI) / kSU * kSU);
    const int tb = max(ta, min(T, (ymax + w - 1 + 2 * SI) / kSU * kSU + kSU));  // ta <= tb <= T: T barriers in all
    for (int t = 0; t < ta; ++t) __syncthreads();
    // the previous sweep's value at step ta - 2 (written before the barrier of step ta - 1; zero before t = 0)
    if (!FIRST) prv = ta >= 2 ? ring_p[(ta - 2) % kUVSlots] : f2v{0.0f, 0.0f};
    for (int t = ta; t < tb; t += kSU) block<0>(t);
    for (int t = tb; t < T; ++t) __syncthreads();
  }
};

template <int S, int G>
__global__ __launch_bounds__(64 * G * (S + kPh)) void k_tv_sysor(TvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int h = a.h, w = a.w;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const SysSorLds L(lds, S, h);
  const int NRU = h + 2;  // (u, v) ring entries per sweep: row y at min(y, h) + 1 (entry 0 = row -1, h + 1 = dump)
  for (int i = threadIdx.x; i < S * NRU * (kUVStride / 8); i += blockDim.x) reinterpret_cast<f2v *>(L.uv)[i] = f2v{0.f, 0.f};
  const int f = blockIdx.x;
  const long fo = (long)f * a.sp;
  const int lim = a.wrap ? w : 1 << 30, rmax = a.wrap ? w - 1 : w + h - 2;
  const int T = ((w - 1) + (h - 1) + 2 * (S - 1) + 1 + kSU - 1) / kSU * kSU;  // SOR steps
  const int NI = kPh + T;                                                    // intervals -kPh .. T - 1
  if (wid < S * G) {
    // ---------------------------------------------------------------- sweep wave (g, s)
    const int g = wid / S, s = wid - g * S;
    const int y = 64 * g + lane, y0 = 64 * g, ymax = min(y0 + 63, h - 1);
    const unsigned ye = (unsigned)min(y, h - 1), ye1 = (unsigned)min(y + 1, h - 1);
    const unsigned eo = (unsigned)min(y, h) + 1, eb = (unsigned)min(y + 1, h) + 1;
    auto setup = [&](auto &st) {
      st.y = y; st.w = w; st.h = h; st.lim = lim; st.rmax = rmax;
      st.crow = L.coef + ye * kCStride;
      st.ctop = L.coef + (unsigned)max(y - 1, 0) * kCStride;
      st.rrow = L.rows + ye * kRowStride;
      st.rrow1 = L.rows + ye1 * kRowStride;
      f2v *uvs = reinterpret_cast<f2v *>(L.uv + (size_t)s * NRU * kUVStride);
      const f2v *uvp = reinterpret_cast<const f2v *>(L.uv + (size_t)(s > 0 ? s - 1 : 0) * NRU * kUVStride);
      st.ring_s = uvs + eo * (kUVStride / 8);
      st.ring_s_top = uvs + (eo - 1) * (kUVStride / 8);
      st.ring_p = uvp + eo * (kUVStride / 8);
      st.ring_pb = uvp + eb * (kUVStride / 8);
      st.top_lds = lane == 0 && g > 0;
      st.notop = y == 0;
      st.border = y == 0 || y >= h - 1;
      st.du = a.du + fo;
      st.dv = a.dv + fo;
      st.omega = a.omega;
      __syncthreads();  // prologue: the producers' first rows
      __syncthreads();  // prologue: s(0), s(1)
      for (int i = 0; i < kPh; ++i) __syncthreads();  // intervals -kPh .. -1: the first coefficients
      st.run(T, y0, ymax);
    };
    if (s == 0) {
      Sweep<S, 0> st;
      setup(st);
    } else if (s == 1) {
      Sweep<S, 1> st;
      setup(st);
    } else {
      Sweep<S, (S > 2 ? 2 : 1)> st;
      setup(st);
    }
    return;
  }
  // ------------------------------------------------------------------ producer wave (g, j)
  const int k = wid - S * G, g = k / kPh, j = k - kPh * g;
  Producer P;
  P.a = a;
  P.y = 64 * g + lane;
  P.w = w;
  P.h = h;
  P.lim = lim;
  P.rmax = rmax;
  P.yin = P.y < h;
  const int ye = min(P.y, h - 1);
  P.o_ye = (unsigned)ye;
  P.o_yu = (unsigned)max(ye - 1, 0);
  P.o_yd = (unsigned)min(ye + 1, h - 1);
  P.rows = L.rows;
  P.sr = L.sr;
  P.coef = L.coef;
  P.first = a.first_iter != 0;
  P.pw[0] = a.wxs + fo; P.pw[1] = a.wys + fo; P.pw[2] = a.du + fo; P.pw[3] = a.dv + fo;
  const long fd = (long)f * a.sp;  // intensity images: one channel plane per frame
  P.pd[0] = a.Ix + fd; P.pd[1] = a.Iy + fd; P.pd[2] = a.Iz + fd; P.pd[3] = a.Ixx + fd;
  P.pd[4] = a.Ixy + fd; P.pd[5] = a.Iyy + fd; P.pd[6] = a.Ixz + fd; P.pd[7] = a.Iyz + fd;
  // prologue: rows 0 .. 2 (wave j < 3: row j), then the loads of this wave's first A (row j + 3, diagonal j)
  for (int r = j; r < 3; r += kPh) {
    P.load_row(r);
    if (P.yin) P.row_at(r, P.o_ye) = P.rowv;
  }
  P.load_row(j + 3);
  P.load_deriv(j);
  __syncthreads();
  if (j < 2) P.smooth(j);  // s(0), s(1): phase A of diagonal d computes s(d + 2)
  __syncthreads();
  // intervals: wave j starts diagonal j at interval j - kPh, then every kPh-th diagonal
  int left = NI;
  for (int i = 0; i < j; ++i, --left) __syncthreads();
  for (int d = j; left >= kPh; d += kPh, left -= kPh) {
    P.phase_a(d);
    P.pin_ab();
    __syncthreads();
    P.pin_ab();
    P.phase_b(d);
    P.pin_bc();
    __syncthreads();
    P.pin_bc();
    P.phase_c();
    P.pin_cd();
    __syncthreads();
    P.pin_cd();
    P.phase_d(d);
    __syncthreads();
  }
  for (; left > 0; --left) __syncthreads();
}

template <int S, int G>
void launch_sysor_sg(const TvArgs &a, hipStream_t s) {
  k_tv_sysor<S, G><<<a.n, 64 * G * (S + kPh), sysor_lds(S, a.h), s>>>(a);
}

}  // namespace

// The fused launch applies to optical flow on intensity images, the exact lexicographic order with 2 or 3 sweeps,
// levels of 2 .. 128 rows and at least 2 columns (option sysor).
bool tv_sysor_ok(const TvArgs &a) {
  return a.sysor && a.nop == 2 && a.noc == 1 && !a.sor_point && !a.sor_redblack && !a.sor_generic &&
         a.sor_variant != 1 && (a.solverit == 2 || a.solverit == 3) && a.h >= 2 && a.h <= 128 && a.w >= 2 &&
         sysor_lds(a.solverit, a.h) <= 160 * 1024;
}

void launch_tv_sysor(const TvArgs &a, hipStream_t s) {
  const bool g2 = a.h > 64;
  if (a.solverit == 2) {
    if (g2) launch_sysor_sg<2, 2>(a, s);
    else launch_sysor_sg<2, 1>(a, s);
  } else {
    if (g2) launch_sysor_sg<3, 2>(a, s);
    else launch_sysor_sg<3, 1>(a, s);
  }
}

}  // namespace ofdis
