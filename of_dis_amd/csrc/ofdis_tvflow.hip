// ofdis_tvflow.hip -- one TV inner iteration (smoothness + system + exact-order SOR) as ONE dataflow launch.
//
// Reference: refine_variational.cpp:192-222 (the inner iteration), opticalflow_aux.c:138-223,408-747
// (compute_smoothness, compute_data / compute_data_DE, sub_laplacian), solver.c:83-433 / :439-471 (sor_coupled /
// the DE point SOR).  Same functions as the two-launch path (ofdis_tv_dev.inc), same operands, same order: the
// same bits.
//
// Why: the two-launch form writes 32 B of coefficients per pixel and inner
// iteration to HBM and reads them back, and in the latency regime (one pair per call, config D's 32 pairs per
// GPU) each of the 18 system launches of a 1080p pair costs ~10 us of a 0.84 ms chain.  Here one workgroup owns
// one frame's level for one inner iteration and every intermediate stays in LDS.  Its waves run free, each in
// its own role, and hand work to each other through LDS rings guarded by per-wave progress counters (workgroup-
// scope release / acquire), not by workgroup barriers -- so no wave waits for the slowest role's step, and a
// role whose per-diagonal work is long (the system: ~12 correctly rounded divisions per pixel) runs on several
// waves round robin:
//
//   M (one wave per row group g of 64 rows): stages the level's skewed rows of (wx, wy, du, dv) into the row
//     ring (global loads issued K rows ahead) and computes the smoothness s of diagonal e (compute_smoothness on
//     uu = wx + du) into the s ring;
//   Y (P waves per row group): the system of diagonal d (diffusivities, data term, sub_laplacian and, OF, the
//     2x2 inverse sor_coupled's first sweep computes -- sys_compute) into the coefficient ring, d = j mod P;
//   SOR (S waves per row group, sweep s): sor_coupled's update of diagonal d = x + y for sweep s, exactly as
//     k_tv_sor_lanes (pixel (x, y) of sweep s needs (x-1, y), (x, y-1) of sweep s and (x+1, y), (x, y+1) of sweep
//     s-1: the diagonal order reproduces the lexicographic raster bit for bit); sweep 0 reads the old (du, dv)
//     from the row ring, the last sweep stores the new ones.
//
// Diagonal d of a w x h level holds pixels (d - y, y); its skewed plane row is d mod w (folded, h <= w) or d.
// Rings are [slot][entry] with entry = y + 1 (entries 0 and 64 G + 1 are the halo rows -1 and 64 G).
// Every wait is bounded: past kFlowSpinLimit polls a wave raises the abort word, every wave leaves its loop and
// the launch ends (a_err counts it) -- a protocol error shows as a failed parity test, never as a hang.
#include "ofdis_internal.h"
#include "ofdis_math.h"

#include <utility>

#pragma clang fp contract(off)

namespace ofdis {
namespace {

#include "ofdis_tv_dev.inc"

constexpr int kFlowRR = 16;  // row ring slots: M runs up to RR - 5 rows ahead of sweep 0
constexpr int kFlowRS = 16;  // s ring slots
constexpr int kFlowRC = 16;  // coefficient ring slots: the system runs up to RC - 2 diagonals ahead of the last sweep
constexpr int kFlowD = 6;    // (u, v) ring slots per sweep
constexpr int kFlowK = 4;    // M's global loads in flight (rows; two per iteration)
constexpr int kFlowSpinLimit = 1 << 22;

// Progress counters live in LDS.  Release = every earlier LDS write of the wave has completed before the counter
// store issues (s_waitcnt lgkmcnt(0)); acquire = the counter read has returned before any later LDS read issues
// (the same wait, and a compiler barrier so no ring read is hoisted above the poll).  LDS only: a workgroup-scope
// fence would also wait for the wave's outstanding global loads (M's prefetch) and stores (the last sweep's).
__device__ __forceinline__ int cnt_load(const int *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void cnt_publish(int *p, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void cnt_acquire() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// The fast forms the SOR waves use.  A wave's LDS instructions are performed in issue order, so (1) a counter store
// issued after the ring stores it publishes is seen after them without waiting for them, and (2) ring reads issued
// after the counter read (in the same round trip) see at least the state the counter showed: a poll that finds its
// counters ready has its operands too.  The empty asm keeps the compiler from reordering the LDS accesses.
__device__ __forceinline__ void cnt_publish_ordered(int *p, int v) {
  asm volatile("" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

template <int NOP, int NOC, int S, int G, int P>
struct Flow {
  static constexpr int NR = 64 * G + 2;  // ring entries per slot
  static constexpr int CW = NOP == 2 ? 2 : 1;
  static constexpr int NW = S * G + G + P * G;
  // progress counters: SOR (s, g) diagonals done; M rows written, s values done; Y (j, g) diagonals done
  static constexpr int C_SOR = 0, C_M = S * G, C_S = S * G + G, C_Y = S * G + 2 * G, C_ABORT = S * G + 2 * G + P * G;
  static constexpr int NCNT = (C_ABORT + 1 + 3) / 4 * 4;
  static constexpr size_t OFF_ROW = 16 * NCNT;                                  // [RR][NR] float4
  static constexpr size_t OFF_COEF = OFF_ROW + sizeof(float4) * kFlowRR * NR;   // [RC][CW][NR] float4
  static constexpr size_t OFF_UV = OFF_COEF + sizeof(float4) * kFlowRC * CW * NR;  // [S][D][NR] f2v
  static constexpr size_t OFF_S = OFF_UV + sizeof(f2v) * S * kFlowD * NR;       // [RS][NR] float
  static constexpr size_t LDS = OFF_S + sizeof(float) * kFlowRS * NR;

  const TvArgs &a;
  int *cnt;
  float4 *row, *coef;
  f2v *uv;
  float *sr;
  int w, h, E, lim;
  unsigned f0;
  bool first;

  __device__ Flow(const TvArgs &a_, char *lds, int frame) : a(a_) {
    cnt = reinterpret_cast<int *>(lds);
    row = reinterpret_cast<float4 *>(lds + OFF_ROW);
    coef = reinterpret_cast<float4 *>(lds + OFF_COEF);
    uv = reinterpret_cast<f2v *>(lds + OFF_UV);
    sr = reinterpret_cast<float *>(lds + OFF_S);
    w = a.w;
    h = a.h;
    E = a.w + a.h - 1;
    lim = a.wrap ? a.w : 1 << 30;
    f0 = (unsigned)((long)frame * a.sp);
    first = a.first_iter != 0;
  }
  __device__ __forceinline__ int prow(int d) const { return d >= lim ? d - lim : d; }  // 0 <= d < E

  // Poll until ok(C) holds, C(i) = counter i: lane i < NCNT reads counter i (one LDS round trip per poll), the
  // checks take them by v_readlane.  false: the launch aborts.
  template <class F>
  __device__ __forceinline__ bool wait(F &&ok) {
    const int lane = threadIdx.x & 63;
    for (int spin = 0;; ++spin) {
      const int v = cnt_load(cnt + (lane < NCNT ? lane : 0));
      auto C = [&](int i) { return __builtin_amdgcn_readlane(v, i); };
      if (ok(C)) {
        cnt_acquire();
        return true;
      }
      if (C(C_ABORT)) return false;
      if (spin > kFlowSpinLimit) {
        cnt_publish(cnt + C_ABORT, 1);
        if (lane == 0 && a.flow_err) atomicAdd(a.flow_err, 1);
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  // min over the row groups of counter block base (sweep s: base = C_SOR + s * G)
  template <class CF>
  __device__ __forceinline__ static int cmin(CF &C, int base) {
    int m = C(base);
#pragma unroll
    for (int g = 1; g < G; ++g) m = min(m, C(base + g));
    return m;
  }

  // ------------------------------------------------------------------------------------------------ M
  // The (wx, wy, du, dv) of diagonal e at lane y (zeros outside the diagonal range: never used).  Only the lanes
  // whose pixel (e - y, y) exists fetch their slot; the others read the row's first one (folded rows hold
  // diagonal e -+ w there; their values are discarded by selects wherever they are read).
  // Diagonals past the last one load the last one (no branch around the loads: they stay in flight across the
  // unrolled steps); rows outside the level are only ever read where a border select discards them.
  __device__ __forceinline__ float4 load_row(int e, int y) const {
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    e = e < E ? e : E - 1;
    const bool in = (unsigned)(e - y) < (unsigned)w && y < h;
    const unsigned o = f0 + (unsigned)(prow(e) * h) + (in ? (unsigned)y : 0u);
    q.x = ldu(a.wxs, o);
    q.z = ldu(a.du, o);
    if (NOP == 2) {
      q.y = ldu(a.wys, o);
      q.w = ldu(a.dv, o);
    }
    return q;
  }

  // s of diagonal e at lane y from rows e - 1, e, e + 1 of the ring (compute_smoothness's replicate border: an
  // absent neighbour is the centre); 0 outside the level
  __device__ __forceinline__ float smooth_at(int e, int y) const {
    const int x = e - y;
    const float4 q1 = row[(e % kFlowRR) * NR + y + 1];                  // centre
    const float4 ql = row[((e + kFlowRR - 1) % kFlowRR) * NR + y + 1];  // left  (x - 1, y)
    const float4 qu = row[((e + kFlowRR - 1) % kFlowRR) * NR + y];      // up    (x, y - 1)
    const float4 qr = row[((e + 1) % kFlowRR) * NR + y + 1];            // right (x + 1, y)
    const float4 qd = row[((e + 1) % kFlowRR) * NR + y + 2];            // down  (x, y + 1)
    float sv = 0.0f;
    if ((unsigned)x < (unsigned)w && y < h) {
      const bool l = x > 0, r = x < w - 1, u = y > 0, dn = y < h - 1;
      const float4 L = l ? ql : q1, Rt = r ? qr : q1, U = u ? qu : q1, D = dn ? qd : q1;
      const float wx5[5] = {q1.x, L.x, Rt.x, U.x, D.x}, du5[5] = {q1.z, L.z, Rt.z, U.z, D.z};
      const float wy5[5] = {q1.y, L.y, Rt.y, U.y, D.y}, dv5[5] = {q1.w, L.w, Rt.w, U.w, D.w};
      sv = smooth_compute<NOP>(a, first, wx5, du5, wy5, dv5);
    }
    return sv;
  }
  // iteration e (even): rows e + 3, e + 4 into the ring (R[2Q], R[2Q + 1] hold them), the loads of rows e + 3 + K,
  // e + 4 + K, and s of diagonals e, e + 1 (rows e - 1 .. e + 2, written by every M wave two iterations ago)
  template <int Q>
  __device__ __forceinline__ bool m_step(int e, int g, int y, float4 (&R)[kFlowK]) {
    if (e >= E) return true;
    // WAR: row e + 4 replaces row e + 4 - RR, read last by the system of diagonal e + 5 - RR (done once sweep 0 is
    // past it); the neighbouring groups' rows <= e + 2 (lanes y -+ 1 at the group edges)
    if (!wait([&](auto &C) {
          bool ok = cmin(C, C_SOR) >= e + 6 - kFlowRR;
          if (G > 1) ok = ok && (g == 0 || C(C_M + g - 1) >= e + 3) && (g == G - 1 || C(C_M + g + 1) >= e + 3);
          return ok;
        }))
      return false;
    row[((e + 3) % kFlowRR) * NR + y + 1] = R[2 * Q];
    row[((e + 4) % kFlowRR) * NR + y + 1] = R[2 * Q + 1];
    R[2 * Q] = load_row(e + 3 + kFlowK, y);
    R[2 * Q + 1] = load_row(e + 4 + kFlowK, y);
    const float s0 = smooth_at(e, y);
    const float s1 = e + 1 < E ? smooth_at(e + 1, y) : 0.0f;
    sr[(e % kFlowRS) * NR + y + 1] = s0;
    sr[((e + 1) % kFlowRS) * NR + y + 1] = s1;
    cnt_publish_ordered(cnt + C_M + g, e + 5);                     // rows 0 .. e + 4 written
    cnt_publish_ordered(cnt + C_S + g, e + 2 < E ? e + 2 : E);     // s of diagonals 0 .. e + 1
    return true;
  }
  __device__ void run_m(int g, int lane) {
    __builtin_amdgcn_s_setprio(2);
    const int y = 64 * g + lane;
    row[0 * NR + y + 1] = load_row(0, y);
    row[1 * NR + y + 1] = load_row(1, y);
    row[2 * NR + y + 1] = load_row(2, y);
    cnt_publish_ordered(cnt + C_M + g, 3);
    float4 R[kFlowK];  // rows 3 .. 3 + K - 1 in flight; iteration e consumes R[2Q], R[2Q + 1], Q = (e / 2) % 2
#pragma unroll
    for (int k = 0; k < kFlowK; ++k) R[k] = load_row(k + 3, y);
    for (int e = 0; e < E; e += 4) {
      if (!m_step<0>(e, g, y, R)) return;
      if (!m_step<1>(e + 2, g, y, R)) return;
    }
  }

  // ------------------------------------------------------------------------------------------------ Y
  struct Der {
    float Ix[NOC], Iy[NOC], Iz[NOC], Ixx[NOC], Ixy[NOC], Iyy[NOC], Ixz[NOC], Iyz[NOC];
  };
  __device__ __forceinline__ void load_der(int d, int y, Der &q) const {
    const int dd = d < E ? d : E - 1;
    const bool in = (unsigned)(dd - y) < (unsigned)w && y < h;
    const unsigned o0 = f0 * (unsigned)NOC + (unsigned)(prow(dd) * h) + (in ? (unsigned)y : 0u);
#pragma unroll
    for (int ch = 0; ch < NOC; ++ch) {
      const unsigned o = o0 + (unsigned)(ch * a.sp);
      q.Ix[ch] = ldu(a.Ix, o); q.Iy[ch] = ldu(a.Iy, o); q.Iz[ch] = ldu(a.Iz, o); q.Ixx[ch] = ldu(a.Ixx, o);
      q.Ixy[ch] = ldu(a.Ixy, o); q.Iyy[ch] = ldu(a.Iyy, o); q.Ixz[ch] = ldu(a.Ixz, o); q.Iyz[ch] = ldu(a.Iyz, o);
    }
  }
  __device__ __forceinline__ bool y_step(int d, int g, int j, int y, Der &cur, Der &nxt) {
    if (d >= E) return true;
    const int sneed = d + 2 < E ? d + 2 : E;  // s of diagonals <= d + 1
    if (!wait([&](auto &C) {
          bool ok = C(C_S + g) >= sneed && cmin(C, C_SOR + (S - 1) * G) >= d - kFlowRC + 2;
          if (G > 1) ok = ok && (g == 0 || C(C_S + g - 1) >= sneed) && (g == G - 1 || C(C_S + g + 1) >= sneed);
          return ok;
        }))
      return false;
    load_der(d + P, y, nxt);  // the next diagonal of this wave, in flight during this one
    const int sm = ((d + kFlowRS - 1) % kFlowRS) * NR, s0 = (d % kFlowRS) * NR, sp1 = ((d + 1) % kFlowRS) * NR;
    const int rm = ((d + kFlowRR - 1) % kFlowRR) * NR, r0 = (d % kFlowRR) * NR, rp1 = ((d + 1) % kFlowRR) * NR;
    // centre, left (x - 1, y), right (x + 1, y), up (x, y - 1), down (x, y + 1)
    const float S5[5] = {sr[s0 + y + 1], sr[sm + y + 1], sr[sp1 + y + 1], sr[sm + y], sr[sp1 + y + 2]};
    const float4 qc = row[r0 + y + 1], ql = row[rm + y + 1], qr = row[rp1 + y + 1], qu = row[rm + y],
                 qd = row[rp1 + y + 2];
    const float X5[5] = {qc.x, ql.x, qr.x, qu.x, qd.x};
    const float Y5[5] = {qc.y, ql.y, qr.y, qu.y, qd.y};
    const int x = d - y;
    const float m = warp_mask(x, y, X5[0], Y5[0], w, h);
    float4 c0, c1;
    sys_compute<NOP, NOC>(a, x, y, S5, X5, Y5, m, qc.z, NOP == 2 ? qc.w : 0.0f, cur.Ix, cur.Iy, cur.Iz, cur.Ixx,
                          cur.Ixy, cur.Iyy, cur.Ixz, cur.Iyz, c0, c1);
    float4 *C = coef + (d % kFlowRC) * CW * NR + y + 1;
    C[0] = c0;
    if (NOP == 2) C[NR] = c1;
    cnt_publish_ordered(cnt + C_Y + j * G + g, d + 1);
    return true;
  }
  __device__ void run_y(int g, int j, int lane) {
    __builtin_amdgcn_s_setprio(0);
    const int y = 64 * g + lane;
    Der b0, b1;
    load_der(j, y, b0);
    for (int d = j; d < E; d += 2 * P) {
      if (!y_step(d, g, j, y, b0, b1)) return;
      if (!y_step(d + P, g, j, y, b1, b0)) return;
    }
  }

  // ------------------------------------------------------------------------------------------------ SOR
  template <int SI>
  __device__ void run_sor(int g, int lane) {
    constexpr bool FIRST = SI == 0, LAST = SI == S - 1;
    constexpr int MODE = NOP == 2 ? 0 : 2;
    const int y = 64 * g + lane;
    const bool border = y == 0 || y >= h - 1, notop = y == 0;
    const bool top_lds = lane == 0 && g > 0;
    const float omega = a.omega;
    f2v pp = f2v{0.0f, 0.0f};  // own (u, v) of the previous diagonal (left neighbour; lane y + 1's top)
    float phr = 0.0f, pvv = 0.0f;
    f2v *ring_s = uv + SI * kFlowD * NR;
    const f2v *ring_p = uv + (SI > 0 ? SI - 1 : 0) * kFlowD * NR;
    __builtin_amdgcn_s_setprio(3);
    const int lane63 = threadIdx.x & 63;
    for (int d = 0; d < E; ++d) {
      const int dn = d + 2 < E ? d + 2 : E;
      const int x = d - y;
      const bool hasl = x > 0, hasr = x < w - 1;
      const int dm = (d + kFlowD - 1) % kFlowD, cm = (d + kFlowRC - 1) % kFlowRC;
      f2v o, rgt, bt, tpl;
      float4 c0, c1;
      float tsvl;
      // one LDS round trip per poll: the counters, then (in issue order) the operands -- valid once they hold
      for (int spin = 0;; ++spin) {
        const int v = cnt_load(cnt + (lane63 < NCNT ? lane63 : 0));
        lds_order();
        if (FIRST) {
          const float4 r0 = row[(d % kFlowRR) * NR + y + 1];
          const float4 r1 = row[((d + 1) % kFlowRR) * NR + y + 1], r2 = row[((d + 1) % kFlowRR) * NR + y + 2];
          o = f2v{r0.z, r0.w};
          rgt = f2v{r1.z, r1.w};
          bt = f2v{r2.z, r2.w};
        } else {
          o = ring_p[(d % kFlowD) * NR + y + 1];
          rgt = ring_p[((d + 1) % kFlowD) * NR + y + 1];
          bt = ring_p[((d + 1) % kFlowD) * NR + y + 2];
        }
        const float4 *Cp = coef + (d % kFlowRC) * CW * NR + y + 1;
        c0 = Cp[0];
        c1 = MODE == 0 ? Cp[NR] : c0;
        if (G > 1) {  // lane 0 of a lower row group: the row above is the group above's
          tpl = ring_s[dm * NR + y];
          tsvl = coef[(cm * CW + CW - 1) * NR + y].w;
        }
        lds_order();
        auto C = [&](int i) { return __builtin_amdgcn_readlane(v, i); };
        bool ok;
        if (FIRST) {
          ok = C(C_Y + (d % P) * G + g) >= d + 1;
        } else {
          ok = C(C_SOR + (SI - 1) * G + g) >= dn;
          if (G > 1 && g + 1 < G) ok = ok && C(C_SOR + (SI - 1) * G + g + 1) >= dn;
        }
        if (G > 1 && g > 0) ok = ok && C(C_SOR + SI * G + g - 1) >= d;  // top of lane 0: diagonal d - 1
        if (!LAST) {
          // WAR: this ring slot's diagonal d - D is read by sweep SI + 1 of this group as its own (at d - D) and
          // right / bottom values (at d - D - 1), by sweep SI + 1 of the group above as lane 63's bottom
          ok = ok && C(C_SOR + (SI + 1) * G + g) >= d - kFlowD + 1;
          if (G > 1 && g > 0) ok = ok && C(C_SOR + (SI + 1) * G + g - 1) >= d - kFlowD;
        }
        // ... and by this sweep's group below as lane 0's top (at d - D + 1)
        if (G > 1 && g + 1 < G) ok = ok && C(C_SOR + SI * G + g + 1) >= d - kFlowD + 2;
        if (ok) break;
        if (C(C_ABORT)) return;
        if (spin > kFlowSpinLimit) {
          cnt_publish(cnt + C_ABORT, 1);
          if (lane63 == 0 && a.flow_err) atomicAdd(a.flow_err, 1);
          return;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      f2v tp = f2v{dpp_from_prev_lane(pp.x), MODE == 0 ? dpp_from_prev_lane(pp.y) : 0.0f};
      float tsv = dpp_from_prev_lane(pvv);
      if (G > 1 && top_lds) {
        tp = tpl;
        tsv = tsvl;
      }
      f2v nw;
      float vv;
      if (MODE == 0) {
        const float hr = c1.z;
        vv = c1.w;
        const f2v bb = f2v{c1.x, c1.y};
        const f2v rr = hasr ? rgt : f2v{0.0f, 0.0f};
        const f2v X = hr * rr, Yv = tsv * tp, Z = vv * bt;
        const f2v l = X + (border ? bb : Yv);
        const f2v rg = (border ? f2v{-0.0f, -0.0f} : bb) + (border ? (notop ? Z : Yv) : Z);
        const f2v srr = l + rg;
        const f2v Bv = hasl ? phr * pp + srr : srr;
        const f2v m_1 = f2v{c0.x, c0.y} * Bv.x, m_2 = f2v{c0.z, c0.w} * Bv.y;
        nw = o + omega * ((m_1 + m_2) - o);
        phr = hr;
      } else {
        const float a11 = c0.x, b1 = c0.y, hr = c0.z;
        vv = c0.w;
        const bool has_top = !notop, has_bot = !(border && has_top);
        const float tu = tp.x, ur = hasr ? rgt.x : 0.0f, hl = phr;
        float su = 0.0f;
        su = has_top ? su - tsv * tu : su;
        su = hasl ? su - hl * pp.x : su;
        su = has_bot ? su - vv * bt.x : su;
        su = hasr ? su - hr * ur : su;
        const float A = a11, Bq = b1 - su;
        nw = f2v{(1.0f - omega) * o.x + omega * (Bq / A), 0.0f};
        phr = hr;
      }
      ring_s[(d % kFlowD) * NR + y + 1] = nw;
      if (LAST && (unsigned)x < (unsigned)w && y < h) {
        const unsigned oo = f0 + (unsigned)(prow(d) * h + y);
        *reinterpret_cast<float *>(reinterpret_cast<char *>(a.du) + (size_t)oo * 4u) = nw.x;
        if (MODE == 0) *reinterpret_cast<float *>(reinterpret_cast<char *>(a.dv) + (size_t)oo * 4u) = nw.y;
      }
      pp = nw;
      pvv = vv;
      cnt_publish_ordered(cnt + C_SOR + SI * G + g, d + 1);
    }
  }
};

template <int NOP, int NOC, int S, int G, int P>
__global__ __launch_bounds__((64 * Flow<NOP, NOC, S, G, P>::NW)) void k_tv_flow(TvArgs a) {
  using F = Flow<NOP, NOC, S, G, P>;
  extern __shared__ __attribute__((aligned(16))) char flow_lds[];
  // zero everything (counters, rings: halo entries and slots of rows -1 / beyond stay finite)
  for (int i = threadIdx.x; i < (int)(F::LDS / 16); i += blockDim.x)
    reinterpret_cast<float4 *>(flow_lds)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  F fl(a, flow_lds, blockIdx.x);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wid < S * G) {  // sweep wid / G of row group wid % G
    const int s = wid / G, g = wid - s * G;
    if (s == 0) fl.template run_sor<0>(g, lane);
    else if (s == 1) fl.template run_sor<(S > 1 ? 1 : 0)>(g, lane);
    else if (s == 2) fl.template run_sor<(S > 2 ? 2 : 0)>(g, lane);
    else fl.template run_sor<(S > 3 ? 3 : 0)>(g, lane);
  } else if (wid < S * G + G) {
    fl.run_m(wid - S * G, lane);
  } else {
    const int k = wid - S * G - G, j = k / G, g = k - j * G;
    fl.run_y(g, j, lane);
  }
}

template <int NOP, int NOC, int S, int G, int P>
void launch_flow(const TvArgs &a, hipStream_t s) {
  using F = Flow<NOP, NOC, S, G, P>;
  static_assert(F::LDS <= 160 * 1024, "LDS");
  k_tv_flow<NOP, NOC, S, G, P><<<a.n, 64 * F::NW, F::LDS, s>>>(a);
}

template <int NOP, int NOC, int S>
bool flow_dispatch(const TvArgs &a, hipStream_t s, bool run) {
  if (a.h <= 64) {
    if (run) launch_flow<NOP, NOC, S, 1, 8>(a, s);
    return true;
  }
  if (a.h <= 128) {
    if (run) launch_flow<NOP, NOC, S, 2, 4>(a, s);
    return true;
  }
  return false;
}

template <int NOP, int NOC>
bool flow_dispatch_s(const TvArgs &a, hipStream_t s, bool run) {
  switch (a.solverit) {
    case 2: return flow_dispatch<NOP, NOC, 2>(a, s, run);
    case 3: return flow_dispatch<NOP, NOC, 3>(a, s, run);
    default: return false;
  }
}

bool flow_go(const TvArgs &a, hipStream_t s, bool run) {
  if (a.nop == 2) return a.noc == 1 ? flow_dispatch_s<2, 1>(a, s, run) : flow_dispatch_s<2, 3>(a, s, run);
  return a.noc == 1 ? flow_dispatch_s<1, 1>(a, s, run) : flow_dispatch_s<1, 3>(a, s, run);
}

}  // namespace

// The dataflow iteration runs where its rings fit: up to 128 rows (two row groups), 2 or 3 sweeps, the exact
// order (not the red-black mode, not the OpenMP build's point SOR), levels of at least 2 x 2 (solver.c's
// border forms) -- and the system kernels would read all eight derivative planes (no smsys_deriv).
bool tv_flow_ok(const TvArgs &a) {
  if (!a.tv_flow || a.sor_redblack || a.sor_point || a.sor_generic || a.sor_variant == 1) return false;
  if (a.w < 2 || a.h < 2) return false;
  return flow_go(a, nullptr, false);
}
void launch_tv_flow(const TvArgs &a, hipStream_t s) { flow_go(a, s, true); }

__device__ int g_flow_err;
int *tv_flow_err_counter() {
  void *p = nullptr;
  return hipGetSymbolAddress(&p, HIP_SYMBOL(g_flow_err)) == hipSuccess ? static_cast<int *>(p) : nullptr;
}
int tv_flow_err_take() {
  int v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_flow_err), sizeof(int)) != hipSuccess) return -1;
  const int z = 0;
  if (v && hipMemcpyToSymbol(HIP_SYMBOL(g_flow_err), &z, sizeof(int)) != hipSuccess) return -1;
  return v;
}

}  // namespace ofdis
