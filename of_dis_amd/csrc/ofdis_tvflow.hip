// ofdis_tvflow.hip -- one TV inner iteration (smoothness + system + exact-order SOR) as ONE dataflow launch.
//
// Reference: refine_variational.cpp:192-222 (the inner iteration), opticalflow_aux.c:77-132 (get_derivatives'
// second-order filters), :138-223,408-747 (compute_smoothness, compute_data / compute_data_DE, sub_laplacian),
// solver.c:83-433 / :439-471 (sor_coupled / the DE point SOR).  Same functions as the two-launch path
// (ofdis_tv_dev.inc), same operands, same order: the same bits.
//
// Why: the two-launch form writes 32 B of coefficients per pixel and inner iteration
// to HBM and reads them back, and in the latency regime (one pair per call, config D's 32 pairs per GPU) each of
// the 18 system launches of a 1080p pair costs ~10 us of a 0.84 ms chain.  Here one workgroup owns one frame's
// level for one inner iteration and every intermediate stays in LDS.  Its waves run free, each in its own role,
// and hand diagonals to each other through LDS rings guarded by per-wave progress counters -- not by workgroup
// barriers, so no wave waits for the slowest role's step, and the role whose work per diagonal is long (the
// system: ~12 correctly rounded divisions per pixel) runs on P waves round robin:
//
//   L (one wave): streams the level's skewed rows (diagonals) of wx, du (wy, dv) -- and, for intensity images,
//     the first derivatives Ix, Iy, Iz -- into the row ring by LDS-DMA (global_load_lds_dwordx4, one instruction
//     per plane row, two batches of rows in flight; no registers, so no compiler wait on a loop-carried prefetch);
//   M (one wave per row group g of 64 rows): the smoothness s of two diagonals per iteration (compute_smoothness
//     on uu = wx + du) into the s ring;
//   Y (P waves per row group): the system of diagonal d (diffusivities, data term -- with the second derivatives
//     filtered from the staged first ones --, sub_laplacian and, OF, the 2x2 inverse sor_coupled's first sweep
//     computes: sys_compute) into the coefficient ring, d = j mod P;
//   SOR (S waves per row group, wave = sweep s): sor_coupled's update of diagonal d = x + y for sweep s, as
//     k_tv_sor_lanes (pixel (x, y) of sweep s needs (x-1, y), (x, y-1) of sweep s and (x+1, y), (x, y+1) of sweep
//     s-1: diagonal order reproduces the lexicographic raster bit for bit); sweep 0 reads the old (du, dv) from
//     the row ring, the last sweep stores the new ones.
//
// Diagonal d of a w x h level holds pixels (d - y, y); its skewed plane row is d mod w (folded, h <= w) or d.
// LDS rings are [slot][plane][entry]: row ring entry y + 4 (16-byte aligned DMA target; entry 3 = row -1), the
// other rings entry y + 1.  Progress counters are LDS words; a poll reads them all in one round trip.
// Every wait is bounded: past kFlowSpinLimit polls a wave raises the abort word, every wave leaves its loop and
// the launch ends (counted in a.flow_err) -- a protocol error shows as a failed parity test, never as a hang.
#include "ofdis_internal.h"
#include "ofdis_math.h"

#include <utility>

#pragma clang fp contract(off)

namespace ofdis {
namespace {

#include "ofdis_tv_dev.inc"

constexpr int kFlowRR = 16;  // row ring slots (power of 2: per-lane filter taps index it with a mask)
constexpr int kFlowRS = 16;  // s ring slots
constexpr int kFlowRC = 12;  // coefficient ring slots: the system runs up to RC - 2 diagonals ahead of the last sweep
constexpr int kFlowD = 4;    // (u, v) ring slots per sweep
constexpr int kFlowLB = 4;   // rows per loader batch (two batches in flight)
constexpr int kFlowSpinLimit = 1 << 22;

// Progress counters live in LDS.  A wave's LDS instructions are performed in issue order, so (1) a counter store
// issued after the ring stores it publishes is seen after them, and (2) ring reads issued after the counter read
// (same round trip) see at least the state the counter showed: a poll that finds its counters ready has its
// operands too.  The empty asm keeps the compiler from reordering the LDS accesses across the counter access.
__device__ __forceinline__ int cnt_load(const int *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void cnt_publish(int *p, int v) {
  asm volatile("" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }
// s_waitcnt vmcnt(N) (gfx9 encoding: vmcnt bits 3:0 and 15:14; expcnt, lgkmcnt left at their maxima)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
// One LDS-DMA of 16 bytes per lane (global_load_lds_dwordx4: lane i's 16 bytes at src land at lds + 16 i).  Written
// as inline asm so that the compiler's wait-count pass does not see an LDS write in flight: through the builtin it
// waits for every outstanding vector-memory operation (vmcnt(0)) before each LDS access of the kernel, the progress
// polls included.  The loader waits for its own transfers explicitly (wait_vmcnt); M0 is set right before.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16(const float *src, unsigned lds_byte_addr) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_byte_addr) : "memory", "m0");
}
#pragma clang diagnostic pop
__device__ __forceinline__ unsigned lds_addr(const void *p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char *)p;
}

#ifdef OFDIS_FLOW_PROBE
// Probe build only (tools/flow_probe.py; never in libofdis.so): frame 0 of every launch records, per wave and
// loop iteration, the shader clock at the iteration's start, when its wait held and when it published, and the
// polls it took.  Layout: [0] launch counter, then [launch < 64][wave < 16][iteration < 256][4].
__device__ unsigned *g_flow_probe;
struct ProbeRec {
  unsigned *p = nullptr;
  unsigned t0 = 0, t1 = 0, spins = 0;
  __device__ __forceinline__ void start() {
    if (p) t0 = (unsigned)__builtin_amdgcn_s_memtime();
  }
  __device__ __forceinline__ void ready(unsigned sp) {
    if (p) {
      t1 = (unsigned)__builtin_amdgcn_s_memtime();
      spins = sp;
    }
  }
  __device__ __forceinline__ void done(int it) {
    if (p && it < 256 && (threadIdx.x & 63) == 0)
      *reinterpret_cast<uint4 *>(p + 4 * it) = make_uint4(t0, t1, (unsigned)__builtin_amdgcn_s_memtime(), spins);
  }
};
#define FLOW_PROBE(x) x
#else
#define FLOW_PROBE(x)
#endif

// NOP 2 (flow) / 1 (depth); NOC channels; S sweeps; NM smoothness waves; P system waves (levels of <= 64 rows:
// lane = row y).  DF (intensity images): the row ring also carries Ix, Iy, Iz and the system filters the second
// derivatives itself (k_tv_prepd then writes only Ix, Iy, Iz); RGB: the system reads the eight derivative planes
// from memory.
template <int NOP, int NOC, int S, int NM, int P>
struct Flow {
  static constexpr bool DF = NOC == 1;
  static constexpr int NR = 66;   // entries per slot of the s / coefficient / (u, v) rings (row y at y + 1)
  static constexpr int NRA = 72;  // entries per plane of the row ring (row y at y + 4; 16-byte multiple)
  static constexpr int CW = NOP == 2 ? 2 : 1;
  static constexpr int NPL = (NOP == 2 ? 4 : 2) + (DF ? 3 : 0);  // wx, du, (wy, dv), (Ix, Iy, Iz)
  static constexpr int PWX = 0, PDU = 1, PWY = 2, PDV = 3, PIX = NOP == 2 ? 4 : 2;
  static constexpr int NW = S + 1 + NM + P;
  static constexpr int C_SOR = 0, C_L = S, C_M = S + 1, C_Y = S + 1 + NM, C_ABORT = S + 1 + NM + P;
  static constexpr int NCNT = (C_ABORT + 1 + 3) / 4 * 4;
  static constexpr size_t OFF_ROW = 16 * NCNT;                                       // [RR][NPL][NRA] float
  static constexpr size_t OFF_COEF = OFF_ROW + sizeof(float) * kFlowRR * NPL * NRA;  // [RC][CW][NR] float4
  static constexpr size_t OFF_UV = OFF_COEF + sizeof(float4) * kFlowRC * CW * NR;    // [S][D][NR] f2v
  static constexpr size_t OFF_S = OFF_UV + sizeof(f2v) * S * kFlowD * NR;           // [RS][NR] float
  static constexpr size_t LDS = OFF_S + sizeof(float) * kFlowRS * NR;
  static constexpr int NDMA = kFlowLB * NPL;  // DMA instructions per loader batch

  // a copy: the fields live in scalar registers (a reference would make every LDS-order compiler barrier -- the
  // empty asm with a memory clobber -- force a kernel-argument reload, an SMEM round trip, in the loops)
  const TvArgs a;
  int *cnt;
  float *row;
  float4 *coef;
  f2v *uv;
  float *sr;
  int w, h, E, lim;
  unsigned f0;
  bool first;
#ifdef OFDIS_FLOW_PROBE
  ProbeRec pr;
#endif

  __device__ Flow(const TvArgs &a_, char *lds, int frame) : a(a_) {
    cnt = reinterpret_cast<int *>(lds);
    row = reinterpret_cast<float *>(lds + OFF_ROW);
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
  // row ring: the first entry of diagonal q's slot (any q >= -RR: slot q mod RR, a uniform offset)
  __device__ __forceinline__ const float *slot(int q) const { return row + (q & (kFlowRR - 1)) * NPL * NRA + 4; }

  // Poll until ok(C) holds, C(i) = counter i: lane i < NCNT reads counter i (one LDS round trip), the checks take
  // them by v_readlane.  false: the launch aborts.
  template <class F>
  __device__ __forceinline__ bool wait(F &&ok) {
    const int lane = threadIdx.x & 63;
    for (int spin = 0;; ++spin) {
      const int v = cnt_load(cnt + (lane < NCNT ? lane : 0));
      auto C = [&](int i) { return __builtin_amdgcn_readlane(v, i); };
      if (ok(C)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        FLOW_PROBE(pr.ready(spin));
        return true;
      }
      if (C(C_ABORT)) return false;
      if (spin > kFlowSpinLimit) {      // counted in a.flow_err at the end of the launch (no global memory op in
        cnt_publish(cnt + C_ABORT, 1);  // a poll loop: the compiler would wait for outstanding loads there)
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }

  // ------------------------------------------------------------------------------------------------ L
  // The plane rows of diagonal q (clamped to the last one) into its ring slot: lane i < ceil(h / 4) moves floats
  // 4i .. 4i + 3 of the skewed plane row (rows 4i .. 4i + 3 of the diagonal; the tail reads into the next plane
  // row or the plane's dump slots and is never used).
  __device__ __forceinline__ void dma_row(int q, int lane) const {
    const int qc = q < E ? q : E - 1;
    const unsigned o = f0 + (unsigned)(prow(qc) * h) + 4u * (unsigned)lane;
    const float *dst = slot(q);
    const float *src[NPL];
    src[PWX] = a.wxs;
    src[PDU] = a.du;
    if (NOP == 2) {
      src[PWY] = a.wys;
      src[PDV] = a.dv;
    }
    if (DF) {
      src[PIX] = a.Ix;
      src[PIX + 1] = a.Iy;
      src[PIX + 2] = a.Iz;
    }
    if (4 * lane < h) {
#pragma unroll
      for (int p = 0; p < NPL; ++p) dma16(src[p] + o, __builtin_amdgcn_readfirstlane(lds_addr(dst + p * NRA)));
    }
  }
  __device__ void run_l(int lane) {
    __builtin_amdgcn_s_setprio(2);
    // batch b = rows b LB .. b LB + LB - 1; two batches in flight: a batch is published once the next is issued
    const int nb = (E + kFlowLB - 1) / kFlowLB;
    for (int b = 0; b <= nb; ++b) {
      FLOW_PROBE(pr.start());
      if (b < nb) {
        const int rlast = b * kFlowLB + kFlowLB - 1;
        // WAR: row r replaces row r - RR, read last by the system of diagonal r - RR + 2 (filter taps d -+ 2):
        // sweep 0 past it
        if (!wait([&](auto &C) { return C(C_SOR) >= rlast - kFlowRR + 3; })) return;
#pragma unroll
        for (int k = 0; k < kFlowLB; ++k) dma_row(b * kFlowLB + k, lane);
        if (b > 0) wait_vmcnt<NDMA>();  // batch b - 1 has landed
      } else {
        wait_vmcnt<0>();
      }
      if (b > 0) {
        const int done = b * kFlowLB < E ? b * kFlowLB : E;
        cnt_publish(cnt + C_L, done);  // rows 0 .. done - 1 in the ring
      }
      FLOW_PROBE(pr.done(b));
    }
  }

  // ------------------------------------------------------------------------------------------------ M
  // s of diagonal e at row y (compute_smoothness on rows e - 1, e, e + 1; its replicate border takes the centre
  // for an absent neighbour: selected here by address, so each value is one read); 0 outside the level
  __device__ __forceinline__ float smooth_at(int e, int y) const {
    const int x = e - y;
    const float *c = slot(e) + y;
    const float *l = x > 0 ? slot(e - 1) + y : c;       // (x - 1, y)
    const float *r = x < w - 1 ? slot(e + 1) + y : c;   // (x + 1, y)
    const float *u = y > 0 ? slot(e - 1) + y - 1 : c;   // (x, y - 1)
    const float *dn = y < h - 1 ? slot(e + 1) + y + 1 : c;  // (x, y + 1)
    const float *q5[5] = {c, l, r, u, dn};
    float wx5[5], du5[5], wy5[5], dv5[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      wx5[k] = q5[k][PWX * NRA];
      du5[k] = q5[k][PDU * NRA];
      wy5[k] = NOP == 2 ? q5[k][PWY * NRA] : 0.0f;
      dv5[k] = NOP == 2 ? q5[k][PDV * NRA] : 0.0f;
    }
    const float sv = smooth_compute<NOP>(a, first, wx5, du5, wy5, dv5);
    return (unsigned)x < (unsigned)w && y < h ? sv : 0.0f;
  }
  __device__ void run_m(int m, int y) {
    __builtin_amdgcn_s_setprio(2);
    for (int e = m; e < E; e += NM) {
      FLOW_PROBE(pr.start());
      // rows <= e + 1 in the ring; WAR: s(e) replaces s(e - RS), read last by the system of diagonal e - RS + 1
      const int need = e + 2 < E ? e + 2 : E;
      if (!wait([&](auto &C) { return C(C_L) >= need && C(C_SOR) >= e - kFlowRS + 2; })) return;
      sr[(e % kFlowRS) * NR + y + 1] = smooth_at(e, y);
      cnt_publish(cnt + C_M + m, e + 1);  // s of this wave's diagonals <= e
      FLOW_PROBE(pr.done((e - m) / NM));
    }
  }

  // ------------------------------------------------------------------------------------------------ Y
  // get_derivatives' 5-tap filter (k_tv_deriv2 / k_tv_smsys<.., DF>'s expression) from the taps at offsets -2 .. 2
  // along one axis, replicate border: a tap past the border takes the border pixel's value, which is one of the
  // taps read (pos = the pixel's coordinate along the axis, n = the level's extent)
  __device__ __forceinline__ static float conv5_clamped(const float (&t)[5], int pos, int n) {
    const float m1 = pos >= 1 ? t[1] : t[2];
    const float m2 = pos >= 2 ? t[0] : m1;
    const float p1 = pos <= n - 2 ? t[3] : t[2];
    const float p2 = pos <= n - 3 ? t[4] : p1;
    return kK5[0] * m2 + ((kK5[1] * m1 + kK5[2] * t[2]) + (kK5[3] * p1 + kK5[4] * p2));
  }
  __device__ __forceinline__ bool y_step(int d, int j, int y) {
    FLOW_PROBE(pr.start());
    if (!wait([&](auto &C) {  // s(d - 1 .. d + 1); WAR: the coefficient slot's diagonal d - RC, read last at d - RC + 1
          bool ok = C(C_SOR + S - 1) >= d - kFlowRC + 2;
#pragma unroll
          for (int k = -1; k <= 1; ++k) {
            const int e = d + k;
            if (e >= 0 && e < E) ok = ok && C(C_M + e % NM) >= e + 1;
          }
          return ok;
        }))
      return false;
    const int x = d - y;
    const int sm = ((d + kFlowRS - 1) % kFlowRS) * NR, s0 = (d % kFlowRS) * NR, sp1 = ((d + 1) % kFlowRS) * NR;
    // centre, left (x - 1, y), right (x + 1, y), up (x, y - 1), down (x, y + 1)
    const float S5[5] = {sr[s0 + y + 1], sr[sm + y + 1], sr[sp1 + y + 1], sr[sm + y], sr[sp1 + y + 2]};
    const float *c = slot(d) + y, *pm = slot(d - 1) + y, *pp = slot(d + 1) + y;
    const float X5[5] = {c[PWX * NRA], pm[PWX * NRA], pp[PWX * NRA], pm[PWX * NRA - 1], pp[PWX * NRA + 1]};
    float Y5[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    if (NOP == 2) {
      const float t[5] = {c[PWY * NRA], pm[PWY * NRA], pp[PWY * NRA], pm[PWY * NRA - 1], pp[PWY * NRA + 1]};
#pragma unroll
      for (int k = 0; k < 5; ++k) Y5[k] = t[k];
    }
    const float u = c[PDU * NRA], v = NOP == 2 ? c[PDV * NRA] : 0.0f;
    const float m = warp_mask(x, y, X5[0], Y5[0], w, h);
    float lIx[NOC], lIy[NOC], lIz[NOC], lIxx[NOC], lIxy[NOC], lIyy[NOC], lIxz[NOC], lIyz[NOC];
    if constexpr (DF) {
      // taps (x + k, y): diagonal d + k, row y; (x, y + k): diagonal d + k, row y + k
      const float *q[5] = {slot(d - 2) + y, pm, c, pp, slot(d + 2) + y};
      float hX[5], vX[5], vY[5], hZ[5], vZ[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        hX[k] = q[k][PIX * NRA];
        vX[k] = q[k][PIX * NRA + k - 2];
        vY[k] = q[k][(PIX + 1) * NRA + k - 2];
        hZ[k] = q[k][(PIX + 2) * NRA];
        vZ[k] = q[k][(PIX + 2) * NRA + k - 2];
      }
      const int xc = (unsigned)x < (unsigned)w ? x : 0, yc = y < h ? y : 0;  // (lanes outside: any valid taps)
      lIx[0] = hX[2];
      lIy[0] = vY[2];
      lIz[0] = hZ[2];
      lIxx[0] = conv5_clamped(hX, xc, w);
      lIxy[0] = conv5_clamped(vX, yc, h);
      lIyy[0] = conv5_clamped(vY, yc, h);
      lIxz[0] = conv5_clamped(hZ, xc, w);
      lIyz[0] = conv5_clamped(vZ, yc, h);
    } else {
      const bool in = (unsigned)x < (unsigned)w && y < h;
      const unsigned o0 = f0 * (unsigned)NOC + (unsigned)(prow(d) * h) + (in ? (unsigned)y : 0u);
#pragma unroll
      for (int ch = 0; ch < NOC; ++ch) {
        const unsigned o = o0 + (unsigned)(ch * a.sp);
        lIx[ch] = ldu(a.Ix, o); lIy[ch] = ldu(a.Iy, o); lIz[ch] = ldu(a.Iz, o); lIxx[ch] = ldu(a.Ixx, o);
        lIxy[ch] = ldu(a.Ixy, o); lIyy[ch] = ldu(a.Iyy, o); lIxz[ch] = ldu(a.Ixz, o); lIyz[ch] = ldu(a.Iyz, o);
      }
    }
    float4 c0, c1;
    sys_compute<NOP, NOC>(a, x, y, S5, X5, Y5, m, u, v, lIx, lIy, lIz, lIxx, lIxy, lIyy, lIxz, lIyz, c0, c1);
    float4 *C = coef + (d % kFlowRC) * CW * NR + y + 1;
    C[0] = c0;
    if (NOP == 2) C[NR] = c1;
    cnt_publish(cnt + C_Y + j, d + 1);
    FLOW_PROBE(pr.done(d / P));
    return true;
  }
  __device__ void run_y(int j, int y) {
    __builtin_amdgcn_s_setprio(0);
    for (int d = j; d < E; d += P)
      if (!y_step(d, j, y)) return;
  }

  // ------------------------------------------------------------------------------------------------ SOR
  template <int SI>
  __device__ void run_sor(int y) {
    constexpr bool FIRST = SI == 0, LAST = SI == S - 1;
    constexpr int MODE = NOP == 2 ? 0 : 2;
    __builtin_amdgcn_s_setprio(3);
    const bool border = y == 0 || y >= h - 1, notop = y == 0;
    const float omega = a.omega;
    f2v pp = f2v{0.0f, 0.0f};  // own (u, v) of the previous diagonal (left neighbour; lane y + 1's top)
    float phr = 0.0f, pvv = 0.0f;
    f2v *ring_s = uv + SI * kFlowD * NR;
    const f2v *ring_p = uv + (SI > 0 ? SI - 1 : 0) * kFlowD * NR;
    for (int d = 0; d < E; ++d) {
      FLOW_PROBE(pr.start());
      const int dn = d + 2 < E ? d + 2 : E;
      const int x = d - y;
      const bool hasl = x > 0, hasr = x < w - 1;
      f2v o, rgt, bt;
      float4 c0, c1;
      // one LDS round trip per poll: the counters, then (in issue order) the operands -- valid once they hold
      for (int spin = 0;; ++spin) {
        const int v = cnt_load(cnt + (y < NCNT ? y : 0));
        lds_order();
        if (FIRST) {
          const float *r0 = slot(d) + y, *r1 = slot(d + 1) + y;
          o = f2v{r0[PDU * NRA], NOP == 2 ? r0[PDV * NRA] : 0.0f};
          rgt = f2v{r1[PDU * NRA], NOP == 2 ? r1[PDV * NRA] : 0.0f};
          bt = f2v{r1[PDU * NRA + 1], NOP == 2 ? r1[PDV * NRA + 1] : 0.0f};
        } else {
          o = ring_p[(d % kFlowD) * NR + y + 1];
          rgt = ring_p[((d + 1) % kFlowD) * NR + y + 1];
          bt = ring_p[((d + 1) % kFlowD) * NR + y + 2];
        }
        const float4 *Cp = coef + (d % kFlowRC) * CW * NR + y + 1;
        c0 = Cp[0];
        c1 = MODE == 0 ? Cp[NR] : c0;
        lds_order();
        auto C = [&](int i) { return __builtin_amdgcn_readlane(v, i); };
        // FIRST: the coefficients of d; later sweeps: the previous sweep's d + 1.  WAR (not the last sweep): this
        // ring slot's diagonal d - D is read by the next sweep as its own (at d - D) and right / bottom values
        // (at d - D - 1)
        bool ok = FIRST ? C(C_Y + d % P) >= d + 1 : C(C_SOR + SI - 1) >= dn;
        if (!LAST) ok = ok && C(C_SOR + SI + 1) >= d - kFlowD + 1;
        if (ok) {
          FLOW_PROBE(pr.ready(spin));
          break;
        }
        if (C(C_ABORT)) return;
        if (spin > kFlowSpinLimit) {
          cnt_publish(cnt + C_ABORT, 1);
          return;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      // the upper neighbour (x, y - 1) of this sweep: lane y - 1's result of the previous diagonal
      const f2v tp = f2v{dpp_from_prev_lane(pp.x), MODE == 0 ? dpp_from_prev_lane(pp.y) : 0.0f};
      const float tsv = dpp_from_prev_lane(pvv);
      f2v nw;
      float vv;
      if (MODE == 0) {
        const float hr = c1.z;
        vv = c1.w;
        const f2v bb = f2v{c1.x, c1.y};
        const f2v rrv = hasr ? rgt : f2v{0.0f, 0.0f};
        const f2v X = hr * rrv, Yv = tsv * tp, Z = vv * bt;
        // solver.c's three border expression trees (sor_rhs), lane-constant operand selects
        const f2v l = X + (border ? bb : Yv);
        const f2v rg = (border ? f2v{-0.0f, -0.0f} : bb) + (border ? (notop ? Z : Yv) : Z);
        const f2v srr = l + rg;
        const f2v Bv = hasl ? phr * pp + srr : srr;
        const f2v m_1 = f2v{c0.x, c0.y} * Bv.x, m_2 = f2v{c0.z, c0.w} * Bv.y;  // (i11,i12), (i12,i22)
        nw = o + omega * ((m_1 + m_2) - o);
        phr = hr;
      } else {
        const float a11 = c0.x, b1 = c0.y, hr = c0.z;
        vv = c0.w;
        const bool has_top = !notop, has_bot = !(border && has_top);
        const float tu = tp.x, ur = hasr ? rgt.x : 0.0f, hl = phr;
        float su = 0.0f;  // (a11 here is a11 + the diffusivities: sys_compute)
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
      cnt_publish(cnt + C_SOR + SI, d + 1);
      FLOW_PROBE(pr.done(d));
    }
  }
};

template <int NOP, int NOC, int S, int NM, int P>
__global__ __launch_bounds__((64 * Flow<NOP, NOC, S, NM, P>::NW)) void k_tv_flow(TvArgs a) {
  using F = Flow<NOP, NOC, S, NM, P>;
  extern __shared__ __attribute__((aligned(16))) char flow_lds[];
  // zero everything (counters, ring halos: the slots of rows -1 / h stay finite)
  for (int i = threadIdx.x; i < (int)(F::LDS / 16); i += blockDim.x)
    reinterpret_cast<float4 *>(flow_lds)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  F fl(a, flow_lds, blockIdx.x);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
#ifdef OFDIS_FLOW_PROBE
  {
    __shared__ unsigned slot;
    if (threadIdx.x == 0) slot = (blockIdx.x == 0 && g_flow_probe) ? atomicAdd(g_flow_probe, 1u) : 64u;
    __syncthreads();
    if (slot < 64u && wid < 16) fl.pr.p = g_flow_probe + 4 + ((size_t)slot * 16 + wid) * 256 * 4;
  }
#endif
  if (wid < S) {  // sweep wid
    if (wid == 0) fl.template run_sor<0>(lane);
    else if (wid == 1) fl.template run_sor<(S > 1 ? 1 : 0)>(lane);
    else if (wid == 2) fl.template run_sor<(S > 2 ? 2 : 0)>(lane);
    else fl.template run_sor<(S > 3 ? 3 : 0)>(lane);
  } else if (wid == S) {
    fl.run_l(lane);
  } else if (wid < S + 1 + NM) {
    fl.run_m(wid - S - 1, lane);
  } else {
    fl.run_y(wid - S - 1 - NM, lane);
  }
  __syncthreads();  // every role has left its loop (each wait is bounded)
  if (threadIdx.x == 0 && cnt_load(fl.cnt + F::C_ABORT) && a.flow_err) atomicAdd(a.flow_err, 1);
}

template <int NOP, int NOC, int S>
void launch_flow(const TvArgs &a, hipStream_t s) {
  constexpr int NM = 3, P = 12 - S;  // 16 waves
  using F = Flow<NOP, NOC, S, NM, P>;
  static_assert(F::LDS <= 160 * 1024, "LDS");
  static_assert(F::NW <= 16, "one workgroup of at most 1024 threads");
  static_assert(2 * F::NDMA < 64, "loader batches in flight");
  k_tv_flow<NOP, NOC, S, NM, P><<<a.n, 64 * F::NW, F::LDS, s>>>(a);
}

template <int NOP, int NOC>
bool flow_dispatch_s(const TvArgs &a, hipStream_t s, bool run) {
  if (a.h > 64) return false;
  switch (a.solverit) {
    case 2:
      if (run) launch_flow<NOP, NOC, 2>(a, s);
      return true;
    case 3:
      if (run) launch_flow<NOP, NOC, 3>(a, s);
      return true;
    default: return false;
  }
}

bool flow_go(const TvArgs &a, hipStream_t s, bool run) {
  if (a.nop == 2) return a.noc == 1 ? flow_dispatch_s<2, 1>(a, s, run) : flow_dispatch_s<2, 3>(a, s, run);
  return a.noc == 1 ? flow_dispatch_s<1, 1>(a, s, run) : flow_dispatch_s<1, 3>(a, s, run);
}

// ==================================================================================================== SOR only
// k_tv_sorflow: the exact-order SOR call (solver.c:83-433 / :439-471) of one frame's level, the system computed
// by the system launch as before, with the sweep-per-wave schedule of k_tv_sor_lanes run barrier-free: the sweep
// waves (S per 64-row group, G <= 2 groups) and one loader wave hand diagonals to each other through LDS rings and
// progress counters, as in k_tv_flow.  The loader streams each diagonal's coefficients (the system launch's
// array-of-structs row) and the old (du, dv) rows into the rings by LDS-DMA, several rows ahead.  A sweep wave
// thus waits only for the two waves it depends on (the previous sweep, the group above) -- not for every wave of
// the workgroup at a barrier -- and never for a global load.  Same update expressions as k_tv_sor_lanes.
constexpr int kSfRC = 8;   // coefficient ring slots
constexpr int kSfRR = 8;   // (du, dv) row ring slots (power of 2)
constexpr int kSfD = 4;    // (u, v) ring slots per sweep
constexpr int kSfLB = 2;   // rows per loader batch (two batches in flight)

template <int S, int MODE, int G>
struct SorFlow {
  static constexpr int CW = MODE == 0 ? 2 : 1;
  static constexpr int NR = 64 * G + 2;   // (u, v) ring entries per slot (row y at y + 1)
  static constexpr int NRA = 64 * G + 8;  // (du, dv) ring entries per plane (row y at y + 4)
  static constexpr int NCR = 64 * G * CW; // coefficient ring float4 per slot (row y at y CW)
  static constexpr int NPL = MODE == 0 ? 2 : 1;
  static constexpr int NW = S * G + 1;
  static constexpr int C_SOR = 0, C_L = S * G, C_ABORT = S * G + 1;
  static constexpr int NCNT = (C_ABORT + 1 + 3) / 4 * 4;
  static constexpr size_t OFF_COEF = 16 * NCNT;                                    // [RC][NCR] float4
  static constexpr size_t OFF_DU = OFF_COEF + sizeof(float4) * kSfRC * NCR;          // [RR][NPL][NRA] float
  static constexpr size_t OFF_UV = OFF_DU + sizeof(float) * kSfRR * NPL * NRA;       // [S][D][NR] f2v
  static constexpr size_t LDS = OFF_UV + sizeof(f2v) * S * kSfD * NR;
  // DMA instructions per row: coefficients 16 h CW bytes (1 KiB each), du / dv h floats each
  static constexpr int NDMA_ROW = (NCR * 16 + 1023) / 1024 + NPL;

  const TvArgs a;
  int *cnt;
  float4 *coef;
  float *dur;
  f2v *uv;
  int w, h, E, lim;
  unsigned f0;

  __device__ SorFlow(const TvArgs &a_, char *lds, int frame) : a(a_) {
    cnt = reinterpret_cast<int *>(lds);
    coef = reinterpret_cast<float4 *>(lds + OFF_COEF);
    dur = reinterpret_cast<float *>(lds + OFF_DU);
    uv = reinterpret_cast<f2v *>(lds + OFF_UV);
    w = a.w;
    h = a.h;
    E = a.w + a.h - 1;
    lim = a.wrap ? a.w : 1 << 30;
    f0 = (unsigned)((long)frame * a.sp);
  }
  __device__ __forceinline__ int prow(int d) const { return d >= lim ? d - lim : d; }
  __device__ __forceinline__ const float *du_slot(int q) const { return dur + (q & (kSfRR - 1)) * NPL * NRA + 4; }

  // loader: diagonal q's coefficient row (16 h CW contiguous bytes) and old du (dv) rows into the ring slots
  __device__ __forceinline__ void dma_row(int q, int lane) const {
    const int qc = q < E ? q : E - 1;
    const unsigned pr = (unsigned)(prow(qc) * h);
    const char *csrc = reinterpret_cast<const char *>(a.coef) + (size_t)(f0 + pr) * CW * 16;
    const unsigned cdst = lds_addr(coef + (q % kSfRC) * NCR);
    // every DMA instruction is issued by every batch (the loader's vmcnt waits count them): all lanes move 16
    // bytes, those past the row re-read its start into slot entries of rows >= h (never read)
    const int cbytes = h * CW * 16;
#pragma unroll
    for (int k = 0; k < (NCR * 16 + 1023) / 1024; ++k) {
      const int off = 1024 * k + 16 * lane;
      dma16(reinterpret_cast<const float *>(csrc + (off < cbytes ? off : 0)), __builtin_amdgcn_readfirstlane(cdst + 1024 * k));
    }
    if (lane < 16 * G) {  // (du, dv): 4 floats per lane, rows 0 .. 64 G - 1 of the slot (lane 0 always issues)
      const float *d = du_slot(q);
      const unsigned lo = 4 * lane < h ? 4u * (unsigned)lane : 0u;
      dma16(a.du + f0 + pr + lo, __builtin_amdgcn_readfirstlane(lds_addr(d)));
      if (MODE == 0) dma16(a.dv + f0 + pr + lo, __builtin_amdgcn_readfirstlane(lds_addr(d + NRA)));
    }
  }
  template <class F>
  __device__ __forceinline__ bool wait(F &&ok) {
    const int lane = threadIdx.x & 63;
    for (int spin = 0;; ++spin) {
      const int v = cnt_load(cnt + (lane < NCNT ? lane : 0));
      auto C = [&](int i) { return __builtin_amdgcn_readlane(v, i); };
      if (ok(C)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        return true;
      }
      if (C(C_ABORT)) return false;
      if (spin > kFlowSpinLimit) {
        cnt_publish(cnt + C_ABORT, 1);
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  template <class CF>
  __device__ __forceinline__ static int cmin(CF &C, int base) {
    int m = C(base);
#pragma unroll
    for (int g = 1; g < G; ++g) m = min(m, C(base + g));
    return m;
  }
  __device__ void run_l(int lane) {
    __builtin_amdgcn_s_setprio(2);
    const int nb = (E + kSfLB - 1) / kSfLB;
    for (int b = 0; b <= nb; ++b) {
      if (b < nb) {
        const int rlast = b * kSfLB + kSfLB - 1;
        // WAR: coefficient slot of diagonal r - RC, read last by the last sweep (and lane 0's upper sv at
        // r - RC + 1); (du, dv) row r - RR, read last by sweep 0 at diagonal r - RR
        if (!wait([&](auto &C) {
              return cmin(C, C_SOR + (S - 1) * G) >= rlast - kSfRC + 2 && cmin(C, C_SOR) >= rlast - kSfRR + 1;
            }))
          return;
#pragma unroll
        for (int k = 0; k < kSfLB; ++k) dma_row(b * kSfLB + k, lane);
        if (b > 0) wait_vmcnt<kSfLB * NDMA_ROW>();  // batch b - 1 has landed (lanes without a row issue fewer)
      } else {
        wait_vmcnt<0>();
      }
      if (b > 0) cnt_publish(cnt + C_L, b * kSfLB < E ? b * kSfLB : E);  // rows 0 .. b LB - 1 in the rings
    }
  }

  template <int SI>
  __device__ void run_sor(int g, int lane) {
    constexpr bool FIRST = SI == 0, LAST = SI == S - 1;
    __builtin_amdgcn_s_setprio(3);
    const int y = 64 * g + lane;
    const bool border = y == 0 || y >= h - 1, notop = y == 0;
    const bool top_lds = lane == 0 && g > 0;
    const float omega = a.omega;
    f2v pp = f2v{0.0f, 0.0f};
    float phr = 0.0f, pvv = 0.0f;
    f2v *ring_s = uv + SI * kSfD * NR;
    const f2v *ring_p = uv + (SI > 0 ? SI - 1 : 0) * kSfD * NR;
    for (int d = 0; d < E; ++d) {
      const int dn = d + 2 < E ? d + 2 : E;
      const int x = d - y;
      const bool hasl = x > 0, hasr = x < w - 1;
      const int dm = (d + kSfD - 1) % kSfD, cm = (d + kSfRC - 1) % kSfRC;
      f2v o, rgt, bt, tpl = f2v{0.f, 0.f};
      float4 c0, c1;
      float tsvl = 0.f;
      for (int spin = 0;; ++spin) {
        const int v = cnt_load(cnt + (lane < NCNT ? lane : 0));
        lds_order();
        if (FIRST) {
          const float *r0 = du_slot(d) + y, *r1 = du_slot(d + 1) + y;
          o = f2v{r0[0], MODE == 0 ? r0[NRA] : 0.0f};
          rgt = f2v{r1[0], MODE == 0 ? r1[NRA] : 0.0f};
          bt = f2v{r1[1], MODE == 0 ? r1[NRA + 1] : 0.0f};
        } else {
          o = ring_p[(d % kSfD) * NR + y + 1];
          rgt = ring_p[((d + 1) % kSfD) * NR + y + 1];
          bt = ring_p[((d + 1) % kSfD) * NR + y + 2];
        }
        const float4 *Cp = coef + (d % kSfRC) * NCR + y * CW;
        c0 = Cp[0];
        c1 = MODE == 0 ? Cp[1] : c0;
        if (G > 1) {  // lane 0 of a lower row group: the row above is the group above's
          tpl = ring_s[dm * NR + y];
          tsvl = coef[cm * NCR + (y - 1) * CW + CW - 1].w;
        }
        lds_order();
        auto C = [&](int i) { return __builtin_amdgcn_readlane(v, i); };
        bool ok;
        if (FIRST) {
          ok = C(C_L) >= dn;  // the coefficients of d, the old rows d and d + 1
        } else {
          ok = C(C_SOR + (SI - 1) * G + g) >= dn;
          if (G > 1 && g + 1 < G) ok = ok && C(C_SOR + (SI - 1) * G + g + 1) >= dn;
        }
        if (G > 1 && g > 0) ok = ok && C(C_SOR + SI * G + g - 1) >= d;  // top of lane 0: diagonal d - 1
        if (!LAST) {
          ok = ok && C(C_SOR + (SI + 1) * G + g) >= d - kSfD + 1;
          if (G > 1 && g > 0) ok = ok && C(C_SOR + (SI + 1) * G + g - 1) >= d - kSfD;
        }
        if (G > 1 && g + 1 < G) ok = ok && C(C_SOR + SI * G + g + 1) >= d - kSfD + 2;
        if (ok) break;
        if (C(C_ABORT)) return;
        if (spin > kFlowSpinLimit) {
          cnt_publish(cnt + C_ABORT, 1);
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
        const f2v rrv = hasr ? rgt : f2v{0.0f, 0.0f};
        const f2v X = hr * rrv, Yv = tsv * tp, Z = vv * bt;
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
      ring_s[(d % kSfD) * NR + y + 1] = nw;
      if (LAST && (unsigned)x < (unsigned)w && y < h) {
        const unsigned oo = f0 + (unsigned)(prow(d) * h + y);
        *reinterpret_cast<float *>(reinterpret_cast<char *>(a.du) + (size_t)oo * 4u) = nw.x;
        if (MODE == 0) *reinterpret_cast<float *>(reinterpret_cast<char *>(a.dv) + (size_t)oo * 4u) = nw.y;
      }
      pp = nw;
      pvv = vv;
      cnt_publish(cnt + C_SOR + SI * G + g, d + 1);
    }
  }
};

template <int S, int MODE, int G>
__global__ __launch_bounds__((64 * SorFlow<S, MODE, G>::NW)) void k_tv_sorflow(TvArgs a) {
  using F = SorFlow<S, MODE, G>;
  extern __shared__ __attribute__((aligned(16))) char sf_lds[];
  for (int i = threadIdx.x; i < (int)(F::LDS / 16); i += blockDim.x)
    reinterpret_cast<float4 *>(sf_lds)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  F fl(a, sf_lds, blockIdx.x);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wid < S * G) {
    const int s = wid / G, g = wid - s * G;
    if (s == 0) fl.template run_sor<0>(g, lane);
    else if (s == 1) fl.template run_sor<(S > 1 ? 1 : 0)>(g, lane);
    else if (s == 2) fl.template run_sor<(S > 2 ? 2 : 0)>(g, lane);
    else fl.template run_sor<(S > 3 ? 3 : 0)>(g, lane);
  } else {
    fl.run_l(lane);
  }
  __syncthreads();
  if (threadIdx.x == 0 && cnt_load(fl.cnt + F::C_ABORT) && a.flow_err) atomicAdd(a.flow_err, 1);
}

template <int S, int MODE, int G>
void launch_sorflow(const TvArgs &a, hipStream_t s) {
  using F = SorFlow<S, MODE, G>;
  static_assert(F::LDS <= 64 * 1024, "LDS");
  static_assert(2 * kSfLB * F::NDMA_ROW < 64, "loader batches in flight");
  k_tv_sorflow<S, MODE, G><<<a.n, 64 * F::NW, F::LDS, s>>>(a);
}
template <int S, int MODE>
bool sorflow_s(const TvArgs &a, hipStream_t s, bool run) {
  if (a.h <= 64) {
    if (run) launch_sorflow<S, MODE, 1>(a, s);
    return true;
  }
  if (a.h <= 128) {
    if (run) launch_sorflow<S, MODE, 2>(a, s);
    return true;
  }
  return false;
}
bool sorflow_go(const TvArgs &a, hipStream_t s, bool run) {
  const int mode = a.nop == 2 ? 0 : 2;
  switch (a.solverit) {
    case 2: return mode == 0 ? sorflow_s<2, 0>(a, s, run) : sorflow_s<2, 2>(a, s, run);
    case 3: return mode == 0 ? sorflow_s<3, 0>(a, s, run) : sorflow_s<3, 2>(a, s, run);
    default: return false;
  }
}

// ================================================================================== SOR, barriers + LDS-DMA
// k_tv_sordma: the exact-order SOR call (solver.c:83-433 / :439-471) of one frame's level in the latency regime
// (a launch of at most one frame per CU).  The sweep-per-wave schedule of k_tv_sor_lanes -- sweep s of row group g
// is one wave, pixel (x, y) of sweep s at wavefront step x + y + 2 s, one workgroup barrier per step -- but sweep 0
// never waits on a global load: a loader wave streams every diagonal's coefficient row (the system launch's
// array-of-structs row) and old (du, dv) rows into LDS rings by LDS-DMA, kDmLA rows ahead, and waits for the rows
// the next step needs (explicit vmcnt) before the barrier that publishes them.  The sweeps read everything from the
// rings; same update expressions as k_tv_sor_lanes / k_tv_sorflow, same bits.
constexpr int kDmLA = 6;   // rows the loader runs ahead of sweep 0
constexpr int kDmRC = 14;  // coefficient ring slots: > kDmLA + 2 S + 1 (a slot is rewritten only after its last read)
constexpr int kDmRR = 16;  // (du, dv) row ring slots (power of 2): > kDmLA + 2

template <int S, int MODE, int G>
struct SorDma {
  static constexpr int CW = MODE == 0 ? 2 : 1;
  static constexpr int NPL = MODE == 0 ? 2 : 1;
  static constexpr int NR = 64 * G + 2;    // (u, v) ring entries per slot (row y at y + 1)
  static constexpr int NRA = 64 * G + 8;   // (du, dv) ring entries per plane (row y at y + 4)
  static constexpr int NCR = 64 * G * CW;  // coefficient ring float4 per slot (row y at y CW)
  static constexpr int D = 4;              // (u, v) ring slots per sweep
  static constexpr int NW = S * G + 1;
  static constexpr size_t OFF_COEF = 0;
  static constexpr size_t OFF_DU = OFF_COEF + sizeof(float4) * kDmRC * NCR;
  static constexpr size_t OFF_UV = OFF_DU + sizeof(float) * kDmRR * NPL * NRA;
  static constexpr size_t LDS = OFF_UV + sizeof(f2v) * S * D * NR;
  static constexpr int NDMA_ROW = (NCR * 16 + 1023) / 1024 + NPL;  // DMA instructions per row
  static_assert(kDmRC > kDmLA + 2 * S + 1 && kDmRR > kDmLA + 2, "ring slots");

  const TvArgs a;
  float4 *coef;
  float *dur;
  f2v *uv;
  int w, h, E, lim;
  unsigned f0;

  __device__ SorDma(const TvArgs &a_, char *lds, int frame) : a(a_) {
    coef = reinterpret_cast<float4 *>(lds + OFF_COEF);
    dur = reinterpret_cast<float *>(lds + OFF_DU);
    uv = reinterpret_cast<f2v *>(lds + OFF_UV);
    w = a.w;
    h = a.h;
    E = a.w + a.h - 1;
    lim = a.wrap ? a.w : 1 << 30;
    f0 = (unsigned)((long)frame * a.sp);
  }
  __device__ __forceinline__ int prow(int d) const { return d >= lim ? d - lim : d; }
  __device__ __forceinline__ const float *du_slot(int q) const { return dur + (q & (kDmRR - 1)) * NPL * NRA + 4; }

  // diagonal q's coefficient row (16 h CW contiguous bytes) and old (du, dv) rows into their ring slots; rows past
  // the last diagonal re-read the last one (never used).  Every DMA instruction issues (lane 0 always has work), so
  // the loader's vmcnt waits count them exactly.
  __device__ __forceinline__ void dma_row(int q, int lane) const {
    const int qc = q < E ? q : E - 1;
    const unsigned pr = (unsigned)(prow(qc) * h);
    const char *csrc = reinterpret_cast<const char *>(a.coef) + (size_t)(f0 + pr) * CW * 16;
    const unsigned cdst = lds_addr(coef + (q % kDmRC) * NCR);
    const int cbytes = h * CW * 16;
#pragma unroll
    for (int k = 0; k < (NCR * 16 + 1023) / 1024; ++k) {
      const int off = 1024 * k + 16 * lane;
      dma16(reinterpret_cast<const float *>(csrc + (off < cbytes ? off : 0)), __builtin_amdgcn_readfirstlane(cdst + 1024 * k));
    }
    if (lane < 16 * G) {
      const float *d = du_slot(q);
      const unsigned lo = 4 * lane < h ? 4u * (unsigned)lane : 0u;
      dma16(a.du + f0 + pr + lo, __builtin_amdgcn_readfirstlane(lds_addr(d)));
      if (MODE == 0) dma16(a.dv + f0 + pr + lo, __builtin_amdgcn_readfirstlane(lds_addr(d + NRA)));
    }
  }

  // T steps; at the barrier ending step t the rows <= t + 2 have landed (sweep 0 at step t + 1 reads rows t + 1
  // and t + 2), rows t + 3 .. t + kDmLA + 1 may still be in flight
  __device__ void run_l(int lane, int T) {
    for (int q = 0; q <= kDmLA; ++q) dma_row(q, lane);
    wait_vmcnt<(kDmLA - 1) * NDMA_ROW>();
    __syncthreads();
    for (int t = 0; t < T; ++t) {
      dma_row(t + kDmLA + 1, lane);
      wait_vmcnt<(kDmLA - 1) * NDMA_ROW>();
      __syncthreads();
    }
    wait_vmcnt<0>();
  }

  template <int SI>
  __device__ void run_sor(int g, int lane, int T) {
    constexpr bool FIRST = SI == 0, LAST = SI == S - 1;
    const int y = 64 * g + lane;
    const bool border = y == 0 || y >= h - 1, notop = y == 0;
    const bool top_lds = lane == 0 && g > 0;
    const float omega = a.omega;
    f2v pp = f2v{0.0f, 0.0f};
    float phr = 0.0f, pvv = 0.0f;
    f2v *ring_s = uv + SI * D * NR;
    const f2v *ring_p = uv + (SI > 0 ? SI - 1 : 0) * D * NR;
    __syncthreads();  // the loader's prologue
    for (int t = 0; t < T; ++t) {
      const int d = t - 2 * SI;
      if (d >= 0 && d < E) {
        const int x = d - y;
        const bool hasl = x > 0, hasr = x < w - 1;
        const int dm = (d + D - 1) % D, cm = (d + kDmRC - 1) % kDmRC;
        f2v o, rgt, bt, tpl = f2v{0.f, 0.f};
        float tsvl = 0.f;
        if (FIRST) {
          const float *r0 = du_slot(d) + y, *r1 = du_slot(d + 1) + y;
          o = f2v{r0[0], MODE == 0 ? r0[NRA] : 0.0f};
          rgt = f2v{r1[0], MODE == 0 ? r1[NRA] : 0.0f};
          bt = f2v{r1[1], MODE == 0 ? r1[NRA + 1] : 0.0f};
        } else {
          o = ring_p[(d % D) * NR + y + 1];
          rgt = ring_p[((d + 1) % D) * NR + y + 1];
          bt = ring_p[((d + 1) % D) * NR + y + 2];
        }
        const float4 *Cp = coef + (d % kDmRC) * NCR + y * CW;
        const float4 c0 = Cp[0];
        const float4 c1 = MODE == 0 ? Cp[1] : c0;
        if (G > 1) {  // lane 0 of a lower row group: the row above is the group above's
          tpl = ring_s[dm * NR + y];
          tsvl = coef[cm * NCR + (y - 1) * CW + CW - 1].w;
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
          const f2v rrv = hasr ? rgt : f2v{0.0f, 0.0f};
          const f2v X = hr * rrv, Yv = tsv * tp, Z = vv * bt;
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
        ring_s[(d % D) * NR + y + 1] = nw;
        if (LAST && (unsigned)x < (unsigned)w && y < h) {
          const unsigned oo = f0 + (unsigned)(prow(d) * h + y);
          *reinterpret_cast<float *>(reinterpret_cast<char *>(a.du) + (size_t)oo * 4u) = nw.x;
          if (MODE == 0) *reinterpret_cast<float *>(reinterpret_cast<char *>(a.dv) + (size_t)oo * 4u) = nw.y;
        }
        pp = nw;
        pvv = vv;
      }
      __syncthreads();
    }
  }
};

template <int S, int MODE, int G>
__global__ __launch_bounds__((64 * SorDma<S, MODE, G>::NW)) void k_tv_sordma(TvArgs a) {
  using F = SorDma<S, MODE, G>;
  extern __shared__ __attribute__((aligned(16))) char sd_lds[];
  for (int i = threadIdx.x; i < (int)(F::LDS / 16); i += blockDim.x)
    reinterpret_cast<float4 *>(sd_lds)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  F fl(a, sd_lds, blockIdx.x);
  const int T = fl.E + 2 * (S - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wid < S * G) {
    const int s = wid / G, g = wid - s * G;
    if (s == 0) fl.template run_sor<0>(g, lane, T);
    else if (s == 1) fl.template run_sor<(S > 1 ? 1 : 0)>(g, lane, T);
    else if (s == 2) fl.template run_sor<(S > 2 ? 2 : 0)>(g, lane, T);
    else fl.template run_sor<(S > 3 ? 3 : 0)>(g, lane, T);
  } else {
    fl.run_l(lane, T);
  }
}

template <int S, int MODE, int G>
void launch_sordma(const TvArgs &a, hipStream_t s) {
  using F = SorDma<S, MODE, G>;
  static_assert(F::LDS <= 160 * 1024, "LDS");
  static_assert(kDmLA * F::NDMA_ROW < 64, "loader rows in flight");
  k_tv_sordma<S, MODE, G><<<a.n, 64 * F::NW, F::LDS, s>>>(a);
}
template <int S, int MODE>
bool sordma_s(const TvArgs &a, hipStream_t s, bool run) {
  if (a.h <= 64) {
    if (run) launch_sordma<S, MODE, 1>(a, s);
    return true;
  }
  if (a.h <= 128) {
    if (run) launch_sordma<S, MODE, 2>(a, s);
    return true;
  }
  return false;
}
bool sordma_go(const TvArgs &a, hipStream_t s, bool run) {
  const int mode = a.nop == 2 ? 0 : 2;
  switch (a.solverit) {
    case 2: return mode == 0 ? sordma_s<2, 0>(a, s, run) : sordma_s<2, 2>(a, s, run);
    case 3: return mode == 0 ? sordma_s<3, 0>(a, s, run) : sordma_s<3, 2>(a, s, run);
    default: return false;
  }
}

}  // namespace

// The dataflow iteration runs where its rings fit: up to 64 rows (lane = row), 2 or 3 sweeps, the
// exact order (not the red-black mode, not the OpenMP build's point SOR), levels of at least 2 x 2 (solver.c's
// border forms); intensity images also need k_tv_prepd (it writes the Ix, Iy, Iz the loader streams).
bool tv_flow_ok(const TvArgs &a) {
  if (!a.tv_flow || a.sor_redblack || a.sor_point || a.sor_generic || a.sor_variant == 1) return false;
  if (a.w < 2 || a.h < 2) return false;
  if (a.noc == 1 && !tv_prepd_ok(a)) return false;
  return flow_go(a, nullptr, false);
}
void launch_tv_flow(const TvArgs &a, hipStream_t s) { flow_go(a, s, true); }

// The barrier SOR fed by LDS-DMA: exact order, 2 or 3 sweeps, 2 .. 128 rows (option sor_dma).
bool tv_sordma_ok(const TvArgs &a) {
  if (!a.sor_dma || a.sor_redblack || a.sor_point || a.sor_generic || a.sor_variant == 1) return false;
  if (a.w < 2 || a.h < 2) return false;
  return sordma_go(a, nullptr, false);
}
void launch_tv_sordma(const TvArgs &a, hipStream_t s) { sordma_go(a, s, true); }

// The barrier-free SOR: exact order, 2 or 3 sweeps, 2 .. 128 rows (option sor_flow); the system launch runs first.
bool tv_sorflow_ok(const TvArgs &a) {
  if (!a.sor_flow || a.sor_redblack || a.sor_point || a.sor_generic || a.sor_variant == 1) return false;
  if (a.w < 2 || a.h < 2) return false;
  return sorflow_go(a, nullptr, false);
}
void launch_tv_sorflow(const TvArgs &a, hipStream_t s) { sorflow_go(a, s, true); }

__device__ int g_flow_err;
#ifdef OFDIS_FLOW_PROBE
extern "C" int ofdis_flow_probe_attach(void *dev_buffer) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_flow_probe), &dev_buffer, sizeof(dev_buffer)) == hipSuccess ? 0 : -1;
}
#endif
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
