// ofdis_runtime.cpp -- contexts, device workspace planning and the coarse-to-fine driver
// (the OFClass constructor, oflow.cpp:31-338, restated for batches of frame pairs on one MI355X).
//
// One context per GPU.  A batch of n frame pairs is processed level by level; every kernel carries
// the frame index in its grid, so even the 30x17 coarsest level of a 1080p frame fills the chip when
// n is large.  All launches go to one stream; nothing synchronises the host unless a capture, the
// verbosity timers or a host-buffer entry point asks for it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ofdis.h"
#include "ofdis_internal.h"

using namespace ofdis;

namespace {

const char *const kKernelNames[] = {"pyr_base", "pyr_down", "pyr_pad_grad", "patch",    "aggregate", "tv_prep",
                                    "tv_deriv", "tv_system", "tv_sor",       "tv_final", "upsample",  "tv_level"};

struct Plan {
  int n = 0, W0 = 0, H0 = 0, Wp = 0, Hp = 0, padl = 0, padt = 0, padw = 0, padh = 0;
  int nop = 2, noc = 1, pad = 8, sc_f = 0, sc_l = 0;
  std::vector<LevelGeom> lv;                       // index s - sc_l
  std::vector<size_t> off_lvl, off_img, off_dx, off_dy, off_flow, off_flow_bw;
  size_t off_piter = 0, off_pw = 0, off_piter_bw = 0, off_pw_bw = 0, off_tv = 0, tv_plane = 0;
  size_t off_init = 0;  // initial flow at the coarsest scale - 1, [n][Hp >> (sc_f+1)][Wp >> (sc_f+1)][nop]
  bool init = false;    // an initial flow is given: divisibility 2^(sc_f+1) (run_dense.cpp:302)
  bool fb = false;      // usefbcon: backward grid, flow and refinement
  bool gradmag = false; // SELECTCHANNEL 2: float level 0 (gradient magnitude) halved down to sc_l
  size_t off_gm = 0;    // its scratch: [2n][Hp][Wp] + [2n][Hp/2][Wp/2] (ping-pong)
  size_t total = 0;
};

inline size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

// Skewed TV plane: w * h slots when the anti-diagonal rows fold modulo w (h <= w), else (w + h - 1) * h,
// plus 64 per-lane dump slots for the SOR kernels; a multiple of 4 floats (16-byte AoS coefficients).
inline long skew_plane(int w, int h) {
  const long slots = h <= w ? (long)w * h : (long)(w + h - 1) * h;
  return (slots + 64 + 3) / 4 * 4;
}

}  // namespace

struct ofdis_context {
  int device = 0;
  hipStream_t stream = nullptr;
  char *ws = nullptr;
  size_t ws_cap = 0;
  // stage capture (frame 0), indexed by scale
  std::vector<float *> cap_dis, cap_tv;
  // kernel timing
  bool timing = false;
  struct Pending {
    int kernel;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
  std::map<int, std::pair<double, long>> acc;
  int opt_sor_generic = 0;
  int opt_sor_pipe = 0;  // 1: force the single-wave-per-row-group register pipeline (A/B)
  int opt_graph = 1;           // replay the whole batch as one HIP graph (captured once per shape / pointers)
  struct GraphKey {
    const void *a = nullptr, *b = nullptr, *out = nullptr, *ws = nullptr, *init = nullptr;
    int n = 0, w = 0, h = 0;
    ofdis_params p{};
  } gkey;
  hipGraphExec_t gexec = nullptr;
  int opt_nt_store = 0;        // upsample output with non-temporal stores (A/B)
  // flow upsample: 0 per-output-row horizontal taps (k_upsample_rows), 1 / 2 once per staged source row (k_upsample_h,
  // 4 / 8 rows), 3 auto: 1 when the frame spans a whole 1024-column block and the call runs on two or more lanes or
  // has fewer than 1024 pairs, else 0 -- measured end to end, alternating on one box each (profiles/r05/s16/NOTE.md):
  // B two lanes 331.4k (1) vs 322.3k (0), one lane of 2048-pair chunks 294.6k vs 306.8k; C 11,260 vs 11,185; D
  // (2 x 128) 226.9k vs 224.1k; the 32-pair shard 64.67k vs 64.37k; A (640 wide) 122.7k vs 124.5k
  int opt_up_form = 3;
  int opt_smsys = 1;           // smoothness + system in one launch (0: two launches, A/B)
  // the fused launch on 2-D tiles for tall levels: 1 on, 0 off (two launches there), 2 auto = on for calls of
  // fewer than 512 pairs (one stream).  Measured at config E: alone on the GPU it cuts the system time 10 %
  // (580 vs 603 ms per 512 pairs on one stream), but beside a second chain (two streams) the LDS-holding
  // fused kernel overlaps worse with the other lane's patch kernel than the two plain launches (561 vs
  // 544-551 ms per step) -- profiles/r02/ab/ab_smsys2d.
  int opt_smsys2d = 2;
  int opt_smsys_march = 1;     // tall levels: smoothness + system as a register march (k_tv_smsys_m)
  int opt_smsys_prefetch = 1;  // fused smoothness + system (gray): derivative images issued before the staging
  int opt_smsys_small = 1;     // fused smoothness + system: small row blocks for launches that cannot fill the chip
  int opt_agg_stage = 1;       // k_aggregate: patch displacements of the tile staged in LDS (0: gathered from p_iter)
  int opt_pad_grad_v = 1;      // colour pyramid pad + gradients: one thread per value (0: per pixel, channels inside)
  int opt_pyr_rgb = 1;         // colour pyramid base by dword loads and masked v_sad_u8 (0: the byte loop)
  int opt_prepd_df = 1;        // smsys_deriv levels: k_tv_prepd_df (Ix, Iy, Iz from a 2-pixel halo, channels in one pass)
  int opt_smsys_deriv = 1;     // fused smoothness + system (gray; colour: the march): second derivatives filtered from Ix, Iy, Iz
  int call_frames = 1;         // pairs of the current call (auto options)
  int call_lanes = 1;          // streams the current call's chunks run on (auto options)
  int opt_sor_cring = 2;       // sweep-per-wave SOR: coefficient ring in LDS (0: every sweep loads its coefficients;
                               // 2: ring sized to the level's row groups, the clamped in-frame load form in launches
                               // that oversubscribe the chip; 3: that load form in every launch; 1: workgroup limit)
  int opt_prepd = 2;           // prep + derivatives in one launch: 1 intensity images, 2 colour images too (0: three launches)
  int opt_sor_rows2 = 1;       // sweep-per-wave SOR with two rows per lane for 321..640-row levels (0: pipeline)
  int opt_wave_per_patch = 0;  // 1: one wave per patch instead of eight lanes (A/B)
  int opt_sor_mode = 0;        // 0 exact lexicographic order (the reference's bits); 1 red-black (opt-in)
  int opt_patch_window = 1;    // eight-lane patches read their bilinear taps from an LDS window (0: L1 gathers)
  int opt_patch_quad = 1;      // windowed gray patches on four lanes per patch (k_patchq; 0: eight, k_patchw)
  int opt_patch_x16 = 1;       // windowed RGB p = 12 patches on sixteen lanes per patch (k_patchx; 0: eight, k_patchw;
                               // 2: k_patchx with the exact square-root evaluation every iteration, parity testing)
  int opt_patch_absw = 1;      // patch kernels that can hand the aggregation its weights directly do (0: loss weights)
  int opt_patch_buf = 1;       // gray p = 12 windows by buffer loads (32-bit offsets) where the image array allows
  int opt_patch_generic = 0;   // 1: every shape on the any-shape patch kernel k_patchg (parity testing)
  int opt_patch_fdiv = 1;      // the LLT solves divide by FMA-corrected pivot reciprocals (0: IEEE divisions)
  int opt_patch_maxres = 1;    // op-point stopping (res_thresh 0, min_iter = max_iter): largest |w| > 0 for mean > 0
  // sub-batch pipelining: chunks of `opt_chunk` frames round-robin over `opt_streams` streams, each with
  // its own workspace, so one chunk's latency-bound wavefront overlaps another chunk's streaming kernels.
  // streams 0 = auto: 2 for batches of >= 512 pairs (measured +7-9 % at 1024 1080p pairs: two 512-pair
  // chains on two streams), else 1; chunk 0 = the batch split evenly over the streams.
  int opt_streams = 0, opt_chunk = 0;
  struct Lane {
    hipStream_t s = nullptr;
    char *ws = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
  };
  std::vector<Lane> lanes;
  hipEvent_t entry = nullptr;
  // call ordering: ev_null hands the legacy NULL stream's queued work to the context's stream; ev_ws marks
  // the end of the previous call's use of the workspaces (a call on another stream waits for it)
  hipEvent_t ev_null = nullptr, ev_ws = nullptr;
  bool ws_pending = false;
  std::mutex mu;
};

namespace {

// OFDIS_TRACE=1: host-side progress lines on stderr (debugging the multi-stream paths)
bool trace_on() {
  static const bool on = std::getenv("OFDIS_TRACE") && std::getenv("OFDIS_TRACE")[0] == '1';
  return on;
}
#define OFDIS_TRACE(...)                  \
  do {                                    \
    if (trace_on()) {                     \
      std::fprintf(stderr, "ofdis: " __VA_ARGS__); \
      std::fputc('\n', stderr);           \
      std::fflush(stderr);                \
    }                                     \
  } while (0)

#define HIP_OK(x)                                                                                \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      std::fprintf(stderr, "ofdis: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, \
                   __LINE__);                                                                    \
      return e_ == hipErrorOutOfMemory ? OFDIS_ERR_OUT_OF_MEMORY : OFDIS_ERR_DEVICE;             \
    }                                                                                            \
  } while (0)

int kernel_index(const char *name) {
  for (int i = 0; i < (int)(sizeof(kKernelNames) / sizeof(kKernelNames[0])); ++i)
    if (std::strcmp(kKernelNames[i], name) == 0) return i;
  return -1;
}

hipEvent_t get_event(ofdis_context *c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

template <class F>
void timed(ofdis_context *c, int kernel, hipStream_t s, F &&f) {
  if (!c->timing) {
    f();
    return;
  }
  hipEvent_t a = get_event(c), b = get_event(c);
  hipEventRecord(a, s);
  f();
  hipEventRecord(b, s);
  c->pending.push_back({kernel, a, b});
}

void drain_timing(ofdis_context *c) {
  for (auto &p : c->pending) {
    hipEventSynchronize(p.b);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, p.a, p.b);
    auto &e = c->acc[p.kernel];
    e.first += ms;
    e.second += 1;
    c->pool.push_back(p.a);
    c->pool.push_back(p.b);
  }
  c->pending.clear();
}

void fill_level(const ofdis_params *p, int Wp, int Hp, int pad, int s, LevelGeom &g) {
  const float sc_fct = (float)std::pow(2.0, -s);  // oflow.cpp:142-153
  g.w = (int)((float)Wp * sc_fct);
  g.h = (int)((float)Hp * sc_fct);
  g.pad = pad;
  g.W = g.w + 2 * pad;
  g.H = g.h + 2 * pad;
  g.level = s;
  g.tmp_lb = -(float)p->p_samp_s / 2;
  g.tmp_ubw = (float)(g.w + p->p_samp_s / 2 - 2);
  g.tmp_ubh = (float)(g.h + p->p_samp_s / 2 - 2);
  const int st0 = (int)std::floor((float)p->p_samp_s * (1 - p->patove));  // oflow.cpp:90
  const int steps = st0 > 1 ? st0 : 1;
  g.nopw = (int)std::ceil((float)g.w / (float)steps);  // patchgrid.cpp:43-46
  g.noph = (int)std::ceil((float)g.h / (float)steps);
  g.offw = (g.w - (g.nopw - 1) * steps) / 2;
  g.offh = (g.h - (g.noph - 1) * steps) / 2;
  g.npatch = g.nopw * g.noph;
}

int steps_of(const ofdis_params *p) {
  const int st0 = (int)std::floor((float)p->p_samp_s * (1 - p->patove));
  return st0 > 1 ? st0 : 1;
}

Plan make_plan(const ofdis_params *p, int n, int Wp, int Hp, int pad, bool init = false) {
  Plan P;
  P.n = n;
  P.Wp = Wp;
  P.Hp = Hp;
  P.nop = p->mode == OFDIS_MODE_OF ? 2 : 1;
  P.noc = p->noc;
  P.pad = pad;
  P.sc_f = p->sc_f;
  P.sc_l = p->sc_l;
  const int nsc = p->sc_f - p->sc_l + 1;
  P.lv.resize(nsc);
  P.off_lvl.resize(nsc);
  P.off_img.resize(nsc);
  P.off_dx.resize(nsc);
  P.off_dy.resize(nsc);
  P.off_flow.resize(nsc);
  P.off_flow_bw.resize(nsc);
  P.fb = p->usefbcon != 0;
  size_t off = 0;
  const int novals = p->noc * p->p_samp_s * p->p_samp_s;
  size_t max_np = 0, max_plane = 0;
  for (int s = p->sc_l; s <= p->sc_f; ++s) {
    const int i = s - p->sc_l;
    fill_level(p, Wp, Hp, pad, s, P.lv[i]);
    const LevelGeom &g = P.lv[i];
    P.off_lvl[i] = off;
    off = align_up(off + sizeof(float) * 2 * (size_t)n * g.w * g.h * P.noc);
    P.off_img[i] = off;  // (+64 floats: the windowed patch kernel's 16-byte row loads may read past the last row)
    off = align_up(off + sizeof(float) * (2 * (size_t)n * g.W * g.H * P.noc + 64));
    P.off_dx[i] = off;
    off = align_up(off + sizeof(float) * 2 * (size_t)n * g.W * g.H * P.noc);
    P.off_dy[i] = off;
    off = align_up(off + sizeof(float) * 2 * (size_t)n * g.W * g.H * P.noc);
    P.off_flow[i] = off;
    off = align_up(off + sizeof(float) * (size_t)n * P.nop * g.w * g.h);
    P.off_flow_bw[i] = off;
    if (P.fb) off = align_up(off + sizeof(float) * (size_t)n * P.nop * g.w * g.h);
    if ((size_t)g.npatch > max_np) max_np = g.npatch;
    if ((size_t)g.w * g.h > max_plane) max_plane = (size_t)g.w * g.h;
  }
  P.off_piter = off;
  off = align_up(off + sizeof(float) * (size_t)n * max_np * P.nop);
  P.off_pw = off;  // loss weights [n][npatch][novals], or the aggregation-weight slot planes [n][A * A][h][w]
  const size_t aslots = (size_t)((p->p_samp_s - 1) / steps_of(p) + 1);
  off = align_up(off + sizeof(float) * (size_t)n * std::max(max_np * novals, aslots * aslots * max_plane));
  P.off_piter_bw = off;
  if (P.fb) off = align_up(off + sizeof(float) * (size_t)n * max_np * P.nop);
  P.off_pw_bw = off;
  if (P.fb) off = align_up(off + sizeof(float) * (size_t)n * max_np * novals);
  P.off_tv = off;
  size_t max_sp = 0;  // skewed TV plane
  for (const LevelGeom &g : P.lv) max_sp = std::max(max_sp, (size_t)skew_plane(g.w, g.h));
  P.tv_plane = max_sp;
  if (p->usetvref) off = align_up(off + sizeof(float) * (size_t)n * max_sp * (14 + 9 * (size_t)P.noc));
  P.off_gm = off;
  if (p->gradmag) {
    P.gradmag = true;
    off = align_up(off + sizeof(float) * 2 * (size_t)n * ((size_t)Wp * Hp + (size_t)(Wp / 2) * (Hp / 2)));
  }
  P.off_init = off;
  if (init) {
    P.init = true;
    off = align_up(off + sizeof(float) * (size_t)n * P.nop * (Wp >> (p->sc_f + 1)) * (Hp >> (p->sc_f + 1)));
  }
  P.total = off;
  return P;
}

// A captured graph bakes in the workspace and lane pointers: drop it before any of them is reallocated.
int drop_graph(ofdis_context *c) {
  if (!c->gexec) return OFDIS_OK;
  HIP_OK(hipDeviceSynchronize());  // it may still run on a caller stream
  HIP_OK(hipGraphExecDestroy(c->gexec));
  c->gexec = nullptr;
  return OFDIS_OK;
}

int ensure_ws(ofdis_context *c, size_t bytes) {
  if (bytes <= c->ws_cap) return OFDIS_OK;
  if (c->ws) {
    int rc = drop_graph(c);
    if (rc) return rc;
    HIP_OK(hipDeviceSynchronize());  // callers may have queued work on their own streams
    HIP_OK(hipFree(c->ws));
    c->ws = nullptr;
    c->ws_cap = 0;
  }
  HIP_OK(hipMalloc(&c->ws, bytes));
  c->ws_cap = bytes;
  return OFDIS_OK;
}

int capture(ofdis_context *c, hipStream_t s, const std::vector<float *> &cap, int scale, const Plan &P,
            const float *flow_planar) {
  if ((int)cap.size() <= scale || !cap[scale]) return OFDIS_OK;
  const LevelGeom &g = P.lv[scale - P.sc_l];
  const size_t plane = (size_t)g.w * g.h;
  std::vector<float> tmp(plane * P.nop);
  HIP_OK(hipMemcpyAsync(tmp.data(), flow_planar, tmp.size() * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  for (size_t i = 0; i < plane; ++i)
    for (int k = 0; k < P.nop; ++k) cap[scale][i * P.nop + k] = tmp[k * plane + i];
  return OFDIS_OK;
}

struct StageTimes {
  double pconst = 0, pinit = 0, poptim = 0, cflow = 0, tvopt = 0;
};

// The coarse-to-fine loop (oflow.cpp:182-330) over device pyramids already in the workspace.
// init: optional coarse initial flow (device, interleaved, (w_f/2)*(h_f/2)*nop per frame).
// The largest float s with sqrtf(s) <= t.  A correctly rounded square root is monotone, so for every float s
// (NaN and inf included) sqrtf(s) > t <=> s > sqrt_le_bound(t): the patch kernels' outlier test compares the
// squared distance against it, bit-for-bit the reference's norm() > outlierthresh without a square root.
static float sqrt_le_bound(float t) {
  if (!(t >= 0.0f) || std::isinf(t)) return t * t;
  float s = t * t;
  while (std::sqrt(std::nextafter(s, INFINITY)) <= t) s = std::nextafter(s, INFINITY);
  while (s > 0.0f && std::sqrt(s) > t) s = std::nextafter(s, -INFINITY);
  return s;
}

int run_levels(ofdis_context *c, char *ws, const Plan &P, const ofdis_params *p, hipStream_t s, const float *init,
               std::vector<StageTimes> *times) {
  const int nop = P.nop, noc = P.noc, n = P.n;
  const int novals = noc * p->p_samp_s * p->p_samp_s;
  const int steps = steps_of(p);
  hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  if (times)
    for (auto &e : ev) HIP_OK(hipEventCreate(&e));
  for (int sl = p->sc_f; sl >= p->sc_l; --sl) {
    const int i = sl - p->sc_l;
    const LevelGeom &g = P.lv[i];
    const size_t fsp = (size_t)g.W * g.H * noc;  // floats per padded frame
    const float *img = (const float *)(ws + P.off_img[i]);
    const float *dxp = (const float *)(ws + P.off_dx[i]);
    const float *dyp = (const float *)(ws + P.off_dy[i]);
    float *flow = (float *)(ws + P.off_flow[i]);
    if (times) HIP_OK(hipEventRecord(ev[0], s));

    PatchArgs pa{};
    pa.img_a = img;
    pa.dx_a = dxp;
    pa.dy_a = dyp;
    pa.img_b = img + (size_t)n * fsp;
    if (sl < p->sc_f) {
      const LevelGeom &gc = P.lv[i + 1];
      pa.prev = (const float *)(ws + P.off_flow[i + 1]);
      pa.prev_frame_stride = (long)nop * gc.w * gc.h;
      pa.prev_comp_stride = gc.w * gc.h;
      pa.prev_elem_stride = 1;
      pa.prev_w = g.w / 2;
    } else if (init) {
      pa.prev = init;
      pa.prev_frame_stride = (long)nop * (g.w / 2) * (g.h / 2);
      pa.prev_comp_stride = 1;
      pa.prev_elem_stride = nop;
      pa.prev_w = g.w / 2;
    }
    pa.p_iter = (float *)(ws + P.off_piter);
    pa.pweight = (float *)(ws + P.off_pw);
    pa.n = n;
    pa.nop = nop;
    pa.noc = noc;
    pa.p = p->p_samp_s;
    pa.novals = novals;
    pa.steps = steps;
    pa.costfct = p->costfct;
    pa.patnorm = p->patnorm;
    pa.max_iter = p->max_iter;
    pa.min_iter = p->min_iter;
    pa.dp_thresh_sq = p->dp_thresh * p->dp_thresh;
    pa.dr_thresh = p->dr_thresh;
    pa.res_thresh = p->res_thresh;
    pa.outlierthresh = (float)p->p_samp_s / 2;
    pa.outlier_sq = sqrt_le_bound(pa.outlierthresh);
    pa.camlr = 0;
    pa.wave_per_patch = c->opt_wave_per_patch;
    pa.window = c->opt_patch_window;
    pa.quad = c->opt_patch_quad;
    pa.x16 = c->opt_patch_x16;
    pa.absw = !P.fb && c->opt_patch_absw;  // usefbcon: the complementary grid's loss weights are read raw
    pa.aslots = (p->p_samp_s - 1) / steps + 1;
    pa.fdiv = c->opt_patch_fdiv;
    pa.maxres = c->opt_patch_maxres && pa.res_thresh == 0.0f && pa.min_iter >= pa.max_iter;
    pa.buf32 = c->opt_patch_buf && (size_t)n * fsp * sizeof(float) + 4096 <= 0xffffffffu;
    pa.generic = c->opt_patch_generic;
    pa.g = g;
    if (times) {  // verbosity 2: pconst / pinit from construction-only launches (their output is overwritten)
      PatchArgs pd = pa;
      pd.stage = 1;
      launch_patch(pd, s);
      HIP_OK(hipEventRecord(ev[1], s));
      pd.stage = 2;
      launch_patch(pd, s);
      HIP_OK(hipEventRecord(ev[2], s));
    }
    bool absw = false;
    timed(c, 3, s, [&] { absw = launch_patch(pa, s); });
    // usefbcon: the backward grid -- template on image b, target image a, right camera (camlr = 1),
    // initialised from the coarser backward flow (oflow.cpp:158-169, 193-196, 209-211, 231-233)
    PatchArgs pb = pa;
    if (P.fb) {
      pb.img_a = img + (size_t)n * fsp;
      pb.dx_a = dxp + (size_t)n * fsp;
      pb.dy_a = dyp + (size_t)n * fsp;
      pb.img_b = img;
      pb.prev = nullptr;
      if (sl < p->sc_f) pb.prev = (const float *)(ws + P.off_flow_bw[i + 1]);
      pb.p_iter = (float *)(ws + P.off_piter_bw);
      pb.pweight = (float *)(ws + P.off_pw_bw);
      pb.camlr = 1;
      timed(c, 3, s, [&] { launch_patch(pb, s); });
    }

    AggArgs ag{};
    ag.p_iter = pa.p_iter;
    ag.pweight = pa.pweight;
    ag.flow = flow;
    ag.n = n;
    ag.nop = nop;
    ag.noc = noc;
    ag.p = p->p_samp_s;
    ag.novals = novals;
    ag.absw = absw;
    ag.aslots = pa.aslots;
    ag.stage = c->opt_agg_stage;
    ag.steps = steps;
    ag.g = g;
    ag.cg_p_iter = P.fb ? pb.p_iter : nullptr;
    ag.cg_pweight = P.fb ? pb.pweight : nullptr;
    float *flow_bw = (float *)(ws + P.off_flow_bw[i]);
    const int n_inner = p->tv_innerit * (sl + 1);  // refine_variational.cpp:36
    // the refinement's arguments for direction dir (dir 1: VarRefClass on the backward flow with the images swapped,
    // oflow.cpp:312-316)
    auto make_tv = [&](int dir) {
      const long sp = skew_plane(g.w, g.h);
      const size_t pl = (size_t)n * sp;
      float *t0 = (float *)(ws + P.off_tv);
      TvArgs tv{};
      tv.img_a = dir == 0 ? img : img + (size_t)n * fsp;
      tv.img_b = dir == 0 ? img + (size_t)n * fsp : img;
      tv.flow = dir == 0 ? flow : flow_bw;
      tv.du = t0;
      tv.dv = t0 + pl;
      tv.mask = t0 + 2 * pl;
      tv.coef = t0 + 3 * pl;  // 8 planes' worth (float4 x 2 per pixel), 16-byte aligned: sp % 4 == 0 ensured
      tv.s = t0 + 11 * pl;
      tv.wxs = t0 + 12 * pl;
      tv.wys = t0 + 13 * pl;
      tv.sp = sp;
      tv.wrap = g.h <= g.w;
      tv.skew_slots = tv.wrap ? g.w * g.h : (g.w + g.h - 1) * g.h;
      float *cp = t0 + 14 * pl;
      const size_t cpl = pl * noc;
      tv.t = cp;
      tv.dt = cp + cpl;
      tv.Iz = tv.dt;
      tv.Ix = cp + 2 * cpl;
      tv.Iy = cp + 3 * cpl;
      tv.Ixx = cp + 4 * cpl;
      tv.Ixy = cp + 5 * cpl;
      tv.Iyy = cp + 6 * cpl;
      tv.Ixz = cp + 7 * cpl;
      tv.Iyz = cp + 8 * cpl;
      tv.n = n;
      tv.nop = nop;
      tv.noc = noc;
      tv.w = g.w;
      tv.h = g.h;
      tv.pad = g.pad;
      tv.W = g.W;
      tv.quarter_alpha = 0.25f * p->tv_alpha;  // refine_variational.cpp:40-43
      tv.hgo3 = p->tv_gamma * 0.5f / 3.0f;
      tv.hdo3 = p->tv_delta * 0.5f / 3.0f;
      tv.omega = p->tv_sor;
      tv.solverit = p->tv_solverit;
      tv.camlr = dir;
      tv.sor_generic = c->opt_sor_generic;
      tv.sor_variant = c->opt_sor_pipe;
      tv.sor_cring = c->opt_sor_cring;
      tv.sor_rows2 = c->opt_sor_rows2;
      tv.smsys = c->opt_smsys;
      tv.smsys2d = c->opt_smsys2d == 2 ? c->call_frames < 512 : c->opt_smsys2d;
      tv.smsys_march = c->opt_smsys_march;
      tv.smsys_prefetch = c->opt_smsys_prefetch;
      tv.smsys_small = c->opt_smsys_small;
      tv.smsys_deriv = c->opt_smsys_deriv;
      tv.prepd_df = c->opt_prepd_df;
      tv.sor_redblack = c->opt_sor_mode == 1;
      tv.sor_point = p->omp_build && nop == 2;  // refine_variational.cpp:202-203
      tv.prepd = c->opt_prepd;
      return tv;
    };
    if (times) HIP_OK(hipEventRecord(ev[3], s));
    timed(c, 4, s, [&] { launch_aggregate(ag, s); });
    const bool bw_level = P.fb && sl > p->sc_l;  // the backward flow is not needed after the last scale
    if (bw_level) {                               // patchgrid.cpp:213-397 with the roles swapped
      AggArgs ab = ag;
      ab.p_iter = pb.p_iter;
      ab.pweight = pb.pweight;
      ab.cg_p_iter = pa.p_iter;
      ab.cg_pweight = pa.pweight;
      ab.flow = flow_bw;
      timed(c, 4, s, [&] { launch_aggregate(ab, s); });
    }
    if (times) HIP_OK(hipEventRecord(ev[4], s));
    int rc = capture(c, s, c->cap_dis, sl, P, flow);
    if (rc) return rc;

    for (int dir = 0; dir < (bw_level ? 2 : 1) && p->usetvref && n_inner > 0; ++dir) {
      TvArgs tv = make_tv(dir);
      // latency form of sor_mode = 1: the whole inner loop and the flow update in one launch per level, prep writing
      // the colour-split layout that launch reads (all eight derivative planes)
      tv.lat = tv_level_rb_ok(tv);
      tv.smsys_deriv = !tv.lat && tv_deriv_fused(tv);  // before the prep launch: it decides which planes prepd writes
      if (tv_prepd_ok(tv)) {
        timed(c, 5, s, [&] { launch_tv_prepd(tv, s); });
      } else {
        timed(c, 5, s, [&] { launch_tv_prep(tv, s); });
        timed(c, 6, s, [&] {
          launch_tv_deriv1(tv, s);
          launch_tv_deriv2(tv, s);
        });
      }
      if (tv.lat) {
        timed(c, 11, s, [&] { launch_tv_level_rb(tv, n_inner, s); });
        continue;
      }
      for (int it = 0; it < n_inner; ++it) {
        tv.first_iter = it == 0;
        timed(c, 7, s, [&] {
          if (tv_smsys_ok(tv)) {
            launch_tv_smsys(tv, s);
          } else {
            launch_tv_smooth(tv, s);
            launch_tv_system(tv, s);
          }
        });
        timed(c, 8, s, [&] { launch_tv_sor(tv, s); });
      }
      timed(c, 9, s, [&] { launch_tv_final(tv, s); });
    }
    if (times) {
      HIP_OK(hipEventRecord(ev[5], s));
      HIP_OK(hipEventSynchronize(ev[5]));
      StageTimes st;
      float t01, t12, t23, t34, t45;
      hipEventElapsedTime(&t01, ev[0], ev[1]);
      hipEventElapsedTime(&t12, ev[1], ev[2]);
      hipEventElapsedTime(&t23, ev[2], ev[3]);
      hipEventElapsedTime(&t34, ev[3], ev[4]);
      hipEventElapsedTime(&t45, ev[4], ev[5]);
      // the optimisation launch repeats construction and initialisation: poptim is the rest of it
      st.pconst = t01;
      st.pinit = std::max(0.0, (double)t12 - t01);
      st.poptim = std::max(0.0, (double)t23 - t12);
      st.cflow = t34;
      st.tvopt = t45;
      times->push_back(st);
    }
    rc = capture(c, s, c->cap_tv, sl, P, flow);
    if (rc) return rc;
  }
  if (times)
    for (auto &e : ev) hipEventDestroy(e);
  return hipGetLastError() == hipSuccess ? OFDIS_OK : OFDIS_ERR_DEVICE;
}

void print_times(const Plan &P, const std::vector<StageTimes> &t, double total_ms, int verbosity) {
  if (verbosity > 1) {
    for (size_t k = 0; k < t.size(); ++k) {
      const int sl = P.sc_f - (int)k;
      const LevelGeom &g = P.lv[sl - P.sc_l];
      const double all = t[k].pconst + t[k].pinit + t[k].poptim + t[k].cflow + t[k].tvopt;
      std::printf("TIME (Sc: %i, #p:%6i, pconst, pinit, poptim, cflow, tvopt, total): %8.2f %8.2f %8.2f %8.2f %8.2f -> %8.2f ms.\n",
                  sl, g.npatch, t[k].pconst, t[k].pinit, t[k].poptim, t[k].cflow, t[k].tvopt, all);
    }
  }
  if (verbosity > 0) std::printf("TIME (O.Flow Run-Time   ) (ms): %3g\n", total_ms);
}

int check_device(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return OFDIS_ERR_NO_DEVICE;
  if (device < 0 || device >= count) return OFDIS_ERR_INVALID_ARGUMENT;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return OFDIS_ERR_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    std::fprintf(stderr, "ofdis: device %d is %s, this build targets gfx950 only\n", device, prop.gcnArchName);
    return OFDIS_ERR_NO_DEVICE;
  }
  return OFDIS_OK;
}

// Pyramid of the batch (run_dense.cpp:299-312,327-328,131-179) into the workspace.
int run_pyramid(ofdis_context *c, char *ws, const Plan &P, const uint8_t *a, const uint8_t *b, hipStream_t s) {
  const int n2 = 2 * P.n;
  if (P.gradmag) {  // SELECTCHANNEL 2 (run_dense.cpp:139-148): float level 0, then 2x2 means down to sc_l
    float *lvl0 = (float *)(ws + P.off_lvl[0]);
    float *bufA = (float *)(ws + P.off_gm), *bufB = bufA + (size_t)n2 * P.Wp * P.Hp;
    PyrGradmagArgs g{};
    g.img_a = a;
    g.img_b = b;
    g.n = P.n;
    g.W0 = P.W0;
    g.H0 = P.H0;
    g.padl = P.padl;
    g.padt = P.padt;
    g.Wp = P.Wp;
    g.Hp = P.Hp;
    g.out = P.sc_l == 0 ? lvl0 : bufA;
    timed(c, 0, s, [&] { launch_pyr_gradmag(g, s); });
    const float *src = bufA;
    int w = P.Wp, h = P.Hp;
    for (int l = 1; l <= P.sc_l; ++l) {
      PyrDownArgs pd{};
      pd.src = src;
      pd.dst = l == P.sc_l ? lvl0 : ((l & 1) ? bufB : bufA);
      pd.n2 = n2;
      pd.w = w /= 2;
      pd.h = h /= 2;
      pd.noc = 1;
      timed(c, 1, s, [&] { launch_pyr_down(pd, s); });
      src = pd.dst;
    }
  } else {
    PyrBaseArgs pb{};
    pb.img_a = a;
    pb.img_b = b;
    pb.n = P.n;
    pb.W0 = P.W0;
    pb.H0 = P.H0;
    pb.noc = P.noc;
    pb.padl = P.padl;
    pb.padt = P.padt;
    pb.log2s = P.sc_l;
    pb.w = P.lv[0].w;
    pb.h = P.lv[0].h;
    pb.out = (float *)(ws + P.off_lvl[0]);
    pb.rgb_sad = c->opt_pyr_rgb;
    timed(c, 0, s, [&] { launch_pyr_base(pb, s); });
  }
  for (size_t i = 1; i < P.lv.size(); ++i) {
    PyrDownArgs pd{};
    pd.src = (const float *)(ws + P.off_lvl[i - 1]);
    pd.dst = (float *)(ws + P.off_lvl[i]);
    pd.n2 = n2;
    pd.w = P.lv[i].w;
    pd.h = P.lv[i].h;
    pd.noc = P.noc;
    timed(c, 1, s, [&] { launch_pyr_down(pd, s); });
  }
  for (size_t i = 0; i < P.lv.size(); ++i) {
    PyrPadGradArgs pg{};
    pg.lvl = (const float *)(ws + P.off_lvl[i]);
    pg.img = (float *)(ws + P.off_img[i]);
    pg.dx = (float *)(ws + P.off_dx[i]);
    pg.dy = (float *)(ws + P.off_dy[i]);
    pg.n2 = n2;
    pg.w = P.lv[i].w;
    pg.h = P.lv[i].h;
    pg.noc = P.noc;
    pg.pad = P.pad;
    pg.per_value = c->opt_pad_grad_v;
    timed(c, 2, s, [&] { launch_pyr_pad_grad(pg, s); });
  }
  return hipGetLastError() == hipSuccess ? OFDIS_OK : OFDIS_ERR_DEVICE;
}

Plan batch_plan(const ofdis_params *p, int n, int width, int height, bool init = false) {
  const int d = 1 << (p->sc_f + (init ? 1 : 0));  // run_dense.cpp:301-302
  const int padw = (width % d) ? d - width % d : 0, padh = (height % d) ? d - height % d : 0;
  Plan P = make_plan(p, n, width + padw, height + padh, p->p_samp_s, init);
  P.W0 = width;
  P.H0 = height;
  P.padw = padw;
  P.padh = padh;
  P.padl = padw / 2;  // copyMakeBorder(floor(padw/2), ceil(padw/2)) (run_dense.cpp:309)
  P.padt = padh / 2;
  return P;
}

}  // namespace

extern "C" {

int ofdis_context_create(int device, ofdis_context **out) {
  if (!out) return OFDIS_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  int rc = check_device(device);
  if (rc) return rc;
  HIP_OK(hipSetDevice(device));
  ofdis_context *c = new ofdis_context();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return OFDIS_ERR_DEVICE;
  }
  // load the kernels' code objects now, not inside the first call's timers (the drop-in CLI's one pair)
  warm_kernels_module(c->stream);
  warm_tvrb_module(c->stream);
  if (hipStreamSynchronize(c->stream) != hipSuccess) {
    hipStreamDestroy(c->stream);
    delete c;
    return OFDIS_ERR_DEVICE;
  }
  *out = c;
  return OFDIS_OK;
}

void ofdis_context_destroy(ofdis_context *c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->gexec) {  // it may still run on a caller stream
    hipDeviceSynchronize();
    hipGraphExecDestroy(c->gexec);
    c->gexec = nullptr;
  }
  if (c->ws_pending) hipEventSynchronize(c->ev_ws);  // the last call's work, on whatever stream it ran
  if (c->stream) hipStreamSynchronize(c->stream);
  drain_timing(c);
  for (auto e : c->pool) hipEventDestroy(e);
  if (c->ws) hipFree(c->ws);
  for (auto &L : c->lanes) {
    if (L.s) hipStreamSynchronize(L.s);
    if (L.ws) hipFree(L.ws);
    if (L.done) hipEventDestroy(L.done);
    if (L.s) hipStreamDestroy(L.s);
  }
  if (c->entry) hipEventDestroy(c->entry);
  if (c->ev_null) hipEventDestroy(c->ev_null);
  if (c->ev_ws) hipEventDestroy(c->ev_ws);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

namespace {

// x 2^sc_l + INTER_LINEAR upsample + crop of the finest level's flow in workspace ws (run_dense.cpp:407-415).
int run_upsample(ofdis_context *c, char *ws, const Plan &P, const ofdis_params *p, float *flow_out, hipStream_t s) {
  UpArgs up{};
  up.flow = (const float *)(ws + P.off_flow[0]);
  up.out = flow_out;
  up.n = P.n;
  up.nop = P.nop;
  up.wl = P.lv[0].w;
  up.hl = P.lv[0].h;
  up.log2s = p->sc_l;
  up.W0 = P.W0;
  up.H0 = P.H0;
  up.offx = P.padl;
  up.offy = P.padt;
  up.nt_store = c->opt_nt_store;
  up.form = c->opt_up_form == 3 ? (P.W0 >= 1024 && (c->call_lanes >= 2 || c->call_frames < 1024) ? 1 : 0)
                                 : c->opt_up_form;
  timed(c, 10, s, [&] { launch_upsample(up, s); });
  return hipGetLastError() == hipSuccess ? OFDIS_OK : OFDIS_ERR_DEVICE;
}

// The initial flow of a chunk (device, full resolution [n][H0][W0][nop]) -> OFClass's initflow input in the
// workspace (run_dense.cpp:356-379, restated: ofo_init_flow_area).
int run_init(ofdis_context *c, char *ws, const Plan &P, const ofdis_params *p, const float *init, hipStream_t s) {
  InitArgs ia{};
  ia.init = init;
  ia.out = (float *)(ws + P.off_init);
  ia.n = P.n;
  ia.nop = P.nop;
  ia.W0 = P.W0;
  ia.H0 = P.H0;
  ia.padl = P.padl;
  ia.padt = P.padt;
  ia.log2k = p->sc_f + 1;
  ia.wo = P.Wp >> (p->sc_f + 1);
  ia.ho = P.Hp >> (p->sc_f + 1);
  ia.sc = (float)std::pow(2.0, -p->sc_f - 1);  // flowinit *= sc_fct (float)
  ia.scale = 1.f / (float)(1 << (2 * (p->sc_f + 1)));
  launch_init_area(ia, s);
  return hipGetLastError() == hipSuccess ? OFDIS_OK : OFDIS_ERR_DEVICE;
}

// One chunk of frames through the whole pipeline on stream s with workspace ws.
int run_chunk(ofdis_context *c, char *ws, const Plan &P, const ofdis_params *p, const uint8_t *img_a,
              const uint8_t *img_b, const float *init, float *flow_out, hipStream_t s) {
  int rc = run_pyramid(c, ws, P, img_a, img_b, s);
  if (rc) return rc;
  if (init && (rc = run_init(c, ws, P, p, init, s))) return rc;
  rc = run_levels(c, ws, P, p, s, init ? (const float *)(ws + P.off_init) : nullptr, nullptr);
  if (rc) return rc;
  return run_upsample(c, ws, P, p, flow_out, s);
}

// k lanes (stream, done event, workspace of `bytes`).
int ensure_lanes(ofdis_context *c, int k, size_t bytes) {
  if ((int)c->lanes.size() < k) c->lanes.resize(k);
  if (!c->entry) HIP_OK(hipEventCreateWithFlags(&c->entry, hipEventDisableTiming));
  for (int i = 0; i < k; ++i) {
    auto &L = c->lanes[i];
    if (!L.s) HIP_OK(hipStreamCreateWithFlags(&L.s, hipStreamNonBlocking));
    if (!L.done) HIP_OK(hipEventCreateWithFlags(&L.done, hipEventDisableTiming));
    if (L.cap < bytes) {
      if (L.ws) {
        int rc = drop_graph(c);
        if (rc) return rc;
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipFree(L.ws));
        L.ws = nullptr;
        L.cap = 0;
      }
      HIP_OK(hipMalloc(&L.ws, bytes));
      L.cap = bytes;
    }
  }
  return OFDIS_OK;
}

// two lanes from 256 pairs (config D, 256 pairs: 223.4-223.7k on one stream, 225.3-226.8k on two; profiles/r05/s22)
int stream_count(const ofdis_context *c, int n) { return c->opt_streams > 0 ? c->opt_streams : (n >= 256 ? 2 : 1); }

// Frames per launch such that every TV plane group (n * noc * sp floats, addressed with 32-bit byte
// offsets by the system kernels' ldu) stays below 2^30 floats.
int tv_frame_cap(const ofdis_params *p, int width, int height) {
  if (!p->usetvref) return 1 << 30;
  const Plan P1 = batch_plan(p, 1, width, height);
  const long per = (long)P1.noc * (long)P1.tv_plane;
  return (int)std::min((long)(1 << 30), ((1L << 30) - 1) / per);  // 0: one frame alone is too large
}

// How one call is issued: the whole batch on one stream and workspace (single), or chunks round-robin over
// lanes (round robin).  Everything the issue needs -- workspaces, lane streams, events -- is allocated by
// prepare(), before any capture begins.  (Round 5's software pipeline over a streaming stream and chain lanes,
// with CU-masked streams and a staggered round robin, measured slower in every form and was removed in round 6.)
struct CallPlan {
  enum Kind { kSingle, kRoundRobin } kind = kSingle;
  int n = 0, width = 0, height = 0, chunk = 0, nchunks = 1, lanes = 0;
  bool init = false;
  Plan whole;               // kSingle
  std::vector<Plan> parts;  // kRoundRobin: one plan per chunk
};

int prepare(ofdis_context *c, const ofdis_params *p, int n, int width, int height, bool init, bool capturing,
            CallPlan &cp) {
  cp.n = n;
  c->call_frames = n;
  c->call_lanes = 1;
  cp.width = width;
  cp.height = height;
  cp.init = init;
  // a stage capture (frame 0's per-scale flow) runs the batch as one launch on one stream, whatever the
  // stream / chunk options; it is refused only for batches beyond the launch-size cap
  const int nstreams = capturing ? 1 : stream_count(c, n);
  int chunk = capturing ? n : c->opt_chunk > 0 ? std::min(c->opt_chunk, n) : (n + nstreams - 1) / nstreams;
  chunk = std::min(chunk, tv_frame_cap(p, width, height));
  if (chunk < 1) return OFDIS_ERR_INVALID_ARGUMENT;
  cp.chunk = chunk;
  cp.nchunks = (n + chunk - 1) / chunk;
  if (cp.nchunks > 1 && capturing) return OFDIS_ERR_UNSUPPORTED;
  if (cp.nchunks == 1) {
    cp.kind = CallPlan::kSingle;
    cp.whole = batch_plan(p, n, width, height, init);
    return ensure_ws(c, cp.whole.total);
  }
  cp.kind = CallPlan::kRoundRobin;
  for (int ch = 0; ch < cp.nchunks; ++ch)
    cp.parts.push_back(batch_plan(p, std::min(chunk, n - ch * chunk), width, height, init));
  cp.lanes = std::min(nstreams, cp.nchunks);
  c->call_lanes = cp.lanes;
  return ensure_lanes(c, cp.lanes, cp.parts[0].total);
}

// Chunks round-robin over the lanes, each chunk's whole pipeline on one lane (fork from s, join into s).
int issue_round_robin(ofdis_context *c, const CallPlan &cp, hipStream_t s, const ofdis_params *p,
                      const uint8_t *img_a, const uint8_t *img_b, const float *init, float *flow_out) {
  const int k = cp.lanes;
  HIP_OK(hipEventRecord(c->entry, s));
  for (int i = 0; i < k; ++i) HIP_OK(hipStreamWaitEvent(c->lanes[i].s, c->entry, 0));
  const size_t in_frame = (size_t)cp.width * cp.height * p->noc;
  const size_t out_frame = (size_t)cp.width * cp.height * cp.parts[0].nop;
  for (int ch = 0; ch < cp.nchunks; ++ch) {
    const size_t f0 = (size_t)ch * cp.chunk;
    auto &L = c->lanes[ch % k];
    int rc = run_chunk(c, L.ws, cp.parts[ch], p, img_a + f0 * in_frame, img_b + f0 * in_frame,
                       init ? init + f0 * out_frame : nullptr, flow_out + f0 * out_frame, L.s);
    if (rc) return rc;
  }
  for (int i = 0; i < k; ++i) {
    HIP_OK(hipEventRecord(c->lanes[i].done, c->lanes[i].s));
    HIP_OK(hipStreamWaitEvent(s, c->lanes[i].done, 0));
  }
  return OFDIS_OK;
}

int issue(ofdis_context *c, const CallPlan &cp, hipStream_t s, const ofdis_params *p, const uint8_t *img_a,
          const uint8_t *img_b, const float *init, float *flow_out) {
  switch (cp.kind) {
    case CallPlan::kRoundRobin: return issue_round_robin(c, cp, s, p, img_a, img_b, init, flow_out);
    default: return run_chunk(c, c->ws, cp.whole, p, img_a, img_b, init, flow_out, s);
  }
}

// Start of a call on stream s: NULL is the legacy default stream (torch's default), which the context's
// non-blocking stream does not order against -- hand its queued work over with an event; and the
// workspaces are shared by every call on this context, whatever its stream -- wait for the previous call.
int call_begin(ofdis_context *c, void *stream, hipStream_t &s) {
  if (!c->ev_null) HIP_OK(hipEventCreateWithFlags(&c->ev_null, hipEventDisableTiming));
  if (!c->ev_ws) HIP_OK(hipEventCreateWithFlags(&c->ev_ws, hipEventDisableTiming));
  s = stream ? (hipStream_t)stream : c->stream;
  if (!stream) {
    HIP_OK(hipEventRecord(c->ev_null, nullptr));
    HIP_OK(hipStreamWaitEvent(s, c->ev_null, 0));
  }
  if (c->ws_pending) HIP_OK(hipStreamWaitEvent(s, c->ev_ws, 0));
  return OFDIS_OK;
}

// End of a call: mark the workspaces' release; a NULL-stream caller's later work waits for the result.
int call_end(ofdis_context *c, void *stream, hipStream_t s) {
  HIP_OK(hipEventRecord(c->ev_ws, s));
  c->ws_pending = true;
  if (!stream) HIP_OK(hipStreamWaitEvent(nullptr, c->ev_ws, 0));
  return OFDIS_OK;
}

int validate_call(const ofdis_params *p, int width, int height, bool init) {
  int rc = ofdis_params_validate(p, -1, -1, -1);
  if (rc) return rc;
  Plan P = batch_plan(p, 1, width, height, init);
  rc = ofdis_params_validate(p, P.Wp, P.Hp, P.pad);
  if (rc) return rc;
  // one frame's TV plane group must stay below 2^30 floats (32-bit byte offsets in the system kernels)
  return tv_frame_cap(p, width, height) >= 1 ? OFDIS_OK : OFDIS_ERR_INVALID_ARGUMENT;
}

// The whole-batch device path on stream s (call ordering done by the caller).
int run_batch(ofdis_context *c, hipStream_t s, const uint8_t *img_a, const uint8_t *img_b, const float *init, int n,
              int width, int height, const ofdis_params *p, float *flow_out) {
  const bool capturing = !c->cap_dis.empty() || !c->cap_tv.empty();
  CallPlan cp;
  int rc = prepare(c, p, n, width, height, init != nullptr, capturing, cp);
  if (rc) return rc;
  OFDIS_TRACE("run_batch: kind %d, %d chunks of %d, %d lanes", (int)cp.kind, cp.nchunks, cp.chunk, cp.lanes);
  // graph 1: capture single-stream batches; graph 2: also the multi-lane (fork / join) issues
  const bool graph = c->opt_graph == 2 || (c->opt_graph == 1 && cp.kind == CallPlan::kSingle);
  if (!graph || capturing || c->timing) return issue(c, cp, s, p, img_a, img_b, init, flow_out);
  // ~80 dependent launches per chunk: record them once as a HIP graph (on the context's own stream -- the
  // caller's may be the legacy NULL stream, which cannot capture) and replay it on the caller's stream while
  // the pointers, sizes, parameters and options stay the same (set_option drops the graph).  Multi-lane
  // issues fork from and join into the capturing stream through events recorded inside the capture.
  ofdis_context::GraphKey key;
  std::memset(&key, 0, sizeof(key));  // padding included: the key is compared bytewise
  key.a = img_a; key.b = img_b; key.out = flow_out; key.ws = c->ws; key.init = init;
  key.n = n; key.w = width; key.h = height; key.p = *p;
  if (!c->gexec || std::memcmp(&key, &c->gkey, sizeof(key)) != 0) {
    if ((rc = drop_graph(c))) return rc;
    OFDIS_TRACE("graph: capture (kind %d, %d chunks of %d)", (int)cp.kind, cp.nchunks, cp.chunk);
    HIP_OK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    rc = issue(c, cp, c->stream, p, img_a, img_b, init, flow_out);
    OFDIS_TRACE("graph: issued rc %d", rc);
    hipGraph_t graph = nullptr;
    const hipError_t ce = hipStreamEndCapture(c->stream, &graph);
    OFDIS_TRACE("graph: captured rc %d end %d", rc, (int)ce);
    if (rc) {
      if (graph) hipGraphDestroy(graph);
      return rc;
    }
    if (ce != hipSuccess || !graph) return OFDIS_ERR_DEVICE;
    const hipError_t ie = hipGraphInstantiate(&c->gexec, graph, nullptr, nullptr, 0);
    OFDIS_TRACE("graph: instantiated %d", (int)ie);
    hipGraphDestroy(graph);
    if (ie != hipSuccess) {
      c->gexec = nullptr;
      return OFDIS_ERR_DEVICE;
    }
    std::memcpy(&c->gkey, &key, sizeof(key));
  }
  HIP_OK(hipGraphLaunch(c->gexec, s));
  OFDIS_TRACE("graph: launched");
  return OFDIS_OK;
}

// verbosity 2, one pair (the CLI): the reference's stdout timers -- pyramid (run_dense.cpp:352), grid
// allocation (oflow.cpp:177), per-scale stages (oflow.cpp:297) and the OFClass total (oflow.cpp:336) --
// from HIP events around eager launches on the context's stream.
int run_verbose(ofdis_context *c, const uint8_t *img_a, const uint8_t *img_b, const float *init, int width,
                int height, const ofdis_params *p, float *flow_out) {
  hipStream_t s = c->stream;
  c->call_frames = 1;
  auto t0 = std::chrono::steady_clock::now();
  Plan P = batch_plan(p, 1, width, height, init != nullptr);
  int rc = ensure_ws(c, P.total);
  if (rc) return rc;
  const double alloc_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, s));
  rc = run_pyramid(c, c->ws, P, img_a, img_b, s);
  if (!rc && init) rc = run_init(c, c->ws, P, p, init, s);
  HIP_OK(hipEventRecord(e1, s));
  HIP_OK(hipEventSynchronize(e1));
  float pyr_ms = 0.0f;
  hipEventElapsedTime(&pyr_ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (rc) return rc;
  std::printf("TIME (Pyramide+Gradients) (ms): %3g\n", pyr_ms);
  std::printf("TIME (Grid Memo. Alloc. ) (ms): %3g\n", alloc_ms);
  auto t1 = std::chrono::steady_clock::now();
  std::vector<StageTimes> times;
  rc = run_levels(c, c->ws, P, p, s, init ? (const float *)(c->ws + P.off_init) : nullptr, &times);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(s));
  const double ms = alloc_ms + std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
  print_times(P, times, ms, p->verbosity);
  return run_upsample(c, c->ws, P, p, flow_out, s);
}

}  // namespace

int ofdis_run_batch_u8(ofdis_context *c, const uint8_t *img_a, const uint8_t *img_b, int n, int width, int height,
                       const ofdis_params *p, float *flow_out, void *stream) {
  return ofdis_run_batch_u8_init(c, img_a, img_b, nullptr, n, width, height, p, flow_out, stream);
}

int ofdis_run_batch_u8_init(ofdis_context *c, const uint8_t *img_a, const uint8_t *img_b, const float *init, int n,
                            int width, int height, const ofdis_params *p, float *flow_out, void *stream) {
  if (!c || !img_a || !img_b || !flow_out || n <= 0 || width <= 0 || height <= 0) return OFDIS_ERR_INVALID_ARGUMENT;
  int rc = validate_call(p, width, height, init != nullptr);
  if (rc) return rc;
  std::lock_guard<std::mutex> lock(c->mu);
  HIP_OK(hipSetDevice(c->device));
  hipStream_t s;
  if ((rc = call_begin(c, stream, s))) return rc;
  rc = run_batch(c, s, img_a, img_b, init, n, width, height, p, flow_out);
  const int rc2 = call_end(c, stream, s);
  return rc ? rc : rc2;
}

int ofdis_run_batch_u8_host(ofdis_context *c, const uint8_t *img_a, const uint8_t *img_b, int n, int width,
                            int height, const ofdis_params *p, float *flow_out) {
  return ofdis_run_batch_u8_init_host(c, img_a, img_b, nullptr, n, width, height, p, flow_out);
}

int ofdis_run_batch_u8_init_host(ofdis_context *c, const uint8_t *img_a, const uint8_t *img_b, const float *init,
                                 int n, int width, int height, const ofdis_params *p, float *flow_out) {
  if (!c || !img_a || !img_b || !flow_out || n <= 0 || width <= 0 || height <= 0 || !p)
    return OFDIS_ERR_INVALID_ARGUMENT;
  HIP_OK(hipSetDevice(c->device));
  const size_t in = (size_t)n * width * height * p->noc;
  const size_t out = (size_t)n * width * height * (p->mode == OFDIS_MODE_OF ? 2 : 1);
  uint8_t *da = nullptr, *db = nullptr;
  float *dout = nullptr, *dinit = nullptr;
  int rc = OFDIS_OK;
  auto step = [&](hipError_t e) {
    if (e != hipSuccess && rc == OFDIS_OK) rc = e == hipErrorOutOfMemory ? OFDIS_ERR_OUT_OF_MEMORY : OFDIS_ERR_DEVICE;
    return rc == OFDIS_OK;
  };
  if (step(hipMalloc(&da, in)) && step(hipMalloc(&db, in)) && step(hipMalloc(&dout, out * sizeof(float))) &&
      (!init || step(hipMalloc(&dinit, out * sizeof(float)))) &&
      step(hipMemcpyAsync(da, img_a, in, hipMemcpyHostToDevice, c->stream)) &&
      step(hipMemcpyAsync(db, img_b, in, hipMemcpyHostToDevice, c->stream)) &&
      (!init || step(hipMemcpyAsync(dinit, init, out * sizeof(float), hipMemcpyHostToDevice, c->stream)))) {
    const bool verbose = p->verbosity > 1 && n == 1 && c->cap_dis.empty() && c->cap_tv.empty() && !c->timing;
    auto t0 = std::chrono::steady_clock::now();
    if (verbose) {
      rc = validate_call(p, width, height, dinit != nullptr);
      if (!rc) {
        std::lock_guard<std::mutex> lock(c->mu);
        hipStream_t s;
        rc = call_begin(c, c->stream, s);
        if (!rc) rc = run_verbose(c, da, db, dinit, width, height, p, dout);
        if (!rc) rc = call_end(c, c->stream, s);
      }
    } else {
      rc = ofdis_run_batch_u8_init(c, da, db, dinit, n, width, height, p, dout, c->stream);
    }
    if (rc == OFDIS_OK && step(hipStreamSynchronize(c->stream))) {
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (p->verbosity == 1) std::printf("TIME (O.Flow Run-Time   ) (ms): %3g\n", ms);
      step(hipMemcpy(flow_out, dout, out * sizeof(float), hipMemcpyDeviceToHost));
    }
  }
  hipFree(da);
  hipFree(db);
  hipFree(dout);
  hipFree(dinit);
  return rc;
}

int ofdis_pyramid_u8_host(ofdis_context *c, const uint8_t *img, int width, int height, const ofdis_params *p,
                          int imgpadding, float *const *img_pyr, float *const *dx_pyr, float *const *dy_pyr) {
  if (!c || !img || !p || width <= 0 || height <= 0) return OFDIS_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lock(c->mu);
  HIP_OK(hipSetDevice(c->device));
  ofdis_params q = *p;
  q.p_samp_s = imgpadding;  // pad by imgpadding
  Plan P = batch_plan(p, 1, width, height);
  P = make_plan(p, 1, P.Wp, P.Hp, imgpadding);
  {
    const int d = 1 << p->sc_f;
    P.W0 = width;
    P.H0 = height;
    P.padw = (width % d) ? d - width % d : 0;
    P.padh = (height % d) ? d - height % d : 0;
    P.padl = P.padw / 2;
    P.padt = P.padh / 2;
  }
  int rc = ensure_ws(c, P.total);
  if (rc) return rc;
  const size_t in = (size_t)width * height * p->noc;
  uint8_t *d = nullptr;
  HIP_OK(hipMalloc(&d, in));
  HIP_OK(hipMemcpy(d, img, in, hipMemcpyHostToDevice));
  hipStream_t st;
  rc = call_begin(c, c->stream, st);
  if (rc == OFDIS_OK) rc = run_pyramid(c, c->ws, P, d, d, st);
  if (rc == OFDIS_OK) rc = call_end(c, c->stream, st);
  if (rc == OFDIS_OK) {
    HIP_OK(hipStreamSynchronize(c->stream));
    for (int s = p->sc_l; s <= p->sc_f; ++s) {
      const LevelGeom &g = P.lv[s - p->sc_l];
      const size_t bytes = sizeof(float) * (size_t)g.W * g.H * p->noc;
      if (img_pyr && img_pyr[s]) HIP_OK(hipMemcpy(img_pyr[s], c->ws + P.off_img[s - p->sc_l], bytes, hipMemcpyDeviceToHost));
      if (dx_pyr && dx_pyr[s]) HIP_OK(hipMemcpy(dx_pyr[s], c->ws + P.off_dx[s - p->sc_l], bytes, hipMemcpyDeviceToHost));
      if (dy_pyr && dy_pyr[s]) HIP_OK(hipMemcpy(dy_pyr[s], c->ws + P.off_dy[s - p->sc_l], bytes, hipMemcpyDeviceToHost));
    }
  }
  hipFree(d);
  (void)q;
  return rc;
}

int ofdis_context_set_stage_capture(ofdis_context *c, float *const *dis_flow, float *const *tv_flow, int nscales) {
  if (!c || nscales < 0) return OFDIS_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lock(c->mu);
  c->cap_dis.assign(nscales, nullptr);
  c->cap_tv.assign(nscales, nullptr);
  bool any = false;
  for (int i = 0; i < nscales; ++i) {
    if (dis_flow) c->cap_dis[i] = dis_flow[i];
    if (tv_flow) c->cap_tv[i] = tv_flow[i];
    any = any || c->cap_dis[i] || c->cap_tv[i];
  }
  if (!any) {  // no capture: the batch runs as usual (chunked, graph-replayed)
    c->cap_dis.clear();
    c->cap_tv.clear();
  }
  return OFDIS_OK;
}

int ofdis_context_set_option(ofdis_context *c, const char *key, int value) {
  if (!c || !key) return OFDIS_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lock(c->mu);
  struct Opt {
    const char *name;
    int ofdis_context::*field;
    int lo, hi;
  };
  static const Opt opts[] = {
      {"sor_generic", &ofdis_context::opt_sor_generic, 0, 1},
      {"sor_pipe", &ofdis_context::opt_sor_pipe, 0, 1},     {"smsys", &ofdis_context::opt_smsys, 0, 1},
      {"sor_cring", &ofdis_context::opt_sor_cring, 0, 3},   {"smsys2d", &ofdis_context::opt_smsys2d, 0, 2},
      {"smsys_march", &ofdis_context::opt_smsys_march, 0, 1},
      {"smsys_prefetch", &ofdis_context::opt_smsys_prefetch, 0, 1},
      {"smsys_small", &ofdis_context::opt_smsys_small, 0, 1},
      {"smsys_deriv", &ofdis_context::opt_smsys_deriv, 0, 1},
      {"prepd_df", &ofdis_context::opt_prepd_df, 0, 1},
      {"pyr_rgb", &ofdis_context::opt_pyr_rgb, 0, 1},
      {"pad_grad_v", &ofdis_context::opt_pad_grad_v, 0, 1},
      {"agg_stage", &ofdis_context::opt_agg_stage, 0, 1},
      {"sor_rows2", &ofdis_context::opt_sor_rows2, 0, 1},   {"prepd", &ofdis_context::opt_prepd, 0, 2},
      {"wave_per_patch", &ofdis_context::opt_wave_per_patch, 0, 1},
      {"nt_store", &ofdis_context::opt_nt_store, 0, 1},     {"up_form", &ofdis_context::opt_up_form, 0, 3},
      {"graph", &ofdis_context::opt_graph, 0, 2},
      {"patch_window", &ofdis_context::opt_patch_window, 0, 1}, {"patch_quad", &ofdis_context::opt_patch_quad, 0, 1},
      {"patch_generic", &ofdis_context::opt_patch_generic, 0, 1}, {"sor_mode", &ofdis_context::opt_sor_mode, 0, 1},
      {"patch_x16", &ofdis_context::opt_patch_x16, 0, 2},  {"patch_absw", &ofdis_context::opt_patch_absw, 0, 1},
      {"patch_buf", &ofdis_context::opt_patch_buf, 0, 1},  {"patch_fdiv", &ofdis_context::opt_patch_fdiv, 0, 1},
      {"patch_maxres", &ofdis_context::opt_patch_maxres, 0, 1},
      {"streams", &ofdis_context::opt_streams, 0, 16},      {"chunk", &ofdis_context::opt_chunk, 0, 1 << 30},
  };
  for (const Opt &o : opts) {
    if (std::strcmp(key, o.name) != 0) continue;
    if (value < o.lo || value > o.hi) return OFDIS_ERR_INVALID_ARGUMENT;
    HIP_OK(hipSetDevice(c->device));
    const int rc = drop_graph(c);  // a captured graph bakes in the options it was recorded with
    if (rc) return rc;
    c->*o.field = (o.hi == 1) ? (value != 0) : value;
    return OFDIS_OK;
  }
  return OFDIS_ERR_INVALID_ARGUMENT;
}

int ofdis_context_enable_kernel_timing(ofdis_context *c, int enable) {
  if (!c) return OFDIS_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lock(c->mu);
  drain_timing(c);
  c->acc.clear();
  c->timing = enable != 0;
  return OFDIS_OK;
}

int ofdis_context_kernel_time(ofdis_context *c, const char *name, double *total_ms, long *launches) {
  if (!c || !name) return OFDIS_ERR_INVALID_ARGUMENT;
  const int k = kernel_index(name);
  if (k < 0) return OFDIS_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lock(c->mu);
  drain_timing(c);
  auto it = c->acc.find(k);
  if (total_ms) *total_ms = it == c->acc.end() ? 0.0 : it->second.first;
  if (launches) *launches = it == c->acc.end() ? 0 : it->second.second;
  return OFDIS_OK;
}

const char *ofdis_kernel_names(void) {
  static const std::string names = [] {
    std::string r;
    for (const char *k : kKernelNames) r += (r.empty() ? "" : ",") + std::string(k);
    return r;
  }();
  return names.c_str();
}

// Byte model of SURVEY §8(d), per frame pair, for the roofline of each kernel family.
int ofdis_algorithmic_bytes(const ofdis_params *p, int width, int height, const char *kernel, double *bytes) {
  if (!p || !kernel || !bytes) return OFDIS_ERR_INVALID_ARGUMENT;
  Plan P = batch_plan(p, 1, width, height);
  const int nop = P.nop, noc = P.noc;
  const int novals = noc * p->p_samp_s * p->p_samp_s;
  double b = 0.0;
  const std::string k(kernel);
  if (("," + std::string(ofdis_kernel_names()) + ",").find("," + k + ",") == std::string::npos)
    return OFDIS_ERR_INVALID_ARGUMENT;
  for (const LevelGeom &g : P.lv) {
    const double px = (double)g.w * g.h;
    const int n_inner = p->usetvref ? p->tv_innerit * (g.level + 1) : 0;
    if (k == "tv_sor") b += n_inner * p->tv_solverit * px * (nop == 2 ? 44.0 : 24.0);
    // fused red-black level (latency form): wx, wy and the eight derivative planes in, the flow out -- once per level
    // (the later inner iterations re-read the derivative planes from the frame's L2-resident copy)
    if (k == "tv_level" && n_inner > 0) b += px * 4.0 * (2 * nop + 8 * noc);
    if (k == "tv_system") b += n_inner * px * (4.0 * (8 * noc + 1 + 2 * nop) + 4.0 * (nop == 2 ? 7 : 4));
    // patch: per patch the template + gradients, ONE (p+1)^2 target window, the outputs (the compulsory bytes;
    // re-reads of the window over the iterations are cache-resident, and the kernel is VALU-issue bound)
    if (k == "patch") b += (double)g.npatch * (12.0 * novals + 4.0 * (p->p_samp_s + 1) * (p->p_samp_s + 1) * noc +
                                               4.0 * (nop + novals));
    if (k == "aggregate") b += px * 4.0 * nop + (double)g.npatch * 4.0 * (nop + novals);
    if (k == "pyr_pad_grad") b += 2.0 * (px * 4.0 * noc + 3.0 * g.W * g.H * 4.0 * noc);
    if (k == "pyr_down" && g.level > p->sc_l) b += 2.0 * noc * 4.0 * (4.0 * px + px);
    if (p->usetvref) {
      if (k == "tv_prep") b += px * 4.0 * (4 * noc + 1 + 3 * nop);
      if (k == "tv_deriv") b += px * 4.0 * noc * (2 + 4 + 2 + 3);
      if (k == "tv_final") b += px * 4.0 * 3 * nop;
    }
  }
  if (k == "pyr_base") b = 2.0 * width * height * noc + 2.0 * 4.0 * P.lv[0].w * P.lv[0].h * noc;
  if (k == "upsample") b = (double)width * height * nop * 4.0;
  *bytes = b;
  return OFDIS_OK;
}

// OFC::OFClass (oflow.h:99-126) with host pointers; one frame pair on device 0.
int ofdis_oflow_compute(const float *const *im_ao, const float *const *im_ao_dx, const float *const *im_ao_dy,
                        const float *const *im_bo, const float *const *im_bo_dx, const float *const *im_bo_dy,
                        int imgpadding, float *outflow, const float *initflow, int width, int height,
                        const ofdis_params *p) {
  if (!im_ao || !im_ao_dx || !im_ao_dy || !im_bo || !outflow) return OFDIS_ERR_INVALID_ARGUMENT;
  int rc = ofdis_params_validate(p, width, height, imgpadding);
  if (rc) return rc;
  for (int s = p->sc_l; s <= p->sc_f; ++s) {
    if (!im_ao[s] || !im_ao_dx[s] || !im_ao_dy[s] || !im_bo[s]) return OFDIS_ERR_INVALID_ARGUMENT;
    // image b's gradients are read only by the backward grid of usefbcon (oflow.cpp:193-196)
    if (p->usefbcon && (!im_bo_dx || !im_bo_dy || !im_bo_dx[s] || !im_bo_dy[s])) return OFDIS_ERR_INVALID_ARGUMENT;
  }
  static std::mutex gmu;
  static ofdis_context *gctx = nullptr;
  std::lock_guard<std::mutex> glock(gmu);
  if (!gctx) {
    rc = ofdis_context_create(0, &gctx);
    if (rc) return rc;
  }
  ofdis_context *c = gctx;
  std::lock_guard<std::mutex> lock(c->mu);
  HIP_OK(hipSetDevice(c->device));
  auto t0 = std::chrono::steady_clock::now();
  Plan P = make_plan(p, 1, width, height, imgpadding);
  rc = ensure_ws(c, P.total);
  if (rc) return rc;
  hipStream_t s;
  if ((rc = call_begin(c, c->stream, s))) return rc;
  for (int sl = p->sc_l; sl <= p->sc_f; ++sl) {
    const LevelGeom &g = P.lv[sl - p->sc_l];
    const size_t fb = sizeof(float) * (size_t)g.W * g.H * p->noc;
    char *img = c->ws + P.off_img[sl - p->sc_l];
    HIP_OK(hipMemcpyAsync(img, im_ao[sl], fb, hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(img + fb, im_bo[sl], fb, hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(c->ws + P.off_dx[sl - p->sc_l], im_ao_dx[sl], fb, hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(c->ws + P.off_dy[sl - p->sc_l], im_ao_dy[sl], fb, hipMemcpyHostToDevice, s));
    if (p->usefbcon) {
      HIP_OK(hipMemcpyAsync(c->ws + P.off_dx[sl - p->sc_l] + fb, im_bo_dx[sl], fb, hipMemcpyHostToDevice, s));
      HIP_OK(hipMemcpyAsync(c->ws + P.off_dy[sl - p->sc_l] + fb, im_bo_dy[sl], fb, hipMemcpyHostToDevice, s));
    }
  }
  float *dinit = nullptr;
  if (initflow) {
    const size_t nb = sizeof(float) * (size_t)(width >> (p->sc_f + 1)) * (height >> (p->sc_f + 1)) * P.nop;
    HIP_OK(hipMalloc(&dinit, nb > 0 ? nb : 4));
    if (nb) HIP_OK(hipMemcpyAsync(dinit, initflow, nb, hipMemcpyHostToDevice, s));
  }
  std::vector<StageTimes> times;
  c->call_frames = 1;
  rc = run_levels(c, c->ws, P, p, s, dinit, p->verbosity > 1 ? &times : nullptr);
  if (rc == OFDIS_OK) {
    const LevelGeom &g = P.lv[0];
    const size_t plane = (size_t)g.w * g.h;
    std::vector<float> tmp(plane * P.nop);
    HIP_OK(hipMemcpyAsync(tmp.data(), c->ws + P.off_flow[0], tmp.size() * sizeof(float), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    for (size_t i = 0; i < plane; ++i)
      for (int k = 0; k < P.nop; ++k) outflow[i * P.nop + k] = tmp[k * plane + i];
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    print_times(P, times, ms, p->verbosity);
  }
  if (rc == OFDIS_OK) rc = call_end(c, c->stream, s);
  if (dinit) hipFree(dinit);
  return rc;
}

int ofdis_max_frames_per_launch(const ofdis_params *p, int width, int height, int *frames) {
  if (!p || !frames || width <= 0 || height <= 0) return OFDIS_ERR_INVALID_ARGUMENT;
  const int rc = ofdis_params_validate(p, -1, -1, -1);
  if (rc) return rc;
  *frames = tv_frame_cap(p, width, height);
  return *frames >= 1 ? OFDIS_OK : OFDIS_ERR_INVALID_ARGUMENT;
}

}  // extern "C"
