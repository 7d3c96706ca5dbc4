// Minimal stand-alone probe of HIP stream capture with the event patterns of ofdis_runtime.cpp's multi-lane
// issues (no ofdis code): does hipStreamEndCapture survive two lanes that wait on each other?
//   mode 0: round robin  -- fork s -> {S, L}, kernels on each, join (what graph=2 captures fine)
//   mode 1: one-way      -- L waits on events recorded on S, S never waits on L until the join
//   mode 2: pipeline     -- S -> L (ev_pyr) and L -> S (ev_lev), chunk by chunk (issue_pipeline's order)
//   mode 3: pipeline with one event per hand-over direction re-recorded every chunk
//   mode 4: mode 2 issued eagerly first (its events recorded outside any capture), then captured
//   mode 5: mode 2 with 40 kernels per stage (a chunk's length)
//   mode 6: mode 2 with no kernels at all (events only)
// Build: hipcc --offload-arch=gfx950 -O2 tools/capture_repro.hip -o tools/bin/capture_repro
//        hipcc --offload-arch=gfx950 -O2 -fPIC -shared -DREPRO_LIB tools/capture_repro.hip -o tools/bin/libcapture_repro.so
// Run:   tools/bin/capture_repro MODE [chunks]   (prints each step; a crash names the last one)
//        python tools/capture_repro_torch.py MODE: the same inside a process that imported torch, whose
//        bundled HIP runtime (torch/lib/libamdhip64.so) then serves every HIP call of the process
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      std::fflush(stdout);                                                                 \
      return 2;                                                                            \
    }                                                                                      \
  } while (0)

__global__ void k_add(float *p, int n, float v) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + v;
}

static void step(const char *what) {
  std::printf("%s\n", what);
  std::fflush(stdout);
}

static int repro(int mode, int nch) {
  const int n = 1 << 16;
  float *buf = nullptr;
  CK(hipMalloc(&buf, sizeof(float) * n * 2));
  CK(hipMemset(buf, 0, sizeof(float) * n * 2));
  hipStream_t s, S, L;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&L, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(2 * nch + 3);
  for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  hipEvent_t entry = ev[2 * nch], doneS = ev[2 * nch + 1], doneL = ev[2 * nch + 2];
  hipEvent_t *ev_pyr = ev.data(), *ev_lev = ev.data() + nch;
  float *a = buf, *b = buf + n;
  const dim3 g(n / 256), blk(256);

  const int kper = mode == 5 ? 40 : (mode == 6 ? 0 : 1);
  const int pattern = mode >= 4 ? 2 : mode;
  auto issue = [&]() -> int {
  CK(hipEventRecord(entry, s));
  CK(hipStreamWaitEvent(S, entry, 0));
  CK(hipStreamWaitEvent(L, entry, 0));
  if (pattern == 0) {
    for (int ch = 0; ch < nch; ++ch) k_add<<<g, blk, 0, (ch & 1) ? L : S>>>((ch & 1) ? b : a, n, 1.f);
  } else if (pattern == 1) {
    for (int ch = 0; ch < nch; ++ch) {
      k_add<<<g, blk, 0, S>>>(a, n, 1.f);
      CK(hipEventRecord(ev_pyr[ch], S));
      CK(hipStreamWaitEvent(L, ev_pyr[ch], 0));
      k_add<<<g, blk, 0, L>>>(b, n, 2.f);
    }
  } else {
    auto pyr = [&](int ch) -> int {
      for (int r = 0; r < kper; ++r) k_add<<<g, blk, 0, S>>>(a, n, 1.f);
      CK(hipEventRecord(mode == 3 ? ev_pyr[0] : ev_pyr[ch], S));
      return 0;
    };
    if (pyr(0)) return 2;
    for (int ch = 0; ch < nch; ++ch) {
      CK(hipStreamWaitEvent(L, mode == 3 ? ev_pyr[0] : ev_pyr[ch], 0));
      for (int r = 0; r < kper; ++r) k_add<<<g, blk, 0, L>>>(b, n, 2.f);
      CK(hipEventRecord(mode == 3 ? ev_lev[0] : ev_lev[ch], L));
      if (ch + 1 < nch && pyr(ch + 1)) return 2;
      CK(hipStreamWaitEvent(S, mode == 3 ? ev_lev[0] : ev_lev[ch], 0));
      for (int r = 0; r < kper; ++r) k_add<<<g, blk, 0, S>>>(a, n, 3.f);
    }
  }
  CK(hipEventRecord(doneS, S));
  CK(hipStreamWaitEvent(s, doneS, 0));
  CK(hipEventRecord(doneL, L));
  CK(hipStreamWaitEvent(s, doneL, 0));
  CK(hipGetLastError());
  return 0;
  };
  if (mode == 4) {
    step("eager issue");
    if (issue()) return 2;
    CK(hipStreamSynchronize(s));
  }
  step("begin capture");
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  if (issue()) return 2;
  step("issued; end capture");
  hipGraph_t graph = nullptr;
  CK(hipStreamEndCapture(s, &graph));
  size_t nodes = 0;
  CK(hipGraphGetNodes(graph, nullptr, &nodes));
  std::printf("captured %zu nodes\n", nodes);
  hipGraphExec_t exec = nullptr;
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  step("instantiated; launch");
  CK(hipGraphLaunch(exec, s));
  CK(hipStreamSynchronize(s));
  step("ok");
  (void)hipGraphExecDestroy(exec);
  (void)hipGraphDestroy(graph);
  (void)hipFree(buf);
  return 0;
}

#ifdef REPRO_LIB
extern "C" int capture_repro(int mode, int nch) { return repro(mode, nch); }
#else
int main(int argc, char **argv) { return repro(argc > 1 ? std::atoi(argv[1]) : 2, argc > 2 ? std::atoi(argv[2]) : 3); }
#endif
