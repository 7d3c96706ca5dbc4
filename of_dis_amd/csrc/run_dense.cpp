// run_dense.cpp -- the run_{OF,DE}_{INT,RGB} command lines (drop-in for the reference's run_dense.cpp).
//
//   run_OF_INT img1 img2 out.flo            operating point 2, coarsest scale chosen automatically
//   run_OF_INT img1 img2 out.flo X          operating point X = 1..4
//   run_OF_INT img1 img2 out.flo p1 .. p20  all 20 parameters explicitly (README.md:54-86)
//   run_OF_INT img1 img2 out.flo p1 .. p20 1 init.flo   ... with an initial flow (run_dense.cpp:293-294)
//
// SELECTMODE (1 flow -> .flo, 2 depth -> .pfm) and SELECTCHANNEL (1 gray, 3 BGR) are compile-time, as in
// the reference's CMakeLists.txt:36-61.  Images: PNG and Netpbm, decoded with cv::imread's semantics
// (ofdis_read_image; OpenCV is not in this image).  Unlike the reference, argv is validated (the
// reference reads past argv for 6 <= argc < 24, run_dense.cpp:270-295).
// OFDIS_CLI_TIMING=1 adds a per-process breakdown on stderr (HIP runtime init + context creation with the code-object
// load, the call, the file write; tools/cli_wall.py): the reference's stdout timers stay as they are.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/ofdis.h"

#ifndef SELECTMODE
#define SELECTMODE 1
#endif
#ifndef SELECTCHANNEL
#define SELECTCHANNEL 1
#endif
// SELECTCHANNEL 1: intensity, 2: gradient magnitude of the intensity image (run_dense.cpp:139-148,
// 194-197), 3: BGR colour
#define NOCHANNELS (SELECTCHANNEL == 3 ? 3 : 1)

// cv::imread(path, CV_LOAD_IMAGE_GRAYSCALE / CV_LOAD_IMAGE_COLOR) (run_dense.cpp:202-206)
static std::vector<uint8_t> load(const char *path, int &w, int &h) {
  int rc = ofdis_read_image(path, nullptr, &w, &h, NOCHANNELS, 0);
  std::vector<uint8_t> px;
  if (rc == OFDIS_OK) {
    px.resize((size_t)w * h * NOCHANNELS);
    rc = ofdis_read_image(path, px.data(), &w, &h, NOCHANNELS, px.size());
  }
  if (rc != OFDIS_OK) {
    std::fprintf(stderr, "cannot read %s (PNG, Netpbm or BMP expected): %s\n", path, ofdis_status_string(rc));
    std::exit(1);
  }
  return px;
}

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char **argv) {
  auto t0 = std::chrono::steady_clock::now();
  const auto tproc = t0;
  const char *tenv = std::getenv("OFDIS_CLI_TIMING");
  const bool cli_timing = tenv && std::atoi(tenv) != 0;
  // argv[24] / argv[25]: "hasinfile" and the initial-flow file, the reference's commented-out plumbing
  // (run_dense.cpp:293-294): a .flo (OF) / float depth .flo (DE) of the input size
  const bool hasinfile = argc == 26 && std::atoi(argv[24]) != 0;
  if (argc != 4 && argc != 5 && argc != 24 && !(argc == 25 && std::atoi(argv[24]) == 0) && !hasinfile) {
    std::fprintf(stderr, "usage: %s img1 img2 out [oppoint 1-4 | 20 parameters [hasinfile(0/1) [init.flo]]]\n",
                 argv[0]);
    return 1;
  }
  int w = 0, h = 0, w2 = 0, h2 = 0;
  std::vector<uint8_t> a = load(argv[1], w, h), b = load(argv[2], w2, h2);
  if (w != w2 || h != h2) {
    std::fprintf(stderr, "image sizes differ\n");
    return 1;
  }
  ofdis_params p;
  int rc;
  if (argc <= 5)
    rc = ofdis_params_oppoint(&p, argc == 5 ? std::atoi(argv[4]) : 2, w, SELECTMODE, NOCHANNELS);
  else
    rc = ofdis_params_from_strings(&p, 20, (const char *const *)(argv + 4), SELECTMODE, NOCHANNELS);
  p.gradmag = SELECTCHANNEL == 2;
#ifdef OFDIS_OMP_BUILD
  p.omp_build = 1;  // the reference's USE_OPENMP build semantics (point SOR), in single-thread order
#endif
  if (rc == OFDIS_OK) rc = ofdis_params_validate(&p, -1, -1, -1);
  if (rc != OFDIS_OK) {
    std::fprintf(stderr, "invalid parameters: %s\n", ofdis_status_string(rc));
    return 1;
  }
  if (p.verbosity > 1)
    std::printf("TIME (Image loading     ) (ms): %3g\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  const double load_ms = ms_since(t0);
  ofdis_context *ctx = nullptr;
  auto tc = std::chrono::steady_clock::now();
  rc = ofdis_context_create(0, &ctx);
  const double ctx_ms = ms_since(tc);
  if (rc != OFDIS_OK) {
    std::fprintf(stderr, "no usable gfx950 device: %s\n", ofdis_status_string(rc));
    return 1;
  }
  const int nop = SELECTMODE == 1 ? 2 : 1;
  std::vector<float> flow((size_t)w * h * nop), init;
  if (hasinfile) {  // ReadFlowFile (run_dense.cpp:85-129) into a w x h x nop image
    int iw = 0, ih = 0;
    init.resize(flow.size());
    if (ofdis_read_flo(argv[25], nullptr, &iw, &ih, nop) != OFDIS_OK || iw != w || ih != h ||
        ofdis_read_flo(argv[25], init.data(), &iw, &ih, nop) != OFDIS_OK) {
      std::fprintf(stderr, "cannot read %s (a %dx%d .flo file expected)\n", argv[25], w, h);
      ofdis_context_destroy(ctx);
      return 1;
    }
  }
  auto tr = std::chrono::steady_clock::now();
  rc = ofdis_run_batch_u8_init_host(ctx, a.data(), b.data(), hasinfile ? init.data() : nullptr, 1, w, h, &p,
                                    flow.data());
  const double run_ms = ms_since(tr);
  tr = std::chrono::steady_clock::now();
  ofdis_context_destroy(ctx);
  const double destroy_ms = ms_since(tr);
  if (rc != OFDIS_OK) {
    std::fprintf(stderr, "flow computation failed: %s\n", ofdis_status_string(rc));
    return 1;
  }
  t0 = std::chrono::steady_clock::now();
  rc = SELECTMODE == 1 ? ofdis_write_flo(argv[3], flow.data(), w, h, 2) : ofdis_write_pfm(argv[3], flow.data(), w, h);
  if (rc != OFDIS_OK) {
    std::fprintf(stderr, "cannot write %s\n", argv[3]);
    return 1;
  }
  const double write_ms = ms_since(t0);
  if (p.verbosity > 1) std::printf("TIME (Saving flow file  ) (ms): %3g\n", write_ms);
  if (cli_timing)
    std::fprintf(stderr,
                 "cli_ms load %.3f context_create %.3f call %.3f context_destroy %.3f write %.3f main_total %.3f\n",
                 load_ms, ctx_ms, run_ms, destroy_ms, write_ms, ms_since(tproc));
  return 0;
}
