// Graph capture of the multi-lane round robin (chunks forked over two streams and joined) through the C ABI, in a
// process of its own (its HIP calls go to the ROCm runtime libofdis.so links, not to a runtime another library
// brought along).  An eager run, then runs with option graph=GMODE (2: capture the multi-lane issues too), each
// compared bitwise with the eager output.  Usage: lanes_capture [GMODE]   (prints "same 1" per run)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ofdis.h"

#define CK(x)                                                        \
  do {                                                               \
    const int r_ = (int)(x);                                         \
    if (r_) {                                                        \
      std::printf("%s:%d %s -> %d\n", __FILE__, __LINE__, #x, r_);   \
      return 2;                                                      \
    }                                                                \
  } while (0)

int main(int argc, char **argv) {
  const int gmode = argc > 1 ? std::atoi(argv[1]) : 2;
  const int w = 320, h = 240, n = 5;
  std::vector<uint8_t> ha((size_t)n * w * h), hb(ha.size());
  for (int f = 0; f < n; ++f)
    CK(ofdis_synth_pair_u8(ha.data() + (size_t)f * w * h, hb.data() + (size_t)f * w * h, w, h, 1, f, 1));
  std::vector<float> o1(ha.size() * 2), o2(o1.size());
  ofdis_params p;
  CK(ofdis_params_oppoint(&p, 2, w, 1, 1));
  ofdis_context *c = nullptr;
  CK(ofdis_context_create(0, &c));
  CK(ofdis_context_set_option(c, "streams", 2));
  CK(ofdis_context_set_option(c, "chunk", 2));
  CK(ofdis_context_set_option(c, "graph", 0));
  CK(ofdis_run_batch_u8_host(c, ha.data(), hb.data(), n, w, h, &p, o1.data()));
  CK(ofdis_context_set_option(c, "graph", gmode));
  for (int rep = 0; rep < 2; ++rep) {
    CK(ofdis_run_batch_u8_host(c, ha.data(), hb.data(), n, w, h, &p, o2.data()));
    std::printf("same %d\n", (int)(std::memcmp(o1.data(), o2.data(), o1.size() * sizeof(float)) == 0));
  }
  ofdis_context_destroy(c);
  return 0;
}
