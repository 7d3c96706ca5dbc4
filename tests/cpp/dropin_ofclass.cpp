// Drop-in check of include/ofdis_oflow.hpp: the reference's run_dense.cpp call sequence (pyramid of both
// frames, then OFC::OFClass with op-point-2 parameters, run_dense.cpp:226-268 / :392-401) written against
// the wrapper.  Usage: dropin_ofclass a.pgm b.pgm out.flo   (flow at the finest computed scale)
#include <cstdio>
#include <vector>

#include "ofdis_oflow.hpp"

int main(int argc, char **argv) {
  if (argc != 4) return 2;
  int w = 0, h = 0, c = 0;
  if (ofdis_read_pnm(argv[1], nullptr, &w, &h, &c, 0) || c != 1) return 3;
  std::vector<uint8_t> a((size_t)w * h), b((size_t)w * h);
  if (ofdis_read_pnm(argv[1], a.data(), &w, &h, &c, a.size()) || ofdis_read_pnm(argv[2], b.data(), &w, &h, &c, b.size()))
    return 3;
  ofdis_params p;
  ofdis_params_oppoint(&p, 2, w, OFDIS_MODE_OF, 1);
  if (w % (1 << p.sc_f) || h % (1 << p.sc_f)) return 4;  // the caller pads (run_dense.cpp:299-312)
  const int pad = p.p_samp_s;
  ofdis_context *ctx = nullptr;
  if (ofdis_context_create(0, &ctx)) return 5;
  std::vector<std::vector<float>> store;
  const float *pa[3][32] = {}, *pb[3][32] = {};
  for (int f = 0; f < 2; ++f) {
    float *dst[3][32] = {};
    for (int s = p.sc_l; s <= p.sc_f; ++s)
      for (int k = 0; k < 3; ++k) {
        store.emplace_back((size_t)((w >> s) + 2 * pad) * ((h >> s) + 2 * pad));
        dst[k][s] = store.back().data();
        (f ? pb : pa)[k][s] = dst[k][s];
      }
    if (ofdis_pyramid_u8_host(ctx, f ? b.data() : a.data(), w, h, &p, pad, dst[0], dst[1], dst[2])) return 6;
  }
  ofdis_context_destroy(ctx);
  std::vector<float> flow((size_t)(w >> p.sc_l) * (h >> p.sc_l) * 2);
  try {
    OFC::OFClass ofc(pa[0], pa[1], pa[2], pb[0], pb[1], pb[2], pad, flow.data(), nullptr, w, h, p.sc_f, p.sc_l,
                     p.max_iter, p.min_iter, p.dp_thresh, p.dr_thresh, p.res_thresh, p.p_samp_s, p.patove, false,
                     p.costfct, 1, p.patnorm, true, p.tv_alpha, p.tv_gamma, p.tv_delta, p.tv_innerit,
                     p.tv_solverit, p.tv_sor, 0);
  } catch (const OFC::OFDisError &e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 7;
  }
  return ofdis_write_flo(argv[3], flow.data(), w >> p.sc_l, h >> p.sc_l, 2) ? 8 : 0;
}
