/*
 * ofdis_oflow.hpp -- header-only drop-in for the reference's oflow.h (namespace OFC, class OFClass).
 *
 * A C++ caller of lordnn/OF_DIS (run_dense.cpp:392-401) swaps `#include "oflow.h"` for this header and
 * links libofdis.so instead of compiling oflow.cpp / patchgrid.cpp / patch.cpp / refine_variational.cpp /
 * FDF1.0.1.  The constructor has the reference's exact signature (oflow.h:99-126) and, like it, computes
 * the flow into `outflow` before returning.  SELECTMODE / SELECTCHANNEL stay compile-time switches here
 * (CMakeLists.txt:36-61) and are forwarded as the runtime fields of ofdis_params.
 *
 * Differences, all at the error channel only: the reference never validates and exit(1)s on OOM; this
 * wrapper throws OFC::OFDisError (with the ofdis_status) for invalid parameters or a missing gfx950
 * device.  No CPU fallback exists.  usefbcon = true runs forward-backward merging on the GPU.
 */
#ifndef OFDIS_OFLOW_HPP
#define OFDIS_OFLOW_HPP

#include <stdexcept>
#include <string>

#include "ofdis.h"

#ifndef SELECTMODE
#define SELECTMODE 1
#endif
#ifndef SELECTCHANNEL
#define SELECTCHANNEL 1
#endif

namespace OFC {

class OFDisError : public std::runtime_error {
 public:
  OFDisError(int code, const char *what)
      : std::runtime_error(std::string(what) + ": " + ofdis_status_string(code)), status(code) {}
  int status;
};

class OFClass {
 public:
  OFClass(const float **im_ao_in, const float **im_ao_dx_in, const float **im_ao_dy_in,
          const float **im_bo_in, const float **im_bo_dx_in, const float **im_bo_dy_in,
          const int imgpadding_in, float *outflow, const float *initflow, const int width_in,
          const int height_in, const int sc_f_in, const int sc_l_in, const int max_iter_in,
          const int min_iter_in, const float dp_thresh_in, const float dr_thresh_in, const float res_thresh_in,
          const int padval_in, const float patove_in, const bool usefbcon_in, const int costfct_in,
          const int noc_in, const int patnorm_in, const bool usetvref_in, const float tv_alpha_in,
          const float tv_gamma_in, const float tv_delta_in, const int tv_innerit_in, const int tv_solverit_in,
          const float tv_sor_in, const int verbosity_in) {
    ofdis_params p = {};
    p.mode = SELECTMODE;
#ifdef _OPENMP
    p.omp_build = 1;  // an OpenMP build of the reference refines with point SOR (refine_variational.cpp:202-203)
#endif
    p.noc = noc_in;
    p.sc_f = sc_f_in;
    p.sc_l = sc_l_in;
    p.max_iter = max_iter_in;
    p.min_iter = min_iter_in;
    p.dp_thresh = dp_thresh_in;
    p.dr_thresh = dr_thresh_in;
    p.res_thresh = res_thresh_in;
    p.p_samp_s = padval_in;
    p.patove = patove_in;
    p.usefbcon = usefbcon_in ? 1 : 0;
    p.costfct = costfct_in;
    p.patnorm = patnorm_in;
    p.usetvref = usetvref_in ? 1 : 0;
    p.tv_alpha = tv_alpha_in;
    p.tv_gamma = tv_gamma_in;
    p.tv_delta = tv_delta_in;
    p.tv_innerit = tv_innerit_in;
    p.tv_solverit = tv_solverit_in;
    p.tv_sor = tv_sor_in;
    p.verbosity = verbosity_in;
    const int rc = ofdis_oflow_compute(im_ao_in, im_ao_dx_in, im_ao_dy_in, im_bo_in, im_bo_dx_in, im_bo_dy_in,
                                       imgpadding_in, outflow, initflow, width_in, height_in, &p);
    if (rc != OFDIS_OK) throw OFDisError(rc, "OFC::OFClass");
  }
};

}  // namespace OFC

#endif  // OFDIS_OFLOW_HPP
