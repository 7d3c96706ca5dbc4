/*
 * ofdis_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the lordnn/OF_DIS hot path, used as the parity checker for the HIP path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
 * (of_dis_amd/libofdis.so) never links or calls it.
 *
 * Pinning: the FDF1.0.1 part (warp, derivatives, smoothness, data term, laplacian, SOR) is checked
 * bit-for-bit against the reference's own FDF1.0.1 sources compiled by oracle/Makefile into
 * oracle/_ref/ (tests/test_oracle_ref.py).  The DIS part (patch.cpp / patchgrid.cpp / oflow.cpp)
 * needs Eigen, which is absent, so it is pinned by known-answer tests only; the OpenCV-side
 * stages (pyramid, INTER_LINEAR upsample) are restatements of OpenCV's documented generic
 * paths with OpenCV absent: parity of those stages w.r.t. OpenCV is unpinned.
 */
#ifndef OFDIS_ORACLE_H
#define OFDIS_ORACLE_H

#include <stdint.h>
#include "../include/ofdis.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Eigen 3.3/3.4 SSE redux order (2 packet accumulators x 4 lanes, then (l0+l2)+(l1+l3)). */
float ofo_eigen_sum(const float *x, int n);

/* run_dense.cpp:181-184 and :226-295 */
int ofo_auto_first_scale(int imgwidth, int fratio, int patchsize);
int ofo_params_oppoint(ofdis_params *p, int oppoint, int width_org, int mode, int noc);

/* Divisibility padding amounts (run_dense.cpp:299-312). */
void ofo_divisibility_pad(int width, int height, int sc_f, int *padw, int *padh);

/* Pyramid of ONE image (run_dense.cpp:131-179) on an already divisibility-padded u8 image.
 * Writes levels s in [sc_l, sc_f] (arrays indexed by s; entries below sc_l untouched), each
 * padded by imgpadding: (w_s+2pad)*(h_s+2pad)*noc floats. */
int ofo_build_pyramid(const uint8_t *img, int width, int height, int noc, int sc_f, int sc_l, int imgpadding,
                      float **img_pyr, float **dx_pyr, float **dy_pyr);

/* Same; gradmag = SELECTCHANNEL 2 (run_dense.cpp:139-148): level 0 is the Sobel gradient magnitude. */
int ofo_build_pyramid_ex(const uint8_t *img, int width, int height, int noc, int sc_f, int sc_l, int imgpadding,
                         int gradmag, float **img_pyr, float **dx_pyr, float **dy_pyr);

/* OFC::OFClass (oflow.cpp:31-338).  Optional per-scale capture of the flow after aggregation
 * and after TV refinement (arrays indexed by scale, w_s*h_s*nop interleaved; may be NULL). */
int ofo_oflow(const float *const *im_ao, const float *const *im_ao_dx, const float *const *im_ao_dy,
              const float *const *im_bo, const float *const *im_bo_dx, const float *const *im_bo_dy,
              int imgpadding, float *outflow, const float *initflow, int width, int height,
              const ofdis_params *p, float *const *cap_dis, float *const *cap_tv);

/* flow *= 2^sc_l; cv::resize(x 2^sc_l, INTER_LINEAR); crop (run_dense.cpp:407-415). */
int ofo_upsample_crop(const float *flow_l, int wl, int hl, int nop, int scale_log2, int padw, int padh,
                      int width_org, int height_org, float *out);

/* Whole pipeline for one frame pair of u8 images [h][w][noc]: output [h][w][nop]. */
int ofo_run_u8(const uint8_t *img_a, const uint8_t *img_b, int width, int height, const ofdis_params *p,
               float *flow_out, float *const *cap_dis, float *const *cap_tv);
/* Same with an optional full-resolution initial flow [h][w][nop] (run_dense.cpp:293-294, 302, 356-379:
 * divisibility 2^(sc_f+1), replicate pad, x 2^-(sc_f+1), INTER_AREA down to the coarsest scale - 1). */
int ofo_run_u8_init(const uint8_t *img_a, const uint8_t *img_b, const float *init, int width, int height,
                    const ofdis_params *p, float *flow_out, float *const *cap_dis, float *const *cap_tv);
int ofo_run_u8_stages(const uint8_t *img_a, const uint8_t *img_b, const float *init, int width, int height,
                      const ofdis_params *p, float *flow_out, float *const *cap_dis, float *const *cap_tv,
                      double *stage_s);
void ofo_init_flow_area(const float *init, int width, int height, int nop, int padw, int padh, int sc_f,
                        float *out);

/* One VarRefClass run at scale `level` on padded interleaved level images; flow w*h*nop in place. */
int ofo_refine_level(const float *im_ao, const float *im_bo, int w, int h, int imgpadding, int level,
                     const ofdis_params *p, float *flow);

/* ---- FDF1.0.1 restatements on planar arrays (stride = width), exported for pinning ---- */
/* image_warp (opticalflow_aux.c:31-75): noc planes of w*h */
void ofo_image_warp(float *dst, float *mask, const float *src, const float *wx, const float *wy, int w, int h,
                    int noc);
/* get_derivatives (opticalflow_aux.c:77-132) per channel plane */
void ofo_get_derivatives(const float *im1, const float *im2, int w, int h, int noc, float *dx, float *dy,
                         float *dt, float *dxx, float *dxy, float *dyy, float *dxt, float *dyt);
/* compute_smoothness (opticalflow_aux.c:138-187) */
void ofo_compute_smoothness(float *dst_h, float *dst_v, const float *uu, const float *vv, int w, int h,
                            float quarter_alpha);
/* sub_laplacian (opticalflow_aux.c:194-223) */
void ofo_sub_laplacian(float *dst, const float *src, const float *wh, const float *wv, int w, int h);
/* compute_data (opticalflow_aux.c:408-594), gray (noc=1) and RGB (noc=3) variants */
void ofo_compute_data(float *a11, float *a12, float *a22, float *b1, float *b2, const float *mask,
                      const float *du, const float *dv, const float *Ix, const float *Iy, const float *Iz,
                      const float *Ixx, const float *Ixy, const float *Iyy, const float *Ixz, const float *Iyz,
                      int w, int h, int noc, float half_delta_over3, float half_gamma_over3);
/* compute_data_DE (opticalflow_aux.c:601-747) */
void ofo_compute_data_de(float *a11, float *b1, const float *mask, const float *du, const float *Ix,
                         const float *Iy, const float *Iz, const float *Ixx, const float *Ixy, const float *Iyy,
                         const float *Ixz, const float *Iyz, int w, int h, int noc, float half_delta_over3,
                         float half_gamma_over3);
/* sor_coupled (solver.c:83-433) incl. its small-image fallback (solver.c:34-78) */
void ofo_sor_coupled(float *du, float *dv, float *a11, float *a12, float *a22, const float *b1, const float *b2,
                     const float *h, const float *v, int w, int hgt, int iterations, float omega);
/* sor_coupled_slow_but_readable (solver.c:34-78), the OpenMP build's optical-flow SOR */
void ofo_sor_point_of(float *du, float *dv, const float *a11, const float *a12, const float *a22, const float *b1,
                      const float *b2, const float *h, const float *v, int w, int hgt, int iterations, float omega);
/* sor_coupled_slow_but_readable_DE (solver.c:439-471) */
void ofo_sor_point_de(float *du, const float *a11, const float *b1, const float *h, const float *v, int w,
                      int hgt, int iterations, float omega);
/* Red-black order of the same updates (NOT a reference function: the checker of the GPU's opt-in sor_mode = 1).
 * ofo_set_sor_order(1) makes every later refinement (ofo_run_u8*, ofo_refine_level) use it; 0 restores solver.c's. */
void ofo_set_sor_order(int order);
int ofo_get_sor_order(void);
void ofo_sor_rb_of(float *du, float *dv, float *a11, float *a12, float *a22, const float *b1, const float *b2,
                   const float *h, const float *v, int w, int hgt, int iterations, float omega);
void ofo_sor_rb_de(float *du, const float *a11, const float *b1, const float *h, const float *v, int w, int hgt,
                   int iterations, float omega);

#ifdef __cplusplus
}
#endif

#endif
