// ofdis_internal.h -- kernel argument blocks and launchers shared by ofdis_kernels.hip and the runtime.
//
// Device data layout (per batch of n frame pairs, all float32 unless noted):
//   pyramid level s   : [2n][H_s][W_s][noc]  padded by `pad` (W_s = w_s + 2 pad); frames 0..n-1 are
//                       image a, n..2n-1 image b (same layout as OFClass's inputs, oflow.h:99-106)
//   patch state       : p_iter [n][npatch][nop], pweight [n][npatch][novals]
//   flow level s      : planar [n][nop][h_s][w_s]  (wx, wy)
//   TV scratch        : planar [n][plane][h][w] for du, dv, mask, a11, a12, a22, b1, b2, sh, sv,
//                       t/dt, and the 8 derivative images (noc planes each)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ofdis {

struct LevelGeom {
  int w, h;        // unpadded level size
  int pad;         // imgpadding
  int W, H;        // padded size
  int nopw, noph, npatch, offw, offh;
  float tmp_lb, tmp_ubw, tmp_ubh;
  int level;       // scale index s
};

struct PyrBaseArgs {
  const uint8_t *img_a, *img_b;  // [n][H0][W0][noc]
  int n, W0, H0, noc;
  int padl, padt;                // divisibility padding offsets (floor halves)
  int log2s;                     // level of the output (sc_l)
  int w, h;                      // output level size
  float *out;                    // unpadded level [2n][h][w][noc]
  int rgb_sad;                   // colour, 2^l = 4..16: k_pyr_base_rgb (option pyr_rgb)
};

// SELECTCHANNEL 2 (run_dense.cpp:139-148): level 0 = Sobel gradient magnitude of the divisibility-padded
// intensity frame, sqrt(dx*dx + dy*dy) (exact up to the correctly rounded sqrt: dx, dy are multiples of
// 1/8 below 2^10, their squares and sum exact in fp32).
struct PyrGradmagArgs {
  const uint8_t *img_a, *img_b;  // [n][H0][W0]
  int n, W0, H0, padl, padt, Wp, Hp;
  float *out;                    // [2n][Hp][Wp]
};

struct PyrDownArgs {
  const float *src;  // [2n][2h][2w][noc]
  float *dst;        // [2n][h][w][noc]
  int n2, w, h, noc;
};

struct PyrPadGradArgs {
  const float *lvl;        // unpadded [2n][h][w][noc]
  float *img, *dx, *dy;    // padded [2n][H][W][noc]
  int n2, w, h, noc, pad;
  int per_value;           // colour: one thread per value (k_pyr_pad_grad_v; option pad_grad_v)
};

struct PatchArgs {
  const float *img_a, *dx_a, *dy_a, *img_b;  // padded level, frame stride = W*H*noc
  const float *prev;                          // coarse flow or NULL
  long prev_frame_stride;                     // floats per frame
  int prev_comp_stride, prev_elem_stride, prev_w;
  float *p_iter;                              // [n][npatch][nop]
  float *pweight;                             // [n][npatch][novals]
  int n, nop, noc, p, novals, steps;
  int costfct, patnorm, max_iter, min_iter;
  float dp_thresh_sq, dr_thresh, res_thresh, outlierthresh;
  float outlier_sq;                           // largest s with sqrt_rn(s) <= outlierthresh: the outlier test
                                              // sqrt(ex^2 + ey^2) > thresh (patch.cpp:197) without the sqrt
  int camlr;
  int wave_per_patch;                         // 1: force the one-wave-per-patch kernel (A/B testing)
  int generic;                                // 1: force the any-shape kernel k_patchg (parity testing)
  int window;                                 // LDS-windowed bilinear taps (k_patchw) where the shape has one
  int quad;                                   // four lanes per patch (k_patchq) where the shape has that form
  int x16;                                    // sixteen lanes per patch (k_patchx) for RGB p = 12 (2: exact evaluations)
  int absw;                                   // 1: write the aggregation weight of every patch pixel into the slot
                                              // planes (agg_plane_off) instead of the loss weights, where the kernel
                                              // can (launch_patch returns whether it did)
  int aslots;                                 // A = (p - 1) / steps + 1: slot planes per axis
  int buf32;                                  // the image array of the launch spans < 2^32 bytes (32-bit buffer offsets)
  int fdiv;                                   // 1: the LLT solves divide by FMA-corrected pivot reciprocals (llt_rcp)
  int maxres;                                 // 1: res_thresh = 0 and min_iter >= max_iter: the four- and sixteen-lane
                                              // kernels test the largest |w| > 0 instead of mean |w| > res_thresh
  int stage;                                  // 0 the whole patch optimisation; timing diagnostics (verbosity 2):
                                              // 1 construction only (pconst), 2 + initialisation (pinit)
  LevelGeom g;
};

struct AggArgs {
  const float *p_iter, *pweight;
  const float *cg_p_iter, *cg_pweight;  // complementary (backward) grid for usefbcon, or NULL
  float *flow;  // planar [n][nop][h][w]
  int n, nop, noc, p, novals, steps;
  int absw;     // 1: pweight holds the patch kernel's aggregation weights as slot planes ([n][A * A][h][w]), 0: loss weights
  int aslots;   // A
  int stage;    // k_aggregate: the tile's patch displacements staged in LDS (option agg_stage)
  LevelGeom g;
};

// TV arrays use a SKEWED (anti-diagonal-major) layout: pixel (x, y) of a w x h level lives at
// (x + y) * h + y of a plane of sp = (w + h - 1) * h floats, so the pixels of one wavefront step
// t = x + y are contiguous (lane = row y).  Both the stencil kernels (neighbours at +-h, +-(h+1)) and the
// exact-order SOR wavefront read it fully coalesced.
struct TvArgs {
  // level images (padded interleaved) and flow
  const float *img_a, *img_b;
  float *flow;                 // planar row-major [n][nop][h][w]  (wx, wy)
  float *wxs, *wys;            // skewed copies of the flow at the start of the level [n][sp]
  float *du, *dv, *mask, *s;   // skewed [n][sp]
  float *coef;                 // AoS per pixel: OF (a11,a12,a22,b1)(b2,sh,sv,-) = 8 floats; DE (a11,b1,sh,sv)
  float *t, *dt;               // skewed [n][noc][sp]
  float *Ix, *Iy, *Iz, *Ixx, *Ixy, *Iyy, *Ixz, *Iyz;  // skewed [n][noc][sp]
  long sp;                     // skewed plane stride: skew_slots + 64 dump slots (SOR), multiple of 4
  int wrap;                    // rows folded modulo w (h <= w): skew_slots = w * h, else (w + h - 1) * h
  int skew_slots;
  int n, nop, noc, w, h, pad, W;
  float quarter_alpha, hdo3, hgo3, omega;
  int first_iter;              // uu = wx (memcpy) on the first inner iteration
  int solverit;
  int camlr;
  int sor_generic;             // force the generic global-memory SOR wavefront (A/B testing)
  int sor_variant;             // 0 auto (sweep-per-wave when it fits), 1 register pipeline (A/B testing)
  int sor_point;               // OpenMP build: point SOR on the raw system (solver.c:34-78) for every size
  int sor_cring;               // lean SOR: coefficients loaded once by sweep 0, passed on through LDS (S <= 3);
                               // 2: the ring sized to the level's row groups
  int sor_rows2;               // lean SOR with two rows per lane for levels of 321..640 rows (else the pipeline)
  int smsys;                   // smoothness + system in one launch (k_tv_smsys)
  int prepd;                   // prep + derivatives in one launch (k_tv_prepd, intensity images; 0: three launches)
  int smsys2d;                 // ... and on 2-D tiles for tall levels (k_tv_smsys2d; 0: two launches there, A/B)
  int smsys_prefetch;          // k_tv_smsys, intensity images: derivative images loaded before the staging
  int smsys_small;             // k_tv_smsys: ~1 pixel per thread when a launch cannot fill the chip
  int smsys_march;             // tall levels: the register march k_tv_smsys_m (takes precedence over smsys2d)
  int smsys_deriv;             // row-block k_tv_smsys, intensity images: Ixx .. Iyz computed from staged Ix, Iy, Iz
  int prepd_df;                // smsys_deriv levels: the prep launch warps on a 2-pixel halo, all channels at once (k_tv_prepd_df)
                               // (k_tv_prepd then writes only Ix, Iy, Iz of the derivative planes); set by the
                               // runtime only where tv_deriv_fused() holds
  int sor_redblack;            // opt-in red-black SOR order (a different iteration: EPE-gated, not bit-exact)
  int lat;                     // sor_mode = 1 latency form (tv_level_rb_ok): k_tv_prepd writes the flow copies and
                               // the eight derivative planes in the colour-split entry layout (lat_idx) that
                               // k_tv_level_rb reads
};

struct UpArgs {
  const float *flow;  // planar [n][nop][hl][wl]
  float *out;         // [n][H0][W0][nop]
  int n, nop, wl, hl, log2s, W0, H0, offx, offy;
  int nt_store;       // non-temporal output stores (A/B option "nt_store")
  int form;           // nop = 2: 0 k_upsample_rows, 1 k_upsample_h<4>, 2 k_upsample_h<8> (option "up_form")
};

// Initial flow (run_dense.cpp:356-379): full-resolution [n][H0][W0][nop] -> replicate-padded, x sc,
// INTER_AREA by k = 2^(sc_f+1) -> [n][ho][wo][nop] interleaved (OFClass's initflow layout).
struct InitArgs {
  const float *init;  // [n][H0][W0][nop]
  float *out;         // [n][ho][wo][nop]
  int n, nop, W0, H0, padl, padt, log2k, wo, ho;
  float sc, scale;    // 2^-(sc_f+1), 1 / k^2
};

void launch_init_area(const InitArgs &a, hipStream_t s);
void warm_kernels_module(hipStream_t s);  // one empty launch per kernel translation unit: loads its code object
void warm_tvrb_module(hipStream_t s);
void launch_pyr_base(const PyrBaseArgs &a, hipStream_t s);
void launch_pyr_gradmag(const PyrGradmagArgs &a, hipStream_t s);
void launch_pyr_down(const PyrDownArgs &a, hipStream_t s);
void launch_pyr_pad_grad(const PyrPadGradArgs &a, hipStream_t s);
bool launch_patch(const PatchArgs &a, hipStream_t s);  // true: wrote aggregation weights (PatchArgs::absw)
void launch_aggregate(const AggArgs &a, hipStream_t s);
void launch_tv_prep(const TvArgs &a, hipStream_t s);
void launch_tv_deriv1(const TvArgs &a, hipStream_t s);
void launch_tv_deriv2(const TvArgs &a, hipStream_t s);
bool tv_prepd_ok(const TvArgs &a);
void launch_tv_prepd(const TvArgs &a, hipStream_t s);
void launch_tv_smooth(const TvArgs &a, hipStream_t s);
void launch_tv_system(const TvArgs &a, hipStream_t s);
bool tv_smsys_ok(const TvArgs &a);
bool tv_deriv_fused(const TvArgs &a);  // the level's derivative filters can move into k_tv_smsys (smsys_deriv)
void launch_tv_smsys(const TvArgs &a, hipStream_t s);
void launch_tv_sor(const TvArgs &a, hipStream_t s);
bool tv_level_rb_ok(const TvArgs &a);  // ofdis_tvrb.hip
void launch_tv_level_rb(const TvArgs &a, int n_inner, hipStream_t s);
void launch_tv_final(const TvArgs &a, hipStream_t s);
void launch_upsample(const UpArgs &a, hipStream_t s);

}  // namespace ofdis
