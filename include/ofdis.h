/*
 * ofdis.h -- C-ABI of the MI355X-native DIS optical-flow / stereo-depth hot path.
 *
 * This is the drop-in boundary for lordnn/OF_DIS.  Every entry point below names the
 * reference interface it replaces (paths relative to the reference tree).  Plain C types
 * only: no torch, no HIP types in any signature (device pointers and streams are void*).
 *
 * Library: of_dis_amd/libofdis.so (built by of_dis_amd/csrc/Makefile, hipcc --offload-arch=gfx950).
 */
#ifndef OFDIS_H
#define OFDIS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OFDIS_ABI_VERSION 2

/* Status codes.  The reference has no error channel (it exit(1)s on OOM, FDF1.0.1/image.cpp:26-27,
 * and never validates parameters); every entry point here returns one of these instead. */
typedef enum ofdis_status {
  OFDIS_OK = 0,
  OFDIS_ERR_INVALID_ARGUMENT = 1, /* bad pointer / size / parameter combination          */
  OFDIS_ERR_UNSUPPORTED = 2,      /* valid in the reference but not implemented here       */
  OFDIS_ERR_OUT_OF_MEMORY = 3,    /* device or host allocation failed                      */
  OFDIS_ERR_DEVICE = 4,           /* a HIP runtime call failed                             */
  OFDIS_ERR_NO_DEVICE = 5,        /* no gfx950 device visible                              */
  OFDIS_ERR_IO = 6                /* file could not be opened / read / written             */
} ofdis_status;

/* SELECTMODE of the reference build (CMakeLists.txt:36-61): 1 = optical flow, 2 = stereo depth. */
enum { OFDIS_MODE_OF = 1, OFDIS_MODE_DE = 2 };

/*
 * Parameters of one run.  Mirrors OFC::optparam's explicitly-set fields (oflow.h:45-66) plus
 * the two compile-time switches SELECTMODE / SELECTCHANNEL, which are runtime fields here.
 * Values are taken exactly as the reference constructor receives them (oflow.cpp:80-104):
 * dp_thresh is NOT squared by the caller, steps/outlier threshold/novals are derived.
 */
typedef struct ofdis_params {
  int mode;         /* OFDIS_MODE_OF (nop = 2) or OFDIS_MODE_DE (nop = 1)                 */
  int noc;          /* channels: 1 = intensity, 3 = BGR interleaved (SELECTCHANNEL 1 / 3)  */
  int sc_f;         /* coarsest scale                                                     */
  int sc_l;         /* finest scale                                                       */
  int max_iter;     /* patch iterations                                                   */
  int min_iter;
  float dp_thresh;  /* early-stop on |delta_p| ratio (squared internally, oflow.cpp:87)    */
  float dr_thresh;  /* early-stop on residual ratio                                        */
  float res_thresh; /* early-stop on mean absolute residual                                */
  int p_samp_s;     /* patch edge length (even)                                            */
  float patove;     /* patch overlap in [0,1)                                              */
  int usefbcon;     /* forward-backward merging (patchgrid.cpp:277-375)                    */
  int costfct;      /* 0 L2, 1 L1, 2 pseudo-Huber (10 = NCC is unimplemented upstream)     */
  int patnorm;      /* mean-normalise patches                                              */
  int usetvref;     /* variational refinement                                              */
  float tv_alpha, tv_gamma, tv_delta;
  int tv_innerit;   /* TV outer iterations per level = tv_innerit * (level + 1)            */
  int tv_solverit;  /* SOR sweeps per TV iteration                                         */
  float tv_sor;     /* SOR relaxation omega                                                */
  int verbosity;    /* 0 silent, 1 total time, 2 per-scale TIME lines (oflow.cpp:297,336)  */
  /* Reference build variants (compile-time there, runtime fields here; 0 = the default build): */
  int omp_build;    /* USE_OPENMP build (CMakeLists.txt:4,17-23): optical-flow refinement runs
                       sor_coupled_slow_but_readable, point SOR (refine_variational.cpp:202-203,
                       solver.c:34-78), in its single-thread order (the multi-threaded build races rows) */
  int gradmag;      /* SELECTCHANNEL 2 (run_dense.cpp:139-148, 194-197): the pyramid is built on each
                       frame's Sobel gradient magnitude instead of its intensity (noc must be 1)          */
} ofdis_params;

/* ------------------------------------------------------------------ parameters */

int ofdis_abi_version(void);
const char *ofdis_status_string(int status);

/* AutoFirstScaleSelect (run_dense.cpp:181-184). */
int ofdis_auto_first_scale(int imgwidth, int fratio, int patchsize);

/* Operating points 1-4 with automatic coarsest scale (run_dense.cpp:226-268). */
int ofdis_params_oppoint(ofdis_params *p, int oppoint, int width_org, int mode, int noc);

/* The 20 explicit positional parameters of run_dense.cpp:270-295, as strings (argv[4..23]). */
int ofdis_params_from_strings(ofdis_params *p, int count, const char *const *values, int mode, int noc);

/* Validation the reference never does: p even and >= 2, p*p*noc divisible by 4 (patch.cpp:230),
 * 0 <= sc_l <= sc_f, width/height divisible by 2^sc_f, costfct in {0,1,2}, noc in {1,3}, gradmag only
 * with noc = 1. */
int ofdis_params_validate(const ofdis_params *p, int width, int height, int imgpadding);

/* ------------------------------------------------------------------ library boundary */

/*
 * OFC::OFClass::OFClass (oflow.h:99-126, oflow.cpp:31-338) with host pointers.
 * im_ao[s] .. im_bo_dy[s] for s in [sc_l, sc_f]: padded (w_s + 2*imgpadding) x (h_s + 2*imgpadding)
 * x noc float arrays (images replicate-padded, gradients zero-padded); entries below sc_l may be NULL.
 * outflow: (width >> sc_l) * (height >> sc_l) * nop floats, interleaved.  initflow: NULL or
 * (width >> (sc_f+1)) * (height >> (sc_f+1)) * nop floats.  Runs on the default device; blocking.
 */
int ofdis_oflow_compute(const float *const *im_ao, const float *const *im_ao_dx, const float *const *im_ao_dy,
                        const float *const *im_bo, const float *const *im_bo_dx, const float *const *im_bo_dy,
                        int imgpadding, float *outflow, const float *initflow, int width, int height,
                        const ofdis_params *p);

/* ------------------------------------------------------------------ batched device path */

typedef struct ofdis_context ofdis_context;

/* One context per GPU (and per host thread using it).  No hidden globals. */
int ofdis_context_create(int device, ofdis_context **out);
void ofdis_context_destroy(ofdis_context *ctx);

/*
 * Whole run_dense.cpp main() hot path for a batch of n independent frame pairs, all on device:
 * divisibility padding (run_dense.cpp:299-312) -> pyramid + Sobel gradients (:131-179) ->
 * OFClass (:392-401) -> x 2^sc_l + INTER_LINEAR upsample + crop (:407-415).
 * img_a/img_b: device u8 [n][height][width][noc] (BGR order when noc = 3).
 * flow_out: device float [n][height][width][nop] (nop = 2 OF, 1 DE).
 * stream: hipStream_t, or NULL for the legacy default stream (torch's default): the call is then ordered
 * after the work already queued there and that stream's later work after the call.  Asynchronous w.r.t. the
 * host.  All calls on one context share its workspaces: a call waits for the previous call of the context
 * whatever stream either was issued on.  A batch is split into launches of at most
 * ofdis_max_frames_per_launch() frames.  n < 1, a non-positive size or a NULL image / flow pointer returns
 * OFDIS_ERR_INVALID_ARGUMENT before anything is enqueued (the context stays usable).
 */
int ofdis_run_batch_u8(ofdis_context *ctx, const uint8_t *img_a, const uint8_t *img_b, int n, int width,
                       int height, const ofdis_params *p, float *flow_out, void *stream);

/* Same with host buffers (CLI path; synchronous). */
int ofdis_run_batch_u8_host(ofdis_context *ctx, const uint8_t *img_a, const uint8_t *img_b, int n, int width,
                            int height, const ofdis_params *p, float *flow_out);

/* The same with an initial flow per pair (OFClass's initflow, oflow.h:106 / oflow.cpp:215-217, fed the way
 * run_dense.cpp's commented-out code prepares it, :293-294, :302, :356-379): init_flow is device float
 * [n][height][width][nop] at full resolution, or NULL (= ofdis_run_batch_u8).  With an initial flow the
 * frames are padded to a multiple of 2^(sc_f+1) and the flow is replicate-padded, scaled by 2^-(sc_f+1)
 * and INTER_AREA-reduced to the grid below the coarsest scale -- e.g. the previous frame's output for
 * video (temporal propagation). */
int ofdis_run_batch_u8_init(ofdis_context *ctx, const uint8_t *img_a, const uint8_t *img_b, const float *init_flow,
                            int n, int width, int height, const ofdis_params *p, float *flow_out, void *stream);
int ofdis_run_batch_u8_init_host(ofdis_context *ctx, const uint8_t *img_a, const uint8_t *img_b,
                                 const float *init_flow, int n, int width, int height, const ofdis_params *p,
                                 float *flow_out);

/* Device pyramid only (run_dense.cpp:131-179 + :299-312): writes, for each level s in [sc_l, sc_f],
 * padded image/dx/dy of frame 0 to host arrays (same layout as ofdis_oflow_compute's inputs). */
int ofdis_pyramid_u8_host(ofdis_context *ctx, const uint8_t *img, int width, int height, const ofdis_params *p,
                          int imgpadding, float *const *img_pyr, float *const *dx_pyr, float *const *dy_pyr);

/* Per-stage capture for parity tests: when set, the next run copies frame 0's flow at scale s after
 * patch aggregation (dis_flow[s]) and after variational refinement (tv_flow[s]), each
 * w_s*h_s*nop interleaved floats, into these host arrays (entries may be NULL).  A capturing run issues
 * the whole batch as one launch on one stream whatever the "streams" / "chunk" options; a batch larger
 * than ofdis_max_frames_per_launch() returns OFDIS_ERR_UNSUPPORTED while a capture is set. */
int ofdis_context_set_stage_capture(ofdis_context *ctx, float *const *dis_flow, float *const *tv_flow, int nscales);

/* Tuning / A-B switches:
 *   "sor_generic" (0/1): force the generic global-memory SOR wavefront;
 *   "sor_pipe" (0/1):    force the one-wave-per-row-group register pipeline (the default for tall levels)
 *                        instead of the sweep-per-wave SOR;
 *   "sor_cring" (0..3, default 2): in the sweep-per-wave SOR, sweep 0 loads each pixel's coefficients once and
 *                        hands them to the later sweeps through LDS (solverit <= 3); 2: the LDS ring sized to
 *                        the level's rows (more frames per CU at 3 sweeps), and in launches with more frames than
 *                        CUs the lanes outside the frame load a slot of their wave's in-frame run (fewer fetched
 *                        lines, one v_med3 per load); 3: that load form in every launch; 1: sized to the
 *                        workgroup limit;
 *   "sor_rows2" (0/1, default 1): levels too tall for one row per lane in a 1024-thread workgroup run the
 *                        sweep-per-wave SOR with two rows per lane -- 321..640 rows at 3 sweeps, 513..1024 at
 *                        2 (else the register pipeline);
 *   "smsys" (0/1, default 1): smoothness and system of a TV iteration in one launch;
 *   "smsys2d" (0/1/2, default 2): the fused launch on 2-D tiles for levels taller than 256 rows (0: two
 *                        launches there; 2 = automatic: on for calls of fewer than 512 pairs);
 *   "smsys_prefetch" (0/1, default 1): the fused launch (levels up to 256 rows, intensity images) issues a
 *                        thread's derivative-image loads before the staging, not after two barriers;
 *   "smsys_small" (0/1, default 1): a fused launch that cannot fill the chip (fewer than 4096 row blocks:
 *                        a few pairs per call) takes ~1 pixel per thread (>= 4 rows per block) instead of 4;
 *   "smsys_deriv" (0/1, default 1): where "prepd" and the fused launch (levels up to 256 rows, intensity images)
 *                        or the register march (taller levels, intensity and colour images) run, the system kernel
 *                        filters Ixx, Ixy, Iyy, Ixz, Iyz from Ix, Iy, Iz and the prep launch does not write those
 *                        five planes (per channel);
 *   "pyr_rgb" (0/1, default 1): colour images, pyramid base levels 2..4: dword loads and per-channel masked byte
 *                        sums (v_sad_u8) instead of the byte loop;
 *   "pad_grad_v" (0/1, default 1): colour images: the pyramid's pad + Sobel launch runs one thread per value
 *                        (0: one per pixel, the channels inside the thread);
 *   "agg_stage" (0/1, default 1): the aggregation stages the displacements of the patches covering each 64 x 16
 *                        tile in LDS (0: every pixel gathers them from the patch array);
 *   "prepd_df" (0/1, default 1): on those levels the prep launch warps a 2-pixel halo with every channel in one pass
 *                        and writes Ix, Iy, It only (k_tv_prepd_df; 0: k_tv_prepd's 4-pixel halo, channel by channel);
 *   "smsys_march" (0/1, default 1): levels taller than 256 rows run smoothness + system as a register march
 *                        (one wave per 60 columns x 64 rows, no LDS; takes precedence over smsys2d);
 *   "prepd" (0..2, default 2): image warp, temporal images and the derivative filters of a level in one launch
 *                        (1: intensity images only, colour images in three launches; 0: three launches);
 *   "sor_mode" (0/1, default 0): 0 = sor_coupled's exact lexicographic order (the reference's bits);
 *                        1 = the latency mode, red-black order (every half-sweep fully parallel):
 *                        levels of at most 8192 pixels run their whole inner loop -- smoothness, system, 2 x solverit
 *                        half-sweeps per inner iteration -- and the flow update in one launch of one workgroup per
 *                        frame (k_tv_level_rb), larger levels the system launches and one launch per half-sweep.
 *                        A different iteration -- NOT the reference's bits: bit-exact against the oracle's
 *                        red-black restatement, end-point error gated against the exact path; the one option
 *                        that changes results.  For calls that cannot fill the chip (one pair, a few dozen);
 *   "wave_per_patch" (0/1): one wave64 per patch instead of eight lanes per patch (patches of at most
 *                        448 values; larger ones always run the any-shape kernel);
 *   "patch_window" (0/1, default 1): p = 8 / 12 patches read their bilinear taps from an LDS copy of the
 *                        sample window (0: eight-lane patches gathering the taps from the L1 cache);
 *   "patch_quad" (0/1, default 1): windowed gray patches (p = 8 / 12) on four lanes per patch, the Eigen
 *                        slot pairs packed (0: eight lanes per patch);
 *   "patch_x16" (0..2, default 1): windowed RGB p = 12 patches on sixteen lanes per patch, the Eigen slot chains
 *                        folded in block order on eight owner lanes (0: eight lanes per patch; 2: sixteen lanes,
 *                        every evaluation on the exact square-root form -- parity testing of the fallback);
 *   "patch_absw" (0/1, default 1): without usefbcon, the four- and sixteen-lane patch kernels store each patch
 *                        pixel's aggregation weight into slot planes ([n][A*A][h][w], A = (p-1)/steps + 1) instead
 *                        of their loss weights, so the aggregation reads coalesced plane rows (0: loss weights);
 *   "patch_buf" (0/1, default 1): gray p = 12 patch windows by buffer loads with 32-bit offsets where the level's
 *                        image array spans less than 4 GiB (0: 64-bit address arithmetic per load);
 *   "patch_fdiv" (0/1, default 1): the 2x2 / 1x1 LLT solves of every patch iteration divide by one correctly
 *                        rounded reciprocal of each pivot per patch plus two FMAs (exact by Markstein's theorem in
 *                        the range the kernels check; tools/divcheck_l.c), IEEE divisions outside it (0: IEEE always);
 *   "patch_maxres" (0/1, default 1): with res_thresh = 0 and min_iter >= max_iter (every op-point) the four- and
 *                        sixteen-lane patch kernels stop on the largest |w| of an evaluation being 0 instead of
 *                        summing |w| (the same decision; NaN and tiny terms redo the evaluation with the sum);
 *   "patch_generic" (0/1, default 0): every patch shape on the any-shape kernel (runtime value loops: the
 *                        default for p*p*noc > 448, e.g. RGB p >= 14, gray p >= 22);
 *   "nt_store" (0/1, default 0): write the full-resolution flow with non-temporal stores;
 *   "up_form" (0..3, default 3): optical-flow upsample: 1 / 2 = each staged source row's horizontal taps once per
 *                        column for blocks of 4 / 8 output rows, 0 = once per output row that reads them (round 4),
 *                        3 = 1 on frames at least 1024 wide for calls on two or more streams or of fewer than
 *                        1024 pairs, else 0 (the faster of the two end to end in each measured regime);
 *   "graph" (0/1/2, default 1): replay a batch as one captured HIP graph while its pointers, sizes and
 *                        parameters repeat (re-captured when they change); 1 captures single-stream
 *                        batches, 2 also the multi-stream ones (chunks forked over lanes and joined);
 *   "streams" (0-16, default 0 = automatic: 2 from 256 pairs, else 1): a batch is cut into chunks that run
 *                        round-robin on that many HIP streams with separate workspaces, overlapping one
 *                        chunk's latency-bound wavefront with another's streaming kernels (1 stream and
 *                        several chunks: the chunks run one after the other);
 *   "chunk" (frames per chunk, 0 to 2^30, default 0 = the batch split evenly over the streams);
 * Setting any option drops the captured graph.  Unknown keys and out-of-range values return
 * OFDIS_ERR_INVALID_ARGUMENT.  Apart from "sor_mode", results never depend on these settings. */
int ofdis_context_set_option(ofdis_context *ctx, const char *key, int value);

/* Largest number of frame pairs one launch of the refinement kernels takes at this size (their plane groups
 * are addressed with 32-bit offsets: frames * noc * plane < 2^30 floats); larger batches are chunked.
 * A size at which one frame alone exceeds that (e.g. ~20k x 20k RGB with sc_l 0) returns
 * OFDIS_ERR_INVALID_ARGUMENT here and from every run entry point. */
int ofdis_max_frames_per_launch(const ofdis_params *p, int width, int height, int *frames);

/* HIP-event timing of individual kernels on the launch stream (used by bench.py for the roofline). */
int ofdis_context_enable_kernel_timing(ofdis_context *ctx, int enable);
/* Accumulated device time (ms) and launch count for kernel `name` since timing was enabled. */
int ofdis_context_kernel_time(ofdis_context *ctx, const char *name, double *total_ms, long *launches);
/* Comma-separated list of kernel names known to the timer. */
const char *ofdis_kernel_names(void);

/* Per-frame algorithmic byte counts of the §8(d) byte model for this workload. */
int ofdis_algorithmic_bytes(const ofdis_params *p, int width, int height, const char *kernel, double *bytes_per_frame);

/* ------------------------------------------------------------------ files and inputs */

/* SaveFlowFile (run_dense.cpp:17-58): "PIEH", int32 w, int32 h, w*h*nc float32 row-major. */
int ofdis_write_flo(const char *path, const float *flow, int width, int height, int nc);
/* SavePFMFile (run_dense.cpp:61-82): "Pf\n%d %d\n%f\n" with -1.0, rows bottom-up, values negated. */
int ofdis_write_pfm(const char *path, const float *depth, int width, int height);
/* ReadFlowFile (run_dense.cpp:85-129). w/h out; flow may be NULL to query the size. */
int ofdis_read_flo(const char *path, float *flow, int *width, int *height, int nc);
/* Binary PGM (P5, noc = 1) / PPM (P6, noc = 3, returned in BGR order like cv::imread). */
int ofdis_read_pnm(const char *path, uint8_t *pixels, int *width, int *height, int *noc, size_t capacity);
/* cv::imread(path, want_noc == 1 ? CV_LOAD_IMAGE_GRAYSCALE : CV_LOAD_IMAGE_COLOR) (run_dense.cpp:202-206)
 * for PNG (zlib inflate; gray / RGB / palette / alpha, 1-16 bit, Adam7; libpng's transform chain as
 * OpenCV configures it, incl. png_set_rgb_to_gray(0.299, 0.587)) and Netpbm P1-P6 (colour -> gray with
 * OpenCV's fixed-point BGR2Gray) and BMP (BmpDecoder: 1/4/8-bit palette, 16-bit 555 / 565, 24-bit, 32-bit,
 * core / info / V4 / V5 headers, bottom-up or top-down; colour -> gray by the same BGR2Gray).  Output
 * [h][w][want_noc], BGR for 3.  pixels may be NULL to query the size (PNG: from the checked chunk structure and
 * header, nothing inflated; a corrupt stream then fails the pixel call).  OFDIS_ERR_UNSUPPORTED for other formats
 * (JPEG, TIFF, RLE-compressed BMP, ...), OFDIS_ERR_IO for corrupt files. */
int ofdis_read_image(const char *path, uint8_t *pixels, int *width, int *height, int want_noc, size_t capacity);

/* Deterministic synthetic frame pair: band-limited texture + noise, frame b is frame
 * a moved along a known smooth flow (OF) or a horizontal disparity (DE).  Host buffers [h][w][noc]. */
int ofdis_synth_pair_u8(uint8_t *img_a, uint8_t *img_b, int width, int height, int noc, int frame, int mode);
/* The same texture and noise, frame b a pure translation of frame a: b(x, y) = a(x - sx, y - sy), i.e. the
 * true flow is (sx, sy) at every pixel (the known-answer setups of SURVEY §4). */
int ofdis_synth_shift_pair_u8(uint8_t *img_a, uint8_t *img_b, int width, int height, int noc, int frame, float sx,
                              float sy);

#ifdef __cplusplus
}
#endif

#endif /* OFDIS_H */
