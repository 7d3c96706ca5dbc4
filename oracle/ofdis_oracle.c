/*
 * ofdis_oracle.c -- TEST INFRASTRUCTURE ONLY (see ofdis_oracle.h).
 *
 * A clean-room, pixel-wise CPU restatement of the reference hot path.  Each function cites the
 * reference file:line it restates.  Floating-point expressions keep the reference's evaluation
 * order exactly (no FMA: build with -ffp-contract=off), so that the HIP kernels, which keep the
 * same order, can be checked bit-for-bit against this file.
 */
#include "ofdis_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <smmintrin.h>
#include <time.h>

/* ------------------------------------------------------------------ helpers */

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
/* std::max(a,b) / std::min(a,b) semantics: (a<b)?b:a and (b<a)?b:a */
static inline float stdmaxf(float a, float b) { return (a < b) ? b : a; }
static inline float stdminf(float a, float b) { return (b < a) ? b : a; }
/* _mm_min_ps / _mm_max_ps semantics: second operand when unordered or equal */
static inline float ssemin(float a, float b) { return (a < b) ? a : b; }
static inline float ssemax(float a, float b) { return (a > b) ? a : b; }

/* Eigen::DenseBase::sum() for a dynamic float vector with SSE packets (redux_impl,
 * LinearVectorizedTraversal, NoUnrolling; aligned start 0): two 4-lane packet accumulators over
 * packet pairs, res0+res1, odd trailing packet, predux = (l0+l2)+(l1+l3), scalar tail. */
static float eigen_dot(const float *x, const float *b, int n);

float ofo_eigen_sum(const float *x, int n) {
  return eigen_dot(x, NULL, n);
}

/* Eigen's vectorised redux as the SSE build runs it, on 4-float packets (every _mm_add_ps / _mm_mul_ps lane
 * rounds like the scalar operation: the same bits as the scalar restatement, at the reference's speed).
 * b == NULL: sum of x; else the sum of the packet products x * b -- what Eigen evaluates for
 * (x.array() * b.array()).sum(): the product packet is formed, then accumulated (no fused multiply-add). */
static float eigen_dot(const float *x, const float *b, int n) {
  const int aligned = (n / 4) * 4, aligned2 = (n / 8) * 8;
#define PK(i) (b ? _mm_mul_ps(_mm_loadu_ps(x + (i)), _mm_loadu_ps(b + (i))) : _mm_loadu_ps(x + (i)))
  if (aligned == 0) {
    float r = b ? x[0] * b[0] : x[0];
    for (int i = 1; i < n; ++i) r = r + (b ? x[i] * b[i] : x[i]);
    return r;
  }
  __m128 r0 = PK(0);
  if (aligned > 4) {
    __m128 r1 = PK(4);
    for (int i = 8; i < aligned2; i += 8) {
      r0 = _mm_add_ps(r0, PK(i));
      r1 = _mm_add_ps(r1, PK(i + 4));
    }
    r0 = _mm_add_ps(r0, r1);
    if (aligned > aligned2) r0 = _mm_add_ps(r0, PK(aligned2));
  }
#undef PK
  /* predux: (l0 + l2) + (l1 + l3) */
  const __m128 t = _mm_add_ps(r0, _mm_movehl_ps(r0, r0));
  float res = _mm_cvtss_f32(_mm_add_ss(t, _mm_shuffle_ps(t, t, 1)));
  for (int i = aligned; i < n; ++i) res = res + (b ? x[i] * b[i] : x[i]);
  return res;
}

/* ------------------------------------------------------------------ parameters */

/* run_dense.cpp:181-184 */
int ofo_auto_first_scale(int imgwidth, int fratio, int patchsize) {
  float r = log2f((2.0f * (float)imgwidth) / ((float)fratio * (float)patchsize));
  int v = (int)floorf(r);
  return v > 0 ? v : 0;
}

/* run_dense.cpp:226-268 */
int ofo_params_oppoint(ofdis_params *p, int oppoint, int width_org, int mode, int noc) {
  memset(p, 0, sizeof(*p));
  p->mode = mode;
  p->noc = noc;
  p->dp_thresh = 0.05f;
  p->dr_thresh = 0.95f;
  p->res_thresh = 0.0f;
  p->usefbcon = 0;
  p->patnorm = 1;
  p->costfct = 0;
  p->tv_alpha = 10.0f;
  p->tv_gamma = 10.0f;
  p->tv_delta = 5.0f;
  p->tv_innerit = 1;
  p->tv_solverit = 3;
  p->tv_sor = 1.6f;
  p->verbosity = 2;
  const int fratio = 5;
  switch (oppoint) {
    case 1:
      p->p_samp_s = 8; p->patove = 0.3f;
      p->sc_f = ofo_auto_first_scale(width_org, fratio, p->p_samp_s);
      p->sc_l = p->sc_f - 2 > 0 ? p->sc_f - 2 : 0;
      p->max_iter = p->min_iter = 16; p->usetvref = 0;
      break;
    case 3:
      p->p_samp_s = 12; p->patove = 0.75f;
      p->sc_f = ofo_auto_first_scale(width_org, fratio, p->p_samp_s);
      p->sc_l = p->sc_f - 4 > 0 ? p->sc_f - 4 : 0;
      p->max_iter = p->min_iter = 16; p->usetvref = 1;
      break;
    case 4:
      p->p_samp_s = 12; p->patove = 0.75f;
      p->sc_f = ofo_auto_first_scale(width_org, fratio, p->p_samp_s);
      p->sc_l = p->sc_f - 5 > 0 ? p->sc_f - 5 : 0;
      p->max_iter = p->min_iter = 128; p->usetvref = 1;
      break;
    case 2:
    default:
      p->p_samp_s = 8; p->patove = 0.4f;
      p->sc_f = ofo_auto_first_scale(width_org, fratio, p->p_samp_s);
      p->sc_l = p->sc_f - 2 > 0 ? p->sc_f - 2 : 0;
      p->max_iter = p->min_iter = 12; p->usetvref = 1;
      break;
  }
  return 0;
}

/* run_dense.cpp:299-312 */
void ofo_divisibility_pad(int width, int height, int sc_f, int *padw, int *padh) {
  int scfct = 1 << sc_f;
  int d = width % scfct;
  *padw = d > 0 ? scfct - d : 0;
  d = height % scfct;
  *padh = d > 0 ? scfct - d : 0;
}

/* ------------------------------------------------------------------ pyramid (run_dense.cpp:131-179) */

/* Sobel ksize 3, scale 1/8, BORDER_REFLECT_101, on an unpadded w x h x noc level.  OpenCV splits it
 * as derivative [-1 0 1] along the axis and smoothing [1 2 1]/8 across it.  Level values are
 * multiples of 4^-level below 256, so every intermediate is exact and the summation order
 * is immaterial up to level 6. */
static inline int reflect101(int i, int n) {
  if (n == 1) return 0;
  if (i < 0) return -i;
  if (i >= n) return 2 * n - 2 - i;
  return i;
}

/* One output value of the Sobel pair at (x, y), any position (reflect-101 border). */
static inline void sobel_px(const float *L, int w, int h, int noc, int x, int y, float *dx, float *dy) {
  int xm = reflect101(x - 1, w), xp = reflect101(x + 1, w);
  int ym = reflect101(y - 1, h), yp = reflect101(y + 1, h);
  for (int c = 0; c < noc; ++c) {
#define PX(xx, yy) L[((yy) * w + (xx)) * noc + c]
    float tm = PX(xp, ym) - PX(xm, ym);
    float t0 = PX(xp, y) - PX(xm, y);
    float tp = PX(xp, yp) - PX(xm, yp);
    dx[(y * w + x) * noc + c] = (tm + tp) * 0.125f + t0 * 0.25f;
    float sm = (PX(xm, ym) + PX(xp, ym)) * 0.125f + PX(x, ym) * 0.25f;
    float sp = (PX(xm, yp) + PX(xp, yp)) * 0.125f + PX(x, yp) * 0.25f;
    dy[(y * w + x) * noc + c] = sp - sm;
#undef PX
  }
}

/* The interior rows run as one contiguous loop over the row's values (the neighbours are fixed offsets: the
 * compiler vectorises it, as OpenCV's SIMD Sobel is), the border pixels through sobel_px: same expressions. */
static void sobel_level(const float *L, int w, int h, int noc, float *dx, float *dy) {
  const int rs = w * noc;
  for (int y = 0; y < h; ++y) {
    if (y == 0 || y == h - 1 || w < 3) {
      for (int x = 0; x < w; ++x) sobel_px(L, w, h, noc, x, y, dx, dy);
      continue;
    }
    sobel_px(L, w, h, noc, 0, y, dx, dy);
    const float *restrict up = L + (size_t)(y - 1) * rs, *restrict mid = up + rs, *restrict dn = mid + rs;
    float *restrict ox = dx + (size_t)y * rs, *restrict oy = dy + (size_t)y * rs;
    for (int i = noc; i < rs - noc; ++i) {
      const float tm = up[i + noc] - up[i - noc], t0 = mid[i + noc] - mid[i - noc], tp = dn[i + noc] - dn[i - noc];
      ox[i] = (tm + tp) * 0.125f + t0 * 0.25f;
      const float sm = (up[i - noc] + up[i + noc]) * 0.125f + up[i] * 0.25f;
      const float sp = (dn[i - noc] + dn[i + noc]) * 0.125f + dn[i] * 0.25f;
      oy[i] = sp - sm;
    }
    sobel_px(L, w, h, noc, w - 1, y, dx, dy);
  }
}

/* copyMakeBorder: the level's rows copied whole, the border columns / rows replicated or zero. */
static void pad_level(const float *L, int w, int h, int noc, int pad, int replicate, float *out) {
  const int W = w + 2 * pad, H = h + 2 * pad;
  for (int y = 0; y < H; ++y) {
    const int sy = clampi(y - pad, 0, h - 1);
    float *o = out + (size_t)y * W * noc;
    const float *src = L + (size_t)sy * w * noc;
    if (!replicate && (y < pad || y >= pad + h)) {
      memset(o, 0, sizeof(float) * (size_t)W * noc);
      continue;
    }
    memcpy(o + (size_t)pad * noc, src, sizeof(float) * (size_t)w * noc);
    for (int x = 0; x < pad; ++x)
      for (int c = 0; c < noc; ++c) {
        o[x * noc + c] = replicate ? src[c] : 0.0f;
        o[(pad + w + x) * noc + c] = replicate ? src[(w - 1) * noc + c] : 0.0f;
      }
  }
}

int ofo_build_pyramid(const uint8_t *img, int width, int height, int noc, int sc_f, int sc_l, int imgpadding,
                      float **img_pyr, float **dx_pyr, float **dy_pyr) {
  return ofo_build_pyramid_ex(img, width, height, noc, sc_f, sc_l, imgpadding, 0, img_pyr, dx_pyr, dy_pyr);
}

int ofo_build_pyramid_ex(const uint8_t *img, int width, int height, int noc, int sc_f, int sc_l, int imgpadding,
                         int gradmag, float **img_pyr, float **dx_pyr, float **dy_pyr) {
  int w = width, h = height;
  float *cur;
  int s0 = 0;
  if (!gradmag && sc_l >= 1) {
    /* convertTo CV_32F (:327) and the first 2x2 mean fused: the u8 values are exact in fp32, so
     * ((a + b) + (d + e)) * 0.25 of the converted samples is computed straight from the bytes */
    const int nw = w / 2, nh = h / 2, rn = nw * noc;
    cur = (float *)malloc(sizeof(float) * (size_t)nw * nh * noc);
    if (!cur) return OFDIS_ERR_OUT_OF_MEMORY;
    for (int y = 0; y < nh; ++y) {
      const uint8_t *r0 = img + (size_t)(2 * y) * w * noc, *r1 = r0 + (size_t)w * noc;
      float *o = cur + (size_t)y * rn;
      if (noc == 1) {
        /* the sums of u8 samples are exact integers (< 2^11): summed as integers, converted once -- the same value
         * as the float sums, in a form the compiler vectorises like OpenCV's resize does */
        for (int x = 0; x < nw; ++x)
          o[x] = (float)(((int)r0[2 * x] + (int)r0[2 * x + 1]) + ((int)r1[2 * x] + (int)r1[2 * x + 1])) * 0.25f;
      } else {
        for (int x = 0; x < nw; ++x)
          for (int c = 0; c < noc; ++c) {
            const int i = 2 * x * noc + c;
            o[x * noc + c] = (((float)r0[i] + (float)r0[i + noc]) + ((float)r1[i] + (float)r1[i + noc])) * 0.25f;
          }
      }
    }
    w = nw;
    h = nh;
    s0 = 1;
  } else {
    cur = (float *)malloc(sizeof(float) * (size_t)w * h * noc);
    if (!cur) return OFDIS_ERR_OUT_OF_MEMORY;
    for (size_t i = 0; i < (size_t)w * h * noc; ++i) cur[i] = (float)img[i]; /* convertTo CV_32F (:327) */
  }
  if (gradmag) { /* SELECTCHANNEL 2 (:139-148): level 0 = sqrt(dx.mul(dx) + dy.mul(dy)), Sobel 3, 1/8 */
    float *gx = (float *)malloc(sizeof(float) * (size_t)w * h * noc);
    float *gy = (float *)malloc(sizeof(float) * (size_t)w * h * noc);
    if (!gx || !gy) { free(gx); free(gy); free(cur); return OFDIS_ERR_OUT_OF_MEMORY; }
    sobel_level(cur, w, h, noc, gx, gy);
    for (size_t i = 0; i < (size_t)w * h * noc; ++i) cur[i] = sqrtf(gx[i] * gx[i] + gy[i] * gy[i]);
    free(gx); free(gy);
  }
  for (int s = s0; s <= sc_f; ++s) {
    if (s > s0) { /* cv::resize(.5, INTER_LINEAR) -> OpenCV area-fast 2x: mean of the 2x2 block */
      int nw = w / 2, nh = h / 2;
      float *nx = (float *)malloc(sizeof(float) * (size_t)nw * nh * noc);
      if (!nx) { free(cur); return OFDIS_ERR_OUT_OF_MEMORY; }
      for (int y = 0; y < nh; ++y) {
        const float *r0 = cur + (size_t)(2 * y) * w * noc, *r1 = r0 + (size_t)w * noc;
        float *o = nx + (size_t)y * nw * noc;
        if (noc == 1) { /* compile-time channel stride: the loop vectorises */
          for (int x = 0; x < nw; ++x) o[x] = ((r0[2 * x] + r0[2 * x + 1]) + (r1[2 * x] + r1[2 * x + 1])) * 0.25f;
          continue;
        }
        for (int x = 0; x < nw; ++x)
          for (int c = 0; c < noc; ++c) {
            const int i = 2 * x * noc + c;
            o[x * noc + c] = ((r0[i] + r0[i + noc]) + (r1[i] + r1[i + noc])) * 0.25f;
          }
      }
      free(cur);
      cur = nx; w = nw; h = nh;
    }
    if (s >= sc_l) {
      float *dx = (float *)malloc(sizeof(float) * (size_t)w * h * noc);
      float *dy = (float *)malloc(sizeof(float) * (size_t)w * h * noc);
      if (!dx || !dy) { free(dx); free(dy); free(cur); return OFDIS_ERR_OUT_OF_MEMORY; }
      sobel_level(cur, w, h, noc, dx, dy);
      pad_level(cur, w, h, noc, imgpadding, 1, img_pyr[s]); /* BORDER_REPLICATE (:167) */
      pad_level(dx, w, h, noc, imgpadding, 0, dx_pyr[s]);   /* BORDER_CONSTANT 0 (:172-173) */
      pad_level(dy, w, h, noc, imgpadding, 0, dy_pyr[s]);
      free(dx); free(dy);
    }
  }
  free(cur);
  return 0;
}

/* ------------------------------------------------------------------ DIS patch (patch.cpp) */

typedef struct {
  int w, h, pad, tmp_w;    /* camparam (oflow.h:30-43) */
  float tmp_lb, tmp_ubw, tmp_ubh;
  int curr_lv;
  int camlr;
} cam_t;

typedef struct {
  int nop, p, novals, noc, costfct, patnorm, max_iter, min_iter, steps;
  float dp_thresh_sq, dr_thresh, res_thresh, outlierthresh;
} opt_t;

/* Eigen LLT<2x2>.solve (unblocked llt_inplace + unrolled triangular solves). */
static void llt2_solve(float H00, float H01, float H11, float b0, float b1, float *x0, float *x1) {
  float L00 = H00, L10 = H01, L11 = H11;
  if (!(H00 <= 0.0f)) {
    L00 = sqrtf(H00);
    L10 = H01 / L00;
    float t = H11 - L10 * L10;
    if (!(t <= 0.0f)) L11 = sqrtf(t);
  }
  float y0 = b0 / L00;
  float y1 = (b1 - L10 * y0) / L11;
  float z1 = y1 / L11;
  float z0 = (y0 - L10 * z1) / L00;
  *x0 = z0;
  *x1 = z1;
}

static float llt1_solve(float H, float b) {
  float L = H;
  if (!(H <= 0.0f)) L = sqrtf(H);
  float y = b / L;
  return y / L;
}

/* getPatchStaticBil (patch.cpp:345-413) + mean normalisation. */
static void patch_sample_bil(const cam_t *c, const opt_t *o, const float *img, const float mid[2], float *out) {
  int pos0 = (int)ceilf(mid[0] + 0.00001f);
  int pos1 = (int)ceilf(mid[1] + 0.00001f);
  int pos2 = (int)floorf(mid[0]);
  int pos3 = (int)floorf(mid[1]);
  float rx = mid[0] - (float)pos2, ry = mid[1] - (float)pos3;
  float w0 = rx * ry, w1 = (1 - rx) * ry, w2 = rx * (1 - ry), w3 = (1 - rx) * (1 - ry);
  pos0 += c->pad;
  pos1 += c->pad;
  const int p = o->p, noc = o->noc, pn = p * noc;
  /* row pointers as in the reference (img_a / img_b = a - noc / img_c = a - row / img_d = c - noc): a patch
   * row is pn contiguous floats, so the value loop is a plain elementwise expression */
  for (int iy = 0; iy < p; ++iy) {
    const int row = pos1 - p / 2 + iy;
    const float *a = img + ((size_t)row * c->tmp_w + pos0 - p / 2) * noc;
    const float *cc = a - (size_t)c->tmp_w * noc;
    float *dst = out + (size_t)iy * pn;
    for (int i = 0; i < pn; ++i) dst[i] = w0 * a[i] + w1 * a[i - noc] + w2 * cc[i] + w3 * cc[i - noc];
  }
  if (o->patnorm > 0) {
    float mean = ofo_eigen_sum(out, o->novals) / (float)o->novals;
    for (int i = 0; i < o->novals; ++i) out[i] = out[i] - mean;
  }
}

/* LossComputeErrorImage (patch.cpp:221-273): in = normalised sample, tmp = template. */
static void patch_loss(const opt_t *o, float *pdiff, float *pweight, const float *tmp) {
  const float bsq = 5.0f * 5.0f, b2sq = bsq * 2.0f;
  for (int i = 0; i < o->novals; ++i) {
    float d = pdiff[i] - tmp[i];
    if (o->costfct == 0) {
      pdiff[i] = d;
      pweight[i] = fabsf(d);
    } else if (o->costfct == 1) {
      float pw = sqrtf(fabsf(d));
      pweight[i] = pw;
      pdiff[i] = copysignf(pw, d);
    } else {
      float pw = sqrtf((sqrtf(1.0f + (d * d) / bsq) - 1.0f) * b2sq);
      pweight[i] = pw;
      pdiff[i] = copysignf(pw, d);
    }
  }
}

typedef struct {
  float pt_ref[2];
  float p_in[2], p_iter[2], delta_p[2], pt_iter[2], pt_st[2];
  float sq, sq_init, mares, mares_old;
  int cnt, converged;
  float H00, H01, H11;
  float *tmp, *dxx, *dyy, *pdiff, *pweight, *scratch;
} patch_t;

/* OptimizeComputeErrImg (patch.cpp:275-295) */
static void patch_err(const cam_t *c, const opt_t *o, const float *im_b, patch_t *P) {
  patch_sample_bil(c, o, im_b, P->pt_iter, P->pdiff);
  patch_loss(o, P->pdiff, P->pweight, P->tmp);
  if (o->nop == 2)
    P->sq = P->delta_p[0] * P->delta_p[0] + P->delta_p[1] * P->delta_p[1];
  else
    P->sq = P->delta_p[0] * P->delta_p[0];
  if (P->cnt == 1) P->sq_init = P->sq;
  P->mares_old = P->mares;
  /* lpNorm<1> = cwiseAbs().sum() (into the pdiff-sized scratch, no allocation per iteration) */
  for (int i = 0; i < o->novals; ++i) P->scratch[i] = fabsf(P->pweight[i]);
  P->mares = ofo_eigen_sum(P->scratch, o->novals) / (float)o->novals;
  int keep = (P->cnt < o->max_iter) & (P->mares > o->res_thresh) &
             ((P->cnt < o->min_iter) | (P->sq / P->sq_init >= o->dp_thresh_sq)) &
             ((P->cnt < o->min_iter) | (P->mares / P->mares_old <= o->dr_thresh));
  if (!keep) P->converged = 1;
}

static inline void paramtopt(const opt_t *o, patch_t *P) {
  if (o->nop == 2) {
    P->pt_iter[0] = P->pt_ref[0] + P->p_iter[0];
    P->pt_iter[1] = P->pt_ref[1] + P->p_iter[1];
  } else {
    P->pt_iter[0] = P->pt_ref[0] + P->p_iter[0];
  }
}

static inline int out_of_bounds(const cam_t *c, const float pt[2]) {
  return pt[0] < c->tmp_lb || pt[1] < c->tmp_lb || pt[0] > c->tmp_ubw || pt[1] > c->tmp_ubh;
}

/* InitializePatch + SetTargetImage + OptimizeIter(p_init, true)
 * (patch.cpp:55-67,69-86,88-115,117-154,156-210). */
static void patch_run(const cam_t *c, const opt_t *o, const float *im_a, const float *im_a_dx,
                      const float *im_a_dy, const float *im_b, const float p_init[2], patch_t *P) {
  const int p = o->p, noc = o->noc, nv = o->novals;
  /* ResetPatch */
  P->pt_st[0] = P->pt_iter[0] = P->pt_ref[0];
  P->pt_st[1] = P->pt_iter[1] = P->pt_ref[1];
  P->p_in[0] = P->p_in[1] = P->p_iter[0] = P->p_iter[1] = P->delta_p[0] = P->delta_p[1] = 0.0f;
  P->sq = P->sq_init = (float)1e-10;
  P->mares = P->mares_old = (float)1e20;
  P->cnt = 0;
  P->converged = 0;
  /* getPatchStaticNNGrad (patch.cpp:297-343) */
  int px = (int)roundf(P->pt_ref[0]) + c->pad, py = (int)roundf(P->pt_ref[1]) + c->pad;
  int k = 0;
  for (int j = -p / 2; j <= p / 2 - 1; ++j)
    for (int i = -p / 2; i <= p / 2 - 1; ++i) {
      size_t idx = ((size_t)(py + j) * c->tmp_w + (px + i)) * noc;
      for (int ch = 0; ch < noc; ++ch, ++k) {
        P->tmp[k] = im_a[idx + ch];
        P->dxx[k] = im_a_dx[idx + ch];
        P->dyy[k] = im_a_dy[idx + ch];
      }
    }
  if (o->patnorm > 0) {
    float mean = ofo_eigen_sum(P->tmp, nv) / (float)nv;
    for (int i = 0; i < nv; ++i) P->tmp[i] = P->tmp[i] - mean;
  }
  /* ComputeHessian (patch.cpp:69-86): (dxx.array() * dxx.array()).sum() etc. */
  P->H00 = eigen_dot(P->dxx, P->dxx, nv);
  if (o->nop == 2) {
    P->H01 = eigen_dot(P->dxx, P->dyy, nv);
    P->H11 = eigen_dot(P->dyy, P->dyy, nv);
    if (P->H00 * P->H11 - P->H01 * P->H01 == 0.0f) {
      P->H00 = (float)((double)P->H00 + 1e-10);
      P->H11 = (float)((double)P->H11 + 1e-10);
    }
  } else {
    if (P->H00 == 0.0f) P->H00 = (float)((double)P->H00 + 1e-10);
  }
  /* OptimizeStart */
  P->p_in[0] = P->p_iter[0] = p_init[0];
  if (o->nop == 2) P->p_in[1] = P->p_iter[1] = p_init[1];
  paramtopt(o, P);
  P->pt_st[0] = P->pt_iter[0];
  P->pt_st[1] = P->pt_iter[1];
  if (out_of_bounds(c, P->pt_iter)) {
    P->converged = 1;
    memcpy(P->pdiff, P->tmp, sizeof(float) * nv);
    /* pweight is never written upstream (uninitialised heap, patch.cpp:133-139): defined as 0 here */
    memset(P->pweight, 0, sizeof(float) * nv);
  } else {
    P->cnt = 0;
    P->sq = P->sq_init = (float)1e-10;
    P->mares = 1e5f;
    P->mares_old = (float)1e20;
    P->converged = 0;
    patch_err(c, o, im_b, P);
  }
  /* OptimizeIter loop */
  while (!P->converged) {
    P->cnt++;
    float b0 = eigen_dot(P->dxx, P->pdiff, nv);  /* (dxx.array() * pdiff.array()).sum() (patch.cpp:170-171) */
    if (o->nop == 2) {
      float b1 = eigen_dot(P->dyy, P->pdiff, nv);
      llt2_solve(P->H00, P->H01, P->H11, b0, b1, &P->delta_p[0], &P->delta_p[1]);
      P->p_iter[0] = P->p_iter[0] - P->delta_p[0];
      P->p_iter[1] = P->p_iter[1] - P->delta_p[1];
    } else {
      P->delta_p[0] = llt1_solve(P->H00, b0);
      P->p_iter[0] = P->p_iter[0] - P->delta_p[0];
      if (c->camlr == 0)
        P->p_iter[0] = stdminf(P->p_iter[0], 0.0f);
      else
        P->p_iter[0] = stdmaxf(P->p_iter[0], 0.0f);
    }
    paramtopt(o, P);
    float ex = P->pt_st[0] - P->pt_iter[0], ey = P->pt_st[1] - P->pt_iter[1];
    if (sqrtf(ex * ex + ey * ey) > o->outlierthresh || out_of_bounds(c, P->pt_iter)) {
      P->p_iter[0] = P->p_in[0];
      if (o->nop == 2) P->p_iter[1] = P->p_in[1];
      paramtopt(o, P);
      P->converged = 1;
    }
    patch_err(c, o, im_b, P);
  }
}

/* ------------------------------------------------------------------ grid (patchgrid.cpp) */

typedef struct {
  int nopw, noph, nopatches, offw, offh, steps;
} grid_t;

/* PatGridClass ctor geometry (patchgrid.cpp:42-75). */
static void grid_geometry(const cam_t *c, const opt_t *o, grid_t *g) {
  g->steps = o->steps;
  g->nopw = (int)ceilf((float)c->w / (float)o->steps);
  g->noph = (int)ceilf((float)c->h / (float)o->steps);
  g->offw = (c->w - (g->nopw - 1) * o->steps) / 2;
  g->offh = (c->h - (g->noph - 1) * o->steps) / 2;
  g->nopatches = g->nopw * g->noph;
}

/* AggregateFlowDense (patchgrid.cpp:213-397): the grid's own patches, then -- forward-backward merging,
 * usefbcon -- the complementary grid's patches splatted bilinearly at their optimised position with the
 * NEGATED displacement (:277-375), then normalisation.  params[ip*nop + k], pweight[ip*novals + i]. */
static void aggregate(const cam_t *c, const opt_t *o, const grid_t *g, const patch_t *pats, const patch_t *cg,
                      float *flowout) {
  const int w = c->w, h = c->h, nop = o->nop, p = o->p;
  float *we = (float *)calloc((size_t)w * h, sizeof(float));
  memset(flowout, 0, sizeof(float) * (size_t)w * h * nop);
  for (int ip = 0; ip < g->nopatches; ++ip) {
    const patch_t *P = &pats[ip];
    const float *pw = P->pweight;
    for (int y = -p / 2; y <= p / 2 - 1; ++y)
      for (int x = -p / 2; x <= p / 2 - 1; ++x, ++pw) {
        int yt = (int)((float)y + P->pt_ref[1]);
        int xt = (int)((float)x + P->pt_ref[0]);
        if (xt >= 0 && yt >= 0 && xt < w && yt < h) {
          int i = yt * w + xt;
          float absw;
          if (o->noc == 1) {
            absw = 1.0f / stdmaxf(2.0f, *pw);
          } else {
            absw = stdmaxf(2.0f, *pw); ++pw;
            absw = absw + stdmaxf(2.0f, *pw); ++pw;
            absw = absw + stdmaxf(2.0f, *pw);
            absw = 1.0f / absw;
          }
          we[i] = we[i] + absw;
          for (int k = 0; k < nop; ++k) flowout[nop * i + k] = flowout[nop * i + k] + P->p_iter[k] * absw;
        }
      }
  }
  if (cg) {
    for (int ip = 0; ip < g->nopatches; ++ip) { /* both grids have the same geometry (oflow.cpp:155-164) */
      const patch_t *P = &cg[ip];
      const float *pw = P->pweight;
      const float rp0 = P->pt_iter[0], rp1 = P->pt_iter[1]; /* GetPointPos: position after optimisation */
      const int pos0 = (int)ceil((double)rp0 + .00001), pos1 = (int)ceil((double)rp1 + .00001);
      const int pos2 = (int)floorf(rp0), pos3 = (int)floorf(rp1);
      const float r0 = rp0 - (float)pos2, r1 = rp1 - (float)pos3;
      const float wb[4] = {r0 * r1, (1 - r0) * r1, r0 * (1 - r1), (1 - r0) * (1 - r1)};
      for (int y = -p / 2; y <= p / 2 - 1; ++y)
        for (int x = -p / 2; x <= p / 2 - 1; ++x, ++pw) {
          int yt = y + pos1, xt = x + pos0;
          if (xt >= 1 && yt >= 1 && xt < w - 1 && yt < h - 1) {
            float absw;
            if (o->noc == 1) {
              absw = 1.0f / stdmaxf(2.0f, *pw);
            } else {
              absw = stdmaxf(2.0f, *pw); ++pw;
              absw = absw + stdmaxf(2.0f, *pw); ++pw;
              absw = absw + stdmaxf(2.0f, *pw);
              absw = 1.0f / absw;
            }
            float fl[2];
            for (int k = 0; k < nop; ++k) fl[k] = P->p_iter[k] * absw;
            const int idx[4] = {xt + yt * w, (xt - 1) + yt * w, xt + (yt - 1) * w, (xt - 1) + (yt - 1) * w};
            for (int q = 0; q < 4; ++q) we[idx[q]] = we[idx[q]] + wb[q] * absw;
            for (int q = 0; q < 4; ++q)
              for (int k = 0; k < nop; ++k) flowout[nop * idx[q] + k] = flowout[nop * idx[q] + k] - wb[q] * fl[k];
          }
        }
    }
  }
  for (int i = 0; i < w * h; ++i)
    if (we[i] > 0)
      for (int k = 0; k < nop; ++k) flowout[nop * i + k] = flowout[nop * i + k] / we[i];
  free(we);
}

/* ------------------------------------------------------------------ FDF1.0.1 restatements */

/* 5-tap / 3-tap separable convolutions, replicate border (image.cpp:419-624): evaluation order
 * c0*s0 + ((c1*s1 + c2*s2) + (c3*s3 + c4*s4)) and c0*s0 + (c1*s1 + c2*s2). */
static const float K5[5] = {1.0f / 12.0f, -8.0f / 12.0f, -0.0f, 8.0f / 12.0f, -1.0f / 12.0f};
static const float K3[3] = {-0.5f, -0.0f, 0.5f};

static void conv5_h(float *dst, const float *src, int w, int h) {
  for (int y = 0; y < h; ++y) {
    const float *s = src + (size_t)y * w;
    for (int x = 0; x < w; ++x) {
      float s0 = s[clampi(x - 2, 0, w - 1)], s1 = s[clampi(x - 1, 0, w - 1)], s2 = s[x];
      float s3 = s[clampi(x + 1, 0, w - 1)], s4 = s[clampi(x + 2, 0, w - 1)];
      dst[(size_t)y * w + x] = K5[0] * s0 + ((K5[1] * s1 + K5[2] * s2) + (K5[3] * s3 + K5[4] * s4));
    }
  }
}
static void conv5_v(float *dst, const float *src, int w, int h) {
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float s0 = src[(size_t)clampi(y - 2, 0, h - 1) * w + x], s1 = src[(size_t)clampi(y - 1, 0, h - 1) * w + x];
      float s2 = src[(size_t)y * w + x];
      float s3 = src[(size_t)clampi(y + 1, 0, h - 1) * w + x], s4 = src[(size_t)clampi(y + 2, 0, h - 1) * w + x];
      dst[(size_t)y * w + x] = K5[0] * s0 + ((K5[1] * s1 + K5[2] * s2) + (K5[3] * s3 + K5[4] * s4));
    }
}
static void conv3_h(float *dst, const float *src, int w, int h) {
  for (int y = 0; y < h; ++y) {
    const float *s = src + (size_t)y * w;
    for (int x = 0; x < w; ++x) {
      float s0 = s[clampi(x - 1, 0, w - 1)], s1 = s[x], s2 = s[clampi(x + 1, 0, w - 1)];
      dst[(size_t)y * w + x] = K3[0] * s0 + (K3[1] * s1 + K3[2] * s2);
    }
  }
}
static void conv3_v(float *dst, const float *src, int w, int h) {
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float s0 = src[(size_t)clampi(y - 1, 0, h - 1) * w + x], s1 = src[(size_t)y * w + x];
      float s2 = src[(size_t)clampi(y + 1, 0, h - 1) * w + x];
      dst[(size_t)y * w + x] = K3[0] * s0 + (K3[1] * s1 + K3[2] * s2);
    }
}

/* image_warp (opticalflow_aux.c:31-75) */
void ofo_image_warp(float *dst, float *mask, const float *src, const float *wx, const float *wy, int w, int h,
                    int noc) {
  const size_t plane = (size_t)w * h;
  for (int j = 0; j < h; ++j)
    for (int i = 0; i < w; ++i) {
      size_t o = (size_t)j * w + i;
      float xx = (float)i + wx[o], yy = (float)j + wy[o];
      int x = (int)floorf(xx), y = (int)floorf(yy);
      float dx = xx - (float)x, dy = yy - (float)y;
      mask[o] = (xx >= 0 && xx <= (float)(w - 1) && yy >= 0 && yy <= (float)(h - 1)) ? 1.0f : 0.0f;
      int x1 = clampi(x, 0, w - 1), x2 = clampi(x + 1, 0, w - 1);
      int y1 = clampi(y, 0, h - 1), y2 = clampi(y + 1, 0, h - 1);
      for (int c = 0; c < noc; ++c) {
        const float *s = src + c * plane;
        dst[c * plane + o] = s[(size_t)y1 * w + x1] * (1.0f - dx) * (1.0f - dy) + s[(size_t)y1 * w + x2] * dx * (1.0f - dy) +
                             s[(size_t)y2 * w + x1] * (1.0f - dx) * dy + s[(size_t)y2 * w + x2] * dx * dy;
      }
    }
}

/* get_derivatives (opticalflow_aux.c:77-132) */
void ofo_get_derivatives(const float *im1, const float *im2, int w, int h, int noc, float *dx, float *dy,
                         float *dt, float *dxx, float *dxy, float *dyy, float *dxt, float *dyt) {
  const size_t plane = (size_t)w * h;
  float *t = (float *)malloc(sizeof(float) * plane);
  for (int c = 0; c < noc; ++c) {
    size_t o = c * plane;
    for (size_t i = 0; i < plane; ++i) {
      t[i] = 0.5f * (im2[o + i] + im1[o + i]);
      dt[o + i] = im2[o + i] - im1[o + i];
    }
    conv5_h(dx + o, t, w, h);
    conv5_v(dy + o, t, w, h);
    conv5_h(dxx + o, dx + o, w, h);
    conv5_v(dxy + o, dx + o, w, h);
    conv5_v(dyy + o, dy + o, w, h);
    conv5_h(dxt + o, dt + o, w, h);
    conv5_v(dyt + o, dt + o, w, h);
  }
  free(t);
}

/* compute_smoothness (opticalflow_aux.c:138-187) */
void ofo_compute_smoothness(float *dst_h, float *dst_v, const float *uu, const float *vv, int w, int h,
                            float quarter_alpha) {
  const size_t n = (size_t)w * h;
  float *ux = (float *)malloc(sizeof(float) * n), *vx = (float *)malloc(sizeof(float) * n);
  float *uy = (float *)malloc(sizeof(float) * n), *vy = (float *)malloc(sizeof(float) * n);
  float *s = (float *)malloc(sizeof(float) * n);
  conv3_h(ux, uu, w, h);
  conv3_h(vx, vv, w, h);
  conv3_v(uy, uu, w, h);
  conv3_v(vy, vv, w, h);
  const float eps = 0.001f * 0.001f;
  for (size_t i = 0; i < n; ++i)
    s[i] = quarter_alpha / sqrtf(eps + ((ux[i] * ux[i] + uy[i] * uy[i]) + (vx[i] * vx[i] + vy[i] * vy[i])));
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      size_t i = (size_t)y * w + x;
      dst_h[i] = (x < w - 1) ? s[i] + s[i + 1] : 0.0f;
      dst_v[i] = (y < h - 1) ? s[i] + s[i + w] : 0.0f;
    }
  free(ux); free(vx); free(uy); free(vy); free(s);
}

/* sub_laplacian (opticalflow_aux.c:194-223): b = ((((b - th[x-1]) + th[x]) - tv[y-1]) + tv[y]) */
void ofo_sub_laplacian(float *dst, const float *src, const float *wh, const float *wv, int w, int h) {
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w - 1; ++x) {
      size_t i = (size_t)y * w + x;
      float t = wh[i] * (src[i + 1] - src[i]);
      dst[i] = dst[i] + t;
      dst[i + 1] = dst[i + 1] - t;
    }
  for (int y = 0; y < h - 1; ++y)
    for (int x = 0; x < w; ++x) {
      size_t i = (size_t)y * w + x;
      float t = wv[i] * (src[i + w] - src[i]);
      dst[i] = dst[i] + t;
      dst[i + w] = dst[i + w] - t;
    }
}

#define DNORM (0.1f * 0.1f)
#define EPS_COLOR (0.001f * 0.001f)
#define EPS_GRAD (0.001f * 0.001f)

/* compute_data (opticalflow_aux.c:408-594).  The RGB branch keeps the upstream slips exactly:
 * channel 1's colour term uses Iy of channel 2, and the gradient robust sum keeps only channel 3. */
static inline __attribute__((always_inline)) void compute_data_body(
    float *restrict a11, float *restrict a12, float *restrict a22, float *restrict b1, float *restrict b2,
    const float *restrict mask, const float *restrict du, const float *restrict dv, const float *restrict Ix,
    const float *restrict Iy, const float *restrict Iz, const float *restrict Ixx, const float *restrict Ixy,
    const float *restrict Iyy, const float *restrict Ixz, const float *restrict Iyz, int w, int h, const int noc,
    float hdo3, float hgo3, const int color) {
  const size_t n = (size_t)w * h;
  for (size_t i = 0; i < n; ++i) {
    float A11 = 0.0f, A12 = 0.0f, A22 = 0.0f, B1 = 0.0f, B2 = 0.0f;
    const float u = du[i], v = dv[i], m = mask[i];
    float tmp, tmp2, tmp3, tmpx, tmpy, tmpxy, n1, n2;
    if (noc == 1) {
      if (color) {
        tmpx = Ix[i]; tmpy = Iy[i];
        tmp2 = (Iz[i] + tmpx * u) + tmpy * v;
        n1 = (DNORM + tmpx * tmpx) + tmpy * tmpy;
        tmp = (tmp2 * tmp2) / n1;
        tmp = (m * hdo3) / sqrtf(EPS_COLOR + 3.0f * tmp);
        tmp3 = tmp / n1;
        tmp2 = tmp3 * tmpx;
        tmp3 = tmp3 * tmpy;
        A11 = A11 + tmp2 * tmpx;
        A12 = A12 + tmp2 * tmpy;
        A22 = A22 + tmp3 * tmpy;
        B1 = B1 - tmp2 * Iz[i];
        B2 = B2 - tmp3 * Iz[i];
      }
      tmpx = Ixx[i]; tmpy = Iyy[i]; tmpxy = Ixy[i];
      tmp2 = (Ixz[i] + tmpx * u) + tmpxy * v;
      tmp3 = (Iyz[i] + tmpxy * u) + tmpy * v;
      tmpxy = tmpxy * tmpxy;
      n1 = (tmpxy + DNORM) + tmpx * tmpx;
      n2 = (tmpxy + DNORM) + tmpy * tmpy;
      tmp = (tmp2 * tmp2) / n1 + (tmp3 * tmp3) / n2;
      tmp = (m * hgo3) / sqrtf(EPS_GRAD + 3.0f * tmp);
      tmp2 = tmp / n2; tmp3 = tmp / n1;
      tmpxy = Ixy[i];
      A12 = A12 + ((tmp3 * tmpx) + tmp2 * tmpy) * tmpxy;
      B1 = (B1 - (tmp3 * tmpx) * Ixz[i]) - (tmp2 * tmpxy) * Iyz[i];
      B2 = (B2 - (tmp2 * tmpy) * Iyz[i]) - (tmp3 * tmpxy) * Ixz[i];
      tmpxy = tmpxy * tmpxy;
      A11 = (A11 + tmp3 * (tmpx * tmpx)) + tmp2 * tmpxy;
      A22 = (A22 + tmp2 * (tmpy * tmpy)) + tmp3 * tmpxy;
      A11 = A11 * 3.0f; A12 = A12 * 3.0f; A22 = A22 * 3.0f; B1 = B1 * 3.0f; B2 = B2 * 3.0f;
    } else {
      const size_t o2 = n, o3 = 2 * n;
      float n3, n4, n5, n6;
      if (color) {
        tmpx = Ix[i]; tmpy = Iy[i];
        tmp2 = (Iz[i] + tmpx * u) + tmpy * v;
        n1 = (DNORM + tmpx * tmpx) + tmpy * tmpy;
        tmp = (tmp2 * tmp2) / n1;
        tmpx = Ix[o2 + i]; tmpy = Iy[o2 + i];
        tmp2 = (Iz[o2 + i] + tmpx * u) + tmpy * v;
        n2 = (DNORM + tmpx * tmpx) + tmpy * tmpy;
        tmp = tmp + (tmp2 * tmp2) / n2;
        tmpx = Ix[o3 + i]; tmpy = Iy[o3 + i];
        tmp2 = (Iz[o3 + i] + tmpx * u) + tmpy * v;
        n3 = (DNORM + tmpx * tmpx) + tmpy * tmpy;
        tmp = tmp + (tmp2 * tmp2) / n3;
        tmp = (m * hdo3) / sqrtf(EPS_COLOR + tmp);
        tmp3 = tmp / n3;
        tmp2 = tmp3 * tmpx;
        tmp3 = tmp3 * tmpy;
        A11 = A11 + tmp2 * tmpx; A12 = A12 + tmp2 * tmpy; A22 = A22 + tmp3 * tmpy;
        B1 = B1 - tmp2 * Iz[o3 + i]; B2 = B2 - tmp3 * Iz[o3 + i];
        tmpx = Ix[o2 + i]; tmpy = Iy[o2 + i];
        tmp3 = tmp / n2;
        tmp2 = tmp3 * tmpx;
        tmp3 = tmp3 * tmpy;
        A11 = A11 + tmp2 * tmpx; A12 = A12 + tmp2 * tmpy; A22 = A22 + tmp3 * tmpy;
        B1 = B1 - tmp2 * Iz[o2 + i]; B2 = B2 - tmp3 * Iz[o2 + i];
        tmpx = Ix[i]; tmpy = Iy[o2 + i]; /* upstream slip: channel 2's Iy */
        tmp3 = tmp / n1;
        tmp2 = tmp3 * tmpx;
        tmp3 = tmp3 * tmpy;
        A11 = A11 + tmp2 * tmpx; A12 = A12 + tmp2 * tmpy; A22 = A22 + tmp3 * tmpy;
        B1 = B1 - tmp2 * Iz[i]; B2 = B2 - tmp3 * Iz[i];
      }
      /* gradient: the robust sum is overwritten per channel (only channel 3 survives) */
      tmpx = Ixx[i]; tmpy = Iyy[i]; tmpxy = Ixy[i];
      tmp2 = (Ixz[i] + tmpx * u) + tmpxy * v;
      tmp3 = (Iyz[i] + tmpxy * u) + tmpy * v;
      tmpxy = tmpxy * tmpxy;
      n1 = (tmpxy + DNORM) + tmpx * tmpx;
      n2 = (tmpxy + DNORM) + tmpy * tmpy;
      tmp = (tmp2 * tmp2) / n1 + (tmp3 * tmp3) / n2;
      tmpx = Ixx[o2 + i]; tmpy = Iyy[o2 + i]; tmpxy = Ixy[o2 + i];
      tmp2 = (Ixz[o2 + i] + tmpx * u) + tmpxy * v;
      tmp3 = (Iyz[o2 + i] + tmpxy * u) + tmpy * v;
      tmpxy = tmpxy * tmpxy;
      n3 = (tmpxy + DNORM) + tmpx * tmpx;
      n4 = (tmpxy + DNORM) + tmpy * tmpy;
      tmp = (tmp2 * tmp2) / n3 + (tmp3 * tmp3) / n4;
      tmpx = Ixx[o3 + i]; tmpy = Iyy[o3 + i]; tmpxy = Ixy[o3 + i];
      tmp2 = (Ixz[o3 + i] + tmpx * u) + tmpxy * v;
      tmp3 = (Iyz[o3 + i] + tmpxy * u) + tmpy * v;
      tmpxy = tmpxy * tmpxy;
      n5 = (tmpxy + DNORM) + tmpx * tmpx;
      n6 = (tmpxy + DNORM) + tmpy * tmpy;
      tmp = (tmp2 * tmp2) / n5 + (tmp3 * tmp3) / n6;
      tmp = (m * hgo3) / sqrtf(EPS_GRAD + tmp);
      /* channel 3 */
      tmp2 = tmp / n6; tmp3 = tmp / n5;
      A11 = (A11 + tmp3 * (tmpx * tmpx)) + tmp2 * tmpxy;
      A22 = (A22 + tmp2 * (tmpy * tmpy)) + tmp3 * tmpxy;
      tmpxy = Ixy[o3 + i];
      A12 = A12 + ((tmp3 * tmpx) + tmp2 * tmpy) * tmpxy;
      B1 = (B1 - (tmp3 * tmpx) * Ixz[o3 + i]) - (tmp2 * tmpxy) * Iyz[o3 + i];
      B2 = (B2 - (tmp2 * tmpy) * Iyz[o3 + i]) - (tmp3 * tmpxy) * Ixz[o3 + i];
      /* channel 2 */
      tmp2 = tmp / n4; tmp3 = tmp / n3;
      tmpx = Ixx[o2 + i]; tmpy = Iyy[o2 + i]; tmpxy = Ixy[o2 + i];
      A12 = A12 + ((tmp3 * tmpx) + tmp2 * tmpy) * tmpxy;
      B1 = (B1 - (tmp3 * tmpx) * Ixz[o2 + i]) - (tmp2 * tmpxy) * Iyz[o2 + i];
      B2 = (B2 - (tmp2 * tmpy) * Iyz[o2 + i]) - (tmp3 * tmpxy) * Ixz[o2 + i];
      tmpxy = tmpxy * tmpxy;
      A11 = (A11 + tmp3 * (tmpx * tmpx)) + tmp2 * tmpxy;
      A22 = (A22 + tmp2 * (tmpy * tmpy)) + tmp3 * tmpxy;
      /* channel 1 */
      tmpx = Ixx[i]; tmpy = Iyy[i];
      tmp2 = tmp / n2; tmp3 = tmp / n1;
      tmpxy = Ixy[i];
      A12 = A12 + ((tmp3 * tmpx) + tmp2 * tmpy) * tmpxy;
      B1 = (B1 - (tmp3 * tmpx) * Ixz[i]) - (tmp2 * tmpxy) * Iyz[i];
      B2 = (B2 - (tmp2 * tmpy) * Iyz[i]) - (tmp3 * tmpxy) * Ixz[i];
      tmpxy = tmpxy * tmpxy;
      A11 = (A11 + tmp3 * (tmpx * tmpx)) + tmp2 * tmpxy;
      A22 = (A22 + tmp2 * (tmpy * tmpy)) + tmp3 * tmpxy;
    }
    a11[i] = A11; a12[i] = A12; a22[i] = A22; b1[i] = B1; b2[i] = B2;
  }
}

/* The per-pixel expression trees of compute_data, one loop per (noc, colour term) so the compiler can
 * vectorise it like the reference's SSE code (per-pixel IEEE operations, same order: bit-identical). */
void ofo_compute_data(float *restrict a11, float *restrict a12, float *restrict a22, float *restrict b1,
                      float *restrict b2, const float *restrict mask, const float *restrict du,
                      const float *restrict dv, const float *restrict Ix, const float *restrict Iy,
                      const float *restrict Iz, const float *restrict Ixx, const float *restrict Ixy,
                      const float *restrict Iyy, const float *restrict Ixz, const float *restrict Iyz,
                      int w, int h, int noc, float hdo3, float hgo3) {
#define OFO_CD(NOC, COL) compute_data_body(a11, a12, a22, b1, b2, mask, du, dv, Ix, Iy, Iz, Ixx, Ixy, Iyy, Ixz, \
                                           Iyz, w, h, NOC, hdo3, hgo3, COL)
  if (noc == 1) {
    if (hdo3 != 0.0f) OFO_CD(1, 1); else OFO_CD(1, 0);
  } else {
    if (hdo3 != 0.0f) OFO_CD(3, 1); else OFO_CD(3, 0);
  }
#undef OFO_CD
}

/* compute_data_DE (opticalflow_aux.c:601-747) */
void ofo_compute_data_de(float *a11, float *b1, const float *mask, const float *du, const float *Ix,
                         const float *Iy, const float *Iz, const float *Ixx, const float *Ixy, const float *Iyy,
                         const float *Ixz, const float *Iyz, int w, int h, int noc, float hdo3, float hgo3) {
  const size_t n = (size_t)w * h;
  for (size_t i = 0; i < n; ++i) {
    float A11 = 0.0f, B1 = 0.0f;
    const float u = du[i], m = mask[i];
    float tmp, tmp2, tmp3, tmpx, tmpy, tmpxy, n1, n2;
    if (noc == 1) {
      if (hdo3 != 0.0f) {
        tmpx = Ix[i]; tmpy = Iy[i];
        tmp2 = Iz[i] + tmpx * u;
        n1 = (DNORM + tmpy * tmpy) + tmpx * tmpx;
        tmp = (tmp2 * tmp2) / n1;
        tmp = (m * hdo3) / sqrtf(EPS_COLOR + 3.0f * tmp);
        tmp2 = (tmp / n1) * tmpx;
        A11 = A11 + tmp2 * tmpx;
        B1 = B1 - tmp2 * Iz[i];
      }
      tmpx = Ixx[i]; tmpy = Iyy[i]; tmpxy = Ixy[i];
      tmp2 = Iyz[i] + tmpxy * u;
      tmpxy = DNORM + tmpxy * tmpxy;
      n1 = tmpxy + tmpx * tmpx;
      n2 = tmpxy + tmpy * tmpy;
      tmp = (tmp2 * tmp2) / n2;
      tmp2 = Ixz[i] + tmpx * u;
      tmp = tmp + (tmp2 * tmp2) / n1;
      tmp = (m * hgo3) / sqrtf(EPS_GRAD + 3.0f * tmp);
      tmpxy = Ixy[i];
      tmp2 = (tmp / n2) * tmpxy; tmp3 = (tmp / n1) * tmpx;
      A11 = (A11 + tmp3 * tmpx) + tmp2 * tmpxy;
      B1 = (B1 - tmp3 * Ixz[i]) - tmp2 * Iyz[i];
      A11 = A11 * 3.0f; B1 = B1 * 3.0f;
    } else {
      const size_t o2 = n, o3 = 2 * n;
      float n3, n4, n5, n6;
      if (hdo3 != 0.0f) {
        tmpx = Ix[i]; tmpy = Iy[i];
        tmp2 = Iz[i] + tmpx * u;
        n1 = (DNORM + tmpy * tmpy) + tmpx * tmpx;
        tmp = (tmp2 * tmp2) / n1;
        tmpx = Ix[o2 + i]; tmpy = Iy[o2 + i];
        tmp2 = Iz[o2 + i] + tmpx * u;
        n2 = (DNORM + tmpy * tmpy) + tmpx * tmpx;
        tmp = tmp + (tmp2 * tmp2) / n2;
        tmpx = Ix[o3 + i]; tmpy = Iy[o3 + i];
        tmp2 = Iz[o3 + i] + tmpx * u;
        n3 = (DNORM + tmpy * tmpy) + tmpx * tmpx;
        tmp = tmp + (tmp2 * tmp2) / n3;
        tmp = (m * hdo3) / sqrtf(EPS_COLOR + tmp);
        tmp2 = (tmp / n3) * tmpx;
        A11 = A11 + tmp2 * tmpx; B1 = B1 - tmp2 * Iz[o3 + i];
        tmpx = Ix[o2 + i];
        tmp2 = (tmp / n2) * tmpx;
        A11 = A11 + tmp2 * tmpx; B1 = B1 - tmp2 * Iz[o2 + i];
        tmpx = Ix[i];
        tmp2 = (tmp / n1) * tmpx;
        A11 = A11 + tmp2 * tmpx; B1 = B1 - tmp2 * Iz[i];
      }
      tmpx = Ixx[i]; tmpy = Iyy[i]; tmpxy = Ixy[i];
      tmp2 = Iyz[i] + tmpxy * u;
      tmpxy = DNORM + tmpxy * tmpxy;
      n1 = tmpxy + tmpx * tmpx;
      n2 = tmpxy + tmpy * tmpy;
      tmp = (tmp2 * tmp2) / n2;
      tmp2 = Ixz[i] + tmpx * u;
      tmp = tmp + (tmp2 * tmp2) / n1;
      tmpx = Ixx[o2 + i]; tmpy = Iyy[o2 + i]; tmpxy = Ixy[o2 + i];
      tmp2 = Iyz[o2 + i] + tmpxy * u;
      tmpxy = DNORM + tmpxy * tmpxy;
      n3 = tmpxy + tmpx * tmpx;
      n4 = tmpxy + tmpy * tmpy;
      tmp = tmp + (tmp2 * tmp2) / n4;
      tmp2 = Ixz[o2 + i] + tmpx * u;
      tmp = tmp + (tmp2 * tmp2) / n3;
      tmpx = Ixx[o3 + i]; tmpy = Iyy[o3 + i]; tmpxy = Ixy[o3 + i];
      tmp2 = Iyz[o3 + i] + tmpxy * u;
      tmpxy = DNORM + tmpxy * tmpxy;
      n5 = tmpxy + tmpx * tmpx;
      n6 = tmpxy + tmpy * tmpy;
      tmp = tmp + (tmp2 * tmp2) / n6;
      tmp2 = Ixz[o3 + i] + tmpx * u;
      tmp = tmp + (tmp2 * tmp2) / n5;
      tmp = (m * hgo3) / sqrtf(EPS_GRAD + tmp);
      tmpxy = Ixy[o3 + i];
      tmp2 = (tmp / n6) * tmpxy; tmp3 = (tmp / n5) * tmpx;
      A11 = (A11 + tmp3 * tmpx) + tmp2 * tmpxy;
      B1 = (B1 - tmp3 * Ixz[o3 + i]) - tmp2 * Iyz[o3 + i];
      tmpx = Ixx[o2 + i]; tmpxy = Ixy[o2 + i];
      tmp2 = (tmp / n4) * tmpxy; tmp3 = (tmp / n3) * tmpx;
      A11 = (A11 + tmp3 * tmpx) + tmp2 * tmpxy;
      B1 = (B1 - tmp3 * Ixz[o2 + i]) - tmp2 * Iyz[o2 + i];
      tmpx = Ixx[i]; tmpxy = Ixy[i];
      tmp2 = (tmp / n2) * tmpxy; tmp3 = (tmp / n1) * tmpx;
      A11 = (A11 + tmp3 * tmpx) + tmp2 * tmpxy;
      B1 = (B1 - tmp3 * Ixz[i]) - tmp2 * Iyz[i];
    }
    a11[i] = A11; b1[i] = B1;
  }
}

/* sor_coupled_slow_but_readable (solver.c:34-78): point SOR, used upstream for tiny images and by the
 * OpenMP build for every image (refine_variational.cpp:202-203; single-thread order). */
void ofo_sor_point_of(float *du, float *dv, const float *a11, const float *a12, const float *a22,
                         const float *b1, const float *b2, const float *hh, const float *vv, int w, int hgt,
                         int iterations, float omega) {
  for (int it = 0; it < iterations; ++it)
    for (int j = 0; j < hgt; ++j)
      for (int i = 0; i < w; ++i) {
        float su = 0.0f, sv = 0.0f, sd = 0.0f;
        size_t o = (size_t)j * w + i;
        if (j > 0) { su -= vv[o - w] * du[o - w]; sv -= vv[o - w] * dv[o - w]; sd += vv[o - w]; }
        if (i > 0) { su -= hh[o - 1] * du[o - 1]; sv -= hh[o - 1] * dv[o - 1]; sd += hh[o - 1]; }
        if (j < hgt - 1) { su -= vv[o] * du[o + w]; sv -= vv[o] * dv[o + w]; sd += vv[o]; }
        if (i < w - 1) { su -= hh[o] * du[o + 1]; sv -= hh[o] * dv[o + 1]; sd += hh[o]; }
        float A11 = a11[o] + sd, A12 = a12[o], A22 = a22[o] + sd;
        float B1 = b1[o] - su, B2 = b2[o] - sv;
        du[o] = (1.0f - omega) * du[o] + omega / A11 * (B1 - A12 * dv[o]);
        dv[o] = (1.0f - omega) * dv[o] + omega / A22 * (B2 - A12 * du[o]);
      }
}

/* sor_coupled (solver.c:83-433): lexicographic block Gauss-Seidel SOR with in-place 2x2 inverse. */
void ofo_sor_coupled(float *du, float *dv, float *a11, float *a12, float *a22, const float *b1, const float *b2,
                     const float *hh, const float *vv, int w, int hgt, int iterations, float omega) {
  if (w < 2 || hgt < 2 || iterations < 1) {
    ofo_sor_point_of(du, dv, a11, a12, a22, b1, b2, hh, vv, w, hgt, iterations, omega);
    return;
  }
  for (int it = 0; it < iterations; ++it)
    for (int y = 0; y < hgt; ++y)
      for (int x = 0; x < w; ++x) {
        size_t o = (size_t)y * w + x;
        const float hl = x > 0 ? hh[o - 1] : 0.0f, hr = hh[o];
        const float ur = x < w - 1 ? du[o + 1] : 0.0f, vr = x < w - 1 ? dv[o + 1] : 0.0f;
        float s1, s2, dpsis;
        if (y == 0) {
          dpsis = hl + (hr + vv[o]);
          s1 = (b1[o] + hr * ur) + vv[o] * du[o + w];
          s2 = (b2[o] + hr * vr) + vv[o] * dv[o + w];
        } else if (y < hgt - 1) {
          const float vt = vv[o - w];
          dpsis = (hl + hr) + (vt + vv[o]);
          s1 = ((hr * ur) + vt * du[o - w]) + (b1[o] + vv[o] * du[o + w]);
          s2 = ((hr * vr) + vt * dv[o - w]) + (b2[o] + vv[o] * dv[o + w]);
        } else {
          const float vt = vv[o - w];
          dpsis = hl + (hr + vt);
          s1 = (b1[o] + hr * ur) + vt * du[o - w];
          s2 = (b2[o] + hr * vr) + vt * dv[o - w];
        }
        if (it == 0) {
          float A11 = a22[o] + dpsis, A22 = a11[o] + dpsis, m12 = a12[o];
          float det = A11 * A22 - m12 * m12;
          a11[o] = A11 / det;
          a22[o] = A22 / det;
          a12[o] = m12 / (0.0f - det);
        }
        float B1, B2;
        if (x == 0) {
          B1 = s1;
          B2 = s2;
        } else {
          B1 = hl * du[o - 1] + s1;
          B2 = hl * dv[o - 1] + s2;
        }
        const float u0 = du[o], v0 = dv[o];
        du[o] = u0 + omega * (a11[o] * B1 + a12[o] * B2 - u0);
        dv[o] = v0 + omega * (a12[o] * B1 + a22[o] * B2 - v0);
      }
}

/* sor_coupled_slow_but_readable_DE (solver.c:439-471) */
void ofo_sor_point_de(float *du, const float *a11, const float *b1, const float *hh, const float *vv, int w,
                      int hgt, int iterations, float omega) {
  for (int it = 0; it < iterations; ++it)
    for (int j = 0; j < hgt; ++j)
      for (int i = 0; i < w; ++i) {
        float su = 0.0f, sd = 0.0f;
        size_t o = (size_t)j * w + i;
        if (j > 0) { su -= vv[o - w] * du[o - w]; sd += vv[o - w]; }
        if (i > 0) { su -= hh[o - 1] * du[o - 1]; sd += hh[o - 1]; }
        if (j < hgt - 1) { su -= vv[o] * du[o + w]; sd += vv[o]; }
        if (i < w - 1) { su -= hh[o] * du[o + 1]; sd += hh[o]; }
        float A11 = a11[o] + sd, B1 = b1[o] - su;
        du[o] = (1.0f - omega) * du[o] + omega * (B1 / A11);
      }
}

/* Red-black order of the same per-pixel SOR updates -- NOT a reference function: the checker of the GPU's opt-in
 * sor_mode = 1 (k_tv_level_rb / k_tv_sor_rb), whose iteration differs from solver.c's lexicographic
 * one.  Same operands and the same rounding order per update as sor_coupled (solver.c:83-433: the in-place 2x2 inverse
 * of :122-128 with the border forms :131-190, the right-hand-side trees :241-300) and the DE point form (solver.c:
 * 439-471); only the order changes: every pixel with x + y even, then every odd one, `iterations` times.  Within a
 * colour the updates are independent (every neighbour has the other colour), so the loop order inside it is free. */
static int g_sor_order = 0; /* 0 lexicographic (the reference), 1 red-black */
void ofo_set_sor_order(int order) { g_sor_order = order; }
int ofo_get_sor_order(void) { return g_sor_order; }

void ofo_sor_rb_of(float *du, float *dv, float *a11, float *a12, float *a22, const float *b1, const float *b2,
                   const float *hh, const float *vv, int w, int hgt, int iterations, float omega) {
  if (w < 2 || hgt < 2 || iterations < 1) {
    ofo_sor_point_of(du, dv, a11, a12, a22, b1, b2, hh, vv, w, hgt, iterations, omega);
    return;
  }
  for (int y = 0; y < hgt; ++y) /* the inverse of sor_coupled's first sweep, for every pixel up front */
    for (int x = 0; x < w; ++x) {
      size_t o = (size_t)y * w + x;
      const float hl = x > 0 ? hh[o - 1] : 0.0f, hr = hh[o];
      float dpsis;
      if (y == 0) dpsis = hl + (hr + vv[o]);
      else if (y < hgt - 1) dpsis = (hl + hr) + (vv[o - w] + vv[o]);
      else dpsis = hl + (hr + vv[o - w]);
      float A11 = a22[o] + dpsis, A22 = a11[o] + dpsis, m12 = a12[o];
      float det = A11 * A22 - m12 * m12;
      a11[o] = A11 / det;
      a22[o] = A22 / det;
      a12[o] = m12 / (0.0f - det);
    }
  for (int it = 0; it < iterations; ++it)
    for (int colour = 0; colour < 2; ++colour)
      for (int y = 0; y < hgt; ++y)
        for (int x = (y + colour) & 1; x < w; x += 2) {
          size_t o = (size_t)y * w + x;
          const float hl = x > 0 ? hh[o - 1] : 0.0f, hr = hh[o];
          const float ur = x < w - 1 ? du[o + 1] : 0.0f, vr = x < w - 1 ? dv[o + 1] : 0.0f;
          float s1, s2;
          if (y == 0) {
            s1 = (b1[o] + hr * ur) + vv[o] * du[o + w];
            s2 = (b2[o] + hr * vr) + vv[o] * dv[o + w];
          } else if (y < hgt - 1) {
            const float vt = vv[o - w];
            s1 = ((hr * ur) + vt * du[o - w]) + (b1[o] + vv[o] * du[o + w]);
            s2 = ((hr * vr) + vt * dv[o - w]) + (b2[o] + vv[o] * dv[o + w]);
          } else {
            const float vt = vv[o - w];
            s1 = (b1[o] + hr * ur) + vt * du[o - w];
            s2 = (b2[o] + hr * vr) + vt * dv[o - w];
          }
          const float B1 = x == 0 ? s1 : hl * du[o - 1] + s1;
          const float B2 = x == 0 ? s2 : hl * dv[o - 1] + s2;
          const float u0 = du[o], v0 = dv[o];
          du[o] = u0 + omega * (a11[o] * B1 + a12[o] * B2 - u0);
          dv[o] = v0 + omega * (a12[o] * B1 + a22[o] * B2 - v0);
        }
}

void ofo_sor_rb_de(float *du, const float *a11, const float *b1, const float *hh, const float *vv, int w, int hgt,
                   int iterations, float omega) {
  for (int it = 0; it < iterations; ++it)
    for (int colour = 0; colour < 2; ++colour)
      for (int j = 0; j < hgt; ++j)
        for (int i = (j + colour) & 1; i < w; i += 2) {
          float su = 0.0f, sd = 0.0f;
          size_t o = (size_t)j * w + i;
          if (j > 0) { su -= vv[o - w] * du[o - w]; sd += vv[o - w]; }
          if (i > 0) { su -= hh[o - 1] * du[o - 1]; sd += hh[o - 1]; }
          if (j < hgt - 1) { su -= vv[o] * du[o + w]; sd += vv[o]; }
          if (i < w - 1) { su -= hh[o] * du[o + 1]; sd += hh[o]; }
          float A11 = a11[o] + sd, B1 = b1[o] - su;
          du[o] = (1.0f - omega) * du[o] + omega * (B1 / A11);
        }
}

/* ------------------------------------------------------------------ VarRefClass (refine_variational.cpp) */

/* VarRefClass ctor + RefLevelOF / RefLevelDE (refine_variational.cpp:25-116, 152-342).
 * flow: w*h*nop interleaved, refined in place.  im_ao/im_bo: padded interleaved level images. */
static int var_refine(const cam_t *c, const opt_t *o, const ofdis_params *p, const float *im_ao,
                      const float *im_bo, float *flow) {
  const int w = c->w, h = c->h, noc = o->noc, nop = o->nop;
  const size_t n = (size_t)w * h;
  const int n_inner = p->tv_innerit * (c->curr_lv + 1);
  const float quarter_alpha = 0.25f * p->tv_alpha;
  const float hgo3 = p->tv_gamma * 0.5f / 3.0f, hdo3 = p->tv_delta * 0.5f / 3.0f;
  const float omega = p->tv_sor;
  float *buf = (float *)calloc(n * (15 + 11 * (size_t)noc), sizeof(float));
  if (!buf) return OFDIS_ERR_OUT_OF_MEMORY;
  float *wx = buf, *wy = wx + n, *du = wy + n, *dv = du + n, *mask = dv + n, *sh = mask + n, *sv = sh + n;
  float *uu = sv + n, *vv = uu + n, *a11 = vv + n, *a12 = a11 + n, *a22 = a12 + n, *b1 = a22 + n, *b2 = b1 + n;
  float *im1 = b2 + n + n, *im2 = im1 + n * noc, *wim2 = im2 + n * noc, *Ix = wim2 + n * noc, *Iy = Ix + n * noc;
  float *Iz = Iy + n * noc, *Ixx = Iz + n * noc, *Ixy = Ixx + n * noc, *Iyy = Ixy + n * noc, *Ixz = Iyy + n * noc;
  float *Iyz = Ixz + n * noc; /* 11*noc planes end here; wy stays zero for DE (wy_dummy) */
  for (size_t i = 0; i < n; ++i) {
    wx[i] = flow[i * nop];
    if (nop == 2) wy[i] = flow[i * nop + 1];
  }
  /* copyimage (refine_variational.cpp:119-149): padded interleaved -> planar unpadded */
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x)
      for (int ch = 0; ch < noc; ++ch) {
        size_t src = ((size_t)(y + c->pad) * c->tmp_w + (x + c->pad)) * noc + ch;
        im1[ch * n + (size_t)y * w + x] = im_ao[src];
        im2[ch * n + (size_t)y * w + x] = im_bo[src];
      }
  ofo_image_warp(wim2, mask, im2, wx, wy, w, h, noc);
  ofo_get_derivatives(im1, wim2, w, h, noc, Ix, Iy, Iz, Ixx, Ixy, Iyy, Ixz, Iyz);
  memset(du, 0, sizeof(float) * n);
  memset(dv, 0, sizeof(float) * n);
  memcpy(uu, wx, sizeof(float) * n);
  memcpy(vv, wy, sizeof(float) * n);
  for (int it = 0; it < n_inner; ++it) {
    ofo_compute_smoothness(sh, sv, uu, vv, w, h, quarter_alpha);
    if (nop == 2) {
      ofo_compute_data(a11, a12, a22, b1, b2, mask, du, dv, Ix, Iy, Iz, Ixx, Ixy, Iyy, Ixz, Iyz, w, h, noc, hdo3,
                       hgo3);
      ofo_sub_laplacian(b1, wx, sh, sv, w, h);
      ofo_sub_laplacian(b2, wy, sh, sv, w, h);
      if (p->omp_build) /* refine_variational.cpp:202-203 (#ifdef _OPENMP) */
        ofo_sor_point_of(du, dv, a11, a12, a22, b1, b2, sh, sv, w, h, p->tv_solverit, omega);
      else if (g_sor_order == 1)
        ofo_sor_rb_of(du, dv, a11, a12, a22, b1, b2, sh, sv, w, h, p->tv_solverit, omega);
      else
        ofo_sor_coupled(du, dv, a11, a12, a22, b1, b2, sh, sv, w, h, p->tv_solverit, omega);
      for (size_t i = 0; i < n; ++i) {
        uu[i] = wx[i] + du[i];
        vv[i] = wy[i] + dv[i];
      }
    } else {
      ofo_compute_data_de(a11, b1, mask, du, Ix, Iy, Iz, Ixx, Ixy, Iyy, Ixz, Iyz, w, h, noc, hdo3, hgo3);
      ofo_sub_laplacian(b1, wx, sh, sv, w, h);
      if (g_sor_order == 1)
        ofo_sor_rb_de(du, a11, b1, sh, sv, w, h, p->tv_solverit, omega);
      else
        ofo_sor_point_de(du, a11, b1, sh, sv, w, h, p->tv_solverit, omega);
      for (size_t i = 0; i < n; ++i)
        uu[i] = (c->camlr == 0) ? ssemin(wx[i] + du[i], 0.0f) : ssemax(wx[i] + du[i], 0.0f);
    }
  }
  for (size_t i = 0; i < n; ++i) {
    flow[i * nop] = uu[i];
    if (nop == 2) flow[i * nop + 1] = vv[i];
  }
  free(buf);
  return 0;
}

/* ------------------------------------------------------------------ OFClass (oflow.cpp:31-338) */

static void fill_opt(const ofdis_params *p, opt_t *o) {
  o->nop = p->mode == OFDIS_MODE_OF ? 2 : 1;
  o->p = p->p_samp_s;
  o->noc = p->noc;
  o->novals = p->noc * p->p_samp_s * p->p_samp_s;
  o->costfct = p->costfct;
  o->patnorm = p->patnorm;
  o->max_iter = p->max_iter;
  o->min_iter = p->min_iter;
  o->dp_thresh_sq = p->dp_thresh * p->dp_thresh;
  o->dr_thresh = p->dr_thresh;
  o->res_thresh = p->res_thresh;
  o->outlierthresh = (float)p->p_samp_s / 2;
  int st = (int)floorf((float)p->p_samp_s * (1 - p->patove));
  o->steps = st > 1 ? st : 1;
}

static void fill_cam(const ofdis_params *p, int width, int height, int imgpadding, int sl, cam_t *c) {
  float sc_fct = (float)pow(2.0, -sl);
  c->w = (int)((float)width * sc_fct);
  c->h = (int)((float)height * sc_fct);
  c->pad = imgpadding;
  c->tmp_lb = -(float)p->p_samp_s / 2;
  c->tmp_ubw = (float)(c->w + p->p_samp_s / 2 - 2);
  c->tmp_ubh = (float)(c->h + p->p_samp_s / 2 - 2);
  c->tmp_w = c->w + 2 * imgpadding;
  c->curr_lv = sl;
  c->camlr = 0;
}

/* One patch grid of a scale (PatGridClass: InitializeGrid, SetTargetImage, InitializeFromCoarserOF,
 * Optimize; patchgrid.cpp:31-211).  prev: coarser flow of this grid's direction, or NULL. */
static patch_t *run_grid(const cam_t *c, const opt_t *o, const grid_t *g, const float *im_a, const float *im_a_dx,
                         const float *im_a_dy, const float *im_b, const float *prev, float **store_out) {
  patch_t *pats = (patch_t *)calloc(g->nopatches, sizeof(patch_t));
  /* five arrays per patch + one scratch array shared by the grid's (sequential) patches */
  float *store = (float *)malloc(sizeof(float) * ((size_t)g->nopatches * o->novals * 5 + o->novals));
  float *scratch = store + (size_t)g->nopatches * o->novals * 5;
  for (int x = 0, i = 0; x < g->nopw; ++x)
    for (int y = 0; y < g->noph; ++y, ++i) {
      pats[i].pt_ref[0] = (float)(x * g->steps + g->offw);
      pats[i].pt_ref[1] = (float)(y * g->steps + g->offh);
      float *s = store + (size_t)i * o->novals * 5;
      pats[i].tmp = s; pats[i].dxx = s + o->novals; pats[i].dyy = s + 2 * o->novals;
      pats[i].pdiff = s + 3 * o->novals; pats[i].pweight = s + 4 * o->novals; pats[i].scratch = scratch;
    }
  for (int i = 0; i < g->nopatches; ++i) {
    float pin[2] = {0.0f, 0.0f};
    if (prev) {
      int x = (int)floorf(pats[i].pt_ref[0] / 2), y = (int)floorf(pats[i].pt_ref[1] / 2);
      int k = y * (c->w / 2) + x;
      for (int d = 0; d < o->nop; ++d) pin[d] = prev[o->nop * k + d] * 2;
    }
    patch_run(c, o, im_a, im_a_dx, im_a_dy, im_b, pin, &pats[i]);
  }
  *store_out = store;
  return pats;
}

int ofo_oflow(const float *const *im_ao, const float *const *im_ao_dx, const float *const *im_ao_dy,
              const float *const *im_bo, const float *const *im_bo_dx, const float *const *im_bo_dy,
              int imgpadding, float *outflow, const float *initflow, int width, int height,
              const ofdis_params *p, float *const *cap_dis, float *const *cap_tv) {
  if (p->costfct < 0 || p->costfct > 2) return OFDIS_ERR_UNSUPPORTED;
  const int fb = p->usefbcon != 0;
  opt_t o;
  fill_opt(p, &o);
  const int nsc = p->sc_f - p->sc_l + 1;
  float **flows = (float **)calloc(nsc, sizeof(float *));
  float **flows_bw = (float **)calloc(nsc, sizeof(float *));
  int rc = 0;
  for (int sl = p->sc_f; sl >= p->sc_l; --sl) {
    const int ii = sl - p->sc_l;
    cam_t c, cr;
    fill_cam(p, width, height, imgpadding, sl, &c);
    cr = c;
    cr.camlr = 1; /* cpr: the right camera of the backward grid (oflow.cpp:155-157) */
    grid_t g;
    grid_geometry(&c, &o, &g);
    const size_t fsz = sizeof(float) * (size_t)c.w * c.h * o.nop;
    flows[ii] = (float *)malloc(fsz);
    if (fb) flows_bw[ii] = (float *)malloc(fsz);
    /* InitializeFromCoarserOF (patchgrid.cpp:195-211) or zero / initflow (oflow.cpp:206-217) */
    float *store = NULL, *store_bw = NULL;
    patch_t *pats = run_grid(&c, &o, &g, im_ao[sl], im_ao_dx[sl], im_ao_dy[sl], im_bo[sl],
                             (sl < p->sc_f) ? flows[ii + 1] : initflow, &store);
    patch_t *pats_bw = NULL;
    if (fb) /* grid_bw: template on image b, target image a, initialised from the coarser backward flow */
      pats_bw = run_grid(&cr, &o, &g, im_bo[sl], im_bo_dx[sl], im_bo_dy[sl], im_ao[sl],
                         (sl < p->sc_f) ? flows_bw[ii + 1] : NULL, &store_bw);
    float *dst = (sl == p->sc_l) ? outflow : flows[ii];
    aggregate(&c, &o, &g, pats, pats_bw, dst);
    if (fb && sl > p->sc_l) aggregate(&cr, &o, &g, pats_bw, pats, flows_bw[ii]); /* oflow.cpp:265-266 */
    if (cap_dis && cap_dis[sl]) memcpy(cap_dis[sl], dst, fsz);
    if (p->usetvref) {
      rc = var_refine(&c, &o, p, im_ao[sl], im_bo[sl], dst);
      if (!rc && fb && sl > p->sc_l) rc = var_refine(&cr, &o, p, im_bo[sl], im_ao[sl], flows_bw[ii]);
    }
    if (cap_tv && cap_tv[sl]) memcpy(cap_tv[sl], dst, fsz);
    if (sl == p->sc_l && dst != flows[ii]) memcpy(flows[ii], dst, fsz);
    free(store); free(pats);
    free(store_bw); free(pats_bw);
    if (rc) break;
  }
  for (int i = 0; i < nsc; ++i) {
    free(flows[i]);
    free(flows_bw[i]);
  }
  free(flows);
  free(flows_bw);
  return rc;
}

/* ------------------------------------------------------------------ upsample + crop (run_dense.cpp:407-415) */

/* cv::resize(INTER_LINEAR) on CV_32FC(nop), generic path (resizeGeneric_ + HResizeLinear + VResizeLinear). */
int ofo_upsample_crop(const float *flow_l, int wl, int hl, int nop, int scale_log2, int padw, int padh,
                      int width_org, int height_org, float *out) {
  const int offx = padw / 2, offy = padh / 2;
  if (scale_log2 == 0) {
    for (int y = 0; y < height_org; ++y)
      for (int x = 0; x < width_org; ++x)
        for (int k = 0; k < nop; ++k)
          out[((size_t)y * width_org + x) * nop + k] = flow_l[((size_t)(y + offy) * wl + (x + offx)) * nop + k];
    return 0;
  }
  const float fct = (float)pow(2.0, scale_log2);
  const int Wd = wl << scale_log2, Hd = hl << scale_log2;
  const double scale = 1.0 / (double)fct;
  const int n = width_org * nop;
  int *xs = (int *)malloc(sizeof(int) * width_org);
  float *xa = (float *)malloc(sizeof(float) * width_org);
  int *xl = (int *)malloc(sizeof(int) * width_org);
  /* per output value: the two source taps (the right one clamped into the row: it is selected away where
   * the horizontal interpolation is not linear), the weights 1 - fx, fx and the linear flag */
  int *i0 = (int *)malloc(sizeof(int) * n), *i1 = (int *)malloc(sizeof(int) * n), *lf = (int *)malloc(sizeof(int) * n);
  float *wa = (float *)malloc(sizeof(float) * n), *wb = (float *)malloc(sizeof(float) * n);
  float *rows[2] = {(float *)malloc(sizeof(float) * n), (float *)malloc(sizeof(float) * n)};
  int rid[2] = {-1, -1};
  int xmax = Wd;
  for (int dx = 0; dx < Wd; ++dx) {
    float fx = (float)((dx + 0.5) * scale - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx + 1 >= wl) {
      if (dx < xmax) xmax = dx;
      if (sx >= wl - 1) { fx = 0; sx = wl - 1; }
    }
    if (dx >= offx && dx < offx + width_org) {
      xs[dx - offx] = sx; xa[dx - offx] = fx; xl[dx - offx] = dx < xmax;
    }
  }
  /* xmax is monotone: re-derive the "linear" flag once the full scan is known */
  for (int x = 0; x < width_org; ++x) xl[x] = (x + offx) < xmax;
  for (int x = 0; x < width_org; ++x)
    for (int k = 0; k < nop; ++k) {
      const int i = x * nop + k;
      i0[i] = xs[x] * nop + k;
      i1[i] = (xs[x] + 1 < wl ? xs[x] + 1 : wl - 1) * nop + k;
      wa[i] = 1.f - xa[x];
      wb[i] = xa[x];
      lf[i] = xl[x];
    }
  for (int y = 0; y < height_org; ++y) {
    int dy = y + offy;
    float fy = (float)((dy + 0.5) * scale - 0.5);
    int sy = (int)floorf(fy);
    fy -= (float)sy;
    int r0 = sy >= 0 ? (sy < hl ? sy : hl - 1) : 0;
    int r1 = sy + 1 >= 0 ? (sy + 1 < hl ? sy + 1 : hl - 1) : 0;
    const float b0 = 1.f - fy, b1 = fy;
    const float *R[2];
    for (int r = 0; r < 2; ++r) {  /* the horizontally resized source row, computed once per source row */
      const int want = r == 0 ? r0 : r1;
      int slot = rid[0] == want ? 0 : (rid[1] == want ? 1 : -1);
      if (slot < 0) {
        slot = (rid[0] == (r == 0 ? r1 : r0)) ? 1 : 0;  /* keep the row the other tap still needs */
        const float *S = flow_l + (size_t)want * wl * nop;
        float *D = rows[slot];
        for (int i = 0; i < n; ++i) {
          const float s0 = S[i0[i]] * fct, s1 = S[i1[i]] * fct;
          const float lin = s0 * wa[i] + s1 * wb[i];
          D[i] = lf[i] ? lin : s0;
        }
        rid[slot] = want;
      }
      R[r] = rows[slot];
    }
    float *O = out + (size_t)y * n;
    for (int i = 0; i < n; ++i) O[i] = R[0][i] * b0 + R[1][i] * b1;
  }
  (void)Hd;
  free(rows[0]); free(rows[1]); free(xs); free(xa); free(xl); free(i0); free(i1); free(lf); free(wa); free(wb);
  return 0;
}

/* ------------------------------------------------------------------ whole pipeline (run_dense.cpp main) */

/* The initial-flow input of run_dense.cpp:356-379 (commented out upstream, restated for the initflow
 * boundary): the full-resolution flow is replicate-padded like the images (:299-312 with divisibility
 * 2^(sc_f+1), :302), scaled by sc_fct = 2^-(sc_f+1) (float) and cv::resize'd by the same factor with
 * INTER_AREA.  The factor is an integer, so OpenCV takes resizeAreaFast: per output value, the k x k block
 * in row-major order, summed four at a time (sum += ((a + b) + c) + d, CV_ENABLE_UNROLLED), times 1/k^2. */
void ofo_init_flow_area(const float *init, int width, int height, int nop, int padw, int padh, int sc_f,
                        float *out) {
  const int k = 1 << (sc_f + 1), area = k * k;
  const int wo = (width + padw) / k, ho = (height + padh) / k, l = padw / 2, t = padh / 2;
  const float sc = (float)pow(2.0, -sc_f - 1), scale = 1.f / (float)area;
  for (int y = 0; y < ho; ++y)
    for (int x = 0; x < wo; ++x)
      for (int c = 0; c < nop; ++c) {
#define IV(j) (init[((size_t)clampi(y * k + (j) / k - t, 0, height - 1) * width + \
                     clampi(x * k + (j) % k - l, 0, width - 1)) * nop + c] * sc)
        float sum = 0.0f;
        int j = 0;
        for (; j <= area - 4; j += 4) sum += IV(j) + IV(j + 1) + IV(j + 2) + IV(j + 3);
        for (; j < area; ++j) sum += IV(j);
#undef IV
        out[((size_t)y * wo + x) * nop + c] = sum * scale;
      }
}

int ofo_run_u8(const uint8_t *img_a, const uint8_t *img_b, int width, int height, const ofdis_params *p,
               float *flow_out, float *const *cap_dis, float *const *cap_tv) {
  return ofo_run_u8_init(img_a, img_b, NULL, width, height, p, flow_out, cap_dis, cap_tv);
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

int ofo_run_u8_init(const uint8_t *img_a, const uint8_t *img_b, const float *init, int width, int height,
                    const ofdis_params *p, float *flow_out, float *const *cap_dis, float *const *cap_tv) {
  return ofo_run_u8_stages(img_a, img_b, init, width, height, p, flow_out, cap_dis, cap_tv, NULL);
}

/* The same with the wall time of each stage (CPU-baseline breakdown): stage_s[0] divisibility padding,
 * [1] pyramid + gradients (both frames), [2] OFClass, [3] upsample + crop. */
int ofo_run_u8_stages(const uint8_t *img_a, const uint8_t *img_b, const float *init, int width, int height,
                      const ofdis_params *p, float *flow_out, float *const *cap_dis, float *const *cap_tv,
                      double *stage_s) {
  double t0 = stage_s ? now_s() : 0.0;
  const int noc = p->noc, nop = p->mode == OFDIS_MODE_OF ? 2 : 1, pad = p->p_samp_s;
  int padw, padh;
  ofo_divisibility_pad(width, height, p->sc_f + (init ? 1 : 0), &padw, &padh);  /* run_dense.cpp:302 */
  const int Wp = width + padw, Hp = height + padh, l = padw / 2, t = padh / 2;
  uint8_t *pa = (uint8_t *)malloc((size_t)Wp * Hp * noc), *pb = (uint8_t *)malloc((size_t)Wp * Hp * noc);
  for (int y = 0; y < Hp; ++y) { /* copyMakeBorder BORDER_REPLICATE (run_dense.cpp:309-310) */
    const size_t sr = (size_t)clampi(y - t, 0, height - 1) * width * noc, dr = (size_t)y * Wp * noc;
    memcpy(pa + dr + (size_t)l * noc, img_a + sr, (size_t)width * noc);
    memcpy(pb + dr + (size_t)l * noc, img_b + sr, (size_t)width * noc);
    for (int x = 0; x < Wp; ++x) {
      if (x >= l && x < l + width) { x = l + width - 1; continue; }
      const size_t so = sr + (size_t)clampi(x - l, 0, width - 1) * noc, d = dr + (size_t)x * noc;
      for (int c = 0; c < noc; ++c) {
        pa[d + c] = img_a[so + c];
        pb[d + c] = img_b[so + c];
      }
    }
  }
  float *pyr[6][32];
  memset(pyr, 0, sizeof(pyr));
  int rc = 0;
  for (int s = p->sc_l; s <= p->sc_f; ++s) {
    size_t n = (size_t)((Wp >> s) + 2 * pad) * ((Hp >> s) + 2 * pad) * noc;
    for (int k = 0; k < 6; ++k) pyr[k][s] = (float *)malloc(sizeof(float) * n);
  }
  if (stage_s) {
    const double t = now_s();
    stage_s[0] = t - t0;
    t0 = t;
  }
  rc = ofo_build_pyramid_ex(pa, Wp, Hp, noc, p->sc_f, p->sc_l, pad, p->gradmag, pyr[0], pyr[1], pyr[2]);
  if (!rc) rc = ofo_build_pyramid_ex(pb, Wp, Hp, noc, p->sc_f, p->sc_l, pad, p->gradmag, pyr[3], pyr[4], pyr[5]);
  if (stage_s) {
    const double t = now_s();
    stage_s[1] = t - t0;
    t0 = t;
  }
  const int wl = Wp >> p->sc_l, hl = Hp >> p->sc_l;
  float *fl = (float *)malloc(sizeof(float) * (size_t)wl * hl * nop);
  float *ini = NULL;
  if (init) {
    ini = (float *)malloc(sizeof(float) * (size_t)(Wp >> (p->sc_f + 1)) * (Hp >> (p->sc_f + 1)) * nop);
    ofo_init_flow_area(init, width, height, nop, padw, padh, p->sc_f, ini);
  }
  if (!rc)
    rc = ofo_oflow((const float *const *)pyr[0], (const float *const *)pyr[1], (const float *const *)pyr[2],
                   (const float *const *)pyr[3], (const float *const *)pyr[4], (const float *const *)pyr[5], pad, fl,
                   ini, Wp, Hp, p, cap_dis, cap_tv);
  if (stage_s) {
    const double t = now_s();
    stage_s[2] = t - t0;
    t0 = t;
  }
  if (!rc) rc = ofo_upsample_crop(fl, wl, hl, nop, p->sc_l, padw, padh, width, height, flow_out);
  if (stage_s) stage_s[3] = now_s() - t0;
  free(fl);
  free(ini);
  for (int s = p->sc_l; s <= p->sc_f; ++s)
    for (int k = 0; k < 6; ++k) free(pyr[k][s]);
  free(pa); free(pb);
  return rc;
}

/* Exported for pinning tests: one VarRefClass run at scale `level` (refine_variational.cpp:25-116). */
int ofo_refine_level(const float *im_ao, const float *im_bo, int w, int h, int imgpadding, int level,
                     const ofdis_params *p, float *flow) {
  opt_t o;
  fill_opt(p, &o);
  cam_t c;
  memset(&c, 0, sizeof(c));
  c.w = w; c.h = h; c.pad = imgpadding; c.tmp_w = w + 2 * imgpadding; c.curr_lv = level; c.camlr = 0;
  return var_refine(&c, &o, p, im_ao, im_bo, flow);
}
