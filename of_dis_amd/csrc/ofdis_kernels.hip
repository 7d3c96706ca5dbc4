// ofdis_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the DIS optical-flow hot path.
//
// Every kernel keeps the reference's floating-point evaluation order (no FMA contraction: the file is
// built with -ffp-contract=off and the pragma below; division and sqrt are the correctly rounded HIP
// defaults), so results are bit-identical to the CPU restatement in oracle/ and hence, for the
// variational part, to the reference's own FDF1.0.1 code.
//
// Kernels (reference function they replace):
//   k_pyr_base      run_dense.cpp:299-312 + :151 (divisibility pad + 2^l box mean, exact in fp32)
//   k_pyr_down      run_dense.cpp:151 (cv::resize .5 = 2x2 mean)
//   k_pyr_pad_grad  run_dense.cpp:157-178 (Sobel/8 reflect-101 + replicate / zero padding)
//   k_patch         patch.cpp:55-295 (one wave64 per patch; Eigen-order reductions through LDS)
//   k_aggregate     patchgrid.cpp:213-275,377-397 (gather form, serial patch order, no atomics)
//   k_tv_prep       opticalflow_aux.c:31-75 + :88-99 (warp, mask, mean / temporal images)
//   k_tv_deriv1/2   opticalflow_aux.c:101-107 (5-tap derivative filters)
//   k_tv_smooth     opticalflow_aux.c:138-160 (robust smoothness weight)
//   k_tv_system     opticalflow_aux.c:161-223,408-747 (diffusivities + data term + laplacian)
//   k_tv_sor_pipe   solver.c:83-433 / :439-471 (exact lexicographic order: register-pipelined wavefront)
//   k_tv_sor        same, generic global-memory wavefront (any size; also solver.c:34-78 fallback)
//   k_tv_final      refine_variational.cpp:209-227,305-323
//   k_upsample      run_dense.cpp:407-415 (x2^l, cv::resize INTER_LINEAR, crop)
#include "ofdis_internal.h"
#include "ofdis_math.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#pragma clang fp contract(off)

namespace ofdis {
// 16-byte vector with 4-byte alignment: dword-aligned global_load_dwordx4 (gfx950 allows unaligned vector loads)
typedef float float4_u __attribute__((ext_vector_type(4), aligned(4)));
typedef float float4_v __attribute__((ext_vector_type(4)));

namespace {

#include "ofdis_tv_dev.inc"  // clampi, ssemin/max, skewed indexing, data term, smoothness, system
#include "ofdis_agg_dev.inc"  // aggregation weights, slot planes, the own-grid gather

inline unsigned ceil_div(long a, long b) { return (unsigned)((a + b - 1) / b); }

// XCD-aware block order (T1 of the CDNA guide): the dispatcher deals workgroups to the 8 XCDs round robin by
// linear id, each XCD with its own L2.  Linear id L runs block number L / 8 of the contiguous eighth of the
// grid (frame-major) that L's XCD serves, so blocks that share data -- neighbouring rows of a skewed plane,
// neighbouring tiles of a frame -- are L2 neighbours.  Bijective for any grid size; uniform (scalar) math.
__device__ __forceinline__ uint3 xcd_block() {
  const unsigned gx = gridDim.x, gy = gridDim.y, gxy = gx * gy, nwg = gxy * gridDim.z;
  const unsigned orig = (blockIdx.z * gy + blockIdx.y) * gx + blockIdx.x;
  const unsigned q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  const unsigned w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  return make_uint3(w % gx, (w / gx) % gy, w / gxy);
}



// ------------------------------------------------------------------------------------------------ pyramid

__global__ __launch_bounds__(256) void k_pyr_base(PyrBaseArgs a) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
  if (x >= a.w) return;
  const long idx = ((long)f * a.h + y) * a.w + x;
  const long fs = (long)a.H0 * a.W0 * a.noc;
  const uint8_t *src = f < a.n ? a.img_a + (long)f * fs : a.img_b + (long)(f - a.n) * fs;
  const int B = 1 << a.log2s;
  // 2^l x 2^l box mean of the replicate-padded u8 image.  The sum is an integer < 2^24 and the scale
  // is a power of two, so this equals the reference's repeated ((a+b)+(c+d))*0.25 exactly (l <= 8).
  const float scale = 1.0f / (float)(1 << (2 * a.log2s));
  const int x0 = x * B - a.padl;
  // fast path: intensity image, block row fully inside and 16-byte aligned -> uint4 loads + v_sad_u8
  if (a.noc == 1 && B >= 16 && x0 >= 0 && x0 + B <= a.W0 && ((((uintptr_t)src) + x0) & 15) == 0 && (a.W0 & 15) == 0) {
    unsigned sum = 0;
    for (int by = 0; by < B; ++by) {
      const int yy = clampi(y * B + by - a.padt, 0, a.H0 - 1);
      const uint4 *row = reinterpret_cast<const uint4 *>(src + (long)yy * a.W0 + x0);
      for (int q = 0; q < B / 16; ++q) {
        const uint4 v = row[q];
        sum = __builtin_amdgcn_sad_u8(v.x, 0u, sum);
        sum = __builtin_amdgcn_sad_u8(v.y, 0u, sum);
        sum = __builtin_amdgcn_sad_u8(v.z, 0u, sum);
        sum = __builtin_amdgcn_sad_u8(v.w, 0u, sum);
      }
    }
    a.out[idx] = (float)sum * scale;
    return;
  }
  for (int c = 0; c < a.noc; ++c) {
    unsigned sum = 0;
    for (int by = 0; by < B; ++by) {
      const int yy = clampi(y * B + by - a.padt, 0, a.H0 - 1);
      const uint8_t *row = src + (long)yy * a.W0 * a.noc + c;
      for (int bx = 0; bx < B; ++bx) sum += row[clampi(x0 + bx, 0, a.W0 - 1) * a.noc];
    }
    a.out[idx * a.noc + c] = (float)sum * scale;
  }
}

// Intensity images, 2^L = 4..32: one output pixel per thread over the flattened [2n][h][w] range (full
// waves even for narrow levels), the 2^L rows of the block unrolled so all loads are in flight at once,
// 4 / 8 / 16-byte loads summed with v_sad_u8.  Blocks that need horizontal clamping take the byte loop.
template <int L>
__global__ __launch_bounds__(256) void k_pyr_base_gray(PyrBaseArgs a) {
  constexpr int B = 1 << L;
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= 2L * a.n * a.h * a.w) return;
  const int x = (int)(t % a.w);
  const long r = t / a.w;
  const int y = (int)(r % a.h), f = (int)(r / a.h);
  const long fs = (long)a.H0 * a.W0;
  const uint8_t *src = f < a.n ? a.img_a + (long)f * fs : a.img_b + (long)(f - a.n) * fs;
  const float scale = 1.0f / (float)(1 << (2 * L));
  const int x0 = x * B - a.padl;
  constexpr int VB = B >= 16 ? 16 : B;  // bytes per load
  unsigned sum = 0;
  if (x0 >= 0 && x0 + B <= a.W0 && ((((uintptr_t)src) + x0) % VB) == 0 && (a.W0 % VB) == 0) {
    unsigned acc[B];
#pragma unroll
    for (int by = 0; by < B; ++by) {
      const int yy = clampi(y * B + by - a.padt, 0, a.H0 - 1);
      const uint8_t *row = src + (long)yy * a.W0 + x0;
      unsigned s2 = 0;
      if (VB == 16) {
#pragma unroll
        for (int q = 0; q < B / 16; ++q) {
          const uint4 v = reinterpret_cast<const uint4 *>(row)[q];
          s2 = __builtin_amdgcn_sad_u8(v.x, 0u, s2);
          s2 = __builtin_amdgcn_sad_u8(v.y, 0u, s2);
          s2 = __builtin_amdgcn_sad_u8(v.z, 0u, s2);
          s2 = __builtin_amdgcn_sad_u8(v.w, 0u, s2);
        }
      } else if (VB == 8) {
        const uint2 v = *reinterpret_cast<const uint2 *>(row);
        s2 = __builtin_amdgcn_sad_u8(v.x, 0u, s2);
        s2 = __builtin_amdgcn_sad_u8(v.y, 0u, s2);
      } else {
        s2 = __builtin_amdgcn_sad_u8(*reinterpret_cast<const unsigned *>(row), 0u, s2);
      }
      acc[by] = s2;
    }
#pragma unroll
    for (int by = 0; by < B; ++by) sum += acc[by];  // integer sum: order-free
  } else {
    for (int by = 0; by < B; ++by) {
      const int yy = clampi(y * B + by - a.padt, 0, a.H0 - 1);
      const uint8_t *row = src + (long)yy * a.W0;
      for (int bx = 0; bx < B; ++bx) sum += row[clampi(x0 + bx, 0, a.W0 - 1)];
    }
  }
  a.out[t] = (float)sum * scale;
}

// Colour images, 2^L = 4..16: one output pixel per thread over the flattened [2n][h][w] range, each of its 2^L rows
// read as 3 * 2^L / 4 dwords (4 pixels' B, G, R per 3 dwords) and each channel's bytes summed by v_sad_u8 under a
// byte mask -- exact integer sums like k_pyr_base's byte loop (the order of an integer sum is free).  Blocks that
// need horizontal clamping or are not dword-aligned take the byte loop.  Config C: 4.22 -> 1.50 ms per step
// (profiles/r06/s37).
template <int L>
__global__ __launch_bounds__(256) void k_pyr_base_rgb(PyrBaseArgs a) {
  constexpr int B = 1 << L, ND = 3 * B / 4;  // dwords per block row
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= 2L * a.n * a.h * a.w) return;
  const int x = (int)(t % a.w);
  const long r = t / a.w;
  const int y = (int)(r % a.h), f = (int)(r / a.h);
  const long fs = (long)a.H0 * a.W0 * 3;
  const uint8_t *src = f < a.n ? a.img_a + (long)f * fs : a.img_b + (long)(f - a.n) * fs;
  const float scale = 1.0f / (float)(1 << (2 * L));
  const int x0 = x * B - a.padl;
  unsigned sum[3] = {0u, 0u, 0u};
  if (x0 >= 0 && x0 + B <= a.W0 && (((uintptr_t)src + 3 * (long)x0) & 3) == 0 && ((3 * a.W0) & 3) == 0) {
    // byte k of a 12-byte group (pixels 4i .. 4i + 3) belongs to channel k % 3: its dword k / 4, byte k % 4
    constexpr unsigned M[3][3] = {{0xFF0000FFu, 0x00FF0000u, 0x0000FF00u},
                                  {0x0000FF00u, 0xFF0000FFu, 0x00FF0000u},
                                  {0x00FF0000u, 0x0000FF00u, 0xFF0000FFu}};
    unsigned v[B][ND];
#pragma unroll
    for (int by = 0; by < B; ++by) {
      const int yy = clampi(y * B + by - a.padt, 0, a.H0 - 1);
      const unsigned *row = reinterpret_cast<const unsigned *>(src + ((long)yy * a.W0 + x0) * 3);
#pragma unroll
      for (int k = 0; k < ND; ++k) v[by][k] = row[k];
    }
#pragma unroll
    for (int by = 0; by < B; ++by)
#pragma unroll
      for (int k = 0; k < ND; ++k)
#pragma unroll
        for (int c = 0; c < 3; ++c) sum[c] = __builtin_amdgcn_sad_u8(v[by][k] & M[c][k % 3], 0u, sum[c]);
  } else {
    for (int c = 0; c < 3; ++c)
      for (int by = 0; by < B; ++by) {
        const int yy = clampi(y * B + by - a.padt, 0, a.H0 - 1);
        const uint8_t *row = src + (long)yy * a.W0 * 3 + c;
        for (int bx = 0; bx < B; ++bx) sum[c] += row[clampi(x0 + bx, 0, a.W0 - 1) * 3];
      }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) a.out[t * 3 + c] = (float)sum[c] * scale;
}

// One thread per output value over the flattened [2n][h][w * noc] range (full waves on narrow levels).
__global__ __launch_bounds__(256) void k_pyr_down(PyrDownArgs a) {
  const int rw = a.w * a.noc;
  const long total = (long)a.n2 * a.h * rw;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
  const long r = t / rw;
  const int xc = (int)(t - r * rw), y = (int)(r % a.h), f = (int)(r / a.h);
  const int x = xc / a.noc, c = xc - x * a.noc;
  const long idx = (((long)f * a.h + y) * a.w + x) * a.noc + c;
  const int sw = 2 * a.w;
  const float *s = a.src + (long)f * (2 * a.h) * sw * a.noc;
  const float p = s[((2 * y) * sw + 2 * x) * a.noc + c], q = s[((2 * y) * sw + 2 * x + 1) * a.noc + c];
  const float u = s[((2 * y + 1) * sw + 2 * x) * a.noc + c], v = s[((2 * y + 1) * sw + 2 * x + 1) * a.noc + c];
  a.dst[idx] = ((p + q) + (u + v)) * 0.25f;
  }
}

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  if (i < 0) return -i;
  if (i >= n) return 2 * n - 2 - i;
  return i;
}

// Gradient-magnitude base level (oracle: ofo_build_pyramid_ex): Sobel ksize 3 x 1/8 with reflect-101 at the
// padded frame's border, on the replicate-padded u8 frame; same expression trees as k_pyr_pad_grad.
__global__ __launch_bounds__(256) void k_pyr_gradmag(PyrGradmagArgs a) {
  const int X = blockIdx.x * blockDim.x + threadIdx.x, Y = blockIdx.y, f = blockIdx.z;
  if (X >= a.Wp) return;
  const long fs = (long)a.H0 * a.W0;
  const uint8_t *src = f < a.n ? a.img_a + (long)f * fs : a.img_b + (long)(f - a.n) * fs;
  const int xm = reflect101(X - 1, a.Wp), xp = reflect101(X + 1, a.Wp);
  const int ym = reflect101(Y - 1, a.Hp), yp = reflect101(Y + 1, a.Hp);
  auto px = [&](int xx, int yy) {  // replicate divisibility padding (run_dense.cpp:307-311)
    return (float)src[(long)clampi(yy - a.padt, 0, a.H0 - 1) * a.W0 + clampi(xx - a.padl, 0, a.W0 - 1)];
  };
  const float tm = px(xp, ym) - px(xm, ym);
  const float t0 = px(xp, Y) - px(xm, Y);
  const float tp = px(xp, yp) - px(xm, yp);
  const float sm = (px(xm, ym) + px(xp, ym)) * 0.125f + px(X, ym) * 0.25f;
  const float sp = (px(xm, yp) + px(xp, yp)) * 0.125f + px(X, yp) * 0.25f;
  const float dx = (tm + tp) * 0.125f + t0 * 0.25f, dy = sp - sm;
  a.out[((long)f * a.Hp + Y) * a.Wp + X] = sqrtf(dx * dx + dy * dy);
}

// One thread per padded pixel over the flattened [2n][H][W] range (full waves on narrow levels: a 136-wide
// padded 1080p level 4 filled 53 % of a row-per-block launch's lanes).
__global__ __launch_bounds__(256) void k_pyr_pad_grad(PyrPadGradArgs a) {
  const int W = a.w + 2 * a.pad, H = a.h + 2 * a.pad;
  const long total = (long)a.n2 * H * W;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
  const long r = t / W;
  const int X = (int)(t - r * W), Y = (int)(r % H), f = (int)(r / H);
  const long idx = ((long)f * H + Y) * W + X;
  const int sx = X - a.pad, sy = Y - a.pad;
  const int noc = a.noc, w = a.w;
  const float *L = a.lvl + (long)f * a.h * a.w * noc;
  const bool inside = sx >= 0 && sx < a.w && sy >= 0 && sy < a.h;
  for (int c = 0; c < noc; ++c) {
    const long o = idx * noc + c;
    if (inside) {
      const int xm = reflect101(sx - 1, a.w), xp = reflect101(sx + 1, a.w);
      const int ym = reflect101(sy - 1, a.h), yp = reflect101(sy + 1, a.h);
#define PX(xx, yy) L[((yy) * w + (xx)) * noc + c]
      const float tm = PX(xp, ym) - PX(xm, ym);
      const float t0 = PX(xp, sy) - PX(xm, sy);
      const float tp = PX(xp, yp) - PX(xm, yp);
      const float sm = (PX(xm, ym) + PX(xp, ym)) * 0.125f + PX(sx, ym) * 0.25f;
      const float sp = (PX(xm, yp) + PX(xp, yp)) * 0.125f + PX(sx, yp) * 0.25f;
      a.img[o] = PX(sx, sy);
      a.dx[o] = (tm + tp) * 0.125f + t0 * 0.25f;
      a.dy[o] = sp - sm;
#undef PX
    } else {
      a.img[o] = L[(clampi(sy, 0, a.h - 1) * w + clampi(sx, 0, a.w - 1)) * noc + c];
      a.dx[o] = 0.0f;
      a.dy[o] = 0.0f;
    }
  }
  }
}

// Colour images: one thread per output VALUE over the flattened [2n][H][W * NOC] range (the loop above runs the
// channels inside a thread: three stride-3 store instructions per array and pixel), the same expressions.  Config
// C: 4.70 -> 3.49 ms per step (profiles/r06/s35).
template <int NOC>
__global__ __launch_bounds__(256) void k_pyr_pad_grad_v(PyrPadGradArgs a) {
  const int W = a.w + 2 * a.pad, H = a.h + 2 * a.pad, RW = W * NOC;
  const long total = (long)a.n2 * H * RW;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const long r = t / RW;
    const int xc = (int)(t - r * RW), Y = (int)(r % H), f = (int)(r / H);
    const int X = xc / NOC, c = xc - X * NOC;
    const int sx = X - a.pad, sy = Y - a.pad;
    const int w = a.w;
    const float *L = a.lvl + (long)f * a.h * a.w * NOC;
    if (sx >= 0 && sx < a.w && sy >= 0 && sy < a.h) {
      const int xm = reflect101(sx - 1, a.w), xp = reflect101(sx + 1, a.w);
      const int ym = reflect101(sy - 1, a.h), yp = reflect101(sy + 1, a.h);
#define PX(xx, yy) L[((yy) * w + (xx)) * NOC + c]
      const float tm = PX(xp, ym) - PX(xm, ym);
      const float t0 = PX(xp, sy) - PX(xm, sy);
      const float tp = PX(xp, yp) - PX(xm, yp);
      const float sm = (PX(xm, ym) + PX(xp, ym)) * 0.125f + PX(sx, ym) * 0.25f;
      const float sp = (PX(xm, yp) + PX(xp, yp)) * 0.125f + PX(sx, yp) * 0.25f;
      a.img[t] = PX(sx, sy);
      a.dx[t] = (tm + tp) * 0.125f + t0 * 0.25f;
      a.dy[t] = sp - sm;
#undef PX
    } else {
      a.img[t] = L[(clampi(sy, 0, a.h - 1) * w + clampi(sx, 0, a.w - 1)) * NOC + c];
      a.dx[t] = 0.0f;
      a.dy[t] = 0.0f;
    }
  }
}

// ------------------------------------------------------------------------------------------------ DIS patches

constexpr int kPatchWaves = 4;

template <int N>
__device__ __forceinline__ float row_shl(float v) {  // lane i <- lane i+N within its 16-lane row (else 0)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x100 + N, 0xF, 0xF, false));
}

// Eigen's SSE redux order for a dynamic vector (redux_impl, LinearVectorizedTraversal): two 4-lane packet
// accumulators over packet pairs, res0 + res1, odd trailing packet, predux (l0 + l2) + (l1 + l3).  Value v
// of a slot chain (slot = v % 8) is accumulated in v order.  R arrays are reduced at once: lanes
// (r = lane / 8, s = lane % 8) walk chain s of array r, then the 8 lanes of a group combine by DPP exactly
// like the packet tree.  Returns the R totals as wave-uniform values.
//
// JM == 1 (n <= 64, one value per lane): the arrays were stored TRANSPOSED (v -> (v % 8) * 8 + v / 8), so a
// chain is 8 contiguous floats: two ds_read_b128 per lane.  JM > 1: stored as lds[r * rs + v].
template <int R, int JM>
__device__ __forceinline__ void eigen_reduce(const float *lds, int rs, int n, int lane, float (&out)[R]) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int r = lane >> 3, s = lane & 7;
  const int pairs = n >> 3;
  const bool odd = ((n >> 2) & 1) != 0;
  float acc = 0.0f, first = 0.0f, tail = 0.0f;
  if (r < R) {
    if (JM == 1) {
      const float4 A = *reinterpret_cast<const float4 *>(lds + r * 64 + s * 8);
      const float4 B = *reinterpret_cast<const float4 *>(lds + r * 64 + s * 8 + 4);
      const float e[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
      first = e[0];
      acc = first;
#pragma unroll
      for (int c = 1; c < 8; ++c)
        if (c < pairs) acc = acc + e[c];
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (c == pairs) tail = e[c];
    } else {
      const float *x = lds + r * rs;
      first = x[s];
      acc = first;
      for (int c = 1; c < pairs; ++c) acc = acc + x[s + 8 * c];
      tail = x[pairs * 8 + s];
    }
  }
  float rl = pairs > 0 ? acc + row_shl<4>(acc) : first;
  if (odd && pairs > 0) rl = rl + tail;
  const float t = rl + row_shl<2>(rl);
  const float tot = t + row_shl<1>(t);
#pragma unroll
  for (int k = 0; k < R; ++k)
    out[k] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tot), k * 8));
  __builtin_amdgcn_wave_barrier();
}

template <int JM>
__device__ __forceinline__ void lds_store(float *lds, int n, int lane, const float (&v)[JM]) {
  if (JM == 1) {
    lds[(lane & 7) * 8 + (lane >> 3)] = lane < n ? v[0] : 0.0f;
    return;
  }
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const int e = lane + 64 * j;
    if (e < n) lds[e] = v[j];
  }
}

// Eigen LLT<2x2> (unblocked llt_inplace: a non-positive pivot stops the factorisation and leaves the raw
// entries) -- the factor depends only on the Hessian, so it is computed once per patch.
struct Llt2 {
  float L00, L10, L11;
};
__device__ __forceinline__ Llt2 llt2_factor(float H00, float H01, float H11) {
  Llt2 f{H00, H01, H11};
  if (!(H00 <= 0.0f)) {
    f.L00 = sqrtf(H00);
    f.L10 = H01 / f.L00;
    const float t = H11 - f.L10 * f.L10;
    if (!(t <= 0.0f)) f.L11 = sqrtf(t);
  }
  return f;
}
// LLT::solve: unrolled lower then upper triangular substitution.
__device__ __forceinline__ void llt2_solve(const Llt2 &f, float b0, float b1, float &x0, float &x1) {
  const float y0 = b0 / f.L00;
  const float y1 = (b1 - f.L10 * y0) / f.L11;
  x1 = y1 / f.L11;
  x0 = (y0 - f.L10 * x1) / f.L00;
}
__device__ __forceinline__ float llt1_factor(float H) { return !(H <= 0.0f) ? sqrtf(H) : H; }
__device__ __forceinline__ float llt1_solve(float L, float b) {
  const float y = b / L;
  return y / L;
}

// The solves' divisions by the patch's constant pivots, three instructions each instead of the IEEE
// sequence (two v_div_scale, v_rcp, five FMAs, v_div_fmas, v_div_fixup): with y = RN(1/L) from one IEEE
// division per patch, q0 = a y, r = fma(-q0, L, a) (exact), q = fma(r, y, q0) is RN(a / L) by Markstein's
// theorem while nothing under- or overflows -- |L| in [2^-30, 2^30], |a| in [2^-60, 2^60] (every residual then
// normal).  tools/divcheck_l.c checks it against IEEE a / L on 6.4e9 pairs of that range (0 mismatches; a
// reciprocal one ulp off gives hundreds).  A lane with any numerator or pivot outside the range (zero, tiny,
// huge, inf, NaN, a failed factorisation) repeats the whole solve with IEEE divisions in a wave-uniform branch.
struct LltRcp {
  float r00, r11;  // RN(1 / L00), RN(1 / L11) (NOP = 1: r00 = RN(1 / L))
  bool ok;         // pivots in range and the fast form enabled
};
__device__ __forceinline__ bool mdiv_in(float a) { return fabsf(a) >= 0x1p-60f && fabsf(a) <= 0x1p60f; }
__device__ __forceinline__ bool mdiv_pivot(float L) { return fabsf(L) >= 0x1p-30f && fabsf(L) <= 0x1p30f; }
__device__ __forceinline__ float mdiv(float a, float L, float y) {
  const float q0 = a * y;
  const float r = __builtin_fmaf(-q0, L, a);
  return __builtin_fmaf(r, y, q0);
}
template <int NOP>
__device__ __forceinline__ LltRcp llt_rcp(const Llt2 &f, float L1, bool enable) {
  LltRcp r;
  if (NOP == 2) {
    r.r00 = 1.0f / f.L00;
    r.r11 = 1.0f / f.L11;
    r.ok = enable && mdiv_pivot(f.L00) && mdiv_pivot(f.L11);
  } else {
    r.r00 = 1.0f / L1;
    r.r11 = 0.0f;
    r.ok = enable && mdiv_pivot(L1);
  }
  return r;
}
__device__ __forceinline__ void llt2_solve_fast(const Llt2 &f, const LltRcp &rc, float b0, float b1, float &x0,
                                                float &x1) {
  const float y0 = mdiv(b0, f.L00, rc.r00);
  const float n1 = b1 - f.L10 * y0;
  const float y1 = mdiv(n1, f.L11, rc.r11);
  x1 = mdiv(y1, f.L11, rc.r11);
  const float n3 = y0 - f.L10 * x1;
  x0 = mdiv(n3, f.L00, rc.r00);
  const bool slow = !(rc.ok && mdiv_in(b0) && mdiv_in(n1) && mdiv_in(y1) && mdiv_in(n3));
  if (__builtin_amdgcn_ballot_w64(slow) != 0 && slow) llt2_solve(f, b0, b1, x0, x1);
}
__device__ __forceinline__ float llt1_solve_fast(float L, const LltRcp &rc, float b) {
  const float y = mdiv(b, L, rc.r00);
  float x = mdiv(y, L, rc.r00);
  const bool slow = !(rc.ok && mdiv_in(b) && mdiv_in(y));
  if (__builtin_amdgcn_ballot_w64(slow) != 0 && slow) x = llt1_solve(L, b);
  return x;
}

template <int JM>
struct PatchCtx {
  const float *B;
  int W, noc, p, pad, novals, lane, rs, costfct, patnorm;
  float *lds;
  int offs[JM];
};

// getPatchStaticBil (patch.cpp:345-413) + mean normalisation + LossComputeErrorImage (patch.cpp:221-273).
// Leaves pdiff / pweight per lane and returns the Eigen sums of |pweight|, dx * pdiff (, dy * pdiff).
template <int NOP, int JM>
__device__ __forceinline__ void patch_eval(const PatchCtx<JM> &c, float mx, float my, const float (&tmp)[JM],
                                           const float (&gx)[JM], const float (&gy)[JM], float (&pd)[JM],
                                           float (&pw)[JM], float (&red)[NOP + 1]) {
  const int pos0 = (int)ceilf(mx + 0.00001f) + c.pad;
  const int pos1 = (int)ceilf(my + 0.00001f) + c.pad;
  const int pos2 = (int)floorf(mx), pos3 = (int)floorf(my);
  const float rx = mx - (float)pos2, ry = my - (float)pos3;
  const float w0 = rx * ry, w1 = (1 - rx) * ry, w2 = rx * (1 - ry), w3 = (1 - rx) * (1 - ry);
  const long base = ((long)(pos1 - c.p / 2) * c.W + (pos0 - c.p / 2)) * c.noc;
  const long rowstep = (long)c.W * c.noc;
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    if (c.lane + 64 * j < c.novals) {
      const float *q = c.B + base + c.offs[j];
      const float A = q[0], Bv = q[-c.noc], C = q[-rowstep], D = q[-rowstep - c.noc];
      pd[j] = w0 * A + w1 * Bv + w2 * C + w3 * D;
    } else {
      pd[j] = 0.0f;
    }
  }
  if (c.patnorm > 0) {
    lds_store<JM>(c.lds, c.novals, c.lane, pd);
    float s[1];
    eigen_reduce<1, JM>(c.lds, c.rs, c.novals, c.lane, s);
    const float mean = s[0] / (float)c.novals;
#pragma unroll
    for (int j = 0; j < JM; ++j) pd[j] = pd[j] - mean;
  }
  float ab[JM], px[JM], py[JM];
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const float d = pd[j] - tmp[j];
    float w;
    if (c.costfct == 0) {
      pd[j] = d;
      w = fabsf(d);
    } else if (c.costfct == 1) {
      w = sqrt_nonneg(fabsf(d));
      pd[j] = copysignf(w, d);
    } else {
      w = sqrt_nonneg((sqrt_nonneg(1.0f + (d * d) / 25.0f) - 1.0f) * 50.0f);
      pd[j] = copysignf(w, d);
    }
    pw[j] = w;
    ab[j] = fabsf(w);
    px[j] = gx[j] * pd[j];
    py[j] = gy[j] * pd[j];
  }
  const int stride = JM == 1 ? 64 : c.rs;
  lds_store<JM>(c.lds, c.novals, c.lane, ab);
  lds_store<JM>(c.lds + stride, c.novals, c.lane, px);
  if (NOP == 2) lds_store<JM>(c.lds + 2 * stride, c.novals, c.lane, py);
  eigen_reduce<NOP + 1, JM>(c.lds, c.rs, c.novals, c.lane, red);
}

// One wave64 per patch: InitializePatch + SetTargetImage + OptimizeIter(p_init, true)
// (patch.cpp:55-210, patchgrid.cpp:98-141,195-211).  JM = values per lane (ceil(p*p*noc / 64)).
template <int NOP, int JM>
__global__ __launch_bounds__(256) void k_patch(PatchArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_all[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const LevelGeom &g = a.g;
  const long gp = (long)blockIdx.x * kPatchWaves + wid;
  if (gp >= (long)a.n * g.npatch) return;  // whole wave exits; the kernel has no block barrier
  const int f = (int)(gp / g.npatch), ip = (int)(gp % g.npatch);
  const int pxi = ip / g.noph, pyi = ip % g.noph;
  const float ptr0 = (float)(pxi * a.steps + g.offw), ptr1 = (float)(pyi * a.steps + g.offh);
  const long fs = (long)g.W * g.H * a.noc;

  PatchCtx<JM> c;
  c.B = a.img_b + f * fs;
  c.W = g.W; c.noc = a.noc; c.p = a.p; c.pad = g.pad; c.novals = a.novals;
  c.lane = lane; c.costfct = a.costfct; c.patnorm = a.patnorm;
  c.rs = ((a.novals + 31) / 32) * 32 + 8;
  c.lds = lds_all + wid * 3 * (JM == 1 ? 64 : c.rs);
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const int e = lane + 64 * j;
    const int ch = e % a.noc, q = e / a.noc;
    c.offs[j] = ((q / a.p) * g.W + (q % a.p)) * a.noc + ch;
  }
  const int stride = JM == 1 ? 64 : c.rs;

  // ---- template + gradients at the integer reference position (getPatchStaticNNGrad, patch.cpp:297-343)
  float tmp[JM], gx[JM], gy[JM], pd[JM], pw[JM];
  {
    const int px = (int)roundf(ptr0) + g.pad, py = (int)roundf(ptr1) + g.pad;
    const long base = ((long)(py - a.p / 2) * g.W + (px - a.p / 2)) * a.noc;
    const float *A = a.img_a + f * fs + base, *DX = a.dx_a + f * fs + base, *DY = a.dy_a + f * fs + base;
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      const bool ok = lane + 64 * j < a.novals;
      tmp[j] = ok ? A[c.offs[j]] : 0.0f;
      gx[j] = ok ? DX[c.offs[j]] : 0.0f;
      gy[j] = ok ? DY[c.offs[j]] : 0.0f;
      pd[j] = 0.0f;
      pw[j] = 0.0f;
    }
  }
  if (a.patnorm > 0) {
    lds_store<JM>(c.lds, a.novals, lane, tmp);
    float s[1];
    eigen_reduce<1, JM>(c.lds, c.rs, a.novals, lane, s);
    const float mean = s[0] / (float)a.novals;
#pragma unroll
    for (int j = 0; j < JM; ++j) tmp[j] = tmp[j] - mean;
  }
  // ---- ComputeHessian (patch.cpp:69-86)
  float H00, H01 = 0.0f, H11 = 0.0f;
  {
    float q0[JM], q1[JM], q2[JM];
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      q0[j] = gx[j] * gx[j];
      q1[j] = gx[j] * gy[j];
      q2[j] = gy[j] * gy[j];
    }
    lds_store<JM>(c.lds, a.novals, lane, q0);
    if (NOP == 2) {
      lds_store<JM>(c.lds + stride, a.novals, lane, q1);
      lds_store<JM>(c.lds + 2 * stride, a.novals, lane, q2);
      float hh[3];
      eigen_reduce<3, JM>(c.lds, c.rs, a.novals, lane, hh);
      H00 = hh[0]; H01 = hh[1]; H11 = hh[2];
      if (H00 * H11 - H01 * H01 == 0.0f) {
        H00 = (float)((double)H00 + 1e-10);
        H11 = (float)((double)H11 + 1e-10);
      }
    } else {
      float hh[1];
      eigen_reduce<1, JM>(c.lds, c.rs, a.novals, lane, hh);
      H00 = hh[0];
      if (H00 == 0.0f) H00 = (float)((double)H00 + 1e-10);
    }
  }
  const Llt2 fac = llt2_factor(H00, H01, H11);
  const float fac1 = llt1_factor(H00);
  const LltRcp lrc = llt_rcp<NOP>(fac, fac1, a.fdiv != 0);
  if (a.stage == 1) {  // timing diagnostic "pconst": construction only; one store keeps the work alive
    if (lane == 0) a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tmp[JM - 1];
    return;
  }
  // ---- initial parameters (InitializeFromCoarserOF, patchgrid.cpp:195-211)
  float pin0 = 0.0f, pin1 = 0.0f;
  if (a.prev) {
    const int x = (int)floorf(ptr0 / 2), y = (int)floorf(ptr1 / 2);
    const float *pv = a.prev + (long)f * a.prev_frame_stride + (long)(y * a.prev_w + x) * a.prev_elem_stride;
    pin0 = pv[0] * 2;
    if (NOP == 2) pin1 = pv[a.prev_comp_stride] * 2;
  }
  if (a.stage == 2) {  // "pconst + pinit": construction and initialisation
    if (lane == 0) a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tmp[JM - 1] + pin0 + pin1;
    return;
  }
  // ---- OptimizeStart (patch.cpp:117-154)
  float p0 = pin0, p1 = pin1, d0 = 0.0f, d1 = 0.0f;
  float pt0 = ptr0 + p0, pt1 = (NOP == 2) ? ptr1 + p1 : ptr1;
  const float st0 = pt0, st1 = pt1;
  float sq = (float)1e-10, sq_init = (float)1e-10, mares = (float)1e20, mares_old = (float)1e20;
  int cnt = 0;
  bool converged = false;
  float b0 = 0.0f, b1 = 0.0f;
  auto oob = [&](float x, float y) { return x < g.tmp_lb || y < g.tmp_lb || x > g.tmp_ubw || y > g.tmp_ubh; };
  auto err = [&]() {  // OptimizeComputeErrImg (patch.cpp:275-295)
    float red[NOP + 1];
    patch_eval<NOP, JM>(c, pt0, pt1, tmp, gx, gy, pd, pw, red);
    sq = (NOP == 2) ? d0 * d0 + d1 * d1 : d0 * d0;
    if (cnt == 1) sq_init = sq;
    mares_old = mares;
    mares = red[0] / (float)a.novals;
    const bool keep = (cnt < a.max_iter) & (mares > a.res_thresh) &
                      ((cnt < a.min_iter) | (sq / sq_init >= a.dp_thresh_sq)) &
                      ((cnt < a.min_iter) | (mares / mares_old <= a.dr_thresh));
    if (!keep) converged = true;
    b0 = red[1];
    if (NOP == 2) b1 = red[NOP];
  };
  if (oob(pt0, pt1)) {
    converged = true;
#pragma unroll
    for (int j = 0; j < JM; ++j) pw[j] = 0.0f;  // never written upstream; defined as 0
  } else {
    mares = 1e5f;
    err();
  }
  // ---- OptimizeIter loop (patch.cpp:156-210)
  while (!converged) {
    ++cnt;
    if (NOP == 2) {
      llt2_solve_fast(fac, lrc, b0, b1, d0, d1);
      p0 = p0 - d0;
      p1 = p1 - d1;
    } else {
      d0 = llt1_solve_fast(fac1, lrc, b0);
      p0 = p0 - d0;
      p0 = (a.camlr == 0) ? stdminf(p0, 0.0f) : stdmaxf(p0, 0.0f);
    }
    pt0 = ptr0 + p0;
    if (NOP == 2) pt1 = ptr1 + p1;
    const float ex = st0 - pt0, ey = st1 - pt1;
    if (ex * ex + ey * ey > a.outlier_sq || oob(pt0, pt1)) {
      p0 = pin0;
      p1 = pin1;
      pt0 = ptr0 + p0;
      if (NOP == 2) pt1 = ptr1 + p1;
      converged = true;
    }
    err();
  }
  // ---- outputs
  if (lane < NOP) a.p_iter[gp * NOP + lane] = lane == 0 ? p0 : p1;
  float *pwo = a.pweight + gp * a.novals;
#pragma unroll
  for (int j = 0; j < JM; ++j)
    if (lane + 64 * j < a.novals) pwo[lane + 64 * j] = pw[j];
}

// ---------------------------------------------------------------- DIS patches, eight lanes per patch
// Eight lanes per patch, eight patches per wave.  Lane s of a patch holds the values v = s + 8k (k < PAIRS)
// and, when p*p*noc is an odd number of 4-float packets, the tail value 8*PAIRS + (s & 3) (duplicated in
// lanes s and s^4).  Eigen's SSE reduction (two 4-lane packet accumulators, res0 + res1, odd packet,
// (l0 + l2) + (l1 + l3)) is then: the lane's own chain sum in registers, and a butterfly over lanes
// s^4, s^2, s^1 (DPP, within the 8-lane group) whose pairings are exactly the packet tree's -- additions
// commute bit-exactly, so every lane ends with the reference's total.  No LDS, and the per-patch scalar
// work (the 2x2 solve, the stopping tests) runs lane-parallel for eight patches at once.
__device__ __forceinline__ float grp_xor4(float v) {  // lane s <- lane s^4 (row_half_mirror, then quad xor 3)
  const int m = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true);
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(m, 0x1B, 0xF, 0xF, true));
}
__device__ __forceinline__ float grp_xor2(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
}
__device__ __forceinline__ float grp_xor1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
}
template <int PAIRS, int ODD>
__device__ __forceinline__ float grp_eigen_sum(const float (&x)[PAIRS + ODD]) {
  float r;
  if (PAIRS > 0) {
    float acc = x[0];
#pragma unroll
    for (int k = 1; k < PAIRS; ++k) acc = acc + x[k];
    r = acc + grp_xor4(acc);             // res0 + res1
    if (ODD) r = r + x[PAIRS];           // odd trailing packet
  } else {
    r = x[0];                            // a single packet
  }
  r = r + grp_xor2(r);                   // l0 + l2, l1 + l3
  return r + grp_xor1(r);                // (l0 + l2) + (l1 + l3)
}

template <int NOP, int PAIRS, int ODD>
__global__ __launch_bounds__(256) void k_patch8(PatchArgs a) {
  constexpr int V = PAIRS + ODD;
  const LevelGeom &g = a.g;
  const int s8 = threadIdx.x & 7;
  const long gp = (long)blockIdx.x * 32 + (threadIdx.x >> 3);
  const bool live = gp < (long)a.n * g.npatch;
  const long gq = live ? gp : 0;
  const int f = (int)(gq / g.npatch), ip = (int)(gq % g.npatch);
  const int pxi = ip / g.noph, pyi = ip % g.noph;
  const float ptr0 = (float)(pxi * a.steps + g.offw), ptr1 = (float)(pyi * a.steps + g.offh);
  const long fs = (long)g.W * g.H * a.noc;
  const int noc = a.noc, P = a.p, W = g.W;
  const float inv_n = 1.0f / (float)a.novals;
  const bool pow2 = (a.novals & (a.novals - 1)) == 0;  // x / n == x * (1/n) exactly for n = 2^k
  auto div_n = [&](float x) { return pow2 ? x * inv_n : x / (float)a.novals; };
  int offs[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int v = k < PAIRS ? s8 + 8 * k : 8 * PAIRS + (s8 & 3);
    const int ch = v % noc, q = v / noc;
    offs[k] = ((q / P) * W + (q % P)) * noc + ch;
  }
  // ---- template + gradients at the integer reference position (getPatchStaticNNGrad, patch.cpp:297-343)
  float tmp[V], gx[V], gy[V], pw[V];
  {
    const int px = (int)roundf(ptr0) + g.pad, py = (int)roundf(ptr1) + g.pad;
    const long base = ((long)(py - P / 2) * W + (px - P / 2)) * noc;
    const float *A = a.img_a + f * fs + base, *DX = a.dx_a + f * fs + base, *DY = a.dy_a + f * fs + base;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      tmp[k] = A[offs[k]];
      gx[k] = DX[offs[k]];
      gy[k] = DY[offs[k]];
      pw[k] = 0.0f;
    }
  }
  if (a.patnorm > 0) {
    const float mean = div_n(grp_eigen_sum<PAIRS, ODD>(tmp));
#pragma unroll
    for (int k = 0; k < V; ++k) tmp[k] = tmp[k] - mean;
  }
  // ---- ComputeHessian (patch.cpp:69-86)
  float H00, H01 = 0.0f, H11 = 0.0f;
  {
    float q0[V], q1[V], q2[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      q0[k] = gx[k] * gx[k];
      q1[k] = gx[k] * gy[k];
      q2[k] = gy[k] * gy[k];
    }
    H00 = grp_eigen_sum<PAIRS, ODD>(q0);
    if (NOP == 2) {
      H01 = grp_eigen_sum<PAIRS, ODD>(q1);
      H11 = grp_eigen_sum<PAIRS, ODD>(q2);
      if (H00 * H11 - H01 * H01 == 0.0f) {
        H00 = (float)((double)H00 + 1e-10);
        H11 = (float)((double)H11 + 1e-10);
      }
    } else if (H00 == 0.0f) {
      H00 = (float)((double)H00 + 1e-10);
    }
  }
  const Llt2 fac = llt2_factor(H00, H01, H11);
  const float fac1 = llt1_factor(H00);
  const LltRcp lrc = llt_rcp<NOP>(fac, fac1, a.fdiv != 0);
  if (a.stage == 1) {  // timing diagnostic "pconst": construction only; one store keeps the work alive
    if (live && s8 == 0) a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tmp[V - 1];
    return;
  }
  // ---- initial parameters (InitializeFromCoarserOF, patchgrid.cpp:195-211)
  float pin0 = 0.0f, pin1 = 0.0f;
  if (a.prev) {
    const int x = (int)floorf(ptr0 / 2), y = (int)floorf(ptr1 / 2);
    const float *pv = a.prev + (long)f * a.prev_frame_stride + (long)(y * a.prev_w + x) * a.prev_elem_stride;
    pin0 = pv[0] * 2;
    if (NOP == 2) pin1 = pv[a.prev_comp_stride] * 2;
  }
  if (a.stage == 2) {  // "pconst + pinit": construction and initialisation
    if (live && s8 == 0) a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tmp[V - 1] + pin0 + pin1;
    return;
  }
  const float *Bimg = a.img_b + f * fs;
  const long rowstep = (long)W * noc;
  // ---- OptimizeStart (patch.cpp:117-154)
  float p0 = pin0, p1 = pin1, d0 = 0.0f, d1 = 0.0f;
  float pt0 = ptr0 + p0, pt1 = (NOP == 2) ? ptr1 + p1 : ptr1;
  const float st0 = pt0, st1 = pt1;
  float sq = (float)1e-10, sq_init = (float)1e-10, mares = (float)1e20, mares_old = (float)1e20;
  int cnt = 0;
  bool converged = !live;
  float b0 = 0.0f, b1 = 0.0f;
  auto oob = [&](float x, float y) { return x < g.tmp_lb || y < g.tmp_lb || x > g.tmp_ubw || y > g.tmp_ubh; };
  auto err = [&]() {  // getPatchStaticBil + LossComputeErrorImage + OptimizeComputeErrImg (patch.cpp:221-413)
    const int pos0 = (int)ceilf(pt0 + 0.00001f) + g.pad;
    const int pos1 = (int)ceilf(pt1 + 0.00001f) + g.pad;
    const int pos2 = (int)floorf(pt0), pos3 = (int)floorf(pt1);
    const float rx = pt0 - (float)pos2, ry = pt1 - (float)pos3;
    const float w0 = rx * ry, w1 = (1 - rx) * ry, w2 = rx * (1 - ry), w3 = (1 - rx) * (1 - ry);
    const float *Q = Bimg + ((long)(pos1 - P / 2) * W + (pos0 - P / 2)) * noc;
    float pd[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float *q = Q + offs[k];
      const float A = q[0], Bv = q[-noc], C = q[-rowstep], D = q[-rowstep - noc];
      pd[k] = w0 * A + w1 * Bv + w2 * C + w3 * D;
    }
    if (a.patnorm > 0) {
      const float mean = div_n(grp_eigen_sum<PAIRS, ODD>(pd));
#pragma unroll
      for (int k = 0; k < V; ++k) pd[k] = pd[k] - mean;
    }
    float ab[V], ex[V], ey[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float d = pd[k] - tmp[k];
      float w, e;
      if (a.costfct == 0) {
        e = d;
        w = fabsf(d);
      } else if (a.costfct == 1) {
        w = sqrt_nonneg(fabsf(d));
        e = copysignf(w, d);
      } else {
        w = sqrt_nonneg((sqrt_nonneg(1.0f + (d * d) / 25.0f) - 1.0f) * 50.0f);
        e = copysignf(w, d);
      }
      pw[k] = w;
      ab[k] = fabsf(w);
      ex[k] = gx[k] * e;
      ey[k] = gy[k] * e;
    }
    const float r0 = grp_eigen_sum<PAIRS, ODD>(ab);
    b0 = grp_eigen_sum<PAIRS, ODD>(ex);
    if (NOP == 2) b1 = grp_eigen_sum<PAIRS, ODD>(ey);
    sq = (NOP == 2) ? d0 * d0 + d1 * d1 : d0 * d0;
    if (cnt == 1) sq_init = sq;
    mares_old = mares;
    mares = div_n(r0);
    const bool keep = (cnt < a.max_iter) & (mares > a.res_thresh) &
                      ((cnt < a.min_iter) | (sq / sq_init >= a.dp_thresh_sq)) &
                      ((cnt < a.min_iter) | (mares / mares_old <= a.dr_thresh));
    if (!keep) converged = true;
  };
  if (!converged) {
    if (oob(pt0, pt1)) {
      converged = true;  // pweight stays 0: never written upstream, defined as 0
    } else {
      mares = 1e5f;
      err();
    }
  }
  // ---- OptimizeIter loop (patch.cpp:156-210)
  while (!converged) {
    ++cnt;
    if (NOP == 2) {
      llt2_solve_fast(fac, lrc, b0, b1, d0, d1);
      p0 = p0 - d0;
      p1 = p1 - d1;
    } else {
      d0 = llt1_solve_fast(fac1, lrc, b0);
      p0 = p0 - d0;
      p0 = (a.camlr == 0) ? stdminf(p0, 0.0f) : stdmaxf(p0, 0.0f);
    }
    pt0 = ptr0 + p0;
    if (NOP == 2) pt1 = ptr1 + p1;
    const float ex = st0 - pt0, ey = st1 - pt1;
    if (ex * ex + ey * ey > a.outlier_sq || oob(pt0, pt1)) {
      p0 = pin0;
      p1 = pin1;
      pt0 = ptr0 + p0;
      if (NOP == 2) pt1 = ptr1 + p1;
      converged = true;
    }
    err();
  }
  // ---- outputs
  if (!live) return;
  if (s8 < NOP) a.p_iter[gp * NOP + s8] = s8 == 0 ? p0 : p1;
  float *pwo = a.pweight + gp * a.novals;
#pragma unroll
  for (int k = 0; k < PAIRS; ++k) pwo[s8 + 8 * k] = pw[k];
  if (ODD && s8 < 4) pwo[8 * PAIRS + s8] = pw[PAIRS];
}

// ---------------------------------------------------------------- DIS patches, any shape (eight lanes per patch)
// k_patch8's lane layout and reduction trees with the values walked by a runtime loop instead of held in
// registers, so every p^2 noc the reference accepts (a multiple of 4, patch.cpp:230) runs, however large:
// lane s of a patch visits v = s + 8k in k order -- exactly Eigen's packet-accumulator chain s -- and then
// its value of the odd trailing packet.  Nothing per value lives in registers or LDS: template, gradients
// and target samples are re-read per pass from the cache-resident pyramid.  The normalised template value
// is the same single subtraction A - mean as InitializePatch's (patch.cpp:341-342), so recomputing it
// gives the stored bits; the bilinear sample is recomputed for the pass after the mean (same bits).
struct ChainAcc {  // one Eigen packet-accumulator chain per lane + the lane's tail-packet value
  float acc = 0.0f, tail = 0.0f;
  __device__ __forceinline__ void add(int k, int pairs, float x) {
    if (k < pairs)
      acc = k == 0 ? x : acc + x;
    else
      tail = x;
  }
  // res0 + res1, odd packet, (l0 + l2) + (l1 + l3): grp_eigen_sum's tree
  __device__ __forceinline__ float total(int pairs, int odd) const {
    float r;
    if (pairs > 0) {
      r = acc + grp_xor4(acc);
      if (odd) r = r + tail;
    } else {
      r = tail;
    }
    r = r + grp_xor2(r);
    return r + grp_xor1(r);
  }
};

// Calls fn(k, off) for chain s8's values in k order (k == pairs: the tail-packet value 8 pairs + (s8 & 3)),
// off = the value's float offset inside a patch window of rows of pn = p * noc floats, rowstep apart.
template <class F>
__device__ __forceinline__ void chain_walk(int s8, int pairs, int odd, int pn, long rowstep, F &&fn) {
  int r = 0, c = s8;
  while (c >= pn) {
    c -= pn;
    ++r;
  }
  for (int k = 0; k < pairs; ++k) {
    fn(k, (long)r * rowstep + c);
    c += 8;
    while (c >= pn) {
      c -= pn;
      ++r;
    }
  }
  if (odd) {
    const int v = 8 * pairs + (s8 & 3);
    fn(pairs, (long)(v / pn) * rowstep + v % pn);
  }
}

template <int NOP>
__global__ __launch_bounds__(256) void k_patchg(PatchArgs a) {
  const LevelGeom &g = a.g;
  const int s8 = threadIdx.x & 7;
  const long gp = (long)blockIdx.x * 32 + (threadIdx.x >> 3);
  const bool live = gp < (long)a.n * g.npatch;
  const long gq = live ? gp : 0;
  const int f = (int)(gq / g.npatch), ip = (int)(gq % g.npatch);
  const int pxi = ip / g.noph, pyi = ip % g.noph;
  const float ptr0 = (float)(pxi * a.steps + g.offw), ptr1 = (float)(pyi * a.steps + g.offh);
  const long fs = (long)g.W * g.H * a.noc;
  const int noc = a.noc, P = a.p, W = g.W, pn = P * noc;
  const int pairs = a.novals >> 3, odd = (a.novals >> 2) & 1;
  const long rowstep = (long)W * noc;
  const float inv_n = 1.0f / (float)a.novals;
  const bool pow2 = (a.novals & (a.novals - 1)) == 0;  // x / n == x * (1/n) exactly for n = 2^k
  auto div_n = [&](float x) { return pow2 ? x * inv_n : x / (float)a.novals; };
  // ---- template + gradients at the integer reference position (getPatchStaticNNGrad, patch.cpp:297-343)
  const int rpx = (int)roundf(ptr0) + g.pad, rpy = (int)roundf(ptr1) + g.pad;
  const long rbase = (long)f * fs + ((long)(rpy - P / 2) * W + (rpx - P / 2)) * noc;
  const float *A = a.img_a + rbase, *DX = a.dx_a + rbase, *DY = a.dy_a + rbase;
  float tmean = 0.0f;
  if (a.patnorm > 0) {
    ChainAcc m;
    chain_walk(s8, pairs, odd, pn, rowstep, [&](int k, long o) { m.add(k, pairs, A[o]); });
    tmean = div_n(m.total(pairs, odd));
  }
  // ---- ComputeHessian (patch.cpp:69-86)
  float H00, H01 = 0.0f, H11 = 0.0f;
  {
    ChainAcc q0, q1, q2;
    chain_walk(s8, pairs, odd, pn, rowstep, [&](int k, long o) {
      const float gx = DX[o], gy = DY[o];
      q0.add(k, pairs, gx * gx);
      q1.add(k, pairs, gx * gy);
      q2.add(k, pairs, gy * gy);
    });
    H00 = q0.total(pairs, odd);
    if (NOP == 2) {
      H01 = q1.total(pairs, odd);
      H11 = q2.total(pairs, odd);
      if (H00 * H11 - H01 * H01 == 0.0f) {
        H00 = (float)((double)H00 + 1e-10);
        H11 = (float)((double)H11 + 1e-10);
      }
    } else if (H00 == 0.0f) {
      H00 = (float)((double)H00 + 1e-10);
    }
  }
  const Llt2 fac = llt2_factor(H00, H01, H11);
  const float fac1 = llt1_factor(H00);
  const LltRcp lrc = llt_rcp<NOP>(fac, fac1, a.fdiv != 0);
  const float tlast = A[0] - tmean;  // keeps the template work alive in the diagnostics below
  if (a.stage == 1) {  // timing diagnostic "pconst": construction only
    if (live && s8 == 0) a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tlast;
    return;
  }
  // ---- initial parameters (InitializeFromCoarserOF, patchgrid.cpp:195-211)
  float pin0 = 0.0f, pin1 = 0.0f;
  if (a.prev) {
    const int x = (int)floorf(ptr0 / 2), y = (int)floorf(ptr1 / 2);
    const float *pv = a.prev + (long)f * a.prev_frame_stride + (long)(y * a.prev_w + x) * a.prev_elem_stride;
    pin0 = pv[0] * 2;
    if (NOP == 2) pin1 = pv[a.prev_comp_stride] * 2;
  }
  if (a.stage == 2) {  // "pconst + pinit"
    if (live && s8 == 0) a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tlast + pin0 + pin1;
    return;
  }
  const float *Bimg = a.img_b + (long)f * fs;
  // getPatchStaticBil + mean + LossComputeErrorImage (patch.cpp:221-273,345-413) at (x, y): the Eigen sums
  // of |w|, dx e (, dy e); with pwo, the loss weights w are written instead
  auto eval = [&](float x, float y, float &r0, float &e0, float &e1, float *pwo) {
    const int pos0 = (int)ceilf(x + 0.00001f) + g.pad;
    const int pos1 = (int)ceilf(y + 0.00001f) + g.pad;
    const int pos2 = (int)floorf(x), pos3 = (int)floorf(y);
    const float rx = x - (float)pos2, ry = y - (float)pos3;
    const float w0 = rx * ry, w1 = (1 - rx) * ry, w2 = rx * (1 - ry), w3 = (1 - rx) * (1 - ry);
    const float *Q = Bimg + ((long)(pos1 - P / 2) * W + (pos0 - P / 2)) * noc;
    auto sample = [&](long o) {
      const float *q = Q + o;
      return w0 * q[0] + w1 * q[-noc] + w2 * q[-rowstep] + w3 * q[-rowstep - noc];
    };
    float mean = 0.0f;
    if (a.patnorm > 0) {
      ChainAcc m;
      chain_walk(s8, pairs, odd, pn, rowstep, [&](int k, long o) { m.add(k, pairs, sample(o)); });
      mean = div_n(m.total(pairs, odd));
    }
    ChainAcc sa, sx, sy;
    chain_walk(s8, pairs, odd, pn, rowstep, [&](int k, long o) {
      float pd = sample(o);
      if (a.patnorm > 0) pd = pd - mean;
      const float tmp = a.patnorm > 0 ? A[o] - tmean : A[o];
      const float d = pd - tmp;
      float w, e;
      if (a.costfct == 0) {
        e = d;
        w = fabsf(d);
      } else if (a.costfct == 1) {
        w = sqrt_nonneg(fabsf(d));
        e = copysignf(w, d);
      } else {
        w = sqrt_nonneg((sqrt_nonneg(1.0f + (d * d) / 25.0f) - 1.0f) * 50.0f);
        e = copysignf(w, d);
      }
      if (pwo) {
        const int v = k < pairs ? s8 + 8 * k : 8 * pairs + (s8 & 3);
        if (k < pairs || s8 < 4) pwo[v] = w;
      } else {
        sa.add(k, pairs, fabsf(w));
        sx.add(k, pairs, DX[o] * e);
        if (NOP == 2) sy.add(k, pairs, DY[o] * e);
      }
    });
    if (!pwo) {
      r0 = sa.total(pairs, odd);
      e0 = sx.total(pairs, odd);
      if (NOP == 2) e1 = sy.total(pairs, odd);
    }
  };
  // ---- OptimizeStart (patch.cpp:117-154)
  float p0 = pin0, p1 = pin1, d0 = 0.0f, d1 = 0.0f;
  float pt0 = ptr0 + p0, pt1 = (NOP == 2) ? ptr1 + p1 : ptr1;
  const float st0 = pt0, st1 = pt1;
  float sq = (float)1e-10, sq_init = (float)1e-10, mares = (float)1e20, mares_old = (float)1e20;
  int cnt = 0;
  bool converged = !live, start_oob = false;
  float b0 = 0.0f, b1 = 0.0f;
  auto oob = [&](float x, float y) { return x < g.tmp_lb || y < g.tmp_lb || x > g.tmp_ubw || y > g.tmp_ubh; };
  auto err = [&]() {  // OptimizeComputeErrImg (patch.cpp:275-295)
    float r0 = 0.0f;
    eval(pt0, pt1, r0, b0, b1, nullptr);
    sq = (NOP == 2) ? d0 * d0 + d1 * d1 : d0 * d0;
    if (cnt == 1) sq_init = sq;
    mares_old = mares;
    mares = div_n(r0);
    const bool keep = (cnt < a.max_iter) & (mares > a.res_thresh) &
                      ((cnt < a.min_iter) | (sq / sq_init >= a.dp_thresh_sq)) &
                      ((cnt < a.min_iter) | (mares / mares_old <= a.dr_thresh));
    if (!keep) converged = true;
  };
  if (!converged) {
    if (oob(pt0, pt1)) {
      converged = start_oob = true;  // pweight never written upstream: defined as 0
    } else {
      mares = 1e5f;
      err();
    }
  }
  // ---- OptimizeIter loop (patch.cpp:156-210)
  while (!converged) {
    ++cnt;
    if (NOP == 2) {
      llt2_solve_fast(fac, lrc, b0, b1, d0, d1);
      p0 = p0 - d0;
      p1 = p1 - d1;
    } else {
      d0 = llt1_solve_fast(fac1, lrc, b0);
      p0 = p0 - d0;
      p0 = (a.camlr == 0) ? stdminf(p0, 0.0f) : stdmaxf(p0, 0.0f);
    }
    pt0 = ptr0 + p0;
    if (NOP == 2) pt1 = ptr1 + p1;
    const float ex = st0 - pt0, ey = st1 - pt1;
    if (ex * ex + ey * ey > a.outlier_sq || oob(pt0, pt1)) {
      p0 = pin0;
      p1 = pin1;
      pt0 = ptr0 + p0;
      if (NOP == 2) pt1 = ptr1 + p1;
      converged = true;
    }
    err();
  }
  // ---- outputs: the loss weights of the last evaluation, i.e. at the final position (a pure function of it)
  if (!live) return;
  if (s8 < NOP) a.p_iter[gp * NOP + s8] = s8 == 0 ? p0 : p1;
  float *pwo = a.pweight + gp * a.novals;
  if (start_oob) {
    chain_walk(s8, pairs, odd, pn, rowstep, [&](int k, long) {
      const int v = k < pairs ? s8 + 8 * k : 8 * pairs + (s8 & 3);
      if (k < pairs || s8 < 4) pwo[v] = 0.0f;
    });
  } else {
    float r0, e0, e1;
    eval(pt0, pt1, r0, e0, e1, pwo);
  }
}

// ---------------------------------------------------------------- DIS patches, windowed (eight lanes per patch)
// Same lane layout, reduction trees and per-patch arithmetic as k_patch8, but the bilinear taps come from
// LDS: per iteration the eight lanes of a patch copy its (p+1) x (p+1) x noc sample window (rows of
// contiguous floats) from the target image with 16-byte loads into an LDS tile, then read the four taps of
// each value there (two ds_read2_b32: (D, C) and (B, A)).  Against four 4-byte gathers per value from L1 this
// issues (p+1) * ceil((p+1) noc / 4) / 8 vector loads per lane instead of 4 p^2 noc / 8 (p = 12: 7 instead
// of 72), which is what bounds the gather form (waves parked on vmcnt).  The loss weights of the last
// evaluation are not kept in registers: one more evaluation at the final position writes them (the
// evaluation is a pure function of the position: the same bits).
template <int P, int NOC>
struct PatchShape {
  static constexpr int NV = P * P * NOC;
  static constexpr int PAIRS = NV / 8;
  static constexpr int ODD = (NV / 4) & 1;
  static constexpr int V = PAIRS + ODD;
  static constexpr int WR = (P + 1) * NOC;  // window row (floats)
  static constexpr int Q4 = (WR + 3) / 4;   // 16-byte loads per window row
  static constexpr int RS = Q4 * 4;         // LDS row stride (floats)
  // LDS floats per patch, padded to 8 (mod 32): a ds_read2_b32 is banked (a/4) mod 32 per 32-lane half, i.e.
  // four patches of eight lanes; with their windows 8 banks apart the 8 consecutive values a patch's lanes
  // read never share a bank with another patch's (a group that wraps a window row still can: 2-way)
  static constexpr int WIN = (P + 1) * RS + (8 - ((P + 1) * RS) % 32 + 32) % 32;
  static constexpr int NQ = (P + 1) * Q4;   // 16-byte loads per window
  static constexpr int LPL = (NQ + 7) / 8;  // ... per lane
  // value v -> v + 8 KP advances the tap offsets by whole patch rows: KP = lcm(8, NV / P) / 8
  static constexpr int ROWV = P * NOC;
  static constexpr int gcd(int a, int b) { return b == 0 ? a : gcd(b, a % b); }
  static constexpr int KP = (8 / gcd(8, ROWV) * ROWV) / 8;
  static constexpr int KROWS = 8 * KP / ROWV;  // patch rows per KP values of a lane
  // big shapes (p = 12 RGB: 54 values per lane) trade registers for LDS reads: the taps are read twice (for
  // the mean, then for the loss) instead of keeping the samples, and the window offsets are recomputed
  static constexpr bool LEAN = V > 24;
};

// Eigen's SSE redux order (see grp_eigen_sum), accumulated value by value: add(k, x) for k = 0 .. V-1 in order.
template <int PAIRS, int ODD>
struct EigenAcc {
  float acc = 0.0f, tail = 0.0f;
  __device__ __forceinline__ void add(int k, float x) {
    if (k < PAIRS)
      acc = k == 0 ? x : acc + x;
    else
      tail = x;
  }
  __device__ __forceinline__ float total() const {
    float r;
    if (PAIRS > 0) {
      r = acc + grp_xor4(acc);
      if (ODD) r = r + tail;
    } else {
      r = tail;
    }
    r = r + grp_xor2(r);
    return r + grp_xor1(r);
  }
};

typedef float f2p __attribute__((ext_vector_type(2)));

// x / c, correctly rounded, for the divisors c = p^2 noc of the windowed shapes that are not powers of two:
// q0 = x * RN(1/c), r = x - q0 c (exact by FMA), q = q0 + r RN(1/c).  Checked against IEEE x / c for every
// finite float x (tools/divcheck.c): identical for x = 0 and 2^-60 <= |x| <= 2^100 when c is 144, 192 or 432;
// any other x of the wave (tiny, huge, inf, NaN) takes the IEEE division in a wave-uniform branch.
template <int C>
__device__ __forceinline__ float div_by_const(float x) {
  static_assert(C == 144 || C == 192 || C == 432, "divisor not checked by tools/divcheck.c");
  constexpr float c = (float)C, y = 1.0f / (float)C;
  const float q0 = x * y;
  const float r = __builtin_fmaf(-q0, c, x);
  float q = __builtin_fmaf(r, y, q0);
  q = x == 0.0f ? x : q;
  const float ax = fabsf(x);
  const bool slow = x != 0.0f && !(ax >= 0x1p-60f && ax <= 0x1p100f);
  if (__builtin_amdgcn_ballot_w64(slow) != 0) q = slow ? x / c : q;
  return q;
}

// Compile-time loops (the index is a constant expression: template arguments, asm immediates).
template <class F, int... Is>
__device__ __forceinline__ void static_for_seq(F &&f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_seq(f, std::make_integer_sequence<int, N>{});
}

// ds_read2_b32 of the dwords at byte address addr + 4 O0 and addr + 4 O1 into one register pair.  The
// compiler's own LDS load combining pairs adjacent dwords only; the packed patch evaluation needs two taps
// that lie whole window rows apart.  The compiler does not track these loads: lds_wait<N>() (at most N LDS /
// scalar-memory operations outstanding; LDS completes in order) then reg_fence() on each result order the
// consumers after the data has arrived.
template <int O0, int O1>
__device__ __forceinline__ f2p lds_read2(unsigned addr) {
  static_assert(O0 >= 0 && O1 >= 0 && O0 <= 255 && O1 <= 255, "ds_read2_b32 offsets are 8-bit dword counts");
  f2p r;
  asm volatile("ds_read2_b32 %0, %1 offset0:%2 offset1:%3" : "=v"(r) : "v"(addr), "n"(O0), "n"(O1) : "memory");
  return r;
}
template <int N>
__device__ __forceinline__ void lds_wait() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt is 4 bits");
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void reg_fence(f2p &x) { asm volatile("" : "+v"(x)); }

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// MINW: waves per SIMD the register allocation must allow (amdgpu_waves_per_eu).  COST: costfct as a
// compile-time constant (a runtime switch inside the unrolled value loop was if-converted: every value paid
// for the L1 and pseudo-Huber losses' square roots and division).
template <int NOP, int P, int NOC, int MINW, int COST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MINW))) void k_patchw(PatchArgs a) {
  const uint3 xb = xcd_block();
  using S = PatchShape<P, NOC>;
  // a big shape (LEAN: samples read twice instead of kept) keeps its samples when compiled for one wave per
  // SIMD (MINW 1): measured faster for the L2 cost, slower for the square-root costs (config C2 / C)
  constexpr bool LEAN = S::LEAN && MINW > 1;
  constexpr int PAIRS = S::PAIRS, ODD = S::ODD, V = S::V, RS = S::RS;
  extern __shared__ __attribute__((aligned(16))) float win_all[];
  const LevelGeom &g = a.g;
  const int s8 = threadIdx.x & 7;
  const long gp = (long)xb.x * 32 + (threadIdx.x >> 3);
  const bool live = gp < (long)a.n * g.npatch;
  const long gq = live ? gp : 0;
  const int f = (int)(gq / g.npatch), ip = (int)(gq % g.npatch);
  const int pxi = ip / g.noph, pyi = ip % g.noph;
  const float ptr0 = (float)(pxi * a.steps + g.offw), ptr1 = (float)(pyi * a.steps + g.offh);
  const long fs = (long)g.W * g.H * NOC;
  const int W = g.W;
  constexpr float inv_n = 1.0f / (float)S::NV;
  constexpr bool pow2 = (S::NV & (S::NV - 1)) == 0;  // x / n == x * (1/n) exactly for n = 2^k
  auto div_n = [&](float x) {
    if constexpr (pow2)
      return x * inv_n;
    else
      return div_by_const<S::NV>(x);
  };
  // PK: the per-value arithmetic of an evaluation on value pairs (k, k + 1) in packed fp32 -- every lane of a
  // v_pk_mul_f32 / v_pk_add_f32 rounds like the scalar instruction, so the pairs keep each value's operation
  // order; the taps of a pair come straight from one ds_read2_b32 into a register pair
  constexpr bool PK = !LEAN && S::ODD == 0 && V % (2 * S::KP) == 0;
  float *win = win_all + (threadIdx.x >> 3) * S::WIN;
  // value of slot k of this lane, and its D-tap offset in the window tile
  auto value = [&](int k) { return k < PAIRS ? s8 + 8 * k : 8 * PAIRS + (s8 & 3); };
  auto dtap = [&](int v) {
    const int ch = v % NOC, q = v / NOC;
    return (q / P) * RS + (q % P) * NOC + ch;
  };
  int dbase[S::KP < V ? S::KP : V];
#pragma unroll
  for (int k = 0; k < (S::KP < V ? S::KP : V); ++k) dbase[k] = dtap(value(k));
  const int dtail = dtap(value(V - 1));
  auto doff = [&](int k) {  // compile-time k
    if (ODD && k == V - 1) return dtail;
    return dbase[k % S::KP] + (k / S::KP) * S::KROWS * RS;
  };
  // ---- template + gradients at the integer reference position (getPatchStaticNNGrad, patch.cpp:297-343)
  float tmp[V], gx[V], gy[V];
  {
    const int px = (int)roundf(ptr0) + g.pad, py = (int)roundf(ptr1) + g.pad;
    const long base = ((long)(py - P / 2) * W + (px - P / 2)) * NOC;
    const float *A = a.img_a + f * fs + base, *DX = a.dx_a + f * fs + base, *DY = a.dy_a + f * fs + base;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const int v = value(k), ch = v % NOC, q = v / NOC;
      const int o = ((q / P) * W + (q % P)) * NOC + ch;
      tmp[k] = A[o];
      gx[k] = DX[o];
      gy[k] = DY[o];
    }
  }
  if (a.patnorm > 0) {
    EigenAcc<PAIRS, ODD> m;
#pragma unroll
    for (int k = 0; k < V; ++k) m.add(k, tmp[k]);
    const float mean = div_n(m.total());
#pragma unroll
    for (int k = 0; k < V; ++k) tmp[k] = tmp[k] - mean;
  }
  // ---- ComputeHessian (patch.cpp:69-86)
  float H00, H01 = 0.0f, H11 = 0.0f;
  {
    EigenAcc<PAIRS, ODD> h0, h1, h2;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      h0.add(k, gx[k] * gx[k]);
      if (NOP == 2) {
        h1.add(k, gx[k] * gy[k]);
        h2.add(k, gy[k] * gy[k]);
      }
    }
    H00 = h0.total();
    if (NOP == 2) {
      H01 = h1.total();
      H11 = h2.total();
      if (H00 * H11 - H01 * H01 == 0.0f) {
        H00 = (float)((double)H00 + 1e-10);
        H11 = (float)((double)H11 + 1e-10);
      }
    } else if (H00 == 0.0f) {
      H00 = (float)((double)H00 + 1e-10);
    }
  }
  const Llt2 fac = llt2_factor(H00, H01, H11);
  const float fac1 = llt1_factor(H00);
  const LltRcp lrc = llt_rcp<NOP>(fac, fac1, a.fdiv != 0);
  if (a.stage == 1) {  // timing diagnostic "pconst": construction only; one store keeps the work alive
    if (live && s8 == 0) a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tmp[V - 1];
    return;
  }
  // ---- initial parameters (InitializeFromCoarserOF, patchgrid.cpp:195-211)
  float pin0 = 0.0f, pin1 = 0.0f;
  if (a.prev) {
    const int x = (int)floorf(ptr0 / 2), y = (int)floorf(ptr1 / 2);
    const float *pv = a.prev + (long)f * a.prev_frame_stride + (long)(y * a.prev_w + x) * a.prev_elem_stride;
    pin0 = pv[0] * 2;
    if (NOP == 2) pin1 = pv[a.prev_comp_stride] * 2;
  }
  if (a.stage == 2) {  // "pconst + pinit": construction and initialisation
    if (live && s8 == 0) a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tmp[V - 1] + pin0 + pin1;
    return;
  }
  // template and gradients as value pairs for the packed form (register pairs; the scalar arrays die here)
  constexpr int V2 = PK ? V / 2 : 1;
  f2p tmp2[V2], gx2[V2], gy2[V2];
  // pair j = (k, k + KP) with k = (j / KP) 2 KP + j mod KP: the lane's values v and v + 8 KP are whole patch
  // rows (KROWS) apart, so their taps are a fixed number of window floats apart whatever the lane
  if (PK) {
#pragma unroll
    for (int j = 0; j < V2; ++j) {
      const int k = (j / S::KP) * 2 * S::KP + j % S::KP;
      tmp2[j] = f2p{tmp[k], tmp[k + S::KP]};
      gx2[j] = f2p{gx[k], gx[k + S::KP]};
      if (NOP == 2) gy2[j] = f2p{gy[k], gy[k + S::KP]};
    }
  }
  auto tmpv = [&](int k) -> float {  // compile-time k
    if constexpr (PK) {
      const int g = k / (2 * S::KP), r = k % (2 * S::KP);
      return r < S::KP ? tmp2[g * S::KP + r].x : tmp2[g * S::KP + r - S::KP].y;
    } else {
      return tmp[k];
    }
  };
  const float *Bimg = a.img_b + f * fs;
  // window loads of this lane: float4 e = s8 + 8 j of the (P+1) x Q4 tile
  constexpr int LPLK = LEAN ? 1 : S::LPL;
  int gofs[LPLK], lofs[LPLK];
  auto woff = [&](int j, int &go, int &lo) {
    const int e = s8 + 8 * j, e2 = e < S::NQ ? e : S::NQ - 1;
    const int row = e2 / S::Q4, c4 = e2 % S::Q4;
    go = row * W * NOC + c4 * 4;
    lo = row * RS + c4 * 4;
  };
  if (!LEAN) {
#pragma unroll
    for (int j = 0; j < LPLK; ++j) woff(j, gofs[j], lofs[j]);
  }
  // ---- OptimizeStart (patch.cpp:117-154)
  float p0 = pin0, p1 = pin1, d0 = 0.0f, d1 = 0.0f;
  float pt0 = ptr0 + p0, pt1 = (NOP == 2) ? ptr1 + p1 : ptr1;
  const float st0 = pt0, st1 = pt1;
  float sq = (float)1e-10, sq_init = (float)1e-10, mares = (float)1e20, mares_old = (float)1e20;
  int cnt = 0;
  bool converged = false;
  float b0 = 0.0f, b1 = 0.0f;
  auto oob = [&](float x, float y) { return x < g.tmp_lb || y < g.tmp_lb || x > g.tmp_ubw || y > g.tmp_ubh; };
  int lpos0 = -0x7fffffff, lpos1 = 0;  // integer tap position of the tile in LDS (none yet)
  // getPatchStaticBil + mean normalisation + LossComputeErrorImage (patch.cpp:221-413) at (pt0, pt1):
  // the residual sums r0 = sum |w|, b0 = sum dx e (, b1 = sum dy e); with `out`, the weights w are stored
  auto evaluate = [&](float &r0, float *out, auto store_t) {
    constexpr int STORE = decltype(store_t)::value;  // 0: the sums only; 1: the weights only, to `out`
    const int pos0 = (int)ceilf(pt0 + 0.00001f) + g.pad;
    const int pos1 = (int)ceilf(pt1 + 0.00001f) + g.pad;
    const int pos2 = (int)floorf(pt0), pos3 = (int)floorf(pt1);
    const float rx = pt0 - (float)pos2, ry = pt1 - (float)pos3;
    const float w0 = rx * ry, w1 = (1 - rx) * ry, w2 = rx * (1 - ry), w3 = (1 - rx) * (1 - ry);
    // window origin: the D tap of value 0, one row above and one column left of the A tap
    const float *Q = Bimg + ((long)(pos1 - P / 2 - 1) * W + (pos0 - P / 2 - 1)) * NOC;
    // the tile is a function of (pos0, pos1) alone: reloaded only when a patch of the wave has moved to
    // another integer tap position since its last load (late iterations mostly stay put)
    if (__builtin_amdgcn_ballot_w64(pos0 != lpos0 || pos1 != lpos1) != 0) {
    lpos0 = pos0;
    lpos1 = pos1;
    wave_lds_sync();  // the previous evaluation's tap reads are done before the tile is overwritten
    if (LEAN) {  // in batches of 4 loads: bounded registers in flight
#pragma unroll
      for (int j0 = 0; j0 < S::LPL; j0 += 4) {
        float4_u t[4];
        int lo[4];
#pragma unroll
        for (int j = j0; j < j0 + 4 && j < S::LPL; ++j) {
          int go;
          woff(j, go, lo[j - j0]);
          t[j - j0] = *reinterpret_cast<const float4_u *>(Q + go);
        }
#pragma unroll
        for (int j = j0; j < j0 + 4 && j < S::LPL; ++j)
          if (s8 + 8 * j < S::NQ) *reinterpret_cast<float4_v *>(win + lo[j - j0]) = t[j - j0];
      }
    } else {
#pragma unroll
      for (int j = 0; j < S::LPL; ++j) {
        const float4_u t = *reinterpret_cast<const float4_u *>(Q + gofs[j]);
        if (s8 + 8 * j < S::NQ) *reinterpret_cast<float4_v *>(win + lofs[j]) = t;
      }
    }
    wave_lds_sync();
    }
    if constexpr (PK && STORE == 0) {
      // value pairs (k, k + KP): tap X of both values is one ds_read2_b32 into a register pair (taps PD floats
      // apart), then ((w0 A + w1 B) + w2 C) + w3 D, (x - mean) - tmp and gx e run two values per packed
      // instruction; the Eigen chains (mean, |w|, gx e, gy e) stay scalar, value by value in order.  Groups of
      // 2 KP values; the next group's 4 KP reads are in flight while a group is computed.
      constexpr int KP = S::KP, PD = S::KROWS * RS, NG = V / (2 * KP);
      const unsigned wb = (unsigned)(uintptr_t)win;
      f2p pd2[V2], q[2][4];
      auto issue = [&](auto jc) {  // the four taps of pair j (in flight: this pair and the next)
        constexpr int j = decltype(jc)::value, i = j % KP, o0 = 2 * (j / KP) * PD;
        constexpr bool imm = o0 + RS + NOC + PD <= 255;  // else the row offset goes into the address
        constexpr int o = imm ? o0 : 0;
        const unsigned b = wb + 4u * (unsigned)dbase[i] + (imm ? 0u : 4u * (unsigned)o0);
        q[j & 1][0] = lds_read2<o, o + PD>(b);                        // D
        q[j & 1][1] = lds_read2<o + NOC, o + NOC + PD>(b);            // C
        q[j & 1][2] = lds_read2<o + RS, o + RS + PD>(b);              // B
        q[j & 1][3] = lds_read2<o + RS + NOC, o + RS + NOC + PD>(b);  // A
      };
      issue(std::integral_constant<int, 0>{});
      static_for<V2>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (j + 1 < V2) {
          issue(std::integral_constant<int, j + 1>{});
          lds_wait<4>();
        } else {
          lds_wait<0>();
        }
        f2p *t = q[j & 1];
        static_for<4>([&](auto ic) { reg_fence(t[decltype(ic)::value]); });
        f2p x = t[3] * w0 + t[2] * w1;
        x = x + t[1] * w2;
        x = x + t[0] * w3;
        pd2[j] = x;
      });
      EigenAcc<PAIRS, ODD> m;
      static_for<V>([&](auto kc) {  // value order: pair g KP + i holds values g 2KP + i (.x), g 2KP + KP + i (.y)
        constexpr int k = decltype(kc)::value, g = k / (2 * KP), r = k % (2 * KP);
        m.add(k, r < KP ? pd2[g * KP + r].x : pd2[g * KP + r - KP].y);
      });
      const float mean = a.patnorm > 0 ? div_n(m.total()) : 0.0f;
      EigenAcc<PAIRS, ODD> ab, ex, ey;
      static_for<NG>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        f2p qx[KP], qy[KP], wv[KP];
        static_for<KP>([&](auto ic) {
          constexpr int i = decltype(ic)::value, j = g * KP + i;
          const f2p d = (pd2[j] - mean) - tmp2[j];
          f2p e;
          if (COST == 0) {
            e = d;
            wv[i] = d;
          } else {
            float w[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const float dh = h ? d.y : d.x;
              w[h] = COST == 1 ? sqrt_nonneg(fabsf(dh))
                               : sqrt_nonneg((sqrt_nonneg(1.0f + (dh * dh) / 25.0f) - 1.0f) * 50.0f);
            }
            wv[i] = f2p{w[0], w[1]};
            e = f2p{copysignf(w[0], d.x), copysignf(w[1], d.y)};
          }
          qx[i] = gx2[j] * e;
          if (NOP == 2) qy[i] = gy2[j] * e;
        });
        static_for<2 * KP>([&](auto rc) {  // the chains in value order: .x halves, then .y halves
          constexpr int r = decltype(rc)::value, i = r % KP, h = r / KP, k = g * 2 * KP + r;
          ab.add(k, fabsf(h ? wv[i].y : wv[i].x));
          ex.add(k, h ? qx[i].y : qx[i].x);
          if (NOP == 2) ey.add(k, h ? qy[i].y : qy[i].x);
        });
      });
      r0 = ab.total();
      b0 = ex.total();
      if (NOP == 2) b1 = ey.total();
    } else {
    // (the compiler packs the products into v_pk_mul_f32 pairs itself; written as explicit float2 pairs
    // within a value -- (B, A), (D, C) -- they cost config E 5 % and made the LEAN shapes spill)
    auto sample = [&](int k) {
      const float *t = win + doff(k);
      const float D = t[0], C = t[NOC], Bv = t[RS], A = t[RS + NOC];
      return w0 * A + w1 * Bv + w2 * C + w3 * D;
    };
    constexpr int VK = LEAN ? 1 : V;
    float pd[VK];
    float mean = 0.0f;
    if (a.patnorm > 0 || !LEAN) {
      EigenAcc<PAIRS, ODD> m;
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const float x = sample(k);
        if (!LEAN) pd[k] = x;
        m.add(k, x);
      }
      if (a.patnorm > 0) mean = div_n(m.total());
    }
    EigenAcc<PAIRS, ODD> ab, ex, ey;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float x = (LEAN ? sample(k) : pd[k]) - mean;  // mean = 0 without normalisation: x - 0 == x
      const float d = x - tmpv(k);
      float w, e;
      if (COST == 0) {
        e = d;
        w = fabsf(d);
      } else if (COST == 1) {
        w = sqrt_nonneg(fabsf(d));
        e = copysignf(w, d);
      } else {
        w = sqrt_nonneg((sqrt_nonneg(1.0f + (d * d) / 25.0f) - 1.0f) * 50.0f);
        e = copysignf(w, d);
      }
      if (STORE == 0) {
        ab.add(k, fabsf(w));
        ex.add(k, gx[k] * e);
        if (NOP == 2) ey.add(k, gy[k] * e);
      } else {
        if (k < PAIRS) out[s8 + 8 * k] = w;
        else if (s8 < 4) out[8 * PAIRS + s8] = w;
      }
    }
    if (STORE == 0) {
      r0 = ab.total();
      b0 = ex.total();
      if (NOP == 2) b1 = ey.total();
    }
    }
  };
  // The evaluation is unrolled over the values; the loop holds one copy of it (start evaluation and every
  // iteration), the final weights-only evaluation another.  Per patch:
  //   OptimizeStart (patch.cpp:117-154): evaluate at the start position (unless it is out of bounds);
  //   OptimizeIter (patch.cpp:156-210): while not converged, solve, update, outlier reset, evaluate;
  //   then one more evaluation at the final position that stores the loss weights.
  float *pwo = a.pweight + gq * S::NV;
  bool start_oob = false, first = true;
  converged = !live;
  if (live && oob(pt0, pt1)) {  // converged at once; pweight never written upstream, defined as 0
#pragma unroll
    for (int k = 0; k < PAIRS; ++k) pwo[s8 + 8 * k] = 0.0f;
    if (ODD && s8 < 4) pwo[8 * PAIRS + s8] = 0.0f;
    converged = true;
    start_oob = true;
  } else {
    mares = 1e5f;
  }
  // (a wave-uniform exit test around a masked body: smaller code than the divergent while, same work)
  for (;;) {
    if (__builtin_amdgcn_ballot_w64(!converged) == 0) break;
    if (!converged) {
      if (!first) {
        ++cnt;
        if (NOP == 2) {
          llt2_solve_fast(fac, lrc, b0, b1, d0, d1);
          p0 = p0 - d0;
          p1 = p1 - d1;
        } else {
          d0 = llt1_solve_fast(fac1, lrc, b0);
          p0 = p0 - d0;
          p0 = (a.camlr == 0) ? stdminf(p0, 0.0f) : stdmaxf(p0, 0.0f);
        }
        pt0 = ptr0 + p0;
        if (NOP == 2) pt1 = ptr1 + p1;
        const float ex = st0 - pt0, ey = st1 - pt1;
        if (ex * ex + ey * ey > a.outlier_sq || oob(pt0, pt1)) {
          p0 = pin0;
          p1 = pin1;
          pt0 = ptr0 + p0;
          if (NOP == 2) pt1 = ptr1 + p1;
          converged = true;
        }
      }
      float r0 = 0.0f;
      evaluate(r0, nullptr, std::integral_constant<int, 0>());
      // OptimizeComputeErrImg (patch.cpp:275-295)
      sq = (NOP == 2) ? d0 * d0 + d1 * d1 : d0 * d0;
      if (cnt == 1) sq_init = sq;
      mares_old = mares;
      mares = div_n(r0);
      // the two rate tests count only from min_iter on: their divisions run in a wave-uniform branch that
      // the op-points (min_iter = max_iter) never enter
      bool rates = true;
      if (__builtin_amdgcn_ballot_w64(cnt >= a.min_iter) != 0)
        rates = (cnt < a.min_iter) | ((sq / sq_init >= a.dp_thresh_sq) & (mares / mares_old <= a.dr_thresh));
      const bool keep = (cnt < a.max_iter) & (mares > a.res_thresh) & rates;
      if (!keep) converged = true;
    }
    first = false;
  }
  if (live && !start_oob) {
    float r0;
    evaluate(r0, pwo, std::integral_constant<int, 1>());
  }
  if (live && s8 < NOP) a.p_iter[gp * NOP + s8] = s8 == 0 ? p0 : p1;
}

// ------------------------------------------------------------------ DIS patches, four lanes per patch (round 3)
// k_patchw replicates the per-patch scalar work of an iteration (bilinear weights, the LLT solve's correctly
// rounded divisions, the stopping tests, the three DPP reductions) on all eight lanes of a patch: at p = 12
// gray that is ~40 % of the VALU instructions of an iteration.  Here four lanes share a patch (sixteen patches
// per wave), so the same per-patch work is spread over twice the values.  Lane s holds Eigen's packet slots s
// and s + 4 -- the values v = s + 8k and v + 4 of every 8-value block k -- as one register pair, so every
// per-value operation is packed fp32 on the pair (v, v + 4) INCLUDING the Eigen chains: the pair of slot
// accumulators (acc_s, acc_{s+4}) takes one v_pk_add_f32 per block, and res0 + res1 is the pair's own
// .x + .y; then (l0 + l2) + (l1 + l3) by two DPP butterflies inside the quad.  Same additions, same order:
// bit-identical to k_patchw (and to the oracle).  With p * noc a multiple of 4 every tap of lane s sits at
// s + (a compile-time offset) in the window tile, so a pair's taps are one ds_read2_b32 off a single base
// address.  Shapes: p * p * noc a multiple of 8 with the pairs' registers in budget (gray p = 8 / 12).
template <int P, int NOC>
struct QuadShape {
  static constexpr int NV = P * P * NOC;
  static constexpr int ROWV = P * NOC;
  static constexpr int K = NV / 8;           // 8-value blocks: lane s holds pair k = (s + 8k, s + 4 + 8k)
  static constexpr int WR = (P + 1) * NOC;   // window row (floats)
  static constexpr int Q4 = (WR + 3) / 4;    // 16-byte loads per window row
  // LDS row stride (floats): the row rounded up to an even count only (8-byte stores): at RS = Q4 * 4 the
  // 64 windows of a workgroup took 53 KB and three workgroups did not fit a CU (the quad form then ran at
  // two thirds of its register occupancy: no faster than the eight-lane form at p = 12)
  static constexpr int RS = (WR + 1) & ~1;
  // windows at a stride of 4 (mod 8) dwords: the 8 patches of a 32-lane half then start on 8 distinct 4-bank
  // groups, and their lanes' 4 consecutive dwords never share a bank
  static constexpr int WIN = (P + 1) * RS + ((4 - ((P + 1) * RS) % 8) + 8) % 8;
  static constexpr int NQ = (P + 1) * Q4;    // 16-byte loads per window
  static constexpr int LPL = (NQ + 3) / 4;   // ... per lane
  static_assert(NV % 8 == 0 && ROWV % 4 == 0, "quad form: p * noc a multiple of 4, p * p * noc of 8");
  // window offset (floats, lane s excluded) of the D tap of value 8k + h (h = 0 or 4)
  static constexpr int dtap(int k, int h) { return ((8 * k + h) / ROWV) * RS + (8 * k + h) % ROWV; }
  // frame offset (floats, lane s excluded) of value 8k + h relative to the patch's top-left pixel
  static constexpr int frow(int k, int h) { return (8 * k + h) / ROWV; }
  static constexpr int fcol(int k, int h) { return (8 * k + h) % ROWV; }
};

// Eigen's total of the quad's slot pairs: res0 + res1 (the pair), then (l0 + l2) + (l1 + l3).
__device__ __forceinline__ float quad_total(f2p acc) {
  float r = acc.x + acc.y;
  r = r + grp_xor2(r);
  return r + grp_xor1(r);
}
__device__ __forceinline__ float quad_max(float m) {
  m = fmaxf(m, grp_xor2(m));
  return fmaxf(m, grp_xor1(m));
}

template <int NOP, int P, int NOC, int MINW, int COST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MINW))) void k_patchq(PatchArgs a) {
  const uint3 xb = xcd_block();
  using S = QuadShape<P, NOC>;
  constexpr int K = S::K, RS = S::RS;
  extern __shared__ __attribute__((aligned(16))) float win_all[];
  const LevelGeom &g = a.g;
  const int s4 = threadIdx.x & 3;
  const long gp = (long)xb.x * 64 + (threadIdx.x >> 2);
  const bool live = gp < (long)a.n * g.npatch;
  const long gq = live ? gp : 0;
  const int f = (int)(gq / g.npatch), ip = (int)(gq % g.npatch);
  const int pxi = ip / g.noph, pyi = ip % g.noph;
  const float ptr0 = (float)(pxi * a.steps + g.offw), ptr1 = (float)(pyi * a.steps + g.offh);
  const long fs = (long)g.W * g.H * NOC;
  const int W = g.W;
  constexpr float inv_n = 1.0f / (float)S::NV;
  constexpr bool pow2 = (S::NV & (S::NV - 1)) == 0;
  auto div_n = [&](float x) {
    if constexpr (pow2)
      return x * inv_n;
    else
      return div_by_const<S::NV>(x);
  };
  float *win = win_all + (threadIdx.x >> 2) * S::WIN;
  // ---- template + gradients at the integer reference position (getPatchStaticNNGrad, patch.cpp:297-343)
  f2p tmp2[K], gx2[K], gy2[NOP == 2 ? K : 1];
  {
    const int px = (int)roundf(ptr0) + g.pad, py = (int)roundf(ptr1) + g.pad;
    const long base = ((long)(py - P / 2) * W + (px - P / 2)) * NOC + s4;
    const float *A = a.img_a + f * fs + base, *DX = a.dx_a + f * fs + base, *DY = a.dy_a + f * fs + base;
    const long rw = (long)W * NOC;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const long o0 = S::frow(k, 0) * rw + S::fcol(k, 0), o1 = S::frow(k, 4) * rw + S::fcol(k, 4);
      tmp2[k] = f2p{A[o0], A[o1]};
      gx2[k] = f2p{DX[o0], DX[o1]};
      if constexpr (NOP == 2) gy2[k] = f2p{DY[o0], DY[o1]};
    }
  }
  if (a.patnorm > 0) {
    f2p m = tmp2[0];
#pragma unroll
    for (int k = 1; k < K; ++k) m = m + tmp2[k];
    const float mean = div_n(quad_total(m));
#pragma unroll
    for (int k = 0; k < K; ++k) tmp2[k] = tmp2[k] - mean;
  }
  // ---- ComputeHessian (patch.cpp:69-86)
  float H00, H01 = 0.0f, H11 = 0.0f;
  {
    f2p h0 = gx2[0] * gx2[0], h1 = {0.0f, 0.0f}, h2 = {0.0f, 0.0f};
    if constexpr (NOP == 2) {
      h1 = gx2[0] * gy2[0];
      h2 = gy2[0] * gy2[0];
    }
#pragma unroll
    for (int k = 1; k < K; ++k) {
      h0 = h0 + gx2[k] * gx2[k];
      if constexpr (NOP == 2) {
        h1 = h1 + gx2[k] * gy2[k];
        h2 = h2 + gy2[k] * gy2[k];
      }
    }
    H00 = quad_total(h0);
    if (NOP == 2) {
      H01 = quad_total(h1);
      H11 = quad_total(h2);
      if (H00 * H11 - H01 * H01 == 0.0f) {
        H00 = (float)((double)H00 + 1e-10);
        H11 = (float)((double)H11 + 1e-10);
      }
    } else if (H00 == 0.0f) {
      H00 = (float)((double)H00 + 1e-10);
    }
  }
  const Llt2 fac = llt2_factor(H00, H01, H11);
  const float fac1 = llt1_factor(H00);
  const LltRcp lrc = llt_rcp<NOP>(fac, fac1, a.fdiv != 0);
  if (a.stage == 1) {  // timing diagnostic "pconst"
    if (live && s4 == 0) a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tmp2[K - 1].y;
    return;
  }
  // ---- initial parameters (InitializeFromCoarserOF, patchgrid.cpp:195-211)
  float pin0 = 0.0f, pin1 = 0.0f;
  if (a.prev) {
    const int x = (int)floorf(ptr0 / 2), y = (int)floorf(ptr1 / 2);
    const float *pv = a.prev + (long)f * a.prev_frame_stride + (long)(y * a.prev_w + x) * a.prev_elem_stride;
    pin0 = pv[0] * 2;
    if (NOP == 2) pin1 = pv[a.prev_comp_stride] * 2;
  }
  if (a.stage == 2) {  // "pconst + pinit"
    if (live && s4 == 0)
      a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tmp2[K - 1].y + pin0 + pin1;
    return;
  }
  const float *Bimg = a.img_b + f * fs;
  // ---- OptimizeStart (patch.cpp:117-154)
  float p0 = pin0, p1 = pin1, d0 = 0.0f, d1 = 0.0f;
  float pt0 = ptr0 + p0, pt1 = (NOP == 2) ? ptr1 + p1 : ptr1;
  const float st0 = pt0, st1 = pt1;
  float sq = (float)1e-10, sq_init = (float)1e-10, mares = (float)1e20, mares_old = (float)1e20;
  int cnt = 0;
  bool converged = false;
  float b0 = 0.0f, b1 = 0.0f;
  auto oob = [&](float x, float y) { return x < g.tmp_lb || y < g.tmp_lb || x > g.tmp_ubw || y > g.tmp_ubh; };
  int lpos0 = -0x7fffffff, lpos1 = 0;
  const unsigned wb = (unsigned)(uintptr_t)win + 4u * (unsigned)s4;  // lane s's taps: wb + 4 * (constant)
  // absw (gray: value v is pixel v): the aggregation weight of the value's pixel into the slot planes
  const int ptxi = (int)ptr0, ptyi = (int)ptr1;
  float *pl = a.absw ? a.pweight + agg_plane_off(f, a.aslots, pxi, pyi, g.w, g.h, ptxi - P / 2, ptyi - P / 2) : nullptr;
  auto put_agg = [&](int v, float wv) {
    const int lx = v % P, ly = v / P, x = ptxi - P / 2 + lx, y = ptyi - P / 2 + ly;
    if (x >= 0 && y >= 0 && x < g.w && y < g.h) pl[ly * g.w + lx] = 1.0f / stdmaxf(2.0f, wv);
  };
  // getPatchStaticBil + mean normalisation + LossComputeErrorImage (patch.cpp:221-413) at (pt0, pt1)
  // MAXR (maxres): r0 = the largest |w| instead of the sum -- see the iteration loop
  auto evaluate = [&](float &r0, float *out, auto store_t, auto maxr_t) {
    constexpr int STORE = decltype(store_t)::value;  // 0: the sums only; 1: the weights only, to `out`
    constexpr bool MAXR = decltype(maxr_t)::value;
    const int pos0 = (int)ceilf(pt0 + 0.00001f) + g.pad;
    const int pos1 = (int)ceilf(pt1 + 0.00001f) + g.pad;
    const int pos2 = (int)floorf(pt0), pos3 = (int)floorf(pt1);
    const float rx = pt0 - (float)pos2, ry = pt1 - (float)pos3;
    const float w0 = rx * ry, w1 = (1 - rx) * ry, w2 = rx * (1 - ry), w3 = (1 - rx) * (1 - ry);
    const float *Q = Bimg + ((long)(pos1 - P / 2 - 1) * W + (pos0 - P / 2 - 1)) * NOC;
    if (__builtin_amdgcn_ballot_w64(pos0 != lpos0 || pos1 != lpos1) != 0) {
      lpos0 = pos0;
      lpos1 = pos1;
      wave_lds_sync();
      bool done = false;
      if constexpr (S::Q4 == 4 && S::LPL == P + 1) {
        if (a.buf32) {
          // window row j is one 16-byte load per lane (column 4 s4) at a wave-uniform row offset: buffer loads off
          // the image array with the lane's 32-bit byte offset and the row in the scalar offset, no per-load
          // address arithmetic.  Stores: row j's floats j RS + 4 s4 .. + 3; lane 3's last two (past the RS = 14
          // columns) land on row j + 1's first two, which lane 0 rewrites with row j + 1 right after (one wave's LDS
          // stores are performed in order; the empty asm keeps the compiler's), the last row's in the padding.
          const __amdgpu_buffer_rsrc_t rsrc =
              __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.img_b), (short)0, (int)0xffffffff, 0x00020000);
          const unsigned vo = ((unsigned)(f * fs) + (unsigned)(((pos1 - P / 2 - 1) * W + (pos0 - P / 2 - 1)) * NOC) +
                               4u * (unsigned)s4) * 4u;
          float4_v t[P + 1];
#pragma unroll
          for (int j = 0; j <= P; ++j)
            t[j] = __builtin_bit_cast(float4_v, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo, j * W * NOC * 4, 0));
          f2p *d = reinterpret_cast<f2p *>(win + 4 * s4);
#pragma unroll
          for (int j = 0; j <= P; ++j) {
            d[j * (RS / 2)] = f2p{t[j].x, t[j].y};
            d[j * (RS / 2) + 1] = f2p{t[j].z, t[j].w};
            asm volatile("" ::: "memory");
          }
          done = true;
        }
      }
      // every load of the tile in flight at once: one round trip to L2 per reload (the 8-lane kernel's count)
      constexpr int NB = S::LPL;
#pragma unroll
      for (int j0 = 0; j0 < (done ? 0 : S::LPL); j0 += NB) {
        float4_u t[NB];
        int lo[NB];
#pragma unroll
        for (int j = j0; j < j0 + NB && j < S::LPL; ++j) {
          const int e = s4 + 4 * j, e2 = e < S::NQ ? e : S::NQ - 1;
          const int row = e2 / S::Q4, c4 = e2 % S::Q4;
          lo[j - j0] = row * RS + c4 * 4;
          t[j - j0] = *reinterpret_cast<const float4_u *>(Q + row * W * NOC + c4 * 4);
        }
#pragma unroll
        for (int j = j0; j < j0 + NB && j < S::LPL; ++j) {  // two 8-byte stores: columns < RS only
          const int e = s4 + 4 * j;
          if (e < S::NQ) {
            f2p *d = reinterpret_cast<f2p *>(win + lo[j - j0]);
            d[0] = f2p{t[j - j0].x, t[j - j0].y};
            if (4 * (e % S::Q4) + 2 < RS) d[1] = f2p{t[j - j0].z, t[j - j0].w};
          }
        }
      }
      wave_lds_sync();
    }
    // taps of pair k: one ds_read2_b32 per tap (D, C, B, A), the next pair's reads in flight
    f2p pd2[K], q[2][4];
    auto issue = [&](auto kc) {
      constexpr int k = decltype(kc)::value, c0 = S::dtap(k, 0), c1 = S::dtap(k, 4);
      constexpr int mx = (c0 > c1 ? c0 : c1) + RS + NOC;
      constexpr int b = mx <= 255 ? 0 : (c0 < c1 ? c0 : c1);  // else part of the offset goes into the address
      const unsigned ad = wb + 4u * (unsigned)b;
      q[k & 1][0] = lds_read2<c0 - b, c1 - b>(ad);                        // D
      q[k & 1][1] = lds_read2<c0 - b + NOC, c1 - b + NOC>(ad);            // C
      q[k & 1][2] = lds_read2<c0 - b + RS, c1 - b + RS>(ad);              // B
      q[k & 1][3] = lds_read2<c0 - b + RS + NOC, c1 - b + RS + NOC>(ad);  // A
    };
    issue(std::integral_constant<int, 0>{});
    f2p macc;
    static_for<K>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if constexpr (k + 1 < K) {
        issue(std::integral_constant<int, k + 1>{});
        lds_wait<4>();
      } else {
        lds_wait<0>();
      }
      f2p *t = q[k & 1];
      static_for<4>([&](auto ic) { reg_fence(t[decltype(ic)::value]); });
      f2p x = t[3] * w0 + t[2] * w1;
      x = x + t[1] * w2;
      x = x + t[0] * w3;
      pd2[k] = x;
      if constexpr (k == 0) macc = x;
      else macc = macc + x;
    });
    const float mean = a.patnorm > 0 ? div_n(quad_total(macc)) : 0.0f;
    float abl = 0.0f, abh = 0.0f;
    f2p ex, ey;
    static_for<K>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const f2p d = (pd2[k] - mean) - tmp2[k];
      f2p wv, e;
      if (COST == 0) {
        wv = d;
        e = d;
      } else {
        float w[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float dh = h ? d.y : d.x;
          w[h] = COST == 1 ? sqrt_nonneg(fabsf(dh))
                           : sqrt_nonneg((sqrt_nonneg(1.0f + (dh * dh) / 25.0f) - 1.0f) * 50.0f);
        }
        wv = f2p{w[0], w[1]};
        e = f2p{copysignf(w[0], d.x), copysignf(w[1], d.y)};
      }
      if constexpr (STORE == 0) {
        const f2p qx = gx2[k] * e;
        f2p qy;
        if constexpr (NOP == 2) qy = gy2[k] * e;
        if constexpr (k == 0) {
          if constexpr (MAXR) {
            abl = fmaxf(fabsf(wv.x), fabsf(wv.y));
          } else {
            abl = fabsf(wv.x);
            abh = fabsf(wv.y);
          }
          ex = qx;
          if (NOP == 2) ey = qy;
        } else {
          if constexpr (MAXR) {
            abl = fmaxf(abl, fmaxf(fabsf(wv.x), fabsf(wv.y)));  // one v_max3_f32 with |.| modifiers per pair
            asm volatile("" : "+v"(abl));  // (else the compiler pairs the pairs: v_max + half a v_max3 per pair)
          } else {
            abl = abl + fabsf(wv.x);
            abh = abh + fabsf(wv.y);
            // two scalar adds with |.| source modifiers; left to itself the compiler packs this chain pair
            // (v_pk_add_f32 after two v_and_b32: three instructions instead of two)
            asm volatile("" : "+v"(abl), "+v"(abh));
          }
          ex = ex + qx;
          if (NOP == 2) ey = ey + qy;
        }
      } else {
        const float wl = COST == 0 ? fabsf(wv.x) : wv.x, wh = COST == 0 ? fabsf(wv.y) : wv.y;
        if (a.absw) {
          put_agg(s4 + 8 * k, wl);
          put_agg(s4 + 4 + 8 * k, wh);
        } else {
          out[s4 + 8 * k] = wl;
          out[s4 + 4 + 8 * k] = wh;
        }
      }
    });
    if constexpr (STORE == 0) {
      if constexpr (MAXR)
        r0 = quad_max(abl);
      else
        r0 = quad_total(f2p{abl, abh});
      b0 = quad_total(ex);
      if (NOP == 2) b1 = quad_total(ey);
    }
  };
  float *pwo = a.pweight + gq * S::NV;
  bool start_oob = false, first = true;
  converged = !live;
  if (live && oob(pt0, pt1)) {  // converged at once; pweight never written upstream, defined as 0
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (a.absw) {
        put_agg(s4 + 8 * k, 0.0f);
        put_agg(s4 + 4 + 8 * k, 0.0f);
      } else {
        pwo[s4 + 8 * k] = 0.0f;
        pwo[s4 + 4 + 8 * k] = 0.0f;
      }
    }
    converged = true;
    start_oob = true;
  } else {
    mares = 1e5f;
  }
  for (;;) {
    if (__builtin_amdgcn_ballot_w64(!converged) == 0) break;
    if (!converged) {
      if (!first) {
        ++cnt;
        if (NOP == 2) {
          llt2_solve_fast(fac, lrc, b0, b1, d0, d1);
          p0 = p0 - d0;
          p1 = p1 - d1;
        } else {
          d0 = llt1_solve_fast(fac1, lrc, b0);
          p0 = p0 - d0;
          p0 = (a.camlr == 0) ? stdminf(p0, 0.0f) : stdmaxf(p0, 0.0f);
        }
        pt0 = ptr0 + p0;
        if (NOP == 2) pt1 = ptr1 + p1;
        const float ex = st0 - pt0, ey = st1 - pt1;
        if (ex * ex + ey * ey > a.outlier_sq || oob(pt0, pt1)) {
          p0 = pin0;
          p1 = pin1;
          pt0 = ptr0 + p0;
          if (NOP == 2) pt1 = ptr1 + p1;
          converged = true;
        }
      }
      float r0 = 0.0f;
      // OptimizeComputeErrImg (patch.cpp:275-295).  maxres (res_thresh = 0, min_iter >= max_iter: every
      // op-point): mares only meets the test mares > 0, and the rate tests only iterations that stop anyway; a sum
      // of |w| >= 0 is positive iff its largest term is, and RN(sum / N) > 0 then too while that term is >= 2^-100.
      // So the evaluation keeps the largest |w| (one v_max3 per value pair instead of two adds, no division);
      // a wave with a NaN (b0 / b1 are NaN iff some residual is) or a term in (0, 2^-100) redoes it with the sum.
      // (shapes whose value count is a power of two divide by a multiplication: there the two adds per pair it
      // saves do not pay for the second evaluation copy's registers -- p = 8 spilled 11 VGPRs with it)
      bool summed = true;
      if (!pow2 && a.maxres) {
        evaluate(r0, nullptr, std::integral_constant<int, 0>(), std::true_type());
        summed = false;
        const bool odd = (r0 > 0.0f && r0 < 0x1p-100f) || b0 != b0 || (NOP == 2 && b1 != b1);
        if (__builtin_amdgcn_ballot_w64(odd) != 0) {
          evaluate(r0, nullptr, std::integral_constant<int, 0>(), std::false_type());
          summed = true;
        }
      } else {
        evaluate(r0, nullptr, std::integral_constant<int, 0>(), std::false_type());
      }
      sq = (NOP == 2) ? d0 * d0 + d1 * d1 : d0 * d0;
      if (cnt == 1) sq_init = sq;
      mares_old = mares;
      mares = summed ? div_n(r0) : r0;
      bool rates = true;
      if (__builtin_amdgcn_ballot_w64(cnt >= a.min_iter) != 0)
        rates = (cnt < a.min_iter) | ((sq / sq_init >= a.dp_thresh_sq) & (mares / mares_old <= a.dr_thresh));
      const bool keep = (cnt < a.max_iter) & (summed ? mares > a.res_thresh : r0 > 0.0f) & rates;
      if (!keep) converged = true;
    }
    first = false;
  }
  if (live && !start_oob) {
    float r0;
    evaluate(r0, pwo, std::integral_constant<int, 1>(), std::false_type());
  }
  if (live && s4 < NOP) a.p_iter[gp * NOP + s4] = s4 == 0 ? p0 : p1;
}

// ------------------------------------------------------------------ DIS patches, sixteen lanes per patch (round 4)
// The big RGB shape (p = 12, 432 values) holds 54 values per lane on eight lanes: template + two gradients alone
// are 162 VGPRs, so k_patchw spills at two waves per SIMD and reads every tap twice (LEAN).  Here sixteen lanes
// share a patch (four patches per wave): lane s holds the values s + 16 m (m = 0 .. NV/16 - 1), which are Eigen
// packet slot j = s & 7 of the 8-value blocks k = 2 m + (s >> 3).  Everything per value -- taps, bilinear sample,
// loss, products -- runs on all sixteen lanes, the samples stay in registers; Eigen's eight slot chains stay
// sequential in block order on the owner lanes s < 8: block 2m is the owner's own value, block 2m + 1 its
// partner's (lane s + 8, moved by DPP row_ror:8), added in that order.  The same additions in the same order as
// k_patchw / k_patch8, so the same bits; the lanes s >= 8 get the totals from their owners by one DPP move.
template <int P, int NOC>
struct XShape {
  static constexpr int NV = P * P * NOC;
  static constexpr int M = NV / 16;         // values per lane
  static constexpr int ROWV = P * NOC;      // values per patch row
  static constexpr int WR = (P + 1) * NOC;  // window row (floats)
  static constexpr int Q4 = (WR + 3) / 4;   // 16-byte loads per window row
  static constexpr int RS = Q4 * 4;         // LDS row stride (floats)
  // windows 16 (mod 32) dwords apart: the two patches of a 32-lane half read disjoint bank halves
  static constexpr int WIN = (P + 1) * RS + (16 - ((P + 1) * RS) % 32 + 32) % 32;
  static constexpr int NQ = (P + 1) * Q4;   // 16-byte loads per window
  static constexpr int LPL = (NQ + 15) / 16;
  static constexpr int gcd(int a, int b) { return b == 0 ? a : gcd(b, a % b); }
  // value m -> m + KP of a lane advances its taps by KROWS whole patch rows
  static constexpr int KP = (16 / gcd(16, ROWV) * ROWV) / 16;
  static constexpr int KROWS = 16 * KP / ROWV;
  // value groups of KP: pairs of groups (2g, 2g + 1) run packed, an odd last group alone
  static constexpr int NPG = M / KP / 2, NPP = NPG * KP, NS = M - 2 * NPP;
  static_assert(NV % 16 == 0, "sixteen-lane form: p * p * noc a multiple of 16");
  // LDS floats of a workgroup: sixteen windows, then the gradients of the odd group's values (NOP per value and
  // lane; in LDS they free registers the compiler otherwise spills to scratch and reloads every iteration)
  static constexpr int lds_floats(int nop) { return 16 * WIN + NS * 256 * nop; }
};

// Eigen's chain of one packet slot, folded on the owner lanes in block order (see above).
struct XAcc {
  float acc = 0.0f;
  // values of blocks 2m (own) and 2m + 1 (partner), in two steps: callers with several chains issue every chain's
  // own() before the partner() adds, so no DPP add reads an accumulator written by the instruction just before
  // it (a DPP source VGPR needs two wait states after its VALU write)
  __device__ __forceinline__ void own(int m, float x) { acc = m == 0 ? x : acc + x; }
  __device__ __forceinline__ void partner(float x) {
    acc = acc + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x128, 0xF, 0xF, true));
  }
  __device__ __forceinline__ void add(int m, float x) {
    own(m, x);
    partner(x);
  }
  // res0 + res1, (l0 + l2) + (l1 + l3) on the owners, then the owners' totals to lanes 8 .. 15
  __device__ __forceinline__ float total() const {
    float r = acc + grp_xor4(acc);
    r = r + grp_xor2(r);
    r = r + grp_xor1(r);
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, r), __builtin_bit_cast(int, r),
                                                                 0x128, 0xF, 0xC, false));
  }
};

template <int NOP, int P, int NOC, int MINW, int COST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MINW))) void k_patchx(PatchArgs a) {
  const uint3 xb = xcd_block();
  using S = XShape<P, NOC>;
  constexpr int M = S::M, RS = S::RS, KP = S::KP;
  constexpr int NPG = S::NPG, NPP = S::NPP, NS = S::NS;
  static_assert(M % KP == 0 && NS <= KP, "sixteen-lane form: whole value groups");
  extern __shared__ __attribute__((aligned(16))) float win_all[];
  const LevelGeom &g = a.g;
  const int s16 = threadIdx.x & 15;
  const long gp = (long)xb.x * 16 + (threadIdx.x >> 4);
  const bool live = gp < (long)a.n * g.npatch;
  const long gq = live ? gp : 0;
  const int f = (int)(gq / g.npatch), ip = (int)(gq % g.npatch);
  const int pxi = ip / g.noph, pyi = ip % g.noph;
  const float ptr0 = (float)(pxi * a.steps + g.offw), ptr1 = (float)(pyi * a.steps + g.offh);
  const long fs = (long)g.W * g.H * NOC;
  const int W = g.W;
  constexpr float inv_n = 1.0f / (float)S::NV;
  constexpr bool pow2 = (S::NV & (S::NV - 1)) == 0;
  auto div_n = [&](float x) {
    if constexpr (pow2)
      return x * inv_n;
    else
      return div_by_const<S::NV>(x);
  };
  float *win = win_all + (threadIdx.x >> 4) * S::WIN;
  // window offset of the D tap of value m: dbase[m mod KP] + (m / KP) KROWS RS
  auto dtap = [&](int v) { return (v / S::ROWV) * RS + v % S::ROWV; };
  int dbase[KP < M ? KP : M];
#pragma unroll
  for (int i = 0; i < (KP < M ? KP : M); ++i) dbase[i] = dtap(s16 + 16 * i);
  // ---- template + gradients at the integer reference position (getPatchStaticNNGrad, patch.cpp:297-343)
  float tmp[M], gx[M], gy[NOP == 2 ? M : 1];
  {
    const int px = (int)roundf(ptr0) + g.pad, py = (int)roundf(ptr1) + g.pad;
    const long base = ((long)(py - P / 2) * W + (px - P / 2)) * NOC;
    const float *A = a.img_a + f * fs + base, *DX = a.dx_a + f * fs + base, *DY = a.dy_a + f * fs + base;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int v = s16 + 16 * m;
      const int o = (v / S::ROWV) * W * NOC + v % S::ROWV;
      tmp[m] = A[o];
      gx[m] = DX[o];
      if constexpr (NOP == 2) gy[m] = DY[o];
    }
  }
  if (a.patnorm > 0) {
    XAcc mc;
#pragma unroll
    for (int m = 0; m < M; ++m) mc.add(m, tmp[m]);
    const float mean = div_n(mc.total());
#pragma unroll
    for (int m = 0; m < M; ++m) tmp[m] = tmp[m] - mean;
  }
  // ---- ComputeHessian (patch.cpp:69-86)
  float H00, H01 = 0.0f, H11 = 0.0f;
  {
    XAcc h0, h1, h2;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float a0 = gx[m] * gx[m], a1 = NOP == 2 ? gx[m] * gy[m] : 0.0f, a2 = NOP == 2 ? gy[m] * gy[m] : 0.0f;
      h0.own(m, a0);
      if constexpr (NOP == 2) {
        h1.own(m, a1);
        h2.own(m, a2);
      }
      h0.partner(a0);
      if constexpr (NOP == 2) {
        h1.partner(a1);
        h2.partner(a2);
      }
    }
    H00 = h0.total();
    if (NOP == 2) {
      H01 = h1.total();
      H11 = h2.total();
      if (H00 * H11 - H01 * H01 == 0.0f) {
        H00 = (float)((double)H00 + 1e-10);
        H11 = (float)((double)H11 + 1e-10);
      }
    } else if (H00 == 0.0f) {
      H00 = (float)((double)H00 + 1e-10);
    }
  }
  const Llt2 fac = llt2_factor(H00, H01, H11);
  const float fac1 = llt1_factor(H00);
  const LltRcp lrc = llt_rcp<NOP>(fac, fac1, a.fdiv != 0);
  if (a.stage == 1) {  // timing diagnostic "pconst"
    if (live && s16 == 0) a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tmp[M - 1];
    return;
  }
  // ---- initial parameters (InitializeFromCoarserOF, patchgrid.cpp:195-211)
  float pin0 = 0.0f, pin1 = 0.0f;
  if (a.prev) {
    const int x = (int)floorf(ptr0 / 2), y = (int)floorf(ptr1 / 2);
    const float *pv = a.prev + (long)f * a.prev_frame_stride + (long)(y * a.prev_w + x) * a.prev_elem_stride;
    pin0 = pv[0] * 2;
    if (NOP == 2) pin1 = pv[a.prev_comp_stride] * 2;
  }
  if (a.stage == 2) {  // "pconst + pinit"
    if (live && s16 == 0) a.p_iter[gp * NOP] = fac.L00 + fac.L10 + fac.L11 + fac1 + tmp[M - 1] + pin0 + pin1;
    return;
  }
  // the scaled FAST evaluation's condition (see evaluate): every nonzero gradient of the wave's patches >= 2^-51
  bool gsmall = false;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    gsmall |= gx[m] != 0.0f && fabsf(gx[m]) < 0x1p-51f;
    if constexpr (NOP == 2) gsmall |= gy[m] != 0.0f && fabsf(gy[m]) < 0x1p-51f;
  }
  const bool xok = __builtin_amdgcn_ballot_w64(gsmall) == 0;
  // template and gradients as value pairs (m, m + KP) of the pair groups, and the values of an odd last group
  // (optical flow: the gradients as (gx, gy) pairs of one value -- ga value m, gb value m + KP -- so a value's two
  // products are one v_pk_mul_f32 and its two chains' own adds one v_pk_add_f32)
  f2p tmp2[NPP > 0 ? NPP : 1], gx2[NOP == 1 && NPP > 0 ? NPP : 1];
  f2p ga[NOP == 2 && NPP > 0 ? NPP : 1], gb[NOP == 2 && NPP > 0 ? NPP : 1];
  float tmps[NS > 0 ? NS : 1];
  // the odd group's gradients: LDS float NOP (i 256 + tid) (+1), written and read by the lane itself only
  float *gsl = win_all + 16 * S::WIN + NOP * threadIdx.x;
#pragma unroll
  for (int j = 0; j < NPP; ++j) {
    const int m = (j / KP) * 2 * KP + j % KP;
    tmp2[j] = f2p{tmp[m], tmp[m + KP]};
    if constexpr (NOP == 2) {
      ga[j] = f2p{gx[m], gy[m]};
      gb[j] = f2p{gx[m + KP], gy[m + KP]};
    } else {
      gx2[j] = f2p{gx[m], gx[m + KP]};
    }
  }
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    tmps[i] = tmp[2 * NPP + i];
    if constexpr (NOP == 2)
      *reinterpret_cast<f2p *>(gsl + 2 * 256 * i) = f2p{gx[2 * NPP + i], gy[2 * NPP + i]};
    else
      gsl[256 * i] = gx[2 * NPP + i];
  }
  const float *Bimg = a.img_b + f * fs;
  // ---- OptimizeStart (patch.cpp:117-154)
  float p0 = pin0, p1 = pin1, d0 = 0.0f, d1 = 0.0f;
  float pt0 = ptr0 + p0, pt1 = (NOP == 2) ? ptr1 + p1 : ptr1;
  const float st0 = pt0, st1 = pt1;
  float sq = (float)1e-10, sq_init = (float)1e-10, mares = (float)1e20, mares_old = (float)1e20;
  int cnt = 0;
  bool converged = false;
  float b0 = 0.0f, b1 = 0.0f;
  auto oob = [&](float x, float y) { return x < g.tmp_lb || y < g.tmp_lb || x > g.tmp_ubw || y > g.tmp_ubh; };
  int lpos0 = -0x7fffffff, lpos1 = 0;
  const unsigned wb = (unsigned)(uintptr_t)win;
  // getPatchStaticBil + mean normalisation + LossComputeErrorImage (patch.cpp:221-413) at (pt0, pt1)
  // FAST: the loss square roots by sqrt_nonneg_s64 (exact below 2^64; a sum that comes out non-finite makes the
  // caller redo the evaluation with sqrt_nonneg)
  // MAXR (maxres, with FAST only): r0 = the largest w instead of the sum -- see the iteration loop
  auto evaluate = [&](float &r0, float *out, auto store_t, auto fast_t, auto maxr_t) {
    constexpr int STORE = decltype(store_t)::value;  // 0: the sums only; 1: the weights only, to `out`
    constexpr bool FAST = decltype(fast_t)::value;
    constexpr bool MAXR = decltype(maxr_t)::value;
    const int pos0 = (int)ceilf(pt0 + 0.00001f) + g.pad;
    const int pos1 = (int)ceilf(pt1 + 0.00001f) + g.pad;
    const int pos2 = (int)floorf(pt0), pos3 = (int)floorf(pt1);
    const float rx = pt0 - (float)pos2, ry = pt1 - (float)pos3;
    const float w0 = rx * ry, w1 = (1 - rx) * ry, w2 = rx * (1 - ry), w3 = (1 - rx) * (1 - ry);
    const float *Q = Bimg + ((long)(pos1 - P / 2 - 1) * W + (pos0 - P / 2 - 1)) * NOC;
    if (__builtin_amdgcn_ballot_w64(pos0 != lpos0 || pos1 != lpos1) != 0) {
      lpos0 = pos0;
      lpos1 = pos1;
      wave_lds_sync();
      // the load offsets are recomputed here (an opaque copy of the lane index): hoisted out of the iteration
      // loop they are 27 more live registers for the whole loop.  Load e of the window is 16-byte column e mod Q4
      // of window row e / Q4; in LDS (row stride RS = 4 Q4) it lands at float 4 e.
      int sl = s16;
      asm volatile("" : "+v"(sl));
      sl &= 15;
      const int gstride = W * NOC - RS;
      float4_u t[S::LPL];
#pragma unroll
      for (int j = 0; j < S::LPL; ++j) {
        const int e = sl + 16 * j, e2 = e < S::NQ ? e : S::NQ - 1;
        t[j] = *reinterpret_cast<const float4_u *>(Q + ((e2 / S::Q4) * gstride + 4 * e2));
      }
#pragma unroll
      for (int j = 0; j < S::LPL; ++j) {
        const int e = sl + 16 * j;
        if (e < S::NQ) *reinterpret_cast<float4_v *>(win + 4 * e) = t[j];
      }
      wave_lds_sync();
    }
    // taps: value pairs (m, m + KP) -- their taps are KROWS patch rows apart whatever the lane, so each tap of a
    // pair is one ds_read2_b32 into a register pair and the bilinear sample runs packed; the values of a last
    // odd group of KP alone, (D, C) and (B, A) per ds_read2_b32.  The next unit's reads are in flight while a
    // unit is computed.
    constexpr int PD = S::KROWS * RS;
    f2p pd2[NPP > 0 ? NPP : 1];
    float pds[NS > 0 ? NS : 1];
    f2p q[2][4];
    auto issue = [&](auto uc) {  // unit u: pairs 0 .. NPP - 1, then singles
      constexpr int u = decltype(uc)::value;
      if constexpr (u < NPP) {
        constexpr int i = u % KP, o0 = 2 * (u / KP) * PD;
        constexpr bool imm = o0 + RS + NOC + PD <= 255;
        constexpr int o = imm ? o0 : 0;
        const unsigned b = wb + 4u * (unsigned)dbase[i] + (imm ? 0u : 4u * (unsigned)o0);
        q[u & 1][0] = lds_read2<o, o + PD>(b);                        // D
        q[u & 1][1] = lds_read2<o + NOC, o + NOC + PD>(b);            // C
        q[u & 1][2] = lds_read2<o + RS, o + RS + PD>(b);              // B
        q[u & 1][3] = lds_read2<o + RS + NOC, o + RS + NOC + PD>(b);  // A
      } else {
        constexpr int i = u - NPP, o0 = (2 * NPP / KP) * PD;
        constexpr bool imm = o0 + RS + NOC <= 255;
        constexpr int o = imm ? o0 : 0;
        const unsigned b = wb + 4u * (unsigned)dbase[i] + (imm ? 0u : 4u * (unsigned)o0);
        q[u & 1][0] = lds_read2<o, o + NOC>(b);            // D, C
        q[u & 1][1] = lds_read2<o + RS, o + RS + NOC>(b);  // B, A
      }
    };
    const f2p w32 = f2p{w3, w2}, w10 = f2p{w1, w0};
    issue(std::integral_constant<int, 0>{});
    static_for<NPP + NS>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if constexpr (u + 1 < NPP + NS) {
        issue(std::integral_constant<int, u + 1>{});
        lds_wait<(u + 1 < NPP ? 4 : 2)>();
      } else {
        lds_wait<0>();
      }
      f2p *t = q[u & 1];
      if constexpr (u < NPP) {
        static_for<4>([&](auto ic) { reg_fence(t[decltype(ic)::value]); });
        f2p x = t[3] * w0 + t[2] * w1;
        x = x + t[1] * w2;
        x = x + t[0] * w3;
        pd2[u] = x;
      } else {
        reg_fence(t[0]);
        reg_fence(t[1]);
        // the tap pairs (D, C), (B, A) as they come: two packed products, then the sum in the reference's order
        const f2p dc = t[0] * w32, ba = t[1] * w10;  // (w3 D, w2 C), (w1 B, w0 A)
        pds[u - NPP] = ((ba.y + ba.x) + dc.y) + dc.x;
      }
    });
    auto pdv = [&](int m) -> float {  // compile-time m: the sample of value m
      const int gi = m / KP, i = m % KP;
      if (gi < 2 * NPG) return gi % 2 == 0 ? pd2[(gi / 2) * KP + i].x : pd2[(gi / 2) * KP + i].y;
      return pds[i];
    };
    float mean = 0.0f;
    if (a.patnorm > 0) {
      XAcc mc;
      static_for<M>([&](auto mc_) {
        constexpr int m = decltype(mc_)::value;
        mc.add(m, pdv(m));
      });
      mean = div_n(mc.total());
    }
    // loss of one value: w (weight) and e (signed residual)
    // FAST (COST > 0): w and e at the 2^32 scale (the last square root's exact rescaling moves to the totals, one
    // multiplication per evaluation instead of per value); the products with the gradients and every partial sum
    // then round exactly as at scale 1 -- no product is subnormal at scale 1 (xok: nonzero gradients >= 2^-51,
    // nonzero w >= 2^-75) and a sum's subnormal result is exact -- so the rescaled totals carry the same bits
    auto loss = [&](float d, float &w, float &e) {
      if (COST == 0) {
        e = d;
        w = fabsf(d);
      } else {
        auto sq = [](float x) { return FAST ? sqrt_nonneg_s64(x) : sqrt_nonneg(x); };
        auto sqo = [](float x) { return FAST ? sqrt_nonneg_s64_x32(x) : sqrt_nonneg(x); };
        w = COST == 1 ? sqo(fabsf(d)) : sqo((sq(1.0f + (d * d) / 25.0f) - 1.0f) * 50.0f);
        e = copysignf(w, d);
      }
    };
    XAcc ab, ex;
    float abm = 0.0f;           // MAXR: the lane's largest w
    f2p exy = f2p{0.0f, 0.0f};  // optical flow: the x and y chains side by side (own adds packed)
    // pair groups: d of both halves packed; the .x halves (values m) go into the chains at once, the .y halves'
    // d (values m + KP) are kept until their turn, after the group's KP .x values
    // chain adds run one value behind the products: a DPP source written by the instruction just before needs wait
    // states (s_nop), the previous value's products were written long before
    float pw = 0.0f, pqx = 0.0f;
    f2p pq = f2p{0.0f, 0.0f};
    auto dppf = [](float x) {
      return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x128, 0xF, 0xF, true));
    };
    auto flush = [&](int m) {  // compile-time m: value m's terms into the chains
      if constexpr (MAXR)
        abm = m == 0 ? pw : fmaxf(abm, pw);
      else
        ab.own(m, pw);  // w >= +0 for every cost (|d| or a square root): |w| == w
      if constexpr (NOP == 2) {
        exy = m == 0 ? pq : exy + pq;  // the x and y chains' own values (XAcc::own, two chains at once)
      } else {
        ex.own(m, pqx);
      }
      if constexpr (!MAXR) ab.partner(pw);
      if constexpr (NOP == 2) {  // XAcc::partner per chain
        exy.x = exy.x + dppf(pq.x);
        exy.y = exy.y + dppf(pq.y);
      } else {
        ex.partner(pqx);
      }
    };
    // g: the value's (gx, gy) (depth: gx in .x)
    auto value_out = [&](int m, float d, f2p g) {  // compile-time m, in increasing order
      float w, e;
      loss(d, w, e);
      if constexpr (STORE == 0) {
        if (m > 0) flush(m - 1);
        pw = w;
        if constexpr (NOP == 2)
          pq = g * f2p{e, e};
        else
          pqx = g.x * e;
      } else {
        out[s16 + 16 * m] = w;
      }
    };
    static_for<NPG>([&](auto gc) {
      constexpr int gg = decltype(gc)::value;
      float dy[KP];
      static_for<KP>([&](auto ic) {
        constexpr int i = decltype(ic)::value, j = gg * KP + i;
        const f2p d = (pd2[j] - mean) - tmp2[j];
        dy[i] = d.y;
        if constexpr (NOP == 2)
          value_out(2 * gg * KP + i, d.x, ga[j]);
        else
          value_out(2 * gg * KP + i, d.x, f2p{gx2[j].x, 0.0f});
      });
      static_for<KP>([&](auto ic) {
        constexpr int i = decltype(ic)::value, j = gg * KP + i;
        if constexpr (NOP == 2)
          value_out(2 * gg * KP + KP + i, dy[i], gb[j]);
        else
          value_out(2 * gg * KP + KP + i, dy[i], f2p{gx2[j].y, 0.0f});
      });
    });
    static_for<NS>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (NOP == 2) {
        const f2p gr = *reinterpret_cast<const f2p *>(gsl + 2 * 256 * i);
        value_out(2 * NPP + i, (pds[i] - mean) - tmps[i], gr);
      } else {
        value_out(2 * NPP + i, (pds[i] - mean) - tmps[i], f2p{gsl[256 * i], 0.0f});
      }
    });
    if (STORE == 0) {
      flush(M - 1);
      constexpr float sc = (FAST && COST != 0) ? 0x1p-32f : 1.0f;
      if constexpr (MAXR) {
        float mx = fmaxf(abm, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, abm), 0x128,
                                                                                0xF, 0xF, true)));
        mx = fmaxf(mx, grp_xor4(mx));
        mx = fmaxf(mx, grp_xor2(mx));
        mx = fmaxf(mx, grp_xor1(mx));
        // at scale 1; a positive maximum that the rescaling would take below 2^-100 stays positive and small
        // (the caller's fallback range)
        r0 = mx > 0.0f ? fmaxf(mx * sc, 0x1p-120f) : mx;
      } else {
        r0 = ab.total() * sc;
      }
      if constexpr (NOP == 2) {
        XAcc tx, ty;
        tx.acc = exy.x;
        ty.acc = exy.y;
        b0 = tx.total() * sc;
        b1 = ty.total() * sc;
      } else {
        b0 = ex.total() * sc;
      }
    }
  };
  // absw: the patch's aggregation weights into the slot planes (agg_plane_off) instead of its loss weights
  float *pwo = a.pweight + gq * S::NV;
  bool start_oob = false, first = true;
  converged = !live;
  if (live && oob(pt0, pt1)) {  // converged at once; pweight never written upstream, defined as 0
    if (!a.absw) {
#pragma unroll
      for (int m = 0; m < M; ++m) pwo[s16 + 16 * m] = 0.0f;
    }
    converged = true;
    start_oob = true;
  } else {
    mares = 1e5f;
  }
  for (;;) {
    if (__builtin_amdgcn_ballot_w64(!converged) == 0) break;
    if (!converged) {
      if (!first) {
        ++cnt;
        if (NOP == 2) {
          llt2_solve_fast(fac, lrc, b0, b1, d0, d1);
          p0 = p0 - d0;
          p1 = p1 - d1;
        } else {
          d0 = llt1_solve_fast(fac1, lrc, b0);
          p0 = p0 - d0;
          p0 = (a.camlr == 0) ? stdminf(p0, 0.0f) : stdmaxf(p0, 0.0f);
        }
        pt0 = ptr0 + p0;
        if (NOP == 2) pt1 = ptr1 + p1;
        const float ex = st0 - pt0, ey = st1 - pt1;
        if (ex * ex + ey * ey > a.outlier_sq || oob(pt0, pt1)) {
          p0 = pin0;
          p1 = pin1;
          pt0 = ptr0 + p0;
          if (NOP == 2) pt1 = ptr1 + p1;
          converged = true;
        }
      }
      float r0 = 0.0f;
      // maxres (res_thresh = 0, min_iter >= max_iter: every op-point) -- mares only meets mares > 0 (see
      // k_patchq): the FAST evaluation keeps the largest w, and a wave with a non-finite b0 / b1 (NaN iff some
      // residual is) or a term in (0, 2^-100) redoes the iteration's evaluation exactly, with the sum.  Without
      // maxres every evaluation is the exact one.
      constexpr float fmx = 3.402823466e38f;
      bool exact = !a.maxres || (COST != 0 && (!xok || a.x16 == 2));
      bool summed = true;
      if (!exact) {
        evaluate(r0, nullptr, std::integral_constant<int, 0>(), std::true_type(), std::true_type());
        summed = false;
        const bool odd = (r0 > 0.0f && r0 < 0x1p-100f) || !(fabsf(b0) <= fmx) || (NOP == 2 && !(fabsf(b1) <= fmx));
        exact = __builtin_amdgcn_ballot_w64(odd) != 0;
      }
      if (exact) {
        evaluate(r0, nullptr, std::integral_constant<int, 0>(), std::false_type(), std::false_type());
        summed = true;
      }
      // OptimizeComputeErrImg (patch.cpp:275-295)
      sq = (NOP == 2) ? d0 * d0 + d1 * d1 : d0 * d0;
      if (cnt == 1) sq_init = sq;
      mares_old = mares;
      mares = summed ? div_n(r0) : r0;
      bool rates = true;
      if (__builtin_amdgcn_ballot_w64(cnt >= a.min_iter) != 0)
        rates = (cnt < a.min_iter) | ((sq / sq_init >= a.dp_thresh_sq) & (mares / mares_old <= a.dr_thresh));
      const bool keep = (cnt < a.max_iter) & (summed ? mares > a.res_thresh : r0 > 0.0f) & rates;
      if (!keep) converged = true;
    }
    first = false;
  }
  if (a.absw) {
    // the loss weights into the patch's LDS window (its tap reads are complete: one wave, LDS in order), then
    // each lane the aggregation weights of pixels s16 + 16 i from there
    if (live && !start_oob) {
      float r0;
      evaluate(r0, win, std::integral_constant<int, 1>(), std::false_type(), std::false_type());
    } else {
#pragma unroll
      for (int m = 0; m < M; ++m) win[s16 + 16 * m] = 0.0f;
    }
    wave_lds_sync();
    if (live) {
      const int ptx = (int)ptr0, pty = (int)ptr1;
      float *pl = a.pweight + agg_plane_off(f, a.aslots, pxi, pyi, g.w, g.h, ptx - P / 2, pty - P / 2);
#pragma unroll
      for (int i = 0; i < (P * P + 15) / 16; ++i) {
        const int q = s16 + 16 * i, lx = q % P, ly = q / P;
        const int x = ptx - P / 2 + lx, y = pty - P / 2 + ly;
        if (q < P * P && x >= 0 && y >= 0 && x < g.w && y < g.h)
          pl[ly * g.w + lx] = agg_weight(win, NOC, P, g.w, g.h, ptx, pty, lx, ly);
      }
    }
  } else if (live && !start_oob) {
    float r0;
    evaluate(r0, pwo, std::integral_constant<int, 1>(), std::false_type(), std::false_type());
  }
  if (live && s16 < NOP) a.p_iter[gp * NOP + s16] = s16 == 0 ? p0 : p1;
}

// ------------------------------------------------------------------------------------------------ aggregation

// Forward-backward merging (usefbcon, patchgrid.cpp:277-375): the complementary grid's patch q, at its
// optimised position pos, splats -displacement * bilinear weight over its footprint; pixel (x, y) receives
// the taps cc, fc, cf, ff of the loop positions (x, y), (x+1, y), (x, y+1), (x+1, y+1) in that order (the
// serial loop's order).  Positions with the target outside [1, w-1) x [1, h-1) are skipped; RGB keeps the
// weight-pointer quirk with those bounds.
struct CgPatch {
  int pos0, pos1;
  float wb[4];
  float fl0, fl1;
};
__device__ __forceinline__ void aggregate_cg_one(const AggArgs &a, const CgPatch &q, const float *pw, int x,
                                                 int y, float &we, float &f0, float &f1) {
  const LevelGeom &g = a.g;
  const int hp = a.p / 2;
  for (int k = 0; k < 4; ++k) {
    const int xt = x + (k & 1), yt = y + (k >> 1);
    const int lx = xt - q.pos0 + hp, ly = yt - q.pos1 + hp;
    if (lx < 0 || lx >= a.p || ly < 0 || ly >= a.p) continue;
    if (!(xt >= 1 && yt >= 1 && xt < g.w - 1 && yt < g.h - 1)) continue;
    float absw;
    if (a.noc == 1) {
      absw = 1.0f / stdmaxf(2.0f, pw[ly * a.p + lx]);
    } else {
      const int lx0 = max(0, 1 - q.pos0 + hp), lx1 = min(a.p, g.w - 1 - q.pos0 + hp);
      const int ly0 = max(0, 1 - q.pos1 + hp), ly1 = min(a.p, g.h - 1 - q.pos1 + hp);
      const int nin = max(0, lx1 - lx0);
      int before_in = max(0, min(ly, ly1) - ly0) * nin;
      if (ly >= ly0 && ly < ly1) before_in += max(0, min(lx, lx1) - lx0);
      const int off = ly * a.p + lx + 2 * before_in;
      absw = stdmaxf(2.0f, pw[off]);
      absw = absw + stdmaxf(2.0f, pw[off + 1]);
      absw = absw + stdmaxf(2.0f, pw[off + 2]);
      absw = 1.0f / absw;
    }
    const float n0 = q.fl0 * absw, n1 = q.fl1 * absw;
    we = we + q.wb[k] * absw;
    f0 = f0 - q.wb[k] * n0;
    if (a.nop == 2) f1 = f1 - q.wb[k] * n1;
  }
}

// 64 x 16 pixel tiles: the patch weights of one patch row are then read by one workgroup (one XCD's L2).
// With a complementary grid, its patches are staged through LDS 256 at a time (all of them, in id order:
// an optimised position is arbitrary) and each pixel tests its reach.
__global__ __launch_bounds__(256) void k_aggregate(AggArgs a) {
  const uint3 xb = xcd_block();
  __shared__ CgPatch cgs[256];
  const LevelGeom &g = a.g;
  const int x = xb.x * 64 + (threadIdx.x & 63), f = xb.z;
  // the displacements of every patch that covers the 64 x 16 tile, staged in LDS (option agg_stage): a wave's
  // gathers of p_iter otherwise touch one line per patch column (p_iter is column-major: stride noph).  Config E's
  // aggregation 12.8 -> 10.3 ms per step, C's 4.44 -> 2.97, B's unchanged (profiles/r06/s33).
  constexpr int kAggStage = 2048;
  __shared__ float pis[kAggStage];
  const int hp = a.p / 2;
  const int tx0 = xb.x * 64, ty0 = xb.y * 16;
  const int PX0 = max(0, -floordiv(-(tx0 - hp + 1 - g.offw), a.steps));
  const int PX1 = min(g.nopw - 1, floordiv(min(tx0 + 63, g.w - 1) + hp - g.offw, a.steps));
  const int PY0 = max(0, -floordiv(-(ty0 - hp + 1 - g.offh), a.steps));
  const int PY1 = min(g.noph - 1, floordiv(min(ty0 + 15, g.h - 1) + hp - g.offh, a.steps));
  const int NPX = PX1 - PX0 + 1, NPY = PY1 - PY0 + 1;
  const bool stage = a.stage && NPX > 0 && NPY > 0 && NPX * NPY * a.nop <= kAggStage;
  if (stage) {
    const float *PI = a.p_iter + (long)f * g.npatch * a.nop;
    const int per = NPY * a.nop;  // a patch column's run: (py, comp) contiguous in p_iter
    for (int i = threadIdx.x; i < NPX * per; i += 256) {
      const int cx = i / per, r = i - cx * per;
      pis[i] = PI[((PX0 + cx) * g.noph + PY0) * a.nop + r];
    }
    __syncthreads();
  }
  float we[4], f0[4], f1[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    we[r] = f0[r] = f1[r] = 0.0f;
    const int y = xb.y * 16 + (threadIdx.x >> 6) + 4 * r;
    if (x < g.w && y < g.h) aggregate_own(a, x, y, f, we[r], f0[r], f1[r], stage ? pis : nullptr, PX0, PY0, NPY);
  }
  if (a.cg_p_iter) {
    const float *CPI = a.cg_p_iter + (long)f * g.npatch * a.nop;
    const float *CPW = a.cg_pweight + (long)f * g.npatch * a.novals;
    for (int c0 = 0; c0 < g.npatch; c0 += 256) {
      const int q = c0 + threadIdx.x;
      if (q < g.npatch) {
        const int pxi = q / g.noph, pyi = q % g.noph;
        const float ptr0 = (float)(pxi * a.steps + g.offw), ptr1 = (float)(pyi * a.steps + g.offh);
        CgPatch e;
        e.fl0 = CPI[q * a.nop];
        e.fl1 = a.nop == 2 ? CPI[q * a.nop + 1] : 0.0f;
        const float rp0 = ptr0 + e.fl0, rp1 = a.nop == 2 ? ptr1 + e.fl1 : ptr1;  // GetPointPos (pt_iter)
        e.pos0 = (int)ceil((double)rp0 + .00001);
        e.pos1 = (int)ceil((double)rp1 + .00001);
        const float r0 = rp0 - (float)(int)floorf(rp0), r1 = rp1 - (float)(int)floorf(rp1);
        e.wb[0] = r0 * r1;
        e.wb[1] = (1 - r0) * r1;
        e.wb[2] = r0 * (1 - r1);
        e.wb[3] = (1 - r0) * (1 - r1);
        cgs[threadIdx.x] = e;
      }
      __syncthreads();
      const int nq = min(256, g.npatch - c0);
      for (int j = 0; j < nq; ++j) {
        const CgPatch &e = cgs[j];
        // reach of the patch: x in [pos0 - p/2 - 1, pos0 + p/2 - 1] (tile-level reject first)
        if (e.pos0 - hp - 1 > tx0 + 63 || e.pos0 + hp - 1 < tx0 || e.pos1 - hp - 1 > ty0 + 15 || e.pos1 + hp - 1 < ty0)
          continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int y = ty0 + (threadIdx.x >> 6) + 4 * r;
          if (x < g.w && y < g.h && x >= e.pos0 - hp - 1 && x <= e.pos0 + hp - 1 && y >= e.pos1 - hp - 1 &&
              y <= e.pos1 + hp - 1)
            aggregate_cg_one(a, e, CPW + (long)(c0 + j) * a.novals, x, y, we[r], f0[r], f1[r]);
        }
      }
      __syncthreads();
    }
  }
  const long plane = (long)g.w * g.h;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int y = xb.y * 16 + (threadIdx.x >> 6) + 4 * r;
    if (x >= g.w || y >= g.h) continue;
    float v0 = f0[r], v1 = f1[r];
    if (we[r] > 0) {
      v0 = v0 / we[r];
      v1 = v1 / we[r];
    }
    float *fl = a.flow + (long)f * a.nop * plane + (long)y * g.w + x;
    fl[0] = v0;
    if (a.nop == 2) fl[plane] = v1;
  }
}

// ------------------------------------------------------------------------------------------------ variational


// image_warp (opticalflow_aux.c:31-75) + the mean / temporal images of get_derivatives (:88-99), plus the
// skewed copies of the level flow and du = dv = 0 (refine_variational.cpp:185-190).  Row-major threads.
// image_warp (opticalflow_aux.c:31-75) + the t / It inputs of get_derivatives (:77-132) for pixel (x, y):
// v = {mask, wx, wy, t[0..noc), dt[0..noc)}.
__device__ __forceinline__ void tv_prep_values(const TvArgs &a, int x, int y, int f, float *v) {
  const long plane = (long)a.w * a.h;
  const long o = (long)y * a.w + x;
  const float wx = a.flow[(long)f * a.nop * plane + o];
  const float wy = a.nop == 2 ? a.flow[(long)f * a.nop * plane + plane + o] : 0.0f;
  const float xx = (float)x + wx, yy = (float)y + wy;
  const int xi = (int)floorf(xx), yi = (int)floorf(yy);
  const float dx = xx - (float)xi, dy = yy - (float)yi;
  v[0] = warp_mask(x, y, wx, wy, a.w, a.h);
  v[1] = wx;
  v[2] = wy;
  const int x1 = clampi(xi, 0, a.w - 1), x2 = clampi(xi + 1, 0, a.w - 1);
  const int y1 = clampi(yi, 0, a.h - 1), y2 = clampi(yi + 1, 0, a.h - 1);
  const long fs = (long)a.W * (a.h + 2 * a.pad) * a.noc;
  const float *B = a.img_b + f * fs, *A = a.img_a + f * fs;
#define SB(xq, yq) B[((long)((yq) + a.pad) * a.W + (xq) + a.pad) * a.noc + ch]
  for (int ch = 0; ch < a.noc; ++ch) {
    const float w2 = SB(x1, y1) * (1.0f - dx) * (1.0f - dy) + SB(x2, y1) * dx * (1.0f - dy) +
                     SB(x1, y2) * (1.0f - dx) * dy + SB(x2, y2) * dx * dy;
    const float i1 = A[((long)(y + a.pad) * a.W + x + a.pad) * a.noc + ch];
    v[3 + ch] = 0.5f * (w2 + i1);
    v[3 + a.noc + ch] = w2 - i1;
  }
#undef SB
}
// The values of pixel (x, y) into the skewed planes (du = dv = 0: the increment starts at zero).  The mask
// is not stored: it is a function of (x, y, wx, wy), which the system kernels recompute (warp_mask) from the
// skewed flow copies they read anyway -- 4 bytes per pixel and inner iteration less.
__device__ __forceinline__ void tv_prep_store(const TvArgs &a, int x, int y, int f, const float *v) {
  const long sk = skw(x, y, a.h, a.w, a.wrap), fk = (long)f * a.sp + sk;
  a.wxs[fk] = v[1];
  a.du[fk] = 0.0f;
  if (a.nop == 2) {
    a.wys[fk] = v[2];
    a.dv[fk] = 0.0f;
  }
  for (int ch = 0; ch < a.noc; ++ch) {
    const long q = ((long)f * a.noc + ch) * a.sp + sk;
    a.t[q] = v[3 + ch];
    a.dt[q] = v[3 + a.noc + ch];
  }
}

// Row-major <-> skewed conversions run on 64 x 16 pixel tiles transposed through LDS: the row-major side
// is read / written by rows, the skewed side by anti-diagonal segments of the tile (16 consecutive floats),
// so neither side scatters 4-byte accesses over 64 cache lines per instruction.  Row pitch 66: the
// diagonal-order accesses (row yy, column dd - yy) hit 16 different banks.
// TH: tile height.  A diagonal's run inside a 64 x TH tile is min(64, TH) pixels long, so the skewed side
// moves TH-float segments (TH = 16: 64-byte half lines, 2-3x the algorithmic bytes on the bus; taller
// tiles cut that).  NP = 3 + 2 noc planes.
constexpr int kTileW = 64, kTileP = 66;
template <int NP, int TH>
__global__ __launch_bounds__(256) void k_tv_prep(TvArgs a) {
  const uint3 xb = xcd_block();
  __shared__ float sm[NP][TH][kTileP];  // mask, wx, wy, t[noc], dt[noc]
  constexpr int TD = kTileW + TH - 1;
  const int x0 = xb.x * kTileW, y0 = xb.y * TH, f = xb.z;
  const int tx = threadIdx.x & 63, np = NP;
  for (int yl = threadIdx.x >> 6; yl < TH; yl += 4) {
    const int x = x0 + tx, y = y0 + yl;
    if (x < a.w && y < a.h) {
      float v[9];
      tv_prep_values(a, x, y, f, v);
      for (int k = 0; k < np; ++k) sm[k][yl][tx] = v[k];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TD * TH; i += 256) {
    const int yy = i & (TH - 1), dd = i / TH, xl = dd - yy;
    const int x = x0 + xl, y = y0 + yy;
    if (xl < 0 || xl >= kTileW || x >= a.w || y >= a.h) continue;
    float v[9];
    for (int k = 0; k < np; ++k) v[k] = sm[k][yy][xl];
    tv_prep_store(a, x, y, f, v);
  }
}


// 5-tap filters (image.cpp:419-624 fast paths) with replicate border, on a skewed plane.
__device__ __forceinline__ float conv5h(const float *s, int x, int y, int w, int h, int wr) {
  const float s0 = s[skw(clampi(x - 2, 0, w - 1), y, h, w, wr)], s1 = s[skw(clampi(x - 1, 0, w - 1), y, h, w, wr)];
  const float s2 = s[skw(x, y, h, w, wr)];
  const float s3 = s[skw(clampi(x + 1, 0, w - 1), y, h, w, wr)], s4 = s[skw(clampi(x + 2, 0, w - 1), y, h, w, wr)];
  return kK5[0] * s0 + ((kK5[1] * s1 + kK5[2] * s2) + (kK5[3] * s3 + kK5[4] * s4));
}
__device__ __forceinline__ float conv5v(const float *s, int x, int y, int w, int h, int wr) {
  const float s0 = s[skw(x, clampi(y - 2, 0, h - 1), h, w, wr)], s1 = s[skw(x, clampi(y - 1, 0, h - 1), h, w, wr)];
  const float s2 = s[skw(x, y, h, w, wr)];
  const float s3 = s[skw(x, clampi(y + 1, 0, h - 1), h, w, wr)], s4 = s[skw(x, clampi(y + 2, 0, h - 1), h, w, wr)];
  return kK5[0] * s0 + ((kK5[1] * s1 + kK5[2] * s2) + (kK5[3] * s3 + kK5[4] * s4));
}


// ---- prep + derivatives in one launch: image_warp and get_derivatives' t / It (opticalflow_aux.c:31-132) on a
// row-major tile with a 4-pixel halo in LDS, the first derivatives Ix, Iy of t on the tile with a 2-pixel halo, then
// per core pixel the remaining 5-tap filters (Ixz, Iyz of It; Ixx, Ixy of Ix; Iyy of Iy) straight from LDS and every
// plane written in skewed order (threads walk the tile's anti-diagonals: contiguous skewed rows).  A halo position
// outside the level holds the value of the clamped position, which is exactly the filters' replicate border; every
// value is the same expression as in k_tv_prep / k_tv_deriv1 / k_tv_deriv2: same bits, t / It / Ix / Iy never go
// through memory.  Intensity images; colour images (color_image_convolve_hv filters every channel alike:
// image.cpp:737-760) take k_tv_prepd_c3 below, every phase over the three channels.
constexpr int kPdW = 64, kPdH = 16;
template <int NOC>
__global__ __launch_bounds__(256) void k_tv_prepd(TvArgs a) {
  const uint3 xb = xcd_block();
  constexpr int H4 = kPdH + 8, W4 = kPdW + 8, H2 = kPdH + 4, W2 = kPdW + 4;
  __shared__ float T[H4][W4], DT[H4][W4], IX[H2][W2], IY[H2][W2], WX[kPdH][kPdW], WY[kPdH][kPdW];
  const int x0 = xb.x * kPdW, y0 = xb.y * kPdH, f = xb.z;
  const int w = a.w, h = a.h;
#pragma unroll 1
  for (int ch = 0; ch < NOC; ++ch) {
    if (ch > 0) __syncthreads();  // the previous channel's phase C has read the tiles
    // phase A: t, It at every halo-4 position (the clamped pixel's values), the flow of the core
    for (int i = threadIdx.x; i < H4 * W4; i += 256) {
      const int ly = i / W4, lx = i - ly * W4;
      const int xx = x0 - 4 + lx, yy = y0 - 4 + ly;
      const int cx = clampi(xx, 0, w - 1), cy = clampi(yy, 0, h - 1);
      float t, it, wx, wy;
      tv_prep_values_ch(a, cx, cy, f, ch, t, it, wx, wy);
      T[ly][lx] = t;
      DT[ly][lx] = it;
      const int cxl = lx - 4, cyl = ly - 4;
      if (ch == 0 && cxl >= 0 && cxl < kPdW && cyl >= 0 && cyl < kPdH) {
        WX[cyl][cxl] = wx;
        WY[cyl][cxl] = wy;
      }
    }
    __syncthreads();
    // phase B: Ix, Iy at every halo-2 position (of the clamped pixel): conv5h / conv5v of t
    for (int i = threadIdx.x; i < H2 * W2; i += 256) {
      const int ly = i / W2, lx = i - ly * W2;
      const int cx = clampi(x0 - 2 + lx, 0, w - 1), cy = clampi(y0 - 2 + ly, 0, h - 1);
      const int tx = cx - x0 + 4, ty = cy - y0 + 4;  // the clamped pixel in T (within the halo)
      IX[ly][lx] = kK5[0] * T[ty][tx - 2] + ((kK5[1] * T[ty][tx - 1] + kK5[2] * T[ty][tx]) +
                                            (kK5[3] * T[ty][tx + 1] + kK5[4] * T[ty][tx + 2]));
      IY[ly][lx] = kK5[0] * T[ty - 2][tx] + ((kK5[1] * T[ty - 1][tx] + kK5[2] * T[ty][tx]) +
                                            (kK5[3] * T[ty + 1][tx] + kK5[4] * T[ty + 2][tx]));
    }
    __syncthreads();
    // phase C: the core pixels in anti-diagonal order
    constexpr int TD = kPdW + kPdH - 1;
    for (int i = threadIdx.x; i < TD * kPdH; i += 256) {
      const int yy = i & (kPdH - 1), dd = i / kPdH, xl = dd - yy;
      const int x = x0 + xl, y = y0 + yy;
      if (xl < 0 || xl >= kPdW || x >= w || y >= h) continue;
      const int tx = xl + 4, ty = yy + 4, ix = xl + 2, iy = yy + 2;
      const float ixz = kK5[0] * DT[ty][tx - 2] + ((kK5[1] * DT[ty][tx - 1] + kK5[2] * DT[ty][tx]) +
                                                 (kK5[3] * DT[ty][tx + 1] + kK5[4] * DT[ty][tx + 2]));
      const float iyz = kK5[0] * DT[ty - 2][tx] + ((kK5[1] * DT[ty - 1][tx] + kK5[2] * DT[ty][tx]) +
                                                 (kK5[3] * DT[ty + 1][tx] + kK5[4] * DT[ty + 2][tx]));
      const float ixx = kK5[0] * IX[iy][ix - 2] + ((kK5[1] * IX[iy][ix - 1] + kK5[2] * IX[iy][ix]) +
                                                 (kK5[3] * IX[iy][ix + 1] + kK5[4] * IX[iy][ix + 2]));
      const float ixy = kK5[0] * IX[iy - 2][ix] + ((kK5[1] * IX[iy - 1][ix] + kK5[2] * IX[iy][ix]) +
                                                 (kK5[3] * IX[iy + 1][ix] + kK5[4] * IX[iy + 2][ix]));
      const float iyy = kK5[0] * IY[iy - 2][ix] + ((kK5[1] * IY[iy - 1][ix] + kK5[2] * IY[iy][ix]) +
                                                 (kK5[3] * IY[iy + 1][ix] + kK5[4] * IY[iy + 2][ix]));
      // lat: the colour-split entry layout of the fused red-black level launch, which keeps (du, dv) in LDS
      const long sk = a.lat ? lat_idx(x, y, w, lat_entries(w, h)) : skw(x, y, h, w, a.wrap), k = (long)f * a.sp + sk;
      if (ch == 0) {
        a.wxs[k] = WX[yy][xl];
        if (a.nop == 2) a.wys[k] = WY[yy][xl];
        if (!a.lat) {
          a.du[k] = 0.0f;
          if (a.nop == 2) a.dv[k] = 0.0f;
        }
      }
      const long q = ((long)f * NOC + ch) * a.sp + sk;
      a.Iz[q] = DT[ty][tx];
      a.Ix[q] = IX[iy][ix];
      a.Iy[q] = IY[iy][ix];
      if (a.smsys_deriv) continue;  // the system kernel filters Ix, Iy, Iz itself
      a.Ixx[q] = ixx;
      a.Ixy[q] = ixy;
      a.Iyy[q] = iyy;
      a.Ixz[q] = ixz;
      a.Iyz[q] = iyz;
    }
  }
}

// Colour images, all eight planes (levels whose system kernel reads them): k_tv_prepd<3> with the three channels in
// each phase instead of the phases once per channel -- the flow, warp position and bilinear weights once per halo
// position (tv_prep_values_all), It kept on the 2-pixel halo only (Ixz / Iyz), and two barriers instead of eight.
// 78 KB of LDS: two workgroups per CU.  Same expressions, same bits.  Config C: 3.36 -> 3.15 ms of prep per
// 512-pair step (r06_s11), the 240 x 135 level 554 -> 471 us per 256 pairs (r06_s12).
__global__ __launch_bounds__(256) void k_tv_prepd_c3(TvArgs a) {
  const uint3 xb = xcd_block();
  constexpr int NOC = 3, H4 = kPdH + 8, W4 = kPdW + 8, H2 = kPdH + 4, W2 = kPdW + 4;
  __shared__ float T[NOC][H4][W4], DT[NOC][H2][W2], IX[NOC][H2][W2], IY[NOC][H2][W2], WX[kPdH][kPdW], WY[kPdH][kPdW];
  const int x0 = xb.x * kPdW, y0 = xb.y * kPdH, f = xb.z;
  const int w = a.w, h = a.h;
  constexpr int NPOS = H4 * W4, NIT = (NPOS + 255) / 256, PB = 4;
#pragma unroll
  for (int j0 = 0; j0 < NIT; j0 += PB) {
    float t[PB][NOC], it[PB][NOC], wx[PB], wy[PB];
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int i = min((int)threadIdx.x + (j0 + j) * 256, NPOS - 1);
      const int ly = i / W4, lx = i - ly * W4;
      const int cx = clampi(x0 - 4 + lx, 0, w - 1), cy = clampi(y0 - 4 + ly, 0, h - 1);
      tv_prep_values_all<NOC>(a, cx, cy, f, t[j], it[j], wx[j], wy[j]);
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int i = (int)threadIdx.x + (j0 + j) * 256;
      if (j0 + j >= NIT || i >= NPOS) break;
      const int ly = i / W4, lx = i - ly * W4;
#pragma unroll
      for (int ch = 0; ch < NOC; ++ch) T[ch][ly][lx] = t[j][ch];
      const int hx = lx - 2, hy = ly - 2;
      if (hx >= 0 && hx < W2 && hy >= 0 && hy < H2) {
#pragma unroll
        for (int ch = 0; ch < NOC; ++ch) DT[ch][hy][hx] = it[j][ch];
      }
      const int cxl = lx - 4, cyl = ly - 4;
      if (cxl >= 0 && cxl < kPdW && cyl >= 0 && cyl < kPdH) {
        WX[cyl][cxl] = wx[j];
        WY[cyl][cxl] = wy[j];
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NOC * H2 * W2; i += 256) {
    const int ch = i / (H2 * W2), r = i - ch * (H2 * W2);
    const int ly = r / W2, lx = r - ly * W2;
    const int cx = clampi(x0 - 2 + lx, 0, w - 1), cy = clampi(y0 - 2 + ly, 0, h - 1);
    const int tx = cx - x0 + 4, ty = cy - y0 + 4;
    IX[ch][ly][lx] = kK5[0] * T[ch][ty][tx - 2] + ((kK5[1] * T[ch][ty][tx - 1] + kK5[2] * T[ch][ty][tx]) +
                                                  (kK5[3] * T[ch][ty][tx + 1] + kK5[4] * T[ch][ty][tx + 2]));
    IY[ch][ly][lx] = kK5[0] * T[ch][ty - 2][tx] + ((kK5[1] * T[ch][ty - 1][tx] + kK5[2] * T[ch][ty][tx]) +
                                                  (kK5[3] * T[ch][ty + 1][tx] + kK5[4] * T[ch][ty + 2][tx]));
  }
  __syncthreads();
  constexpr int TD = kPdW + kPdH - 1;
  for (int i = threadIdx.x; i < TD * kPdH; i += 256) {
    const int yy = i & (kPdH - 1), dd = i / kPdH, xl = dd - yy;
    const int x = x0 + xl, y = y0 + yy;
    if (xl < 0 || xl >= kPdW || x >= w || y >= h) continue;
    const int ix = xl + 2, iy = yy + 2;  // (DT, IX, IY: 2-pixel halo)
    const long sk = a.lat ? lat_idx(x, y, w, lat_entries(w, h)) : skw(x, y, h, w, a.wrap), k = (long)f * a.sp + sk;
    a.wxs[k] = WX[yy][xl];
    if (a.nop == 2) a.wys[k] = WY[yy][xl];
    if (!a.lat) {  // (the latency mode's level launch keeps du, dv in LDS)
      a.du[k] = 0.0f;
      if (a.nop == 2) a.dv[k] = 0.0f;
    }
#pragma unroll
    for (int ch = 0; ch < NOC; ++ch) {
      const float(&D)[H2][W2] = DT[ch];
      const float(&X)[H2][W2] = IX[ch];
      const float(&Y)[H2][W2] = IY[ch];
      const long q = ((long)f * NOC + ch) * a.sp + sk;
      a.Iz[q] = D[iy][ix];
      a.Ix[q] = X[iy][ix];
      a.Iy[q] = Y[iy][ix];
      a.Ixz[q] = kK5[0] * D[iy][ix - 2] + ((kK5[1] * D[iy][ix - 1] + kK5[2] * D[iy][ix]) +
                                          (kK5[3] * D[iy][ix + 1] + kK5[4] * D[iy][ix + 2]));
      a.Iyz[q] = kK5[0] * D[iy - 2][ix] + ((kK5[1] * D[iy - 1][ix] + kK5[2] * D[iy][ix]) +
                                          (kK5[3] * D[iy + 1][ix] + kK5[4] * D[iy + 2][ix]));
      a.Ixx[q] = kK5[0] * X[iy][ix - 2] + ((kK5[1] * X[iy][ix - 1] + kK5[2] * X[iy][ix]) +
                                          (kK5[3] * X[iy][ix + 1] + kK5[4] * X[iy][ix + 2]));
      a.Ixy[q] = kK5[0] * X[iy - 2][ix] + ((kK5[1] * X[iy - 1][ix] + kK5[2] * X[iy][ix]) +
                                          (kK5[3] * X[iy + 1][ix] + kK5[4] * X[iy + 2][ix]));
      a.Iyy[q] = kK5[0] * Y[iy - 2][ix] + ((kK5[1] * Y[iy - 1][ix] + kK5[2] * Y[iy][ix]) +
                                          (kK5[3] * Y[iy + 1][ix] + kK5[4] * Y[iy + 2][ix]));
    }
  }
}

// The same launch where the system kernel filters the second derivatives itself (smsys_deriv: k_tv_smsys<.., DF> /
// k_tv_smsys_m<.., DF>), so only t's first derivatives and It are written: t is needed on a 2-pixel halo (not 4),
// It only at the core (it goes straight to Iz), and every channel is warped in the same pass (the flow, the warp
// position and the bilinear weights once per position, not once per channel; tv_prep_values_all).  One barrier, no
// second-derivative tiles: 1360 warped positions per 64 x 16 tile instead of 1728 per channel, and 37 KB of LDS
// (colour) / 18 KB (intensity); TH = 32 (levels of 256+ rows, 512 threads): 70 / 34 KB.  Ix = conv5h(t), Iy =
// conv5v(t) with the replicate border of the clamped halo: the values of k_tv_prepd's phase B, same bits.
template <int NOC, int TH = kPdH>
__global__ __launch_bounds__(16 * TH) void k_tv_prepd_df(TvArgs a) {
  constexpr int NT = 16 * TH;  // threads: 16 per tile row
  const uint3 xb = xcd_block();
  constexpr int H2 = TH + 4, W2 = kPdW + 4;
  __shared__ float T[NOC][H2][W2], DT[NOC][TH][kPdW], WX[TH][kPdW], WY[TH][kPdW];
  const int x0 = xb.x * kPdW, y0 = xb.y * TH, f = xb.z;
  const int w = a.w, h = a.h;
  // positions in batches of PB per thread with unconditional (index-clamped) loads: PB independent warp chains in
  // flight instead of one
  constexpr int NPOS = H2 * W2, NIT = (NPOS + NT - 1) / NT, PB = TH >= 32 && NOC == 3 ? 5 : 3;
#pragma unroll
  for (int j0 = 0; j0 < NIT; j0 += PB) {
    float t[PB][NOC], it[PB][NOC], wx[PB], wy[PB];
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int i = min((int)threadIdx.x + (j0 + j) * NT, NPOS - 1);
      const int ly = i / W2, lx = i - ly * W2;
      const int cx = clampi(x0 - 2 + lx, 0, w - 1), cy = clampi(y0 - 2 + ly, 0, h - 1);
      tv_prep_values_all<NOC>(a, cx, cy, f, t[j], it[j], wx[j], wy[j]);
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int i = (int)threadIdx.x + (j0 + j) * NT;
      if (j0 + j >= NIT || i >= NPOS) break;
      const int ly = i / W2, lx = i - ly * W2;
#pragma unroll
      for (int ch = 0; ch < NOC; ++ch) T[ch][ly][lx] = t[j][ch];
      const int cxl = lx - 2, cyl = ly - 2;
      if (cxl >= 0 && cxl < kPdW && cyl >= 0 && cyl < TH) {
#pragma unroll
        for (int ch = 0; ch < NOC; ++ch) DT[ch][cyl][cxl] = it[j][ch];
        WX[cyl][cxl] = wx[j];
        WY[cyl][cxl] = wy[j];
      }
    }
  }
  __syncthreads();
  constexpr int TD = kPdW + TH - 1;
  for (int i = threadIdx.x; i < TD * TH; i += NT) {
    const int yy = i & (TH - 1), dd = i / TH, xl = dd - yy;
    const int x = x0 + xl, y = y0 + yy;
    if (xl < 0 || xl >= kPdW || x >= w || y >= h) continue;
    const int tx = xl + 2, ty = yy + 2;
    const long sk = skw(x, y, h, w, a.wrap), k = (long)f * a.sp + sk;
    a.wxs[k] = WX[yy][xl];
    if (a.nop == 2) a.wys[k] = WY[yy][xl];
    a.du[k] = 0.0f;
    if (a.nop == 2) a.dv[k] = 0.0f;
#pragma unroll
    for (int ch = 0; ch < NOC; ++ch) {
      const long q = ((long)f * NOC + ch) * a.sp + sk;
      a.Iz[q] = DT[ch][yy][xl];
      a.Ix[q] = kK5[0] * T[ch][ty][tx - 2] + ((kK5[1] * T[ch][ty][tx - 1] + kK5[2] * T[ch][ty][tx]) +
                                             (kK5[3] * T[ch][ty][tx + 1] + kK5[4] * T[ch][ty][tx + 2]));
      a.Iy[q] = kK5[0] * T[ch][ty - 2][tx] + ((kK5[1] * T[ch][ty - 1][tx] + kK5[2] * T[ch][ty][tx]) +
                                             (kK5[3] * T[ch][ty + 1][tx] + kK5[4] * T[ch][ty + 2][tx]));
    }
  }
}

// decode a skewed-plane thread index; false for holes (unwrapped layout) and the dump slots
__device__ __forceinline__ bool skew_xy(int kk, int w, int h, int wrap, int &x, int &y) {
  const int t = kk / h;
  y = kk - t * h;
  x = t - y;
  if (wrap) {
    if (x < 0) x += w;
    return t < w;
  }
  return x >= 0 && x < w;
}

__device__ __forceinline__ void tv_deriv1_px(const TvArgs &a, long pl, int kk) {
  const long idx = pl * a.sp + kk;
  int x, y;
  if (!skew_xy(kk, a.w, a.h, a.wrap, x, y)) return;
  const float *t = a.t + pl * a.sp, *dt = a.dt + pl * a.sp;
  a.Ix[idx] = conv5h(t, x, y, a.w, a.h, a.wrap);
  a.Iy[idx] = conv5v(t, x, y, a.w, a.h, a.wrap);
  a.Ixz[idx] = conv5h(dt, x, y, a.w, a.h, a.wrap);
  a.Iyz[idx] = conv5v(dt, x, y, a.w, a.h, a.wrap);
}

__device__ __forceinline__ void tv_deriv2_px(const TvArgs &a, long pl, int kk) {
  const long idx = pl * a.sp + kk;
  int x, y;
  if (!skew_xy(kk, a.w, a.h, a.wrap, x, y)) return;
  a.Ixx[idx] = conv5h(a.Ix + pl * a.sp, x, y, a.w, a.h, a.wrap);
  a.Ixy[idx] = conv5v(a.Ix + pl * a.sp, x, y, a.w, a.h, a.wrap);
  a.Iyy[idx] = conv5v(a.Iy + pl * a.sp, x, y, a.w, a.h, a.wrap);
}

__global__ __launch_bounds__(256) void k_tv_deriv1(TvArgs a) {
  const uint3 b = xcd_block();
  const int kk = b.x * blockDim.x + threadIdx.x;
  if (kk < a.sp) tv_deriv1_px(a, b.y, kk);
}
__global__ __launch_bounds__(256) void k_tv_deriv2(TvArgs a) {
  const uint3 b = xcd_block();
  const int kk = b.x * blockDim.x + threadIdx.x;
  if (kk < a.sp) tv_deriv2_px(a, b.y, kk);
}


// compute_smoothness (opticalflow_aux.c:138-160): s = (alpha/4) / sqrt(eps + |grad u|^2 + |grad v|^2)
template <int NOP>
__device__ __forceinline__ void tv_smooth_px(const TvArgs &a, long fr, int kk, bool first) {
  const long f0 = fr * a.sp, idx = f0 + kk;
  int x, y;
  if (!skew_xy(kk, a.w, a.h, a.wrap, x, y)) return;
  const int w = a.w, h = a.h;
  const int wr = a.wrap;
  const long kl = f0 + skw(x > 0 ? x - 1 : 0, y, h, w, wr), kr = f0 + skw(x < w - 1 ? x + 1 : w - 1, y, h, w, wr);
  const long ku = f0 + skw(x, y > 0 ? y - 1 : 0, h, w, wr), kd = f0 + skw(x, y < h - 1 ? y + 1 : h - 1, h, w, wr);
  const unsigned k5[5] = {(unsigned)idx, (unsigned)kl, (unsigned)kr, (unsigned)ku, (unsigned)kd};
  // gather everything first (one memory round trip), then uu = wx (first iteration) or wx + du
  float wx5[5], du5[5], wy5[5], dv5[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    wx5[i] = ldu(a.wxs, k5[i]);
    du5[i] = ldu(a.du, k5[i]);
    if (NOP == 2) {
      wy5[i] = ldu(a.wys, k5[i]);
      dv5[i] = ldu(a.dv, k5[i]);
    }
  }
  a.s[idx] = smooth_compute<NOP>(a, first, wx5, du5, wy5, dv5);
}


// One TV inner iteration's system (refine_variational.cpp:195-199): diffusivities from s
// (opticalflow_aux.c:161-184), data term (:408-747) and sub_laplacian (:194-223).
// All of a pixel's inputs are gathered first with unconditional loads (border neighbours clamped to the
// pixel itself and discarded by selects afterwards): one memory round trip per pixel instead of one per
// data-dependent branch.
template <int NOP, int NOC>
__device__ __forceinline__ void tv_system_px(const TvArgs &a, long fr, int kk) {
  const long idx = fr * a.sp + kk;
  int x, y;
  if (!skew_xy(kk, a.w, a.h, a.wrap, x, y)) return;
  const int w = a.w, h = a.h;
  const bool hasl = x >= 1, hasr = x <= w - 2, hasu = y >= 1, hasd = y <= h - 2;
  const unsigned f0 = (unsigned)(fr * a.sp), ui = (unsigned)idx;
  const unsigned il = hasl ? f0 + (unsigned)skw(x - 1, y, h, w, a.wrap) : ui;
  const unsigned ir = hasr ? f0 + (unsigned)skw(x + 1, y, h, w, a.wrap) : ui;
  const unsigned iu = hasu ? f0 + (unsigned)skw(x, y - 1, h, w, a.wrap) : ui;
  const unsigned id = hasd ? f0 + (unsigned)skw(x, y + 1, h, w, a.wrap) : ui;
  // ---- gather
  const unsigned i5[5] = {ui, il, ir, iu, id};
  float S5[5], X5[5], Y5[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    S5[k] = ldu(a.s, i5[k]);
    X5[k] = ldu(a.wxs, i5[k]);
    Y5[k] = NOP == 2 ? ldu(a.wys, i5[k]) : 0.0f;
  }
  const float u = ldu(a.du, ui), v = NOP == 2 ? ldu(a.dv, ui) : 0.0f;
  const float m = warp_mask(x, y, X5[0], Y5[0], w, h);
  const unsigned q = (unsigned)(fr * NOC * a.sp + kk);
  float lIx[NOC], lIy[NOC], lIz[NOC], lIxx[NOC], lIxy[NOC], lIyy[NOC], lIxz[NOC], lIyz[NOC];
#pragma unroll
  for (int c = 0; c < NOC; ++c) {
    const unsigned o = q + (unsigned)(c * a.sp);
    lIx[c] = ldu(a.Ix, o); lIy[c] = ldu(a.Iy, o); lIz[c] = ldu(a.Iz, o); lIxx[c] = ldu(a.Ixx, o);
    lIxy[c] = ldu(a.Ixy, o); lIyy[c] = ldu(a.Iyy, o); lIxz[c] = ldu(a.Ixz, o); lIyz[c] = ldu(a.Iyz, o);
  }
  // ---- compute
  float4 c0, c1;
  sys_compute<NOP, NOC>(a, x, y, S5, X5, Y5, m, u, v, lIx, lIy, lIz, lIxx, lIxy, lIyy, lIxz, lIyz, c0, c1);
  if (NOP == 2) {
    float4 *C = reinterpret_cast<float4 *>(a.coef) + 2 * idx;
    C[0] = c0;
    C[1] = c1;
  } else {
    reinterpret_cast<float4 *>(a.coef)[idx] = c0;
  }
}

template <int NOP>
__global__ __launch_bounds__(256) void k_tv_smooth(TvArgs a) {
  const uint3 b = xcd_block();
  const int kk = b.x * blockDim.x + threadIdx.x;
  if (kk < a.sp) tv_smooth_px<NOP>(a, b.y, kk, a.first_iter != 0);
}
template <int NOP, int NOC>
__global__ __launch_bounds__(256) void k_tv_system(TvArgs a) {
  const uint3 b = xcd_block();
  const int kk = b.x * blockDim.x + threadIdx.x;
  if (kk < a.sp) tv_system_px<NOP, NOC>(a, b.y, kk);
}

// ---- smoothness + system in one launch (compute_smoothness + the system of refine_variational.cpp:195-199)
// A workgroup takes RB consecutive rows of one frame's skewed plane.  In both layouts the 4-neighbours of a
// row-r pixel lie in rows r - 1 (left: same column, up: column - 1) and r + 1 (right: same column, down:
// column + 1), modulo w when folded.  Phase 0 stages (wx, wy, du, dv) of rows r0-2 .. r0+RB+1 in LDS,
// phase 1 computes s of rows r0-1 .. r0+RB into LDS (smooth_compute, tv_smooth_px's replicate border),
// phase 2 the system of rows r0 .. r0+RB-1 (sys_compute).  s never goes to memory and (wx, wy, du, dv)
// are read once (plus the halo) instead of by two kernels: same functions, same bits.  blockIdx.x is the
// frame, so the row blocks of a frame (which share halo rows) land on one XCD.
__host__ __device__ __forceinline__ int smsys_rows(int w, int h, int wrap) { return wrap ? w : w + h - 1; }
__host__ __device__ __forceinline__ int smsys_rb(int h) { return h >= 1024 ? 1 : (1024 / h > 16 ? 16 : 1024 / h); }
__host__ __device__ __forceinline__ size_t smsys_lds_rb(int h, int rb) {
  return (size_t)(rb + 4) * h * 16 + (size_t)(rb + 2) * h * 4;
}
__host__ __device__ __forceinline__ size_t smsys_lds(int h) { return smsys_lds_rb(h, smsys_rb(h)); }
// Rows per workgroup of a launch: smsys_rb's (up to 1024 pixels, 4 per thread) when the launch has enough
// workgroups to fill the chip (>= 4096), else about one pixel per thread (>= 4 rows): the latency regime
// (the drop-in CLI's single pair, config D's 32 pairs per GPU) then spreads a level over 3-4x the CUs.
__host__ __device__ __forceinline__ int smsys_rb_n(int h, int rows, int n, int small) {
  const int rb = smsys_rb(h);
  if (!small || (long)n * ((rows + rb - 1) / rb) >= 4096) return rb;
  const int r1 = (256 + h - 1) / h;
  return r1 < 4 ? 4 : (r1 < rb ? r1 : rb);
}

// DF (intensity images, option smsys_deriv): Ix, Iy, Iz are staged with (wx, wy, du, dv) -- same rows, same halo
// -- and the five second-order filters of get_derivatives (Ixx, Ixy of Ix; Iyy of Iy; Ixz, Iyz of It = Iz:
// opticalflow_aux.c:77-132, k_tv_deriv2 / k_tv_prepd's expressions and replicate border) are computed per
// pixel from LDS instead of read as five planes (k_tv_prepd then does not write them): 20 bytes per pixel and
// inner iteration less read, 20 per level less written.  A row-r pixel's horizontal neighbour x + k is staged
// row r + k, same column; its vertical neighbour y + k is row r + k, column y + k (k <= 2: inside the halo).
__host__ __device__ __forceinline__ size_t smsys_lds_df(int h, int rb, bool df) {
  return smsys_lds_rb(h, rb) + (df ? (size_t)3 * (rb + 4) * h * 4 : 0);
}
constexpr size_t kSmsysDfCap = 40 * 1024;
template <int NOP, int NOC, bool DF = false>
__global__ __launch_bounds__(256) void k_tv_smsys(TvArgs a) {
  extern __shared__ float4 st[];  // [(RB + 4) * h] (wx, wy, du, dv), then float s[(RB + 2) * h] (DF: Ix, Iy, Iz)
  static_assert(!DF || NOC == 1, "staged derivatives: intensity images");
  const int w = a.w, h = a.h, rows = smsys_rows(w, h, a.wrap);
  int rb = smsys_rb_n(h, rows, a.n, a.smsys_small);
  if (DF)  // four workgroups per CU (five, at 32 KB: slower, r03_s49); the launcher applies the same rule
    while (rb > 1 && smsys_lds_df(h, rb, true) > kSmsysDfCap) --rb;
  float *sl = reinterpret_cast<float *>(st + (rb + 4) * h);
  float *gIx = sl + (rb + 2) * h, *gIy = gIx + (rb + 4) * h, *gIz = gIy + (rb + 4) * h;  // DF
  const int f = blockIdx.x, r0 = blockIdx.y * rb;
  const long f0 = (long)f * a.sp;
  const bool first = a.first_iter != 0;
  // plane row of a staged / s row index (r0 - 2 + i); -1 when it does not exist (unfolded layout)
  auto prow = [&](int r) { return a.wrap ? (r < 0 ? r + w : (r >= w ? r - w : r)) : (r < 0 || r >= rows ? -1 : r); };
  // intensity images: the derivative images of this thread's phase-2 pixels (rb * h <= 1024: at most 4) are
  // loaded first, so they are in flight with the staging loads instead of a second round trip after two barriers
  constexpr int PF = NOC == 1 ? 4 : 1;
  float pre[PF][8];
  const bool pf = NOC == 1 && !DF && a.smsys_prefetch;
  if (pf) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int i = threadIdx.x + j * (int)blockDim.x;
      const int ri = i / h, y = i - ri * h, rr = r0 + ri;
      const bool ok = i < rb * h && rr < rows;
      const unsigned o = (unsigned)((long)f * a.sp + (long)(ok ? rr : 0) * h + (ok ? y : 0));
      pre[j][0] = ldu(a.Ix, o); pre[j][1] = ldu(a.Iy, o); pre[j][2] = ldu(a.Iz, o); pre[j][3] = ldu(a.Ixx, o);
      pre[j][4] = ldu(a.Ixy, o); pre[j][5] = ldu(a.Iyy, o); pre[j][6] = ldu(a.Ixz, o); pre[j][7] = ldu(a.Iyz, o);
    }
  }
  // ---- phase 0: stage
  for (int i = threadIdx.x; i < (rb + 4) * h; i += blockDim.x) {
    const int ri = i / h, y = i - ri * h;
    const int r = prow(r0 - 2 + ri);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    float dx = 0.f, dy = 0.f, dz = 0.f;
    if (r >= 0) {
      const long o = f0 + (long)r * h + y;
      v.x = a.wxs[o];
      v.z = a.du[o];
      if (NOP == 2) {
        v.y = a.wys[o];
        v.w = a.dv[o];
      }
      if (DF) {
        dx = a.Ix[o];
        dy = a.Iy[o];
        dz = a.Iz[o];
      }
    }
    st[i] = v;
    if (DF) {
      gIx[i] = dx;
      gIy[i] = dy;
      gIz[i] = dz;
    }
  }
  __syncthreads();
  // ---- phase 1: s of rows r0 - 1 .. r0 + rb
  auto pix = [&](int r, int y, int &x) {  // plane (row, column) -> pixel x; false outside the level
    if (r < 0) return false;
    x = r - y;
    if (a.wrap) {
      if (x < 0) x += w;
      return true;
    }
    return x >= 0 && x < w;
  };
  for (int i = threadIdx.x; i < (rb + 2) * h; i += blockDim.x) {
    const int ri = i / h, y = i - ri * h;  // s row ri <-> staged row ri + 1
    const int r = prow(r0 - 1 + ri);
    int x;
    float sv = 0.0f;
    if (pix(r, y, x)) {
      const int c = (ri + 1) * h + y;
      const int cl = x > 0 ? c - h : c, cr = x < w - 1 ? c + h : c;
      const int cu = y > 0 ? c - h - 1 : c, cd = y < h - 1 ? c + h + 1 : c;
      const float4 q0 = st[c], q1 = st[cl], q2 = st[cr], q3 = st[cu], q4 = st[cd];
      const float wx5[5] = {q0.x, q1.x, q2.x, q3.x, q4.x}, du5[5] = {q0.z, q1.z, q2.z, q3.z, q4.z};
      const float wy5[5] = {q0.y, q1.y, q2.y, q3.y, q4.y}, dv5[5] = {q0.w, q1.w, q2.w, q3.w, q4.w};
      sv = smooth_compute<NOP>(a, first, wx5, du5, wy5, dv5);
    }
    sl[i] = sv;
  }
  __syncthreads();
  // ---- phase 2: the system of rows r0 .. r0 + rb - 1
#pragma unroll
  for (int j = 0; j < (NOC == 1 ? PF : 1); ++j) {
  for (int i = threadIdx.x + j * (int)blockDim.x; i < rb * h; i += (NOC == 1 ? PF : 1) * (int)blockDim.x) {
    const int ri = i / h, y = i - ri * h;
    const int rr = r0 + ri;
    if (rr >= rows) break;
    int x;
    if (!pix(rr, y, x)) continue;
    const int c = (ri + 1) * h + y, cs = c + h;  // s index (row ri + 1), staged index (row ri + 2)
    const int yu = y > 0 ? -1 : 0, yd = y < h - 1 ? 1 : 0;  // clamped columns; absent neighbours are discarded
    const int s5[5] = {c, c - h, c + h, c - h + yu, c + h + yd};
    const int t5[5] = {cs, cs - h, cs + h, cs - h + yu, cs + h + yd};
    float S5[5], X5[5], Y5[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      S5[k] = sl[s5[k]];
      const float4 q = st[t5[k]];
      X5[k] = q.x;
      Y5[k] = NOP == 2 ? q.y : 0.0f;
    }
    const float4 qc = st[cs];
    const long idx = f0 + (long)rr * h + y;
    const float m = warp_mask(x, y, X5[0], Y5[0], w, h);
    const unsigned qd = (unsigned)((long)f * NOC * a.sp + (long)rr * h + y);
    float lIx[NOC], lIy[NOC], lIz[NOC], lIxx[NOC], lIxy[NOC], lIyy[NOC], lIxz[NOC], lIyz[NOC];
    if constexpr (DF) {
      // replicate border: the clamped tap's staged offset (rows for x, rows + columns for y)
      const int hx0 = (max(x - 2, 0) - x) * h, hx1 = (max(x - 1, 0) - x) * h;
      const int hx3 = (min(x + 1, w - 1) - x) * h, hx4 = (min(x + 2, w - 1) - x) * h;
      const int vy0 = (max(y - 2, 0) - y) * (h + 1), vy1 = (max(y - 1, 0) - y) * (h + 1);
      const int vy3 = (min(y + 1, h - 1) - y) * (h + 1), vy4 = (min(y + 2, h - 1) - y) * (h + 1);
      auto c5h = [&](const float *P) {
        return kK5[0] * P[cs + hx0] + ((kK5[1] * P[cs + hx1] + kK5[2] * P[cs]) + (kK5[3] * P[cs + hx3] + kK5[4] * P[cs + hx4]));
      };
      auto c5v = [&](const float *P) {
        return kK5[0] * P[cs + vy0] + ((kK5[1] * P[cs + vy1] + kK5[2] * P[cs]) + (kK5[3] * P[cs + vy3] + kK5[4] * P[cs + vy4]));
      };
      lIx[0] = gIx[cs];
      lIy[0] = gIy[cs];
      lIz[0] = gIz[cs];
      lIxx[0] = c5h(gIx);
      lIxy[0] = c5v(gIx);
      lIyy[0] = c5v(gIy);
      lIxz[0] = c5h(gIz);
      lIyz[0] = c5v(gIz);
    } else if (pf && i < PF * (int)blockDim.x) {  // (rb * h <= 1024 whenever this kernel runs)
      lIx[0] = pre[j][0]; lIy[0] = pre[j][1]; lIz[0] = pre[j][2]; lIxx[0] = pre[j][3];
      lIxy[0] = pre[j][4]; lIyy[0] = pre[j][5]; lIxz[0] = pre[j][6]; lIyz[0] = pre[j][7];
    } else {
#pragma unroll
      for (int ch = 0; ch < NOC; ++ch) {
        const unsigned o = qd + (unsigned)(ch * a.sp);
        lIx[ch] = ldu(a.Ix, o); lIy[ch] = ldu(a.Iy, o); lIz[ch] = ldu(a.Iz, o); lIxx[ch] = ldu(a.Ixx, o);
        lIxy[ch] = ldu(a.Ixy, o); lIyy[ch] = ldu(a.Iyy, o); lIxz[ch] = ldu(a.Ixz, o); lIyz[ch] = ldu(a.Iyz, o);
      }
    }
    float4 c0, c1;
    sys_compute<NOP, NOC>(a, x, y, S5, X5, Y5, m, qc.z, NOP == 2 ? qc.w : 0.0f, lIx, lIy, lIz, lIxx, lIxy, lIyy,
                          lIxz, lIyz, c0, c1);
    if (NOP == 2) {
      float4 *C = reinterpret_cast<float4 *>(a.coef) + 2 * idx;
      C[0] = c0;
      C[1] = c1;
    } else {
      reinterpret_cast<float4 *>(a.coef)[idx] = c0;
    }
  }
  }
}

// ---- smoothness + system as a register march (tall levels, h > 256; round 3)
// One wave takes 64 consecutive columns (y0 - 2 .. y0 + 61) of one frame's skewed plane and walks a segment of
// kMR rows.  A row-r pixel's 4-neighbours lie in rows r -+ 1 (left / right: same column; up / down: column
// -+ 1), so with the rows r - 1 .. r + 2 of (wx, du, wy, dv) and the rows r - 1 .. r + 1 of s in registers, a
// step loads row r + 2, computes s of row r + 1 and the system of row r; the column -+ 1 operands come from the
// neighbouring lanes (DPP wave shifts).  s is valid on lanes 1 .. 62 and the system on lanes 2 .. 61 (60
// columns per wave).  Everything streams once (plus 4 halo rows per kMR and 4 halo columns per 60): no LDS,
// no barrier, no s round trip; the same functions as k_tv_smooth / k_tv_system, so the same bits.
constexpr int kMR = 64, kMC = 60;
__device__ __forceinline__ float wave_from_prev(float v) {  // lane i <- lane i - 1 (lane 0: its own value)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v),
                                                                0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_from_next(float v) {  // lane i <- lane i + 1 (lane 63: its own value)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v),
                                                                0x130, 0xF, 0xF, false));
}
__host__ __device__ __forceinline__ int march_segments(int rows) { return (rows + kMR - 1) / kMR; }
__host__ __device__ __forceinline__ int march_strips(int h) { return (h + kMC - 1) / kMC; }

// get_derivatives' 5-tap filter from the taps at offsets -2 .. 2 along one axis, replicate border: a tap past the
// border takes the border pixel's value, one of the taps held (pos = the pixel's coordinate on the axis, n = the
// level's extent); k_tv_smsys<.., DF>'s expression (c5h / c5v)
__device__ __forceinline__ float conv5_clamp(const float (&t)[5], int pos, int n) {
  const float m1 = pos >= 1 ? t[1] : t[2];
  const float m2 = pos >= 2 ? t[0] : m1;
  const float p1 = pos <= n - 2 ? t[3] : t[2];
  const float p2 = pos <= n - 3 ? t[4] : p1;
  return kK5[0] * m2 + ((kK5[1] * m1 + kK5[2] * t[2]) + (kK5[3] * p1 + kK5[4] * p2));
}

// DF (option smsys_deriv; intensity images round 4, colour images round 5): the march keeps rows r - 2 .. r + 2 of
// Ix, Iy, Iz (of every channel) in registers and filters the five second derivatives of row r itself: a horizontal
// tap x + k is row r + k of the same lane, a vertical tap y + k row r + k of lane + k (DPP shifts); k_tv_prepd then
// writes 3 of the 8 derivative planes per channel, and a step reads 5 (colour: 11) planes instead of 10 (26).
template <int NOP, int NOC, bool DF = false>
__global__ __launch_bounds__(256) void k_tv_smsys_m(TvArgs a) {
  const int w = a.w, h = a.h, rows = smsys_rows(w, h, a.wrap);
  const int nstrip = march_strips(h), nseg = march_segments(rows);
  const long task = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // (frame, segment, strip), strip fastest
  if (task >= (long)a.n * nseg * nstrip) return;
  const int strip = (int)(task % nstrip), seg = (int)((task / nstrip) % nseg), f = (int)(task / ((long)nstrip * nseg));
  const int lane = threadIdx.x & 63;
  const int y = strip * kMC - 2 + lane;
  const bool ycol = y >= 0 && y < h;
  const bool out_lane = lane >= 2 && lane < 2 + kMC && ycol;
  const int R0 = seg * kMR, R1 = R0 + kMR < rows ? R0 + kMR : rows;
  const unsigned f0 = (unsigned)((long)f * a.sp);
  const bool first = a.first_iter != 0;
  // plane row of row r (-1: not in the plane), pixel x of (r, y) (false: no pixel)
  auto prow = [&](int r) { return a.wrap ? (r < 0 ? r + w : (r >= w ? r - w : r)) : (r < 0 || r >= rows ? -1 : r); };
  auto pix = [&](int r, int &x) {
    const int pr = prow(r);
    if (pr < 0 || !ycol) return false;
    x = pr - y;
    if (a.wrap) {
      if (x < 0) x += w;
      return true;
    }
    return x >= 0 && x < w;
  };
  struct Row {
    float wx, du, wy, dv;
  };
  auto load_row = [&](int r) {
    Row q{0.f, 0.f, 0.f, 0.f};
    const int pr = prow(r);
    if (pr >= 0 && ycol) {
      const unsigned o = f0 + (unsigned)(pr * h + y);
      q.wx = ldu(a.wxs, o);
      q.du = ldu(a.du, o);
      if (NOP == 2) {
        q.wy = ldu(a.wys, o);
        q.dv = ldu(a.dv, o);
      }
    }
    return q;
  };
  // s of row r from rows r - 1 (U0), r (U1), r + 1 (U2): tv_smooth_px's clamped neighbourhood
  auto smooth_row = [&](int r, const Row &U0, const Row &U1, const Row &U2) {
    const float uu0 = smooth_uu<NOP>(a, first, U0.wx, U0.du), uu1 = smooth_uu<NOP>(a, first, U1.wx, U1.du);
    const float uu2 = smooth_uu<NOP>(a, first, U2.wx, U2.du);
    const float uup = wave_from_prev(uu0), uun = wave_from_next(uu2);
    float vv0 = 0.f, vv1 = 0.f, vv2 = 0.f, vvp = 0.f, vvn = 0.f;
    if (NOP == 2) {
      vv0 = smooth_uu<2>(a, first, U0.wy, U0.dv);
      vv1 = smooth_uu<2>(a, first, U1.wy, U1.dv);
      vv2 = smooth_uu<2>(a, first, U2.wy, U2.dv);
      vvp = wave_from_prev(vv0);
      vvn = wave_from_next(vv2);
    }
    int x;
    if (!pix(r, x)) return 0.0f;
    const bool l = x > 0, rr = x < w - 1, u = y > 0, d = y < h - 1;
    const float uu5[5] = {uu1, l ? uu0 : uu1, rr ? uu2 : uu1, u ? uup : uu1, d ? uun : uu1};
    const float vv5[5] = {vv1, l ? vv0 : vv1, rr ? vv2 : vv1, u ? vvp : vv1, d ? vvn : vv1};
    return smooth_from_uu<NOP>(a, uu5, vv5);
  };
  struct Drow {
    float ix[NOC], iy[NOC], iz[NOC];
  };
  auto load_d = [&](int r) {  // DF: Ix, Iy, Iz of row r, every channel (0 outside the plane / the level's columns)
    Drow q;
    const int pr = prow(r);
    const bool in = pr >= 0 && ycol;
    const unsigned o = (unsigned)((long)f * NOC * a.sp + (in ? pr * h + y : 0));
#pragma unroll
    for (int ch = 0; ch < NOC; ++ch) {
      const unsigned oc = o + (unsigned)(ch * a.sp);
      q.ix[ch] = in ? ldu(a.Ix, oc) : 0.f;
      q.iy[ch] = in ? ldu(a.Iy, oc) : 0.f;
      q.iz[ch] = in ? ldu(a.Iz, oc) : 0.f;
    }
    return q;
  };
  Drow D0{}, D1{}, D2{}, D3{}, D4{};  // DF: rows r - 2 .. r + 2
  if constexpr (DF) {
    D0 = load_d(R0 - 2);
    D1 = load_d(R0 - 1);
    D2 = load_d(R0);
    D3 = load_d(R0 + 1);
  }
  Row Um = load_row(R0 - 1), U0 = load_row(R0), U1 = load_row(R0 + 1);
  float Sm = smooth_row(R0 - 1, load_row(R0 - 2), Um, U0);
  float S0 = smooth_row(R0, Um, U0, U1);
  for (int r = R0; r < R1; ++r) {
    // the derivative images of row r (issued first: in flight while s of row r + 1 is computed)
    int x;
    const bool has = pix(r, x);
    float lIx[NOC], lIy[NOC], lIz[NOC], lIxx[NOC], lIxy[NOC], lIyy[NOC], lIxz[NOC], lIyz[NOC];
    const int pr = prow(r);
    if constexpr (DF) {
      D4 = load_d(r + 2);
    } else {
      const unsigned qd = (unsigned)((long)f * NOC * a.sp + (long)(pr < 0 ? 0 : pr) * h + (ycol ? y : 0));
#pragma unroll
      for (int ch = 0; ch < NOC; ++ch) {
        const unsigned o = qd + (unsigned)(ch * a.sp);
        if (has) {
          lIx[ch] = ldu(a.Ix, o); lIy[ch] = ldu(a.Iy, o); lIz[ch] = ldu(a.Iz, o); lIxx[ch] = ldu(a.Ixx, o);
          lIxy[ch] = ldu(a.Ixy, o); lIyy[ch] = ldu(a.Iyy, o); lIxz[ch] = ldu(a.Ixz, o); lIyz[ch] = ldu(a.Iyz, o);
        } else {
          lIx[ch] = lIy[ch] = lIz[ch] = lIxx[ch] = lIxy[ch] = lIyy[ch] = lIxz[ch] = lIyz[ch] = 0.0f;
        }
      }
    }
    const Row U2 = load_row(r + 2);
    const float S1 = smooth_row(r + 1, U0, U1, U2);
    // the system of row r: s, wx, wy of the pixel and its 4-neighbourhood (centre, left, right, up, down)
    const float Sp = wave_from_prev(Sm), Sn = wave_from_next(S1);
    const float Xp = wave_from_prev(Um.wx), Xn = wave_from_next(U1.wx);
    float Yp = 0.f, Yn = 0.f;
    if (NOP == 2) {
      Yp = wave_from_prev(Um.wy);
      Yn = wave_from_next(U1.wy);
    }
    if constexpr (DF) {
      // vertical taps (x, y + k): row r + k, lane + k (every lane shifts: the DPP moves are wave-wide)
      auto vt = [&](float m2, float m1, float c, float p1, float p2, float (&t)[5]) {
        t[0] = wave_from_prev(wave_from_prev(m2));
        t[1] = wave_from_prev(m1);
        t[2] = c;
        t[3] = wave_from_next(p1);
        t[4] = wave_from_next(wave_from_next(p2));
      };
      const int xc = has ? x : 0, yc = ycol ? y : 0;  // (lanes without a pixel: any valid taps)
#pragma unroll
      for (int ch = 0; ch < NOC; ++ch) {
        float vx[5], vy[5], vz[5];
        vt(D0.ix[ch], D1.ix[ch], D2.ix[ch], D3.ix[ch], D4.ix[ch], vx);
        vt(D0.iy[ch], D1.iy[ch], D2.iy[ch], D3.iy[ch], D4.iy[ch], vy);
        vt(D0.iz[ch], D1.iz[ch], D2.iz[ch], D3.iz[ch], D4.iz[ch], vz);
        const float hx[5] = {D0.ix[ch], D1.ix[ch], D2.ix[ch], D3.ix[ch], D4.ix[ch]};
        const float hz[5] = {D0.iz[ch], D1.iz[ch], D2.iz[ch], D3.iz[ch], D4.iz[ch]};
        lIx[ch] = D2.ix[ch];
        lIy[ch] = D2.iy[ch];
        lIz[ch] = D2.iz[ch];
        lIxx[ch] = conv5_clamp(hx, xc, w);
        lIxy[ch] = conv5_clamp(vx, yc, h);
        lIyy[ch] = conv5_clamp(vy, yc, h);
        lIxz[ch] = conv5_clamp(hz, xc, w);
        lIyz[ch] = conv5_clamp(vz, yc, h);
      }
      D0 = D1;
      D1 = D2;
      D2 = D3;
      D3 = D4;
    }
    if (has && out_lane) {
      const float S5[5] = {S0, Sm, S1, Sp, Sn};
      const float X5[5] = {U0.wx, Um.wx, U1.wx, Xp, Xn};
      const float Y5[5] = {U0.wy, Um.wy, U1.wy, Yp, Yn};
      const float m = warp_mask(x, y, X5[0], Y5[0], w, h);
      float4 c0, c1;
      sys_compute<NOP, NOC>(a, x, y, S5, X5, Y5, m, U0.du, NOP == 2 ? U0.dv : 0.0f, lIx, lIy, lIz, lIxx, lIxy, lIyy,
                            lIxz, lIyz, c0, c1);
      const long idx = (long)f0 + (long)pr * h + y;
      if (NOP == 2) {
        float4 *C = reinterpret_cast<float4 *>(a.coef) + 2 * idx;
        C[0] = c0;
        C[1] = c1;
      } else {
        reinterpret_cast<float4 *>(a.coef)[idx] = c0;
      }
    }
    Um = U0;
    U0 = U1;
    U1 = U2;
    Sm = S0;
    S0 = S1;
  }
}

// The same launch on 2-D tiles of the skewed plane for tall levels (h > 256), where whole-row blocks would
// stage RB + 4 rows for RB < 4 computed ones.  A workgroup takes rows r0 .. r0+RB-1 and columns
// y0 .. y0+CB-1; its 4-neighbours lie at (r -+ 1, y) and (r -+ 1, y -+ 1), so it stages (wx, wy, du, dv) of
// rows r0-2 .. r0+RB+1 x columns y0-2 .. y0+CB+1 ((RB+4)(CB+4) for RB CB: 1.33x at 16 x 64) and s of rows
// r0-1 .. r0+RB x columns y0-1 .. y0+CB in LDS.  Against the two launches (smoothness, then system) it
// skips the s round trip and the second read of (wx, du): same functions, same bits.  blockIdx.x is the
// frame, so the tiles of a frame land on one XCD.
constexpr int kS2R = 16, kS2C = 64, kS2CS = kS2C + 4, kS2SS = kS2C + 2;
template <int NOP, int NOC>
__global__ __launch_bounds__(256) void k_tv_smsys2d(TvArgs a) {
  __shared__ float4 st[(kS2R + 4) * kS2CS];  // (wx, wy, du, dv)
  __shared__ float sl[(kS2R + 2) * kS2SS];   // s
  const int w = a.w, h = a.h, rows = smsys_rows(w, h, a.wrap);
  const int f = blockIdx.x, r0 = blockIdx.y * kS2R, y0 = blockIdx.z * kS2C;
  const long f0 = (long)f * a.sp;
  const bool first = a.first_iter != 0;
  auto prow = [&](int r) { return a.wrap ? (r < 0 ? r + w : (r >= w ? r - w : r)) : (r < 0 || r >= rows ? -1 : r); };
  auto pix = [&](int r, int y, int &x) {  // plane (row, column) -> pixel x; false outside the level
    if (r < 0 || y < 0 || y >= h) return false;
    x = r - y;
    if (a.wrap) {
      if (x < 0) x += w;
      return true;
    }
    return x >= 0 && x < w;
  };
  // ---- phase 0: stage
  for (int i = threadIdx.x; i < (kS2R + 4) * kS2CS; i += blockDim.x) {
    const int ri = i / kS2CS, y = y0 - 2 + (i - ri * kS2CS);
    const int r = prow(r0 - 2 + ri);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r >= 0 && y >= 0 && y < h) {
      const long o = f0 + (long)r * h + y;
      v.x = a.wxs[o];
      v.z = a.du[o];
      if (NOP == 2) {
        v.y = a.wys[o];
        v.w = a.dv[o];
      }
    }
    st[i] = v;
  }
  __syncthreads();
  // ---- phase 1: s of rows r0 - 1 .. r0 + RB, columns y0 - 1 .. y0 + CB
  for (int i = threadIdx.x; i < (kS2R + 2) * kS2SS; i += blockDim.x) {
    const int ri = i / kS2SS, yl = i - ri * kS2SS, y = y0 - 1 + yl;  // s (ri, yl) <-> staged (ri + 1, yl + 1)
    int x;
    float sv = 0.0f;
    if (pix(prow(r0 - 1 + ri), y, x)) {
      const int c = (ri + 1) * kS2CS + yl + 1;
      const int cl = x > 0 ? c - kS2CS : c, cr = x < w - 1 ? c + kS2CS : c;
      const int cu = y > 0 ? c - kS2CS - 1 : c, cd = y < h - 1 ? c + kS2CS + 1 : c;
      const float4 q0 = st[c], q1 = st[cl], q2 = st[cr], q3 = st[cu], q4 = st[cd];
      const float wx5[5] = {q0.x, q1.x, q2.x, q3.x, q4.x}, du5[5] = {q0.z, q1.z, q2.z, q3.z, q4.z};
      const float wy5[5] = {q0.y, q1.y, q2.y, q3.y, q4.y}, dv5[5] = {q0.w, q1.w, q2.w, q3.w, q4.w};
      sv = smooth_compute<NOP>(a, first, wx5, du5, wy5, dv5);
    }
    sl[i] = sv;
  }
  __syncthreads();
  // ---- phase 2: the system of rows r0 .. r0 + RB - 1, columns y0 .. y0 + CB - 1
  for (int i = threadIdx.x; i < kS2R * kS2C; i += blockDim.x) {
    const int ri = i / kS2C, yl = i - ri * kS2C, y = y0 + yl;
    const int rr = r0 + ri;
    int x;
    if (rr >= rows || !pix(rr, y, x)) continue;
    const int c = (ri + 1) * kS2SS + yl + 1, cs = (ri + 2) * kS2CS + yl + 2;  // s index, staged index
    const int yu = y > 0 ? -1 : 0, yd = y < h - 1 ? 1 : 0;  // clamped columns; absent neighbours are discarded
    const int s5[5] = {c, c - kS2SS, c + kS2SS, c - kS2SS + yu, c + kS2SS + yd};
    const int t5[5] = {cs, cs - kS2CS, cs + kS2CS, cs - kS2CS + yu, cs + kS2CS + yd};
    float S5[5], X5[5], Y5[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      S5[k] = sl[s5[k]];
      const float4 q = st[t5[k]];
      X5[k] = q.x;
      Y5[k] = NOP == 2 ? q.y : 0.0f;
    }
    const float4 qc = st[cs];
    const long idx = f0 + (long)rr * h + y;
    const float m = warp_mask(x, y, X5[0], Y5[0], w, h);
    const unsigned qd = (unsigned)((long)f * NOC * a.sp + (long)rr * h + y);
    float lIx[NOC], lIy[NOC], lIz[NOC], lIxx[NOC], lIxy[NOC], lIyy[NOC], lIxz[NOC], lIyz[NOC];
#pragma unroll
    for (int ch = 0; ch < NOC; ++ch) {
      const unsigned o = qd + (unsigned)(ch * a.sp);
      lIx[ch] = ldu(a.Ix, o); lIy[ch] = ldu(a.Iy, o); lIz[ch] = ldu(a.Iz, o); lIxx[ch] = ldu(a.Ixx, o);
      lIxy[ch] = ldu(a.Ixy, o); lIyy[ch] = ldu(a.Iyy, o); lIxz[ch] = ldu(a.Ixz, o); lIyz[ch] = ldu(a.Iyz, o);
    }
    float4 c0, c1;
    sys_compute<NOP, NOC>(a, x, y, S5, X5, Y5, m, qc.z, NOP == 2 ? qc.w : 0.0f, lIx, lIy, lIz, lIxx, lIxy, lIyy,
                          lIxz, lIyz, c0, c1);
    if (NOP == 2) {
      float4 *C = reinterpret_cast<float4 *>(a.coef) + 2 * idx;
      C[0] = c0;
      C[1] = c1;
    } else {
      reinterpret_cast<float4 *>(a.coef)[idx] = c0;
    }
  }
}

// Generic exact-order SOR (any size / sweep count): one workgroup per frame, in-place skewed arrays in
// global memory, one barrier per wavefront step.  Pixel (x, y) of sweep s runs at step t = x + y + 2 s:
// its left/top neighbours of the same sweep ran at t-1, its right/bottom neighbours of the previous
// sweep at t-1, and no two pixels of one step touch each other (parity), so this reproduces
// solver.c's raster order bit for bit.  MODE 0: sor_coupled (solver.c:83-433); 1: its point-SOR
// fallback for width < 2 or height < 2 (solver.c:34-78); 2: sor_coupled_slow_but_readable_DE (:439-471).
template <int MODE>
__global__ __launch_bounds__(256) void k_tv_sor(TvArgs a) {
  const int f = blockIdx.x;
  const int w = a.w, h = a.h, S = a.solverit;
  const long fo = (long)f * a.sp;
  float *du = a.du + fo, *dv = a.dv + fo;
  float4 *C = reinterpret_cast<float4 *>(a.coef) + fo * (MODE == 2 ? 1 : 2);
  // AoS accessors: OF (a11, a12, a12, a22) (b1, b2, sh, sv); DE (a11, b1, sh, sv)
#define SH_(o) (MODE == 2 ? C[o].z : C[2 * (o) + 1].z)
#define SV_(o) (MODE == 2 ? C[o].w : C[2 * (o) + 1].w)
  const float omega = a.omega;
  const int items = S * h;
  const int T = (w - 1) + (h - 1) + 2 * (S - 1) + 1;
  for (int t = 0; t < T; ++t) {
    for (int k = threadIdx.x; k < items; k += blockDim.x) {
      const int s = k / h, y = k - s * h;
      const int x = t - y - 2 * s;
      if (x < 0 || x >= w) continue;
      const long o = skw(x, y, h, w, a.wrap);
      // neighbours (clamped coordinates: only read when they exist)
      const long oL = skw(x > 0 ? x - 1 : x, y, h, w, a.wrap), oR = skw(x < w - 1 ? x + 1 : x, y, h, w, a.wrap);
      const long oU = skw(x, y > 0 ? y - 1 : y, h, w, a.wrap), oD = skw(x, y < h - 1 ? y + 1 : y, h, w, a.wrap);
      if (MODE == 0) {
        const float4 c0 = C[2 * o];
        const float4 c1 = C[2 * o + 1];
        const float b1 = c1.x, b2 = c1.y, hr = c1.z, vo = c1.w;
        const float hl = x > 0 ? SH_(oL) : 0.0f;
        const float ur = x < w - 1 ? du[oR] : 0.0f, vr = x < w - 1 ? dv[oR] : 0.0f;
        float s1, s2;
        if (y == 0) {
          s1 = (b1 + hr * ur) + vo * du[oD];
          s2 = (b2 + hr * vr) + vo * dv[oD];
        } else if (y < h - 1) {
          const float vt = SV_(oU);
          s1 = ((hr * ur) + vt * du[oU]) + (b1 + vo * du[oD]);
          s2 = ((hr * vr) + vt * dv[oU]) + (b2 + vo * dv[oD]);
        } else {
          const float vt = SV_(oU);
          s1 = (b1 + hr * ur) + vt * du[oU];
          s2 = (b2 + hr * vr) + vt * dv[oU];
        }
        const float i11 = c0.x, i12 = c0.y, i22 = c0.w;  // inverse precomputed by k_tv_system
        float B1 = s1, B2 = s2;
        if (x > 0) {
          B1 = hl * du[oL] + s1;
          B2 = hl * dv[oL] + s2;
        }
        const float u0 = du[o], v0 = dv[o];
        du[o] = u0 + omega * (i11 * B1 + i12 * B2 - u0);
        dv[o] = v0 + omega * (i12 * B1 + i22 * B2 - v0);
      } else if (MODE == 1) {
        const float4 c0 = C[2 * o], c1 = C[2 * o + 1];
        float su = 0.0f, sv = 0.0f, sd = 0.0f;
        if (y > 0) { const float q = SV_(oU); su -= q * du[oU]; sv -= q * dv[oU]; sd += q; }
        if (x > 0) { const float q = SH_(oL); su -= q * du[oL]; sv -= q * dv[oL]; sd += q; }
        if (y < h - 1) { su -= c1.w * du[oD]; sv -= c1.w * dv[oD]; sd += c1.w; }
        if (x < w - 1) { su -= c1.z * du[oR]; sv -= c1.z * dv[oR]; sd += c1.z; }
        const float A11 = c0.x + sd, A12 = c0.y, A22 = c0.w + sd;
        const float B1 = c1.x - su, B2 = c1.y - sv;
        du[o] = (1.0f - omega) * du[o] + omega / A11 * (B1 - A12 * dv[o]);
        dv[o] = (1.0f - omega) * dv[o] + omega / A22 * (B2 - A12 * du[o]);
      } else {
        const float4 c0 = C[o];
        float su = 0.0f;  // (c0.x = a11 + the diffusivities: sys_compute)
        if (y > 0) { const float q = SV_(oU); su -= q * du[oU]; }
        if (x > 0) { const float q = SH_(oL); su -= q * du[oL]; }
        if (y < h - 1) { su -= c0.w * du[oD]; }
        if (x < w - 1) { su -= c0.z * du[oR]; }
        const float A11 = c0.x, B1 = c0.y - su;
        du[o] = (1.0f - omega) * du[o] + omega * (B1 / A11);
      }
    }
    __syncthreads();
  }
#undef SH_
#undef SV_
}


#ifdef OFDIS_SOR_PROBE
// Step-timing probe of the sweep-per-wave SOR (a separate build, tools/sor_probe.py; never in libofdis.so):
// frame 0 of every launch records, per wave and wavefront step, the shader clock (s_memtime) after the
// previous step's barrier, after the step's LDS reads have arrived, after its update is written to LDS, and
// after the step's barrier.  Layout: [0] launch counter, then [launch < 64][wave < 16][step < 1024][4].
__device__ unsigned *g_sor_probe;
__device__ __forceinline__ unsigned probe_clock() { return (unsigned)__builtin_amdgcn_s_memtime(); }
#endif

// Per-pixel data that sweep 0 loads / derives and sweeps 1..S-1 reuse 2s steps later (register ring).
struct SorPix {
  float i11, i12, i22, b1, b2, hl, hr, vv, vt;
};

// ---------------------------------------------------------------------------------- red-black SOR (opt-in)
// The throughput mode of SURVEY §7 4(ii): the same per-pixel block SOR update as sor_coupled (2x2 inverse
// precomputed by the system kernel, solver.c's right-hand-side trees via sor_rhs) but in red-black order --
// all pixels with x + y even, then all odd ones, 2 * solverit half-sweeps -- instead of the lexicographic
// order, so every half-sweep is fully parallel.  A different iteration: results are NOT the reference's bits;
// the parity gate is an end-point tolerance against the exact path, and bit-exactness against the oracle's
// red-black restatement (ofo_sor_rb_*; tests/test_gpu_redblack.py).  MODE 0: OF block SOR, 2: DE point SOR.
// Levels of at most kLvPix pixels run the whole inner loop in one launch (k_tv_level_rb, ofdis_tvrb.hip); the
// larger ones run the system kernels and these global-memory half-sweeps, one launch each.
template <int MODE>
__device__ __forceinline__ RbPix rb_load(const TvArgs &a, int f, int x, int y) {
  const float4 *C = reinterpret_cast<const float4 *>(a.coef);
  const long fo = (long)f * a.sp;
  const long o = fo + skw(x, y, a.h, a.w, a.wrap);
  RbPix d;
  if (MODE == 0) {
    const float4 c0 = C[2 * o], c1 = C[2 * o + 1];
    d.i11 = c0.x; d.i12 = c0.y; d.i22 = c0.w; d.b1 = c1.x; d.b2 = c1.y; d.hr = c1.z; d.vb = c1.w;
    d.hl = x > 0 ? C[2 * (fo + skw(x - 1, y, a.h, a.w, a.wrap)) + 1].z : 0.0f;
    d.vt = y > 0 ? C[2 * (fo + skw(x, y - 1, a.h, a.w, a.wrap)) + 1].w : 0.0f;
  } else {
    const float4 c0 = C[o];
    d.i11 = c0.x; d.i12 = 0.0f; d.i22 = 0.0f; d.b1 = c0.y; d.b2 = 0.0f; d.hr = c0.z; d.vb = c0.w;
    d.hl = x > 0 ? C[fo + skw(x - 1, y, a.h, a.w, a.wrap)].z : 0.0f;
    d.vt = y > 0 ? C[fo + skw(x, y - 1, a.h, a.w, a.wrap)].w : 0.0f;
  }
  return d;
}
// One half-sweep of one colour over global memory (larger levels): thread = pixel.
template <int MODE>
__global__ __launch_bounds__(256) void k_tv_sor_rb(TvArgs a, int color) {
  const int p = blockIdx.x * 256 + threadIdx.x, f = blockIdx.y, w = a.w, h = a.h;
  if (p >= w * h) return;
  const int x = p % w, y = p / w;
  if (((x + y) & 1) != color) return;
  const long fo = (long)f * a.sp;
  const RbPix d = rb_load<MODE>(a, f, x, y);
  auto at = [&](int xx, int yy) { return fo + skw(xx, yy, h, w, a.wrap); };
  const long o = at(x, y);
  const float ul = x > 0 ? a.du[at(x - 1, y)] : 0.0f, ur = x < w - 1 ? a.du[at(x + 1, y)] : 0.0f;
  const float ut = y > 0 ? a.du[at(x, y - 1)] : 0.0f, ub = y < h - 1 ? a.du[at(x, y + 1)] : 0.0f;
  float vl = 0.0f, vr = 0.0f, vt = 0.0f, vb = 0.0f, v = 0.0f;
  if (MODE == 0) {
    vl = x > 0 ? a.dv[at(x - 1, y)] : 0.0f; vr = x < w - 1 ? a.dv[at(x + 1, y)] : 0.0f;
    vt = y > 0 ? a.dv[at(x, y - 1)] : 0.0f; vb = y < h - 1 ? a.dv[at(x, y + 1)] : 0.0f;
    v = a.dv[o];
  }
  float u = a.du[o];
  rb_update<MODE>(d, x, y, w, h, a.omega, ul, ur, ut, ub, vl, vr, vt, vb, u, v);
  a.du[o] = u;
  if (MODE == 0) a.dv[o] = v;
}

// Register-pipelined exact-order SOR: thread = row y (h <= 1024), one workgroup per frame.  At step t the
// thread runs sweep s on pixel x_s = t - y - 2 s for every s < S.  Left/right/own values come from its own
// registers (results of steps t-1 / t-2), top/bottom values from the neighbouring lanes by DPP (through LDS
// across wave boundaries), coefficients from the skewed array-of-structs (two 16-byte loads per step,
// issued two steps ahead).  The step loop is unrolled by U = lcm(2, 2(S-1)) so that the load buffers, the
// per-step history and the sweep ring are all indexed by compile-time phase: no register copies.  Every
// per-lane condition (borders, inactive lanes) is a select, never a branch: one instruction stream per wave.
// Same arithmetic, same order as k_tv_sor -> bit-identical results.  MODE 0: OF block SOR, 2: DE point SOR.
template <int S, int MODE>
struct SorPipe {
  static constexpr int D = S > 1 ? 2 * (S - 1) : 1;          // sweep ring depth
  static constexpr int U = S > 1 ? D : 2;  // unroll = lcm(2, D); D = 2(S-1) is even
  static constexpr int NV = 2 * S + 1;
  static constexpr int NV4 = (NV + 3) / 4;                   // float4s per published record
  struct Ld {
    float4 c0, c1;   // AoS coefficients: OF (a11, a12, a22, b1), (b2, sh, sv, -); DE (a11, b1, sh, sv)
    float ru, rv, bu, bv;
  };
  // state
  float hu[2][S], hv[2][S];   // sweep results of the last step of each parity
  float own_u[2], own_v[2];   // "right" initial values loaded at a step of each parity
  float hsh[2], hsv[2];       // sh / sv loaded at a step of each parity
  SorPix ring[D];
  Ld L[2];
  // constants
  const float4 *C;
  float *du, *dv;
  float4 (*xtop)[16][NV4], (*xbot)[16][NV4];
  int w, h, y, lane, wv, nw, wrap;
  unsigned dump;
  float omega;
  bool has_top, has_bot, border, notop, get_top, get_bot;

  __device__ __forceinline__ void load(int t, Ld &B) {
    const int x0 = t - y;
    const bool in = y < h && x0 >= 0 && x0 < w;
    const unsigned here = (unsigned)(skrow(t, w, wrap) * h + y);
    const unsigned next = (unsigned)(skrow(t + 1, w, wrap) * h + y);  // row of diagonal t + 1
    const unsigned o = in ? here : dump;
    if (MODE == 0) {
      B.c0 = C[2 * o];
      B.c1 = C[2 * o + 1];
    } else {
      B.c0 = C[o];
    }
    const unsigned ob = in && has_bot ? next + 1 : dump;
    B.bu = du[ob];
    if (MODE == 0) B.bv = dv[ob];
    const unsigned orr = y < h && x0 + 1 >= 0 && x0 + 1 < w ? next : dump;
    B.ru = du[orr];
    if (MODE == 0) B.rv = dv[orr];
  }

  template <int PH>
  __device__ __forceinline__ void step(const int t) {
    constexpr int q = PH & 1, qp = q ^ 1;
    Ld &B = L[q];
    // consume this step's prefetched values, then reuse the buffer for step t + 2
    float c11, c12 = 0, c22 = 0, cb1, cb2 = 0, csh, csv;
    if (MODE == 0) {
      c11 = B.c0.x; c12 = B.c0.y; c22 = B.c0.w; cb1 = B.c1.x; cb2 = B.c1.y; csh = B.c1.z; csv = B.c1.w;
    } else {
      c11 = B.c0.x; cb1 = B.c0.y; csh = B.c0.z; csv = B.c0.w;
    }
    const float cru = B.ru, crv = B.rv, cbu = B.bu, cbv = B.bv;
    load(t + 2, B);
    // neighbour values from the previous step
    float tu[S], tv[S], bu[S], bv[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      tu[s] = dpp_from_prev_lane(hu[qp][s]);
      bu[s] = dpp_from_next_lane(hu[qp][s]);
      if (MODE == 0) {
        tv[s] = dpp_from_prev_lane(hv[qp][s]);
        bv[s] = dpp_from_next_lane(hv[qp][s]);
      } else {
        tv[s] = bv[s] = 0.0f;
      }
    }
    float svt = dpp_from_prev_lane(hsv[qp]);
    if (nw > 1 && t > 0) {  // wave-boundary lanes take the neighbouring wave's values (uniform LDS reads)
      const int par = (t & 1) ^ 1;
      float xt[4 * NV4], xb[4 * NV4];
#pragma unroll
      for (int k = 0; k < NV4; ++k) {
        const float4 a4 = xtop[par][wv > 0 ? wv - 1 : 0][k], b4 = xbot[par][wv < nw - 1 ? wv + 1 : wv][k];
        xt[4 * k] = a4.x; xt[4 * k + 1] = a4.y; xt[4 * k + 2] = a4.z; xt[4 * k + 3] = a4.w;
        xb[4 * k] = b4.x; xb[4 * k + 1] = b4.y; xb[4 * k + 2] = b4.z; xb[4 * k + 3] = b4.w;
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        tu[s] = get_top ? xt[s] : tu[s];
        bu[s] = get_bot ? xb[s] : bu[s];
        if (MODE == 0) {
          tv[s] = get_top ? xt[S + s] : tv[s];
          bv[s] = get_bot ? xb[S + s] : bv[s];
        }
      }
      svt = get_top ? xt[2 * S] : svt;
    }
    float nu[S], nvv[S];
    const int x0 = t - y;
    const float own_u0 = own_u[qp], own_v0 = own_v[qp];
    // ---- sweep 0 on pixel x0.  Its data goes to the ring slot of age 0 only after sweeps 1..S-1 have read theirs: the oldest one (age D) lives in that same slot.
    SorPix d;
    d.b1 = cb1; d.b2 = cb2; d.hr = csh; d.hl = x0 > 0 ? hsh[qp] : 0.0f; d.vv = csv; d.vt = has_top ? svt : 0.0f;
    {
      const float ur = x0 < w - 1 ? cru : 0.0f, vr = x0 < w - 1 ? crv : 0.0f;
      if (MODE == 0) {
        const float s1 = sor_rhs(border, notop, d.b1, d.hr * ur, d.vt * tu[0], d.vv * cbu);
        const float s2 = sor_rhs(border, notop, d.b2, d.hr * vr, d.vt * tv[0], d.vv * cbv);
        d.i11 = c11;  // inverse precomputed by k_tv_system (solver.c:122-128)
        d.i12 = c12;
        d.i22 = c22;
        const float B1 = x0 > 0 ? d.hl * hu[qp][0] + s1 : s1;
        const float B2 = x0 > 0 ? d.hl * hv[qp][0] + s2 : s2;
        nu[0] = own_u0 + omega * (d.i11 * B1 + d.i12 * B2 - own_u0);
        nvv[0] = own_v0 + omega * (d.i12 * B1 + d.i22 * B2 - own_v0);
      } else {
        d.i11 = c11;
        float su = 0.0f;  // (c11 = a11 + the diffusivities: sys_compute)
        su = has_top ? su - d.vt * tu[0] : su;
        su = x0 > 0 ? su - d.hl * hu[qp][0] : su;
        su = has_bot ? su - d.vv * cbu : su;
        su = x0 < w - 1 ? su - d.hr * ur : su;
        const float A = c11, Bv = d.b1 - su;
        nu[0] = (1.0f - omega) * own_u0 + omega * (Bv / A);
        nvv[0] = 0.0f;
      }
    }
    // ---- sweeps 1..S-1 on pixel x0 - 2 s with the data sweep 0 saw 2 s steps ago
#pragma unroll
    for (int s = 1; s < S; ++s) {
      const SorPix &e = ring[(PH + 2 * D - 2 * s) % D];
      const int xs = x0 - 2 * s;
      const float ou = hu[q][s - 1], ov = hv[q][s - 1];          // own value after sweep s-1 (step t-2)
      const float ur = xs < w - 1 ? hu[qp][s - 1] : 0.0f;        // right neighbour after sweep s-1
      const float vr = xs < w - 1 ? hv[qp][s - 1] : 0.0f;
      if (MODE == 0) {
        const float s1 = sor_rhs(border, notop, e.b1, e.hr * ur, e.vt * tu[s], e.vv * bu[s - 1]);
        const float s2 = sor_rhs(border, notop, e.b2, e.hr * vr, e.vt * tv[s], e.vv * bv[s - 1]);
        const float B1 = xs > 0 ? e.hl * hu[qp][s] + s1 : s1;
        const float B2 = xs > 0 ? e.hl * hv[qp][s] + s2 : s2;
        nu[s] = ou + omega * (e.i11 * B1 + e.i12 * B2 - ou);
        nvv[s] = ov + omega * (e.i12 * B1 + e.i22 * B2 - ov);
      } else {
        float su = 0.0f;
        su = has_top ? su - e.vt * tu[s] : su;
        su = xs > 0 ? su - e.hl * hu[qp][s] : su;
        su = has_bot ? su - e.vv * bu[s - 1] : su;
        su = xs < w - 1 ? su - e.hr * ur : su;
        const float A = e.i11, Bv = e.b1 - su;
        nu[s] = (1.0f - omega) * ou + omega * (Bv / A);
        nvv[s] = 0.0f;
      }
    }
    if (S > 1) ring[PH % D] = d;
    // ---- the last sweep's result is final (unconditional store: inactive lanes hit the dump slots)
    {
      const int xl = x0 - 2 * (S - 1);
      const unsigned o = y < h && xl >= 0 && xl < w ? (unsigned)(skrow(t - 2 * (S - 1), w, wrap) * h + y) : dump;
      du[o] = nu[S - 1];
      if (MODE == 0) dv[o] = nvv[S - 1];
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      hu[q][s] = nu[s];
      hv[q][s] = nvv[s];
    }
    own_u[q] = cru;
    own_v[q] = crv;
    hsh[q] = csh;
    hsv[q] = csv;
    // ---- publish wave-boundary values, one barrier per step
    if (nw > 1) {
      const int par = t & 1;
      float rec[4 * NV4];
#pragma unroll
      for (int s = 0; s < S; ++s) { rec[s] = nu[s]; rec[S + s] = nvv[s]; }
      rec[2 * S] = csv;
#pragma unroll
      for (int k = 2 * S + 1; k < 4 * NV4; ++k) rec[k] = 0.0f;
      if (lane == 63) {
#pragma unroll
        for (int k = 0; k < NV4; ++k) xtop[par][wv][k] = make_float4(rec[4 * k], rec[4 * k + 1], rec[4 * k + 2], rec[4 * k + 3]);
      }
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NV4; ++k) xbot[par][wv][k] = make_float4(rec[4 * k], rec[4 * k + 1], rec[4 * k + 2], rec[4 * k + 3]);
      }
      __syncthreads();
    }
  }

  template <int PH>
  __device__ __forceinline__ void steps(const int t) {
    step<PH>(t + PH);
    if constexpr (PH + 1 < U) steps<PH + 1>(t);
  }
};

// MAXT = launch bound: 256 (one wave per SIMD, up to 512 registers) for h <= 256, 512 for h <= 512 (the
// S <= 4 rings fit without spilling in both), 1024 for taller levels.
template <int S, int MODE, int MAXT>
__global__ __launch_bounds__(MAXT) void k_tv_sor_pipe(TvArgs a) {
  using P = SorPipe<S, MODE>;
  __shared__ float4 xtop[2][16][P::NV4];  // published by each wave's lane 63: results of the step, sv
  __shared__ float4 xbot[2][16][P::NV4];  // published by each wave's lane 0
  P st;
  const int f = blockIdx.x;
  st.w = a.w;
  st.h = a.h;
  st.y = threadIdx.x;
  st.lane = st.y & 63;
  st.wv = st.y >> 6;
  st.nw = (int)(blockDim.x >> 6);
  const long fo = (long)f * a.sp;
  st.du = a.du + fo;
  st.dv = a.dv + fo;
  st.C = reinterpret_cast<const float4 *>(a.coef) + fo * (MODE == 0 ? 2 : 1);
  st.xtop = xtop;
  st.xbot = xbot;
  st.omega = a.omega;
  st.has_top = st.y > 0;
  st.has_bot = st.y < a.h - 1;
  st.notop = !st.has_top;
  st.border = !st.has_top || !st.has_bot;
  st.get_top = st.lane == 0 && st.wv > 0;
  st.get_bot = st.lane == 63 && st.wv < st.nw - 1;
  st.wrap = a.wrap;
  st.dump = (unsigned)(a.skew_slots + st.lane);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
#pragma unroll
    for (int s = 0; s < S; ++s) st.hu[q][s] = st.hv[q][s] = 0.0f;
    st.own_u[q] = st.own_v[q] = st.hsh[q] = st.hsv[q] = 0.0f;
  }
  if (st.y == 0 && a.w > 0) {  // row 0 starts at step 0: its first own value has no previous-step load
    st.own_u[1] = st.du[0];
    if (MODE == 0) st.own_v[1] = st.dv[0];
  }
  const int T = (a.w - 1) + (a.h - 1) + 2 * (S - 1) + 1;
  // steps t >= T are past the right border for every lane and sweep (dump-slot traffic only)
  const int TU = (T + P::U - 1) / P::U * P::U;
  st.load(0, st.L[0]);
  st.load(1, st.L[1]);
  for (int t = 0; t < TU; t += P::U) st.template steps<0>(t);
}

// Skewed row of anti-diagonal d for a wave-uniform d (SALU only).  Diagonals outside the frame map to a row
// inside the plane: every lane reading it is outside the frame (its value is never used), and with the
// 64 dump slots after the rows even lanes beyond h stay inside the plane.
// The layout is folded into two wave-uniform constants (branch-free SALU): lim = w (wrapped) or a value
// above every d (unwrapped), rmax = the last row of the plane.
__device__ __forceinline__ int sor_row2(int d, int lim, int rmax) {
  const int dd = max(d, 0);
  return min(dd >= lim ? dd - lim : dd, rmax);
}


// Sweep-per-wave exact-order SOR, one row per lane.  Same wavefront as SorPipe (pixel (x, y) of sweep s at
// step t = x + y + 2 s), but the S sweeps run on S different waves of the workgroup: wave (g, s) owns rows
// 64 g .. 64 g + 63 of sweep s.  Per step every wave computes ONE pixel per lane and publishes its values
// in LDS rings of depth 3 (steps t, t-1, t-2); the wave of sweep s+1 reads its own / right / bottom "old"
// values there, every wave reads its top neighbour there, and its left neighbour is its own result of
// step t-1.  Sweep 0 reads the old values from global memory (the previous SOR call's, never yet
// overwritten: the last sweep writes pixel (x, y) at step x + y + 2 (S-1) > every read of it).  One
// barrier per step.  Arithmetic and order as SorPipe: bit-identical.  MODE 0: OF block SOR (2x2 inverse
// precomputed), 2: DE point SOR.  The form is lean:
//  * addresses are a wave-uniform base (SALU: skewed row of the step's diagonal) plus a per-lane constant:
//    no per-step vector address arithmetic; lanes outside the frame read real plane slots (sor_row) and
//    only the stores are masked;
//  * coefficients are multi-buffered (NB buffers, prefetch distance NB - 1 into the buffer of step t-1);
//    sweep 0's right neighbour is the next step's own value (one load fewer);
//  * the LDS rings hold (u, v) as float2 [row][slot] (24-B lane stride) and sv as float [row][slot]
//    (12-B stride): conflict-free ds_read_b64 / ds_write_b64 / b32, slots a compile-time phase of the
//    unrolled block -> immediate offsets.  (Loading the upper pixel's sv from the coefficients instead
//    measured 40 % slower with 4 frames per CU: the per-sweep coefficient re-reads already load the
//    vector memory path, the LDS much less);
//  * (u, v) pairs run on packed fp32 (v_pk_mul_f32 / v_pk_add_f32: the same roundings as scalar, no FMA);
//  * a wave whose rows are all outside the frame for a whole block only joins the block's barriers.
// SI: sweep index.  CRN > 0: coefficient ring of CRN entries per slot -- sweep 0 loads each pixel's
// coefficients once and passes them to the later sweeps through LDS (slot = diagonal mod 6: a diagonal
// lives from sweep 0's step to sweep S-1's, 2 (S - 1) + 1 <= 6 steps for S <= 3), which also supplies the
// upper pixel's sv; CRN = 0: every sweep loads its own coefficients and keeps an sv ring.
// R: rows per lane.  Wave (g, s) owns rows 64 R g .. 64 R g + 64 R - 1; lane i runs rows y + 64 r (r < R), one
// pixel each per step -- the rows of one step are independent (their top neighbours ran at step t-1 and are in
// the ring), so R = 2 runs levels of up to 640 rows with S <= 3 in 16 waves (E's 544-row level) where R = 1
// would need 27.  Every per-row ring / coefficient-ring offset is a compile-time multiple of 64 entries.
// SEL: load form of the lanes outside the frame (see load()).
template <int S, int MODE, int SI, int NB, int CRN, int R = 1, bool SEL = false>
struct SorLane {
  static constexpr bool FIRST = SI == 0, LAST = SI == S - 1;
  static_assert(CRN == 0 || S <= 3, "coefficient ring depth 6 needs S <= 3");
  static constexpr int PD = NB - 1;                                    // prefetch distance (steps)
  static constexpr int U = NB % 3 == 0 ? (NB < 6 ? 6 : NB) : 3 * NB;  // multiple of 3 (ring) and NB
  static constexpr int CW = MODE == 0 ? 2 : 1;                         // float4s of coefficients per pixel
  struct Ld {
    float4 c0[R], c1[R];
    f2v o[R], b[R];  // sweep 0: old (u, v) of the pixel and of the one below (the right one: next step's o)
  };
  Ld L0, L1, L2, L3, L4, L5;  // buffers as named members (no array: keeps them in registers)
  template <int I>
  __device__ __forceinline__ Ld &buf() {
    static_assert(I < NB && NB <= 6, "buffer index");
    if constexpr (I == 0) return L0;
    else if constexpr (I == 1) return L1;
    else if constexpr (I == 2) return L2;
    else if constexpr (I == 3) return L3;
    else if constexpr (I == 4) return L4;
    else return L5;
  }
  f2v pp[R];      // own (u, v) of step t-1 (left neighbour)
  float phr[R];   // own sh of step t-1 (left neighbour's sh)
  float pvv[R];   // own sv of step t-1 (the lower pixel's upper sv)
  f2v prv[R];     // previous sweep's (u, v) of this row at step t-2: the right neighbour read at step t-1
  // DPT: the upper neighbour's (u, v) and sv come from lane y-1's registers (DPP) instead of the LDS rings;
  // only lane 0 of a row group below the first reads them there (the row above is another wave's)
  static constexpr bool DPT = R == 1;
  bool top_lds;   // DPT: this lane reads its upper neighbour from LDS (lane 0, row group > 0)
  const float4 *C;
  const float *du_r, *dv_r;
  float *du, *dv;
  f2v *ring_s;        // [NR][3] this sweep, lane base = entry y + 1 (entry 0 = row -1 stays zero)
  const f2v *ring_p;  // [NR][3] previous sweep
  float *sv_s;        // [NR][3] this sweep's sv (row y's sv at entry y + 1) (CRN = 0)
  // coefficient ring (CRN > 0), lane base = entry y + 1, slot = diagonal mod 6: [6][CW][CRN] float4.  (Round 4's
  // 28-byte entries for throughput launches -- more frames per CU -- were removed in round 6: with the clamped load
  // form the 32-byte ring runs B's launches 4 % faster and fetches 7 % (A: 30 %) fewer bytes, profiles/r06/s21.)
  float4 *cr;
  int w, h, y, s, lim, rmax, hplane;
  unsigned yc[R];  // !SEL load slot: row y + 64 r clamped into the frame (lanes past h read row h - 1: in the plane)
  bool border[R], notop[R];
  float omega;
#ifdef OFDIS_SOR_PROBE
  unsigned *probe = nullptr;  // this wave's [step][4] records (frame 0 only)
#endif

  __device__ __forceinline__ void load(int t, Ld &B) {
    const int d = t - 2 * s;
    const unsigned r0 = (unsigned)sor_row2(d, lim, rmax) * (unsigned)hplane;
    const unsigned r1 = FIRST ? (unsigned)sor_row2(d + 1, lim, rmax) * (unsigned)hplane : 0u;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      // SEL (launches with more frames than the chip holds at once): a plane row holds h slots, of which the folded
      // layout gives the ones outside the wave's in-frame run to diagonal d -+ w, so lane-constant slots fetch every
      // slot (w + h + 2S - 3) / w ~ 1.6 times per call at B's levels (the PMC fetch excess).  Here
      // the lane's row is clamped into the run [max(d - w + 1, 0), min(d, h - 1)] (bounds in SALU, one v_med3 per
      // lane): a lane outside the frame reads a slot an in-frame lane of its wave reads, so the wave fetches the lines
      // of its run only; every use of such a lane's values is discarded by a select.  (Round 4's form selected the
      // row's first slot: compare, compare, select per load.  An exec-masked load costs the prefetch: the wait-count
      // pass waits for it at the join, tv_sor 135 -> 166 us per launch.)  !SEL (launches whose frames all fit the
      // chip -- the latency regime): the lane-constant slot, no per-step vector address arithmetic at all.
      unsigned yr = yc[r];
      if (SEL) {
        const int lo = min(max(d - w + 1, 0), h - 1), hi = max(min(d, h - 1), 0);
        yr = (unsigned)min(max(y + 64 * r, lo), hi);
      }
      if (FIRST || CRN == 0) {
        const float4 *cp = C + (size_t)r0 * CW;
        B.c0[r] = cp[yr * CW];
        if (MODE == 0) B.c1[r] = cp[yr * CW + 1];
      }
      if (FIRST) {
        const float *u0 = du_r + r0, *u1 = du_r + r1;
        float ov = 0.0f, bv = 0.0f;
        if (MODE == 0) {
          const float *v0 = dv_r + r0, *v1 = dv_r + r1;
          ov = v0[yr];
          bv = v1[yr + 1];
        }
        B.o[r] = f2v{u0[yr], ov};
        B.b[r] = f2v{u1[yr + 1], bv};
      }
    }
  }

  template <int Q>
  __device__ __forceinline__ void step(const int t) {
    constexpr int m0 = Q % 3, m1 = (Q + 2) % 3;  // ring slots of steps t, t-1
#ifdef OFDIS_SOR_PROBE
    const unsigned pt0 = probe_clock();
    unsigned pt1 = 0, pt2 = 0;
#endif
    Ld &B = buf<Q % NB>();
    const Ld &Bn = buf<(Q + 1) % NB>();
    load(t + PD, buf<(Q + PD) % NB>());  // beyond the last step too: sor_row keeps every address in the plane
    const int d = t - 2 * s;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      constexpr int RO = 64 * 3;  // ring entries of the row 64 below, in f2v / float
      const int yr = y + 64 * r;
      const int xp = d - yr;
      const bool hasl = xp > 0, hasr = xp < w - 1;
      f2v o, rgt, bt;
      if (FIRST) {
        o = B.o[r]; rgt = Bn.o[r]; bt = B.b[r];
      } else {  // own value after the previous sweep (step t-2) = the right neighbour read at step t-1
        o = prv[r]; rgt = ring_p[r * RO + m1]; bt = ring_p[r * RO + 3 + m1];
        prv[r] = rgt;
      }
      // coefficients of this pixel and sv of the one above (entry 0, row -1, stays zero)
      constexpr int cs = ((Q - 2 * SI) % 6 + 6) % 6, ct = (cs + 5) % 6;  // slots of diagonals d, d - 1
      float4 c0, c1;
      if (CRN > 0) {
        if (FIRST) {
          c0 = B.c0[r];
          c1 = MODE == 0 ? B.c1[r] : B.c0[r];
          cr[cs * CW * CRN + 64 * r] = c0;
          if (MODE == 0) cr[(cs * CW + 1) * CRN + 64 * r] = c1;
        } else {
          c0 = cr[cs * CW * CRN + 64 * r];
          c1 = MODE == 0 ? cr[(cs * CW + 1) * CRN + 64 * r] : c0;
        }
      } else {
        c0 = B.c0[r];
        c1 = MODE == 0 ? B.c1[r] : B.c0[r];
      }
      // row y - 1 at step t-1: its (u, v) and its sv
      f2v tp;
      float tsv;
      if (DPT) {
        tp = f2v{dpp_from_prev_lane(pp[r].x), MODE == 0 ? dpp_from_prev_lane(pp[r].y) : 0.0f};
        tsv = dpp_from_prev_lane(pvv[r]);
        if (top_lds) {
          tp = ring_s[r * RO + m1 - 3];
          tsv = CRN > 0 ? cr[(ct * CW + CW - 1) * CRN - 1 + 64 * r].w : sv_s[r * RO + m1 - 3];
        }
      } else {
        tp = ring_s[r * RO + m1 - 3];
        tsv = CRN > 0 ? cr[(ct * CW + CW - 1) * CRN - 1 + 64 * r].w : sv_s[r * RO + m1 - 3];
      }
      f2v nw;
      float vv;
#ifdef OFDIS_SOR_PROBE
      {  // the step's LDS operands arrived (a use of each forces the wait): take the clock
        const float dep = ((c0.x + c1.x) + (tp.x + tsv)) + (rgt.x + bt.x);
        asm volatile("; probe use %0" ::"v"(dep) : "memory");
        pt1 = probe_clock();
      }
#endif
      if (MODE == 0) {
        const float hr = c1.z;
        vv = c1.w;
        const f2v bb = f2v{c1.x, c1.y};
        const f2v rr = hasr ? rgt : f2v{0.0f, 0.0f};
        const f2v X = hr * rr, Y = tsv * tp, Z = vv * bt;
        // solver.c's three border expression trees (see sor_rhs), lane-constant operand selects
        const f2v l = X + (border[r] ? bb : Y);
        const f2v rg = (border[r] ? f2v{-0.0f, -0.0f} : bb) + (border[r] ? (notop[r] ? Z : Y) : Z);
        const f2v sr = l + rg;
        const f2v Bv = hasl ? phr[r] * pp[r] + sr : sr;
        const f2v m_1 = f2v{c0.x, c0.y} * Bv.x, m_2 = f2v{c0.z, c0.w} * Bv.y;  // (i11,i12), (i12,i22)
        nw = o + omega * ((m_1 + m_2) - o);
        phr[r] = hr;
      } else {
        const float a11 = c0.x, b1 = c0.y, hr = c0.z;
        vv = c0.w;
        const bool has_top = !notop[r], has_bot = !(border[r] && has_top);
        const float tu = tp.x, ur = hasr ? rgt.x : 0.0f, hl = phr[r];
        float su = 0.0f;  // (a11 here is a11 + the diffusivities: sys_compute)
        su = has_top ? su - tsv * tu : su;
        su = hasl ? su - hl * pp[r].x : su;
        su = has_bot ? su - vv * bt.x : su;
        su = hasr ? su - hr * ur : su;
        const float A = a11, Bq = b1 - su;
        nw = f2v{(1.0f - omega) * o.x + omega * (Bq / A), 0.0f};
        phr[r] = hr;
      }
      ring_s[r * RO + m0] = nw;
      if (CRN == 0) sv_s[r * RO + m0] = vv;
      pvv[r] = vv;
      if (LAST) {
        if ((unsigned)xp < (unsigned)w && yr < h) {
          const unsigned r0 = (unsigned)sor_row2(d, lim, rmax) * (unsigned)hplane;
          du[r0 + (unsigned)yr] = nw.x;
          if (MODE == 0) dv[r0 + (unsigned)yr] = nw.y;
        }
      }
      pp[r] = nw;
    }
#ifdef OFDIS_SOR_PROBE
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pt2 = probe_clock();
#endif
    __syncthreads();
#ifdef OFDIS_SOR_PROBE
    if (probe && (threadIdx.x & 63) == 0 && t < 1024)
      *reinterpret_cast<uint4 *>(probe + 4 * t) = make_uint4(pt0, pt1, pt2, probe_clock());
#endif
  }

  template <int J>
  __device__ __forceinline__ void prologue(const int t) {
    load(t + J, buf<J>());
    if constexpr (J + 1 < PD) prologue<J + 1>(t);
  }
  template <int J>
  __device__ __forceinline__ void block(const int t) {
    step<J>(t + J);
    if constexpr (J + 1 < U) block<J + 1>(t);
  }

  // Steps [0, T), T a multiple of U.  The wave's rows y0..ymax are inside the frame for diagonals
  // d = t - 2s in [y0, ymax + w - 1]; blocks wholly outside that range only join the barriers.
  __device__ __forceinline__ void run(int T, int y0, int ymax) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      pp[r] = f2v{0.0f, 0.0f};
      phr[r] = 0.0f;
      pvv[r] = 0.0f;
    }
    const int ta = max(0, (y0 + 2 * SI) / U * U);
    const int tb = min(T, (ymax + w - 1 + 2 * SI) / U * U + U);
    for (int t = 0; t < ta; ++t) __syncthreads();
    // the previous sweep's value at step ta - 2 (written before the barrier of step ta - 1; zero before t = 0)
    if (!FIRST) {
#pragma unroll
      for (int r = 0; r < R; ++r) prv[r] = ta >= 2 ? ring_p[64 * 3 * r + (ta - 2) % 3] : f2v{0.0f, 0.0f};
    }
    prologue<0>(ta);
    for (int t = ta; t < tb; t += U) block<0>(t);
    for (int t = tb; t < T; ++t) __syncthreads();
  }
};

constexpr size_t kSorLds = 160 * 1024;  // LDS per workgroup (gfx950: 160 KB per CU)
// Compute units of the current device (hipDeviceProp_t::multiProcessorCount; 256 on MI355X), cached per device.
static long device_cus() {
  static long cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int v = 0;
    cus[dev] = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
  }
  return cus[dev];
}
// Entries per slot of the coefficient ring: the most rows a workgroup of MAXT threads holds, + 2 halos
// (a compile-time constant, so every ring offset is an immediate); 0 = no coefficient ring (S > 3).
__host__ __device__ constexpr int sor_crn(int S, int MAXT, int R = 1) {
  return S <= 3 ? 64 * R * (MAXT / (64 * S)) + 2 : 0;
}

// LDS of the lean SOR: S (u, v) rings of NR = 64 R G + 2 entries x 3 slots of float2, then S sv rings
// (CRN = 0) or the coefficient ring (16-byte aligned): 6 slots x CRN entries of 32 (OF, cw = 2) / 16 (DE) bytes.
__host__ __device__ __forceinline__ size_t sor_cring_bytes(int crn, int cw) { return (size_t)6 * crn * (cw == 2 ? 32 : 16); }
__host__ __device__ __forceinline__ size_t sor_lanes_lds(int S, int h, int crn, int cw, int R = 1) {
  const size_t nr = (size_t)((h + 64 * R - 1) / (64 * R)) * 64 * R + 2;
  const size_t uv = sizeof(float) * 2 * 3 * (size_t)S * nr;
  if (crn == 0) return uv + sizeof(float) * 3 * (size_t)S * nr;
  return (uv + 15) / 16 * 16 + sor_cring_bytes(crn, cw);
}

// One frame's SOR call, lean form: 64 * G * S threads, R rows per lane.
template <int S, int MODE, int NB, int CRN, int R, bool SEL = false>
__device__ __forceinline__ void sor_lanes_frame(const TvArgs &a, int frame, f2v *ring) {
  constexpr int CW = MODE == 0 ? 2 : 1;
  const int G = (a.h + 64 * R - 1) / (64 * R);
  const int NR = G * 64 * R + 2;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int g = wid / S, s = wid - g * S;
  float *svr = reinterpret_cast<float *>(ring + S * 3 * NR);
  char *crb = reinterpret_cast<char *>(ring) + (sizeof(f2v) * S * 3 * NR + 15) / 16 * 16;
  float4 *crr = reinterpret_cast<float4 *>(crb);  // [6][CW][CRN] float4
  for (int i = threadIdx.x; i < S * 3 * NR; i += blockDim.x) {
    ring[i] = f2v{0.f, 0.f};
    if (CRN == 0) svr[i] = 0.0f;
  }
  if (CRN > 0) {
    float *z = reinterpret_cast<float *>(crb);
    for (int i = threadIdx.x; i < (int)(sor_cring_bytes(CRN, CW) / 4); i += blockDim.x) z[i] = 0.0f;
  }
  __syncthreads();
#ifdef OFDIS_SOR_PROBE
  __shared__ unsigned probe_slot;
  if (threadIdx.x == 0 && frame == 0) probe_slot = g_sor_probe ? atomicAdd(g_sor_probe, 1u) : 64u;
  __syncthreads();
#endif
  const long fo = (long)frame * a.sp;
  constexpr int U = SorLane<S, MODE, 0, NB, CRN, R>::U;
  const int T = ((a.w - 1) + (a.h - 1) + 2 * (S - 1) + 1 + U - 1) / U * U;
  const int y0 = g * 64 * R, ymax = min(y0 + 64 * R - 1, a.h - 1);
  auto setup = [&](auto &st) {
    st.C = reinterpret_cast<const float4 *>(a.coef) + fo * (MODE == 0 ? 2 : 1);
    st.du_r = a.du + fo;
    st.dv_r = a.dv + fo;
    st.du = a.du + fo;
    st.dv = a.dv + fo;
    const int y = y0 + lane;
    st.ring_s = ring + (s * NR + y + 1) * 3;
    st.ring_p = ring + ((s > 0 ? s - 1 : 0) * NR + y + 1) * 3;
    st.sv_s = svr + (s * NR + y + 1) * 3;
    st.cr = crr + y + 1;
    st.w = a.w; st.h = a.h; st.y = y; st.s = s;  // s == SI
    st.lim = a.wrap ? a.w : 1 << 30;
    st.rmax = a.wrap ? a.w - 1 : a.w + a.h - 2;
    st.hplane = a.h;
    st.top_lds = lane == 0 && y0 > 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int yr = y + 64 * r;
      st.yc[r] = (unsigned)min(yr, a.h - 1);
      st.notop[r] = yr == 0;
      st.border[r] = yr == 0 || yr >= a.h - 1;
    }
    st.omega = a.omega;
#ifdef OFDIS_SOR_PROBE
    if (frame == 0 && probe_slot < 64u && wid < 16)
      st.probe = g_sor_probe + 4 + ((size_t)probe_slot * 16 + wid) * 1024 * 4;
#endif
    st.run(T, y0, ymax);
  };
  if (s == 0) {
    SorLane<S, MODE, 0, NB, CRN, R, SEL> st;
    setup(st);
  } else if (s == 1) {
    SorLane<S, MODE, (S > 1 ? 1 : 0), NB, CRN, R, SEL> st;
    setup(st);
  } else if (s == 2) {
    SorLane<S, MODE, (S > 2 ? 2 : 0), NB, CRN, R, SEL> st;
    setup(st);
  } else {
    SorLane<S, MODE, (S > 3 ? 3 : 0), NB, CRN, R, SEL> st;
    setup(st);
  }
}

// CG > 0: the coefficient ring holds exactly the CG row groups of the level (+ 2 halos) instead of the most a
// workgroup of MAXT threads can hold -- less LDS per frame, more frames per CU.
template <int S, int MODE, int NB, int MAXT, bool CRING, int R = 1, int CG = 0, bool SEL = false>
__global__ __launch_bounds__(MAXT) void k_tv_sor_lanes(TvArgs a) {
  extern __shared__ f2v ring_uv[];  // [S][NR][3], then the sv rings or the coefficient ring
  constexpr int crn = !CRING ? 0 : CG > 0 ? 64 * R * CG + 2 : sor_crn(S, MAXT, R);
  static_assert(CG == 0 || CG * 64 * S <= MAXT, "row groups of the workgroup");
  sor_lanes_frame<S, MODE, NB, crn, R, SEL>(a, blockIdx.x, ring_uv);
}

template <int TH>
__global__ __launch_bounds__(256) void k_tv_final(TvArgs a) {
  const uint3 xb = xcd_block();
  __shared__ float sm[2][TH][kTileP];
  constexpr int TD = kTileW + TH - 1;
  const int x0 = xb.x * kTileW, y0 = xb.y * TH, f = xb.z;
  for (int i = threadIdx.x; i < TD * TH; i += 256) {  // skewed side: diagonal segments
    const int yy = i & (TH - 1), dd = i / TH, xl = dd - yy;
    const int x = x0 + xl, y = y0 + yy;
    if (xl < 0 || xl >= kTileW || x >= a.w || y >= a.h) continue;
    const long fk = (long)f * a.sp + skw(x, y, a.h, a.w, a.wrap);
    if (a.nop == 2) {
      sm[0][yy][xl] = a.wxs[fk] + a.du[fk];
      sm[1][yy][xl] = a.wys[fk] + a.dv[fk];
    } else {
      const float s = a.wxs[fk] + a.du[fk];
      sm[0][yy][xl] = a.camlr == 0 ? ssemin(s, 0.0f) : ssemax(s, 0.0f);
    }
  }
  __syncthreads();
  const int tx = threadIdx.x & 63, x = x0 + tx;
  const long plane = (long)a.w * a.h;
  float *WX = a.flow + (long)f * a.nop * plane;
  for (int yl = threadIdx.x >> 6; yl < TH; yl += 4) {  // row-major side: rows
    const int y = y0 + yl;
    if (x >= a.w || y >= a.h) continue;
    const long o = (long)y * a.w + x;
    WX[o] = sm[0][yl][tx];
    if (a.nop == 2) WX[plane + o] = sm[1][yl][tx];
  }
}

// ------------------------------------------------------------------------------------------------ output

// flow *= 2^l ; cv::resize(INTER_LINEAR) generic float path (HResizeLinear + VResizeLinear) ; crop.
// Horizontal source position / weight of output column dx (resizeGeneric_: fx, sx, xmax clamping).
struct XTap {
  int sx;
  float fx;
  bool lin;
};
__device__ __forceinline__ XTap xtap(int dx, double scale, int wl) {
  XTap r;
  float fx = (float)((dx + 0.5) * scale - 0.5);
  int sx = (int)floorf(fx);
  fx -= (float)sx;
  if (sx < 0) { fx = 0; sx = 0; }
  r.lin = true;
  if (sx + 1 >= wl) {
    r.lin = false;
    if (sx >= wl - 1) { fx = 0; sx = wl - 1; }
  }
  r.sx = sx;
  r.fx = fx;
  return r;
}

__device__ __forceinline__ float up_px(const float *P, long r0, long r1, const XTap &xt, float fct, float b0, float b1) {
  float h0, h1;
  {
    const float *S = P + r0;
    const float s0 = S[xt.sx] * fct;
    h0 = xt.lin ? s0 * (1.f - xt.fx) + (S[xt.sx + 1] * fct) * xt.fx : s0;
  }
  {
    const float *S = P + r1;
    const float s0 = S[xt.sx] * fct;
    h1 = xt.lin ? s0 * (1.f - xt.fx) + (S[xt.sx + 1] * fct) * xt.fx : s0;
  }
  return h0 * b0 + h1 * b1;
}

// Upsample for 2^l >= 2, nop = 2: one block = 1024 output columns x kUpRows output rows, 4 columns (two
// 16-byte stores per row) per thread.  The source rows the block needs are staged in LDS once,
// already multiplied by 2^l.  The OpenCV tap positions fx = (dx + .5) / 2^l - .5 are dyadic rationals, so
// computing them as (2 dx + 1 - 2^l) * 2^-(l+1) in fp32 is exact and equals resizeGeneric_'s double ->
// float value.  Horizontal taps are per source row (HResizeLinear), the vertical blend per output row
// (VResizeLinear), exactly as in OpenCV's generic float path.
constexpr int kUpCols = 1024;
// 4 output rows per block (round 4, profiles/r04/s17): 13 KB of staged source rows, more blocks per CU; B's
// upsample 6.27-6.29 -> 6.00-6.01 ms per 2048-pair launch against 8 rows (2 rows: 6.73, 16 rows: 6.55)
constexpr int kUpRows = 4;
constexpr int kUpSrcRows = kUpRows / 2 + 3;  // source rows a block can touch (2^l >= 2)
typedef float v4f __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_upsample_rows(UpArgs a) {
  __shared__ float src[kUpSrcRows][2][kUpCols / 2 + 8];  // [row][comp][col]
  const int y0 = blockIdx.y * kUpRows, f = blockIdx.z;
  const int dx0 = blockIdx.x * kUpCols + a.offx;  // first output column of the block (uncropped coordinates)
  const int fct_i = 1 << a.log2s;
  const float fct = (float)fct_i, half_inv = 1.0f / (float)(2 * fct_i);
  const long plane = (long)a.wl * a.hl;
  const float *F = a.flow + (long)f * 2 * plane;
  auto src_row = [&](int dy, float &fy) {  // resizeGeneric_Invoker rows: sy, fy (weights not clamped)
    fy = (float)(2 * dy + 1 - fct_i) * half_inv;
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    return sy;
  };
  auto clip_row = [&](int r) { return r >= 0 ? (r < a.hl ? r : a.hl - 1) : 0; };
  const int yl = min(y0 + kUpRows, a.H0) - 1;
  float dummy;
  const int r_first = clip_row(src_row(y0 + a.offy, dummy));
  const int r_last = clip_row(src_row(yl + a.offy, dummy) + 1);
  const int nr = r_last - r_first + 1;
  // source column window of this block
  const int c_lo = max(0, (int)floorf((float)(2 * dx0 + 1 - fct_i) * half_inv));
  const int ncol = kUpCols / fct_i + 2;
  for (int k = threadIdx.x; k < nr * 2 * ncol; k += blockDim.x) {
    const int col = k % ncol, rc = k / ncol;  // rc = row * 2 + comp
    const int r = rc >> 1, comp = rc & 1;
    const int sc = min(c_lo + col, a.wl - 1);
    src[r][comp][col] = F[comp * plane + (long)(r_first + r) * a.wl + sc] * fct;
  }
  __syncthreads();
  // lane i of wave wv owns output columns xb + {2i, 2i+1} and xb + 128 + {2i, 2i+1} (xb = block + 256 wv):
  // each 16-byte store instruction of a wave then covers 1 KiB contiguously (full cache lines).
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int xb = blockIdx.x * kUpCols + wv * 256 + 2 * lane;
  int xs[2] = {xb, xb + 128};
  int cc[4];
  float fxs[4];
  bool lin[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int dx = xs[i >> 1] + (i & 1) + a.offx;
    float fx = (float)(2 * dx + 1 - fct_i) * half_inv;
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { fx = 0; sx = 0; }
    bool l = true;
    if (sx + 1 >= a.wl) {
      l = false;
      if (sx >= a.wl - 1) { fx = 0; sx = a.wl - 1; }
    }
    cc[i] = min(max(sx - c_lo, 0), kUpCols / 2 + 6);  // columns past W0 are computed, never stored
    fxs[i] = fx;
    lin[i] = l;
  }
#pragma unroll
  for (int i = 0; i < kUpRows; ++i) {
    const int y = y0 + i;
    if (y >= a.H0) break;
    float fy;
    const int sy = src_row(y + a.offy, fy);
    const int j0 = clip_row(sy) - r_first, j1 = clip_row(sy + 1) - r_first;
    const float b0 = 1.f - fy, b1 = fy;
    float v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int c = cc[q];
        const float s00 = src[j0][k][c], s10 = src[j1][k][c];
        const float h0 = lin[q] ? s00 * (1.f - fxs[q]) + src[j0][k][c + 1] * fxs[q] : s00;
        const float h1 = lin[q] ? s10 * (1.f - fxs[q]) + src[j1][k][c + 1] * fxs[q] : s10;
        v[q * 2 + k] = h0 * b0 + h1 * b1;
      }
    }
    float *row = a.out + ((long)f * a.H0 + y) * a.W0 * 2;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int x = xs[hh];
      if (x + 2 <= a.W0) {
        const v4f val = v4f{v[4 * hh], v[4 * hh + 1], v[4 * hh + 2], v[4 * hh + 3]};
        if (a.nt_store)
          __builtin_nontemporal_store(val, reinterpret_cast<v4f *>(row + 2 * x));
        else
          *reinterpret_cast<v4f *>(row + 2 * x) = val;
      } else if (x < a.W0) {
        row[2 * x] = v[4 * hh];
        row[2 * x + 1] = v[4 * hh + 1];
      }
    }
  }
}

// k_upsample_h<R>: the same output (same expressions, same lanes and stores) with each staged source row's
// horizontal taps computed once per lane and column instead of once per output row that reads them
// (VResizeLinear blends two HResizeLinear rows; at 2^l = 2 four output rows read four source rows, eight
// horizontal evaluations before), and the staging copy in 16-byte groups with no per-element division:
// B's upsample issued ~500 VALU per wave, 43 % of the whole pipeline's VALU (profiles/r05/s9).  R output rows
// per block (4 or 8).  The staged window starts at the 4-aligned column below the first one the block reads.
template <int R>
__global__ __launch_bounds__(256) void k_upsample_h(UpArgs a) {
  constexpr int NSR = R / 2 + 3;         // source rows a block can touch (2^l >= 2)
  constexpr int SC = kUpCols / 2 + 8;    // staged columns per row (>= the 514 + 3 a block reads at 2^l = 2)
  constexpr int S4 = SC / 4;             // 16-byte groups per staged row
  __shared__ __attribute__((aligned(16))) float src[NSR][2][SC];
  const int y0 = blockIdx.y * R, f = blockIdx.z;
  const int dx0 = blockIdx.x * kUpCols + a.offx;
  const int fct_i = 1 << a.log2s;
  const float fct = (float)fct_i, half_inv = 1.0f / (float)(2 * fct_i);
  const long plane = (long)a.wl * a.hl;
  const float *F = a.flow + (long)f * 2 * plane;
  auto src_row = [&](int dy, float &fy) {  // resizeGeneric_Invoker rows: sy, fy (weights not clamped)
    fy = (float)(2 * dy + 1 - fct_i) * half_inv;
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    return sy;
  };
  auto clip_row = [&](int r) { return r >= 0 ? (r < a.hl ? r : a.hl - 1) : 0; };
  const int yl = min(y0 + R, a.H0) - 1;
  float dummy;
  const int r_first = clip_row(src_row(y0 + a.offy, dummy));
  const int r_last = clip_row(src_row(yl + a.offy, dummy) + 1);
  const int nr = r_last - r_first + 1;
  const int c_lo = max(0, (int)floorf((float)(2 * dx0 + 1 - fct_i) * half_inv));
  const int c0 = c_lo & ~3;                                  // staged column 0
  const int n4 = min(S4, (c_lo - c0 + kUpCols / fct_i + 2 + 3) >> 2);
  const bool vec = (a.wl & 3) == 0 && ((uintptr_t)a.flow & 15) == 0;
  for (int e = threadIdx.x; e < nr * 2 * S4; e += 256) {  // (row, comp) = e / S4: a division by a constant
    const int rc = e / S4, j = e - rc * S4;
    if (j >= n4) continue;
    const int r = rc >> 1, comp = rc & 1, c = c0 + 4 * j;
    const float *row = F + comp * plane + (long)(r_first + r) * a.wl;
    v4f v;
    if (vec && c + 3 < a.wl) {
      v = *reinterpret_cast<const v4f *>(row + c);
    } else {
      v = v4f{row[min(c, a.wl - 1)], row[min(c + 1, a.wl - 1)], row[min(c + 2, a.wl - 1)], row[min(c + 3, a.wl - 1)]};
    }
    *reinterpret_cast<v4f *>(&src[r][comp][4 * j]) = v * fct;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int xb = blockIdx.x * kUpCols + wv * 256 + 2 * lane;
  int xs[2] = {xb, xb + 128};
  int cc[4];
  float fxs[4], gxs[4];
  bool lin[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int dx = xs[i >> 1] + (i & 1) + a.offx;
    float fx = (float)(2 * dx + 1 - fct_i) * half_inv;
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { fx = 0; sx = 0; }
    bool l = true;
    if (sx + 1 >= a.wl) {
      l = false;
      if (sx >= a.wl - 1) { fx = 0; sx = a.wl - 1; }
    }
    cc[i] = min(max(sx - c0, 0), SC - 2);  // columns past W0 are computed, never stored
    fxs[i] = fx;
    gxs[i] = 1.f - fx;
    lin[i] = l;
  }
  auto hrow = [&](int j, float *h) {  // HResizeLinear of staged row j at the lane's 4 columns, both components
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const float s0 = src[j][k][cc[q]];
        h[q * 2 + k] = lin[q] ? s0 * gxs[q] + src[j][k][cc[q] + 1] * fxs[q] : s0;
      }
  };
  float ha[8], hb[8];
  int ja = -1, jb = -1;  // staged rows held in ha / hb (wave-uniform)
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int y = y0 + i;
    if (y >= a.H0) break;
    float fy;
    const int sy = src_row(y + a.offy, fy);
    const int j0 = clip_row(sy) - r_first, j1 = clip_row(sy + 1) - r_first;
    if (j0 != ja) {
      if (j0 == jb) {
#pragma unroll
        for (int t = 0; t < 8; ++t) ha[t] = hb[t];
      } else {
        hrow(j0, ha);
      }
      ja = j0;
    }
    if (j1 != jb) {
      if (j1 == ja) {
#pragma unroll
        for (int t = 0; t < 8; ++t) hb[t] = ha[t];
      } else {
        hrow(j1, hb);
      }
      jb = j1;
    }
    const float b0 = 1.f - fy, b1 = fy;
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = ha[t] * b0 + hb[t] * b1;
    float *orow = a.out + ((long)f * a.H0 + y) * a.W0 * 2;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int x = xs[hh];
      if (x + 2 <= a.W0) {
        const v4f val = v4f{v[4 * hh], v[4 * hh + 1], v[4 * hh + 2], v[4 * hh + 3]};
        if (a.nt_store)
          __builtin_nontemporal_store(val, reinterpret_cast<v4f *>(orow + 2 * x));
        else
          *reinterpret_cast<v4f *>(orow + 2 * x) = val;
      } else if (x < a.W0) {
        orow[2 * x] = v[4 * hh];
        orow[2 * x + 1] = v[4 * hh + 1];
      }
    }
  }
}

// The same for depth (nop = 1): lane i of wave wv owns the four output columns xb + 4i .. xb + 4i + 3
// (xb = block + 256 wv): one 16-byte store per row, 1 KiB contiguous per wave-instruction.
__global__ __launch_bounds__(256) void k_upsample_rows1(UpArgs a) {
  __shared__ float src[kUpSrcRows][kUpCols / 2 + 8];
  const int y0 = blockIdx.y * kUpRows, f = blockIdx.z;
  const int dx0 = blockIdx.x * kUpCols + a.offx;
  const int fct_i = 1 << a.log2s;
  const float fct = (float)fct_i, half_inv = 1.0f / (float)(2 * fct_i);
  const float *F = a.flow + (long)f * a.wl * a.hl;
  auto src_row = [&](int dy, float &fy) {
    fy = (float)(2 * dy + 1 - fct_i) * half_inv;
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    return sy;
  };
  auto clip_row = [&](int r) { return r >= 0 ? (r < a.hl ? r : a.hl - 1) : 0; };
  const int yl = min(y0 + kUpRows, a.H0) - 1;
  float dummy;
  const int r_first = clip_row(src_row(y0 + a.offy, dummy));
  const int r_last = clip_row(src_row(yl + a.offy, dummy) + 1);
  const int nr = r_last - r_first + 1;
  const int c_lo = max(0, (int)floorf((float)(2 * dx0 + 1 - fct_i) * half_inv));
  const int ncol = kUpCols / fct_i + 2;
  for (int k = threadIdx.x; k < nr * ncol; k += blockDim.x) {
    const int col = k % ncol, r = k / ncol;
    src[r][col] = F[(long)(r_first + r) * a.wl + min(c_lo + col, a.wl - 1)] * fct;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int xb = blockIdx.x * kUpCols + wv * 256 + 4 * lane;
  int cc[4];
  float fxs[4];
  bool lin[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int dx = xb + i + a.offx;
    float fx = (float)(2 * dx + 1 - fct_i) * half_inv;
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { fx = 0; sx = 0; }
    bool l = true;
    if (sx + 1 >= a.wl) {
      l = false;
      if (sx >= a.wl - 1) { fx = 0; sx = a.wl - 1; }
    }
    cc[i] = min(max(sx - c_lo, 0), kUpCols / 2 + 6);  // columns past W0 are computed, never stored
    fxs[i] = fx;
    lin[i] = l;
  }
#pragma unroll
  for (int i = 0; i < kUpRows; ++i) {
    const int y = y0 + i;
    if (y >= a.H0) break;
    float fy;
    const int sy = src_row(y + a.offy, fy);
    const int j0 = clip_row(sy) - r_first, j1 = clip_row(sy + 1) - r_first;
    const float b0 = 1.f - fy, b1 = fy;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = cc[q];
      const float s00 = src[j0][c], s10 = src[j1][c];
      const float h0 = lin[q] ? s00 * (1.f - fxs[q]) + src[j0][c + 1] * fxs[q] : s00;
      const float h1 = lin[q] ? s10 * (1.f - fxs[q]) + src[j1][c + 1] * fxs[q] : s10;
      v[q] = h0 * b0 + h1 * b1;
    }
    float *row = a.out + ((long)f * a.H0 + y) * a.W0;
    if (xb + 4 <= a.W0) {
      *reinterpret_cast<v4f *>(row + xb) = v4f{v[0], v[1], v[2], v[3]};
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (xb + q < a.W0) row[xb + q] = v[q];
    }
  }
}

// Generic path (any nop, 2^l = 1, unaligned output): one output pixel per thread.
__global__ __launch_bounds__(256) void k_upsample(UpArgs a) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
  if (x >= a.W0) return;
  const long plane = (long)a.wl * a.hl;
  const float *F = a.flow + (long)f * a.nop * plane;
  float *out = a.out + (((long)f * a.H0 + y) * a.W0 + x) * a.nop;
  if (a.log2s == 0) {
    const long o = (long)(y + a.offy) * a.wl + (x + a.offx);
    out[0] = F[o];
    if (a.nop == 2) out[1] = F[plane + o];
    return;
  }
  const float fct = (float)(1 << a.log2s);
  const double scale = 1.0 / (double)(1 << a.log2s);
  const int dy = y + a.offy;
  float fy = (float)((dy + 0.5) * scale - 0.5);
  const int sy = (int)floorf(fy);
  fy -= (float)sy;
  const long r0 = (long)(sy >= 0 ? (sy < a.hl ? sy : a.hl - 1) : 0) * a.wl;
  const long r1 = (long)(sy + 1 >= 0 ? (sy + 1 < a.hl ? sy + 1 : a.hl - 1) : 0) * a.wl;
  const float b0 = 1.f - fy, b1 = fy;
  const XTap xt = xtap(x + a.offx, scale, a.wl);
  for (int k = 0; k < a.nop; ++k) out[k] = up_px(F + k * plane, r0, r1, xt, fct, b0, b1);
}

}  // namespace

// ------------------------------------------------------------------------------------------------ launchers

void launch_pyr_base(const PyrBaseArgs &a, hipStream_t s) {
  const long total = 2L * a.n * a.h * a.w;
  if (a.noc == 1 && a.log2s >= 2 && a.log2s <= 5) {
    const unsigned blocks = (unsigned)ceil_div(total, 256);
    switch (a.log2s) {
      case 2: k_pyr_base_gray<2><<<blocks, 256, 0, s>>>(a); return;
      case 3: k_pyr_base_gray<3><<<blocks, 256, 0, s>>>(a); return;
      case 4: k_pyr_base_gray<4><<<blocks, 256, 0, s>>>(a); return;
      case 5: k_pyr_base_gray<5><<<blocks, 256, 0, s>>>(a); return;
    }
  }
  if (a.noc == 3 && a.rgb_sad && a.log2s >= 2 && a.log2s <= 4) {
    const unsigned blocks = (unsigned)ceil_div(total, 256);
    switch (a.log2s) {
      case 2: k_pyr_base_rgb<2><<<blocks, 256, 0, s>>>(a); return;
      case 3: k_pyr_base_rgb<3><<<blocks, 256, 0, s>>>(a); return;
      case 4: k_pyr_base_rgb<4><<<blocks, 256, 0, s>>>(a); return;
    }
  }
  k_pyr_base<<<dim3(ceil_div(a.w, 256), a.h, 2 * a.n), 256, 0, s>>>(a);
}
void launch_pyr_gradmag(const PyrGradmagArgs &a, hipStream_t s) {
  k_pyr_gradmag<<<dim3(ceil_div(a.Wp, 256), a.Hp, 2 * a.n), 256, 0, s>>>(a);
}
void launch_pyr_down(const PyrDownArgs &a, hipStream_t s) {
  k_pyr_down<<<std::min(ceil_div((long)a.n2 * a.h * a.w * a.noc, 256), 1u << 22), 256, 0, s>>>(a);  // grid-stride beyond
}
void launch_pyr_pad_grad(const PyrPadGradArgs &a, hipStream_t s) {
  if (a.noc == 3 && a.per_value) {
    k_pyr_pad_grad_v<3><<<std::min(ceil_div((long)a.n2 * (a.h + 2 * a.pad) * (a.w + 2 * a.pad) * 3, 256), 1u << 22),
                          256, 0, s>>>(a);
    return;
  }
  k_pyr_pad_grad<<<std::min(ceil_div((long)a.n2 * (a.h + 2 * a.pad) * (a.w + 2 * a.pad), 256), 1u << 22), 256, 0,
                   s>>>(a);  // grid-stride beyond 2^22 workgroups
}
template <int JM>
static void patch_jm(const PatchArgs &a, hipStream_t s) {
  const long waves = (long)a.n * a.g.npatch;
  const int rs = JM == 1 ? 64 : ((a.novals + 31) / 32) * 32 + 8;
  const size_t lds = sizeof(float) * 3 * rs * kPatchWaves;
  if (a.nop == 2)
    k_patch<2, JM><<<ceil_div(waves, kPatchWaves), 64 * kPatchWaves, lds, s>>>(a);
  else
    k_patch<1, JM><<<ceil_div(waves, kPatchWaves), 64 * kPatchWaves, lds, s>>>(a);
}
template <int PAIRS, int ODD>
static void patch8(const PatchArgs &a, hipStream_t s) {
  const long patches = (long)a.n * a.g.npatch;
  if (a.nop == 2)
    k_patch8<2, PAIRS, ODD><<<ceil_div(patches, 32), 256, 0, s>>>(a);
  else
    k_patch8<1, PAIRS, ODD><<<ceil_div(patches, 32), 256, 0, s>>>(a);
}
// MINW1 / MINW2: waves per SIMD for the depth (nop 1) / flow (nop 2) forms, chosen so that nothing spills
// MINW0: waves per SIMD of the L2-cost (costfct 0) instances
template <int P, int NOC, int MINW1, int MINW2, int MINW0 = 0>
static void patchw(const PatchArgs &a, hipStream_t s) {
  const long patches = (long)a.n * a.g.npatch;
  const size_t lds = sizeof(float) * 32 * PatchShape<P, NOC>::WIN;
  const dim3 grid(ceil_div(patches, 32));
  constexpr int M01 = MINW0 ? MINW0 : MINW1, M02 = MINW0 ? MINW0 : MINW2;
  switch (a.costfct * 2 + (a.nop == 2 ? 1 : 0)) {
    case 0: k_patchw<1, P, NOC, M01, 0><<<grid, 256, lds, s>>>(a); return;
    case 1: k_patchw<2, P, NOC, M02, 0><<<grid, 256, lds, s>>>(a); return;
    case 2: k_patchw<1, P, NOC, MINW1, 1><<<grid, 256, lds, s>>>(a); return;
    case 3: k_patchw<2, P, NOC, MINW2, 1><<<grid, 256, lds, s>>>(a); return;
    case 4: k_patchw<1, P, NOC, MINW1, 2><<<grid, 256, lds, s>>>(a); return;
    default: k_patchw<2, P, NOC, MINW2, 2><<<grid, 256, lds, s>>>(a); return;
  }
}
template <int P, int NOC, int MINW1, int MINW2>
static void patchq(const PatchArgs &a, hipStream_t s) {
  const long patches = (long)a.n * a.g.npatch;
  const size_t lds = sizeof(float) * 64 * QuadShape<P, NOC>::WIN;
  const dim3 grid(ceil_div(patches, 64));
  switch (a.costfct * 2 + (a.nop == 2 ? 1 : 0)) {
    case 0: k_patchq<1, P, NOC, MINW1, 0><<<grid, 256, lds, s>>>(a); return;
    case 1: k_patchq<2, P, NOC, MINW2, 0><<<grid, 256, lds, s>>>(a); return;
    case 2: k_patchq<1, P, NOC, MINW1, 1><<<grid, 256, lds, s>>>(a); return;
    case 3: k_patchq<2, P, NOC, MINW2, 1><<<grid, 256, lds, s>>>(a); return;
    case 4: k_patchq<1, P, NOC, MINW1, 2><<<grid, 256, lds, s>>>(a); return;
    default: k_patchq<2, P, NOC, MINW2, 2><<<grid, 256, lds, s>>>(a); return;
  }
}
template <int P, int NOC, int MINW>
static void patchx(const PatchArgs &a, hipStream_t s) {
  const long patches = (long)a.n * a.g.npatch;
  const size_t lds = sizeof(float) * XShape<P, NOC>::lds_floats(a.nop == 2 ? 2 : 1);
  const dim3 grid(ceil_div(patches, 16));
  switch (a.costfct * 2 + (a.nop == 2 ? 1 : 0)) {
    case 0: k_patchx<1, P, NOC, MINW, 0><<<grid, 256, lds, s>>>(a); return;
    case 1: k_patchx<2, P, NOC, MINW, 0><<<grid, 256, lds, s>>>(a); return;
    case 2: k_patchx<1, P, NOC, MINW, 1><<<grid, 256, lds, s>>>(a); return;
    case 3: k_patchx<2, P, NOC, MINW, 1><<<grid, 256, lds, s>>>(a); return;
    case 4: k_patchx<1, P, NOC, MINW, 2><<<grid, 256, lds, s>>>(a); return;
    default: k_patchx<2, P, NOC, MINW, 2><<<grid, 256, lds, s>>>(a); return;
  }
}
void launch_patch_loss(const PatchArgs &a, hipStream_t s);
bool launch_patch(const PatchArgs &a, hipStream_t s) {
  if (a.window && a.x16 && !a.wave_per_patch && !a.generic && a.p == 12 && a.noc == 3) {  // sixteen lanes per patch
    patchx<12, 3, 3>(a, s);
    return a.absw != 0;
  }
  if (a.window && a.quad && !a.wave_per_patch && !a.generic && a.noc == 1 && (a.p == 8 || a.p == 12)) {
    launch_patch_loss(a, s);  // k_patchq: the aggregation weights too
    return a.absw != 0;
  }
  PatchArgs b = a;
  b.absw = 0;  // the other kernels write the loss weights
  launch_patch_loss(b, s);
  return false;
}
void launch_patch_loss(const PatchArgs &a, hipStream_t s) {
  if (a.window && a.quad && !a.wave_per_patch && !a.generic) {  // four lanes per patch: gray p = 8 / 12
    switch (a.p * 4 + a.noc) {
      case 8 * 4 + 1: patchq<8, 1, 4, 3>(a, s); return;
      case 12 * 4 + 1: patchq<12, 1, 3, 2>(a, s); return;
    }
  }
  if (a.window && !a.wave_per_patch && !a.generic) {  // LDS-windowed eight-lane form for the shapes of the op-points
    switch (a.p * 4 + a.noc) {
      case 8 * 4 + 1: patchw<8, 1, 4, 4>(a, s); return;
      case 12 * 4 + 1: patchw<12, 1, 4, 3>(a, s); return;
      case 8 * 4 + 3: patchw<8, 3, 2, 2>(a, s); return;
      case 12 * 4 + 3: patchw<12, 3, 2, 2, 1>(a, s); return;  // L2 cost: samples kept, one wave per SIMD
    }
  }
  if (!a.wave_per_patch && !a.generic) {
    switch (a.novals) {  // eight lanes per patch for the common shapes
      case 64: patch8<8, 0>(a, s); return;    // p 8, gray
      case 144: patch8<18, 0>(a, s); return;  // p 12, gray
      case 192: patch8<24, 0>(a, s); return;  // p 8, RGB
      case 36: patch8<4, 1>(a, s); return;    // p 6, gray
      case 100: patch8<12, 1>(a, s); return;  // p 10, gray
      case 16: patch8<2, 0>(a, s); return;    // p 4, gray
      case 4: patch8<0, 1>(a, s); return;     // p 2, gray
    }
  }
  const int J = (a.novals + 63) / 64;
  if (a.generic || J > 7) {  // any shape: runtime value loops (p^2 noc > 448, or forced by option patch_generic)
    const unsigned grid = ceil_div((long)a.n * a.g.npatch, 32);
    if (a.nop == 2)
      k_patchg<2><<<grid, 256, 0, s>>>(a);
    else
      k_patchg<1><<<grid, 256, 0, s>>>(a);
    return;
  }
  if (J <= 1)
    patch_jm<1>(a, s);
  else if (J <= 3)
    patch_jm<3>(a, s);
  else
    patch_jm<7>(a, s);
}
void launch_aggregate(const AggArgs &a, hipStream_t s) {
  k_aggregate<<<dim3(ceil_div(a.g.w, 64), ceil_div(a.g.h, 16), a.n), 256, 0, s>>>(a);
}
void launch_tv_prep(const TvArgs &a, hipStream_t s) {
  if (a.noc == 1)
    k_tv_prep<5, 32><<<dim3(ceil_div(a.w, kTileW), ceil_div(a.h, 32), a.n), 256, 0, s>>>(a);
  else
    k_tv_prep<9, 16><<<dim3(ceil_div(a.w, kTileW), ceil_div(a.h, 16), a.n), 256, 0, s>>>(a);
}
// prep + derivatives in one launch: intensity images (option prepd), colour images too with prepd = 2 (default)
// Code-object warm-up: HIP loads a translation unit's code object on the first launch of any of its kernels, which
// in a one-pair-per-process CLI would land inside the reference's first timer (TIME (Pyramide+Gradients),
// run_dense.cpp:315-353).  ofdis_context_create launches this empty kernel of each unit instead.
__global__ void k_warm_kernels(int *p) {
  if (p) *p = 0;
}
void warm_kernels_module(hipStream_t s) { k_warm_kernels<<<1, 64, 0, s>>>(nullptr); }

bool tv_prepd_ok(const TvArgs &a) { return a.prepd && (a.noc == 1 || a.prepd == 2); }
void launch_tv_prepd(const TvArgs &a, hipStream_t s) {
  const dim3 grid(ceil_div(a.w, kPdW), ceil_div(a.h, kPdH), a.n);
  if (a.smsys_deriv && !a.lat && a.prepd_df) {  // tv_deriv_fused(): Ix, Iy, Iz only
    // tall levels (the march's, h >= 256) on 64 x 32 tiles, 512 threads: halo 1.33x -> 1.2x the core, the same
    // occupancy; config E's prep 3.06 -> 2.61 ms per step, C's 3.16 -> 3.04 (profiles/r06/s29); short levels keep
    // 16 rows (B's 68-row levels would compute 96)
    if (a.h >= 256) {
      const dim3 g32(ceil_div(a.w, kPdW), ceil_div(a.h, 32), a.n);
      if (a.noc == 1) k_tv_prepd_df<1, 32><<<g32, 512, 0, s>>>(a);
      else k_tv_prepd_df<3, 32><<<g32, 512, 0, s>>>(a);
    } else if (a.noc == 1) k_tv_prepd_df<1><<<grid, 256, 0, s>>>(a);
    else k_tv_prepd_df<3><<<grid, 256, 0, s>>>(a);
    return;
  }
  if (a.noc == 1) k_tv_prepd<1><<<grid, 256, 0, s>>>(a);
  else k_tv_prepd_c3<<<grid, 256, 0, s>>>(a);
}
void launch_tv_deriv1(const TvArgs &a, hipStream_t s) {
  k_tv_deriv1<<<dim3(ceil_div(a.sp, 256), a.n * a.noc), 256, 0, s>>>(a);
}
void launch_tv_deriv2(const TvArgs &a, hipStream_t s) {
  k_tv_deriv2<<<dim3(ceil_div(a.sp, 256), a.n * a.noc), 256, 0, s>>>(a);
}
void launch_tv_smooth(const TvArgs &a, hipStream_t s) {
  if (a.nop == 2)
    k_tv_smooth<2><<<dim3(ceil_div(a.sp, 256), a.n), 256, 0, s>>>(a);
  else
    k_tv_smooth<1><<<dim3(ceil_div(a.sp, 256), a.n), 256, 0, s>>>(a);
}
// The fused form stages RB + 4 rows for RB computed ones: below RB = 4 (h > 256) the halo re-reads cost
// more than the smoothness round trip saves (config E, h = 544 / 272: 518 vs 299 us per launch).
// Tall levels take the 2-D tiled form (k_tv_smsys2d) unless a.smsys2d = 0 (A/B: two launches there).
// The register march for a level: tall levels (no row block fits).  (Colour levels of 135 rows on the march too: prep
// -0.50 ms, system +0.62 ms per config-C step, r06_s13: not taken.)
static bool smsys_use_march(const TvArgs &a) {
  return a.smsys_march && !(smsys_rb(a.h) >= 4 && smsys_lds(a.h) <= 64 * 1024);
}
bool tv_smsys_ok(const TvArgs &a) {
  return a.smsys && ((smsys_rb(a.h) >= 4 && smsys_lds(a.h) <= 64 * 1024) || a.smsys2d || a.smsys_march);
}
// The derivative filters move into the system kernel where the level runs k_tv_prepd (intensity images) and the
// row-block k_tv_smsys or the march k_tv_smsys_m (round 4); the 2-D tiles and the two-launch form read all eight planes.
// Not where the 40 KB LDS cap of the DF form leaves fewer than 3 rows per block (levels of ~180-256 rows): a
// block would then stage 5-6 rows of seven planes for 1-2 computed ones, 3-5x redundant staging.
bool tv_deriv_fused(const TvArgs &a) {
  if (!(a.smsys_deriv && tv_prepd_ok(a) && a.smsys)) return false;
  if (smsys_use_march(a)) return true;  // the march filters them too
  if (!(smsys_rb(a.h) >= 4 && smsys_lds(a.h) <= 64 * 1024)) return false;
  if (a.noc != 1) return false;  // colour images: the march only (a row block would stage 9 derivative planes)
  int rb = smsys_rb_n(a.h, smsys_rows(a.w, a.h, a.wrap), a.n, a.smsys_small);
  while (rb > 1 && smsys_lds_df(a.h, rb, true) > kSmsysDfCap) --rb;
  return rb >= 3;
}
void launch_tv_smsys(const TvArgs &a, hipStream_t s) {
  if (smsys_use_march(a)) {
    const long waves = (long)a.n * march_segments(smsys_rows(a.w, a.h, a.wrap)) * march_strips(a.h);
    const unsigned grid = ceil_div(waves, 4);
    if (a.smsys_deriv) {  // tv_deriv_fused(): k_tv_prepd wrote Ix, Iy, Iz only
      if (a.noc == 1) {
        if (a.nop == 2) k_tv_smsys_m<2, 1, true><<<grid, 256, 0, s>>>(a);
        else k_tv_smsys_m<1, 1, true><<<grid, 256, 0, s>>>(a);
      } else {
        if (a.nop == 2) k_tv_smsys_m<2, 3, true><<<grid, 256, 0, s>>>(a);
        else k_tv_smsys_m<1, 3, true><<<grid, 256, 0, s>>>(a);
      }
    } else if (a.nop == 2) {
      if (a.noc == 1) k_tv_smsys_m<2, 1><<<grid, 256, 0, s>>>(a);
      else k_tv_smsys_m<2, 3><<<grid, 256, 0, s>>>(a);
    } else {
      if (a.noc == 1) k_tv_smsys_m<1, 1><<<grid, 256, 0, s>>>(a);
      else k_tv_smsys_m<1, 3><<<grid, 256, 0, s>>>(a);
    }
    return;
  }
  if (!(smsys_rb(a.h) >= 4 && smsys_lds(a.h) <= 64 * 1024)) {
    const dim3 g2(a.n, ceil_div(smsys_rows(a.w, a.h, a.wrap), kS2R), ceil_div(a.h, kS2C));
    if (a.nop == 2) {
      if (a.noc == 1) k_tv_smsys2d<2, 1><<<g2, 256, 0, s>>>(a);
      else k_tv_smsys2d<2, 3><<<g2, 256, 0, s>>>(a);
    } else {
      if (a.noc == 1) k_tv_smsys2d<1, 1><<<g2, 256, 0, s>>>(a);
      else k_tv_smsys2d<1, 3><<<g2, 256, 0, s>>>(a);
    }
    return;
  }
  const int rows = smsys_rows(a.w, a.h, a.wrap);
  int rb = smsys_rb_n(a.h, rows, a.n, a.smsys_small);
  if (a.smsys_deriv) {  // the kernel's rule: four workgroups per CU
    while (rb > 1 && smsys_lds_df(a.h, rb, true) > kSmsysDfCap) --rb;
    const dim3 grid(a.n, ceil_div(rows, rb));
    const size_t lds = smsys_lds_df(a.h, rb, true);
    if (a.nop == 2) k_tv_smsys<2, 1, true><<<grid, 256, lds, s>>>(a);
    else k_tv_smsys<1, 1, true><<<grid, 256, lds, s>>>(a);
    return;
  }
  const dim3 grid(a.n, ceil_div(rows, rb));
  const size_t lds = smsys_lds_rb(a.h, rb);
  if (a.nop == 2) {
    if (a.noc == 1)
      k_tv_smsys<2, 1><<<grid, 256, lds, s>>>(a);
    else
      k_tv_smsys<2, 3><<<grid, 256, lds, s>>>(a);
  } else {
    if (a.noc == 1)
      k_tv_smsys<1, 1><<<grid, 256, lds, s>>>(a);
    else
      k_tv_smsys<1, 3><<<grid, 256, lds, s>>>(a);
  }
}
void launch_tv_system(const TvArgs &a, hipStream_t s) {
  const dim3 grid(ceil_div(a.sp, 256), a.n);
  if (a.nop == 2) {
    if (a.noc == 1)
      k_tv_system<2, 1><<<grid, 256, 0, s>>>(a);
    else
      k_tv_system<2, 3><<<grid, 256, 0, s>>>(a);
  } else {
    if (a.noc == 1)
      k_tv_system<1, 1><<<grid, 256, 0, s>>>(a);
    else
      k_tv_system<1, 3><<<grid, 256, 0, s>>>(a);
  }
}
template <int S>
static void sor_pipe(const TvArgs &a, hipStream_t s) {
  const int threads = ((a.h + 63) / 64) * 64;
  if (threads <= 256) {
    if (a.nop == 2)
      k_tv_sor_pipe<S, 0, 256><<<a.n, threads, 0, s>>>(a);
    else
      k_tv_sor_pipe<S, 2, 256><<<a.n, threads, 0, s>>>(a);
  } else if (threads <= 512) {
    if (a.nop == 2)
      k_tv_sor_pipe<S, 0, 512><<<a.n, threads, 0, s>>>(a);
    else
      k_tv_sor_pipe<S, 2, 512><<<a.n, threads, 0, s>>>(a);
  } else {
    if (a.nop == 2)
      k_tv_sor_pipe<S, 0, 1024><<<a.n, threads, 0, s>>>(a);
    else
      k_tv_sor_pipe<S, 2, 1024><<<a.n, threads, 0, s>>>(a);
  }
}
// Sweep-per-wave SOR (k_tv_sor_lanes): 64 * ceil(h / (64 R)) * S threads, one workgroup per frame.  With S <= 3
// sweep 0 hands the coefficients to the later sweeps through an LDS ring (option sor_cring, default on) while
// it fits the LDS.
template <int S, int MAXT, int R>
static void sor_lanes(const TvArgs &a, hipStream_t s) {
  const int G = (a.h + 64 * R - 1) / (64 * R);
  constexpr int crn = sor_crn(S, MAXT, R);
  const int cw = a.nop == 2 ? 2 : 1;
  const bool cring = crn > 0 && a.sor_cring && sor_lanes_lds(S, a.h, crn, cw, R) <= kSorLds;
  const size_t lds = sor_lanes_lds(S, a.h, cring ? crn : 0, cw, R);
  const int th = 64 * G * S;
  if constexpr (S == 3 && R == 1) {
    if (cring && a.sor_cring >= 2) {  // the ring sized to the level's G row groups
      const size_t ldsg = sor_lanes_lds(S, a.h, 64 * G + 2, cw, R);
      // the clamped in-frame load form in throughput launches -- more frames than CUs -- and the lane-constant slots in
      // latency launches, where the per-step v_med3 would sit on the wavefront's critical path (sor_cring 3: everywhere,
      // parity).  Measured (profiles/r06/s5, s21): B's tv_sor 4.16 -> 4.00 ms per step and its counted bytes 1.33x ->
      // 1.23x the compulsory ones, A's 1.82x -> 1.27x; the single pair 0.84 -> 0.91 ms with it everywhere.
      const bool sel = a.sor_cring >= 3 || (long)a.n > device_cus();
      auto go = [&](auto gc) {
        constexpr int CG = decltype(gc)::value;
        if (a.nop == 2) {
          if (sel) k_tv_sor_lanes<S, 0, 3, MAXT, true, R, CG, true><<<a.n, th, ldsg, s>>>(a);
          else k_tv_sor_lanes<S, 0, 3, MAXT, true, R, CG, false><<<a.n, th, ldsg, s>>>(a);
        } else {
          if (sel) k_tv_sor_lanes<S, 2, 3, MAXT, true, R, CG, true><<<a.n, th, ldsg, s>>>(a);
          else k_tv_sor_lanes<S, 2, 3, MAXT, true, R, CG, false><<<a.n, th, ldsg, s>>>(a);
        }
      };
      if constexpr (MAXT == 512) {
        if (G == 1) return go(std::integral_constant<int, 1>{});
        if (G == 2) return go(std::integral_constant<int, 2>{});
      } else {
        if (G == 3) return go(std::integral_constant<int, 3>{});
        if (G == 4) return go(std::integral_constant<int, 4>{});
        if (G == 5) return go(std::integral_constant<int, 5>{});
      }
    }
  }
  // every other form: the same rule for the clamped load form
  const bool sel = a.sor_cring >= 3 || (long)a.n > device_cus();
  auto go2 = [&](auto cr, auto sl) {
    constexpr bool CR = decltype(cr)::value, SL = decltype(sl)::value;
    if (a.nop == 2) k_tv_sor_lanes<S, 0, 3, MAXT, CR, R, 0, SL><<<a.n, th, lds, s>>>(a);
    else k_tv_sor_lanes<S, 2, 3, MAXT, CR, R, 0, SL><<<a.n, th, lds, s>>>(a);
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (cring) {
    if (sel) go2(T_{}, T_{});
    else go2(T_{}, F_{});
  } else {
    if (sel) go2(F_{}, T_{});
    else go2(F_{}, F_{});
  }
}
template <int S>
static void sor_lanes_s(const TvArgs &a, hipStream_t s) {
  if (64 * S * ((a.h + 63) / 64) <= 512)
    sor_lanes<S, 512, 1>(a, s);
  else if (64 * S * ((a.h + 63) / 64) <= 1024)
    sor_lanes<S, 1024, 1>(a, s);
  else
    sor_lanes<S, 1024, 2>(a, s);
}
// Exact-order SOR dispatch: the sweep-per-wave form while its S * ceil(h / 64) waves fit one workgroup,
// the register pipeline (one wave per row group runs all sweeps) for taller levels, the generic
// global-memory wavefront for the point SOR of the OpenMP build and degenerate sizes.
void launch_tv_sor(const TvArgs &a, hipStream_t s) {
  if (a.solverit < 1) return;
  const bool tiny = a.nop == 2 && (a.w < 2 || a.h < 2 || a.sor_point);  // point SOR (solver.c:34-78)
  if (a.sor_redblack && !tiny) {  // opt-in red-black order (not the reference's bits), levels over kLvPix pixels
    const dim3 grid(ceil_div(a.w * a.h, 256), a.n);
    for (int it = 0; it < 2 * a.solverit; ++it) {
      if (a.nop == 2) k_tv_sor_rb<0><<<grid, 256, 0, s>>>(a, it & 1);
      else k_tv_sor_rb<2><<<grid, 256, 0, s>>>(a, it & 1);
    }
    return;
  }
  const int G = (a.h + 63) / 64, G2 = (a.h + 127) / 128;  // row groups at one / two rows per lane
  const bool lanes_fit = G * a.solverit <= 16 || (a.solverit <= 3 && G2 * a.solverit <= 16 && a.sor_rows2);
  if (!tiny && !a.sor_generic && a.sor_variant != 1 && a.solverit >= 2 && a.solverit <= 4 && lanes_fit) {
    switch (a.solverit) {
      case 2: sor_lanes_s<2>(a, s); return;
      case 3: sor_lanes_s<3>(a, s); return;
      case 4: sor_lanes_s<4>(a, s); return;
    }
  }
  if (!tiny && a.h <= 1024 && a.solverit <= 4 && !a.sor_generic) {
    switch (a.solverit) {
      case 1: sor_pipe<1>(a, s); return;
      case 2: sor_pipe<2>(a, s); return;
      case 3: sor_pipe<3>(a, s); return;
      case 4: sor_pipe<4>(a, s); return;
    }
  }
  if (a.nop == 1)
    k_tv_sor<2><<<a.n, 256, 0, s>>>(a);
  else if (tiny)
    k_tv_sor<1><<<a.n, 256, 0, s>>>(a);
  else
    k_tv_sor<0><<<a.n, 256, 0, s>>>(a);
}
void launch_tv_final(const TvArgs &a, hipStream_t s) {
  k_tv_final<32><<<dim3(ceil_div(a.w, kTileW), ceil_div(a.h, 32), a.n), 256, 0, s>>>(a);
}
// OpenCV resizeAreaFast for the initial flow (oracle: ofo_init_flow_area): one thread per output value,
// the k x k block in row-major order, sum += ((a + b) + c) + d four at a time, then x 1/k^2.  The chain is
// serial by definition (exact order); it runs once per batch on the coarsest grid (a few hundred values
// per frame), its loads are issued four ahead of the adds.
__global__ __launch_bounds__(256) void k_init_area(InitArgs a) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)a.wo * a.ho * a.nop;
  if (i >= per * a.n) return;
  const int f = (int)(i / per), r = (int)(i - f * per);
  const int c = r % a.nop, px = r / a.nop, x = px % a.wo, y = px / a.wo;
  const int k = 1 << a.log2k, area = k * k;
  const float *src = a.init + (size_t)f * a.W0 * a.H0 * a.nop + c;
  auto val = [&](int j) {
    const int sy = clampi(y * k + (j >> a.log2k) - a.padt, 0, a.H0 - 1);
    const int sx = clampi(x * k + (j & (k - 1)) - a.padl, 0, a.W0 - 1);
    return src[((size_t)sy * a.W0 + sx) * a.nop] * a.sc;
  };
  float sum = 0.0f;
  int j = 0;
  for (; j <= area - 4; j += 4) {
    const float v0 = val(j), v1 = val(j + 1), v2 = val(j + 2), v3 = val(j + 3);
    sum += ((v0 + v1) + v2) + v3;
  }
  for (; j < area; ++j) sum += val(j);
  a.out[i] = sum * a.scale;
}

void launch_init_area(const InitArgs &a, hipStream_t s) {
  const long total = (long)a.n * a.wo * a.ho * a.nop;
  k_init_area<<<dim3(ceil_div(total, 256)), 256, 0, s>>>(a);
}

void launch_upsample(const UpArgs &a, hipStream_t s) {
  if (a.nop == 2 && a.log2s >= 1 && a.log2s <= 9 && (a.W0 % 4) == 0 && ((uintptr_t)a.out % 16) == 0) {
    if (a.form == 2)
      k_upsample_h<8><<<dim3(ceil_div(a.W0, kUpCols), ceil_div(a.H0, 8), a.n), 256, 0, s>>>(a);
    else if (a.form == 1)
      k_upsample_h<4><<<dim3(ceil_div(a.W0, kUpCols), ceil_div(a.H0, 4), a.n), 256, 0, s>>>(a);
    else
      k_upsample_rows<<<dim3(ceil_div(a.W0, kUpCols), ceil_div(a.H0, kUpRows), a.n), 256, 0, s>>>(a);
  } else if (a.nop == 1 && a.log2s >= 1 && a.log2s <= 9 && (a.W0 % 4) == 0 && ((uintptr_t)a.out % 16) == 0)
    k_upsample_rows1<<<dim3(ceil_div(a.W0, kUpCols), ceil_div(a.H0, kUpRows), a.n), 256, 0, s>>>(a);
  else
    k_upsample<<<dim3(ceil_div(a.W0, 256), a.H0, a.n), 256, 0, s>>>(a);
}

}  // namespace ofdis

#ifdef OFDIS_SOR_PROBE
// Probe build only: point the SOR step probe at a device buffer of 4 + 64 * 16 * 1024 * 4 uints (NULL: off).
extern "C" int ofdis_sor_probe_attach(void *dev_buffer) {
  return hipMemcpyToSymbol(HIP_SYMBOL(ofdis::g_sor_probe), &dev_buffer, sizeof(dev_buffer)) == hipSuccess ? 0 : -1;
}
#endif
