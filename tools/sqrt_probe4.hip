// Exhaustive: which side of the correctly rounded square root the raw v_sqrt_f32 lands on, for the scaled inputs
// sqrt_nonneg_s64 feeds it (x * 2^64, x every non-negative float below 2^64), and whether a ONE-sided
// neighbour test (only s - 1 ulp, or only s + 1 ulp) already gives the correctly rounded result everywhere.
// Build: hipcc --offload-arch=gfx950 -O3 -I of_dis_amd/csrc -o tools/bin/sqrt_probe4 tools/sqrt_probe4.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "ofdis_math.h"

__device__ __forceinline__ float sqrt_lo_only(float x) {  // s may be one ulp above: test s - 1 ulp only
  const float xs = x * 0x1p+64f;
  const float s = __builtin_amdgcn_sqrtf(xs);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u);
  return (__builtin_fmaf(-sm, s, xs) <= 0.0f ? sm : s) * 0x1p-32f;
}
__device__ __forceinline__ float sqrt_hi_only(float x) {  // s may be one ulp below: test s + 1 ulp only
  const float xs = x * 0x1p+64f;
  const float s = __builtin_amdgcn_sqrtf(xs);
  const float sp = __uint_as_float(__float_as_uint(s) + 1u);
  return (__builtin_fmaf(-sp, s, xs) > 0.0f ? sp : s) * 0x1p-32f;
}

// c[0..4]: raw - cr == -1, 0, +1, other; c[5]: lo-only mismatches; c[6]: hi-only mismatches
__global__ void k_probe(unsigned long long *c, unsigned int lo, unsigned int hi) {
  const unsigned int stride = gridDim.x * blockDim.x;
  unsigned int n[7] = {0, 0, 0, 0, 0, 0, 0};
  for (unsigned int i = lo + blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += stride) {
    const float x = __uint_as_float(i);
    const float xs = x * 0x1p+64f;
    const int raw = (int)__float_as_uint(__builtin_amdgcn_sqrtf(xs));
    const float cr = sqrtf(x);
    const int crs = (int)__float_as_uint(cr * 0x1p+32f);
    const int d = raw - crs;
    n[d == -1 ? 0 : d == 0 ? 1 : d == 1 ? 2 : 3]++;
    n[5] += __float_as_uint(sqrt_lo_only(x)) != __float_as_uint(cr);
    n[6] += __float_as_uint(sqrt_hi_only(x)) != __float_as_uint(cr);
  }
  for (int k = 0; k < 7; ++k)
    if (n[k]) atomicAdd(&c[k], (unsigned long long)n[k]);
}

int main() {
  unsigned long long *d, h[7];
  hipMalloc(&d, sizeof(h));
  hipMemset(d, 0, sizeof(h));
  k_probe<<<8192, 256>>>(d, 0u, 0x5f800000u);  // [0, 2^64)
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("v_sqrt_f32(x * 2^64) - correctly rounded, over x in [0, 2^64): -1: %llu  0: %llu  +1: %llu  other: %llu\n",
         h[0], h[1], h[2], h[3]);
  printf("one-sided corrections vs sqrtf: s-1ulp test only: %llu mismatches; s+1ulp test only: %llu mismatches\n",
         h[5], h[6]);
  return 0;
}
