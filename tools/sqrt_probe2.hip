// Exhaustive check over every non-negative float: where does the correction sequence WITHOUT the tiny-input
// scaling (s = v_sqrt_f32(x), then the neighbour ulps s -/+ 1 tested with one fma residual each) differ from
// the correctly rounded sqrtf?  Decides the threshold below which the patch kernels' L1 / pseudo-Huber loss
// must take the scaled form (ofdis_math.h sqrt_nonneg scales below 2^-96).
// Build: hipcc --offload-arch=gfx950 -O3 -o sqrt_probe2 tools/sqrt_probe2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__device__ __forceinline__ float sqrt_unscaled(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u);
  const float sp = __uint_as_float(__float_as_uint(s) + 1u);
  float r = __builtin_fmaf(-sm, s, x) <= 0.0f ? sm : s;
  r = __builtin_fmaf(-sp, s, x) > 0.0f ? sp : r;
  return r;
}

__global__ void k_probe(unsigned long long *bad, unsigned int *maxbad) {
  const unsigned int stride = gridDim.x * blockDim.x;
  unsigned int n = 0, mx = 0;
  for (unsigned int i = blockIdx.x * blockDim.x + threadIdx.x; i <= 0x7f800000u; i += stride) {
    const float x = __uint_as_float(i);
    if (__float_as_uint(sqrt_unscaled(x)) != __float_as_uint(sqrtf(x))) {
      ++n;
      mx = i > mx ? i : mx;
    }
  }
  atomicAdd(bad, (unsigned long long)n);
  atomicMax(maxbad, mx);
}

int main() {
  unsigned long long *d, h;
  unsigned int *m, hm;
  hipMalloc(&d, 8);
  hipMalloc(&m, 4);
  hipMemset(d, 0, 8);
  hipMemset(m, 0, 4);
  k_probe<<<4096, 256>>>(d, m);
  hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  hipMemcpy(&hm, m, 4, hipMemcpyDeviceToHost);
  float fm;
  memcpy(&fm, &hm, 4);
  printf("unscaled correction: %llu mismatches over [0, +inf]; largest mismatching input 0x%08x = %g (2^-96 = %g)\n",
         h, hm, fm, 0x1p-96);
  return 0;
}
