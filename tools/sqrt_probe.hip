// Exhaustive check over every non-negative finite float: is (float) v_sqrt_f64((double) x) the correctly
// rounded sqrtf(x)?  And the raw v_sqrt_f32?  (Decides whether the patch kernels' L1 / pseudo-Huber losses
// can use the short form and stay bit-exact.)  Build: hipcc --offload-arch=gfx950 -O3 -o sqrt_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "../of_dis_amd/csrc/ofdis_math.h"

__global__ void k_probe(unsigned long long *bad64, unsigned long long *bad32, unsigned int *first64,
                        unsigned long long *badnn) {
  const unsigned int stride = gridDim.x * blockDim.x;
  unsigned int n64 = 0, n32 = 0, nnn = 0;
  for (unsigned int i = blockIdx.x * blockDim.x + threadIdx.x; i < 0x7f800000u; i += stride) {
    const float x = __uint_as_float(i);
    const float ref = sqrtf(x);
    const float a = (float)__builtin_amdgcn_sqrt((double)x);
    const float b = __builtin_amdgcn_sqrtf(x);
    if (__float_as_uint(a) != __float_as_uint(ref)) {
      ++n64;
      atomicMin(first64, i);
    }
    if (__float_as_uint(b) != __float_as_uint(ref)) ++n32;
    if (__float_as_uint(ofdis::sqrt_nonneg(x)) != __float_as_uint(ref)) ++nnn;
  }
  {  // +inf and +0 too
    const float xi = __uint_as_float(0x7f800000u);
    if (blockIdx.x == 0 && threadIdx.x == 0 && (ofdis::sqrt_nonneg(xi) != sqrtf(xi) || ofdis::sqrt_nonneg(0.0f) != 0.0f)) ++nnn;
  }
  atomicAdd(badnn, (unsigned long long)nnn);
  atomicAdd(bad64, (unsigned long long)n64);
  atomicAdd(bad32, (unsigned long long)n32);
}

int main() {
  unsigned long long *d, h[3];
  unsigned int *f, hf;
  hipMalloc(&d, 24);
  hipMalloc(&f, 4);
  hipMemset(d, 0, 24);
  hipMemset(f, 0xff, 4);
  k_probe<<<4096, 256>>>(d, d + 1, f, d + 2);
  hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
  hipMemcpy(&hf, f, 4, hipMemcpyDeviceToHost);
  printf("inputs %u  f64-path mismatches %llu (first 0x%08x)  raw-f32 mismatches %llu  sqrt_nonneg mismatches %llu\n",
         0x7f800000u, h[0], hf, h[1], h[2]);
  return h[2] == 0 ? 0 : 1;
}
