// Check of the FMA-corrected division by a per-patch divisor used by the LLT solves of the patch kernels
// (llt_div in ofdis_kernels.hip): with y = RN(1/L) computed once per patch by an IEEE division,
//   q0 = a * y,  r = fma(-q0, L, a),  q = fma(r, y, q0)
// against IEEE a / L, for |L| in [2^-30, 2^30] and |a| in [2^-60, 2^60] (the kernel sends every other
// numerator or divisor -- zero, tiny, huge, inf, NaN -- to the IEEE division in a wave-uniform branch).
// Markstein's theorem (y within half an ulp of 1/L, q0 within an ulp of a/L, no underflow) says q = RN(a/L);
// this program tests it:
//   part 1: every divisor significand (2^23) at a random exponent, 256 random numerators each (2^31 pairs);
//   part 2: every numerator significand (2^23) for 512 divisors (random, near powers of two, all-ones
//           significands), numerator exponents drawn over the whole range (2^32 pairs);
//   part 3: both operands at the ends of their ranges.
// Build: gcc -O2 -fopenmp -ffp-contract=off -mfma -o /tmp/divcheck_l tools/divcheck_l.c -lm;  run: /tmp/divcheck_l
// Prints the pairs checked and the mismatches (expected: 0).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static inline float f_of(uint32_t b) { float x; memcpy(&x, &b, 4); return x; }
static inline uint32_t b_of(float x) { uint32_t b; memcpy(&b, &x, 4); return b; }
static inline uint64_t mix(uint64_t x) {  // splitmix64
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
// float with the given significand bits (23) and unbiased exponent e, sign s
static inline float mk(uint32_t sig, int e, int s) { return f_of(((uint32_t)s << 31) | ((uint32_t)(e + 127) << 23) | (sig & 0x7fffff)); }

static inline int check(float a, float L, float y) {
  volatile float ref = a / L;
  const float q0 = a * y;
  const float r = fmaf(-q0, L, a);
  const float q = fmaf(r, y, q0);
  return b_of(q) != b_of(ref);
}

int main(void) {
  long n1 = 0, bad1 = 0;
#pragma omp parallel for reduction(+ : n1, bad1) schedule(dynamic, 4096)
  for (long sig = 0; sig < (1L << 23); ++sig) {
    uint64_t h = mix((uint64_t)sig * 7919u);
    const float L = mk((uint32_t)sig, (int)(h % 61) - 30, (int)((h >> 8) & 1));
    const float y = 1.0f / L;
    for (int k = 0; k < 256; ++k) {
      h = mix(h + (uint64_t)k);
      const float a = mk((uint32_t)h, (int)((h >> 32) % 121) - 60, (int)((h >> 40) & 1));
      ++n1;
      bad1 += check(a, L, y);
    }
  }
  printf("part 1: %ld pairs, %ld mismatches\n", n1, bad1);

  float Ls[512];
  int nl = 0;
  const uint32_t special[] = {0x000000, 0x7fffff, 0x7ffffe, 0x000001, 0x400000, 0x3fffff, 0x555555, 0x2aaaab, 0x124925};
  for (unsigned i = 0; i < sizeof special / sizeof special[0]; ++i) Ls[nl++] = mk(special[i], 0, 0);
  for (uint64_t i = 1; nl < 512; ++i) Ls[nl++] = mk((uint32_t)mix(i * 31337u), (int)(mix(i) % 61) - 30, (int)(i & 1));
  long n2 = 0, bad2 = 0;
  for (int li = 0; li < nl; ++li) {
    const float L = Ls[li], y = 1.0f / L;
#pragma omp parallel for reduction(+ : n2, bad2) schedule(static)
    for (long sig = 0; sig < (1L << 23); ++sig) {
      const uint64_t h = mix((uint64_t)sig ^ ((uint64_t)li << 40));
      const float a = mk((uint32_t)sig, (int)(h % 121) - 60, (int)((h >> 8) & 1));
      ++n2;
      bad2 += check(a, L, y);
    }
  }
  printf("part 2: %ld pairs, %ld mismatches\n", n2, bad2);

  long n3 = 0, bad3 = 0;
  const int eL[] = {-30, -29, 29, 30}, eA[] = {-60, -59, 59, 60};
#pragma omp parallel for reduction(+ : n3, bad3) schedule(static) collapse(2)
  for (int i = 0; i < 4; ++i)
    for (long s = 0; s < (1L << 20); ++s) {
      const uint64_t h = mix((uint64_t)s * 97u + (uint64_t)i);
      const float L = mk((uint32_t)h, eL[i], (int)((h >> 60) & 1)), y = 1.0f / L;
      for (int j = 0; j < 4; ++j) {
        const float a = mk((uint32_t)(h >> 23), eA[j], (int)((h >> 61) & 1));
        ++n3;
        bad3 += check(a, L, y);
      }
    }
  printf("part 3: %ld pairs, %ld mismatches\n", n3, bad3);
  return (bad1 | bad2 | bad3) != 0;
}
