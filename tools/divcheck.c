// Exhaustive check of the FMA-corrected division by a constant used by k_patchw (div_by_const): for every
// finite float x, q1 = fma(fma(-q0, c, x), y, q0) with q0 = x * y, y = RN(1/c) against IEEE x / c.
// Build: gcc -O2 -fopenmp -ffp-contract=off -mfma -o divcheck tools/divcheck.c -lm;  run: ./divcheck 144 192 432
// (prints the mismatch counts: all of them lie below |x| = 1e-30, i.e. in the range the kernel sends to the
// IEEE division).
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <stdlib.h>
int main(int argc, char **argv) {
  for (int ai = 1; ai < argc; ++ai) {
    const float c = (float)atof(argv[ai]);
    const float y = 1.0f / c;
    long bad = 0, badnorm = 0; uint32_t first = 0;
    #pragma omp parallel for reduction(+:bad,badnorm) schedule(static)
    for (long u = 0; u < (1L << 32); ++u) {
      uint32_t b = (uint32_t)u; float x; memcpy(&x, &b, 4);
      if (!isfinite(x)) continue;
      volatile float ref = x / c;
      float q0 = x * y;
      float r = fmaf(-q0, c, x);
      float q1 = fmaf(r, y, q0);
      uint32_t r1, r2; float rr = ref; memcpy(&r1, &rr, 4); memcpy(&r2, &q1, 4);
      if (r1 != r2) { bad++; if (fabsf(x) >= 1e-30f) badnorm++; }
    }
    printf("c=%g y=%a bad=%ld bad(|x|>=1e-30)=%ld\n", c, y, bad, badnorm);
  }
  return 0;
}
