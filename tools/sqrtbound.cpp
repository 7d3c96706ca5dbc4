// Exhaustive-neighbourhood check behind sqrt_le_bound (ofdis_runtime.cpp): for every outlier threshold p/2 of
// p = 2..64, sqrtf(s) > t <=> s > bound for every float s within 2e5 ulps of the bound (monotonicity covers the
// rest).  g++ -O2 tools/sqrtbound.cpp && ./a.out  ->  "mismatches 0".
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
static float sqrt_le_bound(float t) {
  if (!(t >= 0.0f) || std::isinf(t)) return t * t;
  float s = t * t;
  while (std::sqrt(std::nextafter(s, INFINITY)) <= t) s = std::nextafter(s, INFINITY);
  while (s > 0.0f && std::sqrt(s) > t) s = std::nextafter(s, -INFINITY);
  return s;
}
int main() {
  long bad = 0, n = 0;
  for (int p = 2; p <= 64; ++p) {
    const float t = (float)p / 2, b = sqrt_le_bound(t);
    uint32_t u; std::memcpy(&u, &b, 4);
    for (long k = -200000; k <= 200000; ++k) {  // every float within 2e5 ulps of the bound
      uint32_t v = u + (uint32_t)k; float s; std::memcpy(&s, &v, 4);
      ++n; if ((std::sqrt(s) > t) != (s > b)) ++bad;
    }
    if (p == 8 || p == 12 || p == 16) printf("t=%g bound=%.9g (t*t=%.9g)\n", t, b, t * t);
  }
  printf("checked %ld, mismatches %ld\n", n, bad);
}
