// Device math helpers shared by the kernels and tools/sqrt_probe.hip (which checks them exhaustively).
#pragma once
#include <hip/hip_runtime.h>

namespace ofdis {

// Correctly rounded sqrtf for x >= +0, +inf or NaN: the sequence the compiler expands sqrtf into on gfx950
// (denormal range scaled by 2^32, v_sqrt_f32, then the neighbour ulps s -/+ 1 tested with one fma residual
// each) without its final class test, which only changes the result for negative inputs.  Bit-identical to
// sqrtf over every non-negative float (tools/sqrt_probe.hip); callers pass |d| or sums of squares.
__device__ __forceinline__ float sqrt_nonneg(float x) {
  const bool tiny = x < 0x1p-96f;
  const float xs = tiny ? x * 0x1p+32f : x;
  const float s = __builtin_amdgcn_sqrtf(xs);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u);
  const float sp = __uint_as_float(__float_as_uint(s) + 1u);
  float r = __builtin_fmaf(-sm, s, xs) <= 0.0f ? sm : s;
  r = __builtin_fmaf(-sp, s, xs) > 0.0f ? sp : r;
  return tiny ? r * 0x1p-16f : r;
}

// The same correction at a fixed scale, for 0 <= x < 2^64: x * 2^64 is at least 2^-85 for every non-zero x
// (denormals included), where v_sqrt_f32 plus the two neighbour tests is exact, and sqrt(x 2^64) 2^-32 rounds like
// sqrt(x) (both normal: power-of-two scales commute with the rounding).  Two multiplications instead of the
// compare, selects and multiplication of the conditional scaling.  Bit-identical to sqrtf over [0, 2^64)
// (tools/sqrt_probe3.hip, every float); x >= 2^64 overflows to +inf -- callers detect that and redo the exact form.
// 2^32 sqrt(x), correctly rounded, for 0 <= x < 2^64: sqrt_nonneg_s64 before its exact final scaling (callers that
// keep their sums at the 2^32 scale and rescale the totals)
__device__ __forceinline__ float sqrt_nonneg_s64_x32(float x) {
  const float xs = x * 0x1p+64f;
  const float s = __builtin_amdgcn_sqrtf(xs);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u);
  const float sp = __uint_as_float(__float_as_uint(s) + 1u);
  float r = __builtin_fmaf(-sm, s, xs) <= 0.0f ? sm : s;
  r = __builtin_fmaf(-sp, s, xs) > 0.0f ? sp : r;
  return r;
}
__device__ __forceinline__ float sqrt_nonneg_s64(float x) {
  const float xs = x * 0x1p+64f;
  const float s = __builtin_amdgcn_sqrtf(xs);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u);
  const float sp = __uint_as_float(__float_as_uint(s) + 1u);
  float r = __builtin_fmaf(-sm, s, xs) <= 0.0f ? sm : s;
  r = __builtin_fmaf(-sp, s, xs) > 0.0f ? sp : r;
  return r * 0x1p-32f;
}

}  // namespace ofdis
