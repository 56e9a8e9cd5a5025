// Box-Muller's logf and sqrtf (csrc/mask.hip, efl_dp_noise) over the arguments it can reach.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// logf and sqrtf over the arguments Box-Muller reaches: u1 in [1e-7, 1) and -2 ln u1 in
// [2.38e-7, 32.24], normal and finite. These are the device library's own operations, in its order,
// as the compiler lowers logf / sqrtf for gfx950 (tools/dp_fastmath_check.hip compares both over
// all 2^23 values of u1 on the GPU): v_log_f32 times ln 2 as a double-float, and v_sqrt_f32 with
// the one-ulp correction by the two fma residuals. What is left out is unreachable here: the
// denormal rescaling of both, logf's non-finite select and sqrtf's zero / infinity select, about a
// dozen instructions per pair (round 5).
__device__ __forceinline__ float log_unit(float u) {
#pragma clang fp contract(off)
  const float hi = __uint_as_float(0x3f317217u), lo = __uint_as_float(0x3377d1cfu);   // ln 2 = hi + lo
  const float y = __builtin_amdgcn_logf(u);   // log2 u
  const float h = y * hi;
  float e = __builtin_fmaf(y, hi, -h);
  e = __builtin_fmaf(lo, y, e);
  return __builtin_fmaf(hi, y, e);
}

__device__ __forceinline__ float sqrt_normal(float x) {
#pragma clang fp contract(off)
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float r = __builtin_fmaf(-sm, s, x) <= 0.0f ? sm : s;
  return __builtin_fmaf(-sp, s, x) > 0.0f ? sp : r;
}

// r at the clamp u1 = 1e-7: the value the compiler folds sqrtf(-2 logf(1e-7f)) to (5.677 68...)
constexpr uint32_t kRClampBits = 0x40b5afa8u;

