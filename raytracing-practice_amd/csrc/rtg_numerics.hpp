// rtg_numerics.hpp — correctly rounded fp32 division and square root for the gfx950 kernels, without
// the compiler's special-case steps. Shared by rtg_kernels.hip and the numerics check
// (tests/native/numerics_check.hip), which compares them with hipcc's `x / y` and `sqrtf` bit for bit
// over the operand ranges the kernels use.
#ifndef RTG_NUMERICS_HPP
#define RTG_NUMERICS_HPP
#include <hip/hip_runtime.h>

namespace rtg {
// Correctly rounded fp32 division and square root without the compiler's special-case steps.
// div_rn is the IEEE sequence hipcc emits for `x / y` (rcp, two refinements of the reciprocal and
// of the quotient) minus v_div_scale / v_div_fmas / v_div_fixup, which change nothing unless an
// operand or the quotient lies within 2^64 of the fp32 range ends (or is 0, inf, NaN): in range
// the results are the same bits, 8 VALU instead of 11. Every call site divides by a ray length,
// a radius, a refraction index or a quad denominator (>= 1e-8), and a numerator that is tiny or
// zero yields a root far below tmin either way.
__device__ __forceinline__ float div_rn(float x, float y) {
  const float r0 = __builtin_amdgcn_rcpf(y);
  const float e0 = fmaf(-y, r0, 1.0f);
  const float r = fmaf(e0, r0, r0);
  const float q0 = x * r;
  const float e1 = fmaf(-y, q0, x);
  const float q1 = fmaf(e1, r, q0);
  const float e2 = fmaf(-y, q1, x);
  return fmaf(e2, r, q1);
}
// sqrt_rn: the compiler's correctly rounded sqrt (v_sqrt_f32, then the neighbour whose residual
// changes sign) without its 2^32 pre-scaling of x < 2^-96 and its 0/inf class fix-up: exact for x
// == 0 and 2^-96 <= x < inf, 9 VALU instead of 16. Call sites: 1 - z^2 of a 24-bit uniform, a
// 24-bit uniform, 1 - cos^2 and |1 - |perp|^2| (each 0 or >= 2^-25), and |v|^2 of ray directions
// (camera rays, and scatter directions kept >= 1e-8 per axis by near_zero). The sphere test's
// discriminant, which can be arbitrarily small, keeps sqrtf.
__device__ __forceinline__ float sqrt_rn(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float lo = __int_as_float(__float_as_int(s) - 1);
  const float hi = __int_as_float(__float_as_int(s) + 1);
  const float rlo = fmaf(-lo, s, x);
  const float rhi = fmaf(-hi, s, x);
  const float t = rlo <= 0.0f ? lo : s;
  return rhi > 0.0f ? hi : t;
}
}  // namespace rtg
#endif
