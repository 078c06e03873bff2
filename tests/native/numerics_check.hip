// tests/native/numerics_check.hip — TEST INFRASTRUCTURE: checks the kernels' division and square root
// (raytracing-practice_amd/csrc/rtg_numerics.hpp: div_rn, sqrt_rn) against hipcc's correctly rounded
// `x / y` and `sqrtf`, bit for bit, on random operands from the ranges the kernels use.
// Built into tests/native/libnumcheck.so by raytracing-practice_amd/Makefile; run by
// tests/test_gpu.py::test_numerics_helpers_match_ieee.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rtg_numerics.hpp"

namespace {

__device__ __forceinline__ uint64_t splitmix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// a float with a random sign, a random 23-bit mantissa and an exponent uniform in [emin, emax]
__device__ __forceinline__ float rand_float(uint64_t h, int emin, int emax) {
  const uint32_t mant = static_cast<uint32_t>(h) & 0x7fffffu;
  const int e = emin + static_cast<int>((h >> 23) % static_cast<uint64_t>(emax - emin + 1));
  const uint32_t sign = static_cast<uint32_t>(h >> 63) << 31;
  return __uint_as_float(sign | (static_cast<uint32_t>(e + 127) << 23) | mant);
}

// out[0] division mismatches, out[1] sqrt mismatches (random operands), out[2] sqrt mismatches on
// the kernel's 1 - z^2 / uniform operands, out[3] operands tested, out[4] div_rn mismatches on the
// sphere test's small divisors (2^-100 .. 2^-20); ex[0..3] the last mismatch seen
__global__ void check_kernel(uint64_t n, uint64_t seed, unsigned long long* out, float* ex) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  unsigned long long bad_div = 0, bad_sqrt = 0, bad_kern = 0, bad_wide = 0;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t h0 = splitmix(seed ^ (i * 4 + 0)), h1 = splitmix(seed ^ (i * 4 + 1));
    const uint64_t h2 = splitmix(seed ^ (i * 4 + 2)), h3 = splitmix(seed ^ (i * 4 + 3));
    // division: numerators 2^-60 .. 2^61 (1/64 of them zero, 1/64 exactly one), divisors 2^-30 .. 2^31
    float x = rand_float(h0, -60, 60);
    if ((h2 & 63) == 0) x = 0.0f;
    if ((h2 & 63) == 1) x = 1.0f;
    const float y = rand_float(h1, -30, 30);
    const float q_ieee = x / y;
    const float q = rtg::div_rn(x, y);
    if (__float_as_uint(q) != __float_as_uint(q_ieee)) {
      ++bad_div;
      ex[0] = x, ex[1] = y;
    }
    // the sphere test's near root c / q with the spec's guard (|q| >= 2^-100 reaches the division):
    // numerators 2^-60 .. 2^40, divisors 2^-100 .. 2^-20, quotients below 2^120 (c / q is a
    // distance compared with tmin and the closest hit)
    {
      const float xw = (h2 & 63) == 3 ? 0.0f : rand_float(h3, -60, 40);
      const float yw = rand_float(h0 ^ h1, -100, -20);
      const float qi = xw / yw;
      if (fabsf(qi) < 0x1p120f && __float_as_uint(rtg::div_rn(xw, yw)) != __float_as_uint(qi)) {
        ++bad_wide;
        ex[0] = xw, ex[1] = yw;
      }
    }
    // square root: 0 and 2^-90 .. 2^100
    float s = fabsf(rand_float(h3, -90, 100));
    if ((h2 & 63) == 2) s = 0.0f;
    if (__float_as_uint(rtg::sqrt_rn(s)) != __float_as_uint(sqrtf(s))) {
      ++bad_sqrt;
      ex[2] = s;
    }
    // the kernels' sqrt operands built from 24-bit uniforms: U, 1 - z^2 with z = 1 - 2U (plain and fused)
    const float u = static_cast<float>(static_cast<uint32_t>(h2 >> 40)) * 5.9604644775390625e-8f;
    const float z = 1.0f - 2.0f * u;
    const float a = fmaxf(0.0f, fmaf(-z, z, 1.0f)), b = fmaxf(0.0f, 1.0f - z * z);
    if (__float_as_uint(rtg::sqrt_rn(u)) != __float_as_uint(sqrtf(u)) ||
        __float_as_uint(rtg::sqrt_rn(a)) != __float_as_uint(sqrtf(a)) ||
        __float_as_uint(rtg::sqrt_rn(b)) != __float_as_uint(sqrtf(b))) {
      ++bad_kern;
      ex[3] = u;
    }
  }
  if (bad_div) atomicAdd(&out[0], bad_div);
  if (bad_sqrt) atomicAdd(&out[1], bad_sqrt);
  if (bad_kern) atomicAdd(&out[2], bad_kern);
  if (bad_wide) atomicAdd(&out[4], bad_wide);
}

}  // namespace

// n operands of each kind from `seed`; out[5] as in check_kernel, examples[4]. Returns 0 or a HIP error.
extern "C" int rtg_numerics_check(uint64_t n, uint64_t seed, unsigned long long out[5], float examples[4]) {
  unsigned long long* d_out = nullptr;
  float* d_ex = nullptr;
  hipError_t e = hipMalloc(&d_out, 5 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMalloc(&d_ex, 4 * sizeof(float));
  if (e == hipSuccess) e = hipMemset(d_out, 0, 5 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(d_ex, 0, 4 * sizeof(float));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(check_kernel, dim3(1024), dim3(256), 0, nullptr, n, seed, d_out, d_ex);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(out, d_out, 5 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(examples, d_ex, 4 * sizeof(float), hipMemcpyDeviceToHost);
  out[3] = n;
  if (d_out) (void)hipFree(d_out);
  if (d_ex) (void)hipFree(d_ex);
  return static_cast<int>(e);
}
