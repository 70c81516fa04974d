// fleet_amd/csrc/teacher_math.h -- arithmetic of the sampler's mode-1 teacher
// forward pass, host+device so that tests/native can check it
// on the CPU against the library the reference links.
//
// The teacher is a mojo network (commonLib/cppNN, built -O0 for x86-64 SSE: one
// binary32 rounding per operation, no contraction); its only transcendental is
// std::exp(float), i.e. libm's expf. glibc_expf below restates the expf of the
// reference's libm -- glibc 2.35 (this image), sysdeps/ieee754/flt-32/e_expf.c
// with the __exp2f_data tables of e_exp2f_data.c, in the x86-64 ifunc variant
// selected on CPUs with FMA (__expf_fma: the same C compiled with -mfma, so the
// multiply-adds below are fused). Published algorithm: exp(x) = 2^(k/32) *
// 2^(r/32) with k = round(x*32/ln2), a 32-entry table for 2^(i/32) and a cubic
// in r, all in binary64, rounded once to binary32. Checked against the libm
// expf on all 2^32 inputs (tests/native/digest_ref.cpp fn 18 vs the device
// digest, and tests/test_teacher.py on the CPU).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define FLEET_TM __host__ __device__ __forceinline__
#else
#define FLEET_TM static inline __attribute__((always_inline))
#endif

namespace fleet {

// __exp2f_data.tab[i] = bits(2^(i/32)) - (i << 47)
#define FLEET_EXP2F_TAB                                                                                      \
  {0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,               \
   0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,               \
   0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,               \
   0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,               \
   0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,               \
   0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,               \
   0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,               \
   0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull}

FLEET_TM float glibc_expf(float x) {
  constexpr uint64_t tab[32] = FLEET_EXP2F_TAB;
  constexpr double inv_ln2_n = 0x1.71547652b82fep+0 * 32;  // __exp2f_data.invln2_scaled
  constexpr double shift = 0x1.8p+52;                      // round-to-int by addition
  constexpr double c0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, c1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
                   c2 = 0x1.62e42ff0c52d6p-1 / 32;           // __exp2f_data.poly_scaled
  const uint32_t ux = __builtin_bit_cast(uint32_t, x);
  const uint32_t abstop = (ux >> 20) & 0x7ffu;
  if (abstop >= 0x42bu) {                        // |x| >= 88 or NaN
    if (ux == 0xff800000u) return 0.0f;          // -inf
    if (abstop >= 0x7f8u) return x + x;          // +inf, NaN
    if (x > 0x1.62e42ep6f) return __builtin_inff();  // overflow
    if (x < -0x1.9fe368p6f) return 0.0f;         // underflow
    if (x < -0x1.9d1d9ep6f) return 0x1p-149f;    // __math_may_uflowf: 0x1.4p-75f * 0x1.4p-75f
  }
  const double xd = (double)x;
  double kd = __builtin_fma(inv_ln2_n, xd, shift);
  const uint64_t ki = __builtin_bit_cast(uint64_t, kd);
  kd -= shift;
  const double r = __builtin_fma(inv_ln2_n, xd, -kd);
  const uint64_t t = tab[ki % 32] + (ki << 47);
  const double s = __builtin_bit_cast(double, t);
  const double z = __builtin_fma(c0, r, c1);
  const double r2 = r * r;
  double y = __builtin_fma(c2, r, 1.0);
  y = __builtin_fma(z, r2, y);
  return (float)(y * s);
}

// activation.h:161-176 elu::fc on one value: the bias added, then
// 0.1f*(exp(v) - 1) for v < 0
FLEET_TM float mojo_elu(float x, float bias) {
  const float v = x + bias;
  return v < 0.0f ? 0.1f * (glibc_expf(v) - 1.0f) : v;
}

// x86-64 `(int)x` (cvttss2si): INT_MIN when |x| >= 2^31 or x is NaN
FLEET_TM int32_t mojo_cvtt(float x) { return __builtin_fabsf(x) < 2147483648.0f ? (int32_t)x : INT32_MIN; }

// semi_stochastic_pooling_layer::accumulate_signal (layer.h:481-556) for one
// window: v[] in the reference's scan order (rows, then columns). The largest
// and second largest by strict `<`; the pick is the largest unless
// r = 34909 % 100 = 9 exceeds (int)(100*max/(max+max2)) in a training forward
// (forward(..., _train = 1) in uniformSample, cppNN_backend.cpp:603).
template <int P>
FLEET_TM float mojo_semi_pool(const float (&v)[P * P], bool train) {
  float mx = v[0], mx2 = v[0];
  int mi = 0, mi2 = 0;
#pragma unroll
  for (int i = 0; i < P * P; ++i) {
    if (mx < v[i]) {
      mx2 = mx;
      mi2 = mi;
      mx = v[i];
      mi = i;
    } else if (mx2 < v[i]) {
      mx2 = v[i];
      mi2 = i;
    }
  }
  const float denom = mx + mx2;
  if (denom == 0.0f) return v[mi];
  const int32_t t1 = mojo_cvtt(100.0f * mx / (mx + mx2));
  return (9 <= t1 || !train) ? v[mi] : v[mi2];
}

}  // namespace fleet
