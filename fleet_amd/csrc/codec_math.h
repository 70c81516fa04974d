// fleet_amd/csrc/codec_math.h -- the FLeet decimal fixed-point codec arithmetic,
// host+device (the host build exists only so tests/native can check the fast
// paths exhaustively against the oracle on CPU).
//
// Bit-exact restatement of commonLib/cpp_utils/Base64.cpp:37-103 as the
// reference's x86-64 SSE build computes it: one IEEE binary32 RNE rounding per
// multiply/divide, `(int)` = cvttss2si. Compile with -ffp-contract=off; every
// fused multiply-add below is explicit.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define FLEET_HD __host__ __device__ __forceinline__
#else
#define FLEET_HD static inline __attribute__((always_inline))
#endif
// compile-time evaluable (table images, codec_device.h)
#define FLEET_HDC FLEET_HD constexpr

namespace fleet {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

// RN(0.1) and RN(0.1 - RN(0.1)).
constexpr float kTenthHi = 0x1.99999ap-4f;
constexpr float kTenthLo = -0x1.99999ap-30f;

FLEET_HD uint32_t f2u(float x) { return __builtin_bit_cast(uint32_t, x); }
FLEET_HD float u2f(uint32_t x) { return __builtin_bit_cast(float, x); }

// Correctly rounded t/10 in two ops (mul + fma): t*hi exact inside the fma plus
// RN(t*lo) is within 2^-49 (relative) of t/10, while t/10 is never closer than
// 2^-27.3 to a binary32 rounding midpoint (10*midpoint - t is a nonzero odd
// multiple of the finer ulp). Exhaustively checked for every binary32 t with
// |t| >= 1e-30 (tests/test_native_math.py); int2float never divides values
// below 1e-9 in magnitude. div10(-0.0) = +0.0, as -0.0/10 is not needed:
// int2float starts from (float)code, never -0.0.
FLEET_HD float div10(float t) { return __builtin_fmaf(t, kTenthHi, t * kTenthLo); }

// RN((0.1 - RN(0.1)) / 10): a chain U_j = U_{j-1}/10 may take step j's small
// term U_{j-1}*lo as U_{j-2}*kTenthLo2. U_{j-1} = U_{j-2}/10 * (1 + 2^-24 at
// most), so the addend is within 2^-46 of t*(0.1 - RN(0.1)) relative to t/10 --
// still far inside the 2^-27.3 midpoint margin -- and each step after the
// first is ONE dependent fma (the mul runs a step ahead). Used by q_lat;
// verified with it over its whole domain (tests/native, digest fn 12).
constexpr float kTenthLo2 = -0x1.47ae14p-33f;
FLEET_HD f2 div10x2(f2 t) {
  return __builtin_elementwise_fma(t, f2{kTenthHi, kTenthHi}, t * f2{kTenthLo, kTenthLo});
}

// x86-64 `(int)x` (cvttss2si): INT_MIN when |x| >= 2^31 or x is NaN.
FLEET_HD int32_t cvtt(float x) { return __builtin_fabsf(x) < 2147483648.0f ? (int32_t)x : INT32_MIN; }

// Base64::numDigits (Base64.cpp:37-46): decimal digits of n, '-' counted.
FLEET_HD int num_digits(int32_t n) {
  uint32_t a = n < 0 ? 0u - (uint32_t)n : (uint32_t)n;
  int d = n < 0;
  d += a >= 1u;
  d += a >= 10u;
  d += a >= 100u;
  d += a >= 1000u;
  d += a >= 10000u;
  d += a >= 100000u;
  d += a >= 1000000u;
  d += a >= 10000000u;
  d += a >= 100000000u;
  d += a >= 1000000000u;
  return d;
}

// ------------------------------------------------------------ general, exact

// Base64::int2float (Base64.cpp:91-98): k = 9 - |c % 10| divisions of (float)c.
FLEET_HD float dec(int32_t c) {
  int dd = c % 10;
  dd = dd < 0 ? -dd : dd;
  float t = (float)c;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    float q = div10(t);
    t = (j + dd < 9) ? q : t;
  }
  return t;
}

// Base64::float2int (Base64.cpp:60-73): 9 - d multiplications by 10,
// truncation, last decimal digit replaced by d.
FLEET_HD int32_t enc(float x) {
  int d = num_digits(cvtt(x));
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    float w = x * 10.0f;
    x = (j + d < 9) ? w : x;
  }
  int32_t t = cvtt(x);
  int32_t lsb = t % 10;
  uint32_t u = (uint32_t)t - (uint32_t)lsb;
  u = t >= 0 ? u + (uint32_t)d : u - (uint32_t)d;
  return (int32_t)u;
}

// Q = int2float o float2int: what the next JNI op decodes after an encode.
FLEET_HD float q(float x) { return dec(enc(x)); }

// ------------------------------------------------------------- fast paths
// Exact only under their stated preconditions; callers test the precondition
// per value and send the rest through dec()/q() (kernels.hip, compaction).

// |c| % 10 == 0 (int2float then divides exactly 9 times): modular-inverse
// divisibility test, n % 10 == 0 <=> ror(n * 5^-1 mod 2^32, 1) <= (2^32-1)/10.
FLEET_HD bool dec9_ok(int32_t c) {
  uint32_t a = c < 0 ? 0u - (uint32_t)c : (uint32_t)c;
  uint32_t m = a * 0xCCCCCCCDu;
  uint32_t r = (m >> 1) | (m << 31);
  return r <= 0x19999999u;
}

FLEET_HD float d9(float t) {
#pragma unroll
  for (int j = 0; j < 9; ++j) t = div10(t);
  return t;
}
FLEET_HD f2 d9x2(f2 t) {
#pragma unroll
  for (int j = 0; j < 9; ++j) t = div10x2(t);
  return t;
}

// int2float(c) when dec9_ok(c)
FLEET_HD float dec_fast(int32_t c) { return d9((float)c); }
FLEET_HD f2 dec_fast2(int32_t c0, int32_t c1) { return d9x2(f2{(float)c0, (float)c1}); }

// Q(x) when |x| < 1 (numDigits((int)x) == 0): 9 multiplications, truncation to
// a multiple of 10 (the last digit becomes 0), then 9 divisions. The sign is
// put on (float)code before dividing: code 0 gives -0.0 there, which div10
// turns into +0.0 exactly like int2float(0).
FLEET_HD float q_fast(float x) {
  float X = __builtin_fabsf(x);
#pragma unroll
  for (int j = 0; j < 9; ++j) X = X * 10.0f;
  uint32_t n = (uint32_t)X;  // X < 1e9
  uint32_t c = (n / 10u) * 10u;
  float t = u2f(f2u((float)c) | (f2u(x) & 0x80000000u));
  return d9(t);
}
FLEET_HD f2 q_fast2(f2 x) {
  f2 X = __builtin_elementwise_abs(x);
#pragma unroll
  for (int j = 0; j < 9; ++j) X = X * f2{10.0f, 10.0f};
  uint32_t n0 = (uint32_t)X.x, n1 = (uint32_t)X.y;
  uint32_t c0 = (n0 / 10u) * 10u, c1 = (n1 / 10u) * 10u;
  f2 t = f2{u2f(f2u((float)c0) | (f2u(x.x) & 0x80000000u)), u2f(f2u((float)c1) | (f2u(x.y) & 0x80000000u))};
  return d9x2(t);
}

// precondition of q_fast (also false for NaN)
FLEET_HD bool q_ok(float x) { return __builtin_fabsf(x) < 1.0f; }

// ------------------------------------------------- variable-length fast paths
// For numDigits d <= 9 the reference runs k = 9 - d in [0, 9] multiplications
// and as many divisions. Every chain step is the same operation, so each chain
// is computed as groups of 2, 1, 2 and 4 steps, each kept or dropped by one
// select: with e = (k >= 8) and k' = k - 2e = 4*b2 + 2*b1 + b0, k = 2e + k'.
// 9 steps and 4 selects instead of 9 per-step selects.
struct Steps {
  bool e, b0, b1, b2;
};
FLEET_HDC Steps steps_of(uint32_t k) {
  const bool e = k >= 8u;
  const uint32_t r = k - (e ? 2u : 0u);
  return Steps{e, (r & 1u) != 0, (r & 2u) != 0, (r & 4u) != 0};
}

// Digit-count table indexed by e = frexp exponent (|x| in [2^(e-1), 2^e)):
// numDigits(trunc|x|) = base[e] + (|x| >= 10^base[e]).
struct DigitEntry {
  uint32_t base;
  float thr;
};
#define FLEET_DIGIT_TABLE                                                                                  \
  {{0, __builtin_inff()}, {1, 10.f}, {1, 10.f}, {1, 10.f}, {1, 10.f}, {2, 100.f}, {2, 100.f}, {2, 100.f}, \
   {3, 1e3f}, {3, 1e3f}, {3, 1e3f}, {4, 1e4f}, {4, 1e4f}, {4, 1e4f}, {4, 1e4f}, {5, 1e5f}, {5, 1e5f},     \
   {5, 1e5f}, {6, 1e6f}, {6, 1e6f}, {6, 1e6f}, {7, 1e7f}, {7, 1e7f}, {7, 1e7f}, {7, 1e7f}, {8, 1e8f},      \
   {8, 1e8f}, {8, 1e8f}, {9, 1e9f}, {9, 1e9f}, {9, 1e9f}, {10, 1e10f}}

// 10^i for i = -1..10 (exact in binary32 for i >= 0), indexed i + 1
constexpr float kPow10Tab[12] = {0.1f, 1.f, 10.f, 100.f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
#define kPow10 (kPow10Tab + 1)

FLEET_HD int frexp_exp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_frexp_expf(x);
#else
  int e = 0;
  (void)__builtin_frexpf(x, &e);
  return e;
#endif
}

// numDigits((int)x) for |x| < 2^31 (table: DigitEntry[32])
FLEET_HD int digits_of(float x, const DigitEntry* tab) {
  float ax = __builtin_fabsf(x);
  int e = frexp_exp(ax);
  e = e < 0 ? 0 : e > 31 ? 31 : e;
  const DigitEntry t = tab[e];
  return (int)t.base + (ax >= t.thr) + (x <= -1.0f);
}

// numDigits((int)x) on the q_gen domain by compares only (no table load:
// for latency-bound callers).
FLEET_HD int digits_cmp(float x) {
  const float ax = __builtin_fabsf(x);
  return (ax >= 1.0f) + (ax >= 10.0f) + (ax >= 100.0f) + (ax >= 1e3f) + (ax >= 1e4f) + (ax >= 1e5f) +
         (ax >= 1e6f) + (ax >= 1e7f) + (ax >= 1e8f) + (x <= -1.0f);
}

// Q(x) for -1e8 < x < 1e9 (numDigits((int)x) <= 9).
FLEET_HD bool q_gen_ok(float x) { return x < 1e9f && x > -1e8f; }

FLEET_HD float steps_mul10(float X, Steps s) {
  float Y = X * 10.0f;
  Y = Y * 10.0f;
  X = s.e ? Y : X;
  Y = X * 10.0f;
  X = s.b0 ? Y : X;
  Y = X * 10.0f;
  Y = Y * 10.0f;
  X = s.b1 ? Y : X;
  Y = X * 10.0f;
  Y = Y * 10.0f;
  Y = Y * 10.0f;
  Y = Y * 10.0f;
  return s.b2 ? Y : X;
}
FLEET_HD float steps_div10(float t, Steps s) {
  float u = div10(div10(t));
  t = s.e ? u : t;
  u = div10(t);
  t = s.b0 ? u : t;
  u = div10(div10(t));
  t = s.b1 ? u : t;
  u = div10(div10(div10(div10(t))));
  return s.b2 ? u : t;
}
FLEET_HD f2 sel2(bool a, bool b, f2 y, f2 x) { return f2{a ? y.x : x.x, b ? y.y : x.y}; }
FLEET_HD f2 steps_mul10x2(f2 X, Steps s0, Steps s1) {
  const f2 ten = f2{10.0f, 10.0f};
  f2 Y = X * ten;
  Y = Y * ten;
  X = sel2(s0.e, s1.e, Y, X);
  Y = X * ten;
  X = sel2(s0.b0, s1.b0, Y, X);
  Y = X * ten;
  Y = Y * ten;
  X = sel2(s0.b1, s1.b1, Y, X);
  Y = X * ten;
  Y = Y * ten;
  Y = Y * ten;
  Y = Y * ten;
  return sel2(s0.b2, s1.b2, Y, X);
}
FLEET_HD f2 steps_div10x2(f2 t, Steps s0, Steps s1) {
  f2 u = div10x2(div10x2(t));
  t = sel2(s0.e, s1.e, u, t);
  u = div10x2(t);
  t = sel2(s0.b0, s1.b0, u, t);
  u = div10x2(div10x2(t));
  t = sel2(s0.b1, s1.b1, u, t);
  u = div10x2(div10x2(div10x2(div10x2(t))));
  return sel2(s0.b2, s1.b2, u, t);
}

// |code| = 10*(n/10) + d with n = trunc(|x| * 10^(9-d)) (Base64.cpp:64-70)
FLEET_HD float signed_code_float(uint32_t n, int d, float x) {
  uint32_t c = (n / 10u) * 10u + (uint32_t)d;
  return u2f(f2u((float)c) | (f2u(x) & 0x80000000u));
}

FLEET_HD float q_gen_d(float x, int d) {
  const Steps st = steps_of((uint32_t)(9 - d));
  const float X = steps_mul10(__builtin_fabsf(x), st);
  return steps_div10(signed_code_float((uint32_t)X, d, x), st);
}
// table lookup for the digit count (throughput paths) / compares (latency paths)
FLEET_HD float q_gen(float x, const DigitEntry* tab) { return q_gen_d(x, digits_of(x, tab)); }
FLEET_HD float q_gen_lat(float x) { return q_gen_d(x, digits_cmp(x)); }

// float2int(x) on the q_gen domain: the code itself (client-side encode)
FLEET_HD int32_t enc_gen(float x, const DigitEntry* tab) {
  const int d = digits_of(x, tab);
  const float X = steps_mul10(__builtin_fabsf(x), steps_of((uint32_t)(9 - d)));
  const uint32_t n = (uint32_t)X;
  const uint32_t c = (n / 10u) * 10u + (uint32_t)d;
  return x < 0.0f ? -(int32_t)c : (int32_t)c;
}
// float2int(x) for |x| < 1: 9 multiplications, last digit 0
FLEET_HD int32_t enc_fast(float x) {
  float X = __builtin_fabsf(x);
#pragma unroll
  for (int j = 0; j < 9; ++j) X = X * 10.0f;
  const uint32_t n = (uint32_t)X;
  const uint32_t c = (n / 10u) * 10u;
  return x < 0.0f ? -(int32_t)c : (int32_t)c;
}
FLEET_HD f2 q_gen2(f2 x, const DigitEntry* tab) {
  const int d0 = digits_of(x.x, tab), d1 = digits_of(x.y, tab);
  const Steps s0 = steps_of((uint32_t)(9 - d0)), s1 = steps_of((uint32_t)(9 - d1));
  const f2 X = steps_mul10x2(__builtin_elementwise_abs(x), s0, s1);
  const f2 t = f2{signed_code_float((uint32_t)X.x, d0, x.x), signed_code_float((uint32_t)X.y, d1, x.y)};
  return steps_div10x2(t, s0, s1);
}

// 10*floor(n/10) + d as a signed float, n < 2^30: floor(n/10) = mulhi(n, ceil(2^32/10))
// (error n*0.4/2^32 < 0.1) -- one dependent op less than n/10u.
FLEET_HD float code_float_lat(uint32_t n, uint32_t d, float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t q = __umulhi(n, 0x1999999Au);
#else
  const uint32_t q = (uint32_t)(((uint64_t)n * 0x1999999Au) >> 32);
#endif
  return u2f(f2u((float)(q * 10u + d)) | (f2u(x) & 0x80000000u));
}

// Q(x) on the q_gen domain for the serial accumulation (one value per lane, a
// single wave: bound by issue slots AND the dependent chain, so both are cut).
//   * sign folding: w = 10|x| when x <= -1 ('-' counts as a digit), else |x|;
//     then numDigits((int)x) = #{m in 0..8 : w >= 10^m}. RN(10|x|) < 10^m iff
//     |x| < 10^(m-1) for these powers (10*ulp(f) is 0.625 or 1.25 ulp(10^m)),
//     so nine compares give both d (as carries) and the keep conditions
//     (step j <= k = 9 - d kept iff w < 10^(9-j)).
//   * the 9-step x10 chain runs from |x| unconditionally; a select chain
//     tracking it keeps X_k.
//   * the k-step /10 chain is one dependent fma per step, U_j = fma(U_{j-1},
//     RN(0.1), a_j), with a_{j+1} = U_{j-1} * kTenthLo2 computed alongside (see
//     kTenthLo2); a select chain keeps U_k.
FLEET_HD float q_lat(float x) {
  const float ax = __builtin_fabsf(x);
  const float w = x <= -1.0f ? ax * 10.0f : ax;
  bool big[9];
  int d = 0;
#pragma unroll
  for (int m = 0; m <= 8; ++m) {
    big[m] = w >= kPow10[m];
    d += big[m];
  }
  float X = ax, t = ax;
#pragma unroll
  for (int j = 1; j <= 9; ++j) {
    X = X * 10.0f;
    t = big[9 - j] ? t : X;
  }
  const float cf = code_float_lat((uint32_t)t, (uint32_t)d, x);
  float U = cf, a = cf * kTenthLo, r = cf;
#pragma unroll
  for (int j = 1; j <= 9; ++j) {
    const float Un = __builtin_fmaf(U, kTenthHi, a);  // the only dependent op per step
    a = U * kTenthLo2;                                 // next step's small term, off the chain
    U = Un;
    r = big[9 - j] ? r : U;
  }
  return r;
}

// --------------------------------------- multiplier-table variable-length Q
// The throughput form of q_gen. Measured on gfx950 (scripts/ubench3.hip): f32
// mul/fma issue in ~2.4 cycles per wave64 instruction, integer/convert/select
// ops in ~4, packed f32 ops in ~8 (slower than two scalar ops). So the step
// selection is done with multiplications instead of selects: every value runs
// the full 9-step chains, and a step that the reference does not take
// multiplies by 1 (x10 chain) or computes fma(t, 1, t*0) = t (/10 chain), both
// exact identities. The per-value step multipliers (groups of 2, 1, 2 and 4
// steps, Steps) come from a 16-entry LDS table indexed by the digit count d;
// d itself from a 512-entry table indexed by the top 9 bits of x (sign and
// biased exponent) plus one compare with the power of ten inside that binade.
struct alignas(16) MulEntry {
  float m[4];  // x10 chain group multipliers: 10 (step taken) or 1
  float h[4];  // /10 chain: fma(t, h, t*kTenthLo) = div10(t) (h = RN(0.1), taken) or t (h = 1)
};
// One small term for both kinds of /10 step: a taken step needs t*lo within
// 40 % of t*(0.1 - RN(0.1)) (div10's 2^-27.3 midpoint margin, 2^-26 scale of
// the term), and an identity step fma(t, 1, t*kTenthLo) = RN(t*(1 - 1.5e-9))
// = t because |t*kTenthLo| < half an ulp of t (2^-25 |t| at least); t is never
// +-0 in a chain with identity steps (codes there end in a digit count >= 1).
// Checked over every input by the multiplier-table digests (fn 13-15) and
// tests/native/check_math.cpp mt.
FLEET_HDC MulEntry mul_entry(uint32_t d) {  // d = numDigits; d > 9 (slow marker): identity
  MulEntry e{};
  const bool ok = d <= 9u;
  const Steps s = steps_of(ok ? 9u - d : 0u);
  const bool g[4] = {ok && s.e, ok && s.b0, ok && s.b1, ok && s.b2};
  for (int i = 0; i < 4; ++i) {
    e.m[i] = g[i] ? 10.0f : 1.0f;
    e.h[i] = g[i] ? kTenthHi : 1.0f;
  }
  return e;
}

// Digit table entry i = (sign << 8) | biased exponent of x. The binade holds at
// most one power of ten, thr: numDigits((int)x) is dlo for |x| < thr and dhi =
// dlo + 1 for |x| >= thr ('-' counts, Base64.cpp:37-46). The entry keeps
// base = dlo + 1, so d = base - (|x| < thr) is three integer ops (sub, shift,
// sub) with no select or bit-field extract. d > 9 marks values outside the
// q_gen domain (-1e8 < x < 1e9), NaN and inf (callers send those through the
// general codec): base = 10 where only dhi leaves the domain (dlo = 9), 15
// where both do. The threshold is kept as bits WITH the entry's sign bit: x's
// bits and thr's then share bit 31, so bits - thr borrows exactly when
// |x| < thr and no |x| mask is needed.
struct alignas(8) VarEntry {
  uint32_t thr;  // bits of the threshold | the entry's sign bit
  uint32_t base;
};
constexpr uint32_t kSlowDigits = 15u;
struct DigitPair {
  float thr;
  uint32_t dlo, dhi;  // kSlowDigits when > 9
};
FLEET_HDC DigitPair digit_pair(uint32_t i) {
  constexpr DigitEntry dig[32] = FLEET_DIGIT_TABLE;
  const uint32_t neg = (i >> 8) & 1u;
  const int e = (int)(i & 255u) - 126;  // |x| in [2^(e-1), 2^e) for normal x
  if (e <= 0) return DigitPair{__builtin_inff(), 0u, 0u};  // |x| < 1: (int)x == 0, d = 0
  const DigitEntry t = dig[e > 31 ? 31 : e];
  uint32_t dlo = t.base + neg, dhi = t.base + 1u + neg;
  dlo = dlo > 9u ? kSlowDigits : dlo;
  dhi = dhi > 9u ? kSlowDigits : dhi;
  return DigitPair{t.thr, dlo, dhi};
}
FLEET_HDC VarEntry var_entry(uint32_t i) {
  const DigitPair p = digit_pair(i);
  return VarEntry{__builtin_bit_cast(uint32_t, p.thr) | (((i >> 8) & 1u) << 31),
                  p.dlo <= 9u ? p.dlo + 1u : kSlowDigits};
}

// numDigits((int)x) on the q_gen domain, a value > 9 outside it. bits - thr
// borrows iff |x| < thr (both carry x's sign bit, the magnitudes are below
// 2^31). `ab` (the bits of |x|) is unused, kept for the callers' signature.
FLEET_HD uint32_t var_digits_ab(uint32_t bits, uint32_t ab, const VarEntry* vt) {
  (void)ab;
  const VarEntry v = vt[bits >> 23];
  return v.base - ((bits - v.thr) >> 31);
}
FLEET_HD uint32_t var_digits(float x, const VarEntry* vt) {
  return var_digits_ab(f2u(x), f2u(x) & 0x7fffffffu, vt);
}

FLEET_HD float mul10_mt(float X, const MulEntry& e) {
  X = X * e.m[0];
  X = X * e.m[0];
  X = X * e.m[1];
  X = X * e.m[2];
  X = X * e.m[2];
  X = X * e.m[3];
  X = X * e.m[3];
  X = X * e.m[3];
  return X * e.m[3];
}
FLEET_HD float div10_mt(float t, const MulEntry& e) {
  t = __builtin_fmaf(t, e.h[0], t * kTenthLo);
  t = __builtin_fmaf(t, e.h[0], t * kTenthLo);
  t = __builtin_fmaf(t, e.h[1], t * kTenthLo);
  t = __builtin_fmaf(t, e.h[2], t * kTenthLo);
  t = __builtin_fmaf(t, e.h[2], t * kTenthLo);
  t = __builtin_fmaf(t, e.h[3], t * kTenthLo);
  t = __builtin_fmaf(t, e.h[3], t * kTenthLo);
  t = __builtin_fmaf(t, e.h[3], t * kTenthLo);
  return __builtin_fmaf(t, e.h[3], t * kTenthLo);
}

// |code| = 10*floor(n/10) + d, n = trunc(X): floor(n/10) = mulhi(n, ceil(2^32/10))
// for n < 2^30 (error n*0.4/2^32 < 0.1); the sign of x goes on the float.
FLEET_HD uint32_t div10_u30(uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umulhi(n, 0x1999999Au);
#else
  return (uint32_t)(((uint64_t)n * 0x1999999Au) >> 32);
#endif
}
FLEET_HD float code_float_mt(float X, uint32_t d, float x) {
  const uint32_t c = div10_u30((uint32_t)X) * 10u + d;
  return u2f(f2u((float)c) | (f2u(x) & 0x80000000u));
}

// Q(x) on the q_gen domain (d = var_digits(x) <= 9)
FLEET_HD float q_mt_d(float x, uint32_t d, const MulEntry* mt) {
  const MulEntry e = mt[d];
  return div10_mt(code_float_mt(mul10_mt(__builtin_fabsf(x), e), d, x), e);
}
FLEET_HD float q_mt(float x, const VarEntry* vt, const MulEntry* mt) { return q_mt_d(x, var_digits(x, vt), mt); }
// float2int(x) on the q_gen domain
FLEET_HD int32_t enc_mt(float x, const VarEntry* vt, const MulEntry* mt) {
  const uint32_t d = var_digits(x, vt);
  const uint32_t c = div10_u30((uint32_t)mul10_mt(__builtin_fabsf(x), mt[d])) * 10u + d;
  return x < 0.0f ? -(int32_t)c : (int32_t)c;
}
// int2float(c) for every code: k = 9 - |c % 10| steps, flags from the last digit
FLEET_HD uint32_t last_digit_u(uint32_t a) {  // a % 10 for every uint32
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t q = __umulhi(a, 0xCCCCCCCDu) >> 3;
#else
  const uint32_t q = (uint32_t)(((uint64_t)a * 0xCCCCCCCDu) >> 35);
#endif
  return a - q * 10u;
}
FLEET_HD float dec_mt_r(int32_t c, uint32_t r, const MulEntry* mt) { return div10_mt((float)c, mt[r]); }
FLEET_HD float dec_mt(int32_t c, const MulEntry* mt) {
  return dec_mt_r(c, last_digit_u(c < 0 ? 0u - (uint32_t)c : (uint32_t)c), mt);
}

// Q(x) for |x| < 1 (the fixed 9-step chains), scalar: cheaper than q_fast2
FLEET_HD float q_fast1(float x) {
  float X = __builtin_fabsf(x);
#pragma unroll
  for (int j = 0; j < 9; ++j) X = X * 10.0f;
  const uint32_t c = div10_u30((uint32_t)X) * 10u;
  return d9(u2f(f2u((float)c) | (f2u(x) & 0x80000000u)));
}

// ------------------------------------- byte-table digit count (throughput Q)
// The k_update stages' form of q_mt: the digit count comes from ONE byte load
// indexed by the top 13 bits of x (sign, exponent, 4 mantissa bits; 8 KB), and
// the byte is already the byte offset of the step tables' entry (16 * d), so
// neither the compare against the power of ten nor an address computation
// costs a VALU instruction. A 1/16-binade slice that holds a power of ten (the
// one place where numDigits changes inside a binade) holds kD16Cmp instead: its
// lanes take the compare (var_digits_ab) in a rare divergent fix-up. Values
// outside the q_gen domain map to >= kD16Out (identity chains; the caller
// recomputes them exactly).
constexpr uint32_t kD16Out = 10u << 4;   // first out-of-domain offset
constexpr uint32_t kD16Cmp = 14u << 4;   // the slice holds the power of ten: compare
constexpr uint32_t kD16Slow = 15u << 4;  // numDigits > 9, inf, NaN
FLEET_HDC uint8_t d16_entry(uint32_t i) {  // i = bits >> 19
  const DigitPair p = digit_pair(i >> 4);
  const uint32_t ab_lo = (i << 19) & 0x7fffffffu, ab_hi = ab_lo | 0x7ffffu;
  const uint32_t thr = __builtin_bit_cast(uint32_t, p.thr);
  const uint32_t d_lo = ab_lo < thr ? p.dlo : p.dhi, d_hi = ab_hi < thr ? p.dlo : p.dhi;
  if (d_lo != d_hi) return (uint8_t)kD16Cmp;
  return (uint8_t)(d_lo > 9u ? kD16Slow : d_lo << 4);
}
// step tables at a 16-byte stride, addressed by the d16 byte offset
struct alignas(16) StepTables {
  float m[16][4];     // x10 chain group multipliers (MulEntry::m)
  float h[16][4];     // /10 chain group multipliers (MulEntry::h)
  uint32_t d[16][4];  // d itself (the code's last digit), in .x
};
FLEET_HDC StepTables make_step_tables() {
  StepTables t{};
  for (uint32_t d = 0; d < 16; ++d) {
    const MulEntry e = mul_entry(d);
    for (int k = 0; k < 4; ++k) {
      t.m[d][k] = e.m[k];
      t.h[d][k] = e.h[k];
      t.d[d][k] = d;
    }
  }
  return t;
}
// 16 * (|c| % 10) for every int32 c without a division (the stream kernels' int2float
// step count): 256 = 1 (mod 5) and 2^32 = 1 (mod 5), so with S the sum of the four
// bytes of c's bit pattern u, |c| = u = S (mod 5) for c >= 0 and |c| = 2^32 - u = 1 - S
// (mod 5) for c < 0, while |c| = u (mod 2). One table byte per (S, sign, u & 1):
// index S + 1024 * sign + 2048 * (u & 1), 4 KB. On gfx950 the index is v_alignbit
// (rotl 11 puts bit 0 at 11 and the sign at 10), v_and and v_sad_u8 (the byte sum
// plus those two bits) -- three instructions for the six of the mulhi remainder.
// Checked for every int32 by tests/native/check_math.cpp d16 and GPU digest fn 23.
FLEET_HDC uint8_t ld16_entry(uint32_t i) {
  const uint32_t S = i & 1023u, neg = (i >> 10) & 1u, odd = (i >> 11) & 1u;
  if (S > 1020u) return 0;
  const uint32_t m5 = neg ? (1026u - S) % 5u : S % 5u;  // 1 - S + 5 * 205 >= 6 > 0
  const uint32_t r = (m5 & 1u) == odd ? m5 : m5 + 5u;
  return (uint8_t)(r << 4);
}
FLEET_HD uint32_t ld16_index(int32_t c) {
  const uint32_t u = (uint32_t)c;
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_sad_u8(u, 0u, __builtin_amdgcn_alignbit(u, u, 21) & 0xc00u);
#else
  return (u & 255u) + ((u >> 8) & 255u) + ((u >> 16) & 255u) + (u >> 24) + ((u >> 31) << 10) + ((u & 1u) << 11);
#endif
}

// int2float(c) given r16 = 16 * (|c| % 10): the /10 chain's multipliers at r16
FLEET_HD float dec_d16(int32_t c, uint32_t r16, const StepTables* st) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const char* base = reinterpret_cast<const char*>(st);
  const f4 h = *static_cast<const f4*>(__builtin_assume_aligned(base + sizeof(st->m) + r16, 16));
  const MulEntry me{{1.0f, 1.0f, 1.0f, 1.0f}, {h.x, h.y, h.z, h.w}};
  return div10_mt((float)c, me);
}
// the marker lanes' digit offset (the compare of var_digits_ab)
FLEET_HD uint32_t d16_fix(float x, const VarEntry* vt) {
  return var_digits_ab(f2u(x), f2u(x) & 0x7fffffffu, vt) << 4;
}
// 16 * numDigits((int)x) by the VarEntry compare, total (no marker slices):
// >= kD16Out outside the q_gen domain, like the byte table. The serial
// accumulation's form: its sums fall into a power-of-ten slice of the byte table
// in most waves (1 % of values, 79 % of waves of 192 on the synthetic mix), where
// the byte table's divergent fix-up costs more than this compare for every value.
FLEET_HD uint32_t var_d16(uint32_t bits, const VarEntry* vt) {
  const VarEntry v = vt[bits >> 23];
  return (v.base - ((bits - v.thr) >> 31)) << 4;
}

// Q(x) given e = 16 * numDigits((int)x) <= 144 (garbage, never a fault, for e >= kD16Out)
FLEET_HD float q_d16(float x, uint32_t e, const StepTables* st) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  // e is a multiple of 16 (d16_entry, d16_fix): 16-byte loads at the byte offset itself
  const char* base = reinterpret_cast<const char*>(st);
  const f4 m = *static_cast<const f4*>(__builtin_assume_aligned(base + e, 16));
  const f4 h = *static_cast<const f4*>(__builtin_assume_aligned(base + sizeof(st->m) + e, 16));
  const uint32_t d = *static_cast<const uint32_t*>(__builtin_assume_aligned(base + sizeof(st->m) + sizeof(st->h) + e, 16));
  const MulEntry me{{m.x, m.y, m.z, m.w}, {h.x, h.y, h.z, h.w}};
  return div10_mt(code_float_mt(mul10_mt(__builtin_fabsf(x), me), d, x), me);
}

// float2int(x) given e = 16 * numDigits((int)x) <= 144 (the client encode's form
// of q_d16): the x10 chain's multipliers and d itself at the byte offset e; the
// sign by two integer ops on x's sign mask ((c ^ s) - s), not a compare and select.
FLEET_HD int32_t enc_d16(float x, uint32_t e, const StepTables* st) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const char* base = reinterpret_cast<const char*>(st);
  const f4 m = *static_cast<const f4*>(__builtin_assume_aligned(base + e, 16));
  const uint32_t d = *static_cast<const uint32_t*>(__builtin_assume_aligned(base + sizeof(st->m) + sizeof(st->h) + e, 16));
  const MulEntry me{{m.x, m.y, m.z, m.w}, {1.0f, 1.0f, 1.0f, 1.0f}};
  const uint32_t c = div10_u30((uint32_t)mul10_mt(__builtin_fabsf(x), me)) * 10u + d;
  const uint32_t sm = (uint32_t)((int32_t)f2u(x) >> 31);
  return (int32_t)((c ^ sm) - sm);
}

// ------------------------------------------- one-lookup latency Q (serial chain)
// The serial accumulation A = Q(A + p) runs on ONE wave per tile: it is bound by
// that wave's instruction issue, so the step count matters more than a table
// load on the path. One LDS entry per (sign, biased exponent) of x, clamped to
// 126..158 (|x| < 1 shares the 126 entry), holds everything the step needs:
//   * the chains for k_hi = 9 - dhi steps (dhi = numDigits when |x| >= thr) as
//     group multipliers (groups 2, 1, 2, 4: m = 10 or 1, h = RN(0.1) or 1);
//   * ONE extra step taken iff |x| < thr and dlo = dhi - 1 (then k = k_hi + 1):
//     both chains are order-free (identity steps are exact), so it goes last;
//   * the /10 chain's small terms in the kTenthLo2 form of q_lat (one
//     dependent fma per step): A_1 = U_0*c[0], A_j = U_{j-2}*c[j-1],
//     c = kTenthLo after an identity step, kTenthLo2 after a taken one, 0 for
//     an identity step itself (fma(U, 1, U'*0) = U exactly).
// Entries of values outside the q_gen domain hold identity chains; callers
// flag |x| >= 1e8 (max over the chain) and recompute such values exactly.
constexpr uint32_t kXlSpan = 33;  // biased exponents 126..158 per sign
struct alignas(16) XlEntry {
  float m[4];     // x10 chain group multipliers
  float thr;      // |x| < thr selects dlo and the extra step
  uint32_t dhi, dlo;
  float mx;       // extra x10 step: 10 if dlo + 1 == dhi, else 1
  float c[10];    // small-term multipliers, c[9] for the extra step
  float h[4];     // /10 chain group multipliers
  float hx;       // extra /10 step: RN(0.1) or 1
  float pad;
  // 112-byte stride: seven 16-byte LDS chunks, odd, so the serial consumer's entry reads
  // (one entry per lane, six 16-byte reads) fall on 16 distinct bank offsets before two
  // entries collide (the 96-byte stride repeated every 8 entries)
  float pad2[4];
};
static_assert(sizeof(XlEntry) == 112, "XlEntry stride");
FLEET_HDC XlEntry xl_entry(uint32_t idx) {
  XlEntry x{};
  const uint32_t sign = idx / kXlSpan, be = 126u + idx % kXlSpan;
  const DigitPair v = digit_pair((sign << 8) | be);
  uint32_t dhi = v.dhi, dlo = v.dlo;
  const bool extra = dlo <= 9u && dlo + 1u == dhi;
  if (dhi > 9u) dhi = 9u;  // off the domain: identity chains (flagged by the caller)
  if (dlo > 9u) dlo = 9u;
  const Steps s = steps_of(9u - dhi);
  const bool g[4] = {s.e, s.b0, s.b1, s.b2};
  bool taken[10] = {false, s.e, s.e, s.b0, s.b1, s.b1, s.b2, s.b2, s.b2, s.b2};  // taken[j], steps j = 1..9
  for (int i = 0; i < 4; ++i) {
    x.m[i] = g[i] ? 10.0f : 1.0f;
    x.h[i] = g[i] ? kTenthHi : 1.0f;
  }
  x.thr = v.thr;
  x.dhi = dhi;
  x.dlo = extra ? dlo : dhi;
  x.mx = extra ? 10.0f : 1.0f;
  x.hx = extra ? kTenthHi : 1.0f;
  x.c[0] = taken[1] ? kTenthLo : 0.0f;
  for (int j = 2; j <= 9; ++j) x.c[j - 1] = taken[j] ? (taken[j - 1] ? kTenthLo2 : kTenthLo) : 0.0f;
  x.c[9] = extra ? (taken[9] ? kTenthLo2 : kTenthLo) : 0.0f;
  return x;
}
FLEET_HD uint32_t xl_index(float x) {
  const uint32_t b = f2u(x);
  uint32_t be = (b >> 23) & 0xffu;
  be = be < 126u ? 126u : be > 158u ? 158u : be;
  return (b >> 31) * kXlSpan + be - 126u;
}
// Q(x) for |x| < 1e8 (exact there; garbage, never a fault, elsewhere).
// the entry's sign + clamped exponent: equal keys <=> same entry
FLEET_HD uint32_t xl_key(float x) {
  const uint32_t b = f2u(x);
  uint32_t be = (b >> 23) & 0xffu;
  be = be < 126u ? 126u : be > 158u ? 158u : be;
  return (b & 0x80000000u) | be;
}
// the entry in registers: six 16-byte loads in flight together, and selects
// between loaded values instead of loads under a condition
FLEET_HD XlEntry xl_load(const XlEntry* xt, float x) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u3 __attribute__((ext_vector_type(3)));
  XlEntry e;
  const u4* src = reinterpret_cast<const u4*>(xt + xl_index(x));
  u4* dst = reinterpret_cast<u4*>(&e);
#pragma unroll
  for (int i = 0; i < 5; ++i) dst[i] = src[i];
  // the last 16 bytes without the pad word: a loaded register nobody reads
  // would be reused at once and stall on the load (write-after-write)
  const u3 t = *reinterpret_cast<const u3*>(src + 5);
  e.h[2] = u2f(t.x);
  e.h[3] = u2f(t.y);
  e.hx = u2f(t.z);
  e.pad = 0.0f;
  return e;
}
// Q(x) for |x| < 1e8 given x's entry (exact there; garbage, never a fault,
// elsewhere).
FLEET_HD float q_xl_e(float x, const XlEntry& e) {
  const float ax = __builtin_fabsf(x);
  const bool small = ax < e.thr;
  float X = ax * e.m[0];
  X = X * e.m[0];
  X = X * e.m[1];
  X = X * e.m[2];
  X = X * e.m[2];
  X = X * e.m[3];
  X = X * e.m[3];
  X = X * e.m[3];
  X = X * e.m[3];
  X = X * (small ? e.mx : 1.0f);
  const uint32_t d = small ? e.dlo : e.dhi;
  const float cf = code_float_mt(X, d, x);
  const float H[9] = {e.h[0], e.h[0], e.h[1], e.h[2], e.h[2], e.h[3], e.h[3], e.h[3], e.h[3]};
  float U = cf, a = cf * e.c[0];
#pragma unroll
  for (int j = 1; j <= 9; ++j) {
    const float Un = __builtin_fmaf(U, H[j - 1], a);  // the only dependent op per step
    a = U * (j < 9 ? e.c[j] : (small ? e.c[9] : 0.0f));
    U = Un;
  }
  return __builtin_fmaf(U, small ? e.hx : 1.0f, a);
}
FLEET_HD float q_xl(float x, const XlEntry* xt) { return q_xl_e(x, xl_load(xt, x)); }

// int2float(c) for every code (k = 9 - |c % 10| in [0, 9]) -- total.
FLEET_HD uint32_t last_digit(int32_t c) {
  uint32_t a = c < 0 ? 0u - (uint32_t)c : (uint32_t)c;
  return a - (a / 10u) * 10u;
}
FLEET_HD float dec_gen(int32_t c) { return steps_div10((float)c, steps_of(9u - last_digit(c))); }
FLEET_HD f2 dec_gen2(int32_t c0, int32_t c1) {
  return steps_div10x2(f2{(float)c0, (float)c1}, steps_of(9u - last_digit(c0)), steps_of(9u - last_digit(c1)));
}

}  // namespace fleet
