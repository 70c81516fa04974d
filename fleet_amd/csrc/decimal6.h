// fleet_amd/csrc/decimal6.h -- the decimal round trip of the mode-1 model-version
// copy, host+device: y = strtof(text of `os << v`), with the ostream's default
// precision 6, i.e. strtof(sprintf("%.6g", (double)v)).
//
// descentNative copies the model through its text (Server/src/main/c++/
// cppNN_backend.cpp:367-372: cnnNew->read(cnn.getParams())): network::getParams
// prints every dictionary value and bias with `ss << value` (commonLib/cppNN/
// network.h:611-706) and network::read parses them back with `>>` (:956-997),
// which libstdc++ forwards to strtof. Both conversions are exact-rounding
// operations on rationals, computed here with integers only:
//   1. %.6g: E = floor(log10|v|) (the exponent of the exact value), then
//      N = round-half-even(|v| * 10^(5-E)) in [10^5, 10^6]; a carry to 10^6
//      gives N = 10^5, E + 1 (glibc printf: the exact binary value, rounded in
//      the default round-to-nearest mode).
//   2. strtof: y = the binary32 nearest to N * 10^(E-5), ties to even,
//      subnormals included (glibc strtof).
// Each quotient floor(A / B) is estimated in double and settled with exact
// multiplications on 192-bit integers; the remainder decides the rounding.
// Checked against libc (snprintf + strtof) on every finite binary32: digest
// fn 22 (fleet_selftest_digest) against tests/golden/digests.json, and on the
// CPU by tests/native/check_math.cpp g6.
#pragma once
#include <stdint.h>

#include "codec_math.h"

namespace fleet {

struct U192 {
  uint64_t w[3];  // little-endian 64-bit limbs
};

FLEET_HD U192 u192(uint64_t x) { return U192{{x, 0, 0}}; }

// a * b; the caller guarantees the product fits in 192 bits
FLEET_HD U192 u192_mul(const U192& a, uint64_t b) {
  U192 r;
  unsigned __int128 c = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    c += (unsigned __int128)a.w[i] * b;
    r.w[i] = (uint64_t)c;
    c >>= 64;
  }
  return r;
}

FLEET_HD U192 u192_shl(const U192& a, int s) {  // 0 <= s < 192
  U192 r{{0, 0, 0}};
  const int q = s >> 6, b = s & 63;
#pragma unroll
  for (int i = 2; i >= 0; --i) {
    const int src = i - q;
    if (src < 0) continue;
    uint64_t v = a.w[src] << b;
    if (b && src > 0) v |= a.w[src - 1] >> (64 - b);
    r.w[i] = v;
  }
  return r;
}

FLEET_HD int u192_cmp(const U192& a, const U192& b) {
#pragma unroll
  for (int i = 2; i >= 0; --i)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}

FLEET_HD U192 u192_sub(const U192& a, const U192& b) {  // a >= b
  U192 r;
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint64_t x = a.w[i], y = b.w[i];
    const uint64_t d = x - y - borrow;
    borrow = (x < y) || (x - y < borrow) ? 1u : 0u;
    r.w[i] = d;
  }
  return r;
}

FLEET_HD U192 u192_pow5(int k) {  // 5^k, k <= 82
  U192 r = u192(1);
  while (k > 0) {
    const int s = k > 27 ? 27 : k;  // 5^27 < 2^63
    uint64_t p = 1;
    for (int i = 0; i < s; ++i) p *= 5u;
    r = u192_mul(r, p);
    k -= s;
  }
  return r;
}

// q = floor(A / B) near the estimate q0 (|error| a few units), and the rounding
// of A / B to an integer, ties to even. Returns the rounded quotient; *fl = floor.
FLEET_HD uint64_t div_round_even(const U192& A, const U192& B, uint64_t q0, uint64_t* fl) {
  uint64_t q = q0;
  // settle q: q*B <= A < (q+1)*B
  for (int it = 0; it < 64 && q > 0 && u192_cmp(u192_mul(B, q), A) > 0; ++it) --q;
  for (int it = 0; it < 64 && u192_cmp(u192_mul(B, q + 1), A) <= 0; ++it) ++q;
  *fl = q;
  const U192 R = u192_sub(A, u192_mul(B, q));
  const int c = u192_cmp(u192_shl(R, 1), B);
  return q + ((c > 0 || (c == 0 && (q & 1u))) ? 1u : 0u);
}

// 10^k as a double estimate (k in [-60, 60])
FLEET_HD double pow10_est(int k) {
  double r = 1.0, b = k < 0 ? 0.1 : 10.0;
  int n = k < 0 ? -k : k;
  while (n) {
    if (n & 1) r *= b;
    b *= b;
    n >>= 1;
  }
  return r;
}

FLEET_HD float pow2f(int e) { return u2f((uint32_t)(e + 127) << 23); }  // e in [-126, 127]
FLEET_HD double pow2d(int e) { return __builtin_bit_cast(double, (uint64_t)(e + 1023) << 52); }  // |e| <= 1022

// m * 2^e for an integer m <= 2^24 when the result is an exact binary32 value
// (normal or subnormal): one multiply, or two through a normal intermediate.
FLEET_HD float ldexp_exact(float m, int e) {
  if (e >= -126) return m * pow2f(e);
  return (m * pow2f(e + 64)) * 0x1p-64f;
}

// strtof(sprintf("%.6g", (double)v)) for finite v.
FLEET_HD float g6_roundtrip(float v) {
  const uint32_t bits = f2u(v), a = bits & 0x7fffffffu, sign = bits & 0x80000000u;
  if (a == 0) return v;  // "0" / "-0"
  const uint32_t be = a >> 23, mant = a & 0x7fffffu;
  const uint64_t m = be ? (uint64_t)(mant | 0x800000u) : (uint64_t)mant;
  const int e = be ? (int)be - 150 : -149;  // |v| = m * 2^e
  const double av = (double)u2f(a);
  // 1. E and N: floor(|v| * 10^(5-E)) in [10^5, 10^6), then round half-even
  int E = 0;
  {  // floor(log10|v|) from a double estimate (settled below by the exact floor's range)
    int ee = (int)(((be ? (int)be - 127 : -149)) * 0.30102999566398120) - 1;
    double t = av * pow10_est(-ee);
    while (t >= 10.0) {
      t *= 0.1;
      ++ee;
    }
    while (t < 1.0) {
      t *= 10.0;
      --ee;
    }
    E = ee;
  }
  uint64_t N = 0;
  for (int it = 0; it < 8; ++it) {
    const int k = 5 - E;
    U192 A, B;
    if (k >= 0) {
      A = u192_mul(u192_pow5(k), m);
      const int sh = e + k;
      if (sh >= 0) {
        A = u192_shl(A, sh);
        B = u192(1);
      } else {
        B = u192_shl(u192(1), -sh);
      }
    } else {
      const int j = -k;
      B = u192_pow5(j);
      const int sh = e - j;
      if (sh >= 0) {
        A = u192_shl(u192(m), sh);
      } else {
        A = u192(m);
        B = u192_shl(B, -sh);
      }
    }
    double est = av * pow10_est(k);
    uint64_t q0 = est < 1.0 ? 0u : (uint64_t)est;
    uint64_t fl = 0;
    const uint64_t r = div_round_even(A, B, q0, &fl);
    if (fl < 100000u) {
      --E;
      continue;
    }
    if (fl >= 1000000u) {
      ++E;
      continue;
    }
    N = r;
    if (N == 1000000u) {
      N = 100000u;
      ++E;
    }
    break;
  }
  // 2. strtof: the binary32 nearest to N * 10^p
  const int p = E - 5;
  float y;
  if (p >= 0) {
    const U192 I = u192_mul(u192_pow5(p), N);  // value = I * 2^p
    int L = 0;
    for (int i = 2; i >= 0; --i)
      if (I.w[i]) {
        L = 64 * i + 64 - __builtin_clzll(I.w[i]);
        break;
      }
    if (L <= 24) {
      y = ldexp_exact((float)I.w[0], p);
    } else {
      const int drop = L - 24;
      // mant = I >> drop (24 bits), rem against half = 2^(drop-1)
      U192 sh = I;
      uint64_t mnt = 0;
      {
        const int q = drop >> 6, b = drop & 63;
        uint64_t lo = sh.w[q], hi = q + 1 < 3 ? sh.w[q + 1] : 0;
        mnt = b ? (lo >> b) | (hi << (64 - b)) : lo;
        mnt &= 0xffffffu;
      }
      const U192 back = u192_shl(u192(mnt), drop);
      const U192 rem = u192_sub(I, back);
      const U192 half = u192_shl(u192(1), drop - 1);
      const int c = u192_cmp(rem, half);
      if (c > 0 || (c == 0 && (mnt & 1u))) ++mnt;
      y = ldexp_exact((float)mnt, drop + p);
    }
  } else {
    const int j = -p;
    const U192 B0 = u192_pow5(j);
    // the ulp exponent qe of the result: normal 2^23 <= N*10^p / 2^qe < 2^24, else -149
    const double d = (double)N * pow10_est(p);
    const int lg = (int)((__builtin_bit_cast(uint64_t, d) >> 52) & 0x7ffu) - 1023;  // floor(log2 d), d normal
    int qe = lg - 23;
    if (qe < -149) qe = -149;
    uint64_t M = 0;
    for (int it = 0; it < 8; ++it) {
      const int s = -qe - j;  // R = N * 2^s / 5^j
      U192 A, B = B0;
      if (s >= 0) A = u192_shl(u192(N), s);
      else {
        A = u192(N);
        B = u192_shl(B0, -s);
      }
      const double est = d * pow2d(-qe);
      uint64_t fl = 0;
      const uint64_t r = div_round_even(A, B, est < 1.0 ? 0u : (uint64_t)est, &fl);
      if (fl >= (1u << 24)) {
        ++qe;
        continue;
      }
      if (fl < (1u << 23) && qe > -149) {
        --qe;
        continue;
      }
      M = r;
      break;
    }
    y = ldexp_exact((float)M, qe);
  }
  return u2f(f2u(y) | sign);
}

}  // namespace fleet
