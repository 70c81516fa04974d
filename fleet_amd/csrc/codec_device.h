// fleet_amd/csrc/codec_device.h -- device-side FLeet codec arithmetic for gfx950.
//
// Bit-exact restatement, for CDNA4 VALU, of
//   Base64::numDigits / float2int / int2float  (commonLib/cpp_utils/Base64.cpp:73-139)
//   Base64 text <-> bytes                     (Base64.cpp:56-68,160-205,221-253)
// as the reference's x86-64 SSE build computes them (one IEEE binary32 RNE
// rounding per operation, cvttss2si truncation). Built with
// -ffp-contract=off: every fused multiply-add below is written explicitly.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fleet {

// RN(0.1) and RN(0.1 - RN(0.1)): t*0.1 as an unevaluated pair.
constexpr float kTenthHi = 0x1.99999ap-4f;
constexpr float kTenthLo = -0x1.99999ap-30f;

// Correctly rounded t/10 in two VALU ops (v_mul_f32 + v_fma_f32): the exact
// t*hi plus RN(t*lo) lies within 2^-49 (relative) of t/10, while t/10 is
// never closer than 2^-27.3 to a binary32 rounding midpoint (t has a 24-bit
// significand, so 10*midpoint - t is an odd multiple of the finer ulp).
// Exhaustively checked against IEEE division for every binary32 t with
// |t| >= 1e-30 (tests/test_div10.py); int2float never divides anything
// smaller than 1e-9 in magnitude.
__device__ __forceinline__ float div10(float t) { return __builtin_fmaf(t, kTenthHi, t * kTenthLo); }

// x86-64 `(int)x` (cvttss2si): INT_MIN when |x| >= 2^31 or x is NaN
// (v_cvt_i32_f32 would saturate instead).
__device__ __forceinline__ int32_t cvtt(float x) {
  return __builtin_fabsf(x) < 2147483648.0f ? (int32_t)x : INT32_MIN;
}

// Base64::numDigits (Base64.cpp:73-82): decimal digits of n, '-' counted.
__device__ __forceinline__ int num_digits(int32_t n) {
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

// Base64::int2float, intNum = 1, precision = 9 (Base64.cpp:127-134):
// k = 9 - |c % 10| fp32 divisions by 10 of (float)c.
__device__ __forceinline__ float dec(int32_t c) {
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

// Base64::float2int, intNum = 1, precision = 9 (Base64.cpp:96-109).
__device__ __forceinline__ int32_t enc(float x) {
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

// Q = int2float o float2int: the value the next JNI op decodes after an encode.
__device__ __forceinline__ float q(float x) { return dec(enc(x)); }

// ------------------------------------------------------------------ Base64

// Base64.cpp:56-68 `from_base64`, extended with 0xff for bytes >= 0x80
// (the reference indexes out of bounds there; such text is rejected here).
struct B64Tables {
  uint8_t from[256];
  uint8_t to[64];
};

__device__ __forceinline__ uint8_t b64_from_value(int ch) {
  if (ch >= 'A' && ch <= 'Z') return (uint8_t)(ch - 'A');
  if (ch >= 'a' && ch <= 'z') return (uint8_t)(ch - 'a' + 26);
  if (ch >= '0' && ch <= '9') return (uint8_t)(ch - '0' + 52);
  if (ch == '+' || ch == '-') return 62;
  if (ch == '/' || ch == '_') return 63;
  return 0xff;
}

__device__ __forceinline__ uint8_t b64_to_value(int s) {
  return (uint8_t)(s < 26 ? 'A' + s : s < 52 ? 'a' + s - 26 : s < 62 ? '0' + s - 52 : s == 62 ? '+' : '/');
}

// Fill the block's LDS tables (call from every thread, then __syncthreads()).
__device__ __forceinline__ void b64_tables_init(B64Tables* t) {
  for (int i = threadIdx.x; i < 256; i += blockDim.x) t->from[i] = b64_from_value(i);
  for (int i = threadIdx.x; i < 64; i += blockDim.x) t->to[i] = b64_to_value(i);
}

// One 16-char group -> 12 bytes -> 3 little-endian int32 codes.
// Returns a 16-bit mask of chars that are not in the alphabet (bit i = char i).
__device__ __forceinline__ uint32_t b64_decode_group(uint4 w, const B64Tables* t, int32_t codes[3]) {
  const uint32_t words[4] = {w.x, w.y, w.z, w.w};
  uint32_t V[4];
  uint32_t bad = 0;
#pragma unroll
  for (int qd = 0; qd < 4; ++qd) {
    uint32_t s0 = t->from[words[qd] & 0xff];
    uint32_t s1 = t->from[(words[qd] >> 8) & 0xff];
    uint32_t s2 = t->from[(words[qd] >> 16) & 0xff];
    uint32_t s3 = t->from[words[qd] >> 24];
    bad |= ((s0 >> 7) | ((s1 >> 7) << 1) | ((s2 >> 7) << 2) | ((s3 >> 7) << 3)) << (4 * qd);
    V[qd] = ((s0 & 63) << 18) | ((s1 & 63) << 12) | ((s2 & 63) << 6) | (s3 & 63);
  }
  // bytes of quad q are V[q] big-endian; codes are little-endian int32
  codes[0] = (int32_t)__builtin_amdgcn_perm(V[1], V[0], 0x06000102u);
  codes[1] = (int32_t)__builtin_amdgcn_perm(V[2], V[1], 0x05060001u);
  codes[2] = (int32_t)__builtin_amdgcn_perm(V[3], V[2], 0x04050600u);
  return bad;
}

// 3 codes -> 12 bytes -> 16 chars (Base64.cpp:176-195).
__device__ __forceinline__ uint4 b64_encode_group(const int32_t codes[3], const B64Tables* t) {
  const uint32_t c0 = (uint32_t)codes[0], c1 = (uint32_t)codes[1], c2 = (uint32_t)codes[2];
  // inverse of the perms above: V[q] = 24-bit big-endian view of bytes 3q..3q+2
  uint32_t V[4];
  V[0] = __builtin_amdgcn_perm(0u, c0, 0x0c000102u);  // b0<<16 | b1<<8 | b2
  V[1] = __builtin_amdgcn_perm(c1, c0, 0x0c030405u);  // b3<<16 | b4<<8 | b5
  V[2] = __builtin_amdgcn_perm(c2, c1, 0x0c020304u);  // b6<<16 | b7<<8 | b8
  V[3] = __builtin_amdgcn_perm(0u, c2, 0x0c010203u);  // b9<<16 | b10<<8 | b11
  uint32_t out[4];
#pragma unroll
  for (int qd = 0; qd < 4; ++qd) {
    uint32_t a = t->to[(V[qd] >> 18) & 63];
    uint32_t b = t->to[(V[qd] >> 12) & 63];
    uint32_t c = t->to[(V[qd] >> 6) & 63];
    uint32_t d = t->to[V[qd] & 63];
    out[qd] = a | (b << 8) | (c << 16) | (d << 24);
  }
  return make_uint4(out[0], out[1], out[2], out[3]);
}

// ------------------------------------------------------------- synthetic

// Philox4x32-10 (Salmon et al., SC'11), standard round constants.
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// SURVEY.md §8d value mix (integer ops + bit assembly only).
__device__ __forceinline__ float synth_value(uint64_t seed, uint32_t client, uint32_t element) {
  uint4 u = philox4x32_10(make_uint4(element, client, 0x464C4545u, 0u),
                          make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  uint32_t cls = u.x % 100u;
  int e = cls < 90u ? -20 + (int)(u.y % 14u) : cls < 99u ? -6 + (int)(u.y % 10u) : 4 + (int)(u.y % 17u);
  uint32_t bits = (u.w & 0x80000000u) | ((uint32_t)(e + 127) << 23) | (u.z & 0x7FFFFFu);
  return __uint_as_float(bits);
}

}  // namespace fleet
