// fleet_amd/csrc/codec_device.h -- device-side FLeet codec pieces for gfx950:
//   decimal fixed-point arithmetic (codec_math.h, Base64.cpp:37-103)
//   Base64 text <-> bytes           (Base64.cpp:20-27,124-169,185-217)
//   Philox synthetic gradient source
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "codec_math.h"

namespace fleet {

// ------------------------------------------------------------------ Base64

// Base64.cpp:20-27 `from_base64`, extended with 0xff for bytes >= 0x80
// (the reference indexes out of bounds there; such text is rejected here).
// Every kernel copies this block of tables into LDS at start (b64_tables_init).
struct B64Tables {
  MulEntry mt[16];    // step multipliers by digit count (codec_math.h)
  VarEntry var[512];  // digit count by sign + biased exponent (codec_math.h)
  uint8_t from[256];  // Base64.cpp:20-27, 0xff = not in the alphabet
  uint8_t to[64];
};
static_assert(sizeof(B64Tables) % 16 == 0, "copied as uint4");

FLEET_HDC uint8_t b64_from_value(int ch) {
  if (ch >= 'A' && ch <= 'Z') return (uint8_t)(ch - 'A');
  if (ch >= 'a' && ch <= 'z') return (uint8_t)(ch - 'a' + 26);
  if (ch >= '0' && ch <= '9') return (uint8_t)(ch - '0' + 52);
  if (ch == '+' || ch == '-') return 62;
  if (ch == '/' || ch == '_') return 63;
  return 0xff;
}

FLEET_HDC uint8_t b64_to_value(int s) {
  return (uint8_t)(s < 26 ? 'A' + s : s < 52 ? 'a' + s - 26 : s < 62 ? '0' + s - 52 : s == 62 ? '+' : '/');
}

FLEET_HDC B64Tables make_b64_tables() {
  B64Tables t{};
  for (int d = 0; d < 16; ++d) t.mt[d] = mul_entry((uint32_t)d);
  for (int i = 0; i < 512; ++i) t.var[i] = var_entry((uint32_t)i);
  for (int i = 0; i < 256; ++i) {
    t.from[i] = b64_from_value(i);
  }
  for (int i = 0; i < 64; ++i) t.to[i] = b64_to_value(i);
  return t;
}
// built at compile time; one copy per code object
static __constant__ B64Tables g_b64_tables = make_b64_tables();

// Copy the tables into the block's LDS (call from every thread of an NT-thread
// block, then __syncthreads()): 308 16-byte loads from an L2-resident image.
template <int NT = 256>
__device__ __forceinline__ void b64_tables_init(B64Tables* t) {
  constexpr int n16 = (int)(sizeof(B64Tables) / 16);
  const uint4* src = reinterpret_cast<const uint4*>(&g_b64_tables);
  uint4* dst = reinterpret_cast<uint4*>(t);
#pragma unroll
  for (int i0 = 0; i0 < n16; i0 += NT) {
    const int i = i0 + (int)threadIdx.x;
    if (i < n16) dst[i] = src[i];
  }
}

// One-lookup latency Q entries (codec_math.h q_xl) for the serial consumer.
struct XlTable {
  XlEntry x[2 * kXlSpan];
};
static_assert(sizeof(XlTable) % 16 == 0, "copied as uint4");
FLEET_HDC XlTable make_xl_table() {
  XlTable t{};
  for (uint32_t i = 0; i < 2 * kXlSpan; ++i) t.x[i] = xl_entry(i);
  return t;
}
static __constant__ XlTable g_xl_table = make_xl_table();
template <int NT = 256>
__device__ __forceinline__ void xl_table_init(XlTable* t) {
  constexpr int n16 = (int)(sizeof(XlTable) / 16);
  const uint4* src = reinterpret_cast<const uint4*>(&g_xl_table);
  uint4* dst = reinterpret_cast<uint4*>(t);
#pragma unroll
  for (int i0 = 0; i0 < n16; i0 += NT) {
    const int i = i0 + (int)threadIdx.x;
    if (i < n16) dst[i] = src[i];
  }
}

// The throughput-Q tables of k_update (codec_math.h d16_entry / StepTables):
// 8 KB of digit offsets by the top 13 bits of x, and the stride-16 step tables.
struct alignas(16) D16Table {
  StepTables st;
  uint8_t d16[8192];
};
static_assert(sizeof(D16Table) % 16 == 0, "copied as uint4");
FLEET_HDC D16Table make_d16_table() {
  D16Table t{};
  t.st = make_step_tables();
  for (uint32_t i = 0; i < 8192; ++i) t.d16[i] = d16_entry(i);
  return t;
}
static __constant__ D16Table g_d16_table = make_d16_table();
template <int NT = 256>
__device__ __forceinline__ void d16_table_init(D16Table* t) {
  constexpr int n16 = (int)(sizeof(D16Table) / 16);
  const uint4* src = reinterpret_cast<const uint4*>(&g_d16_table);
  uint4* dst = reinterpret_cast<uint4*>(t);
#pragma unroll
  for (int i0 = 0; i0 < n16; i0 += NT) {
    const int i = i0 + (int)threadIdx.x;
    if (i < n16) dst[i] = src[i];
  }
}

// The stream kernels' extra table: int2float's step count by byte sum (codec_math.h
// ld16_entry), 4 KB beside their D16Table (the tiles, LDS-bound, keep the division).
struct alignas(16) LastDigitTable {
  uint8_t ld16[4096];
};
FLEET_HDC LastDigitTable make_last_digit_table() {
  LastDigitTable t{};
  for (uint32_t i = 0; i < 4096; ++i) t.ld16[i] = ld16_entry(i);
  return t;
}
static __constant__ LastDigitTable g_ld16_table = make_last_digit_table();
template <int NT = 256>
__device__ __forceinline__ void ld16_table_init(LastDigitTable* t) {
  constexpr int n16 = (int)(sizeof(LastDigitTable) / 16);
  const uint4* src = reinterpret_cast<const uint4*>(&g_ld16_table);
  uint4* dst = reinterpret_cast<uint4*>(t);
#pragma unroll
  for (int i0 = 0; i0 < n16; i0 += NT) {
    const int i = i0 + (int)threadIdx.x;
    if (i < n16) dst[i] = src[i];
  }
}

// One 16-char group -> 12 bytes -> 3 little-endian int32 codes.
// Returns a 16-bit mask of chars that are not in the alphabet (bit i = char i).
__device__ __forceinline__ uint32_t b64_decode_group(uint4 w, const B64Tables* t, int32_t codes[3]) {
  const uint32_t words[4] = {w.x, w.y, w.z, w.w};
  uint32_t V[4];
  uint32_t bad = 0;
  // read sign-extended like b64_decode_group_full (the two share their first loads):
  // the invalid marker is -1, bit 31 of its sextet word
  const int8_t* from = reinterpret_cast<const int8_t*>(t->from);
#pragma unroll
  for (int qd = 0; qd < 4; ++qd) {
    const uint32_t s0 = (uint32_t)(int32_t)from[words[qd] & 0xff];
    const uint32_t s1 = (uint32_t)(int32_t)from[(words[qd] >> 8) & 0xff];
    const uint32_t s2 = (uint32_t)(int32_t)from[(words[qd] >> 16) & 0xff];
    const uint32_t s3 = (uint32_t)(int32_t)from[words[qd] >> 24];
    bad |= ((s0 >> 31) | ((s1 >> 31) << 1) | ((s2 >> 31) << 2) | ((s3 >> 31) << 3)) << (4 * qd);
    V[qd] = ((s0 & 63) << 18) | ((s1 & 63) << 12) | ((s2 & 63) << 6) | (s3 & 63);
  }
  // bytes of quad q are V[q] big-endian; codes are little-endian int32
  codes[0] = (int32_t)__builtin_amdgcn_perm(V[1], V[0], 0x06000102u);
  codes[1] = (int32_t)__builtin_amdgcn_perm(V[2], V[1], 0x05060001u);
  codes[2] = (int32_t)__builtin_amdgcn_perm(V[3], V[2], 0x04050600u);
  return bad;
}

// The shift-or assembly of four 6-bit sextets into 24 bits, written out, is re-associated
// by the compiler into four instructions per quad (two shifts, v_lshl_or, v_or3); three
// v_lshl_or are the minimum, so they are written as asm.
// A whole group's four quads (s[4q..4q+3] -> 24 bits, big-endian) in ONE asm block of
// twelve v_lshl_or: every sextet is an input, so the compiler issues all sixteen table
// reads before it (one asm per quad made it wait on each quad's reads in turn)
__device__ __forceinline__ void group24(const uint32_t (&s)[16], uint32_t (&V)[4]) {
  uint32_t a0, b0, a1, b1, a2, b2, a3, b3;
  asm("v_lshl_or_b32 %4, %12, 6, %13\n\t"
      "v_lshl_or_b32 %5, %14, 6, %15\n\t"
      "v_lshl_or_b32 %6, %16, 6, %17\n\t"
      "v_lshl_or_b32 %7, %18, 6, %19\n\t"
      "v_lshl_or_b32 %8, %20, 6, %21\n\t"
      "v_lshl_or_b32 %9, %22, 6, %23\n\t"
      "v_lshl_or_b32 %10, %24, 6, %25\n\t"
      "v_lshl_or_b32 %11, %26, 6, %27\n\t"
      "v_lshl_or_b32 %0, %4, 12, %5\n\t"
      "v_lshl_or_b32 %1, %6, 12, %7\n\t"
      "v_lshl_or_b32 %2, %8, 12, %9\n\t"
      "v_lshl_or_b32 %3, %10, 12, %11"
      : "=v"(V[0]), "=v"(V[1]), "=v"(V[2]), "=v"(V[3]), "=&v"(a0), "=&v"(b0), "=&v"(a1), "=&v"(b1), "=&v"(a2),
        "=&v"(b2), "=&v"(a3), "=&v"(b3)
      : "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]), "v"(s[4]), "v"(s[5]), "v"(s[6]), "v"(s[7]), "v"(s[8]), "v"(s[9]),
        "v"(s[10]), "v"(s[11]), "v"(s[12]), "v"(s[13]), "v"(s[14]), "v"(s[15]));
}

// Same decode for a full group (all 16 chars carry data): returns nonzero if any
// char is outside the alphabet. Sextets compose by shift-or; no per-char mask:
// valid entries are 0..63 and the invalid marker 0xff has bit 6 set, so the OR of
// the group's sextets flags it (the codes are garbage then, and the caller fails).
// The sextets are read sign-extended (ds_read_i8): the invalid marker 0xff becomes -1,
// whose set high bits survive the shift-or assembly in bits 24-31 of the quad's word
// wherever the char sits (s3 or s2 in t2 = s2 << 6 | s3 fill bits 6..31; s1 or s0 in
// t1 fill bits 6..31 / 12..31, shifted by 12 into 18..31 / 24..31), so one OR of the
// four words flags the group; valid quads stay below 2^24.
__device__ __forceinline__ uint32_t b64_decode_group_full(uint4 w, const B64Tables* t, int32_t codes[3]) {
  const uint32_t words[4] = {w.x, w.y, w.z, w.w};
  const int8_t* from = reinterpret_cast<const int8_t*>(t->from);
  uint32_t sx[16], V[4];
#pragma unroll
  for (int qd = 0; qd < 4; ++qd) {
    sx[4 * qd] = (uint32_t)(int32_t)from[words[qd] & 0xff];
    sx[4 * qd + 1] = (uint32_t)(int32_t)from[(words[qd] >> 8) & 0xff];
    sx[4 * qd + 2] = (uint32_t)(int32_t)from[(words[qd] >> 16) & 0xff];
    sx[4 * qd + 3] = (uint32_t)(int32_t)from[words[qd] >> 24];
  }
  group24(sx, V);
  codes[0] = (int32_t)__builtin_amdgcn_perm(V[1], V[0], 0x06000102u);
  codes[1] = (int32_t)__builtin_amdgcn_perm(V[2], V[1], 0x05060001u);
  codes[2] = (int32_t)__builtin_amdgcn_perm(V[3], V[2], 0x04050600u);
  return (V[0] | V[1] | V[2] | V[3]) >> 24;
}

// One code of a group from the two 4-char quads that hold its bytes: value e of
// the group is bytes 4e..4e+3, i.e. quads e and e+1 (w0, w1 = chars 4e..4e+7);
// `sel` = b64_pair_selector(e). For lanes that own one value of a group.
__device__ __forceinline__ uint32_t b64_pair_selector(int e) {
  return e == 0 ? 0x06000102u : e == 1 ? 0x05060001u : 0x04050600u;  // the perms of b64_decode_group
}
// all 8 chars carry data: nonzero if any is outside the alphabet
__device__ __forceinline__ uint32_t b64_decode_pair_full(uint32_t w0, uint32_t w1, uint32_t sel, const B64Tables* t,
                                                         int32_t& code) {
  const uint32_t words[2] = {w0, w1};
  const int8_t* from = reinterpret_cast<const int8_t*>(t->from);  // sign-extended: see b64_decode_group_full
  uint32_t V[2];
#pragma unroll
  for (int qd = 0; qd < 2; ++qd) {
    const uint32_t s0 = (uint32_t)(int32_t)from[words[qd] & 0xff];
    const uint32_t s1 = (uint32_t)(int32_t)from[(words[qd] >> 8) & 0xff];
    const uint32_t s2 = (uint32_t)(int32_t)from[(words[qd] >> 16) & 0xff];
    const uint32_t s3 = (uint32_t)(int32_t)from[words[qd] >> 24];
    V[qd] = (((s0 << 6) | s1) << 12) | ((s2 << 6) | s3);
  }
  code = (int32_t)__builtin_amdgcn_perm(V[1], V[0], sel);
  return (V[0] | V[1]) >> 24;
}
// per-char mask of chars outside the alphabet (bit i = char 4e + i)
__device__ __forceinline__ uint32_t b64_decode_pair(uint32_t w0, uint32_t w1, uint32_t sel, const B64Tables* t,
                                                    int32_t& code) {
  const uint32_t words[2] = {w0, w1};
  const int8_t* from = reinterpret_cast<const int8_t*>(t->from);
  uint32_t V[2], bad = 0;
#pragma unroll
  for (int qd = 0; qd < 2; ++qd) {
    const uint32_t s0 = (uint32_t)(int32_t)from[words[qd] & 0xff];  // sign-extended, as above
    const uint32_t s1 = (uint32_t)(int32_t)from[(words[qd] >> 8) & 0xff];
    const uint32_t s2 = (uint32_t)(int32_t)from[(words[qd] >> 16) & 0xff];
    const uint32_t s3 = (uint32_t)(int32_t)from[words[qd] >> 24];
    bad |= ((s0 >> 31) | ((s1 >> 31) << 1) | ((s2 >> 31) << 2) | ((s3 >> 31) << 3)) << (4 * qd);
    V[qd] = ((s0 & 63) << 18) | ((s1 & 63) << 12) | ((s2 & 63) << 6) | (s3 & 63);
  }
  code = (int32_t)__builtin_amdgcn_perm(V[1], V[0], sel);
  return bad;
}

// 3 codes -> 12 bytes -> 16 chars (Base64.cpp:141-162).
__device__ __forceinline__ uint4 b64_encode_group(const int32_t codes[3], const B64Tables* t) {
  const uint32_t c0 = (uint32_t)codes[0], c1 = (uint32_t)codes[1], c2 = (uint32_t)codes[2];
  // inverse of the perms above: V[q] = 24-bit big-endian view of bytes 3q..3q+2
  uint32_t V[4];
  V[0] = __builtin_amdgcn_perm(0u, c0, 0x0c000102u);  // b0<<16 | b1<<8 | b2
  V[1] = __builtin_amdgcn_perm(c1, c0, 0x0c030405u);  // b3<<16 | b4<<8 | b5
  V[2] = __builtin_amdgcn_perm(c2, c1, 0x0c020304u);  // b6<<16 | b7<<8 | b8
  V[3] = __builtin_amdgcn_perm(0u, c2, 0x0c010203u);  // b9<<16 | b10<<8 | b11
  uint32_t ch[16];
#pragma unroll
  for (int qd = 0; qd < 4; ++qd) {
    ch[4 * qd] = t->to[(V[qd] >> 18) & 63];
    ch[4 * qd + 1] = t->to[(V[qd] >> 12) & 63];
    ch[4 * qd + 2] = t->to[(V[qd] >> 6) & 63];
    ch[4 * qd + 3] = t->to[V[qd] & 63];
  }
  // chars a, b, c, d of a quad -> a | b << 8 | c << 16 | d << 24: three v_lshl_or per
  // word (the OR form takes four), the group's twelve in one asm block (see group24)
  uint32_t out[4], p0, q0, p1, q1, p2, q2, p3, q3;
  asm("v_lshl_or_b32 %4, %13, 8, %12\n\t"
      "v_lshl_or_b32 %5, %15, 8, %14\n\t"
      "v_lshl_or_b32 %6, %17, 8, %16\n\t"
      "v_lshl_or_b32 %7, %19, 8, %18\n\t"
      "v_lshl_or_b32 %8, %21, 8, %20\n\t"
      "v_lshl_or_b32 %9, %23, 8, %22\n\t"
      "v_lshl_or_b32 %10, %25, 8, %24\n\t"
      "v_lshl_or_b32 %11, %27, 8, %26\n\t"
      "v_lshl_or_b32 %0, %5, 16, %4\n\t"
      "v_lshl_or_b32 %1, %7, 16, %6\n\t"
      "v_lshl_or_b32 %2, %9, 16, %8\n\t"
      "v_lshl_or_b32 %3, %11, 16, %10"
      : "=v"(out[0]), "=v"(out[1]), "=v"(out[2]), "=v"(out[3]), "=&v"(p0), "=&v"(q0), "=&v"(p1), "=&v"(q1),
        "=&v"(p2), "=&v"(q2), "=&v"(p3), "=&v"(q3)
      : "v"(ch[0]), "v"(ch[1]), "v"(ch[2]), "v"(ch[3]), "v"(ch[4]), "v"(ch[5]), "v"(ch[6]), "v"(ch[7]), "v"(ch[8]),
        "v"(ch[9]), "v"(ch[10]), "v"(ch[11]), "v"(ch[12]), "v"(ch[13]), "v"(ch[14]), "v"(ch[15]));
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
