// fleet_amd/csrc/kernels.hip -- gfx950 kernels of the FLeet codec / aggregation path.
//
// Data layout in HBM: client uploads are rows of `pitch` bytes
// (pitch % 16 == 0) of Base64 text. One lane owns one 16-char group = 12
// bytes = 3 int32 codes = 3 gradient values, and walks every client row in
// order (the per-element chain is serial across clients, CppNNUpdater.java:
// 420-509); a wave reads 1 KiB contiguous per client row (global_load_dwordx4).
#include "kernels.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>

#include "codec_device.h"
#include "decimal6.h"
#include "teacher_math.h"

// Experiment switches of the stream kernels (r05 A/Bs; the defaults are the product):
// FLEET_TILE_LADDER = 0: the classic / woven tiles without the progress priority ladder.
#ifndef FLEET_TILE_LADDER
#define FLEET_TILE_LADDER 1
#endif

namespace fleet {

// Dev-only phase timestamps (scripts/ubench_tiled.hip builds with FLEET_TIMING);
// compiled out of the library.
#ifdef FLEET_TIMING
__device__ unsigned long long g_fleet_timing[16384 * 8];
#define FLEET_TSTAMP(slot)                                                                  \
  do {                                                                                      \
    if (threadIdx.x == 0) g_fleet_timing[blockIdx.x * 8 + (slot)] = wall_clock64();        \
  } while (0)
#else
#define FLEET_TSTAMP(slot) \
  do {                     \
  } while (0)
#endif
// Dev-only per-wave phase trace of the tile kernels (FLEET_TRACE builds: scripts/tile_trace.py):
// the shader clock at phase boundaries of tiles 0..63, chunk k < 64, wave w < 8, slot s < 4;
// stored by lane 0 with vector stores. Compiled out of the library.
#ifdef FLEET_TRACE
#ifndef FLEET_TRACE_WAVES  // 0: block start / end only (fewer SGPRs: the kernel keeps its residency)
#define FLEET_TRACE_WAVES 1
#endif
static __device__ unsigned long long* g_fleet_trace;
#define FLEET_WTRACE(tile, k, slot)                                                                        \
  do {                                                                                                     \
    if (FLEET_TRACE_WAVES && g_fleet_trace && (tile) < 64 && (k) < 64 && (threadIdx.x & 63) == 0)          \
      g_fleet_trace[((((tile) * 64 + (k)) * 8 + (threadIdx.x >> 6)) * 4) + (slot)] = clock64();          \
  } while (0)
// per block (dispatch order blockIdx.x < 65536): the constant 100 MHz clock at its start and
// end and its hardware id (XCC, SE, CU): residency and rounds of a launch
#define FLEET_BTRACE(slot)                                                                                  \
  do {                                                                                                      \
    if (g_fleet_trace && blockIdx.x < 65536 && threadIdx.x == 0) {                                         \
      unsigned long long* bt_ = g_fleet_trace + 64 * 64 * 8 * 4 + (size_t)blockIdx.x * 4;                 \
      bt_[slot] = wall_clock64();                                                                           \
      if ((slot) == 0)                                                                                      \
        bt_[2] = ((unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) << 32) |  \
                 (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));          \
    }                                                                                                       \
  } while (0)
#else
#define FLEET_WTRACE(tile, k, slot) \
  do {                              \
  } while (0)
#define FLEET_BTRACE(slot) \
  do {                     \
  } while (0)
#endif
// Dev-only per-wave progress trace of the stream kernels' client loop
// (scripts/ubench_window.hip defines it); compiled out of the library.
#ifndef FLEET_CLIENT_HOOK
#define FLEET_CLIENT_HOOK(c, M) \
  do {                          \
  } while (0)
#endif

// 16-byte store of data no later access in this kernel touches and that is far
// larger than the caches (the client texts): a non-temporal store
// (scripts/ubench_stream.hip: the encode's 12 B in / 16 B out pattern 0.414 ->
// 0.395 ms on the headline size)
__device__ __forceinline__ void store_stream16(uint8_t* p, uint4 v) {
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(u4v{v.x, v.y, v.z, v.w}, reinterpret_cast<u4v*>(p));
}
// chars of the group that must be alphabet chars, for r valid int32 values
__device__ __forceinline__ uint32_t needed_chars_mask(int r) {
  return r >= 3 ? 0xffffu : r == 2 ? 0x7ffu : r == 1 ? 0x3fu : 0u;
}

// Base64.cpp:164-166 -- trailing '=' for the missing bytes of a partial group
__device__ __forceinline__ uint4 pad_group(uint4 v, int r) {
  if (r == 1) {  // 4 bytes -> 6 chars + "=="
    v.y = (v.y & 0x0000ffffu) | 0x3d3d0000u;
    v.z = 0;
    v.w = 0;
  } else if (r == 2) {  // 8 bytes -> 11 chars + "="
    v.z = (v.z & 0x00ffffffu) | 0x3d000000u;
    v.w = 0;
  }
  return v;
}

__device__ __forceinline__ int headers_in_group(const int32_t* __restrict__ hdr, int n_hdr, int64_t p0,
                                                bool is_hdr[3]) {
  // hdr is sorted; n_hdr is small (layers), a binary search keeps it O(log n)
  int lo = 0, hi = n_hdr;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (hdr[mid] < p0) lo = mid + 1; else hi = mid;
  }
  int cnt = 0;
#pragma unroll
  for (int e = 0; e < 3; ++e) is_hdr[e] = false;
  for (int i = lo; i < n_hdr && hdr[i] < p0 + 3; ++i) {
    is_hdr[hdr[i] - p0] = true;
    ++cnt;
  }
  return cnt;
}

// bit e set = value slot p0+e is a layout header slot
__device__ __forceinline__ uint32_t header_bits(const int32_t* __restrict__ hdr, int n_hdr, int64_t p0) {
  bool ih[3];
  headers_in_group(hdr, n_hdr, p0, ih);
  return (uint32_t)ih[0] | ((uint32_t)ih[1] << 1) | ((uint32_t)ih[2] << 2);
}

// out[i] = Q(x[i]) for a stage of S values: fixed 9-step chains when the
// whole wave is in |x| < 1, else the multiplier-table chains (codec_math.h:
// no selects, no packed ops -- the cheap encodings on gfx950); the general
// codec, per lane, for the values outside the q_gen domain.
template <int S>
__device__ __forceinline__ void q_stage(float (&out)[S], const float (&x)[S], const B64Tables* tab) {
  // integer magnitude tests (an f32 compare with |.| is a 6-cycle e64 op):
  // the whole wave is in |x| < 1 iff the largest |x| bit pattern is
  uint32_t ab[S], amax = 0;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    ab[i] = f2u(x[i]) & 0x7fffffffu;
    amax = max(amax, ab[i]);
  }
  if (__ballot(amax >= 0x3f800000u) == 0) {
#pragma unroll
    for (int i = 0; i < S; ++i) out[i] = q_fast1(x[i]);
    return;
  }
  uint32_t d[S], dmax = 0;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    d[i] = var_digits_ab(f2u(x[i]), ab[i], tab->var);
    dmax = max(dmax, d[i]);
    out[i] = q_mt_d(x[i], d[i], tab->mt);
  }
  if (__ballot(dmax > 9u) != 0) {  // values outside the q_gen domain (rare): the general codec, per lane
#pragma unroll
    for (int i = 0; i < S; ++i)
      if (d[i] > 9u) out[i] = q(x[i]);
  }
}

// q_stage without the in-stage fallback: values outside the q_gen domain leave
// their lane's results undefined and raise `dmax` above 9; the caller then
// recomputes that lane's whole chain with the general codec (chain_general).
// One max per value instead of the compaction machinery in every stage.
template <int S>
__device__ __forceinline__ void q_stage_off(float (&out)[S], const float (&x)[S], const B64Tables* tab,
                                            uint32_t& dmax) {
  uint32_t ab[S], amax = 0;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    ab[i] = f2u(x[i]) & 0x7fffffffu;
    amax = max(amax, ab[i]);
  }
  if (__ballot(amax >= 0x3f800000u) == 0) {
#pragma unroll
    for (int i = 0; i < S; ++i) out[i] = q_fast1(x[i]);
    return;
  }
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const uint32_t d = var_digits_ab(f2u(x[i]), ab[i], tab->var);
    dmax = max(dmax, d);
    out[i] = q_mt_d(x[i], d, tab->mt);
  }
}

// q_stage_off with the byte-table digit count (codec_math.h q_d16): one byte
// load per value gives the step tables' offset; lanes in a power-of-ten slice
// (rare) take the compare; values outside the q_gen domain raise `dmax` to
// >= kD16Out and leave their results undefined (the caller recomputes them).
template <int S>
__device__ __forceinline__ void q_stage_d16(float (&out)[S], const float (&x)[S], const D16Table* dt,
                                            const VarEntry* vt, uint32_t& dmax) {
  uint32_t e[S], emax = 0;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    e[i] = dt->d16[f2u(x[i]) >> 19];
    emax = max(emax, e[i]);
  }
  if (__ballot(emax >= kD16Out) != 0) {  // compare slices / out of domain (wave-uniform branch)
    emax = 0;
#pragma unroll
    for (int i = 0; i < S; ++i) {
      if (e[i] == kD16Cmp) e[i] = d16_fix(x[i], vt);
      emax = max(emax, e[i]);
    }
  }
  dmax = max(dmax, emax);
#pragma unroll
  for (int i = 0; i < S; ++i) out[i] = q_d16(x[i], e[i], &dt->st);
}

// q_stage_d16 with the digit offsets from the VarEntry compare (var_d16): branch-
// free, for the serial accumulation A = Q(A + p) whose sums hit the byte table's
// compare slices in most waves.
template <int S>
__device__ __forceinline__ void q_stage_v16(float (&out)[S], const float (&x)[S], const D16Table* dt,
                                            const VarEntry* vt, uint32_t& dmax) {
  uint32_t e[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    e[i] = var_d16(f2u(x[i]), vt);
    dmax = max(dmax, e[i]);
  }
#pragma unroll
  for (int i = 0; i < S; ++i) out[i] = q_d16(x[i], e[i], &dt->st);
}

// int2float for the stream kernel: the step multipliers from the stride-16 tables
// by the code's last digit (total, no fast-path test: the table chain costs what
// the fixed one does).
template <int S>
__device__ __forceinline__ void dec_stage_d16(float (&out)[S], const int32_t (&codes)[S], const D16Table* dt) {
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const uint32_t a = codes[i] < 0 ? 0u - (uint32_t)codes[i] : (uint32_t)codes[i];
    out[i] = dec_d16(codes[i], last_digit_u(a) << 4, &dt->st);
  }
}

// dec_stage_d16 with the step count from the byte-sum table (codec_math.h ld16_entry):
// three VALU instructions and one LDS byte read for the six of the mulhi remainder
// (the stream kernels, which have the LDS for its 4 KB)
template <int S>
__device__ __forceinline__ void dec_stage_ld16(float (&out)[S], const int32_t (&codes)[S], const D16Table* dt,
                                               const uint8_t* ld16) {
#pragma unroll
  for (int i = 0; i < S; ++i) out[i] = dec_d16(codes[i], ld16[ld16_index(codes[i])], &dt->st);
}

// q_stage_d16 with the exact in-stage fallback (the general codec per lane for
// values outside the q_gen domain): a drop-in for q_stage where every stage
// output is used (Kardam's side outputs).
template <int S>
__device__ __forceinline__ void q_stage_d16x(float (&out)[S], const float (&x)[S], const D16Table* dt,
                                             const VarEntry* vt) {
  uint32_t e[S], emax = 0;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    e[i] = dt->d16[f2u(x[i]) >> 19];
    emax = max(emax, e[i]);
  }
  if (__ballot(emax >= kD16Out) != 0) {
    emax = 0;
#pragma unroll
    for (int i = 0; i < S; ++i) {
      if (e[i] == kD16Cmp) e[i] = d16_fix(x[i], vt);
      emax = max(emax, e[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < S; ++i) out[i] = q_d16(x[i], e[i], &dt->st);
  if (__ballot(emax >= kD16Out) != 0) {
#pragma unroll
    for (int i = 0; i < S; ++i)
      if (e[i] >= kD16Out) out[i] = q(x[i]);
  }
}

// scalarMultiply(getDampen) (cppNN_backend.cpp:753-777): (float)((double)y * d).
// When d is a binary32 value (1, 1/2, ... -- staleness 0 gives 1 under every
// getDampen policy) the double product of two binary32 values is exact and one
// binary32 multiply rounds it identically. d is uniform (one client per step of
// every lane), and the test and the binary32 bits are integer work on its two
// words -- scalar instructions, no VALU; the volatile asm keeps the f64 side a
// branch (the compiler would otherwise compute both sides and select).
template <int S>
__device__ __forceinline__ void dampen_stage(float (&r)[S], double d) {
  const uint64_t b = __builtin_bit_cast(uint64_t, d);
  const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
  const uint32_t ex = (hi >> 20) & 0x7ffu;
  // a binary32 normal value: f64 biased exponent 897..1150, no mantissa bits below
  // binary32's (+-0 and the rest take the f64 side, exact for every d)
  if ((lo & 0x1fffffffu) == 0 && ex - 897u < 254u) {
    const float df = u2f((hi & 0x80000000u) | ((ex - 896u) << 23) | ((hi & 0xfffffu) << 3) | (lo >> 29));
#pragma unroll
    for (int i = 0; i < S; ++i) r[i] = r[i] * df;
  } else {
    asm volatile("");
#pragma unroll
    for (int i = 0; i < S; ++i) r[i] = (float)((double)r[i] * d);
  }
}

// out[i] = int2float(codes[i]) (Base64.cpp:80-103): fixed 9-step chains when
// every code of the wave ends in 0 (|value| < 1), else step multipliers from
// the last digit. Total: no fallback needed.
template <int S>
__device__ __forceinline__ void dec_stage(float (&out)[S], const int32_t (&codes)[S], const B64Tables* tab) {
  uint32_t r[S], rmax = 0;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const uint32_t a = codes[i] < 0 ? 0u - (uint32_t)codes[i] : (uint32_t)codes[i];
    r[i] = last_digit_u(a);
    rmax = max(rmax, r[i]);
  }
  if (__ballot(rmax != 0u) == 0) {
#pragma unroll
    for (int i = 0; i < S; ++i) out[i] = dec_fast(codes[i]);
  } else {
#pragma unroll
    for (int i = 0; i < S; ++i) out[i] = dec_mt_r(codes[i], r[i], tab->mt);
  }
}


// ----------------------------------------------------------------------------
// One merged slot (mergeFlatGradient, cppNN_backend.cpp:722-750, after
// scalarMultiply(1.0/avgSize), CppNNUpdater.java:507-508): header and unwalked
// slots re-encode the last upload's decoded value, payload slots encode
// Q(f32(f64(A) * inv)). Variable-length chains on their domain, the general
// codec for the rest (divergent, rare).
__device__ __forceinline__ int32_t merged_code(float A, double inv, int32_t last_code, bool keep_last,
                                               const B64Tables* tab) {
  if (keep_last) return enc(dec(last_code));
  const float r = (float)((double)A * inv);
  const uint32_t d = var_digits(r, tab->var);
  if (d <= 9u) {
    const float y = q_mt_d(r, d, tab->mt);
    if (var_digits(y, tab->var) <= 9u) return enc_mt(y, tab->var, tab->mt);
  }
  return enc(q(r));
}

// Keep slots: layout header slots and slots past network::flatGrad's walk take the
// last upload's code in the merged output (mergeFlatGradient, cppNN_backend.cpp:722-750),
// so their running sums are never read. The chain runs on code 0 there (Q(0) = 0; the
// stream kernels keep the last client's codes, which the merged output needs): a header
// value summed over thousands of clients (configs[4]: the bucket size 4,194,304 at
// position 1) would otherwise leave the codec's fast domain and send its lane through
// chain_general -- one straggler wave that doubled the configs[4] window kernels
// (DESIGN.md §5). Bit i of the result = slot p0 + i of the lane is a keep slot.
template <int S>
__device__ __forceinline__ uint32_t keep_bits(uint32_t hbits, bool live, int64_t p0, int64_t walk_end) {
  uint32_t k = hbits;
#pragma unroll
  for (int i = 0; i < S; ++i)
    if (live && p0 + i >= walk_end) k |= 1u << i;
  return k;
}

// The exact chain of one value recomputed from global memory with the general
// codec: the fallback when the serial accumulation leaves the fast domain
// (|A| >= 1e8 or 1e9; never for gradients). Per lane, divergent, slow, exact; the
// next client's group is loaded while the current one is computed.
__device__ __noinline__ float chain_general(const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                            const double* __restrict__ dampen, int64_t g, int e,
                                            const B64Tables* tab) {
  float A = 0.f;
  const uint8_t* row = uploads + 16 * g;
  uint4 nxt = *reinterpret_cast<const uint4*>(row);
  for (int c = 0; c < M; ++c) {
    const uint4 cur = nxt;
    if (c + 1 < M) nxt = *reinterpret_cast<const uint4*>(row + (size_t)(c + 1) * pitch);
    int32_t cc[3];
    b64_decode_group(cur, tab, cc);
    const float y = q(dec(cc[e]));
    const float p = q((float)((double)y * dampen[c]));
    A = c == 0 ? p : q(A + p);
  }
  return A;
}

// ----------------------------------------------------------------------------
// Fused update: CppNNUpdater.update's aggregation (java:420-509) for the
// groups [g_begin, g_end). Per value and client c, in CppNNUpdater order:
//   y = Q(dec(code_c))                  getFlatGradient decode+encode, scalarMul decode
//   p = Q((float)((double)y * d_c))     scalarMultiply(getDampen) encode, add decode
//   A = (c == 0) ? p : Q(A + p)         ByteVec.add encode/decode
// then r = Q((float)((double)A * inv)) (scalarMultiply(1/avgSize) + merge decode) and
// merged code = enc(r); header slots take enc(dec(code_{M-1})) (mergeFlatGradient).
//
// The stream form (update_lane, k_update_mixed): a lane walks one group (or one
// value) down all M client rows, so every wave-wide load of a client row is 1 KiB
// contiguous; the next client's loads are in flight while the current one computes.
// KD = true adds Kardam's bookkeeping of the same picked uploads (CppNNUpdater.java:
// 463-481, Kardam.java:48-106) as side outputs of the client loop
// (KardamOut), so it costs no second pass over the uploads; stages A and B then
// use the exact in-stage fallback (their values feed the side outputs).
//
// Sum of v over each aligned group of TG lanes (16, 32 or 64), valid in the
// group's last lane, by DPP lane moves inside the VALU (no LDS crossbar):
// row_half_mirror + two quad_perms + row_mirror give every lane its 16-lane row's
// sum, row_bcast15 / row_bcast31 then fold rows 0+1, 2+3 and 0..3. Call with
// every lane of the wave active.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_move_f64(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, ROW_MASK, 0xf, false);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int TG>
__device__ __forceinline__ double group_sum_f64(double v) {
  static_assert(TG == 16 || TG == 32 || TG == 64, "DPP group sums over rows of 16 lanes");
  v += dpp_move_f64<0x141, 0xf>(v);  // row_half_mirror
  v += dpp_move_f64<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
  v += dpp_move_f64<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
  v += dpp_move_f64<0x140, 0xf>(v);  // row_mirror: every lane holds its row's sum
  if constexpr (TG >= 32) v += dpp_move_f64<0x142, 0xa>(v);  // row_bcast15 into rows 1, 3
  if constexpr (TG == 64) v += dpp_move_f64<0x143, 0x8>(v);  // row_bcast31 into row 3
  return v;
}

// Two sums at once (Kardam's squared norms): the sums of a and of b over each aligned
// group of TG lanes (16, 32 or 64), a's valid in lane TG/2 - 1 of the group, b's in lane
// TG - 1. One gfx950 half swap (v_permlane32_swap / v_permlane16_swap: the upper half
// of a's group against the lower half of b's) and one add fold the pair into one
// register -- a's group halves summed in the group's lower half, b's in the upper --,
// then one group_sum_f64 of half the width: 3 + 15 instructions for TG = 64 against
// 36 for two group_sum_f64<64>. Every lane of the wave active.
template <int TG>
__device__ __forceinline__ double pair_sum_f64(double a, double b) {
  static_assert(TG == 16 || TG == 32 || TG == 64, "half swaps of 32 or 16 lanes, a row mirror");
  if constexpr (TG == 16) {
    // a 16-lane row: each lane keeps a (lanes 0-7 of the row) or b (8-15) and takes its
    // mirror lane's other value (row_mirror: lane i reads 15 - i, the other half), then
    // the half's three DPP steps: 16 instructions against 24 for two group_sum_f64<16>
    const bool up = (threadIdx.x & 8) != 0;
    double v = (up ? b : a) + dpp_move_f64<0x140, 0xf>(up ? a : b);
    v += dpp_move_f64<0x141, 0xf>(v);  // row_half_mirror
    v += dpp_move_f64<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
    v += dpp_move_f64<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
    return v;
  } else {
    const uint64_t ab = __builtin_bit_cast(uint64_t, a), bb = __builtin_bit_cast(uint64_t, b);
    const uint32_t alo = (uint32_t)ab, ahi = (uint32_t)(ab >> 32), blo = (uint32_t)bb, bhi = (uint32_t)(bb >> 32);
    double x, y;
    if constexpr (TG == 64) {
      const auto lo = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
      const auto hi = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
      x = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
      y = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
    } else {
      const auto lo = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
      const auto hi = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
      x = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
      y = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
    }
    return group_sum_f64<TG / 2>(x + y);
  }
}

// Four sums at once (Kardam's squared norms of two clients): a and b fold into the two
// wave halves and c and d likewise (pair_sum_f64<64>'s first step), one permlane16 swap
// folds the two results into one register by 16-lane rows -- a, c, b, d in rows 0..3 --
// and one group_sum_f64<16> finishes: the sums in lanes 15 (a), 31 (c), 47 (b) and 63
// (d); 21 instructions against 36 for two pair_sum_f64<64>. Every lane of the wave active.
__device__ __forceinline__ double quad_sum_f64(double a, double b, double c, double d) {
  auto fold32 = [](double u, double v) {
    const uint64_t ub = __builtin_bit_cast(uint64_t, u), vb = __builtin_bit_cast(uint64_t, v);
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)ub, (uint32_t)vb, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(ub >> 32), (uint32_t)(vb >> 32), false, false);
    return __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]) +
           __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
  };
  const double x = fold32(a, b), y = fold32(c, d);
  const uint64_t xb = __builtin_bit_cast(uint64_t, x), yb = __builtin_bit_cast(uint64_t, y);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)xb, (uint32_t)yb, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(xb >> 32), (uint32_t)(yb >> 32), false, false);
  return group_sum_f64<16>(__builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]) +
                           __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]));
}

// Kardam's bookkeeping of one client step in a stream lane (KD = true; SURVEY.md f2,
// CppNNUpdater.java:463-481, Kardam.java:48-106): G = Q(f32(f64(p) * lr)) -- the
// picked gradient scalarMultiply(getLrate()) --, its squared norm and that of
// Q(G - prev) (getNorm: float products summed in double), G stored in upload
// coordinates for the next round's difference. `flat` bit i = value slot pos0 + i
// is in the flat gradient (neither a header slot nor past the walk). The wave's
// two per-lane sums are returned (sg, sd); the stream loop reduces them over the wave two
// clients at a time (quad_sum_f64) into the wave's partial slots (k_kardam_reduce sums the waves).
// The worker's previous G at the lane's slots (0 off the flat gradient): loaded a client
// ahead by the stream loop, so the HBM latency of the prev rows overlaps the current
// client's chain instead of stalling it. Returns has_prev[c] (uniform).
template <int S>
__device__ __forceinline__ bool kardam_prev_load(const KardamOut& kd, int c, uint32_t flat, bool live, int64_t pos0,
                                                 int64_t n_up, float (&pv)[S]) {
  typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));
#pragma unroll
  for (int i = 0; i < S; ++i) pv[i] = 0.0f;
  if (!(kd.prev && kd.has_prev[c])) return false;  // uniform
  const float* pr = kd.prev + (size_t)c * kd.vpitch + pos0;
  if constexpr (S == 3) {
    if (live && pos0 + S - 1 < n_up) {  // one 12-byte access per group (rows are 4-byte aligned)
      const f3u t = *reinterpret_cast<const f3u*>(pr);
      pv[0] = t.x;
      pv[1] = t.y;
      pv[2] = t.z;
    } else {
#pragma unroll
      for (int i = 0; i < S; ++i) pv[i] = ((flat >> i) & 1u) ? pr[i] : 0.0f;
    }
  } else {
    pv[0] = (flat & 1u) ? pr[0] : 0.0f;
  }
  return true;
}

// FULL: every lane of the wave has all S slots in the flat gradient (flat = 2^S - 1,
// a whole group in range): no per-slot selects (the common wave, taken by a uniform
// branch hoisted out of the client loop).
template <int S, bool FULL = false>
__device__ __forceinline__ void kardam_lane_step(const float (&p)[S], int c, uint32_t flat, bool live, int64_t pos0,
                                                 int64_t n_up, const KardamOut& kd, const D16Table& dtab,
                                                 const B64Tables& tab, bool hasp, const float (&pv)[S], double& sg,
                                                 double& sd) {
  typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));
  if constexpr (FULL) {
    flat = (1u << S) - 1u;
    live = true;
  }
  float rg[S], G[S];
#pragma unroll
  for (int i = 0; i < S; ++i) rg[i] = p[i];
  dampen_stage<S>(rg, kd.lr);  // lr is uniform
  q_stage_d16x<S>(G, rg, &dtab, tab.var);
  sg = 0.0;
  sd = 0.0;
#pragma unroll
  for (int i = 0; i < S; ++i)
    if ((flat >> i) & 1u) sg += (double)(G[i] * G[i]);
  const bool whole = FULL || (live && pos0 + S - 1 < n_up);
  if (hasp) {  // uniform
    float dv[S], D[S];
#pragma unroll
    for (int i = 0; i < S; ++i) dv[i] = ((flat >> i) & 1u) ? G[i] - pv[i] : 0.0f;
    q_stage_d16x<S>(D, dv, &dtab, tab.var);
#pragma unroll
    for (int i = 0; i < S; ++i)
      if ((flat >> i) & 1u) sd += (double)(D[i] * D[i]);
  }
  if (kd.g_out) {
    float* go = kd.g_out + (size_t)c * kd.vpitch + pos0;
    float gv[S];
#pragma unroll
    for (int i = 0; i < S; ++i) gv[i] = ((flat >> i) & 1u) ? G[i] : 0.0f;
    if constexpr (S == 3) {
      if (whole) {
        *reinterpret_cast<f3u*>(go) = f3u{gv[0], gv[1], gv[2]};
      } else {
#pragma unroll
        for (int i = 0; i < S; ++i)
          if (live && pos0 + i < n_up) go[i] = gv[i];
      }
    } else {
      if (FULL || (live && pos0 < n_up)) go[0] = gv[0];
    }
  }
}

// The wave's norm partials of clients c - 1 and c (held sums sg0, sd0 and this client's
// sg, sd) into their slots, or of client c alone when it is the last and even; nothing
// for an even client with a successor (its sums are held). Every lane of the wave here;
// c uniform.
__device__ __forceinline__ void kardam_wave_partials(int c, int M, double& sg0, double& sd0, double sg, double sd,
                                                     double* __restrict__ part, size_t stride) {
  if (c & 1) {
    const double s = quad_sum_f64(sg0, sd0, sg, sd);
    const int lane = threadIdx.x & 63;
    if ((lane & 15) == 15)  // rows 0..3: (c - 1, g), (c, g), (c - 1, d), (c, d)
      part[(size_t)(c - 1 + ((lane >> 4) & 1)) * stride + (lane >> 5)] = s;
  } else if (c + 1 == M) {
    const double s = pair_sum_f64<64>(sg, sd);
    if ((threadIdx.x & 31) == 31) part[(size_t)c * stride + ((threadIdx.x >> 5) & 1)] = s;
  } else {
    sg0 = sg;
    sd0 = sd;
  }
}

// Client-side encode: rows of fp32 -> rows of Base64 (Base64::encode(vector<float>)).
// One group (3 values) of one row: float2int (fixed chains when the wave is
// in |x| < 1, multiplier-table chains otherwise, the general codec for values
// outside the q_gen domain) and the 16 Base64 chars.
__device__ __forceinline__ uint4 encode_group(const float (&x)[3], int r, const B64Tables* tab,
                                              const D16Table* dt) {
  int32_t codes[3];
  // |x| < 1 for the whole wave iff the largest |x| bit pattern is (integer max,
  // not three 6-cycle e64 compares)
  uint32_t amax = 0;
#pragma unroll
  for (int e = 0; e < 3; ++e) amax = max(amax, f2u(x[e]) & 0x7fffffffu);
  if (__ballot(amax >= 0x3f800000u) == 0) {  // wave-uniform: gradients, |x| < 1
#pragma unroll
    for (int e = 0; e < 3; ++e) codes[e] = enc_fast(x[e]);
  } else {
    // byte-table digit counts (codec_math.h d16_entry): one byte load per value;
    // the power-of-ten slices take the compare, values outside the q_gen
    // domain (|x| >= 1e8/1e9, inf, NaN) the general codec -- both rare, per lane
    uint32_t ofs[3], omax = 0;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      ofs[e] = dt->d16[f2u(x[e]) >> 19];
      omax = max(omax, ofs[e]);
    }
    if (__ballot(omax >= kD16Out) != 0) {
      omax = 0;
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        if (ofs[e] == kD16Cmp) ofs[e] = d16_fix(x[e], tab->var);
        omax = max(omax, ofs[e]);
      }
    }
#pragma unroll
    // offsets >= kD16Out read the tables' identity rows (garbage codes, never a fault;
    // replaced below), so no select is spent on the common path
    for (int e = 0; e < 3; ++e) codes[e] = enc_d16(x[e], ofs[e], &dt->st);
    if (__ballot(omax >= kD16Out) != 0) {
#pragma unroll
      for (int e = 0; e < 3; ++e)
        if (ofs[e] >= kD16Out) codes[e] = enc(x[e]);
    }
  }
  return pad_group(b64_encode_group(codes, tab), r);
}

// The same with the VarEntry digit counts (kernels that keep only B64Tables in LDS)
__device__ __forceinline__ uint4 encode_group(const float (&x)[3], int r, const B64Tables* tab) {
  int32_t codes[3];
  const bool fast = q_ok(x[0]) && q_ok(x[1]) && q_ok(x[2]);
  if (__ballot(!fast) == 0) {  // wave-uniform: gradients, |x| < 1
#pragma unroll
    for (int e = 0; e < 3; ++e) codes[e] = enc_fast(x[e]);
  } else {
#pragma unroll
    for (int e = 0; e < 3; ++e) codes[e] = enc_mt(x[e], tab->var, tab->mt);
    if (!(q_gen_ok(x[0]) && q_gen_ok(x[1]) && q_gen_ok(x[2]))) {  // |x| >= 1e8/1e9, inf, NaN
#pragma unroll
      for (int e = 0; e < 3; ++e) codes[e] = enc(x[e]);
    }
  }
  return pad_group(b64_encode_group(codes, tab), r);
}

// A client-encode job riding in an aggregation launch (k_update_encode,
// k_update_tiled_encode, k_update_pipe): k_encode_f32's grid, flattened x-fastest.
struct EncodeJob {
  const float* values;
  int64_t n;
  size_t vpitch;
  uint8_t* out;
  size_t pitch;
  int64_t groups, gx;
  int rows, rpb;
  int prio = 0;  // the encode blocks' issue priority (the tiles' fused step)
};

// s_setprio takes an immediate
__device__ __forceinline__ void encode_prio(int p) {
  if (p == 1) __builtin_amdgcn_s_setprio(1);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else if (p >= 3) __builtin_amdgcn_s_setprio(3);
}


// Buffer resource word 3 for raw byte-addressed dword loads on gfx9-family parts (gfx950),
// and the cache-policy operand of a non-temporal buffer store (the `nt` bit, as
// __builtin_nontemporal_store gives global stores: store_stream16).
constexpr int kBufferDword3 = 0x00020000;
constexpr int kBufferNT = 2;

// One lane's share of the fused update (the stream path): the values [e0, e0 + S)
// of group g, S = 3 (the whole group) or S = 1 (one value; three lanes of a wave
// share a group). Returns the lane's merged codes in out[S] and its Base64 / layout
// error bits; tables already in LDS. KD: Kardam's side outputs per client
// (kardam_lane_step; kd_part = this wave's slot of client 0, kd_stride between clients).
// LD: the kernel holds the byte-sum step-count table in LDS (ld16; dec_stage_ld16).
template <int S, bool KD = false, int LADDER = 0, bool LD = false>
__device__ __forceinline__ void update_lane(const B64Tables& tab, const D16Table& dtab,
                                            const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                            const double* __restrict__ dampen, double inv_avg, int64_t n_up,
                                            int64_t g, int e0, bool live, int64_t g_safe,
                                            const int32_t* __restrict__ hdr_block, int32_t (&out)[S],
                                            uint32_t& bad, uint32_t& layout_bad, const KardamOut& kd = KardamOut{},
                                            double* __restrict__ kd_part = nullptr, size_t kd_stride = 0,
                                            const uint8_t* __restrict__ ld16 = nullptr) {
  const int n_hdr = hdr_block[1];
  const int64_t walk_end = hdr_block[2];
  const int32_t* hdr = hdr_block + 4;
  // the lane's byte offset in a row as 32 bits (a row is one client's text, < 2^31 bytes:
  // checked by the launchers), so each row's load is a buffer load at this offset from the
  // uniform row address (scalar registers, advanced by SALU) -- no 64-bit VALU address
  // arithmetic per client
  const uint32_t lane_off = (uint32_t)(16 * (live ? g : g_safe)) + (S == 3 ? 0u : 4u * (uint32_t)e0);
  const uint32_t need = needed_chars_mask((int)min<int64_t>(3, max<int64_t>(0, n_up - 3 * g)));
  const uint32_t hbits = live ? (header_bits(hdr, n_hdr, 3 * g) >> e0) & ((1u << S) - 1u) : 0u;
  // Kardam: the lane's value slots in the flat gradient
  uint32_t flatbits = 0;
  if constexpr (KD) {
#pragma unroll
    for (int i = 0; i < S; ++i) {
      const int64_t pos = 3 * g + e0 + i;
      if (live && pos < n_up && pos < walk_end && !((hbits >> i) & 1u)) flatbits |= 1u << i;
    }
  }
  // every lane's slots all in the flat gradient (most waves): kardam_lane_step's FULL form
  const bool kd_full = KD && __ballot(flatbits != (1u << S) - 1u) == 0;
  // waves holding header slots (layout check) or keep slots (keep_bits: their chains run
  // on code 0 up to the last client, whose codes the merged output keeps): wave-uniform
  const bool wave_keep = __ballot(keep_bits<S>(hbits, live, 3 * g + e0, walk_end) != 0) != 0;
  int32_t hfirst[S], codes[S];
  float acc[S];
  uint32_t dmax = 0;
  // one client's step on its group `cur`
  // S = 1: the lane reads and decodes only the two quads that hold its value's
  // bytes (chars 4e..4e+7); the group's three lanes together cover all 16 chars
  const uint32_t sel = b64_pair_selector(e0), need_pair = (need >> (4 * e0)) & 0xffu;
  using Row = typename std::conditional<S == 3, uint4, uint2>::type;
  float kd_pv[S];       // KD: this client's prev values (loaded a client ahead)
  bool kd_hasp = false;
  double kd_sg0 = 0.0, kd_sd0 = 0.0;  // KD: the lane's norm sums of the held (even) client
  auto client = [&](int c, const Row& cur) {
    if constexpr (S == 3) {
      if (need == 0xffffu) bad |= b64_decode_group_full(cur, &tab, codes);
      else bad |= b64_decode_group(cur, &tab, codes) & need;
    } else {
      if (need == 0xffffu) bad |= b64_decode_pair_full(cur.x, cur.y, sel, &tab, codes[0]);
      else bad |= b64_decode_pair(cur.x, cur.y, sel, &tab, codes[0]) & need_pair;
    }
    if (wave_keep) {
      const uint32_t kbits = keep_bits<S>(hbits, live, 3 * g + e0, walk_end);
#pragma unroll
      for (int i = 0; i < S; ++i) {
        if (c == 0) hfirst[i] = codes[i];
        layout_bad |= (((hbits >> i) & 1u) & (uint32_t)(codes[i] != hfirst[i])) << i;
        if (((kbits >> i) & 1u) && c + 1 < M) codes[i] = 0;
      }
    }
    float y0[S], y[S], p[S];
    if constexpr (LD) dec_stage_ld16<S>(y0, codes, &dtab, ld16);
    else dec_stage_d16<S>(y0, codes, &dtab);
    if constexpr (KD) {  // stages A and B feed the side outputs: the exact in-stage fallback
      q_stage_d16x<S>(y, y0, &dtab, tab.var);
      dampen_stage<S>(y, dampen[c]);
      q_stage_d16x<S>(p, y, &dtab, tab.var);
      double sg, sd;
      if (kd_full)
        kardam_lane_step<S, true>(p, c, flatbits, live, 3 * g + e0, n_up, kd, dtab, tab, kd_hasp, kd_pv, sg, sd);
      else
        kardam_lane_step<S>(p, c, flatbits, live, 3 * g + e0, n_up, kd, dtab, tab, kd_hasp, kd_pv, sg, sd);
      kardam_wave_partials(c, M, kd_sg0, kd_sd0, sg, sd, kd_part, kd_stride);
    } else {
      q_stage_d16<S>(y, y0, &dtab, tab.var, dmax);
      dampen_stage<S>(y, dampen[c]);
      q_stage_d16<S>(p, y, &dtab, tab.var, dmax);
    }
    if (c == 0) {
#pragma unroll
      for (int i = 0; i < S; ++i) acc[i] = p[i];
    } else {
      float sm[S];
#pragma unroll
      for (int i = 0; i < S; ++i) sm[i] = acc[i] + p[i];
      q_stage_v16<S>(acc, sm, &dtab, tab.var, dmax);
    }
  };
  auto group_of = [&](int c) {
    // row c as a buffer resource built by SALU from the wave-uniform row address
    const __amdgpu_buffer_rsrc_t row = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(uploads + (size_t)c * pitch), (short)0, 0x7fffffff, kBufferDword3);
    if constexpr (S == 3) {
      typedef uint32_t u4v __attribute__((ext_vector_type(4)));
      const u4v v = __builtin_amdgcn_raw_buffer_load_b128(row, lane_off, 0, 0);
      return make_uint4(v.x, v.y, v.z, v.w);
    } else {  // two dwords at 4e (4-byte aligned only)
      return make_uint2(__builtin_amdgcn_raw_buffer_load_b32(row, lane_off, 0, 0),
                        __builtin_amdgcn_raw_buffer_load_b32(row, lane_off + 4u, 0, 0));
    }
  };
  // two clients per trip, the next client's group always in flight, in alternating
  // registers (no copies between trips)
  Row b0 = group_of(0), b1;
  int c = 0;
  // LADDER: issue priority falls as a wave gets ahead (3 -> 0 at quarters of the
  // client loop), so the waves of a SIMD keep step instead of finishing one by one in
  // age order -- the tail of a one-round grid (profiles/r04/window_traces.txt). The
  // aggregation alone: 828 -> 786 us on synth1m_256 (r04 call a6); inside
  // k_update_encode with the encode's waves at priority 2 (see there)
  // rungs at quarters of the loop; the Kardam form's longer client steps settle later
  // (rungs at 1/2, 3/4, 7/8: 1561 -> 1517 us on synth1m_256, where they cost the fused
  // step 1.8 % and rungs at 1/8, 1/4, 1/2 lose everywhere; r04 call a18)
  const int q1 = KD ? M / 2 : M / 4, q2 = KD ? 3 * M / 4 : M / 2, q3 = KD ? 7 * M / 8 : 3 * M / 4;
  // LADDER = the first rung's priority (0: no ladder); each rung one lower, floor 0
  constexpr int P0 = LADDER, P1 = LADDER > 1 ? LADDER - 1 : 0, P2 = LADDER > 2 ? LADDER - 2 : 0;
  if constexpr (LADDER > 0) __builtin_amdgcn_s_setprio(P0);
  if constexpr (KD) {
    // Kardam: one client per trip, the next one in flight (two per trip: 1840 against
    // 1795 us on synth1m_256, r04 call a13)
    float pn[S];  // the next client's prev values, in flight with its group
    bool hn = kardam_prev_load<S>(kd, 0, flatbits, live, 3 * g + e0, n_up, pn);
    for (; c < M; ++c) {
      if constexpr (LADDER > 0) {
        if (c == q1) __builtin_amdgcn_s_setprio(P1);
        if (c == q2) __builtin_amdgcn_s_setprio(P2);
        if (c == q3) __builtin_amdgcn_s_setprio(0);
      }
      const Row cur = b0;
      kd_hasp = hn;
#pragma unroll
      for (int i = 0; i < S; ++i) kd_pv[i] = pn[i];
      if (c + 1 < M) {
        b0 = group_of(c + 1);
        hn = kardam_prev_load<S>(kd, c + 1, flatbits, live, 3 * g + e0, n_up, pn);
      }
      client(c, cur);
    }
  }
  for (; c + 1 < M; c += 2) {
    FLEET_CLIENT_HOOK(c, M);
    if constexpr (LADDER > 0) {
      if (c == (q1 & ~1)) __builtin_amdgcn_s_setprio(P1);
      if (c == (q2 & ~1)) __builtin_amdgcn_s_setprio(P2);
      if (c == (q3 & ~1)) __builtin_amdgcn_s_setprio(0);
    }
    b1 = group_of(c + 1);
    client(c, b0);
    if (c + 2 < M) b0 = group_of(c + 2);
    client(c + 1, b1);
  }
  if (c < M) client(c, b0);
  FLEET_CLIENT_HOOK(M, M);
  if (__ballot(dmax >= kD16Out) != 0) {  // left the q_gen domain: recompute exactly (never for gradients)
    if (dmax >= kD16Out && live) {
#pragma unroll
      for (int i = 0; i < S; ++i) acc[i] = chain_general(uploads, pitch, M, dampen, g, e0 + i, &tab);
    }
  }
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const int64_t pos = 3 * g + e0 + i;
    const bool keep_last = ((hbits >> i) & 1u) || pos >= walk_end;
    out[i] = (live && pos < n_up) ? merged_code(acc[i], inv_avg, codes[i], keep_last, &tab) : 0;
  }
}

// Block `bid` of the SIMD-balanced stream grid (tables already in LDS).
template <int NT, bool KD = false, int LADDER = 0, bool LD = false>
__device__ __forceinline__ void update_mixed_block(const B64Tables& tab, const D16Table& dtab, int64_t bid,
                                                   const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                                   const double* __restrict__ dampen, double inv_avg, int64_t n_up,
                                                   int64_t g_begin, int64_t g_end,
                                                   const int32_t* __restrict__ hdr_block, uint8_t* __restrict__ merged,
                                                   float* __restrict__ merged_f32, int* __restrict__ err, int nA,
                                                   const KardamOut& kd = KardamOut{},
                                                   const uint8_t* __restrict__ ld16 = nullptr) {
  uint32_t bad = 0, layout_bad = 0;
  // Kardam: this wave's partial slot of client 0; one slot per wave of the grid
  const size_t nw = (size_t)gridDim.x * (NT / 64);
  double* kd_part = KD ? kd.partials + 2 * ((size_t)bid * (NT / 64) + (threadIdx.x >> 6)) : nullptr;
  if (bid < nA) {  // block-uniform: one group per lane
    const int64_t g = g_begin + bid * NT + threadIdx.x;
    const bool live = g < g_end;
    int32_t out[3];
    update_lane<3, KD, LADDER, LD>(tab, dtab, uploads, pitch, M, dampen, inv_avg, n_up, g, 0, live, g_begin, hdr_block,
                                   out, bad, layout_bad, kd, kd_part, 2 * nw, ld16);
    if (!live) return;
    if (bad) atomicOr(err, FLEET_ERRBIT_BASE64);
    if (layout_bad) atomicOr(err, FLEET_ERRBIT_LAYOUT);
    const int r = (int)min<int64_t>(3, n_up - 3 * g);
    *reinterpret_cast<uint4*>(merged + 16 * g) = pad_group(b64_encode_group(out, &tab), r);
    if (merged_f32)
      for (int e = 0; e < r; ++e) merged_f32[3 * g + e] = dec_mt(out[e], tab.mt);
  } else {  // one value per lane, 21 groups per wave
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t g = g_begin + (int64_t)nA * NT + ((bid - nA) * (NT / 64) + wave) * 21 + lane / 3;
    const int e = lane % 3;
    const bool live = lane < 63 && g < g_end;
    int32_t out[1];
    update_lane<1, KD, LADDER, LD>(tab, dtab, uploads, pitch, M, dampen, inv_avg, n_up, g, e, live, g_begin, hdr_block,
                                   out, bad, layout_bad, kd, kd_part, 2 * nw, ld16);
    const int base = lane - e;  // the group's three lanes (lane 63 reads its own)
    const int32_t o0 = __shfl(out[0], base), o1 = __shfl(out[0], base + 1), o2 = __shfl(out[0], base + 2);
    if (!live) return;
    if (bad) atomicOr(err, FLEET_ERRBIT_BASE64);
    if (layout_bad) atomicOr(err, FLEET_ERRBIT_LAYOUT);
    const int r = (int)min<int64_t>(3, n_up - 3 * g);
    if (e == 0) {
      const int32_t o3[3] = {o0, r > 1 ? o1 : 0, r > 2 ? o2 : 0};
      *reinterpret_cast<uint4*>(merged + 16 * g) = pad_group(b64_encode_group(o3, &tab), r);
    }
    if (merged_f32 && e < r) merged_f32[3 * g + e] = dec_mt(out[0], tab.mt);
  }
}

// The stream update with balanced SIMDs. The plain stream grid has
// ceil(groups/64) waves, which leaves some SIMDs one wave more than others for
// the whole kernel (synth1m_256: 5,462 waves on 1,024 SIMDs -> 5 or 6 each). Here
// blocks [0, nA) run whole rounds of group-per-lane waves, and the remaining
// groups go to blocks of one value per lane (21 groups = 63 lanes per wave):
// three times the waves at a third of the work each, spread over every SIMD
// instead of a sixth full wave on some. nA = gridDim.x: the plain grid.
// KD = true adds Kardam's side outputs (kardam_lane_step; partial slots per wave).
// Both forms run the issue-priority ladder (update_lane: synth1m_256 828 -> 786 us
// plain, 1776 -> 1502-1546 us with Kardam's side outputs, r04 call a14);
// its register budget asks for at least 6 waves per SIMD (73 VGPRs, no scratch;
// unconstrained it takes 91 VGPRs: 5 waves, 1922 against 1795 us on synth1m_256; at 7
// or 8 waves it spills 16 / 64 B a lane and runs no faster, r04 call a24).
template <int NT, bool KD>
__global__ void __launch_bounds__(NT, KD ? 6 : 1) k_update_mixed(const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                                     const double* __restrict__ dampen, double inv_avg,
                                                     int64_t n_up, int64_t g_begin, int64_t g_end,
                                                     const int32_t* __restrict__ hdr_block,
                                                     uint8_t* __restrict__ merged, float* __restrict__ merged_f32,
                                                     int* __restrict__ err, int nA, KardamOut kd) {
  __shared__ B64Tables tab;
  __shared__ D16Table dtab;
  __shared__ LastDigitTable ldt;
  b64_tables_init<NT>(&tab);
  d16_table_init<NT>(&dtab);
  ld16_table_init<NT>(&ldt);
  __syncthreads();
  update_mixed_block<NT, KD, 3, true>(tab, dtab, blockIdx.x, uploads, pitch, M, dampen, inv_avg, n_up, g_begin, g_end,
                                      hdr_block, merged, merged_f32, err, nA, kd, ldt.ld16);
}

// D16: the tile also holds the byte-table digit counts (D16Table, 9 KB), and the
// epilogue assembles its merged codes in the tile's p buffer instead of outcodes.
template <bool D16>
struct TileD16 {};
template <>
struct TileD16<true> {
  D16Table dt;
};
template <int TG, int NW = 4, bool D16 = false>
struct TileShared : TileD16<D16> {
  static constexpr int E = 3 * TG;
  B64Tables tab;
  int32_t last_codes[E];            // codes of the last upload (mergeFlatGradient's g)
  int32_t hmin[E], hmax[E];         // header-slot codes over all uploads (layout check)
  uint32_t hmask[TG];               // bit e = slot 3*g+e is a header slot
  int32_t outcodes[D16 ? 1 : E];    // merged codes (epilogue)
};

// Tables, header slots of the tile (every thread checks one header position:
// one independent load each, not a per-group binary search), min/max init.
template <int TG, int NW, bool D16>
__device__ __forceinline__ void tile_init(TileShared<TG, NW, D16>& sh, const int32_t* __restrict__ hdr, int n_hdr,
                                          int64_t g0, int ng) {
  constexpr int E = 3 * TG;
  const int tid = threadIdx.x;
  const int64_t v0 = 3 * g0, v1 = 3 * (g0 + ng);
  int32_t hp = -1;
  if (tid < n_hdr) hp = hdr[tid];
  b64_tables_init<64 * NW>(&sh.tab);
  if constexpr (D16) d16_table_init<64 * NW>(&sh.dt);
  if (tid < TG) sh.hmask[tid] = 0u;
  if (tid < E) {
    sh.hmin[tid] = INT32_MAX;
    sh.hmax[tid] = INT32_MIN;
  }
  __syncthreads();
  for (int i = tid; i < n_hdr; i += 64 * NW) {
    if (i != tid) hp = hdr[i];
    if (hp >= v0 && hp < v1) atomicOr(&sh.hmask[(hp - v0) / 3], 1u << ((hp - v0) % 3));
  }
  __syncthreads();
}

// Client-independent part of the chain for IPT (client, group) items per
// thread: items it0 + h*stride (h < IPT) of the nitems items (client-major:
// item = cc*TG + gl) of clients c_base.. ; p of client c_base+cc, slot 3*gl+e
// goes to pdst[cc*E + 3*gl + e]:
//   p = Q(f32(f64(Q(int2float(code))) * d_c))   (CppNNUpdater.java:463-464)
// Also: Base64 validity, the last upload's codes, header-slot min/max.
// Split in two so a producer can issue the next pass's loads (tile_load)
// before computing the current one (tile_compute).
template <int TG, int IPT>
struct TileItems {
  uint4 w[IPT];
  int cc[IPT], gl[IPT], c_base;
  bool live[IPT];
  int cl[IPT];       // the item's client in the pass, also for dead groups past the tile's last
  bool cvalid[IPT];  // the item's client exists (item < nitems)
};

template <int TG, int IPT>
__device__ __forceinline__ void tile_load(TileItems<TG, IPT>& it, const uint8_t* __restrict__ uploads, size_t pitch,
                                          int64_t g0, int ng, int c_base, int nitems, int it0, int stride) {
  it.c_base = c_base;
#pragma unroll
  for (int h = 0; h < IPT; ++h) {
    const int item = it0 + h * stride;
    it.cvalid[h] = item < nitems;
    it.cl[h] = item / TG;
    it.live[h] = item < nitems && (item % TG) < ng;
    it.cc[h] = it.live[h] ? item / TG : 0;
    it.gl[h] = it.live[h] ? item % TG : 0;
    it.w[h] = *reinterpret_cast<const uint4*>(uploads + (size_t)(c_base + it.cc[h]) * pitch + 16 * (g0 + it.gl[h]));
  }
}

// Kardam's side outputs in a tile producer (CppNNUpdater.java:463-481,
// Kardam.java:48-106): the tile's index among the grid's tiles (partials slot) and
// the end of network::flatGrad's walk (slots past it are not gradient values).
struct TileKd {
  KardamOut kd;
  int64_t tile, ntiles, walk_end;
};

// Per item (one client, one group): the text Kardam.setGrad stores, G =
// Q(f32(f64(p) * lr)), written to g_out; ||G||^2 and, with the worker's previous
// G, ||Q(G - prev)||^2 over the flat gradient's slots (getNorm: float products
// summed in double). A client's W groups of the tile are W consecutive lanes of
// one wave (items are client-major, W in {16, 32, 64} and waves start at multiples of
// 64), so the lane group's sums are the (client, tile) partial: one write per sum, no
// atomics, a fixed order (k_kardam_reduce then sums the tiles in order). Item h: client c[h]
// and group gl[h] (live[h]: a real item), partial slot client cp[h] (cvalid[h]: that
// client exists -- dead groups of a live client still write their lane group's zeros).
template <int IPT, int NW, int TGS, bool D16>
__device__ __forceinline__ void kardam_items(TileShared<TGS, NW, D16>& sh, const int (&c)[IPT], const int (&gl)[IPT],
                                             const bool (&live)[IPT], const int (&cp)[IPT], const bool (&cvalid)[IPT],
                                             const float (&p)[3 * IPT], int W, int64_t n_up, int64_t g0,
                                             const TileKd& tk) {
  constexpr int S = 3 * IPT;
  const KardamOut& kd = tk.kd;
  float rg[S], G[S];
#pragma unroll
  for (int i = 0; i < S; ++i) rg[i] = p[i];
  dampen_stage<S>(rg, kd.lr);  // (float)((double)p * lr), lr uniform
  if constexpr (D16) q_stage_d16x<S>(G, rg, &sh.dt, sh.tab.var);  // exact (in-stage fallback)
  else q_stage<S>(G, rg, &sh.tab);
  // per item: the flat slots, ||G||^2, prev and G - prev, the G row out; then one D stage
  // for all the lane's items (one ballot / fix-up pass, not one per item)
  typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));
  double sg[IPT], sd[IPT];
  float dv[S], D[S];
  uint32_t flat = 0, hasps = 0;
#pragma unroll
  for (int h = 0; h < IPT; ++h) {
    const int64_t gp = 3 * (g0 + gl[h]);
    const uint32_t hm = live[h] ? sh.hmask[gl[h]] : 7u;
    const bool hasp = kd.prev && live[h] && kd.has_prev[c[h]];
    hasps |= (uint32_t)hasp << h;
    sg[h] = 0.0;
    // prev / G rows: one 12-byte access per whole group (rows are 4-byte aligned)
    const bool whole = live[h] && gp + 2 < n_up;
    float pv[3] = {0.0f, 0.0f, 0.0f};
    if (hasp && whole) {
      const f3u t = *reinterpret_cast<const f3u*>(kd.prev + (size_t)c[h] * kd.vpitch + gp);
      pv[0] = t.x;
      pv[1] = t.y;
      pv[2] = t.z;
    }
    float gv[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const int64_t pos = gp + e;
      const bool f = live[h] && !((hm >> e) & 1u) && pos < n_up && pos < tk.walk_end;
      flat |= (uint32_t)f << (3 * h + e);
      const float g = G[3 * h + e];
      if (f) sg[h] += (double)(g * g);
      if (hasp && !whole && f) pv[e] = kd.prev[(size_t)c[h] * kd.vpitch + pos];
      dv[3 * h + e] = (f && hasp) ? g - pv[e] : 0.0f;
      gv[e] = f ? g : 0.0f;
    }
    if (kd.g_out) {
      float* go = kd.g_out + (size_t)c[h] * kd.vpitch + gp;
      if (whole) {
        *reinterpret_cast<f3u*>(go) = f3u{gv[0], gv[1], gv[2]};
      } else {
#pragma unroll
        for (int e = 0; e < 3; ++e)
          if (live[h] && gp + e < n_up) go[e] = gv[e];
      }
    }
  }
  if constexpr (D16) q_stage_d16x<S>(D, dv, &sh.dt, sh.tab.var);
  else q_stage<S>(D, dv, &sh.tab);
#pragma unroll
  for (int h = 0; h < IPT; ++h) {
    sd[h] = 0.0;
#pragma unroll
    for (int e = 0; e < 3; ++e)
      if (((flat >> (3 * h + e)) & 1u) && ((hasps >> h) & 1u)) sd[h] += (double)(D[3 * h + e] * D[3 * h + e]);
    // the client's tile sums (W is block-uniform: one branch per item): sg in the lane
    // group's middle lane, sd in its last
    const int l = threadIdx.x & (W - 1);
    const size_t slot = ((size_t)cp[h] * tk.ntiles + tk.tile) * 2;
    // sc1: the pipelined form's reduce blocks read them in the same launch
    double s;
    if (W == 64) s = pair_sum_f64<64>(sg[h], sd[h]);
    else if (W == 32) s = pair_sum_f64<32>(sg[h], sd[h]);
    else s = pair_sum_f64<16>(sg[h], sd[h]);
    if (cvalid[h] && (l == W - 1 || l == W / 2 - 1))
      __hip_atomic_store(kd.partials + slot + (l == W - 1), s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// kardam_items over a tile producer's TileItems (the classic and pipelined tiles)
template <int TG, int IPT, int NW, bool D16>
__device__ __forceinline__ void tile_kardam(TileShared<TG, NW, D16>& sh, const TileItems<TG, IPT>& it,
                                            const float (&p)[3 * IPT], int64_t n_up, int64_t g0, const TileKd& tk) {
  static_assert(64 % TG == 0 && TG >= 16, "a client's groups in one lane group of 16, 32 or 64");
  int c[IPT], cp[IPT];
#pragma unroll
  for (int h = 0; h < IPT; ++h) {
    c[h] = it.c_base + it.cc[h];
    cp[h] = it.c_base + it.cl[h];
  }
  kardam_items<IPT, NW>(sh, c, it.gl, it.live, cp, it.cvalid, p, TG, n_up, g0, tk);
}

template <int TG, int IPT, int NW, bool KD = false, bool D16 = false>
__device__ __forceinline__ void tile_compute(TileShared<TG, NW, D16>& sh, const TileItems<TG, IPT>& it, int M,
                                             const double* __restrict__ dampen, int64_t n_up, int64_t walk_end,
                                             int64_t g0, float* __restrict__ pdst, uint32_t& badacc,
                                             const TileKd& tk = TileKd{}) {
  constexpr int E = 3 * TG, S = 3 * IPT;
  int32_t codes[S];
#pragma unroll
  for (int h = 0; h < IPT; ++h) {
    const int r = (int)min<int64_t>(3, max<int64_t>(0, n_up - 3 * (g0 + it.gl[h])));
    uint32_t b;
    if (r == 3)
      b = b64_decode_group_full(it.w[h], &sh.tab, codes + 3 * h);
    else
      b = b64_decode_group(it.w[h], &sh.tab, codes + 3 * h) & needed_chars_mask(r);
    if (it.live[h]) {
      badacc |= b;
      if (it.c_base + it.cc[h] == M - 1)
        for (int e = 0; e < 3; ++e) sh.last_codes[3 * it.gl[h] + e] = codes[3 * h + e];
      const uint32_t hm = sh.hmask[it.gl[h]];
      if (hm) {  // header slots (rare lanes): the layout check, then the chain runs on code 0 (keep_bits)
        for (int e = 0; e < 3; ++e)
          if ((hm >> e) & 1u) {
            atomicMin(&sh.hmin[3 * it.gl[h] + e], codes[3 * h + e]);
            atomicMax(&sh.hmax[3 * it.gl[h] + e], codes[3 * h + e]);
            codes[3 * h + e] = 0;
          }
      }
    }
  }
  if (3 * (g0 + TG) > walk_end) {  // block-uniform, rare: slots past the walk run on code 0 too
#pragma unroll
    for (int h = 0; h < IPT; ++h)
#pragma unroll
      for (int e = 0; e < 3; ++e)
        if (3 * (g0 + it.gl[h]) + e >= walk_end) codes[3 * h + e] = 0;
  }
  // stage A: y = Q(int2float(code)); D16: the stream kernel's byte-table stages
  float y0[S], y[S];
  if constexpr (D16) dec_stage_d16<S>(y0, codes, &sh.dt);
  else dec_stage<S>(y0, codes, &sh.tab);
  if constexpr (D16) q_stage_d16x<S>(y, y0, &sh.dt, sh.tab.var);
  else q_stage<S>(y, y0, &sh.tab);
  // stage B: p = Q(f32(f64(y) * d)), per-item client
  float r[S], p[S];
#pragma unroll
  for (int h = 0; h < IPT; ++h) {
    if constexpr (TG % 64 == 0) {
      // a wave's 64 items are 64 groups of one client (items are client-major and
      // every wave starts at a multiple of 64): d is wave-uniform, so the scalar
      // test of dampen_stage applies (a dead lane 0 means a dead wave)
      float t[3] = {y[3 * h], y[3 * h + 1], y[3 * h + 2]};
      dampen_stage<3>(t, dampen[__builtin_amdgcn_readfirstlane(it.c_base + it.cc[h])]);
#pragma unroll
      for (int e = 0; e < 3; ++e) r[3 * h + e] = t[e];
    } else {
      const double d = dampen[it.c_base + it.cc[h]];
#pragma unroll
      for (int e = 0; e < 3; ++e) r[3 * h + e] = (float)((double)y[3 * h + e] * d);
    }
  }
  if constexpr (D16) q_stage_d16x<S>(p, r, &sh.dt, sh.tab.var);
  else q_stage<S>(p, r, &sh.tab);
#pragma unroll
  for (int h = 0; h < IPT; ++h)
    if (it.live[h])
#pragma unroll
      for (int e = 0; e < 3; ++e) pdst[it.cc[h] * E + 3 * it.gl[h] + e] = p[3 * h + e];
  if constexpr (KD) tile_kardam<TG, IPT, NW>(sh, it, p, n_up, g0, tk);
}

template <int TG, int IPT, int NW, bool KD = false, bool D16 = false>
__device__ __forceinline__ void tile_produce(TileShared<TG, NW, D16>& sh, const uint8_t* __restrict__ uploads, size_t pitch,
                                             int M, const double* __restrict__ dampen, int64_t n_up, int64_t walk_end,
                                             int64_t g0, int ng, int c_base, int nitems, int it0, int stride,
                                             float* __restrict__ pdst, uint32_t& badacc, const TileKd& tk) {
  TileItems<TG, IPT> it;
  tile_load<TG, IPT>(it, uploads, pitch, g0, ng, c_base, nitems, it0, stride);
  tile_compute<TG, IPT, NW, KD>(sh, it, M, dampen, n_up, walk_end, g0, pdst, badacc, tk);
}

// Final values of the tile (vals[0..E)) -> merged Base64 (+ fp32), layout
// check. One thread per value computes its merged code (the longest part),
// then one thread per group assembles the 16 Base64 chars. Call from every
// thread of the block (contains a barrier).
// D16: `outc` (E ints, not overlapping vals) takes the merged codes.
template <int TG, int NW, bool D16>
__device__ __forceinline__ void tile_epilogue(TileShared<TG, NW, D16>& sh, const float* __restrict__ vals,
                                              double inv_avg, int64_t n_up, int64_t walk_end, int64_t g0, int ng,
                                              uint8_t* __restrict__ merged, float* __restrict__ merged_f32,
                                              int* __restrict__ err, int32_t* outc = nullptr) {  // outc: E ints of LDS, D16 only
  const int tid = threadIdx.x;
  int32_t* oc;
  if constexpr (D16) oc = outc;
  else oc = sh.outcodes;
  if (tid < 3 * ng) {
    const int gl = tid / 3, e = tid % 3;
    const int64_t p = 3 * g0 + tid;
    int32_t o = 0;
    if (p < n_up) {
      const bool hdr = (sh.hmask[gl] >> e) & 1u;
      if (hdr && sh.hmin[tid] != sh.hmax[tid]) atomicOr(err, FLEET_ERRBIT_LAYOUT);
      o = merged_code(vals[tid], inv_avg, sh.last_codes[tid], hdr || p >= walk_end, &sh.tab);
      if (merged_f32) merged_f32[p] = dec_mt(o, sh.tab.mt);
    }
    oc[tid] = o;
  }
  __syncthreads();
  if (tid < ng) {
    const int64_t g = g0 + tid;
    const int r = (int)min<int64_t>(3, n_up - 3 * g);
    const int32_t out[3] = {oc[3 * tid], oc[3 * tid + 1], oc[3 * tid + 2]};
    *reinterpret_cast<uint4*>(merged + 16 * g) = pad_group(b64_encode_group(out, &sh.tab), r);
  }
}

// Two-phase tile variant for small/medium buckets (MNIST: 7,654 groups -- too
// few lanes to fill 1,024 SIMDs when every lane walks all clients serially).
// A block owns TG groups (E = 3*TG values) and walks the clients in chunks
// of CM:
//   phase 1 -- all 256 threads: p[c][e] for every (client, group) item of the
//              chunk into LDS (tile_produce; independent across clients).
//   phase 2 -- one thread per value: the serial A = Q(A + p_c)
//              (CppNNUpdater.java:490-493), the only part that must follow
//              client order, as straight-line q_lat steps (no per-step
//              branch); a lane that ever leaves the q_lat domain is recomputed
//              by chain_general.
// Layout consistency (all uploads carry the last one's header codes) is
// checked in phase 1 with per-slot LDS min/max of the header codes.
#ifndef FLEET_TILED_PT
#define FLEET_TILED_PT 3072
#endif
// p floats per chunk: 12 KiB (CM = 16 clients at TG = 64, so a chunk is two full
// 512-item passes); with the tables the block fits 7 per CU (measured: 24 KiB
// chunks 0.40 ms, 12 KiB 0.37, 8 KiB 0.50, 16 KiB 0.43 on cifar10_256)
// D16 tiles: 6 KiB (CM = 8 at TG = 64: one full 512-item pass per chunk), so the
// byte table fits with 7 blocks per CU (22.6 KB per block)
#ifndef FLEET_TILED_PT_D16
#define FLEET_TILED_PT_D16 1536
#endif
template <int TG, bool D16 = false>
constexpr int tiled_chunk_clients() { return TG > 0 ? (D16 ? FLEET_TILED_PT_D16 : FLEET_TILED_PT) / (3 * TG) : 0; }

// Tile `bid` of k_update_tiled (LDS state in sh / ptile)
template <int TG, bool KD = false, bool D16 = false>
__device__ __forceinline__ void update_tiled_block(TileShared<TG, 4, D16>& sh, float* ptile, int64_t bid,
                                                   const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                                   const double* __restrict__ dampen, double inv_avg, int64_t n_up,
                                                   int64_t g_begin, int64_t g_end,
                                                   const int32_t* __restrict__ hdr_block, uint8_t* __restrict__ merged,
                                                   float* __restrict__ merged_f32, int* __restrict__ err,
                                                   const TileKd& tk = TileKd{}) {
  constexpr int E = 3 * TG;
  static_assert(E <= 256, "phase 2 is one thread per value");
  constexpr int CM = tiled_chunk_clients<TG, D16>();
  static_assert(CM >= 2, "the epilogue's codes go after the E final values in ptile");
  FLEET_TSTAMP(0);
  const int tid = threadIdx.x;
  const int64_t g0 = g_begin + bid * TG;
  const int ng = (int)min<int64_t>(TG, g_end - g0);
  tile_init(sh, hdr_block + 4, hdr_block[1], g0, ng);
  FLEET_TSTAMP(1);

  float A = 0.f;  // phase-2 value: element tid of the tile (tid < E)
  uint32_t off_domain = 0;
  float amax = 0.f;  // narrow tiles: max |A + p| (q_lat is exact below 1e8 for any sign)
  uint32_t badacc = 0;
  // Issue-priority ladder over the client loop (3 -> 0 at quarters of it), as in the
  // stream kernel: a CU's tiles are all resident at once and the oldest win issue
  // arbitration, so without it they finished one by one -- on cifar10_256 the tiles of
  // one CU ended 118 us apart on a 245 us mean span, the last ones running alone in a
  // latency-bound tail (r05 residency trace, scripts/bt_analyze.py). A tile that gets
  // ahead yields, the lagging ones catch up.
  const int nch = (M + CM - 1) / CM;
  const int r1 = nch / 4, r2 = nch / 2, r3 = 3 * nch / 4;
  if (FLEET_TILE_LADDER) __builtin_amdgcn_s_setprio(3);
  for (int c0 = 0; c0 < M; c0 += CM) {
    const int cm = min(CM, M - c0);
    const int nitems = cm * TG;
    FLEET_WTRACE(bid, c0 / CM, 0);
    if (FLEET_TILE_LADDER) {
      const int k = c0 / CM;
      if (k == r1) __builtin_amdgcn_s_setprio(2);
      if (k == r2) __builtin_amdgcn_s_setprio(1);
      if (k == r3) __builtin_amdgcn_s_setprio(0);
    }
    for (int base = 0; base < nitems; base += 512) {
      tile_produce<TG, 2, 4, KD>(sh, uploads, pitch, M, dampen, n_up, hdr_block[2], g0, ng, c0, nitems, base + tid,
                                 256, ptile, badacc, tk);
      if (base == 0) FLEET_TSTAMP(2);
    }
    FLEET_WTRACE(bid, c0 / CM, 1);
    __syncthreads();
    FLEET_WTRACE(bid, c0 / CM, 2);
    FLEET_TSTAMP(3);
    // phase 2: serial accumulation, one value per thread
    if (tid < E) {
      int k = 0;
      if (c0 == 0) {
        A = ptile[tid];
        k = 1;
      }
      if (TG <= 16) {  // few blocks: the serial chain is the critical path (select-chain Q)
#pragma unroll 4
        for (; k < cm; ++k) {
          const float s = A + ptile[k * E + tid];
          amax = __builtin_fmaxf(amax, __builtin_fabsf(s));
          A = q_lat(s);
        }
      } else {  // many blocks: throughput (multiplier-table Q, fewer instructions)
#pragma unroll 2
        for (; k < cm; ++k) {
          const float s = A + ptile[k * E + tid];
          if constexpr (D16) {  // the stream kernel's stage C (var_d16: branch-free)
            const uint32_t e = var_d16(f2u(s), sh.tab.var);
            off_domain |= (uint32_t)(e >= kD16Out);
            A = q_d16(s, e, &sh.dt.st);
          } else {
            const uint32_t d = var_digits(s, sh.tab.var);
            off_domain |= (uint32_t)(d > 9u);
            A = q_mt_d(s, d, sh.tab.mt);
          }
        }
      }
    }
    FLEET_WTRACE(bid, c0 / CM, 3);
    __syncthreads();
  }
  FLEET_TSTAMP(4);
  if (badacc) atomicOr(err, FLEET_ERRBIT_BASE64);
  off_domain |= (uint32_t)!(amax < 1e8f);
  if (tid >= 3 * ng) off_domain = 0;  // columns past the last group hold no values
  if (__ballot(off_domain != 0)) {    // wave-uniform, never for gradients
    if (off_domain) A = chain_general(uploads, pitch, M, dampen, g0 + tid / 3, tid % 3, &sh.tab);
  }
  if (tid < E) ptile[tid] = A;
  __syncthreads();
  tile_epilogue(sh, ptile, inv_avg, n_up, hdr_block[2], g0, ng, merged, merged_f32, err,
                D16 ? reinterpret_cast<int32_t*>(ptile + E) : nullptr);
  FLEET_TSTAMP(5);
}

// XCD-aware tile order: the dispatcher deals workgroups to the 8 XCDs round robin
// (b % 8; placement is unspecified, so this is for speed only, never correctness).
// Tiles of neighbouring column ranges share the 128-byte lines their 1 KiB row
// segments straddle (rows are only 16-byte aligned); dealt round robin, those
// lines were fetched once per XCD's L2 (PMC traffic 1.11x the algorithmic bytes
// on cifar10_256). Here XCD x runs one contiguous run of tiles instead.
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t nb) {
  if (nb < 16) return b;
  const int64_t q = nb / 8, r = nb % 8, x = b % 8, i = b / 8;
  return x * q + (x < r ? x : r) + i;
}

// ----------------------------------------------------------------------------
// Flat tiles (r05): k_update_tiled's two phases with the tile width W a runtime
// value (up to 64 groups; the planner uses 64, 32 and 16), so one launch deals the
// groups out as ONE round over the CUs' block slots: whole rounds of 64-group tiles,
// then the rest in tiles of the width that leaves the most loaded CU the least work.
// cifar10_256 (104,623 groups, 256 CUs, 7 slots per CU): 1,536 64-group tiles + 198
// 32-group tiles, at most 6 x 64 + 32 = 416 groups on a CU, where the one-width grid
// put 7 x 64 = 448 on most CUs and the compile-time two-width grid (two inlined tile
// bodies: 106 SGPRs, 6 blocks per CU) ran its 16-group tiles as a second round --
// either way the kernel took as long as its most loaded CU (317-320 us against a
// 252 us first round, r05 residency traces). One tile body (92 SGPRs, 22.6 KB of
// LDS): 7 blocks per CU. A tile's (client, group) items are client-major over its W
// groups, 512 per pass (two per thread): floor(512 / W) whole clients per pass, so
// phase 2 is k_update_tiled's.
// The widest flat tile: E = 192 values, one per phase-2 thread. 85-group tiles (six
// whole clients per pass, a fourth phase-2 wave, 23.4 KB of LDS: 6 blocks per CU) were
// slower everywhere: cifar10_256 update 275.5 against 268.4 us, the N = 4 window 250.3
// against 230.6 (r05, profiles/r05/ab_flat_width85.txt).
constexpr int kFlatTG = 64;
constexpr int kFlatPass = 512;  // items per pass
constexpr int kFlatSlots = 7;   // blocks per CU (LDS 22.6 KB, 92 SGPRs; r05 residency traces)

// scalarMultiply(getDampen) for a lane's own client (dampen_stage with a per-lane d: a
// narrow tile's wave spans 64 / W clients): the binary32 multiply when every lane's d is
// a binary32 value (wave-uniform branch), the f64 product otherwise; both exact.
__device__ __forceinline__ void dampen_lane3(float (&r)[3], double d) {
  const uint64_t b = __builtin_bit_cast(uint64_t, d);
  const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
  const uint32_t ex = (hi >> 20) & 0x7ffu;
  const bool f32ok = (lo & 0x1fffffffu) == 0 && ex - 897u < 254u;
  if (__ballot(!f32ok) == 0) {
    const float df = u2f((hi & 0x80000000u) | ((ex - 896u) << 23) | ((hi & 0xfffffu) << 3) | (lo >> 29));
#pragma unroll
    for (int i = 0; i < 3; ++i) r[i] = r[i] * df;
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i) r[i] = (float)((double)r[i] * d);
  }
}

// One pass's items of a thread: items tid and tid + 256 of the pass (client c, group gl)
struct FlatItems {
  uint4 w[2];
  int c[2], gl[2];
  bool live[2];
  bool cvalid[2];  // the item's client exists (its group may be past the tile's last)
};

// p of the thread's two items -> pbuf[item * 3 + e]: tile_compute's stages
// (CppNNUpdater.java:463-464). W = 64: a wave's items are one client (wave-uniform d).
// KD: Kardam's side outputs with p (kardam_items; W in {16, 32, 64}).
template <bool KD = false>
__device__ __forceinline__ void flat_compute(TileShared<kFlatTG, 4, true>& sh, const FlatItems& it, int M,
                                             const double* __restrict__ dampen, int64_t n_up, int64_t walk_end,
                                             int64_t g0, int ng, int W, float* __restrict__ pbuf, int tid,
                                             uint32_t& badacc, const TileKd& tk) {
  const bool W64 = W == 64;
  int32_t codes[6];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = (int)min<int64_t>(3, max<int64_t>(0, n_up - 3 * (g0 + it.gl[h])));
    uint32_t b;
    if (r == 3) b = b64_decode_group_full(it.w[h], &sh.tab, codes + 3 * h);
    else b = b64_decode_group(it.w[h], &sh.tab, codes + 3 * h) & needed_chars_mask(r);
    if (it.live[h]) {
      badacc |= b;
      if (it.c[h] == M - 1)
        for (int e = 0; e < 3; ++e) sh.last_codes[3 * it.gl[h] + e] = codes[3 * h + e];
      const uint32_t hm = sh.hmask[it.gl[h]];
      if (hm) {  // header slots (rare lanes): the layout check, then the chain runs on code 0 (keep_bits)
        for (int e = 0; e < 3; ++e)
          if ((hm >> e) & 1u) {
            atomicMin(&sh.hmin[3 * it.gl[h] + e], codes[3 * h + e]);
            atomicMax(&sh.hmax[3 * it.gl[h] + e], codes[3 * h + e]);
            codes[3 * h + e] = 0;
          }
      }
    }
  }
  if (3 * (g0 + ng) > walk_end) {  // block-uniform, rare: slots past the walk run on code 0 too
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 3; ++e)
        if (3 * (g0 + it.gl[h]) + e >= walk_end) codes[3 * h + e] = 0;
  }
  float y0[6], y[6], r[6], p[6];
  dec_stage_d16<6>(y0, codes, &sh.dt);
  q_stage_d16x<6>(y, y0, &sh.dt, sh.tab.var);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float t[3] = {y[3 * h], y[3 * h + 1], y[3 * h + 2]};
    if (W64) dampen_stage<3>(t, dampen[__builtin_amdgcn_readfirstlane(it.c[h])]);  // block-uniform branch
    else dampen_lane3(t, dampen[it.c[h]]);
#pragma unroll
    for (int e = 0; e < 3; ++e) r[3 * h + e] = t[e];
  }
  q_stage_d16x<6>(p, r, &sh.dt, sh.tab.var);
#pragma unroll
  for (int h = 0; h < 2; ++h)
    if (it.live[h])
#pragma unroll
      for (int e = 0; e < 3; ++e) pbuf[(tid + 256 * h) * 3 + e] = p[3 * h + e];
  if constexpr (KD) kardam_items<2, 4>(sh, it.c, it.gl, it.live, it.c, it.cvalid, p, W, n_up, g0, tk);
}

// Flat tile: groups [g0, g0 + ng) on the item mapping of width W (ng <= W <= kFlatTG;
// a pass holds 512 / W whole clients), pbuf = kFlatPass * 3 floats; `tile` its index
// (Kardam's partial slot; dev traces). KD: Kardam's side outputs (flat_compute).
template <bool KD = false>
__device__ __forceinline__ void update_flat_block(TileShared<kFlatTG, 4, true>& sh, float* pbuf, int64_t tile,
                                                  int64_t g0, int ng, int W, const uint8_t* __restrict__ uploads,
                                                  size_t pitch, int M, const double* __restrict__ dampen,
                                                  double inv_avg, int64_t n_up, const int32_t* __restrict__ hdr_block,
                                                  uint8_t* __restrict__ merged, float* __restrict__ merged_f32,
                                                  int* __restrict__ err, const TileKd& tk = TileKd{}) {
  static_assert(3 * kFlatTG <= 256 && 2 * 3 * kFlatTG <= 3 * kFlatPass, "phase 2 / epilogue fit the block / pbuf");
  const int tid = threadIdx.x;
  const int E = 3 * W;
  const int cpp = kFlatPass / W;  // whole clients per pass (items past cpp * W idle)
  const int64_t walk_end = hdr_block[2];
  tile_init(sh, hdr_block + 4, hdr_block[1], g0, ng);
  float A = 0.f;  // phase-2 value: element tid of the tile (tid < E)
  uint32_t off_domain = 0, badacc = 0;
  // the thread's items: (client offset, group), the same in every pass
  int icl[2], igl[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    icl[h] = (tid + 256 * h) / W;
    igl[h] = (tid + 256 * h) % W;
  }
  // the issue-priority ladder of update_tiled_block (3 -> 0 at quarters of the passes)
  const int npass = (M + cpp - 1) / cpp;
  const int r1 = npass / 4, r2 = npass / 2, r3 = 3 * npass / 4;
  if (FLEET_TILE_LADDER) __builtin_amdgcn_s_setprio(3);
  for (int k = 0; k < npass; ++k) {
    if (FLEET_TILE_LADDER) {
      if (k == r1) __builtin_amdgcn_s_setprio(2);
      if (k == r2) __builtin_amdgcn_s_setprio(1);
      if (k == r3) __builtin_amdgcn_s_setprio(0);
    }
    const int c0 = k * cpp, cm = min(cpp, M - c0);
    FLEET_WTRACE(tile, k, 0);
    FlatItems it;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      it.live[h] = icl[h] < cm && igl[h] < ng;
      it.cvalid[h] = icl[h] < cm;
      it.c[h] = c0 + (icl[h] < cm ? icl[h] : 0);
      it.gl[h] = it.live[h] ? igl[h] : 0;
      it.w[h] = *reinterpret_cast<const uint4*>(uploads + (size_t)it.c[h] * pitch + 16 * (g0 + it.gl[h]));
    }
    if (__ballot(it.live[0]) != 0)  // wave-uniform: only a last pass or a ragged tile has dead waves
      flat_compute<KD>(sh, it, M, dampen, n_up, walk_end, g0, ng, W, pbuf, tid, badacc, tk);
    FLEET_WTRACE(tile, k, 1);
    __syncthreads();
    FLEET_WTRACE(tile, k, 2);
    // phase 2: serial accumulation, one value per thread (k_update_tiled's stage C)
    if (tid < E) {
      int j = 0;
      if (c0 == 0) {
        A = pbuf[tid];
        j = 1;
      }
#pragma unroll 2
      for (; j < cm; ++j) {
        const float s = A + pbuf[j * E + tid];
        const uint32_t e = var_d16(f2u(s), sh.tab.var);
        off_domain |= (uint32_t)(e >= kD16Out);
        A = q_d16(s, e, &sh.dt.st);
      }
    }
    FLEET_WTRACE(tile, k, 3);
    __syncthreads();
  }
  if (badacc) atomicOr(err, FLEET_ERRBIT_BASE64);
  if (tid >= 3 * ng) off_domain = 0;  // columns past the last group hold no values
  if (__ballot(off_domain != 0)) {    // wave-uniform, never for gradients
    if (off_domain) A = chain_general(uploads, pitch, M, dampen, g0 + tid / 3, tid % 3, &sh.tab);
  }
  if (tid < E) pbuf[tid] = A;
  __syncthreads();
  tile_epilogue(sh, pbuf, inv_avg, n_up, walk_end, g0, ng, merged, merged_f32, err,
                reinterpret_cast<int32_t*>(pbuf + 3 * kFlatTG));
}

// The grid of k_update_flat: blocks [0, nW) are tiles of w1 groups, [nW, nU) tiles of
// w2 groups (the last one ragged), each run in XCD-aware order (xcd_tile).
struct FlatGrid {
  int nW, nU, w1, w2;
};
__device__ __forceinline__ void flat_tile_range(int64_t b, const FlatGrid& fg, int64_t g_begin, int64_t g_end,
                                                int64_t* g0, int* ng, int* w) {
  if (b < fg.nW) {
    *g0 = g_begin + fg.w1 * xcd_tile(b, fg.nW);
    *w = fg.w1;
  } else {
    *g0 = g_begin + fg.w1 * (int64_t)fg.nW + fg.w2 * xcd_tile(b - fg.nW, fg.nU - fg.nW);
    *w = fg.w2;
  }
  *ng = (int)min<int64_t>(*w, g_end - *g0);
}

// ----------------------------------------------------------------------------
// Woven tiles (r05): the two phases of k_update_tiled in ONE barrier interval and
// in the same instruction stream. A block of NW waves owns 64 groups (E = 192
// values) and walks the clients in chunks of NW: wave w produces client c0 + w's
// p for the tile's 64 groups (one group per lane, so the dampening factor is
// wave-uniform), while three consumer waves run the serial A = Q(A + p) of the
// PREVIOUS chunk, one value per lane, from the other half of a double-buffered p
// chunk. The serial steps sit between the producer's stages in the source, so
// they share basic blocks with independent work and the scheduler fills their
// dependent latency (k_update_tiled's phase 2 ran one dependent chain per wave
// between two barriers: 2.95 cycles per VALU instruction against the stream
// kernel's 2.42, profiles/r04/sq.json). One barrier per chunk instead of two; the
// next chunk's group is loaded one chunk ahead. NW = 4: the block's fourth wave
// only produces, and which wave that is rotates with the tile (every SIMD of a CU
// carries the same share of serial work).
constexpr int kWeaveTG = 64, kWeaveE = 3 * kWeaveTG;

template <int NW>
struct WeaveShared {
  TileShared<kWeaveTG, NW, true> t;
  float p[2][NW * kWeaveE];  // double-buffered p chunk: client j of the chunk at [j * E + value]
};

// The consumer's serial step A = Q(A + p) (the stream kernel's stage C, var_d16: branch
// free); FIRST: the chain's first client, A = p.
template <bool FIRST>
__device__ __forceinline__ void weave_step(float& A, float p, const D16Table& dt, const VarEntry* vt, uint32_t& emax) {
  if constexpr (FIRST) {
    A = p;
  } else {
    const float s = A + p;
    const uint32_t e = var_d16(f2u(s), vt);
    emax = max(emax, e);
    A = q_d16(s, e, &dt.st);
  }
}

// One producer lane's item: client c (wave-uniform), group g0 + gl of the tile, its
// 16 chars `w` already loaded -> the three p of the item, with the consumer's steps
// of the previous chunk (CS of them, from `pc`, column `col`) woven between the stages.
// CS = 0: produce only. FIRST: the consumed chunk is the chain's first.
template <int NW, int CS, bool FIRST>
__device__ __forceinline__ void weave_item(WeaveShared<NW>& sh, uint4 w, bool live, int c, int gl, int M,
                                           const double* __restrict__ dampen, int64_t n_up, int64_t walk_end,
                                           int64_t g0, float* __restrict__ pdst, uint32_t& badacc, float& A,
                                           const float* __restrict__ pc, int col, uint32_t& emax) {
  TileShared<kWeaveTG, NW, true>& t = sh.t;
  float pp[CS > 0 ? CS : 1];
#pragma unroll
  for (int j = 0; j < CS; ++j) pp[j] = pc[j * kWeaveE + col];  // the consumed chunk's p: loads in flight early
  int32_t codes[3];
  const int64_t gp = 3 * (g0 + gl);
  const int r = (int)min<int64_t>(3, max<int64_t>(0, n_up - gp));
  uint32_t b;
  if (r == 3) b = b64_decode_group_full(w, &t.tab, codes);
  else b = b64_decode_group(w, &t.tab, codes) & needed_chars_mask(r);
  if (live) {
    badacc |= b;
    if (c == M - 1)
#pragma unroll
      for (int e = 0; e < 3; ++e) t.last_codes[3 * gl + e] = codes[e];
    const uint32_t hm = t.hmask[gl];
    if (hm) {  // header slots (rare lanes): the layout check, then the chain runs on code 0 (keep_bits)
#pragma unroll
      for (int e = 0; e < 3; ++e)
        if ((hm >> e) & 1u) {
          atomicMin(&t.hmin[3 * gl + e], codes[e]);
          atomicMax(&t.hmax[3 * gl + e], codes[e]);
          codes[e] = 0;
        }
    }
  }
  if (gp + 3 > walk_end) {  // rare: slots past network::flatGrad's walk run on code 0 too
#pragma unroll
    for (int e = 0; e < 3; ++e)
      if (gp + e >= walk_end) codes[e] = 0;
  }
  // stage A: y = Q(int2float(code))
  float y0[3], y[3];
  dec_stage_d16<3>(y0, codes, &t.dt);
  if constexpr (CS > 0) weave_step<FIRST>(A, pp[0], t.dt, t.tab.var, emax);
  q_stage_d16x<3>(y, y0, &t.dt, t.tab.var);
  if constexpr (CS > 1) weave_step<false>(A, pp[1], t.dt, t.tab.var, emax);
  // stage B: p = Q(f32(f64(y) * d_c)), d wave-uniform (the wave is one client)
  dampen_stage<3>(y, dampen[__builtin_amdgcn_readfirstlane(c < M ? c : M - 1)]);
  float p[3];
  q_stage_d16x<3>(p, y, &t.dt, t.tab.var);
#pragma unroll
  for (int j = 2; j < CS; ++j) weave_step<false>(A, pp[j], t.dt, t.tab.var, emax);
#pragma unroll
  for (int e = 0; e < 3; ++e) pdst[3 * gl + e] = live ? p[e] : 0.0f;
}

// Tile `bid` of the woven grid (LDS state in sh).
template <int NW>
__device__ __forceinline__ void update_weave_block(WeaveShared<NW>& sh, int64_t bid, const uint8_t* __restrict__ uploads,
                                                   size_t pitch, int M, const double* __restrict__ dampen,
                                                   double inv_avg, int64_t n_up, int64_t g_begin, int64_t g_end,
                                                   const int32_t* __restrict__ hdr_block, uint8_t* __restrict__ merged,
                                                   float* __restrict__ merged_f32, int* __restrict__ err) {
  static_assert(NW == 6 || NW == 8, "three consumer waves + producer-only waves (the planned widths)");
  constexpr int E = kWeaveE, CM = NW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t g0 = g_begin + bid * kWeaveTG;
  const int ng = (int)min<int64_t>(kWeaveTG, g_end - g0);
  const int64_t walk_end = hdr_block[2];
  // consumers: three consecutive waves from r = tile mod NW (on three different SIMDs
  // when waves go to SIMDs round robin), so the serial work rotates over the SIMDs
  const int r = (int)(bid % NW);
  const int ci = (wave - r + NW) % NW;  // consumer index 0..2, or a producer-only wave
  const bool consumer = ci < 3;          // wave-uniform
  const int col = (consumer ? ci : 0) * 64 + lane;  // the consumer's value
  const int nchunks = (M + CM - 1) / CM;
  const int gl = lane;
  const bool glive = gl < ng;
  const uint8_t* rowbase = uploads + 16 * (g0 + (glive ? gl : 0));
  auto load = [&](int k) -> uint4 {  // chunk k's group of this lane (client k * CM + wave)
    const int c = k * CM + wave;
    return *reinterpret_cast<const uint4*>(rowbase + (size_t)(c < M ? c : M - 1) * pitch);
  };
  uint4 nxt = load(0);  // in flight while the tables are copied
  tile_init(sh.t, hdr_block + 4, hdr_block[1], g0, ng);
  uint32_t badacc = 0, emax = 0;
  float A = 0.0f;
  // interval 0: produce chunk 0
  {
    const uint4 cur = nxt;
    if (nchunks > 1) nxt = load(1);
    const int c = wave;
    weave_item<NW, 0, false>(sh, cur, glive && c < M, c, gl, M, dampen, n_up, walk_end, g0, sh.p[0] + wave * E, badacc,
                             A, nullptr, col, emax);
  }
  __syncthreads();
  // intervals 1 .. nchunks-1: produce chunk k, consume chunk k-1 (always CM clients);
  // the progress priority ladder of the classic tiles (update_tiled_block)
  const int r1 = nchunks / 4, r2 = nchunks / 2, r3 = 3 * nchunks / 4;
  if (FLEET_TILE_LADDER) __builtin_amdgcn_s_setprio(3);
  for (int k = 1; k < nchunks; ++k) {
    FLEET_WTRACE(bid, k, 0);
    if (FLEET_TILE_LADDER) {
      if (k == r1) __builtin_amdgcn_s_setprio(2);
      if (k == r2) __builtin_amdgcn_s_setprio(1);
      if (k == r3) __builtin_amdgcn_s_setprio(0);
    }
    const uint4 cur = nxt;
    if (k + 1 < nchunks) nxt = load(k + 1);
    const int c = k * CM + wave;
    float* pdst = sh.p[k & 1] + wave * E;
    const float* pc = sh.p[(k - 1) & 1];
    if (consumer) {
      if (k == 1)
        weave_item<NW, CM, true>(sh, cur, glive && c < M, c, gl, M, dampen, n_up, walk_end, g0, pdst, badacc, A, pc,
                                 col, emax);
      else
        weave_item<NW, CM, false>(sh, cur, glive && c < M, c, gl, M, dampen, n_up, walk_end, g0, pdst, badacc, A, pc,
                                  col, emax);
    } else {
      weave_item<NW, 0, false>(sh, cur, glive && c < M, c, gl, M, dampen, n_up, walk_end, g0, pdst, badacc, A,
                               nullptr, col, emax);
    }
    FLEET_WTRACE(bid, k, 1);
    __syncthreads();
    FLEET_WTRACE(bid, k, 2);
  }
  // the last interval: consume the last chunk (cm clients)
  if (consumer) {
    const float* pc = sh.p[(nchunks - 1) & 1];
    const int cm = M - (nchunks - 1) * CM;
    int j = 0;
    if (nchunks == 1) {
      A = pc[col];
      j = 1;
    }
    for (; j < cm; ++j) weave_step<false>(A, pc[j * E + col], sh.t.dt, sh.t.tab.var, emax);
  }
  if (badacc) atomicOr(err, FLEET_ERRBIT_BASE64);
  // a running sum outside the q_gen domain (never for gradients): the whole chain again, exactly
  const bool off = consumer && col < 3 * ng && emax >= kD16Out;
  if (__ballot(off)) {
    if (off) A = chain_general(uploads, pitch, M, dampen, g0 + col / 3, col % 3, &sh.t.tab);
  }
  __syncthreads();  // every consumer is done with the p buffers
  float* finals = sh.p[0];
  if (consumer) finals[col] = A;
  __syncthreads();
  tile_epilogue(sh.t, finals, inv_avg, n_up, walk_end, g0, ng, merged, merged_f32, err,
                reinterpret_cast<int32_t*>(sh.p[1]));
}

template <int NW>
__global__ void __launch_bounds__(64 * NW) k_update_weave(const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                                          const double* __restrict__ dampen, double inv_avg,
                                                          int64_t n_up, int64_t g_begin, int64_t g_end,
                                                          const int32_t* __restrict__ hdr_block,
                                                          uint8_t* __restrict__ merged, float* __restrict__ merged_f32,
                                                          int* __restrict__ err) {
  __shared__ WeaveShared<NW> sh;
  FLEET_BTRACE(0);
  update_weave_block<NW>(sh, xcd_tile(blockIdx.x, gridDim.x), uploads, pitch, M, dampen, inv_avg, n_up, g_begin, g_end,
                         hdr_block, merged, merged_f32, err);
  FLEET_BTRACE(1);
}


// Client-side encode: rows of fp32 -> rows of Base64 (Base64::encode(vector<float>)).
// Block (bx, by) encodes groups [NT*bx, NT*bx+NT) of rows [rpb*by, rpb*by+rpb):
// a lane walks its group down rpb rows (next row's floats loaded while the
// current one is encoded), so the LDS table copy is paid once per rpb rows.
// ROT = true: the rows in flight rotate through registers with a row loop
// unrolled by two (no copies between rows) -- the standalone encode, 467 -> 448 us
// on synth1m_256 (same-box A/B); ROT = false: one register pair copied forward per
// row -- the form the fused step keeps (the rotating loop made it 1 % slower there).
template <bool D16, int NT = 256, bool ROT = false>
__device__ __forceinline__ void encode_rows(const float* __restrict__ values, int64_t n, size_t vpitch,
                                            uint8_t* __restrict__ out, size_t pitch, int64_t groups, int rows,
                                            int rpb, int64_t bx, int by, const B64Tables* tab,
                                            const D16Table* dt) {
  const int64_t g = bx * NT + threadIdx.x;
  if (g >= groups) return;
  const int row0 = by * rpb, row1 = min(rows, row0 + rpb);
  const int r = (int)min<int64_t>(3, n - 3 * g);
  const float* v = values + (size_t)row0 * vpitch + 3 * g;
  // one 12-byte load per full group (a wave instruction spans 768 contiguous
  // bytes once, instead of three dword loads over the same lines); two rows in
  // flight ahead of the one being encoded
  typedef float f3 __attribute__((ext_vector_type(3)));
  // 12*g is only 4-byte aligned: the load's type promises no more than that
  typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));
  auto load = [&](int rr) -> f3 {
    const float* p = v + (size_t)(rr - row0) * vpitch;
    if (r == 3) return *reinterpret_cast<const f3u*>(p);
    return f3{p[0], r > 1 ? p[1] : 0.0f, 0.0f};
  };
  auto emit = [&](int rr, const float (&x)[3]) {
    if constexpr (D16) store_stream16(out + (size_t)rr * pitch + 16 * g, encode_group(x, r, tab, dt));
    else store_stream16(out + (size_t)rr * pitch + 16 * g, encode_group(x, r, tab));
  };
  // the fused steps' encode blocks (D16) on rows padded to whole groups (bench.py's buffers):
  // there the encode's VALU work shares the SIMDs with the aggregation's, and the form
  // below has the fewest instructions; the standalone encode (HBM-bound) keeps two rows in
  // flight ahead of the one it encodes (the form below, one row ahead, measured 3 % slower
  // there: synth1m_256 443 -> 459 us, r06 call a5)
  if (D16 && vpitch >= (size_t)(3 * groups)) {  // block-uniform
    // Every lane loads its 12 bytes (a buffer load from the row's uniform address, SALU-
    // advanced), so the loads need no per-lane form: the rows in flight rotate through
    // the same registers, with no copies between rows (the branchy load made the compiler
    // copy each row twice). The last group's slots past n are masked to +0.0, the value
    // the unpadded load gives them.
    typedef uint32_t u3v __attribute__((ext_vector_type(3)));
    uint32_t m1 = r > 1 ? ~0u : 0u, m2 = r > 2 ? ~0u : 0u;
    asm("" : "+v"(m1), "+v"(m2));  // opaque masks: one v_and per slot, not a v_cndmask_e64 each
    const uint32_t off = (uint32_t)(12 * g);  // a row < 2 GiB (the launchers check)
    auto ld = [&](int rr) -> u3v {
      const __amdgpu_buffer_rsrc_t row = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(values + (size_t)rr * vpitch), (short)0, 0x7fffffff, kBufferDword3);
      return __builtin_amdgcn_raw_buffer_load_b96(row, off, 0, 0);
    };
    const uint32_t ooff = (uint32_t)(16 * g);
    auto emit_u = [&](int rr, const u3v& w) {
      const float x[3] = {u2f(w.x), u2f(w.y & m1), u2f(w.z & m2)};
      const uint4 t = D16 ? encode_group(x, r, tab, dt) : encode_group(x, r, tab);
      typedef uint32_t u4v __attribute__((ext_vector_type(4)));
      const __amdgpu_buffer_rsrc_t orow = __builtin_amdgcn_make_buffer_rsrc(out + (size_t)rr * pitch, (short)0,
                                                                             0x7fffffff, kBufferDword3);
      __builtin_amdgcn_raw_buffer_store_b128(u4v{t.x, t.y, t.z, t.w}, orow, ooff, 0, kBufferNT);
    };
    // a row's registers are reloaded right after it is encoded (the other row in flight
    // meanwhile), so no register is copied between rows; the loads are unconditional
    // (the last row again at the end), so the loop carries no per-lane PHI either
    u3v a = ld(row0), b = ld(min(row0 + 1, row1 - 1));
    for (int row = row0; row < row1; row += 2) {
      emit_u(row, a);
      a = ld(min(row + 2, row1 - 1));
      if (row + 1 < row1) emit_u(row + 1, b);  // block-uniform
      b = ld(min(row + 3, row1 - 1));
    }
    return;
  }
  if constexpr (ROT) {
    f3 buf[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) buf[k] = row0 + k < row1 ? load(row0 + k) : f3{0.0f, 0.0f, 0.0f};
    for (int row = row0; row < row1; row += 2) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int rr = row + k;
        if (rr < row1) {  // block-uniform
          const float x[3] = {buf[k].x, buf[k].y, buf[k].z};
          if (rr + 2 < row1) buf[k] = load(rr + 2);
          emit(rr, x);
        }
      }
    }
  } else {
    f3 n1 = load(row0), n2 = f3{0.0f, 0.0f, 0.0f};
    if (row0 + 1 < row1) n2 = load(row0 + 1);
    for (int row = row0; row < row1; ++row) {
      const float x[3] = {n1.x, n1.y, n1.z};
      n1 = n2;
      if (row + 2 < row1) n2 = load(row + 2);
      emit(row, x);
    }
  }
}

// Kardam's side outputs of the pipelined form (CppNNUpdater.java:463-481,
// Kardam.java:48-106): the tiles' producer waves compute them with p (tile_kardam: G =
// Q(f32(f64(p) * lr)) into g_out, ||G||^2 and ||Q(G - prev)||^2 summed over the tile's
// groups per client, one partial slot per (client, tile)), and M reduce blocks riding
// in the same launch add a client's tile partials in a fixed order -- no second launch
// (a dependent launch costs >= 4.5 us at MNIST size, a quarter of the update).
// Hand-off: a producer wave's partial stores are sc1 (agent-scope relaxed atomics) and
// drained (vmcnt 0) before it publishes the launch's epoch in its flag
// (flags[tile * NPW + wave]); a reduce block polls every flag with relaxed sc1 loads,
// then reads the partials with sc1 loads (no agent-scope release / acquire: their L2
// writeback and invalidate per wave cost more than the whole reduce). Tiles are
// dispatched before every reduce block and never wait on one, so the launch drains;
// the epoch (new per launch, never reused) makes a stale flag never match, so the
// flags need no reset.
struct KardamReduceJob {
  double* norms;    // M pairs
  uint32_t* flags;  // tiles x producer waves
  uint32_t epoch;
  uint32_t wait_skew = 0;  // test hook (fleet_test_kardam_skew): the reduce waits for epoch + skew
};
template <int NT, int NPW>
__device__ __forceinline__ void kardam_reduce_block(const KardamReduceJob& kr, int c, int64_t ntiles,
                                                    const double* partials, double (*red)[NT / 64],
                                                    int* __restrict__ err) {
  // every tile's producers done (bounded ~0.5 s: a flag that never comes sets
  // FLEET_ERRBIT_SYNC, which fleet_update_kardam_device reads after its sync and fails
  // the call; the thread stops waiting at its first missing flag)
  const uint32_t want = kr.epoch + kr.wait_skew;
  bool late = false;
  for (int64_t f = threadIdx.x; f < ntiles * NPW && !late; f += NT) {
    for (uint32_t spin = 0; __hip_atomic_load(kr.flags + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want;
         ++spin) {
      if (spin == (1u << 21)) {
        atomicOr(err, FLEET_ERRBIT_SYNC);
        late = true;
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
  }
  // (the barrier also keeps the compiler from hoisting the partial loads above the polls)
  __syncthreads();
  // the client's tile partials in a fixed order: lane t of the block adds tiles t, t + NT, ...
  const double* p = partials + (size_t)c * ntiles * 2;
  double a = 0.0, b = 0.0;
  for (int64_t t = threadIdx.x; t < ntiles; t += NT) {
    a += __hip_atomic_load(p + 2 * t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    b += __hip_atomic_load(p + 2 * t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  a = group_sum_f64<64>(a);  // valid in lane 63
  b = group_sum_f64<64>(b);
  if ((threadIdx.x & 63) == 63) {
    red[0][threadIdx.x / 64] = a;
    red[1][threadIdx.x / 64] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double sa = 0.0, sb = 0.0;
    for (int i = 0; i < NT / 64; ++i) {
      sa += red[0][i];
      sb += red[1][i];
    }
    kr.norms[2 * c] = sa;
    kr.norms[2 * c + 1] = sb;
  }
}

// Pipelined tile variant (E = 3*TG <= 64): producer waves compute p for passes
// of clients into an LDS ring while wave 0 consumes them in client order (the
// serial A = Q(A + p_c)), so the client-independent work and the serial
// accumulation overlap instead of running back to back.
//   WP = 0: a pass is shared by all producer waves (IPT items per thread);
//   WP = 1: a pass belongs to ONE producer wave (passes dealt round-robin), so
//           a pass is ready after one wave's work -- the consumer starts
//           early -- while the NW-1 producer waves work on successive passes
//           in parallel.
// Blocks [nU, ...): the next batch's client encode (ej; the pipelined step), or with
// KD = true Kardam's reduce blocks: the producers compute Kardam's side outputs with p
// (tile_kardam) and one block per client adds its tile partials (kardam_reduce_block).
// Hand-off through LDS: a producer wave publishes its count of finished passes
// with a workgroup release after its p writes; the consumer acquires it before
// reading a pass, and publishes "passes consumed" so producers never overwrite
// a ring slot still being read. Every wait has a partner that always makes
// progress, so the grid drains.
// p floats in the ring: 12 KiB = four passes of 16 clients at TG = 16, enough for the
// producers to stay ahead (r04: the consumer waits 0.3 us in all), and it keeps the block
// at 34.7 KB of LDS, four per CU, so the step's encode blocks get a slot beside the
// 1.9 tiles per CU of a MNIST-size launch (24 KiB of ring: 46.7 KB, three per CU)
#ifndef FLEET_PIPE_RING
#define FLEET_PIPE_RING 3072
#endif
#ifndef FLEET_KD_RING
#define FLEET_KD_RING 3072
#endif
#ifndef FLEET_PIPE_D16
#define FLEET_PIPE_D16 1
#endif
template <int TG, int IPT, int NW, int WP = 0, bool KD = false>
__global__ void __launch_bounds__(64 * NW) k_update_pipe(const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                                     const double* __restrict__ dampen, double inv_avg,
                                                     int64_t n_up, int64_t g_begin, int64_t g_end,
                                                     const int32_t* __restrict__ hdr_block,
                                                     uint8_t* __restrict__ merged, float* __restrict__ merged_f32,
                                                     int* __restrict__ err, int nU, EncodeJob ej,
                                                     KardamOut kd = KardamOut{},
                                                     KardamReduceJob kr = KardamReduceJob{}) {
  constexpr int E = 3 * TG;
  static_assert(E <= 64, "one consumer wave");
  constexpr int NPW = NW - 1;                                // producer waves
  constexpr int CPP = ((WP ? 1 : NPW) * 64 * IPT) / TG;      // clients per pass
  constexpr int RP = KD ? FLEET_KD_RING : FLEET_PIPE_RING;
  constexpr int RING = (RP / E) / CPP > 0 ? (RP / E) / CPP : 1;  // passes in LDS
  static_assert(RING * CPP >= 1, "the ring holds the epilogue's E codes");
  FLEET_TSTAMP(0);
  // the producers on the byte-table digit counts (D16: the stream kernel's stages; the
  // tiles of a MNIST-size launch, 1.9 per CU, leave the LDS for its 9 KB)
  __shared__ TileShared<TG, NW, (bool)FLEET_PIPE_D16> sh;
  __shared__ XlTable xl;  // the consumer's one-lookup Q
  __shared__ float ptile[RING * CPP * E];
  __shared__ float finals[E];
  __shared__ int prog[NPW];  // passes finished by each producer wave
  __shared__ int consumed;   // passes finished by the consumer
  // wave index made wave-uniform (readfirstlane), so the producer/consumer
  // split below is a scalar branch and the consumer's s_setprio is its own
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  if constexpr (KD) {
    if ((int)blockIdx.x >= nU) {  // block-uniform: Kardam's reduce of one client's tile partials
      __shared__ double kred[2][NW];
      kardam_reduce_block<64 * NW, NPW>(kr, (int)blockIdx.x - nU, nU, kd.partials, kred, err);
      return;
    }
  }
  if ((int)blockIdx.x >= nU) {  // block-uniform: a job riding in the launch
    b64_tables_init<64 * NW>(&sh.tab);
#if FLEET_PIPE_D16
    d16_table_init<64 * NW>(&sh.dt);
#endif
    __syncthreads();
    const int64_t e = (int64_t)blockIdx.x - nU;
    // the next batch's client encode (fleet_update_encode_device), on the byte table too
#if FLEET_PIPE_D16
    encode_rows<true, 64 * NW>(ej.values, ej.n, ej.vpitch, ej.out, ej.pitch, ej.groups, ej.rows, ej.rpb, e % ej.gx,
                               (int)(e / ej.gx), &sh.tab, &sh.dt);
#else
    encode_rows<false, 64 * NW>(ej.values, ej.n, ej.vpitch, ej.out, ej.pitch, ej.groups, ej.rows, ej.rpb, e % ej.gx,
                                (int)(e / ej.gx), &sh.tab, nullptr);
#endif
    return;
  }
  const int64_t g0 = g_begin + (int64_t)blockIdx.x * TG;
  const int ng = (int)min<int64_t>(TG, g_end - g0);
  if (tid < NPW) prog[tid] = 0;
  if (tid == 0) consumed = 0;
  const int npass = (M + CPP - 1) / CPP;
  // producers: the first pass's groups in flight while the tables are copied
  const int w = wave - 1;
  const int step = WP ? NPW : 1;
  const int it0 = WP ? lane : tid - 64, stride = WP ? 64 : NPW * 64;
  int pass = WP ? w : 0;
  TileItems<TG, IPT> nxt;  // the next pass's groups, loaded one pass ahead
  if (wave > 0 && pass < npass)
    tile_load<TG, IPT>(nxt, uploads, pitch, g0, ng, pass * CPP, min(CPP, M - pass * CPP) * TG, it0, stride);
  tile_init(sh, hdr_block + 4, hdr_block[1], g0, ng);
  FLEET_TSTAMP(1);
  uint32_t badacc = 0;

  if (wave > 0) {  // ---------------------------------------------- producers
    int done = 0;
    for (; pass < npass; pass += step) {
      const TileItems<TG, IPT> cur = nxt;
      const int np = pass + step;
      if (np < npass) tile_load<TG, IPT>(nxt, uploads, pitch, g0, ng, np * CPP, min(CPP, M - np * CPP) * TG, it0,
                                         stride);
      if (pass >= RING) {  // ring slot free once the consumer finished pass - RING
        while (__hip_atomic_load(&consumed, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < pass - RING + 1)
          __builtin_amdgcn_s_sleep(1);
      }
      tile_compute<TG, IPT, NW, KD>(sh, cur, M, dampen, n_up, hdr_block[2], g0, ptile + (pass % RING) * CPP * E,
                                    badacc, TileKd{kd, (int64_t)blockIdx.x, (int64_t)nU, (int64_t)hdr_block[2]});
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      ++done;
      if (lane == 0) __hip_atomic_store(&prog[w], done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if constexpr (KD) {  // this wave's Kardam partials are out: the reduce blocks may read them
      // the sc1 stores drained (vmcnt 0), then the flag: no agent-scope release (an L2
      // writeback per wave; 82 us against 19 us for the tiles alone on mnist64, r05 call x2).
      // Hardware order: the partials are agent-scope (sc1) atomic stores, complete at the
      // agent's coherence point once vmcnt reaches 0, and the flag store issues after that.
      // Compiler order: the waitcnt intrinsic is not a memory operation, so an empty asm
      // with a memory clobber keeps every partial store above it (no fence instruction).
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_waitcnt(0);
      if (lane == 0)
        __hip_atomic_store(kr.flags + (size_t)blockIdx.x * NPW + w, kr.epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  } else {  // ---------------------------------------------------- consumer
    // the serial chain is the block's critical path: win VALU issue
    // arbitration against co-resident producer waves (MI355X_MICROARCH.md,
    // two waves per SIMD, item 4)
    __builtin_amdgcn_s_setprio(3);
    // the q_xl table is the consumer's alone: copied while pass 0 is produced,
    // visible to this wave once its own LDS writes are done (no block barrier)
    xl_table_init<64>(&xl);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done
    __builtin_amdgcn_wave_barrier();
    float A = 0.f;
    float amax = 0.f;  // max |A + p| over the chain: q_xl is exact below 1e8
    const int col = tid < E ? tid : 0;
#ifdef FLEET_TIMING
    unsigned long long waited = 0, spun = 0;
#endif
    for (int pass = 0; pass < npass; ++pass) {
#ifdef FLEET_TIMING
      const unsigned long long w0 = wall_clock64();
      bool spin = false;
#endif
      for (;;) {
        bool ready;
        if (WP) {
          ready = __hip_atomic_load(&prog[pass % NPW], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >
                  pass / NPW;
        } else {
          int m = __hip_atomic_load(&prog[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
          for (int v = 1; v < NPW; ++v)
            m = min(m, __hip_atomic_load(&prog[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          ready = m > pass;
        }
        if (ready) break;
#ifdef FLEET_TIMING
        spin = true;
#endif
        __builtin_amdgcn_s_sleep(1);
      }
#ifdef FLEET_TIMING
      if (pass > 0) {  // slot 6: time the consumer waited for producers after the first pass
        waited += wall_clock64() - w0;
        spun += spin;
      }
      if (threadIdx.x == 0) {
        g_fleet_timing[blockIdx.x * 8 + 6] = waited;
        g_fleet_timing[blockIdx.x * 8 + 7] = spun;
      }
#endif
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (pass == 0) {
        FLEET_TSTAMP(2);
        FLEET_TSTAMP(3);
      }
      const float* pt = ptile + (pass % RING) * CPP * E;
      const int cm = min(CPP, M - pass * CPP);
      int k = 0;
      if (pass == 0) {
        A = pt[col];
        k = 1;
      }
#pragma unroll 4
      for (; k < cm; ++k) {
        const float s = A + pt[k * E + col];
        amax = __builtin_fmaxf(amax, __builtin_fabsf(s));  // s is finite: p and A are Q outputs
        A = q_xl(s, xl.x);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&consumed, pass + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const bool off_domain = tid < 3 * ng && !(amax < 1e8f);  // columns past the last group hold no values
    if (__ballot(off_domain)) {                                // wave-uniform, never for gradients
      if (off_domain) A = chain_general(uploads, pitch, M, dampen, g0 + tid / 3, tid % 3, &sh.tab);
    }
    if (tid < E) finals[tid] = A;
  }
  FLEET_TSTAMP(4);
  if (badacc) atomicOr(err, FLEET_ERRBIT_BASE64);
  __syncthreads();
  // (the ring is free after the barrier: the merged codes are assembled there)
  tile_epilogue(sh, finals, inv_avg, n_up, hdr_block[2], g0, ng, merged, merged_f32, err,
                reinterpret_cast<int32_t*>(ptile));
  FLEET_TSTAMP(5);
}

// ----------------------------------------------------------------------------
#ifndef FLEET_STREAM_TU  // (the stream unit needs only the two stream kernels)
__global__ void __launch_bounds__(256) k_encode_f32(const float* __restrict__ values, int64_t n, size_t vpitch,
                                                    uint8_t* __restrict__ out, size_t pitch, int64_t groups,
                                                    int rows, int rpb) {
  __shared__ B64Tables tab;
  b64_tables_init(&tab);
  __syncthreads();
  encode_rows<false, 256, true>(values, n, vpitch, out, pitch, groups, rows, rpb, blockIdx.x, blockIdx.y, &tab, nullptr);
}
#endif

// One launch, two independent jobs on disjoint buffers: the aggregation of the
// uploads already in HBM (blocks [0, nU): k_update_mixed's grid) and the client
// encode of the NEXT batch's rows into another upload buffer (blocks [nU, ...):
// k_encode_f32's grid, flattened x-fastest). The aggregation is VALU-bound and
// leaves HBM mostly idle, the encode is HBM-bound; the dispatcher places the
// aggregation's blocks first (they fit the chip in one round) and streams the
// encode's blocks through the wave slots and issue cycles they leave. Each
// block's results are those of the separate kernels.
template <int NT>
__global__ void __launch_bounds__(NT) k_update_encode(const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                                      const double* __restrict__ dampen, double inv_avg,
                                                      int64_t n_up, int64_t g_begin, int64_t g_end,
                                                      const int32_t* __restrict__ hdr_block,
                                                      uint8_t* __restrict__ merged, float* __restrict__ merged_f32,
                                                      int* __restrict__ err, int nA, int nU, EncodeJob ej) {
  static_assert(NT == 256, "the encode blocks are 256 lanes");
  __shared__ B64Tables tab;
  __shared__ D16Table dtab;
  __shared__ LastDigitTable ldt;
  b64_tables_init<NT>(&tab);
  d16_table_init<NT>(&dtab);
  if ((int)blockIdx.x < nU) ld16_table_init<NT>(&ldt);  // block-uniform: the update blocks read it
  __syncthreads();
  // the update waves run the issue-priority ladder (3 -> 0 as they get ahead) and the
  // encode's waves run at priority 3: the HBM-bound encode issues whenever it can, the
  // update waves that lag next. synth1m_256 step 1129-1133 -> 1119-1120 us with the
  // encode at 2 (r04 call a15), 1171-1176 -> 1153-1158 us from 2 to 3 on
  // another box (gpu_r04_a16.sh); at 0 (r04 a6: 1158 us) or 1 (1138-1142 us) slower, and
  // so were update waves laddered from 2 under the encode's 3 (1134-1141 against
  // 1118-1129 us, gpu_r04_a26.sh)
  if ((int)blockIdx.x < nU) {  // block-uniform
    update_mixed_block<NT, false, 3, true>(tab, dtab, blockIdx.x, uploads, pitch, M, dampen, inv_avg, n_up, g_begin,
                                           g_end, hdr_block, merged, merged_f32, err, nA, KardamOut{}, ldt.ld16);
  } else {
    const int64_t e = (int64_t)blockIdx.x - nU;
    encode_prio(ej.prio);
    encode_rows<true>(ej.values, ej.n, ej.vpitch, ej.out, ej.pitch, ej.groups, ej.rows, ej.rpb, e % ej.gx,
                     (int)(e / ej.gx), &tab, &dtab);
  }
}

// The stream kernels are compiled in their own translation unit
// (stream_kernels.hip: this file under FLEET_STREAM_TU) with the ILP-first
// machine scheduler, which helps them (VALU-issue bound at 5-6 waves per SIMD)
// and hurts the tiled and pipelined kernels; the main unit only
// declares their instantiations.
#if defined(FLEET_STREAM_TU) || defined(FLEET_DEV_ALL_KERNELS)  // (dev tools that include this file: all here)
template __global__ void k_update_mixed<256, false>(const uint8_t* __restrict__, size_t, int,
                                                    const double* __restrict__, double, int64_t, int64_t, int64_t,
                                                    const int32_t* __restrict__, uint8_t* __restrict__,
                                                    float* __restrict__, int* __restrict__, int, KardamOut);
template __global__ void k_update_mixed<256, true>(const uint8_t* __restrict__, size_t, int,
                                                   const double* __restrict__, double, int64_t, int64_t, int64_t,
                                                   const int32_t* __restrict__, uint8_t* __restrict__,
                                                   float* __restrict__, int* __restrict__, int, KardamOut);
template __global__ void k_update_encode<256>(const uint8_t* __restrict__, size_t, int, const double* __restrict__,
                                              double, int64_t, int64_t, int64_t, const int32_t* __restrict__,
                                              uint8_t* __restrict__, float* __restrict__, int* __restrict__, int, int,
                                              EncodeJob);
#else
extern template __global__ void k_update_mixed<256, false>(const uint8_t* __restrict__, size_t, int,
                                                           const double* __restrict__, double, int64_t, int64_t,
                                                           int64_t, const int32_t* __restrict__, uint8_t* __restrict__,
                                                           float* __restrict__, int* __restrict__, int, KardamOut);
extern template __global__ void k_update_mixed<256, true>(const uint8_t* __restrict__, size_t, int,
                                                          const double* __restrict__, double, int64_t, int64_t,
                                                          int64_t, const int32_t* __restrict__, uint8_t* __restrict__,
                                                          float* __restrict__, int* __restrict__, int, KardamOut);
extern template __global__ void k_update_encode<256>(const uint8_t* __restrict__, size_t, int,
                                                     const double* __restrict__, double, int64_t, int64_t, int64_t,
                                                     const int32_t* __restrict__, uint8_t* __restrict__,
                                                     float* __restrict__, int* __restrict__, int, int, EncodeJob);
#endif

#ifndef FLEET_STREAM_TU

// The same pairing for the tiled sizes (CIFAR buckets): blocks [0, nU) are
// k_update_tiled<TG>'s byte-table tiles on one width (every tile is resident at
// once there and the encode's blocks fill the CUs the last partial round leaves:
// the two-width grid measured slower in the fused step), the rest
// the client encode's blocks on the tile's tables (enc_d16, as in k_update_encode).
template <int TG>
__global__ void __launch_bounds__(256) k_update_tiled_encode(const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                                             const double* __restrict__ dampen, double inv_avg,
                                                             int64_t n_up, int64_t g_begin, int64_t g_end,
                                                             const int32_t* __restrict__ hdr_block,
                                                             uint8_t* __restrict__ merged,
                                                             float* __restrict__ merged_f32, int* __restrict__ err,
                                                             int nU, EncodeJob ej) {
  __shared__ TileShared<TG, 4, true> sh;
  __shared__ float ptile[tiled_chunk_clients<TG, true>() * 3 * TG];
  FLEET_BTRACE(0);
  if ((int)blockIdx.x < nU) {  // block-uniform
    update_tiled_block<TG, false, true>(sh, ptile, xcd_tile(blockIdx.x, nU), uploads, pitch, M, dampen, inv_avg, n_up,
                                        g_begin, g_end, hdr_block, merged, merged_f32, err);
    FLEET_BTRACE(1);
  } else {
    b64_tables_init(&sh.tab);
    d16_table_init(&sh.dt);
    __syncthreads();
    encode_prio(ej.prio);
    const int64_t e = (int64_t)blockIdx.x - nU;
    encode_rows<true>(ej.values, ej.n, ej.vpitch, ej.out, ej.pitch, ej.groups, ej.rows, ej.rpb, e % ej.gx,
                      (int)(e / ej.gx), &sh.tab, &sh.dt);
    FLEET_BTRACE(1);
  }
}

// The flat tiles (update_flat_block) on blocks [0, fg.nU); with fg.nU < gridDim.x the
// client encode's blocks follow (the fused step), on the tile's tables as in
// k_update_tiled_encode. (The encode inside the tiles -- the fourth wave encoding the
// tile's columns during phase 2 -- made it the critical path: 449 against 390 us on
// cifar10_256, r05.)
template <bool KD>
__device__ __forceinline__ void flat_kernel(const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                            const double* __restrict__ dampen, double inv_avg, int64_t n_up,
                                            int64_t g_begin, int64_t g_end, const int32_t* __restrict__ hdr_block,
                                            uint8_t* __restrict__ merged, float* __restrict__ merged_f32,
                                            int* __restrict__ err, const FlatGrid& fg, const EncodeJob& ej,
                                            const KardamOut& kd) {
  __shared__ TileShared<kFlatTG, 4, true> sh;
  __shared__ float pbuf[3 * kFlatPass];
  FLEET_BTRACE(0);
  if ((int)blockIdx.x < fg.nU) {  // block-uniform
    int64_t g0;
    int ng, w;
    flat_tile_range(blockIdx.x, fg, g_begin, g_end, &g0, &ng, &w);
    if (ng > 0) {
      update_flat_block<KD>(sh, pbuf, blockIdx.x, g0, ng, w, uploads, pitch, M, dampen, inv_avg, n_up, hdr_block,
                            merged, merged_f32, err,
                            TileKd{kd, (int64_t)blockIdx.x, (int64_t)fg.nU, (int64_t)hdr_block[2]});
    } else if constexpr (KD) {
      // an empty tile (flat_grid makes none today) still owns its (client, tile) partial
      // slots, which k_kardam_reduce sums: zero them explicitly
      for (int c = threadIdx.x; c < M; c += blockDim.x) {
        double* slot = kd.partials + ((size_t)c * fg.nU + blockIdx.x) * 2;
        slot[0] = 0.0;
        slot[1] = 0.0;
      }
    }
  } else if constexpr (!KD) {
    b64_tables_init(&sh.tab);
    d16_table_init(&sh.dt);
    __syncthreads();
    encode_prio(ej.prio);
    const int64_t e = (int64_t)blockIdx.x - fg.nU;
    encode_rows<true>(ej.values, ej.n, ej.vpitch, ej.out, ej.pitch, ej.groups, ej.rows, ej.rpb, e % ej.gx,
                      (int)(e / ej.gx), &sh.tab, &sh.dt);
  }
  FLEET_BTRACE(1);
}

__global__ void __launch_bounds__(256) k_update_flat(const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                                     const double* __restrict__ dampen, double inv_avg, int64_t n_up,
                                                     int64_t g_begin, int64_t g_end,
                                                     const int32_t* __restrict__ hdr_block,
                                                     uint8_t* __restrict__ merged, float* __restrict__ merged_f32,
                                                     int* __restrict__ err, FlatGrid fg, EncodeJob ej) {
  flat_kernel<false>(uploads, pitch, M, dampen, inv_avg, n_up, g_begin, g_end, hdr_block, merged, merged_f32, err, fg,
                     ej, KardamOut{});
}

// The flat tiles with Kardam's side outputs (their partials summed by k_kardam_reduce)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_num_sgpr(84), amdgpu_num_vgpr(72))) k_update_flat_kd(const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                                        const double* __restrict__ dampen, double inv_avg,
                                                        int64_t n_up, int64_t g_begin, int64_t g_end,
                                                        const int32_t* __restrict__ hdr_block,
                                                        uint8_t* __restrict__ merged, float* __restrict__ merged_f32,
                                                        int* __restrict__ err, FlatGrid fg, KardamOut kd) {
  flat_kernel<true>(uploads, pitch, M, dampen, inv_avg, n_up, g_begin, g_end, hdr_block, merged, merged_f32, err, fg,
                    EncodeJob{}, kd);
}

// The woven tiles with the next batch's client encode riding in the launch (the
// pipelined step at CIFAR sizes): blocks [0, nU) are tiles, the rest the encode's
// 64*NW-lane blocks on the tile's tables.
template <int NW>
__global__ void __launch_bounds__(64 * NW) k_update_weave_encode(const uint8_t* __restrict__ uploads, size_t pitch,
                                                                 int M, const double* __restrict__ dampen,
                                                                 double inv_avg, int64_t n_up, int64_t g_begin,
                                                                 int64_t g_end, const int32_t* __restrict__ hdr_block,
                                                                 uint8_t* __restrict__ merged,
                                                                 float* __restrict__ merged_f32, int* __restrict__ err,
                                                                 int nU, EncodeJob ej) {
  __shared__ WeaveShared<NW> sh;
  if ((int)blockIdx.x < nU) {  // block-uniform
    update_weave_block<NW>(sh, xcd_tile(blockIdx.x, nU), uploads, pitch, M, dampen, inv_avg, n_up, g_begin, g_end,
                           hdr_block, merged, merged_f32, err);
  } else {
    b64_tables_init<64 * NW>(&sh.t.tab);
    d16_table_init<64 * NW>(&sh.t.dt);
    __syncthreads();
    encode_prio(ej.prio);
    const int64_t e = (int64_t)blockIdx.x - nU;
    encode_rows<true, 64 * NW>(ej.values, ej.n, ej.vpitch, ej.out, ej.pitch, ej.groups, ej.rows, ej.rpb, e % ej.gx,
                               (int)(e / ej.gx), &sh.t.tab, &sh.t.dt);
  }
}

// getModelParametersNative (Server/src/main/c++/cppNN_backend.cpp:227-242):
// Base64::encode of network::getModelParams (commonLib/cppNN/network.h:708-723)
// = the use_bias() biases repeated `reps` times (the bias loop sits inside the
// loop over layer_graph) followed by the non-null W -- encoded straight from
// the resident model, without materialising the vector.
__global__ void __launch_bounds__(256) k_encode_model_params(const float* __restrict__ weights, int64_t n_w,
                                                             const float* __restrict__ biases, int64_t n_b,
                                                             int64_t reps, uint8_t* __restrict__ out,
                                                             int64_t groups) {
  __shared__ B64Tables tab;
  b64_tables_init(&tab);
  __syncthreads();
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= groups) return;
  const int64_t nbr = n_b * reps, n = nbr + n_w;
  const int r = (int)min<int64_t>(3, n - 3 * g);
  float x[3];
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    const int64_t v = 3 * g + e;
    x[e] = e >= r ? 0.0f : v < nbr ? biases[v % n_b] : weights[v - nbr];
  }
  *reinterpret_cast<uint4*>(out + 16 * g) = encode_group(x, r, &tab);
}

// getMiniBatch (Server/src/main/c++/cppNN_backend.cpp:677-699): Base64::encode
// of the vector uniformSample / nonIIDSample build (:553-675) -- 7 header
// values, then per sample its F features, (mode 1) the teacher's NL class
// probabilities, and its label as float; mode 1 ends with 1234567 --
// encoded straight from the resident dataset by sample index, without
// materialising the vector. An index outside [0, n_images) flags an argument
// error and reads row 0.
struct MiniBatchHeader {
  float v[7];
};
__global__ void __launch_bounds__(256) k_encode_minibatch(const float* __restrict__ images, int64_t n_images, int F,
                                                          const int32_t* __restrict__ labels,
                                                          const int32_t* __restrict__ idx, int B,
                                                          const float* __restrict__ teacher, int NL,
                                                          MiniBatchHeader hdr, uint8_t* __restrict__ out,
                                                          int64_t n, int64_t groups, int* __restrict__ err) {
  __shared__ B64Tables tab;
  b64_tables_init(&tab);
  __syncthreads();
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= groups) return;
  const int per = F + (teacher ? NL : 0) + 1;
  const int r = (int)min<int64_t>(3, n - 3 * g);
  float x[3];
  bool bad = false;
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    const int64_t p = 3 * g + e;
    float v = 0.0f;
    if (e < r) {
      if (p < 7) {
        v = hdr.v[p];
      } else {
        const int64_t q = p - 7, b = q / per;
        const int f = (int)(q - b * per);
        if (b >= B) {
          v = 1234567.0f;  // mode 1 end marker (:611)
        } else {
          int64_t row = idx[b];
          if (row < 0 || row >= n_images) bad = true, row = 0;
          v = f < F ? images[row * F + f] : (teacher && f < F + NL) ? teacher[b * NL + (f - F)] : (float)labels[row];
        }
      }
    }
    x[e] = v;
  }
  if (bad) atomicOr(err, FLEET_ERRBIT_ARG);
  *reinterpret_cast<uint4*>(out + 16 * g) = encode_group(x, r, &tab);
}

hipError_t launch_encode_minibatch(const float* images, int64_t n_images, int F, const int32_t* labels,
                                   const int32_t* idx, int B, const float* teacher, int NL, const float header[7],
                                   uint8_t* out, int* err, hipStream_t s) {
  const int64_t n = 7 + (int64_t)B * (F + (teacher ? NL : 0) + 1) + (teacher ? 1 : 0);
  const int64_t groups = (n + 2) / 3;
  MiniBatchHeader h;
  for (int i = 0; i < 7; ++i) h.v[i] = header[i];
  hipLaunchKernelGGL(k_encode_minibatch, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, images, n_images, F,
                     labels, idx, B, teacher, NL, h, out, n, groups, err);
  return hipGetLastError();
}

hipError_t launch_encode_model_params(const float* weights, int64_t n_w, const float* biases, int64_t n_b, int64_t reps,
                                      uint8_t* out, hipStream_t s) {
  const int64_t groups = (n_b * reps + n_w + 2) / 3;
  if (groups == 0) return hipSuccess;
  hipLaunchKernelGGL(k_encode_model_params, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, weights, n_w, biases,
                     n_b, reps, out, groups);
  return hipGetLastError();
}

// int32 codes -> Base64 (Base64::encode(vector<int>))
__global__ void __launch_bounds__(256) k_encode_i32(const int32_t* __restrict__ codes_in, int64_t n,
                                                    uint8_t* __restrict__ out, int64_t groups) {
  __shared__ B64Tables tab;
  b64_tables_init(&tab);
  __syncthreads();
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= groups) return;
  const int r = (int)min<int64_t>(3, n - 3 * g);
  int32_t codes[3];
#pragma unroll
  for (int e = 0; e < 3; ++e) codes[e] = e < r ? codes_in[3 * g + e] : 0;
  *reinterpret_cast<uint4*>(out + 16 * g) = pad_group(b64_encode_group(codes, &tab), r);
}

// Base64 rows -> fp32 rows (decodeFloat) or int32 (decodeInt, as_codes)
__global__ void __launch_bounds__(256) k_decode(const uint8_t* __restrict__ text, int64_t n, size_t pitch,
                                                void* __restrict__ out, size_t vpitch, int64_t groups,
                                                int as_codes, int* __restrict__ err) {
  __shared__ B64Tables tab;
  b64_tables_init(&tab);
  __syncthreads();
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= groups) return;
  const int64_t row_id = blockIdx.y;
  const int r = (int)min<int64_t>(3, n - 3 * g);
  int32_t codes[3];
  uint32_t bad = b64_decode_group(*reinterpret_cast<const uint4*>(text + row_id * pitch + 16 * g), &tab, codes);
  if (bad & needed_chars_mask(r)) atomicOr(err, FLEET_ERRBIT_BASE64);
  if (as_codes) {
    int32_t* o = (int32_t*)out + row_id * vpitch + 3 * g;
    for (int e = 0; e < r; ++e) o[e] = codes[e];
  } else {
    float* o = (float*)out + row_id * vpitch + 3 * g;
    for (int e = 0; e < r; ++e) o[e] = dec(codes[e]);
  }
}

// ----------------------------------------------------------------------------
// Per-op JNI replacements on equal-length Base64 vectors.
// op 0: x*a (scalarMulNative), 1: a+b (addNative), 2: a-b (subtractNative)
__global__ void __launch_bounds__(256) k_elementwise(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                                                     int op, double s, int64_t n, uint8_t* __restrict__ out,
                                                     int64_t groups, int* __restrict__ err) {
  __shared__ B64Tables tab;
  b64_tables_init(&tab);
  __syncthreads();
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= groups) return;
  const int r = (int)min<int64_t>(3, n - 3 * g);
  int32_t ca[3], cb[3] = {0, 0, 0};
  uint32_t bad = b64_decode_group(*reinterpret_cast<const uint4*>(a + 16 * g), &tab, ca);
  if (op != 0) bad |= b64_decode_group(*reinterpret_cast<const uint4*>(b + 16 * g), &tab, cb);
  if (bad & needed_chars_mask(r)) atomicOr(err, FLEET_ERRBIT_BASE64);
  int32_t o[3];
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    float x = dec(ca[e]);
    float res;
    if (op == 0) res = (float)((double)x * s);
    else if (op == 1) res = x + dec(cb[e]);
    else res = x - dec(cb[e]);
    o[e] = e < r ? enc(res) : 0;
  }
  *reinterpret_cast<uint4*>(out + 16 * g) = pad_group(b64_encode_group(o, &tab), r);
}

// getNorm: per-group (double)(x*x) partial sums; the host finishes the sum.
__global__ void __launch_bounds__(256) k_norm_partials(const uint8_t* __restrict__ a, int64_t n,
                                                       double* __restrict__ partials, int64_t groups,
                                                       int* __restrict__ err) {
  __shared__ B64Tables tab;
  __shared__ double red[256];
  b64_tables_init(&tab);
  __syncthreads();
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double s = 0.0;
  if (g < groups) {
    const int r = (int)min<int64_t>(3, n - 3 * g);
    int32_t ca[3];
    uint32_t bad = b64_decode_group(*reinterpret_cast<const uint4*>(a + 16 * g), &tab, ca);
    if (bad & needed_chars_mask(r)) atomicOr(err, FLEET_ERRBIT_BASE64);
    for (int e = 0; e < r; ++e) {
      float x = dec(ca[e]);
      float sq = x * x;
      s += (double)sq;
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) partials[blockIdx.x] = red[0];
}

// read the code at value position p of a Base64 vector
__device__ __forceinline__ int32_t code_at(const uint8_t* text, int64_t p, const B64Tables* tab, uint32_t* bad) {
  int32_t cc[3];
  uint32_t b = b64_decode_group(*reinterpret_cast<const uint4*>(text + 16 * (p / 3)), tab, cc);
  int e = (int)(p % 3);
  const uint32_t carry[3] = {0x003fu, 0x07e0u, 0xfc00u};  // chars carrying bytes 4e..4e+3
  *bad |= b & carry[e];
  return cc[e];
}

// getFlatGradient: flat[i] = enc(dec(upload[pos(i)])), pos skips header slots
__global__ void __launch_bounds__(256) k_flat(const uint8_t* __restrict__ up, const int32_t* __restrict__ hdr,
                                              int n_hdr, int64_t n_flat, uint8_t* __restrict__ out,
                                              int64_t groups, int* __restrict__ err) {
  __shared__ B64Tables tab;
  b64_tables_init(&tab);
  __syncthreads();
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= groups) return;
  const int r = (int)min<int64_t>(3, n_flat - 3 * g);
  int32_t o[3] = {0, 0, 0};
  uint32_t bad = 0;
  for (int e = 0; e < r; ++e) {
    int64_t pos = 3 * g + e;
    for (int h = 0; h < n_hdr; ++h)
      if (hdr[h] <= pos) ++pos;
    o[e] = enc(dec(code_at(up, pos, &tab, &bad)));
  }
  if (bad) atomicOr(err, FLEET_ERRBIT_BASE64);
  *reinterpret_cast<uint4*>(out + 16 * g) = pad_group(b64_encode_group(o, &tab), r);
}

// mergeFlatGradient: header slots from g, payload slots from flat, all re-encoded
__global__ void __launch_bounds__(256) k_merge(const uint8_t* __restrict__ up, const uint8_t* __restrict__ flat,
                                               const int32_t* __restrict__ hdr, int n_hdr, int64_t walk_end,
                                               int64_t n_up,
                                               uint8_t* __restrict__ out, int64_t groups, int* __restrict__ err) {
  __shared__ B64Tables tab;
  b64_tables_init(&tab);
  __syncthreads();
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= groups) return;
  const int r = (int)min<int64_t>(3, n_up - 3 * g);
  int32_t o[3] = {0, 0, 0};
  uint32_t bad = 0;
  for (int e = 0; e < r; ++e) {
    const int64_t p = 3 * g + e;
    int before = 0;
    bool is_h = false;
    for (int h = 0; h < n_hdr; ++h) {
      if (hdr[h] < p) ++before;
      if (hdr[h] == p) is_h = true;
    }
    if (p >= walk_end) is_h = true;  // outside the layout walk: kept from g
    int32_t c = is_h ? code_at(up, p, &tab, &bad) : code_at(flat, p - before, &tab, &bad);
    o[e] = enc(dec(c));
  }
  if (bad) atomicOr(err, FLEET_ERRBIT_BASE64);
  *reinterpret_cast<uint4*>(out + 16 * g) = pad_group(b64_encode_group(o, &tab), r);
}

// Kardam bookkeeping of CppNNUpdater.update (Server/src/main/java/apps/cppNN/
// CppNNUpdater.java:463-481) for M picked uploads at once:
//   pickedGrad_c = getFlatGradient(upload_c).scalarMultiply(dampen_c)
//   g_c          = pickedGrad_c.scalarMultiply(lr)            -> text out (flat layout)
//   ||g_c||, ||g_c.subtract(prev_c)||                           (Kardam.setGrad, Kardam.java:48-62)
// per flat value i (pos(i) skips the header slots, k_flat):
//   y = Q(dec(code)), p = Q(f32(f64(y) d)), g = enc(f32(f64(p) lr)), G = dec(g),
//   D = dec(enc(G - dec(prev_i))); partial sums of (double)(G*G), (double)(D*D)
// (getNorm, cppNN_backend.cpp:779-795: float products summed in double) per
// block and client; the host adds the partials in index order. Exact general
// codec throughout (side work: once per picked upload, only under staleness
// simulation in the reference).
__global__ void __launch_bounds__(256) k_kardam_grads(const uint8_t* __restrict__ uploads, size_t pitch,
                                                      const int32_t* __restrict__ hdr, int n_hdr, int64_t n_flat,
                                                      const double* __restrict__ dampen, double lr,
                                                      const uint8_t* __restrict__ prev, size_t prev_pitch,
                                                      const uint8_t* __restrict__ has_prev,
                                                      uint8_t* __restrict__ g_out, size_t g_pitch,
                                                      double* __restrict__ partials, int64_t groups,
                                                      int* __restrict__ err) {
  __shared__ B64Tables tab;
  __shared__ double red[2][256];
  b64_tables_init(&tab);
  __syncthreads();
  const int c = blockIdx.y;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint8_t* up = uploads + (size_t)c * pitch;
  const bool hp = prev && has_prev[c];
  const double d = dampen[c];
  double sg = 0.0, sd = 0.0;
  if (g < groups) {
    const int r = (int)min<int64_t>(3, n_flat - 3 * g);
    int32_t o[3] = {0, 0, 0};
    uint32_t bad = 0;
    for (int e = 0; e < r; ++e) {
      const int64_t i = 3 * g + e;
      int64_t pos = i;
      for (int h = 0; h < n_hdr; ++h)
        if (hdr[h] <= pos) ++pos;
      const float y = q(dec(code_at(up, pos, &tab, &bad)));
      const float pv = q((float)((double)y * d));
      o[e] = enc((float)((double)pv * lr));
      const float G = dec(o[e]);
      sg += (double)(G * G);
      if (hp) {
        const float D = q(G - dec(code_at(prev + (size_t)c * prev_pitch, i, &tab, &bad)));
        sd += (double)(D * D);
      }
    }
    if (bad) atomicOr(err, FLEET_ERRBIT_BASE64);
    *reinterpret_cast<uint4*>(g_out + (size_t)c * g_pitch + 16 * g) = pad_group(b64_encode_group(o, &tab), r);
  }
  red[0][threadIdx.x] = sg;
  red[1][threadIdx.x] = sd;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partials[(size_t)c * 2 * gridDim.x + blockIdx.x] = red[0][0];
    partials[(size_t)c * 2 * gridDim.x + gridDim.x + blockIdx.x] = red[1][0];
  }
}

// network::flatGrad's header walk (network.h:1206-1223), one thread.
// out[0] = status (0 ok, 1 malformed), out[1] = n_headers, out[2] = walk end,
// out[4..] = header positions.
__global__ void k_layout_parse(const uint8_t* __restrict__ up, int64_t n, int cap, int32_t* __restrict__ out) {
  __shared__ B64Tables tab;
  b64_tables_init<64>(&tab);
  __syncthreads();
  if (threadIdx.x != 0) return;
  int64_t idx = 0;
  int nh = 0;
  uint32_t bad = 0;
  int status = 0;
  for (int part = 0; part < 2 && !status; ++part) {
    if (idx >= n || nh >= cap) { status = 1; break; }
    out[4 + nh++] = (int32_t)idx;
    int cnt = cvtt(dec(code_at(up, idx++, &tab, &bad)));
    for (int i = 0; i < cnt; ++i) {
      if (idx >= n || nh >= cap) { status = 1; break; }
      out[4 + nh++] = (int32_t)idx;
      int size = cvtt(dec(code_at(up, idx++, &tab, &bad)));
      if (size < 0 || idx + size > n) { status = 1; break; }
      idx += size;
    }
  }
  if (bad) status = 1;
  out[0] = status;
  out[1] = nh;
  out[2] = (int32_t)idx;
  out[3] = 0;
}

// synthetic buckets + layout header values
// elem0: the first element of a column window of a larger problem (its values are
// that problem's columns: the counter is the global element index)
__global__ void __launch_bounds__(256) k_synth(uint64_t seed, int client0, int64_t elem0, int64_t n_up,
                                               float* __restrict__ out, size_t vpitch) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (i < n_up) out[(size_t)c * vpitch + i] = synth_value(seed, (uint32_t)(client0 + c), (uint32_t)(elem0 + i));
}

__global__ void k_synth_headers(float* __restrict__ out, size_t vpitch, const int32_t* __restrict__ hpos,
                                const float* __restrict__ hval, int n_hdr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_hdr) out[(size_t)blockIdx.y * vpitch + hpos[i]] = hval[i];
}

// ----------------------------------------------------------------------------
// descentNative's model step: Server/src/main/c++/
// cppNN_backend.cpp:336-352 -> network::descent(vector), commonLib/cppNN/
// network.h:1185-1202,1334-1353. Per segment: a weight block (kind 0,
// sgd::increment_w, solver.h:88-94: w -= lr*(dW + 0*w)) or a fully-connected
// layer's bias block (kind 1, update_bias, layer.h:241-243: b -= db*lr), each
// op one fp32 rounding as in the reference's SSE build (no contraction).
// NaN results as the reference's x86 SSE build produces them (the GPU's own
// canonical NaN is 0x7FC00000): a NaN operand propagates quieted, the
// instruction's first operand winning; an invalid operation gives 0xFFC00000.
__device__ __forceinline__ float x86_nan(float a, float b, float r) {
  if (r == r) return r;
  if (a != a) return u2f(f2u(a) | 0x00400000u);
  if (b != b) return u2f(f2u(b) | 0x00400000u);
  return u2f(0xFFC00000u);
}

__global__ void __launch_bounds__(256) k_descent(float* __restrict__ weights, float* __restrict__ fc_bias,
                                                 const float* __restrict__ grad, DescentSegs segs, float lr) {
  const int sg = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= segs.len[sg]) return;
  const float g = grad[segs.grad_off[sg] + i];
  if (segs.kind[sg] == 0) {
    float* w = weights + segs.model_off[sg] + i;
    const float x = *w;
    const float t = x86_nan(0.0f, x, 0.0f * x);  // w_decay * w
    const float u = x86_nan(t, g, t + g);        // dW + t (the product is the x86 first operand)
    const float v = x86_nan(lr, u, lr * u);
    *w = x86_nan(x, v, x - v);
  } else {
    float* b = fc_bias + segs.model_off[sg] + i;
    const float v = x86_nan(g, lr, g * lr);
    *b = x86_nan(*b, v, *b - v);
  }
}

hipError_t launch_descent(float* weights, float* fc_bias, const float* grad, const DescentSegs& segs, float lr,
                          hipStream_t s) {
  int64_t mx = 0;
  for (int k = 0; k < segs.n; ++k) mx = std::max(mx, segs.len[k]);
  if (segs.n == 0 || mx == 0) return hipSuccess;
  hipLaunchKernelGGL(k_descent, dim3((unsigned)((mx + 255) / 256), (unsigned)segs.n), dim3(256), 0, s, weights,
                     fc_bias, grad, segs, lr);
  return hipGetLastError();
}

// ---------------------------------------------------------------- launch plan

// Launch-plan overrides (kernels.h): process-wide, set by fleet_set_plan or, once at
// first use, from FLEET_EXPERIMENTS (the same spec) -- the only environment read of
// the launch path. Validated: an unknown key or value rejects the whole spec.
namespace {
std::mutex g_plan_mu;
PlanOverrides g_plan;
std::string g_plan_spec;  // normalised, "" = the measured default plan
std::once_flag g_plan_env_once;

bool parse_int(const std::string& v, int lo, int hi, int* out) {
  if (v.empty() || v.size() > 6 || v.find_first_not_of("0123456789") != std::string::npos) return false;
  const int x = atoi(v.c_str());
  if (x < lo || x > hi) return false;
  *out = x;
  return true;
}

int parse_plan(const char* spec, PlanOverrides* o, std::string* norm, std::string* err) {
  *o = PlanOverrides{};
  norm->clear();
  std::string s = spec ? spec : "";
  for (char& ch : s)
    if (ch == ';' || ch == ' ') ch = ',';
  size_t p = 0;
  while (p <= s.size()) {
    size_t q = s.find(',', p);
    if (q == std::string::npos) q = s.size();
    const std::string item = s.substr(p, q - p);
    p = q + 1;
    if (item.empty()) continue;
    const size_t eq = item.find('=');
    if (eq == std::string::npos) {
      *err = "plan item '" + item + "' is not key=value";
      return -1;
    }
    const std::string k = item.substr(0, eq), v = item.substr(eq + 1);
    bool ok = true;
    if (k == "update") {
      if (v == "auto") o->update = 0;
      else if (v == "stream") o->update = 1;
      else if (v == "tiled") o->update = 2;
      else if (v == "pipe") o->update = 3;
      else ok = false;
    } else if (k == "grid") {
      if (v == "auto") o->grid = 0;
      else if (v == "plain") o->grid = 1;
      else if (v == "lanes") o->grid = 2;
      else if (v == "balanced") o->grid = 3;
      else ok = false;
    } else if (k == "tile") {
      if (v == "auto") o->tile = 0;
      else if (v == "classic") o->tile = 1;
      else if (v == "flat") o->tile = 2;
      else if (v == "weave6") o->tile = 6;
      else if (v == "weave8") o->tile = 8;
      else ok = false;
    } else if (k == "tile_enc_prio") {
      if (v == "auto") o->tile_enc_prio = -1;
      else ok = parse_int(v, 0, 3, &o->tile_enc_prio);
    } else if (k == "flat_w2") {
      if (v == "auto") o->flat_w2 = 0;
      else ok = parse_int(v, 1, kFlatTG, &o->flat_w2);
    } else if (k == "tile_enc_rows") {
      ok = parse_int(v, 1, 4096, &o->tile_enc_rows);
    } else if (k == "fused") {
      if (v == "on") o->fused = 1;
      else if (v == "off") o->fused = 0;
      else ok = false;
    } else if (k == "stage_threads") {
      ok = parse_int(v, 1, 64, &o->stage_threads);
    } else if (k == "stage_pieces") {
      ok = parse_int(v, 1, 64, &o->stage_pieces);
    } else {
      *err = "unknown plan key '" + k + "' (update, grid, tile, flat_w2, tile_enc_prio, tile_enc_rows, fused, "
             "stage_threads, "
             "stage_pieces)";
      return -1;
    }
    if (!ok) {
      *err = "bad value '" + v + "' for plan key '" + k + "'";
      return -1;
    }
    if (!norm->empty()) *norm += ",";
    *norm += k + "=" + v;
  }
  return 0;
}

void plan_env_init() {
  std::call_once(g_plan_env_once, [] {
    const char* e = getenv("FLEET_EXPERIMENTS");
    if (!e || !*e) return;
    PlanOverrides o;
    std::string norm, err;
    if (parse_plan(e, &o, &norm, &err) != 0) {
      fprintf(stderr, "[fleet] FLEET_EXPERIMENTS rejected (%s): the default launch plan is used\n", err.c_str());
      return;
    }
    std::lock_guard<std::mutex> lk(g_plan_mu);
    g_plan = o;
    g_plan_spec = norm;
  });
}
}  // namespace

#ifdef FLEET_TRACE
hipError_t set_trace_buffer(void* p) {
  unsigned long long* q = static_cast<unsigned long long*>(p);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_fleet_trace), &q, sizeof(q));
}
#endif

PlanOverrides plan_overrides() {
  plan_env_init();
  std::lock_guard<std::mutex> lk(g_plan_mu);
  return g_plan;
}

int set_plan_overrides(const char* spec, std::string* err) {
  plan_env_init();
  PlanOverrides o;
  std::string norm;
  if (parse_plan(spec, &o, &norm, err) != 0) return -1;
  std::lock_guard<std::mutex> lk(g_plan_mu);
  g_plan = o;
  g_plan_spec = norm;
  return 0;
}

std::string plan_spec() {
  plan_env_init();
  std::lock_guard<std::mutex> lk(g_plan_mu);
  return g_plan_spec;
}

static inline unsigned blocks_for(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

// The stream kernels address a lane's group by a 32-bit byte offset in its row (buffer
// loads from the row's uniform address): one client's text below 2 GiB (a Java byte[]
// holds less anyway).
static inline bool row_fits(int64_t n_up) { return 16 * ((n_up + 2) / 3) + 16 < (1LL << 31); }

// SIMDs of the current device (4 per CU), cached per device (a process may drive
// several GPUs, one launching thread each; concurrent first calls store the same value)
static int device_simds() {
  static std::atomic<int> simds[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    dev = 0;
  }
  const bool cached = dev >= 0 && dev < 64;
  int v = cached ? simds[dev].load(std::memory_order_relaxed) : 0;
  if (!v) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
      (void)hipGetLastError();
      fprintf(stderr, "[fleet] no CU count for device %d: planning for 256 CUs\n", dev);
      cus = 256;
    }
    v = 4 * cus;
    if (cached) simds[dev].store(v, std::memory_order_relaxed);
  }
  return v;
}

// k_update_flat's grid for `groups` groups: r whole rounds of kFlatTG-group tiles over the
// CUs, the rest in tiles of w2 = kFlatTG, 1/2 or 1/4 of it dealt round robin after them.
// Picks the w2 that leaves the most loaded CU the fewest groups (r * kFlatTG +
// ceil(n2 / CUs) * w2) with every tile resident at once (r + ceil(n2 / CUs) <= kFlatSlots),
// the wider on a tie; more than one round of the widest tiles when the groups do not fit
// one. (On the N = 8 window, 2.7 tiles per CU, the 16-group tiles' extra serial chains
// also hide latency: the update 156-159 us on one width, 143 us with them; r05.)
static FlatGrid flat_grid(int64_t groups, const PlanOverrides& o, bool fused) {
  const int64_t cus = device_simds() / 4, w1 = kFlatTG;
  const int64_t r = groups / (w1 * cus);
  const int64_t rest = groups - r * w1 * cus;
  int best = -1;
  int64_t best_load = INT64_MAX;
  // the fused step: no quarter-width tiles (their extra blocks take the slots the encode's
  // blocks would start in) and half-width ones on a tie (the N = 8 window, 192 groups per
  // CU either way: 175.4 us with quarter-width, 173.1 / 176.6 with half-width against
  // 182.3 with full-width narrow tiles; r05 same-process A/Bs)
  for (int k = 0; k < (fused ? 2 : 3); ++k) {
    const int w2 = o.flat_w2 ? o.flat_w2 : kFlatTG >> k;  // a forced width: that one, even past a round
    const int64_t n2 = (rest + w2 - 1) / w2, per_cu = (n2 + cus - 1) / cus;
    if (r + per_cu > kFlatSlots && !o.flat_w2) continue;
    const int64_t load = r * w1 + per_cu * w2;
    if (load < best_load || (fused && load == best_load)) {  // the fused step: the narrower on a tie
      best_load = load;
      best = w2;
    }
  }
  if (best < 0) best = kFlatTG;  // more than a round: the widest tiles throughout
  const int64_t n2 = (rest + best - 1) / best;
  return FlatGrid{(int)(r * cus), (int)(r * cus + n2), kFlatTG, best};
}

// The aggregation's launch plan for a bucket (or window) of `groups` 3-value groups.
//   stream -- k_update_mixed<256> (fused: k_update_encode<256>): a lane walks its group
//             down all M rows, whole rounds group-per-lane and the rest a value per lane;
//   tiled  -- the one-width 64-group tiles of k_update_tiled_encode<64> (the fused step);
//   flat   -- k_update_flat: two-phase tiles of a runtime width, one balanced round;
//   woven  -- k_update_weave<8> / k_update_weave_encode<8 | 6>: both phases in one barrier
//             interval (small windows, latency-bound);
//   pipe   -- k_update_pipe<16, 1, 5, 0>: 16-group tiles, 4 producer waves + one consumer
//             wave (MNIST-size buckets: the serial chain is the critical path).
// Default ranges (DESIGN.md §4, 256 CUs): the update alone -- stream from 131,072 groups,
// flat above 49,152 (three 64-group tiles per CU), woven 8-wave from 24 k, pipe below;
// the fused step -- stream from 131,072, tiled from 65,536, flat from 40 k, woven 6-wave
// from 32 k, woven 8-wave from 14 k, pipe below; Kardam's side outputs -- stream from
// 131,072, flat from 32 k, pipe below.
struct UpdatePlan {
  int kind;       // 0 stream, 1 tiled, 2 pipe, 3 woven tiles (k_update_weave<nw>), 4 flat tiles
  int nA;         // stream: blocks of group-per-lane waves (the rest a value per lane)
  int64_t blocks; // stream / tiled / pipe grid
  int nw;         // woven tiles: waves per block (6 or 8)
  FlatGrid fg;    // flat tiles
};
static UpdatePlan plan_update(int64_t groups, const PlanOverrides& o, bool fused = false) {
  UpdatePlan p{0, 0, 0, 0, FlatGrid{0, 0, kFlatTG, kFlatTG}};
  if (o.update == 1) p.kind = 0;
  else if (o.update == 2) p.kind = 1;
  else if (o.update == 3) p.kind = 2;
  else {
    // the tiles from 32 k groups; the update alone (auto tiles) from 24 k, where its woven
    // tiles already beat the pipelined ones (cifar10_256's N = 4 window, 26 k groups: 100.8
    // against 141.3 us; 20.9 k: 106.9 / 109.4; 18.4 k and below the pipelined tiles win;
    // r05, profiles/r05/ab_weave_vs_pipe.txt)
    const int64_t tile_min = (!fused && o.tile == 0) ? 24LL * 1024 : 32LL * 1024;
    p.kind = groups >= 256LL * 4 * 2 * 64 ? 0 : groups >= tile_min ? 1 : 2;
  }
  if (p.kind == 1 && o.tile >= 3) {  // the woven tiles (one width)
    p.kind = 3;
    p.nw = o.tile;
  }
  // the flat tiles for the update alone; the fused step keeps the one-width 64-group tiles
  // from 64 k groups, whose free block slots start the encode's blocks beside them
  // (same-process A/B, r05: the update alone 276 -> 261 us on cifar10_256, 241 -> 227 on
  // the N = 4 window, 1133 -> 1099 on cifar100_1024; the fused step 380 against 392 on
  // cifar10_256, but 170.6 against 181.4 us on the N = 8 window)
  // the update alone up to three 64-group tiles per CU (the N = 8 window: 2.7, latency-
  // bound): the woven 8-wave tiles, whose serial steps run between the producers' stages,
  // one round of them at most (synth1m_256's N = 8 window 125.3 against 143.8 us for the
  // flat tiles, cifar10_256's N = 3 122.2 against 146.2; at 3.2 and 3.6 tiles per CU they
  // lose, 190-194 against 161-165 us; r05 same-process A/B, profiles/r05/ab_weave_small.txt)
  if (p.kind == 1 && o.tile == 0 && !fused && groups <= 3LL * 64 * (device_simds() / 4)) {
    p.kind = 3;
    p.nw = 8;
  }
  // the fused step on small windows: the woven tiles with the encode's blocks after them
  // from 14 k to 40 k groups (8 waves up to 32 k, 6 above), the pipelined tiles below
  // (cifar10_256's N = 5 window 134.7 -> 107.5 us, cifar100_1024's N = 4 672.4 -> 463.0,
  // cifar10_256's N = 3 160.2 -> 147.6 against the flat tiles; 13 k groups: 90.0 pipelined
  // against 94.1; r05 same-process A/B, profiles/r05/ab_weave_fused.txt)
  if (fused && o.update == 0 && o.tile == 0 && groups >= 14LL * 1024 && groups < 40LL * 1024) {
    p.kind = 3;
    p.nw = groups < 32LL * 1024 ? 8 : 6;
  }
  if (p.kind == 1 && (o.tile == 2 || (o.tile == 0 && (!fused || groups < 65536)))) p.kind = 4;
  if (p.kind == 2) {
    p.blocks = (groups + 15) / 16;
  } else if (p.kind == 4) {
    p.fg = flat_grid(groups, o, fused);
    p.blocks = p.fg.nU;
  } else if (p.kind == 3) {
    p.blocks = (groups + kWeaveTG - 1) / kWeaveTG;
  } else if (p.kind == 1) {  // one width (the fused step's tiles; the update alone under tile=classic)
    p.blocks = (groups + 63) / 64;
  } else {
    const int64_t plain = (groups + 255) / 256;
    if (o.grid == 1) {
      p.nA = (int)plain;
    } else if (o.grid == 2) {
      p.nA = 0;
    } else {  // whole rounds of group-per-lane waves (a multiple of one wave per SIMD)
      const int simds = device_simds();
      const int64_t waves = (groups + 63) / 64;
      p.nA = waves < simds ? (int)plain : (int)(waves / simds * simds * 64 / 256);
    }
    // the value-per-lane blocks take what the group-per-lane rounds leave (none when
    // the plain grid covers every group: its last block is ragged)
    const int64_t rest = groups - (int64_t)p.nA * 256;
    p.blocks = p.nA + (rest > 0 ? (rest + 83) / 84 : 0);
  }
  return p;
}

std::string update_kernel_name(int64_t groups) {
  const UpdatePlan p = plan_update(groups, plan_overrides());
  char buf[64];
  if (p.kind == 0) snprintf(buf, sizeof buf, "k_update_mixed<256, false>");
  else if (p.kind == 2) snprintf(buf, sizeof buf, "k_update_pipe<16, 1, 5, 0, false>");
  else if (p.kind == 3) snprintf(buf, sizeof buf, "k_update_weave<%d>", p.nw);
  else if (p.kind == 4) snprintf(buf, sizeof buf, "k_update_flat");
  else snprintf(buf, sizeof buf, "k_update_tiled_encode<64>");  // its tiles alone, no encode blocks
  return buf;
}

void update_plan_grid(int64_t groups, int* kind, int64_t* blocks, int64_t* n_a, int64_t* n_w, int64_t* n_n) {
  const UpdatePlan p = plan_update(groups, plan_overrides());
  *kind = p.kind;
  *blocks = p.blocks;
  *n_a = p.nA;
  *n_w = -1;  // one width: blocks = ceil(groups / 64)
  *n_n = 0;
  if (p.kind == 4) {  // flat: n_w tiles of kFlatTG groups, n_n tiles of n_a groups
    *n_a = p.fg.w2;
    *n_w = p.fg.nW;
    *n_n = p.fg.nU - p.fg.nW;
  }
}

std::string update_encode_kernel_name(int64_t groups) {
  const PlanOverrides o = plan_overrides();
  const UpdatePlan p = plan_update(groups, o, true);
  if (!o.fused) return update_kernel_name(groups) + " + k_encode_f32";
  if (p.kind == 0) return "k_update_encode<256>";
  if (p.kind == 1) return "k_update_tiled_encode<64>";
  if (p.kind == 3) return "k_update_weave_encode<" + std::to_string(p.nw) + ">";
  if (p.kind == 4) return "k_update_flat";
  return "k_update_pipe<16, 1, 5, 0, false> (with the encode's blocks)";
}

// The classic one-width tiles alone (tile=classic for the update without the encode):
// k_update_tiled_encode<64> with no encode blocks
static void launch_tiled(const UpdatePlan& p, const uint8_t* uploads, size_t pitch, int M, const double* d_dampen,
                         double inv_avg, int64_t n_up, int64_t g_begin, int64_t g_end, const int32_t* d_hdr_block,
                         uint8_t* merged, float* merged_f32, int* d_err, hipStream_t s) {
  hipLaunchKernelGGL((k_update_tiled_encode<64>), dim3((unsigned)p.blocks), dim3(256), 0, s, uploads, pitch, M, d_dampen,
                     inv_avg, n_up, g_begin, g_end, d_hdr_block, merged, merged_f32, d_err, (int)p.blocks, EncodeJob{});
}

// k_update_weave<nw> (nw = 6 or 8 waves per block)
static void launch_weave(int nw, unsigned blocks, hipStream_t s, const uint8_t* uploads, size_t pitch, int M,
                         const double* d_dampen, double inv_avg, int64_t n_up, int64_t g_begin, int64_t g_end,
                         const int32_t* d_hdr_block, uint8_t* merged, float* merged_f32, int* d_err) {
#define FLEET_WEAVE_LAUNCH(NWV)                                                                                   \
  hipLaunchKernelGGL(k_update_weave<NWV>, dim3(blocks), dim3(64 * NWV), 0, s, uploads, pitch, M, d_dampen, inv_avg, \
                     n_up, g_begin, g_end, d_hdr_block, merged, merged_f32, d_err)
  if (nw == 6) FLEET_WEAVE_LAUNCH(6);
  else FLEET_WEAVE_LAUNCH(8);
#undef FLEET_WEAVE_LAUNCH
}

hipError_t launch_update(const uint8_t* uploads, size_t pitch, int M, const double* d_dampen, double inv_avg,
                         int64_t n_up, int64_t g_begin, int64_t g_end, const int32_t* d_hdr_block,
                         uint8_t* merged, float* merged_f32, int* d_err, hipStream_t s) {
  if (!row_fits(n_up)) return hipErrorInvalidValue;
  if (g_end <= g_begin) return hipSuccess;
  const UpdatePlan p = plan_update(g_end - g_begin, plan_overrides());
  if (p.kind == 2)
    hipLaunchKernelGGL((k_update_pipe<16, 1, 5, 0>), dim3((unsigned)p.blocks), dim3(64 * 5), 0, s, uploads, pitch, M,
                       d_dampen, inv_avg, n_up, g_begin, g_end, d_hdr_block, merged, merged_f32, d_err, INT32_MAX,
                       EncodeJob{});
  else if (p.kind == 1)
    launch_tiled(p, uploads, pitch, M, d_dampen, inv_avg, n_up, g_begin, g_end, d_hdr_block, merged, merged_f32, d_err,
                 s);
  else if (p.kind == 3)
    launch_weave(p.nw, (unsigned)p.blocks, s, uploads, pitch, M, d_dampen, inv_avg, n_up, g_begin, g_end, d_hdr_block,
                 merged, merged_f32, d_err);
  else if (p.kind == 4)
    hipLaunchKernelGGL(k_update_flat, dim3((unsigned)p.blocks), dim3(256), 0, s, uploads, pitch, M, d_dampen,
                       inv_avg, n_up, g_begin, g_end, d_hdr_block, merged, merged_f32, d_err, p.fg, EncodeJob{});
  else
    hipLaunchKernelGGL((k_update_mixed<256, false>), dim3((unsigned)p.blocks), dim3(256), 0, s, uploads, pitch, M,
                       d_dampen, inv_avg, n_up, g_begin, g_end, d_hdr_block, merged, merged_f32, d_err, p.nA,
                       KardamOut{});
  return hipGetLastError();
}

// per client: the (client, wave or tile) partials of the update summed in a fixed
// order. The reduce is pure latency (a few hundred to a few thousand 16-byte pairs
// per client), so a lane issues all of its U loads before the first add (one HBM
// round trip, not one per 8 loads), the pairs fold in a fixed tree, the wave by DPP
// lane moves (group_sum_f64: no LDS crossbar round trips), and the block's waves meet
// in LDS. One wave per client up to 2,048 partials (the tiles), four beyond (the
// stream grid's thousands of waves); past U * NT a strided loop takes the rest.
template <int NT, int U>
__global__ void __launch_bounds__(NT) k_kardam_reduce(const double* __restrict__ partials, int64_t n_waves,
                                                      double* __restrict__ norms) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int c = blockIdx.x;
  const d2* p = reinterpret_cast<const d2*>(partials) + (size_t)c * n_waves;
  d2 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t w = threadIdx.x + (int64_t)u * NT;
    v[u] = w < n_waves ? p[w] : d2{0.0, 0.0};
  }
  for (int64_t w = threadIdx.x + (int64_t)U * NT; w < n_waves; w += NT) v[0] += p[w];
#pragma unroll
  for (int h = U / 2; h > 0; h /= 2)
#pragma unroll
    for (int u = 0; u < h; ++u) v[u] += v[u + h];
  const double a = group_sum_f64<64>(v[0].x), b = group_sum_f64<64>(v[0].y);  // valid in lane 63
  if constexpr (NT == 64) {
    if (threadIdx.x == 63) {
      norms[2 * c] = a;
      norms[2 * c + 1] = b;
    }
  } else {
    __shared__ double red[2][NT / 64];
    if ((threadIdx.x & 63) == 63) {
      red[0][threadIdx.x / 64] = a;
      red[1][threadIdx.x / 64] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double sa = 0.0, sb = 0.0;
      for (int i = 0; i < NT / 64; ++i) {
        sa += red[0][i];
        sb += red[1][i];
      }
      norms[2 * c] = sa;
      norms[2 * c + 1] = sb;
    }
  }
}

// waves per block of the Kardam pipelined form (one consumer, the rest producers): the
// side outputs double the producers' work, and 8 producer waves keep the consumer fed
// where 4 do not (mnist64 under rocprof, r06 call a10: 27.3 us with 4 producer waves,
// 24.4 with 8, 28.3 with 10, 43.2 with 12; the plain update 16.1 us)
#ifndef FLEET_KD_NW
#define FLEET_KD_NW 9
#endif
constexpr int kKdPipeNW = FLEET_KD_NW;

hipError_t launch_update_kardam(const uint8_t* uploads, size_t pitch, int M, const double* d_dampen, double inv_avg,
                                int64_t n_up, int64_t g_begin, int64_t g_end, const int32_t* d_hdr_block,
                                uint8_t* merged, float* merged_f32, int* d_err, const KardamOut& kd, int* n_waves,
                                double* norms, int* norm_parts, int* flag_slots, uint32_t* kd_flags,
                                uint32_t kd_epoch, const PlanOverrides& o, hipStream_t s, uint32_t kd_wait_skew) {
  if (!row_fits(n_up)) return hipErrorInvalidValue;
  const int64_t groups = g_end - g_begin;
  // the update's own launch plan with the side outputs: the pipelined tiles (side outputs
  // from the producers, the reduce blocks in the same launch), the wide tiles (side
  // outputs from the tile producers), or the stream kernel's SIMD-balanced grid
  PlanOverrides ok = o;
  // Kardam's side outputs ride in the flat tiles at every tile size (kardam_items: narrow
  // widths 16 / 32 / 64 only, so another forced width is ignored here), never in the
  // classic or woven ones
  const bool flat_ok = o.flat_w2 == 0 || o.flat_w2 == 16 || o.flat_w2 == 32 || o.flat_w2 == 64;
  ok.tile = 2;
  if (!flat_ok) ok.flat_w2 = 0;
  UpdatePlan p = plan_update(groups, ok);
  if (p.kind == 0 && o.grid == 0) {
    // the stream form on the plain grid unless a grid is asked for: value-per-lane waves
    // pay the per-client wave sums for a third of the values (synth1m_256: 1747 vs
    // 1724 us, r04 call a6)
    p.nA = (int)((groups + 255) / 256);
    p.blocks = p.nA;
  }
  const unsigned blocks = (unsigned)p.blocks;
  // partial slots per client: a wave of the stream grid or a tile
  *n_waves = p.kind == 0 ? (int)blocks * 4 : (int)blocks;
  *flag_slots = p.kind == 2 ? (int)blocks * (kKdPipeNW - 1) : 0;  // the pipelined form's tile flags (per producer wave)
  *norm_parts = 1;                                   // one pair per client
  if (groups <= 0) return hipSuccess;
  if (!kd.partials) return hipErrorInvalidValue;  // sizing call: *n_waves only
  if (p.kind == 2 && !kd_flags) return hipErrorInvalidValue;
  if (p.kind == 2) {  // the tiles, then one reduce block per client
    const KardamReduceJob kr{norms, kd_flags, kd_epoch, kd_wait_skew};
    hipLaunchKernelGGL((k_update_pipe<16, 1, kKdPipeNW, 0, true>), dim3((unsigned)(blocks + (unsigned)M)),
                       dim3(64 * kKdPipeNW), 0, s,
                       uploads, pitch, M, d_dampen, inv_avg, n_up, g_begin, g_end, d_hdr_block, merged, merged_f32,
                       d_err, (int)blocks, EncodeJob{}, kd, kr);
    return hipGetLastError();
  }
  if (p.kind == 4)
    hipLaunchKernelGGL(k_update_flat_kd, dim3(blocks), dim3(256), 0, s, uploads, pitch, M, d_dampen, inv_avg, n_up,
                       g_begin, g_end, d_hdr_block, merged, merged_f32, d_err, p.fg, kd);
  else
    hipLaunchKernelGGL((k_update_mixed<256, true>), dim3(blocks), dim3(256), 0, s, uploads, pitch, M, d_dampen,
                       inv_avg, n_up, g_begin, g_end, d_hdr_block, merged, merged_f32, d_err, p.nA, kd);
  if (*n_waves <= 512)
    hipLaunchKernelGGL((k_kardam_reduce<64, 8>), dim3((unsigned)M), dim3(64), 0, s, kd.partials, (int64_t)*n_waves,
                       norms);
  else if (*n_waves <= 2048)
    hipLaunchKernelGGL((k_kardam_reduce<64, 32>), dim3((unsigned)M), dim3(64), 0, s, kd.partials, (int64_t)*n_waves,
                       norms);
  else
    hipLaunchKernelGGL((k_kardam_reduce<256, 32>), dim3((unsigned)M), dim3(256), 0, s, kd.partials,
                       (int64_t)*n_waves, norms);
  return hipGetLastError();
}

// rows per block of the standalone client encode: about 65,536 blocks in all (a
// lane walks its group down rpb rows, so the LDS table copy is paid once per rpb
// rows). Measured on one box (gpu_encode_rpb.sh (r04 tree), two rows of loads in
// flight): synth1m_256 encodes in 478-480 us at 4-8 rows per block, 483 at 16, 501
// at 2 and 32, 595 at 1; the same access pattern without the codec arithmetic
// (scripts/ubench_stream.hip, 12 B in / 16 B out per lane) runs 452-486 us.
static int encode_rows_per_block(int64_t gx, int rows) {
  return (int)std::min<int64_t>(rows, std::max<int64_t>(1, (gx * rows + 65535) / 65536));
}

// The standalone client encode keeps the VarEntry digit counts: it is HBM-bound, and
// the byte table's 9 KB copy per block costs it more than the VALU it saves (same-box
// A/B on synth1m_256: 460 vs 476 us); k_update_encode, where the VALU is the limit,
// uses the byte table.
hipError_t launch_encode_f32(const float* values, int64_t n, size_t vpitch, int rows, uint8_t* out, size_t pitch,
                             hipStream_t s) {
  if (!row_fits(n)) return hipErrorInvalidValue;
  int64_t groups = (n + 2) / 3;
  if (groups == 0 || rows == 0) return hipSuccess;
  const int64_t gx = blocks_for(groups, 256);
  const int rpb = encode_rows_per_block(gx, rows);
  hipLaunchKernelGGL(k_encode_f32, dim3((unsigned)gx, (unsigned)((rows + rpb - 1) / rpb)), dim3(256), 0, s, values, n,
                     vpitch, out, pitch, groups, rows, rpb);
  return hipGetLastError();
}

// The aggregation of `uploads` and the client encode of `values` into `enc_out`
// (another buffer) in one launch (the pipelined step): k_update_encode on the stream
// grid, k_update_tiled_encode on the wide tiles, the pipelined tiles with the encode's
// blocks after them; plan fused=off runs the two kernels back to back.
hipError_t launch_update_encode(const uint8_t* uploads, size_t pitch, int M, const double* d_dampen, double inv_avg,
                                int64_t n_up, const int32_t* d_hdr_block, uint8_t* merged, float* merged_f32,
                                int* d_err, const float* values, size_t vpitch, uint8_t* enc_out, hipStream_t s) {
  if (!row_fits(n_up)) return hipErrorInvalidValue;
  const int64_t groups = (n_up + 2) / 3;
  const PlanOverrides o = plan_overrides();
  const UpdatePlan p = plan_update(groups, o, true);
  // the tiles' encode blocks at issue priority 3 beside the tiles' ladder (3 -> 0) from
  // 64 k groups, 0 below: cifar10_256 394 -> 380 us, the N = 4 window 319 -> 311,
  // cifar100_1024 1622 -> 1593, the N = 8 window 174.5 -> 178.5 (r05 same-process A/B)
  const int tprio = o.tile_enc_prio >= 0 ? o.tile_enc_prio : groups >= 65536 ? 3 : 0;
  if (groups == 0 || !o.fused) {
    hipError_t e = launch_update(uploads, pitch, M, d_dampen, inv_avg, n_up, 0, groups, d_hdr_block, merged, merged_f32,
                                 d_err, s);
    if (e != hipSuccess) return e;
    return launch_encode_f32(values, n_up, vpitch, M, enc_out, pitch, s);
  }
  if (p.kind == 3) {  // the woven tiles, then the encode's blocks (64 * nw lanes each)
    const int nt = 64 * p.nw;
    const int64_t gx = (groups + nt - 1) / nt;
    // 24 rows per encode block as in the other fused forms (the standalone encode's rule
    // gave these blocks one or two rows each, every block copying the tables for them)
    const int rpb = std::min(M, o.tile_enc_rows > 0 ? o.tile_enc_rows : 24);
    const int64_t nU = p.blocks, nE = gx * ((M + rpb - 1) / rpb);
    const EncodeJob ej{values, n_up, vpitch, enc_out, pitch, groups, gx, M, rpb,
                       o.tile_enc_prio >= 0 ? o.tile_enc_prio : 0};
#define FLEET_WEAVE_ENC_LAUNCH(NWV)                                                                             \
  hipLaunchKernelGGL(k_update_weave_encode<NWV>, dim3((unsigned)(nU + nE)), dim3(64 * NWV), 0, s, uploads, pitch, M, \
                     d_dampen, inv_avg, n_up, (int64_t)0, groups, d_hdr_block, merged, merged_f32, d_err, (int)nU, ej)
    if (p.nw == 6) FLEET_WEAVE_ENC_LAUNCH(6);
    else FLEET_WEAVE_ENC_LAUNCH(8);
#undef FLEET_WEAVE_ENC_LAUNCH
    return hipGetLastError();
  }
  if (p.kind == 4) {  // the flat tiles' round, then the encode's blocks (24 rows each, as below)
    const int64_t gx = blocks_for(groups, 256);
    const int rpb = std::min(M, o.tile_enc_rows > 0 ? o.tile_enc_rows : 24);
    const int64_t nU = p.blocks, nE = gx * ((M + rpb - 1) / rpb);
    const EncodeJob ej{values, n_up, vpitch, enc_out, pitch, groups, gx, M, rpb, tprio};
    hipLaunchKernelGGL(k_update_flat, dim3((unsigned)(nU + nE)), dim3(256), 0, s, uploads, pitch, M, d_dampen,
                       inv_avg, n_up, (int64_t)0, groups, d_hdr_block, merged, merged_f32, d_err, p.fg, ej);
    return hipGetLastError();
  }
  if (p.kind == 1) {  // the wide tiles on one width, then the encode's blocks
    // 24 rows per encode block, as in k_update_encode: each block copies the tile's
    // 14 KB of tables into LDS, so the standalone encode's ~65,536 blocks (2 rows each at
    // CIFAR sizes) spent the step on table copies -- the encode ran mostly after the
    // tiles, 230 us of it on cifar10_256 against 157 us alone (r05 residency trace)
    const int64_t gx = blocks_for(groups, 256);
    const int rpb = std::min(M, o.tile_enc_rows > 0 ? o.tile_enc_rows : 24);
    const int64_t nU = (groups + 63) / 64, nE = gx * ((M + rpb - 1) / rpb);
    const EncodeJob ej{values, n_up, vpitch, enc_out, pitch, groups, gx, M, rpb, tprio};
    hipLaunchKernelGGL((k_update_tiled_encode<64>), dim3((unsigned)(nU + nE)), dim3(256), 0, s, uploads, pitch, M,
                       d_dampen, inv_avg, n_up, (int64_t)0, groups, d_hdr_block, merged, merged_f32, d_err, (int)nU, ej);
    return hipGetLastError();
  }
  if (p.kind == 2) {  // small buckets: the pipelined tiles, the encode's 320-lane blocks after them
    const int64_t gxp = (groups + 319) / 320;
    const int rpb = encode_rows_per_block(gxp, M);
    const EncodeJob ej{values, n_up, vpitch, enc_out, pitch, groups, gxp, M, rpb};
    hipLaunchKernelGGL((k_update_pipe<16, 1, 5, 0>), dim3((unsigned)(p.blocks + gxp * ((M + rpb - 1) / rpb))),
                       dim3(64 * 5), 0, s, uploads, pitch, M, d_dampen, inv_avg, n_up, (int64_t)0, groups, d_hdr_block,
                       merged, merged_f32, d_err, (int)p.blocks, ej);
    return hipGetLastError();
  }
  // the stream grid group-per-lane everywhere: the encode's blocks fill the SIMDs the
  // last round of update waves leaves idle, so the value-per-lane balancing of
  // k_update_mixed only adds instructions here (same-box A/B on synth1m_256: 1172.7 vs
  // 1181.3 us, gpu_fused_ab.sh (r04 tree)). 24 rows per encode block: short blocks that
  // fill the slots the update's waves leave (a lane walks its group down the rows with
  // two loads in flight, so a block of hundreds of rows is a latency-bound straggler);
  // same-box A/B on synth1m_256: 1179 / 1170 us at 6 / 12 rows per block in r03; with
  // the encode's waves at priority 3 (r04) 1130 / 1097-1100 / 1084-1090 us at 6 / 12 /
  // 24, and 48 no better (r04 call a31, a32.sh).
  // (grid=lanes: the update's blocks a value per lane, for experiments on small windows)
  const int64_t gx = blocks_for(groups, 256);
  // Below four waves of group-per-lane update per SIMD (the N = 2 strong window: 2.7) the
  // update alone's SIMD-balanced split -- whole rounds of group-per-lane waves, the rest a
  // value per lane -- also under the encode's blocks (grid=balanced): synth1m_256's N = 2
  // window 635.3 -> 604.3 us, configs[4]'s N = 8 window 11.09 -> 10.05 ms, while the full
  // width (5.3 waves per SIMD) loses with it, 1106.6 -> 1159.8 us; one group-per-lane round
  // fewer loses at N = 2 (624.0 us) (r05 same-process A/B, profiles/r05/ab_fused_balanced.txt)
  const bool lanes = o.grid == 2;
  int nAf = lanes ? 0 : (int)gx, nUf = lanes ? (int)((groups + 83) / 84) : (int)gx;
  const bool balanced = o.grid == 3 || (o.grid == 0 && groups < 4LL * 64 * device_simds());
  if (balanced) {
    PlanOverrides ob = o;
    ob.grid = 0;
    const UpdatePlan pb = plan_update(groups, ob);
    if (pb.kind == 0) {
      nAf = pb.nA;
      nUf = (int)pb.blocks;
    }
  }
  const int rpb = std::min(M, o.tile_enc_rows > 0 ? o.tile_enc_rows : 24);
  const int64_t nE = gx * ((M + rpb - 1) / rpb);
  // the encode's waves at priority 3 over the full width (r04, see k_update_encode), at 0
  // under the balanced split of a small window: there the update waves, 2.7 per SIMD, are
  // the critical path (the N = 2 window 588.9 -> 572.5 us, while the full width loses at 2,
  // 1083.7 -> 1108.4; r05 same-process A/B, profiles/r05/ab_stream_encode_prio.txt)
  const EncodeJob ej{values, n_up, vpitch, enc_out, pitch, groups, gx, M, rpb,
                     o.tile_enc_prio >= 0 ? o.tile_enc_prio : balanced ? 0 : 3};
  hipLaunchKernelGGL((k_update_encode<256>), dim3((unsigned)(nUf + nE)), dim3(256), 0, s, uploads, pitch, M, d_dampen,
                     inv_avg, n_up, (int64_t)0, groups, d_hdr_block, merged, merged_f32, d_err, nAf, nUf, ej);
  return hipGetLastError();
}

hipError_t launch_encode_i32(const int32_t* codes, int64_t n, uint8_t* out, hipStream_t s) {
  int64_t groups = (n + 2) / 3;
  if (groups == 0) return hipSuccess;
  hipLaunchKernelGGL(k_encode_i32, dim3(blocks_for(groups, 256)), dim3(256), 0, s, codes, n, out, groups);
  return hipGetLastError();
}

hipError_t launch_decode(const uint8_t* text, int64_t n, size_t pitch, int rows, void* out, size_t vpitch,
                         int as_codes, int* d_err, hipStream_t s) {
  int64_t groups = (n + 2) / 3;
  if (groups == 0 || rows == 0) return hipSuccess;
  hipLaunchKernelGGL(k_decode, dim3(blocks_for(groups, 256), rows), dim3(256), 0, s, text, n, pitch, out, vpitch,
                     groups, as_codes, d_err);
  return hipGetLastError();
}

hipError_t launch_elementwise(const uint8_t* a, const uint8_t* b, int op, double scale, int64_t n, uint8_t* out,
                              int* d_err, hipStream_t s) {
  int64_t groups = (n + 2) / 3;
  if (groups == 0) return hipSuccess;
  hipLaunchKernelGGL(k_elementwise, dim3(blocks_for(groups, 256)), dim3(256), 0, s, a, b, op, scale, n, out,
                     groups, d_err);
  return hipGetLastError();
}

hipError_t launch_norm_partials(const uint8_t* a, int64_t n, double* partials, int* nblocks, int* d_err,
                                hipStream_t s) {
  int64_t groups = (n + 2) / 3;
  *nblocks = (int)blocks_for(groups, 256);
  if (groups == 0) return hipSuccess;
  hipLaunchKernelGGL(k_norm_partials, dim3(*nblocks), dim3(256), 0, s, a, n, partials, groups, d_err);
  return hipGetLastError();
}

hipError_t launch_kardam_grads(const uint8_t* uploads, size_t pitch, int M, const int32_t* d_hdr, int n_hdr,
                               int64_t n_flat, const double* d_dampen, double lr, const uint8_t* prev,
                               size_t prev_pitch, const uint8_t* d_has_prev, uint8_t* g_out, size_t g_pitch,
                               double* partials, int* nblocks, int* d_err, hipStream_t s) {
  const int64_t groups = (n_flat + 2) / 3;
  *nblocks = (int)blocks_for(groups, 256);
  if (groups == 0 || M == 0) return hipSuccess;
  hipLaunchKernelGGL(k_kardam_grads, dim3((unsigned)*nblocks, (unsigned)M), dim3(256), 0, s, uploads, pitch, d_hdr,
                     n_hdr, n_flat, d_dampen, lr, prev, prev_pitch, d_has_prev, g_out, g_pitch, partials, groups,
                     d_err);
  return hipGetLastError();
}

hipError_t launch_flat(const uint8_t* up, const int32_t* d_hdr, int n_hdr, int64_t n_flat, uint8_t* out,
                       int* d_err, hipStream_t s) {
  int64_t groups = (n_flat + 2) / 3;
  if (groups == 0) return hipSuccess;
  hipLaunchKernelGGL(k_flat, dim3(blocks_for(groups, 256)), dim3(256), 0, s, up, d_hdr, n_hdr, n_flat, out, groups,
                     d_err);
  return hipGetLastError();
}

hipError_t launch_merge(const uint8_t* up, const uint8_t* flat, const int32_t* d_hdr, int n_hdr, int64_t walk_end,
                        int64_t n_up, uint8_t* out, int* d_err, hipStream_t s) {
  int64_t groups = (n_up + 2) / 3;
  if (groups == 0) return hipSuccess;
  hipLaunchKernelGGL(k_merge, dim3(blocks_for(groups, 256)), dim3(256), 0, s, up, flat, d_hdr, n_hdr, walk_end,
                     n_up, out, groups, d_err);
  return hipGetLastError();
}

hipError_t launch_layout_parse(const uint8_t* up, int64_t n, int cap, int32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_layout_parse, dim3(1), dim3(64), 0, s, up, n, cap, out);
  return hipGetLastError();
}

hipError_t launch_synth(uint64_t seed, int client0, int64_t elem0, int rows, int64_t n_up, float* out, size_t vpitch,
                        const int32_t* d_hpos, const float* d_hval, int n_hdr, hipStream_t s) {
  if (rows == 0 || n_up == 0) return hipSuccess;
  hipLaunchKernelGGL(k_synth, dim3(blocks_for(n_up, 256), rows), dim3(256), 0, s, seed, client0, elem0, n_up, out,
                     vpitch);
  if (n_hdr > 0)
    hipLaunchKernelGGL(k_synth_headers, dim3(blocks_for(n_hdr, 256), rows), dim3(256), 0, s, out, vpitch, d_hpos,
                       d_hval, n_hdr);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------
// Self-test: order-independent digests of the device codec arithmetic over
// whole input domains (all 2^32 codes / float bit patterns), compared with
// the oracle's digests (tests/golden/digests.json, tests/native/digest_ref.cpp).
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) k_digest(int fn, unsigned long long* __restrict__ out) {
  __shared__ DigitEntry dig[32];
  __shared__ B64Tables tab;
  __shared__ XlTable xl;
  __shared__ D16Table dtab;
  __shared__ LastDigitTable ldt;
  {
    constexpr DigitEntry init[32] = FLEET_DIGIT_TABLE;
    if (threadIdx.x < 32) dig[threadIdx.x] = init[threadIdx.x];
    b64_tables_init(&tab);
    xl_table_init(&xl);
    d16_table_init(&dtab);
    ld16_table_init(&ldt);
    __syncthreads();
  }
  const VarEntry* var = tab.var;
  const MulEntry* mt = tab.mt;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  uint64_t sum = 0;
  for (uint64_t i = tid; i < (1ull << 32); i += nthreads) {
    const uint32_t u = (uint32_t)i;
    uint32_t o;
    bool use = true;
    switch (fn) {
      case 0: o = f2u(dec((int32_t)u)); break;                       // int2float, all codes
      case 1: o = (uint32_t)enc(u2f(u)); break;                      // float2int, all bit patterns
      case 2: use = (u & 0x7fffffffu) < 0x3f800000u;                 // Q fast path, |x| < 1
              o = use ? f2u(q_fast(u2f(u))) : 0u; break;
      case 3: use = ((int32_t)u % 10) == 0;                          // int2float fast path
              o = use ? f2u(dec_fast((int32_t)u)) : 0u; break;
      case 4: use = u >= 0x0DA24260u && u < 0x7F800000u;             // div10, t >= 1e-30
              o = use ? f2u(div10(u2f(u))) : 0u; break;
      case 5: { f2 v = q_fast2(f2{u2f(u), -u2f(u)});                   // packed Q fast path on (x, -x)
              use = (u & 0x7fffffffu) < 0x3f800000u; o = use ? f2u(v.x) + 3u * f2u(v.y) : 0u; break; }
      case 6: use = q_gen_ok(u2f(u));                                 // variable-length Q, numDigits <= 7
              o = use ? f2u(q_gen(u2f(u), dig)) : 0u; break;
      case 7: o = f2u(dec_gen((int32_t)u)); break;                    // variable-length int2float (total)
      case 8: { const float x = u2f(u);                               // packed variable-length Q on (x, -x/4)
              use = q_gen_ok(x) && q_gen_ok(-0.25f * x);
              const f2 v = q_gen2(f2{x, -0.25f * x}, dig);
              o = use ? f2u(v.x) + 3u * f2u(v.y) : 0u; break; }
      case 9: { const int32_t c = (int32_t)u, c2 = (int32_t)(u * 2654435761u);  // packed int2float
              const f2 v = dec_gen2(c, c2);
              o = f2u(v.x) + 3u * f2u(v.y); break; }
      case 10: use = q_gen_ok(u2f(u));                                // variable-length float2int
               o = use ? (uint32_t)enc_gen(u2f(u), dig) : 0u; break;
      case 11: use = (u & 0x7fffffffu) < 0x3f800000u;                 // float2int fast path, |x| < 1
               o = use ? (uint32_t)enc_fast(u2f(u)) : 0u; break;
      case 12: use = q_gen_ok(u2f(u));                                // select-chain Q (serial accumulation)
               o = use ? f2u(q_lat(u2f(u))) : 0u; break;
      case 13: use = q_gen_ok(u2f(u));                                // multiplier-table Q (same digest as fn 6)
               o = use ? f2u(q_mt(u2f(u), var, mt)) : 0u; break;
      case 14: o = f2u(dec_mt((int32_t)u, mt)); break;                // multiplier-table int2float (as fn 7)
      case 15: use = q_gen_ok(u2f(u));                                // multiplier-table float2int (as fn 10)
               o = use ? (uint32_t)enc_mt(u2f(u), var, mt) : 0u; break;
      case 16: use = (u & 0x7fffffffu) < 0x3f800000u;                 // scalar Q fast path (as fn 2)
               o = use ? f2u(q_fast1(u2f(u))) : 0u; break;
      case 17: { const float x = u2f(u);                              // one-lookup Q on |x| < 1e8 (as fn 6)
               use = q_gen_ok(x);
               o = use ? f2u(__builtin_fabsf(x) < 1e8f ? q_xl(x, xl.x) : q_lat(x)) : 0u; break; }
      case 19: { const float x = u2f(u);                              // byte-table Q of k_update (as fn 6)
               use = q_gen_ok(x);
               uint32_t e = dtab.d16[u >> 19];
               if (e == kD16Cmp) e = d16_fix(x, var);
               o = use ? (e < kD16Out ? f2u(q_d16(x, e, &dtab.st)) : 0xdeadbeefu) : 0u; break; }
      case 20: { const float x = u2f(u);                              // byte-table float2int of the client encode (as fn 10)
               use = q_gen_ok(x);
               uint32_t e = dtab.d16[u >> 19];
               if (e == kD16Cmp) e = d16_fix(x, var);
               o = use ? (e < kD16Out ? (uint32_t)enc_d16(x, e, &dtab.st) : 0xdeadbeefu) : 0u; break; }
      case 21: { const float x = u2f(u);                              // stage C's VarEntry-offset Q (as fn 6)
               use = q_gen_ok(x);
               const uint32_t e = var_d16(u, var);
               o = use ? (e < kD16Out ? f2u(q_d16(x, e, &dtab.st)) : 0xdeadbeefu) : 0u; break; }
      case 23: o = f2u(dec_d16((int32_t)u, ldt.ld16[ld16_index((int32_t)u)], &dtab.st)); break;  // stream int2float (as fn 0)
      case 22: { const float x = u2f(u);                              // strtof("%.6g") of the model-version copy
               use = (u & 0x7f800000u) != 0x7f800000u;
               o = use ? f2u(g6_roundtrip(x)) : 0u; break; }
      case 18: { const float e = glibc_expf(u2f(u));                 // the teacher's expf (libm's)
               o = e != e ? 0x7fc00000u : f2u(e); break; }
      default: o = 0; use = false;
    }
    if (use) sum += splitmix64(((uint64_t)u << 32) | o);
  }
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)sum);
}

hipError_t launch_digest(int fn, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(k_digest, dim3(256 * 16), dim3(256), 0, s, fn, out);
  return hipGetLastError();
}

#endif  // FLEET_STREAM_TU
}  // namespace fleet
