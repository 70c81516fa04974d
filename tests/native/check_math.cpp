// tests/native/check_math.cpp -- CPU check of fleet_amd/csrc/codec_math.h (the
// arithmetic the gfx950 kernels run) against the oracle (oracle/fleet_oracle.c).
//
//   check_math sample      ~1e8 sampled inputs per function (CPU test suite)
//   check_math exhaustive  every input in each fast path's domain (dev check; ~1 min on 8 cores)
//   check_math g6          the model-version copy's %g / strtof round trip (decimal6.h) against
//                          libc's snprintf / strtof on every finite binary32 (~8 min on 8 cores)
//
// Exit status 0 = all bit-identical.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../fleet_amd/csrc/codec_math.h"
#include "../../fleet_amd/csrc/decimal6.h"
extern "C" {
#include "../../oracle/fleet_oracle.h"
}

using namespace fleet;
static std::atomic<long> g_bad{0};
static const StepTables g_st = make_step_tables();

template <typename F>
void par_for(uint64_t begin, uint64_t end, uint64_t stride, F f) {
  unsigned nt = std::max(1u, std::thread::hardware_concurrency());
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([=] {
      for (uint64_t i = begin + t * stride; i < end; i += (uint64_t)nt * stride) f(i);
    });
  for (auto& x : th) x.join();
}

static void report(const char* name, long bad_before) {
  long b = g_bad.load() - bad_before;
  printf("%-28s %s (%ld mismatches)\n", name, b ? "FAIL" : "ok", b);
}

static inline bool same(float a, float b) { return f2u(a) == f2u(b); }

int main(int argc, char** argv) {
  bool exhaustive = argc > 1 && std::string(argv[1]) == "exhaustive";
  if (argc > 1 && std::string(argv[1]) == "qlat") {  // q_lat alone, every input of its domain
    long b = g_bad;
    par_for(0, 1ull << 32, 1, [](uint64_t i) {
      float x = u2f((uint32_t)i);
      if (!q_gen_ok(x)) return;
      if (!same(q_lat(x), fo_int2float(fo_float2int(x)))) g_bad++;
    });
    report("q_lat (exhaustive)", b);
    return g_bad ? 1 : 0;
  }
  if (argc > 1 && std::string(argv[1]) == "xl") {  // one-lookup latency Q, every input of |x| < 1e8
    static XlEntry xt[2 * kXlSpan];
    for (uint32_t i = 0; i < 2 * kXlSpan; ++i) xt[i] = xl_entry(i);
    long b = g_bad;
    par_for(0, 1ull << 32, 1, [](uint64_t i) {
      const float x = u2f((uint32_t)i);
      if (!(__builtin_fabsf(x) < 1e8f)) return;
      if (!same(q_xl(x, xt), fo_int2float(fo_float2int(x)))) g_bad++;
    });
    report("q_xl (exhaustive)", b);
    return g_bad ? 1 : 0;
  }
  if (argc > 1 && std::string(argv[1]) == "mt") {  // multiplier-table functions, every input
    static VarEntry vt[512];
    static MulEntry mt[16];
    for (uint32_t i = 0; i < 512; ++i) vt[i] = var_entry(i);
    for (uint32_t d = 0; d < 16; ++d) mt[d] = mul_entry(d);
    long b = g_bad;
    par_for(0, 1ull << 32, 1, [](uint64_t i) {
      const float x = u2f((uint32_t)i);
      const int32_t c = (int32_t)(uint32_t)i;
      const uint32_t a = c < 0 ? 0u - (uint32_t)c : (uint32_t)c;
      if (!same(dec_mt_r(c, last_digit_u(a), mt), fo_int2float(c))) g_bad++;
      const uint32_t d = var_digits(x, vt);
      if (!q_gen_ok(x)) {
        if (d <= 9u) g_bad++;
        return;
      }
      if (d != (uint32_t)fo_num_digits(fo_cvtt(x))) g_bad++;
      const int32_t e = fo_float2int(x);
      if (!same(q_mt(x, vt, mt), fo_int2float(e)) || enc_mt(x, vt, mt) != e) g_bad++;
      if (q_ok(x) && !same(q_fast1(x), fo_int2float(e))) g_bad++;
    });
    report("q_mt/enc_mt/dec_mt/var_digits/q_fast1 (exhaustive)", b);
    return g_bad ? 1 : 0;
  }
  if (argc > 1 && std::string(argv[1]) == "d16") {  // byte-table digit count + stride-16 Q, every input
    static VarEntry vt[512];
    static uint8_t dt[8192];
    static StepTables st = make_step_tables();
    for (uint32_t i = 0; i < 512; ++i) vt[i] = var_entry(i);
    for (uint32_t i = 0; i < 8192; ++i) dt[i] = d16_entry(i);
    long b = g_bad;
    par_for(0, 1ull << 32, 1, [](uint64_t i) {
      const float x = u2f((uint32_t)i);
      uint32_t e = dt[(uint32_t)i >> 19];
      if (e == kD16Cmp) e = d16_fix(x, vt);
      if (!q_gen_ok(x)) {
        if (e < kD16Out || var_d16((uint32_t)i, vt) < kD16Out) g_bad++;
        return;
      }
      if (e != 16u * (uint32_t)fo_num_digits(fo_cvtt(x))) g_bad++;
      if (var_d16((uint32_t)i, vt) != e) g_bad++;  // stage C's compare form
      if (!same(q_d16(x, e, &st), fo_int2float(fo_float2int(x)))) g_bad++;
      if (enc_d16(x, e, &st) != fo_float2int(x)) g_bad++;  // the client encode's form
    });
    par_for(0, 1ull << 32, 1, [](uint64_t i) {  // int2float from the same tables, every code
      const int32_t c = (int32_t)(uint32_t)i;
      const uint32_t a = c < 0 ? 0u - (uint32_t)c : (uint32_t)c;
      if (!same(dec_d16(c, last_digit_u(a) << 4, &g_st), fo_int2float(c))) g_bad++;
      if (ld16_entry(ld16_index(c)) != last_digit_u(a) << 4) g_bad++;  // the stream kernels' byte-sum form
    });
    long cmp_slices = 0;
    for (uint32_t i = 0; i < 8192; ++i) cmp_slices += dt[i] == kD16Cmp;
    printf("d16 table: %ld compare slices of 8192\n", cmp_slices);
    report("d16 / q_d16 / enc_d16 (exhaustive)", b);
    return g_bad ? 1 : 0;
  }
  if (argc > 1 && std::string(argv[1]) == "g6") {  // %g / strtof round trip, every finite input
    long b = g_bad;
    par_for(0, 1ull << 32, 1, [](uint64_t i) {
      const uint32_t u = (uint32_t)i;
      if ((u & 0x7f800000u) == 0x7f800000u) return;
      char buf[64];
      snprintf(buf, sizeof buf, "%g", (double)u2f(u));
      if (!same(g6_roundtrip(u2f(u)), strtof(buf, nullptr))) g_bad++;
    });
    report("g6_roundtrip (exhaustive)", b);
    return g_bad ? 1 : 0;
  }
  const uint64_t s = exhaustive ? 1 : 97;  // sampling stride (odd, walks every residue class)
  long b0;

  b0 = g_bad;  // div10 vs IEEE division, all positive finite floats >= 1e-30 (0x0DA24260)
  par_for(0x0DA24260ull, 0x7F800000ull, s, [](uint64_t i) {
    float t = u2f((uint32_t)i);
    if (!same(div10(t), t / 10.0f) || !same(div10(-t), -t / 10.0f)) g_bad++;
  });
  report("div10", b0);

  b0 = g_bad;  // dec9_ok vs c % 10 == 0, all int32
  par_for(0, 1ull << 32, s, [](uint64_t i) {
    int32_t c = (int32_t)(uint32_t)i;
    if (dec9_ok(c) != (c % 10 == 0)) g_bad++;
  });
  report("dec9_ok", b0);

  b0 = g_bad;  // dec_fast vs int2float on its domain (multiples of 10)
  par_for(0, 1ull << 32, 10 * s, [](uint64_t i) {
    int32_t c = (int32_t)(uint32_t)i;
    if (c % 10 != 0) return;
    if (!same(dec_fast(c), fo_int2float(c))) g_bad++;
  });
  report("dec_fast", b0);

  b0 = g_bad;  // q_fast (+ packed) vs Q on its domain |x| < 1, both signs
  par_for(0, 0x3F800000ull, s, [](uint64_t i) {
    float x = u2f((uint32_t)i);
    float r = fo_int2float(fo_float2int(x)), rn = fo_int2float(fo_float2int(-x));
    f2 p = q_fast2(f2{x, -x});
    if (!same(q_fast(x), r) || !same(q_fast(-x), rn) || !same(p.x, r) || !same(p.y, rn)) g_bad++;
  });
  report("q_fast/q_fast2 (|x|<1)", b0);

  static const DigitEntry tab[32] = FLEET_DIGIT_TABLE;
  b0 = g_bad;  // digits_of vs numDigits((int)x), |x| < 2^31
  par_for(0, 1ull << 32, s, [](uint64_t i) {
    float x = u2f((uint32_t)i);
    if (!(__builtin_fabsf(x) < 2147483648.0f)) return;
    if (digits_of(x, tab) != fo_num_digits(fo_cvtt(x))) g_bad++;
  });
  report("digits_of", b0);

  b0 = g_bad;  // digits_cmp and q_gen without table on the q_gen domain
  par_for(0, 1ull << 32, s * 3, [](uint64_t i) {
    float x = u2f((uint32_t)i);
    if (!q_gen_ok(x)) return;
    if (digits_cmp(x) != fo_num_digits(fo_cvtt(x))) g_bad++;
    if (!same(q_gen_lat(x), fo_int2float(fo_float2int(x)))) g_bad++;
    if (!same(q_lat(x), fo_int2float(fo_float2int(x)))) g_bad++;
    if (enc_gen(x, tab) != fo_float2int(x)) g_bad++;
    if (q_ok(x) && enc_fast(x) != fo_float2int(x)) g_bad++;
  });
  report("digits_cmp/q_gen_lat/q_lat/enc_gen/enc_fast", b0);

  b0 = g_bad;  // q_gen (+ packed) vs Q on its domain -1e6 < x < 1e7
  par_for(0, 1ull << 32, s, [](uint64_t i) {
    float x = u2f((uint32_t)i);
    if (!q_gen_ok(x)) return;
    float r = fo_int2float(fo_float2int(x));
    f2 p = q_gen2(f2{x, x * 0.5f}, tab);
    float r2 = fo_int2float(fo_float2int(x * 0.5f));
    if (!same(q_gen(x, tab), r) || !same(p.x, r) || !same(p.y, r2)) g_bad++;
  });
  report("q_gen/q_gen2", b0);

  static VarEntry vt[512];
  static MulEntry mt[16];
  for (uint32_t i = 0; i < 512; ++i) vt[i] = var_entry(i);
  for (uint32_t d = 0; d < 16; ++d) mt[d] = mul_entry(d);

  b0 = g_bad;  // var_digits vs numDigits((int)x) on the q_gen domain, slow marker outside it
  par_for(0, 1ull << 32, s, [](uint64_t i) {
    float x = u2f((uint32_t)i);
    const uint32_t d = var_digits(x, vt);
    if (q_gen_ok(x) ? d != (uint32_t)fo_num_digits(fo_cvtt(x)) : d <= 9u) g_bad++;
  });
  report("var_digits", b0);

  b0 = g_bad;  // multiplier-table Q / float2int / fixed scalar Q vs the oracle
  par_for(0, 1ull << 32, s, [](uint64_t i) {
    float x = u2f((uint32_t)i);
    if (!q_gen_ok(x)) return;
    if (!same(q_mt(x, vt, mt), fo_int2float(fo_float2int(x)))) g_bad++;
    if (enc_mt(x, vt, mt) != fo_float2int(x)) g_bad++;
    if (q_ok(x) && !same(q_fast1(x), fo_int2float(fo_float2int(x)))) g_bad++;
  });
  report("q_mt/enc_mt/q_fast1", b0);
  b0 = g_bad;  // byte-table digit offsets + stride-16 Q (k_update's stages) vs the oracle
  {
    static uint8_t dt[8192];
    static StepTables st = make_step_tables();
    for (uint32_t i = 0; i < 8192; ++i) dt[i] = d16_entry(i);
    par_for(0, 1ull << 32, s, [](uint64_t i) {
      const float x = u2f((uint32_t)i);
      uint32_t e = dt[(uint32_t)i >> 19];
      if (e == kD16Cmp) e = d16_fix(x, vt);
      if (!q_gen_ok(x)) {
        if (e < kD16Out || var_d16((uint32_t)i, vt) < kD16Out) g_bad++;
        return;
      }
      if (e != 16u * (uint32_t)fo_num_digits(fo_cvtt(x))) g_bad++;
      if (var_d16((uint32_t)i, vt) != e) g_bad++;  // stage C's compare form
      if (!same(q_d16(x, e, &st), fo_int2float(fo_float2int(x)))) g_bad++;
      if (enc_d16(x, e, &st) != fo_float2int(x)) g_bad++;
    });
    // every power-of-ten slice, densely (where the compare decides)
    for (uint32_t sl = 0; sl < 8192; ++sl)
      if (dt[sl] == kD16Cmp)
        par_for((uint64_t)sl << 19, (uint64_t)(sl + 1) << 19, 1, [](uint64_t i) {
          const float x = u2f((uint32_t)i);
          const uint32_t e = d16_fix(x, vt);
          if (!q_gen_ok(x)) {
            if (e < kD16Out) g_bad++;
            return;
          }
          if (e != 16u * (uint32_t)fo_num_digits(fo_cvtt(x)) || !same(q_d16(x, e, &st), fo_int2float(fo_float2int(x))) ||
              enc_d16(x, e, &st) != fo_float2int(x))
            g_bad++;
        });
  }
  report("d16/q_d16/enc_d16", b0);
  b0 = g_bad;
  {
    static XlEntry xt[2 * kXlSpan];
    for (uint32_t i = 0; i < 2 * kXlSpan; ++i) xt[i] = xl_entry(i);
    par_for(0, 1ull << 32, s, [](uint64_t i) {
      const float x = u2f((uint32_t)i);
      if (__builtin_fabsf(x) < 1e8f && !same(q_xl(x, xt), fo_int2float(fo_float2int(x)))) g_bad++;
    });
  }
  report("q_xl", b0);

  b0 = g_bad;  // multiplier-table int2float, every code
  par_for(0, 1ull << 32, s, [](uint64_t i) {
    int32_t c = (int32_t)(uint32_t)i;
    const uint32_t a = c < 0 ? 0u - (uint32_t)c : (uint32_t)c;
    if (last_digit_u(a) != a % 10u) g_bad++;
    if (!same(dec_mt_r(c, last_digit_u(a), mt), fo_int2float(c))) g_bad++;
    if (!same(dec_d16(c, last_digit_u(a) << 4, &g_st), fo_int2float(c))) g_bad++;
    if (ld16_entry(ld16_index(c)) != (a % 10u) << 4) g_bad++;  // the stream kernels' byte-sum step count
  });
  report("dec_mt/dec_d16/last_digit_u/ld16", b0);

  b0 = g_bad;  // dec_gen (+ packed) vs int2float, every code
  par_for(0, 1ull << 32, s, [](uint64_t i) {
    int32_t c = (int32_t)(uint32_t)i;
    float r = fo_int2float(c);
    int32_t c2 = c / 7 * 3;
    f2 p = dec_gen2(c, c2);
    if (!same(dec_gen(c), r) || !same(p.x, r) || !same(p.y, fo_int2float(c2))) g_bad++;
  });
  report("dec_gen/dec_gen2", b0);

  b0 = g_bad;  // general dec vs int2float, all int32 (sampled more coarsely in sample mode)
  par_for(0, 1ull << 32, exhaustive ? 1 : 1009, [](uint64_t i) {
    int32_t c = (int32_t)(uint32_t)i;
    if (!same(dec(c), fo_int2float(c))) g_bad++;
  });
  report("dec (general)", b0);

  b0 = g_bad;  // general enc vs float2int, all float bit patterns (incl. inf/NaN)
  par_for(0, 1ull << 32, exhaustive ? 1 : 1009, [](uint64_t i) {
    float x = u2f((uint32_t)i);
    if (enc(x) != fo_float2int(x)) g_bad++;
  });
  report("enc (general)", b0);

  b0 = g_bad;  // stage C's VarEntry digit offsets against the byte table's, sampled
  {
    static VarEntry vt2[512];
    static uint8_t dt2[8192];
    for (uint32_t i = 0; i < 512; ++i) vt2[i] = var_entry(i);
    for (uint32_t i = 0; i < 8192; ++i) dt2[i] = d16_entry(i);
    par_for(0, 1ull << 32, s, [](uint64_t i) {
      const float x = u2f((uint32_t)i);
      uint32_t e = dt2[(uint32_t)i >> 19];
      if (e == kD16Cmp) e = d16_fix(x, vt2);
      const uint32_t v = var_d16((uint32_t)i, vt2);
      if (q_gen_ok(x) ? v != e : v < kD16Out) g_bad++;
    });
  }
  report("var_d16", b0);

  b0 = g_bad;  // %g / strtof round trip against libc, sampled
  par_for(0, 1ull << 32, exhaustive ? 1 : 1009, [](uint64_t i) {
    const uint32_t u = (uint32_t)i;
    if ((u & 0x7f800000u) == 0x7f800000u) return;
    char buf[64];
    snprintf(buf, sizeof buf, "%g", (double)u2f(u));
    if (!same(g6_roundtrip(u2f(u)), strtof(buf, nullptr))) g_bad++;
  });
  report("g6_roundtrip", b0);

  printf("%s\n", g_bad ? "FAILED" : "ALL OK");
  return g_bad ? 1 : 0;
}
