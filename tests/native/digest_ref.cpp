// tests/native/digest_ref.cpp -- the oracle's side of fleet_selftest_digest:
// the same order-independent digests, computed with oracle/fleet_oracle.c over
// the same whole input domains (fn 18: the libm expf the reference's mojo
// network calls, against the device's glibc_expf restatement). Writes tests/golden/digests.json (~1 min, 8 cores).
#include <atomic>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <stdint.h>
extern "C" {
#include "../../oracle/fleet_oracle.h"
}

static inline uint32_t f2u(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static inline float u2f(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }
static inline uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline float Q(float x) { return fo_int2float(fo_float2int(x)); }

static uint64_t digest(int fn) {
  unsigned nt = std::max(1u, std::thread::hardware_concurrency());
  std::vector<uint64_t> part(nt, 0);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      uint64_t sum = 0;
      for (uint64_t i = t; i < (1ull << 32); i += nt) {
        uint32_t u = (uint32_t)i, o = 0;
        bool use = true;
        switch (fn) {
          case 0: o = f2u(fo_int2float((int32_t)u)); break;
          case 1: o = (uint32_t)fo_float2int(u2f(u)); break;
          case 2: use = (u & 0x7fffffffu) < 0x3f800000u; if (use) o = f2u(Q(u2f(u))); break;
          case 3: use = ((int32_t)u % 10) == 0; if (use) o = f2u(fo_int2float((int32_t)u)); break;
          case 4: use = u >= 0x0DA24260u && u < 0x7F800000u; if (use) o = f2u(u2f(u) / 10.0f); break;
          case 5: use = (u & 0x7fffffffu) < 0x3f800000u; if (use) o = f2u(Q(u2f(u))) + 3u * f2u(Q(-u2f(u))); break;
          case 6: { float x = u2f(u); use = x < 1e9f && x > -1e8f; if (use) o = f2u(Q(x)); break; }
          case 7: o = f2u(fo_int2float((int32_t)u)); break;
          case 8: { float x = u2f(u), x2 = -0.25f * x;
                    use = x < 1e9f && x > -1e8f && x2 < 1e9f && x2 > -1e8f; if (use) o = f2u(Q(x)) + 3u * f2u(Q(x2)); break; }
          case 9: { int32_t c = (int32_t)u, c2 = (int32_t)(u * 2654435761u);
                    o = f2u(fo_int2float(c)) + 3u * f2u(fo_int2float(c2)); break; }
          case 10: { float x = u2f(u); use = x < 1e9f && x > -1e8f; if (use) o = (uint32_t)fo_float2int(x); break; }
          case 11: use = (u & 0x7fffffffu) < 0x3f800000u; if (use) o = (uint32_t)fo_float2int(u2f(u)); break;
          case 12: { float x = u2f(u); use = x < 1e9f && x > -1e8f; if (use) o = f2u(Q(x)); break; }
          case 18: { float e = expf(u2f(u)); o = e != e ? 0x7fc00000u : f2u(e); break; }  // libm expf
          case 22: {  // libc's %g / strtof round trip (ostream << float, istream >> float)
            use = (u & 0x7f800000u) != 0x7f800000u;
            if (use) {
              char b[64];
              snprintf(b, sizeof b, "%g", (double)u2f(u));
              o = f2u(strtof(b, nullptr));
            }
            break;
          }
        }
        if (use) sum += splitmix64(((uint64_t)u << 32) | o);
      }
      part[t] = sum;
    });
  for (auto& x : th) x.join();
  uint64_t s = 0;
  for (auto p : part) s += p;
  return s;
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "tests/golden/digests.json";
  FILE* f = fopen(path, "w");
  fprintf(f, "{\n  \"generator\": \"tests/native/digest_ref.cpp over oracle/fleet_oracle.c\",\n");
  std::vector<int> fns = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 18, 22};
  if (argc > 2) {  // argv[2..]: print only these functions' digests (no file written)
    for (int a = 2; a < argc; ++a) printf("fn%d %016llx\n", atoi(argv[a]), (unsigned long long)digest(atoi(argv[a])));
    return 0;
  }
  const int nf = (int)fns.size();
  for (int j = 0; j < nf; ++j) {
    const int fn = fns[j];
    uint64_t d = digest(fn);
    fprintf(f, "  \"fn%d\": \"%016llx\"%s\n", fn, (unsigned long long)d, j < nf - 1 ? "," : "");
    printf("fn%d %016llx\n", fn, (unsigned long long)d);
    fflush(stdout);
  }
  fprintf(f, "}\n");
  fclose(f);
  return 0;
}
