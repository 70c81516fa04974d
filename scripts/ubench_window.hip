// scripts/ubench_window.hip -- per-wave progress trace of the stream aggregation on
// one column window (dev tool; VERDICT r03 item 1: configs[4]'s N = 4 window takes
// 0.87 / 6.54 / 26.4 ms at M = 256 / 1024 / 4096).
//
// Every wave stamps the realtime counter (100 MHz) when it reaches clients
// k*M/16, k = 0..16, plus its hardware slot (XCC, SE, CU, SIMD). The host prints
// the kernel time, the spread of wave start / end times, the timeline of active
// waves and their client positions, and per-segment rates, and dumps the raw
// stamps under gpurun_out/.
//
// usage: ubench_window GROUPS M[,M...] [plain|mixed] [rep]
#include <hip/hip_runtime.h>

#include <cstdint>

__device__ unsigned long long* g_wt = nullptr;
__device__ __forceinline__ void fleet_trace_hook(int c, int M) {
  unsigned long long* wt = g_wt;
  if (wt == nullptr) return;
  const int step = M >> 4;  // M % 32 == 0: step is even, c runs over even values
  if (c % step != 0) return;
  const int k = c / step;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) {
    wt[wave * 18 + k] = wall_clock64();
    if (k == 0) {
      const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_ID
      const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);   // XCC_ID
      wt[wave * 18 + 17] = ((unsigned long long)xcc << 32) | hw;
    }
  }
}
#define FLEET_CLIENT_HOOK(c, M) fleet_trace_hook(c, M)
#define FLEET_DEV_ALL_KERNELS 1
#include "../fleet_amd/csrc/kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

using namespace fleet;



__global__ void __launch_bounds__(256) k_probe(const uint8_t* __restrict__ uploads, size_t pitch, int M,
                                               const double* __restrict__ dampen, double inv_avg, int64_t n_up,
                                               int64_t g_begin, int64_t g_end, const int32_t* __restrict__ hdr_block,
                                               uint8_t* __restrict__ merged, float* __restrict__ merged_f32,
                                               int* __restrict__ err, int nA) {
  __shared__ B64Tables tab;
  __shared__ D16Table dtab;
  b64_tables_init<256>(&tab);
  d16_table_init<256>(&dtab);
  __syncthreads();
  update_mixed_block<256>(tab, dtab, blockIdx.x, uploads, pitch, M, dampen, inv_avg, n_up, g_begin, g_end, hdr_block,
                          merged, merged_f32, err, nA);
}

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

static double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  size_t i = (size_t)std::min<double>(v.size() - 1, p * (v.size() - 1));
  return v[i];
}

static void run(int64_t groups, int M, bool plain, const char* tag) {
  const int64_t n_up = 3 * groups;
  const size_t pitch = 16 * (size_t)groups, vpitch = 3 * (size_t)groups;
  float* vals;
  uint8_t *text, *merged;
  float* mf;
  double* damp;
  int32_t* hdr;
  int* err;
  CHK(hipMalloc(&vals, sizeof(float) * vpitch * M));
  CHK(hipMalloc(&text, pitch * M));
  CHK(hipMalloc(&merged, pitch));
  CHK(hipMalloc(&mf, sizeof(float) * vpitch));
  CHK(hipMalloc(&damp, sizeof(double) * M));
  CHK(hipMalloc(&hdr, sizeof(int32_t) * 8));
  CHK(hipMalloc(&err, sizeof(int)));
  std::vector<double> d(M);
  for (int c = 0; c < M; ++c) d[c] = 1.0 / ((c % 3) + 1);
  CHK(hipMemcpy(damp, d.data(), sizeof(double) * M, hipMemcpyHostToDevice));
  const int32_t h[8] = {0, 0, (int32_t)n_up, 0, 0, 0, 0, 0};
  CHK(hipMemcpy(hdr, h, sizeof h, hipMemcpyHostToDevice));
  CHK(hipMemset(err, 0, sizeof(int)));
  CHK(launch_synth(1, 0, 0, M, n_up, vals, vpitch, nullptr, nullptr, 0, 0));
  CHK(launch_encode_f32(vals, n_up, vpitch, M, text, pitch, 0));
  CHK(hipDeviceSynchronize());
  CHK(hipFree(vals));

  // the launch plan of launch_update's stream path
  int nA, blocks;
  const int simds = device_simds();
  const int64_t waves_plain = (groups + 63) / 64;
  if (plain || waves_plain < simds) {
    nA = (int)((groups + 255) / 256);
    blocks = nA;
  } else {
    nA = (int)(waves_plain / simds * simds * 64 / 256);
    blocks = nA + (int)((groups - (int64_t)nA * 256 + 83) / 84);
  }
  const size_t nwaves = (size_t)blocks * 4;
  unsigned long long* wt;
  CHK(hipMalloc(&wt, nwaves * 18 * sizeof(unsigned long long)));
  CHK(hipMemset(wt, 0, nwaves * 18 * sizeof(unsigned long long)));
  auto launch = [&]() {
    hipLaunchKernelGGL(k_probe, dim3((unsigned)blocks), dim3(256), 0, 0, text, pitch, M, damp, 1.0 / M, n_up,
                       (int64_t)0, groups, hdr, merged, mf, err, nA);
  };
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  // untraced (hook reads a null pointer)
  unsigned long long* none = nullptr;
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_wt), &none, sizeof none));
  launch();
  CHK(hipEventRecord(a));
  launch();
  launch();
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms_plain;
  CHK(hipEventElapsedTime(&ms_plain, a, b));
  ms_plain /= 2;
  // traced
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_wt), &wt, sizeof wt));
  CHK(hipEventRecord(a));
  launch();
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms_tr;
  CHK(hipEventElapsedTime(&ms_tr, a, b));
  int herr = 0;
  CHK(hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost));
  std::vector<unsigned long long> t(nwaves * 18);
  CHK(hipMemcpy(t.data(), wt, t.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_wt), &none, sizeof none));

  // raw dump
  {
    char path[256];
    snprintf(path, sizeof path, "gpurun_out/window_%s_g%ld_m%d_%s.bin", tag, (long)groups, M, plain ? "plain" : "mixed");
    if (FILE* f = fopen(path, "wb")) {
      fwrite(t.data(), sizeof(unsigned long long), t.size(), f);
      fclose(f);
    }
  }
  // analysis: waves that stamped client 0 (value-per-lane lane 63 waves too)
  unsigned long long t0 = ~0ull, t1 = 0;
  std::vector<size_t> live;
  for (size_t w = 0; w < nwaves; ++w) {
    if (!t[w * 18] || !t[w * 18 + 16]) continue;
    live.push_back(w);
    t0 = std::min(t0, t[w * 18]);
    t1 = std::max(t1, t[w * 18 + 16]);
  }
  const double span = (t1 - t0) * 0.01;  // us
  std::vector<double> st, en, dur;
  std::map<uint64_t, int> per_simd;
  std::map<uint32_t, int> per_xcc;
  for (size_t w : live) {
    st.push_back((t[w * 18] - t0) * 0.01);
    en.push_back((t[w * 18 + 16] - t0) * 0.01);
    dur.push_back((t[w * 18 + 16] - t[w * 18]) * 0.01);
    const uint64_t id = t[w * 18 + 17];
    const uint32_t hw = (uint32_t)id, xcc = (uint32_t)(id >> 32) & 0xf;
    const uint32_t simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    per_simd[((uint64_t)xcc << 16) | (se << 8) | (sh << 7) | (cu << 2) | simd]++;
    per_xcc[xcc]++;
  }
  std::vector<double> simd_counts;
  for (auto& kv : per_simd) simd_counts.push_back(kv.second);
  printf("== %s groups=%ld M=%d grid=%s blocks=%d (nA=%d) waves=%zu traced=%zu | kernel %.1f us (traced %.1f us), "
         "span %.1f us, %.2f us/client, err=%d\n",
         tag, (long)groups, M, plain ? "plain" : "mixed", blocks, nA, nwaves, live.size(), ms_plain * 1e3, ms_tr * 1e3,
         span, span / M, herr);
  printf("   SIMDs used %zu, waves per SIMD min %.0f med %.0f max %.0f; XCCs:", simd_counts.size(), pct(simd_counts, 0),
         pct(simd_counts, 0.5), pct(simd_counts, 1));
  for (auto& kv : per_xcc) printf(" %u:%d", kv.first, kv.second);
  printf("\n   start us: p0 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f\n", pct(st, 0), pct(st, .5), pct(st, .9), pct(st, .99),
         pct(st, 1));
  printf("   end   us: p0 %.1f p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f\n", pct(en, 0), pct(en, .1), pct(en, .5),
         pct(en, .9), pct(en, .99), pct(en, 1));
  printf("   dur   us: p0 %.1f p50 %.1f p90 %.1f max %.1f\n", pct(dur, 0), pct(dur, .5), pct(dur, .9), pct(dur, 1));
  // per-segment time per client (sixteenths of the client loop), over waves
  printf("   segment us/client (p10/p50/p90):");
  for (int k = 0; k < 16; ++k) {
    std::vector<double> s;
    for (size_t w : live) s.push_back((t[w * 18 + k + 1] - t[w * 18 + k]) * 0.01 / (M / 16.0));
    if (k % 4 == 0 || k == 15) printf(" [%d] %.2f/%.2f/%.2f", k, pct(s, .1), pct(s, .5), pct(s, .9));
  }
  printf("\n");
  // timeline: active waves and client positions (interpolated) in 16 time bins
  printf("   timeline (t us: active waves, client pos p10/p50/p90, finished):\n");
  for (int bi = 1; bi <= 16; ++bi) {
    const double tt = span * bi / 16.0;
    int active = 0, fin = 0;
    std::vector<double> pos;
    for (size_t w : live) {
      const double s0 = (t[w * 18] - t0) * 0.01, e0 = (t[w * 18 + 16] - t0) * 0.01;
      if (tt >= e0) {
        ++fin;
        continue;
      }
      if (tt < s0) continue;
      ++active;
      int k = 0;
      while (k < 16 && (t[w * 18 + k + 1] - t0) * 0.01 <= tt) ++k;
      const double a0 = (t[w * 18 + k] - t0) * 0.01, a1 = (t[w * 18 + k + 1] - t0) * 0.01;
      pos.push_back((k + (a1 > a0 ? (tt - a0) / (a1 - a0) : 0)) * M / 16.0);
    }
    printf("     %8.1f: %6d active  pos %7.1f %7.1f %7.1f  fin %d\n", tt, active, pct(pos, .1), pct(pos, .5),
           pct(pos, .9), fin);
  }
  CHK(hipFree(wt));
  CHK(hipFree(text));
  CHK(hipFree(merged));
  CHK(hipFree(mf));
  CHK(hipFree(damp));
  CHK(hipFree(hdr));
  CHK(hipFree(err));
}

int main(int argc, char** argv) {
  const int64_t groups = argc > 1 ? atoll(argv[1]) : 349526;
  std::vector<int> ms;
  {
    std::string s = argc > 2 ? argv[2] : "256,1024";
    size_t p = 0;
    while (p < s.size()) {
      size_t q = s.find(',', p);
      if (q == std::string::npos) q = s.size();
      ms.push_back(atoi(s.substr(p, q - p).c_str()));
      p = q + 1;
    }
  }
  const bool plain = argc > 3 && !strcmp(argv[3], "plain");
  const char* tag = argc > 4 ? argv[4] : "w";
  for (int M : ms) {
    if (M % 32) {
      fprintf(stderr, "M must be a multiple of 32\n");
      return 2;
    }
    run(groups, M, plain, tag);
    fflush(stdout);
  }
  return 0;
}
