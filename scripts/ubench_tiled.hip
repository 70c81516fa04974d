// scripts/ubench_tiled.hip -- phase timing of the pipelined tiles k_update_pipe (dev tool).
// Builds kernels.hip with FLEET_TIMING and prints per-block phase durations.
#define FLEET_TIMING 1
#define FLEET_DEV_ALL_KERNELS 1
#include "../fleet_amd/csrc/kernels.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace fleet;

template <int TG, bool PIPE, int IPT = 1, int NW = 4, int WP = 0>
static void launch(unsigned blocks, const uint8_t* text, size_t pitch, int M, const double* damp, int64_t n_up,
                   int64_t groups, const int32_t* hdr, uint8_t* merged, float* mf, int* err) {
  static_assert(PIPE, "the classic tiles have no standalone kernel since r06");
  hipLaunchKernelGGL((k_update_pipe<TG, IPT, NW, WP>), dim3(blocks), dim3(64 * NW), 0, 0, text, pitch, M, damp, 1.0 / M,
                     n_up, (int64_t)0, groups, hdr, merged, mf, err, INT32_MAX, EncodeJob{});
}

static std::vector<int32_t> g_hpos;
static std::vector<float> g_hval;

// network.h:1038-1056 layout: [nW, (size_i, dW_i..)*, nB, (size_j, db_j..)*]
static int64_t layout(std::vector<int> w, std::vector<int> b) {
  g_hpos.clear();
  g_hval.clear();
  int64_t p = 0;
  g_hpos.push_back(p++);
  g_hval.push_back((float)w.size());
  for (int x : w) {
    g_hpos.push_back(p);
    g_hval.push_back((float)x);
    p += 1 + x;
  }
  g_hpos.push_back(p++);
  g_hval.push_back((float)b.size());
  for (int x : b) {
    g_hpos.push_back(p);
    g_hval.push_back((float)x);
    p += 1 + x;
  }
  return p;
}

template <int TG, bool PIPE = false, int IPT = 1, int NW = 4, int WP = 0>
void run(int64_t n_up, int M, int reps = 1) {
  const int64_t groups = (n_up + 2) / 3;
  const size_t pitch = 16 * groups, vpitch = 3 * groups;
  float* vals;
  uint8_t *text, *merged;
  float* mf;
  double* damp;
  int32_t* hdr;
  int* err;
  hipMalloc(&vals, sizeof(float) * vpitch * M);
  hipMalloc(&text, pitch * M);
  hipMalloc(&merged, pitch);
  hipMalloc(&mf, sizeof(float) * vpitch);
  hipMalloc(&damp, sizeof(double) * M);
  hipMalloc(&hdr, sizeof(int32_t) * 8);
  hipMalloc(&err, sizeof(int));
  std::vector<double> d(M);
  for (int c = 0; c < M; ++c) d[c] = 1.0 / ((c % 3) + 1);
  hipMemcpy(damp, d.data(), sizeof(double) * M, hipMemcpyHostToDevice);
  const int nh = (int)g_hpos.size();
  hipFree(hdr);
  hipMalloc(&hdr, sizeof(int32_t) * (4 + nh));
  std::vector<int32_t> h = {0, nh, (int32_t)n_up, 0};
  h.insert(h.end(), g_hpos.begin(), g_hpos.end());
  hipMemcpy(hdr, h.data(), sizeof(int32_t) * h.size(), hipMemcpyHostToDevice);
  hipMemset(err, 0, sizeof(int));
  int32_t* dpos = nullptr;
  float* dval = nullptr;
  if (nh) {
    hipMalloc(&dpos, sizeof(int32_t) * nh);
    hipMalloc(&dval, sizeof(float) * nh);
    hipMemcpy(dpos, g_hpos.data(), sizeof(int32_t) * nh, hipMemcpyHostToDevice);
    hipMemcpy(dval, g_hval.data(), sizeof(float) * nh, hipMemcpyHostToDevice);
  }
  launch_synth(1, 0, 0, M, n_up, vals, vpitch, dpos, dval, nh, 0);
  launch_encode_f32(vals, n_up, vpitch, M, text, pitch, 0);
  const unsigned blocks = (unsigned)((groups + TG - 1) / TG);
  for (int rep = 0; rep < 3; ++rep)
    launch<TG, PIPE, IPT, NW, WP>(blocks, text, pitch, M, damp, n_up, groups, hdr, merged, mf, err);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r)
    launch<TG, PIPE, IPT, NW, WP>(blocks, text, pitch, M, damp, n_up, groups, hdr, merged, mf, err);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  int herr = 0;
  hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost);
  if (herr) printf("kernel error flag %d\n", herr);
  std::vector<unsigned long long> t(blocks * 8);
  hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_fleet_timing), sizeof(unsigned long long) * blocks * 8);
  // slots: 0 start, 1 init done, 2 first pass done (thread 0), 3 phase 1 done, 4 phase 2 done, 5 end
  unsigned long long t0 = ~0ull, t5 = 0;
  double seg[5] = {0, 0, 0, 0, 0}, segmax[5] = {0, 0, 0, 0, 0};
  const int from[5] = {0, 1, 2, 3, 4}, to[5] = {1, 2, 3, 4, 5};
  for (unsigned i = 0; i < blocks; ++i) {
    t0 = std::min(t0, t[8 * i]);
    t5 = std::max(t5, t[8 * i + 5]);
    for (int k = 0; k < 5; ++k) {
      double v = (double)(t[8 * i + to[k]] - t[8 * i + from[k]]) * 0.01;  // 100 MHz ticks -> us
      seg[k] += v;
      segmax[k] = std::max(segmax[k], v);
    }
  }
  double wsum = 0, spun = 0;
  if (PIPE)
    for (unsigned i = 0; i < blocks; ++i) {
      wsum += (double)t[8 * i + 6] * 0.01;
      spun += (double)t[8 * i + 7];
    }
  if (PIPE) printf("  consumer waited for producers after pass 0: %.2f us avg, %.2f passes avg\n", wsum / blocks, spun / blocks);
  printf("%s%d/%dw/wp%d TG=%d n=%ld M=%d blocks=%u: event %.1f us, span %.1f us | init %.2f/%.2f | pass0 %.2f/%.2f | "
         "rest of phase1 %.2f/%.2f | phase2 %.2f/%.2f (%.0f ns/client) | epilogue %.2f/%.2f  (avg/max us)\n",
         PIPE ? "pipe" : "tiled", PIPE ? IPT : 2, NW, WP, TG, (long)n_up, M, blocks, ms * 1e3, (t5 - t0) * 0.01, seg[0] / blocks, segmax[0], seg[1] / blocks,
         segmax[1], seg[2] / blocks, segmax[2], seg[3] / blocks, segmax[3], seg[3] / blocks * 1e3 / M,
         seg[4] / blocks, segmax[4]);
  hipFree(vals);
  hipFree(text);
  hipFree(merged);
  hipFree(mf);
  hipFree(damp);
  hipFree(hdr);
  hipFree(err);
}

// back-to-back client encodes of M rows of n floats (k_encode_f32)
static void time_encode(int64_t n_up, int M, int reps) {
  const int64_t groups = (n_up + 2) / 3;
  const size_t pitch = 16 * groups, vpitch = 3 * groups;
  float* vals;
  uint8_t* text;
  hipMalloc(&vals, sizeof(float) * vpitch * M);
  hipMalloc(&text, pitch * M);
  launch_synth(1, 0, 0, M, n_up, vals, vpitch, nullptr, nullptr, 0, 0);
  for (int r = 0; r < 3; ++r) launch_encode_f32(vals, n_up, vpitch, M, text, pitch, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) launch_encode_f32(vals, n_up, vpitch, M, text, pitch, 0);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("encode n=%ld M=%d: %.2f us per launch (%d back-to-back)\n", (long)n_up, M, ms * 1e3 / reps, reps);
  hipFree(vals);
  hipFree(text);
}

int main() {
  const int64_t n = layout({200, 0, 128, 19200, 0, 1920}, {784, 0, 512, 0, 0, 192, 10});
  printf("MNIST layout n_up=%ld headers=%zu\n", (long)n, g_hpos.size());
  for (int M : {64, 256}) run<16, true, 1, 5, 0>(n, M, 200);
  return 0;
}
