// scripts/ubench_mix.hip -- issue cost of v_fma_mix_f32 with an f16 multiplier (the x10 chain's
// multipliers 1 / 10 as halves of one register: a ds_read_b64 per four instead of a b128) against
// v_mul_f32, and ds_read_b64 / b128 broadcast costs (dev tool; harness of ubench3.hip)
#include <hip/hip_runtime.h>

#include <cstdio>

#define ITER 2048
#define CH 8
#define BLOCKS (256 * 8)
#define THREADS 256

__global__ void k_clock(unsigned long long* out) {
  const unsigned long long c0 = clock64(), w0 = wall_clock64();
  float v = threadIdx.x;
  for (int i = 0; i < 200000; ++i) asm volatile("v_mul_f32 %0, %0, %0" : "+v"(v));
  const unsigned long long c1 = clock64(), w1 = wall_clock64();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = w1 - w0;
  }
  if (v == 12345.f) out[2] = 1;
}

#define VK(name, ...)                                                   \
  __global__ void name(float* out, float s) {                            \
    float v[CH];                                                         \
    unsigned u[CH];                                                      \
    for (int i = 0; i < CH; ++i) v[i] = s + threadIdx.x + i, u[i] = threadIdx.x * 7 + i; \
    const float a = s * 1.5f, b = s * 0.25f;                             \
    const unsigned ua = threadIdx.x | 0x55u, ub = 0xff00ff00u;           \
    unsigned long long m = __ballot(threadIdx.x & 1);                    \
    for (int it = 0; it < ITER; ++it) {                                  \
      _Pragma("unroll") for (int i = 0; i < CH; ++i) { __VA_ARGS__; }         \
    }                                                                    \
    float acc = 0.f;                                                     \
    for (int i = 0; i < CH; ++i) acc += v[i] + (float)u[i];              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc + (float)(m & 3);   \
  }


VK(k_mul_vv, asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[i]) : "v"(a)))
VK(k_mix_lo, asm volatile("v_fma_mix_f32 %0, %0, %1, 0 op_sel_hi:[0,1,0]" : "+v"(v[i]) : "v"(ua)))
VK(k_mix_hi, asm volatile("v_fma_mix_f32 %0, %0, %1, 0 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "+v"(v[i]) : "v"(ua)))
VK(k_mix_f32, asm volatile("v_fma_mix_f32 %0, %0, %1, 0" : "+v"(v[i]) : "v"(a)))

template <int W, int MODE>
__global__ void k_ldsw(float* out, float s) {
  __shared__ float4 tab[64];
  if (threadIdx.x < 64) tab[threadIdx.x] = make_float4(s, s + 1, s + 2, s + 3);
  __syncthreads();
  const int e = MODE == 0 ? 0 : (threadIdx.x % 10) * 3;
  float acc = 0.f;
  for (int it = 0; it < ITER; ++it) {
    float x[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int idx = (e + (i % 3) + (it & 1)) & 63;
      if (W == 8) {
        float2 t;
        asm volatile("ds_read_b64 %0, %1" : "=v"(t) : "v"(idx * 16) : "memory");
        x[i] = t.x;
      } else {
        float4 t;
        asm volatile("ds_read_b128 %0, %1" : "=v"(t) : "v"(idx * 16) : "memory");
        x[i] = t.x;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < CH; ++i) acc += x[i];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

static double g_mhz = 2100.0;

template <typename K>
double run(K k, const char* name, int insts_per_body) {
  float* out;
  hipMalloc(&out, sizeof(float) * BLOCKS * THREADS);
  hipLaunchKernelGGL(k, dim3(BLOCKS), dim3(THREADS), 0, 0, out, 1.0001f);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, dim3(BLOCKS), dim3(THREADS), 0, 0, out, 1.0001f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double waves_per_simd = 3.0 * BLOCKS * THREADS / 64 / 1024;
  const double insts = waves_per_simd * (double)ITER * CH * insts_per_body;  // per SIMD
  const double cyc = ms * 1e-3 * g_mhz * 1e6 / insts;
  printf("%-14s %8.3f ms  %5.2f cyc per wave-instruction per SIMD\n", name, ms, cyc);
  hipFree(out);
  return cyc;
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 3 * sizeof(unsigned long long));
  hipLaunchKernelGGL(k_clock, dim3(BLOCKS), dim3(THREADS), 0, 0, d);
  hipLaunchKernelGGL(k_clock, dim3(BLOCKS), dim3(THREADS), 0, 0, d);
  unsigned long long h[2];
  hipMemcpy(h, d, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  g_mhz = (double)h[0] / ((double)h[1] / 100.0);
  printf("shader clock under load: %.0f MHz\n", g_mhz);
  for (int r = 0; r < 2; ++r) {
    run(k_mul_vv, "v_mul_f32", 1);
    run(k_mix_lo, "fma_mix f16lo", 1);
    run(k_mix_hi, "fma_mix f16hi", 1);
    run(k_mix_f32, "fma_mix f32", 1);
    run(k_ldsw<8, 0>, "ds_read_b64 bc", 1);
    run(k_ldsw<16, 0>, "ds_read_b128 bc", 1);
    run(k_ldsw<8, 1>, "ds_read_b64 10e", 1);
    run(k_ldsw<16, 1>, "ds_read_b128 10e", 1);
  }
  return 0;
}
