// scripts/ubench3.hip -- per-encoding VALU / LDS issue costs on gfx950 (dev tool).
// Every kernel: 8 waves per SIMD, 8 independent chains per lane. The shader
// clock under load is measured first (s_memtime vs the 100 MHz wall clock) and
// every result is printed in shader cycles per wave-instruction per SIMD.
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
VK(k_mul_lit, asm volatile("v_mul_f32 %0, 0x41200000, %0" : "+v"(v[i])))
VK(k_mul_abs, asm volatile("v_mul_f32_e64 %0, |%0|, %1" : "+v"(v[i]) : "v"(a)))
VK(k_fmac, asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b)))
VK(k_fmamk, asm volatile("v_fmamk_f32 %0, %0, 0x3dcccccd, %1" : "+v"(v[i]) : "v"(b)))
VK(k_fma3, asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b)))
VK(k_cnd_sgpr, asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "s"(m)))
VK(k_bfi, asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(u[i]) : "v"(ua), "v"(ub)))
VK(k_bfe, asm volatile("v_bfe_u32 %0, %0, 3, 8" : "+v"(u[i])))
VK(k_bfe_i, asm volatile("v_bfe_i32 %0, %0, %1, 1" : "+v"(u[i]) : "v"(ua)))
VK(k_and_or, asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(ua), "v"(ub)))
VK(k_lshl_add, asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(u[i]) : "v"(ua)))
VK(k_mulhi, asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[i]) : "v"(ua)))
VK(k_mullo, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(ua)))
VK(k_mad64, {
  unsigned long long r;
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %3" : "=v"(r) : "v"(u[i]), "v"(ua), "v"((unsigned long long)ub) : "s0", "s1");
  u[i] = (unsigned)r;
})
VK(k_add_u32, asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(ua)))
VK(k_and, asm volatile("v_and_b32 %0, %0, %1" : "+v"(u[i]) : "v"(ua)))
VK(k_lshr, asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(u[i])))
VK(k_cvt_u, asm volatile("v_cvt_u32_f32 %0, %1" : "=v"(u[i]) : "v"(v[i])))
VK(k_cvt_f, asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(v[i]) : "v"(u[i])))
VK(k_pk_mul, {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 t = {v[i], a};
  asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(t) : "v"(f2{a, b}));
  v[i] = t.x;
})
VK(k_pk_fma, {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 t = {v[i], a};
  asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(t) : "v"(f2{a, b}), "v"(f2{b, a}));
  v[i] = t.x;
})
VK(k_cmp_e64, {
  unsigned long long r;
  asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(r) : "v"(v[i]), "v"(a));
  m ^= r;
})
VK(k_cvt_f64, {
  double d;
  asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d) : "v"(v[i]));
  asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(v[i]) : "v"(d));
})
VK(k_mul_f64, {
  double d = v[i];
  asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d) : "v"((double)a));
  v[i] = (float)d;
})

// LDS: 10 x 48-B entries; each lane reads entry (lane % 10) (distinct) or entry 0 (broadcast)
template <int MODE>
__global__ void k_lds(float* out, float s) {
  __shared__ float4 tab[64];
  if (threadIdx.x < 64) tab[threadIdx.x] = make_float4(s, s + 1, s + 2, s + 3);
  __syncthreads();
  const int e = MODE == 0 ? 0 : (threadIdx.x % 10) * 3;
  float acc = 0.f;
  for (int it = 0; it < ITER; ++it) {
    float4 x[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int idx = (e + (i % 3) + (it & 1)) & 63;
      asm volatile("ds_read_b128 %0, %1" : "=v"(x[i]) : "v"(idx * 16) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < CH; ++i) acc += x[i].x;
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
  run(k_mul_vv, "v_mul_f32", 1);
  run(k_mul_lit, "v_mul_f32 lit", 1);
  run(k_mul_abs, "v_mul_f32 |x|", 1);
  run(k_fmac, "v_fmac_f32", 1);
  run(k_fmamk, "v_fmamk_f32", 1);
  run(k_fma3, "v_fma_f32", 1);
  run(k_pk_mul, "v_pk_mul_f32", 1);
  run(k_pk_fma, "v_pk_fma_f32", 1);
  run(k_cnd_sgpr, "v_cndmask e64", 1);
  run(k_bfi, "v_bfi_b32", 1);
  run(k_bfe, "v_bfe_u32", 1);
  run(k_bfe_i, "v_bfe_i32", 1);
  run(k_and_or, "v_and_or_b32", 1);
  run(k_lshl_add, "v_lshl_add_u32", 1);
  run(k_mulhi, "v_mul_hi_u32", 1);
  run(k_mullo, "v_mul_lo_u32", 1);
  run(k_mad64, "v_mad_u64_u32", 1);
  run(k_add_u32, "v_add_u32", 1);
  run(k_and, "v_and_b32", 1);
  run(k_lshr, "v_lshrrev_b32", 1);
  run(k_cvt_u, "v_cvt_u32_f32", 1);
  run(k_cvt_f, "v_cvt_f32_u32", 1);
  run(k_cmp_e64, "v_cmp e64", 1);
  run(k_cvt_f64, "cvt f32<->f64", 2);
  run(k_mul_f64, "f64 mul+cvts", 3);
  run(k_lds<0>, "ds_read_b128 bc", 1);
  run(k_lds<1>, "ds_read_b128 10", 1);
  return 0;
}
