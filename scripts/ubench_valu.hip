// scripts/ubench_valu.hip -- VALU issue-rate microbenchmark on gfx950 (dev tool).
// Each kernel runs 8 independent chains per lane x ITER iterations of one
// instruction kind; reports lane-ops/cycle/CU (wave64 full rate = 64/2cyc per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>

#define ITER 4096
#define CH 8

#define KERNEL(name, TY, INIT, BODY)                                        \
  __global__ void name(TY* out, float s) {                                  \
    TY v[CH];                                                               \
    for (int i = 0; i < CH; ++i) v[i] = INIT;                               \
    for (int it = 0; it < ITER; ++it) {                                     \
      _Pragma("unroll") for (int i = 0; i < CH; ++i) { BODY; }              \
    }                                                                       \
    TY acc = v[0];                                                          \
    for (int i = 1; i < CH; ++i) acc = acc + v[i];                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;                       \
  }

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ inline f2 mk2(float a, float b) { f2 r; r.x = a; r.y = b; return r; }

KERNEL(k_mul_f32, float, s + threadIdx.x, asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[i]) : "v"(s)))
KERNEL(k_fma_f32, float, s + threadIdx.x, asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(s)))
KERNEL(k_pk_mul_f32, f2, mk2(s, s + threadIdx.x), asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(v[i]) : "v"(mk2(s, s))))
KERNEL(k_pk_fma_f32, f2, mk2(s, s + threadIdx.x), asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(mk2(s, s))))
KERNEL(k_mul_hi_u32, unsigned, threadIdx.x, asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[i]) : "v"(0x9E3779B9u)))
KERNEL(k_mul_lo_u32, unsigned, threadIdx.x, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[i]) : "v"(0x9E3779B9u)))
KERNEL(k_mul_u24, unsigned, threadIdx.x, asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[i]) : "v"(0x79B9u)))
KERNEL(k_mul_f64, double, s + threadIdx.x, asm volatile("v_mul_f64 %0, %0, %1" : "+v"(v[i]) : "v"((double)s)))
KERNEL(k_fma_f64, double, s + threadIdx.x, asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(v[i]) : "v"((double)s)))
KERNEL(k_cvt_f32_f64, float, s + threadIdx.x, { double d; asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d) : "v"(v[i])); asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(v[i]) : "v"(d)); })
KERNEL(k_med3_f32, float, s + threadIdx.x, asm volatile("v_med3_f32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(s)))
KERNEL(k_cvt_i32_f32, float, s + threadIdx.x, { int t; asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(t) : "v"(v[i])); asm volatile("v_cvt_f32_i32 %0, %1" : "=v"(v[i]) : "v"(t)); })
KERNEL(k_perm, unsigned, threadIdx.x, asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(0x05040302u)))
KERNEL(k_cndmask, float, s + threadIdx.x, asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(s) : "vcc"))
KERNEL(k_add_u32, unsigned, threadIdx.x, asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(7u)))

template <typename T>
double run(void (*k)(T*, float), const char* name, int ops_per_inst, int insts_per_body) {
  int cus = 256, blocks = cus * 8, threads = 256;
  T* out;
  hipMalloc(&out, sizeof(T) * blocks * threads);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 1.0001f);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 1.0001f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double insts = 5.0 * blocks * threads / 64 * (double)ITER * CH * insts_per_body;  // wave-instructions
  double per_s = insts / (ms * 1e-3);
  // wave-instructions per second per SIMD; full rate = clk/2
  double per_simd = per_s / (cus * 4);
  printf("%-14s %8.3f ms  %.3e wave-inst/s/SIMD  -> %.2f GHz-equivalent at 2 cyc/inst  lane-ops/s %.3e\n", name, ms,
         per_simd, per_simd * 2 / 1e9, per_s * 64 * ops_per_inst);
  hipFree(out);
  return per_simd;
}

int main() {
  run(k_mul_f32, "v_mul_f32", 1, 1);
  run(k_fma_f32, "v_fma_f32", 1, 1);
  run(k_pk_mul_f32, "v_pk_mul_f32", 2, 1);
  run(k_pk_fma_f32, "v_pk_fma_f32", 2, 1);
  run(k_mul_hi_u32, "v_mul_hi_u32", 1, 1);
  run(k_mul_lo_u32, "v_mul_lo_u32", 1, 1);
  run(k_mul_u24, "v_mul_u32_u24", 1, 1);
  run(k_mul_f64, "v_mul_f64", 1, 1);
  run(k_fma_f64, "v_fma_f64", 1, 1);
  run(k_cvt_f32_f64, "cvt f32<->f64", 1, 2);
  run(k_med3_f32, "v_med3_f32", 1, 1);
  run(k_cvt_i32_f32, "cvt i32<->f32", 1, 2);
  run(k_perm, "v_perm_b32", 1, 1);
  run(k_cndmask, "v_cndmask", 1, 1);
  run(k_add_u32, "v_add_u32", 1, 1);
  return 0;
}
