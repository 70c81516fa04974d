// scripts/ubench2.hip -- select / hazard / latency microbenchmarks on gfx950 (dev tool).
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITER 4096

// throughput: 8 independent chains per lane, 8 waves per SIMD
__global__ void k_cnd_vcc(float* out, float s) {
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = s + threadIdx.x + i;
  asm volatile("v_cmp_gt_f32 vcc, %0, %1" ::"v"(v[0]), "v"(s) : "vcc");
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(s));
  }
  float a = 0;
  for (int i = 0; i < 8; ++i) a += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

__global__ void k_cnd_sgpr(float* out, float s) {
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = s + threadIdx.x + i;
  unsigned long long m = __ballot(v[0] > s);
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(v[i]) : "v"(s), "s"(m));
  }
  float a = 0;
  for (int i = 0; i < 8; ++i) a += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

// v_cmp writing an SGPR pair immediately consumed by v_cndmask (the compiler's pattern)
__global__ void k_cmp_cnd(float* out, float s) {
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = s + threadIdx.x + i;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float w = v[i] * 1.0001f;
      v[i] = (w > s) ? w : v[i];
    }
  }
  float a = 0;
  for (int i = 0; i < 8; ++i) a += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

__global__ void k_med3(float* out, float s) {
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = s + threadIdx.x + i;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(s), "v"(v[(i + 1) & 7]));
  }
  float a = 0;
  for (int i = 0; i < 8; ++i) a += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

// latency: ONE dependent chain per lane, 1 wave per SIMD (grid = 256 CUs x 4 waves)
__global__ void k_lat_fma(float* out, float s) {
  float v = s + threadIdx.x;
  for (int it = 0; it < ITER * 8; ++it) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(v) : "v"(s));
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}
__global__ void k_lat_mul(float* out, float s) {
  float v = s + threadIdx.x;
  for (int it = 0; it < ITER * 8; ++it) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v) : "v"(s));
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k_lat_pkfma(float* out, float s) {
  f2 v;
  v.x = s + threadIdx.x;
  v.y = s;
  f2 c;
  c.x = s;
  c.y = s;
  for (int it = 0; it < ITER * 8; ++it) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(v) : "v"(c));
  out[blockIdx.x * blockDim.x + threadIdx.x] = v.x + v.y;
}
__global__ void k_lat_cnd(float* out, float s) {
  float v = s + threadIdx.x;
  unsigned long long m = __ballot(v > s);
  for (int it = 0; it < ITER * 8; ++it) asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(v) : "v"(s), "s"(m));
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}
__global__ void k_lat_cvt(float* out, float s) {
  float v = s + threadIdx.x;
  for (int it = 0; it < ITER * 4; ++it) {
    unsigned t;
    asm volatile("v_cvt_u32_f32 %0, %1" : "=v"(t) : "v"(v));
    asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(v) : "v"(t));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}
__global__ void k_lat_mulhi(float* out, float s) {
  unsigned v = threadIdx.x;
  for (int it = 0; it < ITER * 8; ++it) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v) : "v"(0x9E3779B9u));
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)v;
}

double run(void (*k)(float*, float), const char* name, int blocks, int threads, double wave_insts_per_thread) {
  float* out;
  hipMalloc(&out, sizeof(float) * blocks * threads);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 1.0001f);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 1.0001f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double waves = 3.0 * blocks * threads / 64;
  double per_wave_ns = ms * 1e6 / (waves / (256.0 * 4)) / wave_insts_per_thread;  // ns per inst per SIMD-slot
  printf("%-12s %8.3f ms   %.3f ns per wave-inst per SIMD (x2.2GHz = %.2f cyc)\n", name, ms, per_wave_ns,
         per_wave_ns * 2.2);
  hipFree(out);
  return ms;
}

int main() {
  // throughput (8 waves/SIMD)
  run(k_cnd_vcc, "cnd_vcc", 2048, 256, ITER * 8);
  run(k_cnd_sgpr, "cnd_sgpr", 2048, 256, ITER * 8);
  run(k_cmp_cnd, "mul+cmp+cnd", 2048, 256, ITER * 8 * 3);
  run(k_med3, "med3", 2048, 256, ITER * 8);
  // latency (1 wave/SIMD)
  run(k_lat_fma, "lat fma", 256, 256, ITER * 8);
  run(k_lat_mul, "lat mul", 256, 256, ITER * 8);
  run(k_lat_pkfma, "lat pk_fma", 256, 256, ITER * 8);
  run(k_lat_cnd, "lat cnd", 256, 256, ITER * 8);
  run(k_lat_cvt, "lat cvt2", 256, 256, ITER * 8);
  run(k_lat_mulhi, "lat mulhi", 256, 256, ITER * 8);
  return 0;
}
