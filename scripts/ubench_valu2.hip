// scripts/ubench_valu2.hip -- issue cost of the byte-extraction and bit-assembly forms
// on gfx950 (dev tool): v_bfe / v_lshr / v_and vs the SDWA byte selects, relative to
// v_mul_f32 (2.45 cycles per wave-instruction in profiles/r01/ubench_encoding_costs.log).
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITER 4096
#define CH 8

#define KERNEL(name, BODY)                                                  \
  __global__ void name(unsigned* out, unsigned s) {                         \
    unsigned v[CH];                                                         \
    for (int i = 0; i < CH; ++i) v[i] = s + threadIdx.x * (i + 1);          \
    for (int it = 0; it < ITER; ++it) {                                     \
      _Pragma("unroll") for (int i = 0; i < CH; ++i) { BODY; }              \
    }                                                                       \
    unsigned acc = v[0];                                                    \
    for (int i = 1; i < CH; ++i) acc ^= v[i];                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;                       \
  }

KERNEL(k_mul_f32, asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[i]) : "v"(s)))
KERNEL(k_add_u32, asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(s)))
KERNEL(k_and_b32, asm volatile("v_and_b32 %0, %1, %0" : "+v"(v[i]) : "v"(s)))
KERNEL(k_lshr_b32, asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(v[i])))
KERNEL(k_bfe_u32, asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(v[i])))
KERNEL(k_sdwa_mov, asm volatile("v_mov_b32_sdwa %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "+v"(v[i])))
KERNEL(k_sdwa_add, asm volatile("v_add_u32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "+v"(v[i]) : "v"(s)))
KERNEL(k_sdwa_lshl, asm volatile("v_lshlrev_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(v[i]) : "v"(s)))
KERNEL(k_lshl_or, asm volatile("v_lshl_or_b32 %0, %0, 6, %1" : "+v"(v[i]) : "v"(s)))
KERNEL(k_bfi, asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(v[i]) : "v"(s)))
KERNEL(k_xor, asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(s)))
KERNEL(k_and_or, asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(s)))
KERNEL(k_mad_u24, asm volatile("v_mad_u32_u24 %0, %0, 10, %1" : "+v"(v[i]) : "v"(s)))
KERNEL(k_mul_u24, asm volatile("v_mul_u32_u24 %0, 10, %0" : "+v"(v[i])))
KERNEL(k_cvt_ubyte1, asm volatile("v_cvt_f32_ubyte1 %0, %0" : "+v"(v[i])))
KERNEL(k_cvt_u32_f32, asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(v[i])))
KERNEL(k_cvt_f32_u32, asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(v[i])))
KERNEL(k_mul_hi, asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[i]) : "v"(s)))
KERNEL(k_ashr, asm volatile("v_ashrrev_i32 %0, 31, %0" : "+v"(v[i])))
KERNEL(k_or3, asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(s)))

static float run(void (*k)(unsigned*, unsigned), const char* name, float ref) {
  const int blocks = 256 * 8, threads = 256;
  unsigned* out;
  hipMalloc(&out, sizeof(unsigned) * blocks * threads);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 0x3f800001u);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 0x3f800001u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("%-22s %8.3f ms  %.2f cycles per wave-instruction (v_mul_f32 = 2.45)\n", name, ms,
         ref > 0 ? 2.45 * ms / ref : 2.45);
  hipFree(out);
  return ms;
}

int main() {
  const float ref = run(k_mul_f32, "v_mul_f32", 0);
  run(k_add_u32, "v_add_u32 (VOP2)", ref);
  run(k_and_b32, "v_and_b32 (VOP2)", ref);
  run(k_lshr_b32, "v_lshrrev_b32 (VOP2)", ref);
  run(k_ashr, "v_ashrrev_i32 (VOP2)", ref);
  run(k_xor, "v_xor_b32 (VOP2)", ref);
  run(k_mul_u24, "v_mul_u32_u24 (VOP2)", ref);
  run(k_bfe_u32, "v_bfe_u32 (VOP3)", ref);
  run(k_sdwa_mov, "v_mov_b32_sdwa byte1", ref);
  run(k_sdwa_add, "v_add_u32_sdwa byte2", ref);
  run(k_sdwa_lshl, "v_lshlrev_b32_sdwa", ref);
  run(k_cvt_ubyte1, "v_cvt_f32_ubyte1", ref);
  run(k_lshl_or, "v_lshl_or_b32 (VOP3)", ref);
  run(k_bfi, "v_bfi_b32 (VOP3)", ref);
  run(k_and_or, "v_and_or_b32 (VOP3)", ref);
  run(k_or3, "v_or3_b32 (VOP3)", ref);
  run(k_mad_u24, "v_mad_u32_u24 (VOP3)", ref);
  run(k_mul_hi, "v_mul_hi_u32", ref);
  run(k_cvt_u32_f32, "v_cvt_u32_f32", ref);
  run(k_cvt_f32_u32, "v_cvt_f32_u32", ref);
  return 0;
}
