// scripts/ubench_chain.hip -- latency of the serial accumulation step A = Q(A + p)
// (phase 2 of k_update_tiled) in isolation on gfx950 (dev tool).
// One wave per block, 256 blocks (one per CU), STEPS dependent steps per lane.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "codec_device.h"

using namespace fleet;

#define STEPS 2048

template <int V>
__global__ void __launch_bounds__(64) k_chain(const float* __restrict__ p_in, float* out, int mode) {
  __shared__ float p[STEPS];
  __shared__ DigitEntry dig[32];
  __shared__ uint32_t ws[64];
  constexpr DigitEntry dtab[32] = FLEET_DIGIT_TABLE;
  for (int i = threadIdx.x; i < STEPS; i += 64) p[i] = p_in[i];
  if (threadIdx.x < 32) dig[threadIdx.x] = dtab[threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x;
  float A = p_in[lane];
  uint32_t flag = 0;
#pragma unroll 4
  for (int k = 0; k < STEPS; ++k) {
    const float s = A + p[(k + lane) & (STEPS - 1)];
    if (V == 0) {
      A = q_fast(s);
    } else if (V == 1) {
      A = q_gen_lat(s);
    } else if (V == 2) {
      A = q_gen(s, dig);
    } else if (V == 3) {
      float o[1], x[1] = {s};
      if (__ballot(!q_ok(s)) == 0) {
        A = q_fast(s);
      } else {
        o[0] = q_gen_lat(s);
        uint32_t in[1] = {f2u(s)};
        if (__ballot(!q_gen_ok(s))) o[0] = q(s);
        A = o[0];
      }
    } else if (V == 4) {
      A = q(s);  // general path (reference-shaped loops)
    } else if (V == 5) {
      A = s * 1.0001f;  // LDS read + add + 1 op: loop floor
    } else if (V == 6) {
      A = q_lat(s);
    } else if (V == 7) {
      flag |= !q_gen_ok(s);
      A = q_lat(s);
    }
  }
  out[blockIdx.x * 64 + lane] = A + (float)flag;
}

int main() {
  const int B = 256;
  float *p, *out;
  hipMalloc(&p, STEPS * sizeof(float));
  hipMalloc(&out, B * 64 * sizeof(float));
  float h[STEPS];
  for (int i = 0; i < STEPS; ++i) {
    // gradient-like mix: mostly small, some > 1 (the accumulator leaves the fast domain)
    unsigned r = (unsigned)i * 2654435761u;
    float m = 1e-3f * (float)((r >> 8) & 0xffff) / 65536.0f;
    h[i] = (r & 1) ? m : -m;
    if ((i % 97) == 0) h[i] = 3.5f;
    if ((i % 89) == 0) h[i] = -3.25f;
  }
  hipMemcpy(p, h, sizeof(h), hipMemcpyHostToDevice);
  const char* names[] = {"q_fast", "q_gen_lat", "q_gen(table)", "q_stage_lat-like", "q general", "floor",
                         "q_lat", "q_lat+flag"};
  for (int v = 0; v < 8; ++v) {
    auto run = [&](void) {
      switch (v) {
        case 0: hipLaunchKernelGGL(k_chain<0>, dim3(B), dim3(64), 0, 0, p, out, 0); break;
        case 1: hipLaunchKernelGGL(k_chain<1>, dim3(B), dim3(64), 0, 0, p, out, 0); break;
        case 2: hipLaunchKernelGGL(k_chain<2>, dim3(B), dim3(64), 0, 0, p, out, 0); break;
        case 3: hipLaunchKernelGGL(k_chain<3>, dim3(B), dim3(64), 0, 0, p, out, 0); break;
        case 4: hipLaunchKernelGGL(k_chain<4>, dim3(B), dim3(64), 0, 0, p, out, 0); break;
        case 5: hipLaunchKernelGGL(k_chain<5>, dim3(B), dim3(64), 0, 0, p, out, 0); break;
        case 6: hipLaunchKernelGGL(k_chain<6>, dim3(B), dim3(64), 0, 0, p, out, 0); break;
        case 7: hipLaunchKernelGGL(k_chain<7>, dim3(B), dim3(64), 0, 0, p, out, 0); break;
      }
    };
    run();
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    run();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-18s %8.3f ms  %7.1f ns/step\n", names[v], ms, ms * 1e6 / STEPS);
  }
  return 0;
}
