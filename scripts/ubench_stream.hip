// Dev microbenchmark: HBM ceilings for the encode's access pattern on one MI355X.
//   copy   : 16 B in -> 16 B out per lane (balanced read/write)
//   enc    : 12 B in -> 16 B out per lane (k_encode_f32's mix: 1.07 GB read, 1.43 GB written)
//   write  : 16 B out per lane only
//   read   : 16 B in per lane, one dword out per block
//   enc nt / write nt : the same with non-temporal stores (__builtin_nontemporal_store)
//   enc4 nt: 4 groups per lane (three 16-byte loads, four non-temporal 16-byte stores)
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_stream.hip -o /tmp/ubench_stream
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

typedef float f3 __attribute__((ext_vector_type(3)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
#define NTS(v, p) __builtin_nontemporal_store((u4)(v), reinterpret_cast<u4*>(p))

__global__ void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}
__global__ void k_enc(const float* __restrict__ in, uint4* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const f3 v = *reinterpret_cast<const f3*>(in + 3 * i);
    out[i] = uint4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), 0x41414141u};
  }
}
__global__ void k_write(uint4* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = uint4{(uint32_t)i, 1u, 2u, 3u};
}
__global__ void k_read(const uint4* __restrict__ in, uint32_t* __restrict__ out, int64_t n) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ void k_enc_nt(const float* __restrict__ in, uint4* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const f3 v = *reinterpret_cast<const f3*>(in + 3 * i);
    NTS((u4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), 0x41414141u}), out + i);
  }
}
__global__ void k_write_nt(uint4* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    NTS((u4{(uint32_t)i, 1u, 2u, 3u}), out + i);
}
__global__ void k_enc4_nt(const float* __restrict__ in, uint4* __restrict__ out, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4* src = reinterpret_cast<const uint4*>(in) + 3 * i;
    const uint4 a = src[0], b = src[1], c = src[2];
    NTS((u4{a.x, a.y, a.z, 1u}), out + 4 * i);
    NTS((u4{a.w, b.x, b.y, 2u}), out + 4 * i + 1);
    NTS((u4{b.z, b.w, c.x, 3u}), out + 4 * i + 2);
    NTS((u4{c.y, c.z, c.w, 4u}), out + 4 * i + 3);
  }
}

int main() {
  const int64_t groups = 256LL * 349526;  // synth1m_256: 256 rows x (1048576 + 2) / 3 groups
  float* fin; uint4 *a, *b; uint32_t* sink;
  CK(hipMalloc(&fin, groups * 12));
  CK(hipMalloc(&a, groups * 16));
  CK(hipMalloc(&b, groups * 16));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipMemset(fin, 0, groups * 12));
  CK(hipMemset(a, 0, groups * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int grid : {4096, 16384, 65536}) {
    for (int kind = 0; kind < 7; ++kind) {
      float best = 1e9f;
      for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(e0, 0));
        if (kind == 0) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a, b, groups);
        if (kind == 1) hipLaunchKernelGGL(k_enc, dim3(grid), dim3(256), 0, 0, fin, b, groups);
        if (kind == 2) hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, b, groups);
        if (kind == 3) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, sink, groups);
        if (kind == 4) hipLaunchKernelGGL(k_enc_nt, dim3(grid), dim3(256), 0, 0, fin, b, groups);
        if (kind == 5) hipLaunchKernelGGL(k_write_nt, dim3(grid), dim3(256), 0, 0, b, groups);
        if (kind == 6) hipLaunchKernelGGL(k_enc4_nt, dim3(grid / 4 > 0 ? grid / 4 : 1), dim3(256), 0, 0, fin, b, groups / 4);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
      }
      const double bytes = kind == 0 ? 32.0 * groups : (kind == 1 || kind == 4 || kind == 6) ? 28.0 * groups : 16.0 * groups;
      const char* nm[] = {"copy 16->16", "enc 12->16", "write 16", "read 16", "enc nt", "write nt", "enc4 nt"};
      printf("grid %6d %-12s %.3f ms  %.0f GB/s\n", grid, nm[kind], best, bytes / best / 1e6);
    }
  }
  return 0;
}
