// fleet_amd/csrc/teacher.hip -- the sampler's mode-1 teacher forward pass on the
// device: uniformSample runs teacher.forward(sample,
// TEMPERATURE, -1, 1) per drawn sample and appends its 10 class probabilities
// to the mini-batch (Server/src/main/c++/cppNN_backend.cpp:596-613).
//
// The teacher is the network built by initSampler (cppNN_backend.cpp:494-502):
//   I1  input 28x28x1
//   C1  convolution 5x5, 8 maps, elu        -> 24x24x8
//   P1  semi_stochastic_pool 3, stride 3    -> 8x8x8
//   C2i convolution 1x1, 16 maps, elu       -> 8x8x16
//   C2  convolution 5x5, 48 maps, elu       -> 4x4x48
//   P2  semi_stochastic_pool 2, stride 2    -> 2x2x48
//   FC2 fully connected 192 -> 10, softmax(temperature)
// network::forward (commonLib/cppNN/network.h:523-585) zeroes every node, copies
// the sample into I1 and, layer by layer, activates the layer (bias + activation)
// and accumulates it into the next one. Every sum below runs in the reference's
// order, one binary32 rounding per multiply and per add (no contraction):
//   convolution k x k (layer.h:805-872, core_math.h dotsum_unwrapped_NxN): per
//     output, input channel k outer and kernel tap i = row*5 + col inner, one
//     running sum from 0;
//   convolution 1x1 (layer.h:873-887): input channel k in order;
//   fully connected (layer.h:200-238, core_math.h dot): 0 + sum_i x_i w_i;
//   softmax::fc (activation.h:271-313): the reference's max scan (max is
//     replaced by in[j]/T), sum of expf(in/T - max), then expf(.)/sum; the
//     layer's bias is not added by softmax.
// One 256-thread block per sample, the layers staged through LDS (31 KB).
//
// Weights: w = the non-null W of network order (mojo `W`: C1 [8][25],
// C2i [16*8] at map + k*16, C2 [16][48][25] at (k*48 + map)*25 + tap,
// FC2 [10][192]), b = the biases of the use_bias() layers in layer order
// (C1 8, C2i 16, C2 48, FC2 10) -- the layout getParams / fleet_model keep.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fleet_codec.h"
#include "kernels.h"
#include "teacher_math.h"

namespace fleet {

namespace teacher {
constexpr int kIn = 28, kC1 = 24, kP1 = 8, kC2 = 4, kP2 = 2;
constexpr int kMaps1 = 8, kMaps2i = 16, kMaps2 = 48, kClasses = 10;
constexpr int kFcIn = kP2 * kP2 * kMaps2;  // 192
constexpr int64_t kW1 = 0, kW2i = kW1 + kMaps1 * 25, kW2 = kW2i + kMaps2i * kMaps1, kWfc = kW2 + kMaps2 * kMaps2i * 25;
constexpr int64_t kWTotal = kWfc + kClasses * kFcIn;  // 21448
constexpr int64_t kB1 = 0, kB2i = kB1 + kMaps1, kB2 = kB2i + kMaps2i, kBfc = kB2 + kMaps2;
constexpr int64_t kBTotal = kBfc + kClasses;  // 82
}  // namespace teacher

__global__ void __launch_bounds__(256) k_teacher_forward(const float* __restrict__ w, const float* __restrict__ b,
                                                         const float* __restrict__ images, int64_t n_images, int F,
                                                         const int32_t* __restrict__ idx, float temperature,
                                                         float* __restrict__ probs, int* __restrict__ err) {
  using namespace teacher;
  __shared__ float s_in[kIn * kIn];
  __shared__ float s_c1[kMaps1 * kC1 * kC1];
  __shared__ float s_p1[kMaps1 * kP1 * kP1];
  __shared__ float s_c2i[kMaps2i * kP1 * kP1];
  __shared__ float s_c2[kMaps2 * kC2 * kC2];
  __shared__ float s_p2[kFcIn];
  __shared__ float s_fc[kClasses];
  const int t = threadIdx.x;
  int64_t row = idx ? (int64_t)idx[blockIdx.x] : (int64_t)blockIdx.x;
  if (row < 0 || row >= n_images) {  // block-uniform
    if (t == 0) atomicOr(err, FLEET_ERRBIT_ARG);
    row = 0;
  }
  for (int i = t; i < kIn * kIn; i += 256) s_in[i] = images[row * F + i];
  __syncthreads();

  // C1: 5x5 over the single input channel, then bias + elu
  for (int o = t; o < kMaps1 * kC1 * kC1; o += 256) {
    const int map = o / (kC1 * kC1), p = o % (kC1 * kC1), y = p / kC1, x = p % kC1;
    const float* wm = w + kW1 + map * 25;
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 25; ++i) acc = acc + s_in[(y + i / 5) * kIn + x + i % 5] * wm[i];
    s_c1[o] = mojo_elu(acc, b[kB1 + map]);
  }
  __syncthreads();

  // P1: semi-stochastic 3x3 pool, stride 3
  for (int o = t; o < kMaps1 * kP1 * kP1; o += 256) {
    const int k = o / (kP1 * kP1), p = o % (kP1 * kP1), j = 3 * (p / kP1), i = 3 * (p % kP1);
    float v[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) v[q] = s_c1[k * kC1 * kC1 + (j + q / 3) * kC1 + i + q % 3];
    s_p1[o] = mojo_semi_pool<3>(v, true);
  }
  __syncthreads();

  // C2i: 1x1 over 8 input channels, then bias + elu
  for (int o = t; o < kMaps2i * kP1 * kP1; o += 256) {
    const int map = o / (kP1 * kP1), p = o % (kP1 * kP1);
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < kMaps1; ++k) acc = acc + s_p1[k * kP1 * kP1 + p] * w[kW2i + map + k * kMaps2i];
    s_c2i[o] = mojo_elu(acc, b[kB2i + map]);
  }
  __syncthreads();

  // C2: 5x5 over 16 input channels (channel outer, tap inner), then bias + elu
  for (int o = t; o < kMaps2 * kC2 * kC2; o += 256) {
    const int map = o / (kC2 * kC2), p = o % (kC2 * kC2), y = p / kC2, x = p % kC2;
    float acc = 0.0f;
    for (int k = 0; k < kMaps2i; ++k) {
      const float* wm = w + kW2 + (int64_t)(k * kMaps2 + map) * 25;
      const float* src = s_c2i + k * kP1 * kP1;
#pragma unroll
      for (int i = 0; i < 25; ++i) acc = acc + src[(y + i / 5) * kP1 + x + i % 5] * wm[i];
    }
    s_c2[o] = mojo_elu(acc, b[kB2 + map]);
  }
  __syncthreads();

  // P2: semi-stochastic 2x2 pool, stride 2
  if (t < kFcIn) {
    const int k = t / (kP2 * kP2), p = t % (kP2 * kP2), j = 2 * (p / kP2), i = 2 * (p % kP2);
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = s_c2[k * kC2 * kC2 + (j + q / 2) * kC2 + i + q % 2];
    s_p2[t] = mojo_semi_pool<2>(v, true);
  }
  __syncthreads();

  // FC2: node[j] = 0 + dot(P2, W row j)
  if (t < kClasses) {
    const float* wr = w + kWfc + (int64_t)t * kFcIn;
    float v = 0.0f;
    for (int i = 0; i < kFcIn; ++i) v = v + s_p2[i] * wr[i];
    s_fc[t] = 0.0f + v;
  }
  __syncthreads();

  // softmax with temperature (one lane: ten values, the reference's order)
  if (t == 0) {
    float in[kClasses];
#pragma unroll
    for (int j = 0; j < kClasses; ++j) in[j] = s_fc[j];
    float mx = in[0];
#pragma unroll
    for (int j = 1; j < kClasses; ++j)
      if (in[j] > mx) mx = in[j] / temperature;
    float denom = 0.0f;
#pragma unroll
    for (int j = 0; j < kClasses; ++j) denom = denom + glibc_expf(in[j] / temperature - mx);
#pragma unroll
    for (int j = 0; j < kClasses; ++j) probs[(int64_t)blockIdx.x * kClasses + j] = glibc_expf(in[j] / temperature - mx) / denom;
  }
}

hipError_t launch_teacher_forward(const float* w, const float* b, const float* images, int64_t n_images, int F,
                                  const int32_t* idx, int B, float temperature, float* probs, int* err,
                                  hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (F < teacher::kIn * teacher::kIn) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_teacher_forward, dim3((unsigned)B), dim3(256), 0, s, w, b, images, n_images, F, idx,
                     temperature, probs, err);
  return hipGetLastError();
}

int64_t teacher_weight_count() { return teacher::kWTotal; }
int64_t teacher_bias_count() { return teacher::kBTotal; }

}  // namespace fleet
