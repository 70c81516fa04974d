// fleet_amd/csrc/kernels.h -- internal launchers (fleet_codec.cpp <-> kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

// device error bits (atomicOr into the context's error word, read back by fleet_check)
#define FLEET_ERRBIT_BASE64 1
#define FLEET_ERRBIT_LAYOUT 2
#define FLEET_ERRBIT_ARG 4
#define FLEET_ERRBIT_SYNC 8  // a cross-block hand-off timed out (Kardam reduce blocks)

namespace fleet {

// FLEET_MAX_HEADERS of fleet_codec.h (checked there): header positions a kernel may
// hold in LDS
constexpr int kMaxHeaderSlots = 4096;
// segments of descentNative's model step (k_descent): kind 0 = weight block,
// 1 = fully-connected bias block; offsets in floats
constexpr int kMaxDescentSegs = 64;
struct DescentSegs {
  int n;
  int kind[kMaxDescentSegs];
  int64_t grad_off[kMaxDescentSegs], model_off[kMaxDescentSegs], len[kMaxDescentSegs];
};
hipError_t launch_descent(float* weights, float* fc_bias, const float* grad, const DescentSegs& segs, float lr,
                          hipStream_t s);
hipError_t launch_update(const uint8_t* uploads, size_t pitch, int M, const double* d_dampen, double inv_avg,
                         int64_t n_up, int64_t g_begin, int64_t g_end, const int32_t* d_hdr_block,
                         uint8_t* merged, float* merged_f32, int* d_err, hipStream_t s);
// Kardam's side outputs of the fused update (k_update_mixed<256, true>, the tiles, the
// pipelined tiles): per client c and flat value (upload positions that are neither header slots nor past the walk)
//   G = Q(f32(f64(p) lr))            the decoded Kardam.setGrad text (p = stage B)
//   D = Q(G - prev[c])               the decoded g.subtract(prev) text (has_prev[c])
// partials[(c * n_waves + w) * 2 + {0, 1}] = per-wave (or per-tile) sums of (double)(G*G),
// (double)(D*D); g_out (nullable) = G in upload
// coordinates (M rows of vpitch floats; may be prev itself).
// launch_update_kardam: *n_waves = partial slots per client (sizing call: partials
// NULL), norms = M x *norm_parts pairs of sums, added in order on the host;
// *flag_slots = the u32 tile flags the pipelined form needs (kd_flags: zeroed once at
// allocation, kd_epoch: a value new to them, per launch). The plan
// overrides are the caller's one snapshot, passed to the sizing call and the launch
// alike, so a concurrent fleet_set_plan cannot change the grid between the two.
struct PlanOverrides;
struct KardamOut {
  double lr;
  const float* prev;
  const uint8_t* has_prev;
  size_t vpitch;
  float* g_out;
  double* partials;
};
hipError_t launch_update_kardam(const uint8_t* uploads, size_t pitch, int M, const double* d_dampen, double inv_avg,
                                int64_t n_up, int64_t g_begin, int64_t g_end, const int32_t* d_hdr_block,
                                uint8_t* merged, float* merged_f32, int* d_err, const KardamOut& kd, int* n_waves,
                                double* norms, int* norm_parts, int* flag_slots, uint32_t* kd_flags,
                                uint32_t kd_epoch, const PlanOverrides& o, hipStream_t s,
                                uint32_t kd_wait_skew = 0);
// Launch-plan overrides: experiments, and the tests that run every launch variant on
// small inputs. Process-wide; set by fleet_set_plan (spec "key=value,..." -- update=
// auto|stream|tiled|pipe, grid=auto|plain|lanes|balanced, fused=on|off,
// stage_threads=N, stage_pieces=N, tile=auto|classic|flat|weave6|8, flat_w2=auto|N,
// tile_enc_prio=auto|0..3,
// tile_enc_rows=N) or, once at first
// use, from FLEET_EXPERIMENTS (the
// same spec). The default (empty spec) is the measured plan.
struct PlanOverrides {
  int update = 0;         // 0 auto, 1 stream grid, 2 64-group tiles, 3 16-group pipelined tiles
  int grid = 0;           // stream grid: 0 auto, 1 a group per lane everywhere, 2 a value per lane everywhere
  int tile = 0;           // tiles: 0 auto (flat alone, classic fused), 1 classic, 2 flat, 6/8 woven
  int flat_w2 = 0;        // flat tiles: width of the tiles after the whole 64-group rounds (0 auto)
  int tile_enc_prio = -1; // tiled / flat fused step: the encode blocks' issue priority (-1 auto)
  int tile_enc_rows = 0;  // fused steps (tiles and stream): rows per encode block (0 auto: 24)
  int fused = 1;          // 0: the pipelined step as two launches (update, then encode)
  int stage_threads = 0;  // host staging copy threads (0 auto)
  int stage_pieces = 0;   // host staging H2D parts (0 auto)
};
PlanOverrides plan_overrides();
int set_plan_overrides(const char* spec, std::string* err);  // 0, or -1 (nothing changed)
std::string plan_spec();                                     // normalised active spec, "" = default
// names of the kernels launch_update / launch_update_encode pick for `groups` groups
std::string update_kernel_name(int64_t groups);
void update_plan_grid(int64_t groups, int* kind, int64_t* blocks, int64_t* n_a, int64_t* n_w, int64_t* n_n);
std::string update_encode_kernel_name(int64_t groups);
hipError_t launch_update_encode(const uint8_t* uploads, size_t pitch, int M, const double* d_dampen, double inv_avg,
                                int64_t n_up, const int32_t* d_hdr_block, uint8_t* merged, float* merged_f32,
                                int* d_err, const float* values, size_t vpitch, uint8_t* enc_out, hipStream_t s);
hipError_t launch_encode_f32(const float* values, int64_t n, size_t vpitch, int rows, uint8_t* out, size_t pitch,
                             hipStream_t s);
hipError_t launch_encode_minibatch(const float* images, int64_t n_images, int F, const int32_t* labels,
                                   const int32_t* idx, int B, const float* teacher, int NL, const float header[7],
                                   uint8_t* out, int* err, hipStream_t s);
// the sampler's mode-1 teacher forward (teacher.hip): probs[b*10 + j] for sample
// idx[b] (idx == nullptr: sample b) of the n_images x F rows
hipError_t launch_teacher_forward(const float* w, const float* b, const float* images, int64_t n_images, int F,
                                  const int32_t* idx, int B, float temperature, float* probs, int* err,
                                  hipStream_t s);
int64_t teacher_weight_count();
int64_t teacher_bias_count();
hipError_t launch_encode_model_params(const float* weights, int64_t n_w, const float* biases, int64_t n_b, int64_t reps,
                                      uint8_t* out, hipStream_t s);
hipError_t launch_encode_i32(const int32_t* codes, int64_t n, uint8_t* out, hipStream_t s);
hipError_t launch_decode(const uint8_t* text, int64_t n, size_t pitch, int rows, void* out, size_t vpitch,
                         int as_codes, int* d_err, hipStream_t s);
hipError_t launch_elementwise(const uint8_t* a, const uint8_t* b, int op, double scale, int64_t n, uint8_t* out,
                              int* d_err, hipStream_t s);
hipError_t launch_norm_partials(const uint8_t* a, int64_t n, double* partials, int* nblocks, int* d_err,
                                hipStream_t s);
hipError_t launch_kardam_grads(const uint8_t* uploads, size_t pitch, int M, const int32_t* d_hdr, int n_hdr,
                               int64_t n_flat, const double* d_dampen, double lr, const uint8_t* prev,
                               size_t prev_pitch, const uint8_t* d_has_prev, uint8_t* g_out, size_t g_pitch,
                               double* partials, int* nblocks, int* d_err, hipStream_t s);
hipError_t launch_flat(const uint8_t* up, const int32_t* d_hdr, int n_hdr, int64_t n_flat, uint8_t* out,
                       int* d_err, hipStream_t s);
hipError_t launch_merge(const uint8_t* up, const uint8_t* flat, const int32_t* d_hdr, int n_hdr, int64_t walk_end,
                        int64_t n_up, uint8_t* out, int* d_err, hipStream_t s);
hipError_t launch_layout_parse(const uint8_t* up, int64_t n, int cap, int32_t* out, hipStream_t s);
hipError_t launch_synth(uint64_t seed, int client0, int64_t elem0, int rows, int64_t n_up, float* out, size_t vpitch,
                        const int32_t* d_hpos, const float* d_hval, int n_hdr, hipStream_t s);
hipError_t launch_digest(int fn, unsigned long long* out, hipStream_t s);
#ifdef FLEET_TRACE
hipError_t set_trace_buffer(void* p);  // dev builds: the tile kernels' phase trace (FLEET_WTRACE)
#endif
}  // namespace fleet
