/*
 * include/fleet_codec.h -- C-ABI of the MI355X-native FLeet gradient codec and
 * server-side aggregation path (libfleetcodec.so).
 *
 * This is the drop-in boundary under the reference's JNI layer. Every entry
 * point below replaces a native function of the reference's server backend
 * (libnative.so built from Server/src/main/c++/cppNN_backend.cpp), or the
 * call sequence CppNNUpdater.update drives through them, and produces the
 * same bytes. The JNI shim (fleet_amd/csrc/jni_shim.cpp, libfleet_native.so)
 * re-exports the reference's Java_* symbols on top of this ABI; see
 * INTEGRATION.md for the Java-side binding.
 *
 * Conventions
 *   - Plain pointers and sizes; no torch/HIP types. `stream` arguments are a
 *     hipStream_t passed as void* (NULL = the null/default stream). Host-buffer
 *     entry points run on the context's own stream and return synchronously.
 *   - "Base64" buffers are the reference's wire format: Base64 (RFC 4648
 *     alphabet; '-' and '_' accepted as 62/63 on input, from_base64 at Base64.cpp:20-27) of
 *     little-endian int32 decimal fixed-point codes (Base64::float2int,
 *     Base64.cpp:48-78). Host buffers are NOT NUL-terminated.
 *   - Every function returns FLEET_OK (0) or a negative FLEET_ERR_* code;
 *     fleet_last_error() gives a message. The reference has no error
 *     reporting (malformed input is UB there); here it is rejected.
 *   - Thread safety: a context serialises its own calls with an internal
 *     mutex (the reference serialises all updater natives under
 *     `synchronized(acc)`, CppNNUpdater.java:259,333). Use one context per
 *     thread/GPU for concurrency.
 *   - Input contract: Base64 text produced by Base64::encode -- length a
 *     multiple of 4, '=' only as trailing padding. Anything else returns
 *     FLEET_ERR_BASE64 (the reference would silently drop bytes).
 */
#ifndef FLEET_CODEC_H
#define FLEET_CODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLEET_OK 0
#define FLEET_ERR_ARG (-1)      /* bad argument / size mismatch */
#define FLEET_ERR_BASE64 (-2)   /* text outside the Base64::encode output contract */
#define FLEET_ERR_LAYOUT (-3)   /* gradient layout header inconsistent (network.h:1038-1056) */
#define FLEET_ERR_HIP (-4)      /* HIP runtime failure (or no GPU) */
#define FLEET_ERR_NOMEM (-5)
#define FLEET_ERR_CAPACITY (-6) /* output buffer too small; *out_len holds the size needed */

#define FLEET_MAX_HEADERS 4096

typedef struct fleet_ctx fleet_ctx;

/* Library / context ------------------------------------------------------ */
const char* fleet_version(void);
int fleet_create(int device, fleet_ctx** out);
void fleet_destroy(fleet_ctx* ctx);
const char* fleet_last_error(const fleet_ctx* ctx);
int fleet_sync(fleet_ctx* ctx, void* stream);

/* Base64 length of n int32/fp32 values: 4*ceil(4n/3) (Base64.cpp:129-136). */
size_t fleet_b64_len(size_t n_values);
/* Number of int32 values carried by a Base64::encode output of length len. */
size_t fleet_b64_count(size_t len);

/* Gradient layout (network.h:1038-1056): [nW,(size_i,dW_i..)*,nB,(size_j,db_j..)*].
 * Writes the sorted header slot positions; returns FLEET_OK and *n_headers,
 * *n_up (total floats). */
int fleet_layout_from_sizes(const int32_t* w_sizes, int n_w, const int32_t* b_sizes, int n_b,
                            int32_t* header_pos, int cap, int* n_headers, size_t* n_up);
/* Same, parsed from an upload (Base64 host buffer) by decoding its header
 * slots on the device, exactly as network::flatGrad walks them (:1206-1223).
 * *n_up = the floats the walk covers (= the upload's count for gradients()
 * output); slots past it are carried from the last upload, like headers. */
int fleet_layout_parse(fleet_ctx* ctx, const char* upload, size_t len, int32_t* header_pos, int cap,
                       int* n_headers, size_t* n_up);

/* Codec (Base64.cpp) -- host buffers ------------------------------------- */
/* Base64::encode(std::vector<float>) (:140-142) */
int fleet_encode_f32(fleet_ctx* ctx, const float* values, size_t n, char* out, size_t cap, size_t* out_len);
/* Base64::encode(std::vector<int>) (:145-151) */
int fleet_encode_i32(fleet_ctx* ctx, const int32_t* codes, size_t n, char* out, size_t cap, size_t* out_len);
/* Base64::decodeFloat (:207-209) */
int fleet_decode_f32(fleet_ctx* ctx, const char* text, size_t len, float* out, size_t cap, size_t* n_out);
/* Base64::decodeInt (:211-219) */
int fleet_decode_i32(fleet_ctx* ctx, const char* text, size_t len, int32_t* out, size_t cap, size_t* n_out);

/* Per-op JNI replacements (cppNN_backend.cpp) -- host Base64 buffers ------ */
/* Java_apps_cppNN_CppNNUpdater_getFlatGradient (:701-720) */
int fleet_flat_gradient(fleet_ctx* ctx, const char* g, size_t len, char* out, size_t cap, size_t* out_len);
/* Java_apps_cppNN_CppNNUpdater_mergeFlatGradient (:722-750) */
int fleet_merge_flat_gradient(fleet_ctx* ctx, const char* g, size_t glen, const char* flat, size_t flen,
                              char* out, size_t cap, size_t* out_len);
/* Java_utils_ByteVec_scalarMulNative (:753-777) */
int fleet_scalar_mul(fleet_ctx* ctx, const char* v, size_t len, double a, char* out, size_t cap,
                     size_t* out_len);
/* Java_utils_ByteVec_addNative (:797-846) */
int fleet_add(fleet_ctx* ctx, const char* a, size_t alen, const char* b, size_t blen, char* out, size_t cap,
              size_t* out_len);
/* Java_utils_ByteVec_subtractNative (:848-892) */
int fleet_subtract(fleet_ctx* ctx, const char* a, size_t alen, const char* b, size_t blen, char* out,
                   size_t cap, size_t* out_len);
/* Java_utils_ByteVec_getNorm (:779-795): sqrt(sum_i (double)(x_i*x_i)) in index order */
int fleet_norm(fleet_ctx* ctx, const char* v, size_t len, double* out);

/* The fused update -- host buffers ---------------------------------------
 * One call = the aggregation part of CppNNUpdater.update (CppNNUpdater.java:
 * 420-509): for the M picked uploads in order,
 *   pickedGrad = getFlatGradient(g_i).scalarMultiply(dampen[i]); avg += pickedGrad
 *   merged = mergeFlatGradient(g_{M-1}, avg.scalarMultiply(1.0/M))
 * with every intermediate re-quantised exactly as the per-op JNI chain does.
 * All uploads must share one layout and length. `merged` receives the
 * Base64 the reference returns; `merged_f32` (nullable, n_up floats) receives
 * Base64::decodeFloat(merged), i.e. what descentNative decodes (:336). */
int fleet_update(fleet_ctx* ctx, const char* const* uploads, const size_t* lens, int M, const double* dampen,
                 char* merged, size_t cap, size_t* out_len, float* merged_f32);
/* The same update spread over the GPUs of a node from ONE host process
 * (SURVEY.md §8e element sharding; the reference server is one JVM calling
 * its natives under synchronized(acc), CppNNUpdater.java:333,420-509).
 * ctxs = n_ctx distinct contexts, one per device. Context k takes a
 * contiguous, balanced range of the 16-char / 3-value groups: on its own
 * thread it copies that column window of every upload into its pinned
 * staging, H2Ds it over its own PCIe link, runs the exact chain there and
 * D2Hs its merged slice straight into `merged` / `merged_f32` (disjoint byte
 * ranges). No collective and no reduction crosses devices, so the output is
 * byte-identical to fleet_update's. Errors are reported on ctxs[0]
 * (fleet_last_error), Base64 errors first. */
int fleet_update_multi(fleet_ctx* const* ctxs, int n_ctx, const char* const* uploads, const size_t* lens, int M,
                       const double* dampen, char* merged, size_t cap, size_t* out_len, float* merged_f32);
/* fleet_update / fleet_update_multi over uploads stored as M rows `row_pitch`
 * bytes apart (row i = upload i, `len` Base64 chars): the ingress of a caller
 * that deserialises the uploads into one buffer (a Java direct ByteBuffer,
 * INTEGRATION.md). When the whole row range lies inside ONE live
 * fleet_host_register registration every context DMAs its column window
 * straight from it -- no host copy at all; otherwise the rows are staged as
 * in fleet_update. */
int fleet_update_rows(fleet_ctx* ctx, const char* rows, size_t row_pitch, size_t len, int M, const double* dampen,
                      char* merged, size_t cap, size_t* out_len, float* merged_f32);
int fleet_update_rows_multi(fleet_ctx* const* ctxs, int n_ctx, const char* rows, size_t row_pitch, size_t len, int M,
                            const double* dampen, char* merged, size_t cap, size_t* out_len, float* merged_f32);
/* Page-lock (hipHostRegister, portable to every device) / release a long-lived
 * host buffer, e.g. the upload rows of fleet_update_rows. The registrations
 * are tracked process-wide: registering a range that overlaps a recorded
 * registration releases the old one first. Contract: unregister BEFORE the
 * memory is freed. The library cannot tell a registration whose memory was
 * freed and reused (a collected Java direct buffer, a new allocation at the
 * same addresses) from a live one: rows inside it would be DMA'd from the
 * stale pinned pages. */
int fleet_host_register(fleet_ctx* ctx, void* ptr, size_t bytes);
int fleet_host_unregister(fleet_ctx* ctx, void* ptr);
/* How the last host-buffer update on ctx (fleet_update*, its window on this context)
 * reached HBM: FLEET_INGRESS_STAGED (copied into the context's pinned staging),
 * FLEET_INGRESS_PINNED (one DMA straight from registered rows), or
 * FLEET_INGRESS_NONE before any. ctx NULL: the process's most recent such update
 * on any context (e.g. those of the JNI shim). Diagnostics and tests. */
#define FLEET_INGRESS_NONE 0
#define FLEET_INGRESS_STAGED 1
#define FLEET_INGRESS_PINNED 2
int fleet_last_ingress(fleet_ctx* ctx);

/* Device-resident entry points (all buffers are device pointers) ----------
 * Uploads are stored as M rows of `pitch` bytes (pitch >= 16*ceil(len/16),
 * multiple of 16); each row holds `len` Base64 chars. group_begin/group_end
 * select the 16-char / 3-value groups this call processes (element-range
 * sharding; [0, ceil(len/16)) = everything). `dampen` is a host array of M
 * doubles. Outputs are written for the selected groups only: merged Base64
 * at byte 16*g, merged_f32 (nullable) at value 3*g.
 * Only bytes [16*group_begin, 16*group_end) of each row (and of d_merged,
 * values [3*group_begin, 3*group_end) of d_merged_f32) are dereferenced, so a
 * rank holding just its window of every upload passes the window's address
 * minus 16*group_begin (3*group_begin floats for merged_f32) and pitch >=
 * 16*(group_end - group_begin): fleet_amd/shard.py does exactly that.
 * Graph capture: the dampen and header words live in ONE device buffer per
 * context, re-uploaded (synchronously) whenever a call passes different ones.
 * Every graph captured on the context therefore replays with the parameters of
 * the context's latest call, and a capture cannot introduce new parameters
 * (FLEET_ERR_ARG): make one eager call with them first, and do not change them
 * while captured graphs that must keep the old ones are still replayed. */
int fleet_update_device(fleet_ctx* ctx, const void* d_uploads, size_t pitch, size_t len, int M,
                        const double* dampen, const int32_t* header_pos, int n_headers, size_t group_begin,
                        size_t group_end, void* d_merged, void* d_merged_f32, void* stream);
/* A pipelined step of the device-resident path: fleet_update_device over the
 * whole uploads in d_uploads AND fleet_encode_device of the next batch's M rows
 * of fp32 (d_values, n values, vpitch floats per row) into d_next_uploads (same
 * pitch; must not overlap d_uploads), in ONE launch when the update runs on the
 * stream grid (the aggregation is VALU-bound, the client encode HBM-bound: they
 * share the CUs), else the two kernels back to back. Results equal the two
 * calls' results. Replaces nothing in the reference (its clients encode on
 * their own devices); the bench's steady-state step. */
int fleet_update_encode_device(fleet_ctx* ctx, const void* d_uploads, size_t pitch, size_t len, int M,
                               const double* dampen, const int32_t* header_pos, int n_headers, void* d_merged,
                               void* d_merged_f32, const void* d_values, size_t vpitch, void* d_next_uploads,
                               void* stream);
/* fleet_update_device plus Kardam's bookkeeping of the same picked uploads
 * (CppNNUpdater.java:463-481, Kardam.java:48-106) as side
 * outputs of the one pass over the uploads (no second read of them):
 *   G_c = decodeFloat(getFlatGradient(u_c).scalarMultiply(dampen[c]).scalarMultiply(lr))
 *   norm_g[c]    = G_c's getNorm
 *   norm_diff[c] = getNorm(g_c.subtract(prev_c)) when has_prev[c] (else NaN)
 * with prev_c = the worker's previous G (d_prev: M rows of vpitch floats in
 * upload coordinates, header slots ignored; NULL = none) and, when d_g_out is
 * given, this round's G written there in the same layout (the next round's
 * prev; d_g_out may be d_prev itself: G then replaces prev in place). Whole
 * uploads (all groups); synchronous (the norms are host outputs);
 * not for graph capture. Norms: fixed-order partial sums of the reference's
 * fp64 loop (1e-12 relative, like fleet_norm). */
int fleet_update_kardam_device(fleet_ctx* ctx, const void* d_uploads, size_t pitch, size_t len, int M,
                               const double* dampen, const int32_t* header_pos, int n_headers, double lr,
                               const void* d_prev, const uint8_t* has_prev, void* d_g_out, size_t vpitch,
                               void* d_merged, void* d_merged_f32, double* norm_g, double* norm_diff, void* stream);
/* Client-side encode of M fp32 buckets (rows of `n` floats, `vpitch` floats
 * apart) into Base64 rows of `pitch` bytes: Base64::encode(vector<float>) per row. */
int fleet_encode_device(fleet_ctx* ctx, const void* d_values, size_t n, size_t vpitch, int M, void* d_out,
                        size_t pitch, void* stream);
/* Base64 rows -> fp32 (decodeFloat) per row. */
int fleet_decode_device(fleet_ctx* ctx, const void* d_text, size_t len, size_t pitch, int M, void* d_values,
                        size_t vpitch, void* stream);
/* Deterministic synthetic gradient buckets on the device (SURVEY.md §8d value
 * mix; Philox4x32-10 keyed by seed, counter = (element, client)), with the
 * given layout's header values written in place. Rows of `vpitch` floats. */
int fleet_synth_device(fleet_ctx* ctx, uint64_t seed, int M, int client0, const int32_t* header_pos,
                       const float* header_val, int n_headers, size_t n_up, void* d_values, size_t vpitch,
                       void* stream);
/* The same for a column window of a larger synthetic problem: values n_up columns
 * from element elem0 (the counter is the global element index, so a rank's window
 * holds exactly the fixed problem's values there); header_pos in window coordinates. */
int fleet_synth_window_device(fleet_ctx* ctx, uint64_t seed, int M, int client0, size_t elem0,
                              const int32_t* header_pos, const float* header_val, int n_headers, size_t n_up,
                              void* d_values, size_t vpitch, void* stream);
/* Returns FLEET_ERR_BASE64 / FLEET_ERR_LAYOUT if a device-resident call
 * (fleet_*_device) since the last check saw malformed text or a header that
 * differs from the last upload's (synchronises the stream), and clears the
 * flag. Device-resident calls keep their parameters and error flag in buffers
 * of their own, so host-buffer calls on the same context (its own stream) may
 * be issued while device-resident work is still in flight, and a grown
 * parameter buffer that a captured HIP graph may reference stays allocated
 * until fleet_destroy. */
int fleet_check(fleet_ctx* ctx, void* stream);

/* Self-test of the device codec arithmetic over whole input domains: an
 * order-independent 64-bit digest sum_i splitmix64(i<<32 | f(i)) of
 *   fn 0: int2float over all 2^32 codes      fn 1: float2int over all 2^32 bit patterns
 *   fn 2: Q fast path over |x| < 1           fn 3: int2float fast path (codes % 10 == 0)
 *   fn 4: t/10 (div10) for 1e-30 <= t < inf  fn 5: packed Q fast path
 *   fn 6: variable-length Q (-1e8 < x < 1e9)  fn 7: variable-length int2float (all codes)
 *   fn 8: packed fn 6 on (x, -x/4)            fn 9: packed fn 7 on (c, c*2654435761)
 *   fn 10: variable-length float2int (-1e8 < x < 1e9)   fn 11: float2int fast path (|x| < 1)
 *   fn 12: select-chain Q of the serial accumulation (-1e8 < x < 1e9; same digest as fn 6)
 *   fn 13: multiplier-table Q (as fn 6)   fn 14: multiplier-table int2float (as fn 7)
 *   fn 15: multiplier-table float2int (as fn 10)   fn 16: scalar Q fast path (as fn 2)
 *   fn 17: one-lookup latency Q (q_xl) on |x| < 1e8, fn 12 elsewhere (as fn 6)
 *   fn 18: the teacher forward's expf (glibc 2.35 restated) over all 2^32 inputs,
 *          NaN results as 0x7fc00000 (the libm expf digest of tests/native/digest_ref.cpp)
 *   fn 19: byte-table Q of the stream kernel (q_d16 + compare fix-up; as fn 6)
 *   fn 20: byte-table float2int of the client encode (enc_d16; as fn 10)
 *   fn 21: the serial accumulation's Q with VarEntry digit offsets (var_d16; as fn 6)
 *   fn 22: the model-version copy's strtof("%.6g") round trip over every finite
 *          binary32 (decimal6.h; against libc's snprintf/strtof)
 * computed on the GPU; compare with the oracle's digests. */
int fleet_selftest_digest(fleet_ctx* ctx, int fn, uint64_t* out);

/* DISTILLATION_MODE=1 model codec -- host buffers ----
 * `weights` = the model's W matrices concatenated in W order, `dims` =
 * n_mats x {cols, rows, chans} (W matrices are not channel-aligned: each is
 * cols*rows*chans floats). */
/* network::quantization_weight_model (commonLib/cppNN/network.h:1683-1774,
 * core_math.h:881-912) on a copy of the weights, then getParams' first-occurrence
 * dictionary (float_vector_find, network.h:594-608, |a-b| < 1e-8f) and the
 * selected-index set (network.h:641-692). Outputs, each nullable: quantized[n]
 * (the weights the text describes), dict[n] (entries in creation order, *n_dict
 * of them), index[n] (the printed index; -1 for NaN/inf weights). */
int fleet_model_quantize_index(fleet_ctx* ctx, const float* weights, const int32_t* dims, int n_mats,
                               float* quantized, float* dict, int* n_dict, int32_t* index);
/* The DISTILLATION_MODE=1 weights section of getParams (network.h:641-692) for
 * these weights: "n\nU\n", U pairs "k\nvalue\n" (value as `ostream << float`,
 * i.e. %g), one line of "index " per matrix -- the bytes the reference emits
 * after the bias lines (getParametersNative, Server/.../cppNN_backend.cpp:244-280). */
int fleet_model_weights_text(fleet_ctx* ctx, const float* weights, const int32_t* dims, int n_mats, char* out,
                             size_t cap, size_t* out_len);
/* network::read's DISTILLATION_MODE=1 weights branch (network.h:958-997): such a
 * section back to weights (W[i] = value of the index's dictionary key; a key
 * the dictionary lacks gives 0.0f, std::map::operator[]). */
int fleet_model_read_weights(fleet_ctx* ctx, const char* text, size_t len, const int32_t* dims, int n_mats,
                             float* weights_out);

/* descentNative's DISTILLATION_MODE=1 model copy (Server/src/main/c++/
 * cppNN_backend.cpp:355-372: cnnNew->read(cnn.getParams()) of the unquantised
 * model, network.h:611-706 + 956-997): every weight becomes the %g/strtof
 * round trip of its first-occurrence dictionary entry (|a-b| < 1e-8f), every
 * bias the round trip of itself. The O(n*U) dictionary scans of the reference
 * become a device sort, and the decimal round trips run on the device too
 * (exact integer arithmetic, checked against libc's snprintf/strtof on every
 * finite binary32). Non-finite weights or biases: FLEET_ERR_ARG (the
 * reference's text parse fails on "nan"/"inf"). */
int fleet_model_version(fleet_ctx* ctx, const float* weights, const int32_t* dims, int n_mats, const float* biases,
                        size_t n_biases, float* weights_out, float* biases_out);

/* getModelParametersNative (Server/src/main/c++/cppNN_backend.cpp:227-242, SURVEY.md
 * §8 a20): Base64::encode of network::getModelParams (commonLib/cppNN/network.h:
 * 708-723) = the biases of every use_bias() layer (layer order) repeated
 * graph_edges = layer_graph.size() times -- the bias loop sits inside the loop
 * over layer_graph -- then the non-null W. Output: fleet_b64_len(n_biases *
 * graph_edges + n_weights) bytes. */
int fleet_model_params_device(fleet_ctx* ctx, const float* d_weights, size_t n_weights, const float* d_biases,
                              size_t n_biases, int graph_edges, void* d_out, void* stream);
int fleet_model_params(fleet_ctx* ctx, const float* weights, size_t n_weights, const float* biases, size_t n_biases,
                       int graph_edges, char* out, size_t cap, size_t* out_len);

/* getMiniBatch (Server/src/main/c++/cppNN_backend.cpp:677-699):
 * Base64::encode of the vector uniformSample / nonIIDSample build (:553-675) --
 * header[7] = {E, sigma, C, lr, batchSize, featureSize, numLabels} as float (the
 * caller converts as push_back does), then per sample idx[b] its F features,
 * (DISTILLATION_MODE=1, teacher != NULL) the teacher's num_labels probabilities
 * teacher[b*num_labels ..], and its label as float; with a teacher the vector
 * ends with 1234567 (:611). The index draw (rand() % N, or the non-IID bucket
 * cursor) stays with the caller (fleet_amd/sampler.py mirrors both); the
 * teacher's forward pass is not rebuilt (its outputs are inputs).
 * images: n_images x F fp32 rows; labels: n_images int32. Output:
 * fleet_minibatch_len(F, B, num_labels, teacher != NULL) bytes. */
size_t fleet_minibatch_len(int F, int B, int num_labels, int with_teacher);

/* The sampler's mode-1 teacher forward: uniformSample appends
 * teacher.forward(sample, TEMPERATURE, -1, 1)'s 10 class probabilities per drawn
 * sample (Server/src/main/c++/cppNN_backend.cpp:596-613) for the teacher network
 * initSampler builds (:494-502: I1 28x28, C1 conv 5x5x8 elu, P1 semi-stochastic
 * pool 3, C2i conv 1x1x16 elu, C2 conv 5x5x48 elu, P2 semi-stochastic pool 2,
 * FC2 softmax 10), computed as commonLib/cppNN's network::forward does, bit for
 * bit (expf = glibc 2.35's, fleet_amd/csrc/teacher_math.h). w: the network's
 * non-null W in order (fleet_teacher_weight_count() floats), b: the use_bias()
 * layers' biases in layer order (fleet_teacher_bias_count()); the first 784 of
 * each image's F features are the input; temperature = TEMPERATURE (2,
 * commonLib/cppNN/network.h:53). Replaces the teacher.forward calls; the
 * teacher's training in initSampler stays with the caller. */
size_t fleet_teacher_weight_count(void);
size_t fleet_teacher_bias_count(void);
/* device buffers: probs[b*10 + j] for image d_idx[b] (d_idx NULL: image b);
 * an index outside [0, n_images) is reported by fleet_check as FLEET_ERR_ARG */
int fleet_teacher_forward_device(fleet_ctx* ctx, const void* d_w, const void* d_b, const void* d_images,
                                 size_t n_images, int F, const void* d_idx, int B, float temperature, void* d_probs,
                                 void* stream);
/* host buffers, synchronous: probs[B x 10] for images[idx[b]] */
int fleet_teacher_forward(fleet_ctx* ctx, const float* w, size_t n_w, const float* b, size_t n_b, const float* images,
                          size_t n_images, int F, const int32_t* idx, int B, float temperature, float* probs);

/* Kardam bookkeeping of CppNNUpdater.update (Server/src/main/java/apps/cppNN/
 * CppNNUpdater.java:463-481, utils/Kardam.java:48-62) for the M
 * picked uploads in one call:
 *   g_c = ByteVec(getFlatGradient(upload_c)).scalarMultiply(dampen_c).scalarMultiply(lr)
 * (flat Base64, the text Kardam.setGrad stores), norm_g[c] = g_c.getNorm() and,
 * when prev[c] != NULL (the worker's previous g, same length),
 * norm_diff[c] = g_c.subtract(prev[c]).getNorm(), else NaN. The uploads share
 * the last one's layout (as fleet_update enforces). g_out: M rows of g_pitch
 * bytes (>= *g_len). Norms: partial sums of the reference's fp64 loop in a
 * different order (1e-12 relative). */
int fleet_kardam_grads(fleet_ctx* ctx, const char* const* uploads, const size_t* lens, int M, const double* dampen,
                       double lr, const char* const* prev, char* g_out, size_t g_pitch, size_t* g_len,
                       double* norm_g, double* norm_diff);
/* device-resident dataset, indices (d_idx[B]) and output; an index outside
 * [0, n_images) is reported by fleet_check as FLEET_ERR_ARG */
int fleet_minibatch_device(fleet_ctx* ctx, const void* d_images, size_t n_images, int F, const void* d_labels,
                           const void* d_idx, int B, const void* d_teacher, int num_labels, const float header[7],
                           void* d_out, void* stream);
/* host buffers: the B sampled rows are gathered into pinned staging, encoded on
 * the GPU and returned (synchronous); FLEET_ERR_ARG for an index outside the set */
int fleet_minibatch(fleet_ctx* ctx, const float* images, size_t n_images, int F, const int32_t* labels,
                    const int32_t* idx, int B, const float* teacher, int num_labels, const float header[7],
                    char* out, size_t cap, size_t* out_len);

/* descentNative's model step -------------------------------
 * Server/src/main/c++/cppNN_backend.cpp:336-352: network::descent(vector)
 * (commonLib/cppNN/network.h:1185-1202) walks the gradients() layout of the
 * merged gradient -- w_sizes[n_w] weight blocks, b_sizes[n_b] bias blocks -- and
 * descent() (:1334-1353) applies
 *   sgd::increment_w (solver.h:88-94):  w -= lr*(dW + 0*w)   per weight block i
 *                                         with w_present[i] (W[i] non-null)
 *   update_bias (layer.h:241-243):       b -= db*lr           per layer k with
 *                                         fc_layer[k] (fully_connected_layer)
 * in fp32, one rounding per operation. `weights` = the non-null W concatenated in
 * slot order (the model codec's layout); `fc_bias` = the fully-connected layers'
 * biases concatenated in layer order; `grad` = decodeFloat(merged) (fleet_update's
 * merged_f32), n_up floats. lr = (float)lrates_vec[currEpoch].
 * Device-resident (layout arrays on the host; the header values inside d_grad
 * are not re-read: fleet_update already checked them against the layout). */
int fleet_descent_device(fleet_ctx* ctx, float* d_weights, float* d_fc_bias, const float* d_grad,
                         const int32_t* w_sizes, const uint8_t* w_present, int n_w, const int32_t* b_sizes,
                         const uint8_t* fc_layer, int n_b, float lr, void* stream);
/* The same model step on one element shard (fleet_amd.shard): d_grad_window holds
 * the merged fp32 values [value_begin, value_end) of the upload positions (what
 * fleet_update_device's window mode writes); only the weights and FC biases whose
 * gradient positions fall in the window are updated, in the full-size model
 * arrays -- so N ranks, each on its window, update disjoint parts with no
 * exchange, and together do exactly fleet_descent_device's step. */
int fleet_descent_window_device(fleet_ctx* ctx, float* d_weights, float* d_fc_bias, const float* d_grad_window,
                                size_t value_begin, size_t value_end, const int32_t* w_sizes,
                                const uint8_t* w_present, int n_w, const int32_t* b_sizes, const uint8_t* fc_layer,
                                int n_b, float lr, void* stream);
/* Host buffers, updated in place; checks the header floats of grad against the
 * layout as network::descent(vector) would read them (FLEET_ERR_LAYOUT). */
int fleet_descent(fleet_ctx* ctx, float* weights, size_t n_weights, float* fc_bias, size_t n_fc_bias,
                  const float* grad, size_t n_grad, const int32_t* w_sizes, const uint8_t* w_present, int n_w,
                  const int32_t* b_sizes, const uint8_t* fc_layer, int n_b, float lr);

/* The server's resident model -----------------------
 * The state the reference's updater natives keep in libnative.so globals
 * (Server/src/main/c++/cppNN_backend.cpp: cnn, models, lrates_vec, currEpoch,
 * priority), built on the entry points above. Errors: fleet_model_last_error.
 * distillation_mode = the reference's compile-time DISTILLATION_MODE (1: the
 * quantised dictionary / index-set text; 0: plain values). */
typedef struct fleet_model fleet_model;
/* fetchParamsNative (:282-301): network::read of a getParams text (mojo01 format,
 * commonLib/cppNN/network.h:611-706, 840-1010). Layer types: input,
 * convolution, max_pool, semi_stochastic_pool, fully_connected (FLeet's cppNN
 * models); W shapes follow the layers' new_connection rules (layer.h). */
int fleet_model_load(fleet_ctx* ctx, const char* text, size_t len, int distillation_mode, fleet_model** out);
void fleet_model_destroy(fleet_model* m);
const char* fleet_model_last_error(const fleet_model* m);
/* initUpdater's model part (:161-194): lr = (float)lrates[0], the first version
 * (read(getParams()) of the model) pushed, priority = epoch = 0. */
int fleet_model_init_updater(fleet_model* m, const double* lrates, int n_lrates);
/* descentNative (:329-383): decodeFloat(merged); lr = lrates[epoch] while epoch <
 * n_lrates; network::descent (sgd w -= lr*dW, fully-connected biases b -= db*lr,
 * fleet_descent); epoch++; the new version read(getParams()) appended and the
 * oldest dropped beyond stale_size. The merged gradient's header must describe
 * the model (FLEET_ERR_LAYOUT otherwise; the reference overruns). */
int fleet_model_descent(fleet_model* m, const char* merged, size_t len, int client_batch_size, int stale_size);
/* modelsSize (:324-327) */
int fleet_model_count(fleet_model* m);
/* getParametersNative(version) (:244-280): the full getParams text of
 * models[version] -- header, bias lines (ostream precision 6), weights
 * (mode 1: quantization_weight_model's dictionary and index set, the version
 * itself left unquantised). */
int fleet_model_get_params(fleet_model* m, int version, char* out, size_t cap, size_t* out_len);
/* getModelParametersNative(version) (:227-242): Base64 of getModelParams. */
int fleet_model_get_model_params(fleet_model* m, int version, char* out, size_t cap, size_t* out_len);
/* getCurrEpoch/setCurrEpoch, getPriority/setPriority, getLrate (:129-159) */
int fleet_model_get_epoch(fleet_model* m);
void fleet_model_set_epoch(fleet_model* m, int epoch);
int fleet_model_get_priority(fleet_model* m);
void fleet_model_set_priority(fleet_model* m, int priority);
double fleet_model_get_lrate(fleet_model* m);
/* sizes: non-null W floats, use_bias() biases, layer-graph edges, layers */
int fleet_model_shape(fleet_model* m, size_t* n_weights, size_t* n_biases, int* graph_edges, int* n_layers);
/* weights / biases of models[version] (version -1: the current `cnn`) */
int fleet_model_export(fleet_model* m, int version, float* weights, size_t n_weights, float* biases, size_t n_biases);

/* The offline sampler's state (the CppNNOfflineSampler natives
 * of Server/src/main/c++/cppNN_backend.cpp and the globals they keep). Random
 * draws come from libc rand(), the process-wide generator the reference uses.
 * Errors: fleet_sampler_last_error. */
typedef struct fleet_sampler fleet_sampler;
/* initSampler (:385-479): srand(seed) (the reference's seed is 1, :71), the
 * MNIST training set under data_path (commonLib/cppNN/mnist_parser.h:
 * train-images.idx3-ubyte or train-images-idx3-ubyte and the labels file,
 * pixels (b / 255) * 2 - 1), numLabels = 10, and with iid == 0 the non-IID
 * buckets (:411-479): sort_indexes of the labels (std::sort), with outlier != 0
 * a first bucket of the label-0 samples, then 2*(num_clients - outliers) shards
 * shuffled and dealt two per client, every bucket shuffled (std::random_shuffle
 * over rand() % i). iid, outlier and num_clients are the reference's
 * compile-time globals (:59-61; defaults 0, 0, 10). The teacher's training that
 * follows in DISTILLATION_MODE=1 whatever the sampler (:481-545) is not rebuilt:
 * iid mini-batches take the trained weights from fleet_sampler_set_teacher.
 * ctx may be NULL (host state only; fleet_sampler_minibatch then fails). */
int fleet_sampler_create(fleet_ctx* ctx, const char* data_path, int iid, int outlier, int num_clients,
                         int distillation_mode, int seed, fleet_sampler** out);
/* the same over a dataset in memory: images n x F floats, labels n */
int fleet_sampler_create_from(fleet_ctx* ctx, const float* images, const int32_t* labels, size_t n, int F,
                              int num_labels, int iid, int outlier, int num_clients, int distillation_mode, int seed,
                              fleet_sampler** out);
void fleet_sampler_destroy(fleet_sampler* s);
const char* fleet_sampler_last_error(const fleet_sampler* s);
/* initUpdater's generator side effects (:163, :216/:222): srand(seed), then, when
 * a model was fetched (fetched != 0: fetchParamsNative's set_random_augmentation
 * enabled the random shift, :293), the two rand() draws of cnn.train_class's shift
 * (network.h:1840). Assumes the reference's MNIST network: no dropout layer (whose
 * training forward would draw more, layer.h:608-617) and no flips. */
void fleet_updater_reseed_ex(int seed, int fetched);
/* the original one-argument form: fleet_updater_reseed_ex(seed, 1) (a model was
 * fetched, the reference's server order) -- kept so callers built against it keep
 * their meaning */
void fleet_updater_reseed(int seed);
/* initUpdater's E, sigma, C (:169-171), read by every later mini-batch header */
int fleet_sampler_set_hyper(fleet_sampler* s, int E, double sigma, double C);
/* DISTILLATION_MODE=1 with iid sampling: the trained teacher's weights
 * (fleet_teacher_forward's layout); uniformSample then appends its outputs */
int fleet_sampler_set_teacher(fleet_sampler* s, const float* w, size_t n_w, const float* b, size_t n_b);
/* getMiniBatch (:677-699): B = batch_size * E samples -- uniformSample's
 * rand() % N draws, or nonIIDSample's cursor over the current client's bucket
 * -- the client rotation advanced, header {E, sigma, C, lr, B, F, numLabels}
 * (lr = the updater's cnn.get_learning_rate()), encoded on the GPU
 * (fleet_minibatch). B <= 0 (E = 0 before initUpdater) is FLEET_ERR_ARG: the
 * reference reads sample 0 of an empty batch there. */
int fleet_sampler_minibatch(fleet_sampler* s, int batch_size, float lr, char* out, size_t cap, size_t* out_len);
size_t fleet_sampler_minibatch_len(fleet_sampler* s, int batch_size);
int fleet_sampler_num_labels(const fleet_sampler* s);   /* getNumLabels (:129-132) */
int fleet_sampler_has_outlier(const fleet_sampler* s);  /* hasOutlier (:134-137) */
size_t fleet_sampler_num_samples(const fleet_sampler* s);
/* introspection (tests): bucket `client` (positions in the label-sorted order),
 * the label-sorted order itself, and the last request's image indices */
int fleet_sampler_bucket(fleet_sampler* s, int client, int32_t* out, size_t cap, size_t* n);
int fleet_sampler_sorted_index(fleet_sampler* s, int32_t* out, size_t cap, size_t* n);
int fleet_sampler_last_indices(fleet_sampler* s, int32_t* out, size_t cap, size_t* n);

/* Name of the aggregation kernel fleet_update / fleet_update_device launch for
 * an upload of `len` Base64 bytes (or a group window of that many bytes), exactly
 * as rocprofv3 names it (every template argument spelled out): "k_update_mixed<256,
 * false>", "k_update_flat", "k_update_weave<8>", "k_update_tiled_encode<64>" (tile=classic)
 * or "k_update_pipe<16, 1, 5, 0, false>"; and what fleet_update_encode_device launches
 * ("k_update_encode<256>", "k_update_tiled_encode<64>", "k_update_flat",
 * "k_update_weave_encode<8>", ...; DESIGN.md §4 lists the default per size;
 * profiling aid; thread-local storage, valid until the thread's next call). */
const char* fleet_update_kernel(size_t len);
const char* fleet_update_encode_kernel(size_t len);
/* The same plan's grid (test and profiling aid, no device needed): kind 0 stream
 * (blocks [0, n_a) a group per lane, 256 groups each, the rest a value per lane,
 * 84 groups each), 1 tiled (n_w 64-group tiles then n_n 16-group tiles; n_w = -1:
 * one width, 64-group tiles only), 2 pipelined (16-group tiles), 3 woven tiles
 * (64 groups each), 4 flat tiles (n_w 64-group tiles, then n_n tiles of n_a
 * groups, the last one ragged); *blocks = the aggregation's grid. */
int fleet_update_plan_grid(size_t len, int* kind, int64_t* blocks, int64_t* n_a, int64_t* n_w, int64_t* n_n);

/* Launch-plan overrides, process-wide (experiments, and tests that run every
 * launch variant on small inputs; results are identical under every plan). spec =
 * comma-separated key=value items: update=auto|stream|tiled|pipe, grid=auto|plain|balanced|
 * lanes (the stream grid; lanes = every group a value per lane, the balanced grid's tail
 * form, for tests on small inputs), tile=auto|classic|flat|weave6|weave8 and
 * flat_w2=auto|1..64, tile_enc_prio=auto|0..3 (the tiles' form; the flat grid's
 * narrow width; the tiles' fused encode blocks' issue priority), tile_enc_rows=N,
 * fused=on|off (the pipelined step as one launch or two), stage_threads=1..64,
 * stage_pieces=1..64 (host staging); ""
 * restores the measured default. An unknown key or value rejects the whole spec
 * (FLEET_ERR_ARG, the reason in err) and leaves the plan unchanged. The environment
 * variable FLEET_EXPERIMENTS, read once at first use, takes the same spec; no other
 * environment variable changes a launch. fleet_plan returns the active spec ("" =
 * default; thread-local storage). */
int fleet_set_plan(const char* spec, char* err, size_t cap);
const char* fleet_plan(void);

/* Test hook (no reference counterpart): the pipelined Kardam form's reduce blocks of
 * this context wait for the launch's epoch + skew, which no tile publishes when skew
 * != 0, so their bounded wait times out and fleet_update_kardam_device returns
 * FLEET_ERR_HIP. skew = 0 restores the normal hand-off. */
int fleet_test_kardam_skew(fleet_ctx* ctx, unsigned skew);

#ifdef __cplusplus
}
#endif
#endif
