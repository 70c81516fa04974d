/*
 * oracle/fleet_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference (gdamaskinos/fleet) compressed-SGD
 * gradient codec and server-side aggregation path, used as the parity
 * checker for the HIP path (tests/, __graft_entry__.smoke) and as the
 * `cpu_baseline` "port" leg of bench.py. The product (fleet_amd/) never links
 * or calls this.
 *
 * PARITY UNPINNED for the codec and aggregation chain (rows a1-a14, f2, f4):
 * the reference's Base64.cpp and cppNN_backend.cpp #include <jni.h>, which this
 * image lacks, so they cannot be built here, and the reference ships no tests
 * or fixtures. The restatement is checked against SURVEY.md
 * §8c's known-answer values only. The model-side functions (quantize,
 * dictionary, weights section, descent) ARE pinned to the reference's own
 * header-only mojo network compiled into oracle/_ref/libfleetref_model.so
 * (tests/test_oracle_golden.py).
 *
 * Every function cites the reference file:line it restates.
 */
#ifndef FLEET_ORACLE_H
#define FLEET_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* commonLib/cpp_utils/Base64.cpp:37-46 */
int fo_num_digits(int32_t number);
/* x86-64 `(int) float` (cvttss2si): INT32_MIN when |x| >= 2^31 or NaN. */
int32_t fo_cvtt(float x);
/* Base64.cpp:48-78, intNum == 1, precision == 9 */
int32_t fo_float2int(float x);
/* Base64.cpp:80-103, intNum == 1, precision == 9 */
float fo_int2float(int32_t c);
/* Q = int2float o float2int: what the next JNI op sees after an encode. */
float fo_q(float x);

/* Base64.cpp:124-169: bytes -> text; returns text length (4*ceil(len/3)). */
size_t fo_b64_encode(const uint8_t* buf, size_t len, char* out);
/* Base64.cpp:175-217: text -> bytes (pad/invalid sextets drop bytes). */
size_t fo_b64_decode(const char* s, size_t len, uint8_t* out);
size_t fo_b64_len(size_t n_values);

/* Base64::encode(vector<float>) (:140-142) / decodeFloat (:207-209) / decodeInt (:211-219) */
size_t fo_encode_floats(const float* v, size_t n, char* out);
size_t fo_encode_ints(const int32_t* v, size_t n, char* out);
size_t fo_decode_floats(const char* s, size_t len, float* out);
size_t fo_decode_ints(const char* s, size_t len, int32_t* out);

/* Per-op restatements of Server/src/main/c++/cppNN_backend.cpp (all Base64 in/out).
 * Return the output length, or (size_t)-1 on malformed input. `out` must hold
 * fo_b64_len(decoded values) bytes. */
size_t fo_flat_gradient(const char* g, size_t len, char* out);                                      /* :701-720 */
size_t fo_merge_flat_gradient(const char* g, size_t glen, const char* flat, size_t flen, char* out); /* :722-750 */
size_t fo_scalar_mul(const char* v, size_t len, double a, char* out);                               /* :753-777 */
double fo_norm(const char* v, size_t len);                                                          /* :779-795 */
size_t fo_add(const char* a, size_t alen, const char* b, size_t blen, char* out);                   /* :797-846 */
size_t fo_subtract(const char* a, size_t alen, const char* b, size_t blen, char* out);              /* :848-892 */

/* CppNNUpdater.update (CppNNUpdater.java:420-509) as the per-op string chain
 * (faithful: same op sequence and string round trips as the reference). */
size_t fo_update_faithful(const char* const* uploads, const size_t* lens, int M, const double* dampen,
                          char* merged);

/* The same update computed element-wise (identical results), OpenMP over
 * element groups with `threads` threads (<=0: all cores). `header_mask[i]`
 * (N_up bytes) marks the layout slots of the upload (network.h:1038-1056).
 * Optional merged_f32 receives decodeFloat(merged). */
size_t fo_update_fused(const char* const* uploads, size_t len, int M, const double* dampen,
                       const uint8_t* header_mask, char* merged, float* merged_f32, int threads);

/* Layout of gradients() (network.h:1038-1056): header mask for given sizes. */
size_t fo_layout_n_up(const int32_t* w_sizes, int n_w, const int32_t* b_sizes, int n_b);
void fo_layout_header_mask(const int32_t* w_sizes, int n_w, const int32_t* b_sizes, int n_b, uint8_t* mask);

/* Synthetic inputs: Philox4x32-10 keyed by seed, counter (element, client). */
void fo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
float fo_synth_value(uint64_t seed, uint32_t client, uint32_t element);
/* Full client upload as floats: layout headers + synthetic payload. */
void fo_synth_upload(uint64_t seed, uint32_t client, const int32_t* w_sizes, int n_w, const int32_t* b_sizes,
                     int n_b, float* out);

/* ---- DISTILLATION_MODE=1 model codec ---- */
/* network.h:1683-1774 + core_math.h:881-912: quantise one W matrix in place. */
void fo_quantize_matrix(float* x, int cols, int rows, int chans);
/* network.h:594-608,641-692: first-occurrence dictionary + printed indices. */
int fo_dictionary(const float* w, size_t n, float* dict, int32_t* index);
/* getParams' DISTILLATION_MODE=1 weights section for quantised weights. */
size_t fo_weights_section(const float* w, const int32_t* dims, int n_mats, char* out, size_t cap);
/* network::read's DISTILLATION_MODE=1 weights branch (network.h:958-997). */
int fo_read_weights_section(const char* text, size_t len, const int32_t* dims, int n_mats, float* w_out);

/* ---- SGD epilogue: descentNative's model step ---- */
/* cppNN_backend.cpp:336-352 -> network.h:1185-1202,1334-1353 -> solver.h:88-94, layer.h:241-243 */
/* The sampler's mode-1 teacher forward, one sample:
 * teacher.forward(x, TEMPERATURE, -1, 1) of initSampler's network
 * (Server/src/main/c++/cppNN_backend.cpp:494-502, 603) restated from
 * commonLib/cppNN: network.h:523-585 (forward), layer.h:805-887 (convolution
 * accumulate, 5x5 via core_math.h unwrap_aligned_NxN/dotsum_unwrapped_NxN, 1x1),
 * layer.h:481-556 (semi-stochastic pool, r = 9, train = 1), layer.h:200-238 +
 * core_math.h dot (fully connected), activation.h:161-176 (elu) and :271-313
 * (softmax), with the libm expf the reference calls (std::exp(float)).
 * w: non-null W in network order (21448 floats), b: use_bias() biases in layer
 * order (82), x: 784 floats, probs: 10. Pinned to the reference's own network
 * (oracle/_ref ref_teacher_forward) by tests/test_teacher.py. */
void fo_teacher_forward(const float* w, const float* b, const float* x, float temperature, float* probs);
/* glibc expf over all 2^32 inputs: the order-independent digest of
 * tests/native/digest_ref.cpp fn 18 (NaN results as 0x7fc00000) */
uint64_t fo_expf_digest(void);

int fo_descent(float* weights, size_t n_weights, float* fc_bias, size_t n_fc_bias, const float* g, size_t n_g,
               const uint8_t* w_present, int n_w_slots, const uint8_t* fc_layer, int n_layers, float lr);

#ifdef __cplusplus
}
#endif
#endif
