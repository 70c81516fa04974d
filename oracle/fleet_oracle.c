/*
 * oracle/fleet_oracle.c -- TEST INFRASTRUCTURE ONLY (see fleet_oracle.h).
 *
 * Clean-room C restatement of the FLeet cppNN gradient codec + aggregation
 * path. Compiled with -ffp-contract=off and no fast-math so every float op
 * is one IEEE-754 binary32/binary64 round-to-nearest-even operation, exactly
 * like the reference's x86-64 SSE build (Server/Makefile:2, -O0).
 * Parity status (unpinned for the codec/aggregation chain): fleet_oracle.h.
 */
#include "fleet_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------- scalars */

/* Base64.cpp:37-46 -- '-' counts as a digit; numDigits(0) == 0. */
int fo_num_digits(int32_t number) {
  int digits = 0;
  if (number < 0) digits = 1;
  while (number) {
    number /= 10;
    digits++;
  }
  return digits;
}

/* `(int) x` as compiled for x86-64 (cvttss2si): out of range / NaN -> INT_MIN. */
int32_t fo_cvtt(float x) {
  if (!(fabsf(x) < 2147483648.0f)) return INT32_MIN;
  return (int32_t)x;
}

/* Base64.cpp:48-78 with intNum == 1, precision == 9. */
int32_t fo_float2int(float x) {
  const int precision = 9;
  int digits = fo_num_digits(fo_cvtt(x));
  for (int j = 0; j < precision - digits; j++) x *= 10; /* fp32 multiply, rounded each time */
  int32_t temp = fo_cvtt(x);
  int32_t lsb = temp % 10; /* C: truncating remainder */
  /* `temp - LSB + digits` in 32-bit two's complement (wraps like the x86 build) */
  uint32_t t = (uint32_t)temp - (uint32_t)lsb;
  t = temp >= 0 ? t + (uint32_t)digits : t - (uint32_t)digits;
  return (int32_t)t;
}

/* Base64.cpp:80-103 with intNum == 1, precision == 9. */
float fo_int2float(int32_t c) {
  const int precision = 9;
  int dd = abs(c % 10);
  float t = (float)c;
  for (int j = 0; j < precision - dd; j++) t /= 10; /* fp32 divide, correctly rounded */
  return t;
}

float fo_q(float x) { return fo_int2float(fo_float2int(x)); }

/* ----------------------------------------------------------------- base64 */

/* Base64.cpp:20-27 */
static const uint8_t from_b64[128] = {
    255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255,
    255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255,
    255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 62,  255, 62,  255, 63,
    52,  53,  54,  55,  56,  57,  58,  59,  60,  61,  255, 255, 255, 255, 255, 255,
    255, 0,   1,   2,   3,   4,   5,   6,   7,   8,   9,   10,  11,  12,  13,  14,
    15,  16,  17,  18,  19,  20,  21,  22,  23,  24,  25,  255, 255, 255, 255, 63,
    255, 26,  27,  28,  29,  30,  31,  32,  33,  34,  35,  36,  37,  38,  39,  40,
    41,  42,  43,  44,  45,  46,  47,  48,  49,  50,  51,  255, 255, 255, 255, 255};
static const char to_b64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

size_t fo_b64_len(size_t n_values) { return 4 * ((4 * n_values + 2) / 3); }

/* Base64.cpp:124-169 */
size_t fo_b64_encode(const uint8_t* buf, size_t len, char* out) {
  size_t missing = 0, ret_size = len;
  while (ret_size % 3 != 0) {
    ++ret_size;
    ++missing;
  }
  ret_size = 4 * ret_size / 3;
  for (size_t i = 0; i < ret_size / 4; ++i) {
    size_t idx = i * 3;
    uint8_t b0 = idx + 0 < len ? buf[idx + 0] : 0;
    uint8_t b1 = idx + 1 < len ? buf[idx + 1] : 0;
    uint8_t b2 = idx + 2 < len ? buf[idx + 2] : 0;
    out[4 * i + 0] = to_b64[(b0 & 0xfc) >> 2];
    out[4 * i + 1] = to_b64[((b0 & 0x03) << 4) + ((b1 & 0xf0) >> 4)];
    out[4 * i + 2] = to_b64[((b1 & 0x0f) << 2) + ((b2 & 0xc0) >> 6)];
    out[4 * i + 3] = to_b64[b2 & 0x3f];
  }
  for (size_t i = 0; i < missing; ++i) out[ret_size - i - 1] = '=';
  return ret_size;
}

static uint8_t sextet(char ch) {
  /* `(ch <= 'z') ? from_base64[ch] : 0xff` (Base64.cpp:199-202). Bytes >= 0x80
   * index the table out of bounds in the reference (UB); treated as pad here. */
  unsigned char u = (unsigned char)ch;
  return u <= 'z' ? from_b64[u] : 0xff;
}

/* Base64.cpp:185-217 (the string is first padded with '=' to a multiple of 4) */
size_t fo_b64_decode(const char* s, size_t len, uint8_t* out) {
  size_t n = 0;
  size_t padded = (len + 3) / 4 * 4;
  for (size_t i = 0; i < padded; i += 4) {
    uint8_t b4[4];
    for (int k = 0; k < 4; ++k) b4[k] = i + k < len ? sextet(s[i + k]) : 0xff;
    uint8_t b30 = (uint8_t)(((b4[0] & 0x3f) << 2) + ((b4[1] & 0x30) >> 4));
    uint8_t b31 = (uint8_t)(((b4[1] & 0x0f) << 4) + ((b4[2] & 0x3c) >> 2));
    uint8_t b32 = (uint8_t)(((b4[2] & 0x03) << 6) + ((b4[3] & 0x3f) >> 0));
    if (b4[1] != 0xff) out[n++] = b30;
    if (b4[2] != 0xff) out[n++] = b31;
    if (b4[3] != 0xff) out[n++] = b32;
  }
  return n;
}

/* Base64.cpp:109-115 */
size_t fo_encode_ints(const int32_t* v, size_t n, char* out) {
  return fo_b64_encode((const uint8_t*)v, n * sizeof(int32_t), out);
}
/* Base64.cpp:104-106 */
size_t fo_encode_floats(const float* v, size_t n, char* out) {
  int32_t* codes = (int32_t*)malloc(sizeof(int32_t) * (n ? n : 1));
  for (size_t i = 0; i < n; ++i) codes[i] = fo_float2int(v[i]);
  size_t r = fo_encode_ints(codes, n, out);
  free(codes);
  return r;
}
/* Base64.cpp:175-183 */
size_t fo_decode_ints(const char* s, size_t len, int32_t* out) {
  uint8_t* bytes = (uint8_t*)malloc(len + 4);
  size_t nb = fo_b64_decode(s, len, bytes);
  size_t n = nb / sizeof(int32_t);
  memcpy(out, bytes, n * sizeof(int32_t));
  free(bytes);
  return n;
}
/* Base64.cpp:171-173 */
size_t fo_decode_floats(const char* s, size_t len, float* out) {
  int32_t* codes = (int32_t*)malloc(len + 4);
  size_t n = fo_decode_ints(s, len, codes);
  for (size_t i = 0; i < n; ++i) out[i] = fo_int2float(codes[i]);
  free(codes);
  return n;
}

/* -------------------------------------------------------------- JNI ops */

static float* decode_alloc(const char* s, size_t len, size_t* n) {
  float* v = (float*)malloc(sizeof(float) * (len / 4 * 3 + 4));
  *n = fo_decode_floats(s, len, v);
  return v;
}

/* network.h:1206-1223 (flatGrad); returns flat length or -1 if the header
 * walks past the end (the reference reads out of bounds there). */
static long flat_grad(const float* g, size_t n, float* flat) {
  size_t idx = 0;
  long k = 0;
  for (int part = 0; part < 2; ++part) { /* dW_sets, then dbias_sets */
    if (idx >= n) return -1;
    int cnt = fo_cvtt(g[idx++]);
    for (int i = 0; i < cnt; ++i) {
      if (idx >= n) return -1;
      int size = fo_cvtt(g[idx++]);
      if (size < 0 || idx + (size_t)size > n) return -1;
      for (int j = 0; j < size; ++j) flat[k++] = g[idx++];
    }
  }
  return k;
}

/* network.h:1226-1242 (mergeFlatGrad) */
static int merge_flat_grad(float* g, size_t n, const float* flat, size_t nflat) {
  size_t idx = 0, idx2 = 0;
  for (int part = 0; part < 2; ++part) {
    if (idx >= n) return -1;
    int cnt = fo_cvtt(g[idx++]);
    for (int i = 0; i < cnt; ++i) {
      if (idx >= n) return -1;
      int size = fo_cvtt(g[idx++]);
      if (size < 0 || idx + (size_t)size > n || idx2 + (size_t)size > nflat) return -1;
      for (int j = 0; j < size; ++j) g[idx++] = flat[idx2++];
    }
  }
  return 0;
}

/* cppNN_backend.cpp:701-720 */
size_t fo_flat_gradient(const char* g, size_t len, char* out) {
  size_t n;
  float* v = decode_alloc(g, len, &n);
  float* flat = (float*)malloc(sizeof(float) * (n + 1));
  long k = flat_grad(v, n, flat);
  size_t r = k < 0 ? (size_t)-1 : fo_encode_floats(flat, (size_t)k, out);
  free(v);
  free(flat);
  return r;
}

/* cppNN_backend.cpp:722-750 */
size_t fo_merge_flat_gradient(const char* g, size_t glen, const char* flat, size_t flen, char* out) {
  size_t n, nf;
  float* grad = decode_alloc(g, glen, &n);
  float* fl = decode_alloc(flat, flen, &nf);
  size_t r = merge_flat_grad(grad, n, fl, nf) < 0 ? (size_t)-1 : fo_encode_floats(grad, n, out);
  free(grad);
  free(fl);
  return r;
}

/* cppNN_backend.cpp:753-777: res = ret[i] * a (float * double -> double, stored as float) */
size_t fo_scalar_mul(const char* v, size_t len, double a, char* out) {
  size_t n;
  float* x = decode_alloc(v, len, &n);
  for (size_t i = 0; i < n; ++i) x[i] = (float)((double)x[i] * a);
  size_t r = fo_encode_floats(x, n, out);
  free(x);
  return r;
}

/* cppNN_backend.cpp:779-795: s += ret[i]*ret[i] (fp32 square, fp64 sum) */
double fo_norm(const char* v, size_t len) {
  size_t n;
  float* x = decode_alloc(v, len, &n);
  double s = 0;
  for (size_t i = 0; i < n; ++i) {
    float sq = x[i] * x[i];
    s += sq;
  }
  free(x);
  return sqrt(s);
}

static size_t binop(const char* a, size_t alen, const char* b, size_t blen, char* out, int sub) {
  size_t na, nb;
  float* x = decode_alloc(a, alen, &na);
  float* y = decode_alloc(b, blen, &nb);
  size_t r = (size_t)-1;
  if (nb >= na) { /* the reference reads retB[i] for i < retA.size() */
    for (size_t i = 0; i < na; ++i) x[i] = sub ? x[i] - y[i] : x[i] + y[i];
    r = fo_encode_floats(x, na, out);
  }
  free(x);
  free(y);
  return r;
}
/* cppNN_backend.cpp:797-846 */
size_t fo_add(const char* a, size_t alen, const char* b, size_t blen, char* out) {
  return binop(a, alen, b, blen, out, 0);
}
/* cppNN_backend.cpp:848-892 */
size_t fo_subtract(const char* a, size_t alen, const char* b, size_t blen, char* out) {
  return binop(a, alen, b, blen, out, 1);
}

/* CppNNUpdater.java:420-509 (thresholds 0, Kardam bypassed at :488) */
size_t fo_update_faithful(const char* const* uploads, const size_t* lens, int M, const double* dampen,
                          char* merged) {
  if (M <= 0) return (size_t)-1;
  size_t cap = lens[M - 1] + 16;
  for (int i = 0; i < M; ++i)
    if (lens[i] + 16 > cap) cap = lens[i] + 16;
  char* flat = (char*)malloc(cap);
  char* damp = (char*)malloc(cap);
  char* avg = (char*)malloc(cap);
  char* tmp = (char*)malloc(cap);
  size_t avg_len = 0;
  size_t r = (size_t)-1;
  for (int i = 0; i < M; ++i) {
    size_t fl = fo_flat_gradient(uploads[i], lens[i], flat);             /* :463 */
    if (fl == (size_t)-1) goto done;
    size_t dl = fo_scalar_mul(flat, fl, dampen[i], damp);                 /* :464 */
    if (i == 0) {                                                         /* :490-493 */
      memcpy(avg, damp, dl);
      avg_len = dl;
    } else {
      size_t al = fo_add(avg, avg_len, damp, dl, tmp);
      if (al == (size_t)-1) goto done;
      memcpy(avg, tmp, al);
      avg_len = al;
    }
  }
  {
    size_t sl = fo_scalar_mul(avg, avg_len, (double)1 / M, tmp);         /* :507 */
    r = fo_merge_flat_gradient(uploads[M - 1], lens[M - 1], tmp, sl, merged); /* :508 */
  }
done:
  free(flat);
  free(damp);
  free(avg);
  free(tmp);
  return r;
}

/* ------------------------------------------------------- element-wise chain */

/* decode one 16-char group (3 codes) of an upload, reference semantics for valid text */
static int group_codes(const char* s, size_t len, size_t g, int32_t codes[3]) {
  uint8_t bytes[12];
  size_t off = 16 * g;
  size_t nchars = len - off < 16 ? len - off : 16;
  size_t nb = fo_b64_decode(s + off, nchars, bytes);
  int n = (int)(nb / 4);
  memcpy(codes, bytes, (size_t)n * 4);
  return n;
}

size_t fo_update_fused(const char* const* uploads, size_t len, int M, const double* dampen,
                       const uint8_t* header_mask, char* merged, float* merged_f32, int threads) {
  if (M <= 0 || len % 4 != 0) return (size_t)-1;
  size_t groups = (len + 15) / 16;
  const double inv = (double)1 / M;
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for num_threads(threads) schedule(static)
#endif
  for (long g = 0; g < (long)groups; ++g) {
    int32_t codes[3], out[3] = {0, 0, 0};
    float acc[3] = {0, 0, 0};
    int n = 3;
    for (int c = 0; c < M; ++c) {
      n = group_codes(uploads[c], len, (size_t)g, codes);
      for (int e = 0; e < n; ++e) {
        float y = fo_q(fo_int2float(codes[e]));          /* getFlatGradient: dec, enc; next op decodes */
        float p = fo_q((float)((double)y * dampen[c]));   /* scalarMultiply(d_c) */
        acc[e] = c == 0 ? p : fo_q(acc[e] + p);           /* ByteVec.add */
      }
    }
    for (int e = 0; e < n; ++e) {
      size_t i = 3 * (size_t)g + (size_t)e;
      if (header_mask[i]) {
        out[e] = fo_float2int(fo_int2float(codes[e]));      /* merge keeps the last upload's header */
      } else {
        float f = fo_q((float)((double)acc[e] * inv));      /* scalarMultiply(1/avgSize), merge decodes */
        out[e] = fo_float2int(f);                           /* merge re-encodes */
      }
      if (merged_f32) merged_f32[i] = fo_int2float(out[e]);
    }
    char text[16];
    size_t tl = fo_encode_ints(out, (size_t)n, text);
    memcpy(merged + 16 * g, text, tl);
  }
  return len;
}

/* ------------------------------------------------------------------ layout */

size_t fo_layout_n_up(const int32_t* w_sizes, int n_w, const int32_t* b_sizes, int n_b) {
  size_t n = 2 + (size_t)n_w + (size_t)n_b;
  for (int i = 0; i < n_w; ++i) n += (size_t)w_sizes[i];
  for (int i = 0; i < n_b; ++i) n += (size_t)b_sizes[i];
  return n;
}

/* network.h:1038-1056: [nW, (size_i, dW_i...)*, nB, (size_j, db_j...)*] */
void fo_layout_header_mask(const int32_t* w_sizes, int n_w, const int32_t* b_sizes, int n_b, uint8_t* mask) {
  size_t n = fo_layout_n_up(w_sizes, n_w, b_sizes, n_b), idx = 0;
  memset(mask, 0, n);
  mask[idx++] = 1;
  for (int i = 0; i < n_w; ++i) {
    mask[idx++] = 1;
    idx += (size_t)w_sizes[i];
  }
  mask[idx++] = 1;
  for (int i = 0; i < n_b; ++i) {
    mask[idx++] = 1;
    idx += (size_t)b_sizes[i];
  }
}

/* ------------------------------------------------------------- synthetic */

static inline uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
  uint64_t p = (uint64_t)a * b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

/* Philox4x32-10 (Salmon et al., SC'11), standard constants. */
void fo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, hi1;
    uint32_t lo0 = mulhilo(0xD2511F53u, c0, &hi0);
    uint32_t lo1 = mulhilo(0xCD9E8D57u, c2, &hi1);
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

/* SURVEY.md §8d value mix, integer ops + bit assembly only:
 * 90% |x| = 2^e(1+m/2^23), e in [-20,-7]; 9% e in [-6,3]; 1% e in [4,20]; random sign. */
float fo_synth_value(uint64_t seed, uint32_t client, uint32_t element) {
  uint32_t ctr[4] = {element, client, 0x464C4545u, 0u};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t u[4];
  fo_philox4x32_10(ctr, key, u);
  uint32_t cls = u[0] % 100u;
  int e;
  if (cls < 90u)
    e = -20 + (int)(u[1] % 14u);
  else if (cls < 99u)
    e = -6 + (int)(u[1] % 10u);
  else
    e = 4 + (int)(u[1] % 17u);
  uint32_t bits = (u[3] & 0x80000000u) | ((uint32_t)(e + 127) << 23) | (u[2] & 0x7FFFFFu);
  float x;
  memcpy(&x, &bits, 4);
  return x;
}

void fo_synth_upload(uint64_t seed, uint32_t client, const int32_t* w_sizes, int n_w, const int32_t* b_sizes,
                     int n_b, float* out) {
  size_t n = fo_layout_n_up(w_sizes, n_w, b_sizes, n_b);
  uint8_t* mask = (uint8_t*)malloc(n);
  fo_layout_header_mask(w_sizes, n_w, b_sizes, n_b, mask);
  for (size_t i = 0; i < n; ++i) out[i] = fo_synth_value(seed, client, (uint32_t)i);
  size_t idx = 0;
  out[idx++] = (float)n_w;
  for (int i = 0; i < n_w; ++i) {
    out[idx++] = (float)w_sizes[i];
    idx += (size_t)w_sizes[i];
  }
  out[idx++] = (float)n_b;
  for (int i = 0; i < n_b; ++i) {
    out[idx++] = (float)b_sizes[i];
    idx += (size_t)b_sizes[i];
  }
  free(mask);
}

/* ======================================================================
 * DISTILLATION_MODE=1 model codec.
 * ==================================================================== */

/* network.h:1683-1774 (non-bucketing path) with matrix::min_max
 * (core_math.h:881-899), operator+(float)/operator*(float) (:1045-1056) and
 * round_matrix (:901-912), for one weight matrix of cols*rows*chans floats
 * (W matrices are built with chan_aligned = 0: chan_stride = cols*rows, no
 * padding; layer.h:158,787,1297). In place. */
void fo_quantize_matrix(float* x, int cols, int rows, int chans) {
  const int s = rows * cols;
  const size_t n = (size_t)s * (size_t)chans;
  if (n == 0) return;
  size_t mini = 0, maxi = 0;
  for (size_t i = 0; i < n; ++i) {
    if (x[i] < x[mini]) mini = i;
    if (x[i] > x[maxi]) maxi = i;
  }
  const float mn = x[mini], mx = x[maxi];
  const float alpha = mx - mn, beta = mn;
  const float nbeta = (float)(-1.0 * (double)beta); /* `+ (-1.0) * beta` -> operator+(float) */
  const float ialpha = (float)(1.0 / (double)alpha); /* `* (1.0 / alpha)` -> operator*(float) */
  for (size_t i = 0; i < n; ++i) x[i] = x[i] + nbeta;
  for (size_t i = 0; i < n; ++i) x[i] = x[i] * ialpha;
  const float fs = (float)s;
  const float one_over_s = (float)(1 / s); /* integer division: 1 if s == 1 else 0 */
  for (size_t i = 0; i < n; ++i) {
    if (x[i] - floorf(x[i]) > 0.5f)
      x[i] = floorf(x[i] * fs) / fs + one_over_s;
    else
      x[i] = floorf(x[i] * fs) / fs;
  }
  for (size_t i = 0; i < n; ++i) x[i] = x[i] * alpha;
  for (size_t i = 0; i < n; ++i) x[i] = x[i] + beta;
}

/* network.h:594-608 float_vector_find + the two passes of getParams
 * (:641-692): pass 1 builds the first-occurrence dictionary (an element joins
 * the first entry with fabsf(x - e) < 1e-8f, else is appended); pass 2 prints
 * the first matching entry, -1 when none (NaN/inf never match, not even
 * themselves). Returns U; dict (capacity n) gets the entries in creation
 * order, index[i] the printed index of w[i]. */
int fo_dictionary(const float* w, size_t n, float* dict, int32_t* index) {
  int U = 0;
  for (size_t i = 0; i < n; ++i) {
    int found = 0;
    for (int k = 0; k < U; ++k)
      if (fabsf(w[i] - dict[k]) < 0.00000001f) {
        found = 1;
        break;
      }
    if (!found) dict[U++] = w[i];
  }
  for (size_t i = 0; i < n; ++i) {
    int32_t idx = -1;
    for (int k = 0; k < U; ++k)
      if (fabsf(w[i] - dict[k]) < 0.00000001f) {
        idx = k;
        break;
      }
    index[i] = idx;
  }
  return U;
}

static size_t put(char* out, size_t cap, size_t pos, const char* s) {
  size_t l = strlen(s);
  if (out && pos + l <= cap) memcpy(out + pos, s, l);
  return pos + l;
}

/* The weights section of getParams in DISTILLATION_MODE=1 (network.h:641-692):
 * "loop_counter\nU\n" + U x "k\nvalue\n" (ostream default precision 6 == %g)
 * + per matrix the indices each followed by ' ' and a final '\n'.
 * w = the already quantized weights, dims = n_mats x {cols, rows, chans}.
 * Returns the text length (writes only what fits in cap). */
size_t fo_weights_section(const float* w, const int32_t* dims, int n_mats, char* out, size_t cap) {
  size_t n = 0;
  for (int j = 0; j < n_mats; ++j) n += (size_t)dims[3 * j] * dims[3 * j + 1] * dims[3 * j + 2];
  float* dict = (float*)malloc(sizeof(float) * (n ? n : 1));
  int32_t* index = (int32_t*)malloc(sizeof(int32_t) * (n ? n : 1));
  const int U = fo_dictionary(w, n, dict, index);
  char buf[64];
  size_t pos = 0;
  snprintf(buf, sizeof buf, "%zu\n%d\n", n, U);
  pos = put(out, cap, pos, buf);
  for (int k = 0; k < U; ++k) {
    snprintf(buf, sizeof buf, "%d\n%g\n", k, (double)dict[k]);
    pos = put(out, cap, pos, buf);
  }
  size_t i = 0;
  for (int j = 0; j < n_mats; ++j) {
    const size_t m = (size_t)dims[3 * j] * dims[3 * j + 1] * dims[3 * j + 2];
    for (size_t t = 0; t < m; ++t, ++i) {
      snprintf(buf, sizeof buf, "%d ", index[i]);
      pos = put(out, cap, pos, buf);
    }
    pos = put(out, cap, pos, "\n");
  }
  free(dict);
  free(index);
  return pos;
}

/* network::read's DISTILLATION_MODE=1 branch (network.h:958-997) on a weights
 * section: U pairs (index, value read by `>>` = strtof), then W[i] =
 * unique_mapping[index] (std::map operator[]: 0.0f for an index it lacks).
 * Returns 0, or -1 on malformed text. */
int fo_read_weights_section(const char* text, size_t len, const int32_t* dims, int n_mats, float* w_out) {
  char* s = (char*)malloc(len + 1);
  memcpy(s, text, len);
  s[len] = 0;
  char* p = s;
  char* e;
  long loop_counter = strtol(p, &e, 10);
  if (e == p) goto bad;
  p = e;
  long U = strtol(p, &e, 10);
  if (e == p || U < 0) goto bad;
  p = e;
  (void)loop_counter;
  {
    /* std::map semantics: insert keeps the first value for a repeated key */
    long* keys = (long*)malloc(sizeof(long) * (U ? U : 1));
    float* vals = (float*)malloc(sizeof(float) * (U ? U : 1));
    long nk = 0;
    for (long k = 0; k < U; ++k) {
      long idx = strtol(p, &e, 10);
      if (e == p) { free(keys); free(vals); goto bad; }
      p = e;
      float v = strtof(p, &e);
      if (e == p) { free(keys); free(vals); goto bad; }
      p = e;
      int dup = 0;
      for (long q = 0; q < nk; ++q)
        if (keys[q] == idx) { dup = 1; break; }
      if (!dup) { keys[nk] = idx; vals[nk] = v; ++nk; }
    }
    size_t i = 0;
    for (int j = 0; j < n_mats; ++j) {
      const size_t m = (size_t)dims[3 * j] * dims[3 * j + 1] * dims[3 * j + 2];
      for (size_t t = 0; t < m; ++t, ++i) {
        long idx = strtol(p, &e, 10);
        if (e == p) { free(keys); free(vals); goto bad; }
        p = e;
        float v = 0.0f;
        /* dictionary indices are 0..U-1 in order: direct lookup, else search */
        if (idx >= 0 && idx < nk && keys[idx] == idx)
          v = vals[idx];
        else
          for (long q = 0; q < nk; ++q)
            if (keys[q] == idx) { v = vals[q]; break; }
        w_out[i] = v;
      }
    }
    free(keys);
    free(vals);
  }
  free(s);
  return 0;
bad:
  free(s);
  return -1;
}

/* --------------------------------------------------- SGD epilogue (f1) */

/* descentNative's model step (Server/src/main/c++/cppNN_backend.cpp:336-352):
 * network::descent(vector) (commonLib/cppNN/network.h:1185-1202) reads the
 * dW / dbias blocks of the gradients() layout from g -- sizes are (int) of
 * the decoded header floats -- then descent() (:1334-1353) applies, per
 * weight slot i with a non-empty block and a non-null W[i] (w_present[i]),
 * sgd::increment_w (solver.h:88-94):
 *     w[s] -= lr * (dW[s] + 0.0f * w[s])          (fp32, one rounding per op)
 * and, per layer k that is a fully_connected_layer (fc_layer[k]),
 * update_bias (layer.h:241-243):
 *     b[j] -= db[j] * lr
 * Other layers' update_bias is the base no-op (layer.h:108). `weights` holds
 * the non-null W concatenated in slot order; `fc_bias` the FC layers' biases
 * in layer order. Returns 0, or -1 when g's header does not fit the model. */
/* x86 SSE NaN results (Intel SDM vol. 1, 4.8.3.5), restated so they do not
 * depend on how this file's compiler orders commutative operands: r = a OP b
 * with a the instruction's first (destination) operand as the reference's
 * -O0 build emits it -- a NaN operand propagates quieted, the first one
 * winning; an invalid operation on non-NaN operands gives the default NaN
 * 0xFFC00000. The operand orders below were read off the reference build
 * (tests/golden/descent_mnist.npz case 2). */
static float x86_nan(float a, float b, float r) {
  union { float f; uint32_t u; } x;
  if (r == r) return r;
  if (a != a) { x.f = a; x.u |= 0x00400000u; return x.f; }
  if (b != b) { x.f = b; x.u |= 0x00400000u; return x.f; }
  x.u = 0xFFC00000u;
  return x.f;
}

int fo_descent(float* weights, size_t n_weights, float* fc_bias, size_t n_fc_bias, const float* g, size_t n_g,
               const uint8_t* w_present, int n_w_slots, const uint8_t* fc_layer, int n_layers, float lr) {
  size_t idx = 0, wo = 0, bo = 0;
  if (n_g < 1) return -1;
  const int nw = (int)g[idx++];
  if (nw != n_w_slots) return -1;
  for (int i = 0; i < nw; ++i) {
    if (idx >= n_g) return -1;
    const int size = (int)g[idx++];
    if (size < 0 || idx + (size_t)size > n_g) return -1;
    if (w_present[i] && size > 0) {
      if (wo + (size_t)size > n_weights) return -1;
      for (int s = 0; s < size; ++s) {
        float* w = &weights[wo + (size_t)s];
        const float x = *w, d = g[idx + (size_t)s];
        const float t = x86_nan(0.0f, x, 0.0f * x); /* w_decay * w */
        const float u = x86_nan(t, d, t + d);       /* dW + t: the product is the first operand */
        const float v = x86_nan(lr, u, lr * u);
        *w = x86_nan(x, v, x - v);
      }
    }
    if (w_present[i]) wo += (size_t)size;
    idx += (size_t)size;
  }
  if (idx >= n_g) return -1;
  const int nb = (int)g[idx++];
  if (nb != n_layers) return -1;
  for (int k = 0; k < nb; ++k) {
    if (idx >= n_g) return -1;
    const int size = (int)g[idx++];
    if (size < 0 || idx + (size_t)size > n_g) return -1;
    if (fc_layer[k]) {
      if (bo + (size_t)size > n_fc_bias) return -1;
      for (int j = 0; j < size; ++j) {
        const float d = g[idx + (size_t)j], b = fc_bias[bo + (size_t)j];
        const float v = x86_nan(d, lr, d * lr);
        fc_bias[bo + (size_t)j] = x86_nan(b, v, b - v);
      }
      bo += (size_t)size;
    }
    idx += (size_t)size;
  }
  return 0;
}

/* ------------------------------------------------ mode-1 teacher forward */

static float fo_elu(float x, float bias) { /* activation.h:172-176 */
  if ((x + bias) < 0) return 0.1f * (expf(x + bias) - 1.f);
  return x + bias;
}

/* layer.h:481-556 on a P x P window of a channel (row stride js) */
static float fo_semi_pool(const float* top, int base, int js, int P) {
  int max_i = base, max2_i = base;
  float mx = top[base], mx2 = mx;
  for (int jj = 0; jj < P; jj++)
    for (int ii = 0; ii < P; ii++) {
      const int index = base + ii + jj * js;
      if (mx < top[index]) {
        mx2 = mx;
        max2_i = max_i;
        mx = top[index];
        max_i = index;
      } else if (mx2 < top[index]) {
        mx2 = top[index];
        max2_i = index;
      }
    }
  const int r = 34909 % 100;
  const float denom = mx + mx2;
  if (denom == 0) return top[max_i];
  const int t1 = fo_cvtt(100 * mx / (mx + mx2));
  return (r <= t1) ? top[max_i] : top[max2_i]; /* train == 1 */
}

void fo_teacher_forward(const float* w, const float* b, const float* x, float temperature, float* probs) {
  static const int W1 = 0, W2i = 200, W2 = 328, Wfc = 328 + 19200;
  static const int B1 = 0, B2i = 8, B2 = 24;
  float c1[8 * 576], p1[8 * 64], c2i[16 * 64], c2[48 * 16], p2[192], fc[10];
  /* C1 (the node is zeroed, then one running sum per output) */
  for (int map = 0; map < 8; map++)
    for (int y = 0; y < 24; y++)
      for (int xx = 0; xx < 24; xx++) {
        float c = 0;
        for (int k = 0; k < 5; k++)
          for (int m = 0; m < 5; m++) c += x[(y + k) * 28 + xx + m] * w[W1 + map * 25 + k * 5 + m];
        c1[map * 576 + y * 24 + xx] = c;
      }
  for (int map = 0; map < 8; map++)
    for (int i = 0; i < 576; i++) c1[map * 576 + i] = fo_elu(c1[map * 576 + i], b[B1 + map]);
  /* P1 */
  for (int k = 0, o = 0; k < 8; k++)
    for (int j = 0; j <= 24 - 3; j += 3)
      for (int i = 0; i <= 24 - 3; i += 3) p1[o++] = fo_semi_pool(c1, i + j * 24 + k * 576, 24, 3);
  /* C2i: input channel outer, map, position */
  for (int i = 0; i < 16 * 64; i++) c2i[i] = 0;
  for (int k = 0; k < 8; k++)
    for (int map = 0; map < 16; map++) {
      const float cw = w[W2i + map + k * 16];
      for (int j = 0; j < 64; j++) c2i[j + 64 * map] += p1[k * 64 + j] * cw;
    }
  for (int map = 0; map < 16; map++)
    for (int i = 0; i < 64; i++) c2i[map * 64 + i] = fo_elu(c2i[map * 64 + i], b[B2i + map]);
  /* C2: input channel outer, map, position, tap */
  for (int i = 0; i < 48 * 16; i++) c2[i] = 0;
  for (int k = 0; k < 16; k++)
    for (int map = 0; map < 48; map++)
      for (int y = 0; y < 4; y++)
        for (int xx = 0; xx < 4; xx++) {
          float* c = &c2[map * 16 + y * 4 + xx];
          for (int t = 0; t < 25; t++)
            *c += c2i[k * 64 + (y + t / 5) * 8 + xx + t % 5] * w[W2 + (k * 48 + map) * 25 + t];
        }
  for (int map = 0; map < 48; map++)
    for (int i = 0; i < 16; i++) c2[map * 16 + i] = fo_elu(c2[map * 16 + i], b[B2 + map]);
  /* P2 */
  for (int k = 0, o = 0; k < 48; k++)
    for (int j = 0; j <= 4 - 2; j += 2)
      for (int i = 0; i <= 4 - 2; i += 2) p2[o++] = fo_semi_pool(c2, i + j * 4 + k * 16, 4, 2);
  /* FC2 */
  for (int j = 0; j < 10; j++) {
    float v = 0;
    for (int i = 0; i < 192; i++) v += p2[i] * w[Wfc + j * 192 + i];
    fc[j] = 0;
    fc[j] += v;
  }
  /* softmax */
  float mx = fc[0];
  for (int j = 1; j < 10; j++)
    if (fc[j] > mx) mx = fc[j] / temperature;
  float denom = 0;
  for (int j = 0; j < 10; j++) denom += expf(fc[j] / temperature - mx);
  for (int i = 0; i < 10; i++) probs[i] = expf(fc[i] / temperature - mx) / denom;
}

static uint64_t fo_splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t fo_expf_digest(void) {
  uint64_t sum = 0;
#pragma omp parallel for reduction(+ : sum) schedule(static)
  for (int64_t hi = 0; hi < 65536; ++hi) {
    uint64_t part = 0;
    for (uint32_t lo = 0; lo < 65536; ++lo) {
      const uint32_t u = (uint32_t)(hi << 16) | lo;
      float xv;
      memcpy(&xv, &u, 4);
      const float e = expf(xv);
      uint32_t o;
      memcpy(&o, &e, 4);
      if (e != e) o = 0x7fc00000u;
      part += fo_splitmix64(((uint64_t)u << 32) | o);
    }
    sum += part;
  }
  return sum;
}
