/*
 * oracle/fleet_oracle.c -- TEST INFRASTRUCTURE ONLY (see fleet_oracle.h).
 *
 * Clean-room C restatement of the FLeet cppNN gradient codec + aggregation
 * path. Compiled with -ffp-contract=off and no fast-math so every float op
 * is one IEEE-754 binary32/binary64 round-to-nearest-even operation, exactly
 * like the reference's x86-64 SSE build (Server/Makefile:2, -O0).
 * Parity with the reference's own compiled code: tests/test_oracle_golden.py.
 */
#include "fleet_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------- scalars */

/* Base64.cpp:73-82 -- '-' counts as a digit; numDigits(0) == 0. */
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

/* Base64.cpp:84-114 with intNum == 1, precision == 9. */
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

/* Base64.cpp:116-139 with intNum == 1, precision == 9. */
float fo_int2float(int32_t c) {
  const int precision = 9;
  int dd = abs(c % 10);
  float t = (float)c;
  for (int j = 0; j < precision - dd; j++) t /= 10; /* fp32 divide, correctly rounded */
  return t;
}

float fo_q(float x) { return fo_int2float(fo_float2int(x)); }

/* ----------------------------------------------------------------- base64 */

/* Base64.cpp:56-68 */
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

/* Base64.cpp:160-205 */
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
  /* `(ch <= 'z') ? from_base64[ch] : 0xff` (Base64.cpp:233-236). Bytes >= 0x80
   * index the table out of bounds in the reference (UB); treated as pad here. */
  unsigned char u = (unsigned char)ch;
  return u <= 'z' ? from_b64[u] : 0xff;
}

/* Base64.cpp:221-253 (the string is first padded with '=' to a multiple of 4) */
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

/* Base64.cpp:145-151 */
size_t fo_encode_ints(const int32_t* v, size_t n, char* out) {
  return fo_b64_encode((const uint8_t*)v, n * sizeof(int32_t), out);
}
/* Base64.cpp:140-142 */
size_t fo_encode_floats(const float* v, size_t n, char* out) {
  int32_t* codes = (int32_t*)malloc(sizeof(int32_t) * (n ? n : 1));
  for (size_t i = 0; i < n; ++i) codes[i] = fo_float2int(v[i]);
  size_t r = fo_encode_ints(codes, n, out);
  free(codes);
  return r;
}
/* Base64.cpp:211-219 */
size_t fo_decode_ints(const char* s, size_t len, int32_t* out) {
  uint8_t* bytes = (uint8_t*)malloc(len + 4);
  size_t nb = fo_b64_decode(s, len, bytes);
  size_t n = nb / sizeof(int32_t);
  memcpy(out, bytes, n * sizeof(int32_t));
  free(bytes);
  return n;
}
/* Base64.cpp:207-209 */
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
