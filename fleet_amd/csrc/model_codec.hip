// fleet_amd/csrc/model_codec.hip -- the DISTILLATION_MODE=1 model codec on gfx950
// (SURVEY.md §8 rows a15-a19): per-matrix min-max quantisation, the
// first-occurrence dictionary and the selected-index set that getParams
// prints, and the read-back of that text.
//
// Reference semantics (all restated bit-exactly):
//   quantization_weight_model  commonLib/cppNN/network.h:1683-1774 (non-bucketing path)
//   matrix::min_max             commonLib/cppNN/core_math.h:881-899
//   matrix::round_matrix        core_math.h:901-912 (s = rows*cols: the shadowed parameter)
//   operator+(float), *(float)  core_math.h:1045-1056
//   float_vector_find           network.h:594-608 (first entry with fabsf(x - e) < 1e-8f)
//   getParams mode-1 section    network.h:641-692
//   network::read mode-1 branch network.h:958-997
//
// Layout: the W matrices of a model concatenated in W order (n floats), each
// cols*rows*chans (chan_aligned = 0, no padding), matrix j at offset off[j].
//
// The dictionary is built without the reference's O(n*U) scans: values are
// radix-sorted (stable, so equal values keep index order); a "cluster" is a
// maximal run of sorted neighbours closer than the tolerance. Two values in
// different clusters never match (their float difference is at least the
// gap at the cluster boundary: rounding is monotone), so every cluster is
// resolved alone: a cluster of equal values is one entry created by its
// first occurrence; a cluster of distinct near-equal values (a tolerance
// chain, where non-transitivity matters) replays the reference's sequential
// rule over its members in index order. Entry creators ranked by index give
// the dictionary order; NaN/inf match nothing (fabsf(NaN) < tol is false),
// each creates an entry and prints index -1 (the reference's pass 2).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "model_codec.h"
#include "decimal6.h"

namespace fleet {

// Device-wide sums and the key sort on rocPRIM, AMD's own primitives library (its
// wave-level scans and LDS radix passes are tuned for CDNA; no CUB-compatible layer).
// Each call with tmp == nullptr only sizes the temporary storage, as in rocPRIM.
template <class T>
static hipError_t inclusive_sum(void* tmp, size_t& bytes, const T* in, T* out, size_t n, hipStream_t s) {
  return rocprim::inclusive_scan(tmp, bytes, in, out, n, rocprim::plus<T>(), s);
}
template <class T>
static hipError_t exclusive_sum(void* tmp, size_t& bytes, const T* in, T* out, size_t n, hipStream_t s) {
  return rocprim::exclusive_scan(tmp, bytes, in, out, T(0), n, rocprim::plus<T>(), s);
}
static hipError_t sort_pairs(void* tmp, size_t& bytes, const uint32_t* keys, uint32_t* keys_out, const int32_t* vals,
                             int32_t* vals_out, size_t n, hipStream_t s) {
  return rocprim::radix_sort_pairs(tmp, bytes, keys, keys_out, vals, vals_out, n, 0u, 32u, s);
}
namespace {

constexpr float kTol = 0.00000001f;

struct MatParams {
  float alpha, beta, nbeta, ialpha, fs, one_over_s;
};

__device__ __forceinline__ bool finite_f(float x) { return __builtin_isfinite(x); }

// matrix::min_max: mini/maxi start at 0 and move on a strict < / > -- the
// first index of the extreme value, NaN never selected unless x[0] is NaN.
__global__ void __launch_bounds__(256) k_mm_minmax(const float* __restrict__ w, const int64_t* __restrict__ off,
                                                   const int32_t* __restrict__ dims, MatParams* __restrict__ prm) {
  const int j = blockIdx.x;
  const int64_t o = off[j], n = off[j + 1] - off[j];
  const int s = dims[3 * j] * dims[3 * j + 1];
  __shared__ float smin[256], smax[256];
  __shared__ int64_t simin[256], simax[256];
  float bmin = 0.f, bmax = 0.f;
  int64_t imin = -1, imax = -1;  // -1: nothing seen yet
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    const float x = w[o + i];
    if (x != x) continue;
    if (imin < 0 || x < bmin) bmin = x, imin = i;
    if (imax < 0 || x > bmax) bmax = x, imax = i;
  }
  smin[threadIdx.x] = bmin;
  smax[threadIdx.x] = bmax;
  simin[threadIdx.x] = imin;
  simax[threadIdx.x] = imax;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) {
      const int t = threadIdx.x, u = t + st;
      if (simin[u] >= 0 &&
          (simin[t] < 0 || smin[u] < smin[t] || (smin[u] == smin[t] && simin[u] < simin[t])))
        smin[t] = smin[u], simin[t] = simin[u];
      if (simax[u] >= 0 &&
          (simax[t] < 0 || smax[u] > smax[t] || (smax[u] == smax[t] && simax[u] < simax[t])))
        smax[t] = smax[u], simax[t] = simax[u];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float mn, mx;
    if (n == 0) {
      mn = mx = 0.f;
    } else if (w[o] != w[o]) {  // x[0] NaN: no comparison ever moves mini/maxi off 0
      mn = mx = w[o];
    } else {
      mn = smin[0];
      mx = smax[0];
    }
    MatParams p;
    p.alpha = mx - mn;
    p.beta = mn;
    p.nbeta = (float)(-1.0 * (double)mn);
    p.ialpha = (float)(1.0 / (double)p.alpha);
    p.fs = (float)s;
    p.one_over_s = (float)(1 / s);
    prm[j] = p;
  }
}

__device__ __forceinline__ int mat_of(const int64_t* __restrict__ off, int n_mats, int64_t i) {
  int lo = 0, hi = n_mats;  // off[lo] <= i < off[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (off[mid] <= i) lo = mid; else hi = mid;
  }
  return lo;
}

// x + (-beta); * (1/alpha); round_matrix(s); * alpha; + beta -- one rounding per step.
__global__ void __launch_bounds__(256) k_mm_quantize(const float* __restrict__ w, int64_t n,
                                                     const int64_t* __restrict__ off, int n_mats,
                                                     const MatParams* __restrict__ prm, float* __restrict__ wq) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const MatParams p = prm[mat_of(off, n_mats, i)];
  float x = w[i] + p.nbeta;
  x = x * p.ialpha;
  if (x - floorf(x) > 0.5f)
    x = floorf(x * p.fs) / p.fs + p.one_over_s;
  else
    x = floorf(x * p.fs) / p.fs;
  x = x * p.alpha;
  wq[i] = x + p.beta;
}

// order-preserving key; NaN/inf last (they never match, their order is by index)
__global__ void __launch_bounds__(256) k_dict_keys(const float* __restrict__ w, int64_t n, uint32_t* __restrict__ key,
                                                   int32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float x = w[i];
  uint32_t u = __float_as_uint(x);
  if (!finite_f(x))
    u = 0xFFFFFFFFu;
  else if (u == 0x80000000u)
    u = 0x80000000u;  // -0 sorts with +0 (fabsf(-0 - 0) = 0 < tol)
  else
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  key[i] = u;
  idx[i] = (int32_t)i;
}

// start[k] = 1 where a new cluster begins in sorted order
__global__ void __launch_bounds__(256) k_dict_starts(const float* __restrict__ w, const int32_t* __restrict__ sidx,
                                                     int64_t n, int32_t* __restrict__ start) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  int32_t st = 1;
  if (k > 0) {
    const float a = w[sidx[k - 1]], b = w[sidx[k]];
    if (finite_f(a) && finite_f(b) && fabsf(b - a) < kTol) st = 0;
  }
  start[k] = st;
}

// cluster c spans sorted positions [cbeg[c], cbeg[c+1])
__global__ void __launch_bounds__(256) k_dict_cbeg(const int32_t* __restrict__ start,
                                                   const int32_t* __restrict__ cid_incl, int64_t n,
                                                   int32_t* __restrict__ cbeg) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  if (start[k]) cbeg[cid_incl[k] - 1] = (int32_t)k;
}

// One thread per cluster: creator (original index of the element that created
// the member's dictionary entry) for every member; is_creator flags.
__global__ void __launch_bounds__(256) k_dict_resolve(const float* __restrict__ w, const int32_t* __restrict__ sidx,
                                                      const int32_t* __restrict__ cbeg, int32_t n_clusters,
                                                      int32_t* __restrict__ creator_of_sorted,
                                                      uint8_t* __restrict__ is_creator,
                                                      int32_t* __restrict__ scratch /* n: entry list */) {
  const int32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n_clusters) return;
  const int32_t a = cbeg[c], b = cbeg[c + 1];
  const float va = w[sidx[a]], vb = w[sidx[b - 1]];
  if (!finite_f(va)) {  // NaN / inf: singleton, creates an entry, prints -1
    creator_of_sorted[a] = sidx[a];
    is_creator[sidx[a]] = 1;
    return;
  }
  if (va == vb) {  // all equal (sorted): one entry, created by the first occurrence
    const int32_t cr = sidx[a];  // stable sort: smallest index first
    is_creator[cr] = 1;
    for (int32_t k = a; k < b; ++k) creator_of_sorted[k] = cr;
    return;
  }
  // tolerance chain: the reference's sequential rule over members in index
  // order. Entries (sorted positions) kept in scratch[a..). Members are
  // visited by increasing original index (selection over the run).
  int32_t n_ent = 0;
  int32_t last = -1;
  for (int32_t done = 0; done < b - a; ++done) {
    int32_t kk = -1, best = 0x7FFFFFFF;
    for (int32_t k = a; k < b; ++k) {
      const int32_t id = sidx[k];
      if (id > last && id < best) best = id, kk = k;
    }
    last = best;
    const float x = w[best];
    int32_t cr = -1;
    for (int32_t e = 0; e < n_ent; ++e) {
      const int32_t ek = scratch[a + e];
      if (fabsf(x - w[sidx[ek]]) < kTol) {
        cr = sidx[ek];
        break;
      }
    }
    if (cr < 0) {
      scratch[a + n_ent++] = kk;
      cr = best;
      is_creator[best] = 1;
    }
    creator_of_sorted[kk] = cr;
  }
}

__global__ void __launch_bounds__(256) k_dict_u8_to_i32(const uint8_t* __restrict__ f, int64_t n,
                                                        int32_t* __restrict__ o) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) o[i] = f[i];
}

// dictionary value at each creator's rank; index of every element
__global__ void __launch_bounds__(256) k_dict_emit(const float* __restrict__ w, const int32_t* __restrict__ sidx,
                                                   const int32_t* __restrict__ creator_of_sorted,
                                                   const uint8_t* __restrict__ is_creator,
                                                   const int32_t* __restrict__ rank, int64_t n,
                                                   float* __restrict__ dict, int32_t* __restrict__ index) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const int32_t i = sidx[k];
  if (is_creator[i]) dict[rank[i]] = w[i];
  if (index) index[i] = finite_f(w[i]) ? rank[creator_of_sorted[k]] : -1;
}

// ------------------------------------------------------------ text (a17)

__device__ __forceinline__ int dec_len(int32_t v) {
  uint32_t a = v < 0 ? 0u - (uint32_t)v : (uint32_t)v;
  int d = 1;
  while (a >= 10u) a /= 10u, ++d;
  return d + (v < 0);
}

// bytes of element i in the index section: digits + ' ' (+ '\n' after a matrix's last)
__global__ void __launch_bounds__(256) k_text_len(const int32_t* __restrict__ index, int64_t n,
                                                  const int64_t* __restrict__ off, int n_mats,
                                                  int64_t* __restrict__ len) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int j = mat_of(off, n_mats, i);
  len[i] = dec_len(index[i]) + 1 + (i + 1 == off[j + 1] ? 1 : 0);
}

__global__ void __launch_bounds__(256) k_text_write(const int32_t* __restrict__ index, int64_t n,
                                                    const int64_t* __restrict__ off, int n_mats,
                                                    const int64_t* __restrict__ pos, char* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int j = mat_of(off, n_mats, i);
  int32_t v = index[i];
  char* p = out + pos[i];
  const int l = dec_len(v);
  uint32_t a = v < 0 ? 0u - (uint32_t)v : (uint32_t)v;
  if (v < 0) p[0] = '-';
  for (int q = l - 1; q >= (v < 0); --q) {
    p[q] = (char)('0' + a % 10u);
    a /= 10u;
  }
  p[l] = ' ';
  if (i + 1 == off[j + 1]) p[l + 1] = '\n';
}

// ------------------------------------------------------------ read (a19)

__device__ __forceinline__ bool is_ws(uint8_t c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r'; }
__device__ __forceinline__ bool tok_char(uint8_t c) { return c == '-' || c == '+' || (c >= '0' && c <= '9'); }

__global__ void __launch_bounds__(256) k_read_starts(const uint8_t* __restrict__ t, int64_t len,
                                                     int32_t* __restrict__ st) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= len) return;
  st[p] = tok_char(t[p]) && (p == 0 || is_ws(t[p - 1])) ? 1 : 0;
}

// token number t (from the inclusive scan) -> weight t = value of its key
__global__ void __launch_bounds__(256) k_read_tokens(const uint8_t* __restrict__ t, int64_t len,
                                                     const int32_t* __restrict__ st,
                                                     const int32_t* __restrict__ tok_incl, int64_t n_w,
                                                     const int32_t* __restrict__ keys,
                                                     const float* __restrict__ vals, int32_t n_keys,
                                                     float* __restrict__ w, int* __restrict__ bad) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= len || !st[p]) return;
  const int64_t tk = tok_incl[p] - 1;
  // `ifs >> int`: optional sign, digits; the reference's own texts only
  int64_t q = p;
  bool neg = false;
  if (t[q] == '-' || t[q] == '+') neg = t[q++] == '-';
  int64_t v = 0;
  int nd = 0;
  while (q < len && t[q] >= '0' && t[q] <= '9' && nd < 12) v = v * 10 + (t[q++] - '0'), ++nd;
  if (nd == 0 || nd >= 12 || (q < len && !is_ws(t[q]))) {
    atomicOr(bad, 1);
    return;
  }
  if (neg) v = -v;
  if (tk >= n_w) {
    atomicOr(bad, 2);
    return;
  }
  // std::map<int,float> operator[]: the value of the key, 0.0f when absent
  int32_t lo = 0, hi = n_keys;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (keys[mid] < v) lo = mid + 1; else hi = mid;
  }
  w[tk] = (lo < n_keys && keys[lo] == v) ? vals[lo] : 0.0f;
}

inline unsigned nb(int64_t n) { return (unsigned)((n + 255) / 256); }

template <typename T>
struct DevBuf {
  T* p = nullptr;
  hipError_t alloc(size_t n) { return hipMalloc((void**)&p, sizeof(T) * (n ? n : 1)); }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

#define MC_TRY(x)                      \
  do {                                 \
    hipError_t e_ = (x);               \
    if (e_ != hipSuccess) return e_;   \
  } while (0)

}  // namespace

hipError_t model_quantize_index(const float* d_w, const int32_t* h_dims, int n_mats, float* d_wq, float* d_dict,
                                int32_t* d_index, int32_t* h_U, hipStream_t s, bool quantize) {
  std::vector<int64_t> off(n_mats + 1, 0);
  for (int j = 0; j < n_mats; ++j) off[j + 1] = off[j] + (int64_t)h_dims[3 * j] * h_dims[3 * j + 1] * h_dims[3 * j + 2];
  const int64_t n = off[n_mats];
  *h_U = 0;
  if (n == 0) return hipSuccess;
  DevBuf<int64_t> d_off;
  DevBuf<int32_t> d_dims;
  DevBuf<MatParams> d_prm;
  MC_TRY(d_off.alloc(n_mats + 1));
  MC_TRY(d_dims.alloc(3 * n_mats));
  MC_TRY(d_prm.alloc(n_mats));
  MC_TRY(hipMemcpyAsync(d_off.p, off.data(), sizeof(int64_t) * (n_mats + 1), hipMemcpyHostToDevice, s));
  MC_TRY(hipMemcpyAsync(d_dims.p, h_dims, sizeof(int32_t) * 3 * n_mats, hipMemcpyHostToDevice, s));
  if (quantize) {
    hipLaunchKernelGGL(k_mm_minmax, dim3(n_mats), dim3(256), 0, s, d_w, d_off.p, d_dims.p, d_prm.p);
    hipLaunchKernelGGL(k_mm_quantize, dim3(nb(n)), dim3(256), 0, s, d_w, n, d_off.p, n_mats, d_prm.p, d_wq);
    MC_TRY(hipGetLastError());
  } else {  // the dictionary of the weights as they are (descentNative's model copy)
    d_wq = const_cast<float*>(d_w);
  }

  // dictionary over the quantised weights
  DevBuf<uint32_t> key, key2;
  DevBuf<int32_t> idx, sidx, start, cid, cbeg, creator, scratch, rank, flag32;
  DevBuf<uint8_t> is_creator;
  MC_TRY(key.alloc(n));
  MC_TRY(key2.alloc(n));
  MC_TRY(idx.alloc(n));
  MC_TRY(sidx.alloc(n));
  MC_TRY(start.alloc(n));
  MC_TRY(cid.alloc(n));
  MC_TRY(cbeg.alloc(n + 1));
  MC_TRY(creator.alloc(n));
  MC_TRY(scratch.alloc(n));
  MC_TRY(rank.alloc(n));
  MC_TRY(flag32.alloc(n));
  MC_TRY(is_creator.alloc(n));
  hipLaunchKernelGGL(k_dict_keys, dim3(nb(n)), dim3(256), 0, s, d_wq, n, key.p, idx.p);
  size_t tmp_bytes = 0, t2 = 0, t3 = 0;
  MC_TRY(sort_pairs(nullptr, tmp_bytes, key.p, key2.p, idx.p, sidx.p, n, s));
  MC_TRY(inclusive_sum(nullptr, t2, start.p, cid.p, n, s));
  MC_TRY(exclusive_sum(nullptr, t3, flag32.p, rank.p, n, s));
  tmp_bytes = std::max(tmp_bytes, std::max(t2, t3));
  DevBuf<uint8_t> tmp;
  MC_TRY(tmp.alloc(tmp_bytes));
  MC_TRY(sort_pairs(tmp.p, tmp_bytes, key.p, key2.p, idx.p, sidx.p, n, s));
  hipLaunchKernelGGL(k_dict_starts, dim3(nb(n)), dim3(256), 0, s, d_wq, sidx.p, n, start.p);
  size_t tb = tmp_bytes;
  MC_TRY(inclusive_sum(tmp.p, tb, start.p, cid.p, n, s));
  int32_t n_clusters = 0;
  MC_TRY(hipMemcpyAsync(&n_clusters, cid.p + (n - 1), sizeof(int32_t), hipMemcpyDeviceToHost, s));
  MC_TRY(hipStreamSynchronize(s));
  hipLaunchKernelGGL(k_dict_cbeg, dim3(nb(n)), dim3(256), 0, s, start.p, cid.p, n, cbeg.p);
  const int32_t nn = (int32_t)n;
  MC_TRY(hipMemcpyAsync(cbeg.p + n_clusters, &nn, sizeof(int32_t), hipMemcpyHostToDevice, s));
  MC_TRY(hipMemsetAsync(is_creator.p, 0, n, s));
  hipLaunchKernelGGL(k_dict_resolve, dim3(nb(n_clusters)), dim3(256), 0, s, d_wq, sidx.p, cbeg.p, n_clusters,
                     creator.p, is_creator.p, scratch.p);
  hipLaunchKernelGGL(k_dict_u8_to_i32, dim3(nb(n)), dim3(256), 0, s, is_creator.p, n, flag32.p);
  tb = tmp_bytes;
  MC_TRY(exclusive_sum(tmp.p, tb, flag32.p, rank.p, n, s));
  int32_t last_rank = 0, last_flag = 0;
  MC_TRY(hipMemcpyAsync(&last_rank, rank.p + (n - 1), sizeof(int32_t), hipMemcpyDeviceToHost, s));
  MC_TRY(hipMemcpyAsync(&last_flag, flag32.p + (n - 1), sizeof(int32_t), hipMemcpyDeviceToHost, s));
  hipLaunchKernelGGL(k_dict_emit, dim3(nb(n)), dim3(256), 0, s, d_wq, sidx.p, creator.p, is_creator.p, rank.p, n,
                     d_dict, d_index);
  MC_TRY(hipGetLastError());
  MC_TRY(hipStreamSynchronize(s));
  *h_U = last_rank + last_flag;
  return hipSuccess;
}

// w[i] = vals[index[i]] (index -1, a non-finite weight: 0.0f, std::map::operator[])
__global__ void __launch_bounds__(256) k_dict_gather(const int32_t* __restrict__ index, int64_t n,
                                                     const float* __restrict__ vals, float* __restrict__ w) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int32_t k = index[i];
  w[i] = k >= 0 ? vals[k] : 0.0f;
}

__global__ void __launch_bounds__(256) k_g6_inplace(float* __restrict__ v, int64_t n, int* __restrict__ bad) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float x = v[i];
  if ((f2u(x) & 0x7f800000u) == 0x7f800000u) {  // inf / NaN: the reference's text read fails
    atomicOr(bad, 1);
    return;
  }
  v[i] = g6_roundtrip(x);
}

hipError_t model_g6_inplace(float* d_v, int64_t n, int* d_bad, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_g6_inplace, dim3(nb(n)), dim3(256), 0, s, d_v, n, d_bad);
  return hipGetLastError();
}

hipError_t model_dict_gather(const int32_t* d_index, int64_t n, const float* d_vals, float* d_w, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_dict_gather, dim3(nb(n)), dim3(256), 0, s, d_index, n, d_vals, d_w);
  return hipGetLastError();
}

hipError_t model_index_text(const int32_t* d_index, const int32_t* h_dims, int n_mats, std::vector<char>* out,
                            hipStream_t s) {
  std::vector<int64_t> off(n_mats + 1, 0);
  for (int j = 0; j < n_mats; ++j) off[j + 1] = off[j] + (int64_t)h_dims[3 * j] * h_dims[3 * j + 1] * h_dims[3 * j + 2];
  const int64_t n = off[n_mats];
  // matrices of size 0 still print their '\n' (the reference loops W[j] non-null)
  out->clear();
  if (n == 0) {
    out->assign((size_t)n_mats, '\n');
    return hipSuccess;
  }
  DevBuf<int64_t> d_off, len, pos;
  DevBuf<char> txt;
  MC_TRY(d_off.alloc(n_mats + 1));
  MC_TRY(len.alloc(n));
  MC_TRY(pos.alloc(n));
  MC_TRY(hipMemcpyAsync(d_off.p, off.data(), sizeof(int64_t) * (n_mats + 1), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_text_len, dim3(nb(n)), dim3(256), 0, s, d_index, n, d_off.p, n_mats, len.p);
  size_t tb = 0;
  MC_TRY(exclusive_sum(nullptr, tb, len.p, pos.p, n, s));
  DevBuf<uint8_t> tmp;
  MC_TRY(tmp.alloc(tb));
  MC_TRY(exclusive_sum(tmp.p, tb, len.p, pos.p, n, s));
  int64_t last_pos = 0, last_len = 0;
  MC_TRY(hipMemcpyAsync(&last_pos, pos.p + (n - 1), sizeof(int64_t), hipMemcpyDeviceToHost, s));
  MC_TRY(hipMemcpyAsync(&last_len, len.p + (n - 1), sizeof(int64_t), hipMemcpyDeviceToHost, s));
  MC_TRY(hipStreamSynchronize(s));
  const int64_t total = last_pos + last_len;
  MC_TRY(txt.alloc(total));
  hipLaunchKernelGGL(k_text_write, dim3(nb(n)), dim3(256), 0, s, d_index, n, d_off.p, n_mats, pos.p, txt.p);
  MC_TRY(hipGetLastError());
  // empty matrices print a lone '\n' in their place: stitch them in on the host
  std::vector<char> body((size_t)total);
  MC_TRY(hipMemcpyAsync(body.data(), txt.p, (size_t)total, hipMemcpyDeviceToHost, s));
  MC_TRY(hipStreamSynchronize(s));
  bool any_empty = false;
  for (int j = 0; j < n_mats; ++j) any_empty |= off[j + 1] == off[j];
  if (!any_empty) {
    out->swap(body);
    return hipSuccess;
  }
  // positions of each matrix's text: recompute from the line breaks
  size_t p = 0;
  for (int j = 0; j < n_mats; ++j) {
    if (off[j + 1] == off[j]) {
      out->push_back('\n');
      continue;
    }
    const size_t q = (size_t)(std::find(body.begin() + p, body.end(), '\n') - body.begin()) + 1;
    out->insert(out->end(), body.begin() + p, body.begin() + q);
    p = q;
  }
  return hipSuccess;
}

hipError_t model_read_index(const uint8_t* d_text, int64_t len, int64_t n_w, const int32_t* d_keys,
                            const float* d_vals, int32_t n_keys, float* d_w, int* h_status, hipStream_t s) {
  *h_status = 0;
  if (len == 0) {
    *h_status = n_w ? 2 : 0;
    return hipSuccess;
  }
  DevBuf<int32_t> st, tok;
  DevBuf<int> bad;
  MC_TRY(st.alloc(len));
  MC_TRY(tok.alloc(len));
  MC_TRY(bad.alloc(1));
  MC_TRY(hipMemsetAsync(bad.p, 0, sizeof(int), s));
  hipLaunchKernelGGL(k_read_starts, dim3(nb(len)), dim3(256), 0, s, d_text, len, st.p);
  size_t tb = 0;
  MC_TRY(inclusive_sum(nullptr, tb, st.p, tok.p, (size_t)len, s));
  DevBuf<uint8_t> tmp;
  MC_TRY(tmp.alloc(tb));
  MC_TRY(inclusive_sum(tmp.p, tb, st.p, tok.p, (size_t)len, s));
  hipLaunchKernelGGL(k_read_tokens, dim3(nb(len)), dim3(256), 0, s, d_text, len, st.p, tok.p, n_w, d_keys, d_vals,
                     n_keys, d_w, bad.p);
  MC_TRY(hipGetLastError());
  int32_t n_tok = 0;
  int hbad = 0;
  MC_TRY(hipMemcpyAsync(&n_tok, tok.p + (len - 1), sizeof(int32_t), hipMemcpyDeviceToHost, s));
  MC_TRY(hipMemcpyAsync(&hbad, bad.p, sizeof(int), hipMemcpyDeviceToHost, s));
  MC_TRY(hipStreamSynchronize(s));
  *h_status = hbad ? hbad : (n_tok != n_w ? 2 : 0);
  return hipSuccess;
}

}  // namespace fleet
