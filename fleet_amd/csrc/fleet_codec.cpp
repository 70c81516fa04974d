// fleet_amd/csrc/fleet_codec.cpp -- host side of the C-ABI (include/fleet_codec.h).
//
// Owns device memory, a HIP stream and pinned staging per context; stages
// host Base64 buffers to HBM, launches the gfx950 kernels (kernels.hip) and
// returns bytes identical to the reference's JNI natives. No CPU compute
// path exists: without a GPU every compute entry point returns FLEET_ERR_HIP.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <sched.h>

#include "../../include/fleet_codec.h"
#include "kernels.h"

static_assert(FLEET_MAX_HEADERS == fleet::kMaxHeaderSlots, "the kernels size their LDS header lists by it");
#include "model_codec.h"
#include "codec_device.h"

#define FLEET_VERSION "fleet-mi355x 0.1.0 (gfx950)"

// Persistent host threads for the staging copies of large host-buffer updates
// (one pool per context, created on first use): a thread per part and call
// cost 50-100 us to start on the GPU boxes, more than a part's copy.
class WorkerPool {
 public:
  explicit WorkerPool(int workers) {
    for (int i = 0; i < workers; ++i) ts_.emplace_back([this] { loop(); });
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : ts_) t.join();
  }
  int workers() const { return (int)ts_.size(); }
  // f(i) for every i in [0, n), on the pool's threads and the caller's
  void run(int n, const std::function<void(int)>& f) {
    {
      std::lock_guard<std::mutex> g(m_);
      f_ = &f;
      n_ = n;
      next_.store(0, std::memory_order_relaxed);
      pending_ = (int)ts_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return pending_ == 0; });
    f_ = nullptr;
  }

 private:
  void work() {
    for (int i; (i = next_.fetch_add(1, std::memory_order_relaxed)) < n_;) (*f_)(i);
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      cv_.wait(g, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      g.unlock();
      work();
      g.lock();
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> ts_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* f_ = nullptr;
  int n_ = 0;
  std::atomic<int> next_{0};
  int pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

struct fleet_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::string err;
  // device buffers (grown on demand)
  uint8_t* d_a = nullptr;
  size_t d_a_cap = 0;
  uint8_t* d_b = nullptr;
  size_t d_b_cap = 0;
  uint8_t* d_out = nullptr;
  size_t d_out_cap = 0;
  float* d_f32 = nullptr;
  size_t d_f32_cap = 0;
  double* d_dampen = nullptr;
  size_t d_dampen_cap = 0;
  int32_t* d_hdr = nullptr;  // {status, count, walk_end, 0, positions[FLEET_MAX_HEADERS]}
  int* d_err = nullptr;
  // Device-resident entry points (fleet_*_device) run on the CALLER's stream and
  // may be captured into HIP graphs, so they own parameter buffers of their own:
  // nothing the host-buffer entry points do on the context's stream touches
  // them, and a buffer a captured graph may reference is never freed before
  // fleet_destroy (a grown dampen buffer is retired, not freed).
  double* d_dev_dampen = nullptr;
  size_t d_dev_dampen_cap = 0;
  int32_t* d_dev_hdr = nullptr;
  int* d_dev_err = nullptr;           // read by fleet_check
  std::vector<void*> retired;         // freed in fleet_destroy
  std::vector<double> dev_dampen;     // what d_dev_dampen holds
  std::vector<int32_t> dev_hdr;       // what d_dev_hdr holds
  bool dev_params_valid = false;
  double* d_partials = nullptr;
  size_t d_partials_cap = 0;
  // pinned host staging
  uint8_t* h_stage = nullptr;
  size_t h_stage_cap = 0;
  int32_t* h_hdr = nullptr;
  int* h_err = nullptr;
  std::unique_ptr<WorkerPool> pool;  // staging copy threads (stage_uploads)
  int last_ingress = FLEET_INGRESS_NONE;  // how the last host-buffer update reached HBM
  // the pipelined Kardam form's tile flags (zeroed at allocation) and its launch epoch
  uint32_t* d_kflags = nullptr;
  size_t d_kflags_cap = 0;
  uint32_t kflag_epoch = 0;
  uint32_t kflag_test_skew = 0;       // fleet_test_kardam_skew: reduce blocks wait for a later epoch
};

namespace {

constexpr size_t kHdrWords = FLEET_MAX_HEADERS + 4;  // {status, count, walk_end, 0, positions}

int fail(fleet_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIP_TRY(ctx, expr)                                                                       \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess) return fail((ctx), FLEET_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// Every entry point runs on its context's device and leaves the calling
// thread's current device as it found it (a JVM request thread or a torch
// process keeps its own notion of the current GPU): hipGetDevice on entry,
// hipSetDevice back on every return path.
struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int device) {
    if (hipGetDevice(&prev) != hipSuccess) {
      (void)hipGetLastError();
      prev = -1;
    }
    ok = prev == device || hipSetDevice(device) == hipSuccess;
  }
  ~DeviceGuard() {
    if (ok && prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};
#define DEVICE_SCOPE(ctx)                                                                       \
  DeviceGuard device_guard_((ctx)->device);                                                     \
  if (!device_guard_.ok) return fail((ctx), FLEET_ERR_HIP, "hipSetDevice(%d) failed", (ctx)->device)

template <typename T>
int grow_dev(fleet_ctx* c, T** p, size_t* cap, size_t need_elems) {
  if (need_elems <= *cap) return FLEET_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  size_t n = std::max(need_elems, *cap * 2);
  hipError_t e = hipMalloc((void**)p, n * sizeof(T) + 64);
  if (e != hipSuccess) {
    *cap = 0;
    return fail(c, FLEET_ERR_NOMEM, "hipMalloc(%zu): %s", n * sizeof(T), hipGetErrorString(e));
  }
  *cap = n;
  return FLEET_OK;
}

int grow_pinned(fleet_ctx* c, size_t need) {
  if (need <= c->h_stage_cap) return FLEET_OK;
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  c->h_stage = nullptr;
  size_t n = std::max(need, c->h_stage_cap * 2);
  hipError_t e = hipHostMalloc((void**)&c->h_stage, n + 64, hipHostMallocDefault);
  if (e != hipSuccess) {
    c->h_stage_cap = 0;
    return fail(c, FLEET_ERR_NOMEM, "hipHostMalloc(%zu): %s", n, hipGetErrorString(e));
  }
  c->h_stage_cap = n;
  return FLEET_OK;
}

inline size_t round16(size_t x) { return (x + 15) / 16 * 16; }
inline size_t groups_of(size_t n_values) { return (n_values + 2) / 3; }

// Device-resident entry points run on the caller's stream; NULL is the null
// (default) stream, as in the HIP libraries. Host-buffer entry points use the
// context's own stream.
hipStream_t pick(fleet_ctx*, void* s) { return (hipStream_t)s; }

// Copy host text (len chars) into device buffer padded to 16-byte groups.
int stage_text(fleet_ctx* c, const char* text, size_t len, uint8_t** dbuf, size_t* dcap) {
  size_t padded = round16(len) + 16;
  int rc = grow_dev(c, dbuf, dcap, padded);
  if (rc) return rc;
  HIP_TRY(c, hipMemsetAsync(*dbuf + (len & ~(size_t)15), 0, padded - (len & ~(size_t)15), c->stream));
  if (len) HIP_TRY(c, hipMemcpyAsync(*dbuf, text, len, hipMemcpyHostToDevice, c->stream));
  return FLEET_OK;
}

int check_text_len(fleet_ctx* c, size_t len) {
  if (len % 4 != 0) return fail(c, FLEET_ERR_BASE64, "Base64 length %zu is not a multiple of 4", len);
  return FLEET_OK;
}

int read_err(fleet_ctx* c, hipStream_t s, int* d_errbuf = nullptr) {
  if (!d_errbuf) d_errbuf = c->d_err;
  HIP_TRY(c, hipMemcpyAsync(c->h_err, d_errbuf, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  int e = *c->h_err;
  if (e) {
    HIP_TRY(c, hipMemsetAsync(d_errbuf, 0, sizeof(int), s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  if (e & 1) return fail(c, FLEET_ERR_BASE64, "input is not Base64::encode output (alphabet/padding)");
  if (e & 2) return fail(c, FLEET_ERR_LAYOUT, "uploads disagree on the gradient layout header slots");
  if (e & 4) return fail(c, FLEET_ERR_ARG, "sample index outside the dataset");
  if (e & 8) return fail(c, FLEET_ERR_HIP, "a cross-block hand-off timed out (Kardam reduce blocks)");
  return FLEET_OK;
}

// Parse the layout of the upload at d_text (device) into c->d_hdr / c->h_hdr.
int parse_layout(fleet_ctx* c, const uint8_t* d_text, size_t n_up, int* n_hdr, size_t* walk_end = nullptr) {
  HIP_TRY(c, fleet::launch_layout_parse(d_text, (int64_t)n_up, FLEET_MAX_HEADERS, c->d_hdr, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->h_hdr, c->d_hdr, kHdrWords * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (c->h_hdr[0] != 0)
    return fail(c, FLEET_ERR_LAYOUT, "upload header does not describe a gradient layout (network.h:1038-1056)");
  *n_hdr = c->h_hdr[1];
  if (walk_end) *walk_end = (size_t)c->h_hdr[2];
  return FLEET_OK;
}

int finish_text(fleet_ctx* c, size_t out_len, char* out, size_t cap, size_t* out_len_p) {
  if (out_len_p) *out_len_p = out_len;
  if (cap < out_len) return fail(c, FLEET_ERR_CAPACITY, "output capacity %zu < %zu", cap, out_len);
  if (out_len) HIP_TRY(c, hipMemcpyAsync(out, c->d_out, out_len, hipMemcpyDeviceToHost, c->stream));
  int rc = read_err(c, c->stream);
  return rc;
}

// Host staging copy threads: the plan's stage_threads (fleet_set_plan), else one per
// ~2 MiB of staging, at most 8 and at most the CPUs this process may run on.
int stage_threads(size_t bytes) {
  if (const int t = fleet::plan_overrides().stage_threads) return t;
  int n = 1;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
  return (int)std::max<size_t>(1, std::min<size_t>({bytes >> 21, 8, (size_t)std::max(1, n)}));
}

// f(i) for i in [0, n) on `threads` threads (the caller's and the context's pool).
void parallel_for(fleet_ctx* c, int n, int threads, const std::function<void(int)>& f) {
  threads = std::max(1, std::min(threads, n));
  if (threads == 1) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  if (!c->pool || c->pool->workers() != threads - 1) {
    c->pool.reset();
    c->pool.reset(new WorkerPool(threads - 1));
  }
  c->pool->run(n, f);
}

// Copies bytes [col0, col0 + width) of each of the M uploads into the pinned
// staging rows (pitch apart, zero padded) and queues ONE H2D of [rows |
// tail_bytes already written after the rows] into d_a, in parts, each queued as
// soon as its rows are copied, so the DMA of a part overlaps the copy of the
// next (ingress framing). col0 = 0, width = len stages whole
// uploads; a column window is one GPU's element shard (fleet_update_multi).
// Measured on MI355X (probe_e2e2.py (r04 tree), rocprofv3 memory-copy trace): 1 MiB
// H2D parts run at ~35 GB/s with ~9 us gaps, one 7.8 MB copy at ~53 GB/s; three
// parts gave the shortest host-buffer update for MNIST-64 (0.27 vs 0.32 ms with
// one part). Each part is copied by `threads` workers (the context's pool): one
// thread's memcpy into pinned memory, not PCIe, bounded the host-buffer update
// of large batches (synth1m_256: 56.7 -> 27.9 ms; H2D floor 25.1 ms), and 16
// parts beat 3 there (cifar10_256, 8 threads: 9.37 -> 8.68 ms; floor 7.56 ms;
// gpu_e2e_sweep.sh (r04 tree)). MNIST-64: 4 threads 0.26 ms vs 1 thread 0.39 ms.
int stage_uploads(fleet_ctx* c, const char* const* uploads, size_t col0, size_t width, size_t pitch, int M,
                  size_t tail_bytes, int threads) {
  const size_t total = pitch * (size_t)M;
  int pieces = 3;
  if (total >= (256u << 20)) pieces = (int)std::min<size_t>(16, total / (24u << 20));
  if (const int k = fleet::plan_overrides().stage_pieces) pieces = k;
  if (total < (4u << 20)) pieces = 1;
  pieces = std::min(pieces, M);
  for (int k = 0; k < pieces; ++k) {
    const int r0 = (int)((int64_t)M * k / pieces), r1 = (int)((int64_t)M * (k + 1) / pieces);
    parallel_for(c, r1 - r0, threads, [&](int j) {
      const int i = r0 + j;
      uint8_t* row = c->h_stage + (size_t)i * pitch;
      std::memcpy(row, uploads[i] + col0, width);
      std::memset(row + width, 0, pitch - width);
    });
    const size_t off = (size_t)r0 * pitch;
    const size_t bytes = (size_t)(r1 - r0) * pitch + (r1 == M ? tail_bytes : 0);
    HIP_TRY(c, hipMemcpyAsync(c->d_a + off, c->h_stage + off, bytes, hipMemcpyHostToDevice, c->stream));
  }
  return FLEET_OK;
}

// network::flatGrad's header walk (network.h:1206-1223) over the last upload,
// on the host from the caller's buffer -- the same walk as k_layout_parse:
// words = {status (0 ok, 1 malformed), count, walk end, 0, positions...}.
// The caller's buffer is exactly `len` bytes (a JVM array or Python bytes, no
// padding): the group holding value p is copied into a zero-padded local, so a
// short or truncated upload never reads past the end (bytes at or beyond len
// decode as the device path's zero padding).
int32_t host_code_at(const char* text, size_t len, int64_t p, bool* bad) {
  static constexpr auto tab = [] {
    struct T {
      uint8_t v[256];
    } t{};
    for (int i = 0; i < 256; ++i) t.v[i] = fleet::b64_from_value(i);
    return t;
  }();
  uint8_t g[16] = {0};
  const size_t g0 = 16 * (size_t)(p / 3);
  if (g0 < len) std::memcpy(g, text + g0, std::min<size_t>(16, len - g0));
  const int e = (int)(p % 3);
  const uint32_t carry[3] = {0x003fu, 0x07e0u, 0xfc00u};  // chars carrying bytes 4e..4e+3
  uint8_t bytes[12];
  for (int q = 0; q < 4; ++q) {
    uint32_t w = 0;
    for (int i = 0; i < 4; ++i) {
      const uint8_t v = tab.v[g[4 * q + i]];
      if (v == 0xff && ((carry[e] >> (4 * q + i)) & 1u)) *bad = true;
      w = (w << 6) | (v & 63u);
    }
    bytes[3 * q] = (uint8_t)(w >> 16);
    bytes[3 * q + 1] = (uint8_t)(w >> 8);
    bytes[3 * q + 2] = (uint8_t)w;
  }
  uint32_t u = 0;
  for (int i = 3; i >= 0; --i) u = (u << 8) | bytes[4 * e + i];
  return (int32_t)u;
}
void host_layout_parse(const char* up, size_t len, int64_t n, int cap, int32_t* out) {
  int64_t idx = 0;
  int nh = 0;
  bool bad = false;
  int status = 0;
  for (int part = 0; part < 2 && !status; ++part) {
    if (idx >= n || nh >= cap) {
      status = 1;
      break;
    }
    out[4 + nh++] = (int32_t)idx;
    const int cnt = fleet::cvtt(fleet::dec(host_code_at(up, len, idx++, &bad)));
    for (int i = 0; i < cnt; ++i) {
      if (idx >= n || nh >= cap) {
        status = 1;
        break;
      }
      out[4 + nh++] = (int32_t)idx;
      const int size = fleet::cvtt(fleet::dec(host_code_at(up, len, idx++, &bad)));
      if (size < 0 || idx + size > n) {
        status = 1;
        break;
      }
      idx += size;
    }
  }
  if (bad) status = 1;
  out[0] = status;
  out[1] = nh;
  out[2] = (int32_t)idx;
  out[3] = 0;
}

// fleet_update when the host walk of the last upload's header fails: the
// device flow (parse kernel, update, error flags), so the error reported is
// the same as a full device run's (Base64 errors anywhere take precedence).
int update_host_fallback(fleet_ctx* c, const char* const* uploads, size_t len, int M, const double* dampen,
                         char* merged, float* merged_f32) {
  const size_t n = fleet_b64_count(len), groups = groups_of(n), pitch = round16(len), total = pitch * (size_t)M;
  int rc;
  if ((rc = grow_dev(c, &c->d_dampen, &c->d_dampen_cap, (size_t)M))) return rc;
  if ((rc = grow_dev(c, &c->d_out, &c->d_out_cap, 16 * groups + 16))) return rc;
  if (merged_f32 && (rc = grow_dev(c, &c->d_f32, &c->d_f32_cap, 3 * groups + 3))) return rc;
  if ((rc = stage_uploads(c, uploads, 0, len, pitch, M, 0, stage_threads(total)))) return rc;
  std::memcpy(c->h_stage + total, dampen, sizeof(double) * (size_t)M);
  HIP_TRY(c, hipMemcpyAsync(c->d_dampen, c->h_stage + total, sizeof(double) * (size_t)M, hipMemcpyHostToDevice,
                            c->stream));
  HIP_TRY(c, fleet::launch_layout_parse(c->d_a + (size_t)(M - 1) * pitch, (int64_t)n, FLEET_MAX_HEADERS, c->d_hdr,
                                        c->stream));
  HIP_TRY(c, fleet::launch_update(c->d_a, pitch, M, c->d_dampen, (double)1 / M, (int64_t)n, 0, (int64_t)groups,
                                  c->d_hdr, c->d_out, merged_f32 ? c->d_f32 : nullptr, c->d_err, c->stream));
  HIP_TRY(c, hipMemcpyAsync(merged, c->d_out, len, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->h_hdr, c->d_hdr, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  if ((rc = read_err(c, c->stream))) return rc;
  if (c->h_hdr[0] != 0)
    return fail(c, FLEET_ERR_LAYOUT, "last upload's header does not describe a gradient layout");
  return FLEET_OK;  // not reached for a failed host walk (the device walk is the same)
}

}  // namespace

extern "C" {

const char* fleet_version(void) { return FLEET_VERSION; }

size_t fleet_b64_len(size_t n_values) { return 4 * ((4 * n_values + 2) / 3); }
size_t fleet_b64_count(size_t len) { return 3 * len / 16; }

int fleet_create(int device, fleet_ctx** out) {
  if (!out) return FLEET_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return FLEET_ERR_HIP;
  if (device < 0 || device >= n) return FLEET_ERR_ARG;
  fleet_ctx* c = new fleet_ctx();
  c->device = device;
  int rc = FLEET_OK;
  auto bail = [&](int code) {
    fleet_destroy(c);
    return code;
  };
  DeviceGuard dg(device);
  if (!dg.ok) return bail(FLEET_ERR_HIP);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bail(FLEET_ERR_HIP);
  if (hipMalloc((void**)&c->d_hdr, kHdrWords * sizeof(int32_t)) != hipSuccess) return bail(FLEET_ERR_NOMEM);
  if (hipMalloc((void**)&c->d_err, 64) != hipSuccess) return bail(FLEET_ERR_NOMEM);
  if (hipMemset(c->d_err, 0, 64) != hipSuccess) return bail(FLEET_ERR_HIP);
  if (hipMalloc((void**)&c->d_dev_hdr, kHdrWords * sizeof(int32_t)) != hipSuccess) return bail(FLEET_ERR_NOMEM);
  if (hipMalloc((void**)&c->d_dev_err, 64) != hipSuccess) return bail(FLEET_ERR_NOMEM);
  if (hipMemset(c->d_dev_err, 0, 64) != hipSuccess) return bail(FLEET_ERR_HIP);
  if (hipHostMalloc((void**)&c->h_hdr, kHdrWords * sizeof(int32_t), hipHostMallocDefault) != hipSuccess)
    return bail(FLEET_ERR_NOMEM);
  if (hipHostMalloc((void**)&c->h_err, 64, hipHostMallocDefault) != hipSuccess) return bail(FLEET_ERR_NOMEM);
  (void)rc;
  *out = c;
  return FLEET_OK;
}

void fleet_destroy(fleet_ctx* c) {
  if (!c) return;
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (void* p : {(void*)c->d_a, (void*)c->d_b, (void*)c->d_out, (void*)c->d_f32, (void*)c->d_dampen,
                  (void*)c->d_hdr, (void*)c->d_err, (void*)c->d_partials, (void*)c->d_dev_dampen,
                  (void*)c->d_dev_hdr, (void*)c->d_dev_err, (void*)c->d_kflags})
    if (p) (void)hipFree(p);
  for (void* p : c->retired) (void)hipFree(p);
  for (void* p : {(void*)c->h_stage, (void*)c->h_hdr, (void*)c->h_err})
    if (p) (void)hipHostFree(p);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* fleet_last_error(const fleet_ctx* c) { return c ? c->err.c_str() : "no context"; }

namespace {
std::atomic<int> g_last_ingress{FLEET_INGRESS_NONE};  // the process's most recent one
}

#ifdef FLEET_TRACE
// dev builds only (-DFLEET_TRACE): where the tile kernels write their phase trace
extern "C" __attribute__((visibility("default"))) int fleet_dev_trace(void* d_buf) {
  return fleet::set_trace_buffer(d_buf) == hipSuccess ? FLEET_OK : FLEET_ERR_HIP;
}
#endif

int fleet_last_ingress(fleet_ctx* c) {
  if (!c) return g_last_ingress.load();
  std::lock_guard<std::mutex> lk(c->mu);
  return c->last_ingress;
}

int fleet_sync(fleet_ctx* c, void* stream) {
  if (!c) return FLEET_ERR_ARG;
  HIP_TRY(c, hipStreamSynchronize(pick(c, stream)));
  return FLEET_OK;
}

int fleet_check(fleet_ctx* c, void* stream) {
  if (!c) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  return read_err(c, pick(c, stream), c->d_dev_err);
}

int fleet_layout_from_sizes(const int32_t* w_sizes, int n_w, const int32_t* b_sizes, int n_b, int32_t* header_pos,
                            int cap, int* n_headers, size_t* n_up) {
  if (n_w < 0 || n_b < 0 || (n_w && !w_sizes) || (n_b && !b_sizes)) return FLEET_ERR_ARG;
  size_t idx = 0;
  int nh = 0;
  auto put = [&](size_t p) {
    if (nh < cap && header_pos) header_pos[nh] = (int32_t)p;
    ++nh;
  };
  put(idx++);
  for (int i = 0; i < n_w; ++i) {
    if (w_sizes[i] < 0) return FLEET_ERR_ARG;
    put(idx++);
    idx += (size_t)w_sizes[i];
  }
  put(idx++);
  for (int i = 0; i < n_b; ++i) {
    if (b_sizes[i] < 0) return FLEET_ERR_ARG;
    put(idx++);
    idx += (size_t)b_sizes[i];
  }
  if (n_headers) *n_headers = nh;
  if (n_up) *n_up = idx;
  return nh <= cap ? FLEET_OK : FLEET_ERR_CAPACITY;
}

int fleet_layout_parse(fleet_ctx* c, const char* upload, size_t len, int32_t* header_pos, int cap, int* n_headers,
                       size_t* n_up) {
  if (!c || (!upload && len)) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  int rc = check_text_len(c, len);
  if (rc) return rc;
  size_t n = fleet_b64_count(len);
  if ((rc = stage_text(c, upload, len, &c->d_a, &c->d_a_cap))) return rc;
  int nh = 0;
  size_t walk_end = n;
  if ((rc = parse_layout(c, c->d_a, n, &nh, &walk_end))) return rc;
  if (n_headers) *n_headers = nh;
  if (n_up) *n_up = walk_end;
  if (header_pos) std::memcpy(header_pos, c->h_hdr + 4, sizeof(int32_t) * std::min(nh, cap));
  return nh <= cap ? FLEET_OK : FLEET_ERR_CAPACITY;
}

// ----------------------------------------------------------------- codec

int fleet_encode_f32(fleet_ctx* c, const float* values, size_t n, char* out, size_t cap, size_t* out_len) {
  if (!c || (!values && n)) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  int rc;
  if ((rc = grow_dev(c, &c->d_f32, &c->d_f32_cap, n + 3))) return rc;
  if ((rc = grow_dev(c, &c->d_out, &c->d_out_cap, 16 * groups_of(n) + 16))) return rc;
  if (n) HIP_TRY(c, hipMemcpyAsync(c->d_f32, values, n * sizeof(float), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, fleet::launch_encode_f32(c->d_f32, (int64_t)n, 0, 1, c->d_out, 0, c->stream));
  return finish_text(c, fleet_b64_len(n), out, cap, out_len);
}

int fleet_encode_i32(fleet_ctx* c, const int32_t* codes, size_t n, char* out, size_t cap, size_t* out_len) {
  if (!c || (!codes && n)) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  int rc;
  if ((rc = grow_dev(c, &c->d_a, &c->d_a_cap, 4 * n + 16))) return rc;
  if ((rc = grow_dev(c, &c->d_out, &c->d_out_cap, 16 * groups_of(n) + 16))) return rc;
  if (n) HIP_TRY(c, hipMemcpyAsync(c->d_a, codes, n * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, fleet::launch_encode_i32((const int32_t*)c->d_a, (int64_t)n, c->d_out, c->stream));
  return finish_text(c, fleet_b64_len(n), out, cap, out_len);
}

static int decode_common(fleet_ctx* c, const char* text, size_t len, void* out, size_t cap, size_t* n_out,
                         int as_codes) {
  if (!c || (!text && len)) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  int rc = check_text_len(c, len);
  if (rc) return rc;
  size_t n = fleet_b64_count(len);
  if (n_out) *n_out = n;
  if (cap < n) return fail(c, FLEET_ERR_CAPACITY, "output capacity %zu < %zu values", cap, n);
  if ((rc = stage_text(c, text, len, &c->d_a, &c->d_a_cap))) return rc;
  if ((rc = grow_dev(c, &c->d_f32, &c->d_f32_cap, n + 3))) return rc;
  HIP_TRY(c, fleet::launch_decode(c->d_a, (int64_t)n, 0, 1, c->d_f32, 0, as_codes, c->d_err, c->stream));
  if (n) HIP_TRY(c, hipMemcpyAsync(out, c->d_f32, n * 4, hipMemcpyDeviceToHost, c->stream));
  return read_err(c, c->stream);
}

int fleet_decode_f32(fleet_ctx* c, const char* text, size_t len, float* out, size_t cap, size_t* n_out) {
  return decode_common(c, text, len, out, cap, n_out, 0);
}
int fleet_decode_i32(fleet_ctx* c, const char* text, size_t len, int32_t* out, size_t cap, size_t* n_out) {
  return decode_common(c, text, len, out, cap, n_out, 1);
}

// ------------------------------------------------------------- JNI ops

int fleet_flat_gradient(fleet_ctx* c, const char* g, size_t len, char* out, size_t cap, size_t* out_len) {
  if (!c || (!g && len)) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  int rc = check_text_len(c, len);
  if (rc) return rc;
  size_t n = fleet_b64_count(len);
  if ((rc = stage_text(c, g, len, &c->d_a, &c->d_a_cap))) return rc;
  int nh = 0;
  size_t walk_end = 0;
  if ((rc = parse_layout(c, c->d_a, n, &nh, &walk_end))) return rc;
  // network::flatGrad stops after the last bias block: values past the walk are dropped
  const size_t n_flat = walk_end - (size_t)nh;
  if ((rc = grow_dev(c, &c->d_out, &c->d_out_cap, 16 * groups_of(n_flat) + 16))) return rc;
  HIP_TRY(c, fleet::launch_flat(c->d_a, c->d_hdr + 4, nh, (int64_t)n_flat, c->d_out, c->d_err, c->stream));
  return finish_text(c, fleet_b64_len(n_flat), out, cap, out_len);
}

int fleet_merge_flat_gradient(fleet_ctx* c, const char* g, size_t glen, const char* flat, size_t flen, char* out,
                              size_t cap, size_t* out_len) {
  if (!c || (!g && glen) || (!flat && flen)) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  int rc = check_text_len(c, glen);
  if (rc || (rc = check_text_len(c, flen))) return rc;
  size_t n = fleet_b64_count(glen), nf = fleet_b64_count(flen);
  if ((rc = stage_text(c, g, glen, &c->d_a, &c->d_a_cap))) return rc;
  if ((rc = stage_text(c, flat, flen, &c->d_b, &c->d_b_cap))) return rc;
  int nh = 0;
  size_t walk_end = 0;
  if ((rc = parse_layout(c, c->d_a, n, &nh, &walk_end))) return rc;
  if (nf < walk_end - (size_t)nh)
    return fail(c, FLEET_ERR_ARG, "flat gradient has %zu values, layout needs %zu", nf, walk_end - (size_t)nh);
  if ((rc = grow_dev(c, &c->d_out, &c->d_out_cap, 16 * groups_of(n) + 16))) return rc;
  HIP_TRY(c, fleet::launch_merge(c->d_a, c->d_b, c->d_hdr + 4, nh, (int64_t)walk_end, (int64_t)n, c->d_out,
                                 c->d_err, c->stream));
  return finish_text(c, glen, out, cap, out_len);
}

static int elementwise(fleet_ctx* c, const char* a, size_t alen, const char* b, size_t blen, int op, double s,
                       char* out, size_t cap, size_t* out_len) {
  if (!c || (!a && alen) || (op && !b && blen)) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  int rc = check_text_len(c, alen);
  if (rc) return rc;
  size_t n = fleet_b64_count(alen);
  if ((rc = stage_text(c, a, alen, &c->d_a, &c->d_a_cap))) return rc;
  if (op) {
    if ((rc = check_text_len(c, blen))) return rc;
    if (fleet_b64_count(blen) < n) return fail(c, FLEET_ERR_ARG, "second operand shorter than the first");
    if ((rc = stage_text(c, b, blen, &c->d_b, &c->d_b_cap))) return rc;
  }
  if ((rc = grow_dev(c, &c->d_out, &c->d_out_cap, 16 * groups_of(n) + 16))) return rc;
  HIP_TRY(c, fleet::launch_elementwise(c->d_a, op ? c->d_b : c->d_a, op, s, (int64_t)n, c->d_out, c->d_err,
                                       c->stream));
  return finish_text(c, fleet_b64_len(n), out, cap, out_len);
}

int fleet_scalar_mul(fleet_ctx* c, const char* v, size_t len, double a, char* out, size_t cap, size_t* out_len) {
  return elementwise(c, v, len, nullptr, 0, 0, a, out, cap, out_len);
}
int fleet_add(fleet_ctx* c, const char* a, size_t alen, const char* b, size_t blen, char* out, size_t cap,
              size_t* out_len) {
  return elementwise(c, a, alen, b, blen, 1, 0.0, out, cap, out_len);
}
int fleet_subtract(fleet_ctx* c, const char* a, size_t alen, const char* b, size_t blen, char* out, size_t cap,
                   size_t* out_len) {
  return elementwise(c, a, alen, b, blen, 2, 0.0, out, cap, out_len);
}

int fleet_norm(fleet_ctx* c, const char* v, size_t len, double* out) {
  if (!c || (!v && len) || !out) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  int rc = check_text_len(c, len);
  if (rc) return rc;
  size_t n = fleet_b64_count(len);
  if ((rc = stage_text(c, v, len, &c->d_a, &c->d_a_cap))) return rc;
  size_t blocks = (groups_of(n) + 255) / 256 + 1;
  if ((rc = grow_dev(c, &c->d_partials, &c->d_partials_cap, blocks))) return rc;
  int nb = 0;
  HIP_TRY(c, fleet::launch_norm_partials(c->d_a, (int64_t)n, c->d_partials, &nb, c->d_err, c->stream));
  std::vector<double> part((size_t)nb);
  if (nb) HIP_TRY(c, hipMemcpyAsync(part.data(), c->d_partials, nb * sizeof(double), hipMemcpyDeviceToHost,
                                    c->stream));
  if ((rc = read_err(c, c->stream))) return rc;
  double s = 0;
  for (double p : part) s += p;  // block partials in index order
  *out = __builtin_sqrt(s);
  return FLEET_OK;
}

// ------------------------------------------------------------ fused update

namespace {

// Validation shared by the host-buffer updates; on success *len = the common length.
int check_update_args(fleet_ctx* c, const char* const* uploads, const size_t* lens, int M, size_t cap,
                      size_t* out_len, size_t* len_out) {
  const size_t len = lens[0];
  int rc = check_text_len(c, len);
  if (rc) return rc;
  for (int i = 0; i < M; ++i) {
    if (!uploads[i] || lens[i] != len)
      return fail(c, FLEET_ERR_ARG, "upload %d has length %zu, expected %zu (one model layout)", i, lens[i], len);
  }
  if (out_len) *out_len = len;
  if (cap < len) return fail(c, FLEET_ERR_CAPACITY, "output capacity %zu < %zu", cap, len);
  *len_out = len;
  return FLEET_OK;
}

// The host-buffer update of the groups [gb, ge) on context c (lock held, device
// set): the column window [16*gb, 16*ge) of every upload is staged into pinned
// memory and sent to HBM, the exact chain runs on it, and its merged slice
// (Base64 bytes [16*gb, min(len, 16*ge)), fp32 values [3*gb, min(n, 3*ge))) is
// written into the caller's outputs -- disjoint ranges for disjoint windows.
// hw = the host walk of the last upload's header (whole-upload coordinates).
//   staging block, mirrored on the device in d_a:
//   [window rows M x wpitch | dampen M doubles | header words | err | merged | fp32]
//   one H2D up to err (inclusive, err = 0), one D2H from err on.
// pinned_rows != NULL: the uploads are rows `row_pitch` apart in page-locked
// memory (fleet_host_register, or allocated pinned): the window goes to HBM in
// one 2D DMA straight from them, with no host copy (only the parameter words
// are staged). Bytes past `len` in the last group of a row may hold anything:
// the kernels ignore the chars that carry no value.
int update_window(fleet_ctx* c, const char* const* uploads, size_t len, int M, const double* dampen,
                  const int32_t* hw, size_t gb, size_t ge, char* merged, float* merged_f32, int threads,
                  const char* pinned_rows = nullptr, size_t row_pitch = 0) {
  const size_t n = fleet_b64_count(len);
  const size_t w = ge - gb;
  if (w == 0) return FLEET_OK;
  const size_t wpitch = 16 * w;
  const size_t col0 = 16 * gb, width = std::min(len, 16 * ge) - col0;
  const size_t total = wpitch * (size_t)M;
  const size_t o_damp = total, o_hdr = round16(o_damp + sizeof(double) * (size_t)M);
  const size_t o_err = round16(o_hdr + sizeof(int32_t) * kHdrWords), o_out = o_err + 16;
  const size_t o_f32 = round16(o_out + wpitch + 16), o_end = o_f32 + sizeof(float) * (3 * w + 3);
  int rc;
  if ((rc = grow_pinned(c, o_end + 64))) return rc;
  if ((rc = grow_dev(c, &c->d_a, &c->d_a_cap, o_end + 64))) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));  // staging buffer reuse
  std::memcpy(c->h_stage + o_hdr, hw, sizeof(int32_t) * kHdrWords);
  std::memcpy(c->h_stage + o_damp, dampen, sizeof(double) * (size_t)M);
  std::memset(c->h_stage + o_err, 0, 16);
  c->last_ingress = pinned_rows ? FLEET_INGRESS_PINNED : FLEET_INGRESS_STAGED;
  g_last_ingress.store(c->last_ingress);
  if (pinned_rows) {
    HIP_TRY(c, hipMemcpy2DAsync(c->d_a, wpitch, pinned_rows + col0, row_pitch, width, (size_t)M,
                                hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->d_a + total, c->h_stage + total, o_err + 16 - total, hipMemcpyHostToDevice,
                              c->stream));
  } else if ((rc = stage_uploads(c, uploads, col0, width, wpitch, M, o_err + 16 - total, threads))) {
    return rc;
  }
  uint8_t* d = c->d_a;
  // window mode: row and output pointers shifted back by the window's start
  HIP_TRY(c, fleet::launch_update(d - col0, wpitch, M, reinterpret_cast<const double*>(d + o_damp), (double)1 / M,
                                  (int64_t)n, (int64_t)gb, (int64_t)ge, reinterpret_cast<const int32_t*>(d + o_hdr),
                                  d + o_out - col0,
                                  merged_f32 ? reinterpret_cast<float*>(d + o_f32) - 3 * gb : nullptr,
                                  reinterpret_cast<int*>(d + o_err), c->stream));
  const size_t v0 = 3 * gb, v1 = std::min(n, 3 * ge);
  const size_t back = (merged_f32 ? o_f32 + sizeof(float) * (v1 - v0) : o_out + width) - o_err;
  HIP_TRY(c, hipMemcpyAsync(c->h_stage + o_err, d + o_err, back, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  const int e = *reinterpret_cast<const int*>(c->h_stage + o_err);
  if (e & 1) return fail(c, FLEET_ERR_BASE64, "input is not Base64::encode output (alphabet/padding)");
  if (e & 2) return fail(c, FLEET_ERR_LAYOUT, "uploads disagree on the gradient layout header slots");
  std::memcpy(merged + col0, c->h_stage + o_out, width);
  if (merged_f32) std::memcpy(merged_f32 + v0, c->h_stage + o_f32, sizeof(float) * (v1 - v0));
  return FLEET_OK;
}

}  // namespace

int fleet_update(fleet_ctx* c, const char* const* uploads, const size_t* lens, int M, const double* dampen,
                 char* merged, size_t cap, size_t* out_len, float* merged_f32) {
  if (!c || !uploads || !lens || !dampen || !merged || M <= 0) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  size_t len = 0;
  int rc = check_update_args(c, uploads, lens, M, cap, out_len, &len);
  if (rc) return rc;
  const size_t n = fleet_b64_count(len);
  // layout of the last picked upload (mergeFlatGradient keeps its header), walked on the host
  std::vector<int32_t> hw(kHdrWords);
  host_layout_parse(uploads[M - 1], len, (int64_t)n, FLEET_MAX_HEADERS, hw.data());
  if (hw[0] != 0) return update_host_fallback(c, uploads, len, M, dampen, merged, merged_f32);
  return update_window(c, uploads, len, M, dampen, hw.data(), 0, groups_of(n), merged, merged_f32,
                       stage_threads(round16(len) * (size_t)M));
}

namespace {

// Ranges page-locked by fleet_host_register (process-wide: every context's
// device DMAs from them). The copy-free row path requires the WHOLE row range
// to lie inside ONE recorded registration. A record cannot tell whether its
// memory was freed and reused since (the caller's contract, fleet_codec.h:
// unregister before freeing); it only stops rows that straddle two ranges.
std::mutex g_reg_mu;
std::vector<std::pair<uintptr_t, size_t>> g_registered;  // (base, bytes)

bool in_one_registration(const void* p, size_t bytes) {
  const uintptr_t a = (uintptr_t)p;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  for (const auto& r : g_registered)
    if (a >= r.first && bytes <= r.second && a - r.first <= r.second - bytes) return true;
  return false;
}

int update_multi_impl(fleet_ctx* const* ctxs, int n_ctx, const char* const* uploads, const size_t* lens, int M,
                      const double* dampen, char* merged, size_t cap, size_t* out_len, float* merged_f32,
                      const char* pinned_rows, size_t row_pitch) {
  for (int k = 0; k < n_ctx; ++k) {
    if (!ctxs[k]) return FLEET_ERR_ARG;
    for (int j = 0; j < k; ++j)
      if (ctxs[j] == ctxs[k]) return fail(ctxs[0], FLEET_ERR_ARG, "context %d is passed twice", k);
  }
  fleet_ctx* c0 = ctxs[0];
  size_t len = 0;
  int rc;
  {
    std::lock_guard<std::mutex> lk(c0->mu);
    if ((rc = check_update_args(c0, uploads, lens, M, cap, out_len, &len))) return rc;
  }
  const size_t n = fleet_b64_count(len), groups = groups_of(n);
  std::vector<int32_t> hw(kHdrWords);
  host_layout_parse(uploads[M - 1], len, (int64_t)n, FLEET_MAX_HEADERS, hw.data());
  // a malformed header: the single-device flow reports the same error as a full device run
  if (hw[0] != 0) {
    std::lock_guard<std::mutex> lk(c0->mu);
    DEVICE_SCOPE(c0);
    return update_host_fallback(c0, uploads, len, M, dampen, merged, merged_f32);
  }
  const int threads = std::max(1, stage_threads(round16(len) * (size_t)M) / n_ctx);
  std::vector<int> rcs((size_t)n_ctx, FLEET_OK);
  auto run = [&](int k) {
    // balanced contiguous split of the groups (fleet_amd.shard.group_range)
    const size_t base = groups / (size_t)n_ctx, rem = groups % (size_t)n_ctx;
    const size_t gb = (size_t)k * base + std::min((size_t)k, rem), ge = gb + base + ((size_t)k < rem ? 1 : 0);
    fleet_ctx* c = ctxs[k];
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) {
      rcs[(size_t)k] = fail(c, FLEET_ERR_HIP, "hipSetDevice(%d) failed", c->device);
      return;
    }
    rcs[(size_t)k] = update_window(c, uploads, len, M, dampen, hw.data(), gb, ge, merged, merged_f32,
                                   n_ctx == 1 ? stage_threads(round16(len) * (size_t)M) : threads, pinned_rows,
                                   row_pitch);
  };
  if (n_ctx == 1) {
    run(0);
  } else {
    std::vector<std::thread> ts;
    ts.reserve((size_t)n_ctx);
    for (int k = 0; k < n_ctx; ++k) ts.emplace_back(run, k);
    for (auto& t : ts) t.join();
  }
  // the first failing shard's error (Base64 errors first, as one device reports them)
  int first = -1;
  for (int k = 0; k < n_ctx; ++k)
    if (rcs[(size_t)k] != FLEET_OK &&
        (first < 0 || (rcs[(size_t)k] == FLEET_ERR_BASE64 && rcs[(size_t)first] != FLEET_ERR_BASE64)))
      first = k;
  if (first < 0) return FLEET_OK;
  if (first != 0) {
    std::lock_guard<std::mutex> lk(c0->mu);
    c0->err = ctxs[first]->err;
  }
  return rcs[(size_t)first];
}

int update_rows_impl(fleet_ctx* const* ctxs, int n_ctx, const char* rows, size_t row_pitch, size_t len, int M,
                     const double* dampen, char* merged, size_t cap, size_t* out_len, float* merged_f32) {
  if (row_pitch < len) return fail(ctxs[0], FLEET_ERR_ARG, "row pitch %zu < upload length %zu", row_pitch, len);
  std::vector<const char*> ptrs((size_t)M);
  std::vector<size_t> lens((size_t)M, len);
  for (int i = 0; i < M; ++i) ptrs[(size_t)i] = rows + (size_t)i * row_pitch;
  const bool pinned = in_one_registration(rows, (size_t)(M - 1) * row_pitch + len);
  return update_multi_impl(ctxs, n_ctx, ptrs.data(), lens.data(), M, dampen, merged, cap, out_len, merged_f32,
                           pinned ? rows : nullptr, row_pitch);
}

}  // namespace

int fleet_update_multi(fleet_ctx* const* ctxs, int n_ctx, const char* const* uploads, const size_t* lens, int M,
                       const double* dampen, char* merged, size_t cap, size_t* out_len, float* merged_f32) {
  if (!ctxs || n_ctx <= 0 || !uploads || !lens || !dampen || !merged || M <= 0) return FLEET_ERR_ARG;
  if (n_ctx == 1) return fleet_update(ctxs[0], uploads, lens, M, dampen, merged, cap, out_len, merged_f32);
  return update_multi_impl(ctxs, n_ctx, uploads, lens, M, dampen, merged, cap, out_len, merged_f32, nullptr, 0);
}

int fleet_update_rows(fleet_ctx* c, const char* rows, size_t row_pitch, size_t len, int M, const double* dampen,
                      char* merged, size_t cap, size_t* out_len, float* merged_f32) {
  if (!c || !rows || !dampen || !merged || M <= 0) return FLEET_ERR_ARG;
  return update_rows_impl(&c, 1, rows, row_pitch, len, M, dampen, merged, cap, out_len, merged_f32);
}

int fleet_update_rows_multi(fleet_ctx* const* ctxs, int n_ctx, const char* rows, size_t row_pitch, size_t len, int M,
                            const double* dampen, char* merged, size_t cap, size_t* out_len, float* merged_f32) {
  if (!ctxs || n_ctx <= 0 || !ctxs[0] || !rows || !dampen || !merged || M <= 0) return FLEET_ERR_ARG;
  return update_rows_impl(ctxs, n_ctx, rows, row_pitch, len, M, dampen, merged, cap, out_len, merged_f32);
}

int fleet_host_register(fleet_ctx* c, void* ptr, size_t bytes) {
  if (!c || !ptr || !bytes) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  const uintptr_t a = (uintptr_t)ptr;
  {
    // a live registration overlapping the new range belongs to memory that was
    // freed and reused (a collected direct buffer): it is released first
    std::lock_guard<std::mutex> rk(g_reg_mu);
    for (size_t i = g_registered.size(); i-- > 0;) {
      const auto r = g_registered[i];
      if (r.first < a + bytes && a < r.first + r.second) {
        (void)hipHostUnregister((void*)r.first);
        (void)hipGetLastError();
        g_registered.erase(g_registered.begin() + (long)i);
      }
    }
  }
  HIP_TRY(c, hipHostRegister(ptr, bytes, hipHostRegisterPortable));
  std::lock_guard<std::mutex> rk(g_reg_mu);
  g_registered.emplace_back(a, bytes);
  return FLEET_OK;
}

int fleet_host_unregister(fleet_ctx* c, void* ptr) {
  if (!c || !ptr) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  {
    std::lock_guard<std::mutex> rk(g_reg_mu);
    for (size_t i = g_registered.size(); i-- > 0;)
      if (g_registered[i].first == (uintptr_t)ptr) g_registered.erase(g_registered.begin() + (long)i);
  }
  HIP_TRY(c, hipHostUnregister(ptr));
  return FLEET_OK;
}

// ---------------------------------------------------------- device-resident

namespace {

// The device-resident update's parameters ({status, count, walk_end, 0, positions}
// and dampen): kept resident in the context's own buffers and re-uploaded (one
// sync) only when they change, so steady-state calls are pure kernel launches.
int dev_params(fleet_ctx* c, hipStream_t s, size_t n, int M, const double* dampen, const int32_t* header_pos,
               int n_headers) {
  std::vector<int32_t> hdr_words((size_t)n_headers + 4);
  hdr_words[0] = 0;
  hdr_words[1] = n_headers;
  hdr_words[2] = (int32_t)n;  // the caller's layout covers the whole upload
  hdr_words[3] = 0;
  if (n_headers) std::memcpy(hdr_words.data() + 4, header_pos, sizeof(int32_t) * (size_t)n_headers);
  if (!c->dev_params_valid || c->dev_hdr != hdr_words || c->dev_dampen.size() != (size_t)M ||
      std::memcmp(c->dev_dampen.data(), dampen, sizeof(double) * (size_t)M) != 0) {
    int rc;
    // new parameters are uploaded synchronously, which a stream under capture
    // cannot do (it would invalidate the capture): the caller makes one eager
    // call with them first (fleet_codec.h, device-resident entry points)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone)
      return fail(c, FLEET_ERR_ARG,
                  "dampen / header positions changed while the stream is being captured: make one eager call "
                  "with them before capturing");
    (void)hipGetLastError();
    HIP_TRY(c, hipStreamSynchronize(s));
    if ((size_t)M > c->d_dev_dampen_cap) {  // grow; the old buffer may sit in a captured graph: retire it
      if (c->d_dev_dampen) c->retired.push_back(c->d_dev_dampen);
      c->d_dev_dampen = nullptr;
      c->d_dev_dampen_cap = 0;
      if ((rc = grow_dev(c, &c->d_dev_dampen, &c->d_dev_dampen_cap, (size_t)M))) return rc;
    }
    HIP_TRY(c, hipMemcpy(c->d_dev_dampen, dampen, sizeof(double) * (size_t)M, hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(c->d_dev_hdr, hdr_words.data(), sizeof(int32_t) * hdr_words.size(), hipMemcpyHostToDevice));
    c->dev_dampen.assign(dampen, dampen + M);
    c->dev_hdr = hdr_words;
    c->dev_params_valid = true;
  }
  return FLEET_OK;
}

int check_device_update(fleet_ctx* c, size_t pitch, size_t len, size_t* group_begin, size_t* group_end) {
  int rc = check_text_len(c, len);
  if (rc) return rc;
  const size_t groups = groups_of(fleet_b64_count(len));
  if (*group_end > groups) *group_end = groups;
  if (*group_begin > *group_end) return FLEET_ERR_ARG;
  // only columns [16*group_begin, 16*group_end) of each row are touched: rows
  // must not overlap there (a full row, or a window of just those columns)
  if (pitch % 16 != 0 || pitch < 16 * (*group_end - *group_begin))
    return fail(c, FLEET_ERR_ARG, "pitch must be a multiple of 16 covering the selected groups");
  return FLEET_OK;
}

}  // namespace

int fleet_update_device(fleet_ctx* c, const void* d_uploads, size_t pitch, size_t len, int M, const double* dampen,
                        const int32_t* header_pos, int n_headers, size_t group_begin, size_t group_end,
                        void* d_merged, void* d_merged_f32, void* stream) {
  if (!c || !d_uploads || !dampen || M <= 0 || !d_merged || n_headers < 0 || n_headers > FLEET_MAX_HEADERS ||
      (n_headers && !header_pos))
    return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  int rc = check_device_update(c, pitch, len, &group_begin, &group_end);
  if (rc) return rc;
  const size_t n = fleet_b64_count(len);
  hipStream_t s = pick(c, stream);
  if ((rc = dev_params(c, s, n, M, dampen, header_pos, n_headers))) return rc;
  HIP_TRY(c, fleet::launch_update((const uint8_t*)d_uploads, pitch, M, c->d_dev_dampen, (double)1 / M, (int64_t)n,
                                  (int64_t)group_begin, (int64_t)group_end, c->d_dev_hdr, (uint8_t*)d_merged,
                                  (float*)d_merged_f32, c->d_dev_err, s));
  return FLEET_OK;
}

int fleet_update_encode_device(fleet_ctx* c, const void* d_uploads, size_t pitch, size_t len, int M,
                               const double* dampen, const int32_t* header_pos, int n_headers, void* d_merged,
                               void* d_merged_f32, const void* d_values, size_t vpitch, void* d_next_uploads,
                               void* stream) {
  if (!c || !d_uploads || !dampen || M <= 0 || !d_merged || !d_values || !d_next_uploads || n_headers < 0 ||
      n_headers > FLEET_MAX_HEADERS || (n_headers && !header_pos))
    return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  size_t gb = 0, ge = SIZE_MAX;
  int rc = check_device_update(c, pitch, len, &gb, &ge);
  if (rc) return rc;
  const size_t n = fleet_b64_count(len);
  if (vpitch < n) return fail(c, FLEET_ERR_ARG, "vpitch %zu < %zu values", vpitch, n);
  // the encode writes rows [0, M) of d_next_uploads while the update reads d_uploads
  const uintptr_t u0 = (uintptr_t)d_uploads, u1 = u0 + pitch * (size_t)M;
  const uintptr_t e0 = (uintptr_t)d_next_uploads, e1 = e0 + pitch * (size_t)M;
  if (u0 < e1 && e0 < u1) return fail(c, FLEET_ERR_ARG, "d_next_uploads overlaps d_uploads");
  hipStream_t s = pick(c, stream);
  if ((rc = dev_params(c, s, n, M, dampen, header_pos, n_headers))) return rc;
  HIP_TRY(c, fleet::launch_update_encode((const uint8_t*)d_uploads, pitch, M, c->d_dev_dampen, (double)1 / M,
                                         (int64_t)n, c->d_dev_hdr, (uint8_t*)d_merged, (float*)d_merged_f32,
                                         c->d_dev_err, (const float*)d_values, vpitch, (uint8_t*)d_next_uploads, s));
  return FLEET_OK;
}

int fleet_update_kardam_device(fleet_ctx* c, const void* d_uploads, size_t pitch, size_t len, int M,
                               const double* dampen, const int32_t* header_pos, int n_headers, double lr,
                               const void* d_prev, const uint8_t* has_prev, void* d_g_out, size_t vpitch,
                               void* d_merged, void* d_merged_f32, double* norm_g, double* norm_diff, void* stream) {
  if (!c || !d_uploads || !dampen || M <= 0 || !d_merged || !norm_g || !norm_diff || n_headers < 0 ||
      n_headers > FLEET_MAX_HEADERS || (n_headers && !header_pos) || (d_prev && !has_prev))
    return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  size_t gb = 0, ge = SIZE_MAX;
  int rc = check_device_update(c, pitch, len, &gb, &ge);
  if (rc) return rc;
  const size_t n = fleet_b64_count(len);
  if ((d_prev || d_g_out) && vpitch < n) return fail(c, FLEET_ERR_ARG, "vpitch %zu < %zu values", vpitch, n);
  hipStream_t s = pick(c, stream);
  if ((rc = dev_params(c, s, n, M, dampen, header_pos, n_headers))) return rc;
  // one snapshot of the launch plan for the sizing call and the launch (a concurrent
  // fleet_set_plan must not give the launch more partial slots than were sized)
  const fleet::PlanOverrides plan = fleet::plan_overrides();
  int nw_sz = 0, parts_sz = 1, flags_sz = 0;  // partial slots, norm parts per client, tile flags (sizing call)
  fleet::KardamOut kd0{lr, nullptr, nullptr, 0, nullptr, nullptr};
  (void)fleet::launch_update_kardam(nullptr, pitch, M, nullptr, 0.0, (int64_t)n, 0, (int64_t)ge, nullptr, nullptr,
                                    nullptr, nullptr, kd0, &nw_sz, nullptr, &parts_sz, &flags_sz, nullptr, 0, plan, s);
  (void)hipGetLastError();
  const size_t n_waves = (size_t)std::max(nw_sz, 1), n_parts = (size_t)std::max(parts_sz, 1);
  // scratch: [partials M x slots x 2 | norms M x parts x 2 | has_prev M]; synchronous call (host outputs)
  const size_t o_norm = sizeof(double) * 2 * (size_t)M * n_waves;
  const size_t o_has = o_norm + sizeof(double) * 2 * (size_t)M * n_parts;
  if ((rc = grow_dev(c, &c->d_b, &c->d_b_cap, o_has + (size_t)M + 64))) return rc;
  HIP_TRY(c, hipStreamSynchronize(s));
  double* d_part = reinterpret_cast<double*>(c->d_b);
  double* d_norm = reinterpret_cast<double*>(c->d_b + o_norm);
  uint8_t* d_has = c->d_b + o_has;
  if (d_prev) HIP_TRY(c, hipMemcpy(d_has, has_prev, (size_t)M, hipMemcpyHostToDevice));
  fleet::KardamOut kd{lr, (const float*)d_prev, d_prev ? d_has : nullptr, vpitch, (float*)d_g_out, d_part};
  if ((size_t)flags_sz > c->d_kflags_cap) {  // new flags start at 0, which no launch's epoch is
    if (c->d_kflags) (void)hipFree(c->d_kflags);
    c->d_kflags = nullptr;
    c->d_kflags_cap = 0;
    HIP_TRY(c, hipMalloc(&c->d_kflags, sizeof(uint32_t) * (size_t)flags_sz));
    HIP_TRY(c, hipMemsetAsync(c->d_kflags, 0, sizeof(uint32_t) * (size_t)flags_sz, s));
    c->d_kflags_cap = (size_t)flags_sz;
    c->kflag_epoch = 0;
  }
  if (++c->kflag_epoch == 0) {  // wrapped: every flag back to 0 before epoch 1 is used again
    if (c->d_kflags_cap) HIP_TRY(c, hipMemsetAsync(c->d_kflags, 0, sizeof(uint32_t) * c->d_kflags_cap, s));
    c->kflag_epoch = 1;
  }
  int nw = 0, np = 1, nf = 0;
  HIP_TRY(c, fleet::launch_update_kardam((const uint8_t*)d_uploads, pitch, M, c->d_dev_dampen, (double)1 / M,
                                         (int64_t)n, 0, (int64_t)ge, c->d_dev_hdr, (uint8_t*)d_merged,
                                         (float*)d_merged_f32, c->d_dev_err, kd, &nw, d_norm, &np, &nf, c->d_kflags,
                                         c->kflag_epoch, plan, s, c->kflag_test_skew));
  if ((size_t)np != n_parts || (size_t)std::max(nw, 1) != n_waves)
    return fail(c, FLEET_ERR_HIP, "Kardam launch plan changed between sizing and launch");
  std::vector<double> norms(2 * (size_t)M * n_parts);
  HIP_TRY(c, hipMemcpyAsync(norms.data(), d_norm, sizeof(double) * norms.size(), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_err, c->d_dev_err, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  // the pipelined form's reduce blocks wait on the tiles' flags with a bound: a flag that
  // never came leaves FLEET_ERRBIT_SYNC, and the norms are not to be trusted. The call is
  // synchronous, so it fails now (the bit is cleared; other sticky bits stay for fleet_check)
  if (*c->h_err & FLEET_ERRBIT_SYNC) {
    *c->h_err &= ~FLEET_ERRBIT_SYNC;
    HIP_TRY(c, hipMemcpyAsync(c->d_dev_err, c->h_err, sizeof(int), hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    return fail(c, FLEET_ERR_HIP, "Kardam reduce blocks timed out waiting for the tiles' flags");
  }
  for (int i = 0; i < M; ++i) {
    double a = 0.0, b = 0.0;  // the client's chunk sums, in order
    for (size_t k = 0; k < n_parts; ++k) {
      a += norms[2 * ((size_t)i * n_parts + k)];
      b += norms[2 * ((size_t)i * n_parts + k) + 1];
    }
    norm_g[i] = std::sqrt(a);
    norm_diff[i] = (d_prev && has_prev[i]) ? std::sqrt(b) : std::nan("");
  }
  return FLEET_OK;
}

int fleet_test_kardam_skew(fleet_ctx* c, unsigned skew) {
  if (!c) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  c->kflag_test_skew = skew;
  return FLEET_OK;
}

int fleet_encode_device(fleet_ctx* c, const void* d_values, size_t n, size_t vpitch, int M, void* d_out,
                        size_t pitch, void* stream) {
  if (!c || !d_values || !d_out || M <= 0) return FLEET_ERR_ARG;
  if (pitch % 16 != 0 || pitch < 16 * groups_of(n)) return fail(c, FLEET_ERR_ARG, "bad pitch");
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  HIP_TRY(c, fleet::launch_encode_f32((const float*)d_values, (int64_t)n, vpitch, M, (uint8_t*)d_out, pitch,
                                      pick(c, stream)));
  return FLEET_OK;
}

int fleet_decode_device(fleet_ctx* c, const void* d_text, size_t len, size_t pitch, int M, void* d_values,
                        size_t vpitch, void* stream) {
  if (!c || !d_text || !d_values || M <= 0) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  int rc = check_text_len(c, len);
  if (rc) return rc;
  HIP_TRY(c, fleet::launch_decode((const uint8_t*)d_text, (int64_t)fleet_b64_count(len), pitch, M, d_values,
                                  vpitch, 0, c->d_dev_err, pick(c, stream)));
  return FLEET_OK;
}

int fleet_synth_device(fleet_ctx* c, uint64_t seed, int M, int client0, const int32_t* header_pos,
                       const float* header_val, int n_headers, size_t n_up, void* d_values, size_t vpitch,
                       void* stream) {
  return fleet_synth_window_device(c, seed, M, client0, 0, header_pos, header_val, n_headers, n_up, d_values, vpitch,
                                   stream);
}

int fleet_synth_window_device(fleet_ctx* c, uint64_t seed, int M, int client0, size_t elem0,
                              const int32_t* header_pos, const float* header_val, int n_headers, size_t n_up,
                              void* d_values, size_t vpitch, void* stream) {
  if (!c || !d_values || M <= 0 || n_headers < 0 || n_headers > FLEET_MAX_HEADERS || vpitch < n_up)
    return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  hipStream_t s = pick(c, stream);
  int32_t* d_pos = nullptr;
  float* d_val = nullptr;
  if (n_headers) {
    HIP_TRY(c, hipMalloc((void**)&d_pos, sizeof(int32_t) * (size_t)n_headers));
    HIP_TRY(c, hipMalloc((void**)&d_val, sizeof(float) * (size_t)n_headers));
    HIP_TRY(c, hipMemcpy(d_pos, header_pos, sizeof(int32_t) * (size_t)n_headers, hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(d_val, header_val, sizeof(float) * (size_t)n_headers, hipMemcpyHostToDevice));
  }
  HIP_TRY(c, fleet::launch_synth(seed, client0, (int64_t)elem0, M, (int64_t)n_up, (float*)d_values, vpitch, d_pos,
                                 d_val, n_headers, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  if (d_pos) (void)hipFree(d_pos);
  if (d_val) (void)hipFree(d_val);
  return FLEET_OK;
}

// ------------------------------------------------- mode-1 model codec

namespace {

static int model_total(fleet_ctx* c, const int32_t* dims, int n_mats, size_t* n) {
  if (n_mats < 0 || (n_mats && !dims)) return fail(c, FLEET_ERR_ARG, "bad dims");
  size_t t = 0;
  for (int j = 0; j < n_mats; ++j) {
    if (dims[3 * j] < 0 || dims[3 * j + 1] < 0 || dims[3 * j + 2] < 0) return fail(c, FLEET_ERR_ARG, "negative dim");
    t += (size_t)dims[3 * j] * dims[3 * j + 1] * dims[3 * j + 2];
  }
  if (t > (size_t)INT32_MAX) return fail(c, FLEET_ERR_ARG, "model too large for int32 indices");
  *n = t;
  return FLEET_OK;
}

struct DevMem {
  void* p = nullptr;
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
};

// quantize + dictionary on the device; leaves d_index and the dictionary on the host
static int model_run(fleet_ctx* c, const float* weights, const int32_t* dims, int n_mats, size_t n, float* quantized,
              std::vector<float>* dict_host, int32_t* U, DevMem* d_index_keep) {
  DevMem dw, dq, dd;
  if (n) {
    HIP_TRY(c, hipMalloc(&dw.p, n * sizeof(float)));
    HIP_TRY(c, hipMalloc(&dq.p, n * sizeof(float)));
    HIP_TRY(c, hipMalloc(&dd.p, n * sizeof(float)));
    HIP_TRY(c, hipMalloc(&d_index_keep->p, n * sizeof(int32_t)));
    HIP_TRY(c, hipMemcpyAsync(dw.p, weights, n * sizeof(float), hipMemcpyHostToDevice, c->stream));
  }
  HIP_TRY(c, fleet::model_quantize_index((const float*)dw.p, dims, n_mats, (float*)dq.p, (float*)dd.p,
                                         (int32_t*)d_index_keep->p, U, c->stream));
  if (quantized && n) HIP_TRY(c, hipMemcpyAsync(quantized, dq.p, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  dict_host->resize((size_t)*U);
  if (*U) HIP_TRY(c, hipMemcpyAsync(dict_host->data(), dd.p, (size_t)*U * sizeof(float), hipMemcpyDeviceToHost,
                                    c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FLEET_OK;
}

}  // namespace

int fleet_model_quantize_index(fleet_ctx* c, const float* weights, const int32_t* dims, int n_mats,
                               float* quantized, float* dict, int* n_dict, int32_t* index) {
  if (!c) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  size_t n = 0;
  int rc = model_total(c, dims, n_mats, &n);
  if (rc) return rc;
  if (n && !weights) return FLEET_ERR_ARG;
  std::vector<float> dh;
  int32_t U = 0;
  DevMem di;
  if ((rc = model_run(c, weights, dims, n_mats, n, quantized, &dh, &U, &di))) return rc;
  if (dict && U) std::memcpy(dict, dh.data(), sizeof(float) * (size_t)U);
  if (n_dict) *n_dict = U;
  if (index && n) {
    HIP_TRY(c, hipMemcpy(index, di.p, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  }
  return FLEET_OK;
}

int fleet_model_weights_text(fleet_ctx* c, const float* weights, const int32_t* dims, int n_mats, char* out,
                             size_t cap, size_t* out_len) {
  if (!c) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  size_t n = 0;
  int rc = model_total(c, dims, n_mats, &n);
  if (rc) return rc;
  if (n && !weights) return FLEET_ERR_ARG;
  std::vector<float> dh;
  int32_t U = 0;
  DevMem di;
  if ((rc = model_run(c, weights, dims, n_mats, n, nullptr, &dh, &U, &di))) return rc;
  // header and dictionary lines: `ostream << int` / `ostream << float` (precision 6 == %g),
  // U lines of host formatting; the n index tokens are formatted on the device
  std::string head;
  char buf[64];
  snprintf(buf, sizeof buf, "%zu\n%d\n", n, U);
  head += buf;
  for (int32_t k = 0; k < U; ++k) {
    snprintf(buf, sizeof buf, "%d\n%g\n", k, (double)dh[(size_t)k]);
    head += buf;
  }
  std::vector<char> body;
  HIP_TRY(c, fleet::model_index_text((const int32_t*)di.p, dims, n_mats, &body, c->stream));
  const size_t total = head.size() + body.size();
  if (out_len) *out_len = total;
  if (cap < total) return fail(c, FLEET_ERR_CAPACITY, "output capacity %zu < %zu", cap, total);
  std::memcpy(out, head.data(), head.size());
  if (!body.empty()) std::memcpy(out + head.size(), body.data(), body.size());
  return FLEET_OK;
}

int fleet_model_read_weights(fleet_ctx* c, const char* text, size_t len, const int32_t* dims, int n_mats,
                             float* weights_out) {
  if (!c || (!text && len)) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  size_t n = 0;
  int rc = model_total(c, dims, n_mats, &n);
  if (rc) return rc;
  if (n && !weights_out) return FLEET_ERR_ARG;
  // header: loop_counter and U lines (getcleanline + atoi), then U pairs read
  // with `>>` (int, float = strtof); the std::map keeps the first value of a key
  std::string t(text, len);
  const char* p = t.c_str();
  char* e = nullptr;
  (void)strtol(p, &e, 10);
  if (e == p) return fail(c, FLEET_ERR_ARG, "weights section: no loop counter");
  p = e;
  const long U = strtol(p, &e, 10);
  if (e == p || U < 0) return fail(c, FLEET_ERR_ARG, "weights section: no dictionary size");
  p = e;
  std::vector<std::pair<int32_t, float>> kv;
  kv.reserve((size_t)U);
  for (long k = 0; k < U; ++k) {
    const long key = strtol(p, &e, 10);
    if (e == p) return fail(c, FLEET_ERR_ARG, "weights section: bad dictionary index %ld", k);
    p = e;
    const float v = strtof(p, &e);
    if (e == p) return fail(c, FLEET_ERR_ARG, "weights section: bad dictionary value %ld", k);
    p = e;
    kv.emplace_back((int32_t)key, v);
  }
  std::stable_sort(kv.begin(), kv.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<int32_t> keys;
  std::vector<float> vals;
  for (size_t k = 0; k < kv.size(); ++k)
    if (k == 0 || kv[k].first != kv[k - 1].first) keys.push_back(kv[k].first), vals.push_back(kv[k].second);
  const size_t body = (size_t)(p - t.c_str());
  const size_t blen = len - body;
  DevMem dt, dk, dv, dw;
  if (blen) HIP_TRY(c, hipMalloc(&dt.p, blen));
  HIP_TRY(c, hipMalloc(&dk.p, sizeof(int32_t) * (keys.size() + 1)));
  HIP_TRY(c, hipMalloc(&dv.p, sizeof(float) * (vals.size() + 1)));
  if (n) HIP_TRY(c, hipMalloc(&dw.p, sizeof(float) * n));
  if (blen) HIP_TRY(c, hipMemcpyAsync(dt.p, text + body, blen, hipMemcpyHostToDevice, c->stream));
  if (!keys.empty()) {
    HIP_TRY(c, hipMemcpyAsync(dk.p, keys.data(), sizeof(int32_t) * keys.size(), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(dv.p, vals.data(), sizeof(float) * vals.size(), hipMemcpyHostToDevice, c->stream));
  }
  int status = 0;
  HIP_TRY(c, fleet::model_read_index((const uint8_t*)dt.p, (int64_t)blen, (int64_t)n, (const int32_t*)dk.p,
                                     (const float*)dv.p, (int32_t)keys.size(), (float*)dw.p, &status, c->stream));
  if (status == 1) return fail(c, FLEET_ERR_ARG, "weights section: malformed index token");
  if (status == 2) return fail(c, FLEET_ERR_LAYOUT, "weights section: index count differs from the model size");
  if (n) HIP_TRY(c, hipMemcpy(weights_out, dw.p, sizeof(float) * n, hipMemcpyDeviceToHost));
  return FLEET_OK;
}

// ------------------------------------------ model parameters (getModelParametersNative)

int fleet_model_params_device(fleet_ctx* c, const float* d_weights, size_t n_weights, const float* d_biases,
                              size_t n_biases, int graph_edges, void* d_out, void* stream) {
  if (!c || !d_out || graph_edges < 0 || (n_weights && !d_weights) || (n_biases && graph_edges && !d_biases))
    return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  HIP_TRY(c, fleet::launch_encode_model_params(d_weights, (int64_t)n_weights, d_biases, (int64_t)n_biases,
                                               n_biases ? (int64_t)graph_edges : 0, (uint8_t*)d_out,
                                               pick(c, stream)));
  return FLEET_OK;
}

int fleet_kardam_grads(fleet_ctx* c, const char* const* uploads, const size_t* lens, int M, const double* dampen,
                       double lr, const char* const* prev, char* g_out, size_t g_pitch, size_t* g_len,
                       double* norm_g, double* norm_diff) {
  if (!c || !uploads || !lens || !dampen || M <= 0 || !norm_g || !norm_diff) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  const size_t len = lens[0];
  int rc = check_text_len(c, len);
  if (rc) return rc;
  for (int i = 0; i < M; ++i)
    if (!uploads[i] || lens[i] != len)
      return fail(c, FLEET_ERR_ARG, "upload %d has length %zu, expected %zu (one model layout)", i, lens[i], len);
  const size_t n = fleet_b64_count(len);
  std::vector<int32_t> hw(kHdrWords);
  host_layout_parse(uploads[M - 1], len, (int64_t)n, FLEET_MAX_HEADERS, hw.data());
  if (hw[0] != 0) return fail(c, FLEET_ERR_LAYOUT, "last upload's header does not describe a gradient layout");
  const int nh = hw[1];
  const size_t n_flat = (size_t)hw[2] - (size_t)nh;  // flatGrad stops after the last bias block
  const size_t glen = fleet_b64_len(n_flat), gpad = round16(glen) + 16;
  if (g_len) *g_len = glen;
  if (!g_out || g_pitch < glen) return fail(c, FLEET_ERR_CAPACITY, "g row pitch %zu < %zu", g_pitch, glen);
  const size_t pitch = round16(len);
  bool any_prev = false;
  for (int i = 0; prev && i < M; ++i) any_prev |= prev[i] != nullptr;
  // staging: [uploads | prev rows | has_prev | dampen | header positions]; device adds [g rows | partials]
  const size_t o_prev = pitch * (size_t)M, o_has = o_prev + (any_prev ? gpad * (size_t)M : 0);
  const size_t o_damp = round16(o_has + (size_t)M), o_hdr = round16(o_damp + sizeof(double) * (size_t)M);
  const size_t o_g = round16(o_hdr + sizeof(int32_t) * (size_t)(nh + 1));
  const int64_t groups = (int64_t)groups_of(n_flat);
  const int nblk = (int)((groups + 255) / 256);
  const size_t o_part = round16(o_g + gpad * (size_t)M), o_end = o_part + sizeof(double) * 2 * (size_t)M * (nblk + 1);
  if ((rc = grow_pinned(c, o_end))) return rc;
  if ((rc = grow_dev(c, &c->d_a, &c->d_a_cap, o_end))) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));  // staging buffer reuse
  uint8_t* h = c->h_stage;
  for (int i = 0; i < M; ++i) {
    std::memcpy(h + (size_t)i * pitch, uploads[i], len);
    std::memset(h + (size_t)i * pitch + len, 0, pitch - len);
    h[o_has + i] = (uint8_t)(prev && prev[i]);
    if (any_prev) {
      uint8_t* row = h + o_prev + (size_t)i * gpad;
      std::memset(row, 'A', gpad);
      if (prev[i]) std::memcpy(row, prev[i], glen);
    }
  }
  std::memcpy(h + o_damp, dampen, sizeof(double) * (size_t)M);
  std::memcpy(h + o_hdr, hw.data() + 4, sizeof(int32_t) * (size_t)nh);
  uint8_t* d = c->d_a;
  HIP_TRY(c, hipMemcpyAsync(d, h, o_g, hipMemcpyHostToDevice, c->stream));
  int nb = 0;
  HIP_TRY(c, fleet::launch_kardam_grads(d, pitch, M, (const int32_t*)(d + o_hdr), nh, (int64_t)n_flat,
                                        (const double*)(d + o_damp), lr, any_prev ? d + o_prev : nullptr, gpad,
                                        d + o_has, d + o_g, gpad, (double*)(d + o_part), &nb, c->d_err, c->stream));
  HIP_TRY(c, hipMemcpyAsync(h + o_g, d + o_g, o_end - o_g, hipMemcpyDeviceToHost, c->stream));
  if ((rc = read_err(c, c->stream))) return rc;
  const double* part = (const double*)(h + o_part);
  for (int i = 0; i < M; ++i) {
    std::memcpy(g_out + (size_t)i * g_pitch, h + o_g + (size_t)i * gpad, glen);
    double sg = 0, sd = 0;
    for (int b = 0; b < nb; ++b) {  // block partials in index order
      sg += part[(size_t)i * 2 * nb + b];
      sd += part[(size_t)i * 2 * nb + nb + b];
    }
    norm_g[i] = std::sqrt(sg);
    norm_diff[i] = (prev && prev[i]) ? std::sqrt(sd) : std::nan("");
  }
  return FLEET_OK;
}

size_t fleet_minibatch_len(int F, int B, int num_labels, int with_teacher) {
  if (F < 0 || B < 0 || num_labels < 0) return 0;
  const size_t n = 7 + (size_t)B * ((size_t)F + (with_teacher ? (size_t)num_labels : 0) + 1) + (with_teacher ? 1 : 0);
  return fleet_b64_len(n);
}

int fleet_minibatch_device(fleet_ctx* c, const void* d_images, size_t n_images, int F, const void* d_labels,
                           const void* d_idx, int B, const void* d_teacher, int num_labels, const float header[7],
                           void* d_out, void* stream) {
  if (!c || !d_out || !header || F < 0 || B < 0 || num_labels < 0 || (B && (!d_idx || !d_labels || !d_images)) ||
      (d_teacher && num_labels == 0))
    return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  HIP_TRY(c, fleet::launch_encode_minibatch((const float*)d_images, (int64_t)n_images, F, (const int32_t*)d_labels,
                                            (const int32_t*)d_idx, B, (const float*)d_teacher, num_labels, header,
                                            (uint8_t*)d_out, c->d_dev_err, pick(c, stream)));
  return FLEET_OK;
}

int fleet_minibatch(fleet_ctx* c, const float* images, size_t n_images, int F, const int32_t* labels,
                    const int32_t* idx, int B, const float* teacher, int num_labels, const float header[7],
                    char* out, size_t cap, size_t* out_len) {
  if (!c || !header || F < 0 || B < 0 || num_labels < 0 || (B && (!idx || !labels || !images)) ||
      (teacher && num_labels == 0))
    return FLEET_ERR_ARG;
  const size_t len = fleet_minibatch_len(F, B, num_labels, teacher != nullptr);
  if (out_len) *out_len = len;
  if (cap < len || !out) return fail(c, FLEET_ERR_CAPACITY, "output capacity %zu < %zu", cap, len);
  for (int b = 0; b < B; ++b)
    if (idx[b] < 0 || (size_t)idx[b] >= n_images)
      return fail(c, FLEET_ERR_ARG, "sample %d: index %d outside the %zu images", b, idx[b], n_images);
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  // staging: [B x F features | B labels | 0..B-1 | B x NL teacher]; the device gathers nothing
  const size_t nl = teacher ? (size_t)num_labels : 0;
  const size_t o_lab = round16(sizeof(float) * (size_t)B * (size_t)F), o_idx = o_lab + round16(4 * (size_t)B);
  const size_t o_tea = o_idx + round16(4 * (size_t)B), o_out = o_tea + round16(sizeof(float) * (size_t)B * nl);
  const size_t o_end = o_out + round16(len) + 16;
  int rc;
  if ((rc = grow_pinned(c, o_end))) return rc;
  if ((rc = grow_dev(c, &c->d_a, &c->d_a_cap, o_end))) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));  // staging buffer reuse
  uint8_t* h = c->h_stage;
  for (int b = 0; b < B; ++b) {
    std::memcpy(h + sizeof(float) * (size_t)b * F, images + (size_t)idx[b] * F, sizeof(float) * (size_t)F);
    reinterpret_cast<int32_t*>(h + o_lab)[b] = labels[idx[b]];
    reinterpret_cast<int32_t*>(h + o_idx)[b] = b;
  }
  if (teacher) std::memcpy(h + o_tea, teacher, sizeof(float) * (size_t)B * nl);
  uint8_t* d = c->d_a;
  HIP_TRY(c, hipMemcpyAsync(d, h, o_out, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, fleet::launch_encode_minibatch((const float*)d, (int64_t)B, F, (const int32_t*)(d + o_lab),
                                            (const int32_t*)(d + o_idx), B, teacher ? (const float*)(d + o_tea) : nullptr,
                                            num_labels, header, d + o_out, c->d_err, c->stream));
  HIP_TRY(c, hipMemcpyAsync(h + o_out, d + o_out, len, hipMemcpyDeviceToHost, c->stream));
  if ((rc = read_err(c, c->stream))) return rc;
  std::memcpy(out, h + o_out, len);
  return FLEET_OK;
}

size_t fleet_teacher_weight_count(void) { return (size_t)fleet::teacher_weight_count(); }
size_t fleet_teacher_bias_count(void) { return (size_t)fleet::teacher_bias_count(); }

int fleet_teacher_forward_device(fleet_ctx* c, const void* d_w, const void* d_b, const void* d_images, size_t n_images,
                                 int F, const void* d_idx, int B, float temperature, void* d_probs, void* stream) {
  if (!c || B < 0 || (B && (!d_w || !d_b || !d_images || !d_probs)) || F < 28 * 28) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  HIP_TRY(c, fleet::launch_teacher_forward((const float*)d_w, (const float*)d_b, (const float*)d_images,
                                           (int64_t)n_images, F, (const int32_t*)d_idx, B, temperature,
                                           (float*)d_probs, c->d_dev_err, pick(c, stream)));
  return FLEET_OK;
}

int fleet_teacher_forward(fleet_ctx* c, const float* w, size_t n_w, const float* b, size_t n_b, const float* images,
                          size_t n_images, int F, const int32_t* idx, int B, float temperature, float* probs) {
  if (!c || B < 0 || F < 28 * 28 || (B && (!w || !b || !images || !idx || !probs))) return FLEET_ERR_ARG;
  if (n_w != fleet_teacher_weight_count() || n_b != fleet_teacher_bias_count())
    return fail(c, FLEET_ERR_ARG, "teacher: %zu weights and %zu biases, expected %zu and %zu", n_w, n_b,
                fleet_teacher_weight_count(), fleet_teacher_bias_count());
  for (int i = 0; i < B; ++i)
    if (idx[i] < 0 || (size_t)idx[i] >= n_images)
      return fail(c, FLEET_ERR_ARG, "sample %d: index %d outside the %zu images", i, idx[i], n_images);
  if (B == 0) return FLEET_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  // staging: [w | b | B gathered rows | B x 10 probs]
  const size_t o_b = round16(sizeof(float) * n_w), o_x = o_b + round16(sizeof(float) * n_b);
  const size_t o_p = o_x + round16(sizeof(float) * (size_t)B * (size_t)F);
  const size_t o_end = o_p + round16(sizeof(float) * (size_t)B * 10);
  int rc;
  if ((rc = grow_pinned(c, o_end))) return rc;
  if ((rc = grow_dev(c, &c->d_a, &c->d_a_cap, o_end))) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));  // staging buffer reuse
  uint8_t* h = c->h_stage;
  std::memcpy(h, w, sizeof(float) * n_w);
  std::memcpy(h + o_b, b, sizeof(float) * n_b);
  for (int i = 0; i < B; ++i)
    std::memcpy(h + o_x + sizeof(float) * (size_t)i * F, images + (size_t)idx[i] * F, sizeof(float) * (size_t)F);
  uint8_t* d = c->d_a;
  HIP_TRY(c, hipMemcpyAsync(d, h, o_p, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, fleet::launch_teacher_forward((const float*)d, (const float*)(d + o_b), (const float*)(d + o_x), B, F,
                                           nullptr, B, temperature, (float*)(d + o_p), c->d_err, c->stream));
  HIP_TRY(c, hipMemcpyAsync(h + o_p, d + o_p, sizeof(float) * (size_t)B * 10, hipMemcpyDeviceToHost, c->stream));
  if ((rc = read_err(c, c->stream))) return rc;
  std::memcpy(probs, h + o_p, sizeof(float) * (size_t)B * 10);
  return FLEET_OK;
}

int fleet_model_params(fleet_ctx* c, const float* weights, size_t n_weights, const float* biases, size_t n_biases,
                       int graph_edges, char* out, size_t cap, size_t* out_len) {
  if (!c || graph_edges < 0 || (n_weights && !weights) || (n_biases && !biases)) return FLEET_ERR_ARG;
  const size_t n = n_biases * (size_t)graph_edges + n_weights;
  const size_t len = fleet_b64_len(n);
  if (out_len) *out_len = len;
  if (cap < len || !out) return fail(c, FLEET_ERR_CAPACITY, "output capacity %zu < %zu", cap, len);
  DevMem dw, db, dt;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    DEVICE_SCOPE(c);
    if (n_weights) HIP_TRY(c, hipMalloc(&dw.p, n_weights * sizeof(float)));
    if (n_biases) HIP_TRY(c, hipMalloc(&db.p, n_biases * sizeof(float)));
    HIP_TRY(c, hipMalloc(&dt.p, 16 * groups_of(n) + 16));
    if (n_weights) HIP_TRY(c, hipMemcpyAsync(dw.p, weights, n_weights * sizeof(float), hipMemcpyHostToDevice, c->stream));
    if (n_biases) HIP_TRY(c, hipMemcpyAsync(db.p, biases, n_biases * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, fleet::launch_encode_model_params((const float*)dw.p, (int64_t)n_weights, (const float*)db.p,
                                                 (int64_t)n_biases, n_biases ? (int64_t)graph_edges : 0,
                                                 (uint8_t*)dt.p, c->stream));
    if (len) HIP_TRY(c, hipMemcpyAsync(out, dt.p, len, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  return FLEET_OK;
}

// ------------------------------------------ SGD epilogue (descentNative)

namespace {

// Segments of network::descent(vector)'s walk over the gradients() layout
// (network.h:1185-1202): weight blocks of non-null W, bias blocks of the
// fully-connected layers. Also the layout's total length and the model sizes.
// Segments of the model step; with [vb, ve) only the parts whose gradient
// positions fall in that window of upload values (an element shard), with
// gradient offsets relative to vb.
static int descent_segments(fleet_ctx* c, const int32_t* w_sizes, const uint8_t* w_present, int n_w,
                     const int32_t* b_sizes, const uint8_t* fc_layer, int n_b, size_t* n_up, size_t* n_weights,
                     size_t* n_fc, std::vector<fleet::DescentSegs>* segs, size_t vb = 0, size_t ve = SIZE_MAX) {
  if (n_w < 0 || n_b < 0 || (n_w && (!w_sizes || !w_present)) || (n_b && (!b_sizes || !fc_layer)))
    return fail(c, FLEET_ERR_ARG, "bad descent layout arguments");
  segs->clear();
  auto add = [&](int kind, size_t g, size_t m, size_t len) {
    const size_t lo = std::max(g, vb), hi = std::min(g + len, ve);
    if (lo >= hi) return;
    m += lo - g;
    len = hi - lo;
    g = lo - vb;
    if (segs->empty() || segs->back().n == fleet::kMaxDescentSegs) {
      segs->emplace_back();
      segs->back().n = 0;
    }
    fleet::DescentSegs& d = segs->back();
    d.kind[d.n] = kind;
    d.grad_off[d.n] = (int64_t)g;
    d.model_off[d.n] = (int64_t)m;
    d.len[d.n] = (int64_t)len;
    ++d.n;
  };
  size_t idx = 1, wo = 0, bo = 0;
  for (int i = 0; i < n_w; ++i) {
    if (w_sizes[i] < 0) return fail(c, FLEET_ERR_ARG, "negative weight block size");
    ++idx;
    if (w_present[i] && w_sizes[i] > 0) add(0, idx, wo, (size_t)w_sizes[i]);
    if (w_present[i]) wo += (size_t)w_sizes[i];
    idx += (size_t)w_sizes[i];
  }
  ++idx;
  for (int k = 0; k < n_b; ++k) {
    if (b_sizes[k] < 0) return fail(c, FLEET_ERR_ARG, "negative bias block size");
    ++idx;
    if (fc_layer[k] && b_sizes[k] > 0) add(1, idx, bo, (size_t)b_sizes[k]);
    if (fc_layer[k]) bo += (size_t)b_sizes[k];
    idx += (size_t)b_sizes[k];
  }
  *n_up = idx;
  *n_weights = wo;
  *n_fc = bo;
  return FLEET_OK;
}

}  // namespace

int fleet_descent_device(fleet_ctx* c, float* d_weights, float* d_fc_bias, const float* d_grad,
                         const int32_t* w_sizes, const uint8_t* w_present, int n_w, const int32_t* b_sizes,
                         const uint8_t* fc_layer, int n_b, float lr, void* stream) {
  if (!c || !d_grad) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  size_t n_up = 0, nw = 0, nf = 0;
  std::vector<fleet::DescentSegs> segs;
  int rc = descent_segments(c, w_sizes, w_present, n_w, b_sizes, fc_layer, n_b, &n_up, &nw, &nf, &segs);
  if (rc) return rc;
  if ((nw && !d_weights) || (nf && !d_fc_bias)) return FLEET_ERR_ARG;
  for (const auto& sg : segs)
    HIP_TRY(c, fleet::launch_descent(d_weights, d_fc_bias, d_grad, sg, lr, pick(c, stream)));
  return FLEET_OK;
}

int fleet_descent_window_device(fleet_ctx* c, float* d_weights, float* d_fc_bias, const float* d_grad_window,
                                size_t value_begin, size_t value_end, const int32_t* w_sizes,
                                const uint8_t* w_present, int n_w, const int32_t* b_sizes, const uint8_t* fc_layer,
                                int n_b, float lr, void* stream) {
  if (!c || !d_grad_window || value_end < value_begin) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  size_t n_up = 0, nw = 0, nf = 0;
  std::vector<fleet::DescentSegs> segs;
  int rc = descent_segments(c, w_sizes, w_present, n_w, b_sizes, fc_layer, n_b, &n_up, &nw, &nf, &segs, value_begin,
                            value_end);
  if (rc) return rc;
  if ((nw && !d_weights) || (nf && !d_fc_bias)) return FLEET_ERR_ARG;
  for (const auto& sg : segs)
    HIP_TRY(c, fleet::launch_descent(d_weights, d_fc_bias, d_grad_window, sg, lr, pick(c, stream)));
  return FLEET_OK;
}

int fleet_descent(fleet_ctx* c, float* weights, size_t n_weights, float* fc_bias, size_t n_fc_bias,
                  const float* grad, size_t n_grad, const int32_t* w_sizes, const uint8_t* w_present, int n_w,
                  const int32_t* b_sizes, const uint8_t* fc_layer, int n_b, float lr) {
  if (!c || !grad) return FLEET_ERR_ARG;
  size_t n_up = 0, nw = 0, nf = 0;
  std::vector<fleet::DescentSegs> segs;
  int rc;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    rc = descent_segments(c, w_sizes, w_present, n_w, b_sizes, fc_layer, n_b, &n_up, &nw, &nf, &segs);
  }
  if (rc) return rc;
  if (n_grad != n_up || n_weights != nw || n_fc_bias != nf || (nw && !weights) || (nf && !fc_bias))
    return fail(c, FLEET_ERR_ARG, "descent: sizes do not match the layout (grad %zu/%zu, weights %zu/%zu, bias %zu/%zu)",
                n_grad, n_up, n_weights, nw, n_fc_bias, nf);
  // the header floats network::descent(vector) reads its block sizes from
  size_t idx = 0;
  bool ok = grad[idx++] == (float)n_w;
  for (int i = 0; i < n_w && ok; ++i) {
    ok = grad[idx++] == (float)w_sizes[i];
    idx += (size_t)w_sizes[i];
  }
  ok = ok && grad[idx++] == (float)n_b;
  for (int k = 0; k < n_b && ok; ++k) {
    ok = grad[idx++] == (float)b_sizes[k];
    idx += (size_t)b_sizes[k];
  }
  if (!ok) return fail(c, FLEET_ERR_LAYOUT, "descent: gradient header does not match the model layout");
  DevMem dw, db, dg;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    DEVICE_SCOPE(c);
    if (nw) HIP_TRY(c, hipMalloc(&dw.p, nw * sizeof(float)));
    if (nf) HIP_TRY(c, hipMalloc(&db.p, nf * sizeof(float)));
    HIP_TRY(c, hipMalloc(&dg.p, n_grad * sizeof(float)));
    if (nw) HIP_TRY(c, hipMemcpyAsync(dw.p, weights, nw * sizeof(float), hipMemcpyHostToDevice, c->stream));
    if (nf) HIP_TRY(c, hipMemcpyAsync(db.p, fc_bias, nf * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(dg.p, grad, n_grad * sizeof(float), hipMemcpyHostToDevice, c->stream));
    for (const auto& sg : segs)
      HIP_TRY(c, fleet::launch_descent((float*)dw.p, (float*)db.p, (const float*)dg.p, sg, lr, c->stream));
    if (nw) HIP_TRY(c, hipMemcpyAsync(weights, dw.p, nw * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    if (nf) HIP_TRY(c, hipMemcpyAsync(fc_bias, db.p, nf * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  return FLEET_OK;
}

// descentNative's model copy in DISTILLATION_MODE=1 (cppNN_backend.cpp:355-372):
// cnnNew->read(cnn.getParams()) of the unquantised model. getParams prints the
// biases and the first-occurrence dictionary values with `ostream << float`
// (precision 6 = %g) and read() parses them back (strtof); every weight takes
// its dictionary entry's value. All on the device: the dictionary (sort-based,
// no O(n*U) scans), the %g / strtof round trip of the U values and the biases
// (decimal6.h: exact integer arithmetic, checked against libc on every finite
// binary32, digest fn 22) and the gather; no host round trip of the values.
int fleet_model_version(fleet_ctx* c, const float* weights, const int32_t* dims, int n_mats, const float* biases,
                        size_t n_biases, float* weights_out, float* biases_out) {
  if (!c || (n_biases && (!biases || !biases_out))) return FLEET_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  size_t n = 0;
  int rc = model_total(c, dims, n_mats, &n);
  if (rc) return rc;
  if (n && (!weights || !weights_out)) return FLEET_ERR_ARG;
  DevMem dw, dd, di, db;
  // the biases' text round trip on the device as well (getParams prints them with `<<` too)
  if (n_biases) {
    HIP_TRY(c, hipMalloc(&db.p, n_biases * sizeof(float)));
    HIP_TRY(c, hipMemcpyAsync(db.p, biases, n_biases * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->d_err, 0, sizeof(int), c->stream));
    HIP_TRY(c, fleet::model_g6_inplace((float*)db.p, (int64_t)n_biases, c->d_err, c->stream));
    HIP_TRY(c, hipMemcpyAsync(biases_out, db.p, n_biases * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->h_err, c->d_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (*c->h_err) {
      HIP_TRY(c, hipMemset(c->d_err, 0, sizeof(int)));
      return fail(c, FLEET_ERR_ARG, "non-finite bias: the reference's text read fails");
    }
  }
  if (!n) return FLEET_OK;
  HIP_TRY(c, hipMalloc(&dw.p, n * sizeof(float)));
  HIP_TRY(c, hipMalloc(&dd.p, (n + 1) * sizeof(float)));
  HIP_TRY(c, hipMalloc(&di.p, n * sizeof(int32_t)));
  HIP_TRY(c, hipMemcpyAsync(dw.p, weights, n * sizeof(float), hipMemcpyHostToDevice, c->stream));
  int32_t U = 0;
  HIP_TRY(c, fleet::model_quantize_index((const float*)dw.p, dims, n_mats, nullptr, (float*)dd.p, (int32_t*)di.p,
                                         &U, c->stream, false));
  // the U dictionary values through `<<` / `>>` (decimal6.h), in place, then the gather
  HIP_TRY(c, hipMemsetAsync(c->d_err, 0, sizeof(int), c->stream));
  HIP_TRY(c, fleet::model_g6_inplace((float*)dd.p, (int64_t)U, c->d_err, c->stream));
  HIP_TRY(c, fleet::model_dict_gather((const int32_t*)di.p, (int64_t)n, (const float*)dd.p, (float*)dw.p, c->stream));
  HIP_TRY(c, hipMemcpyAsync(weights_out, dw.p, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->h_err, c->d_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (*c->h_err) {
    HIP_TRY(c, hipMemset(c->d_err, 0, sizeof(int)));
    return fail(c, FLEET_ERR_ARG, "non-finite weight: the reference's text read fails");
  }
  return FLEET_OK;
}

const char* fleet_update_kernel(size_t len) {
  static thread_local std::string name;
  name = fleet::update_kernel_name((int64_t)groups_of(fleet_b64_count(len)));
  return name.c_str();
}

int fleet_update_plan_grid(size_t len, int* kind, int64_t* blocks, int64_t* n_a, int64_t* n_w, int64_t* n_n) {
  if (!kind || !blocks || !n_a || !n_w || !n_n) return FLEET_ERR_ARG;
  fleet::update_plan_grid((int64_t)groups_of(fleet_b64_count(len)), kind, blocks, n_a, n_w, n_n);
  return FLEET_OK;
}

const char* fleet_update_encode_kernel(size_t len) {
  static thread_local std::string name;
  name = fleet::update_encode_kernel_name((int64_t)groups_of(fleet_b64_count(len)));
  return name.c_str();
}

int fleet_set_plan(const char* spec, char* err, size_t cap) {
  std::string e;
  if (fleet::set_plan_overrides(spec, &e) == 0) return FLEET_OK;
  if (err && cap) std::snprintf(err, cap, "%s", e.c_str());
  return FLEET_ERR_ARG;
}

const char* fleet_plan(void) {
  static thread_local std::string spec;
  spec = fleet::plan_spec();
  return spec.c_str();
}

int fleet_selftest_digest(fleet_ctx* c, int fn, uint64_t* out) {
  if (!c || !out) return FLEET_ERR_ARG;
  if (fn < 0 || fn > 23) return fail(c, FLEET_ERR_ARG, "no self-test function %d", fn);
  std::lock_guard<std::mutex> lk(c->mu);
  DEVICE_SCOPE(c);
  unsigned long long* d = nullptr;
  HIP_TRY(c, hipMalloc((void**)&d, sizeof(unsigned long long)));
  HIP_TRY(c, hipMemsetAsync(d, 0, sizeof(unsigned long long), c->stream));
  HIP_TRY(c, fleet::launch_digest(fn, d, c->stream));
  unsigned long long h = 0;
  HIP_TRY(c, hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  (void)hipFree(d);
  *out = h;
  return FLEET_OK;
}

}  // extern "C"
