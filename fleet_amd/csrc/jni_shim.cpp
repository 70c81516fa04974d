// fleet_amd/csrc/jni_shim.cpp -- JNI shim: the reference's native symbol names
// on top of the C-ABI (include/fleet_codec.h). Built as libfleet_native.so.
//
// Drop-in for the updater natives of the reference's server backend
// (Server/src/main/c++/cppNN_backend.cpp, loaded as libnative.so by
// commonLib/utils/JNITest.java:22-53; declared at CppNNUpdater.java:147-162 and
// ByteVec.java:23-26):
//   per-op gradient natives
//     Java_apps_cppNN_CppNNUpdater_getFlatGradient     cppNN_backend.cpp:701-720
//     Java_apps_cppNN_CppNNUpdater_mergeFlatGradient   :722-750
//     Java_utils_ByteVec_scalarMulNative               :753-777
//     Java_utils_ByteVec_getNorm                       :779-795
//     Java_utils_ByteVec_addNative                     :797-846
//     Java_utils_ByteVec_subtractNative                :848-892
//   the model the updater keeps (fleet_model, one per process like `cnn`/`models`)
//     Java_apps_cppNN_CppNNUpdater_fetchParamsNative   :282-301
//     Java_apps_cppNN_CppNNUpdater_initUpdater         :161-225 (model part)
//     Java_apps_cppNN_CppNNUpdater_descentNative       :329-383
//     Java_apps_cppNN_CppNNUpdater_getParametersNative :244-280
//     Java_apps_cppNN_CppNNUpdater_getModelParametersNative :227-242
//     ..._modelsSize, _getPriority/_setPriority, _getCurrEpoch/_setCurrEpoch, _getLrate :129-159,324-327
//     ..._getNumLabels, _hasOutlier                    :129-137
//     ..._printParamsNative                            :304-322
//   the offline sampler (fleet_sampler; dataset, buckets, client rotation, E/sigma/C)
//     Java_apps_cppNN_CppNNOfflineSampler_initSampler  :385-551
//     Java_apps_cppNN_CppNNOfflineSampler_getMiniBatch :677-699
//   plus boolean apps.cppNN.FleetSampler.setTeacherNative(float[] w, float[] b): the
//   mode-1 teacher's trained weights (below)
// so no native of libnative.so is reached any more: every global the
// reference's natives share (the model, E/sigma/C, the libc rand() stream that
// initSampler and initUpdater reseed) lives behind this one library;
// and the batched natives of an updater that makes one call per update:
//   byte[] apps.cppNN.FleetUpdater.aggregateNative(byte[][] uploads, double[] dampen)
//   byte[] apps.cppNN.FleetUpdater.aggregateDirectNative(ByteBuffer rows, int M, int len, int rowPitch,
//                                                          double[] dampen)
//   boolean apps.cppNN.FleetUpdater.registerDirectNative(ByteBuffer rows)
//   void apps.cppNN.FleetUpdater.unregisterDirectNative(ByteBuffer rows)
//
// Environment: FLEET_GPUS = devices the batched natives spread one update over
// (element sharding, fleet_update_multi; default 1, "all" = every visible GPU);
// FLEET_DISTILLATION_MODE = the reference's compile-time DISTILLATION_MODE (default 1);
// FLEET_SAMPLER_IID / FLEET_SAMPLER_OUTLIER / FLEET_SAMPLER_CLIENTS = the
// reference's source-edited sampler globals iid / outlier / numClients
// (cppNN_backend.cpp:59-61; defaults 0, 0, 10). In DISTILLATION_MODE=1 the
// reference's initSampler, after the buckets and whatever the sampler, parses the
// MNIST test set (returning early when it is missing, :485) and trains a teacher
// network (:481-545: 300 rand()-drawn samples through mojo's backward pass). Only
// iid mini-batches carry the teacher's outputs (uniformSample :593-620); nonIIDSample
// sends none. The training is not rebuilt here (it is client-side model compute,
// not the codec path): iid mode-1 mini-batches need the trained weights from the
// JVM through FleetSampler.setTeacherNative, and until then getMiniBatch fails with
// that reason. Its rand() draws do not move the sampler's indices: initUpdater
// reseeds after initSampler.
//
// Same argument meaning and results as the reference; failures return null / 0
// (Java sees a NullPointerException at the caller) and print the C-ABI error
// on stderr -- the reference has no error path at all. JNI rules kept: at most
// the guaranteed 16 local references without EnsureLocalCapacity, no JNI call
// inside a critical region, every Get*ArrayElements released.
#include <jni.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "fleet_codec.h"

namespace {

std::mutex g_mu;
std::vector<fleet_ctx*> g_ctxs;  // [0]: per-op natives, the model; all: the batched update
bool g_init = false;
// the updater's model and the sampler, each used only under its lock (a fetch
// replaces the model while another request thread may be reading it)
std::mutex g_model_mu;
fleet_model* g_model = nullptr;
std::mutex g_sampler_mu;
fleet_sampler* g_sampler = nullptr;
int g_E = 0;  // initUpdater's globals (cppNN_backend.cpp:47-50; zero until it runs)
double g_sigma = 0.0, g_C = 0.0;
constexpr int kSeed = 1;  // cppNN_backend.cpp:71
std::mutex g_rows_mu;
std::vector<char> g_rows;  // row staging of aggregateNative when the JVM cannot grant M local refs

void init_contexts() {
  if (g_init) return;
  g_init = true;
  int want = 1;
  if (const char* e = std::getenv("FLEET_GPUS")) want = std::strcmp(e, "all") == 0 ? 1 << 16 : std::max(1, std::atoi(e));
  for (int d = 0; d < want; ++d) {
    fleet_ctx* c = nullptr;
    if (fleet_create(d, &c) != FLEET_OK) break;
    g_ctxs.push_back(c);
  }
  if (g_ctxs.empty()) std::fprintf(stderr, "[fleet] fleet_create failed: no MI355X visible\n");
}

fleet_ctx* ctx() {
  std::lock_guard<std::mutex> lk(g_mu);
  init_contexts();
  return g_ctxs.empty() ? nullptr : g_ctxs[0];
}

std::vector<fleet_ctx*> all_ctx() {
  std::lock_guard<std::mutex> lk(g_mu);
  init_contexts();
  return g_ctxs;
}

int distillation_mode() {
  const char* e = std::getenv("FLEET_DISTILLATION_MODE");
  return e ? (std::atoi(e) != 0) : 1;
}

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

// JVM byte[] -> host bytes (no NUL terminator needed: lengths are explicit)
struct Bytes {
  JNIEnv* env;
  jbyteArray arr;
  jbyte* p;
  jsize n;
  Bytes(JNIEnv* e, jbyteArray a)
      : env(e), arr(a), p(a ? e->GetByteArrayElements(a, nullptr) : nullptr), n(a ? e->GetArrayLength(a) : 0) {}
  ~Bytes() {
    if (p) env->ReleaseByteArrayElements(arr, p, JNI_ABORT);
  }
  bool ok() const { return p != nullptr; }
  const char* data() const { return reinterpret_cast<const char*>(p); }
};

jbyteArray to_java(JNIEnv* env, const char* v, size_t n) {
  jbyteArray a = env->NewByteArray((jsize)n);
  if (a) env->SetByteArrayRegion(a, 0, (jsize)n, reinterpret_cast<const jbyte*>(v));
  return a;
}

jbyteArray fail(fleet_ctx* c, const char* what, int rc) {
  std::fprintf(stderr, "[fleet] %s failed (%d): %s\n", what, rc, c ? fleet_last_error(c) : "no context");
  return nullptr;
}

jbyteArray mfail(const char* what, int rc) {
  std::fprintf(stderr, "[fleet] %s failed (%d): %s\n", what, rc, g_model ? fleet_model_last_error(g_model) : "no model");
  return nullptr;
}

// one update over every context (FLEET_GPUS), host pointers to the M uploads
int update_ptrs(const std::vector<fleet_ctx*>& cs, const char* const* ups, const size_t* lens, int M, const double* d,
                char* out, size_t cap, size_t* n) {
  if (cs.size() > 1) return fleet_update_multi(cs.data(), (int)cs.size(), ups, lens, M, d, out, cap, n, nullptr);
  return fleet_update(cs[0], ups, lens, M, d, out, cap, n, nullptr);
}

// Direct ByteBuffers page-locked by registerDirectNative, each with a weak global
// reference to its Java object. The library's registration record only knows an
// address range; the weak reference tells whether the buffer that owns the range is
// still alive. A buffer the JVM collected without unregisterDirectNative (its Cleaner
// freed the memory; a later buffer may sit at the same address) leaves a stale page
// lock: aggregateDirectNative finds it by address, sees the referent gone, releases
// the registration and stages the rows instead of DMAing from the stale pages.
struct DirectReg {
  uintptr_t base;
  size_t bytes;
  jweak ref;
};
std::mutex g_direct_mu;
std::vector<DirectReg> g_direct;

// drop the shim's records overlapping [a, a + bytes) (the library released their page
// locks when a new registration covered them)
void forget_overlapping(JNIEnv* env, uintptr_t a, size_t bytes) {
  for (size_t i = g_direct.size(); i-- > 0;) {
    const DirectReg& r = g_direct[i];
    if (r.base < a + bytes && a < r.base + r.bytes) {
      env->DeleteWeakGlobalRef(r.ref);
      g_direct.erase(g_direct.begin() + (long)i);
    }
  }
}

// Before rows [p, p + bytes) of `buf` go to fleet_update_rows: every registration
// they touch must belong to a live buffer. One whose buffer was collected is released
// (library page lock and record), so the library stages those rows.
void release_stale(JNIEnv* env, fleet_ctx* c, jobject buf, const char* p, size_t bytes) {
  const uintptr_t a = (uintptr_t)p;
  std::lock_guard<std::mutex> lk(g_direct_mu);
  for (size_t i = g_direct.size(); i-- > 0;) {
    const DirectReg r = g_direct[i];
    if (!(r.base < a + bytes && a < r.base + r.bytes)) continue;
    // alive: the same buffer, or another live view of the registered memory
    if (env->IsSameObject(r.ref, buf) || !env->IsSameObject(r.ref, nullptr)) continue;
    (void)fleet_host_unregister(c, (void*)r.base);
    env->DeleteWeakGlobalRef(r.ref);
    g_direct.erase(g_direct.begin() + (long)i);
  }
}

int update_rows(const std::vector<fleet_ctx*>& cs, const char* rows, size_t pitch, size_t len, int M, const double* d,
                char* out, size_t cap, size_t* n) {
  if (cs.size() > 1) return fleet_update_rows_multi(cs.data(), (int)cs.size(), rows, pitch, len, M, d, out, cap, n, nullptr);
  return fleet_update_rows(cs[0], rows, pitch, len, M, d, out, cap, n, nullptr);
}

}  // namespace

extern "C" {

// ----------------------------------------------------------- per-op natives

JNIEXPORT jbyteArray JNICALL Java_apps_cppNN_CppNNUpdater_getFlatGradient(JNIEnv* env, jobject, jbyteArray input) {
  fleet_ctx* c = ctx();
  if (!c || !input) return nullptr;
  Bytes in(env, input);
  if (!in.ok()) return nullptr;
  std::vector<char> out((size_t)in.n + 16);
  size_t n = 0;
  int rc = fleet_flat_gradient(c, in.data(), (size_t)in.n, out.data(), out.size(), &n);
  return rc == FLEET_OK ? to_java(env, out.data(), n) : fail(c, "getFlatGradient", rc);
}

JNIEXPORT jbyteArray JNICALL Java_apps_cppNN_CppNNUpdater_mergeFlatGradient(JNIEnv* env, jobject, jbyteArray g,
                                                                            jbyteArray flatG) {
  fleet_ctx* c = ctx();
  if (!c || !g || !flatG) return nullptr;
  Bytes a(env, g), b(env, flatG);
  if (!a.ok() || !b.ok()) return nullptr;
  std::vector<char> out((size_t)a.n + 16);
  size_t n = 0;
  int rc = fleet_merge_flat_gradient(c, a.data(), (size_t)a.n, b.data(), (size_t)b.n, out.data(), out.size(), &n);
  return rc == FLEET_OK ? to_java(env, out.data(), n) : fail(c, "mergeFlatGradient", rc);
}

JNIEXPORT jbyteArray JNICALL Java_utils_ByteVec_scalarMulNative(JNIEnv* env, jobject, jbyteArray input, jdouble a) {
  fleet_ctx* c = ctx();
  if (!c || !input) return nullptr;
  Bytes in(env, input);
  if (!in.ok()) return nullptr;
  std::vector<char> out((size_t)in.n + 16);
  size_t n = 0;
  int rc = fleet_scalar_mul(c, in.data(), (size_t)in.n, (double)a, out.data(), out.size(), &n);
  return rc == FLEET_OK ? to_java(env, out.data(), n) : fail(c, "scalarMulNative", rc);
}

JNIEXPORT jdouble JNICALL Java_utils_ByteVec_getNorm(JNIEnv* env, jobject, jbyteArray input) {
  fleet_ctx* c = ctx();
  if (!c || !input) return 0.0;
  Bytes in(env, input);
  if (!in.ok()) return 0.0;
  double r = 0.0;
  int rc = fleet_norm(c, in.data(), (size_t)in.n, &r);
  if (rc != FLEET_OK) fail(c, "getNorm", rc);
  return r;
}

static jbyteArray binop(JNIEnv* env, jbyteArray a, jbyteArray b, bool sub) {
  fleet_ctx* c = ctx();
  if (!c || !a || !b) return nullptr;
  Bytes x(env, a), y(env, b);
  if (!x.ok() || !y.ok()) return nullptr;
  std::vector<char> out((size_t)x.n + 16);
  size_t n = 0;
  int rc = sub ? fleet_subtract(c, x.data(), (size_t)x.n, y.data(), (size_t)y.n, out.data(), out.size(), &n)
               : fleet_add(c, x.data(), (size_t)x.n, y.data(), (size_t)y.n, out.data(), out.size(), &n);
  return rc == FLEET_OK ? to_java(env, out.data(), n) : fail(c, sub ? "subtractNative" : "addNative", rc);
}

JNIEXPORT jbyteArray JNICALL Java_utils_ByteVec_addNative(JNIEnv* env, jobject, jbyteArray a, jbyteArray b) {
  return binop(env, a, b, false);
}

JNIEXPORT jbyteArray JNICALL Java_utils_ByteVec_subtractNative(JNIEnv* env, jobject, jbyteArray a, jbyteArray b) {
  return binop(env, a, b, true);
}

// ------------------------------------------------------------ batched update

// CppNNUpdater.java:420-509's getFlatGradient/scalarMultiply/add/scalarMultiply(1/M)/
// mergeFlatGradient chain in one call. The M uploads are read in place inside
// one critical region (GetPrimitiveArrayCritical: no copy by the JVM; only
// Get/ReleasePrimitiveArrayCritical are called inside it) after M local
// references are secured with EnsureLocalCapacity. A JVM that cannot grant M
// references gets the other path: one reference at a time, each upload copied
// with GetByteArrayRegion into a row buffer and the reference deleted.
JNIEXPORT jbyteArray JNICALL Java_apps_cppNN_FleetUpdater_aggregateNative(JNIEnv* env, jobject, jobjectArray uploads,
                                                                          jdoubleArray dampen) {
  const std::vector<fleet_ctx*> cs = all_ctx();
  if (cs.empty()) return nullptr;
  if (!uploads || !dampen) return fail(cs[0], "aggregateNative (null argument)", FLEET_ERR_ARG);
  const jsize M = env->GetArrayLength(uploads);
  if (M <= 0 || env->GetArrayLength(dampen) != M) return fail(cs[0], "aggregateNative (argument sizes)", FLEET_ERR_ARG);
  std::vector<double> d((size_t)M);
  env->GetDoubleArrayRegion(dampen, 0, M, d.data());
  std::vector<char> out;
  size_t n = 0;
  int rc;
  if (env->EnsureLocalCapacity(M) == JNI_OK) {
    std::vector<jbyteArray> arrs((size_t)M, nullptr);
    std::vector<size_t> lens((size_t)M);
    bool ok = true;
    for (jsize i = 0; i < M && ok; ++i) {
      arrs[(size_t)i] = (jbyteArray)env->GetObjectArrayElement(uploads, i);
      ok = arrs[(size_t)i] != nullptr;
      if (ok) lens[(size_t)i] = (size_t)env->GetArrayLength(arrs[(size_t)i]);
    }
    std::vector<const char*> ptrs((size_t)M, nullptr);
    jsize pinned = 0;
    if (ok) {
      out.resize(lens[0] + 16);
      for (; pinned < M; ++pinned) {
        ptrs[(size_t)pinned] =
            static_cast<const char*>(env->GetPrimitiveArrayCritical(arrs[(size_t)pinned], nullptr));
        if (!ptrs[(size_t)pinned]) break;
      }
      rc = pinned == M ? update_ptrs(cs, ptrs.data(), lens.data(), (int)M, d.data(), out.data(), out.size(), &n)
                       : FLEET_ERR_NOMEM;
      for (jsize i = pinned; i-- > 0;)
        env->ReleasePrimitiveArrayCritical(arrs[(size_t)i], const_cast<char*>(ptrs[(size_t)i]), JNI_ABORT);
    } else {
      rc = FLEET_ERR_ARG;
    }
    for (jsize i = 0; i < M; ++i)
      if (arrs[(size_t)i]) env->DeleteLocalRef(arrs[(size_t)i]);
    if (!ok) return fail(cs[0], "aggregateNative (null upload)", rc);
  } else {
    env->ExceptionClear();  // the OutOfMemoryError of the refused capacity
    std::lock_guard<std::mutex> rows_lk(g_rows_mu);
    size_t len = 0, pitch = 0;
    rc = FLEET_OK;
    for (jsize i = 0; i < M && rc == FLEET_OK; ++i) {
      jbyteArray a = (jbyteArray)env->GetObjectArrayElement(uploads, i);
      if (!a) {
        rc = FLEET_ERR_ARG;
        break;
      }
      const size_t li = (size_t)env->GetArrayLength(a);
      if (i == 0) {
        len = li;
        pitch = (len + 15) / 16 * 16;
        if (g_rows.size() < pitch * (size_t)M) g_rows.resize(pitch * (size_t)M);
      }
      if (li != len) rc = FLEET_ERR_ARG;
      else env->GetByteArrayRegion(a, 0, (jsize)len, reinterpret_cast<jbyte*>(g_rows.data() + (size_t)i * pitch));
      env->DeleteLocalRef(a);
    }
    if (rc != FLEET_OK) return fail(cs[0], "aggregateNative (null or ragged upload)", rc);
    out.resize(len + 16);
    rc = update_rows(cs, g_rows.data(), pitch, len, (int)M, d.data(), out.data(), out.size(), &n);
  }
  return rc == FLEET_OK ? to_java(env, out.data(), n) : fail(cs[0], "aggregateNative", rc);
}

// The same update over uploads the Java side deserialised into ONE direct
// ByteBuffer, row i at byte i*rowPitch: no JVM array is touched, and when the
// buffer was registered (registerDirectNative) each GPU DMAs its column window
// straight from it (fleet_update_rows: no host copy).
JNIEXPORT jbyteArray JNICALL Java_apps_cppNN_FleetUpdater_aggregateDirectNative(JNIEnv* env, jobject, jobject rows,
                                                                                jint M, jint len, jint rowPitch,
                                                                                jdoubleArray dampen) {
  const std::vector<fleet_ctx*> cs = all_ctx();
  if (cs.empty()) return nullptr;
  if (!rows || !dampen || M <= 0 || len < 0 || rowPitch < len || env->GetArrayLength(dampen) != M)
    return fail(cs[0], "aggregateDirectNative (arguments)", FLEET_ERR_ARG);
  const char* base = static_cast<const char*>(env->GetDirectBufferAddress(rows));
  const jlong cap = env->GetDirectBufferCapacity(rows);
  if (!base || cap < (jlong)rowPitch * (M - 1) + len)
    return fail(cs[0], "aggregateDirectNative (not a direct buffer of M rows)", FLEET_ERR_ARG);
  std::vector<double> d((size_t)M);
  env->GetDoubleArrayRegion(dampen, 0, M, d.data());
  release_stale(env, cs[0], rows, base, (size_t)rowPitch * (size_t)(M - 1) + (size_t)len);
  std::vector<char> out((size_t)len + 16);
  size_t n = 0;
  const int rc = update_rows(cs, base, (size_t)rowPitch, (size_t)len, (int)M, d.data(), out.data(), out.size(), &n);
  return rc == FLEET_OK ? to_java(env, out.data(), n) : fail(cs[0], "aggregateDirectNative", rc);
}

// Page-locks a long-lived direct ByteBuffer (e.g. the rows of aggregateDirectNative).
JNIEXPORT jboolean JNICALL Java_apps_cppNN_FleetUpdater_registerDirectNative(JNIEnv* env, jobject, jobject buf) {
  fleet_ctx* c = ctx();
  if (!c || !buf) return JNI_FALSE;
  void* p = env->GetDirectBufferAddress(buf);
  const jlong cap = env->GetDirectBufferCapacity(buf);
  if (!p || cap <= 0) return JNI_FALSE;
  std::lock_guard<std::mutex> lk(g_direct_mu);
  const int rc = fleet_host_register(c, p, (size_t)cap);
  // the library released any registration overlapping this one before it tried to page-
  // lock the range (p and cap are valid here, so that happened whether or not the lock
  // succeeded): drop their records either way, or a later release would unregister
  // memory the library no longer holds
  forget_overlapping(env, (uintptr_t)p, (size_t)cap);
  if (rc != FLEET_OK) {
    fail(c, "registerDirectNative", rc);
    return JNI_FALSE;
  }
  const jweak ref = env->NewWeakGlobalRef(buf);
  if (ref) g_direct.push_back(DirectReg{(uintptr_t)p, (size_t)cap, ref});
  return JNI_TRUE;
}

// Releases the page lock; the Java side should call it before the buffer is dropped
// (its Cleaner frees the memory). A registration left behind is caught by its weak
// reference: the next aggregateDirectNative over that memory finds the buffer
// collected, releases the registration and stages the rows (release_stale).
JNIEXPORT void JNICALL Java_apps_cppNN_FleetUpdater_unregisterDirectNative(JNIEnv* env, jobject, jobject buf) {
  fleet_ctx* c = ctx();
  if (!c || !buf) return;
  void* p = env->GetDirectBufferAddress(buf);
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_direct_mu);
  for (size_t i = g_direct.size(); i-- > 0;)
    if (g_direct[i].base == (uintptr_t)p) {
      env->DeleteWeakGlobalRef(g_direct[i].ref);
      g_direct.erase(g_direct.begin() + (long)i);
    }
  const int rc = fleet_host_unregister(c, p);
  if (rc != FLEET_OK) fail(c, "unregisterDirectNative", rc);
}

// ------------------------------------------------------------------- model

JNIEXPORT void JNICALL Java_apps_cppNN_CppNNUpdater_fetchParamsNative(JNIEnv* env, jobject, jbyteArray input) {
  fleet_ctx* c = ctx();
  if (!c || !input) return;
  Bytes in(env, input);
  if (!in.ok()) return;
  fleet_model* m = nullptr;
  const int rc = fleet_model_load(c, in.data(), (size_t)in.n, distillation_mode(), &m);
  if (rc != FLEET_OK) {
    fail(c, "fetchParamsNative", rc);
    return;
  }
  std::lock_guard<std::mutex> lk(g_model_mu);
  if (g_model) fleet_model_destroy(g_model);
  g_model = m;
}

// initUpdater (:161-225): srand(seed) and the rand() draws of its
// cnn.train_class (fleet_updater_reseed_ex: two, for the random shift that
// fetchParamsNative's set_random_augmentation enables; none before a fetch), E /
// sigma / C for the sampler's mini-batch headers, and the model part (lrates, the
// first version).
JNIEXPORT void JNICALL Java_apps_cppNN_CppNNUpdater_initUpdater(JNIEnv* env, jobject, jdoubleArray lrates, jint E,
                                                                jdouble sigma, jdouble C) {
  bool fetched;
  {
    std::lock_guard<std::mutex> lk(g_model_mu);
    fetched = g_model != nullptr;
  }
  {
    std::lock_guard<std::mutex> lk(g_sampler_mu);
    fleet_updater_reseed_ex(kSeed, fetched ? 1 : 0);
    g_E = E;
    g_sigma = sigma;
    g_C = C;
    if (g_sampler) fleet_sampler_set_hyper(g_sampler, E, sigma, C);
  }
  std::lock_guard<std::mutex> lk(g_model_mu);
  if (!g_model || !lrates) return;
  const jsize n = env->GetArrayLength(lrates);
  std::vector<double> lr((size_t)std::max<jsize>(n, 0));
  if (n > 0) env->GetDoubleArrayRegion(lrates, 0, n, lr.data());
  const int rc = fleet_model_init_updater(g_model, lr.data(), (int)n);
  if (rc != FLEET_OK) mfail("initUpdater", rc);
}

JNIEXPORT void JNICALL Java_apps_cppNN_CppNNUpdater_descentNative(JNIEnv* env, jobject, jbyteArray input,
                                                                  jint clientBatchSize, jint staleSize) {
  if (!input) return;
  Bytes in(env, input);
  if (!in.ok()) return;
  std::lock_guard<std::mutex> lk(g_model_mu);
  if (!g_model) return;
  const int rc = fleet_model_descent(g_model, in.data(), (size_t)in.n, clientBatchSize, staleSize);
  if (rc != FLEET_OK) mfail("descentNative", rc);
}

static jbyteArray model_text(JNIEnv* env, jint p, bool params) {
  std::lock_guard<std::mutex> lk(g_model_mu);
  if (!g_model) return nullptr;
  auto fn = params ? fleet_model_get_params : fleet_model_get_model_params;
  size_t need = 0;
  int rc = fn(g_model, p, nullptr, 0, &need);
  if (rc != FLEET_OK && rc != FLEET_ERR_CAPACITY) return mfail(params ? "getParametersNative" : "getModelParametersNative", rc);
  std::vector<char> out(need + 1);
  rc = fn(g_model, p, out.data(), out.size(), &need);
  return rc == FLEET_OK ? to_java(env, out.data(), need)
                        : mfail(params ? "getParametersNative" : "getModelParametersNative", rc);
}

JNIEXPORT jbyteArray JNICALL Java_apps_cppNN_CppNNUpdater_getParametersNative(JNIEnv* env, jobject, jint p) {
  return model_text(env, p, true);
}

JNIEXPORT jbyteArray JNICALL Java_apps_cppNN_CppNNUpdater_getModelParametersNative(JNIEnv* env, jobject, jint p) {
  return model_text(env, p, false);
}

JNIEXPORT jint JNICALL Java_apps_cppNN_CppNNUpdater_modelsSize(JNIEnv*, jobject) {
  std::lock_guard<std::mutex> lk(g_model_mu);
  return g_model ? fleet_model_count(g_model) : 0;
}
JNIEXPORT jint JNICALL Java_apps_cppNN_CppNNUpdater_getPriority(JNIEnv*, jobject) {
  std::lock_guard<std::mutex> lk(g_model_mu);
  return g_model ? fleet_model_get_priority(g_model) : 0;
}
JNIEXPORT void JNICALL Java_apps_cppNN_CppNNUpdater_setPriority(JNIEnv*, jobject, jint p) {
  std::lock_guard<std::mutex> lk(g_model_mu);
  if (g_model) fleet_model_set_priority(g_model, p);
}
JNIEXPORT jint JNICALL Java_apps_cppNN_CppNNUpdater_getCurrEpoch(JNIEnv*, jobject) {
  std::lock_guard<std::mutex> lk(g_model_mu);
  return g_model ? fleet_model_get_epoch(g_model) : 0;
}
JNIEXPORT void JNICALL Java_apps_cppNN_CppNNUpdater_setCurrEpoch(JNIEnv*, jobject, jint e) {
  std::lock_guard<std::mutex> lk(g_model_mu);
  if (g_model) fleet_model_set_epoch(g_model, e);
}
JNIEXPORT jdouble JNICALL Java_apps_cppNN_CppNNUpdater_getLrate(JNIEnv*, jobject) {
  std::lock_guard<std::mutex> lk(g_model_mu);
  return g_model ? fleet_model_get_lrate(g_model) : 0.0;
}

// getNumLabels / hasOutlier (:129-137): the sampler's globals (0 / the
// configured outlier flag before initSampler, like the zero-initialised globals)
JNIEXPORT jint JNICALL Java_apps_cppNN_CppNNUpdater_getNumLabels(JNIEnv*, jobject) {
  std::lock_guard<std::mutex> lk(g_sampler_mu);
  return g_sampler ? fleet_sampler_num_labels(g_sampler) : 0;
}
JNIEXPORT jboolean JNICALL Java_apps_cppNN_CppNNUpdater_hasOutlier(JNIEnv*, jobject) {
  return env_int("FLEET_SAMPLER_OUTLIER", 0) != 0 ? JNI_TRUE : JNI_FALSE;
}

// printParamsNative (:304-322): the upload's int32 codes on stdout
JNIEXPORT void JNICALL Java_apps_cppNN_CppNNUpdater_printParamsNative(JNIEnv* env, jobject, jbyteArray input) {
  fleet_ctx* c = ctx();
  if (!c || !input) return;
  Bytes in(env, input);
  if (!in.ok()) return;
  std::vector<int32_t> codes(fleet_b64_count((size_t)in.n) + 3);
  size_t n = 0;
  const int rc = fleet_decode_i32(c, in.data(), (size_t)in.n, codes.data(), codes.size(), &n);
  if (rc != FLEET_OK) {
    fail(c, "printParamsNative", rc);
    return;
  }
  std::string line = "Got Numbers: ";
  char buf[16];
  for (size_t i = 0; i < n; ++i) {
    std::snprintf(buf, sizeof buf, "%d ", codes[i]);
    line += buf;
  }
  std::printf("%s\n", line.c_str());
  std::fflush(stdout);
}

// ----------------------------------------------------------------- sampler

// the MNIST test set parse_test_data reads (mnist_parser.h:153-161: the two file-name spellings)
static bool mnist_test_set_present(const std::string& dir) {
  auto readable = [](const std::string& p) {
    FILE* f = std::fopen(p.c_str(), "rb");
    if (f) std::fclose(f);
    return f != nullptr;
  };
  return (readable(dir + "/t10k-images.idx3-ubyte") || readable(dir + "/t10k-images-idx3-ubyte")) &&
         (readable(dir + "/t10k-labels.idx1-ubyte") || readable(dir + "/t10k-labels-idx1-ubyte"));
}

// initSampler (:385-551) with the reference's source-edited globals taken from
// the environment (FLEET_SAMPLER_*); the dataset stays in this library. The
// sampler lock is held from the srand(seed) on, so its rand() draws (the bucket
// shuffles) cannot interleave with another thread's getMiniBatch / initUpdater.
JNIEXPORT void JNICALL Java_apps_cppNN_CppNNOfflineSampler_initSampler(JNIEnv* env, jobject, jstring prefix) {
  fleet_ctx* c = ctx();
  if (!c || !prefix) return;
  const int iid = env_int("FLEET_SAMPLER_IID", 0) != 0, outlier = env_int("FLEET_SAMPLER_OUTLIER", 0) != 0;
  const int clients = env_int("FLEET_SAMPLER_CLIENTS", 10), mode = distillation_mode();
  std::printf("IID: %d\nOutlier: %d\n", iid, outlier);
  std::fflush(stdout);
  const char* path = env->GetStringUTFChars(prefix, nullptr);
  if (!path) return;
  const std::string data_path(path);
  env->ReleaseStringUTFChars(prefix, path);
  std::lock_guard<std::mutex> lk(g_sampler_mu);
  fleet_sampler* s = nullptr;
  const int rc = fleet_sampler_create(c, data_path.c_str(), iid, outlier, clients, mode, kSeed, &s);
  if (rc != FLEET_OK) return;  // fleet_sampler_create printed the reason
  fleet_sampler_set_hyper(s, g_E, g_sigma, g_C);
  if (g_sampler) fleet_sampler_destroy(g_sampler);
  g_sampler = s;  // the buckets exist from here on, as the reference's globals do
  if (mode) {
    if (!mnist_test_set_present(data_path)) {  // :485: the early return, after the buckets
      std::fprintf(stderr, "error: could not parse test data.\n");
      return;
    }
    std::fprintf(stderr,
                 "[fleet] initSampler: the mode-1 teacher's training (:481-545) is not rebuilt%s\n",
                 iid ? "; iid mini-batches need its trained weights (FleetSampler.setTeacherNative)" : "");
  }
  std::printf("Train data size: %zu\n", fleet_sampler_num_samples(s));
  std::fflush(stdout);
}

// The mode-1 teacher's trained weights (initSampler's network: conv 5x5x8, conv
// 1x1x16, conv 5x5x48, softmax 10; fleet_teacher_weight_count / _bias_count floats in
// mojo's layer order), from a JVM that trained or loaded it. iid mini-batches then
// append its outputs at TEMPERATURE 2 (uniformSample :593-620, k_teacher_forward).
// False (and the reason on stderr) without a sampler or with the wrong sizes.
JNIEXPORT jboolean JNICALL Java_apps_cppNN_FleetSampler_setTeacherNative(JNIEnv* env, jobject, jfloatArray w,
                                                                         jfloatArray b) {
  if (!w || !b) return JNI_FALSE;
  const jsize nw = env->GetArrayLength(w), nb = env->GetArrayLength(b);
  std::vector<float> wv((size_t)std::max<jsize>(nw, 0)), bv((size_t)std::max<jsize>(nb, 0));
  if (nw > 0) env->GetFloatArrayRegion(w, 0, nw, wv.data());
  if (nb > 0) env->GetFloatArrayRegion(b, 0, nb, bv.data());
  std::lock_guard<std::mutex> lk(g_sampler_mu);
  if (!g_sampler) {
    std::fprintf(stderr, "[fleet] setTeacherNative: no sampler (initSampler failed or was not called)\n");
    return JNI_FALSE;
  }
  const int rc = fleet_sampler_set_teacher(g_sampler, wv.data(), wv.size(), bv.data(), bv.size());
  if (rc != FLEET_OK) {
    std::fprintf(stderr, "[fleet] setTeacherNative failed (%d): %s (expected %zu weights, %zu biases)\n", rc,
                 fleet_sampler_last_error(g_sampler), fleet_teacher_weight_count(), fleet_teacher_bias_count());
    return JNI_FALSE;
  }
  return JNI_TRUE;
}

// getMiniBatch (:677-699): batch_size * E samples of the current client, the
// header's learning rate from the updater's model (cnn.get_learning_rate(),
// moved along lrates by descentNative).
JNIEXPORT jbyteArray JNICALL Java_apps_cppNN_CppNNOfflineSampler_getMiniBatch(JNIEnv* env, jobject, jint batch_size) {
  float lr = 0.0f;
  {
    std::lock_guard<std::mutex> lk(g_model_mu);
    if (g_model) lr = (float)fleet_model_get_lrate(g_model);
  }
  std::lock_guard<std::mutex> lk(g_sampler_mu);
  if (!g_sampler) {
    std::fprintf(stderr, "[fleet] getMiniBatch: no sampler (initSampler failed or was not called)\n");
    return nullptr;
  }
  const size_t len = fleet_sampler_minibatch_len(g_sampler, batch_size);
  std::vector<char> out(len + 16);
  size_t n = 0;
  const int rc = fleet_sampler_minibatch(g_sampler, batch_size, lr, out.data(), out.size(), &n);
  if (rc != FLEET_OK) {
    std::fprintf(stderr, "[fleet] getMiniBatch failed (%d): %s\n", rc, fleet_sampler_last_error(g_sampler));
    return nullptr;
  }
  return to_java(env, out.data(), n);
}

}  // extern "C"
