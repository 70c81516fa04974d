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
// and the batched natives of an updater that makes one call per update:
//   byte[] apps.cppNN.FleetUpdater.aggregateNative(byte[][] uploads, double[] dampen)
//   byte[] apps.cppNN.FleetUpdater.aggregateDirectNative(ByteBuffer rows, int M, int len, int rowPitch,
//                                                          double[] dampen)
//   boolean apps.cppNN.FleetUpdater.registerDirectNative(ByteBuffer rows)
// The sampler's natives (initSampler / getMiniBatch, dataset loading) stay in
// the reference's libnative.so (load order, learning-rate note).
//
// Environment: FLEET_GPUS = devices the batched natives spread one update over
// (element sharding, fleet_update_multi; default 1, "all" = every visible GPU);
// FLEET_DISTILLATION_MODE = the reference's compile-time DISTILLATION_MODE (default 1).
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
fleet_model* g_model = nullptr;
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
  const int rc = fleet_host_register(c, p, (size_t)cap);
  if (rc != FLEET_OK) fail(c, "registerDirectNative", rc);
  return rc == FLEET_OK ? JNI_TRUE : JNI_FALSE;
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
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_model) fleet_model_destroy(g_model);
  g_model = m;
}

JNIEXPORT void JNICALL Java_apps_cppNN_CppNNUpdater_initUpdater(JNIEnv* env, jobject, jdoubleArray lrates, jint E,
                                                                jdouble sigma, jdouble C) {
  (void)E, (void)sigma, (void)C;  // the sampler's mini-batch header values (libnative.so keeps them)
  if (!g_model || !lrates) return;
  const jsize n = env->GetArrayLength(lrates);
  std::vector<double> lr((size_t)std::max<jsize>(n, 0));
  if (n > 0) env->GetDoubleArrayRegion(lrates, 0, n, lr.data());
  const int rc = fleet_model_init_updater(g_model, lr.data(), (int)n);
  if (rc != FLEET_OK) mfail("initUpdater", rc);
}

JNIEXPORT void JNICALL Java_apps_cppNN_CppNNUpdater_descentNative(JNIEnv* env, jobject, jbyteArray input,
                                                                  jint clientBatchSize, jint staleSize) {
  if (!g_model || !input) return;
  Bytes in(env, input);
  if (!in.ok()) return;
  const int rc = fleet_model_descent(g_model, in.data(), (size_t)in.n, clientBatchSize, staleSize);
  if (rc != FLEET_OK) mfail("descentNative", rc);
}

static jbyteArray model_text(JNIEnv* env, jint p, bool params) {
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
  return g_model ? fleet_model_count(g_model) : 0;
}
JNIEXPORT jint JNICALL Java_apps_cppNN_CppNNUpdater_getPriority(JNIEnv*, jobject) {
  return g_model ? fleet_model_get_priority(g_model) : 0;
}
JNIEXPORT void JNICALL Java_apps_cppNN_CppNNUpdater_setPriority(JNIEnv*, jobject, jint p) {
  if (g_model) fleet_model_set_priority(g_model, p);
}
JNIEXPORT jint JNICALL Java_apps_cppNN_CppNNUpdater_getCurrEpoch(JNIEnv*, jobject) {
  return g_model ? fleet_model_get_epoch(g_model) : 0;
}
JNIEXPORT void JNICALL Java_apps_cppNN_CppNNUpdater_setCurrEpoch(JNIEnv*, jobject, jint e) {
  if (g_model) fleet_model_set_epoch(g_model, e);
}
JNIEXPORT jdouble JNICALL Java_apps_cppNN_CppNNUpdater_getLrate(JNIEnv*, jobject) {
  return g_model ? fleet_model_get_lrate(g_model) : 0.0;
}

}  // extern "C"
