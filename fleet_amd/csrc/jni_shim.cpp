// fleet_amd/csrc/jni_shim.cpp -- JNI shim: the reference's native symbol names
// on top of the C-ABI (include/fleet_codec.h). Built as libfleet_native.so.
//
// Drop-in for the hot-path natives of the reference's server backend
// (Server/src/main/c++/cppNN_backend.cpp, loaded as libnative.so by
// commonLib/utils/JNITest.java:22-53):
//   Java_apps_cppNN_CppNNUpdater_getFlatGradient     cppNN_backend.cpp:701-720
//   Java_apps_cppNN_CppNNUpdater_mergeFlatGradient   cppNN_backend.cpp:722-750
//   Java_utils_ByteVec_scalarMulNative               cppNN_backend.cpp:753-777
//   Java_utils_ByteVec_getNorm                       cppNN_backend.cpp:779-795
//   Java_utils_ByteVec_addNative                     cppNN_backend.cpp:797-846
//   Java_utils_ByteVec_subtractNative                cppNN_backend.cpp:848-892
// and one batched native for an updater that makes a single call per update
// (INTEGRATION.md):
//   byte[] apps.cppNN.FleetUpdater.aggregateNative(byte[][] uploads, double[] dampen)
// Model-side natives (descentNative, getParametersNative, initUpdater, ...)
// stay in the reference's libnative.so.
//
// Same argument meaning and results as the reference; failures return null
// (Java sees a NullPointerException at the caller) and print the C-ABI error
// on stderr -- the reference has no error path at all.
#include <jni.h>

#include <cstdio>
#include <mutex>
#include <vector>

#include "fleet_codec.h"

namespace {

std::mutex g_mu;
fleet_ctx* g_ctx = nullptr;

fleet_ctx* ctx() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_ctx) {
    int rc = fleet_create(0, &g_ctx);
    if (rc != FLEET_OK) {
      std::fprintf(stderr, "[fleet] fleet_create failed (%d): no MI355X visible\n", rc);
      g_ctx = nullptr;
    }
  }
  return g_ctx;
}

// JVM byte[] -> host bytes (no NUL terminator needed: lengths are explicit)
struct Bytes {
  JNIEnv* env;
  jbyteArray arr;
  jbyte* p;
  jsize n;
  Bytes(JNIEnv* e, jbyteArray a) : env(e), arr(a), p(e->GetByteArrayElements(a, nullptr)), n(e->GetArrayLength(a)) {}
  ~Bytes() { env->ReleaseByteArrayElements(arr, p, 2 /* JNI_ABORT: no copy-back */); }
  const char* data() const { return reinterpret_cast<const char*>(p); }
};

jbyteArray to_java(JNIEnv* env, const std::vector<char>& v, size_t n) {
  jbyteArray a = env->NewByteArray((jsize)n);
  env->SetByteArrayRegion(a, 0, (jsize)n, reinterpret_cast<const jbyte*>(v.data()));
  return a;
}

jbyteArray fail(fleet_ctx* c, const char* what, int rc) {
  std::fprintf(stderr, "[fleet] %s failed (%d): %s\n", what, rc, c ? fleet_last_error(c) : "no context");
  return nullptr;
}

}  // namespace

extern "C" {

JNIEXPORT jbyteArray JNICALL Java_apps_cppNN_CppNNUpdater_getFlatGradient(JNIEnv* env, jobject, jbyteArray input) {
  fleet_ctx* c = ctx();
  if (!c) return nullptr;
  Bytes in(env, input);
  std::vector<char> out((size_t)in.n + 16);
  size_t n = 0;
  int rc = fleet_flat_gradient(c, in.data(), (size_t)in.n, out.data(), out.size(), &n);
  return rc == FLEET_OK ? to_java(env, out, n) : fail(c, "getFlatGradient", rc);
}

JNIEXPORT jbyteArray JNICALL Java_apps_cppNN_CppNNUpdater_mergeFlatGradient(JNIEnv* env, jobject, jbyteArray g,
                                                                            jbyteArray flatG) {
  fleet_ctx* c = ctx();
  if (!c) return nullptr;
  Bytes a(env, g), b(env, flatG);
  std::vector<char> out((size_t)a.n + 16);
  size_t n = 0;
  int rc = fleet_merge_flat_gradient(c, a.data(), (size_t)a.n, b.data(), (size_t)b.n, out.data(), out.size(), &n);
  return rc == FLEET_OK ? to_java(env, out, n) : fail(c, "mergeFlatGradient", rc);
}

JNIEXPORT jbyteArray JNICALL Java_utils_ByteVec_scalarMulNative(JNIEnv* env, jobject, jbyteArray input, jdouble a) {
  fleet_ctx* c = ctx();
  if (!c) return nullptr;
  Bytes in(env, input);
  std::vector<char> out((size_t)in.n + 16);
  size_t n = 0;
  int rc = fleet_scalar_mul(c, in.data(), (size_t)in.n, (double)a, out.data(), out.size(), &n);
  return rc == FLEET_OK ? to_java(env, out, n) : fail(c, "scalarMulNative", rc);
}

JNIEXPORT jdouble JNICALL Java_utils_ByteVec_getNorm(JNIEnv* env, jobject, jbyteArray input) {
  fleet_ctx* c = ctx();
  if (!c) return 0.0;
  Bytes in(env, input);
  double r = 0.0;
  int rc = fleet_norm(c, in.data(), (size_t)in.n, &r);
  if (rc != FLEET_OK) fail(c, "getNorm", rc);
  return r;
}

static jbyteArray binop(JNIEnv* env, jbyteArray a, jbyteArray b, bool sub) {
  fleet_ctx* c = ctx();
  if (!c) return nullptr;
  Bytes x(env, a), y(env, b);
  std::vector<char> out((size_t)x.n + 16);
  size_t n = 0;
  int rc = sub ? fleet_subtract(c, x.data(), (size_t)x.n, y.data(), (size_t)y.n, out.data(), out.size(), &n)
               : fleet_add(c, x.data(), (size_t)x.n, y.data(), (size_t)y.n, out.data(), out.size(), &n);
  return rc == FLEET_OK ? to_java(env, out, n) : fail(c, sub ? "subtractNative" : "addNative", rc);
}

JNIEXPORT jbyteArray JNICALL Java_utils_ByteVec_addNative(JNIEnv* env, jobject, jbyteArray a, jbyteArray b) {
  return binop(env, a, b, false);
}

JNIEXPORT jbyteArray JNICALL Java_utils_ByteVec_subtractNative(JNIEnv* env, jobject, jbyteArray a, jbyteArray b) {
  return binop(env, a, b, true);
}

// The batched update: CppNNUpdater.java:420-509's getFlatGradient/scalarMultiply/
// add/scalarMultiply(1/M)/mergeFlatGradient chain in one device call.
JNIEXPORT jbyteArray JNICALL Java_apps_cppNN_FleetUpdater_aggregateNative(JNIEnv* env, jobject, jobjectArray uploads,
                                                                          jdoubleArray dampen) {
  fleet_ctx* c = ctx();
  if (!c) return nullptr;
  const jsize M = env->GetArrayLength(uploads);
  if (M <= 0 || env->GetArrayLength(dampen) != M) return fail(c, "aggregateNative (argument sizes)", FLEET_ERR_ARG);
  std::vector<jbyteArray> arrs((size_t)M);
  std::vector<jbyte*> ptrs((size_t)M);
  std::vector<const char*> cp((size_t)M);
  std::vector<size_t> lens((size_t)M);
  for (jsize i = 0; i < M; ++i) {
    arrs[i] = (jbyteArray)env->GetObjectArrayElement(uploads, i);
    ptrs[i] = env->GetByteArrayElements(arrs[i], nullptr);
    cp[i] = reinterpret_cast<const char*>(ptrs[i]);
    lens[i] = (size_t)env->GetArrayLength(arrs[i]);
  }
  jdouble* d = env->GetDoubleArrayElements(dampen, nullptr);
  std::vector<char> out(lens[0] + 16);
  size_t n = 0;
  int rc = fleet_update(c, cp.data(), lens.data(), (int)M, d, out.data(), out.size(), &n, nullptr);
  env->ReleaseDoubleArrayElements(dampen, d, 2);
  for (jsize i = 0; i < M; ++i) env->ReleaseByteArrayElements(arrs[i], ptrs[i], 2);
  return rc == FLEET_OK ? to_java(env, out, n) : fail(c, "aggregateNative", rc);
}

}  // extern "C"
