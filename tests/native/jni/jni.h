/*
 * tests/native/jni/jni.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A minimal JNI surface for building and testing fleet_amd's OWN JNI shim
 * (fleet_amd/csrc/jni_shim.cpp) in an image without a JDK: tests/jnifake.py
 * drives the shim's Java_* exports through it. It is never used to compile
 * reference sources. On a server host the shim is built against the JDK's
 * real <jni.h> (JAVA_HOME; fleet_amd/build.py).
 *
 * Arrays are heap blocks {len, payload}. GetByteArrayElements hands out a
 * NUL-terminated copy, so callers that read a byte[] as a C string (as the
 * reference's natives do) see a terminated buffer.
 */
#ifndef FLEET_ORACLE_FAKE_JNI_H
#define FLEET_ORACLE_FAKE_JNI_H

#include <cstdint>
#include <cstdlib>
#include <cstring>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int8_t jbyte;
typedef int32_t jint;
typedef int32_t jsize;
typedef int64_t jlong;
typedef double jdouble;
typedef float jfloat;
typedef uint8_t jboolean;

struct _jobject {};
typedef _jobject* jobject;

struct fake_jarray_hdr {
  jsize len;
  jsize elem;
};

struct _jbyteArray : _jobject {};
struct _jdoubleArray : _jobject {};
struct _jobjectArray : _jobject {};
struct _jstring : _jobject {};
typedef _jbyteArray* jbyteArray;
typedef _jdoubleArray* jdoubleArray;
typedef _jobjectArray* jobjectArray;
typedef _jstring* jstring;
typedef _jobject* jarray;

namespace fakejni {
inline fake_jarray_hdr* hdr(const void* a) { return (fake_jarray_hdr*)a; }
inline char* payload(const void* a) { return (char*)a + sizeof(fake_jarray_hdr); }
inline void* alloc(jsize len, jsize elem) {
  char* p = (char*)std::calloc(1, sizeof(fake_jarray_hdr) + (size_t)len * elem + 1);
  hdr(p)->len = len;
  hdr(p)->elem = elem;
  return p;
}
}  // namespace fakejni

struct JNIEnv {
  jsize GetArrayLength(const void* a) { return fakejni::hdr(a)->len; }

  jbyte* GetByteArrayElements(jbyteArray a, jboolean*) {
    jsize n = fakejni::hdr(a)->len;
    jbyte* c = (jbyte*)std::malloc((size_t)n + 1);
    std::memcpy(c, fakejni::payload(a), (size_t)n);
    c[n] = 0;
    return c;
  }
  void ReleaseByteArrayElements(jbyteArray a, jbyte* c, jint mode) {
    if (mode == 0) std::memcpy(fakejni::payload(a), c, (size_t)fakejni::hdr(a)->len);
    std::free(c);
  }
  jbyteArray NewByteArray(jsize n) { return (jbyteArray)fakejni::alloc(n, 1); }
  void SetByteArrayRegion(jbyteArray a, jsize start, jsize n, const jbyte* src) {
    std::memcpy(fakejni::payload(a) + start, src, (size_t)n);
  }
  jdouble* GetDoubleArrayElements(jdoubleArray a, jboolean*) {
    return (jdouble*)fakejni::payload(a);
  }
  void ReleaseDoubleArrayElements(jdoubleArray, jdouble*, jint) {}
  jobject GetObjectArrayElement(jobjectArray a, jsize i) { return ((jobject*)fakejni::payload(a))[i]; }
  const char* GetStringUTFChars(jstring s, jboolean*) { return fakejni::payload(s); }
  void ReleaseStringUTFChars(jstring, const char*) {}
  void DeleteLocalRef(void*) {}
};

#endif
