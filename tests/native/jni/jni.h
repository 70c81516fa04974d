/*
 * tests/native/jni/jni.h -- TEST INFRASTRUCTURE ONLY.
 *
 * The JNI interface as the JNI specification lays it out, for building and
 * testing fleet_amd's OWN JNI shim (fleet_amd/csrc/jni_shim.cpp) in an image
 * without a JDK. It is ABI-shaped: JNIEnv is a pointer to a table of function
 * pointers (JNINativeInterface_) in the specification's slot order -- four
 * reserved slots, then GetVersion at index 4 ... GetModule at 233 -- and the
 * C++ JNIEnv_ forwards each call through that table, exactly as a JDK's
 * <jni.h> does. So the libfleet_native.so built against this header is the
 * binary a JVM's System.load would bind (the same symbol names, the same
 * calling convention, the same table offsets); tests/native/fakejvm.cpp
 * fills a table with a small in-process "JVM" (arrays, local references,
 * critical regions) that the shim's calls dispatch through.
 *
 * Slot types: the functions the shim and the fake JVM use carry their JNI
 * signatures; every other slot is a plain pointer of the same size, keeping
 * the offsets (checked by the static_asserts at the end).
 * On a server host the shim is built against the JDK's real <jni.h>
 * (JAVA_HOME; fleet_amd/build.py). Never used to compile reference sources.
 */
#ifndef FLEET_TEST_JNI_H
#define FLEET_TEST_JNI_H

#include <stdarg.h>
#include <stddef.h>
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNIIMPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef signed char jbyte;
typedef unsigned char jboolean;
typedef unsigned short jchar;
typedef short jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

#ifdef __cplusplus
class _jobject {};
class _jclass : public _jobject {};
class _jthrowable : public _jobject {};
class _jstring : public _jobject {};
class _jarray : public _jobject {};
class _jbooleanArray : public _jarray {};
class _jbyteArray : public _jarray {};
class _jcharArray : public _jarray {};
class _jshortArray : public _jarray {};
class _jintArray : public _jarray {};
class _jlongArray : public _jarray {};
class _jfloatArray : public _jarray {};
class _jdoubleArray : public _jarray {};
class _jobjectArray : public _jarray {};
typedef _jobject* jobject;
typedef _jclass* jclass;
typedef _jthrowable* jthrowable;
typedef _jstring* jstring;
typedef _jarray* jarray;
typedef _jbooleanArray* jbooleanArray;
typedef _jbyteArray* jbyteArray;
typedef _jcharArray* jcharArray;
typedef _jshortArray* jshortArray;
typedef _jintArray* jintArray;
typedef _jlongArray* jlongArray;
typedef _jfloatArray* jfloatArray;
typedef _jdoubleArray* jdoubleArray;
typedef _jobjectArray* jobjectArray;
#else
struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass, jthrowable, jstring, jarray, jbooleanArray, jbyteArray, jcharArray, jshortArray, jintArray,
    jlongArray, jfloatArray, jdoubleArray, jobjectArray;
#endif
typedef jobject jweak;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_OK 0
#define JNI_ERR (-1)
#define JNI_COMMIT 1
#define JNI_ABORT 2
#define JNI_VERSION_1_8 0x00010008

struct JNINativeInterface_;
#ifdef __cplusplus
struct JNIEnv_;
typedef JNIEnv_ JNIEnv;
#else
typedef const struct JNINativeInterface_* JNIEnv;
#endif

/* the function table, in the JNI specification's order (index in the comment) */
struct JNINativeInterface_ {
  void* reserved0;  /* 0 */
  void* reserved1;
  void* reserved2;
  void* reserved3;
  jint(JNICALL* GetVersion)(JNIEnv*); /* 4 */
  void* DefineClass;
  jclass(JNICALL* FindClass)(JNIEnv*, const char*); /* 6 */
  void* FromReflectedMethod;
  void* FromReflectedField;
  void* ToReflectedMethod;
  void* GetSuperclass; /* 10 */
  void* IsAssignableFrom;
  void* ToReflectedField;
  void* Throw;
  jint(JNICALL* ThrowNew)(JNIEnv*, jclass, const char*); /* 14 */
  void* ExceptionOccurred;
  void* ExceptionDescribe;
  void(JNICALL* ExceptionClear)(JNIEnv*); /* 17 */
  void* FatalError;
  jint(JNICALL* PushLocalFrame)(JNIEnv*, jint); /* 19 */
  jobject(JNICALL* PopLocalFrame)(JNIEnv*, jobject); /* 20 */
  void* NewGlobalRef;
  void* DeleteGlobalRef;
  void(JNICALL* DeleteLocalRef)(JNIEnv*, jobject); /* 23 */
  jboolean(JNICALL* IsSameObject)(JNIEnv*, jobject, jobject); /* 24 */
  void* NewLocalRef;
  jint(JNICALL* EnsureLocalCapacity)(JNIEnv*, jint); /* 26 */
  void* AllocObject;
  void* NewObject;
  void* NewObjectV;
  void* NewObjectA; /* 30 */
  void* GetObjectClass;
  void* IsInstanceOf;
  void* GetMethodID;
  void* CallObjectMethod; /* 34 */
  void* CallObjectMethodV;
  void* CallObjectMethodA;
  void* CallBooleanMethod;
  void* CallBooleanMethodV;
  void* CallBooleanMethodA;
  void* CallByteMethod; /* 40 */
  void* CallByteMethodV;
  void* CallByteMethodA;
  void* CallCharMethod;
  void* CallCharMethodV;
  void* CallCharMethodA;
  void* CallShortMethod;
  void* CallShortMethodV;
  void* CallShortMethodA;
  void* CallIntMethod;
  void* CallIntMethodV; /* 50 */
  void* CallIntMethodA;
  void* CallLongMethod;
  void* CallLongMethodV;
  void* CallLongMethodA;
  void* CallFloatMethod;
  void* CallFloatMethodV;
  void* CallFloatMethodA;
  void* CallDoubleMethod;
  void* CallDoubleMethodV;
  void* CallDoubleMethodA; /* 60 */
  void* CallVoidMethod;
  void* CallVoidMethodV;
  void* CallVoidMethodA;
  void* CallNonvirtualObjectMethod; /* 64 */
  void* CallNonvirtualObjectMethodV;
  void* CallNonvirtualObjectMethodA;
  void* CallNonvirtualBooleanMethod;
  void* CallNonvirtualBooleanMethodV;
  void* CallNonvirtualBooleanMethodA;
  void* CallNonvirtualByteMethod; /* 70 */
  void* CallNonvirtualByteMethodV;
  void* CallNonvirtualByteMethodA;
  void* CallNonvirtualCharMethod;
  void* CallNonvirtualCharMethodV;
  void* CallNonvirtualCharMethodA;
  void* CallNonvirtualShortMethod;
  void* CallNonvirtualShortMethodV;
  void* CallNonvirtualShortMethodA;
  void* CallNonvirtualIntMethod;
  void* CallNonvirtualIntMethodV; /* 80 */
  void* CallNonvirtualIntMethodA;
  void* CallNonvirtualLongMethod;
  void* CallNonvirtualLongMethodV;
  void* CallNonvirtualLongMethodA;
  void* CallNonvirtualFloatMethod;
  void* CallNonvirtualFloatMethodV;
  void* CallNonvirtualFloatMethodA;
  void* CallNonvirtualDoubleMethod;
  void* CallNonvirtualDoubleMethodV;
  void* CallNonvirtualDoubleMethodA; /* 90 */
  void* CallNonvirtualVoidMethod;
  void* CallNonvirtualVoidMethodV;
  void* CallNonvirtualVoidMethodA;
  void* GetFieldID; /* 94 */
  void* GetObjectField;
  void* GetBooleanField;
  void* GetByteField;
  void* GetCharField;
  void* GetShortField;
  void* GetIntField; /* 100 */
  void* GetLongField;
  void* GetFloatField;
  void* GetDoubleField;
  void* SetObjectField;
  void* SetBooleanField;
  void* SetByteField;
  void* SetCharField;
  void* SetShortField;
  void* SetIntField;
  void* SetLongField; /* 110 */
  void* SetFloatField;
  void* SetDoubleField;
  void* GetStaticMethodID;
  void* CallStaticObjectMethod; /* 114 */
  void* CallStaticObjectMethodV;
  void* CallStaticObjectMethodA;
  void* CallStaticBooleanMethod;
  void* CallStaticBooleanMethodV;
  void* CallStaticBooleanMethodA;
  void* CallStaticByteMethod; /* 120 */
  void* CallStaticByteMethodV;
  void* CallStaticByteMethodA;
  void* CallStaticCharMethod;
  void* CallStaticCharMethodV;
  void* CallStaticCharMethodA;
  void* CallStaticShortMethod;
  void* CallStaticShortMethodV;
  void* CallStaticShortMethodA;
  void* CallStaticIntMethod;
  void* CallStaticIntMethodV; /* 130 */
  void* CallStaticIntMethodA;
  void* CallStaticLongMethod;
  void* CallStaticLongMethodV;
  void* CallStaticLongMethodA;
  void* CallStaticFloatMethod;
  void* CallStaticFloatMethodV;
  void* CallStaticFloatMethodA;
  void* CallStaticDoubleMethod;
  void* CallStaticDoubleMethodV;
  void* CallStaticDoubleMethodA; /* 140 */
  void* CallStaticVoidMethod;
  void* CallStaticVoidMethodV;
  void* CallStaticVoidMethodA;
  void* GetStaticFieldID; /* 144 */
  void* GetStaticObjectField;
  void* GetStaticBooleanField;
  void* GetStaticByteField;
  void* GetStaticCharField;
  void* GetStaticShortField;
  void* GetStaticIntField; /* 150 */
  void* GetStaticLongField;
  void* GetStaticFloatField;
  void* GetStaticDoubleField;
  void* SetStaticObjectField;
  void* SetStaticBooleanField;
  void* SetStaticByteField;
  void* SetStaticCharField;
  void* SetStaticShortField;
  void* SetStaticIntField;
  void* SetStaticLongField; /* 160 */
  void* SetStaticFloatField;
  void* SetStaticDoubleField;
  void* NewString; /* 163 */
  void* GetStringLength;
  void* GetStringChars;
  void* ReleaseStringChars;
  void* NewStringUTF;
  void* GetStringUTFLength;
  const char*(JNICALL* GetStringUTFChars)(JNIEnv*, jstring, jboolean*); /* 169 */
  void(JNICALL* ReleaseStringUTFChars)(JNIEnv*, jstring, const char*); /* 170 */
  jsize(JNICALL* GetArrayLength)(JNIEnv*, jarray); /* 171 */
  void* NewObjectArray;
  jobject(JNICALL* GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize); /* 173 */
  void* SetObjectArrayElement;
  void* NewBooleanArray;
  jbyteArray(JNICALL* NewByteArray)(JNIEnv*, jsize); /* 176 */
  void* NewCharArray;
  void* NewShortArray;
  void* NewIntArray;
  void* NewLongArray; /* 180 */
  jfloatArray(JNICALL* NewFloatArray)(JNIEnv*, jsize); /* 181 */
  jdoubleArray(JNICALL* NewDoubleArray)(JNIEnv*, jsize); /* 182 */
  void* GetBooleanArrayElements;
  jbyte*(JNICALL* GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*); /* 184 */
  void* GetCharArrayElements;
  void* GetShortArrayElements;
  jint*(JNICALL* GetIntArrayElements)(JNIEnv*, jintArray, jboolean*); /* 187 */
  void* GetLongArrayElements;
  jfloat*(JNICALL* GetFloatArrayElements)(JNIEnv*, jfloatArray, jboolean*); /* 189 */
  jdouble*(JNICALL* GetDoubleArrayElements)(JNIEnv*, jdoubleArray, jboolean*); /* 190 */
  void* ReleaseBooleanArrayElements;
  void(JNICALL* ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint); /* 192 */
  void* ReleaseCharArrayElements;
  void* ReleaseShortArrayElements;
  void(JNICALL* ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint); /* 195 */
  void* ReleaseLongArrayElements;
  void(JNICALL* ReleaseFloatArrayElements)(JNIEnv*, jfloatArray, jfloat*, jint); /* 197 */
  void(JNICALL* ReleaseDoubleArrayElements)(JNIEnv*, jdoubleArray, jdouble*, jint); /* 198 */
  void* GetBooleanArrayRegion;
  void(JNICALL* GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*); /* 200 */
  void* GetCharArrayRegion;
  void* GetShortArrayRegion;
  void(JNICALL* GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*); /* 203 */
  void* GetLongArrayRegion;
  void(JNICALL* GetFloatArrayRegion)(JNIEnv*, jfloatArray, jsize, jsize, jfloat*); /* 205 */
  void(JNICALL* GetDoubleArrayRegion)(JNIEnv*, jdoubleArray, jsize, jsize, jdouble*); /* 206 */
  void* SetBooleanArrayRegion;
  void(JNICALL* SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*); /* 208 */
  void* SetCharArrayRegion;
  void* SetShortArrayRegion; /* 210 */
  void* SetIntArrayRegion;
  void* SetLongArrayRegion;
  void(JNICALL* SetFloatArrayRegion)(JNIEnv*, jfloatArray, jsize, jsize, const jfloat*); /* 213 */
  void(JNICALL* SetDoubleArrayRegion)(JNIEnv*, jdoubleArray, jsize, jsize, const jdouble*); /* 214 */
  void* RegisterNatives;
  void* UnregisterNatives;
  void* MonitorEnter;
  void* MonitorExit;
  void* GetJavaVM;
  void* GetStringRegion; /* 220 */
  void* GetStringUTFRegion;
  void*(JNICALL* GetPrimitiveArrayCritical)(JNIEnv*, jarray, jboolean*); /* 222 */
  void(JNICALL* ReleasePrimitiveArrayCritical)(JNIEnv*, jarray, void*, jint); /* 223 */
  void* GetStringCritical;
  void* ReleaseStringCritical;
  jweak(JNICALL* NewWeakGlobalRef)(JNIEnv*, jobject); /* 226 */
  void(JNICALL* DeleteWeakGlobalRef)(JNIEnv*, jweak); /* 227 */
  jboolean(JNICALL* ExceptionCheck)(JNIEnv*); /* 228 */
  jobject(JNICALL* NewDirectByteBuffer)(JNIEnv*, void*, jlong); /* 229 */
  void*(JNICALL* GetDirectBufferAddress)(JNIEnv*, jobject); /* 230 */
  jlong(JNICALL* GetDirectBufferCapacity)(JNIEnv*, jobject); /* 231 */
  void* GetObjectRefType;
  void* GetModule; /* 233 */
};

#ifdef __cplusplus
/* the C++ JNIEnv: the table pointer and inline forwarders (as in a JDK's jni.h) */
struct JNIEnv_ {
  const struct JNINativeInterface_* functions;
  jint GetVersion() { return functions->GetVersion(this); }
  jclass FindClass(const char* name) { return functions->FindClass(this, name); }
  jint ThrowNew(jclass c, const char* msg) { return functions->ThrowNew(this, c, msg); }
  void ExceptionClear() { functions->ExceptionClear(this); }
  jint PushLocalFrame(jint capacity) { return functions->PushLocalFrame(this, capacity); }
  jobject PopLocalFrame(jobject result) { return functions->PopLocalFrame(this, result); }
  void DeleteLocalRef(jobject o) { functions->DeleteLocalRef(this, o); }
  jboolean IsSameObject(jobject a, jobject b) { return functions->IsSameObject(this, a, b); }
  jweak NewWeakGlobalRef(jobject o) { return functions->NewWeakGlobalRef(this, o); }
  void DeleteWeakGlobalRef(jweak w) { functions->DeleteWeakGlobalRef(this, w); }
  jint EnsureLocalCapacity(jint capacity) { return functions->EnsureLocalCapacity(this, capacity); }
  const char* GetStringUTFChars(jstring s, jboolean* isCopy) { return functions->GetStringUTFChars(this, s, isCopy); }
  void ReleaseStringUTFChars(jstring s, const char* c) { functions->ReleaseStringUTFChars(this, s, c); }
  jsize GetArrayLength(jarray a) { return functions->GetArrayLength(this, a); }
  jobject GetObjectArrayElement(jobjectArray a, jsize i) { return functions->GetObjectArrayElement(this, a, i); }
  jbyteArray NewByteArray(jsize n) { return functions->NewByteArray(this, n); }
  jfloatArray NewFloatArray(jsize n) { return functions->NewFloatArray(this, n); }
  jdoubleArray NewDoubleArray(jsize n) { return functions->NewDoubleArray(this, n); }
  jbyte* GetByteArrayElements(jbyteArray a, jboolean* isCopy) { return functions->GetByteArrayElements(this, a, isCopy); }
  jint* GetIntArrayElements(jintArray a, jboolean* isCopy) { return functions->GetIntArrayElements(this, a, isCopy); }
  jfloat* GetFloatArrayElements(jfloatArray a, jboolean* isCopy) {
    return functions->GetFloatArrayElements(this, a, isCopy);
  }
  jdouble* GetDoubleArrayElements(jdoubleArray a, jboolean* isCopy) {
    return functions->GetDoubleArrayElements(this, a, isCopy);
  }
  void ReleaseByteArrayElements(jbyteArray a, jbyte* e, jint mode) { functions->ReleaseByteArrayElements(this, a, e, mode); }
  void ReleaseIntArrayElements(jintArray a, jint* e, jint mode) { functions->ReleaseIntArrayElements(this, a, e, mode); }
  void ReleaseFloatArrayElements(jfloatArray a, jfloat* e, jint mode) {
    functions->ReleaseFloatArrayElements(this, a, e, mode);
  }
  void ReleaseDoubleArrayElements(jdoubleArray a, jdouble* e, jint mode) {
    functions->ReleaseDoubleArrayElements(this, a, e, mode);
  }
  void GetByteArrayRegion(jbyteArray a, jsize s, jsize n, jbyte* buf) { functions->GetByteArrayRegion(this, a, s, n, buf); }
  void GetIntArrayRegion(jintArray a, jsize s, jsize n, jint* buf) { functions->GetIntArrayRegion(this, a, s, n, buf); }
  void GetFloatArrayRegion(jfloatArray a, jsize s, jsize n, jfloat* buf) {
    functions->GetFloatArrayRegion(this, a, s, n, buf);
  }
  void GetDoubleArrayRegion(jdoubleArray a, jsize s, jsize n, jdouble* buf) {
    functions->GetDoubleArrayRegion(this, a, s, n, buf);
  }
  void SetByteArrayRegion(jbyteArray a, jsize s, jsize n, const jbyte* buf) {
    functions->SetByteArrayRegion(this, a, s, n, buf);
  }
  void SetFloatArrayRegion(jfloatArray a, jsize s, jsize n, const jfloat* buf) {
    functions->SetFloatArrayRegion(this, a, s, n, buf);
  }
  void SetDoubleArrayRegion(jdoubleArray a, jsize s, jsize n, const jdouble* buf) {
    functions->SetDoubleArrayRegion(this, a, s, n, buf);
  }
  void* GetPrimitiveArrayCritical(jarray a, jboolean* isCopy) { return functions->GetPrimitiveArrayCritical(this, a, isCopy); }
  void ReleasePrimitiveArrayCritical(jarray a, void* p, jint mode) {
    functions->ReleasePrimitiveArrayCritical(this, a, p, mode);
  }
  jboolean ExceptionCheck() { return functions->ExceptionCheck(this); }
  jobject NewDirectByteBuffer(void* p, jlong cap) { return functions->NewDirectByteBuffer(this, p, cap); }
  void* GetDirectBufferAddress(jobject b) { return functions->GetDirectBufferAddress(this, b); }
  jlong GetDirectBufferCapacity(jobject b) { return functions->GetDirectBufferCapacity(this, b); }
};

static_assert(offsetof(JNINativeInterface_, GetVersion) == 4 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, DeleteLocalRef) == 23 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, IsSameObject) == 24 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, EnsureLocalCapacity) == 26 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, GetArrayLength) == 171 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, NewByteArray) == 176 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, GetByteArrayElements) == 184 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, ReleaseDoubleArrayElements) == 198 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, SetByteArrayRegion) == 208 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, GetPrimitiveArrayCritical) == 222 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, NewWeakGlobalRef) == 226 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, ExceptionCheck) == 228 * sizeof(void*), "JNI table layout");
static_assert(offsetof(JNINativeInterface_, GetDirectBufferCapacity) == 231 * sizeof(void*), "JNI table layout");
static_assert(sizeof(JNINativeInterface_) == 234 * sizeof(void*), "JNI table size (JNI 9+)");
#endif

#endif
