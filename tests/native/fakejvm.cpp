// tests/native/fakejvm.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A small in-process stand-in for a JVM's JNI function table (the ABI of
// tests/native/jni/jni.h, the JNI specification's slot order), so the JNI shim
// (fleet_amd/csrc/jni_shim.cpp, libfleet_native.so) can be driven and checked
// through the same table dispatch a JVM would use. It also enforces the JNI
// rules the shim must follow and counts violations:
//   * local references: 16 guaranteed per native frame; every reference a
//     call creates (GetObjectArrayElement, New*Array) beyond the capacity
//     secured with EnsureLocalCapacity / PushLocalFrame is an overflow;
//   * critical regions: no JNI call other than Get/ReleasePrimitiveArrayCritical
//     between them;
//   * Get<Type>ArrayElements hands out copies (as HotSpot does) that must be
//     released; outstanding ones are reported as leaked pins;
//   * an optional limit on EnsureLocalCapacity / PushLocalFrame simulates a
//     JVM that cannot grant a large frame (OutOfMemoryError pending);
//   * weak global references: fakejvm_collect(obj) plays the garbage collector
//     (a weak reference to a collected object then IsSameObject-equals NULL);
//     live weak references are counted.
// Built by tests/jnifake.py with g++ (no JDK exists in the image).
#include <jni.h>

#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

namespace {

enum Kind { BYTES = 1, INTS, FLOATS, DOUBLES, OBJECTS, DIRECT, STRING, CLASS, WEAK };

struct Obj {
  int kind;
  jsize len;
  int elem;
  std::vector<char> data;  // primitive payload
  std::vector<Obj*> objs;  // object array elements
  void* direct = nullptr;  // direct buffer
  jlong cap = 0;
  bool collected = false;  // fakejvm_collect: only weak references may still name it
  Obj* target = nullptr;   // WEAK: the referent
};

struct Frame {
  jint cap;
  std::vector<Obj*> refs;  // local references created in this frame
};

struct State {
  std::vector<Frame> frames;
  long overflows = 0, critical_violations = 0, pins = 0, criticals = 0, max_live = 0, exceptions = 0, weak = 0;
  long frame_limit = 1L << 30;
  int critical_depth = 0;
  bool pending = false;
} g;

long live() { return g.frames.empty() ? 0 : (long)g.frames.back().refs.size(); }

void new_local(Obj* o) {
  if (g.frames.empty()) g.frames.push_back(Frame{16, {}});
  Frame& f = g.frames.back();
  f.refs.push_back(o);
  if ((long)f.refs.size() > f.cap) g.overflows++;
  if (live() > g.max_live) g.max_live = live();
}

void jni_call() {
  if (g.critical_depth > 0) g.critical_violations++;
}

Obj* O(const void* p) { return (Obj*)p; }

Obj* make(int kind, jsize len, int elem) {
  Obj* o = new Obj();
  o->kind = kind;
  o->len = len;
  o->elem = elem;
  o->data.assign((size_t)len * (size_t)elem + 1, 0);
  return o;
}

void raise() {
  g.pending = true;
  g.exceptions++;
}

jint JNICALL GetVersion(JNIEnv*) {
  jni_call();
  return JNI_VERSION_1_8;
}
jclass JNICALL FindClass(JNIEnv*, const char*) {
  jni_call();
  Obj* o = make(CLASS, 0, 1);
  new_local(o);
  return (jclass)o;
}
jint JNICALL ThrowNew(JNIEnv*, jclass, const char*) {
  jni_call();
  raise();
  return 0;
}
void JNICALL ExceptionClear(JNIEnv*) {
  jni_call();
  g.pending = false;
}
jboolean JNICALL ExceptionCheck(JNIEnv*) {
  jni_call();
  return g.pending ? JNI_TRUE : JNI_FALSE;
}
jint JNICALL PushLocalFrame(JNIEnv*, jint cap) {
  jni_call();
  if (cap > g.frame_limit) {
    raise();
    return JNI_ERR;
  }
  g.frames.push_back(Frame{cap < 16 ? 16 : cap, {}});
  return JNI_OK;
}
jobject JNICALL PopLocalFrame(JNIEnv*, jobject result) {
  jni_call();
  if (g.frames.size() > 1) g.frames.pop_back();
  if (result) new_local(O(result));
  return result;
}
void JNICALL DeleteLocalRef(JNIEnv*, jobject o) {
  jni_call();
  if (g.frames.empty() || !o) return;
  auto& r = g.frames.back().refs;
  for (size_t i = r.size(); i-- > 0;)
    if (r[i] == O(o)) {
      r.erase(r.begin() + (long)i);
      return;
    }
}
jint JNICALL EnsureLocalCapacity(JNIEnv*, jint n) {
  jni_call();
  if (n > g.frame_limit) {
    raise();
    return JNI_ERR;
  }
  if (g.frames.empty()) g.frames.push_back(Frame{16, {}});
  Frame& f = g.frames.back();
  if ((long)f.refs.size() + n > f.cap) f.cap = (jint)(f.refs.size() + (size_t)n);
  return JNI_OK;
}
const char* JNICALL GetStringUTFChars(JNIEnv*, jstring s, jboolean* c) {
  jni_call();
  if (c) *c = JNI_FALSE;
  return O(s)->data.data();
}
void JNICALL ReleaseStringUTFChars(JNIEnv*, jstring, const char*) { jni_call(); }
jsize JNICALL GetArrayLength(JNIEnv*, jarray a) {
  jni_call();
  return O(a)->len;
}
jobject JNICALL GetObjectArrayElement(JNIEnv*, jobjectArray a, jsize i) {
  jni_call();
  Obj* o = O(a);
  if (i < 0 || i >= o->len) {
    raise();
    return nullptr;
  }
  Obj* e = o->objs[(size_t)i];
  if (e) new_local(e);
  return (jobject)e;
}
template <int K, int E, class R>
R JNICALL NewArray(JNIEnv*, jsize n) {
  jni_call();
  Obj* o = make(K, n, E);
  new_local(o);
  return (R)o;
}
template <class T>
T* JNICALL GetElements(JNIEnv*, jarray a, jboolean* isCopy) {
  jni_call();
  Obj* o = O(a);
  T* c = (T*)std::malloc((size_t)o->len * sizeof(T) + 1);
  std::memcpy(c, o->data.data(), (size_t)o->len * sizeof(T));
  if (isCopy) *isCopy = JNI_TRUE;
  g.pins++;
  return c;
}
template <class T>
void JNICALL ReleaseElements(JNIEnv*, jarray a, T* e, jint mode) {
  jni_call();
  if (mode != JNI_ABORT) std::memcpy(O(a)->data.data(), e, (size_t)O(a)->len * sizeof(T));
  if (mode != JNI_COMMIT) {
    std::free(e);
    g.pins--;
  }
}
template <class T>
void JNICALL GetRegion(JNIEnv*, jarray a, jsize s, jsize n, T* buf) {
  jni_call();
  Obj* o = O(a);
  if (s < 0 || n < 0 || s + n > o->len) {
    raise();
    return;
  }
  std::memcpy(buf, o->data.data() + (size_t)s * sizeof(T), (size_t)n * sizeof(T));
}
template <class T>
void JNICALL SetRegion(JNIEnv*, jarray a, jsize s, jsize n, const T* buf) {
  jni_call();
  Obj* o = O(a);
  if (s < 0 || n < 0 || s + n > o->len) {
    raise();
    return;
  }
  std::memcpy(o->data.data() + (size_t)s * sizeof(T), buf, (size_t)n * sizeof(T));
}
void* JNICALL GetPrimitiveArrayCritical(JNIEnv*, jarray a, jboolean* isCopy) {
  g.critical_depth++;
  g.criticals++;
  if (isCopy) *isCopy = JNI_FALSE;
  return O(a)->data.data();
}
void JNICALL ReleasePrimitiveArrayCritical(JNIEnv*, jarray, void*, jint) {
  if (g.critical_depth > 0) g.critical_depth--;
}
jobject JNICALL NewDirectByteBuffer(JNIEnv*, void* p, jlong cap) {
  jni_call();
  Obj* o = make(DIRECT, 0, 1);
  o->direct = p;
  o->cap = cap;
  new_local(o);
  return (jobject)o;
}
void* JNICALL GetDirectBufferAddress(JNIEnv*, jobject b) {
  jni_call();
  return O(b)->kind == DIRECT ? O(b)->direct : nullptr;
}
jlong JNICALL GetDirectBufferCapacity(JNIEnv*, jobject b) {
  jni_call();
  return O(b)->kind == DIRECT ? O(b)->cap : -1;
}
// a reference resolved to its object: a weak one to its referent, NULL once collected
Obj* resolve(jobject r) {
  Obj* o = O(r);
  if (o && o->kind == WEAK) o = o->target;
  return o && o->collected ? nullptr : o;
}
jboolean JNICALL IsSameObject(JNIEnv*, jobject a, jobject b) {
  jni_call();
  return resolve(a) == resolve(b) ? JNI_TRUE : JNI_FALSE;
}
jweak JNICALL NewWeakGlobalRef(JNIEnv*, jobject r) {
  jni_call();
  Obj* t = resolve(r);
  if (!t) return nullptr;
  Obj* w = make(WEAK, 0, 1);
  w->target = t;
  g.weak++;
  return (jweak)w;
}
void JNICALL DeleteWeakGlobalRef(JNIEnv*, jweak w) {
  jni_call();
  if (w && O(w)->kind == WEAK) {
    delete O(w);
    g.weak--;
  }
}

JNINativeInterface_ make_table() {
  JNINativeInterface_ t;
  std::memset(&t, 0, sizeof t);
  t.GetVersion = GetVersion;
  t.FindClass = FindClass;
  t.ThrowNew = ThrowNew;
  t.ExceptionClear = ExceptionClear;
  t.ExceptionCheck = ExceptionCheck;
  t.PushLocalFrame = PushLocalFrame;
  t.PopLocalFrame = PopLocalFrame;
  t.DeleteLocalRef = DeleteLocalRef;
  t.EnsureLocalCapacity = EnsureLocalCapacity;
  t.GetStringUTFChars = GetStringUTFChars;
  t.ReleaseStringUTFChars = ReleaseStringUTFChars;
  t.GetArrayLength = GetArrayLength;
  t.GetObjectArrayElement = GetObjectArrayElement;
  t.NewByteArray = NewArray<BYTES, 1, jbyteArray>;
  t.NewFloatArray = NewArray<FLOATS, 4, jfloatArray>;
  t.NewDoubleArray = NewArray<DOUBLES, 8, jdoubleArray>;
  t.GetByteArrayElements = (jbyte * (JNICALL*)(JNIEnv*, jbyteArray, jboolean*)) GetElements<jbyte>;
  t.GetIntArrayElements = (jint * (JNICALL*)(JNIEnv*, jintArray, jboolean*)) GetElements<jint>;
  t.GetFloatArrayElements = (jfloat * (JNICALL*)(JNIEnv*, jfloatArray, jboolean*)) GetElements<jfloat>;
  t.GetDoubleArrayElements = (jdouble * (JNICALL*)(JNIEnv*, jdoubleArray, jboolean*)) GetElements<jdouble>;
  t.ReleaseByteArrayElements = (void(JNICALL*)(JNIEnv*, jbyteArray, jbyte*, jint))ReleaseElements<jbyte>;
  t.ReleaseIntArrayElements = (void(JNICALL*)(JNIEnv*, jintArray, jint*, jint))ReleaseElements<jint>;
  t.ReleaseFloatArrayElements = (void(JNICALL*)(JNIEnv*, jfloatArray, jfloat*, jint))ReleaseElements<jfloat>;
  t.ReleaseDoubleArrayElements = (void(JNICALL*)(JNIEnv*, jdoubleArray, jdouble*, jint))ReleaseElements<jdouble>;
  t.GetByteArrayRegion = (void(JNICALL*)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*))GetRegion<jbyte>;
  t.GetIntArrayRegion = (void(JNICALL*)(JNIEnv*, jintArray, jsize, jsize, jint*))GetRegion<jint>;
  t.GetFloatArrayRegion = (void(JNICALL*)(JNIEnv*, jfloatArray, jsize, jsize, jfloat*))GetRegion<jfloat>;
  t.GetDoubleArrayRegion = (void(JNICALL*)(JNIEnv*, jdoubleArray, jsize, jsize, jdouble*))GetRegion<jdouble>;
  t.SetByteArrayRegion = (void(JNICALL*)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*))SetRegion<jbyte>;
  t.SetFloatArrayRegion = (void(JNICALL*)(JNIEnv*, jfloatArray, jsize, jsize, const jfloat*))SetRegion<jfloat>;
  t.SetDoubleArrayRegion = (void(JNICALL*)(JNIEnv*, jdoubleArray, jsize, jsize, const jdouble*))SetRegion<jdouble>;
  t.GetPrimitiveArrayCritical = GetPrimitiveArrayCritical;
  t.ReleasePrimitiveArrayCritical = ReleasePrimitiveArrayCritical;
  t.IsSameObject = IsSameObject;
  t.NewWeakGlobalRef = NewWeakGlobalRef;
  t.DeleteWeakGlobalRef = DeleteWeakGlobalRef;
  t.NewDirectByteBuffer = NewDirectByteBuffer;
  t.GetDirectBufferAddress = GetDirectBufferAddress;
  t.GetDirectBufferCapacity = GetDirectBufferCapacity;
  return t;
}

const JNINativeInterface_ g_table = make_table();
JNIEnv_ g_env{&g_table};

}  // namespace

extern "C" {

__attribute__((visibility("default"))) JNIEnv* fakejvm_env() { return &g_env; }

// a new native-method frame (the refs the caller passes in are its arguments)
__attribute__((visibility("default"))) void fakejvm_begin_call() {
  g.frames.clear();
  g.frames.push_back(Frame{16, {}});
  g.overflows = g.critical_violations = g.criticals = g.max_live = 0;
  g.critical_depth = 0;
  g.pending = false;
}

__attribute__((visibility("default"))) long fakejvm_stat(const char* what) {
  if (!std::strcmp(what, "overflows")) return g.overflows;
  if (!std::strcmp(what, "critical_violations")) return g.critical_violations;
  if (!std::strcmp(what, "criticals")) return g.criticals;
  if (!std::strcmp(what, "critical_depth")) return g.critical_depth;
  if (!std::strcmp(what, "pins")) return g.pins;
  if (!std::strcmp(what, "weak")) return g.weak;
  if (!std::strcmp(what, "live")) return live();
  if (!std::strcmp(what, "max_live")) return g.max_live;
  if (!std::strcmp(what, "pending")) return g.pending ? 1 : 0;
  return -1;
}

// the largest EnsureLocalCapacity / PushLocalFrame request granted
__attribute__((visibility("default"))) void fakejvm_set_frame_limit(long n) { g.frame_limit = n; }

// kind: 1 byte[], 2 int[], 3 float[], 4 double[]; data = n elements
__attribute__((visibility("default"))) void* fakejvm_new_array(int kind, const void* data, int n) {
  static const int elem[] = {0, 1, 4, 4, 8};
  if (kind < 1 || kind > 4) return nullptr;
  Obj* o = make(kind, n, elem[kind]);
  if (data && n) std::memcpy(o->data.data(), data, (size_t)n * (size_t)elem[kind]);
  return o;
}

__attribute__((visibility("default"))) void* fakejvm_new_object_array(void* const* elems, int n) {
  Obj* o = make(OBJECTS, n, (int)sizeof(void*));
  for (int i = 0; i < n; ++i) o->objs.push_back(O(elems[i]));
  return o;
}

__attribute__((visibility("default"))) void* fakejvm_new_direct(void* p, long cap) {
  Obj* o = make(DIRECT, 0, 1);
  o->direct = p;
  o->cap = cap;
  return o;
}

// the garbage collector reclaims `obj` (the test dropped its last strong reference):
// weak references to it now equal NULL; its memory is kept (handles stay readable)
__attribute__((visibility("default"))) void fakejvm_collect(void* obj) {
  if (obj) O(obj)->collected = true;
}

// a java.lang.String (modified UTF-8 = the bytes given, NUL-terminated)
__attribute__((visibility("default"))) void* fakejvm_new_string(const char* utf) {
  const jsize n = (jsize)std::strlen(utf);
  Obj* o = make(STRING, n, 1);
  std::memcpy(o->data.data(), utf, (size_t)n);
  return o;
}

__attribute__((visibility("default"))) int fakejvm_array_len(const void* a) { return a ? O(a)->len : -1; }
__attribute__((visibility("default"))) const void* fakejvm_array_data(const void* a) {
  return a ? O(a)->data.data() : nullptr;
}

}  // extern "C"
