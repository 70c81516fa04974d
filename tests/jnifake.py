"""ctypes harness for driving libfleet_native.so through a JNI function table.

tests/native/fakejvm.cpp (built here with g++ against tests/native/jni/jni.h,
the JNI specification's table layout) is a small in-process JVM stand-in:
fakejvm_env() is a JNIEnv* whose `functions` table the shim's calls dispatch
through, and it counts the JNI-rule violations the shim must avoid (local
reference overflow, JNI calls inside critical regions, unreleased array
elements). TEST INFRASTRUCTURE ONLY."""
import ctypes as C
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def fakejvm():
    global _lib
    if _lib is not None:
        return _lib
    out = os.path.join(tempfile.mkdtemp(prefix="fakejvm"), "libfakejvm.so")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden",
                           "-I", os.path.join(HERE, "native", "jni"), os.path.join(HERE, "native", "fakejvm.cpp"),
                           "-o", out])
    L = C.CDLL(out)
    vp = C.c_void_p
    L.fakejvm_env.restype = vp
    L.fakejvm_begin_call.restype = None
    L.fakejvm_stat.restype = C.c_long
    L.fakejvm_stat.argtypes = [C.c_char_p]
    L.fakejvm_set_frame_limit.argtypes = [C.c_long]
    L.fakejvm_new_array.restype = vp
    L.fakejvm_new_array.argtypes = [C.c_int, vp, C.c_int]
    L.fakejvm_new_object_array.restype = vp
    L.fakejvm_new_object_array.argtypes = [vp, C.c_int]
    L.fakejvm_collect.restype = None
    L.fakejvm_collect.argtypes = [vp]
    L.fakejvm_new_direct.restype = vp
    L.fakejvm_new_direct.argtypes = [vp, C.c_long]
    L.fakejvm_new_string.restype = vp
    L.fakejvm_new_string.argtypes = [C.c_char_p]
    L.fakejvm_array_len.restype = C.c_int
    L.fakejvm_array_len.argtypes = [vp]
    L.fakejvm_array_data.restype = vp
    L.fakejvm_array_data.argtypes = [vp]
    _lib = L
    return L


def collect(obj) -> None:
    """The garbage collector reclaims obj: weak references to it now equal NULL."""
    fakejvm().fakejvm_collect(obj)


def env():
    return fakejvm().fakejvm_env()


def begin():
    fakejvm().fakejvm_begin_call()


def stat(name: str) -> int:
    return fakejvm().fakejvm_stat(name.encode())


def new_bytes(payload: bytes) -> int:
    return fakejvm().fakejvm_new_array(1, payload, len(payload))


def new_doubles(values) -> int:
    a = np.ascontiguousarray(values, np.float64)
    return fakejvm().fakejvm_new_array(4, a.ctypes.data, len(a))


def new_floats(values) -> int:
    a = np.ascontiguousarray(values, np.float32)
    return fakejvm().fakejvm_new_array(3, a.ctypes.data, len(a))


def new_object_array(ptrs) -> int:
    arr = (C.c_void_p * len(ptrs))(*ptrs)
    return fakejvm().fakejvm_new_object_array(arr, len(ptrs))


def new_direct(buf: np.ndarray) -> int:
    return fakejvm().fakejvm_new_direct(buf.ctypes.data, buf.nbytes)


def new_string(text: str) -> int:
    return fakejvm().fakejvm_new_string(text.encode())


def read_bytes(p: int) -> bytes:
    assert p, "native returned null"
    L = fakejvm()
    return C.string_at(L.fakejvm_array_data(p), L.fakejvm_array_len(p))
