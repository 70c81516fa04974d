"""ctypes helpers for driving libfleet_native.so built against the test JNI
header (tests/native/jni/jni.h): arrays are heap blocks {int32 len, int32 elem, payload}."""
import ctypes as C

import numpy as np

libc = C.CDLL(None)
libc.calloc.restype = C.c_void_p
libc.calloc.argtypes = [C.c_size_t, C.c_size_t]
libc.free.argtypes = [C.c_void_p]

HDR = 8


def new_array(payload: bytes, elem: int = 1) -> int:
    n = len(payload) // elem
    p = libc.calloc(1, HDR + len(payload) + 1)
    C.memmove(p, C.byref(C.c_int32(n)), 4)
    C.memmove(p + 4, C.byref(C.c_int32(elem)), 4)
    C.memmove(p + HDR, payload, len(payload))
    return p


def new_object_array(ptrs) -> int:
    arr = (C.c_void_p * len(ptrs))(*ptrs)
    return new_array(bytes(arr), elem=C.sizeof(C.c_void_p))


def read_bytes(p: int) -> bytes:
    assert p, "native returned null"
    n = C.c_int32.from_address(p).value
    return C.string_at(p + HDR, n)


def new_doubles(values) -> int:
    return new_array(np.ascontiguousarray(values, np.float64).tobytes(), elem=8)
