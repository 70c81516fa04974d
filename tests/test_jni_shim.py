"""The JNI shim (libfleet_native.so): exports the reference's Java_* natives and
returns, through the (test) JNI surface, exactly the bytes of the reference path."""
import ctypes as C
import os

import numpy as np
import pytest

import fleet_amd as F
from fleet_amd.layouts import MNIST, synthetic

JNI = os.path.join(os.path.dirname(F.LIB_PATH), "libfleet_native.so")
SYMBOLS = ["Java_apps_cppNN_CppNNUpdater_getFlatGradient", "Java_apps_cppNN_CppNNUpdater_mergeFlatGradient",
           "Java_utils_ByteVec_scalarMulNative", "Java_utils_ByteVec_getNorm", "Java_utils_ByteVec_addNative",
           "Java_utils_ByteVec_subtractNative", "Java_apps_cppNN_FleetUpdater_aggregateNative"]


def load():
    if not os.path.exists(JNI):
        pytest.skip("libfleet_native.so not built")
    F.lib()  # same HIP runtime as torch
    L = C.CDLL(JNI)
    vp = C.c_void_p
    for s in SYMBOLS:
        getattr(L, s).restype = C.c_double if s.endswith("getNorm") else vp
    L.Java_apps_cppNN_CppNNUpdater_getFlatGradient.argtypes = [vp, vp, vp]
    L.Java_apps_cppNN_CppNNUpdater_mergeFlatGradient.argtypes = [vp, vp, vp, vp]
    L.Java_utils_ByteVec_scalarMulNative.argtypes = [vp, vp, vp, C.c_double]
    L.Java_utils_ByteVec_getNorm.argtypes = [vp, vp, vp]
    L.Java_utils_ByteVec_addNative.argtypes = [vp, vp, vp, vp]
    L.Java_utils_ByteVec_subtractNative.argtypes = [vp, vp, vp, vp]
    L.Java_apps_cppNN_FleetUpdater_aggregateNative.argtypes = [vp, vp, vp, vp]
    return L


def test_shim_exports_reference_symbols():
    L = load()
    for s in SYMBOLS:
        assert hasattr(L, s)


@pytest.mark.gpu
def test_shim_natives_match_oracle(oracle):
    import jnifake as J
    L = load()
    env = J.libc.calloc(1, 64)  # JNIEnv of the test header is stateless
    ups = [oracle.encode_floats(oracle.synth_upload(4, c, list(MNIST.w_sizes), list(MNIST.b_sizes)))
           for c in range(3)]
    a = J.new_array(ups[0])
    flat = J.read_bytes(L.Java_apps_cppNN_CppNNUpdater_getFlatGradient(env, None, a))
    assert flat == oracle.flat_gradient(ups[0])
    f1 = oracle.flat_gradient(ups[1])
    assert J.read_bytes(L.Java_utils_ByteVec_scalarMulNative(env, None, J.new_array(f1), 1 / 3)) == \
        oracle.scalar_mul(f1, 1 / 3)
    assert J.read_bytes(L.Java_utils_ByteVec_addNative(env, None, J.new_array(flat), J.new_array(f1))) == \
        oracle.add(flat, f1)
    assert J.read_bytes(L.Java_utils_ByteVec_subtractNative(env, None, J.new_array(flat), J.new_array(f1))) == \
        oracle.subtract(flat, f1)
    assert abs(L.Java_utils_ByteVec_getNorm(env, None, J.new_array(f1)) - oracle.norm(f1)) <= 1e-12 * oracle.norm(f1)
    assert J.read_bytes(L.Java_apps_cppNN_CppNNUpdater_mergeFlatGradient(env, None, a, J.new_array(f1))) == \
        oracle.merge_flat_gradient(ups[0], f1)
    d = [1.0, 0.5, 1 / 3]
    objs = J.new_object_array([J.new_array(u) for u in ups])
    merged = J.read_bytes(L.Java_apps_cppNN_FleetUpdater_aggregateNative(env, None, objs, J.new_doubles(d)))
    assert merged == oracle.update_faithful(ups, d)
