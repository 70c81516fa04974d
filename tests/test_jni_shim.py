"""The JNI shim (libfleet_native.so): exports the reference's Java_* natives and
returns, through a JNI function table (tests/native/jni/jni.h, the JNI
specification's slot order; tests/native/fakejvm.cpp), exactly the bytes of the
reference path -- while keeping the JNI rules a JVM enforces (local reference
capacity, critical regions, released array elements)."""
import ctypes as C
import os

import numpy as np
import pytest

import fleet_amd as F
from fleet_amd.layouts import MNIST

JNI = os.path.join(os.path.dirname(F.LIB_PATH), "libfleet_native.so")
HERE = os.path.dirname(os.path.abspath(__file__))
UPDATER = "Java_apps_cppNN_CppNNUpdater_"
BYTES_OUT = {
    UPDATER + "getFlatGradient": 1, UPDATER + "mergeFlatGradient": 2, "Java_utils_ByteVec_scalarMulNative": None,
    "Java_utils_ByteVec_addNative": 2, "Java_utils_ByteVec_subtractNative": 2,
    "Java_apps_cppNN_FleetUpdater_aggregateNative": 2, UPDATER + "getParametersNative": None,
    UPDATER + "getModelParametersNative": None, "Java_apps_cppNN_FleetUpdater_aggregateDirectNative": None,
}
SAMPLER = "Java_apps_cppNN_CppNNOfflineSampler_"
SYMBOLS = list(BYTES_OUT) + ["Java_utils_ByteVec_getNorm", UPDATER + "fetchParamsNative", UPDATER + "initUpdater",
                             UPDATER + "descentNative", UPDATER + "modelsSize", UPDATER + "getPriority",
                             UPDATER + "setPriority", UPDATER + "getCurrEpoch", UPDATER + "setCurrEpoch",
                             UPDATER + "getLrate", UPDATER + "getNumLabels", UPDATER + "hasOutlier",
                             UPDATER + "printParamsNative", SAMPLER + "initSampler", SAMPLER + "getMiniBatch",
                             "Java_apps_cppNN_FleetUpdater_registerDirectNative",
                             "Java_apps_cppNN_FleetUpdater_unregisterDirectNative",
                             "Java_apps_cppNN_FleetSampler_setTeacherNative"]


def load():
    if not os.path.exists(JNI):
        pytest.skip("libfleet_native.so not built")
    F.lib()  # same HIP runtime as torch
    L = C.CDLL(JNI)
    vp, i32, f64 = C.c_void_p, C.c_int32, C.c_double
    for s in BYTES_OUT:
        getattr(L, s).restype = vp
    sig = {
        UPDATER + "getFlatGradient": [vp, vp, vp], UPDATER + "mergeFlatGradient": [vp, vp, vp, vp],
        "Java_utils_ByteVec_scalarMulNative": [vp, vp, vp, f64], "Java_utils_ByteVec_getNorm": [vp, vp, vp],
        "Java_utils_ByteVec_addNative": [vp, vp, vp, vp], "Java_utils_ByteVec_subtractNative": [vp, vp, vp, vp],
        "Java_apps_cppNN_FleetUpdater_aggregateNative": [vp, vp, vp, vp],
        "Java_apps_cppNN_FleetUpdater_aggregateDirectNative": [vp, vp, vp, i32, i32, i32, vp],
        "Java_apps_cppNN_FleetUpdater_registerDirectNative": [vp, vp, vp],
        UPDATER + "fetchParamsNative": [vp, vp, vp], UPDATER + "initUpdater": [vp, vp, vp, i32, f64, f64],
        UPDATER + "descentNative": [vp, vp, vp, i32, i32], UPDATER + "getParametersNative": [vp, vp, i32],
        UPDATER + "getModelParametersNative": [vp, vp, i32], UPDATER + "modelsSize": [vp, vp],
        UPDATER + "getCurrEpoch": [vp, vp], UPDATER + "setCurrEpoch": [vp, vp, i32],
        UPDATER + "getPriority": [vp, vp], UPDATER + "setPriority": [vp, vp, i32], UPDATER + "getLrate": [vp, vp],
        UPDATER + "getNumLabels": [vp, vp], UPDATER + "hasOutlier": [vp, vp], UPDATER + "printParamsNative": [vp, vp, vp],
        SAMPLER + "initSampler": [vp, vp, vp], SAMPLER + "getMiniBatch": [vp, vp, i32],
        "Java_apps_cppNN_FleetUpdater_unregisterDirectNative": [vp, vp, vp],
        "Java_apps_cppNN_FleetSampler_setTeacherNative": [vp, vp, vp, vp],
    }
    for s, a in sig.items():
        getattr(L, s).argtypes = a
    L.Java_utils_ByteVec_getNorm.restype = f64
    L.Java_apps_cppNN_CppNNUpdater_getLrate.restype = f64
    L.Java_apps_cppNN_FleetUpdater_registerDirectNative.restype = C.c_uint8
    L.Java_apps_cppNN_CppNNUpdater_hasOutlier.restype = C.c_uint8
    L.Java_apps_cppNN_FleetSampler_setTeacherNative.restype = C.c_uint8
    L.Java_apps_cppNN_CppNNOfflineSampler_getMiniBatch.restype = vp
    L.Java_apps_cppNN_FleetUpdater_unregisterDirectNative.restype = None
    L.Java_apps_cppNN_CppNNUpdater_printParamsNative.restype = None
    for s in ("modelsSize", "getCurrEpoch", "getPriority", "getNumLabels"):
        getattr(L, UPDATER + s).restype = i32
    return L


def test_shim_exports_reference_symbols():
    L = load()
    for s in SYMBOLS:
        assert hasattr(L, s), s


def test_shim_exports_every_reference_native():
    """Every Java_* native of the reference's server backend (cppNN_backend.cpp: 22
    symbols) is served by the shim, so the JVM never binds one of them
    to libnative.so."""
    ref = ["getNumLabels", "hasOutlier", "setCurrEpoch", "getCurrEpoch", "setPriority", "getPriority", "getLrate",
           "initUpdater", "getModelParametersNative", "getParametersNative", "fetchParamsNative",
           "printParamsNative", "modelsSize", "descentNative", "getFlatGradient", "mergeFlatGradient"]
    names = [UPDATER + r for r in ref] + [SAMPLER + "initSampler", SAMPLER + "getMiniBatch"] + [
        "Java_utils_ByteVec_" + r for r in ("scalarMulNative", "getNorm", "addNative", "subtractNative")]
    assert len(names) == 22
    L = load()
    for s in names:
        assert hasattr(L, s), s


def test_fake_jvm_table_is_jni_shaped():
    import jnifake as J
    J.begin()
    e = J.env()
    table = C.cast(C.c_void_p.from_address(e).value, C.POINTER(C.c_void_p))
    assert all(table[i] is None for i in range(4))          # reserved slots
    assert table[171] and table[184] and table[222]         # GetArrayLength, GetByteArrayElements, critical
    assert C.cast(table[4], C.CFUNCTYPE(C.c_int32, C.c_void_p))(e) == 0x00010008  # GetVersion


def test_model_natives_without_a_model_are_inert():
    # before fetchParamsNative the updater's state natives answer like an empty `models`
    L = load()
    import jnifake as J
    J.begin()
    assert L.Java_apps_cppNN_CppNNUpdater_modelsSize(J.env(), None) == 0
    assert L.Java_apps_cppNN_CppNNUpdater_getParametersNative(J.env(), None, 0) is None
    assert J.stat("critical_violations") == 0 and J.stat("overflows") == 0


def check_rules(J):
    assert J.stat("overflows") == 0, "local references beyond the frame's capacity"
    assert J.stat("critical_violations") == 0, "JNI call inside a critical region"
    assert J.stat("critical_depth") == 0, "critical region left open"
    assert J.stat("pins") == 0, "array elements not released"


@pytest.mark.gpu
def test_shim_per_op_natives_match_oracle(oracle):
    import jnifake as J
    L = load()
    env = J.env()
    ups = [oracle.encode_floats(oracle.synth_upload(4, c, list(MNIST.w_sizes), list(MNIST.b_sizes)))
           for c in range(3)]
    J.begin()
    a = J.new_bytes(ups[0])
    flat = J.read_bytes(L.Java_apps_cppNN_CppNNUpdater_getFlatGradient(env, None, a))
    assert flat == oracle.flat_gradient(ups[0])
    f1 = oracle.flat_gradient(ups[1])
    assert J.read_bytes(L.Java_utils_ByteVec_scalarMulNative(env, None, J.new_bytes(f1), 1 / 3)) == \
        oracle.scalar_mul(f1, 1 / 3)
    assert J.read_bytes(L.Java_utils_ByteVec_addNative(env, None, J.new_bytes(flat), J.new_bytes(f1))) == \
        oracle.add(flat, f1)
    assert J.read_bytes(L.Java_utils_ByteVec_subtractNative(env, None, J.new_bytes(flat), J.new_bytes(f1))) == \
        oracle.subtract(flat, f1)
    assert abs(L.Java_utils_ByteVec_getNorm(env, None, J.new_bytes(f1)) - oracle.norm(f1)) <= 1e-12 * oracle.norm(f1)
    assert J.read_bytes(L.Java_apps_cppNN_CppNNUpdater_mergeFlatGradient(env, None, a, J.new_bytes(f1))) == \
        oracle.merge_flat_gradient(ups[0], f1)
    check_rules(J)


@pytest.mark.gpu
@pytest.mark.parametrize("frame_limit", [1 << 30, 8])
def test_shim_aggregate_many_uploads(oracle, frame_limit):
    # 40 uploads: more than the 16 local references JNI guarantees. With a JVM that
    # grants EnsureLocalCapacity(40) the uploads are read in one critical region;
    # with one that refuses (frame_limit 8) one reference at a time.
    import jnifake as J
    L = load()
    env = J.env()
    M = 40
    ups = [oracle.encode_floats(oracle.synth_upload(6, c, list(MNIST.w_sizes), list(MNIST.b_sizes)))
           for c in range(M)]
    d = [1.0 / ((c % 3) + 1) for c in range(M)]
    J.fakejvm().fakejvm_set_frame_limit(frame_limit)
    try:
        J.begin()
        objs = J.new_object_array([J.new_bytes(u) for u in ups])
        merged = J.read_bytes(L.Java_apps_cppNN_FleetUpdater_aggregateNative(env, None, objs, J.new_doubles(d)))
        check_rules(J)
        assert J.stat("max_live") <= (M + 1 if frame_limit > M else 16)
        assert (J.stat("criticals") == M) == (frame_limit > M)
    finally:
        J.fakejvm().fakejvm_set_frame_limit(1 << 30)
    assert merged == oracle.update_faithful(ups, d)
    # a null element: null result, every reference and critical region released
    J.begin()
    bad = J.new_object_array([J.new_bytes(ups[0]), None, J.new_bytes(ups[2])])
    assert L.Java_apps_cppNN_FleetUpdater_aggregateNative(env, None, bad, J.new_doubles(d[:3])) is None
    check_rules(J)


@pytest.mark.gpu
def test_shim_aggregate_direct_buffer(oracle):
    import jnifake as J
    L = load()
    env = J.env()
    M = 5
    ups = [oracle.encode_floats(oracle.synth_upload(8, c, list(MNIST.w_sizes), list(MNIST.b_sizes)))
           for c in range(M)]
    d = [1.0, 0.5, 1 / 3, 1.0, 0.5]
    Lb = len(ups[0])
    pitch = Lb + 5
    rows = np.zeros(M * pitch, np.uint8)
    for i, u in enumerate(ups):
        rows[i * pitch: i * pitch + Lb] = np.frombuffer(u, np.uint8)
    J.begin()
    buf = J.new_direct(rows)
    assert L.Java_apps_cppNN_FleetUpdater_registerDirectNative(env, None, buf) == 1
    out = J.read_bytes(L.Java_apps_cppNN_FleetUpdater_aggregateDirectNative(env, None, buf, M, Lb, pitch,
                                                                             J.new_doubles(d)))
    assert out == oracle.update_faithful(ups, d)
    check_rules(J)


@pytest.mark.gpu
def test_shim_model_natives_match_reference_session(oracle):
    # the updater's model natives through the table, against the reference's own
    # network (tests/golden/session_mnist.npz, see test_gpu_model_state.py)
    import jnifake as J
    L = load()
    env = J.env()
    s = np.load(os.path.join(HERE, "golden", "session_mnist.npz"))
    J.begin()
    L.Java_apps_cppNN_CppNNUpdater_fetchParamsNative(env, None, J.new_bytes(bytes(s["init"])))
    L.Java_apps_cppNN_CppNNUpdater_initUpdater(env, None, J.new_doubles(s["lrates"]), 1, 0.0, 0.0)
    for step in range(4):
        if step:
            L.Java_apps_cppNN_CppNNUpdater_descentNative(env, None, J.new_bytes(bytes(s[f"merged{step - 1}"])),
                                                         int(s["batch"]), int(s["stale"]))
        newest = L.Java_apps_cppNN_CppNNUpdater_modelsSize(env, None) - 1
        assert J.read_bytes(L.Java_apps_cppNN_CppNNUpdater_getParametersNative(env, None, newest)) == \
            bytes(s[f"newest_text{step}"])
        assert J.read_bytes(L.Java_apps_cppNN_CppNNUpdater_getModelParametersNative(env, None, 0)) == \
            oracle.encode_floats(s[f"oldest_params{step}"])
    assert L.Java_apps_cppNN_CppNNUpdater_getCurrEpoch(env, None) == 3
    assert L.Java_apps_cppNN_CppNNUpdater_getLrate(env, None) == float(np.float32(s["lrates"][2]))
    check_rules(J)


@pytest.mark.gpu
def test_shim_print_params(oracle, capfd):
    """printParamsNative (:304-322): the upload's int32 codes on stdout."""
    import jnifake as J
    L = load()
    codes = np.array([100000001, -10000002, 7, 0, 123456789], np.int32)
    J.begin()
    L.Java_apps_cppNN_CppNNUpdater_printParamsNative(J.env(), None, J.new_bytes(oracle.encode_ints(codes)))
    check_rules(J)
    assert "Got Numbers: 100000001 -10000002 7 0 123456789 \n" in capfd.readouterr().out


@pytest.mark.gpu
def test_shim_direct_buffer_reregistration(oracle):
    """A registration outlives nothing: unregisterDirectNative releases it, and a new
    buffer over the same memory re-registers cleanly (the stale one is released)."""
    import jnifake as J
    L = load()
    env = J.env()
    M = 3
    ups = [oracle.encode_floats(oracle.synth_upload(9, c, list(MNIST.w_sizes), list(MNIST.b_sizes)))
           for c in range(M)]
    Lb = len(ups[0])
    rows = np.zeros(M * Lb, np.uint8)
    for i, u in enumerate(ups):
        rows[i * Lb:(i + 1) * Lb] = np.frombuffer(u, np.uint8)
    d = [1.0, 0.5, 0.25]
    J.begin()
    buf = J.new_direct(rows)
    assert L.Java_apps_cppNN_FleetUpdater_registerDirectNative(env, None, buf) == 1
    assert L.Java_apps_cppNN_FleetUpdater_registerDirectNative(env, None, J.new_direct(rows[: 2 * Lb])) == 1
    out = J.read_bytes(L.Java_apps_cppNN_FleetUpdater_aggregateDirectNative(env, None, buf, M, Lb, Lb,
                                                                             J.new_doubles(d)))
    assert out == oracle.update_faithful(ups, d)  # rows now outside the (smaller) registration: staged
    L.Java_apps_cppNN_FleetUpdater_unregisterDirectNative(env, None, buf)
    out = J.read_bytes(L.Java_apps_cppNN_FleetUpdater_aggregateDirectNative(env, None, buf, M, Lb, Lb,
                                                                             J.new_doubles(d)))
    assert out == oracle.update_faithful(ups, d)
    check_rules(J)


@pytest.mark.gpu
def test_shim_collected_registration_is_not_used(oracle):
    """A direct buffer the JVM collected without unregisterDirectNative:
    a new buffer at the same address must not be DMA'd through the old page lock. The
    shim keeps a weak reference per registration; aggregateDirectNative sees the
    referent gone, releases the registration and stages the rows."""
    import jnifake as J
    L = load()
    env = J.env()
    M = 3
    ups = [oracle.encode_floats(oracle.synth_upload(11, c, list(MNIST.w_sizes), list(MNIST.b_sizes)))
           for c in range(M)]
    Lb = len(ups[0])
    rows = np.zeros(M * Lb, np.uint8)
    for i, u in enumerate(ups):
        rows[i * Lb:(i + 1) * Lb] = np.frombuffer(u, np.uint8)
    d = [1.0, 0.5, 0.25]
    want = oracle.update_faithful(ups, d)
    J.begin()
    weak0 = J.stat("weak")
    old = J.new_direct(rows)
    assert L.Java_apps_cppNN_FleetUpdater_registerDirectNative(env, None, old) == 1
    assert J.stat("weak") == weak0 + 1
    # the registered, live buffer: copy-free
    out = J.read_bytes(L.Java_apps_cppNN_FleetUpdater_aggregateDirectNative(env, None, old, M, Lb, Lb,
                                                                             J.new_doubles(d)))
    assert out == want and F.lib().fleet_last_ingress(None) == 2  # FLEET_INGRESS_PINNED
    # another live view of the same memory (a duplicate()): still copy-free
    view = J.new_direct(rows)
    out = J.read_bytes(L.Java_apps_cppNN_FleetUpdater_aggregateDirectNative(env, None, view, M, Lb, Lb,
                                                                             J.new_doubles(d)))
    assert out == want and F.lib().fleet_last_ingress(None) == 2
    # dropped without unregisterDirectNative; a new buffer at the same address
    J.collect(old)
    J.collect(view)
    new = J.new_direct(rows)
    out = J.read_bytes(L.Java_apps_cppNN_FleetUpdater_aggregateDirectNative(env, None, new, M, Lb, Lb,
                                                                             J.new_doubles(d)))
    assert out == want
    assert F.lib().fleet_last_ingress(None) == 1  # FLEET_INGRESS_STAGED: the stale lock was not used
    assert J.stat("weak") == weak0  # the stale record's weak reference was deleted
    # registering the new buffer works, and it is copy-free again
    assert L.Java_apps_cppNN_FleetUpdater_registerDirectNative(env, None, new) == 1
    out = J.read_bytes(L.Java_apps_cppNN_FleetUpdater_aggregateDirectNative(env, None, new, M, Lb, Lb,
                                                                             J.new_doubles(d)))
    assert out == want and F.lib().fleet_last_ingress(None) == 2
    L.Java_apps_cppNN_FleetUpdater_unregisterDirectNative(env, None, new)
    assert J.stat("weak") == weak0
    check_rules(J)
