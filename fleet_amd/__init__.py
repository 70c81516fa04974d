"""fleet_amd -- MI355X-native FLeet gradient codec + server-side aggregation.

Python host layer over the C-ABI of ``include/fleet_codec.h`` (libfleetcodec.so,
gfx950 HIP kernels). It mirrors the reference's native surface:

* :class:`Codec` -- one device context; the JNI natives of the reference's
  server backend (Server/src/main/c++/cppNN_backend.cpp) as methods with the
  same names and argument meaning (``getFlatGradient``, ``mergeFlatGradient``,
  ``scalarMulNative``, ``addNative``, ``subtractNative``, ``getNorm``) plus the
  fused batched ``update`` and the device-resident entry points.
* :class:`ByteVec` -- mirror of Server/src/main/java/utils/ByteVec.java.
* :mod:`fleet_amd.updater` -- mirror of CppNNUpdater's aggregation logic.

There is no CPU compute path: if the HIP library is missing or no GPU is
visible, constructing a :class:`Codec` raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

from .layouts import LAYOUTS, Layout  # noqa: F401

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
# FLEET_CODEC_LIB: load another build of the same C-ABI (A/B experiments on one box)
LIB_PATH = os.environ.get("FLEET_CODEC_LIB") or os.path.join(PKG, "libfleetcodec.so")
HEADER_PATH = os.path.join(ROOT, "include", "fleet_codec.h")

FLEET_OK = 0
FLEET_ERR_ARG = -1
FLEET_ERR_BASE64 = -2
FLEET_ERR_LAYOUT = -3
FLEET_ERR_HIP = -4
FLEET_ERR_NOMEM = -5
FLEET_ERR_CAPACITY = -6
FLEET_MAX_HEADERS = 4096


class FleetError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class Base64Error(FleetError):
    pass


class LayoutError(FleetError):
    pass


_lib = None


def lib() -> C.CDLL:
    """Load libfleetcodec.so (build it with ``python -m fleet_amd.build``)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `python -m fleet_amd.build` (HIP extension not built)")
    # One HIP runtime per process: when torch (ROCm build) is present, load it first so
    # libfleetcodec.so binds to the libamdhip64 torch already mapped (two runtimes in
    # one process cannot share streams/pointers and the second fails to initialise).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    sz, vp, i32, i64 = C.c_size_t, C.c_void_p, C.c_int, C.c_int64
    szp = C.POINTER(C.c_size_t)
    sig = {
        "fleet_version": (C.c_char_p, []),
        "fleet_create": (i32, [i32, C.POINTER(vp)]),
        "fleet_destroy": (None, [vp]),
        "fleet_last_error": (C.c_char_p, [vp]),
        "fleet_sync": (i32, [vp, vp]),
        "fleet_check": (i32, [vp, vp]),
        "fleet_b64_len": (sz, [sz]),
        "fleet_b64_count": (sz, [sz]),
        "fleet_layout_from_sizes": (i32, [vp, i32, vp, i32, vp, i32, C.POINTER(i32), szp]),
        "fleet_layout_parse": (i32, [vp, vp, sz, vp, i32, C.POINTER(i32), szp]),
        "fleet_encode_f32": (i32, [vp, vp, sz, vp, sz, szp]),
        "fleet_encode_i32": (i32, [vp, vp, sz, vp, sz, szp]),
        "fleet_decode_f32": (i32, [vp, vp, sz, vp, sz, szp]),
        "fleet_decode_i32": (i32, [vp, vp, sz, vp, sz, szp]),
        "fleet_flat_gradient": (i32, [vp, vp, sz, vp, sz, szp]),
        "fleet_merge_flat_gradient": (i32, [vp, vp, sz, vp, sz, vp, sz, szp]),
        "fleet_scalar_mul": (i32, [vp, vp, sz, C.c_double, vp, sz, szp]),
        "fleet_add": (i32, [vp, vp, sz, vp, sz, vp, sz, szp]),
        "fleet_subtract": (i32, [vp, vp, sz, vp, sz, vp, sz, szp]),
        "fleet_norm": (i32, [vp, vp, sz, C.POINTER(C.c_double)]),
        "fleet_update": (i32, [vp, vp, vp, i32, vp, vp, sz, szp, vp]),
        "fleet_update_multi": (i32, [vp, i32, vp, vp, i32, vp, vp, sz, szp, vp]),
        "fleet_update_rows": (i32, [vp, vp, sz, sz, i32, vp, vp, sz, szp, vp]),
        "fleet_update_rows_multi": (i32, [vp, i32, vp, sz, sz, i32, vp, vp, sz, szp, vp]),
        "fleet_host_register": (i32, [vp, vp, sz]),
        "fleet_host_unregister": (i32, [vp, vp]),
        "fleet_update_device": (i32, [vp, vp, sz, sz, i32, vp, vp, i32, sz, sz, vp, vp, vp]),
        "fleet_update_encode_device": (i32, [vp, vp, sz, sz, i32, vp, vp, i32, vp, vp, vp, sz, vp, vp]),
        "fleet_update_kardam_device": (i32, [vp, vp, sz, sz, i32, vp, vp, i32, C.c_double, vp, vp, vp, sz, vp, vp,
                                             vp, vp, vp]),
        "fleet_update_kernel": (C.c_char_p, [sz]),
        "fleet_update_plan_grid": (i32, [sz, C.POINTER(C.c_int), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                         C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
        "fleet_update_encode_kernel": (C.c_char_p, [sz]),
        "fleet_set_plan": (i32, [C.c_char_p, vp, sz]),
        "fleet_plan": (C.c_char_p, []),
        "fleet_model_quantize_index": (i32, [vp, vp, vp, i32, vp, vp, vp, vp]),
        "fleet_model_weights_text": (i32, [vp, vp, vp, i32, vp, sz, szp]),
        "fleet_model_read_weights": (i32, [vp, vp, sz, vp, i32, vp]),
        "fleet_encode_device": (i32, [vp, vp, sz, sz, i32, vp, sz, vp]),
        "fleet_decode_device": (i32, [vp, vp, sz, sz, i32, vp, sz, vp]),
        "fleet_synth_device": (i32, [vp, C.c_uint64, i32, i32, vp, vp, i32, sz, vp, sz, vp]),
        "fleet_synth_window_device": (i32, [vp, C.c_uint64, i32, i32, sz, vp, vp, i32, sz, vp, sz, vp]),
        "fleet_selftest_digest": (i32, [vp, i32, C.POINTER(C.c_uint64)]),
        "fleet_descent_device": (i32, [vp, vp, vp, vp, vp, vp, i32, vp, vp, i32, C.c_float, vp]),
        "fleet_descent": (i32, [vp, vp, sz, vp, sz, vp, sz, vp, vp, i32, vp, vp, i32, C.c_float]),
        "fleet_model_params": (i32, [vp, vp, sz, vp, sz, i32, vp, sz, szp]),
        "fleet_model_version": (i32, [vp, vp, vp, i32, vp, sz, vp, vp]),
        "fleet_model_params_device": (i32, [vp, vp, sz, vp, sz, i32, vp, vp]),
        "fleet_minibatch_len": (sz, [i32, i32, i32, i32]),
        "fleet_test_kardam_skew": (i32, [vp, C.c_uint]),
        "fleet_kardam_grads": (i32, [vp, vp, vp, i32, vp, C.c_double, vp, vp, sz, szp, vp, vp]),
        "fleet_descent_window_device": (i32, [vp, vp, vp, vp, sz, sz, vp, vp, i32, vp, vp, i32, C.c_float, vp]),
        "fleet_minibatch_device": (i32, [vp, vp, sz, i32, vp, vp, i32, vp, i32, vp, vp, vp]),
        "fleet_minibatch": (i32, [vp, vp, sz, i32, vp, vp, i32, vp, i32, vp, vp, sz, szp]),
        "fleet_teacher_weight_count": (sz, []),
        "fleet_teacher_bias_count": (sz, []),
        "fleet_teacher_forward_device": (i32, [vp, vp, vp, vp, sz, i32, vp, i32, C.c_float, vp, vp]),
        "fleet_teacher_forward": (i32, [vp, vp, sz, vp, sz, vp, sz, i32, vp, i32, C.c_float, vp]),
        "fleet_model_load": (i32, [vp, vp, sz, i32, C.POINTER(vp)]),
        "fleet_model_destroy": (None, [vp]),
        "fleet_model_last_error": (C.c_char_p, [vp]),
        "fleet_model_init_updater": (i32, [vp, vp, i32]),
        "fleet_model_descent": (i32, [vp, vp, sz, i32, i32]),
        "fleet_model_count": (i32, [vp]),
        "fleet_model_get_params": (i32, [vp, i32, vp, sz, szp]),
        "fleet_model_get_model_params": (i32, [vp, i32, vp, sz, szp]),
        "fleet_model_get_epoch": (i32, [vp]),
        "fleet_model_set_epoch": (None, [vp, i32]),
        "fleet_model_get_priority": (i32, [vp]),
        "fleet_model_set_priority": (None, [vp, i32]),
        "fleet_model_get_lrate": (C.c_double, [vp]),
        "fleet_model_shape": (i32, [vp, szp, szp, C.POINTER(i32), C.POINTER(i32)]),
        "fleet_model_export": (i32, [vp, i32, vp, sz, vp, sz]),
        "fleet_sampler_create": (i32, [vp, C.c_char_p, i32, i32, i32, i32, i32, C.POINTER(vp)]),
        "fleet_sampler_create_from": (i32, [vp, vp, vp, sz, i32, i32, i32, i32, i32, i32, i32, C.POINTER(vp)]),
        "fleet_sampler_destroy": (None, [vp]),
        "fleet_sampler_last_error": (C.c_char_p, [vp]),
        "fleet_last_ingress": (i32, [vp]),
        "fleet_updater_reseed_ex": (None, [i32, i32]),
        "fleet_updater_reseed": (None, [i32]),
        "fleet_sampler_set_hyper": (i32, [vp, i32, C.c_double, C.c_double]),
        "fleet_sampler_set_teacher": (i32, [vp, vp, sz, vp, sz]),
        "fleet_sampler_minibatch": (i32, [vp, i32, C.c_float, vp, sz, szp]),
        "fleet_sampler_minibatch_len": (sz, [vp, i32]),
        "fleet_sampler_num_labels": (i32, [vp]),
        "fleet_sampler_has_outlier": (i32, [vp]),
        "fleet_sampler_num_samples": (sz, [vp]),
        "fleet_sampler_bucket": (i32, [vp, i32, vp, sz, szp]),
        "fleet_sampler_sorted_index": (i32, [vp, vp, sz, szp]),
        "fleet_sampler_last_indices": (i32, [vp, vp, sz, szp]),
    }
    ab_build = bool(os.environ.get("FLEET_CODEC_LIB"))
    for name, (res, args) in sig.items():
        try:
            f = getattr(L, name)
        except AttributeError:
            if ab_build:  # an A/B build from an older commit: entry points it predates stay unbound
                continue
            raise
        f.restype = res
        f.argtypes = args
    _ = i64
    _lib = L
    return L


def exported_symbols_from_header(path: str = HEADER_PATH):
    """Function names declared in include/fleet_codec.h."""
    import re
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fleet_[a-z0-9_]+)\s*\(", text)))


def b64_len(n_values: int) -> int:
    """Base64 length of n int32 values: 4*ceil(4n/3) (Base64.cpp:129-136)."""
    return 4 * ((4 * n_values + 2) // 3)


def b64_count(length: int) -> int:
    return 3 * length // 16


def update_kernel(length: int) -> str:
    """Aggregation kernel the library launches for uploads of `length` bytes."""
    return lib().fleet_update_kernel(length).decode()


def update_plan_grid(length: int) -> dict:
    """The aggregation's launch grid for uploads of `length` bytes (fleet_update_plan_grid):
    kind ("stream" / "tiled" / "pipe" / "weave" / "flat"), blocks, and n_a / n_w / n_n (see fleet_codec.h)."""
    k = C.c_int()
    b, a, w, n = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
    rc = lib().fleet_update_plan_grid(length, C.byref(k), C.byref(b), C.byref(a), C.byref(w), C.byref(n))
    if rc != 0:
        raise FleetError(f"fleet_update_plan_grid: {rc}")
    return {"kind": ("stream", "tiled", "pipe", "weave", "flat")[k.value], "blocks": b.value, "n_a": a.value, "n_w": w.value,
            "n_n": n.value}


def update_encode_kernel(length: int) -> str:
    """What fleet_update_encode_device launches for uploads of `length` bytes: the fused
    k_update_encode on the stream grid, k_update_tiled_encode on the wide tiles,
    k_update_pipe with the encode's blocks appended on the pipelined tiles."""
    return lib().fleet_update_encode_kernel(length).decode()


def set_plan(spec: str = "") -> None:
    """Launch-plan overrides (fleet_set_plan; process-wide): "update=auto|stream|tiled|pipe",
    "grid=auto|plain|balanced|lanes", "tile=auto|classic|flat|weave6|weave8", "flat_w2=auto|N",
    "tile_enc_prio=auto|0..3", "tile_enc_rows=N", "fused=on|off", "stage_threads=N",
    "stage_pieces=N", comma-separated; "" restores the measured default. Results are
    identical under every plan; an invalid spec raises and changes nothing."""
    err = C.create_string_buffer(256)
    rc = lib().fleet_set_plan(spec.encode(), err, 256)
    if rc != FLEET_OK:
        raise FleetError(rc, err.value.decode())


def plan() -> str:
    """The active launch-plan overrides ("" = the measured default)."""
    return lib().fleet_plan().decode()


class plan_override:
    """Context manager: `with plan_override("update=tiled"): ...` restores the previous plan."""

    def __init__(self, spec: str):
        self.spec = spec

    def __enter__(self):
        self.prev = plan()
        set_plan(self.spec)
        return self

    def __exit__(self, *exc):
        set_plan(self.prev)
        return False


def layout_from_sizes(w_sizes: Sequence[int], b_sizes: Sequence[int]):
    """Header slot positions + n_up of the gradients() layout (network.h:1038-1056)."""
    w = np.ascontiguousarray(w_sizes, dtype=np.int32)
    b = np.ascontiguousarray(b_sizes, dtype=np.int32)
    cap = len(w) + len(b) + 2
    pos = np.empty(cap, np.int32)
    nh = C.c_int(0)
    n_up = C.c_size_t(0)
    rc = lib().fleet_layout_from_sizes(w.ctypes.data, len(w), b.ctypes.data, len(b), pos.ctypes.data, cap,
                                       C.byref(nh), C.byref(n_up))
    if rc != FLEET_OK:
        raise FleetError(rc, "bad layout sizes")
    return pos[: nh.value].copy(), int(n_up.value)


def _stream(stream):
    """Device calls default to torch's current stream so they order with torch ops
    (NULL = the null stream, which is torch's default stream)."""
    if stream is not None:
        return C.c_void_p(int(stream)) if int(stream) else None
    try:
        import torch
        if torch.cuda.is_available():
            h = torch.cuda.current_stream().cuda_stream
            return C.c_void_p(h) if h else None
    except ImportError:
        pass
    return None


def _as_bytes(x) -> bytes:
    if isinstance(x, (bytes, bytearray, memoryview)):
        return bytes(x)
    if isinstance(x, np.ndarray):
        return x.tobytes()
    if isinstance(x, str):
        return x.encode("ascii")
    raise TypeError(f"expected Base64 bytes, got {type(x)}")


class Codec:
    """One HIP device context (``fleet_ctx``). Raises if no GPU / library."""

    def __init__(self, device: int = 0):
        L = lib()
        h = C.c_void_p()
        rc = L.fleet_create(device, C.byref(h))
        if rc != FLEET_OK:
            raise FleetError(rc, f"fleet_create(device={device}) failed: no usable MI355X/HIP device")
        self._h = h
        self._L = L
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            self._L.fleet_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- error plumbing -------------------------------------------------------
    def _check(self, rc: int):
        if rc == FLEET_OK:
            return
        msg = self._L.fleet_last_error(self._h).decode(errors="replace")
        if rc == FLEET_ERR_BASE64:
            raise Base64Error(rc, msg)
        if rc == FLEET_ERR_LAYOUT:
            raise LayoutError(rc, msg)
        raise FleetError(rc, msg)

    def _text_call(self, fn, args, cap):
        out = np.empty(max(cap, 1), np.uint8)
        n = C.c_size_t(0)
        rc = fn(self._h, *args, out.ctypes.data, cap, C.byref(n))
        self._check(rc)
        return out[: n.value].tobytes()

    # -- Base64.cpp -------------------------------------------------------------
    def encode_floats(self, v) -> bytes:
        """Base64::encode(std::vector<float>) (Base64.cpp:104-106)."""
        v = np.ascontiguousarray(v, dtype=np.float32)
        return self._text_call(self._L.fleet_encode_f32, (v.ctypes.data, len(v)), b64_len(len(v)))

    def encode_ints(self, v) -> bytes:
        """Base64::encode(std::vector<int>) (Base64.cpp:109-115)."""
        v = np.ascontiguousarray(v, dtype=np.int32)
        return self._text_call(self._L.fleet_encode_i32, (v.ctypes.data, len(v)), b64_len(len(v)))

    def decode_floats(self, text) -> np.ndarray:
        """Base64::decodeFloat (Base64.cpp:171-173)."""
        s = _as_bytes(text)
        out = np.empty(b64_count(len(s)) + 1, np.float32)
        n = C.c_size_t(0)
        self._check(self._L.fleet_decode_f32(self._h, s, len(s), out.ctypes.data, len(out), C.byref(n)))
        return out[: n.value].copy()

    def decode_ints(self, text) -> np.ndarray:
        """Base64::decodeInt (Base64.cpp:175-183)."""
        s = _as_bytes(text)
        out = np.empty(b64_count(len(s)) + 1, np.int32)
        n = C.c_size_t(0)
        self._check(self._L.fleet_decode_i32(self._h, s, len(s), out.ctypes.data, len(out), C.byref(n)))
        return out[: n.value].copy()

    # -- cppNN_backend.cpp natives (same names as the Java declarations) -------
    def getFlatGradient(self, grad) -> bytes:  # noqa: N802  (CppNNUpdater.java:159)
        s = _as_bytes(grad)
        return self._text_call(self._L.fleet_flat_gradient, (s, len(s)), len(s) + 16)

    def mergeFlatGradient(self, grad, flat) -> bytes:  # noqa: N802  (CppNNUpdater.java:160)
        g, f = _as_bytes(grad), _as_bytes(flat)
        return self._text_call(self._L.fleet_merge_flat_gradient, (g, len(g), f, len(f)), len(g) + 16)

    def scalarMulNative(self, v, a: float) -> bytes:  # noqa: N802  (ByteVec.java:26)
        s = _as_bytes(v)
        return self._text_call(self._L.fleet_scalar_mul, (s, len(s), float(a)), len(s) + 16)

    def addNative(self, a, b) -> bytes:  # noqa: N802  (ByteVec.java:25)
        x, y = _as_bytes(a), _as_bytes(b)
        return self._text_call(self._L.fleet_add, (x, len(x), y, len(y)), len(x) + 16)

    def subtractNative(self, a, b) -> bytes:  # noqa: N802  (ByteVec.java:24)
        x, y = _as_bytes(a), _as_bytes(b)
        return self._text_call(self._L.fleet_subtract, (x, len(x), y, len(y)), len(x) + 16)

    def getNorm(self, v) -> float:  # noqa: N802  (ByteVec.java:23)
        s = _as_bytes(v)
        out = C.c_double(0)
        self._check(self._L.fleet_norm(self._h, s, len(s), C.byref(out)))
        return out.value

    def layout_parse(self, upload):
        s = _as_bytes(upload)
        pos = np.empty(FLEET_MAX_HEADERS, np.int32)
        nh = C.c_int(0)
        n_up = C.c_size_t(0)
        self._check(self._L.fleet_layout_parse(self._h, s, len(s), pos.ctypes.data, FLEET_MAX_HEADERS,
                                               C.byref(nh), C.byref(n_up)))
        return pos[: nh.value].copy(), int(n_up.value)

    # -- fused update ------------------------------------------------------------
    def update(self, uploads: Sequence, dampen: Sequence[float], want_f32: bool = False):
        """Aggregation of CppNNUpdater.update (CppNNUpdater.java:420-509) in one call.

        Returns the merged Base64 (what mergeFlatGradient returns) and, with
        ``want_f32``, Base64::decodeFloat of it (what descentNative decodes).
        """
        ups = [_as_bytes(u) for u in uploads]
        M = len(ups)
        if M == 0:
            raise ValueError("no uploads")
        if len(dampen) != M:
            raise ValueError("one dampening factor per upload")
        arr = (C.c_char_p * M)(*ups)
        lens = np.array([len(u) for u in ups], dtype=np.uint64)
        d = np.ascontiguousarray(dampen, dtype=np.float64)
        L = len(ups[0])
        out = np.empty(L + 16, np.uint8)
        n = C.c_size_t(0)
        f32 = np.empty(b64_count(L) + 1, np.float32) if want_f32 else None
        rc = self._L.fleet_update(self._h, C.cast(arr, C.c_void_p), lens.ctypes.data, M, d.ctypes.data,
                                  out.ctypes.data, len(out), C.byref(n), f32.ctypes.data if want_f32 else None)
        self._check(rc)
        merged = out[: n.value].tobytes()
        if want_f32:
            return merged, f32[: b64_count(L)].copy()
        return merged

    def update_rows(self, rows: np.ndarray, length: int, dampen: Sequence[float], want_f32: bool = False):
        """fleet_update over a uint8 host array [M, row_pitch] whose row i holds upload i's
        `length` Base64 chars; page-locked rows (register_host) go to HBM without a host copy."""
        return update_rows([self], rows, length, dampen, want_f32)

    def register_host(self, arr: np.ndarray):
        """Page-lock a host array for copy-free ingress (fleet_host_register)."""
        self._check(self._L.fleet_host_register(self._h, arr.ctypes.data, arr.nbytes))

    def unregister_host(self, arr: np.ndarray):
        self._check(self._L.fleet_host_unregister(self._h, arr.ctypes.data))

    # -- device-resident (torch tensors on this device) -----------------------
    def update_device(self, uploads_u8, length: int, dampen: Sequence[float], header_pos, merged_u8,
                      merged_f32=None, group_begin: int = 0, group_end: Optional[int] = None, stream=None,
                      window: bool = False):
        """uploads_u8: uint8 CUDA tensor [M, pitch]; merged_u8: uint8 [>= 16*groups].

        window=False: the tensors hold whole rows (group 0 at column 0).
        window=True: they hold only the groups [group_begin, group_end) of every
        row (uploads [M, >= 16*(ge-gb)], merged [16*(ge-gb)], merged_f32
        [3*(ge-gb)]); header_pos stay in whole-upload coordinates."""
        M, pitch = uploads_u8.shape
        groups = (b64_count(length) + 2) // 3
        ge = groups if group_end is None else min(group_end, groups)
        hp = np.ascontiguousarray(header_pos, dtype=np.int32)
        d = np.ascontiguousarray(dampen, dtype=np.float64)
        shift_b = 16 * group_begin if window else 0
        shift_f = 3 * 4 * group_begin if window else 0
        if window:
            w = ge - group_begin
            if pitch < 16 * w or merged_u8.numel() < 16 * w or (merged_f32 is not None and merged_f32.numel() < 3 * w):
                raise ValueError("window tensors smaller than the selected groups")
        rc = self._L.fleet_update_device(self._h, uploads_u8.data_ptr() - shift_b, pitch, length, M, d.ctypes.data,
                                         hp.ctypes.data, len(hp), group_begin, ge, merged_u8.data_ptr() - shift_b,
                                         merged_f32.data_ptr() - shift_f if merged_f32 is not None else None,
                                         _stream(stream))
        self._check(rc)

    def update_encode_device(self, uploads_u8, length: int, dampen: Sequence[float], header_pos, merged_u8,
                             merged_f32, values_f32, next_uploads_u8, stream=None):
        """One pipelined step (fleet_update_encode_device): update_device over the whole
        uploads_u8 [M, pitch] and encode_device of values_f32 [M, vpitch] into
        next_uploads_u8 [M, pitch] (a different buffer), in one launch."""
        M, pitch = uploads_u8.shape
        if tuple(next_uploads_u8.shape) != (M, pitch) or values_f32.shape[0] != M:
            raise ValueError("next_uploads / values must have the uploads' rows and pitch")
        hp = np.ascontiguousarray(header_pos, dtype=np.int32)
        d = np.ascontiguousarray(dampen, dtype=np.float64)
        rc = self._L.fleet_update_encode_device(self._h, uploads_u8.data_ptr(), pitch, length, M, d.ctypes.data,
                                                hp.ctypes.data, len(hp), merged_u8.data_ptr(),
                                                merged_f32.data_ptr() if merged_f32 is not None else None,
                                                values_f32.data_ptr(), values_f32.shape[1],
                                                next_uploads_u8.data_ptr(), _stream(stream))
        self._check(rc)

    def update_kardam_device(self, uploads_u8, length: int, dampen: Sequence[float], header_pos, lr: float,
                             merged_u8, merged_f32=None, prev_f32=None, has_prev=None, g_out_f32=None, stream=None):
        """update_device plus Kardam's per-client norms in the same pass (fleet_update_kardam_device):
        returns (norm_g[M], norm_diff[M]); prev_f32 / g_out_f32: float32 CUDA tensors [M, vpitch]
        of decoded Kardam gradients in upload coordinates (g_out_f32 may be prev_f32 itself:
        this round's G then replaces prev in place)."""
        M, pitch = uploads_u8.shape
        hp = np.ascontiguousarray(header_pos, dtype=np.int32)
        d = np.ascontiguousarray(dampen, dtype=np.float64)
        vpitch = (prev_f32 if prev_f32 is not None else g_out_f32).shape[1] if (
            prev_f32 is not None or g_out_f32 is not None) else 0
        hv = None
        if prev_f32 is not None:
            hv = np.ascontiguousarray(has_prev if has_prev is not None else np.ones(M), dtype=np.uint8)
        ng, nd = np.empty(M, np.float64), np.empty(M, np.float64)
        rc = self._L.fleet_update_kardam_device(
            self._h, uploads_u8.data_ptr(), pitch, length, M, d.ctypes.data, hp.ctypes.data, len(hp), float(lr),
            prev_f32.data_ptr() if prev_f32 is not None else None, hv.ctypes.data if hv is not None else None,
            g_out_f32.data_ptr() if g_out_f32 is not None else None, vpitch, merged_u8.data_ptr(),
            merged_f32.data_ptr() if merged_f32 is not None else None, ng.ctypes.data, nd.ctypes.data,
            _stream(stream))
        self._check(rc)
        return ng, nd

    def test_kardam_skew(self, skew: int) -> None:
        """Test hook: the pipelined Kardam form's reduce blocks wait for a later epoch than
        the tiles publish (skew != 0), so the call fails on their bounded wait."""
        self._check(self._L.fleet_test_kardam_skew(self._h, int(skew)))

    def encode_device(self, values_f32, n: int, out_u8, stream=None):
        """values_f32: float32 CUDA tensor [M, vpitch]; out_u8: uint8 [M, pitch]."""
        M, vpitch = values_f32.shape
        _, pitch = out_u8.shape
        rc = self._L.fleet_encode_device(self._h, values_f32.data_ptr(), n, vpitch, M, out_u8.data_ptr(), pitch,
                                         _stream(stream))
        self._check(rc)

    def decode_device(self, text_u8, length: int, out_f32, stream=None):
        M, pitch = text_u8.shape
        _, vpitch = out_f32.shape
        rc = self._L.fleet_decode_device(self._h, text_u8.data_ptr(), length, pitch, M, out_f32.data_ptr(), vpitch,
                                         _stream(stream))
        self._check(rc)

    def synth_device(self, seed: int, values_f32, n_up: int, header_pos, header_val, client0: int = 0,
                     stream=None, elem0: int = 0):
        """Synthetic buckets (fleet_synth_window_device): rows client0.. of a problem whose
        elements elem0 .. elem0 + n_up this tensor holds; header_pos in its coordinates."""
        M, vpitch = values_f32.shape
        hp = np.ascontiguousarray(header_pos, dtype=np.int32)
        hv = np.ascontiguousarray(header_val, dtype=np.float32)
        rc = self._L.fleet_synth_window_device(self._h, seed, M, client0, elem0, hp.ctypes.data, hv.ctypes.data,
                                               len(hp), n_up, values_f32.data_ptr(), vpitch, _stream(stream))
        self._check(rc)

    def selftest_digest(self, fn: int) -> int:
        """Digest of the device codec arithmetic over a whole input domain (fleet_codec.h)."""
        out = C.c_uint64(0)
        self._check(self._L.fleet_selftest_digest(self._h, fn, C.byref(out)))
        return out.value

    def check(self, stream=None):
        self._check(self._L.fleet_check(self._h, _stream(stream)))

    def sync(self, stream=None):
        self._check(self._L.fleet_sync(self._h, _stream(stream)))

    # -- DISTILLATION_MODE=1 model codec ----------------
    @staticmethod
    def _model_args(weights, dims):
        w = np.ascontiguousarray(weights, dtype=np.float32).reshape(-1)
        d = np.ascontiguousarray(dims, dtype=np.int32).reshape(-1)
        if len(d) % 3:
            raise ValueError("dims: (cols, rows, chans) per matrix")
        n = int(sum(int(d[k]) * int(d[k + 1]) * int(d[k + 2]) for k in range(0, len(d), 3)))
        if len(w) != n:
            raise ValueError(f"{len(w)} weights for a model of {n}")
        return w, d, n

    def model_quantize_index(self, weights, dims):
        """quantization_weight_model + getParams' dictionary and selected-index set
        (network.h:594-692, 1683-1774): (quantised weights, dictionary, indices)."""
        w, d, n = self._model_args(weights, dims)
        wq = np.empty(n, np.float32)
        dic = np.empty(max(1, n), np.float32)
        idx = np.empty(n, np.int32)
        U = C.c_int(0)
        self._check(self._L.fleet_model_quantize_index(self._h, w.ctypes.data, d.ctypes.data, len(d) // 3,
                                                       wq.ctypes.data, dic.ctypes.data, C.byref(U), idx.ctypes.data))
        return wq, dic[: U.value].copy(), idx

    def model_weights_text(self, weights, dims) -> bytes:
        """getParams' DISTILLATION_MODE=1 weights section for these (unquantised) weights."""
        w, d, n = self._model_args(weights, dims)
        need = C.c_size_t(0)
        rc = self._L.fleet_model_weights_text(self._h, w.ctypes.data, d.ctypes.data, len(d) // 3, None, 0,
                                              C.byref(need))
        if rc not in (0, FLEET_ERR_CAPACITY):
            self._check(rc)
        buf = np.empty(max(1, need.value), np.uint8)
        self._check(self._L.fleet_model_weights_text(self._h, w.ctypes.data, d.ctypes.data, len(d) // 3,
                                                     buf.ctypes.data, need.value, C.byref(need)))
        return buf[: need.value].tobytes()

    def model_read_weights(self, text, dims) -> np.ndarray:
        """network::read's DISTILLATION_MODE=1 branch: weights section -> weights."""
        t = _as_bytes(text)
        d = np.ascontiguousarray(dims, dtype=np.int32).reshape(-1)
        n = int(sum(int(d[k]) * int(d[k + 1]) * int(d[k + 2]) for k in range(0, len(d), 3)))
        out = np.empty(n, np.float32)
        self._check(self._L.fleet_model_read_weights(self._h, t, len(t), d.ctypes.data, len(d) // 3,
                                                     out.ctypes.data))
        return out

    def model_version(self, weights, dims, biases):
        """descentNative's mode-1 model copy: read(getParams()) of the unquantised model
        (weights via the first-occurrence dictionary, %g/strtof round trips)."""
        w, d, n = self._model_args(weights, dims)
        b = np.ascontiguousarray(biases, dtype=np.float32).reshape(-1)
        wo = np.empty(n, np.float32)
        bo = np.empty(len(b), np.float32)
        self._check(self._L.fleet_model_version(self._h, w.ctypes.data, d.ctypes.data, len(d) // 3, b.ctypes.data,
                                                len(b), wo.ctypes.data, bo.ctypes.data))
        return wo, bo

    def getModelParametersNative(self, weights, biases, graph_edges: int) -> bytes:  # noqa: N802  (java:148)
        """Base64 of network::getModelParams (cppNN_backend.cpp:227-242): the use_bias() biases repeated
        graph_edges (= layer_graph.size()) times, then the non-null W."""
        w = np.ascontiguousarray(weights, dtype=np.float32).reshape(-1)
        b = np.ascontiguousarray(biases, dtype=np.float32).reshape(-1)
        n = len(b) * int(graph_edges) + len(w)
        return self._text_call(self._L.fleet_model_params, (w.ctypes.data, len(w), b.ctypes.data, len(b),
                                                            int(graph_edges)), b64_len(n))

    # -- Kardam bookkeeping ------------------------------------
    def kardam_grads(self, uploads: Sequence, dampen: Sequence[float], lr: float, prev=None):
        """For the M picked uploads (CppNNUpdater.java:463-481): the texts
        g_c = getFlatGradient(u_c).scalarMultiply(d_c).scalarMultiply(lr), their norms and,
        where prev[c] is given, the norms of g_c.subtract(prev[c]) (else NaN)."""
        ups = [_as_bytes(u) for u in uploads]
        M = len(ups)
        if M == 0 or len(dampen) != M:
            raise ValueError("one dampening factor per upload")
        arr = (C.c_char_p * M)(*ups)
        lens = np.array([len(u) for u in ups], dtype=np.uint64)
        d = np.ascontiguousarray(dampen, dtype=np.float64)
        pv = None
        if prev is not None:
            if len(prev) != M:
                raise ValueError("one previous gradient (or None) per upload")
            pv = (C.c_char_p * M)(*[(_as_bytes(x) if x is not None else None) for x in prev])
        pitch = len(ups[0]) + 16
        g = np.empty((M, pitch), np.uint8)
        glen = C.c_size_t(0)
        ng = np.empty(M, np.float64)
        nd = np.empty(M, np.float64)
        self._check(self._L.fleet_kardam_grads(self._h, C.cast(arr, C.c_void_p), lens.ctypes.data, M, d.ctypes.data,
                                               float(lr), C.cast(pv, C.c_void_p) if pv is not None else None,
                                               g.ctypes.data, pitch, C.byref(glen), ng.ctypes.data, nd.ctypes.data))
        return [g[c, : glen.value].tobytes() for c in range(M)], ng, nd

    # -- getMiniBatch -------------------------------------------
    def getMiniBatch(self, images, labels, idx, header, teacher=None) -> bytes:  # noqa: N802  (cppNN_backend.cpp:677)
        """Base64 of the sampler's mini-batch vector (cppNN_backend.cpp:553-699) for the
        sample indices `idx`: header (7 floats, fleet_amd.sampler.minibatch_header),
        per sample its features, (mode 1) the teacher's probabilities, its label."""
        x = np.ascontiguousarray(images, dtype=np.float32)
        n_img, F = x.shape
        lab = np.ascontiguousarray(labels, dtype=np.int32)
        ix = np.ascontiguousarray(idx, dtype=np.int32)
        h = np.ascontiguousarray(header, dtype=np.float32)
        if len(h) != 7:
            raise ValueError("header holds E, sigma, C, lr, batchSize, featureSize, numLabels")
        t, nl = None, 0
        if teacher is not None:
            t = np.ascontiguousarray(teacher, dtype=np.float32)
            nl = t.shape[1]
            if t.shape[0] != len(ix):
                raise ValueError("one teacher row per sample")
        cap = self._L.fleet_minibatch_len(F, len(ix), nl, t is not None)
        return self._text_call(self._L.fleet_minibatch, (x.ctypes.data, n_img, F, lab.ctypes.data, ix.ctypes.data,
                                                         len(ix), t.ctypes.data if t is not None else None, nl,
                                                         h.ctypes.data), cap)

    def minibatch_device(self, images_f32, labels_i32, idx_i32, header, out_u8, teacher_f32=None, stream=None):
        """Device-resident getMiniBatch: CUDA tensors images [N, F], labels [N], idx [B],
        out uint8 [>= fleet_minibatch_len]. Index errors surface at check()."""
        n_img, F = images_f32.shape
        h = np.ascontiguousarray(header, dtype=np.float32)
        nl = teacher_f32.shape[1] if teacher_f32 is not None else 0
        self._check(self._L.fleet_minibatch_device(self._h, images_f32.data_ptr(), n_img, F, labels_i32.data_ptr(),
                                                   idx_i32.data_ptr(), idx_i32.numel(),
                                                   teacher_f32.data_ptr() if teacher_f32 is not None else None, nl,
                                                   h.ctypes.data, out_u8.data_ptr(), _stream(stream)))

    # -- the sampler's mode-1 teacher forward ----------------
    def teacher_forward(self, w, b, images, idx=None, temperature: float = 2.0) -> np.ndarray:
        """uniformSample's teacher.forward(sample, TEMPERATURE, -1, 1) (cppNN_backend.cpp:603)
        for images[idx] (all rows when idx is None): [B, 10] class probabilities of
        initSampler's teacher network with weights w (non-null W in network order) and
        biases b (use_bias() layers in layer order)."""
        wv = np.ascontiguousarray(w, dtype=np.float32).reshape(-1)
        bv = np.ascontiguousarray(b, dtype=np.float32).reshape(-1)
        x = np.ascontiguousarray(images, dtype=np.float32)
        if x.ndim == 1:
            x = x.reshape(1, -1)
        n_img, F = x.shape
        ix = np.arange(n_img, dtype=np.int32) if idx is None else np.ascontiguousarray(idx, dtype=np.int32)
        out = np.empty((len(ix), 10), np.float32)
        self._check(self._L.fleet_teacher_forward(self._h, wv.ctypes.data, len(wv), bv.ctypes.data, len(bv),
                                                  x.ctypes.data, n_img, F, ix.ctypes.data, len(ix),
                                                  float(temperature), out.ctypes.data))
        return out

    def teacher_forward_device(self, w_f32, b_f32, images_f32, probs_f32, idx_i32=None, temperature: float = 2.0,
                               stream=None):
        """Device-resident teacher forward: CUDA tensors w [21448], b [82], images [N, F >= 784],
        probs [B, 10] written for images[idx] (B = N rows when idx is None). Index errors at check()."""
        n_img, F = images_f32.shape
        if w_f32.numel() != self._L.fleet_teacher_weight_count() or b_f32.numel() != self._L.fleet_teacher_bias_count():
            raise ValueError("teacher weights / biases of the wrong size")
        B = idx_i32.numel() if idx_i32 is not None else n_img
        if probs_f32.numel() < 10 * B:
            raise ValueError("probs holds B x 10 floats")
        self._check(self._L.fleet_teacher_forward_device(self._h, w_f32.data_ptr(), b_f32.data_ptr(),
                                                         images_f32.data_ptr(), n_img, F,
                                                         idx_i32.data_ptr() if idx_i32 is not None else None, B,
                                                         float(temperature), probs_f32.data_ptr(), _stream(stream)))

    # -- descentNative's model step ----------------------------
    @staticmethod
    def _layout_args(layout):
        ws = np.ascontiguousarray(layout.w_sizes, dtype=np.int32)
        wp = np.ascontiguousarray(layout.w_present(), dtype=np.uint8)
        bs = np.ascontiguousarray(layout.b_sizes, dtype=np.int32)
        fc = np.ascontiguousarray(layout.fc_flags(), dtype=np.uint8)
        return ws, wp, bs, fc

    def descent(self, weights, fc_bias, grad, layout, lr: float):
        """network::descent(vector) with the sgd solver (cppNN_backend.cpp:336-352): returns the
        updated (weights, fc_bias); `grad` = decodeFloat(merged) in the layout's gradients() order."""
        w = np.array(weights, dtype=np.float32, copy=True).reshape(-1)
        b = np.array(fc_bias, dtype=np.float32, copy=True).reshape(-1)
        g = np.ascontiguousarray(grad, dtype=np.float32).reshape(-1)
        ws, wp, bs, fc = self._layout_args(layout)
        self._check(self._L.fleet_descent(self._h, w.ctypes.data, len(w), b.ctypes.data, len(b), g.ctypes.data,
                                          len(g), ws.ctypes.data, wp.ctypes.data, len(ws), bs.ctypes.data,
                                          fc.ctypes.data, len(bs), float(lr)))
        return w, b

    def descent_window_device(self, weights_f32, fc_bias_f32, grad_window_f32, value_begin: int, value_end: int,
                              layout, lr: float, stream=None):
        """The model step of one element shard: grad_window_f32 holds the merged fp32 values
        [value_begin, value_end); only the parameters those positions cover are updated."""
        ws, wp, bs, fc = self._layout_args(layout)
        self._check(self._L.fleet_descent_window_device(self._h, weights_f32.data_ptr(),
                                                        fc_bias_f32.data_ptr() if fc_bias_f32 is not None else None,
                                                        grad_window_f32.data_ptr(), int(value_begin), int(value_end),
                                                        ws.ctypes.data, wp.ctypes.data, len(ws), bs.ctypes.data,
                                                        fc.ctypes.data, len(bs), float(lr), _stream(stream)))

    def descent_device(self, weights_f32, fc_bias_f32, grad_f32, layout, lr: float, stream=None):
        """Device-resident model step: float32 CUDA tensors updated in place."""
        ws, wp, bs, fc = self._layout_args(layout)
        self._check(self._L.fleet_descent_device(self._h, weights_f32.data_ptr(),
                                                 fc_bias_f32.data_ptr() if fc_bias_f32 is not None else None,
                                                 grad_f32.data_ptr(), ws.ctypes.data, wp.ctypes.data, len(ws),
                                                 bs.ctypes.data, fc.ctypes.data, len(bs), float(lr),
                                                 _stream(stream)))


def update_multi(codecs: Sequence["Codec"], uploads: Sequence, dampen: Sequence[float], want_f32: bool = False):
    """Codec.update spread over several device contexts from one process
    (fleet_update_multi): context k aggregates a contiguous range of the 3-value
    groups of every upload and writes its slice of the output; byte-identical to
    one context's update. The first context reports errors."""
    if not codecs:
        raise ValueError("no contexts")
    ups = [_as_bytes(u) for u in uploads]
    M = len(ups)
    if M == 0:
        raise ValueError("no uploads")
    if len(dampen) != M:
        raise ValueError("one dampening factor per upload")
    L = lib()
    arr = (C.c_char_p * M)(*ups)
    lens = np.array([len(u) for u in ups], dtype=np.uint64)
    d = np.ascontiguousarray(dampen, dtype=np.float64)
    hs = (C.c_void_p * len(codecs))(*[c._h for c in codecs])
    n_len = len(ups[0])
    out = np.empty(n_len + 16, np.uint8)
    n = C.c_size_t(0)
    f32 = np.empty(b64_count(n_len) + 1, np.float32) if want_f32 else None
    rc = L.fleet_update_multi(C.cast(hs, C.c_void_p), len(codecs), C.cast(arr, C.c_void_p), lens.ctypes.data, M,
                              d.ctypes.data, out.ctypes.data, len(out), C.byref(n),
                              f32.ctypes.data if want_f32 else None)
    codecs[0]._check(rc)
    merged = out[: n.value].tobytes()
    if want_f32:
        return merged, f32[: b64_count(n_len)].copy()
    return merged


def update_rows(codecs: Sequence["Codec"], rows: np.ndarray, length: int, dampen: Sequence[float],
                want_f32: bool = False):
    """fleet_update_rows(_multi): the update over uploads stored as the rows of one host
    array (rows[i, :length] = upload i), on one or several device contexts."""
    if rows.ndim != 2 or rows.dtype != np.uint8 or not rows.flags.c_contiguous:
        raise ValueError("rows: a C-contiguous uint8 array [M, row_pitch]")
    M, pitch = rows.shape
    if len(dampen) != M:
        raise ValueError("one dampening factor per upload")
    d = np.ascontiguousarray(dampen, dtype=np.float64)
    out = np.empty(length + 16, np.uint8)
    n = C.c_size_t(0)
    f32 = np.empty(b64_count(length) + 1, np.float32) if want_f32 else None
    L = lib()
    if len(codecs) == 1:
        rc = L.fleet_update_rows(codecs[0]._h, rows.ctypes.data, pitch, length, M, d.ctypes.data, out.ctypes.data,
                                 len(out), C.byref(n), f32.ctypes.data if want_f32 else None)
    else:
        hs = (C.c_void_p * len(codecs))(*[c._h for c in codecs])
        rc = L.fleet_update_rows_multi(C.cast(hs, C.c_void_p), len(codecs), rows.ctypes.data, pitch, length, M,
                                       d.ctypes.data, out.ctypes.data, len(out), C.byref(n),
                                       f32.ctypes.data if want_f32 else None)
    codecs[0]._check(rc)
    merged = out[: n.value].tobytes()
    if want_f32:
        return merged, f32[: b64_count(length)].copy()
    return merged


class Model:
    """The server's resident model (fleet_model): the state the reference's updater
    natives keep in libnative.so (cppNN_backend.cpp: cnn, models, lrates_vec,
    currEpoch, priority), with the natives' names as methods."""

    def __init__(self, codec: "Codec", params_text, distillation_mode: int = 1):
        """fetchParamsNative (cppNN_backend.cpp:282-301): network::read of a getParams text."""
        t = _as_bytes(params_text)
        h = C.c_void_p()
        rc = codec._L.fleet_model_load(codec._h, t, len(t), int(distillation_mode), C.byref(h))
        if rc != FLEET_OK:
            raise FleetError(rc, "fleet_model_load failed (see stderr): not a supported getParams text")
        self._h, self._L, self.codec = h, codec._L, codec

    def close(self):
        if getattr(self, "_h", None):
            self._L.fleet_model_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != FLEET_OK:
            msg = self._L.fleet_model_last_error(self._h).decode(errors="replace")
            raise (LayoutError if rc == FLEET_ERR_LAYOUT else Base64Error if rc == FLEET_ERR_BASE64 else FleetError)(rc, msg)

    def _text(self, fn, version):
        need = C.c_size_t(0)
        rc = fn(self._h, int(version), None, 0, C.byref(need))
        if rc not in (FLEET_OK, FLEET_ERR_CAPACITY):
            self._check(rc)
        out = np.empty(max(1, need.value), np.uint8)
        self._check(fn(self._h, int(version), out.ctypes.data, need.value, C.byref(need)))
        return out[: need.value].tobytes()

    def initUpdater(self, lrates) -> None:  # noqa: N802  (cppNN_backend.cpp:161-225, model part)
        lr = np.ascontiguousarray(lrates, dtype=np.float64)
        self._check(self._L.fleet_model_init_updater(self._h, lr.ctypes.data, len(lr)))

    def descentNative(self, merged, client_batch_size: int, stale_size: int) -> None:  # noqa: N802  (:329-383)
        m = _as_bytes(merged)
        self._check(self._L.fleet_model_descent(self._h, m, len(m), int(client_batch_size), int(stale_size)))

    def modelsSize(self) -> int:  # noqa: N802  (:324-327)
        return self._L.fleet_model_count(self._h)

    def getParametersNative(self, priority: int) -> bytes:  # noqa: N802  (:244-280)
        return self._text(self._L.fleet_model_get_params, priority)

    def getModelParametersNative(self, priority: int) -> bytes:  # noqa: N802  (:227-242)
        return self._text(self._L.fleet_model_get_model_params, priority)

    def getCurrEpoch(self) -> int:  # noqa: N802
        return self._L.fleet_model_get_epoch(self._h)

    def setCurrEpoch(self, e: int) -> None:  # noqa: N802
        self._L.fleet_model_set_epoch(self._h, int(e))

    def getPriority(self) -> int:  # noqa: N802
        return self._L.fleet_model_get_priority(self._h)

    def setPriority(self, p: int) -> None:  # noqa: N802
        self._L.fleet_model_set_priority(self._h, int(p))

    def getLrate(self) -> float:  # noqa: N802
        return self._L.fleet_model_get_lrate(self._h)

    def shape(self):
        nw, nb = C.c_size_t(0), C.c_size_t(0)
        ge, nl = C.c_int(0), C.c_int(0)
        self._check(self._L.fleet_model_shape(self._h, C.byref(nw), C.byref(nb), C.byref(ge), C.byref(nl)))
        return nw.value, nb.value, ge.value, nl.value

    def export(self, version: int = -1):
        """(weights, biases) of models[version]; version -1 = the current model."""
        nw, nb, _, _ = self.shape()
        w, b = np.empty(nw, np.float32), np.empty(nb, np.float32)
        self._check(self._L.fleet_model_export(self._h, int(version), w.ctypes.data, nw, b.ctypes.data, nb))
        return w, b


class ByteVec:
    """Mirror of Server/src/main/java/utils/ByteVec.java: a Base64 vector whose
    arithmetic runs through the natives (here: the HIP codec)."""

    def __init__(self, v, codec: Codec):
        self.v = _as_bytes(v)  # ByteVec.java:33-35 clones
        self.codec = codec

    def add(self, other: "ByteVec") -> "ByteVec":  # :85-88
        return ByteVec(self.codec.addNative(self.v, other.v), self.codec)

    def subtract(self, other: "ByteVec") -> "ByteVec":  # :96-99
        return ByteVec(self.codec.subtractNative(self.v, other.v), self.codec)

    def scalarMultiply(self, a: float) -> "ByteVec":  # noqa: N802  :121-123
        return ByteVec(self.codec.scalarMulNative(self.v, a), self.codec)

    def getNorm(self) -> float:  # noqa: N802  :69-71
        return self.codec.getNorm(self.v)
