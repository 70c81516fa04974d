"""oracle/pyoracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for
  * ``liboracle.so``         -- the clean-room C restatement (fleet_oracle.c), and
  * ``_ref/libfleetref_model.so`` -- the reference's own header-only mojo network
                                (commonLib/cppNN) compiled by oracle/Makefile (present
                                only where /root/reference was available at build time).
The reference's codec (Base64.cpp) and JNI backend (cppNN_backend.cpp) include
<jni.h>, which this image lacks: they have no reference build here.

Only tests/, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of bench.py
import this module. The product package (fleet_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
ORACLE_O0_SO = os.path.join(HERE, "liboracle_O0.so")  # same source at -O0 (bench.py's faithful CPU leg)
REF_MODEL_SO = os.path.join(HERE, "_ref", "libfleetref_model.so")
SAMPLER_SO = os.path.join(HERE, "libsampler_oracle.so")  # initSampler's buckets (sampler_oracle.cpp)

_c_char_pp = C.POINTER(C.c_char_p)


def build(force: bool = False) -> None:
    """Compile liboracle.so (and the reference build when /root/reference exists)."""
    if force or not all(os.path.exists(p) for p in (ORACLE_SO, ORACLE_O0_SO, SAMPLER_SO)):
        subprocess.check_call(["make", "-s", "liboracle.so", "liboracle_O0.so", "libsampler_oracle.so"], cwd=HERE)
    if os.path.isdir("/root/reference/Server") and (force or not os.path.exists(REF_MODEL_SO)):
        subprocess.check_call(["make", "-s", "ref"], cwd=HERE)


def _u8(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def _f32(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _i32(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def _f64(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def b64_len(n_values: int) -> int:
    return 4 * ((4 * n_values + 2) // 3)


class Oracle:
    """The C restatement (fleet_oracle.c)."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(ORACLE_SO) or not os.path.exists(path):
            build()
        L = C.CDLL(path)
        self.lib = L
        sz = C.c_size_t
        L.fo_float2int.restype = C.c_int32
        L.fo_float2int.argtypes = [C.c_float]
        L.fo_int2float.restype = C.c_float
        L.fo_int2float.argtypes = [C.c_int32]
        L.fo_encode_floats.restype = sz
        L.fo_encode_floats.argtypes = [C.c_void_p, sz, C.c_void_p]
        L.fo_encode_ints.restype = sz
        L.fo_encode_ints.argtypes = [C.c_void_p, sz, C.c_void_p]
        L.fo_decode_floats.restype = sz
        L.fo_decode_floats.argtypes = [C.c_void_p, sz, C.c_void_p]
        L.fo_decode_ints.restype = sz
        L.fo_decode_ints.argtypes = [C.c_void_p, sz, C.c_void_p]
        for name in ("fo_flat_gradient",):
            getattr(L, name).restype = sz
            getattr(L, name).argtypes = [C.c_void_p, sz, C.c_void_p]
        L.fo_merge_flat_gradient.restype = sz
        L.fo_merge_flat_gradient.argtypes = [C.c_void_p, sz, C.c_void_p, sz, C.c_void_p]
        L.fo_scalar_mul.restype = sz
        L.fo_scalar_mul.argtypes = [C.c_void_p, sz, C.c_double, C.c_void_p]
        L.fo_norm.restype = C.c_double
        L.fo_norm.argtypes = [C.c_void_p, sz]
        for name in ("fo_add", "fo_subtract"):
            getattr(L, name).restype = sz
            getattr(L, name).argtypes = [C.c_void_p, sz, C.c_void_p, sz, C.c_void_p]
        L.fo_update_faithful.restype = sz
        L.fo_update_faithful.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.fo_update_fused.restype = sz
        L.fo_update_fused.argtypes = [C.c_void_p, sz, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_int]
        L.fo_layout_n_up.restype = sz
        L.fo_layout_n_up.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int]
        L.fo_layout_header_mask.restype = None
        L.fo_layout_header_mask.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
        L.fo_synth_value.restype = C.c_float
        L.fo_synth_value.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32]
        L.fo_synth_upload.restype = None
        L.fo_synth_upload.argtypes = [C.c_uint64, C.c_uint32, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                      C.c_void_p]
        L.fo_philox4x32_10.restype = None
        L.fo_philox4x32_10.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.fo_quantize_matrix.restype = None
        L.fo_quantize_matrix.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
        L.fo_dictionary.restype = C.c_int
        L.fo_dictionary.argtypes = [C.c_void_p, sz, C.c_void_p, C.c_void_p]
        L.fo_weights_section.restype = sz
        L.fo_weights_section.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, sz]
        L.fo_read_weights_section.restype = C.c_int
        L.fo_read_weights_section.argtypes = [C.c_void_p, sz, C.c_void_p, C.c_int, C.c_void_p]
        L.fo_descent.restype = C.c_int
        L.fo_descent.argtypes = [C.c_void_p, sz, C.c_void_p, sz, C.c_void_p, sz, C.c_void_p, C.c_int, C.c_void_p,
                                 C.c_int, C.c_float]
        L.fo_teacher_forward.restype = None
        L.fo_teacher_forward.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_void_p]
        L.fo_expf_digest.restype = C.c_uint64
        L.fo_expf_digest.argtypes = []

    # -- scalars / vectors ------------------------------------------------
    def float2int(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        return np.array([self.lib.fo_float2int(float(v)) for v in x], dtype=np.int32)

    def int2float(self, c: np.ndarray) -> np.ndarray:
        c = np.ascontiguousarray(c, dtype=np.int32)
        return np.array([self.lib.fo_int2float(int(v)) for v in c], dtype=np.float32)

    def encode_floats(self, v: np.ndarray) -> bytes:
        v = np.ascontiguousarray(v, dtype=np.float32)
        out = np.empty(b64_len(len(v)) + 4, np.uint8)
        n = self.lib.fo_encode_floats(v.ctypes.data, len(v), out.ctypes.data)
        return out[:n].tobytes()

    def encode_ints(self, v: np.ndarray) -> bytes:
        v = np.ascontiguousarray(v, dtype=np.int32)
        out = np.empty(b64_len(len(v)) + 4, np.uint8)
        n = self.lib.fo_encode_ints(v.ctypes.data, len(v), out.ctypes.data)
        return out[:n].tobytes()

    def decode_floats(self, s: bytes) -> np.ndarray:
        out = np.empty(len(s) // 4 * 3 + 4, np.float32)
        n = self.lib.fo_decode_floats(s, len(s), out.ctypes.data)
        return out[:n].copy()

    def decode_ints(self, s: bytes) -> np.ndarray:
        out = np.empty(len(s) // 4 * 3 + 4, np.int32)
        n = self.lib.fo_decode_ints(s, len(s), out.ctypes.data)
        return out[:n].copy()

    # -- JNI ops ------------------------------------------------------------
    def _buf(self, nbytes):
        return np.empty(nbytes + 64, np.uint8)

    def flat_gradient(self, g: bytes) -> bytes:
        out = self._buf(len(g))
        n = self.lib.fo_flat_gradient(g, len(g), out.ctypes.data)
        if n == C.c_size_t(-1).value:
            raise ValueError("malformed upload")
        return out[:n].tobytes()

    def merge_flat_gradient(self, g: bytes, flat: bytes) -> bytes:
        out = self._buf(len(g))
        n = self.lib.fo_merge_flat_gradient(g, len(g), flat, len(flat), out.ctypes.data)
        if n == C.c_size_t(-1).value:
            raise ValueError("malformed upload")
        return out[:n].tobytes()

    def scalar_mul(self, v: bytes, a: float) -> bytes:
        out = self._buf(len(v))
        n = self.lib.fo_scalar_mul(v, len(v), a, out.ctypes.data)
        return out[:n].tobytes()

    def add(self, a: bytes, b: bytes) -> bytes:
        out = self._buf(len(a))
        n = self.lib.fo_add(a, len(a), b, len(b), out.ctypes.data)
        return out[:n].tobytes()

    def subtract(self, a: bytes, b: bytes) -> bytes:
        out = self._buf(len(a))
        n = self.lib.fo_subtract(a, len(a), b, len(b), out.ctypes.data)
        return out[:n].tobytes()

    def norm(self, v: bytes) -> float:
        return self.lib.fo_norm(v, len(v))

    def update_faithful(self, uploads, dampen) -> bytes:
        M = len(uploads)
        arr = (C.c_char_p * M)(*uploads)
        lens = np.array([len(u) for u in uploads], dtype=np.uint64)
        d = np.ascontiguousarray(dampen, dtype=np.float64)
        out = self._buf(max(len(u) for u in uploads))
        n = self.lib.fo_update_faithful(C.cast(arr, C.c_void_p), lens.ctypes.data, M, d.ctypes.data,
                                        out.ctypes.data)
        if n == C.c_size_t(-1).value:
            raise ValueError("malformed upload")
        return out[:n].tobytes()

    def update_fused(self, uploads, dampen, header_mask, threads: int = 0, want_f32: bool = False):
        M = len(uploads)
        arr = (C.c_char_p * M)(*uploads)
        d = np.ascontiguousarray(dampen, dtype=np.float64)
        L = len(uploads[0])
        out = self._buf(L)
        hm = np.ascontiguousarray(header_mask, dtype=np.uint8)
        f32 = np.empty(len(hm), np.float32) if want_f32 else None
        n = self.lib.fo_update_fused(C.cast(arr, C.c_void_p), L, M, d.ctypes.data, hm.ctypes.data,
                                     out.ctypes.data, f32.ctypes.data if want_f32 else None, threads)
        if n == C.c_size_t(-1).value:
            raise ValueError("malformed upload")
        return (out[:n].tobytes(), f32) if want_f32 else out[:n].tobytes()

    # -- layout / synthetic ---------------------------------------------------
    def header_mask(self, w_sizes, b_sizes) -> np.ndarray:
        w = np.ascontiguousarray(w_sizes, dtype=np.int32)
        b = np.ascontiguousarray(b_sizes, dtype=np.int32)
        n = self.lib.fo_layout_n_up(w.ctypes.data, len(w), b.ctypes.data, len(b))
        m = np.empty(n, np.uint8)
        self.lib.fo_layout_header_mask(w.ctypes.data, len(w), b.ctypes.data, len(b), m.ctypes.data)
        return m

    def synth_upload(self, seed: int, client: int, w_sizes, b_sizes) -> np.ndarray:
        w = np.ascontiguousarray(w_sizes, dtype=np.int32)
        b = np.ascontiguousarray(b_sizes, dtype=np.int32)
        n = self.lib.fo_layout_n_up(w.ctypes.data, len(w), b.ctypes.data, len(b))
        out = np.empty(n, np.float32)
        self.lib.fo_synth_upload(seed, client, w.ctypes.data, len(w), b.ctypes.data, len(b), out.ctypes.data)
        return out

    # -- DISTILLATION_MODE=1 model codec -----------
    def quantize(self, w, dims) -> np.ndarray:
        """quantization_weight_model over the concatenated matrices (dims: [(cols, rows, chans)])."""
        w = np.array(w, dtype=np.float32, copy=True)
        off = 0
        for c, r, ch in dims:
            n = c * r * ch
            seg = np.ascontiguousarray(w[off:off + n])
            self.lib.fo_quantize_matrix(seg.ctypes.data, c, r, ch)
            w[off:off + n] = seg
            off += n
        return w

    def dictionary(self, w):
        w = np.ascontiguousarray(w, dtype=np.float32)
        d = np.empty(max(1, len(w)), np.float32)
        idx = np.empty(max(1, len(w)), np.int32)
        U = self.lib.fo_dictionary(w.ctypes.data, len(w), d.ctypes.data, idx.ctypes.data)
        return d[:U].copy(), idx[: len(w)].copy()

    def weights_section(self, wq, dims) -> bytes:
        wq = np.ascontiguousarray(wq, dtype=np.float32)
        dm = np.ascontiguousarray(dims, dtype=np.int32).reshape(-1)
        n = self.lib.fo_weights_section(wq.ctypes.data, dm.ctypes.data, len(dm) // 3, None, 0)
        buf = np.empty(n, np.uint8)
        self.lib.fo_weights_section(wq.ctypes.data, dm.ctypes.data, len(dm) // 3, buf.ctypes.data, n)
        return buf.tobytes()

    def read_weights_section(self, text: bytes, dims) -> np.ndarray:
        dm = np.ascontiguousarray(dims, dtype=np.int32).reshape(-1)
        n = int(sum(c * r * ch for c, r, ch in np.asarray(dims).reshape(-1, 3)))
        out = np.empty(n, np.float32)
        if self.lib.fo_read_weights_section(text, len(text), dm.ctypes.data, len(dm) // 3, out.ctypes.data):
            raise ValueError("malformed weights section")
        return out

    def descent(self, weights, fc_bias, g, w_present, fc_layer, lr):
        """descentNative's model step (fo_descent): returns the updated (weights, fc_bias)."""
        w = np.array(weights, dtype=np.float32, copy=True)
        b = np.array(fc_bias, dtype=np.float32, copy=True)
        g = np.ascontiguousarray(g, dtype=np.float32)
        wp = np.ascontiguousarray(w_present, dtype=np.uint8)
        fl = np.ascontiguousarray(fc_layer, dtype=np.uint8)
        rc = self.lib.fo_descent(w.ctypes.data, len(w), b.ctypes.data, len(b), g.ctypes.data, len(g), wp.ctypes.data,
                                 len(wp), fl.ctypes.data, len(fl), float(lr))
        if rc != 0:
            raise ValueError("gradient header does not fit the model")
        return w, b

    def teacher_forward(self, w, b, x, temperature: float = 2.0) -> np.ndarray:
        """fo_teacher_forward per sample: [B, 784] inputs -> [B, 10] probabilities."""
        w = np.ascontiguousarray(w, dtype=np.float32)
        b = np.ascontiguousarray(b, dtype=np.float32)
        x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1, 784)
        out = np.empty((x.shape[0], 10), np.float32)
        for i in range(x.shape[0]):
            self.lib.fo_teacher_forward(w.ctypes.data, b.ctypes.data, x[i].ctypes.data, temperature, out[i].ctypes.data)
        return out

    def expf_digest(self) -> int:
        """The libm expf digest over all 2^32 inputs (fn 18 of the device self-test)."""
        return int(self.lib.fo_expf_digest())

    def philox(self, ctr, key):
        c = np.ascontiguousarray(ctr, dtype=np.uint32)
        k = np.ascontiguousarray(key, dtype=np.uint32)
        o = np.empty(4, np.uint32)
        self.lib.fo_philox4x32_10(c.ctypes.data, k.ctypes.data, o.ctypes.data)
        return o


def minibatch_vector(images, labels, idx, header, teacher=None) -> np.ndarray:
    """The float vector uniformSample / nonIIDSample build (cppNN_backend.cpp:
    553-675): the 7 header values, then per sample its F features, (mode 1) the
    teacher's numLabels probabilities, and its label as float; mode 1 appends
    1234567. `header` = (E, sigma, C, lr, batchSize, featureSize, numLabels)
    already in float, as push_back converts them."""
    images = np.asarray(images, dtype=np.float32)
    parts = [np.asarray(header, dtype=np.float32)]
    for b, i in enumerate(idx):
        parts.append(images[i])
        if teacher is not None:
            parts.append(np.asarray(teacher[b], dtype=np.float32))
        parts.append(np.array([labels[i]], dtype=np.float32))
    if teacher is not None:
        parts.append(np.array([1234567], dtype=np.float32))
    return np.concatenate(parts)


class ReferenceModel:
    """The reference's own DISTILLATION_MODE=1 model codec (oracle/_ref/libfleetref_model.so:
    the header-only mojo network of commonLib/cppNN, compiled by oracle/Makefile)."""

    def __init__(self, path: str = REF_MODEL_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = C.CDLL(path)
        self.lib = L
        sz = C.c_size_t
        L.ref_quantize_params.restype = sz
        L.ref_quantize_params.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, sz]
        L.ref_mnist_roundtrip.restype = sz
        L.ref_mnist_roundtrip.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_void_p, sz]
        L.ref_mnist_version_copy.restype = None
        L.ref_mnist_version_copy.argtypes = [C.c_void_p] * 4
        L.ref_mnist_model_params.restype = C.c_int
        L.ref_mnist_model_params.argtypes = [C.c_void_p] * 4
        L.ref_server_session.restype = sz
        L.ref_server_session.argtypes = [C.c_char_p, sz, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.c_void_p, sz]
        L.ref_teacher_forward.restype = C.c_int
        L.ref_teacher_forward.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.ref_mnist_descent.restype = C.c_int
        L.ref_mnist_descent.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_float] + [C.c_void_p] * 9

    def quantize_params(self, w, dims):
        """(quantised weights, getParams text) of a network whose W are the given matrices."""
        w = np.ascontiguousarray(w, dtype=np.float32)
        dm = np.ascontiguousarray(dims, dtype=np.int32).reshape(-1)
        wq = np.empty_like(w)
        n = self.lib.ref_quantize_params(w.ctypes.data, dm.ctypes.data, len(dm) // 3, None, None, 0)
        buf = np.empty(n, np.uint8)
        self.lib.ref_quantize_params(w.ctypes.data, dm.ctypes.data, len(dm) // 3, wq.ctypes.data,
                                     buf.ctypes.data, n)
        return wq, buf.tobytes()

    def mnist_roundtrip(self, w_in=None):
        """The Driver's MNIST network: dims, initial W, quantised W, getParams text, W read back."""
        nm = C.c_int(0)
        dims = np.zeros(48, np.int32)
        n_text = self.lib.ref_mnist_roundtrip(None, C.byref(nm), dims.ctypes.data, None, None, None, None, 0)
        dims = dims[: 3 * nm.value].reshape(-1, 3)
        n = int(sum(int(c) * int(r) * int(ch) for c, r, ch in dims))
        win = None if w_in is None else np.ascontiguousarray(w_in, dtype=np.float32)
        w0 = np.empty(n, np.float32)
        wq = np.empty(n, np.float32)
        wr = np.empty(n, np.float32)
        if win is not None:
            n_text = self.lib.ref_mnist_roundtrip(win.ctypes.data, C.byref(nm), None, None, None, None, None, 0)
        buf = np.empty(n_text, np.uint8)
        self.lib.ref_mnist_roundtrip(None if win is None else win.ctypes.data, C.byref(nm), None, w0.ctypes.data,
                                     wq.ctypes.data, wr.ctypes.data, buf.ctypes.data, n_text)
        return [tuple(int(v) for v in d) for d in dims], w0, wq, buf.tobytes(), wr

    def mnist_descent(self, g=None, lr=0.01, w_in=None, b_in=None):
        """descentNative's model step on the Driver's MNIST network (ref_mnist_descent):
        dict with the gradients() layout (w_sizes, b_sizes), per layer the FC flag and
        bias length (0 without use_bias()), the non-null W and the use_bias() biases
        (concatenated in layer order) before (w0, b0) and after (w1, b1)."""
        nw, nb = C.c_int(0), C.c_int(0)
        ws, bs, fc = np.zeros(64, np.int32), np.zeros(64, np.int32), np.zeros(64, np.int32)
        w0 = np.empty(1 << 16, np.float32)
        b0 = np.empty(1 << 16, np.float32)
        nl = self.lib.ref_mnist_descent(None, None, None, 0, 0.0, C.byref(nw), ws.ctypes.data, C.byref(nb),
                                        bs.ctypes.data, w0.ctypes.data, b0.ctypes.data, None, None, fc.ctypes.data)
        out = {"w_sizes": ws[: nw.value].copy(), "b_sizes": bs[: nb.value].copy(), "fc": fc[:nl] & 1,
               "bias_len": fc[:nl] >> 1}
        if g is None:
            return out
        g = np.ascontiguousarray(g, dtype=np.float32)
        win = None if w_in is None else np.ascontiguousarray(w_in, dtype=np.float32)
        bin_ = None if b_in is None else np.ascontiguousarray(b_in, dtype=np.float32)
        w1 = np.empty_like(w0)
        b1 = np.empty_like(b0)
        self.lib.ref_mnist_descent(None if win is None else win.ctypes.data,
                                   None if bin_ is None else bin_.ctypes.data, g.ctypes.data, len(g), float(lr),
                                   None, None, None, None, w0.ctypes.data, b0.ctypes.data, w1.ctypes.data,
                                   b1.ctypes.data, None)
        out.update(w0=w0, b0=b0, w1=w1, b1=b1)
        return out

    def mnist_model_params(self, w_in=None, b_in=None):
        """network::getModelParams of the MNIST network: (vector, layer_graph.size())."""
        e = C.c_int(0)
        n = self.lib.ref_mnist_model_params(None, None, None, C.byref(e))
        out = np.empty(n, np.float32)
        win = None if w_in is None else np.ascontiguousarray(w_in, dtype=np.float32)
        bin_ = None if b_in is None else np.ascontiguousarray(b_in, dtype=np.float32)
        self.lib.ref_mnist_model_params(None if win is None else win.ctypes.data,
                                        None if bin_ is None else bin_.ctypes.data, out.ctypes.data, C.byref(e))
        return out, e.value

    def server_session(self, text: bytes, lrates, grads, batch: int = 8, stale: int = 2):
        """The updater's model natives replayed on the reference network
        (ref_server_session): fetchParamsNative(text), initUpdater(lrates), one
        descentNative per merged gradient (decoded floats). Returns
        ([(newest_text, newest_params, oldest_text, oldest_params)] after init and
        each step, models.size())."""
        lr = np.ascontiguousarray(lrates, dtype=np.float64)
        g = np.ascontiguousarray(np.stack(grads) if len(grads) else np.zeros((0, 1)), dtype=np.float32)
        n_g = g.shape[1] if len(grads) else 0
        args = (text, len(text), lr.ctypes.data, len(lr), g.ctypes.data, n_g, len(grads), batch, stale)
        n = self.lib.ref_server_session(*args, None, 0)
        buf = np.empty(n, np.uint8)
        self.lib.ref_server_session(*args, buf.ctypes.data, n)
        raw = buf.tobytes()
        pos, states = 0, []

        def take(kind):
            nonlocal pos
            k = int(np.frombuffer(raw, np.uint64, 1, pos)[0])
            pos += 8
            if kind == "text":
                v = raw[pos:pos + k]
                pos += k
            else:
                v = np.frombuffer(raw, np.float32, k, pos).copy()
                pos += 4 * k
            return v
        for _ in range(len(grads) + 1):
            states.append((take("text"), take("floats"), take("text"), take("floats")))
        n_models = int(np.frombuffer(raw, np.uint64, 1, pos)[0])
        return states, n_models

    def teacher_forward(self, w, b, x) -> np.ndarray:
        """initSampler's teacher with these W / biases, forward(x_i, TEMPERATURE, -1, 1) per sample."""
        w = np.ascontiguousarray(w, dtype=np.float32)
        b = np.ascontiguousarray(b, dtype=np.float32)
        x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1, 784)
        out = np.empty((x.shape[0], 10), np.float32)
        self.lib.ref_teacher_forward(w.ctypes.data, b.ctypes.data, x.ctypes.data, x.shape[0], out.ctypes.data)
        return out

    def mnist_version_copy(self, w_in, b_in):
        """descentNative's mode-1 model copy: read(getParams()) of the MNIST network."""
        w = np.ascontiguousarray(w_in, dtype=np.float32)
        b = np.ascontiguousarray(b_in, dtype=np.float32)
        wo, bo = np.empty_like(w), np.empty_like(b)
        self.lib.ref_mnist_version_copy(w.ctypes.data, b.ctypes.data, wo.ctypes.data, bo.ctypes.data)
        return wo, bo


def sampler_buckets(labels, num_clients: int = 10, outlier: bool = False, seed: int = 1):
    """initSampler's non-IID buckets (sampler_oracle.cpp: the C++ library's own
    std::sort / std::random_shuffle over libc rand() after srand(seed)).
    Returns (sorted_index[n], [bucket positions into the sorted order, per client])."""
    L = C.CDLL(SAMPLER_SO)
    L.fo_sampler_buckets.restype = C.c_int
    L.fo_sampler_buckets.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                     C.c_long, C.c_void_p]
    lab = np.ascontiguousarray(labels, dtype=np.int32)
    n = len(lab)
    srt = np.zeros(n, np.int32)
    flat = np.zeros(n + 1, np.int32)
    lens = np.zeros(num_clients, np.int32)
    k = L.fo_sampler_buckets(lab.ctypes.data, n, num_clients, int(outlier), seed, srt.ctypes.data, flat.ctypes.data,
                             n, lens.ctypes.data)
    if k < 0:
        raise ValueError("dataset too small for the clients")
    out, o = [], 0
    for i in range(k):
        out.append(flat[o:o + lens[i]].copy())
        o += lens[i]
    return srt, out
