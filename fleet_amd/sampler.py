"""Mirror of the offline sampler's mini-batch request.

CppNNOfflineSampler.getSample -> JNI getMiniBatch (Server/src/main/c++/
cppNN_backend.cpp:677-699) draws batch_size*E sample indices -- uniformly with
libc ``rand() % N`` (uniformSample, :553-634) or by walking the client's
non-IID bucket with a cursor (nonIIDSample, :636-675) -- builds the float
vector [E, sigma, C, lr, batchSize, featureSize, numLabels, per sample: features,
(mode 1) teacher probabilities, label] and Base64-encodes it. The index draw is
host logic and stays here; the gather + encode runs on the GPU
(``Codec.getMiniBatch`` / ``Codec.minibatch_device``). The mode-1 teacher's
forward pass (uniformSample's teacher.forward, :603) runs on the GPU too
(``Teacher``: fleet_teacher_forward, bit-identical to the mojo network); its
training in initSampler (:480-546: 300 rand()-drawn MNIST samples) is dataset
plumbing and stays with the caller, who hands over the trained weights.

``NativeSampler`` is the whole sampler state of the reference's backend in the
C-ABI (fleet_amd/csrc/sampler_state.cpp, the fleet_sampler_* entry points the
JNI shim's initSampler / getMiniBatch use): the MNIST set loaded by
initSampler's parser, the non-IID buckets it builds (:409-479: label sort,
2-shard buckets, ``std::random_shuffle`` over libc ``rand()``), the client
rotation and initUpdater's E / sigma / C. ``OfflineSampler`` below takes the
buckets as given (any dataset).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

_libc = None


def _rand() -> int:
    """libc rand() -- the generator uniformSample draws from (srand(seed) in initSampler)."""
    global _libc
    if _libc is None:
        _libc = ctypes.CDLL(None)
        _libc.rand.restype = ctypes.c_int
    return _libc.rand()


def srand(seed: int) -> None:
    """initSampler's srand(seed) (cppNN_backend.cpp:387)."""
    global _libc
    if _libc is None:
        _libc = ctypes.CDLL(None)
        _libc.rand.restype = ctypes.c_int
    _libc.srand(ctypes.c_uint(seed))


def minibatch_header(E: int, sigma: float, C: float, lr: float, batch_size: int, feature_size: int,
                     num_labels: int) -> np.ndarray:
    """The 7 leading values as push_back(float) converts them (:586-592): ints and the
    doubles sigma, C rounded to float; lr is cnn.get_learning_rate() (a float)."""
    return np.array([E, sigma, C, lr, batch_size, feature_size, num_labels], dtype=np.float64).astype(np.float32)


def uniform_indices(n_images: int, count: int, rand=_rand) -> List[int]:
    """uniformSample's draw (:559-563): index = 0 + rand() % (N - 1 - 0 + 1)."""
    return [rand() % n_images for _ in range(count)]


class NonIIDCursor:
    """nonIIDSample's per-client cursor (:645-652): non-overlapping samples from the
    client's bucket, wrapping around."""

    def __init__(self, buckets: Sequence[Sequence[int]]):
        self.buckets = [list(b) for b in buckets]
        self.pos = [0] * len(self.buckets)

    def take(self, client: int, count: int) -> List[int]:
        b = self.buckets[client]
        out = []
        for _ in range(count):
            out.append(b[self.pos[client]])
            self.pos[client] = (self.pos[client] + 1) % len(b)
        return out


class OfflineSampler:
    """CppNNOfflineSampler.getMiniBatch with the sampler state of cppNN_backend.cpp
    (E, sigma, C, lr, iid, the client rotation currClientID, :691)."""

    def __init__(self, codec, images, labels, E: int, sigma: float, C: float, lr=0.01,
                 num_labels: int = 10, iid: bool = False, buckets: Optional[Sequence[Sequence[int]]] = None):
        """``lr``: a number, or a callable / an object with an ``lr`` attribute (the
        FleetUpdater) read at every request -- the reference pushes
        cnn.get_learning_rate() when the request is built (:588, :658), and
        descentNative moves it along lrates_vec every epoch (:345-348)."""
        self.codec = codec
        self.images = np.ascontiguousarray(images, dtype=np.float32)
        self.labels = np.ascontiguousarray(labels, dtype=np.int32)
        self.E, self.sigma, self.C = int(E), float(sigma), float(C)
        self._lr = lr
        self.num_labels = int(num_labels)
        self.iid = bool(iid)
        if not self.iid and not buckets:
            raise ValueError("the non-IID sampler needs the clients' buckets (initSampler)")
        self.cursor = NonIIDCursor(buckets) if buckets else None
        self.num_clients = len(buckets) if buckets else 1
        self.curr_client = 0

    @property
    def lr(self) -> float:
        """The learning rate as of now (cnn.get_learning_rate(), a float)."""
        src = self._lr
        if callable(src):
            src = src()
        elif hasattr(src, "lr"):
            src = src.lr
        return float(np.float32(src))

    def getMiniBatch(self, batch_size: int, teacher=None) -> bytes:  # noqa: N802  (cppNN_backend.cpp:677)
        """``teacher(indices) -> [B, numLabels]`` (e.g. a ``Teacher``) supplies the mode-1
        teacher's probabilities for the IID path (uniformSample runs the teacher there)."""
        B = batch_size * self.E
        if self.iid:
            idx = uniform_indices(len(self.images), B)
        else:
            idx = self.cursor.take(self.curr_client, B)
        self.curr_client = (self.curr_client + 1) % self.num_clients
        hdr = minibatch_header(self.E, self.sigma, self.C, self.lr, B, self.images.shape[1], self.num_labels)
        probs = teacher(idx) if (teacher is not None and self.iid) else None
        return self.codec.getMiniBatch(self.images, self.labels, idx, hdr, teacher=probs)


class Teacher:
    """The sampler's mode-1 teacher (initSampler's network, cppNN_backend.cpp:494-502)
    with trained weights: ``teacher(idx)`` = teacher.forward(images[i], TEMPERATURE, -1, 1)
    for each drawn index (uniformSample, :596-613), on the GPU (Codec.teacher_forward).
    w: the network's non-null W in order (21448 floats), b: the use_bias() layers'
    biases in layer order (82)."""

    TEMPERATURE = 2.0  # commonLib/cppNN/network.h:53

    def __init__(self, codec, w, b, images):
        self.codec = codec
        self.w = np.ascontiguousarray(w, dtype=np.float32).reshape(-1)
        self.b = np.ascontiguousarray(b, dtype=np.float32).reshape(-1)
        self.images = np.ascontiguousarray(images, dtype=np.float32)

    def __call__(self, idx) -> np.ndarray:
        return self.codec.teacher_forward(self.w, self.b, self.images, idx, self.TEMPERATURE)


class NativeSampler:
    """fleet_sampler (include/fleet_codec.h): CppNNOfflineSampler's native state.

    ``NativeSampler(codec, data_path=...)`` is initSampler on an MNIST directory;
    ``NativeSampler(codec, images=..., labels=...)`` the same over a dataset in
    memory. ``codec`` may be None for the host state alone (buckets)."""

    def __init__(self, codec, data_path: Optional[str] = None, images=None, labels=None, num_labels: int = 10,
                 iid: bool = False, outlier: bool = False, num_clients: int = 10, distillation_mode: int = 1,
                 seed: int = 1):
        from . import lib, FleetError
        self._L = L = lib()
        self.codec = codec
        h = ctypes.c_void_p()
        cp = codec._h if codec is not None else None
        if data_path is not None:
            rc = L.fleet_sampler_create(cp, data_path.encode(), int(iid), int(outlier), num_clients,
                                        distillation_mode, seed, ctypes.byref(h))
        else:
            self._images = np.ascontiguousarray(images, dtype=np.float32)
            self._labels = np.ascontiguousarray(labels, dtype=np.int32)
            rc = L.fleet_sampler_create_from(cp, self._images.ctypes.data, self._labels.ctypes.data,
                                             len(self._labels), self._images.shape[1], num_labels, int(iid),
                                             int(outlier), num_clients, distillation_mode, seed, ctypes.byref(h))
        if rc != 0:
            raise FleetError(rc, "fleet_sampler_create failed (see stderr)")
        self._h = h.value

    def close(self):
        if getattr(self, "_h", None):
            self._L.fleet_sampler_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc != 0:
            from . import FleetError
            raise FleetError(rc, self._L.fleet_sampler_last_error(self._h).decode())

    @staticmethod
    def reseed_updater(seed: int = 1, fetched: bool = True) -> None:
        """initUpdater's srand(seed) and, after fetchParamsNative (fetched), its
        train_class's two rand() draws."""
        from . import lib
        lib().fleet_updater_reseed_ex(seed, int(bool(fetched)))

    def set_hyper(self, E: int, sigma: float, C: float) -> None:
        self._check(self._L.fleet_sampler_set_hyper(self._h, int(E), float(sigma), float(C)))

    def set_teacher(self, w, b) -> None:
        self._tw = np.ascontiguousarray(w, dtype=np.float32).reshape(-1)
        self._tb = np.ascontiguousarray(b, dtype=np.float32).reshape(-1)
        self._check(self._L.fleet_sampler_set_teacher(self._h, self._tw.ctypes.data, len(self._tw),
                                                      self._tb.ctypes.data, len(self._tb)))

    def getMiniBatch(self, batch_size: int, lr: float) -> bytes:  # noqa: N802  (cppNN_backend.cpp:677)
        n = self._L.fleet_sampler_minibatch_len(self._h, int(batch_size))
        out = ctypes.create_string_buffer(max(n, 1))
        got = ctypes.c_size_t(0)
        self._check(self._L.fleet_sampler_minibatch(self._h, int(batch_size), float(np.float32(lr)), out, n,
                                                    ctypes.byref(got)))
        return out.raw[:got.value]

    def _ints(self, fn, *args) -> np.ndarray:
        n = ctypes.c_size_t(0)
        fn(self._h, *args, None, 0, ctypes.byref(n))
        a = np.zeros(max(n.value, 1), np.int32)
        self._check(fn(self._h, *args, a.ctypes.data, a.size, ctypes.byref(n)))
        return a[:n.value]

    def bucket(self, client: int) -> np.ndarray:
        """Positions (in the label-sorted order) of the client's bucket."""
        return self._ints(self._L.fleet_sampler_bucket, int(client))

    def sorted_index(self) -> np.ndarray:
        return self._ints(self._L.fleet_sampler_sorted_index)

    def last_indices(self) -> np.ndarray:
        """Image indices (loaded order) of the last mini-batch."""
        return self._ints(self._L.fleet_sampler_last_indices)

    @property
    def num_labels(self) -> int:
        return self._L.fleet_sampler_num_labels(self._h)

    @property
    def num_samples(self) -> int:
        return self._L.fleet_sampler_num_samples(self._h)
