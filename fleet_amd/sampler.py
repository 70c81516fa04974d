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

Bucket construction (initSampler :409-470: label sort, 2-shard buckets,
``std::random_shuffle``) is dataset plumbing outside the hot path; buckets are
given.
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
