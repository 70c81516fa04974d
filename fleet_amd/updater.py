"""Mirror of CppNNUpdater's aggregation path on the MI355X codec.

Server/src/main/java/apps/cppNN/CppNNUpdater.java drives the hot path through
JNI: it buffers client uploads until M have arrived (M-softsync, :383-391),
picks them in FIFO order (:420-421), dampens each by ``getDampen(tau,
similarity)`` (:300-327, :463-464), sums and averages them (:490-507), merges
the average into the last picked upload's layout (:508) and calls
``descentNative`` (:509). :class:`FleetUpdater` keeps that control logic on the
host (it is O(M) and O(labels)) and runs the per-element work as two device
calls: ``Codec.update`` (the exact re-quantised dampen/sum/average/merge chain)
and ``Codec.descent`` (sgd on the resident model).

Scope: the ``staleSize == 0`` branch (``aggregated = acc``, :408-411) with the
pruning thresholds at 0 (their defaults in the quick start). Staleness
simulation (StalenessSimulator), percentile pruning and Kardam's bookkeeping are
the reference's host-side experiment controls and are not rebuilt (SURVEY.md §2
rows 11-13); their O(N) natives (getNorm, subtract) are on :class:`Codec`.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np


def _java_max(a: float, b: float) -> float:
    """Math.max: NaN if either argument is NaN."""
    if a != a or b != b:
        return float("nan")
    return a if a >= b else b


def get_dampen(policy: int, tau: int, similarity: float = 1.0, stale_size: int = 0, alpha: float = 0.0,
               has_outlier: bool = False) -> float:
    """CppNNUpdater.getDampen (:300-327), in Java double arithmetic. (Java's
    Math.exp may differ from libm's exp in the last bit; the factors are inputs
    of the device chain, which is exact for any given value.)"""
    l_tau = 1.0
    if policy == 0:  # average
        l_tau = 1.0
    elif policy == 1:  # inverse
        l_tau = 1 / float(tau + 1)
    elif policy == 2:  # inverse + class-aware
        l_tau = 1 / float(tau + 1)
        if has_outlier and tau > 1.5 * stale_size:
            l_tau /= _java_max(0.1, similarity)
    elif policy == 3:  # exponential
        l_tau = math.exp((-1) * alpha * min(tau, stale_size))
    elif policy == 4:  # exponential + class-aware
        l_tau = math.exp((-1) * alpha * min(tau, stale_size))
        if has_outlier and tau > 1.5 * stale_size:
            l_tau /= _java_max(0.1, similarity)
    return l_tau


def similarity(x: Sequence[int], y: Sequence[int]) -> float:
    """Helpers.similarity (commonLib/utils/Helpers.java:140-161): Bhattacharyya
    coefficient of the two label histograms, each normalised by its sum (an
    all-zero histogram normalises to NaN, as 0.0/0 does in Java)."""
    def norm(v):
        s = float(sum(v))
        return [(a / s) if s != 0 else (float("nan") if a == 0 else math.copysign(math.inf, a)) for a in v]
    b = 0.0
    for a, c in zip(norm(x), norm(y)):
        b += math.sqrt(a) * math.sqrt(c) if a == a and c == c else float("nan")
    return b


class Kardam:
    """utils/Kardam.java's bookkeeping (setGrad :48-62, setModel :93-106, updateLip
    :190-203) with its O(N) vector work on the GPU: the gradient texts and norms of
    all picked uploads come from one ``Codec.kardam_grads`` call,
    the model-difference norm from ``subtractNative`` + ``getNorm``. ``checkByz``
    is not rebuilt: CppNNUpdater bypasses it (``if (true || ...)``, :488)."""

    def __init__(self, codec, workers: int = 10):
        self.codec = codec
        self.workers = workers
        self.grads = {}           # worker -> (g text, epoch)
        self.models = {}          # worker -> model text
        self.model_diff_norm = {}
        self.grad_diff_norm = {}
        self.lips = {}

    def set_grads(self, worker_ids, uploads, dampen, lr: float, epochs):
        """setGrad for each picked upload: one device pass computes every g_c and its
        difference norm to the worker's previous g. Returns the setGrad results."""
        worker_ids = list(worker_ids)
        if len(set(worker_ids)) < len(worker_ids):  # a worker twice in one batch: its pushes in order
            out = []
            for i in range(len(worker_ids)):
                out += self.set_grads(worker_ids[i:i + 1], uploads[i:i + 1], dampen[i:i + 1], lr, epochs[i:i + 1])
            return out
        prev = [self.grads[w][0] if w in self.grads else None for w in worker_ids]
        texts, _, diff = self.codec.kardam_grads(uploads, dampen, lr, prev)
        out = []
        for w, g, dn, ep in zip(worker_ids, texts, diff, epochs):
            if w in self.grads:
                if self.grads[w][1] == ep:  # same epoch as the previous push: ignored
                    out.append(False)
                    continue
                self.grad_diff_norm[w] = float(dn)
                self.grads[w] = (g, ep)
                out.append(True)
            else:
                self.grads[w] = (g, ep)
                out.append(False)
        return out

    def set_model(self, worker: int, model_text: bytes) -> None:
        if worker in self.models:
            norm = self.codec.getNorm(self.codec.subtractNative(model_text, self.models[worker]))
            if norm == 0:  # same model as before: ignored
                return
            self.model_diff_norm[worker] = norm
        self.models[worker] = model_text

    def update_lip(self, worker: int) -> None:
        lip = self.grad_diff_norm[worker] / self.model_diff_norm[worker]
        lst = self.lips.setdefault(worker, [])
        if len(lst) > 25:
            lst.pop(0)
        lst.append(lip)


@dataclass
class Pending:
    upload: bytes
    labels: List[int]
    epoch: int
    client_id: int


class FleetUpdater:
    """CppNNUpdater.update's aggregation + descentNative's model step.

    ``weights`` (the non-null W concatenated in slot order) and ``fc_bias`` (the
    fully-connected layers' biases) are the model the server keeps
    (``cnn`` in cppNN_backend.cpp); ``lrates`` is initUpdater's schedule
    (cppNN_backend.cpp:161-172)."""

    def __init__(self, codec, layout, M: int, lrates: Sequence[float], weights, fc_bias, policy: int = 0,
                 alpha: float = 0.0, stale_size: int = 0, num_labels: int = 10, has_outlier: bool = False):
        if stale_size != 0:
            raise NotImplementedError("staleness simulation (StalenessSimulator) is not rebuilt: staleSize must be 0")
        self.codec = codec
        self.layout = layout
        self.M = M
        self.policy = policy
        self.alpha = alpha
        self.stale_size = stale_size
        self.has_outlier = has_outlier
        self.lrates = [float(v) for v in lrates]
        self.lr = np.float32(self.lrates[0])  # initUpdater: cnn.set_learning_rate(lrates_vec[0])
        self.weights = np.array(weights, dtype=np.float32, copy=True)
        self.fc_bias = np.array(fc_bias, dtype=np.float32, copy=True)
        self.curr_epoch = 0
        self.acc: List[Pending] = []
        self.global_labels = [0] * num_labels
        self.last_merged: Optional[bytes] = None

    def update(self, upload: bytes, labels: Sequence[int], epoch: int, client_id: int = 0) -> Optional[bytes]:
        """One client upload (CppNNUpdater.update, :330-518). Returns the merged
        gradient when this upload completed a batch of M (and the model stepped),
        else None."""
        self.acc.append(Pending(bytes(upload), list(labels), int(epoch), int(client_id)))
        if len(self.acc) < self.M:  # M-softsync (:388-391)
            return None
        picked, dampen = [], []
        window = [0] * len(self.global_labels)
        for _ in range(self.M):  # FIFO (:420-421)
            p = self.acc.pop(0)
            tau = self.curr_epoch - p.epoch
            sim = similarity(p.labels, self.global_labels)
            picked.append(p.upload)
            dampen.append(get_dampen(self.policy, tau, sim, self.stale_size, self.alpha, self.has_outlier))
            for j, v in enumerate(p.labels[: len(window)]):
                window[j] += v
        for j, v in enumerate(window):
            self.global_labels[j] += v
        merged, grad = self.codec.update(picked, dampen, want_f32=True)
        # descentNative (cppNN_backend.cpp:329-353): lr from the schedule, then the model step
        if self.curr_epoch < len(self.lrates):
            self.lr = np.float32(self.lrates[self.curr_epoch])
        self.weights, self.fc_bias = self.codec.descent(self.weights, self.fc_bias, grad, self.layout, self.lr)
        self.curr_epoch += 1
        self.acc.clear()  # aggregated.clear() (:516)
        self.last_merged = merged
        return merged
