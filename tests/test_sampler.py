"""getMiniBatch: the sampler's mini-batch vector and its Base64.

Restates the reference's getMiniBatch (cppNN_backend.cpp:677-699, non-IID
path); tests/golden/minibatch_noniid.npz is a regression fixture of that
restatement (tests/golden/make_golden.py minibatch; parity unpinned: the
reference backend needs <jni.h>, absent here); the GPU gather+encode is compared with that fixture and with the
oracle's restatement (oracle/pyoracle.py minibatch_vector + the C encoder)."""
import os

import numpy as np
import pytest

from fleet_amd.sampler import NonIIDCursor, OfflineSampler, minibatch_header, uniform_indices

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "minibatch_noniid.npz")


def _fixture():
    z = np.load(GOLDEN)
    return {k: z[k] for k in z.files}


def _fixture_indices(z):
    B = int(z["batch"]) * int(z["E"])
    return NonIIDCursor([z["bucket"].tolist()]).take(0, B), B


def test_oracle_minibatch_matches_fixture(oracle):
    import pyoracle
    z = _fixture()
    idx, B = _fixture_indices(z)
    hdr = minibatch_header(int(z["E"]), float(z["sigma"]), float(z["C"]), 0.01, B, z["images"].shape[1],
                           int(z["num_labels"]))
    v = pyoracle.minibatch_vector(z["images"], z["labels"], idx, hdr)
    assert oracle.encode_floats(v) == z["out"].tobytes()


def test_cursor_and_uniform_draw():
    cur = NonIIDCursor([[4, 2, 9], [1]])
    assert cur.take(0, 5) == [4, 2, 9, 4, 2]
    assert cur.take(0, 2) == [9, 4]
    assert cur.take(1, 3) == [1, 1, 1]
    seq = iter([7, 12, 3, 100])
    assert uniform_indices(10, 4, rand=lambda: next(seq)) == [7, 2, 3, 0]
    h = minibatch_header(2, 0.1, 3.0, 0.01, 14, 784, 10)
    assert h.dtype == np.float32 and h[1] == np.float32(0.1) and h[5] == 784.0


def test_sampler_rotation_and_header():
    calls = []

    class FakeCodec:
        def getMiniBatch(self, images, labels, idx, header, teacher=None):  # noqa: N802
            calls.append((list(idx), header.copy(), teacher))
            return b""

    img = np.zeros((6, 3), np.float32)
    s = OfflineSampler(FakeCodec(), img, np.arange(6), E=2, sigma=0.5, C=1.0, buckets=[[0, 1, 2], [3, 4, 5]])
    s.getMiniBatch(2)
    s.getMiniBatch(1)
    s.getMiniBatch(1)
    assert [c[0] for c in calls] == [[0, 1, 2, 0], [3, 4], [1, 2]]
    assert calls[0][1].tolist() == [2.0, 0.5, 1.0, np.float32(0.01), 4.0, 3.0, 10.0]
    with pytest.raises(ValueError):
        OfflineSampler(FakeCodec(), img, np.arange(6), E=1, sigma=0, C=0)


def test_sampler_reads_learning_rate_per_request():
    """The header's lr is cnn.get_learning_rate() when the request is built
    (cppNN_backend.cpp:588,658); descentNative moves it along lrates_vec
    (:345-348), so a schedule change shows in the next request."""
    calls = []

    class FakeCodec:
        def getMiniBatch(self, images, labels, idx, header, teacher=None):  # noqa: N802
            calls.append(header.copy())
            return b""

    class Updater:  # the FleetUpdater attribute the sampler reads
        lr = np.float32(0.05)

    up = Updater()
    img = np.zeros((4, 3), np.float32)
    s = OfflineSampler(FakeCodec(), img, np.arange(4), E=1, sigma=0.0, C=1.0, lr=up, buckets=[[0, 1, 2, 3]])
    s.getMiniBatch(1)
    up.lr = np.float32(0.01)  # the epoch moved on
    s.getMiniBatch(1)
    schedule = iter([0.2, 0.3])
    s2 = OfflineSampler(FakeCodec(), img, np.arange(4), E=1, sigma=0.0, C=1.0, lr=lambda: next(schedule),
                        buckets=[[0, 1, 2, 3]])
    s2.getMiniBatch(1)
    s2.getMiniBatch(1)
    assert [h[3] for h in calls] == [np.float32(0.05), np.float32(0.01), np.float32(0.2), np.float32(0.3)]


@pytest.mark.gpu
def test_device_minibatch_matches_restatement_fixture(codec):
    z = _fixture()
    s = OfflineSampler(codec, z["images"], z["labels"], E=int(z["E"]), sigma=float(z["sigma"]), C=float(z["C"]),
                       num_labels=int(z["num_labels"]), buckets=[z["bucket"].tolist()])
    assert s.getMiniBatch(int(z["batch"])) == z["out"].tobytes()


@pytest.mark.gpu
def test_device_minibatch_teacher_and_edges(codec, oracle):
    """Mode-1 layout (teacher probabilities, end marker), an empty batch, a
    device-resident run, and an index outside the dataset."""
    import pyoracle
    import fleet_amd as F
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(11)
    n, Fd, nl = 50, 785, 10
    img = rng.normal(0, 1, (n, Fd)).astype(np.float32)
    img[:, 0] = 1e9  # outside the fast codec domain
    lab = rng.integers(0, nl, n).astype(np.int32)
    idx = rng.integers(0, n, 23).astype(np.int32)
    teacher = rng.dirichlet(np.ones(nl), len(idx)).astype(np.float32)
    hdr = minibatch_header(1, 0.0, 0.0, 0.01, len(idx), Fd, nl)
    want = oracle.encode_floats(pyoracle.minibatch_vector(img, lab, idx, hdr, teacher))
    assert codec.getMiniBatch(img, lab, idx, hdr, teacher=teacher) == want
    want0 = oracle.encode_floats(pyoracle.minibatch_vector(img, lab, [], hdr))
    assert codec.getMiniBatch(img, lab, np.zeros(0, np.int32), hdr) == want0
    dev = torch.device("cuda", 0)
    L = codec._L.fleet_minibatch_len(Fd, len(idx), nl, 1)
    out = torch.zeros(L + 16, dtype=torch.uint8, device=dev)
    codec.minibatch_device(torch.from_numpy(img).to(dev), torch.from_numpy(lab).to(dev),
                           torch.from_numpy(idx).to(dev), hdr, out, teacher_f32=torch.from_numpy(teacher).to(dev))
    codec.check()
    assert out[:L].cpu().numpy().tobytes() == want
    with pytest.raises(F.FleetError):
        codec.getMiniBatch(img, lab, np.array([0, n], np.int32), hdr)
    bad = torch.tensor([1, n + 5], dtype=torch.int32, device=dev)
    codec.minibatch_device(torch.from_numpy(img).to(dev), torch.from_numpy(lab).to(dev), bad, hdr, out)
    with pytest.raises(F.FleetError):
        codec.check()
