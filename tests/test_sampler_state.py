"""The offline sampler's native state (fleet_sampler, fleet_amd/csrc/sampler_state.cpp)
and the JNI shim's sampler natives (initSampler / getMiniBatch / getNumLabels /
hasOutlier), SURVEY.md §8 f4 and the drop-in boundary (b).

* initSampler's non-IID buckets (Server/src/main/c++/cppNN_backend.cpp:387,
  :411-470) equal the oracle's (oracle/sampler_oracle.cpp: the C++ library's own
  std::sort and std::random_shuffle over libc rand() after srand(1)) -- CPU.
* A server session through the JNI function table, in the reference's call
  order (MasterOrchestrator: initSampler -> CppNNUpdater.initialize's
  fetchParamsNative + initUpdater -> compute requests' getMiniBatch, gradient
  requests' descentNative): every mini-batch header is
  {E, sigma, C, lrates[epoch], batch*E, F, numLabels} and the samples are the
  libc-rand replay of the buckets -- GPU (the encode runs there).
* uniformSample (iid): indices = rand() % N after initUpdater's srand(1) and its
  train_class's two draws (network.h:1840) -- GPU.

Parity: pinned to the reference's call sequence on this image's libstdc++ and
glibc (no reference build exists for cppNN_backend.cpp: it needs <jni.h>)."""
import ctypes as C
import os

import numpy as np
import pytest

import fleet_amd as F
from fleet_amd.sampler import NativeSampler

HERE = os.path.dirname(os.path.abspath(__file__))


def _dataset(n, seed, F_=784, classes=10):
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, classes, n).astype(np.int32)
    pix = rng.integers(0, 256, (n, F_)).astype(np.uint8)
    pix[:, 0] = np.arange(n) % 256  # distinct images (first two pixels encode the index)
    pix[:, 1] = np.arange(n) // 256
    return pix, labels


def _write_mnist(path, pix, labels, dashed=False):
    os.makedirs(path, exist_ok=True)
    n = len(labels)
    sep = "-" if dashed else "."
    with open(os.path.join(path, f"train-images{sep}idx3-ubyte"), "wb") as f:
        f.write(np.array([2051, n, 28, 28], ">i4").tobytes())
        f.write(pix.tobytes())
    with open(os.path.join(path, f"train-labels{sep}idx1-ubyte"), "wb") as f:
        f.write(np.array([2049, n], ">i4").tobytes())
        f.write(labels.astype(np.uint8).tobytes())


def _pixels(pix):
    """mnist_parser.h: (b / 255.0f) * (1 - (-1)) + (-1), in binary32."""
    return (pix.astype(np.float32) / np.float32(255.0)) * np.float32(2.0) + np.float32(-1.0)


@pytest.mark.parametrize("n,clients,outlier", [(600, 10, 0), (600, 10, 1), (1003, 7, 0), (1003, 7, 1),
                                               (60000, 10, 0)])
def test_nonid_buckets_match_oracle(n, clients, outlier):
    import pyoracle
    pyoracle.build()
    pix, labels = _dataset(n, n + clients)
    s = NativeSampler(None, images=_pixels(pix), labels=labels, num_clients=clients, outlier=bool(outlier))
    srt, buckets = pyoracle.sampler_buckets(labels, clients, bool(outlier), seed=1)
    assert np.array_equal(s.sorted_index(), srt)
    assert len(buckets) == clients
    for k, b in enumerate(buckets):
        assert np.array_equal(s.bucket(k), b), k
    # the real generator state after initSampler is the same too: both consumed the same draws
    s.close()


def test_initsampler_parses_mnist_files(tmp_path):
    import pyoracle
    pyoracle.build()
    pix, labels = _dataset(300, 5)
    for dashed in (False, True):  # parse_train_data's two file-name spellings
        d = str(tmp_path / ("dash" if dashed else "dot"))
        _write_mnist(d, pix, labels, dashed)
        s = NativeSampler(None, data_path=d, num_clients=3)
        assert s.num_samples == 300 and s.num_labels == 10
        srt, buckets = pyoracle.sampler_buckets(labels, 3, False, seed=1)
        assert np.array_equal(s.sorted_index(), srt)
        assert all(np.array_equal(s.bucket(k), b) for k, b in enumerate(buckets))
    with pytest.raises(F.FleetError):
        NativeSampler(None, data_path=str(tmp_path / "missing"))
    with pytest.raises(F.FleetError):  # 2 samples cannot make 10 clients' shards
        NativeSampler(None, images=np.zeros((2, 784), np.float32), labels=np.zeros(2, np.int32))


def test_minibatch_needs_a_context():
    pix, labels = _dataset(60, 1)
    s = NativeSampler(None, images=_pixels(pix), labels=labels, num_clients=2)
    s.set_hyper(1, 0.0, 0.0)
    with pytest.raises(F.FleetError):
        s.getMiniBatch(2, 0.01)


# ----------------------------------------------------------------------- GPU

def _decode_samples(text, images_f32, labels, B, with_teacher=False, num_labels=10):
    """Decode a mini-batch text (the oracle's decoder) -> (header[7], sample indices)."""
    import pyoracle
    v = pyoracle.Oracle().decode_floats(text)
    F_ = images_f32.shape[1]
    hdr = v[:7]
    per = F_ + (num_labels if with_teacher else 0) + 1
    key = {(int(round((r[0] + 1) * 127.5)), int(round((r[1] + 1) * 127.5))): i for i, r in enumerate(images_f32)}
    idx = []
    for b in range(B):
        row = v[7 + b * per: 7 + b * per + F_]
        i = key[(int(round((row[0] + 1) * 127.5)), int(round((row[1] + 1) * 127.5)))]
        np.testing.assert_allclose(row, images_f32[i], rtol=0, atol=3e-7)  # Q(x): the codec is lossy
        assert v[7 + b * per + per - 1] == labels[i]
        idx.append(i)
    return hdr, idx


@pytest.mark.gpu
def test_shim_server_session_sampler_and_updater(tmp_path, oracle, monkeypatch):
    """initSampler -> fetchParams -> initUpdater -> getMiniBatch -> descentNative x2 (across an
    lr-schedule step) -> getMiniBatch, through the JNI table: headers and sample indices."""
    import jnifake as J
    import pyoracle
    from test_jni_shim import check_rules, load
    L = load()
    env = J.env()
    n, clients, E, sigma, Cc, batch = 600, 10, 2, 0.5, 3.0, 5
    pix, labels = _dataset(n, 77)
    d = str(tmp_path / "mnist")
    _write_mnist(d, pix, labels)
    images = _pixels(pix)
    monkeypatch.setenv("FLEET_SAMPLER_IID", "0")
    monkeypatch.setenv("FLEET_SAMPLER_OUTLIER", "0")
    monkeypatch.setenv("FLEET_SAMPLER_CLIENTS", str(clients))
    monkeypatch.setenv("FLEET_DISTILLATION_MODE", "1")
    s = np.load(os.path.join(HERE, "golden", "session_mnist.npz"))
    lrates = np.asarray(s["lrates"], np.float64)

    J.begin()
    L.Java_apps_cppNN_CppNNOfflineSampler_initSampler(env, None, J.new_string(d))
    assert L.Java_apps_cppNN_CppNNUpdater_getNumLabels(env, None) == 10
    assert L.Java_apps_cppNN_CppNNUpdater_hasOutlier(env, None) == 0
    L.Java_apps_cppNN_CppNNUpdater_fetchParamsNative(env, None, J.new_bytes(bytes(s["init"])))
    L.Java_apps_cppNN_CppNNUpdater_initUpdater(env, None, J.new_doubles(lrates), E, sigma, Cc)
    check_rules(J)

    srt, buckets = pyoracle.sampler_buckets(labels, clients, False, seed=1)
    cursor = [0] * clients

    def expect(client):
        b = buckets[client]
        out = [int(srt[b[(cursor[client] + j) % len(b)]]) for j in range(batch * E)]
        cursor[client] = (cursor[client] + batch * E) % len(b)
        return out

    def request(lr_expected, client):
        J.begin()
        text = J.read_bytes(L.Java_apps_cppNN_CppNNOfflineSampler_getMiniBatch(env, None, batch))
        check_rules(J)
        hdr, idx = _decode_samples(text, images, labels, batch * E)
        want = np.array([E, sigma, Cc, lr_expected, batch * E, 784, 10], np.float64).astype(np.float32)
        q_want = oracle.decode_floats(oracle.encode_floats(want))  # what the text carries: Q(header)
        assert np.array_equal(hdr.view(np.uint32), q_want.view(np.uint32)), (hdr, want)
        assert idx == expect(client)
        # the text is Base64::encode of exactly that vector
        vec = pyoracle.minibatch_vector(images, labels, idx, want)
        assert text == oracle.encode_floats(vec)

    request(float(np.float32(lrates[0])), 0)
    for step in range(2):
        J.begin()
        L.Java_apps_cppNN_CppNNUpdater_descentNative(env, None, J.new_bytes(bytes(s[f"merged{step}"])),
                                                     int(s["batch"]), int(s["stale"]))
        check_rules(J)
    assert L.Java_apps_cppNN_CppNNUpdater_getCurrEpoch(env, None) == 2
    request(float(np.float32(lrates[1])), 1)  # descent 2 set lr = lrates[1]
    request(float(np.float32(lrates[1])), 2)
    # the model side is unchanged by the sampler (session fixture, test_jni_shim.py)
    newest = L.Java_apps_cppNN_CppNNUpdater_modelsSize(env, None) - 1
    assert J.read_bytes(L.Java_apps_cppNN_CppNNUpdater_getParametersNative(env, None, newest)) == \
        bytes(s["newest_text2"])


def _write_test_set(path, n=10):
    """The MNIST test files parse_test_data reads (mnist_parser.h:153-161)."""
    with open(os.path.join(path, "t10k-images.idx3-ubyte"), "wb") as f:
        f.write(np.array([2051, n, 28, 28], ">i4").tobytes() + bytes(784 * n))
    with open(os.path.join(path, "t10k-labels.idx1-ubyte"), "wb") as f:
        f.write(np.array([2049, n], ">i4").tobytes() + bytes(n))


@pytest.mark.gpu
def test_shim_mode1_test_set_and_empty_batches(tmp_path, monkeypatch, capfd):
    """DISTILLATION_MODE=1 initSampler without the MNIST test set: the reference
    returns after building the buckets (cppNN_backend.cpp:485), so the non-IID
    sampler still serves and "Train data size" is not printed; getMiniBatch with
    batch * E = 0 is refused instead of reading sample 0 of an empty batch."""
    import jnifake as J
    from test_jni_shim import load
    L = load()
    env = J.env()
    pix, labels = _dataset(100, 3)
    d = str(tmp_path / "m")
    _write_mnist(d, pix, labels)
    monkeypatch.setenv("FLEET_SAMPLER_IID", "0")
    monkeypatch.setenv("FLEET_SAMPLER_CLIENTS", "2")
    monkeypatch.setenv("FLEET_DISTILLATION_MODE", "1")
    J.begin()
    L.Java_apps_cppNN_CppNNOfflineSampler_initSampler(env, None, J.new_string(d))
    out = capfd.readouterr()
    assert "error: could not parse test data." in out.err and "Train data size" not in out.out
    L.Java_apps_cppNN_CppNNUpdater_initUpdater(env, None, J.new_doubles([0.1]), 0, 0.0, 0.0)  # E = 0
    J.begin()
    assert L.Java_apps_cppNN_CppNNOfflineSampler_getMiniBatch(env, None, 4) is None  # batch*E = 0: no read of sample 0
    assert "batch_size * E = 0" in capfd.readouterr().err
    L.Java_apps_cppNN_CppNNUpdater_initUpdater(env, None, J.new_doubles([0.1]), 1, 0.0, 0.0)
    J.begin()
    assert L.Java_apps_cppNN_CppNNOfflineSampler_getMiniBatch(env, None, 4)  # the buckets serve
    _write_test_set(d)
    L.Java_apps_cppNN_CppNNOfflineSampler_initSampler(env, None, J.new_string(d))
    assert "Train data size: 100" in capfd.readouterr().out


@pytest.mark.gpu
def test_shim_iid_mode1_session_with_teacher(tmp_path, oracle, monkeypatch, capfd):
    """iid sampling in DISTILLATION_MODE=1 through the JNI table, in the server's call
    order: initSampler (test set present; the teacher's training is not rebuilt) ->
    fetchParamsNative -> initUpdater -> getMiniBatch refused until the JVM hands over
    the trained teacher (FleetSampler.setTeacherNative) -> getMiniBatch x2: indices =
    rand() % N after srand(1) and initUpdater's two train_class draws, teacher outputs
    = the teacher's forward pass, the 1234567 sentinel (uniformSample :553-634)."""
    import jnifake as J
    import pyoracle
    from test_jni_shim import check_rules, load
    L = load()
    env = J.env()
    n, E, batch = 300, 2, 3
    pix, labels = _dataset(n, 19)
    d = str(tmp_path / "iid")
    _write_mnist(d, pix, labels)
    _write_test_set(d)
    images = _pixels(pix)
    monkeypatch.setenv("FLEET_SAMPLER_IID", "1")
    monkeypatch.setenv("FLEET_DISTILLATION_MODE", "1")
    s = np.load(os.path.join(HERE, "golden", "session_mnist.npz"))
    lrates = np.asarray(s["lrates"], np.float64)
    J.begin()
    L.Java_apps_cppNN_CppNNOfflineSampler_initSampler(env, None, J.new_string(d))
    assert "Train data size: 300" in capfd.readouterr().out
    L.Java_apps_cppNN_CppNNUpdater_fetchParamsNative(env, None, J.new_bytes(bytes(s["init"])))
    L.Java_apps_cppNN_CppNNUpdater_initUpdater(env, None, J.new_doubles(lrates), E, 0.5, 2.0)
    J.begin()
    assert L.Java_apps_cppNN_CppNNOfflineSampler_getMiniBatch(env, None, batch) is None
    assert "trained teacher" in capfd.readouterr().err
    z = np.load(os.path.join(HERE, "golden", "teacher_mnist.npz"))
    w, b = z["w0"], z["b0"]
    J.begin()
    assert L.Java_apps_cppNN_FleetSampler_setTeacherNative(env, None, J.new_floats(w[:-1]), J.new_floats(b)) == 0
    assert L.Java_apps_cppNN_FleetSampler_setTeacherNative(env, None, J.new_floats(w), J.new_floats(b)) == 1
    check_rules(J)
    # the generator: initUpdater's srand(1) + two draws, then B = batch * E draws per request.
    # libc's rand() state is the process's, shared with the shim: replay the expected
    # indices first, then put the state back where initUpdater left it
    lc = _libc()
    B = batch * E
    lc.srand(1)
    lc.rand(), lc.rand()
    wants = [[lc.rand() % n for _ in range(B)] for _ in range(2)]
    lc.srand(1)
    lc.rand(), lc.rand()
    hdr = np.array([E, 0.5, 2.0, np.float32(lrates[0]), B, 784, 10], np.float64).astype(np.float32)
    for want in wants:
        J.begin()
        text = J.read_bytes(L.Java_apps_cppNN_CppNNOfflineSampler_getMiniBatch(env, None, batch))
        check_rules(J)
        teacher = oracle.teacher_forward(w, b, images[want])
        assert text == oracle.encode_floats(pyoracle.minibatch_vector(images, labels, want, hdr, teacher))


def test_reseed_without_a_fetched_model_draws_nothing():
    """initUpdater before any fetchParamsNative: the reference's train_class draws its
    random shift only with use_augmentation > 0, which the fetch sets."""
    lc = _libc()
    NativeSampler.reseed_updater(1, fetched=False)
    got = lc.rand()
    lc.srand(1)
    assert got == lc.rand()
    NativeSampler.reseed_updater(1, fetched=True)
    got = lc.rand()
    lc.srand(1)
    lc.rand(), lc.rand()
    assert got == lc.rand()


def test_one_argument_reseed_keeps_its_meaning():
    """fleet_updater_reseed(seed) is the original one-argument symbol: the fetched-model
    form, fleet_updater_reseed_ex(seed, 1) (the ABI must not change under
    the same name)."""
    import fleet_amd
    lc = _libc()
    fleet_amd.lib().fleet_updater_reseed(5)
    got = lc.rand()
    lc.srand(5)
    lc.rand(), lc.rand()
    assert got == lc.rand()


def _libc():
    lc = C.CDLL(None)
    lc.rand.restype = C.c_int
    lc.srand.argtypes = [C.c_uint]
    return lc


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_uniform_sample_replays_libc_rand(codec, oracle, mode):
    """uniformSample (iid): B draws of rand() % N after initUpdater's srand(1) and the two
    draws of its train_class; mode 1 appends the teacher's outputs (given weights) and
    the 1234567 sentinel."""
    import pyoracle
    n, E, batch = 257, 3, 4
    pix, labels = _dataset(n, 11)
    images = _pixels(pix)
    s = NativeSampler(codec, images=images, labels=labels, iid=True, distillation_mode=mode)
    teacher = None
    if mode:
        z = np.load(os.path.join(HERE, "golden", "teacher_mnist.npz"))
        w, b = z["w0"], z["b0"]
        s.set_teacher(w, b)
    lc = _libc()
    lc.srand(1)
    lc.rand(), lc.rand()
    want = [lc.rand() % n for _ in range(batch * E)] + [lc.rand() % n for _ in range(batch * E)]
    NativeSampler.reseed_updater(1)
    s.set_hyper(E, 0.25, 2.0)
    texts = [s.getMiniBatch(batch, 0.125), s.getMiniBatch(batch, 0.125)]
    got = []
    for t in texts:
        B = batch * E
        hdr = np.array([E, 0.25, 2.0, 0.125, B, 784, 10], np.float64).astype(np.float32)
        idx = list(s.last_indices()) if t is texts[-1] else None
        v = oracle.decode_floats(t)
        per = 784 + (10 if mode else 0) + 1
        ids = []
        for bb in range(B):
            row = v[7 + bb * per: 7 + bb * per + 784]
            ids.append(int(round((row[0] + 1) * 127.5)) + 256 * int(round((row[1] + 1) * 127.5)))
        if idx is not None:
            assert ids == idx
        if mode:
            teacher = oracle.teacher_forward(w, b, images[ids])
        assert t == oracle.encode_floats(pyoracle.minibatch_vector(images, labels, ids, hdr, teacher))
        got += ids
    assert got == want
