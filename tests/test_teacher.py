"""The sampler's mode-1 teacher forward: uniformSample's
teacher.forward(sample, TEMPERATURE, -1, 1) (Server/src/main/c++/cppNN_backend.cpp:
596-613) of initSampler's network (:494-502).

Pins, strongest first:
* tests/golden/teacher_mnist.npz holds the class probabilities of the
  reference's OWN mojo network (commonLib/cppNN compiled by oracle/Makefile into
  oracle/_ref, tests/golden/make_golden.py teacher) for seeded weights and inputs;
* the oracle's C restatement (oracle/fleet_oracle.c fo_teacher_forward, libm
  expf) equals that fixture bit for bit, and equals the reference build on fresh
  inputs where oracle/_ref exists (this container);
* the device's expf (teacher_math.h glibc_expf, a restatement of glibc 2.35's)
  equals libm's expf on all 2^32 inputs (digest fn 18, tests/golden/digests.json,
  itself checked against this machine's libm here);
* the device forward equals the fixture bit for bit (NaN rows included: the
  reference's softmax overflows at the largest weight scale).
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "teacher_mnist.npz")
REF_SO = os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libfleetref_model.so")


def _cases():
    z = np.load(GOLDEN)
    n = len([k for k in z.files if k.startswith("probs")])
    return [(z[f"w{i}"], z[f"b{i}"], z[f"x{i}"], z[f"probs{i}"]) for i in range(n)]


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def test_fixture_shape_and_coverage():
    cases = _cases()
    assert len(cases) == 3
    for w, b, x, p in cases:
        assert w.shape == (21448,) and b.shape == (82,) and x.shape[1] == 784 and p.shape == (x.shape[0], 10)
    # typical scales give proper distributions; the largest overflows the softmax as the reference does
    for _, _, _, p in cases[:2]:
        assert np.all(np.isfinite(p)) and np.allclose(p.sum(1), 1.0, atol=1e-5)
    assert np.any(~np.isfinite(cases[2][3]))


def test_oracle_teacher_matches_reference_fixture(oracle):
    for w, b, x, p in _cases():
        assert np.array_equal(_bits(oracle.teacher_forward(w, b, x)), _bits(p))


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref (reference build) absent")
def test_oracle_teacher_matches_reference_build(oracle):
    import pyoracle
    ref = pyoracle.ReferenceModel()
    rng = np.random.default_rng(77)
    for scale in (0.02, 0.1, 0.4):
        w = (rng.standard_normal(21448) * scale).astype(np.float32)
        b = (rng.standard_normal(82) * 0.2).astype(np.float32)
        x = np.where(rng.random((16, 784)) < 0.6, 0.0, rng.random((16, 784))).astype(np.float32)
        assert np.array_equal(_bits(oracle.teacher_forward(w, b, x)), _bits(ref.teacher_forward(w, b, x)))


def test_libm_expf_digest_matches_golden(oracle):
    """digests.json fn 18 is this libm's expf (the reference's std::exp(float))."""
    ref = json.load(open(os.path.join(HERE, "golden", "digests.json")))
    assert f"{oracle.expf_digest():016x}" == ref["fn18"]


def test_teacher_symbols_and_sizes():
    import fleet_amd as F
    L = F.lib()
    assert L.fleet_teacher_weight_count() == 21448
    assert L.fleet_teacher_bias_count() == 82


@pytest.mark.gpu
def test_device_teacher_matches_reference_fixture(codec):
    for w, b, x, p in _cases():
        assert np.array_equal(_bits(codec.teacher_forward(w, b, x)), _bits(p))


@pytest.mark.gpu
def test_device_teacher_indices_device_path_and_errors(codec, oracle):
    import fleet_amd as F
    torch = pytest.importorskip("torch")
    w, b, x, p = _cases()[1]
    rng = np.random.default_rng(3)
    feats = np.concatenate([x, rng.random((x.shape[0], 1)).astype(np.float32)], axis=1)  # F = 785 rows
    idx = rng.integers(0, x.shape[0], 40).astype(np.int32)
    assert np.array_equal(_bits(codec.teacher_forward(w, b, feats, idx)), _bits(p[idx]))
    dev = torch.device("cuda", 0)
    probs = torch.zeros((len(idx), 10), dtype=torch.float32, device=dev)
    codec.teacher_forward_device(torch.from_numpy(w).to(dev), torch.from_numpy(b).to(dev),
                                 torch.from_numpy(feats).to(dev), probs, torch.from_numpy(idx).to(dev))
    codec.check()
    assert np.array_equal(_bits(probs.cpu().numpy()), _bits(p[idx]))
    with pytest.raises(F.FleetError):
        codec.teacher_forward(w, b, feats, np.array([0, x.shape[0]], np.int32))
    with pytest.raises(F.FleetError):
        codec.teacher_forward(w[:-1], b, feats)
    bad = torch.tensor([1, x.shape[0] + 3], dtype=torch.int32, device=dev)
    codec.teacher_forward_device(torch.from_numpy(w).to(dev), torch.from_numpy(b).to(dev),
                                 torch.from_numpy(feats).to(dev), probs, bad)
    with pytest.raises(F.FleetError):
        codec.check()


@pytest.mark.gpu
def test_sampler_minibatch_with_device_teacher(codec, oracle):
    """uniformSample + getMiniBatch in mode 1 end to end: the request text equals the
    oracle's composition with the reference's teacher probabilities."""
    import pyoracle
    from fleet_amd import sampler as S
    w, b, x, p = _cases()[0]
    labels = (np.arange(x.shape[0]) % 10).astype(np.int32)
    s = S.OfflineSampler(codec, x, labels, E=1, sigma=0.0, C=0.0, num_labels=10, lr=0.01, iid=True)
    teacher = S.Teacher(codec, w, b, x)
    S.srand(5)
    text = s.getMiniBatch(12, teacher=teacher)
    S.srand(5)
    idx = S.uniform_indices(x.shape[0], 12)
    hdr = S.minibatch_header(1, 0.0, 0.0, 0.01, 12, 784, 10)
    assert text == oracle.encode_floats(pyoracle.minibatch_vector(x, labels, idx, hdr, p[idx]))
