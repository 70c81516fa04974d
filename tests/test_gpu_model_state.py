"""The server's resident model (fleet_model) against the
reference's own network code: session_mnist.npz is the updater's model natives
(fetchParamsNative, initUpdater, 3 x descentNative, getParametersNative and
getModelParametersNative of the newest and the oldest version after each step;
Server/src/main/c++/cppNN_backend.cpp:161-383) replayed by oracle/_ref on the
mojo network compiled from /root/reference (tests/golden/make_golden.py session).
getParametersNative's whole text is compared for equality, header and bias lines
included."""
import os

import numpy as np
import pytest

import fleet_amd as F

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def session():
    return np.load(os.path.join(HERE, "golden", "session_mnist.npz"))


def test_model_session_matches_reference(codec, oracle, session):
    s = session
    m = F.Model(codec, bytes(s["init"]), distillation_mode=1)
    m.initUpdater(s["lrates"])
    assert m.modelsSize() == 1 and m.getCurrEpoch() == 0
    assert abs(m.getLrate() - float(np.float32(s["lrates"][0]))) == 0

    def check(state):
        newest = m.modelsSize() - 1
        assert m.getParametersNative(newest) == bytes(s[f"newest_text{state}"])
        assert m.getParametersNative(0) == bytes(s[f"oldest_text{state}"])
        for v, key in ((newest, "newest"), (0, "oldest")):
            # Base64::encode of the reference's getModelParams vector (the codec: the oracle)
            assert m.getModelParametersNative(v) == oracle.encode_floats(s[f"{key}_params{state}"])
    check(0)
    for i in range(3):
        m.descentNative(bytes(s[f"merged{i}"]), int(s["batch"]), int(s["stale"]))
        check(i + 1)
    assert m.modelsSize() == int(s["n_models"])
    assert m.getCurrEpoch() == 3
    assert m.getLrate() == float(np.float32(s["lrates"][2]))
    m.close()


def test_model_text_rejects(codec, session):
    init = bytes(session["init"])
    with pytest.raises(F.FleetError):
        F.Model(codec, b"mojo02\n" + init[7:])
    with pytest.raises(F.FleetError):
        F.Model(codec, init.replace(b"semi_stochastic_pool 3 3", b"dropout 3 3", 1))
    m = F.Model(codec, init)
    m.initUpdater([0.1])
    # a merged gradient of another layout (CIFAR-10) does not describe the model
    from fleet_amd.layouts import CIFAR10
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    import pyoracle
    o = pyoracle.Oracle()
    g = o.encode_floats(o.synth_upload(3, 0, list(CIFAR10.w_sizes), list(CIFAR10.b_sizes)))
    with pytest.raises(F.LayoutError):
        m.descentNative(g, 8, 2)
    assert m.modelsSize() == 1
    with pytest.raises(F.FleetError):
        m.getParametersNative(5)
