"""Seeded differential fuzz of the fused update (CppNNUpdater.update's aggregation,
CppNNUpdater.java:420-509) against the oracle's faithful per-op chain.

Each case draws a bucket size (4 .. 150 k values, log-uniform), a client count, a value
mix, dampening factors and a launch plan, so the kernels meet combinations the fixed
parity cases do not: every plan form at sizes its default range never gives it, ragged
last groups, dampening factors that are not binary32 values (the f64 branch of
scalarMultiply), payloads with values past the codec's fast domain (|x| >= 1e8 / 1e9,
infinities, NaN: the general codec per lane), and sums that leave it. The merged text
and Base64::decodeFloat of it must be the oracle's, byte for byte."""
import numpy as np
import pytest

import fleet_amd as F

from fleet_amd.layouts import synthetic

pytestmark = pytest.mark.gpu

PLANS = ["", "update=stream", "update=stream,grid=plain", "update=stream,grid=lanes", "update=tiled,tile=flat",
         "update=tiled,tile=flat,flat_w2=16", "update=tiled,tile=classic", "update=tiled,tile=weave6",
         "update=tiled,tile=weave8", "update=pipe"]
DAMPEN = [1.0, 0.5, 1.0 / 3.0, 0.25, 0.1, 0.7, 2.0, 1e-3, 0.123456789, 1.0 / 7.0]
EDGE = np.array([1e8, -1e8, 99999999.0, 999999999.0, 1e9, -1e9, 2.1e9, 3e9, -3e9, 9.99999e8, 123456.789,
                 float("inf"), float("-inf"), float("nan"), 1e-45, 3.4e38], np.float32)


def _payload(rng, mix, n):
    if mix == 0:  # the synthetic §8d mix as generated (gradient-like, a few large values)
        return None
    if mix == 1:  # wide magnitudes, sums that leave the fast domain
        v = np.exp(rng.uniform(-30, 19, n)) * rng.choice([-1.0, 1.0], n)
        return v.astype(np.float32)
    v = rng.normal(0, 1e-2, n).astype(np.float32)  # gradient-like with edge values sprinkled in
    k = max(1, n // 500)
    v[rng.integers(0, n, k)] = rng.choice(EDGE, k)
    return v


@pytest.mark.parametrize("case", range(48))
def test_update_fuzz_vs_faithful_chain(codec, oracle, plan, case):
    rng = np.random.default_rng(20260 + case)
    n_up = int(np.exp(rng.uniform(np.log(4), np.log(150_000))))
    # the layout header carries N = n_up - 3: sizes whose N the codec does not round-trip
    # (N * 10^(9 - digits) not a binary32 value, e.g. odd N in [134218, 268435]) make the
    # reference's own flatGrad walk misread the bucket, so take the next size that does
    while oracle.decode_floats(oracle.encode_floats(np.array([n_up - 3], np.float32)))[0] != n_up - 3:
        n_up += 1
    M = int(rng.integers(1, 41))
    mix = int(rng.integers(0, 3))
    spec = PLANS[case % len(PLANS)]
    lay = synthetic(n_up)
    ups = []
    for c in range(M):
        v = oracle.synth_upload(1000 + case, c, list(lay.w_sizes), list(lay.b_sizes))
        p = _payload(rng, mix, n_up - 3)
        if p is not None:
            v[2:n_up - 1] = p  # the layout's header ([1, N] and the trailing 0) stays
        ups.append(oracle.encode_floats(v))
    d = [float(x) for x in rng.choice(DAMPEN, M)]
    plan(spec)
    merged, f32 = codec.update(ups, d, want_f32=True)
    exp = oracle.update_faithful(ups, d)
    assert merged == exp, (case, n_up, M, mix, spec)
    assert np.array_equal(f32.view(np.uint32), oracle.decode_floats(exp).view(np.uint32)), (case, n_up, M, mix, spec)


FUSED_PLANS = ["", "update=stream", "update=stream,grid=lanes", "update=tiled", "update=tiled,tile=flat",
               "update=tiled,tile=weave6", "update=tiled,tile=weave8", "update=pipe"]


@pytest.mark.parametrize("case", range(16))
def test_fused_step_fuzz(codec, oracle, plan, case):
    """The pipelined device step (fleet_update_encode_device: this batch's aggregation and
    the next batch's client encode in one launch) on random sizes, payloads and plans: its
    merged text, merged_f32 and next uploads equal the two separate calls, and the next
    uploads are the oracle's Base64::encode of the rows (sampled rows)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(7700 + case)
    n = int(np.exp(rng.uniform(np.log(4), np.log(400_000))))
    while oracle.decode_floats(oracle.encode_floats(np.array([n - 3], np.float32)))[0] != n - 3:
        n += 1
    M = int(rng.integers(1, 17))
    lay = synthetic(n)
    groups = (n + 2) // 3
    dev = torch.device("cuda", 0)

    def batch(seed):
        rows = np.zeros((M, 3 * groups), np.float32)
        for c in range(M):
            v = oracle.synth_upload(seed, c, list(lay.w_sizes), list(lay.b_sizes))
            p = _payload(rng, int(rng.integers(0, 3)), n - 3)
            if p is not None:
                v[2:n - 1] = p
            rows[c, :n] = v
        return rows

    cur, nxt = batch(50 + case), batch(90 + case)
    values_next = torch.from_numpy(nxt).to(dev)
    L = F.b64_len(n)
    text = torch.from_numpy(np.stack([np.frombuffer(oracle.encode_floats(cur[c, :n]), np.uint8) for c in range(M)])
                            ).to(dev).contiguous()
    text = torch.nn.functional.pad(text, (0, 16 * groups - L)).contiguous()
    d = [float(x) for x in rng.choice(DAMPEN, M)]
    hp = np.asarray(lay.header_positions(), np.int32)
    plan(FUSED_PLANS[case % len(FUSED_PLANS)])
    merged_a = torch.zeros(16 * groups, dtype=torch.uint8, device=dev)
    f32_a = torch.zeros(3 * groups, dtype=torch.float32, device=dev)
    codec.update_device(text, L, d, hp, merged_a, f32_a)
    next_a = torch.zeros_like(text)
    codec.encode_device(values_next, n, next_a)
    merged_b, f32_b, next_b = torch.zeros_like(merged_a), torch.zeros_like(f32_a), torch.zeros_like(text)
    codec.update_encode_device(text, L, d, hp, merged_b, f32_b, values_next, next_b)
    torch.cuda.synchronize()
    codec.check()
    assert torch.equal(merged_a, merged_b) and torch.equal(f32_a.view(torch.int32), f32_b.view(torch.int32))
    assert torch.equal(next_a, next_b)
    exp = oracle.update_faithful([oracle.encode_floats(cur[c, :n]) for c in range(M)], d)
    assert merged_b.cpu().numpy()[:L].tobytes() == exp
    for c in sorted({0, M - 1, int(rng.integers(0, M))}):
        assert next_b[c].cpu().numpy()[:L].tobytes() == oracle.encode_floats(nxt[c, :n])


KD_PLANS = ["", "update=stream", "update=stream,grid=lanes", "update=tiled", "update=tiled,flat_w2=16", "update=pipe"]


@pytest.mark.parametrize("case", range(12))
def test_kardam_fuzz(codec, oracle, plan, case):
    """Kardam's side outputs (fleet_update_kardam_device) on random bucket sizes, client
    counts and plans, three rounds each (no prev, prev on every other client, prev
    replaced in place): merged bytes, G rows and norms as test_gpu_kardam_fused checks."""
    from test_gpu_kardam_fused import check_side_outputs
    rng = np.random.default_rng(5150 + case)
    n = int(np.exp(rng.uniform(np.log(8), np.log(200_000))))
    while oracle.decode_floats(oracle.encode_floats(np.array([n - 3], np.float32)))[0] != n - 3:
        n += 1
    plan(KD_PLANS[case % len(KD_PLANS)])
    check_side_outputs(codec, oracle, synthetic(n), int(rng.integers(1, 9)))


@pytest.mark.parametrize("case", range(12))
def test_model_codec_fuzz(codec, oracle, case):
    """The mode-1 model codec (quantisation, first-occurrence dictionary by rocPRIM radix
    sort and scans, the weights section of getParams and network::read of it) on random
    matrix shapes -- single values, thin and wide matrices, sizes either side of the sort's
    single-block limit -- and value mixes (trained-like, few levels, constant matrices,
    +-0, NaN / inf) against the oracle's sequential restatement (network.h:594-706)."""
    rng = np.random.default_rng(9100 + case)
    nm = int(rng.integers(1, 7))
    dims = []
    for _ in range(nm):
        shape = rng.integers(0, 4)
        if shape == 0:
            dims.append((1, 1, 1))
        elif shape == 1:
            dims.append((int(rng.integers(1, 6)), int(rng.integers(1, 6)), int(rng.integers(1, 400))))
        else:
            dims.append((int(rng.integers(1, 40)), int(rng.integers(1, 40)), int(rng.integers(1, 12))))
    n = sum(c * r * ch for c, r, ch in dims)
    mix = case % 4
    if mix == 0:
        w = rng.normal(0, 0.05, n) * np.exp(rng.normal(0, 1, n))
    elif mix == 1:
        w = rng.integers(-4, 5, n) * 0.125 + rng.choice([0.0, 1e-9], n)
    elif mix == 2:
        w = np.full(n, float(rng.normal()))
    else:
        w = rng.normal(0, 1, n)
        k = max(1, n // 50)
        w[rng.integers(0, n, k)] = rng.choice([np.nan, np.inf, -np.inf, 0.0, -0.0], k)
    w = w.astype(np.float32)
    wq, dic, idx = codec.model_quantize_index(w, dims)
    owq = oracle.quantize(w, dims)
    assert np.array_equal(wq.view(np.uint32), owq.view(np.uint32)), (case, dims)
    od, oi = oracle.dictionary(owq)
    assert np.array_equal(dic.view(np.uint32), od.view(np.uint32)) and np.array_equal(idx, oi), (case, dims)
    sec = codec.model_weights_text(w, dims)
    assert sec == oracle.weights_section(owq, dims), (case, dims)
    wr = codec.model_read_weights(sec, dims)
    assert np.array_equal(wr.view(np.uint32), oracle.read_weights_section(sec, dims).view(np.uint32)), (case, dims)
