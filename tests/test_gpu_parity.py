"""HIP path vs the oracle (bit-exact), through the C-ABI (libfleetcodec.so).

The oracle is the C restatement in oracle/ (model side pinned to the reference's
own mojo network; codec/aggregation side unpinned beyond SURVEY.md §8c's known
answers, see oracle/fleet_oracle.h). Every comparison of Base64
output is byte-for-byte; decoded floats are compared bitwise. getNorm is the
one floating-point reduction: the reference sums in index order in fp64, the
GPU in a tree, so it is checked to 1e-12 relative (documented in DESIGN.md).
"""
import math

import numpy as np
import pytest

import fleet_amd as F
from fleet_amd.layouts import CIFAR10, MNIST, Layout, synthetic

pytestmark = pytest.mark.gpu


def edge_floats():
    v = [0.0, -0.0, 1.0, -1.0, 9.99, -9.99, 10.0, -10.0, 1e-9, -1e-9, 9.99999e8, -9.99999e8, 1e-45, -1e-45,
         0.5, 0.05, 123456.789, -123456.789, 0.0168, 99999999.0, 1e8, -1e8, 999999999.0, 1e9, 2.1e9, -2.1e9,
         3e9, -3e9, float("inf"), float("-inf"), float("nan"), 1.17549435e-38, 3.4e38]
    return np.array(v, dtype=np.float32)


def random_floats(rng, n):
    parts = [rng.normal(0, 1e-3, n), rng.normal(0, 1, n), rng.uniform(-1e8, 1e8, n // 4),
             np.exp(rng.uniform(-40, 20, n)) * rng.choice([-1, 1], n)]
    return np.concatenate(parts).astype(np.float32)


def uploads_for(oracle, layout: Layout, M: int, seed: int):
    return [oracle.encode_floats(oracle.synth_upload(seed, c, list(layout.w_sizes), list(layout.b_sizes)))
            for c in range(M)]


def test_encode_floats_bitexact(codec, oracle):
    rng = np.random.default_rng(1)
    for v in (edge_floats(), random_floats(rng, 20000), random_floats(rng, 7)[:7], np.zeros(0, np.float32)):
        assert codec.encode_floats(v) == oracle.encode_floats(v)


def test_decode_bitexact(codec, oracle):
    rng = np.random.default_rng(2)
    codes = np.concatenate([rng.integers(-2**31, 2**31, 30001), np.arange(-30, 30),
                            [2**31 - 1, -2**31, 10, -10, 1000000000, -1000000000]]).astype(np.int32)
    for n in (len(codes), 1, 2, 3, 4, 5):
        text = oracle.encode_ints(codes[:n])
        assert codec.decode_ints(text).tolist() == oracle.decode_ints(text).tolist()
        got = codec.decode_floats(text)
        exp = oracle.decode_floats(text)
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))
    assert codec.encode_ints(codes) == oracle.encode_ints(codes)


def test_url_safe_alphabet_accepted(codec, oracle):
    v = np.arange(-3000, 3000, dtype=np.int32) * 7919
    t = oracle.encode_ints(v)
    u = t.replace(b"+", b"-").replace(b"/", b"_")
    assert codec.decode_ints(u).tolist() == oracle.decode_ints(u).tolist() == v.tolist()


def test_invalid_base64_rejected(codec):
    good = codec.encode_floats(np.ones(30, np.float32))
    for bad in (good[:-1], good[:8] + b"*" + good[9:], good[:20] + b"=" + good[21:]):
        with pytest.raises(F.Base64Error):
            codec.decode_floats(bad)


def test_elementwise_ops_bitexact(codec, oracle):
    rng = np.random.default_rng(3)
    for n in (3000, 3001, 3002, 159):
        a = oracle.encode_floats(random_floats(rng, n)[:n])
        b = oracle.encode_floats(random_floats(rng, n)[:n])
        for s in (0.5, 1 / 3, 1.0, math.exp(-0.7), 7.25):
            assert codec.scalarMulNative(a, s) == oracle.scalar_mul(a, s)
        assert codec.addNative(a, b) == oracle.add(a, b)
        assert codec.subtractNative(a, b) == oracle.subtract(a, b)
        ref = oracle.norm(a)
        assert abs(codec.getNorm(a) - ref) <= 1e-12 * abs(ref)


@pytest.mark.parametrize("layout", [MNIST, synthetic(1000), synthetic(1001), synthetic(1002)])
def test_flat_and_merge_bitexact(codec, oracle, layout):
    ups = uploads_for(oracle, layout, 2, seed=11)
    flat = oracle.flat_gradient(ups[0])
    assert codec.getFlatGradient(ups[0]) == flat
    other = oracle.flat_gradient(ups[1])
    assert codec.mergeFlatGradient(ups[0], other) == oracle.merge_flat_gradient(ups[0], other)
    pos, n_up = codec.layout_parse(ups[0])
    assert n_up == layout.n_up and pos.tolist() == layout.header_positions()


def policy(name, M):
    if name == "avg":
        return [1.0] * M
    if name == "inverse":
        return [1 / ((c % 3) + 1) for c in range(M)]
    if name == "exp":
        return [math.exp(-0.5 * min(c, 4)) for c in range(M)]
    raise KeyError(name)


@pytest.mark.parametrize("M", [1, 2, 8])
@pytest.mark.parametrize("pol", ["avg", "inverse", "exp"])
def test_update_mnist_vs_faithful_chain(codec, oracle, M, pol):
    ups = uploads_for(oracle, MNIST, M, seed=100 + M)
    d = policy(pol, M)
    merged, f32 = codec.update(ups, d, want_f32=True)
    exp = oracle.update_faithful(ups, d)
    assert merged == exp
    assert np.array_equal(f32.view(np.uint32), oracle.decode_floats(exp).view(np.uint32))


@pytest.mark.parametrize("layout,M", [(MNIST, 64), (CIFAR10, 16), (synthetic(100000), 9), (synthetic(99998), 5)])
def test_update_vs_elementwise_oracle(codec, oracle, layout, M):
    ups = uploads_for(oracle, layout, M, seed=7)
    d = policy("inverse", M)
    hm = oracle.header_mask(list(layout.w_sizes), list(layout.b_sizes))
    assert codec.update(ups, d) == oracle.update_fused(ups, d, hm)


@pytest.mark.parametrize("n_up", [3, 4, 5, 6, 7])
@pytest.mark.parametrize("M", [1, 2, 3])
def test_update_tiny_layouts(codec, oracle, n_up, M):
    """The smallest uploads the layout allows (an empty weight block, one or two
    values, one partial Base64 group) through the fused update, against the
    faithful per-op chain; every tile/stream path sees one group."""
    lay = synthetic(n_up)
    ups = uploads_for(oracle, lay, M, seed=n_up * 10 + M)
    d = policy("exp", M)
    merged, f32 = codec.update(ups, d, want_f32=True)
    exp = oracle.update_faithful(ups, d)
    assert merged == exp
    assert np.array_equal(f32.view(np.uint32), oracle.decode_floats(exp).view(np.uint32))


def test_empty_inputs(codec, oracle):
    """Empty texts through the codec and the per-op natives; an update needs at
    least one upload and a header to walk."""
    empty = np.zeros(0, np.float32)
    assert codec.encode_floats(empty) == oracle.encode_floats(empty) == b""
    assert codec.decode_floats(b"").size == 0
    assert codec.decode_ints(b"").size == 0
    assert codec.scalarMulNative(b"", 0.5) == oracle.scalar_mul(b"", 0.5)
    assert codec.addNative(b"", b"") == oracle.add(b"", b"")
    assert codec.getNorm(b"") == 0.0
    with pytest.raises((F.FleetError, ValueError)):
        codec.update([], [])
    with pytest.raises((F.FleetError, ValueError)):
        codec.update([b"", b""], [1.0, 1.0])


def test_update_cifar100_layout(codec, oracle):
    """configs[3]'s layout (CIFAR-100 cppNN, 17 header slots) on a few clients."""
    from fleet_amd.layouts import CIFAR100
    ups = uploads_for(oracle, CIFAR100, 3, seed=17)
    d = policy("exp", 3)
    hm = oracle.header_mask(list(CIFAR100.w_sizes), list(CIFAR100.b_sizes))
    assert codec.update(ups, d) == oracle.update_fused(ups, d, hm)


def test_update_malformed_last_header(codec, oracle):
    """The host walk of the last upload's header fails: the device flow reports the
    same error a full device run would (layout, or Base64 when a char is invalid)."""
    lay = synthetic(3000)
    ups = uploads_for(oracle, lay, 3, seed=5)
    v = oracle.decode_floats(ups[-1])
    v[1] = 5000.0  # the first W block claims more values than the upload holds
    bad_walk = oracle.encode_floats(v)
    with pytest.raises(F.LayoutError):
        codec.update([ups[0], ups[1], bad_walk], [1.0, 1.0, 1.0])
    bad_char = bytearray(bad_walk)
    bad_char[2] = ord("*")  # inside the first group: the header count itself
    with pytest.raises(F.Base64Error):
        codec.update([ups[0], ups[1], bytes(bad_char)], [1.0, 1.0, 1.0])


def test_update_layout_mismatch_rejected(codec, oracle):
    a = uploads_for(oracle, synthetic(3000), 2, seed=3)
    b = uploads_for(oracle, Layout("x", (1000, 1996), ()), 1, seed=3)
    assert len(a[0]) == len(b[0])
    with pytest.raises(F.LayoutError):
        codec.update([a[0], b[0], a[1]], [1.0, 1.0, 1.0])


def test_device_resident_update_sharded(codec, oracle):
    torch = pytest.importorskip("torch")
    lay = synthetic(30001)
    M = 6
    ups = uploads_for(oracle, lay, M, seed=5)
    L = len(ups[0])
    pitch = (L + 15) // 16 * 16
    host = np.zeros((M, pitch), np.uint8)
    for i, u in enumerate(ups):
        host[i, :L] = np.frombuffer(u, np.uint8)
    dev = torch.from_numpy(host).cuda()
    groups = (F.b64_count(L) + 2) // 3
    out = torch.zeros(16 * groups, dtype=torch.uint8, device="cuda")
    f32 = torch.zeros(3 * groups, dtype=torch.float32, device="cuda")
    d = policy("inverse", M)
    hp = lay.header_positions()
    half = groups // 2
    codec.update_device(dev, L, d, hp, out, f32, 0, half)
    codec.update_device(dev, L, d, hp, out, f32, half, groups)
    codec.check()
    torch.cuda.synchronize()
    got = out.cpu().numpy()[:L].tobytes()
    hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
    exp = oracle.update_fused(ups, d, hm)
    assert got == exp
    assert np.array_equal(f32.cpu().numpy()[: lay.n_up].view(np.uint32), oracle.decode_floats(exp).view(np.uint32))


def test_device_and_host_calls_interleaved(codec, oracle):
    """A device-resident update left in flight on the caller's stream, then
    host-buffer calls on the same context (its own stream: flat gradient, an
    update with more clients, a merge) before any sync: the device call keeps its
    own parameter and error buffers, so both results are exact."""
    torch = pytest.importorskip("torch")
    lay = synthetic(30001)
    M = 4
    ups = uploads_for(oracle, lay, M, seed=41)
    L = len(ups[0])
    pitch = (L + 15) // 16 * 16
    host = np.zeros((M, pitch), np.uint8)
    for i, u in enumerate(ups):
        host[i, :L] = np.frombuffer(u, np.uint8)
    dev = torch.from_numpy(host).cuda()
    groups = (F.b64_count(L) + 2) // 3
    out = torch.zeros(16 * groups, dtype=torch.uint8, device="cuda")
    d = policy("inverse", M)
    hp = lay.header_positions()
    hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
    for rep in range(2):
        codec.update_device(dev, L, d, hp, out)
        more = uploads_for(oracle, MNIST, 9, seed=42 + rep)
        dm = policy("exp", 9)
        assert codec.getFlatGradient(more[0]) == oracle.flat_gradient(more[0])
        assert codec.update(more, dm) == oracle.update_fused(more, dm, oracle.header_mask(
            list(MNIST.w_sizes), list(MNIST.b_sizes)))
        codec.check()
        torch.cuda.synchronize()
        assert out.cpu().numpy()[:L].tobytes() == oracle.update_fused(ups, d, hm)
        out.zero_()
    # more clients after the first call grows the device parameter buffer (the old one is retired)
    M2 = 11
    ups2 = uploads_for(oracle, lay, M2, seed=43)
    host2 = np.zeros((M2, pitch), np.uint8)
    for i, u in enumerate(ups2):
        host2[i, :L] = np.frombuffer(u, np.uint8)
    d2 = policy("exp", M2)
    codec.update_device(torch.from_numpy(host2).cuda(), L, d2, hp, out)
    codec.check()
    torch.cuda.synchronize()
    assert out.cpu().numpy()[:L].tobytes() == oracle.update_fused(ups2, d2, hm)


@pytest.mark.parametrize("text", [b"AAAAAA==", b"AAAAAAAAAAAAAAAAAAAAAA==", b"AAAAAAAAAAAAAAAAAAAAAAAA", b"AAAA"])
def test_update_short_uploads(codec, oracle, text):
    """Uploads shorter than a 16-char group or ending inside one: the host
    header walk reads only the caller's bytes (no over-read past a JVM array);
    the result is the oracle's layout verdict: LayoutError for a header that
    runs off the upload, otherwise the faithful chain's bytes."""
    ups = [text, text]
    try:
        exp = oracle.update_faithful(ups, [1.0, 1.0])
    except Exception:
        exp = None
    if exp is None:
        with pytest.raises(F.LayoutError):
            codec.update(ups, [1.0, 1.0])
    else:
        assert codec.update(ups, [1.0, 1.0]) == exp


def test_device_synth_and_encode(codec, oracle):
    torch = pytest.importorskip("torch")
    lay = synthetic(20002)
    M = 3
    vals = torch.zeros((M, lay.n_up + 5), dtype=torch.float32, device="cuda")
    codec.synth_device(1234, vals, lay.n_up, lay.header_positions(), lay.header_values())
    host = vals.cpu().numpy()
    for c in range(M):
        exp = oracle.synth_upload(1234, c, list(lay.w_sizes), list(lay.b_sizes))
        assert np.array_equal(host[c, : lay.n_up].view(np.uint32), exp.view(np.uint32))
    L = F.b64_len(lay.n_up)
    pitch = (L + 15) // 16 * 16
    text = torch.zeros((M, pitch), dtype=torch.uint8, device="cuda")
    codec.encode_device(vals, lay.n_up, text)
    back = torch.zeros((M, lay.n_up + 5), dtype=torch.float32, device="cuda")
    codec.decode_device(text, L, back)
    codec.check()
    t = text.cpu().numpy()
    b = back.cpu().numpy()
    for c in range(M):
        exp = oracle.encode_floats(host[c, : lay.n_up])
        assert t[c, :L].tobytes() == exp
        assert np.array_equal(b[c, : lay.n_up].view(np.uint32), oracle.decode_floats(exp).view(np.uint32))


# fn 13-17, 19, 20 and 21 compute the same functions as fn 6, 7, 10, 2, 6, 6, 10 and 6 by other arithmetic
SAME_DIGEST = {13: 6, 14: 7, 15: 10, 16: 2, 17: 6, 19: 6, 20: 10, 21: 6, 23: 0}


@pytest.mark.parametrize("fn", range(24))
def test_device_codec_exhaustive_digest(codec, fn):
    """Every input of each device codec function's domain (2^32 codes / bit
    patterns), digested on the GPU, equals the oracle's digest."""
    import json
    import os
    ref = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "digests.json")))
    assert f"{codec.selftest_digest(fn):016x}" == ref[f"fn{SAME_DIGEST.get(fn, fn)}"]


@pytest.mark.parametrize("grid", ["auto", "plain", "lanes"])
def test_update_stream_grids(codec, oracle, plan, grid):
    """The stream kernel's grids (a group per lane, a value per lane, and the
    balanced mix the planner picks from one round of waves up) on ragged sizes."""
    plan(f"update=stream,grid={grid}")
    for lay, M in ((synthetic(300001), 3), (synthetic(20000), 7), (MNIST, 5)):
        ups = uploads_for(oracle, lay, M, seed=21)
        d = policy("exp", M)
        hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
        assert codec.update(ups, d) == oracle.update_fused(ups, d, hm)


@pytest.mark.parametrize("spec", ["update=pipe", "update=tiled", "update=stream", "update=stream,grid=plain",
                                  "update=stream,grid=lanes", "update=tiled,tile=classic", "update=tiled,tile=weave6",
                                  "update=tiled,tile=weave8", "update=tiled,tile=flat",
                                  "update=tiled,tile=flat,flat_w2=16"])
def test_update_large_magnitudes_slow_path(codec, oracle, plan, spec):
    """Values far outside the fast path (|x| >= 1, digits != 0, >= 2^31) force
    every compaction pass and the tiled kernel's general-chain fallback (the
    accumulator leaves the q_lat domain); dampening > 1 (class-aware policy) too.
    Ragged tiles (4000 values = 1334 groups) for every tile width."""
    plan(spec)
    rng = np.random.default_rng(8)
    lay = synthetic(4000)
    M = 6
    ups = []
    for c in range(M):
        v = oracle.synth_upload(3, c, list(lay.w_sizes), list(lay.b_sizes))
        big = rng.random(len(v)) < 0.3
        v[big] = (np.exp(rng.uniform(0, 21, big.sum())) * rng.choice([-1, 1], big.sum())).astype(np.float32)
        v[0], v[1], v[-1] = 1.0, float(lay.w_sizes[0]), 0.0
        v[5:9] = [9.99e8, -9.99e8, 2.1e9, 0.999999]
        ups.append(oracle.encode_floats(v))
    d = [1.0, 7.5, 0.25, 10.0, 1 / 3, 1.0]
    hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
    assert codec.update(ups, d) == oracle.update_fused(ups, d, hm) == oracle.update_faithful(ups, d)


@pytest.mark.parametrize("spec", ["update=pipe", "update=tiled", "update=stream", "update=stream,grid=plain",
                                  "update=stream,grid=lanes", "update=tiled,tile=classic", "update=tiled,tile=weave6",
                                  "update=tiled,tile=weave8", "update=tiled,tile=flat",
                                  "update=tiled,tile=flat,flat_w2=16"])
def test_update_modes(codec, oracle, plan, spec):
    """Every aggregation kernel (pipelined and two-phase tiles for small
    buckets, streaming for large ones) on ragged tiles, client counts that wrap
    the LDS ring / chunk several times, and every layout."""
    plan(spec)
    for lay, M in ((MNIST, 70), (synthetic(1000), 1), (synthetic(3001), 129), (synthetic(5002), 2),
                   (synthetic(700), 300), (CIFAR10, 3)):
        ups = uploads_for(oracle, lay, M, seed=M)
        d = policy("inverse", M)
        hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
        assert codec.update(ups, d) == oracle.update_fused(ups, d, hm), (lay.name, M)


@pytest.mark.parametrize("spec", ["update=pipe", "update=tiled", "update=stream", "update=stream,grid=plain",
                                  "update=stream,grid=lanes", "update=tiled,tile=classic", "update=tiled,tile=weave6",
                                  "update=tiled,tile=weave8", "update=tiled,tile=flat",
                                  "update=tiled,tile=flat,flat_w2=16"])
@pytest.mark.parametrize("extra", [200, 201])
def test_update_keep_slots_past_the_walk(codec, oracle, plan, spec, extra):
    """Uploads longer than their layout: mergeFlatGradient (CppNNUpdater.java:508)
    keeps the last upload's values past the header walk, like the header slots. The
    kernels still run the chain on those lanes (on code 0, so no lane of a wave leaves
    the fast path); the values there are large enough (3e8..9.9e8) that a chain on
    the real codes would overflow the digit domain within a few clients. Same bytes
    as the per-op chain and as the fused oracle with those slots masked. The device-
    resident entry points take the caller's header positions as a layout that covers
    the whole upload (fleet_codec.h), so there the tail is payload: the Kardam update's
    merged text is the fused oracle's with only the header slots kept (the tail's
    sums leave the fast domain: the exact general-codec recompute). extra = 201 leaves
    the last group ragged."""
    torch = pytest.importorskip("torch")
    plan(spec)
    lay = synthetic(1000)
    rng = np.random.default_rng(extra)
    M = 8
    ups = []
    for c in range(M):
        v = oracle.synth_upload(17, c, list(lay.w_sizes), list(lay.b_sizes))
        tail = (rng.uniform(3e8, 9.9e8, extra) * rng.choice([-1, 1], extra)).astype(np.float32)
        ups.append(oracle.encode_floats(np.concatenate([v, tail])))
    d = [1.0, 7.5, 0.25, 10.0, 1 / 3, 1.0, 2.0, 0.5]
    hm = np.concatenate([oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes)), np.ones(extra, np.uint8)])
    exp = oracle.update_faithful(ups, d)
    assert exp == oracle.update_fused(ups, d, hm)
    assert codec.update(ups, d) == exp
    L = len(ups[0])
    pitch = 16 * ((L + 15) // 16)
    host = np.zeros((M, pitch), np.uint8)
    for c, u in enumerate(ups):
        host[c, :L] = np.frombuffer(u, np.uint8)
    merged = torch.zeros(pitch, dtype=torch.uint8, device="cuda")
    g_out = torch.zeros((M, lay.n_up + extra + 3), dtype=torch.float32, device="cuda")
    codec.update_kardam_device(torch.from_numpy(host).cuda(), L, d, lay.header_positions(), 0.05, merged, None,
                               None, None, g_out)
    codec.check()
    torch.cuda.synchronize()
    hm_dev = np.concatenate([oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes)), np.zeros(extra, np.uint8)])
    assert merged.cpu().numpy()[:L].tobytes() == oracle.update_fused(ups, d, hm_dev)


def test_device_window_update(codec, oracle):
    """A rank holding only its column window of every upload (fleet_amd.shard)."""
    torch = pytest.importorskip("torch")
    from fleet_amd.shard import ShardedUpdater, byte_range, group_range
    lay = MNIST
    M = 5
    ups = uploads_for(oracle, lay, M, seed=21)
    L = len(ups[0])
    d = policy("exp", M)
    hp = lay.header_positions()
    groups = (F.b64_count(L) + 2) // 3
    exp = oracle.update_faithful(ups, d)
    parts = []
    for r in range(3):
        gb, ge = group_range(groups, 3, r)
        b0, b1 = byte_range(L, gb, ge)
        win = np.zeros((M, 16 * (ge - gb)), np.uint8)
        for c, u in enumerate(ups):
            win[c, : b1 - b0] = np.frombuffer(u, np.uint8)[b0:b1]
        dev = torch.from_numpy(win).cuda()
        out = torch.zeros(16 * (ge - gb), dtype=torch.uint8, device="cuda")
        f32 = torch.zeros(3 * (ge - gb), dtype=torch.float32, device="cuda")
        codec.update_device(dev, L, d, hp, out, f32, gb, ge, window=True)
        codec.check()
        torch.cuda.synchronize()
        parts.append(out.cpu().numpy()[: b1 - b0].tobytes())
        n_loc = min(lay.n_up, 3 * ge) - 3 * gb
        assert np.array_equal(f32.cpu().numpy()[:n_loc].view(np.uint32),
                              oracle.decode_floats(exp)[3 * gb: 3 * gb + n_loc].view(np.uint32))
    assert b"".join(parts) == exp
    # the single-rank driver (no process group): same bytes
    assert ShardedUpdater(codec).update(ups, d) == exp


def test_client_sharded_partials_on_device(codec, oracle):
    """The approximate client-sharded mode's per-rank HIP step (fleet_amd.shard.
    ClientShardedUpdater.local_partial): a block of clients through the exact
    chain on the GPU equals the oracle on that block (bytes and decoded floats);
    with one rank the mode IS the exact chain. Its N-rank combination runs under
    gloo in tests/test_shard_gloo.py."""
    from fleet_amd.shard import ClientShardedUpdater
    lay = MNIST
    M = 7
    ups = uploads_for(oracle, lay, M, seed=23)
    d = policy("inverse", M)
    hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
    cs = ClientShardedUpdater(codec, approx=True)
    hp = cs.layout(ups[-1])
    for cb, ce in ((0, 3), (3, 7)):
        part, text = cs.local_partial(ups[cb:ce], d[cb:ce], hp)
        want = oracle.update_fused(ups[cb:ce], d[cb:ce], hm)
        assert text == want
        assert np.array_equal(part.float().cpu().numpy().view(np.uint32), oracle.decode_floats(want).view(np.uint32))
    assert cs.update(ups, d) == oracle.update_fused(ups, d, hm)
    # the device-resident step (bench.py's approx block) with one rank: the exact chain's text
    torch = pytest.importorskip("torch")
    L = len(ups[0])
    groups = (F.b64_count(L) + 2) // 3
    rows = torch.zeros((M, 16 * groups), dtype=torch.uint8, device="cuda")
    rows[:, :L] = torch.from_numpy(np.frombuffer(b"".join(ups), np.uint8).reshape(M, L).copy()).cuda()
    merged = torch.zeros(16 * groups, dtype=torch.uint8, device="cuda")
    f32 = torch.zeros(3 * groups, dtype=torch.float32, device="cuda")
    out = torch.zeros(16 * groups, dtype=torch.uint8, device="cuda")
    cs.device_step(rows, L, d, hp, M, 0, merged, f32, out)
    torch.cuda.synchronize()
    codec.check()
    assert out.cpu().numpy()[:L].tobytes() == oracle.update_fused(ups, d, hm)


# ---- DISTILLATION_MODE=1 model codec ---------------------------------

def _model_fixture(name):
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", f"model_{name}.npz"))


@pytest.mark.parametrize("name", ["mnist_init", "mnist_seeded"])
def test_model_codec_matches_reference_fixtures(codec, name):
    """quantised weights, the weights section of getParams and network::read's
    weights, bit-exact against the reference's own mojo network (fixtures)."""
    f = _model_fixture(name)
    dims = [tuple(int(v) for v in d) for d in f["dims"]]
    wq, dic, idx = codec.model_quantize_index(f["w"], dims)
    assert np.array_equal(wq.view(np.uint32), f["wq"].view(np.uint32))
    sec = codec.model_weights_text(f["w"], dims)
    assert f["text"].tobytes().endswith(sec)
    wr = codec.model_read_weights(sec, dims)
    assert np.array_equal(wr.view(np.uint32), f["w_read"].view(np.uint32))


def test_model_codec_edge_cases(codec, oracle):
    """NaN/inf (index -1), constant matrices (alpha = 0 -> NaN), s = 1 matrices."""
    f = _model_fixture("generic")
    dims = [tuple(int(v) for v in d) for d in f["dims"]]
    for t in range(4):
        wq, dic, idx = codec.model_quantize_index(f[f"w{t}"], dims)
        assert np.array_equal(wq.view(np.uint32), f[f"wq{t}"].view(np.uint32)), t
        assert b"mojo01\n0\n0\n0\n" + codec.model_weights_text(f[f"w{t}"], dims) == f[f"text{t}"].tobytes(), t
        od, oi = oracle.dictionary(wq)
        assert np.array_equal(dic.view(np.uint32), od.view(np.uint32)) and np.array_equal(idx, oi), t


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_model_dictionary_tolerance_chains(codec, oracle, seed):
    """Long tolerance chains (levels closer than 1e-8 across and within
    matrices), ties, +-0, against the oracle's sequential float_vector_find."""
    rng = np.random.default_rng(seed)
    dims = [(40, 30, 2), (1, 1, 300), (25, 4, 7), (7, 1, 1)]
    n = sum(c * r * ch for c, r, ch in dims)
    kinds = [rng.normal(0, 1e-7, n), rng.integers(-5, 6, n) * 4e-9 + rng.normal(0, 2e-9, n),
             np.where(rng.random(n) < 0.5, 0.0, -0.0) + rng.integers(0, 3, n) * 1e-9]
    w = kinds[seed].astype(np.float32)
    wq, dic, idx = codec.model_quantize_index(w, dims)
    owq = oracle.quantize(w, dims)
    assert np.array_equal(wq.view(np.uint32), owq.view(np.uint32))
    od, oi = oracle.dictionary(owq)
    assert np.array_equal(dic.view(np.uint32), od.view(np.uint32)) and np.array_equal(idx, oi)
    sec = codec.model_weights_text(w, dims)
    assert sec == oracle.weights_section(owq, dims)
    wr = codec.model_read_weights(sec, dims)
    assert np.array_equal(wr.view(np.uint32), oracle.read_weights_section(sec, dims).view(np.uint32))


def test_model_codec_large_random(codec, oracle):
    """A 167k-weight model (conv stacks with few levels, and a 20,000-level FC
    matrix: U ~ 20k) of trained-like weights. The oracle is O(n*U), so the
    model is sized for it, not for the GPU."""
    rng = np.random.default_rng(11)
    dims = [(3, 3, 4096), (3, 3, 4096), (5, 5, 1000), (1, 1, 20000), (200, 100, 1)]
    n = sum(c * r * ch for c, r, ch in dims)
    w = (rng.normal(0, 0.05, n) * np.exp(rng.normal(0, 1, n))).astype(np.float32)
    sec = codec.model_weights_text(w, dims)
    owq = oracle.quantize(w, dims)
    assert sec == oracle.weights_section(owq, dims)
    wr = codec.model_read_weights(sec, dims)
    assert np.array_equal(wr.view(np.uint32), oracle.read_weights_section(sec, dims).view(np.uint32))


# ---- descentNative's model step --------------------------------------------

@pytest.mark.parametrize("case", [0, 1, 2])
def test_descent_matches_reference_fixture(codec, case):
    """sgd increment_w + FC update_bias on the GPU vs the reference's own
    network::descent (MNIST network, fixture from oracle/_ref), bitwise."""
    import os
    from test_oracle_golden import GOLDEN, descent_case
    f = np.load(os.path.join(GOLDEN, "descent_mnist.npz"))
    lay, w0, b0, g, lr, w1, b1 = descent_case(f, case)
    w, b = codec.descent(w0, b0, g, lay, lr)
    assert np.array_equal(w.view(np.uint32), w1.view(np.uint32))
    assert np.array_equal(b.view(np.uint32), b1.view(np.uint32))


def test_descent_device_after_update(codec, oracle):
    """The device-resident server step: fused update -> merged_f32 stays in HBM ->
    descent on the resident CIFAR-10 model, vs the oracle (update chain + fo_descent)."""
    torch = pytest.importorskip("torch")
    lay = CIFAR10
    M = 4
    ups = uploads_for(oracle, lay, M, seed=31)
    d = policy("inverse", M)
    merged, g = codec.update(ups, d, want_f32=True)
    rng = np.random.default_rng(3)
    w0 = rng.normal(0, 0.05, lay.n_weights).astype(np.float32)
    b0 = rng.normal(0, 0.1, lay.n_fc_bias).astype(np.float32)
    lr = np.float32(0.0123)
    ew, eb = oracle.descent(w0, b0, oracle.decode_floats(merged), lay.w_present(), lay.fc_flags(), lr)
    tw, tb, tg = (torch.from_numpy(x).cuda() for x in (w0, b0, g))
    codec.descent_device(tw, tb, tg, lay, lr)
    torch.cuda.synchronize()
    assert np.array_equal(tw.cpu().numpy().view(np.uint32), ew.view(np.uint32))
    assert np.array_equal(tb.cpu().numpy().view(np.uint32), eb.view(np.uint32))


def test_descent_window_shards_compose(codec, oracle):
    """Element-sharded server step: each rank's window update writes merged_f32 of
    its groups, fleet_descent_window_device steps the parameters those positions
    cover; the ranks' steps (run one after another here, 1..4 ranks, ragged splits)
    update disjoint parts and together equal the oracle's whole-model descent."""
    torch = pytest.importorskip("torch")
    from fleet_amd.shard import byte_range, group_range
    lay = CIFAR10
    M = 3
    ups = uploads_for(oracle, lay, M, seed=37)
    L = len(ups[0])
    d = policy("inverse", M)
    hp = lay.header_positions()
    groups = (F.b64_count(L) + 2) // 3
    merged = codec.update(ups, d)
    rng = np.random.default_rng(4)
    w0 = rng.normal(0, 0.05, lay.n_weights).astype(np.float32)
    b0 = rng.normal(0, 0.1, lay.n_fc_bias).astype(np.float32)
    lr = np.float32(0.021)
    ew, eb = oracle.descent(w0, b0, oracle.decode_floats(merged), lay.w_present(), lay.fc_flags(), lr)
    for world in (1, 2, 4):
        tw, tb = torch.from_numpy(w0).cuda(), torch.from_numpy(b0).cuda()
        for r in range(world):
            gb, ge = group_range(groups, world, r)
            b_0, b_1 = byte_range(L, gb, ge)
            win = np.zeros((M, 16 * (ge - gb)), np.uint8)
            for c, u in enumerate(ups):
                win[c, : b_1 - b_0] = np.frombuffer(u, np.uint8)[b_0:b_1]
            out = torch.zeros(16 * (ge - gb), dtype=torch.uint8, device="cuda")
            f32 = torch.zeros(3 * (ge - gb), dtype=torch.float32, device="cuda")
            codec.update_device(torch.from_numpy(win).cuda(), L, d, hp, out, f32, gb, ge, window=True)
            codec.descent_window_device(tw, tb, f32, 3 * gb, 3 * ge, lay, lr)
        torch.cuda.synchronize()
        codec.check()
        assert np.array_equal(tw.cpu().numpy().view(np.uint32), ew.view(np.uint32)), world
        assert np.array_equal(tb.cpu().numpy().view(np.uint32), eb.view(np.uint32)), world


def test_descent_rejects_mismatched_header(codec):
    g = np.zeros(MNIST.n_up, np.float32)
    g[MNIST.header_positions()] = MNIST.header_values()
    g[MNIST.header_positions()[3]] += 1  # one weight block size off
    with pytest.raises(F.LayoutError):
        codec.descent(np.zeros(MNIST.n_weights, np.float32), np.zeros(MNIST.n_fc_bias, np.float32), g, MNIST, 0.1)
    with pytest.raises(F.FleetError):
        codec.descent(np.zeros(5, np.float32), np.zeros(MNIST.n_fc_bias, np.float32), g, MNIST, 0.1)


def test_model_params_matches_reference_fixture(codec):
    """getModelParametersNative (a20) on the GPU: bytes of the reference's own
    getModelParams + Base64::encode (fixture)."""
    import os
    from test_oracle_golden import GOLDEN
    f = np.load(os.path.join(GOLDEN, "model_params_mnist.npz"))
    assert codec.getModelParametersNative(f["w"], f["b"], int(f["graph_edges"][0])) == f["text"].tobytes()
    # ragged lengths and large magnitudes (group boundaries inside the bias repeats)
    rng = np.random.default_rng(1)
    for nb, e, nw in ((7, 3, 11), (1, 1, 0), (0, 5, 4), (10, 6, 1000)):
        b = (rng.normal(0, 1, nb) * 10.0 ** rng.integers(-8, 9, nb)).astype(np.float32)
        w = (rng.normal(0, 1, nw) * 10.0 ** rng.integers(-8, 9, nw)).astype(np.float32)
        from conftest import ROOT  # noqa: F401
        import pyoracle
        exp = pyoracle.Oracle().encode_floats(np.concatenate([np.tile(b, e), w]).astype(np.float32))
        assert codec.getModelParametersNative(w, b, e) == exp, (nb, e, nw)


def test_model_version_matches_reference_fixture(codec):
    """descentNative's mode-1 model copy on the device dictionary == the
    reference's read(getParams()) (fixture), bitwise."""
    import os
    from test_oracle_golden import GOLDEN
    f = np.load(os.path.join(GOLDEN, "version_mnist.npz"))
    dims = [tuple(int(v) for v in d) for d in f["dims"]]
    w, b = codec.model_version(f["w"], dims, f["b"])
    assert np.array_equal(w.view(np.uint32), f["w_out"].view(np.uint32))
    assert np.array_equal(b.view(np.uint32), f["b_out"].view(np.uint32))


@pytest.mark.parametrize("grid", ["auto", "plain", "lanes"])
def test_stream_update_mixed_grid(codec, oracle, plan, grid):
    """The stream kernel's SIMD-balanced grid (k_update_mixed: whole rounds of
    group-per-lane waves, the remaining groups one value per lane) against the
    oracle and against the plain grid: a ragged size whose remainder groups and
    last partial group fall in the value-per-lane blocks, with values outside the
    q_gen domain (1e9, -1e8, inf, NaN, 3e38) and power-of-ten boundaries
    planted in both parts, under the two dampening kinds (binary32-exact and not)."""
    plan(f"update=stream,grid={grid}")
    lay = synthetic(3 * 70000 + 2)  # 70,001 groups: one round of 65,536 + 4,465 in value-per-lane blocks
    M = 4
    n = lay.n_up
    hpos = set(lay.header_positions())
    rng = np.random.default_rng(5)
    special = np.array([1e9, -1e8, np.inf, -np.inf, np.nan, 3e38, 1e8, 9.999999e7, 10.0, -10.0, 1e-45], np.float32)
    ups = []
    for c in range(M):
        v = oracle.synth_upload(70 + c, c, list(lay.w_sizes), list(lay.b_sizes)).copy()
        for region in ((0, 3 * 65536), (3 * 65536, n)):
            pos = [p for p in rng.integers(region[0], region[1], 40) if p not in hpos]
            v[pos] = rng.choice(special, len(pos))
        ups.append(oracle.encode_floats(v))
    hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
    for pol in ("inverse", "exp"):
        d = policy(pol, M)
        got, f32 = codec.update(ups, d, want_f32=True)
        exp = oracle.update_fused(ups, d, hm)
        assert got == exp, pol
        assert np.array_equal(f32.view(np.uint32), oracle.decode_floats(exp).view(np.uint32))


@pytest.mark.parametrize("spec", ["update=stream", "update=stream,grid=plain", "update=tiled"])
def test_update_dampen_kinds(codec, oracle, plan, spec):
    """The dampen step takes one binary32 multiply when d is a binary32 normal
    value (tested on d's bits with scalar instructions where d is wave-uniform:
    the stream kernels, 64-group tiles) and the reference's f64 product
    otherwise: both kinds and their edges (+-0, binary32 subnormal and extreme
    binary32 values, values just off binary32, products that overflow) against
    the oracle, in both parts of the balanced grid and in the tiled kernel."""
    plan(spec)
    f32 = lambda x: float(np.float32(x))  # noqa: E731
    d = [1.0, 0.0, -0.0, -0.5, 2.0 ** -126, 2.0 ** -149, 2.0 ** 127, f32(3.4028235e38), 1 / 3, 1e-300, 0.1,
         f32(0.1), 3.0, -7.25, f32(0.1) * (1 + 2.0 ** -40), 2.0 ** -127]
    lay = synthetic(3 * 70000 + 2)
    ups = uploads_for(oracle, lay, len(d), seed=61)
    hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
    assert codec.update(ups, d) == oracle.update_fused(ups, d, hm)


def test_value_per_lane_decode_checks_every_char(codec, oracle, plan):
    """Lanes that own one value of a group decode only the two quads holding its
    bytes (grid=lanes: every group one value per lane): a char outside
    the alphabet at any of a full group's 16 positions, or at a needed position
    of the last partial group, is still reported; the partial group's '='
    padding is not."""
    plan("update=stream,grid=lanes")
    lay = synthetic(3 * 200 + 2)
    M = 3
    ups = uploads_for(oracle, lay, M, seed=23)
    d = policy("inverse", M)
    hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
    assert codec.update(ups, d) == oracle.update_fused(ups, d, hm)
    hpos = set(lay.header_positions())
    g = next(g for g in range(100, 200) if not {3 * g, 3 * g + 1, 3 * g + 2} & hpos)
    for ch in range(16):
        bad = bytearray(ups[1])
        bad[16 * g + ch] = ord("*")
        with pytest.raises(F.Base64Error):
            codec.update([ups[0], bytes(bad), ups[2]], d)
    last = 16 * (len(ups[0]) // 16 - 1) if len(ups[0]) % 16 == 0 else 16 * (len(ups[0]) // 16)
    assert ups[0][last + 11:last + 12] == b"=" and len(ups[0]) - last in (12, 16)
    for ch in (0, 5, 6, 10):
        bad = bytearray(ups[2])
        bad[last + ch] = ord("*")
        with pytest.raises(F.Base64Error):
            codec.update([ups[0], ups[1], bytes(bad)], d)
    assert codec.update(ups, d) == oracle.update_fused(ups, d, hm)


def test_window_update_on_mixed_grid(codec, oracle, plan):
    """Element windows (the N-GPU shards of fleet_update_multi / torch.distributed)
    through the SIMD-balanced stream grid: each window's merged slice equals the
    same bytes of the whole update."""
    torch = pytest.importorskip("torch")
    from fleet_amd.shard import byte_range, group_range
    plan("update=stream")
    lay = synthetic(3 * 150001 + 1)
    M = 3
    ups = uploads_for(oracle, lay, M, seed=41)
    L = len(ups[0])
    d = policy("exp", M)
    hp = lay.header_positions()
    groups = (F.b64_count(L) + 2) // 3
    whole = codec.update(ups, d)
    for world in (1, 2, 3):
        for r in range(world):
            gb, ge = group_range(groups, world, r)
            b_0, b_1 = byte_range(L, gb, ge)
            win = np.zeros((M, 16 * (ge - gb)), np.uint8)
            for c, u in enumerate(ups):
                win[c, : b_1 - b_0] = np.frombuffer(u, np.uint8)[b_0:b_1]
            out = torch.zeros(16 * (ge - gb), dtype=torch.uint8, device="cuda")
            codec.update_device(torch.from_numpy(win).cuda(), L, d, hp, out, None, gb, ge, window=True)
            torch.cuda.synchronize()
            codec.check()
            assert out.cpu().numpy()[: b_1 - b_0].tobytes() == whole[b_0:b_1], (world, r)
