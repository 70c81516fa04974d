"""The client-chunked stream update (launch_update / launch_update_encode for
many clients: launches of at most FLEET_UPDATE_CHUNK clients, the running sums
handed on through the merged output, NaN for a chain that left the q_gen domain)
against the oracle and against the one-launch update, byte for byte: both grid
forms, values outside the domain in early and late chunks, Base64 and layout
errors in a late chunk, element windows, the device-resident and the pipelined
step. Small chunks (2-3 clients) make every boundary case appear at test sizes."""
import numpy as np
import pytest

import fleet_amd as F
from fleet_amd.layouts import Layout, synthetic

pytestmark = pytest.mark.gpu


def _uploads(oracle, lay, M, seed, special_clients=()):
    rng = np.random.default_rng(seed)
    hpos = set(lay.header_positions())
    special = np.array([1e9, -1e8, np.inf, -np.inf, np.nan, 3e38, 1e8, 9.999999e7, 10.0, -10.0, 1e-45], np.float32)
    ups = []
    for c in range(M):
        v = oracle.synth_upload(seed + c, c, list(lay.w_sizes), list(lay.b_sizes)).copy()
        if c in special_clients:
            pos = [p for p in rng.integers(0, lay.n_up, 60) if p not in hpos]
            v[pos] = rng.choice(special, len(pos))
        ups.append(oracle.encode_floats(v))
    return ups


@pytest.mark.parametrize("mixed", ["1", "2", "0"])
@pytest.mark.parametrize("chunk", ["2", "3"])
def test_chunked_update_vs_oracle(codec, oracle, monkeypatch, mixed, chunk):
    monkeypatch.setenv("FLEET_UPDATE_MODE", "stream")
    monkeypatch.setenv("FLEET_UPDATE_MIXED", mixed)
    monkeypatch.setenv("FLEET_UPDATE_CHUNK", chunk)
    lay = synthetic(3 * 70000 + 2)
    M = 8
    ups = _uploads(oracle, lay, M, 90, special_clients=(1, 6))
    hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
    d = [1 / ((c % 3) + 1) for c in range(M)]
    got, f32 = codec.update(ups, d, want_f32=True)
    exp = oracle.update_fused(ups, d, hm)
    assert got == exp
    assert np.array_equal(f32.view(np.uint32), oracle.decode_floats(exp).view(np.uint32))


def test_chunked_errors_in_a_late_chunk(codec, oracle, monkeypatch):
    monkeypatch.setenv("FLEET_UPDATE_MODE", "stream")
    monkeypatch.setenv("FLEET_UPDATE_CHUNK", "2")
    lay = synthetic(3 * 70000 + 2)
    M = 7
    ups = _uploads(oracle, lay, M, 11)
    d = [1.0] * M
    bad = bytearray(ups[5])
    bad[16 * 40000 + 7] = ord("*")
    with pytest.raises(F.Base64Error):
        codec.update(ups[:5] + [bytes(bad)] + ups[6:], d)
    # client 6 with another header (a layout mismatch only the late chunk sees)
    other = Layout("x", (1000, 3 * 70000 + 2 - 1000 - 4), ())
    alien = oracle.encode_floats(oracle.synth_upload(5, 6, list(other.w_sizes), list(other.b_sizes)))
    assert len(alien) == len(ups[0])
    with pytest.raises(F.LayoutError):
        codec.update(ups[:6] + [alien], d)
    hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
    assert codec.update(ups, d) == oracle.update_fused(ups, d, hm)


def test_chunked_device_window_and_fused_step(codec, oracle, monkeypatch):
    torch = pytest.importorskip("torch")
    from fleet_amd.shard import group_range
    monkeypatch.setenv("FLEET_UPDATE_MODE", "stream")
    lay = synthetic(3 * 150001 + 1)
    M = 9
    n = lay.n_up
    groups = (n + 2) // 3
    dev = torch.device("cuda", 0)
    hp = np.asarray(lay.header_positions(), np.int32)
    hv = np.asarray(lay.header_values(), np.float32)
    vals = torch.empty((M, 3 * groups), dtype=torch.float32, device=dev)
    nxt = torch.empty_like(vals)
    codec.synth_device(5, vals, n, hp, hv)
    codec.synth_device(6, nxt, n, hp, hv)
    text = torch.zeros((M, 16 * groups), dtype=torch.uint8, device=dev)
    codec.encode_device(vals, n, text)
    L = F.b64_len(n)
    d = [1 / ((c % 3) + 1) for c in range(M)]

    def run(chunk):
        monkeypatch.setenv("FLEET_UPDATE_CHUNK", chunk)
        m = torch.zeros(16 * groups, dtype=torch.uint8, device=dev)
        f = torch.zeros(3 * groups, dtype=torch.float32, device=dev)
        codec.update_device(text, L, d, hp, m, f)
        wins = []
        for r in range(3):
            gb, ge = group_range(groups, 3, r)
            mw = torch.zeros(16 * (ge - gb), dtype=torch.uint8, device=dev)
            codec.update_device(text[:, 16 * gb:16 * ge].contiguous(), L, d, hp, mw, None, gb, ge, window=True)
            wins.append(mw)
        mf = torch.zeros_like(m)
        ff = torch.zeros_like(f)
        enc = torch.zeros_like(text)
        codec.update_encode_device(text, L, d, hp, mf, ff, nxt, enc)
        torch.cuda.synchronize()
        codec.check()
        return m, f, torch.cat(wins), mf, ff, enc

    a = run("0")
    b = run("4")
    for x, y in zip(a, b):
        assert torch.equal(x.view(torch.uint8) if x.dtype != torch.uint8 else x,
                           y.view(torch.uint8) if y.dtype != torch.uint8 else y)
    assert torch.equal(a[0], a[2]) and torch.equal(a[0], a[3])
    ref_next = torch.zeros_like(text)
    codec.encode_device(nxt, n, ref_next)
    assert torch.equal(b[5], ref_next)
    # and against the oracle on sampled groups
    ups = [bytes(text[c, :L].cpu().numpy()) for c in range(M)]
    hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
    assert bytes(b[0][:L].cpu().numpy()) == oracle.update_fused(ups, d, hm)

