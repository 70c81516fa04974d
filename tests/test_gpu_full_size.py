"""Parity at BASELINE.json's full sizes (SURVEY.md §8d configs[2]-[4] and the 1 M-float
north-star bucket), by sampled columns.

The aggregation is element-wise (every value's chain runs over all M clients in
client order and no other value enters it), so the merged text of any subset of
3-value groups equals the oracle's fused update (oracle/fleet_oracle.c
fo_update_fused, parity status in oracle/fleet_oracle.h) run on
the uploads cut down to those groups. The full-size uploads are generated and
encoded on the GPU (k_synth, k_encode_f32), aggregated by the kernel the launch
plan picks at that size, and ~1,500 random groups plus the (padded) last group
are checked byte for byte, with merged_f32 at the same positions bitwise.

The same uploads then go through the pipelined step the bench times
(fleet_update_encode_device: k_update_encode<256> on the stream sizes,
k_update_tiled_encode at CIFAR sizes) at the full client count, with a second
synthetic batch as the next round's values: its merged text and merged_f32 are
checked against the same oracle result, and the next batch's uploads it writes
against the oracle's client encode (fo_encode_floats, Base64.cpp:104-169) of the
sampled values -- Base64 groups are independent, so the cut-down text of the
sampled groups is the encode of the sampled values."""
import numpy as np
import pytest

import fleet_amd as F
from fleet_amd.layouts import LAYOUTS

pytestmark = pytest.mark.gpu

# workload -> (layout, clients M, GiB of device memory the test holds at its peak)
FULL = {
    "cifar10_256": ("cifar10", 256, 1),
    "cifar100_1024": ("cifar100", 1024, 4),
    "synth1m_256": ("synth1m", 256, 3),
    "synth4m_4096": ("synth4m", 4096, 152),
}


@pytest.mark.parametrize("name", sorted(FULL))
def test_full_size_sampled_groups(codec, oracle, name):
    torch = pytest.importorskip("torch")
    lay_name, M, gib = FULL[name]
    free, _ = torch.cuda.mem_get_info()
    if free < (gib + 8) * 2**30:
        pytest.skip(f"{name} needs ~{gib} GiB of free device memory")
    lay = LAYOUTS[lay_name]
    n = lay.n_up
    groups = (n + 2) // 3
    L = F.b64_len(n)
    hp = np.asarray(lay.header_positions(), np.int32)
    rng = np.random.default_rng(sum(map(ord, name)))
    dampen = rng.uniform(0.05, 2.0, M)
    dev = torch.device("cuda", 0)
    values = torch.empty((M, 3 * groups), dtype=torch.float32, device=dev)
    codec.synth_device(20261016, values, n, hp, lay.header_values())
    text = torch.empty((M, 16 * groups), dtype=torch.uint8, device=dev)
    codec.encode_device(values, n, text)
    codec.check()
    del values
    torch.cuda.empty_cache()
    merged = torch.zeros(16 * groups, dtype=torch.uint8, device=dev)
    merged_f32 = torch.zeros(3 * groups, dtype=torch.float32, device=dev)
    codec.update_device(text, L, dampen, hp, merged, merged_f32)
    codec.check()

    # sampled groups, the last (padded) group last, so the cut-down texts are valid Base64
    sel = np.sort(rng.choice(groups - 1, size=min(1500, groups - 1), replace=False))
    sel = np.append(sel, groups - 1)
    tail = L - 16 * (groups - 1)  # bytes of the last group
    cols = (16 * sel[:, None] + np.arange(16)[None, :]).reshape(-1)
    cols = cols[: cols.size - (16 - tail)]
    cols_t = torch.from_numpy(cols).to(dev)
    pos = (3 * sel[:, None] + np.arange(3)[None, :]).reshape(-1)
    pos = pos[pos < n]
    pos_t = torch.from_numpy(pos).to(dev)
    sub = text.index_select(1, cols_t).cpu().numpy()
    got = merged.index_select(0, cols_t).cpu().numpy().tobytes()
    got_f32 = merged_f32.index_select(0, pos_t).cpu().numpy()
    del merged, merged_f32

    # the pipelined step at full M: this batch's aggregation + the next batch's encode
    # (peak: the uploads, the next batch's values and its uploads)
    free, _ = torch.cuda.mem_get_info()
    need = M * 16 * groups + M * 12 * groups + 4 * 2**30
    assert free > need, f"{name}: {free / 2**30:.1f} GiB free, the fused step needs {need / 2**30:.1f}"
    values_next = torch.empty((M, 3 * groups), dtype=torch.float32, device=dev)
    codec.synth_device(20261018, values_next, n, hp, lay.header_values())
    text_next = torch.empty_like(text)
    fmerged = torch.zeros(16 * groups, dtype=torch.uint8, device=dev)
    fmerged_f32 = torch.zeros(3 * groups, dtype=torch.float32, device=dev)
    codec.update_encode_device(text, L, dampen, hp, fmerged, fmerged_f32, values_next, text_next)
    torch.cuda.synchronize()
    codec.check()
    kernel = F.update_encode_kernel(L)
    fgot = fmerged.index_select(0, cols_t).cpu().numpy().tobytes()
    fgot_f32 = fmerged_f32.index_select(0, pos_t).cpu().numpy()
    nsub = text_next.index_select(1, cols_t).cpu().numpy()
    nvals = values_next.index_select(1, pos_t).cpu().numpy()
    del text, text_next, values_next, fmerged, fmerged_f32
    torch.cuda.empty_cache()

    hm = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))[pos]
    ups = [sub[c].tobytes() for c in range(M)]
    exp, exp_f32 = oracle.update_fused(ups, dampen, hm, threads=16, want_f32=True)
    assert len(got) == 16 * (sel.size - 1) + tail and len(ups) == M
    assert got == exp, name
    assert np.array_equal(got_f32.view(np.uint32), exp_f32.view(np.uint32)), name
    # the timed kernel (k_update_encode / k_update_tiled_encode) at the full client count
    assert fgot == exp, (name, kernel)
    assert np.array_equal(fgot_f32.view(np.uint32), exp_f32.view(np.uint32)), (name, kernel)
    for c in range(M):
        assert nsub[c].tobytes() == oracle.encode_floats(nvals[c]), (name, kernel, c)
    print(name, M, kernel)


def test_full_size_host_ingress_paths(oracle):
    """synth1m_256 through every host-side entry (fleet_update staged by the worker pool,
    fleet_update_rows from page-locked rows, fleet_update_multi / _rows_multi over three
    contexts) gives the device-resident update's bytes, which test_full_size_sampled_groups
    pins to the oracle; plus the fused Kardam norms at full size vs fleet_kardam_grads
    (rtol 1e-12 as in test_gpu_kardam_fused.py)."""
    torch = pytest.importorskip("torch")
    free, _ = torch.cuda.mem_get_info()
    if free < 12 * 2**30:
        pytest.skip("needs ~12 GiB of free device memory")
    lay = LAYOUTS["synth1m"]
    M = 256
    n = lay.n_up
    groups = (n + 2) // 3
    L = F.b64_len(n)
    hp = np.asarray(lay.header_positions(), np.int32)
    rng = np.random.default_rng(7)
    dampen = rng.uniform(0.05, 2.0, M)
    dev = torch.device("cuda", 0)
    cs = [F.Codec(0) for _ in range(3)]
    try:
        codec = cs[0]
        values = torch.empty((M, 3 * groups), dtype=torch.float32, device=dev)
        codec.synth_device(20261017, values, n, hp, lay.header_values())
        text = torch.empty((M, 16 * groups), dtype=torch.uint8, device=dev)
        codec.encode_device(values, n, text)
        codec.check()
        del values
        merged = torch.zeros(16 * groups, dtype=torch.uint8, device=dev)
        merged_f32 = torch.zeros(3 * groups, dtype=torch.float32, device=dev)
        codec.update_device(text, L, dampen, hp, merged, merged_f32)
        codec.check()
        want = merged.cpu().numpy()[:L].tobytes()
        want_f32 = merged_f32.cpu().numpy()[:n]
        rows = np.ascontiguousarray(text.cpu().numpy())  # [M, 16*groups], rows[i, :L] = upload i
        ups = [rows[i, :L].tobytes() for i in range(M)]

        got, f32 = codec.update(ups, dampen, want_f32=True)
        assert got == want
        assert np.array_equal(f32[:n].view(np.uint32), want_f32.view(np.uint32))
        assert F.update_multi(cs, ups, dampen) == want
        del ups
        codec.register_host(rows)
        try:
            assert codec.update_rows(rows, L, dampen) == want
            assert F.update_rows(cs, rows, L, dampen) == want
        finally:
            codec.unregister_host(rows)
        assert F.update_rows(cs[:2], rows, L, dampen) == want  # pageable rows: staged copy

        # Kardam side outputs at full size on a 16-client slice (kardam_grads is host-paced)
        K = 16
        lr = 0.05
        kd = dampen[:K]
        kmerged = torch.zeros(16 * groups, dtype=torch.uint8, device=dev)
        ng, nd = codec.update_kardam_device(text[:K].contiguous(), L, kd, hp, lr, kmerged,
                                            g_out_f32=torch.zeros((K, n + 3), dtype=torch.float32, device=dev))
        codec.check()
        _, eng, _ = codec.kardam_grads([rows[i, :L].tobytes() for i in range(K)], kd, lr)
        np.testing.assert_allclose(ng, eng, rtol=1e-12, atol=0)
        assert np.all(np.isnan(nd))
        assert kmerged.cpu().numpy()[:L].tobytes() == codec.update([rows[i, :L].tobytes() for i in range(K)], kd)
    finally:
        for c in cs:
            c.close()
        torch.cuda.empty_cache()
