"""Kardam's bookkeeping as side outputs of the fused update (fleet_update_kardam_device,
SURVEY.md §8 f2: CppNNUpdater.java:463-481, Kardam.java:48-106) against the
two-pass path (fleet_kardam_grads, itself checked against the oracle's per-op
chain in test_updater.py): same merged bytes as the plain update, the same
decoded Kardam gradients (bitwise), norms within 1e-12 relative (getNorm's fp64
sum in another order, as for fleet_norm)."""
import numpy as np
import pytest
import torch

import fleet_amd as F
from fleet_amd.layouts import CIFAR10, MNIST, synthetic

pytestmark = pytest.mark.gpu


def scatter_flat(flat, layout):
    """flat (getFlatGradient order) -> upload coordinates, header slots 0."""
    out = np.zeros(layout.n_up, np.float32)
    mask = np.ones(layout.n_up, bool)
    mask[layout.header_positions()] = False
    out[mask] = flat
    return out


# every launch plan of the update carries the side outputs: the pipelined tiles
# (MNIST, small buckets), the wide tiles at TG = 32 and 64 (CIFAR-10 sizes) and
# the stream kernel (1 M floats)
@pytest.mark.parametrize("layout,M", [(MNIST, 6), (synthetic(3001), 4), (CIFAR10, 5), (synthetic(120_001), 3),
                                      (synthetic(1_048_576), 2)])
def test_kardam_side_outputs(codec, oracle, layout, M):
    check_side_outputs(codec, oracle, layout, M)


@pytest.mark.parametrize("spec", ["update=stream,grid=plain", "update=stream,grid=lanes", "update=stream",
                                  "update=tiled", "update=tiled,flat_w2=16", "update=tiled,flat_w2=32",
                                  "update=tiled,flat_w2=21", "update=tiled,tile=classic", "update=pipe"])
def test_kardam_side_outputs_under_plans(codec, oracle, plan, spec):
    """Every launch plan's Kardam form on ragged sizes: the stream kernel's group-per-
    lane and value-per-lane blocks (k_update_mixed<256, true>), the flat tiles with each
    narrow width (k_update_flat_kd; a width other than 16 / 32 / 64, or tile=classic,
    keeps the flat tiles at their planned widths), the pipelined tiles."""
    plan(spec)
    for layout, M in ((synthetic(3001), 4), (synthetic(50_003), 3), (MNIST, 5)):
        check_side_outputs(codec, oracle, layout, M)


def check_side_outputs(codec, oracle, layout, M):
    dev = torch.device("cuda", 0)
    lr = 0.05
    d = [1.0 / ((c % 3) + 1) for c in range(M)]
    L = F.b64_len(layout.n_up)
    pitch = 16 * ((L + 15) // 16)
    vpitch = layout.n_up + 3
    hpos = layout.header_positions()

    def round_(seed, prev_texts, prev_dev, has, in_place=False):
        ups = [oracle.encode_floats(oracle.synth_upload(seed, c, list(layout.w_sizes), list(layout.b_sizes)))
               for c in range(M)]
        host = np.zeros((M, pitch), np.uint8)
        for c, u in enumerate(ups):
            host[c, :L] = np.frombuffer(u, np.uint8)
        t = torch.from_numpy(host).to(dev)
        merged = torch.zeros(pitch, dtype=torch.uint8, device=dev)
        # in_place: this round's G replaces prev in the same rows
        g_out = prev_dev if in_place else torch.zeros((M, vpitch), dtype=torch.float32, device=dev)
        ng, nd = codec.update_kardam_device(t, L, d, hpos, lr, merged, None, prev_dev, has, g_out)
        codec.check()
        print(layout.n_up, M, F.update_kernel(L))
        torch.cuda.synchronize()
        assert merged.cpu().numpy()[:L].tobytes() == codec.update(ups, d)
        prev_arg = None if prev_texts is None else [p if h else None for p, h in zip(prev_texts, has)]
        g_texts, eng, end = codec.kardam_grads(ups, d, lr, prev_arg)
        G = g_out.cpu().numpy()[:, : layout.n_up]
        for c in range(M):
            want = scatter_flat(codec.decode_floats(g_texts[c]), layout)
            assert np.array_equal(G[c].view(np.uint32), want.view(np.uint32))
        np.testing.assert_allclose(ng, eng, rtol=1e-12, atol=0)
        if prev_texts is None:
            assert np.all(np.isnan(nd))
        else:
            for c in range(M):
                if has[c]:
                    np.testing.assert_allclose(nd[c], end[c], rtol=1e-12, atol=1e-300)
                else:
                    assert np.isnan(nd[c])
        return g_texts, g_out

    g1, g1_dev = round_(31, None, None, None)
    has = [c % 2 == 0 for c in range(M)]
    g2, g2_dev = round_(32, g1, g1_dev, has)
    round_(33, g2, g2_dev, [True] * M, in_place=True)


def test_kardam_pipelined_flags_across_sizes(codec, oracle, plan):
    """The pipelined form's finish blocks wait on per-tile epoch flags held by the
    context (k_update_pipe<..., true>): a bigger bucket grows the flags (new ones start
    at 0, and the epoch restarts), a smaller one after it reuses the first flags with a
    newer epoch -- every call equals the two-pass path, none waits on a stale flag."""
    plan("update=pipe")
    for layout, M in ((MNIST, 3), (synthetic(50_003), 2), (synthetic(3001), 5), (MNIST, 3)):
        check_side_outputs(codec, oracle, layout, M)


def test_kardam_pipelined_timeout_fails_the_call(codec, oracle, plan):
    """A tile flag that never arrives (the reduce blocks made to wait for a later
    epoch by the test hook) fails fleet_update_kardam_device itself instead of
    returning norms summed from unfinished tiles; the next call, with the
    normal hand-off, is exact again and the context's error word is clean."""
    plan("update=pipe")
    layout, M = MNIST, 2
    L = F.b64_len(layout.n_up)
    pitch = 16 * ((L + 15) // 16)
    ups = [oracle.encode_floats(oracle.synth_upload(41, c, list(layout.w_sizes), list(layout.b_sizes)))
           for c in range(M)]
    host = np.zeros((M, pitch), np.uint8)
    for c, u in enumerate(ups):
        host[c, :L] = np.frombuffer(u, np.uint8)
    t = torch.from_numpy(host).cuda()
    merged = torch.zeros(pitch, dtype=torch.uint8, device="cuda")
    d = [1.0, 0.5]
    codec.test_kardam_skew(1)
    try:
        with pytest.raises(F.FleetError):
            codec.update_kardam_device(t, L, d, layout.header_positions(), 0.05, merged)
    finally:
        codec.test_kardam_skew(0)
    codec.check()
    ng, _ = codec.update_kardam_device(t, L, d, layout.header_positions(), 0.05, merged)
    codec.check()
    torch.cuda.synchronize()
    assert merged.cpu().numpy()[:L].tobytes() == codec.update(ups, d)
    _, eng, _ = codec.kardam_grads(ups, d, 0.05, None)
    np.testing.assert_allclose(ng, eng, rtol=1e-12, atol=0)
