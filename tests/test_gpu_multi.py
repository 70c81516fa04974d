"""fleet_update_multi: one update spread over several device contexts from one
process (SURVEY.md §8e element sharding through the C-ABI), byte-identical to
the oracle's faithful per-op chain (CppNNUpdater.java:420-509).

The box has one GPU, so the N contexts all live on device 0 -- each with its
own stream, pinned staging and device buffers, exactly as on N devices; the
window split, the per-context staging of column windows from the caller's
buffers and the disjoint D2H slices are what is under test.
"""
import numpy as np
import pytest

import fleet_amd as F
from fleet_amd.layouts import CIFAR10, MNIST, synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def contexts():
    cs = [F.Codec(0) for _ in range(8)]
    yield cs
    for c in cs:
        c.close()


def uploads_for(oracle, layout, M, seed):
    return [oracle.encode_floats(oracle.synth_upload(seed, c, list(layout.w_sizes), list(layout.b_sizes)))
            for c in range(M)]


@pytest.mark.parametrize("N", [1, 2, 3, 8])
@pytest.mark.parametrize("layout,M", [(MNIST, 6), (synthetic(1001), 4), (synthetic(20), 3)])
def test_update_multi_vs_faithful_chain(contexts, oracle, N, layout, M):
    ups = uploads_for(oracle, layout, M, seed=11 + N)
    d = [1.0 / ((c % 3) + 1) for c in range(M)]
    expected = oracle.update_faithful(ups, d)
    merged, f32 = F.update_multi(contexts[:N], ups, d, want_f32=True)
    assert merged == expected
    assert np.array_equal(f32.view(np.uint32), oracle.decode_floats(expected).view(np.uint32))


def test_update_multi_more_contexts_than_groups(contexts, oracle):
    # 7 values = 3 groups over 8 contexts: five contexts get an empty window
    ups = uploads_for(oracle, synthetic(7), 2, seed=5)
    d = [1.0, 0.5]
    assert F.update_multi(contexts, ups, d) == oracle.update_faithful(ups, d)


def test_update_multi_cifar_matches_single(contexts, oracle):
    ups = uploads_for(oracle, CIFAR10, 5, seed=3)
    d = [np.exp(-0.3 * c) for c in range(5)]
    one = contexts[0].update(ups, d)
    assert F.update_multi(contexts[:3], ups, d) == one
    hm = oracle.header_mask(list(CIFAR10.w_sizes), list(CIFAR10.b_sizes))
    assert one == oracle.update_fused(ups, d, hm)


def test_update_multi_errors(contexts, oracle):
    ups = uploads_for(oracle, MNIST, 3, seed=2)
    d = [1.0, 1.0, 1.0]
    # a bad Base64 char inside the LAST context's window is reported on contexts[0]
    bad = bytearray(ups[1])
    bad[len(bad) - 40] = ord("*")
    with pytest.raises(F.Base64Error):
        F.update_multi(contexts[:4], [ups[0], bytes(bad), ups[2]], d)
    # a header slot that differs from the last upload's (layout consistency)
    other = oracle.encode_floats(oracle.synth_upload(2, 0, [200, 0, 128, 19200, 0, 1921], [784, 0, 512, 0, 0, 192, 9]))
    with pytest.raises(F.LayoutError):
        F.update_multi(contexts[:2], [other, ups[1], ups[2]], d)
    with pytest.raises(F.FleetError):
        F.update_multi([contexts[0], contexts[0]], ups, d)
    # the contexts stay usable after an error
    assert F.update_multi(contexts[:4], ups, d) == oracle.update_faithful(ups, d)


@pytest.mark.parametrize("threads,pieces", [("4", "5"), ("3", "1"), ("8", "16")])
def test_update_threaded_staging(contexts, oracle, plan, threads, pieces):
    # the host-buffer path's parallel staging copy (large batches) on a small batch
    plan(f"stage_threads={threads},stage_pieces={pieces}")
    ups = uploads_for(oracle, CIFAR10, 7, seed=9)
    d = [1.0 / ((c % 3) + 1) for c in range(7)]
    hm = oracle.header_mask(list(CIFAR10.w_sizes), list(CIFAR10.b_sizes))
    expected = oracle.update_fused(ups, d, hm)
    assert contexts[0].update(ups, d) == expected
    assert F.update_multi(contexts[:2], ups, d) == expected


@pytest.mark.parametrize("N", [1, 3])
@pytest.mark.parametrize("pad", [0, 3, 16])
@pytest.mark.parametrize("pinned", [False, True])
def test_update_rows(contexts, oracle, N, pad, pinned):
    # uploads as the rows of one host buffer (a direct ByteBuffer's layout); page-locked
    # rows are DMAed per context column window with no host copy
    ups = uploads_for(oracle, MNIST, 5, seed=21 + pad)
    d = [1.0 / ((c % 3) + 1) for c in range(5)]
    L = len(ups[0])
    rows = np.full((5, L + pad), ord("!"), np.uint8)  # bytes past len are never read as values
    for i, u in enumerate(ups):
        rows[i, :L] = np.frombuffer(u, np.uint8)
    if pinned:
        contexts[0].register_host(rows)
    try:
        merged, f32 = F.update_rows(contexts[:N], rows, L, d, want_f32=True)
    finally:
        if pinned:
            contexts[0].unregister_host(rows)
    expected = oracle.update_faithful(ups, d)
    assert merged == expected
    assert np.array_equal(f32.view(np.uint32), oracle.decode_floats(expected).view(np.uint32))


def test_entry_points_keep_the_callers_device(contexts, oracle):
    """Every C-ABI entry restores the calling thread's current device (fleet_codec.cpp
    DeviceGuard): creating a context on the last visible GPU, a multi-context update,
    device-resident and host-buffer calls leave torch's current device as it was."""
    torch = pytest.importorskip("torch")
    n = torch.cuda.device_count()
    before = torch.cuda.current_device()
    last = F.Codec(n - 1)
    try:
        assert torch.cuda.current_device() == before
        ups = uploads_for(oracle, MNIST, 3, seed=5)
        d = [1.0, 0.5, 0.25]
        assert F.update_multi([contexts[0], last] if n > 1 else contexts[:2], ups, d) == oracle.update_faithful(ups, d)
        assert torch.cuda.current_device() == before
        assert last.update(ups, d) == oracle.update_faithful(ups, d)
        assert torch.cuda.current_device() == before
        last.check()
        assert torch.cuda.current_device() == before
    finally:
        last.close()
    assert torch.cuda.current_device() == before
