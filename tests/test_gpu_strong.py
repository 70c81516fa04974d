"""bench.py's strong-scaling value is the N = 1 problem's bytes:
the N ranks' column windows, synthesised as the fixed problem's columns
(fleet_synth_window_device: same seed, global element index) and aggregated by the
bench's own per-rank step (the pipelined launch on the window as a bucket of its
own, headers re-based), concatenate to the merged text of the full-width update of
the same problem on one GPU -- byte for byte. Here every "rank" runs on the one
GPU of the box, one after the other; the all_gather only moves these slices."""
import os
import sys

import numpy as np
import pytest

import fleet_amd as F
from fleet_amd.layouts import LAYOUTS

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def _full_width(bench, torch, codec, layout, M):
    sh = bench.Shard(codec, torch, layout, M, 0, 1)
    sh.encode()
    sh.aggregate()
    torch.cuda.synchronize()
    codec.check()
    return sh.merged.cpu().numpy().copy(), sh


@pytest.mark.parametrize("lay_name,M", [("synth1m", 6), ("cifar10", 5), ("mnist", 7), ("synth1m", 1)])
def test_strong_windows_compose_to_the_one_gpu_text(codec, lay_name, M):
    torch = pytest.importorskip("torch")
    bench = _bench()
    layout = LAYOUTS[lay_name]
    full, whole = _full_width(bench, torch, codec, layout, M)
    G = (layout.n_up + 2) // 3
    for world in (2, 3, 8):
        parts = []
        for rank in range(world):
            sh = bench.Shard(codec, torch, layout, M, rank, world, strong=True)
            # the window's uploads are the full problem's columns
            sh.encode()
            b0 = 16 * sh.gb
            assert torch.equal(sh.text[:, : 16 * sh.groups], whole.text[:, b0: b0 + 16 * sh.groups]), (world, rank)
            # the bench's per-rank step (strong_pipelined's local()): the window as a bucket of its own
            v0 = 3 * sh.gb
            hloc = sh.hpos_global[(sh.hpos_global >= v0) & (sh.hpos_global < v0 + sh.n_local)] - v0
            src = torch.zeros(16 * sh.groups, dtype=torch.uint8, device=sh.text.device)
            nxt = torch.zeros_like(sh.text)
            codec.update_encode_device(sh.text, F.b64_len(sh.n_local), sh.dampen, hloc, src, sh.merged_f32,
                                       sh.values, nxt)
            torch.cuda.synchronize()
            codec.check()
            parts.append(src.cpu().numpy())
            # window mode in the fixed problem's coordinates (strong_device's step) gives the same slice
            sh.aggregate()
            torch.cuda.synchronize()
            codec.check()
            assert np.array_equal(sh.merged[: 16 * sh.groups].cpu().numpy(), parts[-1]), (world, rank)
            del sh, src, nxt
        got = np.concatenate(parts)
        assert got.size == 16 * G
        assert np.array_equal(got, full), (lay_name, M, world)
