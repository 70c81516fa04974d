"""N>1 path on CPU: element-range sharding + all_gather over gloo, world_size 2, 3 and 8
(the node size bench.py's scaling run uses).

fleet_amd.shard.ShardedUpdater is the product's multi-GPU driver; here its two
per-rank compute hooks (layout, local_update) are replaced by the oracle so the
partitioning, windowing, error agreement and the gather run under a real
torch.distributed process group without a GPU. The merged bytes must equal the
single-process oracle's (element sharding is exact: no cross-rank reduction).
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from fleet_amd import b64_count  # noqa: E402
from fleet_amd.layouts import MNIST, synthetic  # noqa: E402
from fleet_amd.shard import byte_range, group_range  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("groups,world", [(0, 2), (1, 2), (2, 3), (7654, 2), (7654, 8), (104623, 8), (5, 8)])
def test_group_range_partition(groups, world):
    spans = [group_range(groups, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == groups
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0
    sizes = [e - b for b, e in spans]
    assert max(sizes) - min(sizes) <= 1
    L = 16 * groups - 8 if groups else 0
    assert sum(e - b for b, e in (byte_range(L, *s) for s in spans)) == L


def _rank_main(rank, world, port, cases, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch

    import pyoracle
    from fleet_amd.shard import ShardedUpdater

    o = pyoracle.Oracle()

    class OracleRank(ShardedUpdater):
        """ShardedUpdater with the oracle standing in for the HIP window update."""

        def __init__(self, layout):
            super().__init__(codec=None, device="cpu")
            self.mask = o.header_mask(list(layout.w_sizes), list(layout.b_sizes))

        def layout(self, last_upload):
            return np.nonzero(self.mask)[0].tolist()

        def local_update(self, window, length, dampen, header_pos, begin, end):
            b0, b1 = byte_range(length, begin, end)
            ups = [window[c, : b1 - b0].tobytes() for c in range(window.shape[0])]
            n = b64_count(b1 - b0)
            mask = np.zeros(n, np.uint8)
            hp = np.asarray(header_pos, np.int64)
            sel = hp[(hp >= 3 * begin) & (hp < 3 * begin + n)] - 3 * begin
            mask[sel] = 1
            got = o.update_fused(ups, dampen, mask, threads=1)
            return torch.frombuffer(bytearray(got), dtype=torch.uint8)

    results = []
    for name, M in cases:
        lay = MNIST if name == "mnist" else synthetic(int(name))
        ups = [o.encode_floats(o.synth_upload(9, c, list(lay.w_sizes), list(lay.b_sizes))) for c in range(M)]
        d = [1.0 / ((c % 3) + 1) for c in range(M)]
        got = OracleRank(lay).update(ups, d)
        results.append(got == o.update_fused(ups, d, o.header_mask(list(lay.w_sizes), list(lay.b_sizes))))
    # error agreement: a failure on one rank raises on every rank (no hang in the gather)
    class Failing(OracleRank):
        def local_update(self, *a):
            if self.rank == world - 1:
                raise ValueError("boom")
            return super().local_update(*a)
    lay = synthetic(3000)
    ups = [o.encode_floats(o.synth_upload(9, c, list(lay.w_sizes), list(lay.b_sizes))) for c in range(2)]
    try:
        Failing(lay).update(ups, [1.0, 1.0])
        results.append(False)
    except (ValueError, RuntimeError):
        results.append(True)
    with open(os.path.join(out_dir, f"rank{rank}.txt"), "w") as f:
        f.write(" ".join("1" if r else "0" for r in results))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_update_gloo_matches_single_process(world, tmp_path):
    import torch.multiprocessing as mp
    cases = [("mnist", 4), ("1000", 3), ("1001", 1), ("4", 2)]
    mp.start_processes(_rank_main, args=(world, _free_port(), cases, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    for r in range(world):
        flags = (tmp_path / f"rank{r}.txt").read_text().split()
        assert flags == ["1"] * (len(cases) + 1), f"rank {r}: {flags}"


def _client_rank_main(rank, world, port, cases, out_dir):
    """ClientShardedUpdater (the opt-in approximate mode) with the oracle standing in
    for the per-rank HIP update and the encode; gloo carries the float64 all_reduce."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch

    import pyoracle
    from fleet_amd.shard import ClientShardedUpdater, deviation, group_range

    o = pyoracle.Oracle()

    class OracleClientRank(ClientShardedUpdater):
        def __init__(self, layout):
            super().__init__(codec=None, device="cpu", approx=True)
            self.mask = o.header_mask(list(layout.w_sizes), list(layout.b_sizes))

        def layout(self, last_upload):
            return np.nonzero(self.mask)[0].tolist()

        def local_partial(self, uploads, dampen, header_pos):
            text = o.update_fused(list(uploads), list(dampen), self.mask, threads=1)
            return torch.from_numpy(o.decode_floats(text).astype(np.float64)), text

        def encode(self, values):
            return o.encode_floats(values.float().numpy())

    class OracleDeviceCodec:
        """update_device / encode_device of the C-ABI on CPU tensors, by the oracle:
        drives ClientShardedUpdater.device_step (bench.py's approx block) under gloo."""

        def __init__(self, mask):
            self.mask = mask

        def update_device(self, rows, length, dampen, header_pos, merged, merged_f32):
            ups = [rows[c, :length].numpy().tobytes() for c in range(rows.shape[0])]
            text = o.update_fused(ups, list(dampen), self.mask, threads=1)
            merged[: len(text)] = torch.from_numpy(np.frombuffer(text, np.uint8).copy())
            f = o.decode_floats(text)
            merged_f32[: len(f)] = torch.from_numpy(f)

        def encode_device(self, vals, n, out):
            text = o.encode_floats(vals[0, :n].numpy())
            out[0, : len(text)] = torch.from_numpy(np.frombuffer(text, np.uint8).copy())

    lines = []
    for name, M in cases:
        lay = MNIST if name == "mnist" else synthetic(int(name))
        ups = [o.encode_floats(o.synth_upload(9, c, list(lay.w_sizes), list(lay.b_sizes))) for c in range(M)]
        d = [1.0 / ((c % 3) + 1) for c in range(M)]
        hm = o.header_mask(list(lay.w_sizes), list(lay.b_sizes))
        exact = o.update_fused(ups, d, hm)
        got = OracleClientRank(lay).update(ups, d)
        # the device-resident form (bench.py's approx block) gives the same text
        cb, ce = group_range(M, world, rank)
        if True:  # every rank joins the all_reduce, with or without clients
            L = len(ups[0])
            groups = (len(o.decode_floats(ups[0])) + 2) // 3
            rows = torch.zeros((ce - cb, 16 * groups), dtype=torch.uint8)
            for i, c in enumerate(range(cb, ce)):
                rows[i, :L] = torch.from_numpy(np.frombuffer(ups[c], np.uint8).copy())
            dev = ClientShardedUpdater(OracleDeviceCodec(hm), device="cpu", approx=True)
            out = torch.zeros(16 * groups, dtype=torch.uint8)
            dev.device_step(rows, L, d[cb:ce], np.nonzero(hm)[0].tolist(), M, cb,
                            torch.zeros(16 * groups, dtype=torch.uint8), torch.zeros(3 * groups),
                            out)
            assert out.numpy()[:L].tobytes() == got, (name, M)
        a, e = o.decode_floats(got), o.decode_floats(exact)
        dv = deviation(a, e)
        ok = (len(got) == len(exact) and np.array_equal(a[hm != 0], e[hm != 0])
              and dv["max_abs"] <= 2e-6 * max(1.0, float(np.abs(e).max())))
        lines.append("%d %s %d %.6g %.6g" % (ok, name, M, dv["frac_differ"], dv["max_abs"]))
    with open(os.path.join(out_dir, f"crank{rank}.txt"), "w") as f:
        f.write("\n".join(lines))
    dist.destroy_process_group()


def test_client_sharded_needs_explicit_approx():
    """The approximate mode refuses to run unless asked for by name (approx=True)."""
    from fleet_amd.shard import ClientShardedUpdater
    cs = ClientShardedUpdater(codec=None, device="cpu")
    with pytest.raises(ValueError, match="approx=True"):
        cs.update([b"AAAA"], [1.0])


@pytest.mark.parametrize("world", [2, 3, 8])
def test_client_sharded_approx_gloo(world, tmp_path):
    """The approximate client-sharded mode: header slots exact, payload within a
    bound of the exact chain (|diff| <= 2e-6 max|exact| on the synthetic mix), the
    same text on every rank; M < world leaves ranks without clients."""
    import torch.multiprocessing as mp
    cases = [("mnist", 8), ("1000", 5), ("5000", 2)]
    mp.start_processes(_client_rank_main, args=(world, _free_port(), cases, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    texts = [(tmp_path / f"crank{r}.txt").read_text().splitlines() for r in range(world)]
    for r in range(world):
        assert all(line.startswith("1 ") for line in texts[r]), texts[r]
        assert texts[r] == texts[0]
