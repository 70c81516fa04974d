"""Element-range sharding of the aggregation over the GPUs of a node.

The per-element chain of CppNNUpdater.update (CppNNUpdater.java:420-509) is
serial across clients but independent across elements, so rank r of N owns a
contiguous range of 16-char / 3-value Base64 groups of EVERY upload, runs the
exact chain there (fleet_update_device on just that window), and the merged
slices are all-gathered -- RCCL over xGMI with the "nccl" backend, gloo on CPU.
No reduction crosses ranks, so the result is byte-identical to one GPU's.

ClientShardedUpdater is the opt-in APPROXIMATE alternative (SURVEY.md §8e's
"approx" mode, the literal "RCCL reduce producing the final model delta"): rank r
aggregates its block of clients with the exact chain, and one all_reduce sums the
ranks' partial averages. That reorders the re-quantised adds of
CppNNUpdater.java:490-493, so its text is NOT the reference's; `deviation`
reports how far it lands from the exact result.

One process per GPU (torch.distributed); every rank receives the full merged
Base64 (the reference returns it to the Java updater on the server host).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import b64_count


def group_range(groups: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced split of `groups` 3-value groups: [begin, end) of `rank`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    base, rem = divmod(groups, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def byte_range(length: int, begin: int, end: int) -> Tuple[int, int]:
    """Base64 bytes of groups [begin, end) in a text of `length` bytes."""
    return min(length, 16 * begin), min(length, 16 * end)


def gather_slices(local, sizes: Sequence[int], group=None):
    """All-gather variable-sized uint8 slices in rank order into one tensor.

    Slices are padded to the largest one so a single all_gather_into_tensor
    (one RCCL call over xGMI) moves them; sizes are known to every rank."""
    import torch
    import torch.distributed as dist
    world = len(sizes)
    mx = max(sizes) if sizes else 0
    buf = torch.zeros(max(mx, 1), dtype=torch.uint8, device=local.device)
    buf[: local.numel()] = local
    out = torch.empty(world * buf.numel(), dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    return torch.cat([out[r * buf.numel(): r * buf.numel() + sizes[r]] for r in range(world)])


class ShardedUpdater:
    """One rank's part of an N-GPU fused update (host uploads in, merged Base64 out).

    update(uploads, dampen) has CppNNUpdater.update's aggregation semantics
    (fleet_update): the same bytes on every rank, whatever N."""

    def __init__(self, codec, group=None, device=None):
        import torch
        import torch.distributed as dist
        self.codec = codec
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)

    # -- per-rank compute (HIP); the CPU tests substitute these two ---------
    def layout(self, last_upload: bytes) -> List[int]:
        """Header slots of the last picked upload (network::flatGrad walk, on device)."""
        pos, walk_end = self.codec.layout_parse(last_upload)
        n = b64_count(len(last_upload))
        # slots past the walk come from the last upload, exactly like header slots
        return [int(p) for p in pos] + list(range(walk_end, n))

    def local_update(self, window: np.ndarray, length: int, dampen, header_pos, begin: int, end: int):
        """Merged Base64 of groups [begin, end) from a host window [M, 16*(end-begin)]."""
        import torch
        dev = torch.from_numpy(window).pin_memory().to(self.device, non_blocking=True)
        merged = torch.empty(16 * (end - begin), dtype=torch.uint8, device=self.device)
        self.codec.update_device(dev, length, dampen, header_pos, merged, None, begin, end, window=True)
        self.codec.check()
        return merged

    def local_step(self, weights, fc_bias, window_f32, begin: int, end: int, layout, lr: float):
        """descentNative's model step on this rank's element shard: window_f32 is the
        merged fp32 of groups [begin, end) (update_device's merged_f32 in window mode);
        only the parameters those gradient positions cover are updated, in the
        full-size resident model, so the ranks' steps are disjoint and need no exchange."""
        self.codec.descent_window_device(weights, fc_bias, window_f32, 3 * begin, 3 * end, layout, lr)

    # -----------------------------------------------------------------------
    def update(self, uploads: Sequence[bytes], dampen: Sequence[float]) -> bytes:
        import torch
        import torch.distributed as dist
        M = len(uploads)
        if M == 0 or len(dampen) != M:
            raise ValueError("need one dampening factor per upload")
        L = len(uploads[0])
        if any(len(u) != L for u in uploads):
            raise ValueError("uploads differ in length (one layout per update)")
        groups = (b64_count(L) + 2) // 3
        begin, end = group_range(groups, self.world, self.rank)
        b0, b1 = byte_range(L, begin, end)
        status = 0
        local = torch.zeros(b1 - b0, dtype=torch.uint8, device=self.device)
        err: Optional[BaseException] = None
        try:
            hpos = self.layout(uploads[-1])
            window = np.zeros((M, 16 * (end - begin)), np.uint8)
            for c, u in enumerate(uploads):
                window[c, : b1 - b0] = np.frombuffer(u, np.uint8, count=b1 - b0, offset=b0)
            if end > begin:
                local = self.local_update(window, L, dampen, hpos, begin, end)[: b1 - b0]
        except Exception as e:  # keep the ranks in step: every rank raises together below
            err, status = e, 1
        if self.world > 1:
            flag = torch.tensor([status], dtype=torch.int32, device=self.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
            status = int(flag.item())
        if status:
            if err is not None:
                raise err
            raise RuntimeError("fleet update failed on another rank")
        if self.world == 1:
            return local.cpu().numpy().tobytes()
        sizes = [byte_range(L, *group_range(groups, self.world, r)) for r in range(self.world)]
        full = gather_slices(local, [s1 - s0 for s0, s1 in sizes], self.group)
        return full.cpu().numpy().tobytes()


class ClientShardedUpdater(ShardedUpdater):
    """Opt-in approximate aggregation sharded over CLIENTS ("approx").

    Rank r takes the contiguous block of picked uploads [cb, ce) (group_range over
    clients) and runs the exact chain of CppNNUpdater.update on them alone
    (fleet_update_device: decode, dampen, serial re-quantised sum, average by its
    own M_r), giving merged_f32_r = dec(merged_r). One all_reduce(SUM) in float64
    (RCCL over xGMI) of (M_r / M) * merged_f32_r gives the average over all M
    clients; header slots (and slots past the layout walk) carry the LAST upload's
    decoded codes, contributed with weight 1 by the rank holding client M-1. The
    sum is encoded (Base64::encode(vector<float>)) on every rank.

    Not bit-exact: the reference adds the M dampened uploads one by one,
    re-quantising after every add (CppNNUpdater.java:490-493); here each rank's
    block is summed that way and the blocks are added in float64 at the end, then
    quantised once. Use `deviation(approx, exact)` to report the difference; the
    exact, byte-identical default is ShardedUpdater (element sharding). Construct
    with approx=True to accept that: without it update() raises, so the mode is
    never mistaken for the exact path."""

    def __init__(self, codec, group=None, device=None, approx: bool = False):
        super().__init__(codec, group, device)
        self.approx = bool(approx)

    def _require_approx(self):
        if not self.approx:
            raise ValueError("ClientShardedUpdater is not the reference's bytes: construct it with approx=True "
                             "(the exact sharded update is ShardedUpdater)")

    def device_step(self, text_rows, length: int, dampen_block, header_pos, M: int, cb: int, merged, merged_f32,
                    out_text, values_buf=None):
        """The same step on device-resident uploads: text_rows [M_r, pitch] holds picked
        uploads [cb, cb + M_r) of M (rows of the full-width texts); dampen_block their
        factors. The rank's exact chain (fleet_update_device, averaged by M_r), the
        float64 all_reduce of its weighted partial (header slots: the last upload's
        values from the rank holding client M-1) and the encode of the float32 sum into
        out_text [>= 16 * groups] (fleet_encode_device). One rank: the exact chain's
        merged text itself. Returns nothing; every rank's out_text holds the result."""
        import torch
        import torch.distributed as dist
        self._require_approx()
        Mr = int(text_rows.shape[0])
        n = b64_count(length)
        if Mr:  # a rank without clients (M < world) still joins the all_reduce
            self.codec.update_device(text_rows, length, dampen_block, header_pos, merged, merged_f32)
        if self.world == 1:
            out_text[: merged.numel()].copy_(merged)
            return
        last = Mr > 0 and cb + Mr == M
        part = merged_f32[:n].double() if Mr else torch.zeros(n, dtype=torch.float64, device=merged_f32.device)
        # the header-slot mask, cached per (n, header positions): a later call with other
        # header positions at the same n must not reuse the old mask
        key = (n, tuple(int(h) for h in header_pos))
        cached = getattr(self, "_keep", None)
        if cached is None or cached[0] != key:
            keep = torch.zeros(n, dtype=torch.bool, device=part.device)
            if len(header_pos):
                keep[torch.as_tensor(np.asarray(header_pos), dtype=torch.long, device=part.device)] = True
            self._keep = cached = (key, keep)
        keep = cached[1]
        acc = torch.where(keep, part if last else torch.zeros_like(part), part * (Mr / M))
        dist.all_reduce(acc, op=dist.ReduceOp.SUM, group=self.group)
        vals = values_buf if values_buf is not None else torch.empty((1, 3 * ((n + 2) // 3)), dtype=torch.float32,
                                                                       device=part.device)
        vals[0, :n].copy_(acc)
        self.codec.encode_device(vals, n, out_text.view(1, -1))

    def local_partial(self, uploads: Sequence[bytes], dampen: Sequence[float], header_pos):
        """This rank's block of uploads through the exact chain: (merged_f32 as a
        float64 tensor of n values, the merged Base64 as bytes)."""
        import torch
        M, L = len(uploads), len(uploads[0])
        groups = (b64_count(L) + 2) // 3
        host = np.zeros((M, 16 * groups), np.uint8)
        for c, u in enumerate(uploads):
            host[c, :L] = np.frombuffer(u, np.uint8)
        dev = torch.from_numpy(host).pin_memory().to(self.device, non_blocking=True)
        merged = torch.empty(16 * groups, dtype=torch.uint8, device=self.device)
        f32 = torch.empty(3 * groups, dtype=torch.float32, device=self.device)
        self.codec.update_device(dev, L, dampen, header_pos, merged, f32)
        self.codec.check()
        return f32[: b64_count(L)].double(), merged[:L].cpu().numpy().tobytes()

    def encode(self, values) -> bytes:
        """Base64 text of the summed average (float32)."""
        return self.codec.encode_floats(values.float().cpu().numpy())

    def update(self, uploads: Sequence[bytes], dampen: Sequence[float]) -> bytes:
        import torch
        import torch.distributed as dist
        self._require_approx()
        M = len(uploads)
        if M == 0 or len(dampen) != M:
            raise ValueError("need one dampening factor per upload")
        L = len(uploads[0])
        if any(len(u) != L for u in uploads):
            raise ValueError("uploads differ in length (one layout per update)")
        n = b64_count(L)
        cb, ce = group_range(M, self.world, self.rank)
        last_owner = next(r for r in range(self.world) if group_range(M, self.world, r)[1] == M)
        acc = torch.zeros(n, dtype=torch.float64, device=self.device)
        status = 0
        err: Optional[BaseException] = None
        try:
            hpos = self.layout(uploads[-1])
            if ce > cb:
                part, text = self.local_partial(uploads[cb:ce], list(dampen[cb:ce]), hpos)
                if self.world == 1:
                    return text  # one rank holds every client: the exact chain
                keep = torch.zeros(n, dtype=torch.bool, device=self.device)
                if hpos:
                    keep[torch.as_tensor(hpos, dtype=torch.long, device=self.device)] = True
                acc = torch.where(keep, part if self.rank == last_owner else torch.zeros_like(part),
                                  part * ((ce - cb) / M))
        except Exception as e:  # every rank raises together below
            err, status = e, 1
        if self.world > 1:
            flag = torch.tensor([status], dtype=torch.int32, device=self.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
            status = int(flag.item())
        if status:
            if err is not None:
                raise err
            raise RuntimeError("fleet update failed on another rank")
        if self.world > 1:
            dist.all_reduce(acc, op=dist.ReduceOp.SUM, group=self.group)
        return self.encode(acc)


def deviation(approx: np.ndarray, exact: np.ndarray) -> dict:
    """How far an approximate merged gradient (decoded float32) lands from the exact
    one: the fraction of values that differ, the largest absolute difference and
    the largest difference relative to max(|exact|, 1e-30)."""
    a = np.asarray(approx, np.float32).astype(np.float64)
    e = np.asarray(exact, np.float32).astype(np.float64)
    if a.shape != e.shape:
        raise ValueError("different lengths")
    if a.size == 0:
        return {"n": 0, "frac_differ": 0.0, "max_abs": 0.0, "max_rel": 0.0}
    d = np.abs(a - e)
    return {"n": int(a.size), "frac_differ": float(np.mean(a != e)), "max_abs": float(d.max()),
            "max_rel": float((d / np.maximum(np.abs(e), 1e-30)).max())}
