#!/usr/bin/env python3
"""bench.py -- gradient GiB/s encode+decode+aggregate (device-resident) on MI355X.

One step = the hot path over one batch of M synthetic client gradient buckets
already resident in HBM:
  1. client-side encode  (Base64::encode(vector<float>) of every bucket)
  2. server aggregation  (CppNNUpdater.update's decode/dampen/sum/average/merge
                          chain, bit-exact) -> merged Base64 + fp32
`value` times the steps software-pipelined over two upload buffers: step i
aggregates batch i and encodes batch i+1 in ONE launch (k_update_encode /
k_update_tiled_encode / k_update_pipe with encode blocks;
fleet_update_encode_device), batch 0 encoded before the clock. The sequential
form (k_encode_f32, then k_update*) is reported beside it (`sequential`;
--sequential makes it the value).

Headline (N=1): synth1m_256, the north-star configuration (1 M-float buckets,
C = 256 clients, 1.43 GB of Base64 >> the 256 MiB Infinity Cache).

Multi-GPU (element-range sharding):
  * `value` is strong scaling of ONE fixed problem, the headline's: synth1m_256
    split over the N ranks by 3-value group ranges; each rank's step is the same
    pipelined launch on its column window (aggregation of batch i + encode of
    batch i+1) followed by the all_gather of the merged slices (RCCL over xGMI)
    inside the timed step, so every rank ends the step holding the whole merged
    text. At N=1 this is exactly the headline step (no gather).
  * `weak` beside it: every rank a full-size synth1m_256 slice of a model N times
    larger, no collective in the timed steps (all_gather timed separately).
  * the `strong` block splits the larger configs over the N ranks: configs[4]
    (synthetic 4 M floats x 4096 clients) device-resident, timed with the
    all_gather of the merged slices inside the step and without it; and
    configs[3] (CIFAR-100 x 1024) host-staged: pinned-host H2D of the rank's
    column window + aggregation + D2H of its merged slice (+ the gather).
  * --strong makes the strong configs[4] gather-inside line the `value`.
  * `python bench.py --gpus N` without a launcher starts its N ranks itself
    (torch.distributed.run as a child process, before anything touches a GPU);
    under a launcher, --gpus must equal WORLD_SIZE.

Output: ONE JSON line on rank 0 (see DESIGN.md §6 for every field).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# workload name -> (layout, clients M, BASELINE.json config index or note)
# timed steps of the small extra workloads at least (see main)
EXTRA_MIN_STEPS = {"mnist64": 200, "cifar10_256": 20}

WORKLOADS = {
    "mnist64": ("mnist", 64, "configs[1]: MNIST cppNN gradient buckets, 64 simulated clients"),
    "cifar10_256": ("cifar10", 256, "configs[2]: CIFAR-10 cppNN gradient buckets, 256 clients"),
    "cifar100_1024": ("cifar100", 1024, "configs[3]: CIFAR-100 cppNN gradient buckets, 1024 clients"),
    "synth1m_256": ("synth1m", 256, "north-star target: 1M-float buckets, C=256 (SURVEY.md §8d)"),
    "synth4m_4096": ("synth4m", 4096, "configs[4]: synthetic 4M-float buckets x 4096 clients"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md:36
HBM_COPY_GBS = 6290.0  # measured copy ceiling, same line (SURVEY.md §8d asks for both)
# what actually bounds each aggregation kernel: none is HBM-bound
LIMITER = {
    "k_update_pipe": "latency of the serial client chain (one consumer wave per tile; DESIGN.md 4.2)",
    "k_update_tiled": "VALU issue (exact chain)",
    "k_update": "VALU issue (exact chain)",
}


def dampen_policy(M: int):
    """policy 1 (inverse, CppNNUpdater.java:307-308) with tau = c mod 3."""
    return [1.0 / ((c % 3) + 1) for c in range(M)]


def group_range(groups: int, world: int, rank: int):
    from fleet_amd.shard import group_range as gr
    return gr(groups, world, rank)


class Shard:
    """One rank's device-resident slice of a workload.

    weak (default): a full-size bucket slice per rank.
    strong: the rank's column window [gb, ge) of the ONE fixed problem, synthesised
    in place as that problem's columns (the same seed on every rank, the global
    element index as the generator's counter, the header slots that fall inside),
    so the N windows together hold exactly the N = 1 problem's uploads."""

    def __init__(self, codec, torch, layout, M, rank, world, seed=1, strong=False):
        import fleet_amd as F
        self.F = F
        self.torch = torch
        self.codec = codec
        self.M = M
        self.strong = strong
        hpos = np.asarray(layout.header_positions(), dtype=np.int32)
        hval = np.asarray(layout.header_values(), dtype=np.float32)
        if strong:
            G = (layout.n_up + 2) // 3
            self.gb, self.ge = group_range(G, world, rank)
            self.groups = self.ge - self.gb
            v0, v1 = 3 * self.gb, min(layout.n_up, 3 * self.ge)
            self.n_local = max(0, v1 - v0)            # values of this window
            self.L = F.b64_len(layout.n_up)           # the fixed problem's upload length
            keep = (hpos >= v0) & (hpos < v1)
            self.hpos_global = hpos
            syn_pos, syn_val = hpos[keep] - v0, hval[keep]
        else:
            self.gb, self.ge = 0, (layout.n_up + 2) // 3
            self.groups = self.ge
            self.n_local = layout.n_up
            self.L = F.b64_len(self.n_local)
            self.hpos_global = hpos
            syn_pos, syn_val = hpos, hval
        self.pitch = 16 * max(1, self.groups)
        self.vpitch = 3 * max(1, self.groups)
        dev = torch.device("cuda", torch.cuda.current_device())
        self.values = torch.empty((M, self.vpitch), dtype=torch.float32, device=dev)
        self.text = torch.zeros((M, self.pitch), dtype=torch.uint8, device=dev)
        self.merged = torch.zeros((self.pitch,), dtype=torch.uint8, device=dev)
        self.merged_f32 = torch.empty((self.vpitch,), dtype=torch.float32, device=dev)
        if self.n_local:
            codec.synth_device(seed, self.values, self.n_local, syn_pos, syn_val,
                               elem0=3 * self.gb if strong else 0)
        self.dampen = np.asarray(dampen_policy(M), dtype=np.float64)
        torch.cuda.synchronize()

    def encode(self):
        if self.n_local:
            self.codec.encode_device(self.values, self.n_local, self.text)

    def aggregate(self):
        if not self.n_local:
            return
        if self.strong:
            self.codec.update_device(self.text, self.L, self.dampen, self.hpos_global, self.merged, self.merged_f32,
                                     self.gb, self.ge, window=True)
        else:
            self.codec.update_device(self.text, self.L, self.dampen, self.hpos_global, self.merged, self.merged_f32)

    def algorithmic_bytes(self):
        """Per launch: k_update reads M*L Base64, writes L Base64 + 4*n fp32;
        k_encode_f32 reads 4*n*M fp32, writes M*L Base64 (L, n of this rank's slice)."""
        L = self.F.b64_len(self.n_local)
        upd = self.M * L + L + 4 * self.n_local
        enc = self.M * (4 * self.n_local + L)
        return upd, enc


def graph_of(torch, fn, reps: int):
    """HIP graph (torch.cuda.CUDAGraph) of `reps` back-to-back calls of fn."""
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    return g


def kernel_ms(torch, fn, reps: int = 10, rounds: int = 3) -> float:
    """Average device time of one launch of fn: HIP events around the replay
    of a graph of `reps` back-to-back launches (on the launch stream), so host
    launch gaps are not counted. Agrees with rocprofv3's kernel trace."""
    g = graph_of(torch, fn, reps)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(rounds):
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best.append(a.elapsed_time(b) / reps)
    del g
    return float(np.mean(best))


def steps_per_graph(steps: int, cap: int = 10) -> int:
    return max(d for d in range(1, min(cap, steps) + 1) if steps % d == 0)


def run_timed(torch, dist, world, body, count):
    """barrier + synchronize on both sides; the clock stops when this rank's
    steps are done (before the closing barrier, whose latency is not step
    time); returns the MAX over ranks."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(count):
        body()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = t1 - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def all_gather_fn(torch, dist, world, src, out):
    def f():
        if world > 1:
            if dist.get_backend() == "gloo":  # CPU-collective rehearsal (FLEET_BENCH_BACKEND=gloo)
                dist.all_gather(list(out.chunk(world)), src)
            else:
                dist.all_gather_into_tensor(out, src)
    return f


def time_pipelined(torch, dist, codec, sh, steps, warmup, world):
    """The same steps software-pipelined over two upload buffers: step i
    aggregates batch i (buffer i % 2) and encodes batch i+1 into the other buffer
    in one launch (fleet_update_encode_device; k_update_encode = the stream
    update's blocks + the client encode's blocks). Per step: one aggregation and
    one client encode, as in the sequential step; batch 0 is encoded before the
    clock starts. Graph-replayed like the sequential step (an even number of
    steps per graph, so every replay starts on buffer 0)."""
    import fleet_amd as F
    if not sh.n_local or sh.strong:
        return None
    bufs = [sh.text, torch.zeros_like(sh.text)]
    state = {"i": 0}

    def step():
        a, b = bufs[state["i"] % 2], bufs[(state["i"] + 1) % 2]
        state["i"] += 1
        codec.update_encode_device(a, sh.L, sh.dampen, sh.hpos_global, sh.merged, sh.merged_f32, sh.values, b)

    sh.encode()
    for _ in range(max(2, warmup)):
        step()
    torch.cuda.synchronize()
    codec.check()
    # an even number of steps per graph (every replay starts on buffer 0); an odd
    # step count ends with a one-step graph (buffer 0 -> 1)
    E = steps - steps % 2
    G = max(d for d in range(2, min(10, E) + 1, 2) if E % d == 0) if E else 0
    state["i"] = 0
    g = graph_of(torch, step, G) if G else None
    state["i"] = 0
    g1 = graph_of(torch, step, 1) if steps % 2 else None
    if g:
        g.replay()
    if g1:
        g1.replay()
    seq = ([g.replay] * (E // G) if G else []) + ([g1.replay] if g1 else [])
    it = iter(seq)
    elapsed = run_timed(torch, dist, world, lambda: next(it)(), len(seq))
    codec.check()
    del g, g1
    fused_ms = kernel_ms(torch, lambda: (step(), step()), reps=5) / 2  # a buffer-0/1 pair per graph entry
    codec.check()
    del bufs[1]
    return {"ms_per_step": elapsed / steps * 1e3,
            "gib_s": world * sh.M * sh.n_local * 4 / (elapsed / steps) / 2**30,
            "steps_per_graph": G, "kernel": F.update_encode_kernel(sh.L), "kernel_ms": fused_ms}


def strong_pipelined(torch, dist, codec, name, steps, warmup, rank, world):
    """`value`: strong scaling of ONE fixed problem. The rank's column window of
    every upload is a bucket of its own (n_local values, the header slots that
    fall inside it): the pipelined step (fleet_update_encode_device on the window,
    the same launch as the N=1 headline step) writes the rank's merged slice
    straight into the padded all_gather source; the all_gather of every rank's
    slice (RCCL) runs inside the timed step. Graph replays of the local
    launch (one graph per buffer parity), the gather eager after each, issued
    asynchronously: step i's all_gather (RCCL's own stream) overlaps step i+1's
    launch, the slice buffers double-buffered by step parity, and the step that
    reuses a slice buffer first waits for the gather that read it (every gather
    completes inside the timed region; FLEET_BENCH_GATHER_OVERLAP=0 runs them in
    line)."""
    import fleet_amd as F
    from fleet_amd.layouts import LAYOUTS
    lay_name, M, note = WORKLOADS[name]
    layout = LAYOUTS[lay_name]
    sh = Shard(codec, torch, layout, M, rank, world, strong=True)
    G = (layout.n_up + 2) // 3
    wmax = max(b - a for a, b in (group_range(G, world, r) for r in range(world)))
    dev = sh.merged.device
    srcs = [torch.zeros(16 * wmax, dtype=torch.uint8, device=dev) for _ in range(2)]
    outs = [torch.empty(world * 16 * wmax, dtype=torch.uint8, device=dev) for _ in range(2)]
    overlap = world > 1 and os.environ.get("FLEET_BENCH_GATHER_OVERLAP", "1") != "0"
    v0 = 3 * sh.gb
    hloc = sh.hpos_global[(sh.hpos_global >= v0) & (sh.hpos_global < v0 + sh.n_local)] - v0
    L_loc = F.b64_len(sh.n_local)
    bufs = [sh.text, torch.zeros_like(sh.text)]
    nb = 16 * sh.groups

    def local(i):  # the rank's merged slice written straight into the all_gather source of its parity
        codec.update_encode_device(bufs[i % 2], L_loc, sh.dampen, hloc, srcs[i % 2], sh.merged_f32, sh.values,
                                   bufs[(i + 1) % 2])

    def gather(k, async_op=False):
        if world == 1:
            return None
        if dist.get_backend() == "gloo":  # CPU-collective rehearsal (FLEET_BENCH_BACKEND=gloo)
            return dist.all_gather(list(outs[k].chunk(world)), srcs[k], async_op=async_op)
        return dist.all_gather_into_tensor(outs[k], srcs[k], async_op=async_op)

    sh.encode()
    for i in range(max(2, warmup)):
        local(i)
        gather(i % 2)
    torch.cuda.synchronize()
    codec.check()
    graphs = [graph_of(torch, lambda: local(0), 1), graph_of(torch, lambda: local(1), 1)]
    graphs[0].replay()
    graphs[1].replay()
    state = {"i": 0}
    works = [None, None]

    def step():
        i = state["i"]
        k = i % 2
        state["i"] += 1
        if not overlap:
            graphs[k].replay()
            gather(k)
            return
        if works[k] is not None:  # the gather of step i-2 read srcs[k]: the stream waits for it
            works[k].wait()
        graphs[k].replay()
        works[k] = gather(k, async_op=True)
        if i == steps - 1:  # the last step: both outstanding gathers complete inside the timed region
            for j in (0, 1):
                if works[j] is not None:
                    works[j].wait()
                    works[j] = None

    elapsed = run_timed(torch, dist, world, step, steps)
    codec.check()
    kl = (steps - 1) % 2
    if world > 1 and not torch.equal(outs[kl][rank * 16 * wmax: rank * 16 * wmax + nb], srcs[kl][:nb]):
        raise RuntimeError("all_gather returned a different merged slice")
    # rank 0's merged text of the whole problem: every rank's slice, trimmed to its width
    gathered = None
    if rank == 0:
        parts = []
        for r in range(world):
            a, b = group_range(G, world, r)
            base = r * 16 * wmax if world > 1 else 0
            parts.append((outs[kl] if world > 1 else srcs[kl])[base: base + 16 * (b - a)])
        gathered = torch.cat(parts).cpu().numpy()
    kern_ms = kernel_ms(torch, lambda: (local(0), local(1)), reps=5) / 2
    res = {"workload": name, "note": note, "clients": M, "n_up_total": layout.n_up, "n_up_per_rank": sh.n_local,
           "groups_per_rank_max": wmax, "ms_per_step": elapsed / steps * 1e3,
           "gib_s": M * layout.n_up * 4 / (elapsed / steps) / 2**30,
           "kernel": F.update_encode_kernel(L_loc), "kernel_ms_rank0": kern_ms,
           # what the step costs beyond rank 0's launch: the all_gather's exposed part plus
           # the step's launch gaps and any rank imbalance (the clock is the max over ranks)
           "exposed_ms": elapsed / steps * 1e3 - kern_ms,
           "step": "pipelined launch on the rank's column window + all_gather of the merged slices (inside; "
                   + ("issued async, overlapping the next step's launch)" if overlap else "in line)")}
    del graphs, bufs, sh, srcs, outs
    torch.cuda.empty_cache()
    res["gathered"] = gathered  # popped by main (rank 0: the parity check)
    return res


def full_width_merged(torch, codec, name):
    """The fixed problem of `name` aggregated at full width on ONE GPU -- the N = 1
    problem (the same synthetic uploads, one fleet_update_device over every group):
    its merged Base64 bytes [16 * groups], the reference the N-rank text is held to."""
    from fleet_amd.layouts import LAYOUTS
    lay_name, M, _ = WORKLOADS[name]
    sh = Shard(codec, torch, LAYOUTS[lay_name], M, 0, 1)
    sh.encode()
    sh.aggregate()
    torch.cuda.synchronize()
    codec.check()
    out = sh.merged.cpu().numpy().copy()
    del sh
    torch.cuda.empty_cache()
    return out


def approx_client_sharded(torch, dist, codec, name, steps, warmup, rank, world, exact):
    """SURVEY.md §8e's opt-in approximate mode timed on the same problem: rank r holds
    the full-width uploads of its block of clients (group_range over clients), runs the
    exact chain on them (fleet_update_device, averaged by its own M_r), one float64
    all_reduce (RCCL) sums the weighted partials, and every rank encodes the sum
    (fleet_amd.shard.ClientShardedUpdater.device_step). Rank 0 reports deviation() of
    its text from the exact text (`exact`: the full-width merged bytes); at N = 1 the
    mode is the exact chain itself."""
    import fleet_amd as F
    from fleet_amd.layouts import LAYOUTS
    from fleet_amd.shard import ClientShardedUpdater, deviation
    lay_name, M, _ = WORKLOADS[name]
    layout = LAYOUTS[lay_name]
    cb, ce = group_range(M, world, rank)
    Mr = ce - cb
    n = layout.n_up
    groups = (n + 2) // 3
    L = F.b64_len(n)
    hpos = np.asarray(layout.header_positions(), dtype=np.int32)
    hval = np.asarray(layout.header_values(), dtype=np.float32)
    dev = torch.device("cuda", torch.cuda.current_device())
    values = torch.empty((Mr, 3 * groups), dtype=torch.float32, device=dev)
    text = torch.zeros((Mr, 16 * groups), dtype=torch.uint8, device=dev)
    codec.synth_device(1, values, n, hpos, hval, client0=cb)
    codec.encode_device(values, n, text)
    del values
    merged = torch.zeros(16 * groups, dtype=torch.uint8, device=dev)
    f32 = torch.zeros(3 * groups, dtype=torch.float32, device=dev)
    out = torch.zeros(16 * groups, dtype=torch.uint8, device=dev)
    vals = torch.zeros((1, 3 * groups), dtype=torch.float32, device=dev)
    cs = ClientShardedUpdater(codec, approx=True)
    d = dampen_policy(M)[cb:ce]

    def step():
        cs.device_step(text, L, d, hpos, M, cb, merged, f32, out, vals)

    for _ in range(max(1, warmup)):
        step()
    torch.cuda.synchronize()
    codec.check()
    el = run_timed(torch, dist, world, step, steps) / steps
    codec.check()
    res = {"workload": name, "clients": M, "clients_per_rank": [e - b for b, e in
                                                                 (group_range(M, world, r) for r in range(world))],
           "ms_per_step": el * 1e3, "gib_s": M * n * 4 / el / 2**30,
           "step": "rank's block of clients through the exact chain (full width) + float64 all_reduce of the "
                   "weighted partial averages + encode of the sum; NOT the reference's bytes"}
    if rank == 0 and exact is not None:
        got = out.cpu().numpy()[:L].tobytes()
        want = bytes(exact[:L])
        res["deviation"] = deviation(codec.decode_floats(got), codec.decode_floats(want))
        res["equals_exact_bytes"] = got == want
    del text, merged, f32, out, vals
    torch.cuda.empty_cache()
    return res


def time_workload(torch, dist, codec, name, steps, warmup, rank, world, graph=True, pipelined_step=True):
    """Weak-scaling measurement of `name`: times `steps` steps. graph=True: a
    step (encode + aggregation) is captured once into a HIP graph of G steps
    and replayed steps/G times; graph=False: eager launches. N>1: the
    all_gather of the merged slices is timed after the steps, on its own
    (exchange_ms)."""
    import fleet_amd as F
    from fleet_amd.layouts import LAYOUTS
    lay_name, M, note = WORKLOADS[name]
    layout = LAYOUTS[lay_name]
    sh = Shard(codec, torch, layout, M, rank, world)
    gathered = torch.empty((world * sh.pitch,), dtype=torch.uint8, device=sh.merged.device) if world > 1 else None

    def local():
        sh.encode()
        sh.aggregate()

    for _ in range(warmup):
        local()
    torch.cuda.synchronize()
    codec.check()

    eager_elapsed = run_timed(torch, dist, world, local, steps)
    codec.check()
    eager_ms = eager_elapsed / steps * 1e3

    # per-kernel device time (roofline): graph of 10 back-to-back launches each
    enc_ms = kernel_ms(torch, sh.encode)
    upd_ms = kernel_ms(torch, sh.aggregate)
    codec.check()

    elapsed = eager_elapsed
    G = 1
    if graph:
        G = steps_per_graph(steps)
        g = graph_of(torch, local, G)
        for _ in range(max(1, warmup // G)):
            g.replay()
        elapsed = run_timed(torch, dist, world, g.replay, steps // G)
        codec.check()
        del g
    pipelined = time_pipelined(torch, dist, codec, sh, steps, warmup, world) if (graph and pipelined_step) else None
    exchange_ms = None
    if world > 1:
        exchange = all_gather_fn(torch, dist, world, sh.merged, gathered)
        exchange()
        exchange_ms = run_timed(torch, dist, world, exchange, 5) / 5 * 1e3
        if not torch.equal(gathered[rank * sh.pitch:(rank + 1) * sh.pitch], sh.merged):
            raise RuntimeError("all_gather returned a different merged slice")
    ms = elapsed / steps * 1e3
    total_bytes_fp32 = world * M * sh.n_local * 4
    gib_s = total_bytes_fp32 / (elapsed / steps) / 2**30
    upd_b, enc_b = sh.algorithmic_bytes()
    res = {
        "workload": name, "note": note, "layout": lay_name, "clients": M, "n_up_per_rank": sh.n_local,
        "ms_per_step": ms, "gib_s": gib_s, "update_kernel_ms": upd_ms, "encode_kernel_ms": enc_ms,
        "graph": graph, "steps": steps, "steps_per_graph": G, "eager_ms_per_step": eager_ms, "exchange_ms": exchange_ms,
        "update_kernel": F.update_kernel(sh.L),
        "update_bytes": upd_b, "encode_bytes": enc_b,
        "update_gbs": upd_b / (upd_ms * 1e-3) / 1e9, "encode_gbs": enc_b / (enc_ms * 1e-3) / 1e9,
        "element_clients_per_s": world * M * sh.n_local / (elapsed / steps),
        "pipelined": pipelined,
    }
    del sh
    torch.cuda.empty_cache()
    return res


def strong_device(torch, dist, codec, name, steps, warmup, rank, world):
    """Strong scaling of ONE fixed problem split over the ranks (device-resident):
    step = encode + aggregation of this rank's window; timed once with the
    all_gather of the merged slices inside every step and once without it."""
    from fleet_amd.layouts import LAYOUTS
    lay_name, M, note = WORKLOADS[name]
    layout = LAYOUTS[lay_name]
    sh = Shard(codec, torch, layout, M, rank, world, strong=True)
    # every rank's slice padded to the largest window (one RCCL call)
    G = (layout.n_up + 2) // 3
    wmax = max(b - a for a, b in (group_range(G, world, r) for r in range(world)))
    src = torch.zeros(16 * wmax, dtype=torch.uint8, device=sh.merged.device)
    out = torch.empty(world * 16 * wmax, dtype=torch.uint8, device=sh.merged.device)
    gather = all_gather_fn(torch, dist, world, src, out)

    def local():
        sh.encode()
        sh.aggregate()

    def with_gather():
        local()
        src[: 16 * sh.groups].copy_(sh.merged[: 16 * sh.groups])
        gather()

    for _ in range(warmup):
        with_gather()
    torch.cuda.synchronize()
    codec.check()
    inside = run_timed(torch, dist, world, with_gather, steps) / steps
    outside = run_timed(torch, dist, world, local, steps) / steps
    codec.check()
    if world > 1 and not torch.equal(out[rank * 16 * wmax: rank * 16 * wmax + 16 * sh.groups],
                                     sh.merged[: 16 * sh.groups]):
        raise RuntimeError("all_gather returned a different merged slice")
    gathered = None
    if rank == 0 and world > 1:
        gathered = torch.cat([out[r * 16 * wmax: r * 16 * wmax + 16 * (b - a)]
                              for r, (a, b) in enumerate(group_range(G, world, q) for q in range(world))]).cpu().numpy()
    fp32 = M * layout.n_up * 4
    res = {"workload": name, "note": note, "clients": M, "n_up_total": layout.n_up,
           "groups_per_rank_max": wmax,
           "gather_inside": {"ms_per_step": inside * 1e3, "gib_s": fp32 / inside / 2**30},
           "gather_outside": {"ms_per_step": outside * 1e3, "gib_s": fp32 / outside / 2**30}}
    del sh, src, out
    torch.cuda.empty_cache()
    if gathered is not None:  # rank 0: the N windows' text against the 1-GPU full-width text
        res["parity"] = bool(np.array_equal(gathered, full_width_merged(torch, codec, name)))
    if world > 1:
        dist.barrier()
    return res


def strong_host(torch, dist, codec, name, steps, rank, world):
    """Strong scaling of ONE fixed problem with host buffers: every step H2Ds this
    rank's column window of the M uploads from pinned host memory, aggregates it,
    D2Hs its merged slice into pinned host memory and (N>1) all-gathers the slices
    -- the PCIe- and gather-inclusive rate of the sharded path."""
    import fleet_amd as F
    from fleet_amd.layouts import LAYOUTS
    lay_name, M, note = WORKLOADS[name]
    layout = LAYOUTS[lay_name]
    sh = Shard(codec, torch, layout, M, rank, world, strong=True)
    sh.encode()
    torch.cuda.synchronize()
    host_up = torch.empty(sh.text.shape, dtype=torch.uint8).pin_memory()
    host_up.copy_(sh.text)
    host_out = torch.empty(sh.merged.shape, dtype=torch.uint8).pin_memory()
    G = (layout.n_up + 2) // 3
    wmax = max(b - a for a, b in (group_range(G, world, r) for r in range(world)))
    src = torch.zeros(16 * wmax, dtype=torch.uint8, device=sh.merged.device)
    out = torch.empty(world * 16 * wmax, dtype=torch.uint8, device=sh.merged.device)
    gather = all_gather_fn(torch, dist, world, src, out)

    def step():
        sh.text.copy_(host_up, non_blocking=True)
        sh.aggregate()
        host_out.copy_(sh.merged, non_blocking=True)
        src[: 16 * sh.groups].copy_(sh.merged[: 16 * sh.groups])
        gather()

    step()
    torch.cuda.synchronize()
    codec.check()
    el = run_timed(torch, dist, world, step, steps) / steps
    codec.check()
    res = {"workload": name, "note": note, "clients": M, "n_up_total": layout.n_up,
           "h2d_bytes_per_rank": M * sh.pitch, "ms_per_step": el * 1e3,
           "gib_s": M * layout.n_up * 4 / el / 2**30,
           "what": "pinned-host H2D of the rank's column window + aggregation + D2H of its merged slice + all_gather"}
    del sh, host_up, host_out, src, out
    torch.cuda.empty_cache()
    return res


def newest_profile(name: str):
    """profiles/rNN/<name>, newest round first."""
    return sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name)), reverse=True)


def kernel_key(kern: dict, kernel: str):
    """The entry of `kernel` in a profile summary: the exact rocprofv3 name, else the
    same kernel with default template arguments spelled differently (k_update_mixed<256> /
    k_update_mixed<256, false>; k_update_tiled_encode<64> /
    k_update_tiled_encode<64, 0>)."""
    if kernel in kern:
        return kernel
    def canon(n):
        return re.sub(r"(,false)?(,0)?(,256)?>$", ">", re.sub(r"\s+", "", n))
    for k in kern:
        if canon(k) == canon(kernel):
            return k
    return None


def sq_valu(workload: str, kernel: str):
    """VALU lane-instructions per (client, value) of the profiled kernel from the
    newest committed SQ_INSTS_VALU pass (profiles/rNN/sq.json), None when absent."""
    for path in newest_profile("sq.json"):
        try:
            with open(path) as f:
                kern = json.load(f)["workloads"][workload]
            v = kern[kernel_key(kern, kernel)]["valu_lane_instr_per_element_client"]
            return float(v), os.path.relpath(path, ROOT)
        except (OSError, KeyError, ValueError):
            continue
    return None


def pmc_traffic(workload: str, kernel: str = ""):
    """HBM bytes per k_update launch for `workload` from the newest committed
    rocprofv3 PMC summary (profiles/rNN/traffic.json, written by
    scripts/pmc_summary.py from separate --pmc FETCH_SIZE / WRITE_SIZE passes,
    FETCH_SIZE doubled per the gfx950 correction). None when absent."""
    for path in newest_profile("traffic.json"):
        try:
            with open(path) as f:
                kern = json.load(f)["workloads"].get(workload, {})
        except (OSError, ValueError, KeyError):
            continue
        # only a profile of the same kernel variant counts
        k = kernel_key(kern, kernel)
        if k and "hbm_bytes" in kern[k]:
            return kern[k]["hbm_bytes"], k, os.path.relpath(path, ROOT)
    return None


def end_to_end(torch, codec, name, reps=None):
    """Host-buffer path (fleet_update: host header walk, pinned staging, H2D of the
    M uploads, update, D2H of the merged Base64 + error check) on the same
    synthetic uploads: the PCIe-inclusive rate the JNI shim sees. Not `value`.
    Beside it, the H2D floor: one pinned-host -> HBM copy of the same bytes."""
    import fleet_amd as F
    from fleet_amd.layouts import LAYOUTS
    lay_name, M, _ = WORKLOADS[name]
    layout = LAYOUTS[lay_name]
    sh = Shard(codec, torch, layout, M, 0, 1)
    sh.encode()
    torch.cuda.synchronize()
    host = sh.text.cpu().numpy()
    L = sh.L
    if reps is None:  # small batches: more repetitions (sub-ms calls, the min of 3 is noisy)
        reps = 3 if M * L >= 64 << 20 else 20
    ups = [host[c, :L].tobytes() for c in range(M)]
    del host
    # H2D floor: the same bytes in one pinned buffer, one copy on torch's stream
    pin = torch.empty(M * L, dtype=torch.uint8).pin_memory()
    dst = sh.text.view(-1)[: M * L]
    dst.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h2d = []
    for _ in range(3):
        a.record()
        dst.copy_(pin, non_blocking=True)
        b.record()
        b.synchronize()
        h2d.append(a.elapsed_time(b) * 1e-3)
    h2d_s = min(h2d)
    del sh, pin, dst
    torch.cuda.empty_cache()
    d = dampen_policy(M)
    codec.update(ups, d)  # warm (allocations, staging)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        merged = codec.update(ups, d)
        times.append(time.perf_counter() - t0)
    dt = min(times)
    # copy-free ingress: the uploads deserialised into one page-locked buffer (a
    # registered direct ByteBuffer on the Java side), DMAed straight to HBM
    rows = np.empty((M, L), np.uint8)
    for c in range(M):
        rows[c] = np.frombuffer(ups[c], np.uint8)
    codec.register_host(rows)
    try:
        if codec.update_rows(rows, L, d) != merged:
            raise RuntimeError("fleet_update_rows differs from fleet_update")
        pt = []
        for _ in range(reps):
            t0 = time.perf_counter()
            codec.update_rows(rows, L, d)
            pt.append(time.perf_counter() - t0)
    finally:
        codec.unregister_host(rows)
    del rows
    pinned = {"ms": min(pt) * 1e3, "gib_s": M * layout.n_up * 4 / min(pt) / 2**30,
              "pcie_gbs_achieved": M * L / min(pt) / 1e9, "x_floor": min(pt) / h2d_s,
              "what": "fleet_update_rows on registered (page-locked) rows: no host copy"}
    multi = None
    ndev = torch.cuda.device_count()
    if ndev > 1:  # one process driving every visible GPU (fleet_update_multi): column windows per device
        codecs = [codec] + [F.Codec(k) for k in range(1, ndev)]
        F.update_multi(codecs, ups, d)
        mt = []
        for _ in range(reps):
            t0 = time.perf_counter()
            if F.update_multi(codecs, ups, d) != merged:
                raise RuntimeError("fleet_update_multi differs from fleet_update")
            mt.append(time.perf_counter() - t0)
        multi = {"devices": ndev, "ms": min(mt) * 1e3, "gib_s": M * layout.n_up * 4 / min(mt) / 2**30,
                 "pcie_gbs_achieved": M * L / min(mt) / 1e9}
        for cd in codecs[1:]:
            cd.close()
    return {"workload": name, "ms": dt * 1e3, "ms_mean": float(np.mean(times)) * 1e3, "pinned_rows": pinned,
            "multi_gpu": multi,
            "gib_s": M * layout.n_up * 4 / dt / 2**30,
            "h2d_bytes": M * L, "d2h_bytes": len(merged),
            "h2d_floor_ms": h2d_s * 1e3, "h2d_floor_gbs": M * L / h2d_s / 1e9,
            "pcie_gbs_achieved": M * L / dt / 1e9, "x_floor": dt / h2d_s}


def cpu_threads():
    threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(threads, int(os.environ.get("OMP_NUM_THREADS", threads))))


def cpu_baseline(workload: str, budget_s: float = 20.0, faithful_clients: int = 4):
    """The reference C++ path's CPU cost on the GPU box's host, for the headline
    workload (kind "port": the C restatement oracle/fleet_oracle.c; the
    reference's own codec and JNI backend (Base64.cpp, cppNN_backend.cpp)
    include <jni.h>, which the image lacks, so there is no reference build to
    time).

    value: the restatement's fused chain with OpenMP on every core this process
           may use, over the FULL workload: client encode (threads over clients)
           + CppNNUpdater.update's aggregation chain.
    also:  the faithful per-op string chain (one JNI op at a time, re-encoding
           between ops, single thread like the synchronized update()) at -O2
           and at -O0 (the reference's own flags, Server/Makefile:2), on the
           first `faithful_clients` clients of the same workload."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from fleet_amd.layouts import LAYOUTS
    lay_name, M, _ = WORKLOADS[workload]
    lay = LAYOUTS[lay_name]
    w, b = list(lay.w_sizes), list(lay.b_sizes)
    o2 = pyoracle.Oracle()
    threads = cpu_threads()
    with ThreadPoolExecutor(threads) as ex:  # ctypes releases the GIL
        floats = list(ex.map(lambda c: o2.synth_upload(1, c, w, b), range(M)))
    hm = o2.header_mask(w, b)
    d = dampen_policy(M)
    fp32 = M * lay.n_up * 4

    reps, t_total = 0, 0.0
    while reps < 3 and t_total < budget_s / 2:
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            ups = list(ex.map(o2.encode_floats, floats))
        o2.update_fused(ups, d, hm, threads=threads)
        t_total += time.perf_counter() - t0
        reps += 1
    per = t_total / reps
    value = fp32 / per / 2**30
    del ups

    also = {}
    Mf = min(faithful_clients, M)
    for tag, path in (("faithful_O2_1core", pyoracle.ORACLE_SO), ("faithful_O0_1core", pyoracle.ORACLE_O0_SO)):
        o = pyoracle.Oracle(path)
        n, t = 0, 0.0
        while n < 3 and t < budget_s / 4:
            t0 = time.perf_counter()
            sub = [o.encode_floats(v) for v in floats[:Mf]]
            o.update_faithful(sub, d[:Mf])
            t += time.perf_counter() - t0
            n += 1
        also[tag] = {"value": Mf * lay.n_up * 4 / (t / n) / 2**30, "unit": "GiB/s", "cores": 1,
                     "s_per_update": t / n, "clients": Mf,
                     "mfloat_per_s": Mf * lay.n_up / (t / n) / 1e6}
    import platform
    cpu = platform.processor() or "x86_64"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": value, "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{workload} in full ({M} clients x {lay.n_up} floats): client encode (threads over clients) + "
                      f"CppNNUpdater.update chain (fused restatement, OpenMP), {reps} rep(s), {per:.2f} s/rep; "
                      f"no reference build (Base64.cpp needs <jni.h>)",
            "cpu_model": cpu, "host_nproc": os.cpu_count(), "also": also}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="synth1m_256", choices=sorted(WORKLOADS))
    ap.add_argument("--extras", default="synth4m_4096,cifar10_256,cifar100_1024,mnist64",
                    help="comma list of extra workloads measured in the same run (N=1 only); '' for none")
    ap.add_argument("--strong", action="store_true",
                    help="value = strong scaling of configs[4] (one fixed problem split over the ranks, "
                         "all_gather of the merged slices inside every step)")
    ap.add_argument("--sequential", action="store_true",
                    help="value = the sequential step (encode, then aggregate) instead of the pipelined one")
    ap.add_argument("--no-strong-block", action="store_true", help="skip the strong-scaling block")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", type=int, default=1,
                    help="1 (default): replay steps from a captured HIP graph; 0: eager launches")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) measurement")
    ap.add_argument("--e2e", default="synth1m_256,cifar10_256,mnist64",
                    help="workloads of the host-buffer (PCIe-inclusive) measurement (N=1)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: start the N ranks as a child torch.distributed.run (this process has
        # touched no GPU) and exit with its status
        import socket
        import subprocess
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
        sys.exit(subprocess.call(cmd))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} (one rank per GPU)")

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N>1 path on a one-GPU box: every rank on device 0, gloo collectives
    # (FLEET_BENCH_SAME_DEVICE=1 FLEET_BENCH_BACKEND=gloo); the driver's runs use one GPU per rank over RCCL
    if os.environ.get("FLEET_BENCH_SAME_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("FLEET_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    import fleet_amd as F
    codec = F.Codec(local)

    main_res = time_workload(torch, dist, codec, args.workload, args.steps, args.warmup, rank, world, args.graph)
    strong_value = None
    exact = None  # rank 0: the N = 1 problem's merged bytes (full width, one GPU)
    if world > 1 and args.graph:
        strong_value = strong_pipelined(torch, dist, codec, args.workload, args.steps, args.warmup, rank, world)
        gathered = strong_value.pop("gathered")
        if rank == 0:
            exact = full_width_merged(torch, codec, args.workload)
            strong_value["parity"] = bool(gathered is not None and np.array_equal(gathered, exact))
            strong_value["parity_check"] = ("rank 0's gathered merged text (every rank's slice) == the full-width "
                                            "1-GPU update of the same problem, byte for byte")
            if not strong_value["parity"]:
                print("bench.py: the N-rank merged text differs from the 1-GPU text of the same problem",
                      file=sys.stderr)
    elif rank == 0:
        exact = full_width_merged(torch, codec, args.workload)
    approx = approx_client_sharded(torch, dist, codec, args.workload, max(3, args.steps // 4), 1, rank, world, exact)
    # the host-buffer paths before the extras: after the 150 GiB synth4m_4096 extra the
    # process's small pinned-host copies run 2-3x slower (measured on MNIST-64: 0.81 vs
    # 0.30 ms), an allocator-state effect that is not the path's
    e2e = None
    if world == 1 and not args.no_e2e:
        e2e = {w: end_to_end(torch, codec, w) for w in args.e2e.split(",") if w}

    extras = {}
    if world == 1 and args.extras:
        for w in [x for x in args.extras.split(",") if x and x != args.workload]:
            # a few steps of the large extras; the small ones get enough steps that the
            # timed region is not one or two graph launches (mnist64's 17 us step: 4 steps
            # timed 22 us per step, 200 steps 17 us)
            n = max(4, args.steps // 8 * 2, EXTRA_MIN_STEPS.get(w, 0))
            extras[w] = time_workload(torch, dist, codec, w, n, 2, rank, world, args.graph)

    strong = None
    if args.strong or not args.no_strong_block:
        ssteps = max(3, args.steps // 4)
        strong = {"scaling": "strong", "n_gpus": world,
                  "device": strong_device(torch, dist, codec, "synth4m_4096", ssteps, 1, rank, world),
                  "host_staged": strong_host(torch, dist, codec, "cifar100_1024", ssteps, rank, world)}

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(args.workload, args.cpu_budget)
    r = main_res
    upd_roof = {"kernel": r["update_kernel"], "achieved": r["update_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": r["update_gbs"] / HBM_PEAK_GBS, "frac_of_copy_ceiling": r["update_gbs"] / HBM_COPY_GBS,
                "limiter": LIMITER.get(r["update_kernel"].split("<")[0], "VALU issue"),
                "bytes_per_launch": r["update_bytes"], "kernel_ms": r["update_kernel_ms"]}
    traffic = pmc_traffic(args.workload, r["update_kernel"]) if world == 1 else None
    sq = sq_valu(args.workload, r["update_kernel"])
    upd_roof.update({"valu_lane_instr_per_element_client": sq[0] if sq else None, "valu_source": sq[1] if sq else None,
                     "traffic": traffic[0] if traffic else None,
                     "traffic_source": f"{traffic[2]} ({traffic[1]})" if traffic else None})
    pipe = r.get("pipelined") if isinstance(r.get("pipelined"), dict) and "gib_s" in r["pipelined"] else None
    value, ms, scaling = r["gib_s"], r["ms_per_step"], "weak"
    step_form = "sequential: k_encode_f32 then the aggregation kernel, per step"
    roofline = dict(upd_roof, bound="hbm", workload=args.workload)
    if pipe and not args.sequential:
        value, ms = pipe["gib_s"], pipe["ms_per_step"]
        step_form = ("pipelined: step i aggregates batch i and encodes batch i+1 into the other upload buffer, "
                     f"one {pipe['kernel']} launch (fleet_update_encode_device); batch 0 encoded before the clock")
        if pipe["kernel"].startswith("k_update_encode"):
            fb = r["update_bytes"] + r["encode_bytes"]
            fgbs = fb / (pipe["kernel_ms"] * 1e-3) / 1e9
            ftr = pmc_traffic(args.workload, pipe["kernel"]) if world == 1 else None
            fsq = sq_valu(args.workload, pipe["kernel"])
            roofline = {"bound": "hbm", "kernel": pipe["kernel"], "achieved": fgbs, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": fgbs / HBM_PEAK_GBS, "frac_of_copy_ceiling": fgbs / HBM_COPY_GBS,
                        "limiter": "VALU issue (the aggregation's exact chain; the encode fills HBM time)",
                        "bytes_per_launch": fb, "bytes_update": r["update_bytes"], "bytes_encode": r["encode_bytes"],
                        "kernel_ms": pipe["kernel_ms"],
                        "valu_lane_instr_per_element_client": fsq[0] if fsq else None,
                        "valu_source": fsq[1] if fsq else None,
                        "traffic": ftr[0] if ftr else None,
                        "traffic_source": f"{ftr[2]} ({ftr[1]})" if ftr else None,
                        "workload": args.workload, "aggregation_alone": upd_roof}
    config = {"workload": args.workload, "layout": r["layout"], "clients": r["clients"],
              "n_up_per_rank": r["n_up_per_rank"], "parallelism": f"element-shard x{world}",
              "dampening": "policy 1 inverse, tau = c mod 3", "step": step_form}
    weak = None
    if strong_value is not None:  # N>1: value = the fixed headline problem split over the ranks
        weak = {"gib_s": value, "ms_per_step": ms, "step": step_form,
                "what": "every rank a full-size slice of a model N times larger; no collective in the timed steps"}
        value, ms, scaling = strong_value["gib_s"], strong_value["ms_per_step"], "strong"
        config = {"workload": args.workload, "layout": r["layout"], "clients": r["clients"],
                  "n_up_total": strong_value["n_up_total"], "n_up_per_rank": strong_value["n_up_per_rank"],
                  "parallelism": f"element-shard x{world}, all_gather of the merged slices inside the step",
                  "dampening": "policy 1 inverse, tau = c mod 3", "step": strong_value["step"]}
    elif world == 1:
        scaling = "strong"  # the N=1 point of the strong curve: the same fixed problem on one GPU
    if args.strong:
        sd = strong["device"]
        value, ms, scaling = sd["gather_inside"]["gib_s"], sd["gather_inside"]["ms_per_step"], "strong"
        config = {"workload": "synth4m_4096", "layout": "synth4m", "clients": sd["clients"],
                  "n_up_total": sd["n_up_total"], "parallelism": f"element-shard x{world}, all_gather inside",
                  "dampening": "policy 1 inverse, tau = c mod 3"}
    line = {
        "metric": "gradient GiB/s encode+decode+aggregate (device-resident); % HBM roofline",
        "value": value,
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Philox4x32-10 value mix, SURVEY.md §8d), device-resident",
        "config": config,
        "roofline": roofline,
        "cpu_baseline": cpu,
        "timing": {"graph": bool(r["graph"]), "steps_per_graph": r["steps_per_graph"],
                   "eager_ms_per_step": r["eager_ms_per_step"],
                   "exchange_ms": r["exchange_ms"],
                   "exchange": "weak-scaling value: none in the timed steps (element shards stay resident); N>1: one "
                               "all_gather of the merged slices timed separately (exchange_ms, max over ranks) and "
                               "checked; the strong block times it inside the step",
                   "kernel_ms": "HIP events around graph replays of 10 back-to-back launches"},
        "kernels": {"k_update_ms": r["update_kernel_ms"], "k_encode_f32_ms": r["encode_kernel_ms"],
                    "k_encode_gbs": r["encode_gbs"], "element_clients_per_s": r["element_clients_per_s"]},
        "sequential": {"gib_s": r["gib_s"], "ms_per_step": r["ms_per_step"]},
        "pipelined": r["pipelined"],
        "strong": strong,
        "weak": weak,
        "strong_value": strong_value,
        "parity": None if strong_value is None else {"n_rank_equals_1_gpu": strong_value["parity"],
                                                     "check": strong_value["parity_check"]},
        "approx": approx,
        "extra": extras,
        # the extras in the headline's own form (the pipelined step), beside their sequential step
        "extra_steps": {w: {"pipelined_ms": (x["pipelined"] or {}).get("ms_per_step"),
                            "pipelined_gib_s": (x["pipelined"] or {}).get("gib_s"),
                            "pipelined_kernel": (x["pipelined"] or {}).get("kernel"),
                            "sequential_ms": x["ms_per_step"], "sequential_gib_s": x["gib_s"],
                            "update_kernel": x["update_kernel"], "update_kernel_ms": x["update_kernel_ms"]}
                        for w, x in extras.items()},
        "end_to_end_host_buffers": e2e,
    }
    if cpu:
        line["vs_cpu_baseline"] = value / cpu["value"]
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
