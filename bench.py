#!/usr/bin/env python3
"""bench.py -- gradient GiB/s encode+decode+aggregate (device-resident) on MI355X.

One step = the hot path over one batch of M synthetic client gradient buckets
already resident in HBM:
  1. client-side encode  (Base64::encode(vector<float>) of every bucket; k_encode_f32)
  2. server aggregation  (CppNNUpdater.update's decode/dampen/sum/average/merge
                          chain, bit-exact; k_update) -> merged Base64 + fp32

Multi-GPU: element-range sharding, weak scaling -- every rank owns
a fixed slice of G 3-value groups of a model N times larger. No collective in the
data path: each rank's merged slice (its share of the model delta) stays
resident on its GPU, as the whole merged vector does at N=1; the all_gather of
the slices (fleet_amd.shard, for a caller that needs the full vector) is timed
separately and reported as `exchange_ms`, after the timed steps.

Output: ONE JSON line on rank 0 (see DESIGN.md §6 for every field).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# workload name -> (layout, clients M, BASELINE.json config index or note)
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
    "k_update_tiled": "VALU issue (exact chain, ~178 VALU instructions per client-value)",
    "k_update": "VALU issue (exact chain, ~172 VALU instructions per client-value)",
}


def dampen_policy(M: int):
    """policy 1 (inverse, CppNNUpdater.java:307-308) with tau = c mod 3."""
    return [1.0 / ((c % 3) + 1) for c in range(M)]


class Shard:
    """One rank's device-resident slice of a workload."""

    def __init__(self, codec, torch, layout, M, rank, world, seed=1):
        import fleet_amd as F
        self.F = F
        self.torch = torch
        self.codec = codec
        self.M = M
        n_up_rank = layout.n_up  # weak scaling: every rank owns one full-size bucket slice
        groups = (n_up_rank + 2) // 3
        self.groups = groups
        self.n_local = n_up_rank
        self.g0 = rank * groups  # global group offset of this slice
        # global layout = the per-rank layout replicated world times; headers of
        # this slice in local coordinates (the slice is one copy of the layout)
        self.hpos = np.asarray(layout.header_positions(), dtype=np.int32)
        self.hval = np.asarray(layout.header_values(), dtype=np.float32)
        self.L = F.b64_len(self.n_local)
        self.pitch = 16 * groups
        self.vpitch = 3 * groups
        dev = torch.device("cuda", torch.cuda.current_device())
        self.values = torch.empty((M, self.vpitch), dtype=torch.float32, device=dev)
        self.text = torch.empty((M, self.pitch), dtype=torch.uint8, device=dev)
        self.merged = torch.empty((self.pitch,), dtype=torch.uint8, device=dev)
        self.merged_f32 = torch.empty((self.vpitch,), dtype=torch.float32, device=dev)
        codec.synth_device(seed + rank * 1000003, self.values, self.n_local, self.hpos, self.hval)
        self.dampen = np.asarray(dampen_policy(M), dtype=np.float64)
        torch.cuda.synchronize()

    def encode(self):
        self.codec.encode_device(self.values, self.n_local, self.text)

    def aggregate(self):
        self.codec.update_device(self.text, self.L, self.dampen, self.hpos, self.merged, self.merged_f32)

    def algorithmic_bytes(self):
        """Per launch: k_update reads M*L Base64, writes L Base64 + 4*n fp32;
        k_encode_f32 reads 4*n*M fp32, writes M*L Base64."""
        upd = self.M * self.L + self.L + 4 * self.n_local
        enc = self.M * (4 * self.n_local + self.L)
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


def time_workload(torch, dist, codec, name, steps, warmup, rank, world, graph=True):
    """Times `steps` steps. graph=True: a step (encode + aggregation) is
    captured once into a HIP graph of G steps and replayed steps/G times;
    graph=False: eager launches (host launch gaps between the small kernels
    included). Both variants are reported. N>1: the all_gather of the merged
    slices is timed after the steps, on its own (exchange_ms)."""
    import fleet_amd as F
    from fleet_amd.layouts import LAYOUTS
    lay_name, M, note = WORKLOADS[name]
    layout = LAYOUTS[lay_name]
    sh = Shard(codec, torch, layout, M, rank, world)
    gathered = None
    if world > 1:
        gathered = torch.empty((world * sh.pitch,), dtype=torch.uint8, device=sh.merged.device)

    def local():
        sh.encode()
        sh.aggregate()

    def exchange():
        if world > 1:
            if dist.get_backend() == "gloo":  # CPU-collective rehearsal (FLEET_BENCH_BACKEND=gloo)
                dist.all_gather(list(gathered.chunk(world)), sh.merged)
            else:
                dist.all_gather_into_tensor(gathered, sh.merged)

    def run_timed(body, count):
        # barrier + synchronize on both sides; the clock stops when this rank's
        # steps are done (before the closing barrier, whose latency is not step
        # time) and the max over ranks is taken by the caller
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
        return t1 - t0

    for _ in range(warmup):
        local()
    torch.cuda.synchronize()
    codec.check()

    eager_elapsed = run_timed(local, steps)
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

        elapsed = run_timed(g.replay, steps // G)
        codec.check()
        del g
    exchange_ms = None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=sh.merged.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # the slices gathered once (RCCL all_gather over xGMI), timed on its own, and
        # checked: this rank's slice of the gathered vector is its merged output
        exchange()
        xt = run_timed(exchange, 5) / 5
        t = torch.tensor([xt], dtype=torch.float64, device=sh.merged.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        exchange_ms = float(t.item()) * 1e3
        if not torch.equal(gathered[rank * sh.pitch:(rank + 1) * sh.pitch], sh.merged):
            raise RuntimeError("all_gather returned a different merged slice")
    ms = elapsed / steps * 1e3
    total_bytes_fp32 = world * M * sh.n_local * 4
    gib_s = total_bytes_fp32 / (elapsed / steps) / 2**30
    upd_b, enc_b = sh.algorithmic_bytes()
    res = {
        "workload": name, "note": note, "layout": lay_name, "clients": M, "n_up_per_rank": sh.n_local,
        "ms_per_step": ms, "gib_s": gib_s, "update_kernel_ms": upd_ms, "encode_kernel_ms": enc_ms,
        "graph": graph, "steps_per_graph": G, "eager_ms_per_step": eager_ms, "exchange_ms": exchange_ms,
        "update_kernel": F.update_kernel(sh.L),
        "update_bytes": upd_b, "encode_bytes": enc_b,
        "update_gbs": upd_b / (upd_ms * 1e-3) / 1e9, "encode_gbs": enc_b / (enc_ms * 1e-3) / 1e9,
        "element_clients_per_s": world * M * sh.n_local / (elapsed / steps),
    }
    del sh
    torch.cuda.empty_cache()
    return res


def sq_valu(workload: str, kernel: str):
    """VALU lane-instructions per (client, value) of the profiled kernel
    (profiles/r01/sq.json, SQ_INSTS_VALU pass), None when not profiled."""
    try:
        with open(os.path.join(ROOT, "profiles", "r01", "sq.json")) as f:
            v = json.load(f)["workloads"][workload][kernel]["valu_lane_instr_per_element_client"]
        return float(v)
    except (OSError, KeyError, ValueError):
        return None


def pmc_traffic(workload: str, kernel: str = ""):
    """HBM bytes per k_update launch for `workload` from the newest committed
    rocprofv3 PMC summary (profiles/rNN/traffic.json, written by
    scripts/pmc_summary.py from separate --pmc FETCH_SIZE / WRITE_SIZE passes,
    FETCH_SIZE doubled per the gfx950 correction). None when absent."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")), reverse=True):
        try:
            with open(path) as f:
                kern = json.load(f)["workloads"].get(workload, {})
        except (OSError, ValueError, KeyError):
            continue
        # only a profile of the same kernel variant counts
        if kernel in kern and "hbm_bytes" in kern[kernel]:
            return kern[kernel]["hbm_bytes"], kernel, os.path.relpath(path, ROOT)
    return None


def end_to_end(torch, codec, name, reps=5):
    """Host-buffer path (fleet_update: pinned staging, H2D of the M uploads, layout
    parse, update, D2H of the merged Base64 + error check) on the same synthetic
    uploads: the PCIe-inclusive rate the JNI shim sees. Not `value`."""
    import fleet_amd as F
    from fleet_amd.layouts import LAYOUTS
    lay_name, M, _ = WORKLOADS[name]
    layout = LAYOUTS[lay_name]
    sh = Shard(codec, torch, layout, M, 0, 1)
    sh.encode()
    torch.cuda.synchronize()
    host = sh.text.cpu().numpy()
    ups = [host[c, : sh.L].tobytes() for c in range(M)]
    del sh
    d = dampen_policy(M)
    codec.update(ups, d)  # warm (allocations, staging)
    t0 = time.perf_counter()
    for _ in range(reps):
        merged = codec.update(ups, d)
    dt = (time.perf_counter() - t0) / reps
    return {"workload": name, "ms": dt * 1e3, "gib_s": M * layout.n_up * 4 / dt / 2**30,
            "h2d_bytes": M * F.b64_len(layout.n_up), "d2h_bytes": len(merged)}


def cpu_baseline(budget_s: float = 20.0):
    """The C restatement's faithful per-op chain (oracle/fleet_oracle.c, -O2), single
    thread (update() is synchronized in the reference). The reference's own codec
    and JNI backend (Base64.cpp, cppNN_backend.cpp) include <jni.h>, which the image
    lacks, so there is no reference build to time (kind "port"). Sample: MNIST
    layout, 64 clients (= configs[1]), client encode + CppNNUpdater.update chain,
    repeated while under budget."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from fleet_amd.layouts import MNIST
    o = pyoracle.Oracle()
    kind = "port"
    M = 64
    floats = [o.synth_upload(1, c, list(MNIST.w_sizes), list(MNIST.b_sizes)) for c in range(M)]
    d = dampen_policy(M)
    reps, t_total = 0, 0.0
    while t_total < budget_s and reps < 10:
        t0 = time.perf_counter()
        ups = [o.encode_floats(v) for v in floats]
        o.update_faithful(ups, d)
        t_total += time.perf_counter() - t0
        reps += 1
        if t_total > budget_s / 2:
            break
    per = t_total / reps
    value = M * MNIST.n_up * 4 / per / 2**30
    # SURVEY.md §8d's OpenMP leg on the same sample (the aggregation chain only):
    # the C restatement's fused chain on all the cores this process may use
    also = {}
    ups = [o.encode_floats(v) for v in floats]

    def rate(fn, budget=3.0):
        n, t = 0, 0.0
        while t < budget and n < 20:
            t0 = time.perf_counter()
            fn()
            t += time.perf_counter() - t0
            n += 1
        return M * MNIST.n_up * 4 / (t / n) / 2**30, t / n
    threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    hm = o.header_mask(list(MNIST.w_sizes), list(MNIST.b_sizes))
    vp, sp = rate(lambda: o.update_fused(ups, d, hm, threads=threads))
    also["port_fused_openmp"] = {"value": vp, "unit": "GiB/s", "cores": threads, "s_per_update": sp}
    also["note"] = "aggregation chain only (CppNNUpdater.update on pre-encoded uploads), same MNIST x 64 sample"
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
    return {"value": value, "unit": "GiB/s", "cores": 1, "kind": kind,
            "sample": f"MNIST layout (22,961 floats) x 64 clients: client encode + CppNNUpdater.update chain, "
                      f"{reps} rep(s), {per:.3f} s/rep, oracle faithful port -O2 (no reference build: Base64.cpp needs <jni.h>)",
            "cpu_model": cpu, "host_nproc": os.cpu_count(), "also": also}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="mnist64", choices=sorted(WORKLOADS))
    ap.add_argument("--extras", default="cifar10_256,synth1m_256",
                    help="comma list of extra workloads measured in the same run (N=1 only); '' for none")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", type=int, default=1,
                    help="1 (default): replay steps from a captured HIP graph; 0: eager launches")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) measurement")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    args = ap.parse_args()

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
    extras = {}
    if world == 1 and args.extras:
        for w in [x for x in args.extras.split(",") if x and x != args.workload]:
            extras[w] = time_workload(torch, dist, codec, w, max(3, args.steps // 4), 2, rank, world, args.graph)

    e2e = None
    if world == 1 and not args.no_e2e:
        e2e = end_to_end(torch, codec, args.workload)

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(args.cpu_budget)
    r = main_res
    achieved = r["update_gbs"]
    traffic = pmc_traffic(args.workload, r["update_kernel"]) if world == 1 else None
    line = {
        "metric": "gradient GiB/s encode+decode+aggregate (device-resident); % HBM roofline",
        "value": r["gib_s"],
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Philox4x32-10 value mix, SURVEY.md §8d), device-resident",
        "config": {"workload": args.workload, "layout": r["layout"], "clients": r["clients"],
                   "n_up_per_rank": r["n_up_per_rank"], "parallelism": f"element-shard x{world}",
                   "dampening": "policy 1 inverse, tau = c mod 3"},
        "roofline": {"bound": "hbm", "kernel": r["update_kernel"], "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "frac_of_copy_ceiling": achieved / HBM_COPY_GBS,
                     "limiter": LIMITER.get(r["update_kernel"].split("<")[0], "VALU issue"),
                     "valu_lane_instr_per_element_client": sq_valu(args.workload, r["update_kernel"]),
                     "traffic": traffic[0] if traffic else None,
                     "traffic_source": f"{traffic[2]} ({traffic[1]})" if traffic else None,
                     "bytes_per_launch": r["update_bytes"], "kernel_ms": r["update_kernel_ms"]},
        "cpu_baseline": cpu,
        "timing": {"graph": bool(r["graph"]), "steps_per_graph": r["steps_per_graph"],
                   "eager_ms_per_step": r["eager_ms_per_step"],
                   "exchange_ms": r["exchange_ms"],
                   "exchange": "none in the timed steps (element shards stay resident); N>1: one all_gather of "
                               "the merged slices timed separately (exchange_ms, max over ranks) and checked",
                   "kernel_ms": "HIP events around graph replays of 10 back-to-back launches"},
        "kernels": {"k_update_ms": r["update_kernel_ms"], "k_encode_f32_ms": r["encode_kernel_ms"],
                    "k_encode_gbs": r["encode_gbs"], "element_clients_per_s": r["element_clients_per_s"]},
        "extra": extras,
        "end_to_end_host_buffers": e2e,
    }
    if cpu:
        line["vs_cpu_baseline"] = r["gib_s"] / cpu["value"]
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
