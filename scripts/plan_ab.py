#!/usr/bin/env python3
"""Dev tool: same-process A/B of launch plans on one window (rank 0's column window of
WORKLOAD split over N ranks, as strong_probe.py): the plans' graphs are timed in turns,
REPS rounds, so clock and thermal drift hit every plan alike. Prints per plan the
median and min of the per-round averages (us per launch).

usage: plan_ab.py WORKLOAD N MODE PLAN [PLAN ...]   (MODE fused | upd; PLAN a fleet_set_plan
spec, '-' for the default; REPS from the environment, default 7)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import fleet_amd as F  # noqa: E402
from fleet_amd.layouts import LAYOUTS  # noqa: E402


def main():
    name, N, mode = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    plans = ["" if p == "-" else p for p in sys.argv[4:]]
    reps = int(os.environ.get("REPS", "7"))
    lay_name, M, _ = bench.WORKLOADS[name]
    codec = F.Codec(0)
    sh = bench.Shard(codec, torch, LAYOUTS[lay_name], M, 0, N, strong=True)
    v0 = 3 * sh.gb
    hloc = sh.hpos_global[(sh.hpos_global >= v0) & (sh.hpos_global < v0 + sh.n_local)] - v0
    L_loc = F.b64_len(sh.n_local)
    bufs = [sh.text, torch.zeros_like(sh.text)]
    sh.encode()

    def local(i):
        if mode == "fused":
            codec.update_encode_device(bufs[i % 2], L_loc, sh.dampen, hloc, sh.merged, sh.merged_f32, sh.values,
                                       bufs[(i + 1) % 2])
        else:
            codec.update_device(bufs[0], L_loc, sh.dampen, hloc, sh.merged, sh.merged_f32)

    ref = None
    kern = {}
    for p in plans:  # every plan's output is the same bytes
        F.set_plan(p)
        kern[p] = F.update_encode_kernel(L_loc) if mode == "fused" else F.update_kernel(L_loc)
        local(0)
        torch.cuda.synchronize()
        codec.check()
        out = sh.merged.cpu().numpy().tobytes()
        assert ref is None or out == ref, f"plan {p!r}: merged text differs"
        ref = out
    t = {p: [] for p in plans}
    for _ in range(reps):
        for p in plans:
            F.set_plan(p)
            t[p].append(bench.kernel_ms(torch, lambda: (local(0), local(1)), reps=5, rounds=2) / 2 * 1e3)
    F.set_plan("")
    print(f"{name} N={N} {mode} groups/rank={sh.groups} reps={reps}", flush=True)
    for p in plans:
        a = np.array(t[p])
        print(f"  {p or 'default':40s} {kern[p]:36s} median {np.median(a):8.1f}  min {a.min():8.1f} us", flush=True)


if __name__ == "__main__":
    main()
