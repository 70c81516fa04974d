#!/usr/bin/env python3
"""Dev tool: the pipelined step of one window as TWO concurrent kernels -- the update
alone on the launch stream and the client encode on a second stream, forked and
joined by events inside the captured graph -- against the one-launch fused step, per
launch plan of the update (same process, graphs timed in turns).

usage: dual_stream_probe.py WORKLOAD N PLAN [PLAN ...]   ('-' = the default plan; REPS)"""
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
    name, N = sys.argv[1], int(sys.argv[2])
    plans = ["" if p == "-" else p for p in sys.argv[3:]]
    reps = int(os.environ.get("REPS", "7"))
    lay_name, M, _ = bench.WORKLOADS[name]
    codec = F.Codec(0)
    sh = bench.Shard(codec, torch, LAYOUTS[lay_name], M, 0, N, strong=True)
    v0 = 3 * sh.gb
    hloc = sh.hpos_global[(sh.hpos_global >= v0) & (sh.hpos_global < v0 + sh.n_local)] - v0
    L_loc = F.b64_len(sh.n_local)
    bufs = [sh.text, torch.zeros_like(sh.text)]
    sh.encode()
    side = torch.cuda.Stream()

    def fused(i):
        codec.update_encode_device(bufs[i % 2], L_loc, sh.dampen, hloc, sh.merged, sh.merged_f32, sh.values,
                                   bufs[(i + 1) % 2])

    def dual(i):
        main_s = torch.cuda.current_stream()
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            codec.encode_device(sh.values, sh.n_local, bufs[(i + 1) % 2])
        codec.update_device(bufs[i % 2], L_loc, sh.dampen, hloc, sh.merged, sh.merged_f32)
        main_s.wait_stream(side)

    def upd(i):
        codec.update_device(bufs[i % 2], L_loc, sh.dampen, hloc, sh.merged, sh.merged_f32)

    forms = {"fused": fused, "dual": dual, "upd": upd}
    ref = None
    for p in plans:  # the merged text is the same under every plan and form
        F.set_plan(p)
        for f in ("fused", "dual"):
            forms[f](0)
            torch.cuda.synchronize()
            codec.check()
            out = sh.merged.cpu().numpy().tobytes()
            assert ref is None or out == ref, (p, f)
            ref = out
    t = {(p, f): [] for p in plans for f in forms}
    for _ in range(reps):
        for p in plans:
            F.set_plan(p)
            for f, fn in forms.items():
                t[(p, f)].append(bench.kernel_ms(torch, lambda: (fn(0), fn(1)), reps=5, rounds=2) / 2 * 1e3)
    F.set_plan("")
    print(f"{name} N={N} groups/rank={sh.groups} reps={reps}", flush=True)
    for p in plans:
        line = "  ".join(f"{f} {np.median(t[(p, f)]):7.1f}" for f in forms)
        print(f"  {p or 'default':36s} {line} us", flush=True)


if __name__ == "__main__":
    main()
