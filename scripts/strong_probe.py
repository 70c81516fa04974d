#!/usr/bin/env python3
"""Dev tool: the per-rank local step of bench.py's strong-scaling value at N = 1, 2, 4, 8
on ONE GPU (rank 0's column window of the fixed problem, the pipelined launch; no
collective): what an N-GPU strong run's kernels cost per rank. Prints one line per N."""
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
    name = sys.argv[1] if len(sys.argv) > 1 else "synth1m_256"
    ns = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4,8").split(",")]
    mode = sys.argv[3] if len(sys.argv) > 3 else "fused"  # fused | upd | enc
    lay_name, M, _ = bench.WORKLOADS[name]
    M = int(os.environ.get("PROBE_M", M))  # experiments: another client count on the same windows
    layout = LAYOUTS[lay_name]
    codec = F.Codec(0)
    base = None
    for N in ns:
        sh = bench.Shard(codec, torch, layout, M, 0, N, strong=True)
        pm = int(os.environ.get("PROBE_PITCH_MULT", "1"))  # experiments: rows pm times wider than the window
        if pm > 1:
            sh.text = torch.zeros((M, sh.pitch * pm), dtype=torch.uint8, device=sh.text.device)  # pitch = pm x window
        v0 = 3 * sh.gb
        hloc = sh.hpos_global[(sh.hpos_global >= v0) & (sh.hpos_global < v0 + sh.n_local)] - v0
        L_loc = F.b64_len(sh.n_local)
        bufs = [sh.text, torch.zeros_like(sh.text)]

        def local(i):
            if mode == "fused":
                codec.update_encode_device(bufs[i % 2], L_loc, sh.dampen, hloc, sh.merged, sh.merged_f32, sh.values,
                                           bufs[(i + 1) % 2])
            elif mode == "upd":
                codec.update_device(bufs[0], L_loc, sh.dampen, hloc, sh.merged, sh.merged_f32)
            else:
                codec.encode_device(sh.values, sh.n_local, bufs[1])
        sh.encode()
        local(0)
        local(1)
        torch.cuda.synchronize()
        codec.check()
        ms = bench.kernel_ms(torch, lambda: (local(0), local(1)), reps=5) / 2
        base = base or ms
        print(f"{name} M={M} pitch x{pm} {mode} N={N} groups/rank={sh.groups} kernel={F.update_encode_kernel(L_loc)} {ms * 1e3:.1f} us  "
              f"speedup {base / ms:.2f} (x{N} ideal)", flush=True)
        del bufs, sh
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
