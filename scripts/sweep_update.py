#!/usr/bin/env python3
"""Dev tool: time k_update / k_update_tiled over layouts, client counts and
launch variants (FLEET_UPDATE_MODE / FLEET_TILE_G / FLEET_UPDATE_K are read at
every launch, so one process sweeps them all). Prints one line per case."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import fleet_amd as F  # noqa: E402
from fleet_amd.layouts import LAYOUTS  # noqa: E402


def run(codec, layout, M, env, reps=20):
    for k in ("FLEET_UPDATE_MODE", "FLEET_TILE_G", "FLEET_UPDATE_K"):
        os.environ.pop(k, None)
    os.environ.update(env)
    n = layout.n_up
    groups = (n + 2) // 3
    dev = torch.device("cuda", 0)
    vals = torch.empty((M, 3 * groups), dtype=torch.float32, device=dev)
    text = torch.empty((M, 16 * groups), dtype=torch.uint8, device=dev)
    merged = torch.empty((16 * groups,), dtype=torch.uint8, device=dev)
    f32 = torch.empty((3 * groups,), dtype=torch.float32, device=dev)
    hpos, hval = layout.header_positions(), layout.header_values()
    codec.synth_device(1, vals, n, hpos, hval)
    codec.encode_device(vals, n, text)
    L = F.b64_len(n)
    d = [1.0 / ((c % 3) + 1) for c in range(M)]
    for _ in range(3):
        codec.update_device(text, L, d, hpos, merged, f32)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        codec.update_device(text, L, d, hpos, merged, f32)
    b.record()
    torch.cuda.synchronize()
    codec.check()
    us = a.elapsed_time(b) / reps * 1e3
    return us, M * n / (us * 1e-6)


def main():
    cases = sys.argv[1] if len(sys.argv) > 1 else "mnist"
    codec = F.Codec(0)
    if cases == "mnist":
        lay = LAYOUTS["mnist"]
        for M in (1, 4, 16, 64):
            for env in ({"FLEET_UPDATE_MODE": "tiled", "FLEET_TILE_G": "16"},
                        {"FLEET_UPDATE_MODE": "tiled", "FLEET_TILE_G": "32"},
                        {"FLEET_UPDATE_MODE": "stream", "FLEET_UPDATE_K": "1"}):
                us, rate = run(codec, lay, M, env)
                print(f"mnist M={M:4d} {env} {us:9.1f} us  {rate / 1e9:7.2f} G elem-client/s", flush=True)
    else:
        lay = LAYOUTS[cases]
        M = int(sys.argv[2]) if len(sys.argv) > 2 else 256
        for env in ({"FLEET_UPDATE_MODE": "tiled", "FLEET_TILE_G": "16"},
                    {"FLEET_UPDATE_MODE": "tiled", "FLEET_TILE_G": "32"},
                    {"FLEET_UPDATE_MODE": "tiled", "FLEET_TILE_G": "64"},
                    {"FLEET_UPDATE_MODE": "stream", "FLEET_UPDATE_K": "1"},
                    {"FLEET_UPDATE_MODE": "stream", "FLEET_UPDATE_K": "2"}):
            us, rate = run(codec, lay, M, env, reps=5)
            print(f"{cases} M={M:4d} {env} {us:9.1f} us  {rate / 1e9:7.2f} G elem-client/s", flush=True)


if __name__ == "__main__":
    main()
