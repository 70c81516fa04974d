#!/usr/bin/env python3
"""Dev tool: board power and clocks while one kernel form runs back to back (no GPU settings
are changed; `amd-smi metric` is only read, from a child process).

usage: power_probe.py WORKLOAD MODE SECONDS   (MODE fused | upd | enc; the full-width N = 1 problem)

Prints, per mode, the launches per second and the median / max of the sampled socket power
and GFX clock, so the clock the chip holds under each job can be set beside its time."""
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import fleet_amd as F  # noqa: E402
from fleet_amd.layouts import LAYOUTS  # noqa: E402


def sample(stop, out):
    while not stop.is_set():
        try:
            r = subprocess.run(["amd-smi", "metric", "-g", "0", "--json"], capture_output=True, text=True,
                               timeout=10)
            out.append(r.stdout)
        except Exception as e:  # noqa: BLE001 -- a dev probe: report and go on
            out.append(f"ERR {e}")
        time.sleep(0.3)


def numbers(raw, keys):
    """every numeric value under a key containing one of `keys` in a JSON blob"""
    vals = {k: [] for k in keys}

    def walk(o, path):
        if isinstance(o, dict):
            for k, v in o.items():
                walk(v, path + [str(k).lower()])
        elif isinstance(o, list):
            for v in o:
                walk(v, path)
        else:
            for k in keys:
                if any(k in p for p in path[-2:]):
                    try:
                        vals[k].append(float(o))
                    except (TypeError, ValueError):
                        pass

    for s in raw:
        try:
            walk(json.loads(s), [])
        except ValueError:
            pass
    return vals


def main():
    name, mode, secs = sys.argv[1], sys.argv[2], float(sys.argv[3])
    lay_name, M, _ = bench.WORKLOADS[name]
    codec = F.Codec(0)
    sh = bench.Shard(codec, torch, LAYOUTS[lay_name], M, 0, 1, strong=True)
    L = F.b64_len(sh.n_local)
    hloc = sh.hpos_global[(sh.hpos_global >= 0) & (sh.hpos_global < sh.n_local)]
    bufs = [sh.text, torch.zeros_like(sh.text)]
    sh.encode()

    def launch(i):
        if mode == "fused":
            codec.update_encode_device(bufs[i % 2], L, sh.dampen, hloc, sh.merged, sh.merged_f32, sh.values,
                                       bufs[(i + 1) % 2])
        elif mode == "upd":
            codec.update_device(bufs[0], L, sh.dampen, hloc, sh.merged, sh.merged_f32)
        else:
            sh.encode()

    for i in range(4):
        launch(i)
    torch.cuda.synchronize()
    raw, stop = [], threading.Event()
    th = threading.Thread(target=sample, args=(stop, raw))
    th.start()
    t0, n = time.time(), 0
    while time.time() - t0 < secs:
        for _ in range(20):
            launch(n)
            n += 1
        torch.cuda.synchronize()
    el = time.time() - t0
    stop.set()
    th.join()
    codec.check()
    v = numbers(raw, ["power", "gfx_clk", "clk"])
    pw = [x for x in v["power"] if 50 < x < 3000]
    ck = [x for x in v["gfx_clk"] if 100 < x < 5000] or [x for x in v["clk"] if 100 < x < 5000]
    print(f"{name} {mode}: {n / el:8.1f} launches/s ({el / n * 1e6:7.1f} us each, eager)  samples {len(raw)}  "
          f"power median {np.median(pw) if pw else float('nan'):6.0f} max {max(pw) if pw else float('nan'):6.0f} W  "
          f"gfx clock median {np.median(ck) if ck else float('nan'):6.0f} MHz", flush=True)
    if not pw:
        print("raw sample:", raw[:1], flush=True)


if __name__ == "__main__":
    main()
