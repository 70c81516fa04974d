#!/usr/bin/env python3
"""Dev tool: per-wave phase trace of the tile kernels (a FLEET_TRACE build of the library,
FLEET_CODEC_LIB=ab/trace.so): shader-clock stamps at the phase boundaries of tiles 0..63,
chunk by chunk, wave by wave (kernels.hip FLEET_WTRACE). Prints, per wave role, the mean
cycles of each phase and of the barrier waits, so the tile's idle time shows where it is.

usage: FLEET_CODEC_LIB=ab/trace.so python3 scripts/tile_trace.py WORKLOAD [N] [upd|fused]
(ab/btrace.so, FLEET_TRACE_WAVES=0: block start / end only, at the product build's SGPR count)
(N: rank 0's window of the workload split over N ranks, as strong_probe.py)"""
import ctypes as C
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
    name = sys.argv[1] if len(sys.argv) > 1 else "cifar10_256"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    mode = sys.argv[3] if len(sys.argv) > 3 else "upd"
    lay_name, M, _ = bench.WORKLOADS[name]
    codec = F.Codec(0)
    L = F.lib()
    L.fleet_dev_trace.argtypes = [C.c_void_p]
    sh = bench.Shard(codec, torch, LAYOUTS[lay_name], M, 0, N, strong=True)
    v0 = 3 * sh.gb
    hloc = sh.hpos_global[(sh.hpos_global >= v0) & (sh.hpos_global < v0 + sh.n_local)] - v0
    L_loc = F.b64_len(sh.n_local)
    nxt = torch.zeros_like(sh.text)
    sh.encode()
    NW = 64 * 64 * 8 * 4
    trace = torch.zeros(NW + 65536 * 4, dtype=torch.int64, device="cuda")

    def run():
        if mode == "fused":
            codec.update_encode_device(sh.text, L_loc, sh.dampen, hloc, sh.merged, sh.merged_f32, sh.values, nxt)
        else:
            codec.update_device(sh.text, L_loc, sh.dampen, hloc, sh.merged, sh.merged_f32)

    run()
    torch.cuda.synchronize()
    assert L.fleet_dev_trace(trace.data_ptr()) == 0
    for _ in range(3):  # the last launch's stamps stay
        trace.zero_()
        run()
    torch.cuda.synchronize()
    codec.check()
    full = trace.cpu().numpy()
    t = full[:NW].reshape(64, 64, 8, 4).astype(np.float64)
    bt = full[NW:].reshape(65536, 4)
    if os.environ.get("TRACE_OUT"):  # the raw block trace for offline analysis
        np.save(os.environ["TRACE_OUT"], bt[bt[:, 0] > 0])
    kern = F.update_kernel(L_loc) if mode == "upd" else F.update_encode_kernel(L_loc)
    print(f"{name} N={N} {mode} kernel={kern} groups/rank={sh.groups}", flush=True)
    waves = [w for w in range(8) if t[:, :, w, 0].any()]
    if not waves:  # a block-only trace build (FLEET_TRACE_WAVES=0): residency alone
        residency(bt)
        return
    chunks = [k for k in range(64) if t[:, k, waves[0], 0].any()]
    print(f"traced tiles 64, chunks {len(chunks)} (k {chunks[0]}..{chunks[-1]}), waves {waves}")
    classic = t[:, :, :, 3].any()
    for w in waves:
        a = t[:, chunks[0]:chunks[-1] + 1, w, :]
        ok = (a[..., 0] > 0) & (a[..., 1] > 0) & (a[..., 2] > 0)
        work = np.where(ok, a[..., 1] - a[..., 0], np.nan)
        wait1 = np.where(ok, a[..., 2] - a[..., 1], np.nan)
        line = f"wave {w}: work {np.nanmean(work):8.0f}  barrier {np.nanmean(wait1):8.0f}"
        if classic:
            ok2 = ok & (a[..., 3] > 0)
            p2 = np.where(ok2, a[..., 3] - a[..., 2], np.nan)
            nxt0 = np.concatenate([a[:, 1:, 0], np.full((64, 1), np.nan)], axis=1)
            wait2 = np.where(ok2 & (nxt0 > 0), nxt0 - a[..., 3], np.nan)
            line += f"  phase2 {np.nanmean(p2):8.0f}  barrier2 {np.nanmean(wait2):8.0f}"
        else:
            nxt0 = np.concatenate([a[:, 1:, 0], np.full((64, 1), np.nan)], axis=1)
            gap = np.where(ok & (nxt0 > 0), nxt0 - a[..., 2], np.nan)
            line += f"  to-next {np.nanmean(gap):6.0f}"
        print(line, flush=True)
    # whole tile: first stamp to last
    first = np.where(t[:, :, :, 0] > 0, t[:, :, :, 0], np.inf).min(axis=(1, 2))
    last = t.max(axis=(1, 2, 3))
    residency(bt)
    print(f"tile span (cycles): mean {np.mean(last - first):.0f}, min {np.min(last - first):.0f}, "
          f"max {np.max(last - first):.0f}; per chunk {np.mean(last - first) / max(1, len(chunks)):.0f}")


def residency(bt):
    """Block start / end (100 MHz clock) of every traced block: rounds of the launch."""
    used = bt[:, 0] > 0
    if not used.any():
        return
    st, en = bt[used, 0].astype(np.float64), bt[used, 1].astype(np.float64)
    t0 = st.min()
    st, en = (st - t0) / 100.0, (en - t0) / 100.0  # us
    n = used.sum()
    hw = bt[used, 2]
    xcc = (hw >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    first = st < 2.0
    print(f"blocks {n}: started in the first 2 us {first.sum()}, start max {st.max():.1f} us, end max {en.max():.1f} us, "
          f"block span mean {np.mean(en - st):.1f} us")
    key = xcc * 64 + se * 16 + cu
    _, counts = np.unique(key[first], return_counts=True)
    print(f"first-round blocks per CU: min {counts.min()} max {counts.max()} mean {counts.mean():.2f} "
          f"({len(counts)} CUs)")
    for lo, hi in ((0, 2), (2, 50), (50, 150), (150, 400), (400, 1e9)):
        m = (st >= lo) & (st < hi)
        if m.any():
            print(f"  start in [{lo}, {hi}) us: {m.sum()} blocks, their end mean {en[m].mean():.1f} us")


if __name__ == "__main__":
    main()
