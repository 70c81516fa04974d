#!/usr/bin/env python3
"""Dev tool: offline analysis of a per-block trace saved by tile_trace.py (TRACE_OUT):
block start / end on the 100 MHz clock and the block's hardware place (XCC, SE, CU).
Prints how a launch's blocks were placed and how their end times depend on the load of
their CU and on their XCC.

usage: bt_analyze.py BT.npy [N_UPDATE_BLOCKS]   (update blocks = the first N in dispatch order)"""
import sys

import numpy as np


def main():
    bt = np.load(sys.argv[1])
    nu = int(sys.argv[2]) if len(sys.argv) > 2 else len(bt)
    bt = bt[:nu]
    st = (bt[:, 0] - bt[:, 0].min()) / 100.0
    en = (bt[:, 1] - bt[:, 0].min()) / 100.0
    hw = bt[:, 2].astype(np.int64)
    xcc = (hw >> 32) & 0xF
    se = (hw >> 13) & 0x7
    cu = (hw >> 8) & 0xF
    key = xcc * 128 + se * 16 + cu
    first = st < 2.0
    print(f"{len(bt)} blocks, {first.sum()} in the first round; end mean {en.mean():.1f} max {en.max():.1f} us; "
          f"span mean {(en - st).mean():.1f} us")
    ks, inv, counts = np.unique(key[first], return_inverse=True, return_counts=True)
    load = counts[inv]  # blocks on this block's CU (first round)
    for c in sorted(set(load)):
        m = load == c
        print(f"  CUs with {c} first-round blocks: {m.sum() // c} CUs, block end mean {en[first][m].mean():.1f} "
              f"max {en[first][m].max():.1f} us")
    for x in sorted(set(xcc)):
        m = xcc == x
        print(f"  XCC {x}: {m.sum()} blocks, end mean {en[m].mean():.1f} max {en[m].max():.1f}, "
              f"span mean {(en[m] - st[m]).mean():.1f} us")
    # within a CU: do the blocks finish together?
    spread = []
    for k in ks:
        m = key == k
        if m.sum() > 1:
            spread.append(en[m].max() - en[m].min())
    if spread:
        print(f"  end spread within a CU: mean {np.mean(spread):.1f} max {np.max(spread):.1f} us")


if __name__ == "__main__":
    main()
