#!/usr/bin/env python3
"""Kardam bookkeeping on a bench workload (argv[1], default synth1m_256): the
update alone (the plan's kernel), the update with Kardam's side outputs in the
same pass (the same kernel with KD = true, + k_kardam_reduce), and the two-pass
path (the update plus fleet_kardam_grads' own pass over the uploads,
k_kardam_grads). Run under `rocprofv3 --kernel-trace --stats` for the
per-kernel averages."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import fleet_amd as F  # noqa: E402
from fleet_amd.layouts import LAYOUTS  # noqa: E402

W = sys.argv[1] if len(sys.argv) > 1 else "synth1m_256"
lay = LAYOUTS[bench.WORKLOADS[W][0]]
M = bench.WORKLOADS[W][1]
codec = F.Codec(0)
sh = bench.Shard(codec, torch, lay, M, 0, 1)
sh.encode()
torch.cuda.synchronize()
d = bench.dampen_policy(M)
lr = 0.05
prev = torch.zeros((M, sh.vpitch), dtype=torch.float32, device="cuda")
g_out = torch.zeros_like(prev)
hpos = sh.hpos_global
for _ in range(20):
    sh.aggregate()
torch.cuda.synchronize()
codec.update_kardam_device(sh.text, sh.L, d, hpos, lr, sh.merged, sh.merged_f32, None, None, prev)
for _ in range(20):
    t0 = time.perf_counter()
    ng, nd = codec.update_kardam_device(sh.text, sh.L, d, hpos, lr, sh.merged, sh.merged_f32, prev, np.ones(M),
                                        g_out)
    print("fused update+kardam (host clock) %.3f ms" % ((time.perf_counter() - t0) * 1e3))
codec.check()
host = sh.text.cpu().numpy()
ups = [host[c, :sh.L].tobytes() for c in range(M)]
g_texts, _, _ = codec.kardam_grads(ups, d, lr)
for _ in range(2):
    codec.kardam_grads(ups, d, lr, g_texts)
print("norms", ng[:3], nd[:3])
