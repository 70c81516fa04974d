"""fleet_update phase times (FLEET_TRACE) on MNIST-64 synthetic uploads (dev probe)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fleet_amd as F
from fleet_amd.layouts import LAYOUTS

lay = LAYOUTS["mnist"]
codec = F.Codec(0)
M = 64
groups = (lay.n_up + 2) // 3
vals = torch.empty((M, 3 * groups), dtype=torch.float32, device="cuda")
text = torch.empty((M, 16 * groups), dtype=torch.uint8, device="cuda")
codec.synth_device(1, vals, lay.n_up, np.asarray(lay.header_positions(), np.int32),
                   np.asarray(lay.header_values(), np.float32))
codec.encode_device(vals, lay.n_up, text)
torch.cuda.synchronize()
L = F.b64_len(lay.n_up)
host = text.cpu().numpy()
ups = [host[c, :L].tobytes() for c in range(M)]
d = [1.0 / ((c % 3) + 1) for c in range(M)]
for _ in range(3):
    codec.update(ups, d)
ts = []
for _ in range(50):
    t = time.perf_counter()
    codec.update(ups, d)
    ts.append(time.perf_counter() - t)
ts.sort()
print(f"codec.update: median {ts[25] * 1e3:.3f} ms, min {ts[0] * 1e3:.3f} ms", file=sys.stderr)
