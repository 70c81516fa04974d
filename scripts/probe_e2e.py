"""Breakdown of the host-buffer update path on the GPU box (dev probe): H2D
rate from pinned memory, host copy rate, and the fleet_update call itself."""
import time

import numpy as np
import torch



n = 7837440
src = torch.empty(n, dtype=torch.uint8).pin_memory()
dst = torch.empty(n, dtype=torch.uint8, device="cuda")
for _ in range(3):
    dst.copy_(src, non_blocking=True)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20):
    dst.copy_(src, non_blocking=True)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 20
print(f"H2D pinned {n/1e6:.1f} MB: {dt*1e3:.3f} ms ({n/dt/1e9:.1f} GB/s)")
back = torch.empty(n, dtype=torch.uint8).pin_memory()
t = time.perf_counter()
for _ in range(20):
    back.copy_(dst, non_blocking=True)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 20
print(f"D2H pinned: {dt*1e3:.3f} ms ({n/dt/1e9:.1f} GB/s)")
ups = [np.random.default_rng(c).integers(65, 90, 122460, dtype=np.uint8).tobytes() for c in range(64)]
buf = np.empty(n, dtype=np.uint8)
t = time.perf_counter()
for _ in range(20):
    for c in range(64):
        buf[c * 122464:c * 122464 + 122460] = np.frombuffer(ups[c], dtype=np.uint8)
dt = (time.perf_counter() - t) / 20
print(f"host copy 64 x 122460 B (numpy, 1 thread): {dt*1e3:.3f} ms")
