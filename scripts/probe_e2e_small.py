"""Dev probe: bench.end_to_end on small workloads with many reps, per staging setting
(FLEET_STAGE_THREADS from the environment), to see the host path's fixed overheads."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import fleet_amd as F  # noqa: E402

codec = F.Codec(0)
for name in sys.argv[1:] or ["mnist64"]:
    r = bench.end_to_end(torch, codec, name, reps=30)
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()
                      if k in ("workload", "ms", "ms_mean", "h2d_floor_ms", "x_floor")}),
          "rows", round(r["pinned_rows"]["ms"], 4), flush=True)
codec.close()
