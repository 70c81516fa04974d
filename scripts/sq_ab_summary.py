#!/usr/bin/env python3
"""Print the mean per-launch SQ counters of the k_update* kernels from scripts/gpu_sq_ab.sh output."""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sqab"
labels = sorted({os.path.basename(d).rsplit("_p", 1)[0] for d in glob.glob(os.path.join(root, "*_p*")) if os.path.isdir(d)})
for lab in labels:
    tot = {}
    name = None
    for d in sorted(glob.glob(os.path.join(root, f"{lab}_p*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        per = {}
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            if not k.startswith("k_update"):
                continue
            name = k
            per.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
            per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
        for c, disp in per.items():
            vals = [v for _, v in sorted(disp.items(), key=lambda t: int(t[0]))][1:] or list(disp.values())
            tot[c] = sum(vals) / len(vals)
    print(f"== {lab} ({name})")
    for c in sorted(tot):
        print(f"   {c:28s} {tot[c]:.4g}")
