#!/usr/bin/env python3
"""Per-launch SQ counters of the aggregation / encode kernels from a rocprofv3
--pmc run (SQ_INSTS_VALU, SQ_INSTS_LDS, SQ_BUSY_CU_CYCLES, SQ_WAVES ...):
VALU instructions per element-client, CU-busy cycles per launch.

usage: sq_summary.py OUT.json WORKLOAD=DIR:ELEMENT_CLIENTS ...
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main():
    res = {"note": "SQ_INSTS_* are wave-instructions; x64 / element-clients = lane-instructions per "
                   "(client, value) step of the chain. Means over the launches after the first.",
           "workloads": {}}
    for spec in sys.argv[2:]:
        wl, rest = spec.split("=", 1)
        d, ec = rest.rsplit(":", 1)
        ec = float(ec)
        per = {}
        with open(os.path.join(d, "run_counter_collection.csv")) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                per.setdefault(k, {}).setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
                per[k][row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
        out = {}
        for k, cs in per.items():
            if not (k.startswith("k_update") or k.startswith("k_encode")):
                continue
            o = {}
            for c, disp in cs.items():
                vals = [v for _, v in sorted(disp.items(), key=lambda t: int(t[0]))]
                vals = vals[1:] if len(vals) > 1 else vals
                o[c] = sum(vals) / len(vals)
            if "SQ_INSTS_VALU" in o:
                o["valu_lane_instr_per_element_client"] = o["SQ_INSTS_VALU"] * 64 / ec
            if "SQ_INSTS_LDS" in o:
                o["lds_lane_instr_per_element_client"] = o["SQ_INSTS_LDS"] * 64 / ec
            out[k] = o
        res["workloads"][wl] = out
    with open(sys.argv[1], "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
