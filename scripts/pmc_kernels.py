#!/usr/bin/env python3
"""Per-kernel means of a rocprofv3 --pmc (+ --kernel-trace) run: every counter, plus
cycles per VALU instruction per SIMD (SQ_BUSY_CU_CYCLES x 4 / SQ_INSTS_VALU, the
measure DESIGN.md §4 quotes), the SQ_WAIT_* / SQ_ACTIVE_INST_ANY shares of
SQ_WAVE_CYCLES, the mean duration and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs /
duration). The first dispatch of each kernel is dropped.

usage: pmc_kernels.py DIR [ELEMENT_CLIENTS]   (DIR holds run_counter_collection.csv)
"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main():
    d = sys.argv[1]
    ec = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    per, dur = {}, {}
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            per.setdefault(k, {}).setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
            per[k][row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    tp = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(tp):
        with open(tp) as f:
            for row in csv.DictReader(f):
                dur.setdefault(short(row["Kernel_Name"]), []).append(
                    (int(row["Dispatch_Id"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    for k, cs in sorted(per.items()):
        o = {}
        for c, disp in cs.items():
            vals = [v for _, v in sorted(disp.items(), key=lambda t: int(t[0]))]
            vals = vals[1:] if len(vals) > 1 else vals
            o[c] = sum(vals) / len(vals)
        line = [k]
        if k in dur:
            ds = [t for _, t in sorted(dur[k])]
            ds = ds[1:] if len(ds) > 1 else ds
            o["dur_us"] = sum(ds) / len(ds) / 1e3
            line.append("%.1f us" % o["dur_us"])
            if "GRBM_GUI_ACTIVE" in o:
                line.append("clock %.2f GHz" % (o["GRBM_GUI_ACTIVE"] / 8 / (o["dur_us"] * 1e3)))
        if "SQ_INSTS_VALU" in o and "SQ_BUSY_CU_CYCLES" in o:
            line.append("cyc/VALU %.2f" % (o["SQ_BUSY_CU_CYCLES"] * 4 / o["SQ_INSTS_VALU"]))
        if ec and "SQ_INSTS_VALU" in o:
            line.append("VALU/(c,v) %.1f" % (o["SQ_INSTS_VALU"] * 64 / ec))
        if ec and "SQ_INSTS_LDS" in o:
            line.append("LDS/(c,v) %.1f" % (o["SQ_INSTS_LDS"] * 64 / ec))
        wc = o.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in o:
                    line.append("%s %.2f" % (c[3:].lower(), o[c] / wc))
        if o.get("SQ_LDS_IDX_ACTIVE"):
            for c in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_UNALIGNED_STALL", "SQ_LDS_ADDR_CONFLICT"):
                if c in o:
                    line.append("%s %.3f" % (c[7:].lower(), o[c] / o["SQ_LDS_IDX_ACTIVE"]))
            line.append("lds_active %.0f" % o["SQ_LDS_IDX_ACTIVE"])
        if "SQ_WAVES" in o:
            line.append("waves %.0f" % o["SQ_WAVES"])
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
