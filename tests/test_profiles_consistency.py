"""The committed headline bench line agrees with the committed rocprof summary.

VERDICT r01 asked that `roofline.frac` equal the kernel's algorithmic bytes
divided by the `profiles/rNN` kernel average and by 8 TB/s, to within 5 %.
This checks that arithmetic on the files this round commits (CPU only: it reads
JSON/CSV, runs nothing on a GPU).
"""
import csv
import glob
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _newest_round():
    """The newest round that committed a headline line together with its kernel trace
    (None where the CSVs do not travel, e.g. a GPU box's snapshot)."""
    rounds = sorted(os.path.dirname(p) for p in glob.glob(os.path.join(ROOT, "profiles", "r*", "bench_default.json"))
                    if os.path.exists(os.path.join(os.path.dirname(p), "synth1m_256_kernel_stats.csv")))
    return rounds[-1] if rounds else None


def _canon(name):
    """A kernel name without spaces and with default trailing template arguments dropped
    (rocprofv3 spells k_update_encode<256, false> where the bench says k_update_encode<256>)."""
    return re.sub(r"(,false)?(,0)?(,256)?>$", ">", re.sub(r"\s+", "", name))


def _kernel_avg_ns(stats_csv, kernel):
    # rocprofv3 spells the full signature: compare the name with its template arguments
    with open(stats_csv, newline="") as f:
        for row in csv.DictReader(f):
            n = row["Name"].split("(")[0].replace("void ", "").replace("fleet::", "")
            if _canon(n) == _canon(kernel):
                return float(row["AverageNs"])
    raise KeyError(kernel)


@pytest.mark.parametrize("line", ["bench_default.json"])
def test_headline_roofline_matches_profile(line):
    PROF = _newest_round()
    if PROF is None:
        pytest.skip("no committed profile round with its kernel trace here")
    path = os.path.join(PROF, line)
    d = json.loads(open(path).read().strip().splitlines()[-1])
    assert d["config"]["workload"] == "synth1m_256"
    assert d["metric"].startswith("gradient GiB/s") and d["unit"] == "GiB/s"
    rf = d["roofline"]
    assert rf["peak"] == 8000.0 and rf["unit"] == "GB/s"
    # algorithmic bytes of the fused step: aggregation M*L + L + 4n, encode 4nM + ML
    M, n = 256, 1 << 20
    L = 4 * ((4 * n + 2) // 3)  # padded Base64 text of the 4n bytes of n int32 codes
    assert rf["bytes_update"] == M * L + L + 4 * n
    assert rf["bytes_encode"] == 4 * n * M + M * L
    assert rf["bytes_per_launch"] == rf["bytes_update"] + rf["bytes_encode"]
    avg_ns = _kernel_avg_ns(os.path.join(PROF, "synth1m_256_kernel_stats.csv"), rf["kernel"])
    frac_prof = rf["bytes_per_launch"] / (avg_ns * 1e-9) / 8e12
    assert abs(rf["frac"] - frac_prof) / frac_prof < 0.05, (rf["frac"], frac_prof)
    # the aggregation kernel on its own, same rule
    ag = rf["aggregation_alone"]
    avg_ns = _kernel_avg_ns(os.path.join(PROF, "synth1m_256_kernel_stats.csv"), ag["kernel"])
    frac_prof = ag["bytes_per_launch"] / (avg_ns * 1e-9) / 8e12
    assert abs(ag["frac"] - frac_prof) / frac_prof < 0.05, (ag["frac"], frac_prof)
    # whole-job value: M * n fp32-equivalent bytes per step
    assert abs(d["value"] - M * n * 4 / 2**30 / (d["ms_per_step"] * 1e-3)) / d["value"] < 1e-6
