# configs[4] N=4 window, update alone: rocprof kernel durations at M=256 / 1024 / 4096 and N=1 at M=1024
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/d10; mkdir -p $O
for m in 256 1024 4096; do
  PROBE_M=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$m -o run -- python3 scripts/strong_probe.py synth4m_4096 4 upd > $O/t$m.log 2>&1 || exit 1
  grep "N=" $O/t$m.log
  python3 - $O/t$m <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_update" in r["Name"]:
            print("   rocprof", r["Name"][:40], r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 1), "min", round(float(r["MinNs"]) / 1e3, 1), "max", round(float(r["MaxNs"]) / 1e3, 1))
PY
done
