# shader clock during the update: GRBM_COUNT (clocks) / kernel duration, configs[4] windows vs the full width
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/d11; mkdir -p $O
run() {  # tag, env..., args
  local tag=$1; shift
  env "$@" timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_COUNT GRBM_GUI_ACTIVE --output-format csv -d $O/$tag -o run -- python3 scripts/strong_probe.py $PARGS > $O/$tag.log 2>&1 || exit 1
  grep "N=" $O/$tag.log
  python3 - $O/$tag <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list); dur = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_update" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_update" in r.get("Kernel_Name", ""):
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
d = sum(dur) / max(1, len(dur))
print("   ", {k: round(sum(v) / len(v)) for k, v in acc.items()}, "dur us", round(d, 1),
      "GRBM_COUNT/us (MHz)", round(sum(acc["GRBM_COUNT"]) / len(acc["GRBM_COUNT"]) / d, 1) if acc.get("GRBM_COUNT") else None)
PY
}
PARGS="synth4m_4096 4 upd" run w256 PROBE_M=256
PARGS="synth4m_4096 4 upd" run w1024 PROBE_M=1024
PARGS="synth4m_4096 1 upd" run f1024 PROBE_M=1024
PARGS="synth1m_256 1 upd" run s256 A=1
