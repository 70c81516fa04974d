# configs[4] N=4 window, update alone: HBM bytes (FETCH_SIZE) and TCC hits at M=256 vs M=1024
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/d9; mkdir -p $O
for m in 256 1024; do
  PROBE_M=$m timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$m -o run -- python3 scripts/strong_probe.py synth4m_4096 4 upd > $O/f$m.log 2>&1 || exit 1
  PROBE_M=$m timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/h$m -o run -- python3 scripts/strong_probe.py synth4m_4096 4 upd > $O/h$m.log 2>&1 || exit 1
  PROBE_M=$m timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/s$m -o run -- python3 scripts/strong_probe.py synth4m_4096 4 upd > $O/s$m.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for tag in ("f256","f1024","h256","h1024","s256","s1024"):
    fs = glob.glob(f"gpurun_out/d9/{tag}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(list)
    for f in fs:
        for r in csv.DictReader(open(f)):
            if "k_update_mixed" in r.get("Kernel_Name", ""):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(tag, {k: (len(v), sum(v) / len(v)) for k, v in acc.items()})
PY
