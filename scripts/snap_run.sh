#!/bin/bash
# Dev tool: run a GPU script on a frozen copy of the tree (.snap/, sent with the tree)
# so that the working tree can change while gpurun waits for a box. Retries only
# when gpurun ran nothing (no box free / transient preparation failure). The copy is
# removed when the call ends, so no later call (the driver's round-end runs included)
# ships it or a stale library inside it.
# usage: scripts/snap_run.sh SCRIPT TIMEOUT LOG
set -u
script=$1; tmo=$2; log=$3
cd /root/repo
rm -rf .snap && mkdir .snap
tar --exclude ./.git --exclude ./.snap --exclude ./gpurun_out --exclude ./ab --exclude './ab6/*.objs' --exclude '__pycache__' --exclude '*.pyc' \
  -cf - . | tar -xf - -C .snap
trap 'rm -rf /root/repo/.snap' EXIT
cmd="export OUTROOT=\$GRAFT_REPO_ROOT/gpurun_out; cd .snap && export GRAFT_REPO_ROOT=\$PWD && bash $script"
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$tmo" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "no free box right now\|stopped responding while being prepared\|taken away by the GPU service\|backing off" "$log"; then
    if ! grep -q "status=ok\|status=fail\|status=error" "$log"; then sleep 120; continue; fi
  fi
  exit $rc
done
exit 3
