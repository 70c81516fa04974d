# final tree: full GPU suite + smoke + default bench
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/gpu_final.sh || exit 1
