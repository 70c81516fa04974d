# round-3 check: full GPU suite + smoke + default bench (scripts/gpu_final.sh), then the Kardam plans
set -u
bash scripts/gpu_final.sh || exit 1
TAG=r03k bash scripts/gpu_kardam_plans.sh
