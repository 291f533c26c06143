#!/bin/bash
# same-box A/B of the lane/wave kernels whose grids are capped at the resident blocks: product vs $EXP_LIBS, twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
C5="--groups 4194304 --replicas 7 --entries 16 --cid-mix"
C3="--groups 262144 --replicas 5 --entries 64 --payload 64 --payload-max 4096 --ring 344064 --history 16"
for r in 1 2; do
  ONLY=append,apply,config_scan,log_adjust KB_ARGS="--rounds 6" bash scripts/exp_run.sh || exit 1
  ONLY=append,apply,config_scan,log_adjust KB_ARGS="$C5 --rounds 6" bash scripts/exp_run.sh || exit 1
  ONLY=validate KB_ARGS="$C3 --rounds 6" bash scripts/exp_run.sh || exit 1
done
