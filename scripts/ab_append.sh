#!/bin/bash
# same-box A/B of the append kernels: product vs $EXP_LIBS at C2 (and C5), three rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
C5="--groups 4194304 --replicas 7 --entries 16 --cid-mix"
for r in 1 2 3; do
  ONLY=append KB_ARGS="--rounds 6" bash scripts/exp_run.sh || exit 1
  if [ "${AB_C5:-0}" = 1 ]; then ONLY=append KB_ARGS="$C5 --rounds 6" bash scripts/exp_run.sh || exit 1; fi
done
