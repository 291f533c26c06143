#!/bin/bash
# same-box A/B of the commit walks at the batch shapes that take the block counter (DYN): product vs $EXP_LIBS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SEG="--groups 4194304 --replicas 5 --entries 16 --history 2 --ring 2448"
for r in 1 2; do
  ONLY=wave_walk_checksum,wave_walk bash scripts/exp_run.sh || exit 1
  ONLY=wave_walk_checksum KB_ARGS="--groups 8388608 --replicas 5 --rounds 4" bash scripts/exp_run.sh || exit 1
  ONLY=short_walk_checksum,short_walk KB_ARGS="$SEG" bash scripts/exp_run.sh || exit 1
done
