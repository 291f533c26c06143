#!/bin/bash
# same-box A/B of the commit walks: product vs $EXP_LIBS, three rounds (C2 wave kernel; C4 shard shape when AB_C4=1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2 3; do
  ONLY=wave_walk_checksum,wave_walk bash scripts/exp_run.sh || exit 1
  if [ "${AB_C4:-0}" = 1 ]; then
    ONLY=wave_walk_checksum KB_ARGS="--groups 8388608 --replicas 5 --rounds 4" bash scripts/exp_run.sh || exit 1
  fi
done
