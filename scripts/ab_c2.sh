#!/bin/bash
# same-box A/B of the C2 wave walk: product vs $EXP_LIBS, three rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2 3; do
  ONLY=wave_walk_checksum,wave_walk bash scripts/exp_run.sh || exit 1
done
