#!/bin/bash
# C5 step: one commit call with APUS_COMMIT_LAST_IT vs --split (apus_last_idx_term_batch), at 3 and 20 steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="timeout -k 10 240 python3 bench.py --workload c5 --no-cpu-baseline"
for r in 1 2; do
  for a in "--steps 20 --warmup 3" "--steps 3 --warmup 1" "--steps 20 --warmup 3 --split"; do
    echo "== $a (round $r)"
    $B $a | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['roofline']['kernel'], round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), 'step', round(d['ms_per_step'],4))" || exit 1
  done
done
