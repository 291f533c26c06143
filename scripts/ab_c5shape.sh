#!/bin/bash
# the segment kernel at C5-like shapes: which of R=7, the configuration mix, the ring size costs time
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
K="timeout -k 10 200 python3 scripts/kbench.py --only short_walk_checksum --groups 8388608 --entries 16 --history 16 --rounds 6"
for r in 1 2; do
  for a in "--replicas 5 --ring 8192" "--replicas 7 --ring 8192" "--replicas 7 --ring 8192 --cid-mix" "--replicas 5 --ring 2448 --history 2"; do
    echo "== $a (round $r)"; $K $a 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
