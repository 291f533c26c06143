#!/bin/bash
# kbench cases ($ONLY) at C2 and C5 shapes (CFGS overrides), one summary line per shape
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra SHAPES <<< "${CFGS:- ;--groups 4194304 --replicas 7 --entries 16 --cid-mix}"
for cfg in "${SHAPES[@]}"; do
  timeout -k 10 300 python3 scripts/kbench.py --rounds ${ROUNDS:-5} $cfg --only $ONLY > gpurun_out/kb.json 2>gpurun_out/kb.err \
    || { tail -3 gpurun_out/kb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/kb.json'))
print(d['groups'], {k: round(v['ms_median'], 3) for k, v in d.items() if isinstance(v, dict)})"
done
