#!/bin/bash
# NC build implementations: parity (quad, lane, 16-lane segments), then C2 / C3 / C5 timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_records.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "${PYK:-nc_build or records or last_idx or vote_rank}" > gpurun_out/ncseg.log 2>&1
rc=$?; tail -3 gpurun_out/ncseg.log; [ $rc -eq 0 ] || exit $rc
for cfg in "" "--groups 262144 --replicas 5 --payload 64 --payload-max 4096 --ring 344064" \
           "--groups 4194304 --replicas 7 --entries 16 --cid-mix"; do
  timeout -k 10 300 python3 scripts/kbench.py --rounds 4 $cfg --only ${ONLY:-nc_build,nc_build_quad,nc_build_lane,last_idx_term,last_idx_term_lane} \
    > gpurun_out/kb_nc.json 2>gpurun_out/kb_nc.err || { tail -3 gpurun_out/kb_nc.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/kb_nc.json'))
print(d['groups'], {k: round(v['ms_median'], 3) for k, v in d.items() if isinstance(v, dict)})"
done
