#!/bin/bash
# Same-box A/B of the commit call's tail launch (round 4): C5 shape (2^23
# groups x R=7, 16 entries, configuration mix) failover cases and the C2 tail,
# for the product library and each experiment build given in EXP_LIBS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C5="--groups 8388608 --replicas 7 --entries 16 --ring 8192 --cid-mix"
for pass in 1 2; do
for lib in rdma-paxos_amd/libapus_gpu.so ${EXP_LIBS:-}; do
  n=$(basename $lib .so)
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 300 python3 scripts/kbench.py --rounds ${ROUNDS:-6} $C5 \
    --only ${ONLY5:-tail,fail_tail,tail_with_fail,short_step_fused,short_step_calls,vote_tally,vote_rank} \
    > gpurun_out/abt_${n}_c5_$pass.json 2>gpurun_out/abt_err.log || { tail -5 gpurun_out/abt_err.log; exit 1; }
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/kbench.py --rounds ${ROUNDS:-6} \
    --only ${ONLY2:-tail,step_fused,wave_walk_checksum} > gpurun_out/abt_${n}_c2_$pass.json 2>gpurun_out/abt_err.log \
    || { tail -5 gpurun_out/abt_err.log; exit 1; }
  python3 - "$n" "$pass" <<'PY'
import json, sys
n, p = sys.argv[1], sys.argv[2]
for sh in ("c5", "c2"):
    d = json.load(open(f"gpurun_out/abt_{n}_{sh}_{p}.json"))
    print(n, sh, p, {k: round(v["ms_median"], 4) for k, v in d.items() if isinstance(v, dict) and "ms_median" in v})
PY
done
done
