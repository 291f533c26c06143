#!/bin/bash
# Same-box A/B of validate_kernel at the C3 wave (2^19 groups, 4 followers x 64
# determinants, ring sized for the batch): product library vs EXP_LIBS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C3="--groups 524288 --replicas 5 --entries 64 --payload 64 --payload-max 4096 --ring 272960 --history 16 --history-max 64"
for pass in 1 2; do
for lib in rdma-paxos_amd/libapus_gpu.so ${EXP_LIBS:-}; do
  n=$(basename $lib .so)
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 300 python3 scripts/kbench.py --rounds ${ROUNDS:-8} $C3 \
    --only ${ONLY3:-validate,validate_lead} > gpurun_out/abv_${n}_$pass.json 2>gpurun_out/abv_err.log || { tail -5 gpurun_out/abv_err.log; exit 1; }
  python3 - "$n" "$pass" <<'PY'
import json, sys
n, p = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/abv_{n}_{p}.json"))
print(n, "c3", p, {k: (round(v["ms_median"], 4), round(v.get("GBps_alg", 0) / 8000, 3)) for k, v in d.items() if isinstance(v, dict) and "ms_median" in v})
PY
done
done
