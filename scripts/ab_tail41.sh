#!/bin/bash
# Same-box A/B of the commit call's tail launch at the C4 1-GPU point (2^26
# groups x R=5, 16 entries on 2,448-B rings): the tail alone (median +
# pruning) and the walk + tail call, product library and EXP_LIBS builds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C41="--groups 67108864 --replicas 5 --entries 16 --ring 2448 --history 2"
for pass in 1 2; do
for lib in rdma-paxos_amd/libapus_gpu.so ${EXP_LIBS:-}; do
  n=$(basename $lib .so)
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 300 python3 scripts/kbench.py --rounds ${ROUNDS:-4} $C41 \
    --only ${ONLY:-tail,short_walk_checksum} > gpurun_out/ab41_${n}_$pass.json 2>gpurun_out/ab41_err.log \
    || { tail -5 gpurun_out/ab41_err.log; exit 1; }
  python3 - "$n" "$pass" <<'PY'
import json, sys
n, p = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/ab41_{n}_{p}.json"))
print(n, p, {k: round(v["ms_median"], 4) for k, v in d.items() if isinstance(v, dict) and "ms_median" in v})
PY
done
done
