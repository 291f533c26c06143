#!/bin/bash
# Same-box A/B of append_kernel (round 4: a wrapping batch's two fast prefixes
# in one round trip) at the C2 shape (2^20 groups x 64 SEND messages of 64 B
# on 16-KiB rings) and the C5 shape (2^22 groups x R=7, 16 messages).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pass in 1 2; do
for lib in rdma-paxos_amd/libapus_gpu.so ${EXP_LIBS:-}; do
  n=$(basename $lib .so)
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 200 python3 scripts/kbench.py --rounds ${ROUNDS:-5} --only append \
    > gpurun_out/abap_${n}_c2_$pass.json 2>gpurun_out/abap_err.log || { tail -5 gpurun_out/abap_err.log; exit 1; }
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 200 python3 scripts/kbench.py --rounds ${ROUNDS:-5} --only append \
    --groups 4194304 --replicas 7 --entries 16 --ring 8192 --cid-mix \
    > gpurun_out/abap_${n}_c5_$pass.json 2>gpurun_out/abap_err.log || { tail -5 gpurun_out/abap_err.log; exit 1; }
  python3 - "$n" "$pass" <<'PY'
import json, sys
n, p = sys.argv[1], sys.argv[2]
for sh in ("c2", "c5"):
    d = json.load(open(f"gpurun_out/abap_{n}_{sh}_{p}.json"))
    print(n, sh, p, {k: round(v["ms_median"], 4) for k, v in d.items() if isinstance(v, dict) and "ms_median" in v})
PY
done
done
