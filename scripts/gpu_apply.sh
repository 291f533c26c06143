#!/bin/bash
# apply / config scan: GPU parity, then C5 timings against build_exp/ libraries
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_apply.py > gpurun_out/apply_parity.log 2>&1
rc=$?; tail -2 gpurun_out/apply_parity.log; [ $rc -ne 0 ] && exit $rc
for lib in rdma-paxos_amd/libapus_gpu.so build_exp/libapus_*.so; do
  [ -f "$lib" ] || continue
  echo "== $lib"
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 200 python scripts/kbench.py --rounds 5 --groups 4194304 --replicas 7 \
    --entries 16 --ring 8192 --cid-mix --only apply,config_scan > gpurun_out/kb_apply_c5_$(basename $lib .so).log 2>&1 || exit $?
  grep -A1 '"apply"\|"config_scan"' gpurun_out/kb_apply_c5_$(basename $lib .so).log | grep -v "^--"
done
