#!/bin/bash
# append / persist: GPU parity, then kbench timings (C2 shape)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_append.py tests/test_apply.py > gpurun_out/append_parity.log 2>&1
rc=$?; tail -3 gpurun_out/append_parity.log; [ $rc -ne 0 ] && exit $rc
for lib in rdma-paxos_amd/libapus_gpu.so build_exp/libapus_*.so; do
  [ -f "$lib" ] || continue
  echo "== $lib"
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 200 python scripts/kbench.py --rounds 6 --only append,persist ${KB_ARGS:-} \
    > gpurun_out/kb_append_$(basename $lib .so).log 2>&1
  rc=$?; grep -A3 '"append"\|"persist"' gpurun_out/kb_append_$(basename $lib .so).log; [ $rc -ne 0 ] && exit $rc
done
exit 0
