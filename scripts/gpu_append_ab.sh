#!/bin/bash
# append experiments: parity of every build (product + build_exp/), then kbench append timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in rdma-paxos_amd/libapus_gpu.so build_exp/libapus_*.so; do
  [ -f "$lib" ] || continue
  n=$(basename $lib .so)
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -m gpu tests/test_append.py tests/test_apply.py > gpurun_out/ab_parity_$n.log 2>&1
  rc=$?; echo "== $n parity: $(tail -1 gpurun_out/ab_parity_$n.log)"; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
for lib in rdma-paxos_amd/libapus_gpu.so build_exp/libapus_*.so; do
  n=$(basename $lib .so)
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 200 python scripts/kbench.py --rounds 6 --only append ${KB_ARGS:-} \
    > gpurun_out/kb_append_$n.log 2>&1
  rc=$?; echo "$n $(grep -A1 '"append"' gpurun_out/kb_append_$n.log | tail -1)"; [ $rc -ne 0 ] && exit $rc
done
done
exit 0
