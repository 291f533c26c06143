#!/bin/bash
# quad walkers (nc_build, local idx/term): parity, then C5/C3 timings against the lane kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_log_image.py tests/test_golden.py \
  -k "nc_build or validate or golden or gpu_matches or vote_rank or log_image" > gpurun_out/ncq_parity.log 2>&1
rc=$?; tail -3 gpurun_out/ncq_parity.log; [ $rc -ne 0 ] && exit $rc
for lib in rdma-paxos_amd/libapus_gpu.so build_exp/libapus_*.so; do
  [ -f "$lib" ] || continue
  echo "== $lib"
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 200 python scripts/kbench.py --rounds 5 --groups 4194304 --replicas 7 \
    --entries 16 --ring 8192 --cid-mix --only last_idx_term,nc_build > gpurun_out/kb_ncq_c5_$(basename $lib .so).log 2>&1 || exit $?
  grep -A1 '"last_idx_term"\|"nc_build"' gpurun_out/kb_ncq_c5_$(basename $lib .so).log | grep -v "^--"
done
