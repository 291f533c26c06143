#!/bin/bash
# nc_build quad kernel: parity, then timings against the lane kernel (C2, C3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_log_image.py tests/test_golden.py tests/test_full_size.py \
  -k "nc_build or validate or golden or gpu_matches or full_size or log_image" > gpurun_out/ncq_parity.log 2>&1
rc=$?; tail -3 gpurun_out/ncq_parity.log; [ $rc -ne 0 ] && exit $rc
for lib in rdma-paxos_amd/libapus_gpu.so build_exp/libapus_*.so; do
  [ -f "$lib" ] || continue
  echo "== $lib"
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 200 python scripts/kbench.py --rounds 6 --only nc_build,validate \
    > gpurun_out/kb_ncq_c2_$(basename $lib .so).log 2>&1 || exit $?
  grep -A1 '"nc_build"\|"validate"' gpurun_out/kb_ncq_c2_$(basename $lib .so).log | grep -v "^--"
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 300 python scripts/kbench.py --rounds 3 --groups 262144 --replicas 5 \
    --payload 64 --payload-max 4096 --ring 344064 --only nc_build,validate > gpurun_out/kb_ncq_c3_$(basename $lib .so).log 2>&1 || exit $?
  grep -A1 '"nc_build"\|"validate"' gpurun_out/kb_ncq_c3_$(basename $lib .so).log | grep -v "^--"
done
