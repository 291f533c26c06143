#!/bin/bash
# A/B of the commit kernel on one box: GPU parity of the commit path with the
# product build, then kbench of every build_exp/libapus_*.so and the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_streams.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:-} > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log
  if [ $rc -ne 0 ]; then grep -E "Error|error|assert" gpurun_out/ab_tests.log | head -20; exit $rc; fi
fi
for lib in ${LIBS:-rdma-paxos_amd/libapus_gpu.so build_exp/libapus_*.so}; do
  n=$(basename $lib .so)
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/kbench.py --rounds ${ROUNDS:-10} --only ${ONLY:-wave_walk_checksum,wave_walk} ${KB_ARGS:-} > gpurun_out/ab_$n.json 2>gpurun_out/ab_err.log
  rc=$?
  if [ $rc -ne 0 ]; then echo "$n rc=$rc"; tail -5 gpurun_out/ab_err.log; exit $rc; fi
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$n.json'))
print('$n', {k:(round(v['ms_median'],4) if isinstance(v,dict) else v) for k,v in d.items() if isinstance(v,dict) and 'ms_median' in v})"
done
