#!/bin/bash
# commit kernel experiments: parity of every build_exp library on the commit tests, then C2 / C3 timings, twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in build_exp/libapus_*.so; do
  n=$(basename $lib .so)
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -m gpu tests/test_gpu_parity.py tests/test_golden.py -k "commit or vectors" > gpurun_out/cab_$n.log 2>&1
  rc=$?; echo "== $n parity: $(tail -1 gpurun_out/cab_$n.log)"; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
  ROUNDS=8 bash scripts/exp_run.sh || exit 1
  ROUNDS=4 ONLY=var_walk_checksum KB_ARGS="--groups 262144 --replicas 5 --payload 64 --payload-max 4096 --ring 344064" bash scripts/exp_run.sh || exit 1
done
