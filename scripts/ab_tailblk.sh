#!/bin/bash
# segment kernel: 16-group tail blocks on the counter path (product) vs none (build_exp/libapus_notb.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 400 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_full_size.py tests/test_gpu_parity.py -k "partial_last_block or c4_one_gpu or c5 or commit" > gpurun_out/tb_pytest.log 2>&1 || { tail -20 gpurun_out/tb_pytest.log; exit 1; }
tail -2 gpurun_out/tb_pytest.log
for r in 1 2; do
  echo "#### C5 shape, round $r"
  ONLY=short_walk_checksum ROUNDS=8 KB_ARGS="--groups 8388608 --replicas 7 --entries 16 --history 16 --ring 8192 --cid-mix" bash scripts/exp_run.sh || exit 1
  echo "#### C4 1-GPU shape 2^22, round $r"
  ONLY=short_walk_checksum ROUNDS=8 KB_ARGS="--groups 4194304 --replicas 5 --entries 16 --history 2 --ring 2448" bash scripts/exp_run.sh || exit 1
done
