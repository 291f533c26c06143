#!/bin/bash
# the commit tail launch: parity of the product and of build_exp/libapus_taildyn.so, then their steps at C2 and the C4 1-GPU point
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="python3 scripts/gpu_steps.py"
T="tests/test_gpu_parity.py -k commit"
$S "pytest_tail@600=pytest:$T" || exit 1
APUS_GPU_LIB=$PWD/build_exp/libapus_taildyn.so $S "pytest_taildyn@600=pytest:$T" || exit 1
for r in 1 2; do
  $S "b41_$r=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" "b2_$r=bench:--no-cpu-baseline" || exit 1
  APUS_GPU_LIB=$PWD/build_exp/libapus_taildyn.so $S "b41d_$r=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" "b2d_$r=bench:--no-cpu-baseline" || exit 1
done
