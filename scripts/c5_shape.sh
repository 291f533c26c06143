#!/bin/bash
# the C5 walk against the C4 1-GPU shape: which difference costs (seq_probe.py
# --rings 2, one process per shape, every shape twice)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/c5shape
for round in 1 2; do
  for s in c5 c5_nolit c5_dense c4_sparse c4_1gpu_2e23; do
    echo "== round $round $s"
    timeout -k 10 180 python3 scripts/seq_probe.py --rings 2 --n 6 --shape $s 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
