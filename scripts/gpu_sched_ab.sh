#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for r in 1 2 3; do
for lib in build_exp/libapus_a_memclause.so build_exp/libapus_z_base.so; do
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/kbench.py --rounds 10 --only wave_walk_checksum > gpurun_out/ab_$r.json 2>gpurun_out/ab_err.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$r.json')); print('$lib', round(d['wave_walk_checksum']['ms_median'],4))"
done
done
