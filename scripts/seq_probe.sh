#!/bin/bash
# scripts/seq_probe.py under a kernel trace, for the product library and each
# EXP_LIBS build; prints one JSON line per library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in rdma-paxos_amd/libapus_gpu.so ${EXP_LIBS:-}; do
  n=$(basename $lib .so)
  d=gpurun_out/seq_$n
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- \
    python3 scripts/seq_probe.py --n ${N:-20} > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "$n $(python3 scripts/seq_probe.py --trace $d --n ${N:-20})"
done
