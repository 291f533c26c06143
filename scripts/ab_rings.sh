#!/bin/bash
# same-box A/B of the C5 segment walk over three ring allocations (seq_probe.py --rings 3):
# the product library against build_exp/libapus_$1.so, two processes each
set -u
cd "$(dirname "$0")/.."
for round in 1 2; do
  for lib in rdma-paxos_amd/libapus_gpu.so build_exp/libapus_$1.so; do
    echo "== round $round $lib"
    APUS_GPU_LIB=$PWD/$lib timeout -k 10 150 python3 scripts/seq_probe.py --rings 3 --n 6 || exit $?
  done
done
