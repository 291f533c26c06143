#!/bin/bash
# same-box A/B of the scalar drop-ins: the product library and an experiment build
set -u
cd "$(dirname "$0")/.."
for round in 1 2; do
  for lib in rdma-paxos_amd/libapus_gpu.so build_exp/libapus_qmap.so; do
    echo "== round $round $lib"
    APUS_GPU_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/scalar_latency.py --calls 3000 || exit $?
  done
done
