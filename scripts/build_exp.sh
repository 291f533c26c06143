#!/bin/bash
# Experimental builds of libapus_gpu (kernel A/B timing only; never the product):
#   build_exp/libapus_<name>.so compiled with -D<macro>; load with APUS_GPU_LIB=...
# The APUS_EXP_* branches were taken out of the product sources (round 5); to
# rebuild an experiment, first restore them in a scratch checkout with
#   git apply profiles/r04/exp_knobs.diff (round 4) or profiles/r05/exp_knobs.diff (round 5)
set -eu
cd "$(dirname "$0")/.."
mkdir -p build_exp
SRC=rdma-paxos_amd/csrc
build() {
  local name=$1; shift
  local objs=""
  for f in $(cd $SRC && ls *.hip | sed 's/\.hip$//'); do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c $SRC/$f.hip -o build_exp/${name}_$f.o &
    objs="$objs build_exp/${name}_$f.o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_exp/libapus_$name.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  rm -f $objs
}
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  build "$name" $flags
done
