#!/bin/bash
# Time the commit kernel of each experimental build (scripts/build_exp.sh) + the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in rdma-paxos_amd/libapus_gpu.so ${EXP_LIBS:-build_exp/libapus_*.so}; do
  echo "== $lib"
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/kbench.py --rounds ${ROUNDS:-8} --only ${ONLY:-wave_walk_checksum,wave_walk} ${KB_ARGS:-} > gpurun_out/exp_$(basename $lib .so).json 2>gpurun_out/exp_err.log
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -5 gpurun_out/exp_err.log; exit $rc; fi
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/exp_$(basename $lib .so).json'))
print({k:(round(v['ms_median'],4) if isinstance(v,dict) else v) for k,v in d.items() if k not in ('wave_stats',)})"
done
