#!/bin/bash
# PMC passes + kernel trace of the commit kernel (one counter group per pass;
# never combined with --sys-trace / runtime traces).  Output: gpurun_out/prof/*
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
KB="python3 scripts/kbench.py --rounds ${ROUNDS:-3} --only ${ONLY:-wave_walk_checksum} ${KB_ARGS:-}"
run() {
  local name=$1; shift
  echo "== $name"; date +%T
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- $KB > $OUT/$name.log 2>&1
  local rc=$?; echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run trace --kernel-trace --stats
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY
run sq2 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run grbm --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum
python3 scripts/parse_pmc.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
