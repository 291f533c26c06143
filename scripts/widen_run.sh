#!/bin/bash
# Per-kernel timings at the other BASELINE configs (one process each, every
# GPU step under its own time limit, stop at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 limit=$2; shift 2
  echo "== $name"; date +%T
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
for s in ${STEPS:-kb_c2 kb_c5}; do
  case $s in
    t_append) run t_append 300 python -u -m pytest tests/test_append.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
    kb_c2) run kb_c2 300 python scripts/kbench.py --rounds 5 ${KB2:-} ;;
    kb_app) run kb_app 300 python scripts/kbench.py --rounds 5 --only append,persist --ring 32768 ;;
    kb_c3) run kb_c3 400 python scripts/kbench.py --rounds 3 --groups 524288 --replicas 5 --payload 64 --payload-max 4096 --ring 272960 --history-max 64 --only wave_walk_checksum,wave_walk,var_walk_checksum,var_walk,median,prune,nc_build_quad,validate,validate_lead,last_idx_term ;;
    kb_rec) run kb_rec 300 python scripts/kbench.py --rounds 5 --only records_store,records_load,records_store_lane,records_load_lane ;;
    kb_c5) run kb_c5 300 python scripts/kbench.py --rounds 5 --groups 4194304 --replicas 7 --entries 16 --ring 8192 --cid-mix --only vote_tally,vote_rank,last_idx_term,median,prune,wave_walk_checksum,short_walk_checksum,apply,config_scan,nc_build,nc_build_quad,lr_completion,log_adjust ${KB5:-} ;;
    kb_lr) run kb_lr 300 python scripts/kbench.py --rounds 5 --only lr_completion,log_adjust ;;
    kb_lr5) run kb_lr5 300 python scripts/kbench.py --rounds 5 --groups 4194304 --replicas 7 --entries 16 --ring 8192 --cid-mix --only lr_completion,log_adjust ;;
    t_lr) run t_lr 300 python -u -m pytest tests/test_lr_step.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    bench_c4) run bench_c4 600 python bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline ;;
  esac
done
echo "== done"
