#!/bin/bash
# Named GPU plans for gpurun (each a list of scripts/gpu_steps.py steps):
#   bash scripts/gpu_plan.sh PLAN
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="python3 scripts/gpu_steps.py"
SEG="--groups 4194304 --replicas 5 --entries 16 --history 2 --ring 2448"
SQ="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY"
case "${1:-round}" in
  round)   # the round-end evidence: suite, smoke, C2 bench + profile, C3 bench + profile
    $S "pytest_gpu@900=pytest" "smoke@300=smoke" "bench_c2=bench:" "prof_c2=prof:--no-cpu-baseline" \
       "bench_c3=bench:--workload c3 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c3=prof:--workload c3 --steps 20 --warmup 3 --no-cpu-baseline" ;;
  nc)      # NC determinants from the walk, validation on leader determinants, fused step A/B
    $S "pytest_nc=pytest:tests/test_gpu_parity.py -k 'commit_walk_checksum_median or malformed or validate_and_nc'" \
       "kb_c2_fuse2=kb:--only step_fused,step_separate,wave_walk_checksum --rounds 12" \
       "bench_c2_fused=bench:--no-cpu-baseline" "bench_c2_sep=bench:--no-cpu-baseline --separate" \
       "bench_c3_fused=bench:--workload c3 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c3_sep=bench:--workload c3 --steps 20 --warmup 3 --no-cpu-baseline --separate" ;;
  pmc)     # instruction mix + traffic: short-walk kernel (C4 1-GPU shape) and wave kernel (C2)
    $S "avail@60=avail" \
       "seg_sq=pmc:$SQ|kbench.py --only short_walk_checksum $SEG --rounds 2" \
       "seg_fetch=pmc:FETCH_SIZE|kbench.py --only short_walk_checksum $SEG --rounds 2" \
       "seg_write=pmc:WRITE_SIZE|kbench.py --only short_walk_checksum $SEG --rounds 2" \
       "wav_sq=pmc:$SQ|kbench.py --only wave_walk_checksum --rounds 2" ;;
  *) echo "unknown plan $1"; exit 2 ;;
esac
