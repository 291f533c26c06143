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
  walk)    # commit walks (wave + segment kernels): parity everywhere the walk runs, then timings
    $S "pytest_walk@900=pytest:tests/test_gpu_parity.py tests/test_full_size.py tests/test_log_image.py tests/test_golden.py tests/test_append.py tests/test_gpu_streams.py" \
       "kb_c2_walk=kb:--only wave_walk_checksum,wave_walk --rounds 12" \
       "kb_seg_2448_g22=kb:--only short_walk_checksum,short_walk $SEG --rounds 8" \
       "kb_seg_16k_g22=kb:--only short_walk_checksum,short_walk --groups 4194304 --replicas 5 --entries 16 --history 16 --ring 16384 --rounds 8" \
       "bench_c2=bench:--no-cpu-baseline" \
       "bench_c4_1gpu=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" ;;
  c4)      # the C4 per-GPU shard: time, HBM traffic and address-translation counters (C2 beside it)
    TLB="TCP_UTCL1_TRANSLATION_MISS_sum,TCP_UTCL1_TRANSLATION_HIT_sum,TCP_UTCL1_REQUEST_sum,GRBM_UTCL2_BUSY,GRBM_GUI_ACTIVE"
    B4="bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline"
    B2="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
    $S "bench_c4=bench:--workload c4 --steps 20 --warmup 3 --no-cpu-baseline" \
       "c4_fetch@240=pmc:FETCH_SIZE|$B4" "c4_write@240=pmc:WRITE_SIZE|$B4" "c4_tlb@240=pmc:$TLB|$B4" \
       "c2_tlb@240=pmc:$TLB|$B2" ;;
  exp)     # same-box A/B of the experimental builds in build_exp/ (scripts/build_exp.sh) against the product
    ONLY=wave_walk_checksum,wave_walk bash scripts/exp_run.sh && \
    ONLY=short_walk_checksum,short_walk KB_ARGS="$SEG" bash scripts/exp_run.sh && \
    ONLY=short_walk_checksum,short_walk KB_ARGS="--groups 4194304 --replicas 5 --entries 16 --history 16 --ring 16384" bash scripts/exp_run.sh && \
    ONLY=wave_walk_checksum,wave_walk bash scripts/exp_run.sh ;;
  exppmc)  # instruction mix of the product and each experimental build (short-walk kernel, C4 1-GPU shape)
    SQ2="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU"
    for lib in rdma-paxos_amd/libapus_gpu.so build_exp/libapus_*.so; do
      n=$(basename $lib .so)
      APUS_GPU_LIB=$PWD/$lib $S "pmc_seg_$n=pmc:$SQ2|kbench.py --only short_walk_checksum,short_walk $SEG --rounds 2" || exit 1
    done ;;
  walkexp) # the walk parity suite, then the same-box A/B of build_exp/ (the "exp" plan)
    $S "pytest_walk@900=pytest:tests/test_gpu_parity.py tests/test_full_size.py tests/test_log_image.py tests/test_golden.py tests/test_append.py" && \
    bash "$0" exp ;;
  expseg)  # same-box A/B of build_exp/ on the short-walk kernel only (C4 1-GPU shape)
    ONLY=short_walk_checksum,short_walk KB_ARGS="$SEG" bash scripts/exp_run.sh && \
    ONLY=short_walk_checksum,short_walk KB_ARGS="$SEG" bash scripts/exp_run.sh ;;
  ev1)     # round evidence 1: the suite, smoke, C2 and C3 benches with profiles and traffic passes
    $S "pytest_gpu@900=pytest" "smoke@300=smoke" "bench_c2=bench:" "prof_c2=prof:--no-cpu-baseline" \
       "pmc_c2_fetch@240=pmc:FETCH_SIZE|bench.py --no-cpu-baseline --steps 5 --warmup 1" \
       "pmc_c2_write@240=pmc:WRITE_SIZE|bench.py --no-cpu-baseline --steps 5 --warmup 1" \
       "bench_c3=bench:--workload c3 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c3=prof:--workload c3 --steps 20 --warmup 3 --no-cpu-baseline" \
       "pmc_c3_fetch@300=pmc:FETCH_SIZE|bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c3_write@300=pmc:WRITE_SIZE|bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1" ;;
  ev2)     # round evidence 2: the 64M-group batch on one GPU, the C4 shard (traffic, translation), scalar latency
    TLB="TCP_UTCL1_TRANSLATION_MISS_sum,TCP_UTCL1_TRANSLATION_HIT_sum,TCP_UTCL1_REQUEST_sum,GRBM_UTCL2_BUSY,GRBM_GUI_ACTIVE"
    $S "bench_c4_1gpu=bench:--workload c4_1gpu --steps 20 --warmup 3 --cpu-seconds 8" \
       "prof_c4_1gpu=prof:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" \
       "pmc_c41_fetch@300=pmc:FETCH_SIZE|bench.py --workload c4_1gpu --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c41_write@300=pmc:WRITE_SIZE|bench.py --workload c4_1gpu --no-cpu-baseline --steps 3 --warmup 1" \
       "bench_c4=bench:--workload c4 --steps 20 --warmup 3 --cpu-seconds 6" \
       "pmc_c4_fetch@300=pmc:FETCH_SIZE|bench.py --workload c4 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c4_write@300=pmc:WRITE_SIZE|bench.py --workload c4 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c4_tlb@300=pmc:$TLB|bench.py --workload c4 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c2_tlb@240=pmc:$TLB|bench.py --no-cpu-baseline --steps 3 --warmup 1" \
       "scalar=scalar:--calls 1000" ;;
  app)     # append: parity of both kernels, then C2 and C5 timings (product and build_exp/libapus_prev.so)
    C5="--groups 4194304 --replicas 7 --entries 16 --cid-mix"
    $S "pytest_append@600=pytest:tests/test_append.py tests/test_log_image.py" && \
    EXP_LIBS=build_exp/libapus_prev.so ONLY=append,append_per_group KB_ARGS="--rounds 10" bash scripts/exp_run.sh && \
    EXP_LIBS=build_exp/libapus_prev.so ONLY=append,append_per_group KB_ARGS="$C5 --rounds 10" bash scripts/exp_run.sh && \
    EXP_LIBS=build_exp/libapus_prev.so ONLY=append,append_per_group KB_ARGS="$C5 --rounds 10" bash scripts/exp_run.sh ;;
  appab)   # append A/B only: product vs build_exp/libapus_prev.so at C2 and C5, then phases (build_exp/libapus_phases.so)
    C5="--groups 4194304 --replicas 7 --entries 16 --cid-mix"
    $S "pytest_append@600=pytest:tests/test_append.py" && \
    EXP_LIBS=build_exp/libapus_prev.so ONLY=append,append_per_group KB_ARGS="--rounds 10" bash scripts/exp_run.sh && \
    EXP_LIBS=build_exp/libapus_prev.so ONLY=append,append_per_group KB_ARGS="$C5 --rounds 10" bash scripts/exp_run.sh && \
    EXP_LIBS=build_exp/libapus_prev.so ONLY=append,append_per_group KB_ARGS="--rounds 10" bash scripts/exp_run.sh && \
    APUS_GPU_LIB=$PWD/build_exp/libapus_phases.so timeout -k 10 120 python3 scripts/phase_probe.py --append ;;
  tail)    # the one-launch commit tail: parity, then the step A/B against the round's previous build (split step)
    P="APUS_GPU_LIB=$PWD/build_exp/libapus_prev.so"
    $S "pytest_tail@900=pytest:tests/test_gpu_parity.py tests/test_full_size.py tests/test_gpu_streams.py tests/test_log_image.py tests/test_golden.py" \
       "smoke@300=smoke" "bench_c2=bench:--no-cpu-baseline" && \
    env $P $S "bench_c2_prev=bench:--no-cpu-baseline --split" && \
    $S "bench_c2_b=bench:--no-cpu-baseline" "bench_c41=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" && \
    env $P $S "bench_c41_prev=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline --split" && \
    $S "prof_c2=prof:--no-cpu-baseline" "prof_c41=prof:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" ;;
  tail2)   # tail kernel rework: parity of the commit / pruning paths, then C2 and C4 1-GPU steps
    $S "pytest_t2@900=pytest:tests/test_gpu_parity.py -k 'commit or prune or vote_rank' tests/test_full_size.py" \
       "bench_c2=bench:--no-cpu-baseline" "bench_c41=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" \
       "prof_c2=prof:--no-cpu-baseline --steps 20" ;;
  seg3)    # short-walk kernel rework (one exclusion pass, SGPR piece offsets) + the tail rework: parity, then A/B
    P="APUS_GPU_LIB=$PWD/build_exp/libapus_prev.so"
    $S "pytest_s3@900=pytest:tests/test_gpu_parity.py tests/test_full_size.py tests/test_log_image.py tests/test_golden.py" && \
    ONLY=short_walk_checksum,short_walk KB_ARGS="$SEG" EXP_LIBS=build_exp/libapus_prev.so bash scripts/exp_run.sh && \
    $S "bench_c41=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" "bench_c2=bench:--no-cpu-baseline" && \
    env $P $S "bench_c41_prev=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline --split" && \
    ONLY=short_walk_checksum,short_walk KB_ARGS="$SEG" EXP_LIBS=build_exp/libapus_prev.so bash scripts/exp_run.sh && \
    $S "prof_c41=prof:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" ;;
  tail3)   # LDS-staged tail: the commit / pruning parity, then C2 and C4 1-GPU steps against the lane-per-group tail
    $S "pytest_t3@900=pytest:tests/test_gpu_parity.py tests/test_full_size.py tests/test_log_image.py tests/test_golden.py tests/test_gpu_streams.py" \
       "bench_c2=bench:--no-cpu-baseline" "bench_c41=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" \
       "prof_c2=prof:--no-cpu-baseline --steps 20" "prof_c41=prof:--workload c4_1gpu --steps 10 --warmup 2 --no-cpu-baseline" && \
    env APUS_GPU_LIB=$PWD/build_exp/libapus_lanetail.so $S "bench_c2_lane=bench:--no-cpu-baseline" \
       "bench_c41_lane=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" ;;
  ev3)     # round evidence 3: the suite, smoke, every single-GPU workload with its rocprof summary
    $S "pytest_gpu@900=pytest" "smoke@300=smoke" "bench_c2=bench:" "prof_c2=prof:--no-cpu-baseline" \
       "bench_c2_split=bench:--no-cpu-baseline --split" \
       "bench_c3=bench:--workload c3 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c3=prof:--workload c3 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c4=bench:--workload c4 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c4=prof:--workload c4 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c4_1gpu=bench:--workload c4_1gpu --steps 20 --warmup 3 --cpu-seconds 8" \
       "prof_c4_1gpu=prof:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" ;;
  c3ab)    # the C3 hop walk and the C2 wave walk: product vs the round-2 build (build_exp/libapus_r2.so), twice
    C3="--groups 262144 --replicas 5 --entries 64 --payload 64 --payload-max 4096 --ring 344064 --history 16"
    for r in 1 2; do
      ONLY=var_walk_checksum,var_walk KB_ARGS="$C3" EXP_LIBS=build_exp/libapus_r2.so bash scripts/exp_run.sh || exit 1
      ONLY=wave_walk_checksum,wave_walk EXP_LIBS=build_exp/libapus_r2.so bash scripts/exp_run.sh || exit 1
    done ;;
  win)     # wave-kernel window / occupancy variants (build_exp/libapus_w*.so) against the product at C2, twice
    for r in 1 2; do
      ONLY=wave_walk_checksum,wave_walk EXP_LIBS="build_exp/libapus_w7168.so build_exp/libapus_w6144.so" bash scripts/exp_run.sh || exit 1
    done ;;
  tail4)   # the tail with branch-free input loads: C2 / C4 1-GPU steps and their rocprof summaries
    $S "bench_c2=bench:--no-cpu-baseline" "prof_c2=prof:--no-cpu-baseline" \
       "bench_c41=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" \
       "prof_c41=prof:--workload c4_1gpu --steps 10 --warmup 2 --no-cpu-baseline" "bench_c2_b=bench:--no-cpu-baseline" && \
    STEPS="kb_c2 kb_c3 kb_c5" bash scripts/widen_run.sh ;;
  segab)   # short-walk kernel: walk parity, then product vs $EXP_LIBS at the C4 1-GPU shape (2^22 groups), twice
    $S "pytest_seg@600=pytest:tests/test_gpu_parity.py tests/test_golden.py tests/test_log_image.py" && \
    for r in 1 2; do
      ONLY=short_walk_checksum,short_walk KB_ARGS="$SEG" bash scripts/exp_run.sh || exit 1
    done && $S "bench_c41=bench:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" ;;
  waveab)  # wave kernel (C2) and hop walk (C3): walk parity, then product vs $EXP_LIBS, twice
    C3="--groups 262144 --replicas 5 --entries 64 --payload 64 --payload-max 4096 --ring 344064 --history 16"
    $S "pytest_walk@600=pytest:tests/test_gpu_parity.py tests/test_golden.py tests/test_log_image.py" && \
    for r in 1 2; do
      ONLY=wave_walk_checksum,wave_walk bash scripts/exp_run.sh || exit 1
      ONLY=var_walk_checksum,var_walk KB_ARGS="$C3" bash scripts/exp_run.sh || exit 1
    done && $S "bench_c2=bench:--no-cpu-baseline" ;;
  appprof) # append at C2: cycle phases (build_exp/libapus_phases.so), HBM traffic and instruction mix
    SQA="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY"
    APUS_GPU_LIB=$PWD/build_exp/libapus_phases.so timeout -k 10 120 python3 scripts/phase_probe.py --append > gpurun_out/app_phases.json && \
    $S "app_fetch=pmc:FETCH_SIZE|kbench.py --only append --rounds 2" "app_write=pmc:WRITE_SIZE|kbench.py --only append --rounds 2" \
       "app_sq=pmc:$SQA|kbench.py --only append --rounds 2" ;;
  appab2)  # append + records: parity, then product vs $EXP_LIBS at C2 and C5 (append) and C2 (records), twice
    C5="--groups 4194304 --replicas 7 --entries 16 --cid-mix"
    $S "pytest_app@600=pytest:tests/test_append.py tests/test_log_image.py tests/test_records.py" && \
    for r in 1 2; do
      ONLY=append KB_ARGS="--rounds 8" bash scripts/exp_run.sh || exit 1
      ONLY=append KB_ARGS="$C5 --rounds 8" bash scripts/exp_run.sh || exit 1
      ONLY=records_store,records_load KB_ARGS="--rounds 8" bash scripts/exp_run.sh || exit 1
    done ;;
  ev5)     # round evidence 5 (end of round 3): suite, smoke, every workload with its rocprof summary, C5 traffic
    $S "pytest_gpu@900=pytest" "smoke@300=smoke" "bench_c2=bench:" "prof_c2=prof:--no-cpu-baseline" \
       "bench_c3=bench:--workload c3 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c3=prof:--workload c3 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c4=bench:--workload c4 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c4=prof:--workload c4 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c4_1gpu=bench:--workload c4_1gpu --steps 20 --warmup 3 --cpu-seconds 8" \
       "prof_c4_1gpu=prof:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c5=bench:--workload c5 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c5=prof:--workload c5 --steps 20 --warmup 3 --no-cpu-baseline" \
       "pmc_c5_fetch@300=pmc:FETCH_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c5_write@300=pmc:WRITE_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" ;;
  ev6)     # round evidence 6 (final code of round 3): ev5 plus the C2 traffic passes
    bash "$0" ev5 && \
    $S "pmc_c2_fetch@240=pmc:FETCH_SIZE|bench.py --no-cpu-baseline --steps 5 --warmup 1" \
       "pmc_c2_write@240=pmc:WRITE_SIZE|bench.py --no-cpu-baseline --steps 5 --warmup 1" ;;
  ev7)     # round 4 evidence, call 1: the suite, smoke, C2 and C3 (one wave and the whole batch) with
           # rocprof summaries and traffic passes
    $S "pytest_gpu@900=pytest" "smoke@300=smoke" "bench_c2=bench:" "prof_c2=prof:--no-cpu-baseline" \
       "pmc_c2_fetch@240=pmc:FETCH_SIZE|bench.py --no-cpu-baseline --steps 5 --warmup 1" \
       "pmc_c2_write@240=pmc:WRITE_SIZE|bench.py --no-cpu-baseline --steps 5 --warmup 1" \
       "bench_c3=bench:--workload c3 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c3=prof:--workload c3 --steps 20 --warmup 3 --no-cpu-baseline" \
       "pmc_c3_fetch@300=pmc:FETCH_SIZE|bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c3_write@300=pmc:WRITE_SIZE|bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1" \
       "bench_c3_full@900=bench:--workload c3_full --steps 2 --warmup 1 --no-cpu-baseline" ;;
  ev8)     # round 4 evidence, call 2: C4 (shard and the 64M-group batch on one GPU) and C5, rocprof and traffic
    $S "bench_c4=bench:--workload c4 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c4=prof:--workload c4 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c4_1gpu=bench:--workload c4_1gpu --steps 20 --warmup 3 --cpu-seconds 8" \
       "prof_c4_1gpu=prof:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c5=bench:--workload c5 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c5=prof:--workload c5 --steps 20 --warmup 3 --no-cpu-baseline" \
       "pmc_c5_fetch@300=pmc:FETCH_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c5_write@300=pmc:WRITE_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_app_fetch=pmc:FETCH_SIZE|kbench.py --only append --rounds 2" \
       "pmc_app_write=pmc:WRITE_SIZE|kbench.py --only append --rounds 2" \
       "scalar=scalar:--calls 1000" ;;
  tailpmc) # the tail's request counts against the segment walk's (C4 1-GPU shape at 2^22 groups)
    K="kbench.py --only tail,short_walk_checksum $SEG --rounds 2"
    $S "tp_tcc@120=pmc:TCC_REQ_sum,TCC_HIT_sum,TCC_MISS_sum,TCC_TAG_STALL_sum|$K" \
       "tp_tcp@120=pmc:TCP_TCC_READ_REQ_sum,TCP_TCC_WRITE_REQ_sum,TCP_PENDING_STALL_CYCLES_sum,TCP_TCP_TA_DATA_STALL_CYCLES_sum|$K" \
       "tp_ta@120=pmc:TA_TA_BUSY_sum,TA_ADDR_STALLED_BY_TC_CYCLES_sum,GRBM_GUI_ACTIVE|$K" \
       "tp_fetch@120=pmc:FETCH_SIZE|$K" "tp_write@120=pmc:WRITE_SIZE|$K" ;;
  ev9)     # round 4 final evidence: the suite, smoke, every workload with its rocprof summary, C5 traffic
    $S "pytest_gpu@900=pytest" "smoke@300=smoke" "bench_c2=bench:" "prof_c2=prof:--no-cpu-baseline" \
       "bench_c3=bench:--workload c3 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c3=prof:--workload c3 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c4=bench:--workload c4 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c4=prof:--workload c4 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c4_1gpu=bench:--workload c4_1gpu --steps 20 --warmup 3 --cpu-seconds 8" \
       "prof_c4_1gpu=prof:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c5=bench:--workload c5 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c5=prof:--workload c5 --steps 20 --warmup 3 --no-cpu-baseline" \
       "pmc_c5_fetch@300=pmc:FETCH_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c5_write@300=pmc:WRITE_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" ;;
  ev10)    # round 4 final evidence after the tail grid change: ev9's steps
    bash "$0" ev9 ;;
  ev11)    # round 4 final evidence after the tail's col_ld / col_st experiment hooks: ev9's steps
    bash "$0" ev9 ;;
  ev12)    # round 4 final evidence after the median's replica-slot path: ev9's steps
    bash "$0" ev9 ;;
  ev13)    # round 4 final evidence on the final tree (tests added after ev12): ev9's steps
    bash "$0" ev9 ;;
  ev14)    # round 4 final evidence after prune_calc (prune_of's arithmetic returned, for the deferred-store experiment)
    bash "$0" ev9 ;;
  r5ev)    # round 5 final evidence: the suite, smoke, every workload (c3_full with its CPU baseline) with its
           # rocprof summary, C2 / C5 traffic, the scalar drop-ins' latency
    $S "pytest_gpu@900=pytest" "smoke@300=smoke" "bench_c2=bench:" "prof_c2=prof:--no-cpu-baseline" \
       "bench_c3=bench:--workload c3 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c3=prof:--workload c3 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c3_full@900=bench:--workload c3_full --steps 3 --warmup 1 --cpu-seconds 10" \
       "bench_c4=bench:--workload c4 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c4=prof:--workload c4 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c4_1gpu=bench:--workload c4_1gpu --steps 20 --warmup 3 --cpu-seconds 8" \
       "prof_c4_1gpu=prof:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c5=bench:--workload c5 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c5=prof:--workload c5 --steps 20 --warmup 3 --no-cpu-baseline" \
       "pmc_c2_fetch@300=pmc:FETCH_SIZE|bench.py --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c2_write@300=pmc:WRITE_SIZE|bench.py --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c5_fetch@300=pmc:FETCH_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c5_write@300=pmc:WRITE_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" \
       "scalar=scalar:--calls 3000" ;;
  r5traf)  # round 5: HBM traffic passes of C3, the C4 shard and the 64M-group batch on the final tree
    $S "pmc_c3_fetch@300=pmc:FETCH_SIZE|bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c3_write@300=pmc:WRITE_SIZE|bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c4_fetch@300=pmc:FETCH_SIZE|bench.py --workload c4 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c4_write@300=pmc:WRITE_SIZE|bench.py --workload c4 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c41_fetch@400=pmc:FETCH_SIZE|bench.py --workload c4_1gpu --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c41_write@400=pmc:WRITE_SIZE|bench.py --workload c4_1gpu --no-cpu-baseline --steps 3 --warmup 1" ;;
  r5c3)    # round 5: the hop build's 12-KiB windows: the suite, smoke, C3 and the whole C3 batch with profiles and traffic
    $S "pytest_gpu@900=pytest" "smoke@300=smoke" \
       "bench_c3=bench:--workload c3 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c3=prof:--workload c3 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c3_full@900=bench:--workload c3_full --steps 3 --warmup 1 --cpu-seconds 10" \
       "pmc_c3_fetch@300=pmc:FETCH_SIZE|bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c3_write@300=pmc:WRITE_SIZE|bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1" ;;
  r5seg)   # round 5: the segment walk's checksum builds at 3 waves per SIMD: the suite, smoke, a same-ring A/B
           # against the previous build, C5 and the 64M-group batch with profiles and traffic
    $S "pytest_gpu@900=pytest" "smoke@300=smoke" \
       "ab_seg3@400=sh:ab_seg3.sh" \
       "bench_c5=bench:--workload c5 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c5=prof:--workload c5 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c4_1gpu=bench:--workload c4_1gpu --steps 20 --warmup 3 --cpu-seconds 8" \
       "prof_c4_1gpu=prof:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" \
       "pmc_c5_fetch@300=pmc:FETCH_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c5_write@300=pmc:WRITE_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c41_fetch@400=pmc:FETCH_SIZE|bench.py --workload c4_1gpu --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c41_write@400=pmc:WRITE_SIZE|bench.py --workload c4_1gpu --no-cpu-baseline --steps 3 --warmup 1" ;;
  r5final) # round 5, the final tree: r5ev plus the C3, C4-shard and 64M-group traffic passes
    bash scripts/gpu_plan.sh r5ev && bash scripts/gpu_plan.sh r5traf ;;
  r6ev)    # round 6 evidence: the suite, smoke, every workload (c3_full with its CPU baseline) with its rocprof
           # summary, C5 with the packed request rows, and every workload's FETCH_SIZE / WRITE_SIZE passes
    $S "pytest_gpu@900=pytest" "smoke@300=smoke" "bench_c2=bench:" "prof_c2=prof:--no-cpu-baseline" \
       "bench_c3=bench:--workload c3 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c3=prof:--workload c3 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c3_full@900=bench:--workload c3_full --steps 3 --warmup 1 --cpu-seconds 10" \
       "bench_c4=bench:--workload c4 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c4=prof:--workload c4 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c4_1gpu=bench:--workload c4_1gpu --steps 20 --warmup 3 --cpu-seconds 8" \
       "prof_c4_1gpu=prof:--workload c4_1gpu --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c5=bench:--workload c5 --steps 20 --warmup 3 --cpu-seconds 6" \
       "prof_c5=prof:--workload c5 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c5_sit=bench:--workload c5 --steps 20 --warmup 3 --no-cpu-baseline --vote-sit" \
       "pmc_c2_fetch@300=pmc:FETCH_SIZE|bench.py --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c2_write@300=pmc:WRITE_SIZE|bench.py --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c5_fetch@300=pmc:FETCH_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c5_write@300=pmc:WRITE_SIZE|bench.py --workload c5 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c3_fetch@300=pmc:FETCH_SIZE|bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c3_write@300=pmc:WRITE_SIZE|bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c4_fetch@300=pmc:FETCH_SIZE|bench.py --workload c4 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c4_write@300=pmc:WRITE_SIZE|bench.py --workload c4 --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c41_fetch@400=pmc:FETCH_SIZE|bench.py --workload c4_1gpu --no-cpu-baseline --steps 3 --warmup 1" \
       "pmc_c41_write@400=pmc:WRITE_SIZE|bench.py --workload c4_1gpu --no-cpu-baseline --steps 3 --warmup 1" ;;
  r6kb)    # round 6: every kernel at C2 / C3 / C5 (kbench, one process per shape), append / persist, records,
           # the scalar drop-ins' latency
    $S "kb_c2@400=kb:--rounds 5" \
       "kb_c5@400=kb:--rounds 5 --groups 4194304 --replicas 7 --entries 16 --ring 8192 --cid-mix --only vote_tally,vote_rank,last_idx_term,median,prune,short_walk_checksum,apply,config_scan,nc_build,nc_build_quad,lr_completion,log_adjust,append,persist" \
       "kb_c3@500=kb:--rounds 3 --groups 524288 --replicas 5 --payload 64 --payload-max 4096 --ring 272960 --history-max 64 --only var_walk_checksum,var_walk,median,prune,nc_build_quad,validate,validate_lead,last_idx_term" \
       "kb_rec@300=kb:--rounds 5 --only records_store,records_load,records_store_lane,records_load_lane" \
       "kb_app@300=kb:--rounds 5 --only append,persist" \
       "scalar=scalar:--calls 3000" ;;
  r6chk)   # round 6: the rebuilt tree on a fresh box -- the suite, smoke, C2 with its profile, C5
    $S "pytest_gpu@900=pytest" "smoke@300=smoke" "bench_c2=bench:" "prof_c2=prof:--no-cpu-baseline" \
       "bench_c5=bench:--workload c5 --steps 20 --warmup 3 --no-cpu-baseline" \
       "bench_c2_rccl=bench:--rccl --no-cpu-baseline --steps 20 --warmup 0" \
       "trun_c2_rccl=trun:--rccl --no-cpu-baseline --steps 20 --warmup 1" ;;
  r6whole) # round 6: every group of every full-size BASELINE batch against oracle/_ref (the reference's code)
    $S "whole@1100=pytest:tests/test_whole_batch.py -v --durations=0" ;;
  r6app2)  # round 6: append + persist at kbench's C2 / C5 shapes, every group, against oracle/_ref
    $S "whole_app@900=pytest:tests/test_whole_batch.py -v --durations=0 -k append" ;;
  r6f2)    # round 6: apply + config scan at the C2 / C5 shapes, every group, against oracle/_ref
    $S "whole_f2@900=pytest:tests/test_whole_batch.py -v --durations=0 -k apply_config" ;;
  r6win)   # round 6: the C5 shard's election win, every group, against oracle/_ref
    $S "whole_win@900=pytest:tests/test_whole_batch.py -v --durations=0 -k election_win" ;;
  r6fin)   # round 6, the final tree: the whole suite (whole-batch parity included), smoke, C2 with its profile
    $S "pytest_gpu@1100=pytest:tests --durations=25" "smoke@300=smoke" "bench_c2=bench:" "prof_c2=prof:--no-cpu-baseline" ;;
  r6app)   # round 6: append / persist at the C2 shape
    $S "kb_app@300=kb:--rounds 5 --only append,persist" ;;
  *) echo "unknown plan $1"; exit 2 ;;
esac
