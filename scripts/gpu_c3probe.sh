#!/bin/bash
# C3 commit-kernel ceiling: read probe of the C3 access pattern, per-phase
# cycle accounting (APUS_EXP_PHASES build) and the product kernel's timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/stream_probe_c3 > gpurun_out/c3_probe.log 2>&1 || exit $?
cat gpurun_out/c3_probe.log
APUS_GPU_LIB=$PWD/build_exp/libapus_phases.so timeout -k 10 200 python3 scripts/phase_probe.py --c3 > gpurun_out/c3_phases.json 2>gpurun_out/c3_phases.err || { tail -5 gpurun_out/c3_phases.err; exit 1; }
cat gpurun_out/c3_phases.json
timeout -k 10 300 python3 scripts/kbench.py --rounds 3 --groups 262144 --replicas 5 --payload 64 --payload-max 4096 --ring 344064 --only wave_walk_checksum,wave_walk > gpurun_out/c3_kb.json 2>gpurun_out/c3_kb.err || { tail -5 gpurun_out/c3_kb.err; exit 1; }
grep -A3 '"wave_walk' gpurun_out/c3_kb.json
