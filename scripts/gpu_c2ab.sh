#!/bin/bash
# commit_wave_kernel A/B on one box: parity of the product build's commit
# paths, then kernel timings of the product and build_exp/ libraries, then
# the phase-instrumented build (if present)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_golden.py tests/test_log_image.py -k "commit or golden or gpu_matches or log_image" \
  > gpurun_out/ab_parity.log 2>&1
rc=$?; tail -2 gpurun_out/ab_parity.log; [ $rc -ne 0 ] && exit $rc
ONLY=${ONLY:-wave_walk_checksum} ROUNDS=${ROUNDS:-12} bash scripts/exp_run.sh || exit $?
if [ -f build_exp/libapus_phases.so ]; then
  APUS_GPU_LIB=$PWD/build_exp/libapus_phases.so timeout -k 10 200 python scripts/phase_probe.py > gpurun_out/phases.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/phases.log | grep -v "frac"; exit $rc
fi
