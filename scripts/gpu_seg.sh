#!/bin/bash
# commit_seg_kernel bring-up: parity of every commit implementation, then C5 timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "commit" > gpurun_out/seg_parity.log 2>&1
rc=$?; tail -3 gpurun_out/seg_parity.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_log_image.py > gpurun_out/seg_log_image.log 2>&1
rc=$?; tail -3 gpurun_out/seg_log_image.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/kbench.py --groups 4194304 --replicas 7 --entries 16 --cid-mix --rounds 8 \
  --only wave_walk_checksum,wave_walk,short_walk_checksum,short_walk > gpurun_out/kb_c5_seg.log 2>&1
rc=$?; cat gpurun_out/kb_c5_seg.log | grep -v amdgpu.ids; exit $rc
