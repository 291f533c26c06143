#!/bin/bash
# commit kernel change check: commit parity tests, then C2 and C3 kernel timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_log_image.py tests/test_full_size.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/hop_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/hop_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/kbench.py --rounds 5 --only wave_walk_checksum,var_walk_checksum > gpurun_out/hop_kb_c2.json 2>gpurun_out/hop_kb.err || { tail -5 gpurun_out/hop_kb.err; exit 1; }
grep -A2 "_walk" gpurun_out/hop_kb_c2.json
timeout -k 10 300 python3 scripts/kbench.py --rounds 5 --groups 262144 --replicas 5 --payload 64 --payload-max 4096 --ring 344064 --only wave_walk_checksum,var_walk_checksum,var_walk > gpurun_out/hop_kb_c3.json 2>gpurun_out/hop_kb.err || { tail -5 gpurun_out/hop_kb.err; exit 1; }
grep -A2 "_walk" gpurun_out/hop_kb_c3.json
