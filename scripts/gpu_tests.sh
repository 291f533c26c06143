#!/bin/bash
# GPU pytest run (optionally a subset: TESTS="tests/test_x.py ..."), log under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
NAME=${NAME:-pytest_gpu}
timeout -k 10 ${LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > "gpurun_out/$NAME.log" 2>&1
rc=$?
tail -n 5 "gpurun_out/$NAME.log"
exit $rc
