#!/bin/bash
# Counters of append_kernel / persist_kernel at C2 from short kbench runs, one
# rocprofv3 --pmc pass per argument (default: FETCH_SIZE, then WRITE_SIZE);
# an argument is a space-separated counter list that fits one pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
[ $# -gt 0 ] || set -- FETCH_SIZE WRITE_SIZE
i=0
for pass in "$@"; do
  i=$((i + 1))
  d=gpurun_out/pmc_app_$i
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $d -o run --output-format csv -- \
    python3 scripts/kbench.py --rounds 2 --only ${KB_ONLY:-append,persist} ${KBARGS:-} > $d.log 2>&1 || exit $?
  python3 scripts/pmc_kernels.py $d ${PMC_KERNELS:-append_kernel persist_kernel}
done
