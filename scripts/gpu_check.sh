#!/bin/bash
# One gpurun session: GPU parity tests, smoke, a bench line and (optionally)
# a rocprofv3 kernel-trace of the bench.  Every GPU step has its own time
# limit; a step that faults / aborts / times out ends the script (test
# FAILURES, exit 1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="${STEPS:-pytest smoke bench}"
step() {
  local name=$1 limit=$2; shift 2
  echo "== $name: $*" ; date +%T
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    pytest) step pytest_gpu 1500 python -m pytest tests -m gpu -q -x -p no:cacheprovider ${PYTEST_ARGS:-} ;;
    smoke)  step smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 900 python bench.py ${BENCH_ARGS:-} ;;
    prof)   export TMPDIR=/tmp
            step prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} ;;
    pmc_fetch) export TMPDIR=/tmp
            step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 ${BENCH_ARGS:-} ;;
    pmc_write) export TMPDIR=/tmp
            step pmc_write 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 ${BENCH_ARGS:-} ;;
  esac
done
echo "== done"
