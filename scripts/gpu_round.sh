#!/bin/bash
# Round evidence: full GPU suite, smoke, C2 bench (+ rocprof), C3 bench (+ rocprof).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 limit=$2; shift 2
  echo "== $name"; date +%T
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for s in ${STEPS:-pytest smoke bench prof bench_c3 prof_c3}; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench_c2 600 python bench.py ;;
    prof) step prof_c2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline ;;
    bench_c3) step bench_c3 600 python bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 6 ;;
    prof_c3) step prof_c3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline ;;
    pmc_c3_fetch) step pmc_c3_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c3_fetch -o run --output-format csv -- python3 bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1 ;;
    pmc_c3_write) step pmc_c3_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_c3_write -o run --output-format csv -- python3 bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1 ;;
  esac
done
echo "== done"
