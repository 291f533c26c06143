#!/bin/bash
# Same-box A/B by kernel trace over bench.py: WORKLOADS (default c4_1gpu) under
# rocprofv3 --kernel-trace --stats for the product library and each EXP_LIBS
# build, twice; prints the apus kernels' calls and average durations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pass in 1 2; do
for wl in ${WORKLOADS:-c4_1gpu}; do
for lib in rdma-paxos_amd/libapus_gpu.so ${EXP_LIBS:-}; do
  n=$(basename $lib .so)
  d=gpurun_out/abb_${wl}_${n}_$pass
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
    python3 bench.py --workload $wl --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  python3 - "$n" "$pass" "$d" "$wl" <<'PY'
import csv, glob, sys
n, p, d, wl = sys.argv[1:]
f = glob.glob(f"{d}/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    nm = r["Name"]
    if "apus::" not in nm or "gen_" in nm:
        continue
    print(wl, n, p, nm.split("(")[0][:70], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4), "ms")
PY
done
done
done
