#!/bin/bash
# Same-box A/B by kernel trace: kbench cases (ONLY, KB_ARGS) under
# rocprofv3 --kernel-trace --stats for the product library and each EXP_LIBS
# build; prints every kernel's calls and average duration per library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pass in 1 2; do
for lib in rdma-paxos_amd/libapus_gpu.so ${EXP_LIBS:-}; do
  n=$(basename $lib .so)
  d=gpurun_out/abp_${n}_$pass
  APUS_GPU_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
    python3 scripts/kbench.py --rounds ${ROUNDS:-8} $KB_ARGS --only $ONLY > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  python3 - "$n" "$pass" "$d" <<'PY'
import csv, glob, sys
n, p, d = sys.argv[1:]
f = glob.glob(f"{d}/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    nm = r["Name"]
    if "gen_" in nm or "elementwise" in nm or "fill" in nm.lower():
        continue
    print(n, p, nm[:90], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4), "ms")
PY
done
done
