#!/bin/bash
# Process-to-process spread of the C5 segment walk against its address
# translation: N processes, each one rocprofv3 pass with the kernel trace and
# the UTCL1 counters, over kbench's short_walk_checksum at the C5 shard shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C5="--groups 8388608 --replicas 7 --entries 16 --ring 8192 --cid-mix"
for p in $(seq 1 ${N:-4}); do
  d=gpurun_out/tlbv_$p
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE \
    -d $d -o run --output-format csv -- python3 scripts/kbench.py --rounds 3 $C5 --only short_walk_checksum > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  python3 - "$d" "$p" <<'PY'
import csv, glob, sys
d, p = sys.argv[1:]
t = {}
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "commit_seg" in r["Kernel_Name"]:
            t.setdefault("ms", []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
c = {}
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "commit_seg" in r["Kernel_Name"]:
            c.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
print(p, {k: [round(x, 3) for x in v] for k, v in t.items()}, {k: [round(x / 1e6, 2) for x in v] for k, v in c.items()})
PY
done
