"""Summarise rocprofv3 csv output (kernel trace + PMC passes) per kernel.
usage: python scripts/parse_pmc.py <dir with pass subdirs>"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
pmc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("apus::", "")
        pmc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = defaultdict(list)
for f in glob.glob(os.path.join(root, "*", "*kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("apus::", "")
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
for k in sorted(set(pmc) | set(dur)):
    print(f"## {k}")
    if dur.get(k):
        d = sorted(dur[k])
        print(f"  dispatches={len(d)} avg_ms={sum(d)/len(d):.4f} min_ms={d[0]:.4f} max_ms={d[-1]:.4f}")
    c = {n: sum(v) / len(v) for n, v in pmc[k].items()}
    for n in sorted(c):
        print(f"  {n:28s} {c[n]:.6g}")
    if "SQ_WAVES" in c and c.get("SQ_WAVES"):
        w = c["SQ_WAVES"]
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
            if n in c:
                print(f"  per-wave {n:20s} {c[n]/w:.1f}")
    if "FETCH_SIZE" in c:
        print(f"  FETCH_SIZE*2 (gfx950 wide-read correction) bytes = {c['FETCH_SIZE']*1024*2:.4g}")
    if "WRITE_SIZE" in c:
        print(f"  WRITE_SIZE bytes = {c['WRITE_SIZE']*1024:.4g}")
