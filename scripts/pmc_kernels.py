"""Average FETCH_SIZE / WRITE_SIZE per dispatch (gfx950 x2 read correction)
of the kernels in a rocprofv3 --pmc output directory whose name contains one
of the given substrings.  usage: python scripts/pmc_kernels.py <dir> <substr>..."""
import csv
import glob
import os
import sys
from collections import defaultdict

root, keys = sys.argv[1], sys.argv[2:]
d = defaultdict(list)
for f in glob.glob(os.path.join(root, "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if any(s in k for s in keys):
            d[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    if c in ("FETCH_SIZE", "WRITE_SIZE"):
        scale = 1024 * (2 if c == "FETCH_SIZE" else 1)
        print(f"{k} {c} dispatches={len(v)} avg={sum(v) / len(v) * scale / 1e9:.3f} GB")
    else:
        print(f"{k} {c} dispatches={len(v)} avg={sum(v) / len(v):.6g}")
