"""HBM traffic of the dominant commit kernel per launch from two rocprofv3
--pmc passes (FETCH_SIZE, WRITE_SIZE; their own runs), written as the
profiles/traffic_commit_<workload>.json that bench.py reports as
roofline.traffic.  FETCH_SIZE is doubled (gfx950 wide-read correction,
MI355X_MICROARCH.md HBM section); both are in KiB.

usage: python3 scripts/traffic_json.py WORKLOAD GROUPS KERNEL_SUBSTR FETCH_DIR WRITE_DIR [BENCH_LOG]

The same passes' rows of quorum_tail_kernel (the commit call's second
launch) go under "tail" with the same correction: its lane-per-group column
loads arrive as whole 128-B lines, as the walk's do (TCP_TCC_READ_REQ x 128 B
= FETCH_SIZE x 2 at the tail, profiles/r04/tail_pmc/).
"""
import csv
import glob
import json
import os
import sys


def avg(d, counter, key):
    v = []
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"] and r["Counter_Name"] == counter:
                v.append(float(r["Counter_Value"]))
    if not v:
        raise SystemExit(f"no {counter} rows for {key} in {d}")
    return sum(v) / len(v), len(v)


def main():
    wl, groups, key, fdir, wdir = sys.argv[1:6]
    fkb, nf = avg(fdir, "FETCH_SIZE", key)
    wkb, nw = avg(wdir, "WRITE_SIZE", key)
    out = {"workload": wl, "groups": int(groups), "kernel": key, "fetch_size_kb": fkb, "write_size_kb": wkb,
           "hbm_bytes_per_launch": fkb * 1024 * 2 + wkb * 1024,
           "method": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes ({nf} / {nw} dispatches); "
                     "FETCH_SIZE x1024 x2 (gfx950 wide-read correction) + WRITE_SIZE x1024",
           "source": f"{fdir}, {wdir}", "round": int(os.environ.get("APUS_ROUND", "4"))}
    b = None
    if len(sys.argv) > 6:
        t = open(sys.argv[6]).read()
        b = json.loads(t[t.index("{"):])
        out["alg_bytes_per_launch"] = b["roofline"]["alg_bytes_per_launch"]
        out["traffic_over_alg"] = out["hbm_bytes_per_launch"] / out["alg_bytes_per_launch"]
    try:
        tf, ntf = avg(fdir, "FETCH_SIZE", "quorum_tail_kernel")
        tw, ntw = avg(wdir, "WRITE_SIZE", "quorum_tail_kernel")
        out["tail"] = {"kernel": "quorum_tail_kernel", "fetch_size_kb": tf, "write_size_kb": tw,
                       "hbm_bytes_per_launch": tf * 1024 * 2 + tw * 1024, "dispatches": [ntf, ntw]}
        if b is not None and (b["roofline"].get("tail") or {}).get("alg_bytes_per_launch"):
            out["tail"]["alg_bytes_per_launch"] = b["roofline"]["tail"]["alg_bytes_per_launch"]
            out["tail"]["traffic_over_alg"] = out["tail"]["hbm_bytes_per_launch"] / out["tail"]["alg_bytes_per_launch"]
    except SystemExit:
        pass
    json.dump(out, open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                     f"traffic_commit_{wl}.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
