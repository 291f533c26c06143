"""Does commit_seg_kernel's time at the C5 shard depend on what ran before it?

The tail's nontemporal-load experiment (profiles/r04/tail_nt/) made the C5
tail slower and the walk that follows it faster (3.14 against 3.37 ms, both
passes).  Here one process, one batch (bench.py's C5 shard: 2^23 groups x
R=7, 16 entries after 16 history entries, 8,192-B rings, short-walk hint),
four phases of PHASE calls each, run under rocprofv3 --kernel-trace:
  walk        the walk alone (walk + checksum + local (idx, term)), back to back
  fused       the whole C5 step (walk + the fused tail), back to back
  walk_sleep  the walk alone, each followed by an idle kernel of the fused
              tail's length (torch.cuda._sleep)
  walk_copy   the walk alone, each followed by a device copy of 2.6 GB
              (HBM busy for about the fused tail's length, no arithmetic)
The script then reads the kernel trace it was run under (--trace DIR after
the run) and prints the walk's mean / min / max duration per phase.

--batches K: instead, K copies of the same batch (each its own allocation,
generated alike) walked in turn, N rounds: the walk's time per copy, in one
process.  --alloc hip / contig: the rings from hipExtMallocWithFlags with
the default / the contiguous flag instead of torch's allocator.  --rings K:
one batch's columns and K copies of its rings (device copies), walked in
turn, timed by the walk kernel's own start / end (apus_commit_mark_walk;
the round-4 and early round-5 runs timed the whole call, the tail launch
included).  --ab FLAGS: each ring also walked with FLAGS OR-ed into the
batch flags, alternately.
"""
import argparse
import csv
import ctypes as C
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHASES = ("walk", "fused", "walk_sleep", "walk_copy")


def run(n):
    import torch

    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi
    eng = pkg.Engine(0)
    lib = eng.lib
    G, R = 1 << 23, 7
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(8192))
    cfg = pkg.batch.gen_cfg(seed=2026, n_entries=16, n_history=16, len_min=64, len_max=64, ring_len=8192,
                            p_full_ack=0.9, straggler=True, cid_mix=True)
    eng.gen(db, cfg)
    bs = db.struct()
    bs.flags = abi.BATCH_SHORT_WALKS
    out = eng.alloc_commit_out(G, 15 | abi.COMMIT_LAST_IT | abi.COMMIT_VOTE | abi.COMMIT_RANK)
    o = eng.commit_struct(out)
    W, CK, MD, PR = abi.COMMIT_WALK, abi.COMMIT_CHECKSUM, abi.COMMIT_MEDIAN, abi.COMMIT_PRUNE
    LIT, VT, RK = abi.COMMIT_LAST_IT, abi.COMMIT_VOTE, abi.COMMIT_RANK
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    src = torch.empty(1300 << 20, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)

    def walk():
        abi.check(lib.apus_commit_batch(eng.ctx, C.byref(bs), C.byref(o), W | CK | LIT, sp), "walk")

    def fused():
        abi.check(lib.apus_commit_batch(eng.ctx, C.byref(bs), C.byref(o), W | CK | MD | PR | LIT | VT | RK, sp),
                  "fused")
    for _ in range(3):
        fused()
    torch.cuda.synchronize()
    for ph in PHASES:
        for _ in range(n):
            if ph == "fused":
                fused()
            else:
                walk()
            if ph == "walk_sleep":
                torch.cuda._sleep(3_000_000)
            elif ph == "walk_copy":
                dst.copy_(src)
        torch.cuda.synchronize()
        torch.cuda._sleep(50_000_000)          # a marker gap between phases
        torch.cuda.synchronize()
    eng.close()


class _Dev:
    """a device allocation made outside torch (hipExtMallocWithFlags)"""
    def __init__(self, size, flags):
        self.hip = C.CDLL("libamdhip64.so")
        self.p = C.c_void_p()
        rc = self.hip.hipExtMallocWithFlags(C.byref(self.p), C.c_size_t(size), C.c_uint(flags))
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags({size}, {flags:#x}) = {rc}")

    def data_ptr(self):
        return self.p.value


def run_batches(n, k, alloc):
    import torch

    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi
    eng = pkg.Engine(0)
    lib = eng.lib
    G, R = 1 << 23, 7
    cfg = pkg.batch.gen_cfg(seed=2026, n_entries=16, n_history=16, len_min=64, len_max=64, ring_len=8192,
                            p_full_ack=0.9, straggler=True, cid_mix=True)
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_LAST_IT
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    cps = []
    for _ in range(k):
        db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(8192),
                                   fields=["state", "self_idx", "remote_end", "lr_step", "fail_count"])
        if alloc != "torch":
            db.ring = None
            torch.cuda.empty_cache()
            db.ring = _Dev(G * db.stride, {"hip": 0x0, "contig": 0x4}[alloc])
        eng.gen(db, cfg)
        bs = db.struct()
        bs.flags = abi.BATCH_SHORT_WALKS
        out = eng.alloc_commit_out(G, flags)
        cps.append((db, bs, out, eng.commit_struct(out)))
        print("batch at", hex(db.ring.data_ptr()), flush=True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ms = [[] for _ in range(k)]
    for _ in range(n):
        for i, (db, bs, out, o) in enumerate(cps):
            ev[0].record()
            abi.check(lib.apus_commit_batch(eng.ctx, C.byref(bs), C.byref(o), flags, sp), "walk")
            ev[1].record()
            torch.cuda.synchronize()
            ms[i].append(ev[0].elapsed_time(ev[1]))
    print(json.dumps({"batches": [[round(sum(m) / len(m), 4), round(min(m), 4), round(max(m), 4)] for m in ms]}))
    eng.close()


SHAPES = {
    "c5": dict(G=1 << 23, R=7, E=16, H=16, ring=8192, cid_mix=True, short=True, lit=True),
    "c2": dict(G=1 << 20, R=3, E=64, H=16, ring=16384, cid_mix=False, short=False, lit=False),
    "c4_1gpu_2e23": dict(G=1 << 23, R=5, E=16, H=2, ring=2448, cid_mix=False, short=True, lit=False),
    # what separates the C5 walk from the C4 1-GPU shape's (same bytes per group):
    # the (idx, term) rows, the configuration mix and R = 7, the 8-KiB ring stride
    "c5_nolit": dict(G=1 << 23, R=7, E=16, H=16, ring=8192, cid_mix=True, short=True, lit=False),
    "c5_dense": dict(G=1 << 23, R=7, E=16, H=2, ring=2448, cid_mix=True, short=True, lit=True),
    "c3": dict(G=1 << 19, R=5, E=64, H=16, ring=272960, cid_mix=False, short=False, lit=False, Lmax=4096, Hmax=64,
               var=True),
    "c3_nc": dict(G=1 << 19, R=5, E=64, H=16, ring=272960, cid_mix=False, short=False, lit=False, Lmax=4096, Hmax=64,
                  var=True, nc=True),
    "c4": dict(G=1 << 23, R=5, E=64, H=16, ring=16384, cid_mix=False, short=False, lit=False),
    "c4_sparse": dict(G=1 << 23, R=5, E=16, H=16, ring=8192, cid_mix=False, short=True, lit=False),
}


def run_rings(n, k, shape, stride=0, ab=0, ab_lib=""):
    """one batch's columns; its rings copied into K allocations, walked in turn"""
    import torch

    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi
    eng = pkg.Engine(0)
    lib = eng.lib
    sh = SHAPES[shape]
    G, R = sh["G"], sh["R"]
    cfg = pkg.batch.gen_cfg(seed=2026, n_entries=sh["E"], n_history=sh["H"], len_min=64, len_max=sh.get("Lmax", 64),
                            ring_len=sh["ring"], p_full_ack=0.9, straggler=True, cid_mix=sh["cid_mix"],
                            hist_len_max=sh.get("Hmax", 0))
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | (abi.COMMIT_LAST_IT if sh["lit"] else 0) | \
        (abi.COMMIT_NC if sh.get("nc") else 0)
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    db = pkg.batch.DeviceBatch(G, R, stride or pkg.batch.ring_stride_for(sh["ring"]),
                               fields=["state", "self_idx", "remote_end", "lr_step", "fail_count"])
    eng.gen(db, cfg)
    rings = [db.ring] + [db.ring.clone() for _ in range(k - 1)]
    out = eng.alloc_commit_out(G, flags, nc_max=sh["E"] if sh.get("nc") else 0)
    o = eng.commit_struct(out)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in ev:                                 # created at their first record
        e.record()
    torch.cuda.synchronize()
    # ab: each ring walked with the batch flags as they are and with ab OR-ed
    # in, alternately (a same-allocation A/B of two walk forms); ab_lib:
    # and by another build of the library loaded beside this one (its own
    # context, the same device memory)
    variants = [(0, lib, eng.ctx)] + ([(ab, lib, eng.ctx)] if ab else [])
    if ab_lib:
        lib2 = abi.load_library(ab_lib)
        h2 = C.c_void_p()
        abi.check(lib2.apus_ctx_create(0, C.byref(h2)), "apus_ctx_create (ab lib)")
        variants.append((0, lib2, h2))
    ms = [[[] for _ in variants] for _ in range(k)]
    for _ in range(n):
        for i, r in enumerate(rings):
            for vi, (extra, vlib, vctx) in enumerate(variants):
                bs = db.struct()
                bs.flags = (abi.BATCH_SHORT_WALKS if sh["short"] else 0) | (abi.BATCH_VAR_LEN if sh.get("var") else 0) | extra
                bs.ring = r.data_ptr()
                # the walk kernel's own start / end (apus_commit_mark_walk), not the tail launch
                abi.check(vlib.apus_commit_mark_walk(vctx, C.c_void_p(ev[0].cuda_event),
                                                     C.c_void_p(ev[1].cuda_event)), "mark_walk")
                abi.check(vlib.apus_commit_batch(vctx, C.byref(bs), C.byref(o), flags, sp), "walk")
                torch.cuda.synchronize()
                ms[i][vi].append(ev[0].elapsed_time(ev[1]))
    st = lambda m: [round(sum(m) / len(m), 4), round(min(m), 4), round(max(m), 4)]
    res = {"shape": shape, "stride": db.stride, "rings": [st(m[0]) for m in ms], "at": [hex(r.data_ptr()) for r in rings]}
    if ab:
        res["ab_flag"] = hex(ab)
        res["rings_ab"] = [st(m[1]) for m in ms]
    if ab_lib:
        res["ab_lib"] = ab_lib
        res["rings_ab_lib"] = [st(m[-1]) for m in ms]
        lib2.apus_ctx_destroy(h2)
    print(json.dumps(res))
    eng.close()


def chan_report(d, k):
    """--chan DIR: per walk dispatch (ring i = dispatch j mod K), the per-channel
    TCC -> EA read requests of a pass with scripts/chan_counters.yaml's counters:
    the spread over the channels (max / mean, coefficient of variation)"""
    import numpy as np
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if "commit_seg_kernel" not in r["Kernel_Name"] and "commit_wave_kernel" not in r["Kernel_Name"]:
            continue
        per.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(per)
    res = {}
    for j, di in enumerate(ids):
        c = per[di]
        ring = j % k
        for fam, keys in (("ch", [f"APUS_RDREQ_CH{i}" for i in range(16)]),
                          ("xcd", [f"APUS_RDREQ_XCD{x}" for x in range(8)]),
                          ("xc", [f"APUS_RDREQ_X{x}C{i}" for x in range(8) for i in range(16)]),
                          ("hit", ["TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum"]),
                          ("dram", ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_LEVEL_sum",
                                    "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "TCC_TAG_STALL_sum", "GRBM_GUI_ACTIVE"])):
            if not all(x in c for x in keys):
                continue
            v = np.array([c[x] for x in keys])
            e = res.setdefault(ring, {}).setdefault(fam, [])
            if fam == "dram":
                # mean requests in flight per cycle over the TCC instances, and
                # the mean cycles a read request waits (LEVEL / RDREQ)
                e.append({"rdreq": v[0], "cycles": v[4], "lat_cycles": round(v[1] / max(v[0], 1), 1),
                          "credit_stall": v[2], "tag_stall": v[3]})
            elif fam == "hit":
                e.append({"hit_rate": round(v[0] / max(v[0] + v[1], 1), 4), "hit": v[0], "miss": v[1], "rdreq": v[2]})
            else:
                e.append({"total": v.sum(), "max_over_mean": round(v.max() / v.mean(), 4),
                          "cv": round(v.std() / v.mean(), 4), "min_over_mean": round(v.min() / v.mean(), 4),
                          "values": [int(x) for x in v] if fam != "xc" else None})
        # any other counters of the pass, as collected
        rest = {k: c[k] for k in sorted(c) if not k.startswith("APUS_")}
        if rest:
            res.setdefault(ring, {}).setdefault("raw", []).append(rest)
    print(json.dumps(res, indent=1))


def report(d, n):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    calls = []                                   # [walk ms, the tail launch after it (ms) or 0]
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        if "commit_seg_kernel" in r["Kernel_Name"]:
            calls.append([d, 0.0])
        elif "quorum_tail_kernel" in r["Kernel_Name"] and calls:
            calls[-1][1] = d
    calls = calls[3:]                            # the warm-up calls
    res = {}
    for i, ph in enumerate(PHASES):
        w = [c[0] for c in calls[i * n:(i + 1) * n]]
        t = [c[1] for c in calls[i * n:(i + 1) * n]]
        res[ph] = {"walk_ms": [round(sum(w) / len(w), 4), round(min(w), 4), round(max(w), 4)],
                   "tail_ms": round(sum(t) / len(t), 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--trace", default="")
    ap.add_argument("--batches", type=int, default=0)
    ap.add_argument("--rings", type=int, default=0)
    ap.add_argument("--shape", default="c5", choices=sorted(SHAPES))
    ap.add_argument("--stride", type=int, default=0, help="ring stride (default ring_stride_for(ring))")
    ap.add_argument("--alloc", default="torch", choices=["torch", "hip", "contig"])
    ap.add_argument("--ab", default="0", help="--rings: also walk each ring with these batch flags OR-ed in")
    ap.add_argument("--ab-lib", default="", help="--rings: also walk each ring with this build of the library")
    ap.add_argument("--chan", default="", help="report a per-channel counter pass (DIR) of a --rings K run")
    a = ap.parse_args()
    if a.chan:
        chan_report(a.chan, a.rings)
    elif a.rings:
        run_rings(a.n, a.rings, a.shape, a.stride, int(a.ab, 0), a.ab_lib)
    elif a.batches:
        run_batches(a.n, a.batches, a.alloc)
    elif a.trace:
        report(a.trace, a.n)
    else:
        run(a.n)
