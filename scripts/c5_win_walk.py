"""The C5 walk before and after the election win, on the same rings (one process).

bench.py --workload c5 times its steps on the logs the cold step's
apus_vote_win_batch left: every candidate's commit moved to its tally's, and
every winner's log one blank entry (CONFIG / NOOP, 64 B) longer.  This script
times the commit call's walk kernel (its own start / end events,
apus_commit_mark_walk) with the bench's C5 flags on the generated logs, then
runs the win call once and times the same walk again: the walk's ms, its
algorithmic bytes (every walked entry, counted from the logs as they are) and
the fraction of the 8 TB/s peak, both ways.

Usage: python scripts/c5_win_walk.py [--n 10]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10)
    a = ap.parse_args()
    import torch

    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi
    eng = pkg.Engine(0)
    lib = eng.lib
    G, R, E, L = 1 << 23, 7, 16, 8192
    stride = pkg.batch.ring_stride_for(L)
    db = pkg.batch.DeviceBatch(G, R, stride)
    eng.gen(db, pkg.batch.gen_cfg(seed=2026, n_entries=E, n_history=16, len_min=64, len_max=64, ring_len=L,
                                  p_full_ack=0.9, straggler=True, cid_mix=True, p_vote_ack=0.6))
    b = db.struct()
    b.flags = abi.BATCH_SHORT_WALKS
    flags = (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PUBLISH | abi.COMMIT_PRUNE |
             abi.COMMIT_STATS_FRESH | abi.COMMIT_LAST_IT | abi.COMMIT_VOTE | abi.COMMIT_RANK)
    out = eng.alloc_commit_out(G, flags)
    o = eng.commit_struct(out)
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in ev:
        e.record()
    torch.cuda.synchronize()

    def walked():
        dets, ln = eng.log_entries_to_nc_buf(db, E + 2)
        d3 = dets.view(torch.int64).view(G, E + 2, 3)
        live = torch.arange(E + 2, device="cuda").view(1, -1) < ln.view(G, 1).to(torch.int64)
        at = torch.arange(G, device="cuda").view(G, 1) * stride + d3[:, :, 2]
        at = torch.where(live, at, torch.zeros_like(at))
        typ = db.ring[at + 26].to(torch.int64)
        clen = db.ring[at + 48].to(torch.int64) | (db.ring[at + 49].to(torch.int64) << 8)
        el = 64 + torch.where((typ == abi.NOOP) | (typ == abi.CONFIG) | (typ == abi.HEAD), 0, clen)
        n = ln.to(torch.int64)
        return int(torch.where(live, el, torch.zeros_like(el)).sum().item()), int((n > E).sum().item())

    def time_walk():
        ms = []
        for _ in range(a.n):
            abi.check(lib.apus_commit_mark_walk(eng.ctx, C.c_void_p(ev[0].cuda_event), C.c_void_p(ev[1].cuda_event)),
                      "mark")
            abi.check(lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), flags, sp), "commit")
            torch.cuda.synchronize()
            ms.append(ev[0].elapsed_time(ev[1]))
        return ms

    res = {}
    for phase in ("generated", "after_win"):
        wb, long_ = walked()
        ms = time_walk()
        mean = sum(ms) / len(ms)
        alg = wb + (64 + 1 + 17 + 16) * G
        res[phase] = {"walk_ms_mean": round(mean, 4), "walk_ms_min": round(min(ms), 4),
                      "walked_bytes": wb, "alg_bytes": alg, "frac": round(alg / (mean * 1e-3) / 8e12, 4),
                      "groups_over_16_entries": long_}
        if phase == "generated":
            t = torch
            z = lambda dt, n=1: torch.zeros(G * n, dtype=dt, device="cuda")   # noqa: E731
            st64 = db.arrays["state"].view(torch.int64).view(G, 8)
            wio = {"won": out["vote"]["won"], "voters": out["vote"]["voters"],
                   "new_commit": out["vote"]["new_commit"], "cid_offset": st64[:, 2].clone(),
                   "cid_idx": z(t.int64), "req_id": z(t.int64), "clt_id": z(t.int16),
                   "last_applied": z(t.int64, 3), "last_csm_idx": z(t.int64), "last_write_csm_idx": z(t.int64),
                   "outcome": z(t.uint8), "events": z(t.uint8), "departed": z(t.int16), "n_applied": z(t.int32),
                   "n_cfg": z(t.int32)}
            eng.become_leader(db, wio, bstruct=b)
            torch.cuda.synchronize()
    print(json.dumps(res))
    eng.close()


if __name__ == "__main__":
    main()
