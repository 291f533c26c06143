"""Can the C5 tail's walk-independent work (the vote tally and log_pruning's
minimum: neither reads what the walk produces) run beside the walk on a second
stream?  Times, on the C5 shard (2^23 groups x R = 7, 16 entries, cid mix):
  fused    the bench's one commit call (walk + checksum + median + publish +
           pruning + LIT + tally + ranking)
  seq      the commit call without tally / pruning, then apus_vote_batch and
           apus_prune_batch on the same stream
  overlap  the same three, the tally and the pruning on a second stream that
           starts with the commit call (events both ways)
each the median of interleaved rounds (HIP events around the whole), plus the
walk kernel's own duration in each (apus_commit_mark_walk).
usage: python scripts/overlap_probe.py [--groups N] [--rounds 8]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1 << 23)
    ap.add_argument("--rounds", type=int, default=8)
    args = ap.parse_args()
    import torch

    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi
    eng = pkg.Engine(0)
    lib = eng.lib
    G, R = args.groups, 7
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(8192))
    cfg = pkg.batch.gen_cfg(seed=2026, n_entries=16, n_history=16, len_min=64, len_max=64, ring_len=8192,
                            p_full_ack=0.9, straggler=True, cid_mix=True, p_vote_ack=0.6)
    eng.gen(db, cfg)
    torch.cuda.synchronize()
    W, CK, MD, PR, PUB = abi.COMMIT_WALK, abi.COMMIT_CHECKSUM, abi.COMMIT_MEDIAN, abi.COMMIT_PRUNE, abi.COMMIT_PUBLISH
    LIT, VT, RK = abi.COMMIT_LAST_IT, abi.COMMIT_VOTE, abi.COMMIT_RANK
    full = W | CK | MD | PR | PUB | LIT | VT | RK
    part = W | CK | MD | PUB | LIT | RK
    out = eng.alloc_commit_out(G, full)
    o = eng.commit_struct(out)
    b = db.struct()
    b.flags = abi.BATCH_SHORT_WALKS
    vo = {"won": eng._z(G, torch.uint8), "vote_count": eng._z(G, torch.uint8, 2),
          "new_commit": eng._z(G, torch.int64), "voters": eng._z(G, torch.int16)}
    vos = abi.VoteOut(won=vo["won"].data_ptr(), vote_count=vo["vote_count"].data_ptr(),
                      new_commit=vo["new_commit"].data_ptr(), voters=vo["voters"].data_ptr())
    pout = {"new_head": eng._z(G, torch.int64), "append_head": eng._z(G, torch.uint8),
            "min_apply": eng._z(G, torch.int64)}
    s1 = torch.cuda.current_stream()
    s2 = torch.cuda.Stream()
    p1, p2 = C.c_void_p(s1.cuda_stream), C.c_void_p(s2.cuda_stream)
    mk = lambda: torch.cuda.Event(enable_timing=True)   # noqa: E731

    def run(case):
        a, z, wa, wz = mk(), mk(), mk(), mk()
        wa.record(s1)                  # (torch creates an event at its first record)
        wz.record(s1)
        a.record(s1)
        lib.apus_commit_mark_walk(eng.ctx, C.c_void_p(wa.cuda_event), C.c_void_p(wz.cuda_event))
        if case == "fused":
            lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), full, p1)
        elif case == "seq":
            lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), part, p1)
            lib.apus_vote_batch(eng.ctx, C.byref(b), C.byref(vos), p1)
            eng.log_pruning(db, out=pout, bstruct=b, stream=s1)
        else:
            s2.wait_event(a)
            lib.apus_vote_batch(eng.ctx, C.byref(b), C.byref(vos), p2)
            eng.log_pruning(db, out=pout, bstruct=b, stream=s2)
            lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), part, p1)
            e2 = mk()
            e2.record(s2)
            s1.wait_event(e2)
        z.record(s1)
        return a, z, wa, wz

    cases = ("fused", "seq", "overlap")
    for c in cases:
        run(c)
    torch.cuda.synchronize()
    res = {c: ([], []) for c in cases}
    for _ in range(args.rounds):
        for c in cases:
            ev = run(c)
            torch.cuda.synchronize()
            res[c][0].append(ev[0].elapsed_time(ev[1]))
            res[c][1].append(ev[2].elapsed_time(ev[3]))
    print(json.dumps({c: {"ms_median": float(np.median(v[0])), "ms_min": float(np.min(v[0])),
                          "walk_ms_median": float(np.median(v[1]))} for c, v in res.items()}, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
