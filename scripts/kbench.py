"""Per-kernel timing of the libapus_gpu entry points on one batch (HIP events,
interleaved rounds in one process).  Usage:
  python scripts/kbench.py [--workload c2] [--groups N] [--rounds 10]
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
    ap.add_argument("--groups", type=int, default=1 << 20)
    ap.add_argument("--replicas", type=int, default=3)
    ap.add_argument("--entries", type=int, default=64)
    ap.add_argument("--payload", type=int, default=64)
    ap.add_argument("--payload-max", type=int, default=0)
    ap.add_argument("--ring", type=int, default=16384)
    ap.add_argument("--history", type=int, default=16)
    ap.add_argument("--history-max", type=int, default=0, help="history commands at most this long (C3: 64)")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--cid-mix", action="store_true", help="STABLE / EXTENDED / TRANSIT configurations (C5)")
    args = ap.parse_args()
    import torch

    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi
    eng = pkg.Engine(0)
    lib = eng.lib
    G, R = args.groups, args.replicas
    pmax = args.payload_max or args.payload
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(args.ring))
    cfg = pkg.batch.gen_cfg(seed=2026, n_entries=args.entries, n_history=args.history, len_min=args.payload,
                            len_max=pmax, ring_len=args.ring, p_full_ack=0.9, straggler=True,
                            cid_mix=args.cid_mix, hist_len_max=args.history_max)
    s = torch.cuda.current_stream()
    sp = C.c_void_p(s.cuda_stream)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    eng.gen(db, cfg)
    t1.record()
    torch.cuda.synchronize()
    gen_ms = t0.elapsed_time(t1)

    bw = db.struct()
    bl = db.struct()
    bl.flags = abi.BATCH_LANE_IMPL
    bs = db.struct()
    bs.flags = abi.BATCH_SHORT_WALKS
    bv = db.struct()
    bv.flags = abi.BATCH_VAR_LEN
    out = eng.alloc_commit_out(G, 15 | abi.COMMIT_LAST_IT | abi.COMMIT_VOTE | abi.COMMIT_RANK)
    o = eng.commit_struct(out)
    vo = {"won": eng._z(G, torch.uint8), "vote_count": eng._z(G, torch.uint8, 2),
          "new_commit": eng._z(G, torch.int64), "voters": eng._z(G, torch.int16)}
    vos = abi.VoteOut(won=vo["won"].data_ptr(), vote_count=vo["vote_count"].data_ptr(),
                      new_commit=vo["new_commit"].data_ptr(), voters=vo["voters"].data_ptr())
    pout = {"new_head": eng._z(G, torch.int64), "append_head": eng._z(G, torch.uint8),
            "min_apply": eng._z(G, torch.int64)}
    W, CK, MD, PR = abi.COMMIT_WALK, abi.COMMIT_CHECKSUM, abi.COMMIT_MEDIAN, abi.COMMIT_PRUNE

    def step_separate(bs_):
        lib.apus_commit_batch(eng.ctx, C.byref(bs_), C.byref(o), W | CK, sp)
        lib.apus_commit_batch(eng.ctx, C.byref(bs_), C.byref(o), MD, sp)
        return eng.log_pruning(db, out=pout, bstruct=bs_)
    LIT, VT, RK = abi.COMMIT_LAST_IT, abi.COMMIT_VOTE, abi.COMMIT_RANK
    # the failover pass on the generator's local (idx, term) (no walk: the
    # tail alone), and C5's whole step as one call or as the round-3 calls
    bf = db.struct()
    bf.flags = abi.BATCH_SHORT_WALKS
    bfl = db.struct()
    bfl.flags = abi.BATCH_SHORT_WALKS
    bfl.last_idx_term = out["last_idx_term"].data_ptr()

    def step_calls():
        lib.apus_commit_batch(eng.ctx, C.byref(bs), C.byref(o), W | CK | MD | PR | LIT, sp)
        lib.apus_vote_batch(eng.ctx, C.byref(bs), C.byref(o.vote), sp)
        return lib.apus_vote_rank_batch(eng.ctx, C.byref(bfl), C.byref(o.rank), sp)
    cases = {
        "tail": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bw), C.byref(o), MD | PR, sp),
        "fail_tail": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bf), C.byref(o), VT | RK, sp),
        "tail_with_fail": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bf), C.byref(o), MD | PR | VT | RK, sp),
        "short_step_fused": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bs), C.byref(o),
                                                          W | CK | MD | PR | LIT | VT | RK, sp),
        "short_step_calls": step_calls,
        # bench.py's step: walk + checksum + median + pruning as one call (the
        # walk, then one tail launch) or as three calls (round 2)
        "step_fused": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bw), C.byref(o), W | CK | MD | PR, sp),
        "step_separate": lambda: step_separate(bw),
        "short_step_separate": lambda: step_separate(bs),
        "wave_walk_checksum": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bw), C.byref(o), W | CK, sp),
        "wave_walk": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bw), C.byref(o), W, sp),
        "var_walk_checksum": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bv), C.byref(o), W | CK, sp),
        "var_walk": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bv), C.byref(o), W, sp),
        "short_walk_checksum": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bs), C.byref(o), W | CK, sp),
        "short_walk": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bs), C.byref(o), W, sp),
        "lane_walk_checksum": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bl), C.byref(o), W | CK, sp),
        "lane_walk": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bl), C.byref(o), W, sp),
        "median": lambda: lib.apus_commit_batch(eng.ctx, C.byref(bw), C.byref(o), MD, sp),
        "vote_tally": lambda: lib.apus_vote_batch(eng.ctx, C.byref(bw), C.byref(vos), sp),
        "prune": lambda: eng.log_pruning(db, out=pout, bstruct=bw),
    }
    # ---- a9 / a8 / a6: NC determinants of every group's [commit, end), then
    # per follower a copy whose terms match a prefix m_r ~ U[0, E] and differ
    # after it, validated against the local log
    want0 = set(args.only.split(",")) if args.only else None
    if want0 is None or want0 & {"nc_build", "nc_build_quad", "nc_build_lane", "validate", "validate_lead", "vote_rank",
                                 "last_idx_term", "last_idx_term_lane"}:
        E, F = args.entries, R - 1
        nc_dets = eng._z(G, torch.uint8, E * 24)
        nc_len = eng._z(G, torch.int32)
        cases["nc_build"] = lambda: lib.apus_nc_build_batch(eng.ctx, C.byref(bw), C.c_void_p(nc_dets.data_ptr()), E,
                                                            C.c_void_p(nc_len.data_ptr()), sp)
        cases["nc_build_quad"] = lambda: lib.apus_nc_build_batch(eng.ctx, C.byref(bv), C.c_void_p(nc_dets.data_ptr()),
                                                                 E, C.c_void_p(nc_len.data_ptr()), sp)
        cases["nc_build_lane"] = lambda: lib.apus_nc_build_batch(eng.ctx, C.byref(bl), C.c_void_p(nc_dets.data_ptr()),
                                                                 E, C.c_void_p(nc_len.data_ptr()), sp)
        cases["nc_build"]()
        torch.cuda.synchronize()
        gq = torch.Generator(device="cuda").manual_seed(11)
        dv = nc_dets.view(torch.int64).view(G, 1, E, 3).repeat(1, F, 1, 1).contiguous()
        m_r = torch.randint(0, E + 1, (G, F, 1), device="cuda", generator=gq)
        ar = torch.arange(E, device="cuda").view(1, 1, E)
        dv[..., 1] += (ar >= m_r).to(torch.int64)
        v_dets = dv.view(torch.uint8).view(-1)
        v_len = nc_len.view(G, 1).repeat(1, F).contiguous().view(-1)
        selfv = db.arrays["self_idx"].view(G, 1).to(torch.int64)
        fol = (selfv + 1 + torch.arange(F, device="cuda").view(1, F)) % R
        v_fol = fol.to(torch.uint8).contiguous().view(-1)
        v_out = eng._z(G, torch.int64, F)
        ncb = abi.NcBatch(n_followers=F, max_dets=E, dets=v_dets.data_ptr(), det_len=v_len.data_ptr(),
                          follower=v_fol.data_ptr())
        cases["validate"] = lambda: lib.apus_validate_batch(eng.ctx, C.byref(bw), C.byref(ncb),
                                                            C.c_void_p(v_out.data_ptr()), sp)
        # bench.py's C3 form: the leader's own determinants (the walk's NC
        # epilogue) given, so a follower determinant at the leader's offset
        # needs no header gather
        ncl = abi.NcBatch(n_followers=F, max_dets=E, dets=v_dets.data_ptr(), det_len=v_len.data_ptr(),
                          follower=v_fol.data_ptr(), leader_dets=nc_dets.data_ptr(),
                          leader_len=nc_len.data_ptr(), leader_max=E)
        cases["validate_lead"] = lambda: lib.apus_validate_batch(eng.ctx, C.byref(bw), C.byref(ncl),
                                                                 C.c_void_p(v_out.data_ptr()), sp)
        # a6 with preallocated outputs; the local (idx, term) of every group
        # (dare_server.c:1598-1620) is its own case
        lit = eng._z(G, torch.int64, 2)
        br = db.struct()
        br.last_idx_term = lit.data_ptr()
        ro = {"outcome": eng._z(G, torch.uint8), "new_sid": eng._z(G, torch.int64),
              "new_cid": eng._z(G, torch.uint8, 16), "cleared": eng._z(G, torch.int16)}
        rso = abi.RankOut(outcome=ro["outcome"].data_ptr(), new_sid=ro["new_sid"].data_ptr(),
                          new_cid=ro["new_cid"].data_ptr(), cleared=ro["cleared"].data_ptr())
        cases["last_idx_term"] = lambda: lib.apus_last_idx_term_batch(eng.ctx, C.byref(bw),
                                                                      C.c_void_p(lit.data_ptr()), sp)
        cases["vote_rank"] = lambda: lib.apus_vote_rank_batch(eng.ctx, C.byref(br), C.byref(rso), sp)
        cases["last_idx_term_lane"] = lambda: lib.apus_last_idx_term_batch(eng.ctx, C.byref(bl),
                                                                           C.c_void_p(lit.data_ptr()), sp)
    # ---- 8f.1: append M = --entries SEND messages of --payload bytes per
    # group (messages generated on the device), then every follower persists
    # them; state / cursors are restored outside the timed region
    want = set(args.only.split(",")) if args.only else set()
    # ---- 8f.2: apply scan over [head, commit) (the history entries) and the
    # config scan over [head, end); state restored outside the timed region
    if not want or want & {"apply", "config_scan"}:
        stv0 = db.arrays["state"].view(torch.int64).view(G, 8)
        st_a = db.arrays["state"].clone()
        st_a.view(torch.int64).view(G, 8)[:, 1] = stv0[:, 0]            # apply = head
        MC = 4
        a_t = {"req_id": eng._z(G, torch.int64), "clt_id": eng._z(G, torch.int16),
               "last_applied": eng._z(G, torch.int64, 3), "last_csm_idx": eng._z(G, torch.int64),
               "n_applied": eng._z(G, torch.int32), "departed": eng._z(G, torch.int16),
               "events": eng._z(G, torch.uint8), "cfg_entries": eng._z(G, torch.uint8, 24 * MC),
               "cfg_payload": eng._z(G, torch.uint8, 16 * MC), "n_cfg": eng._z(G, torch.int32)}
        aio = abi.ApplyIO(max_cfg=MC, **{k: v.data_ptr() for k, v in a_t.items()})
        c_off = stv0[:, 0].clone()
        c_t = {"cid_offset": c_off.clone(), "cid_idx": eng._z(G, torch.int64), "req_id": eng._z(G, torch.int64),
               "clt_id": eng._z(G, torch.int16), "departed": eng._z(G, torch.int16)}
        cio = abi.ConfigIO(**{k: v.data_ptr() for k, v in c_t.items()})

        def do_apply():
            db.arrays["state"].copy_(st_a)
            t0.record()
            lib.apus_apply_batch(eng.ctx, C.byref(bw), C.byref(aio), sp)
            t1.record()
            return "timed"

        def do_config():
            db.arrays["state"].copy_(st_a)
            c_t["cid_offset"].copy_(c_off)
            t0.record()
            lib.apus_config_scan_batch(eng.ctx, C.byref(bw), C.byref(cio), sp)
            t1.record()
            return "timed"
        cases["apply"] = do_apply
        cases["config_scan"] = do_config
    # ---- 8f.2 step machine: every server at a random step 1..6 with its send
    # flag armed, NC buffers = the group's own determinants (a SET_END server
    # walks all of them), completions for half the pairs; the mutated columns
    # are restored outside the timed region
    if not want or want & {"lr_completion", "log_adjust"}:
        E = args.entries
        gq = torch.Generator(device="cuda").manual_seed(13)
        lr_dets = eng._z(G, torch.uint8, E * 24)
        lr_dl = eng._z(G, torch.int32)
        lib.apus_nc_build_batch(eng.ctx, C.byref(bw), C.c_void_p(lr_dets.data_ptr()), E,
                                C.c_void_p(lr_dl.data_ptr()), sp)
        lr_nc = lr_dets.view(torch.int64).view(G, 1, E, 3).repeat(1, R, 1, 1).contiguous()
        lr_len = lr_dl.to(torch.int64).view(G, 1).repeat(1, R).contiguous()
        step0 = torch.randint(1, 7, (G * R,), device="cuda", generator=gq).to(torch.uint8)
        lr_t = {"send_flag": torch.ones(G * R, dtype=torch.uint8, device="cuda"),
                "send_count": torch.randint(0, 3, (G * R,), device="cuda", generator=gq).to(torch.uint8),
                "wc": (torch.randint(0, 2, (G * R,), device="cuda", generator=gq)).to(torch.uint8),
                "ssn": eng._z(G, torch.int64), "post": eng._z(G, torch.uint8, R)}
        lio = abi.LrIO(send_flag=lr_t["send_flag"].data_ptr(), send_count=lr_t["send_count"].data_ptr(),
                       wc=lr_t["wc"].data_ptr(), rc_connected=None, nc_len=lr_len.data_ptr(),
                       nc_dets=lr_nc.data_ptr(), ssn=lr_t["ssn"].data_ptr(), post=lr_t["post"].data_ptr(),
                       max_dets=E)
        st_l = db.arrays["state"].clone()
        sc0 = lr_t["send_count"].clone()

        def lr_reset():
            db.arrays["state"].copy_(st_l)
            db.arrays["lr_step"].copy_(step0)
            lr_t["send_flag"].fill_(1)
            lr_t["send_count"].copy_(sc0)

        def do_completion():
            lr_reset()
            t0.record()
            lib.apus_lr_completion_batch(eng.ctx, C.byref(bw), C.byref(lio), sp)
            t1.record()
            return "timed"

        def do_adjust():
            lr_reset()
            t0.record()
            lib.apus_log_adjust_batch(eng.ctx, C.byref(bw), C.byref(lio), sp)
            t1.record()
            return "timed"
        cases["lr_completion"] = do_completion
        cases["log_adjust"] = do_adjust
    if want & {"append", "append_per_group", "persist"}:
        M, L = args.entries, args.payload
        n = G * M
        need = 2 + L
        g = torch.Generator(device="cuda").manual_seed(7)
        ent = torch.zeros(n, 24, dtype=torch.uint8, device="cuda")
        e64 = ent.view(torch.int64).view(n, 3)
        e64[:, 0] = torch.randint(0, 1 << 62, (n,), device="cuda", generator=g)
        e64[:, 1] = torch.arange(n, device="cuda", dtype=torch.int64) * need
        e64[:, 2] = torch.randint(0, 1 << 16, (n,), device="cuda", generator=g) | (5 << 16)
        payload = torch.randint(0, 256, (n * need,), dtype=torch.uint8, device="cuda", generator=g)
        pv = payload.view(n, need)
        pv[:, 0] = L & 0xFF
        pv[:, 1] = L >> 8
        st0 = db.arrays["state"].clone()
        out_idx = eng._z(G, torch.int64, M)
        out_last = eng._z(G, torch.int64)
        ai = abi.AppendIn(entries=ent.data_ptr(), n_entries=None, term=None, payload=payload.data_ptr(),
                          payload_bytes=payload.numel(), max_entries=M)
        ao = abi.AppendOut(idx=out_idx.data_ptr(), last_idx=out_last.data_ptr())
        stv = db.arrays["state"].view(torch.int64).view(G, 8)
        oe0 = stv[:, 3].repeat_interleave(R).contiguous()      # each copy resumes at the pre-append end
        old_end = oe0.clone()
        pin = abi.PersistIn(old_end=old_end.data_ptr(), limit=None)

        ai_pg = abi.AppendIn(entries=ent.data_ptr(), n_entries=None, term=None, payload=payload.data_ptr(),
                             payload_bytes=payload.numel(), max_entries=M, flags=abi.APPEND_PER_GROUP)

        def do_append(a=ai):
            db.arrays["state"].copy_(st0)
            t0.record()
            lib.apus_append_batch(eng.ctx, C.byref(bw), C.byref(a), C.byref(ao), sp)
            t1.record()
            return "timed"

        def do_persist():
            old_end.copy_(oe0)
            t0.record()
            lib.apus_persist_batch(eng.ctx, C.byref(bw), C.byref(pin), sp)
            t1.record()
            return "timed"
        cases["append"] = do_append
        cases["append_per_group"] = lambda: do_append(ai_pg)
        cases["persist"] = do_persist
    # ---- 8f.3: the proxy's stable-storage records of every entry from head
    # (store: cursor and lengths reset outside the timed region), then the
    # snapshots replayed (load)
    if want & {"records_store", "records_load", "records_store_lane", "records_load_lane"}:
        RC = 64 * (args.entries + 16) + 64
        r_cur0 = db.arrays["state"].view(torch.int64).view(G, 8)[:, 0].clone()
        r_cur = r_cur0.clone()
        r_dump = eng._z(G, torch.uint8, RC)
        r_len = eng._z(G, torch.int32)
        r_n = eng._z(G, torch.int32)
        rio = abi.RecordsIO(cursor=r_cur.data_ptr(), dump=r_dump.data_ptr(), cap=RC, dump_len=r_len.data_ptr(),
                            n_records=r_n.data_ptr())
        MP = args.entries + 16
        l_out = {"plan": eng._z(G, torch.uint8, 16 * MP), "n_records": eng._z(G, torch.int32),
                 "counts": eng._z(G, torch.int32, 3), "status": eng._z(G, torch.int32)}
        rlio = abi.RecordsLoadIO(dump=r_dump.data_ptr(), stride=RC, size=r_len.data_ptr(), n=G,
                                plan=l_out["plan"].data_ptr(), max_plan=MP, n_records=l_out["n_records"].data_ptr(),
                                counts=l_out["counts"].data_ptr(), status=l_out["status"].data_ptr())

        def do_rstore():
            r_cur.copy_(r_cur0)
            r_len.zero_()
            t0.record()
            lib.apus_records_store_batch(eng.ctx, C.byref(bw), C.byref(rio), sp)
            t1.record()
            return "timed"
        lio_lane = abi.RecordsLoadIO(dump=r_dump.data_ptr(), stride=RC, size=r_len.data_ptr(), n=G,
                                     plan=l_out["plan"].data_ptr(), max_plan=MP, flags=abi.BATCH_LANE_IMPL,
                                     n_records=l_out["n_records"].data_ptr(), counts=l_out["counts"].data_ptr(),
                                     status=l_out["status"].data_ptr())

        def do_rstore_lane():
            r_cur.copy_(r_cur0)
            r_len.zero_()
            t0.record()
            lib.apus_records_store_batch(eng.ctx, C.byref(bl), C.byref(rio), sp)
            t1.record()
            return "timed"
        cases["records_store"] = do_rstore
        cases["records_store_lane"] = do_rstore_lane
        cases["records_load"] = lambda: lib.apus_records_load_batch(eng.ctx, C.byref(rlio), sp)
        cases["records_load_lane"] = lambda: lib.apus_records_load_batch(eng.ctx, C.byref(lio_lane), sp)
    if args.only:
        cases = {k: v for k, v in cases.items() if k in want}
    times = {k: [] for k in cases}
    for r in range(args.rounds):
        for k, f in cases.items():
            if k in ("append", "append_per_group", "persist", "apply", "config_scan", "lr_completion", "log_adjust",
                     "records_store", "records_store_lane"):  # they record their own events
                f()
                torch.cuda.synchronize()
                times[k].append(t0.elapsed_time(t1))
                continue
            t0.record()
            rc = f()
            t1.record()
            torch.cuda.synchronize()
            assert rc in (0, None) or isinstance(rc, dict), (k, rc)
            times[k].append(t0.elapsed_time(t1))
    per_group = args.entries * (64 + (args.payload + pmax) / 2) + 82
    res = {"groups": G, "gen_ms": gen_ms}
    eng.stats_reset()
    lib.apus_commit_batch(eng.ctx, C.byref(bw), C.byref(o), W | CK, sp)
    res["wave_stats"] = [int(x) for x in eng.stats()]
    # append: per message 24 B record + 2 + L payload read, 64 - 8 + L bytes
    # of the entry written (sender@27 and 41..47 untouched); persist: per
    # entry and copy the type / cmd.len bytes read and one byte written,
    # counted as one 64-B header line per entry per copy
    alg = {"append": G * args.entries * (24 + 2 + args.payload + 56 + args.payload) + G * 64,
           "persist": G * R * args.entries * 64,
           # (R-1) E 24 determinants + E 16 local idx/term + 8 (R-1) out
           "validate": G * ((R - 1) * args.entries * 24 + args.entries * 16 + 8 * (R - 1)),
           # per entry walked: its 64-B header line read, a 24-B determinant written
           "nc_build": G * args.entries * (64 + 24),
           "nc_build_quad": G * args.entries * (64 + 24),
           "nc_build_lane": G * args.entries * (64 + 24),
           # 40R vote_req + 8R + 8 + 16 + 64 in, 1 + 8 + 16 + 2 out, + last (idx, term)
           "vote_rank": G * (48 * R + 88 + 27),
           # state row + the header of every entry walked from commit to end
           # (the last one's (idx, term) among them), 16 B out
           "last_idx_term": G * (64 + args.entries * 64 + 16),
           "last_idx_term_lane": G * (64 + args.entries * 64 + 16),
           # per entry walked one 64-B header line; state row in, ~40 B out
           "apply": G * (16 * 64 + 64 + 40),
           "config_scan": G * ((16 + args.entries) * 64 + 64 + 32),
           # per pair wc / step / send_flag / send_count read, 3 bytes written
           "lr_completion": G * R * 7,
           # per group state row, self, ssn r/w; per server fail / flag / step /
           # post bytes, vote_ack, nc_len, remote commit / end; the SET_END
           # servers (1/6) walk E determinants + E 16-B local (idx, term)
           "log_adjust": G * (64 + 1 + 16 + R * (4 + 32)) + G * R * args.entries * 40 // 6,
           # every entry from head: its header line read, a 24-B SEND record written (R <= 4)
           "records_store": G * (args.entries + 16) * (64 + 24) + G * 24,
           # every 24-B record read, a 16-B plan entry written
           "records_load": G * (args.entries + 16) * (24 + 16) + G * 16}
    alg["records_store_lane"], alg["records_load_lane"] = alg["records_store"], alg["records_load"]
    alg["append_per_group"] = alg["append"]
    alg["validate_lead"] = alg["validate"]
    for k, v in times.items():
        med = float(np.median(v[1:] if len(v) > 1 else v))
        res[k] = {"ms_median": med, "ms_min": float(np.min(v)),
                  "GBps_alg_commit": per_group * G / (med * 1e-3) / 1e9}
        if k in alg:
            res[k]["GBps_alg"] = alg[k] / (med * 1e-3) / 1e9
            res[k]["Mentries_per_s"] = G * args.entries / (med * 1e-3) / 1e6
    print(json.dumps(res, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
