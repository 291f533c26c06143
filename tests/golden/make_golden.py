"""Generate tests/golden/*.json (run in the build container, needs /root/reference).

Every expected value here comes from oracle/_ref/libapusref.so: the
reference's own src/include/dare/dare_log.h compiled from /root/reference
(log_append_entry builds the logs; log_get_entry / log_fit_entry /
log_entry_len / log_is_offset_larger / log_get_tail / log_entries_to_nc_buf /
log_find_remote_end_offset evaluate them) with the hot-path loops of
dare_ibv_rc.c / dare_server.c restated on those primitives.

1. scenarios.json  -- the reference results SURVEY.md §8c records, rebuilt:
   commit 640 (R=3, 5 of 8 128-B entries acked), wrap commit 128 (len 1000,
   ghost header at 896), 7-replica vote 3 acks win / 2 acks lose, TRANSIT 5->7
   {1,2} lose / {1,2,5} win, find_remote_end 192 at the first term mismatch,
   pruning head 128 + HEAD entry (end 448).
2. vectors.json    -- seeded synthetic batches (the generator spec in
   oracle/apus_oracle.c); stores a SHA-256 of the generated inputs and the
   per-group outputs of the reference-composed oracle, plus each group's
   build-defined checksum (the reference has none): zlib's
   Adler-32 over the entries the reference's log_entries_to_nc_buf lists from
   commit to end, each entry's bytes [0, 27) ++ 21 zero bytes ++ [48, len),
   taken from where log_fit_entry places it -- computed here with zlib, not
   with the oracle's or the kernels' Adler code.

3. records.json    -- the proxy's stable-storage records (round 4, records()).
4. tail_vectors.json -- the publish and force_log_pruning (round 5, tail()).
5. win_vectors.json  -- poll_vote_count whole: the tally and the election-win
   transition (round 6, win()).

Usage: python tests/golden/make_golden.py [scenarios] [vectors] [records] [tail] [win]
"""
import ctypes as C
import hashlib
import json
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
import apus_pkg  # noqa: E402

orc = apus_pkg.load_oracle()
pkg = apus_pkg.load_package()


def P(a):
    return C.c_void_p(a.ctypes.data)


def ref():
    r = orc.ref()
    if r is None:
        raise SystemExit("oracle/_ref missing: run `make -C oracle` with /root/reference present")
    return r


def cid_bytes(epoch=0, s0=3, s1=0, state=0, bitmask=0x1FFF):
    return np.frombuffer(np.array([(epoch, s0, s1, state, 0, bitmask)],
                                  dtype=pkg.batch.CID_DT).tobytes(), np.uint8).copy()


def build_log(ln, start, types, clens, terms=None):
    """real log_append_entry; returns ring image, final state, entry offsets"""
    R = ref()
    n = len(types)
    t = np.array(types, np.uint8)
    c = np.array(clens, np.uint16)
    tm = np.array(terms if terms is not None else [1] * n, np.uint64)
    ring = np.zeros(ln + 64, np.uint8)
    st = np.zeros(6, np.uint64)
    off = np.zeros(n, np.uint64)
    assert R.ref_append_seq(ln, start, n, P(t), P(c), P(tm), P(cid_bytes()), P(ring), P(st), P(off)) == 0
    return ring, st, [int(x) for x in off]


def scenarios():
    R = ref()
    out = []

    # A: R=3, eight 128-B SEND entries, follower 1 acked the first five
    ring, st, off = build_log(4096, 4096, [5] * 8, [64] * 8)
    for k in range(5):
        ring[off[k] + 28 + 1] = 1
    st6 = np.array([0, 0, 0, st[3], st[4], 4096], np.uint64)
    cm = C.c_int(0)
    got = R.ref_commit_walk(P(ring), P(st6), P(cid_bytes(s0=3)), 0, C.byref(cm))
    out.append(dict(name="commit_640", kind="commit", ring_len=4096, types=[5] * 8, clens=[64] * 8, start=4096,
                    acks={"1": [0, 1, 2, 3, 4]}, state=[int(x) for x in st6], cid=[0, 3, 0, 0, 0x1FFF], self=0,
                    expect_commit=int(got), expect_committed=cm.value))
    assert got == 640

    # B: len 1000, one 128-B entry appended at end 896: ghost header at 896, entry at 0
    ring, st, off = build_log(1000, 896, [5], [64])
    assert off == [0] and ring[896 + 26] == 5
    ring[0 + 28 + 1] = 1
    st6 = np.array([0, 0, 896, st[3], st[4], 1000], np.uint64)
    got = R.ref_commit_walk(P(ring), P(st6), P(cid_bytes(s0=3)), 0, C.byref(cm))
    out.append(dict(name="wrap_commit_128", kind="commit", ring_len=1000, types=[5], clens=[64], start=896,
                    acks={"1": [0]}, state=[int(x) for x in st6], cid=[0, 3, 0, 0, 0x1FFF], self=0,
                    expect_commit=int(got), expect_committed=cm.value))
    assert got == 128

    # C/D: vote tallies
    for name, sizes, state, acks, want in [("vote7_3acks", (7, 0), 0, [1, 2, 3], 1),
                                           ("vote7_2acks", (7, 0), 0, [1, 2], 0),
                                           ("transit_5_7_acks12", (5, 7), 1, [1, 2], 0),
                                           ("transit_5_7_acks125", (5, 7), 1, [1, 2, 5], 1)]:
        ln = 4096
        va = np.full(13, ln, np.uint64)
        for a in acks:
            va[a] = 0
        st6 = np.array([0, 0, 0, 64, 0, ln], np.uint64)
        vc = np.zeros(2, np.uint8)
        nc = C.c_uint64(0)
        won = R.ref_vote_tally(P(st6), P(cid_bytes(s0=sizes[0], s1=sizes[1], state=state)), 0, P(va), P(vc),
                               C.byref(nc))
        assert won == want
        out.append(dict(name=name, kind="vote", ring_len=ln, state=[int(x) for x in st6],
                        cid=[0, sizes[0], sizes[1], state, 0x1FFF], self=0, vote_ack=[int(x) for x in va],
                        expect_won=won, expect_vc=[int(vc[0]), int(vc[1])], expect_commit=nc.value))

    # E: four 64-B entries; the follower's 4th determinant has another term
    ring, st, off = build_log(4096, 4096, [0, 0, 0, 0], [0, 0, 0, 0], terms=[3, 3, 3, 3])
    st6 = np.array([0, 0, 0, st[3], st[4], 4096], np.uint64)
    d = np.array([[1, 3, 0], [2, 3, 64], [3, 3, 128], [4, 4, 192]], np.uint64).ravel()
    got = R.ref_find_remote_end(P(ring), P(st6), P(d), 4)
    assert got == 192
    out.append(dict(name="find_remote_end_192", kind="validate", ring_len=4096, types=[0] * 4, clens=[0] * 4,
                    terms=[3] * 4, start=4096, state=[int(x) for x in st6], dets=[int(x) for x in d],
                    expect_end=int(got)))

    # F: three 128-B entries, replicas applied up to 128 / 256: head 0 -> 128, HEAD entry appended
    ring, st, off = build_log(4096, 4096, [5, 5, 5], [64, 64, 64])
    st6 = np.array([0, 384, 384, st[3], st[4], 4096], np.uint64)
    ap = np.array([384, 128, 256] + [0] * 10, np.uint64)
    nh = C.c_uint64(0)
    app = C.c_int(0)
    mn = R.ref_min_apply(P(ring), P(st6), P(cid_bytes(s0=3, bitmask=0x7)), P(ap), 0, C.byref(nh), C.byref(app))
    assert nh.value == 128 and app.value == 1
    ring2, st2, _ = build_log(4096, 4096, [5, 5, 5, 3], [64, 64, 64, 0])
    out.append(dict(name="prune_head_128", kind="prune", ring_len=4096, types=[5, 5, 5], clens=[64] * 3,
                    start=4096, state=[int(x) for x in st6], cid=[0, 3, 0, 0, 7], apply_offsets=[384, 128, 256],
                    expect_min=int(mn), expect_head=nh.value, expect_append=app.value,
                    expect_end_after_head_entry=int(st2[3])))
    assert int(st2[3]) == 448
    return out


VECTOR_CFGS = {
    "c2": (3, dict(seed=501, n_entries=64, n_history=16, len_min=64, len_max=64, ring_len=16384, p_full_ack=0.9,
                   straggler=True)),
    "c2_skew": (5, dict(seed=502, n_entries=64, n_history=16, len_min=64, len_max=64, ring_len=16384,
                        p_full_ack=0.5, garbage_reply=0.02, self_random=True, straggler=True)),
    "c3_var": (5, dict(seed=503, n_entries=64, n_history=8, len_min=64, len_max=4096, ring_len=600000,
                       straggler=True, p_full_ack=0.8)),
    "c5_reconf": (7, dict(seed=505, n_entries=16, n_history=8, len_min=32, len_max=64, ring_len=8192,
                          cid_mix=True, self_random=True, p_vote_ack=0.6, type_mix=True)),
    "tiny_wrap": (5, dict(seed=506, n_entries=5, n_history=1, len_min=3, len_max=45, ring_len=777,
                          cid_mix=True, self_random=True, p_full_ack=0.0, straggler=True)),
    # round 3: the C4 one-GPU shape (16-entry batches on 2,448-B rings: most wrap), mixed types and
    # lengths, spans of several 9-KiB windows, and small 16-B aligned rings that wrap inside a window
    "c4_short": (5, dict(seed=507, n_entries=16, n_history=2, len_min=64, len_max=64, ring_len=2448,
                         p_full_ack=0.9, straggler=True)),
    "mixed_small": (7, dict(seed=508, n_entries=24, n_history=8, len_min=0, len_max=90, ring_len=6000,
                            type_mix=True, cid_mix=True, self_random=True, garbage_reply=0.05, p_full_ack=0.5)),
    "multiwin": (3, dict(seed=509, n_entries=40, n_history=4, len_min=200, len_max=1000, ring_len=65536,
                         p_full_ack=0.7, straggler=True)),
    "wrap_aligned": (5, dict(seed=510, n_entries=12, n_history=3, len_min=0, len_max=100, ring_len=4096,
                             type_mix=True, cid_mix=True, self_random=True, p_full_ack=0.6, straggler=True,
                             garbage_reply=0.03)),
}
G_VEC = 160
N_DETS = 1024          # the reference's nc_buf capacity (dare_log.h: dare_nc_buf_t.entries[1024])


def image_digest(ring, st6, dets, n):
    """zlib.adler32 of the checksum image of the n entries the reference's
    log_entries_to_nc_buf recorded (offset before the ghost test)"""
    ln = int(st6[5])
    img = bytearray()
    for k in range(n):
        o = int(dets[3 * k + 2])
        t = int(ring[o + 26])
        clen = int(ring[o + 48]) | (int(ring[o + 49]) << 8)
        el = 64 if t in (0, 2, 3) else 64 + clen          # log_entry_len: NOOP / CONFIG / HEAD are bare
        if ln - o < el:                                    # !log_fit_entry: the entry lies at 0
            o = 0
        e = bytes(ring[o:o + el])
        img += e[:27] + bytes(21) + e[48:]
    return zlib.adler32(bytes(img)) & 0xFFFFFFFF


def input_digest(hb):
    h = hashlib.sha256(hb.ring.tobytes())
    for k in sorted(hb.arrays):
        h.update(hb.arrays[k].tobytes())
    return h.hexdigest()


def vectors():
    R_ = ref()
    res = {}
    for name, (R, kw) in VECTOR_CFGS.items():
        cfg = pkg.batch.gen_cfg(**kw)
        hb = orc.host_batch(G_VEC, R, kw["ring_len"])
        orc.gen(hb, cfg)
        ent = {"replicas": R, "groups": G_VEC, "cfg": kw, "input_sha256": input_digest(hb), "groups_out": []}
        ap0 = hb.apply_offsets.copy()
        for g in range(G_VEC):
            s = hb.state[g]
            st6 = np.array([s["head"], s["apply"], s["commit"], s["end"], s["tail"], s["len"]], np.uint64)
            cid = np.frombuffer(hb.state[g:g + 1].tobytes()[48:64], np.uint8).copy()
            me = int(hb.self_idx[g])
            ring = hb.group_ring(g)
            cm = C.c_int(0)
            commit = R_.ref_commit_walk(P(ring), P(st6), P(cid), me, C.byref(cm))
            sl = slice(g * R, (g + 1) * R)
            # keep every array passed by address alive across the call
            rend, lrs, fc = hb.remote_end[sl].copy(), hb.lr_step[sl].copy(), hb.fail_count[sl].copy()
            med = R_.ref_median(P(st6), P(cid), me, P(rend), P(lrs), P(fc))
            vc = np.zeros(2, np.uint8)
            vcm = C.c_uint64(0)
            vack = hb.vote_ack[sl].copy()
            won = R_.ref_vote_tally(P(st6), P(cid), me, P(vack), P(vc), C.byref(vcm))
            lit = np.zeros(2, np.uint64)
            R_.ref_last_idx_term(P(ring), P(st6), P(lit))
            ns = C.c_uint64(0)
            ncid = np.zeros(16, np.uint8)
            clr = C.c_uint16(0)
            req = np.frombuffer(hb.vote_req[sl].tobytes(), np.uint64).copy()
            hbv = hb.hb[sl].copy()
            oc = R_.ref_vote_rank(P(st6), P(cid), me, int(hb.sid[g]), P(hbv), R, P(req), int(lit[0]),
                                  int(lit[1]), C.byref(ns), P(ncid), C.byref(clr))
            ap = ap0[sl].copy()
            nh = C.c_uint64(0)
            app = C.c_int(0)
            mn = R_.ref_min_apply(P(ring), P(st6), P(cid), P(ap), int(hb.prev_head[g]), C.byref(nh), C.byref(app))
            d = np.zeros(N_DETS * 3, np.uint64)
            nnc = R_.ref_nc_build(P(ring), P(st6), P(d), N_DETS)
            fre = R_.ref_find_remote_end(P(ring), P(st6), P(d), nnc) if nnc else None
            ent["groups_out"].append(dict(commit=int(commit), committed=cm.value, median=int(med), won=won,
                                          vc=[int(vc[0]), int(vc[1])], vote_commit=vcm.value, lit=[int(lit[0]),
                                          int(lit[1])], rank=oc, new_sid=ns.value, cleared=clr.value,
                                          min_apply=int(mn), new_head=nh.value, append=app.value,
                                          nc_len=int(nnc), find_end=None if fre is None else int(fre),
                                          digest=image_digest(ring, st6, d, int(nnc))))
        res[name] = ent
    return res


def tail():
    """tail_vectors.json (round 5) -- update_remote_logs' lazy remote-commit
    publish (dare_ibv_rc.c:1760-1822) and force_log_pruning
    (dare_server.c:2069-2122) from oracle/_ref: both bodies transcribed on the
    reference's own primitives (ref_compose.c, drift-checked) on the commit
    the reference-composed walk leaves, over tests/test_publish_force.py's
    batches (generated, then perturbed with its seeded rng); SHA-256 digests
    of every output and of every array the two write in place, the action
    counts, and the first groups' values in clear."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_publish_force as tp
    R_ = ref()
    abi = pkg.abi
    flags = abi.COMMIT_PUBLISH | abi.COMMIT_FORCE_PRUNE
    res = {}
    for ci, (kw, R) in enumerate(tp.FULL):
        hb = orc.host_batch(G_TAIL, R, kw["ring_len"])
        orc.gen(hb, pkg.batch.gen_cfg(**kw))
        tp.perturb(hb, np.random.default_rng(100 + ci))
        ent = {"replicas": R, "groups": G_TAIL, "cfg": kw, "input_sha256": input_digest(hb)}
        commit = np.zeros(G_TAIL, np.uint64)
        for g in range(G_TAIL):
            s = hb.state[g]
            st6 = np.array([s["head"], s["apply"], s["commit"], s["end"], s["tail"], s["len"]], np.uint64)
            cid = np.frombuffer(hb.state[g:g + 1].tobytes()[48:64], np.uint8).copy()
            cm = C.c_int(0)
            commit[g] = R_.ref_commit_walk(P(hb.group_ring(g)), P(st6), P(cid), int(hb.self_idx[g]), C.byref(cm))
        rq = np.arange(G_TAIL, dtype=np.uint64) + 7
        cl = (np.arange(G_TAIL) % 60000 + 3).astype(np.uint16)
        out, wm, bad = orc.ref_tail(hb, flags, commit, out=orc.tail_out(G_TAIL, flags, req_id=rq, clt_id=cl))
        sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()   # noqa: E731
        ent["commit_sha256"] = sha(commit)
        ent["out_sha256"] = {k: sha(out[k]) for k in ("new_head", "append_head", "min_apply", "publish", "ssn")}
        ent["force_sha256"] = {k: sha(v) for k, v in out["force"].items()}
        ent["after_sha256"] = {k: sha(hb.arrays[k]) for k in ("state", "apply_offsets", "remote_commit",
                                                               "prev_head")}
        ent["ring_after_sha256"] = sha(hb.ring)
        ent["watermark"], ent["corrupt"] = int(wm), int(bad)
        ent["actions"] = [int(x) for x in np.bincount(out["force"]["action"], minlength=3)]
        ent["first"] = [dict(publish=int(out["publish"][g]), action=int(out["force"]["action"][g]),
                             target=int(out["force"]["target"][g]), cfg_idx=int(out["force"]["cfg_idx"][g]),
                             new_head=int(out["new_head"][g]), append=int(out["append_head"][g]),
                             min_apply=int(out["min_apply"][g])) for g in range(8)]
        res[f"full{ci}"] = ent
    return res


G_TAIL = 384


WIN_OUT = ("cid_offset", "req_id", "clt_id", "last_applied", "last_csm_idx", "last_write_csm_idx", "outcome",
           "events", "departed", "n_applied", "n_cfg")
WIN_AFTER = ("state", "sid", "remote_commit", "lr_step", "apply_offsets", "prev_head")


def win():
    """win_vectors.json (round 6) -- poll_vote_count (dare_server.c:1327-1518)
    from oracle/_ref: the tally and the election-win transition transcribed
    whole on the reference's own primitives, log_append_entry and config
    macros (ref_compose.c region vote_count, drift-checked), over
    tests/test_vote_win.py's seeded batches; SHA-256 digests of the inputs,
    of every output and of every array it writes in place, the outcome
    counts, and the first groups' values in clear."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_vote_win as tw
    ref()
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()   # noqa: E731
    res = {}
    for name in tw.CASES:
        hb, io = tw.build(pkg, orc, name)
        ent = {"groups": hb.G, "replicas": hb.R, "input_sha256": input_digest(hb),
               "io_in_sha256": sha(np.concatenate([io[k].view(np.uint8) for k in sorted(io)]))}
        bad = orc.ref_vote_count(hb, io)
        ent["out_sha256"] = {k: sha(io[k]) for k in WIN_OUT}
        ent["after_sha256"] = {k: sha(hb.arrays[k]) for k in WIN_AFTER}
        ent["ring_after_sha256"] = sha(hb.ring)
        ent["corrupt"] = int(bad)
        ent["outcomes"] = [int(x) for x in np.bincount(io["outcome"], minlength=8)]
        ent["first"] = [dict(outcome=int(io["outcome"][g]), last_write_csm_idx=int(io["last_write_csm_idx"][g]),
                             cid_offset=int(io["cid_offset"][g]), events=int(io["events"][g]),
                             departed=int(io["departed"][g]), n_cfg=int(io["n_cfg"][g])) for g in range(8)]
        res[name] = ent
    return res


def records():
    """records.json (round 4) -- the proxy's stable-storage records from
    oracle/_ref: persist_new_entries' walk on the reference's dare_log.h
    handing every entry to stablestorage_save_request restated on the
    reference's proxy.h (store, oracle/ref_compose.c + oracle/ref_records.c),
    and stablestorage_load_records likewise (load), over the traces of
    tests/test_records.py (snapshots from head at each capacity), the
    known-answer dumps and the random snapshots; SHA-256 digests of every
    output array."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_records as tr
    ref()
    res = {"store": {}}
    for name, (R, G, kw) in tr.TRACES.items():
        hb = orc.host_batch(G, R, kw["ring_len"])
        orc.gen(hb, pkg.batch.gen_cfg(**kw))
        for cap in tr.GOLDEN_CAPS:
            cur = hb.state["head"].copy()
            dump, dl, n, bad = orc.ref_records_store(hb, cur, cap)
            e = tr.store_digests(dump, dl, n, cur, bad)
            e["input_sha256"] = tr.sha(hb.ring) + ":" + tr.sha(hb.state)
            e["load"] = tr.load_digests(orc.ref_records_load(dump, dl, tr.GOLDEN_PLAN))
            res["store"][f"{name}/{cap}"] = e
    dumps, sizes = tr.random_snapshots()
    res["load_random"] = {"dumps_sha256": tr.sha(dumps), "sizes_sha256": tr.sha(sizes),
                          "load": tr.load_digests(orc.ref_records_load(dumps, sizes, 32))}
    d, s_, _ = tr._known_dumps()
    res["load_known"] = tr.load_digests(orc.ref_records_load(d, s_, 8))
    return res


if __name__ == "__main__":
    only = sys.argv[1:]
    if not only or "scenarios" in only:
        with open(os.path.join(HERE, "scenarios.json"), "w") as f:
            json.dump(scenarios(), f, indent=1)
    if not only or "vectors" in only:
        with open(os.path.join(HERE, "vectors.json"), "w") as f:
            json.dump(vectors(), f)
    if not only or "tail" in only:
        with open(os.path.join(HERE, "tail_vectors.json"), "w") as f:
            json.dump(tail(), f, indent=1)
    if not only or "win" in only:
        with open(os.path.join(HERE, "win_vectors.json"), "w") as f:
            json.dump(win(), f, indent=1)
    if not only or "records" in only:
        with open(os.path.join(HERE, "records.json"), "w") as f:
            json.dump(records(), f, indent=1)
    print("wrote", only or "scenarios.json, vectors.json, records.json")
