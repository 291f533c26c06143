"""Full-size BASELINE configurations on one MI355X (C5 added in round 2).

C4 (BASELINE.json configs[3]): the per-GPU shard of 64M groups over 8 GPUs,
2^23 groups x R=5, 64 x 128-B entries (a 137-GB ring batch resident in HBM):
commit walk + Adler-32 + median and the pruning minimum / watermark.
C3 (configs[2]): one resident wave of the 10M-group batch, 2^19 groups x R=5,
entries of 64 B - 4 KB on 266.6-KiB rings (143 GB), straggler acks: commit walk
+ Adler-32 + median, the leader's NC determinants (log_entries_to_nc_buf) and
the followers' (idx, term) validation (log_find_remote_end_offset) against
perturbed copies.

The oracle cannot walk these batches whole in test time, so per-group
outputs are compared bit-exactly on sampled group ranges (the generator is
keyed by group id, so a host batch with gid_base = g0 holds exactly groups
g0.. of the device batch), and the whole batch is checked through
size-independent properties: the statistics equal the sums / minimum of the
per-group outputs.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def test_c4_shard_full_size(pkg, orc, eng):
    import torch
    abi = pkg.abi
    G, R, L = 1 << 23, 5, 16384
    kw = dict(seed=4004, n_entries=64, n_history=16, len_min=64, len_max=64, ring_len=L, p_full_ack=0.9,
              straggler=True)
    fields = ["state", "self_idx", "remote_end", "lr_step", "fail_count", "apply_offsets", "prev_head", "abs_base"]
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L), fields=fields)
    eng.gen(db, pkg.batch.gen_cfg(**kw))
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN
    eng.stats_reset()
    out = eng.update_remote_logs(db, flags)
    po = eng.log_pruning(db)
    torch.cuda.synchronize()
    st = eng.stats()
    n_ent = out["n_entries"].cpu().numpy().view(np.uint32)
    committed = out["committed"].cpu().numpy()
    assert st[abi.STAT_DECISIONS] == G
    assert st[abi.STAT_COMMITTED] == int(n_ent.astype(np.uint64).sum())
    assert st[abi.STAT_ADVANCED] == int((committed == 1).sum())
    assert st[abi.STAT_CORRUPT] == 0 and st[abi.STAT_SLOW] == 0
    # the pruning watermark is the minimum over every group of abs_base + new_head
    wm = (db.download("abs_base") + _u64(po["new_head"])).min()
    assert st[abi.STAT_MIN_WATERMARK] == int(wm)
    S = 2000
    for g0 in (0, G // 3 + 777, G - S):
        hb = orc.host_batch(S, R, L, fields=fields)
        orc.gen(hb, pkg.batch.gen_cfg(gid_base=g0, **kw))
        # the reference's own code, too
        assert _ref_groups(orc, hb, g0, 256, out, None, None, po) or not _REF_SO, "oracle/_ref built but not loaded"
        ref = orc.commit(hb, flags)
        sl = slice(g0, g0 + S)
        assert np.array_equal(_u64(out["new_commit"][sl]), ref["new_commit"]), g0
        assert np.array_equal(committed[sl], ref["committed"]), g0
        assert np.array_equal(n_ent[sl], ref["n_entries"]), g0
        assert np.array_equal(out["digest"][sl].cpu().numpy().view(np.uint32), ref["digest"]), g0
        assert np.array_equal(_u64(out["median"][sl]), ref["median"]), g0
        rp, _ = orc.prune(hb)
        assert np.array_equal(_u64(po["new_head"][sl]), rp["new_head"]), g0
        assert np.array_equal(po["append_head"][sl].cpu().numpy(), rp["append_head"]), g0
        assert np.array_equal(_u64(po["min_apply"][sl]), rp["min_apply"]), g0
    del db, out, po
    torch.cuda.empty_cache()


def _conn_of(g):
    """rc_connected of group g (numpy or torch int64 ids): all connected but
    every 7th group, whose bits come from the id"""
    h = (g * 2654435761) % (1 << 32)
    return ((h >> 8) % 7 == 0) * ((h >> 12) & 0xFFFF) + ((h >> 8) % 7 != 0) * 0xFFFF


def test_c4_shard_force_full_size(pkg, orc, eng):
    """the C4 shard (2^23 groups x R=5, 16-KiB rings) with the
    rings 81% full (64 new entries after 40 history entries): walk + Adler-32
    + median + update_remote_logs' publish, log->commit updated, then
    force_log_pruning on that log (its own call).  Whole batch: the statistics and the watermark
    equal the per-group sums / minimum, every outcome occurs, ssn moves exactly
    where something was posted; three sampled ranges bit-exact against the
    oracle on every output and every byte written in place."""
    import torch
    abi = pkg.abi
    G, R, L = 1 << 23, 5, 16384
    kw = dict(seed=4014, n_entries=64, n_history=40, len_min=64, len_max=64, ring_len=L, p_full_ack=0.9,
              straggler=True)
    fields = ["state", "self_idx", "remote_end", "remote_commit", "lr_step", "fail_count", "apply_offsets",
              "prev_head", "abs_base", "sid"]
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L), fields=fields)
    eng.gen(db, pkg.batch.gen_cfg(**kw))
    conn = db.add("rc_connected").view(torch.int16)
    conn.copy_(_conn_of(torch.arange(G, dtype=torch.int64, device="cuda")).to(torch.int16))
    flags = (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PUBLISH |
             abi.COMMIT_FORCE_PRUNE | abi.COMMIT_STATS_FRESH)
    out = eng.alloc_commit_out(G, flags)
    out["ssn"].copy_(torch.arange(G, dtype=torch.int64, device="cuda") * 2)
    out["force"]["req_id"].copy_(torch.arange(G, dtype=torch.int64, device="cuda") + 11)
    out["force"]["clt_id"].copy_((torch.arange(G, dtype=torch.int64, device="cuda") % 30000 + 1).to(torch.int16))
    eng.stats_reset()
    eng.commit_then_force(db, flags, out=out)
    torch.cuda.synchronize()
    st = eng.stats()
    n_ent = out["n_entries"].cpu().numpy().view(np.uint32)
    committed = out["committed"].cpu().numpy()
    act = out["force"]["action"].cpu().numpy()
    pub = out["publish"].cpu().numpy().view(np.uint16)
    assert st[abi.STAT_DECISIONS] == G
    assert st[abi.STAT_COMMITTED] == int(n_ent.astype(np.uint64).sum())
    assert st[abi.STAT_ADVANCED] == int((committed == 1).sum())
    assert st[abi.STAT_SLOW] == 0
    wm = (db.download("abs_base") + _u64(out["new_head"])).min()
    assert st[abi.STAT_MIN_WATERMARK] == int(wm)
    assert {abi.FORCE_NONE, abi.FORCE_PRUNE, abi.FORCE_REMOVE} <= set(np.unique(act).tolist()), np.bincount(act)
    ssn = _u64(out["ssn"])
    assert np.array_equal(ssn - np.arange(G, dtype=np.uint64) * 2, (pub != 0).astype(np.uint64))
    S = 2000
    for g0 in (0, G // 3 + 777, G - S):
        hb = orc.host_batch(S, R, L, fields=fields)
        orc.gen(hb, pkg.batch.gen_cfg(gid_base=g0, **kw))
        hb.add("rc_connected")[:] = _conn_of(np.arange(g0, g0 + S, dtype=np.int64)).astype(np.uint16)
        ref = orc.commit(hb, flags & (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN))
        sl = slice(g0, g0 + S)
        assert np.array_equal(_u64(out["new_commit"][sl]), ref["new_commit"]), g0
        assert np.array_equal(committed[sl], ref["committed"]), g0
        assert np.array_equal(n_ent[sl], ref["n_entries"]), g0
        assert np.array_equal(out["digest"][sl].cpu().numpy().view(np.uint32), ref["digest"]), g0
        assert np.array_equal(_u64(out["median"][sl]), ref["median"]), g0
        tf = abi.COMMIT_PUBLISH | abi.COMMIT_FORCE_PRUNE
        rq = np.arange(g0, g0 + S, dtype=np.uint64) + 11
        cl = (np.arange(g0, g0 + S) % 30000 + 1).astype(np.uint16)
        to, _, _ = orc.tail(hb, tf, ref["new_commit"],
                            out=orc.tail_out(S, tf, req_id=rq, clt_id=cl,
                                             ssn=np.arange(g0, g0 + S, dtype=np.uint64) * 2))
        hb.state["commit"] = ref["new_commit"]            # the caller's log->commit update between the calls
        assert np.array_equal(pub[sl], to["publish"]), g0
        assert np.array_equal(ssn[sl], to["ssn"]), g0
        for k in ("new_head", "min_apply"):
            assert np.array_equal(_u64(out[k][sl]), to[k]), (g0, k)
        assert np.array_equal(out["append_head"][sl].cpu().numpy(), to["append_head"]), g0
        for k in ("action", "target"):
            assert np.array_equal(out["force"][k][sl].cpu().numpy(), to["force"][k]), (g0, k)
        assert np.array_equal(_u64(out["force"]["cfg_idx"][sl]), to["force"]["cfg_idx"]), g0
        assert np.array_equal(_u64(out["force"]["req_id"][sl]), to["force"]["req_id"]), g0
        assert np.array_equal(out["force"]["clt_id"][sl].cpu().numpy().view(np.uint16), to["force"]["clt_id"]), g0
        # every byte written in place: the rings (CONFIG entries), the state rows, the columns
        stride = db.stride
        assert np.array_equal(db.ring[g0 * stride:(g0 + S) * stride].cpu().numpy(), hb.ring), g0
        for k, per in (("state", 64), ("apply_offsets", 8 * R), ("remote_commit", 8 * R), ("prev_head", 1)):
            got = db.arrays[k][g0 * per:(g0 + S) * per].cpu().numpy()
            assert got.tobytes() == hb.arrays[k].tobytes(), (g0, k)
    del db, out, conn
    torch.cuda.empty_cache()


def test_c4_one_gpu_64m_groups(pkg, orc, eng):
    """north_star's ">= 64M groups per batch on 1 GPU" (the
    1-GPU point; VERDICT r2 missing #2): 2^26 groups x R=5, 16-entry batches
    of 128-B entries after 2 history entries on 2,448-B rings (165 GB of
    rings), commit walk + Adler-32 on the short-walk kernel, median, pruning.
    Statistics equal the per-group sums / minimum over all 67M groups, no
    group leaves the segment kernel, and three sampled ranges are bit-exact
    against the oracle.  bench.py --workload c4_1gpu measures this batch."""
    import torch
    abi = pkg.abi
    G, R, L = 1 << 26, 5, 2448
    kw = dict(seed=2026, n_entries=16, n_history=2, len_min=64, len_max=64, ring_len=L, p_full_ack=0.9,
              straggler=True)
    fields = ["state", "self_idx", "remote_end", "lr_step", "fail_count", "apply_offsets", "prev_head", "abs_base"]
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L), fields=fields)
    eng.gen(db, pkg.batch.gen_cfg(**kw))
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN
    b = db.struct()
    b.flags = abi.BATCH_SHORT_WALKS
    eng.stats_reset()
    out = eng.update_remote_logs(db, flags, bstruct=b)
    po = eng.log_pruning(db)
    torch.cuda.synchronize()
    st = eng.stats()
    committed = out["committed"]
    assert st[abi.STAT_DECISIONS] == G
    assert st[abi.STAT_COMMITTED] == int(out["n_entries"].to(torch.int64).sum().item())
    assert st[abi.STAT_ADVANCED] == int((committed == 1).sum().item())
    assert st[abi.STAT_CORRUPT] == 0 and st[abi.STAT_SLOW] == 0
    wm = (db.download("abs_base") + _u64(po["new_head"])).min()
    assert st[abi.STAT_MIN_WATERMARK] == int(wm)
    S = 2000
    for g0 in (0, G // 3 + 777, G - S):
        hb = orc.host_batch(S, R, L, fields=fields)
        orc.gen(hb, pkg.batch.gen_cfg(gid_base=g0, **kw))
        ref = orc.commit(hb, flags)
        sl = slice(g0, g0 + S)
        assert np.array_equal(_u64(out["new_commit"][sl]), ref["new_commit"]), g0
        assert np.array_equal(committed[sl].cpu().numpy(), ref["committed"]), g0
        assert np.array_equal(out["n_entries"][sl].cpu().numpy().view(np.uint32), ref["n_entries"]), g0
        assert np.array_equal(out["digest"][sl].cpu().numpy().view(np.uint32), ref["digest"]), g0
        assert np.array_equal(_u64(out["median"][sl]), ref["median"]), g0
        rp, _ = orc.prune(hb)
        assert np.array_equal(_u64(po["new_head"][sl]), rp["new_head"]), g0
        assert np.array_equal(po["append_head"][sl].cpu().numpy(), rp["append_head"]), g0
    del db, out, po, committed
    torch.cuda.empty_cache()


def test_c3_wave_full_size(pkg, orc, eng):
    import torch
    abi = pkg.abi
    # bench.py's C3 wave: 2^19 groups on 272,960-B rings (history commands of
    # at most 64 B, the batch of 64 x 64 B - 4 KB at its worst + a wrap gap)
    G, R, E, L = 1 << 19, 5, 64, 272960
    F = R - 1
    kw = dict(seed=3003, n_entries=E, n_history=16, len_min=64, len_max=4096, ring_len=L, p_full_ack=0.9,
              straggler=True, hist_len_max=64)
    fields = ["state", "self_idx", "remote_end", "remote_commit", "lr_step", "fail_count"]
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L), fields=fields)
    eng.gen(db, pkg.batch.gen_cfg(**kw))
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN
    eng.stats_reset()
    out = eng.update_remote_logs(db, flags)
    dets, ln = eng.log_entries_to_nc_buf(db, E)
    torch.cuda.synchronize()
    st = eng.stats()
    n_ent = out["n_entries"].cpu().numpy().view(np.uint32)
    assert st[abi.STAT_DECISIONS] == G
    assert st[abi.STAT_COMMITTED] == int(n_ent.astype(np.uint64).sum())
    assert st[abi.STAT_ADVANCED] == int((out["committed"].cpu().numpy() == 1).sum())
    assert st[abi.STAT_CORRUPT] == 0
    # the hop walk (APUS_BATCH_VAR_LEN, the hint this config's variable entries
    # call for) equals the speculative walk on every group, with no deferral
    bv = db.struct()
    bv.flags = abi.BATCH_VAR_LEN
    eng.stats_reset()
    out_v = eng.update_remote_logs(db, abi.COMMIT_WALK | abi.COMMIT_CHECKSUM, bstruct=bv)
    torch.cuda.synchronize()
    for k in ("new_commit", "committed", "n_entries", "digest"):
        assert torch.equal(out_v[k], out[k]), k
    sv = eng.stats()
    assert sv[abi.STAT_SLOW] == 0 and sv[abi.STAT_COMMITTED] == st[abi.STAT_COMMITTED]
    del out_v
    # followers: the leader's determinants with the term changed from a
    # random position m on (m = n: an exact copy), some truncated, some empty
    gq = torch.Generator(device="cuda").manual_seed(33)
    dv = dets.view(torch.int64).view(G, 1, E, 3).repeat(1, F, 1, 1).contiguous()
    m_r = torch.randint(0, E + 1, (G, F, 1), device="cuda", generator=gq)
    dv[..., 1] += (torch.arange(E, device="cuda").view(1, 1, E) >= m_r).to(torch.int64)
    lens = ln.view(G, 1).repeat(1, F).contiguous()
    cut = torch.randint(0, 8, (G, F), device="cuda", generator=gq)
    lens = torch.where(cut == 0, torch.zeros_like(lens), torch.where(cut == 1, lens // 2, lens)).contiguous()
    fol = ((db.arrays["self_idx"].view(G, 1).to(torch.int64) + 1 + torch.arange(F, device="cuda").view(1, F)) % R)
    fol = fol.to(torch.uint8).contiguous()
    eng.stats_reset()
    rend = eng.log_find_remote_end_offset(db, dv.view(torch.uint8).view(-1), lens.view(-1), fol.view(-1), E)
    torch.cuda.synchronize()
    assert eng.stats()[abi.STAT_MISMATCHES] > 0
    S = 300
    for g0 in (0, G // 2 + 4321, G - S):
        hb = orc.host_batch(S, R, L, fields=fields)
        orc.gen(hb, pkg.batch.gen_cfg(gid_base=g0, **kw))
        ref = orc.commit(hb, flags)
        sl = slice(g0, g0 + S)
        assert np.array_equal(_u64(out["new_commit"][sl]), ref["new_commit"]), g0
        assert np.array_equal(out["digest"][sl].cpu().numpy().view(np.uint32), ref["digest"]), g0
        assert np.array_equal(_u64(out["median"][sl]), ref["median"]), g0
        rd, rl = orc.nc_build(hb, E)
        gl = ln[sl].cpu().numpy().view(np.uint32)
        assert np.array_equal(gl, rl), g0
        gd = dets.view(torch.int64).view(G, E * 3)[sl].cpu().numpy().view(np.uint64)
        for g in range(S):
            n = int(rl[g])
            assert np.array_equal(gd[g, :3 * n], rd[g * E * 3:g * E * 3 + 3 * n]), (g0, g)
        fd = dv[sl].cpu().numpy().reshape(-1).view(np.uint64)
        fl = lens[sl].cpu().numpy().reshape(-1).astype(np.int32)
        ff = fol[sl].cpu().numpy().reshape(-1)
        rv = orc.validate(hb, fd, fl, ff, F, E)
        assert np.array_equal(_u64(rend.view(G, F)[sl].reshape(-1)), rv), g0
    del db, out, dets, dv, rend
    torch.cuda.empty_cache()

_REF_SO = os.path.exists(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                                      "libapusref.so"))


def _ref_groups(orc, hb, g0, n, out, vo, ro, po):
    """the first n groups of a sampled range against the reference's own code
    (oracle/_ref: its compiled dare_log.h with the transcribed loop bodies,
    per group on the group's ring, state and columns -- the .so travels with
    the tree, so this runs on the GPU box too); returns False without _ref"""
    import ctypes as C
    ref = orc.ref()
    if ref is None:
        return False
    R = hb.R
    P = lambda a: C.c_void_p(a.ctypes.data)   # noqa: E731
    nc_o, cm_o = _u64(out["new_commit"]), out["committed"].cpu().numpy()
    med_o = _u64(out["median"])
    if vo is not None:
        won_o, vc_o, vn_o = vo["won"].cpu().numpy(), vo["vote_count"].cpu().numpy(), _u64(vo["new_commit"])
    if ro is not None:
        lit_o, oc_o, ns_o = _u64(ro["last_idx_term"]), ro["outcome"].cpu().numpy(), _u64(ro["new_sid"])
        cid_o, clr_o = ro["new_cid"].cpu().numpy(), ro["cleared"].cpu().numpy().view(np.uint16)
    nh_o, ah_o, mn_o = _u64(po["new_head"]), po["append_head"].cpu().numpy(), _u64(po["min_apply"])
    for g in range(n):
        G_ = g0 + g
        s_ = hb.state[g]
        st = np.array([s_["head"], s_["apply"], s_["commit"], s_["end"], s_["tail"], s_["len"]], np.uint64)
        cid = np.frombuffer(hb.state[g:g + 1].tobytes()[48:64], np.uint8).copy()
        self_ = int(hb.self_idx[g])
        ring = hb.group_ring(g)
        committed = C.c_int(0)
        assert ref.ref_commit_walk(P(ring), P(st), P(cid), self_, C.byref(committed)) == nc_o[G_], G_
        assert committed.value == cm_o[G_], G_
        cols = {k: getattr(hb, k)[g * R:(g + 1) * R].copy() for k in ("remote_end", "lr_step", "fail_count",
                                                                        "vote_ack", "hb", "apply_offsets")
                if k in hb.arrays}
        assert ref.ref_median(P(st), P(cid), self_, P(cols["remote_end"]), P(cols["lr_step"]),
                              P(cols["fail_count"])) == med_o[G_], G_
        if vo is not None:
            vc, vn = np.zeros(2, np.uint8), C.c_uint64(0)
            won = ref.ref_vote_tally(P(st), P(cid), self_, P(cols["vote_ack"]), P(vc), C.byref(vn))
            assert won == won_o[G_] and list(vc) == list(vc_o[2 * G_:2 * G_ + 2]) and vn.value == vn_o[G_], G_
        if ro is not None:
            lit = np.zeros(2, np.uint64)
            ref.ref_last_idx_term(P(ring), P(st), P(lit))
            assert list(lit) == list(lit_o[2 * G_:2 * G_ + 2]), G_
            req = np.frombuffer(hb.vote_req[g * R:(g + 1) * R].tobytes(), np.uint64).copy()
            ns, ncid, clr = C.c_uint64(0), np.zeros(16, np.uint8), C.c_uint16(0)
            oc = ref.ref_vote_rank(P(st), P(cid), self_, int(hb.sid[g]), P(cols["hb"]), R, P(req), int(lit[0]),
                                   int(lit[1]), C.byref(ns), P(ncid), C.byref(clr))
            assert oc == oc_o[G_] and ns.value == ns_o[G_] and clr.value == clr_o[G_], G_
            assert bytes(ncid) == bytes(cid_o[16 * G_:16 * G_ + 16]), G_
        nh, app = C.c_uint64(0), C.c_int(0)
        mn = ref.ref_min_apply(P(ring), P(st), P(cid), P(cols["apply_offsets"]), int(hb.prev_head[g]),
                               C.byref(nh), C.byref(app))
        assert mn == mn_o[G_] and nh.value == nh_o[G_] and app.value == ah_o[G_], G_
    return True


def test_c5_shard_full_size(pkg, orc, eng):
    """C5 (BASELINE.json configs[4]): the per-GPU shard of 64M 7-replica groups
    over 8 GPUs, 2^23 groups x R=7, 16-entry batches, STABLE / EXTENDED /
    TRANSIT configurations, vote acks with p=0.6 (76 GB resident): the commit
    walk + Adler-32 on the short-walk kernel (four groups per wave), the median
    quorum, the vote tally, the vote-request ranking with the local (idx, term)
    derived from each log, and the pruning minimum."""
    import torch
    abi = pkg.abi
    G, R, L = 1 << 23, 7, 8192
    kw = dict(seed=5005, n_entries=16, n_history=16, len_min=64, len_max=64, ring_len=L, p_full_ack=0.9,
              straggler=True, cid_mix=True, p_vote_ack=0.6)
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, pkg.batch.gen_cfg(**kw))
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN
    b = db.struct()
    b.flags = abi.BATCH_SHORT_WALKS
    eng.stats_reset()
    out = eng.update_remote_logs(db, flags, bstruct=b)
    vo = eng.poll_vote_count(db)
    ro = eng.poll_vote_requests(db, derive_local=True)
    po = eng.log_pruning(db)
    torch.cuda.synchronize()
    st = eng.stats()
    n_ent = out["n_entries"].cpu().numpy().view(np.uint32)
    committed = out["committed"].cpu().numpy()
    won = vo["won"].cpu().numpy()
    assert st[abi.STAT_DECISIONS] == G
    assert st[abi.STAT_COMMITTED] == int(n_ent.astype(np.uint64).sum())
    assert st[abi.STAT_ADVANCED] == int((committed == 1).sum())
    assert st[abi.STAT_VOTES_WON] == int(won.astype(np.uint64).sum())
    # every 16-entry walk fits the segment window: no group left the fast path
    assert st[abi.STAT_CORRUPT] == 0 and st[abi.STAT_SLOW] == 0
    wm = (db.download("abs_base") + _u64(po["new_head"])).min()
    assert st[abi.STAT_MIN_WATERMARK] == int(wm)
    S = 1500
    for g0 in (0, G // 2 + 4321, G - S):
        hb = orc.host_batch(S, R, L)
        orc.gen(hb, pkg.batch.gen_cfg(gid_base=g0, **kw))
        sl = slice(g0, g0 + S)
        # (the full-size shard against the reference's own code too)
        assert _ref_groups(orc, hb, g0, 256, out, vo, ro, po) or not _REF_SO, "oracle/_ref built but not loaded"
        ref = orc.commit(hb, flags)
        assert np.array_equal(_u64(out["new_commit"][sl]), ref["new_commit"]), g0
        assert np.array_equal(committed[sl], ref["committed"]), g0
        assert np.array_equal(n_ent[sl], ref["n_entries"]), g0
        assert np.array_equal(out["digest"][sl].cpu().numpy().view(np.uint32), ref["digest"]), g0
        assert np.array_equal(_u64(out["median"][sl]), ref["median"]), g0
        rv = orc.vote(hb)
        assert np.array_equal(won[sl], rv["won"]), g0
        assert np.array_equal(vo["vote_count"].view(G, 2)[sl].cpu().numpy().reshape(-1), rv["vote_count"]), g0
        assert np.array_equal(_u64(vo["new_commit"][sl]), rv["new_commit"]), g0
        assert np.array_equal(_u64(ro["last_idx_term"].view(G, 2)[sl]).reshape(-1), orc.last_idx_term(hb)), g0
        rr = orc.rank(hb)
        assert np.array_equal(ro["outcome"][sl].cpu().numpy(), rr["outcome"]), g0
        assert np.array_equal(_u64(ro["new_sid"][sl]), rr["new_sid"]), g0
        assert np.array_equal(ro["new_cid"].view(G, 16)[sl].cpu().numpy().reshape(-1), rr["new_cid"].reshape(-1)), g0
        rp, _ = orc.prune(hb)
        assert np.array_equal(_u64(po["new_head"][sl]), rp["new_head"]), g0
        assert np.array_equal(po["append_head"][sl].cpu().numpy(), rp["append_head"]), g0
    # bench.py's C5 step: ONE call -- walk + checksum, then one tail launch for
    # the median, pruning, local (idx, term), vote tally and vote-request
    # ranking -- equals the separate calls above on every group
    # (round 5: with update_remote_logs' lazy remote-commit publish, the bench's C5 set)
    fused = (flags | abi.COMMIT_PRUNE | abi.COMMIT_LAST_IT | abi.COMMIT_VOTE | abi.COMMIT_RANK |
             abi.COMMIT_PUBLISH | abi.COMMIT_STATS_FRESH)
    del committed, n_ent
    fo = eng.update_remote_logs(db, fused, bstruct=b)
    torch.cuda.synchronize()
    sf = eng.stats()
    pub = fo["publish"].cpu().numpy().view(np.uint16)
    assert (pub != 0).any() and np.array_equal(_u64(fo["ssn"]), (pub != 0).astype(np.uint64))
    for g0 in (0, G // 2 + 4321, G - S):
        hb = orc.host_batch(S, R, L)
        orc.gen(hb, pkg.batch.gen_cfg(gid_base=g0, **kw))
        sl = slice(g0, g0 + S)
        ref = orc.commit(hb, flags)
        to, _, _ = orc.tail(hb, abi.COMMIT_PUBLISH, ref["new_commit"])
        assert np.array_equal(pub[sl], to["publish"]), g0
        rc = db.arrays["remote_commit"][g0 * R * 8:(g0 + S) * R * 8].cpu().numpy().view(np.uint64)
        assert np.array_equal(rc, hb.remote_commit), g0
    for k in ("new_commit", "committed", "n_entries", "digest", "median"):
        assert torch.equal(fo[k], out[k]), k
    for k in ("new_head", "append_head", "min_apply"):
        assert torch.equal(fo[k], po[k]), k
    assert torch.equal(fo["last_idx_term"], ro["last_idx_term"])
    for k in ("won", "vote_count", "new_commit", "voters"):
        assert torch.equal(fo["vote"][k], vo[k]), k
    for k in ("outcome", "new_sid", "new_cid", "cleared"):
        assert torch.equal(fo["rank"][k], ro[k]), k
    for k in (abi.STAT_DECISIONS, abi.STAT_COMMITTED, abi.STAT_ADVANCED, abi.STAT_VOTES_WON, abi.STAT_MIN_WATERMARK,
              abi.STAT_SLOW, abi.STAT_CORRUPT):
        assert sf[k] == st[k], k
    del db, out, vo, ro, po, fo
    torch.cuda.empty_cache()


@pytest.mark.parametrize("short", [False, True])
def test_block_counter_partial_last_block(pkg, orc, eng, short):
    """Batches large enough for the walks' block counter (>= 8 blocks of 64
    groups per wave: commit_wave_kernel / commit_seg_kernel with DYN), with a
    partial last block (G = 2^22 + 37): every group walked once (statistics =
    per-group sums), sampled ranges -- the first, a middle one and the partial
    last block -- bit-exact against the oracle, and on the segment kernel the
    local (idx, term) of APUS_COMMIT_LAST_IT against apus_last_idx_term_batch."""
    import torch
    abi = pkg.abi
    G, R, L = (1 << 22) + 37, 5, 2048
    kw = dict(seed=4242, n_entries=8 if not short else 12, n_history=2, len_min=64, len_max=64, ring_len=L,
              p_full_ack=0.8, straggler=True, cid_mix=short)
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, pkg.batch.gen_cfg(**kw))
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | (abi.COMMIT_LAST_IT if short else 0)
    b = db.struct()
    b.flags = abi.BATCH_SHORT_WALKS if short else 0
    eng.stats_reset()
    out = eng.update_remote_logs(db, flags, bstruct=b)
    lit = eng.last_idx_term(db) if short else None
    torch.cuda.synchronize()
    st = eng.stats()
    n_ent = out["n_entries"].cpu().numpy().view(np.uint32)
    committed = out["committed"].cpu().numpy()
    assert st[abi.STAT_DECISIONS] == G
    assert st[abi.STAT_COMMITTED] == int(n_ent.astype(np.uint64).sum())
    assert st[abi.STAT_ADVANCED] == int((committed == 1).sum())
    assert st[abi.STAT_CORRUPT] == 0
    if short:
        assert torch.equal(out["last_idx_term"], lit)
    S = 700
    for g0 in (0, G // 2 + 1234, G - S):
        hb = orc.host_batch(S, R, L)
        orc.gen(hb, pkg.batch.gen_cfg(gid_base=g0, **kw))
        ref = orc.commit(hb, flags & ~abi.COMMIT_LAST_IT)
        sl = slice(g0, g0 + S)
        assert np.array_equal(_u64(out["new_commit"][sl]), ref["new_commit"]), g0
        assert np.array_equal(committed[sl], ref["committed"]), g0
        assert np.array_equal(n_ent[sl], ref["n_entries"]), g0
        assert np.array_equal(out["digest"][sl].cpu().numpy().view(np.uint32), ref["digest"]), g0
        assert np.array_equal(_u64(out["median"][sl]), ref["median"]), g0
        if short:
            assert np.array_equal(_u64(out["last_idx_term"].view(G, 2)[sl]).reshape(-1), orc.last_idx_term(hb)), g0
    del db, out
    torch.cuda.empty_cache()
