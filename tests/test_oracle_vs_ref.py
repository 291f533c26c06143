"""Pin the clean-room oracle against the reference's own code (CPU only).

oracle/_ref/libapusref.so is the reference's src/include/dare/dare_log.h
compiled from /root/reference with the hot-path loops of dare_ibv_rc.c /
dare_server.c restated on its real primitives (oracle/ref_compose.c).  Every
test here drives both on identical synthetic logs -- small rings so that the
header-wrap and ghost-header paths (dare_log.h:316-332, 502-538) are hit
constantly -- and requires identical results.
"""
import ctypes as C

import numpy as np
import pytest

CONFIGS = [
    dict(seed=11, ring_len=16384, n_entries=64, n_history=16),                     # C2 shape
    dict(seed=12, ring_len=6000, n_entries=24, n_history=8, len_min=0, len_max=90,
         type_mix=True, self_random=True, garbage_reply=0.05, p_full_ack=0.5),
    dict(seed=13, ring_len=2600, n_entries=12, n_history=4, len_min=1, len_max=60,
         type_mix=True, cid_mix=True, self_random=True, straggler=True, p_full_ack=0.3),
    dict(seed=14, ring_len=1500, n_entries=6, n_history=2, len_min=0, len_max=64,
         type_mix=True, cid_mix=True, self_random=True, garbage_reply=0.2),
    dict(seed=15, ring_len=777, n_entries=5, n_history=1, len_min=3, len_max=45,
         cid_mix=True, self_random=True, p_full_ack=0.0, straggler=True),
]


def _batch(orc, pkg, R, **kw):
    cfg = pkg.batch.gen_cfg(**kw)
    hb = orc.host_batch(256, R, kw["ring_len"])
    orc.gen(hb, cfg)
    return hb, cfg


def _st6(hb, g):
    s = hb.state[g]
    return np.array([s["head"], s["apply"], s["commit"], s["end"], s["tail"], s["len"]], np.uint64)


def _cid(hb, g):
    return np.frombuffer(hb.state[g:g + 1].tobytes()[48:64], np.uint8).copy()


def P(a):
    return C.c_void_p(a.ctypes.data)


@pytest.mark.parametrize("R", [3, 5, 7])
@pytest.mark.parametrize("ci", range(len(CONFIGS)))
def test_commit_walk_median_vote(orc, ref, pkg, R, ci):
    kw = dict(CONFIGS[ci])
    if R < 5 and kw.get("cid_mix"):
        kw["cid_mix"] = True
    hb, _ = _batch(orc, pkg, R, **kw)
    out = orc.commit(hb, 1 | 4)
    vo = orc.vote(hb)
    hits = {"adv": 0, "wrap": 0}
    for g in range(hb.G):
        st, cid, self_ = _st6(hb, g), _cid(hb, g), int(hb.self_idx[g])
        ring = hb.group_ring(g)
        committed = C.c_int(0)
        rc = ref.ref_commit_walk(P(ring), P(st), P(cid), self_, C.byref(committed))
        assert rc == out["new_commit"][g], (g, rc, out["new_commit"][g])
        assert committed.value == out["committed"][g]
        hits["adv"] += committed.value
        hits["wrap"] += int(st[3] < st[2])
        rend = hb.remote_end[g * R:(g + 1) * R].copy()
        step = hb.lr_step[g * R:(g + 1) * R].copy()
        fail = hb.fail_count[g * R:(g + 1) * R].copy()
        med = ref.ref_median(P(st), P(cid), self_, P(rend), P(step), P(fail))
        assert med == out["median"][g]
        ack = hb.vote_ack[g * R:(g + 1) * R].copy()
        vc = np.zeros(2, np.uint8)
        nc = C.c_uint64(0)
        won = ref.ref_vote_tally(P(st), P(cid), self_, P(ack), P(vc), C.byref(nc))
        assert won == vo["won"][g]
        assert list(vc) == list(vo["vote_count"][2 * g:2 * g + 2])
        assert nc.value == vo["new_commit"][g]
    assert hits["adv"] > 0 and hits["wrap"] > 0


@pytest.mark.parametrize("ci", range(len(CONFIGS)))
def test_rank_prune_tail(orc, ref, pkg, ci):
    R = 5
    hb, _ = _batch(orc, pkg, R, **CONFIGS[ci])
    lit = orc.last_idx_term(hb)
    # the generator's last_idx_term must equal the reference's derivation
    for g in range(hb.G):
        o = np.zeros(2, np.uint64)
        ref.ref_last_idx_term(P(hb.group_ring(g)), P(_st6(hb, g)), P(o))
        assert list(o) == list(lit[2 * g:2 * g + 2])
    assert np.array_equal(lit, hb.last_idx_term)
    ro = orc.rank(hb)
    ap_before = hb.apply_offsets.copy()
    po, wm = orc.prune(hb)
    outcomes = set()
    for g in range(hb.G):
        st, cid, self_ = _st6(hb, g), _cid(hb, g), int(hb.self_idx[g])
        hbv = hb.hb[g * R:(g + 1) * R].copy()
        req = np.frombuffer(hb.vote_req[g * R:(g + 1) * R].tobytes(), np.uint64).copy()
        ns = C.c_uint64(0)
        ncid = np.zeros(16, np.uint8)
        clr = C.c_uint16(0)
        oc = ref.ref_vote_rank(P(st), P(cid), self_, int(hb.sid[g]), P(hbv), R, P(req),
                               int(lit[2 * g]), int(lit[2 * g + 1]), C.byref(ns), P(ncid), C.byref(clr))
        assert oc == ro["outcome"][g]
        assert ns.value == ro["new_sid"][g]
        assert clr.value == ro["cleared"][g]
        assert bytes(ncid) == bytes(ro["new_cid"][16 * g:16 * g + 16])
        outcomes.add(oc)
        ap = ap_before[g * R:(g + 1) * R].copy()
        nh = C.c_uint64(0)
        app = C.c_int(0)
        mn = ref.ref_min_apply(P(hb.group_ring(g)), P(st), P(cid), P(ap), int(hb.prev_head[g]),
                               C.byref(nh), C.byref(app))
        assert mn == po["min_apply"][g]
        assert nh.value == po["new_head"][g] and app.value == po["append_head"][g]
        assert np.array_equal(ap, hb.apply_offsets[g * R:(g + 1) * R])     # OFF-server side effect
        assert ref.ref_get_tail(P(hb.group_ring(g)), P(st)) == orc.lib().apus_oracle_log_get_tail(
            P(hb.group_ring(g)), C.c_void_p(hb.state.ctypes.data + 64 * g))
    assert wm == min(int(hb.abs_base[g]) + int(po["new_head"][g]) for g in range(hb.G))
    assert len(outcomes) >= 3


@pytest.mark.parametrize("ci", range(len(CONFIGS)))
def test_nc_and_find_remote_end(orc, ref, pkg, ci):
    R, F, M = 5, 4, 256
    hb, cfg = _batch(orc, pkg, R, **CONFIGS[ci])
    dets, ln = orc.nc_build(hb, M)
    for g in range(hb.G):
        rd = np.zeros(M * 3, np.uint64)
        n = ref.ref_nc_build(P(hb.group_ring(g)), P(_st6(hb, g)), P(rd), M)
        assert n == ln[g]
        assert np.array_equal(rd[:3 * n], dets[g * M * 3:g * M * 3 + 3 * n])
    fd, fl, ff = orc.gen_nc(hb, cfg, F, M)
    out = orc.validate(hb, fd, fl, ff, F, M)
    seen_mismatch = 0
    for g in range(hb.G):
        for f in range(F):
            gf = g * F + f
            n = int(fl[gf])
            if n == 0:
                assert out[gf] == hb.remote_commit[g * R + int(ff[gf])]
                continue
            d = fd[gf * M * 3:gf * M * 3 + 3 * n].copy()
            r = ref.ref_find_remote_end(P(hb.group_ring(g)), P(_st6(hb, g)), P(d), n)
            assert r == out[gf]
            seen_mismatch += int(r != (d[3 * (n - 1) + 2]))
    assert seen_mismatch > 0


def test_placement_matches_log_append_entry(orc, ref, pkg):
    """the generator's placement rule == the reference's log_append_entry"""
    rng = np.random.default_rng(5)
    for trial in range(300):
        ln = int(rng.integers(300, 5000))
        n = int(rng.integers(1, 24))
        types = rng.choice([0, 2, 3, 4, 5, 6], size=n).astype(np.uint8)
        clens = rng.integers(0, 200, size=n).astype(np.uint16)
        clens[np.isin(types, [0, 2, 3])] = 0
        elen = (64 + clens.astype(np.uint32)).astype(np.uint32)
        if int(elen.sum()) + 300 >= ln:
            continue
        start = int(rng.integers(0, ln)) if trial % 5 else ln        # ln = empty log
        off = np.zeros(n, np.uint64)
        gh = np.zeros(n, np.uint64)
        end = C.c_uint64(0)
        orc.lib().apus_oracle_place_seq(ln, start, n, P(elen), P(off), P(gh), C.byref(end))
        rring = np.zeros(ln + 64, np.uint8)
        rst = np.zeros(6, np.uint64)
        roff = np.zeros(n, np.uint64)
        cid = np.zeros(16, np.uint8)
        terms = np.ones(n, np.uint64)
        assert ref.ref_append_seq(ln, start, n, P(types), P(clens), P(terms), P(cid), P(rring), P(rst),
                                  P(roff)) == 0
        assert np.array_equal(off, roff), (trial, off, roff)
        assert int(rst[3]) == end.value
        for k in range(n):       # ghost headers exist exactly where the oracle puts them
            if gh[k] != np.uint64(2 ** 64 - 1):
                g0 = int(gh[k])
                assert rring[g0 + 26] == types[k]
                assert int.from_bytes(bytes(rring[g0 + 48:g0 + 50]), "little") == clens[k]


def test_primitives(orc, ref):
    rng = np.random.default_rng(9)
    L = orc.lib()
    for _ in range(2000):
        ln = int(rng.integers(64, 1 << 20))
        end = int(rng.integers(0, ln + 1))
        a, b = (int(x) for x in rng.integers(0, ln + 1, size=2))
        st = np.array([0, 0, 0, end, ln, ln], np.uint64)
        assert ref.ref_dist(P(st), a) == L.apus_oracle_dist(end, ln, a)
        assert ref.ref_larger(P(st), a, b) == L.apus_oracle_larger(end, ln, a, b)
