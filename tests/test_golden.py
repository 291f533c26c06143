"""Golden fixtures (tests/golden/*.json, written by tests/golden/make_golden.py
from the reference's own dare_log.h compiled in oracle/_ref) checked against

  * the CPU oracle            (not gpu: pins the restatement), and
  * the HIP path via the ABI  (gpu:     parity of the product).

scenarios.json holds the reference results SURVEY.md §8c records (commit 640,
wrap commit 128, 7-replica and TRANSIT 5->7 vote tallies, find_remote_end 192,
pruning to head 128 + HEAD entry); vectors.json holds 160 groups of nine seeded
configurations with the SHA-256 of their generated inputs.  Nothing here
reads /root/reference at run time.
"""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SCEN = json.load(open(os.path.join(HERE, "scenarios.json")))
VECS = json.load(open(os.path.join(HERE, "vectors.json")))
BY_NAME = {s["name"]: s for s in SCEN}

E_IDX, E_TERM, E_TYPE, E_REPLY, E_DATA = 0, 8, 26, 28, 48
BARE = (0, 2, 3)                                     # NOOP, CONFIG, HEAD


def P(a):
    return C.c_void_p(a.ctypes.data)


def _elen(t, c):
    return 64 if t in BARE else 64 + c


def build_ring(orc, ln, start, types, clens, terms=None):
    """log_append_entry placement (oracle place_seq) + header bytes, ghost
    headers included; returns (ring, end, offsets)"""
    n = len(types)
    el = np.array([_elen(t, c) for t, c in zip(types, clens)], np.uint32)
    off = np.zeros(n, np.uint64)
    gh = np.zeros(n, np.uint64)
    end = C.c_uint64(0)
    orc.lib().apus_oracle_place_seq(ln, start, n, P(el), P(off), P(gh), C.byref(end))
    ring = np.zeros(ln + 64, np.uint8)
    terms = terms or [1] * n
    for k in range(n):
        hdr = np.zeros(64, np.uint8)
        hdr[E_IDX:E_IDX + 8] = np.frombuffer(np.uint64(k + 1).tobytes(), np.uint8)
        hdr[E_TERM:E_TERM + 8] = np.frombuffer(np.uint64(terms[k]).tobytes(), np.uint8)
        hdr[E_TYPE] = types[k]
        hdr[E_DATA:E_DATA + 2] = np.frombuffer(np.uint16(clens[k]).tobytes(), np.uint8)
        if gh[k] != np.uint64(2 ** 64 - 1):
            ring[int(gh[k]):int(gh[k]) + 64] = hdr
        ring[int(off[k]):int(off[k]) + 64] = hdr
    return ring, int(end.value), [int(o) for o in off]


def state_of(pkg, st6, cid):
    s = np.zeros(1, pkg.batch.STATE_DT)
    for k, v in zip(("head", "apply", "commit", "end", "tail", "len"), st6):
        s[k] = v
    s["cid"]["epoch"], s["cid"]["size0"], s["cid"]["size1"], s["cid"]["state"], s["cid"]["bitmask"] = cid
    return s


def scenario_ring(orc, sc):
    ring, end, off = build_ring(orc, sc["ring_len"], sc["start"], sc["types"], sc["clens"], sc.get("terms"))
    for r, ks in sc.get("acks", {}).items():
        for k in ks:
            ring[off[k] + E_REPLY + int(r)] = 1
    return ring, end


# ------------------------------------------------------------------ CPU side
def test_scenarios_cover_survey_results():
    assert BY_NAME["commit_640"]["expect_commit"] == 640
    assert BY_NAME["wrap_commit_128"]["expect_commit"] == 128
    assert [BY_NAME[n]["expect_won"] for n in ("vote7_3acks", "vote7_2acks", "transit_5_7_acks12",
                                               "transit_5_7_acks125")] == [1, 0, 0, 1]
    assert BY_NAME["find_remote_end_192"]["expect_end"] == 192
    p = BY_NAME["prune_head_128"]
    assert (p["expect_head"], p["expect_append"], p["expect_end_after_head_entry"]) == (128, 1, 448)


@pytest.mark.parametrize("name", ["commit_640", "wrap_commit_128"])
def test_oracle_commit_scenarios(orc, pkg, name):
    sc = BY_NAME[name]
    ring, end = scenario_ring(orc, sc)
    assert end == sc["state"][3]                       # same placement as log_append_entry
    st = state_of(pkg, sc["state"], sc["cid"])
    adv, n, bad = C.c_int(0), C.c_uint32(0), C.c_int(0)
    got = orc.lib().apus_oracle_commit_walk(P(ring), P(st), sc["self"], C.byref(adv), C.byref(n), C.byref(bad))
    assert got == sc["expect_commit"] and adv.value == sc["expect_committed"] and bad.value == 0


@pytest.mark.parametrize("name", ["vote7_3acks", "vote7_2acks", "transit_5_7_acks12", "transit_5_7_acks125"])
def test_oracle_vote_scenarios(orc, pkg, name):
    sc = BY_NAME[name]
    st = state_of(pkg, sc["state"], sc["cid"])
    va = np.array(sc["vote_ack"], np.uint64)
    vc = np.zeros(2, np.uint8)
    nc, voters = C.c_uint64(0), C.c_uint16(0)
    won = orc.lib().apus_oracle_vote_tally(P(st), sc["self"], P(va), P(vc), C.byref(nc), C.byref(voters))
    assert won == sc["expect_won"] and list(vc) == sc["expect_vc"] and nc.value == sc["expect_commit"]


def test_oracle_find_remote_end_scenario(orc, pkg):
    sc = BY_NAME["find_remote_end_192"]
    ring, end = scenario_ring(orc, sc)
    st = state_of(pkg, sc["state"], [0, 3, 0, 0, 0x1FFF])
    d = np.array(sc["dets"], np.uint64)
    out = C.c_uint64(0)
    orc.lib().apus_oracle_find_remote_end(P(ring), P(st), P(d), len(d) // 3, C.byref(out))
    assert out.value == sc["expect_end"]


def test_oracle_prune_scenario(orc, pkg):
    sc = BY_NAME["prune_head_128"]
    ring, end = scenario_ring(orc, sc)
    st = state_of(pkg, sc["state"], sc["cid"])
    ap = np.zeros(13, np.uint64)
    ap[:3] = sc["apply_offsets"]
    nh, app = C.c_uint64(0), C.c_int(0)
    mn = orc.lib().apus_oracle_min_apply(P(ring), P(st), P(ap), 0, C.byref(nh), C.byref(app))
    assert (mn, nh.value, app.value) == (sc["expect_min"], sc["expect_head"], sc["expect_append"])
    _, end2, _ = build_ring(orc, 4096, 4096, [5, 5, 5, 3], [64, 64, 64, 0])
    assert end2 == sc["expect_end_after_head_entry"]


def input_digest(hb):
    h = hashlib.sha256(hb.ring.tobytes())
    for k in sorted(hb.arrays):
        h.update(hb.arrays[k].tobytes())
    return h.hexdigest()


def _host(orc, pkg, ent):
    hb = orc.host_batch(ent["groups"], ent["replicas"], ent["cfg"]["ring_len"])
    orc.gen(hb, pkg.batch.gen_cfg(**ent["cfg"]))
    return hb


def _col(ent, k):
    return np.array([g[k] for g in ent["groups_out"]], np.uint64)


@pytest.mark.parametrize("name", sorted(VECS))
def test_oracle_matches_vectors(orc, pkg, name):
    ent = VECS[name]
    hb = _host(orc, pkg, ent)
    assert input_digest(hb) == ent["input_sha256"]       # generator is stable
    G = hb.G
    c = orc.commit(hb, pkg.abi.COMMIT_WALK | pkg.abi.COMMIT_CHECKSUM | pkg.abi.COMMIT_MEDIAN)
    assert np.array_equal(c["new_commit"], _col(ent, "commit"))
    # Adler-32 of the entries the reference lists from commit to end (zlib, in make_golden.py)
    assert np.array_equal(c["digest"].astype(np.uint64), _col(ent, "digest"))
    assert np.array_equal(c["committed"], _col(ent, "committed"))
    assert np.array_equal(c["median"], _col(ent, "median"))
    v = orc.vote(hb)
    assert np.array_equal(v["won"], _col(ent, "won"))
    assert np.array_equal(v["vote_count"].reshape(G, 2), np.array([g["vc"] for g in ent["groups_out"]]))
    assert np.array_equal(v["new_commit"], _col(ent, "vote_commit"))
    assert np.array_equal(orc.last_idx_term(hb).reshape(G, 2),
                          np.array([g["lit"] for g in ent["groups_out"]], np.uint64))
    dets, ln = orc.nc_build(hb, 256)
    assert np.array_equal(ln, _col(ent, "nc_len"))
    for g in range(G):
        n = int(ln[g])
        if n:
            out = C.c_uint64(0)
            st = C.c_void_p(hb.state.ctypes.data + 64 * g)
            dg = dets[g * 256 * 3:(g + 1) * 256 * 3].copy()
            orc.lib().apus_oracle_find_remote_end(P(hb.group_ring(g)), st, P(dg), n, C.byref(out))
            assert out.value == ent["groups_out"][g]["find_end"]
    r = orc.rank(hb)
    assert np.array_equal(r["outcome"], _col(ent, "rank"))
    assert np.array_equal(r["new_sid"], _col(ent, "new_sid"))
    assert np.array_equal(r["cleared"], _col(ent, "cleared"))
    p, _ = orc.prune(_host(orc, pkg, ent))
    assert np.array_equal(p["min_apply"], _col(ent, "min_apply"))
    assert np.array_equal(p["new_head"], _col(ent, "new_head"))
    assert np.array_equal(p["append_head"], _col(ent, "append"))


# ------------------------------------------------------------------ GPU side
@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(VECS))
def test_gpu_matches_vectors(pkg, eng, name):
    import torch
    ent = VECS[name]
    G, R, L = ent["groups"], ent["replicas"], ent["cfg"]["ring_len"]
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, pkg.batch.gen_cfg(**ent["cfg"]))
    torch.cuda.synchronize()
    h = hashlib.sha256(db.download("ring").tobytes())
    for k in sorted(db.arrays):
        h.update(db.download(k).tobytes())
    assert h.hexdigest() == ent["input_sha256"]           # device generator == fixture inputs
    W, MD, CK = pkg.abi.COMMIT_WALK, pkg.abi.COMMIT_MEDIAN, pkg.abi.COMMIT_CHECKSUM
    c = eng.update_remote_logs(db, W | CK | MD)
    b_sh = db.struct()
    b_sh.flags = pkg.abi.BATCH_SHORT_WALKS
    c_sh = eng.update_remote_logs(db, W | CK, bstruct=b_sh)
    b_hp = db.struct()
    b_hp.flags = pkg.abi.BATCH_VAR_LEN
    c_hp = eng.update_remote_logs(db, W | CK, bstruct=b_hp)
    v = eng.poll_vote_count(db)
    dets, ln = eng.log_entries_to_nc_buf(db, 256)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(c["new_commit"]), _col(ent, "commit"))
    assert np.array_equal(c["committed"].cpu().numpy(), _col(ent, "committed"))
    assert np.array_equal(c["digest"].cpu().numpy().view(np.uint32).astype(np.uint64), _col(ent, "digest"))
    assert np.array_equal(_u64(c_sh["new_commit"]), _col(ent, "commit"))
    assert np.array_equal(c_sh["digest"].cpu().numpy().view(np.uint32).astype(np.uint64), _col(ent, "digest"))
    assert np.array_equal(_u64(c_hp["new_commit"]), _col(ent, "commit"))
    assert np.array_equal(c_hp["digest"].cpu().numpy().view(np.uint32).astype(np.uint64), _col(ent, "digest"))
    assert np.array_equal(_u64(c["median"]), _col(ent, "median"))
    assert np.array_equal(v["won"].cpu().numpy(), _col(ent, "won"))
    assert np.array_equal(_u64(v["new_commit"]), _col(ent, "vote_commit"))
    assert np.array_equal(ln.cpu().numpy().view(np.uint32), _col(ent, "nc_len"))
    # validate every group's own NC buffer as follower 1's (no mismatch: end of last entry)
    d = dets.cpu().numpy()
    l32 = ln.cpu().numpy().view(np.int32).copy()
    fol = np.ones(G, np.uint8)
    out = eng.log_find_remote_end_offset(db, torch.from_numpy(d).cuda(), torch.from_numpy(l32).cuda(),
                                         torch.from_numpy(fol).cuda(), 256)
    r = eng.poll_vote_requests(db, derive_local=True)
    torch.cuda.synchronize()
    got_end = _u64(out)
    for g in range(G):
        if ent["groups_out"][g]["find_end"] is not None:
            assert got_end[g] == ent["groups_out"][g]["find_end"], g
    assert np.array_equal(_u64(r["last_idx_term"]).reshape(G, 2),
                          np.array([g["lit"] for g in ent["groups_out"]], np.uint64))
    assert np.array_equal(r["outcome"].cpu().numpy(), _col(ent, "rank"))
    assert np.array_equal(_u64(r["new_sid"]), _col(ent, "new_sid"))
    assert np.array_equal(r["cleared"].cpu().numpy().view(np.uint16), _col(ent, "cleared"))
    db2 = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db2, pkg.batch.gen_cfg(**ent["cfg"]))
    p = eng.log_pruning(db2)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(p["min_apply"]), _col(ent, "min_apply"))
    assert np.array_equal(_u64(p["new_head"]), _col(ent, "new_head"))
    assert np.array_equal(p["append_head"].cpu().numpy(), _col(ent, "append"))
    # the same results from one commit call (walk, then the tail launch's median and pruning)
    db3 = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db3, pkg.batch.gen_cfg(**ent["cfg"]))
    t = eng.update_remote_logs(db3, W | CK | MD | pkg.abi.COMMIT_PRUNE | pkg.abi.COMMIT_STATS_FRESH)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(t["new_commit"]), _col(ent, "commit"))
    assert np.array_equal(_u64(t["median"]), _col(ent, "median"))
    assert np.array_equal(_u64(t["min_apply"]), _col(ent, "min_apply"))
    assert np.array_equal(_u64(t["new_head"]), _col(ent, "new_head"))
    assert np.array_equal(t["append_head"].cpu().numpy(), _col(ent, "append"))


def _one_group(pkg, orc, ring, st6, cid, R, self_idx=0):
    ln = int(st6[5])
    hb = orc.host_batch(1, R, ln)
    hb.ring[:ln] = ring[:ln]
    s = state_of(pkg, st6, cid)
    hb.state[:] = s
    hb.self_idx[0] = self_idx
    return hb


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["commit_640", "wrap_commit_128"])
def test_gpu_commit_scenarios(pkg, orc, eng, name):
    import torch
    sc = BY_NAME[name]
    ring, _ = scenario_ring(orc, sc)
    hb = _one_group(pkg, orc, ring, sc["state"], sc["cid"], 3, sc["self"])
    for lane in (False, True):
        db = pkg.batch.DeviceBatch(1, 3, hb.stride)
        db.upload(hb)
        b = db.struct()
        if lane:
            b.flags = pkg.abi.BATCH_LANE_IMPL
        out = eng.update_remote_logs(db, pkg.abi.COMMIT_WALK, bstruct=b)
        torch.cuda.synchronize()
        assert _u64(out["new_commit"])[0] == sc["expect_commit"]
        assert out["committed"].cpu().numpy()[0] == sc["expect_committed"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["vote7_3acks", "vote7_2acks", "transit_5_7_acks12", "transit_5_7_acks125"])
def test_gpu_vote_scenarios(pkg, orc, eng, name):
    import torch
    sc = BY_NAME[name]
    R = 7
    hb = _one_group(pkg, orc, np.zeros(sc["ring_len"] + 64, np.uint8), sc["state"], sc["cid"], R, sc["self"])
    hb.vote_ack[:] = sc["vote_ack"][:R]
    db = pkg.batch.DeviceBatch(1, R, hb.stride)
    db.upload(hb)
    v = eng.poll_vote_count(db)
    torch.cuda.synchronize()
    assert v["won"].cpu().numpy()[0] == sc["expect_won"]
    assert list(v["vote_count"].cpu().numpy()) == sc["expect_vc"]
    assert _u64(v["new_commit"])[0] == sc["expect_commit"]


@pytest.mark.gpu
def test_gpu_find_remote_end_and_prune_scenarios(pkg, orc, eng):
    import torch
    sc = BY_NAME["find_remote_end_192"]
    ring, _ = scenario_ring(orc, sc)
    hb = _one_group(pkg, orc, ring, sc["state"], [0, 3, 0, 0, 0x1FFF], 3)
    db = pkg.batch.DeviceBatch(1, 3, hb.stride)
    db.upload(hb)
    d = np.zeros(256 * 3, np.uint64)
    d[:len(sc["dets"])] = sc["dets"]
    out = eng.log_find_remote_end_offset(db, torch.from_numpy(d.view(np.uint8)).cuda(),
                                         torch.tensor([len(sc["dets"]) // 3], dtype=torch.int32).cuda(),
                                         torch.tensor([1], dtype=torch.uint8).cuda(), 256)
    torch.cuda.synchronize()
    assert _u64(out)[0] == sc["expect_end"]

    sc = BY_NAME["prune_head_128"]
    ring, _ = scenario_ring(orc, sc)
    hb = _one_group(pkg, orc, ring, sc["state"], sc["cid"], 3)
    hb.apply_offsets[:] = sc["apply_offsets"]
    db = pkg.batch.DeviceBatch(1, 3, hb.stride)
    db.upload(hb)
    p = eng.log_pruning(db)
    torch.cuda.synchronize()
    assert _u64(p["min_apply"])[0] == sc["expect_min"]
    assert _u64(p["new_head"])[0] == sc["expect_head"]
    assert p["append_head"].cpu().numpy()[0] == sc["expect_append"]


# ---- tail_vectors.json: update_remote_logs' publish + force_log_pruning (round 5)
TAIL = json.load(open(os.path.join(HERE, "tail_vectors.json")))


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _tail_batch(orc, pkg, name):
    import test_publish_force as tp
    ent = TAIL[name]
    ci = int(name[4:])
    kw, R = tp.FULL[ci]
    assert kw == ent["cfg"] and R == ent["replicas"]
    G = ent["groups"]
    hb = orc.host_batch(G, R, kw["ring_len"])
    orc.gen(hb, pkg.batch.gen_cfg(**kw))
    tp.perturb(hb, np.random.default_rng(100 + ci))
    h = hashlib.sha256(hb.ring.tobytes())
    for k in sorted(hb.arrays):
        h.update(hb.arrays[k].tobytes())
    assert h.hexdigest() == ent["input_sha256"]
    return ent, hb


def _tail_check(ent, out, hb, wm, bad):
    for k, v in ent["out_sha256"].items():
        assert _sha(out[k]) == v, k
    for k, v in ent["force_sha256"].items():
        assert _sha(out["force"][k]) == v, k
    for k, v in ent["after_sha256"].items():
        assert _sha(hb[k] if isinstance(hb, dict) else hb.arrays[k]) == v, k
    assert wm == ent["watermark"] and bad == ent["corrupt"]


@pytest.mark.parametrize("name", sorted(TAIL))
def test_oracle_matches_tail_vectors(orc, pkg, name):
    abi = pkg.abi
    ent, hb = _tail_batch(orc, pkg, name)
    G = hb.G
    commit = orc.commit(hb, abi.COMMIT_WALK)["new_commit"]
    assert _sha(commit) == ent["commit_sha256"]
    flags = abi.COMMIT_PUBLISH | abi.COMMIT_FORCE_PRUNE
    rq = np.arange(G, dtype=np.uint64) + 7
    cl = (np.arange(G) % 60000 + 3).astype(np.uint16)
    out, wm, bad = orc.tail(hb, flags, commit, out=orc.tail_out(G, flags, req_id=rq, clt_id=cl))
    _tail_check(ent, out, hb, wm, bad)
    assert _sha(hb.ring) == ent["ring_after_sha256"]
    assert [int(x) for x in np.bincount(out["force"]["action"], minlength=3)] == ent["actions"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(TAIL))
def test_gpu_matches_tail_vectors(orc, pkg, eng, name):
    """the commit call (walk + publish) and force_log_pruning on the log its
    commit leaves (apus_commit_batch takes them as two calls) reproduce the
    reference-composed vectors, in-place writes included"""
    import torch
    abi = pkg.abi
    ent, hb = _tail_batch(orc, pkg, name)
    G = hb.G
    db = pkg.batch.DeviceBatch(G, hb.R, hb.stride)
    db.add("rc_connected")
    db.upload(hb)
    flags = abi.COMMIT_WALK | abi.COMMIT_PUBLISH | abi.COMMIT_FORCE_PRUNE
    out = eng.alloc_commit_out(G, flags)
    rq = np.arange(G, dtype=np.uint64) + 7
    cl = (np.arange(G) % 60000 + 3).astype(np.uint16)
    out["force"]["req_id"].copy_(torch.from_numpy(rq.view(np.int64)))
    out["force"]["clt_id"].copy_(torch.from_numpy(cl.view(np.int16)))
    eng.stats_reset()
    eng.commit_then_force(db, flags, out=out)
    # the vectors hash the state rows as the reference-composed tail leaves them
    # (it does not write log->commit): the commit column restored for the hash
    eng.set_commit(db, torch.from_numpy(hb.state["commit"].view(np.int64)).cuda())
    torch.cuda.synchronize()
    u = lambda t, dt: t.cpu().numpy().view(dt)   # noqa: E731
    host = {"new_head": u(out["new_head"], np.uint64), "append_head": u(out["append_head"], np.uint8),
            "min_apply": u(out["min_apply"], np.uint64), "publish": u(out["publish"], np.uint16),
            "ssn": u(out["ssn"], np.uint64),
            "force": {"action": u(out["force"]["action"], np.uint8), "target": u(out["force"]["target"], np.uint8),
                      "cfg_idx": u(out["force"]["cfg_idx"], np.uint64),
                      "req_id": u(out["force"]["req_id"], np.uint64),
                      "clt_id": u(out["force"]["clt_id"], np.uint16)}}
    assert _sha(u(out["new_commit"], np.uint64)) == ent["commit_sha256"]
    after = {k: db.download(k) for k in ent["after_sha256"]}
    st = eng.stats()
    _tail_check(ent, host, after, int(st[abi.STAT_MIN_WATERMARK]), int(st[abi.STAT_CORRUPT]))
    assert _sha(db.download("ring")) == ent["ring_after_sha256"]


# ---- win_vectors.json: poll_vote_count whole, the election-win transition (round 6)
WIN = json.load(open(os.path.join(HERE, "win_vectors.json")))


def _win_batch(orc, pkg, name):
    import test_vote_win as tw
    ent = WIN[name]
    hb, io = tw.build(pkg, orc, name)
    assert (hb.G, hb.R) == (ent["groups"], ent["replicas"])
    h = hashlib.sha256(hb.ring.tobytes())
    for k in sorted(hb.arrays):
        h.update(hb.arrays[k].tobytes())
    assert h.hexdigest() == ent["input_sha256"], "trace drifted from the fixture's"
    assert _sha(np.concatenate([io[k].view(np.uint8) for k in sorted(io)])) == ent["io_in_sha256"]
    return ent, hb, io


def _win_check(ent, io, after, ring, bad):
    for k, v in ent["out_sha256"].items():
        assert _sha(io[k]) == v, k
    for k, v in ent["after_sha256"].items():
        assert _sha(after[k]) == v, k
    assert _sha(ring) == ent["ring_after_sha256"]
    assert bad == ent["corrupt"]
    assert [int(x) for x in np.bincount(io["outcome"], minlength=8)] == ent["outcomes"]


@pytest.mark.parametrize("name", sorted(WIN))
def test_oracle_matches_win_vectors(orc, pkg, name):
    """the clean-room tally + win transition reproduce the reference-composed
    poll_vote_count's vectors (tests/golden/make_golden.py win)"""
    ent, hb, io = _win_batch(orc, pkg, name)
    bad = orc.vote_win(hb, io)
    _win_check(ent, io, hb.arrays, hb.ring, bad)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(WIN))
def test_gpu_matches_win_vectors(orc, pkg, eng, name):
    """apus_vote_batch then apus_vote_win_batch on the device reproduce them,
    every byte written in place included"""
    ent, hb, io = _win_batch(orc, pkg, name)
    db = pkg.batch.DeviceBatch(hb.G, hb.R, hb.stride)
    db.upload(hb)
    vo = eng.poll_vote_count(db)
    dio = dict(io)
    for k in ("won", "voters", "new_commit"):
        dio[k] = vo[k]
    eng.stats_reset()
    got = eng.become_leader(db, dio)
    after = {k: db.download(k) for k in ent["after_sha256"]}
    _win_check(ent, got, after, db.download("ring"), int(eng.stats()[pkg.abi.STAT_CORRUPT]))
