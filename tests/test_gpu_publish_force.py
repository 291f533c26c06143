"""update_remote_logs' lazy remote-commit publish (APUS_COMMIT_PUBLISH,
dare_ibv_rc.c:1760-1822) and force_log_pruning (APUS_COMMIT_FORCE_PRUNE,
dare_server.c:2069-2122) in the commit call's tail launch, through the C ABI,
against the oracle (apus_oracle_tail_batch, itself pinned to the transcribed
reference bodies by tests/test_publish_force.py).  Bit-exact: every output,
and every byte the call writes in place (remote_commit, apply_offsets, the
CONFIG entry in the ring, end / tail / cid, prev_head).

The batches are test_publish_force.py's (rings near or past 75% full, every
branch perturbed in), over the four walk kernels: a group the walk kernel
defers (commit_seg_kernel defers every walk longer than its window) is walked
by the tail lane that finishes it, so its new commit feeds the publish.
"""
import numpy as np
import pytest

from test_publish_force import FULL, perturb

pytestmark = pytest.mark.gpu

IMPL_FLAGS = {"wave": 0, "lane": 0x1, "wave_short": 0x2, "wave_hop": 0x8}


@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def _host(pkg, orc, ci, G=2048):
    kw, R = FULL[ci]
    hb = orc.host_batch(G, R, kw["ring_len"])
    orc.gen(hb, pkg.batch.gen_cfg(**kw))
    perturb(hb, np.random.default_rng(500 + ci))
    return hb


def _device(pkg, hb):
    db = pkg.batch.DeviceBatch(hb.G, hb.R, hb.stride)
    db.add("rc_connected")
    db.upload(hb)
    return db


def _run(pkg, orc, eng, hb, flags, impl):
    """the device call and the oracle on copies of the same batch"""
    import torch
    abi = pkg.abi
    G = hb.G
    db = _device(pkg, hb)
    b = db.struct()
    b.flags = IMPL_FLAGS[impl]
    out = eng.alloc_commit_out(G, flags)
    rq = np.arange(G, dtype=np.uint64) * 3 + 1
    cl = (np.arange(G) % 50000 + 9).astype(np.uint16)
    if flags & abi.COMMIT_FORCE_PRUNE:
        out["force"]["req_id"].copy_(torch.from_numpy(rq.view(np.int64)))
        out["force"]["clt_id"].copy_(torch.from_numpy(cl.view(np.int16)))
    ssn0 = np.arange(G, dtype=np.uint64) * 5
    if flags & abi.COMMIT_PUBLISH:
        out["ssn"].copy_(torch.from_numpy(ssn0.view(np.int64)))
    eng.stats_reset()
    if flags & abi.COMMIT_FORCE_PRUNE:
        # the walk call, log->commit = its commit, the force_log_pruning call
        eng.commit_then_force(db, flags, out=out, bstruct=b)
    else:
        eng.update_remote_logs(db, flags, out=out, bstruct=b)
    torch.cuda.synchronize()
    # the oracle: the walk, then (on the walk's commit) the publish and force_log_pruning
    ref = orc.commit(hb, flags & (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN))
    tf = flags & (abi.COMMIT_PUBLISH | abi.COMMIT_FORCE_PRUNE)
    rp = wm = None
    if (flags & abi.COMMIT_PRUNE) and not (flags & abi.COMMIT_FORCE_PRUNE):
        rp, wm = orc.prune(hb)
    to, twm, bad = orc.tail(hb, tf, ref["new_commit"], out=orc.tail_out(G, tf, req_id=rq, clt_id=cl, ssn=ssn0))
    if flags & abi.COMMIT_FORCE_PRUNE:
        hb.state["commit"] = ref["new_commit"]          # the caller's log->commit update between the calls
    return db, out, ref, rp, wm, to, twm, bad


def _check(pkg, db, hb, out, ref, rp, to, flags):
    abi = pkg.abi
    assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"])
    assert np.array_equal(out["committed"].cpu().numpy(), ref["committed"])
    assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"])
    assert np.array_equal(_u64(out["median"]), ref["median"])
    if flags & abi.COMMIT_PUBLISH:
        assert np.array_equal(out["publish"].cpu().numpy().view(np.uint16), to["publish"])
        assert np.array_equal(_u64(out["ssn"]), to["ssn"])
    pr = rp if rp is not None else to
    if flags & (abi.COMMIT_PRUNE | abi.COMMIT_FORCE_PRUNE):
        assert np.array_equal(_u64(out["new_head"]), pr["new_head"])
        assert np.array_equal(out["append_head"].cpu().numpy(), pr["append_head"])
        assert np.array_equal(_u64(out["min_apply"]), pr["min_apply"])
    if flags & abi.COMMIT_FORCE_PRUNE:
        f = out["force"]
        assert np.array_equal(f["action"].cpu().numpy(), to["force"]["action"])
        assert np.array_equal(f["target"].cpu().numpy(), to["force"]["target"])
        assert np.array_equal(_u64(f["cfg_idx"]), to["force"]["cfg_idx"])
        assert np.array_equal(_u64(f["req_id"]), to["force"]["req_id"])
        assert np.array_equal(f["clt_id"].cpu().numpy().view(np.uint16), to["force"]["clt_id"])
    # every byte written in place
    assert np.array_equal(db.download("ring"), hb.ring)
    for k in ("state", "apply_offsets", "remote_commit", "prev_head"):
        assert db.download(k).tobytes() == hb.arrays[k].tobytes(), k


@pytest.mark.parametrize("impl", list(IMPL_FLAGS))
@pytest.mark.parametrize("ci", range(len(FULL)))
def test_publish_force_commit_call(pkg, orc, eng, ci, impl):
    """walk + checksum + median + publish, then force_log_pruning on the log
    the walk's commit leaves (two calls: apus_commit_batch refuses the pair in
    one, dare_server.c:1100-1123) at R = 3, 5, 7"""
    abi = pkg.abi
    hb = _host(pkg, orc, ci)
    flags = (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PUBLISH |
             abi.COMMIT_FORCE_PRUNE)
    db, out, ref, rp, _, to, twm, bad = _run(pkg, orc, eng, hb, flags, impl)
    _check(pkg, db, hb, out, ref, rp, to, flags)
    s = eng.stats()
    assert s[abi.STAT_MIN_WATERMARK] == twm
    assert s[abi.STAT_CORRUPT] == bad + int((ref["committed"] == 0xFF).sum())
    assert s[abi.STAT_DECISIONS] == hb.G
    if impl == "wave_short" and FULL[ci][0]["n_entries"] > 16:
        assert s[abi.STAT_SLOW] > 0          # deferred walks finished by the tail lanes
    acts = set(to["force"]["action"].tolist())
    if ci < 5:
        assert acts == {abi.FORCE_NONE, abi.FORCE_PRUNE, abi.FORCE_REMOVE}


@pytest.mark.parametrize("impl", ["wave", "wave_short"])
@pytest.mark.parametrize("ci", [0, 1, 3])
def test_publish_with_pruning(pkg, orc, eng, ci, impl):
    """publish beside log_pruning (the C2 bench step's flag set)"""
    abi = pkg.abi
    hb = _host(pkg, orc, ci)
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PRUNE | abi.COMMIT_PUBLISH
    db, out, ref, rp, wm, to, _, _ = _run(pkg, orc, eng, hb, flags, impl)
    _check(pkg, db, hb, out, ref, rp, to, flags)
    assert eng.stats()[abi.STAT_MIN_WATERMARK] == wm


@pytest.mark.parametrize("ci", [1, 2, 3])
def test_publish_force_with_failover(pkg, orc, eng, ci):
    """the failover pass (vote tally, ranking on the walk's local (idx, term))
    in the same tail as the publish and force_log_pruning (the FAIL
    instantiation, the C5 step's set with the segment walk's rows)"""
    import torch
    abi = pkg.abi
    hb = _host(pkg, orc, ci)
    for extra in (abi.COMMIT_PRUNE, abi.COMMIT_FORCE_PRUNE):
        h = hb if extra == abi.COMMIT_FORCE_PRUNE else _host(pkg, orc, ci)
        flags = (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_LAST_IT | abi.COMMIT_VOTE |
                 abi.COMMIT_RANK | abi.COMMIT_PUBLISH | extra)
        rv, rr = orc.vote(h), orc.rank(h, use_lit=False)
        db, out, ref, rp, _, to, _, _ = _run(pkg, orc, eng, h, flags, "wave_short")
        torch.cuda.synchronize()
        _check(pkg, db, h, out, ref, rp, to, flags)
        assert np.array_equal(out["vote"]["won"].cpu().numpy(), rv["won"])
        assert np.array_equal(out["rank"]["outcome"].cpu().numpy(), rr["outcome"])
        assert np.array_equal(_u64(out["rank"]["new_sid"]), rr["new_sid"])


def test_publish_force_refusals(pkg, eng):
    """the flags' inputs are checked before anything launches"""
    import ctypes as C
    abi = pkg.abi
    db = pkg.batch.DeviceBatch(64, 3, 1024, fields=["state", "self_idx", "apply_offsets", "remote_end", "lr_step",
                                                     "fail_count"])
    out = eng.alloc_commit_out(64, abi.COMMIT_WALK | abi.COMMIT_PUBLISH | abi.COMMIT_FORCE_PRUNE)
    o = eng.commit_struct(out)
    b = db.struct()
    lib = eng.lib
    s = eng._stream()
    # publish without remote_commit; force without sid
    assert lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), abi.COMMIT_PUBLISH, s) == abi.APUS_ERROR
    assert lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), abi.COMMIT_FORCE_PRUNE, s) == abi.APUS_ERROR
    # a walking call without new_commit
    db2 = pkg.batch.DeviceBatch(64, 3, 1024)
    b2 = db2.struct()
    assert lib.apus_commit_batch(eng.ctx, C.byref(b2), C.byref(o), abi.COMMIT_WALK | abi.COMMIT_FORCE_PRUNE,
                                 s) == abi.APUS_ERROR      # force_log_pruning never beside a walk
    o.new_commit = None
    assert lib.apus_commit_batch(eng.ctx, C.byref(b2), C.byref(o), abi.COMMIT_WALK | abi.COMMIT_PUBLISH,
                                 s) == abi.APUS_ERROR


@pytest.mark.parametrize("ci", [0, 2, 4])
def test_leader_poll_walk_apply_force(pkg, orc, eng, ci):
    """polling()'s leader order (dare_server.c:1100-1124): the
    commit call (walk + checksum + median + publish), log->commit = its commit,
    apply_committed_entries on that log (apus_apply_batch, then its CONFIG
    re-appends through apus_append_batch), then force_log_pruning on the
    applied log -- its minimum starts from the new log->apply.  The oracle runs
    the same sequence; every output and every byte in place bit-exact."""
    import torch
    abi = pkg.abi
    hb = _host(pkg, orc, ci)
    G = hb.G
    db = _device(pkg, hb)
    b = db.struct()
    f1 = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PUBLISH
    out = eng.alloc_commit_out(G, f1 | abi.COMMIT_FORCE_PRUNE)
    rq = np.arange(G, dtype=np.uint64) * 7 + 3
    cl = (np.arange(G) % 40000 + 11).astype(np.uint16)
    ssn0 = np.arange(G, dtype=np.uint64) * 2
    out["force"]["req_id"].copy_(torch.from_numpy(rq.view(np.int64)))
    out["force"]["clt_id"].copy_(torch.from_numpy(cl.view(np.int16)))
    out["ssn"].copy_(torch.from_numpy(ssn0.view(np.int64)))
    apply0 = hb.state["apply"].copy()
    eng.stats_reset()
    # the device: commit call, log->commit, apply (+ its CONFIG re-appends), force_log_pruning
    eng.update_remote_logs(db, f1, out=out, bstruct=b)
    eng.set_commit(db, out["new_commit"])
    aio = orc.apply_io(G, 4)
    dio = eng.apply_committed_entries(db, aio)
    eng.log_append_entry(db, torch.from_numpy(dio["cfg_entries"].view(np.uint8).copy()).cuda(),
                         torch.from_numpy(dio["cfg_payload"]).cuda(), 4,
                         n_entries=torch.from_numpy(dio["n_cfg"]).cuda())
    eng.update_remote_logs(db, abi.COMMIT_FORCE_PRUNE, out=out, bstruct=b)
    torch.cuda.synchronize()
    # the oracle, the same order
    ref = orc.commit(hb, abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN)
    tp, _, _ = orc.tail(hb, abi.COMMIT_PUBLISH, ref["new_commit"], out=orc.tail_out(G, abi.COMMIT_PUBLISH, ssn=ssn0))
    hb.state["commit"] = ref["new_commit"]
    orc.apply(hb, aio)
    orc.append(hb, aio["cfg_entries"], aio["cfg_payload"], 4, n_entries=aio["n_cfg"])
    tf, twm, bad = orc.tail(hb, abi.COMMIT_FORCE_PRUNE, hb.state["commit"],
                            out=orc.tail_out(G, abi.COMMIT_FORCE_PRUNE, req_id=rq, clt_id=cl))
    assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"])
    assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"])
    assert np.array_equal(out["publish"].cpu().numpy().view(np.uint16), tp["publish"])
    assert np.array_equal(_u64(out["ssn"]), tp["ssn"])
    for k in ("req_id", "clt_id", "last_applied", "last_csm_idx", "n_applied", "departed", "events", "n_cfg"):
        assert np.array_equal(dio[k], aio[k]), k
    f = out["force"]
    assert np.array_equal(f["action"].cpu().numpy(), tf["force"]["action"])
    assert np.array_equal(f["target"].cpu().numpy(), tf["force"]["target"])
    assert np.array_equal(_u64(f["cfg_idx"]), tf["force"]["cfg_idx"])
    assert np.array_equal(_u64(f["req_id"]), tf["force"]["req_id"])
    assert np.array_equal(f["clt_id"].cpu().numpy().view(np.uint16), tf["force"]["clt_id"])
    assert np.array_equal(_u64(out["new_head"]), tf["new_head"])
    assert np.array_equal(_u64(out["min_apply"]), tf["min_apply"])
    assert np.array_equal(db.download("ring"), hb.ring)
    for k in ("state", "apply_offsets", "remote_commit", "prev_head"):
        assert db.download(k).tobytes() == hb.arrays[k].tobytes(), k
    assert eng.stats()[abi.STAT_MIN_WATERMARK] == twm
    # the apply moved log->apply on some groups before the forced pruning read it
    assert (hb.state["apply"] != apply0).any()
    assert len(set(tf["force"]["action"].tolist())) >= 2
