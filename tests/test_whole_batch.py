"""Every group of every full-size BASELINE batch against the REFERENCE's own
code (north_star: "bit-exact commit indices and vote outcomes for >= 64M
groups per batch").

Each test generates the batch in HBM exactly as `bench.py --workload X` does,
downloads its inputs chunk by chunk BEFORE the step and runs
oracle/_ref's ref_check_batch on them (the reference's dare_log.h compiled
from its sources, with the transcribed dare_ibv_rc.c / dare_server.c loop
bodies on top; the .so travels with the tree), then runs the bench's own step
-- ONE apus_commit_batch call with the bench's flags -- and requires every
output of every group, and every column the step writes in place
(remote_commit by the publish, the OFF servers' apply_offsets by the
pruning), to equal the reference's.  tests/test_ref_check.py pins
ref_check_batch to the clean-room oracle.

Host memory: one chunk of inputs (<= ~17 GB) plus the reference's outputs
(~150 B per group) at a time.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_REF_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                       "libapusref.so")

# bench.py's own workload table (the same generator parameters; the flags below are its step's)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import WORKLOADS as _W  # noqa: E402
_IN = ("state", "self_idx", "remote_end", "remote_commit", "lr_step", "fail_count", "apply_offsets", "prev_head")
_VIN = ("vote_ack", "hb", "vote_req", "sid")


@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _per_group_bytes(pkg, name, R):
    f = {x[0]: (x[1], x[2]) for x in pkg.batch.FIELDS}[name]
    return np.dtype(f[0]).itemsize * f[1](R)


def _np(t, dt):
    return t.cpu().numpy().view(dt)


@pytest.mark.parametrize("workload", ["c2", "c5", "c4", "c3", "c4_1gpu"])
def test_whole_batch_equals_reference(pkg, orc, eng, workload):
    import torch
    if not os.path.exists(_REF_SO):
        pytest.skip("oracle/_ref not built (no /root/reference where the tree was built)")
    abi = pkg.abi
    wl = _W[workload]
    G, R, votes = wl["G"], wl["R"], wl.get("votes", False)
    stride = pkg.batch.ring_stride_for(wl["ring"])
    fields = list(_IN) + (list(_VIN) + ["last_idx_term", "abs_base"] if votes else ["abs_base"])
    db = pkg.batch.DeviceBatch(G, R, stride, fields=fields)
    cfg = pkg.batch.gen_cfg(seed=2026, n_entries=wl["E"], n_history=wl["H"], len_min=wl["L"],
                            len_max=wl.get("Lmax", wl["L"]), ring_len=wl["ring"], p_full_ack=0.9, straggler=True,
                            cid_mix=wl.get("cid_mix", False), p_vote_ack=0.6, hist_len_max=wl.get("Hmax", 0))
    eng.gen(db, cfg)
    var = wl.get("var_len", False)
    E, F = wl["E"], R - 1
    if var:
        # C3: each follower's NC buffer as bench.py builds it -- the leader's
        # determinants with the term changed from m_r ~ U[0, E] on, some
        # buffers emptied or halved; followers self + 1 .. self + F
        dets, ln = eng.log_entries_to_nc_buf(db, E)
        gq = torch.Generator(device="cuda:0").manual_seed(33)
        dv = dets.view(torch.int64).view(G, 1, E, 3).repeat(1, F, 1, 1).contiguous()
        m_r = torch.randint(0, E + 1, (G, F, 1), device=dv.device, generator=gq)
        dv[..., 1] += (torch.arange(E, device=dv.device).view(1, 1, E) >= m_r).to(torch.int64)
        cut = torch.randint(0, 8, (G, F), device=dv.device, generator=gq)
        nl = ln.view(G, 1).repeat(1, F)
        nl = torch.where(cut == 0, torch.zeros_like(nl), torch.where(cut == 1, nl // 2, nl)).contiguous()
        fol = ((db.arrays["self_idx"].view(G, 1).to(torch.int64) + 1 +
                torch.arange(F, device=dv.device).view(1, F)) % R).to(torch.uint8).contiguous()
        del dets, ln, m_r, cut
    torch.cuda.synchronize()

    # 1. the reference's results on the inputs as generated, chunk by chunk
    chunk = max(1, min(G, (16 << 30) // (stride + 512)))
    ref = None
    for c0 in range(0, G, chunk):
        c1 = min(G, c0 + chunk)
        ins = {"ring": db.ring[c0 * stride:c1 * stride].cpu().numpy()}
        for k in _IN + (_VIN if votes else ()):
            pb = _per_group_bytes(pkg, k, R)
            ins[k] = db.arrays[k][c0 * pb:c1 * pb].cpu().numpy()
        folw = None
        if var:
            folw = (dv[c0:c1].cpu().numpy().reshape(-1).view(np.uint64), nl[c0:c1].cpu().numpy().reshape(-1)
                    .view(np.uint32), fol[c0:c1].cpu().numpy().reshape(-1), F, E)
        rc = orc.ref_check(c1 - c0, R, stride, ins, votes, nc_max=E if var else 0, followers=folw)
        del ins, folw
        if ref is None:
            ref = {k: np.zeros(v.size // (c1 - c0) * G, v.dtype) for k, v in rc.items()}
        for k, v in rc.items():
            per = v.size // (c1 - c0)
            ref[k][c0 * per:c1 * per] = v
        del rc

    # 2. bench.py's step: one commit call with the bench's flags
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PUBLISH | abi.COMMIT_PRUNE | \
        abi.COMMIT_STATS_FRESH
    b = db.struct()
    nc_max = 0
    if wl.get("var_len"):
        b.flags = abi.BATCH_VAR_LEN
        flags |= abi.COMMIT_NC                  # the bench's C3 walk writes the NC determinants too
        nc_max = wl["E"]
    elif wl.get("short"):
        b.flags = abi.BATCH_SHORT_WALKS
    if votes:
        flags |= abi.COMMIT_LAST_IT | abi.COMMIT_VOTE | abi.COMMIT_RANK
    out = eng.update_remote_logs(db, flags, bstruct=b, nc_max=nc_max)
    if var:
        # the bench's validation call, on the leader's determinants the walk wrote
        vout = eng.log_find_remote_end_offset(db, dv.view(torch.uint8), nl, fol, E,
                                              leader=(out["nc_dets"], out["nc_len"], E))
    torch.cuda.synchronize()
    st = eng.stats()
    assert st[abi.STAT_DECISIONS] == G and st[abi.STAT_CORRUPT] == 0

    # 3. every group, every output
    def eq(dev, dt, key):
        a = _np(dev, dt)
        if not np.array_equal(a, ref[key]):
            bad = np.flatnonzero(a != ref[key])
            raise AssertionError(f"{workload} {key}: {bad.size} differ, first at {bad[0]}: "
                                 f"gpu {a[bad[0]]} reference {ref[key][bad[0]]}")
    eq(out["new_commit"], np.uint64, "new_commit")
    eq(out["committed"], np.uint8, "committed")
    eq(out["digest"], np.uint32, "digest")
    eq(out["median"], np.uint64, "median")
    eq(out["publish"], np.uint16, "publish")
    eq(out["ssn"], np.uint64, "ssn")
    eq(db.arrays["remote_commit"], np.uint64, "rcommit_out")
    eq(out["new_head"], np.uint64, "new_head")
    eq(out["append_head"], np.uint8, "append_head")
    eq(out["min_apply"], np.uint64, "min_apply")
    eq(db.arrays["apply_offsets"], np.uint64, "apply_out")
    assert (ref["committed"] == 1).sum() > G // 2 and (ref["publish"] != 0).any()
    if var:
        eq(out["nc_len"], np.uint32, "nc_len")
        ln_ = ref["nc_len"].astype(np.int64)
        live = (np.arange(E)[None, :] < ln_[:, None]).repeat(3, axis=1).reshape(-1)
        got = _np(out["nc_dets"], np.uint64)
        assert np.array_equal(np.where(live, got, 0), np.where(live, ref["nc_dets"], 0)), "nc_dets"
        eq(vout, np.uint64, "rend_follow")
        assert (ref["rend_follow"] != ~np.uint64(0)).all() and np.unique(ref["rend_follow"][:1 << 16]).size > 100
        del dv, nl, fol, vout
    if votes:
        v, r = out["vote"], out["rank"]
        eq(v["won"], np.uint8, "won")
        eq(v["vote_count"], np.uint8, "vc")
        eq(v["new_commit"], np.uint64, "vote_commit")
        eq(out["last_idx_term"], np.uint64, "lit")
        eq(r["outcome"], np.uint8, "outcome")
        eq(r["new_sid"], np.uint64, "new_sid")
        eq(r["new_cid"], np.uint8, "new_cid")
        eq(r["cleared"], np.uint16, "cleared")
        assert set(np.unique(ref["outcome"])) >= {0, 2, 3, 4} and ref["won"].any()
    del db, out, ref
    torch.cuda.empty_cache()


def test_whole_c5_election_win_equals_reference(pkg, orc, eng):
    """bench.py --workload c5's cold step: the commit call's tally, then
    apus_vote_win_batch on every group of the 2^23-group shard (the
    candidates that won become leaders: SID L bit, configuration scan, apply,
    the blank entry, apply_offsets = head) against oracle/_ref's
    poll_vote_count -- transcribed whole on the reference's log primitives --
    run on the pre-transition copy of every group: every ring byte, state row,
    column and output."""
    import torch
    if not os.path.exists(_REF_SO):
        pytest.skip("oracle/_ref not built (no /root/reference where the tree was built)")
    abi = pkg.abi
    wl = _W["c5"]
    G, R = wl["G"], wl["R"]
    stride = pkg.batch.ring_stride_for(wl["ring"])
    db = pkg.batch.DeviceBatch(G, R, stride)
    eng.gen(db, pkg.batch.gen_cfg(seed=2026, n_entries=wl["E"], n_history=wl["H"], len_min=wl["L"], len_max=wl["L"],
                                  ring_len=wl["ring"], p_full_ack=0.9, straggler=True, cid_mix=True, p_vote_ack=0.6))
    b = db.struct()
    b.flags = abi.BATCH_SHORT_WALKS
    flags = (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PUBLISH | abi.COMMIT_PRUNE |
             abi.COMMIT_STATS_FRESH | abi.COMMIT_LAST_IT | abi.COMMIT_VOTE | abi.COMMIT_RANK)
    out = eng.update_remote_logs(db, flags, bstruct=b)
    dev = torch.device("cuda:0")
    z = lambda dt, n=1: torch.zeros(G * n, dtype=dt, device=dev)   # noqa: E731
    st64 = db.arrays["state"].view(torch.int64).view(G, 8)
    dio = {"won": out["vote"]["won"], "voters": out["vote"]["voters"], "new_commit": out["vote"]["new_commit"],
           "cid_offset": st64[:, 2].clone(), "cid_idx": z(torch.int64), "req_id": z(torch.int64),
           "clt_id": z(torch.int16), "last_applied": z(torch.int64, 3), "last_csm_idx": z(torch.int64),
           "last_write_csm_idx": z(torch.int64), "outcome": z(torch.uint8), "events": z(torch.uint8),
           "departed": z(torch.int16), "n_applied": z(torch.int32), "n_cfg": z(torch.int32)}
    keys = ("state", "sid", "remote_commit", "lr_step", "apply_offsets", "prev_head")
    pre = {k: db.arrays[k].clone() for k in keys}
    pre["ring"] = db.ring.clone()                  # the rings as the transition finds them (HBM holds both)
    pre_off = dio["cid_offset"].clone()
    eng.stats_reset()
    eng.become_leader(db, dio, bstruct=b)
    torch.cuda.synchronize()
    assert eng.stats()[abi.STAT_CORRUPT] == 0

    io_dt = {"cid_offset": np.uint64, "cid_idx": np.uint64, "req_id": np.uint64, "clt_id": np.uint16,
             "last_applied": np.uint64, "last_csm_idx": np.uint64, "last_write_csm_idx": np.uint64,
             "outcome": np.uint8, "events": np.uint8, "departed": np.uint16, "n_applied": np.uint32,
             "n_cfg": np.uint32}
    col_dt = {"state": np.uint8, "sid": np.uint64, "remote_commit": np.uint64, "lr_step": np.uint8,
              "apply_offsets": np.uint64, "prev_head": np.uint8, "self_idx": np.uint8, "vote_ack": np.uint64}
    counts = np.zeros(8, np.int64)
    chunk = 1 << 20
    for c0 in range(0, G, chunk):
        c1 = min(G, c0 + chunk)
        n = c1 - c0
        arr = {"ring": pre["ring"][c0 * stride:c1 * stride].cpu().numpy()}
        for k, dt in col_dt.items():
            pb = _per_group_bytes(pkg, k, R)
            src = pre[k] if k in pre else db.arrays[k]      # self_idx / vote_ack: not written by the transition
            arr[k] = src[c0 * pb:c1 * pb].cpu().numpy().view(dt)
        io = {k: np.zeros(n * (3 if k == "last_applied" else 1), dt) for k, dt in io_dt.items()}
        io["cid_offset"][:] = pre_off[c0:c1].cpu().numpy().view(np.uint64)
        orc.ref_vote_count_batch(n, R, stride, arr, io)
        ring_dev = db.ring[c0 * stride:c1 * stride].cpu().numpy()
        if not np.array_equal(ring_dev, arr["ring"]):
            bad = np.flatnonzero(ring_dev != arr["ring"])
            raise AssertionError(f"ring bytes differ: {bad.size}, first in group {c0 + bad[0] // stride}")
        del ring_dev
        for k in keys:
            pb = _per_group_bytes(pkg, k, R)
            got = db.arrays[k][c0 * pb:c1 * pb].cpu().numpy().view(col_dt[k])
            assert np.array_equal(got, arr[k]), (k, c0, np.flatnonzero(got != arr[k])[:4])
        for k, dt in io_dt.items():
            w = 3 if k == "last_applied" else 1
            got = dio[k][c0 * w:c1 * w].cpu().numpy().view(dt)
            assert np.array_equal(got, io[k]), (k, c0, np.flatnonzero(got != io[k])[:4])
        counts += np.bincount(io["outcome"], minlength=8)
        del arr, io
    # every branch of the blank-entry decision happens in the shard (not NOOP:
    # the generator writes no un-applied CONFIG entry past cid_idx)
    for o in (abi.WIN_NOT_CANDIDATE, abi.WIN_LOST, abi.WIN_CONFIG, abi.WIN_TRANSIT, abi.WIN_STABLE,
              abi.WIN_UNDEFINED):
        assert counts[o] > 0, (o, counts)
    assert counts[abi.WIN_CORRUPT] == 0 and counts.sum() == G
    del db, out, dio, pre
    torch.cuda.empty_cache()


@pytest.mark.parametrize("shape", ["c2", "c5"])
def test_whole_append_persist_equals_reference(pkg, orc, eng, shape):
    """SURVEY 8f.1 at scripts/kbench.py's shapes: every group appends M SEND
    messages of 64 B with apus_append_batch (C2: 2^20 groups x 64 messages,
    the wave kernel; C5: 2^22 7-replica groups x 16, the four-groups-per-wave
    kernel), then every replica copy persists from the pre-append end with
    apus_persist_batch -- against the reference's OWN log_append_entry
    (dare_log.h:466-558, compiled from its sources: ref_append_batch) and the
    persist walk (ref_persist_batch) run on the pre-append copy: every ring
    byte, end / tail / prev_head, each message's index, last_idx, the cursors."""
    import torch
    if not os.path.exists(_REF_SO):
        pytest.skip("oracle/_ref not built (no /root/reference where the tree was built)")
    G, R, E, ring, M, cid = {"c2": (1 << 20, 3, 64, 16384, 64, False), "c5": (1 << 22, 7, 16, 8192, 16, True)}[shape]
    L = 64
    stride = pkg.batch.ring_stride_for(ring)
    db = pkg.batch.DeviceBatch(G, R, stride)
    eng.gen(db, pkg.batch.gen_cfg(seed=2026, n_entries=E, n_history=16, ring_len=ring, p_full_ack=0.9,
                                  straggler=True, cid_mix=cid, p_vote_ack=0.6))
    # kbench's messages: random req / clt ids, type SEND, back-to-back payloads
    n, need = G * M, 2 + L
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
    keys = ("state", "prev_head")
    pre = {k: db.arrays[k].clone() for k in keys}
    pre["ring"] = db.ring.clone()
    end0 = db.arrays["state"].view(torch.int64).view(G, 8)[:, 3].clone()
    old_end = end0.repeat_interleave(R).contiguous()
    eng.stats_reset()
    ao = eng.log_append_entry(db, ent.view(-1), payload, M)
    eng.persist_new_entries(db, old_end)
    torch.cuda.synchronize()
    assert eng.stats()[pkg.abi.STAT_CORRUPT] == 0

    pay_h = payload.cpu().numpy()
    ent_h = ent.cpu().numpy().reshape(-1)
    del payload, ent, pv, e64
    chunk = 1 << 20
    full = appended = 0
    for c0 in range(0, G, chunk):
        c1 = min(G, c0 + chunk)
        k = c1 - c0
        arr = {"ring": pre["ring"][c0 * stride:c1 * stride].cpu().numpy(),
               "state": pre["state"][64 * c0:64 * c1].cpu().numpy(),
               "prev_head": pre["prev_head"][c0:c1].cpu().numpy(),
               "sid": db.arrays["sid"][8 * c0:8 * c1].cpu().numpy().view(np.uint64),
               "self_idx": db.arrays["self_idx"][c0:c1].cpu().numpy()}
        idx, last, bad = orc.ref_append_batch(k, stride, arr, ent_h[24 * M * c0:24 * M * c1], pay_h, M)
        assert bad == 0
        oe = np.repeat(end0[c0:c1].cpu().numpy().view(np.uint64), R)
        assert orc.ref_persist_batch(k, R, stride, arr, oe) == 0
        got = db.ring[c0 * stride:c1 * stride].cpu().numpy()
        if not np.array_equal(got, arr["ring"]):
            b = np.flatnonzero(got != arr["ring"])
            raise AssertionError(f"{shape}: {b.size} ring bytes differ, first in group {c0 + b[0] // stride}")
        del got
        for key in keys:
            pb = _per_group_bytes(pkg, key, R)
            assert np.array_equal(db.arrays[key][c0 * pb:c1 * pb].cpu().numpy(), arr[key].view(np.uint8)), key
        assert np.array_equal(_np(ao["idx"][c0 * M:c1 * M], np.uint64), idx), "idx"
        assert np.array_equal(_np(ao["last_idx"][c0:c1], np.uint64), last), "last_idx"
        assert np.array_equal(_np(old_end[c0 * R:c1 * R], np.uint64), oe), "old_end"
        full += int((idx.reshape(k, M) == 0).any(axis=1).sum())
        appended += int((idx != 0).sum())
        del arr
    # C2's 16-KiB rings fill up: appends that return 0 (a full log) occur
    assert appended > G * M // 2 and (full > 0 or shape != "c2"), (appended, full)
    del db, pre, old_end, ao
    torch.cuda.empty_cache()


@pytest.mark.parametrize("shape", ["c2", "c5"])
def test_whole_apply_config_scan_equals_reference(pkg, orc, eng, shape):
    """SURVEY 8f.2 on every group at the C2 shape (2^20 groups x R=3, 16-KiB
    rings) and the C5 shape (2^22 x R=7, 8-KiB): logs with every entry type
    (NOOP / CONFIG / HEAD / client entries of 0-64 B), STABLE / EXTENDED /
    TRANSIT configurations, leaders and followers, the state row's cid changed
    on half the groups (more servers on; a later epoch on some) so CONFIG
    entries move the configuration.  apus_apply_batch from head
    (apply_committed_entries, max_cfg = 4 re-appends recorded) and
    apus_config_scan_batch from head (poll_config_entries), each on the same
    pre-state, against the transcribed reference bodies on the reference's
    own primitives (ref_apply_batch / ref_config_scan_batch): every state row
    and every output."""
    import torch
    if not os.path.exists(_REF_SO):
        pytest.skip("oracle/_ref not built (no /root/reference where the tree was built)")
    G, R, E, ring = {"c2": (1 << 20, 3, 64, 16384), "c5": (1 << 22, 7, 16, 8192)}[shape]
    stride = pkg.batch.ring_stride_for(ring)
    db = pkg.batch.DeviceBatch(G, R, stride)
    eng.gen(db, pkg.batch.gen_cfg(seed=2027, n_entries=E, n_history=16, len_min=0, len_max=64, ring_len=ring,
                                  p_full_ack=0.9, straggler=True, cid_mix=True, type_mix=True, self_random=True))
    dev = torch.device("cuda:0")
    gq = torch.Generator(device="cuda").manual_seed(21)
    st64 = db.arrays["state"].view(torch.int64).view(G, 8)
    st64[:, 1] = st64[:, 0]                                          # apply = head
    sb = db.arrays["state"].view(G, 64)
    bm = sb[:, 60:64].contiguous().view(torch.int32).view(G)
    more = torch.rand(G, device=dev, generator=gq) < 0.5
    sb[:, 60:64] = torch.where(more, bm | 0xFF, bm).view(torch.uint8).view(G, 4)
    later = torch.rand(G, device=dev, generator=gq) < 0.25
    st64[:, 6] += later.to(torch.int64)                              # cid.epoch
    self_ = db.arrays["self_idx"].to(torch.int64)
    lead = torch.rand(G, device=dev, generator=gq) < 0.6
    term = torch.randint(1, 50, (G,), device=dev, generator=gq)
    idx = torch.where(lead, self_, (self_ + 1) % R)
    db.arrays["sid"].view(torch.int64).copy_((term << 9) | (lead.to(torch.int64) << 8) | idx)
    pre = db.arrays["state"].clone()
    MC = 4
    z = lambda dt, n=1: torch.zeros(G * n, dtype=dt, device=dev)   # noqa: E731
    aio = {"req_id": z(torch.int64), "clt_id": z(torch.int16), "last_applied": z(torch.int64, 3),
           "last_csm_idx": z(torch.int64), "n_applied": z(torch.int32), "departed": z(torch.int16),
           "events": z(torch.uint8), "cfg_entries": z(torch.uint8, 24 * MC), "cfg_payload": z(torch.uint8, 16 * MC),
           "n_cfg": z(torch.int32), "max_cfg": MC}
    eng.stats_reset()
    eng.apply_committed_entries(db, aio)
    post_apply = db.arrays["state"].clone()
    db.arrays["state"].copy_(pre)
    cio = {"cid_offset": st64[:, 0].clone(), "cid_idx": z(torch.int64), "req_id": z(torch.int64),
           "clt_id": z(torch.int16), "departed": z(torch.int16)}
    eng.poll_config_entries(db, cio)
    torch.cuda.synchronize()
    assert eng.stats()[pkg.abi.STAT_CORRUPT] == 0
    a_dt = {"req_id": np.uint64, "clt_id": np.uint16, "last_applied": np.uint64, "last_csm_idx": np.uint64,
            "n_applied": np.uint32, "departed": np.uint16, "events": np.uint8, "cfg_entries": np.uint8,
            "cfg_payload": np.uint8, "n_cfg": np.uint32}
    c_dt = {"cid_offset": np.uint64, "cid_idx": np.uint64, "req_id": np.uint64, "clt_id": np.uint16,
            "departed": np.uint16}
    per = {"last_applied": 3, "cfg_entries": 24 * MC, "cfg_payload": 16 * MC}
    chunk = 1 << 20
    seen = {"n_cfg": 0, "departed_apply": 0, "departed_scan": 0, "req_scan": 0}
    for c0 in range(0, G, chunk):
        c1 = min(G, c0 + chunk)
        k = c1 - c0
        rg = db.ring[c0 * stride:c1 * stride].cpu().numpy()
        s_a = pre[64 * c0:64 * c1].cpu().numpy()
        s_c = s_a.copy()
        io = {key: np.zeros(k * per.get(key, 1), dt) for key, dt in a_dt.items()}
        io["max_cfg"] = MC
        assert orc.ref_apply_batch(k, stride, rg, s_a, db.arrays["self_idx"][c0:c1].cpu().numpy(),
                                   db.arrays["sid"][8 * c0:8 * c1].cpu().numpy().view(np.uint64), io) == 0
        assert np.array_equal(post_apply[64 * c0:64 * c1].cpu().numpy(), s_a), "apply: state rows"
        # the records' data_off index the batch's payload rows: j = g * max_cfg + k over the whole batch
        rec = io["cfg_entries"].view(pkg.batch.APPEND_DT).reshape(k, MC)
        live = np.arange(MC)[None, :] < io["n_cfg"][:, None].astype(np.int64)
        rec["data_off"] += np.where(live, np.uint64(16 * MC * c0), np.uint64(0))
        for key, dt in a_dt.items():
            cnt = per.get(key, 1)
            got = aio[key][c0 * cnt:c1 * cnt].cpu().numpy().view(dt)
            assert np.array_equal(got, io[key]), ("apply", key, c0)
        cc = {key: np.zeros(k, dt) for key, dt in c_dt.items()}
        cc["cid_offset"][:] = s_c.view(np.uint64).reshape(k, 8)[:, 0]
        assert orc.ref_config_scan_batch(k, stride, rg, s_c, cc) == 0
        assert np.array_equal(db.arrays["state"][64 * c0:64 * c1].cpu().numpy(), s_c), "config scan: state rows"
        for key, dt in c_dt.items():
            assert np.array_equal(cio[key][c0:c1].cpu().numpy().view(dt), cc[key]), ("config scan", key, c0)
        seen["n_cfg"] += int(io["n_cfg"].sum())
        seen["departed_apply"] += int((io["departed"] != 0).sum())
        seen["departed_scan"] += int((cc["departed"] != 0).sum())
        seen["req_scan"] += int((cc["req_id"] != 0).sum())
        del rg, s_a, s_c
    assert all(v > 0 for v in seen.values()), seen
    del db, pre, post_apply, aio, cio
    torch.cuda.empty_cache()


@pytest.mark.parametrize("shape", ["c2", "c5"])
def test_whole_log_adjust_completion_equals_reference(pkg, orc, eng, shape):
    """SURVEY 8f.2's replication step machine on every group at the C2 shape
    (2^20 x R=3, 64 determinants per NC buffer) and the C5 shape (2^22 x R=7,
    16): tests/test_lr_step.py's column model drawn on the device (steps 0..7
    and 255, fail counts around PERMANENT_FAILURE, send flags, rc_connected
    masks, vote ACKs, every server's NC buffer the leader's determinants with a
    term mismatch, truncated, empty or longer than max_dets), then
    apus_log_adjust_batch and apus_lr_completion_batch on the posts it made,
    against the transcribed log_adjustment / handle_lr_work_completion on the
    reference's own primitives (ref_log_adjust_batch / ref_lr_completion_batch):
    every state row, column and output."""
    import torch
    if not os.path.exists(_REF_SO):
        pytest.skip("oracle/_ref not built (no /root/reference where the tree was built)")
    G, R, E, ring = {"c2": (1 << 20, 3, 64, 16384), "c5": (1 << 22, 7, 16, 8192)}[shape]
    M = E
    stride = pkg.batch.ring_stride_for(ring)
    db = pkg.batch.DeviceBatch(G, R, stride)
    eng.gen(db, pkg.batch.gen_cfg(seed=2028, n_entries=E, n_history=16, len_min=0, len_max=64, ring_len=ring,
                                  p_full_ack=0.9, straggler=True, cid_mix=True, type_mix=True, self_random=True))
    dev = torch.device("cuda:0")
    gq = torch.Generator(device="cuda").manual_seed(31)
    n = G * R
    rnd = lambda *s: torch.rand(*s, device=dev, generator=gq)              # noqa: E731
    rint = lambda lo, hi, *s: torch.randint(lo, hi, s, device=dev, generator=gq)   # noqa: E731
    st64 = db.arrays["state"].view(torch.int64).view(G, 8)
    lens = st64[:, 5].repeat_interleave(R)
    db.arrays["lr_step"].copy_(torch.where(rnd(n) < 0.05, 255, rint(0, 8, n)).to(torch.uint8))
    db.arrays["fail_count"].copy_(torch.tensor([0, 0, 0, 1, 2, 3], device=dev)[rint(0, 6, n)].to(torch.uint8))
    db.arrays["vote_ack"].view(torch.int64).copy_(torch.where(rnd(n) < 0.25, lens, rint(0, 1 << 40, n) % lens))
    db.arrays["remote_commit"].view(torch.int64).copy_(rint(0, 1 << 40, n) % lens)
    db.arrays["remote_end"].view(torch.int64).copy_(rint(0, 1 << 40, n) % lens)
    dets, dl = eng.log_entries_to_nc_buf(db, M)
    nc = dets.view(torch.int64).view(G, 1, M, 3).repeat(1, R, 1, 1).contiguous()
    del dets
    k0 = dl.to(torch.int64).view(G, 1).expand(G, R)
    mode = rint(0, 5, G, R)
    m = (rnd(G, R) * k0.to(torch.float64)).to(torch.int64).clamp(max=M - 1)
    mis = (mode == 1) & (k0 > 0)
    nc[..., 1] += (mis.view(G, R, 1) & (torch.arange(M, device=dev).view(1, 1, M) == m.view(G, R, 1))).to(torch.int64)
    nc_len = torch.where(mode == 2, (rnd(G, R) * (k0 + 1).to(torch.float64)).to(torch.int64).clamp(max=k0),
                         torch.where(mode == 3, torch.zeros_like(k0), torch.where(mode == 4, M + rint(1, 50, G, R),
                                                                                   k0)))
    nc_len = nc_len.contiguous().view(-1)
    dio = {"send_flag": (rnd(n) < 0.8).to(torch.uint8), "send_count": rint(0, 4, n).to(torch.uint8),
           "wc": torch.zeros(n, dtype=torch.uint8, device=dev),
           "rc_connected": torch.where(rnd(G) < 0.8, 0xFFFF, rint(0, 1 << 16, G)).to(torch.int16),
           "nc_len": nc_len, "nc_dets": nc.view(-1), "ssn": rint(0, 1 << 50, G),
           "post": torch.zeros(n, dtype=torch.uint8, device=dev), "max_dets": M}
    cols = ("lr_step", "remote_commit", "remote_end")
    pre = {k: db.arrays[k].clone() for k in cols + ("state",)}
    pre_io = {k: dio[k].clone() for k in ("send_flag", "send_count", "ssn")}
    eng.log_adjustment(db, dio)
    torch.cuda.synchronize()
    # the posted writes complete (success, or a seeded failure)
    dio["wc"] = torch.where(dio["post"] != 0, torch.where(rnd(n) < 0.85, 1, 2), 0).to(torch.uint8)
    mid = {k: db.arrays[k].clone() for k in cols + ("state",)}
    mid_io = {k: dio[k].clone() for k in ("ssn", "post")}
    eng.handle_lr_work_completion(db, dio)
    torch.cuda.synchronize()

    chunk = 1 << 20
    posted = [0, 0, 0, 0]
    moved = 0
    for c0 in range(0, G, chunk):
        c1 = min(G, c0 + chunk)
        k = c1 - c0
        sl, slr = slice(c0, c1), slice(c0 * R, c1 * R)
        arr = {"ring": db.ring[c0 * stride:c1 * stride].cpu().numpy(),
               "state": pre["state"][64 * c0:64 * c1].cpu().numpy(),
               "self_idx": db.arrays["self_idx"][sl].cpu().numpy(),
               "fail_count": db.arrays["fail_count"][slr].cpu().numpy(),
               "lr_step": pre["lr_step"][slr].cpu().numpy(),
               "vote_ack": db.arrays["vote_ack"][8 * c0 * R:8 * c1 * R].cpu().numpy().view(np.uint64),
               "remote_commit": pre["remote_commit"][8 * c0 * R:8 * c1 * R].cpu().numpy().view(np.uint64),
               "remote_end": pre["remote_end"][8 * c0 * R:8 * c1 * R].cpu().numpy().view(np.uint64)}
        io = {"send_flag": pre_io["send_flag"][slr].cpu().numpy(), "send_count": pre_io["send_count"][slr].cpu().numpy(),
              "rc_connected": dio["rc_connected"][sl].cpu().numpy().view(np.uint16),
              "nc_len": nc_len[slr].cpu().numpy().view(np.uint64), "nc_dets": nc[sl].cpu().numpy().reshape(-1)
              .view(np.uint64), "ssn": pre_io["ssn"][sl].cpu().numpy().view(np.uint64),
              "post": np.zeros(k * R, np.uint8), "max_dets": M}
        s0 = arr["state"].copy()
        orc.ref_log_adjust_batch(k, R, stride, arr, io)
        assert np.array_equal(mid["state"][64 * c0:64 * c1].cpu().numpy(), arr["state"]), ("adjust: state", c0)
        for key in cols:
            pb = _per_group_bytes(pkg, key, R)
            got = mid[key][c0 * pb:c1 * pb].cpu().numpy().view(arr[key].dtype)
            assert np.array_equal(got, arr[key]), ("adjust", key, c0)
        assert np.array_equal(mid_io["ssn"][sl].cpu().numpy().view(np.uint64), io["ssn"]), ("adjust: ssn", c0)
        assert np.array_equal(mid_io["post"][slr].cpu().numpy(), io["post"]), ("adjust: post", c0)
        io["wc"] = dio["wc"][slr].cpu().numpy()
        orc.ref_lr_completion_batch(arr["lr_step"], io)
        assert np.array_equal(db.arrays["lr_step"][slr].cpu().numpy(), arr["lr_step"]), ("completion: lr_step", c0)
        for key in ("send_flag", "send_count"):
            assert np.array_equal(dio[key][slr].cpu().numpy(), io[key]), ("completion", key, c0)
        posted = [a + int((io["post"] == v).sum()) for a, v in zip(posted, range(4))]
        moved += int((arr["state"].view(np.uint64).reshape(k, 8)[:, 2] != s0.view(np.uint64).reshape(k, 8)[:, 2]).sum())
        del arr, io
    assert all(v > 0 for v in posted[1:]) and moved > 0, (posted, moved)
    del db, nc, dio, pre, mid
    torch.cuda.empty_cache()


@pytest.mark.parametrize("impl", [0, 0x1])
@pytest.mark.parametrize("shape", ["c2", "c5"])
def test_whole_records_equal_reference(pkg, orc, eng, shape, impl):
    """SURVEY 8f.3 on every group at kbench's records shapes (C2: 2^20 groups,
    16-KiB rings; C5: 2^22 7-replica groups, whose acks in reply[4..5] are the
    proxy's data length): apus_records_store_batch from head over every entry
    type (snapshot capacities that stop some groups on a full snapshot),
    then apus_records_load_batch replays the snapshots -- both kernels (16-lane
    segments, a lane per chain) -- against persist_new_entries' walk with
    stablestorage_save_request / stablestorage_load_records restated on the
    reference's proxy.h (ref_records_store_batch / ref_records_load_batch):
    every snapshot byte, length, count, cursor and replay plan."""
    import torch
    if not os.path.exists(_REF_SO):
        pytest.skip("oracle/_ref not built (no /root/reference where the tree was built)")
    G, R, E, ring = {"c2": (1 << 20, 3, 64, 16384), "c5": (1 << 22, 7, 16, 8192)}[shape]
    stride = pkg.batch.ring_stride_for(ring)
    db = pkg.batch.DeviceBatch(G, R, stride, fields=["state", "self_idx", "remote_end", "lr_step", "fail_count",
                                                     "remote_commit"])
    eng.gen(db, pkg.batch.gen_cfg(seed=2029, n_entries=E, n_history=16, len_min=0, len_max=90, ring_len=ring,
                                  p_full_ack=0.5, straggler=True, cid_mix=True, type_mix=True, self_random=True))
    cap, MP = {"c2": 1600, "c5": 1344}[shape], E + 16
    st64 = db.arrays["state"].view(torch.int64).view(G, 8)
    cur = st64[:, 0].clone()
    dump = torch.zeros(G * cap, dtype=torch.uint8, device="cuda")
    dlen = torch.zeros(G, dtype=torch.int32, device="cuda")
    nrec = torch.zeros(G, dtype=torch.int32, device="cuda")
    eng.stats_reset()
    eng.records_store(db, cur, dump, cap, dlen, nrec, flags=impl)
    lo = eng.records_load(dump, cap, dlen, MP, flags=impl)
    torch.cuda.synchronize()
    corrupt = int(eng.stats()[pkg.abi.STAT_CORRUPT])
    chunk = 1 << 20
    bad = recs = 0
    for c0 in range(0, G, chunk):
        c1 = min(G, c0 + chunk)
        k = c1 - c0
        rg = db.ring[c0 * stride:c1 * stride].cpu().numpy()
        stt = db.arrays["state"][64 * c0:64 * c1].cpu().numpy()
        c_ref = stt.view(np.uint64).reshape(k, 8)[:, 0].copy()
        d_ref, l_ref, n_ref = np.zeros(k * cap, np.uint8), np.zeros(k, np.uint32), np.zeros(k, np.uint32)
        bad += orc.ref_records_store_batch(k, stride, rg, stt, c_ref, d_ref, cap, l_ref, n_ref)
        assert np.array_equal(_np(cur[c0:c1], np.uint64), c_ref), ("cursor", c0)
        assert np.array_equal(_np(dlen[c0:c1], np.uint32), l_ref), ("dump_len", c0)
        assert np.array_equal(_np(nrec[c0:c1], np.uint32), n_ref), ("n_records", c0)
        assert np.array_equal(dump[c0 * cap:c1 * cap].cpu().numpy(), d_ref), ("snapshot bytes", c0)
        rl = orc.ref_records_load_batch(d_ref, cap, l_ref, MP)
        for key in ("n_records", "status", "stop"):
            assert np.array_equal(_np(lo[key][c0:c1], np.uint32), rl[key]), ("load", key, c0)
        assert np.array_equal(_np(lo["counts"][3 * c0:3 * c1], np.uint32), rl["counts"]), ("load counts", c0)
        assert np.array_equal(lo["plan"][16 * MP * c0:16 * MP * c1].cpu().numpy(), rl["plan"]), ("plan", c0)
        recs += int(n_ref.sum())
        del rg, d_ref
    assert bad == corrupt and bad > 0 and recs > G, (bad, corrupt, recs)
    del db, dump, lo
    torch.cuda.empty_cache()


def test_whole_force_log_pruning_equals_reference(pkg, orc, eng):
    """force_log_pruning (dare_server.c:2069-2122) on every group of a 2^21-group
    batch of 5-replica logs 81% full (64 entries of 128 B after 40 history
    entries on 16-KiB rings; some servers disconnected): the commit call with
    the publish, log->commit set to its result, then the FORCE call
    (engine.commit_then_force's order) -- against the transcribed
    force_log_pruning on the reference's own primitives and log_append_entry
    (ref_force_prune_batch) run on the pre-FORCE copy: every ring byte (the
    CONFIG entries a removal appends), state row, apply offset, prev_head and
    output."""
    import torch
    from test_full_size import _conn_of
    if not os.path.exists(_REF_SO):
        pytest.skip("oracle/_ref not built (no /root/reference where the tree was built)")
    abi = pkg.abi
    G, R, L = 1 << 21, 5, 16384
    stride = pkg.batch.ring_stride_for(L)
    fields = ["state", "self_idx", "remote_end", "remote_commit", "lr_step", "fail_count", "apply_offsets",
              "prev_head", "abs_base", "sid"]
    db = pkg.batch.DeviceBatch(G, R, stride, fields=fields)
    eng.gen(db, pkg.batch.gen_cfg(seed=4024, n_entries=64, n_history=40, len_min=64, len_max=64, ring_len=L,
                                  p_full_ack=0.9, straggler=True))
    ar = torch.arange(G, dtype=torch.int64, device="cuda")
    db.add("rc_connected").view(torch.int16).copy_(_conn_of(ar).to(torch.int16))
    flags = (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PUBLISH |
             abi.COMMIT_FORCE_PRUNE | abi.COMMIT_STATS_FRESH)
    out = eng.alloc_commit_out(G, flags)
    out["force"]["req_id"].copy_(ar + 11)
    out["force"]["clt_id"].copy_((ar % 30000 + 1).to(torch.int16))
    eng.update_remote_logs(db, flags & ~abi.COMMIT_FORCE_PRUNE, out=out)
    eng.set_commit(db, out["new_commit"])
    keys = ("state", "apply_offsets", "prev_head")
    pre = {k: db.arrays[k].clone() for k in keys}
    pre["ring"] = db.ring.clone()
    pre_rq, pre_cl = out["force"]["req_id"].clone(), out["force"]["clt_id"].clone()
    eng.stats_reset()
    eng.update_remote_logs(db, abi.COMMIT_FORCE_PRUNE, out=out)
    torch.cuda.synchronize()
    corrupt = int(eng.stats()[abi.STAT_CORRUPT])
    chunk = 1 << 20
    bad = 0
    acts = np.zeros(4, np.int64)
    for c0 in range(0, G, chunk):
        c1 = min(G, c0 + chunk)
        k = c1 - c0
        sl = slice(c0, c1)
        arr = {"ring": pre["ring"][c0 * stride:c1 * stride].cpu().numpy(),
               "state": pre["state"][64 * c0:64 * c1].cpu().numpy(),
               "self_idx": db.arrays["self_idx"][sl].cpu().numpy(),
               "sid": db.arrays["sid"][8 * c0:8 * c1].cpu().numpy().view(np.uint64),
               "apply_offsets": pre["apply_offsets"][8 * R * c0:8 * R * c1].cpu().numpy().view(np.uint64),
               "prev_head": pre["prev_head"][sl].cpu().numpy()}
        rq, cl = _np(pre_rq[sl], np.uint64).copy(), _np(pre_cl[sl], np.uint16).copy()
        ro, b = orc.ref_force_prune_batch(k, R, stride, arr, rq, cl)
        bad += b
        got = db.ring[c0 * stride:c1 * stride].cpu().numpy()
        if not np.array_equal(got, arr["ring"]):
            d = np.flatnonzero(got != arr["ring"])
            raise AssertionError(f"ring bytes differ: {d.size}, first in group {c0 + d[0] // stride}")
        del got
        for key in keys:
            pb = _per_group_bytes(pkg, key, R)
            assert np.array_equal(db.arrays[key][c0 * pb:c1 * pb].cpu().numpy(), arr[key].view(np.uint8)), (key, c0)
        for key, dt in (("new_head", np.uint64), ("append_head", np.uint8), ("min_apply", np.uint64)):
            assert np.array_equal(_np(out[key][sl], dt), ro[key]), (key, c0)
        for key, dt in (("action", np.uint8), ("target", np.uint8), ("cfg_idx", np.uint64)):
            assert np.array_equal(_np(out["force"][key][sl], dt), ro[key]), (key, c0)
        assert np.array_equal(_np(out["force"]["req_id"][sl], np.uint64), rq), ("req_id", c0)
        assert np.array_equal(_np(out["force"]["clt_id"][sl], np.uint16), cl), ("clt_id", c0)
        acts += np.bincount(ro["action"], minlength=4)[:4]
        del arr
    assert bad == corrupt
    assert acts[abi.FORCE_NONE] > 0 and acts[abi.FORCE_PRUNE] > 0 and acts[abi.FORCE_REMOVE] > 0, acts
    del db, out, pre
    torch.cuda.empty_cache()
