"""Log append + ack production: log_append_entry
(src/include/dare/dare_log.h:466-558, driven by get_tailq_message,
src/dare/dare_ibv_ud.c:780-790) and persist_new_entries
(src/dare/dare_server.c:1792-1810 with rc_send_entries_reply,
src/dare/dare_ibv_rc.c:1828-1863).

CPU: the clean-room oracle against the reference's own log_append_entry
(oracle/_ref, compiled from /root/reference) and its persist loop restated on
the reference primitives.  GPU: apus_append_batch / apus_persist_batch
through the C ABI against the oracle, bit-exact on every ring byte, offset,
index and flag; and the whole producer -> consumer pipeline (append, acks,
commit walk + checksum) on C2-shaped batches.
"""
import zlib

import numpy as np
import pytest

# name: (initial logs, replicas, groups, messages per group, message mix)
#   gen:   logs built by the trace generator (history + uncommitted batch)
#   fresh: log_new() state (head = apply = commit = 0, end = tail = len)
CASES = {
    "c2": dict(init=("gen", dict(seed=201, n_entries=8, n_history=8, len_min=64, len_max=64, ring_len=16384)),
               R=3, G=128, M=64, msg=dict(len_min=64, len_max=64)),
    "mixed": dict(init=("gen", dict(seed=202, n_entries=6, n_history=4, len_min=0, len_max=90, ring_len=6000,
                                    type_mix=True, cid_mix=True, self_random=True)),
                  R=5, G=256, M=40, msg=dict(len_min=0, len_max=60, type_mix=True)),
    # more bytes than the ring holds: end runs past head without ever
    # equalling it (is_log_full tests equality only), so the append laps the
    # ring and overwrites live entries exactly as the reference would.  The
    # chain the persist cursors sit on is gone: append-only.
    "mixed_lap": dict(init=("gen", dict(seed=205, n_entries=6, n_history=4, len_min=0, len_max=90, ring_len=6000,
                                        type_mix=True, cid_mix=True, self_random=True)),
                      R=5, G=256, M=40, msg=dict(len_min=0, len_max=200, type_mix=True), persist=False),
    # all-SEND chunks that fit without a wrap take the kernel's lane-parallel
    # path: odd lengths (unaligned headers, byte copies) and 4-B aligned records
    "csm_var": dict(init=("gen", dict(seed=206, n_entries=8, n_history=8, len_min=64, len_max=64, ring_len=65536)),
                    R=3, G=96, M=150, msg=dict(len_min=1, len_max=255)),
    "c2_al4": dict(init=("gen", dict(seed=207, n_entries=8, n_history=8, len_min=64, len_max=64, ring_len=32768)),
                   R=3, G=128, M=100, msg=dict(len_min=60, len_max=60, align=4)),
    "c3_var": dict(init=("gen", dict(seed=203, n_entries=4, n_history=4, len_min=64, len_max=4096,
                                     ring_len=600000)),
                   R=5, G=24, M=24, msg=dict(len_min=64, len_max=4096)),
    # small rings from log_new(): the ring fills, wraps (header wrap and ghost
    # headers) and runs full (end == head) -- every branch of log_append_entry
    "fresh_tiny": dict(init=("fresh", 777), R=3, G=256, M=24, msg=dict(len_min=0, len_max=120, type_mix=True)),
    "fresh_small": dict(init=("fresh", 4096), R=7, G=128, M=70, msg=dict(len_min=0, len_max=300, type_mix=True)),
    # SEND-only batches of odd lengths on small generated rings: the fast
    # path's wraps at the ring end (header wrap to 0, ghost header) with the
    # tail's index known; "send_wrap_lap" runs past head several times
    "send_wrap": dict(init=("gen", dict(seed=208, n_entries=4, n_history=4, len_min=0, len_max=120, ring_len=5000)),
                      R=3, G=256, M=20, msg=dict(len_min=0, len_max=200)),
    "send_wrap_lap": dict(init=("gen", dict(seed=209, n_entries=4, n_history=4, len_min=0, len_max=120,
                                            ring_len=5000)),
                          R=3, G=256, M=80, msg=dict(len_min=0, len_max=200), persist=False),
    # batches of <= 16 messages: four groups per wave (append_quad_kernel),
    # the groups whose batch is not one straight run handed to the per-group
    # kernel.  C5-shaped (7 replicas, 16 x 128-B SENDs, most batches fit),
    # odd lengths on small rings (wraps and ghosts: many groups handed back),
    # commands scattered over the arena (one load per command), type mixes and
    # log_new() rings that fill
    "c5_short": dict(init=("gen", dict(seed=210, n_entries=4, n_history=4, len_min=64, len_max=64, ring_len=16384,
                                       cid_mix=True)),
                     R=7, G=512, M=16, msg=dict(len_min=64, len_max=64)),
    "short_wrap": dict(init=("gen", dict(seed=211, n_entries=4, n_history=4, len_min=0, len_max=120, ring_len=5000)),
                       R=3, G=512, M=16, msg=dict(len_min=0, len_max=200)),
    "short_scatter": dict(init=("gen", dict(seed=212, n_entries=4, n_history=4, len_min=0, len_max=200,
                                            ring_len=16384)),
                          R=5, G=384, M=13, msg=dict(len_min=1, len_max=255, scatter=True)),
    "short_mix": dict(init=("gen", dict(seed=213, n_entries=6, n_history=4, len_min=0, len_max=90, ring_len=6000,
                                        type_mix=True, cid_mix=True, self_random=True)),
                      R=5, G=256, M=8, msg=dict(len_min=0, len_max=60, type_mix=True)),
    "short_fresh": dict(init=("fresh", 3000), R=3, G=256, M=16, msg=dict(len_min=0, len_max=120)),
    # tail == len with entries in the log: the index comes from log_get_tail's scan
    "tail_scan": dict(init=("gen_tail_unknown", dict(seed=204, n_entries=5, n_history=5, len_min=0, len_max=80,
                                                     ring_len=3000, type_mix=True)),
                      R=3, G=256, M=12, msg=dict(len_min=0, len_max=50, type_mix=True)),
}


def _clone(pkg, hb):
    c = pkg.batch.HostBatch(hb.G, hb.R, hb.stride, fields=list(hb.arrays))
    c.ring[:] = hb.ring
    for k, v in hb.arrays.items():
        c.arrays[k][:] = v
    return c


def build(pkg, orc, name):
    c = CASES[name]
    kind, arg = c["init"]
    G, R, M = c["G"], c["R"], c["M"]
    if kind.startswith("gen"):
        hb = orc.host_batch(G, R, arg["ring_len"])
        orc.gen(hb, pkg.batch.gen_cfg(**arg))
        if kind == "gen_tail_unknown":
            hb.state["tail"][:] = hb.state["len"]
    else:
        hb = orc.host_batch(G, R, arg)
        rng = np.random.default_rng(7)
        hb.ring[:] = rng.integers(0, 256, hb.ring.size, dtype=np.uint8)   # sender / pad bytes must survive
        st = hb.state
        st["head"] = st["apply"] = st["commit"] = 0
        st["end"] = st["tail"] = st["len"] = arg
        hb.self_idx[:] = rng.integers(0, R, G, dtype=np.uint8)
        hb.sid[:] = rng.integers(1, 64, G, dtype=np.uint64) << np.uint64(9)
        hb.prev_head[:] = 1
    ent, payload = pkg.batch.make_messages(G, M, seed=zlib.crc32(name.encode()) & 0xFFFF, **c["msg"])
    rng = np.random.default_rng(11)
    n_entries = rng.integers(0, M + 1, G, dtype=np.uint32)
    n_entries[: G // 2] = M
    hb.end0 = hb.state["end"].copy()
    return hb, ent, payload, M, n_entries


def persist_inputs(hb, seed, end0):
    """per replica copy: a persist cursor on the log's entry chain (the commit
    offset, the end before the append -- len on a fresh log, whose chain
    starts at 0 -- or the current end) and a straggler limit.  Cursors off
    the chain are outside the contract (apus_gpu.h): the reference's replica
    copies would each see only their own writes."""
    rng = np.random.default_rng(seed)
    G, R = hb.G, hb.R
    st = hb.state
    choice = rng.integers(0, 3, G * R)
    old_end = np.where(choice == 0, np.repeat(end0, R),
                       np.where(choice == 1, np.repeat(st["commit"], R), np.repeat(st["end"], R))).astype(np.uint64)
    limit = np.where(rng.random(G * R) < 0.8, 0xFFFFFFFF, rng.integers(0, 20, G * R)).astype(np.uint32)
    return old_end, limit


def _same_batch(a, b, what):
    assert np.array_equal(a.ring, b.ring), f"{what}: ring bytes differ"
    for k in ("end", "tail"):
        assert np.array_equal(a.state[k], b.state[k]), f"{what}: state.{k} differs"
    assert np.array_equal(a.prev_head, b.prev_head), f"{what}: prev_head differs"


# ------------------------------------------------------------------- CPU
@pytest.mark.parametrize("name", list(CASES))
def test_oracle_append_matches_reference(pkg, orc, ref, name):
    hb, ent, payload, M, n_entries = build(pkg, orc, name)
    h2 = _clone(pkg, hb)
    idx, last, bad = orc.append(hb, ent, payload, M, n_entries=n_entries)
    ridx, rlast, rbad = orc.ref_append(h2, ent, payload, M, n_entries=n_entries)
    _same_batch(hb, h2, name)
    assert np.array_equal(idx, ridx) and np.array_equal(last, rlast) and bad == rbad
    # the cases reach what they are meant to reach
    if name.startswith("fresh"):
        assert (idx.reshape(hb.G, M) == 0).any(), "no full log reached"
    assert (idx > 0).sum() > hb.G


PERSIST_CASES = [k for k, v in CASES.items() if v.get("persist", True)]


@pytest.mark.parametrize("name", PERSIST_CASES)
def test_oracle_persist_matches_reference(pkg, orc, ref, name):
    hb, ent, payload, M, n_entries = build(pkg, orc, name)
    orc.append(hb, ent, payload, M, n_entries=n_entries)
    old_end, limit = persist_inputs(hb, 5, hb.end0)
    h2 = _clone(pkg, hb)
    oe2 = old_end.copy()
    bad = orc.persist(hb, old_end, limit)
    rbad = orc.ref_persist(h2, oe2, limit)
    assert np.array_equal(hb.ring, h2.ring) and np.array_equal(old_end, oe2) and bad == rbad


@pytest.mark.parametrize("name", PERSIST_CASES)
def test_reference_append_persist_batch_equals_per_group(pkg, orc, ref, name):
    """oracle/_ref's batch forms (tests/test_whole_batch.py's checkers: one
    image cleared once, the append on one thread, the persist over OpenMP)
    leave every byte, offset and output as the per-group calls do"""
    hb, ent, payload, M, n_entries = build(pkg, orc, name)
    h2 = _clone(pkg, hb)
    last0 = np.arange(hb.G, dtype=np.uint64) * 3
    idx, last, bad = orc.ref_append(hb, ent, payload, M, n_entries=n_entries, last_idx=last0)
    arr = {"ring": h2.ring, "state": h2.state.view(np.uint8), "prev_head": h2.prev_head, "sid": h2.sid,
           "self_idx": h2.self_idx}
    bidx, blast, bbad = orc.ref_append_batch(h2.G, h2.stride, arr, ent.view(np.uint8), payload, M,
                                             n_entries=n_entries, last_idx=last0)
    _same_batch(hb, h2, name)
    assert np.array_equal(idx, bidx) and np.array_equal(last, blast) and bad == bbad
    old_end, limit = persist_inputs(hb, 5, hb.end0)
    oe2 = old_end.copy()
    pbad = orc.ref_persist(hb, old_end, limit)
    assert orc.ref_persist_batch(h2.G, h2.R, h2.stride, arr, oe2, limit, threads=4) == pbad
    assert np.array_equal(hb.ring, h2.ring) and np.array_equal(old_end, oe2)


def test_oracle_append_stops_on_bad_messages(pkg, orc, ref):
    hb, ent, payload, M, n_entries = build(pkg, orc, "mixed")
    ent = ent.copy()
    ent["data_off"][5] = payload.nbytes + 1                       # data outside the arena
    ent["type"][3 * M + 2] = 5
    ent["data_off"][3 * M + 2] = payload.nbytes - 1                # sm_cmd_t.len cut off
    n_entries[:] = M
    h2 = _clone(pkg, hb)
    idx, last, bad = orc.append(hb, ent, payload, M, n_entries=n_entries)
    ridx, rlast, rbad = orc.ref_append(h2, ent, payload, M, n_entries=n_entries)
    _same_batch(hb, h2, "bad messages")
    assert np.array_equal(idx, ridx) and np.array_equal(last, rlast) and bad == rbad == 2
    assert (idx[5:M] == 0).all() and (idx[3 * M + 2:4 * M] == 0).all()


def test_oracle_pipeline_acks_commit_everything(pkg, orc):
    """append on fresh logs, every replica persists everything, then the
    APUS commit walk commits exactly the appended entries"""
    G, R, L, M = 64, 5, 65536, 48
    hb = orc.host_batch(G, R, L)
    st = hb.state
    st["end"] = st["tail"] = st["len"] = L
    st["cid"]["size0"] = R
    hb.self_idx[:] = np.arange(G) % R
    hb.sid[:] = np.uint64(3 << 9)
    ent, payload = pkg.batch.make_messages(G, M, seed=3, len_min=10, len_max=400)
    idx, _, bad = orc.append(hb, ent, payload, M)
    assert bad == 0 and np.array_equal(idx.reshape(G, M), np.tile(np.arange(1, M + 1, dtype=np.uint64), (G, 1)))
    old_end = np.full(G * R, L, np.uint64)
    assert orc.persist(hb, old_end) == 0
    assert np.array_equal(old_end, np.repeat(st["end"], R))
    out = orc.commit(hb, pkg.abi.COMMIT_WALK)
    assert np.array_equal(out["new_commit"], st["end"]) and (out["n_entries"] == M).all()


# ------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _dev(pkg, hb):
    db = pkg.batch.DeviceBatch(hb.G, hb.R, hb.stride)
    db.upload(hb)
    return db


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_gpu_append_persist_match_oracle(pkg, orc, eng, name):
    import torch
    hb, ent, payload, M, n_entries = build(pkg, orc, name)
    db = _dev(pkg, hb)
    last0 = np.arange(hb.G, dtype=np.uint64) * 3
    d_ent = torch.from_numpy(ent.view(np.uint8).copy()).cuda()
    d_pay = torch.from_numpy(payload).cuda()
    d_n = torch.from_numpy(n_entries.view(np.int32).copy()).cuda()
    d_last = torch.from_numpy(last0.view(np.int64).copy()).cuda()
    eng.stats_reset()
    out = eng.log_append_entry(db, d_ent, d_pay, M, n_entries=d_n, last_idx=d_last)
    idx, last, bad = orc.append(hb, ent, payload, M, n_entries=n_entries, last_idx=last0)
    torch.cuda.synchronize()
    assert np.array_equal(db.download("ring"), hb.ring), "ring bytes differ after append"
    dst = db.download("state")
    for k in ("end", "tail", "head", "commit"):
        assert np.array_equal(dst[k], hb.state[k]), k
    assert np.array_equal(db.download("prev_head"), hb.prev_head)
    assert np.array_equal(out["idx"].cpu().numpy().view(np.uint64), idx)
    assert np.array_equal(out["last_idx"].cpu().numpy().view(np.uint64), last)
    assert int(eng.stats()[pkg.abi.STAT_CORRUPT]) == bad
    if not CASES[name].get("persist", True):
        return

    old_end, limit = persist_inputs(hb, 9, hb.end0)
    d_oe = torch.from_numpy(old_end.view(np.int64).copy()).cuda()
    d_lim = torch.from_numpy(limit.view(np.int32).copy()).cuda()
    eng.stats_reset()
    eng.persist_new_entries(db, d_oe, d_lim)
    pbad = orc.persist(hb, old_end, limit)
    torch.cuda.synchronize()
    assert np.array_equal(db.download("ring"), hb.ring), "ring bytes differ after persist"
    assert np.array_equal(d_oe.cpu().numpy().view(np.uint64), old_end)
    assert int(eng.stats()[pkg.abi.STAT_CORRUPT]) == pbad


SHORT_CASES = [k for k, v in CASES.items() if v["M"] <= 16]


@pytest.mark.gpu
@pytest.mark.parametrize("name", SHORT_CASES)
def test_gpu_append_short_batches_both_kernels(pkg, orc, eng, name):
    """max_entries <= 16: the four-groups-per-wave kernel (and the groups it
    hands back) and the one-group-per-wave kernel (APPEND_PER_GROUP) both
    bit-exact with the oracle"""
    import torch
    hb, ent, payload, M, n_entries = build(pkg, orc, name)
    last0 = np.arange(hb.G, dtype=np.uint64) * 5
    idx, last, bad = orc.append(_clone(pkg, hb), ent, payload, M, n_entries=n_entries, last_idx=last0.copy())
    ref = _clone(pkg, hb)
    orc.append(ref, ent, payload, M, n_entries=n_entries, last_idx=last0.copy())
    for flags in (0, pkg.abi.APPEND_PER_GROUP):
        db = _dev(pkg, hb)
        d_last = torch.from_numpy(last0.view(np.int64).copy()).cuda()
        eng.stats_reset()
        out = eng.log_append_entry(db, torch.from_numpy(ent.view(np.uint8).copy()).cuda(),
                                   torch.from_numpy(payload).cuda(), M,
                                   n_entries=torch.from_numpy(n_entries.view(np.int32).copy()).cuda(),
                                   last_idx=d_last, flags=flags)
        torch.cuda.synchronize()
        what = f"{name} flags={flags}"
        assert np.array_equal(db.download("ring"), ref.ring), what
        dst = db.download("state")
        for k in ("end", "tail"):
            assert np.array_equal(dst[k], ref.state[k]), (what, k)
        assert np.array_equal(db.download("prev_head"), ref.prev_head), what
        assert np.array_equal(out["idx"].cpu().numpy().view(np.uint64), idx), what
        assert np.array_equal(out["last_idx"].cpu().numpy().view(np.uint64), last), what
        st = eng.stats()
        assert int(st[pkg.abi.STAT_CORRUPT]) == bad, what
        handed = int(st[pkg.abi.STAT_APPEND_SLOW])
        if flags:
            assert handed == 0, what
        else:
            appending = int((n_entries > 0).sum())
            if name.endswith("fresh") or name == "tail_scan":   # tail == len: every index from log_get_tail
                assert handed == appending, (what, handed, appending)
            else:                           # both paths taken
                assert 0 < handed < appending, (what, handed, appending)
            if name == "c5_short":
                assert handed < appending // 4, (what, handed, appending)


@pytest.mark.gpu
def test_gpu_append_stops_on_bad_messages(pkg, orc, eng):
    import torch
    hb, ent, payload, M, n_entries = build(pkg, orc, "mixed")
    ent = ent.copy()
    ent["data_off"][5] = payload.nbytes + 1
    n_entries[:] = M
    db = _dev(pkg, hb)
    eng.stats_reset()
    out = eng.log_append_entry(db, torch.from_numpy(ent.view(np.uint8).copy()).cuda(),
                               torch.from_numpy(payload).cuda(), M,
                               n_entries=torch.from_numpy(n_entries.view(np.int32).copy()).cuda())
    idx, last, bad = orc.append(hb, ent, payload, M, n_entries=n_entries)
    torch.cuda.synchronize()
    assert bad == 1 and int(eng.stats()[pkg.abi.STAT_CORRUPT]) == 1
    assert np.array_equal(out["idx"].cpu().numpy().view(np.uint64), idx)
    assert np.array_equal(db.download("ring"), hb.ring)


@pytest.mark.gpu
def test_gpu_pipeline_c2(pkg, orc, eng):
    """C2-shaped producer -> consumer on the device: generated logs, 64 new
    128-B SEND entries appended per group, followers persist with straggler
    limits, then the commit walk + checksum -- all bit-exact with the oracle"""
    import torch
    G, R, L, M = 2048, 3, 16384, 64
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, pkg.batch.gen_cfg(seed=301, n_entries=4, n_history=8, ring_len=L, p_full_ack=1.0))
    db = _dev(pkg, hb)
    ent, payload = pkg.batch.make_messages(G, M, seed=302, len_min=64, len_max=64)
    eng.log_append_entry(db, torch.from_numpy(ent.view(np.uint8).copy()).cuda(), torch.from_numpy(payload).cuda(), M)
    orc.append(hb, ent, payload, M)
    rng = np.random.default_rng(303)
    old_end = np.repeat(hb.state["commit"], R).astype(np.uint64)
    limit = np.where(rng.random(G * R) < 0.7, 0xFFFFFFFF, rng.integers(0, M, G * R)).astype(np.uint32)
    d_oe = torch.from_numpy(old_end.view(np.int64).copy()).cuda()
    eng.persist_new_entries(db, d_oe, torch.from_numpy(limit.view(np.int32).copy()).cuda())
    orc.persist(hb, old_end, limit)
    flags = pkg.abi.COMMIT_WALK | pkg.abi.COMMIT_CHECKSUM
    out = eng.update_remote_logs(db, flags)
    ref = orc.commit(hb, flags)
    torch.cuda.synchronize()
    assert np.array_equal(db.download("ring"), hb.ring)
    assert np.array_equal(out["new_commit"].cpu().numpy().view(np.uint64), ref["new_commit"])
    assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"])
    assert np.array_equal(out["n_entries"].cpu().numpy().view(np.uint32), ref["n_entries"])
    assert ref["n_entries"].sum() > G * M // 2
