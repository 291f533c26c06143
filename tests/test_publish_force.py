"""update_remote_logs' lazy remote-commit publish (dare_ibv_rc.c:1760-1822)
and force_log_pruning (dare_server.c:2069-2122): the clean-room oracle
(apus_oracle_tail_batch) against the reference-composed one (oracle/_ref:
both bodies transcribed on the reference's own primitives, drift-checked in
test_transcription.py), CPU only.

The batches are the generator's, then perturbed so every branch is taken:
rings at least 75% full (and some just below), remote commits equal to the
remote end / the leader's commit / anything else, rc_connected bits cleared,
tail == len (log_get_tail scans), prev_log_entry_head set, full logs
(end == head), the leader index beyond the replicas.
"""
import copy

import numpy as np
import pytest

# (generator config, R): small rings with many entries -> log_size near len
FULL = [
    (dict(seed=31, ring_len=16384, n_entries=64, n_history=40), 3),                 # C2 entries, 81% full
    (dict(seed=32, ring_len=6000, n_entries=24, n_history=16, len_min=60, len_max=80, type_mix=True,
          self_random=True, garbage_reply=0.05, p_full_ack=0.5), 5),
    (dict(seed=33, ring_len=2600, n_entries=12, n_history=8, len_min=40, len_max=56, type_mix=True,
          cid_mix=True, self_random=True, straggler=True, p_full_ack=0.3), 5),
    (dict(seed=34, ring_len=1500, n_entries=6, n_history=6, len_min=30, len_max=50, cid_mix=True,
          self_random=True, garbage_reply=0.2), 7),
    (dict(seed=35, ring_len=777, n_entries=4, n_history=3, len_min=20, len_max=30, cid_mix=True,
          self_random=True, p_full_ack=0.0, straggler=True), 3),
    (dict(seed=36, ring_len=4096, n_entries=20, n_history=4, len_min=60, len_max=60), 7),   # 73%: below
]


def clone(hb):
    c = copy.copy(hb)
    c.ring = hb.ring.copy()
    c.arrays = {k: v.copy() for k, v in hb.arrays.items()}
    return c


def perturb(hb, rng):
    """every branch of the publish and of force_log_pruning"""
    G, R = hb.G, hb.R
    st = hb.state
    rc = hb.remote_commit.reshape(G, R)
    rend = hb.remote_end.reshape(G, R)
    pick = rng.integers(0, 4, size=(G, R))
    rnd = rng.integers(0, st["len"][:, None], size=(G, R)).astype(np.uint64)
    rc[:] = np.where(pick == 0, rend, np.where(pick == 1, st["commit"][:, None], np.where(pick == 2, rnd, rc)))
    conn = hb.add("rc_connected")
    conn[:] = np.where(rng.random(G) < 0.8, 0xFFFF, rng.integers(0, 1 << 16, size=G)).astype(np.uint16)
    # tail unknown (log_get_tail scans from commit / apply / head)
    sel = rng.random(G) < 0.3
    st["tail"][sel] = st["len"][sel]
    # a full log: end == head
    full = rng.random(G) < 0.05
    st["head"][full] = st["end"][full]
    # the leader beyond the replica columns
    far = rng.random(G) < 0.03
    hb.self_idx[far] = R + 1
    # apply offsets: the leader's own sometimes the smallest
    ap = hb.apply_offsets.reshape(G, R)
    lead = rng.random(G) < 0.15
    ap[lead] = st["end"][lead][:, None]


def _commit(orc, hb):
    return orc.commit(hb, 1)["new_commit"]


@pytest.mark.parametrize("ci", range(len(FULL)))
def test_publish_force_oracle_vs_ref(orc, ref, pkg, ci):
    abi = pkg.abi
    kw, R = FULL[ci]
    hb = orc.host_batch(384, R, kw["ring_len"])
    orc.gen(hb, pkg.batch.gen_cfg(**kw))
    perturb(hb, np.random.default_rng(100 + ci))
    commit = _commit(orc, hb)
    flags = abi.COMMIT_PUBLISH | abi.COMMIT_FORCE_PRUNE
    a, b = clone(hb), clone(hb)
    rq = np.arange(hb.G, dtype=np.uint64) + 7
    cl = (np.arange(hb.G) % 60000 + 3).astype(np.uint16)
    oa, wa, ba = orc.tail(a, flags, commit, out=orc.tail_out(hb.G, flags, req_id=rq, clt_id=cl))
    ob, wb, bb = orc.ref_tail(b, flags, commit, out=orc.tail_out(hb.G, flags, req_id=rq, clt_id=cl))
    for k in ("new_head", "append_head", "min_apply", "publish", "ssn"):
        assert np.array_equal(oa[k], ob[k]), k
    for k in oa["force"]:
        assert np.array_equal(oa["force"][k], ob["force"][k]), k
    assert wa == wb and ba == bb
    assert np.array_equal(a.ring, b.ring)
    for k in ("state", "apply_offsets", "remote_commit", "prev_head"):
        assert np.array_equal(a.arrays[k], b.arrays[k]), k
    act = oa["force"]["action"]
    # coverage: every outcome, posts, a CONFIG entry that landed
    if ci < 5:
        assert {abi.FORCE_NONE, abi.FORCE_PRUNE, abi.FORCE_REMOVE} <= set(act.tolist()), np.bincount(act)
        assert (oa["force"]["cfg_idx"] > 0).any()
    assert (oa["publish"] != 0).any() and (oa["publish"] == 0).any()
    assert (oa["ssn"] == (oa["publish"] != 0)).all()


def test_publish_semantics_by_hand(orc, pkg):
    """a hand-built group: which servers get the commit write, and the clamp"""
    abi = pkg.abi
    R = 5
    hb = orc.host_batch(1, R, 4096)
    st = hb.state
    st["head"], st["apply"], st["commit"], st["end"], st["tail"], st["len"] = 0, 0, 1000, 2000, 1900, 4096
    st["cid"]["size0"], st["cid"]["state"], st["cid"]["bitmask"] = 5, 0, 0b11101     # server 1 OFF
    hb.self_idx[0] = 0
    hb.lr_step[:] = abi.LR_UPDATE_LOG
    hb.remote_end[:] = [2000, 1500, 1200, 1800, 2000]
    hb.remote_commit[:] = [5, 5, 1200, 1500, 1500]          # 2: commit == end -> skipped
    conn = hb.add("rc_connected")
    conn[0] = 0b01111                                       # 4 not connected
    out, _, _ = orc.tail(hb, abi.COMMIT_PUBLISH, np.array([1600], np.uint64))
    # 0 self, 1 OFF, 2 commit == end, 4 not connected; 3: 1600 (its end 1800 is beyond)
    assert out["publish"][0] == 0b01000
    assert list(hb.remote_commit) == [5, 5, 1200, 1600, 1500]
    # the clamp: the leader's commit past a server's end
    hb.remote_commit[3] = 7
    hb.remote_end[3] = 1400
    out, _, _ = orc.tail(hb, abi.COMMIT_PUBLISH, np.array([1600], np.uint64))
    assert out["publish"][0] == 0b01000 and hb.remote_commit[3] == 1400
    # up to date: nothing posted, ssn unchanged
    out, _, _ = orc.tail(hb, abi.COMMIT_PUBLISH, np.array([1400], np.uint64))
    assert out["publish"][0] == 0 and out["ssn"][0] == 0


def test_force_threshold_exact(orc, pkg):
    """log_size < 0.75 * len, compared as the reference compares it"""
    abi = pkg.abi
    for ln, size, fire in ((4096, 3071, False), (4096, 3072, True), (1000, 749, False), (1000, 750, True),
                           (777, 582, False), (777, 583, True)):
        hb = orc.host_batch(1, 3, ln)
        st = hb.state
        st["head"], st["apply"], st["commit"], st["end"], st["tail"], st["len"] = 0, 0, 0, size, 0, ln
        st["cid"]["size0"], st["cid"]["bitmask"] = 3, 7
        hb.apply_offsets[:] = 0
        out, _, _ = orc.tail(hb, abi.COMMIT_FORCE_PRUNE)
        assert (out["force"]["action"][0] != abi.FORCE_NONE) == fire, (ln, size)


@pytest.mark.parametrize("ci", range(len(FULL)))
def test_reference_force_batch_equals_per_group(orc, ref, pkg, ci):
    """oracle/_ref's ref_force_prune_batch (tests/test_whole_batch.py's
    checker: light log images, the state rows in place) equals ref_tail's
    per-group force_log_pruning"""
    abi = pkg.abi
    kw, R = FULL[ci]
    hb = orc.host_batch(384, R, kw["ring_len"])
    orc.gen(hb, pkg.batch.gen_cfg(**kw))
    perturb(hb, np.random.default_rng(100 + ci))
    commit = _commit(orc, hb)
    a, b = clone(hb), clone(hb)
    rq = np.arange(hb.G, dtype=np.uint64) + 7
    cl = (np.arange(hb.G) % 60000 + 3).astype(np.uint16)
    f = abi.COMMIT_FORCE_PRUNE
    oa, _, ba = orc.ref_tail(a, f, commit, out=orc.tail_out(hb.G, f, req_id=rq, clt_id=cl))
    a.state["commit"] = commit
    b.state["commit"] = commit
    rq2, cl2 = rq.copy(), cl.copy()
    arr = {"ring": b.ring, "state": b.state.view(np.uint8), "self_idx": b.self_idx, "sid": b.sid,
           "apply_offsets": b.apply_offsets, "prev_head": b.prev_head}
    ob, bb = orc.ref_force_prune_batch(b.G, b.R, b.stride, arr, rq2, cl2)
    for k in ("new_head", "append_head", "min_apply"):
        assert np.array_equal(oa[k], ob[k]), k
    for k in ("action", "target", "cfg_idx"):
        assert np.array_equal(oa["force"][k], ob[k]), k
    assert np.array_equal(oa["force"]["req_id"], rq2) and np.array_equal(oa["force"]["clt_id"], cl2)
    assert ba == bb and np.array_equal(a.ring, b.ring)
    for k in ("state", "apply_offsets", "prev_head"):
        assert np.array_equal(a.arrays[k], b.arrays[k]), k
