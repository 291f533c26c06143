"""The commit call's tail with eight lanes per group (quorum_row_kernel,
APUS_BATCH_TAIL_ROWS, for the bench flag sets at R = 3, 5, 7) against the
default one-lane form and the oracle: every output and every byte written in
place (apply_offsets, remote_commit, last_idx_term, the statistics) bit-exact.

The batches are test_publish_force.py's (rings near or past 75% full, publish
branches perturbed in) with configuration sizes, states and bitmasks
scrambled in a tenth of the groups: sizes 0..12 (past 8: the groups the row
kernel hands to the list launch), TRANSIT and EXTENDED states (the median's
second configuration, the extended group size), replicas OFF, the leader index
beyond the replicas, SIDs with the L bit and heartbeats of the possible leader.
"""
import numpy as np
import pytest

from test_publish_force import FULL, clone, perturb

pytestmark = pytest.mark.gpu

IMPL = {"wave": 0, "wave_short": 0x2}


@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _scramble(hb, rng):
    G, R = hb.G, hb.R
    st = hb.state
    sel = np.flatnonzero(rng.random(G) < 0.1)
    cid = st["cid"]
    cid["size0"][sel] = rng.integers(0, 13, size=sel.size)
    cid["size1"][sel] = rng.integers(0, 13, size=sel.size)
    cid["state"][sel] = rng.integers(0, 3, size=sel.size)
    cid["bitmask"][sel] = rng.integers(0, 1 << 12, size=sel.size)
    far = rng.random(G) < 0.03
    hb.self_idx[far] = rng.integers(R, 9, size=int(far.sum()))
    sid = hb.sid
    lbit = rng.random(G) < 0.1
    sid[lbit] |= np.uint64(1 << 8)
    # a heartbeat of the possible leader (sid & 0xFF) with the SID's term
    hbm = hb.hb.reshape(G, R)
    pl = (sid & np.uint64(0xFF)).astype(np.int64)
    adopt = np.flatnonzero((rng.random(G) < 0.1) & (pl < R))
    hbm[adopt, pl[adopt]] = (sid[adopt] | np.uint64(7)) & ~np.uint64(1 << 8)


def _host(pkg, orc, ci, G=4096):
    kw, R = FULL[ci]
    hb = orc.host_batch(G, R, kw["ring_len"])
    orc.gen(hb, pkg.batch.gen_cfg(**kw))
    rng = np.random.default_rng(900 + ci)
    perturb(hb, rng)
    _scramble(hb, rng)
    return hb


def _flags(abi, name):
    f = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PRUNE
    if name in ("c5", "c5p"):
        f |= abi.COMMIT_LAST_IT | abi.COMMIT_VOTE | abi.COMMIT_RANK
    if name in ("c2p", "c5p"):
        f |= abi.COMMIT_PUBLISH
    return f


def _flat(out, pre=""):
    r = {}
    for k, v in out.items():
        if isinstance(v, dict):
            r.update(_flat(v, pre + k + "."))
        elif hasattr(v, "cpu"):
            r[pre + k] = v.cpu().numpy().copy()
    return r


def _run(pkg, eng, hb, flags, impl, lanes):
    import torch
    abi = pkg.abi
    db = pkg.batch.DeviceBatch(hb.G, hb.R, hb.stride)
    db.add("rc_connected")
    db.upload(hb)
    b = db.struct()
    b.flags = IMPL[impl] | (0 if lanes else abi.BATCH_TAIL_ROWS)
    out = eng.alloc_commit_out(hb.G, flags)
    if flags & abi.COMMIT_PUBLISH:
        out["ssn"].copy_(torch.arange(hb.G, dtype=torch.int64) * 3)
    eng.stats_reset()
    eng.update_remote_logs(db, flags, out=out, bstruct=b)
    torch.cuda.synchronize()
    r = _flat(out)
    for k in ("state", "apply_offsets", "remote_commit", "prev_head"):
        r["in_place." + k] = db.download(k)
    r["stats"] = eng.stats()
    return r


@pytest.mark.parametrize("name", ["c2", "c5", "c2p", "c5p"])
@pytest.mark.parametrize("ci", range(len(FULL)))
def test_row_tail_vs_lane_tail(pkg, orc, eng, ci, name):
    abi = pkg.abi
    hb = _host(pkg, orc, ci)
    flags = _flags(abi, name)
    cid = hb.state["cid"]
    for impl in (["wave_short"] if name in ("c5", "c5p") else ["wave", "wave_short"]):
        rows = _run(pkg, eng, hb, flags, impl, lanes=False)
        lanes = _run(pkg, eng, hb, flags, impl, lanes=True)
        assert rows.keys() == lanes.keys()
        for k in rows:
            assert np.array_equal(rows[k], lanes[k]), (impl, k)
        # the oracle on the same batch, on the groups inside the reference's
        # domain: configuration sizes at most R (the reference indexes its
        # servers' columns by i < size, so a size past the replica count reads
        # columns a batch row does not have -- the oracle reads the next
        # group's there, the device none) and no empty configuration in use
        # (the median of size 0 is offsets[(0 - 1) / 2], an element the
        # reference never wrote)
        ok = ((cid["size0"] >= 1) & (cid["size0"] <= hb.R) & (cid["size1"] <= hb.R) &
              ((cid["state"] != 1) | (cid["size1"] >= 1)))
        ref = orc.commit(hb, flags & (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN))
        # (the oracle's in-place legs on a copy whose other groups are clamped
        # into the domain, so none writes into a neighbour's columns)
        dom = clone(hb)
        dc = dom.state["cid"]
        dc["size0"] = np.minimum(dc["size0"], hb.R)
        dc["size1"] = np.minimum(dc["size1"], hb.R)
        assert np.array_equal(rows["new_commit"].view(np.uint64), ref["new_commit"])
        assert np.array_equal(rows["median"].view(np.uint64)[ok], ref["median"][ok])
        if not flags & abi.COMMIT_FORCE_PRUNE:
            rp, _ = orc.prune(clone(dom))
            assert np.array_equal(rows["new_head"].view(np.uint64)[ok], rp["new_head"][ok])
            assert np.array_equal(rows["min_apply"].view(np.uint64)[ok], rp["min_apply"][ok])
        if flags & abi.COMMIT_VOTE:
            rv = orc.vote(clone(dom))
            assert np.array_equal(rows["vote.won"][ok], rv["won"][ok])
            assert np.array_equal(rows["vote.new_commit"].view(np.uint64)[ok], rv["new_commit"][ok])
            assert np.array_equal(rows["vote.voters"].view(np.uint16)[ok], rv["voters"][ok])
            rr = orc.rank(clone(dom), use_lit=True)
            assert np.array_equal(rows["rank.outcome"][ok], rr["outcome"][ok])
            assert np.array_equal(rows["rank.new_sid"].view(np.uint64)[ok], rr["new_sid"][ok])
            assert np.array_equal(rows["rank.cleared"].view(np.uint16)[ok], rr["cleared"][ok])
        if flags & abi.COMMIT_PUBLISH:
            tf = flags & (abi.COMMIT_PUBLISH | abi.COMMIT_FORCE_PRUNE)
            to, _, _ = orc.tail(clone(dom), tf, ref["new_commit"],
                                out=orc.tail_out(hb.G, tf, ssn=np.arange(hb.G) * 3))
            assert np.array_equal(rows["publish"].view(np.uint16)[ok], to["publish"][ok])
            assert np.array_equal(rows["ssn"].view(np.uint64)[ok], to["ssn"][ok])
            if tf & abi.COMMIT_FORCE_PRUNE:
                for k in ("new_head", "min_apply"):
                    assert np.array_equal(rows[k].view(np.uint64)[ok], to[k][ok]), k
                assert np.array_equal(rows["append_head"][ok], to["append_head"][ok])
                for k in ("action", "target"):
                    assert np.array_equal(rows["force." + k][ok], to["force"][k][ok]), k
                assert np.array_equal(rows["force.cfg_idx"].view(np.uint64)[ok], to["force"]["cfg_idx"][ok])
                acts = set(rows["force.action"][ok].tolist())
                if ci < 5:
                    assert {abi.FORCE_NONE, abi.FORCE_PRUNE, abi.FORCE_REMOVE} <= acts, acts
    # coverage of the scramble: groups past 8 in size and TRANSIT ones exist
    assert ((cid["size0"] > 8) | (cid["size1"] > 8)).any()
    assert (cid["state"] == 1).any()
