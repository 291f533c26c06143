"""oracle/_ref's whole-batch checker (ref_check_batch, the reference's own
code over every group of a batch: tests/test_whole_batch.py runs it against
the GPU step on the full BASELINE batches) agrees with the clean-room oracle
on every output, so the GPU comparison has two independent CPU paths behind
it.  Runs in this container (it needs the _ref build) on small batches of the
C2 and C5 shapes."""
import numpy as np
import pytest

from test_full_size import _conn_of


def _ins(hb):
    d = {k: hb.arrays[k] for k in hb.arrays}
    d["ring"] = hb.ring
    return d


@pytest.mark.parametrize("shape", ["c2", "c5", "c3"])
def test_ref_check_equals_oracle(pkg, orc, shape):
    if orc.ref() is None:
        pytest.skip("oracle/_ref not built (no /root/reference)")
    abi = pkg.abi
    votes, var = shape == "c5", shape == "c3"
    G, R, L, E = {"c2": (3000, 3, 16384, 64), "c5": (3000, 7, 8192, 16), "c3": (300, 5, 272960, 64)}[shape]
    cfg = pkg.batch.gen_cfg(seed=77 if votes else 76, n_entries=E, n_history=16, len_min=64,
                            len_max=4096 if var else 64, ring_len=L, p_full_ack=0.9, straggler=True, cid_mix=votes,
                            p_vote_ack=0.6, hist_len_max=64 if var else 0)
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, cfg)
    conn = hb.add("rc_connected")
    conn[:] = _conn_of(np.arange(G, dtype=np.int64)).astype(np.uint16)
    F = R - 1
    nc = orc.gen_nc(hb, cfg, F, E) if var else None
    rc = orc.ref_check(G, R, hb.stride, _ins(hb), votes, threads=4, nc_max=E if var else 0,
                       followers=nc + (F, E) if var else None)
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN
    ref = orc.commit(hb, flags)
    for k in ("new_commit", "committed", "digest", "median"):
        assert np.array_equal(rc[k], ref[k]), k
    if votes:
        rv = orc.vote(hb)
        assert np.array_equal(rc["won"], rv["won"])
        assert np.array_equal(rc["vc"], rv["vote_count"])
        assert np.array_equal(rc["vote_commit"], rv["new_commit"])
        lit = orc.last_idx_term(hb)
        assert np.array_equal(rc["lit"], lit)
        hb.arrays["last_idx_term"][:] = lit
        rr = orc.rank(hb)
        for k in ("outcome", "new_sid", "new_cid", "cleared"):
            assert np.array_equal(rc[k], rr[k]), k
        assert set(np.unique(rc["outcome"])) >= {2, 3, 4}
    rp, _ = orc.prune(hb)                       # OFF servers' apply offsets reset in place
    for k in ("new_head", "append_head", "min_apply"):
        assert np.array_equal(rc[k], rp[k]), k
    assert np.array_equal(rc["apply_out"], hb.apply_offsets)
    to, _, _ = orc.tail(hb, abi.COMMIT_PUBLISH, ref["new_commit"])   # remote_commit written in place
    assert np.array_equal(rc["publish"], to["publish"]) and (rc["publish"] != 0).any()
    assert np.array_equal(rc["ssn"], to["ssn"])
    assert np.array_equal(rc["rcommit_out"], hb.remote_commit)
    if var:
        dets, ln = orc.nc_build(hb, E)
        assert np.array_equal(rc["nc_len"], ln) and ln.max() == E
        live = (np.arange(E)[None, :] < ln[:, None]).repeat(3, axis=1).reshape(-1)
        assert np.array_equal(np.where(live, rc["nc_dets"], 0), np.where(live, dets, 0))
        rv = orc.validate(hb, *nc, F, E)          # on the published remote_commit, as the bench's step
        assert np.array_equal(rc["rend_follow"], rv)
