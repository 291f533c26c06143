"""Several rounds of the leader's data path on the device, state carried from
round to round, each round bit-exact with the oracle on every ring byte,
state row and output (SURVEY 8(a) + 8f.1-8f.2 in sequence):

  get_tailq_message -> log_append_entry      apus_append_batch      (dare_ibv_ud.c:780-790, dare_log.h:466-558)
  persist_new_entries (each replica copy)    apus_persist_batch     (dare_server.c:1792-1810)
  update_remote_logs: commit walk + Adler-32, the median, log_pruning's minimum, one call
                                             apus_commit_batch      (dare_ibv_rc.c:1650-1758, dare_server.c:2026-2058)
  the new commit offset installed            (dare_ibv_rc.c:1744-1758: the caller's log->commit = min_offset)
  apply_committed_entries                    apus_apply_batch       (dare_server.c:1815-1974)
  poll_config_entries                        apus_config_scan_batch (dare_server.c:2133-2187)

A quarter of the followers lag in every round (straggler limits), the rings
(4,096 B) wrap within the first rounds, and the messages mix every entry type.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def _valid_configs(pkg, ent, payload, R, r):
    """CONFIG messages carry a well-formed dare_cid_t: STABLE over the R
    servers, a new epoch each round (the reference reads cid.size as a server
    count: random bytes there would index past its arrays)"""
    cfg = np.nonzero(ent["type"] == 2)[0]
    cid = np.zeros(1, pkg.batch.CID_DT)
    cid["epoch"] = r + 1
    cid["size0"] = R
    cid["state"] = 0
    cid["bitmask"] = (1 << R) - 1
    b = cid.view(np.uint8)
    for k in cfg:
        o = int(ent["data_off"][k])
        payload[o:o + 16] = b


@pytest.mark.gpu
@pytest.mark.parametrize("R", [3, 5])
def test_rounds_append_persist_commit_apply_scan(pkg, orc, eng, R):
    import torch
    abi = pkg.abi
    G, L, M, ROUNDS = 1024, 4096, 6, 5
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, pkg.batch.gen_cfg(seed=911, n_entries=3, n_history=6, ring_len=L, len_min=16, len_max=120,
                                  p_full_ack=1.0, type_mix=True))
    db = pkg.batch.DeviceBatch(G, R, hb.stride)
    db.upload(hb)
    rng = np.random.default_rng(912)
    old_end = np.repeat(hb.state["commit"], R).astype(np.uint64)
    d_oe = torch.from_numpy(old_end.view(np.int64).copy()).cuda()
    io_o = orc.apply_io(G, 4)
    io_d = orc.apply_io(G, 4)
    cfg_o = orc.config_io(G, hb.state["head"].copy(), np.zeros(G, np.uint64))
    cfg_d = orc.config_io(G, hb.state["head"].copy(), np.zeros(G, np.uint64))
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PRUNE
    wrapped = 0
    committed = 0
    for r in range(ROUNDS):
        # the leader appends this round's messages
        ent, payload = pkg.batch.make_messages(G, M, seed=1000 + r, len_min=8, len_max=150, type_mix=True)
        _valid_configs(pkg, ent, payload, R, r)
        eng.log_append_entry(db, torch.from_numpy(ent.view(np.uint8).copy()).cuda(),
                             torch.from_numpy(payload).cuda(), M)
        orc.append(hb, ent, payload, M)
        # every follower copy acks from its cursor (some stop early)
        limit = np.where(rng.random(G * R) < 0.75, 0xFFFFFFFF, rng.integers(0, M, G * R)).astype(np.uint32)
        eng.persist_new_entries(db, d_oe, torch.from_numpy(limit.view(np.int32).copy()).cuda())
        orc.persist(hb, old_end, limit)
        # the commit call, then the caller installs the new commit offset
        out = eng.update_remote_logs(db, flags)
        ref = orc.commit(hb, flags)
        rp, _ = orc.prune(hb)
        torch.cuda.synchronize()
        assert np.array_equal(db.download("ring"), hb.ring), r
        assert np.array_equal(_u64(d_oe), old_end), r
        for k in ("new_commit", "median"):
            assert np.array_equal(_u64(out[k]), ref[k]), (r, k)
        assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"]), r
        assert np.array_equal(out["n_entries"].cpu().numpy().view(np.uint32), ref["n_entries"]), r
        assert np.array_equal(_u64(out["new_head"]), rp["new_head"]), r
        assert np.array_equal(out["append_head"].cpu().numpy(), rp["append_head"]), r
        committed += int(ref["n_entries"].sum())
        hb.state["commit"] = ref["new_commit"]
        db.arrays["state"].view(torch.int64).view(G, 8)[:, 2] = out["new_commit"].view(torch.int64)
        # the state machine and the configuration catch up
        io_d = eng.apply_committed_entries(db, io_d)
        orc.apply(hb, io_o)
        for k in ("req_id", "clt_id", "last_applied", "last_csm_idx", "n_applied", "departed", "events", "n_cfg"):
            assert np.array_equal(io_d[k], io_o[k]), (r, k)
        cfg_d = eng.poll_config_entries(db, cfg_d)
        orc.config_scan(hb, cfg_o)
        for k in ("cid_offset", "req_id", "clt_id", "departed"):
            assert np.array_equal(cfg_d[k], cfg_o[k]), (r, k)
        assert np.array_equal(db.download("state"), hb.state), r
        wrapped += int((hb.state["end"] < hb.state["commit"]).sum())
    assert committed > G * M and wrapped > 0, (committed, wrapped)
