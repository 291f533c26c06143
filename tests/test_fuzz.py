"""Randomized parity sweep (round 4): generator configurations drawn at
random -- replica counts 3 ... 11, ring lengths 1 KiB - 16 KiB, 1 - 64 new
entries after 0 - 16 history entries of 0 - 400 B commands, entry-type and
configuration mixes, stragglers, garbage reply bytes, random self indices --
each through the one commit call that carries everything (walk + Adler-32,
median, pruning, the candidates' local (idx, term), vote tally, ranking) on
every walk kernel, against the oracle on every output; and (round 5) through
walk + median + the lazy remote-commit publish + force_log_pruning, every byte
those write in place included.  Seeds are fixed, so
a failure reproduces; a configuration the generator rejects is redrawn.
"""
import numpy as np
import pytest

N_CASES = 64
IMPLS = {"wave": 0x0, "lane": 0x1, "segments": 0x2, "hop": 0x8}


@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def _draw(pkg, orc, k):
    """case k's configuration: the first draw of seed 7000 + k onward that
    the generator accepts"""
    for t in range(64):
        rng = np.random.default_rng(7000 + 97 * k + t)
        R = int(rng.choice([3, 4, 5, 6, 7, 8, 11]))
        ring = int(rng.integers(1024, 16385)) & ~15
        lmin = int(rng.integers(0, 200))
        kw = dict(seed=int(rng.integers(1, 1 << 30)), n_entries=int(rng.integers(1, 65)),
                  n_history=int(rng.integers(0, 17)), len_min=lmin, len_max=lmin + int(rng.integers(0, 200)),
                  ring_len=ring, p_full_ack=float(rng.choice([0.3, 0.7, 0.95, 1.0])),
                  straggler=bool(rng.random() < 0.5), type_mix=bool(rng.random() < 0.5),
                  cid_mix=bool(rng.random() < 0.5), garbage_reply=float(rng.choice([0.0, 0.02])),
                  self_random=bool(rng.random() < 0.5))
        cfg = pkg.batch.gen_cfg(**kw)
        G = 512
        hb = orc.host_batch(G, R, ring)
        try:
            orc.gen(hb, cfg)
        except ValueError:
            continue
        return G, R, ring, cfg, hb, kw
    pytest.skip("no accepted configuration")


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(N_CASES))
def test_fused_commit_random_configs(pkg, orc, eng, k):
    import torch
    abi = pkg.abi
    G, R, ring, cfg, hb, kw = _draw(pkg, orc, k)
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(ring))
    eng.gen(db, cfg)
    assert np.array_equal(db.download("ring"), hb.ring), kw
    flags = (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PRUNE |
             abi.COMMIT_LAST_IT | abi.COMMIT_VOTE | abi.COMMIT_RANK)
    ref = orc.commit(hb, abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN)
    lit = orc.last_idx_term(hb)
    rv = orc.vote(hb)
    hb.arrays["last_idx_term"][:] = lit
    rr = orc.rank(hb)
    rp, wm = orc.prune(hb)
    ap_after = hb.apply_offsets.copy()
    ap_before = db.download("apply_offsets").copy()
    for impl, bf in IMPLS.items():
        db.arrays["apply_offsets"].copy_(torch.from_numpy(ap_before.view(np.uint8).copy()).cuda())
        b = db.struct()
        b.flags = bf
        out = eng.update_remote_logs(db, flags | abi.COMMIT_STATS_FRESH, bstruct=b)
        torch.cuda.synchronize()
        st = eng.stats()
        tag = (impl, kw)
        assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"]), tag
        assert np.array_equal(out["committed"].cpu().numpy(), ref["committed"]), tag
        assert np.array_equal(out["n_entries"].cpu().numpy().view(np.uint32), ref["n_entries"]), tag
        assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"]), tag
        assert np.array_equal(_u64(out["median"]), ref["median"]), tag
        assert np.array_equal(_u64(out["last_idx_term"]).reshape(-1), lit), tag
        for key in ("won", "vote_count"):
            assert np.array_equal(out["vote"][key].cpu().numpy(), rv[key]), (key, tag)
        assert np.array_equal(_u64(out["vote"]["new_commit"]), rv["new_commit"]), tag
        assert np.array_equal(out["rank"]["outcome"].cpu().numpy(), rr["outcome"]), tag
        assert np.array_equal(_u64(out["rank"]["new_sid"]), rr["new_sid"]), tag
        assert np.array_equal(out["rank"]["new_cid"].cpu().numpy(), rr["new_cid"]), tag
        assert np.array_equal(out["rank"]["cleared"].cpu().numpy().view(np.uint16), rr["cleared"]), tag
        assert np.array_equal(_u64(out["new_head"]), rp["new_head"]), tag
        assert np.array_equal(out["append_head"].cpu().numpy(), rp["append_head"]), tag
        assert np.array_equal(_u64(out["min_apply"]), rp["min_apply"]), tag
        assert np.array_equal(db.download("apply_offsets"), ap_after), tag
        assert st[abi.STAT_DECISIONS] == G and st[abi.STAT_MIN_WATERMARK] == wm, tag
        assert st[abi.STAT_COMMITTED] == int(ref["n_entries"].sum()), tag
        assert st[abi.STAT_VOTES_WON] == int(rv["won"].sum()), tag


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(N_CASES))
def test_publish_force_random_configs(pkg, orc, eng, k):
    """the same random configurations through walk + checksum + median +
    update_remote_logs' publish, then force_log_pruning on the walked log (its
    own call) on every walk kernel: every output and every byte written in place (ring, state,
    apply_offsets, remote_commit, prev_head) against the oracle"""
    import torch
    import test_publish_force as tp
    abi = pkg.abi
    G, R, ring, cfg, hb, kw = _draw(pkg, orc, k)
    rng = np.random.default_rng(8000 + k)
    conn = hb.add("rc_connected")
    conn[:] = np.where(rng.random(G) < 0.7, 0xFFFF, rng.integers(0, 1 << 16, size=G)).astype(np.uint16)
    flags = (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PUBLISH |
             abi.COMMIT_FORCE_PRUNE)
    ref = orc.commit(hb, abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN)
    want = tp.clone(hb)
    tf = abi.COMMIT_PUBLISH | abi.COMMIT_FORCE_PRUNE
    ssn0 = np.arange(G, dtype=np.uint64)
    to, twm, bad = orc.tail(want, tf, ref["new_commit"], out=orc.tail_out(G, tf, ssn=ssn0))
    want.state["commit"] = ref["new_commit"]                # the caller's log->commit update between the calls
    for impl, bf in IMPLS.items():
        db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(ring))
        db.add("rc_connected")
        db.upload(hb)
        b = db.struct()
        b.flags = bf
        out = eng.alloc_commit_out(G, flags)
        out["ssn"].copy_(torch.from_numpy(ssn0.view(np.int64)))
        eng.stats_reset()
        out = eng.commit_then_force(db, flags, out=out, bstruct=b)
        torch.cuda.synchronize()
        st = eng.stats()
        tag = (impl, kw)
        assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"]), tag
        assert np.array_equal(_u64(out["median"]), ref["median"]), tag
        assert np.array_equal(out["publish"].cpu().numpy().view(np.uint16), to["publish"]), tag
        assert np.array_equal(_u64(out["ssn"]), to["ssn"]), tag
        for key in ("new_head", "min_apply"):
            assert np.array_equal(_u64(out[key]), to[key]), (key, tag)
        assert np.array_equal(out["append_head"].cpu().numpy(), to["append_head"]), tag
        for key in ("action", "target"):
            assert np.array_equal(out["force"][key].cpu().numpy(), to["force"][key]), (key, tag)
        assert np.array_equal(_u64(out["force"]["cfg_idx"]), to["force"]["cfg_idx"]), tag
        assert np.array_equal(db.download("ring"), want.ring), tag
        for key in ("state", "apply_offsets", "remote_commit", "prev_head"):
            assert db.download(key).tobytes() == want.arrays[key].tobytes(), (key, tag)
        assert st[abi.STAT_MIN_WATERMARK] == twm, tag


def _draw_append(pkg, orc, k):
    """append case k: a generated log (or a fresh log_new() ring) and a queue
    of messages, sizes drawn so that about half the batches wrap"""
    for t in range(64):
        rng = np.random.default_rng(9100 + 131 * k + t)
        R = int(rng.choice([3, 5, 7]))
        M = int(rng.choice([4, 8, 16, 24, 40, 64]))
        lmax = int(rng.integers(1, 260))
        ring = int(rng.integers(max(1024, 64 * M // 2), max(2048, 130 * M + 600)))
        G = 384
        if rng.random() < 0.2:
            hb = orc.host_batch(G, R, ring)
            hb.ring[:] = rng.integers(0, 256, hb.ring.size, dtype=np.uint8)   # bytes the append must keep
            st = hb.state
            st["head"] = st["apply"] = st["commit"] = 0
            st["end"] = st["tail"] = st["len"] = ring
            hb.self_idx[:] = rng.integers(0, R, G, dtype=np.uint8)
            hb.sid[:] = rng.integers(1, 64, G, dtype=np.uint64) << np.uint64(9)
            hb.prev_head[:] = 1
        else:
            lmin = int(rng.integers(0, 120))
            kw = dict(seed=int(rng.integers(1, 1 << 30)), n_entries=int(rng.integers(1, 12)),
                      n_history=int(rng.integers(0, 8)), len_min=lmin, len_max=lmin + int(rng.integers(0, 100)),
                      ring_len=ring, type_mix=bool(rng.random() < 0.4), cid_mix=bool(rng.random() < 0.4),
                      self_random=True)
            hb = orc.host_batch(G, R, ring)
            try:
                orc.gen(hb, pkg.batch.gen_cfg(**kw))
            except ValueError:
                continue
            if rng.random() < 0.2:
                hb.state["tail"][:] = hb.state["len"]               # the tail's index unknown: log_get_tail
        ent, payload = pkg.batch.make_messages(G, M, seed=int(rng.integers(1, 1 << 30)), len_min=0, len_max=lmax,
                                               type_mix=bool(rng.random() < 0.5),
                                               align=int(rng.choice([1, 1, 4, 8])), scatter=bool(rng.random() < 0.3))
        n_entries = rng.integers(0, M + 1, G, dtype=np.uint32)
        n_entries[: G // 2] = M
        return hb, ent, payload, M, n_entries
    pytest.skip("no accepted configuration")


def _clone_host(pkg, hb):
    c = pkg.batch.HostBatch(hb.G, hb.R, hb.stride, fields=list(hb.arrays))
    c.ring[:] = hb.ring
    for key, v in hb.arrays.items():
        c.arrays[key][:] = v
    return c


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(N_CASES))
def test_append_random_batches(pkg, orc, eng, k):
    """log_append_entry over random queues on random rings (wraps, ghost
    headers, full logs, unknown tails, every entry type, unaligned and
    scattered payloads): every ring byte, end / tail, prev_head, returned
    index and the corrupt count equal the oracle's, for the default kernel
    choice (the four-groups-per-wave kernel on short queues) and the
    one-group-per-wave kernel (APPEND_PER_GROUP)"""
    import torch
    abi = pkg.abi
    hb, ent, payload, M, n_entries = _draw_append(pkg, orc, k)
    ref = _clone_host(pkg, hb)
    last0 = np.arange(hb.G, dtype=np.uint64) * 7
    idx, last, bad = orc.append(ref, ent, payload, M, n_entries=n_entries, last_idx=last0.copy())
    for flags in (0, abi.APPEND_PER_GROUP):
        db = pkg.batch.DeviceBatch(hb.G, hb.R, hb.stride)
        db.upload(hb)
        d_last = torch.from_numpy(last0.view(np.int64).copy()).cuda()
        eng.stats_reset()
        out = eng.log_append_entry(db, torch.from_numpy(ent.view(np.uint8).copy()).cuda(),
                                   torch.from_numpy(payload).cuda(), M,
                                   n_entries=torch.from_numpy(n_entries.view(np.int32).copy()).cuda(),
                                   last_idx=d_last, flags=flags)
        torch.cuda.synchronize()
        tag = (k, flags)
        assert np.array_equal(db.download("ring"), ref.ring), tag
        dst = db.download("state")
        for key in ("end", "tail", "head"):
            assert np.array_equal(dst[key], ref.state[key]), (tag, key)
        assert np.array_equal(db.download("prev_head"), ref.prev_head), tag
        assert np.array_equal(out["idx"].cpu().numpy().view(np.uint64), idx), tag
        assert np.array_equal(out["last_idx"].cpu().numpy().view(np.uint64), last), tag
        assert int(eng.stats()[abi.STAT_CORRUPT]) == bad, tag
