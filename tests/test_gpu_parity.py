"""Parity of the HIP kernels (through the libapus_gpu C ABI) with the CPU oracle.

Bit-exact for every output: this path is integer / byte arithmetic only.
Sizes: the oracle finishes each case in seconds; the full-size C2 batch
(2^20 groups) is checked on a sampled group range plus size-independent
properties (stats == sums of the per-group outputs).
"""
import ctypes as C

import numpy as np
import pytest
from conftest import ScalarLog

pytestmark = pytest.mark.gpu

CFGS = {
    "c2": dict(seed=101, n_entries=64, n_history=16, len_min=64, len_max=64, ring_len=16384),
    "c2_skew": dict(seed=102, n_entries=64, n_history=16, len_min=64, len_max=64, ring_len=16384,
                    straggler=True, p_full_ack=0.5, garbage_reply=0.02, self_random=True),
    # (history entries of 64 B - 1 KB: hist_len_max, rings sized for the batch as bench.py's C3)
    "c3_var": dict(seed=103, n_entries=64, n_history=8, len_min=64, len_max=4096, ring_len=600000,
                   straggler=True, p_full_ack=0.8, hist_len_max=1024),
    "mixed_small": dict(seed=104, n_entries=24, n_history=8, len_min=0, len_max=90, ring_len=6000,
                        type_mix=True, cid_mix=True, self_random=True, garbage_reply=0.05,
                        p_full_ack=0.5),
    "tiny_wrap": dict(seed=105, n_entries=5, n_history=1, len_min=3, len_max=45, ring_len=777,
                      cid_mix=True, self_random=True, p_full_ack=0.0, straggler=True),
    "history_only": dict(seed=106, n_entries=0, n_history=12, len_min=10, len_max=300, ring_len=8192,
                         type_mix=True),
    # 16-B aligned small rings: most groups wrap inside one window
    "wrap_aligned": dict(seed=107, n_entries=12, n_history=3, len_min=0, len_max=100, ring_len=4096,
                         type_mix=True, cid_mix=True, self_random=True, p_full_ack=0.6, straggler=True,
                         garbage_reply=0.03),
    # spans of several windows with the wrap (and its ghost header) anywhere in them
    "multiwin": dict(seed=108, n_entries=40, n_history=4, len_min=200, len_max=1000, ring_len=65536,
                     p_full_ack=0.7, straggler=True),
    # C5's shape (BASELINE configs[4]): 7 replicas, 16-entry batches, STABLE / EXTENDED / TRANSIT mix
    "c5": dict(seed=109, n_entries=16, n_history=16, len_min=64, len_max=64, ring_len=16384,
               cid_mix=True, p_full_ack=0.9, straggler=True),
    # short walks of mixed types and lengths, many wrapping inside one 2,304-B segment window
    "short_mixed": dict(seed=110, n_entries=16, n_history=4, len_min=0, len_max=60, ring_len=3000,
                        type_mix=True, cid_mix=True, self_random=True, garbage_reply=0.03, p_full_ack=0.6,
                        straggler=True),
}
RS = {"c2": 3, "c2_skew": 5, "c3_var": 5, "mixed_small": 7, "tiny_wrap": 5, "history_only": 3,
      "wrap_aligned": 5, "multiwin": 3, "c5": 7, "short_mixed": 5}
GS = {"c2": 4096, "c2_skew": 4096, "c3_var": 512, "mixed_small": 4096, "tiny_wrap": 4096, "history_only": 1024,
      "wrap_aligned": 4096, "multiwin": 1024, "c5": 8192, "short_mixed": 8192}
# configurations whose every walk fits commit_seg_kernel's 2,304-B window
# (APUS_BATCH_SHORT_WALKS); longer walks are deferred to the exact lane walk
SHORT_FIT = {"c5", "short_mixed", "tiny_wrap", "wrap_aligned", "history_only"}


@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _pair(pkg, orc, eng, name):
    kw = CFGS[name]
    G, R, L = GS[name], RS[name], kw["ring_len"]
    cfg = pkg.batch.gen_cfg(**kw)
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, cfg)
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, cfg)
    return db, hb, cfg


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("name", list(CFGS))
def test_device_generator_matches_oracle(pkg, orc, eng, name):
    db, hb, _ = _pair(pkg, orc, eng, name)
    assert np.array_equal(db.download("ring"), hb.ring)
    for f in pkg.batch.ALL_FIELDS:
        assert db.download(f).tobytes() == hb.arrays[f].tobytes(), f


IMPL_FLAGS = {"wave": 0, "lane": 0x1, "wave_short": 0x2, "wave_hop": 0x8}   # BATCH_LANE_IMPL / SHORT_WALKS / VAR_LEN


@pytest.mark.parametrize("prune", [False, True])
@pytest.mark.parametrize("impl", list(IMPL_FLAGS))
@pytest.mark.parametrize("name", list(CFGS))
def test_commit_walk_checksum_median(pkg, orc, eng, name, impl, prune):
    """the walk + checksum + median, and with prune the pruning minimum and the
    NC determinants in the same call (APUS_COMMIT_PRUNE | APUS_COMMIT_NC: the
    median and the pruning run in the call's one tail launch, the
    determinants come from the walk; rows of 40 cut C2's 64-entry chains)"""
    import torch
    abi = pkg.abi
    db, hb, _ = _pair(pkg, orc, eng, name)
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN
    if prune:
        flags |= abi.COMMIT_PRUNE | abi.COMMIT_NC
    M = 40
    b = db.struct()
    b.flags = IMPL_FLAGS[impl]
    eng.stats_reset()
    out = eng.update_remote_logs(db, flags, bstruct=b, nc_max=M)
    torch.cuda.synchronize()
    ref = orc.commit(hb, flags)
    assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"])
    assert np.array_equal(out["committed"].cpu().numpy(), ref["committed"])
    assert np.array_equal(out["n_entries"].cpu().numpy().view(np.uint32), ref["n_entries"])
    assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"])
    assert np.array_equal(_u64(out["median"]), ref["median"])
    st = eng.stats()
    assert st[abi.STAT_DECISIONS] == hb.G
    assert st[abi.STAT_COMMITTED] == int(ref["n_entries"].sum())
    assert st[abi.STAT_ADVANCED] == int((ref["committed"] == 1).sum())
    assert st[abi.STAT_CORRUPT] == 0
    # well-formed rings never leave the wave kernel's fast path (nor the
    # segment kernel's, when their walks fit its window)
    if impl in ("wave", "wave_hop") or (impl == "wave_short" and name in SHORT_FIT):
        assert st[abi.STAT_SLOW] == 0
    if prune:
        rd, rl = orc.nc_build(hb, M)
        ln = out["nc_len"].cpu().numpy().view(np.uint32)
        assert np.array_equal(ln, rl)
        got = out["nc_dets"].cpu().numpy().view(np.uint64).reshape(hb.G, 3 * M)
        want = rd.reshape(hb.G, 3 * M)
        live = np.arange(3 * M)[None, :] < 3 * rl.astype(np.int64)[:, None]
        assert np.array_equal(np.where(live, got, 0), np.where(live, want, 0))
        rp, wm = orc.prune(hb)                 # resets OFF servers' apply offsets in hb, as on the device
        assert np.array_equal(_u64(out["new_head"]), rp["new_head"])
        assert np.array_equal(out["append_head"].cpu().numpy(), rp["append_head"])
        assert np.array_equal(_u64(out["min_apply"]), rp["min_apply"])
        assert np.array_equal(db.download("apply_offsets"), hb.apply_offsets)
        assert st[abi.STAT_MIN_WATERMARK] == wm


@pytest.mark.parametrize("ck", [True, False])
@pytest.mark.parametrize("impl", list(IMPL_FLAGS))
@pytest.mark.parametrize("name", list(CFGS))
def test_commit_last_idx_term(pkg, orc, eng, name, impl, ck):
    """APUS_COMMIT_LAST_IT: the candidate's local (idx, term) (poll_vote_requests,
    dare_server.c:1598-1620) from the commit call -- the segment kernel's
    checksum walk records where the last NC determinant lies (ghost headers
    included) and the tail reads it; every other walk leaves it to the tail's
    determinant walk -- equal to the oracle and to apus_last_idx_term_batch"""
    import torch
    abi = pkg.abi
    db, hb, _ = _pair(pkg, orc, eng, name)
    flags = abi.COMMIT_WALK | abi.COMMIT_LAST_IT | (abi.COMMIT_CHECKSUM if ck else 0)
    b = db.struct()
    b.flags = IMPL_FLAGS[impl]
    out = eng.update_remote_logs(db, flags | abi.COMMIT_MEDIAN, bstruct=b)
    lit = eng.last_idx_term(db)
    torch.cuda.synchronize()
    want = orc.last_idx_term(hb)
    assert np.array_equal(_u64(out["last_idx_term"]).reshape(-1), want)
    assert np.array_equal(_u64(lit).reshape(-1), want)
    ref = orc.commit(hb, flags | abi.COMMIT_MEDIAN)
    assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"])
    assert np.array_equal(_u64(out["median"]), ref["median"])
    if ck:
        assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"])


@pytest.mark.parametrize("name", ["c5", "short_mixed", "tiny_wrap", "mixed_small"])
def test_commit_last_idx_term_wide_values(pkg, orc, eng, name):
    """The segment walk's (idx, term) record holds an index below 2^32 and a
    term below 2^16 and leaves every other value to the tail's exact walk:
    determinant headers rewritten (the same bytes on host and device) to an
    index past 32 bits, terms at and past 0xFFFF, the largest values that fit,
    and a term past 40 bits -- ghost headers included -- still give the
    oracle's (idx, term), on the fused failover call as well"""
    import torch
    abi = pkg.abi
    db, hb, _ = _pair(pkg, orc, eng, name)
    M = 4096
    dets, ln = orc.nc_build(hb, M)
    d3 = dets.reshape(hb.G, M, 3)
    for g in range(hb.G):
        n = int(ln[g])
        if n == 0 or g % 6 == 0:
            continue
        ring = hb.group_ring(g)
        for k in range(n):
            idx, term, off = (int(x) for x in d3[g, k])
            cls = g % 6
            if cls == 1:
                idx += 1 << 32
            elif cls == 2:
                term = 0xFFFF + (g % 3)
            elif cls == 3:
                idx, term = 0xFFFFFFFF, 0xFFFE
            elif cls == 4:
                term += 1 << 40
            else:
                idx, term = 0xFFFFFFFF, 0xFFFF
            ring[off:off + 8] = np.frombuffer(np.uint64(idx).tobytes(), np.uint8)
            ring[off + 8:off + 16] = np.frombuffer(np.uint64(term).tobytes(), np.uint8)
    db.upload(hb)
    b = db.struct()
    b.flags = IMPL_FLAGS["wave_short"]
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_LAST_IT | abi.COMMIT_MEDIAN
    out = eng.update_remote_logs(db, flags, bstruct=b)
    torch.cuda.synchronize()
    want = orc.last_idx_term(hb)
    got = _u64(out["last_idx_term"]).reshape(-1)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]
    ref = orc.commit(hb, flags)
    assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"])
    # wide values reached the record path's every class
    w2 = want.reshape(-1, 2)
    assert (w2[:, 0] >= (1 << 32)).any() and (w2[:, 1] >= 0xFFFF).any() and (w2[:, 0] == 0xFFFFFFFF).any()
    # the ranking on those values, in the same call
    fl2 = flags | abi.COMMIT_VOTE | abi.COMMIT_RANK
    out2 = eng.update_remote_logs(db, fl2, bstruct=b)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(out2["last_idx_term"]).reshape(-1), want)
    _check_vote_rank(orc, hb, out2["vote"], out2["rank"], lit_given=want)


def test_commit_walk_info(pkg, eng):
    """apus_commit_walk_info names the walk kernel a call launches (the bench's
    rocprof labels): the batch hints choose lane / wave / segment kernels, the
    hop walk and the NC epilogue follow the flags, the segment kernel records
    the (idx, term) rows only on checksum walks with LAST_IT, and blocks are
    handed out by the counter only on checksum walks of >= 8 blocks per wave"""
    abi = pkg.abi
    db = pkg.batch.DeviceBatch(1024, 3, pkg.batch.ring_stride_for(4096))
    W, CK, NC, LIT = abi.COMMIT_WALK, abi.COMMIT_CHECKSUM, abi.COMMIT_NC, abi.COMMIT_LAST_IT

    def info(impl, flags, G=None):
        b = db.struct()
        b.flags = IMPL_FLAGS[impl]
        if G is not None:
            b.n_groups = G          # sizing only: nothing is launched
        return eng.commit_walk_info(b, flags)

    assert info("lane", W | CK)["kind"] == "lane"
    w = info("wave", W | CK)
    assert (w["kind"], w["hop"], w["nc"], w["dyn"]) == ("wave", False, False, False)
    assert info("wave", W | CK | NC)["nc"] and not info("wave", W | NC)["nc"]
    h = info("wave_hop", W | CK | NC)
    assert (h["kind"], h["hop"], h["nc"]) == ("wave", True, True)
    sg = info("wave_short", W | CK | LIT)
    assert (sg["kind"], sg["rows"], sg["nc"]) == ("segment", True, False)
    assert not info("wave_short", W | LIT)["rows"] and not info("wave_short", W | CK)["rows"]
    big = 1 << 23
    assert info("wave", W | CK, big)["dyn"] and not info("wave", W, big)["dyn"]
    assert info("wave_short", W | CK, big)["dyn"] and not info("wave_short", W | CK)["dyn"]
    b = db.struct()
    b.flags = IMPL_FLAGS["wave_short"]
    b.n_groups = big
    assert eng.walk_kernel_name(b, W | CK | LIT) == "commit_seg_kernel<true, true, true>"
    b.flags = IMPL_FLAGS["wave_hop"]
    b.n_groups = 1024
    assert eng.walk_kernel_name(b, W | CK | NC) == "commit_wave_kernel<true, 12288, true, 4u, false>"


@pytest.mark.parametrize("impl", ["wave", "lane", "wave_short"])
def test_commit_stats_fresh_and_walk_events(pkg, orc, eng, impl):
    """APUS_COMMIT_STATS_FRESH replaces the accumulated statistics (the tail's
    last arriving block writes them; 65,536 groups = 256 tail blocks), and
    apus_commit_mark_walk's events bracket the walk kernel of the next call"""
    import torch
    abi = pkg.abi
    kw = dict(CFGS["c2_skew"])
    G, R, L = 65536, RS["c2_skew"], kw["ring_len"]
    cfg = pkg.batch.gen_cfg(**kw)
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, cfg)
    b = db.struct()
    b.flags = IMPL_FLAGS[impl]
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PRUNE
    eng.stats_reset()
    out = eng.update_remote_logs(db, flags, bstruct=b)
    torch.cuda.synchronize()
    one = eng.stats().copy()
    assert one[abi.STAT_DECISIONS] == G
    # accumulate, then replace
    eng.update_remote_logs(db, flags, bstruct=b)
    torch.cuda.synchronize()
    two = eng.stats()
    assert two[abi.STAT_DECISIONS] == 2 * G and two[abi.STAT_COMMITTED] == 2 * one[abi.STAT_COMMITTED]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in ev:
        e.record()
    torch.cuda.synchronize()
    assert eng.lib.apus_commit_mark_walk(eng.ctx, C.c_void_p(ev[0].cuda_event), C.c_void_p(ev[1].cuda_event)) == 0
    out2 = eng.update_remote_logs(db, flags | abi.COMMIT_STATS_FRESH, bstruct=b)
    torch.cuda.synchronize()
    three = eng.stats()
    assert np.array_equal(three, one), (three, one)
    assert ev[0].query() and ev[1].query() and ev[0].elapsed_time(ev[1]) > 0
    for k in ("new_commit", "committed", "n_entries", "digest", "median", "new_head", "append_head"):
        assert torch.equal(out[k], out2[k]), k
    # a pending pair is consumed by one call: the next call records nothing
    t = ev[0].elapsed_time(ev[1])
    eng.update_remote_logs(db, flags, bstruct=b)
    torch.cuda.synchronize()
    assert ev[0].elapsed_time(ev[1]) == t
    # without the pruning the fresh watermark is the reset value
    eng.update_remote_logs(db, abi.COMMIT_WALK | abi.COMMIT_STATS_FRESH, bstruct=b)
    torch.cuda.synchronize()
    four = eng.stats()
    assert four[abi.STAT_MIN_WATERMARK] == np.uint64(2 ** 64 - 1) and four[abi.STAT_DECISIONS] == G
    # a half pair is refused
    assert eng.lib.apus_commit_mark_walk(eng.ctx, C.c_void_p(ev[0].cuda_event), None) != 0


@pytest.mark.parametrize("name", ["c2_skew", "c5", "mixed_small"])
@pytest.mark.parametrize("shift", [0, 8])
def test_tail_remainder_and_unaligned(pkg, orc, eng, name, shift):
    """the tail launch's median and pruning: G % 64 != 0 (whole 64-group
    blocks staged through LDS, the remainder one lane per group), and with
    shift=8 replica columns that are not 16-B aligned (every group one lane
    per group, inputs loaded directly)"""
    import torch
    abi = pkg.abi
    kw = CFGS[name]
    G, R, L = 3000 + 37, RS[name], kw["ring_len"]
    cfg = pkg.batch.gen_cfg(**kw)
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, cfg)
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, cfg)
    b = db.struct()
    keep = []
    if shift:
        for f in ("remote_end", "apply_offsets"):
            t = db.arrays[f]
            u = torch.zeros(t.numel() + 16, dtype=torch.uint8, device=t.device)
            u[shift:shift + t.numel()] = t
            keep.append((f, u))
            setattr(b, f, u.data_ptr() + shift)
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PRUNE | abi.COMMIT_STATS_FRESH
    out = eng.update_remote_logs(db, flags, bstruct=b)
    torch.cuda.synchronize()
    ref = orc.commit(hb, abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN)
    assert np.array_equal(_u64(out["median"]), ref["median"])
    assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"])
    rp, wm = orc.prune(hb)
    assert np.array_equal(_u64(out["new_head"]), rp["new_head"])
    assert np.array_equal(out["append_head"].cpu().numpy(), rp["append_head"])
    assert np.array_equal(_u64(out["min_apply"]), rp["min_apply"])
    ap = keep[1][1][shift:shift + G * R * 8] if shift else db.arrays["apply_offsets"]
    assert np.array_equal(ap.cpu().numpy().view(np.uint64), hb.apply_offsets.reshape(-1))
    st = eng.stats()
    assert st[abi.STAT_DECISIONS] == G and st[abi.STAT_MIN_WATERMARK] == wm


def _malformed(pkg, orc, G, seed, all_groups):
    """tiny_wrap batches with corrupted headers / ends: chains that overshoot
    end, ghost headers in the wrong place, garbage types and lengths"""
    kw = dict(CFGS["tiny_wrap"], seed=seed)
    R, L = RS["tiny_wrap"], kw["ring_len"]
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, pkg.batch.gen_cfg(**kw))
    rng = np.random.default_rng(seed)
    st = hb.state
    for g in range(G):
        if not all_groups and rng.random() < 0.5:
            continue
        ring = hb.group_ring(g)
        c, e = int(st["commit"][g]), int(st["end"][g])
        kind = rng.integers(0, 4) if not all_groups else 0
        if kind == 0:                       # end moved inside an entry: the chain overshoots it
            st["end"][g] = (e + 1 + rng.integers(0, 40)) % L
            if st["end"][g] == c:
                st["end"][g] = (c + 3) % L
        elif kind == 1:                     # garbage type / cmd.len at the commit offset
            o = c if L - c >= 64 else 0
            ring[o + 26] = rng.integers(0, 256)
            ring[o + 48:o + 50] = rng.integers(0, 256, 2)
        elif kind == 2:                     # random commit
            st["commit"][g] = rng.integers(0, L)
        else:                               # garbage everywhere
            ring[:L] = rng.integers(0, 256, L)
    return hb


@pytest.mark.parametrize("G,all_groups", [(4096, False), (160000, True)])
def test_commit_malformed_rings(pkg, orc, eng, G, all_groups):
    """the wave kernel's exact slow path (per-wave list and its overflow)
    against the oracle and the lane kernel, with and without the checksum"""
    import torch
    abi = pkg.abi
    hb = _malformed(pkg, orc, G, 9 + G, all_groups)
    for flags in (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM, abi.COMMIT_WALK):
        ref = orc.commit(hb, flags)
        for impl in IMPL_FLAGS:
            db = pkg.batch.DeviceBatch(G, hb.R, hb.stride)
            db.upload(hb)
            b = db.struct()
            b.flags = IMPL_FLAGS[impl]
            eng.stats_reset()
            out = eng.update_remote_logs(db, flags, bstruct=b)
            torch.cuda.synchronize()
            assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"]), impl
            assert np.array_equal(out["committed"].cpu().numpy(), ref["committed"]), impl
            assert np.array_equal(out["n_entries"].cpu().numpy().view(np.uint32), ref["n_entries"]), impl
            if flags & abi.COMMIT_CHECKSUM:
                assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"]), impl
                # the walk's NC determinants against the lane NC walk on the same
                # corrupted rings (the oracle reads past a ring where both stop)
                M = 24
                bl = db.struct()
                bl.flags = abi.BATCH_LANE_IMPL
                dl, ll = eng.log_entries_to_nc_buf(db, M, bstruct=bl)
                eng.stats_reset()
                out = eng.update_remote_logs(db, flags | abi.COMMIT_NC, bstruct=b, nc_max=M)
                torch.cuda.synchronize()
                lw, lr = out["nc_len"].cpu().numpy(), ll.cpu().numpy()
                assert np.array_equal(lw, lr), impl
                gw = out["nc_dets"].cpu().numpy().view(np.uint64).reshape(G, 3 * M)
                gr = dl.cpu().numpy().view(np.uint64).reshape(G, 3 * M)
                live = np.arange(3 * M)[None, :] < 3 * lr.astype(np.int64)[:, None]
                assert np.array_equal(np.where(live, gw, 0), np.where(live, gr, 0)), impl
                assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"]), impl
                # the local (idx, term) from the walk against the determinant
                # walk of apus_last_idx_term_batch on the same corrupted rings
                lt = eng.last_idx_term(db, bstruct=bl)
                eng.stats_reset()
                out = eng.update_remote_logs(db, flags | abi.COMMIT_LAST_IT, bstruct=b)
                torch.cuda.synchronize()
                assert torch.equal(out["last_idx_term"], lt), impl
            st = eng.stats()
            assert st[abi.STAT_DECISIONS] == G
            assert st[abi.STAT_CORRUPT] == int((ref["committed"] == 0xFF).sum())
            assert st[abi.STAT_ADVANCED] == int((ref["committed"] == 1).sum())
            assert st[abi.STAT_COMMITTED] == int(ref["n_entries"].sum())


@pytest.mark.parametrize("name", ["c2_skew", "mixed_small", "tiny_wrap"])
def test_commit_walk_only(pkg, orc, eng, name):
    """APUS_COMMIT_WALK alone stops at the first failing entry (no checksum)"""
    import torch
    abi = pkg.abi
    db, hb, _ = _pair(pkg, orc, eng, name)
    out = eng.update_remote_logs(db, abi.COMMIT_WALK)
    torch.cuda.synchronize()
    ref = orc.commit(hb, abi.COMMIT_WALK)
    assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"])
    assert np.array_equal(out["committed"].cpu().numpy(), ref["committed"])


@pytest.mark.parametrize("name", list(CFGS))
def test_vote_rank_prune(pkg, orc, eng, name):
    import torch
    abi = pkg.abi
    db, hb, _ = _pair(pkg, orc, eng, name)
    eng.stats_reset()
    vo = eng.poll_vote_count(db)
    ro = eng.poll_vote_requests(db, derive_local=True)
    po = eng.log_pruning(db)
    torch.cuda.synchronize()
    rv = orc.vote(hb)
    assert np.array_equal(vo["won"].cpu().numpy(), rv["won"])
    assert np.array_equal(vo["vote_count"].cpu().numpy(), rv["vote_count"])
    assert np.array_equal(_u64(vo["new_commit"]), rv["new_commit"])
    assert np.array_equal(vo["voters"].cpu().numpy().view(np.uint16), rv["voters"])
    lit = orc.last_idx_term(hb)
    assert np.array_equal(_u64(ro["last_idx_term"]), lit)
    rr = orc.rank(hb)
    assert np.array_equal(ro["outcome"].cpu().numpy(), rr["outcome"])
    assert np.array_equal(_u64(ro["new_sid"]), rr["new_sid"])
    assert np.array_equal(ro["new_cid"].cpu().numpy(), rr["new_cid"])
    assert np.array_equal(ro["cleared"].cpu().numpy().view(np.uint16), rr["cleared"])
    rp, wm = orc.prune(hb)
    assert np.array_equal(_u64(po["new_head"]), rp["new_head"])
    assert np.array_equal(po["append_head"].cpu().numpy(), rp["append_head"])
    assert np.array_equal(_u64(po["min_apply"]), rp["min_apply"])
    # OFF servers' apply offsets are reset in place, as the reference does
    assert db.download("apply_offsets").tobytes() == hb.apply_offsets.tobytes()
    st = eng.stats()
    assert st[abi.STAT_VOTES_WON] == int(rv["won"].sum())
    assert st[abi.STAT_MIN_WATERMARK] == wm


def _check_vote_rank(orc, hb, vo, ro, lit_given=None):
    rv = orc.vote(hb)
    assert np.array_equal(vo["won"].cpu().numpy(), rv["won"])
    assert np.array_equal(vo["vote_count"].cpu().numpy(), rv["vote_count"])
    assert np.array_equal(_u64(vo["new_commit"]), rv["new_commit"])
    assert np.array_equal(vo["voters"].cpu().numpy().view(np.uint16), rv["voters"])
    if lit_given is not None:                  # the ranking's local (idx, term) input
        hb.arrays["last_idx_term"][:] = lit_given
    rr = orc.rank(hb)
    assert np.array_equal(ro["outcome"].cpu().numpy(), rr["outcome"])
    assert np.array_equal(_u64(ro["new_sid"]), rr["new_sid"])
    assert np.array_equal(ro["new_cid"].cpu().numpy(), rr["new_cid"])
    assert np.array_equal(ro["cleared"].cpu().numpy().view(np.uint16), rr["cleared"])
    return rv


# R beyond the configuration's own: 6 and 8 take the tail's 8-slot form
# with per-replica guards, 11 the 16-slot form
FAIL_R = {"c5": [7, 6, 11], "mixed_small": [7, 8], "short_mixed": [5, 4], "tiny_wrap": [5, 11], "c2_skew": [5, 3]}


@pytest.mark.parametrize("lit", [True, False])
@pytest.mark.parametrize("impl", ["wave", "wave_short", "lane"])
@pytest.mark.parametrize("name,R", [(n, r) for n, rs in FAIL_R.items() for r in rs])
def test_commit_fused_failover(pkg, orc, eng, name, R, impl, lit):
    """APUS_COMMIT_VOTE | APUS_COMMIT_RANK: the vote tally (a5) and the
    vote-request ranking (a6) in the commit call's tail launch equal the
    oracle and the separate apus_vote_batch / apus_vote_rank_batch calls on
    the same batch; the ranking takes the local (idx, term) of the same call
    (APUS_COMMIT_LAST_IT) or, without it, b->last_idx_term; votes won reach
    APUS_STAT_VOTES_WON with the walk's statistics"""
    import torch
    abi = pkg.abi
    kw = CFGS[name]
    G, L = 2048 + 37, kw["ring_len"]
    cfg = pkg.batch.gen_cfg(**kw)
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, cfg)
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, cfg)
    b = db.struct()
    b.flags = IMPL_FLAGS[impl]
    flags = (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PRUNE | abi.COMMIT_VOTE |
             abi.COMMIT_RANK | abi.COMMIT_STATS_FRESH | (abi.COMMIT_LAST_IT if lit else 0))
    out = eng.update_remote_logs(db, flags, bstruct=b)
    torch.cuda.synchronize()
    st = eng.stats().copy()
    ref = orc.commit(hb, abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN)
    assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"])
    assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"])
    assert np.array_equal(_u64(out["median"]), ref["median"])
    if lit:
        assert np.array_equal(_u64(out["last_idx_term"]).reshape(-1), orc.last_idx_term(hb))
    rv = _check_vote_rank(orc, hb, out["vote"], out["rank"],
                          lit_given=orc.last_idx_term(hb) if lit else db.download("last_idx_term").reshape(-1))
    rp, wm = orc.prune(hb)
    assert np.array_equal(_u64(out["new_head"]), rp["new_head"])
    assert st[abi.STAT_DECISIONS] == G and st[abi.STAT_VOTES_WON] == int(rv["won"].sum())
    assert st[abi.STAT_COMMITTED] == int(ref["n_entries"].sum()) and st[abi.STAT_MIN_WATERMARK] == wm
    # the separate calls on the same batch (apply_offsets already reset in
    # place: the reset is idempotent)
    bs = db.struct()
    if lit:
        bs.last_idx_term = out["last_idx_term"].data_ptr()
    eng.stats_reset()
    vo = eng.poll_vote_count(db)
    ro = {k: torch.zeros_like(v) for k, v in out["rank"].items()}
    abi.check(eng.lib.apus_vote_rank_batch(eng.ctx, C.byref(bs), C.byref(eng.rank_struct(ro)), None), "rank")
    torch.cuda.synchronize()
    for k in vo:
        assert torch.equal(vo[k], out["vote"][k]), k
    for k in ro:
        assert torch.equal(ro[k], out["rank"][k]), k
    assert eng.stats()[abi.STAT_VOTES_WON] == st[abi.STAT_VOTES_WON]
    # the failover pass alone (no walk): the tail launch by itself
    out2 = eng.update_remote_logs(db, abi.COMMIT_VOTE | abi.COMMIT_RANK | abi.COMMIT_STATS_FRESH, bstruct=bs)
    torch.cuda.synchronize()
    for k in vo:
        assert torch.equal(out2["vote"][k], vo[k]), k
    for k in ro:
        assert torch.equal(out2["rank"][k], ro[k]), k
    s2 = eng.stats()
    assert s2[abi.STAT_VOTES_WON] == st[abi.STAT_VOTES_WON] and s2[abi.STAT_DECISIONS] == 0


@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("name,R", [("c5", 7), ("mixed_small", 7), ("short_mixed", 5)])
def test_fused_failover_staged_rows_unaligned(pkg, orc, eng, name, R, packed):
    """the C5 tail's request rows staged in LDS by DMA (round 6): 16-B pieces
    when the rows' base is 16-B aligned and the wave is whole, 4-B pieces for a
    partial last wave or a base at 8 mod 16 -- the same results either way
    (the records or the packed vote_sit rows, the winner's cid from the slab),
    and the in-place sid clears land on the relocated rows"""
    import torch
    abi = pkg.abi
    kw = CFGS[name]
    G, L = 2048 + 37, kw["ring_len"]
    cfg = pkg.batch.gen_cfg(**kw)
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, cfg)
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, cfg)
    if packed:
        db.fill_vote_sit()
    key = "vote_sit" if packed else "vote_req"
    src = db.arrays[key].view(torch.uint8).reshape(-1)
    # the rows again at 8 mod 16
    buf = torch.zeros(src.numel() + 32, dtype=torch.uint8, device=src.device)
    off = (8 - buf.data_ptr()) % 16
    moved = buf[off:off + src.numel()]
    moved.copy_(src)
    assert moved.data_ptr() % 16 == 8
    flags = (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PRUNE | abi.COMMIT_VOTE |
             abi.COMMIT_RANK | abi.COMMIT_LAST_IT | abi.COMMIT_STATS_FRESH)
    b = db.struct()
    b.flags = IMPL_FLAGS["wave_short"]
    out = eng.update_remote_logs(db, flags, bstruct=b)
    torch.cuda.synchronize()
    rv = _check_vote_rank(orc, hb, out["vote"], out["rank"], lit_given=orc.last_idx_term(hb))
    assert int(rv["won"].sum()) > 0
    bm = db.struct()
    bm.flags = IMPL_FLAGS["wave_short"]
    if packed:
        bm.vote_sit = moved.data_ptr()
    else:
        bm.vote_req = moved.data_ptr()
    out2 = eng.update_remote_logs(db, flags, bstruct=bm)
    torch.cuda.synchronize()
    for part in ("vote", "rank"):
        for k in out[part]:
            assert torch.equal(out2[part][k], out[part][k]), (part, k)
    if not packed:
        assert torch.equal(moved, db.arrays["vote_req"].view(torch.uint8).reshape(-1))


@pytest.mark.parametrize("R", [3, 5, 7, 11])
@pytest.mark.parametrize("rows", [False, True])
def test_vote_sit_packed_requests(pkg, orc, eng, R, rows):
    """apus_batch_t.vote_sit (ABI 6): the ranking on the packed (sid, index,
    term) rows equals the ranking on the 40-B vote_req records -- the fused
    C5 call (lane and row tails), the separate apus_vote_rank_batch -- and the
    oracle"""
    import torch
    abi = pkg.abi
    kw = CFGS["c5"]
    G, L = 4096 + 5, kw["ring_len"]
    cfg = pkg.batch.gen_cfg(**kw)
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, cfg)
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, cfg)
    flags = (abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PRUNE | abi.COMMIT_LAST_IT |
             abi.COMMIT_VOTE | abi.COMMIT_RANK | abi.COMMIT_STATS_FRESH)
    ap0 = db.arrays["apply_offsets"].clone()
    outs = []
    for packed in (False, True):
        db.arrays["apply_offsets"].copy_(ap0)
        if packed:
            db.fill_vote_sit()
        b = db.struct()
        b.flags = abi.BATCH_SHORT_WALKS | (abi.BATCH_TAIL_ROWS if rows else 0)
        if not packed:
            b.vote_sit = None
        outs.append(eng.update_remote_logs(db, flags, bstruct=b))
        torch.cuda.synchronize()
        # the separate ranking call on the same rows
        bs = db.struct()
        if not packed:
            bs.vote_sit = None
        bs.last_idx_term = outs[-1]["last_idx_term"].data_ptr()
        ro = {k: torch.zeros_like(v) for k, v in outs[-1]["rank"].items()}
        abi.check(eng.lib.apus_vote_rank_batch(eng.ctx, C.byref(bs), C.byref(eng.rank_struct(ro)), None), "rank")
        torch.cuda.synchronize()
        for k in ro:
            assert torch.equal(ro[k], outs[-1]["rank"][k]), (packed, k)
    a, p = outs
    for k in a["rank"]:
        assert torch.equal(a["rank"][k], p["rank"][k]), k
    for k in a["vote"]:
        assert torch.equal(a["vote"][k], p["vote"][k]), k
    hs = db.download("vote_sit").reshape(G, R, 3)
    assert np.array_equal(hs[..., 0], hb.vote_req["sid"].reshape(G, R))
    _check_vote_rank(orc, hb, p["vote"], p["rank"], lit_given=orc.last_idx_term(hb))


def test_commit_fused_failover_refusals(pkg, eng):
    """the failover flags refuse a batch without their columns"""
    abi = pkg.abi
    db = pkg.batch.DeviceBatch(64, 3, pkg.batch.ring_stride_for(4096))
    out = eng.alloc_commit_out(64, abi.COMMIT_VOTE | abi.COMMIT_RANK)
    o = eng.commit_struct(out)
    b = db.struct()
    b.vote_ack = None
    assert eng.lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), abi.COMMIT_VOTE, None) == abi.APUS_ERROR
    b = db.struct()
    b.last_idx_term = None
    assert eng.lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), abi.COMMIT_RANK, None) == abi.APUS_ERROR
    b.hb = None
    assert eng.lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), abi.COMMIT_RANK | abi.COMMIT_LAST_IT,
                                     None) == abi.APUS_ERROR


@pytest.mark.parametrize("name", ["c2", "c3_var", "mixed_small", "tiny_wrap", "wrap_aligned", "short_mixed",
                                  "history_only", "malformed"])
def test_nc_build_quad_and_lane(pkg, orc, eng, name):
    """log_entries_to_nc_buf: the 16-lane speculative segments (default), the
    four-lanes-per-group kernel (APUS_BATCH_VAR_LEN) and the lane-per-group
    walk (APUS_BATCH_LANE_IMPL) against the oracle, buffers
    larger and smaller than the chains.  On corrupted rings
    (undefined in the reference; the oracle reads past the ring where the
    device stops at it) the two device kernels must agree with each other."""
    import torch
    abi = pkg.abi
    if name == "malformed":
        hb = _malformed(pkg, orc, 4096, 77, False)
        db = pkg.batch.DeviceBatch(hb.G, hb.R, hb.stride)
        db.upload(hb)
    else:
        db, hb, _ = _pair(pkg, orc, eng, name)
    res = {}
    for impl in (0, abi.BATCH_LANE_IMPL, abi.BATCH_VAR_LEN):
        out = {}
        for cap in (256, 13, 1):
            b = db.struct()
            b.flags = impl
            dets, ln = eng.log_entries_to_nc_buf(db, cap, bstruct=b)
            torch.cuda.synchronize()
            ln = ln.cpu().numpy().view(np.uint32).copy()
            got = dets.cpu().numpy().view(np.uint64).reshape(hb.G, cap * 3).copy()
            for g in range(hb.G):                     # entries past the length are not outputs
                got[g, 3 * int(ln[g]):] = 0
            out[cap] = (ln, got)
        res[impl] = out
    # 0: 16-lane segments (default); LANE_IMPL: a lane per group; VAR_LEN: the quad kernel
    q, lane, quad = res[0], res[abi.BATCH_LANE_IMPL], res[abi.BATCH_VAR_LEN]
    for cap in (256, 13, 1):
        for other, nm in ((lane, "lane"), (quad, "quad")):
            assert np.array_equal(q[cap][0], other[cap][0]), (nm, cap)
            assert np.array_equal(q[cap][1], other[cap][1]), (nm, cap)
    if name == "malformed":
        return
    for cap in (256, 13, 1):
        rd, rl = orc.nc_build(hb, cap)
        ref = rd.reshape(hb.G, cap * 3).copy()
        for g in range(hb.G):
            ref[g, 3 * int(rl[g]):] = 0
        assert np.array_equal(q[cap][0], rl), cap
        assert np.array_equal(q[cap][1], ref), cap


@pytest.mark.parametrize("name", ["c2_skew", "c3_var", "mixed_small", "tiny_wrap"])
def test_validate_and_nc_build(pkg, orc, eng, name):
    import torch
    abi = pkg.abi
    db, hb, cfg = _pair(pkg, orc, eng, name)
    F, M = RS[name] - 1, 256
    dets, ln = eng.log_entries_to_nc_buf(db, M)
    torch.cuda.synchronize()
    rd, rl = orc.nc_build(hb, M)
    assert np.array_equal(ln.cpu().numpy().view(np.uint32), rl)
    got = dets.cpu().numpy().view(np.uint64)
    for g in range(hb.G):
        n = int(rl[g])
        assert np.array_equal(got[g * M * 3:g * M * 3 + 3 * n], rd[g * M * 3:g * M * 3 + 3 * n])
    # a buffer smaller than the chain: the walk stops at max_dets mid-step
    for cap in (1, 7, 70):
        dets_c, ln_c = eng.log_entries_to_nc_buf(db, cap)
        torch.cuda.synchronize()
        if cap == 7:
            dets_c7, ln_c7 = dets_c, ln_c
        rdc, rlc = orc.nc_build(hb, cap)
        assert np.array_equal(ln_c.cpu().numpy().view(np.uint32), rlc)
        gc = dets_c.cpu().numpy().view(np.uint64).reshape(hb.G, cap * 3)
        rc = rdc.reshape(hb.G, cap * 3)
        for g in range(hb.G):
            n = int(rlc[g])
            assert np.array_equal(gc[g, :3 * n], rc[g, :3 * n]), (cap, g)
    fd, fl, ff = orc.gen_nc(hb, cfg, F, M)
    eng.stats_reset()
    t = torch.from_numpy(fd.view(np.uint8)).cuda()
    tl = torch.from_numpy(fl.view(np.int32)).cuda()
    tf = torch.from_numpy(ff).cuda()
    out = eng.log_find_remote_end_offset(db, t, tl, tf, M)
    torch.cuda.synchronize()
    ref = orc.validate(hb, fd, fl, ff, F, M)
    assert np.array_equal(_u64(out), ref)
    # mismatches: followers whose validated end stops before the end of their
    # last determinant's entry (a mismatch or a missing entry was found)
    exp = 0
    for gf in range(hb.G * F):
        n = int(fl[gf])
        if n:
            exp += int(not _all_match(hb, gf // F, fd[gf * M * 3:gf * M * 3 + 3 * n]))
    assert eng.stats()[abi.STAT_MISMATCHES] == exp
    # with the leader's own determinants (whole rows, and rows cut at 7 so the
    # rest gather): the same ends and mismatch counts
    for ld, ll, lm in ((dets, ln, M), (dets_c7, ln_c7, 7)):
        eng.stats_reset()
        out_l = eng.log_find_remote_end_offset(db, t, tl, tf, M, leader=(ld, ll, lm))
        torch.cuda.synchronize()
        assert np.array_equal(_u64(out_l), ref), lm
        assert eng.stats()[abi.STAT_MISMATCHES] == exp, lm


def _all_match(hb, g, d):
    """True when every determinant matches the leader's entry (no early return)"""
    ring = hb.group_ring(g)
    s = hb.state[g]
    ln, end = int(s["len"]), int(s["end"])
    for k in range(len(d) // 3):
        off = int(d[3 * k + 2])
        dist = 0 if end == ln else (end - off if end >= off else ln - (off - end))
        if end == ln or dist == 0:
            return False
        if ln - off < 64:
            off = 0
        idx = int.from_bytes(bytes(ring[off:off + 8]), "little")
        term = int.from_bytes(bytes(ring[off + 8:off + 16]), "little")
        if idx != int(d[3 * k]) or term != int(d[3 * k + 1]):
            return False
    return True


def _end_after(hb, g, off):
    ring = hb.group_ring(g)
    ln = int(hb.state[g]["len"])
    if ln - off < 64:
        off = 0
    t = ring[off + 26]
    clen = int(ring[off + 48]) | (int(ring[off + 49]) << 8)
    el = 64 if t in (0, 2, 3) else 64 + clen
    return (0 if ln - off < el else off) + el


def test_full_size_c2_sampled(pkg, orc, eng):
    """BASELINE config 2 at full size (2^20 groups, R=3, E=64, 64-B SET entries):
    per-group outputs of a sampled range equal the oracle's; stats equal the
    sums of the per-group outputs."""
    import torch
    abi = pkg.abi
    G, R, L = 1 << 20, 3, 16384
    kw = dict(seed=7, n_entries=64, n_history=16, len_min=64, len_max=64, ring_len=L,
              p_full_ack=0.9, straggler=True)
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L),
                               fields=["state", "self_idx", "remote_end", "lr_step", "fail_count"])
    eng.gen(db, pkg.batch.gen_cfg(**kw))
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN
    eng.stats_reset()
    out = eng.update_remote_logs(db, flags)
    torch.cuda.synchronize()
    st = eng.stats()
    n_ent = out["n_entries"].cpu().numpy().view(np.uint32)
    assert st[abi.STAT_DECISIONS] == G
    assert st[abi.STAT_COMMITTED] == int(n_ent.astype(np.uint64).sum())
    assert st[abi.STAT_ADVANCED] == int((out["committed"].cpu().numpy() == 1).sum())
    for g0 in (0, G // 2 + 12345, G - 3000):
        S = 3000
        hb = orc.host_batch(S, R, L, fields=["state", "self_idx", "remote_end", "lr_step", "fail_count"])
        orc.gen(hb, pkg.batch.gen_cfg(gid_base=g0, **kw))
        ref = orc.commit(hb, flags)
        assert np.array_equal(_u64(out["new_commit"][g0:g0 + S]), ref["new_commit"])
        assert np.array_equal(out["digest"][g0:g0 + S].cpu().numpy().view(np.uint32), ref["digest"])
        assert np.array_equal(_u64(out["median"][g0:g0 + S]), ref["median"])


# ------------------------------------------------------------- scalar ABI
def _ref_shaped(pkg, hb, g, mode="heap"):
    """build a dare_log_t / server_config_t / ctrl_data_t byte image for group
    g; the log is a caller heap buffer (staged) or an apus_log_new log"""
    abi = pkg.abi
    st = hb.state[g]
    ln = int(st["len"])
    lg = ScalarLog(pkg, ln, mode).load(hb, g)
    lg.log.old_end = int(st["end"])
    R = hb.R
    servers = (abi.Server * 13)()
    for i in range(R):
        servers[i].fail_count = int(hb.fail_count[g * R + i])
        servers[i].next_lr_step = int(hb.lr_step[g * R + i])
    cfg = abi.ServerConfig()
    C.memmove(C.addressof(cfg.cid), hb.state[g:g + 1].tobytes()[48:64], 16)
    cfg.idx = int(hb.self_idx[g])
    cfg.len = 13
    cfg.servers = servers
    ctrl = abi.CtrlData()
    ctrl.sid = int(hb.sid[g])
    for i in range(13):
        ctrl.vote_ack[i] = int(hb.vote_ack[g * R + i]) if i < R else ln
    for i in range(R):
        ctrl.log_offsets[i].end = int(hb.remote_end[g * R + i])
        ctrl.log_offsets[i].commit = int(hb.remote_commit[g * R + i])
        ctrl.apply_offsets[i] = int(hb.apply_offsets[g * R + i])
        ctrl.hb[i] = int(hb.hb[g * R + i])
        C.memmove(C.addressof(ctrl.vote_req[i]), hb.vote_req[g * R + i:g * R + i + 1].tobytes(), 40)
    return lg, cfg, servers, ctrl


@pytest.mark.parametrize("unk", [False, True])
@pytest.mark.parametrize("mode", ["heap", "owned"])
@pytest.mark.parametrize("name", ["c2_skew", "mixed_small", "tiny_wrap", "c3_var"])
def test_scalar_dropins(pkg, orc, eng, name, mode, unk):
    """every scalar drop-in against the oracle: the one-launch calls (state,
    columns and the walked ring bytes in the kernel arguments) and the staged
    path they fall back to (c3_var's walks exceed the argument window; unk:
    tail == len on every other log, so the pruning minimum's log_get_tail
    scans the chains from commit / apply / head)"""
    abi = pkg.abi
    lib = abi.load_library()
    kw = dict(CFGS[name])
    R = RS[name]
    G = 64 if name != "c3_var" else 16
    cfg = pkg.batch.gen_cfg(**kw)
    hb = orc.host_batch(G, R, kw["ring_len"])
    orc.gen(hb, cfg)
    if unk:
        hb.state["tail"][::2] = hb.state["len"][::2]
        # the pruning minimum at end on some logs: log_get_tail decides
        ap = hb.apply_offsets.reshape(G, R)
        ap[1::3] = hb.state["end"][1::3][:, None]
        hb.state["apply"][1::3] = hb.state["end"][1::3]
    ref = orc.commit(hb, abi.COMMIT_WALK | abi.COMMIT_MEDIAN)
    rv = orc.vote(hb)
    rr = orc.rank(hb, use_lit=False)
    ap0 = hb.apply_offsets.copy()
    rp, _ = orc.prune(hb)                      # resets OFF servers' apply offsets in hb
    ap1 = hb.apply_offsets.copy()
    dets, ln = orc.nc_build(hb, 1024)
    for g in range(G):
        lg, scfg, servers, ctrl = _ref_shaped(pkg, hb, g, mode)
        for i in range(R):
            ctrl.apply_offsets[i] = int(ap0[g * R + i])
        sids = [ctrl.vote_req[i].sid for i in range(13)]
        logp = lg.ptr
        nc = C.c_uint64(0)
        cm = C.c_int(0)
        assert lib.apus_commit_reply_walk(logp, C.byref(scfg), C.byref(nc), C.byref(cm)) == 0
        assert nc.value == ref["new_commit"][g] and cm.value == ref["committed"][g]
        md = C.c_uint64(0)
        assert lib.apus_commit_median(logp, C.byref(scfg), C.byref(ctrl), C.byref(md)) == 0
        assert md.value == ref["median"][g]
        vc = (C.c_uint8 * 2)()
        vcm = C.c_uint64(0)
        vm = C.c_uint16(0)
        won = lib.apus_vote_tally(logp, C.byref(scfg), C.byref(ctrl), vc, C.byref(vcm), C.byref(vm))
        assert won == rv["won"][g] and vcm.value == rv["new_commit"][g] and vm.value == rv["voters"][g]
        oc = C.c_uint8(0)
        ns = C.c_uint64(0)
        ncid = abi.Cid()
        clr = C.c_uint16(0)
        assert lib.apus_vote_rank(logp, C.byref(scfg), C.byref(ctrl), C.byref(oc), C.byref(ns), C.byref(ncid),
                                  C.byref(clr)) == 0
        assert oc.value == rr["outcome"][g] and ns.value == rr["new_sid"][g] and clr.value == rr["cleared"][g]
        # consumed / dropped requests are cleared in place, as the reference does
        assert [ctrl.vote_req[i].sid for i in range(13)] == [0 if clr.value >> i & 1 else sids[i] for i in range(13)]
        nh = C.c_uint64(0)
        ap = C.c_int(0)
        assert lib.apus_min_apply(logp, C.byref(scfg), C.byref(ctrl), int(hb.prev_head[g]), C.byref(nh),
                                  C.byref(ap)) == 0
        assert nh.value == rp["new_head"][g] and ap.value == rp["append_head"][g]
        assert [ctrl.apply_offsets[i] for i in range(R)] == [int(x) for x in ap1[g * R:(g + 1) * R]]
        ncb = abi.NcBuf()
        assert lib.apus_entries_to_nc_buf(logp, C.byref(ncb)) == 0
        n = int(ln[g])
        assert ncb.len == n
        got = np.frombuffer(bytes(ncb.entries)[:24 * n], np.uint64)
        assert np.array_equal(got, dets[g * 1024 * 3:g * 1024 * 3 + 3 * n])
        if n:
            fe = C.c_uint64(0)
            assert lib.apus_find_remote_end(logp, C.byref(ncb), C.byref(fe)) == 0
            exp = C.c_uint64(0)
            orc.lib().apus_oracle_find_remote_end(C.c_void_p(hb.group_ring(g).ctypes.data),
                                                  C.c_void_p(hb.state.ctypes.data + 64 * g),
                                                  C.c_void_p(got.ctypes.data), n, C.byref(exp))
            assert fe.value == exp.value
        lg.free()


@pytest.mark.parametrize("R", [3, 5, 7])
def test_median_config_sizes(pkg, orc, eng, R):
    """The median (and the pruning minimum beside it) with every configuration
    the batch can hold: sizes size[0], size[1] drawn from 1 ... R independently,
    STABLE / EXTENDED / TRANSIT, random bitmasks -- the tail's rank selection
    over the R replica slots (both sizes <= R, group_ops.h median_of) against
    the oracle (dare_ibv_rc.c:1650-1723), in the bench's flag set (walk +
    checksum + median + pruning: the compile-time-flag tail instantiation)"""
    import torch
    abi = pkg.abi
    G, L = 4096, 8192
    cfg = pkg.batch.gen_cfg(seed=211 + R, n_entries=16, n_history=8, len_min=16, len_max=100, ring_len=L,
                            cid_mix=True, straggler=True, p_full_ack=0.7, self_random=True)
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, cfg)
    rng = np.random.default_rng(300 + R)
    cid = hb.state["cid"]
    cid["size0"] = rng.integers(1, R + 1, G)
    cid["size1"] = rng.integers(1, R + 1, G)
    cid["state"] = rng.integers(0, 3, G)
    cid["bitmask"] = rng.integers(0, 1 << R, G)
    db = pkg.batch.DeviceBatch(G, R, hb.stride)
    db.upload(hb)
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PRUNE
    eng.stats_reset()
    out = eng.update_remote_logs(db, flags)
    torch.cuda.synchronize()
    ref = orc.commit(hb, flags)
    rp, wm = orc.prune(hb)
    assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"])
    assert np.array_equal(_u64(out["median"]), ref["median"])
    assert np.array_equal(_u64(out["new_head"]), rp["new_head"])
    assert np.array_equal(out["append_head"].cpu().numpy(), rp["append_head"])
    assert np.array_equal(_u64(out["min_apply"]), rp["min_apply"])
    assert np.array_equal(db.download("apply_offsets"), hb.apply_offsets)
    assert eng.stats()[abi.STAT_MIN_WATERMARK] == wm
    # the draw reaches both sizes below R, unequal sizes and TRANSIT
    assert ((cid["size0"] != cid["size1"]) & (cid["state"] == 1)).sum() > 100      # APUS_CID_TRANSIT


@pytest.mark.parametrize("mode", ["heap", "owned"])
def test_scalar_walk_malformed(pkg, orc, mode):
    """the one-launch reply walk (the wave form: lane 0 follows the chain,
    the lanes count the replies) and its exact serial fallback on corrupted
    logs: ends inside entries, garbage types and lengths at the commit
    offset, random commits, garbage rings -- against the oracle's walk,
    the corrupt flag (0xFF) included"""
    import test_publish_force as tp
    abi = pkg.abi
    lib = abi.load_library()
    G = 256
    hb = _malformed(pkg, orc, G, 77, False)
    if mode == "heap":
        # a caller heap log is staged: the call sees the ranges Stager::chain
        # copies ([commit, end), wrapped, and the header at 0) and the poison
        # byte everywhere else, so a chain that leaves them (an end moved
        # inside an entry) walks poison -- the oracle on that image
        hb = tp.clone(hb)
        st = hb.state
        for g in range(G):
            ring = hb.group_ring(g)
            L, c, e = int(st["len"][g]), int(st["commit"][g]), int(st["end"][g])
            keep = np.zeros(L, bool)
            if not (e >= L or c == e):
                if c < e:
                    keep[c:e] = True
                else:
                    keep[c:] = True
                    keep[:e] = True
                keep[:64] = True
            ring[:L][~keep] = 0xFF
    ref = orc.commit(hb, abi.COMMIT_WALK)
    assert (ref["committed"] == 0xFF).any() and (ref["committed"] == 1).any()
    for g in range(G):
        lg, scfg, servers, ctrl = _ref_shaped(pkg, hb, g, mode)
        nc, cm = C.c_uint64(0), C.c_int(0)
        rc = lib.apus_commit_reply_walk(lg.ptr, C.byref(scfg), C.byref(nc), C.byref(cm))
        if ref["committed"][g] == 0xFF:
            assert rc == abi.APUS_ERROR, g          # a corrupt chain (the walk's step guard)
        else:
            assert rc == 0 and (nc.value, cm.value) == (ref["new_commit"][g], ref["committed"][g]), g
        lg.free()


@pytest.mark.parametrize("mode", ["heap", "owned"])
@pytest.mark.parametrize("ci", [0, 2, 3, 4])
def test_scalar_publish_force(pkg, orc, ci, mode):
    """apus_publish_commit and apus_force_log_pruning on reference-shaped
    structs against the oracle's publish / force_log_pruning (rings near or
    past 75% full: every outcome, the CONFIG entry written into the caller's
    log, its end / tail / cid / req_id / clt_id / apply offsets updated)"""
    import test_publish_force as tp
    abi = pkg.abi
    lib = abi.load_library()
    kw, R = tp.FULL[ci]
    G = 48
    hb = orc.host_batch(G, R, kw["ring_len"])
    orc.gen(hb, pkg.batch.gen_cfg(**kw))
    tp.perturb(hb, np.random.default_rng(900 + ci))
    hb.self_idx[hb.self_idx >= R] = 0            # the scalar structs hold 13 servers: keep the leader a replica
    want = tp.clone(hb)
    rq = np.arange(G, dtype=np.uint64) + 11
    cl = (np.arange(G) + 5).astype(np.uint16)
    flags = abi.COMMIT_PUBLISH | abi.COMMIT_FORCE_PRUNE
    to, _, _ = orc.tail(want, flags, None, out=orc.tail_out(G, flags, req_id=rq, clt_id=cl))
    seen = set()
    for g in range(G):
        lg, scfg, servers, ctrl = _ref_shaped(pkg, hb, g, mode)
        scfg.req_id, scfg.clt_id = int(rq[g]), int(cl[g])
        conn = int(hb.rc_connected[g])
        ssn = C.c_uint64(5)
        post = C.c_uint16(0)
        assert lib.apus_publish_commit(lg.ptr, C.byref(scfg), C.byref(ctrl), conn, C.byref(ssn), C.byref(post)) == 0
        assert post.value == to["publish"][g]
        assert ssn.value == 5 + (1 if to["publish"][g] else 0)
        assert [ctrl.log_offsets[i].commit for i in range(R)] == [int(x) for x in want.remote_commit[g * R:(g + 1) * R]]
        prev = C.c_int(int(hb.prev_head[g]))
        tg, ci_, nh, app = C.c_uint8(0), C.c_uint64(0), C.c_uint64(0), C.c_int(0)
        act = lib.apus_force_log_pruning(lg.ptr, C.byref(scfg), C.byref(ctrl), C.byref(prev), C.byref(tg),
                                         C.byref(ci_), C.byref(nh), C.byref(app))
        f = to["force"]
        assert act == f["action"][g], (g, act, f["action"][g])
        seen.add(act)
        if act:
            assert tg.value == f["target"][g] and ci_.value == f["cfg_idx"][g]
            assert nh.value == to["new_head"][g] and app.value == to["append_head"][g]
        assert prev.value == want.prev_head[g]
        assert scfg.req_id == f["req_id"][g] and scfg.clt_id == f["clt_id"][g]
        st = want.state[g]
        assert (lg.log.end, lg.log.tail) == (int(st["end"]), int(st["tail"]))
        assert bytes(scfg.cid) == want.state[g:g + 1].tobytes()[48:64]
        assert [ctrl.apply_offsets[i] for i in range(R)] == [int(x) for x in want.apply_offsets[g * R:(g + 1) * R]]
        ln = int(st["len"])
        assert np.array_equal(lg.buf[lg.hdr:lg.hdr + ln], want.group_ring(g)[:ln])
        lg.free()
    assert abi.FORCE_REMOVE in seen and abi.FORCE_NONE in seen
