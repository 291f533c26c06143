"""the reference's dare_log_t as a device-resident RDMA target.

Each group is a whole dare_log_t image in HBM (src/include/dare/dare_log.h:
77-103: the 319,656-B header with head/apply/commit/end/tail/old_end/
old_commit/len and nc_buf[13], then entries[]), the layout the reference
registers for RDMA (dare_ibv_rc.c:240-276).  The followers' acks are the
reply[i] bytes their rc_send_entries_reply RDMA-writes into the leader's
entries (dare_ibv_rc.c:1828-1863).  Here those writes are made by a copy on a
separate stream -- standing in for a GPUDirect NIC writing into HBM -- and
the commit walk, median, vote tally and pruning read the images in place
(APUS_BATCH_LOG_IMAGE), with no 64-B state row.  Every output is compared
bit-exactly with the CPU oracle, before the acks land (nothing commits past
the straggler-free prefix the replies allow) and after.
"""
import numpy as np
import pytest

CFGS = {
    "c2": (dict(seed=801, n_entries=64, n_history=16, len_min=64, len_max=64, ring_len=16384, straggler=True,
                p_full_ack=0.8), 3, 2048),
    "mixed": (dict(seed=802, n_entries=24, n_history=8, len_min=0, len_max=90, ring_len=6000, type_mix=True,
                   cid_mix=True, self_random=True, garbage_reply=0.05, p_full_ack=0.5), 7, 2048),
    "wrap": (dict(seed=803, n_entries=12, n_history=3, len_min=0, len_max=100, ring_len=4096, type_mix=True,
                  cid_mix=True, self_random=True, p_full_ack=0.6, straggler=True), 5, 2048),
}


def _host(pkg, orc, name):
    kw, R, G = CFGS[name]
    hb = orc.host_batch(G, R, kw["ring_len"])
    orc.gen(hb, pkg.batch.gen_cfg(**kw))
    return hb


def _reply_sites(hb, orc):
    """flat (group, ring offset) of every reply[] byte of the entries in
    [commit, end): where the followers' RDMA writes land"""
    dets, ln = orc.nc_build(hb, 1024)
    dets = np.asarray(dets).reshape(hb.G, 1024, 3)
    g_idx, off = [], []
    for g in range(hb.G):
        n = int(ln[g])
        o = dets[g, :n, 2].astype(np.int64)
        g_idx.append(np.full(n, g, np.int64))
        off.append(o)
    g_idx, off = np.concatenate(g_idx), np.concatenate(off)
    k = np.arange(13, dtype=np.int64)
    return np.repeat(g_idx, 13), (off[:, None] + 28 + k[None, :]).reshape(-1)


def test_log_image_layout_cpu(pkg):
    """the image stride keeps entries[] 16-B aligned and the pad after len"""
    s = pkg.batch.log_image_stride(16384)
    assert s % 256 == 0 and s >= pkg.abi.LOG_HDR_BYTES + 16384 + 16
    assert (pkg.abi.LOG_HDR_BYTES + 8) % 16 == 0          # images at 8 mod 16


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
@pytest.mark.parametrize("impl", [0, 0x1, 0x2, 0x8])
@pytest.mark.parametrize("name", list(CFGS))
def test_acks_land_in_hbm_log_images(pkg, orc, eng, name, impl):
    import torch
    abi = pkg.abi
    hb = _host(pkg, orc, name)
    G, R = hb.G, hb.R
    img = pkg.batch.LogImageBatch(G, R, CFGS[name][0]["ring_len"])
    img.fill_from(hb)
    gi, ro = _reply_sites(hb, orc)
    flat = torch.from_numpy(gi * img.stride + img.off + abi.LOG_HDR_BYTES + ro).cuda()
    acks = torch.from_numpy(hb.ring[gi * hb.stride + ro].copy()).cuda()
    img.buf[flat] = 0                                       # no follower has acked yet
    torch.cuda.synchronize()
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_LAST_IT

    def run():
        b = img.struct()
        b.flags |= impl
        eng.stats_reset()
        out = eng.update_remote_logs(img, flags, bstruct=b)
        out["lit_batch"] = eng.last_idx_term(img, bstruct=b)   # before the pruning moves head
        vo = eng.poll_vote_count(img)
        po = eng.log_pruning(img)
        torch.cuda.synchronize()
        return out, vo, po

    def check(out, vo, po, h):
        ref = orc.commit(h, flags)
        assert np.array_equal(_u64(out["new_commit"]), ref["new_commit"])
        assert np.array_equal(out["committed"].cpu().numpy(), ref["committed"])
        assert np.array_equal(out["n_entries"].cpu().numpy().view(np.uint32), ref["n_entries"])
        assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"])
        assert np.array_equal(_u64(out["median"]), ref["median"])
        # APUS_COMMIT_LAST_IT on dare_log_t images: the tail reads b.ring + g*stride + row
        want = orc.last_idx_term(h)
        assert np.array_equal(_u64(out["last_idx_term"]).reshape(-1), want)
        assert np.array_equal(_u64(out["lit_batch"]).reshape(-1), want)
        rv = orc.vote(h)
        assert np.array_equal(vo["won"].cpu().numpy(), rv["won"])
        assert np.array_equal(_u64(vo["new_commit"]), rv["new_commit"])
        rp, wm = orc.prune(h)
        assert np.array_equal(_u64(po["new_head"]), rp["new_head"])
        assert np.array_equal(po["append_head"].cpu().numpy(), rp["append_head"])
        st = eng.stats()
        assert st[abi.STAT_COMMITTED] == int(ref["n_entries"].sum())
        return ref

    # before the acks: the oracle on the same log with every reply[] zeroed
    h0 = pkg.batch.HostBatch(G, R, hb.stride, fields=list(hb.arrays))
    h0.ring[:] = hb.ring
    for k, v in hb.arrays.items():
        h0.arrays[k][:] = v
    h0.ring[gi * hb.stride + ro] = 0
    ref0 = check(*run(), h0)
    hb.apply_offsets[:] = h0.apply_offsets                 # the pruning reset OFF servers' offsets in place
    # the followers' reply writes, issued on another stream (the NIC)
    nic = torch.cuda.Stream()
    with torch.cuda.stream(nic):
        img.buf[flat] = acks
        landed = torch.cuda.Event()
        landed.record(nic)
    torch.cuda.current_stream().wait_event(landed)
    ref1 = check(*run(), hb)
    assert (ref1["n_entries"] >= ref0["n_entries"]).all() and ref1["n_entries"].sum() > ref0["n_entries"].sum()


@pytest.mark.gpu
def test_log_image_validate_and_nc_build(pkg, orc, eng):
    """log_entries_to_nc_buf and log_find_remote_end_offset on log images"""
    import torch
    hb = _host(pkg, orc, "wrap")
    G, R = hb.G, hb.R
    F, M = R - 1, 64
    img = pkg.batch.LogImageBatch(G, R, CFGS["wrap"][0]["ring_len"])
    img.fill_from(hb)
    dets, ln = eng.log_entries_to_nc_buf(img, M)
    torch.cuda.synchronize()
    rd, rl = orc.nc_build(hb, M)
    assert np.array_equal(ln.cpu().numpy().view(np.uint32), rl)
    got = dets.cpu().numpy().view(np.uint64).reshape(G, M * 3)
    for g in range(G):
        assert np.array_equal(got[g, :3 * int(rl[g])], rd[g * M * 3:g * M * 3 + 3 * int(rl[g])])
    fd, fl, ff = orc.gen_nc(hb, pkg.batch.gen_cfg(**CFGS["wrap"][0]), F, M)
    out = eng.log_find_remote_end_offset(img, torch.from_numpy(fd.view(np.uint8)).cuda(),
                                         torch.from_numpy(fl.view(np.int32)).cuda(), torch.from_numpy(ff).cuda(), M)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(out), orc.validate(hb, fd, fl, ff, F, M))


@pytest.mark.gpu
def test_log_image_refused_by_generator(pkg, orc, eng):
    """the synthetic generator writes state rows: it refuses image batches
    (every other writer updates the image header in place)"""
    import ctypes as C
    abi = pkg.abi
    hb = _host(pkg, orc, "wrap")
    img = pkg.batch.LogImageBatch(hb.G, hb.R, CFGS["wrap"][0]["ring_len"])
    b = img.struct()
    cfg = pkg.batch.gen_cfg(**CFGS["wrap"][0])
    assert eng.lib.apus_gen_batch(eng.ctx, C.byref(b), C.byref(cfg), eng._stream()) == abi.APUS_ERROR


def _image_of(pkg, hb, L):
    img = pkg.batch.LogImageBatch(hb.G, hb.R, L)
    img.fill_from(hb)
    return img


def _rings_equal(img, hb, L):
    return np.array_equal(img.download("ring"), hb.ring.reshape(hb.G, hb.stride)[:, :L])


def _state_equal(img, hb, keys=("head", "apply", "commit", "end", "tail", "len")):
    st = img.download("state")
    for k in keys:
        assert np.array_equal(st[k], hb.state[k]), k
    assert st["cid"].tobytes() == hb.state["cid"].tobytes(), "cid"


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c2", "csm_var", "fresh_tiny", "tail_scan"])
def test_writers_append_persist_on_log_images(pkg, orc, eng, name):
    """log_append_entry / persist_new_entries on dare_log_t images: the
    entries land in each image's entries[] and end / tail in its header
    (dare_log.h:466-558), bit-exact against the oracle"""
    import torch
    import test_append as ta
    hb, ent, payload, M, n_entries = ta.build(pkg, orc, name)
    L = int(hb.state["len"][0])
    assert (hb.state["len"] == L).all()
    img = _image_of(pkg, hb, L)
    d_ent = torch.from_numpy(ent.view(np.uint8).copy()).cuda()
    d_pay = torch.from_numpy(payload).cuda()
    d_n = torch.from_numpy(n_entries.view(np.int32).copy()).cuda()
    eng.stats_reset()
    out = eng.log_append_entry(img, d_ent, d_pay, M, n_entries=d_n)
    idx, last, bad = orc.append(hb, ent, payload, M, n_entries=n_entries)
    torch.cuda.synchronize()
    assert _rings_equal(img, hb, L), "entries[] differ after append"
    _state_equal(img, hb)
    assert np.array_equal(img.download("prev_head"), hb.prev_head)
    assert np.array_equal(out["idx"].cpu().numpy().view(np.uint64), idx)
    assert int(eng.stats()[pkg.abi.STAT_CORRUPT]) == bad
    if not ta.CASES[name].get("persist", True):
        return
    old_end, limit = ta.persist_inputs(hb, 9, hb.end0)
    d_oe = torch.from_numpy(old_end.view(np.int64).copy()).cuda()
    d_lim = torch.from_numpy(limit.view(np.int32).copy()).cuda()
    eng.persist_new_entries(img, d_oe, d_lim)
    orc.persist(hb, old_end, limit)
    torch.cuda.synchronize()
    assert _rings_equal(img, hb, L), "entries[] differ after persist"
    assert np.array_equal(d_oe.cpu().numpy().view(np.uint64), old_end)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["mixed", "wrap_small"])
def test_writers_apply_config_scan_on_log_images(pkg, orc, eng, name):
    """apply_committed_entries / poll_config_entries on images: apply and head
    advance in each image's header, config.cid in the cid array"""
    import test_apply as tp
    hb, off, cidx = tp.build(pkg, orc, name)
    L = int(hb.state["len"][0])
    h2 = tp._clone(pkg, hb)
    img = _image_of(pkg, hb, L)
    io = orc.config_io(hb.G, off, cidx)
    out = eng.poll_config_entries(img, io)
    orc.config_scan(hb, io)
    for k in ("cid_offset", "req_id", "clt_id", "departed"):
        assert np.array_equal(out[k], io[k]), k
    _state_equal(img, hb)
    img2 = _image_of(pkg, h2, L)
    io2 = orc.apply_io(h2.G, 4)
    out2 = eng.apply_committed_entries(img2, io2)
    orc.apply(h2, io2)
    for k in ("req_id", "clt_id", "last_applied", "last_csm_idx", "n_applied", "departed", "events", "n_cfg",
              "cfg_payload", "cfg_entries"):
        assert np.array_equal(out2[k], io2[k]), k
    _state_equal(img2, h2)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["r5_mix", "r7_c5"])
def test_writers_log_adjust_on_log_images(pkg, orc, eng, name):
    """log_adjustment on images: the leader's commit advances in the image
    header (dare_ibv_rc.c:1340-1352), the step columns as on state rows"""
    import test_lr_step as tl
    hb, io = tl.build(pkg, orc, name)
    L = int(hb.state["len"][0])
    img = _image_of(pkg, hb, L)
    out = eng.log_adjustment(img, tl._clone_io(io))
    orc.log_adjust(hb, io)
    _state_equal(img, hb)
    for k in ("lr_step", "remote_commit", "remote_end"):
        assert np.array_equal(img.download(k), getattr(hb, k)), k
    for k in tl.IO_KEYS:
        if k in out:
            assert np.array_equal(out[k], io[k]), k


@pytest.mark.gpu
def test_log_image_len_beyond_capacity(pkg, orc, eng):
    """a dare_log_t image whose header len exceeds its entries[]
    capacity (image stride - header) but not the stride.  Without the
    capacity bound, append would write into the next image's header and past
    the batch for the last group.  Such a group is CORRUPT: append and the
    commit walk leave it, every other group is the oracle's, and the next
    image's header and entries are untouched; the readers (pruning, NC build,
    validation, last (idx, term)) stay inside the group's ring."""
    import torch
    import test_append as ta
    abi = pkg.abi
    hb, ent, payload, M, n_entries = ta.build(pkg, orc, "c2")
    L = int(hb.state["len"][0])
    G = hb.G
    img = _image_of(pkg, hb, L)
    cap = img.stride - abi.LOG_HDR_BYTES
    bad_g = [G // 2, G - 1]
    hdr = img.header()
    for g in bad_g:
        hdr[g, 7] = cap + 8                                   # len: above capacity, below the stride
    img.images[:, :64] = hdr.view(torch.uint8).view(G, 64)
    before = img.images.clone()
    d_ent = torch.from_numpy(ent.view(np.uint8).copy()).cuda()
    d_pay = torch.from_numpy(payload).cuda()
    d_n = torch.from_numpy(n_entries.view(np.int32).copy()).cuda()
    eng.stats_reset()
    out = eng.log_append_entry(img, d_ent, d_pay, M, n_entries=d_n)
    idx, last, bad = orc.append(hb, ent, payload, M, n_entries=n_entries)
    torch.cuda.synchronize()
    assert int(eng.stats()[abi.STAT_CORRUPT]) == bad + int((n_entries[bad_g] > 0).sum())
    ok = np.setdiff1d(np.arange(G), bad_g)
    got_idx = out["idx"].cpu().numpy().view(np.uint64).reshape(G, -1)
    assert np.array_equal(got_idx[ok], idx.reshape(G, -1)[ok])
    assert not got_idx[bad_g].any()
    for g in bad_g:                                           # the corrupt images are untouched
        assert torch.equal(img.images[g], before[g]), g
    rings = img.download("ring")
    assert np.array_equal(rings[ok], hb.ring.reshape(G, hb.stride)[ok, :L])
    st = img.download("state")
    for k in ("head", "apply", "commit", "end", "tail"):
        assert np.array_equal(st[k][ok], hb.state[k][ok]), k
    # the commit walk: CORRUPT for those groups (0xFF), the oracle elsewhere
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM
    for impl in (0, abi.BATCH_LANE_IMPL, abi.BATCH_SHORT_WALKS):
        b = img.struct()
        b.flags |= impl
        eng.stats_reset()
        co = eng.update_remote_logs(img, flags, bstruct=b)
        torch.cuda.synchronize()
        ref = orc.commit(hb, flags)
        cm = co["committed"].cpu().numpy()
        assert (cm[bad_g] == 0xFF).all(), impl
        assert np.array_equal(cm[ok], ref["committed"][ok]), impl
        assert np.array_equal(_u64(co["new_commit"])[ok], ref["new_commit"][ok]), impl
        assert np.array_equal(co["digest"].cpu().numpy().view(np.uint32)[ok], ref["digest"][ok]), impl
        assert int(eng.stats()[abi.STAT_CORRUPT]) == len(bad_g), impl
    # the readers stay in bounds (their results for the corrupt groups are not the reference's)
    po = eng.log_pruning(img)
    dets, ln = eng.log_entries_to_nc_buf(img, 64)
    torch.cuda.synchronize()
    rp, _ = orc.prune(hb)
    assert np.array_equal(_u64(po["new_head"])[ok], rp["new_head"][ok])
    rd, rl = orc.nc_build(hb, 64)
    assert np.array_equal(ln.cpu().numpy().view(np.uint32)[ok], rl[ok])
