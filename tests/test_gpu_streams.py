"""Context hygiene: one
context on several streams at once, scalar drop-ins from short-lived threads
at once, a caller stream honoured by the engine's uploads and read-backs, and
the scalar drop-ins' two ring paths -- a caller heap log (staged) reused with
a longer ring, logs sharing a page, and apus_log_new logs read in place.
Every result is compared with the CPU oracle."""
import ctypes as C
import threading

import numpy as np
import pytest
from conftest import ScalarLog

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _batch(pkg, orc, eng, G, R, seed, L=16384, **kw):
    cfg = pkg.batch.gen_cfg(seed=seed, n_entries=64, n_history=16, len_min=64, len_max=64, ring_len=L,
                            straggler=True, p_full_ack=0.8, **kw)
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, cfg)
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, cfg)
    return db, hb


def test_one_context_two_streams(pkg, orc, eng):
    """commit + checksum + median and pruning of two batches issued on two
    streams of one context, interleaved; each stream's scratch is its own,
    the shared statistics hold the sum over both batches"""
    import torch
    abi = pkg.abi
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN
    G = 1 << 16
    dbs, hbs = zip(*[_batch(pkg, orc, eng, G, 3 + 2 * k, 300 + k, self_random=True) for k in range(2)])
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    eng.stats_reset()
    torch.cuda.synchronize()
    outs, pouts = [None, None], [None, None]
    for rep in range(3):                       # several launches in flight per stream
        for k in range(2):
            outs[k] = eng.update_remote_logs(dbs[k], flags, stream=streams[k])
            pouts[k] = eng.log_pruning(dbs[k], stream=streams[k])
    torch.cuda.synchronize()
    for k in range(2):
        ref = orc.commit(hbs[k], flags)
        assert np.array_equal(outs[k]["new_commit"].cpu().numpy().view(np.uint64), ref["new_commit"])
        assert np.array_equal(outs[k]["digest"].cpu().numpy().view(np.uint32), ref["digest"])
        assert np.array_equal(outs[k]["median"].cpu().numpy().view(np.uint64), ref["median"])
        rp, _ = orc.prune(hbs[k])
        assert np.array_equal(pouts[k]["new_head"].cpu().numpy().view(np.uint64), rp["new_head"])
    st = eng.stats()
    assert st[abi.STAT_DECISIONS] == 3 * 2 * G
    exp = sum(int(orc.commit(h, flags)["n_entries"].sum()) for h in hbs)
    assert st[abi.STAT_COMMITTED] == 3 * exp


def test_engine_honours_caller_stream(pkg, orc, eng):
    """log_adjustment / completion with a non-default stream: uploads,
    launches and read-backs all ordered on it"""
    import torch
    from test_lr_step import _clone_io, build
    hb, io = build(pkg, orc, "r5_mix")
    db = pkg.batch.DeviceBatch(hb.G, hb.R, hb.stride)
    db.upload(hb)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    dio = _clone_io(io)
    for _ in range(3):
        dio = eng.log_adjustment(db, dio, stream=s)
        orc.log_adjust(hb, io)
        dio["wc"] = np.where(io["post"] != 0, 1, 0).astype(np.uint8)
        io["wc"][:] = dio["wc"]
        dio = eng.handle_lr_work_completion(db, dio, stream=s)
        orc.lr_completion(hb, io)
        for k in ("send_flag", "send_count", "ssn", "post"):
            assert np.array_equal(dio[k], io[k]), k
    s.synchronize()
    for k in ("state", "lr_step", "remote_commit", "remote_end"):
        assert np.array_equal(db.download(k), getattr(hb, k)), k


def test_engine_requires_max_dets(pkg, orc, eng):
    from test_lr_step import build
    hb, io = build(pkg, orc, "r3_wrap")
    db = pkg.batch.DeviceBatch(hb.G, hb.R, hb.stride)
    db.upload(hb)
    io.pop("max_dets")
    with pytest.raises(KeyError):
        eng.log_adjustment(db, io)


def _cfg_of(pkg, hb, g):
    cfg = pkg.abi.ServerConfig()
    C.memmove(C.addressof(cfg.cid), hb.state[g:g + 1].tobytes()[48:64], 16)
    cfg.idx = int(hb.self_idx[g])
    return cfg


def _walk(lib, p, cfg):
    nc, cm = C.c_uint64(0), C.c_int(0)
    assert lib.apus_commit_reply_walk(p, C.byref(cfg), C.byref(nc), C.byref(cm)) == 0
    return nc.value, cm.value


def _path_stats(lib):
    a, b, n = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
    assert lib.apus_scalar_path_stats(C.byref(a), C.byref(b), C.byref(n), None) == 0
    return a.value, b.value, n.value


@pytest.mark.parametrize("mode", ["heap", "owned"])
def test_scalar_dropins_from_threads(pkg, orc, eng, mode):
    """apus_commit_reply_walk from 6 plain threads at once (ctypes drops the
    GIL), which then exit: the scalar scratch is serialised, every answer is
    the oracle's.  Heap logs are staged, apus_log_new logs read in place."""
    abi = pkg.abi
    lib = abi.load_library()
    G, R, L = 48, 5, 4096
    cfg = pkg.batch.gen_cfg(seed=77, n_entries=20, n_history=4, len_min=0, len_max=90, ring_len=L,
                            type_mix=True, cid_mix=True, self_random=True, p_full_ack=0.5)
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, cfg)
    ref = orc.commit(hb, abi.COMMIT_WALK)
    logs = [ScalarLog(pkg, L, mode).load(hb, g) for g in range(G)]
    cfgs = [_cfg_of(pkg, hb, g) for g in range(G)]
    errors = []
    before = _path_stats(lib)

    def worker(t):
        try:
            for rep in range(4):
                for g in range(t, G, 6):
                    assert _walk(lib, logs[g].ptr, cfgs[g]) == (ref["new_commit"][g], ref["committed"][g]), g
        except Exception as e:          # noqa: BLE001 -- reported below
            errors.append(e)
    threads = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    after = _path_stats(lib)
    for lg in logs:
        lg.free()
    assert not errors, errors[0]
    k = 0 if mode == "owned" else 1
    assert after[k] - before[k] == 4 * G and after[1 - k] == before[1 - k]


def test_scalar_log_reused_with_longer_ring(pkg, orc, eng):
    """one caller buffer holding first a small log, then a log with a 32x
    longer ring: the staging image grows and the walk reads the new ring"""
    abi = pkg.abi
    lib = abi.load_library()
    R = 3
    small = orc.host_batch(1, R, 2048)
    orc.gen(small, pkg.batch.gen_cfg(seed=5, n_entries=8, n_history=2, len_min=64, len_max=64, ring_len=2048))
    big = orc.host_batch(1, R, 65536)
    orc.gen(big, pkg.batch.gen_cfg(seed=6, n_entries=150, n_history=50, len_min=64, len_max=200,
                                   ring_len=65536, p_full_ack=1.0))
    hdr = C.sizeof(abi.LogHeader)
    buf = np.zeros(hdr + 65536 + 64, np.uint8)
    for hb in (small, big):
        st = hb.state[0]
        ln = int(st["len"])
        log = abi.LogHeader.from_buffer(buf)
        for k in ("head", "apply", "commit", "end", "tail", "len"):
            setattr(log, k, int(st[k]))
        buf[hdr:hdr + ln] = hb.group_ring(0)[:ln]
        ref = orc.commit(hb, abi.COMMIT_WALK)
        assert _walk(lib, C.c_void_p(buf.ctypes.data), _cfg_of(pkg, hb, 0)) == (ref["new_commit"][0],
                                                                                  ref["committed"][0])


def test_scalar_logs_sharing_a_page(pkg, orc, eng):
    """two dare_log_t images carved out of one allocation so that the last
    page of the first is the first page of the second, walked alternately,
    then the allocation is freed and reused: the library maps none of it
    (it stages the bytes a call reads), so nothing is left mapped"""
    abi = pkg.abi
    lib = abi.load_library()
    R, L = 3, 4096
    hdr = C.sizeof(abi.LogHeader)
    hbs = []
    for seed in (41, 42):
        hb = orc.host_batch(1, R, L)
        orc.gen(hb, pkg.batch.gen_cfg(seed=seed, n_entries=20, n_history=6, len_min=0, len_max=60, ring_len=L,
                                      p_full_ack=0.8, straggler=True))
        hbs.append(hb)
    span = hdr + L
    for rep in range(2):
        arena = np.zeros(2 * span + 3 * 4096, np.uint8)
        a0 = (-arena.ctypes.data) % 4096 + 100            # log 0 starts 100 B into a page
        a1 = a0 + span + 8                                # log 1 starts in log 0's last page
        assert (arena.ctypes.data + a0 + span - 1) // 4096 == (arena.ctypes.data + a1) // 4096
        logs = []
        for hb, at in zip(hbs, (a0, a1)):
            st = hb.state[0]
            log = abi.LogHeader.from_buffer(arena, at)
            for k in ("head", "apply", "commit", "end", "tail", "len"):
                setattr(log, k, int(st[k]))
            arena[at + hdr:at + hdr + L] = hb.group_ring(0)[:L]
            logs.append((C.c_void_p(arena.ctypes.data + at), _cfg_of(pkg, hb, 0), orc.commit(hb, abi.COMMIT_WALK)))
        for k in (0, 1, 0, 1, 1, 0):
            p, cfg, ref = logs[k]
            assert _walk(lib, p, cfg) == (ref["new_commit"][0], ref["committed"][0]), k
        del logs, arena                                   # freed while the next round allocates


def test_log_new_in_place(pkg, orc, eng):
    """apus_log_new is log_new (dare_log.h:120-137) in pinned, mapped memory:
    the walk reads it in place, so a follower's reply[] byte written into the
    host log after a call is seen by the next call, as an RDMA write into the
    reference's registered log is; apus_log_free refuses foreign pointers"""
    abi = pkg.abi
    lib = abi.load_library()
    R, L = 3, 8192
    hb = orc.host_batch(1, R, L)
    orc.gen(hb, pkg.batch.gen_cfg(seed=9, n_entries=24, n_history=4, len_min=64, len_max=64, ring_len=L,
                                  p_full_ack=0.0, straggler=False))
    lg = ScalarLog(pkg, L, "owned").load(hb, 0)
    cfg = _cfg_of(pkg, hb, 0)
    try:
        ref = orc.commit(hb, abi.COMMIT_WALK)
        got = _walk(lib, lg.ptr, cfg)
        assert got == (ref["new_commit"][0], ref["committed"][0])
        # ack every uncommitted entry from every replica, in the host image and in hb
        dets, ln = orc.nc_build(hb, 1024)
        for e in range(int(ln[0])):
            off = int(dets[3 * e + 2])
            for i in range(R):
                lg.buf[lg.hdr + off + 28 + i] = 1
                hb.group_ring(0)[off + 28 + i] = 1
        ref2 = orc.commit(hb, abi.COMMIT_WALK)
        assert ref2["new_commit"][0] != ref["new_commit"][0] or int(ln[0]) == 0
        assert _walk(lib, lg.ptr, cfg) == (ref2["new_commit"][0], ref2["committed"][0])
    finally:
        lg.free()
    junk = np.zeros(64, np.uint8)
    assert lib.apus_log_free(C.c_void_p(junk.ctypes.data)) == abi.APUS_INSUCCESS
    p = C.c_void_p()
    assert lib.apus_log_new(16, C.byref(p)) == abi.APUS_ERROR       # shorter than one entry header


def test_more_streams_than_scratch_slots(pkg, orc, eng):
    """launches on 24 distinct streams in turn (the context keeps
    scratch for 16): the 17th and later take over the least recently used
    stream's scratch, and every result is the oracle's"""
    import torch
    abi = pkg.abi
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM
    db, hb = _batch(pkg, orc, eng, 4096, 3, 910)
    torch.cuda.synchronize()
    ref = orc.commit(hb, flags)
    streams = [torch.cuda.Stream() for _ in range(24)]
    eng.stats_reset()
    torch.cuda.synchronize()
    outs = []
    for rep in range(2):
        for s in streams:
            outs.append(eng.update_remote_logs(db, flags, stream=s))
    torch.cuda.synchronize()
    for out in outs:
        assert np.array_equal(out["new_commit"].cpu().numpy().view(np.uint64), ref["new_commit"])
        assert np.array_equal(out["digest"].cpu().numpy().view(np.uint32), ref["digest"])
    assert eng.stats()[abi.STAT_DECISIONS] == 48 * 4096
