"""Context hygiene: one context on several
streams at once, scalar drop-ins from several threads at once, a caller
stream honoured by the engine's uploads and read-backs, and the scalar
drop-ins' host registration re-validated when a log at the same address
grows.  Every result is compared with the CPU oracle."""
import ctypes as C

import numpy as np
import pytest
from conftest import host_pool, keep_host

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


def _ref_log(pkg, hb, g, pad=64):
    abi = pkg.abi
    st = hb.state[g]
    ln = int(st["len"])
    hdr = C.sizeof(abi.LogHeader)
    buf = keep_host(np.zeros(hdr + ln + pad, np.uint8))
    log = abi.LogHeader.from_buffer(buf)
    for k in ("head", "apply", "commit", "end", "tail", "len"):
        setattr(log, k, int(st[k]))
    buf[hdr:hdr + ln] = hb.group_ring(g)[:ln]
    cfg = abi.ServerConfig()
    C.memmove(C.addressof(cfg.cid), hb.state[g:g + 1].tobytes()[48:64], 16)
    cfg.idx = int(hb.self_idx[g])
    return buf, log, cfg


def test_scalar_dropins_from_threads(pkg, orc, eng):
    """apus_commit_reply_walk from 6 threads at once (ctypes drops the GIL):
    the scalar scratch is serialised, every answer is the oracle's"""
    abi = pkg.abi
    lib = abi.load_library()
    G, R, L = 48, 5, 4096
    cfg = pkg.batch.gen_cfg(seed=77, n_entries=20, n_history=4, len_min=0, len_max=90, ring_len=L,
                            type_mix=True, cid_mix=True, self_random=True, p_full_ack=0.5)
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, cfg)
    ref = orc.commit(hb, abi.COMMIT_WALK)
    logs = [_ref_log(pkg, hb, g) for g in range(G)]
    errors = []

    def worker(t):
        try:
            for rep in range(4):
                for g in range(t, G, 6):
                    buf, _, scfg = logs[g]
                    nc, cm = C.c_uint64(0), C.c_int(0)
                    assert lib.apus_commit_reply_walk(C.c_void_p(buf.ctypes.data), C.byref(scfg), C.byref(nc),
                                                      C.byref(cm)) == 0
                    assert nc.value == ref["new_commit"][g] and cm.value == ref["committed"][g], g
        except Exception as e:          # noqa: BLE001 -- reported below
            errors.append(e)
    # the worker threads live for the whole session (conftest.host_pool): each
    # thread that calls into HIP gets per-thread runtime state, and the runs
    # whose next test faulted on its first host-to-device copies had just
    # seen these threads exit
    pool = host_pool(6)
    for f in [pool.submit(worker, t) for t in range(6)]:
        f.result()
    for buf, _, _ in logs:
        lib.apus_host_unregister(C.c_void_p(buf.ctypes.data))
    assert not errors, errors[0]


def test_scalar_registration_grows_with_len(pkg, orc, eng):
    """a log whose ring grows at the same address (a new dare_log_t in the
    same allocation) is registered afresh: the walk reads the whole new ring"""
    abi = pkg.abi
    lib = abi.load_library()
    R = 3
    small = orc.host_batch(1, R, 2048)
    orc.gen(small, pkg.batch.gen_cfg(seed=5, n_entries=8, n_history=2, len_min=64, len_max=64, ring_len=2048))
    big = orc.host_batch(1, R, 65536)
    orc.gen(big, pkg.batch.gen_cfg(seed=6, n_entries=150, n_history=50, len_min=64, len_max=200,
                                   ring_len=65536, p_full_ack=1.0))
    hdr = C.sizeof(abi.LogHeader)
    buf = keep_host(np.zeros(hdr + 65536 + 64, np.uint8))
    for hb in (small, big):
        st = hb.state[0]
        ln = int(st["len"])
        log = abi.LogHeader.from_buffer(buf)
        for k in ("head", "apply", "commit", "end", "tail", "len"):
            setattr(log, k, int(st[k]))
        buf[hdr:hdr + ln] = hb.group_ring(0)[:ln]
        cfg = abi.ServerConfig()
        C.memmove(C.addressof(cfg.cid), hb.state[0:1].tobytes()[48:64], 16)
        cfg.idx = int(hb.self_idx[0])
        nc, cm = C.c_uint64(0), C.c_int(0)
        assert lib.apus_commit_reply_walk(C.c_void_p(buf.ctypes.data), C.byref(cfg), C.byref(nc), C.byref(cm)) == 0
        ref = orc.commit(hb, abi.COMMIT_WALK)
        assert nc.value == ref["new_commit"][0] and cm.value == ref["committed"][0]
    assert lib.apus_host_register(C.c_void_p(buf.ctypes.data)) == 0
    assert lib.apus_host_unregister(C.c_void_p(buf.ctypes.data)) == 0


def test_scalar_logs_sharing_a_page(pkg, orc, eng):
    """two dare_log_t images carved out of one allocation so that the last
    page of the first is the first page of the second.  The runtime pins and
    maps whole pages: the library never holds both registrations at once
    (mapping a page twice, then unmapping it with one of them, would leave
    the other log's ring partly unmapped on the GPU).  Walks alternate
    between the logs, one log is unregistered while the other is in use, and
    every answer is the oracle's."""
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
    arena = keep_host(np.zeros(2 * span + 3 * 4096, np.uint8))
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
        cfg = abi.ServerConfig()
        C.memmove(C.addressof(cfg.cid), hb.state[0:1].tobytes()[48:64], 16)
        cfg.idx = int(hb.self_idx[0])
        logs.append((C.c_void_p(arena.ctypes.data + at), cfg, orc.commit(hb, abi.COMMIT_WALK)))

    def walk(k):
        p, cfg, ref = logs[k]
        nc, cm = C.c_uint64(0), C.c_int(0)
        assert lib.apus_commit_reply_walk(p, C.byref(cfg), C.byref(nc), C.byref(cm)) == 0
        assert nc.value == ref["new_commit"][0] and cm.value == ref["committed"][0], k
    for k in (0, 1, 0, 1, 1, 0):
        walk(k)
    assert lib.apus_host_register(logs[1][0]) == 0     # takes the shared page from log 0
    lib.apus_host_unregister(logs[0][0])               # no longer registered: nothing to release
    walk(1)
    walk(0)
    for p, _, _ in logs:
        lib.apus_host_unregister(p)
