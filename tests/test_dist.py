"""N>1 path on CPU: two or four gloo ranks each own a contiguous gid shard (gid_base =
rank * G, rdma-paxos_amd/shard.py), run the hot path on it (the oracle stands in
for the device here: no GPU in this suite) and all-reduce the batch statistics
with the SUM/MIN semantics of apus_stats_allreduce.  The sharded result must
equal one process running the unsharded (world x G)-group batch: per-group outputs
concatenate to the same arrays, and the reduced stats (decisions, committed
entries, advanced groups, global pruning watermark) are identical.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

G, R = 96, 3
KW = dict(seed=77, n_entries=24, n_history=6, len_min=16, len_max=200, ring_len=12000, straggler=True,
          type_mix=True, p_full_ack=0.7)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_shard(orc, pkg, gid_base, n):
    abi = pkg.abi
    hb = orc.host_batch(n, R, KW["ring_len"])
    orc.gen(hb, pkg.batch.gen_cfg(gid_base=gid_base, **KW))
    c = orc.commit(hb, abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN)
    v = orc.vote(hb)
    p, wm = orc.prune(hb)
    # log_adjustment on the shard: every server's step a function
    # of its global id, NC buffers = the group's own determinants
    gid = np.arange(gid_base, gid_base + n, dtype=np.int64)
    hb.lr_step[:] = ((gid[:, None] * R + np.arange(R)[None, :]) % 6 + 1).reshape(-1).astype(np.uint8)
    M = 32
    dets, dl = orc.nc_build(hb, M)
    nc = np.repeat(np.asarray(dets).view(pkg.batch.DET_DT).reshape(n, 1, M), R, axis=1).reshape(-1)
    io = orc.lr_io(n, R, M, send_flag=np.ones(n * R, np.uint8), nc_len=np.repeat(np.asarray(dl), R),
                   nc_dets=nc, ssn=gid.astype(np.uint64))
    orc.log_adjust(hb, io)
    st = np.zeros(abi.STAT_COUNT, np.uint64)
    st[abi.STAT_DECISIONS] = n
    st[abi.STAT_COMMITTED] = c["n_entries"].sum()
    st[abi.STAT_ADVANCED] = c["committed"].sum()
    st[abi.STAT_VOTES_WON] = v["won"].sum()
    st[abi.STAT_MIN_WATERMARK] = wm
    outs = {"commit": c["new_commit"], "digest": c["digest"], "median": c["median"], "won": v["won"],
            "new_head": p["new_head"], "lr_post": io["post"], "lr_step": hb.lr_step.copy(),
            "lr_remote_end": hb.remote_end.copy(), "lr_commit": hb.state["commit"].copy(), "lr_ssn": io["ssn"]}
    return st, outs


def _worker(rank, world, port, resdir):
    import torch.distributed as dist

    import apus_pkg
    pkg, orc = apus_pkg.load_package(), apus_pkg.load_oracle()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        base, n = pkg.shard.gid_range(rank, G)
        st, outs = _run_shard(orc, pkg, base, n)
        red = pkg.shard.allreduce_stats(st)
        np.savez(os.path.join(resdir, f"r{rank}.npz"), stats=red, **outs)
    finally:
        dist.destroy_process_group()


def test_gid_range_and_combine(pkg):
    assert pkg.shard.gid_range(3, 1000) == (3000, 1000)
    a = np.array([1, 2, 3, 4, 5, 6, 100, 1, 5], np.uint64)
    b = np.array([10, 20, 30, 40, 50, 60, 7, 2, 6], np.uint64)
    c = np.array([0, 0, 0, 0, 0, 0, 2 ** 64 - 1, 0, 0], np.uint64)
    got = pkg.shard.combine([a, b, c])
    assert list(got[:6]) == [11, 22, 33, 44, 55, 66] and got[6] == 7 and got[7] == 3 and got[8] == 11


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_gloo_shards_equal_unsharded(tmp_path, orc, pkg, world):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    full_st, full = _run_shard(orc, pkg, 0, G * world)
    for r in range(world):
        assert np.array_equal(res[r]["stats"], full_st), (r, res[r]["stats"], full_st)
    for k in full:
        assert np.array_equal(np.concatenate([res[r][k] for r in range(world)]), full[k]), k
    assert full_st[pkg.abi.STAT_MIN_WATERMARK] != np.uint64(2 ** 64 - 1)


@pytest.mark.gpu
@pytest.mark.timeout(120)
def test_gpu_rccl_stats_allreduce_world1(pkg, orc):
    """bench.py's N>1 plumbing on one GPU: torch's RCCL process group, the
    unique id broadcast, libapus_gpu's own communicator (apus_comm_init_rank)
    and apus_stats_allreduce over it.  With one rank SUM and MIN are the
    identity, so the all-reduced statistics equal the local ones."""
    import ctypes as C

    import torch
    import torch.distributed as dist
    abi = pkg.abi
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        eng = pkg.Engine(0)
        lib = eng.lib
        uid = C.create_string_buffer(128)
        abi.check(lib.apus_comm_get_unique_id(uid), "apus_comm_get_unique_id")
        obj = [bytes(uid.raw)]
        dist.broadcast_object_list(obj, src=0)
        abi.check(lib.apus_comm_init_rank(eng.ctx, 1, C.create_string_buffer(obj[0], 128), 0),
                  "apus_comm_init_rank")
        n = 512
        db = pkg.batch.DeviceBatch(n, R, pkg.batch.ring_stride_for(KW["ring_len"]))
        cfg = pkg.batch.gen_cfg(**KW)
        eng.gen(db, cfg)
        eng.stats_reset()
        eng.update_remote_logs(db, abi.COMMIT_WALK | abi.COMMIT_CHECKSUM)
        eng.log_pruning(db)
        torch.cuda.synchronize()
        before = np.array(eng.stats(), np.uint64)
        s = torch.cuda.current_stream()
        abi.check(lib.apus_stats_allreduce(eng.ctx, C.c_void_p(s.cuda_stream)), "apus_stats_allreduce")
        torch.cuda.synchronize()
        after = np.array(eng.stats(), np.uint64)
        assert np.array_equal(before, after)
        # SURVEY 8(b)'s name for the same call
        abi.check(lib.apus_allreduce_stats(eng.ctx, C.c_void_p(s.cuda_stream)), "apus_allreduce_stats")
        torch.cuda.synchronize()
        assert np.array_equal(before, np.array(eng.stats(), np.uint64))
        assert int(after[abi.STAT_DECISIONS]) == n
        hb = orc.host_batch(n, R, KW["ring_len"])
        orc.gen(hb, cfg)
        c = orc.commit(hb, abi.COMMIT_WALK | abi.COMMIT_CHECKSUM)
        assert int(after[abi.STAT_COMMITTED]) == int(c["n_entries"].sum())
        eng.close()
    finally:
        dist.destroy_process_group()
