"""Benchmark: quorum commit decisions/s + achieved HBM GB/s on MI355X.

Workload (BASELINE.json configs[1], "c2"): per GPU 2^20 independent consensus
groups x 3 replicas, 64-entry batches of 64-byte Redis SET entries (128 B per
entry), commit index + checksum.  A step is one pass of the hot path over the
batch resident in HBM:
  1. commit walk + Adler-32 checksum (fused, one wave per group)   [dominant]
  2. DARE median-offset quorum (one lane per group)
  3. update_remote_logs' lazy remote-commit publish (dare_ibv_rc.c:1760-1822)
  4. log-pruning minimum + global watermark (one lane per group)
  5. N > 1: RCCL all-reduce of the per-batch statistics (SUM) and of the
     pruning watermark (MIN) over xGMI
(2-4 run in the commit call's one tail launch.)
Groups are sharded by id across ranks (weak scaling, no data-path exchange).

`--workload c4` runs BASELINE configs[3]'s per-GPU shard instead (2^23 groups
x 5 replicas, same entries, log_pruning's minimum and watermark each batch); `--workload c4_1gpu` the whole 64M-group batch on
one GPU (2^26 groups x 5 replicas, 16 entries of 128 B: commit_seg_kernel).  `--workload c3` runs one wave of BASELINE
configs[2] (2^19 groups x 5 replicas, 64 entries of 128 B - 4,160 B, one
straggler follower): the step adds the followers' (idx, term) validation, and
the commit walk runs with the APUS_BATCH_VAR_LEN hint (hop walk).
`--workload c3_full` walks configs[2]'s whole 10M-group batch as 20
consecutive resident waves of 2^19 groups (each generated outside the timed
region); its step is one pass over all of them.  `--workload c5` runs configs[4]'s per-GPU shard (2^23 groups x
7 replicas, 16-entry batches, STABLE / EXTENDED / TRANSIT configurations): the
step adds the failover pass (vote tally, local (idx, term), vote-request
ranking on the 40-B vote_req_t records) and the election-win transition
(apus_vote_win_batch: the groups whose candidate won become leaders -- on the
first step; the cold step is timed on its own and reported under "failover").

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       N > 1: one rank per GPU.  Under torch.distributed.run (WORLD_SIZE set)
       the world must equal N; run directly, bench.py starts
       torch.distributed.run --nproc-per-node N itself (a child process,
       before anything touches the GPU) and exits with its status.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md)
WORKLOADS = {
    "c2": dict(G=1 << 20, R=3, E=64, H=16, L=64, ring=16384),
    # configs[3]: the pruning configuration -- log_pruning's minimum and the
    # cross-GPU watermark each batch (force_log_pruning runs after
    # apply_committed_entries in polling(), dare_server.c:1100-1123: never
    # beside the walk, apus_commit_batch)
    "c4": dict(G=1 << 23, R=5, E=64, H=16, L=64, ring=16384),
    # configs[2]: one resident wave (2^19 groups) of the 10M-group batch; the
    # 16 committed history entries carry commands of at most 64 B (Hmax), so
    # the 272,960-B ring holds the worst-case batch of 64 x 4,160 B + a wrap
    # gap (143 GB resident).  c3_full walks the whole 10M groups as 20 waves
    "c3": dict(G=1 << 19, R=5, E=64, H=16, Hmax=64, L=64, Lmax=4096, ring=272960, var_len=True),
    "c3_full": dict(G=1 << 19, total=10_000_000, wave=1 << 19, R=5, E=64, H=16, Hmax=64, L=64, Lmax=4096,
                    ring=272960, var_len=True),
    # north_star's ">= 64M groups per batch ... on 1 GPU" (SURVEY 8d C4, 1-GPU
    # point): 2^26 groups x 5 replicas, 16-entry batches after 2 history
    # entries on the smallest ring the generator accepts (2,448 B: 18 entries
    # of 128 B + a wrap gap), 165 GB of rings; short walks, four groups per wave
    "c4_1gpu": dict(G=1 << 26, R=5, E=16, H=2, L=64, ring=2448, short=True),
    # configs[4]: the per-GPU shard of 64M 7-replica groups
    # over 8 GPUs, 16-entry batches, 60% STABLE / 20% EXTENDED / 20% TRANSIT
    # configurations (joint old/new quorum), vote acks p=0.6; the step adds
    # the failover pass: vote tally (a5), each log's local (idx, term) and the
    # vote-request ranking (a6), then the election-win transition
    "c5": dict(G=1 << 23, R=7, E=16, H=16, L=64, ring=8192, short=True, cid_mix=True, votes=True, win=True),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2", choices=list(WORKLOADS))
    ap.add_argument("--groups", type=int, default=0, help="override groups per GPU")
    ap.add_argument("--impl", default="wave", choices=["wave", "lane"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--vote-sit", action="store_true",
                    help="A/B only: C5's ranking on packed (sid, index, term) rows derived from the 40-B vote_req "
                         "records outside the timed region (apus_batch_t.vote_sit) instead of the records")
    ap.add_argument("--no-win", action="store_true",
                    help="A/B only (c5): the step without the election-win transition call")
    ap.add_argument("--round4-tail", action="store_true",
                    help="A/B only: the round-4 tail (median + log_pruning; no publish, no force_log_pruning)")
    ap.add_argument("--tail-rows", action="store_true",
                    help="the commit tail eight lanes per group (APUS_BATCH_TAIL_ROWS, the A/B of the lane form)")
    ap.add_argument("--split", action="store_true",
                    help="A/B only: the round-2 step (stats reset, walk call, median call, pruning call)")
    ap.add_argument("--failover-calls", action="store_true",
                    help="A/B only (c5): the round-3 step (vote tally and ranking as their own calls after the "
                         "commit call)")
    ap.add_argument("--rccl", action="store_true",
                    help="run the N > 1 path (RCCL process group and all-reduce) even at N = 1 (a rehearsal)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--traffic", default=None, help="PMC traffic summary (default profiles/traffic_commit_<workload>.json)")
    return ap.parse_args()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launcher_cmd(argv, n, port):
    """the torch.distributed.run command line that runs this script on n
    ranks of one node (argv: this process's arguments, --gpus included)"""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def world_plan(gpus, env):
    """('launch', n): start n ranks; ('run', world): this process is a rank.
    Refuses (ValueError) a world that differs from --gpus."""
    if gpus < 1:
        raise ValueError(f"--gpus {gpus}: need at least 1")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return ("launch", gpus) if gpus > 1 else ("run", 1)
    if int(ws) != gpus:
        raise ValueError(f"WORLD_SIZE={ws} but --gpus {gpus}: one rank per GPU")
    return ("run", int(ws))


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def cpu_baseline(pkg, wl, seconds):
    """The GPU step's work on the host cores, over a bounded sample of the
    workload (same trace generator, same per-group work: commit walk + the
    build-defined Adler-32 + median + remote-commit publish + pruning minimum;
    C3: + the followers' (idx, term) validation; C5: + vote tally + local
    (idx, term) + vote-request ranking).

    value (kind "reference"): the reference's own code -- oracle/_ref, the
    reference's dare_log.h compiled from its sources with the transcribed
    loop bodies of dare_ibv_rc.c / dare_server.c on top (ref_compose.c,
    drift-checked) -- over per-group dare_log_t images in the reference's
    shapes (server_t, ctrl_data), -O2, OpenMP static partition over every
    thread this process may use: the CPUs in its affinity mask, capped by the
    CPU share the box allots (OMP_NUM_THREADS: 16 per GPU on the GPU pool).
    legs: the same at 1 thread (-O2 and -O0, the level the reference builds at,
    target/src/dare/subdir.mk) and without the checksum (the reference has
    none); the clean-room restatement (oracle/apus_oracle.c, kind "port") at
    the same thread count and at 1 thread; the cache-hot per-group cost of walk
    + median + pruning minimum on both; the host's DRAM read bandwidth.
    Without the _ref build (the reference tree absent where it was built) the
    port's figure is the value (kind "port")."""
    import apus_pkg
    orc = apus_pkg.load_oracle()
    abi = pkg.abi
    aff = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(aff, share) if share > 0 else aff)
    S = max(1024, min(65536, (2 << 30) // wl["ring"]))      # at most ~2 GiB of host rings
    lmax = wl.get("Lmax", wl["L"])
    cfg = pkg.batch.gen_cfg(seed=2026, n_entries=wl["E"], n_history=wl["H"], len_min=wl["L"], len_max=lmax,
                            ring_len=wl["ring"], p_full_ack=0.9, straggler=True, cid_mix=wl.get("cid_mix", False),
                            p_vote_ack=0.6, hist_len_max=wl.get("Hmax", 0))
    var_len, votes = wl.get("var_len", False), wl.get("votes", False)
    # remote_commit: the publish (and the validation's empty-buffer rule)
    fields = ["state", "self_idx", "remote_end", "remote_commit", "lr_step", "fail_count", "apply_offsets",
              "prev_head", "abs_base"]
    if votes:
        fields += ["vote_ack", "vote_req", "hb", "sid"]
    hb = orc.host_batch(S, wl["R"], wl["ring"], fields=fields)
    orc.gen(hb, cfg, threads)
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM | abi.COMMIT_MEDIAN | abi.COMMIT_PUBLISH
    # the GPU step's other legs: C3's validation of R - 1 followers' NC
    # buffers (each the leader's determinants, truncated and with the term
    # changed from a random entry on: oracle gen_nc); C5's vote tally and
    # local (idx, term) + vote-request ranking
    nc = None
    if var_len:
        F, M = wl["R"] - 1, wl["E"]
        nc = orc.gen_nc(hb, cfg, F, M) + (F, M)

    def timed(fn, secs):
        fn(1)                                  # untimed: first touch of the sample
        t1 = fn(1)
        reps = max(1, int(secs / max(t1, 1e-6)))
        t = fn(reps)
        return S * reps / t, reps, t

    def port(th, opt="O2"):
        return lambda reps: orc.time_step(hb, flags, reps, th, opt, votes=votes, nc=nc)

    legs = {}
    kind, v, reps, t = "port", None, 0, 0.0
    rb = orc.RefBench(hb, "O2", nc=nc)
    if rb.ok:
        _, d0 = rb.time(1, threads)
        port_d0 = int(orc.commit(hb, abi.COMMIT_WALK | abi.COMMIT_CHECKSUM)["digest"][0])
        assert d0 == port_d0, ("reference-composed and restated checksums differ", d0, port_d0)
        kind = "reference"
        v, reps, t = timed(lambda r: rb.time(r, threads)[0], seconds * 0.45)
        legs["ref_O2_1thread"] = timed(lambda r: rb.time(r, 1)[0], seconds * 0.08)[0]
        legs[f"ref_O2_{threads}thread_no_checksum"] = timed(lambda r: rb.time(r, threads, False)[0], seconds * 0.05)[0]
        rb.close()
        r0 = orc.RefBench(hb, "O0", nc=nc)
        legs["ref_O0_1thread"] = timed(lambda r: r0.time(r, 1)[0], seconds * 0.08)[0]
        legs[f"ref_O0_{threads}thread"] = timed(lambda r: r0.time(r, threads)[0], seconds * 0.05)[0]
        r0.close()
        pv, preps, pt = timed(port(threads), seconds * 0.1)
        legs[f"port_O2_{threads}thread"] = pv
    else:
        v, reps, t = timed(port(threads), seconds * 0.6)
    legs["port_O2_1thread"] = timed(port(1), seconds * 0.06)[0]
    legs["port_O0_1thread"] = timed(port(1, "O0"), seconds * 0.06)[0]
    sample_g = list(range(0, S, S // 64))
    for side, name in ((False, "port"), (True, "ref")):
        for opt in ("O2", "O0"):
            ts = [orc.time_group(hb, g, 400, opt=opt, ref_side=side) for g in sample_g]
            if ts[0] is not None:
                legs[f"{name}_{opt}_hot_ns_per_group"] = float(np.mean(ts)) / 400 * 1e9
    legs["host_dram_read_GBs"] = orc.host_read_bw(1 << 30, threads) / 1e9
    what = ("oracle/_ref: the reference's dare_log.h + transcribed dare_ibv_rc.c / dare_server.c bodies over "
            "per-group dare_log_t images" if kind == "reference" else "oracle/apus_oracle.c (restatement)")
    return {"value": v, "unit": "decisions/s", "cores": threads, "kind": kind,
            "host_cpus": aff, "thread_cap": share or None,
            "threads_of_host": f"{threads} of {aff} CPUs",
            "sample": f"{S} groups x {reps} passes of the GPU step's work (commit walk + Adler-32 + median + "
                      f"remote-commit publish + pruning minimum"
                      + (f" + (idx, term) validation of {wl['R'] - 1} followers' NC buffers" if var_len else "")
                      + (" + vote tally + local (idx, term) walk + vote-request ranking" if votes else "")
                      + f"; {wl['R']} replicas, {wl['E']} x {64 + wl['L']}"
                      + (f"-{64 + lmax}" if lmax != wl["L"] else "") + "-B entries), "
                      f"{what}, -O2 OpenMP {threads} threads, {t:.1f} s, {_cpu_model()}",
            "legs": legs,
            "legs_note": "ref_*: the reference's code (oracle/_ref); port_*: the clean-room restatement; "
                         "*_1thread: one thread; *_no_checksum: without the build-defined Adler-32 (the "
                         "reference has none); *_hot_ns_per_group: walk + median + pruning minimum repeated on "
                         "one cache-resident group"}


def main():
    args = parse()
    try:
        plan, n = world_plan(args.gpus, os.environ)
    except ValueError as e:
        sys.exit(f"bench.py: {e}")
    if plan == "launch":
        # nothing has touched the GPU yet: the ranks run as child processes
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.call(launcher_cmd(sys.argv[1:], n, free_port()), env=env))
    import torch
    import torch.distributed as dist

    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi

    world = n
    # --rccl: the N > 1 plumbing (torch's RCCL group, libapus_gpu's own
    # communicator, the per-step all-reduce, barriers, the all-gather of the
    # ranks' times) at world 1 -- a rehearsal of the multi-GPU path on one GPU
    dist_on = world > 1 or args.rccl
    if dist_on and "MASTER_ADDR" not in os.environ:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if dist_on:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))

    wl = dict(WORKLOADS[args.workload])
    if args.groups:
        wl["G"] = args.groups
    G, R = wl["G"], wl["R"]
    eng = pkg.Engine(local)
    lib = eng.lib

    # libapus_gpu's own RCCL communicator for the stats all-reduce
    if dist_on:
        uid = C.create_string_buffer(128)
        if rank == 0:
            abi.check(lib.apus_comm_get_unique_id(uid), "apus_comm_get_unique_id")
        obj = [bytes(uid.raw) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        abi.check(lib.apus_comm_init_rank(eng.ctx, world, C.create_string_buffer(obj[0], 128), rank),
                  "apus_comm_init_rank")

    var_len = wl.get("var_len", False)
    votes = wl.get("votes", False)
    win = wl.get("win", False) and not args.no_win
    sep_fail = votes and (args.split or args.failover_calls)
    E = wl["E"]
    stride = pkg.batch.ring_stride_for(wl["ring"])
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream)
    if dist_on:
        # RCCL connects its channels on a communicator's first collective: done
        # here, so no timed step pays it whatever --warmup is
        abi.check(lib.apus_stats_allreduce(eng.ctx, sp), "apus_stats_allreduce")
        eng.stats_reset()
        torch.cuda.synchronize()

    def walked_of(db, Gw, maxd):
        """the bytes a checksum walk reads from every log as it is: each entry
        of [commit, end) (log_entries_to_nc_buf's list, 64-B header +
        cmd.len), and the entry count"""
        dets, ln = eng.log_entries_to_nc_buf(db, maxd)
        d3 = dets.view(torch.int64).view(Gw, maxd, 3)
        live = torch.arange(maxd, device=d3.device).view(1, maxd) < ln.view(Gw, 1).to(torch.int64)
        at = torch.arange(Gw, device=d3.device).view(Gw, 1) * stride + d3[:, :, 2]
        at = torch.where(live, at, torch.zeros_like(at))
        rv = db.ring
        typ = rv[at + 26].to(torch.int64)
        clen = rv[at + 48].to(torch.int64) | (rv[at + 49].to(torch.int64) << 8)
        elen = 64 + torch.where((typ == abi.NOOP) | (typ == abi.CONFIG) | (typ == abi.HEAD), 0, clen)
        return int(torch.where(live, elen, torch.zeros_like(elen)).sum().item()), dets, ln

    def tail_bytes(Gw):
        """algorithmic bytes of the commit call's tail launch (SURVEY 8d's
        per-decision figures for the modes the step runs; each input column
        once): state row 64 + self_idx 1 + the walk's commit 8; median:
        remote_end 8R, lr_step R, fail_count R -> 8 out; publish:
        remote_commit 8R (the posted writes not counted) -> 2 out; log_pruning:
        apply_offsets 8R, prev_head 1, abs_base 8 -> 17 out; C5's failover
        pass: the walk's (idx, term) row 16, vote_ack 8R, sid 8, hb 8R, the
        vote_req_t records 40R (--vote-sit: 24R + the winner's 16-B cid) ->
        13 out (tally) + 27 out (ranking)"""
        b = 64 + 1 + 8 + (10 * R + 8) + (8 * R + 2) + (8 * R + 1 + 8 + 17)
        if votes:
            b += 16 + 8 * R + 8 + 8 * R + (24 * R + 16 if args.vote_sit else 40 * R) + 13 + 27
        return b * Gw

    def run_wave(gid_base, Gw, warmup, steps):
        """one resident batch of Gw groups (ids gid_base..): generated on the
        device, then `warmup` untimed and `steps` timed steps; returns the
        timed wall seconds, the walk kernel's mean ms, its algorithmic bytes
        per launch, the last step's statistics and the walk kernel's name"""
        fields = ["state", "self_idx", "remote_end", "remote_commit", "lr_step", "fail_count", "apply_offsets",
                  "prev_head", "abs_base"]
        if votes:
            fields = pkg.batch.ALL_FIELDS   # every column: the vote and ranking kernels read vote_ack / vote_req / sid
        db = pkg.batch.DeviceBatch(Gw, R, stride, device=f"cuda:{local}", fields=fields)
        cfg = pkg.batch.gen_cfg(seed=2026, gid_base=gid_base, n_entries=wl["E"], n_history=wl["H"],
                                len_min=wl["L"], len_max=wl.get("Lmax", wl["L"]), ring_len=wl["ring"],
                                p_full_ack=0.9, straggler=True, cid_mix=wl.get("cid_mix", False), p_vote_ack=0.6,
                                hist_len_max=wl.get("Hmax", 0))
        eng.gen(db, cfg)
        if votes and args.vote_sit:
            # A/B only: the ranking's (sid, index, term) packed beside the 40-B
            # records (apus_batch_t.vote_sit; derived from them outside the
            # timed region -- the default step reads the records themselves)
            db.fill_vote_sit()
        torch.cuda.synchronize()
        flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM
        bst = db.struct()
        if args.impl == "lane":
            bst.flags = abi.BATCH_LANE_IMPL
        elif var_len:
            bst.flags = abi.BATCH_VAR_LEN
        elif wl.get("short"):
            bst.flags = abi.BATCH_SHORT_WALKS
        if args.tail_rows:
            bst.flags |= abi.BATCH_TAIL_ROWS
        walked_bytes = n_dets = val_bytes = 0
        ncs = vout = None
        keep = []
        if var_len:
            # C3: each follower's NC determinants are the leader's with the term
            # changed from a random position m_r ~ U[0, E] on; some
            # buffers truncated or empty.  Built outside the timed region.
            F = R - 1
            dets, ln = eng.log_entries_to_nc_buf(db, E)
            gq = torch.Generator(device=f"cuda:{local}").manual_seed(33 + gid_base)
            dv = dets.view(torch.int64).view(Gw, 1, E, 3).repeat(1, F, 1, 1).contiguous()
            m_r = torch.randint(0, E + 1, (Gw, F, 1), device=dv.device, generator=gq)
            dv[..., 1] += (torch.arange(E, device=dv.device).view(1, 1, E) >= m_r).to(torch.int64)
            del m_r
            cut = torch.randint(0, 8, (Gw, F), device=dv.device, generator=gq)
            nl = ln.view(Gw, 1).repeat(1, F)
            nl = torch.where(cut == 0, torch.zeros_like(nl), torch.where(cut == 1, nl // 2, nl)).contiguous()
            fol = ((db.arrays["self_idx"].view(Gw, 1).to(torch.int64) + 1 +
                    torch.arange(F, device=dv.device).view(1, F)) % R).to(torch.uint8).contiguous()
            keep += [dv, nl, fol]
            ncs = abi.NcBatch(n_followers=F, max_dets=E, dets=dv.data_ptr(), det_len=nl.data_ptr(),
                              follower=fol.data_ptr())
            vout = eng._z(Gw, torch.int64, F)
            # the walked bytes (every entry from commit to end: header + cmd.len)
            walked_bytes = walked_of(db, Gw, E)[0]
            n_dets = int(ln.to(torch.int64).sum().item())
            # the validation's bytes: every follower determinant compared (24 B,
            # up to its buffer's length), the leader's determinants (24 B each),
            # det_len 4 + follower 1 in and the remote end 8 out per follower
            val_bytes = 24 * int(nl.to(torch.int64).sum().item()) + 24 * n_dets + 13 * F * Gw
            del dets, ln
        if var_len and args.impl == "wave":
            # C3: the walk also writes the leader's NC determinants (a9) from the
            # headers it streams, and the validation reads them instead of
            # gathering the leader's headers (apus_nc_batch_t.leader_dets)
            flags |= abi.COMMIT_NC
            ncs.leader_max = E
        # the tail's work besides the median: update_remote_logs' publish and
        # log_pruning's minimum
        tail = abi.COMMIT_PUBLISH | abi.COMMIT_PRUNE
        if args.round4_tail:
            tail = abi.COMMIT_PRUNE                       # A/B only: the round-4 step (no publish, log_pruning)
        cout = eng.alloc_commit_out(Gw, flags | abi.COMMIT_MEDIAN | tail |
                                    (abi.COMMIT_LAST_IT | abi.COMMIT_VOTE | abi.COMMIT_RANK if votes else 0), nc_max=E)
        if flags & abi.COMMIT_NC:
            ncs.leader_dets, ncs.leader_len = cout["nc_dets"].data_ptr(), cout["nc_len"].data_ptr()
        ost = eng.commit_struct(cout)
        ost_med = abi.CommitOut(median=cout["median"].data_ptr())
        pout = {k: cout[k] for k in ("new_head", "append_head", "min_apply")}

        fused = flags | abi.COMMIT_MEDIAN | tail | abi.COMMIT_STATS_FRESH
        if votes:
            # C5's failover pass, outputs preallocated: the local (idx, term) of
            # every log from the commit call's own walk (APUS_COMMIT_LAST_IT), the
            # vote tally (poll_vote_count) and the vote-request ranking
            # (poll_vote_requests) on the same batch, in the commit call's tail
            # launch (APUS_COMMIT_VOTE | APUS_COMMIT_RANK); --failover-calls / --split:
            # as calls of their own after it (the round-3 step)
            fused |= abi.COMMIT_LAST_IT | (0 if sep_fail else abi.COMMIT_VOTE | abi.COMMIT_RANK)
            lit = cout["last_idx_term"]
            brk = db.struct()
            brk.flags = bst.flags
            brk.last_idx_term = lit.data_ptr()
            vos, rso = ost.vote, ost.rank
        wio = None
        if win:
            # the election-win transition on the tally just made (apus_vote_win_batch:
            # poll_vote_count after the tally, dare_server.c:1355-1362,1389-1510);
            # the configuration scans start at each log's commit (cid_offset)
            t = torch
            z = lambda dt, n=1: torch.zeros(Gw * n, dtype=dt, device=f"cuda:{local}")   # noqa: E731
            st64 = db.arrays["state"].view(torch.int64).view(Gw, 8)
            wt = {"won": cout["vote"]["won"], "voters": cout["vote"]["voters"], "new_commit": cout["vote"]["new_commit"],
                  "cid_offset": st64[:, 2].clone(), "cid_idx": z(t.int64), "req_id": z(t.int64),
                  "clt_id": z(t.int16), "last_applied": z(t.int64, 3), "last_csm_idx": z(t.int64),
                  "last_write_csm_idx": z(t.int64), "outcome": z(t.uint8), "n_cfg": z(t.int32)}
            keep.append(wt)
            wio = abi.WinIO(**{k: (wt[k].data_ptr() if k in wt else None) for k in abi.WIN_KEYS})

        def step(ev=None, tev=None, wev=None):
            if args.split:
                # round-2 form (A/B only): reset, walk call, median call, pruning call
                eng.stats_reset(stream)
                if ev is not None:
                    ev[0].record(stream)
                abi.check(lib.apus_commit_batch(eng.ctx, C.byref(bst), C.byref(ost), flags, sp), "commit")
                if ev is not None:
                    ev[1].record(stream)
                abi.check(lib.apus_commit_batch(eng.ctx, C.byref(bst), C.byref(ost_med), abi.COMMIT_MEDIAN, sp),
                          "median")
                eng.log_pruning(db, out=pout, bstruct=bst)
                if votes:
                    abi.check(lib.apus_last_idx_term_batch(eng.ctx, C.byref(bst), C.c_void_p(lit.data_ptr()), sp),
                              "apus_last_idx_term_batch")
            else:
                # one call: the walk kernel (its HIP events recorded by the library
                # right around it), then one tail launch for the deferred walks,
                # median, pruning (C5: the failover pass) and the statistics,
                # which replace the last batch's
                if ev is not None:
                    abi.check(lib.apus_commit_mark_walk(eng.ctx, C.c_void_p(ev[0].cuda_event),
                                                        C.c_void_p(ev[1].cuda_event)), "apus_commit_mark_walk")
                if tev is not None:
                    abi.check(lib.apus_commit_mark_tail(eng.ctx, C.c_void_p(tev[0].cuda_event),
                                                        C.c_void_p(tev[1].cuda_event)), "apus_commit_mark_tail")
                abi.check(lib.apus_commit_batch(eng.ctx, C.byref(bst), C.byref(ost), fused, sp), "commit")
            if var_len:
                abi.check(lib.apus_validate_batch(eng.ctx, C.byref(bst), C.byref(ncs), C.c_void_p(vout.data_ptr()),
                                                  sp), "validate")
            if sep_fail:
                abi.check(lib.apus_vote_batch(eng.ctx, C.byref(bst), C.byref(vos), sp), "apus_vote_batch")
                abi.check(lib.apus_vote_rank_batch(eng.ctx, C.byref(brk), C.byref(rso), sp), "apus_vote_rank_batch")
            if win:
                if wev is not None:
                    wev[0].record(stream)
                abi.check(lib.apus_vote_win_batch(eng.ctx, C.byref(bst), C.byref(wio), sp), "apus_vote_win_batch")
                if wev is not None:
                    wev[1].record(stream)
            if dist_on:
                abi.check(lib.apus_stats_allreduce(eng.ctx, sp), "apus_stats_allreduce")

        mk = lambda: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))   # noqa: E731
        failover = None
        if win:
            # the cold step: every candidate's transition happens here (its
            # winners are leaders from then on, as in the reference)
            cold = mk()
            step(wev=cold)
            torch.cuda.synchronize()
            oc = np.bincount(wt["outcome"].cpu().numpy(), minlength=8)
            failover = {"cold_win_ms": cold[0].elapsed_time(cold[1]),
                        "outcomes": {n: int(oc[i]) for i, n in enumerate(
                            ("not_candidate", "lost", "config", "noop", "transit", "stable", "undefined",
                             "corrupt"))},
                        "transitions": int(oc[2:7].sum()),
                        "blank_entries_appended": int((wt["last_write_csm_idx"][wt["outcome"] >= 2] != 0).sum()),
                        "config_reappends": int(wt["n_cfg"].to(torch.int64).sum().item())}
        for _ in range(warmup):
            step()
        eng.stats_reset()
        torch.cuda.synchronize()
        if win:
            # the timed steps' walks start from the commits the cold step left
            # (the tally's, on every candidate) and reach the blank entries the
            # winners appended: their bytes counted from the logs as they are
            walked_bytes = walked_of(db, Gw, E + 2)[0]
        evs = [mk() for _ in range(steps)]
        tevs = [mk() for _ in range(steps)]
        wevs = [mk() for _ in range(steps)] if win else [None] * steps
        for pair in evs + tevs + [w for w in wevs if w is not None]:   # create the events (at their first record)
            pair[0].record(stream)
            pair[1].record(stream)
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(evs[i], tevs[i] if not (args.split or args.tail_rows) else None, wevs[i])
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        tail_ms = None if (args.split or args.tail_rows) else float(np.mean([a.elapsed_time(b) for a, b in tevs]))
        win_ms = float(np.mean([a.elapsed_time(b) for a, b in wevs])) if win else None
        st = eng.stats()
        # algorithmic bytes of ONE launch of the dominant kernel:
        # every walked entry (64 B header + cmd.len) + 64 B group state + 1 B
        # self_idx in; 8 + 1 + 4 + 4 B out per group
        alg = (walked_bytes if (var_len or win) else wl["E"] * (64 + wl["L"]) * Gw) + (64 + 1 + 17) * Gw
        if flags & abi.COMMIT_NC:
            alg += n_dets * 24 + 4 * Gw                   # the determinants and their counts written
        # the walk kernel the library launched (its rocprof name)
        name = eng.walk_kernel_name(bst, flags if args.split else fused)
        # the whole step's algorithmic bytes: walk, tail, validation and the win
        # call's candidate test (sid 8 + self_idx 1 in; outcome 1 + n_cfg 4 out
        # per group; the few candidates' own walks not counted)
        step_bytes = alg + tail_bytes(Gw) + val_bytes + (14 * Gw if win else 0)
        del keep, cout, db
        return dict(elapsed=elapsed, kern_ms=kern_ms, alg=alg, st=st, name=name, tail_ms=tail_ms,
                    tail_alg=tail_bytes(Gw), val_bytes=val_bytes, win_ms=win_ms, step_bytes=step_bytes,
                    failover=failover)

    # C3's whole batch (c3_full): consecutive resident waves of wl["wave"]
    # groups, each generated outside the timed region; a step is one pass over
    # every wave, its time the sum of the waves' timed steps
    if wl.get("total"):
        total, wave = wl["total"], wl["wave"]
        waves = [(w, min(wave, total - w)) for w in range(0, total, wave)]
        G = total
    else:
        waves = [(0, G)]
    elapsed = kern_ms = 0.0
    tail_ms = 0.0
    alg_bytes = tail_alg = step_bytes = val_bytes = 0
    decided = 0
    wave_log = []
    for w0, Gw in waves:
        r = run_wave(rank * G + w0, Gw, args.warmup, args.steps)
        st, walk_name = r["st"], r["name"]
        elapsed += r["elapsed"]
        kern_ms += r["kern_ms"]
        alg_bytes += r["alg"]
        tail_ms = None if r["tail_ms"] is None or tail_ms is None else tail_ms + r["tail_ms"]
        tail_alg += r["tail_alg"]
        step_bytes += r["step_bytes"]
        val_bytes += r["val_bytes"]
        decided += int(st[abi.STAT_DECISIONS])
        wave_log.append({"groups": Gw, "ms_per_step": r["elapsed"] / args.steps * 1e3, "kernel_ms": r["kern_ms"],
                         "tail_ms": r["tail_ms"]})
        torch.cuda.empty_cache()

    per_rank = [(elapsed, kern_ms)]
    if dist_on:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=f"cuda:{local}")
        allt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        per_rank = [(float(a[0]), float(a[1])) for a in allt]
        elapsed = max(e for e, _ in per_rank)
        kern_ms = max(k for _, k in per_rank)

    # decisions: every group of every rank decides once per step; each wave's
    # last all-reduced statistics must say so
    decisions = G * world * args.steps
    assert decided == G * world, (decided, G * world)
    value = decisions / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    # the whole step against the roofline: every kernel's algorithmic bytes
    # (walk + tail + validation + the win call) over the wall time per step
    step_achieved = step_bytes / (ms_per_step * 1e-3) / 1e9
    traffic = tail_traffic = None
    try:
        with open(args.traffic or os.path.join(ROOT, "profiles", f"traffic_commit_{args.workload}.json")) as f:
            tj = json.load(f)
        if tj.get("groups") == G and tj.get("workload") == args.workload:
            traffic = tj.get("hbm_bytes_per_launch")
            tail_traffic = (tj.get("tail") or {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    out = {
        "metric": "quorum commit decisions/sec + achieved HBM GB/s",
        "value": value,
        "unit": "decisions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u64",
        "data": "synthetic (device-generated SplitMix64 traces, reference byte layout)",
        "config": {"workload": f"{args.workload}: {G} groups/GPU x {R} replicas, {wl['E']} x "
                               + (f"{64 + wl['L']}-{64 + wl['Lmax']}-B entries/batch, commit index + checksum + "
                                  f"(idx, term) validation of {R - 1} followers" if var_len else
                                  f"{64 + wl['L']}-B entries/batch, commit index + checksum")
                               + " + median + remote-commit publish + pruning minimum"
                               + (" + vote tally + vote-request ranking (STABLE / EXTENDED / TRANSIT "
                                  "configurations, vote_req_t records" + (" packed to vote_sit rows outside the "
                                  "timed region" if args.vote_sit else "") + ")" if votes else "")
                               + (" + election-win transition" if win else "")
                               + (f", {len(waves)} resident waves of <= {waves[0][1]} groups" if len(waves) > 1
                                  else "")
                               + (" + RCCL stats/watermark allreduce" if dist_on else ""),
                   "groups_per_gpu": G, "replicas": R, "entries": wl["E"], "payload_bytes": wl["L"],
                   "ring_bytes": wl["ring"], "parallelism": f"group-sharded x{world}",
                   "impl": args.impl},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": walk_name,
                     "kernel_ms": kern_ms, "alg_bytes_per_launch": alg_bytes,
                     "kernel_ms_per_rank": [k for _, k in per_rank],
                     "tail": None if tail_ms is None else {
                         "kernel": "quorum_tail_kernel", "kernel_ms": tail_ms, "alg_bytes_per_launch": tail_alg,
                         "achieved": tail_alg / (tail_ms * 1e-3) / 1e9,
                         "frac": tail_alg / (tail_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": tail_traffic},
                     "step_alg_bytes": step_bytes, "step_achieved": step_achieved,
                     "step_frac": step_achieved / HBM_PEAK_GBS,
                     "step_note": "step_frac = (walk + tail" + (" + validation" if var_len else "")
                                  + (" + win-call" if (votes and wl.get("win") and not args.no_win) else "")
                                  + " algorithmic bytes) / ms_per_step / peak"},
        "cpu_baseline": None,
        "ms_per_step_per_rank": [e / args.steps * 1e3 for e, _ in per_rank],
        "stats": {"committed_entries": int(st[abi.STAT_COMMITTED]), "advanced": int(st[abi.STAT_ADVANCED]),
                  "decisions": int(st[abi.STAT_DECISIONS]), "min_watermark": int(st[abi.STAT_MIN_WATERMARK]),
                  "deferred_to_lane_walk": int(st[abi.STAT_SLOW]), "corrupt": int(st[abi.STAT_CORRUPT]),
                  **({"votes_won": int(st[abi.STAT_VOTES_WON])} if votes else {})},
    }
    if win:
        out["failover"] = dict(r["failover"], win_call_ms_steady=r["win_ms"],
                               note="apus_vote_win_batch after the commit call's tally: the cold (first) step "
                                    "makes every winning candidate leader (timed on its own, cold_win_ms); the "
                                    "timed steps run it on the logs that step left (no candidate won again)")
    if var_len:
        out["roofline"]["validation_alg_bytes"] = val_bytes
    if len(waves) > 1:
        out["waves"] = wave_log
        #  what c3_full's number is: each wave is generated on the
        # device outside the timed region and walked while resident; getting
        # the ~2.7 TB of rings of the whole batch into HBM is not timed
        out["config"]["throughput"] = ("resident-wave throughput: every wave generated in HBM outside the timed "
                                       "region, then walked `steps` times; staging the batch into HBM excluded")
        if wl.get("Hmax"):
            out["config"]["history_cmd_max_bytes"] = wl["Hmax"]
        out["roofline"]["note"] = ("kernel_ms and alg_bytes_per_launch are sums over the waves (one launch per "
                                   "wave per step); stats are the last wave's")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pkg, wl, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
