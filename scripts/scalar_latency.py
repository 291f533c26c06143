"""Latency of the scalar drop-ins: one call on one
reference-shaped dare_log_t, as the reference's commit loop would make it
(dare_ibv_rc.c:1870-1948 calls the walk up to 1000 times per
rc_write_remote_logs), against the CPU cost of the same work.

Shape: SURVEY §6's probe -- R = 3, entries of 128 B, the walk covering a few
entries -- on a 16-KiB ring.  GPU: wall time per call from Python (ctypes
overhead, measured on apus_version, included and reported), after a warm-up
call, for both ring paths: a caller heap log (the call stages the bytes it
reads) and an apus_log_new log (read in place).  First call: the default
context's creation.
CPU: the restatement's and the reference primitives' cache-hot cost of walk
+ median + pruning minimum on the same group (oracle timing libraries).

Usage: python scripts/scalar_latency.py [--calls 2000]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ref_shaped(abi, lib, hb, g, mode):
    st = hb.state[g]
    ln = int(st["len"])
    hdr = C.sizeof(abi.LogHeader)
    if mode == "owned":
        p = C.c_void_p()
        assert lib.apus_log_new(ln, C.byref(p)) == 0
        buf = np.ctypeslib.as_array((C.c_uint8 * (hdr + ln)).from_address(p.value))
    else:
        buf = np.zeros(hdr + ln + 64, np.uint8)
    log = abi.LogHeader.from_address(buf.ctypes.data)
    for k in ("head", "apply", "commit", "end", "tail", "len"):
        setattr(log, k, int(st[k]))
    buf[hdr:hdr + ln] = hb.group_ring(g)[:ln]
    R = hb.R
    servers = (abi.Server * 13)()
    for i in range(R):
        servers[i].fail_count = int(hb.fail_count[g * R + i])
        servers[i].next_lr_step = int(hb.lr_step[g * R + i])
    cfg = abi.ServerConfig()
    C.memmove(C.addressof(cfg.cid), hb.state[g:g + 1].tobytes()[48:64], 16)
    cfg.idx = int(hb.self_idx[g])
    cfg.len = R
    cfg.servers = servers
    ctrl = abi.CtrlData()
    for i in range(13):
        ctrl.vote_ack[i] = int(hb.vote_ack[g * R + i]) if i < R else ln
    for i in range(R):
        ctrl.log_offsets[i].end = int(hb.remote_end[g * R + i])
        ctrl.apply_offsets[i] = int(hb.apply_offsets[g * R + i])
    return buf, cfg, servers, ctrl


def per_call_us(fn, n):
    fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--entries", type=int, default=8)
    args = ap.parse_args()
    import apus_pkg
    pkg = apus_pkg.load_package()
    orc = apus_pkg.load_oracle()
    abi = pkg.abi
    lib = abi.load_library()
    R, L, G = 3, 16384, 16
    cfg = pkg.batch.gen_cfg(seed=606, n_entries=args.entries, n_history=4, len_min=64, len_max=64, ring_len=L,
                            p_full_ack=0.7, straggler=True)
    hb = orc.host_batch(G, R, L)
    orc.gen(hb, cfg)
    ref = orc.commit(hb, abi.COMMIT_WALK)
    g = int(np.argmax(ref["committed"] == 1))
    nc, cm = C.c_uint64(0), C.c_int(0)
    md = C.c_uint64(0)
    nh, aph = C.c_uint64(0), C.c_int(0)
    vc, vcm, vm = (C.c_uint8 * 2)(), C.c_uint64(0), C.c_uint16(0)
    res = {"shape": f"R={R}, {args.entries} x 128-B entries after 4 history entries, {L}-B ring, group {g}",
           "ctypes_overhead_us": per_call_us(lambda: lib.apus_version(), args.calls), "gpu_us_per_call": {}}
    for mode in ("heap", "owned"):
        buf, scfg, servers, ctrl = ref_shaped(abi, lib, hb, g, mode)
        logp = C.c_void_p(buf.ctypes.data)
        t0 = time.perf_counter()
        assert lib.apus_commit_reply_walk(logp, C.byref(scfg), C.byref(nc), C.byref(cm)) == 0
        res.setdefault("first_call_us", (time.perf_counter() - t0) * 1e6)
        assert nc.value == ref["new_commit"][g], "scalar walk != oracle"
        res["gpu_us_per_call"][mode] = {
            "apus_commit_reply_walk": per_call_us(
                lambda: lib.apus_commit_reply_walk(logp, C.byref(scfg), C.byref(nc), C.byref(cm)), args.calls),
            "apus_commit_median": per_call_us(
                lambda: lib.apus_commit_median(logp, C.byref(scfg), C.byref(ctrl), C.byref(md)), args.calls),
            "apus_vote_tally": per_call_us(
                lambda: lib.apus_vote_tally(logp, C.byref(scfg), C.byref(ctrl), vc, C.byref(vcm), C.byref(vm)),
                args.calls),
            "apus_min_apply": per_call_us(
                lambda: lib.apus_min_apply(logp, C.byref(scfg), C.byref(ctrl), 0, C.byref(nh), C.byref(aph)),
                args.calls),
        }
        if mode == "owned":
            assert lib.apus_log_free(logp) == 0
    reps = 20000
    cpu = {}
    for side, name in ((False, "port"), (True, "ref")):
        for opt in ("O2", "O0"):
            t = orc.time_group(hb, g, reps, opt=opt, ref_side=side)
            if t is not None:
                cpu[f"{name}_{opt}_walk_median_prune_ns"] = t / reps * 1e9
    res["cpu_ns_per_group"] = cpu
    walk3 = sum(res["gpu_us_per_call"]["heap"][k] for k in ("apus_commit_reply_walk", "apus_commit_median",
                                                     "apus_min_apply"))
    best_cpu = min(cpu.values()) if cpu else None
    res["gpu_walk_median_prune_us"] = walk3
    if best_cpu:
        res["gpu_over_cpu"] = walk3 * 1e3 / best_cpu
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
