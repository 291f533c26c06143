"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front end of oracle/liboracle.so (clean-room C restatement of the APUS
hot path + the synthetic trace generator) and, where present, of
oracle/_ref/libapusref.so (the reference's own dare_log.h compiled from
/root/reference, with the hot-path loops restated on its primitives).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "liboracle.so")
REF = os.path.join(HERE, "_ref", "libapusref.so")

_lib = None
_ref = None


def _pkg():
    import sys
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import apus_pkg
    return apus_pkg.load_package()


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        abi = _pkg().abi
        L = C.CDLL(LIB)
        vp, u64, u32, u8 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint8
        P = C.POINTER
        sig = {
            "apus_oracle_dist": (u64, [u64, u64, u64]),
            "apus_oracle_larger": (C.c_int, [u64, u64, u64, u64]),
            "apus_oracle_adler32": (u32, [vp, C.c_size_t, u32]),
            "apus_oracle_checksum": (u32, [vp, vp]),
            "apus_oracle_place_seq": (C.c_int, [u64, u64, u32, vp, vp, vp, P(u64)]),
            "apus_oracle_gen_check": (C.c_int, [P(abi.Batch), P(abi.GenCfg)]),
            "apus_oracle_gen_batch": (None, [P(abi.Batch), P(abi.GenCfg), u64, u64, C.c_int]),
            "apus_oracle_commit_batch": (None, [P(abi.Batch), P(abi.CommitOut), u32, u64, u64, C.c_int]),
            "apus_oracle_vote_batch": (None, [P(abi.Batch), P(abi.VoteOut), u64, u64]),
            "apus_oracle_rank_batch": (None, [P(abi.Batch), P(abi.RankOut), u64, u64]),
            "apus_oracle_prune_batch": (None, [P(abi.Batch), P(abi.PruneOut), u64, u64, P(u64)]),
            "apus_oracle_validate_batch": (None, [P(abi.Batch), P(abi.NcBatch), vp, u64, u64]),
            "apus_oracle_nc_build_batch": (None, [P(abi.Batch), vp, u32, vp, u64, u64]),
            "apus_oracle_gen_nc": (None, [P(abi.Batch), P(abi.GenCfg), P(abi.NcBatch), u64, u64]),
            "apus_oracle_last_idx_term": (None, [vp, vp, vp]),
            "apus_oracle_log_get_tail": (u64, [vp, vp]),
            "apus_oracle_find_remote_end": (C.c_int, [vp, vp, vp, u64, P(u64)]),
            "apus_oracle_append_batch": (None, [P(abi.Batch), P(abi.AppendIn), P(abi.AppendOut), P(u64)]),
            "apus_oracle_persist_batch": (None, [P(abi.Batch), P(abi.PersistIn), P(u64)]),
            "apus_oracle_records_store_batch": (None, [P(abi.Batch), P(abi.RecordsIO), P(u64)]),
            "apus_oracle_records_load_batch": (None, [P(abi.RecordsLoadIO)]),
            "apus_oracle_config_scan_batch": (None, [P(abi.Batch), P(abi.ConfigIO), u64, u64, P(u64)]),
            "apus_oracle_apply_batch": (None, [P(abi.Batch), P(abi.ApplyIO), u64, u64, P(u64)]),
            "apus_oracle_vote_win_batch": (None, [P(abi.Batch), P(abi.WinIO), u64, u64, P(u64)]),
            "apus_oracle_lr_completion_batch": (None, [P(abi.Batch), P(abi.LrIO), u64, u64]),
            "apus_oracle_log_adjust_batch": (None, [P(abi.Batch), P(abi.LrIO), u64, u64]),
            "apus_oracle_time_commit": (C.c_double, [P(abi.Batch), P(abi.CommitOut), u32, C.c_int, C.c_int]),
            "apus_oracle_tail_batch": (None, [P(abi.Batch), P(abi.CommitOut), u32, vp, u64, u64, P(u64), P(u64)]),
        }
        for n, (r, a) in sig.items():
            f = getattr(L, n)
            f.restype, f.argtypes = r, a
        _lib = L
    return _lib


def ref():
    """reference-composed oracle, or None when /root/reference was absent at build"""
    global _ref
    if _ref is None:
        if not os.path.exists(REF):
            return None
        R = C.CDLL(REF)
        vp, u64, u8 = C.c_void_p, C.c_uint64, C.c_uint8
        sig = {
            "ref_layout": (C.c_int, [vp, C.c_int]),
            "ref_dist": (u64, [vp, u64]),
            "ref_larger": (C.c_int, [vp, u64, u64]),
            "ref_commit_walk": (u64, [vp, vp, vp, u8, vp]),
            "ref_median": (u64, [vp, vp, u8, vp, vp, vp]),
            "ref_vote_tally": (C.c_int, [vp, vp, u8, vp, vp, vp]),
            "ref_last_idx_term": (None, [vp, vp, vp]),
            "ref_vote_rank": (C.c_int, [vp, vp, u8, u64, vp, C.c_int, vp, u64, u64, vp, vp, vp]),
            "ref_min_apply": (u64, [vp, vp, vp, vp, C.c_int, vp, vp]),
            "ref_find_remote_end": (u64, [vp, vp, vp, u64]),
            "ref_nc_build": (u64, [vp, vp, vp, u64]),
            "ref_get_tail": (u64, [vp, vp]),
            "ref_append_seq": (C.c_int, [u64, u64, C.c_int, vp, vp, vp, vp, vp, vp, vp]),
            "ref_append_group": (C.c_int, [vp, u64, vp, vp, u64, vp, C.c_uint32, vp, u64, vp, vp]),
            "ref_persist_one": (C.c_int, [vp, u64, vp, u8, C.c_uint32, vp, C.c_uint32]),
            "ref_config_scan": (C.c_int, [vp, vp, vp, vp, u64, vp, vp, vp]),
            "ref_lr_completion": (None, [u8, vp, vp, vp]),
            "ref_log_adjust": (None, [vp, vp, vp, u8, C.c_uint32, vp, vp, vp, C.c_uint16, vp, vp, vp, vp, vp,
                                      C.c_uint32, vp, vp]),
            "ref_apply": (C.c_int, [vp, vp, vp, u8, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                    C.c_uint32, vp]),
            "ref_records_store_one": (C.c_int, [vp, vp, vp, vp, u64, vp, vp]),
            "ref_records_load_one": (C.c_int, [vp, C.c_uint32, vp, C.c_uint32, vp, vp, vp]),
            "ref_publish": (None, [vp, vp, u8, C.c_uint32, u64, vp, vp, vp, vp, C.c_uint16, vp, vp]),
            "ref_force_prune": (C.c_int, [vp, u64, vp, vp, u8, C.c_uint32, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                          vp]),
            "ref_vote_count": (C.c_int, [vp, u64, vp, vp, u8, C.c_uint32, vp, vp, vp, vp, vp, vp, vp, u64, vp, vp,
                                         vp, vp, vp, vp, vp, vp, vp]),
        }
        for n, (r, a) in sig.items():
            f = getattr(R, n)
            f.restype, f.argtypes = r, a
        _ref = R
    return _ref


def p(a):
    return C.c_void_p(a.ctypes.data)


_CHECK_IN = ("rings", "state", "self", "step", "fail", "prev", "conn", "rend", "rcommit", "apply", "vote_ack", "hb",
             "req", "sid")
# (output, numpy dtype, per-group count); with_votes: only on vote batches
_CHECK_OUT = (("new_commit", np.uint64, 1, False), ("median", np.uint64, 1, False), ("ssn", np.uint64, 1, False),
              ("rcommit_out", np.uint64, "R", False), ("new_head", np.uint64, 1, False),
              ("min_apply", np.uint64, 1, False), ("apply_out", np.uint64, "R", False),
              ("vote_commit", np.uint64, 1, True), ("lit", np.uint64, 2, True), ("new_sid", np.uint64, 1, True),
              ("committed", np.uint8, 1, False), ("append_head", np.uint8, 1, False), ("won", np.uint8, 1, True),
              ("vc", np.uint8, 2, True), ("outcome", np.uint8, 1, True), ("new_cid", np.uint8, 16, True),
              ("digest", np.uint32, 1, False), ("publish", np.uint16, 1, False), ("cleared", np.uint16, 1, True))


class RefCheckIO(C.Structure):
    _fields_ = ([("n", C.c_uint64), ("ring_stride", C.c_uint64), ("R", C.c_uint32), ("votes", C.c_uint32)] +
                [(k, C.c_void_p) for k in _CHECK_IN] + [(o[0], C.c_void_p) for o in _CHECK_OUT] +
                [("nc_max", C.c_uint32), ("F", C.c_uint32), ("M", C.c_uint32), ("pad", C.c_uint32)] +
                [(k, C.c_void_p) for k in ("nc_dets_out", "nc_len_out", "dets", "det_len", "follower",
                                          "rend_follow")])


def ref_check(n, R, stride, ins, votes, threads=0, nc_max=0, followers=None):
    """The GPU step's per-group results from the REFERENCE's own code
    (oracle/_ref ref_check_batch: walk + the build's Adler-32 + median + publish
    on the walk's commit + pruning minimum; with votes the tally, the local
    (idx, term) and the ranking) over n groups given as numpy byte / word
    arrays: ring [n*stride], state [n*64 B], self_idx, remote_end,
    remote_commit, lr_step, fail_count, apply_offsets, prev_head, rc_connected
    (optional), and with votes vote_ack, hb, vote_req [n*R*40 B], sid.
    nc_max: also the leader's NC buffer (out nc_dets [n*nc_max*3] u64, nc_len);
    followers = (dets [n*F*M*3] u64, det_len [n*F] u32, follower [n*F] u8, F,
    M): also each follower's validated remote end (out rend_follow [n*F]).
    Returns {output: numpy array}, or None without the _ref build."""
    R_ = ref()
    if R_ is None:
        return None
    f = R_.ref_check_batch
    f.restype, f.argtypes = C.c_int, [C.POINTER(RefCheckIO), C.c_int]
    keep = []

    def q(a, dt=None):
        if a is None:
            return None
        a = np.ascontiguousarray(a if dt is None else a.view(dt))
        keep.append(a)
        return a.ctypes.data
    io = RefCheckIO(n=n, ring_stride=stride, R=R, votes=1 if votes else 0)
    io.rings, io.state, io.self = q(ins["ring"], np.uint8), q(ins["state"], np.uint8), q(ins["self_idx"], np.uint8)
    io.step, io.fail, io.prev = q(ins["lr_step"], np.uint8), q(ins["fail_count"], np.uint8), q(ins["prev_head"], np.uint8)
    io.conn = q(ins.get("rc_connected"), np.uint16)
    io.rend, io.rcommit = q(ins["remote_end"], np.uint64), q(ins["remote_commit"], np.uint64)
    io.apply = q(ins["apply_offsets"], np.uint64)
    if votes:
        io.vote_ack, io.hb = q(ins["vote_ack"], np.uint64), q(ins["hb"], np.uint64)
        io.req, io.sid = q(ins["vote_req"], np.uint64), q(ins["sid"], np.uint64)
    out = {}
    for name, dt, per, wv in _CHECK_OUT:
        k = R if per == "R" else per
        a = np.zeros(n * k if (votes or not wv) else 1, dt)
        out[name] = a
        setattr(io, name, a.ctypes.data)
    res = {k: v for k, v in out.items() if votes or k not in {o[0] for o in _CHECK_OUT if o[3]}}
    if nc_max:
        io.nc_max = nc_max
        res["nc_dets"], res["nc_len"] = np.zeros(n * nc_max * 3, np.uint64), np.zeros(n, np.uint32)
        io.nc_dets_out, io.nc_len_out = res["nc_dets"].ctypes.data, res["nc_len"].ctypes.data
    if followers is not None:
        dets, det_len, fol, F, M = followers
        io.F, io.M = F, M
        io.dets, io.det_len, io.follower = q(dets, np.uint64), q(det_len, np.uint32), q(fol, np.uint8)
        res["rend_follow"] = np.zeros(n * F, np.uint64)
        io.rend_follow = res["rend_follow"].ctypes.data
    if f(C.byref(io), int(threads)) != 0:
        raise MemoryError("ref_check_batch: no memory for a thread's log image")
    return res


# ---------------------------------------------------------- CPU baseline legs
_timing = {}


def timing_lib(opt="O2", ref_side=False):
    """the restatement (liboracle[_O0].so) or the reference-composed oracle
    (_ref/libapusref[_O0].so) for the bench's CPU-baseline legs; None when
    that build is absent"""
    key = (opt, ref_side)
    if key not in _timing:
        suf = "" if opt == "O2" else "_" + opt
        path = os.path.join(HERE, "_ref", f"libapusref{suf}.so") if ref_side else os.path.join(HERE, f"liboracle{suf}.so")
        if not os.path.exists(path):
            _timing[key] = None
            return None
        abi = _pkg().abi
        L = C.CDLL(path)
        vp, u64, u8, i = C.c_void_p, C.c_uint64, C.c_uint8, C.c_int
        if ref_side:
            L.ref_time_group.restype = C.c_double
            L.ref_time_group.argtypes = [vp, vp, vp, u8, vp, vp, vp, vp, i]
            L.ref_bench_new.restype = vp
            L.ref_bench_new.argtypes = [u64, C.c_uint32, u64, vp, u64] + [vp] * 14 + [C.c_uint32, C.c_uint32, vp, vp,
                                                                                     vp]
            L.ref_bench_time.restype = C.c_double
            L.ref_bench_time.argtypes = [vp, i, i, i, C.POINTER(u64)]
            L.ref_bench_free.restype = None
            L.ref_bench_free.argtypes = [vp]
        else:
            L.apus_oracle_gen_check.restype, L.apus_oracle_gen_check.argtypes = i, [C.POINTER(abi.Batch),
                                                                                   C.POINTER(abi.GenCfg)]
            L.apus_oracle_gen_batch.restype = None
            L.apus_oracle_gen_batch.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.GenCfg), u64, u64, i]
            L.apus_oracle_time_step.restype = C.c_double
            L.apus_oracle_time_step.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.CommitOut),
                                                C.POINTER(abi.PruneOut), C.c_uint32, i, i]
            L.apus_oracle_time_step_full.restype = C.c_double
            L.apus_oracle_time_step_full.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.CommitOut),
                                                     C.POINTER(abi.PruneOut), C.POINTER(abi.VoteOut),
                                                     C.POINTER(abi.RankOut), C.POINTER(abi.NcBatch), vp,
                                                     C.c_uint32, i, i]
            L.apus_oracle_time_group.restype = C.c_double
            L.apus_oracle_time_group.argtypes = [vp, vp, u8, vp, vp, vp, vp, i]
            L.apus_oracle_host_read_bw.restype = C.c_double
            L.apus_oracle_host_read_bw.argtypes = [u64, i, i]
        _timing[key] = L
    return _timing[key]


def time_step(hb, flags, reps, threads, opt="O2", votes=False, nc=None):
    """seconds for `reps` passes of the bench step (commit walk / checksum /
    median per `flags`, then the pruning minimum) over the whole batch; with
    votes the vote tally and the local (idx, term) walk + vote-request
    ranking of every group, with nc = (dets, det_len, follower, F, M) the
    followers' (idx, term) validation (apus_oracle_time_step_full)"""
    L = timing_lib(opt)
    G = hb.G
    out = {"new_commit": np.zeros(G, np.uint64), "committed": np.zeros(G, np.uint8),
           "n_entries": np.zeros(G, np.uint32), "digest": np.zeros(G, np.uint32), "median": np.zeros(G, np.uint64)}
    abi = _pkg().abi
    co = abi.CommitOut(**{k: v.ctypes.data for k, v in out.items()})
    pout = {"new_head": np.zeros(G, np.uint64), "append_head": np.zeros(G, np.uint8),
            "min_apply": np.zeros(G, np.uint64)}
    po = abi.PruneOut(**{k: v.ctypes.data for k, v in pout.items()})
    s = hb.struct()
    if not votes and nc is None:
        return L.apus_oracle_time_step(C.byref(s), C.byref(co), C.byref(po), flags, reps, threads)
    vo = ro = ncs = rend = None
    keep = []
    if votes:
        vb = {"won": np.zeros(G, np.uint8), "vote_count": np.zeros(2 * G, np.uint8),
              "new_commit": np.zeros(G, np.uint64), "voters": np.zeros(G, np.uint16)}
        rb = {"outcome": np.zeros(G, np.uint8), "new_sid": np.zeros(G, np.uint64),
              "new_cid": np.zeros(16 * G, np.uint8), "cleared": np.zeros(G, np.uint16)}
        keep += [vb, rb]
        vo = C.byref(abi.VoteOut(**{k: v.ctypes.data for k, v in vb.items()}))
        ro = C.byref(abi.RankOut(**{k: v.ctypes.data for k, v in rb.items()}))
    if nc is not None:
        dets, det_len, follower, F, M = nc
        rend = np.zeros(G * F, np.uint64)
        keep.append(rend)
        ncs = C.byref(abi.NcBatch(n_followers=F, max_dets=M, dets=dets.ctypes.data, det_len=det_len.ctypes.data,
                                  follower=follower.ctypes.data))
        rend = p(rend)
    return L.apus_oracle_time_step_full(C.byref(s), C.byref(co), C.byref(po), vo, ro, ncs, rend, flags, reps,
                                        threads)


def time_group(hb, g, reps, opt="O2", ref_side=False):
    """seconds for `reps` cache-hot repetitions of walk + median + pruning
    minimum on group g (restatement, or the reference's primitives)"""
    L = timing_lib(opt, ref_side)
    if L is None:
        return None
    R = hb.R
    st = hb.state[g:g + 1]
    ring = hb.group_ring(g)
    rend = hb.remote_end[g * R:(g + 1) * R].copy()
    step = hb.lr_step[g * R:(g + 1) * R].copy()
    fail = hb.fail_count[g * R:(g + 1) * R].copy()
    ap = np.zeros(16, np.uint64)
    ap[:R] = hb.apply_offsets[g * R:(g + 1) * R]
    pad = lambda a, dt: np.concatenate([a, np.zeros(16 - len(a), dt)])   # noqa: E731
    rend, step, fail = pad(rend, np.uint64), pad(step, np.uint8), pad(fail, np.uint8)
    self_ = int(hb.self_idx[g])
    if ref_side:
        st6 = np.array([st["head"][0], st["apply"][0], st["commit"][0], st["end"][0], st["tail"][0], st["len"][0]],
                       np.uint64)
        cid16 = np.frombuffer(st.tobytes()[48:64], np.uint8).copy()
        return L.ref_time_group(p(ring), p(st6), p(cid16), self_, p(rend), p(step), p(fail), p(ap), reps)
    return L.apus_oracle_time_group(p(ring), p(st), self_, p(rend), p(step), p(fail), p(ap), reps)


class RefBench:
    """the step's work on the reference's own code over a host batch's groups
    (oracle/_ref ref_bench_*: one dare_log_t image per group, the reference's
    server_t / ctrl_data shapes, built once); None-safe: `ok` is False when
    the _ref build is absent"""

    def __init__(self, hb, opt="O2", nc=None):
        self.L = timing_lib(opt, ref_side=True)
        self.h = None
        if self.L is None:
            return
        G, R = hb.G, hb.R
        st = hb.state
        st6 = np.stack([st[k] for k in ("head", "apply", "commit", "end", "tail", "len")], axis=1).astype(np.uint64)
        st6 = np.ascontiguousarray(st6)
        cid = np.ascontiguousarray(np.frombuffer(st.tobytes(), np.uint8).reshape(G, 64)[:, 48:64])
        A = hb.arrays
        votes = "vote_ack" in A and "vote_req" in A and "sid" in A and "hb" in A
        self._keep = [st6, cid]

        def q(a):
            if a is None:
                return None
            a = np.ascontiguousarray(a)
            self._keep.append(a)
            return p(a)
        F = M = 0
        dets = det_len = fol = None
        if nc is not None:
            dets, det_len, fol, F, M = nc
        self.h = self.L.ref_bench_new(G, R, int(st["len"][0]), p(hb.ring), hb.stride, p(st6), p(cid), q(hb.self_idx),
                                      q(A["remote_end"]), q(A["remote_commit"]), q(A["lr_step"]), q(A["fail_count"]),
                                      q(A["apply_offsets"]), q(A["prev_head"]), q(A.get("rc_connected")),
                                      q(A["vote_ack"]) if votes else None, q(A["hb"]) if votes else None,
                                      q(A["vote_req"].view(np.uint64)) if votes else None,
                                      q(A["sid"]) if votes else None, F, M, q(dets), q(det_len), q(fol))
        self.G = G

    @property
    def ok(self):
        return bool(self.h)

    def time(self, reps, threads, checksum=True):
        """(seconds for `reps` passes, group 0's checksum)"""
        d = C.c_uint64(0)
        t = self.L.ref_bench_time(self.h, reps, threads, 1 if checksum else 0, C.byref(d))
        return t, d.value

    def close(self):
        if self.h:
            self.L.ref_bench_free(self.h)
            self.h = None


def host_read_bw(nbytes, threads, reps=3):
    return timing_lib("O2").apus_oracle_host_read_bw(nbytes, threads, reps)


# ---------------------------------------------------------------- batches
def host_batch(G, R, ring_len, fields=None):
    b = _pkg().batch
    kw = {} if fields is None else {"fields": fields}
    return b.HostBatch(G, R, b.ring_stride_for(ring_len), **kw)


def gen(hb, cfg, threads=0):
    s = hb.struct()
    L = lib()
    if L.apus_oracle_gen_check(C.byref(s), C.byref(cfg)) != 0:
        raise ValueError("generator config rejected")
    L.apus_oracle_gen_batch(C.byref(s), C.byref(cfg), 0, hb.G, threads)


def commit(hb, flags, threads=0):
    abi = _pkg().abi
    G = hb.G
    out = {"new_commit": np.zeros(G, np.uint64), "committed": np.zeros(G, np.uint8),
           "n_entries": np.zeros(G, np.uint32), "digest": np.zeros(G, np.uint32),
           "median": np.zeros(G, np.uint64)}
    o = abi.CommitOut(new_commit=out["new_commit"].ctypes.data, committed=out["committed"].ctypes.data,
                      n_entries=out["n_entries"].ctypes.data, digest=out["digest"].ctypes.data,
                      median=out["median"].ctypes.data)
    s = hb.struct()
    lib().apus_oracle_commit_batch(C.byref(s), C.byref(o), flags, 0, G, threads)
    return out


def vote(hb):
    abi = _pkg().abi
    G = hb.G
    out = {"won": np.zeros(G, np.uint8), "vote_count": np.zeros(2 * G, np.uint8),
           "new_commit": np.zeros(G, np.uint64), "voters": np.zeros(G, np.uint16)}
    o = abi.VoteOut(**{k: v.ctypes.data for k, v in out.items()})
    s = hb.struct()
    lib().apus_oracle_vote_batch(C.byref(s), C.byref(o), 0, G)
    return out


def rank(hb, use_lit=True):
    abi = _pkg().abi
    G = hb.G
    out = {"outcome": np.zeros(G, np.uint8), "new_sid": np.zeros(G, np.uint64),
           "new_cid": np.zeros(16 * G, np.uint8), "cleared": np.zeros(G, np.uint16)}
    o = abi.RankOut(**{k: v.ctypes.data for k, v in out.items()})
    s = hb.struct()
    if not use_lit:
        s.last_idx_term = None
    lib().apus_oracle_rank_batch(C.byref(s), C.byref(o), 0, G)
    return out


def prune(hb):
    abi = _pkg().abi
    G = hb.G
    out = {"new_head": np.zeros(G, np.uint64), "append_head": np.zeros(G, np.uint8),
           "min_apply": np.zeros(G, np.uint64)}
    o = abi.PruneOut(**{k: v.ctypes.data for k, v in out.items()})
    wm = C.c_uint64(0)
    s = hb.struct()
    lib().apus_oracle_prune_batch(C.byref(s), C.byref(o), 0, G, C.byref(wm))
    return out, wm.value


def gen_nc(hb, cfg, F, M):
    abi = _pkg().abi
    dets = np.zeros(hb.G * F * M * 3, np.uint64)
    det_len = np.zeros(hb.G * F, np.uint32)
    follower = np.zeros(hb.G * F, np.uint8)
    nc = abi.NcBatch(n_followers=F, max_dets=M, dets=dets.ctypes.data, det_len=det_len.ctypes.data,
                     follower=follower.ctypes.data)
    s = hb.struct()
    lib().apus_oracle_gen_nc(C.byref(s), C.byref(cfg), C.byref(nc), 0, hb.G)
    return dets, det_len, follower


def validate(hb, dets, det_len, follower, F, M):
    abi = _pkg().abi
    out = np.zeros(hb.G * F, np.uint64)
    nc = abi.NcBatch(n_followers=F, max_dets=M, dets=dets.ctypes.data, det_len=det_len.ctypes.data,
                     follower=follower.ctypes.data)
    s = hb.struct()
    lib().apus_oracle_validate_batch(C.byref(s), C.byref(nc), p(out), 0, hb.G)
    return out


def nc_build(hb, M):
    dets = np.zeros(hb.G * M * 3, np.uint64)
    ln = np.zeros(hb.G, np.uint32)
    s = hb.struct()
    lib().apus_oracle_nc_build_batch(C.byref(s), p(dets), M, p(ln), 0, hb.G)
    return dets, ln


def last_idx_term(hb):
    out = np.zeros(2 * hb.G, np.uint64)
    st = hb.state
    for g in range(hb.G):
        o = np.zeros(2, np.uint64)
        lib().apus_oracle_last_idx_term(p(hb.group_ring(g)), C.c_void_p(st.ctypes.data + 64 * g), p(o))
        out[2 * g:2 * g + 2] = o
    return out


def time_commit(hb, flags, reps, threads):
    abi = _pkg().abi
    G = hb.G
    bufs = [np.zeros(G, np.uint64), np.zeros(G, np.uint8), np.zeros(G, np.uint32), np.zeros(G, np.uint32)]
    o = abi.CommitOut(new_commit=bufs[0].ctypes.data, committed=bufs[1].ctypes.data,
                      n_entries=bufs[2].ctypes.data, digest=bufs[3].ctypes.data, median=None)
    s = hb.struct()
    return lib().apus_oracle_time_commit(C.byref(s), C.byref(o), flags, reps, threads)


# ------------------------------------------------- log append + persist (8f.1)
def append(hb, entries, payload, max_entries, n_entries=None, term=None, last_idx=None):
    """log_append_entry over every group's queue (in place on hb).  Returns
    (idx [G*M] u64, last_idx [G] u64, groups stopped)."""
    abi = _pkg().abi
    G = hb.G
    idx = np.zeros(G * max_entries, np.uint64)
    last = np.zeros(G, np.uint64) if last_idx is None else last_idx.copy()
    ai = abi.AppendIn(entries=entries.ctypes.data, n_entries=None if n_entries is None else n_entries.ctypes.data,
                      term=None if term is None else term.ctypes.data, payload=payload.ctypes.data,
                      payload_bytes=payload.nbytes, max_entries=max_entries)
    ao = abi.AppendOut(idx=idx.ctypes.data, last_idx=last.ctypes.data)
    bad = C.c_uint64(0)
    s = hb.struct()
    lib().apus_oracle_append_batch(C.byref(s), C.byref(ai), C.byref(ao), C.byref(bad))
    return idx, last, bad.value


def persist(hb, old_end, limit=None):
    """persist_new_entries for every replica copy (in place on hb and old_end)"""
    abi = _pkg().abi
    pi = abi.PersistIn(old_end=old_end.ctypes.data, limit=None if limit is None else limit.ctypes.data)
    bad = C.c_uint64(0)
    s = hb.struct()
    lib().apus_oracle_persist_batch(C.byref(s), C.byref(pi), C.byref(bad))
    return bad.value


def records_store(hb, cursor, cap, dump=None, dump_len=None):
    """stablestorage_save_request over persist_new_entries' walk (proxy.c:
    269-291, dare_server.c:1792-1810): cursor [G] uint64 (in/out), dumps
    [G, cap]; returns dump, dump_len, n_records, corrupt"""
    abi = _pkg().abi
    G = hb.G
    dump = np.zeros((G, cap), np.uint8) if dump is None else dump
    dump_len = np.zeros(G, np.uint32) if dump_len is None else dump_len
    n = np.zeros(G, np.uint32)
    io = abi.RecordsIO(cursor=cursor.ctypes.data, dump=dump.ctypes.data, cap=cap, dump_len=dump_len.ctypes.data,
                       n_records=n.ctypes.data)
    bad = C.c_uint64(0)
    s = hb.struct()
    lib().apus_oracle_records_store_batch(C.byref(s), C.byref(io), C.byref(bad))
    return dump, dump_len, n, bad.value


def records_load(dumps, size, max_plan):
    """stablestorage_load_records (proxy.c:306-336) over dumps [n, stride]"""
    abi = _pkg().abi
    n = dumps.shape[0]
    plan = np.zeros((n, max(max_plan, 1)), np.dtype([("offset", "<u4"), ("data_len", "<u4"),
                                                    ("connection_id", "<u2"), ("action", "u1"),
                                                    ("pad", "u1", (5,))]))
    out = {"n_records": np.zeros(n, np.uint32), "counts": np.zeros((n, 3), np.uint32),
           "status": np.zeros(n, np.uint32), "stop": np.zeros(n, np.uint32)}
    size = np.ascontiguousarray(size, np.uint32)
    io = abi.RecordsLoadIO(dump=dumps.ctypes.data, stride=dumps.shape[1], size=size.ctypes.data, n=n,
                           plan=plan.ctypes.data if max_plan else None, max_plan=max_plan,
                           n_records=out["n_records"].ctypes.data, counts=out["counts"].ctypes.data,
                           status=out["status"].ctypes.data, stop=out["stop"].ctypes.data)
    lib().apus_oracle_records_load_batch(C.byref(io))
    out["plan"] = plan[:, :max_plan]
    return out


def ref_records_store(hb, cursor, cap, dump=None, dump_len=None):
    """records_store through oracle/_ref: persist_new_entries' walk on the
    reference's dare_log.h with stablestorage_save_request restated on its
    proxy.h (ref_compose.c, ref_records.c); same returns"""
    R = ref()
    G = hb.G
    dump = np.zeros((G, cap), np.uint8) if dump is None else dump
    dump_len = np.zeros(G, np.uint32) if dump_len is None else dump_len
    n = np.zeros(G, np.uint32)
    bad = 0
    for g in range(G):
        st6 = _st6(hb, g)
        c = np.array([cursor[g]], np.uint64)
        dl = np.array([dump_len[g]], np.uint32)
        k = np.zeros(1, np.uint32)
        row = np.ascontiguousarray(dump[g])
        bad += R.ref_records_store_one(p(hb.group_ring(g)), p(st6), p(c), p(row), cap, p(dl), p(k))
        dump[g] = row
        cursor[g], dump_len[g], n[g] = c[0], dl[0], k[0]
    return dump, dump_len, n, bad


def ref_records_store_batch(n, stride, ring, state, cursor, dump, cap, dump_len, n_rec):
    """ref_records_store_one on every group in C (oracle/_ref, one thread); in
    place on cursor [n] u64, dump [n*cap] u8, dump_len / n_rec [n] u32.
    Returns the groups that stopped."""
    R_ = ref()
    if R_ is None:
        return None
    f = R_.ref_records_store_batch
    f.restype = C.c_uint64
    f.argtypes = [C.c_uint64, C.c_uint64] + [C.c_void_p] * 4 + [C.c_uint64, C.c_void_p, C.c_void_p]
    return int(f(n, stride, p(ring), p(state), p(cursor), p(dump), cap, p(dump_len), p(n_rec)))


def ref_records_load_batch(dumps, stride, size, max_plan):
    """ref_records_load_one on every snapshot in C; returns the same dict as
    records_load with plan as bytes [n*max_plan*16]"""
    R_ = ref()
    if R_ is None:
        return None
    n = size.size
    f = R_.ref_records_load_batch
    f.restype = None
    f.argtypes = [C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32] + [C.c_void_p] * 4
    out = {"plan": np.zeros(n * max(max_plan, 1) * 16, np.uint8), "n_records": np.zeros(n, np.uint32),
           "counts": np.zeros(3 * n, np.uint32), "status": np.zeros(n, np.uint32), "stop": np.zeros(n, np.uint32)}
    sz = np.ascontiguousarray(size, np.uint32)
    f(n, p(dumps), stride, p(sz), p(out["plan"]) if max_plan else None, max_plan, p(out["n_records"]),
      p(out["counts"]), p(out["status"]), p(out["stop"]))
    return out


def ref_records_load(dumps, size, max_plan):
    """records_load through oracle/_ref: stablestorage_load_records restated on
    the reference's proxy.h (ref_records.c); same returns"""
    R = ref()
    n = dumps.shape[0]
    plan = np.zeros((n, max(max_plan, 1)), np.dtype([("offset", "<u4"), ("data_len", "<u4"),
                                                    ("connection_id", "<u2"), ("action", "u1"),
                                                    ("pad", "u1", (5,))]))
    out = {"n_records": np.zeros(n, np.uint32), "counts": np.zeros((n, 3), np.uint32),
           "status": np.zeros(n, np.uint32), "stop": np.zeros(n, np.uint32)}
    for k in range(n):
        sz = min(int(size[k]), dumps.shape[1])            # apus_gpu.h: a size above the stride reads the stride
        row = np.ascontiguousarray(dumps[k])
        pr = np.zeros(max(max_plan, 1), plan.dtype)
        nr, st = np.zeros(1, np.uint32), np.zeros(1, np.uint32)
        cnt = np.zeros(3, np.uint32)
        out["status"][k] = R.ref_records_load_one(p(row), sz, p(pr) if max_plan else None, max_plan, p(nr), p(cnt),
                                                  p(st))
        out["n_records"][k], out["stop"][k], out["counts"][k] = nr[0], st[0], cnt
        plan[k] = pr
    out["plan"] = plan[:, :max_plan]
    return out


def ref_append(hb, entries, payload, max_entries, n_entries=None, term=None, last_idx=None):
    """the same through the reference's own log_append_entry (oracle/_ref)"""
    R = ref()
    G = hb.G
    st_all = hb.state
    idx = np.zeros(G * max_entries, np.uint64)
    last = np.zeros(G, np.uint64) if last_idx is None else last_idx.copy()
    bad = 0
    for g in range(G):
        st = np.array([st_all["head"][g], st_all["apply"][g], st_all["commit"][g], st_all["end"][g],
                       st_all["tail"][g], st_all["len"][g]], np.uint64)
        ph = np.array([hb.prev_head[g]], np.uint8)
        n = max_entries if n_entries is None else min(int(n_entries[g]), max_entries)
        t = int(term[g]) if term is not None else int(hb.sid[g]) >> 9
        lg = np.array([last[g]], np.uint64)
        ring = hb.group_ring(g)
        q = entries[g * max_entries:(g + 1) * max_entries]
        out = np.zeros(max(n, 1), np.uint64)
        bad += R.ref_append_group(p(ring), hb.stride, p(st), p(ph), t, C.c_void_p(q.ctypes.data), n,
                                  p(payload), payload.nbytes, p(out), p(lg))
        idx[g * max_entries:g * max_entries + n] = out[:n]
        st_all["end"][g], st_all["tail"][g] = st[3], st[4]
        hb.prev_head[g] = ph[0]
        last[g] = lg[0]
    return idx, last, bad


def ref_append_batch(n, stride, arr, entries, payload, max_entries, n_entries=None, term=None, last_idx=None):
    """ref_append (the reference's own log_append_entry) over every group in C
    (oracle/_ref ref_append_batch, one thread): arr = writable numpy ring,
    state (64-B rows), prev_head, sid, in place.  Returns (idx [n*M], last
    [n], stopped groups), or None without _ref."""
    R_ = ref()
    if R_ is None:
        return None
    f = R_.ref_append_batch
    f.restype = C.c_int
    f.argtypes = [C.c_uint64, C.c_uint64] + [C.c_void_p] * 6 + [C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64] + \
        [C.c_void_p] * 3
    for k in ("ring", "state", "prev_head"):
        assert arr[k].flags["C_CONTIGUOUS"] and arr[k].flags["WRITEABLE"], k
    idx = np.zeros(n * max_entries, np.uint64)
    last = np.zeros(n, np.uint64) if last_idx is None else np.array(last_idx, np.uint64).copy()
    stopped = np.zeros(n, np.uint8)
    keep = [np.ascontiguousarray(x) for x in (entries, payload, arr["sid"])]
    ne = None if n_entries is None else np.ascontiguousarray(n_entries, np.uint32)
    tm = None if term is None else np.ascontiguousarray(term, np.uint64)
    if f(n, stride, p(arr["ring"]), p(arr["state"]), p(arr["prev_head"]), None if tm is None else p(tm),
         p(keep[2]), p(keep[0]), max_entries, None if ne is None else p(ne), p(keep[1]), keep[1].nbytes, p(idx),
         p(last), p(stopped)) != 0:
        raise MemoryError("ref_append_batch")
    return idx, last, int(stopped.sum())


def ref_persist_batch(n, R, stride, arr, old_end, limit=None, threads=0):
    """ref_persist (every replica copy's walk) over every group in C, OpenMP
    (oracle/_ref ref_persist_batch): arr = writable numpy ring, state,
    self_idx; old_end [n*R] in place.  Returns the copies that stopped."""
    R_ = ref()
    if R_ is None:
        return None
    f = R_.ref_persist_batch
    f.restype = C.c_int
    f.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64] + [C.c_void_p] * 6 + [C.c_int]
    assert old_end.dtype == np.uint64 and old_end.flags["C_CONTIGUOUS"] and old_end.flags["WRITEABLE"]
    corrupt = np.zeros(n, np.uint32)
    lim = None if limit is None else np.ascontiguousarray(limit, np.uint32)
    if f(n, R, stride, p(arr["ring"]), p(arr["state"]), p(arr["self_idx"]), p(old_end),
         None if lim is None else p(lim), p(corrupt), int(threads)) != 0:
        raise MemoryError("ref_persist_batch")
    return int(corrupt.sum())


def ref_persist(hb, old_end, limit=None):
    R = ref()
    G, NR = hb.G, hb.R
    st_all = hb.state
    bad = 0
    for g in range(G):
        st = np.array([st_all["head"][g], st_all["apply"][g], st_all["commit"][g], st_all["end"][g],
                       st_all["tail"][g], st_all["len"][g]], np.uint64)
        ring = hb.group_ring(g)
        for i in range(NR):
            oe = np.array([old_end[g * NR + i]], np.uint64)
            lim = 0xFFFFFFFF if limit is None else int(limit[g * NR + i])
            bad += R.ref_persist_one(p(ring), hb.stride, p(st), int(hb.self_idx[g]), i, p(oe), lim)
            old_end[g * NR + i] = oe[0]
    return bad


# ---------------------------------------------------------------- 8f.2
def config_io(G, cid_offset, cid_idx, req_id=None, clt_id=None):
    """host arrays of apus_config_io_t (copies; returned dict is updated in place)"""
    return {"cid_offset": np.array(cid_offset, np.uint64).copy(), "cid_idx": np.array(cid_idx, np.uint64).copy(),
            "req_id": np.zeros(G, np.uint64) if req_id is None else np.array(req_id, np.uint64).copy(),
            "clt_id": np.zeros(G, np.uint16) if clt_id is None else np.array(clt_id, np.uint16).copy(),
            "departed": np.zeros(G, np.uint16)}


def config_scan(hb, io):
    """poll_config_entries on every group (in place on hb.state and io); returns the corrupt count"""
    abi = _pkg().abi
    c = abi.ConfigIO(**{k: io[k].ctypes.data for k in ("cid_offset", "cid_idx", "req_id", "clt_id", "departed")})
    bad = C.c_uint64(0)
    s = hb.struct()
    lib().apus_oracle_config_scan_batch(C.byref(s), C.byref(c), 0, hb.G, C.byref(bad))
    return bad.value


def apply_io(G, max_cfg, req_id=None, clt_id=None, last_applied=None, last_csm_idx=None):
    APPEND_DT = _pkg().batch.APPEND_DT
    return {"req_id": np.zeros(G, np.uint64) if req_id is None else np.array(req_id, np.uint64).copy(),
            "clt_id": np.zeros(G, np.uint16) if clt_id is None else np.array(clt_id, np.uint16).copy(),
            "last_applied": np.zeros(3 * G, np.uint64) if last_applied is None
            else np.array(last_applied, np.uint64).copy(),
            "last_csm_idx": np.zeros(G, np.uint64) if last_csm_idx is None
            else np.array(last_csm_idx, np.uint64).copy(),
            "n_applied": np.zeros(G, np.uint32), "departed": np.zeros(G, np.uint16),
            "events": np.zeros(G, np.uint8), "cfg_entries": np.zeros(G * max_cfg, APPEND_DT),
            "cfg_payload": np.zeros(G * max_cfg * 16, np.uint8), "n_cfg": np.zeros(G, np.uint32),
            "max_cfg": max_cfg}


def apply(hb, io):
    """apply_committed_entries on every group (in place on hb.state and io); returns the corrupt count"""
    abi = _pkg().abi
    keys = ("req_id", "clt_id", "last_applied", "last_csm_idx", "n_applied", "departed", "events",
            "cfg_entries", "cfg_payload", "n_cfg")
    a = abi.ApplyIO(max_cfg=io["max_cfg"], **{k: io[k].ctypes.data for k in keys})
    bad = C.c_uint64(0)
    s = hb.struct()
    lib().apus_oracle_apply_batch(C.byref(s), C.byref(a), 0, hb.G, C.byref(bad))
    return bad.value


def _st6(hb, g):
    st = hb.state
    return np.array([st["head"][g], st["apply"][g], st["commit"][g], st["end"][g], st["tail"][g], st["len"][g]],
                    np.uint64)


def ref_config_scan_batch(n, stride, ring, state, io):
    """ref_config_scan on every group in C (oracle/_ref, one thread): ring,
    state (64-B rows, writable) numpy; io as config_io builds it; in place.
    Returns the corrupt count (None without _ref)."""
    R_ = ref()
    if R_ is None:
        return None
    f = R_.ref_config_scan_batch
    f.restype, f.argtypes = C.c_uint64, [C.c_uint64, C.c_uint64] + [C.c_void_p] * 7
    return int(f(n, stride, p(ring), p(state), p(io["cid_offset"]), p(io["cid_idx"]), p(io["req_id"]),
                 p(io["clt_id"]), p(io["departed"])))


def ref_apply_batch(n, stride, ring, state, self_idx, sid, io):
    """ref_apply on every group in C (oracle/_ref, one thread): ring, state
    (64-B rows, writable), self_idx, sid numpy; io as apply_io builds it
    (the CONFIG re-appends as apus_append_batch records); in place.
    Returns the corrupt count (None without _ref)."""
    R_ = ref()
    if R_ is None:
        return None
    f = R_.ref_apply_batch
    f.restype = C.c_uint64
    f.argtypes = [C.c_uint64, C.c_uint64] + [C.c_void_p] * 13 + [C.c_uint32, C.c_void_p]
    keys = ("req_id", "clt_id", "last_applied", "last_csm_idx", "n_applied", "departed", "events", "cfg_entries",
            "cfg_payload")
    return int(f(n, stride, p(ring), p(state), p(self_idx), p(sid), *[p(io[k]) for k in keys], int(io["max_cfg"]),
                 p(io["n_cfg"])))


def ref_config_scan(hb, io):
    """the same through oracle/_ref (reference primitives + equal_cid / CID macros)"""
    R = ref()
    bad = 0
    for g in range(hb.G):
        st = _st6(hb, g)
        cid = hb.state["cid"][g:g + 1].view(np.uint8).copy()
        off = io["cid_offset"][g:g + 1].copy()
        rq = io["req_id"][g:g + 1].copy()
        cl = io["clt_id"][g:g + 1].copy()
        dep = np.zeros(1, np.uint16)
        bad += R.ref_config_scan(p(hb.group_ring(g)), p(st), p(cid), p(off), int(io["cid_idx"][g]), p(rq), p(cl),
                                 p(dep))
        hb.state["head"][g] = st[0]
        hb.state["cid"][g:g + 1] = cid.view(hb.state.dtype["cid"])
        io["cid_offset"][g], io["req_id"][g], io["clt_id"][g], io["departed"][g] = off[0], rq[0], cl[0], dep[0]
    return bad


def ref_apply(hb, io):
    """the same through oracle/_ref; cfg records are rebuilt in apus_append_batch's format"""
    R = ref()
    M = io["max_cfg"]
    bad = 0
    for g in range(hb.G):
        st = _st6(hb, g)
        cid = hb.state["cid"][g:g + 1].view(np.uint8).copy()
        rq = io["req_id"][g:g + 1].copy()
        cl = io["clt_id"][g:g + 1].copy()
        la = io["last_applied"][3 * g:3 * g + 3].copy()
        lc = io["last_csm_idx"][g:g + 1].copy()
        na, nc = np.zeros(1, np.uint32), np.zeros(1, np.uint32)
        dep, ev = np.zeros(1, np.uint16), np.zeros(1, np.uint8)
        creq, cclt = np.zeros(max(M, 1), np.uint64), np.zeros(max(M, 1), np.uint16)
        ccid = np.zeros(16 * max(M, 1), np.uint8)
        bad += R.ref_apply(p(hb.group_ring(g)), p(st), p(cid), int(hb.self_idx[g]), int(hb.sid[g]), p(rq), p(cl),
                           p(la), p(lc), p(na), p(dep), p(ev), p(creq), p(cclt), p(ccid), M, p(nc))
        hb.state["apply"][g] = st[1]
        hb.state["cid"][g:g + 1] = cid.view(hb.state.dtype["cid"])
        io["req_id"][g], io["clt_id"][g], io["last_csm_idx"][g] = rq[0], cl[0], lc[0]
        io["last_applied"][3 * g:3 * g + 3] = la
        io["n_applied"][g], io["departed"][g], io["events"][g], io["n_cfg"][g] = na[0], dep[0], ev[0], nc[0]
        ce = io["cfg_entries"]
        for k in range(int(nc[0])):
            j = g * M + k
            ce["req_id"][j], ce["clt_id"][j], ce["type"][j], ce["data_off"][j] = creq[k], cclt[k], 2, 16 * j
            io["cfg_payload"][16 * (g * M + k):16 * (g * M + k + 1)] = ccid[16 * k:16 * k + 16]
    return bad


# ------------------------------------------- 8f.2 replication step machine
LR_KEYS = ("send_flag", "send_count", "wc", "rc_connected", "nc_len", "nc_dets", "ssn", "post")


def lr_io(G, R, max_dets, send_flag=None, send_count=None, wc=None, rc_connected=None, nc_len=None,
          nc_dets=None, ssn=None):
    """host arrays of apus_lr_io_t (copies; the returned dict is updated in place)"""
    DET_DT = _pkg().batch.DET_DT

    def c(a, n, dt):
        return np.zeros(n, dt) if a is None else np.array(a, dt).copy()
    return {"send_flag": c(send_flag, G * R, np.uint8), "send_count": c(send_count, G * R, np.uint8),
            "wc": c(wc, G * R, np.uint8),
            "rc_connected": None if rc_connected is None else np.array(rc_connected, np.uint16).copy(),
            "nc_len": c(nc_len, G * R, np.uint64),
            "nc_dets": np.zeros(G * R * max(max_dets, 1), DET_DT) if nc_dets is None else nc_dets.copy(),
            "ssn": c(ssn, G, np.uint64), "post": np.zeros(G * R, np.uint8), "max_dets": max_dets}


def _lr_struct(io):
    abi = _pkg().abi
    return abi.LrIO(max_dets=io["max_dets"],
                    **{k: (None if io[k] is None else io[k].ctypes.data) for k in LR_KEYS})


def lr_completion(hb, io):
    """handle_lr_work_completion on every (group, server) pair (in place on hb.lr_step and io)"""
    s, li = hb.struct(), _lr_struct(io)
    lib().apus_oracle_lr_completion_batch(C.byref(s), C.byref(li), 0, hb.G)


def log_adjust(hb, io):
    """log_adjustment on every group (in place on hb and io)"""
    s, li = hb.struct(), _lr_struct(io)
    lib().apus_oracle_log_adjust_batch(C.byref(s), C.byref(li), 0, hb.G)


def ref_lr_completion(hb, io):
    R = ref()
    for k in range(hb.G * hb.R):
        st, sf, sc = (np.array([v], np.uint8) for v in (hb.lr_step[k], io["send_flag"][k], io["send_count"][k]))
        R.ref_lr_completion(int(io["wc"][k]), p(st), p(sf), p(sc))
        hb.lr_step[k], io["send_flag"][k], io["send_count"][k] = st[0], sf[0], sc[0]


def ref_log_adjust_batch(n, R, stride, arr, io):
    """ref_log_adjust on every group in C (oracle/_ref, one thread): arr =
    writable numpy ring, state (64-B rows), self_idx, fail_count, lr_step,
    vote_ack, remote_commit, remote_end; io as lr_io builds it; in place."""
    R_ = ref()
    if R_ is None:
        return None
    f = R_.ref_log_adjust_batch
    f.restype = None
    f.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64] + [C.c_void_p] * 12 + [C.c_uint32, C.c_void_p, C.c_void_p]
    a = arr
    f(n, R, stride, p(a["ring"]), p(a["state"]), p(a["self_idx"]), p(a["fail_count"]), p(a["lr_step"]),
      p(io["send_flag"]), None if io.get("rc_connected") is None else p(io["rc_connected"]), p(a["vote_ack"]),
      p(a["remote_commit"]), p(a["remote_end"]), p(io["nc_len"]), p(io["nc_dets"]), io["max_dets"], p(io["ssn"]),
      p(io["post"]))


def ref_lr_completion_batch(step, io):
    """ref_lr_completion on every (group, server) pair in C (oracle/_ref): step
    = lr_step numpy, io's wc / send_flag / send_count; in place"""
    R_ = ref()
    if R_ is None:
        return None
    f = R_.ref_lr_completion_batch
    f.restype, f.argtypes = None, [C.c_uint64] + [C.c_void_p] * 4
    f(step.size, p(io["wc"]), p(step), p(io["send_flag"]), p(io["send_count"]))


def ref_log_adjust(hb, io):
    """the same through oracle/_ref (real log_is_offset_larger / log_find_remote_end_offset)"""
    R = ref()
    NR, M = hb.R, io["max_dets"]
    for g in range(hb.G):
        st = _st6(hb, g)
        cid = hb.state["cid"][g:g + 1].view(np.uint8).copy()
        sl = slice(g * NR, (g + 1) * NR)
        fc, step, sf = hb.fail_count[sl].copy(), hb.lr_step[sl].copy(), io["send_flag"][sl].copy()
        va, rcm, rend = hb.vote_ack[sl].copy(), hb.remote_commit[sl].copy(), hb.remote_end[sl].copy()
        ncl = io["nc_len"][sl].copy()
        dets = io["nc_dets"][g * NR * M:(g + 1) * NR * M].copy()
        ssn = io["ssn"][g:g + 1].copy()
        post = np.zeros(NR, np.uint8)
        conn = 0xFFFF if io["rc_connected"] is None else int(io["rc_connected"][g])
        R.ref_log_adjust(p(hb.group_ring(g)), p(st), p(cid), int(hb.self_idx[g]), NR, p(fc), p(step), p(sf), conn,
                         p(va), p(rcm), p(rend), p(ncl), p(dets), M, p(ssn), p(post))
        hb.state["commit"][g] = st[2]
        hb.lr_step[sl], io["send_flag"][sl], hb.remote_commit[sl], hb.remote_end[sl] = step, sf, rcm, rend
        io["ssn"][g], io["post"][sl] = ssn[0], post


# ------------------------ update_remote_logs' publish + force_log_pruning
def tail_out(G, flags, req_id=None, clt_id=None, ssn=None):
    """host outputs of APUS_COMMIT_PUBLISH / APUS_COMMIT_FORCE_PRUNE (+ the pruning outputs)"""
    out = {"new_head": np.zeros(G, np.uint64), "append_head": np.zeros(G, np.uint8),
           "min_apply": np.zeros(G, np.uint64), "publish": np.zeros(G, np.uint16),
           "ssn": np.zeros(G, np.uint64) if ssn is None else np.array(ssn, np.uint64).copy(),
           "force": {"action": np.zeros(G, np.uint8), "target": np.zeros(G, np.uint8),
                     "cfg_idx": np.zeros(G, np.uint64),
                     "req_id": np.zeros(G, np.uint64) if req_id is None else np.array(req_id, np.uint64).copy(),
                     "clt_id": np.zeros(G, np.uint16) if clt_id is None else np.array(clt_id, np.uint16).copy()}}
    return out


def tail(hb, flags, commit=None, out=None):
    """the publish and force_log_pruning of a commit call (apus_oracle_tail_batch),
    in place on hb; commit: the walk's new commit per group (None: state.commit).
    Returns (out, watermark, corrupt)."""
    abi = _pkg().abi
    G = hb.G
    out = tail_out(G, flags) if out is None else out
    f = out["force"]
    co = abi.CommitOut(new_head=out["new_head"].ctypes.data, append_head=out["append_head"].ctypes.data,
                       min_apply=out["min_apply"].ctypes.data, publish=out["publish"].ctypes.data,
                       ssn=out["ssn"].ctypes.data,
                       force=abi.ForceOut(**{k: v.ctypes.data for k, v in f.items()}))
    wm, bad = C.c_uint64(0), C.c_uint64(0)
    s = hb.struct()
    cm = None if commit is None else np.ascontiguousarray(commit, np.uint64)
    lib().apus_oracle_tail_batch(C.byref(s), C.byref(co), flags, None if cm is None else p(cm), 0, G, C.byref(wm),
                                 C.byref(bad))
    return out, wm.value, bad.value


def ref_tail(hb, flags, commit=None, out=None):
    """the same through oracle/_ref: the publish (dare_ibv_rc.c:1761-1794) and
    force_log_pruning (dare_server.c:2073-2121) transcribed on the reference's
    own primitives (ref_compose.c)"""
    abi = _pkg().abi
    R = ref()
    G, NR = hb.G, hb.R
    out = tail_out(G, flags) if out is None else out
    f = out["force"]
    wm, bad = (1 << 64) - 1, 0
    for g in range(G):
        st = _st6(hb, g)
        c = int(st[2]) if commit is None else int(commit[g])
        cid = hb.state["cid"][g:g + 1].view(np.uint8).copy()
        sl = slice(g * NR, (g + 1) * NR)
        self_ = int(hb.self_idx[g])
        if flags & abi.COMMIT_PUBLISH:
            rc = hb.remote_commit[sl].copy()
            rend, step, fail = hb.remote_end[sl].copy(), hb.lr_step[sl].copy(), hb.fail_count[sl].copy()
            m, ssn = np.zeros(1, np.uint16), out["ssn"][g:g + 1].copy()
            conn = 0xFFFF if "rc_connected" not in hb.arrays else int(hb.rc_connected[g])
            R.ref_publish(p(st), p(cid), self_, NR, c, p(rend), p(rc), p(step), p(fail), conn, p(m), p(ssn))
            hb.remote_commit[sl] = rc
            out["publish"][g], out["ssn"][g] = m[0], ssn[0]
        if flags & abi.COMMIT_FORCE_PRUNE:
            st2 = st.copy()
            st2[2] = c
            ap = hb.apply_offsets[sl].copy()
            ph = np.array([hb.prev_head[g] if "prev_head" in hb.arrays else 0], np.uint8)
            rq, cl = f["req_id"][g:g + 1].copy(), f["clt_id"][g:g + 1].copy()
            nh, app, mn = np.zeros(1, np.uint64), np.zeros(1, np.int32), np.zeros(1, np.uint64)
            tg, ci, bd = np.zeros(1, np.uint8), np.zeros(1, np.uint64), np.zeros(1, np.int32)
            a = R.ref_force_prune(p(hb.group_ring(g)), hb.stride, p(st2), p(cid), self_, NR, int(hb.sid[g]), p(ap),
                                  p(ph), p(rq), p(cl), p(nh), p(app), p(mn), p(tg), p(ci), p(bd))
            hb.state["end"][g], hb.state["tail"][g] = st2[3], st2[4]
            hb.state["cid"][g:g + 1] = cid.view(hb.state.dtype["cid"])
            hb.apply_offsets[sl] = ap
            if "prev_head" in hb.arrays:
                hb.prev_head[g] = ph[0]
            f["action"][g], f["target"][g], f["cfg_idx"][g] = a, tg[0], ci[0]
            f["req_id"][g], f["clt_id"][g] = rq[0], cl[0]
            out["new_head"][g], out["append_head"][g], out["min_apply"][g] = nh[0], app[0], mn[0]
            if "abs_base" in hb.arrays:
                wm = min(wm, (int(hb.abs_base[g]) + int(nh[0])) & ((1 << 64) - 1))
            bad += int(bd[0])
    return out, wm, bad


def ref_force_prune_batch(n, R, stride, arr, req_id, clt_id):
    """ref_force_prune on every group in C (oracle/_ref, one thread): arr =
    writable numpy ring, state (64-B rows, commit already the walk's),
    self_idx, sid, apply_offsets, prev_head; req_id / clt_id [n] in place.
    Returns (outputs dict, corrupt count)."""
    R_ = ref()
    if R_ is None:
        return None
    f = R_.ref_force_prune_batch
    f.restype = C.c_uint64
    f.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64] + [C.c_void_p] * 14
    out = {"new_head": np.zeros(n, np.uint64), "append_head": np.zeros(n, np.uint8),
           "min_apply": np.zeros(n, np.uint64), "target": np.zeros(n, np.uint8), "cfg_idx": np.zeros(n, np.uint64),
           "action": np.zeros(n, np.uint8)}
    a = arr
    bad = f(n, R, stride, p(a["ring"]), p(a["state"]), p(a["self_idx"]), p(a["sid"]), p(a["apply_offsets"]),
            p(a["prev_head"]), p(req_id), p(clt_id), p(out["new_head"]), p(out["append_head"]), p(out["min_apply"]),
            p(out["target"]), p(out["cfg_idx"]), p(out["action"]))
    return out, int(bad)


# ------------------------------------ election-win transition (config 5)
def win_io(G, won, voters, new_commit, cid_offset, cid_idx, req_id=None, clt_id=None, last_applied=None,
           last_csm_idx=None, last_write_csm_idx=None):
    """host arrays of apus_win_io_t (copies; the returned dict is updated in place)"""
    def c(a, n, dt):
        return np.zeros(n, dt) if a is None else np.array(a, dt).copy()
    return {"won": c(won, G, np.uint8), "voters": c(voters, G, np.uint16), "new_commit": c(new_commit, G, np.uint64),
            "cid_offset": c(cid_offset, G, np.uint64), "cid_idx": c(cid_idx, G, np.uint64),
            "req_id": c(req_id, G, np.uint64), "clt_id": c(clt_id, G, np.uint16),
            "last_applied": c(last_applied, 3 * G, np.uint64), "last_csm_idx": c(last_csm_idx, G, np.uint64),
            "last_write_csm_idx": c(last_write_csm_idx, G, np.uint64), "outcome": np.zeros(G, np.uint8),
            "events": np.zeros(G, np.uint8), "departed": np.zeros(G, np.uint16), "n_applied": np.zeros(G, np.uint32),
            "n_cfg": np.zeros(G, np.uint32)}


def vote_win(hb, io):
    """the election-win transition on every group (in place on hb and io); returns the corrupt count"""
    abi = _pkg().abi
    w = abi.WinIO(**{k: io[k].ctypes.data for k in abi.WIN_KEYS})
    bad = C.c_uint64(0)
    s = hb.struct()
    lib().apus_oracle_vote_win_batch(C.byref(s), C.byref(w), 0, hb.G, C.byref(bad))
    return bad.value


def ref_vote_count_batch(n, R, stride, arr, io):
    """ref_vote_count on every group, in C (oracle/_ref ref_vote_count_batch):
    arr = numpy arrays ring, state (64-B rows), self_idx, sid, vote_ack,
    remote_commit, lr_step, apply_offsets, prev_head; io as win_io builds it.
    In place on arr and io (each array must be a writable contiguous buffer of
    its field's bytes); returns the corrupt count, or None without _ref."""
    R_ = ref()
    if R_ is None:
        return None
    f = R_.ref_vote_count_batch
    f.restype = C.c_int
    f.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64] + [C.c_void_p] * 21
    for k, v in list(arr.items()) + list(io.items()):
        assert v.flags["C_CONTIGUOUS"] and v.flags["WRITEABLE"], k
    a, i = arr, io
    rc = f(n, R, stride, p(a["ring"]), p(a["state"]), p(a["self_idx"]), p(a["sid"]), p(a["vote_ack"]),
           p(a["remote_commit"]), p(a["lr_step"]), p(a["apply_offsets"]), p(a["prev_head"]), p(i["cid_offset"]),
           p(i["cid_idx"]), p(i["req_id"]), p(i["clt_id"]), p(i["last_applied"]), p(i["last_csm_idx"]),
           p(i["last_write_csm_idx"]), p(i["events"]), p(i["departed"]), p(i["n_applied"]), p(i["n_cfg"]),
           p(i["outcome"]))
    if rc != 0:
        raise MemoryError("ref_vote_count_batch")
    return int((io["outcome"] == 7).sum())


def ref_vote_count(hb, io):
    """poll_vote_count whole (the tally, then the win transition) through
    oracle/_ref, on the same io (won / voters / new_commit are not read: the
    transcription tallies itself); in place on hb and io"""
    R = ref()
    NR = hb.R
    bad = 0
    st_all = hb.state
    for g in range(hb.G):
        st = _st6(hb, g)
        cid = st_all["cid"][g:g + 1].view(np.uint8).copy()
        sl = slice(g * NR, (g + 1) * NR)
        sid = hb.sid[g:g + 1].copy()
        rcm, step, ap = hb.remote_commit[sl].copy(), hb.lr_step[sl].copy(), hb.apply_offsets[sl].copy()
        ph = np.array([hb.prev_head[g] if "prev_head" in hb.arrays else 0], np.uint8)
        one = {k: io[k][g:g + 1].copy() for k in ("cid_offset", "req_id", "clt_id", "last_csm_idx",
                                                 "last_write_csm_idx", "events", "departed", "n_applied", "n_cfg")}
        la = io["last_applied"][3 * g:3 * g + 3].copy()
        oc = R.ref_vote_count(p(hb.group_ring(g)), hb.stride, p(st), p(cid), int(hb.self_idx[g]), NR, p(sid),
                              p(hb.vote_ack[sl].copy()), p(rcm), p(step), p(ap), p(ph), p(one["cid_offset"]),
                              int(io["cid_idx"][g]), p(one["req_id"]), p(one["clt_id"]), p(la), p(one["last_csm_idx"]),
                              p(one["last_write_csm_idx"]), p(one["events"]), p(one["departed"]), p(one["n_applied"]),
                              p(one["n_cfg"]))
        for k, i in (("head", 0), ("apply", 1), ("commit", 2), ("end", 3), ("tail", 4)):
            st_all[k][g] = st[i]
        st_all["cid"][g:g + 1] = cid.view(st_all.dtype["cid"])
        hb.sid[g] = sid[0]
        hb.remote_commit[sl], hb.lr_step[sl], hb.apply_offsets[sl] = rcm, step, ap
        if "prev_head" in hb.arrays:
            hb.prev_head[g] = ph[0]
        for k, v in one.items():
            io[k][g] = v[0]
        io["last_applied"][3 * g:3 * g + 3] = la
        io["outcome"][g] = oc
        bad += oc == 7
    return bad
