"""Host-side mirror of the reference's hot-path operations over HBM batches.

Method names follow the reference functions whose semantics the kernels
reproduce (paths relative to the reference tree):

  update_remote_logs        src/dare/dare_ibv_rc.c:1650-1822  (commit walk,
                            optional Adler-32 checksum, optional DARE median,
                            the lazy remote-commit publish)
  force_log_pruning         src/dare/dare_server.c:2069-2122  (APUS_COMMIT_FORCE_PRUNE)
  poll_vote_count           src/dare/dare_server.c:1327-1373
  poll_vote_requests        src/dare/dare_server.c:1526-1655
  log_pruning               src/dare/dare_server.c:1996-2067
  log_find_remote_end_offset src/include/dare/dare_log.h:367-394
  log_entries_to_nc_buf     src/include/dare/dare_log.h:339-359
  handle_lr_work_completion src/dare/dare_ibv_rc.c:3126-3196
  log_adjustment            src/dare/dare_ibv_rc.c:1292-1451

Every call goes through libapus_gpu (HIP kernels); nothing is computed here.
"""
import ctypes as C
import functools
import inspect

import numpy as np

from . import abi
from .batch import DET_DT, ptr


def _streamed(fn):
    """run the method's torch work (output allocation, uploads, read-backs)
    on the stream its kernels are launched on, so a caller-supplied stream
    orders everything (no zero-fill or copy on another stream can race it)"""
    sig = inspect.signature(fn)

    @functools.wraps(fn)
    def wrap(self, *a, **kw):
        st = sig.bind(self, *a, **kw).arguments.get("stream")
        with self._on(st):
            return fn(self, *a, **kw)
    return wrap


class Engine:
    def __init__(self, device=0):
        import torch
        self.torch = torch
        self.lib = abi.load_library()
        self.device = device
        torch.cuda.set_device(device)
        h = C.c_void_p()
        abi.check(self.lib.apus_ctx_create(device, C.byref(h)), "apus_ctx_create")
        self.ctx = h

    def close(self):
        if self.ctx:
            self.lib.apus_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self, stream=None):
        s = stream if stream is not None else self.torch.cuda.current_stream()
        return C.c_void_p(s.cuda_stream)

    def _on(self, stream):
        """context manager: torch work (uploads, downloads, temporaries) on
        the stream the kernels are launched on"""
        import contextlib
        return self.torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()

    def _z(self, G, dt, n=1):
        return self.torch.zeros(G * n, dtype=dt, device=f"cuda:{self.device}")

    # ------------------------------------------------------------------ gen
    @_streamed
    def gen(self, dbatch, cfg, stream=None):
        b = dbatch.struct()
        abi.check(self.lib.apus_gen_batch(self.ctx, C.byref(b), C.byref(cfg), self._stream(stream)),
                  "apus_gen_batch")

    # --------------------------------------------------------------- commit
    def alloc_commit_out(self, G, flags, nc_max=0):
        t = self.torch
        out = {"new_commit": self._z(G, t.int64), "committed": self._z(G, t.uint8),
               "n_entries": self._z(G, t.int32)}
        if flags & abi.COMMIT_CHECKSUM:
            out["digest"] = self._z(G, t.int32)
        if flags & abi.COMMIT_MEDIAN:
            out["median"] = self._z(G, t.int64)
        if flags & abi.COMMIT_PRUNE:             # log_pruning in the same pass (apus_prune_batch's outputs)
            out["new_head"] = self._z(G, t.int64)
            out["append_head"] = self._z(G, t.uint8)
            out["min_apply"] = self._z(G, t.int64)
        if flags & abi.COMMIT_NC:                # log_entries_to_nc_buf from the same pass
            assert nc_max > 0, "APUS_COMMIT_NC needs nc_max (determinants per group row)"
            out["nc_dets"] = self._z(G, t.uint8, nc_max * DET_DT.itemsize)
            out["nc_len"] = self._z(G, t.int32)
            out["nc_max"] = nc_max
        if flags & abi.COMMIT_LAST_IT:           # the local (idx, term) from the same pass
            out["last_idx_term"] = self._z(G, t.int64, 2)
        if flags & abi.COMMIT_VOTE:              # poll_vote_count in the same tail (apus_vote_batch's outputs)
            out["vote"] = {"won": self._z(G, t.uint8), "vote_count": self._z(G, t.uint8, 2),
                           "new_commit": self._z(G, t.int64), "voters": self._z(G, t.int16)}
        if flags & abi.COMMIT_RANK:              # poll_vote_requests in the same tail (apus_vote_rank_batch's)
            out["rank"] = {"outcome": self._z(G, t.uint8), "new_sid": self._z(G, t.int64),
                           "new_cid": self._z(G, t.uint8, 16), "cleared": self._z(G, t.int16)}
        if flags & abi.COMMIT_PUBLISH:           # update_remote_logs' lazy remote-commit publish
            out["publish"] = self._z(G, t.int16)
            out["ssn"] = self._z(G, t.int64)
        if flags & abi.COMMIT_FORCE_PRUNE:       # force_log_pruning (replaces log_pruning's outputs)
            out.setdefault("new_head", self._z(G, t.int64))
            out.setdefault("append_head", self._z(G, t.uint8))
            out.setdefault("min_apply", self._z(G, t.int64))
            out["force"] = {"action": self._z(G, t.uint8), "target": self._z(G, t.uint8),
                            "cfg_idx": self._z(G, t.int64), "req_id": self._z(G, t.int64),
                            "clt_id": self._z(G, t.int16)}
        return out

    def commit_struct(self, out):
        return abi.CommitOut(new_commit=ptr(out.get("new_commit")), committed=ptr(out.get("committed")),
                             n_entries=ptr(out.get("n_entries")), digest=ptr(out.get("digest")),
                             median=ptr(out.get("median")), new_head=ptr(out.get("new_head")),
                             append_head=ptr(out.get("append_head")), min_apply=ptr(out.get("min_apply")),
                             nc_dets=ptr(out.get("nc_dets")), nc_len=ptr(out.get("nc_len")),
                             nc_max=int(out.get("nc_max", 0)), last_idx_term=ptr(out.get("last_idx_term")),
                             vote=self.vote_struct(out.get("vote") or {}), rank=self.rank_struct(out.get("rank") or {}),
                             publish=ptr(out.get("publish")), ssn=ptr(out.get("ssn")),
                             force=self.force_struct(out.get("force") or {}))

    @staticmethod
    def force_struct(f):
        return abi.ForceOut(action=ptr(f.get("action")), target=ptr(f.get("target")), cfg_idx=ptr(f.get("cfg_idx")),
                            req_id=ptr(f.get("req_id")), clt_id=ptr(f.get("clt_id")))

    @staticmethod
    def vote_struct(v):
        return abi.VoteOut(won=ptr(v.get("won")), vote_count=ptr(v.get("vote_count")),
                           new_commit=ptr(v.get("new_commit")), voters=ptr(v.get("voters")))

    @staticmethod
    def rank_struct(r):
        return abi.RankOut(outcome=ptr(r.get("outcome")), new_sid=ptr(r.get("new_sid")),
                           new_cid=ptr(r.get("new_cid")), cleared=ptr(r.get("cleared")))

    def commit_walk_info(self, bstruct, flags):
        """the walk kernel apus_commit_batch launches for this batch and these
        flags: {"kind": lane|wave|segment, "hop", "dyn", "grid", "nc", "rows"}"""
        info = (C.c_uint32 * 6)()
        abi.check(self.lib.apus_commit_walk_info(self.ctx, C.byref(bstruct), flags, info), "apus_commit_walk_info")
        return {"kind": ("lane", "wave", "segment")[info[0]], "hop": bool(info[1]), "dyn": bool(info[2]),
                "grid": int(info[3]), "nc": bool(info[4]), "rows": bool(info[5])}

    def walk_kernel_name(self, bstruct, flags):
        """the walk kernel's name as rocprof lists it (template arguments)"""
        w = self.commit_walk_info(bstruct, flags)
        ck = "true" if flags & abi.COMMIT_CHECKSUM else "false"
        tf = lambda x: "true" if x else "false"   # noqa: E731
        if w["kind"] == "lane":
            return f"commit_lane_kernel<{ck}>"
        if w["kind"] == "segment":
            return f"commit_seg_kernel<{ck}, {tf(w['rows'])}, {tf(w['dyn'])}>"
        win = 12288 if w["hop"] else 9216          # kWinHop / kWin (apus_commit.hip)
        return f"commit_wave_kernel<{ck}, {win}, {tf(w['hop'])}, {4 if w['nc'] else 0}u, {tf(w['dyn'])}>"

    @_streamed
    def update_remote_logs(self, dbatch, flags=abi.COMMIT_WALK, out=None, stream=None, bstruct=None,
                           ostruct=None, nc_max=0):
        if out is None and ostruct is None:
            out = self.alloc_commit_out(dbatch.G, flags, nc_max)
        b = bstruct if bstruct is not None else dbatch.struct()
        o = ostruct if ostruct is not None else self.commit_struct(out)
        abi.check(self.lib.apus_commit_batch(self.ctx, C.byref(b), C.byref(o), flags, self._stream(stream)),
                  "apus_commit_batch")
        return out

    def set_commit(self, dbatch, commit):
        """log->commit = commit (int64 tensor [G]) on every group's state row:
        the caller's update after the commit rule (dare_ibv_rc.c:1744-1757)"""
        dbatch.arrays["state"].view(self.torch.int64).view(dbatch.G, 8)[:, 2].copy_(commit)

    @_streamed
    def commit_then_force(self, dbatch, flags, out=None, stream=None, bstruct=None):
        """a walking commit call and force_log_pruning, as the library takes
        them (apus_commit_batch refuses APUS_COMMIT_FORCE_PRUNE beside a walk:
        polling() runs apply_committed_entries between the two,
        dare_server.c:1100-1123): the commit call with `flags` less
        FORCE_PRUNE, log->commit = its new commit (set_commit), then the
        FORCE_PRUNE call on that log -- force_log_pruning on the log as given
        (apply as it is; apus_apply_batch between the two is the reference's
        full poll).  Statistics accumulate over both calls."""
        f1 = flags & ~abi.COMMIT_FORCE_PRUNE
        out = self.update_remote_logs(dbatch, f1, out=out, stream=stream, bstruct=bstruct)
        self.set_commit(dbatch, out["new_commit"])
        return self.update_remote_logs(dbatch, abi.COMMIT_FORCE_PRUNE, out=out, stream=stream, bstruct=bstruct)

    # ----------------------------------------------------------------- vote
    @_streamed
    def poll_vote_count(self, dbatch, stream=None):
        t = self.torch
        G = dbatch.G
        out = {"won": self._z(G, t.uint8), "vote_count": self._z(G, t.uint8, 2),
               "new_commit": self._z(G, t.int64), "voters": self._z(G, t.int16)}
        o = abi.VoteOut(won=ptr(out["won"]), vote_count=ptr(out["vote_count"]),
                        new_commit=ptr(out["new_commit"]), voters=ptr(out["voters"]))
        b = dbatch.struct()
        abi.check(self.lib.apus_vote_batch(self.ctx, C.byref(b), C.byref(o), self._stream(stream)),
                  "apus_vote_batch")
        return out

    @_streamed
    def last_idx_term(self, dbatch, stream=None, bstruct=None):
        out = self._z(dbatch.G, self.torch.int64, 2)
        b = bstruct if bstruct is not None else dbatch.struct()
        abi.check(self.lib.apus_last_idx_term_batch(self.ctx, C.byref(b), C.c_void_p(out.data_ptr()),
                                                    self._stream(stream)), "apus_last_idx_term_batch")
        return out

    @_streamed
    def poll_vote_requests(self, dbatch, derive_local=True, stream=None):
        t = self.torch
        G = dbatch.G
        b = dbatch.struct()
        lit = None
        if derive_local:
            lit = self.last_idx_term(dbatch, stream)
            b.last_idx_term = lit.data_ptr()
        out = {"outcome": self._z(G, t.uint8), "new_sid": self._z(G, t.int64),
               "new_cid": self._z(G, t.uint8, 16), "cleared": self._z(G, t.int16)}
        o = abi.RankOut(outcome=ptr(out["outcome"]), new_sid=ptr(out["new_sid"]),
                        new_cid=ptr(out["new_cid"]), cleared=ptr(out["cleared"]))
        abi.check(self.lib.apus_vote_rank_batch(self.ctx, C.byref(b), C.byref(o), self._stream(stream)),
                  "apus_vote_rank_batch")
        if lit is not None:
            out["last_idx_term"] = lit
        return out

    # -------------------------------------------------------------- pruning
    @_streamed
    def log_pruning(self, dbatch, stream=None, out=None, bstruct=None):
        t = self.torch
        G = dbatch.G
        if out is None:
            out = {"new_head": self._z(G, t.int64), "append_head": self._z(G, t.uint8),
                   "min_apply": self._z(G, t.int64)}
        o = abi.PruneOut(new_head=ptr(out["new_head"]), append_head=ptr(out["append_head"]),
                         min_apply=ptr(out["min_apply"]))
        b = bstruct if bstruct is not None else dbatch.struct()
        abi.check(self.lib.apus_prune_batch(self.ctx, C.byref(b), C.byref(o), self._stream(stream)),
                  "apus_prune_batch")
        return out

    # ----------------------------------------------------------- validation
    @_streamed
    def log_find_remote_end_offset(self, dbatch, dets, det_len, follower, max_dets, stream=None, leader=None):
        """dets: uint8 tensor [G*F*max_dets*24]; det_len int32 [G*F]; follower uint8 [G*F];
        leader: optional (dets, len, max) -- the leader's own NC determinants
        (log_entries_to_nc_buf / APUS_COMMIT_NC), read instead of gathering headers"""
        F = det_len.numel() // dbatch.G
        out = self._z(dbatch.G, self.torch.int64, F)
        nc = abi.NcBatch(n_followers=F, max_dets=max_dets, dets=dets.data_ptr(), det_len=det_len.data_ptr(),
                         follower=follower.data_ptr())
        if leader is not None:
            nc.leader_dets, nc.leader_len, nc.leader_max = leader[0].data_ptr(), leader[1].data_ptr(), int(leader[2])
        b = dbatch.struct()
        abi.check(self.lib.apus_validate_batch(self.ctx, C.byref(b), C.byref(nc), C.c_void_p(out.data_ptr()),
                                               self._stream(stream)), "apus_validate_batch")
        return out

    @_streamed
    def log_entries_to_nc_buf(self, dbatch, max_dets=abi.MAX_NC_ENTRIES, stream=None, bstruct=None):
        t = self.torch
        dets = self._z(dbatch.G, t.uint8, max_dets * DET_DT.itemsize)
        ln = self._z(dbatch.G, t.int32)
        b = bstruct if bstruct is not None else dbatch.struct()
        abi.check(self.lib.apus_nc_build_batch(self.ctx, C.byref(b), C.c_void_p(dets.data_ptr()), max_dets,
                                               C.c_void_p(ln.data_ptr()), self._stream(stream)),
                  "apus_nc_build_batch")
        return dets, ln

    # ----------------------------------------------- log append + persist
    @_streamed
    def log_append_entry(self, dbatch, entries, payload, max_entries, n_entries=None, term=None,
                         last_idx=None, stream=None, flags=0):
        """apus_append_batch: entries = uint8 tensor of APPEND_DT records
        [G*max_entries], payload = uint8 tensor; n_entries / term / last_idx
        optional device tensors (int32 / int64 / int64); flags: APPEND_*.
        Updates dbatch in place; returns {"idx", "last_idx"}."""
        t = self.torch
        G = dbatch.G
        out = {"idx": self._z(G, t.int64, max_entries),
               "last_idx": last_idx if last_idx is not None else self._z(G, t.int64)}
        ai = abi.AppendIn(entries=entries.data_ptr(), n_entries=ptr(n_entries), term=ptr(term),
                          payload=payload.data_ptr(), payload_bytes=payload.numel(), max_entries=max_entries,
                          flags=flags)
        ao = abi.AppendOut(idx=out["idx"].data_ptr(), last_idx=out["last_idx"].data_ptr())
        b = dbatch.struct()
        abi.check(self.lib.apus_append_batch(self.ctx, C.byref(b), C.byref(ai), C.byref(ao), self._stream(stream)),
                  "apus_append_batch")
        return out

    @_streamed
    def persist_new_entries(self, dbatch, old_end, limit=None, stream=None, flags=0):
        """apus_persist_batch: old_end int64 tensor [G*R] (in/out), limit
        optional int32 tensor [G*R]; flags: extra batch flags"""
        pi = abi.PersistIn(old_end=old_end.data_ptr(), limit=ptr(limit))
        b = dbatch.struct()
        b.flags |= flags
        abi.check(self.lib.apus_persist_batch(self.ctx, C.byref(b), C.byref(pi), self._stream(stream)),
                  "apus_persist_batch")
        return old_end

    # ----------------------------- the proxy's stable-storage records (8f.3)
    @_streamed
    def records_store(self, dbatch, cursor, dump, cap, dump_len, n_records=None, stream=None, flags=0):
        """apus_records_store_batch: cursor int64 [G] and dump_len int32 [G]
        (in/out), dump uint8 [G*cap]; n_records int32 [G] (out) or None;
        flags: extra batch flags (BATCH_VAR_LEN: the lane-per-group kernel)"""
        io = abi.RecordsIO(cursor=cursor.data_ptr(), dump=dump.data_ptr(), cap=cap, dump_len=dump_len.data_ptr(),
                           n_records=ptr(n_records))
        b = dbatch.struct()
        b.flags |= flags
        abi.check(self.lib.apus_records_store_batch(self.ctx, C.byref(b), C.byref(io), self._stream(stream)),
                  "apus_records_store_batch")
        return dump_len

    @_streamed
    def records_load(self, dump, stride, size, max_plan, stream=None, flags=0):
        """apus_records_load_batch over n = size.numel() dumps at dump +
        k*stride: returns device tensors plan (uint8 [n*max_plan*16]),
        n_records, counts [n*3], status, stop"""
        t = self.torch
        n = size.numel()
        out = {"plan": self._z(n, t.uint8, 16 * max(max_plan, 1)), "n_records": self._z(n, t.int32),
               "counts": self._z(n, t.int32, 3), "status": self._z(n, t.int32), "stop": self._z(n, t.int32)}
        io = abi.RecordsLoadIO(dump=dump.data_ptr(), stride=stride, size=size.data_ptr(), n=n,
                               plan=out["plan"].data_ptr() if max_plan else None, max_plan=max_plan, flags=flags,
                               n_records=out["n_records"].data_ptr(), counts=out["counts"].data_ptr(),
                               status=out["status"].data_ptr(), stop=out["stop"].data_ptr())
        abi.check(self.lib.apus_records_load_batch(self.ctx, C.byref(io), self._stream(stream)),
                  "apus_records_load_batch")
        return out

    # ------------------------------------------------ apply / config scan
    def _io_dev(self, io, keys):
        """numpy or torch arrays -> device tensors (numpy inputs are copied)"""
        t = self.torch
        d = {}
        for k in keys:
            v = io.get(k)
            if v is None:
                d[k] = None
            elif isinstance(v, np.ndarray):
                d[k] = t.from_numpy(np.ascontiguousarray(v).view(np.uint8).copy()).to(self.device)
            else:
                d[k] = v
        return d

    @staticmethod
    def _io_host(io, d):
        # scalars (max_dets, max_cfg) and absent columns pass through unchanged;
        # .cpu() runs on the current stream, which the callers set to the
        # launch stream (self._on), so it waits for the kernel
        out = {k: v for k, v in io.items() if k not in d}
        for k, v in d.items():
            if v is None:
                continue
            ref = io.get(k)
            out[k] = v.cpu().numpy().view(ref.dtype) if isinstance(ref, np.ndarray) else v
        return out

    @_streamed
    def poll_config_entries(self, dbatch, io, stream=None, bstruct=None):
        """apus_config_scan_batch.  io: dict of cid_offset, cid_idx, req_id,
        clt_id (+ departed) as numpy (returned as numpy) or device tensors;
        bstruct: the batch struct (its flags choose the kernel)"""
        keys = ("cid_offset", "cid_idx", "req_id", "clt_id", "departed")
        d = self._io_dev(io, keys)
        c = abi.ConfigIO(**{k: ptr(d[k]) for k in keys})
        b = dbatch.struct() if bstruct is None else bstruct
        abi.check(self.lib.apus_config_scan_batch(self.ctx, C.byref(b), C.byref(c), self._stream(stream)),
                  "apus_config_scan_batch")
        return self._io_host(io, d)

    @_streamed
    def apply_committed_entries(self, dbatch, io, stream=None):
        """apus_apply_batch.  io: dict as oracle.apply_io builds it (numpy,
        returned as numpy) or device tensors, plus max_cfg"""
        keys = ("req_id", "clt_id", "last_applied", "last_csm_idx", "n_applied", "departed", "events",
                "cfg_entries", "cfg_payload", "n_cfg")
        d = self._io_dev(io, keys)
        a = abi.ApplyIO(max_cfg=int(io["max_cfg"]), **{k: ptr(d[k]) for k in keys})
        b = dbatch.struct()
        abi.check(self.lib.apus_apply_batch(self.ctx, C.byref(b), C.byref(a), self._stream(stream)),
                  "apus_apply_batch")
        return self._io_host(io, d)

    @_streamed
    def become_leader(self, dbatch, io, stream=None, bstruct=None):
        """apus_vote_win_batch: the rest of poll_vote_count after the tally
        (dare_server.c:1355-1362,1389-1510).  io: dict as oracle.win_io builds
        it (numpy, returned as numpy) or device tensors -- won / voters /
        new_commit are the tally's outputs (poll_vote_count's dict, or the
        commit call's "vote").  dbatch (sid, state, ring, remote_commit,
        lr_step, apply_offsets, prev_head) is updated in place."""
        d = self._io_dev(io, abi.WIN_KEYS)
        w = abi.WinIO(**{k: ptr(d[k]) for k in abi.WIN_KEYS})
        b = dbatch.struct() if bstruct is None else bstruct
        abi.check(self.lib.apus_vote_win_batch(self.ctx, C.byref(b), C.byref(w), self._stream(stream)),
                  "apus_vote_win_batch")
        return self._io_host(io, d)

    # ------------------------------------ replication step machine (8f.2)
    LR_KEYS =("send_flag", "send_count", "wc", "rc_connected", "nc_len", "nc_dets", "ssn", "post")

    def _lr(self, fn, name, dbatch, io, stream, need_max_dets=False):
        if need_max_dets and "max_dets" not in io:
            raise KeyError(f"{name}: io['max_dets'] is required (the row length of nc_dets)")
        d = self._io_dev(io, self.LR_KEYS)
        li = abi.LrIO(max_dets=int(io.get("max_dets", 0)), **{k: ptr(d[k]) for k in self.LR_KEYS})
        if not need_max_dets:
            li.nc_dets = None                     # the completion never reads the NC buffer
        b = dbatch.struct()
        abi.check(fn(self.ctx, C.byref(b), C.byref(li), self._stream(stream)), name)
        return self._io_host(io, d)

    @_streamed
    def handle_lr_work_completion(self, dbatch, io, stream=None):
        """apus_lr_completion_batch.  io: dict of send_flag, send_count, wc
        ([G*R] numpy, returned as numpy, or device tensors); dbatch.lr_step
        is updated in place"""
        return self._lr(self.lib.apus_lr_completion_batch, "apus_lr_completion_batch", dbatch, io, stream)

    @_streamed
    def log_adjustment(self, dbatch, io, stream=None):
        """apus_log_adjust_batch.  io: dict as oracle.lr_io builds it; dbatch
        state.commit, lr_step, remote_commit and remote_end are updated in place"""
        return self._lr(self.lib.apus_log_adjust_batch, "apus_log_adjust_batch", dbatch, io, stream,
                        need_max_dets=True)

    # ---------------------------------------------------------------- stats
    @_streamed
    def stats_reset(self, stream=None):
        abi.check(self.lib.apus_stats_reset(self.ctx, self._stream(stream)), "apus_stats_reset")

    def stats_ptr(self):
        return self.lib.apus_ctx_stats(self.ctx)

    @_streamed
    def stats(self, stream=None):
        arr = (C.c_uint64 * abi.STAT_COUNT)()
        abi.check(self.lib.apus_stats_read(self.ctx, arr, self._stream(stream)), "apus_stats_read")
        return np.array(arr[:], dtype=np.uint64)
