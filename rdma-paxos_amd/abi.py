"""ctypes mirror of include/apus_gpu.h (the libapus_gpu C ABI).

Python is plumbing here: it allocates device memory (torch), picks streams and
calls the C ABI.  Every result comes from the HIP kernels in csrc/.  If the
shared library is missing the import fails loudly -- there is no CPU fallback.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# APUS_GPU_LIB: load another build of the library (kernel experiments, scripts/build_exp.sh)
_DEFAULT_LIB = os.path.join(HERE, "libapus_gpu.so")
LIB_PATH = os.environ.get("APUS_GPU_LIB") or _DEFAULT_LIB

APUS_OK, APUS_ERROR, APUS_INSUCCESS = 0, 1, -1
MAX_SERVER_COUNT = 13
MAX_NC_ENTRIES = 1024
ENTRY_HDR = 64
NOOP, CSM, CONFIG, HEAD = 0, 1, 2, 3
CID_STABLE, CID_TRANSIT, CID_EXTENDED = 0, 1, 2
LR_GET_WRITE, LR_GET_NCE_LEN, LR_GET_NCE, LR_SET_END, LR_UPDATE_LOG, LR_UPDATE_END = 1, 2, 3, 4, 5, 6
PERMANENT_FAILURE = 2

COMMIT_WALK, COMMIT_CHECKSUM, COMMIT_MEDIAN, COMMIT_PRUNE, COMMIT_NC = 0x1, 0x2, 0x4, 0x8, 0x10
COMMIT_STATS_FRESH = 0x20
COMMIT_LAST_IT = 0x40
COMMIT_VOTE = 0x80
COMMIT_RANK = 0x100
COMMIT_PUBLISH = 0x200
COMMIT_FORCE_PRUNE = 0x400
FORCE_NONE, FORCE_PRUNE, FORCE_REMOVE, FORCE_REFUSED = 0, 1, 2, 3
ABI_VERSION = 7
BATCH_LANE_IMPL = 0x1
BATCH_SHORT_WALKS = 0x2
BATCH_LOG_IMAGE = 0x4
BATCH_VAR_LEN = 0x8
BATCH_TAIL_ROWS = 0x10
APPEND_PER_GROUP = 0x1
LOG_HDR_BYTES = 319656
RANK_LEADER_KNOWN, RANK_ADOPT_HB, RANK_NO_BETTER, RANK_RAISE_TERM, RANK_VOTE = 0, 1, 2, 3, 4
(STAT_DECISIONS, STAT_COMMITTED, STAT_ADVANCED, STAT_VOTES_WON, STAT_MISMATCHES,
 STAT_CORRUPT, STAT_MIN_WATERMARK, STAT_SLOW, STAT_APPEND_SLOW) = range(9)
STAT_COUNT = 9

u8, u16, u32, u64, vp = C.c_uint8, C.c_uint16, C.c_uint32, C.c_uint64, C.c_void_p


class Cid(C.Structure):
    _fields_ = [("epoch", u64), ("size", u8 * 2), ("state", u8), ("pad", u8 * 1), ("bitmask", u32)]


class CmdData(C.Structure):
    _fields_ = [("len", u16), ("cmd", u8 * 14)]


class EntryData(C.Union):
    _fields_ = [("cmd", CmdData), ("cid", Cid), ("head", u64)]


class LogEntry(C.Structure):
    _fields_ = [("idx", u64), ("term", u64), ("req_id", u64), ("clt_id", u16), ("type", u8),
                ("sender", u8), ("reply", u8 * MAX_SERVER_COUNT), ("data", EntryData)]


class EntryDet(C.Structure):
    _fields_ = [("idx", u64), ("term", u64), ("offset", u64)]


class NcBuf(C.Structure):
    _fields_ = [("len", u64), ("entries", EntryDet * MAX_NC_ENTRIES)]


class LogHeader(C.Structure):
    """dare_log_t without the flexible entries[] array."""
    _fields_ = [("head", u64), ("apply", u64), ("commit", u64), ("end", u64), ("tail", u64),
                ("old_end", u64), ("old_commit", u64), ("len", u64),
                ("nc_buf", NcBuf * MAX_SERVER_COUNT)]


class Server(C.Structure):
    _fields_ = [("next_wr_id", u64), ("cached_end_offset", u64), ("last_get_read_ssn", u64),
                ("ep", vp), ("fail_count", u8), ("next_lr_step", u8), ("send_flag", u8),
                ("send_count", u8)]


class ServerConfig(C.Structure):
    _fields_ = [("cid", Cid), ("cid_offset", u64), ("cid_idx", u64), ("req_id", u64),
                ("servers", C.POINTER(Server)), ("clt_id", u16), ("idx", u8), ("len", u8)]


class VoteReq(C.Structure):
    _fields_ = [("sid", u64), ("index", u64), ("term", u64), ("cid", Cid)]


class LogOffsets(C.Structure):
    _fields_ = [("head", u64), ("apply", u64), ("commit", u64), ("end", u64)]


class SmRep(C.Structure):
    _fields_ = [("sid", u64), ("raddr", u64), ("rkey", u32), ("len", u32)]


R13 = MAX_SERVER_COUNT


class CtrlData(C.Structure):
    _fields_ = [("sid", u64), ("vote_req", VoteReq * R13), ("log_offsets", LogOffsets * R13),
                ("sm_rep", SmRep * R13), ("sm_req", u64 * R13), ("hb", u64 * R13),
                ("vote_ack", u64 * R13), ("rsid", u64 * R13), ("apply_offsets", u64 * R13),
                ("prv_data", u64 * R13)]


class GroupState(C.Structure):
    _fields_ = [("head", u64), ("apply", u64), ("commit", u64), ("end", u64), ("tail", u64),
                ("len", u64), ("cid", Cid)]


class Batch(C.Structure):
    _fields_ = [("n_groups", u64), ("n_replicas", u32), ("flags", u32), ("ring_stride", u64),
                ("ring", vp), ("state", vp), ("self_idx", vp), ("remote_end", vp),
                ("remote_commit", vp), ("lr_step", vp), ("fail_count", vp), ("vote_ack", vp),
                ("apply_offsets", vp), ("vote_req", vp), ("hb", vp), ("sid", vp),
                ("last_idx_term", vp), ("prev_head", vp), ("abs_base", vp), ("cid", vp), ("rc_connected", vp),
                ("vote_sit", vp)]


class VoteOut(C.Structure):
    _fields_ = [("won", vp), ("vote_count", vp), ("new_commit", vp), ("voters", vp)]


class RankOut(C.Structure):
    _fields_ = [("outcome", vp), ("new_sid", vp), ("new_cid", vp), ("cleared", vp)]


class ForceOut(C.Structure):
    _fields_ = [("action", vp), ("target", vp), ("cfg_idx", vp), ("req_id", vp), ("clt_id", vp)]


class CommitOut(C.Structure):
    _fields_ = [("new_commit", vp), ("committed", vp), ("n_entries", vp), ("digest", vp),
                ("median", vp), ("new_head", vp), ("append_head", vp), ("min_apply", vp),
                ("nc_dets", vp), ("nc_len", vp), ("nc_max", u32), ("pad", u32), ("last_idx_term", vp),
                ("vote", VoteOut), ("rank", RankOut), ("publish", vp), ("ssn", vp), ("force", ForceOut)]


class PruneOut(C.Structure):
    _fields_ = [("new_head", vp), ("append_head", vp), ("min_apply", vp)]


class NcBatch(C.Structure):
    _fields_ = [("n_followers", u32), ("max_dets", u32), ("dets", vp), ("det_len", vp),
                ("follower", vp), ("leader_dets", vp), ("leader_len", vp), ("leader_max", u32), ("pad", u32)]


class GenCfg(C.Structure):
    _fields_ = [("seed", u64), ("gid_base", u64), ("n_entries", u32), ("n_history", u32),
                ("len_min", u32), ("len_max", u32), ("ring_len", u32), ("p_full_ack", u32),
                ("straggler", u32), ("type_mix", u32), ("cid_mix", u32), ("garbage_reply", u32),
                ("self_random", u32), ("p_vote_ack", u32), ("fill_garbage", u32), ("hist_len_max", u32)]


class AppendEntry(C.Structure):
    _fields_ = [("req_id", u64), ("data_off", u64), ("clt_id", u16), ("type", u8), ("pad", u8 * 5)]


class AppendIn(C.Structure):
    _fields_ = [("entries", vp), ("n_entries", vp), ("term", vp), ("payload", vp),
                ("payload_bytes", u64), ("max_entries", u32), ("flags", u32)]


class AppendOut(C.Structure):
    _fields_ = [("idx", vp), ("last_idx", vp)]


class PersistIn(C.Structure):
    _fields_ = [("old_end", vp), ("limit", vp)]


class ConfigIO(C.Structure):
    """apus_config_io_t (poll_config_entries)"""
    _fields_ = [("cid_offset", vp), ("cid_idx", vp), ("req_id", vp), ("clt_id", vp), ("departed", vp)]


class ApplyIO(C.Structure):
    """apus_apply_io_t (apply_committed_entries)"""
    _fields_ = [("req_id", vp), ("clt_id", vp), ("last_applied", vp), ("last_csm_idx", vp),
                ("n_applied", vp), ("departed", vp), ("events", vp), ("cfg_entries", vp),
                ("cfg_payload", vp), ("n_cfg", vp), ("max_cfg", C.c_uint32), ("pad", C.c_uint32)]


class WinIO(C.Structure):
    """apus_win_io_t (poll_vote_count's election-win transition)"""
    _fields_ = [("won", vp), ("voters", vp), ("new_commit", vp), ("cid_offset", vp), ("cid_idx", vp),
                ("req_id", vp), ("clt_id", vp), ("last_applied", vp), ("last_csm_idx", vp),
                ("last_write_csm_idx", vp), ("outcome", vp), ("events", vp), ("departed", vp),
                ("n_applied", vp), ("n_cfg", vp)]


WIN_KEYS = ("won", "voters", "new_commit", "cid_offset", "cid_idx", "req_id", "clt_id", "last_applied",
            "last_csm_idx", "last_write_csm_idx", "outcome", "events", "departed", "n_applied", "n_cfg")
(WIN_NOT_CANDIDATE, WIN_LOST, WIN_CONFIG, WIN_NOOP, WIN_TRANSIT, WIN_STABLE, WIN_UNDEFINED,
 WIN_CORRUPT) = range(8)


class LrIO(C.Structure):
    """apus_lr_io_t (handle_lr_work_completion / log_adjustment)"""
    _fields_ = [("send_flag", vp), ("send_count", vp), ("wc", vp), ("rc_connected", vp), ("nc_len", vp),
                ("nc_dets", vp), ("ssn", vp), ("post", vp), ("max_dets", u32), ("pad", u32)]


class RecordsIO(C.Structure):
    """apus_records_io_t (stablestorage_save_request over persist_new_entries' walk)"""
    _fields_ = [("cursor", vp), ("dump", vp), ("cap", u64), ("dump_len", vp), ("n_records", vp)]


class RecordRef(C.Structure):
    _fields_ = [("offset", u32), ("data_len", u32), ("connection_id", u16), ("action", u8), ("pad", u8 * 5)]


class RecordsLoadIO(C.Structure):
    """apus_records_load_io_t (stablestorage_load_records)"""
    _fields_ = [("dump", vp), ("stride", u64), ("size", vp), ("n", u64), ("plan", vp), ("max_plan", u32),
                ("flags", u32), ("n_records", vp), ("counts", vp), ("status", vp), ("stop", vp)]


REC_CONNECT_BYTES, REC_SEND_BYTES, REC_DATA_OFF = 4, 24, 8
PROXY_CONNECT, PROXY_SEND, PROXY_CLOSE = 4, 5, 6

WC_NONE, WC_SUCCESS, WC_FAILED, WC_STALE = 0, 1, 2, 3
LR_POST_NONE, LR_POST_READ_NC_LEN, LR_POST_READ_NC, LR_POST_WRITE_END = 0, 1, 2, 3
EV_CFG_REPLY, EV_JOIN_REPLY, EV_SELF_REMOVED, EV_CFG_FULL = 1, 2, 4, 8


P = C.POINTER
# (name, restype, argtypes) of every exported symbol of include/apus_gpu.h
SIGNATURES = [
    ("apus_version", C.c_char_p, []),
    ("apus_abi_version", C.c_int, []),
    ("apus_set_log", None, [vp]),
    ("apus_ctx_create", C.c_int, [C.c_int, P(vp)]),
    ("apus_ctx_destroy", C.c_int, [vp]),
    ("apus_ctx_stats", vp, [vp]),
    ("apus_stats_reset", C.c_int, [vp, vp]),
    ("apus_stats_read", C.c_int, [vp, P(u64), vp]),
    ("apus_commit_batch", C.c_int, [vp, P(Batch), P(CommitOut), u32, vp]),
    ("apus_commit_mark_walk", C.c_int, [vp, vp, vp]),
    ("apus_commit_mark_tail", C.c_int, [vp, vp, vp]),
    ("apus_commit_walk_info", C.c_int, [vp, P(Batch), u32, vp]),
    ("apus_vote_batch", C.c_int, [vp, P(Batch), P(VoteOut), vp]),
    ("apus_vote_rank_batch", C.c_int, [vp, P(Batch), P(RankOut), vp]),
    ("apus_last_idx_term_batch", C.c_int, [vp, P(Batch), vp, vp]),
    ("apus_prune_batch", C.c_int, [vp, P(Batch), P(PruneOut), vp]),
    ("apus_validate_batch", C.c_int, [vp, P(Batch), P(NcBatch), vp, vp]),
    ("apus_nc_build_batch", C.c_int, [vp, P(Batch), vp, u32, vp, vp]),
    ("apus_append_batch", C.c_int, [vp, P(Batch), P(AppendIn), P(AppendOut), vp]),
    ("apus_persist_batch", C.c_int, [vp, P(Batch), P(PersistIn), vp]),
    ("apus_config_scan_batch", C.c_int, [vp, P(Batch), P(ConfigIO), vp]),
    ("apus_apply_batch", C.c_int, [vp, P(Batch), P(ApplyIO), vp]),
    ("apus_vote_win_batch", C.c_int, [vp, P(Batch), P(WinIO), vp]),
    ("apus_lr_completion_batch", C.c_int, [vp, P(Batch), P(LrIO), vp]),
    ("apus_log_adjust_batch", C.c_int, [vp, P(Batch), P(LrIO), vp]),
    ("apus_gen_batch", C.c_int, [vp, P(Batch), P(GenCfg), vp]),
    ("apus_records_store_batch", C.c_int, [vp, P(Batch), P(RecordsIO), vp]),
    ("apus_records_load_batch", C.c_int, [vp, P(RecordsLoadIO), vp]),
    ("apus_comm_get_unique_id", C.c_int, [C.c_char_p]),
    ("apus_comm_init_rank", C.c_int, [vp, C.c_int, C.c_char_p, C.c_int]),
    ("apus_stats_allreduce", C.c_int, [vp, vp]),
    ("apus_allreduce_stats", C.c_int, [vp, vp]),
    ("apus_log_new", C.c_int, [u64, P(vp)]),
    ("apus_log_free", C.c_int, [vp]),
    ("apus_scalar_path_stats", C.c_int, [P(u64), P(u64), P(u64), P(u32)]),
    ("apus_commit_reply_walk", C.c_int, [vp, P(ServerConfig), P(u64), P(C.c_int)]),
    ("apus_commit_median", C.c_int, [vp, P(ServerConfig), P(CtrlData), P(u64)]),
    ("apus_vote_tally", C.c_int, [vp, P(ServerConfig), P(CtrlData), P(u8), P(u64), P(u16)]),
    ("apus_vote_rank", C.c_int, [vp, P(ServerConfig), P(CtrlData), P(u8), P(u64), P(Cid), P(u16)]),
    ("apus_min_apply", C.c_int, [vp, P(ServerConfig), P(CtrlData), C.c_int, P(u64), P(C.c_int)]),
    ("apus_find_remote_end", C.c_int, [vp, P(NcBuf), P(u64)]),
    ("apus_log_adjustment", C.c_int, [vp, P(ServerConfig), P(CtrlData), u16, P(u64), P(u8)]),
    ("apus_publish_commit", C.c_int, [vp, P(ServerConfig), P(CtrlData), u16, P(u64), P(u16)]),
    ("apus_force_log_pruning", C.c_int, [vp, P(ServerConfig), P(CtrlData), P(C.c_int), P(u8), P(u64), P(u64),
                                         P(C.c_int)]),
    ("apus_lr_work_completion", C.c_int, [P(Server), C.c_int]),
    ("apus_entries_to_nc_buf", C.c_int, [vp, P(NcBuf)]),
]

_lib = None


def load_library(path=None):
    """Load libapus_gpu.so (built by __graft_entry__.build()).  Raises if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"libapus_gpu.so not built at {p}: run __graft_entry__.build()")
    lib = C.CDLL(p)
    for name, res, args in SIGNATURES:
        f = getattr(lib, name, None)
        if f is None:
            # an experimental build of an older source (APUS_GPU_LIB, A/B timing
            # only) may lack a newer entry point; the product library may not
            if os.environ.get("APUS_GPU_LIB") and p != _DEFAULT_LIB:
                continue
            raise RuntimeError(f"{p} does not export {name}")
        f.restype = res
        f.argtypes = args
    # the structs above are this layout revision (apus_gpu.h APUS_ABI_VERSION)
    if hasattr(lib, "apus_abi_version") and lib.apus_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{p}: ABI {lib.apus_abi_version()} != {ABI_VERSION} of abi.py")
    if path is None:
        _lib = lib
    return lib


def check(rc, what):
    if rc != APUS_OK:
        raise RuntimeError(f"{what} failed with rc={rc}")
