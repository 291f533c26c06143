"""The C-ABI boundary, without a GPU: libapus_gpu.so loads, exports every
function include/apus_gpu.h declares, and the mirror structs have the
reference's byte layout (checked against the reference's own headers through
oracle/_ref when the reference tree is present)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "apus_gpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(apus_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_function(pkg):
    lib = pkg.load_library()
    names = declared_functions()
    assert len(names) >= 25
    nm = subprocess.run(["nm", "-D", "--defined-only", pkg.abi.LIB_PATH], capture_output=True, text=True,
                        check=True).stdout
    exported = set(re.findall(r"\bT (apus_\w+)", nm))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        getattr(lib, n)
    # and the ctypes mirror declares exactly these
    assert sorted(n for n, _, _ in pkg.abi.SIGNATURES) == names
    assert lib.apus_version().startswith(b"libapus_gpu")


def test_no_cpu_fallback_symbols(pkg):
    """the product library links no oracle code and has no host compute path"""
    nm = subprocess.run(["nm", "-D", pkg.abi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "apus_oracle" not in nm and "ref_" not in nm
    ldd = subprocess.run(["ldd", pkg.abi.LIB_PATH], capture_output=True, text=True).stdout
    assert "liboracle" not in ldd and "libapusref" not in ldd


SIZES = {"Cid": 16, "LogEntry": 64, "EntryDet": 24, "NcBuf": 24584, "LogHeader": 319656, "Server": 40,
         "ServerConfig": 56, "VoteReq": 40, "LogOffsets": 32, "SmRep": 24, "CtrlData": 1880,
         "GroupState": 64, "Batch": 168, "CommitOut": 216, "VoteOut": 32,
         "RankOut": 32, "NcBatch": 56, "ForceOut": 40, "WinIO": 120}


@pytest.mark.parametrize("name,size", sorted(SIZES.items()))
def test_struct_sizes(pkg, name, size):
    assert C.sizeof(getattr(pkg.abi, name)) == size


def test_layout_matches_reference_headers(pkg, ref):
    """offsets of our mirrors == offsetof() in the reference's dare_log.h /
    dare_config.h (ref_layout is compiled from /root/reference)"""
    a = pkg.abi
    v = np.zeros(64, np.uint64)
    n = ref.ref_layout(C.c_void_p(v.ctypes.data), 64)
    got = [int(x) for x in v[:n]]
    E, L, Cd, S = a.LogEntry, a.LogHeader, a.Cid, a.ServerConfig
    mine = [C.sizeof(E), E.idx.offset, E.term.offset, E.req_id.offset, E.clt_id.offset, E.type.offset,
            E.sender.offset, E.reply.offset, E.data.offset, C.sizeof(a.EntryDet), C.sizeof(a.NcBuf),
            a.NcBuf.entries.offset, C.sizeof(L), L.head.offset, L.apply.offset, L.commit.offset,
            L.end.offset, L.tail.offset, L.old_end.offset, L.old_commit.offset, L.len.offset,
            L.nc_buf.offset, C.sizeof(L), C.sizeof(Cd), Cd.epoch.offset, Cd.size.offset, Cd.state.offset,
            Cd.bitmask.offset, C.sizeof(S), S.cid.offset, S.cid_offset.offset, S.cid_idx.offset,
            S.req_id.offset, S.servers.offset, S.clt_id.offset, S.idx.offset, S.len.offset,
            C.sizeof(a.LogOffsets), 16384 * 4096, 13, 1024]
    assert got == mine


def test_header_compiles_as_c_and_matches(tmp_path):
    """include/apus_gpu.h is plain C (gcc -std=c99) with the documented sizes"""
    src = tmp_path / "t.c"
    src.write_text('''#include "apus_gpu.h"
#include <stddef.h>
_Static_assert(sizeof(apus_log_entry_t) == 64, "entry");
_Static_assert(offsetof(apus_log_entry_t, reply) == 28, "reply");
_Static_assert(offsetof(apus_log_entry_t, data) == 48, "data");
_Static_assert(offsetof(apus_log_t, entries) == 319656, "log");
_Static_assert(sizeof(apus_ctrl_data_t) == 1880, "ctrl");
_Static_assert(offsetof(apus_ctrl_data_t, vote_ack) == 1464, "vote_ack");
_Static_assert(offsetof(apus_ctrl_data_t, apply_offsets) == 1672, "apply");
_Static_assert(sizeof(apus_server_config_t) == 56, "cfg");
_Static_assert(sizeof(apus_group_state_t) == 64, "state");
_Static_assert(sizeof(apus_batch_t) == 168 && offsetof(apus_batch_t, cid) == 144 &&
               offsetof(apus_batch_t, rc_connected) == 152 && offsetof(apus_batch_t, vote_sit) == 160, "batch");
_Static_assert(APUS_LOG_HDR_BYTES == offsetof(apus_log_t, entries), "log image header");
_Static_assert(sizeof(apus_commit_out_t) == 216 && offsetof(apus_commit_out_t, nc_max) == 80 &&
               offsetof(apus_commit_out_t, last_idx_term) == 88 && offsetof(apus_commit_out_t, vote) == 96 &&
               offsetof(apus_commit_out_t, rank) == 128 && offsetof(apus_commit_out_t, publish) == 160 &&
               offsetof(apus_commit_out_t, ssn) == 168 && offsetof(apus_commit_out_t, force) == 176,
               "commit out");
_Static_assert(sizeof(apus_force_out_t) == 40 && APUS_ABI_VERSION == 7, "force out");
_Static_assert(sizeof(apus_win_io_t) == 120 && offsetof(apus_win_io_t, outcome) == 80, "win io");
_Static_assert(sizeof(apus_nc_batch_t) == 56 && offsetof(apus_nc_batch_t, leader_max) == 48, "nc batch");
int main(void) { return 0; }
''')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src),
                    "-o", str(tmp_path / "t")], check=True)


def test_batch_dtypes(pkg):
    b = pkg.batch
    assert b.STATE_DT.itemsize == C.sizeof(pkg.abi.GroupState)
    assert b.VOTE_REQ_DT.itemsize == C.sizeof(pkg.abi.VoteReq)
    assert b.DET_DT.itemsize == C.sizeof(pkg.abi.EntryDet)
    assert b.ring_stride_for(16384) % 16 == 0 and b.ring_stride_for(16384) >= 16384 + 16


def test_abi_version(pkg):
    """the library reports the layout revision the ctypes mirror is written for"""
    lib = pkg.abi.load_library()
    assert lib.apus_abi_version() == pkg.abi.ABI_VERSION
    assert b"ABI %d" % pkg.abi.ABI_VERSION in lib.apus_version()


def test_header_constants_match_ctypes_mirror(pkg):
    """every flag / code #define of include/apus_gpu.h that abi.py mirrors
    (APUS_X -> abi.X) has the same value there"""
    import re
    abi = pkg.abi
    text = open(os.path.join(ROOT, "include", "apus_gpu.h")).read()
    seen = 0
    for name, val in re.findall(r"^#define\s+APUS_([A-Z0-9_]+)\s+\(?(-?(?:0x[0-9a-fA-F]+|\d+))u?\)?", text, re.M):
        if hasattr(abi, name):
            assert getattr(abi, name) == int(val, 0), name
            seen += 1
    for must in ("BATCH_TAIL_ROWS", "COMMIT_PUBLISH", "COMMIT_FORCE_PRUNE", "FORCE_REMOVE", "FORCE_REFUSED",
                 "ABI_VERSION", "WIN_STABLE", "WIN_UNDEFINED"):
        assert hasattr(abi, must), must
    assert seen >= 30, seen


def test_batched_entries_refuse_null_arguments(pkg):
    """every batched entry point (and the communicator / marker calls) given
    no context, batch or I/O struct returns APUS_ERROR -- the reference's
    RC_ERROR, 1 (dare_ibv_rc.c:27-29) -- before it touches a device: this
    runs without a GPU"""
    import ctypes as C
    abi = pkg.abi
    lib = abi.load_library()
    checked = 0
    for name, _, argtypes in abi.SIGNATURES:
        if not (name.endswith("_batch") or name in ("apus_ctx_destroy", "apus_commit_mark_walk",
                                                       "apus_commit_mark_tail", "apus_commit_walk_info",
                                                       "apus_stats_allreduce", "apus_allreduce_stats",
                                                       "apus_comm_init_rank")):
            continue
        args = [0 if t in (C.c_int, C.c_uint32, C.c_uint64, C.c_int64, C.c_uint8, C.c_uint16) else None
                for t in argtypes]
        assert getattr(lib, name)(*args) == abi.APUS_ERROR, name
        checked += 1
    assert checked >= 24
