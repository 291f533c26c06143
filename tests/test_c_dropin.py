"""The drop-in boundary from C: examples/dare_poll.c, a C program
linked against libapus_gpu.so, builds one leader's dare_log_t (apus_log_new:
pinned mapped memory the GPU reads in place), server_config_t and
ctrl_data_t as the reference lays them out and calls the scalar drop-ins in
polling()'s order -- the commit walk, the median, the publish on the walk's
commit, the pruning minimum, the vote tally, log_entries_to_nc_buf and
log_find_remote_end_offset on a follower's buffer.  It dumps the inputs
before any call; this test runs the reference's own code (oracle/_ref: its
compiled dare_log.h with the transcribed loop bodies) on the dump and
requires every result to be equal.  Seeds cover batches that wrap (ghost
headers, header wraps), failing followers and missing vote acks.
"""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "dare_poll")
LEN, R = 16384, 3


def _parse(path):
    b = np.fromfile(path, np.uint8)
    o = 0

    def take(n):
        nonlocal o
        v = b[o:o + n]
        o += n
        return v
    hdr = take(64).view(np.uint64)
    st6 = np.array([hdr[0], hdr[1], hdr[2], hdr[3], hdr[4], hdr[7]], np.uint64)
    ring = take(LEN).copy()
    cfg = take(56)
    cid = cfg[:16].copy()
    self_ = int(cfg[50])
    srv = take(13 * 40).reshape(13, 40)
    fail, step = srv[:R, 32].copy(), srv[:R, 33].copy()
    ctrl = take(1880)
    lo = ctrl[528:528 + 13 * 32].view(np.uint64).reshape(13, 4)
    rend, rcommit = lo[:R, 3].copy(), lo[:R, 2].copy()
    vote_ack = ctrl[1464:1464 + 104].view(np.uint64)[:R].copy()
    apply = ctrl[1672:1672 + 104].view(np.uint64)[:R].copy()
    n = int(take(8).view(np.uint64)[0])
    dets = take(24 * n).view(np.uint64).copy()
    return dict(st=st6, ring=ring, cid=cid, self=self_, fail=fail, step=step, rend=rend, rcommit=rcommit,
                vote_ack=vote_ack, apply=apply, nc_len=n, dets=dets)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(1, 17))
def test_c_program_equals_reference(orc, tmp_path, seed):
    import ctypes as C
    if not os.path.exists(EXE):
        pytest.fail("examples/dare_poll not built: run __graft_entry__.build()")
    ref = orc.ref()
    if ref is None:
        pytest.skip("oracle/_ref not built (no /root/reference where the tree was built)")
    dump = tmp_path / "in.bin"
    r = subprocess.run([EXE, str(seed), str(dump)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout.strip().splitlines()[-1])
    d = _parse(dump)
    P = lambda a: C.c_void_p(a.ctypes.data)   # noqa: E731
    st, ring, cid, self_ = d["st"], d["ring"], d["cid"], d["self"]
    committed = C.c_int(0)
    new_commit = ref.ref_commit_walk(P(ring), P(st), P(cid), self_, C.byref(committed))
    assert got["new_commit"] == new_commit and got["committed"] == committed.value
    assert got["median"] == ref.ref_median(P(st), P(cid), self_, P(d["rend"]), P(d["step"]), P(d["fail"]))
    rc, mask, ssn = d["rcommit"].copy(), np.zeros(1, np.uint16), np.zeros(1, np.uint64)
    ref.ref_publish(P(st), P(cid), self_, R, new_commit, P(d["rend"]), P(rc), P(d["step"]), P(d["fail"]), 0xFFFF,
                    P(mask), P(ssn))
    assert got["publish"] == int(mask[0]) and got["ssn"] == int(ssn[0]) and got["remote_commit"] == rc.tolist()
    nh, app = C.c_uint64(0), C.c_int(0)
    ref.ref_min_apply(P(ring), P(st), P(cid), P(d["apply"].copy()), 0, C.byref(nh), C.byref(app))
    assert got["new_head"] == nh.value and got["append_head"] == app.value
    vc, vn = np.zeros(2, np.uint8), C.c_uint64(0)
    won = ref.ref_vote_tally(P(st), P(cid), self_, P(d["vote_ack"]), P(vc), C.byref(vn))
    assert got["won"] == won and got["vc"] == vc.tolist() and got["vote_commit"] == vn.value
    # voters: the servers poll_vote_count counted (i != self, i < size, an ack present)
    size = int(cid[8])
    voters = sum(1 << i for i in range(size) if i != self_ and int(d["vote_ack"][i]) != int(st[5]))
    assert got["voters"] == voters
    dets = np.zeros(3 * 1024, np.uint64)
    n = ref.ref_nc_build(P(ring), P(st), P(dets), 1024)
    assert got["nc_len"] == n and n == d["nc_len"]
    assert got["nc_last"] == [int(dets[3 * (n - 1)]), int(dets[3 * (n - 1) + 2])]
    assert got["remote_end"] == ref.ref_find_remote_end(P(ring), P(st), P(d["dets"]), d["nc_len"])


def test_c_program_builds_and_links():
    """the C program is built against the in-tree library (no GPU needed to check the link)"""
    if not os.path.exists(EXE):
        pytest.skip("examples/dare_poll not built")
    r = subprocess.run(["ldd", EXE], capture_output=True, text=True)
    assert "libapus_gpu.so" in r.stdout and "not found" not in r.stdout.split("libapus_gpu.so")[1].splitlines()[0]
