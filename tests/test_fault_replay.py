"""CPU replay of the address arithmetic of log_adjust_kernel and
lr_completion_kernel (VERDICT r1 "next" #1).

One full `pytest -m gpu` run in round 1 stopped with an illegal-address fault
inside test_gpu_adjust_completion_pipeline[r5_mix], on the first
wave-cooperative log_adjust_kernel (commit 243d5ac).  This module replays,
lane by lane and wave by wave, every global-memory access both versions of
the kernel make (243d5ac and the current apus_quorum.hip), plus the dword
and byte paths of lr_completion_kernel, over the exact seeded inputs of the
GPU tests that launch them:

  test_gpu_log_adjust_matches_oracle / _matches_golden_digests  (round 0)
  test_gpu_adjust_completion_pipeline, all 6 adjust -> completion rounds
  test_gpu_scalar_dropins (G = 1, 13 server slots, 1024-entry NC rows)

and checks each access against the extent of the buffer it addresses:
  state[g] (64 B), self_idx, rc_connected, fail_count / send_flag / lr_step /
  vote_ack / remote_commit / remote_end / post [g*R + i], nc_len[k_gi],
  nc_dets[k_gi*max_dets + k] (24 B), ssn[g], and ring bytes, which must stay
  inside the walking group's own [g*stride, g*stride + len) -- the 16-B
  ld_idx_term / 5-dword funnel, type@26 and cmd.len@48..49.

The kernels' lane logic (ballots, readlane / shfl selection of the pending
(group, server) walks, segment bookkeeping, the first-mismatch rule) is
restated from the HIP source; the walked results are checked against the
oracle so the model provably follows the same control flow as the device.
The state the device sees in round r is the oracle's state after round r-1,
which the GPU tests assert bit-exact.  Result: no access of
either kernel version leaves its buffer on any of these inputs.
"""
import numpy as np
import pytest

from test_lr_step import CASES, _all_pairs, _clone_io, build

M64 = (1 << 64) - 1
HDR = 64
LR_GET_WRITE, LR_GET_NCE_LEN, LR_GET_NCE, LR_SET_END, LR_UPDATE_LOG = 1, 2, 3, 4, 5
STABLE = 0


class Mem:
    """extents of the device buffers one launch addresses"""

    def __init__(self, sizes):
        self.sizes = dict(sizes)
        self.n = 0

    def acc(self, buf, lo, nbytes):
        self.n += 1
        assert 0 <= lo and lo + nbytes <= self.sizes[buf], f"{buf}[{lo}:{lo + nbytes}) past {self.sizes[buf]}"


def dist(end, ln, o):
    if end == ln:
        return 0
    return (end - o) & M64 if end >= o else (ln - ((o - end) & M64)) & M64


def get_entry(end, ln, o, version):
    """RingView::get_entry; returns (ok, o).  243d5ac tested o + 64 <= len in
    u64 arithmetic (wraps near 2^64), the current code o <= len - 64"""
    if end == ln or dist(end, ln, o) == 0:
        return False, o
    if ((ln - o) & M64) < HDR:
        o = 0
    if version == "243d5ac":
        return ((o + HDR) & M64) <= ln, o
    return ln >= HDR and o <= ln - HDR, o


def ext_group_size(st):
    s0, s1 = int(st["cid"]["size0"]), int(st["cid"]["size1"])
    return s0 if int(st["cid"]["state"]) == STABLE else max(s0, s1)


def ring_hdr_reads(mem, ring, g, stride, ln, off):
    """the ring bytes one walk step reads at entry offset off (ld_idx_term,
    then e[26] and ld_u16(e + 48) when idx/term match)"""
    base = g * stride
    a = off
    if a % 8 == 0:
        lo, n = a, 16
    else:
        lo, n = a & ~3, 20                 # 5-dword funnel from the aligned word
    mem.acc("ring", base + lo, n)
    assert lo >= 0 and lo + n <= ln, f"group {g}: ring read [{lo},{lo + n}) outside [0,{ln})"
    e = ring[base + off: base + off + HDR]
    return int(e[0:8].view(np.uint64)[0]), int(e[8:16].view(np.uint64)[0]), e


def entry_len_at(mem, ring, g, stride, ln, off, e):
    base = g * stride
    mem.acc("ring", base + off + 26, 1)
    mem.acc("ring", base + off + 48, 2)
    assert off + 50 <= ln
    t = int(e[26])
    clen = int(e[48]) | (int(e[49]) << 8)
    return HDR if t in (0, 2, 3) else HDR + clen


def phase1(hb, io, mem, g, R, M):
    """the per-lane part of log_adjust_kernel (identical in both versions);
    returns the pending-walk mask"""
    st = hb.state[g]
    mem.acc("state", 64 * g, 64)
    mem.acc("self_idx", g, 1)
    self_ = int(hb.self_idx[g])
    size = ext_group_size(st)
    if io["rc_connected"] is not None:
        mem.acc("rc_connected", 2 * g, 2)
        conn = int(io["rc_connected"][g])
    else:
        conn = 0xFFFF
    ln, bitmask = int(st["len"]), int(st["cid"]["bitmask"])
    gR = g * R
    for i in range(R):
        for b, w in (("fail_count", 1), ("send_flag", 1), ("lr_step", 1), ("vote_ack", 8)):
            mem.acc(b, (gR + i) * w, w)
    walk, init = 0, False
    for i in range(R):
        k = gR + i
        p = 0
        if (i < size and i != self_ and (bitmask >> i) & 1 and int(hb.fail_count[k]) < 2 and io["send_flag"][k]
                and (conn >> i) & 1):
            rc = int(hb.vote_ack[k])
            if rc != ln:
                s = int(hb.lr_step[k])
                if not init and s < LR_UPDATE_LOG:
                    init = True
                    mem.acc("ssn", 8 * g, 8)
                if s == LR_GET_WRITE:
                    mem.acc("remote_commit", 8 * k, 8)
                    s = LR_GET_NCE_LEN
                if s == LR_GET_NCE_LEN:
                    p = 1
                elif s == LR_GET_NCE:
                    mem.acc("nc_len", 8 * k, 8)
                    if int(io["nc_len"][k]) == 0:
                        mem.acc("remote_commit", 8 * k, 8)
                        mem.acc("remote_end", 8 * k, 8)
                    else:
                        p = 2
                elif s == LR_SET_END:
                    mem.acc("nc_len", 8 * k, 8)
                    if int(io["nc_len"][k]) and M and ln <= hb.stride:
                        walk |= 1 << i
                    else:
                        mem.acc("remote_commit", 8 * k, 8)
                        mem.acc("remote_end", 8 * k, 8)
                    p = 3
                mem.acc("lr_step", k, 1)
                if p:
                    mem.acc("send_flag", k, 1)
        mem.acc("post", gR + i, 1)
    mem.acc("state", 64 * g + 16, 8)
    return walk


def step_at(hb, io, mem, gL, R, M, myI, k, det, version):
    """one lane's check of determinant k of walk (gL, myI): (bad, ro, nx)"""
    st = hb.state[gL]
    end, ln = int(st["end"]), int(st["len"])
    off = int(det["offset"])
    ok, off = get_entry(end, ln, off, version)
    if not ok:
        return True, off, 0
    l_idx, l_term, e = ring_hdr_reads(mem, hb.ring, gL, hb.stride, ln, off)
    if l_idx != int(det["idx"]) or l_term != int(det["term"]):
        return True, off, 0
    el = entry_len_at(mem, hb.ring, gL, hb.stride, ln, off, e)
    return False, 0, ((0 if ln - off < el else off) + el) & M64


def det_read(io, mem, k_gi, M, k):
    idx = k_gi * M + k
    mem.acc("nc_dets", 24 * idx, 24)
    return io["nc_dets"][idx]


def walks_current(hb, io, mem, base, walk, R, M, res):
    """apus_quorum.hip log_adjust_kernel cooperative pass (S = 16 when
    max_dets <= 16, else 64)"""
    G = hb.G
    S = 16 if M <= 16 else 64
    W = 64 // S
    while any(walk):
        bal = [L for L in range(64) if walk[L]]
        wmine = [((w & -w).bit_length() - 1) if w else 0 for w in walk]
        myL, myI = [64] * 64, [0] * 64
        m = list(bal)
        for j in range(W):
            if m:
                Lj = m.pop(0)
                ij = wmine[Lj]
                for lane in range(j * S, (j + 1) * S):
                    myL[lane], myI[lane] = Lj, ij
                walk[Lj] &= walk[Lj] - 1
        for j in range(W):
            lanes = range(j * S, (j + 1) * S)
            L = myL[j * S]
            if not (L < 64 and base + L < G):
                continue
            gL, iL = base + L, myI[j * S]
            k_gi = gL * R + iL
            det0 = [det_read(io, mem, k_gi, M, sl) if sl < M else None for sl in range(S)]
            mem.acc("nc_len", 8 * k_gi, 8)
            n = min(int(io["nc_len"][k_gi]), M)
            out = None
            k0 = 0
            while k0 < n:
                bad_any = None
                last = 0
                for sl in range(S):
                    k = k0 + sl
                    if k >= n:
                        continue
                    det = det0[sl] if k0 == 0 else det_read(io, mem, k_gi, M, k)
                    bad, ro, nx = step_at(hb, io, mem, gL, R, M, iL, k, det, "current")
                    if bad and bad_any is None:
                        bad_any = ro
                    if k == n - 1:
                        last = nx
                if bad_any is not None:
                    out = bad_any
                    break
                if k0 + S >= n:
                    out = last
                k0 += S
            mem.acc("remote_end", 8 * k_gi, 8)
            res[k_gi] = out
            assert all(myL[x] == L for x in lanes)


def walks_243d5ac(hb, io, mem, base, walk, R, M, res):
    """243d5ac: one pending walk per wave step, 64 determinants per chunk"""
    while any(walk):
        L = next(x for x in range(64) if walk[x])
        iL = (walk[L] & -walk[L]).bit_length() - 1
        gL = base + L
        k_gi = gL * R + iL
        mem.acc("nc_len", 8 * k_gi, 8)
        n = min(int(io["nc_len"][k_gi]), M)
        out, k0 = 0, 0
        while k0 < n:
            bad_any, last = None, 0
            for lane in range(64):
                k = k0 + lane
                if k >= n:
                    continue
                bad, ro, nx = step_at(hb, io, mem, gL, R, M, iL, k, det_read(io, mem, k_gi, M, k), "243d5ac")
                if bad and bad_any is None:
                    bad_any = ro
                if k == n - 1:
                    last = nx
            if bad_any is not None:
                out = bad_any
                break
            if k0 + 64 >= n:
                out = last
            k0 += 64
        mem.acc("remote_end", 8 * k_gi, 8)
        res[k_gi] = out
        walk[L] &= walk[L] - 1


def sizes_of(hb, io):
    G, R, M = hb.G, hb.R, io["max_dets"]
    s = {"state": 64 * G, "self_idx": G, "ring": G * hb.stride, "ssn": 8 * G,
         "nc_len": 8 * G * R, "nc_dets": io["nc_dets"].nbytes, "post": G * R}
    for b in ("fail_count", "send_flag", "lr_step"):
        s[b] = G * R
    for b in ("vote_ack", "remote_commit", "remote_end"):
        s[b] = 8 * G * R
    if io["rc_connected"] is not None:
        s["rc_connected"] = 2 * G
    assert io["nc_dets"].size >= G * R * max(M, 1)
    return s


def replay_log_adjust(hb, io, version):
    """every access of one log_adjust_kernel launch; returns (remote ends the
    walks wrote, number of accesses checked)"""
    G, R, M = hb.G, hb.R, io["max_dets"]
    mem = Mem(sizes_of(hb, io))
    res = {}
    for base in range(0, G, 64):                    # every wave of the grid-stride loop
        walk = [phase1(hb, io, mem, base + ln, R, M) if base + ln < G else 0 for ln in range(64)]
        (walks_current if version == "current" else walks_243d5ac)(hb, io, mem, base, walk, R, M, res)
    return res, mem.n


def replay_lr_completion(pairs, aligned=True, grid=None):
    """lr_completion_kernel<VEC>: every byte index each column access covers"""
    if grid is None:
        grid = min(-(-((pairs + 3) // 4 if aligned else pairs) // 256), 256 * 8)
    stride = grid * 256
    mx = -1
    n = 0
    for t in range(stride):
        tt = t
        if aligned:
            words = pairs >> 2
            for w in range(t, words, stride):
                mx = max(mx, 4 * w + 3)
                n += 1
            tt = t + (words << 2)
            if tt >= pairs:
                continue
        for k in range(tt, pairs, stride):
            mx = max(mx, k)
            n += 1
    assert mx < pairs, f"lr_completion touches byte {mx} of {pairs}"
    return n


def _check_walk_results(hb, io, res, orc):
    """the model's walk results equal the oracle's remote ends (same control flow)"""
    h2, io2 = _clone(hb), _clone_io(io)
    orc.log_adjust(h2, io2)
    for k, v in res.items():
        assert int(h2.remote_end[k]) == v & M64, f"walk model != oracle at pair {k}"


def _clone(hb):
    import apus_pkg
    pkg = apus_pkg.load_package()
    c = pkg.batch.HostBatch(hb.G, hb.R, hb.stride, fields=list(hb.arrays))
    c.ring[:] = hb.ring
    for k, v in hb.arrays.items():
        c.arrays[k][:] = v
    return c


@pytest.mark.parametrize("version", ["243d5ac", "current"])
@pytest.mark.parametrize("name", list(CASES))
def test_replay_adjust_completion_pipeline(pkg, orc, name, version):
    """all 6 rounds of test_gpu_adjust_completion_pipeline (and so round 0 =
    test_gpu_log_adjust_matches_oracle's launch)"""
    hb, io = build(pkg, orc, name)
    rng = np.random.default_rng(5)
    walks = 0
    for r in range(6):
        res, n = replay_log_adjust(hb, io, version)
        assert n > 0
        walks += len(res)
        _check_walk_results(hb, io, res, orc)
        orc.log_adjust(hb, io)
        io["wc"][:] = np.where(io["post"] != 0, np.where(rng.random(io["post"].size) < 0.85, 1, 2), 0).astype(
            np.uint8)
        replay_lr_completion(hb.G * hb.R)
        orc.lr_completion(hb, io)
    assert walks > 0, "trace never reaches an LR_SET_END walk"


@pytest.mark.parametrize("R", [4, 3])
def test_replay_lr_completion_paths(R):
    """test_gpu_lr_completion_exhaustive / _unaligned_columns shapes:
    G*R = 8192 (R = 4) and 8193 (R = 3, a ragged tail); dword and byte paths"""
    pairs = -(-(4 * 256 * 2 * 4) // R) * R
    replay_lr_completion(pairs, aligned=True)
    replay_lr_completion(pairs, aligned=False)
    for p in (1, 2, 3, 5, 4097):
        replay_lr_completion(p, aligned=True)


def test_replay_all_pairs_shape(pkg, orc):
    hb, io = _all_pairs(pkg, orc, 3)
    assert hb.G * hb.R % 4 == 1
    replay_lr_completion(hb.G * hb.R)


@pytest.mark.parametrize("name", ["r5_mix", "r7_c5"])
def test_replay_scalar_dropin_shape(pkg, orc, name):
    """apus_log_adjustment: G = 1 batches over 13 server slots, ring_stride =
    len, max_dets = 1024 (64-lane segments, the speculative det0 load of
    d[0..63] from each server's 1024-entry scratch row)"""
    hb, io = build(pkg, orc, name)
    M, R = io["max_dets"], hb.R
    io["nc_len"][:] = np.minimum(io["nc_len"], M)
    for g in range(48):
        ln = int(hb.state[g]["len"])
        one = pkg.batch.HostBatch(1, 13, ln, fields=list(hb.arrays))
        one.ring[:ln] = hb.group_ring(g)[:ln]
        one.state[:] = hb.state[g]
        one.self_idx[:] = hb.self_idx[g]
        for k in ("fail_count", "lr_step", "vote_ack", "remote_commit", "remote_end"):
            one.arrays[k][:R] = hb.arrays[k][g * R:(g + 1) * R]
        one.vote_ack[R:] = ln
        dets = np.zeros(13 * 1024, pkg.batch.DET_DT)
        nc_len = np.zeros(13, np.uint64)
        sf = np.zeros(13, np.uint8)
        for i in range(R):
            n = int(io["nc_len"][g * R + i])
            nc_len[i] = n
            dets[i * 1024:i * 1024 + n] = io["nc_dets"][(g * R + i) * M:(g * R + i) * M + n]
            sf[i] = io["send_flag"][g * R + i]
        rc = None if io["rc_connected"] is None else io["rc_connected"][g:g + 1].copy()
        sio = {"send_flag": sf, "send_count": np.zeros(13, np.uint8), "wc": np.zeros(13, np.uint8),
               "rc_connected": rc, "nc_len": nc_len, "nc_dets": dets, "ssn": io["ssn"][g:g + 1].copy(),
               "post": np.zeros(13, np.uint8), "max_dets": 1024}
        res, _ = replay_log_adjust(one, sio, "current")
        _check_walk_results(one, sio, res, orc)
