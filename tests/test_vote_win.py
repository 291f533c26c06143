"""The election-win transition (BASELINE config 5's reconfiguration):
poll_vote_count after the tally, src/dare/dare_server.c:1355-1362 and
1389-1510 -- the tally's side effects, the SID's L bit, poll_config_entries,
the leader's apply_committed_entries with its CONFIG re-appends, the blank
entry (CONFIG / NOOP / EXTENDED -> TRANSIT / -> STABLE with the server
removals) and become_leader's apply_offsets = head.

CPU: the clean-room oracle (the tally of apus_oracle_vote_batch, then
apus_oracle_vote_win) against oracle/_ref's poll_vote_count, transcribed whole
on the reference's own log primitives, log_append_entry and config macros
(region vote_count of tests/test_transcription.py), bit-exact on every ring
byte and every output.
GPU: apus_vote_batch then apus_vote_win_batch against the oracle, bit-exact.

The traces are test_apply's (wraps, ghost headers, every entry type, CONFIG
entries with redrawn cids: epochs around the group's, STABLE / TRANSIT /
EXTENDED, joint sizes, req_id 0 or not), with SIDs making most groups
candidates (and some leaders, followers and IS_NONE servers), some logs full
(head == end: the blank entry returns 0), some tails unknown (tail == len:
log_get_tail), and the configuration scans starting from head, apply or
commit.
"""
import numpy as np
import pytest

from test_apply import CASES as APPLY_CASES
from test_apply import build as apply_build

CASES = dict(APPLY_CASES)
CASES["tight"] = dict(G=384, R=5, gen=dict(seed=304, n_entries=6, n_history=10, len_min=0, len_max=30,
                                           ring_len=1700, type_mix=True, cid_mix=True, self_random=True))

OUT_KEYS = ("cid_offset", "req_id", "clt_id", "last_applied", "last_csm_idx", "last_write_csm_idx", "outcome",
            "events", "departed", "n_applied", "n_cfg")
HB_KEYS = ("ring", "state", "sid", "remote_commit", "lr_step", "apply_offsets", "prev_head")


def build(pkg, orc, name):
    """a host batch and the win io (the tally already run by the oracle)"""
    c = CASES[name]
    hb, cid_offset, cid_idx = apply_build(pkg, orc, name, c)
    G, R = hb.G, hb.R
    rng = np.random.default_rng(c["gen"]["seed"] + 1000)
    st = hb.state
    term = rng.integers(1, 60, G).astype(np.uint64)
    kind = rng.choice(4, G, p=[0.72, 0.1, 0.1, 0.08])       # candidate, leader, follower, IS_NONE
    idx = np.where(kind == 2, (hb.self_idx.astype(np.int64) + 1) % R, hb.self_idx).astype(np.uint64)
    term = np.where(kind == 3, 0, term).astype(np.uint64)
    hb.sid[:] = (term << np.uint64(9)) | ((kind == 1).astype(np.uint64) << np.uint64(8)) | idx
    # the last entry's data.cid.state byte (@58) set to CID_EXTENDED on some
    # logs: the blank entry's EXTENDED -> TRANSIT branch reads it (:1456)
    for g in np.nonzero(rng.random(G) < 0.2)[0]:
        t = int(st["tail"][g])
        if t + 64 <= int(st["len"][g]):
            hb.group_ring(g)[t + 58] = 2
    # some logs full (is_log_full: the blank entry returns 0), some tails unknown
    full = rng.random(G) < 0.04
    st["head"] = np.where(full, st["end"], st["head"])
    st["tail"] = np.where(rng.random(G) < 0.1, st["len"], st["tail"])
    hb.prev_head[:] = rng.random(G) < 0.3
    # some vote acks at end: the tally's commit reaches end (cid_offset there)
    sel = rng.random(G * R) < 0.08
    ends = np.repeat(st["end"], R)
    hb.vote_ack[:] = np.where(sel & (hb.vote_ack != np.repeat(st["len"], R)), ends, hb.vote_ack)
    v = orc.vote(hb)
    last = rng.integers(0, 1 << 40, 3 * G).astype(np.uint64)
    io = orc.win_io(G, v["won"], v["voters"], v["new_commit"], cid_offset, cid_idx,
                    req_id=rng.integers(0, 1 << 20, G), clt_id=rng.integers(0, 1 << 16, G),
                    last_applied=last, last_csm_idx=last[:G], last_write_csm_idx=last[G:2 * G])
    return hb, io


def _clone(pkg, hb):
    c = pkg.batch.HostBatch(hb.G, hb.R, hb.stride, fields=list(hb.arrays))
    c.ring[:] = hb.ring
    for k, v in hb.arrays.items():
        c.arrays[k][:] = v
    return c


def _cmp_io(a, b):
    for k in OUT_KEYS:
        assert np.array_equal(a[k], b[k]), k


def _cmp_hb(a, b):
    assert np.array_equal(a.ring, b.ring), "ring"
    for k in HB_KEYS[1:]:
        assert np.array_equal(a.arrays[k], b.arrays[k]), k


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_vote_win_matches_reference(pkg, orc, ref, name):
    hb, io = build(pkg, orc, name)
    h2 = _clone(pkg, hb)
    io2 = {k: v.copy() for k, v in io.items()}
    bad = orc.vote_win(hb, io)
    assert orc.ref_vote_count(h2, io2) == bad
    _cmp_io(io, io2)
    _cmp_hb(hb, h2)
    abi = pkg.abi
    seen = set(np.unique(io["outcome"]).tolist())
    assert {abi.WIN_NOT_CANDIDATE, abi.WIN_LOST, abi.WIN_CONFIG} <= seen, np.bincount(io["outcome"])


@pytest.mark.parametrize("name", list(CASES))
def test_reference_vote_count_batch_equals_per_group(pkg, orc, ref, name):
    """oracle/_ref's ref_vote_count_batch (one log image cleared once, the
    non-candidates skipped: tests/test_whole_batch.py's checker) leaves every
    byte and output as ref_vote_count called group by group does"""
    hb, io = build(pkg, orc, name)
    h2 = _clone(pkg, hb)
    io2 = {k: v.copy() for k, v in io.items()}
    bad = orc.ref_vote_count(hb, io)
    arr = {k: h2.arrays[k] for k in HB_KEYS[1:] + ("self_idx", "vote_ack")}
    arr["ring"] = h2.ring
    arr["state"] = h2.state.view(np.uint8)
    assert orc.ref_vote_count_batch(h2.G, h2.R, h2.stride, arr, io2) == bad
    _cmp_io(io, io2)
    _cmp_hb(hb, h2)


def test_oracle_vote_win_covers_every_outcome(pkg, orc, ref):
    """across the traces: every outcome of the blank-entry decision, the
    removals and a self-removal, CONFIG re-appends in the apply, full logs"""
    abi = pkg.abi
    seen, ev, dep, ncfg, zero = set(), 0, 0, 0, 0
    for name in CASES:
        hb, io = build(pkg, orc, name)
        orc.vote_win(hb, io)
        won = io["outcome"] >= abi.WIN_CONFIG
        seen |= set(np.unique(io["outcome"]).tolist())
        ev |= int(np.bitwise_or.reduce(io["events"]))
        dep |= int((io["departed"][won] != 0).sum())
        ncfg += int(io["n_cfg"].sum())
        zero += int(((io["last_write_csm_idx"] == 0) & (io["outcome"] >= abi.WIN_CONFIG) &
                     (io["outcome"] <= abi.WIN_STABLE)).sum())
    assert {abi.WIN_NOT_CANDIDATE, abi.WIN_LOST, abi.WIN_CONFIG, abi.WIN_NOOP, abi.WIN_TRANSIT,
            abi.WIN_STABLE, abi.WIN_UNDEFINED} <= seen, seen
    assert ev & abi.EV_SELF_REMOVED and dep > 0 and ncfg > 0 and zero > 0, (ev, dep, ncfg, zero)


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _dev(pkg, hb):
    db = pkg.batch.DeviceBatch(hb.G, hb.R, hb.stride)
    db.upload(hb)
    return db


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_gpu_vote_win_matches_oracle(pkg, orc, eng, name):
    """apus_vote_batch on the device, its outputs fed to apus_vote_win_batch:
    every output and every byte of the batch as the oracle leaves them"""
    hb, io = build(pkg, orc, name)
    db = _dev(pkg, hb)
    vo = eng.poll_vote_count(db)
    for k in ("won", "new_commit"):
        assert np.array_equal(vo[k].cpu().numpy().view(io[k].dtype), io[k]), k
    assert np.array_equal(vo["voters"].cpu().numpy().view(np.uint16), io["voters"])
    dio = dict(io)
    for k in ("won", "voters", "new_commit"):
        dio[k] = vo[k]
    eng.stats_reset()
    got = eng.become_leader(db, dio)
    bad = orc.vote_win(hb, io)
    _cmp_io(got, io)
    for k in HB_KEYS:
        assert np.array_equal(db.download(k), hb.ring if k == "ring" else hb.arrays[k]), k
    assert eng.stats()[pkg.abi.STAT_CORRUPT] == bad


@pytest.mark.gpu
def test_gpu_vote_win_guard(pkg, orc, eng):
    """rings whose end was moved off the entry chain: the scans lap the ring to
    the step guard and the groups stop where the oracle stops them"""
    hb, io = build(pkg, orc, "mixed")
    rng = np.random.default_rng(9)
    st = hb.state
    sel = rng.random(hb.G) < 0.25
    st["end"] = np.where(sel, (st["end"].astype(np.int64) + 8) % st["len"].astype(np.int64),
                         st["end"]).astype(np.uint64)
    db = _dev(pkg, hb)
    eng.stats_reset()
    got = eng.become_leader(db, io)
    bad = orc.vote_win(hb, io)
    _cmp_io(got, io)
    for k in HB_KEYS:
        assert np.array_equal(db.download(k), hb.ring if k == "ring" else hb.arrays[k]), k
    assert bad > 0 and eng.stats()[pkg.abi.STAT_CORRUPT] == bad


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["mixed", "wrap_small"])
def test_gpu_vote_win_on_log_images(pkg, orc, eng, name):
    """the same transition on dare_log_t images (APUS_BATCH_LOG_IMAGE): the
    offsets move in each image's header, the blank entries land in its
    entries[], config.cid in the cid array"""
    hb, io = build(pkg, orc, name)
    L = int(hb.state["len"][0])
    assert (hb.state["len"] == L).all()
    img = pkg.batch.LogImageBatch(hb.G, hb.R, L)
    img.fill_from(hb)
    got = eng.become_leader(img, io)
    orc.vote_win(hb, io)
    _cmp_io(got, io)
    assert np.array_equal(img.download("ring"), hb.ring.reshape(hb.G, hb.stride)[:, :L]), "entries[]"
    st = img.download("state")
    for k in ("head", "apply", "commit", "end", "tail", "len"):
        assert np.array_equal(st[k], hb.state[k]), k
    assert st["cid"].tobytes() == hb.state["cid"].tobytes(), "cid"
    for k in HB_KEYS[2:]:
        assert np.array_equal(img.download(k), hb.arrays[k]), k
