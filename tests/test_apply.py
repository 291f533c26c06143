"""Apply / config scan: apply_committed_entries
(src/dare/dare_server.c:1815-1974) and poll_config_entries (:2133-2187, with
update_cid :2193-2226).

CPU: the clean-room oracle against the reference-composed restatement on
the reference's own log primitives and equal_cid / CID macros (oracle/_ref).
GPU: apus_apply_batch / apus_config_scan_batch against the oracle, bit-exact
on every output, then the leader's CONFIG re-appends fed to
apus_append_batch (the reconfiguration step of BASELINE config 5).

The traces are the generator's logs (wraps, ghost headers, every entry type)
with every CONFIG entry's dare_cid_t redrawn: epochs around the group's,
STABLE / TRANSIT / EXTENDED (and an undefined state 3), joint sizes, req_id 0
or not; groups are leaders or followers, and the scans start from head,
apply or commit.
"""
import numpy as np
import pytest

CASES = {
    "mixed": dict(G=384, R=7, gen=dict(seed=301, n_entries=10, n_history=14, len_min=0, len_max=90, ring_len=4000,
                                       type_mix=True, cid_mix=True, self_random=True)),
    "wrap_small": dict(G=384, R=5, gen=dict(seed=302, n_entries=4, n_history=8, len_min=0, len_max=40,
                                            ring_len=2000, type_mix=True, cid_mix=True, self_random=True)),
    "c5": dict(G=256, R=7, gen=dict(seed=303, n_entries=16, n_history=16, len_min=64, len_max=64, ring_len=8192,
                                    type_mix=True, cid_mix=True)),
}


def _chain(hb, g, start):
    """entry offsets from `start` to end (log_get_entry / log_fit_entry walk)"""
    st = hb.state[g]
    ring = hb.group_ring(g)
    end, ln = int(st["end"]), int(st["len"])
    o, out = int(start), []
    for _ in range(ln // 64 + 4):
        if end == ln or (end - o if end >= o else ln - (o - end)) == 0:
            break
        if ln - o < 64:
            o = 0
        t = ring[o + 26]
        el = 64 if t in (0, 2, 3) else 64 + int(ring[o + 48]) + (int(ring[o + 49]) << 8)
        out.append(o)
        if ln - o < el:
            o = 0
        o += el
    return out


def build(pkg, orc, name, case=None):
    c = CASES[name] if case is None else case
    G, R = c["G"], c["R"]
    hb = orc.host_batch(G, R, c["gen"]["ring_len"])
    orc.gen(hb, pkg.batch.gen_cfg(**c["gen"]))
    rng = np.random.default_rng(c["gen"]["seed"])
    st = hb.state
    # leaders (SID_GET_L, idx == self) and followers
    lead = rng.random(G) < 0.6
    term = rng.integers(1, 50, G).astype(np.uint64)
    idx = np.where(lead, hb.self_idx, (hb.self_idx.astype(np.int64) + 1) % R).astype(np.uint64)
    hb.sid[:] = (term << np.uint64(9)) | (lead.astype(np.uint64) << np.uint64(8)) | idx
    # the scans start at head (everything), or the apply the generator set
    from_head = rng.random(G) < 0.5
    st["apply"] = np.where(from_head, st["head"], st["apply"])
    cid_dt = st.dtype["cid"]
    for g in range(G):
        ring = hb.group_ring(g)
        for o in _chain(hb, g, st["head"][g]):
            if ring[o + 26] != 2:
                continue
            c16 = np.zeros(1, cid_dt)
            c16["epoch"] = max(0, int(st["cid"]["epoch"][g]) + int(rng.integers(-1, 2)))
            c16["state"] = rng.choice([0, 1, 2, 3], p=[0.3, 0.3, 0.35, 0.05])
            s0 = int(rng.integers(3, 8))
            c16["size0"] = s0
            c16["size1"] = int(rng.integers(0, 8)) if c16["state"][0] != 0 else 0
            c16["bitmask"] = int(rng.integers(0, 1 << 8))
            ring[o + 48:o + 64] = c16.view(np.uint8)
            if rng.random() < 0.3:
                ring[o + 16:o + 24] = 0                                    # req_id 0
    G_ = np.arange(G)
    starts = rng.integers(0, 3, G)
    cid_offset = np.where(starts == 0, st["head"], np.where(starts == 1, st["apply"], st["commit"]))
    base_idx = np.array([int.from_bytes(hb.group_ring(g)[int(st["commit"][g]) % max(int(st["len"][g]) - 64, 1):][:8]
                                        .tobytes(), "little") for g in G_], np.uint64)
    cid_idx = np.where(rng.random(G) < 0.5, 0, base_idx - rng.integers(0, 12, G).astype(np.uint64))
    return hb, cid_offset.astype(np.uint64), cid_idx.astype(np.uint64)


def _clone(pkg, hb):
    c = pkg.batch.HostBatch(hb.G, hb.R, hb.stride, fields=list(hb.arrays))
    c.ring[:] = hb.ring
    for k, v in hb.arrays.items():
        c.arrays[k][:] = v
    return c


def _same(a, b, keys):
    for k in keys:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_config_scan_matches_reference(pkg, orc, ref, name):
    hb, off, cidx = build(pkg, orc, name)
    h2 = _clone(pkg, hb)
    io = orc.config_io(hb.G, off, cidx)
    io2 = orc.config_io(hb.G, off, cidx)
    assert orc.config_scan(hb, io) == orc.ref_config_scan(h2, io2) == 0
    _same(io, io2, ("cid_offset", "req_id", "clt_id", "departed"))
    assert np.array_equal(hb.state, h2.state)
    assert io["departed"].any() and (io["req_id"] != 0).any(), "trace exercises no cid update"


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("max_cfg", [1, 4])
def test_oracle_apply_matches_reference(pkg, orc, ref, name, max_cfg):
    hb, _, _ = build(pkg, orc, name)
    h2 = _clone(pkg, hb)
    io = orc.apply_io(hb.G, max_cfg)
    io2 = orc.apply_io(hb.G, max_cfg)
    assert orc.apply(hb, io) == orc.ref_apply(h2, io2) == 0
    _same(io, io2, ("req_id", "clt_id", "last_applied", "last_csm_idx", "n_applied", "departed", "events",
                    "n_cfg", "cfg_payload"))
    assert np.array_equal(io["cfg_entries"], io2["cfg_entries"])
    assert np.array_equal(hb.state, h2.state)
    assert io["n_cfg"].any() and io["n_applied"].any()


@pytest.mark.parametrize("name", list(CASES))
def test_reference_batch_forms_equal_per_group(pkg, orc, ref, name):
    """oracle/_ref's ref_config_scan_batch / ref_apply_batch (the whole-batch
    checkers of tests/test_whole_batch.py: the light log image, the records
    written in C) leave every state row and output as the per-group calls do"""
    hb, off, cidx = build(pkg, orc, name)
    h2 = _clone(pkg, hb)
    io, io2 = orc.config_io(hb.G, off, cidx), orc.config_io(hb.G, off, cidx)
    assert orc.ref_config_scan(hb, io) == orc.ref_config_scan_batch(h2.G, h2.stride, h2.ring, h2.state.view(np.uint8),
                                                                     io2) == 0
    _same(io, io2, ("cid_offset", "req_id", "clt_id", "departed"))
    assert np.array_equal(hb.state, h2.state)
    hb, _, _ = build(pkg, orc, name)
    h2 = _clone(pkg, hb)
    io, io2 = orc.apply_io(hb.G, 2), orc.apply_io(hb.G, 2)
    assert orc.ref_apply(hb, io) == orc.ref_apply_batch(h2.G, h2.stride, h2.ring, h2.state.view(np.uint8),
                                                        h2.self_idx, h2.sid, io2) == 0
    _same(io, io2, ("req_id", "clt_id", "last_applied", "last_csm_idx", "n_applied", "departed", "events", "n_cfg",
                    "cfg_payload"))
    assert io["cfg_entries"].tobytes() == io2["cfg_entries"].tobytes()
    assert np.array_equal(hb.state, h2.state)


def test_oracle_apply_resumes_after_cfg_full(pkg, orc):
    """max_cfg = 1 run repeatedly (appending nothing) ends where one unbounded run ends"""
    hb, _, _ = build(pkg, orc, "mixed")
    h2 = _clone(pkg, hb)
    big = orc.apply_io(hb.G, 64)
    orc.apply(hb, big)
    io = orc.apply_io(h2.G, 1)
    n_cfg = np.zeros(h2.G, np.uint32)
    for _ in range(64):
        orc.apply(h2, io)
        n_cfg += io["n_cfg"]
        if not (io["events"] & 8).any():
            break
    assert np.array_equal(h2.state["apply"], hb.state["apply"])
    assert np.array_equal(h2.state["cid"], hb.state["cid"])
    assert np.array_equal(n_cfg, big["n_cfg"])


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
def test_gpu_config_scan_matches_oracle(pkg, orc, eng, name):
    hb, off, cidx = build(pkg, orc, name)
    db = _dev(pkg, hb)
    io = orc.config_io(hb.G, off, cidx)
    out = eng.poll_config_entries(db, io)
    orc.config_scan(hb, io)
    for k in ("cid_offset", "req_id", "clt_id", "departed"):
        assert np.array_equal(out[k], io[k]), k
    assert np.array_equal(db.download("state"), hb.state)


@pytest.mark.gpu
def test_gpu_config_scan_guard_and_malformed(pkg, orc, eng):
    """the step guard stops both kernels at the oracle's entry: on rings
    whose end was moved off the entry chain the scan laps the ring until the
    guard, and the groups count as corrupt with the oracle's partial updates
    (the configurations adopted and servers departed on the way).  (A scan
    started past len, which the reference would read out of bounds, is
    refused by the device and not compared.)"""
    hb, off, cidx = build(pkg, orc, "mixed")
    rng = np.random.default_rng(7)
    st = hb.state
    G = hb.G
    sel = rng.random(G) < 0.3
    # end inside an entry: the walk never meets it and runs to the guard
    st["end"] = np.where(sel, (st["end"].astype(np.int64) + 8) % st["len"].astype(np.int64), st["end"]).astype(np.uint64)
    db = _dev(pkg, hb)
    io = orc.config_io(hb.G, off, cidx)
    eng.stats_reset()
    out = eng.poll_config_entries(db, io)
    bad = orc.config_scan(hb, io)
    for k in ("cid_offset", "req_id", "clt_id", "departed"):
        assert np.array_equal(out[k], io[k]), k
    assert np.array_equal(db.download("state"), hb.state)
    assert bad > 0 and eng.stats()[pkg.abi.STAT_CORRUPT] == bad


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("max_cfg", [1, 4])
def test_gpu_apply_then_append_matches_oracle(pkg, orc, eng, name, max_cfg):
    hb, _, _ = build(pkg, orc, name)
    db = _dev(pkg, hb)
    io = orc.apply_io(hb.G, max_cfg)
    out = eng.apply_committed_entries(db, io)
    orc.apply(hb, io)
    for k in ("req_id", "clt_id", "last_applied", "last_csm_idx", "n_applied", "departed", "events", "n_cfg",
              "cfg_payload"):
        assert np.array_equal(out[k], io[k]), k
    assert np.array_equal(out["cfg_entries"], io["cfg_entries"])
    assert np.array_equal(db.download("state"), hb.state)
    # the reference's log_append_entry(..., CONFIG, &cid) for each request, in order
    import torch
    eng.log_append_entry(db, torch.from_numpy(io["cfg_entries"].view(np.uint8).copy()).cuda(),
                         torch.from_numpy(io["cfg_payload"]).cuda(), max_cfg,
                         n_entries=torch.from_numpy(io["n_cfg"]).cuda())
    orc.append(hb, io["cfg_entries"], io["cfg_payload"], max_cfg, n_entries=io["n_cfg"])
    assert np.array_equal(db.download("ring"), hb.ring)
    assert np.array_equal(db.download("state"), hb.state)
