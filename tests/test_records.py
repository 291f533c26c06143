"""The proxy's stable-storage records -- the BDB record format.

persist_new_entries (src/dare/dare_server.c:1792-1810) hands every persisted
entry to stablestorage_save_request (src/proxy/proxy.c:269-291), which stores
the bytes from entry->clt_id as one proxy message record; dump_records
(src/db/db-interface.c:98-129) concatenates them into the snapshot that
stablestorage_load_records (proxy.c:306-336) replays.

CPU: the message layout against the reference's own proxy.h (compiled here,
oracle/_ref/proxy_layout); known answers for the load walk; the oracle's
store against an independent Python model of the walk (the entry chain from
the cursor, the record of each CONNECT / SEND / CLOSE entry), and store ->
load round trips.  Parity pin (round 4): the oracle against the
reference-composed records of oracle/_ref -- persist_new_entries' walk on the
reference's own dare_log.h handing every entry to stablestorage_save_request
restated on its own proxy.h (oracle/ref_compose.c, oracle/ref_records.c),
and stablestorage_load_records likewise -- directly where /root/reference is
present, and everywhere through tests/golden/records.json, which
tests/golden/make_golden.py wrote from oracle/_ref.
GPU: apus_records_store_batch / apus_records_load_batch against the oracle,
bit-exact on every dump byte, cursor, length and replay-plan field, on state
rows and dare_log_t images, including stops (records past the log, a full
dump, unknown actions, truncated snapshots), and against records.json.
"""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
LAYOUT = os.path.join(HERE, "..", "oracle", "_ref", "proxy_layout")
GOLDEN = os.path.join(HERE, "golden", "records.json")
GOLDEN_CAPS = (4096, 1024, 300)        # snapshot capacities of the fixture (300 and 1024 stop groups: a full dump)
GOLDEN_PLAN = 48

TRACES = {
    # R = 3: reply[4..5] = 0, every SEND record is the 24 bytes entry[24, 48)
    "r3_mix": (3, 256, dict(seed=901, n_entries=24, n_history=8, len_min=0, len_max=90, ring_len=6000, type_mix=True,
                            self_random=True)),
    # R = 7: acks in reply[4..5] make data.cmd.len 1, 256, 257, ... (garbage 2s too)
    "r7_mix": (7, 256, dict(seed=902, n_entries=20, n_history=8, len_min=0, len_max=200, ring_len=8192,
                            type_mix=True, cid_mix=True, self_random=True, garbage_reply=0.2, p_full_ack=0.5)),
    # small wrapping rings: ghost headers, header wraps, records running past len
    "wrap": (6, 512, dict(seed=903, n_entries=10, n_history=3, len_min=0, len_max=100, ring_len=3000, type_mix=True,
                          self_random=True, p_full_ack=0.7)),
}


def _host(pkg, orc, name):
    R, G, kw = TRACES[name]
    hb = orc.host_batch(G, R, kw["ring_len"])
    orc.gen(hb, pkg.batch.gen_cfg(**kw))
    return hb


def _py_store(hb, g, cursor, cap):
    """independent model: the entry chain from the cursor (log_get_entry /
    log_fit_entry), each CONNECT / CLOSE entry's 4 bytes and each SEND
    entry's 24 + u16(entry + 32) bytes from entry + 24"""
    st = hb.state[g]
    ring = hb.group_ring(g)
    end, ln = int(st["end"]), int(st["len"])
    o, out, n = int(cursor), bytearray(), 0
    for _ in range(ln // 64 + 4):
        if end == ln or (end - o if end >= o else ln - (o - end)) == 0:
            return bytes(out), n, o, 0
        if ln - o < 64:
            o = 0
        t = int(ring[o + 26])
        el = 64 if t in (0, 2, 3) else 64 + int(ring[o + 48]) + (int(ring[o + 49]) << 8)
        if ln - o < el:
            o = 0
            continue
        nb = 4 if t in (4, 6) else 24 + int(ring[o + 32]) + (int(ring[o + 33]) << 8) if t == 5 else 0
        if nb:
            if 24 + nb > ln - o or len(out) + nb > cap:
                return bytes(out), n, o, 1
            out += ring[o + 24:o + 24 + nb].tobytes()
            n += 1
        o += el
    return bytes(out), n, o, 1


def test_layout_matches_reference_proxy_h(pkg):
    if not os.path.exists(LAYOUT):
        pytest.skip("oracle/_ref/proxy_layout not built (reference tree absent on this machine)")
    lay = json.loads(subprocess.run([LAYOUT], capture_output=True, text=True, check=True).stdout)
    abi = pkg.abi
    assert lay["header"] == lay["connect"] == lay["close"] == abi.REC_CONNECT_BYTES
    assert lay["send"] == abi.REC_SEND_BYTES and lay["send_data"] == abi.REC_DATA_OFF
    assert (lay["connection_id"], lay["action"]) == (0, 2)                 # clt_id@24, type@26 of the entry
    assert (lay["CONNECT"], lay["SEND"], lay["CLOSE"]) == (abi.PROXY_CONNECT, abi.PROXY_SEND, abi.PROXY_CLOSE)


def _known_dumps():
    """CONNECT(7); SEND(7, "hello"); CLOSE(7) -- then an unknown action, then
    a SEND whose cmd.len runs past the snapshot, then a 3-byte tail"""
    def hdr(conn, action):
        return bytes([conn & 0xFF, conn >> 8, action, 0])
    send = hdr(7, 5) + bytes(4) + (5).to_bytes(2, "little") + b"hello" + bytes(24 - 10)
    good = hdr(7, 4) + send + hdr(7, 6)
    dumps = np.zeros((4, 64), np.uint8)
    sizes = []
    for k, blob in enumerate((good, good + hdr(9, 3) + hdr(9, 4), good + send[:20], good + b"\x01\x02\x03")):
        dumps[k, :len(blob)] = np.frombuffer(blob, np.uint8)
        sizes.append(len(blob))
    return dumps, np.array(sizes, np.uint32), len(good)


def random_snapshots(n=3000, S=512, seed=5):
    """snapshots of mostly valid records with the odd unknown action and
    truncated tails (the GPU garbage test and records.json share them)"""
    rng = np.random.default_rng(seed)
    dumps = np.zeros((n, S), np.uint8)
    sizes = np.zeros(n, np.uint32)
    for k in range(n):
        blob = bytearray()
        while len(blob) < S - 300:
            a = int(rng.choice([4, 5, 6, 5, 5, 1]))
            conn = int(rng.integers(0, 1 << 16))
            if a == 5:
                ln = int(rng.integers(0, 200))
                blob += bytes([conn & 0xFF, conn >> 8, 5, 0]) + bytes(4) + ln.to_bytes(2, "little") + \
                    rng.integers(0, 256, 14 + ln, dtype=np.uint8).tobytes()
            else:
                blob += bytes([conn & 0xFF, conn >> 8, a, 0])
        sizes[k] = min(len(blob), S) - int(rng.integers(0, 3)) * int(rng.random() < 0.3)
        dumps[k, :min(len(blob), S)] = np.frombuffer(bytes(blob[:S]), np.uint8)
    return dumps, sizes


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def store_digests(dump, dump_len, n, cursor, bad):
    return {"dump_sha256": sha(dump), "dump_len_sha256": sha(dump_len), "n_sha256": sha(n),
            "cursor_sha256": sha(cursor), "corrupt": int(bad), "records": int(np.asarray(n).sum())}


def load_digests(out):
    return {k: sha(out[k]) for k in ("n_records", "status", "stop", "counts", "plan")}


def _check_known(out, n_good):
    assert list(out["n_records"]) == [3, 3, 3, 3]
    assert list(out["status"]) == [0, 1, 2, 2]
    assert list(out["stop"]) == [n_good] * 4
    for k in range(4):
        pl = out["plan"][k]
        assert [(int(r["offset"]), int(r["data_len"]), int(r["connection_id"]), int(r["action"])) for r in pl[:3]] == \
            [(0, 0, 7, 4), (4, 5, 7, 5), (33, 0, 7, 6)]
        assert list(out["counts"][k]) == [1, 1, 1]


def test_load_known_answers(orc):
    dumps, sizes, n_good = _known_dumps()
    _check_known(orc.records_load(dumps, sizes, 8), n_good)


@pytest.mark.parametrize("name", list(TRACES))
def test_oracle_store_matches_model_and_round_trips(pkg, orc, name):
    hb = _host(pkg, orc, name)
    G = hb.G
    cap = 4096
    cursor = hb.state["head"].copy()
    c0 = cursor.copy()
    dump, dl, n, bad = orc.records_store(hb, cursor, cap)
    n_bad = 0
    for g in range(G):
        exp, en, eo, eb = _py_store(hb, g, c0[g], cap)
        assert dump[g, :dl[g]].tobytes() == exp and n[g] == en and cursor[g] == eo, g
        n_bad += eb
    assert bad == n_bad
    ld = orc.records_load(dump, dl, 64)
    assert np.array_equal(ld["n_records"], n)
    assert (ld["status"] == 0).all() and np.array_equal(ld["stop"], dl)
    assert ld["counts"].sum() == n.sum()


def _fixture():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.mark.parametrize("name", list(TRACES))
def test_oracle_matches_records_fixture(pkg, orc, name):
    """the oracle's store and load equal the reference-composed results
    records.json holds (written from oracle/_ref by make_golden.py)"""
    fx = _fixture()
    hb = _host(pkg, orc, name)
    for cap in GOLDEN_CAPS:
        e = fx["store"][f"{name}/{cap}"]
        assert e["input_sha256"] == sha(hb.ring) + ":" + sha(hb.state), "trace generator drifted"
        cur = hb.state["head"].copy()
        dump, dl, n, bad = orc.records_store(hb, cur, cap)
        got = store_digests(dump, dl, n, cur, bad)
        assert got == {k: e[k] for k in got}, (name, cap)
        assert load_digests(orc.records_load(dump, dl, GOLDEN_PLAN)) == e["load"], (name, cap)


def test_oracle_load_matches_records_fixture(orc):
    fx = _fixture()["load_random"]
    dumps, sizes = random_snapshots()
    assert sha(dumps) == fx["dumps_sha256"] and sha(sizes) == fx["sizes_sha256"]
    assert load_digests(orc.records_load(dumps, sizes, 32)) == fx["load"]
    d, s, _ = _known_dumps()
    assert load_digests(orc.records_load(d, s, 8)) == _fixture()["load_known"]


def _have_ref(orc):
    if orc.ref() is None or not hasattr(orc.ref(), "ref_records_store_one"):
        pytest.skip("oracle/_ref not built (reference tree absent on this machine)")


@pytest.mark.parametrize("name", list(TRACES))
def test_oracle_matches_reference_composed_records(pkg, orc, name):
    """store (every capacity of the fixture and the two-call form of the GPU
    test) and load, the oracle against oracle/_ref directly"""
    _have_ref(orc)
    hb = _host(pkg, orc, name)
    for cap in GOLDEN_CAPS:
        c1, c2 = hb.state["head"].copy(), hb.state["head"].copy()
        a = orc.records_store(hb, c1, cap)
        b = orc.ref_records_store(hb, c2, cap)
        assert store_digests(*a[:3], c1, a[3]) == store_digests(*b[:3], c2, b[3]), (name, cap)
        assert load_digests(orc.records_load(a[0], a[1], GOLDEN_PLAN)) == \
            load_digests(orc.ref_records_load(a[0], a[1], GOLDEN_PLAN))


@pytest.mark.parametrize("name", list(TRACES))
def test_reference_batch_forms_equal_per_group(pkg, orc, name):
    """oracle/_ref's ref_records_store_batch / ref_records_load_batch (the
    whole-batch checkers of tests/test_whole_batch.py) equal the per-group calls"""
    _have_ref(orc)
    hb = _host(pkg, orc, name)
    cap = 1024
    c1, c2 = hb.state["head"].copy(), hb.state["head"].copy()
    a = orc.ref_records_store(hb, c1, cap)
    dump, dl, nr = np.zeros(hb.G * cap, np.uint8), np.zeros(hb.G, np.uint32), np.zeros(hb.G, np.uint32)
    bad = orc.ref_records_store_batch(hb.G, hb.stride, hb.ring, hb.state.view(np.uint8), c2, dump, cap, dl, nr)
    assert store_digests(*a[:3], c1, a[3]) == store_digests(dump.reshape(hb.G, cap), dl, nr, c2, bad)
    r1 = orc.ref_records_load(a[0], a[1], GOLDEN_PLAN)
    r2 = orc.ref_records_load_batch(dump, cap, dl, GOLDEN_PLAN)
    for k in ("n_records", "status", "stop"):
        assert np.array_equal(r1[k], r2[k]), k
    assert np.array_equal(r1["counts"].reshape(-1), r2["counts"])
    assert np.ascontiguousarray(r1["plan"]).tobytes() == r2["plan"].tobytes()


@pytest.mark.parametrize("G,all_groups", [(2048, False), (1024, True)])
def test_oracle_matches_reference_composed_on_malformed(pkg, orc, G, all_groups):
    """corrupt logs and random cursors: the oracle's stops are the
    reference-composed walk's (its BUILD-ONLY guards)"""
    _have_ref(orc)
    import test_gpu_parity as tg
    hb = tg._malformed(pkg, orc, G, 77 + G, all_groups)
    rng = np.random.default_rng(G)
    L = int(hb.state["len"][0])
    cur = np.where(rng.random(G) < 0.5, hb.state["head"], rng.integers(0, L + 1, G)).astype(np.uint64)
    c1, c2 = cur.copy(), cur.copy()
    a = orc.records_store(hb, c1, 1536)
    b = orc.ref_records_store(hb, c2, 1536)
    assert store_digests(*a[:3], c1, a[3]) == store_digests(*b[:3], c2, b[3])
    assert a[3] > 0
    dumps, sizes = random_snapshots(n=600, seed=G)
    assert load_digests(orc.records_load(dumps, sizes, 16)) == load_digests(orc.ref_records_load(dumps, sizes, 16))


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def eng(pkg):
    import torch
    assert torch.cuda.is_available()
    e = pkg.Engine(0)
    yield e
    e.close()


def _gpu_store(pkg, eng, batch, G, cursor, cap, dump=None, dump_len=None, flags=0):
    import torch
    d_cur = torch.from_numpy(cursor.view(np.int64).copy()).cuda()
    d_dump = torch.zeros(G * cap, dtype=torch.uint8, device="cuda") if dump is None else \
        torch.from_numpy(dump.reshape(-1).copy()).cuda()
    d_len = torch.zeros(G, dtype=torch.int32, device="cuda") if dump_len is None else \
        torch.from_numpy(dump_len.view(np.int32).copy()).cuda()
    d_n = torch.zeros(G, dtype=torch.int32, device="cuda")
    eng.records_store(batch, d_cur, d_dump, cap, d_len, d_n, flags=flags)
    torch.cuda.synchronize()
    return (d_dump.cpu().numpy().reshape(G, cap), d_len.cpu().numpy().view(np.uint32),
            d_n.cpu().numpy().view(np.uint32), d_cur.cpu().numpy().view(np.uint64))


# 0: 16-lane speculative segments; 0x1 (APUS_BATCH_LANE_IMPL): a lane per chain
IMPLS = [0, 0x1]


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("image", [False, True])
@pytest.mark.parametrize("name", list(TRACES))
def test_gpu_store_then_load_match_oracle(pkg, orc, eng, name, image, impl):
    import torch
    abi = pkg.abi
    hb = _host(pkg, orc, name)
    G, L = hb.G, TRACES[name][2]["ring_len"]
    if image:
        batch = pkg.batch.LogImageBatch(G, hb.R, L)
        batch.fill_from(hb)
    else:
        batch = pkg.batch.DeviceBatch(G, hb.R, hb.stride)
        batch.upload(hb)
    # two calls: the history [head, commit) first (end moved to commit), then
    # the rest; the second appends to the first's dumps.  A small cap stops
    # some groups (a full dump).
    cap = 1024 if name == "r7_mix" else 2048
    h1 = orc.host_batch(G, hb.R, L)
    h1.ring[:] = hb.ring
    for k, v in hb.arrays.items():
        h1.arrays[k][:] = v
    h1.state["end"] = hb.state["commit"]
    cur = hb.state["head"].copy()
    exp_dump, exp_len, exp_n, bad1 = orc.records_store(h1, cur, cap)
    if image:
        b1 = pkg.batch.LogImageBatch(G, hb.R, L)
        b1.fill_from(h1)
    else:
        b1 = pkg.batch.DeviceBatch(G, hb.R, hb.stride)
        b1.upload(h1)
    eng.stats_reset()
    got_dump, got_len, got_n, got_cur = _gpu_store(pkg, eng, b1, G, hb.state["head"].copy(), cap, flags=impl)
    assert np.array_equal(got_cur, cur) and np.array_equal(got_len, exp_len) and np.array_equal(got_n, exp_n)
    assert np.array_equal(got_dump, exp_dump)
    assert int(eng.stats()[abi.STAT_CORRUPT]) == bad1
    exp_dump, exp_len, exp_n, bad2 = orc.records_store(hb, cur, cap, exp_dump, exp_len)
    eng.stats_reset()
    got_dump, got_len, got_n, got_cur2 = _gpu_store(pkg, eng, batch, G, got_cur, cap, got_dump, got_len, flags=impl)
    assert np.array_equal(got_cur2, cur) and np.array_equal(got_len, exp_len) and np.array_equal(got_n, exp_n)
    assert np.array_equal(got_dump, exp_dump)
    assert int(eng.stats()[abi.STAT_CORRUPT]) == bad2
    assert exp_n.sum() > 0
    # the snapshots replayed
    M = 48
    ref = orc.records_load(exp_dump, exp_len, M)
    out = eng.records_load(torch.from_numpy(exp_dump.reshape(-1).copy()).cuda(), cap,
                           torch.from_numpy(exp_len.view(np.int32).copy()).cuda(), M, flags=impl)
    torch.cuda.synchronize()
    for k in ("n_records", "status", "stop"):
        assert np.array_equal(out[k].cpu().numpy().view(np.uint32), ref[k]), k
    assert np.array_equal(out["counts"].cpu().numpy().view(np.uint32).reshape(G, 3), ref["counts"])
    assert out["plan"].cpu().numpy().tobytes() == np.ascontiguousarray(ref["plan"]).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
def test_gpu_load_known_answers_and_garbage(pkg, orc, eng, impl):
    import torch
    dumps, sizes, n_good = _known_dumps()
    out = eng.records_load(torch.from_numpy(dumps.reshape(-1).copy()).cuda(), dumps.shape[1],
                           torch.from_numpy(sizes.view(np.int32).copy()).cuda(), 8, flags=impl)
    torch.cuda.synchronize()
    host = {k: (v.cpu().numpy().view(np.uint32) if k != "plan" else
                v.cpu().numpy().view(orc.records_load(dumps, sizes, 8)["plan"].dtype).reshape(4, 8))
            for k, v in out.items()}
    host["counts"] = host["counts"].reshape(4, 3)
    _check_known(host, n_good)
    # random snapshots: mostly valid records with the odd garbage byte
    dumps, sizes = random_snapshots()
    S = dumps.shape[1]
    ref = orc.records_load(dumps, sizes, 32)
    out = eng.records_load(torch.from_numpy(dumps.reshape(-1).copy()).cuda(), S,
                           torch.from_numpy(sizes.view(np.int32).copy()).cuda(), 32, flags=impl)
    torch.cuda.synchronize()
    for k in ("n_records", "status", "stop"):
        assert np.array_equal(out[k].cpu().numpy().view(np.uint32), ref[k]), k
    assert out["plan"].cpu().numpy().tobytes() == np.ascontiguousarray(ref["plan"]).tobytes()
    assert set(np.unique(ref["status"])) >= {0, 1}
    # and the reference-composed replay of the same snapshots (records.json)
    gd = {k: out[k].cpu().numpy().view(np.uint32) for k in ("n_records", "status", "stop")}
    gd["counts"] = out["counts"].cpu().numpy().view(np.uint32).reshape(-1, 3)
    gd["plan"] = out["plan"].cpu().numpy()
    assert load_digests(gd) == _fixture()["load_random"]["load"]


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("name", list(TRACES))
def test_gpu_store_matches_records_fixture(pkg, orc, eng, name, impl):
    """apus_records_store_batch from head, one call per capacity, and the
    replay of its snapshots: digests equal to records.json (the
    reference-composed results)"""
    import torch
    fx = _fixture()
    hb = _host(pkg, orc, name)
    G = hb.G
    db = pkg.batch.DeviceBatch(G, hb.R, hb.stride)
    db.upload(hb)
    for cap in GOLDEN_CAPS:
        e = fx["store"][f"{name}/{cap}"]
        eng.stats_reset()
        dump, dl, n, cur = _gpu_store(pkg, eng, db, G, hb.state["head"].copy(), cap, flags=impl)
        bad = int(eng.stats()[pkg.abi.STAT_CORRUPT])
        got = store_digests(dump, dl, n, cur, bad)
        assert got == {k: e[k] for k in got}, (name, cap)
        out = eng.records_load(torch.from_numpy(dump.reshape(-1).copy()).cuda(), cap,
                               torch.from_numpy(dl.view(np.int32).copy()).cuda(), GOLDEN_PLAN, flags=impl)
        torch.cuda.synchronize()
        gd = {k: out[k].cpu().numpy().view(np.uint32) for k in ("n_records", "status", "stop")}
        gd["counts"] = out["counts"].cpu().numpy().view(np.uint32).reshape(G, 3)
        gd["plan"] = out["plan"].cpu().numpy()
        assert load_digests(gd) == e["load"], (name, cap)


@pytest.mark.gpu
@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("G,all_groups", [(2048, False), (1024, True)])
def test_gpu_store_on_malformed_rings(pkg, orc, eng, G, all_groups, impl):
    """corrupt logs (end inside an entry: a walk the reference never leaves;
    garbage types and lengths; random cursors) stop exactly where the
    one-lane oracle walk stops, on every cursor, length and dump byte"""
    import test_gpu_parity as tg
    abi = pkg.abi
    hb = tg._malformed(pkg, orc, G, 77 + G, all_groups)
    rng = np.random.default_rng(G)
    L = int(hb.state["len"][0])
    cur = np.where(rng.random(G) < 0.5, hb.state["head"], rng.integers(0, L + 1, G)).astype(np.uint64)
    cap = 1536
    db = pkg.batch.DeviceBatch(G, hb.R, hb.stride)
    db.upload(hb)
    eng.stats_reset()
    got_dump, got_len, got_n, got_cur = _gpu_store(pkg, eng, db, G, cur.copy(), cap, flags=impl)
    exp_dump, exp_len, exp_n, bad = orc.records_store(hb, cur, cap)
    assert np.array_equal(got_cur, cur) and np.array_equal(got_len, exp_len) and np.array_equal(got_n, exp_n)
    assert np.array_equal(got_dump, exp_dump)
    assert int(eng.stats()[abi.STAT_CORRUPT]) == bad and bad > 0
