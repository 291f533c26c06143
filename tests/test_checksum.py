"""Pin the build-defined checksum (no checksum exists in the reference):
Adler-32 as specified by RFC 1950 / implemented by zlib, over the concatenated
images of the walked entries (each entry's whole span with the RDMA-rewritten
bytes 27..47 -- sender, reply[], pad -- read as zero).  zlib.adler32 is an independent
implementation of the same published algorithm."""
import ctypes as C
import zlib

import numpy as np


def test_adler32_known_answers(orc):
    L = orc.lib()
    for data, want in [(b"", 1), (b"a", 0x00620062), (b"abc", 0x024D0127), (b"Wikipedia", 0x11E60398),
                       (b"message digest", 0x29750586)]:
        buf = np.frombuffer(data + b"\0", np.uint8)
        assert L.apus_oracle_adler32(C.c_void_p(buf.ctypes.data), len(data), 1) == want == zlib.adler32(data)


def test_adler32_vs_zlib_random(orc):
    L = orc.lib()
    rng = np.random.default_rng(3)
    for n in [1, 15, 16, 17, 255, 5552, 5553, 65536, 200001]:
        d = rng.integers(0, 256, n).astype(np.uint8)
        d[: n // 3] = 255                          # stress the modulo
        assert L.apus_oracle_adler32(C.c_void_p(d.ctypes.data), n, 1) == zlib.adler32(d.tobytes())


def _images(hb, g):
    """independent Python restatement of the image rule over the walk chain"""
    ring = hb.group_ring(g)
    s = hb.state[g]
    ln, end, m = int(s["len"]), int(s["end"]), int(s["commit"])

    def dist(o):
        return 0 if end == ln else (end - o if end >= o else ln - (o - end))
    out = bytearray()
    steps = 0
    while dist(m) and steps < ln // 64 + 4:
        steps += 1
        if ln - m < 64:
            m = 0
        t = int(ring[m + 26])
        clen = int(ring[m + 48]) | (int(ring[m + 49]) << 8)
        el = 64 if t in (0, 2, 3) else 64 + clen
        if ln - m < el:
            m = 0
            continue
        out += bytes(ring[m:m + 27]) + bytes(21) + bytes(ring[m + 48:m + el])
        m += el
    return bytes(out)


def test_group_checksum_is_adler32_of_images(orc, pkg):
    for kw in [dict(seed=31, ring_len=16384), dict(seed=32, ring_len=4500, n_entries=20, n_history=4, len_min=0,
                                                   len_max=80, type_mix=True, cid_mix=True)]:
        cfg = pkg.batch.gen_cfg(**kw)
        hb = orc.host_batch(200, 5, kw["ring_len"])
        orc.gen(hb, cfg)
        out = orc.commit(hb, pkg.abi.COMMIT_CHECKSUM)
        for g in range(hb.G):
            assert out["digest"][g] == zlib.adler32(_images(hb, g)), g
