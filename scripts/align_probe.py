"""Walk time against the ring array's base offset (experiment): the C5 shard
shape (2^23 groups x R=7, 16 entries, 8-KiB rings, configuration mix) on
commit_seg_kernel (walk + checksum), the ring placed at several byte offsets
from the start of one larger allocation, each generated in place and timed
with HIP events; the same offsets twice, interleaved.  Prints one JSON line
per offset: the base address mod 2 MiB and the median of the timed calls."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--offsets", default="0,256,1024,4096,16384,65536,262144,1048576")
    ap.add_argument("--groups", type=int, default=1 << 23)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi
    eng = pkg.Engine(0)
    lib = eng.lib
    G, R = args.groups, 7
    stride = pkg.batch.ring_stride_for(8192)
    offs = [int(x) for x in args.offsets.split(",")]
    db = pkg.batch.DeviceBatch(G, R, stride, fields=["state", "self_idx", "remote_end", "lr_step", "fail_count"])
    big = torch.empty(G * stride + max(offs), dtype=torch.uint8, device="cuda")
    db.ring = None
    torch.cuda.empty_cache()
    cfg = pkg.batch.gen_cfg(seed=2026, n_entries=16, n_history=16, len_min=64, len_max=64, ring_len=8192,
                            p_full_ack=0.9, straggler=True, cid_mix=True)
    flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM
    out = eng.alloc_commit_out(G, flags)
    o = eng.commit_struct(out)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = {}
    for rnd in range(2):
        for off in offs:
            db.ring = big[off:off + G * stride]
            eng.gen(db, cfg)
            b = db.struct()
            b.flags = abi.BATCH_SHORT_WALKS
            ms = []
            for _ in range(args.reps + 1):
                ev[0].record()
                abi.check(lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), flags, None), "commit")
                ev[1].record()
                torch.cuda.synchronize()
                ms.append(ev[0].elapsed_time(ev[1]))
            res.setdefault(off, []).append(float(np.median(ms[1:])))
            print(json.dumps({"round": rnd, "offset": off, "base_mod_2M": db.ring.data_ptr() % (1 << 21),
                              "ms": round(float(np.median(ms[1:])), 4)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
