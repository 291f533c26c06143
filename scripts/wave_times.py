"""(Needs the APUS_EXP_* branches restored first: git apply profiles/r04/exp_knobs.diff
in a scratch checkout; the product sources no longer carry them.)
Per-wave start / end timestamps of commit_seg_kernel (and commit_wave_kernel) (the
ramp and drain of the 2^23-group C5 walk against the 2^26-group batch).

Needs an experiment build with -DAPUS_EXP_WAVE_TIMES (scripts/build_exp.sh
wt=-DAPUS_EXP_WAVE_TIMES), loaded through APUS_GPU_LIB.  For each shape: a
few walk + checksum calls (APUS_BATCH_SHORT_WALKS), then the last launch's
per-wave s_memrealtime (100 MHz) at entry and exit, the blocks each walked
and its XCD; prints one JSON line per shape:
  span_us       first entry to last exit
  ramp_us       first to last entry
  busy          sum of wave lifetimes / (waves x span): 1 - idle share
  end_pct       exit times (us after the first entry) at 50/90/99/100 %
  blocks        blocks per wave: min / mean / max
  xcd_end_us    mean exit per XCD
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {
    # commit_wave_kernel (no hint): C2 and the C4 shard
    "c2": dict(G=1 << 20, R=3, E=64, H=16, ring=16384, cid_mix=False, short=False),
    "c4": dict(G=1 << 23, R=5, E=64, H=16, ring=16384, cid_mix=False, short=False),
    "c5": dict(G=1 << 23, R=7, E=16, H=16, ring=8192, cid_mix=True),
    "c4_1gpu": dict(G=1 << 26, R=5, E=16, H=2, ring=2448, cid_mix=False),
    "c4_1gpu_2e23": dict(G=1 << 23, R=5, E=16, H=2, ring=2448, cid_mix=False),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="c5,c4_1gpu")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi
    eng = pkg.Engine(0)
    lib = eng.lib
    f = lib.apus_exp_wave_times
    f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_uint32]
    for name in args.shapes.split(","):
        s = SHAPES[name]
        G, R = s["G"], s["R"]
        db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(s["ring"]),
                                   fields=["state", "self_idx", "remote_end", "lr_step", "fail_count"])
        cfg = pkg.batch.gen_cfg(seed=2026, n_entries=s["E"], n_history=s["H"], len_min=64, len_max=64,
                                ring_len=s["ring"], p_full_ack=0.9, straggler=True, cid_mix=s["cid_mix"])
        eng.gen(db, cfg)
        b = db.struct()
        b.flags = abi.BATCH_SHORT_WALKS if s.get("short", True) else 0
        flags = abi.COMMIT_WALK | abi.COMMIT_CHECKSUM
        w = eng.commit_walk_info(b, flags)
        out = eng.alloc_commit_out(G, flags)
        o = eng.commit_struct(out)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ms = []
        for _ in range(args.reps):
            ev[0].record()
            abi.check(lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), flags, None), "commit")
            ev[1].record()
            torch.cuda.synchronize()
            ms.append(ev[0].elapsed_time(ev[1]))
        nw = w["grid"] * 4
        buf = np.zeros(4 * nw, np.uint64)
        assert f(C.c_void_p(buf.ctypes.data), nw) == 0
        t = buf.reshape(nw, 4).astype(np.int64)
        st, en, nb = t[:, 0], t[:, 1], t[:, 2]
        xcd = (t[:, 3] >> 32) & 0xF
        t0 = st.min()
        span = (en.max() - t0) / 100.0            # 100 MHz ticks -> us
        busy = float((en - st).sum()) / (nw * (en.max() - t0))
        rel = (en - t0) / 100.0
        res = {"shape": name, "groups": G, "walk": w, "call_ms": [round(x, 4) for x in ms],
               "waves": int(nw), "span_us": round(span, 1), "ramp_us": round((st.max() - t0) / 100.0, 1),
               "busy": round(busy, 4),
               "end_pct": {str(p): round(float(np.percentile(rel, p)), 1) for p in (50, 90, 99, 100)},
               "start_pct": {str(p): round(float(np.percentile((st - t0) / 100.0, p)), 1) for p in (50, 90, 99, 100)},
               "blocks": [int(nb.min()), round(float(nb.mean()), 2), int(nb.max())],
               "xcd_end_us": {int(x): round(float(rel[xcd == x].mean()), 1) for x in np.unique(xcd)}}
        print(json.dumps(res), flush=True)
        del db, out
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
