"""Experiment builds only (scripts/build_exp.sh phases=-DAPUS_EXP_PHASES): where
commit_wave_kernel's cycles go per group, C2 batch.  Usage:
  APUS_GPU_LIB=$PWD/build_exp/libapus_phases.so python scripts/phase_probe.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi
    eng = pkg.Engine(0)
    lib = eng.lib
    G, R, L = 1 << 20, 3, 16384
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, pkg.batch.gen_cfg(seed=2026, n_entries=64, n_history=16, len_min=64, len_max=64, ring_len=L,
                                  p_full_ack=0.9, straggler=True))
    out = eng.alloc_commit_out(G, 7)
    o = eng.commit_struct(out)
    b = db.struct()
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    ph = (C.c_uint64 * 8)()
    lib.apus_exp_phases(ph)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    runs = 5
    lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), abi.COMMIT_WALK | abi.COMMIT_CHECKSUM, sp)
    torch.cuda.synchronize()
    lib.apus_exp_phases(ph)
    t0.record()
    for _ in range(runs):
        lib.apus_commit_batch(eng.ctx, C.byref(b), C.byref(o), abi.COMMIT_WALK | abi.COMMIT_CHECKSUM, sp)
    t1.record()
    torch.cuda.synchronize()
    assert lib.apus_exp_phases(ph) == 0
    v = [int(x) for x in ph]
    n = v[6]
    names = ["stage", "prefetch_issue", "walk", "fold", "group_epilogue", "block_epilogue", "groups", "data_wait"]
    res = {"ms_per_launch": t0.elapsed_time(t1) / runs, "groups": n}
    tot = sum(v[k] for k in (0, 1, 2, 3, 4, 5, 7))
    for k, nm in enumerate(names):
        if k == 6:
            continue
        res[nm + "_cycles_per_group"] = v[k] / max(n, 1)
        res[nm + "_frac"] = v[k] / max(tot, 1)
    print(json.dumps(res, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
