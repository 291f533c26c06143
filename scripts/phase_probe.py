"""(Needs the APUS_EXP_* branches restored first: git apply profiles/r04/exp_knobs.diff
in a scratch checkout; the product sources no longer carry them.)
Experiment builds only (scripts/build_exp.sh phases=-DAPUS_EXP_PHASES): where
commit_wave_kernel's (or, with --append, append_kernel's) cycles go per group,
C2 batch (--c3: a C3 wave).  Usage:
  APUS_GPU_LIB=$PWD/build_exp/libapus_phases.so python scripts/phase_probe.py [--append | --c3]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def append_main():
    import torch
    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi
    eng = pkg.Engine(0)
    lib = eng.lib
    G, R, L, M, P = 1 << 20, 3, 16384, 64, 64
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, pkg.batch.gen_cfg(seed=2026, n_entries=64, n_history=16, len_min=64, len_max=64, ring_len=L,
                                  p_full_ack=0.9, straggler=True))
    n = G * M
    need = 2 + P
    g = torch.Generator(device="cuda").manual_seed(7)
    ent = torch.zeros(n, 24, dtype=torch.uint8, device="cuda")
    e64 = ent.view(torch.int64).view(n, 3)
    e64[:, 0] = torch.randint(0, 1 << 62, (n,), device="cuda", generator=g)
    e64[:, 1] = torch.arange(n, device="cuda", dtype=torch.int64) * need
    e64[:, 2] = torch.randint(0, 1 << 16, (n,), device="cuda", generator=g) | (5 << 16)
    payload = torch.randint(0, 256, (n * need,), dtype=torch.uint8, device="cuda", generator=g)
    pv = payload.view(n, need)
    pv[:, 0] = P
    pv[:, 1] = 0
    st0 = db.arrays["state"].clone()
    out_idx = eng._z(G, torch.int64, M)
    ai = abi.AppendIn(entries=ent.data_ptr(), n_entries=None, term=None, payload=payload.data_ptr(),
                      payload_bytes=payload.numel(), max_entries=M)
    ao = abi.AppendOut(idx=out_idx.data_ptr(), last_idx=None)
    b = db.struct()
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    ph = (C.c_uint64 * 8)()
    runs = 3
    tot_ms = 0.0
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(runs + 1):
        db.arrays["state"].copy_(st0)
        torch.cuda.synchronize()
        if r == 1:
            lib.apus_exp_append_phases(ph)
        t0.record()
        lib.apus_append_batch(eng.ctx, C.byref(b), C.byref(ai), C.byref(ao), sp)
        t1.record()
        torch.cuda.synchronize()
        if r >= 1:
            tot_ms += t0.elapsed_time(t1)
    assert lib.apus_exp_append_phases(ph) == 0
    v = [int(x) for x in ph]
    # fast_prefixes includes span_issue + span_wait + span_build (+ stores)
    names = ["group_setup", "fast_prefixes", "general_steps", "group_end", "groups", "span_issue", "span_wait",
             "span_build"]
    res = {"ms_per_launch": tot_ms / runs, "groups": v[4]}
    tot = sum(v[k] for k in range(4))
    for k, nm in enumerate(names):
        if nm == "groups":
            continue
        res[nm + "_cycles_per_group"] = v[k] / max(v[4], 1)
        res[nm + "_frac"] = round(v[k] / max(tot, 1), 4)
    print(json.dumps(res, indent=1))
    eng.close()


def main():
    if "--append" in sys.argv:
        return append_main()
    import torch
    import apus_pkg
    pkg = apus_pkg.load_package()
    abi = pkg.abi
    eng = pkg.Engine(0)
    lib = eng.lib
    # --c3: BASELINE configs[2]'s wave (2^18 groups, R=5, 64 entries of 128 B - 4 KiB, 336-KiB rings)
    c3 = "--c3" in sys.argv
    G, R, L = (1 << 18, 5, 344064) if c3 else (1 << 20, 3, 16384)
    pmax = 4096 if c3 else 64
    db = pkg.batch.DeviceBatch(G, R, pkg.batch.ring_stride_for(L))
    eng.gen(db, pkg.batch.gen_cfg(seed=2026, n_entries=64, n_history=16, len_min=64, len_max=pmax, ring_len=L,
                                  p_full_ack=0.9, straggler=True))
    out = eng.alloc_commit_out(G, 7)
    o = eng.commit_struct(out)
    b = db.struct()
    if c3 and "--no-hop" not in sys.argv:
        b.flags = abi.BATCH_VAR_LEN
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
