"""The one-launch scalar kernel's phases (argument load, compute, result
stores) on the GPU's constant clock, from an APUS_EXP_QTIME build
(scripts/build_exp.sh qtime=-DAPUS_EXP_QTIME; its kernel prints them):
walk / median calls on scalar_latency.py's log, for 1, 8 and 16 entries.

usage: APUS_GPU_LIB=build_exp/libapus_qtime.so python3 scripts/scalar_phases.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from scalar_latency import ref_shaped  # noqa: E402


def main():
    import apus_pkg
    pkg = apus_pkg.load_package()
    orc = apus_pkg.load_oracle()
    abi = pkg.abi
    lib = abi.load_library()
    R, L, G = 3, 16384, 16
    for entries in (1, 8, 16):
        cfg = pkg.batch.gen_cfg(seed=606, n_entries=entries, n_history=4, len_min=64, len_max=64, ring_len=L,
                                p_full_ack=0.7, straggler=True)
        hb = orc.host_batch(G, R, L)
        orc.gen(hb, cfg)
        ref = orc.commit(hb, abi.COMMIT_WALK)
        g = int(np.argmax(ref["committed"] == 1))
        buf, scfg, servers, ctrl = ref_shaped(abi, lib, hb, g, "heap")
        logp = C.c_void_p(buf.ctypes.data)
        nc, cm, md = C.c_uint64(0), C.c_int(0), C.c_uint64(0)
        print(f"== entries {entries}: walk x 20, median x 5", flush=True)
        for _ in range(20):
            assert lib.apus_commit_reply_walk(logp, C.byref(scfg), C.byref(nc), C.byref(cm)) == 0
        for _ in range(5):
            assert lib.apus_commit_median(logp, C.byref(scfg), C.byref(ctrl), C.byref(md)) == 0
        C.CDLL("libamdhip64.so").hipDeviceSynchronize()       # the kernels' printf drained
        sys.stdout.flush()


if __name__ == "__main__":
    main()
