"""Generate tests/golden/lr_vectors.json (run in the build container, needs
oracle/_ref built from /root/reference).

For every trace of tests/test_lr_step.py (seeded, rebuilt identically on any
box) this records the SHA-256 of the inputs and of every output of
log_adjustment (dare_ibv_rc.c:1292-1451) and of a following
handle_lr_work_completion pass (:3126-3196), computed by the
reference-composed oracle (oracle/ref_compose.c: ref_log_adjust /
ref_lr_completion on the reference's own dare_log.h primitives).  The GPU
tests check libapus_gpu against these digests on boxes without the reference.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def digests(hb, io):
    out = {k: sha(getattr(hb, k)) for k in ("state", "lr_step", "remote_commit", "remote_end")}
    out.update({k: sha(io[k]) for k in ("send_flag", "send_count", "ssn", "post")})
    return out


def input_digest(hb, io):
    h = hashlib.sha256(hb.ring.tobytes())
    for k in sorted(hb.arrays):
        h.update(hb.arrays[k].view(np.uint8).tobytes())
    for k in ("send_flag", "send_count", "wc", "nc_len", "nc_dets", "ssn"):
        h.update(np.ascontiguousarray(io[k]).view(np.uint8).tobytes())
    return h.hexdigest()


def completion_wc(io):
    """the WRs just posted complete: success, or failure for every 7th pair"""
    n = io["post"].size
    return np.where(io["post"] != 0, np.where(np.arange(n) % 7 == 3, 2, 1), 0).astype(np.uint8)


def main():
    import apus_pkg
    from oracle import oracle as orc
    import test_lr_step as T
    pkg = apus_pkg.load_package()
    assert orc.ref() is not None, "oracle/_ref not built"
    res = {}
    for name in T.CASES:
        hb, io = T.build(pkg, orc, name)
        rec = {"input": input_digest(hb, io)}
        orc.ref_log_adjust(hb, io)
        rec["adjust"] = digests(hb, io)
        io["wc"][:] = completion_wc(io)
        orc.ref_lr_completion(hb, io)
        rec["completion"] = digests(hb, io)
        res[name] = rec
    with open(os.path.join(HERE, "lr_vectors.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("wrote lr_vectors.json:", ", ".join(res))


if __name__ == "__main__":
    main()
