"""Dump the groups where the wave kernel and the oracle disagree on the
malformed-ring batch of tests/test_gpu_parity.py (debugging aid)."""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import apus_pkg  # noqa: E402

pkg, orc = apus_pkg.load_package(), apus_pkg.load_oracle()
spec = importlib.util.spec_from_file_location("tg", os.path.join(ROOT, "tests", "test_gpu_parity.py"))
tg = importlib.util.module_from_spec(spec)
spec.loader.exec_module(tg)
import torch  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
hb = tg._malformed(pkg, orc, G, 9 + G, G > 100000)
eng = pkg.Engine(0)
abi = pkg.abi
res = {}
for flags in (3, 1):
    ref = orc.commit(hb, flags)
    db = pkg.batch.DeviceBatch(G, hb.R, hb.stride)
    db.upload(hb)
    out = eng.update_remote_logs(db, flags)
    torch.cuda.synchronize()
    got = {k: v.cpu().numpy() for k, v in out.items()}
    nc = got["new_commit"].view(np.uint64)
    bad = np.nonzero((nc != ref["new_commit"]) | (got["committed"] != ref["committed"]))[0]
    print("flags", flags, "mismatches", len(bad))
    for g in bad[:12]:
        s = hb.state[g]
        print(" g", g, "commit", s["commit"], "end", s["end"], "len", s["len"], "self", hb.self_idx[g],
              "ref", ref["new_commit"][g], ref["committed"][g], ref["n_entries"][g],
              "got", nc[g], got["committed"][g], got["n_entries"].view(np.uint32)[g])
    res[f"bad{flags}"] = bad
    res[f"got_nc{flags}"] = nc
    res[f"got_cm{flags}"] = got["committed"]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "malformed.npz"), **res)
eng.close()
