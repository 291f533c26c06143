"""Debug helper: run one tests/test_append.py case on the GPU and print where
device and oracle rings differ after persist."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import apus_pkg
import test_append as T
pkg = apus_pkg.load_package(); orc = apus_pkg.load_oracle()
eng = pkg.Engine(0)
name = sys.argv[1] if len(sys.argv) > 1 else "mixed"
hb, ent, payload, M, n_entries = T.build(pkg, orc, name)
db = T._dev(pkg, hb)
eng.log_append_entry(db, torch.from_numpy(ent.view(np.uint8).copy()).cuda(), torch.from_numpy(payload).cuda(), M,
                     n_entries=torch.from_numpy(n_entries.view(np.int32).copy()).cuda())
orc.append(hb, ent, payload, M, n_entries=n_entries)
torch.cuda.synchronize()
print("append ring equal:", np.array_equal(db.download("ring"), hb.ring))
old_end, limit = T.persist_inputs(hb, 9, hb.end0)
oe0 = old_end.copy()
d_oe = torch.from_numpy(old_end.view(np.int64).copy()).cuda()
eng.persist_new_entries(db, d_oe, torch.from_numpy(limit.view(np.int32).copy()).cuda())
orc.persist(hb, old_end, limit)
torch.cuda.synchronize()
dr = db.download("ring"); doe = d_oe.cpu().numpy().view(np.uint64)
print("old_end equal:", np.array_equal(doe, old_end))
bad = np.nonzero(dr != hb.ring)[0]
print("differing bytes:", bad.size)
R = hb.R
for pos in bad[:20]:
    g, o = divmod(int(pos), hb.stride)
    st = hb.state[g]
    print(f"g={g} off={o} dev={dr[pos]} orc={hb.ring[pos]} self={hb.self_idx[g]} end={st['end']} len={st['len']} "
          f"commit={st['commit']} oe0={oe0[g*R:(g+1)*R]} lim={limit[g*R:(g+1)*R]} oe_dev={doe[g*R:(g+1)*R]} oe_orc={old_end[g*R:(g+1)*R]}")
