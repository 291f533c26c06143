"""Summarise bench.py JSON lines from gpurun_out/<name>.log files:
    python3 scripts/bsum.py NAME [NAME ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for n in sys.argv[1:]:
    p = os.path.join(ROOT, "gpurun_out", n + ".log")
    try:
        d = json.loads(open(p).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError) as e:
        print(n, "--", type(e).__name__)
        continue
    r = d["roofline"]
    t = r.get("tail") or {}
    f = d.get("failover") or {}
    cb = d.get("cpu_baseline") or {}
    print(f"{n:12s} step {d['ms_per_step']:.4f} ms  walk {r['kernel_ms']:.4f} ({r['frac']:.3f})  "
          f"tail {t.get('kernel_ms', 0):.4f} ({t.get('frac', 0):.3f})  step_frac {r.get('step_frac', 0):.3f}  "
          f"value {d['value']:.3e}" + (f"  win cold {f['cold_win_ms']:.3f} steady {f['win_call_ms_steady']:.4f} "
                                       f"transitions {f['transitions']}" if f else "")
          + (f"  cpu {cb.get('value', 0):.3e} {cb.get('kind')}" if cb else ""))
