"""GPU-box step runner: every GPU command of this repository's gpurun calls.

    python3 scripts/gpu_steps.py STEP [STEP ...]
    STEP  := NAME[@SECONDS]=KIND[:ARGS]
    KIND  := pytest   ARGS: pytest arguments (default: tests); -m gpu, -x, a per-test timeout added
           | smoke    __graft_entry__.smoke()
           | bench    ARGS: bench.py arguments
           | trun     ARGS: bench.py arguments, as one rank under torch.distributed.run (the driver's launch)
           | kb       ARGS: scripts/kbench.py arguments
           | scalar   ARGS: scripts/scalar_latency.py arguments
           | prof     ARGS: bench.py arguments, under rocprofv3 --kernel-trace --stats (csv in gpurun_out/NAME/)
           | profkb   ARGS: kbench.py arguments, the same
           | profpy   ARGS: SCRIPT ARGS (a script under scripts/), the same
           | sh       ARGS: SCRIPT ARGS (a bash script under scripts/: A/B runs of several builds)
           | avail    rocprofv3 --list-avail (the counters this GPU offers)
           | pmc      ARGS: COUNTER[,COUNTER...]|PROGRAM ARGS (PROGRAM bench.py or kbench.py), one
                      rocprofv3 --pmc pass (counters only, no tracing), killed after SECONDS
           | pmce     ARGS: YAML|COUNTER[,COUNTER...]|PROGRAM ARGS: the same with derived counters
                      defined in YAML (rocprofv3 -E)
Each step runs under its own time limit (default 600 s; pmc 120 s) with its
output in gpurun_out/NAME.log; the first step that fails, times out or
crashes ends the run (nothing else touches the GPU after it).  This process
never initialises the GPU itself: every step is a child process.
"""
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PY = "python3"


def command(name, kind, args):
    a = shlex.split(args)
    prof = ["rocprofv3", "--kernel-trace", "--stats", "-d", os.path.join(OUT, name), "-o", "run",
            "--output-format", "csv", "--"]
    if kind == "pytest":
        return [PY, "-u", "-m", "pytest"] + (a or ["tests"]) + ["-m", "gpu", "-x", "-q", "-p", "no:cacheprovider",
                                                                  "--timeout", "300", "--timeout-method", "thread"]
    if kind == "avail":
        return ["rocprofv3", "--list-avail"]
    if kind == "smoke":
        return [PY, "-c", "import __graft_entry__ as g; g.smoke()"]
    if kind == "bench":
        return [PY, "bench.py"] + a
    if kind == "trun":
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        return [PY, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr", "127.0.0.1",
                "--master-port", str(port), "bench.py", "--gpus", "1"] + a
    if kind == "kb":
        return [PY, "scripts/kbench.py"] + a
    if kind == "scalar":
        return [PY, "scripts/scalar_latency.py"] + a
    if kind == "prof":
        return prof + [PY, "bench.py"] + a
    if kind == "profkb":
        return prof + [PY, "scripts/kbench.py"] + a
    if kind == "sh":
        return ["bash", "scripts/" + a[0]] + a[1:]
    if kind == "profpy":
        return prof + [PY, "scripts/" + a[0]] + a[1:]
    if kind in ("pmc", "pmce"):
        extra = []
        if kind == "pmce":
            yml, args = args.split("|", 1)
            extra = ["-E", yml]
        counters, prog = args.split("|", 1)
        p = shlex.split(prog)
        script = p[0] if p[0].startswith("scripts/") or p[0] == "bench.py" else "scripts/" + p[0]
        return ["rocprofv3"] + extra + ["--pmc"] + counters.split(",") + ["-d", os.path.join(OUT, name), "-o", "run",
                                                                "--output-format", "csv", "--", PY, script] + p[1:]
    raise SystemExit(f"unknown step kind {kind!r}")


def main():
    os.chdir(ROOT)
    os.makedirs(OUT, exist_ok=True)
    os.environ.setdefault("TMPDIR", "/tmp")
    for step in sys.argv[1:]:
        head, _, rest = step.partition("=")
        name, _, limit = head.partition("@")
        kind, _, args = rest.partition(":")
        secs = int(limit) if limit else (120 if kind in ("pmc", "pmce") else 600)
        cmd = command(name, kind, args)
        log = os.path.join(OUT, name + ".log")
        print(f"== {name} ({secs} s): {' '.join(cmd)}", flush=True)
        t0 = time.time()
        with open(log, "w") as f:
            p = subprocess.Popen(cmd, stdout=f, stderr=subprocess.STDOUT, start_new_session=True)
            try:
                rc = p.wait(timeout=secs)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, 9)
                p.wait()
                rc = 124
        with open(log) as f:
            tail = f.read()[-1500:]
        print(tail, flush=True)
        print(f"== {name} rc={rc} {time.time() - t0:.0f} s", flush=True)
        if rc != 0:
            sys.exit(rc)
    print("== done", flush=True)


if __name__ == "__main__":
    main()
