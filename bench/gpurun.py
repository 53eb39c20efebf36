#!/usr/bin/env python3
"""One entry point for every GPU study: `python bench/gpurun.py <study> [--dry]`.

A study is a list of steps (name, time limit, command).  This script writes them as one bash
script under bench/.runs/ (part of the snapshot gpurun uploads) and runs it on the MI355X box with
/usr/local/graft/bin/gpurun.  Each step runs under its own `timeout -k 10`, writes its output to
gpurun_out/<study>/<step>.log, and the script stops at the first step that crashed, faulted or hit
its limit (exit codes 124/134/137/139 or >128); an ordinary non-zero exit (a failing test) is
recorded and the next step still runs.  Results land in gpurun_out/<study>/ on this machine;
copy the summaries worth keeping into profiles/.

Studies that back kept profiles name themselves in the profile's README.
"""
from __future__ import annotations

import argparse
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GPURUN = "/usr/local/graft/bin/gpurun"
PYTEST = "python -u -m pytest -x -v --timeout 170 --timeout-method thread"
ROCPROF = "rocprofv3 --kernel-trace --stats"


def bench(args: str) -> str:
    return f"python -u bench.py {args}"


def pmc(counters: str, cmd: str, out: str) -> str:
    # counters in their own pass, kernel trace only (never with sys/runtime traces)
    return f"timeout -s KILL 90 rocprofv3 --pmc {counters} -d gpurun_out/{out} -o pmc -- {cmd}"


STUDIES: dict[str, list[tuple[str, int, str]]] = {
    # round-3 first contact: launch path, ladder, accuracy; the default bench; an 8-rank rehearsal
    "launch": [
        ("pytest_launch", 420, f"{PYTEST} tests/test_gpu_launch_path.py"),
        ("bench_default", 300, bench("--gpus 1 --steps 20 --warmup 5")),
        ("share8", 420, bench("--gpus 8 --share-gpu --M 4096 --N 4096 --steps 20 --warmup 5")),
    ],
    # the whole GPU suite as the driver runs it
    "pytest_gpu": [
        ("pytest_gpu", 1100, f"{PYTEST} tests -m gpu"),
    ],
    "bench": [
        ("bench_default", 300, bench("--gpus 1 --steps 20 --warmup 5")),
        ("bench_200", 300, bench("--gpus 1 --steps 200 --warmup 20 --no-tol-solve")),
    ],
    "profile_default": [
        ("rocprof_bench", 300, f"{ROCPROF} -d gpurun_out/profile_default/rp -o run -- "
                               + bench("--gpus 1 --steps 60 --warmup 10 --no-tol-solve")),
    ],
}


def script(name: str, steps) -> str:
    lines = ["#!/bin/bash", "set -u", f"mkdir -p gpurun_out/{name}", "status=0"]
    for step, limit, cmd in steps:
        log = f"gpurun_out/{name}/{step}.log"
        lines += [
            f"echo '== {step} (limit {limit} s)'",
            f"timeout -k 10 {limit} {cmd} > {log} 2>&1",
            "rc=$?",
            f"echo \"{step} rc=$rc\" | tee -a gpurun_out/{name}/status.txt",
            "tail -3 " + log,
            "if [ $rc -ge 124 ]; then echo 'stopping: crash/fault/time limit'; exit $rc; fi",
            "if [ $rc -ne 0 ]; then status=$rc; fi",
        ]
    lines.append("exit $status")
    return "\n".join(lines) + "\n"


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("study", choices=sorted(STUDIES))
    ap.add_argument("--dry", action="store_true", help="write and print the script, do not run it")
    ap.add_argument("--timeout", type=int, default=0, help="gpurun limit (default: sum of the steps + 120 s)")
    a = ap.parse_args()
    steps = STUDIES[a.study]
    os.makedirs(os.path.join(ROOT, "bench", ".runs"), exist_ok=True)
    path = os.path.join("bench", ".runs", f"{a.study}.sh")
    with open(os.path.join(ROOT, path), "w") as f:
        f.write(script(a.study, steps))
    limit = a.timeout or min(1200, sum(s[1] for s in steps) + 120)
    cmd = [GPURUN, "--timeout", str(limit), "--", f"bash {shlex.quote(path)}"]
    print(" ".join(cmd), flush=True)
    if a.dry:
        print(open(os.path.join(ROOT, path)).read())
        return 0
    return subprocess.call(cmd, cwd=ROOT)


if __name__ == "__main__":
    sys.exit(main())
