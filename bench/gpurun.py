#!/usr/bin/env python3
"""One entry point for every GPU study: `python bench/gpurun.py <study> [--dry]`.

A study is a list of steps (name, time limit, command).  This script writes them as one bash
script under bench/.runs/ (part of the snapshot gpurun uploads) and runs it on the MI355X box with
/usr/local/graft/bin/gpurun.  Each step runs under its own `timeout -k 10`, writes its output to
gpurun_out/<study>/<step>.log, and the script stops at the first step that crashed, faulted or hit
its limit (exit codes 124/134/137/139 or >128); an ordinary non-zero exit (a failing test) is
recorded and the next step still runs.  Results land in gpurun_out/<study>/ on this machine;
copy the summaries worth keeping into profiles/.

Fixed studies (STUDIES) and parametrised ones (`<study> -- <arguments>`):
    ab        -- bench/ab_env.py arguments: interleaved same-box A/B of PMX_* knobs
    pmc       -- tag:ENV=V,... configurations, --args for bench.py, --passes (PMC_PASSES)
    timeline  -- grids MxN: rocprofv3 kernel trace of the CLI + bench/trace_timeline.py
    validate  -- GPU suite, smoke(), default bench
    share     -- rank counts: supervised multi-rank rehearsal on the one GPU
    cli       -- quoted pmx argument strings
    loopback  -- GPUS:RANK[:ENV=V,..]: one rank of an N-GPU job alone on the GPU (per-rank iteration)
    ca_ab     -- bench/probe/ca_env_ab.py arguments: same-process A/B of s-step knobs
    algos     -- MxN:algo:dtype: bench.py per grid x algorithm x storage
    counters  -- kernel trace + SQ / EA counter passes of one bench.py configuration
    cmds      -- ad-hoc steps 'tag:seconds:command'
Studies that back kept profiles name themselves in the profile's README; bench/RETIRED.md maps
the round-1/2 one-off gpu_*.sh scripts onto these.
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


# The Python processes (tests, bench.py) run torch's bundled HIP runtime and RCCL (ROCm 7.0 builds,
# SONAMEs libamdhip64.so.7 / librccl.so.1, loaded by `import torch` before _pmx.so); the CLI and the
# probes link /opt/rocm (7.2).  TORCH_RT + cmd + "'" runs a probe on torch's runtime instead.
TORCH_RT = ("bash -c 'TL=$(python3 -c \"import torch, os; print(os.path.dirname(torch.__file__))\")/lib; "
            "mkdir -p /tmp/pmx_torchrt && ln -sf $TL/libamdhip64.so /tmp/pmx_torchrt/libamdhip64.so.7 && "
            "LD_LIBRARY_PATH=/tmp/pmx_torchrt:$TL ")


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
    "ipc": [
        ("pytest_ipc", 600, f"{PYTEST} tests/test_gpu_dist.py -k 'ipc or share'"),
        ("pytest_launch", 420, f"{PYTEST} tests/test_gpu_launch_path.py -k 'bench'"),
        ("share8", 420, bench("--gpus 8 --share-gpu --M 4096 --N 4096 --steps 20 --warmup 5")),
    ],
    "pytest_gpu": [
        ("pytest_gpu", 1100, f"{PYTEST} tests -m gpu"),
    ],
    "bench": [
        ("bench_default", 300, bench("--gpus 1 --steps 20 --warmup 5")),
        ("bench_200", 300, bench("--gpus 1 --steps 200 --warmup 20 --no-tol-solve")),
    ],
    # binary A/B against a build of the previous commit copied to bench/ab/pmx_base (gitignored)
    "pf_ab": [
        ("fp64", 600, "python -u bench/ab_env.py --shape 16384x16384 --shape 2048x16384 --cfg base: "
                      "--cfg pf2:PMX_PCG1_PF=2 --cfg pf2w1:PMX_PCG1_PF=2,PMX_PCG1_PF_W=1 --rounds 4 --iters 300"),
        ("fp32", 600, "python -u bench/ab_env.py --shape 16384x16384 --shape 32768x32768 --dtype fp32 --cfg base: "
                      "--cfg pf2:PMX_PCG1_PF=2 --cfg pf3:PMX_PCG1_PF=3 --cfg pf2w1:PMX_PCG1_PF=2,PMX_PCG1_PF_W=1 "
                      "--cfg pf3w2:PMX_PCG1_PF=3,PMX_PCG1_PF_W=2 --cfg pf3w1:PMX_PCG1_PF=3,PMX_PCG1_PF_W=1 "
                      "--rounds 3 --iters 200"),
    ],
    "pf_ab2": [
        ("fp64", 900, "python -u bench/ab_env.py --shape 16384x16384 --shape 8192x16384 --shape 4096x16384 "
                      "--shape 2048x16384 --cfg base: --cfg pf2:PMX_PCG1_PF=2 --rounds 5 --iters 300"),
        ("fp32", 600, "python -u bench/ab_env.py --shape 16384x16384 --shape 32768x32768 --shape 2048x16384 "
                      "--dtype fp32 --cfg r24: --cfg r16:PMX_PCG1_ROWS=16 --cfg r20:PMX_PCG1_ROWS=20 "
                      "--cfg r32:PMX_PCG1_ROWS=32 --cfg pf1:PMX_PCG1_PF=1 --rounds 3 --iters 200"),
    ],
    "bin_ab_tests": [
        ("pytest_pcg1", 600, f"{PYTEST} tests/test_gpu_pcg1.py tests/test_gpu_solver.py tests/test_gpu_launch_path.py"),
        ("fp64", 600, "python -u bench/ab_env.py --pkg old=bench/ab/pmx_base --shape 16384x16384 "
                      "--shape 2048x16384 --cfg old@old: --cfg new: --rounds 4 --iters 300"),
        ("fp32", 600, "python -u bench/ab_env.py --pkg old=bench/ab/pmx_base --shape 16384x16384 "
                      "--shape 32768x32768 --dtype fp32 --cfg old@old: --cfg new: --rounds 3 --iters 200"),
    ],
    "bin_ab": [
        ("fp64", 600, "python -u bench/ab_env.py --pkg old=bench/ab/pmx_base --shape 16384x16384 "
                      "--shape 2048x16384 --cfg old@old: --cfg new: --rounds 4 --iters 300"),
        ("fp32", 600, "python -u bench/ab_env.py --pkg old=bench/ab/pmx_base --shape 16384x16384 "
                      "--shape 32768x32768 --dtype fp32 --cfg old@old: --cfg new: --rounds 3 --iters 200"),
    ],
    # standalone bench records (BASELINE configs 2/5 and the headline)
    "records": [
        ("bench_default", 300, bench("--gpus 1 --steps 20 --warmup 5")),
        ("fp32_16384", 300, bench("--gpus 1 --dtype fp32 --steps 200 --warmup 20")),
        ("fp32_32768", 500, bench("--gpus 1 --dtype fp32 --M 32768 --N 32768 --steps 100 --warmup 10")),
        ("fp64_4096", 200, bench("--gpus 1 --M 4096 --N 4096 --steps 200 --warmup 20")),
    ],
    "profile_default": [
        ("rocprof_bench", 300, f"{ROCPROF} -d gpurun_out/profile_default/rp -o run -- "
                               + bench("--gpus 1 --steps 60 --warmup 10 --no-tol-solve")),
    ],
}


PMC_PASSES = {
    "ea_rd": "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum",
    "ea_wr": "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum",
    "sq1": "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES "
           "SQ_WAIT_INST_ANY",
    "sq2": "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY "
           "SQ_INST_LEVEL_VMEM SQ_IFETCH SQ_INSTS_VALU_FMA_F64",
    "lat": "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT",
    "icache": "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE",
    "sq3": "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY "
           "SQ_IFETCH",
}


def pmc_study(study: str, configs: dict[str, str], args: str, passes=("ea_rd", "ea_wr")):
    """One rocprofv3 counter pass per (config, pass), kernel counters only, each under its own
    SIGKILL limit; then bench/pmc_summary.py over the study directory."""
    steps = []
    for tag, env in configs.items():
        for p in passes:
            pre = f"env PMX_STUDY=1 {env} "  # the library applies PMX_* knobs only in study mode
            steps.append((f"{tag}_{p}", 100, f"{pre}timeout -s KILL 90 rocprofv3 --pmc {PMC_PASSES[p]} "
                                              f"--output-format csv -d gpurun_out/{study}/{tag}_{p} -o run -- "
                                              f"python3 bench.py {args}"))
    steps.append(("summary", 60, f"python3 bench/pmc_summary.py gpurun_out/{study}"))
    return steps


PMC_ARGS = "--steps 6 --warmup 1 --graph-batch 0 --no-tol-solve"


# ---- parametrised studies: `python bench/gpurun.py <study> -- <study arguments>` ----
def _ab(argv):
    """interleaved same-box A/B of environment knobs: the arguments go to bench/ab_env.py"""
    return [("ab", 1000, "python -u bench/ab_env.py " + " ".join(shlex.quote(a) for a in argv))]


def _pmc(argv):
    """counter passes per configuration: tag:ENV=V,ENV=V ... [--args 'bench.py args'] [--passes a,b]"""
    ap = argparse.ArgumentParser(prog="pmc")
    ap.add_argument("cfg", nargs="+")
    ap.add_argument("--args", default=PMC_ARGS)
    ap.add_argument("--passes", default="ea_rd,ea_wr")
    a = ap.parse_args(argv)
    cfgs = {c.split(":", 1)[0]: " ".join(c.split(":", 1)[1].split(",")) if ":" in c else "" for c in a.cfg}
    return pmc_study("pmc", cfgs, a.args, tuple(a.passes.split(",")))


def _timeline(argv):
    """kernel durations and gaps per iteration: rocprofv3 --kernel-trace of the pmx CLI per grid
    (MxN ...), then bench/trace_timeline.py; extra pmx arguments after --pmx.  --case TAG 'M N args'
    (repeatable) adds runs with their own pmx arguments; --ranks P passes P subdomains to every run
    (LocalComm on the one GPU) and per-subdomain sweep times to the summary."""
    ap = argparse.ArgumentParser(prog="timeline")
    ap.add_argument("grids", nargs="*")
    ap.add_argument("--iters", type=int, default=600)
    ap.add_argument("--pmx", default="")
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--case", nargs=2, action="append", default=[], metavar=("TAG", "ARGS"))
    a = ap.parse_args(argv)
    cases = [(g, " ".join(g.split("x")) + " " + a.pmx) for g in a.grids] + [tuple(c) for c in a.case]
    rk = f" --ranks {a.ranks}" if a.ranks > 1 else ""
    steps = []
    for tag, args in cases:
        steps.append((f"trace_{tag}", 150, f"rocprofv3 --kernel-trace --output-format csv -d gpurun_out/timeline/{tag} "
                                           f"-o run -- poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx {args} "
                                           f"--max-iter {a.iters} --json{rk}"))
        steps.append((f"timeline_{tag}", 60, f"python3 bench/trace_timeline.py gpurun_out/timeline/{tag}/run_kernel_trace.csv "
                                             f"--skip 50{rk}"))
    return steps


def _validate(argv):
    """the round-end tiers: GPU suite, smoke(), default bench (+ optional extra bench.py args)"""
    keep = "--keep-going" in argv  # every failure of the suite, not only the first
    extra = " ".join(a for a in argv if a != "--keep-going")
    py = PYTEST.replace(" -x ", " ") if keep else PYTEST
    return [("pytest_gpu", 1100, f"{py} tests -m gpu"),
            ("smoke", 200, "python -c 'import __graft_entry__ as g; g.smoke()'"),
            ("bench_default", 300, bench(f"--gpus 1 --steps 20 --warmup 5 {extra}"))]


def _share(argv):
    """multi-rank rehearsal on the one GPU under the supervisor: ranks ... [-- bench.py args]"""
    lead = 0  # rank counts are the leading integers; everything after goes to bench.py
    while lead < len(argv) and argv[lead].isdigit():
        lead += 1
    ranks = [int(x) for x in argv[:lead]] or [2, 4, 8]
    extra = " ".join(argv[lead:])
    return [(f"share{n}", 420, bench(f"--gpus {n} --share-gpu --steps 20 --warmup 5 {extra}")) for n in ranks]


def _cli(argv):
    """pmx CLI runs, one step per quoted argument string: 'M N --flags' ..."""
    return [(f"pmx{i}", 600, f"poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx {a} --json") for i, a in enumerate(argv)]


def _loopback(argv):
    """one rank of an N-GPU job alone on the GPU (bench.py --loopback-rank): per-rank iteration time of
    the real schedule.  Arguments: GPUS:RANK[:ENV=V,ENV=V] ... [-- bench.py args]"""
    cut = argv.index("--") if "--" in argv else len(argv)
    extra = " ".join(argv[cut + 1:]) or "--steps 60 --warmup 6"
    steps = []
    for spec in argv[:cut]:
        parts = spec.split(":")
        g, r = parts[0], parts[1]
        env = " ".join(parts[2].split(",")) if len(parts) > 2 else ""
        pre = f"env PMX_STUDY=1 {env} " if env else ""
        tag = f"g{g}r{r}" + ("_" + parts[2].replace("=", "").replace(",", "_").replace("PMX_", "") if env else "")
        steps.append((tag, 150, pre + bench(f"--gpus {g} --loopback-rank {r} {extra}")))
    return steps


def _ca_ab(argv):
    """same-process A/B of s-step knobs: the arguments go to bench/probe/ca_env_ab.py"""
    return [("ca_ab", 1000, "python -u bench/probe/ca_env_ab.py " + " ".join(shlex.quote(a) for a in argv))]


def _algos(argv):
    """bench.py per grid x algorithm x dtype: MxN:algo:dtype ... [-- bench.py args]"""
    cut = argv.index("--") if "--" in argv else len(argv)
    extra = " ".join(argv[cut + 1:]) or "--steps 20 --warmup 5"
    steps = []
    for spec in argv[:cut]:
        g, algo, dt = spec.split(":")
        m, n = g.split("x")
        steps.append((f"{g}_{algo}_{dt}", 300, bench(f"--gpus 1 --M {m} --N {n} --algo {algo} --dtype {dt} {extra}")))
    return steps


def _counters(argv):
    """kernel trace + SQ instruction / wait mix + EA traffic of one bench.py configuration:
    [--args 'bench.py args'] [--env ENV=V,...]; summary by bench/pmc_summary.py"""
    ap = argparse.ArgumentParser(prog="counters")
    ap.add_argument("--args", default="--steps 30 --warmup 3 --graph-batch 0 --no-tol-solve")
    ap.add_argument("--env", default="")
    a = ap.parse_args(argv)
    env = " ".join(a.env.split(",")) if a.env else ""
    pre = f"env PMX_STUDY=1 {env} " if env else ""
    steps = [("kt", 200, f"{pre}{ROCPROF} --output-format csv -d gpurun_out/counters/kt -o run -- python3 bench.py {a.args}")]
    return steps + pmc_study("counters", {"c": env}, a.args, ("sq1", "sq2", "ea_rd", "ea_wr"))


def _cmds(argv):
    """ad-hoc steps, one per argument 'tag:seconds:command' (python commands of this repo)"""
    steps = []
    for a in argv:
        tag, lim, cmd = a.split(":", 2)
        steps.append((tag, int(lim), cmd))
    return steps


PARAMETRISED = {"cmds": _cmds, "ab": _ab, "pmc": _pmc, "timeline": _timeline, "validate": _validate, "share": _share, "cli": _cli,
                "loopback": _loopback, "ca_ab": _ca_ab, "algos": _algos, "counters": _counters}


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


# Rounds 3-5: the one-off studies (arith32 ... r4ba, r5a ... r5i) and round 5's bench/runs/*.sh
# scripts were defined here / there; the profile READMEs that cite them name the study, and the
# definitions stay in git history (bench/RETIRED.md).


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("study", choices=sorted(STUDIES) + sorted(PARAMETRISED))
    ap.add_argument("--dry", action="store_true", help="write and print the script, do not run it")
    ap.add_argument("--timeout", type=int, default=0, help="gpurun limit (default: sum of the steps + 120 s)")
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    a = ap.parse_args(argv[:cut])
    rest = argv[cut + 1:]  # arguments of a parametrised study
    steps = PARAMETRISED[a.study](rest) if a.study in PARAMETRISED else STUDIES[a.study]
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
