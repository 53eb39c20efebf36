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
            pre = f"env {env} " if env else ""
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
    extra = " ".join(argv)
    return [("pytest_gpu", 1100, f"{PYTEST} tests -m gpu"),
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


# round 3: fp32 stencil arithmetic on fp32 storage (PMX_ARITH32) against the fp64-register sweep,
# and the per-rank cost of the reference 2x4 blocks vs row strips (LocalComm, 8 subdomains)
STUDIES["arith32"] = [
    ("ab", 900, "python -u bench/ab_env.py --dtype fp32 --shape 16384x16384 --shape 32768x32768 "
                "--cfg f64arith: --cfg f32arith:PMX_ARITH32=1 --rounds 3 --iters 100 --tol"),
    ("bench_800", 200, "env PMX_ARITH32=1 " + bench("--gpus 1 --M 800 --N 1200 --dtype fp32 --steps 20 --warmup 5")),
    ("bench_16k", 300, "env PMX_ARITH32=1 " + bench("--gpus 1 --dtype fp32 --steps 20 --warmup 5")),
]
# fp32 arithmetic: tile height, prefetch depth, and a 5-waves/SIMD plain sweep (package copy
# bench/ab/w5 built with PMX_EXTRA_HIP_FLAGS=-DPMX_PCG1_F32_WAVES=5)
STUDIES["f32tune"] = [
    ("ab", 1100, "python -u bench/ab_env.py --dtype fp32 --shape 16384x16384 --shape 32768x32768 --pkg w5=bench/ab/w5 "
                 "--cfg base:PMX_ARITH32=1 --cfg w5@w5:PMX_ARITH32=1 --cfg r32:PMX_ARITH32=1,PMX_PCG1_ROWS=32 "
                 "--cfg r48:PMX_ARITH32=1,PMX_PCG1_ROWS=48 --cfg r16:PMX_ARITH32=1,PMX_PCG1_ROWS=16 "
                 "--cfg pf3:PMX_ARITH32=1,PMX_PCG1_PF=3 --cfg pf1:PMX_ARITH32=1,PMX_PCG1_PF=1 --rounds 3 --iters 60"),
]
# allocation placement: subdomains 5-7 of an 8-way LocalComm run sweep ~8-10% faster than 0-4
STUDIES["placement"] = [
    ("multi", 300, "python -u bench/probe/placement.py --multi 6"),
    ("hold", 600, "python -u bench/probe/placement.py --hold 0 --hold 16 --hold 48 --hold 120 --rounds 2"),
    ("pytest_f32", 300, f"{PYTEST} tests/test_gpu_pcg1.py -k 'fp32' tests/test_gpu_cli.py"),
]
STUDIES["alloc"] = [
    ("multi8", 400, "env PMX_DEBUG_ALLOC=1 python -u bench/probe/placement.py --multi 8"),
]
# placement probe (GpuSubdomainSolver::place_fields): off vs the default 4 candidates, fresh processes
STUDIES["place"] = [
    ("probe_ab", 600, "python -u bench/probe/placement.py --rounds 3 --cfg off:PMX_PLACEMENT=1 --cfg k4: "
                      "--cfg k2:PMX_PLACEMENT=2"),
    ("bench_default", 300, bench("--gpus 1 --steps 20 --warmup 5")),
    ("bench_fp32_16k", 300, bench("--gpus 1 --dtype fp32 --steps 20 --warmup 5")),
    ("bench_fp32_32k", 400, bench("--gpus 1 --M 32768 --N 32768 --dtype fp32 --steps 20 --warmup 5")),
]
STUDIES["hiphold"] = [
    ("hold", 900, "env PMX_PLACEMENT=1 PLACEMENT_HOLD_API=hip python -u bench/probe/placement.py --rounds 1 "
                  "--hold 0 --hold 12 --hold 24 --hold 48 --hold 96"),
    ("hold32k", 900, "env PMX_PLACEMENT=1 PLACEMENT_HOLD_API=hip python -u bench/probe/placement.py --rounds 1 "
                     "--M 32768 --N 32768 --dtype fp32 --iters 30 --hold 0 --hold 24 --hold 48 --hold 96"),
]
STUDIES["place2"] = [
    ("probe32k", 900, "python -u bench/probe/placement.py --rounds 3 --M 32768 --N 32768 --dtype fp32 --iters 30 "
                      "--cfg off:PMX_PLACEMENT=1 --cfg k5:"),
    ("probe16k", 600, "python -u bench/probe/placement.py --rounds 3 --cfg off:PMX_PLACEMENT=1 --cfg k5:"),
]
# BASELINE config 4's 2D blocks on the bench path: 8 supervised ranks sharing the GPU, reference 2x4
STUDIES["share_ref"] = [
    ("pytest_new", 300, f"{PYTEST} tests/test_gpu_pcg1.py -k 'placement or fp32'"),
    ("share8_ref", 420, bench("--gpus 8 --share-gpu --M 4096 --N 4096 --split reference --steps 20 --warmup 5")),
    ("share8_ref16k", 420, bench("--gpus 8 --share-gpu --split reference --steps 20 --warmup 5 --no-tol-solve")),
]
# binary A/B of the working tree against bench/ab/base (a build of the last commit)
STUDIES["bin_ab2"] = [
    ("fp64", 600, "python -u bench/ab_env.py --pkg base=bench/ab/base --shape 16384x16384 --shape 2048x16384 "
                  "--cfg old@base: --cfg new: --rounds 3 --iters 100"),
    ("fp32", 600, "python -u bench/ab_env.py --dtype fp32 --pkg base=bench/ab/base --shape 16384x16384 "
                  "--shape 32768x32768 --cfg old@base: --cfg new: --rounds 3 --iters 60"),
]
# round 3, after the SGPR-base addressing: fp64 tile height / prefetch, fp32 w sweep at 3 waves
STUDIES["tune3"] = [
    ("fp64", 800, "python -u bench/ab_env.py --shape 16384x16384 --shape 2048x16384 --cfg base: "
                  "--cfg pf2:PMX_PCG1_PF=2,PMX_PCG1_PF_W=1 --cfg r6:PMX_PCG1_ROWS=6 --cfg r10:PMX_PCG1_ROWS=10 "
                  "--cfg r12:PMX_PCG1_ROWS=12 --rounds 3 --iters 100"),
    ("fp32", 600, "python -u bench/ab_env.py --dtype fp32 --pkg w3=bench/ab/w3 --shape 16384x16384 "
                  "--shape 32768x32768 --cfg new: --cfg w3@w3: --rounds 3 --iters 60"),
]
STUDIES["fresh_ab"] = [
    ("fp64", 1000, "python -u bench/ab_env.py --fresh --pkg base=bench/ab/base --shape 16384x16384 --shape 2048x16384 "
                   "--cfg old@base: --cfg new: --cfg r10:PMX_PCG1_ROWS=10 --cfg r12:PMX_PCG1_ROWS=12 --rounds 3 --iters 100"),
]
STUDIES["manyk"] = [
    ("k", 900, "python -u bench/probe/placement.py --rounds 2 --cfg k5: --cfg k12:PMX_PLACEMENT=12 "
               "--cfg k20:PMX_PLACEMENT=20"),
]
STUDIES["records3"] = [
    ("fp32_16k", 300, bench("--gpus 1 --dtype fp32 --steps 20 --warmup 5")),
    ("fp32_32k", 400, bench("--gpus 1 --M 32768 --N 32768 --dtype fp32 --steps 20 --warmup 5")),
    ("fp64_4096", 200, bench("--gpus 1 --M 4096 --N 4096 --steps 20 --warmup 5")),
    ("strip_2048", 200, bench("--gpus 1 --M 2048 --N 16384 --steps 200 --warmup 20 --no-tol-solve")),
]
STUDIES["ranks3"] = [
    ("strip_8192", 200, bench("--gpus 1 --M 8192 --N 16384 --steps 100 --warmup 20 --no-tol-solve")),
    ("strip_4096", 200, bench("--gpus 1 --M 4096 --N 16384 --steps 200 --warmup 20 --no-tol-solve")),
    ("block_8192x4096", 200, bench("--gpus 1 --M 8192 --N 4096 --steps 200 --warmup 20 --no-tol-solve")),
    ("timeline_2048", 150, "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ranks3/tl2048 -o run -- "
                           "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 2048 16384 --max-iter 600 --json"),
    ("timeline_2048_sum", 60, "python3 bench/trace_timeline.py gpurun_out/ranks3/tl2048/run_kernel_trace.csv --skip 200"),
]
STUDIES["batch4"] = [
    ("ntp", 700, "python -u bench/ab_env.py --fresh --pkg ntp=bench/ab/ntp --shape 16384x16384 --shape 2048x16384 "
                 "--cfg base: --cfg ntp@ntp: --rounds 4 --iters 200"),
    ("fp32_16k", 300, bench("--gpus 1 --dtype fp32 --steps 20 --warmup 5")),
    ("fp32_32k", 400, bench("--gpus 1 --M 32768 --N 32768 --dtype fp32 --steps 20 --warmup 5")),
    ("fp64_32k", 400, bench("--gpus 1 --M 32768 --N 32768 --steps 20 --warmup 5 --tol-time-cap 200")),
]
STUDIES["blocks8"] = [
    ("ab_ref", 600, "python -u bench/ab_env.py --ranks 8 --split reference --shape 16384x16384 --cfg ref: "
                    "--rounds 3 --iters 100"),
    ("ab_rows", 600, "python -u bench/ab_env.py --ranks 8 --split rows --shape 16384x16384 --cfg rows: "
                     "--rounds 3 --iters 100"),
] + _timeline(["--ranks", "8", "--iters", "300", "--case", "ref", "16384 16384 --split reference",
               "--case", "rows", "16384 16384 --split rows"])

# round 4: placement mechanism -- per-candidate TLB and memory-side counters of the probe's sweeps
PLACEMENT_PASSES = {
    "utcl1": "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum "
             "TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum",
    "utcl1b": "TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum "
              "TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum",
    "lat": "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT",
    "ea": "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_sum",
}


def placement_pmc_steps(study: str, k: int = 24) -> list:
    steps = []
    for tag, counters in PLACEMENT_PASSES.items():
        steps.append((tag, 100, f"bash -c 'timeout -s KILL 90 rocprofv3 --pmc {counters} --output-format csv "
                                f"-d gpurun_out/{study}/{tag} -o run -- python3 bench/probe/placement_pmc.py child "
                                f"--k {k} > gpurun_out/{study}/{tag}.json'"))
    steps.append(("summary", 60, f"python3 bench/probe/placement_pmc.py summary gpurun_out/{study}"))
    return steps


# round 4, first contact: the suite (abort guards, serialized comm schedule, reduction stress,
# opt-in placement), smoke, the default bench (bounded probe) against the round-3 probe, a kernel
# profile, and the placement counter passes
STUDIES["r4a"] = [
    ("pytest_gpu", 700, f"{PYTEST} tests -m gpu"),
    ("smoke", 120, "python -c 'import __graft_entry__ as g; g.smoke()'"),
    ("bench_default", 300, bench("--gpus 1 --steps 20 --warmup 5")),
    ("bench_probe_r3", 300, bench("--gpus 1 --steps 20 --warmup 5 --placement 160 --placement-budget 60 "
                                  "--placement-keep-free 0.125 --no-tol-solve")),
    ("bench_noprobe", 300, bench("--gpus 1 --steps 20 --warmup 5 --placement 0 --no-tol-solve")),
] + [
    # per-rank cost of the 8-GPU iteration on one GPU (verdict r3 item 2): the middle strip of 8 and
    # an interior 2x4 block, against the strip with no neighbours
    ("loop_strip3", 200, bench("--gpus 8 --loopback-rank 3 --steps 300 --warmup 30")),
    ("loop_strip3_packed", 200, "env PMX_DIRECT_ROWS=0 " + bench("--gpus 8 --loopback-rank 3 --steps 300 --warmup 30")),
    ("loop_block5", 200, bench("--gpus 8 --loopback-rank 5 --split reference --steps 300 --warmup 30")),
    ("strip_alone", 200, bench("--gpus 1 --M 2048 --N 16384 --steps 300 --warmup 30 --no-tol-solve")),
    ("tl_strip3", 200, "rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4a/tl_strip3 "
                       "-o run -- python3 bench.py --gpus 8 --loopback-rank 3 --steps 300 --warmup 30"),
    ("tl_strip3_sum", 60, "python3 bench/loopback_timeline.py gpurun_out/r4a/tl_strip3"),
    ("tl_block5", 200, "rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4a/tl_block5 "
                       "-o run -- python3 bench.py --gpus 8 --loopback-rank 5 --split reference --steps 300 --warmup 30"),
    ("tl_block5_sum", 60, "python3 bench/loopback_timeline.py gpurun_out/r4a/tl_block5"),
    ("tl_alone", 200, "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4a/tl_alone -o run -- "
                      "python3 bench.py --gpus 1 --M 2048 --N 16384 --steps 300 --warmup 30 --no-tol-solve"),
    ("tl_alone_sum", 60, "python3 bench/loopback_timeline.py gpurun_out/r4a/tl_alone"),
    ("persist_800", 200, bench("--gpus 1 --M 800 --N 1200 --steps 500 --warmup 50")),
    ("persist_1600", 200, bench("--gpus 1 --M 1600 --N 2400 --steps 500 --warmup 50")),
    ("graphs_800", 200, bench("--gpus 1 --M 800 --N 1200 --steps 500 --warmup 50 --persistent off")),
    # verdict r3 item 7, LAST (a host segfault ends the call): the forked-graph shape without pmx code
    ("graph_fork_default", 60, "bench/probe/graph_fork 3 20 4"),
    ("graph_fork_torchrt", 60, TORCH_RT + "bench/probe/graph_fork 3 20 4'"),
    ("graph_fork_hwq1", 60, "env GPU_MAX_HW_QUEUES=1 bench/probe/graph_fork 3 20 4"),
    ("graph_fork_hwq1_torchrt", 60, TORCH_RT + "GPU_MAX_HW_QUEUES=1 bench/probe/graph_fork 3 20 4'"),
]

STUDIES["r4p"] = placement_pmc_steps("r4p")
# round 4, second contact: the full suite after the fixes, the persistent kernel's anatomy (write-
# through stores vs non-temporal + release fence), the loopback strip (Dirichlet ghosts) + timeline
STUDIES["r4c"] = [
    ("pytest_gpu", 800, f"{PYTEST} tests -m gpu"),
    ("persist_trace", 200, "python3 -u bench/probe/persist_trace.py 800x1200 1600x2400 2400x3200"),
    ("persist_trace_nowt", 200, "env PMX_PERSIST_WT=0 python3 -u bench/probe/persist_trace.py 800x1200 1600x2400"),
    ("loop_strip3", 200, bench("--gpus 8 --loopback-rank 3 --steps 300 --warmup 30")),
    ("loop_strip3_packed", 200, "env PMX_DIRECT_ROWS=0 " + bench("--gpus 8 --loopback-rank 3 --steps 300 --warmup 30")),
    ("tl_strip3", 200, "rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4c/tl_strip3 "
                       "-o run -- python3 bench.py --gpus 8 --loopback-rank 3 --steps 300 --warmup 30"),
    ("tl_strip3_sum", 60, "python3 bench/loopback_timeline.py gpurun_out/r4c/tl_strip3"),
]
# round 4, third contact: the suite, the persistent kernel with cut-row carry + LPT schedule, the
# loopback rank with one fill launch per exchange: split sweep vs halo-under-all-reduce, with and
# without transfer / all-reduce stand-in delays; then the placement counter passes
_LB = "--gpus 8 --loopback-rank 3 --steps 300 --warmup 30"
_LB5 = "--gpus 8 --loopback-rank 5 --split reference --steps 300 --warmup 30"
_DELAY = "env PMX_LOOPBACK_AR_US=15 PMX_LOOPBACK_HALO_US=20 "
STUDIES["suite"] = [("pytest_gpu", 1000, f"{PYTEST} tests -m gpu")]
STUDIES["r4d"] = [
    ("persist_trace", 200, "python3 -u bench/probe/persist_trace.py 800x1200 1600x2400 2400x3200"),
    ("lb3_split", 120, bench(_LB)),
    ("lb3_nosplit", 120, "env PMX_PCG1_SPLIT=0 " + bench(_LB)),
    ("lb3_split_d", 120, _DELAY + bench(_LB)),
    ("lb3_nosplit_d", 120, _DELAY + "PMX_PCG1_SPLIT=0 " + bench(_LB)),
    ("lb3_packed_nosplit_d", 120, _DELAY + "PMX_PCG1_SPLIT=0 PMX_DIRECT_ROWS=0 " + bench(_LB)),
    ("lb5_split", 120, bench(_LB5)),
    ("lb5_nosplit", 120, "env PMX_PCG1_SPLIT=0 " + bench(_LB5)),
    ("lb5_nosplit_d", 120, _DELAY + "PMX_PCG1_SPLIT=0 " + bench(_LB5)),
    ("block_alone", 200, bench("--gpus 1 --M 8192 --N 4096 --steps 300 --warmup 30 --no-tol-solve")),
    ("tl_lb3", 200, "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4d/tl_lb3 -o run -- "
                    "python3 bench.py " + _LB),
    ("tl_lb3_sum", 60, "python3 bench/loopback_timeline.py gpurun_out/r4d/tl_lb3"),
] + placement_pmc_steps("r4d")

# the split sweep without the pack join (direct rows), then the suite
STUDIES["r4e"] = [
    ("lb3_split", 120, bench(_LB)),
    ("lb3_split_d", 120, _DELAY + bench(_LB)),
    ("lb5_split", 120, bench(_LB5)),
    ("pytest_gpu", 900, f"{PYTEST} tests -m gpu"),
]

STUDIES["r4f"] = [
    ("pytest_gpu", 600, f"{PYTEST} tests -m gpu"),
    ("persist_pf2", 150, "env PMX_PCG1_PF=2 python3 -u bench/probe/persist_trace.py 800x1200 1600x2400"),
    ("phases_800", 120, bench("--gpus 1 --M 800 --N 1200 --steps 200 --warmup 20 --profile-phases 200")),
    ("phases_1600", 120, bench("--gpus 1 --M 1600 --N 2400 --steps 200 --warmup 20 --profile-phases 200")),
    ("phases_2400", 120, bench("--gpus 1 --M 2400 --N 3200 --steps 200 --warmup 20 --profile-phases 200")),
    ("tl_800", 120, "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4f/tl_800 -o run -- "
                    "python3 bench.py --gpus 1 --M 800 --N 1200 --steps 300 --warmup 30 --persistent off --no-tol-solve"),
    ("tl_800_sum", 60, "python3 bench/loopback_timeline.py gpurun_out/r4f/tl_800"),
]

# instruction supply: k_pcg1 is ~350 KB of code per variant (the I-cache is 64 KB per 2 CUs); is
# the march fetch-bound?  16384^2 and 800x1200 (graph path), counters per dispatch
_SMALL = "--M 800 --N 1200 --steps 30 --warmup 3 --graph-batch 0 --no-tol-solve --persistent off"
STUDIES["r4g"] = (pmc_study("r4g", {"big": ""}, PMC_ARGS + " --placement 0", ("icache", "sq3"))[:-1]
                  + pmc_study("r4g", {"small": ""}, _SMALL, ("icache", "sq3"))[:-1]
                  + [("summary_big", 60, "python3 bench/pmc_summary.py gpurun_out/r4g --n 16384"),
                     ("summary_small", 60, "python3 bench/pmc_summary.py gpurun_out/r4g --n 1000"),
                     ("pytest_gpu", 700, f"{PYTEST} tests -m gpu")])

# latency-bound grids: shorter tiles = more waves and fewer serial row steps per wave
_G8 = "--gpus 1 --M 800 --N 1200 --steps 500 --warmup 50 --no-tol-solve"
_G16 = "--gpus 1 --M 1600 --N 2400 --steps 500 --warmup 50 --no-tol-solve"
STUDIES["r4h"] = [
    ("g800_rows4", 60, bench(_G8 + " --persistent off")),
    ("g800_rows2", 60, "env PMX_PCG1_ROWS=2 PMX_PCG1_ROWS_W=2 " + bench(_G8 + " --persistent off")),
    ("g800_rows1", 60, "env PMX_PCG1_ROWS=1 PMX_PCG1_ROWS_W=1 " + bench(_G8 + " --persistent off")),
    ("p800", 60, bench(_G8)),
    ("p800_rows2", 60, "env PMX_PERSIST_ROWS=2 " + bench(_G8)),
    ("g1600_rows8", 60, bench(_G16 + " --persistent off")),
    ("g1600_rows4", 60, "env PMX_PCG1_ROWS=4 PMX_PCG1_ROWS_W=4 " + bench(_G16 + " --persistent off")),
    ("g1600_rows2", 60, "env PMX_PCG1_ROWS=2 PMX_PCG1_ROWS_W=2 " + bench(_G16 + " --persistent off")),
    ("phases_800", 120, bench("--gpus 1 --M 800 --N 1200 --steps 200 --warmup 20 --profile-phases 200")),
    ("phases_1600", 120, bench("--gpus 1 --M 1600 --N 2400 --steps 200 --warmup 20 --profile-phases 200")),
    ("phases_2400", 120, bench("--gpus 1 --M 2400 --N 3200 --steps 200 --warmup 20 --profile-phases 200")),
    ("pytest_gpu", 700, f"{PYTEST} tests -m gpu"),
]

_G4 = "--gpus 1 --M 400 --N 600 --steps 500 --warmup 50 --no-tol-solve"
_G24 = "--gpus 1 --M 2400 --N 3200 --steps 500 --warmup 50 --no-tol-solve"
STUDIES["r4i"] = [
    ("g400", 60, bench(_G4 + " --persistent off")),
    ("p400", 60, bench(_G4 + " --persistent on")),
    ("g800", 60, bench(_G8 + " --persistent off")),
    ("p800", 60, bench(_G8 + " --persistent on")),
    ("g1600", 60, bench(_G16 + " --persistent off")),
    ("g2400", 60, bench(_G24 + " --persistent off")),
    ("g400_b", 60, bench(_G4 + " --persistent off")),
    ("p400_b", 60, bench(_G4 + " --persistent on")),
    ("g800_b", 60, bench(_G8 + " --persistent off")),
    ("p800_b", 60, bench(_G8 + " --persistent on")),
    ("pytest_gpu", 700, f"{PYTEST} tests -m gpu"),
]

STUDIES["r4j"] = [
    ("ckpt_probe", 120, "python3 -u bench/probe/ckpt_probe.py"),
    ("pytest_gpu", 900, f"{PYTEST} tests -m gpu"),
]

# the per-rank iteration of the 2/4/8-GPU jobs on one box, against the same subdomain with no
# neighbours (same box, same binary): middle ranks, split sweep (the RCCL default), with and
# without the transfer / all-reduce stand-ins
_ALONE = "--gpus 1 --steps 300 --warmup 30 --no-tol-solve --placement 0"
STUDIES["r4k"] = [
    ("alone_8192", 120, bench(_ALONE + " --M 8192 --N 16384")),
    ("lb2_r0", 120, bench("--gpus 2 --loopback-rank 0 --steps 300 --warmup 30 --placement 0")),
    ("lb2_r0_d", 120, _DELAY + bench("--gpus 2 --loopback-rank 0 --steps 300 --warmup 30 --placement 0")),
    ("alone_4096", 120, bench(_ALONE + " --M 4096 --N 16384")),
    ("lb4_r1", 120, bench("--gpus 4 --loopback-rank 1 --steps 300 --warmup 30 --placement 0")),
    ("lb4_r1_d", 120, _DELAY + bench("--gpus 4 --loopback-rank 1 --steps 300 --warmup 30 --placement 0")),
    ("alone_2048", 120, bench(_ALONE + " --M 2048 --N 16384")),
    ("lb8_r3", 120, bench(_LB + " --placement 0")),
    ("lb8_r3_d", 120, _DELAY + bench(_LB + " --placement 0")),
    ("lb8_r3_nosplit", 120, "env PMX_PCG1_SPLIT=0 " + bench(_LB + " --placement 0")),
    ("alone_2048_b", 120, bench(_ALONE + " --M 2048 --N 16384")),
    ("lb8_r3_b", 120, bench(_LB + " --placement 0")),
    ("tl_lb8_r3", 200, "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4k/tl_lb8_r3 -o run -- "
                       "python3 bench.py " + _LB + " --placement 0"),
    ("tl_lb8_r3_sum", 60, "python3 bench/loopback_timeline.py gpurun_out/r4k/tl_lb8_r3"),
    ("tl_alone_2048", 200, "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4k/tl_alone_2048 -o run -- "
                           "python3 bench.py " + _ALONE + " --M 2048 --N 16384"),
    ("tl_alone_2048_sum", 60, "python3 bench/loopback_timeline.py gpurun_out/r4k/tl_alone_2048"),
    ("pytest_gpu", 600, f"{PYTEST} tests -m gpu"),
]

PYTEST_ALL = "python -u -m pytest -v --timeout 170 --timeout-method thread"
STUDIES["r4l"] = [
    ("threaded_failure_alone", 120, f"{PYTEST} tests/test_gpu_solver.py -m gpu -k threaded_failure"),
    ("block_alone", 120, bench(_ALONE + " --M 8192 --N 4096")),
    ("lb5_split", 120, bench(_LB5 + " --placement 0")),
    ("lb5_split_d", 120, _DELAY + bench(_LB5 + " --placement 0")),
    ("lb8_r3", 120, bench(_LB + " --placement 0")),
    ("pytest_gpu_all", 800, f"{PYTEST_ALL} tests -m gpu"),
]

STUDIES["r4m"] = [
    ("fixed", 200, f"{PYTEST} tests/test_gpu_solver.py tests/test_gpu_launch_path.py -m gpu "
                   "-k 'threaded_failure or progress_counters or serialized or comm_sequence'"),
    ("pytest_gpu_all", 800, f"{PYTEST_ALL} tests -m gpu"),
]

# the w sweep: recover p^{k-2} with an extra stencil (default) or re-read it (PMX_PAIR_W=2, +8 B/pt,
# fewer VGPRs); both with the bounded placement probe, fresh processes
STUDIES["r4n"] = [
    ("ab_pairw", 600, "python -u bench/ab_env.py --fresh --shape 16384x16384 --shape 2048x16384 "
                      "--cfg base:PMX_PLACEMENT=12 --cfg rr:PMX_PLACEMENT=12,PMX_PAIR_W=2 --rounds 4 --iters 200"),
    ("smoke", 120, "python -c 'import __graft_entry__ as g; g.smoke()'"),
]

# (r4o / r4q / r4r: historical -- the spacer and prewarm knobs they set were removed after r4r)
# placement: does the sweep rate follow the physical region the allocator reaches?  Candidates
# allocated after a spacer of 0 / 120 / 170 / 220 GB held untouched (PMX_PLACEMENT_SPACER_GB)
_SP = "--gpus 1 --steps 20 --warmup 5 --no-tol-solve --placement 12 --placement-budget 5 --placement-keep-free 0.02"
STUDIES["r4o"] = [(f"sp{g}", 150, f"env PMX_PLACEMENT_SPACER_GB={g} " + bench(_SP)) for g in (0, 120, 170, 220)] + [
    ("sp0_b", 150, "env PMX_PLACEMENT_SPACER_GB=0 " + bench(_SP)),
    ("sp170_b", 150, "env PMX_PLACEMENT_SPACER_GB=170 " + bench(_SP)),
]

# the bench defaults after r4o: 8 candidates past a 100-GB spacer, 0.5 s of timed sweeps, 30% of
# the free memory kept free; fresh driver-command runs + the 2-GPU per-rank block
STUDIES["r4p2"] = [
    ("driver_1", 300, bench("--gpus 1 --steps 20 --warmup 5")),
    ("driver_2", 300, bench("--gpus 1 --steps 20 --warmup 5 --no-tol-solve")),
    ("driver_3", 300, bench("--gpus 1 --steps 20 --warmup 5 --no-tol-solve")),
    ("alone_8192", 120, bench("--gpus 1 --steps 300 --warmup 30 --no-tol-solve --M 8192 --N 16384")),
    ("alone_8192_nosp", 120, bench("--gpus 1 --steps 300 --warmup 30 --no-tol-solve --M 8192 --N 16384 "
                                   "--placement-spacer 0")),
    ("fp32_16k", 200, bench("--gpus 1 --steps 20 --warmup 5 --dtype fp32 --no-tol-solve")),
    ("mixed_32k", 300, bench("--gpus 1 --steps 20 --warmup 5 --dtype mixed --M 32768 --N 32768 --no-tol-solve")),
]

# placement: is "fast" the memory the driver had to clear?  Pre-written scratch (freed before the
# candidates) vs none, each with and without the spacer, repeated
_PW = "--gpus 1 --steps 20 --warmup 5 --no-tol-solve --placement 8"
STUDIES["r4q"] = [
    ("ctrl_1", 150, bench(_PW)),
    ("pw150_1", 150, "env PMX_PLACEMENT_PREWARM_GB=150 " + bench(_PW)),
    ("pw150_nosp_1", 150, "env PMX_PLACEMENT_PREWARM_GB=150 " + bench(_PW + " --placement-spacer 0")),
    ("ctrl_2", 150, bench(_PW)),
    ("pw150_2", 150, "env PMX_PLACEMENT_PREWARM_GB=150 " + bench(_PW)),
    ("pw150_nosp_2", 150, "env PMX_PLACEMENT_PREWARM_GB=150 " + bench(_PW + " --placement-spacer 0")),
    ("pw250_nosp", 150, "env PMX_PLACEMENT_PREWARM_GB=250 " + bench(_PW + " --placement-spacer 0")),
    ("ctrl_3", 150, bench(_PW)),
]

# the probe times 6 real iterations per candidate: does its ranking now predict the bench rate?
STUDIES["r4r"] = [
    ("sp_1", 150, bench(_PW)),
    ("nosp_1", 150, bench(_PW + " --placement-spacer 0")),
    ("sp_2", 150, bench(_PW)),
    ("nosp_2", 150, bench(_PW + " --placement-spacer 0")),
    ("sp_3", 150, bench(_PW)),
    ("nosp_3", 150, bench(_PW + " --placement-spacer 0")),
    ("p16_half", 150, bench(_PW + " --placement 16 --placement-spacer 0 --placement-keep-free 0.5")),
]

# the bench defaults after r4r (12 candidates timed by 6 real iterations, half of the free HBM)
STUDIES["r4s"] = [
    ("driver_1", 300, bench("--gpus 1 --steps 20 --warmup 5")),
    ("driver_2", 200, bench("--gpus 1 --steps 20 --warmup 5 --no-tol-solve")),
    ("driver_3", 200, bench("--gpus 1 --steps 20 --warmup 5 --no-tol-solve")),
    ("pytest_gpu", 700, f"{PYTEST} tests -m gpu"),
]

# (historical: the PMX_PLACEMENT_PERMS knob was removed after r4t -- permutations do not matter)
# placement: does the assignment of the five fields to the block's slots decide the rate?
_PP = "--gpus 1 --steps 20 --warmup 5 --no-tol-solve --placement-budget 5"
STUDIES["r4t"] = [
    ("perm24_k1_a", 150, "env PMX_PLACEMENT_PERMS=24 " + bench(_PP + " --placement 1")),
    ("perm24_k1_b", 150, "env PMX_PLACEMENT_PERMS=24 " + bench(_PP + " --placement 1")),
    ("perm8_k4", 150, "env PMX_PLACEMENT_PERMS=8 " + bench(_PP + " --placement 4")),
    ("perm24_k1_c", 150, "env PMX_PLACEMENT_PERMS=24 " + bench(_PP + " --placement 1")),
]

# after stripping the persistent variants: its tests + trace, then the suite
STUDIES["r4u"] = [
    ("persist_tests", 200, f"{PYTEST} tests/test_gpu_persist.py -m gpu"),
    ("persist_trace", 120, "python3 -u bench/probe/persist_trace.py 400x600 800x1200"),
    ("pytest_gpu", 700, f"{PYTEST} tests -m gpu"),
]

# block tiles for the latency-bound grids: correctness first, then the rate against the march
_B8 = "--gpus 1 --M 800 --N 1200 --steps 500 --warmup 50 --no-tol-solve --persistent off"
_B16 = "--gpus 1 --M 1600 --N 2400 --steps 500 --warmup 50 --no-tol-solve --persistent off"
_B24 = "--gpus 1 --M 2400 --N 3200 --steps 500 --warmup 50 --no-tol-solve --persistent off"
_BON = "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS="
STUDIES["r4v"] = [
    ("block_tests", 300, f"{PYTEST} tests/test_gpu_block.py -m gpu"),
] + [(f"{g}_{tag}", 60, (f"{_BON}{tag[1:]} " if tag != "m" else "") + bench(a))
     for g, a in (("g800", _B8), ("g1600", _B16), ("g2400", _B24)) for tag in ("m", "b4", "b8")]

_VAR = {"m": "", "b8w8": "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=8 PMX_PCG1_BLOCK_WAVES=8 ",
        "b8w16": "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=8 PMX_PCG1_BLOCK_WAVES=16 ",
        "b16w8": "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=16 PMX_PCG1_BLOCK_WAVES=8 ",
        "b16w16": "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=16 PMX_PCG1_BLOCK_WAVES=16 "}
STUDIES["r4w"] = [
    ("block_tests", 300, f"{PYTEST} tests/test_gpu_block.py -m gpu"),
] + [(f"{g}_{tag}", 60, pre + bench(a)) for g, a in (("g800", _B8), ("g1600", _B16), ("g2400", _B24))
     for tag, pre in _VAR.items()]

_G4b = "--gpus 1 --M 400 --N 600 --steps 500 --warmup 50 --no-tol-solve"
STUDIES["r4x"] = [
    ("g400_pers", 60, bench(_G4b)),
    ("g400_block", 60, bench(_G4b + " --persistent off")),
    ("g400_march", 60, "env PMX_PCG1_BLOCK=0 " + bench(_G4b + " --persistent off")),
    ("g800_block", 60, bench(_B8)),
    ("g800_march", 60, "env PMX_PCG1_BLOCK=0 " + bench(_B8)),
    ("g800_block_unfused", 60, "env PMX_PCG1_BLOCK_FUSED=0 " + bench(_B8)),
    ("g800_tol", 120, bench("--gpus 1 --M 800 --N 1200 --steps 200 --warmup 20")),
    ("pytest_gpu_all", 800, f"{PYTEST_ALL} tests -m gpu"),
]

# block tiles with the cut-first order: shapes x grids against the march
_SH = {"m": "env PMX_PCG1_BLOCK=0 ", "b4": "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=4 ",
       "b8": "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=8 ", "b16": "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=16 "}
STUDIES["r4y"] = [(f"{g}_{tag}", 60, pre + bench(a)) for g, a in
                  (("g400", _G4b + " --persistent off"), ("g800", _B8), ("g1600", _B16), ("g2400", _B24))
                  for tag, pre in _SH.items()] + [
    ("g3200", 60, "env PMX_PCG1_BLOCK=1 " + bench("--gpus 1 --M 3200 --N 4800 --steps 300 --warmup 30 --no-tol-solve")),
    ("g3200_m", 60, "env PMX_PCG1_BLOCK=0 " + bench("--gpus 1 --M 3200 --N 4800 --steps 300 --warmup 30 --no-tol-solve")),
]

# final round-4 validation: suite, smoke, driver bench, the reference grids' full solves
STUDIES["r4z"] = [
    ("pytest_gpu_all", 800, f"{PYTEST_ALL} tests -m gpu"),
    ("smoke", 120, "python -c 'import __graft_entry__ as g; g.smoke()'"),
    ("bench_driver", 300, bench("--gpus 1 --steps 20 --warmup 5")),
    ("ref_800", 60, "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 800 1200 --json"),
    ("ref_1600", 60, "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 1600 2400 --json"),
    ("ref_2400", 60, "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 2400 3200 --json"),
    ("phases_800", 120, bench("--gpus 1 --M 800 --N 1200 --steps 200 --warmup 20 --profile-phases 200")),
]

# block tiles: every global load issued before stage A, column constants only for cut tiles
STUDIES["r4aa"] = [
    ("block_tests", 300, f"{PYTEST} tests/test_gpu_block.py -m gpu"),
    ("g400", 60, bench(_G4b + " --persistent off")),
    ("g800", 60, bench(_B8)),
    ("g800_b", 60, bench(_B8)),
    ("g1600_b16", 60, _SH["b16"] + bench(_B16)),
    ("g1600_b8", 60, _SH["b8"] + bench(_B16)),
    ("g1600_m", 60, bench(_B16)),
]

STUDIES["r4ab"] = [
    ("g800_b12", 60, "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=12 " + bench(_B8)),
    ("g800_b8", 60, bench(_B8)),
    ("g1600_b12", 60, "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=12 " + bench(_B16)),
    ("g1600_b16", 60, _SH["b16"] + bench(_B16)),
    ("g1600_m", 60, bench(_B16)),
    ("g1200", 60, bench("--gpus 1 --M 1200 --N 1800 --steps 500 --warmup 50 --no-tol-solve")),
    ("g1200_m", 60, "env PMX_PCG1_BLOCK=0 " + bench("--gpus 1 --M 1200 --N 1800 --steps 500 --warmup 50 --no-tol-solve")),
    ("g1200_b", 60, "env PMX_PCG1_BLOCK=1 " + bench("--gpus 1 --M 1200 --N 1800 --steps 500 --warmup 50 --no-tol-solve")),
]

_B12 = "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=12 "
STUDIES["r4ac"] = [
    ("g400_b12", 60, _B12 + bench(_G4b + " --persistent off")),
    ("g400_b8", 60, _SH["b8"] + bench(_G4b + " --persistent off")),
    ("g1200_b12", 60, _B12 + bench("--gpus 1 --M 1200 --N 1800 --steps 500 --warmup 50 --no-tol-solve")),
    ("g1600_b12", 60, _B12 + bench(_B16)),
    ("g1600_m", 60, "env PMX_PCG1_BLOCK=0 " + bench(_B16)),
    ("g2000_b12", 60, _B12 + bench("--gpus 1 --M 2000 --N 3000 --steps 500 --warmup 50 --no-tol-solve")),
    ("g2000_m", 60, "env PMX_PCG1_BLOCK=0 " + bench("--gpus 1 --M 2000 --N 3000 --steps 500 --warmup 50 --no-tol-solve")),
    ("g2400_b12", 60, _B12 + bench(_B24)),
    ("g2400_m", 60, "env PMX_PCG1_BLOCK=0 " + bench(_B24)),
    ("g800_b12", 60, _B12 + bench(_B8)),
]

STUDIES["r4ad"] = [
    ("block_tests", 300, f"{PYTEST} tests/test_gpu_block.py -m gpu"),
    ("ref_800", 60, "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 800 1200 --json"),
    ("ref_1600", 60, "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 1600 2400 --json"),
    ("ref_2400", 60, "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 2400 3200 --json"),
    ("phases_800", 120, bench("--gpus 1 --M 800 --N 1200 --steps 200 --warmup 20 --profile-phases 200")),
    ("phases_1600", 120, bench("--gpus 1 --M 1600 --N 2400 --steps 200 --warmup 20 --profile-phases 200")),
    ("phases_2400", 120, bench("--gpus 1 --M 2400 --N 3200 --steps 200 --warmup 20 --profile-phases 200")),
    ("pytest_gpu_all", 800, f"{PYTEST_ALL} tests -m gpu"),
]

STUDIES["r4ae"] = [
    ("phases_800", 120, bench("--gpus 1 --M 800 --N 1200 --steps 200 --warmup 20 --profile-phases 200")),
    ("phases_1600", 120, bench("--gpus 1 --M 1600 --N 2400 --steps 200 --warmup 20 --profile-phases 200")),
    ("cli_tests", 300, f"{PYTEST} tests/test_gpu_cli.py tests/test_gpu_block.py -m gpu"),
]

# kernel statistics of the default path on the reference grids (block tiles) and at 16384^2
STUDIES["r4af"] = [
    ("stats_800", 120, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4af/stats_800 -o run -- "
                       "python3 bench.py --gpus 1 --M 800 --N 1200 --steps 500 --warmup 50 --no-tol-solve"),
    ("stats_1600", 120, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4af/stats_1600 -o run -- "
                        "python3 bench.py --gpus 1 --M 1600 --N 2400 --steps 500 --warmup 50 --no-tol-solve"),
    ("tl_800_sum", 60, "python3 bench/loopback_timeline.py gpurun_out/r4af/stats_800"),
    ("pmc_800_sq", 100, "timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS "
                        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM --output-format csv "
                        "-d gpurun_out/r4af/pmc_800_sq -o run -- python3 bench.py --gpus 1 --M 800 --N 1200 "
                        "--steps 30 --warmup 3 --graph-batch 0 --no-tol-solve"),
    ("pmc_800_sum", 60, "python3 bench/pmc_summary.py gpurun_out/r4af --n 1000 --kernel k_pcg1_block"),
]

STUDIES["r4ag"] = [
    ("block_tests", 300, f"{PYTEST} tests/test_gpu_block.py -m gpu"),
    ("g400", 60, bench(_G4b + " --persistent off")),
    ("g800", 60, bench(_B8)),
    ("g1200", 60, bench("--gpus 1 --M 1200 --N 1800 --steps 500 --warmup 50 --no-tol-solve")),
    ("g1600", 60, bench(_B16)),
    ("g2000_b12", 60, _B12 + bench("--gpus 1 --M 2000 --N 3000 --steps 500 --warmup 50 --no-tol-solve")),
    ("g2000_m", 60, "env PMX_PCG1_BLOCK=0 " + bench("--gpus 1 --M 2000 --N 3000 --steps 500 --warmup 50 --no-tol-solve")),
    ("stats_1600", 120, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ag/stats_1600 -o run -- "
                        "python3 bench.py --gpus 1 --M 1600 --N 2400 --steps 500 --warmup 50 --no-tol-solve"),
]

STUDIES["r4ah"] = [
    ("stats_1600_m", 120, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ah/stats_1600_m -o run -- "
                          "python3 bench.py --gpus 1 --M 1600 --N 2400 --steps 500 --warmup 50 --no-tol-solve --block-tiles off"),
    ("stats_1200_m", 120, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ah/stats_1200_m -o run -- "
                          "python3 bench.py --gpus 1 --M 1200 --N 1800 --steps 500 --warmup 50 --no-tol-solve --block-tiles off"),
    ("stats_800_m", 120, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ah/stats_800_m -o run -- "
                         "python3 bench.py --gpus 1 --M 800 --N 1200 --steps 500 --warmup 50 --no-tol-solve --block-tiles off"),
]

STUDIES["r4ai"] = [
    ("pytest_gpu_all", 800, f"{PYTEST_ALL} tests -m gpu"),
    ("smoke", 120, "python -c 'import __graft_entry__ as g; g.smoke()'"),
    ("bench_driver", 300, bench("--gpus 1 --steps 20 --warmup 5")),
    ("loopback8", 120, bench(_LB + " --placement 0")),
]

# cross-stream events with a device-scope fence (PMX_EVENT_FENCE) on the loopback rank's split sweep
_F = lambda f: f"env PMX_EVENT_FENCE={f} "  # noqa: E731
STUDIES["r4aj"] = [
    ("lb8_f0", 120, _F(0) + bench(_LB + " --placement 0")),
    ("lb8_f1", 120, _F(1) + bench(_LB + " --placement 0")),
    ("lb8_f2", 120, _F(2) + bench(_LB + " --placement 0")),
    ("lb8_f0b", 120, _F(0) + bench(_LB + " --placement 0")),
    ("lb8_f1b", 120, _F(1) + bench(_LB + " --placement 0")),
    ("lb5_f0", 120, _F(0) + bench(_LB5 + " --placement 0")),
    ("lb5_f1", 120, _F(1) + bench(_LB5 + " --placement 0")),
    ("tests_f1", 400, "env PMX_EVENT_FENCE=1 " + f"{PYTEST} tests/test_gpu_pcg1.py tests/test_gpu_launch_path.py tests/test_gpu_dist.py -m gpu"),
]

# march tile height / prefetch on the 8-GPU strip rank (loopback) and on 1600x2400
_R = lambda r, w=None: f"env PMX_PCG1_ROWS={r} PMX_PCG1_ROWS_W={w or r} "  # noqa: E731
STUDIES["r4ak"] = [
    ("lb8_r4", 120, _R(4) + bench(_LB + " --placement 0")),
    ("lb8_r6", 120, _R(6) + bench(_LB + " --placement 0")),
    ("lb8_r8", 120, _R(8) + bench(_LB + " --placement 0")),
    ("lb8_r12", 120, _R(12) + bench(_LB + " --placement 0")),
    ("lb8_r16", 120, _R(16) + bench(_LB + " --placement 0")),
    ("lb8_r8_12", 120, _R(8, 12) + bench(_LB + " --placement 0")),
    ("lb8_r12_8", 120, _R(12, 8) + bench(_LB + " --placement 0")),
    ("lb8_pf2", 120, "env PMX_PCG1_PF=2 PMX_PCG1_PF_W=2 " + bench(_LB + " --placement 0")),
    ("lb8_r8b", 120, _R(8) + bench(_LB + " --placement 0")),
]

# frame tiles on the comm stream ahead of their exchange (PMX_FRAME_ON_COMM): 2 cross-stream edges
# per iteration instead of 4
_FC = lambda f: f"env PMX_FRAME_ON_COMM={f} "  # noqa: E731
STUDIES["r4al"] = [
    ("lb8_fc0", 120, _FC(0) + bench(_LB + " --placement 0")),
    ("lb8_fc1", 120, _FC(1) + bench(_LB + " --placement 0")),
    ("lb8_fc0b", 120, _FC(0) + bench(_LB + " --placement 0")),
    ("lb8_fc1b", 120, _FC(1) + bench(_LB + " --placement 0")),
    ("lb8_fc0_d", 120, _FC(0) + _DELAY + bench(_LB + " --placement 0")),
    ("lb8_fc1_d", 120, _FC(1) + _DELAY + bench(_LB + " --placement 0")),
    ("lb5_fc0", 120, _FC(0) + bench(_LB5 + " --placement 0")),
    ("lb5_fc1", 120, _FC(1) + bench(_LB5 + " --placement 0")),
    ("lb2_fc0", 120, _FC(0) + bench("--gpus 2 --loopback-rank 0 --steps 300 --warmup 30 --placement 0")),
    ("lb2_fc1", 120, _FC(1) + bench("--gpus 2 --loopback-rank 0 --steps 300 --warmup 30 --placement 0")),
    ("tl_fc1", 120, "env PMX_FRAME_ON_COMM=1 rocprofv3 --kernel-trace --stats --output-format csv "
                    "-d gpurun_out/r4al/tl_fc1 -o run -- python3 bench.py " + _LB + " --placement 0"),
    ("tl_fc1_sum", 60, "python3 bench/loopback_timeline.py gpurun_out/r4al/tl_fc1"),
    ("tests_fc1", 500, "env PMX_FRAME_ON_COMM=1 " + f"{PYTEST} tests/test_gpu_pcg1.py tests/test_gpu_launch_path.py "
                       "tests/test_gpu_dist.py tests/test_gpu_solver.py -m gpu"),
]

# block tiles: two tiles per workgroup (PMX_PCG1_BLOCK_NT=2, both tiles' loads up front, one partial)
_NT = lambda n: f"env PMX_PCG1_BLOCK_NT={n} "  # noqa: E731
_G12 = "--gpus 1 --M 1200 --N 1800 --steps 500 --warmup 50 --no-tol-solve"
_G24 = "--gpus 1 --M 2400 --N 3200 --steps 500 --warmup 50 --no-tol-solve"
STUDIES["r4am"] = [
    ("g1600_nt1", 60, _NT(1) + bench(_B16)),
    ("g1600_nt2", 60, _NT(2) + bench(_B16)),
    ("g800_nt1", 60, _NT(1) + bench(_B8)),
    ("g800_nt2", 60, _NT(2) + bench(_B8)),
    ("g1200_nt1", 60, _NT(1) + bench(_G12)),
    ("g1200_nt2", 60, _NT(2) + bench(_G12)),
    ("g2400_b12_nt2", 60, _NT(2) + _B12 + bench(_G24)),
    ("g2400_m", 60, bench(_G24)),
    ("g1600_nt2_b", 60, _NT(2) + bench(_B16)),
    ("g1600_nt1_b", 60, _NT(1) + bench(_B16)),
    ("ref_800_nt2", 60, _NT(2) + "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 800 1200 --json"),
    ("ref_1600_nt2", 60, _NT(2) + "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 1600 2400 --json"),
    ("block_tests", 300, f"{PYTEST} tests/test_gpu_block.py -m gpu"),
]

# block tiles: dispatch slot read in the state's load batch (one round trip fewer per workgroup)
STUDIES["r4an"] = [
    ("g1600", 60, bench(_B16)),
    ("g800", 60, bench(_B8)),
    ("g1200", 60, bench(_G12)),
    ("g400", 60, bench(_G4b + " --persistent off")),
    ("g1600_b", 60, bench(_B16)),
    ("g800_b", 60, bench(_B8)),
    ("block_tests", 300, f"{PYTEST} tests/test_gpu_block.py -m gpu"),
]

# block tiles: cut tiles' row constants staged in LDS with the tile's loads (no scalar round trip per stage)
STUDIES["r4ao"] = [
    ("g800", 60, bench(_B8)),
    ("g1600", 60, bench(_B16)),
    ("g1200", 60, bench(_G12)),
    ("g400", 60, bench(_G4b + " --persistent off")),
    ("g800_b", 60, bench(_B8)),
    ("g1600_b", 60, bench(_B16)),
    ("g1600_unfused", 60, "env PMX_PCG1_BLOCK_FUSED=0 " + bench(_B16)),
    ("g1200_unfused", 60, "env PMX_PCG1_BLOCK_FUSED=0 " + bench(_G12)),
    ("block_tests", 300, f"{PYTEST} tests/test_gpu_block.py -m gpu"),
]

# block tiles: reduction folded into the sweep (default) vs a separate k_reduce_n, by grid
_UF = "env PMX_PCG1_BLOCK_FUSED=0 "
STUDIES["r4ap"] = [
    ("g800_f", 60, bench(_B8)),
    ("g800_u", 60, _UF + bench(_B8)),
    ("g400_f", 60, bench(_G4b + " --persistent off")),
    ("g400_u", 60, _UF + bench(_G4b + " --persistent off")),
    ("g1200_f", 60, bench(_G12)),
    ("g1200_u", 60, _UF + bench(_G12)),
    ("g1600_f", 60, bench(_B16)),
    ("g1600_u", 60, _UF + bench(_B16)),
    ("g800_f2", 60, bench(_B8)),
    ("g800_u2", 60, _UF + bench(_B8)),
    ("g2000_u", 60, "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=12 " + _UF +
     bench("--gpus 1 --M 2000 --N 3000 --steps 500 --warmup 50 --no-tol-solve")),
    ("g2000_m", 60, bench("--gpus 1 --M 2000 --N 3000 --steps 500 --warmup 50 --no-tol-solve")),
    ("g2400_u", 60, "env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS=12 " + _UF + bench(_G24)),
    ("g2400_m", 60, bench(_G24)),
]

# the fused/separate reduction rule by tile count; reference grids end to end
STUDIES["r4aq"] = [
    ("block_tests", 300, f"{PYTEST} tests/test_gpu_block.py tests/test_gpu_cli.py -m gpu"),
    ("g1600", 60, bench(_B16)),
    ("g1200", 60, bench(_G12)),
    ("g800", 60, bench(_B8)),
    ("g400", 60, bench(_G4b + " --persistent off")),
    ("ref_800", 60, "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 800 1200 --json"),
    ("ref_1600", 60, "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 1600 2400 --json"),
    ("ref_2400", 60, "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 2400 3200 --json"),
    ("phases_800", 120, bench("--gpus 1 --M 800 --N 1200 --steps 200 --warmup 20 --profile-phases 200")),
    ("phases_1600", 120, bench("--gpus 1 --M 1600 --N 2400 --steps 200 --warmup 20 --profile-phases 200")),
]

# block-tile shapes again, with the separate reduction above 1,500 tiles
_BR = lambda r, w=8: f"env PMX_PCG1_BLOCK=1 PMX_PCG1_BLOCK_ROWS={r} PMX_PCG1_BLOCK_WAVES={w} "  # noqa: E731
STUDIES["r4ar"] = [
    ("g1600_r12", 60, _BR(12) + bench(_B16)),
    ("g1600_r16", 60, _BR(16) + bench(_B16)),
    ("g1600_r16w16", 60, _BR(16, 16) + bench(_B16)),
    ("g1600_r8", 60, _BR(8) + bench(_B16)),
    ("g1200_r16", 60, _BR(16) + bench(_G12)),
    ("g1200_r12", 60, _BR(12) + bench(_G12)),
    ("g2000_r16", 60, _BR(16) + bench("--gpus 1 --M 2000 --N 3000 --steps 500 --warmup 50 --no-tol-solve")),
    ("g2000_r12", 60, _BR(12) + bench("--gpus 1 --M 2000 --N 3000 --steps 500 --warmup 50 --no-tol-solve")),
    ("g2000_m", 60, bench("--gpus 1 --M 2000 --N 3000 --steps 500 --warmup 50 --no-tol-solve")),
    ("g800_r16", 60, _BR(16) + bench(_B8)),
]

# final validation after the frame-on-comm schedule and the block-tile changes
STUDIES["r4as"] = [
    ("pytest_gpu_all", 800, f"{PYTEST_ALL} tests -m gpu"),
    ("smoke", 120, "python -c 'import __graft_entry__ as g; g.smoke()'"),
    ("bench_driver", 300, bench("--gpus 1 --steps 20 --warmup 5")),
    ("loopback8", 120, bench(_LB + " --placement 0")),
]

# one-workgroup reduction for <= 4096 partials (PMX_REDUCE_ONE) vs the ticketed multi-block k_reduce_n
_RO = lambda v: f"env PMX_REDUCE_ONE={v} "  # noqa: E731
STUDIES["r4at"] = [
    ("g1600_1", 60, _RO(1) + bench(_B16)),
    ("g1600_0", 60, _RO(0) + bench(_B16)),
    ("g1200_1", 60, _RO(1) + bench(_G12)),
    ("g1200_0", 60, _RO(0) + bench(_G12)),
    ("g800m_1", 60, _RO(1) + bench(_B8 + " --block-tiles off")),
    ("g800m_0", 60, _RO(0) + bench(_B8 + " --block-tiles off")),
    ("g1600_1b", 60, _RO(1) + bench(_B16)),
    ("g1600_0b", 60, _RO(0) + bench(_B16)),
    ("tests", 400, f"{PYTEST} tests/test_gpu_block.py tests/test_gpu_pcg1.py tests/test_gpu_solver.py -m gpu"),
]

# block tiles: stage B on the rows of the wave's own stage A (r^{k-1}, p^{k-1} from registers, no sRo;
# sPo only on w sweeps)
STUDIES["r4au"] = [
    ("g1600", 60, bench(_B16)),
    ("g800", 60, bench(_B8)),
    ("g1200", 60, bench(_G12)),
    ("g400", 60, bench(_G4b + " --persistent off")),
    ("g1600_b", 60, bench(_B16)),
    ("g800_b", 60, bench(_B8)),
    ("tests", 300, f"{PYTEST} tests/test_gpu_block.py -m gpu"),
]

# final validation of the round's last state (k_reduce_1 added after r4as)
STUDIES["r4av"] = [
    ("pytest_gpu_all", 800, f"{PYTEST_ALL} tests -m gpu"),
    ("smoke", 120, "python -c 'import __graft_entry__ as g; g.smoke()'"),
    ("bench_driver", 300, bench("--gpus 1 --steps 20 --warmup 5")),
    ("loopback8", 120, bench(_LB + " --placement 0")),
    ("g1600", 60, bench(_B16)),
]

# deeper placement probes on a box whose first half of HBM has no fast block
_DRV = "--gpus 1 --steps 20 --warmup 5"
STUDIES["r4aw"] = [
    ("drv_default", 300, bench(_DRV)),
    ("drv_p20_q25", 300, bench(_DRV + " --placement 20 --placement-keep-free 0.25")),
    ("drv_p24_q15", 300, bench(_DRV + " --placement 24 --placement-keep-free 0.15")),
    ("drv_default_b", 300, bench(_DRV)),
    ("drv_p20_q25_b", 300, bench(_DRV + " --placement 20 --placement-keep-free 0.25")),
]

# the driver's commands with the new placement defaults
STUDIES["r4ax"] = [
    ("bench_driver", 300, bench("--gpus 1 --steps 20 --warmup 5")),
    ("bench_noflags", 400, "python bench.py"),
    ("smoke", 120, "python -c 'import __graft_entry__ as g; g.smoke()'"),
]

# kernel statistics of the final default on the reference grids
STUDIES["r4ay"] = [
    ("stats_1600", 120, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ay/stats_1600 -o run -- "
                        "python3 bench.py --gpus 1 --M 1600 --N 2400 --steps 500 --warmup 50 --no-tol-solve"),
    ("stats_800", 120, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ay/stats_800 -o run -- "
                       "python3 bench.py --gpus 1 --M 800 --N 1200 --steps 500 --warmup 50 --no-tol-solve"),
    ("stats_1200", 120, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ay/stats_1200 -o run -- "
                        "python3 bench.py --gpus 1 --M 1200 --N 1800 --steps 500 --warmup 50 --no-tol-solve"),
]

# bench-driving GPU tests after the placement default change
STUDIES["r4az"] = [
    ("bench_tests", 500, f"{PYTEST} tests/test_gpu_launch_path.py tests/test_gpu_dist.py tests/test_gpu_cli.py -m gpu"),
]

# k_reduce_1 with 256 vs 1024 threads
_RT = lambda t: f"env PMX_REDUCE_ONE_THREADS={t} "  # noqa: E731
STUDIES["r4ba"] = [
    ("g1600_1024", 60, _RT(1024) + bench(_B16)),
    ("g1600_256", 60, _RT(256) + bench(_B16)),
    ("g1200_1024", 60, _RT(1024) + bench(_G12)),
    ("g1200_256", 60, _RT(256) + bench(_G12)),
    ("g1600_1024b", 60, _RT(1024) + bench(_B16)),
    ("g1600_256b", 60, _RT(256) + bench(_B16)),
    ("tests_256", 300, _RT(256) + f"{PYTEST} tests/test_gpu_block.py -m gpu"),
]

# round 4: the reference's Table 2 buckets at its own grids (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:956-980),
# BASELINE config 5's per-rank shape in fp32 / mixed (4096x32768 = the 8-rank strip of 32768^2)
STUDIES["r4b"] = [
    ("bench_driver_1", 300, bench("--gpus 1 --steps 20 --warmup 5")),
    ("bench_driver_2", 300, bench("--gpus 1 --steps 20 --warmup 5")),
    ("phases_800", 200, bench("--gpus 1 --M 800 --N 1200 --steps 200 --warmup 20 --profile-phases 200")),
    ("phases_1600", 200, bench("--gpus 1 --M 1600 --N 2400 --steps 200 --warmup 20 --profile-phases 200")),
    ("phases_2400", 200, bench("--gpus 1 --M 2400 --N 3200 --steps 200 --warmup 20 --profile-phases 200")),
    ("strip32k_fp32", 200, bench("--gpus 1 --M 4096 --N 32768 --dtype fp32 --steps 200 --warmup 20 --no-tol-solve")),
    ("strip32k_mixed", 200, bench("--gpus 1 --M 4096 --N 32768 --dtype mixed --steps 200 --warmup 20 --no-tol-solve")),
    ("strip32k_fp64", 200, bench("--gpus 1 --M 4096 --N 32768 --steps 200 --warmup 20 --no-tol-solve")),
    ("plan_device", 60, "poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx 32768 32768 --plan --gpus 8 --split auto"),
]

PARAMETRISED = {"ab": _ab, "pmc": _pmc, "timeline": _timeline, "validate": _validate, "share": _share, "cli": _cli}


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


# round 5: march occupancy / prefetch depth (bench/probe/dma_march.hip showed the access pattern
# runs 9% faster at 8-10 than at 16 waves per CU); the shared-prologue tests
_AB5 = "python -u bench/ab_env.py --fresh --shape 16384x16384 --rounds 2 --iters 200 "
STUDIES["r5a"] = [
    ("probe", 240, "bench/probe/dma_march 16384 3 10"),
    ("tests_block", 400, f"{PYTEST} tests/test_gpu_block.py"),
    ("ab_pf", 900, _AB5 + "--cfg base: --cfg pf2:PMX_PCG1_PF=2,PMX_PCG1_PF_W=1 "
                    "--cfg pf2w12:PMX_PCG1_PF=2,PMX_PCG1_PF_W=1,PMX_PCG1_WPCU=12 "
                    "--cfg pf2w10:PMX_PCG1_PF=2,PMX_PCG1_PF_W=1,PMX_PCG1_WPCU=10 "
                    "--cfg pf3w12:PMX_PCG1_PF=3,PMX_PCG1_PF_W=1,PMX_PCG1_WPCU=12 "
                    "--cfg pf3w10:PMX_PCG1_PF=3,PMX_PCG1_PF_W=1,PMX_PCG1_WPCU=10 "
                    "--cfg wpf2w10:PMX_PCG1_PF_W=2,PMX_PCG1_WPCU_W=10"),
]


STUDIES["r5c"] = [
    ("tests_dma", 600, f"{PYTEST} tests/test_gpu_pcg1.py -k 'dma or goldens'"),
    ("ab_dma", 900, _AB5 + "--cfg base: --cfg d2:PMX_PCG1_DMA=2 --cfg d3:PMX_PCG1_DMA=3 "
                    "--cfg d2w12:PMX_PCG1_DMA=2,PMX_PCG1_WPCU=12,PMX_PCG1_WPCU_W=10 "
                    "--cfg d3w12:PMX_PCG1_DMA=3,PMX_PCG1_WPCU=12,PMX_PCG1_WPCU_W=10 "
                    "--cfg d2w10:PMX_PCG1_DMA=2,PMX_PCG1_WPCU=10,PMX_PCG1_WPCU_W=8 "
                    "--cfg d2p:PMX_PCG1_DMA=2,PMX_PCG1_DMA_W=0"),
]


STUDIES["r5e"] = [
    ("tests_loop", 600, f"{PYTEST} tests/test_gpu_block.py -k 'looping or goldens'"),
    ("ab_loop", 600, "python -u bench/ab_env.py --shape 800x1200 --shape 1200x1800 --shape 1600x2400 "
                     "--shape 2400x3200 --rounds 3 --iters 600 --warmup 50 --cfg base: --cfg b0:PMX_PCG1_BLOCK=1 "
                     "--cfg l1:PMX_PCG1_BLOCK=1,PMX_PCG1_BLOCK_LOOP=1 --cfg l2:PMX_PCG1_BLOCK=1,PMX_PCG1_BLOCK_LOOP=2 "
                     "--cfg l2f:PMX_PCG1_BLOCK=1,PMX_PCG1_BLOCK_LOOP=2,PMX_PCG1_BLOCK_FUSED=1 "
                     "--cfg l3:PMX_PCG1_BLOCK=1,PMX_PCG1_BLOCK_LOOP=3"),
]


STUDIES["r5f"] = [
    ("tests_lock", 600, f"{PYTEST} tests/test_gpu_pcg1.py -k 'lockstep or goldens'"),
    ("ab_lock", 900, _AB5 + "--shape 2048x16384 --cfg base: --cfg w8:PMX_PCG1_WAVES=8 "
                     "--cfg w8w8:PMX_PCG1_WAVES=8,PMX_PCG1_WAVES_W=8 --cfg w4:PMX_PCG1_WAVES=4 "
                     "--cfg w8r4:PMX_PCG1_WAVES=8,PMX_PCG1_ROWS=4 --cfg w8r12:PMX_PCG1_WAVES=8,PMX_PCG1_ROWS=12"),
]


STUDIES["r5g"] = [
    ("ab_lock2", 900, _AB5 + "--cfg base: --cfg w4r12:PMX_PCG1_WAVES=4,PMX_PCG1_ROWS=12 "
                      "--cfg w8r16:PMX_PCG1_WAVES=8,PMX_PCG1_ROWS=16 --cfg w4r16:PMX_PCG1_WAVES=4,PMX_PCG1_ROWS=16 "
                      "--cfg r12:PMX_PCG1_ROWS=12"),
]


STUDIES["r5h"] = [
    ("ab_rows", 1100, "python -u bench/ab_env.py --fresh --shape 16384x16384 --rounds 3 --iters 200 "
                      "--cfg base: --cfg r12:PMX_PCG1_ROWS=12 --cfg w4r12:PMX_PCG1_WAVES=4,PMX_PCG1_ROWS=12 "
                      "--cfg w4r12w1:PMX_PCG1_WAVES=4,PMX_PCG1_ROWS=12,PMX_PCG1_WAVES_W=1 "
                      "--cfg w4r10:PMX_PCG1_WAVES=4,PMX_PCG1_ROWS=10 --cfg w4r14:PMX_PCG1_WAVES=4,PMX_PCG1_ROWS=14 "
                      "--cfg r14:PMX_PCG1_ROWS=14"),
]


STUDIES["r5i"] = [
    ("ab_rows_probe", 1100, "python -u bench/ab_env.py --fresh --shape 16384x16384 --shape 2048x16384 --rounds 2 "
                            "--iters 200 --cfg base:PMX_PLACEMENT=20 --cfg r12:PMX_PLACEMENT=20,PMX_PCG1_ROWS=12 "
                            "--cfg w4r12:PMX_PLACEMENT=20,PMX_PCG1_WAVES=4,PMX_PCG1_ROWS=12 "
                            "--cfg w4r14:PMX_PLACEMENT=20,PMX_PCG1_WAVES=4,PMX_PCG1_ROWS=14"),
    ("bench_w4r12", 300, "env PMX_PCG1_WAVES=4 PMX_PCG1_ROWS=12 " + bench("--gpus 1 --steps 20 --warmup 5")),
    ("bench_base", 300, bench("--gpus 1 --steps 20 --warmup 5")),
]


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
