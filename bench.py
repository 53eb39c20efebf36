#!/usr/bin/env python3
"""Flagship benchmark: fused-HIP PCG throughput on the BASELINE.json headline config.

Metric (BASELINE.json): grid-point updates per second (MLUPS) + iterations-to-tolerance on a
16384^2 grid at 1/2/4/8 MI355X.  One "step" = one full PCG iteration (halo exchange, A p with
(Ap,p), w/r update with ||dw|| and (z,r), the all-reduce, p update) -- nothing skipped.
MLUPS = (M-1)(N-1) * steps / time / 1e6, whole-job aggregate.  The grid is fixed as N grows
(strong scaling).  Synthetic data = the reference problem itself: F = 1 in the ellipse
x^2 + 4y^2 < 1, zero initial guess (there is no dataset).

    python bench.py --gpus 1 --steps 200 --warmup 20
    python bench.py --gpus 8                  # spawns 8 ranks itself (one per GPU)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29500 bench.py --gpus 8 --steps 200 --warmup 20

Multi-GPU runs are supervised (reference lifecycle: stage4-mpi+cuda/poisson_mpi_cuda_f.cu:986-1039).
The process(es) started by the user or by torchrun never touch the GPU: they start the measuring
ranks as child processes and walk a fallback ladder of transports, each rung in fresh processes:
    rung 1  native RCCL, iterations captured in hipGraphs, split sweep, ghost exchange on its own
            communicator and stream, overlapped with the sweep (the production path)
    rung 2  native RCCL, fully serialized: eager launches, ONE communicator, every call on the compute
            stream in a fixed order (all-reduce, then the send/recv group: the reference's own
            ordering, stage4-mpi+cuda/poisson_mpi_cuda_f.cu:851-943) -- no two RCCL kernels are ever
            in flight together, which removes the two-communicator interlock rung 1 could hit
    rung 3  native IPC transport (peer arenas mapped with hipIpcOpenMemHandle, epoch flags; no
            RCCL at all), graphs and split sweep
    rung 4  torch.distributed ProcessGroupNCCL (= RCCL) driving the same native kernels
A --share-gpu rehearsal (every rank on GPU 0) starts at rung 3, then rung 4 over gloo.
Every rank runs under a progress watchdog: each phase (setup, comm-init, canary iteration, first
graph batch, warmup, timed region, tolerance solve) has a deadline (DEADLINES); on expiry the rank
prints the phase and the device's own progress counters (sweeps reduced, ghost exchanges packed /
unpacked) and exits, and the supervisor moves on.  Failures are classified by the phase the failing
rank was in: a rung that fails in comm-init (the RCCL communicator initialisation) skips the other
RCCL rung, whose initialisation is identical.  The whole ladder runs within --ladder-budget seconds
(540: rung caps RUNG_CAP, each hang ends at its phase deadline), so even a rung-1 hang plus a rung-2
hang leave rung 3 its full cap.  The JSON line names the rung that produced it, the transport
(`comm`), `rccl_graph`, `split_sweep`, every attempt with its phase, and whether the timed region
replayed graphs (`timed_path`); if every rung fails it is still printed, with value null and
valid false.  A run whose rank count differs from --gpus fails; it never measures fewer GPUs than it
reports.

After the timed region a full solve to ||w^{k+1}-w^k|| < 1e-6 reports iters-to-tol and the error
of the solution against the analytic u = (1 - x^2 - 4y^2)/10 (l2_error, max_error; disable with
--no-tol-solve).  That stop rule is the reference's absolute one: at fine grids it ends well before
discretisation accuracy (32768^2: L2 error 5.7e-3), exactly as the reference's solver would.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time

BASELINE_MLUPS = 2450.0  # best published reference rate: 2x P100, 2400x3200
METRIC = "grid-point updates/sec (MLUPS) + iters-to-tol, 16384^2 grid at 1/2/4/8 MI355X"
TOL_NOTE = ("stop rule ||w^{k+1}-w^k|| < delta absolute (reference rule); at fine grids the solve ends "
            "before discretisation accuracy")

# fallback ladder (see the module docstring); `split` None = the driver's default for the transport,
# `overlap` None = --overlap
RUNGS = {
    1: dict(comm="native", rccl_graph=True, split=None, overlap=None),
    2: dict(comm="native", rccl_graph=False, split=0, overlap=False),
    3: dict(comm="ipc", rccl_graph=False, split=None, overlap=None),
    4: dict(comm="torch", rccl_graph=False, split=0, overlap=None),
}
# Per-phase watchdog deadlines (seconds, x --deadline-scale); comm-init is set by DistGpuPCG (its RCCL
# / IPC initialisation watchdog + 15 s).  No phase of a healthy 16384^2 run comes close: setup
# (process group, solver, placement probe) takes ~5-20 s, the rest is sub-second per poll.
DEADLINES = {"setup": 120, "comm-init": 105, "canary": 60, "first-batch": 60, "warmup": 60, "timed": 60,
             "tol-solve": 60, "accuracy": 90, "profile": 300, "report": 60, "shutdown": 60}
COMM_INIT_TIMEOUT = 90.0  # DistGpuPCG's own watchdog around the blocking RCCL / IPC initialisation
# Hard per-rung limits of the supervisor (a rung normally ends far earlier: success in ~30-60 s, a
# hang at its phase deadline).  Worst case rung 1 + rung 2 = 360 s of a 540-s ladder budget.
RUNG_CAP = {1: 210.0, 2: 150.0, 3: 240.0, 4: 240.0}
LADDER_BUDGET = 540.0


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--breakdown-tol", type=float, default=1e-15,
                    help="CG guard on (Ap,p) (reference: 1e-15; grids beyond ~100000^2 need a smaller value)")
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32", "mixed"],
                    help="mixed = fp32: fp32 storage, fp64 arithmetic and reductions")
    ap.add_argument("--comm", default="native", choices=["native", "ipc", "torch"],
                    help="first rung of the ladder: native RCCL (rung 1), the IPC transport (rung 3) or "
                         "torch.distributed (rung 4)")
    ap.add_argument("--ladder", default="on", choices=["on", "off"],
                    help="multi-GPU: fall back to the next transport when a rung fails or stalls")
    ap.add_argument("--split", default="auto", choices=["reference", "auto", "rows", "cols"],
                    help="process grid: auto = row strips while every strip keeps >= 128 rows, else the "
                         "least ghost perimeter (16384^2: 2x1, 4x1, 8x1 for 2/4/8 ranks); reference = the "
                         "reference's choose_process_grid (1x2, 2x2, 2x4)")
    ap.add_argument("--kernel", default="wave", choices=["wave"],
                    help="wave: wave-tile kernels with DPP lane shifts (the round-1 lds kernels are retired)")
    ap.add_argument("--block", type=int, default=256, help="unused (the retired lds kernels' tile width)")
    ap.add_argument("--vec", type=int, default=0, help="wave kernels: columns per lane (0 = per-kernel best)")
    ap.add_argument("--vec-b", type=int, default=0, help="pcg_b columns per lane (0 = follow --vec / auto)")
    ap.add_argument("--tile-rows-b", type=int, default=-1, help="pcg_b tile height (-1 = auto)")
    ap.add_argument("--b-kernel", default="rows", choices=["rows", "ring"],
                    help="pcg_b: ring-free 2-row tiles (default) or the software-pipelined ring kernel")
    ap.add_argument("--waves", type=int, default=4, help="wave kernels: wave tiles per workgroup")
    ap.add_argument("--tile-rows", type=int, default=0, help="tile height (0 = auto)")
    ap.add_argument("--algo", default="auto", choices=["auto", "pcg1", "pcg2", "ca"],
                    help="iteration algorithm: auto (the library's choice: the s-step PCG on big fp64 grids and "
                         "row strips where its fields fit, else pcg1 / pcg2), pcg1, pcg2, or ca = the s-step PCG")
    ap.add_argument("--ca-s", type=int, default=3, choices=[2, 3], help="s-step PCG: iterations per block")
    ap.add_argument("--graph-batch", type=int, default=32,
                    help="iterations per captured hipGraph; the timed region replays graphs for any --steps "
                         "(full batches plus one remainder graph, all captured during warmup)")
    ap.add_argument("--overlap", default="on", choices=["on", "off"],
                    help="ghost exchange on a second HIP stream, overlapped with the sweep")
    ap.add_argument("--exact", action="store_true", help="reference arithmetic order in the fused kernels")
    ap.add_argument("--tol-solve", dest="tol_solve", action="store_true", default=True)
    ap.add_argument("--no-tol-solve", dest="tol_solve", action="store_false")
    ap.add_argument("--tol-time-cap", type=float, default=100.0, help="seconds allowed for the tol solve")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="test the launch/ladder/timing/reporting flow on CPU (gloo, plain-PyTorch PCG); "
                         "prints a JSON line marked data=cpu-dry-run, not a measurement")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal: all ranks on GPU 0, native kernels, gloo comm staged through host "
                         "memory (valid=false: not a multi-GPU measurement)")
    ap.add_argument("--rccl-graph", default="on", choices=["on", "off"],
                    help="rung 1: capture the RCCL calls into the hipGraph batches (off: start at rung 2)")
    ap.add_argument("--profile-phases", type=int, default=0,
                    help="after the run: N eager iterations timed per phase, MAX over ranks, printed as "
                         "the reference's stage-4 buckets on stderr and added to the JSON line")
    ap.add_argument("--deadline-scale", type=float, default=1.0,
                    help="multiplies every progress-watchdog deadline")
    ap.add_argument("--rung-timeout", type=float, default=0.0,
                    help="supervisor: hard limit (s) for one rung's processes (0 = RUNG_CAP per rung)")
    ap.add_argument("--ladder-budget", type=float, default=LADDER_BUDGET,
                    help="supervisor: wall-clock budget (s) of the whole ladder")
    ap.add_argument("--placement", type=int, default=20,
                    help="placement probe: candidate field blocks timed, the fastest kept (0 = off; "
                         "bounded by --placement-budget and --placement-keep-free; off when ranks share a GPU). "
                         "20 with 1/4 of HBM kept free: on boxes whose fast blocks lie past the first half of "
                         "HBM, 1.804 vs 1.942 ms/step at 16384^2 (profiles/r4/placement/r4aw_*)")
    ap.add_argument("--block-tiles", default="auto", choices=["auto", "on", "off"],
                    help="block-tile sweeps (pcg1_block.hip): auto = undecomposed fp64 grids with < 10,000 "
                         "four-row march tiles")
    ap.add_argument("--loopback-rank", type=int, default=-1,
                    help="timing rehearsal on ONE GPU (valid=false): rank R of the --gpus-rank decomposition "
                         "alone, ghosts filled by device copies of the real sizes (from zeros), all-reduce "
                         "skipped -- the real per-rank schedule (split sweep, frame stream, copies) at full speed")
    ap.add_argument("--placement-budget", type=float, default=0.5, help="placement probe: seconds of probing")
    ap.add_argument("--placement-keep-free", type=float, default=0.25,
                    help="placement probe: fraction of the free device memory left free")
    return ap.parse_args(argv)


# =============================================================================================
# progress watchdog (every measuring rank)
# =============================================================================================
class Watch:
    """Per-phase deadlines.  A rank stuck in a phase (a collective whose peer never posts, a kernel
    that never finishes) cannot be interrupted from Python; this thread reports where it is and ends
    the process, which is what lets the supervisor move on instead of burning the lease.  The current
    phase is also written to `phase_file` (when given), so the supervisor can classify a failure by
    the phase the rank died in."""

    EXIT_CODE = 87

    def __init__(self, rank: int, scale: float = 1.0, phase_file: str | None = None):
        self.rank, self.scale, self.phase_file = rank, scale, phase_file
        self.name, self.deadline, self.t0 = "start", None, time.monotonic()
        self.progress = None  # callable -> device progress tuple, or None
        self.on_phase = None  # fault-injection hook: called with the phase name after it is entered
        self._lock = threading.Lock()
        threading.Thread(target=self._run, daemon=True, name="pmx-watch").start()

    def phase(self, name: str, seconds: float | None = None):
        seconds = DEADLINES[name] if seconds is None else seconds
        with self._lock:
            self.name, self.t0 = name, time.monotonic()
            self.deadline = self.t0 + seconds * self.scale
        if self.phase_file:
            try:
                with open(self.phase_file + ".tmp", "w") as f:
                    f.write(name)
                os.replace(self.phase_file + ".tmp", self.phase_file)
            except OSError:
                pass
        if self.on_phase:
            self.on_phase(name)

    def _run(self):
        while True:
            time.sleep(0.25)
            with self._lock:
                name, dl, t0 = self.name, self.deadline, self.t0
            if dl is not None and time.monotonic() > dl:
                dev = ""
                try:
                    pr = self.progress() if self.progress else None
                    if pr is not None:
                        dev = (f"; device progress: {pr[0]} sweeps reduced, {pr[1]} ghost exchanges packed, "
                               f"{pr[2]} unpacked")
                except Exception as e:  # the diagnosis must not mask the exit
                    dev = f"; device progress unreadable ({e})"
                print(f"[bench] rank {self.rank}: no progress in phase '{name}' for "
                      f"{time.monotonic() - t0:.0f} s{dev}; aborting this rank", file=sys.stderr, flush=True)
                os._exit(self.EXIT_CODE)


def _fault(rung: int, rank: int):
    """Fault injection for the ladder tests: PMX_BENCH_FAULT='1:hang,2:fail' (optionally '1:hang@0',
    rank 0 only) -> (kind, phase) for this rung/rank: kind in hang|fail|crash, phase "canary"
    (hang), "setup" (fail) or, with the suffix -init ('1:hang-init'), "comm-init"."""
    spec = os.environ.get("PMX_BENCH_FAULT", "")
    for item in filter(None, (x.strip() for x in spec.split(","))):
        r, _, what = item.partition(":")
        what, _, who = what.partition("@")
        if int(r) == rung and (not who or int(who) == rank):
            kind, _, tag = what.partition("-")
            return kind, ("comm-init" if tag == "init" else "canary" if kind == "hang" else "setup")
    return None, None


# =============================================================================================
# supervisor (never touches the GPU): starts the measuring ranks, walks the ladder
# =============================================================================================
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _child_env(rank: int, local_rank: int, world: int, port: int, rung: int, result: str) -> dict:
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(RANK=str(rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PMX_BENCH_ROLE="child", PMX_BENCH_RUNG=str(rung),
               PMX_BENCH_RESULT=result)
    return env


def _spawn(env: dict):
    # children print their diagnostics to our stderr; the only stdout line is the supervisor's
    return subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                            stdout=sys.stderr, start_new_session=True)


def _kill(p, sig=signal.SIGKILL):
    if p.poll() is None:
        try:
            os.killpg(p.pid, sig)
        except ProcessLookupError:
            pass


def _ladder(args) -> list[int]:
    if args.comm == "torch":
        first = 4
    elif args.comm == "ipc" or args.share_gpu:  # RCCL refuses two ranks on one device
        first = 3
    else:
        first = 1 if args.rccl_graph == "on" else 2
    rungs = [r for r in (1, 2, 3, 4) if r >= first]
    return rungs if args.ladder == "on" else rungs[:1]


# phases in the order a rank passes them (the least advanced rank of a failed rung is its cause: the
# others wait for it in a collective and time out in a later phase)
PHASE_ORDER = ("start", "setup", "comm-init", "canary", "first-batch", "warmup", "timed", "tol-solve",
               "accuracy", "profile", "report", "shutdown")


def least_advanced(phases) -> str:
    known = [p for p in phases if p in PHASE_ORDER]
    return min(known, key=PHASE_ORDER.index) if known else (list(phases) or [""])[0]


def _read_phase(result: str, rank: int) -> str:
    try:
        with open(f"{result}.phase.{rank}") as f:
            return f.read().strip() or "start"
    except OSError:
        return "start"  # died before its watchdog wrote anything (interpreter start, imports)


def skipped_after(rung: int, phase: str, remaining: list[int]) -> list[int]:
    """Rungs made pointless by a failure of `rung` in `phase`: an RCCL rung that failed while
    initialising its communicator takes the other RCCL rung with it (identical ncclCommInitRank;
    rung 2 only changes the schedule AFTER initialisation)."""
    if phase == "comm-init" and RUNGS[rung]["comm"] == "native":
        return [r for r in remaining if RUNGS[r]["comm"] == "native"]
    return []


KILL_GRACE = 10.0  # after a failure or the cap: SIGTERM, then SIGKILL this much later


def rung_cap(args, rung: int, budget_left: float) -> float:
    cap = args.rung_timeout if args.rung_timeout > 0 else RUNG_CAP[rung]
    return max(0.0, min(cap, budget_left - KILL_GRACE))


def worst_case_ladder_seconds(args) -> float:
    """Upper bound of the ladder's wall time with rungs 1 and 2 hanging and rung 3 succeeding: each
    rung ends at its cap at the latest, the supervisor adds its 10-s kill grace (deadline scale 1)."""
    ladder = _ladder(args)
    t = 0.0
    for r in ladder[:3]:
        t += rung_cap(args, r, args.ladder_budget - t) + KILL_GRACE
    return t


def _run_rung_local(args, rung: int, result: str, cap: float) -> tuple[bool, str, str]:
    """All ranks are children of this process (no launcher).  -> (ok, reason, phase of the failure)."""
    world = args.gpus
    port = _free_port()
    procs = [_spawn(_child_env(r, r, world, port, rung, result)) for r in range(world)]
    t0, failed_at, reason, phase = time.monotonic(), None, "", ""
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad and failed_at is None:
            failed_at = time.monotonic()
            phase = least_advanced([_read_phase(result, r) for r in range(world)])
            reason = (f"rank {bad[0][0]} exited with status {bad[0][1]} in phase '{_read_phase(result, bad[0][0])}'"
                      f" (least advanced rank: '{phase}')")
            print(f"[bench] rung {rung}: {reason}; stopping the other ranks", file=sys.stderr, flush=True)
            for p in procs:
                _kill(p, signal.SIGTERM)
        if all(c is not None for c in codes):
            break
        if failed_at is not None and time.monotonic() - failed_at > KILL_GRACE:
            for p in procs:
                _kill(p)
        if failed_at is None and time.monotonic() - t0 > cap:
            failed_at = time.monotonic()
            phase = least_advanced([_read_phase(result, r) for r in range(world)])
            reason = f"rung timeout ({cap:.0f} s) in phase '{phase}'"
            print(f"[bench] rung {rung}: {reason}; killing its ranks", file=sys.stderr, flush=True)
            for p in procs:
                _kill(p)
        time.sleep(0.2)
    ok = failed_at is None and all(p.returncode == 0 for p in procs)
    if not ok and not reason:
        reason = f"exit status {[p.returncode for p in procs]}"
    return ok, reason, phase


def _run_rung_torchrun(args, rung: int, result: str, cap: float, store, rank: int,
                       local_rank: int) -> tuple[bool, str, str]:
    """One supervisor per rank (torchrun started them): each runs its own rank's child; the
    supervisors share torchrun's store to agree on a port and to stop early when any rank fails.
    The first failure's reason and phase go through the store, so every supervisor walks the
    ladder identically."""
    import torch
    import torch.distributed as dist

    world = args.gpus
    key = f"pmx/rung{rung}"
    if rank == 0:
        store.set(f"{key}/port", str(_free_port()))
    port = int(store.get(f"{key}/port").decode())
    p = _spawn(_child_env(rank, local_rank, world, port, rung, result))
    t0, mine = time.monotonic(), ""

    def report(reason):
        store.compare_set(f"{key}/fail", "", reason)

    while True:
        c = p.poll()
        if c is not None:
            if c != 0:
                mine = f"rank {rank} exited with status {c} in phase '{_read_phase(result, rank)}'"
                report(mine)
            break
        if store.check([f"{key}/fail"]):
            time.sleep(5)  # let this rank's own watchdog / error path report first
            _kill(p, signal.SIGTERM)
            time.sleep(2)
            _kill(p)
            p.wait()
            break
        if time.monotonic() - t0 > cap:
            mine = f"rank {rank}: rung timeout ({cap:.0f} s) in phase '{_read_phase(result, rank)}'"
            report(mine)
            _kill(p)
            p.wait()
            break
        time.sleep(0.2)
    store.set(f"{key}/phase/{rank}", _read_phase(result, rank))
    bad = torch.tensor([0 if (p.returncode == 0 and not mine) else 1], dtype=torch.int32)
    dist.all_reduce(bad, op=dist.ReduceOp.MAX)  # after it, every rank's phase is in the store
    ok = int(bad.item()) == 0
    if ok:
        return True, "", ""
    phase = least_advanced([store.get(f"{key}/phase/{r}").decode() for r in range(world)])
    reason = store.get(f"{key}/fail").decode() if store.check([f"{key}/fail"]) else mine or "failed"
    return False, f"{reason} (least advanced rank: '{phase}')", phase


def _failed_record(args, attempts) -> dict:
    """The JSON line when every rung failed: no measurement, the ladder's reasons."""
    return {"metric": METRIC, "value": None, "unit": "MLUPS", "n_gpus": args.gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": args.dtype,
            "data": "none: every rung of the transport ladder failed (see ladder)",
            "config": {"model": f"fictitious-domain Poisson ellipse, Jacobi-PCG, {args.M}x{args.N}",
                       "global_batch": 1, "seq_len": (args.M - 1) * (args.N - 1),
                       "parallelism": f"domain{args.gpus}", "split": args.split, "grid": [args.M, args.N],
                       "rung": None},
            "valid": False, "baseline_mlups": BASELINE_MLUPS,
            "error": "every rung of the ladder failed: " + "; ".join(
                f"rung {a['rung']}: {a.get('reason', 'skipped')}" for a in attempts)}


def supervise(args) -> int:
    world = args.gpus
    launched = "WORLD_SIZE" in os.environ
    rank = int(os.environ.get("RANK", 0))
    store = None
    if launched:
        if int(os.environ["WORLD_SIZE"]) != world:
            print(f"[bench] --gpus {world} but {os.environ['WORLD_SIZE']} rank(s) came up (WORLD_SIZE); refusing "
                  "to report a different GPU count", file=sys.stderr, flush=True)
            return 2
        import datetime

        import torch.distributed as dist

        # gloo prints its connection banner on stdout; the supervisor's stdout carries only the JSON
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=60))
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        store = dist.distributed_c10d._get_default_store()
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    tmp = tempfile.mkdtemp(prefix="pmx_bench_")
    attempts, final = [], None
    ladder = _ladder(args)
    skip = set()
    t_ladder = time.monotonic()
    for i, rung in enumerate(ladder):
        if rung in skip:
            attempts.append(dict(rung=rung, **RUNGS[rung], ok=False, skipped=True,
                                 reason="skipped: an earlier rung failed in its identical comm-init"))
            continue
        left = args.ladder_budget - (time.monotonic() - t_ladder)
        cap = rung_cap(args, rung, left)
        if cap < 30.0:
            attempts.append(dict(rung=rung, **RUNGS[rung], ok=False, skipped=True,
                                 reason=f"skipped: ladder budget spent ({left:.0f} s left)"))
            continue
        result = os.path.join(tmp, f"rung{rung}.json")
        t0 = time.monotonic()
        if launched:
            ok, reason, phase = _run_rung_torchrun(args, rung, result, cap, store, rank, local_rank)
        else:
            ok, reason, phase = _run_rung_local(args, rung, result, cap)
        att = dict(rung=rung, **RUNGS[rung], ok=ok, seconds=round(time.monotonic() - t0, 1))
        if not ok:
            att["reason"], att["phase"] = reason, phase
        attempts.append(att)
        if ok:
            if rank == 0:
                with open(result) as f:
                    final = json.loads(f.read().strip().splitlines()[-1])
            break
        skip |= set(skipped_after(rung, phase, ladder[i + 1:]))
        print(f"[bench] rung {rung} ({RUNGS[rung]}) failed: {reason}", file=sys.stderr, flush=True)
    rc = 0
    if rank == 0:
        if final is None:
            print(f"[bench] every rung of the ladder failed: {attempts}", file=sys.stderr, flush=True)
            final = _failed_record(args, attempts)
            rc = 1
        final["ladder"] = attempts
        final["ladder_seconds"] = round(time.monotonic() - t_ladder, 1)
        line = json.dumps(final)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if launched:
        import torch
        import torch.distributed as dist

        t = torch.tensor([rc], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rc = int(t.item())
        dist.destroy_process_group()
    return rc


# =============================================================================================
# measuring rank
# =============================================================================================
def measure(args) -> int:
    import importlib

    import torch
    import torch.distributed as dist

    pkg_name = "poisson-ellipse-openmp-mpi-cuda-new_amd"
    pmx = importlib.import_module(pkg_name)
    launch = importlib.import_module(pkg_name + ".parallel.launch")
    ds = importlib.import_module(pkg_name + ".parallel.dist_solver")
    process_grid = importlib.import_module(pkg_name + ".parallel.decomp").process_grid

    supervised = os.environ.get("PMX_BENCH_ROLE") == "child"
    rung = int(os.environ.get("PMX_BENCH_RUNG", "1"))
    cfg = RUNGS[rung]
    dry = args.cpu_dry_run
    share = args.share_gpu and not dry
    env = launch.env_info()
    result_path = os.environ.get("PMX_BENCH_RESULT")
    watch = Watch(env.rank, args.deadline_scale,
                  phase_file=f"{result_path}.phase.{env.rank}" if supervised and result_path else None)
    fault, fault_phase = _fault(rung, env.rank) if supervised else (None, None)
    if fault == "crash":
        os._exit(3)

    def on_phase(name):  # fault injection at the phase it names
        if fault and name == fault_phase:
            if fault == "hang":
                time.sleep(10 ** 6)  # the watchdog ends this rank
            raise RuntimeError(f"injected failure (PMX_BENCH_FAULT) at rung {rung}, phase {name}")

    watch.on_phase = on_phase
    watch.phase("setup")
    if env.world != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but {env.world} rank(s) came up (WORLD_SIZE); refusing to "
                         "report a different GPU count")
    # Python-level coordination (uid broadcast, agreement, barriers, MAX over ranks) stays on gloo for
    # the native transports: no third (torch) RCCL communicator next to the solver's
    backend = "nccl" if (not dry and not share and cfg["comm"] == "torch") else "gloo"
    info = launch.init_distributed(backend=backend if env.world > 1 else None,
                                   device_type="cpu" if (dry or share or backend == "gloo") else None)
    world = info.world
    device = 0 if share else info.local_rank
    if not dry:
        if not torch.cuda.is_available():
            raise SystemExit("bench.py needs an MI355X (no HIP device visible)")
        if not share and torch.cuda.device_count() < world:
            raise SystemExit(f"[bench] {world} ranks need {world} visible GPUs, found {torch.cuda.device_count()}")
        torch.cuda.set_device(device)
    split_sweep = -1 if cfg["split"] is None else int(cfg["split"])  # pcg1 split sweep of this rung
    overlap = (args.overlap == "on") if cfg["overlap"] is None else cfg["overlap"]
    tdev = "cuda" if info.backend == "nccl" else "cpu"

    def device_sync():
        if not dry:
            torch.cuda.synchronize()

    problem = pmx.PoissonEllipse(M=args.M, N=args.N, breakdown_tol=args.breakdown_tol)
    kw = dict(split=args.split, dtype=args.dtype, kernel=args.kernel, block=args.block, vec=args.vec,
              waves=args.waves, tile_rows=args.tile_rows, exact=args.exact, graph_batch=args.graph_batch,
              overlap=overlap, vec_b=args.vec_b, tile_rows_b=args.tile_rows_b,
              b_ring=args.b_kernel == "ring")
    pkw = dict(placement=0 if share else args.placement, placement_budget_s=args.placement_budget,
               placement_keep_free=args.placement_keep_free)
    dkw = dict(kw, **pkw, phase=watch.phase, init_timeout=COMM_INIT_TIMEOUT, ca_s=args.ca_s,
               split_sweep=split_sweep)
    # --algo auto: the library decides (choose_algo) -- the s-step PCG (ca_kernels.hip) where it applies
    # and wins (the fast arithmetic, >= 6M points, undecomposed, row strips or 2-D blocks -- BASELINE
    # config 4, `--split reference` -- on a native transport: RCCL or IPC, not torch) and its 7 fields
    # fit, else pcg1 / pcg2.  The JSON's config.tile.algo says which ran.
    ca_ok = not args.exact and (world == 1 or cfg["comm"] in ("native", "ipc"))
    if args.algo == "ca" and not ca_ok:
        raise SystemExit("[bench] --algo ca (the s-step PCG) needs the RCCL or IPC transport")
    algo_id = {"auto": -1, "pcg1": 1, "pcg2": 2, "ca": 3}[args.algo]
    if dry:
        tp = importlib.import_module(pkg_name + ".models.torch_pcg")
        comm = importlib.import_module(pkg_name + ".parallel.comm")
        watch.phase("comm-init")
        runner = ds.TorchRunner(tp.TorchPCG(problem, comm=comm.TorchComm() if world > 1 else None,
                                            split=args.split), problem, info)
        comm_used = "gloo" if world > 1 else "self"
    elif world == 1:
        models = importlib.import_module(pkg_name + ".models")

        runner = ds.SessionRunner(models.make_session(problem, ranks=1, device=info.local_rank,
                                                      block_tiles={"auto": -1, "on": 1, "off": 0}[args.block_tiles],
                                                      algo=algo_id, ca_s=args.ca_s, **pkw, **kw), problem, info)
        comm_used = "self"
    elif share and cfg["comm"] == "ipc":
        runner = ds.DistGpuPCG(problem, info, comm="ipc", device=0, algo=algo_id, **dkw)
        comm_used = "ipc"
    elif share:
        runner = ds.DistGpuPCG(problem, info, comm="torch", device=0, **dkw)
        comm_used = "gloo-host-staged"
    elif cfg["comm"] == "ipc":
        runner = ds.DistGpuPCG(problem, info, comm="ipc", algo=algo_id, **dkw)
        comm_used = "ipc"
    elif cfg["comm"] == "native":
        runner = ds.DistGpuPCG(problem, info, comm="native", rccl_graph=cfg["rccl_graph"], algo=algo_id, **dkw)
        comm_used = "rccl"
    else:
        runner = ds.DistGpuPCG(problem, info, comm="torch", **dkw)
        comm_used = "torch-nccl"
    watch.progress = getattr(runner, "progress", None)

    def barrier():
        if world > 1:
            dist.barrier()

    # ---------------- canary: one eager iteration, then the first graph batch ----------------
    watch.phase("canary")
    runner.init()
    it0 = runner.state()["it"]
    runner.step_eager(1)
    runner.synchronize()
    stc = runner.state()
    if stc["it"] != it0 + 1 and not stc["done"]:
        raise RuntimeError(f"canary iteration: device iteration counter {it0} -> {stc['it']}")
    watch.phase("first-batch")
    if getattr(runner, "graphs", False):
        runner.prepare(args.graph_batch)
        runner.step(args.graph_batch)
        runner.synchronize()

    # ---------------- warmup (captures every graph the timed region replays) ----------------
    watch.phase("warmup", DEADLINES["warmup"] + 0.05 * args.warmup)
    runner.init()
    runner.step(args.warmup)
    runner.synchronize()
    prepared = runner.prepare(args.steps) if getattr(runner, "graphs", False) else False
    st0 = runner.state()
    runner.reset_path_stats()

    # ---------------- timed region ----------------
    watch.phase("timed", DEADLINES["timed"] + 0.05 * args.steps)
    barrier()
    device_sync()
    t0 = time.perf_counter()
    runner.step(args.steps)
    runner.synchronize()
    device_sync()
    barrier()
    t1 = time.perf_counter()
    dt = t1 - t0
    st1 = runner.state()
    path = runner.path_stats()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    timed_path = ("graph" if path["eager_iters"] == 0 and path["graph_iters"] > 0 else
                  "eager" if path["graph_iters"] == 0 else "mixed")
    tile_desc = dict(runner.tile())
    probe = tile_desc.pop("placement_probe_ms", None)
    if probe and isinstance(tile_desc.get("placement"), dict) and len(probe) <= 32:
        tile_desc["placement"] = dict(tile_desc["placement"], probe_ms=[round(float(x), 3) for x in probe])
    if isinstance(tile_desc.get("placement"), dict):
        cls = placement_class(tile_desc["placement"].get("kept_ms"), (args.M - 1) * (args.N - 1), args.dtype,
                              tile_desc.get("algo", "pcg1"))
        if cls:
            tile_desc["placement"]["class"] = cls
    valid = (not st1["done"]) and (st1["it"] - st0["it"] == args.steps) and not st1["nan"]
    pts = (args.M - 1) * (args.N - 1)
    mlups = pts * args.steps / dt / 1e6

    # ---------------- iterations to tolerance + accuracy ----------------
    tol = {}
    if args.tol_solve:
        watch.phase("tol-solve")
        runner.init()
        barrier()
        device_sync()
        ts = time.perf_counter()
        launched, batch = 0, max(args.graph_batch, 32)
        max_iter = problem.effective_max_iter()
        capped = False
        while True:
            runner.step(batch)
            launched += batch
            st = runner.state()
            watch.phase("tol-solve")
            stop = 2 if (st["done"] or launched > max_iter + batch) else 0
            if not stop and time.perf_counter() - ts > args.tol_time_cap:
                stop = 1
            if world > 1:  # one decision for all ranks: a rank that stops alone would hang the rest
                flag = torch.tensor([stop], dtype=torch.int32, device=tdev)
                dist.all_reduce(flag, op=dist.ReduceOp.MAX)
                stop = int(flag.item())
            if stop:
                capped = stop == 1
                break
        runner.synchronize()
        barrier()
        tsolve = time.perf_counter() - ts
        watch.phase("accuracy")
        err = runner.error_norms()
        tol = dict(iters_to_tol=int(st["iters"]) if st["done"] else None, tol_status=st["status"],
                   tol_final_diff=st["diff"], tol_solve_seconds=round(tsolve, 4),
                   tol_solve_mlups=round(pts * (st["iters"] if st["done"] else st["it"]) / tsolve / 1e6, 1),
                   tol_time_capped=capped, l2_error=err["l2_error"], max_error=err["max_error"],
                   max_w=err["max_w"], tol_note=TOL_NOTE)

    phases = {}
    if args.profile_phases > 0 and not dry:
        watch.phase("profile")
        ph = runner.profile(args.profile_phases)
        ca = tile_desc.get("algo") == "ca"
        phases = {"phase_seconds_per_iter_max_over_ranks": {k: v / args.profile_phases for k, v in ph.items()},
                  "phase_note": ("compute = the s-step passes (pass 1 / the fused pass: basis + Gram products; "
                                 "pass 2: p, z, w); dot = the block reductions and scalars; comm = the 21-double "
                                 "all-reduce + ghost-row exchange per block" if ca else
                                 "compute = the whole fused sweep (A p, update, D^-1, A z); dot = the device "
                                 "reduction; comm = all-reduce + ghost exchange") +
                                "; copy and precond are 0 by construction (no host staging, D^-1 fused into "
                                "the sweep)"}
        if info.rank == 0:
            print(f"[bench] {args.profile_phases} profiled iterations (MAX over {world} ranks):\n"
                  + ds.phase_table(ph), file=sys.stderr, flush=True)

    watch.phase("report")
    if info.rank == 0:
        out = {
            "metric": METRIC,
            "value": round(mlups, 1),
            "unit": "MLUPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(mlups / BASELINE_MLUPS, 2),
            "dtype": args.dtype,
            "data": "cpu-dry-run (plain-PyTorch PCG on CPU: flow test, not a measurement)" if dry else
                    (f"share-gpu rehearsal (all ranks on one GPU, {comm_used} transport: not a measurement)"
                     if share else "synthetic (reference problem: F=1 in ellipse x^2+4y^2<1, zero initial guess)"),
            "config": {
                "model": f"fictitious-domain Poisson ellipse, Jacobi-PCG, {args.M}x{args.N}",
                "global_batch": 1,
                "seq_len": pts,
                "parallelism": f"domain{world}" if world > 1 else "single",
                "split": args.split,
                "process_grid": list(process_grid(world, args.M, args.N, args.split)),
                "grid": [args.M, args.N],
                "comm": comm_used,
                "rung": rung if world > 1 else None,
                "rccl_graph": bool(comm_used == "rccl" and cfg["rccl_graph"]),
                "split_sweep": bool(getattr(runner, "split_sweep", False)),
                "kernel": args.kernel,
                "tile": tile_desc,
                "graph_batch": args.graph_batch,
                "overlap": "on" if overlap else "off",
                "rccl_communicators": (2 if overlap else 1) if comm_used == "rccl" else None,
                "exact": args.exact,
            },
            "timed_path": timed_path,
            "timed_graph_lengths": path.get("graph_lengths", []),
            "timed_graph_iters": path["graph_iters"],
            "timed_eager_iters": path["eager_iters"],
            "graphs_prepared": bool(prepared),
            "valid": valid and not share,
            "baseline_mlups": BASELINE_MLUPS,
            **tol,
            **phases,
        }
        line = json.dumps(out)
        if supervised and result_path:
            with open(result_path, "w") as f:
                f.write(line + "\n")
        else:
            print(line, flush=True)
            if args.json_out:
                with open(args.json_out, "w") as f:
                    f.write(line + "\n")
    watch.phase("shutdown")
    launch.shutdown()
    return 0


def measure_loopback(args) -> int:
    """One rank of the --gpus-rank job alone on this GPU (LoopbackComm): per-rank iteration time of
    the real schedule.  Prints one JSON line (valid=false: not a multi-GPU measurement)."""
    import importlib

    import torch

    pkg_name = "poisson-ellipse-openmp-mpi-cuda-new_amd"
    pmx = importlib.import_module(pkg_name)
    native = pmx.load_native()
    if not torch.cuda.is_available():
        raise SystemExit("--loopback-rank needs an MI355X")
    if not 0 <= args.loopback_rank < args.gpus:
        raise SystemExit("--loopback-rank must be in [0, --gpus)")
    problem = pmx.PoissonEllipse(M=args.M, N=args.N, breakdown_tol=args.breakdown_tol)
    # the algorithm the real N-GPU run would use (see measure: the s-step PCG on big fp64 row strips)
    ca_ok = not args.exact
    if args.algo == "ca" and not ca_ok:
        raise SystemExit("[bench] --algo ca (the s-step PCG) runs the fast arithmetic")
    algo_id = {"auto": -1, "pcg1": 1, "pcg2": 2, "ca": 3}[args.algo]  # auto: the library's choose_algo
    s = native.Session(problem.to_native(), world=args.gpus, comm="loopback", split=getattr(native.Split, args.split),
                       ranks=[args.loopback_rank], devices=[0], dtype=args.dtype, graph_batch=args.graph_batch,
                       overlap=args.overlap == "on", placement=args.placement,
                       placement_budget_s=args.placement_budget, placement_keep_free=args.placement_keep_free,
                       algo=algo_id, ca_s=args.ca_s)
    sd = s.subdomain(0)
    s.init()
    s.step(args.warmup)
    s.synchronize()
    prepared = s.prepare(args.steps)
    st0 = s.state(0)
    s.reset_path_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.step(args.steps)
    s.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st1 = s.state(0)
    path = s.path_stats()
    pts = sd["nx"] * sd["ny"]
    tile = dict(s.tile)
    tile.pop("placement_probe_ms", None)
    out = {
        "metric": "per-rank iteration time of one rank of a multi-GPU decomposition (loopback rehearsal)",
        "value": round(dt / args.steps * 1e6, 2), "unit": "us/iteration", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": False,
        "dtype": args.dtype,
        "data": f"loopback: rank {args.loopback_rank} of {args.gpus} alone, ghosts written as zeros (Dirichlet) "
                "by one fill launch per exchange; all-reduce and transfer stand-ins: "
                f"{os.environ.get('PMX_LOOPBACK_AR_US', '0')} / {os.environ.get('PMX_LOOPBACK_HALO_US', '0')} us",
        "config": {"grid": [args.M, args.N], "world": args.gpus, "rank": args.loopback_rank, "split": args.split,
                   "process_grid": list(s.grid), "subdomain": [sd["nx"], sd["ny"]], "comm": s.comm_name,
                   "split_sweep": bool(s.split_sweep), "direct_rows": bool(s.direct_rows), "tile": tile,
                   "graph_batch": args.graph_batch, "overlap": args.overlap},
        "rank_mlups": round(pts * args.steps / dt / 1e6, 1),
        "timed_path": "graph" if path["eager_iters"] == 0 else "mixed",
        "graphs_prepared": bool(prepared),
        "iterations_ran": int(st1["it"] - st0["it"]), "stopped": bool(st1["done"]),
        "valid": False,
    }
    print(json.dumps(out), flush=True)
    return 0


# Placement classes of a kept field block (GpuSubdomainSolver::place_fields times 6 real iterations
# per candidate).  At 16384^2 fp64 the blocks fall into ~three rates (profiles/r3/placement/,
# profiles/r4/placement/): ~10.7 ms per 6 iterations (1.78-1.80 ms/step), ~11.0-11.3, and
# ~11.55-11.65 (1.92-1.95 ms/step), i.e. ~6.65 / ~6.9 / ~7.2 ps per point and iteration.  The
# class says which one the timed run got, so a driver record can be read against the others.
PLACEMENT_CLASS_PS = ((6.80, "fast"), (7.05, "mid"))
# s-step PCG (6 iterations = 2 fused blocks per candidate, round 6): provisional limits from the
# 16384^2 same-process A/Bs, whose sessions ran at ~0.95 or ~1.01-1.02 ms/iteration (fused pass ~2.85 /
# ~3.05 ms: ~3.55 / ~3.8 ps per point and iteration, profiles/r6/shape/)
PLACEMENT_CLASS_PS_CA = ((3.65, "fast"), (3.85, "mid"))


def placement_class(kept_ms, points, dtype, algo="pcg1"):
    """'fast' / 'mid' / 'slow' for fp64 grids of >= 8192^2 points (bandwidth-bound), else None."""
    if not kept_ms or dtype != "fp64" or points < 8192 * 8192:
        return None
    ps = float(kept_ms) / 6.0 / points * 1e9
    for lim, name in (PLACEMENT_CLASS_PS_CA if algo == "ca" else PLACEMENT_CLASS_PS):
        if ps < lim:
            return name
    return "slow"


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.loopback_rank >= 0:
        sys.exit(measure_loopback(args))
    if os.environ.get("PMX_BENCH_ROLE") != "child" and args.gpus > 1:
        sys.exit(supervise(args))
    if os.environ.get("PMX_BENCH_ROLE") != "child" and int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but {os.environ.get('WORLD_SIZE')} rank(s) came up "
                         "(WORLD_SIZE); refusing to report a different GPU count")
    sys.exit(measure(args))


if __name__ == "__main__":
    main()
