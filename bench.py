#!/usr/bin/env python3
"""Flagship benchmark: fused-HIP PCG throughput on the BASELINE.json headline config.

Metric (BASELINE.json): grid-point updates per second (MLUPS) + iterations-to-tolerance on a
16384^2 grid at 1/2/4/8 MI355X.  One "step" = one full PCG iteration (halo exchange, A p with
(Ap,p), w/r update with ||dw|| and (z,r), both all-reduces, p update) -- nothing skipped.
MLUPS = (M-1)(N-1) * steps / time / 1e6, whole-job aggregate.  The grid is fixed as N grows
(strong scaling).  Synthetic data = the reference problem itself: F = 1 in the ellipse
x^2 + 4y^2 < 1, zero initial guess (there is no dataset).

    python bench.py --gpus 1 --steps 200 --warmup 20
    python bench.py --gpus 8                  # spawns 8 ranks itself (one per GPU)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 200 --warmup 20

Without a launcher (no WORLD_SIZE in the environment) and --gpus N > 1, this process starts the N
ranks itself -- before anything touches the GPU -- and exits with their status.  A run whose rank
count differs from --gpus fails; it never measures fewer GPUs than it reports.

After the timed region a full solve to ||w^{k+1}-w^k|| < 1e-6 reports iters-to-tol and the
accuracy against the analytic solution (disable with --no-tol-solve).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_MLUPS = 2450.0  # best published reference rate: 2x P100, 2400x3200
METRIC = "grid-point updates/sec (MLUPS) + iters-to-tol, 16384^2 grid at 1/2/4/8 MI355X"


def parse():
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
    ap.add_argument("--comm", default="native", choices=["native", "torch"])
    ap.add_argument("--split", default="auto", choices=["reference", "auto", "rows", "cols"],
                    help="process grid: auto = least ghost volume (1x1, 2x1, 4x1, 4x2 blocks for 1/2/4/8 "
                         "ranks at 16384^2: wide per-rank blocks run the sweep faster, e.g. 4096x8192 "
                         "0.388 ms vs the reference's 8192x4096 0.403 ms); reference = the reference's "
                         "choose_process_grid (1x2, 2x2, 2x4)")
    ap.add_argument("--kernel", default="wave", choices=["wave", "lds"],
                    help="wave: wave-tile kernels with DPP lane shifts; lds: workgroup tiles + LDS row ring")
    ap.add_argument("--block", type=int, default=256, help="lds kernels: tile width")
    ap.add_argument("--vec", type=int, default=0, help="wave kernels: columns per lane (0 = per-kernel best)")
    ap.add_argument("--vec-b", type=int, default=0, help="pcg_b columns per lane (0 = follow --vec / auto)")
    ap.add_argument("--tile-rows-b", type=int, default=-1, help="pcg_b tile height (-1 = auto)")
    ap.add_argument("--b-kernel", default="rows", choices=["rows", "ring"],
                    help="pcg_b: ring-free 2-row tiles (default) or the software-pipelined ring kernel")
    ap.add_argument("--waves", type=int, default=4, help="wave kernels: wave tiles per workgroup")
    ap.add_argument("--tile-rows", type=int, default=0, help="tile height (0 = auto)")
    ap.add_argument("--graph-batch", type=int, default=32)
    ap.add_argument("--overlap", default="on", choices=["on", "off"],
                    help="ghost exchange on a second HIP stream, overlapped with the w/r update kernel")
    ap.add_argument("--exact", action="store_true", help="reference arithmetic order in the fused kernels")
    ap.add_argument("--tol-solve", dest="tol_solve", action="store_true", default=True)
    ap.add_argument("--no-tol-solve", dest="tol_solve", action="store_false")
    ap.add_argument("--tol-time-cap", type=float, default=300.0, help="seconds allowed for the tol solve")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="test the launch/timing/reporting flow on CPU (gloo, plain-PyTorch PCG); "
                         "prints a JSON line marked data=cpu-dry-run, not a measurement")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal: all ranks on GPU 0, native kernels, gloo comm staged through host "
                         "memory (valid=false: not a multi-GPU measurement)")
    ap.add_argument("--rccl-graph", default="on", choices=["on", "off"],
                    help="multi-rank native path: capture the RCCL calls into the hipGraph batches")
    ap.add_argument("--profile-phases", type=int, default=0,
                    help="after the run: N eager iterations timed per phase, MAX over ranks, printed as "
                         "the reference's stage-4 buckets on stderr and added to the JSON line")
    return ap.parse_args()


def spawn_ranks(n: int) -> int:
    """Start n ranks of this script (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set) and return their
    status.  Runs before any GPU call in this process; a failing rank stops the others."""
    import signal
    import socket
    import subprocess

    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PMX_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc, failed_at = 0, None
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad and failed_at is None:
            rc, failed_at = bad[0], time.time()
            print(f"[bench] a rank exited with status {rc}; stopping the others", file=sys.stderr, flush=True)
            for p in procs:
                if p.poll() is None:
                    p.send_signal(signal.SIGTERM)
        if all(c is not None for c in codes):
            break
        if failed_at is not None and time.time() - failed_at > 20:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.2)
    return rc or max(p.returncode for p in procs)


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    import importlib

    import torch
    import torch.distributed as dist

    pmx = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
    from importlib import import_module

    launch = import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.parallel.launch")
    ds = import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.parallel.dist_solver")
    process_grid = import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.parallel.decomp").process_grid
    dry = args.cpu_dry_run
    share = args.share_gpu and not dry
    info = launch.init_distributed(device_type="cpu" if (dry or share) else None)
    world = info.world
    if world != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but {world} rank(s) came up (WORLD_SIZE); refusing to "
                         "report a different GPU count")
    device = 0 if share else info.local_rank
    if not dry:
        if not torch.cuda.is_available():
            raise SystemExit("bench.py needs an MI355X (no HIP device visible)")
        if not share and torch.cuda.device_count() < world:
            raise SystemExit(f"[bench] {world} ranks need {world} visible GPUs, found {torch.cuda.device_count()}")
        torch.cuda.set_device(device)

    def device_sync():
        if not dry:
            torch.cuda.synchronize()

    problem = pmx.PoissonEllipse(M=args.M, N=args.N, breakdown_tol=args.breakdown_tol)
    kw = dict(split=args.split, dtype=args.dtype, kernel=args.kernel, block=args.block, vec=args.vec,
              waves=args.waves, tile_rows=args.tile_rows, exact=args.exact, graph_batch=args.graph_batch,
              overlap=args.overlap == "on", vec_b=args.vec_b, tile_rows_b=args.tile_rows_b,
              b_ring=args.b_kernel == "ring")
    comm_used = args.comm
    if dry:
        tp = import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.models.torch_pcg")
        comm = import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.parallel.comm")
        runner = tp.TorchPCG(problem, comm=comm.TorchComm() if world > 1 else None, split=args.split)
        runner.tile = lambda: dict(kind="torch-cpu")
        comm_used = "gloo" if world > 1 else "self"
    elif world == 1:
        models = import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.models")
        sess = models.make_session(problem, ranks=1, device=info.local_rank, **kw)

        class Runner:
            init = sess.init
            step = sess.step
            synchronize = sess.synchronize

            @staticmethod
            def tile():
                return sess.tile

            @staticmethod
            def state():
                return sess.state(0)

            @staticmethod
            def profile(n):
                sess.init()
                ph = sess.profile(int(n))
                return {"compute": ph["t_kernel_a"] + ph["t_kernel_b"], "copy": 0.0, "comm": ph["t_comm"],
                        "precond": 0.0, "dot": ph["t_reduce"]}

        runner = Runner()
        comm_used = "self"
    else:
        if share:
            runner = ds.DistGpuPCG(problem, info, comm="torch", device=0, **kw)
            comm_used = "gloo-host-staged"
        else:
            try:  # setup and RCCL init are agreed collectively: every rank raises, or none does
                runner = ds.DistGpuPCG(problem, info, comm=args.comm, rccl_graph=args.rccl_graph == "on", **kw)
            except RuntimeError as e:  # native RCCL bootstrap failed -> portable torch.distributed path
                if args.comm != "native":
                    raise
                print(f"[bench] native RCCL comm failed ({e}); falling back to torch.distributed", file=sys.stderr)
                runner = ds.DistGpuPCG(problem, info, comm="torch", **kw)
                comm_used = "torch"

    def barrier():
        if world > 1:
            dist.barrier()

    # ---------------- timed region ----------------
    runner.init()
    runner.step(args.warmup)
    runner.synchronize()
    st0 = runner.state()
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
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cpu" if (dry or share) else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    tile_desc = runner.tile() if hasattr(runner, "tile") else dict(rows=args.tile_rows, vec=args.vec)
    valid = (not st1["done"]) and (st1["it"] - st0["it"] == args.steps) and not st1["nan"]
    pts = (args.M - 1) * (args.N - 1)
    mlups = pts * args.steps / dt / 1e6

    # ---------------- iterations to tolerance ----------------
    tol = {}
    if args.tol_solve:
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
            stop = 2 if (st["done"] or launched > max_iter + batch) else 0
            if not stop and time.perf_counter() - ts > args.tol_time_cap:
                stop = 1
            if world > 1:  # one decision for all ranks: a rank that stops alone would hang the rest
                flag = torch.tensor([stop], dtype=torch.int32, device="cpu" if (dry or share) else "cuda")
                dist.all_reduce(flag, op=dist.ReduceOp.MAX)
                stop = int(flag.item())
            if stop:
                capped = stop == 1
                break
        runner.synchronize()
        barrier()
        tsolve = time.perf_counter() - ts
        tol = dict(iters_to_tol=int(st["iters"]) if st["done"] else None, tol_status=st["status"],
                   tol_final_diff=st["diff"], tol_solve_seconds=round(tsolve, 4),
                   tol_solve_mlups=round(pts * (st["iters"] if st["done"] else st["it"]) / tsolve / 1e6, 1),
                   tol_time_capped=capped)

    phases = {}
    if args.profile_phases > 0 and not dry and hasattr(runner, "profile"):
        ph = runner.profile(args.profile_phases)
        phases = {"phase_seconds_per_iter_max_over_ranks": {k: v / args.profile_phases for k, v in ph.items()}}
        if info.rank == 0:
            print(f"[bench] {args.profile_phases} profiled iterations (MAX over {world} ranks):\n"
                  + ds.phase_table(ph), file=sys.stderr, flush=True)

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
                    ("share-gpu rehearsal (all ranks on one GPU, gloo host-staged comm: not a measurement)"
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
                "kernel": args.kernel,
                "tile": tile_desc,
                "graph_batch": args.graph_batch,
                "overlap": args.overlap,
                "exact": args.exact,
            },
            "valid": valid and not share,
            "baseline_mlups": BASELINE_MLUPS,
            **tol,
            **phases,
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    launch.shutdown()


if __name__ == "__main__":
    main()
