"""Solver entry points for every execution strategy of the reference.

=================  =====================================  ==========================================
backend            reference stage                        implementation
=================  =====================================  ==========================================
``cpu``            stage 0 serial (Withoutopenmp*.cpp)    native C++ oracle (csrc/cpu/cpu_pcg.cpp)
``omp``            stage 1 OpenMP (Withopenmp*.cpp)       native C++ oracle, OpenMP threads
``cpu-decomposed`` stage 2 MPI / stage 3 hybrid           native CpuSubdomain x P, in-process
                                                          lock-step (bin/pmx_mpi for real MPI)
``hip``            stage 4 MPI+CUDA                       native fused HIP kernels, SelfComm /
                                                          LocalComm (P subdomains on one GPU)
``torch``          (none: PyTorch reference)              models/torch_pcg.py, any device
=================  =====================================  ==========================================
Multi-process GPU runs (one rank per MI355X, RCCL) live in parallel/dist_solver.py.
"""
from __future__ import annotations

import dataclasses
import time
from typing import Optional

import numpy as np

from ..utils.native import load as _native
from .problem import PoissonEllipse


@dataclasses.dataclass
class Result:
    iters: int
    status: str
    diff: float
    seconds: float                 # solver wall time (excludes setup where measurable)
    w: Optional[np.ndarray] = None  # (M+1) x (N+1), boundary rows/cols zero
    backend: str = ""
    ranks: int = 1
    init_seconds: float = 0.0
    extra: dict = dataclasses.field(default_factory=dict)

    @property
    def converged(self) -> bool:
        return self.status == "converged"

    def mlups(self, problem: PoissonEllipse) -> float:
        return problem.interior_points * self.iters / max(self.seconds, 1e-12) / 1e6


def solve(problem: PoissonEllipse, backend: str = "hip", **kw) -> Result:
    if backend in ("cpu", "serial"):
        return solve_cpu(problem, threads=1, **kw)
    if backend in ("omp", "openmp"):
        return solve_cpu(problem, **kw)
    if backend in ("cpu-decomposed", "mpi", "hybrid"):
        return solve_cpu_decomposed(problem, **kw)
    if backend == "hip":
        return solve_hip(problem, **kw)
    if backend == "torch":
        from .torch_pcg import TorchPCG

        return TorchPCG(problem, **kw).solve()
    raise ValueError(f"unknown backend {backend!r}")


def solve_cpu(problem: PoissonEllipse, threads: int = 1, keep_solution: bool = True) -> Result:
    r = _native().cpu_solve(problem.to_native(), int(threads), bool(keep_solution))
    return Result(r["iters"], r["status"], r["diff"], r["seconds"], r.get("w"),
                  backend="cpu" if threads <= 1 else f"omp{threads}")


def solve_cpu_decomposed(problem: PoissonEllipse, ranks: int = 4, split: str = "reference",
                         threads: int = 1, keep_solution: bool = True) -> Result:
    n = _native()
    r = n.cpu_solve_decomposed(problem.to_native(), int(ranks), getattr(n.Split, split), int(threads),
                               bool(keep_solution))
    return Result(r["iters"], r["status"], r["diff"], r["seconds"], r.get("w"),
                  backend="cpu-decomposed", ranks=ranks)


def make_session(problem: PoissonEllipse, ranks: int = 1, split: str = "reference", device: int = 0,
                 dtype: str = "fp64", kernel: str = "wave", block: int = 256, vec: int = 0, waves: int = 4,
                 tile_rows: int = 0, exact: bool = False, graph_batch: int = 32, check: bool = False,
                 overlap: bool = True, vec_b: int = 0, waves_b: int = 0, tile_rows_b: int = -1,
                 poison_halos: bool = False, b_ring: bool = False, placement: int = 0,
                 placement_budget_s: float = 0.5, placement_keep_free: float = 0.5, block_tiles: int = -1,
                 algo: str | int = -1, ca_s: int = 3):
    """Native GPU session with `ranks` subdomains on one device (LocalComm when ranks > 1).

    overlap: ghost exchange on a second stream concurrent with pcg_b (only matters for ranks > 1).

    kernel="wave": wave-tile kernels with DPP neighbour shifts (vec columns/lane, `waves` tiles per
    workgroup; the round-1 "lds" kernels are retired, bench/RETIRED.md).  vec=0 picks the measured
    best per kernel (pcg_a 4, pcg_b 2 in fp64); *_b override pcg_b's shape alone.
    pcg_b runs the ring-free 2-row kernel by default; b_ring=True selects the pipelined one.

    placement: up to this many candidate field blocks are timed and the fastest kept (0 = off, the
    default; bounded by placement_budget_s seconds and by leaving placement_keep_free of the free
    device memory free -- see GpuSubdomainSolver::place_fields).

    block_tiles: -1 = auto (block-tile sweeps, pcg1_block.hip, on small undecomposed fp64 grids), 0 = off,
    1 = on for any undecomposed fp64 grid.

    algo: -1 / "auto" (the library's choice: the s-step on grids of >= 6M points -- one GPU, row strips
    or 2-D blocks -- when its fields fit, else pcg1 / pcg2), "pcg1" / 1, "pcg2" / 2, or "ca" / 3 -- the
    s-step PCG (ca_kernels.hip: ca_s = 2 or 3 iterations per fused pass and one reduction; fp64, fp32
    or mixed storage, fp64 basis and sums)."""
    n = _native()
    algo = {"auto": -1, "pcg1": 1, "pcg2": 2, "ca": 3}.get(algo, algo) if isinstance(algo, str) else algo
    return n.Session(problem.to_native(), world=int(ranks), comm="self" if ranks == 1 else "local",
                     split=getattr(n.Split, split), device=device, kernel=kernel, block=block, vec=vec,
                     waves=waves, tile_rows=tile_rows, dtype=dtype, exact=exact, graph_batch=graph_batch,
                     check=check, overlap=overlap, vec_b=vec_b, waves_b=waves_b, tile_rows_b=tile_rows_b,
                     poison_halos=poison_halos, b_ring=b_ring, placement=placement,
                     placement_budget_s=placement_budget_s, placement_keep_free=placement_keep_free,
                     block_tiles=block_tiles, algo=int(algo), ca_s=int(ca_s))


def solve_hip(problem: PoissonEllipse, ranks: int = 1, keep_solution: bool = True, poll_batches: int = 1,
              **session_kw) -> Result:
    t0 = time.perf_counter()
    s = make_session(problem, ranks=ranks, **session_kw)
    st = s.solve(poll_batches)
    w = s.gather_local_w() if keep_solution else None
    r = Result(st["iters"], st["status"], st["diff"], st["solve_seconds"], w, backend="hip", ranks=ranks,
               init_seconds=st["init_seconds"],
               extra=dict(launched=st["launched"], nan=st["nan"], setup_seconds=time.perf_counter() - t0,
                          comm=s.comm_name, grid=s.grid, device_bytes=s.device_bytes))
    del s
    return r
