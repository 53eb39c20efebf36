"""Multi-process GPU PCG: one process per MI355X, one subdomain per process.

Two communicators, same fused HIP kernels:

* ``comm="native"`` -- the production path.  Rank 0 creates an ncclUniqueId, it is broadcast
  over torch.distributed, and every rank builds its own RCCL communicator inside the native
  Session (csrc/comm/comm.hip).  Halos (ncclSend/ncclRecv in one group) and the two scalar
  all-reduces per iteration are issued from C++ on the solver's stream, optionally captured in a
  hipGraph together with the kernels.
* ``comm="torch"`` -- the portable path.  The native SubdomainSolver runs its kernels on torch's
  current stream and keeps its scalars/halo buffers in a torch-allocated arena; the all-reduces
  and the ghost exchange go through torch.distributed (ProcessGroupNCCL = RCCL).

Replaces the reference's MPI+CUDA driver (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:688-983,986-1039):
no host staging, no per-iteration host synchronisation, explicit rank->device binding.
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.distributed as dist

from ..models.solvers import Result
from ..utils.native import load as _native
from .comm import TorchComm
from .decomp import process_grid
from .launch import DistInfo


class DistGpuPCG:
    def __init__(self, problem, info: DistInfo, comm: str = "native", split: str = "reference",
                 dtype: str = "fp64", kernel: str = "wave", block: int = 256, vec: int = 0, waves: int = 4,
                 tile_rows: int = 0, exact: bool = False, graph_batch: int = 32, rccl_graph: bool = False,
                 overlap: bool = True, vec_b: int = 0, waves_b: int = 0, tile_rows_b: int = -1,
                 b_ring: bool = False):
        self.problem = problem
        self.info = info
        self.comm_kind = comm
        self.device = info.local_rank
        self.n = _native()
        self.spec = problem.to_native()
        self.Px, self.Py = process_grid(info.world, problem.M, problem.N, split)
        self.graph_batch = graph_batch
        torch.cuda.set_device(self.device)
        if comm == "native":
            uid = [self.n.rccl_unique_id() if info.rank == 0 else None]
            if info.world > 1:
                dist.broadcast_object_list(uid, src=0)
            self.session = self.n.Session(self.spec, world=info.world, comm="rccl",
                                          split=getattr(self.n.Split, split), device=self.device,
                                          kernel=kernel, block=block, vec=vec, waves=waves,
                                          tile_rows=tile_rows, dtype=dtype, exact=exact,
                                          graph_batch=graph_batch if rccl_graph else 0, uid=uid[0],
                                          ranks=[info.rank], devices=[self.device], rccl_graph=rccl_graph,
                                          overlap=overlap, vec_b=vec_b, waves_b=waves_b, tile_rows_b=tile_rows_b,
                                          b_ring=b_ring)
            self.sd = self.session.subdomain(0)
        elif comm == "torch":
            lay = self.n.comm_layout(problem.M, problem.N, self.Px, self.Py, info.rank, dtype)
            self.arena = torch.zeros(lay["bytes"] + 256, dtype=torch.uint8, device=f"cuda:{self.device}")
            base = self.arena.data_ptr()
            pad = (-base) % 256
            self.arena_view = self.arena[pad:pad + lay["bytes"]]
            self.solver = self.n.SubdomainSolver(self.spec, self.Px, self.Py, info.rank, device=self.device,
                                                 kernel=kernel, block=block, vec=vec, waves=waves,
                                                 tile_rows=tile_rows, dtype=dtype, exact=exact, arena=base + pad,
                                                 vec_b=vec_b, waves_b=waves_b, tile_rows_b=tile_rows_b,
                                                 b_ring=b_ring)
            self.sd = self.solver.subdomain()
            tdt = torch.float64 if dtype == "fp64" else torch.float32
            el = lay["elem"]
            so = lay["state_off"]
            self.red_a = self.arena_view[so + lay["red_a_off"]: so + lay["red_a_off"] + 8].view(torch.float64)
            self.red_b = self.arena_view[so + lay["red_b_off"]: so + lay["red_b_off"] + 16].view(torch.float64)
            self.sends = [self.arena_view[o:o + n * el].view(tdt) for o, n in zip(lay["send_off"], lay["edge_len"])]
            self.recvs = [self.arena_view[o:o + n * el].view(tdt) for o, n in zip(lay["recv_off"], lay["edge_len"])]
            self.nbs = [self.sd[k] for k in ("nb_xlo", "nb_xhi", "nb_ylo", "nb_yhi")]
            self.tcomm = TorchComm() if info.world > 1 else None
        else:
            raise ValueError(f"unknown comm {comm!r}")

    def tile(self) -> dict:
        if self.comm_kind == "native":
            return self.session.tile
        return dict(ntiles=self.solver.ntiles)

    # ---- torch-comm path ----
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _comm_b(self):
        if self.tcomm is None:
            return
        self.tcomm.allreduce_(self.red_b)
        self.tcomm.exchange(self.sends, self.recvs, self.nbs)

    def init(self):
        if self.comm_kind == "native":
            self.session.init()
            return
        self.solver.enqueue_init(self._stream())
        self._comm_b()
        torch.cuda.synchronize(self.device)

    def step(self, n: int):
        if self.comm_kind == "native":
            self.session.step(n)
            return
        s = self._stream()
        for _ in range(n):
            self.solver.enqueue_phase_a(s)
            if self.tcomm is not None:
                self.tcomm.allreduce_(self.red_a)
            self.solver.enqueue_phase_b(s)
            self._comm_b()

    def synchronize(self):
        if self.comm_kind == "native":
            self.session.synchronize()
        torch.cuda.synchronize(self.device)

    def state(self) -> dict:
        if self.comm_kind == "native":
            return self.session.state(0)
        return self.solver.read_state(self._stream())

    def local_w(self) -> np.ndarray:
        if self.comm_kind == "native":
            g = self.session.gather_local_w()
            sd = self.sd
            return g[sd["i_start"]:sd["i_end"] + 1, sd["j_start"]:sd["j_end"] + 1].copy()
        return self.solver.download_w(self._stream())

    def solve(self, gather: bool = True, batch: int | None = None) -> Result:
        batch = batch or max(self.graph_batch, 16)
        t0 = time.perf_counter()
        self.init()
        t1 = time.perf_counter()
        launched = 0
        max_iter = self.problem.effective_max_iter()
        while True:
            self.step(batch)
            launched += batch
            st = self.state()
            if st["done"]:
                break
            if launched > max_iter + 2 * batch:
                raise RuntimeError("device stop flag never raised")
        self.synchronize()
        t2 = time.perf_counter()
        res = Result(st["iters"], st["status"], st["diff"], t2 - t1, None, backend=f"hip-{self.comm_kind}",
                     ranks=self.info.world, init_seconds=t1 - t0, extra=dict(launched=launched, nan=st["nan"]))
        if gather:
            res.w = gather_solution(self.problem, self.sd, self.local_w(), self.info)
        return res


def gather_solution(problem, sd: dict, local: np.ndarray, info: DistInfo):
    """Assemble the global (M+1)x(N+1) solution on rank 0 (None elsewhere)."""
    pieces = [(sd, local)]
    if info.world > 1:
        out = [None] * info.world if info.rank == 0 else None
        dist.gather_object((sd, local), out, dst=0)
        pieces = out
    if info.rank != 0:
        return None
    g = np.zeros((problem.M + 1, problem.N + 1))
    for s, w in pieces:
        g[s["i_start"]:s["i_end"] + 1, s["j_start"]:s["j_end"] + 1] = w
    return g
