"""TorchPCG: the plain-PyTorch PCG (device-agnostic reference / distributed CPU path).

Mirrors stage2-mpi/poisson_mpi_decomp.cpp:356-460 (weighted norm, |denom| guard) or stage 0
(unweighted) on a 2D-decomposed grid, with torch tensors and a pluggable communicator
(parallel/comm.py).  With gloo it is the multi-process CPU path exercised by the test-suite;
with RCCL it runs on GPUs.  Not the fast path: the native HIP solver is.
"""
from __future__ import annotations

import math
import time

import torch

from ..ops import reference as R
from ..parallel.comm import SingleComm, edge_view, neighbours
from ..parallel.decomp import process_grid, subdomain
from .solvers import Result


class TorchPCG:
    def __init__(self, problem, device="cpu", dtype=torch.float64, comm=None, split="reference"):
        self.p = problem
        self.comm = comm or SingleComm()
        self.device = torch.device(device)
        self.dtype = dtype
        Px, Py = process_grid(self.comm.world, problem.M, problem.N, split)
        self.sd = subdomain(problem.M, problem.N, Px, Py, self.comm.rank)
        self.a, self.b, self.B = R.assemble(problem, self.sd, self.device, dtype)
        self.nbs = neighbours(self.sd)

    def _exchange(self, p: torch.Tensor):
        sends = [edge_view(p, s, ghost=False).contiguous() for s in range(4)]
        recvs = [torch.zeros_like(sends[s]) for s in range(4)]
        self.comm.exchange(sends, recvs, self.nbs)
        for s in range(4):
            g = edge_view(p, s, ghost=True)
            g.copy_(recvs[s] if self.nbs[s] >= 0 else torch.zeros_like(g))

    def _allsum(self, x: torch.Tensor) -> float:
        t = x.reshape(1).to(torch.float64)
        return float(self.comm.allreduce_(t).item())

    def solve(self, keep_solution: bool = True) -> Result:
        P = self.p
        h1, h2 = P.h1, P.h2
        weighted = P.norm == "weighted"
        a, b = self.a, self.b
        shape = self.B.shape
        w = torch.zeros(shape, dtype=self.dtype, device=self.device)
        r = self.B.clone()
        p = torch.zeros_like(w)
        t0 = time.perf_counter()
        z = R.precond(r, a, b, h1, h2)
        p[1:-1, 1:-1] = z
        zr_old = self._allsum(R.dot(z, r[1:-1, 1:-1], h1, h2))
        status, iters, diff = "max_iter", 0, float("nan")
        for k in range(1, P.effective_max_iter() + 1):
            iters = k
            self._exchange(p)
            Ap = R.apply_A(p, a, b, h1, h2)
            denom = self._allsum(R.dot(Ap, p[1:-1, 1:-1], h1, h2))
            if (abs(denom) < 1e-15) if weighted else (denom < 1e-15):
                status = "breakdown"
                break
            alpha = zr_old / denom
            w_old = w[1:-1, 1:-1].clone()
            w[1:-1, 1:-1] += alpha * p[1:-1, 1:-1]
            r[1:-1, 1:-1] -= alpha * Ap
            z = R.precond(r, a, b, h1, h2)
            zr_new = self._allsum(R.dot(z, r[1:-1, 1:-1], h1, h2))
            dw = w[1:-1, 1:-1] - w_old
            dsum = self._allsum((dw * dw).sum(dtype=torch.float64))
            diff = math.sqrt(dsum * h1 * h2) if weighted else math.sqrt(dsum)
            if diff < P.delta:
                status = "converged"
                break
            beta = zr_new / zr_old
            zr_old = zr_new
            p[1:-1, 1:-1] = z + beta * p[1:-1, 1:-1]
        seconds = time.perf_counter() - t0
        wl = None
        if keep_solution:
            wl = w[1:-1, 1:-1].to(torch.float64).cpu().numpy()
        res = Result(iters, status, diff, seconds, None, backend="torch", ranks=self.comm.world)
        res.extra["local_w"] = wl
        res.extra["subdomain"] = self.sd
        if keep_solution and self.comm.world == 1:
            import numpy as np

            g = np.zeros((P.M + 1, P.N + 1))
            g[1:P.M, 1:P.N] = wl
            res.w = g
        return res
