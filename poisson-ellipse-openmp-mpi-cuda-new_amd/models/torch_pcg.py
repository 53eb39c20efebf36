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

    # ---- stepwise interface (same contract as the native Session: init / step / state) ----
    def init(self):
        P = self.p
        h1, h2 = P.h1, P.h2
        self.w = torch.zeros(self.B.shape, dtype=self.dtype, device=self.device)
        self.r = self.B.clone()
        self.pv = torch.zeros_like(self.w)
        z = R.precond(self.r, self.a, self.b, h1, h2)
        self.pv[1:-1, 1:-1] = z
        self.zr_old = self._allsum(R.dot(z, self.r[1:-1, 1:-1], h1, h2))
        self.k = 1
        self.done = False
        self.status, self.iters, self.diff = "max_iter", 0, float("nan")

    def step(self, n: int = 1):
        """Run up to n iterations (no-ops once the stop rule fired, like the device flag)."""
        P = self.p
        h1, h2 = P.h1, P.h2
        weighted = P.norm == "weighted"
        a, b, w, r, p = self.a, self.b, self.w, self.r, self.pv
        for _ in range(n):
            if self.done:
                return
            if self.k > P.effective_max_iter():
                self.done, self.status = True, "max_iter"
                return
            k = self.k
            self.iters = k
            self._exchange(p)
            Ap = R.apply_A(p, a, b, h1, h2)
            denom = self._allsum(R.dot(Ap, p[1:-1, 1:-1], h1, h2))
            tol = P.breakdown_tol
            if (abs(denom) < tol) if weighted else (denom < tol):
                self.done, self.status = True, "breakdown"
                return
            alpha = self.zr_old / denom
            w_old = w[1:-1, 1:-1].clone()
            w[1:-1, 1:-1] += alpha * p[1:-1, 1:-1]
            r[1:-1, 1:-1] -= alpha * Ap
            z = R.precond(r, a, b, h1, h2)
            zr_new = self._allsum(R.dot(z, r[1:-1, 1:-1], h1, h2))
            dw = w[1:-1, 1:-1] - w_old
            dsum = self._allsum((dw * dw).sum(dtype=torch.float64))
            self.diff = math.sqrt(dsum * h1 * h2) if weighted else math.sqrt(dsum)
            self.k = k + 1
            if self.diff < P.delta:
                self.done, self.status = True, "converged"
                return
            beta = zr_new / self.zr_old
            self.zr_old = zr_new
            p[1:-1, 1:-1] = z + beta * p[1:-1, 1:-1]

    def state(self) -> dict:
        return dict(it=self.k, done=self.done, iters=self.iters, status=self.status, diff=self.diff, nan=False)

    def local_error_stats(self) -> dict:
        """Unreduced (sum e^2, max |e|, max w) of this rank's block vs the analytic solution."""
        wl = self.w[1:-1, 1:-1].to(torch.float64).cpu().numpy()
        return self.p.local_error_stats(self.sd, wl)

    def synchronize(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def solve(self, keep_solution: bool = True) -> Result:
        P = self.p
        t0 = time.perf_counter()
        self.init()
        while not self.done:
            self.step(64)
        seconds = time.perf_counter() - t0
        iters, status, diff = self.iters, self.status, self.diff
        wl = None
        if keep_solution:
            wl = self.w[1:-1, 1:-1].to(torch.float64).cpu().numpy()
        res = Result(iters, status, diff, seconds, None, backend="torch", ranks=self.comm.world)
        res.extra["local_w"] = wl
        res.extra["subdomain"] = self.sd
        if keep_solution and self.comm.world == 1:
            import numpy as np

            g = np.zeros((P.M + 1, P.N + 1))
            g[1:P.M, 1:P.N] = wl
            res.w = g
        return res
