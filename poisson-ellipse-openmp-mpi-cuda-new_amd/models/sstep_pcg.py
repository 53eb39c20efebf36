"""TorchSStepPCG: the s-step Jacobi-PCG of csrc/hip/ca_kernels.hip in plain PyTorch (fp64, any device).

The CPU oracle of the native s-step solver (GpuOptions::algo 3) and the executable statement of its
algorithm.  Every block of s iterations:

  pass 1   the Chebyshev basis Y = [P_0..P_s, Z_0..Z_{s-1}] of p_k and z_k = D^-1 r_k,
           P_0 = p, P_1 = L~ p, P_{i+1} = 2 L~ P_i - P_{i-1} with L~ = D^-1 A - I (spectrum in (-1, 1)),
           and the Gram matrices G_D = Y^T D Y (all vectors) and G_0 = Y^T Y (P_0..P_{s-1}, Z_0..Z_{s-2});
  scalars  the classic loop's s iterations on coordinate vectors (p = Y a, z = Y b, w - w_k = Y c):
           alpha = b^T G_D b / a^T G_D T a, ||p||^2 = a^T G_0 a, b -= alpha T a, beta = ..., with
           the breakdown guard, max_iter and the stop test exactly where stage0/Withoutopenmp1.cpp:124-169
           (and stage4-mpi+cuda/poisson_mpi_cuda_f.cu:847-943) has them;
  pass 2   p, z, w <- Y a_n, Y b_n, w + Y c_n.

The iterates equal the classic loop's (models/torch_pcg.py) in exact arithmetic; tests/test_sstep.py
checks iteration counts and solutions against it and against the native CPU oracle.
"""
from __future__ import annotations

import math
import time

import torch

from ..ops import reference as R
from .solvers import Result


def shift_matrix(s: int) -> torch.Tensor:
    """T with L Y = Y T on the columns that stay in the basis (L Q_0 = Q_0 + Q_1,
    L Q_i = Q_i + (Q_{i-1} + Q_{i+1}) / 2, for the P and the Z chain)."""
    n = 2 * s + 1
    T = torch.zeros(n, n, dtype=torch.float64)
    for base, m in ((0, s + 1), (s + 1, s)):
        for i in range(m - 1):
            T[base + i, base + i] = 1.0
            T[base + i + 1, base + i] = 1.0 if i == 0 else 0.5
            if i >= 1:
                T[base + i - 1, base + i] = 0.5
    return T


def g0_members(s: int) -> list[int]:
    """Basis vectors p can use within a block (the rows / columns of G_0)."""
    return list(range(s)) + list(range(s + 1, 2 * s))


class TorchSStepPCG:
    def __init__(self, problem, s: int = 3, device="cpu"):
        if s < 1:
            raise ValueError("s must be >= 1")
        self.p = problem
        self.s = s
        self.device = torch.device(device)
        sd = dict(i_start=1, i_end=problem.M - 1, j_start=1, j_end=problem.N - 1)
        self.a, self.b, B = R.assemble(problem, sd, self.device, torch.float64)
        self.B = B[1:-1, 1:-1].contiguous()
        h1, h2 = problem.h1, problem.h2
        self.D = R.diag(self.a, self.b, h1, h2)
        self.T = shift_matrix(s)

    def _lt(self, v: torch.Tensor) -> torch.Tensor:
        """L~ v = D^-1 A v - v with zero Dirichlet ghosts."""
        g = torch.nn.functional.pad(v, (1, 1, 1, 1))
        return R.apply_A(g, self.a, self.b, self.p.h1, self.p.h2) / self.D - v

    def _cheb(self, v: torch.Tensor, n: int) -> list:
        Q = [v]
        if n > 1:
            Q.append(self._lt(v))
        while len(Q) < n:
            Q.append(2.0 * self._lt(Q[-1]) - Q[-2])
        return Q

    def init(self):
        self.w = torch.zeros_like(self.B)
        self.z = self.B / self.D
        self.pv = self.z.clone()
        self.k = 0
        self.done = False
        self.status, self.iters, self.diff = "max_iter", 0, float("nan")

    def block(self, nmax: int | None = None):
        """One block: up to min(s, nmax) iterations."""
        P, s = self.p, self.s
        nmax = s if nmax is None else min(s, nmax)
        h = P.h1 * P.h2
        wdiff = h if P.norm == "weighted" else 1.0
        weighted = P.norm == "weighted"
        Y = self._cheb(self.pv, s + 1) + self._cheb(self.z, s)
        n = len(Y)
        GD = torch.empty(n, n, dtype=torch.float64)
        G0 = torch.zeros(n, n, dtype=torch.float64)
        mem = g0_members(s)
        for j in range(n):
            dy = self.D * Y[j]
            for i in range(j + 1):
                GD[i, j] = GD[j, i] = float((Y[i] * dy).sum()) * h
                if i in mem and j in mem:
                    G0[i, j] = G0[j, i] = float((Y[i] * Y[j]).sum()) * wdiff
        a = torch.zeros(n, dtype=torch.float64); a[0] = 1.0
        b = torch.zeros(n, dtype=torch.float64); b[s + 1] = 1.0
        c = torch.zeros(n, dtype=torch.float64)
        g = float(GD[s + 1, s + 1])
        nupd = 0
        for j in range(nmax):
            kk = self.k + j + 1
            if kk > P.effective_max_iter():
                self.done, self.status, self.iters = True, "max_iter", kk - 1
                break
            Ta = self.T @ a
            den = float(a @ GD @ Ta)
            if (abs(den) < P.breakdown_tol) if weighted else (den < P.breakdown_tol):
                self.done, self.status, self.iters = True, "breakdown", kk
                break
            alpha = g / den
            c = c + alpha * a
            nupd = j + 1
            self.diff = abs(alpha) * math.sqrt(max(float(a @ G0 @ a), 0.0))
            if self.diff < P.delta:
                self.done, self.status, self.iters = True, "converged", kk
                break
            b = b - alpha * Ta
            gn = float(b @ GD @ b)
            a = b + (gn / g) * a
            g = gn
        self.k += nupd
        if nupd:
            self.w = self.w + sum(float(c[i]) * Y[i] for i in range(n))
            self.pv = sum(float(a[i]) * Y[i] for i in range(n))
            self.z = sum(float(b[i]) * Y[i] for i in range(n))

    def step(self, n: int = 1):
        while n > 0 and not self.done:
            m = min(self.s, n)
            self.block(m)
            n -= m

    def solve(self) -> Result:
        t0 = time.perf_counter()
        self.init()
        while not self.done:
            self.step(self.s * 16)
        g = torch.zeros(self.p.M + 1, self.p.N + 1, dtype=torch.float64)
        g[1:-1, 1:-1] = self.w.cpu()
        return Result(self.iters, self.status, self.diff, time.perf_counter() - t0, g.numpy(),
                      backend=f"torch-sstep{self.s}")
