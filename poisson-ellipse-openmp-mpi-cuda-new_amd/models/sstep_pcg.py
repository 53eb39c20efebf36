"""TorchSStepPCG: the s-step Jacobi-PCG of csrc/hip/ca_kernels.hip in plain PyTorch (fp64, any device).

The CPU oracle of the native s-step solver (GpuOptions::algo 3) and the executable statement of its
algorithm.  Every block of s iterations:

  pass 1   the Chebyshev basis Y = [P_0..P_s, Z_0..Z_{s-1}] of p_k and z_k = D^-1 r_k,
           P_0 = p, P_1 = L~ p, P_{i+1} = 2 L~ P_i - P_{i-1} with L~ = D^-1 A - I (spectrum in (-1, 1)),
           and the Gram matrix G = Y^T D Y from its 6s Chebyshev moments (moment_gram);
  scalars  the classic loop's s iterations on coordinate vectors (p = Y a, z = Y b, w - w_k = Y c):
           alpha = b^T G b / a^T G T a, b -= alpha T a, beta = ..., with the breakdown guard and
           max_iter where stage0/Withoutopenmp1.cpp:124-169 (and stage4-mpi+cuda/poisson_mpi_cuda_f.cu:
           847-943) has them;
  pass 2   p, z, w <- Y a_n, Y b_n, w + Y c_n, and ||Y a_j|| for the stop test |alpha_j| ||p_{k+j}|| < delta
           (on the device one reduction later; a stop inside the block takes w back to w_k + Y c_{j+1}).

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


def moment_gram(Y: list, D: torch.Tensor, s: int, h: float) -> torch.Tensor:
    """G_D from 3s products instead of (2s+1)(2s+2)/2, via the Chebyshev product rule
    T_a T_b = (T_{a+b} + T_{|a-b|}) / 2 and the D-self-adjointness of L~:
    <P_a, P_b>_D = (mu_{a+b} + mu_{|a-b|}) / 2 with mu_m = <T_m(L~) p, p>_D (and likewise nu for z,
    rho for <T_m p, z>_D).  The moments beyond the basis degree come from the last products:
    mu_{2i} = 2 <P_i, P_i> - mu_0, mu_{2i-1} = 2 <P_i, P_{i-1}> - mu_1."""
    P, Z = Y[: s + 1], Y[s + 1:]
    dot = lambda x, y: float((x * D * y).sum()) * h  # noqa: E731
    mu = [dot(P[m], P[0]) for m in range(s + 1)]
    for m in range(s + 1, 2 * s + 1):  # from <P_i, P_j>, i + j = m, |i - j| <= 1
        i, j = (m + 1) // 2, m // 2
        mu.append(2.0 * dot(P[i], P[j]) - mu[i - j])
    nu = [dot(Z[m], Z[0]) for m in range(s)]
    for m in range(s, 2 * s - 1):
        i, j = (m + 1) // 2, m // 2
        nu.append(2.0 * dot(Z[i], Z[j]) - nu[i - j])
    rho = [dot(P[m], Z[0]) for m in range(s + 1)]
    for m in range(s + 1, 2 * s):  # <P_s, Z_b> = (rho_{s+b} + rho_{s-b}) / 2
        b = m - s
        rho.append(2.0 * dot(P[s], Z[b]) - rho[s - b])
    n = 2 * s + 1
    G = torch.empty(n, n, dtype=torch.float64)
    for a in range(s + 1):
        for b in range(s + 1):
            G[a, b] = 0.5 * (mu[a + b] + mu[abs(a - b)])
        for b in range(s):
            G[a, s + 1 + b] = G[s + 1 + b, a] = 0.5 * (rho[a + b] + rho[abs(a - b)])
    for a in range(s):
        for b in range(s):
            G[s + 1 + a, s + 1 + b] = 0.5 * (nu[a + b] + nu[abs(a - b)])
    return G


class TorchSStepPCG:
    def __init__(self, problem, s: int = 3, device="cpu", gram: str = "moments"):
        self.gram = gram
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
        """One block: up to min(s, nmax) iterations, as the device runs it -- the recurrences first
        (max_iter and the |denominator| guard), then the stop test of each iteration with the explicit
        ||p_{k+j}|| (the device's pass 2 sums), w taken to the first iteration that meets it."""
        P, s = self.p, self.s
        nmax = s if nmax is None else min(s, nmax)
        h = P.h1 * P.h2
        wdiff = h if P.norm == "weighted" else 1.0
        weighted = P.norm == "weighted"
        Y = self._cheb(self.pv, s + 1) + self._cheb(self.z, s)
        n = len(Y)
        if self.gram == "moments":
            GD = moment_gram(Y, self.D, s, h)
        else:
            GD = torch.empty(n, n, dtype=torch.float64)
            for j in range(n):
                dy = self.D * Y[j]
                for i in range(j + 1):
                    GD[i, j] = GD[j, i] = float((Y[i] * dy).sum()) * h
        a = torch.zeros(n, dtype=torch.float64); a[0] = 1.0
        b = torch.zeros(n, dtype=torch.float64); b[s + 1] = 1.0
        c = torch.zeros(n, dtype=torch.float64)
        g = float(GD[s + 1, s + 1])
        left = P.effective_max_iter() - self.k
        if left <= 0:
            self.done, self.status, self.iters = True, "max_iter", self.k
            return
        its = []  # (alpha_j, a_j, c_{j+1})
        after = None
        for j in range(min(nmax, left)):
            Ta = self.T @ a
            den = float(a @ GD @ Ta)
            if (abs(den) < P.breakdown_tol) if weighted else (den < P.breakdown_tol):
                after = ("breakdown", self.k + j + 1)
                break
            alpha = g / den
            c = c + alpha * a
            its.append((alpha, a.clone(), c.clone()))
            b = b - alpha * Ta
            gn = float(b @ GD @ b)
            a = b + (gn / g) * a
            g = gn
        if not its:
            self.done, self.status, self.iters = True, after[0], after[1]
            return
        if after is None and self.k + len(its) >= P.effective_max_iter():
            after = ("max_iter", P.effective_max_iter())
        comb = lambda v: sum(float(v[i]) * Y[i] for i in range(n))  # noqa: E731
        for j, (alpha, aj, cj) in enumerate(its):
            self.diff = abs(alpha) * math.sqrt(float((comb(aj) ** 2).sum()) * wdiff)
            if self.diff < P.delta:
                self.w = self.w + comb(cj)
                self.k += j + 1
                self.done, self.status, self.iters = True, "converged", self.k
                return
        self.w = self.w + comb(its[-1][2])
        self.pv = comb(a)
        self.z = comb(b)
        self.k += len(its)
        if after is not None:
            self.done, self.status, self.iters = True, after[0], after[1]

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
