"""Problem family: 2D Poisson -Δu = F in an ellipse, fictitious-domain PCG.

This is the one "model family" of the reference (MSU course project, variant 9): every stage
solves the same discrete problem (stage0/Withoutopenmp1.cpp:9-61) and
differs only in execution strategy.  ``PoissonEllipse`` carries the problem; ``STAGES`` maps
each reference stage to the execution strategy that reproduces it here.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Optional

import numpy as np

from ..utils.native import load as _native


@dataclasses.dataclass
class PoissonEllipse:
    M: int = 40
    N: int = 40
    A1: float = -1.0
    B1: float = 1.0
    A2: float = -0.6
    B2: float = 0.6
    ax: float = 1.0          # ellipse semi-axis along x   (reference: x^2 + 4y^2 < 1)
    by: float = 0.5          # ellipse semi-axis along y
    F: float = 1.0
    delta: float = 1e-6      # stage0/Withoutopenmp1.cpp:178
    max_iter: Optional[int] = None   # None -> (M-1)(N-1)  (stage0/Withoutopenmp1.cpp:182)
    norm: str = "weighted"   # "weighted" (stages 1-4) | "unweighted" (stage 0)
    breakdown_tol: float = 1e-15     # CG guard on (Ap,p) (stage0/Withoutopenmp1.cpp:130); see spec.hpp

    def __post_init__(self):
        if self.norm not in ("weighted", "unweighted"):
            raise ValueError(f"norm must be weighted|unweighted, got {self.norm!r}")
        if self.M < 2 or self.N < 2:
            raise ValueError("grid must be at least 2x2 cells")

    # ---- derived quantities (stage0/Withoutopenmp1.cpp:107-108) ----
    @property
    def h1(self) -> float:
        return (self.B1 - self.A1) / self.M

    @property
    def h2(self) -> float:
        return (self.B2 - self.A2) / self.N

    @property
    def eps(self) -> float:
        return max(self.h1, self.h2) ** 2

    @property
    def interior_points(self) -> int:
        return (self.M - 1) * (self.N - 1)

    def effective_max_iter(self) -> int:
        return self.max_iter if self.max_iter is not None else (self.M - 1) * (self.N - 1)

    def is_reference_ellipse(self) -> bool:
        return self.ax == 1.0 and self.by == 0.5

    def to_native(self):
        n = _native()
        s = n.ProblemSpec()
        for f in ("M", "N", "A1", "B1", "A2", "B2", "ax", "by", "F", "delta", "breakdown_tol"):
            setattr(s, f, getattr(self, f))
        s.max_iter = -1 if self.max_iter is None else int(self.max_iter)
        s.norm = n.Norm.weighted if self.norm == "weighted" else n.Norm.unweighted
        return s

    # ---- geometry on the host (numpy) ----
    def coords(self):
        x = self.A1 + np.arange(self.M + 1) * self.h1
        y = self.A2 + np.arange(self.N + 1) * self.h2
        return x, y

    def exact_solution(self, x, y):
        """u = F (1 - x²/ax² - y²/by²) / (2/ax² + 2/by²) inside D, 0 outside.

        For the reference ellipse this is (1 - x² - 4y²)/10 (итоговый отчёт/Этап_4_1213.pdf p.1)."""
        q = 1.0 - (x / self.ax) ** 2 - (y / self.by) ** 2
        c = self.F / (2.0 / self.ax ** 2 + 2.0 / self.by ** 2)
        return np.where(q > 0, c * q, 0.0)

    def inside_mask(self):
        x, y = self.coords()
        X, Y = np.meshgrid(x, y, indexing="ij")
        if self.is_reference_ellipse():
            return X * X + 4.0 * Y * Y < 1.0
        return (X / self.ax) ** 2 + (Y / self.by) ** 2 < 1.0

    def local_error_stats(self, sd: dict, local: np.ndarray) -> dict:
        """Unreduced error statistics of one subdomain's interior block (nx x ny, global nodes
        i_start..i_end x j_start..j_end): the host twin of the device k_error_norms."""
        x, y = self.coords()
        X, Y = np.meshgrid(x[sd["i_start"]:sd["i_end"] + 1], y[sd["j_start"]:sd["j_end"] + 1], indexing="ij")
        u = self.exact_solution(X, Y)
        m = (X * X + 4.0 * Y * Y < 1.0) if self.is_reference_ellipse() else \
            ((X / self.ax) ** 2 + (Y / self.by) ** 2 < 1.0)
        e = np.where(m, local - u, 0.0)
        return {"sum_e2": float((e * e).sum()), "max_error": float(np.abs(e).max(initial=0.0)),
                "max_w": float(local.max(initial=-np.inf))}

    def error_norms(self, w: np.ndarray) -> dict:
        """L2 (h-weighted) and max error of a (M+1)x(N+1) solution vs the analytic one, in D."""
        x, y = self.coords()
        X, Y = np.meshgrid(x, y, indexing="ij")
        u = self.exact_solution(X, Y)
        m = self.inside_mask()
        e = np.where(m, w - u, 0.0)
        return {
            "l2_error": float(math.sqrt(float((e * e).sum()) * self.h1 * self.h2)),
            "max_error": float(np.abs(e).max()),
            "max_w": float(w.max()),
        }


# Reference stage -> (execution strategy, stop norm).  SURVEY §0 table.
STAGES = {
    "stage0": dict(backend="cpu", threads=1, norm="unweighted",
                   ref="stage0/Withoutopenmp1.cpp"),
    "stage1": dict(backend="omp", norm="weighted", ref="stage1-openmp/Withopenmp1.cpp"),
    "stage2": dict(backend="cpu-decomposed", threads=1, norm="weighted",
                   ref="stage2-mpi/poisson_mpi_decomp.cpp"),
    "stage3": dict(backend="cpu-decomposed", norm="weighted", ref="stage3-openmp+mpi/hybrid.cpp"),
    "stage4": dict(backend="hip", norm="weighted", ref="stage4-mpi+cuda/poisson_mpi_cuda_f.cu"),
}


def stage_problem(stage: str, M: int, N: int, **kw) -> PoissonEllipse:
    if stage not in STAGES:
        raise KeyError(f"unknown stage {stage!r}; choose from {sorted(STAGES)}")
    return PoissonEllipse(M=M, N=N, norm=STAGES[stage]["norm"], **kw)
