"""Plain-PyTorch reference implementations of every device op.

Used (a) as the numerics oracle for the HIP kernels in tests (fp64 reference of the same op) and
(b) by TorchPCG, the device-agnostic PCG (CPU or GPU, gloo or RCCL).  The formulas follow the
reference line by line:

  coefficients  stage0/Withoutopenmp1.cpp:51-54 (face length -> a_ij, b_ij)
  RHS           stage0/Withoutopenmp1.cpp:60
  operator A    stage0/Withoutopenmp1.cpp:83-85
  D^-1          stage0/Withoutopenmp1.cpp:98-99
  dot           stage0/Withoutopenmp1.cpp:64-72

Local arrays have a 1-cell ghost ring: shape (nx+2, ny+2), interior [1:-1, 1:-1].
"""
from __future__ import annotations

import torch

from ..utils.native import load as _native


def face_tables(problem, device="cpu"):
    """The six 1D tables of csrc/include/pmx/geometry.hpp as fp64 tensors (global index)."""
    t = _native().face_tables(problem.to_native())
    return {k: torch.as_tensor(v, dtype=torch.float64, device=device) for k, v in t.items()}


def _clip_len(lo, hi, root):
    # max(0, min(hi, root) - max(lo, -root)) with std::min/std::max tie semantics
    mn = torch.where(root < hi, root, hi)
    nr = -root
    mx = torch.where(lo < nr, nr, lo)
    d = mn - mx
    return torch.where(0.0 < d, d, torch.zeros_like(d))


def _face_coef(l, h, eps):
    inv_eps = 1.0 / eps
    frac = (l / h) + (1.0 - l / h) / eps
    out = torch.where(l < 1e-9, torch.full_like(l, inv_eps), frac)
    return torch.where(torch.abs(l - h) < 1e-9, torch.ones_like(l), out)


def local_index(sd):
    """Global node indices (gi, gj) of a subdomain's local arrays including ghosts."""
    gi = torch.arange(sd["i_start"] - 1, sd["i_end"] + 2)
    gj = torch.arange(sd["j_start"] - 1, sd["j_end"] + 2)
    return gi, gj


def assemble(problem, sd, device="cpu", dtype=torch.float64):
    """a, b over the local array incl. ghosts, B (RHS) on the interior.  Shapes (nx+2, ny+2)."""
    T = face_tables(problem, device)
    gi, gj = local_index(sd)
    gi, gj = gi.to(device), gj.to(device)
    ylo, yhi, rv = T["ylo"][gj][None, :], T["yhi"][gj][None, :], T["rv"][gi][:, None]
    xlo, xhi, rh = T["xlo"][gi][:, None], T["xhi"][gi][:, None], T["rh"][gj][None, :]
    a = _face_coef(_clip_len(ylo, yhi, rv), problem.h2, problem.eps)
    b = _face_coef(_clip_len(xlo, xhi, rh), problem.h1, problem.eps)
    x, y = T["x"][gi][:, None], T["y"][gj][None, :]
    if problem.is_reference_ellipse():
        inside = x * x + 4.0 * y * y < 1.0
    else:
        inside = (x / problem.ax) ** 2 + (y / problem.by) ** 2 < 1.0
    B = torch.where(inside, torch.full_like(x * y, problem.F), torch.zeros_like(x * y))
    B[0, :] = 0
    B[-1, :] = 0
    B[:, 0] = 0
    B[:, -1] = 0
    return a.to(dtype), b.to(dtype), B.to(dtype)


def apply_A(p, a, b, h1, h2):
    """(A p) on the interior; p must carry valid ghosts.  Returns (nx, ny)."""
    c = p[1:-1, 1:-1]
    ax = -1.0 / h1 * (a[2:, 1:-1] * (p[2:, 1:-1] - c) / h1 - a[1:-1, 1:-1] * (c - p[:-2, 1:-1]) / h1)
    ay = -1.0 / h2 * (b[1:-1, 2:] * (p[1:-1, 2:] - c) / h2 - b[1:-1, 1:-1] * (c - p[1:-1, :-2]) / h2)
    return ax + ay


def diag(a, b, h1, h2):
    return (a[2:, 1:-1] + a[1:-1, 1:-1]) / (h1 * h1) + (b[1:-1, 2:] + b[1:-1, 1:-1]) / (h2 * h2)


def precond(r, a, b, h1, h2):
    """z = D^-1 r on the interior.  Returns (nx, ny)."""
    D = diag(a, b, h1, h2)
    return torch.where(D != 0, r[1:-1, 1:-1] / D, torch.zeros_like(D))


def dot(u, v, h1, h2):
    """Weighted inner product over the interior (u, v are (nx, ny) or ghosted with interior=True)."""
    return (u * v).sum(dtype=torch.float64) * h1 * h2
