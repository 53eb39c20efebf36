"""2D block domain decomposition (Python mirror of csrc/include/pmx/decomp.hpp).

Reference: choose_process_grid  stage2-mpi/poisson_mpi_decomp.cpp:60-64
           decompose_2d         stage2-mpi/poisson_mpi_decomp.cpp:75-111
The native and Python versions are cross-checked in tests/test_decomp.py.
"""
from __future__ import annotations

import math


MIN_STRIP_ROWS = 128  # decomp.hpp kMinStripRows


def choose_process_grid(size: int) -> tuple[int, int]:
    if size < 1:
        raise ValueError("process count must be >= 1")
    px = int(math.sqrt(float(size)))
    while px > 1 and size % px != 0:
        px -= 1
    return px, size // px


def process_grid(size: int, M: int, N: int, split: str = "reference") -> tuple[int, int]:
    if split == "reference":
        return choose_process_grid(size)
    if split == "rows":
        return size, 1
    if split == "cols":
        return 1, size
    if split == "auto":  # mirror of make_process_grid (decomp.hpp): row strips while >= 128 rows
        if (M - 1) // size >= MIN_STRIP_ROWS:
            return size, 1
        best, cost_best = (size, 1), float("inf")
        for px in range(1, size + 1):
            if size % px:
                continue
            py = size // px
            nx, ny = (M - 1) / px, (N - 1) / py
            cost = (2.0 * ny if px > 1 else 0.0) + (2.0 * nx * 1.0001 if py > 1 else 0.0)
            if cost < cost_best:
                best, cost_best = (px, py), cost
        return best
    raise ValueError(f"unknown split {split!r}")


def _split(total: int, parts: int, idx: int) -> tuple[int, int]:
    base, rem = divmod(total, parts)
    off = 1 + sum(base + (1 if k < rem else 0) for k in range(idx))
    n = base + (1 if idx < rem else 0)
    return off, off + n - 1


def subdomain(M: int, N: int, Px: int, Py: int, rank: int) -> dict:
    if not 0 <= rank < Px * Py:
        raise ValueError(f"rank {rank} outside {Px}x{Py} grid")
    if M - 1 < Px or N - 1 < Py:
        raise ValueError(f"grid {M}x{N} too small for {Px}x{Py} ranks")
    px, py = rank % Px, rank // Px
    i0, i1 = _split(M - 1, Px, px)
    j0, j1 = _split(N - 1, Py, py)
    nx, ny = i1 - i0 + 1, j1 - j0 + 1
    return dict(M=M, N=N, Px=Px, Py=Py, rank=rank, px=px, py=py, i_start=i0, i_end=i1, j_start=j0,
                j_end=j1, nx=nx, ny=ny,
                nb_xlo=rank - 1 if px > 0 else -1, nb_xhi=rank + 1 if px < Px - 1 else -1,
                nb_ylo=rank - Px if py > 0 else -1, nb_yhi=rank + Px if py < Py - 1 else -1,
                aspect=max(nx, ny) / min(nx, ny))


# halo slots (csrc/include/pmx/device_types.hpp kHaloSlots): 4 sides, then 4 corners
SLOT_OFFSETS = ((-1, 0), (1, 0), (0, -1), (0, 1), (-1, -1), (-1, 1), (1, -1), (1, 1))


def opposite_slot(s: int) -> int:
    return s ^ 1 if s < 4 else 11 - s


def peers(sd: dict) -> list[int]:
    """Rank across each of the 8 halo slots (-1 = none); mirror of Subdomain::peer."""
    out = []
    for dx, dy in SLOT_OFFSETS:
        qx, qy = sd["px"] + dx, sd["py"] + dy
        out.append(qy * sd["Px"] + qx if 0 <= qx < sd["Px"] and 0 <= qy < sd["Py"] else -1)
    return out
