"""Torch-facing wrappers of the hand-written HIP ops (csrc/hip/ops_kernels.hip).

Each op takes/returns ghosted torch tensors of shape (nx+2, ny+2) on ``cuda:<device>`` and runs
on torch's current stream.  They fail loudly when the native extension or the GPU is missing --
there is no silent PyTorch fallback (tests compare them against ops/reference.py instead).
"""
from __future__ import annotations

import torch

from ..utils.native import load as _native


class DeviceOps:
    def __init__(self, problem, Px: int = 1, Py: int = 1, rank: int = 0, device: int = 0):
        if not torch.cuda.is_available():
            raise RuntimeError("DeviceOps needs a GPU (HIP device)")
        self.problem = problem
        self.device = torch.device("cuda", device)
        n = _native()
        sd = n.decompose_2d(problem.M, problem.N, Px, Py, rank)
        self.sd = sd
        self.shape = (sd["nx"] + 2, sd["ny"] + 2)
        self.ctx = n.OpContext(problem.to_native(), Px, Py, rank, sd["ny"] + 2, device)

    def _check(self, *ts):
        for t in ts:
            if t.shape != self.shape or not t.is_contiguous() or t.device != self.device:
                raise ValueError(f"expected contiguous {self.shape} tensor on {self.device}, got "
                                 f"{tuple(t.shape)} on {t.device}")
            if t.dtype not in (torch.float64, torch.float32):
                raise TypeError(f"unsupported dtype {t.dtype}")

    @property
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def empty(self, dtype=torch.float64):
        return torch.zeros(self.shape, dtype=dtype, device=self.device)

    def assemble(self):
        """a, b (incl. ghosts) and B (interior) exactly as the reference's fic_reg."""
        a, b, B = self.empty(), self.empty(), self.empty()
        self.ctx.assemble(a.data_ptr(), b.data_ptr(), B.data_ptr(), self._stream)
        return a, b, B

    def apply_A(self, p: torch.Tensor, exact: bool = False) -> torch.Tensor:
        self._check(p)
        out = torch.zeros_like(p)
        self.ctx.apply_a(p.data_ptr(), out.data_ptr(), p.dtype == torch.float32, exact, self._stream)
        return out

    def precond(self, r: torch.Tensor, exact: bool = True) -> torch.Tensor:
        self._check(r)
        out = torch.zeros_like(r)
        self.ctx.precond(r.data_ptr(), out.data_ptr(), r.dtype == torch.float32, exact, self._stream)
        return out

    def dot(self, x: torch.Tensor, y: torch.Tensor) -> float:
        """Unweighted interior sum of x*y (deterministic block partials, fp64 accumulation)."""
        self._check(x, y)
        if x.dtype != y.dtype:
            raise TypeError("dot operands must share a dtype")
        return self.ctx.dot(x.data_ptr(), y.data_ptr(), x.dtype == torch.float32, self._stream)
