"""Python-side communicators over torch.distributed (``nccl`` == RCCL on ROCm, or ``gloo``).

* ``SingleComm``  -- world size 1: nothing to exchange.
* ``TorchComm``   -- torch.distributed collectives on torch tensors: scalar all-reduce
                     (MPI_Allreduce, stage2-mpi/poisson_mpi_decomp.cpp:396,412,435,439) and the
                     4-neighbour ghost exchange (stage2-mpi/poisson_mpi_decomp.cpp:241-347) as one
                     batched isend/irecv group.  Works with gloo (CPU tests) and nccl/RCCL (GPU).

The native GPU path has its own RCCL communicator (csrc/comm/comm.hip); this module is the
portable/testing path and the fallback when the native communicator cannot be created.
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.distributed as dist

# side order everywhere: 0 x-lo, 1 x-hi, 2 y-lo, 3 y-hi (opposite = side ^ 1)
SIDES = ("nb_xlo", "nb_xhi", "nb_ylo", "nb_yhi")


def neighbours(sd: dict) -> list[int]:
    return [sd[k] for k in SIDES]


def edge_view(f: torch.Tensor, side: int, ghost: bool) -> torch.Tensor:
    """View of the interior edge (ghost=False) or the ghost line (ghost=True) of a ghosted array."""
    nx, ny = f.shape[0] - 2, f.shape[1] - 2
    if side == 0:
        return f[0 if ghost else 1, 1:ny + 1]
    if side == 1:
        return f[nx + 1 if ghost else nx, 1:ny + 1]
    if side == 2:
        return f[1:nx + 1, 0 if ghost else 1]
    return f[1:nx + 1, ny + 1 if ghost else ny]


class SingleComm:
    rank = 0
    world = 1

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def exchange(self, sends: Sequence[torch.Tensor | None], recvs: Sequence[torch.Tensor | None],
                 nbs: Sequence[int]) -> None:
        assert all(n < 0 for n in nbs), "SingleComm with neighbours"

    def barrier(self):
        pass


class TorchComm:
    def __init__(self, group=None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised (see parallel.launch.init_distributed)")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def exchange(self, sends, recvs, nbs) -> None:
        """sends[s] -> neighbour nbs[s] (it lands in that rank's recvs[s^1]); recvs[s] <- nbs[s]."""
        ops = []
        for s, nb in enumerate(nbs):
            if nb < 0:
                continue
            ops.append(dist.P2POp(dist.isend, sends[s], nb, self.group))
            ops.append(dist.P2POp(dist.irecv, recvs[s], nb, self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()

    def barrier(self):
        dist.barrier(group=self.group)
