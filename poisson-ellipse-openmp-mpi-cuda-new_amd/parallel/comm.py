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
    """torch.distributed collectives.  ``stage_host`` (default: on for a gloo group) copies device
    tensors through host memory around each call -- gloo has no device P2P -- which is how several
    ranks that share ONE GPU exercise the native multi-rank solver (RCCL refuses two ranks on one
    device)."""

    def __init__(self, group=None, stage_host: bool | None = None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised (see parallel.launch.init_distributed)")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.stage_host = (self.backend == "gloo") if stage_host is None else stage_host

    def _host(self, t: torch.Tensor) -> torch.Tensor:
        return t.cpu() if (self.stage_host and t.device.type != "cpu") else t

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        h = self._host(t)
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
        if h is not t:
            t.copy_(h)
        return t

    def exchange(self, sends, recvs, nbs) -> None:
        """sends[s] -> rank nbs[s] (it lands in that rank's recvs[opposite(s)]); recvs[s] <- nbs[s].
        Any number of slots (4 sides for pcg2 / TorchPCG, 4 sides + 4 corners for pcg1)."""
        ops, back = [], []
        for s, nb in enumerate(nbs):
            if nb < 0 or sends[s] is None or sends[s].numel() == 0:
                continue
            snd, rcv = self._host(sends[s]), self._host(recvs[s])
            if rcv is not recvs[s]:
                back.append((recvs[s], rcv))
            ops.append(dist.P2POp(dist.isend, snd, nb, self.group))
            ops.append(dist.P2POp(dist.irecv, rcv, nb, self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        for dev, host in back:
            dev.copy_(host)

    def barrier(self):
        dist.barrier(group=self.group)
