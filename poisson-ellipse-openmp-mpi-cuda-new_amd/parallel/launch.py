"""Process-group bootstrap: one process per MI355X (torchrun / torch.distributed.run).

Reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the environment.  The
reference bound ranks to GPUs implicitly through LSF and never called cudaSetDevice;
here each rank pins ``cuda:LOCAL_RANK`` explicitly before touching the device.
"""
from __future__ import annotations

import dataclasses
import os

import torch
import torch.distributed as dist


@dataclasses.dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"

    @property
    def is_distributed(self) -> bool:
        return self.world > 1


def env_info() -> DistInfo:
    return DistInfo(rank=int(os.environ.get("RANK", 0)), world=int(os.environ.get("WORLD_SIZE", 1)),
                    local_rank=int(os.environ.get("LOCAL_RANK", 0)))


def init_distributed(backend: str | None = None, device_type: str | None = None) -> DistInfo:
    """Initialise torch.distributed from env vars when WORLD_SIZE > 1 (no-op otherwise).

    backend None -> "nccl" (RCCL) when GPUs are visible, else "gloo"."""
    info = env_info()
    if info.world <= 1:
        return info
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    use_gpu = (device_type or ("cuda" if torch.cuda.is_available() else "cpu")) == "cuda"
    if use_gpu:
        torch.cuda.set_device(info.local_rank)
    backend = backend or ("nccl" if use_gpu else "gloo")
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", info.local_rank)
        dist.init_process_group(backend=backend, rank=info.rank, world_size=info.world, **kw)
    info.backend = backend
    return info


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()
