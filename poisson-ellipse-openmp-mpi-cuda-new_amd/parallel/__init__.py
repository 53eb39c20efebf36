"""Parallelism: 2D domain decomposition, communicators, process launch, distributed GPU solver."""
from .decomp import choose_process_grid, process_grid, subdomain  # noqa: F401
from .launch import DistInfo, env_info, init_distributed, shutdown  # noqa: F401
