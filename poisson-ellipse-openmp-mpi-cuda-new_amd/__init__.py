"""pmx -- MI355X-native fictitious-domain Poisson solver (PCG, Jacobi preconditioner).

Same capabilities as mxy-kit/poisson-ellipse-openmp-mpi-cuda-new (stages 0-4: serial, OpenMP,
MPI, MPI+OpenMP, MPI+CUDA), redesigned for gfx950: fused HIP kernels, device-resident scalars,
hipGraph-batched iterations, RCCL halos/all-reduces over xGMI.

Import with ``importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")`` (the directory
name is not a Python identifier) or via the repo-root shim ``pmx.py``.
"""
from .models import STAGES, PoissonEllipse, Result, make_session, solve, stage_problem  # noqa: F401
from .utils.native import gpu_available, load as load_native  # noqa: F401

__version__ = "0.1.0"
