"""Device ops: hand-written HIP kernels (kernels.py) and their PyTorch references (reference.py)."""
from . import reference  # noqa: F401


def DeviceOps(*a, **kw):  # lazy: importing the GPU wrapper needs the native extension
    from .kernels import DeviceOps as _D

    return _D(*a, **kw)
