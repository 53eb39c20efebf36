"""Repo-root import shim: ``import pmx`` -> the ``poisson-ellipse-openmp-mpi-cuda-new_amd`` package."""
import importlib
import sys

_pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
sys.modules[__name__] = _pkg
