"""Runs the native C++ unit tests (csrc/tests/unit_tests.cpp, built as bin/pmx_unit_tests)."""
import os
import subprocess

from conftest import ROOT


def test_native_unit_tests(pkg):
    import importlib

    importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.utils.build").build()
    exe = os.path.join(ROOT, "poisson-ellipse-openmp-mpi-cuda-new_amd", "bin", "pmx_unit_tests")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert " 0 failed" in p.stdout
