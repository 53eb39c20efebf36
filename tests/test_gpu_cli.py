"""`pmx --backend hip`: stage-4 compatible stdout, phase buckets, JSON, ASCII dump, dtypes."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
PMX = os.path.join(ROOT, "poisson-ellipse-openmp-mpi-cuda-new_amd", "bin", "pmx")


def run(*args):
    p = subprocess.run([PMX, *map(str, args)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


def last_json(out):
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


def test_stage4_format_and_phase_buckets():
    out = run(400, 600, "--backend", "hip", "--ranks", 2, "--profile-phases", 30, "--json")
    lines = out.splitlines()
    assert lines[0] == "MPI + CUDA 2D run with 2 processes; M=400, N=600"
    assert "Converged after 546 iterations (||w(k+1)-w(k)|| < 1e-06)." in out
    for label in ("GPU compute time", "Host<->Device copy time", "MPI halo exchange time",
                  "Preconditioner CPU part time", "Dot products time"):
        assert any(label in l for l in lines), label
    assert any(l.startswith("M=400, N=600 | Iter=546 | Total Time=") for l in lines)
    j = last_json(out)
    assert j["iters"] == 546 and j["ranks"] == 2 and j["comm"] == "local"
    # single pass: no second sweep, so its bucket is exactly 0 (no event pair around nothing)
    for k in ("phase_kernel_a_s", "phase_reduce_s", "phase_allreduce_s", "phase_halo_s"):
        assert j[k] > 0, k
    assert j["phase_kernel_b_s"] == 0
    assert abs(j["l2_error"] - 3.0607e-4) < 2e-7
    # the two-sweep iteration (--exact) times its second sweep; one rank times no communication
    j2 = last_json(run(400, 600, "--backend", "hip", "--ranks", 2, "--exact", "--profile-phases", 30, "--json"))
    assert j2["phase_kernel_b_s"] > 0 and j2["phase_halo_s"] > 0
    j1 = last_json(run(400, 600, "--backend", "hip", "--profile-phases", 30, "--json"))
    assert j1["phase_allreduce_s"] == 0 and j1["phase_halo_s"] == 0 and j1["phase_kernel_a_s"] > 0


@pytest.mark.parametrize("dtype", ["fp32", "mixed"])
def test_mixed_precision_cli(dtype):
    j = last_json(run(800, 1200, "--backend", "hip", "--dtype", dtype, "--json"))
    assert j["dtype"] == dtype and j["status"] == "converged"  # fp32: fp32 stencil arithmetic, mixed: fp64
    assert j["l2_error"] < 3e-4  # fp64: 1.9157e-4


def test_hip_ascii_dump_matches_cpu(tmp_path):
    f_hip, f_cpu = tmp_path / "hip.txt", tmp_path / "cpu.txt"
    run(40, 40, "--backend", "hip", "--dump", f_hip)
    run(40, 40, "--backend", "cpu", "--dump", f_cpu)
    a = np.loadtxt(f_hip)
    b = np.loadtxt(f_cpu)
    assert a.shape == b.shape == (41 * 41, 5)
    assert np.abs(a - b).max() < 1e-9
