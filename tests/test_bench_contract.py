"""bench.py contract (driver-facing): flags, one JSON line on rank 0, required keys, torchrun
launch with one process per rank.  Runs the CPU dry-run mode (gloo + plain-PyTorch PCG), which
shares the launch / barrier / timing / MAX-over-ranks / reporting code with the GPU path."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, free_port

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check(j, n, steps, warmup):
    assert KEYS <= set(j)
    assert j["n_gpus"] == n and j["steps"] == steps and j["warmup"] == warmup
    assert j["higher_is_better"] is True and j["unit"] == "MLUPS" and j["dtype"] == "fp64"
    assert j["metric"].startswith("grid-point updates/sec (MLUPS)")
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(j["config"])
    assert j["valid"] and j["tol_status"] == "converged"
    assert "dry-run" in j["data"]


def test_bench_single_process_dry_run():
    p = subprocess.run([sys.executable, "bench.py", "--cpu-dry-run", "--M", "64", "--N", "64", "--steps", "5",
                        "--warmup", "2"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    _check(lines[0], 1, 5, 2)


@pytest.mark.parametrize("n", [2, 4])
def test_bench_torchrun_dry_run(n):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", str(n),
           "--cpu-dry-run", "--M", "64", "--N", "96", "--steps", "6", "--warmup", "2"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # rank 0 only
    _check(lines[0], n, 6, 2)
    assert lines[0]["config"]["parallelism"] == f"domain{n}"
    pg = lines[0]["config"]["process_grid"]  # default split "auto": row strips while >= 128 rows, else least halo perimeter
    assert lines[0]["config"]["split"] == "auto" and pg[0] * pg[1] == n


def test_bench_spawns_its_own_ranks():
    """Without a launcher, --gpus N starts N ranks itself (before any GPU call) and reports N."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--cpu-dry-run", "--M", "64", "--N", "96",
                        "--steps", "4", "--warmup", "1"], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    _check(lines[0], 2, 4, 1)
    assert lines[0]["config"]["parallelism"] == "domain2"


def test_bench_refuses_rank_count_mismatch():
    """A launcher that brings up fewer ranks than --gpus is an error, not a warning."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--cpu-dry-run", "--M", "32", "--N", "32",
                        "--steps", "2", "--warmup", "1"], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=env)
    assert p.returncode != 0
    assert "refusing" in p.stderr
    assert not _json_lines(p.stdout)


def test_bench_spawner_propagates_rank_failure():
    """One failing rank fails the whole job (and the spawner stops the other rank)."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--cpu-dry-run", "--M", "1", "--N", "32",
                        "--steps", "2", "--warmup", "1"], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=env)
    assert p.returncode != 0
