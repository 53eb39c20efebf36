"""bench.py multi-GPU supervision (CPU dry runs): the fallback ladder and the progress watchdog.

The supervisor (bench.py itself, or one process per rank under torchrun) never touches the GPU; it
starts the measuring ranks as fresh child processes, one rung of the ladder at a time: native
RCCL + graphs + split sweep -> native eager -> native IPC transport -> torch.distributed.  Faults
are injected with PMX_BENCH_FAULT ('<rung>:<hang|fail|crash>[@rank]'); a hang must be ended by the per-phase watchdog
(exit 87, phase printed) and the JSON must name the rung that produced it and the failed rungs.
Reference rank lifecycle: stage4-mpi+cuda/poisson_mpi_cuda_f.cu:986-1039."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, free_port

BASE = ["--cpu-dry-run", "--M", "64", "--N", "96", "--steps", "4", "--warmup", "1", "--deadline-scale", "0.05"]


def _env(fault=None):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PMX_BENCH_ROLE", "PMX_BENCH_FAULT"):
        env.pop(k, None)
    if fault:
        env["PMX_BENCH_FAULT"] = fault
    return env


def _spawned(n, fault=None, extra=()):
    return subprocess.run([sys.executable, "bench.py", "--gpus", str(n), *BASE, *extra], cwd=ROOT,
                          capture_output=True, text=True, timeout=300, env=_env(fault))


def _torchrun(n, fault=None, extra=()):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", str(n), *BASE, *extra]
    return subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400, env=_env(fault))


def _one_json(p):
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout  # the supervisor's stdout carries the JSON line only
    return lines[0]


def test_ladder_advances_past_hang_and_failure():
    p = _spawned(2, "1:hang@1,2:fail")
    assert p.returncode == 0, p.stderr[-3000:]
    j = _one_json(p)
    assert j["config"]["rung"] == 3
    lad = j["ladder"]
    assert [a["rung"] for a in lad] == [1, 2, 3] and [a["ok"] for a in lad] == [False, False, True]
    assert "status 87" in lad[0]["reason"] and lad[0]["phase"] == "canary"  # the watchdog ended the hung rung
    assert "status 1" in lad[1]["reason"] and lad[1]["phase"] in ("start", "setup")
    assert "no progress in phase 'canary'" in p.stderr
    assert j["valid"] and j["tol_status"] == "converged" and j["n_gpus"] == 2
    # rung 2 is the serialized schedule (overlap off, one communicator); rung 1 the overlapped one
    assert lad[1]["overlap"] is False and lad[0]["overlap"] is None


def test_comm_init_failure_skips_the_other_rccl_rung():
    """A rung that hangs in comm-init (the RCCL communicator initialisation) takes the other RCCL
    rung with it -- rung 2 would repeat the identical initialisation -- and the ladder goes straight
    to the IPC transport (rung 3)."""
    p = _spawned(2, "1:hang-init@0")
    assert p.returncode == 0, p.stderr[-3000:]
    j = _one_json(p)
    lad = j["ladder"]
    assert j["config"]["rung"] == 3 and [a["rung"] for a in lad] == [1, 2, 3]
    # rank 1 times out first (in 'canary', waiting for rank 0); the stuck rank 0 names the phase
    assert lad[0]["phase"] == "comm-init" and "least advanced rank: 'comm-init'" in lad[0]["reason"]
    assert lad[1].get("skipped") and "comm-init" in lad[1]["reason"] and "seconds" not in lad[1]
    # a failure in any later phase does NOT skip rung 2 (its schedule is what differs)
    q = _spawned(2, "1:fail-init@1")
    j = _one_json(q)
    assert j["config"]["rung"] == 3 and j["ladder"][1].get("skipped")
    r = _spawned(2, "1:hang@0")
    assert _one_json(r)["config"]["rung"] == 2


def test_ladder_fits_the_lease():
    """Deadlines and rung caps are sized so the worst ladder -- rung 1 hangs, rung 2 hangs, rung 3
    succeeds -- ends within 540 s at full scale (driver lease: 600 s), and each phase deadline stays
    well inside its rung's cap."""
    sys.path.insert(0, ROOT)
    import bench

    for n in (2, 4, 8):
        a = bench.parse(["--gpus", str(n)])
        assert bench.worst_case_ladder_seconds(a) <= 540.0
        assert bench._ladder(a)[:3] == [1, 2, 3]
    d = bench.DEADLINES
    assert bench.COMM_INIT_TIMEOUT <= 90.0
    # a hang in any single phase is caught by its watchdog before the rung cap of rungs 1 and 2
    worst_phase = max(v for k, v in d.items() if k != "profile")
    assert d["setup"] + worst_phase + 10 < min(bench.RUNG_CAP[1], bench.RUNG_CAP[2]) + d["setup"]
    # rung 3 keeps >= 150 s after two rungs hung to their caps (a healthy 16384^2 rung takes ~30-60 s)
    assert bench.LADDER_BUDGET - (bench.RUNG_CAP[1] + bench.RUNG_CAP[2] + 20) >= 150
    # rung 2 is fully serialized, and comm-init failures of rung 1 skip it
    assert bench.RUNGS[2]["overlap"] is False and bench.RUNGS[2]["rccl_graph"] is False
    assert bench.skipped_after(1, "comm-init", [2, 3, 4]) == [2]
    assert bench.skipped_after(1, "canary", [2, 3, 4]) == []
    assert bench.skipped_after(3, "comm-init", [4]) == []


def test_two_hung_rungs_still_produce_rung3_json():
    p = _spawned(2, "1:hang,2:hang")
    assert p.returncode == 0, p.stderr[-3000:]
    j = _one_json(p)
    assert j["config"]["rung"] == 3 and [a["ok"] for a in j["ladder"]] == [False, False, True]
    assert all(a["phase"] == "canary" for a in j["ladder"][:2])
    assert j["ladder_seconds"] < 120  # deadline scale 0.05


def test_ladder_under_torchrun():
    """One supervisor per torchrun rank: they agree on a fresh port per rung through torchrun's store
    and stop their children when any rank fails."""
    p = _torchrun(2, "1:crash@0,2:hang")
    assert p.returncode == 0, p.stderr[-3000:]
    j = _one_json(p)
    assert j["config"]["rung"] == 3
    assert [a["ok"] for a in j["ladder"]] == [False, False, True]
    assert "status 3" in j["ladder"][0]["reason"] and "status 87" in j["ladder"][1]["reason"]


def test_ladder_first_rung_success_records_path():
    p = _spawned(2)
    assert p.returncode == 0, p.stderr[-3000:]
    j = _one_json(p)
    assert j["config"]["rung"] == 1 and len(j["ladder"]) == 1 and j["ladder"][0]["ok"]
    for k in ("timed_path", "timed_graph_iters", "timed_eager_iters", "l2_error", "max_error", "tol_note"):
        assert k in j
    assert j["timed_path"] == "eager" and j["timed_eager_iters"] == 4  # the CPU runner has no graphs
    assert {"comm", "rccl_graph", "split_sweep", "rung"} <= set(j["config"])
    # the analytic-solution error of the tol solve (64x96: ~2e-3, far above the solve tolerance)
    assert 1e-4 < j["l2_error"] < 1e-2 and j["max_error"] >= j["l2_error"] / 2


def test_every_rung_failing_fails_the_job():
    """Still ONE JSON line -- value null, valid false, the ladder's reasons -- and a failing exit."""
    p = _spawned(2, "1:fail,2:fail,3:crash,4:fail")
    assert p.returncode != 0
    j = _one_json(p)
    assert j["value"] is None and j["valid"] is False and j["n_gpus"] == 2
    assert [a["rung"] for a in j["ladder"]] == [1, 2, 3, 4] and not any(a["ok"] for a in j["ladder"])
    assert "status 3" in j["ladder"][2]["reason"] and "every rung" in j["error"]
    assert "every rung of the ladder failed" in p.stderr


def test_ladder_off_stops_at_the_first_rung():
    p = _spawned(2, "1:fail", extra=("--ladder", "off"))
    assert p.returncode != 0
    j = _one_json(p)
    assert j["valid"] is False and len(j["ladder"]) == 1


@pytest.mark.parametrize("comm,first", [("torch", 4), ("ipc", 3)])
def test_comm_flag_picks_the_first_rung(comm, first):
    p = _spawned(2, extra=("--comm", comm))
    assert p.returncode == 0, p.stderr[-3000:]
    j = _one_json(p)
    assert j["config"]["rung"] == first and [a["rung"] for a in j["ladder"]] == [first]


def test_single_rank_watchdog_reports_phase():
    """A single rank (no supervisor) is watched too: an injected hang ends with the phase named."""
    env = _env("1:hang")
    env["PMX_BENCH_ROLE"] = "child"  # as a supervised rank, so the fault hook is armed
    p = subprocess.run([sys.executable, "bench.py", *BASE], cwd=ROOT, capture_output=True, text=True,
                       timeout=120, env=env)
    assert p.returncode == 87
    assert "no progress in phase 'canary'" in p.stderr
