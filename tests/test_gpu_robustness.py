"""Checkpoint/resume and the halo-poison debug mode (§5.2) on the GPU path."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, sub

pytestmark = pytest.mark.gpu
PMX = os.path.join(ROOT, "poisson-ellipse-openmp-mpi-cuda-new_amd", "bin", "pmx")


@pytest.mark.parametrize("ranks,dtype", [(1, "fp64"), (4, "fp64"), (2, "fp32")])
def test_resume_from_mid_solve_checkpoint_is_bitwise(pkg, tmp_path, ranks, dtype):
    models = sub("models")
    p = pkg.PoissonEllipse(M=400, N=600)
    path = str(tmp_path / "ck.bin")
    a = models.make_session(p, ranks=ranks, dtype=dtype)
    ra = a.solve_checkpointed(path, every=100)
    wa = a.gather_local_w()
    files = [path] if ranks == 1 else [f"{path}.rank{r}" for r in range(ranks)]
    assert all(os.path.exists(f) for f in files)
    # the last periodic checkpoint is mid-solve: resuming replays the remaining iterations
    b = models.make_session(p, ranks=ranks, dtype=dtype)
    rb = b.solve_checkpointed(path, every=0, resume=True)
    assert rb["iters"] == ra["iters"] and rb["status"] == "converged"
    assert rb["launched"] < ra["launched"]
    assert np.array_equal(b.gather_local_w(), wa)


def test_checkpoint_rejects_other_grid(pkg, tmp_path):
    models = sub("models")
    path = str(tmp_path / "ck.bin")
    s = models.make_session(pkg.PoissonEllipse(M=100, N=120))
    s.init()
    s.save_checkpoint(path)
    t = models.make_session(pkg.PoissonEllipse(M=120, N=100))
    with pytest.raises(RuntimeError, match="different grid"):
        t.load_checkpoint(path)


def test_cli_checkpoint_resume(tmp_path):
    ck = tmp_path / "cli.ck"
    out = subprocess.run([PMX, "400", "600", "--backend", "hip", "--ranks", "2", "--checkpoint", str(ck),
                          "--checkpoint-every", "100"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert os.path.exists(f"{ck}.rank0") and os.path.exists(f"{ck}.rank1")
    res = subprocess.run([PMX, "400", "600", "--backend", "hip", "--ranks", "2", "--resume", str(ck)],
                         capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr
    assert "| Iter=546 |" in res.stdout


@pytest.mark.parametrize("overlap", [False, True])
def test_poisoned_halos_change_nothing_when_exchange_is_complete(pkg, overlap):
    models = sub("models")
    p = pkg.PoissonEllipse(M=260, N=390)
    ref = pkg.solve(p, "hip", ranks=4, overlap=overlap)
    s = models.make_session(p, ranks=4, overlap=overlap, poison_halos=True)
    assert s.poisoned
    st = s.solve()
    assert st["iters"] == ref.iters and not st["nan"]
    assert np.array_equal(s.gather_local_w(), ref.w)


@pytest.mark.parametrize("algo", [1, 2])
def test_poisoned_halo_without_exchange_raises_nan_flag(pkg, native, algo):
    """A ghost that never arrives stays NaN and trips the device NaN flag in the reductions
    (pcg2 reads the receive buffers directly; pcg1 unpacks them into the ghost cells)."""
    p = pkg.PoissonEllipse(M=200, N=300)
    s0 = native.SubdomainSolver(p.to_native(), Px=1, Py=2, rank=0, algo=algo)
    assert s0.single_pass == (algo == 1)
    s0.enqueue_init(0)
    s0.enqueue_poison_recv(0)  # ... and no exchange
    s0.enqueue_halo_unpack(0)  # pcg1 only (no-op for pcg2)
    s0.enqueue_phase_a(0)
    st = s0.read_state(0)
    assert st["nan"]


@pytest.mark.parametrize("steps", [7, 8])
def test_resume_with_pending_w_step_is_bitwise(pkg, tmp_path, steps):
    """A checkpoint taken mid-cycle holds deferred w steps (pcg1 fp64 moves w on one sweep in
    three: 1 or 2 steps pending); the resumed solve -- whose host iteration counter comes from the
    checkpoint and picks the plain / w sweep kernels and graph phase -- must apply them exactly like
    the uninterrupted one."""
    models = sub("models")
    p = pkg.PoissonEllipse(M=400, N=600)
    path = str(tmp_path / "ck.bin")
    ref = models.make_session(p)
    rr = ref.solve_checkpointed(str(tmp_path / "unused.bin"), every=0)
    # stop at exactly `steps`: eager launches
    a = models.make_session(p, graph_batch=0)
    a.init()
    a.step(steps)
    a.synchronize()
    assert a.state()["w_pend"] == steps and a.state()["w_pend_n"] == steps % 3
    a.save_checkpoint(path)
    b = models.make_session(p)
    rb = b.solve_checkpointed(path, every=0, resume=True)
    assert rb["iters"] == rr["iters"] == 546
    assert np.array_equal(b.gather_local_w(), ref.gather_local_w())
