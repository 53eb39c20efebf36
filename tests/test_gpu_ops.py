"""HIP ops vs plain-PyTorch fp64 references of the same op (ops/reference.py)."""
import numpy as np
import pytest
import torch

from conftest import sub

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(pkg):
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch.device("cuda", 0)


@pytest.mark.parametrize("M,N,P,rank", [(40, 40, 1, 0), (400, 600, 1, 0), (257, 130, 4, 3), (64, 1000, 2, 1)])
def test_assemble_bitwise(pkg, native, dev, M, N, P, rank):
    p = pkg.PoissonEllipse(M=M, N=N)
    Px, Py = sub("parallel.decomp").choose_process_grid(P)
    ops = pkg.ops.DeviceOps(p, Px, Py, rank) if hasattr(pkg, "ops") else sub("ops").DeviceOps(p, Px, Py, rank)
    a, b, B = ops.assemble()
    sd = ops.sd
    ra, rb, rB = sub("ops.reference").assemble(p, sd)
    assert torch.equal(a.cpu(), ra) and torch.equal(b.cpu(), rb)
    assert torch.equal(B[1:-1, 1:-1].cpu(), rB[1:-1, 1:-1])


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-13), (torch.float32, 3e-6)])
@pytest.mark.parametrize("exact", [True, False])
def test_apply_A_and_precond(pkg, dev, dtype, tol, exact):
    p = pkg.PoissonEllipse(M=300, N=211)
    ops = sub("ops").DeviceOps(p)
    R = sub("ops.reference")
    a, b, _ = R.assemble(p, ops.sd)
    g = torch.Generator().manual_seed(0)
    x = torch.rand(ops.shape, generator=g, dtype=torch.float64)
    x[0, :] = x[-1, :] = 0
    x[:, 0] = x[:, -1] = 0
    xd = x.to(dev, dtype)
    Ap = ops.apply_A(xd, exact=exact).cpu().double()[1:-1, 1:-1]
    ref = R.apply_A(xd.cpu().double(), a, b, p.h1, p.h2)
    scale = ref.abs().max()
    assert (Ap - ref).abs().max() / scale < tol
    if exact and dtype == torch.float64:
        assert torch.equal(Ap, ref)  # same arithmetic order, no FP contraction -> bitwise
    z = ops.precond(xd, exact=exact).cpu().double()[1:-1, 1:-1]
    zr = R.precond(xd.cpu().double(), a, b, p.h1, p.h2)
    assert ((z - zr).abs() / zr.abs().clamp_min(1e-300)).max() < tol


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_dot(pkg, dev, dtype):
    p = pkg.PoissonEllipse(M=513, N=771)
    ops = sub("ops").DeviceOps(p)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(ops.shape, generator=g, dtype=torch.float64)
    y = torch.randn(ops.shape, generator=g, dtype=torch.float64)
    xd, yd = x.to(dev, dtype), y.to(dev, dtype)
    got = ops.dot(xd, yd)
    ref = (xd.cpu().double()[1:-1, 1:-1] * yd.cpu().double()[1:-1, 1:-1]).sum().item()
    assert abs(got - ref) <= 1e-10 * (x.abs() * y.abs()).sum().item()


def test_ops_reject_bad_shapes(pkg, dev):
    p = pkg.PoissonEllipse(M=20, N=20)
    ops = sub("ops").DeviceOps(p)
    with pytest.raises(ValueError):
        ops.apply_A(torch.zeros(5, 5, device=dev, dtype=torch.float64))


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-13), (torch.float32, 2e-5)])
def test_mfma_wave_reductions(native, dev, dtype, tol):
    """Matrix-core wave64 sums (single and packed pair) vs torch fp64 sums per wave."""
    nw = 1000
    g = torch.Generator().manual_seed(1)
    x = (torch.rand(nw * 64, generator=g, dtype=torch.float64) - 0.3).to(dtype)
    out = torch.zeros(nw * 3, dtype=dtype, device=dev)
    xd = x.to(dev)
    native.mfma_wave_sums(xd.data_ptr(), out.data_ptr(), nw, dtype == torch.float32,
                          torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    xr = x.double().view(nw, 64)
    ref = torch.stack([xr.sum(1), xr.sum(1), (xr * xr).sum(1)], 1).flatten()
    o = out.cpu().double()
    scale = torch.stack([xr.abs().sum(1)] * 2 + [(xr * xr).sum(1)], 1).flatten()
    assert ((o - ref).abs() <= tol * scale).all(), (o - ref).abs().max()


@pytest.mark.parametrize("nq", [5, 2, 1])
def test_reduction_handoff_stress(native, nq):
    """The multi-block reductions hand their chunk sums to the last-arriving block (sc1 stores, a
    vmcnt wait, an agent-scope ticket; the last block reads with sc1 loads -- a measured-valid
    inter-workgroup hand-off on gfx950, MI355X_MICROARCH.md 'Valid forms', row 1).  Stress it the way
    a stale chunk would show: 64 blocks, 200 back-to-back launches on ONE workspace with new data
    each time, under uneven load (a bandwidth-heavy kernel on another stream).  Every result must
    match the exactly rounded host sum to fp64 summation accuracy -- a stale chunk of the previous
    launch would be off by ~1/64 of the sum -- and two runs must agree bitwise (fixed order)."""
    import math

    n, nsets = 40000, 200  # n / 512 >= 64: the maximum block count
    g = torch.Generator(device="cuda").manual_seed(nq)
    parts = torch.rand(nsets, n, nq, dtype=torch.float64, device="cuda", generator=g) + 0.5
    side = torch.cuda.Stream()
    hog = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
    outs = []
    for rep in range(2):
        out = torch.zeros(nsets, nq, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            for _ in range(20):
                hog.mul_(1.0000001)
        native.reduce_stress(parts.data_ptr(), n, nq, nsets, out.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    host = parts.cpu().numpy()
    for j in range(nsets):
        for q in range(nq):
            exact = math.fsum(host[j, :, q])
            assert abs(outs[0][j, q] - exact) <= 1e-13 * exact, (j, q, outs[0][j, q], exact)
