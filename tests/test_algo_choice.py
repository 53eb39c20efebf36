"""The iteration algorithm auto picks (choose_algo, gpu_solver.hip) and the memory plan it is sized
by -- pure host functions, no device.  SURVEY §5.7: grids sized against 288 GB of HBM per MI355X."""
import pytest


@pytest.fixture(scope="module")
def spec(pkg):
    return lambda M, N, **kw: pkg.PoissonEllipse(M=M, N=N, **kw).to_native()


def test_auto_picks_the_sstep_on_big_fp64_grids_and_strips(native, spec):
    assert native.choose_algo(spec(16384, 16384)) == 3
    assert native.choose_algo(spec(16384, 16384), world=8) == 3           # 8 row strips (split auto)
    assert native.choose_algo(spec(2600, 2600)) == 3                      # >= 6M points
    assert native.choose_algo(spec(1600, 2400)) == 1                      # the reference grids: pcg1
    assert native.choose_algo(spec(800, 1200)) == 1


def test_auto_keeps_pcg1_where_the_sstep_does_not_apply(native, spec):
    big = spec(16384, 16384)
    assert native.choose_algo(big, world=8, split=native.Split.reference) == 3  # 2 x 4 blocks (config 4)
    assert native.choose_algo(spec(3000, 3000), world=64, split=native.Split.reference) == 3  # 375 x 375 blocks
    assert native.choose_algo(spec(2600, 2600), world=1024, split=native.Split.rows) == 1  # 2-row strips
    assert native.choose_algo(big, dtype="fp32") == 3      # fp32 fields, fp64 basis and sums
    assert native.choose_algo(big, dtype="mixed") == 3
    assert native.choose_algo(spec(800, 1200), dtype="fp32") == 1
    assert native.choose_algo(big, exact=True) == 2                       # reference arithmetic order
    assert native.choose_algo(big, algo=1) == 1 and native.choose_algo(big, algo=2) == 2
    assert native.choose_algo(spec(800, 1200), algo=3) == 3                # explicit


def test_memory_fallback_to_pcg1(native, spec):
    """The s-step's 7 fields must fit (with 5% headroom), else auto falls back to pcg1's 5, then pcg2."""
    s = spec(16384, 16384)
    ca = native.estimate_device_bytes(s, algo=3)
    p1 = native.estimate_device_bytes(s, algo=1)
    p2 = native.estimate_device_bytes(s, algo=2)
    assert ca > p1 > p2
    assert 7 * 8 * 16383 ** 2 < ca < 1.05 * 7 * 8 * 16383 ** 2
    assert native.choose_algo(s, device_bytes=288e9) == 3
    assert native.choose_algo(s, device_bytes=ca / 0.95 * 1.001) == 3
    assert native.choose_algo(s, device_bytes=ca / 0.95 * 0.99) == 1     # s-step no longer fits: pcg1
    assert native.choose_algo(s, device_bytes=p1 / 0.95 * 0.99) == 2     # pcg1 neither: pcg2
    # ranks sharing one device count together
    assert native.choose_algo(s, world=8, device_bytes=288e9, per_device=8) == 3
    assert native.choose_algo(s, world=8, device_bytes=ca / 0.95, per_device=8) == 1


def test_max_square_grid_by_algorithm(native):
    g1 = native.max_square_grid(288e9, 1, "fp64", 0.1, 1)
    g3 = native.max_square_grid(288e9, 1, "fp64", 0.1, 3)
    auto = native.max_square_grid(288e9, 1, "fp64", 0.1)
    assert auto == g1 > g3 > 60000          # auto falls back to pcg1: its 5 fields bound the grid
    assert native.max_square_grid(288e9, 8, "fp64", 0.1, 3) > 2.8 * g3
    assert native.max_square_grid(288e9, 1, "fp32", 0.1, 1) > 1.4 * g1
