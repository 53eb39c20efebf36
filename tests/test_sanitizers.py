"""Host-code AddressSanitizer + UBSan run of the CPU oracle and CLI.

GPU sanitizers are not available on this pool; the device code is covered by the poison-halo
mode and the fp64 numerics tests instead."""
import importlib
import json
import os
import subprocess

import pytest

from conftest import PKG_NAME


@pytest.fixture(scope="module")
def asan_bin():
    b = importlib.import_module(PKG_NAME + ".utils.build")
    try:
        return str(b.build_sanitized())
    except RuntimeError as e:  # toolchain without libasan
        pytest.skip(f"sanitizer build unavailable: {e}")


@pytest.mark.parametrize("args,iters", [
    (["40", "40", "--backend", "cpu"], 50),
    (["40", "40", "--backend", "cpu", "--norm", "unweighted"], 61),
    (["60", "90", "--backend", "omp", "--threads", "3"], None),
    (["60", "90", "--backend", "cpu", "--ranks", "4", "--split", "auto"], None),
])
def test_cli_clean_under_asan_ubsan(asan_bin, args, iters, tmp_path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    dump = tmp_path / "w.txt"
    p = subprocess.run([asan_bin, *args, "--json", "--dump", str(dump)], capture_output=True, text=True,
                       timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    assert "AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-4000:]
    j = json.loads(p.stdout.strip().splitlines()[-1])
    assert j["status"] == "converged"
    if iters is not None:
        assert j["iters"] == iters
    assert dump.exists()
