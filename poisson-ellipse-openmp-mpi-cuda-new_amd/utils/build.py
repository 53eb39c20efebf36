"""Native build driver: compiles the C++/HIP core for gfx950 in-tree.

Products (all inside the package directory, so they travel with the repo snapshot):
  * ``_pmx.<EXT_SUFFIX>``  -- Python extension (pybind11), HIP kernels + RCCL + CPU oracle
  * ``bin/pmx``            -- standalone C++ CLI (stage0..stage4-compatible output)
  * ``bin/pmx_mpi``        -- optional MPI CPU backend (stage 2/3 parity), when mpicxx exists

No torch.utils.cpp_extension/JIT cache: the objects are plain hipcc/g++ outputs, rebuilt
incrementally by mtime (any header change rebuilds everything).
"""
from __future__ import annotations

import concurrent.futures as cf
import contextlib
import fcntl
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent.parent
CSRC = PKG_DIR / "csrc"
BUILD_DIR = PKG_DIR / "build"
BIN_DIR = PKG_DIR / "bin"
EXT_NAME = "_pmx" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so")
EXT_PATH = PKG_DIR / EXT_NAME

ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = os.environ.get("HIPCC", str(ROCM / "bin" / "hipcc"))
ARCH = os.environ.get("PMX_ARCH", "gfx950")

HIP_SOURCES = [
    "hip/pcg_kernels.hip",
    "hip/pcg_kernels_dpp.hip",
    "hip/pcg1_kernels.hip",
    "hip/pcg1_block.hip",
    "hip/ca_kernels.hip",
    "hip/ops_kernels.hip",
    "hip/gpu_solver.hip",
    "hip/pcg_driver.hip",
    "hip/ca_solver.hip",
    "hip/pcg1_driver.hip",
    "hip/session.hip",
    "comm/comm.hip",
    "comm/ipc_comm.hip",
]
CPU_SOURCES = ["cpu/cpu_pcg.cpp"]
BIND_SOURCES = ["bindings/module.cpp"]

COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC / 'include'}", "-Wall", "-Wno-unused-result"]
HIP_FLAGS = [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
# study builds only (e.g. a package copy under bench/ab/ with other compile-time kernel bounds):
# extra hipcc flags such as -DPMX_PCG1_F32_WAVES=5
HIP_FLAGS += os.environ.get("PMX_EXTRA_HIP_FLAGS", "").split()
CPU_FLAGS = ["-fopenmp", "-ffp-contract=off"]
# host-only translation units that use the HIP runtime API (bindings, CLI): plain g++
HOST_HIP_FLAGS = ["-D__HIP_PLATFORM_AMD__", "-DPMX_WITH_HIP", f"-I{ROCM / 'include'}"]


def _headers():
    return list((CSRC / "include").rglob("*.hpp")) + list((CSRC / "hip").glob("*.hpp"))


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print("+", " ".join(str(c) for c in cmd), flush=True)
    p = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"build step failed ({p.returncode}): {' '.join(map(str, cmd))}\n{p.stdout}\n{p.stderr}")
    return p


def _compile(src: str, kind: str, verbose: bool, force: bool) -> Path:
    srcp = CSRC / src
    obj = BUILD_DIR / (src.replace("/", "_") + ".o")
    deps = [srcp] + _headers()
    if not force and not _stale(obj, deps):
        return obj
    obj.parent.mkdir(parents=True, exist_ok=True)
    if kind == "hip":
        cmd = [HIPCC, *HIP_FLAGS, *COMMON_FLAGS, "-c", srcp, "-o", obj]
    elif kind == "bind":
        import pybind11

        py_inc = sysconfig.get_paths()["include"]
        cmd = ["g++", *COMMON_FLAGS, *HOST_HIP_FLAGS, f"-I{pybind11.get_include()}", f"-I{py_inc}",
               "-fvisibility=hidden", "-c", srcp, "-o", obj]
    else:
        cmd = ["g++", *COMMON_FLAGS, *CPU_FLAGS, "-c", srcp, "-o", obj]
    _run(cmd, verbose)
    return obj


@contextlib.contextmanager
def _build_lock():
    """Serialise concurrent builds (pytest-xdist workers, parallel shells) on one lock file."""
    BUILD_DIR.mkdir(exist_ok=True)
    with open(BUILD_DIR / ".lock", "w") as fh:
        fcntl.flock(fh, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(fh, fcntl.LOCK_UN)


def build(verbose: bool = False, force: bool = False, jobs: int | None = None, apps: bool = True) -> Path:
    """Compile every native source for gfx950 and link the extension (and CLI apps)."""
    with _build_lock():
        return _build(verbose, force, jobs, apps)


def _build(verbose: bool, force: bool, jobs: int | None, apps: bool) -> Path:
    BUILD_DIR.mkdir(exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 4)
    todo = [(s, "hip") for s in HIP_SOURCES] + [(s, "cpu") for s in CPU_SOURCES] + \
           [(s, "bind") for s in BIND_SOURCES]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda a: _compile(a[0], a[1], verbose, force), todo))
    core_objs = objs[: len(HIP_SOURCES) + len(CPU_SOURCES)]
    link_libs = [f"-L{ROCM / 'lib'}", "-lrccl", "-lrocprofiler-sdk-roctx", "-lamdhip64", "-lgomp",
                 f"-Wl,-rpath,{ROCM / 'lib'}"]
    if force or _stale(EXT_PATH, objs):
        _run([HIPCC, "-shared", "-fPIC", *objs, "-o", EXT_PATH, *link_libs], verbose)
    if apps:
        _build_apps(core_objs, link_libs, verbose, force)
    return EXT_PATH


def _build_apps(core_objs, link_libs, verbose, force):
    BIN_DIR.mkdir(exist_ok=True)
    lib = BUILD_DIR / "libpmx.a"
    if force or _stale(lib, core_objs):
        if lib.exists():
            lib.unlink()
        _run(["ar", "rcs", lib, *core_objs], verbose)
    app_src = CSRC / "apps" / "pmx.cpp"
    exe = BIN_DIR / "pmx"
    if app_src.exists() and (force or _stale(exe, [app_src, lib] + _headers())):
        app_obj = BUILD_DIR / "apps_pmx.o"
        _run(["g++", *COMMON_FLAGS, *HOST_HIP_FLAGS, "-c", app_src, "-o", app_obj], verbose)
        _run([HIPCC, app_obj, lib, "-o", exe, *link_libs], verbose)
    unit_src = CSRC / "tests" / "unit_tests.cpp"
    exe_unit = BIN_DIR / "pmx_unit_tests"
    if unit_src.exists() and (force or _stale(exe_unit, [unit_src, CSRC / "cpu" / "cpu_pcg.cpp"] + _headers())):
        _run(["g++", "-O2", "-std=c++17", "-fopenmp", "-ffp-contract=off", "-Wall", f"-I{CSRC / 'include'}",
              unit_src, CSRC / "cpu" / "cpu_pcg.cpp", "-o", exe_unit], verbose)
    mpi_src = CSRC / "apps" / "pmx_mpi.cpp"
    exe_mpi = BIN_DIR / "pmx_mpi"
    mpi = _mpi_flags()
    if mpi_src.exists() and mpi and (force or _stale(exe_mpi, [mpi_src, CSRC / "cpu" / "cpu_pcg.cpp"] + _headers())):
        try:
            _run(["g++", "-O3", "-std=c++17", "-fopenmp", "-ffp-contract=off", f"-I{CSRC / 'include'}", *mpi[0],
                  mpi_src, CSRC / "cpu" / "cpu_pcg.cpp", "-o", exe_mpi, *mpi[1]], verbose)
        except RuntimeError as e:  # MPI is optional (stage-2/3 parity only)
            print(f"[pmx build] skipping pmx_mpi: {e}", file=sys.stderr)


def build_sanitized(verbose: bool = False, force: bool = False) -> Path:
    """bin/pmx_asan: the CLI with AddressSanitizer + UBSan on the HOST code.

    The CPU oracle and the CLI are recompiled with -fsanitize=address,undefined; the HIP objects
    are linked unchanged (their device code is never instrumented: GPU sanitizers are not used on
    this pool).  Meant for `--backend cpu|omp` runs, e.g. in tests/test_sanitizers.py."""
    build(verbose=verbose, apps=True)
    with _build_lock():
        return _build_sanitized(verbose, force)


def _build_sanitized(verbose: bool, force: bool) -> Path:
    san = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]
    exe = BIN_DIR / "pmx_asan"
    srcs = [CSRC / "apps" / "pmx.cpp", CSRC / "cpu" / "cpu_pcg.cpp"]
    hip_objs = [BUILD_DIR / (s.replace("/", "_") + ".o") for s in HIP_SOURCES]
    if not (force or _stale(exe, srcs + hip_objs + _headers())):
        return exe
    objs = []
    for src, extra in ((srcs[0], HOST_HIP_FLAGS), (srcs[1], CPU_FLAGS)):
        obj = BUILD_DIR / ("asan_" + src.name + ".o")
        _run(["g++", "-O1", "-g", "-std=c++17", f"-I{CSRC / 'include'}", *extra, *san, "-c", src, "-o", obj],
             verbose)
        objs.append(obj)
    _run(["g++", *san, *objs, *hip_objs, "-o", exe, "-fopenmp", f"-L{ROCM / 'lib'}", "-lrccl",
          "-lrocprofiler-sdk-roctx", "-lamdhip64", f"-Wl,-rpath,{ROCM / 'lib'}"], verbose)
    return exe


def _mpi_flags():
    """(cflags, ldflags) of an MPI installation, using the host g++ (the conda mpicxx wrapper
    points at a cross compiler that is not installed).  The MPI runtime libraries are reached
    through symlinks in bin/mpilib so that the executable's RUNPATH does not expose the MPI
    prefix's (older) libstdc++.  None when no MPI is found."""
    for root in [os.environ.get("MPI_HOME"), "/opt/conda", "/usr/lib/x86_64-linux-gnu/openmpi", "/usr"]:
        if not root:
            continue
        inc, lib = Path(root) / "include", Path(root) / "lib"
        so = sorted(lib.glob("libmpi.so.[0-9]*"))
        if not ((inc / "mpi.h").exists() and so):
            continue
        priv = BIN_DIR / "mpilib"
        priv.mkdir(parents=True, exist_ok=True)
        for pattern in ("libmpi.so.[0-9]*", "libgfortran.so.[0-9]*", "libquadmath.so.[0-9]*"):
            for f in lib.glob(pattern):
                link = priv / f.name
                if not link.exists():
                    link.symlink_to(f)
        return [f"-I{inc}"], [str(so[0]), "-Wl,-rpath,$ORIGIN/mpilib"]
    return None


def extension_built() -> bool:
    return EXT_PATH.exists()


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--no-apps", action="store_true")
    ap.add_argument("--asan", action="store_true", help="also build bin/pmx_asan (host ASan+UBSan)")
    a = ap.parse_args()
    print(build(verbose=a.verbose, force=a.force, apps=not a.no_apps))
    if a.asan:
        print(build_sanitized(verbose=a.verbose, force=a.force))
