"""Multi-process GPU PCG: one process per MI355X, one subdomain per process.

Two communicators, same fused HIP kernels:

* ``comm="native"`` -- the production path.  Rank 0 creates an ncclUniqueId, it is broadcast
  over torch.distributed, and every rank builds its own RCCL communicator inside the native
  Session (csrc/comm/comm.hip).  Halos (ncclSend/ncclRecv in one group) and the scalar
  all-reduce(s) are issued from C++ on the solver's streams and captured in the hipGraph
  together with the kernels (``rccl_graph=True``, the default).
* ``comm="torch"`` -- the portable path.  The native SubdomainSolver runs its kernels on torch's
  current stream and keeps its scalars/halo buffers in a torch-allocated arena; the all-reduces
  and the ghost exchange go through torch.distributed: ProcessGroupNCCL (= RCCL) on GPUs, or
  gloo with the buffers staged through host memory -- which lets 2..16 processes share ONE GPU
  and run the real native multi-rank iteration (RCCL refuses two ranks on one device).

Lifecycle hardening (reference: MPI_Init/MPI_Finalize, stage4-mpi+cuda/poisson_mpi_cuda_f.cu:
987-1037): the native path builds every rank's solver first, agrees collectively that all ranks
succeeded, and only then enters the blocking RCCL initialisation, under a watchdog that ends the
process if the initialisation hangs (the launcher then stops the other ranks).

Replaces the reference's MPI+CUDA driver (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:688-983,986-1039):
no host staging, no per-iteration host synchronisation, explicit rank->device binding.
"""
from __future__ import annotations

import os
import sys
import threading
import time

import numpy as np
import torch
import torch.distributed as dist

from ..models.solvers import Result
from ..utils.native import load as _native
from .comm import TorchComm
from .decomp import process_grid, subdomain
from .launch import DistInfo

# stage-4 Table 2 buckets (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:956-980)
PHASE_BUCKETS = ("compute", "copy", "comm", "precond", "dot")
PHASE_LABELS = {
    "compute": "GPU compute time (Ap + D^{-1}r, max over ranks)",
    "copy": "Host<->Device copy time (max over ranks)       ",
    "comm": "MPI halo exchange time (max over ranks)        ",
    "precond": "Preconditioner CPU part time (max over ranks)  ",
    "dot": "Dot products time (max over ranks)             ",
}


def _comm_device(info: DistInfo, device: int):
    """Device for torch.distributed tensors: the GPU for nccl, host memory for gloo."""
    return torch.device("cuda", device) if info.backend == "nccl" else torch.device("cpu")


def agree(info: DistInfo, ok: bool, what: str, device: int = 0) -> None:
    """Collective success check: raises on EVERY rank if any rank reports failure."""
    if info.world > 1:
        t = torch.tensor([0 if ok else 1], dtype=torch.int32, device=_comm_device(info, device))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        bad = int(t.item())
    else:
        bad = 0 if ok else 1
    if bad:
        raise RuntimeError(f"{what} failed on at least one rank (rank {info.rank}: {'ok' if ok else 'failed'})")


class _Watchdog:
    """Ends the process if a blocking collective setup does not finish in time: a rank stuck in
    ncclCommInitRank cannot be interrupted, and a dead rank is what lets the launcher (torchrun or
    bench.py's spawner) stop the others instead of hanging the job."""

    def __init__(self, seconds: float, what: str):
        self.what = what
        self.timer = threading.Timer(seconds, self._fire) if seconds > 0 else None

    def _fire(self):
        print(f"[pmx] {self.what} did not finish in time; aborting this rank", file=sys.stderr, flush=True)
        os._exit(86)

    def __enter__(self):
        if self.timer:
            self.timer.daemon = True
            self.timer.start()
        return self

    def __exit__(self, *exc):
        if self.timer:
            self.timer.cancel()
        return False


class DistGpuPCG:
    def __init__(self, problem, info: DistInfo, comm: str = "native", split: str = "reference",
                 dtype: str = "fp64", kernel: str = "wave", block: int = 256, vec: int = 0, waves: int = 4,
                 tile_rows: int = 0, exact: bool = False, graph_batch: int = 32, rccl_graph: bool = True,
                 overlap: bool = True, vec_b: int = 0, waves_b: int = 0, tile_rows_b: int = -1,
                 b_ring: bool = False, algo: int = -1, init_timeout: float = 90.0, device: int | None = None,
                 placement: int = 0, placement_budget_s: float = 0.5, placement_keep_free: float = 0.5,
                 phase=None, ca_s: int = 3, split_sweep: int = -1):
        """placement: candidate field blocks of the placement probe (0 = off; forced off when ranks share
        a device).  phase(name, seconds): progress-watchdog hook (bench.py's Watch.phase); called with
        "comm-init" before the blocking communicator initialisation, whose own watchdog is
        init_timeout.  overlap=False is the serialized schedule: one RCCL communicator, every call on
        the compute stream in a fixed order.  algo: -1 = auto (the library's choose_algo: the s-step
        PCG on big fp64 row strips where its fields fit), 1 / 2 / 3; ca_s: the s-step block size;
        split_sweep: pcg1's split sweep (-1 = the transport's default, 0 off, 1 on)."""
        self.problem = problem
        self.info = info
        self.comm_kind = comm
        self.native = comm in ("native", "ipc")  # the native Session drives the iteration
        self.device = info.local_rank if device is None else device
        self.n = _native()
        self.spec = problem.to_native()
        self.Px, self.Py = process_grid(info.world, problem.M, problem.N, split)
        self.graph_batch = graph_batch
        torch.cuda.set_device(self.device)
        # ranks sharing this device (an explicit device, or more local ranks than GPUs): no placement
        # probe (its candidate blocks would crowd the peers), and the pcg1/pcg2 choice counts them all
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", info.world))
        self.shared = device is not None or local_world > torch.cuda.device_count()
        sharing = info.world if self.shared else 1
        placement = 0 if self.shared else placement
        phase = phase or (lambda name, seconds: None)
        if comm == "native":
            uid = [self.n.rccl_unique_id() if info.rank == 0 else None]
            if info.world > 1:
                dist.broadcast_object_list(uid, src=0)
            self.session, err = None, None
            try:
                self.session = self.n.Session(
                    self.spec, world=info.world, comm="rccl", split=getattr(self.n.Split, split),
                    device=self.device, kernel=kernel, block=block, vec=vec, waves=waves, tile_rows=tile_rows,
                    dtype=dtype, exact=exact, graph_batch=graph_batch if rccl_graph else 0, uid=uid[0],
                    ranks=[info.rank], devices=[self.device], rccl_graph=rccl_graph, overlap=overlap,
                    vec_b=vec_b, waves_b=waves_b, tile_rows_b=tile_rows_b, b_ring=b_ring, algo=algo,
                    defer_connect=True, placement=placement, placement_budget_s=placement_budget_s,
                    placement_keep_free=placement_keep_free, sharing=sharing, ca_s=ca_s,
                    split_sweep=split_sweep)
            except Exception as e:  # sizing / allocation: reported collectively below
                err = e
            agree(info, err is None, f"native solver setup ({err})" if err else "native solver setup",
                  self.device)
            phase("comm-init", init_timeout + 15)
            with _Watchdog(init_timeout, "RCCL communicator initialisation"):
                try:
                    self.session.connect()
                    err = None
                except Exception as e:
                    err = e
                agree(info, err is None, f"RCCL communicator initialisation ({err})", self.device)
            self.sd = self.session.subdomain(0)
            self.single_pass = self.session.tile["algo"] == "pcg1"
        elif comm == "ipc":
            # device-resident transport without RCCL (csrc/comm/ipc_comm.hip): every rank exports its
            # comm arena and flag block with hipIpcGetMemHandle, the handles travel over
            # torch.distributed, and every rank maps its peers'
            self.session, err = None, None
            try:
                self.session = self.n.Session(
                    self.spec, world=info.world, comm="ipc", split=getattr(self.n.Split, split),
                    device=self.device, kernel=kernel, block=block, vec=vec, waves=waves, tile_rows=tile_rows,
                    dtype=dtype, exact=exact, graph_batch=graph_batch, ranks=[info.rank], devices=[self.device],
                    overlap=overlap, vec_b=vec_b, waves_b=waves_b, tile_rows_b=tile_rows_b, b_ring=b_ring,
                    algo=algo, defer_connect=True, placement=placement, placement_budget_s=placement_budget_s,
                    placement_keep_free=placement_keep_free, sharing=sharing, ca_s=ca_s, split_sweep=split_sweep)
                mine = self.session.ipc_export()
            except Exception as e:
                err, mine = e, b""
            agree(info, err is None, f"native solver setup ({err})" if err else "native solver setup", self.device)
            exports = [None] * info.world
            if info.world > 1:
                dist.all_gather_object(exports, mine)
            else:
                exports = [mine]
            phase("comm-init", init_timeout + 15)
            with _Watchdog(init_timeout, "IPC transport setup"):
                try:
                    self.session.connect_ipc(exports)
                    err = None
                except Exception as e:
                    err = e
                agree(info, err is None, f"IPC transport setup ({err})", self.device)
            self.sd = self.session.subdomain(0)
            self.single_pass = self.session.tile["algo"] == "pcg1"
        elif comm == "torch":
            # ranks sharing this device (share-gpu rehearsal: all of them) count against its memory
            # in the pcg1/pcg2 choice, which every rank makes identically from global data
            lay = self.n.comm_layout(self.spec, self.Px, self.Py, info.rank, dtype=dtype, kernel=kernel,
                                     exact=exact, device=self.device, algo=algo, sharing=sharing)
            self.single_pass = bool(lay["single_pass"])
            self.solver, err = None, None
            try:  # sizing / allocation: reported collectively, so no rank waits alone in a collective
                self.arena = torch.zeros(lay["bytes"] + 256, dtype=torch.uint8, device=f"cuda:{self.device}")
                base = self.arena.data_ptr()
                pad = (-base) % 256
                self.arena_view = self.arena[pad:pad + lay["bytes"]]
                self.solver = self.n.SubdomainSolver(
                    self.spec, self.Px, self.Py, info.rank, device=self.device, kernel=kernel, block=block,
                    vec=vec, waves=waves, tile_rows=tile_rows, dtype=dtype, exact=exact, arena=base + pad,
                    vec_b=vec_b, waves_b=waves_b, tile_rows_b=tile_rows_b, b_ring=b_ring,
                    algo=1 if self.single_pass else 2)
            except Exception as e:
                err = e
            agree(info, err is None, f"solver setup ({err})" if err else "solver setup", self.device)
            assert self.solver.single_pass == self.single_pass
            self.path = {"graph_iters": 0, "eager_iters": 0, "graph_lengths": []}
            self.sd = self.solver.subdomain()
            tdt = torch.float64 if dtype == "fp64" else torch.float32
            el = lay["elem"]
            so = lay["state_off"]

            def scal(off, n):
                return self.arena_view[so + off: so + off + 8 * n].view(torch.float64)

            self.red_a, self.red_b, self.red_c = scal(lay["red_a_off"], 1), scal(lay["red_b_off"], 2), \
                scal(lay["red_c_off"], 5)
            self.sends = [self.arena_view[o:o + n * el].view(tdt) for o, n in zip(lay["send_off"], lay["edge_len"])]
            self.recvs = [self.arena_view[o:o + n * el].view(tdt) for o, n in zip(lay["recv_off"], lay["edge_len"])]
            self.peers = [p if n > 0 else -1 for p, n in zip(lay["peer"], lay["edge_len"])]
            phase("comm-init", init_timeout + 15)
            self.tcomm = TorchComm() if info.world > 1 else None
        else:
            raise ValueError(f"unknown comm {comm!r}")

    # ---- launch path / progress / accuracy ----
    @property
    def split_sweep(self) -> bool:
        return bool(self.session.split_sweep) if self.native else False

    @property
    def graphs(self) -> bool:
        return self.native and self.graph_batch > 0

    def prepare(self, n: int) -> bool:
        """Capture the graphs step(n) will replay (native path); False when it runs eagerly."""
        return bool(self.session.prepare(int(n))) if self.native else False

    def step_eager(self, n: int):
        if self.native:
            self.session.step_eager(int(n))
        else:
            self.step(n)

    def path_stats(self) -> dict:
        return dict(self.session.path_stats()) if self.native else dict(self.path)

    def reset_path_stats(self):
        if self.native:
            self.session.reset_path_stats()
        else:
            self.path = {"graph_iters": 0, "eager_iters": 0, "graph_lengths": []}

    def progress(self):
        """(sweeps reduced, exchanges packed, exchanges unpacked) from host-mapped device counters, or
        None.  Reads host memory only: safe from a watchdog thread while the main thread blocks."""
        if not self.native:
            return None
        v = self.session.progress(0)
        return None if v[0] < 0 else tuple(int(x) for x in v)

    def local_error_stats(self) -> dict:
        if self.native:
            return dict(self.session.error_norms())
        torch.cuda.synchronize(self.device)
        return dict(self.solver.error_norms(self._stream()))

    def error_norms(self) -> dict:
        """L2 (h-weighted) and max error vs the analytic solution, max w -- over all ranks."""
        return reduce_error_stats(self.local_error_stats(), self.problem, self.info, self.device)

    def tile(self) -> dict:
        if self.native:
            return self.session.tile
        return dict(ntiles=self.solver.ntiles, algo="pcg1" if self.single_pass else "pcg2")

    # ---- torch-comm path ----
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _allreduce(self, t):
        if self.tcomm is not None:
            self.tcomm.allreduce_(t)

    def _exchange(self):
        if self.tcomm is not None:
            self.tcomm.exchange(self.sends, self.recvs, self.peers)

    def _halo1(self, s):
        """pcg1 radius-2 ghosts: pack -> torch.distributed P2P -> unpack (all on torch's stream)."""
        if self.tcomm is None:
            return
        self.solver.enqueue_halo_pack(s)
        self._exchange()
        self.solver.enqueue_halo_unpack(s)

    def init(self):
        if self.native:
            self.session.init()
            return
        s = self._stream()
        self.solver.enqueue_init(s)
        if self.single_pass:  # same order as PcgDriver::init
            self._halo1(s)
            self.solver.enqueue_phase_a(s)
            self._allreduce(self.red_c)
            self._halo1(s)
        else:
            self._allreduce(self.red_b)
            self._exchange()
        torch.cuda.synchronize(self.device)

    def step(self, n: int):
        if self.native:
            self.session.step(n)
            return
        s = self._stream()
        self.path["eager_iters"] += int(n)
        for _ in range(n):
            self.solver.enqueue_phase_a(s)
            if self.single_pass:
                self._allreduce(self.red_c)
                self._halo1(s)
            else:
                self._allreduce(self.red_a)
                self.solver.enqueue_phase_b(s)
                self._allreduce(self.red_b)
                self._exchange()

    def synchronize(self):
        if self.native:
            self.session.synchronize()
        torch.cuda.synchronize(self.device)

    def state(self) -> dict:
        if self.native:
            return self.session.state(0)
        return self.solver.read_state(self._stream())

    def local_w(self) -> np.ndarray:
        """This rank's interior block of w (nx x ny, fp64)."""
        if self.native:
            return self.session.local_w(0)
        return self.solver.download_w(self._stream())

    def profile(self, n: int) -> dict:
        """Per-phase times of n eager iterations (native path), reduced with MAX over ranks and
        mapped onto the reference's 5 stage-4 buckets (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:
        956-980).  Restarts the solver (init) first; values are seconds for the n iterations."""
        if self.native:
            self.session.init()
            ph = self.session.profile(int(n))
            vals = {"compute": ph["t_kernel_a"] + ph["t_kernel_b"], "copy": 0.0, "comm": ph["t_comm"],
                    "precond": 0.0, "dot": ph["t_reduce"]}
        else:
            vals = self._profile_torch(int(n))
        return reduce_max(vals, self.info, self.device)

    def _profile_torch(self, n: int) -> dict:
        """Eager iterations on torch's stream with events between the steps (the torch-comm twin of
        PcgDriver::profile_phases).  With gloo the all-reduce and the ghost exchange include their
        device<->host staging, which lands in the comm bucket."""
        self.init()
        s = self._stream()
        t = {k: 0.0 for k in PHASE_BUCKETS}

        def ev():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e

        marks = []
        for _ in range(n):
            e0 = ev()
            self.solver.enqueue_kernel_a(s)
            e1 = ev()
            self.solver.enqueue_reduce_a(s)
            e2 = ev()
            if self.single_pass:
                self._allreduce(self.red_c)
                e3 = ev()
                self._halo1(s)
                marks.append((e0, e1, e2, e3, ev(), None, None))
            else:
                self._allreduce(self.red_a)
                e3 = ev()
                self.solver.enqueue_kernel_b(s)
                e4 = ev()
                self.solver.enqueue_reduce_b(s)
                e5 = ev()
                self._allreduce(self.red_b)
                self._exchange()
                marks.append((e0, e1, e2, e3, e4, e5, ev()))
        torch.cuda.synchronize(self.device)
        ms = lambda a, b: a.elapsed_time(b) * 1e-3  # noqa: E731
        for m in marks:
            if self.single_pass:
                e0, e1, e2, e3, e4 = m[:5]
                t["compute"] += ms(e0, e1)
                t["dot"] += ms(e1, e2)
                t["comm"] += ms(e2, e3) + ms(e3, e4)
            else:
                e0, e1, e2, e3, e4, e5, e6 = m
                t["compute"] += ms(e0, e1) + ms(e3, e4)
                t["dot"] += ms(e1, e2) + ms(e4, e5)
                t["comm"] += ms(e2, e3) + ms(e5, e6)
        return t

    def solve(self, gather: bool = True, batch: int | None = None) -> Result:
        batch = batch or max(self.graph_batch, 16)
        t0 = time.perf_counter()
        self.init()
        t1 = time.perf_counter()
        launched = 0
        max_iter = self.problem.effective_max_iter()
        while True:
            self.step(batch)
            launched += batch
            st = self.state()
            if st["done"]:
                break
            if launched > max_iter + 2 * batch:
                raise RuntimeError("device stop flag never raised")
        self.synchronize()
        t2 = time.perf_counter()
        res = Result(st["iters"], st["status"], st["diff"], t2 - t1, None, backend=f"hip-{self.comm_kind}",
                     ranks=self.info.world, init_seconds=t1 - t0,
                     extra=dict(launched=launched, nan=st["nan"], algo=self.tile().get("algo")))
        if gather:
            res.w = gather_solution(self.problem, self.sd, self.local_w(), self.info, self.device)
        return res


class SessionRunner:
    """bench.py's runner interface over a single-process native Session (1 GPU, self comm)."""

    def __init__(self, session, problem, info: DistInfo):
        self.s, self.problem, self.info = session, problem, info
        self.graphs = True

    def init(self):
        self.s.init()

    def step(self, n: int):
        self.s.step(int(n))

    def step_eager(self, n: int):
        self.s.step_eager(int(n))

    def synchronize(self):
        self.s.synchronize()

    def state(self) -> dict:
        return self.s.state(0)

    def tile(self) -> dict:
        return self.s.tile

    def prepare(self, n: int) -> bool:
        return bool(self.s.prepare(int(n)))

    def path_stats(self) -> dict:
        return dict(self.s.path_stats())

    def reset_path_stats(self):
        self.s.reset_path_stats()

    @property
    def split_sweep(self) -> bool:
        return bool(self.s.split_sweep)

    def progress(self):
        v = self.s.progress(0)
        return None if v[0] < 0 else tuple(int(x) for x in v)

    def error_norms(self) -> dict:
        return reduce_error_stats(dict(self.s.error_norms()), self.problem, self.info)

    def profile(self, n: int) -> dict:
        self.s.init()
        ph = self.s.profile(int(n))
        return {"compute": ph["t_kernel_a"] + ph["t_kernel_b"], "copy": 0.0, "comm": ph["t_comm"],
                "precond": 0.0, "dot": ph["t_reduce"]}


class TorchRunner:
    """bench.py's runner interface over the plain-PyTorch PCG (CPU dry runs: flow tests)."""

    graphs = False
    split_sweep = False

    def __init__(self, pcg, problem, info: DistInfo):
        self.pcg, self.problem, self.info = pcg, problem, info
        self.path = {"graph_iters": 0, "eager_iters": 0, "graph_lengths": []}

    def init(self):
        self.pcg.init()

    def step(self, n: int):
        self.path["eager_iters"] += int(n)
        self.pcg.step(int(n))

    step_eager = step

    def synchronize(self):
        self.pcg.synchronize()

    def state(self) -> dict:
        return self.pcg.state()

    def tile(self) -> dict:
        return dict(kind="torch-cpu")

    def prepare(self, n: int) -> bool:
        return False

    def path_stats(self) -> dict:
        return dict(self.path)

    def reset_path_stats(self):
        self.path = {"graph_iters": 0, "eager_iters": 0, "graph_lengths": []}

    def progress(self):
        return None

    def error_norms(self) -> dict:
        return reduce_error_stats(self.pcg.local_error_stats(), self.problem, self.info)


def reduce_max(vals: dict, info: DistInfo, device: int = 0) -> dict:
    """MAX over ranks of a dict of floats (MPI_Reduce(MAX), stage4-mpi+cuda/poisson_mpi_cuda_f.cu:963-967)."""
    keys = list(vals)
    if info.world > 1:
        t = torch.tensor([float(vals[k]) for k in keys], dtype=torch.float64, device=_comm_device(info, device))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return {k: float(v) for k, v in zip(keys, t.tolist())}
    return dict(vals)


def reduce_error_stats(local: dict, problem, info: DistInfo, device: int = 0) -> dict:
    """Finish per-rank (sum e^2, max |e|, max w) into l2_error / max_error / max_w over all ranks."""
    if info.world > 1:
        cdev = _comm_device(info, device)
        t = torch.tensor([float(local["sum_e2"])], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        m = torch.tensor([float(local["max_error"]), float(local["max_w"])], dtype=torch.float64, device=cdev)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        sum_e2, max_e, max_w = float(t.item()), float(m[0].item()), float(m[1].item())
    else:
        sum_e2, max_e, max_w = float(local["sum_e2"]), float(local["max_error"]), float(local["max_w"])
    return {"l2_error": float(np.sqrt(sum_e2 * problem.h1 * problem.h2)), "max_error": max_e, "max_w": max_w}


def phase_table(buckets: dict, scale: float = 1.0) -> str:
    """The stage-4 Table 2 lines (reference stdout, stage4-mpi+cuda/poisson_mpi_cuda_f.cu:970-979)."""
    return "\n".join(f"   {PHASE_LABELS[k]} ~ {buckets[k] * scale:.6f} s" for k in PHASE_BUCKETS)


def gather_solution(problem, sd: dict, local: np.ndarray, info: DistInfo, device: int = 0):
    """Assemble the global (M+1)x(N+1) solution on rank 0 (None elsewhere).

    Rank by rank over point-to-point tensors (device tensors for nccl, host for gloo): rank 0 holds
    the global array plus ONE block at a time, and nothing is pickled."""
    if info.rank == 0:
        g = np.zeros((problem.M + 1, problem.N + 1))
        g[sd["i_start"]:sd["i_end"] + 1, sd["j_start"]:sd["j_end"] + 1] = local
    if info.world == 1:
        return g
    cdev = _comm_device(info, device)
    Px, Py = sd["Px"], sd["Py"]
    if info.rank == 0:
        for r in range(1, info.world):
            s = subdomain(problem.M, problem.N, Px, Py, r)
            buf = torch.empty(s["nx"] * s["ny"], dtype=torch.float64, device=cdev)
            dist.recv(buf, src=r)
            g[s["i_start"]:s["i_end"] + 1, s["j_start"]:s["j_end"] + 1] = \
                buf.cpu().numpy().reshape(s["nx"], s["ny"])
            del buf
        return g
    t = torch.from_numpy(np.ascontiguousarray(local, dtype=np.float64).reshape(-1)).to(cdev)
    dist.send(t, dst=0)
    return None
