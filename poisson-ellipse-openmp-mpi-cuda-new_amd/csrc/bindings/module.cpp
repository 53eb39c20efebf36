#include <algorithm>
// Python bindings of the native pmx library (module `_pmx`).
//
// The binding layer is deliberately thin: device buffers are passed as integer pointers and
// streams as integer hipStream_t handles, so the Python side can hand in torch tensors
// (tensor.data_ptr(), torch.cuda.current_stream().cuda_stream) without linking libtorch.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "pmx/common.hpp"
#include "pmx/cpu_pcg.hpp"
#include "pmx/decomp.hpp"
#include "pmx/gpu_solver.hpp"
#include "pmx/kernels.hpp"
#include "pmx/session.hpp"

namespace py = pybind11;
using namespace pmx;

namespace {

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

py::array_t<double> to_numpy(const std::vector<double>& v, std::vector<py::ssize_t> shape) {
  py::array_t<double> a(shape);
  std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(double));
  return a;
}

py::dict sd_dict(const Subdomain& s) {
  py::dict d;
  d["M"] = s.M; d["N"] = s.N; d["Px"] = s.grid.Px; d["Py"] = s.grid.Py;
  d["rank"] = s.rank; d["px"] = s.px; d["py"] = s.py;
  d["i_start"] = s.i_start; d["i_end"] = s.i_end; d["j_start"] = s.j_start; d["j_end"] = s.j_end;
  d["nx"] = s.nx; d["ny"] = s.ny;
  d["nb_xlo"] = s.nb_xlo; d["nb_xhi"] = s.nb_xhi; d["nb_ylo"] = s.nb_ylo; d["nb_yhi"] = s.nb_yhi;
  d["aspect"] = s.aspect();
  return d;
}

py::dict result_dict(const SolveResult& r, const ProblemSpec& s, bool with_w) {
  py::dict d;
  d["iters"] = r.iters;
  d["status"] = std::string(status_name(r.status));
  d["diff"] = r.last_diff;
  d["seconds"] = r.seconds;
  if (with_w && !r.w.empty()) d["w"] = to_numpy(r.w, {s.M + 1, s.N + 1});
  return d;
}

py::dict state_dict(const PcgState& st) {
  py::dict d;
  d["red_a"] = st.red_a[0];
  d["red_b"] = py::make_tuple(st.red_b[0], st.red_b[1]);
  d["zr"] = py::make_tuple(st.zr[0], st.zr[1]);
  d["diff"] = st.diff;
  d["it"] = st.it;
  d["iters"] = st.iters;
  d["done"] = bool(st.done);
  d["status"] = std::string(status_name(Status(st.status)));
  d["nan"] = bool(st.nan_flag);
  d["w_pend"] = st.w_pend;
  d["w_pend_n"] = st.w_pend_n;
  d["w_cycle"] = st.w_cycle;
  d["red_c"] = py::make_tuple(st.red_c[0], st.red_c[1], st.red_c[2], st.red_c[3], st.red_c[4]);
  d["alpha1"] = py::make_tuple(st.alpha1[0], st.alpha1[1], st.alpha1[2], st.alpha1[3]);
  d["beta1"] = py::make_tuple(st.beta1[0], st.beta1[1], st.beta1[2], st.beta1[3]);
  d["halo_k"] = st.halo_k;
  return d;
}

py::dict error_dict(const ErrorStats& e) {
  py::dict d;
  d["sum_e2"] = e.sum_e2;
  d["max_error"] = e.max_e;
  d["max_w"] = e.max_w;
  return d;
}

py::dict stats_dict(const RunStats& r) {
  py::dict d;
  d["iters"] = r.iters;
  d["status"] = std::string(status_name(r.status));
  d["diff"] = r.diff;
  d["init_seconds"] = r.init_seconds;
  d["solve_seconds"] = r.solve_seconds;
  d["launched"] = r.launched;
  d["nan"] = r.nan;
  d["t_kernel_a"] = r.t_kernel_a;
  d["t_kernel_b"] = r.t_kernel_b;
  d["t_comm"] = r.t_comm;
  d["t_reduce"] = r.t_reduce;
  d["t_allreduce"] = r.t_allreduce;
  d["t_halo"] = r.t_halo;
  return d;
}

py::dict layout_dict(const CommLayout& L) {
  py::dict d;
  py::list so, ro, el, pe;
  for (int s = 0; s < kHaloSlots; ++s) {
    so.append(L.send_off[s]);
    ro.append(L.recv_off[s]);
    el.append(L.edge_len[s]);
    pe.append(L.peer[s]);
  }
  d["state_off"] = L.state_off;
  d["send_off"] = py::tuple(so);
  d["recv_off"] = py::tuple(ro);
  d["edge_len"] = py::tuple(el);
  d["peer"] = py::tuple(pe);  // rank across each slot (-1: none); slot s pairs with opposite_slot(s)
  d["opposite"] = py::make_tuple(opposite_slot(0), opposite_slot(1), opposite_slot(2), opposite_slot(3),
                                 opposite_slot(4), opposite_slot(5), opposite_slot(6), opposite_slot(7));
  d["elem"] = L.elem;
  d["bytes"] = L.bytes;
  d["single_pass"] = L.single_pass;
  d["algo"] = L.single_pass ? "pcg1" : "pcg2";
  d["state_bytes"] = sizeof(PcgState);
  d["red_a_off"] = offsetof(PcgState, red_a);
  d["red_b_off"] = offsetof(PcgState, red_b);
  d["red_c_off"] = offsetof(PcgState, red_c);
  return d;
}

// Raw-pointer ops on caller-owned buffers (torch tensors of shape (nx+2, pitch)).
class OpContext {
 public:
  OpContext(const ProblemSpec& spec, int Px, int Py, int rank, int64_t pitch, int device)
      : spec_(spec), device_(device) {
    spec_.validate();
    HIP_CHECK(hipSetDevice(device));
    sd_ = decompose_2d(spec.M, spec.N, ProcGrid{Px, Py}, rank);
    PMX_CHECK(pitch >= sd_.ny + 2, "pitch " << pitch << " < ny+2 = " << sd_.ny + 2);
    geom_ = make_dev_geom(spec_, sd_, pitch);
    tables_ = upload_tables(spec_, &buf_);
    HIP_CHECK(hipMalloc(&partials_, 4096 * sizeof(double)));
  }
  ~OpContext() {
    (void)hipSetDevice(device_);
    if (buf_) (void)hipFree(buf_);
    if (partials_) (void)hipFree(partials_);
  }
  py::dict subdomain() const { return sd_dict(sd_); }
  void assemble(uintptr_t a, uintptr_t b, uintptr_t B, uintptr_t s) {
    HIP_CHECK(hipSetDevice(device_));
    launch_assemble(geom_, tables_, (double*)a, (double*)b, (double*)B, geom_.pitch, as_stream(s));
  }
  void apply_a(uintptr_t p, uintptr_t Ap, bool fp32, bool exact, uintptr_t s) {
    HIP_CHECK(hipSetDevice(device_));
    if (fp32) launch_apply_a<float>(geom_, tables_, (const float*)p, (float*)Ap, exact, as_stream(s));
    else launch_apply_a<double>(geom_, tables_, (const double*)p, (double*)Ap, exact, as_stream(s));
  }
  void precond(uintptr_t r, uintptr_t z, bool fp32, bool exact, uintptr_t s) {
    HIP_CHECK(hipSetDevice(device_));
    if (fp32) launch_precond<float>(geom_, tables_, (const float*)r, (float*)z, exact, as_stream(s));
    else launch_precond<double>(geom_, tables_, (const double*)r, (double*)z, exact, as_stream(s));
  }
  double dot(uintptr_t x, uintptr_t y, bool fp32, uintptr_t s) {
    HIP_CHECK(hipSetDevice(device_));
    const hipStream_t st = as_stream(s);
    const int nb = fp32 ? launch_dot_partials<float>(geom_, (const float*)x, (const float*)y, partials_, 4096, st)
                        : launch_dot_partials<double>(geom_, (const double*)x, (const double*)y, partials_, 4096, st);
    std::vector<double> h(nb);
    HIP_CHECK(hipMemcpyAsync(h.data(), partials_, nb * sizeof(double), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    double sum = 0.0;
    for (double v : h) sum += v;
    return sum;
  }

 private:
  ProblemSpec spec_;
  int device_;
  Subdomain sd_;
  DevGeom geom_{};
  DevTables tables_{};
  double* buf_ = nullptr;
  double* partials_ = nullptr;
};

GpuOptions make_options(int device, const std::string& kernel, int block, int vec, int waves,
                        int tile_rows, const std::string& dtype, bool exact, int graph_batch, bool check,
                        bool overlap = true, int vec_b = 0, int waves_b = 0, int tile_rows_b = -1,
                        bool poison_halos = false, bool b_ring = false, int algo = -1, int placement = 0,
                        double placement_budget_s = 0.5, double placement_keep_free = 0.5, int block1 = -1,
                        int ca_s = 3) {
  GpuOptions o;
  o.ca_s = ca_s;
  o.block1 = block1;
  o.placement = placement;
  o.placement_budget_s = placement_budget_s;
  o.placement_keep_free = placement_keep_free;
  o.algo = algo;
  o.device = device;
  PMX_CHECK(kernel == "wave", "kernel must be wave (the round-1 lds kernels are retired, bench/RETIRED.md), got " << kernel);
  o.kernel = 1;
  o.vec = vec;
  o.waves = waves;
  o.block = block;
  o.tile_rows = tile_rows;
  PMX_CHECK(dtype == "fp64" || dtype == "fp32" || dtype == "mixed",
            "dtype must be fp64, fp32 (fp32 storage and stencil arithmetic) or mixed (fp32 storage, fp64 "
            "arithmetic), got " << dtype);
  o.dtype = dtype == "fp64" ? DType::kFp64 : DType::kFp32;
  o.arith32 = dtype == "fp32" ? 1 : 0;
  o.exact = exact;
  o.graph_batch = graph_batch;
  o.check = check;
  o.overlap = overlap;
  o.vec_b = vec_b;
  o.waves_b = waves_b;
  o.tile_rows_b = tile_rows_b;
  o.poison_halos = poison_halos;
  o.b_ring = b_ring ? 1 : 0;
  return o;
}

}  // namespace

PYBIND11_MODULE(_pmx, m) {
  m.doc() = "pmx: MI355X-native fictitious-domain Poisson PCG (native core)";
  // module-local types: a second copy of the package (an older build, bench/ab_env.py --pkg) can be
  // imported into the same process for same-box binary A/B runs
  py::register_exception<pmx::Error>(m, "PmxError", PyExc_RuntimeError);

  py::enum_<Norm>(m, "Norm", py::module_local()).value("weighted", Norm::kWeighted).value("unweighted", Norm::kUnweighted);
  py::enum_<Split>(m, "Split", py::module_local())
      .value("reference", Split::kReference).value("auto", Split::kAuto)
      .value("rows", Split::kRows).value("cols", Split::kCols);

  py::class_<ProblemSpec>(m, "ProblemSpec", py::module_local())
      .def(py::init<>())
      .def_readwrite("M", &ProblemSpec::M).def_readwrite("N", &ProblemSpec::N)
      .def_readwrite("A1", &ProblemSpec::A1).def_readwrite("B1", &ProblemSpec::B1)
      .def_readwrite("A2", &ProblemSpec::A2).def_readwrite("B2", &ProblemSpec::B2)
      .def_readwrite("ax", &ProblemSpec::ax).def_readwrite("by", &ProblemSpec::by)
      .def_readwrite("F", &ProblemSpec::F).def_readwrite("delta", &ProblemSpec::delta)
      .def_readwrite("breakdown_tol", &ProblemSpec::breakdown_tol)
      .def_readwrite("max_iter", &ProblemSpec::max_iter).def_readwrite("norm", &ProblemSpec::norm)
      .def("effective_max_iter", &ProblemSpec::effective_max_iter)
      .def("validate", &ProblemSpec::validate);

  m.def("grid_info", [](const ProblemSpec& s) {
    const GridInfo g(s);
    py::dict d;
    d["h1"] = g.h1; d["h2"] = g.h2; d["eps"] = g.eps; d["inv_eps"] = g.inv_eps; d["h1h2"] = g.h1h2;
    return d;
  });
  m.def("face_tables", [](const ProblemSpec& s) {
    const GridInfo g(s);
    const geo::FaceTables t(s, g);
    py::dict d;
    auto arr = [](const std::vector<double>& v) { return to_numpy(v, {py::ssize_t(v.size())}); };
    d["rv"] = arr(t.rv); d["xlo"] = arr(t.xlo); d["xhi"] = arr(t.xhi); d["x"] = arr(t.x);
    d["rh"] = arr(t.rh); d["ylo"] = arr(t.ylo); d["yhi"] = arr(t.yhi); d["y"] = arr(t.y);
    return d;
  });

  // ---- decomposition ----
  m.def("choose_process_grid", [](int size) {
    const ProcGrid g = choose_process_grid(size);
    return py::make_tuple(g.Px, g.Py);
  });
  m.def("make_process_grid", [](int size, int M, int N, Split split) {
    const ProcGrid g = make_process_grid(size, M, N, split);
    return py::make_tuple(g.Px, g.Py);
  });
  m.def("decompose_2d", [](int M, int N, int Px, int Py, int rank) {
    return sd_dict(decompose_2d(M, N, ProcGrid{Px, Py}, rank));
  });

  // ---- CPU oracle ----
  m.def("cpu_solve", [](const ProblemSpec& s, int threads, bool keep) {
          SolveResult r;
          { py::gil_scoped_release nogil; r = cpu_solve(s, threads, keep); }
          return result_dict(r, s, keep);
        }, py::arg("spec"), py::arg("threads") = 1, py::arg("keep_solution") = true);
  m.def("cpu_solve_decomposed", [](const ProblemSpec& s, int nranks, Split split, int threads, bool keep) {
          SolveResult r;
          { py::gil_scoped_release nogil; r = cpu_solve_decomposed(s, nranks, split, threads, keep); }
          return result_dict(r, s, keep);
        }, py::arg("spec"), py::arg("nranks"), py::arg("split") = Split::kReference,
        py::arg("threads") = 1, py::arg("keep_solution") = true);
  m.def("cpu_assemble", [](const ProblemSpec& s) {
    std::vector<double> a, b, B;
    cpu_assemble(s, a, b, B);
    return py::make_tuple(to_numpy(a, {s.M + 2, s.N + 2}), to_numpy(b, {s.M + 2, s.N + 2}),
                          to_numpy(B, {s.M + 1, s.N + 1}));
  });

  // ---- GPU ----
  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return 0; }
    return n;
  });
  m.def("mfma_wave_sums", [](uintptr_t x, uintptr_t out, int nwaves, bool fp32, uintptr_t stream) {
    if (fp32) launch_wave_sums<float>(reinterpret_cast<const float*>(x), reinterpret_cast<float*>(out), nwaves, as_stream(stream));
    else launch_wave_sums<double>(reinterpret_cast<const double*>(x), reinterpret_cast<double*>(out), nwaves, as_stream(stream));
  }, py::arg("x"), py::arg("out"), py::arg("nwaves"), py::arg("fp32") = false, py::arg("stream") = 0);
  // Reduction hand-off stress (tests): `nsets` back-to-back launches of the multi-block ticketed
  // reduction on ONE workspace (as a solver does), set j reducing parts[j] (n x nq interleaved
  // doubles) into out[j * nq ..]; nq = 5: k_reduce_n (pcg1), nq = 1 or 2: k_reduce (pcg2).
  m.def("reduce_stress", [](uintptr_t parts, int n, int nq, int nsets, uintptr_t out, uintptr_t stream) {
    PMX_CHECK(nq == 1 || nq == 2 || nq == 5, "nq must be 1, 2 or 5");
    hipStream_t s = as_stream(stream);
    double* ws = nullptr;
    PcgState* st = nullptr;
    HIP_CHECK(hipMalloc(&ws, kReduceWsDoubles * sizeof(double)));
    HIP_CHECK(hipMalloc(&st, sizeof(PcgState)));
    HIP_CHECK(hipMemsetAsync(ws, 0, kReduceWsDoubles * sizeof(double), s));
    HIP_CHECK(hipMemsetAsync(st, 0, sizeof(PcgState), s));
    const double ones[5] = {1.0, 1.0, 1.0, 1.0, 1.0};
    const double* P = reinterpret_cast<const double*>(parts);
    double* O = reinterpret_cast<double*>(out);
    for (int j = 0; j < nsets; ++j) {
      if (nq == 5)
        launch_reduce_n(P + size_t(j) * n * nq, n, nq, ones, O + size_t(j) * nq, st, 0, ws, s);
      else
        launch_reduce(P + size_t(j) * n * nq, n, nq, 1.0, 1.0, O + size_t(j) * nq, st, 0, ws, s);
    }
    HIP_CHECK(hipStreamSynchronize(s));
    HIP_CHECK(hipFree(ws));
    HIP_CHECK(hipFree(st));
  }, py::arg("parts"), py::arg("n"), py::arg("nq"), py::arg("nsets"), py::arg("out"), py::arg("stream") = 0);
  m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
  // Arena layout for a Python-orchestrated solver (DistGpuPCG comm="torch").  The iteration
  // algorithm is resolved exactly as the solver will (options + environment + device size), so
  // pass the returned "algo" on to SubdomainSolver(algo=...).
  m.def("comm_layout", [](const ProblemSpec& s, int Px, int Py, int rank, const std::string& dtype,
                          const std::string& kernel, bool exact, int device, int algo, int sharing) {
          GpuOptions o = make_options(device, kernel, 256, 0, 4, 0, dtype, exact, 0, false);
          o.algo = algo;
          o = resolve_options(o);
          double total = 0.0;
          if (o.algo == -1) {
            HIP_CHECK(hipSetDevice(device));
            size_t fb = 0, tb = 0;
            HIP_CHECK(hipMemGetInfo(&fb, &tb));
            total = double(tb);
          }
          const ProcGrid g{Px, Py};
          const bool sp = choose_single_pass(s, g, o, total, std::max(1, sharing));
          const Subdomain sd = decompose_2d(s.M, s.N, g, rank);
          return layout_dict(GpuSubdomainSolver::comm_layout(sd, o.dtype, sp));
        }, py::arg("spec"), py::arg("Px"), py::arg("Py"), py::arg("rank"), py::arg("dtype") = "fp64",
        py::arg("kernel") = "wave", py::arg("exact") = false, py::arg("device") = 0, py::arg("algo") = -1,
        py::arg("sharing") = 1);
  m.def("record_comm_sequence", [](const ProblemSpec& s, int world, Split split, int graph_batch, int64_t iters,
                                   const std::string& dtype, int device, bool overlap, int algo, int ca_s) {
          GpuOptions o = make_options(device, "wave", 256, 0, 4, 0, dtype, false, graph_batch, false, overlap);
          o.algo = algo;
          o.ca_s = ca_s;
          std::vector<std::vector<CommEvent>> logs;
          {
            py::gil_scoped_release nogil;
            HIP_CHECK(hipSetDevice(device));
            logs = record_comm_sequence(s, world, split, o, iters);
          }
          py::list out;
          for (auto& l : logs) {
            py::list r;
            for (auto& e : l) r.append(py::make_tuple(e.comm, e.op, e.count, e.peer, e.stream));
            out.append(r);
          }
          return out;
        }, py::arg("spec"), py::arg("world"), py::arg("split") = Split::kAuto, py::arg("graph_batch") = 4,
        py::arg("iters") = 8, py::arg("dtype") = "fp64", py::arg("device") = 0, py::arg("overlap") = true,
        py::arg("algo") = -1, py::arg("ca_s") = 3,
        "every rank's communication calls on a recording comm (init + iters iterations, captured when "
        "graph_batch > 0): (comm, op, count, peer, stream) tuples");
  m.def("max_square_grid", [](double bytes_per_gpu, int gpus, const std::string& dtype, double reserve, int algo) {
    return max_square_grid(bytes_per_gpu, gpus, dtype == "fp64" ? DType::kFp64 : DType::kFp32, reserve, algo);
  }, py::arg("bytes_per_gpu"), py::arg("gpus"), py::arg("dtype") = "fp64", py::arg("reserve") = 0.1,
     py::arg("algo") = -1);
  // the iteration algorithm a Session would pick (choose_algo), without building one: 1 pcg1, 2 pcg2,
  // 3 the s-step PCG.  device_bytes = 0 skips the memory test.
  m.def("choose_algo", [](const ProblemSpec& s, int world, Split split, const std::string& dtype, double device_bytes,
                          int per_device, int algo, bool exact) {
    GpuOptions o = make_options(0, "wave", 256, 0, 4, 0, dtype, exact, 32, false);
    o.algo = algo;
    o = resolve_options(o);
    return choose_algo(s, make_process_grid(world, s.M, s.N, split), o, device_bytes, std::max(1, per_device), true);
  }, py::arg("spec"), py::arg("world") = 1, py::arg("split") = Split::kAuto, py::arg("dtype") = "fp64",
     py::arg("device_bytes") = 0.0, py::arg("per_device") = 1, py::arg("algo") = -1, py::arg("exact") = false);
  m.def("estimate_device_bytes", [](const ProblemSpec& s, int world, Split split, int rank, const std::string& dtype,
                                    int algo) {
    const Subdomain sd = decompose_2d(s.M, s.N, make_process_grid(world, s.M, s.N, split), rank);
    return GpuSubdomainSolver::estimate_device_bytes_algo(s, sd, dtype == "fp64" ? DType::kFp64 : DType::kFp32, algo);
  }, py::arg("spec"), py::arg("world") = 1, py::arg("split") = Split::kAuto, py::arg("rank") = 0,
     py::arg("dtype") = "fp64", py::arg("algo") = 1);

  py::class_<OpContext>(m, "OpContext", py::module_local())
      .def(py::init<const ProblemSpec&, int, int, int, int64_t, int>(), py::arg("spec"),
           py::arg("Px"), py::arg("Py"), py::arg("rank"), py::arg("pitch"), py::arg("device") = 0)
      .def("subdomain", &OpContext::subdomain)
      .def("assemble", &OpContext::assemble)
      .def("apply_a", &OpContext::apply_a)
      .def("precond", &OpContext::precond)
      .def("dot", &OpContext::dot);

  // Single subdomain solver on caller-chosen streams/arena (Python-orchestrated comm path).
  py::class_<GpuSubdomainSolver>(m, "SubdomainSolver", py::module_local())
      .def(py::init([](const ProblemSpec& s, int Px, int Py, int rank, int device,
                       const std::string& kernel, int block, int vec, int waves, int tile_rows,
                       const std::string& dtype, bool exact, uintptr_t arena, bool check, int vec_b,
                       int waves_b, int tile_rows_b, bool b_ring, int algo) {
             const Subdomain sd = decompose_2d(s.M, s.N, ProcGrid{Px, Py}, rank);
             return std::make_unique<GpuSubdomainSolver>(
                 s, sd, make_options(device, kernel, block, vec, waves, tile_rows, dtype, exact, 0, check,
                                     true, vec_b, waves_b, tile_rows_b, false, b_ring, algo),
                 arena);
           }),
           py::arg("spec"), py::arg("Px") = 1, py::arg("Py") = 1, py::arg("rank") = 0,
           py::arg("device") = 0, py::arg("kernel") = "wave", py::arg("block") = 256,
           py::arg("vec") = 0, py::arg("waves") = 4, py::arg("tile_rows") = 0,
           py::arg("dtype") = "fp64", py::arg("exact") = false, py::arg("arena") = 0,
           py::arg("check") = false, py::arg("vec_b") = 0, py::arg("waves_b") = 0,
           py::arg("tile_rows_b") = -1, py::arg("b_ring") = false, py::arg("algo") = -1)
      .def("enqueue_init", [](GpuSubdomainSolver& g, uintptr_t s) { g.enqueue_init(as_stream(s)); })
      // pcg1: the exchange's target sweep (its buffer parity); default: the sweep the host enqueues
      // next (host_k, bumped by each reduction) -- what PcgDriver passes
      .def("enqueue_halo_pack",
           [](GpuSubdomainSolver& g, uintptr_t s, long long target) {
             g.set_halo_target(target < 0 ? g.host_k() : target);
             g.enqueue_halo_pack(as_stream(s));
           },
           py::arg("stream"), py::arg("target") = -1)
      .def("enqueue_halo_unpack",
           [](GpuSubdomainSolver& g, uintptr_t s, long long target) {
             g.set_halo_target(target < 0 ? g.host_k() : target);
             g.enqueue_halo_unpack(as_stream(s));
           },
           py::arg("stream"), py::arg("target") = -1)
      .def_property_readonly("single_pass", &GpuSubdomainSolver::single_pass)
      .def("enqueue_phase_a", [](GpuSubdomainSolver& g, uintptr_t s) { g.enqueue_phase_a(as_stream(s)); })
      .def("enqueue_kernel_a", [](GpuSubdomainSolver& g, uintptr_t s) { g.enqueue_kernel_a(as_stream(s)); })
      .def("enqueue_reduce_a", [](GpuSubdomainSolver& g, uintptr_t s) { g.enqueue_reduce_a(as_stream(s)); })
      .def("enqueue_kernel_b", [](GpuSubdomainSolver& g, uintptr_t s) { g.enqueue_kernel_b(as_stream(s), true); })
      .def("enqueue_reduce_b", [](GpuSubdomainSolver& g, uintptr_t s) { g.enqueue_reduce_b(as_stream(s)); })
      .def("enqueue_phase_b", [](GpuSubdomainSolver& g, uintptr_t s, bool pack) {
             g.enqueue_phase_b(as_stream(s), pack);
           }, py::arg("stream"), py::arg("pack") = true)
      .def("enqueue_pack", [](GpuSubdomainSolver& g, uintptr_t s) { g.enqueue_pack(as_stream(s)); })
      .def("enqueue_poison_recv", [](GpuSubdomainSolver& g, uintptr_t s) { g.enqueue_poison_recv(as_stream(s)); })
      .def("read_state", [](GpuSubdomainSolver& g, uintptr_t s) { return state_dict(g.read_state(as_stream(s))); })
      .def("download_w", [](GpuSubdomainSolver& g, uintptr_t s) {
        return to_numpy(g.download_w(as_stream(s)), {g.sd().nx, g.sd().ny});
      })
      .def("download_field", [](GpuSubdomainSolver& g, int which, uintptr_t s) {
        return to_numpy(g.download_field(which, as_stream(s)), {g.sd().nx + 2, g.sd().ny + 2});
      })
      .def("error_norms", [](GpuSubdomainSolver& g, uintptr_t s) {
        ErrorStats e;
        { py::gil_scoped_release nogil; e = g.error_norms(as_stream(s)); }
        return error_dict(e);
      })
      .def("layout", [](GpuSubdomainSolver& g) { return layout_dict(g.layout()); })
      .def("subdomain", [](GpuSubdomainSolver& g) { return sd_dict(g.sd()); })
      .def_property_readonly("arena_ptr", &GpuSubdomainSolver::arena_ptr)
      .def_property_readonly("device_bytes", &GpuSubdomainSolver::device_bytes)
      .def_property_readonly("ntiles", [](GpuSubdomainSolver& g) { return g.tiles().ntiles(); });

  py::class_<Session>(m, "Session", py::module_local())
      .def(py::init([](const ProblemSpec& s, int world, const std::string& comm, Split split,
                       int device, const std::string& kernel, int block, int vec, int waves,
                       int tile_rows, const std::string& dtype, bool exact, int graph_batch,
                       bool check, py::object uid, std::vector<int> ranks, std::vector<int> devices,
                       bool rccl_graph, bool overlap, int vec_b, int waves_b, int tile_rows_b,
                       bool poison_halos, bool b_ring, int algo, bool defer_connect, int threaded,
                       int placement, double placement_budget_s, double placement_keep_free, int sharing,
                       int block_tiles, int ca_s, int split_sweep) {
             SessionConfig c;
             c.sharing = sharing;
             c.spec = s;
             c.opt = make_options(device, kernel, block, vec, waves, tile_rows, dtype, exact,
                                  graph_batch, check, overlap, vec_b, waves_b, tile_rows_b, poison_halos,
                                  b_ring, algo, placement, placement_budget_s, placement_keep_free,
                                  block_tiles, ca_s);
             c.opt.split_sweep = split_sweep;
             c.defer_connect = defer_connect;
             c.threaded = threaded;
             c.split = split;
             c.world = world;
             if (comm == "self") c.comm = CommKind::kSelf;
             else if (comm == "local") c.comm = CommKind::kLocal;
             else if (comm == "rccl") c.comm = CommKind::kRccl;
             else if (comm == "ipc") c.comm = CommKind::kIpc;
             else if (comm == "loopback") c.comm = CommKind::kLoopback;
             else PMX_CHECK(false, "unknown comm " << comm);
             if (!uid.is_none()) c.rccl_uid = uid.cast<std::string>();
             c.ranks = ranks;
             c.devices = devices;
             c.rccl_graph = rccl_graph;
             py::gil_scoped_release nogil;
             return std::make_unique<Session>(c);
           }),
           py::arg("spec"), py::arg("world") = 1, py::arg("comm") = "self",
           py::arg("split") = Split::kReference, py::arg("device") = 0, py::arg("kernel") = "wave",
           py::arg("block") = 256, py::arg("vec") = 0, py::arg("waves") = 4,
           py::arg("tile_rows") = 0, py::arg("dtype") = "fp64", py::arg("exact") = false,
           py::arg("graph_batch") = 32, py::arg("check") = false, py::arg("uid") = py::none(),
           py::arg("ranks") = std::vector<int>{}, py::arg("devices") = std::vector<int>{},
           py::arg("rccl_graph") = false, py::arg("overlap") = true, py::arg("vec_b") = 0,
           py::arg("waves_b") = 0, py::arg("tile_rows_b") = -1, py::arg("poison_halos") = false,
           py::arg("b_ring") = false, py::arg("algo") = -1, py::arg("defer_connect") = false,
           py::arg("threaded") = -1, py::arg("placement") = 0, py::arg("placement_budget_s") = 0.5,
           py::arg("placement_keep_free") = 0.5, py::arg("sharing") = 0, py::arg("block_tiles") = -1,
           py::arg("ca_s") = 3, py::arg("split_sweep") = -1)
      .def("ca_probe",
           [](Session& s, int i, py::array_t<double, py::array::c_style | py::array::forcecast> z,
              py::array_t<double, py::array::c_style | py::array::forcecast> p,
              py::array_t<double, py::array::c_style | py::array::forcecast> w,
              py::array_t<double, py::array::c_style | py::array::forcecast> coef,
              py::array_t<double, py::array::c_style | py::array::forcecast> pa, bool fused) {
             auto vec = [](const py::array_t<double, py::array::c_style | py::array::forcecast>& a) {
               return std::vector<double>(a.data(), a.data() + a.size());
             };
             GpuSubdomainSolver& g = s.solver(i);
             GpuSubdomainSolver::CaProbe r;
             {
               const auto vz = vec(z), vp = vec(p), vw = vec(w), vc = vec(coef), va = vec(pa);
               py::gil_scoped_release nogil;
               r = g.ca_probe(vz, vp, vw, vc, va, fused, s.stream_of(i));
             }
             const py::ssize_t nx = g.sd().nx, ny = g.sd().ny;
             py::dict d;
             d["gram"] = to_numpy(r.gram, {py::ssize_t(r.gram.size())});
             d["norms"] = to_numpy(r.norms, {py::ssize_t(r.norms.size())});
             d["p"] = to_numpy(r.p, {nx, ny});
             d["z"] = to_numpy(r.z, {nx, ny});
             d["w"] = to_numpy(r.w, {nx, ny});
             return d;
           },
           py::arg("i"), py::arg("z"), py::arg("p"), py::arg("w"), py::arg("coef"), py::arg("pa"),
           py::arg("fused") = false,
           "s-step kernel probe (tests): one pass 1 + pass 2 (or the fused pass) on the given fields")
      .def("ca_ghost_rows", [](Session& s, int i) { return s.solver(i).ca_ghost_rows(); }, py::arg("i") = 0)
      .def("ipc_export", [](Session& s) { return py::bytes(s.ipc_export()); },
           "IPC session: this rank's memory handles (pass every rank's to connect_ipc)")
      .def("connect_ipc", [](Session& s, std::vector<py::bytes> ex) {
             std::vector<std::string> v;
             for (auto& b : ex) v.push_back(std::string(b));
             s.set_ipc_exports(v);
             py::gil_scoped_release g;
             s.connect();
           })
      .def("connect", [](Session& s) { py::gil_scoped_release g; s.connect(); },
           "create the communicator and driver (sessions built with defer_connect=True)")
      .def_property_readonly("connected", &Session::connected)
      .def_property_readonly("threaded", &Session::threaded)
      .def("local_w", [](Session& s, int i) {
             std::vector<double> w;
             { py::gil_scoped_release g; w = s.local_w(i); }
             return to_numpy(w, {s.solver(i).sd().nx, s.solver(i).sd().ny});
           }, py::arg("i") = 0)
      .def("partials", [](Session& s, int i) {
             std::vector<double> v;
             { py::gil_scoped_release g; v = s.partials(i); }
             return to_numpy(v, {py::ssize_t(v.size() / 5), 5});
           }, py::arg("i") = 0, "per-tile partial sums of the last sweep (tests of the reduction hand-off)")
      .def("init", [](Session& s) { py::gil_scoped_release g; s.init(); })
      .def("step", [](Session& s, int64_t n) { py::gil_scoped_release g; s.step(n); })
      .def("synchronize", [](Session& s) { py::gil_scoped_release g; s.synchronize(); })
      .def("solve", [](Session& s, int poll) {
             RunStats r;
             { py::gil_scoped_release g; r = s.solve(poll); }
             return stats_dict(r);
           }, py::arg("poll_batches") = 1)
      .def("solve_checkpointed", [](Session& s, const std::string& path, int64_t every, bool resume,
                                    int poll) {
             RunStats r;
             { py::gil_scoped_release g; r = s.solve_checkpointed(path, every, resume ? path : "", poll); }
             return stats_dict(r);
           }, py::arg("path"), py::arg("every") = 0, py::arg("resume") = false,
           py::arg("poll_batches") = 1)
      .def("save_checkpoint", [](Session& s, const std::string& path) {
             py::gil_scoped_release g;
             s.save_checkpoint(path);
           })
      .def("load_checkpoint", [](Session& s, const std::string& path) {
             py::gil_scoped_release g;
             s.load_checkpoint(path);
           })
      .def("profile", [](Session& s, int64_t n) {
             RunStats r;
             { py::gil_scoped_release g; r = s.profile(n); }
             return stats_dict(r);
           })
      .def("state", [](Session& s, int i) {
             PcgState st;
             { py::gil_scoped_release g; st = s.state(i); }  // blocks on the device: a watchdog thread must run
             return state_dict(st);
           }, py::arg("i") = 0)
      .def("prepare", [](Session& s, int64_t n) { py::gil_scoped_release g; return s.prepare(n); },
           "capture every graph step(n) would replay now (no execution); False if graphs are off")
      .def("step_eager", [](Session& s, int64_t n) { py::gil_scoped_release g; s.step_eager(n); })
      .def("path_stats", [](Session& s) {
             const PcgDriver::PathStats p = s.path_stats();
             py::dict d;
             d["graph_iters"] = p.graph_iters;
             d["eager_iters"] = p.eager_iters;
             d["graph_lengths"] = p.graph_lengths;
             return d;
           })
      .def("reset_path_stats", &Session::reset_path_stats)
      .def_property_readonly("split_sweep", &Session::split_sweep)
      .def_property_readonly("direct_rows", &Session::direct_rows)
      .def("progress", [](Session& s, int i) {
             long long v[3];
             s.progress(i, v);  // host memory only: callable while another thread blocks in the session
             return py::make_tuple(v[0], v[1], v[2]);
           }, py::arg("i") = 0)
      .def("error_norms", [](Session& s) {
             ErrorStats e;
             { py::gil_scoped_release g; e = s.error_norms(); }
             return error_dict(e);
           })
      .def("bench_kernel", [](Session& s, int which, int abl, int reps) {
             py::gil_scoped_release g;
             s.synchronize();
             return s.solver(0).bench_kernel(which, abl, reps, nullptr);
           }, py::arg("which"), py::arg("abl") = 0, py::arg("reps") = 20,
           "time k_pcg_a (0) / k_pcg_b (1) alone; invalidates the solver state")
      .def("gather_local_w", [](Session& s) {
             const auto& sp = s.solver(0).spec();
             return to_numpy(s.gather_local_w(), {sp.M + 1, sp.N + 1});
           })
      .def("subdomain", [](Session& s, int i) { return sd_dict(s.solver(i).sd()); }, py::arg("i") = 0)
      .def_property_readonly("num_local", &Session::num_local)
      .def_property_readonly("comm_name", &Session::comm_name)
      .def_property_readonly("overlapped", [](Session& s) { return s.overlapped(); })
      .def_property_readonly("poisoned", [](Session& s) { return s.poisoned(); })
      .def_property_readonly("device_bytes", &Session::device_bytes)
      .def_property_readonly("grid", [](Session& s) { return py::make_tuple(s.grid().Px, s.grid().Py); })
      .def_property_readonly("ntiles", [](Session& s) {
        return s.solver(0).ca() ? s.solver(0).ca_tiles().ntiles() : s.solver(0).tiles().ntiles();
      })
      .def_property_readonly("tile", [](Session& s) {
        auto one = [](const TileCfg& t) {
          py::dict d;
          d["kind"] = t.kind == 0 ? "lds" : t.kind == 1 ? "wave" : t.kind == 2 ? "wave-rows" : "pcg1";
          d["block"] = t.block; d["rows"] = t.rows;
          d["vec"] = t.vec; d["waves"] = t.waves; d["tiles_i"] = t.tiles_i; d["tiles_j"] = t.tiles_j;
          if (t.kind == 3) d["pf"] = t.pf;
          if (t.kind == 3 && t.dpf) d["dpf"] = t.dpf;
          if (t.kind == 3 && t.lds_pad) d["lds_pad"] = t.lds_pad;
          return d;
        };
        py::dict d = one(s.solver(0).tiles());
        if (s.solver(0).block_tiles()) d["block_tiles"] = true;
        if (s.solver(0).ca()) {  // s-step PCG: its own wave tiles
          const CaTiles& c = s.solver(0).ca_tiles();
          d = py::dict();
          d["kind"] = "ca";
          d["s"] = c.s;
          d["block"] = c.wo;
          d["rows"] = c.rows;
          d["rows_upd"] = c.rows2;
          d["vec"] = 2;
          d["waves"] = 1;
          d["tiles_i"] = c.tiles_i;
          d["tiles_j"] = c.tiles_j;
          d["algo"] = "ca";
          d["fused"] = c.fuse != 0;
          if (c.fuse) {  // the fused pass's own tiling (k_ca_fused: two-wave workgroups)
            d["rows_fused"] = c.rows_f;
            d["block_fused"] = c.wo_f;
            d["tiles_fused"] = c.ntilesf();
          }
        } else {
          if (!s.solver(0).single_pass()) d["b"] = one(s.solver(0).tiles_b());
          d["algo"] = s.solver(0).single_pass() ? "pcg1" : "pcg2";
        }
        if (!s.solver(0).placement_ms().empty()) {
          // real iterations per candidate field block, the fastest kept (the slowest under
          // GpuOptions::placement_pick = 1)
          std::vector<float> v = s.solver(0).placement_ms();
          py::list l;
          for (float x : v) l.append(x);
          d["placement_probe_ms"] = l;
          const bool slowest = s.solver(0).options().placement_pick == 1;
          const auto mn = slowest ? std::max_element(v.begin(), v.end()) : std::min_element(v.begin(), v.end());
          if (slowest) d["placement_pick"] = "slowest";
          py::dict q;
          q["candidates"] = v.size();
          q["kept"] = size_t(mn - v.begin());
          q["kept_ms"] = *mn;
          q["first_ms"] = v[0];
          std::sort(v.begin(), v.end());
          q["median_ms"] = v[v.size() / 2];
          q["seconds"] = s.solver(0).placement_seconds();
          d["placement"] = q;
        }
        return d;
      });
}
