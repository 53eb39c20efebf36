// Session: decomposition + solvers + comm + driver.  See pmx/session.hpp.
#include "pmx/session.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <exception>
#include <fstream>
#include <mutex>
#include <set>
#include <thread>

#include "pmx/common.hpp"

namespace pmx {

Session::Session(const SessionConfig& cfg) : cfg_(cfg) {
  cfg_.spec.validate();
  PMX_CHECK(cfg_.world >= 1, "world size must be >= 1");
  pg_ = make_process_grid(cfg_.world, cfg_.spec.M, cfg_.spec.N, cfg_.split);
  if (cfg_.ranks.empty()) {
    if (cfg_.comm == CommKind::kRccl) {
      PMX_CHECK(false, "RCCL sessions must list the ranks they own");
    }
    for (int r = 0; r < cfg_.world; ++r) cfg_.ranks.push_back(r);
  }
  if (cfg_.devices.empty()) cfg_.devices.assign(cfg_.ranks.size(), cfg_.opt.device);
  PMX_CHECK(cfg_.devices.size() == cfg_.ranks.size(), "one device per owned rank");
  if (cfg_.comm == CommKind::kSelf)
    PMX_CHECK(cfg_.world == 1, "self comm needs world == 1 (use local or rccl)");
  if (cfg_.comm == CommKind::kLocal)
    PMX_CHECK(int(cfg_.ranks.size()) == cfg_.world, "local comm owns every rank");
  if (cfg_.comm == CommKind::kIpc)
    PMX_CHECK(cfg_.ranks.size() == 1, "the IPC transport runs one rank per process");
  if (cfg_.comm == CommKind::kLoopback)
    PMX_CHECK(cfg_.ranks.size() == 1, "loopback runs exactly one rank of the decomposition");

  // one iteration algorithm for every subdomain (and every process: the choice only depends on
  // global data, see choose_algo)
  GpuOptions pre = cfg_.opt;
  // a multi-process RCCL run tracks device progress for its hang watchdog (GpuOptions::progress)
  if ((cfg_.comm == CommKind::kRccl || cfg_.comm == CommKind::kIpc) && cfg_.world > 1) pre.progress = 1;
  GpuOptions base = resolve_options(pre);
  if (base.algo == -1) {
    HIP_CHECK(hipSetDevice(cfg_.devices[0]));
    size_t free_b = 0, total_b = 0;
    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    int per_device = 0;  // subdomains sharing the busiest device
    for (int d : cfg_.devices) per_device = std::max<int>(per_device, int(std::count(cfg_.devices.begin(), cfg_.devices.end(), d)));
    per_device = std::max(per_device, cfg_.sharing);
    // every transport of a Session moves ghost rows straight between the fields (direct rows)
    base.algo = choose_algo(cfg_.spec, pg_, base, double(total_b), per_device, true);
  }
  for (size_t i = 0; i < cfg_.ranks.size(); ++i) {
    GpuOptions o = base;
    o.device = cfg_.devices[i];
    if (cfg_.comm == CommKind::kLoopback) o.ca_dirichlet = 1;  // see GpuOptions::ca_dirichlet
    const Subdomain sd = decompose_2d(cfg_.spec.M, cfg_.spec.N, pg_, cfg_.ranks[i]);
    solvers_.push_back(std::make_unique<GpuSubdomainSolver>(cfg_.spec, sd, o));
  }
  if (!cfg_.defer_connect) connect();
}

std::string Session::ipc_export() {
  PMX_CHECK(cfg_.comm == CommKind::kIpc, "ipc_export needs an IPC session");
  if (!comm_) comm_ = make_ipc_comm(solvers_[0].get(), cfg_.world);
  return pmx::ipc_export(comm_.get());
}

void Session::connect() {
  PMX_CHECK(drivers_.empty(), "session already connected");
  std::vector<GpuSubdomainSolver*> raw;
  for (auto& s : solvers_) raw.push_back(s.get());
  switch (cfg_.comm) {
    case CommKind::kIpc:
      if (!comm_) comm_ = make_ipc_comm(raw[0], cfg_.world);
      if (cfg_.world == 1 && cfg_.ipc_exports.empty()) cfg_.ipc_exports.push_back(pmx::ipc_export(comm_.get()));
      ipc_attach(comm_.get(), cfg_.ipc_exports);
      break;
    case CommKind::kSelf: comm_ = make_self_comm(); break;
    case CommKind::kLoopback: comm_ = make_loopback_comm(); break;
    case CommKind::kLocal: comm_ = make_local_comm(raw); break;
    case CommKind::kRccl:
      // overlap off = the serialized schedule: one communicator, every call on the compute stream
      comm_ = make_rccl_comm(cfg_.rccl_uid, cfg_.world, cfg_.ranks, cfg_.devices, cfg_.rccl_graph, cfg_.opt.overlap);
      break;
  }
  // one host thread per GPU.  Several owned ranks on distinct devices (pmx --gpus G)
  // get a driver each -- own streams, own graph captured by its own thread -- so no device's
  // launches queue behind another's on one host thread.
  const std::set<int> devs(cfg_.devices.begin(), cfg_.devices.end());
  const bool auto_threads = cfg_.comm == CommKind::kRccl && raw.size() > 1 && devs.size() == raw.size();
  threaded_ = cfg_.threaded == 1 || (cfg_.threaded == -1 && auto_threads);
  PMX_CHECK(!threaded_ || cfg_.comm == CommKind::kRccl, "threaded drivers need the RCCL communicator");
  if (!threaded_) {
    drivers_.push_back(std::make_unique<PcgDriver>(raw, comm_.get(), cfg_.opt.graph_batch));
    return;
  }
  for (size_t i = 0; i < raw.size(); ++i) {
    views_.push_back(comm_->rank_view(int(i)));
    HIP_CHECK(hipSetDevice(raw[i]->device()));
    drivers_.push_back(std::make_unique<PcgDriver>(std::vector<GpuSubdomainSolver*>{raw[i]}, views_.back().get(),
                                                   cfg_.opt.graph_batch));
  }
}

Session::~Session() {
  drivers_.clear();
  views_.clear();
  comm_.reset();
  solvers_.clear();
}

void Session::for_drivers(const std::function<void(size_t, PcgDriver&)>& f) {
  require_connected();
  if (!threaded_) {
    f(0, *drivers_[0]);
    return;
  }
  std::exception_ptr err;
  std::mutex mu;
  std::vector<std::thread> th;
  th.reserve(drivers_.size());
  for (size_t i = 0; i < drivers_.size(); ++i)
    th.emplace_back([&, i] {
      try {
        HIP_CHECK(hipSetDevice(solvers_[i]->device()));
        f(i, *drivers_[i]);
      } catch (...) {
        bool first = false;
        {
          std::lock_guard<std::mutex> lk(mu);
          if (!err) {
            err = std::current_exception();
            first = true;
          }
        }
        // The other threads may be blocked on collectives this rank will never post: abort the
        // communicator so they return with an error and the join below cannot hang.
        if (first && comm_) comm_->abort();
      }
    });
  for (auto& t : th) t.join();
  if (err) std::rethrow_exception(err);
}

hipStream_t Session::stream_of(int i) const {
  require_connected();
  return threaded_ ? drivers_.at(size_t(i))->streams()[0] : drivers_[0]->streams().at(size_t(i));
}

bool Session::prepare(int64_t n) {
  std::vector<char> ok(drivers_.size(), 0);
  for_drivers([&](size_t i, PcgDriver& d) { ok[i] = d.prepare(n) ? 1 : 0; });
  bool all = true;
  for (char c : ok) all &= c != 0;
  return all;
}

void Session::step_eager(int64_t n) {
  for_drivers([n](size_t, PcgDriver& d) { d.enqueue_eager(n); });
}

PcgDriver::PathStats Session::path_stats() const {
  require_connected();
  PcgDriver::PathStats p = drivers_[0]->path_stats();
  for (auto& d : drivers_)
    PMX_CHECK(d->path_stats().graph_iters == p.graph_iters && d->path_stats().eager_iters == p.eager_iters,
              "drivers disagree on the launch path");
  return p;
}

void Session::reset_path_stats() {
  for (auto& d : drivers_) d->reset_path_stats();
}

bool Session::split_sweep() const {
  require_connected();
  return drivers_[0]->split_sweep();
}

bool Session::direct_rows() const {
  require_connected();
  return drivers_[0]->direct_rows();
}

void Session::progress(int i, long long out[3]) const { solvers_.at(size_t(i))->progress(out); }

ErrorStats Session::error_norms() {
  synchronize();
  ErrorStats t;
  t.max_w = -HUGE_VAL;
  for (size_t i = 0; i < solvers_.size(); ++i) {
    const ErrorStats e = solvers_[i]->error_norms(stream_of(int(i)));
    t.sum_e2 += e.sum_e2;
    t.max_e = std::max(t.max_e, e.max_e);
    t.max_w = std::max(t.max_w, e.max_w);
  }
  return t;
}

void Session::init() {
  for_drivers([](size_t, PcgDriver& d) { d.init(); });
}

void Session::step(int64_t n) {
  for_drivers([n](size_t, PcgDriver& d) { d.enqueue_iterations(n); });
}

void Session::synchronize() {
  for_drivers([](size_t, PcgDriver& d) { d.synchronize(); });
}

PcgState Session::state(int i) {
  require_connected();
  return threaded_ ? drivers_.at(size_t(i))->state(0) : drivers_[0]->state(i);
}

RunStats Session::solve_impl(int poll_batches, bool do_init, int64_t every, const std::string& save_path) {
  // every rank's driver iterates to the same device stop decision (the all-reduced scalars are
  // identical everywhere); rank 0's statistics are returned
  std::vector<RunStats> st(drivers_.size());
  for_drivers([&](size_t i, PcgDriver& d) {
    std::function<void(const PcgState&)> cb;
    if (every > 0 && !save_path.empty()) {
      cb = [&, i](const PcgState&) {
        if (!threaded_) {
          save_checkpoint(save_path);
          return;
        }
        const std::string f = checkpoint_file(save_path, solvers_[i]->sd().rank), tmp = f + ".tmp";
        {
          std::ofstream os(tmp, std::ios::binary | std::ios::trunc);
          PMX_CHECK(os.good(), "cannot open checkpoint file " << tmp);
          solvers_[i]->save_checkpoint(os, d.streams()[0]);
        }
        PMX_CHECK(std::rename(tmp.c_str(), f.c_str()) == 0, "cannot rename " << tmp << " -> " << f);
      };
    }
    st[i] = d.solve(poll_batches, do_init, every, cb);
  });
  for (const RunStats& r : st)
    PMX_CHECK(r.iters == st[0].iters && r.status == st[0].status,
              "ranks disagree on the stop decision (" << r.iters << " vs " << st[0].iters << " iterations)");
  return st[0];
}

RunStats Session::solve(int poll_batches) { return solve_impl(poll_batches, true, 0, ""); }

RunStats Session::profile(int64_t n) {
  std::vector<RunStats> st(drivers_.size());
  for_drivers([&](size_t i, PcgDriver& d) { st[i] = d.profile_phases(n); });
  RunStats m = st[0];
  for (const RunStats& r : st) {  // MAX over ranks, as the reference reports its buckets
    m.t_kernel_a = std::max(m.t_kernel_a, r.t_kernel_a);
    m.t_kernel_b = std::max(m.t_kernel_b, r.t_kernel_b);
    m.t_reduce = std::max(m.t_reduce, r.t_reduce);
    m.t_allreduce = std::max(m.t_allreduce, r.t_allreduce);
    m.t_halo = std::max(m.t_halo, r.t_halo);
    m.t_comm = std::max(m.t_comm, r.t_comm);
  }
  return m;
}

size_t Session::device_bytes() const {
  size_t b = 0;
  for (auto& s : solvers_) b += s->device_bytes();
  return b;
}

std::vector<double> Session::local_w(int i) {
  synchronize();
  return solvers_.at(size_t(i))->download_w(stream_of(i));
}

std::vector<double> Session::partials(int i) {
  synchronize();
  return solvers_.at(size_t(i))->read_partials(stream_of(i));
}

std::vector<double> Session::gather_local_w() {
  const int M = cfg_.spec.M, N = cfg_.spec.N;
  std::vector<double> g(size_t(M + 1) * (N + 1), 0.0);
  for (size_t i = 0; i < solvers_.size(); ++i) {
    auto& s = *solvers_[i];
    const Subdomain& sd = s.sd();
    const std::vector<double> w = s.download_w(stream_of(int(i)));
    for (int li = 1; li <= sd.nx; ++li)
      for (int lj = 1; lj <= sd.ny; ++lj)
        g[size_t(sd.gi0() + li) * (N + 1) + sd.gj0() + lj] = w[size_t(li - 1) * sd.ny + lj - 1];
  }
  return g;
}

std::string Session::checkpoint_file(const std::string& path, int rank) const {
  return cfg_.world == 1 ? path : path + ".rank" + std::to_string(rank);
}

void Session::save_checkpoint(const std::string& path) {
  synchronize();
  for (size_t i = 0; i < solvers_.size(); ++i) {
    const std::string f = checkpoint_file(path, solvers_[i]->sd().rank);
    const std::string tmp = f + ".tmp";
    {
      std::ofstream os(tmp, std::ios::binary | std::ios::trunc);
      PMX_CHECK(os.good(), "cannot open checkpoint file " << tmp);
      solvers_[i]->save_checkpoint(os, stream_of(int(i)));
    }
    PMX_CHECK(std::rename(tmp.c_str(), f.c_str()) == 0, "cannot rename " << tmp << " -> " << f);
  }
}

void Session::load_checkpoint(const std::string& path) {
  synchronize();
  for (size_t i = 0; i < solvers_.size(); ++i) {
    const std::string f = checkpoint_file(path, solvers_[i]->sd().rank);
    std::ifstream is(f, std::ios::binary);
    PMX_CHECK(is.good(), "cannot open checkpoint file " << f);
    solvers_[i]->load_checkpoint(is, stream_of(int(i)));
  }
}

RunStats Session::solve_checkpointed(const std::string& save_path, int64_t every,
                                     const std::string& resume_path, int poll_batches) {
  const bool resume = !resume_path.empty();
  if (resume) load_checkpoint(resume_path);
  return solve_impl(poll_batches, !resume, every, save_path);
}

std::vector<std::vector<CommEvent>> record_comm_sequence(const ProblemSpec& spec, int world, Split split,
                                                         const GpuOptions& opt, int64_t iters) {
  const ProcGrid pg = make_process_grid(world, spec.M, spec.N, split);
  GpuOptions o = resolve_options(opt);
  if (o.algo == -1) o.algo = choose_algo(spec, pg, o, 0.0, world, true);
  std::vector<std::unique_ptr<GpuSubdomainSolver>> solvers;
  std::vector<std::vector<CommEvent>> logs(static_cast<size_t>(world));
  std::vector<std::unique_ptr<Comm>> comms;
  std::vector<std::unique_ptr<PcgDriver>> drivers;
  for (int r = 0; r < world; ++r) {
    solvers.push_back(std::make_unique<GpuSubdomainSolver>(spec, decompose_2d(spec.M, spec.N, pg, r), o));
    comms.push_back(make_recording_comm(&logs[size_t(r)], world, o.overlap));
    drivers.push_back(std::make_unique<PcgDriver>(std::vector<GpuSubdomainSolver*>{solvers.back().get()},
                                                  comms.back().get(), o.graph_batch));
  }
  // each rank's driver on its own (nothing is exchanged; the values are garbage, the call
  // sequence is what counts): init, then `iters` iterations -- captured when graph_batch > 0
  for (auto& d : drivers) {
    d->init();
    d->enqueue_iterations(iters);
    d->synchronize();
  }
  return logs;
}

int64_t max_square_grid(double bytes_per_gpu, int gpus, DType dtype, double reserve_fraction, int algo) {
  // pcg1 keeps 5 fields in either precision, the s-step PCG (fp64) 5 fields plus 2 fp64 face fields,
  // pcg2 4 fields; +1% pitch.  Auto (-1): the largest grid that fits SOME algorithm -- pcg1, to which
  // auto falls back when the s-step's fields do not fit (choose_algo)
  const double elem = dtype == DType::kFp64 ? 8.0 : 4.0;
  const double bpp = (algo == 3 ? 5.0 * elem + 16.0 : algo == 2 ? 4.0 * elem : 5.0 * elem) * 1.01;
  const double pts = bytes_per_gpu * (1.0 - reserve_fraction) * gpus / bpp;
  return int64_t(std::floor(std::sqrt(pts)));
}

}  // namespace pmx
