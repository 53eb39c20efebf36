// Session: decomposition + solvers + comm + driver.  See pmx/session.hpp.
#include "pmx/session.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <fstream>

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

  // one iteration algorithm for every subdomain (and every process: the choice only depends on
  // global data, see choose_single_pass)
  GpuOptions base = resolve_options(cfg_.opt);
  if (base.algo == -1) {
    HIP_CHECK(hipSetDevice(cfg_.devices[0]));
    size_t free_b = 0, total_b = 0;
    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    int per_device = 0;  // subdomains sharing the busiest device
    for (int d : cfg_.devices) per_device = std::max<int>(per_device, int(std::count(cfg_.devices.begin(), cfg_.devices.end(), d)));
    base.algo = choose_single_pass(cfg_.spec, pg_, base, double(total_b), per_device) ? 1 : 2;
  }
  for (size_t i = 0; i < cfg_.ranks.size(); ++i) {
    GpuOptions o = base;
    o.device = cfg_.devices[i];
    const Subdomain sd = decompose_2d(cfg_.spec.M, cfg_.spec.N, pg_, cfg_.ranks[i]);
    solvers_.push_back(std::make_unique<GpuSubdomainSolver>(cfg_.spec, sd, o));
  }
  if (!cfg_.defer_connect) connect();
}

void Session::connect() {
  PMX_CHECK(driver_ == nullptr, "session already connected");
  std::vector<GpuSubdomainSolver*> raw;
  for (auto& s : solvers_) raw.push_back(s.get());
  switch (cfg_.comm) {
    case CommKind::kSelf: comm_ = make_self_comm(); break;
    case CommKind::kLocal: comm_ = make_local_comm(raw); break;
    case CommKind::kRccl:
      comm_ = make_rccl_comm(cfg_.rccl_uid, cfg_.world, cfg_.ranks, cfg_.devices, cfg_.rccl_graph);
      break;
  }
  driver_ = std::make_unique<PcgDriver>(raw, comm_.get(), cfg_.opt.graph_batch);
}

Session::~Session() {
  driver_.reset();
  comm_.reset();
  solvers_.clear();
}

size_t Session::device_bytes() const {
  size_t b = 0;
  for (auto& s : solvers_) b += s->device_bytes();
  return b;
}

std::vector<double> Session::local_w(int i) {
  drv().synchronize();
  return solvers_.at(size_t(i))->download_w(driver_->streams()[size_t(i)]);
}

std::vector<double> Session::gather_local_w() {
  const int M = cfg_.spec.M, N = cfg_.spec.N;
  std::vector<double> g(size_t(M + 1) * (N + 1), 0.0);
  for (size_t i = 0; i < solvers_.size(); ++i) {
    auto& s = *solvers_[i];
    const Subdomain& sd = s.sd();
    const std::vector<double> w = s.download_w(drv().streams()[i]);
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
  drv().synchronize();
  for (size_t i = 0; i < solvers_.size(); ++i) {
    const std::string f = checkpoint_file(path, solvers_[i]->sd().rank);
    const std::string tmp = f + ".tmp";
    {
      std::ofstream os(tmp, std::ios::binary | std::ios::trunc);
      PMX_CHECK(os.good(), "cannot open checkpoint file " << tmp);
      solvers_[i]->save_checkpoint(os, driver_->streams()[i]);
    }
    PMX_CHECK(std::rename(tmp.c_str(), f.c_str()) == 0, "cannot rename " << tmp << " -> " << f);
  }
}

void Session::load_checkpoint(const std::string& path) {
  drv().synchronize();
  for (size_t i = 0; i < solvers_.size(); ++i) {
    const std::string f = checkpoint_file(path, solvers_[i]->sd().rank);
    std::ifstream is(f, std::ios::binary);
    PMX_CHECK(is.good(), "cannot open checkpoint file " << f);
    solvers_[i]->load_checkpoint(is, driver_->streams()[i]);
  }
}

RunStats Session::solve_checkpointed(const std::string& save_path, int64_t every,
                                     const std::string& resume_path, int poll_batches) {
  const bool resume = !resume_path.empty();
  if (resume) load_checkpoint(resume_path);
  std::function<void(const PcgState&)> cb;
  if (every > 0 && !save_path.empty()) cb = [&](const PcgState&) { save_checkpoint(save_path); };
  return drv().solve(poll_batches, !resume, every, cb);
}

int64_t max_square_grid(double bytes_per_gpu, int gpus, DType dtype, double reserve_fraction) {
  // the default iteration (pcg1) keeps 5 fields in either precision; +1% pitch
  const double bpp = 5.0 * (dtype == DType::kFp64 ? 8.0 : 4.0) * 1.01;
  const double pts = bytes_per_gpu * (1.0 - reserve_fraction) * gpus / bpp;
  return int64_t(std::floor(std::sqrt(pts)));
}

}  // namespace pmx
