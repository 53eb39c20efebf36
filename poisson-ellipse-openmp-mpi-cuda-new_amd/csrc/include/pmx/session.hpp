// A solve session: decomposition + per-subdomain GPU solvers + comm backend + driver.
// Shared by the C++ CLI (apps/pmx.cpp) and the Python bindings.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "pmx/common.hpp"
#include "pmx/gpu_solver.hpp"

namespace pmx {

enum class CommKind : int { kSelf = 0, kLocal = 1, kRccl = 2 };

struct SessionConfig {
  ProblemSpec spec;
  GpuOptions opt;
  Split split = Split::kReference;
  CommKind comm = CommKind::kSelf;
  int world = 1;                 // total ranks (subdomains)
  std::vector<int> ranks;        // ranks owned by this process (default: all for self/local)
  std::vector<int> devices;      // device per owned rank (default: opt.device)
  std::string rccl_uid;          // for kRccl
  bool rccl_graph = false;       // capture RCCL calls into the hipGraph
  // Build the solvers only; the communicator and driver are created by Session::connect().  A
  // multi-process caller checks that every rank allocated its subdomain before any rank enters
  // the (blocking, collective) RCCL initialisation, so one failing rank cannot hang the others.
  bool defer_connect = false;
};

class Session {
 public:
  explicit Session(const SessionConfig& cfg);
  ~Session();
  void connect();  // comm + driver (called by the constructor unless cfg.defer_connect)
  bool connected() const { return driver_ != nullptr; }

  void init() { drv().init(); }
  void step(int64_t n) { drv().enqueue_iterations(n); }
  void synchronize() { drv().synchronize(); }
  RunStats solve(int poll_batches = 1) { return drv().solve(poll_batches); }
  // solve with periodic checkpoints to `save_path` (every `every` iterations; none if empty or
  // every == 0), optionally continuing from `resume_path` instead of starting from w = 0
  RunStats solve_checkpointed(const std::string& save_path, int64_t every,
                              const std::string& resume_path, int poll_batches = 1);
  // One file per owned subdomain: `path` when world == 1, else `path.rank<r>`.
  void save_checkpoint(const std::string& path);
  void load_checkpoint(const std::string& path);
  std::string checkpoint_file(const std::string& path, int rank) const;
  RunStats profile(int64_t n) { return drv().profile_phases(n); }
  PcgState state(int i = 0) { return drv().state(i); }

  const ProcGrid& grid() const { return pg_; }
  int num_local() const { return int(solvers_.size()); }
  GpuSubdomainSolver& solver(int i) { return *solvers_.at(size_t(i)); }
  const std::string comm_name() const { return comm_ ? comm_->name() : "unconnected"; }
  bool overlapped() const { return driver_ && driver_->overlapped(); }
  bool poisoned() const { return driver_ && driver_->poisoned(); }
  size_t device_bytes() const;
  // global (M+1) x (N+1) solution filled with the subdomains owned by this process
  std::vector<double> gather_local_w();
  // local interior (nx x ny, row-major) of owned subdomain i
  std::vector<double> local_w(int i = 0);

 private:
  PcgDriver& drv() const {
    PMX_CHECK(driver_ != nullptr, "session not connected (Session::connect)");
    return *driver_;
  }
  SessionConfig cfg_;
  ProcGrid pg_;
  std::vector<std::unique_ptr<GpuSubdomainSolver>> solvers_;
  std::unique_ptr<Comm> comm_;
  std::unique_ptr<PcgDriver> driver_;
};

// Largest square grid whose fields fit into `bytes_per_gpu` on `gpus` devices (SURVEY §5.7:
// subgrids sized against 288 GB HBM per MI355X).  fp64 (single pass): 5 fields x 8 B/pt; fp32
// (two sweeps): 4 x 4 B/pt.
int64_t max_square_grid(double bytes_per_gpu, int gpus, DType dtype, double reserve_fraction = 0.1);

}  // namespace pmx
