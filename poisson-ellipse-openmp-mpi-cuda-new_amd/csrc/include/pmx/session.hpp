// A solve session: decomposition + per-subdomain GPU solvers + comm backend + driver.
// Shared by the C++ CLI (apps/pmx.cpp) and the Python bindings.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "pmx/common.hpp"
#include "pmx/gpu_solver.hpp"

namespace pmx {

enum class CommKind : int { kSelf = 0, kLocal = 1, kRccl = 2, kIpc = 3, kLoopback = 4 };

struct SessionConfig {
  ProblemSpec spec;
  GpuOptions opt;
  Split split = Split::kReference;
  CommKind comm = CommKind::kSelf;
  int world = 1;                 // total ranks (subdomains)
  std::vector<int> ranks;        // ranks owned by this process (default: all for self/local)
  std::vector<int> devices;      // device per owned rank (default: opt.device)
  std::string rccl_uid;          // for kRccl
  std::vector<std::string> ipc_exports;  // for kIpc: every rank's Session::ipc_export(), by rank
  bool rccl_graph = false;       // capture RCCL calls into the hipGraph
  // Build the solvers only; the communicator and driver are created by Session::connect().  A
  // multi-process caller checks that every rank allocated its subdomain before any rank enters
  // the (blocking, collective) RCCL initialisation, so one failing rank cannot hang the others.
  bool defer_connect = false;
  // One host thread (and one driver, graph and stream set) per owned rank: -1 = auto (RCCL with
  // several owned ranks on distinct devices, i.e. `pmx --gpus G`), 1 = always (RCCL only; with a
  // single rank it exercises the threaded path on one GPU), 0 = one host thread drives all ranks.
  int threaded = -1;
  // Subdomains of the whole job that share the busiest device (0 = count this session's own
  // `devices`).  A multi-process job whose ranks share one GPU (bench.py --share-gpu, IPC
  // rehearsals) passes its world size, so every rank sizes the iteration algorithm's fields against
  // the device it shares (choose_algo; the torch path's comm_layout(sharing=...) likewise).
  int sharing = 0;
};

class Session {
 public:
  explicit Session(const SessionConfig& cfg);
  ~Session();
  void connect();  // comm + driver (called by the constructor unless cfg.defer_connect)
  // kIpc (defer_connect): this rank's IPC export; hand every rank's to set_ipc_exports, then connect
  std::string ipc_export();
  void set_ipc_exports(const std::vector<std::string>& e) { cfg_.ipc_exports = e; }
  bool connected() const { return !drivers_.empty(); }

  void init();
  void step(int64_t n);
  void synchronize();
  RunStats solve(int poll_batches = 1);
  // solve with periodic checkpoints to `save_path` (every `every` iterations; none if empty or
  // every == 0), optionally continuing from `resume_path` instead of starting from w = 0
  RunStats solve_checkpointed(const std::string& save_path, int64_t every,
                              const std::string& resume_path, int poll_batches = 1);
  // One file per owned subdomain: `path` when world == 1, else `path.rank<r>`.
  void save_checkpoint(const std::string& path);
  void load_checkpoint(const std::string& path);
  std::string checkpoint_file(const std::string& path, int rank) const;
  RunStats profile(int64_t n);  // threaded: every bucket is the MAX over the owned ranks
  PcgState state(int i = 0);
  bool threaded() const { return threaded_; }  // one host thread per owned rank
  // capture every graph step(n) would replay now, without running (PcgDriver::prepare)
  bool prepare(int64_t n);
  void step_eager(int64_t n);  // n iterations as individual launches (canary)
  PcgDriver::PathStats path_stats() const;
  void reset_path_stats();
  bool split_sweep() const;
  bool direct_rows() const;
  // host-mapped device progress of owned rank i (GpuSubdomainSolver::progress); no HIP call
  void progress(int i, long long out[3]) const;
  // error vs the analytic solution over the owned subdomains (sum of e^2, max |e|, max w)
  ErrorStats error_norms();

  const ProcGrid& grid() const { return pg_; }
  int num_local() const { return int(solvers_.size()); }
  GpuSubdomainSolver& solver(int i) { return *solvers_.at(size_t(i)); }
  const std::string comm_name() const { return comm_ ? comm_->name() : "unconnected"; }
  // the iteration algorithm the solvers run: "ca" (s-step PCG), "pcg1" or "pcg2"
  std::string algo_name() const {
    return solvers_[0]->ca() ? "ca" : solvers_[0]->single_pass() ? "pcg1" : "pcg2";
  }
  bool overlapped() const { return !drivers_.empty() && drivers_[0]->overlapped(); }
  bool poisoned() const { return !drivers_.empty() && drivers_[0]->poisoned(); }
  size_t device_bytes() const;
  // global (M+1) x (N+1) solution filled with the subdomains owned by this process
  std::vector<double> gather_local_w();
  // local interior (nx x ny, row-major) of owned subdomain i
  std::vector<double> local_w(int i = 0);
  // the per-tile partial sums (5 per tile slot) the last sweep wrote (tests of the reduction hand-off)
  std::vector<double> partials(int i = 0);
  hipStream_t stream_of(int i) const;  // the compute stream of owned rank i

 private:
  void require_connected() const {
    PMX_CHECK(!drivers_.empty(), "session not connected (Session::connect)");
  }
  // f(driver index, driver) for every driver: inline, or one host thread per driver (each bound
  // to its rank's device) in threaded mode; the first exception is rethrown after all joined
  void for_drivers(const std::function<void(size_t, PcgDriver&)>& f);
  RunStats solve_impl(int poll_batches, bool do_init, int64_t every, const std::string& save_path);

  SessionConfig cfg_;
  ProcGrid pg_;
  std::vector<std::unique_ptr<GpuSubdomainSolver>> solvers_;
  std::unique_ptr<Comm> comm_;
  std::vector<std::unique_ptr<Comm>> views_;            // threaded: per-rank communicators
  std::vector<std::unique_ptr<PcgDriver>> drivers_;     // one (all ranks) or one per rank
  bool threaded_ = false;
};

// Largest square grid whose fields fit into `bytes_per_gpu` on `gpus` devices (SURVEY §5.7:
// subgrids sized against 288 GB HBM per MI355X): the default single pass keeps 5 fields, 8 B/pt
// each in fp64 and 4 B/pt in fp32.
// Every rank's communication calls for `iters` iterations of its own driver on a RecordingComm (all
// ranks on the current device of opt.device, nothing exchanged): the test that every rank issues the
// same sequence of collectives and matching send/recv groups per captured batch.
std::vector<std::vector<CommEvent>> record_comm_sequence(const ProblemSpec& spec, int world, Split split,
                                                         const GpuOptions& opt, int64_t iters);

int64_t max_square_grid(double bytes_per_gpu, int gpus, DType dtype, double reserve_fraction = 0.1, int algo = -1);

}  // namespace pmx
