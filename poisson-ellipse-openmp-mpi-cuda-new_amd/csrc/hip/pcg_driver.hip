// The iteration driver (PcgDriver, see pmx/gpu_solver.hpp): one compute stream per local subdomain
// (plus a comm stream when the ghost exchange overlaps), the per-iteration schedule of pcg1 / pcg2
// (the s-step's is in ca_solver.hip, pcg1's decomposed schedules in pcg1_driver.hip), hipGraph
// batches keyed by phase and length, the device-side stop test polled once per batch, and the
// reference's five stage-4 timing buckets (profile_phases).
// Reference loop being replaced: stage4-mpi+cuda/poisson_mpi_cuda_f.cu:843-943 (iteration),
// :956-980 and :1022-1035 (timing buckets).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pmx/common.hpp"
#include "pmx/gpu_solver.hpp"
#include "pmx/session.hpp"
#include "pmx/trace.hpp"

namespace pmx {

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

PcgDriver::PcgDriver(std::vector<GpuSubdomainSolver*> local, Comm* comm, int graph_batch)
    : local_(std::move(local)), comm_(comm), graph_batch_(graph_batch) {
  PMX_CHECK(!local_.empty(), "no local subdomains");
  bool same_device = true;
  for (auto* s : local_) same_device &= s->device() == local_[0]->device();
  const size_t nstreams = same_device ? 1 : local_.size();
  for (size_t i = 0; i < nstreams; ++i) {
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    hipStream_t st;
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    roctxNameHipStream("pmx:compute", st);
    streams_.push_back(st);
  }
  if (same_device) streams_.resize(local_.size(), streams_[0]);
  bool any_nb = false;
  for (auto* s : local_) any_nb |= s->geom().nb != 0;
  any_nb_ = any_nb;
  single_pass_ = local_[0]->single_pass();
  ca_ = local_[0]->ca();
  for (auto* s : local_)
    PMX_CHECK(s->single_pass() == single_pass_ && s->ca() == ca_,
              "local subdomains disagree on the iteration algorithm");

  overlap_ = any_nb && local_[0]->options().overlap;
  // Direct-row ghost exchange (row strips): no pack/unpack launches; PMX_DIRECT_ROWS=0 turns it off
  // (A/B).  Every local solver must qualify (they exchange with each other under LocalComm).
  bool direct = (single_pass_ || ca_) && any_nb && comm_->direct_rows();
  for (auto* s : local_) direct &= s->can_direct_rows();
  if (const char* d = study_env("PMX_DIRECT_ROWS"); d && d[0] == '0') direct = false;
  direct_ = direct;
  for (auto* s : local_) s->set_direct_rows(direct_);
  // s-step: row strips move their ghost rows directly where the transport can; otherwise (2-D blocks, or
  // a transport without direct rows) the packed slots carry rows, columns and corners (k_ca_halo)
  // One hardware queue per process (GPU_MAX_HW_QUEUES=1): every stream lands on it, so forking the
  // halo / frame work onto side streams cannot overlap anything -- and ROCm 7.2 segfaults inside
  // hipGraphLaunch on a captured graph with forked branches in that configuration (traced with
  // PMX_DEBUG_GRAPH, bench/probe/hwq_probe.py).  The driver then runs the unforked schedule.
  // PMX_FORK_ONE_QUEUE=1 keeps the forks (eager only) to test that their event ordering needs no
  // concurrently resident streams.
  if (const char* q = std::getenv("GPU_MAX_HW_QUEUES"); q && std::atoi(q) == 1) {
    const char* keep = study_env("PMX_FORK_ONE_QUEUE");
    if (keep && keep[0] == '1') {
      bool forked = overlap_;
      for (auto* s : local_) forked |= s->ca_side_stream();
      graph_failed_ = forked;  // forked schedule, eager launches
    } else {
      overlap_ = false;
      // the s-step passes fork their frame tiles onto a side stream inside every block: run them
      // in-stream instead (a forked graph on one queue is the crashing configuration)
      for (auto* s : local_) s->drop_side_stream();
    }
  }
  const char* env = std::getenv("PMX_POISON_HALOS");
  poison_ = any_nb && (local_[0]->options().poison_halos || (env && env[0] == '1'));
  if (overlap_) {
    for (size_t i = 0; i < nstreams; ++i) {
      HIP_CHECK(hipSetDevice(local_[i]->device()));
      hipStream_t st;
      HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      roctxNameHipStream("pmx:comm", st);
      comm_streams_.push_back(st);
      hipEvent_t e0, e1;
      HIP_CHECK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
      ev_packed_.push_back(e0);
      ev_halo_.push_back(e1);
    }
    if (same_device) comm_streams_.resize(local_.size(), comm_streams_[0]);
  }
  // Split sweep: interior tiles on the compute stream while the previous sweep's ghost exchange is
  // in flight, frame tiles on their own stream once it has landed.  Default: on with RCCL, whose
  // xGMI exchange is the long pole; off with LocalComm, whose device copies are cheaper than the
  // extra launch (16384^2 as 2x2 subdomains on one GPU: 2.647 vs 2.602 ms; 2 strips: 2.416 vs
  // 2.430).  GpuOptions::split_sweep (study: PMX_PCG1_SPLIT) forces it.
  const int sw = local_[0]->options().split_sweep;
  const bool split_default = comm_->prefers_split();
  split_ = overlap_ && single_pass_ && (sw >= 0 ? sw == 1 : split_default);
  if (split_) {
    auto ev = [](std::vector<hipEvent_t>& v) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      v.push_back(e);
    };
    for (size_t i = 0; i < nstreams; ++i) {
      HIP_CHECK(hipSetDevice(local_[i]->device()));
      hipStream_t st;
      HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      roctxNameHipStream("pmx:frame", st);
      frame_streams_.push_back(st);
      ev(ev_ar_);
      ev(ev_fdone_);
      ev(ev_swept_);
    }
    if (same_device) frame_streams_.resize(local_.size(), frame_streams_[0]);
    // default on: loopback rank 3 of 8 284.2 / 284.5 vs 288.0 / 286.9 us, 301.8 vs 308.4 with the
    // 20 / 15-us exchange / all-reduce stand-ins (profiles/r4/loopback/r4al_*); PMX_FRAME_ON_COMM=0
    // restores the separate frame stream
    const char* fc = study_env("PMX_FRAME_ON_COMM");
    frame_on_comm_ = !(fc && fc[0] == '0');
  }
}

PcgDriver::~PcgDriver() {
  for (auto e : execs_) (void)hipGraphExecDestroy(e);
  for (auto g : graphs_) (void)hipGraphDestroy(g);
  for (auto* v : {&streams_, &comm_streams_, &frame_streams_}) {
    hipStream_t last = nullptr;
    for (auto s : *v) {
      if (s != last) (void)hipStreamDestroy(s);
      last = s;
    }
  }
  for (auto* v : {&ev_packed_, &ev_halo_, &ev_ar_, &ev_fdone_, &ev_swept_})
    for (auto e : *v) (void)hipEventDestroy(e);
}

void PcgDriver::synchronize() {
  hipStream_t last = nullptr;
  for (size_t i = 0; i < streams_.size(); ++i) {
    if (streams_[i] == last) continue;
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    HIP_CHECK(hipStreamSynchronize(streams_[i]));
    last = streams_[i];
  }
}

void PcgDriver::init() {
  TraceRange tr("pmx:init");
  if (ca_) {  // fields, state and set 0 of the first block (and its ghost rows)
    for (size_t i = 0; i < local_.size(); ++i) {
      HIP_CHECK(hipSetDevice(local_[i]->device()));
      local_[i]->enqueue_init(streams_[i]);
    }
    if (any_nb_) ca_exchange(streams_);
    synchronize();
    return;
  }
  // pcg2's k_init packs r^0 into the send slots
  if (!single_pass_ && any_nb_) comm_->before_pack(local_, streams_);
  for (size_t i = 0; i < local_.size(); ++i) local_[i]->enqueue_init(streams_[i]);
  if (single_pass_) {
    // ghosts of r^0 -> sweep 0 ((z^0, r^0), (A z^0, z^0); it 0 -> 1) -> all-reduce -> ghosts of
    // sweep 0's outputs, which sweep 1 reads
    if (any_nb_) halo_exchange_pcg1(streams_, local_[0]->host_k());
    for (size_t i = 0; i < local_.size(); ++i) {
      HIP_CHECK(hipSetDevice(local_[i]->device()));
      local_[i]->enqueue_phase_a(streams_[i]);
    }
    comm_->allreduce(local_, 2, streams_);
    if (any_nb_) halo_exchange_pcg1(streams_, local_[0]->host_k());
  } else {
    comm_->allreduce(local_, 1, streams_);
    poison(streams_);
    comm_->halo(local_, streams_);
  }
  synchronize();
}

void PcgDriver::poison(std::vector<hipStream_t>& streams) {
  if (!poison_) return;
  for (size_t i = 0; i < local_.size(); ++i) {
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    local_[i]->enqueue_poison_recv(streams[i]);
  }
}

void PcgDriver::enqueue_one_iteration() {
  if (ca_) {
    enqueue_ca(1);
    return;
  }
  if (split_) {
    enqueue_split_iteration();
    return;
  }
  if (single_pass_) {
    // Single pass.  Every tile of sweep k+1 needs alpha_{k+1}, i.e. the all-reduced sums of
    // sweep k, so no part of the next sweep can start before the all-reduce; what CAN run
    // concurrently is the ghost exchange, which only needs sweep k's outputs:
    //   compute stream  sweep k -> reduce_n -> all-reduce(red_c, 5 doubles) -> join -> sweep k+1
    //   comm stream             `-> pack -> send/recv (8 slots) -> unpack ---'
    if (!any_nb_ || !overlap_) {
      for (size_t i = 0; i < local_.size(); ++i) {
        HIP_CHECK(hipSetDevice(local_[i]->device()));
        local_[i]->enqueue_phase_a(streams_[i]);
      }
      comm_->allreduce(local_, 2, streams_);  // no-op for SelfComm
      if (any_nb_) halo_exchange_pcg1(streams_, local_[0]->host_k());  // the reduction bumped host_k
      return;
    }
    for (size_t i = 0; i < local_.size(); ++i) {
      HIP_CHECK(hipSetDevice(local_[i]->device()));
      local_[i]->enqueue_kernel_a(streams_[i]);
    }
    for_each_stream([&](size_t i, size_t u) {
      HIP_CHECK(hipEventRecord(ev_packed_[u], streams_[i]));
      HIP_CHECK(hipStreamWaitEvent(comm_streams_[i], ev_packed_[u], 0));
    });
    halo_exchange_pcg1(comm_streams_, local_[0]->host_k() + 1);  // before the reduction's bump
    for_each_stream([&](size_t i, size_t u) { HIP_CHECK(hipEventRecord(ev_halo_[u], comm_streams_[i])); });
    for (size_t i = 0; i < local_.size(); ++i) {
      HIP_CHECK(hipSetDevice(local_[i]->device()));
      local_[i]->enqueue_reduce_a(streams_[i]);
    }
    comm_->allreduce(local_, 2, streams_);
    for_each_stream([&](size_t i, size_t u) { HIP_CHECK(hipStreamWaitEvent(streams_[i], ev_halo_[u], 0)); });
    return;
  }
  for (size_t i = 0; i < local_.size(); ++i) {
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    local_[i]->enqueue_phase_a(streams_[i]);
  }
  comm_->allreduce(local_, 0, streams_);
  if (!overlap_) {
    if (any_nb_) comm_->before_pack(local_, streams_);  // k_pcg_b packs the send slots
    for (size_t i = 0; i < local_.size(); ++i) {
      HIP_CHECK(hipSetDevice(local_[i]->device()));
      local_[i]->enqueue_phase_b(streams_[i]);
    }
    comm_->allreduce(local_, 1, streams_);
    poison(streams_);
    comm_->halo(local_, streams_);
    return;
  }
  // Overlapped: compute stream  [edge r -> send bufs] -> pcg_b -> reduce -> all-reduce(b) -> join
  //             comm stream           `-> halo send/recv ------------------------------'
  // The next pcg_a is the only reader of the recv buffers and the next edge kernel the next
  // writer of the send buffers; both come after the join.
  comm_->before_pack(local_, streams_);
  for (size_t i = 0; i < local_.size(); ++i) {
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    local_[i]->enqueue_pack(streams_[i]);
  }
  for_each_stream([&](size_t i, size_t u) {
    HIP_CHECK(hipEventRecord(ev_packed_[u], streams_[i]));
    HIP_CHECK(hipStreamWaitEvent(comm_streams_[i], ev_packed_[u], 0));
  });
  poison(comm_streams_);
  comm_->halo(local_, comm_streams_);
  for_each_stream([&](size_t i, size_t u) { HIP_CHECK(hipEventRecord(ev_halo_[u], comm_streams_[i])); });
  for (size_t i = 0; i < local_.size(); ++i) {
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    local_[i]->enqueue_phase_b(streams_[i], /*pack=*/false);
  }
  comm_->allreduce(local_, 1, streams_);
  for_each_stream([&](size_t i, size_t u) { HIP_CHECK(hipStreamWaitEvent(streams_[i], ev_halo_[u], 0)); });
}

void PcgDriver::advance_host_k(long long n) {
  for (auto* s : local_) s->set_host_k(s->host_k() + n);
}

// Captures `len` iterations starting at w-cycle phase `phase` (the phase of the host iteration
// counter now).  The capture enqueues nothing for execution, so the host counters are restored
// afterwards; each launch of the graph advances them by `len`.
namespace {
// PMX_DEBUG_GRAPH=1: one stderr line per graph API step (locating failures inside the HIP runtime)
bool debug_graph() {
  static const bool on = [] {
    const char* e = std::getenv("PMX_DEBUG_GRAPH");
    return e && e[0] == '1';
  }();
  return on;
}
#define PMX_GDBG(...)                      \
  do {                                     \
    if (debug_graph()) {                   \
      std::fprintf(stderr, "[pmx-graph] "); \
      std::fprintf(stderr, __VA_ARGS__);   \
      std::fprintf(stderr, "\n");          \
      std::fflush(stderr);                 \
    }                                      \
  } while (0)
}  // namespace

hipGraphExec_t PcgDriver::build_graph(int phase, int len) {
  TraceRange tr("pmx:build_graph");
  PMX_GDBG("build phase %d len %d", phase, len);
  (void)phase;
  bool single_stream = true;
  for (auto s : streams_) single_stream &= s == streams_[0];
  if (graph_batch_ <= 0 || len <= 0 || !single_stream || !comm_->graph_capturable()) return nullptr;
  for (auto* s : local_)
    if (s->options().check) return nullptr;
  HIP_CHECK(hipSetDevice(local_[0]->device()));
  hipGraph_t g = nullptr;
  if (hipStreamBeginCapture(streams_[0], hipStreamCaptureModeThreadLocal) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  std::vector<long long> k0, b0;
  std::vector<bool> pr0;
  for (auto* s : local_) {
    k0.push_back(s->host_k());
    b0.push_back(s->ca_blocks());
    pr0.push_back(s->ca_primed());
  }
  PMX_CHECK(!halo_pending_, "graph capture with an unjoined ghost exchange");
  PMX_GDBG("capture begun");
  try {
    if (ca_) enqueue_ca(len);
    else for (int k = 0; k < len; ++k) enqueue_one_iteration();
    join_halo();  // a captured batch is self-contained: every forked stream rejoins
  } catch (...) {  // e.g. an aborted communicator: end the capture so the stream stays usable
    halo_pending_ = false;
    for (size_t i = 0; i < local_.size(); ++i) {
      local_[i]->set_host_k(k0[i]);
      local_[i]->set_ca_blocks(b0[i]);
      local_[i]->set_ca_primed(pr0[i]);
    }
    hipGraph_t dead = nullptr;
    (void)hipStreamEndCapture(streams_[0], &dead);
    if (dead) (void)hipGraphDestroy(dead);
    (void)hipGetLastError();
    throw;
  }
  for (size_t i = 0; i < local_.size(); ++i) {
    local_[i]->set_host_k(k0[i]);
    local_[i]->set_ca_blocks(b0[i]);
    local_[i]->set_ca_primed(pr0[i]);
  }
  PMX_GDBG("enqueued; ending capture");
  if (hipStreamEndCapture(streams_[0], &g) != hipSuccess || !g) {
    (void)hipGetLastError();
    return nullptr;
  }
  hipGraphExec_t e = nullptr;
  if (debug_graph()) {
    size_t nn = 0;
    (void)hipGraphGetNodes(g, nullptr, &nn);
    PMX_GDBG("captured %zu nodes; instantiating", nn);
  }
  if (hipGraphInstantiate(&e, g, nullptr, nullptr, 0) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipGraphDestroy(g);
    return nullptr;
  }
  PMX_GDBG("instantiated");
  graphs_.push_back(g);
  execs_.push_back(e);
  return e;
}

hipGraphExec_t PcgDriver::graph_for(int phase, int len) {
  if (graph_batch_ <= 0 || graph_failed_) return nullptr;
  const auto key = std::make_pair(phase, len);
  auto it = exec_by_key_.find(key);
  if (it != exec_by_key_.end()) return it->second;
  hipGraphExec_t e = build_graph(phase, len);
  if (!e) {
    graph_failed_ = true;  // not capturable (multi-stream, comm, check mode): eager from now on
    return nullptr;
  }
  exec_by_key_[key] = e;
  return e;
}

void PcgDriver::note_graph(int len) {
  path_.graph_iters += len;
  auto& v = path_.graph_lengths;
  if (std::find(v.begin(), v.end(), len) == v.end()) v.push_back(len);
}

bool PcgDriver::prepare(int64_t n) {
  TraceRange tr("pmx:prepare");
  const int cyc = graph_period();
  std::vector<long long> k0, b0;
  std::vector<bool> pr0;
  for (auto* s : local_) {
    k0.push_back(s->host_k());
    b0.push_back(s->ca_blocks());
    pr0.push_back(s->ca_primed());
  }
  bool ok = graph_batch_ > 0 && !graph_failed_;
  const int gb = ca_ ? ca_batch() : graph_batch_;
  int64_t done = 0, blocks = 0;  // s-step: blocks enqueued by the batches before `done`
  auto at = [&](int64_t off) {  // host counters as they will be `off` iterations from now
    for (size_t i = 0; i < local_.size(); ++i) {
      local_[i]->set_host_k(k0[i] + off);
      local_[i]->set_ca_blocks(b0[i] + blocks);
      // after a batch the fused s-step schedule is primed
      local_[i]->set_ca_primed(off > 0 ? local_[i]->ca_fused() : bool(pr0[i]));
    }
  };
  auto phase = [&]() { return ca_ ? ca_phase() : int((k0[0] + done) % cyc); };
  const int s = ca_ ? local_[0]->ca_s() : 1;
  while (ok && done + gb <= n) {
    at(done);
    ok = graph_for(phase(), gb) != nullptr;
    done += gb;
    blocks += (gb + s - 1) / s;
  }
  if (ok && done < n) {
    at(done);
    ok = graph_for(phase(), int(n - done)) != nullptr;
  }
  blocks = 0;
  at(0);
  return ok;
}

void PcgDriver::enqueue_eager(int64_t n) {
  if (ca_) enqueue_ca(n);
  else for (int64_t k = 0; k < n; ++k) enqueue_one_iteration();
  path_.eager_iters += n;
  join_halo();
}

void PcgDriver::enqueue_iterations(int64_t n) {
  TraceRange tr("pmx:enqueue_iterations");
  const int cyc = graph_period();
  for (auto* s : local_) PMX_CHECK(s->host_k() == local_[0]->host_k(), "local solvers out of step");
  int64_t done = 0;
  const int gb = ca_ ? ca_batch() : graph_batch_;
  while (done < n) {
    const int len = int(std::min<int64_t>(gb, n - done));
    hipGraphExec_t e = len > 0 ? graph_for(ca_ ? ca_phase() : int(local_[0]->host_k() % cyc), len) : nullptr;
    if (!e) break;
    PMX_GDBG("launch len %d", len);
    HIP_CHECK(hipGraphLaunch(e, streams_[0]));
    PMX_GDBG("launched");
    advance_host_k(len);
    if (ca_) {
      const int s = local_[0]->ca_s();
      for (auto* g : local_) {
        g->set_ca_blocks(g->ca_blocks() + (len + s - 1) / s);
        g->set_ca_primed(g->ca_fused());  // the batch ended with a fused pass
      }
    }
    note_graph(len);
    done += len;
  }
  if (ca_) enqueue_ca(n - done);
  else for (int64_t k = done; k < n; ++k) enqueue_one_iteration();
  path_.eager_iters += n - done;
  join_halo();
}

PcgState PcgDriver::state(int idx) {
  TraceRange tr("pmx:poll_state");
  comm_->check_health();
  return local_[idx]->read_state(streams_[idx]);
}

RunStats PcgDriver::solve(int poll_batches, bool do_init, int64_t ckpt_every,
                          const std::function<void(const PcgState&)>& on_checkpoint) {
  TraceRange tr("pmx:solve");
  RunStats st;
  const double t0 = now_s();
  if (do_init) init();
  const double t1 = now_s();
  st.init_seconds = t1 - t0;
  const int64_t base = ca_ ? ca_batch() : graph_batch_ > 0 ? graph_batch_ : 16;
  const int64_t batch = base * std::max(1, poll_batches);
  const int64_t max_iter = local_[0]->spec().effective_max_iter();
  PcgState s = state(0);
  int64_t last_ckpt = s.it;
  const int64_t budget = max_iter - s.it + 1 + 2 * batch;
  while (!s.done) {
    enqueue_iterations(batch);
    st.launched += batch;
    s = state(0);
    if (s.done) break;
    PMX_CHECK(st.launched <= budget, "device stop flag never raised");
    if (ckpt_every > 0 && on_checkpoint && s.it - last_ckpt >= ckpt_every) {
      synchronize();
      TraceRange trc("pmx:checkpoint");
      on_checkpoint(s);
      last_ckpt = s.it;
    }
  }
  synchronize();
  st.solve_seconds = now_s() - t1;
  st.iters = s.iters;
  st.status = Status(s.status);
  st.diff = s.diff;
  st.nan = s.nan_flag != 0;
  return st;
}

RunStats PcgDriver::profile_phases(int64_t n) {
  TraceRange tr("pmx:profile_phases");
  // Eager iterations with an event after every step that enqueues work, all on the compute
  // stream(s) (no overlap, so each step's time is its own).  Events on the first device's stream;
  // on a multi-device driver the other streams are joined by the collectives.  Single pass:
  // kernel_a = the sweep, kernel_b = 0, reduce = the 5-value reduction, allreduce = red_c, halo =
  // pack + exchange + unpack.  A step with nothing to enqueue (the all-reduce of one rank, the
  // exchange of an undecomposed grid, pcg2's second half in pcg1) records no event: two back-to-back
  // timing events cost ~5 us of marker latency, which would otherwise show up as that bucket's time.
  // s-step PCG: per block pass 1 (or the fused pass) = kernel_a, pass 2 = kernel_b, the reduction(s)
  // and the scalars = reduce, the 21-double all-reduce, and the ghost-row exchange of strips
  RunStats st;
  HIP_CHECK(hipSetDevice(local_[0]->device()));
  hipStream_t s0 = streams_[0];
  enum Bucket { kA = kPhA, kB = kPhB, kRed = kPhRed, kAr = kPhAr, kHalo = kPhHalo };
  const bool ar = comm_->world_size() > 1;
  std::vector<hipEvent_t> ev(size_t(n) * 7 + 16);
  std::vector<int> bucket(ev.size(), -1);
  for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
  size_t ne = 0;
  auto mark = [&](int b) {
    bucket[ne] = b;
    HIP_CHECK(hipEventRecord(ev[ne++], s0));
  };
  auto each = [&](auto&& f) {
    for (size_t i = 0; i < local_.size(); ++i) {
      HIP_CHECK(hipSetDevice(local_[i]->device()));
      f(local_[i], streams_[i]);
    }
    HIP_CHECK(hipSetDevice(local_[0]->device()));
  };
  mark(-1);
  if (ca_) enqueue_ca(n, mark);
  for (int64_t k = 0; k < n && !ca_; ++k) {
    each([](GpuSubdomainSolver* g, hipStream_t s) { g->enqueue_kernel_a(s); });
    mark(kA);
    each([](GpuSubdomainSolver* g, hipStream_t s) { g->enqueue_reduce_a(s); });
    if (!local_[0]->reduction_in_sweep()) mark(kRed);  // else the sweep's own tail: compute
    if (ar) {
      comm_->allreduce(local_, single_pass_ ? 2 : 0, streams_);
      mark(kAr);
    }
    if (!single_pass_) {
      each([](GpuSubdomainSolver* g, hipStream_t s) { g->enqueue_kernel_b(s, true); });
      mark(kB);
      each([](GpuSubdomainSolver* g, hipStream_t s) { g->enqueue_reduce_b(s); });
      mark(kRed);
      if (ar) {
        comm_->allreduce(local_, 1, streams_);
        mark(kAr);
      }
    }
    if (any_nb_) {
      if (single_pass_) halo_exchange_pcg1(streams_, local_[0]->host_k());
      else comm_->halo(local_, streams_);
      mark(kHalo);
    }
  }
  synchronize();
  double t[5] = {0, 0, 0, 0, 0};
  for (size_t i = 1; i < ne; ++i) {
    float v = 0.f;
    HIP_CHECK(hipEventElapsedTime(&v, ev[i - 1], ev[i]));
    t[bucket[i]] += double(v) * 1e-3;
  }
  st.t_kernel_a = t[kA];
  st.t_kernel_b = t[kB];
  st.t_reduce = t[kRed];
  st.t_allreduce = t[kAr];
  st.t_halo = t[kHalo];
  st.t_comm = st.t_allreduce + st.t_halo;
  for (auto& e : ev) (void)hipEventDestroy(e);
  st.launched = n;
  return st;
}

}  // namespace pmx
