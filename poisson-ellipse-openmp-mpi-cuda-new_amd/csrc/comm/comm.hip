// Communication backends for the GPU PCG (§5.8).
//
// Reference: host-staged halos (cudaMemcpy D2H -> blocking MPI_Sendrecv -> H2D, re-allocated
// pageable buffers every call: stage4-mpi+cuda/poisson_mpi_cuda_f.cu:331-500) and three 8-byte
// MPI_Allreduce per iteration (:843,872,893,926).
//
// Here:
//  * RcclComm  — RCCL over xGMI straight from device buffers: ncclSend/ncclRecv pairs inside one
//                ncclGroup for the active halo slots on a split halo communicator, and in-place
//                ncclAllReduce of the PCG scalars.  Single-pass iteration: ONE 40-byte all-reduce
//                (red_c) and up to 8 peers (4 sides with 2 lines of r and p, 4 corners).
//                Two-sweep iteration: 2 all-reduces (1 double, then (sum dw^2, (z,r))) and the 4
//                sides with one line of r (packed by k_edge_r / k_pcg_b).  Graph-capturable.
//  * LocalComm — P subdomains in one process on one device: halos are D2D copies, the
//                all-reduce is a deterministic rank-ordered sum kernel.  The fake cluster used to
//                test multi-rank logic on a 1-GPU box.
//  * SelfComm  — P = 1.
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <sstream>

#include "pmx/common.hpp"
#include "pmx/gpu_solver.hpp"

#define RCCL_CHECK(expr)                                                                \
  do {                                                                                  \
    ncclResult_t pmx_r_ = (expr);                                                       \
    if (pmx_r_ != ncclSuccess)                                                          \
      ::pmx::fail(__FILE__, __LINE__, std::string(#expr " -> ") + ncclGetErrorString(pmx_r_)); \
  } while (0)

namespace pmx {

std::unique_ptr<Comm> Comm::rank_view(int) {
  PMX_CHECK(false, name() << " communicator has no per-rank view (threaded drivers need RCCL)");
  return nullptr;
}

namespace {

// The neighbour's message that pairs with `m` (opposite slot, same field).
const HaloMsg& partner(const HaloMsgs& theirs, const HaloMsg& m) {
  for (int q = 0; q < theirs.n; ++q)
    if (theirs.m[q].slot == opposite_slot(m.slot) && theirs.m[q].field == m.field) {
      PMX_CHECK(theirs.m[q].count == m.count, "ghost message sizes disagree across slot " << m.slot);
      return theirs.m[q];
    }
  PMX_CHECK(false, "no partner message for slot " << m.slot << " field " << m.field);
  return theirs.m[0];
}

class SelfComm final : public Comm {
 public:
  void allreduce(std::vector<GpuSubdomainSolver*>&, int, std::vector<hipStream_t>&) override {}
  void halo(std::vector<GpuSubdomainSolver*>& local, std::vector<hipStream_t>&) override {
    for (auto* s : local) PMX_CHECK(s->geom().nb == 0, "SelfComm used with a decomposed grid");
  }
  std::string name() const override { return "self"; }
  int world_size() const override { return 1; }
};

class LocalComm final : public Comm {
 public:
  explicit LocalComm(std::vector<GpuSubdomainSolver*>& local) : n_(int(local.size())) {
    const int dev = local[0]->device();
    for (size_t i = 0; i < local.size(); ++i) {
      PMX_CHECK(local[i]->device() == dev, "LocalComm needs every subdomain on one device");
      PMX_CHECK(local[i]->sd().rank == int(i), "LocalComm needs local[i].rank == i");
    }
    HIP_CHECK(hipSetDevice(dev));
    // device table of the all-reduce buffers: [which][rank] for red_a, red_b, red_c and the s-step
    // sums (nullptr without the s-step solver: never all-reduced then)
    std::vector<double*> p;
    for (int which = 0; which < 4; ++which)
      for (auto* s : local) p.push_back(s->reduce_buf(which));
    HIP_CHECK(hipMalloc(&ptrs_, p.size() * sizeof(double*)));
    HIP_CHECK(hipMemcpy(ptrs_, p.data(), p.size() * sizeof(double*), hipMemcpyHostToDevice));
  }
  ~LocalComm() override { if (ptrs_) (void)hipFree(ptrs_); }

  void allreduce(std::vector<GpuSubdomainSolver*>&, int which,
                 std::vector<hipStream_t>& streams) override {
    if (n_ == 1) return;
    launch_local_allreduce(ptrs_ + which * n_, n_, GpuSubdomainSolver::reduce_len(which), streams[0]);
  }
  void halo(std::vector<GpuSubdomainSolver*>& local, std::vector<hipStream_t>& streams) override {
    for (auto* s : local) {
      const HaloMsgs mine = s->halo_msgs();
      for (int q = 0; q < mine.n; ++q) {
        const HaloMsg& m = mine.m[q];
        const HaloMsg& o = partner(local[m.peer]->halo_msgs(), m);
        HIP_CHECK(hipMemcpyAsync(m.recv, o.send, size_t(m.count) * s->layout().elem, hipMemcpyDeviceToDevice,
                                 streams[0]));
      }
    }
  }
  bool direct_rows() const override { return true; }
  std::string name() const override { return "local"; }
  int world_size() const override { return n_; }

 private:
  int n_;
  double** ptrs_ = nullptr;
};

// Shared by an RcclComm and its rank views: set once ncclCommAbort has released the communicators.
// Every entry point checks it first, so a driver thread that returns from a blocked call after
// another thread's abort gets an error instead of touching freed handles.
using AbortFlag = std::shared_ptr<std::atomic<bool>>;

void require_live(const AbortFlag& f) {
  PMX_CHECK(!f->load(), "RCCL communicator was aborted after a failure on another driver thread; this "
                        "session cannot communicate any more");
}

void check_async(ncclComm_t c) {
  ncclResult_t async = ncclSuccess;
  RCCL_CHECK(ncclCommGetAsyncError(c, &async));
  if (async != ncclSuccess && async != ncclInProgress)
    ::pmx::fail(__FILE__, __LINE__, std::string("RCCL asynchronous error: ") + ncclGetErrorString(async));
}

// The halo send/recv pairs of one rank (GpuSubdomainSolver::halo_msgs order: by slot, then field;
// a neighbour issues its partner messages in the same order, so RCCL pairs them per peer).
void rccl_halo_calls(GpuSubdomainSolver* s, ncclComm_t comm, hipStream_t stream) {
  const ncclDataType_t t = s->layout().elem == 8 ? ncclFloat64 : ncclFloat32;
  const HaloMsgs ms = s->halo_msgs();
  for (int q = 0; q < ms.n; ++q) {
    const HaloMsg& m = ms.m[q];
    RCCL_CHECK(ncclSend(m.send, size_t(m.count), t, m.peer, comm, stream));
    RCCL_CHECK(ncclRecv(m.recv, size_t(m.count), t, m.peer, comm, stream));
  }
}

// See make_loopback_comm.
// Loopback exchange: ONE launch writes every receive span of the exchange, a workgroup per
// message -- the shape of an RCCL send/recv group (one kernel, a channel block per peer), not of
// per-message blits, which queue hundreds of workgroups behind a running sweep (profiles/r4/loopback).
// `delay` (100 MHz ticks, PMX_LOOPBACK_HALO_US) holds each block resident first, standing in for
// the xGMI transfer; the all-reduce stand-in (PMX_LOOPBACK_AR_US) is the same kernel with no spans.
struct LoopbackSpans {
  unsigned* dst[2 * kHaloSlots];
  unsigned words[2 * kHaloSlots];
  int n;
  unsigned long long delay;
};

__global__ void __launch_bounds__(256) k_loopback_fill(LoopbackSpans sp) {
  if (sp.delay) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < sp.delay) __builtin_amdgcn_s_sleep(8);
  }
  if (int(blockIdx.x) >= sp.n) return;
  unsigned* d = sp.dst[blockIdx.x];
  const unsigned n = sp.words[blockIdx.x];
  for (unsigned i = threadIdx.x; i < n; i += blockDim.x) d[i] = 0u;  // Dirichlet zero ghosts
}

unsigned long long loopback_ticks(const char* env) {
  const char* v = study_env(env);  // loopback stand-in delays are a study setting
  return v && v[0] ? static_cast<unsigned long long>(std::atof(v) * 100.0) : 0ull;  // 100 MHz clock
}

class LoopbackComm final : public Comm {
 public:
  void allreduce(std::vector<GpuSubdomainSolver*>&, int, std::vector<hipStream_t>& streams) override {
    if (!ar_delay_) return;
    LoopbackSpans sp{};
    sp.delay = ar_delay_;
    hipLaunchKernelGGL(k_loopback_fill, dim3(1), dim3(64), 0, streams[0], sp);
    HIP_CHECK(hipGetLastError());
  }
  void halo(std::vector<GpuSubdomainSolver*>& local, std::vector<hipStream_t>& streams) override {
    PMX_CHECK(local.size() == 1, "the loopback comm stands for one rank");
    const HaloMsgs ms = local[0]->halo_msgs();
    const size_t elem = local[0]->layout().elem;
    LoopbackSpans sp{};
    sp.delay = halo_delay_;
    // every ghost becomes a Dirichlet zero: each rank solves a well-posed problem on its own block
    for (int q = 0; q < ms.n; ++q) {
      const size_t bytes = size_t(ms.m[q].count) * elem;
      PMX_CHECK(bytes % 4 == 0 && reinterpret_cast<uintptr_t>(ms.m[q].recv) % 4 == 0,
                "loopback: receive span not word aligned");
      sp.dst[sp.n] = static_cast<unsigned*>(ms.m[q].recv);
      sp.words[sp.n++] = static_cast<unsigned>(bytes / 4);
    }
    if (sp.n == 0) return;
    hipLaunchKernelGGL(k_loopback_fill, dim3(sp.n), dim3(256), 0, streams[0], sp);
    HIP_CHECK(hipGetLastError());
  }
  bool prefers_split() const override { return true; }  // as RCCL
  bool direct_rows() const override { return true; }
  std::string name() const override { return "loopback"; }
  int world_size() const override { return 1; }

 private:
  unsigned long long halo_delay_ = loopback_ticks("PMX_LOOPBACK_HALO_US");
  unsigned long long ar_delay_ = loopback_ticks("PMX_LOOPBACK_AR_US");
};

// One local rank of an RcclComm, driven by its own host thread: its collectives need no
// ncclGroupStart/End across local ranks (RCCL matches them per communicator, whichever thread
// issues them); the send/recv pairs of its halo slots still form one group.
class RcclRankView final : public Comm {
 public:
  RcclRankView(ncclComm_t comm, ncclComm_t halo_comm, int nranks, bool capturable, Comm* owner, AbortFlag aborted)
      : comm_(comm), halo_comm_(halo_comm), nranks_(nranks), capturable_(capturable), owner_(owner),
        aborted_(std::move(aborted)) {}
  void abort() override { owner_->abort(); }  // every rank view of the process shares the fate
  bool prefers_split() const override { return true; }
  void allreduce(std::vector<GpuSubdomainSolver*>& local, int which,
                 std::vector<hipStream_t>& streams) override {
    require_live(aborted_);
    PMX_CHECK(local.size() == 1, "a rank view drives one subdomain");
    double* buf = local[0]->reduce_buf(which);
    RCCL_CHECK(ncclAllReduce(buf, buf, GpuSubdomainSolver::reduce_len(which), ncclFloat64, ncclSum, comm_,
                             streams[0]));
  }
  void halo(std::vector<GpuSubdomainSolver*>& local, std::vector<hipStream_t>& streams) override {
    require_live(aborted_);
    PMX_CHECK(local.size() == 1, "a rank view drives one subdomain");
    RCCL_CHECK(ncclGroupStart());
    rccl_halo_calls(local[0], halo_comm_, streams[0]);
    RCCL_CHECK(ncclGroupEnd());
  }
  bool graph_capturable() const override { return capturable_; }
  bool direct_rows() const override { return true; }
  void check_health() override {
    require_live(aborted_);
    check_async(comm_);
    if (halo_comm_ != comm_) check_async(halo_comm_);
  }
  std::string name() const override { return "rccl"; }
  int world_size() const override { return nranks_; }

 private:
  ncclComm_t comm_, halo_comm_;
  int nranks_;
  bool capturable_;
  Comm* owner_;
  AbortFlag aborted_;
};

class RcclComm final : public Comm {
 public:
  RcclComm(const std::string& uid, int nranks, const std::vector<int>& ranks,
           const std::vector<int>& devices, bool capturable, bool split_halo)
      : nranks_(nranks), capturable_(capturable), split_(split_halo) {
    PMX_CHECK(uid.size() == sizeof(ncclUniqueId), "bad ncclUniqueId size " << uid.size());
    PMX_CHECK(ranks.size() == devices.size() && !ranks.empty(), "ranks/devices mismatch");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    comms_.resize(ranks.size());
    if (ranks.size() == 1) {
      HIP_CHECK(hipSetDevice(devices[0]));
      RCCL_CHECK(ncclCommInitRank(&comms_[0], nranks, id, ranks[0]));
    } else {
      RCCL_CHECK(ncclGroupStart());
      for (size_t i = 0; i < ranks.size(); ++i) {
        HIP_CHECK(hipSetDevice(devices[i]));
        RCCL_CHECK(ncclCommInitRank(&comms_[i], nranks, id, ranks[i]));
      }
      RCCL_CHECK(ncclGroupEnd());
    }
    if (!split_halo) {  // serialized schedule: one communicator for everything
      halo_comms_ = comms_;
      return;
    }
    // A second communicator (same ranks) carries the halos, so the ghost exchange on the comm
    // stream and the all-reduce on the compute stream never queue behind each other.
    halo_comms_.resize(comms_.size());
    RCCL_CHECK(ncclGroupStart());
    for (size_t i = 0; i < comms_.size(); ++i) {
      HIP_CHECK(hipSetDevice(devices[i]));
      RCCL_CHECK(ncclCommSplit(comms_[i], 0, ranks[i], &halo_comms_[i], nullptr));
    }
    RCCL_CHECK(ncclGroupEnd());
  }
  ~RcclComm() override {
    if (aborted_->load()) return;  // ncclCommAbort already released them
    if (split_) for (auto c : halo_comms_) (void)ncclCommDestroy(c);
    for (auto c : comms_) (void)ncclCommDestroy(c);
  }
  void abort() override {
    if (aborted_->exchange(true)) return;
    if (split_) for (auto c : halo_comms_) (void)ncclCommAbort(c);
    for (auto c : comms_) (void)ncclCommAbort(c);
  }
  bool prefers_split() const override { return true; }

  void allreduce(std::vector<GpuSubdomainSolver*>& local, int which,
                 std::vector<hipStream_t>& streams) override {
    require_live(aborted_);
    RCCL_CHECK(ncclGroupStart());
    for (size_t i = 0; i < local.size(); ++i) {
      double* buf = local[i]->reduce_buf(which);
      RCCL_CHECK(ncclAllReduce(buf, buf, GpuSubdomainSolver::reduce_len(which), ncclFloat64, ncclSum,
                               comms_[i], streams[i]));
    }
    RCCL_CHECK(ncclGroupEnd());
  }

  void halo(std::vector<GpuSubdomainSolver*>& local, std::vector<hipStream_t>& streams) override {
    require_live(aborted_);
    RCCL_CHECK(ncclGroupStart());
    for (size_t i = 0; i < local.size(); ++i) rccl_halo_calls(local[i], halo_comms_[i], streams[i]);
    RCCL_CHECK(ncclGroupEnd());
  }

  bool graph_capturable() const override { return capturable_; }
  bool direct_rows() const override { return true; }
  std::unique_ptr<Comm> rank_view(int i) override {
    PMX_CHECK(i >= 0 && i < int(comms_.size()), "rank view index");
    return std::make_unique<RcclRankView>(comms_[size_t(i)], halo_comms_[size_t(i)], nranks_, capturable_, this,
                                          aborted_);
  }
  void check_health() override {
    require_live(aborted_);
    for (auto c : comms_) check_async(c);
    if (split_) for (auto c : halo_comms_) check_async(c);
  }
  std::string name() const override { return "rccl"; }
  int world_size() const override { return nranks_; }

 private:
  int nranks_;
  bool capturable_;
  bool split_;                          // halo_comms_ are their own communicators
  std::vector<ncclComm_t> comms_;       // scalar all-reduces (compute stream)
  std::vector<ncclComm_t> halo_comms_;  // ghost exchange (comm stream when overlapped); == comms_ unsplit
  AbortFlag aborted_ = std::make_shared<std::atomic<bool>>(false);
};

// See make_recording_comm.
class RecordingComm final : public Comm {
 public:
  RecordingComm(std::vector<CommEvent>* log, int world, bool split_halo)
      : log_(log), world_(world), halo_id_(split_halo ? 1 : 0) {}
  void allreduce(std::vector<GpuSubdomainSolver*>& local, int which, std::vector<hipStream_t>& streams) override {
    PMX_CHECK(local.size() == 1, "a recording comm stands for one rank");
    log_->push_back({0, "allreduce", GpuSubdomainSolver::reduce_len(which), -1, sid(streams)});
  }
  void halo(std::vector<GpuSubdomainSolver*>& local, std::vector<hipStream_t>& streams) override {
    PMX_CHECK(local.size() == 1, "a recording comm stands for one rank");
    const long long st = sid(streams);
    log_->push_back({halo_id_, "group_start", 0, -1, st});
    const HaloMsgs ms = local[0]->halo_msgs();
    for (int q = 0; q < ms.n; ++q) {  // the order RcclComm::halo issues them
      log_->push_back({halo_id_, "send", ms.m[q].count, ms.m[q].peer, st});
      log_->push_back({halo_id_, "recv", ms.m[q].count, ms.m[q].peer, st});
    }
    log_->push_back({halo_id_, "group_end", 0, -1, st});
  }
  bool prefers_split() const override { return true; }
  bool direct_rows() const override { return true; }
  std::string name() const override { return "recording"; }
  int world_size() const override { return world_; }

 private:
  static long long sid(const std::vector<hipStream_t>& s) {
    return static_cast<long long>(reinterpret_cast<uintptr_t>(s.at(0)));
  }
  std::vector<CommEvent>* log_;
  int world_;
  int halo_id_;
};

}  // namespace

std::unique_ptr<Comm> make_self_comm() { return std::make_unique<SelfComm>(); }
std::unique_ptr<Comm> make_loopback_comm() { return std::make_unique<LoopbackComm>(); }

std::unique_ptr<Comm> make_recording_comm(std::vector<CommEvent>* log, int world, bool split_halo) {
  return std::make_unique<RecordingComm>(log, world, split_halo);
}

std::unique_ptr<Comm> make_local_comm(std::vector<GpuSubdomainSolver*>& local) {
  return std::make_unique<LocalComm>(local);
}

std::unique_ptr<Comm> make_rccl_comm(const std::string& unique_id, int nranks,
                                     const std::vector<int>& ranks, const std::vector<int>& devices,
                                     bool capturable, bool split_halo) {
  return std::make_unique<RcclComm>(unique_id, nranks, ranks, devices, capturable, split_halo);
}

std::string rccl_unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

}  // namespace pmx
