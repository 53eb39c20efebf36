// IpcComm: a device-resident multi-process transport without RCCL (SURVEY §5.8 "peer-mapped direct
// halo stores"; verdict r2 item 6).
//
// One rank per process, ranks on one GPU (the 1-GPU test box) or on several (peer access over
// xGMI): every rank exports its comm arena (the send/recv halo slots and the PcgState scalars) and a
// small IpcBlock of flags with hipIpcGetMemHandle, opens its peers' with hipIpcOpenMemHandle, and
// then moves data with its own kernels, ordered by monotonic epoch flags:
//
//   all-reduce   publish the local sums into IpcBlock::pub[c & 1], raise red_flag = c, wait until
//                every rank's red_flag >= c, sum the published values in rank order (the LocalComm
//                order: results are bitwise those of LocalComm / one process with P subdomains)
//   halo         before packing exchange e: wait until every neighbour acknowledged exchange e-1
//                (ack >= e-1 posts); pack (the solver's own kernels); post: halo_flag = e;
//                pull: wait for each neighbour's halo_flag >= e, copy its send slot into our recv
//                slot; ack[slot] = e; unpack (the solver's own kernel)
//
// The parity-indexed pub[] and the acks are what make the schedule race-free with the overlapped
// and split sweeps: a rank may be a whole sweep ahead of a neighbour, never two exchanges.  Waits
// spin on system-scope acquire loads with a wall-clock timeout (PMX_IPC_TIMEOUT_MS, default 20 s):
// on expiry the kernel records the error, stops the solve (done flag, status breakdown) and
// check_health() throws, so a dead peer cannot hang the GPU.  Remote data is read with
// non-temporal loads after the acquire (no stale cache line of an earlier epoch is reused).
// Graph-capturable: every operation is a kernel with fixed arguments, epochs live on the device.
//
// Memory model across devices (peers on other GPUs over xGMI, or processes sharing one GPU):
//  * Flags (IpcBlock) live in UNCACHED device memory (hipExtMallocWithFlags(hipDeviceMallocUncached),
//    MTYPE UC): every load and store of a flag goes to the owning device's memory, whichever GPU
//    issues it, so a spinning peer never polls a line cached in its own (per-XCD, non-coherent) L2
//    and a flag store is visible to every device once it completes.  Coarse-grained hipMalloc
//    memory would only be coherent where the caches happen to be written back / invalidated;
//    PMX_IPC_COARSE=1 restores it (A/B).
//  * Payload (the send slots of the comm arena, coarse-grained, read by peers in place): written by
//    the pack kernel with plain stores.  Every kernel boundary writes the XCD L2s back (gfx950:
//    the per-XCD L2s are not coherent, so the end-of-kernel release covers all of them), and
//    k_ipc_post -- a later kernel in stream order -- raises the flag with a system-scope release
//    (buffer_wbl2 sc0 sc1 + the store): when a peer sees the flag, the payload is in memory.
//  * The reader acquires at system scope (ld_acq: the load plus buffer_inv sc0 sc1 -- its L1 and its
//    L2's lines of non-local memory are invalidated) and then reads the payload with non-temporal
//    loads: no line of an earlier epoch can be served from its caches.
//  * Reuse: a rank packs exchange e only after every neighbour acknowledged e-1 (k_ipc_wait_acks),
//    so a payload is never overwritten while a peer may still read it.
//  * Same-GPU ranks (the one-GPU box) take the same path; there the peer is the same L2 hierarchy
//    and the uncached flags only cost a few hundred ns per poll.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pmx/common.hpp"
#include "pmx/gpu_solver.hpp"

namespace pmx {

namespace {

struct alignas(256) IpcBlock {
  unsigned long long red_flag;   // all-reduces published by this rank
  unsigned long long halo_flag;  // ghost exchanges posted by this rank
  unsigned long long red_count;  // this rank's own counters (only its kernels touch them)
  unsigned long long halo_count;
  unsigned long long ack[kHaloSlots];  // exchanges pulled from the neighbour across slot s
  int err;                             // 1 = a wait timed out
  int pad;
  double pub[2][24];                   // published local sums, by all-reduce parity
};
constexpr int kIpcMaxReduce = 24;

constexpr int kMaxIpcRanks = 64;

struct IpcPeers {
  IpcBlock* all[kMaxIpcRanks];  // every rank's block (ours included), IPC-mapped
  IpcBlock* nbr[kHaloSlots];    // block of the neighbour across slot s (nullptr: none)
  const void* src[kHaloSlots];  // its send slot facing us (opposite slot), IPC-mapped
  void* dst[kHaloSlots];        // our recv slot
  int len[kHaloSlots];          // elements
};

__device__ inline unsigned long long ld_acq(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void st_rel(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Spin until *flag >= target or the wall clock (100 MHz) passes the deadline.  On timeout: record
// the error and stop the solve.  Called by one lane.
__device__ bool wait_ge(const unsigned long long* flag, unsigned long long target, long long timeout_ticks,
                        IpcBlock* own, PcgState* S) {
  const long long t0 = wall_clock64();
  while (ld_acq(flag) < target) {
    if (wall_clock64() - t0 > timeout_ticks) {
      __hip_atomic_store(&own->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      S->nan_flag = 1;
      S->status = int(Status::kBreakdown);
      S->done = 1;
      return false;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  return true;
}

__global__ void k_ipc_allreduce(IpcPeers P, int world, int me, double* buf, int n, PcgState* S,
                                long long timeout) {
  if (threadIdx.x != 0) return;
  IpcBlock* own = P.all[me];
  const unsigned long long c = own->red_count + 1;
  own->red_count = c;
  const int par = int(c & 1);
  for (int q = 0; q < n; ++q) own->pub[par][q] = buf[q];
  st_rel(&own->red_flag, c);
  for (int r = 0; r < world; ++r)
    if (!wait_ge(&P.all[r]->red_flag, c, timeout, own, S)) return;
  for (int q = 0; q < n; ++q) {  // rank order, as LocalComm
    double s = 0.0;
    for (int r = 0; r < world; ++r) s += __builtin_nontemporal_load(&P.all[r]->pub[par][q]);
    buf[q] = s;
  }
}

// before packing exchange e = halo_count + 1: every neighbour pulled exchange e - 1
__global__ void k_ipc_wait_acks(IpcPeers P, int me, PcgState* S, long long timeout) {
  if (threadIdx.x != 0) return;
  IpcBlock* own = P.all[me];
  const unsigned long long posted = own->halo_count;
  for (int s = 0; s < kHaloSlots; ++s)
    if (P.nbr[s] && !wait_ge(&P.nbr[s]->ack[opposite_slot(s)], posted, timeout, own, S)) return;
}

__global__ void k_ipc_post(IpcPeers P, int me) {
  if (threadIdx.x != 0) return;
  IpcBlock* own = P.all[me];
  const unsigned long long c = own->halo_count + 1;
  own->halo_count = c;
  st_rel(&own->halo_flag, c);  // the pack kernel before us has finished: its slots are in memory
}

// grid (blocks per slot, 8 slots): every block's lane 0 waits for the neighbour's post, then the
// block copies its share of the slot (non-temporal loads of the remote slot)
template <typename T>
__global__ void __launch_bounds__(256) k_ipc_pull(IpcPeers P, int me, PcgState* S, long long timeout) {
  const int s = blockIdx.y;
  if (!P.nbr[s]) return;
  __shared__ int ok;
  IpcBlock* own = P.all[me];
  if (threadIdx.x == 0) ok = wait_ge(&P.nbr[s]->halo_flag, own->halo_count, timeout, own, S) ? 1 : 0;
  __syncthreads();
  if (!ok) return;
  const T* src = static_cast<const T*>(P.src[s]);
  T* dst = static_cast<T*>(P.dst[s]);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < P.len[s]; i += gridDim.x * 256)
    dst[i] = __builtin_nontemporal_load(src + i);
}

// s-step strips (direct rows): the spans of one exchange.  Pack: our edge rows -> our staging buffer
// (nbr = nullptr, no wait); pull: the neighbour's staging buffer -> our ghost rows (after its post).
struct IpcSpans {
  const IpcBlock* nbr[4];
  const void* src[4];
  void* dst[4];
  int len[4];
};

template <typename T>
__global__ void __launch_bounds__(256) k_ipc_pull_spans(IpcPeers P, IpcSpans S4, int me, PcgState* S,
                                                        long long timeout) {
  const int q = blockIdx.y;
  __shared__ int ok;
  IpcBlock* own = P.all[me];
  if (threadIdx.x == 0) ok = !S4.nbr[q] || wait_ge(&S4.nbr[q]->halo_flag, own->halo_count, timeout, own, S) ? 1 : 0;
  __syncthreads();
  if (!ok) return;
  const T* src = static_cast<const T*>(S4.src[q]);
  T* dst = static_cast<T*>(S4.dst[q]);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < S4.len[q]; i += gridDim.x * 256)
    dst[i] = __builtin_nontemporal_load(src + i);
}

__global__ void k_ipc_ack(IpcPeers P, int me) {
  if (threadIdx.x != 0) return;
  IpcBlock* own = P.all[me];
  for (int s = 0; s < kHaloSlots; ++s)
    if (P.nbr[s]) st_rel(&own->ack[s], own->halo_count);
}

std::string handle_bytes(void* p) {
  hipIpcMemHandle_t h;
  HIP_CHECK(hipIpcGetMemHandle(&h, p));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void* open_handle(const std::string& b) {
  PMX_CHECK(b.size() == sizeof(hipIpcMemHandle_t), "bad IPC handle size " << b.size());
  hipIpcMemHandle_t h;
  std::memcpy(&h, b.data(), sizeof(h));
  void* p = nullptr;
  HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return p;
}

class IpcComm final : public Comm {
 public:
  IpcComm(GpuSubdomainSolver* local, int world) : local_(local), world_(world) {
    PMX_CHECK(world >= 1 && world <= kMaxIpcRanks, "IpcComm supports 1.." << kMaxIpcRanks << " ranks");
    HIP_CHECK(hipSetDevice(local->device()));
    const char* coarse = study_env("PMX_IPC_COARSE");
    if (coarse && coarse[0] == '1')
      HIP_CHECK(hipMalloc(&block_, sizeof(IpcBlock)));
    else  // flags every device reads and writes coherently (see the memory-model notes above)
      HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&block_), sizeof(IpcBlock), hipDeviceMallocUncached));
    HIP_CHECK(hipMemset(block_, 0, sizeof(IpcBlock)));
    if (ca_) {
      const HaloMsgs ms = local_->ca_halo_msgs(0);
      ca_count_ = ms.n ? ms.m[0].count : 0;
      HIP_CHECK(hipMalloc(&ca_buf_, std::max<size_t>(256, size_t(4) * size_t(ca_count_) * sizeof(double))));
    }
    const char* t = std::getenv("PMX_IPC_TIMEOUT_MS");
    timeout_ = (t && t[0] ? std::atoll(t) : 20000LL) * 100000LL;  // wall_clock64: 100 MHz
  }
  ~IpcComm() override {
    (void)hipSetDevice(local_->device());
    (void)hipDeviceSynchronize();
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    if (block_) (void)hipFree(block_);
    if (ca_buf_) (void)hipFree(ca_buf_);
  }

  // this rank's exports: device id, arena handle, block handle
  std::string export_handles() const {
    const int dev = local_->device();
    std::string out(reinterpret_cast<const char*>(&dev), sizeof(dev));
    out += handle_bytes(reinterpret_cast<void*>(local_->arena_ptr()));
    out += handle_bytes(block_);
    if (ca_) out += handle_bytes(ca_buf_);  // s-step strips: the staging buffer of our edge rows
    return out;
  }

  // every rank's export_handles(), indexed by rank
  void attach(const std::vector<std::string>& peers) {
    PMX_CHECK(int(peers.size()) == world_, "IpcComm::attach needs one export per rank");
    const int me = local_->sd().rank;
    const size_t hs = sizeof(hipIpcMemHandle_t);
    std::vector<char*> arenas(size_t(world_), nullptr);
    std::memset(&P_, 0, sizeof(P_));
    const CommLayout& L0 = local_->layout();
    for (int r = 0; r < world_; ++r) {
      const std::string& e = peers[size_t(r)];
      PMX_CHECK(e.size() == sizeof(int) + 2 * hs + (ca_ ? hs : 0), "bad IPC export of rank " << r);
      if (r == me) {
        arenas[size_t(r)] = reinterpret_cast<char*>(local_->arena_ptr());
        P_.all[r] = block_;
        continue;
      }
      int dev = 0;
      std::memcpy(&dev, e.data(), sizeof(int));
      if (dev != local_->device()) {  // peer GPU: map its memory over xGMI
        const hipError_t pe = hipDeviceEnablePeerAccess(dev, 0);
        if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) HIP_CHECK(pe);
        (void)hipGetLastError();
      }
      arenas[size_t(r)] = static_cast<char*>(open_handle(e.substr(sizeof(int), hs)));
      opened_.push_back(arenas[size_t(r)]);
      P_.all[r] = static_cast<IpcBlock*>(open_handle(e.substr(sizeof(int) + hs, hs)));
      opened_.push_back(P_.all[r]);
      if (ca_) {
        for (int s = 0; s < 2; ++s) {
          if (L0.peer[s] != r) continue;
          ca_peer_buf_[s] = static_cast<char*>(open_handle(e.substr(sizeof(int) + 2 * hs, hs)));
          opened_.push_back(ca_peer_buf_[s]);
        }
      }
    }
    const CommLayout& L = local_->layout();
    for (int s = 0; s < kHaloSlots; ++s) {
      if (!L.active(s)) continue;
      const int q = L.peer[s];
      PMX_CHECK(q >= 0 && q < world_ && q != me, "IpcComm: bad neighbour " << q << " on slot " << s);
      // the neighbour's layout mirrors ours across the shared edge: its slot opposite(s) carries
      // the same number of elements at its own send offset, which a rank computes locally from the
      // neighbour's subdomain (comm_layout is a pure function of it)
      const Subdomain nsd = decompose_2d(local_->spec().M, local_->spec().N, local_->sd().grid, q);
      const CommLayout NL = GpuSubdomainSolver::comm_layout(nsd, local_->options().dtype, local_->single_pass() || local_->ca(),
                                                            local_->ca() ? local_->ca_ghost_rows() : 0);
      const int os = opposite_slot(s);
      PMX_CHECK(NL.edge_len[os] == L.edge_len[s], "IpcComm: slot lengths disagree with rank " << q);
      P_.nbr[s] = P_.all[q];
      P_.src[s] = arenas[size_t(q)] + NL.send_off[os];
      P_.dst[s] = local_->recv_dev(s);
      P_.len[s] = L.edge_len[s];
      maxlen_ = std::max(maxlen_, L.edge_len[s]);
    }
    attached_ = true;
  }

  void allreduce(std::vector<GpuSubdomainSolver*>& local, int which, std::vector<hipStream_t>& streams) override {
    require(local);
    if (world_ == 1) return;
    PMX_CHECK(GpuSubdomainSolver::reduce_len(which) <= kIpcMaxReduce, "IpcComm: all-reduce longer than IpcBlock::pub");
    hipLaunchKernelGGL(k_ipc_allreduce, dim3(1), dim3(64), 0, streams[0], P_, world_, local_->sd().rank,
                       local_->reduce_buf(which), GpuSubdomainSolver::reduce_len(which), local_->state_dev(),
                       timeout_);
    HIP_CHECK(hipGetLastError());
  }
  void before_pack(std::vector<GpuSubdomainSolver*>& local, std::vector<hipStream_t>& streams) override {
    require(local);
    if (maxlen_ == 0) return;
    hipLaunchKernelGGL(k_ipc_wait_acks, dim3(1), dim3(64), 0, streams[0], P_, local_->sd().rank,
                       local_->state_dev(), timeout_);
    HIP_CHECK(hipGetLastError());
  }
  void halo(std::vector<GpuSubdomainSolver*>& local, std::vector<hipStream_t>& streams) override {
    require(local);
    if (maxlen_ == 0) return;
    const int me = local_->sd().rank;
    if (ca_) {
      // the s edge rows of z and p of the current set: wait until every neighbour pulled the last
      // exchange, stage ours, post, pull the neighbours' staged rows into our ghost rows, acknowledge.
      // (Mapping the neighbours' whole field allocations instead hung hipIpcOpenMemHandle with 4
      // ranks of a 16384^2 grid on one GPU; the staging copy is ~1.5 MB per block.)
      const HaloMsgs ms = local_->halo_msgs();
      IpcSpans pack{}, pull{};
      int maxc = 0;
      PMX_CHECK(ms.n <= 4, "IpcComm: more than 4 s-step spans");
      for (int q = 0; q < ms.n; ++q) {
        const HaloMsg& m = ms.m[q];
        PMX_CHECK(m.count == ca_count_ && ca_peer_buf_[m.slot] && P_.nbr[m.slot], "IpcComm: bad s-step span on slot " << m.slot);
        const size_t el = local_->layout().elem;  // fp64 or fp32 fields
        const size_t mine = size_t(m.slot * 2 + m.field) * size_t(ca_count_) * el;
        const size_t theirs = size_t(opposite_slot(m.slot) * 2 + m.field) * size_t(ca_count_) * el;
        pack.nbr[q] = nullptr;
        pack.src[q] = m.send;
        pack.dst[q] = ca_buf_ + mine;
        pack.len[q] = m.count;
        pull.nbr[q] = P_.nbr[m.slot];
        pull.src[q] = ca_peer_buf_[m.slot] + theirs;
        pull.dst[q] = m.recv;
        pull.len[q] = m.count;
        maxc = std::max(maxc, m.count);
      }
      if (ms.n) {
        const dim3 grid(std::max(1, std::min(64, (maxc + 255) / 256)), ms.n);
        hipLaunchKernelGGL(k_ipc_wait_acks, dim3(1), dim3(64), 0, streams[0], P_, me, local_->state_dev(), timeout_);
        auto spans = [&](const IpcSpans& sp) {
          if (local_->layout().elem == 8)
            hipLaunchKernelGGL(k_ipc_pull_spans<double>, grid, dim3(256), 0, streams[0], P_, sp, me,
                               local_->state_dev(), timeout_);
          else
            hipLaunchKernelGGL(k_ipc_pull_spans<float>, grid, dim3(256), 0, streams[0], P_, sp, me,
                               local_->state_dev(), timeout_);
        };
        spans(pack);
        hipLaunchKernelGGL(k_ipc_post, dim3(1), dim3(64), 0, streams[0], P_, me);
        spans(pull);
        hipLaunchKernelGGL(k_ipc_ack, dim3(1), dim3(64), 0, streams[0], P_, me);
      }
      HIP_CHECK(hipGetLastError());
      return;
    }
    hipLaunchKernelGGL(k_ipc_post, dim3(1), dim3(64), 0, streams[0], P_, me);
    const int bx = std::max(1, std::min(64, (maxlen_ + 255) / 256));
    if (local_->layout().elem == 8)
      hipLaunchKernelGGL(k_ipc_pull<double>, dim3(bx, kHaloSlots), dim3(256), 0, streams[0], P_, me,
                         local_->state_dev(), timeout_);
    else
      hipLaunchKernelGGL(k_ipc_pull<float>, dim3(bx, kHaloSlots), dim3(256), 0, streams[0], P_, me,
                         local_->state_dev(), timeout_);
    hipLaunchKernelGGL(k_ipc_ack, dim3(1), dim3(64), 0, streams[0], P_, me);
    HIP_CHECK(hipGetLastError());
  }
  void check_health() override {
    int err = 0;
    HIP_CHECK(hipMemcpy(&err, &block_->err, sizeof(int), hipMemcpyDeviceToHost));
    PMX_CHECK(err == 0, "IPC transport: a wait for a peer rank timed out (PMX_IPC_TIMEOUT_MS); the solve "
                        "was stopped");
  }
  bool prefers_split() const override { return true; }
  bool direct_rows() const override { return ca_; }  // s-step strips: spans of the fields (staged)
  std::string name() const override { return "ipc"; }
  int world_size() const override { return world_; }

 private:
  void require(std::vector<GpuSubdomainSolver*>& local) const {
    PMX_CHECK(attached_, "IpcComm used before attach()");
    PMX_CHECK(local.size() == 1 && local[0] == local_, "IpcComm drives exactly its own rank");
  }
  GpuSubdomainSolver* local_;
  int world_;
  IpcBlock* block_ = nullptr;
  IpcPeers P_{};
  std::vector<void*> opened_;
  int maxlen_ = 0;
  long long timeout_ = 0;
  bool attached_ = false;
  // s-step strips: each x neighbour's fields allocation (mapped) and its span offsets [set][slot][field]
  // s-step strips: our staging buffer of edge rows ([slot][field] spans of ca_count_ elements) and each
  // x neighbour's (mapped)
  bool ca_ = local_->ca() && local_->can_direct_rows();  // s-step strips (2-D blocks: the packed slots)
  int ca_count_ = 0;
  char* ca_buf_ = nullptr;
  char* ca_peer_buf_[2] = {nullptr, nullptr};
};

}  // namespace

std::unique_ptr<Comm> make_ipc_comm(GpuSubdomainSolver* local, int world) {
  return std::make_unique<IpcComm>(local, world);
}
std::string ipc_export(Comm* c) {
  auto* ic = dynamic_cast<IpcComm*>(c);
  PMX_CHECK(ic, "not an IPC communicator");
  return ic->export_handles();
}
void ipc_attach(Comm* c, const std::vector<std::string>& peers) {
  auto* ic = dynamic_cast<IpcComm*>(c);
  PMX_CHECK(ic, "not an IPC communicator");
  ic->attach(peers);
}

}  // namespace pmx
