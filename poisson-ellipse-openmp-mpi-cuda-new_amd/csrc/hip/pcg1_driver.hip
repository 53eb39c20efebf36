// pcg1's schedules on decomposed grids (GpuOptions::algo 1; kernels in pcg1_kernels.hip): the
// radius-2 ghost exchange (pack -> send/recv -> unpack, or direct rows) and the split sweep, whose
// interior tiles overlap the previous exchange while the frame tiles wait for it.
// Reference: the halo exchange of stage4-mpi+cuda/poisson_mpi_cuda_f.cu:331-500, called at :851.
#include <algorithm>
#include <cstring>
#include <functional>
#include <vector>

#include "pmx/common.hpp"
#include "pmx/gpu_solver.hpp"
#include "pmx/trace.hpp"

namespace pmx {

void PcgDriver::set_halo_target(long long k) {
  for (auto* s : local_) s->set_halo_target(k);
}

void PcgDriver::halo_exchange_pcg1(std::vector<hipStream_t>& streams, long long target) {
  set_halo_target(target);
  comm_->before_pack(local_, streams);
  for (size_t i = 0; i < local_.size(); ++i) {
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    local_[i]->enqueue_halo_pack(streams[i]);
  }
  poison(streams);
  comm_->halo(local_, streams);
  for (size_t i = 0; i < local_.size(); ++i) {
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    local_[i]->enqueue_halo_unpack(streams[i]);
  }
}

// Split sweep k (pcg1, decomposed, overlap on).  Default schedule: see frame_on_comm_ below.
// With PMX_FRAME_ON_COMM=0, streams C (compute), F (frame), H (comm):
//   C: [all-reduce k-1] -> ev_ar -> interior tiles of sweep k ----------> wait F -> ev_swept ->
//   F:                     wait ev_ar (+ ev_halo of k-1) -> frame tiles -'
//   C: reduce -> all-reduce k (no join: see the end of enqueue_split_iteration)
//   H: wait ev_swept -> pack -> send/recv -> unpack -> ev_halo (joined by the next F, or
//      by C at the end of the batch: join_halo)
// So the ghost exchange of sweep k runs under the reduction, the all-reduce AND the interior of
// sweep k+1; only the frame tiles (a few % of the sweep) wait for it.
void PcgDriver::enqueue_split_iteration() {
  // frame_on_comm_ (default): F is the comm stream H itself.  The exchange of sweep k reads only edge lines
  // the frame tiles own (rows / columns 1, 2 and n-1, n: every tile whose march reaches a ghost cell
  // is a frame tile, pcg1_tiles) and writes only ghost cells, which no interior tile reads; so H
  // runs frame k -> exchange k -> (wait all-reduce k) frame k+1 in its own order, and the compute
  // stream joins it once per iteration, before the reduction:
  //   C: ev_ar -> interior k -> wait ev_fdone -> reduce -> all-reduce k -> ev_ar ...
  //   H: wait ev_ar -> frame k -> ev_fdone -> pack -> send/recv -> unpack -> ev_halo
  const bool fc = frame_on_comm_;
  auto fstream = [&](size_t i) { return fc ? comm_streams_[i] : frame_streams_[i]; };
  for_each_stream([&](size_t i, size_t u) {
    HIP_CHECK(hipEventRecord(ev_ar_[u], streams_[i]));
    HIP_CHECK(hipStreamWaitEvent(fstream(i), ev_ar_[u], 0));
    if (halo_pending_ && !fc) HIP_CHECK(hipStreamWaitEvent(frame_streams_[i], ev_halo_[u], 0));
  });
  for (size_t i = 0; i < local_.size(); ++i) {
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    local_[i]->enqueue_kernel_a_part(streams_[i], 1);
    local_[i]->enqueue_kernel_a_part(fstream(i), 2);
  }
  for_each_stream([&](size_t i, size_t u) {
    HIP_CHECK(hipEventRecord(ev_fdone_[u], fstream(i)));
    HIP_CHECK(hipStreamWaitEvent(streams_[i], ev_fdone_[u], 0));
    if (!fc) {
      HIP_CHECK(hipEventRecord(ev_swept_[u], streams_[i]));
      HIP_CHECK(hipStreamWaitEvent(comm_streams_[i], ev_swept_[u], 0));
    }
  });
  set_halo_target(local_[0]->host_k() + 1);  // the sweep just enqueued is host_k; the next reads its outputs
  comm_->before_pack(local_, comm_streams_);
  for (size_t i = 0; i < local_.size(); ++i) {
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    local_[i]->enqueue_halo_pack(comm_streams_[i]);
  }
  poison(comm_streams_);
  comm_->halo(local_, comm_streams_);
  for (size_t i = 0; i < local_.size(); ++i) {
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    local_[i]->enqueue_halo_unpack(comm_streams_[i]);
  }
  for_each_stream([&](size_t i, size_t u) { HIP_CHECK(hipEventRecord(ev_halo_[u], comm_streams_[i])); });
  halo_pending_ = true;
  for (size_t i = 0; i < local_.size(); ++i) {
    HIP_CHECK(hipSetDevice(local_[i]->device()));
    local_[i]->enqueue_reduce_a(streams_[i]);
  }
  comm_->allreduce(local_, 2, streams_);
  // No join of the comm stream here: the exchange (packed or direct rows) reads the edge lines of
  // r_{k+1}, p_{k+1} and writes their ghost cells, with the buffer parity in its launch arguments;
  // sweep k+1 writes the other parity (r_{k+2}, p_{k+2}), its interior tiles read no ghost cell and
  // its frame tiles wait for ev_halo (or follow the exchange on H).  Sweep k+2, the next writer of these buffers, follows the
  // all-reduce of k+1, which follows that frame.  So the next interior starts right after the
  // all-reduce: one cross-queue wait per iteration instead of two (loopback strip 3 of 8: 293 ->
  // 266 us, profiles/r4/loopback/).
}

void PcgDriver::join_halo() {
  if (!halo_pending_) return;
  for_each_stream([&](size_t i, size_t u) { HIP_CHECK(hipStreamWaitEvent(streams_[i], ev_halo_[u], 0)); });
  halo_pending_ = false;
}

}  // namespace pmx
