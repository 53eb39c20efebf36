// The s-step PCG's solver steps and driver schedule (GpuOptions::algo 3; kernels in ca_kernels.hip):
// the passes (pass 1, pass 2, the fused pass) with their frame tiles on a side stream, the block
// reductions and scalars, the ghost-row messages of row strips, the kernel test hook, and
// PcgDriver::enqueue_ca -- blocks of s iterations per batch, with or without the fused pass, on one
// grid or on strips (all-reduce of the 21 sums, overlapped ghost-row exchange).
// Reference loop being regrouped: stage4-mpi+cuda/poisson_mpi_cuda_f.cu:843-943.
#include <algorithm>
#include <cstring>
#include <functional>
#include <vector>

#include "pmx/common.hpp"
#include "pmx/gpu_solver.hpp"
#include "pmx/trace.hpp"

namespace pmx {

// One s-step pass (kind 0: pass 1, 1: pass 2, 2: the fused pass): with the split kernels the frame tiles
// run on a side stream, concurrently with the interior (their few long marches would otherwise trail
// the pass by ~0.1 ms).  The first pass after a ghost exchange (pass 1 or the fused pass; with the fused
// schedule also the batch's last pass 2) waits for it in the tiles that read ghost rows.
template <typename T>
void GpuSubdomainSolver::ca_pass_impl(hipStream_t s, int kind) {
  T* w = static_cast<T*>(field_base(0));
  T* z0 = static_cast<T*>(field_base(1));
  T* z1 = reinterpret_cast<T*>(r2_ + field_off_ * elem_);
  T* p0 = static_cast<T*>(field_base(2));
  T* p1 = static_cast<T*>(field_base(3));
  hipEvent_t wait = ca_frame_wait_;
  ca_frame_wait_ = nullptr;
  auto launch = [&](hipStream_t side) {
    if (kind == 2)
      launch_ca_fused<T>(ca_geom_, w, z0, z1, p0, p1, partials_, ca_state_, ca_tiles_, s, side, wait);
    else
      launch_ca_sweep<T>(ca_geom_, ca_tables_, w, z0, z1, p0, p1, partials_, state_, ca_state_, ca_tiles_, kind == 1,
                         s, side, wait);
  };
  if (ca_side_) {
    HIP_CHECK(hipEventRecord(ca_ev_fork_, s));
    HIP_CHECK(hipStreamWaitEvent(ca_side_, ca_ev_fork_, 0));
    launch(ca_side_);
    HIP_CHECK(hipEventRecord(ca_ev_join_, ca_side_));
    HIP_CHECK(hipStreamWaitEvent(s, ca_ev_join_, 0));
  } else {
    launch(nullptr);
  }
  after_launch(s);
}

void GpuSubdomainSolver::drop_side_stream() {
  if (!ca_side_) return;
  HIP_CHECK(hipSetDevice(opt_.device));
  HIP_CHECK(hipStreamSynchronize(ca_side_));
  HIP_CHECK(hipStreamDestroy(ca_side_));
  HIP_CHECK(hipEventDestroy(ca_ev_fork_));
  HIP_CHECK(hipEventDestroy(ca_ev_join_));
  ca_side_ = nullptr;
  ca_ev_fork_ = ca_ev_join_ = nullptr;
}

void GpuSubdomainSolver::enqueue_ca_pass(hipStream_t s, bool upd) {
  PMX_CHECK(ca_, "not an s-step solver");
  if (elem_ == 8) ca_pass_impl<double>(s, upd ? 1 : 0);
  else ca_pass_impl<float>(s, upd ? 1 : 0);
}

void GpuSubdomainSolver::enqueue_ca_fused(hipStream_t s) {
  PMX_CHECK(ca_fused(), "not an s-step solver with the fused pass");
  if (elem_ == 8) ca_pass_impl<double>(s, 2);
  else ca_pass_impl<float>(s, 2);
}

void GpuSubdomainSolver::enqueue_ca_reduce(hipStream_t s, int n, bool check_only, bool finish, bool fused) {
  PMX_CHECK(ca_, "not an s-step solver");
  PMX_CHECK(!fused || ca_fused(), "fused reduction without the fused pass");
  const double wdiff = spec_.norm == Norm::kWeighted ? g_.h1h2 : 1.0;
  // after the fused pass both the Gram products and the norms come from its tiling
  const int n1 = fused ? ca_tiles_.ntilesf() : ca_tiles_.ntiles();
  const int n2 = fused ? ca_tiles_.ntilesf() : ca_tiles_.ntiles2();
  launch_ca_reduce(partials_, n1, n2, ca_tiles_.s, g_.h1h2, wdiff,
                   check_only ? 1 : n, check_only, state_, ca_state_, ca_chunk_, s, progress_dev_, finish);
  after_launch(s);
  if (!check_only) {  // a block the device applies (unless it stopped): the set its pass 2 writes
    ++ca_blk_;
    host_k_ += n;
  }
}

void GpuSubdomainSolver::enqueue_ca_finish(hipStream_t s, int n, bool check_only) {
  PMX_CHECK(ca_, "not an s-step solver");
  const double wdiff = spec_.norm == Norm::kWeighted ? g_.h1h2 : 1.0;
  launch_ca_finish(ca_tiles_.s, g_.h1h2, wdiff, check_only ? 1 : n, check_only, state_, ca_state_, s, progress_dev_);
  after_launch(s);
}

GpuSubdomainSolver::CaProbe GpuSubdomainSolver::ca_probe(const std::vector<double>& z, const std::vector<double>& p,
                                                         const std::vector<double>& w, const std::vector<double>& coef,
                                                         const std::vector<double>& pa, bool fused, hipStream_t s) {
  PMX_CHECK(ca_ && elem_ == 8, "ca_probe: not an fp64 s-step solver");
  PMX_CHECK(!fused || ca_fused(), "ca_probe: the fused pass runs undecomposed grids");
  const int S = ca_tiles_.s, NB = 2 * S + 1, NQ = 6 * S;
  const size_t rows = size_t(sd_.nx + 2 * gh_), cols = size_t(sd_.ny + 2);
  PMX_CHECK(z.size() == rows * cols && p.size() == rows * cols && w.size() == rows * cols,
            "ca_probe: fields must be (nx + 2 gh) x (ny + 2)");
  PMX_CHECK(coef.size() == size_t(3 * NB) && pa.size() == size_t(S * NB), "ca_probe: coefficient shapes");
  HIP_CHECK(hipSetDevice(opt_.device));
  enqueue_init(s);
  HIP_CHECK(hipStreamSynchronize(s));
  auto put = [&](void* base, const std::vector<double>& v) {
    char* dst = static_cast<char*>(base) + int64_t(1 - gh_) * geom_.pitch * 8;
    HIP_CHECK(hipMemcpy2D(dst, size_t(geom_.pitch) * 8, v.data(), cols * 8, cols * 8, rows, hipMemcpyHostToDevice));
  };
  put(field_base(1), z);
  put(field_base(2), p);
  put(field_base(0), w);
  CaProbe out;
  auto sums = [&](int64_t base, int nq, int n) {
    const std::vector<double> h = read_partials(s);
    std::vector<double> r(size_t(nq), 0.0);
    for (int q = 0; q < nq; ++q)
      for (int i = 0; i < n; ++i) r[size_t(q)] += h[size_t(base + int64_t(q) * n + i)];
    return r;
  };
  CaState c{};
  HIP_CHECK(hipMemcpy(&c, ca_state_, sizeof(CaState), hipMemcpyDeviceToHost));
  c.blk = 1;  // as after the block's reduction: pass 2 / the fused pass read set 0, write set 1
  c.nupd = S;
  for (int k = 0; k < 3; ++k)
    for (int i = 0; i < NB; ++i) c.coef[k][i] = coef[size_t(k * NB + i)];
  for (int j = 0; j < S; ++j)
    for (int i = 0; i < NB; ++i) c.pa[j][i] = pa[size_t(j * NB + i)];
  if (!fused) {
    enqueue_ca_pass(s, false);
    HIP_CHECK(hipStreamSynchronize(s));
    out.gram = sums(0, NQ, ca_tiles_.ntiles());
    HIP_CHECK(hipMemcpy(ca_state_, &c, sizeof(CaState), hipMemcpyHostToDevice));
    enqueue_ca_pass(s, true);
    HIP_CHECK(hipStreamSynchronize(s));
    out.norms = sums(int64_t(NQ) * ca_tiles_.ntiles(), S, ca_tiles_.ntiles2());
  } else {
    HIP_CHECK(hipMemcpy(ca_state_, &c, sizeof(CaState), hipMemcpyHostToDevice));
    enqueue_ca_fused(s);
    HIP_CHECK(hipStreamSynchronize(s));
    const std::vector<double> gn = sums(0, NQ + S, ca_tiles_.ntilesf());
    out.gram.assign(gn.begin(), gn.begin() + NQ);
    out.norms.assign(gn.begin() + NQ, gn.end());
  }
  auto get = [&](const void* base) {
    std::vector<double> h(size_t(sd_.nx) * sd_.ny);
    const char* src = static_cast<const char*>(base) + (geom_.pitch + 1) * 8;
    HIP_CHECK(hipMemcpy2D(h.data(), size_t(sd_.ny) * 8, src, size_t(geom_.pitch) * 8, size_t(sd_.ny) * 8,
                          size_t(sd_.nx), hipMemcpyDeviceToHost));
    return h;
  };
  out.p = get(field_base(3));
  out.z = get(r2_ + field_off_ * elem_);
  out.w = get(field_base(0));
  return out;
}

HaloMsgs GpuSubdomainSolver::ca_halo_msgs(int set) const {
  PMX_CHECK(ca_, "ca_halo_msgs: not an s-step solver");
  HaloMsgs out;
  // s-step strips: the gh owned edge rows of z and p of the set the next block reads (CaState::blk
  // & 1, mirrored by ca_blk_) into the neighbour's gh ghost rows (gh = s, 2s with the fused pass), as
  // ONE span per field: rows q .. q+gh-2 whole, row q+gh-1's columns 0 .. ny+1 (columns <= 0 and >= ny+1
  // are Dirichlet on a strip)
  const int s = gh_;
  char* fz = set ? r2_ + field_off_ * elem_ : static_cast<char*>(field_base(1));
  char* fp = static_cast<char*>(field_base(set ? 3 : 2));
  const int64_t P = geom_.pitch;
  const int count = int((s - 1) * P + sd_.ny + 2);
  for (int slot = 0; slot < 2; ++slot) {
    if (layout_.peer[slot] < 0) continue;
    const int64_t srow = slot == 0 ? 1 : sd_.nx - s + 1, rrow = slot == 0 ? 1 - s : sd_.nx + 1;
    for (int f = 0; f < 2; ++f) {
      char* base = f == 0 ? fz : fp;
      out.m[out.n++] = HaloMsg{slot, f, layout_.peer[slot], count, base + srow * P * int64_t(elem_),
                               base + rrow * P * int64_t(elem_)};
    }
  }
  return out;
}

// One s-step ghost exchange on `streams`: direct rows (strips), or packed (2-D blocks): pack -> send /
// recv of the slots -> unpack
void PcgDriver::ca_exchange(std::vector<hipStream_t>& streams) {
  if (direct_) {
    comm_->halo(local_, streams);
    return;
  }
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
  HIP_CHECK(hipSetDevice(local_[0]->device()));
}

int PcgDriver::ca_batch() const {
  const int s = local_[0]->ca_s();
  const int b = graph_batch_ > 0 ? graph_batch_ : 16;
  return (b + s - 1) / s * s;  // whole blocks per captured batch
}

void PcgDriver::enqueue_ca(int64_t n, const std::function<void(int)>& mark) {
  const int s = local_[0]->ca_s();
  HIP_CHECK(hipSetDevice(local_[0]->device()));
  if (n <= 0) return;
  auto mk = [&](int b) {
    if (mark) mark(b);
  };
  auto each = [&](auto&& f) {
    for (size_t i = 0; i < local_.size(); ++i) {
      HIP_CHECK(hipSetDevice(local_[i]->device()));
      f(local_[i], streams_[i]);
    }
    HIP_CHECK(hipSetDevice(local_[0]->device()));
  };
  // The fused schedule is carried across batches: a batch ends with a fused pass, which applies its
  // last block AND sums the next block's Gram products, so the next batch starts at the reduction
  // (primed) and only a solve's first batch runs pass 1.  Every block then costs one fused pass and one
  // reduction wherever the batch boundaries fall (pass 1 + pass 2 at each boundary cost ~0.84 ms more
  // than one fused pass at 16384^2).  The stop test of the batch's last block still runs at its end (a
  // check-only reduction of the fused pass's norms, and the rewind), so w and the PcgState are exact
  // at every batch end; the extra Gram sums of a solve's last fused pass are the one wasted half-pass.
  const bool fused = local_[0]->ca_fused();
  const bool primed = fused && local_[0]->ca_primed();
  auto set_primed = [&](bool v) {
    for (auto* g : local_) g->set_ca_primed(v);
  };
  if (!any_nb_ && local_.size() == 1 && comm_->world_size() == 1) {
    // One grid: pass 1 -> reduce -> pass 2 per block, or with the fused pass
    //   [pass 1 unless primed] -> reduce -> (fused -> reduce) x (blocks - 1) -> fused
    // and then the last block's stop test (and its rewind): the state is exact at every batch end
    GpuSubdomainSolver* g = local_[0];
    hipStream_t st = streams_[0];
    bool first = true;
    while (n > 0) {
      const int m = int(std::min<int64_t>(s, n));
      if (fused && !first) g->enqueue_ca_fused(st);
      else if (!primed) g->enqueue_ca_pass(st, false);
      if (!(first && primed)) mk(kPhA);
      g->enqueue_ca_reduce(st, m, false, true, fused && !(first && !primed));
      mk(kPhRed);
      if (!fused) {
        g->enqueue_ca_pass(st, true);
        mk(kPhB);
      }
      first = false;
      n -= m;
    }
    if (fused) {
      g->enqueue_ca_fused(st);
      mk(kPhA);
    }
    g->enqueue_ca_reduce(st, 1, true, true, fused);
    mk(kPhRed);
    g->enqueue_ca_pass(st, true);  // rewind (a no-op unless the test stopped inside the last block)
    mk(kPhB);
    set_primed(fused);
    return;
  }
  // decomposed: every rank's sums are all-reduced between the reduction and the scalars, and the s
  // ghost rows of the new (z, p) set are exchanged after pass 2 (strips: direct rows, one span per field;
  // 2-D blocks: ghost rows, columns and corners through the packed slots, ca_exchange).
  // With the overlapped schedule the exchange runs on the comm stream: the next pass 1's interior
  // tiles (which read no ghost row) start at once, its frame tiles wait for the exchange.  The batch
  // joins the comm stream at its end, so a captured graph has no edge into the next one.
  const bool ovl = any_nb_ && overlap_ && !comm_streams_.empty() && !mark;
  bool pending = false;
  auto frame_waits = [&](bool on) {  // every solver, by the index of its (possibly shared) stream
    size_t u = 0;
    for (size_t i = 0; i < local_.size(); ++i) {
      if (i > 0 && streams_[i] != streams_[i - 1]) ++u;
      local_[i]->set_ca_frame_wait(on ? ev_halo_[u] : nullptr);
    }
  };
  const bool ar = comm_->world_size() > 1;
  // the s ghost rows of the (z, p) set just written (2s with the fused pass)
  auto exchange = [&] {
    if (any_nb_ && ovl) {
      for_each_stream([&](size_t i, size_t u) {
        HIP_CHECK(hipEventRecord(ev_packed_[u], streams_[i]));
        HIP_CHECK(hipStreamWaitEvent(comm_streams_[i], ev_packed_[u], 0));
      });
      ca_exchange(comm_streams_);
      for_each_stream([&](size_t i, size_t u) { HIP_CHECK(hipEventRecord(ev_halo_[u], comm_streams_[i])); });
      frame_waits(true);
      pending = true;
    } else if (any_nb_) {
      ca_exchange(streams_);
      mk(kPhHalo);
    }
  };
  // Unfused, per block: pass 1 -> reduce -> all-reduce -> scalars -> pass 2 -> exchange.  Fused: pass 1
  // (unless primed) -> reduce -> all-reduce -> scalars, then per further block fused pass -> exchange
  // (under the reduction, all-reduce and scalars) -> ..., and a last fused pass -> exchange.  Every rank
  // runs the same schedule (ca_fused() is decided from global data, primed by the same batches).
  bool first = true;
  while (n > 0) {
    const int m = int(std::min<int64_t>(s, n));
    const bool f = fused && !first;
    if (f) each([&](GpuSubdomainSolver* g, hipStream_t st) { g->enqueue_ca_fused(st); });
    else if (!primed) each([&](GpuSubdomainSolver* g, hipStream_t st) { g->enqueue_ca_pass(st, false); });
    if (!(first && primed)) mk(kPhA);
    if (f) exchange();
    each([&](GpuSubdomainSolver* g, hipStream_t st) { g->enqueue_ca_reduce(st, m, false, false, f || primed); });
    mk(kPhRed);
    comm_->allreduce(local_, 3, streams_);
    if (ar) mk(kPhAr);
    each([&](GpuSubdomainSolver* g, hipStream_t st) { g->enqueue_ca_finish(st, m, false); });
    mk(kPhRed);
    if (!fused) {
      each([&](GpuSubdomainSolver* g, hipStream_t st) { g->enqueue_ca_pass(st, true); });
      mk(kPhB);
      exchange();
    }
    first = false;
    n -= m;
  }
  if (fused) {
    each([&](GpuSubdomainSolver* g, hipStream_t st) { g->enqueue_ca_fused(st); });
    mk(kPhA);
    exchange();
  }
  each([&](GpuSubdomainSolver* g, hipStream_t st) { g->enqueue_ca_reduce(st, 1, true, false, fused); });
  mk(kPhRed);
  comm_->allreduce(local_, 3, streams_);
  if (ar) mk(kPhAr);
  each([&](GpuSubdomainSolver* g, hipStream_t st) { g->enqueue_ca_finish(st, 1, true); });
  mk(kPhRed);
  each([&](GpuSubdomainSolver* g, hipStream_t st) { g->enqueue_ca_pass(st, true); });  // rewind
  mk(kPhB);
  if (pending) {  // the last block's exchange ran next to the check
    for_each_stream([&](size_t i, size_t u) { HIP_CHECK(hipStreamWaitEvent(streams_[i], ev_halo_[u], 0)); });
    frame_waits(false);
  }
  set_primed(fused);
}

// the key of a captured s-step batch: the (z, p) set parity on decomposed grids (the exchange's spans),
// and whether the batch starts primed (no pass 1)
int PcgDriver::ca_phase() const {
  return (any_nb_ ? int(local_[0]->ca_blocks() & 1) : 0) + (local_[0]->ca_primed() ? 2 : 0);
}

}  // namespace pmx
