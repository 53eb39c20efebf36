// Persistent single-pass PCG for latency-bound grids ("pcg1p"): ONE launch runs many iterations.
//
// Where the reference actually published (800x1200 .. 2400x3200, stage4-mpi+cuda/poisson_mpi_cuda_f.cu:
// 847-943; итоговый отчёт/Этап_4_1213.pdf p.11) the five fields are 38-230 MB: they sit in the 256 MB
// Infinity Cache and the bandwidth floor of a sweep is a few microseconds.  The launch-per-sweep path
// (k_pcg1 + k_reduce_n, replayed from hipGraphs) pays per iteration two kernel boundaries, the ramp
// and drain of ~2000-8000 short-lived waves and a separate reduction launch: 53.6 us/iteration at
// 800x1200 (README).  Here a fixed set of workgroups (one 512-thread workgroup per CU: 8 waves, 2 per
// SIMD) stays resident for a whole batch of iterations:
//
//   sweep k:  every wave marches its tiles of the pcg1 tiling (pcg1_march: the same arithmetic as
//             k_pcg1, so every point gets bit-identical values for equal scalars);
//   publish:  the wave sums -> one 5-value partial per workgroup (sc1 stores); the fields are stored
//             write-through (sc1 buffer stores) and every wave drains them (vmcnt 0) before its
//             workgroup arrives, so no L2 writeback fence is needed (k_pcg1's non-temporal stores +
//             one agent-scope release per workgroup measured 57.1 vs 59.6 us at 800x1200, and
//             prefetch depth 2 45.4 vs 46.6 with an unchanged march: both removed, profiles/r4/persist/);
//   barrier:  one monotonic arrival counter (relaxed agent-scope add, relaxed polls with s_sleep,
//             bounded by a wall-clock timeout that stops the solve instead of hanging the GPU);
//   acquire:  one agent-scope acquire per workgroup, then every workgroup sums the NWG partials in
//             the same fixed order (wave 0, sc1 loads, MFMA wave sum) -> identical scalars everywhere;
//   scalars:  alpha, beta, the w schedule and the stop test of sweep k+1 from those sums, exactly as
//             k_pcg1's prologue and k_reduce_n's finish; workgroup 0 mirrors them into PcgState so the
//             host-side state (download_w, error norms, checkpoints) is that of the graph path.
//
// Inter-workgroup hand-offs follow MI355X_MICROARCH.md 'Workgroup dispatch, XCD placement &
// inter-workgroup visibility' (producer: drain + agent release before the counter add; consumer:
// relaxed poll, ONE agent acquire, then plain loads; every polled word zeroed by a memset before each
// launch).  Residency: one workgroup per CU is always admitted, so the grid barrier cannot strand a
// workgroup; the timeout covers the impossible case too.  Reduction order differs from k_reduce_n's
// (per workgroup, then over workgroups), so sums may differ in the last bit from the graph path:
// iteration counts are checked against the reference goldens (tests/test_gpu_pcg1.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <functional>
#include <queue>
#include <utility>
#include <vector>

#include "pcg1_march.hpp"
#include "pcg_device.hpp"
#include "pmx/common.hpp"
#include "pmx/kernels.hpp"
#include "pmx/spec.hpp"

namespace pmx {

namespace {

constexpr int kPersistWaves = kPersistThreads / 64;

struct PersistArgs {
  int TI, tiles_j, ntiles;
  const Pcg1Slot* order;  // the static schedule: wave w marches order[offs[w] .. offs[w+1])
  const int* offs;
  long long k_end;        // the last sweep index this launch may run
  double wt[kNq];         // weights of the 5 sums (h1 h2, and the stop-test norm weight)
  long long timeout;      // barrier wait limit in wall_clock64 ticks (100 MHz)
  // diagnostics (PMX_PERSIST_TRACE=k): wall-clock stamps of sweep `trace_k` -- per wave its march
  // start / end, per workgroup its barrier arrival / exit (100 MHz ticks); nullptr = off
  unsigned long long* trace;
  long long trace_k;
};

unsigned long long* g_trace = nullptr;  // host copy of the trace buffer (one per process)
int g_trace_n = 0;

__device__ __forceinline__ unsigned long long ld_relaxed(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Field stores write-through (sc1, pcg1_march's WT): the publish needs no L2 writeback fence.
template <typename T, typename C>
__global__ void __launch_bounds__(kPersistThreads, kPersistWaves / 4)
k_pcg1_persist(DevGeom G, DevTables Tb, T* __restrict__ w, T* r, T* r2, T* p0, T* p1, PcgState* S,
               PersistWs* ws, PersistArgs A) {
  constexpr int VEC = 2;
  constexpr int WO = 64 * VEC - 4;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int nwg = int(gridDim.x);
  const int gwave = int(blockIdx.x) * kPersistWaves + wave;
  const int nwaves = nwg * kPersistWaves;
  __shared__ double s_col[kPersistWaves * 4 * VEC * 64];
  __shared__ double s_ring[kPersistWaves * 3 * VEC * 4 * 64];  // cut-row coefficient carry (pcg1_march CC)
  __shared__ double s_sum[kPersistWaves][kNq];
  __shared__ int s_stop;
  double* scol = s_col + wave * (4 * VEC * 64);
  double* kring = s_ring + wave * (3 * VEC * 4 * 64);
  const ArithF AF{float(G.cx), float(G.cy), float(G.dinv_in), float(G.dinv_out), float(G.inv_eps)};

  // state at entry (written by earlier kernels: visible at this kernel's start).  The PCG scalars
  // live in LDS between sweeps: held in SGPRs across the marches they spill by the hundred.
  __shared__ double rc[kNq], al[4], be[4], zr[2];
  if (S->done) return;
  long long k = S->it;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int q = 0; q < kNq; ++q) rc[q] = S->red_c[q];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      al[q] = S->alpha1[q];
      be[q] = S->beta1[q];
    }
    zr[0] = S->zr[0];
    zr[1] = S->zr[1];
  }
  __syncthreads();
  const double s_delta = S->delta, s_bd_tol = S->bd_tol, s_pmb = S->pair_min_beta;
  const long long s_max_iter = S->max_iter;
  const int s_norm = S->norm, cyc = S->w_cycle;
  const bool leader = blockIdx.x == 0 && threadIdx.x == 0;  // mirrors the scalars into PcgState
  unsigned long long gen = 0;

  for (; k <= A.k_end; ++k) {
    // ---- scalars of sweep k (k_pcg1's prologue; every workgroup computes the same values)
    double alpha = 0.0, beta = 0.0, c1 = 0.0, c2 = 0.0;
    int wm = 0;
    if (k > 0) {
      const double rho = rc[0];
      double diff = 0.0;
      if (k >= 2) {
        diff = fabs(al[(k - 1) & 3]) * sqrt(rc[4]);
        const bool bad = !(diff == diff) || !(rho == rho);
        if (bad || diff < s_delta || k > s_max_iter) {
          if (leader) {
            S->diff = diff;
            S->iters = k - 1;
            S->status = bad ? int(Status::kBreakdown) : (diff < s_delta ? int(Status::kConverged) : int(Status::kMaxIter));
            if (bad) S->nan_flag = 1;
            S->done = 1;
          }
          return;
        }
        beta = rho / zr[k & 1];
      }
      const double denom = rc[1] + beta * (2.0 * rc[2] + beta * rc[3]);
      const bool bd = s_norm == int(Norm::kWeighted) ? fabs(denom) < s_bd_tol : denom < s_bd_tol;
      if (bd || !(denom == denom)) {
        if (leader) {
          if (k >= 2) S->diff = diff;
          S->iters = k;
          S->status = int(Status::kBreakdown);
          if (!(denom == denom)) S->nan_flag = 1;
          S->done = 1;
        }
        return;
      }
      alpha = rho / denom;
      const int ph = int(k % cyc);
      if (ph == 0) {
        c1 = al[(k - 1) & 3];
        wm = 1;
        if (cyc == 3) {
          const double bprev = be[(k - 1) & 3];
          const double a2 = al[(k - 2) & 3];
          if (fabs(bprev) >= s_pmb) { wm = 2; c2 = a2 / bprev; }
          else { wm = 3; c2 = a2; }
        }
      }
      __syncthreads();  // every wave has read the rings before thread 0 rewrites them
      if (threadIdx.x == 0) {
        zr[(k - 1) & 1] = rho;
        al[k & 3] = alpha;
        be[k & 3] = beta;
      }
      if (leader) {
        S->zr[(k - 1) & 1] = rho;
        S->alpha1[k & 3] = alpha;
        S->beta1[k & 3] = beta;
        if (k >= 2) S->diff = diff;
        S->w_pend = ph ? k : 0;
        S->w_pend_n = ph;
      }
    }
    if (leader) S->halo_k = k + 1;
    const bool tr = A.trace && k == A.trace_k;
    if (tr && lane == 0) A.trace[2 * gwave] = wall_clock64();

    // ---- sweep k: this wave's tiles
    T* pnew = (k & 1) ? p1 : p0;
    const T* pold = (k & 1) ? p0 : p1;
    const T* rold = (k & 1) ? r2 : r;
    T* rnew = (k & 1) ? r : r2;
    double acc[kNq] = {0.0, 0.0, 0.0, 0.0, 0.0};
    const int q0 = A.offs[gwave], q1 = A.offs[gwave + 1];
    for (int pos = q0; pos < q1; ++pos) {
      const int id = A.order[pos].id;
      const unsigned long long ocls = A.order[pos].cls;
      const int ti = id / A.tiles_j, tj = id - ti * A.tiles_j;
      const int i0 = 1 + ti * A.TI, i1 = min(i0 + A.TI - 1, G.nx);
      const int j0 = 1 + tj * WO, j1 = min(j0 + WO - 1, G.ny);
      const bool fast = j1 == j0 + WO - 1 && G.gi0 + i0 - 2 >= 1 && G.gi0 + i1 + 2 <= G.M - 1 &&
                        G.gj0 + j0 - 2 >= 1 && G.gj0 + j0 + 64 * VEC - 3 <= G.N - 1;
      const bool use_cls = A.TI + 5 <= 64 / 2;
      double t[kNq] = {0.0, 0.0, 0.0, 0.0, 0.0};
#define PMX_PMARCH(E, F)                                                                                        \
  pcg1_march<T, C, VEC, 1, E, F, true, true>(G, Tb, AF, w, rold, rnew, pold, pnew, i0, i1, j0, j1, alpha, beta, c1, \
                                            c2, t, scol, ocls, use_cls, kring)
#define PMX_PMARCH_W(F)                  \
  switch (wm) {                          \
    case 0: PMX_PMARCH(0, F); break;     \
    case 1: PMX_PMARCH(1, F); break;     \
    case 2: PMX_PMARCH(2, F); break;     \
    default: PMX_PMARCH(3, F); break;    \
  }
      if (fast) {
        PMX_PMARCH_W(true)
      } else {
        PMX_PMARCH_W(false)
      }
#undef PMX_PMARCH_W
#undef PMX_PMARCH
#pragma unroll
      for (int q = 0; q < kNq; ++q) acc[q] += t[q];
    }

    if (tr && lane == 0) A.trace[2 * gwave + 1] = wall_clock64();
    // ---- publish: wave sums -> workgroup partial (fixed order), field stores drained and released
    wave_sum2_mfma(acc[0], acc[1]);
    wave_sum2_mfma(acc[2], acc[3]);
    acc[4] = wave_sum_mfma(acc[4]);
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < kNq; ++q) s_sum[wave][q] = acc[q];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its field stores
    __syncthreads();
    ++gen;
    double* slot = ws->part[gen & 1] + kNq * blockIdx.x;
    if (threadIdx.x == 0) {
#pragma unroll
      for (int q = 0; q < kNq; ++q) {
        double v = 0.0;  // fixed order over the waves
#pragma unroll
        for (int wv = 0; wv < kPersistWaves; ++wv) v += s_sum[wv][q];
        st_publish(slot + q, v);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial's sc1 stores
      __hip_atomic_fetch_add(&ws->arrive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tr) A.trace[2 * nwaves + 2 * blockIdx.x] = wall_clock64();
      // ---- grid barrier: every workgroup of sweep `gen` has arrived
      const unsigned long long target = gen * (unsigned long long)nwg;
      const long long t0 = wall_clock64();
      int stop = 0;
      while (ld_relaxed(&ws->arrive) < target) {
        if (wall_clock64() - t0 > A.timeout || ld_relaxed(&ws->err) != 0) {
          __hip_atomic_store(&ws->err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          stop = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // ONE acquire: this CU's L1 drops stale lines
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      s_stop = stop;
      if (tr) A.trace[2 * nwaves + 2 * blockIdx.x + 1] = wall_clock64();
    }
    __syncthreads();
    if (s_stop) {  // a workgroup never arrived: stop the solve (the host sees status breakdown + NaN)
      if (leader) {
        S->iters = k;
        S->status = int(Status::kBreakdown);
        S->nan_flag = 1;
        S->done = 1;
      }
      return;
    }

    // ---- every workgroup reduces the NWG partials in the same order -> identical sums
    if (wave == 0) {
      const double* part = ws->part[gen & 1];
      double s[kNq];
#pragma unroll
      for (int q = 0; q < kNq; ++q) s[q] = 0.0;
      for (int b = lane; b < nwg; b += 64) {
#pragma unroll
        for (int q = 0; q < kNq; ++q) s[q] += ld_published(part + kNq * b + q);
      }
      bool bad = false;
#pragma unroll
      for (int q = 0; q < kNq; ++q) {
        s[q] = wave_sum_mfma(s[q]);
        bad |= !(s[q] == s[q]) || isinf(s[q]);
      }
      if (lane == 0) {
#pragma unroll
        for (int q = 0; q < kNq; ++q) rc[q] = s[q] * A.wt[q];
        if (leader && bad) S->nan_flag = 1;
      }
    }
    __syncthreads();
    if (leader) {
#pragma unroll
      for (int q = 0; q < kNq; ++q) S->red_c[q] = rc[q];
      S->it = k + 1;
    }
  }
}

}  // namespace

template <typename T>
int launch_pcg1_persist(const DevGeom& G, const DevTables& Tb, T* w, T* r, T* r2, T* p0, T* p1, PcgState* S,
                        PersistWs* ws, const TileCfg& tc, const Pcg1Slot* sched, const int* offs, int nwg,
                        long long k_end, const double* weights, hipStream_t s) {
  PMX_CHECK(tc.kind == 3 && tc.vec == 2 && tc.waves == 1 && tc.order0, "pcg1p needs VEC 2 wave tiles with an order");
  PMX_CHECK(nwg >= 1 && nwg <= kPersistMaxWg, "pcg1p: 1.." << kPersistMaxWg << " workgroups");
  PMX_CHECK(G.nb == 0, "pcg1p runs undecomposed grids only");
  PersistArgs A{};
  A.TI = tc.rows;
  A.tiles_j = tc.tiles_j;
  A.ntiles = tc.ntiles();
  A.order = sched;
  A.offs = offs;
  A.k_end = k_end;
  for (int q = 0; q < kNq; ++q) A.wt[q] = weights[q];
  A.timeout = 200000000LL;  // 2 s of wall clock per barrier wait
  static const long long trace_k = [] {
    const char* e = std::getenv("PMX_PERSIST_TRACE");
    return e && e[0] ? std::atoll(e) : -1LL;
  }();
  if (trace_k >= 0) {
    const int n = 2 * nwg * (kPersistThreads / 64) + 2 * nwg;
    if (!g_trace || g_trace_n < n) {
      if (g_trace) HIP_CHECK(hipFree(g_trace));
      HIP_CHECK(hipMalloc(&g_trace, size_t(n) * 8));
      g_trace_n = n;
    }
    HIP_CHECK(hipMemsetAsync(g_trace, 0, size_t(n) * 8, s));
    A.trace = g_trace;
    A.trace_k = trace_k;
  }
  // every polled word zeroed before EVERY launch (a memset node when captured)
  HIP_CHECK(hipMemsetAsync(ws, 0, kPersistPolled, s));
  static_assert(sizeof(T) == 8, "pcg1p: fp64 storage");
  hipLaunchKernelGGL((k_pcg1_persist<T, double>), dim3(nwg), dim3(kPersistThreads), 0, s, G, Tb, w, r, r2, p0,
                     p1, S, ws, A);
  HIP_CHECK(hipGetLastError());
  return nwg;
}

std::vector<unsigned long long> pcg1_persist_trace() {
  std::vector<unsigned long long> h(static_cast<size_t>(g_trace_n));
  if (g_trace_n) HIP_CHECK(hipMemcpy(h.data(), g_trace, h.size() * 8, hipMemcpyDeviceToHost));
  return h;
}

int pcg1_persist_max_wg(int device) {
  int cus = 0;
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  return std::min(cus, kPersistMaxWg);  // one workgroup per CU: always resident together
}

template int launch_pcg1_persist<double>(const DevGeom&, const DevTables&, double*, double*, double*, double*,
                                         double*, PcgState*, PersistWs*, const TileCfg&, const Pcg1Slot*,
                                         const int*, int, long long, const double*, hipStream_t);

void pcg1_persist_schedule(const TileCfg& tc, int nwaves, double cut_row_cost, Pcg1Slot* d_sched, int* d_offs) {
  const int n = tc.ntiles();
  std::vector<Pcg1Slot> ord(static_cast<size_t>(n));
  HIP_CHECK(hipMemcpy(ord.data(), tc.order0, ord.size() * sizeof(Pcg1Slot), hipMemcpyDeviceToHost));
  // cost of a tile in row steps: TI + 4 marched rows, each cut row (class 0) cut_row_cost more
  const int rows = tc.rows + 5;  // classes of rows i0-3 .. i1+2 (Pcg1Slot), when they fit 64 bits
  std::vector<double> cost(ord.size());
  for (size_t t = 0; t < ord.size(); ++t) {
    int ncut = 0;
    if (rows <= 32) {
      for (int q = 0; q < rows; ++q) ncut += ((ord[t].cls >> (2 * q)) & 3ull) == 0;
    }
    cost[t] = tc.rows + 4 + cut_row_cost * ncut;
  }
  // longest-processing-time-first onto the least loaded wave (ties: the lowest wave index), so the
  // slowest wave -- the sweep -- carries as little as a static schedule allows; fixed, so every run
  // and every sweep sums the same partials in the same order
  std::vector<int> idx(ord.size());
  for (size_t t = 0; t < idx.size(); ++t) idx[t] = int(t);
  std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return cost[size_t(a)] > cost[size_t(b)]; });
  typedef std::pair<double, int> Load;
  std::priority_queue<Load, std::vector<Load>, std::greater<Load>> heap;
  for (int w = 0; w < nwaves; ++w) heap.push({0.0, w});
  std::vector<std::vector<int>> per(static_cast<size_t>(nwaves));
  for (int t : idx) {
    Load l = heap.top();
    heap.pop();
    per[size_t(l.second)].push_back(t);
    heap.push({l.first + cost[size_t(t)], l.second});
  }
  std::vector<Pcg1Slot> sched;
  std::vector<int> offs(1, 0);
  sched.reserve(ord.size());
  for (auto& v : per) {
    for (int t : v) sched.push_back(ord[size_t(t)]);
    offs.push_back(int(sched.size()));
  }
  HIP_CHECK(hipMemcpy(d_sched, sched.data(), sched.size() * sizeof(Pcg1Slot), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_offs, offs.data(), offs.size() * sizeof(int), hipMemcpyHostToDevice));
}

}  // namespace pmx
