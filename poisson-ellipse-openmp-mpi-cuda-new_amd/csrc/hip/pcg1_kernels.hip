// Single-pass PCG iteration ("pcg1"): ONE streaming kernel and ONE 5-value reduction per
// iteration, instead of pcg_a + pcg_b with two reductions (pcg_kernels_dpp.hip).
//
// The reference iteration (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:847-943; stage0/
// Withoutopenmp1.cpp:124-169) needs the global (A p^k, p^k) before it can update r, which is
// what forces two sweeps.  pcg1 gets that denominator from the previous sweep instead:
//   p^k = z^{k-1} + beta_k p^{k-1}
//   (A p^k, p^k) = (A z, z) + 2 beta_k (A z, p^{k-1}) + beta_k^2 (A p^{k-1}, p^{k-1}),  z = z^{k-1}
// so sweep k-1 also accumulates (A z^{k-1}, z^{k-1}) and (A z^{k-1}, p^{k-1}) next to (z, r) and
// (A p, p).  Sweep k then has alpha_k before it starts and does everything in one pass:
//   p^k = z + beta p;  A p^k (explicit 5-point stencil, not a recurrence);  r^k = r - alpha A p^k;
//   z^k = D^-1 r^k;  A z^k;  partials (z^k, r^k), (A z^k, z^k), (A z^k, p^k), (A p^k, p^k), |p^k|^2.
// r is updated with an explicitly computed A p^k exactly as in the reference, only alpha's
// denominator is formed differently.  Measured in fp64 the expanded denominator differs from the
// direct one by <= 1.4e-15 relative, and every iteration count is unchanged: the reference grids
// 15/26/50/546/989/1858/2449 are GPU tests (tests/test_gpu_pcg1.py), and 32768^2 takes 14,316
// iterations with both pcg1 and pcg2 (profiles/r2/big_32768_records.md).
//
// Mapping (CDNA4): one wave64 marches a tile of TI rows x (64*VEC - 4) owned columns with a
// 3-stage row pipeline (A: p^k of row m, B: A p^k / r^k / z^k of row m-1, C: A z^k of row m-2).
// The dependency radius is 2 (A z^k needs z^k of the neighbours, which needs A p^k there), so a
// tile loads 2 extra columns on each side (overlapped tiles: the edge lanes compute values that
// only feed their neighbours, DPP lane shifts supply j +- 1) and marches 2 extra rows above and
// below.  Loads are 2-column chunks (16 B in fp64), aligned because tiles start at even offsets.
// w uses the paired update of k_pcg_b_rows_paired: odd iterations skip w, even ones apply
// alpha_{k-1} p^{k-1} + alpha_k p^k, and p^{k-1} is the p_old this kernel reads anyway.
// HBM traffic: r, p read + written (32 B) + w every other iteration (8 B) = 40 B/pt/iteration
// (pcg_a + pcg_b: 56), one deterministic reduction and one all-reduce per iteration (pcg2: two).
//
// Decomposed grids: the radius-2 dependency needs r^{k-1} and p^{k-1} on the owned block grown by
// a diamond of radius 2 -- two ghost lines per side plus ONE corner value per diagonal neighbour
// ((0,0), (0,ny+1), (nx+1,0), (nx+1,ny+1)).  Fields carry 2 ghost rows above/below and 2 ghost
// columns left/right (column -1 sits in the previous row's padding); k_pcg1_halo packs/unpacks
// them (8 slots: 4 sides, 4 corners) and the sweep reads ghosts like interior values, deciding
// "interior vs Dirichlet" on global indices.  Values outside the diamond (e.g. (-1, 0)) are never
// exchanged: they only feed columns/rows that are not owned, which are neither stored nor summed.
#include <algorithm>
#include <cmath>
#include <type_traits>
#include <utility>
#include <vector>

#include "pcg1_march.hpp"
#include "pcg_device.hpp"
#include "pmx/common.hpp"
#include "pmx/kernels.hpp"
#include "pmx/spec.hpp"

namespace pmx {

using namespace dev;

namespace {

constexpr int kPcg1AutoPf = 1;
// waves/SIMD bounds of the fp32-arithmetic sweeps (plain, w)
#ifndef PMX_PCG1_F32_WAVES
#define PMX_PCG1_F32_WAVES 4
#endif
#ifndef PMX_PCG1_F32_WAVES_W
#define PMX_PCG1_F32_WAVES_W 4
#endif
constexpr int kPcg1F32Waves = PMX_PCG1_F32_WAVES, kPcg1F32WavesW = PMX_PCG1_F32_WAVES_W;

#ifdef PMX_WAVE_TRACE
// Diagnostic build only (bench/wave_trace.sh): per-wave start/end wall clock, XCC and HW ids and
// tile of ONE chosen sweep, to see how the wave population ramps up and drains.
__device__ unsigned long long* g_wtrace = nullptr;
__device__ long long g_wtrace_it = -1;
#endif

// Waves per SIMD the register allocation must allow (VEC=2, 1 wave/workgroup):
//  * fp64: 139 VGPRs at PF=1 and 153 at PF=2 fit 3 waves/SIMD with no spills; forcing 4 (127
//    VGPRs, 4 spilled) is 2.65% slower (NOTES #36).  PF >= 3 runs at 2.
//  * fp32 storage (half the prefetch registers): PF=1 -- 32768^2 4.54 vs 5.03 ms at 3 waves/SIMD
//    with PF=2 (NOTES #37).
// Other shapes: whatever the allocator picks.
//  * The sweeps that move w (WS, one in w_cycle) are a kernel of their own: without the w paths
//    the plain sweep needs 113 VGPRs in fp64 / 111 in fp32 and runs at 4 waves/SIMD; the w sweep
//    with the triple paths (149 / 135 VGPRs) at 3 (profiles/r2/prologue/, profiles/r2/fp32_w3/).
//  * (round 3) the plain sweeps with deeper prefetch still fit 4 waves/SIMD: fp32 PF 2/3 (119 / 121
//    VGPRs) and fp64 PF 2 (131 free, 128 forced).
//  * fp32 arithmetic (C = float): the fp32 pipeline needs about half the registers; whatever the
//    allocator picks at the 4-wave bound of the plain sweep (see kPcg1F32Waves).
template <typename T, typename C, int VEC, int WAVES, int PF, bool WS>
constexpr int pcg1_min_waves() {
  // lockstep workgroups (WAVES 4 / 8, fp64, prefetch 1): the plain sweep at 4 waves per SIMD (2
  // eight-wave or 4 four-wave workgroups per CU), the w sweep at 3 with four-wave workgroups
  if (VEC == 2 && (WAVES == 4 || WAVES == 8) && PF == 1 && std::is_same_v<C, double>)
    return WS ? (WAVES == 4 ? 3 : 2) : 4;
  if (VEC != 2 || WAVES != 1) return 1;
  if (std::is_same_v<C, float>) return WS ? kPcg1F32WavesW : kPcg1F32Waves;
  if (!WS && (PF == 1 || (sizeof(T) == 4 && PF <= 3) || (sizeof(T) == 8 && PF == 2))) return 4;
  return PF <= 2 ? 3 : 2;  // the w sweeps (triple paths) and fp64 PF 3
}

// Which tiles a launch covers (launch_pcg1's part) and where tile k of that launch sits.
struct Pcg1Part {
  int part;  // 0 all, 1 interior rectangle, 2 frame
  int tiles_i, ti_lo, ti_hi, tj_lo, tj_hi;
  const Pcg1Slot* order;  // position -> tile + row classes (pcg1_build_order), or nullptr: pcg1_tile's order
  int count;         // tiles of this launch
};

// k-th tile of the part -> (ti, tj); false past the end.  The frame is enumerated as: tile rows
// above the interior rectangle, tile rows below it, then the left and right columns beside it.
__host__ __device__ inline bool pcg1_tile(int k, const Pcg1Part& P, int tiles_j, int& ti, int& tj) {
  if (P.part == 0) {
    ti = k / tiles_j;
    tj = k - ti * tiles_j;
    return ti < P.tiles_i;
  }
  const int h = P.ti_hi - P.ti_lo;
  if (P.part == 1) {
    const int wj = P.tj_hi - P.tj_lo;
    if (wj <= 0 || k >= h * wj) return false;
    ti = P.ti_lo + k / wj;
    tj = P.tj_lo + k % wj;
    return true;
  }
  const int ntop = P.ti_lo * tiles_j;
  if (k < ntop) { ti = k / tiles_j; tj = k % tiles_j; return true; }
  k -= ntop;
  const int nbot = (P.tiles_i - P.ti_hi) * tiles_j;
  if (k < nbot) { ti = P.ti_hi + k / tiles_j; tj = k % tiles_j; return true; }
  k -= nbot;
  if (P.tj_lo > 0 && k < h * P.tj_lo) { ti = P.ti_lo + k / P.tj_lo; tj = k % P.tj_lo; return true; }
  k -= h * P.tj_lo;
  const int wr = tiles_j - P.tj_hi;
  if (wr > 0 && k < h * wr) { ti = P.ti_lo + k / wr; tj = P.tj_hi + k % wr; return true; }
  return false;
}

template <typename T, typename C, int VEC, int WAVES, int PF, bool WS, int DPF = 0>
__global__ void __launch_bounds__(64 * WAVES, (pcg1_min_waves<T, C, VEC, WAVES, PF, WS>()))
k_pcg1(DevGeom G, DevTables Tb, T* __restrict__ w, T* r, T* r2, T* p0, T* p1,
       double* __restrict__ partials, PcgState* S, int TI, int tiles_j, int ntiles, Pcg1Part part) {
  constexpr int WO = 64 * VEC - 4;  // owned columns per tile
#ifdef PMX_WAVE_TRACE
  const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime();
#endif
  // Prologue: ONE batch of independent scalar loads (kernel arguments; then the state through the
  // constant address space and the tile's dispatch slot), then the shared control logic
  // (pcg1_march.hpp: pcg1_scalars -- stop test, breakdown guard, w-phase check, ring writes).
  asm volatile("" ::"s"(S), "s"(part.order), "s"(part.count), "s"(gridDim.x));  // kernel arguments: one batch
  const int pos = xcd_remap(blockIdx.x, gridDim.x) * WAVES + __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  // branch-free: without an order the load reads a valid dummy (the state's first 16 bytes)
  const Pcg1Slot* obase = part.order ? part.order : reinterpret_cast<const Pcg1Slot*>(S);
  const int oi = part.order ? min(pos, part.count - 1) : 0;
  const int ord = ld_uniform(&obase[oi].id, 0);
  const unsigned long long ocls = ld_uniform(&obase[oi].cls, 0);
  const Pcg1Pro pro = pcg1_load_state(S);
  pcg1_batch(pro, ord, ocls);
  Pcg1Sweep sw;
  if (!pcg1_scalars<WS>(pro, S, blockIdx.x == 0 && threadIdx.x == 0, sw)) return;
  const long long k = sw.k;
  const double alpha = sw.alpha, beta = sw.beta, c1 = sw.c1, c2 = sw.c2;
  const int wm = sw.wm;
  int ti = 0, tj = 0;
  if (part.order) {  // slow (ellipse-cut) tiles first, so they do not trail the sweep
    if (pos >= part.count || ord < 0) return;  // ord -1: an unused slot of a lockstep group
    ti = ord / tiles_j;
    tj = ord - ti * tiles_j;
  } else if (!pcg1_tile(pos, part, tiles_j, ti, tj)) {
    return;
  }
  const int id = ti * tiles_j + tj;  // the tile's partials slot, whichever launch covers it
  (void)ntiles;
  const int i0 = 1 + ti * TI, i1 = min(i0 + TI - 1, G.nx);
  const int j0 = 1 + tj * WO, j1 = min(j0 + WO - 1, G.ny);
  T* pnew = (k & 1) ? p1 : p0;
  const T* pold = (k & 1) ? p0 : p1;
  const T* rold = (k & 1) ? r2 : r;
  T* rnew = (k & 1) ? r : r2;
  double acc[kNq] = {0.0, 0.0, 0.0, 0.0, 0.0};
#ifdef PMX_WAVE_TRACE
  const unsigned long long wtm = __builtin_amdgcn_s_memrealtime();  // end of the prologue
#endif
  __shared__ double s_col[WAVES * 4 * VEC * 64];  // 4 KB per wave (VEC 2)
  double* scol = s_col + __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)) * (4 * VEC * 64);
  // interior tile: full width, and the marched rows i0-2..i1+2 / columns j0-2..j0+64*VEC-3 lie
  // strictly inside the global domain (no Dirichlet node in reach)
  const bool fast = VEC == 2 && j1 == j0 + WO - 1 && G.gi0 + i0 - 2 >= 1 && G.gi0 + i1 + 2 <= G.M - 1 &&
                    G.gj0 + j0 - 2 >= 1 && G.gj0 + j0 + 64 * VEC - 3 <= G.N - 1;
  const bool use_cls = part.order != nullptr && TI + 5 <= 64 / 2;  // 2 bits for each of the TI+5 rows
  const ArithF AF{float(G.cx), float(G.cy), float(G.dinv_in), float(G.dinv_out), float(G.inv_eps)};
#define PMX_MARCH(E, F)                                                                                       \
  pcg1_march<T, C, VEC, PF, E, F, 0, (WAVES > 1)>(G, Tb, AF, w, rold, rnew, pold, pnew, i0, i1, j0, j1, alpha, beta, \
                                                c1, c2, acc, scol, ocls, use_cls)
  // LDS-DMA ring of the FAST march (pcg1_march's DPF mode): DPF slots of r, p (, w) rows per wave
  constexpr int kRingDoubles = DPF > 0 ? DPF * (WS ? 3 : 2) * 128 : 2;
  __shared__ double s_ring[WAVES * kRingDoubles];
  double* dring = s_ring + __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)) * kRingDoubles;
  (void)dring;
#define PMX_MARCH_D(E)                                                                                            \
  pcg1_march<T, C, VEC, PF, E, true, DPF>(G, Tb, AF, w, rold, rnew, pold, pnew, i0, i1, j0, j1, alpha, beta, c1, c2, \
                                          acc, scol, ocls, use_cls, dring)
#define PMX_MARCH_W(F)                                     \
  if constexpr (!WS) {                                     \
    PMX_MARCH(0, F);                                       \
  } else {                                                 \
    switch (wm) {                                          \
      case 1: PMX_MARCH(1, F); break;                      \
      case 2: PMX_MARCH(2, F); break;                      \
      default: PMX_MARCH(3, F); break;                     \
    }                                                      \
  }
  if constexpr (DPF > 0 && sizeof(T) == 8 && VEC == 2) {
    if (fast && i1 - i0 + 1 >= DPF && (!WS || wm == 1 || wm == 2)) {
      if constexpr (!WS) {
        PMX_MARCH_D(0);
      } else {
        if (wm == 1) PMX_MARCH_D(1);
        else PMX_MARCH_D(2);
      }
      goto marched;
    }
  }
  if (fast) {
    PMX_MARCH_W(true)
  } else {
    PMX_MARCH_W(false)
  }
marched:
#undef PMX_MARCH_D
#undef PMX_MARCH_W
#undef PMX_MARCH
  wave_sum2_mfma(acc[0], acc[1]);
  wave_sum2_mfma(acc[2], acc[3]);
  acc[4] = wave_sum_mfma(acc[4]);
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int q = 0; q < kNq; ++q) partials[int64_t(kNq) * id + q] = acc[q];
  }
#ifdef PMX_WAVE_TRACE
  if (g_wtrace && k == g_wtrace_it && (threadIdx.x & 63) == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    unsigned long long* o = g_wtrace + 5 * int64_t(blockIdx.x);
    o[0] = wt0;
    o[1] = t1;
    o[2] = (static_cast<unsigned long long>(xcc) << 32) | hw;
    o[3] = static_cast<unsigned long long>(id) | (static_cast<unsigned long long>(part.part) << 40);
    o[4] = wtm;
  }
#endif
}

// Radius-2 ghost exchange of the single-pass iteration (see the header): pack (unpack = 0) copies
// the owned edge lines of the buffers the NEXT sweep reads -- sweep kk (the exchange's target,
// known on the host and baked into captured graphs, which are therefore keyed by its parity) reads
// r^{k-1} = (kk & 1 ? r2 : r) and p^{k-1} = (kk & 1 ? p0 : p1) -- into the send slots; unpack
// copies the receive slots into the ghost cells of the same buffers.  No device state is read, so
// the next sweep (which writes S) never has to wait for a pack.  Slot layout: sides
// [field][line][pos] (field 0 = r, 1 = p; line q = ghost row/column -1+q on the receiving side,
// ordered by increasing index), corners [field].  Grid: (ceil(max(nx, ny) / 256), 8 slots,
// 4 = (field, line)).  Tiny and stream-ordered; launched by the driver between two sweeps.
template <typename T>
__global__ void __launch_bounds__(256)
k_pcg1_halo(DevGeom G, T* r, T* r2, T* p0, T* p1, HaloBufs<T> H, long long kk, int unpack,
            long long* progress) {
  const int slot = blockIdx.y;
  // host-visible progress (hang diagnosis): [1] = exchanges packed, [2] = exchanges unpacked --
  // counted, since kk is baked into graphs that replay at later iterations of the same parity
  if (progress && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0)
    __hip_atomic_fetch_add(progress + (unpack ? 2 : 1), 1ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (!((G.nb >> slot) & 1)) return;
  const int f = blockIdx.z >> 1, q = blockIdx.z & 1;
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int nx = G.nx, ny = G.ny;
  int li, lj, idx;
  if (slot < 2) {          // x sides: rows
    if (t >= ny) return;
    li = slot == 0 ? (unpack ? -1 + q : 1 + q) : (unpack ? nx + 1 + q : nx - 1 + q);
    lj = 1 + t;
    idx = (f * 2 + q) * ny + t;
  } else if (slot < 4) {   // y sides: columns
    if (t >= nx) return;
    li = 1 + t;
    lj = slot == 2 ? (unpack ? -1 + q : 1 + q) : (unpack ? ny + 1 + q : ny - 1 + q);
    idx = (f * 2 + q) * nx + t;
  } else {                 // corners: one value per field
    if (t != 0 || q != 0) return;
    const bool xhi = slot >= 6, yhi = slot == 5 || slot == 7;
    li = xhi ? (unpack ? nx + 1 : nx) : (unpack ? 0 : 1);
    lj = yhi ? (unpack ? ny + 1 : ny) : (unpack ? 0 : 1);
    idx = f;
  }
  T* fld = f == 0 ? ((kk & 1) ? r2 : r) : ((kk & 1) ? p0 : p1);
  const int64_t o = int64_t(li) * G.pitch + lj;
  if (unpack)
    fld[o] = H.recv[slot][idx];
  else
    H.send[slot][idx] = fld[o];
}

// Deterministic reduction of n partial vectors of NQ values (fixed chunk order, MFMA wave sums),
// multi-block with a ticketed last-block finish like k_reduce (pcg_kernels.hip).
struct ReduceWeights {
  double w[8];
};

template <int NQ>
__global__ void __launch_bounds__(256)
k_reduce_n(const double* __restrict__ part, int n, ReduceWeights wt, double* out, PcgState* S,
           int mode, double* chunk, unsigned* ticket, long long* progress) {
  __shared__ double lds[NQ][256 / kWave];
  __shared__ int last;
  if ((mode & kSkipIfDone) && S->done) return;
  const int nb = int(gridDim.x);
  const int lo = int(int64_t(n) * blockIdx.x / nb);
  const int hi = int(int64_t(n) * (blockIdx.x + 1) / nb);
  double s[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) s[q] = 0.0;
#pragma unroll 4
  for (int i = lo + int(threadIdx.x); i < hi; i += 256) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) s[q] += part[int64_t(i) * NQ + q];
  }
  const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    s[q] = wave_sum_mfma(s[q]);
    if (lane == 0) lds[q][wid] = s[q];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      st_publish(chunk + NQ * blockIdx.x + q, (lds[q][0] + lds[q][1]) + (lds[q][2] + lds[q][3]));
    last = ticket_arrive_last(ticket, nb);
  }
  __syncthreads();
  if (!last || threadIdx.x >= kWave) return;  // wave 0 of the last block finishes (full EXEC)
  const int l = int(threadIdx.x);
  double t[NQ];
  bool bad = false;
#pragma unroll
  for (int q = 0; q < NQ; ++q) t[q] = l < nb ? ld_published(chunk + NQ * l + q) : 0.0;  // all in flight
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    t[q] = wave_sum_mfma(t[q]);
    bad |= !(t[q] == t[q]) || isinf(t[q]);
  }
  if (l == 0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) out[q] = t[q] * wt.w[q];
    if (bad) S->nan_flag = 1;
    if (mode & kBumpIter) S->it += 1;
    // host-visible progress (hang diagnosis): [0] = sweeps reduced (the device iteration counter)
    if (progress) __hip_atomic_store(progress, S->it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    *ticket = 0u;  // re-arm for the next launch (stream order makes this visible to it)
  }
}

// Small n (<= kReduceOneMax partials): ONE workgroup of 1024 threads reads every partial (at most 3
// per thread, all in flight) and finishes on its own -- no chunk hand-off, no ticket, one memory
// round trip instead of three.  Same finish as k_reduce_n; the fixed summation order is
// thread-strided, then waves in order.
constexpr int kReduceOneMax = 3072;  // 1200x1800 blocks (2250): 36.3 vs 37.1 us; march 800x1200 (4000): 42.1 vs 41.8

template <int NQ, int NT>
__global__ void __launch_bounds__(NT)
k_reduce_1(const double* __restrict__ part, int n, ReduceWeights wt, double* out, PcgState* S, int mode,
           long long* progress) {
  __shared__ double lds[NQ][NT / kWave];
  if ((mode & kSkipIfDone) && S->done) return;
  double s[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) s[q] = 0.0;
#pragma unroll 4
  for (int i = int(threadIdx.x); i < n; i += NT) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) s[q] += part[int64_t(i) * NQ + q];
  }
  const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    s[q] = wave_sum_mfma(s[q]);
    if (lane == 0) lds[q][wid] = s[q];
  }
  __syncthreads();
  if (threadIdx.x >= kWave) return;  // wave 0 finishes (full EXEC)
  double t[NQ];
  bool bad = false;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    t[q] = wave_sum_mfma(lane < NT / kWave ? lds[q][lane] : 0.0);
    bad |= !(t[q] == t[q]) || isinf(t[q]);
  }
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) out[q] = t[q] * wt.w[q];
    if (bad) S->nan_flag = 1;
    if (mode & kBumpIter) S->it += 1;
    if (progress) __hip_atomic_store(progress, S->it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Per tile: the coefficient class of each row its march visits (rows i0-3 .. i1+2 over the tile's
// loaded columns, 2 bits per row, see Pcg1Slot) and whether any of them is "cut" (class 0: those
// rows rebuild every face from the tables, and such a tile takes 3-5x the median tile time,
// profiles/r2/small_shapes/README.md).  One thread per tile, the same rows and column window as
// pcg1_march.
__global__ void k_pcg1_tile_classes(DevGeom G, DevTables Tb, int TI, int tiles_i, int tiles_j, int vec,
                                    unsigned long long* cls, unsigned char* cut) {
  const int id = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (id >= tiles_i * tiles_j) return;
  const int ti = id / tiles_j, tj = id - ti * tiles_j;
  const int i0 = 1 + ti * TI, i1 = min(i0 + TI - 1, G.nx);
  const int j0 = 1 + tj * (64 * vec - 4);
  const int gjlo = max(G.gj0 + j0 - 2, 0), gjhi = min(G.gj0 + j0 - 2 + 64 * vec - 1, G.N);
  unsigned char c = 0;
  unsigned long long bits = 0;
  for (int m = i0 - 3; m <= i1 + 2; ++m) {
    const int gi = min(max(G.gi0 + m, 0), G.M);
    RowConst rc;
    for (int q = 0; q < 4; ++q) {
      rc.ca0[q] = Tb.acls[4 * gi + q];
      rc.ca1[q] = Tb.acls[4 * (gi + 1) + q];
      rc.cb[q] = Tb.bcls[4 * gi + q];
    }
    const int u = row_class(rc, gjlo, gjhi);
    c |= u == 0;
    const int r = m - (i0 - 3);
    if (r < 32) bits |= static_cast<unsigned long long>(u) << (2 * r);
  }
  cut[id] = c;
  cls[id] = bits;
}

}  // namespace

size_t pcg1_order_slots(const TileCfg& tc) {
  // one group per tc.waves tiles of a tile row at most: per part ntiles + tiles_i * (waves - 1) slots
  const size_t per = size_t(tc.ntiles()) + size_t(tc.tiles_i + 2) * size_t(tc.waves);
  return 3 * per;
}

int pcg1_build_order(const DevGeom& G, const DevTables& Tb, TileCfg& tc, Pcg1Slot* d_order, bool slow_first,
                     hipStream_t s) {
  tc.order0 = tc.order1 = tc.order2 = nullptr;
  tc.groups[0] = tc.groups[1] = tc.groups[2] = 0;
  const int n = tc.ntiles();
  if (n == 0) return 0;
  const int gw = tc.waves;  // slots per group (1: every tile its own workgroup)
  unsigned char* d_cut = nullptr;
  unsigned long long* d_cls = nullptr;
  HIP_CHECK(hipMalloc(&d_cut, size_t(n)));
  HIP_CHECK(hipMalloc(&d_cls, size_t(n) * sizeof(unsigned long long)));
  hipLaunchKernelGGL(k_pcg1_tile_classes, dim3((n + 255) / 256), dim3(256), 0, s, G, Tb, tc.rows, tc.tiles_i,
                     tc.tiles_j, tc.vec, d_cls, d_cut);
  HIP_CHECK(hipGetLastError());
  std::vector<unsigned char> cut(static_cast<size_t>(n));
  std::vector<unsigned long long> cls(static_cast<size_t>(n));
  HIP_CHECK(hipMemcpyAsync(cut.data(), d_cut, size_t(n), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(cls.data(), d_cls, size_t(n) * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  HIP_CHECK(hipFree(d_cut));
  HIP_CHECK(hipFree(d_cls));
  const size_t per = pcg1_order_slots(tc) / 3;
  std::vector<Pcg1Slot> order(3 * per, Pcg1Slot{-1, 0, 0ull});
  int nslow = 0;
  for (int part = 0; part <= 2; ++part) {
    const Pcg1Part P{part, tc.tiles_i, tc.ti_lo, tc.ti_hi, tc.tj_lo, tc.tj_hi, nullptr, 0};
    const int count = part == 0 ? n : part == 1 ? tc.interior_tiles() : n - tc.interior_tiles();
    // groups: runs of up to gw consecutive tiles of the part's enumeration within one tile row
    std::vector<std::vector<int>> groups;
    for (int k = 0, last_ti = -1; k < count; ++k) {
      int ti = 0, tj = 0;
      PMX_CHECK(pcg1_tile(k, P, tc.tiles_j, ti, tj), "pcg1_build_order: tile enumeration");
      if (groups.empty() || ti != last_ti || int(groups.back().size()) == gw) groups.emplace_back();
      groups.back().push_back(ti * tc.tiles_j + tj);
      last_ti = ti;
    }
    const int ng = int(groups.size());
    PMX_CHECK(size_t(ng) * size_t(gw) <= per, "pcg1_build_order: order capacity");
    tc.groups[part] = gw > 1 ? ng : 0;
    Pcg1Slot* o = order.data() + size_t(part) * per;
    auto has_cut = [&](const std::vector<int>& g) {
      for (int id : g)
        if (cut[size_t(id)]) return true;
      return false;
    };
    // the groups of XCD x (xcd_remap over ng workgroups): [x (q+1), ...) as in xcd_remap
    const int q = ng / 8, r = ng % 8;
    for (int x = 0, start = 0; x < 8; ++x) {
      const int len = q + (x < r ? 1 : 0);
      int w = start;
      for (int pass = 0; pass < (slow_first ? 2 : 1); ++pass)  // slow groups first, then the rest
        for (int g = start; g < start + len; ++g)
          if (!slow_first || has_cut(groups[size_t(g)]) == (pass == 0)) {
            for (size_t u = 0; u < groups[size_t(g)].size(); ++u) {
              const int id = groups[size_t(g)][u];
              o[size_t(w) * gw + u] = Pcg1Slot{id, 0, cls[size_t(id)]};
              if (slow_first && pass == 0 && part == 0 && cut[size_t(id)]) ++nslow;
            }
            ++w;
          }
      start += len;
    }
  }
  HIP_CHECK(hipMemcpyAsync(d_order, order.data(), order.size() * sizeof(Pcg1Slot), hipMemcpyHostToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));
  tc.order0 = d_order;
  tc.order1 = d_order + per;
  tc.order2 = d_order + 2 * per;
  return nslow;
}

TileCfg make_pcg1_tiles(const DevGeom& G, int vec, int waves, int rows, int pf, int elem) {
  PMX_CHECK(vec == 2 || vec == 4, "pcg1: vec must be 2 or 4");
  PMX_CHECK(pf >= 0 && pf <= 4, "pcg1: prefetch depth must be 0 (auto) or 1..4");
  PMX_CHECK(pf <= 1 || (vec == 2 && waves == 1), "pcg1: prefetch depth > 1 needs vec 2 x 1 wave");
  PMX_CHECK(waves == 1 || waves == 2 || waves == 4 || waves == 8, "pcg1: waves must be 1, 2, 4 or 8");
  PMX_CHECK(vec == 2 || waves == 1, "pcg1: VEC 4 runs 1 wave per workgroup");
  TileCfg t;
  t.kind = 3;
  t.vec = vec;
  t.waves = waves;
  t.block = 64 * vec - 4;  // owned columns per tile
  // fp32 storage: 24-row tiles (profiles/r2/fp32_pcg1_sweep.txt)
  const bool fp32 = elem == 4;
  // fp32 storage: prefetch 2 rows (its plain sweep still fits 4 waves/SIMD at 117 VGPRs); half-size
  // rows keep too few bytes in flight at depth 1: 32768^2 -10%, 16384^2 -3% (profiles/r3/prefetch/)
  t.pf = pf ? pf : (vec == 2 && waves == 1 ? (fp32 ? 2 : kPcg1AutoPf) : 1);
  t.tiles_j = (G.ny + t.block - 1) / t.block;
  if (rows <= 0) {
    // tall tiles keep the 4 extra marched rows cheap; shorter only when the grid is small
    // (>= ~8K tiles keep 3 waves/SIMD busy for a few rounds)
    // fp64, interleaved same-box A/B (profiles/r2/pcg1_rows_sweep.txt): 16384^2 8 rows = 12 rows
    // (+-0.1%), 16 rows +1.4%, 32 rows +7%; the 8-GPU per-rank shape 4096x8192: 8 rows 374 us,
    // 12 rows 388 us (shorter tiles shrink the last, partly filled round of waves).  Short tiles
    // keep fewer DRAM rows in flight and win despite the 4 extra marched rows.
    rows = fp32 ? 24 : 8;
    while (rows > 4 && int64_t((G.nx + rows - 1) / rows) * t.tiles_j < 8192) rows /= 2;
    // (round 5) fp64 grids with >= 16K twelve-row tiles: 12 rows.  Fresh-process A/B, 3 rounds:
    // 16384^2 2093.8 -> 2060.7 us (-1.6%) without the probe, 1939.3 -> 1903.5 (-1.8%) with it;
    // 2048x16384 (the 8-GPU strip) 261.6 either way (studies r5h, r5i; NOTES #101)
    if (!fp32 && int64_t((G.nx + 11) / 12) * t.tiles_j >= 16384) rows = 12;
    // the reference's smallest grid (800x1200: 2000 tiles of 4 rows, ~2 waves per SIMD) is bound by
    // one wave's serial row march: 2-row tiles double the waves and cut the march from 8 row steps
    // to 6 -- 50.1 -> 41.6 us/iteration; 1 row (5 steps, 4x the rows marched) 47.1; at 1600x2400
    // (8000 tiles of 4 rows) 2 rows lose, 60.8 -> 73.1 (profiles/r4/persist/rows_*.log)
    if (rows == 4 && int64_t((G.nx + 3) / 4) * t.tiles_j < 4096) rows = 2;
  }
  PMX_CHECK(rows >= 1 && rows <= 4096, "pcg1: tile rows must be in [1, 4096]");
  t.rows = rows;
  t.tiles_i = (G.nx + rows - 1) / rows;
  // interior rectangle: tiles whose marched rows i0-2 .. i1+2 and loaded columns j0-2 ..
  // j0+64*vec-3 stay clear of the ghost cells of every side that has a neighbour
  auto cdiv = [](int a, int b) { return a <= 0 ? 0 : (a + b - 1) / b; };
  t.ti_lo = (G.nb & kNbXlo) ? (rows == 1 ? 2 : 1) : 0;
  t.ti_hi = (G.nb & kNbXhi) ? std::max(0, cdiv(G.nx - 1, rows) - 1) : t.tiles_i;
  t.tj_lo = (G.nb & kNbYlo) ? 1 : 0;
  t.tj_hi = (G.nb & kNbYhi) ? cdiv(G.ny + 3 - 64 * vec, t.block) : t.tiles_j;
  t.ti_lo = std::min(t.ti_lo, t.tiles_i);
  t.ti_hi = std::min(std::max(t.ti_hi, t.ti_lo), t.tiles_i);
  t.tj_lo = std::min(t.tj_lo, t.tiles_j);
  t.tj_hi = std::min(std::max(t.tj_hi, t.tj_lo), t.tiles_j);
  return t;
}

int pcg1_lds_pad(int wpcu, int waves) {
  if (wpcu <= 0) return 0;
  constexpr int kLdsPerCu = 160 * 1024;
  const int per_wg = (kLdsPerCu / std::max(1, wpcu / std::max(1, waves))) & ~511;  // 512-B granules
  return std::max(0, per_wg - waves * 4096);
}

template <typename T>
void launch_pcg1(const DevGeom& G, const DevTables& Tb, T* w, T* r, T* r2, T* p0, T* p1,
                 double* partials, PcgState* S, const TileCfg& tc, hipStream_t s, int part, bool wsweep) {
  PMX_CHECK(tc.kind == 3, "launch_pcg1 needs make_pcg1_tiles");
  PMX_CHECK(part >= 0 && part <= 2, "launch_pcg1: part must be 0, 1 or 2");
  const int tiles = part == 0 ? tc.ntiles() : part == 1 ? tc.interior_tiles() : tc.ntiles() - tc.interior_tiles();
  const Pcg1Slot* ord = part == 0 ? tc.order0 : part == 1 ? tc.order1 : tc.order2;
  // lockstep workgroups: one per group of the order (tc.groups), tc.waves slots each
  const bool grouped = tc.waves > 1 && ord != nullptr;
  PMX_CHECK(tc.waves == 1 || grouped, "pcg1: workgroups of several waves need the grouped dispatch order");
  const int nb = grouped ? tc.groups[part] : tiles;
  const int count = grouped ? nb * tc.waves : tiles;
  const Pcg1Part P{part, tc.tiles_i, tc.ti_lo, tc.ti_hi, tc.tj_lo, tc.tj_hi, ord, count};
  if (tiles == 0) return;
  PMX_CHECK(G.nb == 0 || (G.nx >= 2 && G.ny >= 2), "pcg1 on a decomposed grid needs subdomains >= 2 x 2");
  const int bs = 64 * tc.waves;
#define PMX_PCG1_CD(C, V, WV, PF, D)                                                                     \
  do {                                                                                                   \
    if (wsweep)                                                                                          \
      hipLaunchKernelGGL((k_pcg1<T, C, V, WV, PF, true, D>), dim3(nb), dim3(bs), tc.lds_pad, s, G, Tb, w, r, r2, \
                         p0, p1, partials, S, tc.rows, tc.tiles_j, tc.ntiles(), P);                      \
    else                                                                                                 \
      hipLaunchKernelGGL((k_pcg1<T, C, V, WV, PF, false, D>), dim3(nb), dim3(bs), tc.lds_pad, s, G, Tb, w, r, r2, \
                         p0, p1, partials, S, tc.rows, tc.tiles_j, tc.ntiles(), P);                      \
  } while (0)
  // the LDS-DMA march (tc.dpf rows ahead): fp64 storage and arithmetic, the default tile shape
#define PMX_PCG1_C(C, V, WV, PF)                                                                         \
  do {                                                                                                   \
    if constexpr (sizeof(T) == 8 && std::is_same_v<C, double> && V == 2 && WV == 1 && PF == 1) {        \
      if (tc.dpf == 2) { PMX_PCG1_CD(C, V, WV, PF, 2); break; }                                          \
      if (tc.dpf == 3) { PMX_PCG1_CD(C, V, WV, PF, 3); break; }                                          \
    }                                                                                                    \
    PMX_CHECK(tc.dpf == 0, "pcg1: the LDS-DMA march needs fp64, VEC 2 x 1 wave, prefetch 1 and dpf 2 or 3"); \
    PMX_PCG1_CD(C, V, WV, PF, 0);                                                                        \
  } while (0)
  // fp32 arithmetic: fp32 storage only, the default tile shape (VEC 2, 1 wave) and prefetch 1-3
#define PMX_PCG1(V, WV, PF)                                                                              \
  do {                                                                                                   \
    if constexpr (std::is_same_v<T, float> && V == 2 && WV == 1 && PF <= 3) {                            \
      if (tc.arith32) { PMX_PCG1_C(float, V, WV, PF); break; }                                           \
    }                                                                                                    \
    PMX_CHECK(!tc.arith32, "pcg1: fp32 arithmetic needs fp32 storage, VEC 2 x 1 wave and prefetch <= 3"); \
    PMX_PCG1_C(double, V, WV, PF);                                                                       \
  } while (0)
  // instantiated shapes: the default (VEC 2, 1 wave, prefetch 1) and prefetch 2.  The other
  // shapes of the round-1/2 sweeps (prefetch 3-4, 2 or 4 waves per workgroup, VEC 4: all slower,
  // NOTES #23, #40) need a PMX_PCG1_ALL_SHAPES build
  if (tc.vec == 2 && tc.waves == 1 && tc.pf == 1) PMX_PCG1(2, 1, 1);
  else if (tc.vec == 2 && tc.waves == 1 && tc.pf == 2) PMX_PCG1(2, 1, 2);
  else if (tc.vec == 2 && tc.waves == 1 && tc.pf == 3) PMX_PCG1(2, 1, 3);
  else if (tc.vec == 2 && tc.waves == 8 && tc.pf == 1) PMX_PCG1(2, 8, 1);
  else if (tc.vec == 2 && tc.waves == 4 && tc.pf == 1) PMX_PCG1(2, 4, 1);
#ifdef PMX_PCG1_ALL_SHAPES
  else if (tc.vec == 2 && tc.waves == 1) PMX_PCG1(2, 1, 4);
  else if (tc.vec == 2 && tc.waves == 2) PMX_PCG1(2, 2, 1);
  else PMX_PCG1(4, 1, 1);
#else
  else PMX_CHECK(false, "pcg1 shape vec " << tc.vec << " x " << tc.waves << " waves, prefetch " << tc.pf
                                          << " is only instantiated in a PMX_PCG1_ALL_SHAPES build");
#endif
#undef PMX_PCG1
#undef PMX_PCG1_C
#undef PMX_PCG1_CD
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_pcg1_halo(const DevGeom& G, T* r, T* r2, T* p0, T* p1, HaloBufs<T> H, long long target,
                      bool unpack, hipStream_t s, long long* progress) {
  if (G.nb == 0) return;
  const int len = std::max(G.nx, G.ny);
  hipLaunchKernelGGL(k_pcg1_halo<T>, dim3((len + 255) / 256, kHaloSlots, 4), dim3(256), 0, s, G, r, r2,
                     p0, p1, H, target, unpack ? 1 : 0, progress);
  HIP_CHECK(hipGetLastError());
}

void launch_reduce_n(const double* partials, int n, int nq, const double* weights, double* out,
                     PcgState* S, int mode, double* ws, hipStream_t s, long long* progress) {
  PMX_CHECK(nq == kNq, "launch_reduce_n: nq must be " << kNq);
  // ~512 partials per block: the loads of a block are 2 rounds per thread, not a latency chain
  // (4096x8192 fp64: 22.9K tiles, 11 -> 44 blocks)
  const int nb = std::max(1, std::min(kReduceMaxBlocks, n / 512));
  double* chunk = ws + kReduceNOffset;
  unsigned* ticket = reinterpret_cast<unsigned*>(chunk + 8 * kReduceMaxBlocks);
  ReduceWeights wt{};
  for (int q = 0; q < nq; ++q) wt.w[q] = weights[q];
  if (n <= kReduceOneMax)
    hipLaunchKernelGGL((k_reduce_1<kNq, 1024>), dim3(1), dim3(1024), 0, s, partials, n, wt, out, S, mode, progress);
  else
    hipLaunchKernelGGL(k_reduce_n<kNq>, dim3(nb), dim3(256), 0, s, partials, n, wt, out, S, mode, chunk, ticket,
                       progress);
  HIP_CHECK(hipGetLastError());
}

#ifdef PMX_WAVE_TRACE
void* pcg1_wave_trace_setup(long long it, int nwaves) {
  void* buf = nullptr;
  HIP_CHECK(hipMalloc(&buf, size_t(nwaves) * 40));
  HIP_CHECK(hipMemset(buf, 0, size_t(nwaves) * 40));
  HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_wtrace), &buf, sizeof(buf)));
  HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_wtrace_it), &it, sizeof(it)));
  return buf;
}
#endif

template void launch_pcg1<double>(const DevGeom&, const DevTables&, double*, double*, double*, double*,
                                  double*, double*, PcgState*, const TileCfg&, hipStream_t, int, bool);
template void launch_pcg1_halo<double>(const DevGeom&, double*, double*, double*, double*, HaloBufs<double>,
                                        long long, bool, hipStream_t, long long*);
template void launch_pcg1_halo<float>(const DevGeom&, float*, float*, float*, float*, HaloBufs<float>,
                                       long long, bool, hipStream_t, long long*);
template void launch_pcg1<float>(const DevGeom&, const DevTables&, float*, float*, float*, float*, float*,
                                 double*, PcgState*, const TileCfg&, hipStream_t, int, bool);

}  // namespace pmx
