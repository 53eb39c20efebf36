// Device building blocks of the single-pass PCG sweep (pcg1): column loads/stores, coefficient
// classes, stencil arithmetic in fp64 or fp32, the sweep prologue (scalars, stop test, breakdown
// guard, w schedule) and pcg1_march -- one wave's march over one tile.  Shared by the march kernel
// k_pcg1 (pcg1_kernels.hip) and the block-tile kernel k_pcg1_block (pcg1_block.hip).  See
// pcg1_kernels.hip's header for the algorithm.
#pragma once

#include <type_traits>
#include <utility>

#include "pcg_device.hpp"
#include "pmx/common.hpp"
#include "pmx/kernels.hpp"

namespace pmx {

using namespace dev;

namespace {

constexpr int kNq = 5;  // rho, (Az,z), (Az,p), (Ap,p), |p|^2

// ---- sweep prologue: ONE copy of the pcg1 control logic, used by k_pcg1 and k_pcg1_block --------
// (the reference's loop control, stage4-mpi+cuda/poisson_mpi_cuda_f.cu:847-943: the stop test, the
// |denominator| guard, alpha and beta -- here evaluated at the start of the sweep that needs them)

// The PcgState fields a sweep reads.  Every one is a field the sweep does not write (the rings
// alpha1 / beta1 / zr are written at slot k, read at k-1 / k-2), so the constant address space view
// is exact and the loads are scalar.
struct Pcg1Pro {
  int done, norm, cyc;
  long long k, max_iter;
  double rc[kNq], al[4], be[4];
  double zr0, zr1, delta, bd_tol, pmb;
};

__device__ __forceinline__ Pcg1Pro pcg1_load_state(const PcgState* S) {
  typedef const __attribute__((address_space(4))) PcgState CState;
  const CState* Sc = (const CState*)S;  // NOLINT: address-space cast
  Pcg1Pro v;
  v.done = Sc->done;
  v.k = Sc->it;  // 0 = the init sweep (alpha = beta = 0: sums of r^0, z^0 only)
#pragma unroll
  for (int q = 0; q < kNq; ++q) v.rc[q] = Sc->red_c[q];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v.al[q] = Sc->alpha1[q];
    v.be[q] = Sc->beta1[q];
  }
  v.zr0 = Sc->zr[0];
  v.zr1 = Sc->zr[1];
  v.delta = Sc->delta;
  v.bd_tol = Sc->bd_tol;
  v.pmb = Sc->pair_min_beta;
  v.max_iter = Sc->max_iter;
  v.norm = Sc->norm;
  v.cyc = Sc->w_cycle;
  return v;
}

// Every state value (and the tile's dispatch slot, id / cls) consumed by one empty asm, so the
// compiler issues all those scalar loads as ONE batch instead of sinking each below the branch that
// first needs it: read field by field with waits in between, the state cost ~8 dependent memory round
// trips, ~7 us of a ~25-us wave (wave traces, profiles/r2/prologue/).
__device__ __forceinline__ void pcg1_batch(const Pcg1Pro& v, int id, unsigned long long cls) {
  asm volatile("" ::"s"(v.done), "s"(v.k), "s"(id), "s"(cls), "s"(v.rc[0]), "s"(v.rc[1]), "s"(v.rc[2]), "s"(v.rc[3]),
               "s"(v.rc[4]), "s"(v.al[0]), "s"(v.al[1]), "s"(v.al[2]), "s"(v.al[3]), "s"(v.be[0]), "s"(v.be[1]),
               "s"(v.be[2]), "s"(v.be[3]), "s"(v.zr0), "s"(v.zr1), "s"(v.delta), "s"(v.bd_tol), "s"(v.pmb),
               "s"(v.max_iter), "s"(v.norm), "s"(v.cyc));
}

// What sweep k runs with.  wm: the w schedule of this sweep (0 = w untouched; 1 = pairs; 2 = triples
// with p^{k-2} recovered; 3 = triples re-reading p^{k-2}; see pcg1_march's WM).
struct Pcg1Sweep {
  long long k;
  double alpha, beta, c1, c2;
  int wm;
};

__device__ __forceinline__ double pcg1_ring4(const double (&v)[4], long long i) {
  const int j = int(i & 3);
  return j == 0 ? v[0] : j == 1 ? v[1] : j == 2 ? v[2] : v[3];
}

// The scalars of sweep k from the reduced sums of sweep k-1 (every workgroup computes the same
// values).  Returns false when the sweep must not run: the solve is done, iteration k-1 met the stop
// test or max_iter, alpha's denominator broke down, or the host launched the w kernel (WS) on the
// wrong phase.  `leader` (one lane of the whole launch) records the outcome and the rings in S.
template <bool WS>
__device__ __forceinline__ bool pcg1_scalars(const Pcg1Pro& v, PcgState* S, bool leader, Pcg1Sweep& o) {
  o = Pcg1Sweep{v.k, 0.0, 0.0, 0.0, 0.0, 0};
  if (v.done) return false;
  const long long k = v.k;
  if (k > 0) {
    const double rho = v.rc[0];  // rho_{k-1} = (z^{k-1}, r^{k-1})
    double diff = 0.0;
    if (k >= 2) {
      // stop test of iteration k-1: ||w^k - w^{k-1}|| = |alpha_{k-1}| ||p^{k-1}||
      diff = fabs(pcg1_ring4(v.al, k - 1)) * sqrt(v.rc[4]);
      const bool bad = !(diff == diff) || !(rho == rho);
      if (bad || diff < v.delta || k > v.max_iter) {
        if (leader) {
          S->diff = diff;
          S->iters = k - 1;
          S->status = bad ? int(Status::kBreakdown) : (diff < v.delta ? int(Status::kConverged) : int(Status::kMaxIter));
          if (bad) S->nan_flag = 1;
          S->done = 1;
        }
        return false;
      }
      o.beta = rho / ((k & 1) ? v.zr1 : v.zr0);  // rho_{k-2} sits in slot k & 1
    }
    // (A p^k, p^k) expanded from sweep k-1's sums (see pcg1_kernels.hip's header)
    const double beta = o.beta;
    const double denom = v.rc[1] + beta * (2.0 * v.rc[2] + beta * v.rc[3]);
    const bool bd = v.norm == int(Norm::kWeighted) ? fabs(denom) < v.bd_tol : denom < v.bd_tol;
    if (bd || !(denom == denom)) {
      if (leader) {
        if (k >= 2) S->diff = diff;
        S->iters = k;
        S->status = int(Status::kBreakdown);
        if (!(denom == denom)) S->nan_flag = 1;
        S->done = 1;
      }
      return false;
    }
    o.alpha = rho / denom;
    // w schedule.  Pairs (w_cycle 2): even sweeps add alpha_{k-1} p^{k-1} + alpha_k p^k, p^{k-1}
    // being the p_old the sweep reads anyway.  Triples (w_cycle 3, default): sweeps k = 0 mod 3
    // also add alpha_{k-2} p^{k-2}, recovered without reading it: sweep k-1 formed
    // p^{k-1} = D^-1 r^{k-2} + beta_{k-1} p^{k-2} and r^{k-1} = r^{k-2} - alpha_{k-1} A p^{k-1}, so
    // p^{k-2} = (p^{k-1} - D^-1 (r^{k-1} + alpha_{k-1} A p^{k-1})) / beta_{k-1} -- one more stencil,
    // on the p_old this sweep already holds.  Its rounding error grows like eps / |beta_{k-1}|, so
    // below pair_min_beta the sweep re-reads p^{k-2} from the buffer it is about to overwrite.
    // w moves on one sweep in three: 37.3 instead of 40 B/pt per iteration.  The stop test uses
    // |alpha| ||p||, so the schedule changes no iteration count, only w's rounding.
    const int ph = int(k % v.cyc);
    // the host launches the w-sweep kernel (WS) exactly on the sweeps k = 0 mod w_cycle; a
    // mismatch (host and device iteration counters out of step) must not pass silently
    if ((ph == 0) != WS) {
      if (leader) {
        S->iters = k;
        S->status = int(Status::kBreakdown);
        S->nan_flag = 1;
        S->done = 1;
      }
      return false;
    }
    if (ph == 0) {
      o.c1 = pcg1_ring4(v.al, k - 1);
      o.wm = 1;
      if (v.cyc == 3) {
        const double bprev = pcg1_ring4(v.be, k - 1);
        const double a2 = pcg1_ring4(v.al, k - 2);
        if (fabs(bprev) >= v.pmb) {
          o.wm = 2;
          o.c2 = a2 / bprev;
        } else {
          o.wm = 3;
          o.c2 = a2;
        }
      }
    }
    if (leader) {
      S->zr[(k - 1) & 1] = rho;  // slot of k-1 (read as rho_{k-2} by the next sweep)
      S->alpha1[k & 3] = o.alpha;
      S->beta1[k & 3] = o.beta;
      if (k >= 2) S->diff = diff;
      S->w_pend = ph ? k : 0;
      S->w_pend_n = ph;
    }
  }
  if (leader) S->halo_k = k + 1;  // the next exchange fills sweep k+1's inputs
  return true;
}

// VEC columns from c0 (c0 - 1 even, so every 2-column chunk is 2-element aligned); chunks are
// clamped to start <= cmax (cmax - 1 even, cmax + 1 inside the padded row).
// Addresses: the row pointer is wave-uniform and every column index is >= -2, so row - 2 plus an
// UNSIGNED 32-bit byte offset lets the compiler use the SGPR-base form (global_load v, voff, s[base])
// instead of a 64-bit VGPR address per access (two VALU adds each).
template <typename T>
__device__ __forceinline__ const T* col_ptr(const T* row, int c) {
  return reinterpret_cast<const T*>(reinterpret_cast<const char*>(row - 2) + unsigned(c + 2) * unsigned(sizeof(T)));
}
template <typename T>
__device__ __forceinline__ T* col_ptr(T* row, int c) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(row - 2) + unsigned(c + 2) * unsigned(sizeof(T)));
}

template <typename T, int VEC>
__device__ __forceinline__ void load_cols(const T* row, int c0, int cmax, T (&out)[VEC]) {
#pragma unroll
  for (int q = 0; q < VEC / 2; ++q) {
    T v[2];
    vload_raw<T, 2>(col_ptr(row, min(c0 + 2 * q, cmax)), v);
    out[2 * q] = v[0];
    out[2 * q + 1] = v[1];
  }
}

// Field stores carry the non-temporal hint (global_store ... nt): nothing re-reads them in this
// sweep, and fewer dirty lines sit in the XCD L2s when the sweep ends (the kernel-end writeback is
// part of every kernel boundary).  Fresh-process A/B, 4 rounds: 16384^2 fp64 1845.9 -> 1796.3 us
// (-2.7%, every nt run below every plain-store run), 2048x16384 263.4 -> 254.5 us
// (profiles/r3/nt_stores/).  Non-temporal LOADS lose (+10-22%: the L2 reuse of halo rows and
// overlapping columns matters, NOTES #60-61).
template <typename T, int VEC>
__device__ __forceinline__ void store_cols(T* row, int c0, const T (&in)[VEC], bool all,
                                           const bool (&own)[VEC]) {
  if (all) {
#pragma unroll
    for (int q = 0; q < VEC / 2; ++q) {
      typedef T V __attribute__((ext_vector_type(2)));
      const V v = {in[2 * q], in[2 * q + 1]};
      __builtin_nontemporal_store(v, reinterpret_cast<V*>(col_ptr(row, c0 + 2 * q)));
    }
  } else {
#pragma unroll
    for (int u = 0; u < VEC; ++u)
      if (own[u]) __builtin_nontemporal_store(in[u], col_ptr(row, c0 + u));
  }
}

// One row of the tile: its table row and wave-uniform coefficient class.  Only these 2 scalars
// travel down the 3-stage pipeline; the row's face constants (20 SGPRs) are re-read from the
// tables on the rare rows the ellipse cuts, which keeps 3 live rows from spilling SGPRs.  The
// per-column coefficients are rebuilt where they are used (class fast path, or the exact formula).
struct RowCo {
  int gi;
  int ucls;
};

__device__ __forceinline__ RowCo row_co(const DevTables& Tb, int gi, int gjlo, int gjhi) {
  return RowCo{gi, row_class(load_row(Tb, gi), gjlo, gjhi)};
}

// Column constants of a tile's lanes parked in LDS (lane-private slots [4 u + q][lane]) the first
// time the tile meets a row the ellipse cuts: the cut-row path then reads them with ds_reads
// instead of 4 vector loads per column and stage, whose waits (vmcnt is in-order) would also
// drain the row prefetch three times per row.
__device__ __forceinline__ ColConst col_lds(const double* scol, int u, int lane, int gj) {
  return ColConst{scol[(4 * u) * 64 + lane], scol[(4 * u + 1) * 64 + lane], scol[(4 * u + 2) * 64 + lane],
                  scol[(4 * u + 3) * 64 + lane], gj};
}

__device__ __forceinline__ void coef(const RowCo& c, const DevTables& Tb, const DevGeom& G, const double* scol,
                                     int u, int lane, int gj, double& a0, double& a1, double& b0, double& b1) {
  if (c.ucls != 0) {
    a0 = a1 = b0 = b1 = c.ucls == 1 ? 1.0 : G.inv_eps;
  } else {
    const RowConst rc = load_row(Tb, c.gi);
    const ColConst cc = col_lds(scol, u, lane, gj);
    a0 = face_a0c(cc, rc, G);
    a1 = face_a1c(cc, rc, G);
    b0 = face_b0c(cc, rc, G);
    b1 = face_b1c(cc, rc, G);
  }
}

// Stencil arithmetic in the sweep's compute type C.  C = double: the shared helpers of
// pcg_device.hpp, bit-identical to every other fp64 kernel.  C = float (fp32 storage with fp32
// arithmetic, GpuOptions::arith32): the same formulas in fp32 with the class coefficients, 1/h^2
// and 1/D rounded once to fp32 (ArithF, built per wave from DevGeom); cut faces are evaluated
// exactly in fp64 and rounded.  The 5 partial sums stay fp64 in both (products of two fp32 values
// are exact in fp64).  Half the registers of the fp64 pipeline and packed-fp32 friendly: the fp32
// sweep is issue-bound in fp64 arithmetic (profiles/r3/kernel_ab/pmc_fp32_16384.md).
struct ArithF {
  float cx, cy, dinv_in, dinv_out, inv_eps;
};

__device__ __forceinline__ double fma_c(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fma_c(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

template <typename C>
__device__ __forceinline__ void coef_c(const RowCo& c, const DevTables& Tb, const DevGeom& G, const ArithF& F,
                                       const double* scol, int u, int lane, int gj, C& a0, C& a1, C& b0, C& b1) {
  if constexpr (std::is_same_v<C, double>) {
    coef(c, Tb, G, scol, u, lane, gj, a0, a1, b0, b1);
  } else {
    if (c.ucls != 0) {
      a0 = a1 = b0 = b1 = c.ucls == 1 ? 1.0f : F.inv_eps;
    } else {
      double d0, d1, e0, e1;
      coef(c, Tb, G, scol, u, lane, gj, d0, d1, e0, e1);
      a0 = float(d0); a1 = float(d1); b0 = float(e0); b1 = float(e1);
    }
  }
}

template <typename C>
__device__ __forceinline__ C zdiv_c(int ucls, C r, C a0, C a1, C b0, C b1, const DevGeom& G, const ArithF& F) {
  if constexpr (std::is_same_v<C, double>) {
    return zdiv_u<false>(ucls, r, a0, a1, b0, b1, G);
  } else {
    if (ucls == 1) return r * F.dinv_in;
    if (ucls == 2) return r * F.dinv_out;
    const bool in = (a0 == 1.0f) & (a1 == 1.0f) & (b0 == 1.0f) & (b1 == 1.0f);
    const bool out = (a0 == F.inv_eps) & (a1 == F.inv_eps) & (b0 == F.inv_eps) & (b1 == F.inv_eps);
    if (in) return r * F.dinv_in;
    if (out) return r * F.dinv_out;
    return r / __builtin_fmaf(a1 + a0, F.cx, (b1 + b0) * F.cy);
  }
}

template <typename C>
__device__ __forceinline__ C apply_c(C pc, C pim, C pip, C pjm, C pjp, C a0, C a1, C b0, C b1, const DevGeom& G,
                                     const ArithF& F) {
  if constexpr (std::is_same_v<C, double>) {
    return apply_a<false>(pc, pim, pip, pjm, pjp, a0, a1, b0, b1, G);
  } else {
    const float x = __builtin_fmaf(a1, pc - pip, a0 * (pc - pim));
    const float y = __builtin_fmaf(b1, pc - pjp, b0 * (pc - pjm));
    return __builtin_fmaf(F.cx, x, F.cy * y);
  }
}

// A x on the VEC columns of a lane: centre xc, rows i-1 / i+1 xim / xip, the lane neighbours'
// edge columns left / right (DPP).  fp32 with VEC = 2: both columns in packed fp32 (v_pk_*), the
// same per-column fmaf sequence as apply_c (bit-identical results).
template <typename C, int VEC>
__device__ __forceinline__ void apply_row(const C (&xc)[VEC], const C (&xim)[VEC], const C (&xip)[VEC], C left,
                                          C right, const C (&a0)[VEC], const C (&a1)[VEC], const C (&b0)[VEC],
                                          const C (&b1)[VEC], const DevGeom& G, const ArithF& F, C (&out)[VEC]) {
  if constexpr (std::is_same_v<C, float> && VEC == 2) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 pc = {xc[0], xc[1]}, pim = {xim[0], xim[1]}, pip = {xip[0], xip[1]};
    const f2 pjm = {left, xc[0]}, pjp = {xc[1], right};
    const f2 A0 = {a0[0], a0[1]}, A1 = {a1[0], a1[1]}, B0 = {b0[0], b0[1]}, B1 = {b1[0], b1[1]};
    const f2 x = __builtin_elementwise_fma(A1, pc - pip, A0 * (pc - pim));
    const f2 y = __builtin_elementwise_fma(B1, pc - pjp, B0 * (pc - pjm));
    const f2 cx = {F.cx, F.cx}, cy = {F.cy, F.cy};
    const f2 r = __builtin_elementwise_fma(cx, x, cy * y);
    out[0] = r.x;
    out[1] = r.y;
  } else {
#pragma unroll
    for (int u = 0; u < VEC; ++u)
      out[u] = apply_c<C>(xc[u], xim[u], xip[u], u == 0 ? left : xc[u - 1], u == VEC - 1 ? right : xc[u + 1], a0[u],
                          a1[u], b0[u], b1[u], G, F);
  }
}

// f(integral_constant<int, 0>) && f(integral_constant<int, 1>) && ... (N calls at most, stops at
// the first false): a loop body whose step number is a compile-time constant
template <typename F, int... I>
__device__ __forceinline__ bool static_for_while_impl(F&& f, std::integer_sequence<int, I...>) {
  return (f(std::integral_constant<int, I>{}) && ...);
}
template <int N, typename F>
__device__ __forceinline__ bool static_for_while(F&& f) {
  return static_for_while_impl(f, std::make_integer_sequence<int, N>{});
}

// ---- LDS-DMA row prefetch (pcg1_march's DPF mode) ----
// global_load_lds_dwordx4: 16 B per lane from base + voff into LDS at lds + 16 * lane, no VGPR
// destination.  Inline asm on purpose: hipcc does not see the load, so it emits no wait for it --
// the march counts vmcnt itself (wait_vmcnt), exactly, stores included.  M0 (the LDS base) is
// saved and restored inside the statement (cdna_hip_programming.md: M0 is compiler-reserved).
__device__ __forceinline__ void dma16(const void* base, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(base), "s"(lds)
               : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <typename T, int VEC>
struct Pcg1Row {
  T r[VEC], p[VEC], w[VEC], q[VEC];  // q: p^{k-2} (WM 3 only)
};

// w schedule of one sweep (template WM of pcg1_march): 0 = w untouched; 1 = pairs, w += c1 p^{k-1}
// + alpha p^k; 2 = triples with p^{k-2} recovered, w += c2 (p^{k-1} - z^{k-2}) + c1 p^{k-1} +
// alpha p^k (c2 = alpha_{k-2} / beta_{k-1}); 3 = triples re-reading p^{k-2}, w += c2 p^{k-2} + ...
// (c2 = alpha_{k-2}).  See k_pcg1.


// FAST: an interior tile (full width, every marched row and column strictly inside the global
// domain, VEC = 2): no Dirichlet masks, and ownership is a fixed lane set (lanes 1..62 own both
// their columns, lanes 0 and 63 none), so the sums accumulate unmasked and are masked once at the
// end.  Same arithmetic as the general path, so a point's values never depend on its tile.
// The tile marches top-down, rows i0-2 .. i1+2.  (Bottom-up and alternating marches, super-row and
// banded dispatch orders were tried to make vertically adjacent tiles share their halo rows in L2:
// all slower, NOTES #30, #46-48.)
//
// DPF > 0 (FAST tiles of fp64 storage, VEC 2, WM 0-2, at least DPF rows): the rows are prefetched
// DPF ahead by LDS-DMA into a per-wave ring `dring` (DPF slots of r, p [, w] rows, 1 KiB each)
// instead of registers.  Why: with compiler-visible loads the march waits, every row, for the
// previous row's STORES -- the stores sit in a branch (owned rows only), so at the merge hipcc
// cannot count them and its vmcnt wait for the prefetched row covers them too: a full store round
// trip per row per wave (bench/probe/dma_march.hip, isa of k_reg).  Here hipcc sees no load at all
// and the march waits with exact counts: the loop is split into 3 steps without stores, DPF ramp
// steps and a steady loop whose every step stores, so each wait's number of younger operations
// (later DMAs and stores) is a compile-time constant.  Same arithmetic, bit-identical fields.
//
// LOCK (lockstep workgroups, k_pcg1 with several waves): the waves of a workgroup march side-by-side
// tiles of one tile row and meet at an s_barrier after every row step, so the workgroup reads and
// writes each row as ONE contiguous span of 8 x 1 KiB per field instead of as independent 1-KiB
// pieces at different times (bench/probe/dma_march.hip k_lock: 16384^2, 16 waves per CU, 1.846 ->
// 1.688 ms per sweep).  Pure pacing: no data passes between the waves, every wave of a workgroup
// marches the same number of rows (one tile row), and a wave that has left no longer counts.
template <typename T, typename C, int VEC, int PF, int WM, bool FAST, int DPF = 0, bool LOCK = false>
__device__ __forceinline__ void pcg1_march(const DevGeom& G, const DevTables& Tb, const ArithF& F, T* __restrict__ w,
                                           const T* __restrict__ rold, T* __restrict__ rnew,
                                           const T* __restrict__ pold,
                                           T* pnew, int i0, int i1, int j0, int j1,
                                           double alpha_d, double beta_d, double c1_d, double c2_d,
                                           double (&acc)[kNq], double* __restrict__ scol,
                                           unsigned long long cls, bool use_cls, double* dring = nullptr) {
  constexpr bool WUP = WM != 0;
  static_assert(DPF == 0 || (FAST && VEC == 2 && sizeof(T) == 8 && WM <= 2), "LDS-DMA march: fp64 FAST tiles, WM 0-2");
  constexpr bool PK = std::is_same_v<C, float> && VEC == 2;  // packed fp32 stencils (apply_row)
  const C alpha = C(alpha_d), beta = C(beta_d), c1 = C(c1_d), c2 = C(c2_d);
  const int64_t P = G.pitch;
  const int lane = threadIdx.x & 63;
  const int c0 = j0 - 2 + lane * VEC;
  const int cmax = G.ny + 1 + (G.ny & 1);  // last odd column <= ny + 2 (second ghost column)
  // Interior / Dirichlet is decided on GLOBAL indices: the ghost rows/columns of a decomposed
  // subdomain hold its neighbours' values (k_pcg1_halo), those on the domain boundary are 0.
  bool colin[VEC], own[VEC];
  int gj[VEC];
#pragma unroll
  for (int u = 0; u < VEC; ++u) {
    const int c = c0 + u, g = G.gj0 + c;
    colin[u] = g >= 1 && g <= G.N - 1;
    own[u] = c >= j0 && c <= j1;
    gj[u] = min(max(g, 0), G.N);
  }
  const bool own_all = own[0] && own[VEC - 1];
  bool own_any = false;
#pragma unroll
  for (int u = 0; u < VEC; ++u) own_any |= own[u];
  const int gjlo = max(G.gj0 + j0 - 2, 0), gjhi = min(G.gj0 + j0 - 2 + 64 * VEC - 1, G.N);
  auto grow = [&](int m) { return min(max(G.gi0 + m, 0), G.M); };  // table row of local row m
  // row m's class: from the slot's bits (Pcg1Slot) or from the tables
  auto row_of = [&](int m) {
    if (use_cls) return RowCo{grow(m), int((cls >> (2 * (m - i0 + 3))) & 3ull)};
    return row_co(Tb, grow(m), gjlo, gjhi);
  };
  auto interior_row = [&](int m) { return G.gi0 + m >= 1 && G.gi0 + m <= G.M - 1; };
  // coefficients of a row in stage B / C, rebuilt (class fast path or the exact face formulas)
  auto coef_at = [&](const RowCo& c, int m, int u, C& a0, C& a1, C& b0, C& b1) {
    (void)m;
    coef_c<C>(c, Tb, G, F, scol, u, lane, gj[u], a0, a1, b0, b1);
  };

  auto fetch = [&](int m, Pcg1Row<T, VEC>& b) {
    const int mc = min(max(m, -1), G.nx + 2);  // rows -1 .. nx+2 exist (2 ghost layers)
    load_cols<T, VEC>(rold + int64_t(mc) * P, c0, cmax, b.r);
    load_cols<T, VEC>(pold + int64_t(mc) * P, c0, cmax, b.p);
    if constexpr (WUP) {  // w of the row stage B handles next step
      const int wc = min(max(m - 1, -1), G.nx + 2);
      load_cols<T, VEC>(w + int64_t(wc) * P, c0, cmax, b.w);
      // p^{k-2} still sits in the buffer this sweep overwrites with p^k: the owner of a point
      // reads it here, before its own store of that row (rows it does not own are never used)
      if constexpr (WM == 3) load_cols<T, VEC>(pnew + int64_t(wc) * P, c0, cmax, b.q);
    }
  };

  // pipeline registers
  C Pm2[VEC], Pm1[VEC], Zm3[VEC], Zm2[VEC], ro1[VEC], po1[VEC], po2[VEC];
#pragma unroll
  for (int u = 0; u < VEC; ++u) Pm2[u] = Pm1[u] = Zm3[u] = Zm2[u] = ro1[u] = po1[u] = po2[u] = C(0);
  RowCo cB = row_of(i0 - 3);  // rows m-1, m-2
  RowCo cC = cB;
  bool parked = false;  // column constants in LDS (see col_lds)
  auto park_cols = [&]() {
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      const ColConst cc = load_col(Tb, gj[u]);
      scol[(4 * u) * 64 + lane] = cc.ylo;
      scol[(4 * u + 1) * 64 + lane] = cc.yhi;
      scol[(4 * u + 2) * 64 + lane] = cc.rh0;
      scol[(4 * u + 3) * 64 + lane] = cc.rh1;
    }
    parked = true;
  };
  if (cB.ucls == 0) park_cols();

  const int mfirst = i0 - 2, mlast = i1 + 2;
  // one row step of the 3-stage pipeline on row m's loaded values
  auto core = [&](int m, const Pcg1Row<T, VEC>& cur) {
    // ---- stage A: p^k of row m
    const bool rowA = FAST || interior_row(m);
    const RowCo cA = row_of(m);
    if (cA.ucls == 0 && !parked) park_cols();
    C Pm[VEC], rom[VEC], pom[VEC];
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      const bool in = FAST || (rowA && colin[u]);
      rom[u] = in ? C(cur.r[u]) : C(0);
      pom[u] = in ? C(cur.p[u]) : C(0);
      C a0, a1, b0, b1;
      coef_c<C>(cA, Tb, G, F, scol, u, lane, gj[u], a0, a1, b0, b1);
      const C z = zdiv_c<C>(cA.ucls, rom[u], a0, a1, b0, b1, G, F);
      const C v = fma_c(beta, pom[u], z);
      Pm[u] = in ? C(static_cast<T>(v)) : C(0);  // the stored (rounded) p^k is the one used
    }
    // ---- stage B: A p^k, r^k, z^k of row m-1 (j neighbours by DPP; edge lanes get 0, their
    // results only feed columns that are not owned).  Rows i-1 / i+1 of it: Pm2 / Pm.
    const int mb = m - 1;
    const bool rowB = FAST || interior_row(mb);
    const bool ownB = mb >= i0 && mb <= i1;
    C Zm1[VEC];
    T rs[VEC], ps[VEC], ws[VEC];
    {
      const C left = dpp_shift<kWaveShr1>(Pm1[VEC - 1], C(0));
      const C right = dpp_shift<kWaveShl1>(Pm1[0], C(0));
      C oleft = C(0), oright = C(0);
      if constexpr (WM == 2) {
        oleft = dpp_shift<kWaveShr1>(po1[VEC - 1], C(0));
        oright = dpp_shift<kWaveShl1>(po1[0], C(0));
      }
      // packed fp32: the row's coefficients first, then both columns' stencils in v_pk_* ops; fp64
      // keeps the per-column interleaving (fewer live registers)
      C a0[VEC], a1[VEC], b0[VEC], b1[VEC], Ap[VEC], Apo[VEC];
      if constexpr (PK) {
#pragma unroll
        for (int u = 0; u < VEC; ++u) coef_at(cB, mb, u, a0[u], a1[u], b0[u], b1[u]);
        apply_row<C, VEC>(Pm1, Pm2, Pm, left, right, a0, a1, b0, b1, G, F, Ap);
        // p^{k-2} recovery (WM 2): A p^{k-1}
        if constexpr (WM == 2)
          apply_row<C, VEC>(po1, po2, pom, oleft, oright, a0, a1, b0, b1, G, F, Apo);
      }
#pragma unroll
      for (int u = 0; u < VEC; ++u) {
        if constexpr (!PK) {
          coef_at(cB, mb, u, a0[u], a1[u], b0[u], b1[u]);
          Ap[u] = apply_c<C>(Pm1[u], Pm2[u], Pm[u], u == 0 ? left : Pm1[u - 1],
                             u == VEC - 1 ? right : Pm1[u + 1], a0[u], a1[u], b0[u], b1[u], G, F);
          if constexpr (WM == 2)
            Apo[u] = apply_c<C>(po1[u], po2[u], pom[u],
                                u == 0 ? oleft : po1[u - 1], u == VEC - 1 ? oright : po1[u + 1], a0[u], a1[u], b0[u],
                                b1[u], G, F);
        }
        const bool in = FAST || (rowB && colin[u]);
        const C rn = C(static_cast<T>(fma_c(-alpha, Ap[u], ro1[u])));  // = upd_r<false>
        rs[u] = static_cast<T>(in ? rn : C(0));
        const C zn = zdiv_c<C>(cB.ucls, rn, a0[u], a1[u], b0[u], b1[u], G, F);
        Zm1[u] = in ? zn : C(0);
        ps[u] = static_cast<T>(Pm1[u]);
        if constexpr (WM == 1) {
          ws[u] = static_cast<T>(fma_c(alpha, Pm1[u], fma_c(c1, po1[u], C(cur.w[u]))));
        } else if constexpr (WM == 2) {
          // r^{k-2} = r^{k-1} + alpha_{k-1} A p^{k-1};  p^{k-2} = (p^{k-1} - D^-1 r^{k-2}) / beta_{k-1}
          const C zo = zdiv_c<C>(cB.ucls, fma_c(c1, Apo[u], ro1[u]), a0[u], a1[u], b0[u], b1[u], G, F);
          const C t = fma_c(c2, po1[u] - zo, C(cur.w[u]));
          ws[u] = static_cast<T>(fma_c(alpha, Pm1[u], fma_c(c1, po1[u], t)));
        } else if constexpr (WM == 3) {
          const C t = fma_c(c2, C(cur.q[u]), C(cur.w[u]));
          ws[u] = static_cast<T>(fma_c(alpha, Pm1[u], fma_c(c1, po1[u], t)));
        }
        if (ownB && (FAST || own[u])) {
          acc[0] += double(Zm1[u]) * double(rn);
          acc[3] += double(Ap[u]) * double(Pm1[u]);
          acc[4] += double(Pm1[u]) * double(Pm1[u]);
        }
      }
    }
    if (ownB && (FAST ? own_all : own_any)) {
      const int64_t o = int64_t(mb) * P;
      store_cols<T, VEC>(rnew + o, c0, rs, FAST || own_all, own);
      store_cols<T, VEC>(pnew + o, c0, ps, FAST || own_all, own);
      if constexpr (WUP) store_cols<T, VEC>(w + o, c0, ws, FAST || own_all, own);
    }
    // ---- stage C: A z^k of row m-2
    const int mcr = m - 2;
    if (mcr >= i0 && mcr <= i1) {
      const C left = dpp_shift<kWaveShr1>(Zm2[VEC - 1], C(0));
      const C right = dpp_shift<kWaveShl1>(Zm2[0], C(0));
      C a0[VEC], a1[VEC], b0[VEC], b1[VEC], Az[VEC];
      if constexpr (PK) {
#pragma unroll
        for (int u = 0; u < VEC; ++u) coef_at(cC, mcr, u, a0[u], a1[u], b0[u], b1[u]);
        apply_row<C, VEC>(Zm2, Zm3, Zm1, left, right, a0, a1, b0, b1, G, F, Az);
      }
#pragma unroll
      for (int u = 0; u < VEC; ++u) {
        if constexpr (!PK) {
          coef_at(cC, mcr, u, a0[u], a1[u], b0[u], b1[u]);
          Az[u] = apply_c<C>(Zm2[u], Zm3[u], Zm1[u], u == 0 ? left : Zm2[u - 1],
                             u == VEC - 1 ? right : Zm2[u + 1], a0[u], a1[u], b0[u], b1[u], G, F);
        }
        if (FAST || own[u]) {
          acc[1] += double(Az[u]) * double(Zm2[u]);
          acc[2] += double(Az[u]) * double(Pm2[u]);
        }
      }
    }
    // ---- shift the pipeline
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      Pm2[u] = Pm1[u]; Pm1[u] = Pm[u];
      Zm3[u] = Zm2[u]; Zm2[u] = Zm1[u];
      ro1[u] = rom[u];
      if constexpr (WM == 2) po2[u] = po1[u];
      po1[u] = pom[u];
    }
    cC = cB;
    cB = cA;
  };

  if constexpr (DPF > 0) {
    // ---- LDS-DMA ring (see the template comment).  Row mfirst + t sits in slot t % DPF.
    constexpr int ND = WUP ? 3 : 2;  // DMAs per row: r, p (, w of the row above)
    constexpr int NS = WUP ? 3 : 2;  // stores per storing step: r, p (, w)
    const unsigned voff = unsigned(c0 + 2) * 8u;  // bytes from row - 2 (col_ptr's unsigned form)
    const unsigned lds0 = unsigned(reinterpret_cast<uintptr_t>(dring));
    auto dma_row = [&](int m, int slot) {
      const unsigned l = lds0 + unsigned(slot) * (ND * 1024u);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's previous ds_reads have returned
      dma16(rold + int64_t(m) * P - 2, voff, l);
      dma16(pold + int64_t(m) * P - 2, voff, l + 1024u);
      if constexpr (WUP) dma16(w + int64_t(m - 1) * P - 2, voff, l + 2048u);
    };
    typedef double d2 __attribute__((ext_vector_type(2)));
    const int h = i1 - i0 + 1;  // rows stored: steps t = 3 .. h + 2 (the caller guarantees h >= DPF)
    int slot = 0;
    // step t: wait for its row (younger: the later rows' DMAs and KS steps' stores), read it from
    // the ring, refill the slot DPF rows ahead (the last row again past the end: a cache hit), run
    // the pipeline
    auto dstep = [&](int t, auto ks) {
      constexpr int KS = decltype(ks)::value;
      wait_vmcnt<(DPF - 1) * ND + KS * NS>();
      const double* sl = dring + slot * (ND * 128);
      Pcg1Row<T, VEC> cur;
      const d2 rv = *reinterpret_cast<const d2*>(sl + 2 * lane);
      const d2 pv = *reinterpret_cast<const d2*>(sl + 128 + 2 * lane);
      cur.r[0] = rv.x; cur.r[1] = rv.y;
      cur.p[0] = pv.x; cur.p[1] = pv.y;
      if constexpr (WUP) {
        const d2 wv = *reinterpret_cast<const d2*>(sl + 256 + 2 * lane);
        cur.w[0] = wv.x; cur.w[1] = wv.y;
      }
      dma_row(min(mfirst + t + DPF, mlast), slot);
      slot = slot + 1 == DPF ? 0 : slot + 1;
      core(mfirst + t, cur);
    };
#pragma unroll
    for (int q = 0; q < DPF; ++q) dma_row(mfirst + q, q);
    using K0 = std::integral_constant<int, 0>;
    dstep(0, K0{});
    dstep(1, K0{});
    dstep(2, K0{});
    // ramp: step 3 + K has the stores of K steps behind its row's DMA
    static_for_while<DPF>([&](auto k) {
      dstep(3 + decltype(k)::value, k);
      return true;
    });
    for (int t = 3 + DPF; t <= h + 3; ++t) dstep(t, std::integral_constant<int, DPF>{});
    wait_vmcnt<0>();  // no DMA may land after the wave has moved on (its LDS is the next tile's)
  } else {
    // ring of PF + 1 row buffers, unrolled by its size so no buffer is ever copied: step m reads
    // slot q and refills the slot step m - 1 consumed
    Pcg1Row<T, VEC> buf[PF + 1];
#pragma unroll
    for (int q = 0; q < PF; ++q) fetch(min(mfirst + q, mlast), buf[q]);
    bool more = true;
    for (int m = mfirst; more && m <= mlast; m += PF + 1) {
#pragma unroll
      for (int q = 0; q <= PF; ++q) {
        if (m + q > mlast) {
          more = false;
          break;
        }
        // PF rows ahead, unconditional (a branch around loads forces vmcnt(0)); past the tile's
        // last row re-read that row (a cache hit) instead of the next tile's rows
        fetch(min(m + q + PF, mlast), buf[(q + PF) % (PF + 1)]);
        core(m + q, buf[q]);
        if constexpr (LOCK) __builtin_amdgcn_s_barrier();
      }
    }
  }
  if constexpr (FAST) {  // lanes 0 and 63 own no column
#pragma unroll
    for (int q = 0; q < kNq; ++q) acc[q] = own_all ? acc[q] : 0.0;
  }
}

}  // namespace
}  // namespace pmx
