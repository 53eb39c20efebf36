// Fused PCG kernels, wave-tile variant ("dpp" kernel family) for CDNA4.
//
// Same dataflow and scalar protocol as pcg_kernels.hip (k_pcg_a / k_pcg_b), different mapping:
//  * one wave64 owns a tile of `rows` x (64*VEC) nodes and marches it alone: no LDS ring and no
//    workgroup barrier inside the march (waves of a workgroup are independent tiles);
//  * every lane holds VEC adjacent columns (VEC*sizeof(T) = 16 B vector loads/stores in fp64);
//  * the j-neighbours of a row come from the lanes on either side through DPP `wave_shr:1` /
//    `wave_shl:1` moves (a VALU op, no LDS traffic); the two columns just outside the tile enter
//    through the DPP `old` operand (lane 0 / lane 63 keep it when their source lane is missing);
//  * the halo columns of p^k (k_pcg_a) are computed once per tile, one row per lane, and
//    broadcast per row with v_readlane;
//  * rows are software-pipelined one row ahead (all loads of row i+1 issue before row i is used).
#include <cmath>
#include <type_traits>

#include "pcg_device.hpp"
#include "pmx/common.hpp"
#include "pmx/kernels.hpp"
#include "pmx/spec.hpp"

namespace pmx {

using namespace dev;

namespace {

constexpr int kMaxWaveRows = 256;


struct WaveTile {
  int i0, iend, j0, jend, id;
  bool live;
};

__device__ __forceinline__ WaveTile wave_tile(int waves, int tiles_j, int ntiles, int TI, int W,
                                              const DevGeom& G, int abl) {
  WaveTile t;
  // readfirstlane makes the wave index provably wave-uniform: without it the compiler treats the
  // whole march as a divergent loop (row tables become per-lane vector loads, loop-carried
  // values get copied through VGPRs every row)
  t.id = ((abl & kAblNoXcd) ? int(blockIdx.x) : xcd_remap(blockIdx.x, gridDim.x)) * waves +
         __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  t.live = t.id < ntiles;
  const int ti = t.id / tiles_j, tj = t.id - ti * tiles_j;
  t.i0 = 1 + ti * TI;
  t.iend = min(t.i0 + TI - 1, G.nx);
  t.j0 = 1 + tj * W;
  t.jend = min(t.j0 + W - 1, G.ny);
  return t;
}

// The PCG scalar prologue of k_pcg_a (stop test of iteration k-1 and beta); identical protocol to
// pcg_kernels.hip.  Returns false when the iteration must not run.
__device__ __forceinline__ bool prologue_a(PcgState* S, long long& k, bool& first, double& beta) {
  if (S->done) return false;
  k = S->it;
  first = (k == 1);
  const double zr_prev = S->red_b[1];
  beta = 0.0;
  if (!first) {
    const double diff = sqrt(S->red_b[0]);
    const bool bad = !(diff == diff) || !(zr_prev == zr_prev);
    if (bad || diff < S->delta || k > S->max_iter) {
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        S->diff = diff;
        S->iters = k - 1;
        S->status = bad ? int(Status::kBreakdown)
                        : (diff < S->delta ? int(Status::kConverged) : int(Status::kMaxIter));
        if (bad) S->nan_flag = 1;
        S->done = 1;
      }
      return false;
    }
    beta = zr_prev / S->zr[k & 1];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S->zr[(k - 1) & 1] = zr_prev;
    if (!first) S->diff = sqrt(S->red_b[0]);
  }
  return true;
}

}  // namespace

// ---------------------------------------------------------------------------
// k_pcg_a (wave-tile): p^k = D^-1 r + beta p^{k-1};  partial (A p^k, p^k)
//
// Memory-pipeline rules (each one fixed a measured stall, see profiles/):
//  * every global load is unconditional and branch-free (addresses clamped, results masked where
//    used): a load inside a divergent branch forces an `s_waitcnt vmcnt(0)` at the join;
//  * prefetched registers are never copied: the row loop is unrolled by the ring size and every
//    ring slot is a compile-time index, because copying a register with an outstanding load makes
//    the wave wait for that load, which serialised the whole march (vmcnt(0) every row).
// ---------------------------------------------------------------------------
// Column constants of a wave tile, parked in LDS: the face ends / clip roots of each lane's
// columns are read only on rows cut by the ellipse, so holding them in VGPRs (9 per column) cost
// occupancy on every row.  Lane-private slots (no barrier); LDS reads count on lgkmcnt and never
// wait for the row prefetch (vmcnt).
template <int VEC>
struct ColLds {
  // slot u*64 + l: lane l's column u (lane-contiguous: conflict-free); 64*VEC + l: lane l's halo column
  double ylo[64 * VEC + 64], yhi[64 * VEC + 64], rh0[64 * VEC + 64], rh1[64 * VEC + 64];
  __device__ void put(int slot, const ColConst& c) {
    ylo[slot] = c.ylo; yhi[slot] = c.yhi; rh0[slot] = c.rh0; rh1[slot] = c.rh1;
  }
  __device__ ColConst get(int slot, int gj) const {
    return ColConst{ylo[slot], yhi[slot], rh0[slot], rh1[slot], gj};
  }
};

template <typename T, int VEC>
struct RowA {
  T rv[VEC], po[VEC];  // r and p^{k-1} of the lane's columns (storage precision)
  T hrv, hpo;          // the same for this lane's halo column
};

template <typename T, int VEC, int WAVES, bool EXACT>
__global__ void __launch_bounds__(64 * WAVES, (VEC == 4 && WAVES == 4 && !EXACT) ? 3 : 1)
k_pcg_a_wave(DevGeom G, DevTables Tb, const T* __restrict__ r, T* p0, T* p1, HaloBufs<T> H,
             double* __restrict__ partials, PcgState* S, int TI, int tiles_j, int ntiles, int abl) {
  constexpr int W = 64 * VEC;
  __shared__ ColLds<VEC> col_lds[WAVES];
  long long k;
  bool first;
  double beta;
  if (!prologue_a(S, k, first, beta)) return;
  const WaveTile t = wave_tile(WAVES, tiles_j, ntiles, TI, W, G, abl);
  if (!t.live) return;
  T* pnew = (k & 1) ? p1 : p0;
  const T* pold = (k & 1) ? p0 : p1;
  const int64_t P = G.pitch;
  const int lane = threadIdx.x & 63;

  const int jl = t.j0 + lane * VEC;
  // clamp for loads: the largest column start with jl's alignment whose VEC columns stay inside
  // the row (the field pitch is padded by >= VEC columns)
  const int jlc = min(jl, 1 + ((G.ny - 1) / VEC) * VEC);
  ColLds<VEC>& L = col_lds[threadIdx.x >> 6];
  bool valid[VEC];
  int gjc[VEC];
#pragma unroll
  for (int u = 0; u < VEC; ++u) {
    valid[u] = jl + u <= t.jend;
    gjc[u] = G.gj0 + min(jl + u, t.jend);
    L.put(u * 64 + lane, load_col(Tb, gjc[u]));
  }
  const bool lane_full = valid[VEC - 1];
  // halo column of this lane: j0-1 for even lanes, jend+1 for odd lanes (computed every row by
  // all lanes, broadcast with v_readlane; the neighbouring tile loads those lines too -> L2 hits)
  const int jh = (lane & 1) ? t.jend + 1 : t.j0 - 1;
  const int gjh = G.gj0 + jh;
  const bool h_dir = gjh <= 0 || gjh >= G.N || (abl & (kAblHalo | kAblHaloLoads));
  const int gjh_c = h_dir ? G.gj0 + t.j0 : gjh;
  L.put(W + lane, load_col(Tb, gjh_c));
  const bool h_store = lane < 2 && ((jh == 0 && (G.nb & kNbYlo)) || (jh == G.ny + 1 && (G.nb & kNbYhi)));
  const int ilast = t.iend + 1;

  // branch-free row fetch (addresses always valid; rows outside [0, nx+1] never requested)
  auto fetch = [&](int i, RowA<T, VEC>& b) {
    const int ic = min(i, G.nx + 1);
    const T* rrow = (ic == 0) ? (H.recv[0] - 1) : (ic == G.nx + 1) ? (H.recv[1] - 1) : (r + int64_t(ic) * P);
    if (!(G.nb & kNbXlo) && ic == 0) rrow = r + P;           // Dirichlet ghost row: any valid row
    if (!(G.nb & kNbXhi) && ic == G.nx + 1) rrow = r + P;
    vload_raw<T, VEC>(rrow + jlc, b.rv);
    vload_raw<T, VEC>(pold + int64_t(ic) * P + jlc, b.po);
    const int ih = min(max(ic, 1), G.nx);
    const T* hp = (jh == 0 && (G.nb & kNbYlo)) ? (H.recv[2] + ih - 1)
                : (jh == G.ny + 1 && (G.nb & kNbYhi)) ? (H.recv[3] + ih - 1)
                : (r + int64_t(ih) * P + min(max(jh, 1), G.ny));
    b.hrv = *hp;
    b.hpo = pold[int64_t(ih) * P + min(max(jh, 0), G.ny + 1)];
  };

  // Row history for A p.  EXACT keeps the reference formula, so it carries rows i-1 and i-2 of
  // p and row i-1's four coefficients.  The fast path starts A p of row i as soon as p^k of row i
  // exists (every term except the one with row i+1) and finishes it one row later with
  // a1(i) = a0(i+1): it carries one partial per column instead of five rows of history, which
  // keeps the VEC=4 kernel's VGPRs inside one wave's budget.
  constexpr int NH = EXACT ? VEC : 1;
  double pm1[VEC], part[VEC], pm2[NH], qa0[NH], qa1[NH], qb0[NH], qb1[NH];
#pragma unroll
  for (int u = 0; u < VEC; ++u) pm1[u] = part[u] = 0.0;
#pragma unroll
  for (int u = 0; u < NH; ++u) pm2[u] = qa0[u] = qa1[u] = qb0[u] = qb1[u] = 0.0;
  double hl_m1 = 0.0, hr_m1 = 0.0;  // halo values of row i-1 (EXACT path)
  double acc = 0.0;
  RowA<T, VEC> buf[2];
  fetch(t.i0 - 1, buf[0]);
  RowConst rc = load_row(Tb, G.gi0 + t.i0 - 1);

  auto step = [&](int i, const RowA<T, VEC>& cur, RowA<T, VEC>& nxt) {
    fetch(min(i + 1, ilast), nxt);  // unconditional: a branch around loads forces vmcnt(0)
    const RowConst rc_n = load_row(Tb, G.gi0 + min(i + 1, ilast));
    const int gi = G.gi0 + i;
    const bool own_row = i >= t.i0 && i <= t.iend;
    const bool live_row = gi > 0 && gi < G.M;
    const int ucls = (EXACT || (abl & kAblCoef)) ? 0 : row_class(rc, G.gj0 + t.j0 - 1, G.gj0 + t.jend + 1);
    const double uval = ucls == 1 ? 1.0 : G.inv_eps;
    // halo column values of this row
    double hv = 0.0;
    if (own_row && live_row) {
      double ha0 = uval, ha1 = uval, hb0 = uval, hb1 = uval;
      if (ucls == 0) {
        const ColConst ch = L.get(W + lane, gjh_c);
        ha0 = face_a0c(ch, rc, G); ha1 = face_a1c(ch, rc, G);
        hb0 = face_b0c(ch, rc, G); hb1 = face_b1c(ch, rc, G);
      }
      const double z = zdiv_u<EXACT>(ucls, double(cur.hrv), ha0, ha1, hb0, hb1, G);
      hv = first ? z : z + beta * double(cur.hpo);
      if (h_dir) hv = 0.0;
      if (h_store && !h_dir) pnew[int64_t(i) * P + jh] = static_cast<T>(hv);
      hv = double(static_cast<T>(hv));
    }
    const double hl_i = readlane_t(hv, 0);
    const double hr_i = readlane_t(hv, 1);
    double a0[VEC], a1[VEC], b0[VEC], b1[VEC], pc[VEC];
    T st[VEC];
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      if (abl & kAblCoef) {
        a0[u] = a1[u] = b0[u] = b1[u] = 1.0;
      } else if (ucls != 0) {
        a0[u] = a1[u] = b0[u] = b1[u] = uval;
      } else {
        const ColConst c = L.get(u * 64 + lane, gjc[u]);
        a0[u] = face_a0c(c, rc, G);
        a1[u] = face_a1c(c, rc, G);
        b0[u] = face_b0c(c, rc, G);
        b1[u] = face_b1c(c, rc, G);
      }
      double v = 0.0;
      if (valid[u] && live_row) {
        const double z = zdiv_u<EXACT>(ucls, double(cur.rv[u]), a0[u], a1[u], b0[u], b1[u], G);
        v = first ? z : z + beta * double(cur.po[u]);
      }
      st[u] = static_cast<T>(v);
      v = double(st[u]);
      // the column right after the tile's last one carries the right halo value, so the DPP
      // shift below hands it to column jend for partial tiles too
      if (jl + u == t.jend + 1) v = hr_i;
      pc[u] = v;
    }
    if (!(abl & kAblStore) &&
        live_row && (own_row || (i == 0 && (G.nb & kNbXlo)) || (i == G.nx + 1 && (G.nb & kNbXhi)))) {
      if (lane_full) {
        vstore<T, VEC>(pnew + int64_t(i) * P + jl, st);
      } else {
#pragma unroll
        for (int u = 0; u < VEC; ++u)
          if (valid[u]) pnew[int64_t(i) * P + jl + u] = st[u];
      }
    }
    if constexpr (EXACT) {
      // A p^k for row i-1 (pm1), neighbours: rows i-2 (pm2), i (pc); columns by DPP
      if (i - 1 >= t.i0 && !(abl & kAblAp)) {
        const double left = dpp_shift_f64<kWaveShr1>(pm1[VEC - 1], hl_m1);
        const double right = dpp_shift_f64<kWaveShl1>(pm1[0], hr_m1);
#pragma unroll
        for (int u = 0; u < VEC; ++u) {
          const double pjm = u == 0 ? left : pm1[u - 1];
          const double pjp = u == VEC - 1 ? right : pm1[u + 1];
          if (valid[u])
            acc += apply_a<true>(pm1[u], pm2[u], pc[u], pjm, pjp, qa0[u], qa1[u], qb0[u], qb1[u], G) * pm1[u];
        }
      }
#pragma unroll
      for (int u = 0; u < NH; ++u) {
        pm2[u] = pm1[u];
        qa0[u] = a0[u]; qa1[u] = a1[u]; qb0[u] = b0[u]; qb1[u] = b1[u];
      }
      hl_m1 = hl_i; hr_m1 = hr_i;
    } else if (!(abl & kAblAp)) {
      // finish row i-1: + cx a1(i-1) (p(i-1) - p(i)), with a1(i-1) = a0(i)
      if (i - 1 >= t.i0) {
#pragma unroll
        for (int u = 0; u < VEC; ++u)
          if (valid[u]) acc += __builtin_fma(G.cx * a0[u], pm1[u] - pc[u], part[u]) * pm1[u];
      }
      // start row i: every term but the one with row i+1
      if (own_row) {
        const double left = dpp_shift_f64<kWaveShr1>(pc[VEC - 1], hl_i);
        const double right = dpp_shift_f64<kWaveShl1>(pc[0], hr_i);
#pragma unroll
        for (int u = 0; u < VEC; ++u) {
          const double pjm = u == 0 ? left : pc[u - 1];
          const double pjp = u == VEC - 1 ? right : pc[u + 1];
          const double y = __builtin_fma(b1[u], pc[u] - pjp, b0[u] * (pc[u] - pjm));
          part[u] = __builtin_fma(G.cx * a0[u], pc[u] - pm1[u], G.cy * y);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < VEC; ++u) pm1[u] = pc[u];
    rc = rc_n;
  };
  // unrolled by the ring size: buf[0]/buf[1] are never copied
  for (int i = t.i0 - 1; i <= ilast; i += 2) {
    step(i, buf[0], buf[1]);
    if (i + 1 > ilast) break;
    step(i + 1, buf[1], buf[0]);
  }
  acc = wave_sum(acc);
  if (lane == 0) partials[t.id] = acc;
}

// ---------------------------------------------------------------------------
// k_pcg_b (wave-tile): alpha, A p^k, w/r update, sum dw^2, (z, r), halo pack
// Ring of 4 p rows (i-1, i, i+1 in use, i+2 in flight) and 2 w/r rows; the loop is unrolled by 4
// so every ring slot is a compile-time register set (see k_pcg_a_wave).
// ---------------------------------------------------------------------------
template <typename T, int VEC, int WAVES, bool EXACT>
__global__ void __launch_bounds__(64 * WAVES)
k_pcg_b_wave(DevGeom G, DevTables Tb, T* __restrict__ w, T* __restrict__ r, const T* p0,
             const T* p1, HaloBufs<T> H, double* __restrict__ partials, PcgState* S, int TI,
             int tiles_j, int ntiles, int abl) {
  constexpr int W = 64 * VEC;
  if (S->done) return;
  const long long k = S->it;
  const double denom = S->red_a[0];
  const bool bd = S->norm == int(Norm::kWeighted) ? fabs(denom) < S->bd_tol : denom < S->bd_tol;
  if (bd || !(denom == denom)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      S->iters = k;
      S->status = int(Status::kBreakdown);
      if (!(denom == denom)) S->nan_flag = 1;
      S->done = 1;
    }
    return;
  }
  const double alpha = S->zr[(k - 1) & 1] / denom;
  const WaveTile t = wave_tile(WAVES, tiles_j, ntiles, TI, W, G, abl);
  if (!t.live) return;
  const T* __restrict__ pn = (k & 1) ? p1 : p0;
  const int64_t P = G.pitch;
  const int lane = threadIdx.x & 63;
  const int jl = t.j0 + lane * VEC;
  bool valid[VEC];
  ColConst cc[VEC];
#pragma unroll
  for (int u = 0; u < VEC; ++u) {
    valid[u] = jl + u <= t.jend;
    cc[u] = load_col(Tb, G.gj0 + min(jl + u, t.jend));
  }
  const bool lane_any = valid[0];
  const bool lane_full = valid[VEC - 1];
  // p columns exist up to ny+1 (ghost); w/r loads stay within the interior.  The pitch is padded
  // by >= VEC columns, so a VEC-wide load starting at <= ny+1 stays inside the row.
  const int jlp = min(jl, 1 + (G.ny / VEC) * VEC);
  const int jlw = min(jl, 1 + ((G.ny - 1) / VEC) * VEC);
  const int jr = t.jend + 1;
  const bool edges = !(abl & (kAblHalo | kAblHaloLoads));

  T pr[4][VEC];             // p rows ring (storage precision)
  T wr[2][VEC], rr[2][VEC];
  T er[2][2];               // [slot][left/right edge]
  auto load_p = [&](int i, T (&out)[VEC]) { vload_raw<T, VEC>(pn + int64_t(i) * P + jlp, out); };
  auto load_wr = [&](int i, T (&wo)[VEC], T (&ro)[VEC], T (&e)[2]) {
    vload_raw<T, VEC>(w + int64_t(i) * P + jlw, wo);
    vload_raw<T, VEC>(r + int64_t(i) * P + jlw, ro);
    e[0] = pn[int64_t(i) * P + t.j0 - 1];
    e[1] = pn[int64_t(i) * P + jr];
  };
  load_p(t.i0 - 1, pr[3]);
  load_p(t.i0, pr[0]);
  load_p(t.i0 + 1, pr[1]);
  load_wr(t.i0, wr[0], rr[0], er[0]);
  RowConst rc = load_row(Tb, G.gi0 + t.i0);
  double acur[VEC];
#pragma unroll
  for (int u = 0; u < VEC; ++u) acur[u] = face_a0c(cc[u], rc, G);
  double dacc = 0.0, zacc = 0.0;

  // S = slot of row i in the p ring; row i's w/r live in slot S & 1
  auto step = [&](auto SC, int i) {
    constexpr int S0 = decltype(SC)::value;
    constexpr int SM = (S0 + 3) & 3, SP = (S0 + 1) & 3, SN = (S0 + 2) & 3, WC = S0 & 1, WN = WC ^ 1;
    const bool more = i < t.iend;
    // unconditional (rows clamped at the tile end): a branch around loads forces vmcnt(0)
    load_p(min(i + 2, t.iend + 1), pr[SN]);
    load_wr(min(i + 1, t.iend), wr[WN], rr[WN], er[WN]);
    const RowConst rc_n = load_row(Tb, G.gi0 + (more ? i + 1 : i));
    const int ucls = (EXACT || (abl & kAblCoef)) ? 0 : row_class(rc, G.gj0 + t.j0, G.gj0 + t.jend);
    const double uval = ucls == 1 ? 1.0 : G.inv_eps;
    const double left = double(dpp_shift<kWaveShr1>(pr[S0][VEC - 1], edges ? er[WC][0] : T(0)));
    const double right = double(dpp_shift<kWaveShl1>(pr[S0][0], edges ? er[WC][1] : T(0)));
    T ws[VEC], rs[VEC];
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      const double pjm = u == 0 ? left : double(pr[S0][u - 1]);
      const double pjp = u == VEC - 1 ? right : double(pr[S0][u + 1]);
      double a0, a1, b0, b1;
      if (abl & kAblCoef) {
        a0 = a1 = b0 = b1 = 1.0;
      } else if (ucls != 0) {
        a0 = a1 = b0 = b1 = uval;
      } else {
        a0 = acur[u];
        a1 = face_a1c(cc[u], rc, G);
        b0 = face_b0c(cc[u], rc, G);
        b1 = face_b1c(cc[u], rc, G);
      }
      const double pc = double(pr[S0][u]);
      const double Ap = apply_a<EXACT>(pc, double(pr[SM][u]), double(pr[SP][u]), pjm, pjp, a0, a1, b0,
                                       b1, G);
      const double wo = double(wr[WC][u]), ro = double(rr[WC][u]);
      ws[u] = static_cast<T>(upd_w<EXACT>(wo, alpha, pc));
      rs[u] = static_cast<T>(upd_r<EXACT>(ro, alpha, Ap));
      if (valid[u]) {
        const double dw = double(ws[u]) - wo;
        dacc += dw * dw;
        const double rq = double(rs[u]);
        const double z = zdiv_u<EXACT>(ucls, rq, a0, a1, b0, b1, G);
        zacc += z * rq;
      }
      acur[u] = a1;
    }
    const int64_t c = int64_t(i) * P + jl;
    if (abl & kAblStore) {
    } else if (lane_full) {
      vstore<T, VEC>(w + c, ws);
      vstore<T, VEC>(r + c, rs);
    } else {
#pragma unroll
      for (int u = 0; u < VEC; ++u)
        if (valid[u]) { w[c + u] = ws[u]; r[c + u] = rs[u]; }
    }
    if (lane_any) {
      if (i == 1 && (G.nb & kNbXlo)) {
#pragma unroll
        for (int u = 0; u < VEC; ++u) if (valid[u]) H.send[0][jl + u - 1] = rs[u];
      }
      if (i == G.nx && (G.nb & kNbXhi)) {
#pragma unroll
        for (int u = 0; u < VEC; ++u) if (valid[u]) H.send[1][jl + u - 1] = rs[u];
      }
      if (jl == 1 && (G.nb & kNbYlo)) H.send[2][i - 1] = rs[0];
#pragma unroll
      for (int u = 0; u < VEC; ++u)
        if (jl + u == G.ny && (G.nb & kNbYhi)) H.send[3][i - 1] = rs[u];
    }
    rc = rc_n;
  };
  for (int i = t.i0; i <= t.iend; i += 4) {
    step(std::integral_constant<int, 0>{}, i);
    if (i + 1 > t.iend) break;
    step(std::integral_constant<int, 1>{}, i + 1);
    if (i + 2 > t.iend) break;
    step(std::integral_constant<int, 2>{}, i + 2);
    if (i + 3 > t.iend) break;
    step(std::integral_constant<int, 3>{}, i + 3);
  }
  wave_sum2_mfma(dacc, zacc);
  if (lane == 0) {
    partials[2 * t.id] = dacc;
    partials[2 * t.id + 1] = zacc;
  }
}

// ---------------------------------------------------------------------------
// k_pcg_b_rows (TileCfg kind 2, the default pcg_b): the same update without a register ring:
// every row loads its three p rows (two of them L1/L2 hits: the neighbouring 2-row tiles of the
// band run at the same time on the same XCD), w and r, and computes; latency is hidden by
// occupancy (4 waves/SIMD) instead of software pipelining.  2-row tiles in XCD-banded row-major
// order keep the concurrent DRAM footprint to a narrow band of rows: 5.24 TB/s effective vs
// 5.04 for the ring kernel's 24-row marches (profiles/NOTES_perf_experiments.md #19).
//
// Paired w updates (fast mode).  w is not part of the CG recurrence (r is updated recursively),
// so its update can be deferred: an odd iteration k leaves alpha_k p^k pending (PcgState::w_pend)
// and does not touch w, the next (even) iteration applies both steps in one read-modify-write:
//   w^{k+1} = w^{k-1} + alpha_{k-1} p^{k-1} + alpha_k p^k.
// p^{k-1} is not re-read: k_pcg_a formed p^k = z^{k-1} + beta_k p^{k-1}, and this kernel already
// holds r^{k-1} (its input r), so p^{k-1} = (p^k - z^{k-1}) / beta_k and
//   w^{k+1} = w^{k-1} + c1 p^k - c2 z^{k-1},  c2 = alpha_{k-1} / beta_k,  c1 = alpha_k + c2.
// The recovery's rounding error is eps |p^k| / beta_k; for |beta_k| < S->pair_min_beta (1e-3) the
// kernel reads p^{k-1} from the other ping-pong buffer instead (still intact: k_pcg_a(k) only
// read it).  GpuOptions::pair_w = 0 launches the unpaired kernel (w updated every iteration).
// Traffic per iteration pair: 40 + 24 B/pt instead of 2 x 40 (the iteration is 64 -> 56 B/pt).
// ||w^{k+1} - w^k|| is computed as ||alpha_k p^k|| (the same quantity without the rounding of w).
// Readers of w materialise a pending step (GpuSubdomainSolver::download_w).
// ---------------------------------------------------------------------------
enum BwMode : int { kBwEvery = 0, kBwPend = 1, kBwRecover = 2, kBwLoad = 3 };

template <typename T, int VEC, bool EXACT, int MODE>
__device__ __forceinline__ void pcg_b_rows_march(const DevGeom& G, const DevTables& Tb, T* __restrict__ w,
                                                 T* __restrict__ r, const T* __restrict__ pn,
                                                 const T* __restrict__ pprev, const HaloBufs<T>& H,
                                                 const WaveTile& t, double alpha, double c1, double c2,
                                                 double& dacc, double& zacc) {
  const int64_t P = G.pitch;
  const int lane = threadIdx.x & 63;
  const int jl = t.j0 + lane * VEC;
  bool valid[VEC];
  int gjc[VEC];
#pragma unroll
  for (int u = 0; u < VEC; ++u) {
    valid[u] = jl + u <= t.jend;
    gjc[u] = G.gj0 + min(jl + u, t.jend);
  }
  const bool lane_any = valid[0];
  const bool lane_full = valid[VEC - 1];
  const int jlp = min(jl, 1 + (G.ny / VEC) * VEC);
  const int jlw = min(jl, 1 + ((G.ny - 1) / VEC) * VEC);
  const int jr = t.jend + 1;
  constexpr bool kReadW = MODE != kBwPend;
  for (int i = t.i0; i <= t.iend; ++i) {
    T pm[VEC], pc[VEC], pp[VEC], wr[VEC], rr[VEC], pv[VEC];
    vload_raw<T, VEC>(pn + int64_t(i - 1) * P + jlp, pm);
    vload_raw<T, VEC>(pn + int64_t(i) * P + jlp, pc);
    vload_raw<T, VEC>(pn + int64_t(i + 1) * P + jlp, pp);
    if constexpr (kReadW) vload_raw<T, VEC>(w + int64_t(i) * P + jlw, wr);
    if constexpr (MODE == kBwLoad) vload_raw<T, VEC>(pprev + int64_t(i) * P + jlw, pv);
    vload_raw<T, VEC>(r + int64_t(i) * P + jlw, rr);
    const T el = pn[int64_t(i) * P + t.j0 - 1], er = pn[int64_t(i) * P + jr];
    const RowConst rc = load_row(Tb, G.gi0 + i);
    const int ucls = EXACT ? 0 : row_class(rc, G.gj0 + t.j0, G.gj0 + t.jend);
    const double uval = ucls == 1 ? 1.0 : G.inv_eps;
    const double left = double(dpp_shift<kWaveShr1>(pc[VEC - 1], el));
    const double right = double(dpp_shift<kWaveShl1>(pc[0], er));
    T ws[VEC], rs[VEC];
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      const double pjm = u == 0 ? left : double(pc[u - 1]);
      const double pjp = u == VEC - 1 ? right : double(pc[u + 1]);
      double a0, a1, b0, b1;
      if (ucls != 0) {
        a0 = a1 = b0 = b1 = uval;
      } else {
        const ColConst c = load_col(Tb, gjc[u]);
        a0 = face_a0c(c, rc, G);
        a1 = face_a1c(c, rc, G);
        b0 = face_b0c(c, rc, G);
        b1 = face_b1c(c, rc, G);
      }
      const double pcu = double(pc[u]);
      const double Ap = apply_a<EXACT>(pcu, double(pm[u]), double(pp[u]), pjm, pjp, a0, a1, b0, b1, G);
      const double ro = double(rr[u]);
      double dw;
      if constexpr (MODE == kBwEvery) {
        const double wo = double(wr[u]);
        ws[u] = static_cast<T>(upd_w<EXACT>(wo, alpha, pcu));
        dw = double(ws[u]) - wo;
      } else {
        dw = alpha * pcu;
        if constexpr (MODE == kBwRecover) {
          const double zo = zdiv_u<EXACT>(ucls, ro, a0, a1, b0, b1, G);  // z^{k-1}, as in k_pcg_a
          ws[u] = static_cast<T>(__builtin_fma(c1, pcu, __builtin_fma(-c2, zo, double(wr[u]))));
        } else if constexpr (MODE == kBwLoad) {
          ws[u] = static_cast<T>(__builtin_fma(alpha, pcu, __builtin_fma(c2, double(pv[u]), double(wr[u]))));
        }
      }
      rs[u] = static_cast<T>(upd_r<EXACT>(ro, alpha, Ap));
      if (valid[u]) {
        dacc += dw * dw;
        const double rq = double(rs[u]);
        zacc += zdiv_u<EXACT>(ucls, rq, a0, a1, b0, b1, G) * rq;
      }
    }
    const int64_t c = int64_t(i) * P + jl;
    if (lane_full) {
      if constexpr (kReadW) vstore<T, VEC>(w + c, ws);
      vstore<T, VEC>(r + c, rs);
    } else {
#pragma unroll
      for (int u = 0; u < VEC; ++u)
        if (valid[u]) {
          if constexpr (kReadW) w[c + u] = ws[u];
          r[c + u] = rs[u];
        }
    }
    if (lane_any) {
      if (i == 1 && (G.nb & kNbXlo)) {
#pragma unroll
        for (int u = 0; u < VEC; ++u) if (valid[u]) H.send[0][jl + u - 1] = rs[u];
      }
      if (i == G.nx && (G.nb & kNbXhi)) {
#pragma unroll
        for (int u = 0; u < VEC; ++u) if (valid[u]) H.send[1][jl + u - 1] = rs[u];
      }
      if (jl == 1 && (G.nb & kNbYlo)) H.send[2][i - 1] = rs[0];
#pragma unroll
      for (int u = 0; u < VEC; ++u)
        if (jl + u == G.ny && (G.nb & kNbYhi)) H.send[3][i - 1] = rs[u];
    }
  }
}

template <typename T, int VEC, int WAVES, bool EXACT, bool PAIRW>
__device__ __forceinline__ void pcg_b_rows_body(const DevGeom& G, const DevTables& Tb, T* __restrict__ w,
                                                T* __restrict__ r, const T* p0, const T* p1,
                                                const HaloBufs<T>& H, double* __restrict__ partials,
                                                PcgState* S, int TI, int tiles_j, int ntiles, int abl) {
  constexpr int W = 64 * VEC;
  if (S->done) return;
  const long long k = S->it;
  const double denom = S->red_a[0];
  const bool bd = S->norm == int(Norm::kWeighted) ? fabs(denom) < S->bd_tol : denom < S->bd_tol;
  if (bd || !(denom == denom)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      S->iters = k;
      S->status = int(Status::kBreakdown);
      if (!(denom == denom)) S->nan_flag = 1;
      S->done = 1;
    }
    return;
  }
  const double alpha = S->zr[(k - 1) & 1] / denom;
  // pairing: odd k defers its w step, even k applies two (slot k & 1 of alpha is written here and
  // slot (k - 1) & 1 only read, so no block can see a half-written value)
  const bool odd = k & 1;
  double alpha_prev = 0.0, beta = 0.0;
  bool recover = false;
  if constexpr (PAIRW) {
    alpha_prev = S->alpha[(k - 1) & 1];
    beta = S->zr[(k - 1) & 1] / S->zr[k & 1];  // beta_k of k_pcg_a(k)
    recover = !odd && fabs(beta) >= S->pair_min_beta;
  }
  if (PAIRW && blockIdx.x == 0 && threadIdx.x == 0) {
    S->alpha[k & 1] = alpha;
    S->w_pend = odd ? k : 0;
  }
  const WaveTile t = wave_tile(WAVES, tiles_j, ntiles, TI, W, G, abl);
  if (!t.live) return;
  const T* __restrict__ pn = (k & 1) ? p1 : p0;
  const T* __restrict__ pprev = (k & 1) ? p0 : p1;
  double dacc = 0.0, zacc = 0.0;
  if constexpr (!PAIRW) {
    pcg_b_rows_march<T, VEC, EXACT, kBwEvery>(G, Tb, w, r, pn, pprev, H, t, alpha, 0.0, 0.0, dacc, zacc);
  } else if (odd) {
    pcg_b_rows_march<T, VEC, EXACT, kBwPend>(G, Tb, w, r, pn, pprev, H, t, alpha, 0.0, 0.0, dacc, zacc);
  } else if (recover) {
    const double c2 = alpha_prev / beta;
    pcg_b_rows_march<T, VEC, EXACT, kBwRecover>(G, Tb, w, r, pn, pprev, H, t, alpha, alpha + c2, c2,
                                                 dacc, zacc);
  } else {
    pcg_b_rows_march<T, VEC, EXACT, kBwLoad>(G, Tb, w, r, pn, pprev, H, t, alpha, alpha, alpha_prev,
                                              dacc, zacc);
  }
  wave_sum2_mfma(dacc, zacc);
  if ((threadIdx.x & 63) == 0) {
    partials[2 * t.id] = dacc;
    partials[2 * t.id + 1] = zacc;
  }
}

template <typename T, int VEC, int WAVES, bool EXACT>
__global__ void __launch_bounds__(64 * WAVES)
k_pcg_b_rows(DevGeom G, DevTables Tb, T* __restrict__ w, T* __restrict__ r, const T* p0,
             const T* p1, HaloBufs<T> H, double* __restrict__ partials, PcgState* S, int TI,
             int tiles_j, int ntiles, int abl) {
  pcg_b_rows_body<T, VEC, WAVES, EXACT, false>(G, Tb, w, r, p0, p1, H, partials, S, TI, tiles_j,
                                               ntiles, abl);
}

template <typename T, int VEC, int WAVES, bool EXACT>
__global__ void __launch_bounds__(64 * WAVES)
k_pcg_b_rows_paired(DevGeom G, DevTables Tb, T* __restrict__ w, T* __restrict__ r, const T* p0,
                    const T* p1, HaloBufs<T> H, double* __restrict__ partials, PcgState* S, int TI,
                    int tiles_j, int ntiles, int abl) {
  static_assert(!EXACT, "exact mode keeps the reference's per-iteration w update");
  pcg_b_rows_body<T, VEC, WAVES, false, true>(G, Tb, w, r, p0, p1, H, partials, S, TI, tiles_j,
                                              ntiles, abl);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
TileCfg make_row_tiles(const DevGeom& G, int vec, int waves, int rows) {
  TileCfg t = make_wave_tiles(G, vec, waves, rows == 0 ? 2 : rows);
  t.kind = 2;
  return t;
}

TileCfg make_wave_tiles(const DevGeom& G, int vec, int waves, int rows, int max_auto_rows,
                        int target_tiles) {
  PMX_CHECK(vec == 1 || vec == 2 || vec == 4, "vec must be 1, 2 or 4");
  PMX_CHECK(waves >= 1 && waves <= 16, "waves per block must be in [1,16]");
  PMX_CHECK(rows >= 0 && rows <= kMaxWaveRows, "wave tile rows must be in [0, 256] (0 = auto)");
  TileCfg t;
  t.kind = 1;
  t.vec = vec;
  t.waves = waves;
  t.block = 64 * vec;  // columns per tile
  t.tiles_j = (G.ny + t.block - 1) / t.block;
  if (rows == 0) {
    // Auto height (bench/tile_sweep.py at the per-rank shapes of 1/2/4/8 GPUs: 16384^2,
    // 16384x8192, 8192^2, 8192x4096): about `target_tiles` tiles per launch (pcg_a 22K = ~7
    // rounds of its 3072 wave slots, pcg_b 66K) balances the halo re-reads of short tiles against
    // the tail of tall ones; never shorter than 12 rows while that still leaves >= 6K tiles;
    // small grids go down to 2.
    const int64_t cells = int64_t(G.nx) * t.tiles_j;  // tile-rows x tile-columns at 1 row/tile
    const int64_t want = (cells + target_tiles / 2) / target_tiles;
    const int64_t floor_rows = std::min<int64_t>(12, std::max<int64_t>(2, cells / 6144));
    rows = int(std::min<int64_t>(max_auto_rows, std::max(want, floor_rows)));
  }
  t.rows = rows;
  t.tiles_i = (G.nx + rows - 1) / rows;
  return t;
}

#define PMX_WAVE_DISPATCH(tc, EX, KERNEL, ...)                                                  \
  do {                                                                                          \
    const int nb_ = (tc.ntiles() + tc.waves - 1) / tc.waves;                                    \
    if (tc.vec == 2 && tc.waves == 4)                                                           \
      hipLaunchKernelGGL((KERNEL<T, 2, 4, EX>), dim3(nb_), dim3(256), 0, s, __VA_ARGS__);       \
    else if (tc.vec == 1 && tc.waves == 4)                                                      \
      hipLaunchKernelGGL((KERNEL<T, 1, 4, EX>), dim3(nb_), dim3(256), 0, s, __VA_ARGS__);       \
    else if (tc.vec == 2 && tc.waves == 1)                                                      \
      hipLaunchKernelGGL((KERNEL<T, 2, 1, EX>), dim3(nb_), dim3(64), 0, s, __VA_ARGS__);        \
    else if (tc.vec == 4 && tc.waves == 4)                                                      \
      hipLaunchKernelGGL((KERNEL<T, 4, 4, EX>), dim3(nb_), dim3(256), 0, s, __VA_ARGS__);       \
    else if (tc.vec == 2 && tc.waves == 8)                                                      \
      hipLaunchKernelGGL((KERNEL<T, 2, 8, EX>), dim3(nb_), dim3(512), 0, s, __VA_ARGS__);       \
    else                                                                                        \
      PMX_CHECK(false, "unsupported wave-tile config vec=" << tc.vec << " waves=" << tc.waves); \
  } while (0)

template <typename T>
void launch_pcg_a_wave(const DevGeom& G, const DevTables& Tb, const T* r, T* p0, T* p1,
                       HaloBufs<T> H, double* partials, PcgState* S, const TileCfg& tc, bool exact,
                       hipStream_t s) {
  if (exact)
    PMX_WAVE_DISPATCH(tc, true, k_pcg_a_wave, G, Tb, r, p0, p1, H, partials, S, tc.rows,
                      tc.tiles_j, tc.ntiles(), tc.abl);
  else
    PMX_WAVE_DISPATCH(tc, false, k_pcg_a_wave, G, Tb, r, p0, p1, H, partials, S, tc.rows,
                      tc.tiles_j, tc.ntiles(), tc.abl);
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_pcg_b_wave(const DevGeom& G, const DevTables& Tb, T* w, T* r, const T* p0,
                       const T* p1, HaloBufs<T> H, double* partials, PcgState* S,
                       const TileCfg& tc, bool exact, hipStream_t s) {
  if (tc.kind == 2) {  // ring-free row kernel
    if (exact)
      PMX_WAVE_DISPATCH(tc, true, k_pcg_b_rows, G, Tb, w, r, p0, p1, H, partials, S, tc.rows,
                        tc.tiles_j, tc.ntiles(), tc.abl);
    else if (tc.pair_w)
      PMX_WAVE_DISPATCH(tc, false, k_pcg_b_rows_paired, G, Tb, w, r, p0, p1, H, partials, S, tc.rows,
                        tc.tiles_j, tc.ntiles(), tc.abl);
    else
      PMX_WAVE_DISPATCH(tc, false, k_pcg_b_rows, G, Tb, w, r, p0, p1, H, partials, S, tc.rows,
                        tc.tiles_j, tc.ntiles(), tc.abl);
  } else if (exact)
    PMX_WAVE_DISPATCH(tc, true, k_pcg_b_wave, G, Tb, w, r, p0, p1, H, partials, S, tc.rows,
                      tc.tiles_j, tc.ntiles(), tc.abl);
  else
    PMX_WAVE_DISPATCH(tc, false, k_pcg_b_wave, G, Tb, w, r, p0, p1, H, partials, S, tc.rows,
                      tc.tiles_j, tc.ntiles(), tc.abl);
  HIP_CHECK(hipGetLastError());
}

template void launch_pcg_a_wave<double>(const DevGeom&, const DevTables&, const double*, double*,
                                        double*, HaloBufs<double>, double*, PcgState*,
                                        const TileCfg&, bool, hipStream_t);
template void launch_pcg_b_wave<double>(const DevGeom&, const DevTables&, double*, double*,
                                        const double*, const double*, HaloBufs<double>, double*,
                                        PcgState*, const TileCfg&, bool, hipStream_t);
template void launch_pcg_a_wave<float>(const DevGeom&, const DevTables&, const float*, float*,
                                       float*, HaloBufs<float>, double*, PcgState*,
                                       const TileCfg&, bool, hipStream_t);
template void launch_pcg_b_wave<float>(const DevGeom&, const DevTables&, float*, float*,
                                       const float*, const float*, HaloBufs<float>, double*,
                                       PcgState*, const TileCfg&, bool, hipStream_t);

}  // namespace pmx
