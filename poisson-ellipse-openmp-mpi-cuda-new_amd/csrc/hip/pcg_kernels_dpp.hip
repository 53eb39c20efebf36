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

#include "pcg_device.hpp"
#include "pmx/common.hpp"
#include "pmx/kernels.hpp"
#include "pmx/spec.hpp"

namespace pmx {

using namespace dev;

namespace {

constexpr int kMaxWaveRows = 64;  // halo values for one tile live one-per-lane

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(int(b), lane);
  const int hi = __builtin_amdgcn_readlane(int(b >> 32), lane);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}

// DPP wave shifts on a double: lane l receives lane l-1's (SHR) / l+1's (SHL) value; the edge lane
// that has no source keeps `edge`.
constexpr int kWaveShl1 = 0x130;
constexpr int kWaveShr1 = 0x138;
template <int CTRL>
__device__ __forceinline__ double dpp_shift_f64(double v, double edge) {
  const long long b = __double_as_longlong(v);
  const long long e = __double_as_longlong(edge);
  const int lo = __builtin_amdgcn_update_dpp(int(e), int(b), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(int(e >> 32), int(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}

template <typename T, int VEC> struct VecT;
template <> struct VecT<double, 1> { using type = double; };
template <> struct VecT<double, 2> { using type = double2; };
template <> struct VecT<double, 4> { using type = double4; };
template <> struct VecT<float, 1> { using type = float; };
template <> struct VecT<float, 2> { using type = float2; };
template <> struct VecT<float, 4> { using type = float4; };

template <typename T, int VEC>
__device__ __forceinline__ void vload(const T* p, double (&out)[VEC]) {
  using V = typename VecT<T, VEC>::type;
  const V v = *reinterpret_cast<const V*>(p);
  const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
  for (int u = 0; u < VEC; ++u) out[u] = double(e[u]);
}

template <typename T, int VEC>
__device__ __forceinline__ void vstore(T* p, const T (&in)[VEC]) {
  using V = typename VecT<T, VEC>::type;
  V v;
  T* e = reinterpret_cast<T*>(&v);
#pragma unroll
  for (int u = 0; u < VEC; ++u) e[u] = in[u];
  *reinterpret_cast<V*>(p) = v;
}

struct WaveTile {
  int i0, iend, j0, jend, id;
  bool live;
};

__device__ __forceinline__ WaveTile wave_tile(int waves, int tiles_j, int ntiles, int TI, int W,
                                              const DevGeom& G) {
  WaveTile t;
  t.id = blockIdx.x * waves + (threadIdx.x >> 6);
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
// ---------------------------------------------------------------------------
template <typename T, int VEC, int WAVES, bool EXACT>
__global__ void __launch_bounds__(64 * WAVES)
k_pcg_a_wave(DevGeom G, DevTables Tb, const T* __restrict__ r, T* p0, T* p1, HaloBufs<T> H,
             double* __restrict__ partials, PcgState* S, int TI, int tiles_j, int ntiles) {
  constexpr int W = 64 * VEC;
  long long k;
  bool first;
  double beta;
  if (!prologue_a(S, k, first, beta)) return;
  const WaveTile t = wave_tile(WAVES, tiles_j, ntiles, TI, W, G);
  if (!t.live) return;
  T* pnew = (k & 1) ? p1 : p0;
  const T* pold = (k & 1) ? p0 : p1;
  const int64_t P = G.pitch;
  const int lane = threadIdx.x & 63;

  // (1) halo columns j0-1 (hl) and jend+1 (hr): lane l holds row i0+l
  double hl = 0.0, hr = 0.0;
  {
    const int ii = t.i0 + lane;
    if (ii <= t.iend) {
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const int jj = side ? t.jend + 1 : t.j0 - 1;
        const int gi = G.gi0 + ii, gj = G.gj0 + jj;
        double v = 0.0;
        if (!dirichlet(G, gi, gj)) {
          double rv;
          if (jj == 0) rv = double(H.recv[2][ii - 1]);
          else if (jj == G.ny + 1) rv = double(H.recv[3][ii - 1]);
          else rv = double(r[int64_t(ii) * P + jj]);
          const double a0 = coef_a(Tb, G, gi, gj), a1 = coef_a(Tb, G, gi + 1, gj);
          const double b0 = coef_b(Tb, G, gi, gj), b1 = coef_b(Tb, G, gi, gj + 1);
          const double z = rv / diag<EXACT>(a0, a1, b0, b1, G);
          v = first ? z : z + beta * double(pold[int64_t(ii) * P + jj]);
          if ((jj == 0 && (G.nb & kNbYlo)) || (jj == G.ny + 1 && (G.nb & kNbYhi)))
            pnew[int64_t(ii) * P + jj] = static_cast<T>(v);
          v = double(static_cast<T>(v));
        }
        if (side) hr = v; else hl = v;
      }
    }
  }

  // (2) march.  Lane columns jl..jl+VEC-1.
  const int jl = t.j0 + lane * VEC;
  bool valid[VEC];
  ColConst cc[VEC];
  double rhn = 0.0;  // rh[gj+VEC] for the last column's b(i, j+1)
#pragma unroll
  for (int u = 0; u < VEC; ++u) {
    valid[u] = jl + u <= t.jend;
    cc[u] = load_col(Tb, G.gj0 + min(jl + u, t.jend));
  }
  const bool lane_any = valid[0];
  const bool lane_full = valid[VEC - 1];
  const int ilast = t.iend + 1;

  auto fetch = [&](int i, double (&rv)[VEC], double (&po)[VEC]) {
#pragma unroll
    for (int u = 0; u < VEC; ++u) { rv[u] = 0.0; po[u] = 0.0; }
    const int gi = G.gi0 + i;
    if (!lane_any || i > ilast || gi <= 0 || gi >= G.M) return;
    if (i == 0 || i == G.nx + 1) {
      const T* src = H.recv[i == 0 ? 0 : 1];
#pragma unroll
      for (int u = 0; u < VEC; ++u)
        if (valid[u]) rv[u] = double(src[jl + u - 1]);
    } else if (lane_full) {
      vload<T, VEC>(r + int64_t(i) * P + jl, rv);
    } else {
#pragma unroll
      for (int u = 0; u < VEC; ++u)
        if (valid[u]) rv[u] = double(r[int64_t(i) * P + jl + u]);
    }
    if (!first) {
      if (lane_full) {
        vload<T, VEC>(pold + int64_t(i) * P + jl, po);
      } else {
#pragma unroll
        for (int u = 0; u < VEC; ++u)
          if (valid[u]) po[u] = double(pold[int64_t(i) * P + jl + u]);
      }
    }
  };

  double pm2[VEC], pm1[VEC], qa0[VEC], qa1[VEC], qb0[VEC], qb1[VEC];
#pragma unroll
  for (int u = 0; u < VEC; ++u) { pm2[u] = pm1[u] = qa0[u] = qa1[u] = qb0[u] = qb1[u] = 0.0; }
  double hl_m1 = 0.0, hr_m1 = 0.0;  // halo values of row i-1
  double acc = 0.0;
  double rv_c[VEC], po_c[VEC];
  fetch(t.i0 - 1, rv_c, po_c);
  RowConst rc = load_row(Tb, G.gi0 + t.i0 - 1);
  for (int i = t.i0 - 1; i <= ilast; ++i) {
    double rv_n[VEC], po_n[VEC];
    fetch(i + 1, rv_n, po_n);
    const RowConst rc_n = load_row(Tb, G.gi0 + min(i + 1, ilast));
    const int gi = G.gi0 + i;
    const bool own_row = i >= t.i0 && i <= t.iend;
    const double hl_i = own_row ? readlane_f64(hl, i - t.i0) : 0.0;
    const double hr_i = own_row ? readlane_f64(hr, i - t.i0) : 0.0;
    double a0[VEC], a1[VEC], b0[VEC], b1[VEC], pc[VEC];
    const bool live_row = gi > 0 && gi < G.M;
    T st[VEC];
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      a0[u] = face_a(cc[u], rc.rv0, G);
      a1[u] = face_a(cc[u], rc.rv1, G);
      b0[u] = face_b(rc, cc[u].rh0, G);
      b1[u] = face_b(rc, cc[u].rh1, G);
      double v = 0.0;
      if (valid[u] && live_row) {
        const double z = rv_c[u] / diag<EXACT>(a0[u], a1[u], b0[u], b1[u], G);
        v = first ? z : z + beta * po_c[u];
      }
      st[u] = static_cast<T>(v);
      v = double(st[u]);
      // the column right after the tile's last one carries the right halo value, so the DPP
      // shift below hands it to column jend for partial tiles too
      if (jl + u == t.jend + 1) v = hr_i;
      pc[u] = v;
    }
    if (live_row && (own_row || (i == 0 && (G.nb & kNbXlo)) || (i == G.nx + 1 && (G.nb & kNbXhi)))) {
      if (lane_full) {
        vstore<T, VEC>(pnew + int64_t(i) * P + jl, st);
      } else {
#pragma unroll
        for (int u = 0; u < VEC; ++u)
          if (valid[u]) pnew[int64_t(i) * P + jl + u] = st[u];
      }
    }
    // A p^k for row i-1 (pm1), neighbours: rows i-2 (pm2), i (pc); columns by DPP
    if (i - 1 >= t.i0) {
      const double left = dpp_shift_f64<kWaveShr1>(pm1[VEC - 1], hl_m1);
      const double right = dpp_shift_f64<kWaveShl1>(pm1[0], hr_m1);
#pragma unroll
      for (int u = 0; u < VEC; ++u) {
        const double pjm = u == 0 ? left : pm1[u - 1];
        const double pjp = u == VEC - 1 ? right : pm1[u + 1];
        if (valid[u])
          acc += apply_a<EXACT>(pm1[u], pm2[u], pc[u], pjm, pjp, qa0[u], qa1[u], qb0[u], qb1[u], G) * pm1[u];
      }
    }
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      pm2[u] = pm1[u]; pm1[u] = pc[u];
      qa0[u] = a0[u]; qa1[u] = a1[u]; qb0[u] = b0[u]; qb1[u] = b1[u];
      rv_c[u] = rv_n[u]; po_c[u] = po_n[u];
    }
    hl_m1 = hl_i; hr_m1 = hr_i;
    rc = rc_n;
  }
  (void)rhn;
  acc = wave_sum(acc);
  if (lane == 0) partials[t.id] = acc;
}

// ---------------------------------------------------------------------------
// k_pcg_b (wave-tile): alpha, A p^k, w/r update, sum dw^2, (z, r), halo pack
// ---------------------------------------------------------------------------
template <typename T, int VEC, int WAVES, bool EXACT>
__global__ void __launch_bounds__(64 * WAVES)
k_pcg_b_wave(DevGeom G, DevTables Tb, T* __restrict__ w, T* __restrict__ r, const T* p0,
             const T* p1, HaloBufs<T> H, double* __restrict__ partials, PcgState* S, int TI,
             int tiles_j, int ntiles) {
  constexpr int W = 64 * VEC;
  if (S->done) return;
  const long long k = S->it;
  const double denom = S->red_a[0];
  const bool bd = S->norm == int(Norm::kWeighted) ? fabs(denom) < 1e-15 : denom < 1e-15;
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
  const WaveTile t = wave_tile(WAVES, tiles_j, ntiles, TI, W, G);
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
  // columns that exist in memory (<= ny+1): the partial tile's right halo column is a real load
  bool mem[VEC];
#pragma unroll
  for (int u = 0; u < VEC; ++u) mem[u] = jl + u <= t.jend + 1;
  const bool lane_mem_full = mem[VEC - 1];
  const int jr = t.jend + 1;

  auto load_p = [&](int i, double (&out)[VEC]) {
#pragma unroll
    for (int u = 0; u < VEC; ++u) out[u] = 0.0;
    if (lane_mem_full) {
      vload<T, VEC>(pn + int64_t(i) * P + jl, out);
    } else {
#pragma unroll
      for (int u = 0; u < VEC; ++u)
        if (mem[u]) out[u] = double(pn[int64_t(i) * P + jl + u]);
    }
  };
  auto load_f = [&](const T* f, int i, double (&out)[VEC]) {
#pragma unroll
    for (int u = 0; u < VEC; ++u) out[u] = 0.0;
    if (lane_full) {
      vload<T, VEC>(f + int64_t(i) * P + jl, out);
    } else {
#pragma unroll
      for (int u = 0; u < VEC; ++u)
        if (valid[u]) out[u] = double(f[int64_t(i) * P + jl + u]);
    }
  };

  double pm[VEC], pc[VEC], pp[VEC], wo[VEC], ro[VEC];
  load_p(t.i0 - 1, pm);
  load_p(t.i0, pc);
  load_p(t.i0 + 1, pp);
  load_f(w, t.i0, wo);
  load_f(r, t.i0, ro);
  double el = double(pn[int64_t(t.i0) * P + t.j0 - 1]);  // left edge (column j0-1)
  double er = double(pn[int64_t(t.i0) * P + jr]);        // right edge (column jend+1)
  RowConst rc = load_row(Tb, G.gi0 + t.i0);
  double acur[VEC];
#pragma unroll
  for (int u = 0; u < VEC; ++u) acur[u] = face_a(cc[u], rc.rv0, G);
  double dacc = 0.0, zacc = 0.0;
  for (int i = t.i0; i <= t.iend; ++i) {
    const bool more = i < t.iend;
    double pp_n[VEC], wo_n[VEC], ro_n[VEC];
    double el_n = 0.0, er_n = 0.0;
    if (more) {
      load_p(i + 2, pp_n);
      load_f(w, i + 1, wo_n);
      load_f(r, i + 1, ro_n);
      el_n = double(pn[int64_t(i + 1) * P + t.j0 - 1]);
      er_n = double(pn[int64_t(i + 1) * P + jr]);
    } else {
#pragma unroll
      for (int u = 0; u < VEC; ++u) pp_n[u] = wo_n[u] = ro_n[u] = 0.0;
    }
    const RowConst rc_n = load_row(Tb, G.gi0 + (more ? i + 1 : i));
    const double left = dpp_shift_f64<kWaveShr1>(pc[VEC - 1], el);
    const double right = dpp_shift_f64<kWaveShl1>(pc[0], er);
    T ws[VEC], rs[VEC];
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      const double pjm = u == 0 ? left : pc[u - 1];
      const double pjp = u == VEC - 1 ? right : pc[u + 1];
      const double a0 = acur[u], a1 = face_a(cc[u], rc.rv1, G);
      const double b0 = face_b(rc, cc[u].rh0, G), b1 = face_b(rc, cc[u].rh1, G);
      const double Ap = apply_a<EXACT>(pc[u], pm[u], pp[u], pjm, pjp, a0, a1, b0, b1, G);
      ws[u] = static_cast<T>(wo[u] + alpha * pc[u]);
      rs[u] = static_cast<T>(ro[u] - alpha * Ap);
      if (valid[u]) {
        const double dw = double(ws[u]) - wo[u];
        dacc += dw * dw;
        const double rq = double(rs[u]);
        const double z = rq / diag<EXACT>(a0, a1, b0, b1, G);
        zacc += z * rq;
      }
      acur[u] = a1;
    }
    const int64_t c = int64_t(i) * P + jl;
    if (lane_full) {
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
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      pm[u] = pc[u]; pc[u] = pp[u]; pp[u] = pp_n[u]; wo[u] = wo_n[u]; ro[u] = ro_n[u];
    }
    el = el_n; er = er_n; rc = rc_n;
  }
  dacc = wave_sum(dacc);
  zacc = wave_sum(zacc);
  if (lane == 0) {
    partials[2 * t.id] = dacc;
    partials[2 * t.id + 1] = zacc;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
TileCfg make_wave_tiles(const DevGeom& G, int vec, int waves, int rows) {
  PMX_CHECK(vec == 1 || vec == 2 || vec == 4, "vec must be 1, 2 or 4");
  PMX_CHECK(waves >= 1 && waves <= 16, "waves per block must be in [1,16]");
  PMX_CHECK(rows >= 0 && rows <= kMaxWaveRows, "wave tile rows must be in [0, 64] (0 = auto)");
  TileCfg t;
  t.kind = 1;
  t.vec = vec;
  t.waves = waves;
  t.block = 64 * vec;  // columns per tile
  t.tiles_j = (G.ny + t.block - 1) / t.block;
  if (rows == 0) {
    constexpr int64_t kTargetWaves = 8192;  // 256 CUs x 32 wave slots
    const int64_t want = (int64_t(G.nx) * t.tiles_j + kTargetWaves - 1) / kTargetWaves;
    rows = int(std::min<int64_t>(64, std::max<int64_t>(2, want)));
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
                      tc.tiles_j, tc.ntiles());
  else
    PMX_WAVE_DISPATCH(tc, false, k_pcg_a_wave, G, Tb, r, p0, p1, H, partials, S, tc.rows,
                      tc.tiles_j, tc.ntiles());
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_pcg_b_wave(const DevGeom& G, const DevTables& Tb, T* w, T* r, const T* p0,
                       const T* p1, HaloBufs<T> H, double* partials, PcgState* S,
                       const TileCfg& tc, bool exact, hipStream_t s) {
  if (exact)
    PMX_WAVE_DISPATCH(tc, true, k_pcg_b_wave, G, Tb, w, r, p0, p1, H, partials, S, tc.rows,
                      tc.tiles_j, tc.ntiles());
  else
    PMX_WAVE_DISPATCH(tc, false, k_pcg_b_wave, G, Tb, w, r, p0, p1, H, partials, S, tc.rows,
                      tc.tiles_j, tc.ntiles());
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
