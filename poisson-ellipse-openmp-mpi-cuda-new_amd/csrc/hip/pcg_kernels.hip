// Fused PCG kernels for CDNA4 (gfx950).  See pmx/kernels.hpp for the dataflow.
//
// Replaces the reference's per-op CUDA kernels (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:507-676):
//   apply_A_kernel + dot_kernel(Ap,p) + update_p_kernel       -> k_pcg_a
//   update_w_r_kernel + apply_Dinv_kernel + dot_kernel(z,r)   -> k_pcg_b
//   host partial-sum loops dot_gpu/reduce_diff (:772-797)     -> k_reduce (device, deterministic)
//   CPU fic_reg + H2D copies (:713-760)                       -> k_init + on-the-fly coefficients
//
// Mapping: one workgroup = one tile of `rows` x BLOCK nodes; thread t owns column j0+t (the
// contiguous axis, so every wave64 load/store is one coalesced 512-B (fp64) segment) and
// marches down the rows.  The i-neighbours of the stencil live in registers, the j-neighbours
// of the freshly computed p row in a 3-slot LDS ring (one barrier per row).
#include <algorithm>
#include <cmath>

#include "pcg_device.hpp"
#include "pmx/common.hpp"
#include "pmx/kernels.hpp"
#include "pmx/spec.hpp"

namespace pmx {

using namespace dev;

constexpr int kMaxRows = 256;

TileCfg make_tiles(const DevGeom& G, int block, int rows) {
  PMX_CHECK(block == 256 || block == 128 || block == 512, "unsupported block " << block);
  PMX_CHECK(rows >= 0 && rows <= kMaxRows, "tile rows must be in [0, " << kMaxRows << "] (0 = auto)");
  TileCfg t;
  t.block = block;
  t.tiles_j = (G.ny + block - 1) / block;
  if (rows == 0) {
    // auto: enough workgroups to fill 256 CUs x 8 resident blocks, but marching tiles no
    // taller than 64 rows (the tile-height sweep in profiles/ shows 32-64 as the plateau)
    constexpr int64_t kTargetBlocks = 2048;
    const int64_t want = (int64_t(G.nx) * t.tiles_j + kTargetBlocks - 1) / kTargetBlocks;
    rows = int(std::min<int64_t>(64, std::max<int64_t>(2, want)));
  }
  t.rows = rows;
  t.tiles_i = (G.nx + rows - 1) / rows;
  return t;
}

// ---------------------------------------------------------------------------
// r = B, w = 0, partial (z0, r0) with z0 = D^-1 r0, pack r edges
// ---------------------------------------------------------------------------
template <typename T, int BLOCK>
__global__ void __launch_bounds__(BLOCK)
k_init(DevGeom G, DevTables Tb, T* __restrict__ w, T* __restrict__ r, HaloBufs<T> H,
       double* __restrict__ partials, int TI, int tiles_j) {
  __shared__ double lds[2 * BLOCK / kWave];
  const Tile t = tile_of(blockIdx.x, tiles_j, TI, BLOCK, G);
  const int j = t.j0 + threadIdx.x;
  double acc = 0.0, unused = 0.0;
  if (j <= t.jend) {
    const int gj = G.gj0 + j;
    const ColConst cc = load_col(Tb, gj);
    const double yj = Tb.y[gj];
    for (int i = t.i0; i <= t.iend; ++i) {
      const int gi = G.gi0 + i;
      const RowConst rc = load_row(Tb, gi);
      const double a0 = face_a(cc, rc.rv0, G), a1 = face_a(cc, rc.rv1, G);
      const double b0 = face_b(rc, cc.rh0, G), b1 = face_b(rc, cc.rh1, G);
      // B_ij = F inside D (stage0/Withoutopenmp1.cpp:60)
      const double B = geo::inside(Tb.x[gi], yj, G.ax, G.by, G.ref_ellipse != 0) ? G.F : 0.0;
      const T Bs = static_cast<T>(B);
      const double Bq = static_cast<double>(Bs);
      const double D = diag<true>(a0, a1, b0, b1, G);
      const double z = (D != 0.0) ? Bq / D : 0.0;
      acc += z * Bq;
      const int64_t c = int64_t(i) * G.pitch + j;
      r[c] = Bs;
      w[c] = T(0);
      if (i == 1 && (G.nb & kNbXlo)) H.send[0][j - 1] = Bs;
      if (i == G.nx && (G.nb & kNbXhi)) H.send[1][j - 1] = Bs;
      if (j == 1 && (G.nb & kNbYlo)) H.send[2][i - 1] = Bs;
      if (j == G.ny && (G.nb & kNbYhi)) H.send[3][i - 1] = Bs;
    }
  }
  block_sum2<BLOCK>(acc, unused, lds);
  if (threadIdx.x == 0) {
    partials[2 * t.id] = 0.0;
    partials[2 * t.id + 1] = acc;
  }
}

// ---------------------------------------------------------------------------
// k_pcg_a: scalar prologue (stop test, beta), p^k = z + beta p^{k-1}, (A p^k, p^k) partial
// ---------------------------------------------------------------------------
template <typename T, int BLOCK, bool EXACT>
__global__ void __launch_bounds__(BLOCK)
k_pcg_a(DevGeom G, DevTables Tb, const T* __restrict__ r, T* p0, T* p1, HaloBufs<T> H,
        double* __restrict__ partials, PcgState* S, int TI, int tiles_j) {
  __shared__ double ring[3][BLOCK + 2];
  __shared__ double halo[2][kMaxRows];
  __shared__ double lds[2 * BLOCK / kWave];

  if (S->done) return;
  const long long k = S->it;
  const bool first = (k == 1);
  const double zr_prev = S->red_b[1];  // zr_{k-1}
  double beta = 0.0;
  if (!first) {
    // stop rule of iteration k-1 (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:890-906)
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
      return;
    }
    beta = zr_prev / S->zr[k & 1];  // zr_{k-1} / zr_{k-2}
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S->zr[(k - 1) & 1] = zr_prev;
    if (!first) S->diff = sqrt(S->red_b[0]);
  }

  T* pnew = (k & 1) ? p1 : p0;  // p^k lives in buffer k & 1
  const T* pold = (k & 1) ? p0 : p1;
  const Tile t = tile_of(blockIdx.x, tiles_j, TI, BLOCK, G);
  const int nrows = t.iend - t.i0 + 1;
  const int64_t P = G.pitch;

  // (1) p^k on the two halo columns j0-1 / jend+1 (ghost columns come from the recv buffers)
  for (int idx = threadIdx.x; idx < 2 * nrows; idx += BLOCK) {
    const int side = idx >= nrows ? 1 : 0;
    const int ii = t.i0 + (side ? idx - nrows : idx);
    const int jj = side ? t.jend + 1 : t.j0 - 1;
    const int gi = G.gi0 + ii, gj = G.gj0 + jj;
    double v = 0.0;
    if (!dirichlet(G, gi, gj)) {
      double rv;
      if (jj == 0) rv = H.recv[2][ii - 1];
      else if (jj == G.ny + 1) rv = H.recv[3][ii - 1];
      else rv = r[int64_t(ii) * P + jj];
      const double a0 = coef_a(Tb, G, gi, gj), a1 = coef_a(Tb, G, gi + 1, gj);
      const double b0 = coef_b(Tb, G, gi, gj), b1 = coef_b(Tb, G, gi, gj + 1);
      const double z = zdiv<EXACT>(rv, a0, a1, b0, b1, G);
      v = first ? z : z + beta * double(pold[int64_t(ii) * P + jj]);
      if ((jj == 0 && (G.nb & kNbYlo)) || (jj == G.ny + 1 && (G.nb & kNbYhi)))
        pnew[int64_t(ii) * P + jj] = static_cast<T>(v);
    }
    halo[side][ii - t.i0] = v;
  }
  __syncthreads();

  // (2) march down the rows.  Row i+1's loads (r, p^{k-1}, row tables) are issued before row
  // i is computed, so every wave keeps two rows of HBM traffic in flight across the barrier.
  const int tid = threadIdx.x;
  const int j = t.j0 + tid;
  const bool valid = j <= t.jend;
  const int gj = G.gj0 + (valid ? j : t.jend);
  const ColConst cc = load_col(Tb, gj);
  const int rpos = t.jend - t.j0 + 2;  // LDS ring index of the right halo column
  const int ilast = t.iend + 1;
  auto fetch = [&](int i, double& rv, double& po) {
    rv = 0.0;
    po = 0.0;
    const int gi = G.gi0 + i;
    if (valid && i <= ilast && gi > 0 && gi < G.M) {
      rv = (i == 0) ? double(H.recv[0][j - 1])
                    : (i == G.nx + 1) ? double(H.recv[1][j - 1]) : double(r[int64_t(i) * P + j]);
      if (!first) po = double(pold[int64_t(i) * P + j]);
    }
  };
  double pm2 = 0.0, pm1 = 0.0;         // p^k at rows i-2, i-1
  double qa0 = 0.0, qa1 = 0.0, qb0 = 0.0, qb1 = 0.0;  // coefficients of row i-1
  double acc = 0.0;
  double rv_c, po_c;
  fetch(t.i0 - 1, rv_c, po_c);
  RowConst rc = load_row(Tb, G.gi0 + t.i0 - 1);
  for (int i = t.i0 - 1; i <= ilast; ++i) {
    double rv_n, po_n;
    fetch(i + 1, rv_n, po_n);
    const RowConst rc_n = load_row(Tb, G.gi0 + min(i + 1, ilast));
    const int gi = G.gi0 + i;
    const double a0 = face_a0c(cc, rc, G), a1 = face_a1c(cc, rc, G);
    const double b0 = face_b0c(cc, rc, G), b1 = face_b1c(cc, rc, G);
    double pc = 0.0;
    const int slot = (i - t.i0 + 1) % 3;
    if (valid) {
      if (gi > 0 && gi < G.M) {
        const double z = zdiv<EXACT>(rv_c, a0, a1, b0, b1, G);
        pc = first ? z : z + beta * po_c;
        const bool own = i >= t.i0 && i <= t.iend;
        const bool ghost = (i == 0 && (G.nb & kNbXlo)) || (i == G.nx + 1 && (G.nb & kNbXhi));
        if (own || ghost) pnew[int64_t(i) * P + j] = static_cast<T>(pc);
      }
      pc = double(static_cast<T>(pc));  // use the stored precision in A p (fp32 mode)
      ring[slot][tid + 1] = pc;
    }
    if (tid == 0 && i >= t.i0 && i <= t.iend) {
      ring[slot][0] = halo[0][i - t.i0];
      ring[slot][rpos] = halo[1][i - t.i0];
    }
    __syncthreads();
    if (valid && i - 1 >= t.i0) {
      const int sm = (i - t.i0) % 3;  // slot of row i-1
      const double pjm = ring[sm][tid], pjp = ring[sm][tid + 2];
      const double Ap = apply_a<EXACT>(pm1, pm2, pc, pjm, pjp, qa0, qa1, qb0, qb1, G);
      acc += Ap * pm1;
    }
    pm2 = pm1; pm1 = pc;
    qa0 = a0; qa1 = a1; qb0 = b0; qb1 = b1;
    rv_c = rv_n; po_c = po_n; rc = rc_n;
  }
  double unused = 0.0;
  block_sum2<BLOCK>(acc, unused, lds);
  if (threadIdx.x == 0) partials[t.id] = acc;
}

// ---------------------------------------------------------------------------
// k_pcg_b: alpha, A p (recomputed), w/r update, sum dw^2, (z, r), halo pack of r
// ---------------------------------------------------------------------------
template <typename T, int BLOCK, bool EXACT>
__global__ void __launch_bounds__(BLOCK)
k_pcg_b(DevGeom G, DevTables Tb, T* __restrict__ w, T* __restrict__ r, const T* p0, const T* p1,
        HaloBufs<T> H, double* __restrict__ partials, PcgState* S, int TI, int tiles_j) {
  __shared__ double lds[2 * BLOCK / kWave];
  if (S->done) return;
  const long long k = S->it;
  const double denom = S->red_a[0];
  // breakdown guard: |denom| < tol (stages 2-4) or denom < tol (stage 0), tol = 1e-15 by default
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
  const T* pn = (k & 1) ? p1 : p0;
  const Tile t = tile_of(blockIdx.x, tiles_j, TI, BLOCK, G);
  const int j = t.j0 + threadIdx.x;
  double dacc = 0.0, zacc = 0.0;
  if (j <= t.jend) {
    // software-pipelined march: row i+1's five loads are in flight while row i is computed
    const int64_t P = G.pitch;
    const int gj = G.gj0 + j;
    const ColConst cc = load_col(Tb, gj);
    double pm = double(pn[int64_t(t.i0 - 1) * P + j]);
    int64_t c = int64_t(t.i0) * P + j;
    double pc = double(pn[c]);
    double pp = double(pn[c + P]), pjm = double(pn[c - 1]), pjp = double(pn[c + 1]);
    double wo = double(w[c]), ro = double(r[c]);
    RowConst rc = load_row(Tb, G.gi0 + t.i0);
    double acur = face_a0c(cc, rc, G);
    for (int i = t.i0; i <= t.iend; ++i) {
      const int64_t cn = c + P;
      const bool more = i < t.iend;
      double pp_n = 0.0, pjm_n = 0.0, pjp_n = 0.0, wo_n = 0.0, ro_n = 0.0;
      if (more) {
        pp_n = double(pn[cn + P]);
        pjm_n = double(pn[cn - 1]);
        pjp_n = double(pn[cn + 1]);
        wo_n = double(w[cn]);
        ro_n = double(r[cn]);
      }
      const RowConst rc_n = load_row(Tb, G.gi0 + (more ? i + 1 : i));
      const double a0 = acur, a1 = face_a1c(cc, rc, G);
      const double b0 = face_b0c(cc, rc, G), b1 = face_b1c(cc, rc, G);
      const double Ap = apply_a<EXACT>(pc, pm, pp, pjm, pjp, a0, a1, b0, b1, G);
      const T ws = static_cast<T>(upd_w<EXACT>(wo, alpha, pc));
      const T rs = static_cast<T>(upd_r<EXACT>(ro, alpha, Ap));
      const double dw = double(ws) - wo;
      dacc += dw * dw;
      const double rq = double(rs);
      const double z = zdiv<EXACT>(rq, a0, a1, b0, b1, G);
      zacc += z * rq;
      w[c] = ws;
      r[c] = rs;
      if (i == 1 && (G.nb & kNbXlo)) H.send[0][j - 1] = rs;
      if (i == G.nx && (G.nb & kNbXhi)) H.send[1][j - 1] = rs;
      if (j == 1 && (G.nb & kNbYlo)) H.send[2][i - 1] = rs;
      if (j == G.ny && (G.nb & kNbYhi)) H.send[3][i - 1] = rs;
      pm = pc; pc = pp; acur = a1;
      pp = pp_n; pjm = pjm_n; pjp = pjp_n; wo = wo_n; ro = ro_n; rc = rc_n;
      c = cn;
    }
  }
  block_sum2<BLOCK>(dacc, zacc, lds);
  if (threadIdx.x == 0) {
    partials[2 * t.id] = dacc;
    partials[2 * t.id + 1] = zacc;
  }
}

// ---------------------------------------------------------------------------
// k_edge_r: the r update of k_pcg_b restricted to the edge lines that feed a neighbour (one
// thread per edge node).  Same inputs, coefficient values and expression as k_pcg_b, so the
// packed values equal the r that k_pcg_b stores.  It reads p, r and the scalars only, so it
// is enqueued right before k_pcg_b and the halo send waits on it alone.
// ---------------------------------------------------------------------------
template <typename T, bool EXACT>
__global__ void __launch_bounds__(256)
k_edge_r(DevGeom G, DevTables Tb, const T* __restrict__ r, const T* p0, const T* p1, HaloBufs<T> H,
         const PcgState* S) {
  if (S->done) return;
  const long long k = S->it;
  const double denom = S->red_a[0];
  const bool bd = S->norm == int(Norm::kWeighted) ? fabs(denom) < S->bd_tol : denom < S->bd_tol;
  if (bd || !(denom == denom)) return;  // k_pcg_b records the breakdown
  const double alpha = S->zr[(k - 1) & 1] / denom;
  const T* pn = (k & 1) ? p1 : p0;
  int idx = blockIdx.x * 256 + threadIdx.x;
  int side = 0;
  for (; side < 4; ++side) {
    const int len = side < 2 ? G.ny : G.nx;
    if (idx < len) break;
    idx -= len;
  }
  if (side == 4 || !(G.nb & (1 << side))) return;  // kNbXlo..kNbYhi == 1 << side
  const int i = side == 0 ? 1 : side == 1 ? G.nx : idx + 1;
  const int j = side < 2 ? idx + 1 : side == 2 ? 1 : G.ny;
  const int gi = G.gi0 + i, gj = G.gj0 + j;
  const int64_t P = G.pitch, c = int64_t(i) * P + j;
  const double a0 = coef_a(Tb, G, gi, gj), a1 = coef_a(Tb, G, gi + 1, gj);
  const double b0 = coef_b(Tb, G, gi, gj), b1 = coef_b(Tb, G, gi, gj + 1);
  const double pc = double(pn[c]);
  const double Ap = apply_a<EXACT>(pc, double(pn[c - P]), double(pn[c + P]), double(pn[c - 1]),
                                   double(pn[c + 1]), a0, a1, b0, b1, G);
  const double ro = double(r[c]);
  H.send[side][idx] = static_cast<T>(upd_r<EXACT>(ro, alpha, Ap));
}

// ---------------------------------------------------------------------------
// Deterministic multi-block finish of the block partials.  Block c sums the fixed chunk
// [c*n/nb, (c+1)*n/nb) and stores it; the last block to finish (atomic ticket) adds the nb chunk
// sums in chunk order on the matrix cores.  Same bits on every run and every nb-invariant
// launch; ~64 CUs stream the partials instead of one (the pcg_b partials of a 16384^2 tile
// grid are 1.4 MB: 26 us on a single workgroup).
// ---------------------------------------------------------------------------
template <int NQ>
__global__ void __launch_bounds__(256)
k_reduce(const double* __restrict__ part, int n, double w0, double w1, double* out, PcgState* S,
         int mode, double* chunk, unsigned* ticket) {
  __shared__ double lds[2 * 256 / kWave];
  __shared__ int last;
  if ((mode & kSkipIfDone) && S->done) return;
  const int nb = int(gridDim.x);
  const int lo = int(int64_t(n) * blockIdx.x / nb);
  const int hi = int(int64_t(n) * (blockIdx.x + 1) / nb);
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  int i = lo + int(threadIdx.x);
  for (; i + 3 * 256 < hi; i += 4 * 256) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s0[u] += part[int64_t(i + u * 256) * NQ];
      if (NQ == 2) s1[u] += part[int64_t(i + u * 256) * NQ + 1];
    }
  }
  for (; i < hi; i += 256) {
    s0[0] += part[int64_t(i) * NQ];
    if (NQ == 2) s1[0] += part[int64_t(i) * NQ + 1];
  }
  double a = (s0[0] + s0[1]) + (s0[2] + s0[3]);
  double b = (s1[0] + s1[1]) + (s1[2] + s1[3]);
  block_sum2<256>(a, b, lds);
  if (threadIdx.x == 0) {
    st_publish(chunk + 2 * blockIdx.x, a);
    st_publish(chunk + 2 * blockIdx.x + 1, b);
    last = ticket_arrive_last(ticket, nb);
  }
  __syncthreads();
  if (!last || threadIdx.x >= kWave) return;  // wave 0 of the last block finishes (full EXEC)
  const int l = int(threadIdx.x);
  double ta = l < nb ? ld_published(chunk + 2 * l) : 0.0;
  double tb = l < nb ? ld_published(chunk + 2 * l + 1) : 0.0;
  wave_sum2_mfma(ta, tb);
  if (l == 0) {
    out[0] = ta * w0;
    if (NQ == 2) out[1] = tb * w1;
    if (!(ta == ta) || !(tb == tb) || isinf(ta) || isinf(tb)) S->nan_flag = 1;
    if (mode & kBumpIter) S->it += 1;
    *ticket = 0u;  // re-arm for the next launch (stream order makes this visible to it)
  }
}

__global__ void k_local_allreduce(double* const* bufs, int nranks, int nq) {
  if (threadIdx.x != 0) return;
  for (int q = 0; q < nq; ++q) {
    double s = 0.0;
    for (int rk = 0; rk < nranks; ++rk) s += bufs[rk][q];
    for (int rk = 0; rk < nranks; ++rk) bufs[rk][q] = s;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
#define PMX_BLOCK_DISPATCH(block, ...)                                  \
  switch (block) {                                                      \
    case 128: { constexpr int B = 128; __VA_ARGS__; } break;            \
    case 256: { constexpr int B = 256; __VA_ARGS__; } break;            \
    case 512: { constexpr int B = 512; __VA_ARGS__; } break;            \
    default: PMX_CHECK(false, "unsupported block " << block);           \
  }

template <typename T>
void launch_init(const DevGeom& G, const DevTables& Tb, T* w, T* r, HaloBufs<T> H,
                 double* partials, const TileCfg& tc, hipStream_t s) {
  PMX_BLOCK_DISPATCH(tc.block,
      hipLaunchKernelGGL((k_init<T, B>), dim3(tc.ntiles()), dim3(B), 0, s, G, Tb, w, r, H,
                         partials, tc.rows, tc.tiles_j));
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_pcg_a(const DevGeom& G, const DevTables& Tb, const T* r, T* p0, T* p1, HaloBufs<T> H,
                  double* partials, PcgState* S, const TileCfg& tc, bool exact, hipStream_t s) {
  if (exact) {
    PMX_BLOCK_DISPATCH(tc.block,
        hipLaunchKernelGGL((k_pcg_a<T, B, true>), dim3(tc.ntiles()), dim3(B), 0, s, G, Tb, r, p0,
                           p1, H, partials, S, tc.rows, tc.tiles_j));
  } else {
    PMX_BLOCK_DISPATCH(tc.block,
        hipLaunchKernelGGL((k_pcg_a<T, B, false>), dim3(tc.ntiles()), dim3(B), 0, s, G, Tb, r, p0,
                           p1, H, partials, S, tc.rows, tc.tiles_j));
  }
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_pcg_b(const DevGeom& G, const DevTables& Tb, T* w, T* r, const T* p0, const T* p1,
                  HaloBufs<T> H, double* partials, PcgState* S, const TileCfg& tc, bool exact,
                  hipStream_t s) {
  if (exact) {
    PMX_BLOCK_DISPATCH(tc.block,
        hipLaunchKernelGGL((k_pcg_b<T, B, true>), dim3(tc.ntiles()), dim3(B), 0, s, G, Tb, w, r,
                           p0, p1, H, partials, S, tc.rows, tc.tiles_j));
  } else {
    PMX_BLOCK_DISPATCH(tc.block,
        hipLaunchKernelGGL((k_pcg_b<T, B, false>), dim3(tc.ntiles()), dim3(B), 0, s, G, Tb, w, r,
                           p0, p1, H, partials, S, tc.rows, tc.tiles_j));
  }
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_edge_r(const DevGeom& G, const DevTables& Tb, const T* r, const T* p0, const T* p1,
                   HaloBufs<T> H, const PcgState* S, bool exact, hipStream_t s) {
  const int n = 2 * G.nx + 2 * G.ny;
  const dim3 grid((n + 255) / 256);
  if (exact) hipLaunchKernelGGL((k_edge_r<T, true>), grid, dim3(256), 0, s, G, Tb, r, p0, p1, H, S);
  else hipLaunchKernelGGL((k_edge_r<T, false>), grid, dim3(256), 0, s, G, Tb, r, p0, p1, H, S);
  HIP_CHECK(hipGetLastError());
}

void launch_reduce(const double* partials, int n, int nq, double w0, double w1, double* out,
                   PcgState* S, int mode, double* ws, hipStream_t s) {
  PMX_CHECK(nq == 1 || nq == 2, "nq must be 1 or 2");
  const int nb = std::max(1, std::min(kReduceMaxBlocks, n / 2048));
  double* chunk = ws;
  unsigned* ticket = reinterpret_cast<unsigned*>(ws + 2 * kReduceMaxBlocks);
  if (nq == 1)
    hipLaunchKernelGGL(k_reduce<1>, dim3(nb), dim3(256), 0, s, partials, n, w0, w1, out, S, mode, chunk, ticket);
  else
    hipLaunchKernelGGL(k_reduce<2>, dim3(nb), dim3(256), 0, s, partials, n, w0, w1, out, S, mode, chunk, ticket);
  HIP_CHECK(hipGetLastError());
}

void launch_local_allreduce(double* const* bufs, int nranks, int nq, hipStream_t s) {
  hipLaunchKernelGGL(k_local_allreduce, dim3(1), dim3(64), 0, s, bufs, nranks, nq);
  HIP_CHECK(hipGetLastError());
}

#define PMX_INST(T)                                                                              \
  template void launch_init<T>(const DevGeom&, const DevTables&, T*, T*, HaloBufs<T>, double*,  \
                               const TileCfg&, hipStream_t);                                     \
  template void launch_pcg_a<T>(const DevGeom&, const DevTables&, const T*, T*, T*, HaloBufs<T>, \
                                double*, PcgState*, const TileCfg&, bool, hipStream_t);          \
  template void launch_pcg_b<T>(const DevGeom&, const DevTables&, T*, T*, const T*, const T*,    \
                                HaloBufs<T>, double*, PcgState*, const TileCfg&, bool,           \
                                hipStream_t);                                                    \
  template void launch_edge_r<T>(const DevGeom&, const DevTables&, const T*, const T*, const T*, \
                                 HaloBufs<T>, const PcgState*, bool, hipStream_t);
PMX_INST(double)
PMX_INST(float)
#undef PMX_INST

}  // namespace pmx
