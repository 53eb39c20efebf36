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
  PMX_CHECK(rows >= 1 && rows <= kMaxRows, "tile rows must be in [1, " << kMaxRows << "]");
  TileCfg t;
  t.block = block;
  t.rows = rows;
  t.tiles_i = (G.nx + rows - 1) / rows;
  t.tiles_j = (G.ny + block - 1) / block;
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
      const double z = rv / diag<EXACT>(a0, a1, b0, b1, G);
      v = first ? z : z + beta * double(pold[int64_t(ii) * P + jj]);
      if ((jj == 0 && (G.nb & kNbYlo)) || (jj == G.ny + 1 && (G.nb & kNbYhi)))
        pnew[int64_t(ii) * P + jj] = static_cast<T>(v);
    }
    halo[side][ii - t.i0] = v;
  }
  __syncthreads();

  // (2) march down the rows
  const int tid = threadIdx.x;
  const int j = t.j0 + tid;
  const bool valid = j <= t.jend;
  const int gj = G.gj0 + (valid ? j : t.jend);
  const ColConst cc = load_col(Tb, gj);
  const int rpos = t.jend - t.j0 + 2;  // LDS ring index of the right halo column
  double pm2 = 0.0, pm1 = 0.0;         // p^k at rows i-2, i-1
  double qa0 = 0.0, qa1 = 0.0, qb0 = 0.0, qb1 = 0.0;  // coefficients of row i-1
  double acc = 0.0;
  for (int i = t.i0 - 1; i <= t.iend + 1; ++i) {
    const int gi = G.gi0 + i;
    const RowConst rc = load_row(Tb, gi);
    const double a0 = face_a(cc, rc.rv0, G), a1 = face_a(cc, rc.rv1, G);
    const double b0 = face_b(rc, cc.rh0, G), b1 = face_b(rc, cc.rh1, G);
    double pc = 0.0;
    const int slot = (i - t.i0 + 1) % 3;
    if (valid) {
      if (gi > 0 && gi < G.M) {
        double rv;
        if (i == 0) rv = H.recv[0][j - 1];
        else if (i == G.nx + 1) rv = H.recv[1][j - 1];
        else rv = r[int64_t(i) * P + j];
        const double z = rv / diag<EXACT>(a0, a1, b0, b1, G);
        pc = first ? z : z + beta * double(pold[int64_t(i) * P + j]);
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
  // breakdown guard: |denom| < 1e-15 (stages 2-4) or denom < 1e-15 (stage 0)
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
  const T* pn = (k & 1) ? p1 : p0;
  const Tile t = tile_of(blockIdx.x, tiles_j, TI, BLOCK, G);
  const int j = t.j0 + threadIdx.x;
  double dacc = 0.0, zacc = 0.0;
  if (j <= t.jend) {
    const int64_t P = G.pitch;
    const int gj = G.gj0 + j;
    const ColConst cc = load_col(Tb, gj);
    double pm = double(pn[int64_t(t.i0 - 1) * P + j]);
    double pc = double(pn[int64_t(t.i0) * P + j]);
    double acur = face_a(cc, Tb.rv[G.gi0 + t.i0], G);
    for (int i = t.i0; i <= t.iend; ++i) {
      const int64_t c = int64_t(i) * P + j;
      const double pp = double(pn[c + P]);
      const double pjm = double(pn[c - 1]), pjp = double(pn[c + 1]);
      const int gi = G.gi0 + i;
      const RowConst rc = load_row(Tb, gi);
      const double a0 = acur, a1 = face_a(cc, rc.rv1, G);
      const double b0 = face_b(rc, cc.rh0, G), b1 = face_b(rc, cc.rh1, G);
      const double Ap = apply_a<EXACT>(pc, pm, pp, pjm, pjp, a0, a1, b0, b1, G);
      const double wo = double(w[c]), ro = double(r[c]);
      const T ws = static_cast<T>(wo + alpha * pc);
      const T rs = static_cast<T>(ro - alpha * Ap);
      const double dw = double(ws) - wo;
      dacc += dw * dw;
      const double rq = double(rs);
      const double z = rq / diag<EXACT>(a0, a1, b0, b1, G);
      zacc += z * rq;
      w[c] = ws;
      r[c] = rs;
      if (i == 1 && (G.nb & kNbXlo)) H.send[0][j - 1] = rs;
      if (i == G.nx && (G.nb & kNbXhi)) H.send[1][j - 1] = rs;
      if (j == 1 && (G.nb & kNbYlo)) H.send[2][i - 1] = rs;
      if (j == G.ny && (G.nb & kNbYhi)) H.send[3][i - 1] = rs;
      pm = pc; pc = pp; acur = a1;
    }
  }
  block_sum2<BLOCK>(dacc, zacc, lds);
  if (threadIdx.x == 0) {
    partials[2 * t.id] = dacc;
    partials[2 * t.id + 1] = zacc;
  }
}

// ---------------------------------------------------------------------------
// deterministic single-block finish of block partials
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_reduce(const double* __restrict__ part, int n, int nq, double w0, double w1, double* out,
         PcgState* S, int mode) {
  __shared__ double lds[2 * 256 / kWave];
  if ((mode & kSkipIfDone) && S->done) return;
  double s0 = 0.0, s1 = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    s0 += part[int64_t(i) * nq];
    if (nq == 2) s1 += part[int64_t(i) * nq + 1];
  }
  block_sum2<256>(s0, s1, lds);
  if (threadIdx.x == 0) {
    out[0] = s0 * w0;
    if (nq == 2) out[1] = s1 * w1;
    if (!(s0 == s0) || !(s1 == s1) || isinf(s0) || isinf(s1)) S->nan_flag = 1;
    if (mode & kBumpIter) S->it += 1;
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

void launch_reduce(const double* partials, int n, int nq, double w0, double w1, double* out,
                   PcgState* S, int mode, hipStream_t s) {
  PMX_CHECK(nq == 1 || nq == 2, "nq must be 1 or 2");
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(256), 0, s, partials, n, nq, w0, w1, out, S, mode);
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
                                hipStream_t);
PMX_INST(double)
PMX_INST(float)
#undef PMX_INST

}  // namespace pmx
