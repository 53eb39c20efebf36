// Setup and reduction kernels shared by both iterations (pcg1, pcg2) on CDNA4 (gfx950):
//   CPU fic_reg + H2D copies (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:713-760) -> k_init (w = 0,
//     r = B, z^0 partials, coefficients rebuilt on the fly from the 1-D face tables)
//   host partial-sum loops dot_gpu / reduce_diff (:772-797)                 -> k_reduce (device,
//     deterministic, ticketed multi-block finish)
//   k_edge_r (pcg2 with a second stream: the edge lines of r a neighbour needs, packed ahead of
//     the sweep), k_local_allreduce (LocalComm's in-process "all-reduce").
// Tiles: one workgroup = `rows` x BLOCK nodes, thread t owns column j0+t (the contiguous axis: every
// wave64 access is one coalesced segment).  The round-1 LDS-ring iteration kernels (k_pcg_a /
// k_pcg_b, `--kernel lds`) are retired (bench/RETIRED.md): the wave kernels replaced them.
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
  template void launch_edge_r<T>(const DevGeom&, const DevTables&, const T*, const T*, const T*, \
                                 HaloBufs<T>, const PcgState*, bool, hipStream_t);
PMX_INST(double)
PMX_INST(float)
#undef PMX_INST

}  // namespace pmx
