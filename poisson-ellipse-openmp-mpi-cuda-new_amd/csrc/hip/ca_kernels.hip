// s-step Jacobi-PCG ("ca", communication-avoiding CG): s iterations per TWO streaming passes and one
// reduction, instead of s single-pass sweeps (pcg1_kernels.hip) and s reductions.
//
// Same iteration as the reference (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:847-943; z = D^-1 r,
// alpha = (r, z) / (A p, p), w += alpha p, r -= alpha A p, beta = (r', z') / (r, z), p = z' + beta p,
// stop when ||w^{k+1} - w^k|| = |alpha| ||p|| < delta), regrouped by blocks of s iterations.  In
// the D-inner product <x, y> = x^T D y the preconditioned operator L = D^-1 A is self-adjoint, and
// after j < s iterations of a block p, z = D^-1 r and w - w_k lie in the span of the Krylov basis
//   Y = [P_0 .. P_s, Z_0 .. Z_{s-1}],  P_i = T_i(L - I) p_k,  Z_i = T_i(L - I) z_k
// (Chebyshev polynomials T_i: L - I has its spectrum in (-1, 1) -- Gershgorin on the M-matrix A --
// so the basis stays well conditioned; a monomial basis would not).  With p = Y a, z = Y b,
// w - w_k = Y c and L Y = Y T (T: the Chebyshev three-term recurrence, exact in the columns that stay
// in the basis), every scalar of the s iterations comes from two small Gram matrices:
//   (r, z) = b^T G_D b,   (A p, p) = a^T G_D T a,   ||p||^2 = a^T G_0 a,
//   G_D = Y^T D Y (all 2s+1 vectors),  G_0 = Y^T Y (the 2s-1 vectors p can use, P_0..P_{s-1}, Z_0..Z_{s-2}).
// So a block is:
//   pass 1 (k_ca_sweep<.., false>): per tile, the basis on the fly from p_k, z_k (radius s) and
//          the (2s+1)(2s+2)/2 + (2s-1)2s/2 Gram partials (s = 3: 28 + 15);
//   reduce (k_ca_reduce): the partials summed in a fixed order, then ONE lane runs the s iterations
//          on the coefficient vectors (alpha, beta, the breakdown guard and the stop test of every
//          iteration, exactly where the classic loop has them) and leaves a_n, b_n, c_n in CaState;
//   pass 2 (k_ca_sweep<.., true>): the basis again, p = Y a_n, z = Y b_n, w += Y c_n.
// HBM traffic per block: pass 1 reads p, z (16 B/pt), pass 2 reads p, z, w and writes them (48 B/pt):
// 64 B/pt for s iterations -- 21.3 B/pt/iteration at s = 3 against pcg1's 37.3.  The price is
// arithmetic: 2 x (2s - 1) stencils and ~50 Gram FMAs per point and block.
// The iterates equal the classic loop's in exact arithmetic; in fp64 the Gram-based scalars differ
// at rounding level, and every reference iteration count (546 / 989 / 1858 / 2449) and 16384^2's
// 10,363 is reproduced (tests/test_gpu_ca.py, bench/probe/ca_pcg_proto.py).
//
// Mapping (CDNA4): one wave64 marches a tile of TI rows x WO owned columns, 2 columns per lane.  The
// dependency radius is s in both directions: the tile loads HE >= s extra columns per side (HE even,
// so every 2-column chunk is 16-B aligned; the outermost lanes compute values that only feed the
// next level's inner lanes) and marches s extra rows above and below.  Level l of both chains is
// formed l rows behind the loaded row (a register window of the last rows of every level), so a
// loaded row's Gram products / updates happen s rows later.  Basis values at a point use only that
// point's coefficients (uniform formula when its four faces are equal, else the general one), so
// every tile computes identical values where tiles overlap.
// Fields: w, and two sets of (z, p): pass 1 and 2 of block b read set b & 1, pass 2 writes the other
// (neighbouring tiles still read the old p, z of the rows a tile writes); CaState::blk tracks b on
// the device, so captured graphs replay at any block.
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

template <int S>
struct CaShape {
  static constexpr int NB = 2 * S + 1;           // basis vectors
  static constexpr int NGD = NB * (NB + 1) / 2;  // G_D upper triangle
  static constexpr int N0 = 2 * S - 1;           // vectors of G_0: P_0..P_{S-1}, Z_0..Z_{S-2}
  static constexpr int NG0 = N0 * (N0 + 1) / 2;
  static constexpr int NQ = NGD + NG0;           // partials per tile
  static constexpr int HE = (S + 1) & ~1;        // extra columns per side (even: aligned chunks)
  static constexpr int WO = 128 - 2 * HE;        // owned columns per wave tile (2 per lane)
  static constexpr int AGES = S + 1 > 3 ? S + 1 : 3;  // rows of every level kept in the window
};

// G_0 position of basis vector i (-1: not in G_0)
template <int S>
__host__ __device__ constexpr int ca_g0_pos(int i) {
  return i < S ? i : (i > S && i < 2 * S) ? i - 1 : -1;
}

// Per-wave constants of the uniform-stencil formula: at a point whose four faces are equal,
// L~ v = A v / D - v = -(cxh (v_{i-1} + v_{i+1}) + cyh (v_{j-1} + v_{j+1})), whatever the face value.
struct CaK {
  double cxh, cyh, d_in, d_out;
};

__device__ __forceinline__ CaK ca_consts(const DevGeom& G) {
  CaK k;
  const double den = 2.0 * (G.cx + G.cy);
  k.cxh = G.cx / den;
  k.cyh = G.cy / den;
  k.d_in = diag<false>(1.0, 1.0, 1.0, 1.0, G);
  k.d_out = diag<false>(G.inv_eps, G.inv_eps, G.inv_eps, G.inv_eps, G);
  return k;
}

// Columns c0 .. c0 + 127 of a row, 2 per lane (c0 - 1 even: 16-B aligned chunks); chunks clamped to
// start <= cmax.  The row pointer is wave-uniform and every column is >= -HE, so row - 4 plus an
// unsigned byte offset keeps the SGPR-base addressing of pcg1_march's col_ptr.
template <typename T>
__device__ __forceinline__ const T* ca_col(const T* row, int c) {
  return reinterpret_cast<const T*>(reinterpret_cast<const char*>(row - 4) + unsigned(c + 4) * unsigned(sizeof(T)));
}
template <typename T>
__device__ __forceinline__ T* ca_col(T* row, int c) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(row - 4) + unsigned(c + 4) * unsigned(sizeof(T)));
}

template <typename T>
__device__ __forceinline__ void ca_load2(const T* row, int c, int cmax, T (&out)[2]) {
  vload_raw<T, 2>(ca_col(row, min(c, cmax)), out);
}

template <typename T>
__device__ __forceinline__ void ca_store2(T* row, int c, const T (&in)[2], bool all, const bool (&own)[2]) {
  typedef T V __attribute__((ext_vector_type(2)));
  if (all) {
    const V v = {in[0], in[1]};
    __builtin_nontemporal_store(v, reinterpret_cast<V*>(ca_col(row, c)));
  } else {
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (own[u]) __builtin_nontemporal_store(in[u], ca_col(row, c + u));
  }
}

// row classes of the tile columns: 2 bits per local row m (0 cut, 1 all faces inside, 2 all
// outside over the tile's loaded columns), 16 rows per word, words of tile column tj at
// tbl + tj * words; row m at bit 2 * ((m + kCaRowOff) % 16) of word (m + kCaRowOff) / 16
constexpr int kCaRowOff = 8;

__device__ __forceinline__ int ca_row_cls(const unsigned* tbl, int m) {
  const int r = m + kCaRowOff;
  const unsigned wd = ld_uniform(tbl, r >> 4);
  return int((wd >> (2 * (r & 15))) & 3u);
}

// L~ v on a lane's 2 columns at one row: centre c, rows above / below im / ip, lane neighbours'
// edge columns left / right.  ucls: the row's class (!= 0: every point of the row is uniform).
__device__ __forceinline__ void ca_lt(int ucls, int gi, const double (&c)[2], const double (&im)[2],
                                      const double (&ip)[2], double left, double right, const CaK& K,
                                      const DevGeom& G, const DevTables& Tb, const double* scol, int lane,
                                      const int (&gj)[2], double (&out)[2]) {
  const double jm[2] = {left, c[0]}, jp[2] = {c[1], right};
  if (ucls != 0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) out[u] = -__builtin_fma(K.cyh, jm[u] + jp[u], K.cxh * (im[u] + ip[u]));
    return;
  }
  const RowCo rc{gi, 0};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    double a0, a1, b0, b1;
    coef(rc, Tb, G, scol, u, lane, gj[u], a0, a1, b0, b1);
    if (a0 == a1 && a0 == b0 && a0 == b1) {
      out[u] = -__builtin_fma(K.cyh, jm[u] + jp[u], K.cxh * (im[u] + ip[u]));
    } else {
      const double av = apply_a<false>(c[u], im[u], ip[u], jm[u], jp[u], a0, a1, b0, b1, G);
      out[u] = av / diag<false>(a0, a1, b0, b1, G) - c[u];
    }
  }
}

// D at a lane's 2 columns of a row (the Gram weight)
__device__ __forceinline__ void ca_diag(int ucls, int gi, const CaK& K, const DevGeom& G, const DevTables& Tb,
                                        const double* scol, int lane, const int (&gj)[2], double (&d)[2]) {
  if (ucls != 0) {
    d[0] = d[1] = ucls == 1 ? K.d_in : K.d_out;
    return;
  }
  const RowCo rc{gi, 0};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    double a0, a1, b0, b1;
    coef(rc, Tb, G, scol, u, lane, gj[u], a0, a1, b0, b1);
    d[u] = diag<false>(a0, a1, b0, b1, G);
  }
}

template <typename T, int S, bool UPD>
struct CaRow {
  T p[2], z[2], w[2];
};

// One wave's march over one tile (see the header).  UPD = false: Gram partials into acc; true:
// p, z, w updated with the block's coefficient vectors ca / cb / cc.
template <typename T, int S, bool UPD, bool FAST>
__device__ __forceinline__ void ca_march(const DevGeom& G, const DevTables& Tb, const CaK& K,
                                         const T* __restrict__ pin, const T* __restrict__ zin, T* __restrict__ pout,
                                         T* __restrict__ zout, T* __restrict__ w, int i0, int i1, int j0, int j1,
                                         const unsigned* __restrict__ ctbl, const double* scol,
                                         double (&acc)[CaShape<S>::NQ], const double (&ca)[CaShape<S>::NB],
                                         const double (&cb)[CaShape<S>::NB], const double (&cc)[CaShape<S>::NB]) {
  using Sh = CaShape<S>;
  constexpr int NB = Sh::NB, A = Sh::AGES;
  const int64_t P = G.pitch;
  const int lane = threadIdx.x & 63;
  const int c0 = j0 - Sh::HE + 2 * lane;
  const int cmax = G.ny + 1 + (G.ny & 1);
  bool colin[2], own[2];
  int gj[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = c0 + u, g = G.gj0 + c;
    colin[u] = g >= 1 && g <= G.N - 1;
    own[u] = c >= j0 && c <= j1;
    gj[u] = min(max(g, 0), G.N);
  }
  const bool own_all = own[0] && own[1];
  const bool own_any = own[0] || own[1];
  auto grow = [&](int m) { return min(max(G.gi0 + m, 0), G.M); };
  auto interior_row = [&](int m) { return G.gi0 + m >= 1 && G.gi0 + m <= G.M - 1; };

  auto fetch = [&](int m, CaRow<T, S, UPD>& b) {
    const int mc = min(max(m, -1), G.nx + 2);  // rows -1 .. nx+2 exist
    ca_load2<T>(pin + int64_t(mc) * P, c0, cmax, b.p);
    ca_load2<T>(zin + int64_t(mc) * P, c0, cmax, b.z);
    if constexpr (UPD) {  // w of the row this step updates (S rows behind)
      const int wc = min(max(m - S, -1), G.nx + 2);
      ca_load2<T>(w + int64_t(wc) * P, c0, cmax, b.w);
    }
  };

  // windows: X[l][a] = level l at row (m - l - a) after step m
  double XP[S + 1][A][2], XZ[S][A][2];
#pragma unroll
  for (int l = 0; l <= S; ++l)
#pragma unroll
    for (int a = 0; a < A; ++a) XP[l][a][0] = XP[l][a][1] = 0.0;
#pragma unroll
  for (int l = 0; l < S; ++l)
#pragma unroll
    for (int a = 0; a < A; ++a) XZ[l][a][0] = XZ[l][a][1] = 0.0;
  int ch[S + 1];  // class of rows m, m-1, .., m-S
#pragma unroll
  for (int a = 0; a <= S; ++a) ch[a] = 0;

  const int mfirst = i0 - S, mlast = i1 + S;
  // one level of a chain: X[l][0] (row m - l) from X[l-1] rows m-l-1 .. m-l+1 and X[l-2] row m-l
  auto level = [&](auto& X, int l, int m) {
    const int r = m - l;
    const double(&ctr)[2] = X[l - 1][1];
    const double left = dpp_shift<kWaveShr1>(ctr[1], 0.0);
    const double right = dpp_shift<kWaveShl1>(ctr[0], 0.0);
    double lt[2];
    ca_lt(ch[l], grow(r), ctr, X[l - 1][2], X[l - 1][0], left, right, K, G, Tb, scol, lane, gj, lt);
    const bool rin = FAST || interior_row(r);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const double v = l == 1 ? lt[u] : __builtin_fma(2.0, lt[u], -X[l >= 2 ? l - 2 : 0][2][u]);
      X[l][0][u] = (FAST || (rin && colin[u])) ? v : 0.0;
    }
  };

  auto core = [&](int m, const CaRow<T, S, UPD>& cur) {
    // shift the windows and the class history
#pragma unroll
    for (int a = A - 1; a >= 1; --a) {
#pragma unroll
      for (int l = 0; l <= S; ++l) {
        XP[l][a][0] = XP[l][a - 1][0];
        XP[l][a][1] = XP[l][a - 1][1];
      }
#pragma unroll
      for (int l = 0; l < S; ++l) {
        XZ[l][a][0] = XZ[l][a - 1][0];
        XZ[l][a][1] = XZ[l][a - 1][1];
      }
    }
#pragma unroll
    for (int a = S; a >= 1; --a) ch[a] = ch[a - 1];
    ch[0] = ca_row_cls(ctbl, m);
    const bool rin = FAST || interior_row(m);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool in = FAST || (rin && colin[u]);
      XP[0][0][u] = in ? double(cur.p[u]) : 0.0;
      XZ[0][0][u] = in ? double(cur.z[u]) : 0.0;
    }
#pragma unroll
    for (int l = 1; l <= S; ++l) level(XP, l, m);
#pragma unroll
    for (int l = 1; l < S; ++l) level(XZ, l, m);
    // row g = m - S: every level of both chains
    const int g = m - S;
    if (g < i0 || g > i1) return;
    double Y[NB][2];
#pragma unroll
    for (int l = 0; l <= S; ++l) {
      Y[l][0] = XP[l][S - l][0];
      Y[l][1] = XP[l][S - l][1];
    }
#pragma unroll
    for (int l = 0; l < S; ++l) {
      Y[S + 1 + l][0] = XZ[l][S - l][0];
      Y[S + 1 + l][1] = XZ[l][S - l][1];
    }
    if constexpr (!UPD) {
      double d[2];
      ca_diag(ch[S], grow(g), K, G, Tb, scol, lane, gj, d);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (!(FAST || own[u])) continue;
        int q = 0;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const double dy = d[u] * Y[j][u];
#pragma unroll
          for (int i = 0; i <= j; ++i) {
            acc[q] = __builtin_fma(Y[i][u], dy, acc[q]);
            ++q;
          }
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if (ca_g0_pos<S>(j) < 0) continue;
#pragma unroll
          for (int i = 0; i <= j; ++i) {
            if (ca_g0_pos<S>(i) < 0) continue;
            acc[q] = __builtin_fma(Y[i][u], Y[j][u], acc[q]);
            ++q;
          }
        }
      }
    } else {
      T pn[2], zn[2], wn[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        double sp = 0.0, sz = 0.0, sw = double(cur.w[u]);
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          sp = __builtin_fma(ca[i], Y[i][u], sp);
          sz = __builtin_fma(cb[i], Y[i][u], sz);
          sw = __builtin_fma(cc[i], Y[i][u], sw);
        }
        pn[u] = static_cast<T>(sp);
        zn[u] = static_cast<T>(sz);
        wn[u] = static_cast<T>(sw);
      }
      if (FAST ? own_all : own_any) {
        const int64_t o = int64_t(g) * P;
        ca_store2<T>(pout + o, c0, pn, FAST || own_all, own);
        ca_store2<T>(zout + o, c0, zn, FAST || own_all, own);
        ca_store2<T>(w + o, c0, wn, FAST || own_all, own);
      }
    }
  };

  // two row buffers: step m reads one and refills the other one row ahead (unconditional loads,
  // the last row re-read past the end)
  CaRow<T, S, UPD> buf[2];
  fetch(mfirst, buf[0]);
  for (int m = mfirst; m <= mlast; m += 2) {
    fetch(min(m + 1, mlast), buf[1]);
    core(m, buf[0]);
    if (m + 1 > mlast) break;
    fetch(min(m + 2, mlast), buf[0]);
    core(m + 1, buf[1]);
  }
  if constexpr (FAST && !UPD) {  // only the lanes that own both columns summed
#pragma unroll
    for (int q = 0; q < Sh::NQ; ++q) acc[q] = own_all ? acc[q] : 0.0;
  }
}

template <int S, bool UPD>
constexpr int ca_min_waves() {
  return UPD ? 3 : 2;
}

template <typename T, int S, bool UPD>
__global__ void __launch_bounds__(64, (ca_min_waves<S, UPD>()))
k_ca_sweep(DevGeom G, DevTables Tb, T* w, T* z0, T* z1, T* p0, T* p1, double* __restrict__ partials,
           const PcgState* St, const CaState* C, int TI, int tiles_j, const unsigned* __restrict__ ctbl,
           int cwords) {
  using Sh = CaShape<S>;
  constexpr int NB = Sh::NB;
  typedef const __attribute__((address_space(4))) PcgState CPS;
  typedef const __attribute__((address_space(4))) CaState CCS;
  const int done = ((CPS*)St)->done;    // NOLINT
  const long long blk = ((CCS*)C)->blk;  // NOLINT
  const int nupd = ((CCS*)C)->nupd;      // NOLINT
  double ca[NB], cb[NB], cc[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    ca[i] = UPD ? ((CCS*)C)->coef[0][i] : 0.0;  // NOLINT
    cb[i] = UPD ? ((CCS*)C)->coef[1][i] : 0.0;  // NOLINT
    cc[i] = UPD ? ((CCS*)C)->coef[2][i] : 0.0;  // NOLINT
  }
  if (UPD ? nupd == 0 : done != 0) return;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int ti = id / tiles_j, tj = id - ti * tiles_j;
  const int i0 = 1 + ti * TI, i1 = min(i0 + TI - 1, G.nx);
  const int j0 = 1 + tj * Sh::WO, j1 = min(j0 + Sh::WO - 1, G.ny);
  // pass 1 reads set blk & 1; pass 2 runs after the reduction advanced blk: reads set (blk - 1) & 1
  const int in = int((UPD ? blk - 1 : blk) & 1);
  const T* pin = in ? p1 : p0;
  const T* zin = in ? z1 : z0;
  T* pout = in ? p0 : p1;
  T* zout = in ? z0 : z1;
  const CaK K = ca_consts(G);
  const int lane = threadIdx.x & 63;
  // column constants of the lane's columns for the cut rows (coef's LDS slots)
  __shared__ double scol[4 * 2 * 64];
  {
    const int c0 = j0 - Sh::HE + 2 * lane;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const ColConst cc0 = load_col(Tb, min(max(G.gj0 + c0 + u, 0), G.N));
      scol[(4 * u) * 64 + lane] = cc0.ylo;
      scol[(4 * u + 1) * 64 + lane] = cc0.yhi;
      scol[(4 * u + 2) * 64 + lane] = cc0.rh0;
      scol[(4 * u + 3) * 64 + lane] = cc0.rh1;
    }
  }
  const unsigned* tbl = ctbl + int64_t(tj) * cwords;
  const bool fast = j1 == j0 + Sh::WO - 1 && G.gi0 + i0 - S >= 1 && G.gi0 + i1 + S <= G.M - 1 &&
                    G.gj0 + j0 - Sh::HE >= 1 && G.gj0 + j0 - Sh::HE + 127 <= G.N - 1;
  double acc[Sh::NQ];
#pragma unroll
  for (int q = 0; q < Sh::NQ; ++q) acc[q] = 0.0;
  if (fast)
    ca_march<T, S, UPD, true>(G, Tb, K, pin, zin, pout, zout, w, i0, i1, j0, j1, tbl, scol, acc, ca, cb, cc);
  else
    ca_march<T, S, UPD, false>(G, Tb, K, pin, zin, pout, zout, w, i0, i1, j0, j1, tbl, scol, acc, ca, cb, cc);
  if constexpr (!UPD) {
#pragma unroll
    for (int q = 0; q + 1 < Sh::NQ; q += 2) wave_sum2_mfma(acc[q], acc[q + 1]);
    if constexpr (Sh::NQ & 1) acc[Sh::NQ - 1] = wave_sum_mfma(acc[Sh::NQ - 1]);
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < Sh::NQ; ++q) partials[int64_t(Sh::NQ) * id + q] = acc[q];
    }
  }
}

// Row classes of every tile column (one thread per 16-row word): 2 bits per local row, over the
// columns the tile loads, as pcg1's k_pcg1_tile_classes.
__global__ void k_ca_row_classes(DevGeom G, DevTables Tb, int he, int wo, int tiles_j, int cwords, unsigned* out) {
  const int t = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (t >= tiles_j * cwords) return;
  const int tj = t / cwords, wd = t - tj * cwords;
  const int j0 = 1 + tj * wo;
  const int gjlo = max(G.gj0 + j0 - he, 0), gjhi = min(G.gj0 + j0 - he + 127, G.N);
  unsigned bits = 0;
  for (int q = 0; q < 16; ++q) {
    const int m = wd * 16 + q - kCaRowOff;
    const int gi = min(max(G.gi0 + m, 0), G.M);
    RowConst rc;
    for (int k = 0; k < 4; ++k) {
      rc.ca0[k] = Tb.acls[4 * gi + k];
      rc.ca1[k] = Tb.acls[4 * (gi + 1) + k];
      rc.cb[k] = Tb.bcls[4 * gi + k];
    }
    bits |= unsigned(row_class(rc, gjlo, gjhi)) << (2 * q);
  }
  out[t] = bits;
}

// z^0 = D^-1 r^0 in place and p^0 = z^0 (set 0): the state the first block starts from.
template <typename T>
__global__ void __launch_bounds__(256) k_ca_init(DevGeom G, DevTables Tb, T* z, T* p) {
  const int lj = 1 + int(blockIdx.x * blockDim.x + threadIdx.x);
  const int li = 1 + int(blockIdx.y);
  if (lj > G.ny) return;
  const int gi = G.gi0 + li, gj = G.gj0 + lj;
  const double a0 = coef_a(Tb, G, gi, gj), a1 = coef_a(Tb, G, gi + 1, gj);
  const double b0 = coef_b(Tb, G, gi, gj), b1 = coef_b(Tb, G, gi, gj + 1);
  const int64_t o = int64_t(li) * G.pitch + lj;
  const double v = dirichlet(G, gi, gj) ? 0.0 : double(z[o]) / diag<false>(a0, a1, b0, b1, G);
  z[o] = static_cast<T>(v);
  p[o] = static_cast<T>(v);
}

// The block's scalars from the reduced Gram sums t (raw): the s iterations of the classic loop on
// the coefficient vectors, in the classic order of tests (max_iter, breakdown guard, stop test).
template <int S>
__device__ void ca_finish(const double* t, double h, double wdiff, int nmax, PcgState* St, CaState* C) {
  using Sh = CaShape<S>;
  constexpr int NB = Sh::NB;
  if (St->done) {
    C->nupd = 0;
    return;
  }
  double GD[NB][NB], G0[NB][NB];
  {
    int q = 0;
    for (int j = 0; j < NB; ++j)
      for (int i = 0; i <= j; ++i) {
        GD[i][j] = GD[j][i] = t[q++] * h;
      }
    for (int j = 0; j < NB; ++j)
      for (int i = 0; i < NB; ++i) G0[i][j] = 0.0;
    for (int j = 0; j < NB; ++j) {
      if (ca_g0_pos<S>(j) < 0) continue;
      for (int i = 0; i <= j; ++i) {
        if (ca_g0_pos<S>(i) < 0) continue;
        G0[i][j] = G0[j][i] = t[q++] * wdiff;
      }
    }
  }
  auto quad = [&](const double (&M)[NB][NB], const double* x, const double* y) {
    double s = 0.0;
    for (int i = 0; i < NB; ++i) {
      double r = 0.0;
      for (int j = 0; j < NB; ++j) r = __builtin_fma(M[i][j], y[j], r);
      s = __builtin_fma(x[i], r, s);
    }
    return s;
  };
  // L Y = Y T: L P_0 = P_0 + P_1, L P_i = P_i + (P_{i-1} + P_{i+1}) / 2; the same for Z
  auto shiftT = [&](const double* x, double* y) {
    for (int base = 0; base <= S + 1; base += S + 1) {
      const int n = base == 0 ? S + 1 : S;
      for (int r = 0; r < n; ++r) {
        double v = x[base + r];
        if (r >= 1) v += (r == 1 ? 1.0 : 0.5) * x[base + r - 1];
        if (r + 1 < n) v += 0.5 * x[base + r + 1];
        y[base + r] = v;
      }
    }
  };
  double a[NB], b[NB], c[NB], Ta[NB];
  for (int i = 0; i < NB; ++i) a[i] = b[i] = c[i] = 0.0;
  a[0] = 1.0;
  b[S + 1] = 1.0;
  double g = GD[S + 1][S + 1];
  const long long k = St->it;
  const bool weighted = St->norm == int(Norm::kWeighted);
  int nupd = 0, status = -1;
  long long iters = 0;
  bool nan = !(g == g);
  double diff = St->diff;
  for (int j = 0; j < S && j < nmax; ++j) {
    const long long kk = k + j + 1;
    if (nan) {
      status = int(Status::kBreakdown);
      iters = kk;
      break;
    }
    if (kk > St->max_iter) {
      status = int(Status::kMaxIter);
      iters = kk - 1;
      break;
    }
    shiftT(a, Ta);
    const double den = quad(GD, a, Ta);
    if (!(den == den) || (weighted ? fabs(den) < St->bd_tol : den < St->bd_tol)) {
      status = int(Status::kBreakdown);
      iters = kk;
      nan = !(den == den);
      break;
    }
    const double alpha = g / den;
    for (int i = 0; i < NB; ++i) c[i] = __builtin_fma(alpha, a[i], c[i]);
    nupd = j + 1;
    const double pp = quad(G0, a, a);
    diff = fabs(alpha) * sqrt(pp);
    if (!(diff == diff)) {
      status = int(Status::kBreakdown);
      iters = kk;
      nan = true;
      break;
    }
    if (diff < St->delta) {
      status = int(Status::kConverged);
      iters = kk;
      break;
    }
    for (int i = 0; i < NB; ++i) b[i] = __builtin_fma(-alpha, Ta[i], b[i]);
    const double gn = quad(GD, b, b);
    const double beta = gn / g;
    for (int i = 0; i < NB; ++i) a[i] = __builtin_fma(beta, a[i], b[i]);
    g = gn;
    nan = !(g == g);
  }
  for (int i = 0; i < NB; ++i) {
    C->coef[0][i] = a[i];
    C->coef[1][i] = b[i];
    C->coef[2][i] = c[i];
  }
  C->nupd = nupd;
  if (nupd > 0) C->blk += 1;
  St->it = k + nupd;
  St->diff = diff;
  if (status >= 0) {
    St->iters = iters;
    St->status = status;
    if (nan) St->nan_flag = 1;
    St->done = 1;
  }
}

// Deterministic reduction of the pass-1 partials (n tiles x NQ) + the scalar finish: blocks sum
// contiguous tile ranges (thread-strided, then waves in order), publish NQ chunk sums, and the last
// block to arrive (ticket) sums the chunks in block order and runs ca_finish.  Hand-off as k_reduce_n.
template <int S>
__global__ void __launch_bounds__(256)
k_ca_reduce(const double* __restrict__ part, int n, double h, double wdiff, int nmax, PcgState* St, CaState* C,
            double* chunk, long long* progress) {
  constexpr int NQ = CaShape<S>::NQ;
  __shared__ double lds[NQ][256 / kWave];
  __shared__ double tot[NQ];
  __shared__ int last;
  if (St->done) {
    if (blockIdx.x == 0 && threadIdx.x == 0) C->nupd = 0;
    return;
  }
  const int nb = int(gridDim.x);
  const int lo = int(int64_t(n) * blockIdx.x / nb);
  const int hi = int(int64_t(n) * (blockIdx.x + 1) / nb);
  double s[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) s[q] = 0.0;
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
  if (nb == 1) {
    if (threadIdx.x == 0) {
      for (int q = 0; q < NQ; ++q) tot[q] = (lds[q][0] + lds[q][1]) + (lds[q][2] + lds[q][3]);
      ca_finish<S>(tot, h, wdiff, nmax, St, C);
      if (progress) __hip_atomic_store(progress, St->it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  if (threadIdx.x == 0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      st_publish(chunk + NQ * blockIdx.x + q, (lds[q][0] + lds[q][1]) + (lds[q][2] + lds[q][3]));
    last = ticket_arrive_last(&C->ticket, nb);
  }
  __syncthreads();
  if (!last || threadIdx.x >= kWave) return;  // wave 0 of the last block finishes (full EXEC)
  const int l = int(threadIdx.x);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const double v = l < nb ? ld_published(chunk + NQ * l + q) : 0.0;
    const double sum = wave_sum_mfma(v);
    if (l == 0) tot[q] = sum;
  }
  if (l == 0) {
    ca_finish<S>(tot, h, wdiff, nmax, St, C);
    if (progress) __hip_atomic_store(progress, St->it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    C->ticket = 0u;  // re-arm for the next launch (stream order makes this visible to it)
  }
}

}  // namespace

CaTiles make_ca_tiles(const DevGeom& G, int s, int rows) {
  PMX_CHECK(s == 2 || s == 3, "s-step PCG: s must be 2 or 3");
  CaTiles t;
  t.s = s;
  t.he = (s + 1) & ~1;
  t.wo = 128 - 2 * t.he;
  t.tiles_j = (G.ny + t.wo - 1) / t.wo;
  if (rows <= 0) {
    // tall tiles keep the 2s re-marched halo rows cheap (their basis levels are recomputed); shorter
    // only when the grid has too few tiles to fill the chip a few times over
    rows = 64;
    while (rows > 8 && int64_t((G.nx + rows - 1) / rows) * t.tiles_j < 4096) rows /= 2;
  }
  PMX_CHECK(rows >= 1 && rows <= 4096, "s-step PCG: tile rows must be in [1, 4096]");
  t.rows = rows;
  t.tiles_i = (G.nx + rows - 1) / rows;
  t.cwords = (G.nx + 2 * s + 2 * kCaRowOff + 15) / 16 + 1;
  return t;
}

int ca_nq(int s) { return s == 2 ? CaShape<2>::NQ : CaShape<3>::NQ; }

void ca_build_classes(const DevGeom& G, const DevTables& Tb, const CaTiles& t, unsigned* tbl, hipStream_t s) {
  const int n = t.tiles_j * t.cwords;
  hipLaunchKernelGGL(k_ca_row_classes, dim3((n + 255) / 256), dim3(256), 0, s, G, Tb, t.he, t.wo, t.tiles_j,
                     t.cwords, tbl);
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_ca_init(const DevGeom& G, const DevTables& Tb, T* z, T* p, hipStream_t s) {
  PMX_CHECK(G.nx <= 65535, "k_ca_init: grid.y limit");
  hipLaunchKernelGGL(k_ca_init<T>, dim3((G.ny + 255) / 256, G.nx), dim3(256), 0, s, G, Tb, z, p);
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_ca_sweep(const DevGeom& G, const DevTables& Tb, T* w, T* z0, T* z1, T* p0, T* p1, double* partials,
                     const PcgState* S, const CaState* C, const CaTiles& t, bool upd, hipStream_t s) {
  PMX_CHECK(G.nb == 0, "s-step PCG runs undecomposed grids");
  PMX_CHECK(t.tbl != nullptr, "s-step PCG: row-class table missing");
  const int n = t.ntiles();
#define PMX_CA(SS)                                                                                              \
  do {                                                                                                          \
    if (upd)                                                                                                    \
      hipLaunchKernelGGL((k_ca_sweep<T, SS, true>), dim3(n), dim3(64), 0, s, G, Tb, w, z0, z1, p0, p1, partials, \
                         S, C, t.rows, t.tiles_j, t.tbl, t.cwords);                                             \
    else                                                                                                        \
      hipLaunchKernelGGL((k_ca_sweep<T, SS, false>), dim3(n), dim3(64), 0, s, G, Tb, w, z0, z1, p0, p1,         \
                         partials, S, C, t.rows, t.tiles_j, t.tbl, t.cwords);                                   \
  } while (0)
  if (t.s == 2) PMX_CA(2);
  else PMX_CA(3);
#undef PMX_CA
  HIP_CHECK(hipGetLastError());
}

void launch_ca_reduce(const double* partials, int n, int s_, double h, double wdiff, int nmax, PcgState* S,
                      CaState* C, double* chunk, hipStream_t s, long long* progress) {
  PMX_CHECK(nmax >= 1 && nmax <= s_, "s-step PCG: a block runs 1..s iterations");
  const int nb = std::max(1, std::min(kReduceMaxBlocks, n / 256));
  if (s_ == 2)
    hipLaunchKernelGGL(k_ca_reduce<2>, dim3(nb), dim3(256), 0, s, partials, n, h, wdiff, nmax, S, C, chunk, progress);
  else
    hipLaunchKernelGGL(k_ca_reduce<3>, dim3(nb), dim3(256), 0, s, partials, n, h, wdiff, nmax, S, C, chunk, progress);
  HIP_CHECK(hipGetLastError());
}

template void launch_ca_init<double>(const DevGeom&, const DevTables&, double*, double*, hipStream_t);
template void launch_ca_sweep<double>(const DevGeom&, const DevTables&, double*, double*, double*, double*, double*,
                                      double*, const PcgState*, const CaState*, const CaTiles&, bool, hipStream_t);

}  // namespace pmx
