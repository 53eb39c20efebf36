// s-step Jacobi-PCG ("ca", communication-avoiding CG): s iterations per TWO streaming passes and one
// reduction, instead of s single-pass sweeps (pcg1_kernels.hip) and s reductions.
//
// Same iteration as the reference (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:847-943; z = D^-1 r,
// alpha = (r, z) / (A p, p), w += alpha p, r -= alpha A p, beta = (r', z') / (r, z), p = z' + beta p,
// stop when ||w^{k+1} - w^k|| = |alpha| ||p|| < delta), regrouped by blocks of s iterations.  In
// the D-inner product <x, y>_D = x^T D y the preconditioned operator L = D^-1 A is self-adjoint, and
// after j < s iterations of a block p, z = D^-1 r and w - w_k lie in the span of the Krylov basis
//   Y = [P_0 .. P_s, Z_0 .. Z_{s-1}],  P_i = T_i(L~) p_k,  Z_i = T_i(L~) z_k,  L~ = L - I
// (Chebyshev polynomials T_i: L~ has its spectrum in (-1, 1) -- Gershgorin on the M-matrix A -- so
// the basis stays well conditioned; a monomial basis would not).  With p = Y a, z = Y b,
// w - w_k = Y c and L Y = Y T (T: the Chebyshev three-term recurrence, exact in the columns that stay
// in the basis), alpha's numerator and denominator come from one Gram matrix:
//   (r, z) = b^T G b,   (A p, p) = a^T G T a,   G = Y^T D Y,
// and G itself from 6s products: the Chebyshev product rule T_a T_b = (T_{a+b} + T_{|a-b|}) / 2 and
// the D-self-adjointness of L~ give <P_a, P_b>_D = (mu_{a+b} + mu_{|a-b|}) / 2 with
// mu_m = <T_m(L~) p, p>_D (likewise nu for z, rho for <T_m p, z>_D); mu_0..mu_s are products with P_0,
// the higher moments come from <P_i, P_j> with i + j = m (s = 3: 18 products for 28 entries).
// The stop test needs the plain norm ||p_{k+j}||, which has no such symmetry: pass 2 forms
// p_{k+j} = Y a_j explicitly and sums its squares, and the test of a block's iterations runs in the
// NEXT reduction (or in a check after the last block of a batch).  A stop at iteration j < n of a
// block rewinds w to w_k + Y c_{j+1} with one more pass over the block's inputs, which are still intact
// (the next pass 2 has not overwritten that set).  So a block is:
//   pass 1 (k_ca_sweep<.., false>): per tile, the basis on the fly from p_k, z_k (radius s) and the
//          6s Gram products;
//   reduce (k_ca_reduce): the partials summed in a fixed order, then ONE lane runs the pending stop
//          test of the previous block and the s iterations of this one on the coefficient vectors
//          (alpha, beta, the breakdown guard, max_iter) and leaves a_n, b_n, c_n in CaState;
//   pass 2 (k_ca_sweep<.., true>): the basis again, p = Y a_n, z = Y b_n, w += Y c_n, ||Y a_j||^2.
// HBM traffic per block: pass 1 reads p, z (16 B/pt), pass 2 reads p, z, w and writes them (48 B/pt):
// 64 B/pt for s iterations -- 21.3 B/pt/iteration at s = 3 against pcg1's 37.3.  The price is
// arithmetic: 2 x (2s - 1) stencils and ~6s Gram FMAs per point and block.
// The iterates equal the classic loop's in exact arithmetic; in fp64 the Gram-based scalars differ
// at rounding level, and every reference iteration count (546 / 989 / 1858 / 2449) and 16384^2's
// 10,363 is reproduced (tests/test_gpu_ca.py; models/sstep_pcg.py is the PyTorch statement).
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
  static constexpr int NB = 2 * S + 1;     // basis vectors
  static constexpr int NQ = 6 * S;         // Gram products per tile (pass 1)
  static constexpr int NN = S;             // ||p_{k+j}||^2 partials per tile (pass 2)
  static constexpr int HE = (S + 1) & ~1;  // extra columns per side (even: aligned chunks)
  static constexpr int WO = 128 - 2 * HE;  // owned columns per wave tile (2 per lane)
  static constexpr int AGES = S + 1 > 3 ? S + 1 : 3;  // rows of every level kept in the window
};

// Gram product q = <Y_i, Y_j>_D (basis index: P_m = m, Z_m = S + 1 + m), in the order
//   mu:  <P_m, P_0> m = 0..S, then <P_{(m+1)/2}, P_{m/2}> m = S+1..2S
//   nu:  <Z_m, Z_0> m = 0..S-1, then <Z_{(m+1)/2}, Z_{m/2}> m = S..2S-2
//   rho: <P_m, Z_0> m = 0..S, then <P_S, Z_b> b = 1..S-1
template <int S>
__host__ __device__ constexpr int ca_prod_i(int q) {
  if (q <= 2 * S) return q <= S ? q : (q + 1) / 2;
  q -= 2 * S + 1;
  if (q <= 2 * S - 2) return S + 1 + (q <= S - 1 ? q : (q + 1) / 2);
  q -= 2 * S - 1;
  return q <= S ? q : S;
}
template <int S>
__host__ __device__ constexpr int ca_prod_j(int q) {
  if (q <= 2 * S) return q <= S ? 0 : q / 2;
  q -= 2 * S + 1;
  if (q <= 2 * S - 2) return S + 1 + (q <= S - 1 ? 0 : q / 2);
  q -= 2 * S - 1;
  return q <= S ? S + 1 : S + 1 + (q - S);
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
// start <= cmax.  The row pointer is wave-uniform and every column is >= -HE >= -8, so row - 8 plus
// an unsigned byte offset keeps the SGPR-base addressing of pcg1_march's col_ptr.
template <typename T>
__device__ __forceinline__ const T* ca_col(const T* row, int c) {
  return reinterpret_cast<const T*>(reinterpret_cast<const char*>(row - 8) + unsigned(c + 8) * unsigned(sizeof(T)));
}
template <typename T>
__device__ __forceinline__ T* ca_col(T* row, int c) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(row - 8) + unsigned(c + 8) * unsigned(sizeof(T)));
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

// Face coefficients of the rows the ellipse cuts come from two precomputed fields (k_ca_faces:
// fa = a(gi, gj), fb = b(gi, gj) at every local node, pitch as the solution fields): four vector loads
// per lane instead of rebuilding the faces from the 1D tables, which would keep the row constants
// and the clip arithmetic live next to the register windows (the kernel spilled with it).
struct CaFaces {
  const double* a;
  const double* b;
  int gh;  // ghost rows (and, on 2-D blocks, columns) on each side of the fields: 2 undecomposed, s or 2s
};

// The last odd column a lane's 2-column load may start at (loads clamp to it; column 1 is 16-B
// aligned, so pairs start at odd columns): the first odd column >= ny + 1 (the Dirichlet column) --
// or, with a neighbour across y-hi (2-D blocks), the one whose pair reaches the last ghost column
// ny + gh.  Lanes past it hold clamped copies; they only feed columns beyond the owned ones.
__device__ __forceinline__ int ca_cmax(const DevGeom& G, const CaFaces& F) {
  return (G.nb & kNbYhi) ? ((G.ny + F.gh - 1) | 1) : G.ny + 1 + (G.ny & 1);
}

// the coefficients of a lane's 2 columns at local row r (clamped into the allocated rows; rows
// outside the grid only feed masked values)
__device__ __forceinline__ void ca_faces(const CaFaces& F, const DevGeom& G, int r, int c0, int cmax,
                                         double (&a0)[2], double (&a1)[2], double (&b0)[2], double (&b1)[2]) {
  const int rc = min(max(r, 1 - F.gh), G.nx + F.gh - 1);
  const double* ra = F.a + int64_t(rc) * G.pitch;
  const double* rb = F.b + int64_t(rc) * G.pitch;
  vload<double, 2>(ca_col(ra, min(c0, cmax)), a0);
  vload<double, 2>(ca_col(ra + G.pitch, min(c0, cmax)), a1);
  vload<double, 2>(ca_col(rb, min(c0, cmax)), b0);
  b1[0] = b0[1];
  b1[1] = *ca_col(rb, min(c0 + 2, cmax + 1));
}

// L~ v on a lane's 2 columns at one row: centre c, rows above / below im / ip, lane neighbours'
// edge columns left / right.  ucls: the row's class (!= 0: every point of the row is uniform).
__device__ __forceinline__ void ca_lt(int ucls, int r, const double (&c)[2], const double (&im)[2],
                                      const double (&ip)[2], double left, double right, const CaK& K,
                                      const DevGeom& G, const CaFaces& F, int c0, int cmax, double (&out)[2]) {
  const double jm[2] = {left, c[0]}, jp[2] = {c[1], right};
  if (ucls != 0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) out[u] = -__builtin_fma(K.cyh, jm[u] + jp[u], K.cxh * (im[u] + ip[u]));
    return;
  }
  double a0[2], a1[2], b0[2], b1[2];
  ca_faces(F, G, r, c0, cmax, a0, a1, b0, b1);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (a0[u] == a1[u] && a0[u] == b0[u] && a0[u] == b1[u]) {
      out[u] = -__builtin_fma(K.cyh, jm[u] + jp[u], K.cxh * (im[u] + ip[u]));
    } else {
      const double av = apply_a<false>(c[u], im[u], ip[u], jm[u], jp[u], a0[u], a1[u], b0[u], b1[u], G);
      out[u] = av / diag<false>(a0[u], a1[u], b0[u], b1[u], G) - c[u];
    }
  }
}

// D at a lane's 2 columns of a row (the Gram weight)
__device__ __forceinline__ void ca_diag(int ucls, int r, const CaK& K, const DevGeom& G, const CaFaces& F, int c0,
                                        int cmax, double (&d)[2]) {
  if (ucls != 0) {
    d[0] = d[1] = ucls == 1 ? K.d_in : K.d_out;
    return;
  }
  double a0[2], a1[2], b0[2], b1[2];
  ca_faces(F, G, r, c0, cmax, a0, a1, b0, b1);
#pragma unroll
  for (int u = 0; u < 2; ++u) d[u] = diag<false>(a0[u], a1[u], b0[u], b1[u], G);
}

// Wave lane shift of a double with zero fill at the edge lane (DPP bound_ctrl: no old value to set up)
template <int CTRL>
__device__ __forceinline__ double dpp_shift0(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp(int(b), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(int(b >> 32), CTRL, 0xf, 0xf, true);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}

template <typename T, int S, bool UPD>
struct CaRow {
  T p[2], z[2], w[2];
};

// One wave's march over one tile (see the header).  UPD = false: the Gram products into acc; true:
// p, z, w updated with the block's coefficient vectors ca / cb / cc and ||Y pa_j||^2 into acc
// (REW: w += Y cc only).
template <typename T, int S, bool UPD, bool FAST, int PF, bool REW, int DPF = 0, int HE = CaShape<S>::HE>
__device__ __forceinline__ void ca_march(const DevGeom& G, const DevTables& Tb, const CaK& K,
                                         const T* __restrict__ pin, const T* __restrict__ zin, T* __restrict__ pout,
                                         T* __restrict__ zout, T* __restrict__ w, int i0, int i1, int j0, int j1,
                                         const unsigned* __restrict__ ctbl, const CaFaces& F,
                                         double (&acc)[CaShape<S>::NQ], const double (&ca)[CaShape<S>::NB],
                                         const double (&cb)[CaShape<S>::NB], const double (&cc)[CaShape<S>::NB],
                                         const double (&pa)[S][CaShape<S>::NB], double* dring = nullptr) {
  using Sh = CaShape<S>;
  constexpr int NB = Sh::NB, A = Sh::AGES;
  const int64_t P = G.pitch;
  const int lane = threadIdx.x & 63;
  const int c0 = j0 - HE + 2 * lane;
  const int cmax = ca_cmax(G, F);
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
    const int mc = min(max(m, 1 - F.gh), G.nx + F.gh);  // the allocated rows
    ca_load2<T>(pin + int64_t(mc) * P, c0, cmax, b.p);
    ca_load2<T>(zin + int64_t(mc) * P, c0, cmax, b.z);
    if constexpr (UPD) {  // w of the row this step updates (S rows behind)
      const int wc = min(max(m - S, 1 - F.gh), G.nx + F.gh);
      ca_load2<T>(w + int64_t(wc) * P, c0, cmax, b.w);
    }
  };

  // windows: level l at row r sits in slot (r - mfirst) & 3 of X[l] (every level keeps at most 4
  // consecutive rows alive), and the march is unrolled by 4, so every slot index is a compile-time
  // constant and no row is ever moved between registers
  static_assert(Sh::AGES <= 4, "ca_march: window deeper than 4 rows");
  double XP[S + 1][4][2], XZ[S][4][2];
#pragma unroll
  for (int l = 0; l <= S; ++l)
#pragma unroll
    for (int a = 0; a < 4; ++a) XP[l][a][0] = XP[l][a][1] = 0.0;
#pragma unroll
  for (int l = 0; l < S; ++l)
#pragma unroll
    for (int a = 0; a < 4; ++a) XZ[l][a][0] = XZ[l][a][1] = 0.0;
  int ch[4] = {0, 0, 0, 0};  // row classes, same slots

  const int mfirst = i0 - S, mlast = i1 + S;
  // one level of a chain at step m (slot q = (m - mfirst) & 3): level l at row m - l from level l-1
  // at rows m-l-1 .. m-l+1 and level l-2 at row m-l
  auto level = [&](auto& X, auto lc, auto qc, int m) {
    constexpr int l = decltype(lc)::value, q = decltype(qc)::value;
    constexpr int sc = (q - l) & 3, sm = (q - l - 1) & 3, sp = (q - l + 1) & 3;
    const int r = m - l;
    const double(&ctr)[2] = X[l - 1][sc];
    const double left = dpp_shift0<kWaveShr1>(ctr[1]);
    const double right = dpp_shift0<kWaveShl1>(ctr[0]);
    double lt[2];
    ca_lt(ch[sc], r, ctr, X[l - 1][sm], X[l - 1][sp], left, right, K, G, F, c0, cmax, lt);
    const bool rin = FAST || interior_row(r);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      double v;
      if constexpr (l == 1) v = lt[u];
      else v = __builtin_fma(2.0, lt[u], -X[l - 2][sc][u]);
      X[l][sc][u] = (FAST || (rin && colin[u])) ? v : 0.0;
    }
  };

  auto core = [&](auto qc, int m, const CaRow<T, S, UPD>& cur) {
    constexpr int q = decltype(qc)::value;
    ch[q] = ca_row_cls(ctbl, m);
    const bool rin = FAST || interior_row(m);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool in = FAST || (rin && colin[u]);
      XP[0][q][u] = in ? double(cur.p[u]) : 0.0;
      XZ[0][q][u] = in ? double(cur.z[u]) : 0.0;
    }
    static_for_while<S>([&](auto l1) {
      level(XP, std::integral_constant<int, decltype(l1)::value + 1>{}, qc, m);
      return true;
    });
    static_for_while<S - 1>([&](auto l1) {
      level(XZ, std::integral_constant<int, decltype(l1)::value + 1>{}, qc, m);
      return true;
    });
    // row g = m - S: every level of both chains
    const int g = m - S;
    if (g < i0 || g > i1) return;
    constexpr int sg = (q - S) & 3;
    double Y[NB][2];
#pragma unroll
    for (int l = 0; l <= S; ++l) {
      Y[l][0] = XP[l][sg][0];
      Y[l][1] = XP[l][sg][1];
    }
#pragma unroll
    for (int l = 0; l < S; ++l) {
      Y[S + 1 + l][0] = XZ[l][sg][0];
      Y[S + 1 + l][1] = XZ[l][sg][1];
    }
    if constexpr (!UPD) {
      double d[2];
      ca_diag(ch[sg], g, K, G, F, c0, cmax, d);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (!(FAST || own[u])) continue;
#pragma unroll
        for (int q = 0; q < Sh::NQ; ++q)  // the compiler shares d * Y_j between products
          acc[q] = __builtin_fma(Y[ca_prod_i<S>(q)][u], d[u] * Y[ca_prod_j<S>(q)][u], acc[q]);
      }
    } else {
      T pn[2], zn[2], wn[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        double sp = 0.0, sz = 0.0, sw = double(cur.w[u]);
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          if constexpr (!REW) {
            sp = __builtin_fma(ca[i], Y[i][u], sp);
            sz = __builtin_fma(cb[i], Y[i][u], sz);
          }
          sw = __builtin_fma(cc[i], Y[i][u], sw);
        }
        pn[u] = static_cast<T>(sp);
        zn[u] = static_cast<T>(sz);
        wn[u] = static_cast<T>(sw);
        if constexpr (!REW) {
          // ||p_{k+j}||^2, p_{k+j} = Y a_j: a_j lives on P_0..P_j, Z_0..Z_{j-1} (a_0 = e_0)
          if (FAST || own[u]) {
            acc[0] = __builtin_fma(Y[0][u], Y[0][u], acc[0]);
#pragma unroll
            for (int j = 1; j < S; ++j) {
              double v = 0.0;
#pragma unroll
              for (int i = 0; i <= j; ++i) v = __builtin_fma(pa[j][i], Y[i][u], v);
#pragma unroll
              for (int i = 0; i < j; ++i) v = __builtin_fma(pa[j][S + 1 + i], Y[S + 1 + i][u], v);
              acc[j] = __builtin_fma(v, v, acc[j]);
            }
          }
        }
      }
      if (FAST ? own_all : own_any) {
        const int64_t o = int64_t(g) * P;
        if constexpr (!REW) {
          ca_store2<T>(pout + o, c0, pn, FAST || own_all, own);
          ca_store2<T>(zout + o, c0, zn, FAST || own_all, own);
        }
        ca_store2<T>(w + o, c0, wn, FAST || own_all, own);
      }
    }
  };

  // PF + 1 row buffers: step m reads one and refills the one step m - 1 consumed with row m + PF
  // (unconditional loads, the last row re-read past the end).  Unrolled by 4 = the window depth
  // (and a multiple of PF + 1), so the window shifts and the ring are register renames, not moves.
  static_assert(PF == 1 || PF == 3, "ca_march: prefetch depth 1 or 3");
  if constexpr (DPF > 0) {
    // LDS-DMA ring (pass 1 of fp64 FAST tiles): row mfirst + t in slot t & 3, DPF = 4 rows ahead, no
    // VGPR buffers.  global_load_lds_dwordx4 is invisible to hipcc (pcg1_march.hpp: dma16), so the
    // march counts vmcnt itself: pass 1 issues no other vector memory operation in the loop (row
    // classes and cut-row constants are scalar / LDS loads), so before reading row m exactly the
    // DMAs of rows m+1 .. m+3 may still be in flight.
    static_assert(DPF == 4 && !UPD && FAST && sizeof(T) == 8, "ca_march: LDS-DMA for pass 1 FAST tiles, 4 rows");
    const unsigned voff = unsigned(c0 + 4) * 8u;  // bytes from row - 4 (ca_col's unsigned form)
    const unsigned lds0 = unsigned(reinterpret_cast<uintptr_t>(dring));
    auto dma_row = [&](int m, int slot) {
      const unsigned l = lds0 + unsigned(slot) * 2048u;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's previous ds_reads have returned
      dma16(pin + int64_t(m) * P - 4, voff, l);
      dma16(zin + int64_t(m) * P - 4, voff, l + 1024u);
    };
    typedef double d2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int q = 0; q < DPF; ++q) dma_row(min(mfirst + q, mlast), q);
    bool more = true;
    for (int m = mfirst; more && m <= mlast; m += 4) {
      more = static_for_while<4>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        if (m + q > mlast) return false;
        wait_vmcnt<(DPF - 1) * 2>();
        const double* sl = dring + q * 256;
        CaRow<T, S, UPD> cur;
        const d2 pv = *reinterpret_cast<const d2*>(sl + 2 * lane);
        const d2 zv = *reinterpret_cast<const d2*>(sl + 128 + 2 * lane);
        cur.p[0] = pv.x;
        cur.p[1] = pv.y;
        cur.z[0] = zv.x;
        cur.z[1] = zv.y;
        dma_row(min(m + q + DPF, mlast), q);
        core(qc, m + q, cur);
        return true;
      });
    }
    wait_vmcnt<0>();  // no DMA may land after the wave has moved on
    if constexpr (FAST) {
#pragma unroll
      for (int q = 0; q < Sh::NQ; ++q) acc[q] = own_all ? acc[q] : 0.0;
    }
    return;
  }
  constexpr int NBUF = PF + 1;
  CaRow<T, S, UPD> buf[NBUF];
#pragma unroll
  for (int q = 0; q < PF; ++q) fetch(min(mfirst + q, mlast), buf[q]);
  bool more = true;
  for (int m = mfirst; more && m <= mlast; m += 4) {
    more = static_for_while<4>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      if (m + q > mlast) return false;
      fetch(min(m + q + PF, mlast), buf[(q + PF) % NBUF]);
      core(qc, m + q, buf[q % NBUF]);
#ifdef PMX_CA_SCHED_BARRIER
      __builtin_amdgcn_sched_barrier(0);  // one row step at a time: bounded live ranges
#endif
      return true;
    });
  }
  if constexpr (FAST) {  // only the lanes that own both columns summed
#pragma unroll
    for (int q = 0; q < Sh::NQ; ++q) acc[q] = own_all ? acc[q] : 0.0;
  }
}

#ifndef PMX_CA_PF_GRAM
#define PMX_CA_PF_GRAM 3
#endif
#ifndef PMX_CA_PF_UPD
#define PMX_CA_PF_UPD 1
#endif
constexpr int kCaPfGram = PMX_CA_PF_GRAM, kCaPfUpd = PMX_CA_PF_UPD;


// Which tiles a launch covers: the interior rectangle [ti_lo, ti_hi) x [tj_lo, tj_hi) of a pass's
// tiling (every tile there is "fast": no Dirichlet node or partial width in reach), or the frame
// around it.  Part 0 (all tiles) is the general kernel over the whole tiling.
struct CaPart {
  int part;  // 0 all, 1 interior, 2 frame
  int tiles_i, ti_lo, ti_hi, tj_lo, tj_hi;
};

// k-th tile of a part -> (ti, tj); the frame: tile rows above the rectangle, below it, then the
// columns left and right of it
__device__ __forceinline__ void ca_part_tile(int k, const CaPart& P, int tiles_j, int& ti, int& tj) {
  if (P.part == 0) {
    ti = k / tiles_j;
    tj = k - ti * tiles_j;
    return;
  }
  const int h = P.ti_hi - P.ti_lo, wj = P.tj_hi - P.tj_lo;
  if (P.part == 1) {
    ti = P.ti_lo + k / wj;
    tj = P.tj_lo + k % wj;
    return;
  }
  const int ntop = P.ti_lo * tiles_j;
  if (k < ntop) { ti = k / tiles_j; tj = k % tiles_j; return; }
  k -= ntop;
  const int nbot = (P.tiles_i - P.ti_hi) * tiles_j;
  if (k < nbot) { ti = P.ti_hi + k / tiles_j; tj = k % tiles_j; return; }
  k -= nbot;
  if (k < h * P.tj_lo) { ti = P.ti_lo + k / P.tj_lo; tj = k % P.tj_lo; return; }
  k -= h * P.tj_lo;
  const int wr = tiles_j - P.tj_hi;
  ti = P.ti_lo + k / wr;
  tj = P.tj_hi + k % wr;
}

// MW: waves per SIMD the register allocation must allow; DMA: pass 1's interior tiles prefetch by
// LDS-DMA (4 rows ahead) instead of registers; PART 1: the interior tiles only, compiled without the
// Dirichlet / partial-tile paths (whose registers would otherwise cap every tile's occupancy).
template <typename T, int S, bool UPD, int MW, bool DMA, int PART>
__global__ void __launch_bounds__(64, MW)
k_ca_sweep(DevGeom G, DevTables Tb, T* w, T* z0, T* z1, T* p0, T* p1, double* __restrict__ partials,
           const PcgState* St, const CaState* C, int TI, int tiles_j, const unsigned* __restrict__ ctbl,
           int cwords, int64_t pbase, CaFaces faces, CaPart part, int ntiles) {
  using Sh = CaShape<S>;
  constexpr int NB = Sh::NB;
  typedef const __attribute__((address_space(4))) PcgState CPS;
  typedef const __attribute__((address_space(4))) CaState CCS;
  const int done = ((CPS*)St)->done;    // NOLINT
  const long long blk = ((CCS*)C)->blk;  // NOLINT
  const int nupd = ((CCS*)C)->nupd;      // NOLINT
  double ca[NB], cb[NB], cc[NB], pa[S][NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    ca[i] = UPD ? ((CCS*)C)->coef[0][i] : 0.0;  // NOLINT
    cb[i] = UPD ? ((CCS*)C)->coef[1][i] : 0.0;  // NOLINT
    cc[i] = UPD ? ((CCS*)C)->coef[2][i] : 0.0;  // NOLINT
#pragma unroll
    for (int j = 0; j < S; ++j) pa[j][i] = UPD ? ((CCS*)C)->pa[j][i] : 0.0;  // NOLINT
  }
  if (UPD ? nupd == 0 : done != 0) return;
  int ti = 0, tj = 0;
  ca_part_tile(xcd_remap(blockIdx.x, gridDim.x), part, tiles_j, ti, tj);
  const int id = ti * tiles_j + tj;  // the tile's partials slot, whichever launch covers it
  const int i0 = 1 + ti * TI, i1 = min(i0 + TI - 1, G.nx);
  const int j0 = 1 + tj * Sh::WO, j1 = min(j0 + Sh::WO - 1, G.ny);
  // pass 1 reads set blk & 1; pass 2 runs after the reduction advanced blk: reads set (blk - 1) & 1
  // (a rewind leaves blk alone: the set the stopped block read)
  const int in = int((UPD ? blk - 1 : blk) & 1);
  const T* pin = in ? p1 : p0;
  const T* zin = in ? z1 : z0;
  T* pout = in ? p0 : p1;
  T* zout = in ? z0 : z1;
  const CaK K = ca_consts(G);
  const int lane = threadIdx.x & 63;
  // pass 1's LDS-DMA row ring (4 slots of p, z rows, 2 KiB each)
  __shared__ double s_ring[(!UPD && DMA) ? 4 * 256 : 2];
  const unsigned* tbl = ctbl + int64_t(tj) * cwords;
  const bool fast = PART == 1 || (j1 == j0 + Sh::WO - 1 && G.gi0 + i0 - S >= 1 && G.gi0 + i1 + S <= G.M - 1 &&
                                   G.gj0 + j0 - Sh::HE >= 1 && G.gj0 + j0 - Sh::HE + 127 <= G.N - 1);
  double acc[Sh::NQ];
#pragma unroll
  for (int q = 0; q < Sh::NQ; ++q) acc[q] = 0.0;
  // rows in flight: pass 1 (2 fields, compute-heavy) 3 rows ahead; pass 2 (3 fields) 1
  constexpr int PF = UPD ? kCaPfUpd : kCaPfGram;
#define PMX_CA_MARCH(F, R) \
  ca_march<T, S, UPD, F, PF, R>(G, Tb, K, pin, zin, pout, zout, w, i0, i1, j0, j1, tbl, faces, acc, ca, cb, cc, pa)
  if constexpr (UPD) {
    if (nupd < 0) {  // rewind: w only
      if constexpr (PART == 1) PMX_CA_MARCH(true, true);
      else if (fast) PMX_CA_MARCH(true, true);
      else PMX_CA_MARCH(false, true);
      return;
    }
  }
  if constexpr (PART == 1) {
    if constexpr (!UPD && DMA && sizeof(T) == 8)  // pass 1: rows prefetched by LDS-DMA
      ca_march<T, S, UPD, true, PF, false, 4>(G, Tb, K, pin, zin, pout, zout, w, i0, i1, j0, j1, tbl, faces, acc, ca,
                                              cb, cc, pa, s_ring);
    else
      PMX_CA_MARCH(true, false);
    goto marched;
  }
  if constexpr (!UPD && DMA && sizeof(T) == 8) {
    if (fast) {  // pass 1, interior tiles: rows prefetched by LDS-DMA
      ca_march<T, S, UPD, true, PF, false, 4>(G, Tb, K, pin, zin, pout, zout, w, i0, i1, j0, j1, tbl, faces, acc, ca,
                                              cb, cc, pa, s_ring);
      goto marched;
    }
  }
  if (fast) PMX_CA_MARCH(true, false);
  else PMX_CA_MARCH(false, false);
marched:
#undef PMX_CA_MARCH
  // partials, one array per quantity: Gram products q (pass 1, n1 tiles) at [q][tile], norms j (pass
  // 2, its own n2 tiles) at pbase + [j][tile], pbase = NQ n1
  constexpr int NOUT = UPD ? Sh::NN : Sh::NQ;
#pragma unroll
  for (int q = 0; q + 1 < NOUT; q += 2) wave_sum2_mfma(acc[q], acc[q + 1]);
  if constexpr (NOUT & 1) acc[NOUT - 1] = wave_sum_mfma(acc[NOUT - 1]);
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < NOUT; ++q) partials[pbase + int64_t(q) * ntiles + id] = acc[q];
  }
}

// ---- the fused pass: pass 2 of block b and pass 1 of block b + 1 in ONE march ----
// Pass 1 of block b + 1 reads exactly the (p, z) that pass 2 of block b writes, so one wave can form
// them and go on: stage 1 builds block b's basis from (p_b, z_b) (radius s), forms p_{b+1}, z_{b+1}
// (and w, and block b's norms on the owned rows), and stage 2 builds block b+1's basis from those
// values still in registers (radius s again) and sums its Gram products.  The tile loads radius 2s
// (2s extra rows above and below, HE = 2s extra columns per side), and the block costs 48 B/pt of
// HBM traffic (read p, z, w; write p, z, w) instead of 64: pass 1's re-read of p, z disappears.  The
// reduction that follows sees what it saw after pass 1 (the Gram partials of block b + 1) plus the
// norms of block b, which the pass 2 of the unfused schedule left; the scalars are unchanged.
template <int S>
struct CaFuseShape {
  static constexpr int HE = 2 * S;         // even: 16-B aligned column chunks
  static constexpr int WO = 128 - 2 * HE;  // owned columns per wave tile
};

template <typename T>
struct CaFRow {
  T p[2], z[2], w[2];
};

// The two halves run in two waves of one workgroup: wave 0 (the producer) marches stage 1 and writes
// each new (p, z) row into a 2-slot LDS ring, wave 1 (the consumer) marches stage 2 from the ring, one
// workgroup barrier per row step.  One wave holding both chains' register windows, the Gram sums and
// the prefetch rows needs ~300 VGPRs (1 wave per SIMD, latency-bound: measured 1.38-2.3 ms/iteration
// against 1.20 unfused at 16384^2); split, each wave holds half and the SIMDs keep 3 of them.
template <typename T, int S, bool FAST, int PF, int ROLE, int RG = 1>
__device__ __forceinline__ void ca_march_fused(const DevGeom& G, const CaK& K, const T* __restrict__ pin,
                                               const T* __restrict__ zin, T* __restrict__ pout, T* __restrict__ zout,
                                               T* __restrict__ w, int i0, int i1, int j0, int j1,
                                               const unsigned* __restrict__ ctbl, const CaFaces& F,
                                               double (&acc)[CaShape<S>::NQ], double (&nacc)[S],
                                               const double (&ca)[CaShape<S>::NB], const double (&cb)[CaShape<S>::NB],
                                               const double (&cc)[CaShape<S>::NB],
                                               const double (&pa)[S][CaShape<S>::NB], double* ring,
                                               unsigned long long* tm = nullptr, double* dring = nullptr) {
  using Sh = CaShape<S>;
  constexpr int NB = Sh::NB, HE = CaFuseShape<S>::HE;
  const int64_t P = G.pitch;
  const int lane = threadIdx.x & 63;
  const int c0 = j0 - HE + 2 * lane;
  const int cmax = ca_cmax(G, F);
  bool colin[2], own[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = c0 + u, g = G.gj0 + c;
    colin[u] = g >= 1 && g <= G.N - 1;
    own[u] = c >= j0 && c <= j1;
  }
  const bool own_all = own[0] && own[1];
  const bool own_any = own[0] || own[1];
  auto interior_row = [&](int m) { return G.gi0 + m >= 1 && G.gi0 + m <= G.M - 1; };
  // ring slot k: the new p row at ring + k * 256, z at + 128 (2 doubles per lane).  2 RG slots: the
  // waves meet once per RG row steps (the producer after its group's last step, the consumer before
  // its group's first), so one wave's slow row is absorbed by the other's group; step t = m - mfirst
  // uses slot t mod 2 RG (rhi: the unrolled iteration's offset, for RG = 4)
  static_assert(RG == 1 || RG == 2 || RG == 4, "ca_march_fused: 1, 2 or 4 row steps per barrier");
  int rhi = 0;
  auto slot_of = [&](auto qc) {
    constexpr int q = decltype(qc)::value;
    if constexpr (RG == 4) return rhi + q;
    else return q & (2 * RG - 1);
  };
  typedef double d2 __attribute__((ext_vector_type(2)));
#ifdef PMX_CAF_TIMING  // study builds: s_memtime ticks a wave spends in the row barriers
  unsigned long long t_sync = 0;
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
  auto sync = [&] {
    const unsigned long long a = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    t_sync += __builtin_amdgcn_s_memtime() - a;
  };
  auto tdone = [&] {
    if (tm) {
      tm[0] = __builtin_amdgcn_s_memtime() - t_start;
      tm[1] = t_sync;
    }
  };
#else
  auto sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  auto tdone = [] {};
#endif

  // register windows as ca_march's: level l of a chain at row r in slot (r - mfirst) & 3.  The
  // producer's chain (block b's basis) trails the loaded row by l rows, the consumer's (block b+1's)
  // trails the producer's output row by l more.
  double XP[S + 1][4][2], XZ[S][4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int l = 0; l <= S; ++l) XP[l][a][u] = 0.0;
#pragma unroll
      for (int l = 0; l < S; ++l) XZ[l][a][u] = 0.0;
    }
  int ch[4] = {0, 0, 0, 0};  // row classes, same slots

  const int mfirst = i0 - 2 * S, mlast = i1 + 2 * S;
  // level l of a chain at row rb - l (slot q = slot of row rb) from level l-1 at rows rb-l-1 .. rb-l+1
  // and level l-2 at row rb-l
  auto level = [&](auto lc, auto qc, int rb, auto& X) {
    constexpr int l = decltype(lc)::value, q = decltype(qc)::value;
    constexpr int sc = (q - l) & 3, sm = (q - l - 1) & 3, sp = (q - l + 1) & 3;
    const int r = rb - l;
    const double(&ctr)[2] = X[l - 1][sc];
    const double left = dpp_shift0<kWaveShr1>(ctr[1]);
    const double right = dpp_shift0<kWaveShl1>(ctr[0]);
    double lt[2];
    ca_lt(ch[sc], r, ctr, X[l - 1][sm], X[l - 1][sp], left, right, K, G, F, c0, cmax, lt);
    const bool rin = FAST || interior_row(r);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      double v;
      if constexpr (l == 1) v = lt[u];
      else v = __builtin_fma(2.0, lt[u], -X[l - 2][sc][u]);
      X[l][sc][u] = (FAST || (rin && colin[u])) ? v : 0.0;
    }
  };
  auto chains = [&](auto qc, int rb) {
    static_for_while<S>([&](auto l1) {
      level(std::integral_constant<int, decltype(l1)::value + 1>{}, qc, rb, XP);
      return true;
    });
    static_for_while<S - 1>([&](auto l1) {
      level(std::integral_constant<int, decltype(l1)::value + 1>{}, qc, rb, XZ);
      return true;
    });
  };
  auto gather = [&](auto sc, double (&Y)[NB][2]) {
    constexpr int sl = decltype(sc)::value;
#pragma unroll
    for (int l = 0; l <= S; ++l) {
      Y[l][0] = XP[l][sl][0];
      Y[l][1] = XP[l][sl][1];
    }
#pragma unroll
    for (int l = 0; l < S; ++l) {
      Y[S + 1 + l][0] = XZ[l][sl][0];
      Y[S + 1 + l][1] = XZ[l][sl][1];
    }
  };

  if constexpr (ROLE == 0) {
    // ---- producer: rows mfirst .. mlast of (p_b, z_b); at step m the basis of row g1 = m - S is
    // complete: the new (p, z) of rows i0 - S .. i1 + S into the ring, w and block b's norms on the
    // owned rows
    auto fetch = [&](int m, CaFRow<T>& b) {
      const int mc = min(max(m, 1 - F.gh), G.nx + F.gh);
      ca_load2<T>(pin + int64_t(mc) * P, c0, cmax, b.p);
      ca_load2<T>(zin + int64_t(mc) * P, c0, cmax, b.z);
      const int wc = min(max(m - S, 1 - F.gh), G.nx + F.gh);
      ca_load2<T>(w + int64_t(wc) * P, c0, cmax, b.w);
    };
    auto core = [&](auto qc, int m, const CaFRow<T>& cur) {
      constexpr int q = decltype(qc)::value;
      ch[q] = ca_row_cls(ctbl, m);
      const bool rin = FAST || interior_row(m);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const bool in = FAST || (rin && colin[u]);
        XP[0][q][u] = in ? double(cur.p[u]) : 0.0;
        XZ[0][q][u] = in ? double(cur.z[u]) : 0.0;
      }
      chains(qc, m);
      const int g1 = m - S;
      if (g1 < i0 - S) return;
      double Y[NB][2];
      gather(std::integral_constant<int, (q - S) & 3>{}, Y);
      T pn[2], zn[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        double sp = 0.0, sz = 0.0;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          sp = __builtin_fma(ca[i], Y[i][u], sp);
          sz = __builtin_fma(cb[i], Y[i][u], sz);
        }
        pn[u] = static_cast<T>(sp);
        zn[u] = static_cast<T>(sz);
      }
      double* sl = ring + slot_of(qc) * 256;
      *reinterpret_cast<d2*>(sl + 2 * lane) = d2{double(pn[0]), double(pn[1])};
      *reinterpret_cast<d2*>(sl + 128 + 2 * lane) = d2{double(zn[0]), double(zn[1])};
      if (g1 < i0 || g1 > i1) return;
      // an owned row: w, the stores and block b's ||p_{k+j}||^2
      T wn[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        double sw = double(cur.w[u]);
#pragma unroll
        for (int i = 0; i < NB; ++i) sw = __builtin_fma(cc[i], Y[i][u], sw);
        wn[u] = static_cast<T>(sw);
        if (FAST || own[u]) {
          nacc[0] = __builtin_fma(Y[0][u], Y[0][u], nacc[0]);
#pragma unroll
          for (int j = 1; j < S; ++j) {
            double v = 0.0;
#pragma unroll
            for (int i = 0; i <= j; ++i) v = __builtin_fma(pa[j][i], Y[i][u], v);
#pragma unroll
            for (int i = 0; i < j; ++i) v = __builtin_fma(pa[j][S + 1 + i], Y[S + 1 + i][u], v);
            nacc[j] = __builtin_fma(v, v, nacc[j]);
          }
        }
      }
      if (FAST ? own_all : own_any) {
        const int64_t o = int64_t(g1) * P;
        ca_store2<T>(pout + o, c0, pn, FAST || own_all, own);
        ca_store2<T>(zout + o, c0, zn, FAST || own_all, own);
        ca_store2<T>(w + o, c0, wn, FAST || own_all, own);
      }
    };
    static_assert(PF == 1 || PF == 3 || PF == 4, "ca_march_fused: prefetch depth 1 or 3 (registers), 4 (LDS-DMA)");
    if constexpr (PF == 4) {
      // LDS-DMA ring (fp64 FAST tiles): row mfirst + t of p, z (and w of row t - S) in slot t & 3, 4 rows
      // ahead, no VGPR buffers.  global_load_lds_dwordx4 is invisible to hipcc, so the march counts
      // vmcnt itself (as pcg1_march's DMA mode): before reading row m, the ops younger than its DMAs
      // are the DMAs of rows m+1 .. m+3 (3 each) and the stores of the steps m-4 .. m-1 that stored
      // (p, z, w of an owned row: 3 each).  Other vector ops (cut-row face loads) only add younger
      // ops, and hipcc's own waits for them only drain more.
      static_assert(FAST && sizeof(T) == 8, "ca_march_fused: LDS-DMA rows for fp64 FAST tiles");
      constexpr int D = 4;
      const unsigned voff = unsigned(c0 + 8) * 8u;  // bytes from row - 8 (ca_col's unsigned form)
      const unsigned lds0 = unsigned(reinterpret_cast<uintptr_t>(dring));
      auto dma_row = [&](int m, int slot) {
        const unsigned l = lds0 + unsigned(slot) * 3072u;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's previous ds_reads have returned
        const int mc = min(max(m, 1 - F.gh), G.nx + F.gh);
        const int wc = min(max(m - S, 1 - F.gh), G.nx + F.gh);
        dma16(pin + int64_t(mc) * P - 8, voff, l);
        dma16(zin + int64_t(mc) * P - 8, voff, l + 1024u);
        dma16(w + int64_t(wc) * P - 8, voff, l + 2048u);
      };
      // step t stores iff its row t - S is owned
      auto stores = [&](int t) { return t >= mfirst && t - S >= i0 && t - S <= i1 ? 1 : 0; };
#pragma unroll
      for (int q = 0; q < D; ++q) dma_row(min(mfirst + q, mlast), q);
      bool more = true;
      for (int m = mfirst; more && m <= mlast; m += 4) {
        rhi = (m - mfirst) & 4;
        more = static_for_while<4>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          const int mm = m + q;
          if (mm > mlast) return false;
          const int nst = stores(mm - 4) + stores(mm - 3) + stores(mm - 2) + stores(mm - 1);
          switch (nst) {
            case 0: wait_vmcnt<3 * (D - 1)>(); break;
            case 1: wait_vmcnt<3 * (D - 1) + 3>(); break;
            case 2: wait_vmcnt<3 * (D - 1) + 6>(); break;
            case 3: wait_vmcnt<3 * (D - 1) + 9>(); break;
            default: wait_vmcnt<3 * (D - 1) + 12>(); break;
          }
          const double* sl = dring + q * 384;
          const d2 pv = *reinterpret_cast<const d2*>(sl + 2 * lane);
          const d2 zv = *reinterpret_cast<const d2*>(sl + 128 + 2 * lane);
          const d2 wv = *reinterpret_cast<const d2*>(sl + 256 + 2 * lane);
          CaFRow<T> cur;
          cur.p[0] = pv.x;
          cur.p[1] = pv.y;
          cur.z[0] = zv.x;
          cur.z[1] = zv.y;
          cur.w[0] = wv.x;
          cur.w[1] = wv.y;
          dma_row(min(mm + D, mlast), q);
          core(qc, mm, cur);
          if (q % RG == RG - 1 || mm == mlast) sync();
          return true;
        });
      }
      wait_vmcnt<0>();  // no DMA may land after the wave has moved on (its LDS is the next tile's)
#pragma unroll
      for (int j = 0; j < S; ++j) nacc[j] = own_all ? nacc[j] : 0.0;
      tdone();
      return;
    }
    constexpr int NBUF = PF + 1;
    CaFRow<T> buf[NBUF];
#pragma unroll
    for (int q = 0; q < PF; ++q) fetch(min(mfirst + q, mlast), buf[q]);
    bool more = true;
    for (int m = mfirst; more && m <= mlast; m += 4) {
      rhi = (m - mfirst) & 4;
      more = static_for_while<4>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        if (m + q > mlast) return false;
        fetch(min(m + q + PF, mlast), buf[(q + PF) % NBUF]);
        core(qc, m + q, buf[q % NBUF]);
        // the group's rows are in the ring; the consumer has read the slots the next group rewrites
        if (q % RG == RG - 1 || m + q == mlast) sync();
        return true;
      });
    }
    if constexpr (FAST) {
#pragma unroll
      for (int j = 0; j < S; ++j) nacc[j] = own_all ? nacc[j] : 0.0;
    }
    tdone();
  } else {
    // ---- consumer: after the producer's step m, row g1 = m - S of the new (p, z) is in the ring: block
    // b+1's basis from it (exactly as pass 1 would build it from the stored values) and, S rows
    // behind, the Gram products of the owned rows
    auto core = [&](auto qc, int m) {
      constexpr int q = decltype(qc)::value;
      const int g1 = m - S;
      if (g1 < i0 - S) return;
      constexpr int s1 = (q - S) & 3;
      const double* sl = ring + slot_of(qc) * 256;
      const d2 pv = *reinterpret_cast<const d2*>(sl + 2 * lane);
      const d2 zv = *reinterpret_cast<const d2*>(sl + 128 + 2 * lane);
      ch[s1] = ca_row_cls(ctbl, g1);
      XP[0][s1][0] = pv.x;
      XP[0][s1][1] = pv.y;
      XZ[0][s1][0] = zv.x;
      XZ[0][s1][1] = zv.y;
      chains(std::integral_constant<int, s1>{}, g1);
      const int g2 = g1 - S;
      if (g2 < i0) return;
      constexpr int s2 = (q - 2 * S) & 3;
      double Y2[NB][2];
      gather(std::integral_constant<int, s2>{}, Y2);
      double d[2];
      ca_diag(ch[s2], g2, K, G, F, c0, cmax, d);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (!(FAST || own[u])) continue;
#pragma unroll
        for (int qq = 0; qq < Sh::NQ; ++qq)
          acc[qq] = __builtin_fma(Y2[ca_prod_i<S>(qq)][u], d[u] * Y2[ca_prod_j<S>(qq)][u], acc[qq]);
      }
    };
    bool more = true;
    for (int m = mfirst; more && m <= mlast; m += 4) {
      rhi = (m - mfirst) & 4;
      more = static_for_while<4>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        if (m + q > mlast) return false;
        if (q % RG == 0) sync();
        core(qc, m + q);
        return true;
      });
    }
    if constexpr (FAST) {
#pragma unroll
      for (int q = 0; q < Sh::NQ; ++q) acc[q] = own_all ? acc[q] : 0.0;
    }
    tdone();
  }
}

#ifndef PMX_CA_PF_FUSE
#define PMX_CA_PF_FUSE 1
#endif

// The fused pass (see ca_march_fused): one workgroup of two waves per tile.  After the reduction of
// block b (CaState::nupd > 0) it applies block b and sums block b+1's Gram products; after a reduction
// that stopped inside block b - 1 (nupd < 0) wave 0 rewinds w, as pass 2 would.  Partials: the Gram
// products q at [q][tile] (wave 1), block b's norms j at NQ * ntiles + [j][tile] (wave 0): the
// reduction's n = n2 = ntiles.
template <typename T, int S, int MW, int PART, int RG, bool DMAF = false>
__global__ void __launch_bounds__(128, MW)
k_ca_fused(DevGeom G, T* w, T* z0, T* z1, T* p0, T* p1, double* __restrict__ partials, const CaState* C, int TI,
           int tiles_j, const unsigned* __restrict__ ctbl, int cwords, CaFaces faces, CaPart part, int ntiles) {
  using Sh = CaShape<S>;
  using Fs = CaFuseShape<S>;
  constexpr int NB = Sh::NB;
  typedef const __attribute__((address_space(4))) CaState CCS;
  const long long blk = ((CCS*)C)->blk;  // NOLINT
  const int nupd = ((CCS*)C)->nupd;      // NOLINT
  if (nupd == 0) return;
  const int role = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
  double ca[NB], cb[NB], cc[NB], pa[S][NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    ca[i] = ((CCS*)C)->coef[0][i];  // NOLINT
    cb[i] = ((CCS*)C)->coef[1][i];  // NOLINT
    cc[i] = ((CCS*)C)->coef[2][i];  // NOLINT
#pragma unroll
    for (int j = 0; j < S; ++j) pa[j][i] = ((CCS*)C)->pa[j][i];  // NOLINT
  }
  int ti = 0, tj = 0;
  ca_part_tile(xcd_remap(blockIdx.x, gridDim.x), part, tiles_j, ti, tj);
  const int id = ti * tiles_j + tj;
  const int i0 = 1 + ti * TI, i1 = min(i0 + TI - 1, G.nx);
  const int j0 = 1 + tj * Fs::WO, j1 = min(j0 + Fs::WO - 1, G.ny);
  // the reduction advanced blk: block b's (p, z) are set (blk - 1) & 1 (a rewind leaves blk alone)
  const int in = int((blk - 1) & 1);
  T* pin = in ? p1 : p0;
  T* zin = in ? z1 : z0;
  T* pout = in ? p0 : p1;
  T* zout = in ? z0 : z1;
  const CaK K = ca_consts(G);
  const int lane = threadIdx.x & 63;
  const unsigned* tbl = ctbl + int64_t(tj) * cwords;
  const bool fast = PART == 1 || (j1 == j0 + Fs::WO - 1 && G.gi0 + i0 - 2 * S >= 1 && G.gi0 + i1 + 2 * S <= G.M - 1 &&
                                   G.gj0 + j0 - Fs::HE >= 1 && G.gj0 + j0 - Fs::HE + 127 <= G.N - 1);
  double acc[Sh::NQ], nacc[S];
#pragma unroll
  for (int q = 0; q < Sh::NQ; ++q) acc[q] = 0.0;
#pragma unroll
  for (int j = 0; j < S; ++j) nacc[j] = 0.0;
  if (nupd < 0) {  // rewind: w only, by wave 0 (no barrier on this path)
    if (role != 0) return;
    double pz[S][NB] = {};
    if (PART == 1 || fast)
      ca_march<T, S, true, true, kCaPfUpd, true, 0, Fs::HE>(G, DevTables{}, K, pin, zin, pout, zout, w, i0, i1, j0, j1,
                                                            tbl, faces, acc, ca, cb, cc, pz);
    else if constexpr (PART != 1)
      ca_march<T, S, true, false, kCaPfUpd, true, 0, Fs::HE>(G, DevTables{}, K, pin, zin, pout, zout, w, i0, i1, j0,
                                                             j1, tbl, faces, acc, ca, cb, cc, pz);
    return;
  }
  __shared__ double ring[2 * RG * 256];
  // the producer's LDS-DMA rows (DMAF: fp64 interior tiles): 4 slots of p, z, w rows
  __shared__ double dring[DMAF ? 4 * 384 : 2];
  static_assert(!DMAF || (PART == 1 && sizeof(T) == 8), "k_ca_fused: LDS-DMA rows for fp64 interior tiles");
  constexpr int PF = PMX_CA_PF_FUSE;
  unsigned long long tm[2] = {0, 0};
#define PMX_CAF_MARCH(FA, R)                                                                                        \
  ca_march_fused<T, S, FA, PF, R, RG>(G, K, pin, zin, pout, zout, w, i0, i1, j0, j1, tbl, faces, acc, nacc, ca, cb, \
                                      cc, pa, ring, tm)
  if (role == 0) {
    if constexpr (DMAF)
      ca_march_fused<T, S, true, 4, 0, RG>(G, K, pin, zin, pout, zout, w, i0, i1, j0, j1, tbl, faces, acc, nacc, ca, cb,
                                           cc, pa, ring, tm, dring);
    else if (PART == 1 || fast) PMX_CAF_MARCH(true, 0);
    else if constexpr (PART != 1) PMX_CAF_MARCH(false, 0);
#pragma unroll
    for (int j = 0; j + 1 < S; j += 2) wave_sum2_mfma(nacc[j], nacc[j + 1]);
    if constexpr (S & 1) nacc[S - 1] = wave_sum_mfma(nacc[S - 1]);
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < S; ++j) partials[int64_t(Sh::NQ + j) * ntiles + id] = nacc[j];
    }
  } else {
    if (PART == 1 || fast) PMX_CAF_MARCH(true, 1);
    else if constexpr (PART != 1) PMX_CAF_MARCH(false, 1);
#pragma unroll
    for (int q = 0; q + 1 < Sh::NQ; q += 2) wave_sum2_mfma(acc[q], acc[q + 1]);
    if constexpr (Sh::NQ & 1) acc[Sh::NQ - 1] = wave_sum_mfma(acc[Sh::NQ - 1]);
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < Sh::NQ; ++q) partials[int64_t(q) * ntiles + id] = acc[q];
    }
  }
#undef PMX_CAF_MARCH
#ifdef PMX_CAF_TIMING
  if (lane == 0 && blk == 7 && id % 499 == 0)
    printf("caf part %d role %d tile %d fast %d total %llu sync %llu\n", PART, role, id, int(fast), tm[0], tm[1]);
#endif
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

// The face coefficients of every local node (rows 1-gh .. nx+gh, columns -1 .. ny+2; on 2-D blocks
// with neighbours across y also the ghost columns: -8 .. ny+gh+2): a(gi, gj) and b(gi, gj) by the exact
// formula (the class fast values are bit-identical to it).
__global__ void __launch_bounds__(256) k_ca_faces(DevGeom G, DevTables Tb, double* fa, double* fb, int gh) {
  const int jlo = (G.nb & kNbYlo) ? -8 : -1, jhi = (G.nb & kNbYhi) ? G.ny + gh + 2 : G.ny + 2;
  const int lj = jlo + int(blockIdx.x * blockDim.x + threadIdx.x);
  const int li = 1 - gh + int(blockIdx.y);
  if (lj > jhi) return;
  const int gi = min(max(G.gi0 + li, 0), G.M), gj = min(max(G.gj0 + lj, 0), G.N);
  const int64_t o = int64_t(li) * G.pitch + lj;
  fa[o] = coef_a(Tb, G, gi, gj);
  fb[o] = coef_b(Tb, G, gi, gj);
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

// The scalars of one reduction: first the pending stop test of the previous block (its ||p_{k+j}||^2
// sums u, its alpha_j from CaState), then -- unless the solve ended there or check_only -- the s
// iterations of this block on the coefficient vectors, from the Gram products t (raw sums), in the
// classic loop's order of tests (max_iter, the |denominator| guard; the stop test follows in the next
// reduction).  One lane; writes CaState (pass 2's coefficients and mode) and the PcgState outcome.
template <int S>
__device__ void ca_finish(const double* t, const double* u, double h, double wdiff, int nmax, bool check_only,
                          PcgState* St, CaState* C) {
  using Sh = CaShape<S>;
  constexpr int NB = Sh::NB;
  C->nupd = 0;
  if (St->done) return;
  // ---- (i) the pending stop test: ||w^{k+j+1} - w^{k+j}|| = |alpha_j| ||p_{k+j}||
  if (C->pend_n > 0) {
    const int n = C->pend_n;
    double diff = 0.0;
    for (int j = 0; j < n; ++j) {
      diff = fabs(C->alpha[j]) * sqrt(u[j] * wdiff);
      const bool bad = !(diff == diff);
      if (bad || diff < St->delta) {
        const long long kk = C->pend_k + j + 1;
        if (j + 1 < n) {  // w went past the stop: back to w_k + Y c_{j+1}
          for (int i = 0; i < NB; ++i) C->coef[2][i] = C->pc[j][i] - C->pc[n - 1][i];
          C->nupd = -1;
        }
        St->it = kk;
        St->iters = kk;
        St->diff = diff;
        St->status = bad ? int(Status::kBreakdown) : int(Status::kConverged);
        if (bad) St->nan_flag = 1;
        St->done = 1;
        C->pend_n = 0;
        return;
      }
    }
    St->diff = diff;
    C->pend_n = 0;
    if (C->after_status != 0) {  // the pending block ended at a breakdown or at max_iter
      St->iters = C->after_iters;
      St->status = C->after_status;
      St->done = 1;
      C->after_status = 0;
      return;
    }
  }
  if (check_only) return;
  // ---- (ii) this block's iterations
  const long long k = St->it;
  const long long left = St->max_iter - k;
  if (left <= 0) {
    St->iters = k;
    St->status = int(Status::kMaxIter);
    St->done = 1;
    return;
  }
  const int nm = int(left < nmax ? left : nmax);
  // G = Y^T D Y from the moments (see the header)
  double mu[2 * S + 1], nu[2 * S - 1], rho[2 * S];
  bool nan = false;
  for (int q = 0; q < Sh::NQ; ++q) nan |= !(t[q] == t[q]) || isinf(t[q]);
  for (int m = 0; m <= S; ++m) mu[m] = t[m] * h;
  for (int m = S + 1; m <= 2 * S; ++m) mu[m] = 2.0 * t[m] * h - mu[m & 1];
  for (int m = 0; m < S; ++m) nu[m] = t[2 * S + 1 + m] * h;
  for (int m = S; m <= 2 * S - 2; ++m) nu[m] = 2.0 * t[2 * S + 1 + m] * h - nu[m & 1];
  for (int m = 0; m <= S; ++m) rho[m] = t[4 * S + m] * h;
  for (int b = 1; b < S; ++b) rho[S + b] = 2.0 * t[5 * S + b] * h - rho[S - b];
  double Gm[NB][NB];
  for (int a = 0; a <= S; ++a) {
    for (int b = 0; b <= S; ++b) Gm[a][b] = 0.5 * (mu[a + b] + mu[a > b ? a - b : b - a]);
    for (int b = 0; b < S; ++b)
      Gm[a][S + 1 + b] = Gm[S + 1 + b][a] = 0.5 * (rho[a + b] + rho[a > b ? a - b : b - a]);
  }
  for (int a = 0; a < S; ++a)
    for (int b = 0; b < S; ++b) Gm[S + 1 + a][S + 1 + b] = 0.5 * (nu[a + b] + nu[a > b ? a - b : b - a]);
  auto quad = [&](const double* x, const double* y) {
    double r = 0.0;
    for (int i = 0; i < NB; ++i) {
      double v = 0.0;
      for (int j = 0; j < NB; ++j) v = __builtin_fma(Gm[i][j], y[j], v);
      r = __builtin_fma(x[i], v, r);
    }
    return r;
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
  double g = Gm[S + 1][S + 1];
  const bool weighted = St->norm == int(Norm::kWeighted);
  int n = 0;
  for (int j = 0; j < nm; ++j) {
    shiftT(a, Ta);
    const double den = quad(a, Ta);
    if (nan || !(den == den) || !(g == g) || (weighted ? fabs(den) < St->bd_tol : den < St->bd_tol)) {
      C->after_status = int(Status::kBreakdown);
      C->after_iters = k + j + 1;
      if (nan || !(den == den) || !(g == g)) St->nan_flag = 1;
      break;
    }
    const double alpha = g / den;
    for (int i = 0; i < NB; ++i) {
      C->pa[j][i] = a[i];
      c[i] = __builtin_fma(alpha, a[i], c[i]);
      C->pc[j][i] = c[i];
    }
    C->alpha[j] = alpha;
    n = j + 1;
    for (int i = 0; i < NB; ++i) b[i] = __builtin_fma(-alpha, Ta[i], b[i]);
    const double gn = quad(b, b);
    const double beta = gn / g;
    for (int i = 0; i < NB; ++i) a[i] = __builtin_fma(beta, a[i], b[i]);
    g = gn;
  }
  if (n == 0) {  // breakdown in the block's first iteration: nothing to apply or to test
    St->iters = C->after_iters;
    St->status = C->after_status;
    St->done = 1;
    C->after_status = 0;
    return;
  }
  if (C->after_status == 0 && k + n >= St->max_iter) {
    C->after_status = int(Status::kMaxIter);
    C->after_iters = St->max_iter;
  }
  for (int i = 0; i < NB; ++i) {
    C->coef[0][i] = a[i];
    C->coef[1][i] = b[i];
    C->coef[2][i] = c[i];
  }
  C->nupd = n;
  C->blk += 1;
  C->pend_n = n;
  C->pend_k = k;
  St->it = k + n;
}

// ca_finish's one lane reads and writes ~40 words of PcgState / CaState in a dependent order: on the
// device structs that is a chain of L2 round trips (~19 us per reduction at 1600x2400).  The
// finishing wave stages both structs in LDS (all lanes, one round trip), lane 0 runs on the copies,
// the wave writes them back.
template <typename X>
__device__ __forceinline__ void wave_copy(X* dst, const X* src, int lane) {
  static_assert(sizeof(X) % 8 == 0, "wave_copy: whole 8-byte words");
  const unsigned long long* a = reinterpret_cast<const unsigned long long*>(src);
  unsigned long long* b = reinterpret_cast<unsigned long long*>(dst);
  for (int i = lane; i < int(sizeof(X) / 8); i += kWave) b[i] = a[i];
}
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Deterministic reduction of the partials (one array of n tile values per quantity: the Gram
// products of pass 1, then the norms of the previous pass 2) + ca_finish.  Blocks sum contiguous tile
// ranges (thread-strided, then waves in order) and publish their chunk sums; the last block to arrive
// (ticket) sums the chunks in block order, one quantity per lane.  check_only: the norms alone (the
// pending test after a batch's last block).  Hand-off as k_reduce_n (pcg_device.hpp).
template <int S>
__global__ void __launch_bounds__(256)
k_ca_reduce(const double* __restrict__ part, int n, int n2, double h, double wdiff, int nmax, int check_only,
            int finish, PcgState* St, CaState* C, double* chunk, long long* progress) {
  using Sh = CaShape<S>;
  constexpr int NT = Sh::NQ + Sh::NN;
  __shared__ double lds[NT][256 / kWave];
  __shared__ double tot[NT];
  __shared__ int last;
  if (St->done) {
    if (blockIdx.x == 0 && threadIdx.x == 0) C->nupd = 0;
    return;
  }
  const int q0 = check_only ? Sh::NQ : 0;  // first quantity summed
  const int nb = int(gridDim.x);
  double s[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) s[q] = 0.0;
  if (!check_only) {  // the Gram products of pass 1's n tiles
    const int lo = int(int64_t(n) * blockIdx.x / nb), hi = int(int64_t(n) * (blockIdx.x + 1) / nb);
    for (int i = lo + int(threadIdx.x); i < hi; i += 256) {
#pragma unroll
      for (int q = 0; q < Sh::NQ; ++q) s[q] += part[int64_t(q) * n + i];
    }
  }
  {  // the norms of pass 2's n2 tiles
    const double* p2 = part + int64_t(Sh::NQ) * n;
    const int lo = int(int64_t(n2) * blockIdx.x / nb), hi = int(int64_t(n2) * (blockIdx.x + 1) / nb);
    for (int i = lo + int(threadIdx.x); i < hi; i += 256) {
#pragma unroll
      for (int q = Sh::NQ; q < NT; ++q) s[q] += p2[int64_t(q - Sh::NQ) * n2 + i];
    }
  }
  const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    s[q] = wave_sum_mfma(s[q]);
    if (lane == 0) lds[q][wid] = s[q];
  }
  __syncthreads();
  if (nb > 1) {
    if (threadIdx.x == 0) {
#pragma unroll
      for (int q = 0; q < NT; ++q)
        st_publish(chunk + NT * blockIdx.x + q, (lds[q][0] + lds[q][1]) + (lds[q][2] + lds[q][3]));
      last = ticket_arrive_last(&C->ticket, nb);
    }
    __syncthreads();
    if (!last || threadIdx.x >= kWave) return;  // wave 0 of the last block finishes (full EXEC)
    // lane l sums chunks l, l + 64, .. (all NT loads of a round in flight together), then the wave
    double t[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) t[q] = 0.0;
    for (int r = 0; r < (nb + kWave - 1) / kWave; ++r) {
      const int c = lane + kWave * r;
#pragma unroll
      for (int q = 0; q < NT; ++q)
        if (q >= q0) t[q] += c < nb ? ld_published(chunk + NT * c + q) : 0.0;
    }
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      t[q] = wave_sum_mfma(t[q]);
      if (lane == 0) tot[q] = t[q];
    }
  } else {
    if (threadIdx.x >= kWave) return;
    if (lane < NT) tot[lane] = (lds[lane][0] + lds[lane][1]) + (lds[lane][2] + lds[lane][3]);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (finish) {
    __shared__ PcgState sst;
    __shared__ CaState sc;
    wave_copy(&sst, St, lane);
    wave_copy(&sc, C, lane);
    wave_lds_sync();
    if (lane == 0) {
      ca_finish<S>(tot, tot + Sh::NQ, h, wdiff, nmax, check_only != 0, &sst, &sc);
      if (progress) __hip_atomic_store(progress, sst.it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      sc.ticket = 0u;  // re-arm for the next launch (every block has arrived; stream order publishes it)
    }
    wave_lds_sync();
    wave_copy(St, &sst, lane);
    wave_copy(C, &sc, lane);
  } else if (lane == 0) {  // decomposed: the rank's sums, all-reduced before k_ca_finish
    for (int q = 0; q < NT; ++q) C->red[q] = tot[q];
    if (nb > 1) C->ticket = 0u;
  }
}

// The same reduction in ONE workgroup of 16 waves, for up to kCaReduce1Max tiles (the reference grids,
// strips of 8 ranks): no chunk hand-off between workgroups (ticket, published chunks, a second wave
// sum: ~7 of the ~19 us the multi-block reduction takes at 1600x2400), and the last wave stages the
// solver state in LDS while the others still load partials.  Fixed order: thread-strided sums, wave
// sums, then the 16 waves in index order.
template <int S>
__global__ void __launch_bounds__(1024)
k_ca_reduce1(const double* __restrict__ part, int n, int n2, double h, double wdiff, int nmax, int check_only,
             int finish, PcgState* St, CaState* C, long long* progress) {
  using Sh = CaShape<S>;
  constexpr int NT = Sh::NQ + Sh::NN, NW = 1024 / kWave;
  __shared__ double lds[NT][NW];
  __shared__ double tot[NT];
  __shared__ PcgState sst;
  __shared__ CaState sc;
  if (St->done) {
    if (threadIdx.x == 0) C->nupd = 0;
    return;
  }
  const int wid = int(threadIdx.x) / kWave, lane = int(threadIdx.x) % kWave;
  if (finish && wid == NW - 1) {
    wave_copy(&sst, St, lane);
    wave_copy(&sc, C, lane);
  }
  double sm[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) sm[q] = 0.0;
  if (!check_only) {
    for (int i = int(threadIdx.x); i < n; i += 1024) {
#pragma unroll
      for (int q = 0; q < Sh::NQ; ++q) sm[q] += part[int64_t(q) * n + i];
    }
  }
  const double* p2 = part + int64_t(Sh::NQ) * n;
  for (int i = int(threadIdx.x); i < n2; i += 1024) {
#pragma unroll
    for (int q = Sh::NQ; q < NT; ++q) sm[q] += p2[int64_t(q - Sh::NQ) * n2 + i];
  }
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    sm[q] = wave_sum_mfma(sm[q]);
    if (lane == 0) lds[q][wid] = sm[q];
  }
  __syncthreads();
  if (wid != 0) return;
  if (lane < NT) {
    double v = 0.0;
    for (int w = 0; w < NW; ++w) v += lds[lane][w];
    tot[lane] = v;
  }
  wave_lds_sync();
  if (finish) {
    if (lane == 0) {
      ca_finish<S>(tot, tot + Sh::NQ, h, wdiff, nmax, check_only != 0, &sst, &sc);
      if (progress) __hip_atomic_store(progress, sst.it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    wave_lds_sync();
    wave_copy(St, &sst, lane);
    wave_copy(C, &sc, lane);
  } else if (lane < NT) {  // decomposed: the rank's sums, all-reduced before k_ca_finish
    C->red[lane] = tot[lane];
  }
}

// Decomposed grids: ca_finish on the all-reduced sums (CaState::red), after the all-reduce.
template <int S>
__global__ void __launch_bounds__(64)
k_ca_finish(double h, double wdiff, int nmax, int check_only, PcgState* St, CaState* C, long long* progress) {
  const int lane = int(threadIdx.x);
  __shared__ PcgState sst;
  __shared__ CaState sc;
  wave_copy(&sst, St, lane);
  wave_copy(&sc, C, lane);
  wave_lds_sync();
  if (lane == 0) {
    if (sst.done) {
      sc.nupd = 0;
    } else {
      double t[7 * S];
      bool bad = false;
      for (int q = 0; q < 7 * S; ++q) {
        t[q] = sc.red[q];
        bad |= !(t[q] == t[q]) || isinf(t[q]);
      }
      if (bad) sst.nan_flag = 1;
      ca_finish<S>(t, t + 6 * S, h, wdiff, nmax, check_only != 0, &sst, &sc);
      if (progress) __hip_atomic_store(progress, sst.it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  wave_lds_sync();
  wave_copy(St, &sst, lane);
  wave_copy(C, &sc, lane);
}

// Ghost exchange of the s-step on 2-D blocks (packed slots of the comm arena, 8 slots: 4 sides, 4
// corners): the gh owned edge lines of z and p of one set, and the gh x gh corner blocks, once per
// block of s iterations.  Slot layout [field][line q][pos]: x sides line q = row 1+q (x-lo) / nx-gh+1+q
// (x-hi) when packing, ghost row 1-gh+q / nx+1+q when unpacking, pos = column - 1; y sides likewise
// with columns; corners [field][q][t] = (row, column) offsets q, t into the gh x gh block.  A message
// of slot s lands in the neighbour's opposite_slot(s) in the same order.  Grid: (ceil(max(nx, ny) /
// 256), 8, 2 gh).
template <typename T>
__global__ void __launch_bounds__(256)
k_ca_halo(DevGeom G, T* z, T* p, HaloBufs<T> H, int gh, int unpack, long long* progress) {
  const int slot = blockIdx.y;
  if (progress && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0)
    __hip_atomic_fetch_add(progress + (unpack ? 2 : 1), 1ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (!((G.nb >> slot) & 1)) return;
  const int f = int(blockIdx.z) / gh, q = int(blockIdx.z) % gh;
  const int t = int(blockIdx.x) * 256 + int(threadIdx.x);
  const int nx = G.nx, ny = G.ny;
  int li, lj;
  int64_t idx;
  if (slot < 2) {  // x sides: rows
    if (t >= ny) return;
    li = slot == 0 ? (unpack ? 1 - gh + q : 1 + q) : (unpack ? nx + 1 + q : nx - gh + 1 + q);
    lj = 1 + t;
    idx = (int64_t(f) * gh + q) * ny + t;
  } else if (slot < 4) {  // y sides: columns
    if (t >= nx) return;
    li = 1 + t;
    lj = slot == 2 ? (unpack ? 1 - gh + q : 1 + q) : (unpack ? ny + 1 + q : ny - gh + 1 + q);
    idx = (int64_t(f) * gh + q) * nx + t;
  } else {  // corners: gh x gh blocks
    if (t >= gh) return;
    const bool xhi = slot >= 6, yhi = slot == 5 || slot == 7;
    li = xhi ? (unpack ? nx + 1 + q : nx - gh + 1 + q) : (unpack ? 1 - gh + q : 1 + q);
    lj = yhi ? (unpack ? ny + 1 + t : ny - gh + 1 + t) : (unpack ? 1 - gh + t : 1 + t);
    idx = (int64_t(f) * gh + q) * gh + t;
  }
  T* fld = f == 0 ? z : p;
  const int64_t o = int64_t(li) * G.pitch + lj;
  if (unpack)
    fld[o] = H.recv[slot][idx];
  else
    H.send[slot][idx] = fld[o];
}

}  // namespace

template <typename T>
void launch_ca_halo(const DevGeom& G, T* z, T* p, const HaloBufs<T>& H, int gh, bool unpack, hipStream_t s,
                    long long* progress) {
  PMX_CHECK(gh >= 1 && G.nx >= gh && G.ny >= gh, "s-step ghost exchange: blocks of at least gh x gh nodes");
  const int n = std::max(G.nx, G.ny);
  hipLaunchKernelGGL(k_ca_halo<T>, dim3((n + 255) / 256, kHaloSlots, 2 * gh), dim3(256), 0, s, G, z, p, H, gh,
                     unpack ? 1 : 0, progress);
  HIP_CHECK(hipGetLastError());
}

CaTiles make_ca_tiles(const DevGeom& G, int s, int rows, int rows2, int rows_f) {
  PMX_CHECK(s == 2 || s == 3, "s-step PCG: s must be 2 or 3");
  CaTiles t;
  t.s = s;
  t.he = (s + 1) & ~1;
  t.wo = 128 - 2 * t.he;
  t.tiles_j = (G.ny + t.wo - 1) / t.wo;
  if (rows <= 0) {
    // tall tiles keep the 2s re-marched halo rows cheap (their basis levels are recomputed); shorter
    // when the grid has fewer than ~4 rounds of tiles (3 waves x 4 SIMDs x 256 CUs = 3072 at a time):
    // a tile's march is ~1.5 us per row with the SIMD shared, so a last round of long tiles trails.
    // 8-GPU strip of 16384^2 (2048 rows): 64-row tiles (4050) 284 us per pass 1, 32-row 225 us;
    // loopback per-rank iteration 8 GPUs 240 -> 221 us, 4 GPUs 388 -> 371 (profiles/r5/ca/rows/).
    rows = 64;
    while (rows > 8 && int64_t((G.nx + rows - 1) / rows) * t.tiles_j < 12288) rows /= 2;
  }
  PMX_CHECK(rows >= 1 && rows <= 4096, "s-step PCG: tile rows must be in [1, 4096]");
  t.rows = rows;
  t.tiles_i = (G.nx + rows - 1) / rows;
  // pass 2 (memory-bound, no Gram) marches shorter tiles: fewer DRAM rows in flight per wave and a
  // finer load balance win over the extra halo rows (16384^2: pass 2 2.87 ms at 32 rows, 2.66 at 16;
  // pass 1 1.78 at 32, 1.77 at 64, 2.17 at 16 -- profiles/r5/ca/)
  if (rows2 <= 0) {
    rows2 = 16;
    while (rows2 > 8 && int64_t((G.nx + rows2 - 1) / rows2) * t.tiles_j < 4096) rows2 /= 2;
  }
  PMX_CHECK(rows2 >= 1 && rows2 <= 4096, "s-step PCG: pass-2 tile rows must be in [1, 4096]");
  t.rows2 = rows2;
  t.tiles_i2 = (G.nx + rows2 - 1) / rows2;
  // interior rectangles (k_ca_sweep's `fast`): rows i0 - s .. i1 + s and columns j0 - he .. j0 - he + 127
  // strictly inside the grid, full width.  i0 = 1 + ti rows: ti >= 1 and (ti + 1) rows <= nx - s; j0 = 1 +
  // tj wo: tj >= 1 and tj wo + 128 - he <= ny.  Checked tile by tile against the kernel's condition.
  auto fast = [&](int ti, int tj, int r) {
    const int i0 = 1 + ti * r, i1 = std::min(i0 + r - 1, G.nx);
    const int j0 = 1 + tj * t.wo, j1 = std::min(j0 + t.wo - 1, G.ny);
    return j1 == j0 + t.wo - 1 && G.gi0 + i0 - s >= 1 && G.gi0 + i1 + s <= G.M - 1 && G.gj0 + j0 - t.he >= 1 &&
           G.gj0 + j0 - t.he + 127 <= G.N - 1;
  };
  t.tj_lo = std::min(1, t.tiles_j);
  t.tj_hi = std::max(t.tj_lo, std::min(t.tiles_j, (G.ny - 128 + t.he) / t.wo + 1));
  auto rect = [&](int r, int tiles_i, int& lo, int& hi) {
    // i0 - s >= 1: with tiles shorter than s the interior starts further down, so no interior tile
    // reads a ghost row (they do not wait for the ghost exchange on strips)
    lo = std::min((s + r - 1) / r, tiles_i);
    hi = std::max(lo, std::min(tiles_i, (G.nx - s) / r));
    if (hi <= lo || t.tj_hi <= t.tj_lo) { lo = hi = 0; return; }
    for (int ti = 0; ti < tiles_i; ++ti)
      for (int tj = 0; tj < t.tiles_j; ++tj) {
        const bool in = ti >= lo && ti < hi && tj >= t.tj_lo && tj < t.tj_hi;
        PMX_CHECK(!in || fast(ti, tj, r), "s-step PCG: interior tile (" << ti << ", " << tj << ") is not fast");
      }
  };
  rect(rows, t.tiles_i, t.ti_lo, t.ti_hi);
  rect(rows2, t.tiles_i2, t.ti_lo2, t.ti_hi2);
  if (t.ti_hi <= t.ti_lo || t.ti_hi2 <= t.ti_lo2) t.split = t.split_upd = 0;
  // rows up to nx + 2s (the fused march's lowest loaded row), 16 per word from row -kCaRowOff
  t.cwords = (G.nx + 4 * s + 2 * kCaRowOff + 15) / 16 + 1;
  // the fused tiling: radius 2s (he_f = 2s columns per side), rows_f rows.  Auto: 64 (16384^2 at 3
  // waves per SIMD, ms/iteration: 16 rows 1.41, 32 1.13, 64 1.01), halved while the grid has fewer
  // than ~4 rounds of tiles (1536 two-wave workgroups at a time): loopback per-rank ms/iteration of
  // the 16384^2 strips, 8 GPUs (2048 rows) 16 / 32 / 48 / 64 rows 0.226 / 0.199 / 0.202 / 0.209,
  // 4 GPUs 0.399 / 0.338 / 0.329 / 0.330 (profiles/r6/loopback/)
  t.he_f = 2 * s;
  t.wo_f = 128 - 2 * t.he_f;
  t.tiles_j_f = (G.ny + t.wo_f - 1) / t.wo_f;
  if (rows_f <= 0) {
    // 96 rows where that still leaves >= 20,000 tiles (~13 rounds of 1536 workgroups): a tile marches
    // rows_f + 4s rows, so 96 instead of 64 cuts the redundant halo row steps from 19% to 12.5%.
    // 16384^2 same-process A/B, fastest of 20 probed blocks per session, ms/iteration over 11
    // sessions: 64 rows median 1.015, 96 rows 0.950 (each bimodal by placement: 0.94-0.95 / 1.01-1.02);
    // fp32 32768^2 3.43 -> 3.13 ms, mixed 16384^2 0.942 -> 0.893 (profiles/r6/shape/).  The 2-GPU strip
    // (12,212 tiles at 96 rows) keeps 64: loopback 0.576 (64) vs 0.586 ms (96).
    rows_f = int64_t((G.nx + 95) / 96) * t.tiles_j_f >= 20000 ? 96 : 64;
    while (rows_f > 16 && rows_f <= 64 && int64_t((G.nx + rows_f - 1) / rows_f) * t.tiles_j_f < 6000) rows_f /= 2;
  }
  PMX_CHECK(rows_f >= 1 && rows_f <= 4096, "s-step PCG: fused tile rows must be in [1, 4096]");
  t.rows_f = rows_f;
  t.tiles_i_f = (G.nx + rows_f - 1) / rows_f;
  {
    const int r = 2 * s;  // the fused kernel's radius
    auto fastf = [&](int ti, int tj) {
      const int i0 = 1 + ti * rows_f, i1 = std::min(i0 + rows_f - 1, G.nx);
      const int j0 = 1 + tj * t.wo_f, j1 = std::min(j0 + t.wo_f - 1, G.ny);
      return j1 == j0 + t.wo_f - 1 && G.gi0 + i0 - r >= 1 && G.gi0 + i1 + r <= G.M - 1 && G.gj0 + j0 - t.he_f >= 1 &&
             G.gj0 + j0 - t.he_f + 127 <= G.N - 1;
    };
    t.tj_lo_f = std::min(1, t.tiles_j_f);
    t.tj_hi_f = std::max(t.tj_lo_f, std::min(t.tiles_j_f, (G.ny - 128 + t.he_f) / t.wo_f + 1));
    t.ti_lo_f = std::min((r + rows_f - 1) / rows_f, t.tiles_i_f);  // i0 - r >= 1
    t.ti_hi_f = std::max(t.ti_lo_f, std::min(t.tiles_i_f, (G.nx - r) / rows_f));
    if (t.ti_hi_f <= t.ti_lo_f || t.tj_hi_f <= t.tj_lo_f) {
      t.ti_lo_f = t.ti_hi_f = t.tj_lo_f = t.tj_hi_f = 0;
      t.split_f = 0;
    }
    for (int ti = t.ti_lo_f; ti < t.ti_hi_f; ++ti)
      for (int tj = t.tj_lo_f; tj < t.tj_hi_f; ++tj)
        PMX_CHECK(fastf(ti, tj), "s-step PCG: interior fused tile (" << ti << ", " << tj << ") is not fast");
  }
  return t;
}

int ca_nq(int s) { return s == 2 ? CaShape<2>::NQ + CaShape<2>::NN : CaShape<3>::NQ + CaShape<3>::NN; }

void ca_build_classes(const DevGeom& G, const DevTables& Tb, const CaTiles& t, unsigned* tbl, hipStream_t s,
                      bool fused) {
  const int tj = fused ? t.tiles_j_f : t.tiles_j;
  const int n = tj * t.cwords;
  hipLaunchKernelGGL(k_ca_row_classes, dim3((n + 255) / 256), dim3(256), 0, s, G, Tb, fused ? t.he_f : t.he,
                     fused ? t.wo_f : t.wo, tj, t.cwords, tbl);
  HIP_CHECK(hipGetLastError());
}

void ca_build_faces(const DevGeom& G, const DevTables& Tb, double* fa, double* fb, int gh, hipStream_t s) {
  PMX_CHECK(G.nx + 2 * gh <= 65535, "k_ca_faces: grid.y limit");
  hipLaunchKernelGGL(k_ca_faces, dim3((G.ny + gh + 12 + 255) / 256, G.nx + 2 * gh), dim3(256), 0, s, G, Tb, fa, fb, gh);
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
                     const PcgState* S, const CaState* C, const CaTiles& t, bool upd, hipStream_t s,
                     hipStream_t sframe, hipEvent_t frame_wait) {
  PMX_CHECK(G.nb == 0 || t.gh >= t.s, "s-step PCG: a decomposed grid needs s ghost rows / columns");
  if (!sframe) sframe = s;
  PMX_CHECK(t.tbl != nullptr && t.fa != nullptr && t.fb != nullptr, "s-step PCG: row-class / face tables missing");
  PMX_CHECK(sizeof(T) == 8 || !t.dma, "s-step PCG: LDS-DMA rows need fp64");
  const int n = upd ? t.ntiles2() : t.ntiles();
  const int rows = upd ? t.rows2 : t.rows;
  const int64_t pbase = upd ? int64_t(ca_nq(t.s) - t.s) * t.ntiles() : 0;  // norms after the Gram products
  const int ti_lo = upd ? t.ti_lo2 : t.ti_lo, ti_hi = upd ? t.ti_hi2 : t.ti_hi;
  const int tiles_i = upd ? t.tiles_i2 : t.tiles_i;
  const int nin = (ti_hi - ti_lo) * (t.tj_hi - t.tj_lo);
  const CaFaces F{t.fa, t.fb, t.gh};
  const CaPart P1{1, tiles_i, ti_lo, ti_hi, t.tj_lo, t.tj_hi}, P2{2, tiles_i, ti_lo, ti_hi, t.tj_lo, t.tj_hi},
      P0{0, tiles_i, 0, 0, 0, 0};
#define PMX_CA_K(SS, U, MW, D, PT, PP, NB)                                                                          \
  do {                                                                                                              \
    if ((NB) > 0)                                                                                                   \
      hipLaunchKernelGGL((k_ca_sweep<T, SS, U, MW, (D) && sizeof(T) == 8, PT>), dim3(NB), dim3(64), 0,            \
                         (PT) == 2 ? sframe : s, G, Tb, w,                                                           \
                         z0, z1, p0, p1, partials, S, C, rows, t.tiles_j, t.tbl, t.cwords, pbase, F, PP, n);        \
  } while (0)
  // split (default): the interior tiles with the fast-only kernel at 3 waves per SIMD, the frame with
  // the general one at 2; else every tile general at waves_gram / waves_upd
  // the tiles that read ghost rows -- the frame on sframe, or every tile on s -- wait for frame_wait
  const bool split = (upd ? t.split_upd : t.split) && nin > 0;
  if (frame_wait) HIP_CHECK(hipStreamWaitEvent(split ? sframe : s, frame_wait, 0));
#define PMX_CA(SS)                                                                                                   \
  do {                                                                                                               \
    if (split) {                                                                                                     \
      if (upd) {                                                                                                     \
        PMX_CA_K(SS, true, 2, false, 2, P2, n - nin);                                                                \
        PMX_CA_K(SS, true, 3, false, 1, P1, nin);                                                                    \
      } else {                                                                                                       \
        PMX_CA_K(SS, false, 2, false, 2, P2, n - nin);                                                               \
        if (t.dma) PMX_CA_K(SS, false, 3, true, 1, P1, nin);                                                         \
        else PMX_CA_K(SS, false, 2, false, 1, P1, nin); /* register rows: 3 waves would spill */                     \
      }                                                                                                              \
    } else if (upd) {                                                                                                \
      if (t.waves_upd == 2) PMX_CA_K(SS, true, 2, false, 0, P0, n);                                                  \
      else PMX_CA_K(SS, true, 3, false, 0, P0, n);                                                                   \
    } else if (t.dma) {                                                                                              \
      if (t.waves_gram == 3) PMX_CA_K(SS, false, 3, true, 0, P0, n);                                                 \
      else PMX_CA_K(SS, false, 2, true, 0, P0, n);                                                                   \
    } else {                                                                                                         \
      if (t.waves_gram == 3) PMX_CA_K(SS, false, 3, false, 0, P0, n);                                                \
      else PMX_CA_K(SS, false, 2, false, 0, P0, n);                                                                  \
    }                                                                                                                \
  } while (0)
  if (t.s == 2) PMX_CA(2);
  else PMX_CA(3);
#undef PMX_CA
#undef PMX_CA_K
  HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_ca_fused(const DevGeom& G, T* w, T* z0, T* z1, T* p0, T* p1, double* partials, const CaState* C,
                     const CaTiles& t, hipStream_t s, hipStream_t sframe, hipEvent_t frame_wait) {
  PMX_CHECK(G.nb == 0 || t.gh >= 2 * t.s, "the fused s-step pass needs 2 s ghost rows / columns on a decomposed grid");
  PMX_CHECK(t.fuse && t.tbl_f != nullptr && t.fa != nullptr && t.fb != nullptr,
            "s-step PCG: fused tiling / row classes / face tables missing");
  if (!sframe) sframe = s;
  const int n = t.ntilesf();
  const int nin = (t.ti_hi_f - t.ti_lo_f) * (t.tj_hi_f - t.tj_lo_f);
  const CaFaces F{t.fa, t.fb, t.gh};
  const CaPart P1{1, t.tiles_i_f, t.ti_lo_f, t.ti_hi_f, t.tj_lo_f, t.tj_hi_f},
      P2{2, t.tiles_i_f, t.ti_lo_f, t.ti_hi_f, t.tj_lo_f, t.tj_hi_f}, P0{0, t.tiles_i_f, 0, 0, 0, 0};
#define PMX_CAF_KD(SS, MW, PT, PP, NB, RG, DM)                                                                     \
  do {                                                                                                              \
    if ((NB) > 0)                                                                                                   \
      hipLaunchKernelGGL((k_ca_fused<T, SS, MW, PT, RG, DM>), dim3(NB), dim3(128), 0, (PT) == 2 ? sframe : s, G, w, \
                         z0, z1, p0, p1, partials, C, t.rows_f, t.tiles_j_f, t.tbl_f, t.cwords, F, PP, n);          \
  } while (0)
#define PMX_CAF_K(SS, MW, PT, PP, NB, RG) PMX_CAF_KD(SS, MW, PT, PP, NB, RG, false)
  constexpr bool kDmaOk = sizeof(T) == 8;
  const bool split = t.split_f && nin > 0;
  if (frame_wait) HIP_CHECK(hipStreamWaitEvent(split ? sframe : s, frame_wait, 0));
  // interior kernel: rows per barrier group (rg_f), 3 waves per SIMD (2: RG 1 only)
#define PMX_CAF(SS)                                                 \
  do {                                                              \
    if (split) {                                                    \
      if (t.frame_first_f) PMX_CAF_K(SS, 2, 2, P2, n - nin, 1);     \
      if (t.waves_f == 2) PMX_CAF_K(SS, 2, 1, P1, nin, 1);          \
      else if (t.rg_f == 4) PMX_CAF_K(SS, 3, 1, P1, nin, 4);        \
      else if (t.rg_f == 2) PMX_CAF_K(SS, 3, 1, P1, nin, 2);        \
      else if (kDmaOk && t.dma_f) PMX_CAF_KD(SS, 3, 1, P1, nin, 1, kDmaOk); \
      else PMX_CAF_K(SS, 3, 1, P1, nin, 1);                         \
      if (!t.frame_first_f) PMX_CAF_K(SS, 2, 2, P2, n - nin, 1);    \
    } else if (t.waves_f == 3) {                                    \
      PMX_CAF_K(SS, 3, 0, P0, n, 1);                                \
    } else {                                                        \
      PMX_CAF_K(SS, 2, 0, P0, n, 1);                                \
    }                                                               \
  } while (0)
  if (t.s == 2) PMX_CAF(2);
  else PMX_CAF(3);
#undef PMX_CAF
#undef PMX_CAF_K
#undef PMX_CAF_KD
  HIP_CHECK(hipGetLastError());
}

void launch_ca_reduce(const double* partials, int n, int n2, int s_, double h, double wdiff, int nmax,
                      bool check_only, PcgState* S, CaState* C, double* chunk, hipStream_t s, long long* progress,
                      bool finish) {
  PMX_CHECK(nmax >= 1 && nmax <= s_, "s-step PCG: a block runs 1..s iterations");
  const int nb = std::max(1, std::min(kCaReduceMaxBlocks, std::max(n, n2) / 512));
  const int co = check_only ? 1 : 0, fi = finish ? 1 : 0;
  if (std::max(n, n2) <= kCaReduce1Max) {
    if (s_ == 2)
      hipLaunchKernelGGL(k_ca_reduce1<2>, dim3(1), dim3(1024), 0, s, partials, n, n2, h, wdiff, nmax, co, fi, S, C,
                         progress);
    else
      hipLaunchKernelGGL(k_ca_reduce1<3>, dim3(1), dim3(1024), 0, s, partials, n, n2, h, wdiff, nmax, co, fi, S, C,
                         progress);
    HIP_CHECK(hipGetLastError());
    return;
  }
  if (s_ == 2)
    hipLaunchKernelGGL(k_ca_reduce<2>, dim3(nb), dim3(256), 0, s, partials, n, n2, h, wdiff, nmax, co, fi, S, C, chunk,
                       progress);
  else
    hipLaunchKernelGGL(k_ca_reduce<3>, dim3(nb), dim3(256), 0, s, partials, n, n2, h, wdiff, nmax, co, fi, S, C, chunk,
                       progress);
  HIP_CHECK(hipGetLastError());
}

void launch_ca_finish(int s_, double h, double wdiff, int nmax, bool check_only, PcgState* S, CaState* C,
                      hipStream_t s, long long* progress) {
  const int co = check_only ? 1 : 0;
  if (s_ == 2)
    hipLaunchKernelGGL(k_ca_finish<2>, dim3(1), dim3(64), 0, s, h, wdiff, nmax, co, S, C, progress);
  else
    hipLaunchKernelGGL(k_ca_finish<3>, dim3(1), dim3(64), 0, s, h, wdiff, nmax, co, S, C, progress);
  HIP_CHECK(hipGetLastError());
}

// fp64 and fp32 storage of w, z, p (the basis, the updates and the Gram sums in fp64 registers either way)
#define PMX_CA_INST(T)                                                                                            \
  template void launch_ca_init<T>(const DevGeom&, const DevTables&, T*, T*, hipStream_t);                         \
  template void launch_ca_sweep<T>(const DevGeom&, const DevTables&, T*, T*, T*, T*, T*, double*, const PcgState*, \
                                   const CaState*, const CaTiles&, bool, hipStream_t, hipStream_t, hipEvent_t);   \
  template void launch_ca_halo<T>(const DevGeom&, T*, T*, const HaloBufs<T>&, int, bool, hipStream_t,          \
                                  long long*);                                                                   \
  template void launch_ca_fused<T>(const DevGeom&, T*, T*, T*, T*, T*, double*, const CaState*, const CaTiles&,    \
                                   hipStream_t, hipStream_t, hipEvent_t);
PMX_CA_INST(double)
PMX_CA_INST(float)
#undef PMX_CA_INST

}  // namespace pmx
