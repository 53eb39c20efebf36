// Small-grid single-pass sweep ("block" tiles): the three pipeline stages of pcg1_march run
// row-parallel across the waves of a workgroup instead of row-serial inside one wave.
//
// Why: at the reference's published grids (800x1200 .. 2400x3200, stage4-mpi+cuda/
// poisson_mpi_cuda_f.cu:847-943) the launch-per-sweep path is bound by one wave's row march: a
// 2-row tile marches 6 row steps (its rows plus the stencil halo of the 3-stage pipeline), each
// ~1.8 us of dependent loads and fp64 arithmetic, and a sweep lasts as long as its slowest tile
// (profiles/r4/persist/).  Here a workgroup of kBlkWaves waves owns TR rows x 124 columns:
//
//   stage A (rows i0-2 .. i1+2):  p^k = D^-1 r^{k-1} + beta p^{k-1}   -> LDS (with r^{k-1}, p^{k-1})
//   barrier
//   stage B (rows i0-1 .. i1+1):  A p^k, r^k = r^{k-1} - alpha A p^k, z^k = D^-1 r^k  -> LDS;
//                                 owned rows store r^k, p^k (and w on the w sweeps)
//   barrier
//   stage C (rows i0 .. i1):      A z^k and the five partial sums
//
// so a tile costs ~3 row latencies instead of TR + 4.  Every value is computed by the same helper
// calls in the same order as pcg1_march (coef_c, zdiv_c, apply_c, fma_c, the same roundings to the
// storage type), so the fields are bit-identical to k_pcg1's; only the partial sums are added in a
// different order (per workgroup instead of per wave tile), as in the persistent kernel.
// Undecomposed fp64 grids only (every ghost is a Dirichlet zero); the prologue is k_pcg1's
// (pcg1_kernels.hip), including the stop test, the breakdown guard and the w-phase check.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "pcg1_march.hpp"

namespace pmx {
namespace {

// The reduction of the sweep's partials folded into the sweep (BlockReduce::ticket non-null): every
// workgroup publishes its partial write-through and takes a ticket; the last one sums all partials
// in a fixed order and finishes as k_reduce_n does (weights, NaN flag, S->it bump, progress word,
// ticket re-armed) -- one launch per iteration instead of two.  Hand-off as k_reduce_n's
// (pcg_device.hpp: st_publish, vmcnt drain, relaxed ticket add, sc1 loads after a barrier).
struct BlockReduce {
  double wt[kNq];
  unsigned* ticket;      // nullptr: plain partials for a separate k_reduce_n
  long long* progress;   // host-mapped progress words or nullptr
};

template <typename T, int TR, int W, bool WS>
__global__ void __launch_bounds__(64 * W)
k_pcg1_block(DevGeom G, DevTables Tb, T* __restrict__ w, T* r, T* r2, T* p0, T* p1,
             double* __restrict__ partials, PcgState* S, int tiles_j, int ntiles, BlockReduce R,
             const Pcg1Slot* __restrict__ order) {
  using C = double;
  constexpr int VEC = 2, WO = 64 * VEC - 4, NA = TR + 4, NB = TR + 2;
  constexpr int kBlkWaves = W;
  constexpr int PA = (NA + W - 1) / W, PB = (NB + W - 1) / W;  // rows per wave in stages A / B
  __shared__ double sP[NA][VEC][64];   // p^k of rows i0-2 .. i1+2 (stage A)
  __shared__ double sPo[NA][VEC][64];  // p^{k-1} of the same rows
  __shared__ double sRo[NA][VEC][64];  // r^{k-1} of the same rows
  __shared__ double sZ[NB][VEC][64];   // z^k of rows i0-1 .. i1+1 (stage B)
  __shared__ double s_col[4 * VEC * 64];
  __shared__ RowConst s_row[TR + 5];   // row constants of rows i0-3 .. i1+2 (tiles with cut rows)
  __shared__ double s_sum[kBlkWaves][kNq];

  // ---- prologue: k_pcg1's (pcg1_march.hpp: one batch of scalar loads, then pcg1_scalars); the
  // dispatch slot is read in the same batch as the state, so the tile's loads wait for one round trip
  asm volatile("" ::"s"(S), "s"(order), "s"(gridDim.x));  // kernel arguments: one batch
  const int pos = xcd_remap(int(blockIdx.x), int(gridDim.x));
  const int id0 = ld_uniform(&order[pos].id, 0);  // pos < gridDim.x = ntiles (launch_pcg1_block)
  const unsigned long long ocls0 = ld_uniform(&order[pos].cls, 0);
  const Pcg1Pro pro = pcg1_load_state(S);
  pcg1_batch(pro, id0, ocls0);
  Pcg1Sweep sw;
  if (!pcg1_scalars<WS>(pro, S, blockIdx.x == 0 && threadIdx.x == 0, sw)) return;
  const long long k = sw.k;
  const double alpha = sw.alpha, beta = sw.beta, c1 = sw.c1, c2 = sw.c2;
  const int wm = sw.wm;
  if (pos >= ntiles) return;  // the grid is exactly ntiles workgroups

  T* pnew = (k & 1) ? p1 : p0;
  const T* pold = (k & 1) ? p0 : p1;
  const T* rold = (k & 1) ? r2 : r;
  T* rnew = (k & 1) ? r : r2;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const ArithF AF{float(G.cx), float(G.cy), float(G.dinv_in), float(G.dinv_out), float(G.inv_eps)};
  const int64_t P = G.pitch;
  const int cmax = G.ny + 1 + (G.ny & 1);
  auto grow = [&](int m) { return min(max(G.gi0 + m, 0), G.M); };
  auto interior_row = [&](int m) { return G.gi0 + m >= 1 && G.gi0 + m <= G.M - 1; };
  const bool wload = WS && wm != 0;

  // every global load of the tile first: stage A's rows, stage B's w (and p^{k-2}) rows -- one
  // latency for the whole tile
  struct Rows {
    T rr[PA][VEC], pp[PA][VEC], wv[PB][VEC], qv[PB][VEC];
  };
  auto load_tile = [&](int id, Rows& L) {
    const int ti = id / tiles_j, tj = id - ti * tiles_j;
    const int i0 = 1 + ti * TR, c0 = 1 + tj * WO - 2 + lane * VEC;
#pragma unroll
    for (int x = 0; x < PA; ++x) {
      const int a = min(wave + x * W, NA - 1);  // past the last row: a harmless repeat
      const int mc = min(max(i0 - 2 + a, -1), G.nx + 2);
      load_cols<T, VEC>(rold + int64_t(mc) * P, c0, cmax, L.rr[x]);
      load_cols<T, VEC>(pold + int64_t(mc) * P, c0, cmax, L.pp[x]);
    }
    if (wload) {
#pragma unroll
      for (int x = 0; x < PB; ++x) {
        const int wc = min(max(i0 - 1 + min(wave + x * W, NB - 1), -1), G.nx + 2);
        load_cols<T, VEC>(w + int64_t(wc) * P, c0, cmax, L.wv[x]);
        // p^{k-2} still sits in the buffer this sweep overwrites with p^k: read before the store
        if (wm == 3) load_cols<T, VEC>(pnew + int64_t(wc) * P, c0, cmax, L.qv[x]);
      }
    }
  };

  double acc[kNq] = {0.0, 0.0, 0.0, 0.0, 0.0};
  // ---- one tile: its three stages on rows L, sums into acc
  auto run_tile = [&](int id, unsigned long long ocls, const Rows& L) {
    const int ti = id / tiles_j, tj = id - ti * tiles_j;
    const int i0 = 1 + ti * TR, i1 = min(i0 + TR - 1, G.nx);
    const int j0 = 1 + tj * WO, j1 = min(j0 + WO - 1, G.ny);
    const int c0 = j0 - 2 + lane * VEC;
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
    const bool own_any = own[0] || own[VEC - 1];
    // row m's class from the slot's 2 bits per row (rows i0-3 .. i1+2; TR + 5 <= 32)
    auto row_of = [&](int m) { return RowCo{grow(m), int((ocls >> (2 * (m - i0 + 3))) & 3ull)}; };
    // does any row of the tile (i0-3 .. i1+2) have cut faces (class 0)?  Only then are the
    // column constants needed
    bool tile_cut = false;
#pragma unroll
    for (int q = 0; q < TR + 5; ++q) tile_cut |= ((ocls >> (2 * q)) & 3ull) == 0;
    // column constants of the tile's lanes and row constants of its rows, for the exact (cut-face)
    // coefficients: one copy per workgroup, lane-private column slots as pcg1_march's park_cols; the
    // rows' constants come in with the tile's loads instead of a scalar round trip in every stage
    if (tile_cut) {
      if (wave == 0) {
#pragma unroll
        for (int u = 0; u < VEC; ++u) {
          const ColConst cc = load_col(Tb, gj[u]);
          s_col[(4 * u) * 64 + lane] = cc.ylo;
          s_col[(4 * u + 1) * 64 + lane] = cc.yhi;
          s_col[(4 * u + 2) * 64 + lane] = cc.rh0;
          s_col[(4 * u + 3) * 64 + lane] = cc.rh1;
        }
      } else if (wave == 1 && lane < TR + 5) {  // the fields of load_row, one row per lane
        const int gi = grow(i0 - 3 + lane);
        RowConst rc;
        rc.rv0 = Tb.rv[gi];
        rc.rv1 = Tb.rv[gi + 1];
        rc.xlo = Tb.xlo[gi];
        rc.xhi = Tb.xhi[gi];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          rc.ca0[q] = Tb.acls[4 * gi + q];
          rc.ca1[q] = Tb.acls[4 * (gi + 1) + q];
          rc.cb[q] = Tb.bcls[4 * gi + q];
        }
        s_row[lane] = rc;
      }
      __syncthreads();
    }
    // coef() with the row's constants from s_row (row m, class c)
    auto coef_t = [&](const RowCo& c, int m, int u, C& a0, C& a1, C& b0, C& b1) {
      if (c.ucls != 0) {
        a0 = a1 = b0 = b1 = c.ucls == 1 ? 1.0 : G.inv_eps;
      } else {
        const RowConst rc = s_row[m - i0 + 3];
        const ColConst cc = col_lds(s_col, u, lane, gj[u]);
        a0 = face_a0c(cc, rc, G);
        a1 = face_a1c(cc, rc, G);
        b0 = face_b0c(cc, rc, G);
        b1 = face_b1c(cc, rc, G);
      }
    };

    // ---- stage A: p^k of rows i0-2 .. i1+2
#pragma unroll
    for (int x = 0; x < PA; ++x) {
      const int a = wave + x * W;
      if (a >= NA) break;
      const int m = i0 - 2 + a;
      const bool rowA = interior_row(m);
      const RowCo cA = row_of(m);
#pragma unroll
      for (int u = 0; u < VEC; ++u) {
        const bool in = rowA && colin[u];
        const C rom = in ? C(L.rr[x][u]) : C(0), pom = in ? C(L.pp[x][u]) : C(0);
        C a0, a1, b0, b1;
        coef_t(cA, m, u, a0, a1, b0, b1);
        const C z = zdiv_c<C>(cA.ucls, rom, a0, a1, b0, b1, G, AF);
        const C v = fma_c(beta, pom, z);
        sP[a][u][lane] = in ? C(static_cast<T>(v)) : C(0);
        sPo[a][u][lane] = pom;
        sRo[a][u][lane] = rom;
      }
    }
    __syncthreads();

    // ---- stage B: A p^k, r^k, z^k of rows i0-1 .. i1+1; stores and three sums on owned rows
    auto stage_b = [&](auto wm_c) {
      constexpr int WM = decltype(wm_c)::value;
      constexpr bool WUP = WM != 0;
#pragma unroll
      for (int x = 0; x < PB; ++x) {
        const int b = wave + x * W;
        if (b >= NB) break;
        const int mb = i0 - 1 + b, a = b + 1;
        const bool ownB = mb >= i0 && mb <= i1;
        const T (&wv)[VEC] = L.wv[x];
        const T (&qv)[VEC] = L.qv[x];
        (void)qv;
        C Pm1[VEC], Pm2[VEC], Pm[VEC], po1[VEC], po2[VEC], pom[VEC], ro1[VEC];
#pragma unroll
        for (int u = 0; u < VEC; ++u) {
          Pm1[u] = sP[a][u][lane];
          Pm2[u] = sP[a - 1][u][lane];
          Pm[u] = sP[a + 1][u][lane];
          po1[u] = sPo[a][u][lane];
          po2[u] = sPo[a - 1][u][lane];
          pom[u] = sPo[a + 1][u][lane];
          ro1[u] = sRo[a][u][lane];
        }
        const bool rowB = interior_row(mb);
        const RowCo cB = row_of(mb);
        const C left = dpp_shift<kWaveShr1>(Pm1[VEC - 1], C(0));
        const C right = dpp_shift<kWaveShl1>(Pm1[0], C(0));
        C oleft = C(0), oright = C(0);
        if constexpr (WM == 2) {
          oleft = dpp_shift<kWaveShr1>(po1[VEC - 1], C(0));
          oright = dpp_shift<kWaveShl1>(po1[0], C(0));
        }
        T rs[VEC], ps[VEC], ws[VEC];
#pragma unroll
        for (int u = 0; u < VEC; ++u) {
          C a0, a1, b0, b1;
          coef_t(cB, mb, u, a0, a1, b0, b1);
          const C Ap = apply_c<C>(Pm1[u], Pm2[u], Pm[u], u == 0 ? left : Pm1[u - 1],
                                  u == VEC - 1 ? right : Pm1[u + 1], a0, a1, b0, b1, G, AF);
          const bool in = rowB && colin[u];
          const C rn = C(static_cast<T>(fma_c(-alpha, Ap, ro1[u])));
          rs[u] = static_cast<T>(in ? rn : C(0));
          const C zn = zdiv_c<C>(cB.ucls, rn, a0, a1, b0, b1, G, AF);
          sZ[b][u][lane] = in ? zn : C(0);
          ps[u] = static_cast<T>(Pm1[u]);
          if constexpr (WM == 1) {
            ws[u] = static_cast<T>(fma_c(C(alpha), Pm1[u], fma_c(C(c1), po1[u], C(wv[u]))));
          } else if constexpr (WM == 2) {
            const C Apo = apply_c<C>(po1[u], po2[u], pom[u], u == 0 ? oleft : po1[u - 1],
                                     u == VEC - 1 ? oright : po1[u + 1], a0, a1, b0, b1, G, AF);
            const C zo = zdiv_c<C>(cB.ucls, fma_c(C(c1), Apo, ro1[u]), a0, a1, b0, b1, G, AF);
            const C t = fma_c(C(c2), po1[u] - zo, C(wv[u]));
            ws[u] = static_cast<T>(fma_c(C(alpha), Pm1[u], fma_c(C(c1), po1[u], t)));
          } else if constexpr (WM == 3) {
            const C t = fma_c(C(c2), C(qv[u]), C(wv[u]));
            ws[u] = static_cast<T>(fma_c(C(alpha), Pm1[u], fma_c(C(c1), po1[u], t)));
          }
          if (ownB && own[u]) {
            acc[0] += double(in ? zn : C(0)) * double(rn);
            acc[3] += double(Ap) * double(Pm1[u]);
            acc[4] += double(Pm1[u]) * double(Pm1[u]);
          }
        }
        if (ownB && own_any) {
          const int64_t o = int64_t(mb) * P;
          store_cols<T, VEC>(rnew + o, c0, rs, own_all, own);
          store_cols<T, VEC>(pnew + o, c0, ps, own_all, own);
          if constexpr (WUP) store_cols<T, VEC>(w + o, c0, ws, own_all, own);
        }
      }
    };
    if constexpr (!WS) {
      stage_b(std::integral_constant<int, 0>{});
    } else {
      switch (wm) {
        case 1: stage_b(std::integral_constant<int, 1>{}); break;
        case 2: stage_b(std::integral_constant<int, 2>{}); break;
        case 3: stage_b(std::integral_constant<int, 3>{}); break;
        default: stage_b(std::integral_constant<int, 0>{}); break;  // k = 0: no w step yet
      }
    }
    __syncthreads();

    // ---- stage C: A z^k of the owned rows, (A z, z) and (A z, p)
    for (int c = wave; c < TR; c += W) {
      const int mc = i0 + c;
      if (mc > i1) break;
      const int b = c + 1;
      C Zc[VEC], Zm[VEC], Zp[VEC];
#pragma unroll
      for (int u = 0; u < VEC; ++u) {
        Zc[u] = sZ[b][u][lane];
        Zm[u] = sZ[b - 1][u][lane];
        Zp[u] = sZ[b + 1][u][lane];
      }
      const RowCo cC = row_of(mc);
      const C left = dpp_shift<kWaveShr1>(Zc[VEC - 1], C(0));
      const C right = dpp_shift<kWaveShl1>(Zc[0], C(0));
#pragma unroll
      for (int u = 0; u < VEC; ++u) {
        C a0, a1, b0, b1;
        coef_t(cC, mc, u, a0, a1, b0, b1);
        const C Az = apply_c<C>(Zc[u], Zm[u], Zp[u], u == 0 ? left : Zc[u - 1], u == VEC - 1 ? right : Zc[u + 1],
                                a0, a1, b0, b1, G, AF);
        if (own[u]) {
          acc[1] += double(Az) * double(Zc[u]);
          acc[2] += double(Az) * double(sP[c + 2][u][lane]);
        }
      }
    }
  };

  {
    Rows L;
    load_tile(id0, L);
    run_tile(id0, ocls0, L);
  }

  // ---- partials: wave sums, then the waves in a fixed order -> one 5-value partial per tile
  const int slot = id0;
  const int nslots = ntiles;
  wave_sum2_mfma(acc[0], acc[1]);
  wave_sum2_mfma(acc[2], acc[3]);
  acc[4] = wave_sum_mfma(acc[4]);
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < kNq; ++q) s_sum[wave][q] = acc[q];
  }
  __syncthreads();
  if (!R.ticket) {
    if (threadIdx.x < kNq) {
      double v = 0.0;
#pragma unroll
      for (int wv = 0; wv < kBlkWaves; ++wv) v += s_sum[wv][threadIdx.x];
      partials[int64_t(kNq) * slot + threadIdx.x] = v;
    }
    return;
  }
  __shared__ int s_last;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int q = 0; q < kNq; ++q) {
      double v = 0.0;
#pragma unroll
      for (int wv = 0; wv < kBlkWaves; ++wv) v += s_sum[wv][q];
      st_publish(partials + int64_t(kNq) * slot + q, v);
    }
    s_last = ticket_arrive_last(R.ticket, nslots);
  }
  __syncthreads();
  if (!s_last) return;
  // the last workgroup: every wave sums a fixed slice of the partials, then the waves in order
  double t[kNq];
#pragma unroll
  for (int q = 0; q < kNq; ++q) t[q] = 0.0;
  for (int l = wave * 64 + lane; l < nslots; l += 64 * W) {
#pragma unroll
    for (int q = 0; q < kNq; ++q) t[q] += ld_published(partials + int64_t(kNq) * l + q);
  }
  wave_sum2_mfma(t[0], t[1]);
  wave_sum2_mfma(t[2], t[3]);
  t[4] = wave_sum_mfma(t[4]);
  __syncthreads();  // s_sum is reused
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < kNq; ++q) s_sum[wave][q] = t[q];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    bool bad = false;
#pragma unroll
    for (int q = 0; q < kNq; ++q) {
      double v = 0.0;
#pragma unroll
      for (int wv = 0; wv < kBlkWaves; ++wv) v += s_sum[wv][q];
      bad |= !(v == v) || isinf(v);
      S->red_c[q] = v * R.wt[q];
    }
    if (bad) S->nan_flag = 1;
    S->it = k + 1;
    if (R.progress) __hip_atomic_store(R.progress, k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    *R.ticket = 0u;  // re-arm for the next launch (stream order makes this visible to it)
  }
}

}  // namespace

bool pcg1_block_shape_ok(int rows, int waves) {
  return (waves == 8 && (rows == 4 || rows == 8 || rows == 12 || rows == 16)) ||
         (waves == 16 && (rows == 8 || rows == 16));
}

template <typename T>
void launch_pcg1_block(const DevGeom& G, const DevTables& Tb, T* w, T* r, T* r2, T* p0, T* p1, double* partials,
                       PcgState* S, const TileCfg& tc, hipStream_t s, bool wsweep, const double* weights,
                       unsigned* ticket, long long* progress) {
  static_assert(sizeof(T) == 8, "pcg1 block tiles: fp64 storage");
  PMX_CHECK(tc.kind == 3 && tc.vec == 2 && G.nb == 0, "pcg1 block tiles: VEC-2 tiling of an undecomposed grid");
  PMX_CHECK(tc.block == 124 && tc.tiles_j == (G.ny + 123) / 124, "pcg1 block tiles: 124-column tiles");
  PMX_CHECK(tc.order0 && tc.rows + 5 <= 32, "pcg1 block tiles: a dispatch order with row classes");
  const int n = tc.ntiles();
  const int grid = n;
  BlockReduce R{};
  for (int q = 0; q < kNq; ++q) R.wt[q] = weights ? weights[q] : 1.0;
  R.ticket = ticket;
  R.progress = progress;
#define PMX_BLK(TR, W)                                                                                             \
  if (wsweep) {                                                                                                    \
    hipLaunchKernelGGL((k_pcg1_block<T, TR, W, true>), dim3(grid), dim3(64 * W), 0, s, G, Tb, w, r, r2, p0, p1,    \
                       partials, S, tc.tiles_j, n, R, tc.order0);                                                  \
  } else {                                                                                                         \
    hipLaunchKernelGGL((k_pcg1_block<T, TR, W, false>), dim3(grid), dim3(64 * W), 0, s, G, Tb, w, r, r2, p0, p1,   \
                       partials, S, tc.tiles_j, n, R, tc.order0);                                                  \
  }
  PMX_CHECK(pcg1_block_shape_ok(tc.rows, tc.bwaves), "pcg1 block tiles: no " << tc.rows << "-row x " << tc.bwaves << "-wave variant");
  if (tc.rows == 4 && tc.bwaves == 8) PMX_BLK(4, 8)
  else if (tc.rows == 8 && tc.bwaves == 8) PMX_BLK(8, 8)
  else if (tc.rows == 8 && tc.bwaves == 16) PMX_BLK(8, 16)
  else if (tc.rows == 12 && tc.bwaves == 8) PMX_BLK(12, 8)
  else if (tc.rows == 16 && tc.bwaves == 8) PMX_BLK(16, 8)
  else if (tc.rows == 16 && tc.bwaves == 16) PMX_BLK(16, 16)
#undef PMX_BLK
  HIP_CHECK(hipGetLastError());
}

template void launch_pcg1_block<double>(const DevGeom&, const DevTables&, double*, double*, double*, double*, double*,
                                        double*, PcgState*, const TileCfg&, hipStream_t, bool, const double*,
                                        unsigned*, long long*);

}  // namespace pmx
