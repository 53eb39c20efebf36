// LDS-DMA row prefetch vs register prefetch on the k_pcg1 access pattern (study probe).
//
// Each wave marches one tile of TI rows x 124 owned columns (128 loaded, 2 halo columns per side)
// over rows i0-2 .. i1+2 like pcg1_march: per row it reads r and p (1 KiB each per wave), and from
// the third row on stores rnew / pnew of the row above (62 lanes x 16 B, non-temporal).  Tiles are
// dealt to XCDs in contiguous row-major bands (xcd_remap), one wave per workgroup, like k_pcg1.
//   reg : register ring, PF rows ahead (the current march: PF 1)
//   dma : global_load_lds_dwordx4 into a per-wave LDS ring of PF slots, counted vmcnt waits
// A few fp64 FMAs and DPP lane shifts per row stand in for the stencil work.  Dynamic LDS caps the
// waves per CU (the real plain sweep runs 4 waves/SIMD = 16 per CU).
// Several candidate field blocks are allocated and every variant is timed on each: the question is
// whether deeper in-flight prefetch closes the gap between fast and slow placements
// (profiles/r4/placement/: slow blocks +3.4% TCP->TCC latency, +7% sweep time).
// Usage: dma_march [n] [candidates] [reps] [work]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);          \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int q = nb / 8, r = nb % 8;
  const int xcd = b % 8, idx = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ double shl(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x130, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x130, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

template <int WORK>
__device__ __forceinline__ void work(double (&x)[2], double (&y)[2], double a) {
#pragma unroll
  for (int k = 0; k < WORK; ++k) {
    x[0] = __builtin_fma(a, y[1], x[0]);
    x[1] = __builtin_fma(a, y[0], x[1]);
    y[0] = __builtin_fma(-a, x[1], y[0]);
    y[1] = __builtin_fma(-a, x[0], y[1]);
  }
}

typedef double d2v __attribute__((ext_vector_type(2)));

struct Geo {
  int n, pitch, TI, tiles_i, tiles_j, halo;  // halo 0: march rows i0 .. i1+1 only (one extra row)
  int order;  // 0: XCD bands of tile rows (xcd_remap, as k_pcg1); 1: block b = tile b (XCDs interleaved)
};

__device__ __forceinline__ void tile_of(const Geo& g, int& i0, int& i1, int& c0) {
  const int id = g.order == 0 ? xcd_remap(blockIdx.x, gridDim.x) : int(blockIdx.x);
  const int ti = id / g.tiles_j, tj = id - ti * g.tiles_j;
  i0 = 2 + ti * g.TI;
  i1 = min(i0 + g.TI - 1, g.n - 3);
  c0 = 2 + tj * 124 - 2 + 2 * (threadIdx.x & 63);  // loaded column of the lane (16-B aligned)
}

template <int PF, int WORK>
__global__ void __launch_bounds__(64) k_reg(Geo g, const double* __restrict__ r, const double* __restrict__ p,
                                            double* __restrict__ rn, double* __restrict__ pn, double a,
                                            double* sink) {
  extern __shared__ double cap[];
  int i0, i1, c0;
  tile_of(g, i0, i1, c0);
  const int lane = threadIdx.x & 63;
  const bool own = lane >= 1 && lane <= 62 && c0 + 1 < g.n;
  const int mfirst = g.halo ? i0 - 2 : i0, mlast = g.halo ? i1 + 2 : i1 + 1;
  double2 br[PF + 1], bp[PF + 1];
  auto fetch = [&](int m, double2& x, double2& y) {
    m = min(m, mlast);
    x = *reinterpret_cast<const double2*>(r + size_t(m) * g.pitch + c0);
    y = *reinterpret_cast<const double2*>(p + size_t(m) * g.pitch + c0);
  };
#pragma unroll
  for (int q = 0; q < PF; ++q) fetch(mfirst + q, br[q], bp[q]);
  double acc = 0.0;
  double x[2] = {0, 0}, y[2] = {0, 0};
  for (int m = mfirst; m <= mlast; m += PF + 1) {
#pragma unroll
    for (int q = 0; q <= PF; ++q) {
      const int mm = m + q;
      if (mm > mlast) goto done;
      fetch(mm + PF, br[(q + PF) % (PF + 1)], bp[(q + PF) % (PF + 1)]);
      x[0] += br[q].x; x[1] += br[q].y; y[0] += bp[q].x; y[1] += bp[q].y;
      work<WORK>(x, y, a);
      x[0] += shl(y[1]);
      if (mm - 1 >= i0 && mm - 1 <= i1 && own) {
        const size_t o = size_t(mm - 1) * g.pitch + c0;
        __builtin_nontemporal_store((d2v){x[0], x[1]}, reinterpret_cast<d2v*>(rn + o));
        __builtin_nontemporal_store((d2v){y[0], y[1]}, reinterpret_cast<d2v*>(pn + o));
      }
      acc += x[0] * y[1];
    }
  }
done:
  if (acc == 12345.678) sink[0] = acc + cap[0];
}

// r and p interleaved in one array (per 2-column pair: r r p p), rows 2*pitch apart: a wave reads
// and writes one contiguous 2 KiB chunk per row instead of two 1-KiB chunks 1 field apart
template <int PF, int WORK>
__global__ void __launch_bounds__(64) k_il(Geo g, const double* __restrict__ rp, const double* __restrict__ unused,
                                           double* __restrict__ rpn, double* __restrict__ unused2, double a,
                                           double* sink) {
  extern __shared__ double cap[];
  int i0, i1, c0;
  tile_of(g, i0, i1, c0);
  const int lane = threadIdx.x & 63;
  const bool own = lane >= 1 && lane <= 62 && c0 + 1 < g.n;
  const int mfirst = g.halo ? i0 - 2 : i0, mlast = g.halo ? i1 + 2 : i1 + 1;
  const size_t P2 = size_t(2) * g.pitch;
  double2 br[PF + 1], bp[PF + 1];
  auto fetch = [&](int m, double2& x, double2& y) {
    m = min(m, mlast);
    const double* q = rp + size_t(m) * P2 + 2 * c0;
    x = *reinterpret_cast<const double2*>(q);
    y = *reinterpret_cast<const double2*>(q + 2);
  };
#pragma unroll
  for (int q = 0; q < PF; ++q) fetch(mfirst + q, br[q], bp[q]);
  double acc = 0.0;
  double x[2] = {0, 0}, y[2] = {0, 0};
  for (int m = mfirst; m <= mlast; m += PF + 1) {
#pragma unroll
    for (int q = 0; q <= PF; ++q) {
      const int mm = m + q;
      if (mm > mlast) goto done;
      fetch(mm + PF, br[(q + PF) % (PF + 1)], bp[(q + PF) % (PF + 1)]);
      x[0] += br[q].x; x[1] += br[q].y; y[0] += bp[q].x; y[1] += bp[q].y;
      work<WORK>(x, y, a);
      x[0] += shl(y[1]);
      if (mm - 1 >= i0 && mm - 1 <= i1 && own) {
        double* o = rpn + size_t(mm - 1) * P2 + 2 * c0;
        __builtin_nontemporal_store((d2v){x[0], x[1]}, reinterpret_cast<d2v*>(o));
        __builtin_nontemporal_store((d2v){y[0], y[1]}, reinterpret_cast<d2v*>(o + 2));
      }
      acc += x[0] * y[1];
    }
  }
done:
  if (acc == 12345.678) sink[0] = acc + cap[0];
}

// Register prefetch (PF 1) like k_reg, but the march split into phases (3 steps without stores, a
// steady loop whose every step stores, one last step without) and the stores issued for all 64
// lanes as buffer stores whose non-owned lanes get an out-of-range offset (dropped by the range
// check): no store is conditional, so the compiler's vmcnt wait for the prefetched row counts the
// previous step's stores as younger ops instead of waiting for their acknowledgement.
__device__ __forceinline__ void st_rows(const double* base, unsigned voff, d2v v) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), 0, 0x7fffffff, 0x00020000);
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), rs, voff, 0, 2);  // aux 2: nt
}

template <int WORK>
__global__ void __launch_bounds__(64) k_regp(Geo g, const double* __restrict__ r, const double* __restrict__ p,
                                             double* __restrict__ rn, double* __restrict__ pn, double a,
                                             double* sink) {
  extern __shared__ double cap[];
  int i0, i1, c0;
  tile_of(g, i0, i1, c0);
  const int lane = threadIdx.x & 63;
  const bool own = lane >= 1 && lane <= 62 && c0 + 1 < g.n;
  const unsigned soff = own ? unsigned(c0) * 8u : 0x80000000u;  // dropped lanes: out of range
  const int mfirst = i0 - 2, mlast = i1 + 2;
  const int h = i1 - i0 + 1;
  double2 br[2], bp[2];
  auto fetch = [&](int m, double2& x, double2& y) {
    m = min(m, mlast);
    x = *reinterpret_cast<const double2*>(r + size_t(m) * g.pitch + c0);
    y = *reinterpret_cast<const double2*>(p + size_t(m) * g.pitch + c0);
  };
  double acc = 0.0;
  double x[2] = {0, 0}, y[2] = {0, 0};
  auto body = [&](int t, const double2& cr, const double2& cp, bool store) {
    x[0] += cr.x; x[1] += cr.y; y[0] += cp.x; y[1] += cp.y;
    work<WORK>(x, y, a);
    x[0] += shl(y[1]);
    if (store) {
      const size_t o = size_t(mfirst + t - 1) * g.pitch;
      st_rows(rn + o, soff, (d2v){x[0], x[1]});
      st_rows(pn + o, soff, (d2v){y[0], y[1]});
    }
    acc += x[0] * y[1];
  };
  fetch(mfirst, br[0], bp[0]);
  // steps 0 .. 2: no stores
  fetch(mfirst + 1, br[1], bp[1]); body(0, br[0], bp[0], false);
  fetch(mfirst + 2, br[0], bp[0]); body(1, br[1], bp[1], false);
  fetch(mfirst + 3, br[1], bp[1]); body(2, br[0], bp[0], false);
  // steps 3 .. h+2: every step stores (two steps per trip, so the ring needs no copies)
  int t = 3;
  for (; t + 1 <= h + 2; t += 2) {
    fetch(mfirst + t + 1, br[0], bp[0]); body(t, br[1], bp[1], true);
    fetch(mfirst + t + 2, br[1], bp[1]); body(t + 1, br[0], bp[0], true);
  }
  if (t <= h + 2) {
    fetch(mfirst + t + 1, br[0], bp[0]); body(t, br[1], bp[1], true);
    body(t + 1, br[0], bp[0], false);  // the last step (t + 1 = h + 3)
  } else {
    body(t, br[1], bp[1], false);
  }
  if (acc == 12345.678) sink[0] = acc + cap[0];
}

// NW waves per workgroup march NW side-by-side column tiles of one tile row in lockstep (an
// s_barrier per row step): each row step of the workgroup reads NW KiB contiguous per field.
template <int NW, int WORK>
__global__ void __launch_bounds__(64 * NW) k_lock(Geo g, const double* __restrict__ r, const double* __restrict__ p,
                                                 double* __restrict__ rn, double* __restrict__ pn, double a,
                                                 double* sink) {
  extern __shared__ double cap[];
  const int wid = int(threadIdx.x >> 6);
  const int gtj = (g.tiles_j + NW - 1) / NW;  // workgroup tiles per tile row
  const int id = g.order == 0 ? xcd_remap(blockIdx.x, gridDim.x) : int(blockIdx.x);
  const int ti = id / gtj, tjg = id - ti * gtj;
  const int tj = min(tjg * NW + wid, g.tiles_j - 1);
  const int i0 = 2 + ti * g.TI, i1 = min(i0 + g.TI - 1, g.n - 3);
  const int lane = threadIdx.x & 63;
  const int c0 = tj * 124 + 2 * lane;
  const bool own = lane >= 1 && lane <= 62 && c0 + 1 < g.n && tjg * NW + wid < g.tiles_j;
  const int mfirst = i0 - 2, mlast = i1 + 2;
  double2 br[2], bp[2];
  auto fetch = [&](int m, double2& x, double2& y) {
    m = min(m, mlast);
    x = *reinterpret_cast<const double2*>(r + size_t(m) * g.pitch + c0);
    y = *reinterpret_cast<const double2*>(p + size_t(m) * g.pitch + c0);
  };
  fetch(mfirst, br[0], bp[0]);
  double acc = 0.0;
  double x[2] = {0, 0}, y[2] = {0, 0};
  for (int m = mfirst; m <= mlast; m += 2) {
#pragma unroll
    for (int q = 0; q <= 1; ++q) {
      const int mm = m + q;
      if (mm > mlast) goto done;
      fetch(mm + 1, br[q ^ 1], bp[q ^ 1]);
      x[0] += br[q].x; x[1] += br[q].y; y[0] += bp[q].x; y[1] += bp[q].y;
      work<WORK>(x, y, a);
      x[0] += shl(y[1]);
      if (mm - 1 >= i0 && mm - 1 <= i1 && own) {
        const size_t o = size_t(mm - 1) * g.pitch + c0;
        __builtin_nontemporal_store((d2v){x[0], x[1]}, reinterpret_cast<d2v*>(rn + o));
        __builtin_nontemporal_store((d2v){y[0], y[1]}, reinterpret_cast<d2v*>(pn + o));
      }
      acc += x[0] * y[1];
      __builtin_amdgcn_s_barrier();
    }
  }
done:
  if (acc == 12345.678) sink[0] = acc + cap[0];
}

// one field only (r read, rn written): half the concurrent streams of k_reg
template <int WORK>
__global__ void __launch_bounds__(64) k_one(Geo g, const double* __restrict__ r, const double* __restrict__ p,
                                            double* __restrict__ rn, double* __restrict__ pn, double a,
                                            double* sink) {
  extern __shared__ double cap[];
  int i0, i1, c0;
  tile_of(g, i0, i1, c0);
  const int lane = threadIdx.x & 63;
  const bool own = lane >= 1 && lane <= 62 && c0 + 1 < g.n;
  const int mfirst = g.halo ? i0 - 2 : i0, mlast = g.halo ? i1 + 2 : i1 + 1;
  double2 br[2];
  br[0] = *reinterpret_cast<const double2*>(r + size_t(mfirst) * g.pitch + c0);
  double acc = 0.0;
  double x[2] = {0, 0}, y[2] = {0, 0};
  for (int m = mfirst; m <= mlast; m += 2) {
#pragma unroll
    for (int q = 0; q <= 1; ++q) {
      const int mm = m + q;
      if (mm > mlast) goto done;
      br[q ^ 1] = *reinterpret_cast<const double2*>(r + size_t(min(mm + 1, mlast)) * g.pitch + c0);
      x[0] += br[q].x; x[1] += br[q].y;
      work<WORK>(x, y, a);
      x[0] += shl(y[1]);
      if (mm - 1 >= i0 && mm - 1 <= i1 && own) {
        const size_t o = size_t(mm - 1) * g.pitch + c0;
        __builtin_nontemporal_store((d2v){x[0], x[1]}, reinterpret_cast<d2v*>(rn + o));
      }
      acc += x[0] * y[1];
    }
  }
done:
  if (acc == 12345.678) sink[0] = acc + cap[0];
}

// LDS-DMA: row m of r / p -> slot (m - mfirst) % PF of this wave's ring (1 KiB per field)
__device__ __forceinline__ void dma16(const double* base, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(base), "s"(lds)
               : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int PF, int WORK>
__global__ void __launch_bounds__(64) k_dma(Geo g, const double* __restrict__ r, const double* __restrict__ p,
                                            double* __restrict__ rn, double* __restrict__ pn, double a,
                                            double* sink) {
  extern __shared__ double ring[];  // [PF][2][64][2] doubles, then the occupancy cap
  int i0, i1, c0;
  tile_of(g, i0, i1, c0);
  const int lane = threadIdx.x & 63;
  const bool own = lane >= 1 && lane <= 62 && c0 + 1 < g.n;
  const int mfirst = i0 - 2, mlast = i1 + 2;
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(unsigned(reinterpret_cast<uintptr_t>(ring)));
  const unsigned voff = unsigned(c0) * 8u;
  auto fetch = [&](int m, int slot) {
    m = min(m, mlast);
    const double* rb = r + size_t(m) * g.pitch;
    const double* pb = p + size_t(m) * g.pitch;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this slot's ds_reads have returned
    dma16(rb, voff, lds0 + unsigned(slot) * 2048u);
    dma16(pb, voff, lds0 + unsigned(slot) * 2048u + 1024u);
  };
#pragma unroll
  for (int q = 0; q < PF; ++q) fetch(mfirst + q, q);
  double acc = 0.0;
  double x[2] = {0, 0}, y[2] = {0, 0};
  // stores happen on steps t = 3 .. h+2 (h = i1 - i0 + 1); the wait for row t must count the
  // stores issued after its DMA: steps t-PF .. t-1 (2 store instructions each)
  const int h = i1 - i0 + 1;
  int slot = 0;
  auto step = [&](int t, auto ks) {
    constexpr int KS = decltype(ks)::value;
    wait_vm<2 * (PF - 1) + 2 * KS>();
    const double* sl = ring + slot * 256;
    const double2 rv = *reinterpret_cast<const double2*>(sl + 2 * lane);
    const double2 pv = *reinterpret_cast<const double2*>(sl + 128 + 2 * lane);
    fetch(mfirst + t + PF, slot);
    slot = slot + 1 == PF ? 0 : slot + 1;
    x[0] += rv.x; x[1] += rv.y; y[0] += pv.x; y[1] += pv.y;
    work<WORK>(x, y, a);
    x[0] += shl(y[1]);
    const int mm = mfirst + t;
    if (t >= 3 && t <= h + 2) {
      if (own) {
        const size_t o = size_t(mm - 1) * g.pitch + c0;
        __builtin_nontemporal_store((d2v){x[0], x[1]}, reinterpret_cast<d2v*>(rn + o));
        __builtin_nontemporal_store((d2v){y[0], y[1]}, reinterpret_cast<d2v*>(pn + o));
      }
    }
    acc += x[0] * y[1];
  };
  using I0 = std::integral_constant<int, 0>;
  step(0, I0{});
  step(1, I0{});
  step(2, I0{});
  // ramp: the first PF store steps (t = 3 .. 2+PF) see 0 .. PF-1 stores behind their row's DMA
  [&]<int... K>(std::integer_sequence<int, K...>) {
    (step(3 + K, std::integral_constant<int, K>{}), ...);
  }(std::make_integer_sequence<int, PF>{});
  for (int t = 3 + PF; t <= h + 3; ++t) step(t, std::integral_constant<int, PF>{});
  wait_vm<0>();
  if (acc == 12345.678) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 16384;
  const int ncand = argc > 2 ? atoi(argv[2]) : 8;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  const int pitch = ((n + 128 + 31) / 32) * 32;  // the last column tile loads up to column n + 111
  const size_t fb = size_t(n) * pitch * 8;
  std::vector<double*> blocks;
  for (int c = 0; c < ncand; ++c) {
    double* b = nullptr;
    CK(hipMalloc(&b, 4 * fb));
    CK(hipMemset(b, 0, 4 * fb));
    blocks.push_back(b);
  }
  double* sink = nullptr;
  CK(hipMalloc(&sink, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V {
    const char* name;
    void (*k)(Geo, const double*, const double*, double*, double*, double, double*);
    int pf, dma;
  };
  const V vars[] = {
      {"reg1", k_reg<1, 6>, 1, 0}, {"lock2", k_lock<2, 6>, 1, 2}, {"lock4", k_lock<4, 6>, 1, 4},
      {"lock8", k_lock<8, 6>, 1, 8},
  };
  const int tis[] = {4, 8};
  const int wpcu[] = {8, 12, 16};
  printf("n=%d pitch=%d candidates=%d reps=%d (ms per sweep; GB/s at 32 B/pt)\n", n, pitch, ncand, reps);
  for (int order = 0; order <= 0; ++order)
  for (int TI : tis) {
    Geo g{n, pitch, TI, (n - 4 + TI - 1) / TI, (n - 4 + 123) / 124, 1, order};
    for (int wc : wpcu) {
      for (const V& v : vars) {
        // lock variants: v.dma = waves per workgroup (side-by-side column tiles)
        const bool lock = v.name[0] == 'l';
        const int nw = lock ? v.dma : 1;
        const int nb = lock ? g.tiles_i * ((g.tiles_j + nw - 1) / nw) : g.tiles_i * g.tiles_j;
        const int bs = 64 * nw;
        const size_t ring = (v.dma && !lock) ? size_t(v.pf) * 2048 : 0;
        const size_t lds = std::min(size_t(163840), std::max(ring, (size_t(163840 / wc) * nw) & ~size_t(255)));
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(v.k), hipFuncAttributeMaxDynamicSharedMemorySize,
                               int(lds)));
        printf("order=%d TI=%2d waves/CU=%2d %-5s:", order, TI, wc, v.name);
        std::vector<float> ms;
        for (int c = 0; c < ncand; ++c) {
          double* b = blocks[c];
          double *r = b, *p = b + fb / 8, *rn = b + 2 * (fb / 8), *pn = b + 3 * (fb / 8);
          hipLaunchKernelGGL(v.k, dim3(nb), dim3(bs), lds, 0, g, r, p, rn, pn, 1e-3, sink);
          CK(hipEventRecord(e0));
          for (int k = 0; k < reps; ++k) {
            if (k & 1)
              hipLaunchKernelGGL(v.k, dim3(nb), dim3(bs), lds, 0, g, rn, pn, r, p, 1e-3, sink);
            else
              hipLaunchKernelGGL(v.k, dim3(nb), dim3(bs), lds, 0, g, r, p, rn, pn, 1e-3, sink);
          }
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float t = 0;
          CK(hipEventElapsedTime(&t, e0, e1));
          ms.push_back(t / reps);
          printf(" %.3f", t / reps);
        }
        const float mn = *std::min_element(ms.begin(), ms.end()), mx = *std::max_element(ms.begin(), ms.end());
        printf(" | min %.3f max %.3f ratio %.3f  %.0f GB/s\n", mn, mx, mx / mn,
               32.0 * (n - 4.0) * (n - 4.0) / (mn * 1e-3) / 1e9);
        fflush(stdout);
      }
    }
  }
  // correctness of the DMA ring: the two kernels must store identical rn/pn
  {
    Geo g{n, pitch, 8, (n - 4 + 7) / 8, (n - 4 + 123) / 124, 1, 0};
    const int nb = g.tiles_i * g.tiles_j;
    double* b = blocks[0];
    double *r = b, *p = b + fb / 8, *rn = b + 2 * (fb / 8), *pn = b + 3 * (fb / 8);
    std::vector<double> h(size_t(n) * pitch);
    for (size_t i = 0; i < h.size(); ++i) h[i] = double((i * 2654435761u) % 1000) * 1e-3;
    CK(hipMemcpy(r, h.data(), fb, hipMemcpyHostToDevice));
    for (size_t i = 0; i < h.size(); ++i) h[i] = double((i * 40503u) % 777) * 1e-3;
    CK(hipMemcpy(p, h.data(), fb, hipMemcpyHostToDevice));
    std::vector<double> a1(h.size()), a2(h.size());
    CK(hipMemset(rn, 0, fb));
    hipLaunchKernelGGL((k_reg<1, 6>), dim3(nb), dim3(64), 0, 0, g, r, p, rn, pn, 1e-3, sink);
    CK(hipMemcpy(a1.data(), rn, fb, hipMemcpyDeviceToHost));
    for (int pf = 2; pf <= 4; ++pf) {
      CK(hipMemset(rn, 0, fb));
      auto k = pf == 2 ? k_dma<2, 6> : pf == 3 ? k_dma<3, 6> : k_dma<4, 6>;
      hipLaunchKernelGGL(k, dim3(nb), dim3(64), pf * 2048, 0, g, r, p, rn, pn, 1e-3, sink);
      CK(hipMemcpy(a2.data(), rn, fb, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (size_t i = 0; i < a1.size(); ++i) bad += a1[i] != a2[i];
      printf("check dma%d vs reg1: %zu mismatches of %zu\n", pf, bad, a1.size());
    }
  }
  return 0;
}
