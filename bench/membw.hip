// Memory-system ceiling study for the PCG access pattern on MI355X.
//
// Measures, on fp64 arrays of N x N (pitch N+32):
//   copy      : 1 read + 1 write, contiguous grid-stride, 16 B/lane
//   stream5   : 3 reads + 2 writes (the k_pcg_b traffic), contiguous grid-stride, 16 B/lane
//   march5    : the same 5 streams, but each 256-thread block marches `rows` rows of a
//               512-column strip (the tile-marching order of the fused kernels)
//   rowband5  : 5 streams, one block per (row, 512-col chunk), rows assigned so that each XCD
//               works on its own contiguous band of rows (T1-style XCD-aware mapping)
//   mix_2r2w  : the k_pcg1 odd-iteration traffic: read 2 arrays, write 2 OTHER arrays (rowband
//               mapping, XCD-aware); mix_3r3w: the even one (+ a third array read and written
//               in place)
// Usage: membw [N] [rows] [reps] [fill]   (reps = timed launches per kernel, default 10; fill 1 =
// non-zero data: HBM power depends on the bit patterns, and sustained runs of >= 1 s show the
// clock/power-limited steady state instead of the first-launch burst)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);          \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void __launch_bounds__(256) k_copy(const double2* a, double2* b, size_t n2) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n2; i += size_t(gridDim.x) * 256) b[i] = a[i];
}

__global__ void __launch_bounds__(256)
k_stream5(const double2* p, double2* w, double2* r, size_t n2, double al) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n2; i += size_t(gridDim.x) * 256) {
    double2 pv = p[i], wv = w[i], rv = r[i];
    wv.x += al * pv.x; wv.y += al * pv.y;
    rv.x -= al * pv.y; rv.y -= al * pv.x;
    w[i] = wv; r[i] = rv;
  }
}

// tile = rows x 512 columns, 256 threads x 2 columns, marching down
__global__ void __launch_bounds__(256)
k_march5(const double* p, double* w, double* r, int n, int pitch, int rows, int tiles_j, double al) {
  const int ti = blockIdx.x / tiles_j, tj = blockIdx.x % tiles_j;
  const int j = tj * 512 + 2 * threadIdx.x;
  const int i0 = ti * rows;
  for (int i = i0; i < i0 + rows && i < n; ++i) {
    const size_t c = size_t(i) * pitch + j;
    double2 pv = *(const double2*)(p + c), wv = *(double2*)(w + c), rv = *(double2*)(r + c);
    wv.x += al * pv.x; wv.y += al * pv.y;
    rv.x -= al * pv.y; rv.y -= al * pv.x;
    *(double2*)(w + c) = wv;
    *(double2*)(r + c) = rv;
  }
}

// wave tiles: each wave marches `rows` rows of a (64*VEC)-column strip; layout 0 = row-major
// (pitch), layout 1 = panel-major (each strip's rows contiguous: one sequential stream per wave)
template <int VEC>
__global__ void __launch_bounds__(256)
k_wavemarch5(const double* p, double* w, double* r, int n, int pitch, int rows, int tiles_j,
             int layout, double al) {
  constexpr int W = 64 * VEC;
  const int wid = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int ti = wid / tiles_j, tj = wid % tiles_j;
  const int i0 = ti * rows;
  if (i0 >= n) return;
  for (int i = i0; i < i0 + rows && i < n; ++i) {
    size_t c;
    if (layout == 0) c = size_t(i) * pitch + tj * W + lane * VEC;
    else c = (size_t(tj) * n + i) * W + lane * VEC;
#pragma unroll
    for (int u = 0; u < VEC; u += 2) {
      double2 pv = *(const double2*)(p + c + u), wv = *(double2*)(w + c + u), rv = *(double2*)(r + c + u);
      wv.x += al * pv.x; wv.y += al * pv.y;
      rv.x -= al * pv.y; rv.y -= al * pv.x;
      *(double2*)(w + c + u) = wv;
      *(double2*)(r + c + u) = rv;
    }
  }
}

// one block per (row, 512-col chunk); block b -> XCD b%8 gets rows [xcd*n/8, (xcd+1)*n/8)
__global__ void __launch_bounds__(256)
k_rowband5(const double* p, double* w, double* r, int n, int pitch, int chunks, double al, int xcd_aware) {
  int b = blockIdx.x;
  const int nb = gridDim.x;
  if (xcd_aware) {
    const int per = nb / 8;  // nb multiple of 8
    b = (blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  const int i = b / chunks, jc = b % chunks;
  if (i >= n) return;
  const int j = jc * 512 + 2 * threadIdx.x;
  const size_t c = size_t(i) * pitch + j;
  double2 pv = *(const double2*)(p + c), wv = *(double2*)(w + c), rv = *(double2*)(r + c);
  wv.x += al * pv.x; wv.y += al * pv.y;
  rv.x -= al * pv.y; rv.y -= al * pv.x;
  *(double2*)(w + c) = wv;
  *(double2*)(r + c) = rv;
}

struct Ptrs {
  double* a[5];
};
// reads a[0..NR-1]; writes a[NR], a[NR+1] (separate arrays) and, if WIN, a[NR-1] in place
template <int NR, bool WIN>
__global__ void __launch_bounds__(256) k_mix(Ptrs P, int n, int pitch, int chunks) {
  const int nb = gridDim.x, per = nb / 8;
  const int b = (blockIdx.x % 8) * per + blockIdx.x / 8;
  const int i = b / chunks, jc = b % chunks;
  if (i >= n) return;
  const size_t c = size_t(i) * pitch + jc * 512 + 2 * threadIdx.x;
  double2 v[NR];
#pragma unroll
  for (int q = 0; q < NR; ++q) v[q] = *(const double2*)(P.a[q] + c);
  double2 o0 = v[0], o1 = v[1];
  o0.x += 0.5 * v[1].y; o1.y -= 0.5 * v[0].x;
  *(double2*)(P.a[NR] + c) = o0;
  *(double2*)(P.a[NR + 1] + c) = o1;
  if constexpr (WIN) {
    double2 wv = v[NR - 1];
    wv.x += 0.25 * o0.y; wv.y += 0.25 * o1.x;
    *(double2*)(P.a[NR - 1] + c) = wv;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 16384;
  const int rows = argc > 2 ? atoi(argv[2]) : 64;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  const int fill = argc > 4 ? atoi(argv[4]) : 0;
  const int pitch = n + 32;
  const size_t elems = size_t(n) * pitch;
  const size_t bytes = elems * 8;
  double *p, *w, *r;
  CK(hipMalloc(&p, bytes));
  CK(hipMalloc(&w, bytes));
  CK(hipMalloc(&r, bytes));
  CK(hipMemset(p, 0, bytes));
  CK(hipMemset(w, 0, bytes));
  CK(hipMemset(r, 0, bytes));
  if (fill) {  // pseudo-random doubles in [0.5, 1): the +/-0.5 updates keep them finite
    std::vector<double> h(elems);
    unsigned long long x = 88172645463325252ull;
    for (auto& v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = 0.5 + double(x >> 11) * 0x1.0p-54; }
    CK(hipMemcpy(p, h.data(), bytes, hipMemcpyHostToDevice));
    CK(hipMemcpy(w, h.data(), bytes, hipMemcpyHostToDevice));
    CK(hipMemcpy(r, h.data(), bytes, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double gb, auto launch) {
    for (int w_ = 0; w_ < 3; ++w_) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int k = 0; k < reps; ++k) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("{\"kernel\": \"%s\", \"n\": %d, \"reps\": %d, \"fill\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n", name, n,
           reps, fill, ms, gb / ms);
    fflush(stdout);
  };
  const size_t n2 = elems / 2;
  const double gb_copy = 2.0 * bytes / 1e9, gb5 = 5.0 * bytes / 1e9;
  timeit("copy", gb_copy, [&] { hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, (const double2*)p, (double2*)w, n2); });
  timeit("stream5", gb5, [&] { hipLaunchKernelGGL(k_stream5, dim3(8192), dim3(256), 0, 0, (const double2*)p, (double2*)w, (double2*)r, n2, 0.5); });
  const int tiles_j = n / 512;
  for (int rw : {rows, 16, 4, 1}) {
    const int tiles_i = (n + rw - 1) / rw;
    char name[64];
    snprintf(name, sizeof name, "march5_rows%d", rw);
    timeit(name, gb5, [&] { hipLaunchKernelGGL(k_march5, dim3(tiles_i * tiles_j), dim3(256), 0, 0, p, w, r, n, pitch, rw, tiles_j, 0.5); });
  }
  for (int layout : {0, 1}) {
    for (int rw : {64, 16}) {
      {
        const int tj = n / 128, waves = tj * ((n + rw - 1) / rw);
        char name[96];
        snprintf(name, sizeof name, "wavemarch5_v2_rows%d_%s", rw, layout ? "panel" : "rowmajor");
        timeit(name, gb5, [&] { hipLaunchKernelGGL((k_wavemarch5<2>), dim3((waves + 3) / 4), dim3(256), 0, 0, p, w, r, n, pitch, rw, tj, layout, 0.5); });
      }
      {
        const int tj = n / 512, waves = tj * ((n + rw - 1) / rw);
        char name[96];
        snprintf(name, sizeof name, "wavemarch5_v8_rows%d_%s", rw, layout ? "panel" : "rowmajor");
        timeit(name, gb5, [&] { hipLaunchKernelGGL((k_wavemarch5<8>), dim3((waves + 3) / 4), dim3(256), 0, 0, p, w, r, n, pitch, rw, tj, layout, 0.5); });
      }
    }
  }
  const int chunks = n / 512;
  timeit("rowband5_rowmajor", gb5, [&] { hipLaunchKernelGGL(k_rowband5, dim3(n * chunks), dim3(256), 0, 0, p, w, r, n, pitch, chunks, 0.5, 0); });
  timeit("rowband5_xcd", gb5, [&] { hipLaunchKernelGGL(k_rowband5, dim3(n * chunks), dim3(256), 0, 0, p, w, r, n, pitch, chunks, 0.5, 1); });
  {
    double *c, *d;
    CK(hipMalloc(&c, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemcpy(c, p, bytes, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(d, p, bytes, hipMemcpyDeviceToDevice));
    const int nblk = ((n * chunks + 7) / 8) * 8;
    Ptrs odd{{p, r, c, d, nullptr}}, even{{p, r, w, c, d}};
    timeit("mix_2r2w", 4.0 * bytes / 1e9, [&] { hipLaunchKernelGGL((k_mix<2, false>), dim3(nblk), dim3(256), 0, 0, odd, n, pitch, chunks); });
    timeit("mix_3r3w", 6.0 * bytes / 1e9, [&] { hipLaunchKernelGGL((k_mix<3, true>), dim3(nblk), dim3(256), 0, 0, even, n, pitch, chunks); });
    CK(hipFree(c));
    CK(hipFree(d));
  }
  return 0;
}
