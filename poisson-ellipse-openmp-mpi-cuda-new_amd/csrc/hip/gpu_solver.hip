// GPU PCG subdomain solver (GpuSubdomainSolver: fields, tables, placement probe, kernels, checkpoints).
// See pmx/gpu_solver.hpp.  The iteration driver (PcgDriver: streams, graphs, batches, phase buckets)
// is in pcg_driver.hip; the s-step solver's passes and its driver schedule in ca_solver.hip, pcg1's
// decomposed-grid schedules in pcg1_driver.hip.
//
// Reference call stack being replaced (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:688-983): CPU
// assembly + 3 H2D copies, 8 cudaMallocs, and per iteration 8 launches each followed by
// cudaDeviceSynchronize, 3x256-KiB partial D2H copies with host summation, host-staged halos.
// Here per iteration: 4 launches (2 streaming + 2 single-block reductions), zero host syncs,
// replayed from a hipGraph in batches.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <unistd.h>
#include <string>
#include <vector>
#include <istream>
#include <ostream>

#include "pmx/common.hpp"
#include "pmx/gpu_solver.hpp"
#include "pmx/session.hpp"
#include "pmx/trace.hpp"

namespace pmx {

namespace {
size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

DevGeom make_dev_geom(const ProblemSpec& spec, const Subdomain& sd, int64_t pitch) {
  const GridInfo g(spec);
  DevGeom G{};
  G.nx = sd.nx;
  G.ny = sd.ny;
  G.pitch = pitch;
  G.gi0 = sd.gi0();
  G.gj0 = sd.gj0();
  G.M = spec.M;
  G.N = spec.N;
  G.nb = 0;  // slot s <-> bit 1 << s (kNbXlo .. kNbXhiYhi)
  for (int s = 0; s < kHaloSlots; ++s) G.nb |= sd.peer(s) >= 0 ? 1 << s : 0;
  G.ref_ellipse = spec.reference_ellipse() ? 1 : 0;
  G.h1 = g.h1; G.h2 = g.h2; G.eps = g.eps; G.inv_eps = g.inv_eps; G.h1h2 = g.h1h2;
  G.cx = 1.0 / (g.h1 * g.h1);
  G.cy = 1.0 / (g.h2 * g.h2);
  G.dinv_in = 1.0 / ((1.0 + 1.0) * G.cx + (1.0 + 1.0) * G.cy);
  G.dinv_out = 1.0 / ((g.inv_eps + g.inv_eps) * G.cx + (g.inv_eps + g.inv_eps) * G.cy);
  G.ax = spec.ax; G.by = spec.by; G.F = spec.F;
  return G;
}

DevTables upload_tables(const ProblemSpec& spec, double** owner) {
  const GridInfo g(spec);
  const geo::FaceTables ft(spec, g);
  const size_t nxT = spec.M + 2, nyT = spec.N + 2;
  const size_t ndbl = 4 * nxT + 4 * nyT, nint = 8 * nxT;
  HIP_CHECK(hipMalloc(owner, ndbl * sizeof(double) + nint * sizeof(int)));
  std::vector<double> host(ndbl);
  double* h = host.data();
  std::memcpy(h + 0 * nxT, ft.rv.data(), nxT * 8);
  std::memcpy(h + 1 * nxT, ft.xlo.data(), nxT * 8);
  std::memcpy(h + 2 * nxT, ft.xhi.data(), nxT * 8);
  std::memcpy(h + 3 * nxT, ft.x.data(), nxT * 8);
  double* hy = h + 4 * nxT;
  std::memcpy(hy + 0 * nyT, ft.rh.data(), nyT * 8);
  std::memcpy(hy + 1 * nyT, ft.ylo.data(), nyT * 8);
  std::memcpy(hy + 2 * nyT, ft.yhi.data(), nyT * 8);
  std::memcpy(hy + 3 * nyT, ft.y.data(), nyT * 8);
  HIP_CHECK(hipMemcpy(*owner, host.data(), ndbl * 8, hipMemcpyHostToDevice));
  const double* d = *owner;
  const double* dy = d + 4 * nxT;
  int* cls = reinterpret_cast<int*>(*owner + ndbl);
  DevTables T{d, d + nxT, d + 2 * nxT, d + 3 * nxT, dy, dy + nyT, dy + 2 * nyT, dy + 3 * nyT,
              cls, cls + 4 * nxT};
  // classify every row on the device with the exact coefficient formulas
  Subdomain whole;
  whole.M = spec.M; whole.N = spec.N; whole.nx = spec.M - 1; whole.ny = spec.N - 1;
  launch_classify(make_dev_geom(spec, whole, spec.N + 2), T, cls, cls + 4 * nxT, nullptr);
  HIP_CHECK(hipDeviceSynchronize());
  return T;
}

namespace {
bool study_mode() {
  const char* e = std::getenv("PMX_STUDY");
  return e && e[0] == '1';
}
// one warning per process for knob variables that are set outside study mode
void warn_ignored_knobs() {
  static std::once_flag once;
  std::call_once(once, [] {
    std::string names;
    for (char** e = ::environ; e && *e; ++e) {
      const std::string kv = *e;
      const std::string k = kv.substr(0, kv.find('='));
      static const char* knobs[] = {"PMX_ALGO", "PMX_PAIR_W", "PMX_PCG1_", "PMX_CA_", "PMX_ARITH32", "PMX_PLACEMENT",
                                    "PMX_DIRECT_ROWS", "PMX_FRAME_ON_COMM", "PMX_FORK_ONE_QUEUE", "PMX_LOOPBACK_",
                                    "PMX_IPC_COARSE", "PMX_PROGRESS"};
      for (const char* p : knobs)
        if (k.rfind(p, 0) == 0) names += (names.empty() ? "" : ", ") + k;
    }
    if (!names.empty())
      std::fprintf(stderr, "pmx: ignoring %s (kernel / schedule study knobs apply only with PMX_STUDY=1)\n",
                   names.c_str());
  });
}
}  // namespace

const char* study_env(const char* name) {
  if (!study_mode()) {
    warn_ignored_knobs();
    return nullptr;
  }
  return std::getenv(name);
}

GpuOptions resolve_options(const GpuOptions& in) {
  if (in.resolved) return in;
  GpuOptions o = in;
  const bool study = study_mode();
  if (!study) warn_ignored_knobs();
  auto env_int = [study](const char* name, int& v) {
    if (!study) return;
    if (const char* e = std::getenv(name); e && e[0]) v = std::atoi(e);
  };
  env_int("PMX_PAIR_W", o.pair_w);
  env_int("PMX_ALGO", o.algo);
  env_int("PMX_PCG1_VEC", o.vec1);
  env_int("PMX_PCG1_ROWS", o.rows1);
  env_int("PMX_PCG1_ROWS_W", o.rows1w);
  env_int("PMX_PCG1_PF_W", o.pf1w);
  env_int("PMX_PCG1_WAVES", o.waves1);
  env_int("PMX_PCG1_WAVES_W", o.waves1w);
  env_int("PMX_PCG1_PF", o.pf1);
  env_int("PMX_PCG1_ORDER", o.order1);
  env_int("PMX_PCG1_WCYCLE", o.wcycle1);
  env_int("PMX_PROGRESS", o.progress);
  env_int("PMX_ARITH32", o.arith32);
  env_int("PMX_PLACEMENT", o.placement);
  env_int("PMX_PCG1_WPCU", o.wpcu1);
  env_int("PMX_PCG1_WPCU_W", o.wpcu1w);
  env_int("PMX_PCG1_BLOCK", o.block1);
  env_int("PMX_PCG1_BLOCK_ROWS", o.block_rows1);
  env_int("PMX_PCG1_BLOCK_WAVES", o.block_waves1);
  env_int("PMX_PCG1_BLOCK_FUSED", o.block_fused1);
  PMX_CHECK(o.block1 >= -1 && o.block1 <= 1, "block tiles must be -1 (auto), 0 or 1");
  PMX_CHECK(o.block_rows1 == 0 || pcg1_block_shape_ok(o.block_rows1, o.block_waves1),
            "block tiles: no " << o.block_rows1 << "-row x " << o.block_waves1 << "-wave variant (4/8/12/16 x 8, 8/16 x 16)");
  PMX_CHECK(o.block_waves1 == 8 || o.block_waves1 == 16, "block tiles: 8 or 16 waves per workgroup");
  PMX_CHECK(o.block_fused1 >= -1 && o.block_fused1 <= 1, "block-tile fused reduction must be -1 (auto), 0 or 1");
  env_int("PMX_CA_S", o.ca_s);
  env_int("PMX_CA_ROWS", o.ca_rows);
  env_int("PMX_CA_ROWS_UPD", o.ca_rows2);
  PMX_CHECK(o.ca_s == 2 || o.ca_s == 3, "s-step PCG: s must be 2 or 3");
  PMX_CHECK(o.ca_rows >= 0 && o.ca_rows <= 4096, "s-step PCG: tile rows must be 0 (auto) .. 4096");
  env_int("PMX_CA_DMA", o.ca_dma);
  env_int("PMX_CA_SPLIT", o.ca_split);
  env_int("PMX_CA_SPLIT_UPD", o.ca_split_upd);
  env_int("PMX_CA_FRAME_STREAM", o.ca_frame_stream);
  env_int("PMX_CA_FUSE", o.ca_fuse);
  env_int("PMX_CA_ROWS_F", o.ca_rows_f);
  PMX_CHECK(o.ca_fuse >= -1 && o.ca_fuse <= 1, "s-step PCG: ca_fuse must be -1, 0 or 1");
  PMX_CHECK(o.ca_rows_f >= 0 && o.ca_rows_f <= 4096, "s-step PCG: fused tile rows must be 0 (auto) .. 4096");
  env_int("PMX_CA_DIRICHLET", o.ca_dirichlet);
  if (const char* pk = study ? std::getenv("PMX_PLACEMENT_PICK") : nullptr; pk && pk[0])
    o.placement_pick = std::string(pk) == "slowest" ? 1 : 0;
  env_int("PMX_PCG1_SPLIT", o.split_sweep);
  PMX_CHECK(o.split_sweep >= -1 && o.split_sweep <= 1, "split_sweep must be -1, 0 or 1");
  PMX_CHECK(o.ca_split >= -1 && o.ca_split <= 1, "s-step PCG: ca_split must be -1, 0 or 1");
  PMX_CHECK(o.ca_split_upd >= -1 && o.ca_split_upd <= 1, "s-step PCG: ca_split_upd must be -1, 0 or 1");
  env_int("PMX_CA_WAVES_GRAM", o.ca_waves_gram);
  env_int("PMX_CA_WAVES_UPD", o.ca_waves_upd);
  PMX_CHECK(o.ca_dma >= -1 && o.ca_dma <= 1, "s-step PCG: ca_dma must be -1, 0 or 1");
  PMX_CHECK((o.ca_waves_gram == 2 || o.ca_waves_gram == 3) && (o.ca_waves_upd == 2 || o.ca_waves_upd == 3),
            "s-step PCG: waves per SIMD must be 2 or 3");
  env_int("PMX_PCG1_DMA", o.dma1);
  env_int("PMX_PCG1_DMA_W", o.dma1w);
  PMX_CHECK(o.dma1 == 0 || o.dma1 == 2 || o.dma1 == 3, "pcg1 LDS-DMA prefetch depth must be 0, 2 or 3");
  PMX_CHECK(o.dma1w == -1 || o.dma1w == 0 || o.dma1w == 2 || o.dma1w == 3,
            "pcg1 w-sweep LDS-DMA prefetch depth must be -1, 0, 2 or 3");
  PMX_CHECK(o.wpcu1 >= 0 && o.wpcu1 <= 32 && o.wpcu1w >= 0 && o.wpcu1w <= 32, "pcg1 waves per CU must be 0..32");
  PMX_CHECK(o.wcycle1 == 2 || o.wcycle1 == 3, "pcg1 w cycle must be 2 or 3");
  PMX_CHECK(o.pair_w >= 0 && o.pair_w <= 2, "pair_w must be 0, 1 or 2");
  PMX_CHECK(o.algo >= -1 && o.algo <= 3 && o.algo != 0, "algo must be -1, 1, 2 or 3");
  o.resolved = true;
  return o;
}

bool choose_single_pass(const ProblemSpec& spec, const ProcGrid& grid, const GpuOptions& o,
                        double device_total_bytes, int subdomains_per_device) {
  PMX_CHECK(o.resolved, "choose_single_pass needs resolve_options()");
  if (o.algo == 2 || o.algo == 3) return false;
  // the radius-2 halo takes two owned lines from every neighbour: each block needs >= 2 x 2
  const bool thick = grid.size() == 1 || ((spec.M - 1) / grid.Px >= 2 && (spec.N - 1) / grid.Py >= 2);
  const bool ok = !o.exact && o.kernel == 1 && thick;
  PMX_CHECK(o.algo != 1 || ok,
            "pcg1 needs the wave kernels, the fast arithmetic and subdomains of at least 2 x 2 nodes");
  if (o.algo == 1) return true;
  // auto: every storage type.  (Round 1 kept pcg2 for fp32 -- 32768^2: pcg1 8.99 ms vs pcg2 7.69 --
  // but with the scalar-cache row tables and short tiles pcg1 wins there too: 5.20 vs 7.08 ms,
  // 16384^2 1.41 vs 2.00 ms, profiles/r2/fp32_pcg1_sweep.txt)
  if (!ok) return false;
  if (device_total_bytes > 0) {  // the 5th field must fit (rank 0 holds the largest block)
    const Subdomain sd0 = decompose_2d(spec.M, spec.N, grid, 0);
    const double need = double(GpuSubdomainSolver::estimate_device_bytes(spec, sd0, o.dtype, true)) *
                        std::max(1, subdomains_per_device);
    if (need > 0.95 * device_total_bytes) return false;
  }
  return true;
}

int choose_algo(const ProblemSpec& spec, const ProcGrid& grid, const GpuOptions& o, double device_total_bytes,
                int subdomains_per_device, bool direct_rows) {
  PMX_CHECK(o.resolved, "choose_algo needs resolve_options()");
  if (o.algo == 3) return 3;  // validated by the solver
  if (o.algo == -1) {
    // one grid, or (native transports) row strips of >= 8 rows / 2-D blocks of >= 8 x 8 nodes (BASELINE
    // config 4: packed ghost rows, columns and corners once per block of s iterations)
    const bool strips = grid.size() == 1 || (direct_rows && (spec.M - 1) / grid.Px >= 8 &&
                                             (grid.Py == 1 || (spec.N - 1) / grid.Py >= 8));
    // every storage type: with fp32 / mixed fields the s-step keeps its basis and sums in fp64 registers
    // and beats pcg1 too (16384^2 0.951 vs 1.093 ms, 32768^2 3.356 vs 3.831; NOTES #124)
    bool ca = !o.exact && o.kernel == 1 && strips && int64_t(spec.M - 1) * (spec.N - 1) >= kCaAutoPoints;
    if (ca && device_total_bytes > 0) {  // rank 0 holds the largest strip
      const Subdomain sd0 = decompose_2d(spec.M, spec.N, grid, 0);
      const double need = double(GpuSubdomainSolver::estimate_device_bytes_algo(spec, sd0, o.dtype, 3)) *
                          std::max(1, subdomains_per_device);
      ca = need <= 0.95 * device_total_bytes;
    }
    if (ca) return 3;
  }
  return choose_single_pass(spec, grid, o, device_total_bytes, subdomains_per_device) ? 1 : 2;
}

CommLayout GpuSubdomainSolver::comm_layout(const Subdomain& sd, DType dtype, bool single_pass, int ca_gh) {
  CommLayout L;
  L.elem = dtype == DType::kFp64 ? 8 : 4;
  L.single_pass = single_pass;
  size_t off = 0;
  L.state_off = 0;
  off = round_up(sizeof(PcgState), 256);
  for (int s = 0; s < kHaloSlots; ++s) {
    L.peer[s] = sd.peer(s);
    // pcg2: one line of r per side; pcg1: 2 lines x (r, p) per side, one (r, p) per corner
    const int line = s < 2 ? sd.ny : sd.nx;
    L.edge_len[s] = single_pass ? (s < 4 ? 4 * line : 2) : (s < 4 ? line : 0);
    // s-step (packed, k_ca_halo): ca_gh lines x (z, p) per side, a ca_gh x ca_gh block per corner
    if (ca_gh > 0) L.edge_len[s] = 2 * ca_gh * (s < 4 ? line : ca_gh);
  }
  for (int s = 0; s < kHaloSlots; ++s) {
    L.send_off[s] = off;
    off = round_up(off + L.edge_len[s] * L.elem, 256);
  }
  for (int s = 0; s < kHaloSlots; ++s) {
    L.recv_off[s] = off;
    off = round_up(off + L.edge_len[s] * L.elem, 256);
  }
  L.bytes = off;
  return L;
}

GpuSubdomainSolver::GpuSubdomainSolver(const ProblemSpec& spec, const Subdomain& sd,
                                       const GpuOptions& opt, uintptr_t external_arena)
    : spec_(spec), sd_(sd), opt_(resolve_options(opt)), g_(spec) {
  spec.validate();
  PMX_CHECK(sd.nx >= 1 && sd.ny >= 1, "empty subdomain");
  HIP_CHECK(hipSetDevice(opt_.device));
  try {
    construct(external_arena);
  } catch (...) {
    release();  // the destructor does not run for a throwing constructor
    throw;
  }
}


void GpuSubdomainSolver::construct(uintptr_t external_arena) {
  const GpuOptions& opt = opt_;
  const ProblemSpec& spec = spec_;
  const Subdomain& sd = sd_;
  elem_ = opt.dtype == DType::kFp64 ? 8 : 4;
  const size_t align_elems = 256 / elem_;
  size_t free_b = 0, total_b = 0;
  HIP_CHECK(hipMemGetInfo(&free_b, &total_b));

  // iteration algorithm (see GpuOptions::algo); a Session resolves it once for all its solvers
  // (a standalone decomposed solver cannot know its transport: no s-step by auto there)
  if (opt_.algo == -1) opt_.algo = choose_algo(spec, sd.grid, opt_, double(total_b), 1, false);
  pcg1_ = opt_.algo == 1;
  ca_ = opt_.algo == 3;
  PMX_CHECK(!ca_ || (!opt.exact && sd.nx >= opt.ca_s && (sd.grid.Py == 1 || sd.ny >= opt.ca_s)),
            "s-step PCG (algo 3) runs the fast arithmetic, on subdomains of at least s rows (and s columns on "
            "2-D blocks)");
  // the s-step's fused pass (GpuOptions::ca_fuse) reads radius 2s: every subdomain must hold 2s rows (and
  // columns on 2-D blocks) -- decided from global data, so every rank runs the same schedule
  const bool fuse_ok = sd.grid.size() == 1 || ((spec.M - 1) / sd.grid.Px >= 2 * opt_.ca_s &&
                                               (sd.grid.Py == 1 || (spec.N - 1) / sd.grid.Py >= 2 * opt_.ca_s));
  PMX_CHECK(!ca_ || opt_.ca_fuse != 1 || fuse_ok, "the fused s-step pass needs subdomains of at least 2 s rows / columns");
  ca_fuse_ = ca_ && (opt_.ca_fuse == 1 || (opt_.ca_fuse == -1 && fuse_ok));
  // ghost rows per side: 2 (the single-pass radius-2 halo); a decomposed s-step subdomain needs s, 2s with
  // the fused pass (rows, and columns on 2-D blocks)
  gh_ = ca_ && sd.grid.size() > 1 ? (ca_fuse_ ? 2 * opt_.ca_s : opt_.ca_s) : 2;
  const bool ca_cols = ca_ && sd.grid.Py > 1;  // ghost columns: gh_ per side
  PMX_CHECK(!pcg1_ || (!opt.exact && opt.kernel == 1 && (sd.grid.size() == 1 || (sd.nx >= 2 && sd.ny >= 2))),
            "pcg1 needs the wave kernels, the fast arithmetic and a subdomain of at least 2 x 2 nodes");

  // +8 columns of padding: vector loads of VEC <= 4 columns starting at <= ny+3 stay in the row,
  // and the last padding element of a row is column -1 of the next one
  // (s-step blocks: + 2 gh + 8, so that the right ghost columns ny+1 .. ny+gh of a row and the left ones of
  // the next row -- that row's padding read as columns -gh .. -1 -- never overlap)
  geom_ = make_dev_geom(spec, sd,
                        int64_t(round_up(size_t(sd.ny + 2 + 8 + (ca_cols ? 2 * gh_ + 8 : 0)), align_elems)));
  const DevGeom& G = geom_;

  // fields: element (li, lj), li = -1 .. nx+2, at base[li*pitch + lj]; base = alloc + pitch +
  // (align-1) so that every interior row starts 256-B aligned (lj = 1)
  field_off_ = size_t(gh_ - 1) * size_t(G.pitch) + align_elems - 1;
  field_bytes_ = round_up((align_elems - 1 + size_t(sd.nx + 2 * gh_) * G.pitch) * elem_, 256);
  {  // fail with a sizing message instead of a bare hipErrorOutOfMemory
    const size_t need = estimate_device_bytes_algo(spec, sd, opt.dtype, opt_.algo);
    PMX_CHECK(need <= free_b,
              "subdomain " << sd.nx << "x" << sd.ny << " (" << (ca_ ? "s-step, 7" : pcg1_ ? "pcg1, 5" : "pcg2, 4")
                           << " fields) needs " << need / 1e9 << " GB on device " << opt.device
                           << " but only " << free_b / 1e9 << " of " << total_b / 1e9
                           << " GB are free; the largest square grid for this precision on one such "
                              "device is ~"
                           << max_square_grid(double(total_b), 1, opt.dtype) << "^2 (pmx --plan)");
  }
  // One allocation for all fields (field f at fields_ + f * field_bytes_).  The offset between the
  // fields (0 ... 8 MiB of stagger) and physically contiguous memory were measured: no gain
  // (profiles/r3/placement/stagger.log); where the block lands is what matters (place_fields).
  field_stride_ = field_bytes_;
  const int nfields = pcg1_ || ca_ ? 5 : 4;
  HIP_CHECK(hipMalloc(&fields_, size_t(nfields) * field_stride_));
  if (const char* e = std::getenv("PMX_DEBUG_ALLOC"); e && e[0] == '1')
    std::fprintf(stderr, "pmx alloc: fields %p (%zu B, mod 1G %zu, mod 2M %zu)\n", static_cast<void*>(fields_),
                 size_t(nfields) * field_stride_, size_t(reinterpret_cast<uintptr_t>(fields_) % (size_t(1) << 30)),
                 size_t(reinterpret_cast<uintptr_t>(fields_) % (size_t(1) << 21)));

  // 1D face tables
  tables_ = upload_tables(spec, &tables_buf_);
  ca_geom_ = geom_;
  ca_tables_ = tables_;
  if (ca_ && opt_.ca_dirichlet) {  // see ca_tables_
    const int o = geom_.gi0;
    ca_geom_.nb = 0;
    ca_geom_.gi0 = 0;
    ca_geom_.M = sd.nx + 1;
    if (sd.grid.Py > 1) {  // 2-D blocks: also Dirichlet across y, on the problem's columns 1 .. ny
      ca_geom_.gj0 = 0;
      ca_geom_.N = sd.ny + 1;
    }
    for (const double** t : {&ca_tables_.rv, &ca_tables_.xlo, &ca_tables_.xhi, &ca_tables_.x}) *t += o;
    ca_tables_.acls += 4 * o;
    ca_tables_.bcls += 4 * o;
  }
  ca_gh_ = ca_geom_.nb ? gh_ : 2;

  PMX_CHECK(opt.kernel == 1, "kernel must be 1 (wave tiles); the round-1 LDS-ring kernels are retired (bench/RETIRED.md)");
  // tile shapes per kernel (profiles/tile_counters_16384_fp64.md: pcg_a is fastest with 4
  // columns/lane, pcg_b with 2 in fp64; fp32 moves 16 B with 4 columns)
  const bool fp64 = opt.dtype == DType::kFp64;
  const int vec_a = opt.vec ? opt.vec : (opt.waves == 4 ? 4 : 2);  // (4, 4) is instantiated
  const int vec_b = opt.vec_b ? opt.vec_b : opt.vec ? opt.vec : (fp64 || opt.waves != 4 ? 2 : 4);
  const int waves_b = opt.waves_b ? opt.waves_b : opt.waves;
  const int rows_b = opt.tile_rows_b >= 0 ? opt.tile_rows_b : opt.tile_rows;
  // auto tile heights (caps and tile-count targets from bench/tile_sweep.py, see make_wave_tiles)
  tiles_ = make_wave_tiles(G, vec_a, opt.waves, opt.tile_rows, 32, 22000);
  if (opt.b_ring)
    tiles_b_ = make_wave_tiles(G, vec_b, waves_b, rows_b, 24, 66000);
  else  // default: ring-free 2-row tiles, independent of the pcg_a height
    tiles_b_ = make_row_tiles(G, vec_b, waves_b, opt.tile_rows_b >= 0 ? opt.tile_rows_b : 0);
  tiles_b_.pair_w = tiles_b_.kind == 2 && !opt.exact && opt_.pair_w != 0;

  if (pcg1_) {
    // block tiles (pcg1_block.hip): undecomposed fp64 grids, the three pipeline stages row-parallel
    // across a workgroup's 8 waves.  Auto where the march is latency-bound, by its four-row tile
    // count T4 (study r4ac, profiles/r4/block/, us/iteration block vs march): T4 < 1000 8-row tiles
    // (400x600 17.3 vs 37.1), T4 < 10000 12-row tiles (800x1200 23.9 vs 42.0, 1200x1800 39.1 vs
    // 54.1, 1600x2400 59.9 vs 61.2); above, the march (2000x3000 85.7 vs 76.1).  PMX_PCG1_BLOCK=0/1
    // forces it, PMX_PCG1_BLOCK_ROWS=4|8|12|16 and PMX_PCG1_BLOCK_WAVES=8|16 pick the shape.
    const int blk = opt_.block1;
    const int64_t t4 = int64_t((G.nx + 3) / 4) * ((G.ny + 123) / 124);
    if (G.nb == 0 && elem_ == 8 && (blk == 1 || (blk == -1 && t4 < 10000))) {
      const int rows = opt_.block_rows1 ? opt_.block_rows1 : t4 < 1000 ? 8 : 12;
      PMX_CHECK(pcg1_block_shape_ok(rows, opt_.block_waves1),
                "block tiles: no " << rows << "-row x " << opt_.block_waves1 << "-wave variant");
      block1_ = true;
      // the reduction folded into the sweep costs every workgroup a drain of its stores and a ticket
      // round trip while it holds its LDS: cheaper than a k_reduce_n launch when the tiles run in
      // about one round (400x600 16.8 vs 18.3 us, 800x1200 23.3 vs 24.6), dearer over several
      // (1200x1800 37.5 vs 37.2, 1600x2400 57.3 vs 54.9; study r4ap).  PMX_PCG1_BLOCK_FUSED=0/1 forces it.
      const int64_t nblk = int64_t((G.nx + rows - 1) / rows) * ((G.ny + 123) / 124);
      block_fused_ = opt_.block_fused1 >= 0 ? opt_.block_fused1 == 1 : nblk < 1500;
      opt_.rows1 = rows;
      opt_.rows1w = rows;
      opt_.vec1 = 2;
      opt_.waves1 = 1;
      opt_.waves1w = 1;
      opt_.pf1 = opt_.pf1w = 1;
    }
    tiles1_ = make_pcg1_tiles(G, opt_.vec1, opt_.waves1, opt_.rows1, opt_.pf1, int(elem_));
#ifdef PMX_WAVE_TRACE
    if (const char* e = std::getenv("PMX_WAVE_TRACE_IT"); e && e[0]) {
      wtrace_n_ = tiles1_.ntiles();
      wtrace_ = pcg1_wave_trace_setup(std::atoll(e), wtrace_n_);
    }
#endif
    r2_ = field_raw(4);
    tiles1_.arith32 = elem_ == 4 && opt_.arith32 ? 1 : 0;
    const int waves_w = opt_.waves1w ? opt_.waves1w : (opt_.waves1 == 8 ? 4 : opt_.waves1);
    tiles1w_ = make_pcg1_tiles(G, opt_.vec1, waves_w, opt_.rows1w ? opt_.rows1w : tiles1_.rows,
                               opt_.pf1w ? opt_.pf1w : tiles1_.pf, int(elem_));
    tiles1w_.arith32 = tiles1_.arith32;
    tiles1_.lds_pad = pcg1_lds_pad(opt_.wpcu1, tiles1_.waves);
    tiles1w_.lds_pad = pcg1_lds_pad(opt_.wpcu1w, tiles1w_.waves);
    if (block1_) tiles1_.bwaves = tiles1w_.bwaves = opt_.block_waves1;
    // the LDS-DMA march: fp64 with the default shape only (VEC 2, 1 wave, register prefetch 1)
    auto dma_ok = [&](const TileCfg& t) { return elem_ == 8 && t.vec == 2 && t.waves == 1 && t.pf == 1; };
    if (dma_ok(tiles1_)) tiles1_.dpf = opt_.dma1;
    if (dma_ok(tiles1w_)) tiles1w_.dpf = opt_.dma1w >= 0 ? opt_.dma1w : opt_.dma1;
    const bool same_w = tiles1w_.rows == tiles1_.rows && tiles1w_.waves == tiles1_.waves;
    // dispatch order tables with the tiles' row classes; order1: the ellipse-cut tiles first
    // within each XCD's share (their 3-5x longer tiles would trail the sweep)
    HIP_CHECK(hipMalloc(&tile_order_, pcg1_order_slots(tiles1_) * sizeof(Pcg1Slot)));
    slow_tiles_ = pcg1_build_order(G, tables_, tiles1_, tile_order_, opt_.order1 != 0, nullptr);
    if (same_w) {
      tiles1w_.order0 = tiles1_.order0;
      tiles1w_.order1 = tiles1_.order1;
      tiles1w_.order2 = tiles1_.order2;
      for (int q = 0; q < 3; ++q) tiles1w_.groups[q] = tiles1_.groups[q];
    } else {
      HIP_CHECK(hipMalloc(&tile_order_w_, pcg1_order_slots(tiles1w_) * sizeof(Pcg1Slot)));
      (void)pcg1_build_order(G, tables_, tiles1w_, tile_order_w_, opt_.order1 != 0, nullptr);
    }
  }

  if (ca_) {
    r2_ = field_raw(4);  // the second z buffer
    ca_tiles_ = make_ca_tiles(ca_geom_, opt_.ca_s, opt_.ca_rows, opt_.ca_rows2, opt_.ca_rows_f);
    ca_tiles_.fuse = ca_fuse_ ? 1 : 0;
    if (const char* e = study_env("PMX_CA_WAVES_F"); e && e[0]) ca_tiles_.waves_f = std::atoi(e);
    if (const char* e = study_env("PMX_CA_SPLIT_F"); e && e[0]) ca_tiles_.split_f = std::atoi(e);
    if (const char* e = study_env("PMX_CA_RG_F"); e && e[0]) ca_tiles_.rg_f = std::atoi(e);
    if (const char* e = study_env("PMX_CA_DMA_F"); e && e[0]) ca_tiles_.dma_f = std::atoi(e);
    if (const char* e = study_env("PMX_CA_FRAME_FIRST_F"); e && e[0]) ca_tiles_.frame_first_f = std::atoi(e);
    PMX_CHECK(ca_tiles_.dma_f == 0 || ca_tiles_.dma_f == 1, "s-step PCG: fused LDS-DMA rows must be 0 or 1");
    PMX_CHECK(ca_tiles_.rg_f == 1 || ca_tiles_.rg_f == 2 || ca_tiles_.rg_f == 4,
              "s-step PCG: fused row steps per barrier must be 1, 2 or 4");
    PMX_CHECK(ca_tiles_.waves_f == 2 || ca_tiles_.waves_f == 3, "s-step PCG: fused waves per SIMD must be 2 or 3");
    // the face coefficients of every node, read on the rows the ellipse cuts (2 more field-sized arrays)
    // fp64 whatever the fields' storage, in the fields' pitch (elements); column 1 of every row 256-B aligned
    const size_t face_off = size_t(gh_ - 1) * size_t(geom_.pitch) + 31;
    ca_face_bytes_ = round_up((31 + size_t(sd.nx + 2 * gh_) * size_t(geom_.pitch)) * 8, 256);
    HIP_CHECK(hipMalloc(&ca_faces_, 2 * ca_face_bytes_));
    ca_tiles_.fa = reinterpret_cast<const double*>(ca_faces_ + face_off * 8);
    ca_tiles_.fb = reinterpret_cast<const double*>(ca_faces_ + ca_face_bytes_ + face_off * 8);
    ca_tiles_.gh = ca_gh_;
    ca_build_faces(ca_geom_, ca_tables_, const_cast<double*>(ca_tiles_.fa), const_cast<double*>(ca_tiles_.fb), ca_gh_, nullptr);
    const bool split = opt_.ca_split == -1 ? geom_.nb != 0 : opt_.ca_split == 1;  // see GpuOptions::ca_split
    if (!split) ca_tiles_.split = 0;
    if (!(opt_.ca_split_upd == -1 ? split : opt_.ca_split_upd == 1)) ca_tiles_.split_upd = 0;
    if (!ca_tiles_.split) ca_tiles_.split_upd = ca_tiles_.split_upd && opt_.ca_split_upd == 1;
    ca_tiles_.dma = elem_ == 8 ? (opt_.ca_dma == -1 ? int(split) : opt_.ca_dma) : 0;  // LDS-DMA rows: fp64
    if (ca_tiles_.split && opt_.ca_frame_stream) {
      HIP_CHECK(hipStreamCreateWithFlags(&ca_side_, hipStreamNonBlocking));
      HIP_CHECK(hipEventCreateWithFlags(&ca_ev_fork_, hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&ca_ev_join_, hipEventDisableTiming));
    }
    ca_tiles_.waves_gram = opt_.ca_waves_gram;
    ca_tiles_.waves_upd = opt_.ca_waves_upd;
    HIP_CHECK(hipMalloc(&ca_tbl_, size_t(ca_tiles_.tiles_j) * ca_tiles_.cwords * sizeof(unsigned)));
    ca_tiles_.tbl = ca_tbl_;
    ca_build_classes(ca_geom_, ca_tables_, ca_tiles_, ca_tbl_, nullptr);
    if (ca_tiles_.fuse) {
      HIP_CHECK(hipMalloc(&ca_tbl_f_, size_t(ca_tiles_.tiles_j_f) * ca_tiles_.cwords * sizeof(unsigned)));
      ca_tiles_.tbl_f = ca_tbl_f_;
      ca_build_classes(ca_geom_, ca_tables_, ca_tiles_, ca_tbl_f_, nullptr, true);
    }
    HIP_CHECK(hipStreamSynchronize(nullptr));
    HIP_CHECK(hipMalloc(&ca_state_, sizeof(CaState)));
    HIP_CHECK(hipMemset(ca_state_, 0, sizeof(CaState)));
    HIP_CHECK(hipMalloc(&ca_chunk_, size_t(kCaReduceMaxBlocks) * ca_nq(ca_tiles_.s) * sizeof(double)));
  }
  init_tiles_ = make_tiles(G, 256, 0);
  // partials: 5 doubles per slot (the s-step Gram partials take ca_nq per tile)
  const int ca_slots =
      ca_ ? int((std::max(int64_t(ca_tiles_.ntiles()) * (ca_nq(ca_tiles_.s) - ca_tiles_.s) +
                              int64_t(ca_tiles_.ntiles2()) * ca_tiles_.s,
                          int64_t(ca_tiles_.fuse ? ca_tiles_.ntilesf() : 0) * ca_nq(ca_tiles_.s)) + 4) / 5)
          : 0;
  const size_t npart = size_t(std::max({tiles_.ntiles(), tiles_b_.ntiles(), init_tiles_.ntiles(),
                                        pcg1_ ? std::max(tiles1_.ntiles(), tiles1w_.ntiles()) : 0, ca_slots}));
  npart_ = npart;
  HIP_CHECK(hipMalloc(&partials_, (npart * 5 + kReduceWsDoubles) * sizeof(double)));
  reduce_ws_ = partials_ + npart * 5;
  HIP_CHECK(hipMemset(reduce_ws_, 0, kReduceWsDoubles * sizeof(double)));

  layout_ = comm_layout(sd, opt.dtype, pcg1_ || ca_, ca_ && sd.grid.size() > 1 ? gh_ : 0);
  if (external_arena) {
    arena_ = reinterpret_cast<char*>(external_arena);
    own_arena_ = false;
    PMX_CHECK(external_arena % 256 == 0, "external comm arena must be 256-B aligned");
  } else {
    HIP_CHECK(hipMalloc(&arena_, layout_.bytes));
    own_arena_ = true;
  }
  HIP_CHECK(hipMemset(arena_, 0, layout_.bytes));
  state_ = reinterpret_cast<PcgState*>(arena_ + layout_.state_off);
  HIP_CHECK(hipHostMalloc(&host_state_, 2 * sizeof(PcgState), hipHostMallocDefault));
  if (opt_.progress) {
    HIP_CHECK(hipHostMalloc(&progress_host_, 64, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(progress_host_, 0, 64);
    void* d = nullptr;
    HIP_CHECK(hipHostGetDevicePointer(&d, progress_host_, 0));
    progress_dev_ = static_cast<long long*>(d);
  }
  if (pcg1_ || ca_) place_fields();
}

// Field placement probe.  On MI355X the same sweep runs at one of (at least) three rates depending
// on WHERE its fields were allocated: a property of the allocation, stable for its lifetime and
// across passes (8 sessions alive in one process, timed forward then in reverse).  At 16384^2 fp64,
// 3 plain sweeps of a candidate block take ~5.45, ~4.97 or ~4.55-4.63 ms, and the iteration runs
// at ~2150 / ~1995 / ~1810 us -- profiles/r3/placement/, profiles/r4/placement/.  So the solver may
// allocate candidate blocks and keep the fastest: at most opt.placement of them (GpuOptions), while
// opt.placement_keep_free of the memory that was free stays free and for at most
// opt.placement_budget_s seconds of timing; blocks under 256 MB are not probed (latency-bound
// grids).  Each candidate: 6 real iterations (probe_iterations; init() resets everything afterwards).
// Construction time only; nothing in the iteration changes.  Off by default (the library) and for
// ranks that share a device; skipped with an external (IPC-shared) arena.
// One candidate's rate: the iteration itself, in its real buffer roles -- init, two untimed
// iterations, then 6 timed ones (a whole parity x w-cycle period: plain and w sweeps with r / r2 and
// p0 / p1 in both assignments).  Round 4: the earlier probe (3 plain sweeps with the fields in
// rotating roles) ranked blocks whose iteration rates differ by 7% within 1% of each other
// (profiles/r4/placement/).  No ghost exchange (timing only); the driver's init() resets everything.
void GpuSubdomainSolver::probe_iterations(hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  enqueue_init(s);
  if (ca_ && ca_fused()) {  // fused schedule: pass 1 + reduction untimed, then two fused blocks -- the
    // kernels a solve actually runs (pass 1 / pass 2 rank blocks differently from the fused pass:
    // round 6, a probe of the unfused passes kept blocks on which the fused pass ran ~6% slower)
    enqueue_ca_pass(s, false);
    enqueue_ca_reduce(s, ca_tiles_.s, false, true);
    HIP_CHECK(hipEventRecord(e0, s));
    for (int k = 0; k < 2; ++k) {
      enqueue_ca_fused(s);
      enqueue_ca_reduce(s, ca_tiles_.s, false, true, true);
    }
    HIP_CHECK(hipEventRecord(e1, s));
    return;
  }
  if (ca_) {  // s-step: one untimed block, then two (2 s iterations); strips: this rank's sums only
    const auto block = [&] {
      enqueue_ca_pass(s, false);
      enqueue_ca_reduce(s, ca_tiles_.s, false, true);
      enqueue_ca_pass(s, true);
    };
    block();
    HIP_CHECK(hipEventRecord(e0, s));
    for (int k = 0; k < 2; ++k) block();
    HIP_CHECK(hipEventRecord(e1, s));
    return;
  }
  for (int k = 0; k < 2; ++k) enqueue_phase_a(s);
  HIP_CHECK(hipEventRecord(e0, s));
  for (int k = 0; k < 6; ++k) enqueue_phase_a(s);
  HIP_CHECK(hipEventRecord(e1, s));
}

void GpuSubdomainSolver::place_fields() {
  const int K = opt_.placement;
  const size_t block = 5 * field_stride_;
  if (K <= 1 || !own_arena_ || block < (size_t(256) << 20)) return;  // small grids: latency-bound
  const double t0 = now_s();
  std::vector<char*> cand{fields_};
  size_t free0 = 0, total_b = 0;
  HIP_CHECK(hipMemGetInfo(&free0, &total_b));
  const size_t keep = std::max(size_t(double(free0) * std::clamp(opt_.placement_keep_free, 0.0, 1.0)),
                               size_t(4) << 30);
  while (int(cand.size()) < K) {
    size_t free_b = 0;
    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    if (free_b < block + keep) break;
    char* p = nullptr;
    if (hipMalloc(&p, block) != hipSuccess) {
      (void)hipGetLastError();
      break;
    }
    cand.push_back(p);
  }
  if (cand.size() == 1) {
    placement_s_ = now_s() - t0;
    return;
  }
  // the time budget bounds the timed sweeps; allocation (the driver clears reused VRAM) is reported
  // in placement_seconds but not charged to it
  const double t_probe = now_s();
  auto keep_only = [&](size_t keep) {  // free every other candidate, point the fields at `keep`
    for (size_t c = 0; c < cand.size(); ++c)
      if (c != keep) (void)hipFree(cand[c]);
    fields_ = cand[keep];
    r2_ = field_raw(4);
  };
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  try {
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    placement_ms_.clear();
    for (size_t c = 0; c < cand.size(); ++c) {
      if (c > 0 && now_s() - t_probe > opt_.placement_budget_s) break;  // time budget: the rest stay untimed
      placement_ms_.push_back(0.f);
      fields_ = cand[c];
      r2_ = field_raw(4);
      probe_iterations(s, e0, e1);
      HIP_CHECK(hipEventSynchronize(e1));
      HIP_CHECK(hipEventElapsedTime(&placement_ms_[c], e0, e1));
    }
  } catch (...) {  // keep the first block (the solver's own), release the candidates, then report
    if (s) (void)hipStreamSynchronize(s);
    keep_only(0);
    placement_ms_.clear();
    throw;
  }
  const auto pick = opt_.placement_pick == 1 ? std::max_element(placement_ms_.begin(), placement_ms_.end())
                                             : std::min_element(placement_ms_.begin(), placement_ms_.end());
  keep_only(size_t(pick - placement_ms_.begin()));
  HIP_CHECK(hipEventDestroy(e0));
  HIP_CHECK(hipEventDestroy(e1));
  HIP_CHECK(hipStreamDestroy(s));
  placement_s_ = now_s() - t0;
}

void GpuSubdomainSolver::progress(long long out[3]) const {
  for (int q = 0; q < 3; ++q)
    out[q] = progress_host_ ? __atomic_load_n(progress_host_ + q, __ATOMIC_RELAXED) : -1;
}

ErrorStats GpuSubdomainSolver::error_norms(hipStream_t s) const {
  HIP_CHECK(hipSetDevice(opt_.device));
  const PcgState st = read_state(s);
  // pending w steps, exactly as download_w applies them
  const void* pp[2] = {nullptr, nullptr};
  double a[2] = {0.0, 0.0};
  int npend = 0;
  if (pcg1_ && st.w_pend_n > 0 && st.w_pend > 0) {
    npend = st.w_pend_n;
    for (int q = 0; q < npend; ++q) {
      const long long j = st.w_pend - (npend - 1) + q;
      pp[q] = field_base((j & 1) ? 3 : 2);
      a[q] = st.alpha1[j & 3];
    }
  } else if (!pcg1_ && st.w_pend > 0) {
    npend = 1;
    pp[0] = field_base((st.w_pend & 1) ? 3 : 2);
    a[0] = st.alpha[st.w_pend & 1];
  }
  constexpr int kMaxBlocks = 1024;
  double* d_out = nullptr;
  HIP_CHECK(hipMalloc(&d_out, 3 * kMaxBlocks * sizeof(double)));
  int nb = 0;
  if (elem_ == 8)
    nb = launch_error_norms<double>(geom_, tables_, static_cast<const double*>(field_base(0)),
                                    static_cast<const double*>(pp[0]), a[0], static_cast<const double*>(pp[1]),
                                    a[1], npend, d_out, kMaxBlocks, s);
  else
    nb = launch_error_norms<float>(geom_, tables_, static_cast<const float*>(field_base(0)),
                                   static_cast<const float*>(pp[0]), a[0], static_cast<const float*>(pp[1]),
                                   a[1], npend, d_out, kMaxBlocks, s);
  std::vector<double> h(3 * size_t(nb));
  HIP_CHECK(hipMemcpyAsync(h.data(), d_out, h.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  HIP_CHECK(hipFree(d_out));
  ErrorStats e;
  e.max_w = -HUGE_VAL;
  for (int b = 0; b < nb; ++b) {  // block order: deterministic
    e.sum_e2 += h[3 * size_t(b)];
    e.max_e = std::max(e.max_e, h[3 * size_t(b) + 1]);
    e.max_w = std::max(e.max_w, h[3 * size_t(b) + 2]);
  }
  return e;
}

void GpuSubdomainSolver::release() noexcept {
  (void)hipSetDevice(opt_.device);
  (void)hipDeviceSynchronize();
  if (fields_) (void)hipFree(fields_);
  if (tile_order_) (void)hipFree(tile_order_);
  if (tile_order_w_) (void)hipFree(tile_order_w_);
  if (ca_tbl_) (void)hipFree(ca_tbl_);
  if (ca_tbl_f_) (void)hipFree(ca_tbl_f_);
  ca_tbl_f_ = nullptr;
  if (ca_faces_) (void)hipFree(ca_faces_);
  if (ca_side_) (void)hipStreamDestroy(ca_side_);
  if (ca_ev_fork_) (void)hipEventDestroy(ca_ev_fork_);
  if (ca_ev_join_) (void)hipEventDestroy(ca_ev_join_);
  ca_side_ = nullptr;
  ca_ev_fork_ = ca_ev_join_ = nullptr;
  ca_faces_ = nullptr;
  if (ca_state_) (void)hipFree(ca_state_);
  if (ca_chunk_) (void)hipFree(ca_chunk_);
  ca_tbl_ = nullptr;
  ca_state_ = nullptr;
  ca_chunk_ = nullptr;
  if (tables_buf_) (void)hipFree(tables_buf_);
  if (partials_) (void)hipFree(partials_);
  if (own_arena_ && arena_) (void)hipFree(arena_);
  if (host_state_) (void)hipHostFree(host_state_);
  if (progress_host_) (void)hipHostFree(progress_host_);
  progress_host_ = progress_dev_ = nullptr;
  fields_ = r2_ = nullptr;
  arena_ = nullptr;
  tables_buf_ = partials_ = nullptr;
  tile_order_ = tile_order_w_ = nullptr;
  host_state_ = nullptr;
}

GpuSubdomainSolver::~GpuSubdomainSolver() {
#ifdef PMX_WAVE_TRACE
  if (wtrace_) {  // one line per wave: start end xcc hw_id tile part prologue_end (100 MHz ticks)
    std::vector<unsigned long long> h(size_t(wtrace_n_) * 5);
    if (hipMemcpy(h.data(), wtrace_, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      const char* fn = std::getenv("PMX_WAVE_TRACE_OUT");
      if (FILE* f = std::fopen(fn && fn[0] ? fn : "wave_trace.txt", "w")) {
        for (int b = 0; b < wtrace_n_; ++b) {
          const unsigned long long* o = &h[size_t(b) * 5];
          if (o[1]) std::fprintf(f, "%llu %llu %llu %llu %llu %llu %llu\n", o[0], o[1], o[2] >> 32, o[2] & 0xffffffffull,
                                 o[3] & 0xffffffffffull, o[3] >> 40, o[4]);
        }
        std::fclose(f);
      }
    }
    (void)hipFree(wtrace_);
  }
#endif
  release();
}

size_t GpuSubdomainSolver::estimate_device_bytes(const ProblemSpec& spec, const Subdomain& sd,
                                                 DType dtype, bool single_pass) {
  const size_t elem = dtype == DType::kFp64 ? 8 : 4, align = 256 / elem;
  const size_t pitch = round_up(size_t(sd.ny + 2 + 8), align);
  const size_t field = round_up((align - 1 + size_t(sd.nx + 4) * pitch) * elem, 256);
  const size_t tables = (4 * size_t(spec.M + 2) + 4 * size_t(spec.N + 2)) * 8 + 8 * size_t(spec.M + 2) * 4;
  // partials: at most one per 2 rows x 64 columns tile (the smallest auto tile), 5 doubles each
  const size_t partials = (size_t(sd.nx + 1) / 2 + 1) * (size_t(sd.ny) / 64 + 1) * 40;
  return (single_pass ? 5 : 4) * field + tables + partials + comm_layout(sd, dtype, single_pass).bytes +
         (1u << 20);
}

size_t GpuSubdomainSolver::estimate_device_bytes_algo(const ProblemSpec& spec, const Subdomain& sd, DType dtype,
                                                      int algo) {
  if (algo != 3) return estimate_device_bytes(spec, sd, dtype, algo == 1);
  // s-step: w, two (z, p) sets and the two face fields, rows -gh+1 .. nx+gh (gh = 2s = 6 on strips: the
  // fused pass)
  const size_t elem = dtype == DType::kFp64 ? 8 : 4, align = 256 / elem;
  const int gh = sd.grid.size() > 1 ? 2 * kCaMaxS : 2;
  const size_t pitch = round_up(size_t(sd.ny + 2 + 8 + (sd.grid.Py > 1 ? 2 * gh + 8 : 0)), align);
  const size_t field = round_up((align - 1 + size_t(sd.nx + 2 * gh) * pitch) * elem, 256);
  const size_t face = round_up((31 + size_t(sd.nx + 2 * gh) * pitch) * 8, 256);
  const size_t tables = (4 * size_t(spec.M + 2) + 4 * size_t(spec.N + 2)) * 8 + 8 * size_t(spec.M + 2) * 4;
  // partials: 21 doubles per 8-row tile of 116 columns (the smallest tiling), row-class words
  const size_t partials = (size_t(sd.nx) / 8 + 1) * (size_t(sd.ny) / 116 + 1) * 21 * 8 * 2;
  return 5 * field + 2 * face + tables + partials +
         comm_layout(sd, dtype, true, sd.grid.size() > 1 ? gh : 0).bytes + (1u << 20);
}

size_t GpuSubdomainSolver::device_bytes() const {
  const size_t tables = (4 * size_t(spec_.M + 2) + 4 * size_t(spec_.N + 2)) * sizeof(double) +
                        8 * size_t(spec_.M + 2) * sizeof(int);
  return (r2_ ? 5 : 4) * field_stride_ + tables + (npart_ * 5 + kReduceWsDoubles) * sizeof(double) +
         (own_arena_ ? layout_.bytes : 0) + (ca_faces_ ? 2 * ca_face_bytes_ : 0);
}

void* GpuSubdomainSolver::field_base(int which) const {
  PMX_CHECK(which >= 0 && which < 4, "field index");
  return field_raw(which) + field_off_ * elem_;
}

template <typename T>
HaloBufs<T> GpuSubdomainSolver::halo() const {
  HaloBufs<T> H;
  for (int s = 0; s < kHaloSlots; ++s) {
    H.send[s] = reinterpret_cast<T*>(arena_ + layout_.send_off[s]);
    H.recv[s] = reinterpret_cast<T*>(arena_ + layout_.recv_off[s]);
  }
  return H;
}

void GpuSubdomainSolver::after_launch(hipStream_t s) const {
  if (opt_.check) {
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(s));
  }
}

template <typename T>
void GpuSubdomainSolver::init_impl(hipStream_t s) {
  for (int f = 0; f < 4; ++f) HIP_CHECK(hipMemsetAsync(field_raw(f), 0, field_bytes_, s));
  if (r2_) HIP_CHECK(hipMemsetAsync(r2_, 0, field_bytes_, s));
  HIP_CHECK(hipMemsetAsync(arena_, 0, layout_.bytes, s));
  PcgState& st = host_state_[1];  // template (never rewritten while a copy is in flight)
  std::memset(&st, 0, sizeof(st));
  st.delta = spec_.delta;
  st.bd_tol = spec_.breakdown_tol;
  st.it = pcg1_ || ca_ ? 0 : 1;  // pcg1: sweep 0 (enqueued by the driver) forms (z^0, r^0), (A z^0, z^0)
  st.halo_k = 0;          // pcg1: the first ghost exchange fills sweep 0's inputs
  st.max_iter = spec_.effective_max_iter();
  st.norm = int(spec_.norm);
  st.pair_w = opt_.pair_w ? 1 : 0;
  st.pair_min_beta = opt_.pair_w == 2 ? HUGE_VAL : 1e-3;
  st.w_cycle = w_cycle();
  host_k_ = st.it;
  if (progress_host_) {  // the device has finished with them: init follows a synchronised state
    for (int q = 0; q < 3; ++q) __atomic_store_n(progress_host_ + q, 0LL, __ATOMIC_RELAXED);
  }
  HIP_CHECK(hipMemcpyAsync(state_, &st, sizeof(PcgState), hipMemcpyHostToDevice, s));
  T* w = static_cast<T*>(field_base(0));
  T* r = static_cast<T*>(field_base(1));
  // k_init packs r^0 into the two-sweep send buffers; pcg1 packs its own radius-2 halo
  DevGeom G = geom_;
  if (pcg1_) G.nb = 0;
  launch_init<T>(G, tables_, w, r, halo<T>(), partials_, init_tiles_, s);
  after_launch(s);
  launch_reduce(partials_, init_tiles_.ntiles(), 2, 0.0, g_.h1h2, state_->red_b, state_, 0, reduce_ws_, s);
  after_launch(s);
  if (ca_) {  // set 0: z^0 = D^-1 r^0 (in r's buffer), p^0 = z^0; block counter 0
    std::memset(&ca_init_, 0, sizeof(CaState));
    ca_init_.s = ca_tiles_.s;  // (checked by load_checkpoint)
    HIP_CHECK(hipMemcpyAsync(ca_state_, &ca_init_, sizeof(CaState), hipMemcpyHostToDevice, s));
    ca_blk_ = 0;
    ca_primed_ = false;
    launch_ca_init<T>(ca_geom_, ca_tables_, static_cast<T*>(field_base(1)), static_cast<T*>(field_base(2)), s);
    after_launch(s);
  }
}

template <typename T>
void GpuSubdomainSolver::halo_impl(hipStream_t s, bool unpack) {
  launch_pcg1_halo<T>(geom_, static_cast<T*>(field_base(1)), reinterpret_cast<T*>(r2_ + field_off_ * elem_),
                      static_cast<T*>(field_base(2)), static_cast<T*>(field_base(3)), halo<T>(), halo_target_,
                      unpack, s, progress_dev_);
  after_launch(s);
}

// 2-D blocks (no direct rows): pack / unpack the gh edge lines and corners of the set ca_halo_msgs would
// name (the set the next block reads, CaState::blk & 1 mirrored by ca_blk_) through the arena slots
void GpuSubdomainSolver::ca_halo_impl(hipStream_t s, bool unpack) {
  const int set = int(ca_blk_ & 1);
  char* fz = set ? r2_ + field_off_ * elem_ : static_cast<char*>(field_base(1));
  char* fp = static_cast<char*>(field_base(set ? 3 : 2));
  if (elem_ == 8)
    launch_ca_halo<double>(geom_, reinterpret_cast<double*>(fz), reinterpret_cast<double*>(fp), halo<double>(), gh_,
                           unpack, s, progress_dev_);
  else
    launch_ca_halo<float>(geom_, reinterpret_cast<float*>(fz), reinterpret_cast<float*>(fp), halo<float>(), gh_, unpack,
                          s, progress_dev_);
  after_launch(s);
}

void GpuSubdomainSolver::set_direct_rows(bool on) {
  PMX_CHECK(!on || can_direct_rows(), "direct-row ghost exchange needs pcg1 on a row strip (x neighbours only)");
  direct_rows_ = on;
}

HaloMsgs GpuSubdomainSolver::halo_msgs() const {
  HaloMsgs out;
  if (!direct_rows_) {  // the packed slot buffers of the comm arena
    for (int slot = 0; slot < kHaloSlots; ++slot)
      if (layout_.active(slot))
        out.m[out.n++] = HaloMsg{slot, 0, layout_.peer[slot], layout_.edge_len[slot], send_dev(slot), recv_dev(slot)};
    return out;
  }
  if (ca_) return ca_halo_msgs(int(ca_blk_ & 1));
  // sweep t reads r^{t-1} from (t & 1 ? r2 : r) and p^{t-1} from (t & 1 ? p0 : p1) (k_pcg1)
  const long long t = halo_target_;
  char* fr = (t & 1) ? r2_ + field_off_ * elem_ : static_cast<char*>(field_base(1));
  char* fp = static_cast<char*>(field_base((t & 1) ? 2 : 3));
  const int64_t P = geom_.pitch;
  // rows q, q+1 as one span: row q whole (its padding ends with column -1 of row q+1) and row q+1's
  // columns 0 .. ny+1; on a row strip the ghost columns are Dirichlet zeros on both sides
  const int count = int(P + sd_.ny + 2);
  for (int slot = 0; slot < 2; ++slot) {
    if (layout_.peer[slot] < 0) continue;
    const int64_t srow = slot == 0 ? 1 : sd_.nx - 1, rrow = slot == 0 ? -1 : sd_.nx + 1;
    for (int f = 0; f < 2; ++f) {
      char* base = f == 0 ? fr : fp;
      out.m[out.n++] = HaloMsg{slot, f, layout_.peer[slot], count, base + srow * P * int64_t(elem_),
                               base + rrow * P * int64_t(elem_)};
    }
  }
  return out;
}

void GpuSubdomainSolver::enqueue_halo_pack(hipStream_t s) {
  if (ca_ && geom_.nb != 0 && !direct_rows_) {
    ca_halo_impl(s, false);
    return;
  }
  if (!pcg1_ || geom_.nb == 0 || direct_rows_) return;
  if (opt_.dtype == DType::kFp64) halo_impl<double>(s, false); else halo_impl<float>(s, false);
}

void GpuSubdomainSolver::enqueue_halo_unpack(hipStream_t s) {
  if (ca_ && geom_.nb != 0 && !direct_rows_) {
    ca_halo_impl(s, true);
    return;
  }
  if (!pcg1_ || geom_.nb == 0 || direct_rows_) return;
  if (opt_.dtype == DType::kFp64) halo_impl<double>(s, true); else halo_impl<float>(s, true);
}

template <typename T>
void GpuSubdomainSolver::phase_a_impl(hipStream_t s) {
  enqueue_kernel_a(s);
  enqueue_reduce_a(s);
}

template <typename T>
void GpuSubdomainSolver::phase_a_kernel_only(hipStream_t s, int part) {
  if constexpr (sizeof(T) == 8) {
    if (block1_) {
      PMX_CHECK(part == 0, "block tiles run whole sweeps (undecomposed grids)");
      const double h = g_.h1h2, wdiff = spec_.norm == Norm::kWeighted ? g_.h1h2 : 1.0;
      const double wts[5] = {h, h, h, h, wdiff};
      // the reduce_n ticket (never in flight together with this sweep: same stream)
      unsigned* ticket = block_fused_ ? reinterpret_cast<unsigned*>(reduce_ws_ + kReduceNOffset + 8 * kReduceMaxBlocks)
                                      : nullptr;
      launch_pcg1_block<T>(geom_, tables_, static_cast<T*>(field_base(0)), static_cast<T*>(field_base(1)),
                           reinterpret_cast<T*>(r2_ + field_off_ * elem_), static_cast<T*>(field_base(2)),
                           static_cast<T*>(field_base(3)), partials_, state_, tiles1_for(w_sweep_next()), s,
                           w_sweep_next(), wts, ticket, progress_dev_);
      return;
    }
  }
  if (pcg1_)
    launch_pcg1<T>(geom_, tables_, static_cast<T*>(field_base(0)), static_cast<T*>(field_base(1)),
                   reinterpret_cast<T*>(r2_ + field_off_ * elem_), static_cast<T*>(field_base(2)), static_cast<T*>(field_base(3)), partials_, state_,
                   tiles1_for(w_sweep_next()), s, part, w_sweep_next());
  else
    launch_pcg_a_wave<T>(geom_, tables_, static_cast<const T*>(field_base(1)),
                         static_cast<T*>(field_base(2)), static_cast<T*>(field_base(3)), halo<T>(),
                         partials_, state_, tiles_, opt_.exact, s);
}

template <typename T>
void GpuSubdomainSolver::phase_b_impl(hipStream_t s, bool pack) {
  enqueue_kernel_b(s, pack);
  enqueue_reduce_b(s);
}

template <typename T>
void GpuSubdomainSolver::phase_b_kernel_only(hipStream_t s, bool pack) {
  if (pcg1_) return;  // the single sweep ran in phase a
  // pcg_b reads G.nb only to pack the send buffers: clearing it skips the packing
  DevGeom G = geom_;
  if (!pack) G.nb = 0;
  launch_pcg_b_wave<T>(G, tables_, static_cast<T*>(field_base(0)),
                       static_cast<T*>(field_base(1)), static_cast<const T*>(field_base(2)),
                       static_cast<const T*>(field_base(3)), halo<T>(), partials_, state_, tiles_b_,
                       opt_.exact, s);
}

void GpuSubdomainSolver::enqueue_init(hipStream_t s) {
  HIP_CHECK(hipSetDevice(opt_.device));
  if (opt_.dtype == DType::kFp64) init_impl<double>(s); else init_impl<float>(s);
}
void GpuSubdomainSolver::enqueue_phase_a(hipStream_t s) {
  if (opt_.dtype == DType::kFp64) phase_a_impl<double>(s); else phase_a_impl<float>(s);
}
void GpuSubdomainSolver::enqueue_phase_b(hipStream_t s, bool pack) {
  if (opt_.dtype == DType::kFp64) phase_b_impl<double>(s, pack); else phase_b_impl<float>(s, pack);
}
void GpuSubdomainSolver::enqueue_kernel_a(hipStream_t s) {
  if (opt_.dtype == DType::kFp64) phase_a_kernel_only<double>(s); else phase_a_kernel_only<float>(s);
  after_launch(s);
}
void GpuSubdomainSolver::enqueue_kernel_a_part(hipStream_t s, int part) {
  PMX_CHECK(pcg1_, "interior/frame sweeps are a pcg1 feature");
  if (opt_.dtype == DType::kFp64) phase_a_kernel_only<double>(s, part); else phase_a_kernel_only<float>(s, part);
  after_launch(s);
}
void GpuSubdomainSolver::enqueue_reduce_a(hipStream_t s) {
  if (block1_ && block_fused_) {  // the sweep finished its own reduction
    ++host_k_;
    return;
  }
  if (pcg1_) {
    const double h = g_.h1h2, wdiff = spec_.norm == Norm::kWeighted ? g_.h1h2 : 1.0;
    const double wts[5] = {h, h, h, h, wdiff};
    // the sweep just enqueued (host_k not bumped yet) wrote one partial per tile of its tiling
    launch_reduce_n(partials_, tiles1_for(w_sweep_next()).ntiles(), 5, wts, state_->red_c, state_,
                    kSkipIfDone | kBumpIter,
                    reduce_ws_, s, progress_dev_);
    ++host_k_;  // mirrors the S->it bump (see host_k())
    after_launch(s);
    return;
  }
  launch_reduce(partials_, tiles_.ntiles(), 1, g_.h1h2, 0.0, state_->red_a, state_, kSkipIfDone,
                reduce_ws_, s);
  after_launch(s);
}
void GpuSubdomainSolver::enqueue_kernel_b(hipStream_t s, bool pack) {
  if (opt_.dtype == DType::kFp64) phase_b_kernel_only<double>(s, pack);
  else phase_b_kernel_only<float>(s, pack);
  after_launch(s);
}
void GpuSubdomainSolver::enqueue_reduce_b(hipStream_t s) {
  if (pcg1_) return;
  const double wdiff = spec_.norm == Norm::kWeighted ? g_.h1h2 : 1.0;
  launch_reduce(partials_, tiles_b_.ntiles(), 2, wdiff, g_.h1h2, state_->red_b, state_,
                kSkipIfDone | kBumpIter, reduce_ws_, s);
  after_launch(s);
}

template <typename T>
static void pack_impl(const GpuSubdomainSolver& g, HaloBufs<T> H, hipStream_t s) {
  launch_edge_r<T>(g.geom(), g.tables(), static_cast<const T*>(g.field_base(1)),
                   static_cast<const T*>(g.field_base(2)), static_cast<const T*>(g.field_base(3)), H,
                   g.state_dev(), g.options().exact, s);
}

void GpuSubdomainSolver::enqueue_poison_recv(hipStream_t s) {
  if (direct_rows_) {  // the ghost rows the next exchange writes
    const HaloMsgs ms = halo_msgs();
    for (int q = 0; q < ms.n; ++q)
      HIP_CHECK(hipMemsetAsync(ms.m[q].recv, 0xFF, size_t(ms.m[q].count) * elem_, s));
    return;
  }
  const size_t off = layout_.recv_off[0];
  HIP_CHECK(hipMemsetAsync(arena_ + off, 0xFF, layout_.bytes - off, s));  // all-ones = NaN
}

namespace {
struct CkptHeader {
  char magic[8];
  int32_t version, M, N, gi0, gj0, rank, elem, norm;
  int64_t nx, ny, pitch, field_bytes, arena_bytes, max_iter;
  double delta;
};
constexpr char kCkptMagic[8] = {'P', 'M', 'X', 'C', 'K', 'P', 'T', '1'};
}  // namespace

// The version names the iteration algorithm and layout: v3 pcg2 (4 fields with 2 ghost rows), v5 pcg1
// (+ its w-cycle state, r2 appended), v6 the s-step PCG (r2 = the second z buffer appended, then
// CaState).  A checkpoint is written between batches, where every algorithm's state is exact: for the
// s-step no block's stop test is pending and w holds every applied block.
int GpuSubdomainSolver::ckpt_version() const { return ca_ ? 7 : pcg1_ ? 5 : 3; }

void GpuSubdomainSolver::save_checkpoint(std::ostream& os, hipStream_t s) const {
  HIP_CHECK(hipSetDevice(opt_.device));
  HIP_CHECK(hipStreamSynchronize(s));
  CkptHeader h{};
  std::memcpy(h.magic, kCkptMagic, 8);
  h.version = ckpt_version();
  h.M = spec_.M; h.N = spec_.N; h.gi0 = sd_.gi0(); h.gj0 = sd_.gj0();
  h.rank = sd_.rank; h.elem = int32_t(elem_); h.norm = int32_t(spec_.norm);
  h.nx = sd_.nx; h.ny = sd_.ny; h.pitch = geom_.pitch; h.field_bytes = int64_t(field_bytes_);
  h.arena_bytes = int64_t(layout_.bytes); h.max_iter = spec_.effective_max_iter(); h.delta = spec_.delta;
  os.write(reinterpret_cast<const char*>(&h), sizeof(h));
  std::vector<char> buf(std::max(4 * field_bytes_, layout_.bytes));
  for (int f = 0; f < 4; ++f)
    HIP_CHECK(hipMemcpy(buf.data() + size_t(f) * field_bytes_, field_raw(f), field_bytes_, hipMemcpyDeviceToHost));
  os.write(buf.data(), std::streamsize(4 * field_bytes_));
  HIP_CHECK(hipMemcpy(buf.data(), arena_, layout_.bytes, hipMemcpyDeviceToHost));
  os.write(buf.data(), std::streamsize(layout_.bytes));
  if (pcg1_ || ca_) {
    HIP_CHECK(hipMemcpy(buf.data(), r2_, field_bytes_, hipMemcpyDeviceToHost));
    os.write(buf.data(), std::streamsize(field_bytes_));
  }
  if (ca_) {
    CaState c{};
    HIP_CHECK(hipMemcpy(&c, ca_state_, sizeof(CaState), hipMemcpyDeviceToHost));
    PMX_CHECK(c.pend_n == 0 && c.nupd <= 0, "s-step checkpoint inside a batch (a block's stop test is pending)");
    os.write(reinterpret_cast<const char*>(&c), sizeof(c));
    // a carried fused schedule: the next block's Gram partials (so a resume continues bitwise)
    const int32_t primed = ca_primed_ ? 1 : 0;
    os.write(reinterpret_cast<const char*>(&primed), sizeof(primed));
    if (primed) {
      std::vector<double> part(ca_primed_doubles());
      HIP_CHECK(hipMemcpy(part.data(), partials_, part.size() * sizeof(double), hipMemcpyDeviceToHost));
      os.write(reinterpret_cast<const char*>(part.data()), std::streamsize(part.size() * sizeof(double)));
    }
  }
  PMX_CHECK(os.good(), "checkpoint write failed");
}

void GpuSubdomainSolver::load_checkpoint(std::istream& is, hipStream_t s) {
  HIP_CHECK(hipSetDevice(opt_.device));
  CkptHeader h{};
  is.read(reinterpret_cast<char*>(&h), sizeof(h));
  PMX_CHECK(is.good() && std::memcmp(h.magic, kCkptMagic, 8) == 0 && h.version == ckpt_version(),
            "not a pmx checkpoint of this iteration algorithm and layout (v3 pcg2, v5 pcg1, v7 s-step; file v"
                << h.version << ", solver v" << ckpt_version() << ")");
  PMX_CHECK(h.M == spec_.M && h.N == spec_.N && h.gi0 == sd_.gi0() && h.gj0 == sd_.gj0() &&
                h.nx == sd_.nx && h.ny == sd_.ny && h.rank == sd_.rank,
            "checkpoint is for a different grid/decomposition (M=" << h.M << " N=" << h.N << " rank "
                                                                  << h.rank << ")");
  PMX_CHECK(h.elem == int32_t(elem_) && h.pitch == geom_.pitch &&
                h.field_bytes == int64_t(field_bytes_) && h.arena_bytes == int64_t(layout_.bytes),
            "checkpoint precision/layout differs from this solver");
  PMX_CHECK(h.norm == int32_t(spec_.norm) && h.delta == spec_.delta &&
                h.max_iter == spec_.effective_max_iter(),
            "checkpoint was written with a different stop rule (norm/delta/max_iter)");
  std::vector<char> buf(std::max(4 * field_bytes_, layout_.bytes));
  is.read(buf.data(), std::streamsize(4 * field_bytes_));
  PMX_CHECK(is.good(), "truncated checkpoint (fields)");
  HIP_CHECK(hipStreamSynchronize(s));
  for (int f = 0; f < 4; ++f)
    HIP_CHECK(hipMemcpy(field_raw(f), buf.data() + size_t(f) * field_bytes_, field_bytes_, hipMemcpyHostToDevice));
  is.read(buf.data(), std::streamsize(layout_.bytes));
  PMX_CHECK(is.good(), "truncated checkpoint (scalars/halos)");
  HIP_CHECK(hipMemcpy(arena_, buf.data(), layout_.bytes, hipMemcpyHostToDevice));
  PcgState ck{};
  std::memcpy(&ck, buf.data() + layout_.state_off, sizeof(PcgState));
  host_k_ = ck.it;
  if (pcg1_ || ca_) {
    is.read(buf.data(), std::streamsize(field_bytes_));
    PMX_CHECK(is.good(), "truncated checkpoint (r2 / second z buffer)");
    HIP_CHECK(hipMemcpy(r2_, buf.data(), field_bytes_, hipMemcpyHostToDevice));
  }
  if (ca_) {
    CaState c{};
    is.read(reinterpret_cast<char*>(&c), sizeof(c));
    PMX_CHECK(is.good(), "truncated checkpoint (s-step state)");
    PMX_CHECK(c.s == ca_tiles_.s, "checkpoint was written with s = " << c.s << ", this solver runs s = " << ca_tiles_.s);
    c.ticket = 0u;
    HIP_CHECK(hipMemcpy(ca_state_, &c, sizeof(CaState), hipMemcpyHostToDevice));
    ca_blk_ = c.blk;  // the (z, p) set the next block reads
    int32_t primed = 0;
    is.read(reinterpret_cast<char*>(&primed), sizeof(primed));
    PMX_CHECK(is.good() && (primed == 0 || (primed == 1 && ca_fused())), "checkpoint: bad s-step schedule flag");
    if (primed) {
      std::vector<double> part(ca_primed_doubles());
      is.read(reinterpret_cast<char*>(part.data()), std::streamsize(part.size() * sizeof(double)));
      PMX_CHECK(is.good(), "truncated checkpoint (carried Gram partials)");
      HIP_CHECK(hipMemcpy(partials_, part.data(), part.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    ca_primed_ = primed != 0;
  }
}

void GpuSubdomainSolver::enqueue_pack(hipStream_t s) {
  if (geom_.nb == 0 || pcg1_) return;
  if (opt_.dtype == DType::kFp64) pack_impl<double>(*this, halo<double>(), s);
  else pack_impl<float>(*this, halo<float>(), s);
  after_launch(s);
}

double GpuSubdomainSolver::bench_kernel(int which, int abl, int reps, hipStream_t s) {
  PMX_CHECK(!ca_, "not available for the s-step solver");
  HIP_CHECK(hipSetDevice(opt_.device));
  PcgState& st = host_state_[1];
  std::memset(&st, 0, sizeof(st));
  st.delta = 0.0;
  // a mid-solve iteration: beta path, p^{k-1} read.  which = 2: pcg_b on an odd iteration (w
  // step deferred, see k_pcg_b_rows); which = 1 is the even (paired w update) one
  st.it = which == 2 ? 3 : 2;
  st.max_iter = int64_t(1) << 40;
  st.norm = int(spec_.norm);
  st.red_a[0] = 1.0;
  st.red_b[0] = 1.0;
  st.red_b[1] = 1e-3;
  st.zr[0] = st.zr[1] = 1e-3;
  st.alpha[0] = st.alpha[1] = 1.0;
  for (int q = 0; q < 4; ++q) st.alpha1[q] = st.beta1[q] = 1.0;
  st.w_cycle = w_cycle();
  host_k_ = st.it;
  st.red_c[0] = 1e-3;
  st.red_c[1] = st.red_c[3] = st.red_c[4] = 1.0;
  st.pair_w = opt_.pair_w ? 1 : 0;
  st.pair_min_beta = opt_.pair_w == 2 ? HUGE_VAL : 1e-3;
  const TileCfg saved = tiles_, saved_b = tiles_b_;
  tiles_.abl = abl;
  tiles_b_.abl = abl;
  auto launch = [&]() {
    HIP_CHECK(hipMemcpyAsync(state_, &st, sizeof(PcgState), hipMemcpyHostToDevice, s));
    if (which == 0 || pcg1_) {
      if (opt_.dtype == DType::kFp64) phase_a_kernel_only<double>(s); else phase_a_kernel_only<float>(s);
    } else {
      if (opt_.dtype == DType::kFp64) phase_b_kernel_only<double>(s); else phase_b_kernel_only<float>(s);
    }
  };
  launch();
  launch();
  HIP_CHECK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  float total = 0.f;
  for (int k = 0; k < reps; ++k) {
    HIP_CHECK(hipMemcpyAsync(state_, &st, sizeof(PcgState), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipEventRecord(e0, s));
    if (which == 0 || pcg1_) {
      if (opt_.dtype == DType::kFp64) phase_a_kernel_only<double>(s); else phase_a_kernel_only<float>(s);
    } else {
      if (opt_.dtype == DType::kFp64) phase_b_kernel_only<double>(s); else phase_b_kernel_only<float>(s);
    }
    HIP_CHECK(hipEventRecord(e1, s));
    HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    total += ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  tiles_ = saved;
  tiles_b_ = saved_b;
  return double(total) / reps;
}

PcgState GpuSubdomainSolver::read_state(hipStream_t s) const {
  HIP_CHECK(hipSetDevice(opt_.device));
  HIP_CHECK(hipMemcpyAsync(&host_state_[0], state_, sizeof(PcgState), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return host_state_[0];
}

std::vector<double> GpuSubdomainSolver::read_partials(hipStream_t s) const {
  HIP_CHECK(hipSetDevice(opt_.device));
  std::vector<double> h(npart_ * 5);
  HIP_CHECK(hipMemcpyAsync(h.data(), partials_, h.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return h;
}

std::vector<double> GpuSubdomainSolver::download_field(int which, hipStream_t s) const {
  HIP_CHECK(hipSetDevice(opt_.device));
  const size_t n = size_t(sd_.nx + 2) * geom_.pitch;
  std::vector<char> raw(n * elem_);
  HIP_CHECK(hipMemcpyAsync(raw.data(), field_base(which), raw.size(), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  std::vector<double> out(size_t(sd_.nx + 2) * (sd_.ny + 2));
  for (int li = 0; li <= sd_.nx + 1; ++li)
    for (int lj = 0; lj <= sd_.ny + 1; ++lj) {
      const size_t src = size_t(li) * geom_.pitch + lj;
      out[size_t(li) * (sd_.ny + 2) + lj] =
          elem_ == 8 ? reinterpret_cast<const double*>(raw.data())[src]
                     : double(reinterpret_cast<const float*>(raw.data())[src]);
    }
  return out;
}

std::vector<double> GpuSubdomainSolver::download_w(hipStream_t s) const {
  const std::vector<double> f = download_field(0, s);
  // Paired w updates (k_pcg_b_rows): an odd iteration leaves w^{k+1} = w^k + alpha_k p^k pending
  // in device memory; apply it here, rounded to the storage type like a device update.
  // pcg1 (k_pcg1) leaves w_pend_n (1 or 2) steps pending, p^j in p[j & 1], alpha_j in alpha1[j & 3].
  const PcgState st = read_state(s);
  std::vector<double> pk[2];
  double a[2] = {0.0, 0.0};
  int npend = 0;
  if (pcg1_ && st.w_pend_n > 0 && st.w_pend > 0) {
    npend = st.w_pend_n;
    for (int q = 0; q < npend; ++q) {  // q = 0: the oldest pending step
      const long long j = st.w_pend - (npend - 1) + q;
      pk[q] = download_field((j & 1) ? 3 : 2, s);
      a[q] = st.alpha1[j & 3];
    }
  } else if (!pcg1_ && st.w_pend > 0) {
    npend = 1;
    pk[0] = download_field((st.w_pend & 1) ? 3 : 2, s);
    a[0] = st.alpha[st.w_pend & 1];
  }
  std::vector<double> out(size_t(sd_.nx) * sd_.ny);
  for (int li = 1; li <= sd_.nx; ++li)
    for (int lj = 1; lj <= sd_.ny; ++lj) {
      const size_t src = size_t(li) * (sd_.ny + 2) + lj;
      double v = f[src];
      for (int q = 0; q < npend; ++q) v = std::fma(a[q], pk[q][src], v);
      if (npend && elem_ == 4) v = double(float(v));
      out[size_t(li - 1) * sd_.ny + (lj - 1)] = v;
    }
  return out;
}

}  // namespace pmx
