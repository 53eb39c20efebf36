// GPU PCG: per-subdomain device state + the host orchestrator
// (components C9, X1-X4, P3/P4/P6 of SURVEY §2; replaces gradient_solver_mpi,
// stage4-mpi+cuda/poisson_mpi_cuda_f.cu:688-983).
//
// * GpuSubdomainSolver owns one subdomain's fields on one device: w, r and a ping-pong pair
//   p0/p1 (4 arrays, 32 B/pt in fp64), the 1D face tables, the block-partials scratch and a
//   "comm arena" holding the PcgState scalars (the all-reduce buffers) and the packed
//   send/recv halo buffers.  The arena may be supplied externally (e.g. a torch tensor) so a
//   Python-side communicator can operate on it.
// * PcgDriver steps a set of local subdomains through the PCG iteration with a Comm backend,
//   optionally replaying hipGraph-captured batches of iterations.  The host never waits per
//   iteration: the stop test runs on the device and later launches become no-ops.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <iosfwd>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "pmx/decomp.hpp"
#include "pmx/device_types.hpp"
#include "pmx/geometry.hpp"
#include "pmx/kernels.hpp"
#include "pmx/spec.hpp"

namespace pmx {

enum class DType : int { kFp64 = 0, kFp32 = 1 };

// Kernel-side view of a subdomain whose fields use row pitch `pitch` (elements).
DevGeom make_dev_geom(const ProblemSpec& spec, const Subdomain& sd, int64_t pitch);
// Upload the 1D face tables (pmx/geometry.hpp) to the current device; *owner receives the
// allocation (caller frees).
DevTables upload_tables(const ProblemSpec& spec, double** owner);

struct GpuOptions {
  int device = 0;
  int kernel = 1;         // 0: LDS-ring workgroup tiles, 1: wave tiles with DPP lane shifts
  int block = 256;        // kernel 0: tile width (threads per workgroup)
  // Tile shapes.  pcg_a and pcg_b are separate launches, so each gets its own shape; the *_b
  // fields default to "same as pcg_a" when the pcg_a field is set explicitly.
  int vec = 0;            // kernel 1, pcg_a: columns per lane (0 = auto: 4 = 32-B fp64 accesses)
  int waves = 4;          // kernel 1: wave tiles per workgroup
  int tile_rows = 0;      // tile height (marching length), 0 = auto-size for occupancy
  int vec_b = 0;          // pcg_b columns per lane (0 = vec if set, else auto: 2 fp64 / 4 fp32)
  int waves_b = 0;        // pcg_b wave tiles per workgroup (0 = waves)
  int tile_rows_b = -1;   // pcg_b tile height (-1 = tile_rows, or 2 for the row kernel)
  int b_ring = 0;         // kernel 1: 0 = ring-free row kernel for pcg_b (default), 1 = ring kernel
  DType dtype = DType::kFp64;
  bool exact = false;     // reference arithmetic order inside the fused kernels
  int graph_batch = 32;   // iterations per captured hipGraph (0 = eager launches)
  bool check = false;     // PMX_CHECK mode: synchronise + error-check after every launch
  bool overlap = true;    // halo exchange on a comm stream, overlapped with pcg_b
  // Debug: fill the ghost receive buffers with NaN before every exchange, so a
  // ghost value that the exchange failed to deliver poisons the reductions and raises the
  // device NaN flag.  Also enabled by the environment variable PMX_POISON_HALOS=1.
  bool poison_halos = false;
  // Paired w updates in the pcg_b row kernel (pcg_kernels_dpp.hip): 1 = on (default), 0 = w
  // updated every iteration, 2 = paired but always re-reading p^{k-1} (no recovery; test and
  // ablation).  The environment variable PMX_PAIR_W=0|1|2 overrides it.
  int pair_w = 1;
  // Iteration algorithm: 2 = pcg2 (k_pcg_a + k_pcg_b, two reductions, radius-1 halo), 1 = pcg1
  // (single-pass k_pcg1, one 5-value reduction, radius-2 halo with corners), -1 = auto (pcg1
  // where it applies: wave kernels, not exact, any storage type, every subdomain >= 2 x 2 and the 5th
  // field fits into the device).  The choice depends only on global data (problem, process grid,
  // options, device size), so every rank of a distributed run makes the same one.
  // PMX_ALGO=-1|1|2 overrides.  pcg1 matches the reference iteration counts and pcg2's solution
  // (tests/test_gpu_pcg1.py) and moves 40 instead of 56 B/pt per iteration.
  // 3 = s-step PCG (ca_kernels.hip: s iterations per two passes and one reduction, 21.3 B/pt per
  // iteration at s = 3; undecomposed fp64 grids), never chosen by auto.
  int algo = -1;
  // s-step PCG: block size (2 or 3) and tile height (0 = auto).  PMX_CA_S / PMX_CA_ROWS.
  int ca_s = 3, ca_rows = 0, ca_rows2 = 0;  // (ca_rows2: pass 2's tile rows, PMX_CA_ROWS_UPD)
  // s-step pass shapes: pass 1 rows by LDS-DMA (1) or registers (0); waves per SIMD each pass's
  // registers must allow (2 or 3).  PMX_CA_DMA / PMX_CA_WAVES_GRAM / PMX_CA_WAVES_UPD.  Same-process
  // A/B at 16384^2 (profiles/r5/ca/): pass 1 1712 us with registers vs 1815 with LDS-DMA, 2407 at 3
  // waves (spills); pass 2 3025 at 2 waves vs 3105 at 3 (56 B of spills) -- within noise
  // ca_dma -1: LDS-DMA rows with the split kernels (below), registers without
  int ca_dma = -1, ca_waves_gram = 2, ca_waves_upd = 3;
  // s-step: the interior tiles of a pass by a kernel without the Dirichlet / partial-tile paths, whose
  // registers fit 3 waves per SIMD (pass 1 with LDS-DMA rows), the frame by the general kernel on a
  // side stream (1), or every tile by the general kernel (0); -1 = split on row strips only.
  // PMX_CA_SPLIT / PMX_CA_SPLIT_UPD (pass 2; -1: as pass 1).  16384^2, every session on the fastest
  // of 20 probed blocks, 5 same-process rounds: 1169 us/iteration with pass 1 split and pass 2 one
  // kernel, 1178 both split, 1222 neither (profiles/r5/ca/split/placed_ab16384.log; without the probe
  // the placement lottery hid the difference).  On row strips pass 1's frame tiles also wait for the
  // ghost exchange while its interior runs.
  int ca_split = 1;
  int ca_split_upd = 0;
  // ... the frame kernel on a side stream, overlapping the interior (1), or after it (0).  PMX_CA_FRAME_STREAM.
  int ca_frame_stream = 1;
  // s-step: pass 2 of block b and pass 1 of block b+1 as ONE fused pass (k_ca_fused, 48 instead of 64
  // B/pt per block) between the first pass 1 and the last pass 2 of every batch: 1 on, 0 off, -1 auto
  // (undecomposed grids).  ca_rows_f: its tile rows (0 = auto).
  int ca_fuse = -1, ca_rows_f = 0;
  // s-step kernels see the subdomain's ghost rows as a Dirichlet boundary (nb = 0) while the driver
  // keeps the decomposed schedule: the loopback rehearsal, whose zero ghosts would otherwise break
  // the basis recurrence (its redundant ghost-row levels need the neighbour's real rows).  Set by the
  // Session for comm="loopback"; numerically a different (local) problem, timing-equivalent.
  int ca_dirichlet = 0;
  // pcg1 tile shape (rows1 = 0: auto).  VEC=2 x 1 wave/workgroup won the 16384^2 sweeps
  // (bench/gpu_pcg1_sweep.sh; VEC=4 needs 256 VGPRs and is 35% slower).
  int vec1 = 2, waves1 = 1, rows1 = 0;
  // waves per workgroup of the w sweep (0 = as waves1, but 4 where waves1 is 8: the w sweep's
  // registers allow 3 waves per SIMD, i.e. one 8-wave workgroup per CU).  PMX_PCG1_WAVES_W.
  int waves1w = 0;
  // the w-moving sweep (one in w_cycle, a kernel of its own at 3 waves/SIMD) may use its own tile
  // height and prefetch depth: 0 = as the plain sweep (PMX_PCG1_ROWS_W, PMX_PCG1_PF_W)
  int rows1w = 0, pf1w = 0;
  // pcg1 prefetch depth: rows loaded ahead of the row being computed (1..4).  The sweep is
  // latency-bound at 2 waves/SIMD; deeper prefetch spends VGPRs that occupancy does not use.
  int pf1 = 0;  // 0 = auto
  // pcg1 with fp32 storage: 1 = the sweep's stencil arithmetic in fp32 too (fp64 partial sums,
  // reductions and PCG scalars), 0 = fp64 registers (the default "fp32 storage" path).  fp64 storage
  // ignores it.  PMX_ARITH32=0|1 overrides.
  int arith32 = 0;
  // pcg1 dispatch order: 1 = tiles cut by the ellipse first within each XCD's share, 0 = natural
  int order1 = 1;
  // pcg1 w schedule: w is read and written on one sweep in wcycle1 (3 = triples, 2 = pairs).
  // Triples recover p^{k-2} from p^{k-1} and r^{k-1} (one extra stencil), or re-read it when
  // |beta_{k-1}| < 1e-3 or pair_w == 2.  PMX_PCG1_WCYCLE=2|3 overrides.
  int wcycle1 = 3;
  // Host-mapped progress counters written by the device (sweeps reduced, ghost exchanges packed /
  // unpacked), readable without any HIP call -- how a hang watchdog tells which step a stuck rank
  // is in.  One 8-B system-scope store per kernel; on for multi-rank RCCL sessions.  PMX_PROGRESS
  // overrides.
  int progress = 0;
  // Field placement probe (GpuSubdomainSolver::place_fields): up to `placement` candidate field
  // blocks are allocated and timed and the fastest is kept; 0 or 1 = off (the library default: a
  // probe briefly takes device memory a co-resident process might need).  Bounded by
  // placement_budget_s of probing and by keeping placement_keep_free of the free memory free.
  // bench.py turns it on unless ranks share the device.  PMX_PLACEMENT=K overrides.
  int placement = 0;
  // Block tiles for the pcg1 sweep (pcg1_block.hip): -1 = auto (undecomposed fp64 grids with fewer
  // than 10,000 four-row march tiles, ~1600x2400), 0 = off, 1 = on for any undecomposed fp64 grid.
  // PMX_PCG1_BLOCK overrides.
  int block1 = -1;
  // block-tile shape and reduction: rows per tile (0 = auto: 8 below 1,000 four-row tiles, else 12),
  // waves per workgroup (8 or 16), the reduction folded into the sweep (-1 = auto: below 1,500
  // tiles).  PMX_PCG1_BLOCK_ROWS / _WAVES / _FUSED.
  int block_rows1 = 0, block_waves1 = 8, block_fused1 = -1;
  // pcg1 march sweeps: resident waves per CU (0 = as many as the registers allow: 16 for the plain
  // sweep, 12 for the w sweep).  A cap is enforced with padding LDS per workgroup.  Fewer streams
  // in flight keep more DRAM rows open per access (bench/probe/dma_march.hip).
  // PMX_PCG1_WPCU / PMX_PCG1_WPCU_W override.
  int wpcu1 = 0, wpcu1w = 0;
  // pcg1 march, interior (FAST) tiles in fp64: rows prefetched dma1 ahead by LDS-DMA into a per-wave
  // LDS ring with exact vmcnt counting (2 or 3), 0 = register prefetch.  dma1w: the w sweep (-1 = as
  // dma1).  PMX_PCG1_DMA / PMX_PCG1_DMA_W override.
  int dma1 = 0, dma1w = -1;
  // pcg1 split sweep on decomposed grids (interior tiles overlap the previous ghost exchange, the frame
  // waits for it): -1 = the transport's default (Comm::prefers_split: RCCL on), 0 off, 1 on
  int split_sweep = -1;
  double placement_budget_s = 0.5;
  double placement_keep_free = 0.5;
  // which probed block to keep: 0 the fastest (default), 1 the slowest -- for slow-class A/Bs and
  // counter tables on one box (PMX_PLACEMENT_PICK=slowest)
  int placement_pick = 0;
  bool resolved = false;  // environment overrides already applied (resolve_options)
};

// "fp64", "fp32" (fp32 storage + fp32 stencil arithmetic) or "mixed" (fp32 storage, fp64 arithmetic)
inline const char* dtype_name(const GpuOptions& o) {
  return o.dtype == DType::kFp64 ? "fp64" : (o.arith32 ? "fp32" : "mixed");
}

// Validates `opt` and marks it resolved.  Study mode (PMX_STUDY=1 in the environment) first applies
// the kernel / schedule overrides of bench/ studies (PMX_ALGO, PMX_PAIR_W, PMX_PCG1_*, PMX_CA_*,
// PMX_PLACEMENT*); without it those variables are ignored (one warning on stderr), so a stray
// variable cannot change what a run or a test measures.
GpuOptions resolve_options(const GpuOptions& opt);
// getenv(name) in study mode, nullptr otherwise (driver-level study knobs: PMX_DIRECT_ROWS,
// PMX_PCG1_SPLIT, PMX_FRAME_ON_COMM, PMX_FORK_ONE_QUEUE, PMX_CA_WAVES_F, PMX_CA_SPLIT_F)
const char* study_env(const char* name);
// Single-pass (pcg1) or two-sweep (pcg2) iteration for this problem/process grid/options.  A pure
// function of global data (see GpuOptions::algo); `device_total_bytes` = 0 skips the size test.
// `subdomains_per_device` subdomains share one device (LocalComm: all of them).
bool choose_single_pass(const ProblemSpec& spec, const ProcGrid& grid, const GpuOptions& resolved,
                        double device_total_bytes, int subdomains_per_device);
// The iteration algorithm (GpuOptions::algo) a run uses: an explicit 1 / 2 / 3 as given, auto (-1) the
// s-step PCG (3) where it applies and wins -- the fast arithmetic (any storage), undecomposed or row strips
// of >= 8 rows on a transport that moves ghost rows between fields (`direct_rows`), at least
// kCaAutoPoints grid points (below, pcg1's block tiles are faster: profiles/r5/ca/small.log) -- and
// whose 7 fields fit into the device (`device_total_bytes` > 0; else no size test), otherwise
// choose_single_pass.  A pure function of global data: every rank makes the same choice.
constexpr int64_t kCaAutoPoints = 6000000;
int choose_algo(const ProblemSpec& spec, const ProcGrid& grid, const GpuOptions& resolved, double device_total_bytes,
                int subdomains_per_device, bool direct_rows = true);

// The comm arena: PcgState (the all-reduce buffers) and one send + one receive buffer per halo
// slot (pmx/device_types.hpp kHaloSlots), all sends first, then all receives.
// Error of the local solution against the analytic one (k_error_norms), before any reduction
// over ranks: l2_error = sqrt(h1 h2 sum_e2) once summed over all ranks.
struct ErrorStats {
  double sum_e2 = 0.0;  // sum of (w - u)^2 over the owned nodes in D
  double max_e = 0.0;   // max |w - u| over the owned nodes in D
  double max_w = 0.0;   // max w over the owned nodes
};

// One ghost message of a rank: `count` elements from `send` go to the neighbour across `slot`
// (rank `peer`), and `count` elements from that neighbour land at `recv`.  `field` orders the
// messages of one slot (0 = r, 1 = p in the direct-row exchange; 0 for packed slots): the
// neighbour's message with slot opposite_slot(slot) and the same field is the partner.
struct HaloMsg {
  int slot, field, peer, count;
  void* send;
  void* recv;
};
struct HaloMsgs {
  HaloMsg m[2 * kHaloSlots];
  int n = 0;
};

struct CommLayout {
  size_t state_off = 0;          // PcgState
  size_t send_off[kHaloSlots] = {};
  size_t recv_off[kHaloSlots] = {};
  int edge_len[kHaloSlots] = {};  // elements per message (0: slot unused by this algorithm)
  int peer[kHaloSlots] = {-1, -1, -1, -1, -1, -1, -1, -1};  // rank across the slot, -1 = none
  size_t elem = 8;               // bytes per halo element
  size_t bytes = 0;              // total arena size
  bool single_pass = false;
  // slot s carries a message in this layout
  bool active(int s) const { return peer[s] >= 0 && edge_len[s] > 0; }
};

class GpuSubdomainSolver {
 public:
  GpuSubdomainSolver(const ProblemSpec& spec, const Subdomain& sd, const GpuOptions& opt,
                     uintptr_t external_arena = 0);
  ~GpuSubdomainSolver();
  GpuSubdomainSolver(const GpuSubdomainSolver&) = delete;
  GpuSubdomainSolver& operator=(const GpuSubdomainSolver&) = delete;

  // ca_gh > 0: the s-step's packed slots (ca_gh ghost lines of z and p per side, ca_gh x ca_gh corners)
  static CommLayout comm_layout(const Subdomain& sd, DType dtype, bool single_pass, int ca_gh = 0);
  // Upper bound of the device memory a solver for `sd` allocates (fields -- 4, or 5 for the
  // single-pass iteration -- tables, partials, comm arena).  Checked against hipMemGetInfo before
  // allocating; used by `pmx --plan` and the pcg1/pcg2 choice.
  static size_t estimate_device_bytes(const ProblemSpec& spec, const Subdomain& sd, DType dtype,
                                      bool single_pass);
  // ... for iteration algorithm `algo` (1 pcg1, 2 pcg2, 3 the s-step PCG: 5 fields with s ghost rows on
  // strips, plus the two face-coefficient fields)
  static size_t estimate_device_bytes_algo(const ProblemSpec& spec, const Subdomain& sd, DType dtype, int algo);

  // r=B, w=0, p=0, state reset, red_b <- (0, zr_0).  Single-pass: the driver then runs the ghost
  // exchange of r^0 (decomposed grids), sweep 0 (enqueue_phase_a) and the all-reduce of red_c.
  void enqueue_init(hipStream_t s);
  void enqueue_phase_a(hipStream_t s);  // k_pcg_a + reduce -> red_a
  // the two halves of each phase, for per-step timing (PcgDriver::profile_phases)
  void enqueue_kernel_a(hipStream_t s);
  // pcg1 only: the interior (part 1) or frame (part 2) tiles of the sweep, see launch_pcg1
  void enqueue_kernel_a_part(hipStream_t s, int part);
  bool has_interior_split() const { return pcg1_ && geom_.nb != 0; }
  void enqueue_reduce_a(hipStream_t s);
  void enqueue_kernel_b(hipStream_t s, bool pack);
  void enqueue_reduce_b(hipStream_t s);
  // k_pcg_b + reduce -> red_b, it += 1.  pack=false: the edges were packed by enqueue_pack.
  void enqueue_phase_b(hipStream_t s, bool pack = true);
  void enqueue_pack(hipStream_t s);     // pcg2, k_edge_r: r^{k+1} edges -> send buffers
  // pcg1: radius-2 edges (2 lines of r and p per side, corner values) of the buffers the next
  // sweep reads -> send buffers / receive buffers -> ghost cells of those buffers
  void enqueue_halo_pack(hipStream_t s);
  void enqueue_halo_unpack(hipStream_t s);
  void enqueue_poison_recv(hipStream_t s);  // recv buffers <- NaN (poison_halos debug mode)

  // Direct-row ghost exchange (pcg1 on row strips: x neighbours only, no y / corner neighbours).
  // The two owned edge rows of r^k and p^k are sent straight from the fields and received straight
  // into the two ghost rows of the buffers sweep k+1 reads: no pack / unpack kernels, no slot
  // buffers (a row span, padding included, is contiguous).  The driver turns it on when its
  // communicator moves arbitrary device spans (Comm::direct_rows).
  bool can_direct_rows() const {
    return (pcg1_ || ca_) && (geom_.nb & ~(kNbXlo | kNbXhi)) == 0 && sd_.nx >= (ca_ ? gh_ : 2);
  }
  void set_direct_rows(bool on);
  bool direct_rows() const { return direct_rows_; }
  // pcg1: the next Comm::halo call fills the inputs of sweep k (r^{k-1}, p^{k-1}); the driver sets
  // it before every exchange (the direct-row spans alternate between the double buffers)
  void set_halo_target(long long k) { halo_target_ = k; }
  long long halo_target() const { return halo_target_; }
  // this rank's messages of the next exchange, in the order every transport issues them
  HaloMsgs halo_msgs() const;
  // s-step strips: the messages of an exchange of (z, p) set `set` (halo_msgs() = the current set's)
  HaloMsgs ca_halo_msgs(int set) const;
  int ca_halo_set() const { return int(ca_blk_ & 1); }
  // s-step strips: the next pass 1 runs its interior tiles at once and its frame tiles (the only ones
  // that read ghost rows) after event e -- the ghost exchange on the driver's comm stream.  Without a
  // frame stream the whole pass waits.  One-shot.
  void set_ca_frame_wait(hipEvent_t e) { ca_frame_wait_ = e; }
  // s-step: the frame tiles of a split pass run on a side stream (forked and joined inside every
  // block); drop_side_stream() runs them in-stream from now on (one hardware queue: no forks)
  bool ca_side_stream() const { return ca_side_ != nullptr; }
  void drop_side_stream();

  // Checkpoint: the fields with ghosts (pcg1 / s-step: also the second r / z buffer),
  // the PCG scalars, the halo buffers and the s-step's CaState, i.e. everything the next iteration
  // reads.  Synchronous; written at batch boundaries.
  void save_checkpoint(std::ostream& os, hipStream_t s) const;
  void load_checkpoint(std::istream& is, hipStream_t s);
  int ckpt_version() const;  // file version of this solver's algorithm (3 pcg2, 5 pcg1, 7 s-step)

  PcgState read_state(hipStream_t s) const;  // synchronous D2H of the scalars
  std::vector<double> read_partials(hipStream_t s) const;  // the partials buffer (5 per tile slot)
  // device-side error norms of the current w (pending steps applied); synchronous
  ErrorStats error_norms(hipStream_t s) const;
  // host-mapped progress counters (GpuOptions::progress): sweeps reduced, ghost exchanges packed,
  // exchanges unpacked.  Plain host reads, no HIP call: safe from a watchdog thread.  All -1 when
  // progress tracking is off.
  void progress(long long out[3]) const;
  bool progress_enabled() const { return progress_dev_ != nullptr; }
  // Kernel isolation benchmark: pins the scalar state to a mid-solve iteration and launches
  // k_pcg_a (which=0) or k_pcg_b (which=1) alone `reps` times; returns ms per launch.  Leaves
  // the solver state invalid (call enqueue_init afterwards).
  double bench_kernel(int which, int abl, int reps, hipStream_t s);
  PcgState* state_dev() const { return state_; }
  double* red_a_dev() const { return state_->red_a; }
  double* red_b_dev() const { return state_->red_b; }
  double* red_c_dev() const { return state_->red_c; }
  // all-reduce buffer `which` (0: red_a, 1 value; 1: red_b, 2; 2: red_c, 5; 3: the s-step sums,
  // CaState::red, 21 -- nullptr without the s-step solver) and its length
  double* reduce_buf(int which) const {
    return which == 0 ? red_a_dev() : which == 1 ? red_b_dev() : which == 2 ? red_c_dev()
                                                    : (ca_state_ ? ca_state_->red : nullptr);
  }
  static int reduce_len(int which) { return which == 0 ? 1 : which == 1 ? 2 : which == 2 ? 5 : 7 * kCaMaxS; }
  void* send_dev(int side) const { return arena_ + layout_.send_off[side]; }
  void* recv_dev(int side) const { return arena_ + layout_.recv_off[side]; }
  const CommLayout& layout() const { return layout_; }
  uintptr_t arena_ptr() const { return reinterpret_cast<uintptr_t>(arena_); }

  // local interior of w (nx x ny, row-major) as fp64 on the host
  std::vector<double> download_w(hipStream_t s) const;
  // any local field (0 w, 1 r, 2 p0, 3 p1) including ghosts: (nx+2) x (ny+2)
  std::vector<double> download_field(int which, hipStream_t s) const;

  const Subdomain& sd() const { return sd_; }
  const ProblemSpec& spec() const { return spec_; }
  const GpuOptions& options() const { return opt_; }
  bool block_tiles() const { return block1_; }  // pcg1 sweeps as block tiles (pcg1_block.hip)
  bool reduction_in_sweep() const { return block1_ && block_fused_; }  // no separate reduce launch
  const DevGeom& geom() const { return geom_; }
  const DevTables& tables() const { return tables_; }
  const TileCfg& tiles() const { return pcg1_ ? tiles1_ : tiles_; }  // pcg_a (or pcg1)
  bool single_pass() const { return pcg1_; }
  // s-step PCG (GpuOptions::algo 3): a block of n <= ca_s() iterations is pass 1 -> reduction (+ the
  // block's scalars) -> pass 2; host_k() counts iterations enqueued
  bool ca() const { return ca_; }
  int ca_s() const { return ca_ ? ca_tiles_.s : 0; }
  const CaTiles& ca_tiles() const { return ca_tiles_; }
  // the same block in steps, for decomposed grids (the driver all-reduces CaState::red between
  // reduce and finish, and exchanges the s ghost rows of the new (z, p) set after pass 2)
  void enqueue_ca_pass(hipStream_t s, bool upd);
  // the fused pass (ca_fused()): pass 2 of the block just reduced + pass 1 of the next; its reduction
  // is enqueue_ca_reduce(.., fused = true)
  void enqueue_ca_fused(hipStream_t s);
  bool ca_fused() const { return ca_ && ca_tiles_.fuse != 0; }
  void enqueue_ca_reduce(hipStream_t s, int n, bool check_only, bool finish, bool fused = false);
  void enqueue_ca_finish(hipStream_t s, int n, bool check_only);
  // Kernel test hook (tests/test_gpu_ca_gram.py): set 0 <- (z, p) and w <- w0 from host arrays of
  // (nx + 2 gh) x (ny + 2) values (local rows 1-gh .. nx+gh, columns 0 .. ny+1, gh = ca_ghost_rows()),
  // then pass 1 and pass 2 -- or the fused pass -- once each with pass 2's coefficient vectors coef
  // (a, b, c: 3 x (2s+1)) and pa (s x (2s+1)).  Returns pass 1's 6s Gram sums over the tiles (the fused
  // pass: of the NEW basis), pass 2's s norm sums, and the new p, z, w (nx x ny).  Resets the solver.
  struct CaProbe {
    std::vector<double> gram, norms, p, z, w;
  };
  CaProbe ca_probe(const std::vector<double>& z, const std::vector<double>& p, const std::vector<double>& w,
                   const std::vector<double>& coef, const std::vector<double>& pa, bool fused, hipStream_t s);
  int ca_ghost_rows() const { return gh_; }
  // host mirror of CaState::blk (blocks enqueued): the (z, p) set the next exchange sends
  long long ca_blocks() const { return ca_blk_; }
  void set_ca_blocks(long long b) { ca_blk_ = b; }
  // fused schedule carried across batches: a batch ends with a fused pass (block b applied AND block
  // b+1's Gram partials summed), so the next batch starts at the reduction instead of pass 1 -- and the
  // batch boundary no longer costs pass 1 + pass 2 in place of one fused pass.  init clears it.
  bool ca_primed() const { return ca_primed_; }
  void set_ca_primed(bool v) { ca_primed_ = v; }
  size_t ca_primed_doubles() const { return size_t(ca_nq(ca_tiles_.s)) * size_t(ca_tiles_.ntilesf()); }
  // pcg1: host mirror of the device iteration counter S->it -- the index of the next sweep this
  // solver enqueues.  init sets it to 0, every enqueued reduction (which bumps S->it on the
  // device) advances it, load_checkpoint reads it from the checkpoint.  It picks the plain or the
  // w-moving k_pcg1 (see launch_pcg1); captured graphs depend on its phase modulo w_cycle().
  long long host_k() const { return host_k_; }
  void set_host_k(long long k) { host_k_ = k; }
  int w_cycle() const { return pcg1_ ? opt_.wcycle1 : 1; }
  bool w_sweep_next() const { return pcg1_ && host_k_ > 0 && host_k_ % w_cycle() == 0; }
  const TileCfg& tiles_b() const { return tiles_b_; }  // pcg_b
  int device() const { return opt_.device; }
  size_t field_bytes() const { return field_bytes_; }
  const std::vector<float>& placement_ms() const { return placement_ms_; }
  double placement_seconds() const { return placement_s_; }  // wall time of the probe (0: off)
  void* field_base(int which) const;  // pointer to local (0,0)
  size_t device_bytes() const;        // total device memory owned

 private:
  template <typename T> void init_impl(hipStream_t s);
  template <typename T> void phase_a_impl(hipStream_t s);
  template <typename T> void phase_b_impl(hipStream_t s, bool pack);
  template <typename T> void phase_a_kernel_only(hipStream_t s, int part = 0);
  template <typename T> void phase_b_kernel_only(hipStream_t s, bool pack = true);
  template <typename T> HaloBufs<T> halo() const;
  void ca_halo_impl(hipStream_t s, bool unpack);  // k_ca_halo on the (z, p) set the next block reads
  template <typename T> void halo_impl(hipStream_t s, bool unpack);
  void after_launch(hipStream_t s) const;
  void construct(uintptr_t external_arena);
  void release() noexcept;  // frees every allocation (destructor, failed constructor)

  ProblemSpec spec_;
  Subdomain sd_;
  GpuOptions opt_;
  GridInfo g_;
  DevGeom geom_{};
  DevTables tables_{};
  TileCfg tiles_{};    // pcg_a
  TileCfg tiles_b_{};  // pcg_b
  TileCfg tiles1_{};   // pcg1
  TileCfg tiles1w_{};  // pcg1, the w-moving sweeps (GpuOptions::rows1w / pf1w)
  const TileCfg& tiles1_for(bool wsweep) const { return wsweep ? tiles1w_ : tiles1_; }
  bool pcg1_ = false;
  bool ca_ = false;             // s-step PCG
  CaTiles ca_tiles_{};
  unsigned* ca_tbl_ = nullptr;  // its row-class table
  unsigned* ca_tbl_f_ = nullptr;  // ... of the fused pass's tiling
  char* ca_faces_ = nullptr;    // its face-coefficient fields (a, b)
  hipStream_t ca_side_ = nullptr;  // the frame tiles' stream (split kernels)
  hipEvent_t ca_ev_fork_ = nullptr, ca_ev_join_ = nullptr;
  hipEvent_t ca_frame_wait_ = nullptr;  // one-shot: the next pass 1's frame tiles wait for it
  template <typename T> void ca_pass_impl(hipStream_t s, int kind);  // 0 pass 1, 1 pass 2, 2 fused
  size_t ca_face_bytes_ = 0;    // one face-coefficient field (fp64)
  CaState* ca_state_ = nullptr;
  CaState ca_init_{};           // host template of the state init() uploads
  double* ca_chunk_ = nullptr;  // its reduction's chunk sums
  long long ca_blk_ = 0;        // blocks enqueued since init (CaState::blk's host mirror)
  bool ca_primed_ = false;      // partials_ hold the next block's Gram sums from a batch-ending fused pass
  int gh_ = 2;                  // ghost rows of the fields on each side
  bool ca_fuse_ = false;        // the s-step's fused pass (GpuOptions::ca_fuse, decided at construction)
  // the s-step kernels' geometry and face tables: geom_ / tables_, or under ca_dirichlet a standalone
  // grid of the subdomain's rows (gi0 = 0, M = nx + 1, tables shifted by gi0), whose rows 0 and nx + 1
  // are boundary rows (the kernels tell boundary from interior rows by the global row index)
  DevGeom ca_geom_{};
  DevTables ca_tables_{};
  int ca_gh_ = 2;               // ghost rows the s-step kernels compute on
  long long host_k_ = 0;
  bool direct_rows_ = false;
  long long halo_target_ = 0;
  TileCfg init_tiles_{};
  CommLayout layout_{};
  size_t elem_ = 8, field_bytes_ = 0, field_off_ = 0;
  // Fields w, r, p0, p1 (and pcg1's r2) in ONE allocation, field f at fields_ + f * field_stride_;
  // rows -1 .. nx+2 each.
  char* fields_ = nullptr;
  char* r2_ = nullptr;      // pcg1 only: the second r buffer (r is double-buffered there)
  size_t field_stride_ = 0;
  bool block1_ = false;       // pcg1 sweeps as block tiles (pcg1_block.hip)
  bool block_fused_ = false;  // ... which also finish the reduction (no k_reduce_n launch)
  char* field_raw(int f) const { return fields_ + size_t(f) * field_stride_; }
  void place_fields();                // placement probe (see gpu_solver.hip)
  void probe_iterations(hipStream_t s, hipEvent_t e0, hipEvent_t e1);
  std::vector<float> placement_ms_;   // probe: ms per candidate block (the kept one is the min)
  double placement_s_ = 0.0;
  double* tables_buf_ = nullptr;
  double* partials_ = nullptr;
  size_t npart_ = 0;
  double* reduce_ws_ = nullptr;  // k_reduce chunk sums + ticket (inside the partials allocation)
  char* arena_ = nullptr;
  bool own_arena_ = true;
  PcgState* state_ = nullptr;
  Pcg1Slot* tile_order_ = nullptr;    // pcg1 dispatch order + row classes (pcg1_build_order)
  Pcg1Slot* tile_order_w_ = nullptr;  // ... of tiles1w_ when its shape differs
  int slow_tiles_ = 0;
#ifdef PMX_WAVE_TRACE
  void* wtrace_ = nullptr;
  int wtrace_n_ = 0;
#endif
  PcgState* host_state_ = nullptr;  // pinned
  long long* progress_host_ = nullptr;  // host-mapped, coherent (GpuOptions::progress)
  long long* progress_dev_ = nullptr;   // its device address, or nullptr (off)
};

// ---------------------------------------------------------------------------
// Communication backends (RcclComm / LocalComm / SelfComm)
// ---------------------------------------------------------------------------
class Comm {
 public:
  virtual ~Comm() = default;
  // in-place sum of red_a (which=0, 1 double) or red_b (which=1, 2 doubles) over all ranks
  virtual void allreduce(std::vector<GpuSubdomainSolver*>& local, int which,
                         std::vector<hipStream_t>& streams) = 0;
  // send[s] of every rank -> recv[opposite side] of its neighbour
  virtual void halo(std::vector<GpuSubdomainSolver*>& local, std::vector<hipStream_t>& streams) = 0;
  virtual bool graph_capturable() const { return true; }
  // Failure detection: called by the driver at every host poll (once per batch);
  // throws if the communicator reported an asynchronous error (RCCL: ncclCommGetAsyncError).
  virtual void check_health() {}
  virtual std::string name() const = 0;
  virtual int world_size() const = 0;
  // Called before every kernel that writes this rank's send slots (the next exchange's pack): a
  // transport whose peers read those slots in place (IpcComm) waits here until they have.
  virtual void before_pack(std::vector<GpuSubdomainSolver*>&, std::vector<hipStream_t>&) {}
  // The transport moves any device span a rank's halo_msgs() names (not only its packed slot
  // buffers), so the driver may use the direct-row exchange (GpuSubdomainSolver::set_direct_rows).
  virtual bool direct_rows() const { return false; }
  // The pcg1 split sweep is the default with this transport (its exchange is the long pole).
  virtual bool prefers_split() const { return false; }
  // Error path of a threaded driver set: make every operation in flight or blocked on this
  // communicator return (RCCL: ncclCommAbort), so the other driver threads fail instead of
  // waiting for a rank that will never post.  The communicator is unusable afterwards.
  virtual void abort() {}
  // A communicator for local rank i alone, for a driver thread that owns just that rank (one host
  // thread per device).  Non-owning: valid while this communicator lives.
  virtual std::unique_ptr<Comm> rank_view(int i);
};

std::unique_ptr<Comm> make_self_comm();
// bench.py --loopback-rank: ONE rank of a P-rank decomposition alone on this device.  Every ghost
// message is a device copy of the real size on the exchange's stream -- from a zero buffer, so the
// rank solves its block with Dirichlet ghosts (a well-posed problem that runs as long as the real
// one) -- and the all-reduce is skipped: the real per-rank schedule (split sweep, frame stream,
// events, copies) runs at full speed as a timing rehearsal.
std::unique_ptr<Comm> make_loopback_comm();
std::unique_ptr<Comm> make_local_comm(std::vector<GpuSubdomainSolver*>& local);
// RCCL: one communicator per local solver.  `unique_id` is the 128-byte ncclUniqueId,
// `ranks` the global ranks of the local solvers, `nranks` the world size.  `split_halo`: a second
// communicator (ncclCommSplit) carries the ghost exchange, so the exchange on the comm stream and the
// all-reduce on the compute stream never queue behind each other (overlapped schedules).  Without it
// every call goes through ONE communicator -- the serialized schedule (overlap off), where halo and
// all-reduce are issued on one stream in a fixed order and no two RCCL kernels are ever in flight
// together (bench.py rung 2).
std::unique_ptr<Comm> make_rccl_comm(const std::string& unique_id, int nranks,
                                     const std::vector<int>& ranks, const std::vector<int>& devices,
                                     bool capturable, bool split_halo = true);
std::string rccl_unique_id();

// IPC transport (comm/ipc_comm.hip): one rank per process, peers' arenas mapped with
// hipIpcOpenMemHandle.  Two-phase setup: construct, ipc_export() on every rank, exchange the
// strings out of band, ipc_attach() with all of them (indexed by rank).
std::unique_ptr<Comm> make_ipc_comm(GpuSubdomainSolver* local, int world);
std::string ipc_export(Comm* ipc);
void ipc_attach(Comm* ipc, const std::vector<std::string>& exports);

// One communication call as a rank's driver issued it (RecordingComm, tests): comm 0 = the
// scalar communicator, 1 = the halo communicator (0 too without a split halo communicator); op
// "allreduce" (count = doubles), or a halo group ("group_start", "send"/"recv" with element count
// and peer rank, "group_end"); `stream` = the HIP stream the call was issued on.
struct CommEvent {
  int comm;
  std::string op;
  int count;
  int peer;
  long long stream;
};
// Records the calls instead of communicating (no data moves).  Mimics RCCL's driver defaults
// (prefers_split) and its communicator layout (`split_halo` as make_rccl_comm), so a driver on it
// issues exactly the sequence it would issue on RCCL.
std::unique_ptr<Comm> make_recording_comm(std::vector<CommEvent>* log, int world, bool split_halo = true);

struct RunStats {
  int64_t iters = 0;
  Status status = Status::kRunning;
  double diff = 0.0;
  double init_seconds = 0.0;
  double solve_seconds = 0.0;
  int64_t launched = 0;    // iterations enqueued (>= iters; the rest were device no-ops)
  bool nan = false;
  // per-step times (seconds, summed over the profiled iterations; only profile_phases() fills
  // them).  Mapped onto the reference's 5 buckets (stage4-mpi+cuda/poisson_mpi_cuda_f.cu:956-980)
  // by the CLI: compute = kernel_a + kernel_b, comm = allreduce + halo (incl. edge pack),
  // dot = reduce; copy and precond are 0 by construction (no H2D/D2H in the loop, D^-1 fused).
  double t_kernel_a = 0, t_kernel_b = 0, t_reduce = 0, t_allreduce = 0, t_halo = 0, t_comm = 0;
};

class PcgDriver {
 public:
  // All local solvers must run the same iteration algorithm (checked).  The single-pass
  // iteration runs: sweep -> 5-value reduction -> ONE all-reduce (red_c); on decomposed grids the
  // radius-2 ghost exchange (pack -> send/recv -> unpack) runs on the comm stream, overlapped with
  // the reduction and the all-reduce, and the next sweep waits for it.
  PcgDriver(std::vector<GpuSubdomainSolver*> local, Comm* comm, int graph_batch);
  ~PcgDriver();

  void init();                       // enqueue init on all ranks, all-reduce, halo; sync
  void enqueue_iterations(int64_t n);  // no host sync (graph replays when possible)
  void synchronize();
  // init (or continue from the current device state when do_init is false, e.g. after a
  // checkpoint load) + iterate until the device says done; on_checkpoint is called every
  // ckpt_every iterations (at batch granularity) with the device idle
  RunStats solve(int poll_batches = 1, bool do_init = true, int64_t ckpt_every = 0,
                 const std::function<void(const PcgState&)>& on_checkpoint = {});
  RunStats profile_phases(int64_t n);    // eager iterations with events around each phase
  PcgState state(int idx = 0);
  std::vector<hipStream_t>& streams() { return streams_; }
  bool overlapped() const { return overlap_; }
  bool poisoned() const { return poison_; }
  // pcg1 split sweep in use (interior tiles overlap the previous exchange, see enqueue_split_iteration)
  bool split_sweep() const { return split_; }
  bool direct_rows() const { return direct_; }

  // Which path ran: iterations replayed from captured graphs / enqueued as individual launches
  // since the last reset, and the graph lengths used (bench.py reports them for its timed region).
  struct PathStats {
    int64_t graph_iters = 0, eager_iters = 0;
    std::vector<int> graph_lengths;  // distinct lengths, in first-use order
  };
  const PathStats& path_stats() const { return path_; }
  void reset_path_stats() { path_ = PathStats{}; }
  // Capture -- without running anything -- every graph that enqueue_iterations(n) issued now would
  // replay (full batches of graph_batch and the remainder), so a timed region replays graphs only
  // and pays no capture.  False when this driver cannot capture (graph_batch 0, check mode, a
  // non-capturable comm, several streams).
  bool prepare(int64_t n);
  // n iterations as individual launches, never from a graph (the bench's canary iteration)
  void enqueue_eager(int64_t n);

 private:
  void enqueue_one_iteration();
  // s-step PCG: n iterations as blocks of ca_s() (the last one shorter), graphs of ca_batch().  mark:
  // profile_phases' event hook, called after every step with its bucket (PhaseBucket); with a hook the
  // ghost exchange runs on the compute stream (each step's time is its own)
  enum PhaseBucket { kPhA = 0, kPhB, kPhRed, kPhAr, kPhHalo };
  void enqueue_ca(int64_t n, const std::function<void(int)>& mark = {});
  int ca_batch() const;
  void ca_exchange(std::vector<hipStream_t>& streams);
  int ca_phase() const;  // captured s-step batches on decomposed grids depend on the (z, p) set parity
  // pack -> comm -> unpack, filling the inputs of sweep `target` (direct rows: comm only)
  void halo_exchange_pcg1(std::vector<hipStream_t>& streams, long long target);
  void set_halo_target(long long k);
  // captured batches depend on the w-cycle phase of their first sweep, and with direct rows also on
  // its parity (the exchanged spans alternate between the double buffers)
  // pcg1 with neighbours: every exchange names its target sweep's buffer parity in its launch
  // arguments (direct spans or pack/unpack), so a captured batch is only valid at its parity
  int graph_period() const { return ca_ ? 1 : local_[0]->w_cycle() * (single_pass_ && any_nb_ ? 2 : 1); }
  void enqueue_split_iteration();  // pcg1, decomposed, overlap: interior/frame sweep split
  void join_halo();                // compute stream waits for a pending ghost exchange
  // captured batch of `len` iterations starting at w-cycle phase `phase`, built on first use;
  // nullptr when capture is impossible (graph_failed_ is then set)
  hipGraphExec_t graph_for(int phase, int len);
  hipGraphExec_t build_graph(int phase, int len);
  // f(index of the first solver using a stream, index of that unique stream) per distinct stream
  template <typename F>
  void for_each_stream(F&& f) {
    size_t u = 0;
    for (size_t i = 0; i < streams_.size(); ++i) {
      if (i > 0 && streams_[i] == streams_[i - 1]) continue;
      HIP_CHECK(hipSetDevice(local_[i]->device()));
      f(i, u++);
    }
  }
  void poison(std::vector<hipStream_t>& streams);

  std::vector<GpuSubdomainSolver*> local_;
  Comm* comm_;
  int graph_batch_;
  std::vector<hipStream_t> streams_;
  // halo/compute overlap: one comm stream per compute stream, fork/join events per iteration
  bool overlap_ = false;
  bool poison_ = false;
  bool single_pass_ = false;
  bool ca_ = false;  // s-step PCG (one undecomposed subdomain)
  bool any_nb_ = false;
  bool direct_ = false;  // direct-row ghost exchange (GpuSubdomainSolver::set_direct_rows)
  std::vector<hipStream_t> comm_streams_;
  std::vector<hipEvent_t> ev_packed_, ev_halo_;
  // split sweep (pcg1 with neighbours and overlap): the frame tiles run on their own stream
  bool split_ = false;
  bool halo_pending_ = false;  // a ghost exchange on the comm stream not yet joined
  std::vector<hipStream_t> frame_streams_;
  std::vector<hipEvent_t> ev_ar_, ev_fdone_, ev_swept_;
  // frame tiles on the comm stream, ahead of the exchange that reads their edge lines (two
  // cross-stream edges per iteration instead of four; enqueue_split_iteration)
  bool frame_on_comm_ = false;
  bool graph_failed_ = false;  // capture is not possible for this driver: eager launches
  std::vector<hipGraph_t> graphs_;
  std::vector<hipGraphExec_t> execs_;
  // captured batches by (phase of the w cycle at their first sweep, length): pcg1 bakes the plain /
  // w sweep kernel choice into the graph
  std::map<std::pair<int, int>, hipGraphExec_t> exec_by_key_;
  PathStats path_;
  void note_graph(int len);
  void advance_host_k(long long n);
};

}  // namespace pmx
