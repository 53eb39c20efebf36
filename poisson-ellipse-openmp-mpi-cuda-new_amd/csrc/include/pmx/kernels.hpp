// Host-side launchers of the HIP kernels (csrc/hip/*.hip).
//
// Fused PCG iteration (redesigned to 2 streaming kernels / iteration):
//   pcg_a : p^k = D^-1 r + beta p^{k-1} on the tile + 1-cell ring (LDS row ring), A p^k on the
//           tile, block partial (A p^k, p^k)        [replaces K7 + K1 + K3(Ap,p) of the reference]
//   pcg_b : A p^k recomputed from p^k, w += alpha p, r -= alpha A p, z = D^-1 r (not stored),
//           block partials sum dw^2 and (z, r), halo pack of r  [replaces K6 + K2 + K3(z,r) + D1]
//   reduce: deterministic single-block finish of the block partials into the PcgState scalars.
// HBM traffic: 3 T/pt for pcg_a (r, p_old read, p write) + 5 T/pt for pcg_b (p, w, r read,
// w, r write) = 64 B/pt/iter in fp64 vs ~176 B/pt in the reference.
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "pmx/device_types.hpp"

namespace pmx {

// One dispatch slot of a pcg1 order table: the tile, and the coefficient class (2 bits: 0 cut,
// 1 all faces inside D, 2 all outside) of each row r = 0..31 the tile's march visits, row r being
// local row i0 - 3 + r (the pipeline's initial row, then rows i0-2 .. i1+2).  With the classes in
// the slot a wave finds a row's class with a shift instead of ~11 scalar loads and ~20 compares.
struct Pcg1Slot {
  int id;
  int pad;
  unsigned long long cls;
};

struct TileCfg {
  int kind = 0;       // 0: workgroup tile + LDS row ring (pcg_kernels.hip)
                      // 1: wave tile + DPP lane shifts, software-pipelined register ring
                      // 2: wave tile + DPP lane shifts, ring-free short tiles (pcg_b only)
                      // 3: single-pass pcg1 tiles (overlapped by 2 columns, 3-stage row pipeline)
  int block = 256;    // columns per tile (kind 0: = threads per block; kind 1: = 64*vec)
  int rows = 0;       // rows per tile (marching length); 0 = auto
  int vec = 1;        // kind 1: columns per lane
  int waves = 1;      // kind 1: independent wave tiles per workgroup
  int abl = 0;        // kernel-isolation ablation bits (kAbl*), 0 in production
  int pair_w = 0;     // kind 2: paired w updates (k_pcg_b_rows_paired, pcg_kernels_dpp.hip)
  int pf = 1;         // kind 3: rows prefetched ahead of the computed row
  int tiles_i = 0, tiles_j = 0;
  // kind 3 on decomposed grids: the tiles [ti_lo, ti_hi) x [tj_lo, tj_hi) read no ghost cell of a
  // side that has a neighbour ("interior"); the rest form the frame (see launch_pcg1's part)
  int ti_lo = 0, ti_hi = 0, tj_lo = 0, tj_hi = 0;
  // kind 3: dispatch order of the whole-grid (order0) and interior (order1) launches: position
  // -> tile id, the tiles the ellipse cuts first within each XCD's share (pcg1_build_order);
  // nullptr = natural order
  const Pcg1Slot* order0 = nullptr;
  const Pcg1Slot* order1 = nullptr;
  const Pcg1Slot* order2 = nullptr;  // the frame tiles
  int groups[3] = {0, 0, 0};  // waves > 1: workgroups of each part (lockstep groups, pcg1_build_order)
  int arith32 = 0;  // kind 3 with fp32 storage: 1 = fp32 stencil arithmetic (GpuOptions::arith32)
  int lds_pad = 0;  // kind 3: dynamic LDS bytes per workgroup that cap the resident waves per CU
  int dpf = 0;      // kind 3: FAST tiles prefetch their rows dpf ahead by LDS-DMA (0 = registers)
  int bwaves = 8;   // kind 3 block tiles (pcg1_block.hip): waves per workgroup
  int interior_tiles() const { return (ti_hi - ti_lo) * (tj_hi - tj_lo); }
  int ntiles() const { return tiles_i * tiles_j; }
};

TileCfg make_tiles(const DevGeom& G, int block, int rows);
// rows = 0: auto, about target_tiles tiles but no taller than max_auto_rows
TileCfg make_wave_tiles(const DevGeom& G, int vec, int waves, int rows, int max_auto_rows = 32,
                        int target_tiles = 22000);
// kind 2 tiles for k_pcg_b_rows (rows = 0: 2)
TileCfg make_row_tiles(const DevGeom& G, int vec, int waves, int rows);
// kind 3 tiles for k_pcg1: 64*vec - 4 owned columns, rows = 0: auto
TileCfg make_pcg1_tiles(const DevGeom& G, int vec, int waves, int rows, int pf = 0, int elem = 8);
// padding LDS (bytes per workgroup) that lets at most wpcu workgroups of k_pcg1 (static LDS: 4 KiB
// per wave) share a CU; 0 for no cap
int pcg1_lds_pad(int wpcu, int waves);

enum ReduceMode : int { kSkipIfDone = 1, kBumpIter = 2 };

// Ablation bits for the kernel-isolation benchmark (GpuSubdomainSolver::bench_kernel): each
// switches off one part of the wave-tile kernels so its cost can be measured.  Results are
// numerically meaningless with any bit set.
enum AblBits : int {
  kAblHalo = 1, kAblAp = 2, kAblCoef = 4, kAblStore = 8,
  kAblHaloLoads = 16,  // skip the halo-column loads (k_pcg_a) / edge loads (k_pcg_b)
  kAblNoXcd = 64,      // identity workgroup -> tile mapping instead of the XCD-aware remap
};

template <typename T>
void launch_init(const DevGeom& G, const DevTables& Tb, T* w, T* r, HaloBufs<T> H,
                 double* partials, const TileCfg& tc, hipStream_t s);

template <typename T>
void launch_pcg_a_wave(const DevGeom& G, const DevTables& Tb, const T* r, T* p0, T* p1,
                       HaloBufs<T> H, double* partials, PcgState* S, const TileCfg& tc, bool exact,
                       hipStream_t s);
template <typename T>
void launch_pcg_b_wave(const DevGeom& G, const DevTables& Tb, T* w, T* r, const T* p0,
                       const T* p1, HaloBufs<T> H, double* partials, PcgState* S,
                       const TileCfg& tc, bool exact, hipStream_t s);

// Single-pass PCG iteration (pcg1_kernels.hip): p^k, A p^k, w, r^k, z^k, A z^k in one sweep,
// 5 partials per tile (rho, (Az,z), (Az,p), (Ap,p), |p|^2).  S->it == 0 is the init sweep.
// r is double-buffered (overlapped tiles read neighbour rows/columns of r^{k-1} while others
// write r^k): sweep k reads (k & 1 ? r2 : r).  Decomposed grids read the radius-2 ghosts that
// launch_pcg1_halo unpacked into the fields.
// part: 0 = every tile; 1 = the interior tiles only (they read no ghost cell, so they may run
// while the previous sweep's ghost exchange is still in flight); 2 = the frame tiles only.
// Parts 1 and 2 of one sweep may run concurrently on two streams: they write disjoint partials.
// wsweep: launch the kernel that moves w; it must be set exactly on the sweeps k >= 1 with
// k % S->w_cycle == 0 (the caller mirrors the device iteration counter; a mismatch stops the solve
// with status breakdown and the NaN flag).
// Builds tc.order0/order1/order2 in d_order (pcg1_order_slots(tc) slots): per launch part, the
// tiles of each XCD's share of the positions with their row classes; slow_first: the tiles with
// cut (slow-path) rows go first within each share.  Returns the number of such tiles.
// tc.waves > 1 (lockstep workgroups): the positions come in groups of tc.waves -- up to tc.waves
// adjacent tiles of ONE tile row, marched side by side by the waves of one workgroup; unused slots
// hold id -1; tc.groups[part] = the workgroups of each part, the XCD shares and the cut-first
// ordering are per group.
int pcg1_build_order(const DevGeom& G, const DevTables& Tb, TileCfg& tc, Pcg1Slot* d_order, bool slow_first,
                     hipStream_t s);
size_t pcg1_order_slots(const TileCfg& tc);  // d_order capacity pcg1_build_order needs

template <typename T>
void launch_pcg1(const DevGeom& G, const DevTables& Tb, T* w, T* r, T* r2, T* p0, T* p1,
                 double* partials, PcgState* S, const TileCfg& tc, hipStream_t s, int part = 0,
                 bool wsweep = false);

// pcg1 sweep with block tiles (pcg1_block.hip): one workgroup per tc.rows x 124 tile, the three
// pipeline stages row-parallel; undecomposed fp64 grids; partial sums per tile as k_pcg1.  With a ticket the sweep also finishes the reduction (red_c =
// sums * weights, S->it + 1, progress[0]), replacing launch_reduce_n.
bool pcg1_block_shape_ok(int rows, int waves);  // an instantiated (rows, waves per workgroup) variant
template <typename T>
void launch_pcg1_block(const DevGeom& G, const DevTables& Tb, T* w, T* r, T* r2, T* p0, T* p1, double* partials,
                       PcgState* S, const TileCfg& tc, hipStream_t s, bool wsweep, const double* weights = nullptr,
                       unsigned* ticket = nullptr, long long* progress = nullptr);

// s-step PCG (ca_kernels.hip): s iterations per block of pass 1 (basis + Gram partials), one
// reduction that also runs the block's scalar recurrences, and pass 2 (p, z, w updated).
// Undecomposed fp64 grids; fields w and two (z, p) sets, the set read by a block in CaState::blk.
struct CaTiles {
  int s = 3;        // block size = basis degree (2 or 3)
  int he = 4;       // extra columns loaded per side ((s + 1) & ~1)
  int wo = 120;     // owned columns per wave tile (128 - 2 he)
  int rows = 0;     // rows per tile (pass 1)
  int tiles_i = 0, tiles_j = 0;
  int rows2 = 0, tiles_i2 = 0;  // pass 2's tile rows (same columns)
  int cwords = 0;   // row-class words per tile column (16 rows each)
  unsigned* tbl = nullptr;  // row classes (ca_build_classes), tiles_j * cwords words, owned by the caller
  const double* fa = nullptr;  // face coefficients a, b at every local node (ca_build_faces), pitched as
  const double* fb = nullptr;  // the fields, local (0, 0); read on the rows the ellipse cuts
  int gh = 2;                  // ghost rows of the fields on each side: 2, or 3 = s on a decomposed strip
  // interior rectangles of the two tilings (every tile "fast": no Dirichlet node or partial width in
  // reach): [ti_lo, ti_hi) x [tj_lo, tj_hi) for pass 1, [ti_lo2, ti_hi2) x (same columns) for pass 2
  int ti_lo = 0, ti_hi = 0, tj_lo = 0, tj_hi = 0, ti_lo2 = 0, ti_hi2 = 0;
  int split = 1;       // interior tiles by a fast-only kernel at 3 waves per SIMD, the frame by the general one
  int split_upd = 1;   // the same for pass 2
  int dma = 1;         // pass 1: interior tiles prefetch their rows by LDS-DMA (0: registers)
  int waves_gram = 2;  // waves per SIMD the pass-1 registers must allow (2 or 3)
  int waves_upd = 3;   // ... pass 2 (2 or 3)
  // fused pass (k_ca_fused: pass 2 of block b + pass 1 of block b+1 in one march, radius 2s): its own
  // tiling of rows_f x wo_f (= 128 - 4 s) tiles, its interior rectangle and its row-class table
  int fuse = 0;
  int rows_f = 0, tiles_i_f = 0, tiles_j_f = 0, wo_f = 116, he_f = 6;
  int ti_lo_f = 0, ti_hi_f = 0, tj_lo_f = 0, tj_hi_f = 0;
  int split_f = 1;     // interior tiles by the fast-only kernel, the frame by the general one
  int waves_f = 3;     // waves per SIMD the fused interior kernel's registers must allow (2 or 3)
  int rg_f = 1;        // fused interior tiles: row steps per producer / consumer barrier (1, 2, 4)
  // split fused pass: the frame kernel launched before (1) or after (0) the interior.  In a captured
  // graph the first-launched node starts first: frame first delayed the interior by up to ~140 us and
  // ran it slower; driver command 1.004-1.013 (frame first) vs 0.965-0.970 ms/step (frame last), three
  // interleaved fresh-process runs each (profiles/r6/frame_order/)
  int frame_first_f = 0;
  int dma_f = 0;       // fp64 fused interior tiles: the producer's rows by LDS-DMA, 4 ahead (0: registers, 1 ahead)
  unsigned* tbl_f = nullptr;
  int ntiles() const { return tiles_i * tiles_j; }
  int ntiles2() const { return tiles_i2 * tiles_j; }
  int ntilesf() const { return tiles_i_f * tiles_j_f; }
};
// rows_f: the fused tiling's rows (0 = auto)
CaTiles make_ca_tiles(const DevGeom& G, int s, int rows, int rows2 = 0, int rows_f = 0);
int ca_nq(int s);  // partials per tile (pass 1's Gram products + pass 2's norms)
// fused: the classes of the fused tiling (t.he_f, t.wo_f, t.tiles_j_f columns) instead of pass 1/2's
void ca_build_classes(const DevGeom& G, const DevTables& Tb, const CaTiles& t, unsigned* tbl, hipStream_t s,
                      bool fused = false);
// fa / fb: local (0, 0) of two field-sized arrays (rows -1 .. nx+2 allocated)
void ca_build_faces(const DevGeom& G, const DevTables& Tb, double* fa, double* fb, int gh, hipStream_t s);
// the s-step's packed ghost exchange on 2-D blocks (k_ca_halo): pack z, p of one set into the send
// slots, or unpack the receive slots into the ghost rows / columns / corners
template <typename T>
void launch_ca_halo(const DevGeom& G, T* z, T* p, const HaloBufs<T>& H, int gh, bool unpack, hipStream_t s,
                    long long* progress);
// z = D^-1 r in place, p = z (the first block's set 0)
template <typename T>
void launch_ca_init(const DevGeom& G, const DevTables& Tb, T* z, T* p, hipStream_t s);
template <typename T>
// sframe: the stream of the frame tiles' kernel with t.split (nullptr: s); the caller forks and joins it.
// frame_wait: an event the tiles that read ghost rows wait for (the frame on sframe, or the whole pass)
void launch_ca_sweep(const DevGeom& G, const DevTables& Tb, T* w, T* z0, T* z1, T* p0, T* p1, double* partials,
                     const PcgState* S, const CaState* C, const CaTiles& t, bool upd, hipStream_t s,
                     hipStream_t sframe = nullptr, hipEvent_t frame_wait = nullptr);
// the fused pass (undecomposed grids, t.fuse): after the reduction of block b, block b's update and
// block b+1's Gram partials (the reduction then takes n = n2 = t.ntilesf()); a pending rewind instead
// rewinds w.  t.tbl_f: the fused tiling's row classes (ca_build_classes with fused = true).
template <typename T>
void launch_ca_fused(const DevGeom& G, T* w, T* z0, T* z1, T* p0, T* p1, double* partials, const CaState* C,
                     const CaTiles& t, hipStream_t s, hipStream_t sframe = nullptr, hipEvent_t frame_wait = nullptr);
// chunk: kCaReduceMaxBlocks * ca_nq(s) doubles of workspace; nmax: iterations this block may run
constexpr int kCaReduceMaxBlocks = 256;
// up to this many tiles the s-step reduction runs in one workgroup (k_ca_reduce1: no chunk hand-off)
constexpr int kCaReduce1Max = 12288;
// check_only: the pending stop test alone (after the last block of a batch; pass 2 then rewinds w if
// the test stopped inside that block)
// n / n2: pass 1 / pass 2 tiles (the partials of each)
// finish = false (decomposed grids): the rank's sums go to CaState::red for the all-reduce, and
// launch_ca_finish runs the scalars on the reduced sums afterwards
void launch_ca_reduce(const double* partials, int n, int n2, int s_, double h, double wdiff, int nmax,
                      bool check_only, PcgState* S, CaState* C, double* chunk, hipStream_t s,
                      long long* progress = nullptr, bool finish = true);
void launch_ca_finish(int s_, double h, double wdiff, int nmax, bool check_only, PcgState* S, CaState* C,
                      hipStream_t s, long long* progress = nullptr);

// pcg1 ghost exchange: pack (unpack=false) the radius-2 edges of the buffers sweep `target` reads
// (parity of target) into H.send, or unpack H.recv into their ghost cells.
#ifdef PMX_WAVE_TRACE
void* pcg1_wave_trace_setup(long long it, int nwaves);
#endif

template <typename T>
void launch_pcg1_halo(const DevGeom& G, T* r, T* r2, T* p0, T* p1, HaloBufs<T> H, long long target,
                      bool unpack, hipStream_t s, long long* progress = nullptr);

// Halo/compute overlap: r^{k+1} on the subdomain edges that have a neighbour,
// written to the send buffers only, with exactly the arithmetic of pcg_b.  Runs first so the
// ghost exchange on the comm stream overlaps pcg_b, which then skips its own packing.
template <typename T>
void launch_edge_r(const DevGeom& G, const DevTables& Tb, const T* r, const T* p0, const T* p1,
                   HaloBufs<T> H, const PcgState* S, bool exact, hipStream_t s);

// Deterministic reduction of n block partials (nq interleaved values each) into out[0..nq),
// scaled by w0/w1.  `ws` is a per-solver workspace of kReduceWsDoubles doubles whose ticket
// word starts zeroed; the kernel re-arms it.  One workspace per stream (launches on a workspace
// must be stream-ordered).
constexpr int kReduceMaxBlocks = 64;
// k_reduce: chunk sums [0, 2*64) + ticket; k_reduce_n: its own chunk sums + ticket after that
constexpr int kReduceNOffset = 2 * kReduceMaxBlocks + 2;
constexpr int kReduceWsDoubles = kReduceNOffset + 8 * kReduceMaxBlocks + 2;
void launch_reduce(const double* partials, int n, int nq, double w0, double w1, double* out,
                   PcgState* S, int mode, double* ws, hipStream_t s);
// the same for nq = 5 interleaved values (k_pcg1 partials), out[q] = sum_q * weights[q].
// progress: optional host-mapped counters (GpuSubdomainSolver::progress): [0] <- S->it after the
// bump; launch_pcg1_halo counts [1] (exchanges packed) and [2] (exchanges unpacked).
void launch_reduce_n(const double* partials, int n, int nq, const double* weights, double* out,
                     PcgState* S, int mode, double* ws, hipStream_t s, long long* progress = nullptr);

// Deterministic in-process "all-reduce" across P subdomains on one device (LocalComm):
// out_k[q] = sum_r in_r[q] for every k, summed in rank order.
void launch_local_allreduce(double* const* bufs, int nranks, int nq, hipStream_t s);

// Per-row coefficient classes (see DevTables::acls); rows gi = 0..M+1, columns j = 0..N+1.
void launch_classify(const DevGeom& Gglobal, const DevTables& Tb, int* acls, int* bcls, hipStream_t s);

// MFMA wave reductions on test data: per wave64 w, out[3w..3w+2] = (sum x, sum x, sum x^2)
template <typename T>
void launch_wave_sums(const T* x, T* out, int nwaves, hipStream_t s);

// ---- unfused ops (tests, naive solver mode, bit-equality checks) ----
// All fields are local arrays with ghost ring: element (li,lj) at f[li*pitch+lj].
void launch_assemble(const DevGeom& G, const DevTables& Tb, double* a, double* b, double* B,
                     int64_t pitch_ab, hipStream_t s);
template <typename T>
void launch_apply_a(const DevGeom& G, const DevTables& Tb, const T* p, T* Ap, bool exact,
                    hipStream_t s);
template <typename T>
void launch_precond(const DevGeom& G, const DevTables& Tb, const T* r, T* z, bool exact,
                    hipStream_t s);
// partial sums of x*y over the interior into partials[nblocks]; returns nblocks used
template <typename T>
int launch_dot_partials(const DevGeom& G, const T* x, const T* y, double* partials, int max_blocks,
                        hipStream_t s);

// Error vs the analytic solution (k_error_norms): per block (sum e^2 in D, max |e| in D, max w)
// into out[3 * nblocks]; w_eff = w + ca pa (+ cb pb) for npend = 1 (2) pending w steps.  Returns
// the number of blocks used.
template <typename T>
int launch_error_norms(const DevGeom& G, const DevTables& Tb, const T* w, const T* pa, double ca,
                       const T* pb, double cb, int npend, double* out, int max_blocks, hipStream_t s);

}  // namespace pmx
