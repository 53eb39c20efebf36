// Plain-old-data structs shared by host orchestration and HIP kernels.
#pragma once

#include <cstdint>

namespace pmx {

// Device pointers to the 1D face tables of pmx/geometry.hpp, indexed by GLOBAL node index.
struct DevTables {
  const double* rv;   // vertical-face clip root at x_i - h1/2   (M+2)
  const double* xlo;  // x_i - h1/2                               (M+2)
  const double* xhi;  // x_i + h1/2                               (M+2)
  const double* x;    // x_i                                      (M+2)
  const double* rh;   // horizontal-face clip root at y_j - h2/2  (N+2)
  const double* ylo;  // y_j - h2/2                               (N+2)
  const double* yhi;  // y_j + h2/2                               (N+2)
  const double* y;    // y_j                                      (N+2)
  // Per-row coefficient classes (4 ints per GLOBAL row gi = 0..M+1), built on the device by
  // k_classify from the exact formulas: for j < c[0] or j > c[3] the coefficient is exactly
  // 1/eps (face outside D), for c[1] <= j <= c[2] exactly 1 (face inside D), otherwise the face
  // is cut by the ellipse and the exact formula is evaluated.  acls: a(gi, j), bcls: b(gi, j).
  const int* acls;
  const int* bcls;
};

// Neighbour bits: the 4 sides, then the 4 diagonal neighbours (only the single-pass iteration,
// whose stencil radius is 2, needs the corner values of the diagonal ranks).
enum NbBits : int {
  kNbXlo = 1, kNbXhi = 2, kNbYlo = 4, kNbYhi = 8,
  kNbXloYlo = 16, kNbXloYhi = 32, kNbXhiYlo = 64, kNbXhiYhi = 128,
};
// Halo slots: 0 x-lo, 1 x-hi, 2 y-lo, 3 y-hi, 4 (x-lo, y-lo), 5 (x-lo, y-hi), 6 (x-hi, y-lo),
// 7 (x-hi, y-hi).  Slot s of a rank talks to the rank whose slot opposite_slot(s) faces back.
constexpr int kHaloSlots = 8;
inline constexpr int opposite_slot(int s) { return s < 4 ? (s ^ 1) : 11 - s; }

// One subdomain's geometry as seen by a kernel.  Local node (li, lj), li = -1..nx+2,
// lj = -1..ny+2, lives at field[li * pitch + lj]; global index gi = gi0 + li.  Rows -1 and nx+2
// and columns -1 and ny+2 are the second ghost layer of the single-pass iteration (column -1 of
// row li is the last padding element of row li-1, pitch >= ny + 10).
struct DevGeom {
  int nx, ny;
  int64_t pitch;
  int gi0, gj0;
  int M, N;
  int nb;  // NbBits: neighbour exists on that side / corner (else Dirichlet ghost)
  int ref_ellipse;
  double h1, h2, eps, inv_eps, h1h2;
  double cx, cy;  // 1/h1^2, 1/h2^2
  double dinv_in, dinv_out;  // 1/D for all-inside / all-outside stencils (fast mode)
  double ax, by, F;
};

// Device-resident PCG scalars.  The host never reads these inside the loop; it
// polls `done` once per graph batch (SURVEY §7.1 "graphs + predication").
struct alignas(64) PcgState {
  double red_a[2];   // [0] = (Ap,p) (weighted).  All-reduce buffer A.
  double red_b[2];   // [0] = sum dw^2 (weighted per norm), [1] = (z,r).  All-reduce buffer B.
  double zr[2];      // zr_m stored at slot m & 1
  double diff;       // last ||w^{k+1} - w^k||
  double delta;      // tolerance
  double bd_tol;     // breakdown guard on (A p, p)
  long long it;      // iteration currently executing (1-based)
  long long max_iter;
  long long iters;   // final iteration count (valid when done)
  int done;
  int status;        // pmx::Status
  int norm;          // pmx::Norm
  int nan_flag;      // set when a reduction produced NaN/Inf (failure detection)
  // Paired w updates (fast row kernel): odd iterations leave w^{k+1} = w^k + alpha_k p^k pending
  // and the next (even) iteration applies both steps in one read-modify-write of w.
  double alpha[2];   // alpha_k at slot k & 1
  long long w_pend;  // k whose alpha_k p^k is not yet in w (0 = w is current); p^k is in p[k & 1]
  double pair_min_beta;  // |beta_k| below which p^{k-1} is re-read instead of recovered
  int pair_w;            // 0: w updated every iteration, 1: paired updates (GpuOptions::pair_w)
  // Single-pass iteration (pcg1_kernels.hip): all-reduce buffer C = (z,r), (Az,z), (Az,p),
  // (Ap,p) (weighted) and |p|^2 (weighted per norm) of the last sweep.
  double red_c[5];
  // Single-pass halo: index of the sweep whose input buffers (r^{k-1}, p^{k-1}) the next ghost
  // exchange fills.  Written by sweep k (= k + 1) and by init (= 0) for diagnostics; the exchange
  // kernels take their target from the host (round 4), so nothing on the device reads it.
  long long halo_k;
  long long halo_k_unpack;  // unused since round 4 (kept: checkpoint files hold PcgState)
  // Single-pass w schedule (pcg1): w is read and written on one sweep in w_cycle (2 = pairs, 3 =
  // triples, see k_pcg1).  alpha1/beta1 hold alpha_k / beta_k at slot k & 3; w_pend_n steps
  // (p^{w_pend - w_pend_n + 1} .. p^{w_pend}, both still in the two p buffers) are not yet in w.
  double alpha1[4];
  double beta1[4];
  int w_cycle;
  int w_pend_n;
};

// s-step PCG (ca_kernels.hip): the per-block scalars next to PcgState.  Basis of a block: Chebyshev
// polynomials of L = D^-1 A in p and z, Y = [P_0..P_s, Z_0..Z_{s-1}] (2s+1 vectors); p, z and w - w_k
// after j iterations are Y a_j, Y b_j, Y c_j.  The stop test of a block's iterations needs ||p_{k+j}||,
// which pass 2 forms explicitly: it is checked one reduction later ("pending"), and a stop inside the
// block rewinds w to c_{j+1} with one more pass over the block's (still intact) inputs.
constexpr int kCaMaxS = 3;
constexpr int kCaMaxNb = 2 * kCaMaxS + 1;
struct alignas(64) CaState {
  double coef[3][kCaMaxNb];     // pass 2: a_n, b_n, c_n (rewind: w += Y coef[2])
  double pa[kCaMaxS][kCaMaxNb];  // a_j (p_{k+j} = Y a_j) of the block's iterations: pass 2's norms
  double pc[kCaMaxS][kCaMaxNb];  // c_{j+1} of the pending block (the rewind target)
  double alpha[kCaMaxS];         // alpha_j of the pending block
  double red[7 * kCaMaxS];       // decomposed grids: this rank's Gram + norm sums, all-reduced before the finish
  long long blk;          // blocks applied: pass 1 reads (p, z) from set blk & 1, pass 2 writes set (blk & 1)
  long long pend_k;       // iterations done before the pending block
  long long after_iters;  // iteration count reported with after_status
  int nupd;               // pass 2: n > 0 apply n iterations, 0 nothing, -1 rewind w only
  int pend_n;             // iterations of the block whose stop test is pending (0: none)
  int after_status;       // 0, or the status (breakdown / max_iter) that ends the solve once the pending test passes
  int s;                  // block size (basis degree)
  unsigned ticket;        // the reduction's last-block ticket (re-armed by the finishing block)
  int pad;
};

// Pointers for the halo ("ghost") exchange, one per slot (see kHaloSlots).  Two-sweep iteration:
// slots 0-3 hold one line of r (ny values for x sides, nx for y sides).  Single-pass iteration:
// two lines of r and of p per side (4 ny / 4 nx values) and one (r, p) pair per corner.
template <typename T>
struct HaloBufs {
  T* send[kHaloSlots];
  T* recv[kHaloSlots];
};

}  // namespace pmx
