"""s-step (communication-avoiding) Jacobi-PCG prototype in plain PyTorch fp64: does it reproduce the
classic loop's iteration counts?

Classic PCG (models/torch_pcg.py) streams r, p (and w) once per iteration.  The s-step form runs s
iterations per two passes over the fields:

  pass 1  build the Chebyshev basis Y = [P_0..P_s, Z_0..Z_{s-1}] of p_k and z_k = D^-1 r_k
          (P_{i+1} = 2 L~ P_i - P_{i-1}, L~ = D^-1 A - I, spectrum in (-1, 1)) and the two Gram
          matrices G_D = Y^T D Y, G_0 = Y^T Y (one reduction)
  scalars the s iterations run on coordinate vectors: p_{k+j} = Y a_j, z_{k+j} = Y b_j,
          w_{k+j} - w_k = Y c_j; (r, z) = b^T G_D b, (p, Ap) = a^T G_D T a, ||p||^2 = a^T G_0 a
  pass 2  p, z, w <- Y a_s, Y b_s, w + Y c_s  (or c_{j+1} at the stop)

Usage: python bench/probe/ca_pcg_proto.py M N [--device cuda] [--no-classic] [s ...]
"""
from __future__ import annotations

import argparse
import importlib
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
R = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.ops.reference")


def setup(M, N, dev):
    P = pkg.PoissonEllipse(M=M, N=N)
    sd = dict(i_start=1, i_end=M - 1, j_start=1, j_end=N - 1)
    a, b, B = (t.to(dev) for t in R.assemble(P, sd))
    h1, h2 = P.h1, P.h2
    aE, aW = a[2:, 1:-1] / (h1 * h1), a[1:-1, 1:-1] / (h1 * h1)
    bN, bS = b[1:-1, 2:] / (h2 * h2), b[1:-1, 1:-1] / (h2 * h2)
    D = aE + aW + bN + bS
    del a, b

    def A(u):
        g = torch.nn.functional.pad(u, (1, 1, 1, 1))
        return D * u - aE * g[2:, 1:-1] - aW * g[:-2, 1:-1] - bN * g[1:-1, 2:] - bS * g[1:-1, :-2]
    return P, A, B[1:-1, 1:-1].contiguous(), D


def dot(x, y):
    return float((x * y).sum())


def classic(P, A, B, D):
    h = P.h1 * P.h2
    w = torch.zeros_like(B)
    r = B.clone()
    z = r / D
    p = z.clone()
    zr = dot(z, r) * h
    for k in range(1, P.effective_max_iter() + 1):
        Ap = A(p)
        alpha = zr / (dot(Ap, p) * h)
        w += alpha * p
        r -= alpha * Ap
        z = r / D
        zr_new = dot(z, r) * h
        if abs(alpha) * math.sqrt(dot(p, p) * h) < P.delta:
            return k, w
        p = z + (zr_new / zr) * p
        zr = zr_new
    return -1, w


def cheb(L, v, n):
    """v, L~v, ... (n vectors): Q_0 = v, Q_1 = L~ v, Q_{i+1} = 2 L~ Q_i - Q_{i-1}."""
    Q = [v]
    if n > 1:
        Q.append(L(v) - v)
    while len(Q) < n:
        Q.append(2.0 * (L(Q[-1]) - Q[-1]) - Q[-2])
    return Q


def shift_matrix(s):
    """T with L Y = Y T on the columns that stay in the basis (Chebyshev recurrence:
    L Q_0 = Q_0 + Q_1, L Q_i = Q_i + Q_{i+1}/2 + Q_{i-1}/2)."""
    n = 2 * s + 1
    T = [[0.0] * n for _ in range(n)]
    for base, m in ((0, s + 1), (s + 1, s)):
        for i in range(m - 1):
            T[base + i][base + i] = 1.0
            T[base + i + 1][base + i] = 1.0 if i == 0 else 0.5
            if i >= 1:
                T[base + i - 1][base + i] = 0.5
    return torch.tensor(T, dtype=torch.float64)


def sstep(P, A, B, D, s):
    h = P.h1 * P.h2
    L = lambda u: A(u) / D  # noqa: E731
    w = torch.zeros_like(B)
    z = B / D
    p = z.clone()
    T = shift_matrix(s)
    n = 2 * s + 1
    k = 0
    maxit = P.effective_max_iter()
    t0 = time.time()
    while k < maxit:
        if k % 600 < s:
            print(f"  s={s} k={k} ({time.time() - t0:.0f} s)", flush=True)
        Y = cheb(L, p, s + 1) + cheb(L, z, s)
        GD = torch.empty(n, n, dtype=torch.float64)
        G0 = torch.empty(n, n, dtype=torch.float64)
        DY = [D * y for y in Y]
        for i in range(n):
            for j in range(i, n):
                GD[i, j] = GD[j, i] = dot(Y[i], DY[j])
                G0[i, j] = G0[j, i] = dot(Y[i], Y[j])
        del DY
        a = torch.zeros(n, dtype=torch.float64); a[0] = 1.0
        b = torch.zeros(n, dtype=torch.float64); b[s + 1] = 1.0
        c = torch.zeros(n, dtype=torch.float64)
        g = float(b @ GD @ b)
        stop = False
        for j in range(s):
            k += 1
            Ta = T @ a
            alpha = g / float(a @ GD @ Ta)
            c = c + alpha * a
            diff = abs(alpha) * math.sqrt(max(float(a @ G0 @ a), 0.0) * h)
            if diff < P.delta or k >= maxit:
                stop = True
                break
            b = b - alpha * Ta
            g_new = float(b @ GD @ b)
            a = b + (g_new / g) * a
            g = g_new
        for i in range(n):
            w += float(c[i]) * Y[i]
        if stop:
            return k, w
        p = sum(float(a[i]) * Y[i] for i in range(n))
        z = sum(float(b[i]) * Y[i] for i in range(n))
        del Y
    return -1, w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("M", type=int)
    ap.add_argument("N", type=int)
    ap.add_argument("s", type=int, nargs="*", default=[2, 3, 4])
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--no-classic", action="store_true")
    args = ap.parse_args()
    M, N = args.M, args.N
    P, A, B, D = setup(M, N, args.device)
    wc = None
    if not args.no_classic:
        t = time.time()
        kc, wc = classic(P, A, B, D)
        print(f"{M}x{N} classic: {kc} iterations ({time.time() - t:.1f} s)", flush=True)
    for s in args.s:
        t = time.time()
        ks, ws = sstep(P, A, B, D, s)
        msg = f"{M}x{N} s={s}: {ks} iterations"
        if wc is not None:
            msg += f", max|w_s - w_c|/max|w_c| = {float((ws - wc).abs().max() / wc.abs().max()):.2e}"
        print(msg + f" ({time.time() - t:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
