"""Where the fused s-step march waits: run a build of the package made with
PMX_EXTRA_HIP_FLAGS=-DPMX_CAF_TIMING (k_ca_fused prints, for block 7 and every 499th tile, the
s_memtime ticks each wave spent in total and inside the producer / consumer row barriers) and
summarise the lines per role.

  python bench/probe/caf_timing.py bench/ab/pmx_timing [--n 16384] [--m 0]
"""
import argparse
import importlib.util
import os
import re
import statistics
import subprocess
import sys

CHILD = r"""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(sys.argv[1]))
pkg = importlib.import_module(os.path.basename(sys.argv[1]))
s = pkg.make_session(pkg.PoissonEllipse(M=int(sys.argv[2]), N=int(sys.argv[3])), algo="ca", graph_batch=0)
s.init()
s.step(30)
s.synchronize()
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pkgdir")
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--m", type=int, default=0)
    a = ap.parse_args()
    env = dict(os.environ, PMX_STUDY="1")
    p = subprocess.run([sys.executable, "-c", CHILD, os.path.abspath(a.pkgdir), str(a.m or a.n), str(a.n)],
                       capture_output=True, text=True, timeout=300, env=env)
    print(p.stderr[-2000:], file=sys.stderr)
    pat = re.compile(r"caf part (\d) role (\d) tile (\d+) fast (\d) total (\d+) sync (\d+)")
    rows = [tuple(int(x) for x in m.groups()) for m in pat.finditer(p.stdout)]
    print(f"{len(rows)} timing lines")
    for part in (0, 1, 2):
        for role in (0, 1):
            sel = [r for r in rows if r[0] == part and r[1] == role]
            if not sel:
                continue
            tot = [r[4] for r in sel]
            syn = [r[5] for r in sel]
            frac = [s / t for s, t in zip(syn, tot) if t]
            print(f"part {part} role {role} ({'producer' if role == 0 else 'consumer'}): n={len(sel)} "
                  f"total median {statistics.median(tot):.0f} ticks, in barriers median {statistics.median(syn):.0f} "
                  f"({100 * statistics.median(frac):.1f}%)")
    return p.returncode


if __name__ == "__main__":
    sys.exit(main())
