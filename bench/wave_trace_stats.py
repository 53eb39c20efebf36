"""Summarise a k_pcg1 wave trace (bench/bin/pmx_wtrace, PMX_WAVE_TRACE_OUT): how the wave
population ramps up, holds and drains during one sweep, per XCC.

usage: python bench/wave_trace_stats.py trace.txt [--slots N]
Lines: start end xcc hw_id tile part [prologue_end] (100-MHz wall-clock ticks, 10 ns).
"""
from __future__ import annotations

import statistics
import sys

import numpy as np


def main():
    path = sys.argv[1]
    a = np.loadtxt(path, dtype=np.int64, ndmin=2)
    st, en, xcc = a[:, 0], a[:, 1], a[:, 2]
    t0 = st.min()
    st_us, en_us = (st - t0) / 100.0, (en - t0) / 100.0
    span = en_us.max()
    dur = en_us - st_us
    n = len(st)
    print(f"{path}: {n} waves, sweep span {span:.1f} us (first start -> last end)")
    print(f"wave duration: median {np.median(dur):.1f} us, p10 {np.percentile(dur, 10):.1f}, "
          f"p90 {np.percentile(dur, 90):.1f}, max {dur.max():.1f}")
    if a.shape[1] > 6:  # prologue: kernel entry -> tile decoded, before the first row loads
        pro = (a[:, 6] - st) / 100.0
        print(f"prologue: median {np.median(pro):.2f} us, p90 {np.percentile(pro, 90):.2f} "
              f"({np.median(pro) / np.median(dur):.1%} of the median wave)")
    # resident waves over time (1-us bins)
    nb = int(np.ceil(span)) + 1
    occ = np.zeros(nb + 1)
    np.add.at(occ, np.floor(st_us).astype(int), 1)
    np.add.at(occ, np.floor(en_us).astype(int), -1)
    occ = np.cumsum(occ)[:nb]
    peak = occ.max()
    slots = int(sys.argv[sys.argv.index("--slots") + 1]) if "--slots" in sys.argv else int(peak)
    full = occ >= 0.9 * slots
    first_full = int(np.argmax(full)) if full.any() else nb
    last_full = nb - 1 - int(np.argmax(full[::-1])) if full.any() else 0
    print(f"resident waves: peak {peak:.0f}, mean {occ.mean():.0f} ({occ.mean() / slots:.1%} of {slots} slots)")
    print(f"ramp: {first_full} us to reach 90% of the slots; drain: {span - last_full:.1f} us below 90% at the end")
    lost = np.sum(np.maximum(0, slots - occ)) / slots
    print(f"slot-time lost below full occupancy: {lost:.1f} us-equivalents ({lost / span:.1%} of the span)")
    print("occupancy by tenth of the span:", " ".join(f"{occ[int(i * nb / 10):int((i + 1) * nb / 10)].mean() / slots:.2f}"
                                                  for i in range(10)))
    # duration by start-time decile
    order = np.argsort(st_us)
    dec = np.array_split(order, 10)
    print("median wave duration by start decile (us):", " ".join(f"{np.median(dur[d]):.1f}" for d in dec))
    print("per XCC: waves, first start, last end (us), median duration")
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        print(f"  xcc {x}: {m.sum():6d}  {st_us[m].min():7.1f}  {en_us[m].max():7.1f}  {statistics.median(dur[m].tolist()):6.1f}")


if __name__ == "__main__":
    main()
