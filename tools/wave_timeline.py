"""Analyse VR_STATS_DUMP records.  Layout (u64): per wave 6 words [t_entry, after the staging
barrier, after the table barrier, t_start (prologue done), t_end, xcc] for nw waves, then per lane 2 words [iters | loads << 32, jumps | 1 << 63];
times from s_memrealtime (100 MHz).  Waves that never reached the end (culled tiles) have t_end 0."""
import sys

import numpy as np

d = np.fromfile(sys.argv[1], dtype=np.uint64)
nw = len(d) // (6 + 128)
wv = d[:6 * nw].reshape(nw, 6).astype(np.int64)
ln = d[6 * nw:].reshape(nw, 64, 2)
valid = (ln[:, :, 1] >> np.uint64(63)).astype(bool)
loads = (ln[:, :, 0] >> np.uint64(32)).astype(np.int64) * valid
t_in, tb1, tb2, t0, t1, xcc = (wv[:, k] for k in range(6))
ok = t1 > 0
t_in, tb1, tb2, t0, t1, xcc, loads, valid = (a[ok] for a in (t_in, tb1, tb2, t0, t1, xcc, loads, valid))
base = t_in.min()
t_in, tb1, tb2, t0, t1 = t_in - base, tb1 - base, tb2 - base, t0 - base, t1 - base
span = t1.max()
wmax = loads.max(axis=1)
busy = wmax > 0
print(f"waves {len(t1)}  span {span} ticks = {span / 100:.1f} us  (s_memrealtime, 100 MHz)")
pro, mar = t0 - t_in, t1 - t0
for name, m in [("marching", busy), ("no samples", ~busy)]:
    if m.sum():
        q = lambda a: (np.percentile(a[m], [10, 50, 90, 99, 100]) / 100).round(2)  # noqa: E731
        print(f"{name:10s} n={m.sum():6d} prologue us p10/50/90/99/max {q(pro)}  march us {q(mar)}")
        print(f"{'':10s}   staging+init (to barrier 1) {q(tb1 - t_in)}  table (to barrier 2) {q(tb2 - tb1)}  "
              f"entry search {q(t0 - tb2)}")
eff = loads[busy].sum() / max(1, (wmax[busy][:, None] * valid[busy]).sum())
print(f"lane efficiency of the sample loads (sum / wave max x lanes): {eff:.2f}")
iters = (ln[:, :, 0] & np.uint64(0xffffffff)).astype(np.int64)[ok] * valid
imax = iters.max(axis=1)
ieff = iters[busy].sum() / max(1, (imax[busy][:, None] * valid[busy]).sum())
# batches a wave runs while some of its lanes are finished: what refilling finished lanes could recover
print(f"lane efficiency of the batches (sum / wave max x lanes): {ieff:.2f}  "
      f"(batches per marching wave p50/90/max {np.percentile(imax[busy], [50, 90, 100]).round(0)})")
bins = np.linspace(0, span, 21)
for i in range(20):
    a, b = bins[i], bins[i + 1]
    live = ((t_in < b) & (t1 > a)).sum()
    started = ((t_in >= a) & (t_in < b)).sum()
    print(f"  t {a / 100:6.1f}-{b / 100:6.1f} us: live waves {live:6d} started {started:6d}")
for x in np.unique(xcc):
    m = xcc == x
    print(f"xcc {x}: waves {m.sum()} last end {t1[m].max() / 100:.1f} us")
