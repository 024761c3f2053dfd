"""Analyse VR_STATS_DUMP per-wave records: [u32 max_iters, u32 max_loads][t_start][t_end][xcc]."""
import sys

import numpy as np

d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4)
it = (d[:, 0] & 0xFFFFFFFF).astype(np.int64)
ld = (d[:, 0] >> 32).astype(np.int64)
t0, t1, xcc = d[:, 1].astype(np.int64), d[:, 2].astype(np.int64), d[:, 3].astype(np.int64)
ok = t1 > 0
t0, t1, it, ld, xcc = t0[ok], t1[ok], it[ok], ld[ok], xcc[ok]
base = t0.min()
t0 -= base
t1 -= base
dur = t1 - t0
busy = it > 0
print(f"waves {len(t0)}  busy {busy.sum()}  span {t1.max()} ticks")
for name, m in [("busy", busy), ("idle", ~busy)]:
    if m.sum():
        q = np.percentile(dur[m], [10, 50, 90, 99, 100])
        print(f"{name:5s} duration ticks p10/50/90/99/max {q.astype(int)}  mean iters {it[m].mean():.1f} loads {ld[m].mean():.1f}")
# concurrency over time
T = t1.max()
bins = np.linspace(0, T, 21)
for i in range(20):
    a, b = bins[i], bins[i + 1]
    live = ((t0 < b) & (t1 > a)).sum()
    lb = ((t0 < b) & (t1 > a) & busy).sum()
    started = ((t0 >= a) & (t0 < b)).sum()
    print(f"  t {int(a):>8d}-{int(b):>8d}: live {live:6d} (busy {lb:6d}) started {started:6d}")
for x in range(8):
    m = xcc == x
    if m.sum():
        print(f"xcc {x}: waves {m.sum()} busy {(m & busy).sum()} last end {t1[m].max()} sum iters {it[m].sum()}")
