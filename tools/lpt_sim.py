"""What-if for the dispatch order, from a VR_STATS_DUMP wave timeline: replay the recorded workgroup
durations through list scheduling on the chip's resident slots, in the recorded order, longest
first (LPT) and random.  Durations were measured under the recorded concurrency, so this bounds what
a better order could buy rather than predicting it.

usage: python tools/lpt_sim.py gpurun_out/waves.bin [slots]
"""
import heapq
import sys

import numpy as np


def makespan(durations, slots):
    h = [0.0] * slots
    heapq.heapify(h)
    mk = 0.0
    for d in durations:
        t = heapq.heappop(h) + d
        mk = max(mk, t)
        heapq.heappush(h, t)
    return mk


def main():
    d = np.fromfile(sys.argv[1], dtype=np.uint64)
    slots = int(sys.argv[2]) if len(sys.argv) > 2 else 256 * 7
    nw = len(d) // (6 + 128)
    wv = d[:6 * nw].reshape(nw, 6).astype(np.int64)
    nb = nw // 4
    tin, te = wv[:nb * 4, 0].reshape(nb, 4), wv[:nb * 4, 4].reshape(nb, 4)
    ok = (te > 0).all(axis=1)
    start, end = tin.min(axis=1)[ok], te.max(axis=1)[ok]
    durs = (end - start) / 100.0
    print(f"workgroups recorded {ok.sum()} of {nb}; recorded span {(end.max() - start.min()) / 100:.1f} us")
    print(f"durations us p50 {np.percentile(durs, 50):.1f} p90 {np.percentile(durs, 90):.1f} max {durs.max():.1f}; "
          f"sum / slots {durs.sum() / slots:.1f}")
    print(f"replayed makespan us: recorded order {makespan(durs, slots):.1f}, "
          f"longest first {makespan(np.sort(durs)[::-1], slots):.1f}, "
          f"random {makespan(np.random.default_rng(0).permutation(durs), slots):.1f}")


if __name__ == "__main__":
    main()
