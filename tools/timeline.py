"""Dispatch timeline of the march kernel from a rocprofv3 --kernel-trace CSV: for the dispatches
[first, first + n) of the march (e.g. bench.py's timed steps after its warm-up), each launch's start
and end relative to the first start, its duration and the idle gap before it, and the summed busy
time of the window.  usage: python tools/timeline.py <kernel_trace.csv> [first] [n]"""
import csv
import sys

MARCH = ("vrc_march_kernel", "test_march_kernel", "test_axis_kernel", "test_axz_kernel")


def main():
    path = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = [r for r in csv.DictReader(open(path)) if any(m in r["Kernel_Name"] for m in MARCH)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sel = rows[first:first + n]
    if not sel:
        raise SystemExit("no march dispatches in that range")
    t0 = int(sel[0]["Start_Timestamp"])
    prev_end = None
    busy_until = t0
    busy = 0
    for r in sel:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        gap = None if prev_end is None else s - prev_end
        print(f"start {s / 1e3:8.2f} us  end {e / 1e3:8.2f} us  dur {(e - s) / 1e3:7.2f} us  "
              f"gap {'' if gap is None else f'{gap / 1e3:7.2f}'}")
        # union of busy intervals
        s_abs, e_abs = s + t0, e + t0
        if e_abs > busy_until:
            busy += e_abs - max(s_abs, busy_until)
            busy_until = e_abs
        prev_end = e
    span = int(sel[-1]["End_Timestamp"]) - t0
    print(f"window {span / 1e3:.2f} us for {len(sel)} launches = {span / 1e3 / len(sel):.2f} us per launch; "
          f"device busy {busy / span:.1%} of it")


if __name__ == "__main__":
    main()
