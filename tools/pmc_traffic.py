#!/usr/bin/env python3
"""HBM traffic per march-kernel launch from PMC counters, for bench.py's roofline.traffic.

Runs bench.py twice under rocprofv3, one counter per pass (FETCH_SIZE, then WRITE_SIZE; the
guide: never combine --pmc with tracing, FETCH_SIZE and WRITE_SIZE do not fit one pass), averages
the counter over every dispatch of the march kernel and applies the gfx950 corrections of
MI355X_MICROARCH.md section HBM:
  * both counters are in KiB (x 1024);
  * FETCH_SIZE reports half the bytes of a wide coalesced read (128-B requests counted as 64 B),
    so it is doubled.  The march's reads are 1-byte gathers (a width the guide leaves
    uncalibrated), so the raw value is kept alongside.
Writes profiles/traffic_latest.json, or $TRAFFIC_OUT (read by bench.py when the workload key matches).

usage: python tools/pmc_traffic.py [bench args ...]   (on the GPU box)
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pass(counter, bench_args, outdir):
    d = os.path.join(outdir, counter)
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", counter, "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "1", "--cpu-baseline", "0",
           "--traffic-json", "/dev/null", "--extra", "0"] + bench_args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=dict(os.environ, TMPDIR="/tmp"))
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
        raise SystemExit(r.returncode)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    vals = []
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            if "march_kernel" in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} samples for the march kernel")
    return sum(vals) / len(vals), len(vals), json.loads(line)


def main():
    bench_args = sys.argv[1:]
    out = tempfile.mkdtemp(prefix="vr_pmc_", dir="/tmp")
    try:
        fetch_kib, nf, bl = run_pass("FETCH_SIZE", bench_args, out)
        write_kib, nw, _ = run_pass("WRITE_SIZE", bench_args, out)
    finally:
        shutil.rmtree(out, ignore_errors=True)
    cfg = bl["config"]
    flags = 0
    fl = [a for a in bench_args]
    # reconstruct the workload key bench.py uses
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", default="ess,ert")
    ap.add_argument("--mode", default="vrc")
    ap.add_argument("--volume", default="mni")
    a, _ = ap.parse_known_args(fl)
    for f in a.flags.split(","):
        flags |= {"ess": 1, "ert": 2, "shade": 8}.get(f.strip().lower(), 0)
    key = f"{a.volume}:{cfg['width']}x{cfg['height']}x{cfg['samples_per_ray']}:{a.mode}:{flags}:n{bl['n_gpus']}"
    fetch_b = fetch_kib * 1024.0
    write_b = write_kib * 1024.0
    res = {
        "workload_key": key,
        "kernel": bl["roofline"]["kernel"],
        "dispatches": {"FETCH_SIZE": nf, "WRITE_SIZE": nw},
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib_raw": write_kib,
        "hbm_read_bytes_corrected": 2.0 * fetch_b,
        "hbm_write_bytes": write_b,
        "hbm_bytes_per_launch": 2.0 * fetch_b + write_b,
        "hbm_bytes_per_launch_uncorrected": fetch_b + write_b,
        "algorithmic_bytes_per_launch": bl["roofline"]["algorithmic_bytes_per_launch"],
        "kernel_ms_mean_profiled": bl["roofline"]["kernel_ms_mean"],
        "note": "FETCH_SIZE x2 per MI355X_MICROARCH.md (128-B requests tallied at 64 B); the march's "
                "1-byte gathers are an uncalibrated width, raw values kept.",
    }
    dest = os.environ.get("TRAFFIC_OUT") or os.path.join(ROOT, "profiles", "traffic_latest.json")
    os.makedirs(os.path.dirname(dest), exist_ok=True)
    with open(dest, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
