#!/usr/bin/env python3
"""HBM traffic and SQ stall split per march-kernel launch from PMC counters (bench.py's roofline).

Runs bench.py under rocprofv3 once per counter group (the guide: never combine --pmc with tracing;
FETCH_SIZE and WRITE_SIZE do not fit one pass):
  pass 1  FETCH_SIZE
  pass 2  WRITE_SIZE
  pass 3  SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
          SQ_INSTS_VMEM_RD SQ_INSTS_LDS                                   (8 SQ counters, one pass)
  pass 4  TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr
          TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE  (L1 / L2 hit rates, texture-address busy;
          optional: a failure leaves "cache": null)
averages each counter over every dispatch of the march kernel and applies the gfx950 corrections of
MI355X_MICROARCH.md section HBM:
  * FETCH_SIZE / WRITE_SIZE are in KiB (x 1024);
  * FETCH_SIZE reports half the bytes of a wide coalesced read (128-B requests counted as 64 B), so
    it is doubled.  The march's reads are 1-byte gathers (a width the guide leaves uncalibrated),
    so the raw value is kept alongside.
  * SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (ready, issue-stalled) +
    SQ_ACTIVE_INST_ANY (issuing) ~= SQ_WAVE_CYCLES; the split is reported as fractions.
Writes $TRAFFIC_OUT (default profiles/traffic_latest.json; bench.py attaches it when the workload
key matches) and, with $PMC_CSV, the per-dispatch counter rows of the march kernel as CSV.

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
sys.path.insert(0, ROOT)
CACHE = ["TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "TCC_HIT_sum", "TCC_MISS_sum", "TA_BUSY_avr",
         "TA_BUFFER_READ_WAVEFRONTS_sum", "GRBM_GUI_ACTIVE"]
# the per-frame march kernels (VRC, TEST generic, TEST z-axis plane march)
MARCH_KERNELS = ("vrc_march_kernel", "test_march_kernel", "test_axis_kernel", "test_axz_kernel")
SQ = ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_SALU",
      "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS"]


def is_march(name):
    """A timed march launch: not the counting instantiation of vr_count_work (STATS = 2, the last
    template argument of every march kernel), which bench.py runs once after the timed region."""
    return any(k in name for k in MARCH_KERNELS) and ", 2>(" not in name


def run_pass(counters, bench_args, outdir, tag, rows, timeout=600):
    d = os.path.join(outdir, tag)
    cmd = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", tag, "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "1", "--cpu-baseline", "0",
           "--traffic-json", "/dev/null", "--extra", "0"] + bench_args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=dict(os.environ, TMPDIR="/tmp"))
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
        raise SystemExit(r.returncode)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    vals = {c: [] for c in counters}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            if is_march(row["Kernel_Name"]) and row["Counter_Name"] in vals:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
                rows.append({"pass": tag, "kernel": row["Kernel_Name"][:80], "dispatch": row.get("Dispatch_Id", ""),
                             "counter": row["Counter_Name"], "value": row["Counter_Value"]})
    for c, v in vals.items():
        if not v:
            raise SystemExit(f"no {c} samples for the march kernel")
    return {c: sum(v) / len(v) for c, v in vals.items()}, {c: len(v) for c, v in vals.items()}, json.loads(line)


def main():
    bench_args = sys.argv[1:]
    out = tempfile.mkdtemp(prefix="vr_pmc_", dir="/tmp")
    rows = []
    try:
        f, nf, bl = run_pass(["FETCH_SIZE"], bench_args, out, "fetch", rows)
        w, nw, _ = run_pass(["WRITE_SIZE"], bench_args, out, "write", rows)
        sq, nsq, _ = run_pass(SQ, bench_args, out, "sq", rows)
        try:
            cache, _, _ = run_pass(CACHE, bench_args, out, "cache", rows, timeout=120)
        except (SystemExit, subprocess.TimeoutExpired) as e:
            sys.stderr.write(f"cache pass skipped: {e}\n")
            cache = None
    finally:
        shutil.rmtree(out, ignore_errors=True)
    import argparse
    import bench
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", default="ess,ert")
    ap.add_argument("--mode", default="vrc")
    ap.add_argument("--volume", default="mni")
    ap.add_argument("--camera", default="default")
    a, _ = ap.parse_known_args(bench_args)
    flags = 0
    for fl in a.flags.split(","):
        flags |= {"ess": 1, "ert": 2, "shade": 8}.get(fl.strip().lower(), 0)
    cfg = bl["config"]
    key = bench.workload_key(a.volume, cfg["width"], cfg["height"], cfg["samples_per_ray"], a.mode, flags,
                             bl["n_gpus"], a.camera)
    fetch_b = f["FETCH_SIZE"] * 1024.0
    write_b = w["WRITE_SIZE"] * 1024.0
    wc = sq["SQ_WAVE_CYCLES"]
    ms = bl["roofline"]["kernel_ms_mean"]
    hbm = 2.0 * fetch_b + write_b
    res = {
        "workload_key": key,
        "workload": cfg["workload"],
        "kernel": bl["roofline"]["kernel"],
        "dispatches": {"FETCH_SIZE": nf["FETCH_SIZE"], "WRITE_SIZE": nw["WRITE_SIZE"], "SQ": nsq["SQ_WAVE_CYCLES"]},
        "fetch_size_kib_raw": f["FETCH_SIZE"],
        "write_size_kib_raw": w["WRITE_SIZE"],
        "hbm_read_bytes_corrected": 2.0 * fetch_b,
        "hbm_write_bytes": write_b,
        "hbm_bytes_per_launch": hbm,
        "hbm_bytes_per_launch_uncorrected": fetch_b + write_b,
        "kernel_ms_mean_under_pmc": ms,
        "model_bytes_per_launch": bl["roofline"].get("model_bytes_per_launch"),
        "sq": sq,
        "sq_split": {"wait_any (s_waitcnt/barrier)": sq["SQ_WAIT_ANY"] / wc,
                     "wait_inst_any (ready, not issued)": sq["SQ_WAIT_INST_ANY"] / wc,
                     "active_inst_any (issuing)": sq["SQ_ACTIVE_INST_ANY"] / wc},
        "cache": None if cache is None else {
            **cache,
            "l1_hit_rate": 1.0 - cache["TCP_TCC_READ_REQ_sum"] / max(1.0, cache["TCP_TOTAL_CACHE_ACCESSES_sum"]),
            "l2_hit_rate": cache["TCC_HIT_sum"] / max(1.0, cache["TCC_HIT_sum"] + cache["TCC_MISS_sum"]),
            "ta_busy_frac": cache["TA_BUSY_avr"] / max(1.0, cache["GRBM_GUI_ACTIVE"]),
        },
        "note": "FETCH_SIZE x2 per MI355X_MICROARCH.md (128-B requests tallied at 64 B); the march's "
                "1-byte gathers are an uncalibrated width, raw values kept.  Counter passes serialise the "
                "dispatches, so kernel_ms_mean_under_pmc is not a duration to divide by: bench.py divides "
                "hbm_bytes_per_launch by its own live HIP-event time.  SQ cycles are quad-cycles "
                "summed over waves; the split is their ratio to SQ_WAVE_CYCLES.",
    }
    dest = os.environ.get("TRAFFIC_OUT") or os.path.join(ROOT, "profiles", "traffic_latest.json")
    os.makedirs(os.path.dirname(dest), exist_ok=True)
    with open(dest, "w") as fh:
        json.dump(res, fh, indent=1)
    if os.environ.get("PMC_CSV"):
        with open(os.environ["PMC_CSV"], "w", newline="") as fh:
            wr = csv.DictWriter(fh, fieldnames=["pass", "kernel", "dispatch", "counter", "value"])
            wr.writeheader()
            wr.writerows(rows)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
