#!/usr/bin/env bash
# Measurement of one workload on the GPU box: PMC passes (HBM traffic + SQ stall split,
# tools/pmc_traffic.py), a rocprofv3 kernel-trace --stats run and the bench line with that traffic
# attached.  Every step has its own time limit; the script stops at the first failure.
# Output: gpurun_out/prof_<tag>/ (traffic.json, pmc.csv, kt/..._kernel_stats.csv, bench.json).
# usage: tools/round_profile.sh <tag> [bench args ...]
set -e
tag="$1"; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out="gpurun_out/prof_$tag"
mkdir -p "$out"
step() { echo "[$(date +%T)] $tag: $*"; }
step "PMC passes"
TRAFFIC_OUT="$PWD/$out/traffic.json" PMC_CSV="$PWD/$out/pmc.csv" timeout -k 10 900 python3 tools/pmc_traffic.py "$@" \
    > "$out/pmc.log" 2>&1
step "kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- \
    python3 bench.py "$@" --cpu-baseline 0 --extra 0 --traffic-json "$out/traffic.json" \
    > "$out/kt_bench.json" 2> "$out/kt_bench.err"
step "bench"
timeout -k 10 600 python3 bench.py "$@" --cpu-baseline 0 --traffic-json "$out/traffic.json" \
    > "$out/bench.json" 2> "$out/bench.err"
step "done"
