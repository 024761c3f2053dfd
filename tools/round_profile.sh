#!/usr/bin/env bash
# End-of-milestone measurement on the GPU box: PMC HBM traffic, rocprofv3 kernel-trace stats and
# the bench lines for C3 (the headline workload) and C5 (the HBM-roofline run).  Every step has its
# own time limit; the script stops at the first failure.  Output: gpurun_out/round_<tag>/.
# usage: tools/round_profile.sh <tag> [c5]
set -e
tag="$1"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out="gpurun_out/round_$tag"
mkdir -p "$out"
step() { echo "[$(date +%T)] $*"; }
step "C3 PMC traffic"
TRAFFIC_OUT="$PWD/profiles/traffic_latest.json" timeout -k 10 600 python3 tools/pmc_traffic.py > "$out/traffic_c3.log" 2>&1
cp profiles/traffic_latest.json "$out/traffic_c3.json"
step "C3 kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- \
    python3 bench.py --steps 50 --warmup 5 --cpu-baseline 0 --extra 0 > "$out/kt_bench.json" 2> "$out/kt_bench.err"
step "C3 bench"
timeout -k 10 400 python3 bench.py > "$out/bench_c3.json" 2> "$out/bench_c3.err"
if [ "$2" = "c5" ]; then
  C5="--volume c5 --width 3840 --height 2160 --samples 4096"
  step "C5 PMC traffic"
  TRAFFIC_OUT="$PWD/$out/traffic_c5.json" timeout -k 10 900 python3 tools/pmc_traffic.py $C5 > "$out/traffic_c5.log" 2>&1
  step "C5 kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt_c5" -o kt -- \
      python3 bench.py $C5 --steps 10 --warmup 2 --cpu-baseline 0 --extra 0 > "$out/kt_c5.json" 2> "$out/kt_c5.err"
  step "C5 bench"
  timeout -k 10 600 python3 bench.py $C5 --steps 10 --warmup 2 --traffic-json "$out/traffic_c5.json" \
      > "$out/bench_c5.json" 2> "$out/bench_c5.err"
fi
step "done"
