#!/usr/bin/env bash
# Profiles bench.py's C3 workload: kernel-trace stats, then separate PMC passes (never combined
# with tracing domains).  Output under gpurun_out/prof_<tag>/.  usage: tools/profile_round.sh <tag> [bench args]
tag="$1"; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out="gpurun_out/prof_$tag"
mkdir -p "$out"
B="bench.py --steps 20 --warmup 3 --cpu-baseline 0 $*"
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- python3 $B > "$out/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o fetch -- python3 $B > "$out/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o write -- python3 $B > "$out/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/tcc" -o tcc -- python3 $B > "$out/tcc.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv -d "$out/sq" -o sq -- python3 $B > "$out/sq.log" 2>&1
echo "profile $tag done"
find "$out" -name "*.csv" | head -50
