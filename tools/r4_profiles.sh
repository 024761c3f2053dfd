#!/usr/bin/env bash
# Round-4 profiles on the GPU box: for each workload, tools/round_profile.sh (PMC passes -> traffic.json,
# rocprofv3 kernel trace + stats, the bench line with that traffic).  Which workloads: $WL (default
# all), names below.  Stops at the first failing step.  Results: gpurun_out/prof_<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
run() { tag=$1; shift; if [[ ",${WL:-all}," == *",all,"* || ",${WL}," == *",$tag,"* ]]; then
  timeout -k 10 1000 bash tools/round_profile.sh "$tag" --steps 20 --warmup 5 "$@"; fi; }
run r4_c3                                                    # the headline (C3 ESS + ERT, default camera)
run r4_c3obl   --camera oblique
run r4_c3test  --mode test
run r4_c3testo --mode test --camera oblique
run r4_c5exact --volume c5 --width 3840 --height 2160 --samples 4096 --flags exact
run r4_c5exact8 --volume c5 --width 3840 --height 2160 --samples 4096 --flags exact --options class_bits=8
run r4_c5exact_rw1 --volume c5 --width 3840 --height 2160 --samples 4096 --flags exact --options run_words=1
run r4_c5      --volume c5 --width 3840 --height 2160 --samples 4096
