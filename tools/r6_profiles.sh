#!/usr/bin/env bash
# Round-6 profiles on the GPU box: for each workload, tools/round_profile.sh (PMC passes -> traffic.json,
# rocprofv3 kernel trace + stats, the bench line with that traffic).  Which workloads: $WL (default
# all), names below.  Stops at the first failing step.  Results: gpurun_out/prof_<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
run() { tag=$1; shift; if [[ ",${WL:-all}," == *",all,"* || ",${WL}," == *",$tag,"* ]]; then
  timeout -k 10 1000 bash tools/round_profile.sh "$tag" --steps 20 --warmup 5 "$@"; fi; }
run r6_c3                                                    # the headline (C3 ESS + ERT, default camera)
run r6_c3obl   --camera oblique --extra-configs ''
run r6_c3s1    --samples 1 --extra-configs ''               # the fixed per-frame cost
run r6_c3test  --mode test --extra-configs ''
run r6_c3testo --mode test --camera oblique --extra-configs ''
run r6_c4      --volume r512 --samples 1024 --extra-configs ''   # BASELINE configs[3] on one GPU
run r6_c5      --volume c5 --width 3840 --height 2160 --samples 4096 --extra-configs ''
