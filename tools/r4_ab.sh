#!/usr/bin/env bash
# Round-4 A/B session on the GPU box: compact class volumes (class_bits 8 vs auto) and the round-3
# library (build_ab/base.so, built from the round-3 tree) on the same configs, in one call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFG="${CFG:-c3obl,c3oblx,c3obls,c3,c3exact,c2,c3s1,t3e,t3eo,t3x,t3xo}"
exec bash tools/gpu_session.sh \
  "300|sweep_cb|python -u tools/sweep.py --rounds 5 --variants \"class_bits=8;class_bits=0;run_words=2\" --configs $CFG" \
  "300|sweep_base|VR_LIB=$PWD/build_ab/base.so python -u tools/sweep.py --rounds 5 --configs $CFG"
