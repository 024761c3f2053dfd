#!/usr/bin/env bash
# A/B of library builds in build_ab/ (same box, sequential processes, alternating twice).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for lib in build_ab/*.so; do
    echo "### $lib (rep $rep)"
    VR_LIB=$PWD/$lib timeout -k 10 120 python tools/sweep.py --rounds 3 --configs "${CONFIGS:-c3,c3exact,c3obl,c3oblx,c2}" --variants "${VARIANTS:-batch=8;batch=16}" | grep median || exit $?
  done
done
