#!/usr/bin/env bash
# Runs a list of GPU steps on the gpurun box; each step has its own time limit.  A step that
# ends with 0 (ok) or 1 (test failures) lets the next one run; anything else (fault, abort,
# segfault, timeout) stops the session immediately.
# usage: tools/gpu_session.sh "<seconds>|<name>|<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] ($secs s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start )) s" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping session after [$name] rc=$rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
exit 0
