#!/usr/bin/env bash
# PMC passes (one rocprofv3 run per counter group, never combined with tracing) over a command.
# usage: tools/pmc.sh <outdir> "<counters group 1>" "<group 2>" ... -- <command...>
out="$1"; shift
groups=()
while [ "$1" != "--" ]; do groups+=("$1"); shift; done
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p "$out"
i=0
for g in "${groups[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $g --output-format csv -d "$out/g$i" -o g$i -- "$@" > "$out/g$i.log" 2>&1 || exit $?
  i=$((i+1))
done
echo "pmc done: $out"
