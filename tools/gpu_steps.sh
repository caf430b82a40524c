#!/bin/bash
# Run GPU steps one after another on the gpurun box; each step has its own time limit and its
# output under gpurun_out/.  A fault, abort, segfault or time limit ends the script at once.
#   tools/gpu_steps.sh "name:seconds:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - start )) s)"
  tail -n 5 "gpurun_out/$name.log"
  case $rc in
    124|134|137|139|143) echo "=== fatal exit $rc: stopping"; exit $rc ;;
  esac
done
exit 0
