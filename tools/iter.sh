#!/bin/bash
# One development iteration on the GPU box: named steps, each under its own time limit,
# logs under gpurun_out/iter/.  Stops at the first fatal exit (timeout / abort / crash).
# usage: tools/iter.sh 'name|timeout|command' ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
mkdir -p gpurun_out/iter
# heartbeat: a step that is silent for minutes (first torch import, synthetic data build) is not hung
( while sleep 50; do date +%T >> gpurun_out/iter/heartbeat.log; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/iter/$name.log" 2>&1
  rc=$?
  echo "step $name exit $rc" | tee -a gpurun_out/iter/steps.log
  case "$rc" in 124|137|134|139|143) echo "fatal exit in $name"; exit "$rc";; esac
done
exit 0
