#!/bin/bash
# Round-end bench lines (with CPU baselines) of a set of configs -> gpurun_out/r2bench/<name>.log.
# usage: tools/round2_bench.sh small|m64|big
# Each run under its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2bench
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
run() {  # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python bench.py "$@" > "gpurun_out/r2bench/$name.log" 2>&1
  local rc=$?
  echo "step $name exit $rc" | tee -a gpurun_out/r2bench/steps.log
  [ $rc -eq 0 ] || exit $rc
}
case "$1" in
  small)
    run ml1m 600
    run yelp 600 --config yelp-ncf --cpu-baseline-seconds 15 ;;
  m64)
    run m64 900 --config 20m-mf64 --steps 5 --warmup 1 --cpu-baseline-seconds 20 ;;
  big)
    run mf256 600 --config 20m-mf256 --shard-of 8 --steps 3 --warmup 1 --cpu-baseline-seconds 20
    run ncf256 600 --config 20m-ncf256 --shard-of 8 --steps 3 --warmup 1 --cpu-baseline-seconds 20 ;;
esac
