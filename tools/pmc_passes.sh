#!/bin/bash
# PMC passes (one rocprofv3 run per pass, counters only + kernel trace) of one bench
# config, restricted to the kernels matching a regex.
# usage: tools/pmc_passes.sh <config> <tag> <kernel-regex> <pass>... [-- extra bench args]
#   each <pass> is a quoted, space-separated counter list (<= 8 SQ, <= 4 TCC per pass)
#   -> gpurun_out/<tag>/pmc<i>/run_counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
cfg=$1; tag=$2; re=$3; shift 3
passes=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do passes+=("$1"); shift; done
[ $# -gt 0 ] && shift
out=gpurun_out/$tag
mkdir -p "$out"
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $p --kernel-include-regex "$re" -d "$out/pmc$i" -o run --output-format csv -- \
    python3 bench.py --config "$cfg" --no-cpu-baseline --steps 1 --warmup 0 "$@" > "$out/pmc$i.log" 2>&1
  rc=$?
  echo "pass $i ($p) exit $rc" | tee -a "$out/steps.log"
  [ $rc -eq 0 ] || exit $rc
done
