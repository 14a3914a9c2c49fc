#!/bin/bash
# PMC passes (one rocprofv3 run each, counters + kernel trace only) over a short bench run.
# usage: tools/pmc2.sh <kernel-regex> <tag> "<bench args>" "<pass counters>"...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
re=$1; tag=$2; bargs=$3; shift 3
mkdir -p gpurun_out/pmc2
i=0
for p in "$@"; do
  i=$((i+1))
  timeout -k 10 100 rocprofv3 --pmc $p --kernel-include-regex "$re" -d "gpurun_out/pmc2/${tag}_$i" -o run \
      --output-format csv -- python3 bench.py --no-cpu-baseline $bargs > "gpurun_out/pmc2/${tag}_$i.log" 2>&1
  rc=$?
  echo "pmc pass $i ($p) exit $rc"
  [ $rc -eq 0 ] || exit $rc
done
