#!/bin/bash
# Round-6 GPU check: the full -m gpu suite (durations), then the default headline bench line.
# Every step under its own time limit; the first failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
out=gpurun_out/${TAG:-r6}
mkdir -p "$out"
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1
  local rc=$?
  echo "step $n exit $rc" | tee -a "$out/steps.log"
  [ $rc -eq 0 ] || exit $rc
}
step tests ${TEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=60 ${TESTS:-}
step bench_ml1m 300 python bench.py
tail -1 "$out/bench_ml1m.log"
