#!/bin/bash
# Round 6, config-4 scoring kernel: MF k in {32, 64} parity tests with the in-tree library, then a
# same-box A/B of library builds on 20m-mf64 (tools/ab_quick.sh).  usage: tools/r6_m64.sh <tag> <lib>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "mf64 or config4 or MF-64 or MF-32 or 1-64 or 1-32 or every_built or 4-64 or 6-64 or 4-32 or 6-32" > "$out/tests.log" 2>&1
rc=$?; echo "tests exit $rc"; grep -E "passed|failed" "$out/tests.log" | tail -3; [ $rc -eq 0 ] || exit $rc
bash tools/ab_quick.sh 20m-mf64 "$@" -- --steps 10 --warmup 2 --spinup-seconds 5
