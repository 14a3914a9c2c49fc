#!/bin/bash
# Same-box A/B of library builds, bench phase times only (no profiler): one bench run per
# library (path or "-" for the in-tree libfia.so).  usage: tools/ab_quick.sh <config> <lib>... [-- bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
cfg=$1; shift
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ $# -gt 0 ] && shift
mkdir -p gpurun_out/abq
for lib in "${libs[@]}"; do
  if [ "$lib" = "-" ]; then unset FIA_LIB; else export FIA_LIB=$(realpath "$lib"); fi
  log=gpurun_out/abq/$(basename "$lib" .so)_$cfg.log
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline "$@" > "$log" 2>&1 || { echo "bench $lib failed"; tail -5 "$log"; exit 1; }
  tail -1 "$log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-36s' % '$lib', round(d['value']), round(d['ms_per_step'], 4), {k: round(v, 4) for k, v in d['phases_ms_per_launch'].items()}, 'score_ev', round(d['roofline'].get('kernel_ms', 0) if d['roofline'].get('phase') == 'score' else d['roofline']['score_hbm']['kernel_ms'], 4))"
done
