#!/bin/bash
# A/B of one bench config: run A (env as given) and B (with the extra env assignment),
# print value, ms/step, scoring-kernel ms and per-launch phases of each.
# usage: tools/ab_bench.sh <config> "<VAR=value for B>" [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
cfg=$1; benv=$2; shift 2
mkdir -p gpurun_out/ab
timeout -k 10 300 python bench.py --config "$cfg" --no-cpu-baseline --steps 5 --warmup 2 "$@" > gpurun_out/ab/A.log 2>&1 || exit $?
env $benv timeout -k 10 300 python bench.py --config "$cfg" --no-cpu-baseline --steps 5 --warmup 2 "$@" > gpurun_out/ab/B.log 2>&1 || exit $?
for f in A B; do
  tail -1 gpurun_out/ab/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value']), round(d['ms_per_step'], 3), round(d['roofline']['kernel_ms'], 4), {k: round(v, 4) for k, v in d['phases_ms_per_launch'].items()})"
done
