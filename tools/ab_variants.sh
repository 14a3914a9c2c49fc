#!/bin/bash
# Same-box comparison of library variants selected by environment knobs: one bench run per
# "VAR=value ..." argument (use "-" for the default build), in order, each printed as
#   <label> value ms/step scoring-kernel-ms phases
# usage: tools/ab_variants.sh <config> <variant>... [-- extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
cfg=$1; shift
vars=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do vars+=("$1"); shift; done
[ $# -gt 0 ] && shift
mkdir -p gpurun_out/abv
i=0
for v in "${vars[@]}"; do
  i=$((i+1))
  e=(); [ "$v" != "-" ] && e=($v)
  env "${e[@]}" timeout -k 10 300 python bench.py --config "$cfg" --no-cpu-baseline --steps 5 --warmup 2 "$@" > gpurun_out/abv/$i.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/abv/$i.log; exit 1; }
  tail -1 gpurun_out/abv/$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-40s' % '$v', round(d['value']), round(d['ms_per_step'], 3), round(d['roofline']['kernel_ms'], 4), {k: round(v, 4) for k, v in d['phases_ms_per_launch'].items()})"
done
