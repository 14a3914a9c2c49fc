#!/bin/bash
# Batches-in-flight A/B: bench lines at --inflight 1 and 2 (and more) for the given configs.
# usage: tools/ab_inflight.sh "<bench args>" <inflight>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
a=$1; shift
mkdir -p gpurun_out/infl
for n in "$@"; do
  log=gpurun_out/infl/$(echo "$a" | tr -c 'a-z0-9' '_')_$n.log
  timeout -k 10 300 python bench.py --no-cpu-baseline $a --inflight $n > "$log" 2>&1 || { echo fail $n; tail -5 "$log"; exit 1; }
  tail -1 "$log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; h=r if r.get('phase')=='score' else r['score_hbm']; print('$a', $n, round(d['value']/1e6,3), 'Mq/s', round(d['ms_per_step'],4), 'ms', r.get('phase'), 'score_ms', round(h.get('kernel_ms',0),4), 'frac', r.get('frac'), {k: round(v,4) for k,v in d['phases_ms_per_launch'].items()})"
done
