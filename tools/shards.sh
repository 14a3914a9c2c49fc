#!/bin/bash
# One bench run per shard of an S-way strong-scaling split on one GPU (what each rank of an
# S-GPU job answers): gpurun_out/shards/<config>_<r>.json.  usage: tools/shards.sh <config> <S> [steps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
cfg=$1; S=$2; steps=${3:-3}
mkdir -p gpurun_out/shards
for r in $(seq 0 $((S - 1))); do
  timeout -k 10 600 python bench.py --config "$cfg" --shard-of "$S" --shard-index "$r" --no-cpu-baseline \
      --steps "$steps" --warmup 1 --spinup-seconds 5 > "gpurun_out/shards/${cfg}_$r.log" 2>&1
  rc=$?
  echo "shard $r exit $rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 "gpurun_out/shards/${cfg}_$r.log" > "gpurun_out/shards/${cfg}_$r.json"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['config']['queries_per_rank'], round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_step'].items()})" "gpurun_out/shards/${cfg}_$r.json" "$r"
done
