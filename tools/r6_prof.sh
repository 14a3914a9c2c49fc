#!/bin/bash
# Round-6 profiles at HEAD.  usage: tools/r6_prof.sh pmc|stats <name>...
#   pmc   : the FETCH_SIZE and WRITE_SIZE passes (separate rocprofv3 runs, short bench runs)
#           -> gpurun_out/r6prof/<name>/{fetch,write}   (then tools/traffic_json.py on the host)
#   stats : the bench command itself under rocprofv3 --kernel-trace --stats; its JSON line is
#           the committed bench line (HIP-event kernel times and the rocprof averages of one run)
#           -> gpurun_out/r6prof/<name>/{stats,bench.json}
# names: ml1m yelp m64 m64i2 mf256 ncf256 ml1m8 (ml1m8: one shard of the 8-way split; m64i2:
# config 4 with two batches in flight)
# Every step under its own time limit; the first failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
declare -A ARGS=(
  [ml1m]="--config ml1m-mf"
  [ml1m8]="--config ml1m-mf --shard-of 8 --shard-index 0"
  [yelp]="--config yelp-ncf"
  [m64]="--config 20m-mf64"
  [m64i2]="--config 20m-mf64 --inflight 2"
  [mf256]="--config 20m-mf256 --shard-of 8"
  [ncf256]="--config 20m-ncf256 --shard-of 8"
)
mode=$1; shift
step() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  mkdir -p "$(dirname "$n")"
  timeout -k 10 "$t" "$@" > "$n.log" 2>&1
  local rc=$?
  echo "step $n exit $rc" | tee -a gpurun_out/r6prof/steps.log
  [ $rc -eq 0 ] || exit $rc
}
mkdir -p gpurun_out/r6prof
for n in "$@"; do
  a=${ARGS[$n]}
  o=gpurun_out/r6prof/$n
  if [ "$mode" = pmc ]; then
    step "$o/fetch" 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$o/fetch" -o run --output-format csv -- \
      python3 bench.py $a --no-cpu-baseline --steps 2 --warmup 1 --spinup-seconds 0
    step "$o/write" 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$o/write" -o run --output-format csv -- \
      python3 bench.py $a --no-cpu-baseline --steps 2 --warmup 1 --spinup-seconds 0
  else
    step "$o/stats" 600 rocprofv3 --kernel-trace --stats -d "$o/stats" -o run --output-format csv -- \
      python3 bench.py $a ${BENCH_EXTRA:-}
    grep '^{"metric"' "$o/stats.log" | tail -1 > "$o/bench.json"
    # keep the summary (kernel stats), drop the per-dispatch trace (tens of MB)
    find "$o/stats" -name '*kernel_trace.csv' -delete
  fi
done
