#!/bin/bash
# Round profile pass: for each config, a rocprofv3 kernel-trace --stats run and the two PMC
# traffic passes (FETCH_SIZE, WRITE_SIZE; separate runs) -> gpurun_out/rprof/<name>/{stats,fetch,write}.
# usage: tools/round_prof.sh [name ...]   (names: ml1m yelp m64 mf256 ncf256; default all)
# Each step under its own time limit; the first failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
declare -A ARGS=(
  [ml1m]="--config ml1m-mf"
  [yelp]="--config yelp-ncf"
  [m64]="--config 20m-mf64"
  [mf256]="--config 20m-mf256 --shard-of 8"
  [ncf256]="--config 20m-ncf256 --shard-of 8"
)
names=("$@"); [ ${#names[@]} -eq 0 ] && names=(ml1m yelp m64 mf256 ncf256)
step() {  # dir timeout cmd...
  local n=$1 t=$2; shift 2
  mkdir -p "$(dirname "$n")"
  timeout -k 10 "$t" "$@" > "$n.log" 2>&1
  local rc=$?
  echo "step $n exit $rc" | tee -a gpurun_out/rprof/steps.log
  [ $rc -eq 0 ] || exit $rc
}
mkdir -p gpurun_out/rprof
for n in "${names[@]}"; do
  a=${ARGS[$n]}
  o=gpurun_out/rprof/$n
  step "$o/stats" 600 rocprofv3 --kernel-trace --stats -d "$o/stats" -o run --output-format csv -- \
    python3 bench.py $a --no-cpu-baseline --steps 3 --warmup 1 --spinup-seconds 0
  step "$o/fetch" 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$o/fetch" -o run --output-format csv -- \
    python3 bench.py $a --no-cpu-baseline --steps 1 --warmup 0 --spinup-seconds 0
  step "$o/write" 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$o/write" -o run --output-format csv -- \
    python3 bench.py $a --no-cpu-baseline --steps 1 --warmup 0 --spinup-seconds 0
done
