#!/bin/bash
# Round-3 measurement of one config on the GPU box: bench line, kernel-trace stats, and the
# FETCH_SIZE / WRITE_SIZE passes (separate runs) of its scoring, solve and prepare kernels.
# usage: tools/round3_prof.sh <config> <tag> [extra bench args]
#   -> gpurun_out/r3/<tag>/{bench.json, stats/, fetch/, write/}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
cfg=$1; tag=$2; shift 2
out=gpurun_out/r3/$tag
mkdir -p "$out"
re="k_score|k_solve|k_gram|k_ncf_gram|k_big|k_bs_|k_resid|k_ncf_rows"
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1
  local rc=$?
  echo "step $tag/$n exit $rc" | tee -a gpurun_out/r3/steps.log
  [ $rc -eq 0 ] || exit $rc
}
step stats 900 rocprofv3 --kernel-trace --stats -d "$out/stats" -o run --output-format csv -- \
  python3 bench.py --config "$cfg" --no-cpu-baseline "$@"
step fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$re" -d "$out/fetch" -o run --output-format csv -- \
  python3 bench.py --config "$cfg" --no-cpu-baseline --steps 1 --warmup 0 --spinup-seconds 0 "$@"
step write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$re" -d "$out/write" -o run --output-format csv -- \
  python3 bench.py --config "$cfg" --no-cpu-baseline --steps 1 --warmup 0 --spinup-seconds 0 "$@"
