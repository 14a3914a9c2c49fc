#!/bin/bash
# Round-5 iteration on the GPU box: the parity tests (optionally a -k filter), the headline bench
# and a kernel-trace profile of the same bench.  Each step under its own limit; stops at the
# first failure.
# usage: tools/r5_check.sh <outdir> [pytest -k expr] [bench config]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/$1; kexpr=${2:-}; cfg=${3:-ml1m-mf}
mkdir -p "$out"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
step() { local n=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "step $n exit $rc"; tail -3 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
if [ -n "$kexpr" ]; then
  step tests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$kexpr"
fi
step bench 300 python bench.py --config "$cfg" --no-cpu-baseline --steps 20 --warmup 5
step stats 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python3 bench.py --config "$cfg" --no-cpu-baseline --steps 20 --warmup 3
p=$(dirname "$(find "$out/prof" -name run_kernel_stats.csv | head -1)"); python3 tools/summarize_profile.py "$out/kernels.md" "$p" || true
head -30 "$out/kernels.md"
