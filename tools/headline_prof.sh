#!/bin/bash
# Headline measurement on the GPU box: bench (with CPU baseline), kernel-trace stats of the
# same command, FETCH_SIZE / WRITE_SIZE passes.  Each step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/head
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/head/$n.log" 2>&1; local rc=$?; echo "step $n exit $rc"; [ $rc -eq 0 ] || exit $rc; }
step bench 600 python bench.py
step stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/head/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline
step fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/head/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1
step write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/head/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1
