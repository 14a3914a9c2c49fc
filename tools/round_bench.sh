#!/bin/bash
# Full measurement pass on the GPU box: tests, smoke, every bench config, headline rocprof.
# Each GPU step under its own time limit; stops at the first timeout / crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/round
export TMPDIR=/tmp
fatal() { case "$1" in 124|137|134|139|143) return 0;; *) return 1;; esac; }
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/round/$name.log" 2>&1
  local rc=$?
  echo "step $name exit $rc" | tee -a gpurun_out/round/steps.log
  if fatal "$rc"; then echo "fatal exit in $name"; exit "$rc"; fi
}
run tests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_ml1m 600 python bench.py
run bench_yelp 600 python bench.py --config yelp-ncf --cpu-baseline-seconds 15
run bench_20m64 900 python bench.py --config 20m-mf64 --steps 5 --warmup 1 --cpu-baseline-seconds 20
run bench_mf256 600 python bench.py --config 20m-mf256 --shard-of 8 --steps 3 --warmup 1 --no-cpu-baseline
run bench_ncf256 600 python bench.py --config 20m-ncf256 --shard-of 8 --steps 2 --warmup 1 --no-cpu-baseline
run prof_ml1m 600 rocprofv3 --kernel-trace --stats -d gpurun_out/round/prof_ml1m -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3
exit 0
