#!/bin/bash
# One GPU-box session: gpu tests, smoke, bench (+ optional rocprof), each step
# under its own time limit.  Stops at the first timeout / abort / crash; test
# failures (exit 1) are recorded and the remaining steps still run.
# usage: [TAG=suffix] tools/gpu_check.sh [tests|smoke|bench|bench-<config>|prof|pmc ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
steps=("$@")
[ ${#steps[@]} -eq 0 ] && steps=(tests smoke bench)

fatal() {  # exit codes that mean: do not touch the GPU again in this call
  case "$1" in 124|137|134|139|143) return 0;; *) return 1;; esac
}

for s in "${steps[@]}"; do
  case "$s" in
    tests) timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench) timeout -k 10 600 python bench.py > gpurun_out/bench${TAG:-}.log 2>&1 ;;
    bench-*) timeout -k 10 900 python bench.py --config "${s#bench-}" --no-cpu-baseline > "gpurun_out/bench_${s#bench-}.log" 2>&1 ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof${TAG:-} -o run --output-format csv -- \
            python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/prof${TAG:-}.log 2>&1 ;;
    pmc) timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch${TAG:-} -o run --output-format csv -- \
            python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/pmc_fetch.log 2>&1 && \
         timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write${TAG:-} -o run --output-format csv -- \
            python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/pmc_write.log 2>&1 ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  rc=$?
  echo "step $s exit $rc" | tee -a gpurun_out/steps.log
  if fatal "$rc"; then echo "fatal exit in $s; stopping"; exit "$rc"; fi
done
exit 0
