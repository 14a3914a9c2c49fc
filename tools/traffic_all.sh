#!/bin/bash
# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes, separate runs) of the scoring kernel of
# the yelp-ncf and 20m-mf64 configs -> gpurun_out/traf/<config>_{fetch,write}.  Each pass
# under its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/traf
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/traf/$n.log" 2>&1; local rc=$?; echo "step $n exit $rc"; [ $rc -eq 0 ] || exit $rc; }
step yelp_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/traf/yelp_fetch -o run --output-format csv -- python3 bench.py --config yelp-ncf --no-cpu-baseline --steps 5 --warmup 1
step yelp_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/traf/yelp_write -o run --output-format csv -- python3 bench.py --config yelp-ncf --no-cpu-baseline --steps 5 --warmup 1
step m64_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/traf/m64_fetch -o run --output-format csv -- python3 bench.py --config 20m-mf64 --no-cpu-baseline --steps 1 --warmup 0
step m64_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/traf/m64_write -o run --output-format csv -- python3 bench.py --config 20m-mf64 --no-cpu-baseline --steps 1 --warmup 0
