#!/bin/bash
# Same-box A/B of the headline step: default, no timed-region events, HIP graph replay, and the
# driver's default 20 steps with / without a 1 s spin-up.  gpurun_out/evt/*.json
export FIA_SYNTH_CACHE=/tmp/fia_synth TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/evt
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/evt/ev_$i.json 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-timed-events --steps 200 --warmup 20 > gpurun_out/evt/noev_$i.json 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --warmup 20 --graph > gpurun_out/evt/graph_$i.json 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/evt/d20_$i.json 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --spinup-seconds 1 > gpurun_out/evt/d20spin_$i.json 2>&1 || exit 1
done
for f in gpurun_out/evt/*.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))" $f
done
