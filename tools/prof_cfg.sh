#!/bin/bash
# Kernel-trace stats + PMC passes of one bench config on the GPU box.
# usage: tools/prof_cfg.sh <config> <tag> <kernel-regex> [extra bench args...]
#   -> gpurun_out/<tag>/{bench.log, stats/, pmc_*}
# Every step under its own time limit; the first failing step ends the script.
# PMC passes are separate runs (counter-slot limits: 8 SQ, 4 TCC incl. FETCH_SIZE=3 / WRITE_SIZE=2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
cfg=$1; tag=$2; re=$3; shift 3
out=gpurun_out/$tag
mkdir -p "$out"
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1
  local rc=$?
  echo "step $n exit $rc" | tee -a "$out/steps.log"
  [ $rc -eq 0 ] || exit $rc
}
step bench 900 python bench.py --config "$cfg" --no-cpu-baseline "$@"
step stats 600 rocprofv3 --kernel-trace --stats -d "$out/stats" -o run --output-format csv -- \
  python3 bench.py --config "$cfg" --no-cpu-baseline "$@"
[ "${PMC:-1}" = "1" ] || exit 0
i=0
for p in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  step "pmc$i" 300 rocprofv3 --pmc $p --kernel-include-regex "$re" -d "$out/pmc$i" -o run --output-format csv -- \
    python3 bench.py --config "$cfg" --no-cpu-baseline --steps 1 --warmup 0 "$@"
done
