#!/bin/bash
# PMC passes over a short bench run (counters only, kernel trace; no sys/runtime trace).
# usage: tools/pmc.sh <kernel-regex> <tag> [bench args...]
# (TA_* counters hung rocprofv3 on this pool: not collected)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
re="${1:-k_score}"; tag="${2:-score}"; shift 2 || true
mkdir -p gpurun_out
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
  "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $p --kernel-include-regex "$re" -d "gpurun_out/pmc_${tag}_$i" -o run \
      --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" \
      > "gpurun_out/pmc_${tag}_$i.log" 2>&1
  rc=$?
  echo "pmc pass $i ($p) exit $rc"
  case "$rc" in 0) ;; *) exit "$rc";; esac
done
