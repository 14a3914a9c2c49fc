#!/bin/bash
# SQ counters of the headline's prepare / solve kernels (one rocprofv3 pass each, kernel trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-pmcg}; cfg=${2:-ml1m-mf}; re=${3:-k_gram|k_solve_tps|k_score_mf_runs}
mkdir -p "$out"
i=0
for p in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $p --kernel-include-regex "$re" -d "$out/p$i" -o run --output-format csv -- \
      python3 bench.py --config "$cfg" --no-cpu-baseline --steps 3 --warmup 1 > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i exit $rc"
  [ $rc -eq 0 ] || exit $rc
  python3 tools/pmc_table.py $(find "$out/p$i" -name "run_counter_collection.csv") | tee -a "$out/table.txt"
done
