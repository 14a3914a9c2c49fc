#!/bin/bash
# Same-box A/B of library builds: one bench run + kernel-trace stats per library (path or "-" for
# the in-tree libfia.so), in order.
# usage: tools/ab_libs.sh <outdir> <config> <lib>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FIA_SYNTH_CACHE=/tmp/fia_synth
out=gpurun_out/$1; cfg=$2; shift 2
mkdir -p "$out"
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = "-" ]; then unset FIA_LIB; else export FIA_LIB=$(realpath "$lib"); fi
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps 20 --warmup 5 > "$out/b$i.log" 2>&1 || { echo "bench $lib failed"; tail -5 "$out/b$i.log"; exit 1; }
  tail -1 "$out/b$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-28s' % '$lib', round(d['value']), round(d['ms_per_step'], 4), {k: round(v, 4) for k, v in d['phases_ms_per_launch'].items()})"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/p$i" -o run --output-format csv -- python3 bench.py --config $cfg --no-cpu-baseline --steps 20 --warmup 3 > "$out/p$i.log" 2>&1 || { echo "prof $lib failed"; exit 1; }
  python3 - "$(find "$out/p$i" -name run_kernel_stats.csv | head -1)" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:9]:
    print("   %8.1f us x %4s  %s" % (float(r["AverageNs"]) / 1e3, r["Calls"], r["Name"][:70]))
PY
done
unset FIA_LIB
