#!/bin/bash
# Per-kernel register / LDS / occupancy summary of one HIP source (gfx950).
# usage: tools/resusage.sh <file.hip> [kernel-regex]
f=$1; re=${2:-.}
cd "$(dirname "$f")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$(dirname "$0")/../include" -I/root/repo/include \
  -munsafe-fp-atomics -mllvm -pragma-unroll-threshold=200000 -c "$(basename "$f")" -o /dev/null \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None; rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m: cur = {"name": m.group(1)}; rows.append(cur); continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\S+)", line)
    if m and cur is not None: cur[m.group(1).strip()] = m.group(2)
    elif "error" in line: print(line.rstrip())
for r in rows:
    if re.search(sys.argv[1], r["name"]):
        print("%-70s V%-4s A%-4s scr%-4s occ%-2s vspill%-3s lds%s" % (r["name"][:70], r.get("VGPRs"), r.get("AGPRs"),
              r.get("ScratchSize [bytes/lane]"), r.get("Occupancy [waves/SIMD]"), r.get("VGPRs Spill"), r.get("LDS Size [bytes/block]")))
' "$re"
