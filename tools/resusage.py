"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per kernel.
usage: python tools/resusage.py fia-kdd-19_amd/csrc/bigk.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
inc = __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "include")
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + inc,
                      "-mllvm", "-pragma-unroll-threshold=200000", "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dem = re.sub(r"fia::\(anonymous namespace\)::", "", dem)
        dem = dem.split("(")[0]
        cur = {"name": dem}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt and flt not in r["name"]:
        continue
    print("%-58s V%-4s A%-4s VS%-3s scr %-5s LDS %-7s occ %s" % (r["name"][:58], r.get("VGPRs"), r.get("AGPRs"),
          r.get("VGPRs Spill"), r.get("ScratchSize [bytes/lane]"), r.get("LDS Size [bytes/block]"), r.get("Occupancy [waves/SIMD]")))
