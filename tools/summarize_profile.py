"""Summarise rocprofv3 outputs (kernel stats + PMC passes) into a markdown file
under profiles/.

    python tools/summarize_profile.py <out.md> <prof_dir> [pmc_dir ...]

prof_dir holds run_kernel_stats.csv (rocprofv3 --kernel-trace --stats
--output-format csv); each pmc_dir holds run_counter_collection.csv.  HBM bytes
follow MI355X_MICROARCH.md: FETCH_SIZE (KB) is doubled (gfx950 reports half of
a wide coalesced read), WRITE_SIZE (KB) is taken as is.
"""
import collections
import csv
import os
import sys


def short(name, n=70):
    name = name.replace("fia::(anonymous namespace)::", "")
    return name if len(name) <= n else name[:n] + "..."


def main():
    out, prof = sys.argv[1], sys.argv[2]
    pmcs = sys.argv[3:]
    lines = ["# rocprofv3 summary", "", "source: `%s` %s" % (prof, " ".join("`%s`" % p for p in pmcs)), ""]
    ks = os.path.join(prof, "run_kernel_stats.csv")
    if os.path.exists(ks):
        rows = list(csv.DictReader(open(ks)))
        lines += ["## Kernel time (--kernel-trace --stats)", "",
                  "| kernel | calls | avg us | total % |", "|---|---:|---:|---:|"]
        for r in rows:
            lines.append("| `%s` | %s | %.1f | %.2f |" % (short(r["Name"]), r["Calls"], float(r["AverageNs"]) / 1e3,
                                                       float(r["Percentage"])))
        lines.append("")
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in pmcs:
        f = os.path.join(p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if agg:
        lines += ["## PMC (per-dispatch averages)", ""]
        for k, cs in sorted(agg.items()):
            if "rocclr" in k or "rocprim" in k:
                continue
            lines.append("### `%s`" % k)
            lines.append("")
            for c, v in sorted(cs.items()):
                lines.append("- %s = %.6g (n=%d)" % (c, sum(v) / len(v), len(v)))
            if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
                fb = 2 * sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024
                wb = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
                lines.append("- HBM bytes per dispatch (2*FETCH_SIZE + WRITE_SIZE) = %.4g" % (fb + wb))
            lines.append("")
    open(out, "w").write("\n".join(lines) + "\n")
    print("wrote", out)


if __name__ == "__main__":
    main()
