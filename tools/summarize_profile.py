"""Summarise rocprofv3 outputs (kernel stats + PMC passes) into a markdown file
under profiles/.

    python tools/summarize_profile.py <out.md> <prof_dir> [pmc_dir ...] [--bench bench.json]

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


def crosscheck(bench, stats_rows, agg):
    """The bench line's roofline against this profile: the line's bytes (traffic.json, PMC) over
    the rocprofv3 average duration of the same kernel, beside the line's HIP-event figure."""
    import json
    import re
    d = json.loads(open(bench).read())
    r = d["roofline"]
    h = r if r.get("phase") == "score" else r["score_hbm"]
    out = ["## Roofline cross-check (bench line vs this profile)", "",
           "bench line: `%s` -- %.4g queries/s, %.4f ms/step, batches in flight %s" % (
               os.path.basename(bench), d["value"], d["ms_per_step"], d["config"].get("batches_in_flight", 1)), ""]
    avg = {}
    for row in stats_rows:
        m = re.search(r"\b(k_[a-z0-9_]+)[<(]", row["Name"])
        if m:
            avg.setdefault(m.group(1), float(row["AverageNs"]) / 1e3)
    out += ["| kernel | PMC bytes / launch | HIP-event ms (line) | frac (line) | rocprof avg ms | frac (PMC / rocprof avg) |",
            "|---|---:|---:|---:|---:|---:|"]
    def row(name, traffic, ev_ms, frac):
        a = avg.get(name)
        fp = traffic / (a * 1e-6) / 8e12 if (traffic and a) else None
        out.append("| `%s` | %s | %.4f | %s | %s | %s |" % (
            name, "%.4g" % traffic if traffic else "-", ev_ms, "%.3f" % frac if frac is not None else "-",
            "%.4f" % (a / 1e3) if a else "-", "%.3f" % fp if fp is not None else "-"))
    row(h["kernel"], h.get("traffic"), h["kernel_ms"], h.get("frac"))
    if "isolated" in h:
        out.append("")
        out.append("un-overlapped (instrumented steps): %.4f ms, frac %s" % (
            h["isolated"]["kernel_ms"], "%.3f" % h["isolated"]["frac"] if h["isolated"].get("frac") else "-"))
    if r.get("phase") != "score":
        out += ["", "dominant phase `%s` (%s): %.4f ms per launch, %.4g TFLOP/s = %.3f of FP64, phase PMC bytes %s" % (
            r["phase"], r["kernel"], r["kernel_ms"], r["achieved"], r["frac"],
            "%.4g" % r["traffic"] if r.get("traffic") else "-")]
    out.append("")
    return out


def main():
    args = sys.argv[1:]
    bench = None
    if "--bench" in args:
        i = args.index("--bench")
        bench = args[i + 1]
        args = args[:i] + args[i + 2:]
    out, prof = args[0], args[1]
    pmcs = args[2:]
    lines = ["# rocprofv3 summary", "", "source: `%s` %s" % (prof, " ".join("`%s`" % p for p in pmcs)), ""]
    import glob
    kss = glob.glob(os.path.join(prof, "**", "*kernel_stats.csv"), recursive=True)
    ks = kss[0] if kss else os.path.join(prof, "run_kernel_stats.csv")
    rows = []
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
        fs = glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True)
        if not fs:
            continue
        f = fs[0]
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if bench:
        lines += crosscheck(bench, rows, agg)
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
