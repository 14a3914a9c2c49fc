"""HBM traffic per dispatch of kernels from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE, separate runs) -> profiles/traffic.json, {config: {kernel: entry}}.

    python tools/traffic_json.py <config> <fetch_dir> <write_dir> <out.json> <kernel>...

A <kernel> argument NAME=k1+k2+...[/anchor] records a phase: the bytes of all dispatches of k1,
k2, ... divided by the dispatch count of the anchor (default k1; a kernel launched once per
phase), as entry NAME (e.g. prepare_phase=k_gram_mf_stream+k_gram_combine,
solve_phase=k_bs_dupd+k_bs_dfac+k_bs_trail+k_bs_back/k_big_prologue).

MI355X_MICROARCH.md: FETCH_SIZE (KB) reports half the bytes of a wide coalesced read
on gfx950 -> doubled; WRITE_SIZE (KB) taken as is."""
import csv
import glob
import json
import os
import re
import sys


def dispatch_values(d, counter, kernel):
    # whole-name match: the kernel identifier followed by its template or parameter list
    # (k_score_mf must not pick up k_score_mf_mfma)
    pat = re.compile(r"\b%s[<(]" % re.escape(kernel))
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and pat.search(r["Kernel_Name"])]


def per_dispatch(d, counter, kernel):
    if "=" in kernel:                       # a phase: all its kernels per dispatch of the anchor
        spec = kernel.split("=", 1)[1]
        spec, anchor = spec.split("/", 1) if "/" in spec else (spec, None)
        ks = spec.split("+")
        first = dispatch_values(d, counter, anchor or ks[0])
        if not first:
            return None, 0
        return sum(sum(dispatch_values(d, counter, k)) for k in ks) / len(first), len(first)
    vals = dispatch_values(d, counter, kernel)
    if not vals:
        return None, 0
    return sum(vals) / len(vals), len(vals)


def main():
    cfg, fdir, wdir, out = sys.argv[1:5]
    kernels = sys.argv[5:]
    allres = {}
    if os.path.exists(out):
        try:
            allres = json.load(open(out))
        except Exception:
            allres = {}
    entry = allres.get(cfg, {})
    if "kernel" in entry:                      # round-2 layout {config: entry}
        entry = {entry["kernel"]: entry}
    for kern in kernels:
        f, nf = per_dispatch(fdir, "FETCH_SIZE", kern)
        w, nw = per_dispatch(wdir, "WRITE_SIZE", kern)
        if f is None or w is None:
            print("no dispatches of %s" % kern, file=sys.stderr)
            continue
        name = kern.split("=", 1)[0]
        res = {"config": cfg, "kernel": name, "hbm_bytes_per_launch": (2 * f + w) * 1024.0,
               "fetch_bytes_per_launch": 2 * f * 1024.0, "write_bytes_per_launch": w * 1024.0,
               "dispatches": [nf, nw],
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (short bench.py "
                         "runs); FETCH_SIZE(KB) x2 (gfx950 correction, MI355X_MICROARCH.md) + WRITE_SIZE(KB), "
                         "x1024, per-dispatch average"}
        if "=" in kern:
            spec = kern.split("=", 1)[1]
            spec, anchor = spec.split("/", 1) if "/" in spec else (spec, None)
            res["kernels"] = spec.split("+")
            res["scope"] = "phase %s: every dispatch of %s per dispatch of %s" % (
                name, " + ".join(res["kernels"]), anchor or res["kernels"][0])
        entry[name] = res
        print(json.dumps(res))
    allres[cfg] = entry
    json.dump(allres, open(out, "w"), indent=2)


if __name__ == "__main__":
    main()
