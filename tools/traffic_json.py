"""HBM traffic per dispatch of one kernel from two rocprofv3 PMC passes
(FETCH_SIZE and WRITE_SIZE, separate runs) -> profiles/score_traffic.json (one entry per config).

    python tools/traffic_json.py <config> <kernel-substring> <fetch_dir> <write_dir> <out.json>

MI355X_MICROARCH.md: FETCH_SIZE (KB) reports half the bytes of a wide coalesced read
on gfx950 -> doubled; WRITE_SIZE (KB) taken as is."""
import csv
import json
import os
import re
import sys


def per_dispatch(d, counter, kernel):
    # whole-name match: the kernel identifier followed by its template or parameter list
    # (k_score_mf must not pick up k_score_mf_mfma)
    pat = re.compile(r"\b%s[<(]" % re.escape(kernel))
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv")))
            if r["Counter_Name"] == counter and pat.search(r["Kernel_Name"])]
    return sum(vals) / len(vals), len(vals)


def main():
    cfg, kern, fdir, wdir, out = sys.argv[1:6]
    f, nf = per_dispatch(fdir, "FETCH_SIZE", kern)
    w, nw = per_dispatch(wdir, "WRITE_SIZE", kern)
    res = {"config": cfg, "kernel": kern, "hbm_bytes_per_launch": (2 * f + w) * 1024.0,
           "fetch_bytes_per_launch": 2 * f * 1024.0, "write_bytes_per_launch": w * 1024.0,
           "dispatches": [nf, nw],
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (short bench.py runs); "
                     "FETCH_SIZE(KB) x2 (gfx950 correction, MI355X_MICROARCH.md) + WRITE_SIZE(KB), x1024, "
                     "per-dispatch average"}
    # one entry per config: {config: {...}} (an older single-entry file is converted)
    allres = {}
    if os.path.exists(out):
        try:
            old = json.load(open(out))
            allres = {old["config"]: old} if "config" in old else old
        except Exception:
            allres = {}
    allres[cfg] = res
    json.dump(allres, open(out, "w"), indent=2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
