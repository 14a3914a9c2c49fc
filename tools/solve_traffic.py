"""Record the side-solve phase's PMC HBM bytes per solve launch in profiles/traffic.json.

    python tools/solve_traffic.py <config> <summary.md>

summary.md: tools/summarize_profile.py output of a FETCH_SIZE and a WRITE_SIZE pass over
the k_bs_* kernels and k_big_score_mfma (tools/g35.sh).  A solve launch (one query batch)
dispatches each k_bs_* kernel many times (one per 64-column panel and slab chunk); the
scoring kernel runs once per batch, so dispatches per launch = n(kernel) / n(score).
Bytes follow MI355X_MICROARCH.md: FETCH_SIZE (KB) x 2 + WRITE_SIZE (KB), x 1024.
"""
import json
import os
import re
import sys


def parse(md):
    out, cur = {}, None
    for line in open(md):
        m = re.match(r"### `(.+?)`", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.match(r"- (FETCH_SIZE|WRITE_SIZE) = ([0-9.e+]+) \(n=(\d+)\)", line)
        if m and cur:
            out[cur][m.group(1)] = (float(m.group(2)), int(m.group(3)))
    return out


def main():
    config, md = sys.argv[1], sys.argv[2]
    k = parse(md)
    score = [v for n, v in k.items() if "k_big_score_mfma" in n][0]
    n_launch = score["FETCH_SIZE"][1]
    total, parts = 0.0, {}
    for name, v in k.items():
        if "k_bs_" not in name or "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
            continue
        per = (2.0 * v["FETCH_SIZE"][0] + v["WRITE_SIZE"][0]) * 1024.0
        disp = v["FETCH_SIZE"][1] / n_launch
        short = re.sub(r"^void ", "", name).split("(")[0]
        parts[short] = {"bytes_per_dispatch": per, "dispatches_per_launch": disp}
        total += per * disp
    path = os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json")
    tj = json.load(open(path))
    tj.setdefault(config, {})["solve_phase"] = {
        "config": config, "kernel": "solve_phase", "hbm_bytes_per_launch": total,
        "scope": "side-solve phase per launch (one query batch): k_bs_dupd + k_bs_dfac + k_bs_trail + k_bs_back",
        "parts": parts,
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/g35.sh, %s); FETCH_SIZE(KB) x2 + "
                  "WRITE_SIZE(KB), x1024, per-dispatch averages x dispatches per batch" % os.path.basename(md)}
    json.dump(tj, open(path, "w"), indent=1)
    print(config, "%.3e bytes per solve launch" % total, parts)


if __name__ == "__main__":
    main()
