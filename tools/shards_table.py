"""Markdown table of a one-GPU-per-shard measurement (tools/shards.sh output,
gpurun_out/shards/<config>_<r>.json) with the predicted S-GPU step (the slowest shard: the
ranks run independently and the top-K all_gather overlaps the next step).

    python tools/shards_table.py <config> <S> <N=1 ms/step> [dir]   -> markdown on stdout"""
import json
import os
import sys


def main():
    cfg, S, n1 = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
    d = sys.argv[4] if len(sys.argv) > 4 else "gpurun_out/shards"
    rows = [json.load(open(os.path.join(d, "%s_%d.json" % (cfg, r)))) for r in range(S)]
    out = ["## %s" % cfg, "", "| shard | queries | ms/step | prepare | chunks | solve | score | top-K |",
           "|---:|---:|---:|---:|---:|---:|---:|---:|"]
    for r, j in enumerate(rows):
        p = j["phases_ms_per_step"]
        out.append("| %d | %d | %.4f | %.4f | %.4f | %.4f | %.4f | %.4f |" % (
            r, j["config"]["queries_per_rank"][0], j["ms_per_step"], p.get("prepare", 0), p.get("chunks", 0),
            p.get("solve", 0), p.get("score", 0), p.get("topk", 0)))
    mx = max(j["ms_per_step"] for j in rows)
    nq = sum(j["config"]["queries_per_rank"][0] for j in rows)
    out += ["", "Predicted %d-GPU step = max over shards = %.4f ms (N=1 step %.4f ms, ideal N1/%d = %.4f ms, "
            "max / ideal = %.3f): predicted speed-up %.2fx, %.0f %% of linear; %d queries in all shards."
            % (S, mx, n1, S, n1 / S, mx / (n1 / S), n1 / mx, 100 * n1 / mx / S, nq), ""]
    print("\n".join(out))


if __name__ == "__main__":
    main()
