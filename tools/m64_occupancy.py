"""Config 4 (20M MF k=64) scoring work-item statistics on the host: how full the f64-MFMA tiles
of k_score_mf_mfma are, and the issue floors that follow (profiles/round5_m64.md).

A work item of k_score_mf_mfma is (<= kMfmaCPI = 4 list chunks of kChunk = 256 ratings of one
entity) x (<= kMfmaQB = 16 batch queries sharing that entity; 15 + the entity's own row before
round 6's Gram-pass residuals); per 16-rating tile it runs k/4 MFMAs whose A rows are the block's
queries.  This script rebuilds the
bench's batches (item-major order, --batch-rows 2^29 related ratings) from the same synthetic
draw and counts, per batch: work items, 16-rating tiles, live query rows per tile, outputs.
usage: python tools/m64_occupancy.py   (about a minute: the 20M draw)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fia-kdd-19_amd"))
from influence import synth  # noqa: E402

QB, CPI, CHUNK, K = 16, 4, 256, 64
BATCH_ROWS = 1 << 29


def main():
    d = synth.make_20m(seed=0)
    tu, ti, _ = d["train"]
    U, I = d["U"], d["I"]
    qu, qi, _ = d["test"]
    order = np.lexsort((qu, qi))
    qu, qi = qu[order].astype(np.int64), qi[order].astype(np.int64)
    du = np.bincount(tu, minlength=U).astype(np.int64)
    di = np.bincount(ti, minlength=I).astype(np.int64)
    n_q = du[qu] + di[qi]
    cum = np.concatenate([[0], np.cumsum(n_q)])
    bounds = [0]
    while bounds[-1] < qu.size:
        b0 = bounds[-1]
        b1 = int(np.searchsorted(cum, cum[b0] + BATCH_ROWS, side="right")) - 1
        bounds.append(min(qu.size, max(b1, b0 + 1)))
    tot = dict(items=0, tiles=0, live=0, outputs=0, tiles_u=0, live_u=0, tiles_i=0, live_i=0)
    for b0, b1 in zip(bounds[:-1], bounds[1:]):
        for side, ids, deg in ((0, qu[b0:b1], du), (1, qi[b0:b1], di)):
            ent, nq = np.unique(ids, return_counts=True)
            L = deg[ent]
            chunks = (L + CHUNK - 1) // CHUNK
            blocks = (nq + QB - 1) // QB
            tiles_per_ent = (L + 15) // 16           # 16-rating tiles over the entity's list
            items = ((chunks + CPI - 1) // CPI) * blocks
            tiles = tiles_per_ent * blocks
            live = tiles_per_ent * nq                 # query rows summed over the tiles
            tot["items"] += int(items.sum())
            tot["tiles"] += int(tiles.sum())
            tot["live"] += int(live.sum())
            tot["outputs"] += int((L * nq).sum())
            tot["tiles_u" if side == 0 else "tiles_i"] += int(tiles.sum())
            tot["live_u" if side == 0 else "live_i"] += int(live.sum())
    nb = len(bounds) - 1
    mfma = tot["tiles"] * (K // 4)                    # 16x16x4 f64 MFMAs (k/4 per tile)
    simds, clk = 256 * 4, 2.4e9
    print("batches %d, queries %d, outputs %.3f G" % (nb, qu.size, tot["outputs"] / 1e9))
    print("per batch: work items %.0f, 16-rating tiles %.0f, MFMAs %.0f" % (tot["items"] / nb, tot["tiles"] / nb,
                                                                          mfma / nb))
    print("live query rows per 16-row tile: %.2f of 16 (user side %.2f, item side %.2f)" % (
        tot["live"] / tot["tiles"], tot["live_u"] / max(tot["tiles_u"], 1), tot["live_i"] / max(tot["tiles_i"], 1)))
    print("tiles: user side %.1f %%, item side %.1f %%" % (100 * tot["tiles_u"] / tot["tiles"],
                                                            100 * tot["tiles_i"] / tot["tiles"]))
    print("MFMA floor per batch: %.3f ms (64 cycles per MFMA, %d SIMDs, %.1f GHz)" % (
        mfma / nb * 64 / simds / clk * 1e3, simds, clk / 1e9))
    out_b = tot["outputs"] / nb * 12
    print("output bytes per batch %.2f GB -> %.3f ms at 8 TB/s" % (out_b / 1e9, out_b / 8e12 * 1e3))


if __name__ == "__main__":
    main()
