"""Where a single query's wall time goes (RQ2, ml-1m-ex MF test_idx 59): the facade call with
the RQ2 timers, the one-sync path without them, and the library calls alone (median of 50)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fia-kdd-19_amd"))
sys.path.insert(0, ROOT)


def med(f, n=50):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


def main():
    import torch
    from scripts import RQ2
    from scripts.load_movielens import load_movielens_synthetic
    ds = load_movielens_synthetic(0)
    cfg = dict(RQ2.configs)
    m = RQ2.build("movielens", "MF", cfg, ds, train_dir="/tmp/rq2b")
    t = 59
    N = ds["train"].labels.shape[0]
    ar = np.arange(N)
    m.get_influence_on_test_loss([t], ar)
    print("facade call (RQ2 timers)   %.1f us" % med(lambda: m.get_influence_on_test_loss([t], ar)))
    print("  its own wall (last_timing) %.1f us" % (m.last_timing["wall_s"] * 1e6))
    print("one-sync path, no timers   %.1f us" % med(lambda: m._one_query(t)))
    b = m._one_bufs
    u, i = m._test_pair(t)
    n = int(m._deg_u[u] + m._deg_i[i])
    qu, qi = b["q"][0:1], b["q"][1:2]
    s = torch.cuda.current_stream()

    def lib_only():
        m.ctx.count_related(qu, qi, b["off"], want_total=False)
        m.ctx.query_batch(qu, qi, b["off"], n, b["rel"], b["infl"], b["x"], 0, None, None, None)
        s.synchronize()
    print("library calls + sync       %.1f us" % med(lib_only))

    def sync_only():
        s.synchronize()
    print("stream sync alone          %.1f us" % med(sync_only))

    def copies():
        b["din"][:8].copy_(b["hin_all"][:8], non_blocking=True)
        b["hout"].copy_(b["dout"], non_blocking=True)
        s.synchronize()
    print("H2D + D2H copies + sync    %.1f us" % med(copies))
    m.ctx.close()


if __name__ == "__main__":
    main()
