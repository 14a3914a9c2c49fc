"""Per-panel durations of the k_bs_* slab-solve kernels from a rocprofv3 --kernel-trace CSV:
dispatches of each kernel are grouped by template (panel width) and by position within a
chunk's panel sequence.  usage: python tools/trail_panels.py <kernel_trace.csv>"""
import collections
import csv
import re
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    seq = collections.defaultdict(list)
    pos = collections.Counter()
    for r in rows:
        n = r["Kernel_Name"]
        if "k_bs_" not in n:
            if "k_big_prologue" in n:
                pos.clear()
            continue
        m = re.search(r"k_bs_\w+<[^>]*>", n)
        short = m.group(0).replace("fia::", "") if m else n[:40]
        if "k_bs_back" in n:
            pos.clear()
            seq[(short, 0)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            continue
        p = pos[short]
        pos[short] += 1
        seq[(short, p)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (k, p), v in sorted(seq.items()):
        print("%-52s panel %2d  n=%4d  avg %8.1f us" % (k[:52], p, len(v), sum(v) / len(v)))


if __name__ == "__main__":
    main()
