"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (one row per dispatch x counter)."""
import csv
import sys
from collections import defaultdict

for path in sys.argv[1:]:
    acc = defaultdict(lambda: defaultdict(list))
    for row in csv.DictReader(open(path)):
        acc[row["Kernel_Name"][:60]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    print("##", path)
    for k, cs in acc.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        n = len(next(iter(cs.values())))
        line = " ".join("%s=%.4g" % (c, v) for c, v in sorted(avg.items()))
        print("%s (n=%d): %s" % (k, n, line))
