"""Per-kernel averages of rocprofv3 counter-collection CSVs (diagnostic tool).
usage: python3 tools/pmc_summary.py <dir with */run_counter_collection.csv> [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[(r["Kernel_Name"].split("(")[0][:48], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:48s} {c:24s} n={len(v):3d} avg={sum(v) / len(v):.6g}")
