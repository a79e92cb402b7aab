"""Median duration (us) of a kernel's calls in a rocprofv3 kernel trace, split by call parity
(the loss kernel alternates training / eval calls in the bench epoch).
usage: python3 tools/trace_split.py <run_kernel_trace.csv> <name-substring> [period]"""
import csv
import statistics
import sys

path, pat = sys.argv[1], sys.argv[2]
period = int(sys.argv[3]) if len(sys.argv) > 3 else 2
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
     for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
print(f"{pat}: {len(d)} calls;", " ".join(
    f"phase{p} med {statistics.median(d[p::period]):.1f}" for p in range(period) if d[p::period]))
