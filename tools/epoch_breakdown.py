"""Per-epoch kernel breakdown from a rocprofv3 kernel trace (diagnostic tool, host side).

usage: python3 tools/epoch_breakdown.py gpurun_out/<dir>/trace [marker-kernel-substring]

An epoch is taken between the last two launches of the marker kernel (default: eval's
first-layer GEMM over Â X, `k_xs_nn_ring<38, false, false, false, false[, true]>`).  Prints the epoch's span, the
sum of its kernel times, the gaps between launches and the per-kernel times in launch order.
"""
import collections
import csv
import os
import sys

trace_dir = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_xs_nn_ring<38, false, false, false, false"
rows = list(csv.DictReader(open(os.path.join(trace_dir, "run_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
if len(idx) < 2:
    sys.exit(f"fewer than two launches of {marker!r}")
a, b = idx[-2], idx[-1]
ep = rows[a:b]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
t0, t1 = int(ep[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
gaps = [(int(ep[i + 1]["Start_Timestamp"]) - int(ep[i]["End_Timestamp"])) / 1e3
        for i in range(len(ep) - 1)]
print(f"epoch span {(t1 - t0) / 1e3:.1f} us, kernel sum {sum(dur(r) for r in ep):.1f} us, "
      f"{len(ep)} launches, gaps {sum(gaps):.1f} us")
agg = collections.OrderedDict()
for r in ep:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pgcn::", "")
    agg.setdefault(k, []).append(round(dur(r), 1))
for k, v in agg.items():
    print(f"{k:42s} {sum(v):7.1f}  {v}")
