"""GraphSum roofline fraction two ways from ONE bench run (diagnostic tool, host side):
rocprofv3 --kernel-trace of `bench.py` (not --profile-only) gives the kernel durations of the
bench's two HIP-event-profiled epochs, the last `calls` GraphSum calls (prescale when launched +
k_graphsum_ring + k_gs_lds_combine, the launches the events bracket); the bench's JSON line
gives the event-timed figure of the same calls.  Prints one JSON object with both fractions.

usage: python3 tools/gs_fraction.py <trace_dir> <bench.json> [calls=10]
"""
import csv
import json
import os
import sys

trace, bench = sys.argv[1], sys.argv[2]
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 10
rows = list(csv.DictReader(open(os.path.join(trace, "run_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
GS = ("k_ring_prescale", "k_graphsum_ring", "k_gs_lds_combine")
per_call, cur = [], 0.0
for r in rows:
    name = r["Kernel_Name"]
    if any(k in name for k in GS):
        cur += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "k_gs_lds_combine" in name:
            per_call.append(cur)
            cur = 0.0
per_call = per_call[-calls:]
b = json.load(open(bench))
roof = b["roofline"]
bytes_call = roof["algorithmic_bytes_per_call"]
prof_us = sum(per_call) / len(per_call)
out = {
    "calls": len(per_call),
    "rocprof_us_per_call": prof_us,
    "rocprof_frac": bytes_call / (prof_us * 1e-6) / 1e9 / roof["peak"],
    "events_us_per_call": roof["avg_call_ms"] * 1e3,
    "events_frac": roof["frac"],
    "per_call_us": per_call,
    "value": b["value"],
}
out["difference"] = out["events_frac"] - out["rocprof_frac"]
print(json.dumps(out))
