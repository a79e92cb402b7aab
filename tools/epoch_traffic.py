"""HBM traffic of one whole epoch by kernel family from rocprofv3 PMC passes (diagnostic tool,
host side; the 4-layer model's d = 128 GraphSums).

usage: python3 tools/epoch_traffic.py gpurun_out/<dir> [marker-substring]
<dir> holds scripts/profile.sh's fetch/ and write/ passes.  The epoch is the dispatches from
the second-to-last launch of the marker kernel (default k_mask_nibbles: the 4-layer training
forward's first-layer mask layout; the 2-layer epoch has no such pass since r05 late -- pass
another marker there) up to the last.  Bytes as tools/traffic.py: FETCH_SIZE x 2 +
WRITE_SIZE (KB).  Prints one JSON object: per family {launches, fetch_MB, write_MB, hbm_MB}.
"""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_mask_nibbles"
FAMILIES = (("graphsum", ("k_graphsum_ring", "k_gs_lds_combine", "k_ring_prescale", "k_graphsum",
                          "k_gs_")),
            ("gemm", ("k_gemm", "k_xs_", "k_xstream")),
            ("loss", ("k_xent", "k_out_xent", "k_reduce_scalars")),
            ("dropout", ("k_dropout", "k_mask_nibbles", "k_relu")),
            ("other", ("",)))


def load(counter):
    f = glob.glob(os.path.join(root, counter, "**", "run_counter_collection.csv"), recursive=True)
    rows = {}
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"].startswith(counter.upper()):
            d = int(r["Dispatch_Id"])
            rows.setdefault(d, [r["Kernel_Name"], 0.0])[1] += float(r["Counter_Value"])
    return rows


fetch, write = load("fetch"), load("write")


def epoch(rows):
    ids = sorted(rows)
    marks = [d for d in ids if marker in rows[d][0]]
    return [d for d in ids if marks[-2] <= d < marks[-1]]


out = {}
for name, rows, mult in (("fetch", fetch, 2.0), ("write", write, 1.0)):
    for d in epoch(rows):
        k = rows[d][0]
        fam = next(f for f, subs in FAMILIES if any(s in k for s in subs))
        e = out.setdefault(fam, {"launches": 0, "fetch_MB": 0.0, "write_MB": 0.0})
        if name == "fetch":
            e["launches"] += 1
        e[name + "_MB"] += rows[d][1] * mult * 1024 / 1e6
for e in out.values():
    e["hbm_MB"] = round(e["fetch_MB"] + e["write_MB"], 1)
    e["fetch_MB"] = round(e["fetch_MB"], 1)
    e["write_MB"] = round(e["write_MB"], 1)
print(json.dumps(out))
