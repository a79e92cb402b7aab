"""HBM traffic per GraphSum call from rocprofv3 PMC passes (diagnostic tool, run on the host
after scripts/profile.sh's fetch/write passes).

usage: python3 tools/traffic.py gpurun_out/<dir> [epoch_calls] [--write <round>]
           [--key <workload>] [--hidden <dims, '+'-separated>] [--epoch <calls per epoch>]

--epoch C (r06): the bytes of every GraphSum-family launch (the wide passes' prescale and
combines included) between the last two Adam launches (k_adam_multi or k_adam_mask) -- one epoch -- divided by the
epoch's C GraphSum calls; the 4-layer model's d = 128 calls are 8 ring passes each.  --key: the
entry of profiles/traffic_graphsum.json to write (default reddit-114M); --write merges it into
the file when the file's source stamp matches (else the file starts afresh).

With --write, profiles/traffic_graphsum.json is rewritten with the bytes, the round tag and
the source stamp of the kernel the passes measured (tools/stamp.py): bench.py reports the
bytes as roofline.traffic only while that stamp matches the sources it runs.

A GraphSum call is its prescale (k_ring_prescale, or k_gs_prescale on the window-1 schedule;
absent when a fused epilogue staged the table) + k_graphsum_ring / k_graphsum_lds +
k_gs_lds_combine (the launches the bench's HIP events bracket).  Only the last `epoch_calls` calls (default 20: 4 epochs x 5) are
counted, so the engine-build calls (Â X precompute) are left out.  Bytes follow
MI355X_MICROARCH.md's HBM section: FETCH_SIZE x 2 (gfx950 tallies the 128-B requests of
16-B/lane streams at 64 B) + WRITE_SIZE, both in KB.  Prints one JSON object.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from stamp import REPO, graphsum_stamp  # noqa: E402

argv = list(sys.argv[1:])


def opt(name, default=None):
    if name in argv:
        i = argv.index(name)
        v = argv[i + 1]
        del argv[i:i + 2]
        return v
    return default


write_round = opt("--write")
# the entry: the bench workload, and its hidden dims when not the 2-layer hidden-16 model
# (written with '+' for ',': "--hidden 128+128+128" -> "reddit-114M hidden=128,128,128")
hid = opt("--hidden", "16").replace("+", ",")
key = opt("--key", "reddit-114M") + ("" if hid == "16" else f" hidden={hid}")
per_epoch = opt("--epoch")
root = argv[0]
n_calls = int(argv[1]) if len(argv) > 1 else 20
GS_FAMILY = ("k_gs_prescale", "k_ring_prescale", "k_graphsum_lds", "k_graphsum_ring",
             "k_gs_lds_combine")


def per_dispatch(counter):
    rows = []
    for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    return rows


out = {}
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    allrows = per_dispatch(counter)
    rows = [r for r in allrows if any(k in r[1] for k in GS_FAMILY)]
    if per_epoch:  # one epoch between the last two Adam launches, per GraphSum call
        adam = [d for d, name, _ in allrows if "k_adam_multi" in name or "k_adam_mask" in name]
        lo, hi = adam[-2], adam[-1]
        tot = sum(v for d, _, v in rows if lo < d < hi)
        out[counter + "_KB_per_call"] = tot / int(per_epoch)
        out[counter + "_calls"] = int(per_epoch)
        continue
    calls, cur = [], 0.0
    for _, name, v in rows:
        cur += v
        if "k_gs_lds_combine" in name:
            calls.append(cur)
            cur = 0.0
    calls = calls[-n_calls:]
    out[counter + "_KB_per_call"] = sum(calls) / max(len(calls), 1)
    out[counter + "_calls"] = len(calls)
out["hbm_bytes_per_call"] = (2 * out["FETCH_SIZE_KB_per_call"] + out["WRITE_SIZE_KB_per_call"]) * 1024
out["source_stamp"] = graphsum_stamp()
print(json.dumps(out))
if write_round:
    path = os.path.join(REPO, "profiles", "traffic_graphsum.json")
    try:
        old = json.load(open(path))
    except (OSError, ValueError):
        old = {}
    keep = old if old.get("source_stamp") == out["source_stamp"] else {}
    entries = {k: v for k, v in keep.items() if k.startswith("reddit")}
    raw = dict(keep.get("raw_per_call_KB_by_key", {}))
    entries[key] = out["hbm_bytes_per_call"]
    raw[key] = {"FETCH_SIZE": out["FETCH_SIZE_KB_per_call"],
                "WRITE_SIZE": out["WRITE_SIZE_KB_per_call"], "calls": out["FETCH_SIZE_calls"]}
    doc = dict(entries)
    doc.update({
        "source_stamp": out["source_stamp"],
        "round": write_round,
        "_doc": "HBM-side bytes per GraphSum call (ring prescale when not staged by a fused "
                "epilogue + k_graphsum_ring + k_gs_lds_combine, the launches the bench's HIP "
                "events bracket), averaged over the last %d GraphSum calls of bench.py "
                "--profile-only on reddit-114M with the engine defaults (engine-build A X calls "
                "excluded). Separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; "
                "scripts/profile.sh), corrected as MI355X_MICROARCH.md prescribes: FETCH_SIZE x2 "
                "+ WRITE_SIZE. source_stamp = tools/stamp.py over the kernel's sources; bench.py "
                "reports null when it no longer matches." % n_calls,
        "raw_per_call_KB_by_key": raw,
    })
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
