"""Epochs/s on the small datasets (cora, citeseer, pubmed_synth) on one GPU, beside the
reference's own sequential epoch on this host ("epochs/sec on
citeseer/cora/pubmed/reddit").  Diagnostic tool; bench.py stays the reddit headline.

usage: python3 tools/datasets_bench.py [--epochs 200] [--graph 0|1|both] [--out file.json]

Two GPU numbers per dataset:
  * "async": epoch_async() back to back (metrics go to the device results ring, one host
    sync at the end) -- the engine's throughput;
  * "reference_loop": train_epoch() + eval(2) with their host reads of loss/accuracy every
    epoch, i.e. the reference's own run() loop (src/gcn.cu:363-375), timed per epoch and
    reported as 100 / sum of epoch times like TMR_TRAIN.
The CPU leg is oracle/_ref (the reference's hpdga sources, 1 thread) when built, else the C
restatement.  Inputs come from the committed fixtures (tests/golden/data).

Launch floor: these epochs are a few dozen short kernels each, so next to epochs/s the tool
reports the kernel launches per epoch (the library's launch counter, pgcn_debug_path_count
"launches") times the time of one empty kernel launched back to back the same way
(pgcn_debug_empty_launches), i.e. the epochs/s an epoch of empty kernels would reach, and
the measured rate as a fraction of it.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime per process: torch's)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if "--lib" in sys.argv:  # an A/B build of the library (as PGCN_LIB), set before it loads
    os.environ["PGCN_LIB"] = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402


def gpu_rates(pg, ds, epochs, graph):
    pg.lib.pgcn_debug_set(b"epoch_graph", graph)
    g = pg.GCN(pg.make_params(ds), ds, device=0)
    for _ in range(5):
        g.epoch_async()
    g.sync()
    t0 = time.perf_counter()
    for _ in range(epochs):
        g.epoch_async()
    g.sync()
    async_rate = epochs / (time.perf_counter() - t0)
    res = g.results(1)
    total = 0.0
    for _ in range(min(epochs, 100)):
        t0 = time.perf_counter()
        g.train_epoch()
        g.eval(2)
        total += time.perf_counter() - t0
    g.close()
    pg.lib.pgcn_debug_set(b"epoch_graph", 0)
    return async_rate, min(epochs, 100) / total, res


def launch_floor_us(pg, n=2000):
    """microseconds per empty kernel launched back to back from the host (best of 3)."""
    import ctypes
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    pg.check(pg.lib.pgcn_debug_empty_launches(100, sp), "empty")
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        pg.check(pg.lib.pgcn_debug_empty_launches(n, sp), "empty")
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n * 1e6
        best = dt if best is None else min(best, dt)
    return best


def launches_per_epoch(pg, ds, epochs=20):
    g = pg.GCN(pg.make_params(ds), ds, device=0)
    for _ in range(3):
        g.epoch_async()
    g.sync()
    pg.reset_path_counts()
    for _ in range(epochs):
        g.epoch_async()
    g.sync()
    n = pg.path_counts()["launches"] / epochs
    g.close()
    return n


def cpu_rate(ds, reps):
    import bench
    kind, times = bench.cpu_baseline(ds, reps)[:2]
    return kind, len(times) / sum(times)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=200)
    ap.add_argument("--graph", default="both", choices=["0", "1", "both"])
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="one dataset (e.g. under rocprofv3)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--lib", default=None, help="another build of libpgcn.so (A/B)")
    ap.add_argument("--set", action="append", default=[], metavar="KNOB=VALUE",
                    help="engine knob (pgcn_debug_set) for every engine built (A/B runs)")
    args = ap.parse_args()
    sys.path.insert(0, REPO)
    pg = helpers.pgcn()
    for kv in args.set:
        k, v = kv.split("=")
        pg.check(pg.lib.pgcn_debug_set(k.encode(), int(v)), "knob " + k)
    modes = [0, 1] if args.graph == "both" else [int(args.graph)]
    out = {}
    floor_us = launch_floor_us(pg)
    out["empty_launch_us"] = floor_us
    print("empty launch", round(floor_us, 3), "us", flush=True)
    with tempfile.TemporaryDirectory() as root:
        for name in ((args.only,) if args.only else ("cora", "citeseer", "pubmed_synth")):
            dname = helpers.materialize_dataset(name, root)
            ds = pg.Dataset.load(root, dname)
            row = {"nodes": int(ds.num_nodes), "adjacency_nnz": int(ds.graph_indptr[-1])}
            for m in modes:
                a, r, res = gpu_rates(pg, ds, args.epochs, m)
                key = "graph" if m else "eager"
                row[f"{key}_async_epochs_s"] = a
                row[f"{key}_reference_loop_epochs_s"] = r
                row[f"{key}_last"] = [float(v) for v in np.asarray(res).ravel()]
            lpe = launches_per_epoch(pg, ds)
            row["launches_per_epoch"] = lpe
            row["launch_floor_epochs_s"] = 1e6 / (lpe * floor_us)
            if "eager_async_epochs_s" in row:
                row["eager_frac_of_launch_floor"] = row["eager_async_epochs_s"] / row["launch_floor_epochs_s"]
            if not args.no_cpu:
                kind, c = cpu_rate(ds, args.cpu_reps)
                row["cpu_epochs_s"] = c
                row["cpu_kind"] = kind
            out[name] = row
            print(name, json.dumps(row), flush=True)
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
