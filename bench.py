#!/usr/bin/env python3
"""bench.py -- training epochs/sec of the 2-layer GCN (hidden 16) on reddit-shaped data.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1 launched with
torch.distributed.run, one process per GPU.  A "step" is one reference epoch:
GCN::train_epoch() + GCN::eval(2) (hpdga-spring23/src/gcn.cpp:221-232, src/gcn.cu:363-375)
over the whole graph.  Rank 0 prints ONE JSON line.

Workload (BASELINE.json configs[2]/[3]): reddit-shaped SYNTHETIC graph -- N = 232,965
nodes, F = 602 dense features, C = 41 classes, Chung-Lu power-law adjacency with 114,615,892
directed slots (+ N implicit self loops = 114,848,857 = nnz of Â), seed 1 (the reddit files
are not in the reference tree).  Inputs are resident in HBM before the timed region.

Multi-GPU: edge-cut (contiguous nnz-balanced node ranges), RCCL reduce-scatter per GraphSum
and all-reduce of weight grads inside the C++ engine; the graph is fixed, so scaling is
STRONG (value = epochs of the whole graph per second, all ranks together).

Extra fields: "roofline" for the dominant kernel (GraphSum: algorithmic bytes per call over
its HIP-event-timed duration on the engine's stream, peak 8 TB/s) and "cpu_baseline" (the
reference's own sequential code, oracle/_ref/libhpdga_ref.so, on a bounded sample of the
same workload on this host, 1 thread).  "engine_options" lists the epoch reorganisations the
engine applies (train-ahead, output-layer row restriction, eval's first layer
from Â X computed once; all exact algebra, no work whose result reaches the loss, accuracy or
weights is skipped) and "value_reorganisations_off" times the same epoch with them off.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
# torch before libpgcn.so: its bundled HIP runtime / RCCL (same SONAMEs) then serve both,
# so the process holds one HIP runtime.  torch is only control plumbing here.
import torch  # noqa: F401

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "tests"))

N_NODES, N_FEAT, N_CLASS = 232965, 602, 41
WORKLOADS = {
    # undirected edges (directed slots / 2) -- SURVEY.md §8 / BASELINE.md §1
    "reddit-114M": 57307946,
    "reddit-11.6M": 11606919,
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def load_pkg():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "pgcn_amd", os.path.join(REPO, "parallel-gcn_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["pgcn_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def cpu_baseline(ds, epochs):
    """The reference's sequential epoch (train_epoch + eval(2)) on this host, 1 thread.
    Prefers oracle/_ref (the reference's own sources); falls back to the C restatement."""
    import helpers
    n, f, c = ds.num_nodes, ds.input_dim, ds.output_dim
    args = [ds.graph_indptr, ds.graph_indices, ds.feat_indptr, ds.feat_indices, ds.feat_values,
            ds.label, ds.split]
    ref = helpers.ref_lib()
    times = []
    if ref is not None:
        kind = "reference"
        h = ref.ref_create(n, f, 16, c, 0.5, 0.01, 5e-4, 100, helpers.ptr(args[0]),
                           helpers.ptr(args[1]), int(ds.graph_indptr[-1]), helpers.ptr(args[2]),
                           helpers.ptr(args[3]), helpers.ptr(args[4]), int(ds.feat_indptr[-1]),
                           helpers.ptr(args[5]), helpers.ptr(args[6]))
        out = np.zeros(2, np.float32)
        for _ in range(epochs):
            t0 = time.perf_counter()
            ref.ref_train_epoch(h, helpers.ptr(out))
            ref.ref_eval(h, 2, helpers.ptr(out))
            times.append(time.perf_counter() - t0)
        ref.ref_free(h)
    else:
        kind = "port"
        g = helpers.OracleGCN(helpers.ds_dict(ds))
        for _ in range(epochs):
            t0 = time.perf_counter()
            g.train_epoch()
            g.eval(2)
            times.append(time.perf_counter() - t0)
        del g
    return kind, times


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="reddit-114M", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-epochs", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--edge-cut", action="store_true",
                    help="one GPU through the multi-GPU engine (partition, RCCL at world 1)")
    ap.add_argument("--profile-only", action="store_true",
                    help="only run warmup+steps (for rocprofv3), no JSON extras")
    ap.add_argument("--hidden", default="16",
                    help="hidden dims, comma-separated (BASELINE configs[4]: 128,128,128)")
    ap.add_argument("--no-plain", action="store_true",
                    help="skip the secondary measurement with the epoch reorganisations off")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world != 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dist = None
    # this rank's GPU before anything touches HIP through torch (torch.cuda.synchronize()
    # below would otherwise open a context on GPU 0 from every rank)
    torch.cuda.set_device(local_rank)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    pgcn = load_pkg()
    t_gen = time.perf_counter()
    ds = pgcn.Dataset.synthetic(N_NODES, N_FEAT, N_CLASS, WORKLOADS[args.workload], seed=1)
    t_gen = time.perf_counter() - t_gen
    hidden = tuple(int(h) for h in args.hidden.split(","))
    params = pgcn.make_params(ds, hidden_dims=hidden, dropouts=(0.5,) * (len(hidden) + 1))
    model = (f"{len(hidden) + 1}-layer GCN, hidden={hidden[0]}" if len(set(hidden)) == 1
             else f"{len(hidden) + 1}-layer GCN, hidden={args.hidden}")
    t_build = time.perf_counter()
    if world > 1:
        uid = [pgcn.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        g = pgcn.GCN(params, ds, device=local_rank, rank=rank, world=world, unique_id=uid[0])
    elif args.edge_cut:
        g = pgcn.GCN(params, ds, device=local_rank, rank=0, world=1,
                     unique_id=pgcn.comm_unique_id())
    else:
        g = pgcn.GCN(params, ds, device=local_rank)
    t_build = time.perf_counter() - t_build

    def barrier():
        g.sync()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        g.epoch_async()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g.epoch_async()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = g.results(min(args.steps, 4))

    if args.profile_only:
        if rank == 0:
            print(json.dumps({"elapsed_s": elapsed, "steps": args.steps}))
        return

    # roofline of the dominant kernel: GraphSum, timed with HIP events on the engine stream
    g.profile(True)
    for _ in range(2):
        g.epoch_async()
    gs_ms, gs_calls, gs_bytes = g.profile_read()
    g.profile(False)
    avg_ms = gs_ms / max(gs_calls, 1)
    bytes_per_call = gs_bytes / max(gs_calls, 1)
    achieved = bytes_per_call / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic = None
    tpath = os.path.join(REPO, "profiles", "traffic_graphsum.json")
    if os.path.exists(tpath) and hidden == (16,):  # PMC passes exist for the headline model
        try:
            traffic = json.load(open(tpath)).get(args.workload)
        except Exception:
            traffic = None

    out = {
        "metric": f"training epochs/sec ({model}) on reddit",
        "value": args.steps / elapsed,
        "unit": "epochs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic reddit-shaped (Chung-Lu power-law graph, dense N(0,1) features, seed 1)",
        "config": {"workload": f"{args.workload} {model} dropout=0.5 Adam",
                   "nodes": N_NODES, "features": N_FEAT, "classes": N_CLASS,
                   "adjacency_nnz": int(ds.graph_indptr[-1]),
                   "parallelism": (f"edge-cut x{world}" if world > 1 or args.edge_cut
                                   else "single GPU"),
                   "step": "train_epoch + eval(2)"},
        "roofline": {"kernel": "graphsum", "bound": "hbm", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "avg_call_ms": avg_ms,
                     "algorithmic_bytes_per_call": bytes_per_call, "calls": gs_calls},
        "last_epoch": {"train_loss": float(res[-1, 0]), "train_acc": float(res[-1, 1]),
                       "val_loss": float(res[-1, 2]), "val_acc": float(res[-1, 3])},
        "setup_s": {"generate": t_gen, "build": t_build},
    }
    g.close()
    # the same epoch with the engine's epoch reorganisations off (train-ahead, output-layer
    # row restriction, eval from Â X): every module runs the reference's full
    # per-epoch work, for comparison (same synthetic data, fewer steps)
    opts = {"train_ahead": 1, "split_rows": 1, "eval_ax": 1, "reassociate_last": 1}
    out["engine_options"] = opts
    if not args.no_plain and world == 1 and not args.edge_cut:
        for k in ("train_ahead", "split_rows", "eval_ax"):
            pgcn.lib.pgcn_debug_set(k.encode(), 0)
        g2 = pgcn.GCN(params, ds, device=local_rank)
        steps2 = max(1, min(args.steps, 10))
        for _ in range(2):
            g2.epoch_async()
        g2.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps2):
            g2.epoch_async()
        g2.sync()
        torch.cuda.synchronize()
        el2 = time.perf_counter() - t0
        g2.close()
        for k in ("train_ahead", "split_rows", "eval_ax"):
            pgcn.lib.pgcn_debug_set(k.encode(), 1)
        out["value_reorganisations_off"] = steps2 / el2
        out["reorganisations_off_steps"] = steps2
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        kind, times = cpu_baseline(ds, args.cpu_epochs)
        out["cpu_baseline"] = {"value": len(times) / sum(times), "unit": "epochs/s", "cores": 1,
                               "kind": kind,
                               "sample": f"{len(times)} full epoch(s) (train_epoch + eval(2)) of "
                                         f"{args.workload}, sequential, 1 thread",
                               "host_cpus": os.cpu_count()}
    if rank == 0:
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
