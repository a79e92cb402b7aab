"""Per-rank epoch of the edge-cut engine at world W, timed on ONE GPU (diagnostic tool for the
DESIGN.md §6 scaling model; no multi-GPU box needed).

For each world in WORLDS and each rank in RANKS, builds that rank's engine on reddit-114M
with a timing-only communicator (pgcn_debug_gcn_create_solo: the rank's own partition, chunk
graphs, kernels and stream order; a reduce-scatter keeps the rank's own share, an all-reduce
is skipped) and times `steps` reference epochs (train_epoch + eval(2)).  Also reports the
collectives one epoch enqueues and the bytes the rank sends into them (ring algorithm), from
which the model adds the transfer time at an assumed xGMI bus bandwidth.  One JSON line.

usage: python3 tools/rank_epoch.py [worlds=1,2,4,8] [ranks=0] [hidden=16]
"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

pg = helpers.pgcn()
# RANK_KNOBS="rs_chunks=1,...": engine knobs for every engine built here
for kv in filter(None, os.environ.get("RANK_KNOBS", "").split(",")):
    k, v = kv.split("=")
    pg.check(pg.lib.pgcn_debug_set(k.encode(), int(v)), "knob " + k)
worlds = [int(w) for w in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,8").split(",")]
ranks = [int(r) for r in (sys.argv[2] if len(sys.argv) > 2 else "0").split(",")]
hidden = tuple(int(h) for h in (sys.argv[3] if len(sys.argv) > 3 else "16").split(","))
steps = int(os.environ.get("RANK_STEPS", "10"))
warmup = int(os.environ.get("RANK_WARMUP", "2"))  # the clock settles over ~18 epochs
ds = pg.Dataset.synthetic(232965, 602, 41, 57307946, 1)
params = pg.make_params(ds, hidden_dims=hidden, dropouts=(0.5,) * (len(hidden) + 1))
out = {"hidden": list(hidden), "steps": steps, "ranks": {}}
for w in worlds:
    for r in ranks:
        if r >= w:
            continue
        g = pg.GCN(params, ds, device=0, rank=r, world=w, solo=True)
        for _ in range(warmup):
            g.epoch_async()
        g.sync()
        torch.cuda.synchronize()
        c0, b0 = g.query("comm_calls"), g.query("comm_bytes")
        t0 = time.perf_counter()
        for _ in range(steps):
            g.epoch_async()
        g.sync()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        calls = (g.query("comm_calls") - c0) / steps
        mb = (g.query("comm_bytes") - b0) / steps / 1e6
        g.close()
        out["ranks"][f"w{w}r{r}"] = {"ms_per_epoch": dt * 1e3, "collectives_per_epoch": calls,
                                     "sent_mb_per_epoch": mb}
        print(f"world {w} rank {r}: {dt * 1e3:.3f} ms/epoch, {calls:.0f} collectives, "
              f"{mb:.1f} MB sent", file=sys.stderr)
print(json.dumps(out))
