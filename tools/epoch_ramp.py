#!/usr/bin/env python3
"""Per-epoch wall times of the headline engine from its first epoch on (reddit-114M, 2-layer
H 16): where the "first ~15 epochs are slower" ramp of the bench window comes from.

Phases (each epoch: epoch_async + sync, host wall clock):
  cold    -- right after the engine build
  idle    -- after 2 s of host sleep (the GPU idles)
  busy    -- after ~300 ms of unrelated GPU work (torch matmuls) with no idle gap
Prints one JSON object."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import bench  # noqa: E402


def epochs(g, n):
    out = []
    for _ in range(n):
        t0 = time.perf_counter()
        g.epoch_async()
        g.sync()
        out.append((time.perf_counter() - t0) * 1e3)
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    torch.cuda.set_device(0)
    pgcn = bench.load_pkg()
    ds = pgcn.Dataset.synthetic(bench.N_NODES, bench.N_FEAT, bench.N_CLASS,
                                bench.WORKLOADS["reddit-114M"], seed=1)
    g = pgcn.GCN(pgcn.make_params(ds), ds, device=0)
    res = {"cold": epochs(g, n)}
    time.sleep(2.0)
    res["idle"] = epochs(g, n)
    a = torch.randn(4096, 4096, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        a = (a @ a).clamp_(-1, 1)
    torch.cuda.synchronize()
    res["busy"] = epochs(g, n)
    g.close()
    summ = {k: {"first5": sum(v[:5]) / 5, "last10": sum(v[-10:]) / 10} for k, v in res.items()}
    print(json.dumps({"ms": res, "summary": summ}))


if __name__ == "__main__":
    main()
