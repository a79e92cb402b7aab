"""One rank of the multi-process peer-exchange test (tests/test_gpu_peer_procs.py).

usage: python peer_worker.py <rank> <world> <port> <spec.json> <out.npz>

Joins a gloo group on 127.0.0.1:<port> (the host channel), builds the edge-cut engine over
peer-mapped memory (pgcn_gcn_create_peer: the peers' receive slots opened with hipIpc handles
exchanged over that channel), runs the spec's epochs and writes its epoch lines, eval(3),
its node range, its rows of the logits and W1."""
import json
import os
import sys

import numpy as np


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    spec = json.load(open(sys.argv[4]))
    out = sys.argv[5]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch  # noqa: F401  (before libpgcn.so: one HIP runtime)
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import helpers
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pg = helpers.pgcn()
    for k, v in spec.get("knobs", {}).items():
        pg.check(pg.lib.pgcn_debug_set(k.encode(), int(v)), k)
    if "synthetic" in spec:
        s = spec["synthetic"]
        ds = pg.Dataset.synthetic(s["n"], s["f"], s["c"], s["edges"], s["seed"])
    else:
        ds = pg.Dataset.load(spec["root"], spec["name"])
    p = pg.make_params(ds)
    g = pg.GCN(p, ds, device=spec.get("device", 0), rank=rank, world=world,
               allgather=pg.torch_allgather())
    info = [g.query(k) for k in ("world", "rank", "comm", "graphsum_lds", "peer_uncached")]
    lines = [g.train_epoch() + g.eval(2) for _ in range(spec["epochs"])]
    for _ in range(spec.get("async", 0)):
        g.epoch_async()
    if spec.get("async", 0):
        lines += [tuple(x) for x in g.results(spec["async"])]
    test = g.eval(3)
    lo, hi = g.node_range()
    logits = g.get_var(g.num_vars() - 1)
    w1 = g.get_var(2)
    calls = g.query("comm_calls")
    g.close()
    np.savez(out, info=np.array(info), lines=np.array(lines, np.float64),
             test=np.array(test, np.float64), range=np.array([lo, hi]), logits=logits, w1=w1,
             calls=np.array([calls]))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
