"""A/B of GraphSum schedule knobs on the reddit bench graphs (diagnostic tool, GPU box):
per arm, a graph built with that arm's knobs (pgcn_graph_create; the LDS schedule is built at
its first call), then the arms timed interleaved -- rounds x (arm A calls, arm B calls, ...)
with HIP events over `calls` back-to-back calls each -- and every arm's output compared with
the first arm's (max |diff| relative to the row's magnitude).

usage: python3 tools/gs_ab.py <workload: 114M|11.6M> <dim> <arm> [<arm> ...]
arm: name=knob:value,knob:value (e.g. base=ring_pair:0 pair=ring_pair:1).  One JSON line."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

EDGES = {"114M": 57307946, "11.6M": 11606919}
wl, dim = sys.argv[1], int(sys.argv[2])
arms = []
for a in sys.argv[3:]:
    name, _, kv = a.partition("=")
    arms.append((name, [(k, int(v)) for k, v in (x.split(":") for x in kv.split(",") if x)]))
calls, rounds = int(os.environ.get("GS_CALLS", "10")), int(os.environ.get("GS_ROUNDS", "3"))
pg = helpers.pgcn()
ds = pg.Dataset.synthetic(232965, 2, 41, EDGES[wl], 1)
n = ds.num_nodes
ip, ix = ds.graph_indptr, ds.graph_indices
ld = (dim + 3) // 4 * 4
x = torch.randn(n, ld, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
graphs, outs = [], []
for name, knobs in arms:
    with helpers.knobs(pg, **dict(knobs)):
        g = ctypes.c_void_p()
        pg.check(pg.lib.pgcn_graph_create(n, helpers.ptr(ip), helpers.ptr(ix), ctypes.byref(g)),
                 "graph")
        o = torch.zeros(n, ld, device="cuda")
        pg.check(pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), ld,
                                      ctypes.c_void_p(o.data_ptr()), ld, dim, st), "graphsum")
        torch.cuda.synchronize()
    graphs.append(g)
    outs.append(o)
mag = (x[:, :dim].abs().mean() * torch.from_numpy((ip[1:] - ip[:-1]).astype("float32")).cuda()
       .sqrt()[:, None])
times = {name: [] for name, _ in arms}
for _ in range(rounds):
    for (name, _), g, o in zip(arms, graphs, outs):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(calls):
            pg.check(pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), ld,
                                          ctypes.c_void_p(o.data_ptr()), ld, dim, st), "gs")
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / calls * 1e3)
nnz = int(ip[-1])
algo = 4.0 * (n + 1) + 8.0 * nnz + 8.0 * n * dim
res = {"workload": wl, "dim": dim, "calls": calls, "rounds": rounds, "arms": {}}
for (name, knobs), o in zip(arms, outs):
    us = sorted(times[name])
    res["arms"][name] = {"knobs": dict(knobs), "us_per_call": us, "median_us": us[len(us) // 2],
                         "frac_8tbs": algo / (us[len(us) // 2] * 1e-6) / 8e12,
                         "max_rel_diff_vs_first": float(((o[:, :dim] - outs[0][:, :dim]).abs()
                                                         / (mag + 1e-30)).max())}
print(json.dumps(res))
for g in graphs:
    pg.lib.pgcn_graph_destroy(g)
