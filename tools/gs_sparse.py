"""d = 16 GraphSum on the report-comparable reddit-11.6M graph (232,965 nodes, 11.6 M undirected edges)
through the C ABI, per path: the ring (default), the plain gather kernels with their per-XCD
column blocks (k_graphsum16, and k_graphsum<4, 16> with interleaved neighbour slots: knob
gs16_gather 1 / 2).  HIP events over
`calls` back-to-back calls; each path on a fresh graph object (schedules are cached per graph).
usage: python3 tools/gs_sparse.py [calls] [undirected_edges]; one JSON line (GPU box)."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
edges = int(sys.argv[2]) if len(sys.argv) > 2 else 11606919
pg = helpers.pgcn()
ds = pg.Dataset.synthetic(232965, 16, 41, edges, 1)
n = ds.num_nodes
ip, ix = ds.graph_indptr, ds.graph_indices
x = torch.randn(n, 16, device="cuda")
o = torch.empty(n, 16, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
PATHS = {"ring": {}, "plain_blocked": {"lds_min_kb": 1 << 30, "gs16_gather": 1},
         "plain_blocked_interleaved": {"lds_min_kb": 1 << 30, "gs16_gather": 2}}
out = {"nodes": n, "nnz": int(ip[-1]), "calls": calls}
ref = None
for name, kn in PATHS.items():
    with helpers.knobs(pg, **kn):
        g = ctypes.c_void_p()
        pg.check(pg.lib.pgcn_graph_create(n, helpers.ptr(ip), helpers.ptr(ix), ctypes.byref(g)),
                 "graph")

        def call():
            pg.check(pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), 16,
                                          ctypes.c_void_p(o.data_ptr()), 16, 16, st), "graphsum")

        call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(calls):
            call()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_us"] = e0.elapsed_time(e1) * 1e3 / calls
        res = o.clone()
        if ref is None:
            ref = res
        out[name + "_maxdiff"] = float((res - ref).abs().max())
        pg.lib.pgcn_graph_destroy(g)
print(json.dumps(out))
