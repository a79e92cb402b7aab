"""Times the d = 16 GraphSum of the reddit-114M bench graph through the C ABI (pgcn_graphsum:
prescale + k_graphsum_ring + combine), HIP events over `calls` back-to-back calls on one
stream.  usage: python3 tools/gs_call.py [calls] [width]; prints one JSON object (GPU box)."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dim = int(sys.argv[2]) if len(sys.argv) > 2 else 16
pg = helpers.pgcn()
ds = pg.Dataset.synthetic(232965, 602, 41, 57307946, 1)
n = ds.num_nodes
ip, ix = ds.graph_indptr, ds.graph_indices
x = torch.randn(n, dim, device="cuda")
o = torch.empty(n, dim, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
g = ctypes.c_void_p()
pg.check(pg.lib.pgcn_graph_create(n, helpers.ptr(ip), helpers.ptr(ix), ctypes.byref(g)), "graph")


def call():
    pg.check(pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), dim,
                                  ctypes.c_void_p(o.data_ptr()), dim, dim, st), "graphsum")


call()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(calls):
    call()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / calls
nnz = int(ip[-1])
algo = 4.0 * (n + 1) + 8.0 * nnz + 8.0 * n * dim
print(json.dumps({"dim": dim, "calls": calls, "ms_per_call": ms,
                  "algorithmic_bytes": algo, "frac_8tbs": algo / (ms * 1e-3) / 8e12}))
pg.lib.pgcn_graph_destroy(g)
