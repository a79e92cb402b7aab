"""Ring schedule knob sweep on reddit-114M, d = 16 (GPU box): per-call GraphSum time for
(ring_spread, ring_balance, graphsum_ring_prio) settings given as argv triples "s,b,p".
Prints one JSON object."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

pg = helpers.pgcn()
ds = pg.Dataset.synthetic(232965, 602, 41, 57307946, 1)
n = ds.num_nodes
ip, ix = np.ascontiguousarray(ds.graph_indptr), np.ascontiguousarray(ds.graph_indices)
x = torch.randn(n, 16, device="cuda")
o = torch.empty(n, 16, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
pg.lib.pgcn_debug_set(b"graphsum_lds_window", 5)
out = {}
for cfg in sys.argv[1:]:
    vals = [int(v) for v in cfg.split(",")]
    s, b, p = vals[:3]
    pg.lib.pgcn_debug_set(b"ring_spread", s)
    pg.lib.pgcn_debug_set(b"ring_balance", b)
    pg.lib.pgcn_debug_set(b"graphsum_ring_prio", p)
    g = ctypes.c_void_p()
    pg.check(pg.lib.pgcn_graph_create(n, helpers.ptr(ip), helpers.ptr(ix), ctypes.byref(g)), "g")

    def call():
        pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), 16, ctypes.c_void_p(o.data_ptr()),
                             16, 16, st)
    call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        call()
    e1.record()
    torch.cuda.synchronize()
    out[cfg] = e0.elapsed_time(e1) / 20
    print(cfg, out[cfg], flush=True)
    pg.lib.pgcn_graph_destroy(g)
print(json.dumps(out))
