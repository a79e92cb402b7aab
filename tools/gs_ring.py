"""Ring schedule (graphsum_lds_window 5) vs the window-1 LDS schedule on reddit-114M, d = 16
(run on the GPU box): per-call time with HIP events (prescale + kernel + combine) and the
difference of the two outputs relative to sum_j |coef_ij x_j|.  Prints one JSON object."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

pg = helpers.pgcn()
t0 = time.time()
ds = pg.Dataset.synthetic(232965, 602, 41, int(sys.argv[1]) if len(sys.argv) > 1 else 57307946, 1)
n = ds.num_nodes
ip = np.ascontiguousarray(ds.graph_indptr)
ix = np.ascontiguousarray(ds.graph_indices)
res = {"nnz": int(ip[-1]), "gen_s": time.time() - t0}
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
x = torch.randn(n, 16, device="cuda")
xa = torch.abs(x)
outs = {}
for window in (1, 5, 1, 5):
    pg.lib.pgcn_debug_set(b"graphsum_lds_window", window)
    g = ctypes.c_void_p()
    t1 = time.time()
    pg.check(pg.lib.pgcn_graph_create(n, helpers.ptr(ip), helpers.ptr(ix), ctypes.byref(g)), "g")
    o = torch.empty(n, 16, device="cuda")
    oa = torch.empty(n, 16, device="cuda")
    pg.check(pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), 16,
                                  ctypes.c_void_p(o.data_ptr()), 16, 16, s), "gs")
    torch.cuda.synchronize()
    build_s = time.time() - t1
    pg.lib.pgcn_graphsum(g, ctypes.c_void_p(xa.data_ptr()), 16, ctypes.c_void_p(oa.data_ptr()),
                         16, 16, s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), 16, ctypes.c_void_p(o.data_ptr()),
                             16, 16, s)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    outs[window] = (o.clone(), oa.clone())
    res.setdefault(f"w{window}_ms", []).append(ms)
    res[f"w{window}_build_s"] = build_s
    pg.lib.pgcn_graph_destroy(g)
    print(window, ms, flush=True)
o1, a1 = outs[1]
o5, _ = outs[5]
res["max_diff_over_abs"] = float((torch.abs(o1 - o5) / (a1 + 1e-30)).max())
bytes_call = 4 * (n + 1) + 8 * int(ip[-1]) + 8 * n * 16
for w in (1, 5):
    res[f"w{w}_frac"] = bytes_call / (min(res[f"w{w}_ms"]) * 1e-3) / 8e12
pg.lib.pgcn_debug_set(b"graphsum_lds_window", 1)
print(json.dumps(res))
