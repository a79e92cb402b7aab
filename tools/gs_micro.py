"""GraphSum ablation micro-benchmark on the reddit-shaped graph (run on the GPU box).

Times pgcn_graphsum (kernel + combine) per call with HIP events on torch's stream for:
dim 16 (blocked schedule), the same without XCD column blocking, no-gather and folded-table
ablations, and dim 32 (128-B rows).  Prints one JSON object.
"""
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
edges = 57307946
ONLY = sys.argv[1] if len(sys.argv) > 1 else None  # run one configuration (for PMC passes)
t0 = time.time()
ds = pg.Dataset.synthetic(232965, 602, 41, edges, 1)
n = ds.num_nodes
ip = np.ascontiguousarray(ds.graph_indptr)
ix = np.ascontiguousarray(ds.graph_indices)
gen_s = time.time() - t0


def make_graph():
    g = ctypes.c_void_p()
    pg.check(pg.lib.pgcn_graph_create(n, helpers.ptr(ip), helpers.ptr(ix), ctypes.byref(g)), "g")
    return g


def timeit(g, dim, reps=10):
    ld = (dim + 3) // 4 * 4
    x = torch.randn(n, ld, device="cuda")
    o = torch.empty(n, ld, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(2):
        pg.check(pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), ld,
                                      ctypes.c_void_p(o.data_ptr()), ld, dim, s), "gs")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), ld, ctypes.c_void_p(o.data_ptr()),
                             ld, dim, s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {"nnz": int(ip[-1]), "gen_s": gen_s}
if ONLY:
    variant = {"nogather": 1, "table4096": 2}.get(ONLY, 0)
    if ONLY == "v3":
        pg.lib.pgcn_debug_set(b"graphsum_lds", 0)
    if ONLY == "plain":
        pg.lib.pgcn_debug_set(b"graphsum_plain", 1)
    pg.lib.pgcn_debug_set(b"graphsum_variant", variant)
    g = make_graph()
    res[ONLY + "_ms"] = timeit(g, 32 if ONLY == "d32" else 16, reps=5)
    print(json.dumps(res))
    sys.exit(0)
g = make_graph()
ld = 16
x = torch.randn(n, ld, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run_once(dim=16):
    o = torch.empty(n, ld, device="cuda")
    pg.check(pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), ld,
                                  ctypes.c_void_p(o.data_ptr()), ld, dim, st), "gs")
    torch.cuda.synchronize()
    return o


t1 = time.time()
o_lds = run_once()
res["lds_build_plus_first_call_s"] = time.time() - t1
res["d16_lds_ms"] = timeit(g, 16)
pg.lib.pgcn_debug_set(b"graphsum_lds_sync", 0)
res["d16_lds_barriers_ms"] = timeit(g, 16)
res["d16_lds_again_ms"] = timeit(g, 16)
pg.lib.pgcn_debug_set(b"graphsum_lds_sync", 1)
res["d16_lds_flags_again_ms"] = timeit(g, 16)

# window 2 (two-slot runs, exec-masked adds) on a fresh graph
pg.lib.pgcn_debug_set(b"graphsum_lds_window", 2)
g2 = make_graph()
o_w2 = torch.empty(n, ld, device="cuda")
pg.check(pg.lib.pgcn_graphsum(g2, ctypes.c_void_p(x.data_ptr()), ld,
                              ctypes.c_void_p(o_w2.data_ptr()), ld, 16, st), "gs")
torch.cuda.synchronize()
res["d16_lds_window2_ms"] = timeit(g2, 16)
pg.lib.pgcn_debug_set(b"graphsum_lds_diag", 6)
res["d16_lds_window2_notouch_ms"] = timeit(g2, 16)
pg.lib.pgcn_debug_set(b"graphsum_lds_diag", 0)
res["window2_vs_window1_max_rel"] = ((o_w2 - o_lds).abs().max() / o_lds.abs().max()).item()
pg.lib.pgcn_debug_set(b"graphsum_lds_window", 1)
for dg, name in ((1, "stage1of16"), (2, "noreads"), (3, "oneadd")):
    pg.lib.pgcn_debug_set(b"graphsum_lds_diag", dg)
    res[f"d16_lds_{name}_ms"] = timeit(g, 16)
pg.lib.pgcn_debug_set(b"graphsum_lds_diag", 0)
pg.lib.pgcn_debug_set(b"graphsum_lds", 0)
o_v3 = run_once()
res["d16_v3_ms"] = timeit(g, 16)
rel = ((o_lds - o_v3).abs().max() / o_v3.abs().max()).item()
res["lds_vs_v3_max_rel"] = rel
print(json.dumps(res))
