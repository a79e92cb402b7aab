"""Per-rank GraphSum of the edge-cut engine at world N, timed on one GPU (diagnostic tool).

For world in WORLDS, builds rank 0's reduce-scatter chunk graphs of reddit-114M exactly as the
engine does (pgcn_debug_rank_graph: rows world*maxrows/chunks, columns = the rank's nodes) and
times one d = 16 GraphSum call (every chunk) on each kernel path the shape admits:
  * "default"  -- the engine's choice (LDS ring schedule when the rank's table exceeds 4 MB,
                  else the plain gather kernel);
  * "lds"      -- the LDS ring schedule forced (lds_min_kb 0);
  * "plain"    -- the plain gather kernel (lds_min_kb huge).
Prints one JSON object: ms per GraphSum call (all chunks) per (world, path).

usage: python3 tools/rank_graphsum.py [worlds=2,4,8] [chunks=2]
"""
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
worlds = [int(w) for w in (sys.argv[1] if len(sys.argv) > 1 else "2,4,8").split(",")]
chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ds = pg.Dataset.synthetic(232965, 602, 41, 57307946, 1)
n = ds.num_nodes
ip = np.ascontiguousarray(ds.graph_indptr, np.int32)
ix = np.ascontiguousarray(ds.graph_indices, np.int32)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
PATHS = {"default": {}, "lds": {"lds_min_kb": 0}, "plain": {"lds_min_kb": 1 << 30}}
if os.environ.get("RANK_GS_PATHS"):  # e.g. "lds_b8:lds_blocks=8,lds_min_kb=0;lds_b16:lds_blocks=16"
    PATHS = {}
    for item in os.environ["RANK_GS_PATHS"].split(";"):
        name, _, kv = item.partition(":")
        PATHS[name] = {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}


def time_path(world, knobs, reps=20):
    for k, v in knobs.items():
        pg.lib.pgcn_debug_set(k.encode(), v)
    graphs, shapes = [], []
    try:
        for c in range(chunks):
            g, r, cc = ctypes.c_void_p(), ctypes.c_int(), ctypes.c_int()
            pg.check(pg.lib.pgcn_debug_rank_graph(n, helpers.ptr(ip), helpers.ptr(ix), world, 0,
                                                  chunks, c, ctypes.byref(g), ctypes.byref(r),
                                                  ctypes.byref(cc)), "rank_graph")
            graphs.append(g)
            shapes.append((r.value, cc.value))
        x = torch.randn(shapes[0][1], 16, device="cuda")
        outs = [torch.empty(s[0], 16, device="cuda") for s in shapes]

        def call():
            for g, o in zip(graphs, outs):
                pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), 16,
                                     ctypes.c_void_p(o.data_ptr()), 16, 16, st)
        call()  # builds the schedules
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        nnz = sum(pg.lib.pgcn_graph_nnz(g) for g in graphs)
        return e0.elapsed_time(e1) / reps, shapes, nnz
    finally:
        for g in graphs:
            pg.lib.pgcn_graph_destroy(g)
        pg.lib.pgcn_debug_set(b"lds_min_kb", -1)  # the defaults
        pg.lib.pgcn_debug_set(b"lds_blocks", 0)


out = {"chunks": chunks}
for w in worlds:
    row = {}
    for name, knobs in PATHS.items():
        ms, shapes, nnz = time_path(w, knobs)
        row[name + "_ms"] = ms
        row["shapes"] = shapes
        row["nnz"] = int(nnz)
    out[f"world{w}"] = row
    print(w, json.dumps(row), flush=True)
print(json.dumps(out))
