"""GraphSum d=16 LDS kernel option sweep on the reddit-shaped graph (diagnostic tool, GPU box).

For each schedule window (env GS_WINDOWS, default "1") and each value of the
"graphsum_lds_opt" knob (argv, default 3): the per-call time (prescale + k_graphsum_lds +
combine, HIP events on torch's stream, 10 calls), the max relative difference against the
v3 TA-gather kernel (a different summation order: ~1e-6 expected), and the in-kernel cycle
stamps (graphsum_lds_diag = 4).  Prints one JSON object.
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
ds = pg.Dataset.synthetic(232965, 602, 41, 57307946, 1)
n = ds.num_nodes
ip, ix = np.ascontiguousarray(ds.graph_indptr), np.ascontiguousarray(ds.graph_indices)
g = ctypes.c_void_p()
x = torch.randn(n, 16, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def call(o):
    pg.check(pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), 16,
                                  ctypes.c_void_p(o.data_ptr()), 16, 16, st), "gs")


def timeit(reps=10):
    o = torch.empty(n, 16, device="cuda")
    call(o)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call(o)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def stamps():
    o = torch.empty(n, 16, device="cuda")
    pg.lib.pgcn_debug_set(b"graphsum_lds_diag", 4)
    call(o)
    call(o)
    torch.cuda.synchronize()
    pg.lib.pgcn_debug_set(b"graphsum_lds_diag", 0)
    cnt = pg.lib.pgcn_debug_read(b"graphsum_lds_stamps", None, 0)
    buf = np.zeros(cnt, np.uint64)
    pg.lib.pgcn_debug_read(b"graphsum_lds_stamps", buf.ctypes.data_as(ctypes.c_void_p), cnt)
    s = buf.reshape(-1, 16, 8).astype(np.float64)
    summ, load = s[:, :15], s[:, 15]
    return {"sum_loop_cyc_mean": summ[:, :, 0].mean(),
            "sum_wait_frac": summ[:, :, 1].sum() / summ[:, :, 0].sum(),
            "loader_stage_wait_cyc_mean": load[:, 2].mean(),
            "loader_done_wait_cyc_mean": load[:, 1].mean(),
            "blocks_per_wave_mean": summ[:, :, 3].mean()}


res = {}
o_ref = torch.empty(n, 16, device="cuda")
windows = [int(w) for w in os.environ.get("GS_WINDOWS", "1").split()]
blocks = [int(b) for b in os.environ.get("GS_BLOCKS", "0").split()]  # 0: by shape
configs = [(w, b) for w in windows for b in blocks]
for wi, (window, nblk) in enumerate(configs):
    # a fresh graph per configuration: the LDS schedule is built at its first d = 16 call
    pg.lib.pgcn_debug_set(b"graphsum_lds_window", window)
    pg.lib.pgcn_debug_set(b"lds_blocks", nblk)
    if g.value:
        pg.lib.pgcn_graph_destroy(g)
    pg.check(pg.lib.pgcn_graph_create(n, helpers.ptr(ip), helpers.ptr(ix), ctypes.byref(g)), "g")
    if wi == 0:
        pg.lib.pgcn_debug_set(b"graphsum_lds", 0)
        call(o_ref)
        torch.cuda.synchronize()
        pg.lib.pgcn_debug_set(b"graphsum_lds", 1)
    for opt in [int(a) for a in (sys.argv[1:] or ["3"])]:
        pg.lib.pgcn_debug_set(b"graphsum_lds_opt", opt)
        o = torch.empty(n, 16, device="cuda")
        call(o)
        torch.cuda.synchronize()
        r = {"ms": timeit(), "max_rel_vs_v3": ((o - o_ref).abs().max() / o_ref.abs().max()).item()}
        r["ms_again"] = timeit()
        r.update(stamps())
        res[f"w{window}_b{nblk}_opt{opt}"] = r
        print(json.dumps({f"w{window}_b{nblk}_opt{opt}": r}), file=sys.stderr, flush=True)
# ablations (window 1 schedule, timing only): DIAG 1 = 1/16 of each slice staged, 2 = no table
# reads, 3 = one add per read, 5 = 1 + 2, 7 = 5 without the entry stream
diags = [int(d) for d in os.environ.get("GS_DIAGS", "").split()]
if diags:
    pg.lib.pgcn_debug_set(b"graphsum_lds_window", 1)
    pg.lib.pgcn_graph_destroy(g)
    pg.check(pg.lib.pgcn_graph_create(n, helpers.ptr(ip), helpers.ptr(ix), ctypes.byref(g)), "g")
    o = torch.empty(n, 16, device="cuda")
    call(o)
    res["w1_base_ms"] = timeit()
    for d in diags:
        pg.lib.pgcn_debug_set(b"graphsum_lds_diag", d)
        res[f"w1_diag{d}_ms"] = timeit()
    pg.lib.pgcn_debug_set(b"graphsum_lds_diag", 0)
    res["w1_base_again_ms"] = timeit()
print(json.dumps(res))
