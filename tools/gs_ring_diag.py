"""Ring schedule diagnostics on reddit-114M, d = 16 (GPU box): per-call time of the ring
kernel (window 5) and of its timing-only ablations (graphsum_lds_diag 1: no table reads;
2: the loader stages 1/8 of each slice), and the in-kernel cycle stamps (diag 4).
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
window = int(os.environ.get("RING_WINDOW", "5"))
ds = pg.Dataset.synthetic(232965, 602, 41, 57307946, 1)
n = ds.num_nodes
ip, ix = np.ascontiguousarray(ds.graph_indptr), np.ascontiguousarray(ds.graph_indices)
pg.lib.pgcn_debug_set(b"graphsum_lds_window", window)
g = ctypes.c_void_p()
pg.check(pg.lib.pgcn_graph_create(n, helpers.ptr(ip), helpers.ptr(ix), ctypes.byref(g)), "g")
x = torch.randn(n, 16, device="cuda")
o = torch.empty(n, 16, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def call():
    pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), 16, ctypes.c_void_p(o.data_ptr()),
                         16, 16, st)


def timed(reps=20):
    call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


out = {"window": window}
ref = None
for pipe in [int(x) for x in os.environ.get("RING_PRIOS", "1,0").split(",")]:
    pg.lib.pgcn_debug_set(b"graphsum_ring_prio", pipe)
    for diag in [int(d) for d in os.environ.get("RING_DIAGS", "0,1,2,0").split(",")]:
        pg.lib.pgcn_debug_set(b"graphsum_lds_diag", diag)
        out[f"prio{pipe}_diag{diag}_ms"] = timed()
    pg.lib.pgcn_debug_set(b"graphsum_lds_diag", 0)
    call()
    torch.cuda.synchronize()
    if ref is None:
        ref = o.clone()
    else:  # both loops add the same rows in the same order per accumulator
        out["prio_max_abs_diff"] = float(torch.abs(o - ref).max())
pg.lib.pgcn_debug_set(b"graphsum_ring_prio", int(os.environ.get("RING_PRIO", "1")))
pg.lib.pgcn_debug_set(b"graphsum_lds_diag", 4)
call()
call()
torch.cuda.synchronize()
pg.lib.pgcn_debug_set(b"graphsum_lds_diag", 0)
cnt = pg.lib.pgcn_debug_read(b"graphsum_lds_stamps", None, 0)
buf = np.zeros(cnt, np.uint64)
pg.lib.pgcn_debug_read(b"graphsum_lds_stamps", buf.ctypes.data_as(ctypes.c_void_p), cnt)
s = buf.reshape(-1, 16, 8).astype(np.float64)
summ, load = s[:, :15], s[:, 15]
out.update({
    "wgs": int(s.shape[0]),
    "sum_loop_cyc_mean": summ[:, :, 0].mean(), "sum_loop_cyc_max": summ[:, :, 0].max(),
    "sum_handoff_wait_frac": summ[:, :, 1].sum() / summ[:, :, 0].sum(),
    "sum_ring_wait_frac": summ[:, :, 2].sum() / summ[:, :, 0].sum(),
    "blocks_per_wave_mean": summ[:, :, 3].mean(),
    "cyc_per_block_excl_waits": ((summ[:, :, 0] - summ[:, :, 1] - summ[:, :, 2]).sum() /
                                 summ[:, :, 3].sum()),
    "loader_free_wait_cyc_mean": load[:, 1].mean(), "loader_land_wait_cyc_mean": load[:, 2].mean(),
    "visits": summ[:, :, 4].mean(),
    "wg_loop_max_over_mean": float(summ[:, :, 0].max(1).max() / summ[:, :, 0].max(1).mean()),
    "per_wave_wait_frac": [round(float(x), 3) for x in
                           (summ[:, :, 1].sum(0) / summ[:, :, 0].sum(0))],
    "per_wave_blocks": [round(float(x), 1) for x in summ[:, :, 3].mean(0)],
    "per_wave_cyc_per_block": [round(float(x), 1) for x in
                               ((summ[:, :, 0] - summ[:, :, 1]).sum(0) / summ[:, :, 3].sum(0))],
})
pg.lib.pgcn_debug_set(b"graphsum_lds_window", 1)
print(json.dumps(out))
