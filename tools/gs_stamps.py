"""In-kernel cycle stamps of k_graphsum_lds (graphsum_lds_diag = 4) on the reddit-shaped graph
(diagnostic tool, GPU box).  Prints per-role averages of loop / barrier / ring-wait cycles."""
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
pg.check(pg.lib.pgcn_graph_create(n, helpers.ptr(ip), helpers.ptr(ix), ctypes.byref(g)), "g")
x = torch.randn(n, 16, device="cuda")
o = torch.empty(n, 16, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
call = lambda: pg.lib.pgcn_graphsum(g, ctypes.c_void_p(x.data_ptr()), 16,  # noqa: E731
                                    ctypes.c_void_p(o.data_ptr()), 16, 16, st)
call()
out = {}
for sync in (1, 0):  # slice hand-off words / a workgroup barrier per slice
    pg.lib.pgcn_debug_set(b"graphsum_lds_sync", sync)
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
    res = {
        "wgs": int(s.shape[0]),
        "sum_loop_cyc_mean": summ[:, :, 0].mean(), "sum_loop_cyc_max": summ[:, :, 0].max(),
        "sum_wait_frac": summ[:, :, 1].sum() / summ[:, :, 0].sum(),
        "sum_ringwait_frac": summ[:, :, 2].sum() / summ[:, :, 0].sum(),
        "blocks_per_wave_mean": summ[:, :, 3].mean(),
        "cyc_per_block_excl_waits": ((summ[:, :, 0] - summ[:, :, 1] - summ[:, :, 2]).sum() /
                                     summ[:, :, 3].sum()),
        "loader_stage_wait_cyc_mean": load[:, 2].mean(), "loader_wait_cyc_mean": load[:, 1].mean(),
        "slices_mean": summ[:, :, 4].mean(),
        "wg_loop_imbalance_max_over_mean": float(summ[:, :, 0].max(1).max() /
                                                 summ[:, :, 0].max(1).mean()),
    }
    out["flags" if sync else "barriers"] = res
pg.lib.pgcn_debug_set(b"graphsum_lds_sync", 1)
print(json.dumps(out))
