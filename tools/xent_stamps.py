"""Phase timeline of the loss kernel (diagnostic; needs a library built with
-DPGCN_XENT_STAMPS, e.g. scripts/build_ab.sh ab_xst -DPGCN_XENT_STAMPS, loaded by PGCN_LIB).

Runs the bench's reddit-114M 2-layer engine, then one train_epoch and one eval(2), reading the
per-wave stamps after each: shader-clock cycles between the phase boundaries (median and p90
over waves) and the wall-clock spread of wave starts / ends within the launch."""
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
fn = pg.lib.pgcn_debug_xent_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
ds = pg.Dataset.synthetic(232965, 602, 41, 57307946, 1)
params = pg.make_params(ds, hidden_dims=(16,), dropouts=(0.5, 0.5))
g = pg.GCN(params, ds, device=0)
for _ in range(3):
    g.train_epoch()
    g.eval(2)
names = ["start", "W staged", "logits in tile", "softmax", "logits out", "grad in tile",
         "dH", "dWp + grad out", "partials", "end"]
out = {}
for tag, run in (("train", g.train_epoch), ("eval", lambda: g.eval(2))):
    run()
    torch.cuda.synchronize()
    buf = np.zeros(16384 * 12, np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    st = buf.reshape(16384, 12).astype(np.int64)
    st = st[st[:, 0] != 0]
    res = {"waves": int(len(st))}
    for k in range(1, 10):
        d = st[:, k] - st[:, k - 1]
        ok = (st[:, k] != 0) & (st[:, k - 1] != 0)
        if ok.any():
            res[f"{names[k - 1]} -> {names[k]}"] = [int(np.median(d[ok])), int(np.percentile(d[ok], 90))]
    tot = st[:, 9] - st[:, 0]
    res["total cycles med/p90"] = [int(np.median(tot)), int(np.percentile(tot, 90))]
    w0, w1 = st[:, 10], st[:, 11]  # 100 MHz wall clock
    t0 = w0.min()
    res["launch span us"] = float((w1.max() - t0) / 100.0)
    res["wave start us p10/p50/p90"] = [float(np.percentile(w0 - t0, p) / 100.0) for p in (10, 50, 90)]
    res["wave life us med"] = float(np.median(w1 - w0) / 100.0)
    hist = np.histogram((w0 - t0) / 100.0, bins=10)
    res["start histogram"] = [int(x) for x in hist[0]]
    res["start bins us"] = [round(float(x), 1) for x in hist[1]]
    out[tag] = res
g.close()
print(json.dumps(out, indent=1))
