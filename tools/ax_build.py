"""Device time of the eval_ax precompute (Â X over reddit-114M's 602 columns: 38 d = 16
GraphSums) in three engines built one after another in one process (GPU box): the first build
runs on a GPU that has been idle through the host-side data generation.  One JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

pg = helpers.pgcn()
ds = pg.Dataset.synthetic(232965, 602, 41, 57307946, 1)
params = pg.make_params(ds)
out = []
for i in range(3):
    g = pg.GCN(params, ds)
    out.append(g.query("eval_ax_us") / 1000.0)
    if i == 1:  # a few epochs between builds: the clocks stay up
        for _ in range(5):
            g.epoch_async()
        g.sync()
    g.close()
print(json.dumps({"eval_ax_build_ms": out}))
