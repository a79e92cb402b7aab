"""Diagnostic: per-variable max relative deviation from the oracle after one training epoch
(and after eval) for a dataset + hidden width.  usage: tools/var_diff.py name hidden [seed]"""
import os
import sys
import tempfile

import numpy as np
import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

name, hidden = sys.argv[1], int(sys.argv[2])
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 0
pg = helpers.pgcn()
for knob in (b"split_rows",):
    pg.lib.pgcn_debug_set(knob, 0)
with tempfile.TemporaryDirectory() as root:
    ds = pg.Dataset.load(root, helpers.materialize_dataset(name, root))
    p = pg.make_params(ds, hidden_dims=(hidden,), dropouts=(0.6, 0.6), seed=seed,
                       reassociate_last=False)
    g = pg.GCN(p, ds)
    ref = helpers.OracleGCN(helpers.ds_dict(ds), hidden_dims=(hidden,), dropouts=(0.6, 0.6),
                            seed=seed)
    print("train", g.train_epoch(), ref.train_epoch())
    for i in range(g.num_vars()):
        for w in (0, 1):
            a = np.asarray(g.get_var(i, w), np.float64)
            b = np.asarray(ref.var(i, w), np.float64).ravel()[: a.size]
            if a.size == 0 or b.size == 0:
                continue
            d = np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)
            print(f"var {i} {'grad' if w else 'data'} n={a.size} maxrel={d:.3e}")
    print("eval", g.eval(2), ref.eval(2))
    for i in range(g.num_vars()):
        a = np.asarray(g.get_var(i, 0), np.float64)
        b = np.asarray(ref.var(i, 0), np.float64).ravel()[: a.size]
        if a.size:
            print(f"eval var {i} maxrel={np.abs(a - b).max() / max(np.abs(b).max(), 1e-30):.3e}")
