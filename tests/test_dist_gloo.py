"""World-size-2 (gloo, CPU) check of the edge-cut decomposition the multi-GPU engine uses.

Two processes each own one contiguous nnz-balanced node range of cora, build their column
block of Â with the product's partition plan, and run the 2-layer GCN forward (eval and
train splits) and backward through GraphSum partials + reduce-scatter and all-reduced
scalars / weight gradients (tests/dist_worker.py).  The result must equal the single-process
oracle (the reference's sequential algorithm) at the same initial weights: losses rtol 1e-5,
accuracy exact, weight gradients rtol 1e-4 (fp64 numpy vs the oracle's fp32)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

import dist_worker
import helpers


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_edge_cut_world2_matches_oracle(datasets, loaded, tmp_path):
    root, names = datasets
    ds = loaded["cora"]
    orc = helpers.OracleGCN(helpers.ds_dict(ds), dropouts=(0.0, 0.0))
    shared = {"w1": orc.var(2).reshape(ds.input_dim, 16), "w2": orc.var(5).reshape(16, ds.output_dim)}
    ev = orc.eval(2)
    tr = orc.train_epoch()  # dropout p = 0: the mask keeps everything, grads are the pure ones
    gw1, gw2 = orc.var(2, 1), orc.var(5, 1)

    mp.start_processes(dist_worker.run, args=(2, _free_port(), root, names["cora"], shared,
                                              str(tmp_path)),
                       nprocs=2, join=True, start_method="spawn")
    got = np.load(os.path.join(tmp_path, "dist.npz"))
    np.testing.assert_allclose(got["eval_loss"], ev[0], rtol=1e-5)
    assert abs(got["eval_acc"] - ev[1]) * got["eval_count"] < 0.5
    np.testing.assert_allclose(got["train_loss"], tr[0], rtol=1e-5)
    np.testing.assert_allclose(got["gw2"].ravel(), gw2, rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(got["gw1"].ravel(), gw1, rtol=1e-4, atol=1e-7)
