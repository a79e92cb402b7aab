"""Rank body of the world-size-2 gloo test (tests/test_dist_gloo.py).

Restates, in numpy on CPU, the edge-cut schedule the C++ engine runs over RCCL
(csrc/host/comm.cpp, csrc/host/gcn.cpp dist branch), using the PRODUCT's partition plan
(pgcn_partition_bounds / pgcn_partition_subgraph):
  * every rank owns a contiguous nnz-balanced node range [lo, hi);
  * GraphSum: partial = (rank's column block of Â, padded rows) x V[lo:hi], then a
    reduce-scatter over the padded row blocks (gloo has no reduce_scatter for CPU tensors:
    all_reduce + own slice, same arithmetic);
  * loss / wrong-count scalars and weight gradients: all_reduce.
"""
import os

import numpy as np


def _graphsum(dist, torch, sub, v_loc, rank, maxrows, nloc):
    part = torch.from_numpy(np.ascontiguousarray(sub @ v_loc))
    dist.all_reduce(part)
    return part.numpy()[rank * maxrows:rank * maxrows + nloc]


def run(rank, world, port, root, name, shared, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import scipy.sparse as sps
    import torch
    import torch.distributed as dist
    import helpers
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pg = helpers.pgcn()
        ds = pg.Dataset.load(root, name)
        n, f, c = ds.num_nodes, ds.input_dim, ds.output_dim
        w1, w2 = shared["w1"].astype(np.float64), shared["w2"].astype(np.float64)
        h = w1.shape[1]
        b, maxrows = pg.partition_bounds(ds.graph_indptr, world)
        lo, hi = int(b[rank]), int(b[rank + 1])
        nloc = hi - lo
        sp_, si, sv = pg.partition_subgraph(ds.graph_indptr, ds.graph_indices, world, rank)
        sub = sps.csr_matrix((sv.astype(np.float64), si, sp_), shape=(world * maxrows, nloc))
        x = sps.csr_matrix((ds.feat_values.astype(np.float64), ds.feat_indices, ds.feat_indptr),
                           shape=(n, f))[lo:hi]
        label, split = ds.label[lo:hi], ds.split[lo:hi]
        gs = lambda v: _graphsum(dist, torch, sub, v, rank, maxrows, nloc)  # noqa: E731

        def forward(which):
            z1 = np.asarray(x @ w1)
            a1 = gs(z1)
            hid = np.maximum(a1, 0)
            logits = gs(hid @ w2)
            truth = np.where(split == which, label, -1)
            lab = truth >= 0
            lg = logits[lab]
            m = lg.max(1, keepdims=True)
            lse = np.log(np.exp(lg - m).sum(1)) + m[:, 0]
            nll = lse - lg[np.arange(lg.shape[0]), truth[lab]]
            wrong = (lg > lg[np.arange(lg.shape[0]), truth[lab]][:, None]).any(1)
            s = torch.tensor([nll.sum(), float(lab.sum()), float(wrong.sum())], dtype=torch.float64)
            dist.all_reduce(s)
            total, count, nwrong = s.tolist()
            return dict(z1=z1, a1=a1, hid=hid, logits=logits, truth=truth, lab=lab,
                        loss=total / count, count=count, acc=1 - nwrong / count)

        l2 = 5e-4 * float((shared["w1"].astype(np.float64) ** 2).sum()) / 2
        ev = forward(2)
        tr = forward(1)
        # backward (training split, no dropout): d logits = (softmax - onehot) / global count
        lg = tr["logits"]
        p = np.exp(lg - lg.max(1, keepdims=True))
        p /= p.sum(1, keepdims=True)
        p[tr["lab"], tr["truth"][tr["lab"]]] -= 1.0
        p[~tr["lab"]] = 0.0
        dout = p / tr["count"]
        dz2 = gs(dout)  # Â symmetric: the backward GraphSum is the same edge-cut op
        gw2 = torch.from_numpy(tr["hid"].T @ dz2)
        dhid = (dz2 @ w2.T) * (tr["a1"] > 0)
        dz1 = gs(dhid)
        gw1 = torch.from_numpy(np.asarray(x.T @ dz1))
        dist.all_reduce(gw1)
        dist.all_reduce(gw2)
        if rank == 0:
            np.savez(os.path.join(out_dir, "dist.npz"), eval_loss=ev["loss"] + l2,
                     eval_acc=ev["acc"], eval_count=ev["count"], train_loss=tr["loss"] + l2,
                     gw1=gw1.numpy(), gw2=gw2.numpy(), h=h)
    finally:
        dist.destroy_process_group()
