"""The edge-cut engine at world 2 over RCCL (rank r on GPU r), against the single-GPU engine.
Needs two GPUs: RCCL refuses two ranks on one device ("Duplicate GPU detected", measured on
the one-GPU box, r01), so on one GPU the N > 1 path is covered by the gloo restatement
(tests/test_dist_gloo.py) and the world-1 RCCL engine tests only.

usage: python3 tools/rccl_world2.py [--dataset cora|synthetic] [--epochs 5]
The parent starts two rank processes (this file with --rank), rank 0 writes the RCCL unique
id to a file that rank 1 reads; each rank runs train_epoch + eval(2) and saves its lines.
The parent prints the lines next to the single-process reference and exits 1 when the
losses differ by more than 1e-4 relative.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def load(pg, args, root):
    import helpers
    if args.dataset == "synthetic":
        return pg.Dataset.synthetic(60000, 32, 8, 1500000, 4)
    return pg.Dataset.load(root, helpers.materialize_dataset(args.dataset, root))


def rank_main(args):
    import torch  # noqa: F401
    import helpers
    pg = helpers.pgcn()
    with tempfile.TemporaryDirectory() as root:
        ds = load(pg, args, root)
        uid_path = os.path.join(args.dir, "uid")
        if args.rank == 0:
            with open(uid_path + ".tmp", "wb") as f:
                f.write(pg.comm_unique_id())
            os.rename(uid_path + ".tmp", uid_path)
        t0 = time.time()
        while not os.path.exists(uid_path):
            if time.time() - t0 > 60:
                sys.exit("no unique id")
            time.sleep(0.1)
        uid = open(uid_path, "rb").read()
        g = pg.GCN(pg.make_params(ds), ds, device=args.rank, rank=args.rank, world=2,
                   unique_id=uid)
        lines = [g.train_epoch() + g.eval(2) for _ in range(args.epochs)]
        for _ in range(3):
            g.epoch_async()
        lines += [tuple(r) for r in g.results(3)]
        np.save(os.path.join(args.dir, f"rank{args.rank}.npy"), np.array(lines, np.float64))
        g.close()


def parent_main(args):
    import helpers
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, __file__, "--rank", str(r), "--dir", d,
                                   "--dataset", args.dataset, "--epochs", str(args.epochs)])
                 for r in (0, 1)]
        rcs = [p.wait(timeout=240) for p in procs]
        if any(rcs):
            print("rank exit codes", rcs)
            sys.exit(2)
        ranks = [np.load(os.path.join(d, f"rank{r}.npy")) for r in (0, 1)]
    import torch  # noqa: F401
    pg = helpers.pgcn()
    with tempfile.TemporaryDirectory() as root:
        ds = load(pg, args, root)
        g = pg.GCN(pg.make_params(ds), ds, device=0)
        single = [g.train_epoch() + g.eval(2) for _ in range(args.epochs)]
        for _ in range(3):
            g.epoch_async()
        single += [tuple(r) for r in g.results(3)]
        g.close()
    single = np.array(single, np.float64)
    ok = np.array_equal(ranks[0], ranks[1])
    rel = np.abs(ranks[0][:, [0, 2]] - single[:, [0, 2]]) / np.abs(single[:, [0, 2]])
    acc = np.abs(ranks[0][:, [1, 3]] - single[:, [1, 3]])
    out = {"ranks_identical": bool(ok), "max_rel_loss": float(rel.max()),
           "max_acc_diff": float(acc.max()), "world2": ranks[0].tolist(),
           "single": single.tolist()}
    print(json.dumps(out))
    sys.exit(0 if ok and rel.max() <= 1e-4 and acc.max() <= 0.01 else 1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=-1)
    ap.add_argument("--dir", default="")
    ap.add_argument("--dataset", default="cora")
    ap.add_argument("--epochs", type=int, default=5)
    a = ap.parse_args()
    rank_main(a) if a.rank >= 0 else parent_main(a)
