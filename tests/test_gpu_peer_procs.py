"""The edge-cut engine over peer-mapped memory with one PROCESS per rank (pgcn_gcn_create_peer,
DESIGN.md §6): every rank's receive slots are opened in every other process with hipIpc
handles exchanged over a gloo group, and a GraphSum's partial sums are stored straight into
their owner's slot by the kernel that forms them.  On this one-GPU box all ranks share the
device -- the same code, handles, flags and kernels as one process per GPU over xGMI.

Checked against the in-process loopback ranks (the same kernels over raw pointers): epoch lines,
eval(3), every rank's rows of the logits and W1 bit-identical; and cora against the reference's
golden lines."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_procs(world, spec, tmp_path):
    port = _free_port()
    sp = os.path.join(str(tmp_path), "spec.json")
    with open(sp, "w") as f:
        json.dump(spec, f)
    outs = [os.path.join(str(tmp_path), f"rank{r}.npz") for r in range(world)]
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "peer_worker.py"), str(r),
                               str(world), str(port), sp, outs[r]], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=300)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} rc {p.returncode}:\n{logs[r][-3000:]}"
    return [dict(np.load(o)) for o in outs]


def _run_loopback(pgcn, ds, world, spec):
    group = pgcn.LoopbackGroup(world)
    p = pgcn.make_params(ds)

    def rank_fn(r):
        g = pgcn.GCN(p, ds, device=0, rank=r, loopback=group)
        lines = [g.train_epoch() + g.eval(2) for _ in range(spec["epochs"])]
        for _ in range(spec.get("async", 0)):
            g.epoch_async()
        if spec.get("async", 0):
            lines += [tuple(x) for x in g.results(spec["async"])]
        test = g.eval(3)
        out = dict(lines=np.array(lines, np.float64), test=np.array(test, np.float64),
                   range=np.array(g.node_range()), logits=g.get_var(g.num_vars() - 1),
                   w1=g.get_var(2))
        g.close()
        return out
    with helpers.knobs(pgcn, **spec.get("knobs", {})):
        return pgcn.run_ranks(world, rank_fn)


def _same(procs, loop, world):
    for r in range(world):
        a, b = procs[r], loop[r]
        assert list(a["info"][:3]) == [world, r, 4]  # world, rank, comm = peer (IPC)
        np.testing.assert_array_equal(a["range"], b["range"])
        np.testing.assert_array_equal(a["lines"], b["lines"])
        np.testing.assert_array_equal(a["test"], b["test"])
        np.testing.assert_array_equal(a["logits"], b["logits"])
        np.testing.assert_array_equal(a["w1"], b["w1"])
        np.testing.assert_array_equal(a["lines"], procs[0]["lines"])  # all-reduced scalars


def test_peer_procs_cora_world2(pgcn, datasets, loaded, tmp_path):
    root, names = datasets
    spec = {"root": root, "name": names["cora"], "epochs": 10, "async": 2}
    procs = _run_procs(2, spec, tmp_path)
    _same(procs, _run_loopback(pgcn, loaded["cora"], 2, spec), 2)
    gold = helpers.golden("cora")["epoch_lines"].reshape(-1, 4)
    cnt = helpers.split_counts(loaded["cora"])
    for e, ours in enumerate(procs[0]["lines"][:10]):
        helpers.assert_line_close(ours, gold[e], cnt, what=f"peer procs epoch {e + 1}")


@pytest.mark.parametrize("world,tail,uncached", [(2, 0, 0), (4, 0, 0), (4, 1, 0), (2, 0, 1)])
def test_peer_procs_lds_graph(pgcn, world, tail, uncached, tmp_path):
    """140k nodes: every rank's column block takes the LDS ring GraphSum, whose combine pushes
    the partial sums into the owners' slots (k_gs_lds_combine's push mode).  tail 1: the eval
    pass's last exchange and output layer on the comm stream beside the next epoch (eval_tail),
    the same bits as the in-process ranks (which never take it).  uncached 1: the receive
    slots in uncached memory (peer_uncached), the same bits."""
    syn = dict(n=140000, f=64, c=41, edges=1500000, seed=31)
    spec = {"synthetic": syn, "epochs": 3, "async": 2,
            "knobs": {"eval_tail": tail, "peer_uncached": uncached}}
    procs = _run_procs(world, spec, tmp_path)
    assert procs[0]["info"][3] == 1  # graphsum_lds
    assert procs[0]["info"][4] == uncached  # the slots' memory as asked
    ds = pgcn.Dataset.synthetic(syn["n"], syn["f"], syn["c"], syn["edges"], syn["seed"])
    _same(procs, _run_loopback(pgcn, ds, world, spec), world)
