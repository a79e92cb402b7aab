"""The edge-cut engine at worlds 2, 4 and 8 on ONE GPU through the in-process loopback
ranks (SURVEY.md §4 "fake RCCL"; RCCL itself refuses two ranks on one device).

Each rank is an engine created and driven by its own host thread; its collectives are the
peer-mapped exchange's kernels (PeerComm, k_peer.hip) over raw device pointers -- the same
pushes, flags and rank-order sums as one process per GPU.  Everything else is the multi-GPU
path the 8-GPU bench runs: nnz-balanced contiguous node ranges, GraphSum partials pushed into
their owners' slots by the combine, dropout masks drawn at the global stream offsets of each
rank's elements, per-rank Â X for eval, the training split's column-subset backward, the
weight-gradient all-reduce.  Compared with the oracle (single process, the reference's algorithm)
with dropout 0.5 at the north star's 1e-4 on the losses.
"""
import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu


def _run_world(pgcn, ds, world, epochs, params=None, asynchronous=0):
    group = pgcn.LoopbackGroup(world)
    p = params or pgcn.make_params(ds)

    def rank_fn(r):
        g = pgcn.GCN(p, ds, device=0, rank=r, loopback=group)
        info = {k: g.query(k) for k in ("world", "rank", "comm", "graphsum_lds", "reassociated")}
        lines = [g.train_epoch() + g.eval(2) for _ in range(epochs)]
        for _ in range(asynchronous):
            g.epoch_async()
        if asynchronous:
            lines += [tuple(x) for x in g.results(asynchronous)]
        test = g.eval(3)
        rng = g.node_range()
        w1 = g.get_var(2)
        g.close()
        return dict(info=info, lines=lines, test=test, range=rng, w1=w1)
    return pgcn.run_ranks(world, rank_fn)


def _check_ranks(res, world, n):
    bounds = [r["range"] for r in res]
    assert bounds[0][0] == 0 and bounds[-1][1] == n
    for a, b in zip(bounds, bounds[1:]):
        assert a[1] == b[0] and a[0] < a[1]
    for r, x in enumerate(res):
        assert x["info"]["world"] == world and x["info"]["rank"] == r
        assert x["info"]["comm"] == 2  # loopback
        # every rank reports the same all-reduced scalars and holds the same weights
        np.testing.assert_array_equal(np.asarray(x["lines"]), np.asarray(res[0]["lines"]))
        np.testing.assert_array_equal(x["w1"], res[0]["w1"])


@pytest.mark.parametrize("world", [2, 4])
def test_loopback_cora_matches_reference_lines(loaded, pgcn, world):
    ds = loaded["cora"]
    res = _run_world(pgcn, ds, world, 20, asynchronous=3)
    _check_ranks(res, world, ds.num_nodes)
    gold = helpers.golden("cora")["epoch_lines"].reshape(-1, 4)
    cnt = helpers.split_counts(ds)
    for e, ours in enumerate(res[0]["lines"]):
        helpers.assert_line_close(ours, gold[e], cnt, what=f"world {world} epoch {e + 1}")


@pytest.fixture(scope="module")
def big_ds(pgcn):
    # 140k nodes: a rank's columns (70k / 35k / 17.5k at world 2 / 4 / 8) take the LDS GraphSum
    # (tables above 1 MB); the gather kernel case forces the plain path
    return pgcn.Dataset.synthetic(140000, 64, 41, 1500000, 31)


@pytest.fixture(scope="module")
def big_oracle(big_ds):
    """4 epoch lines, eval(3), and the oracle's near-tied rows of every pass (the accuracy
    tolerance, helpers.near_ties)."""
    ref = helpers.OracleGCN(helpers.ds_dict(big_ds))
    c = big_ds.output_dim
    runs = [ref.epoch_with_ties(big_ds.label, big_ds.split, c) for _ in range(4)]
    test, tt = ref.eval_with_ties(3, big_ds.label, big_ds.split, c)
    return [r[0] for r in runs], [r[1] for r in runs], test, {1: tt, 2: tt}


@pytest.mark.parametrize("world,split_rows,lds", [(2, 0, 1), (2, 1, 1), (4, 0, 1), (8, 0, 1),
                                                  (4, 0, 0), (4, 1, 1)])
def test_loopback_lds_graph_matches_oracle(pgcn, big_ds, big_oracle, world, split_rows, lds):
    """lds 1: every rank's column block takes the LDS ring GraphSum, whose combine pushes the
    partial sums into the owners' receive slots (PeerComm); lds 0: the plain kernels, whose
    partials go through the generic push / wait / rank-order sum; split_rows 1: the output
    layer's forward over the split's rows (the generic path too)."""
    with helpers.knobs(pgcn, split_rows=split_rows, lds_min_kb=-1 if lds else 1 << 20):
        res = _run_world(pgcn, big_ds, world, 4)
    _check_ranks(res, world, big_ds.num_nodes)
    assert res[0]["info"]["graphsum_lds"] == lds
    assert res[0]["info"]["reassociated"] == 1
    cnt = helpers.split_counts(big_ds)
    lines, ties, test, test_ties = big_oracle
    for e, (ours, want, tie) in enumerate(zip(res[0]["lines"], lines, ties)):
        helpers.assert_line_close(ours, want, cnt, what=f"world {world} epoch {e + 1}", ties=tie)
    t = res[0]["test"]
    helpers.assert_line_close(t + t, test * 2, {1: cnt[3], 2: cnt[3]}, what="test",
                              ties=test_ties)


def test_loopback_hidden_above_128(pgcn, big_ds):
    """A hidden width above 128 on the LDS path at world 2: 16 passes of 16 columns, each pass's
    combine pushing its columns into the owners' slots and only the last one signalling; those
    GraphSums prescale per pass (the batched prescale takes <= 128 columns)."""
    dims, drops = (256,), (0.5, 0.5)
    p = pgcn.make_params(big_ds, hidden_dims=dims, dropouts=drops)
    res = _run_world(pgcn, big_ds, 2, 2, params=p)
    _check_ranks(res, 2, big_ds.num_nodes)
    assert res[0]["info"]["graphsum_lds"] == 1
    ref = helpers.OracleGCN(helpers.ds_dict(big_ds), hidden_dims=dims, dropouts=drops)
    cnt = helpers.split_counts(big_ds)
    for e in range(2):
        want, ties = ref.epoch_with_ties(big_ds.label, big_ds.split, big_ds.output_dim,
                                         helpers.DEEP_TIE_TOL)
        helpers.assert_line_close(res[0]["lines"][e], want, cnt, what=f"epoch {e + 1}", ties=ties)


# BASELINE configs[4] (4 layers, hidden 128) on the edge-cut path: 140k nodes, so a rank's
# column block takes the LDS GraphSum at world 8 too (17.5k columns x 64 B > 1 MB); every
# d = 128 GraphSum then runs as 16-column LDS passes over the rank's chunk graphs, each chunk
# reduce-scattered on the comm stream
DEEP = dict(n=140000, f=32, c=41, edges=1500000, seed=33)
DEEP_DIMS, DEEP_DROPS = (128, 128, 128), (0.5, 0.5, 0.5, 0.5)


@pytest.fixture(scope="module")
def deep_ds(pgcn):
    return pgcn.Dataset.synthetic(DEEP["n"], DEEP["f"], DEEP["c"], DEEP["edges"], DEEP["seed"])


@pytest.fixture(scope="module")
def deep_oracle(deep_ds):
    ref = helpers.OracleGCN(helpers.ds_dict(deep_ds), hidden_dims=DEEP_DIMS, dropouts=DEEP_DROPS)
    c = deep_ds.output_dim
    tol = helpers.DEEP_TIE_TOL
    runs = [ref.epoch_with_ties(deep_ds.label, deep_ds.split, c, tol) for _ in range(2)]
    test, tt = ref.eval_with_ties(3, deep_ds.label, deep_ds.split, c, tol)
    return [r[0] for r in runs], [r[1] for r in runs], test, {1: tt, 2: tt}


@pytest.mark.parametrize("world", [2, 8])
def test_loopback_deep_wide_matches_oracle(pgcn, deep_ds, deep_oracle, world):
    """4-layer hidden-128 model (BASELINE configs[4]) on the edge-cut engine at worlds 2 and 8
    (loopback communicator): 128-wide GraphSums on the ranks' chunk graphs with their
    reduce-scatters, the hidden layers' Matmul weight gradients all-reduced, against the
    oracle's L-layer restatement (hpdga's algorithm, src/gcn.cu:85-112's layer builder)."""
    p = pgcn.make_params(deep_ds, hidden_dims=DEEP_DIMS, dropouts=DEEP_DROPS)
    res = _run_world(pgcn, deep_ds, world, 2, params=p)
    _check_ranks(res, world, deep_ds.num_nodes)
    assert res[0]["info"]["graphsum_lds"] == 1
    cnt = helpers.split_counts(deep_ds)
    lines, ties, test, test_ties = deep_oracle
    for e, (ours, want, tie) in enumerate(zip(res[0]["lines"], lines, ties)):
        helpers.assert_line_close(ours, want, cnt, what=f"world {world} epoch {e + 1}", ties=tie)
    t = res[0]["test"]
    helpers.assert_line_close(t + t, test * 2, {1: cnt[3], 2: cnt[3]}, what="test", ties=test_ties)


# ------------------------------------------------------------------ reddit's feature width
def _run_world_rw(pgcn, ds, world, epochs, params=None):
    """_run_world plus, per rank, the logits of its rows after eval(3) and the launch counts
    of its own host thread (the rank's kernels only)."""
    group = pgcn.LoopbackGroup(world)
    p = params or pgcn.make_params(ds)

    def rank_fn(r):
        pgcn.reset_path_counts(thread=True)
        g = pgcn.GCN(p, ds, device=0, rank=r, loopback=group)
        info = {k: g.query(k) for k in ("world", "rank", "comm", "graphsum_lds", "reassociated")}
        lines = [g.train_epoch() + g.eval(2) for _ in range(epochs)]
        test = g.eval(3)
        paths = pgcn.path_counts(thread=True)
        rng = g.node_range()
        logits = g.get_var(g.num_vars() - 1)
        w1 = g.get_var(2)
        g.close()
        return dict(info=info, lines=lines, test=test, range=rng, w1=w1, logits=logits,
                    paths=paths)
    return pgcn.run_ranks(world, rank_fn)


@pytest.mark.parametrize("world", [2, 8])
def test_loopback_reddit_width_matches_oracle(pgcn, rw_ds, rw_oracle, world):
    """The edge-cut engine at reddit's feature width (F = 602, 41 classes, 100 k nodes, 3.1 M
    slots) at worlds 2 and 8: every rank's first layer runs the loader / MFMA-wave X-stream
    kernels on its own row range (k_xs_nn_ring for the masked training product and eval's
    (Â X) W1, k_xs_tn_ring for its W1.grad partial), proven by each rank thread's launch
    counters; 3 epochs + eval(3), every rank's rows of the logits and the weights against the
    oracle (hpdga gcn.cpp:179-212, module.cpp:49-72)."""
    res = _run_world_rw(pgcn, rw_ds, world, 3)
    _check_ranks(res, world, rw_ds.num_nodes)
    cnt = helpers.split_counts(rw_ds)
    want = rw_oracle
    for e, (ours, ref, tie) in enumerate(zip(res[0]["lines"], want["lines"], want["ties"])):
        helpers.assert_line_close(ours, ref, cnt, what=f"world {world} epoch {e + 1}", ties=tie)
    t = res[0]["test"]
    helpers.assert_line_close(t + t, want["test"] * 2, {1: cnt[3], 2: cnt[3]}, what="test",
                              ties=want["test_ties"])
    c = rw_ds.output_dim
    ref_logits = want["logits"].reshape(-1, c)
    for r, x in enumerate(res):
        lo, hi = x["range"]
        np.testing.assert_allclose(x["logits"].reshape(-1, c), ref_logits[lo:hi], rtol=1e-4,
                                   atol=1e-4, err_msg=f"rank {r} logits")
        p = x["paths"]
        # per epoch: training drop(X) W1 + eval (Â X) W1 on NN, W1.grad on TN; + eval(3)
        assert p["xs_nn_ring"] >= 7 and p["xs_tn_ring"] == 3, (r, p)
        assert p["xs_nn"] == 0 and p["xs_tn"] == 0, (r, p)
    w1, scale = res[0]["w1"], np.abs(want["w1"]).max()
    err = np.abs(w1 - want["w1"])
    assert np.quantile(err, 0.99) <= 1e-3 * scale and np.median(err) <= 1e-4 * scale


def test_loopback_deep_reddit_width_matches_oracle(pgcn):
    """4 layers x hidden 128 at reddit's feature width (F = 602) on the edge-cut engine at
    world 2: each rank's first layer (masked product, eval (Â X) W1, W1.grad partial) and
    hidden layers on the wide MFMA kernels over its own rows, 128-wide GraphSums reduce-
    scattered, weight grads all-reduced -- against the oracle's L-layer restatement
    (src/gcn.cu:85-112, hpdga gcn.cpp:179-212)."""
    ds = pgcn.Dataset.synthetic(24000, 602, 41, 240000, 43)
    dims, drops = (128, 128, 128), (0.5, 0.5, 0.5, 0.5)
    p = pgcn.make_params(ds, hidden_dims=dims, dropouts=drops)
    res = _run_world_rw(pgcn, ds, 2, 2, params=p)
    _check_ranks(res, 2, ds.num_nodes)
    ref = helpers.OracleGCN(helpers.ds_dict(ds), hidden_dims=dims, dropouts=drops)
    cnt = helpers.split_counts(ds)
    for e in range(2):
        want, ties = ref.epoch_with_ties(ds.label, ds.split, ds.output_dim,
                                         helpers.DEEP_TIE_TOL)
        helpers.assert_line_close(res[0]["lines"][e], want, cnt, what=f"epoch {e + 1}", ties=ties)
    for r, x in enumerate(res):
        q = x["paths"]
        # per epoch on every rank: the wide NN for X W1 (training) and (Â X) W1 (eval) and the
        # hidden layers' products; the wide TN for the first layer's and hidden weight grads
        assert q["gemm_nn_w"] >= 2 * 8 and q["gemm_tn_w"] >= 2 * 3, (r, q)
