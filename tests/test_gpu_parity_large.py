"""Parity of the MEASURED path: the default engine on graphs whose feature table takes the
LDS GraphSum (n_cols * 64 B above 1 MB and >= 32 k rows, graph.hpp kLdsMinBytes), with dense
features (X-stream MFMA kernels + nibble dropout masks), 41 classes (the output layer runs
reassociated as (Â H) W2 over every row, its backward over the training split's columns),
eval's first layer from Â X, train-ahead -- against the oracle (the C restatement of
hpdga-spring23/src/gcn.cpp:179-212, pinned bit-exact to the reference build) at the north
star's 1e-4 on the losses.  Also the diagnostic row restriction (split_rows), the dual
X-stream pass (eval_ax off), the 4-layer hidden-128 model (16-column LDS passes inside a
deep stack), the edge-cut engine at world 1, and reddit's own feature width (F = 602), the
only width the loader / MFMA-wave X-stream kernels (k_xs_nn_ring, k_xs_tn_ring) take.

Accuracies: a row may differ from the oracle's verdict only where the oracle's logits of that
pass are within 1e-5 of a tie (helpers.near_ties); the tests count those rows and allow
exactly that many.

Sizes: the oracle finishes an epoch of these graphs in about a second (2-layer, F = 64), a
few seconds (4 x 128, F = 602); the reddit-114M epoch itself is compared by bench.py (its
"parity" key).
"""
import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu

# N > 62,500 (LDS path), hubs from the Chung-Lu power law, ~3.1 M adjacency slots
LDS_GRAPH = dict(n=120000, f=64, c=41, edges=1500000, seed=21)
EPOCHS = 5


def _synthetic(pgcn, g):
    return pgcn.Dataset.synthetic(g["n"], g["f"], g["c"], g["edges"], g["seed"])


@pytest.fixture(scope="module")
def lds_ds(pgcn):
    return _synthetic(pgcn, LDS_GRAPH)


@pytest.fixture(scope="module")
def oracle_lines(lds_ds):
    return helpers.oracle_run(lds_ds, EPOCHS)


def _check_lines(ds, lines, test, want, what):
    cnt = helpers.split_counts(ds)
    for e, (ours, ref, ties) in enumerate(zip(lines, want["lines"], want["ties"])):
        helpers.assert_line_close(ours, ref, cnt, what=f"{what} epoch {e + 1}", ties=ties)
    helpers.assert_line_close(test + test, want["test"] * 2, {1: cnt[3], 2: cnt[3]},
                              what=f"{what} test", ties=want["test_ties"])


def _engine_lines(pgcn, ds, epochs=EPOCHS, **make):
    g = pgcn.GCN(pgcn.make_params(ds), ds, **make)
    assert g.query("graphsum_lds") == 1, "the graph must take the LDS GraphSum path"
    assert g.query("reassociated") == 1
    lines = [g.train_epoch() + g.eval(2) for _ in range(epochs)]
    test = g.eval(3)
    return g, lines, test


@pytest.mark.parametrize("config", ["default", "split_rows", "eval_ax_off", "async"])
def test_lds_graph_matches_oracle(pgcn, lds_ds, oracle_lines, config):
    knobs = {"split_rows": dict(split_rows=1), "eval_ax_off": dict(eval_ax=0)}.get(config, {})
    with helpers.knobs(pgcn, **knobs):
        if config == "async":  # the bench loop: epoch_async, results from the device ring
            g = pgcn.GCN(pgcn.make_params(lds_ds), lds_ds)
            for _ in range(EPOCHS):
                g.epoch_async()
            lines = [tuple(r) for r in g.results(EPOCHS)]
            test = g.eval(3)
        else:
            g, lines, test = _engine_lines(pgcn, lds_ds)
        _check_lines(lds_ds, lines, test, oracle_lines, config)
        if config != "split_rows":
            # every row's logits after eval(3) (max-shifted in place on the labelled rows, as
            # the reference's loss does)
            np.testing.assert_allclose(g.get_var(6), oracle_lines["logits"], rtol=1e-4,
                                       atol=1e-4)
        np.testing.assert_allclose(g.get_var(5), oracle_lines["w2"], rtol=1e-3, atol=1e-6)
        g.close()


def test_lds_graph_edge_cut_world1_matches_oracle(pgcn, lds_ds, oracle_lines):
    """The edge-cut engine (chunk graphs, reduce-scatters on the comm stream, per-rank Â X,
    column-subset backward chunks) at world 1 on the same LDS-path graph."""
    cnt = helpers.split_counts(lds_ds)
    g = pgcn.GCN(pgcn.make_params(lds_ds), lds_ds, device=0, rank=0, world=1,
                 unique_id=pgcn.comm_unique_id())
    assert g.query("world") == 1 and g.query("comm") == 1
    for e, (want, ties) in enumerate(zip(oracle_lines["lines"], oracle_lines["ties"])):
        helpers.assert_line_close(g.train_epoch() + g.eval(2), want, cnt, what=f"epoch {e + 1}",
                                  ties=ties)
    g.close()


def test_deep_wide_lds_graph_matches_oracle(pgcn):
    """4 layers x hidden 128 (BASELINE configs[4]) on a graph that takes the LDS path: every
    d = 128 GraphSum runs as 16-column LDS passes, the eval first layer as (Â X) W1 on MFMA."""
    ds = pgcn.Dataset.synthetic(64000, 32, 41, 1000000, 23)
    dims, drops = (128, 128, 128), (0.5, 0.5, 0.5, 0.5)
    g = pgcn.GCN(pgcn.make_params(ds, hidden_dims=dims, dropouts=drops), ds)
    assert g.query("graphsum_lds") == 1
    ref = helpers.OracleGCN(helpers.ds_dict(ds), hidden_dims=dims, dropouts=drops)
    cnt = helpers.split_counts(ds)
    for e in range(2):
        want, ties = ref.epoch_with_ties(ds.label, ds.split, ds.output_dim,
                                         helpers.DEEP_TIE_TOL)
        helpers.assert_line_close(g.train_epoch() + g.eval(2), want, cnt, what=f"epoch {e + 1}",
                                  ties=ties)
    g.close()


# ------------------------------------------------------------------ reddit's feature width
# (rw_ds / rw_oracle: tests/conftest.py, shared with the edge-cut tests)
def test_reddit_width_epoch_matches_oracle(pgcn, rw_ds, rw_oracle):
    """The measured configuration at F = 602 (reddit's width), 41 classes, 100 k nodes, 3.1 M
    slots, every engine default: 3 epochs + eval(3) + every row of the logits + the weights
    against the oracle, and the launch counters prove the first layer ran on the loader / MFMA-
    wave X-stream kernels (k_xs_nn_ring for the masked training product and eval's (Â X) W1,
    k_xs_tn_ring for W1.grad), never on the register-streamed ones (hpdga gcn.cpp:179-212,
    module.cpp:49-72)."""
    pgcn.reset_path_counts()
    g, lines, test = _engine_lines(pgcn, rw_ds, epochs=3)
    paths = pgcn.path_counts()
    _check_lines(rw_ds, lines, test, rw_oracle, "F=602")
    np.testing.assert_allclose(g.get_var(6), rw_oracle["logits"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(g.get_var(5), rw_oracle["w2"], rtol=1e-3, atol=1e-6)
    w1, scale = g.get_var(2), np.abs(rw_oracle["w1"]).max()
    err = np.abs(w1 - rw_oracle["w1"])
    assert np.quantile(err, 0.99) <= 1e-3 * scale and np.median(err) <= 1e-4 * scale
    g.close()
    # per epoch: training drop(X) W1 and eval (Â X) W1 on NN, W1.grad on TN; + eval(3)
    assert paths["xs_nn_ring"] >= 7 and paths["xs_tn_ring"] == 3, paths
    assert paths["xs_nn"] == 0 and paths["xs_tn"] == 0, paths
    assert paths["gs_ring"] > 0 and paths["out_xent"] >= 7, paths


def test_xstream_ring_engine_matches_register_kernels(pgcn, rw_ds):
    """The loader / MFMA-wave X-stream kernels (k_xstream_lds.hip, the default at F = 602)
    against the register-streamed k_xstream_nn / k_xstream_tn (xstream_ring 0) in a whole run
    at reddit's width: the launch counters show each arm ran its own kernels; the forward
    products are bit-identical (epoch 1's training line), W1.grad sums the same rows in
    another order, so later lines agree to float rounding."""
    lines, paths = {}, {}
    for ring in (1, 0):
        with helpers.knobs(pgcn, xstream_ring=ring):
            pgcn.reset_path_counts()
            g = pgcn.GCN(pgcn.make_params(rw_ds), rw_ds)
            lines[ring] = np.array([g.train_epoch() + g.eval(2) for _ in range(3)], np.float64)
            paths[ring] = pgcn.path_counts()
            g.close()
    assert paths[1]["xs_nn_ring"] > 0 and paths[1]["xs_tn_ring"] > 0, paths[1]
    assert paths[1]["xs_nn"] == 0 and paths[1]["xs_tn"] == 0, paths[1]
    assert paths[0]["xs_nn_ring"] == 0 and paths[0]["xs_tn_ring"] == 0, paths[0]
    assert paths[0]["xs_nn"] > 0 and paths[0]["xs_tn"] > 0, paths[0]
    np.testing.assert_array_equal(lines[1][0, :2], lines[0][0, :2])  # epoch 1 forward: NN only
    np.testing.assert_allclose(lines[1][:, [0, 2]], lines[0][:, [0, 2]], rtol=2e-5)
    cnt = helpers.split_counts(rw_ds)  # a near-tied row may flip: at most 3 rows per split
    for col, sp in ((1, 1), (3, 2)):
        assert np.abs(lines[1][:, col] - lines[0][:, col]).max() * cnt[sp] <= 3 + 1e-3


def test_deep_reddit_width_matches_oracle(pgcn):
    """4 layers x hidden 128 at reddit's feature width (F = 602, 10 k-chunks of 64): the first
    layer's product and weight gradient run on the wide MFMA kernels (k_gemm_wide.hip) with
    the input dropout in the nibble layout, the hidden layers' products and gradients on them
    too (unmasked), against the oracle at 1e-4 (hpdga gcn.cpp:179-212 generalised to L layers,
    src/gcn.cu:85-112)."""
    ds = pgcn.Dataset.synthetic(24000, 602, 41, 240000, 43)
    dims, drops = (128, 128, 128), (0.5, 0.5, 0.5, 0.5)
    pgcn.reset_path_counts()
    g = pgcn.GCN(pgcn.make_params(ds, hidden_dims=dims, dropouts=drops), ds)
    ref = helpers.OracleGCN(helpers.ds_dict(ds), hidden_dims=dims, dropouts=drops)
    cnt = helpers.split_counts(ds)
    for e in range(2):
        want, ties = ref.epoch_with_ties(ds.label, ds.split, ds.output_dim,
                                         helpers.DEEP_TIE_TOL)
        helpers.assert_line_close(g.train_epoch() + g.eval(2), want, cnt, what=f"epoch {e + 1}",
                                  ties=ties)
    paths = pgcn.path_counts()
    g.close()
    # per epoch: the wide NN for X W1 (training, masked), (Â X) W1 (eval), the hidden layers'
    # products (train + eval) and input grads; the wide TN for every hidden weight gradient
    assert paths["gemm_nn_w"] >= 2 * 8 and paths["gemm_tn_w"] >= 2 * 3, paths
    assert paths["gemm_nn"] == 0 or paths["gemm_nn"] < paths["gemm_nn_w"], paths
