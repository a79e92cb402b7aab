"""Pin the C restatement (oracle/pgcn_oracle.c) against the reference's own outputs.

The golden fixtures were produced by the reference's sequential sources
(hpdga-spring23/src/*.cpp, compiled by oracle/Makefile; tests/golden/make_golden.py).  The
restatement must reproduce them BIT-FOR-BIT: every epoch line of 100 epochs, the glorot
weights, every epoch-1 activation and gradient, the xorshift stream.  Only after this holds
is the oracle trusted as the checker of the HIP engine.
"""
import numpy as np
import pytest

import helpers

DATASETS = ["cora", "citeseer", "pubmed_synth"]


@pytest.fixture(scope="module")
def runs(loaded):
    out = {}
    for name in DATASETS:
        ds = helpers.ds_dict(loaded[name])
        g = helpers.OracleGCN(ds)
        init = [g.var(i) for i in range(7)]
        lines, e1 = [], None
        for e in range(100):
            tl, ta = g.train_epoch()
            if e == 0:
                e1 = {"vars": [g.var(i) for i in range(7)], "grads": [g.var(i, 1) for i in range(7)]}
            vl, va = g.eval(2)
            if e == 0:
                e1["eval_logits"] = g.var(6)
            lines.append([tl, ta, vl, va])
        test = g.eval(3)
        out[name] = dict(init=init, e1=e1, lines=np.array(lines, np.float32), test=test,
                         final_w1=g.var(2), final_w2=g.var(5))
    return out


@pytest.mark.parametrize("name", DATASETS)
def test_epoch_lines_bit_exact(runs, name):
    gold = helpers.golden(name)
    np.testing.assert_array_equal(runs[name]["lines"], gold["epoch_lines"].reshape(-1, 4))
    np.testing.assert_array_equal(np.array(runs[name]["test"], np.float32), gold["test_scalars"])


@pytest.mark.parametrize("name", DATASETS)
def test_weights_bit_exact(runs, name):
    gold = helpers.golden(name)
    r = runs[name]
    np.testing.assert_array_equal(r["init"][2], gold["init_W1"])
    np.testing.assert_array_equal(r["init"][5], gold["init_W2"])
    np.testing.assert_array_equal(r["final_w1"], gold["final_W1"])
    np.testing.assert_array_equal(r["final_w2"], gold["final_W2"])


@pytest.mark.parametrize("name", ["cora", "citeseer"])
def test_epoch1_tensors_bit_exact(runs, name):
    gold = helpers.golden(name)
    e1 = runs[name]["e1"]
    names = ["input", "l1_var1", "W1", "l1_var2", "l2_var1", "W2", "output"]
    for i, n in enumerate(names):
        if n in ("W1", "W2"):
            np.testing.assert_array_equal(e1["grads"][i], gold[f"e1_{n}_grad"])
            np.testing.assert_array_equal(e1["vars"][i], gold[f"e1_{n}_after_step"])
            continue
        np.testing.assert_array_equal(e1["vars"][i], gold[f"e1_{n}"], err_msg=n)
        if n != "input":
            np.testing.assert_array_equal(e1["grads"][i], gold[f"e1_{n}_grad"], err_msg=n + " grad")
    np.testing.assert_array_equal(e1["eval_logits"], gold["e1_eval_logits"])


def test_golden_lines_text_matches_binary():
    # the printed %.5f lines (what the reference prints) agree with the binary fixture
    for name in DATASETS:
        gold = helpers.golden(name)["epoch_lines"].reshape(-1, 4)
        txt = helpers.golden_lines(name)
        for e, line in enumerate(txt[:100]):
            g = gold[e]
            assert line == (f"epoch={e + 1} train_loss={g[0]:.5f} train_acc={g[1]:.5f} "
                            f"val_loss={g[2]:.5f} val_acc={g[3]:.5f}")


def test_rng_stream_matches_reference():
    lib = helpers.oracle()
    gold = helpers.golden("cora")
    s = np.zeros(2, np.uint64)
    lib.or_rng_seed(helpers.ptr(s))
    np.testing.assert_array_equal(s, gold["rng_seed_state"])
    draws = np.array([lib.or_rng_next(helpers.ptr(s)) for _ in range(64)], np.int32)
    np.testing.assert_array_equal(draws, gold["rng_first64"])


def test_anchor_lines_from_survey():
    # SURVEY.md §8c anchor lines (the reference binary run in the survey container)
    assert helpers.golden_lines("cora")[0] == ("epoch=1 train_loss=1.95362 train_acc=0.17798 "
                                               "val_loss=1.94780 val_acc=0.52000")
    assert helpers.golden_lines("cora")[100] == "test_loss=1.08953 test_acc=0.81900"
    assert helpers.golden_lines("citeseer")[100] == "test_loss=1.21826 test_acc=0.77000"
