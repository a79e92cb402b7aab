import os
import sys

import pytest
# torch first: its bundled libamdhip64.so.7 / librccl.so.1 then satisfy libpgcn.so's
# dependencies (same SONAMEs), so one process never holds two HIP runtimes.
import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import helpers  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def datasets(tmp_path_factory):
    """Root directory holding data/<name>.* for cora, citeseer and pubmed (synthetic
    features), materialised from tests/golden/data."""
    root = str(tmp_path_factory.mktemp("datasets"))
    names = {}
    for n in ("cora", "citeseer", "pubmed_synth"):
        names[n] = helpers.materialize_dataset(n, root)
    return root, names


@pytest.fixture(scope="session")
def pgcn():
    return helpers.pgcn()


@pytest.fixture(scope="session")
def loaded(datasets, pgcn):
    root, names = datasets
    return {k: pgcn.Dataset.load(root, v) for k, v in names.items()}


@pytest.fixture(scope="session")
def rw_ds(pgcn):
    """reddit's feature width (F = 602) and 41 classes on a 100 k-node power-law graph."""
    g = helpers.RW_GRAPH
    return pgcn.Dataset.synthetic(g["n"], g["f"], g["c"], g["edges"], g["seed"])


@pytest.fixture(scope="session")
def rw_oracle(rw_ds):
    """3 oracle epochs + eval(3) on rw_ds (shared by the single-GPU and edge-cut tests)."""
    return helpers.oracle_run(rw_ds, 3)
