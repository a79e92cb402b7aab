"""Generate the committed golden fixtures under tests/golden/ (run in the build container).

Provenance: every expected value here is produced by the reference's OWN sequential CPU code
(hpdga-spring23/src/*.cpp compiled where it lies by `make -C oracle ref` into
oracle/_ref/ref_golden, driven by oracle/ref_harness.cpp).  Nothing from the reference's
source text is stored; the reference's own dataset files (data/cora.*, data/citeseer.*,
data/pubmed.{graph,split}) are stored gzipped as input fixtures.

pubmed: the reference tree lacks data/pubmed.svmlight (.MISSING_LARGE_BLOBS:1), so
`pubmed_synth_svmlight()` below writes a SEEDED SYNTHETIC one (19,717 rows, 500 dims, 3
classes, ~50 nnz/row, row-normalised TF-IDF-like values).  Its golden lines are labelled
"pubmed_synth" and pin our engine against the reference on the real pubmed graph with
synthetic features.

Usage:  python tests/golden/make_golden.py [--ref /root/reference]
"""
import argparse
import gzip
import hashlib
import json
import os
import shutil
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
DATA_OUT = os.path.join(HERE, "data")

KEEP = [
    # (file stem in harness output, dtype)
    ("dims", np.int32), ("rng_seed_state", np.uint64), ("rng_first64", np.int32),
    ("rng_after_ctor", np.uint64), ("rng_after_e1_fwd", np.uint64), ("rng_after_e1", np.uint64),
    ("init_W1", np.float32), ("init_W2", np.float32),
    ("e1_input", np.float32),
    ("e1_l1_var1", np.float32), ("e1_l1_var1_grad", np.float32),
    ("e1_W1_grad", np.float32),
    ("e1_l1_var2", np.float32), ("e1_l1_var2_grad", np.float32),
    ("e1_l2_var1", np.float32), ("e1_l2_var1_grad", np.float32),
    ("e1_W2_grad", np.float32),
    ("e1_output", np.float32), ("e1_output_grad", np.float32),
    ("e1_W1_after_step", np.float32), ("e1_W2_after_step", np.float32),
    ("e1_train_scalars", np.float32), ("e1_eval_logits", np.float32),
    ("e1_eval_scalars", np.float32),
    ("epoch_lines", np.float32), ("final_W1", np.float32), ("final_W2", np.float32),
    ("final_eval_logits", np.float32), ("test_scalars", np.float32),
    ("final_test_logits", np.float32),
]
HASHED = [("graph_indptr", np.int32), ("graph_indices", np.int32), ("feat_indptr", np.int32),
          ("feat_indices", np.int32), ("feat_values", np.float32), ("label", np.int32),
          ("split", np.int32)]

PUBMED_SEED = 20230606


def pubmed_synth_svmlight(path, n_rows=19717, dims=500, classes=3, nnz=50, seed=PUBMED_SEED):
    """Seeded synthetic pubmed features (the real file is missing from the reference).

    Each row: label uniform in [0, classes); 50 distinct feature ids, 10 of them drawn from a
    label-specific band so the model has signal; values ~ TF-IDF-like positive weights,
    L1-normalised per row, written with 8 significant digits, ids ascending.
    """
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, classes, size=n_rows)
    band = dims // classes
    lines = []
    for i in range(n_rows):
        lab = int(labels[i])
        own = rng.choice(np.arange(lab * band, (lab + 1) * band), size=10, replace=False)
        rest = rng.choice(dims, size=nnz, replace=False)
        ids = np.unique(np.concatenate([own, rest]))[:nnz]
        vals = rng.gamma(2.0, 1.0, size=ids.size)
        vals = vals / vals.sum()
        toks = " ".join(f"{int(k)}:{v:.8g}" for k, v in zip(ids, vals))
        lines.append(f"{lab} {toks}\n")
    with open(path, "w") as f:
        f.writelines(lines)


def gz_copy(src, dst):
    with open(src, "rb") as fi, open(dst, "wb") as raw:
        with gzip.GzipFile(filename="", mode="wb", fileobj=raw, compresslevel=9, mtime=0) as fo:
            shutil.copyfileobj(fi, fo)


def run_harness(ref_golden, root, name, outdir, epochs=100):
    subprocess.run([ref_golden, root, name, outdir, str(epochs)], check=True,
                   stdout=subprocess.DEVNULL)


# pubmed's per-node intermediates are large; keep only what pins the epoch end to end.
SMALL = {"dims", "rng_seed_state", "rng_first64", "rng_after_ctor", "rng_after_e1_fwd",
         "rng_after_e1", "init_W1", "init_W2", "e1_W1_grad", "e1_W2_grad", "e1_output",
         "e1_W1_after_step", "e1_W2_after_step", "e1_train_scalars", "e1_eval_scalars",
         "epoch_lines", "final_W1", "final_W2", "test_scalars"}


def package(outdir, tag, small=False):
    arrs, hashes = {}, {}
    for stem, dt in KEEP:
        if small and stem not in SMALL:
            continue
        arrs[stem] = np.fromfile(os.path.join(outdir, stem + ".bin"), dtype=dt)
    for stem, dt in HASHED:
        raw = open(os.path.join(outdir, stem + ".bin"), "rb").read()
        hashes[stem] = {"sha256": hashlib.sha256(raw).hexdigest(),
                        "count": len(raw) // np.dtype(dt).itemsize}
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **arrs)
    lines = open(os.path.join(outdir, "epoch_lines.txt")).read()
    with open(os.path.join(HERE, f"{tag}_epoch_lines.txt"), "w") as f:
        f.write(lines)
    return hashes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True,
                   stdout=subprocess.DEVNULL)
    ref_golden = os.path.join(REPO, "oracle", "_ref", "ref_golden")
    os.makedirs(DATA_OUT, exist_ok=True)
    manifest = {"generator": "tests/golden/make_golden.py",
                "oracle": "oracle/_ref/ref_golden (reference hpdga-spring23 sources, g++ -O3 -std=c++11)",
                "datasets": {}}
    with tempfile.TemporaryDirectory() as tmp:
        for ds in ["cora", "citeseer"]:
            for ext in ["graph", "split", "svmlight"]:
                gz_copy(os.path.join(args.ref, "data", f"{ds}.{ext}"),
                        os.path.join(DATA_OUT, f"{ds}.{ext}.gz"))
            out = os.path.join(tmp, ds)
            run_harness(ref_golden, args.ref, ds, out)
            manifest["datasets"][ds] = {"parsed": package(out, ds), "features": "reference file"}
        # pubmed: real graph/split + seeded synthetic features
        root = os.path.join(tmp, "pm")
        os.makedirs(os.path.join(root, "data"))
        for ext in ["graph", "split"]:
            shutil.copy(os.path.join(args.ref, "data", f"pubmed.{ext}"),
                        os.path.join(root, "data", f"pubmed.{ext}"))
            gz_copy(os.path.join(args.ref, "data", f"pubmed.{ext}"),
                    os.path.join(DATA_OUT, f"pubmed.{ext}.gz"))
        pubmed_synth_svmlight(os.path.join(root, "data", "pubmed.svmlight"))
        out = os.path.join(tmp, "pubmed")
        run_harness(ref_golden, root, "pubmed", out)
        svm_hash = hashlib.sha256(open(os.path.join(root, "data", "pubmed.svmlight"), "rb").read()).hexdigest()
        manifest["datasets"]["pubmed_synth"] = {
            "parsed": package(out, "pubmed_synth", small=True),
            "features": f"SYNTHETIC (seed {PUBMED_SEED}); svmlight sha256 {svm_hash}"}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
