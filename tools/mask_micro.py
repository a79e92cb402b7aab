"""Input-dropout mask kernels alone on reddit's shape (232,965 x 602 elements, p = 0.5), timed
with HIP events over repeated launches on the current stream (run on the GPU; PGCN_LIB selects
another build for A/B).  One JSON line: us per launch of the fused bitmap + nibble kernel
(pgcn_dropout_mask_nib) and of the two-launch form (pgcn_dropout_mask + pgcn_mask_nibbles)."""
import ctypes
import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
spec = importlib.util.spec_from_file_location(
    "pgcn", os.path.join(HERE, "..", "parallel-gcn_amd", "__init__.py"),
    submodule_search_locations=[os.path.join(HERE, "..", "parallel-gcn_amd")])
pgcn = importlib.util.module_from_spec(spec)
sys.modules["pgcn"] = pgcn
spec.loader.exec_module(pgcn)

ROWS, F = 232965, 602
REPS = int(os.environ.get("REPS", "30"))


def vp(t):
    return ctypes.c_void_p(t.data_ptr())


def main():
    dev = "cuda"
    n_elems = ROWS * F
    nch = (n_elems + 63) // 64
    rng = np.random.default_rng(5)
    states = torch.from_numpy(rng.integers(1, 2**62, (nch, 2), dtype=np.int64)).to(dev)
    table = torch.from_numpy(pgcn.rng_jump_table(144_000_000).view(np.int64)).to(dev)
    mask = torch.zeros(nch + 1, dtype=torch.int64, device=dev)
    nib = torch.zeros((ROWS, 16), dtype=torch.int64, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def fused():
        pgcn.check(pgcn.lib.pgcn_dropout_mask_nib(vp(states), nch, n_elems, 0, 0.5, vp(mask),
                                                  vp(table), 0, F, ROWS, vp(nib), st), "nib")

    def two():
        pgcn.check(pgcn.lib.pgcn_dropout_mask(vp(states), nch, n_elems, 0, 0.5, vp(mask),
                                              vp(table), st), "mask")
        pgcn.check(pgcn.lib.pgcn_mask_nibbles(vp(mask), 0, F, ROWS, F, vp(nib), st), "nibbles")

    out = {"rows": ROWS, "features": F, "reps": REPS, "lib": os.environ.get("PGCN_LIB", "in-tree")}
    for name, fn in (("fused_us", fused), ("two_launch_us", two)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REPS):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) * 1e3 / REPS
    print(json.dumps(out))


if __name__ == "__main__":
    main()
