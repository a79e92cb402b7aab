"""X-stream NN grid sweep on the reddit shape (diagnostic; GPU box): times pgcn_gemm_xstream
(drop(X) W1 and X W1, X = [232965][604] fp32) for the default grid, the balanced grid
(xstream_nn_balance 1) and fixed workgroup counts.  One JSON line: ms per call, TB/s of X."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

pg = helpers.pgcn()
lib = pg.lib
M, K, N, LDA = 232965, 602, 16, 604
X = torch.zeros(M, LDA, device="cuda")
X[:, :K] = torch.randn(M, K, device="cuda")
W = torch.randn(K, N, device="cuda")
Z = torch.empty(M, N, device="cuda")
nib = torch.randint(-2**62, 2**62, (M, 16), dtype=torch.int64, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def run(masked):
    pg.check(lib.pgcn_gemm_xstream(M, N, K, vp(X), LDA, vp(W), N, 0, vp(Z), N,
                                   vp(nib) if masked else None, 2.0, st), "xnn")


def timeit(masked, reps=30):
    for _ in range(3):
        run(masked)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run(masked)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {}
settings = [0, 1] + [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else
                                      "256,384,456,512,640,768,1024").split(",")]
for rep in range(2):
    for b in settings:
        lib.pgcn_debug_set(b"xstream_nn_balance", b)
        for masked in (True, False):
            ms = timeit(masked)
            key = f"{'masked' if masked else 'plain'}_b{b}"
            res.setdefault(key, []).append(round(ms * 1000, 1))
lib.pgcn_debug_set(b"xstream_nn_balance", 0)
res["tb_s_at_100us"] = 4.0 * M * K / 100e-6 / 1e12
print(json.dumps(res))
