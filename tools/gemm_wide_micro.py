"""Wide-output GEMM timing on the reddit hidden-128 shapes (GPU box): pgcn_gemm (NN) and
pgcn_gemm_tn (TN) at M = 232,965 for (K, N) = (602, 128) masked, (128, 128), (128, 41 via
trans B) -- the 4-layer hidden-128 model's contractions -- with the wide kernels
(r05: the general-kernel arm was removed).  HIP events on torch's stream; one JSON line with ms
per call and TF/s against the 157.3 TF fp32 MFMA peak."""
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
M = 232965
dev = "cuda"
torch.manual_seed(0)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {"M": M}
for (K, N, masked, tb) in ((602, 128, True, 0), (602, 128, False, 0), (128, 128, False, 0),
                           (41, 128, False, 1), (128, 41, False, 0)):
    lda = (K + 3) // 4 * 4
    A = torch.zeros(M, lda, device=dev)
    A[:, :K] = torch.randn(M, K, device=dev)
    B = torch.randn(N, K, device=dev) if tb else torch.randn(K, N, device=dev)
    G = torch.randn(M, N, device=dev)
    mask = torch.randint(-2**62, 2**62, ((M * K + 63) // 64 + 1,), dtype=torch.int64, device=dev)
    C = torch.empty(M, N, device=dev)
    dW = torch.empty(K, N, device=dev)
    ws = torch.empty(lib.pgcn_gemm_tn_workspace(M, N, K) // 4 + 64, device=dev)
    flops = 2.0 * M * N * K
    for variant in (0,):  # (r05: the general-kernel arm "gemm_variant" 1 was removed)

        def nn():
            pg.check(lib.pgcn_gemm(M, N, K, vp(A), lda, vp(B), K if tb else N, tb, vp(C), N,
                                   vp(mask) if masked else None, 0, K, 2.0, st), "gemm")

        def tn():
            pg.check(lib.pgcn_gemm_tn(M, N, K, vp(A), lda, vp(G), N, vp(dW), N,
                                      vp(mask) if masked else None, 0, K, 2.0, vp(ws), st), "tn")
        for name, fn in (("nn", nn), ("tn", tn)):
            ms = timeit(fn)
            res[f"{name}_K{K}_N{N}{'m' if masked else ''}_v{variant}"] = {"ms": round(ms, 4),
                                                   "tflops": round(flops / ms / 1e9, 1),
                                                   "frac": round(flops / ms / 1e9 / 157.3, 3)}
print(json.dumps(res))
