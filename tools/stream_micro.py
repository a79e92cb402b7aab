"""Streaming-read ceiling on this box (run on the GPU): torch reductions / copies / hipBLASLt
GEMM over the reddit-shaped X [232965][604] fp32 (563 MB), ms and GB/s.  One JSON line."""
import json

import torch

M, LDA, K, N = 232965, 604, 602, 16
X = torch.randn(M, LDA, device="cuda")
W = torch.randn(K, N, device="cuda")
Y = torch.empty_like(X)
nbytes = X.numel() * 4


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {}
for name, fn, b in (("sum", lambda: X.sum(), nbytes), ("copy", lambda: Y.copy_(X), 2 * nbytes),
                    ("mm_f32", lambda: X[:, :K] @ W, nbytes),
                    ("colsum", lambda: X.sum(0), nbytes)):
    ms = timeit(fn)
    res[name + "_ms"] = ms
    res[name + "_GBs"] = b / ms / 1e6
print(json.dumps(res))
