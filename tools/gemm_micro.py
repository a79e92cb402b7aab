"""X-stream GEMM micro-benchmark on the reddit shape (run on the GPU box).

Times pgcn_gemm (Z = drop(X) W1, the forward of the first layer) and pgcn_gemm_tn (W1.grad =
drop(X)^T dZ) on X = [232965][604] fp32 (602 features), masked and unmasked, for the N <= 16
streaming kernels (gemm_variant 0) and the general kernels (gemm_variant 1), with HIP events
on torch's stream.  Reports ms per call, GB/s of algorithmic bytes (X + mask bits + the small
operands) and the max relative difference between the two kernel families.  One JSON line.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

pg = helpers.pgcn()
lib = pg.lib
M, K, N, LDA = 232965, 602, 16, 604
dev = "cuda"
torch.manual_seed(0)
X = torch.zeros(M, LDA, device=dev)
X[:, :K] = torch.randn(M, K, device=dev)
W = torch.randn(K, N, device=dev)
G = torch.randn(M, N, device=dev)
nbits = M * K
mask = torch.randint(-2**62, 2**62, ((nbits + 63) // 64 + 1,), dtype=torch.int64, device=dev)
Z = torch.empty(M, N, device=dev)
dW = torch.empty(K, N, device=dev)
ws = torch.empty(lib.pgcn_gemm_tn_workspace(M, N, K) // 4 + 64, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def nn(masked):
    pg.check(lib.pgcn_gemm(M, N, K, vp(X), LDA, vp(W), N, 0, vp(Z), N,
                           vp(mask) if masked else None, 0, K, 2.0, st), "gemm")


def tn(masked):
    pg.check(lib.pgcn_gemm_tn(M, N, K, vp(X), LDA, vp(G), N, vp(dW), N,
                              vp(mask) if masked else None, 0, K, 2.0, vp(ws), st), "tn")


nib = torch.empty(M, 16, dtype=torch.int64, device=dev)


def xnn(masked):
    if masked:
        pg.check(lib.pgcn_mask_nibbles(vp(mask), 0, K, M, K, vp(nib), st), "nib")
    pg.check(lib.pgcn_gemm_xstream(M, N, K, vp(X), LDA, vp(W), N, 0, vp(Z), N,
                                   vp(nib) if masked else None, 2.0, st), "xnn")


def xtn(masked):
    pg.check(lib.pgcn_gemm_tn_xstream(M, N, K, vp(X), LDA, vp(G), N, vp(dW), N,
                                      vp(nib) if masked else None, 2.0, vp(ws), st), "xtn")


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


x_bytes = 4.0 * M * K
res = {"M": M, "K": K, "N": N}
outs = {}
for variant in (0, 1):
    lib.pgcn_debug_set(b"gemm_variant", variant)
    for masked in (False, True):
        tag = f"v{variant}_{'masked' if masked else 'plain'}"
        b = x_bytes + 4.0 * M * N + (nbits / 8 if masked else 0)
        ms = timeit(lambda: nn(masked))
        res[f"nn_{tag}_ms"] = ms
        res[f"nn_{tag}_GBs"] = b / ms / 1e6
        outs[("nn", variant, masked)] = Z.clone()
        ms = timeit(lambda: tn(masked))
        res[f"tn_{tag}_ms"] = ms
        res[f"tn_{tag}_GBs"] = b / ms / 1e6
        outs[("tn", variant, masked)] = dW.clone()
lib.pgcn_debug_set(b"gemm_variant", 0)
for masked in (False, True):  # the engine's path: xstream kernels, nibble masks
    tag = f"xs_{'masked' if masked else 'plain'}"
    b = x_bytes + 4.0 * M * N + (M * 128 if masked else 0)
    ms = timeit(lambda: xnn(masked))
    res[f"nn_{tag}_ms"] = ms
    res[f"nn_{tag}_GBs"] = b / ms / 1e6
    outs[("xnn", masked)] = Z.clone()
    ms = timeit(lambda: xtn(masked))
    res[f"tn_{tag}_ms"] = ms
    res[f"tn_{tag}_GBs"] = b / ms / 1e6
    outs[("xtn", masked)] = dW.clone()
for kind in ("nn", "tn"):
    for masked in (False, True):
        a, b = outs[("x" + kind, masked)], outs[(kind, 1, masked)]
        res[f"x{kind}_{'masked' if masked else 'plain'}_vs_v1_max_rel"] = (
            ((a - b).abs().max() / b.abs().max()).item())
for kind in ("nn", "tn"):
    for masked in (False, True):
        a, b = outs[(kind, 0, masked)], outs[(kind, 1, masked)]
        res[f"{kind}_{'masked' if masked else 'plain'}_v0_vs_v1_max_rel"] = (
            ((a - b).abs().max() / b.abs().max()).item())
ref = X[:, :K] @ W
res["nn_plain_vs_torch_max_rel"] = ((outs[("nn", 0, False)] - ref).abs().max() /
                                    ref.abs().max()).item()
print(json.dumps(res))
