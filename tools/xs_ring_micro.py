"""X-stream kernels on the reddit shape through the C ABI (run on the GPU box): ms per call of
pgcn_gemm_xstream (Z = drop(X) W1, unmasked and with nibble keep bits) and pgcn_gemm_tn_xstream
(W1.grad = drop(X)^T dZ) for each value of the "xstream_ring" knob (1: loader / MFMA-wave
split, k_xstream_lds.hip, TN in its K-split form or not; 0: register-streamed kernels; diag 1 / 2: consumers without MFMAs / loaders without DMAs, timing only), with HIP
events on torch's stream.
One JSON line.

usage: python3 tools/xs_ring_micro.py [lda=604]
"""
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
M, K, N = 232965, 602, 16
LDA = int(sys.argv[1]) if len(sys.argv) > 1 else 604
dev = "cuda"
torch.manual_seed(0)
X = torch.zeros(M, LDA, device=dev)
X[:, :K] = torch.randn(M, K, device=dev)
W = torch.randn(K, N, device=dev)
G = torch.randn(M, N, device=dev)
nib = torch.randint(-2**62, 2**62, (M, 16), dtype=torch.int64, device=dev)
Z = torch.empty(M, N, device=dev)
dW = torch.empty(K, N, device=dev)
ws = torch.empty(lib.pgcn_gemm_tn_workspace(M, N, K) // 4 + 64, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def nn(masked):
    pg.check(lib.pgcn_gemm_xstream(M, N, K, vp(X), LDA, vp(W), N, 0, vp(Z), N,
                                   vp(nib) if masked else None, 2.0, st), "xnn")


def tn(masked):
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


out = {"M": M, "K": K, "lda": LDA}
for ring, split, diag in ((1, 1, 0), (1, 0, 0), (0, 0, 0), (1, 1, 1), (1, 1, 2)):
    with helpers.knobs(pg, xstream_ring=ring, xstream_tn_split=split, xstream_ring_diag=diag):
        for name, fn in (("nn", lambda: nn(False)), ("nn_masked", lambda: nn(True)),
                         ("tn_masked", lambda: tn(True))):
            out[f"{name}_ring{ring}_split{split}" + (f"_diag{diag}" if diag else "") + "_ms"] = \
                round(timeit(fn), 4)
print(json.dumps(out))
