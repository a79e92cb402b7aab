"""X-stream pass time against the row count (diagnostic tool, one GPU): the first layer's
products Z = X W1 (pgcn_gemm_xstream) and W1.grad = X^T dZ (pgcn_gemm_tn_xstream, with its
ordered reduce) over reddit's feature width (K = 602, N = 16) at M = the full graph's rows and
its 1/2, 1/4, 1/8 (an edge-cut rank's share at W = 2, 4, 8).  Times each call by HIP events on
the stream it runs on, median of `reps`, and prints the fixed part: t(M) - t(M_full) * M /
M_full.  One JSON line.

usage: python3 tools/xs_scale.py [reps=30] [library path (A/B: another build, as PGCN_LIB)]
                                [nocheck]
"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2:
    os.environ["PGCN_LIB"] = os.path.abspath(sys.argv[2])
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

pg = helpers.pgcn()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
K, N, MF = 602, 16, 232965
lda = (K + 3) // 4 * 4
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(1)
A = torch.randn(MF, lda, device=dev, generator=g)
W = torch.randn(K, N, device=dev, generator=g)
dZ = torch.randn(MF, N, device=dev, generator=g)
C = torch.empty(MF, N, device=dev)
WG = torch.empty(K, N, device=dev)
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
s = torch.cuda.Stream()
vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
sp = ctypes.c_void_p(s.cuda_stream)


def nn(M):
    pg.check(pg.lib.pgcn_gemm_xstream(M, N, K, vp(A), lda, vp(W), N, 0, vp(C), N, None,
                                      ctypes.c_float(1.0), sp), "xstream")


def tn(M):
    pg.check(pg.lib.pgcn_gemm_tn_xstream(M, N, K, vp(A), lda, vp(dZ), N, vp(WG), N, None,
                                         ctypes.c_float(1.0), vp(ws), sp), "tn")


def timed(fn, M):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    with torch.cuda.stream(s):
        for _ in range(3):
            fn(M)
        for a, b in ev:
            a.record(s)
            fn(M)
            b.record(s)
    s.synchronize()
    t = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return t[len(t) // 2]


out = {}
# the products against torch's fp32 (a sanity check of the build under test, not a parity test)
for M in (MF, MF // 8):
    with torch.cuda.stream(s):
        nn(M)
        tn(M)
    s.synchronize()
    Xm = A[:M, :K].double()
    e_nn = ((C[:M] - (Xm @ W.double()).float()).abs().max() / C[:M].abs().max()).item()
    e_tn = ((WG - (Xm.T @ dZ[:M].double()).float()).abs().max() / WG.abs().max()).item()
    out[f"check_M{M}"] = {"nn_rel": e_nn, "tn_rel": e_tn}
    if "nocheck" not in sys.argv[3:]:  # (timing-only ablation builds compute nothing)
        assert e_nn < 1e-5 and e_tn < 1e-5, out
arms = (("nn", nn), ("tn", tn))
if not os.environ.get("XS_RING_ONLY"):  # the register-streamed kernels too (xstream_ring 0)
    def _plain(fn):
        def run(M):
            pg.lib.pgcn_debug_set(b"xstream_ring", 0)
            try:
                fn(M)
            finally:
                pg.lib.pgcn_debug_set(b"xstream_ring", 1)
        return run
    arms += (("nn_plain", _plain(nn)), ("tn_plain", _plain(tn)))
for name, fn in arms:
    full = timed(fn, MF)
    row = {"full_us": round(full, 1)}
    for d in (2, 4, 8, 16, 32, 64):
        M = MF // d
        t = timed(fn, M)
        row[f"1/{d}_us"] = round(t, 1)
        row[f"1/{d}_fixed_us"] = round(t - full / d, 1)
    out[name] = row
    print(name, row, file=sys.stderr)
print(json.dumps(out))
