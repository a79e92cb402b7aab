"""Kernel-level parity of the HIP path through the C ABI (include/pgcn.h) vs the oracle.

Device memory comes from torch (plumbing only); every compute call goes through libpgcn.so.
Tolerances: integer/bit work bit-exact (dropout masks, RNG states, CSR transposes); Adam
bit-exact (double temporaries as hpdga optim.cpp); sparse-X SpMM bit-exact (CSR order, no
FMA); GraphSum / MFMA GEMMs within 1e-5 relative to sum|terms| (fp32 reordering only).
"""
import ctypes

import numpy as np
import pytest
import torch

import helpers

pytestmark = pytest.mark.gpu

DEV = "cuda"


def vp(t):
    return ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def random_graph(n, avg_deg, seed, hubs=0, hub_deg=0, empty_rows=0):
    """Symmetric random graph in the hpdga CSR form (self loop first, duplicates allowed)."""
    rng = np.random.default_rng(seed)
    m = n * avg_deg // 2
    u = rng.integers(0, n, m)
    v = rng.integers(0, n, m)
    if hubs:
        hu = rng.integers(0, n, hubs)
        extra_u = np.repeat(hu, hub_deg)
        extra_v = rng.integers(0, n, hubs * hub_deg)
        u, v = np.concatenate([u, extra_u]), np.concatenate([v, extra_v])
    keep = u != v
    u, v = u[keep], v[keep]
    src = np.concatenate([u, v, np.arange(n)])
    dst = np.concatenate([v, u, np.arange(n)])
    order = np.lexsort((dst, src != dst, src))  # self loop first within a row
    src, dst = src[order], dst[order]
    indptr = np.zeros(n + 1, np.int64)
    np.add.at(indptr, src + 1, 1)
    indptr = np.cumsum(indptr).astype(np.int32)
    return indptr, dst.astype(np.int32)


def _merge_graphs(ip1, ix1, ip2, ix2):
    """Row-wise concatenation of two CSR patterns on the same nodes (symmetric if both are)."""
    n = len(ip1) - 1
    ip = np.zeros(n + 1, np.int64)
    ip[1:] = np.cumsum(np.diff(ip1) + np.diff(ip2))
    ix = np.concatenate([np.concatenate([ix1[ip1[i]:ip1[i + 1]], ix2[ip2[i]:ip2[i + 1]]])
                         for i in range(n)])
    return ip.astype(np.int32), ix.astype(np.int32)


def oracle_graphsum(indptr, indices, x, dim):
    lib = helpers.oracle()
    n = len(indptr) - 1
    out = np.zeros((n, dim), np.float32)
    xin = np.ascontiguousarray(x[:, :dim], np.float32)
    lib.or_graphsum(n, helpers.ptr(indptr), helpers.ptr(indices), helpers.ptr(xin),
                    helpers.ptr(out), dim)
    return out


def abs_bound(indptr, indices, x, dim):
    """sum_j |coef_ij * x_j| per output element (scale of the fp32 reordering error)."""
    n = len(indptr) - 1
    deg = np.diff(indptr).astype(np.float64)
    rows = np.repeat(np.arange(n), np.diff(indptr))
    coef = 1.0 / np.sqrt(deg[rows] * deg[indices])
    out = np.zeros((n, dim))
    np.add.at(out, rows, np.abs(coef)[:, None] * np.abs(x[indices, :dim]))
    return out


@pytest.mark.parametrize("n,deg,dim,hubs", [
    (3000, 6, 16, 0),        # cora-like, plain schedule
    (120000, 40, 16, 20),    # table > 4 MB: XCD-blocked schedule, hub rows split in chunks
    (20000, 12, 41, 5),      # C = 41 (ld 44): whole-wave items
    (5000, 8, 3, 2),         # pubmed-like C = 3
    (5000, 8, 7, 2),         # cora C = 7
    (20000, 10, 128, 3),     # 4-layer hidden 128
    (120000, 40, 16, 20),    # the same graph, LDS ring path (the table exceeds 1 MB)
    (150000, 60, 16, 40),    # LDS ring path, more hubs (spread rows over 2..16 lane groups)
])
def test_graphsum_vs_oracle(pgcn, n, deg, dim, hubs):
    indptr, indices = random_graph(n, deg, seed=n + dim, hubs=hubs, hub_deg=3000)
    ld = (dim + 3) // 4 * 4
    rng = np.random.default_rng(7)
    x = np.zeros((n, ld), np.float32)
    x[:, :dim] = rng.standard_normal((n, dim)).astype(np.float32)
    g = ctypes.c_void_p()
    pgcn.check(pgcn.lib.pgcn_graph_create(n, helpers.ptr(indptr), helpers.ptr(indices),
                                          ctypes.byref(g)), "graph_create")
    xin = torch.from_numpy(x).to(DEV)
    out = torch.full((n, ld), float("nan"), device=DEV)
    for _ in range(2):  # twice: partial buffers and schedules are reused across calls
        pgcn.check(pgcn.lib.pgcn_graphsum(g, vp(xin), ld, vp(out), ld, dim, stream()), "graphsum")
    torch.cuda.synchronize()
    ours = out.cpu().numpy()
    ref = oracle_graphsum(indptr, indices, x, dim)
    bound = abs_bound(indptr, indices, x, dim)
    err = np.abs(ours[:, :dim] - ref)
    assert (err <= 1e-5 * bound + 1e-30).all(), f"max err/bound {(err / (bound + 1e-30)).max():.3g}"
    np.testing.assert_array_equal(ours[:, dim:], 0.0)  # padding columns stay zero
    # deterministic: identical bits on a rerun
    out2 = torch.empty_like(out)
    pgcn.lib.pgcn_graphsum(g, vp(xin), ld, vp(out2), ld, dim, stream())
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    pgcn.lib.pgcn_graph_destroy(g)


@pytest.mark.parametrize("n,deg,dim,hubs", [
    (120000, 40, 16, 20),    # LDS ring path
    (150000, 60, 16, 40),    # more hubs (spread rows)
    (120000, 40, 128, 20),   # 8 ring passes (the 4-layer model's width)
])
def test_graphsum_ring_pair_vs_oracle(pgcn, n, deg, dim, hubs):
    """ring_pair 1: rowsets in lockstep pairs, both blocks' table reads in flight
    (k_graphsum_ring<16, true>): the oracle's sums within the reordering bound, reruns
    bit-identical."""
    with helpers.knobs(pgcn, ring_pair=1):
        test_graphsum_vs_oracle(pgcn, n, deg, dim, hubs)


@pytest.mark.parametrize("n,deg,dim,hubs", [
    (120000, 40, 16, 20),    # LDS ring path
    (150000, 60, 16, 40),    # more hubs (spread rows)
    (120000, 40, 128, 20),   # 8 ring passes
])
def test_graphsum_ring_window2_vs_oracle(pgcn, n, deg, dim, hubs):
    """ring_window 2: visits read two resident slices and the loader runs two slices ahead
    (k_graphsum_ring<16, false, 2>): the oracle's sums within the reordering bound, reruns
    bit-identical."""
    with helpers.knobs(pgcn, ring_window=2):
        test_graphsum_vs_oracle(pgcn, n, deg, dim, hubs)


@pytest.mark.parametrize("dim", [16, 7, 41])
def test_graphsum_split_rows_in_kernel(pgcn, dim):
    """Rows longer than one work item on the plain path (cora's hubs): gs_split 1 (default: the
    last of a row's items to finish adds the row's slots, one launch) gives gs_split 0's bits
    (the combine launch) on every call at the same item length (gs_item_iters 32) -- the arrival
    counters are left at zero for the next one; short items (8 iterations: more split rows,
    more arrivals), gs_split 2 (long rows as one item) and the default gs_split 3 (rows of up
    to 8 workgroup iterations summed by one workgroup, longer ones split with arrivals) agree
    with the oracle and repeat their bits."""
    n = 4000
    # hubs of ~300 (workgroup items at d <= 16) and ~2,000 neighbours (split at every width)
    indptr, indices = random_graph(n, 6, seed=dim, hubs=12, hub_deg=300)
    i2, x2 = random_graph(n, 1, seed=dim + 1, hubs=6, hub_deg=2000)
    indptr, indices = _merge_graphs(indptr, indices, i2, x2)
    ld = (dim + 3) // 4 * 4
    x = np.zeros((n, ld), np.float32)
    x[:, :dim] = np.random.default_rng(dim).standard_normal((n, dim)).astype(np.float32)
    xin = torch.from_numpy(x).to(DEV)
    outs = {}
    try:
        for mode in (0, 1, 2, 3, 4, 5):  # mode 5: the defaults (item length by shape)
            assert pgcn.lib.pgcn_debug_set(b"gs_split", (0, 1, 2, 1, 3, 3)[mode]) == 0
            assert pgcn.lib.pgcn_debug_set(b"gs_item_iters", (32, 32, 32, 8, 8, 0)[mode]) == 0
            g = ctypes.c_void_p()
            pgcn.check(pgcn.lib.pgcn_graph_create(n, helpers.ptr(indptr), helpers.ptr(indices),
                                                  ctypes.byref(g)), "graph_create")
            pgcn.reset_path_counts()
            res = []
            for _ in range(3):
                out = torch.full((n, ld), float("nan"), device=DEV)
                pgcn.check(pgcn.lib.pgcn_graphsum(g, vp(xin), ld, vp(out), ld, dim, stream()), "gs")
                res.append(out)
            torch.cuda.synchronize()
            outs[mode] = (res, pgcn.path_counts()["launches"])
            pgcn.lib.pgcn_graph_destroy(g)
    finally:
        pgcn.lib.pgcn_debug_set(b"gs_split", 3)
        pgcn.lib.pgcn_debug_set(b"gs_item_iters", 0)
    for r in outs[1][0] + outs[0][0][1:]:
        assert torch.equal(r, outs[0][0][0])
    assert outs[1][1] < outs[0][1], (outs[1][1], outs[0][1])  # no combine launches
    ref = oracle_graphsum(indptr, indices, x, dim)
    bound = abs_bound(indptr, indices, x, dim)
    for mode in (3, 4, 5):
        for r in outs[mode][0][1:]:
            assert torch.equal(r, outs[mode][0][0])
    for mode in (0, 2, 3, 4, 5):
        err = np.abs(outs[mode][0][2].cpu().numpy()[:, :dim] - ref)
        assert (err <= 1e-5 * bound + 1e-30).all(), (mode, (err / (bound + 1e-30)).max())


@pytest.mark.parametrize("kind", ["coef", "random", "directed"])
def test_graphsum_with_values(pgcn, kind):
    """pgcn_graph_create_values (the reference's GraphSum contract: any dev_graph_value array,
    include/module.cuh:82): the parser's own coefficients take the LDS ring path and give
    pgcn_graph_create's bits; arbitrary values (and a directed pattern) take the gather
    kernels; every case against a float64 CSR product of the given values."""
    n, dim = 120000, 16
    indptr, indices = random_graph(n, 30, seed=3, hubs=10, hub_deg=2000)
    if kind == "directed":  # drop every other slot of each row past the self loop
        keep = np.ones(len(indices), bool)
        keep[1::2] = False
        rows = np.repeat(np.arange(n), np.diff(indptr))
        keep[indptr[:-1]] = True
        indices = np.ascontiguousarray(indices[keep])
        indptr = np.zeros(n + 1, np.int32)
        np.add.at(indptr, rows[keep] + 1, 1)
        indptr = np.ascontiguousarray(np.cumsum(indptr).astype(np.int32))
    deg = np.diff(indptr)
    rows = np.repeat(np.arange(n), np.diff(indptr))
    if kind == "coef":
        # graph_coef's expression (src/parser.cpp:164-181): float sqrt of the int product,
        # double division, stored to float
        prod = (deg[rows].astype(np.int64) * deg[indices].astype(np.int64)).astype(np.float32)
        vals = (1.0 / np.sqrt(prod).astype(np.float64)).astype(np.float32)
        g0 = ctypes.c_void_p()
        pgcn.check(pgcn.lib.pgcn_graph_create(n, helpers.ptr(indptr), helpers.ptr(indices),
                                              ctypes.byref(g0)), "graph_create")
    else:
        vals = np.random.default_rng(9).uniform(-1, 1, len(indices)).astype(np.float32)
    vals = np.ascontiguousarray(vals)
    g = ctypes.c_void_p()
    st = pgcn.lib.pgcn_graph_create_values(n, helpers.ptr(indptr), helpers.ptr(indices),
                                           helpers.ptr(vals), ctypes.byref(g))
    pgcn.check(st, "graph_create_values")
    x = np.random.default_rng(4).standard_normal((n, dim)).astype(np.float32)
    xin = torch.from_numpy(x).to(DEV)
    out = torch.full((n, dim), float("nan"), device=DEV)
    pgcn.reset_path_counts()
    pgcn.check(pgcn.lib.pgcn_graphsum(g, vp(xin), dim, vp(out), dim, dim, stream()), "graphsum")
    torch.cuda.synchronize()
    paths = pgcn.path_counts()
    ref = np.zeros((n, dim))
    np.add.at(ref, rows, vals[:, None].astype(np.float64) * x[indices].astype(np.float64))
    bound = np.zeros((n, dim))
    np.add.at(bound, rows, np.abs(vals[:, None].astype(np.float64) * x[indices]))
    err = np.abs(out.cpu().numpy() - ref)
    assert (err <= 1e-5 * bound + 1e-30).all(), (err / (bound + 1e-30)).max()
    if kind == "coef":
        # the parser's coefficients bit for bit: the ring path, pgcn_graph_create's bits
        assert paths["gs_ring"] >= 1, paths
        out0 = torch.empty_like(out)
        pgcn.check(pgcn.lib.pgcn_graphsum(g0, vp(xin), dim, vp(out0), dim, dim, stream()), "gs0")
        torch.cuda.synchronize()
        assert torch.equal(out, out0)
        pgcn.lib.pgcn_graph_destroy(g0)
    else:
        assert paths["gs_ring"] == 0 and paths["gs_gather"] >= 1, paths
    pgcn.lib.pgcn_graph_destroy(g)


@pytest.mark.parametrize("blocks", [2, 8, 16, 32])
def test_graphsum_lds_column_blocks(pgcn, blocks):
    """The LDS ring schedule with other column-block counts than the shape rule picks (4 for
    square graphs, 8 for row subsets): the same sums (XCD mapping: workgroup w serves block
    w % B).  At 32 blocks: 7-8 slices per block, so the ring's prologue and drain (the loader's
    last W - 1 iterations) make up much of each sweep."""
    assert pgcn.lib.pgcn_debug_set(b"lds_blocks", blocks) == 0
    try:
        n, dim = 120000, 16
        indptr, indices = random_graph(n, 40, seed=blocks, hubs=20, hub_deg=3000)
        x = np.random.default_rng(3).standard_normal((n, dim)).astype(np.float32)
        g = ctypes.c_void_p()
        pgcn.check(pgcn.lib.pgcn_graph_create(n, helpers.ptr(indptr), helpers.ptr(indices),
                                              ctypes.byref(g)), "graph_create")
        xin = torch.from_numpy(x).to(DEV)
        out = torch.full((n, dim), float("nan"), device=DEV)
        pgcn.check(pgcn.lib.pgcn_graphsum(g, vp(xin), dim, vp(out), dim, dim, stream()), "gs")
        torch.cuda.synchronize()
        ref = oracle_graphsum(indptr, indices, x, dim)
        bound = abs_bound(indptr, indices, x, dim)
        err = np.abs(out.cpu().numpy() - ref)
        assert (err <= 1e-5 * bound + 1e-30).all()
        pgcn.lib.pgcn_graph_destroy(g)
    finally:
        pgcn.lib.pgcn_debug_set(b"lds_blocks", 0)


@pytest.mark.parametrize("gather16", [0, 1, 2])
def test_graphsum_blocked_gather16(pgcn, gather16):
    """d = 16 on the plain path's XCD-blocked layout (the LDS ring switched off by lds_min_kb):
    k_graphsum16 (gs16_gather 1) and k_graphsum<4, 16> with interleaved neighbour slots
    (gs16_gather 2; 0 = by shape, here the interleaved one: 40 slots per row over 8 column
    blocks), hub rows split over several items, against the oracle; the same bits on a
    rerun."""
    n, dim = 120000, 16
    indptr, indices = random_graph(n, 40, seed=11, hubs=20, hub_deg=3000)
    x = np.random.default_rng(5).standard_normal((n, dim)).astype(np.float32)
    with helpers.knobs(pgcn, lds_min_kb=1 << 30, gs16_gather=gather16):
        g = ctypes.c_void_p()
        pgcn.check(pgcn.lib.pgcn_graph_create(n, helpers.ptr(indptr), helpers.ptr(indices),
                                              ctypes.byref(g)), "graph_create")
        xin = torch.from_numpy(x).to(DEV)
        pgcn.reset_path_counts()
        outs = []
        for _ in range(2):
            out = torch.full((n, dim), float("nan"), device=DEV)
            pgcn.check(pgcn.lib.pgcn_graphsum(g, vp(xin), dim, vp(out), dim, dim, stream()), "gs")
            outs.append(out)
        torch.cuda.synchronize()
        paths = pgcn.path_counts()
        pgcn.lib.pgcn_graph_destroy(g)
    assert paths["gs_ring"] == 0 and paths["gs_gather"] == 2, paths
    ref = oracle_graphsum(indptr, indices, x, dim)
    bound = abs_bound(indptr, indices, x, dim)
    err = np.abs(outs[0].cpu().numpy() - ref)
    assert (err <= 1e-5 * bound + 1e-30).all(), (err / (bound + 1e-30)).max()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("dim,ld", [(128, 128), (41, 44), (24, 24)])
def test_graphsum_lds_wide_rows(pgcn, dim, ld):
    """Rows wider than 16 on a graph that takes the LDS GraphSum: one 16-column LDS pass per
    chunk (the last one overlapping), against the oracle; padding columns stay zero;
    deterministic (the same bits on a rerun)."""
    n = 120000
    indptr, indices = random_graph(n, 30, seed=dim, hubs=10, hub_deg=3000)
    x = np.zeros((n, ld), np.float32)
    x[:, :dim] = np.random.default_rng(dim).standard_normal((n, dim))
    g = ctypes.c_void_p()
    pgcn.check(pgcn.lib.pgcn_graph_create(n, helpers.ptr(indptr), helpers.ptr(indices),
                                          ctypes.byref(g)), "graph_create")
    xin = torch.from_numpy(x).to(DEV)
    outs = []
    # runs 0, 1: every pass's table prescaled by one launch (the batched prescale); then each
    # 16-column pass as a d = 16 call of its own (its own prescale launch): the same products,
    # so the same bits
    for _ in range(2):
        out = torch.full((n, ld), float("nan"), device=DEV)
        pgcn.check(pgcn.lib.pgcn_graphsum(g, vp(xin), ld, vp(out), ld, dim, stream()), "gs")
        torch.cuda.synchronize()
        outs.append(out)
    assert torch.equal(outs[0], outs[1])
    for c0 in range(0, dim, 16):
        c = min(c0, ld - 16)
        one = torch.full((n, 16), float("nan"), device=DEV)
        pgcn.check(pgcn.lib.pgcn_graphsum(g, vp(xin[:, c:]), ld, vp(one), 16, 16, stream()), "gs16")
        torch.cuda.synchronize()
        assert torch.equal(one, outs[0][:, c:c + 16]), c
    ours = outs[0].cpu().numpy()
    ref = oracle_graphsum(indptr, indices, x, dim)
    bound = abs_bound(indptr, indices, x, dim)
    assert (np.abs(ours[:, :dim] - ref) <= 1e-5 * bound + 1e-30).all()
    np.testing.assert_array_equal(ours[:, dim:], 0.0)
    pgcn.lib.pgcn_graph_destroy(g)


def test_graphsum_linearity_large(pgcn):
    """Size-independent property at reddit-like density: GraphSum(a x + b y) == a GS(x) + b GS(y)."""
    n = 200000
    indptr, indices = random_graph(n, 100, seed=3, hubs=10, hub_deg=20000)
    g = ctypes.c_void_p()
    pgcn.check(pgcn.lib.pgcn_graph_create(n, helpers.ptr(indptr), helpers.ptr(indices),
                                          ctypes.byref(g)), "graph_create")
    x = torch.randn(n, 16, device=DEV)
    y = torch.randn(n, 16, device=DEV)
    outs = []
    for inp in (x, y, 2.0 * x - 3.0 * y):
        o = torch.empty(n, 16, device=DEV)
        pgcn.lib.pgcn_graphsum(g, vp(inp), 16, vp(o), 16, 16, stream())
        outs.append(o)
    torch.cuda.synchronize()
    lhs, rhs = outs[2], 2.0 * outs[0] - 3.0 * outs[1]
    scale = (outs[0].abs() + outs[1].abs()).max()
    assert (lhs - rhs).abs().max() <= 1e-5 * scale
    # ones in -> row sums of coefficients (checked against float64 numpy)
    ones = torch.ones(n, 16, device=DEV)
    o = torch.empty(n, 16, device=DEV)
    pgcn.lib.pgcn_graphsum(g, vp(ones), 16, vp(o), 16, 16, stream())
    torch.cuda.synchronize()
    deg = np.diff(indptr).astype(np.float64)
    rows = np.repeat(np.arange(n), np.diff(indptr))
    rs = np.bincount(rows, weights=1.0 / np.sqrt(deg[rows] * deg[indices]), minlength=n)
    np.testing.assert_allclose(o[:, 0].cpu().numpy(), rs, rtol=2e-5)
    pgcn.lib.pgcn_graph_destroy(g)


def mask_bits(mask_words, n):
    b = np.unpackbits(mask_words.view(np.uint8), bitorder="little")
    return b[:n].astype(bool)


def test_dropout_masks_bit_exact(pgcn):
    """Chunk states + GPU mask kernel reproduce the sequential xorshift128+ stream exactly,
    across two 'epochs' (state advance by the period through the byte tables)."""
    lib = helpers.oracle()
    offset, n, period = 12345, 100_003, 250_007
    # sequential reference: draws offset .. offset+n (epoch 1) and offset+period .. (epoch 2)
    s = np.zeros(2, np.uint64)
    lib.or_rng_seed(helpers.ptr(s))
    seq = np.array([lib.or_rng_next(helpers.ptr(s)) for _ in range(offset + period + n)], np.int64)
    thr = int(np.float32(0.5) * np.float32(0x7FFFFFFF))
    ref1 = seq[offset:offset + n] >= thr
    ref2 = seq[offset + period:offset + period + n] >= thr
    nch = (n + 63) // 64
    states = np.zeros((nch, 2), np.uint64)
    st = pgcn.rng_jump(pgcn.rng_seed(), offset)
    for c in range(nch):
        states[c] = st
        st = pgcn.rng_jump(st, 64)
    table = torch.from_numpy(pgcn.rng_jump_table(period).view(np.int64)).to(DEV)
    dstates = torch.from_numpy(states.view(np.int64)).to(DEV)
    mask = torch.zeros(nch + 1, dtype=torch.int64, device=DEV)
    for ref in (ref1, ref2):
        pgcn.check(pgcn.lib.pgcn_dropout_mask(vp(dstates), nch, n, 0, 0.5, vp(mask), vp(table),
                                              stream()), "dropout_mask")
        torch.cuda.synchronize()
        ours = mask_bits(mask.cpu().numpy()[:nch].view(np.uint64), n)
        np.testing.assert_array_equal(ours, ref)


def test_dropout_apply(pgcn):
    n = 10_007
    x = torch.randn(n, device=DEV)
    words = torch.randint(-2**62, 2**62, ((n + 63) // 64 + 1,), dtype=torch.int64, device=DEV)
    ref = x.cpu().numpy().copy()
    bits = mask_bits(words.cpu().numpy().view(np.uint64), n)
    ref = ref * np.where(bits, np.float32(2.0), np.float32(0.0))
    pgcn.lib.pgcn_dropout_apply(vp(x), n, vp(words), 2.0, stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(x.cpu().numpy(), ref.astype(np.float32))


def mask_window(mask, base, M, K):
    """bits base .. base + M*K of a flat bitmap as an (M, K) bool array"""
    return mask_bits(mask, base + M * K)[base:].reshape(M, K)


# every shape on the kernel the product dispatches it to: N <= 16 streaming (X-stream) kernels,
# 33..128 the wide MFMA kernels, the general MFMA kernels elsewhere (17..32, > 128)
@pytest.mark.parametrize("M,N,K,drop,base", [(1000, 16, 602, True, 0), (777, 41, 16, False, 0),
                                             (400, 24, 100, True, 3), (999, 32, 602, True, 0),
                                             (513, 16, 41, False, 0), (300, 128, 128, False, 0),
                                             (64, 16, 1433, True, 0), (2011, 16, 602, True, 37),
                                             (99, 13, 70, True, 63), (5, 16, 602, True, 1),
                                             (500, 200, 72, True, 5), (300, 300, 41, False, 0),
                                             (257, 136, 16, False, 0)])
def test_gemm_nn(pgcn, M, N, K, drop, base):
    rng = np.random.default_rng(M + N + K)
    lda = (K + 3) // 4 * 4
    A = np.zeros((M, lda), np.float32)
    A[:, :K] = rng.standard_normal((M, K))
    A[:, K:] = np.nan  # ld padding is never read into the result
    B = rng.standard_normal((K, N)).astype(np.float32)
    # exactly as many words as the bits need: the kernels must not read past the bitmap
    mask = rng.integers(0, 2**63, (base + M * K + 63) // 64, dtype=np.uint64)
    Ae = A[:, :K].astype(np.float64)
    if drop:
        Ae = Ae * np.where(mask_window(mask, base, M, K), 2.0, 0.0)
    ref = Ae @ B.astype(np.float64)
    dA, dB = torch.from_numpy(A).to(DEV), torch.from_numpy(B).to(DEV)
    dm = torch.from_numpy(mask.view(np.int64)).to(DEV)
    ldc = (N + 3) // 4 * 4
    C = torch.full((M, ldc), float("nan"), device=DEV)
    pgcn.check(pgcn.lib.pgcn_gemm(M, N, K, vp(dA), lda, vp(dB), N, 0, vp(C), ldc,
                                  vp(dm) if drop else None, base, K, 2.0, stream()), "gemm")
    # transposed B: C2 = A * (B^T)^T with B^T stored [N][K]
    dBt = torch.from_numpy(np.ascontiguousarray(B.T)).to(DEV)
    C2 = torch.empty((M, ldc), device=DEV)
    pgcn.check(pgcn.lib.pgcn_gemm(M, N, K, vp(dA), lda, vp(dBt), K, 1, vp(C2), ldc,
                                  vp(dm) if drop else None, base, K, 2.0, stream()), "gemm_t")
    torch.cuda.synchronize()
    bound = np.abs(Ae) @ np.abs(B.astype(np.float64))
    for out in (C, C2):
        o = out.cpu().numpy()
        assert (np.abs(o[:, :N] - ref) <= 1e-5 * bound + 1e-30).all()
        np.testing.assert_array_equal(o[:, N:], 0.0)


@pytest.mark.parametrize("M,N,K,drop,base", [(5000, 16, 602, True, 0), (3000, 41, 16, False, 0),
                                             (2000, 24, 100, True, 3), (3001, 32, 602, True, 0),
                                             (2000, 128, 128, False, 0), (100, 16, 1433, True, 0),
                                             (70000, 16, 602, False, 0), (4099, 16, 602, True, 29),
                                             (333, 16, 200, True, 63), (7, 11, 602, True, 5),
                                             (3000, 128, 602, True, 0), (2000, 80, 300, True, 3),
                                             (1000, 200, 72, True, 3), (600, 136, 16, False, 0)])
def test_gemm_tn(pgcn, M, N, K, drop, base):
    rng = np.random.default_rng(M + 3 * N + K)
    lda = (K + 3) // 4 * 4
    A = np.zeros((M, lda), np.float32)
    A[:, :K] = rng.standard_normal((M, K))
    A[:, K:] = np.nan
    Gm = rng.standard_normal((M, N)).astype(np.float32)
    mask = rng.integers(0, 2**63, (base + M * K + 63) // 64, dtype=np.uint64)
    Ae = A[:, :K].astype(np.float64)
    if drop:
        Ae = Ae * np.where(mask_window(mask, base, M, K), 2.0, 0.0)
    ref = Ae.T @ Gm.astype(np.float64)
    ws = torch.empty(pgcn.lib.pgcn_gemm_tn_workspace(M, N, K) // 4 + 16, device=DEV)
    dA, dG = torch.from_numpy(A).to(DEV), torch.from_numpy(Gm).to(DEV)
    dm = torch.from_numpy(mask.view(np.int64)).to(DEV)
    C = torch.full((K, N), float("nan"), device=DEV)
    pgcn.check(pgcn.lib.pgcn_gemm_tn(M, N, K, vp(dA), lda, vp(dG), N, vp(C), N,
                                     vp(dm) if drop else None, base, K, 2.0, vp(ws), stream()),
               "tn")
    torch.cuda.synchronize()
    bound = np.abs(Ae).T @ np.abs(Gm.astype(np.float64))
    assert (np.abs(C.cpu().numpy() - ref) <= 1e-5 * bound + 1e-30).all()


def nibble_mask_ref(mask, base, M, K):
    """maskT[m][j] nibble c = keep bits of (m, 64c + 4j .. +3), zero past K (numpy)"""
    bits = np.zeros((M, 1024), np.uint64)
    bits[:, :K] = mask_window(mask, base, M, K)
    nib = bits.reshape(M, 16, 16, 4)  # [m][c][j][t]: k = 64c + 4j + t
    vals = (nib << np.arange(4, dtype=np.uint64)).sum(-1)  # [m][c][j]
    out = np.zeros((M, 16), np.uint64)
    for c in range(16):
        out |= vals[:, c, :] << np.uint64(4 * c)
    return out


@pytest.mark.parametrize("M,N,K,base", [(3001, 16, 602, 0), (40009, 16, 602, 9),
                                        (1000, 16, 602, 41), (77, 12, 100, 63),
                                        (129, 16, 640, 5), (20, 3, 7, 0),
                                        # lda 628..640: 2 NN ring slots for 2 loader waves, and
                                        # >= 3 groups per workgroup (the loader
                                        # waited for its own unpublished group)
                                        (40009, 16, 636, 3), (50001, 7, 629, 0)])
def test_gemm_xstream(pgcn, M, N, K, base):
    """X-stream NN/TN kernels with nibble-layout dropout bits vs fp64 references (the loader /
    MFMA-wave split of k_xstream_lds.hip and the register-streamed kernels); the dual NN
    kernel bit-identical to the plain and masked ones; on the loader-wave shapes the flat
    bitmap (pgcn_gemm_*xstream_flat, the engine's form) bit-identical to the nibbles."""
    rng = np.random.default_rng(7 * M + K)
    lda = (K + 3) // 4 * 4
    ring = 577 <= K <= 640  # the loader / MFMA-wave kernels' shapes
    A = np.zeros((M, lda), np.float32)
    A[:, :K] = rng.standard_normal((M, K))
    A[:, K:] = np.nan
    B = rng.standard_normal((K, N)).astype(np.float32)
    Gm = rng.standard_normal((M, N)).astype(np.float32)
    mask = rng.integers(0, 2**63, (base + M * K + 63) // 64, dtype=np.uint64)
    mask = np.concatenate([mask, np.zeros(len(mask) % 2, np.uint64)])  # whole 16-B pieces (flat)
    keep = mask_window(mask, base, M, K)
    dA, dB, dG = (torch.from_numpy(a).to(DEV) for a in (A, B, Gm))
    dm = torch.from_numpy(mask.view(np.int64)).to(DEV)
    nib = torch.empty((M, 16), dtype=torch.int64, device=DEV)
    pgcn.check(pgcn.lib.pgcn_mask_nibbles(vp(dm), base, K, M, K, vp(nib), stream()), "nib")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(nib.cpu().numpy().view(np.uint64),
                                  nibble_mask_ref(mask, base, M, K))
    ldc = (N + 3) // 4 * 4
    ws = torch.empty(pgcn.lib.pgcn_gemm_tn_workspace(M, N, K) // 4 + 16, device=DEV)
    outs = {}
    for drop in (False, True):
        Ae = A[:, :K].astype(np.float64) * (np.where(keep, 2.0, 0.0) if drop else 1.0)
        C = torch.full((M, ldc), float("nan"), device=DEV)
        pgcn.check(pgcn.lib.pgcn_gemm_xstream(M, N, K, vp(dA), lda, vp(dB), N, 0, vp(C), ldc,
                                              vp(nib) if drop else None, 2.0, stream()), "xnn")
        W = torch.full((K, N), float("nan"), device=DEV)
        pgcn.check(pgcn.lib.pgcn_gemm_tn_xstream(M, N, K, vp(dA), lda, vp(dG), N, vp(W), N,
                                                 vp(nib) if drop else None, 2.0, vp(ws),
                                                 stream()), "xtn")
        # the register-streamed kernels (xstream_ring 0): NN bit-identical to the loader /
        # MFMA-wave split (default), TN the same sums in another order
        C0 = torch.full((M, ldc), float("nan"), device=DEV)
        W0 = torch.full((K, N), float("nan"), device=DEV)
        with helpers.knobs(pgcn, xstream_ring=0):
            pgcn.check(pgcn.lib.pgcn_gemm_xstream(M, N, K, vp(dA), lda, vp(dB), N, 0, vp(C0),
                                                  ldc, vp(nib) if drop else None, 2.0, stream()),
                       "xnn regs")
            pgcn.check(pgcn.lib.pgcn_gemm_tn_xstream(M, N, K, vp(dA), lda, vp(dG), N, vp(W0), N,
                                                     vp(nib) if drop else None, 2.0, vp(ws),
                                                     stream()), "xtn regs")
        torch.cuda.synchronize()
        np.testing.assert_array_equal(C0.cpu().numpy(), C.cpu().numpy())
        ref = Ae @ B.astype(np.float64)
        bound = np.abs(Ae) @ np.abs(B.astype(np.float64))
        o = C.cpu().numpy()
        assert (np.abs(o[:, :N] - ref) <= 1e-5 * bound + 1e-30).all()
        np.testing.assert_array_equal(o[:, N:], 0.0)
        ref_t = Ae.T @ Gm.astype(np.float64)
        bound_t = np.abs(Ae).T @ np.abs(Gm.astype(np.float64))
        for tn in (W, W0):  # the same products, rows summed in different orders
            assert (np.abs(tn.cpu().numpy() - ref_t) <= 1e-5 * bound_t + 1e-30).all()
        if drop and ring:
            # the flat bitmap staged by the loader waves (the engine's form on these shapes):
            # the same bits as the nibble layout
            Cf = torch.full((M, ldc), float("nan"), device=DEV)
            Wf = torch.full((K, N), float("nan"), device=DEV)
            pgcn.check(pgcn.lib.pgcn_gemm_xstream_flat(M, N, K, vp(dA), lda, vp(dB), N, 0, vp(Cf),
                                                       None, ldc, vp(dm), base, len(mask), 2.0,
                                                       stream()), "xnn flat")
            pgcn.check(pgcn.lib.pgcn_gemm_tn_xstream_flat(M, N, K, vp(dA), lda, vp(dG), N, vp(Wf),
                                                          N, vp(dm), base, len(mask), 2.0, vp(ws),
                                                          stream()), "xtn flat")
            torch.cuda.synchronize()
            assert torch.equal(Cf, C) and torch.equal(Wf, W)
        outs[drop] = C
    # the dual kernel (eval + next training product in one pass) is bit-identical to both
    C1 = torch.full((M, ldc), float("nan"), device=DEV)
    C2 = torch.full((M, ldc), float("nan"), device=DEV)
    pgcn.check(pgcn.lib.pgcn_gemm_xstream_dual(M, N, K, vp(dA), lda, vp(dB), N, 0, vp(C1), vp(C2),
                                               ldc, vp(nib), 2.0, stream()), "xnn dual")
    torch.cuda.synchronize()
    assert torch.equal(C1, outs[False]) and torch.equal(C2, outs[True])
    if ring:
        C1.fill_(float("nan"))
        C2.fill_(float("nan"))
        pgcn.check(pgcn.lib.pgcn_gemm_xstream_flat(M, N, K, vp(dA), lda, vp(dB), N, 0, vp(C1),
                                                   vp(C2), ldc, vp(dm), base, len(mask), 2.0,
                                                   stream()), "xnn dual flat")
        torch.cuda.synchronize()
        assert torch.equal(C1, outs[False]) and torch.equal(C2, outs[True])
    else:  # the flat form exists for the loader-wave kernels' shapes only
        assert pgcn.lib.pgcn_gemm_xstream_flat(M, N, K, vp(dA), lda, vp(dB), N, 0, vp(C1), None,
                                               ldc, vp(dm), base, len(mask), 2.0, stream()) != 0


def test_spmm_csr_and_csc_bit_exact(pgcn, loaded):
    """Sparse-X SpMM fwd and W-grad are bit-identical to hpdga's loops (cora features)."""
    ds = loaded["cora"]
    lib = helpers.oracle()
    n, F, p = ds.num_nodes, ds.input_dim, 16
    rng = np.random.default_rng(1)
    W = rng.standard_normal((F, p)).astype(np.float32)
    Gm = rng.standard_normal((n, p)).astype(np.float32)
    ip, ix, xv = (np.ascontiguousarray(a) for a in (ds.feat_indptr, ds.feat_indices, ds.feat_values))
    nnz = len(ix)
    mask = rng.integers(0, 2**63, (nnz + 63) // 64 + 1, dtype=np.uint64)
    xd = xv * np.where(mask_bits(mask, nnz), np.float32(2.0), np.float32(0.0)).astype(np.float32)
    ref_c = np.zeros((n, p), np.float32)
    lib.or_spmm_fwd(n, helpers.ptr(ip), helpers.ptr(ix), helpers.ptr(xd), helpers.ptr(W),
                    helpers.ptr(ref_c), p)
    ref_w = np.zeros((F, p), np.float32)
    lib.or_spmm_bwd(n, F, helpers.ptr(ip), helpers.ptr(ix), helpers.ptr(xd), helpers.ptr(ref_w),
                    helpers.ptr(Gm), p)
    cp, cr, cpos = pgcn.csr_transpose(ip, ix, F)
    t = {k: torch.from_numpy(v).to(DEV) for k, v in
         dict(ip=ip, ix=ix, xv=xv, W=W, G=Gm, cp=cp, cr=cr, cpos=cpos).items()}
    dm = torch.from_numpy(mask.view(np.int64)).to(DEV)
    c = torch.empty((n, p), device=DEV)
    wg = torch.empty((F, p), device=DEV)
    pgcn.check(pgcn.lib.pgcn_spmm_csr(n, p, vp(t["ip"]), vp(t["ix"]), vp(t["xv"]), vp(dm), 2.0,
                                      vp(t["W"]), vp(c), stream()), "spmm")
    pgcn.check(pgcn.lib.pgcn_spmm_csc_bwd(F, p, vp(t["cp"]), vp(t["cr"]), vp(t["cpos"]),
                                          vp(t["xv"]), vp(dm), 2.0, vp(t["G"]), vp(wg), stream()),
               "csc")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(c.cpu().numpy(), ref_c)
    np.testing.assert_array_equal(wg.cpu().numpy(), ref_w)


@pytest.mark.parametrize("p", [16, 41, 128])
def test_spmm_csc_long_columns_bit_exact(pgcn, p):
    """The W-grad kernel on columns of ~1,000 entries (several 256-entry LDS chunks), widths
    that are not 16 (several column groups; an ld that is not a multiple of 4): the same bits
    as hpdga's scatter loop."""
    lib = helpers.oracle()
    rng = np.random.default_rng(p)
    n, F = 3000, 37
    dense = rng.random((n, F)) < 0.33
    ip = np.concatenate([[0], np.cumsum(dense.sum(1))]).astype(np.int32)
    ix = np.nonzero(dense)[1].astype(np.int32)
    xv = rng.standard_normal(len(ix)).astype(np.float32)
    nnz = len(ix)
    Gm = rng.standard_normal((n, p)).astype(np.float32)
    mask = rng.integers(0, 2**63, (nnz + 63) // 64 + 1, dtype=np.uint64)
    xd = xv * np.where(mask_bits(mask, nnz), np.float32(2.0), np.float32(0.0)).astype(np.float32)
    ref_w = np.zeros((F, p), np.float32)
    lib.or_spmm_bwd(n, F, helpers.ptr(ip), helpers.ptr(ix), helpers.ptr(xd), helpers.ptr(ref_w),
                    helpers.ptr(Gm), p)
    cp, cr, cpos = pgcn.csr_transpose(ip, ix, F)
    t = {k: torch.from_numpy(v).to(DEV) for k, v in
         dict(xv=xv, G=Gm, cp=cp, cr=cr, cpos=cpos).items()}
    dm = torch.from_numpy(mask.view(np.int64)).to(DEV)
    wg = torch.full((F, p), float("nan"), device=DEV)
    pgcn.check(pgcn.lib.pgcn_spmm_csc_bwd(F, p, vp(t["cp"]), vp(t["cr"]), vp(t["cpos"]),
                                          vp(t["xv"]), vp(dm), 2.0, vp(t["G"]), vp(wg), stream()),
               "csc")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(wg.cpu().numpy(), ref_w)


def test_adam_bit_exact(pgcn):
    lib = helpers.oracle()
    rng = np.random.default_rng(5)
    n = 9632
    w = rng.standard_normal(n).astype(np.float32) * 0.1
    m = np.zeros(n, np.float32)
    v = np.zeros(n, np.float32)
    dw, dm_, dv = (torch.from_numpy(a.copy()).to(DEV) for a in (w, m, v))
    for t in range(1, 6):
        g = rng.standard_normal(n).astype(np.float32) * 0.01
        ss = lib.or_adam_step_size(0.01, 0.9, 0.999, t)
        assert np.float32(ss) == np.float32(pgcn.lib.pgcn_adam_step_size(0.01, 0.9, 0.999, t))
        lib.or_adam_update(helpers.ptr(w), helpers.ptr(g), helpers.ptr(m), helpers.ptr(v),
                           ctypes.c_long(n), ctypes.c_float(ss), ctypes.c_float(0.9),
                           ctypes.c_float(0.999), ctypes.c_float(1e-8), ctypes.c_float(5e-4), 1)
        dg = torch.from_numpy(g).to(DEV)
        pgcn.check(pgcn.lib.pgcn_adam(vp(dw), vp(dg), vp(dm_), vp(dv), n, ss, 0.9, 0.999, 1e-8,
                                      5e-4, 1, stream()), "adam")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dw.cpu().numpy(), w)
    np.testing.assert_array_equal(dm_.cpu().numpy(), m)
    np.testing.assert_array_equal(dv.cpu().numpy(), v)


def test_exp_nonpos_matches_expf(pgcn):
    """The loss kernel's exp of max-shifted logits (x <= 0) is the device expf's sequence
    without the overflow select: bit-identical to expf over every x <= 0 it can see -- a dense
    sweep of [-110, 0] (through the underflow cut at -103.97), denormal and tiny inputs, -0."""
    rng = np.random.default_rng(5)
    x = np.concatenate([
        -np.linspace(0.0, 110.0, 2_000_001, dtype=np.float32),
        -rng.exponential(5.0, 1_000_000).astype(np.float32),
        -np.abs(rng.standard_normal(100_000).astype(np.float32)) * 1e-30,
        np.array([-0.0, -1e-45, -103.972076, -103.97208, -103.97209, -87.33655, -88.7],
                 np.float32)])
    dx = torch.from_numpy(x).to(DEV)
    mine = torch.empty_like(dx)
    lib = torch.empty_like(dx)
    pgcn.check(pgcn.lib.pgcn_debug_exp_check(vp(dx), x.size, vp(mine), vp(lib), stream()),
               "exp_check")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mine.cpu().numpy().view(np.uint32),
                                  lib.cpu().numpy().view(np.uint32))


def test_div_rn_matches_ieee(pgcn):
    """The loss kernel's quotients (prob = e / sum and prob / count, div_rn) against IEEE fp32
    division (numpy, round to nearest, subnormals kept): dense a in (0, 1] -- every 97th bit
    pattern, so subnormal, tiny and normal numerators alike -- over b in [1, 128] (random
    reals and every integer count)."""
    rng = np.random.default_rng(5)
    bits = np.arange(1, 0x3f800001, 97, dtype=np.uint32)
    a = bits.view(np.float32)
    b = np.where(rng.random(a.size) < 0.5, rng.uniform(1.0, 128.0, a.size),
                 rng.integers(1, 129, a.size)).astype(np.float32)
    want = (a / b).astype(np.float32)
    da, db = torch.from_numpy(a).to(DEV), torch.from_numpy(b).to(DEV)
    q = torch.empty_like(da)
    pgcn.check(pgcn.lib.pgcn_debug_div_check(vp(da), vp(db), a.size, vp(q), stream()),
               "div_check")
    torch.cuda.synchronize()
    got = q.cpu().numpy()
    bad = np.flatnonzero(got.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, (bad.size, a[bad[:5]], b[bad[:5]], got[bad[:5]], want[bad[:5]])


@pytest.mark.parametrize("n,c", [(2708, 7), (50000, 41), (1000, 3), (3000, 60), (2000, 113)])
def test_xent_vs_oracle(pgcn, n, c):
    lib = helpers.oracle()
    rng = np.random.default_rng(n)
    ld = (c + 3) // 4 * 4
    logits = np.zeros((n, ld), np.float32)
    logits[:, :c] = rng.standard_normal((n, c)) * 3
    truth = np.where(rng.random(n) < 0.4, rng.integers(0, c, n), -1).astype(np.int32)
    count = int((truth >= 0).sum())
    ref_l = np.ascontiguousarray(logits[:, :c])
    ref_g = np.zeros((n, c), np.float32)
    ref_loss = lib.or_xent_fwd(helpers.ptr(ref_l), helpers.ptr(ref_g), helpers.ptr(truth), n, c, 1)
    ref_acc = lib.or_accuracy(helpers.ptr(ref_l), helpers.ptr(truth), n, c)
    dl = torch.from_numpy(logits).to(DEV)
    dg = torch.full((n, ld), float("nan"), device=DEV)
    dt = torch.from_numpy(truth).to(DEV)
    nb = pgcn.lib.pgcn_xent_blocks(n)
    part = torch.zeros(2 * nb + 2, device=DEV)
    out4 = torch.zeros(4, device=DEV)
    w = torch.zeros(1, device=DEV)
    pgcn.check(pgcn.lib.pgcn_xent_fwd(vp(dl), ld, vp(dg), vp(dt), n, c, count, 1, vp(part),
                                      stream()), "xent")
    pgcn.check(pgcn.lib.pgcn_finalize(vp(part), nb, count, vp(w), 1, 0.0, vp(out4), stream()),
               "finalize")
    torch.cuda.synchronize()
    o = out4.cpu().numpy()
    assert abs(o[0] - ref_loss) <= 1e-5 * abs(ref_loss)
    assert abs(o[1] - ref_acc) * count <= 1.0 + 1e-6
    np.testing.assert_allclose(dl.cpu().numpy()[:, :c], ref_l, rtol=0, atol=0)  # shift exact
    np.testing.assert_allclose(dg.cpu().numpy()[:, :c], ref_g, rtol=1e-5, atol=1e-9)
    np.testing.assert_array_equal(dg.cpu().numpy()[:, c:], 0.0)
