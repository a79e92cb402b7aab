"""Rowsets formed by per-slice signature instead of consecutive degree order (diagnostic tool,
host only; VERDICT r04 item 2's suggestion, DESIGN.md §3 "r05: where the ring's padding comes
from").  A variant of tools/ring_padding_sim.py (W 3, G 4, 512-row slices): inside consecutive
groups of GRP rows of one spread class, rows are re-sorted by a signature of their per-slice
edge counts -- "proj" a random projection of the count vector, "first" its centre of mass --
before the rowsets are cut.  usage: python3 tools/ring_rowset_sim.py [base|proj|first] [GRP]
"""
import os, sys
import numpy as np
sys.path.insert(0, "/root/repo")
import bench
mode = sys.argv[1] if len(sys.argv) > 1 else "base"
GRP = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
W, G, SR = 3, 4, 512
pg = bench.load_pkg()
ds = pg.Dataset.synthetic(bench.N_NODES, 2, bench.N_CLASS, bench.WORKLOADS["reddit-114M"], 1)
ip = np.asarray(ds.graph_indptr, np.int64); ix = np.asarray(ds.graph_indices, np.int64)
n, nnz, deg = len(ip) - 1, len(ix), np.diff(ip)
B, thr = 4, 6.0
rows = np.repeat(np.arange(n, dtype=np.int64), deg)
six = ix[np.argsort(rows * n + ix, kind="stable")]
colcnt = np.bincount(six, minlength=n).astype(np.int64); cc = np.concatenate([[0], np.cumsum(colcnt)])
cut = [0]
for b in range(1, B):
    c = int(np.searchsorted(cc, nnz * b / B)); cut.append(max((c + SR // 2) // SR * SR, cut[-1]))
cut.append(n)
lam = deg * 512.0 / n
spread = np.zeros(n, np.int64)
for _ in range(4): spread += lam / (1 << spread) > thr
order = np.lexsort((-deg, -spread))
# signature: per-slice counts over the whole row (all blocks), coarse: counts per slice
if mode != "base":
    T = (n + SR - 1) // SR
    sl = six // SR
    cnt = np.zeros((n, T), np.int16)
    np.add.at(cnt, (rows, sl), 1)
    rng = np.random.default_rng(0)
    if mode == "proj":
        key = cnt.astype(np.float32) @ rng.standard_normal(T).astype(np.float32)
    elif mode == "first":  # center of mass of the row's slices
        key = (cnt.astype(np.float32) * np.arange(T)).sum(1) / np.maximum(1, cnt.sum(1))
    # re-sort inside consecutive groups of GRP rows of the same spread
    o2 = order.copy()
    for s in range(5):
        idx = np.where(spread[order] == s)[0]
        for g0 in range(0, len(idx), GRP):
            seg = idx[g0:g0 + GRP]
            rr = order[seg]
            o2[seg] = rr[np.argsort(key[rr], kind="stable")]
    order = o2
unit = np.zeros(n, np.int64); nunits = 0
for s in range(4, -1, -1):
    rws = order[spread[order] == s]
    if len(rws) == 0: continue
    m, per = 1 << s, 16 >> s
    k = np.arange(len(rws))
    unit[rws] = nunits + (k // per) * 16 + (k % per) * m
    nunits += (len(rws) + per - 1) // per * 16
nrs = nunits // 16; m_of = 1 << spread
slots = edges = 0
for b in range(B):
    c0, c1 = cut[b], cut[b + 1]; T = (c1 - c0 + SR - 1) // SR
    sel = (six >= c0) & (six < c1); er, ec = rows[sel], six[sel]
    first = np.searchsorted(er, np.arange(n), side="left"); j = np.arange(len(er)) - first[er]
    lane = unit[er] + j % m_of[er]
    cnt = np.bincount(lane * T + (ec - c0) // SR, minlength=nunits * T).reshape(nrs, 16, T)
    edges += len(er); rem = cnt.astype(np.int32)
    for v in range(T):
        S = G * ((rem[:, :, v].max(1) + G - 1) // G); slots += 16 * int(S.sum())
        c = np.repeat(S[:, None], 16, 1)
        for u in range(v, min(T, v + W)):
            take = np.minimum(c, rem[:, :, u]); rem[:, :, u] -= take; c -= take
print(mode, GRP, f"{slots / edges:.3f}")
