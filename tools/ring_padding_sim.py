#!/usr/bin/env python3
"""Lockstep padding of the d = 16 ring schedule as a function of its shape (diagnostic tool,
host only; DESIGN.md §3 "r05: where the ring's padding comes from").

A numpy restatement of host/ring.cpp's per-(rowset, visit) step-count rule on reddit-114M's
synthetic graph (the bench's, seed 1): rows sorted by spread then degree into rowsets of 16
lane groups, hub rows spread over 2..16 lane groups, 4 nnz-balanced column blocks cut on slice
boundaries; per visit v a rowset runs S_v steps, S_v = the most edges any of its lanes still has
in slice v rounded up to a multiple of G, and every lane spends the S_v steps on its earliest
edges among slices v .. v + W - 1 (first in, first out).  The builder additionally gives the 4
lane groups of one LDS cycle distinct bank quarters, which costs ~0.14 slot per edge on top
(2.03 measured by pgcn_debug_lds_check against 1.89 here at W 3, G 4).

usage: python3 tools/ring_padding_sim.py [W=3] [G=4] [SR=512]
prints: slots per edge, entry blocks (ceil(S_v / 4) per rowset and visit), the floor from the
rowsets' degree imbalance alone (no window, G = 1).
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    SR = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    import bench
    pg = bench.load_pkg()
    # the adjacency does not depend on the feature width
    ds = pg.Dataset.synthetic(bench.N_NODES, 2, bench.N_CLASS, bench.WORKLOADS["reddit-114M"], 1)
    ip = np.asarray(ds.graph_indptr, np.int64)
    ix = np.asarray(ds.graph_indices, np.int64)
    n, nnz, deg = len(ip) - 1, len(ix), np.diff(ip)
    B, spread_thr = 4, 6.0  # host/ring.cpp: 4 column blocks, kRingSpread / 10
    rows = np.repeat(np.arange(n, dtype=np.int64), deg)
    six = ix[np.argsort(rows * n + ix, kind="stable")]
    colcnt = np.bincount(six, minlength=n).astype(np.int64)
    cc = np.concatenate([[0], np.cumsum(colcnt)])
    cut = [0]
    for b in range(1, B):
        c = int(np.searchsorted(cc, nnz * b / B))
        cut.append(max((c + SR // 2) // SR * SR, cut[-1]))
    cut.append(n)
    lam = deg * 512.0 / n
    spread = np.zeros(n, np.int64)
    for _ in range(4):
        spread += lam / (1 << spread) > spread_thr
    order = np.lexsort((-deg, -spread))
    unit = np.zeros(n, np.int64)
    nunits = 0
    for s in range(4, -1, -1):
        rws = order[spread[order] == s]
        if len(rws) == 0:
            continue
        m, per = 1 << s, 16 >> s
        k = np.arange(len(rws))
        unit[rws] = nunits + (k // per) * 16 + (k % per) * m
        nunits += (len(rws) + per - 1) // per * 16
    nrs = nunits // 16
    m_of = 1 << spread
    slots = blocks = edges = lower = 0
    for b in range(B):
        c0, c1 = cut[b], cut[b + 1]
        T = (c1 - c0 + SR - 1) // SR
        sel = (six >= c0) & (six < c1)
        er, ec = rows[sel], six[sel]
        first = np.searchsorted(er, np.arange(n), side="left")
        j = np.arange(len(er)) - first[er]
        lane = unit[er] + j % m_of[er]
        cnt = np.bincount(lane * T + (ec - c0) // SR, minlength=nunits * T).reshape(nrs, 16, T)
        edges += len(er)
        lower += int(cnt.sum(2).max(1).sum()) * 16
        rem = cnt.astype(np.int32)
        for v in range(T):
            S = G * ((rem[:, :, v].max(1) + G - 1) // G)
            slots += 16 * int(S.sum())
            blocks += int(((S + 3) // 4).sum())
            c = np.repeat(S[:, None], 16, 1)
            for u in range(v, min(T, v + W)):
                take = np.minimum(c, rem[:, :, u])
                rem[:, :, u] -= take
                c -= take
        assert rem.sum() == 0
    print(f"W {W} G {G} SR {SR}: {slots / edges:.3f} slots per edge, {blocks} entry blocks "
          f"({blocks * 64 / edges:.3f} block slots per edge); floor (degree imbalance) "
          f"{lower / edges:.3f}")


if __name__ == "__main__":
    main()
