#!/usr/bin/env python3
"""CPU model of neighbour-row derivation for sparse all-pairs builds.

Take an independent set I of low-degree vertices (on a BA graph with m = 3 every vertex of degree 3
qualifies: preferential attachment never links two of them). Only the rows of the other vertices
("core") run the SSSP kernel. For s in I and t != s, every path leaves s through a neighbour k, so

    D[s][t] = min_k w(s,k) + D[k][t]                                           (exact, w >= 1)

and the canonical predecessor -- argmin (D[s][u], u) over the tight in-arcs u -> t, i.e. the largest
arc weight, then the smallest u (topology.c:1679-1701 up to igraph's heap order) --
is the best of the optimal neighbours' own canonical arcs into t (the ordering key (-w, u) does not
depend on the row, and an arc is tight for s exactly when it is tight for some optimal k), with the
direct arc (s, t) when t is a neighbour. The reliability must still be the path-order product from s
(topology.c:1364-1365), so it is re-formed from these predecessors, not taken from k's row.

This script checks both claims against the oracle's Dijkstra rows on a small BA graph, then prints
the traffic model of the C5 split. usage: python tools/c5_derive_model.py [n]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import oracle  # noqa: E402
from shadow_amd import graphs  # noqa: E402


def canon_csr(g):
    """canonical undirected arcs: min latency per pair (lowest edge index on ties), no self-loops"""
    off = g.src != g.dst
    s = np.concatenate([g.src[off], g.dst[off]])
    d = np.concatenate([g.dst[off], g.src[off]])
    lat = np.concatenate([g.lat_ns[off], g.lat_ns[off]])
    r = 1.0 - np.concatenate([g.loss[off], g.loss[off]])
    eidx = np.concatenate([np.nonzero(off)[0]] * 2)
    o = np.lexsort((eidx, lat, d, s))
    s, d, lat, r = s[o], d[o], lat[o], r[o]
    keep = np.ones(len(s), bool)
    keep[1:] = (s[1:] != s[:-1]) | (d[1:] != d[:-1])
    s, d, lat, r = s[keep], d[keep], lat[keep], r[keep]
    q = int(np.gcd.reduce(lat))
    ptr = np.searchsorted(s, np.arange(g.n + 1))
    return ptr, d.astype(np.int64), (lat // q).astype(np.int64), r, q


def independent_low_degree(ptr, col, maxdeg):
    n = len(ptr) - 1
    deg = np.diff(ptr)
    blocked = np.zeros(n, bool)
    inI = np.zeros(n, bool)
    for v in np.argsort(deg, kind="stable"):
        if deg[v] > maxdeg:
            break
        if blocked[v]:
            continue
        inI[v] = True
        blocked[v] = True
        blocked[col[ptr[v]:ptr[v + 1]]] = True
    return inI


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    g = graphs.barabasi_albert(n, seed=5)
    ptr, col, w, r, q = canon_csr(g)
    inI = independent_low_degree(ptr, col, 4)
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    rows = oracle.sssp_rows(el, 0, n, nthreads=8, want_pred=True)
    D = (rows["lat_int"] // np.uint64(q)).astype(np.int64)
    P = rows["pred"]
    I = np.nonzero(inI)[0]
    wq = {}
    for v in range(n):
        for k in range(ptr[v], ptr[v + 1]):
            wq[(v, int(col[k]))] = int(w[k])
    bad_d = bad_p = 0
    for s in I:
        nb = col[ptr[s]:ptr[s + 1]]
        ws = w[ptr[s]:ptr[s + 1]]
        assert not inI[nb].any(), "not independent"
        cand = ws[:, None] + D[nb]  # [deg, n]
        dd = cand.min(axis=0)
        dd[s] = 0
        bad_d += int((dd != D[s]).sum())
        for t in range(n):
            if t == s:
                continue
            best = None
            for i, k in enumerate(nb):
                if cand[i, t] != dd[t]:
                    continue
                if t == k:
                    key = (-int(ws[i]), int(s))  # the direct arc (s, k)
                else:
                    u = int(P[k, t])
                    key = (-wq[(u, t)], u)
                best = key if best is None or key < best else best
            if best is None or best[1] != int(P[s, t]):
                bad_p += 1
    print(f"BA n={n}: |I| = {len(I)} ({len(I) / n:.1%}), derived distances wrong: {bad_d}, "
          f"derived predecessors wrong: {bad_p}")
    # C5 traffic model (n = 100,000, m = 3): |I| and the mean degree in I from the real graph
    big = graphs.barabasi_albert(100_000, seed=5)
    bp, bc, _, _, _ = canon_csr(big)
    bI = independent_low_degree(bp, bc, 4)
    N = big.n
    nI = int(bI.sum())
    mdeg = float(np.diff(bp)[bI].mean())
    row_u32 = 4 * N
    per_row = mdeg * 2 * row_u32 + row_u32 + 4 * N + 8 * N  # k lat + k arc-code rows in; lat, pred, r out
    sweeps = 8 * N + 4 * N + 8 * N  # rel in/out + pred, one pass of the sweeps
    print(f"C5: |I| = {nI} of {N} ({nI / N:.1%}), mean degree in I {mdeg:.2f}; SSSP rows "
          f"{N - nI}; derivation {nI * per_row / 1e9:.1f} GB + sweeps {nI * sweeps / 1e9:.1f} GB "
          f"+ arc codes of the core rows {(N - nI) * 4 * N / 1e9:.1f} GB")


if __name__ == "__main__":
    main()
