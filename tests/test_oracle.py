"""The CPU oracle against the golden vectors (it must be pinned before it judges the GPU path)."""
import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN
from shadow_amd import graphs

MS = 1_000_000


def _edges_from_case(case):
    e = np.array(case["edges"], dtype=np.float64)
    return oracle.EdgeList(case["n"], case["directed"], e[:, 0].astype(np.int32),
                           e[:, 1].astype(np.int32), (e[:, 2] * MS).astype(np.int64), e[:, 3])


def test_known_answers_single_vertex():
    """topology.c:1431-1576 self-loop rule on the reference's own test graphs."""
    cases = json.load(open(os.path.join(GOLDEN, "known_answers.json")))
    lat = {"50 ms": 50 * MS, "1 ms": MS, "10 ms": 10 * MS}
    assert len(cases) == 5
    for c in cases:
        (l,) = [v for k, v in lat.items() if f'latency "{k}"' in c["gml"]]
        loss = 0.25 if "packet_loss 0.25" in c["gml"] else 0.0
        directed = "directed 1" in c["gml"]
        el = oracle.EdgeList(1, directed, [0], [0], [l], [loss])
        t = oracle.table(el)
        for s, d, lat_ns, rel in c["pairs"]:
            assert int(t["lat_int"][s, d]) == lat_ns
            assert int(t["lat_ref"][s, d]) == lat_ns
            assert t["rel"][s, d] == rel, c["name"]


@pytest.mark.parametrize("case", json.load(open(os.path.join(GOLDEN, "ties.json"))),
                         ids=lambda c: c["name"])
def test_tie_graphs(case):
    t = oracle.table(_edges_from_case(case), raw=True)
    for s, d, lat_ns, rel in case["pairs"]:
        assert int(t["lat_int"][s, d]) == lat_ns, (s, d)
        assert t["rel"][s, d] == rel, (s, d)


def test_c1_regression_and_modes():
    g = graphs.complete_graph(50, seed=1, lat_max=300, self_max=10, loss_max=500)
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    exp = np.load(os.path.join(GOLDEN, "c1_expected.npz"))
    for mode in (oracle.ORC_INT_NS, oracle.ORC_F64_MS):
        t = oracle.table(el, True, mode, nthreads=2, raw=True)
        assert np.array_equal(t["lat_int"], exp["lat_ns"])
        assert np.array_equal(t["rel"], exp["rel"])
        served = oracle.table(el, True, mode, nthreads=2)
        assert np.array_equal(served["rel"], exp["rel_served_ascending"])
    # whole-ms graph: exact integer ns equals the reference's ceil(ms * 1e6) (worker.c:551)
    assert np.array_equal(t["lat_ref"], t["lat_int"])
    # undirected: latency is symmetric; each source's own reliability is not, bit for bit (the
    # reversed product, and ties): the first source run decides what a pair serves
    assert np.array_equal(exp["lat_ns"], exp["lat_ns"].T)
    assert np.array_equal(exp["rel_served_ascending"], exp["rel_served_ascending"].T)
    assert not np.array_equal(exp["rel"], exp["rel"].T)


def test_c1_against_networkx():
    nx = pytest.importorskip("networkx")
    g = graphs.complete_graph(50, seed=1)
    exp = np.load(os.path.join(GOLDEN, "c1_expected.npz"))
    G = nx.Graph()
    for e in range(g.m):
        if g.src[e] != g.dst[e]:
            G.add_edge(int(g.src[e]), int(g.dst[e]), weight=int(g.lat_ns[e]))
    for s, dist in nx.all_pairs_dijkstra_path_length(G, weight="weight"):
        for t, d in dist.items():
            if s != t:
                assert int(exp["lat_ns"][s, t]) == d


def test_sub_ms_quirk_documented():
    """Sub-millisecond latencies: the reference sums f64 ms and rounds up (worker.c:551), which
    can exceed the exact integer sum by 1 ns (0.1 + 0.2 ms). This pins that class on a 3-vertex
    path. The GPU build reproduces lat_ref: with a sub-ms quantum it also forms the path-order f64
    ms table (tables.hip path_sweeps_kernel), checked in tests/test_gpu_dropin.py."""
    el = oracle.EdgeList(3, False, [0, 1], [1, 2], [100_000, 200_000], [0.0, 0.0])
    t = oracle.table(el)
    assert int(t["lat_int"][0, 2]) == 300_000
    assert int(t["lat_ref"][0, 2]) == 300_001  # ceil(0.30000000000000004 * 1e6)


def test_direct_mode():
    g = graphs.complete_graph(12, seed=9)
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    t = oracle.table(el, use_shortest_path=False)
    w, r = graphs.complete_dense(12, 9)
    assert np.array_equal(t["lat_int"], w.astype(np.uint64) * MS)
    assert np.array_equal(t["rel"], r)


def test_rows_threads_agree():
    g = graphs.random_geometric(400, seed=3)
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    a = oracle.sssp_rows(el, 10, 60, nthreads=1, want_pred=True)
    b = oracle.sssp_rows(el, 10, 60, nthreads=4, want_pred=True)
    for k in a:
        assert np.array_equal(a[k], b[k])


def test_complete_sample_matches_edge_list_oracle():
    """The dense CPU-baseline Dijkstra (bench.py cpu_baseline) equals the edge-list oracle."""
    n, seed = 300, 2
    g = graphs.complete_graph(n, seed=seed, lat_max=300, self_max=10, loss_max=500)
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    src = np.array([0, 7, 150, 299], np.int32)
    lat, rel, _, _ = oracle.complete_sample(n, seed, 300, 10, 500, src, nthreads=2)
    for i, s in enumerate(src):
        rows = oracle.sssp_rows(el, int(s), int(s) + 1)
        assert np.array_equal(lat[i], rows["lat_int"][0])
        assert np.array_equal(rel[i], rows["rel"][0])


def _scipy_crosscheck(g):
    """An independent implementation pins the oracle: scipy's Dijkstra gives every distance, and
    on every pair whose shortest path is unique (where igraph's heap order and the canonical tie
    rule cannot differ) the path-order product of (1 - loss) along scipy's predecessor chain,
    formed left to right from the source (topology.c:1364-1365), gives the reliability."""
    sp = pytest.importorskip("scipy.sparse")
    csgraph = pytest.importorskip("scipy.sparse.csgraph")
    n = g.n
    off = g.src != g.dst
    w = (g.lat_ns[off] // MS).astype(np.float64)
    W = sp.coo_matrix((w, (g.src[off], g.dst[off])), shape=(n, n)).tocsr()
    R = {(int(a), int(b)): 1.0 - float(x) for a, b, x in zip(g.src[off], g.dst[off], g.loss[off])}
    if not g.directed:
        W = W.maximum(W.T)
        R.update({(b, a): x for (a, b), x in list(R.items())})
    D, P = csgraph.dijkstra(W, directed=True, return_predecessors=True)
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    t = oracle.table(el, nthreads=4, raw=True)
    Wd = W.toarray()
    checked = 0
    for s in range(n):
        reach = np.isfinite(D[s])
        for v in range(n):
            if v != s and reach[v]:
                assert int(t["lat_int"][s, v]) == int(D[s, v]) * MS, (s, v)
        # uniqueness and the path product, in increasing distance order
        order = np.argsort(D[s], kind="stable")
        uniq = np.zeros(n, bool)
        rel = np.zeros(n)
        uniq[s], rel[s] = True, 1.0
        for v in order:
            if v == s or not reach[v]:
                continue
            tight = [u for u in np.nonzero(Wd[:, v])[0]
                     if reach[u] and D[s, u] + Wd[u, v] == D[s, v] and u != v]
            u = int(P[s, v])
            uniq[v] = len(tight) == 1 and uniq[u]
            rel[v] = rel[u] * R[(u, v)]
            if uniq[v]:  # every row is its own source's
                assert t["rel"][s, v] == rel[v], (s, v)
                checked += 1
    return checked


@pytest.mark.parametrize("which", ["c1", "rgg300", "ba400", "complete120_ties"])
def test_oracle_against_scipy_dijkstra(which):
    if which == "c1":
        g = graphs.complete_graph(50, seed=1)
    elif which == "rgg300":
        g = graphs.random_geometric(300, seed=3)
    elif which == "ba400":
        g = graphs.barabasi_albert(400, seed=5)
    else:  # small latencies: many equal-length paths, so many pairs are skipped as tied
        g = graphs.complete_graph(120, seed=11, lat_max=8)
    checked = _scipy_crosscheck(g)
    assert checked > 0


def test_lazy_cache_ascending_order_is_the_served_table():
    """oracle/lazy_cache.py (the reference's lazy cache, topology.c:1900-1981) pinned on C1: with
    every vertex attached and lookups (s, t) issued in increasing source order, each pair is served
    from the row of min(s, t) -- exactly orc_table's served table; the reverse order serves the
    row of max(s, t). Every source runs once, and the packet counts land on one Path per pair."""
    from oracle.lazy_cache import LazyPathCache
    g = graphs.complete_graph(50, seed=1, lat_max=300, self_max=10, loss_max=500)
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    raw = oracle.table(el, True, raw=True)
    exp = np.load(os.path.join(GOLDEN, "c1_expected.npz"))
    for order in (1, -1):
        sim = LazyPathCache(raw, directed=False)
        for v in range(g.n):
            sim.attach(v, v)
        got = np.empty((g.n, g.n))
        for s in range(g.n)[::order]:
            for t in range(g.n)[::order]:
                got[s, t] = sim.get_reliability(s, t)
                sim.increment(t, s)
        if order == 1:
            assert np.array_equal(got, exp["rel_served_ascending"])
        else:  # the row of max(s, t): the transpose of the ascending lower triangle
            up = np.triu_indices(g.n, 1)
            assert np.array_equal(got[up], raw["rel"].T[up])
        assert sim.source_runs == g.n - 1  # the last source finds every pair cached
        assert all(p.packets == (2 if p.src != p.dst else 1)
                   for c in sim.cache.values() for p in c.values())


def test_lazy_cache_directed_serves_the_first_run():
    """Directed: the reference checks only (s, t) before computing (topology.c:1919), but falls
    back to (t, s) after (:1963-1967) -- so lookup(s, t) after t's source ran returns t -> s."""
    from oracle.lazy_cache import LazyPathCache
    el = oracle.EdgeList(3, True, [0, 1, 1, 2, 0, 0, 1, 2], [1, 0, 2, 0, 2, 0, 1, 2],
                         np.array([1, 5, 1, 1, 10, 50, 50, 50]) * MS, [0.1, 0.2, 0.3, 0.4, 0.5,
                                                                       0.0, 0.0, 0.0])
    raw = oracle.table(el, True, raw=True)
    sim = LazyPathCache(raw, directed=True)
    for v in range(3):
        sim.attach(v, v)
    assert sim.get_latency(1, 0) == 2.0            # source 1 runs: 1 -> 2 -> 0
    assert sim.get_latency(0, 1) == 2.0            # served the 1 -> 0 path, not 0 -> 1 (1 ms)
    assert raw["lat_ms"][0, 1] == 1.0
    assert sim.get_latency(0, 2) == 2.0            # source 0 ran too: its own 0 -> 1 -> 2
    assert sim.source_runs == 2
