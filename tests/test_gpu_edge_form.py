"""The edge-list form of the dense build (build.hip canon_from_edges / dense_scatter, tables.hip
scatter kernels): a dense-shaped graph's edges go to the device and the canonical arc rule of
graph.c (per ordered pair the minimum latency, the lowest edge index among equal latencies, both
directions of an undirected edge, the same rule for self-loops on the diagonal; topology.c:377-396)
is applied there by atomics. Checked against the host canonical form (the sparse build of the same
graph, which reads graph.c's CSR) and the oracle's rows; the fallbacks (too few distinct arcs for
the dense choice, invalid edges) reach the host form and its errors."""
import numpy as np
import pytest

import oracle
from shadow_amd import graphs
from shadow_amd._lib import ALGO_DENSE_FW, ALGO_SPARSE_SSSP
from shadow_amd.topology import build_tables

pytestmark = pytest.mark.gpu
MS = 1_000_000
REL_TOL = 1e-12


def _rel_err(a, b):
    return float((np.abs(a - b) / np.maximum(np.abs(b), 1e-300)).max())


def _multigraph(n, directed, seed):
    """a dense random multigraph: parallel edges with equal latencies and different losses,
    unequal latencies, several self-loops per vertex"""
    rng = np.random.default_rng(seed)
    m = n * n // 6
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    dup = rng.integers(0, m, m // 4)  # parallel copies of existing edges
    src = np.concatenate([src, src[dup], np.arange(n), np.arange(n)])
    dst = np.concatenate([dst, dst[dup], np.arange(n), np.arange(n)])
    lat = rng.integers(1, 40, len(src)) * MS
    lat[m:m + len(dup)] = np.where(rng.random(len(dup)) < 0.5, lat[dup], lat[m:m + len(dup)])
    loss = rng.integers(0, 500, len(src)) / 10000.0
    ring = np.arange(n)
    src = np.concatenate([src, ring]).astype(np.int32)
    dst = np.concatenate([dst, (ring + 1) % n]).astype(np.int32)
    lat = np.concatenate([lat, np.full(n, 40 * MS)]).astype(np.int64)
    loss = np.concatenate([loss, np.zeros(n)])
    return graphs.Graph(n, directed, src, dst, lat, loss)


@pytest.mark.parametrize("directed", [False, True])
def test_edge_form_matches_host_canonical_form(gpu, directed):
    g = _multigraph(2560, directed, 7 + directed)
    lat_d, rel_d, st = build_tables(g.n, directed, g.src, g.dst, g.lat_ns, g.loss)
    assert st.algo == ALGO_DENSE_FW
    lat_s, rel_s, st2 = build_tables(g.n, directed, g.src, g.dst, g.lat_ns, g.loss,
                                     algo=ALGO_SPARSE_SSSP)
    assert st2.algo == ALGO_SPARSE_SSSP
    assert np.array_equal(lat_d, lat_s)
    assert np.array_equal(rel_d, rel_s)
    el = oracle.EdgeList(g.n, directed, g.src, g.dst, g.lat_ns, g.loss)
    rows = [0, 1, 777, g.n - 1]
    o = oracle.sssp_list(el, rows, nthreads=4)
    for k, s in enumerate(rows):  # the oracle's raw rows hold 0 / 1 at the source itself
        off = np.arange(g.n) != s
        assert np.array_equal(lat_d[s][off], o["lat_int"][k][off]), s
        assert _rel_err(rel_d[s][off], o["rel"][k][off]) <= REL_TOL, s


def test_edge_form_direct_mode_diagonal_and_ties(gpu):
    """use_shortest_path = false: the tables ARE the canonical arcs (topology.c:1816-1858)"""
    g = graphs.complete_graph(300, seed=9)
    # a second copy of every edge: equal latency (the first, lower index wins), other loss
    src = np.concatenate([g.src, g.src])
    dst = np.concatenate([g.dst, g.dst])
    lat = np.concatenate([g.lat_ns, g.lat_ns])
    loss = np.concatenate([g.loss, np.full(len(g.loss), 0.3)])
    lat_ns, rel, _ = build_tables(g.n, False, src, dst, lat, loss, use_shortest_path=False)
    lat0, rel0, _ = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss, use_shortest_path=False)
    assert np.array_equal(lat_ns, lat0) and np.array_equal(rel, rel0)
    i = np.arange(g.n)
    assert np.all(rel[i, i] > 0)  # the self-loops on the diagonal


@pytest.mark.parametrize("ranks", [1, 3])
def test_edge_form_falls_back_when_arcs_are_few(gpu, monkeypatch, ranks):
    """edge count says dense, distinct arcs say sparse: the host canonical form decides. On 3
    virtual ranks no rank holds every row, so the ranks sum their exact arc counts and fall back
    together (before, a multi-rank build kept the dense FW path here)"""
    n = 3000
    ring = np.arange(n)
    rng = np.random.default_rng(3)
    k = n * n // 28
    pick = rng.integers(0, n, k)
    src = np.concatenate([ring, pick]).astype(np.int32)
    dst = np.concatenate([(ring + 1) % n, (pick + 1) % n]).astype(np.int32)
    lat = (rng.integers(1, 30, len(src)) * MS).astype(np.int64)
    loss = rng.integers(0, 300, len(src)) / 10000.0
    if ranks > 1:
        monkeypatch.setenv("SRT_VIRTUAL_RANKS", str(ranks))
    lat_ns, rel, st = build_tables(n, False, src, dst, lat, loss, ngpus=ranks if ranks > 1 else None)
    assert st.algo == ALGO_SPARSE_SSSP
    el = oracle.EdgeList(n, False, src, dst, lat, loss)
    rows = [0, 1500, n - 1]
    o = oracle.sssp_list(el, rows, nthreads=4)
    for j, s in enumerate(rows):
        off = np.arange(n) != s
        assert np.array_equal(lat_ns[s][off], o["lat_int"][j][off]), s
        assert _rel_err(rel[s][off], o["rel"][j][off]) <= REL_TOL, s


def test_edge_form_invalid_edges_report_like_the_host_form(gpu):
    g = graphs.complete_graph(64, seed=2)
    lat = g.lat_ns.copy()
    lat[100] = 0
    with pytest.raises(Exception, match="non-positive latency"):
        build_tables(g.n, False, g.src, g.dst, lat, g.loss)
    dst = g.dst.copy()
    dst[5] = 64
    with pytest.raises(Exception, match="out of range"):
        build_tables(g.n, False, g.src, dst, g.lat_ns, g.loss)
