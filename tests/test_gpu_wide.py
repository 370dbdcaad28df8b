"""Graphs whose shortest-path latencies may pass the u32 tables' SRT_INF = 2^31 - 1 quanta: the u64 rows of
wide.hip (dist_enc 4) against the oracle's i64-ns Dijkstra (oracle.sssp_list, restating
topology.c:1578-1814 with the f64-ms path-order sums of topology.c:1308/:1364).

The u32 `lat` table saturates at SRT_INF - 1 = 0x7FFFFFFE quanta for reachable pairs; the reference's value is
the f64 ms table, which must match bit for bit, as must the path-order reliability."""
import os

import numpy as np
import pytest

import oracle
from shadow_amd import graphs
from shadow_amd._lib import ALGO_AUTO, ALGO_DENSE_FW, ALGO_SPARSE_SSSP
from shadow_amd.topology import build_tables_subset

pytestmark = pytest.mark.gpu
SAT = 0x7FFFFFFE     # SRT_INF - 1: reachable pairs beyond the u32 table's range
INF32 = 0x7FFFFFFF   # SRT_INF: unreachable


def _el(g):
    return oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)


def _wide_chain(n=3000, chords=40, directed=False, seed=5):
    """A long path of ~4 ms hops in odd nanoseconds (quantum 1 ns: 1.2e10 quanta end to end) with a
    few long chords (0.6-1.0 s; an arc stays below 2^30 quanta) -- true distances pass the u32
    table's 2^31 - 1."""
    rng = np.random.default_rng(seed)
    a = np.arange(n - 1)
    src = [a, rng.integers(0, n, chords)]
    dst = [a + 1, rng.integers(0, n, chords)]
    lat = [rng.integers(3_500_000, 4_500_000, n - 1) | 1, rng.integers(600_000_000, 1_000_000_000, chords)]
    if directed:  # some backward arcs, so part of each row is unreachable
        b = rng.integers(1, n, n // 10)
        src.append(b)
        dst.append(b - 1 - rng.integers(0, np.minimum(b, 5)))
        lat.append(rng.integers(1_500_000, 2_500_000, len(b)) | 1)
    src = np.concatenate(src).astype(np.int32)
    dst = np.concatenate(dst).astype(np.int32)
    lat = np.concatenate(lat).astype(np.int64)
    loss = rng.integers(0, 300, len(src)) / 10000.0
    return graphs.Graph(n, directed, src, dst, lat, loss, f"wide{n}{'d' if directed else ''}")


def _check(g, verts, lat, rel, ms, q):
    exp = oracle.sssp_list(_el(g), verts, nthreads=16)
    vv = np.asarray(verts)
    li = exp["lat_int"][:, vv]
    reach = li != np.uint64(oracle.U64_MAX)
    raw = lat // np.uint64(q)
    want = np.where(reach, np.minimum(li // np.uint64(q), np.uint64(SAT)), np.uint64(INF32))
    off = ~np.eye(len(vv), dtype=bool)
    assert np.array_equal(raw[off], want[off])
    assert np.array_equal(rel[off].view(np.uint64), exp["rel"][:, vv][off].view(np.uint64))
    m = off & reach
    assert np.array_equal(ms[m], exp["lat_ms"][:, vv][m]), np.argwhere((ms != exp["lat_ms"][:, vv]) & m)[:5]
    # the diagonal: its own rule, its latency in ms from its quanta
    d = np.diag(raw).astype(np.float64)
    assert np.array_equal(np.diag(ms), np.array([float(int(x) * q) / 1e6 for x in d]))
    return int(reach[off].sum()), int((li[off & reach] // np.uint64(q) > np.uint64(SAT)).sum())


@pytest.mark.parametrize("directed", [False, True])
def test_wide_chain_full_table(gpu, directed):
    g = _wide_chain(directed=directed)
    lat, rel, ms, _, st = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                              algo=ALGO_AUTO, want_ms=True)
    assert st.dist_enc == 4
    q = int(np.gcd.reduce(g.lat_ns))
    assert q == 1
    reach, beyond = _check(g, np.arange(g.n, dtype=np.int32), lat, rel, ms, q)
    assert beyond > 0, "the graph should have distances beyond u32 quanta"
    if directed:
        assert reach < g.n * (g.n - 1)


def test_wide_subset_and_virtual_ranks(gpu):
    g = _wide_chain(n=2500, chords=30, seed=9)
    rng = np.random.default_rng(1)
    verts = np.sort(rng.choice(g.n, 97, replace=False)).astype(np.int32)
    lat, rel, ms, _, st = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                              verts=verts, algo=ALGO_SPARSE_SSSP, want_ms=True)
    assert st.dist_enc == 4
    _check(g, verts, lat, rel, ms, 1)
    os.environ["SRT_VIRTUAL_RANKS"] = "2"
    try:
        lat2, rel2, ms2, _, _ = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                                    verts=verts, algo=ALGO_AUTO, ngpus=2, want_ms=True)
    finally:
        del os.environ["SRT_VIRTUAL_RANKS"]
    assert np.array_equal(lat, lat2) and np.array_equal(rel, rel2) and np.array_equal(ms, ms2)


def test_wide_refusals(gpu):
    """A wide graph never lands silently in a u32 table: a dense request, or no f64 ms output
    to carry the values, is refused (SRT_E_RANGE)."""
    g = _wide_chain(n=600, chords=10)
    with pytest.raises(RuntimeError, match="SRT_E_RANGE"):
        build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss, algo=ALGO_DENSE_FW,
                            want_ms=True)
    with pytest.raises(RuntimeError, match="SRT_E_RANGE"):
        build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss, algo=ALGO_AUTO)
    # the device-row entry points without an f64 ms output (they used to saturate)
    import torch
    from shadow_amd.topology import SparseGraph
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss, device=0)
    try:
        lat = torch.empty((4, g.n), dtype=torch.int32, device="cuda")
        rel = torch.empty((4, g.n), dtype=torch.float64, device="cuda")
        srcs = torch.arange(4, dtype=torch.int32, device="cuda")
        with pytest.raises(RuntimeError, match="SRT_E_RANGE"):
            sg.rows(0, 4, lat.data_ptr(), rel.data_ptr())
        with pytest.raises(RuntimeError, match="SRT_E_RANGE"):
            sg.rows_list(srcs.data_ptr(), 4, lat.data_ptr(), rel.data_ptr())
    finally:
        sg.free()


@pytest.mark.parametrize("directed", [False, True])
def test_ba100k_microsecond_latencies(gpu, directed):
    """VERDICT r02 #3's case: a 100k BA graph with 1..100,000 us latencies (q = 1 us), undirected
    (the hop bound keeps it in u32 quanta) and directed (arcs new -> old: not strongly connected,
    so the bound is (n - 1) max_w > SRT_INF and the u64 rows build it); sampled rows vs the oracle."""
    b = graphs.barabasi_albert(100_000, m=3, seed=5)
    rng = np.random.default_rng(7)
    lat = rng.integers(1, 100_001, b.m).astype(np.int64) * 1000
    g = graphs.Graph(b.n, directed, b.src, b.dst, lat, b.loss, "ba100k_us")
    verts = np.sort(rng.choice(g.n, 48, replace=False)).astype(np.int32)
    lat_t, rel, ms, _, st = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                                verts=verts, algo=ALGO_AUTO, want_ms=True)
    assert st.dist_enc == (4 if directed else st.dist_enc)
    q = int(np.gcd.reduce(lat))
    assert q == 1000
    _check(g, verts, lat_t, rel, ms, q)
