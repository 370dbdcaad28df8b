"""Multi-source shared-frontier SSSP (shadow_amd/csrc/msssp.hip, srt_build_stats.dist_enc 3):
64 sources per workgroup, one per lane, pulls to a fixed point with delta-stepping over the lane
minimum. AUTO takes it for local graphs (C3-shaped RGGs); SRT_FORM kernel=ms forces it on any graph.

Every row is its own source's (topology.c:1578-1814, no mirror), compared with oracle/ off the
diagonal: latency bit-exact in integer ns, reliability bit-exact (the product is formed in path
order along the canonical predecessor, like the single-source kernels; north_star allows 1e-12).
"""
import numpy as np
import pytest
from conftest import form_env, set_form

import oracle
from shadow_amd import graphs
from shadow_amd._lib import ALGO_SPARSE_SSSP, BuildStats
from shadow_amd.topology import SparseGraph, build_tables

pytestmark = pytest.mark.gpu


def _el(g):
    return oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)


def _unreached_as_oracle(lat_ns, g):
    """The tables mark an unreachable pair SRT_INF quanta; the oracle marks it UINT64_MAX ns."""
    q = int(np.gcd.reduce(g.lat_ns[g.lat_ns > 0]))
    return np.where(lat_ns == np.uint64(0x7FFFFFFF * q), np.uint64(0xFFFFFFFFFFFFFFFF), lat_ns)


def _directed_ring_graph(n=400, m=3000, seed=12, wmax=20):
    rng = np.random.default_rng(seed)
    ring = np.arange(n)
    src = np.concatenate([rng.integers(0, n, m), ring, ring]).astype(np.int32)
    dst = np.concatenate([rng.integers(0, n, m), (ring + 1) % n, ring]).astype(np.int32)
    lat = (rng.integers(1, wmax, len(src)) * 1_000_000).astype(np.int64)
    loss = rng.integers(0, 300, len(src)) / 10000.0
    return graphs.Graph(n, True, src, dst, lat, loss, "dring")


def _two_components(n=1500, seed=4):
    """Two RGGs side by side with no edge between them: half of every row is unreachable."""
    a = graphs.random_geometric(n, seed=seed)
    b = graphs.random_geometric(n, seed=seed + 1)
    return graphs.Graph(2 * n, False, np.concatenate([a.src, b.src + n]).astype(np.int32),
                        np.concatenate([a.dst, b.dst + n]).astype(np.int32),
                        np.concatenate([a.lat_ns, b.lat_ns]), np.concatenate([a.loss, b.loss]),
                        "two_rgg")


def _reweighted(g, lo, hi, seed=9):
    """g's structure with latencies U{lo..hi} ms (self-loops keep theirs)."""
    rng = np.random.default_rng(seed)
    lat = g.lat_ns.copy()
    off = g.src != g.dst
    lat[off] = rng.integers(lo, hi + 1, int(off.sum())) * 1_000_000
    return graphs.Graph(g.n, g.directed, g.src, g.dst, lat, g.loss, f"{g.name}_w{lo}_{hi}")


def _graph(which):
    if which == "rgg3000":
        return graphs.random_geometric(3000, seed=3)
    if which == "ba2000":
        return graphs.barabasi_albert(2000, seed=5)
    if which == "dring":
        return _directed_ring_graph()
    if which == "drgg2000":
        return graphs.directed_rgg(2000, seed=7)
    if which == "two_rgg":
        return _two_components()
    if which == "rgg2000_w1_2":
        return _reweighted(graphs.random_geometric(2000, seed=3), 1, 2)
    if which == "rgg2000_w1_5000":
        return _reweighted(graphs.random_geometric(2000, seed=3), 1, 5000)
    raise KeyError(which)


@pytest.mark.parametrize("which", ["rgg3000", "ba2000", "dring", "drgg2000", "two_rgg",
                                   "rgg2000_w1_2", "rgg2000_w1_5000"])
def test_msssp_full_tables(gpu, monkeypatch, which):
    """Forced multi-source kernel: the whole raw table (every source's own row) equals the
    oracle's, on undirected / directed / power-law / disconnected graphs and tie-heavy (1..2 ms)
    and wide (1..5000 ms, max weight >= 256) weights."""
    set_form(monkeypatch, kernel="ms")
    g = _graph(which)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_SPARSE_SSSP)
    assert st.dist_enc == 3, st.dist_enc
    exp = oracle.table(_el(g), True, oracle.ORC_INT_NS, 8, raw=True)
    lat = _unreached_as_oracle(lat, g)
    assert np.array_equal(lat, exp["lat_int"]), which
    assert np.array_equal(rel.view(np.uint64), exp["rel"].view(np.uint64)), which


@pytest.mark.parametrize("scale", [1, 40])
def test_msssp_distance_widths(gpu, monkeypatch, scale):
    """16-bit working distances where the graph's distance bound is below 0xFFFF (a candidate
    past it reads as not reached yet), 32-bit ones past it (the same graph with ~40x latencies,
    still in 1-ms quanta):
    the oracle's tables either way, the width reported in fw_block bit 16."""
    set_form(monkeypatch, kernel="ms")
    g0 = graphs.random_geometric(2200, seed=13)
    odd = (np.arange(g0.m) % 2) * 1_000_000 * (scale > 1)  # keep the quantum at 1 ms
    g = graphs.Graph(g0.n, g0.directed, g0.src, g0.dst, g0.lat_ns * scale + odd, g0.loss)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_SPARSE_SSSP)
    assert st.dist_enc == 3
    assert bool(st.fw_block & 16) == (scale == 1), st.fw_block
    exp = oracle.table(_el(g), True, oracle.ORC_INT_NS, 8, raw=True)
    assert np.array_equal(lat, exp["lat_int"])
    assert np.array_equal(rel.view(np.uint64), exp["rel"].view(np.uint64))


@pytest.mark.parametrize("slots", ["1", "3"])
def test_msssp_persistent_slots(gpu, monkeypatch, slots):
    """SRT_FORM ms_slots: one workgroup (or three) runs every batch in turn, so every batch after
    the first starts from the previous batch's working rows (re-initialised to INF)."""
    set_form(monkeypatch, kernel="ms")
    set_form(monkeypatch, ms_slots=slots)
    g = graphs.random_geometric(1200, seed=21)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_SPARSE_SSSP)
    exp = oracle.table(_el(g), True, oracle.ORC_INT_NS, 8, raw=True)
    assert np.array_equal(lat, exp["lat_int"])
    assert np.array_equal(rel.view(np.uint64), exp["rel"].view(np.uint64))


def _near(g_n, seed, x0, y0, k):
    """The k vertices of random_geometric(g_n, seed) nearest (x0, y0): a compact source set."""
    idx = np.arange(g_n, dtype=np.uint64)
    x, y = graphs._rand01(seed, 4, idx), graphs._rand01(seed, 5, idx)
    return np.argsort((x - x0) ** 2 + (y - y0) ** 2)[:k].astype(np.int32)


def test_msssp_c3_compact_sources_and_ties(gpu):
    """C3 itself (n = 20,000) with AUTO: a compact set of 300 sources (five batches, the last one
    partial) takes the multi-source kernel and is exact, with the tied-pair count equal to the
    wave kernel's on the same rows. A range of original ids is scattered across the square
    (random positions): small batches within the batch budget, the single-source kernels with a
    zero budget; both exact."""
    import os
    import torch
    g = graphs.random_geometric(20000, seed=3)
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    el = _el(g)
    srcs = _near(g.n, 3, 0.62, 0.41, 300)
    ds = torch.from_numpy(srcs).cuda()
    lat = torch.empty((len(srcs), g.n), dtype=torch.int32, device="cuda")
    rel = torch.empty((len(srcs), g.n), dtype=torch.float64, device="cuda")
    st = BuildStats()
    st.count_ties = 1
    sg.rows_list(ds.data_ptr(), len(srcs), lat.data_ptr(), rel.data_ptr(), None, st)
    torch.cuda.synchronize()
    assert st.dist_enc == 3, st.dist_enc
    got = lat.cpu().numpy().view(np.uint32).astype(np.uint64) * np.uint64(sg.quantum_ns)
    exp = oracle.sssp_list(el, srcs, nthreads=16)
    off = np.arange(g.n)[None, :] != srcs[:, None]
    assert np.array_equal(np.where(off, got, 0), np.where(off, exp["lat_int"], 0))
    r = rel.cpu().numpy()
    assert np.array_equal(r[off].view(np.uint64), exp["rel"][off].view(np.uint64))
    with form_env(kernel="wave"):
        st1 = BuildStats()
        st1.count_ties = 1
        sg.rows_list(ds.data_ptr(), len(srcs), lat.data_ptr(), rel.data_ptr(), None, st1)
        torch.cuda.synchronize()
    assert st1.dist_enc == 1 and st1.tied_pairs == st.tied_pairs, (st1.tied_pairs, st.tied_pairs)
    # 100 original ids: random positions, so small clusters -- batches of their own within the
    # batch budget, the single-source kernels without one
    exp = oracle.sssp_rows(el, 0, 100, nthreads=16)
    off = np.arange(g.n)[None, :] != np.arange(100)[:, None]
    st2 = BuildStats()
    sg.rows(0, 100, lat.data_ptr(), rel.data_ptr(), None, st2)
    torch.cuda.synchronize()
    assert st2.dist_enc == 3, st2.dist_enc
    got = lat[:100].cpu().numpy().view(np.uint32).astype(np.uint64) * np.uint64(sg.quantum_ns)
    assert np.array_equal(np.where(off, got, 0), np.where(off, exp["lat_int"], 0))
    r = rel[:100].cpu().numpy()
    assert np.array_equal(r[off].view(np.uint64), exp["rel"][off].view(np.uint64))
    sg.free()


@pytest.mark.parametrize("which", ["rgg3000", "dring"])
def test_msssp_source_list(gpu, monkeypatch, which):
    """srt_sparse_graph_rows_list with an unordered source list of 150 scattered vertices (small
    clusters, each a batch of its own within the batch budget): row i is source srcs[i]."""
    import torch
    set_form(monkeypatch, kernel="ms")
    g = _graph(which)
    rng = np.random.default_rng(77)
    srcs = rng.choice(g.n, 150, replace=False).astype(np.int32)
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    ds = torch.from_numpy(srcs).cuda()
    lat = torch.empty((len(srcs), g.n), dtype=torch.int32, device="cuda")
    rel = torch.empty((len(srcs), g.n), dtype=torch.float64, device="cuda")
    st = BuildStats()
    sg.rows_list(ds.data_ptr(), len(srcs), lat.data_ptr(), rel.data_ptr(), None, st)
    torch.cuda.synchronize()
    assert st.dist_enc == 3
    got = lat.cpu().numpy().view(np.uint32).astype(np.uint64) * np.uint64(sg.quantum_ns)
    exp = oracle.sssp_list(_el(g), srcs, nthreads=16)
    off = np.arange(g.n)[None, :] != srcs[:, None]
    assert np.array_equal(np.where(off, got, 0), np.where(off, exp["lat_int"], 0))
    r = rel.cpu().numpy()
    assert np.array_equal(r[off].view(np.uint64), exp["rel"][off].view(np.uint64))
    sg.free()


def test_msssp_compact_and_scattered_sources(gpu, monkeypatch):
    """A source list mixing a compact region (the 200 vertices nearest a point of the unit
    square) with 40 scattered vertices: clusters that fill 48 lanes within the hop radius and the
    small ones all take the multi-source kernel while the batches fit the budget (two per CU)."""
    import torch
    set_form(monkeypatch, kernel="ms")
    n = 4000
    g = graphs.random_geometric(n, seed=3)
    idx = np.arange(n, dtype=np.uint64)
    x, y = graphs._rand01(3, 4, idx), graphs._rand01(3, 5, idx)
    near = np.argsort((x - 0.3) ** 2 + (y - 0.6) ** 2)[:200]
    rng = np.random.default_rng(5)
    far = rng.choice(np.setdiff1d(np.arange(n), near), 40, replace=False)
    srcs = rng.permutation(np.concatenate([near, far])).astype(np.int32)
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    ds = torch.from_numpy(srcs).cuda()
    lat = torch.empty((len(srcs), g.n), dtype=torch.int32, device="cuda")
    rel = torch.empty((len(srcs), g.n), dtype=torch.float64, device="cuda")
    st = BuildStats()
    sg.rows_list(ds.data_ptr(), len(srcs), lat.data_ptr(), rel.data_ptr(), None, st)
    torch.cuda.synchronize()
    assert st.dist_enc == 3, st.dist_enc
    got = lat.cpu().numpy().view(np.uint32).astype(np.uint64) * np.uint64(sg.quantum_ns)
    exp = oracle.sssp_list(_el(g), srcs, nthreads=16)
    off = np.arange(g.n)[None, :] != srcs[:, None]
    assert np.array_equal(np.where(off, got, 0), np.where(off, exp["lat_int"], 0))
    r = rel.cpu().numpy()
    assert np.array_equal(r[off].view(np.uint64), exp["rel"][off].view(np.uint64))
    sg.free()


def test_msssp_past_the_batch_budget(gpu):
    """Every source of a 40,000-vertex RGG in one call: more clusters than the batch budget (two
    per CU), so the batches past it go to the single-source kernels and are scattered to their
    rows. Sampled rows from the whole range against the oracle."""
    import torch
    g = graphs.random_geometric(40000, seed=17)
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    lat = torch.empty((g.n, g.n), dtype=torch.int32, device="cuda")
    rel = torch.empty((g.n, g.n), dtype=torch.float64, device="cuda")
    st = BuildStats()
    sg.rows(0, g.n, lat.data_ptr(), rel.data_ptr(), None, st)
    torch.cuda.synchronize()
    assert st.dist_enc == 3, st.dist_enc
    rows = np.random.default_rng(4).choice(g.n, 64, replace=False).astype(np.int32)
    idx = torch.from_numpy(rows.astype(np.int64)).cuda()
    got = lat.index_select(0, idx).cpu().numpy().view(np.uint32).astype(np.uint64) \
        * np.uint64(sg.quantum_ns)
    r = rel.index_select(0, idx).cpu().numpy()
    del lat, rel
    exp = oracle.sssp_list(_el(g), rows, nthreads=16)
    off = np.arange(g.n)[None, :] != rows[:, None]
    assert np.array_equal(np.where(off, got, 0), np.where(off, exp["lat_int"], 0))
    assert np.array_equal(r[off].view(np.uint64), exp["rel"][off].view(np.uint64))
    sg.free()
