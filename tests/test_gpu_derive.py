"""Neighbour-row derivation (shadow_amd/csrc/derive.hip): in a full-table sparse build on the
workgroup kernel, the rows of an independent set of low-degree vertices come from their
neighbours' rows -- distances as neighbour minimums, canonical predecessors as the best of the
optimal neighbours' canonical arcs, reliability re-formed in path order from the source -- and the
rest ("core") from the kernel, which also emits its canonical arcs.

Checked against the oracle's Dijkstra (oracle.c, restating topology.c:1578-1814) bit for bit in
latency and within 1e-12 in reliability, and against the same build with SRT_FORM derive=0 (the
kernel for every row): identical tables and tied-pair counts."""
import numpy as np
import pytest
from conftest import set_form

import oracle
from shadow_amd import graphs
from shadow_amd._lib import ALGO_SPARSE_SSSP, BuildStats
from shadow_amd.topology import SparseGraph, build_tables

pytestmark = pytest.mark.gpu
REL_TOL = 1e-12
DERIVED = 64  # srt_build_stats.fw_block bit of a build with derived rows


def _el(g):
    return oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)


@pytest.mark.parametrize("lat_max", [1, 2, 20, 100])
def test_derived_rows_full_table_small(gpu, monkeypatch, lat_max):
    """BA 2,500 (m = 3) on the workgroup kernel: ~46% of the rows derived. lat_max = 1-2 makes
    nearly every pair tied (the canonical rule decides), 100 is C5's distribution."""
    set_form(monkeypatch, kernel="wg")
    g = graphs.barabasi_albert(2500, seed=31, lat_max=lat_max)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_SPARSE_SSSP)
    assert st.dist_enc == 2 and st.fw_block & DERIVED, (st.dist_enc, st.fw_block)
    exp = oracle.table(_el(g), True, oracle.ORC_INT_NS, 8, raw=True)
    assert np.array_equal(lat, exp["lat_int"])
    err = np.abs(rel - exp["rel"]) / np.maximum(np.abs(exp["rel"]), 1e-300)
    assert float(err.max()) <= REL_TOL
    set_form(monkeypatch, derive="0")
    lat0, rel0, st0 = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                   algo=ALGO_SPARSE_SSSP)
    assert not st0.fw_block & DERIVED
    assert np.array_equal(lat, lat0) and np.array_equal(rel, rel0)


def test_derived_rows_ba40000_device(gpu, monkeypatch):
    """BA 40,000 through srt_sparse_graph_rows (the bench's entry point, AUTO: the workgroup
    kernel): every entry equal to the all-kernel build, the tied-pair count too, and sampled
    derived and core rows against the oracle."""
    import torch
    g = graphs.barabasi_albert(40_000, seed=7)
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    n = g.n
    lat = torch.empty((n, n), dtype=torch.int32, device="cuda")
    rel = torch.empty((n, n), dtype=torch.float64, device="cuda")
    st = BuildStats()
    st.count_ties = 1
    sg.rows(0, n, lat.data_ptr(), rel.data_ptr(), None, st)
    torch.cuda.synchronize()
    assert st.dist_enc == 2 and st.fw_block & DERIVED, (st.dist_enc, st.fw_block)
    # sampled rows: degree-3 vertices (derived) and hubs (core)
    deg = np.bincount(np.concatenate([g.src[g.src != g.dst], g.dst[g.src != g.dst]]),
                      minlength=n)
    rows = np.unique(np.concatenate([np.nonzero(deg == 3)[0][::2000], np.argsort(-deg)[:6],
                                     [0, 1, n - 1]])).astype(np.int32)
    idx = torch.from_numpy(rows.astype(np.int64)).cuda()
    glat = lat.index_select(0, idx).cpu().numpy().view(np.uint32).astype(np.uint64) \
        * np.uint64(sg.quantum_ns)
    grel = rel.index_select(0, idx).cpu().numpy()
    exp = oracle.sssp_list(_el(g), rows, nthreads=16)
    off = np.arange(n)[None, :] != rows[:, None]
    assert np.array_equal(np.where(off, glat, 0), np.where(off, exp["lat_int"], 0))
    err = np.abs(grel - exp["rel"]) / np.maximum(np.abs(exp["rel"]), 1e-300)
    assert float(err[off].max()) <= REL_TOL
    # the all-kernel build into a second pair of tables: identical
    set_form(monkeypatch, derive="0")
    lat0 = torch.empty_like(lat)
    rel0 = torch.empty_like(rel)
    st0 = BuildStats()
    st0.count_ties = 1
    sg.rows(0, n, lat0.data_ptr(), rel0.data_ptr(), None, st0)
    torch.cuda.synchronize()
    assert not st0.fw_block & DERIVED
    assert torch.equal(lat, lat0)
    assert torch.equal(rel.view(torch.int64), rel0.view(torch.int64))
    assert st.tied_pairs == st0.tied_pairs
    sg.free()


def test_derived_rows_c5_full_size(gpu):
    """C5 itself -- the 100,000-vertex BA graph (m = 3, U{1..100} ms, seed 5, the
    bench's graph) -- through srt_sparse_graph_rows(0, n), the bench's default form: the core
    rows by the workgroup kernel and ~46% of the rows derived from their neighbours' (120 GB of
    tables on one MI355X). Sampled derived (degree-3) and core (hub and other) rows against the
    oracle's Dijkstra, bit for bit in latency and within 1e-12 in reliability; the derived-row
    count is the one the bench reports."""
    import torch
    g = graphs.barabasi_albert(100_000, seed=5)
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    n = g.n
    lat = torch.empty((n, n), dtype=torch.int32, device="cuda")
    rel = torch.empty((n, n), dtype=torch.float64, device="cuda")
    st = BuildStats()
    sg.rows(0, n, lat.data_ptr(), rel.data_ptr(), None, st)
    torch.cuda.synchronize()
    assert st.dist_enc == 2 and st.fw_block & DERIVED, (st.dist_enc, st.fw_block)
    assert 40_000 < st.n_derived < 50_000, st.n_derived
    deg = np.bincount(np.concatenate([g.src[g.src != g.dst], g.dst[g.src != g.dst]]),
                      minlength=n)
    rng = np.random.default_rng(5)
    rows = np.unique(np.concatenate([rng.choice(np.nonzero(deg == 3)[0], 12, replace=False),
                                     rng.choice(np.nonzero(deg >= 5)[0], 8, replace=False),
                                     np.argsort(-deg)[:4], [0, 1, n - 1]])).astype(np.int32)
    idx = torch.from_numpy(rows.astype(np.int64)).cuda()
    glat = lat.index_select(0, idx).cpu().numpy().view(np.uint32).astype(np.uint64) \
        * np.uint64(sg.quantum_ns)
    grel = rel.index_select(0, idx).cpu().numpy()
    del lat, rel
    torch.cuda.empty_cache()
    exp = oracle.sssp_list(_el(g), rows, nthreads=16)
    off = np.arange(n)[None, :] != rows[:, None]
    bad = np.argwhere(np.where(off, glat, 0) != np.where(off, exp["lat_int"], 0))
    assert bad.size == 0, f"{len(bad)} latency mismatches, first {bad[:5].tolist()}"
    err = np.abs(grel - exp["rel"]) / np.maximum(np.abs(exp["rel"]), 1e-300)
    assert float(err[off].max()) <= REL_TOL
    sg.free()
