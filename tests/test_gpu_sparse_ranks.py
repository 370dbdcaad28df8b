"""The source-sharded sparse build at 4 and 8 ranks: each rank settles its block of
sources with the sparse kernels, then the rows are all-gathered (srt_sparse_allgather /
ncclAllGather). Ranks are virtual (SRT_VIRTUAL_RANKS: R ranks on device 0, collectives as device
copies), so the schedule, the shard boundaries and the gather run as they would on R GPUs.

Against oracle.sssp_list (the restatement of topology.c:1578-1814's per-source Dijkstra):
latency bit-exact in integer ns, reliability within 1e-12 relative (north_star)."""
import numpy as np
import pytest

import oracle
from shadow_amd import graphs
from shadow_amd._lib import ALGO_AUTO, ALGO_SPARSE_SSSP
from shadow_amd.topology import build_tables, build_tables_subset

pytestmark = pytest.mark.gpu
REL_TOL = 1e-12


def _el(g):
    return oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)


def _rel_err(got, exp):
    return float((np.abs(got - exp) / np.maximum(np.abs(exp), 1e-300)).max())


def test_c5_attached_2000_eight_virtual_ranks(gpu, monkeypatch):
    """C5 (100,000-vertex BA graph) with ~2,000 attached vertices on 8 ranks: each rank builds
    ~250 sources' rows over the whole graph, the sub-table is all-gathered; the same sub-table as
    one GPU and as the oracle."""
    g = graphs.barabasi_albert(100_000, seed=5)
    rng = np.random.default_rng(808)
    verts = np.unique(np.concatenate([rng.choice(g.n, 2000, replace=False), [0, 1, 99_999]]))
    verts = verts.astype(np.int32)
    lat1, rel1, _, mn1, st1 = build_tables_subset(g.n, False, g.src, g.dst, g.lat_ns, g.loss,
                                                  verts=verts, algo=ALGO_AUTO)
    assert st1.algo == ALGO_SPARSE_SSSP
    monkeypatch.setenv("SRT_VIRTUAL_RANKS", "8")
    lat8, rel8, _, mn8, st8 = build_tables_subset(g.n, False, g.src, g.dst, g.lat_ns, g.loss,
                                                  verts=verts, algo=ALGO_AUTO, ngpus=8)
    assert st8.algo == ALGO_SPARSE_SSSP
    assert np.array_equal(lat1, lat8) and np.array_equal(rel1, rel8) and mn1 == mn8
    rows = oracle.sssp_list(_el(g), verts, nthreads=16)
    elat = rows["lat_int"][:, verts]
    erel = rows["rel"][:, verts]
    off = ~np.eye(len(verts), dtype=bool)
    assert np.array_equal(lat8[off], elat[off])
    assert _rel_err(rel8[off], erel[off]) <= REL_TOL


def test_c3_full_table_four_virtual_ranks(gpu, monkeypatch):
    """C3 (20,000-vertex RGG, the multi-source kernel) full table on 4 ranks: 5,000 source rows
    per rank, all-gathered into the 20,000 x 20,000 table; every row against the oracle (in
    blocks of 2,000 rows)."""
    g = graphs.random_geometric(20000, seed=3)
    monkeypatch.setenv("SRT_VIRTUAL_RANKS", "4")
    lat, rel, st = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss, algo=ALGO_AUTO,
                                ngpus=1)
    assert st.algo == ALGO_SPARSE_SSSP
    el = _el(g)
    worst = 0.0
    for s0 in range(0, g.n, 2000):
        s1 = min(g.n, s0 + 2000)
        exp = oracle.sssp_rows(el, s0, s1, nthreads=16)
        off = np.arange(g.n)[None, :] != np.arange(s0, s1)[:, None]
        assert np.array_equal(np.where(off, lat[s0:s1], 0), np.where(off, exp["lat_int"], 0)), \
            f"latency mismatch in rows {s0}..{s1}"
        worst = max(worst, _rel_err(np.where(off, rel[s0:s1], 1.0),
                                    np.where(off, exp["rel"], 1.0)))
    assert worst <= REL_TOL, worst
