"""Sparse SSSP through the device C-ABI (srt_sparse_graph_*) and the table builds, every kernel
form: the wave-per-source bucket kernel (C3-shaped RGG), the workgroup-per-source kernel with the
distance row packed in LDS (C5-shaped 100k-node Barabasi-Albert graph), and the block kernel
(sparse.hip: LDS working set, HBM past ~20k vertices, bucket overflows).

Latency bit-exact in integer ns, reliability within 1e-12 relative (north_star). Every row is its
own source's (no mirror), compared with oracle.sssp_rows / the oracle's raw table off the
diagonal.
"""
import numpy as np
import pytest
from conftest import set_form

import oracle
from shadow_amd import graphs
from shadow_amd._lib import ALGO_SPARSE_SSSP
from shadow_amd.topology import SparseGraph, build_tables

pytestmark = pytest.mark.gpu
REL_TOL = 1e-12


@pytest.fixture(autouse=True)
def _single_source_kernels(monkeypatch):
    """These tests pin the single-source kernels (SRT_FORM kernel=wave unless a test names
    another); the multi-source kernel that AUTO gives local graphs (msssp.hip, dist_enc 3) has
    its own file, tests/test_gpu_msssp.py."""
    set_form(monkeypatch, kernel="wave")


def _rows_on_gpu(sg, s0, s1, torch, stats=None):
    lat = torch.empty((s1 - s0, sg.n), dtype=torch.int32, device="cuda")
    rel = torch.empty((s1 - s0, sg.n), dtype=torch.float64, device="cuda")
    sg.rows(s0, s1, lat.data_ptr(), rel.data_ptr(), None, stats)
    torch.cuda.synchronize()
    return (lat.cpu().numpy().view(np.uint32).astype(np.uint64) * np.uint64(sg.quantum_ns),
            rel.cpu().numpy())


def _check_rows(g, ranges, torch, want_enc=None):
    from shadow_amd._lib import BuildStats
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    for s0, s1 in ranges:
        st = BuildStats()
        lat, rel = _rows_on_gpu(sg, s0, s1, torch, st)
        if want_enc is not None:
            assert st.dist_enc == want_enc, (s0, s1, st.dist_enc)
        exp = oracle.sssp_rows(el, s0, s1, nthreads=8)
        off = np.arange(g.n)[None, :] != np.arange(s0, s1)[:, None]
        assert np.array_equal(np.where(off, lat, 0), np.where(off, exp["lat_int"], 0)), (s0, s1)
        err = np.abs(rel - exp["rel"]) / np.maximum(exp["rel"], 1e-300)
        assert float(err[off].max()) <= REL_TOL, (s0, s1)
    sg.free()


def test_c3_shape_rgg_20000_wave_kernel_rows(gpu):
    import torch
    g = graphs.random_geometric(20000, seed=3)
    _check_rows(g, [(0, 96), (9_950, 10_050), (19_900, 20_000)], torch, want_enc=1)


def test_c5_shape_ba_100000_workgroup_kernel_rows(gpu, monkeypatch):
    """C5's graph takes the workgroup kernel (srt_build_stats.dist_enc == 2 for sparse builds)."""
    import torch
    set_form(monkeypatch, kernel="auto")
    g = graphs.barabasi_albert(100_000, seed=5)
    _check_rows(g, [(0, 48), (50_000, 50_016), (99_984, 100_000)], torch, want_enc=2)


@pytest.mark.parametrize("which", ["rgg21000", "ba21000", "directed21000"])
def test_block_kernel_hbm_workset_rows(gpu, monkeypatch, which):
    """The block kernel past srt_sparse_max_n() (~20,160 vertices): its working set in a
    per-workgroup HBM slot instead of LDS, on sampled row ranges."""
    import torch
    set_form(monkeypatch, kernel="block")
    n = 21000
    if which == "rgg21000":
        g = graphs.random_geometric(n, seed=3)
    elif which == "ba21000":
        g = graphs.barabasi_albert(n, seed=5)
    else:
        rng = np.random.default_rng(12)
        m = 8 * n
        ring = np.arange(n)
        src = np.concatenate([rng.integers(0, n, m), ring, ring]).astype(np.int32)
        dst = np.concatenate([rng.integers(0, n, m), (ring + 1) % n, ring]).astype(np.int32)
        lat = (rng.integers(1, 20, len(src)) * 1_000_000).astype(np.int64)
        loss = rng.integers(0, 300, len(src)) / 10000.0
        g = graphs.Graph(n, True, src, dst, lat, loss)
    _check_rows(g, [(0, 48), (n - 48, n)], torch)


@pytest.mark.parametrize("which", ["rgg3000", "directed"])
@pytest.mark.parametrize("bcap", ["3", "64"])
def test_wave_kernel_bucket_overflow_fallback(gpu, monkeypatch, which, bcap):
    """Wave-per-source bucket kernel (wsssp.hip) with tiny bucket capacities: sources whose
    buckets overflow are recomputed by the workgroup kernel, and the table stays exact."""
    set_form(monkeypatch, bcap=bcap)
    if which == "rgg3000":
        g = graphs.random_geometric(3000, seed=3)
    else:
        rng = np.random.default_rng(12)
        n, m = 400, 3000
        ring = np.arange(n)
        src = np.concatenate([rng.integers(0, n, m), ring, ring]).astype(np.int32)
        dst = np.concatenate([rng.integers(0, n, m), (ring + 1) % n, ring]).astype(np.int32)
        lat = (rng.integers(1, 20, len(src)) * 1_000_000).astype(np.int64)
        loss = rng.integers(0, 300, len(src)) / 10000.0
        g = graphs.Graph(n, True, src, dst, lat, loss)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_SPARSE_SSSP)
    exp = oracle.table(oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss),
                       True, oracle.ORC_INT_NS, 8, raw=True)
    assert np.array_equal(lat, exp["lat_int"])
    err = np.abs(rel - exp["rel"]) / np.maximum(np.abs(exp["rel"]), 1e-300)
    assert float(err.max()) <= REL_TOL
    if bcap == "3":
        assert st.ess_arcs > 0, "expected some sources to overflow and be recomputed"


def test_wave_kernel_matches_block_kernel_c3_rows(gpu, monkeypatch):
    """The two sparse kernels agree bit for bit on C3-shaped rows (the wave kernel is the default,
    SRT_FORM kernel=block selects the block kernel)."""
    import torch
    g = graphs.random_geometric(20000, seed=3)
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    a = _rows_on_gpu(sg, 5000, 5256, torch)
    set_form(monkeypatch, kernel="block")
    b = _rows_on_gpu(sg, 5000, 5256, torch)
    sg.free()
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("which", ["rgg3000", "rgg6000", "ba20000", "directed"])
def test_wave_kernel_working_row_forms(gpu, which):
    """The wave kernel's forms: working distance row in LDS while eight rows fit a CU (n <= 4,096)
    or in global memory, and reliability kept in a relabelled row gathered at the end (local
    graphs) or written to the output rows at settle time (ba20000, not local). The same exact
    rows either way (fw_block bits 1 and 2 name the form)."""
    import torch
    from shadow_amd._lib import BuildStats
    if which == "rgg3000":
        g = graphs.random_geometric(3000, seed=3)
    elif which == "rgg6000":
        g = graphs.random_geometric(6000, seed=4)
    elif which == "ba20000":
        g = graphs.barabasi_albert(20000, seed=5)
    else:
        rng = np.random.default_rng(12)
        n, m = 400, 3000
        ring = np.arange(n)
        src = np.concatenate([rng.integers(0, n, m), ring, ring]).astype(np.int32)
        dst = np.concatenate([rng.integers(0, n, m), (ring + 1) % n, ring]).astype(np.int32)
        lat = (rng.integers(1, 20, len(src)) * 1_000_000).astype(np.int64)
        loss = rng.integers(0, 300, len(src)) / 10000.0
        g = graphs.Graph(n, True, src, dst, lat, loss)
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    st = BuildStats()
    _rows_on_gpu(sg, 0, 1, torch, st)
    sg.free()
    want = {"rgg3000": 3, "rgg6000": 2, "ba20000": 0, "directed": 3}[which]
    assert st.fw_block & 3 == want, st.fw_block
    _check_rows(g, [(0, 64), (g.n - 64, g.n)], torch, want_enc=1)


@pytest.mark.parametrize("which", ["ba2000", "ba3000_w20", "rgg3000"])
def test_workgroup_kernel_packed_rows(gpu, monkeypatch, which):
    """SRT_FORM kernel=wg: the workgroup-per-source kernel (distance row packed 3 x 10 bits in LDS)
    on any undirected graph whose probe source shows every distance fits (2 ecc <= 1022); else
    the wave kernel. Either way the exact tables."""
    set_form(monkeypatch, kernel="wg")
    if which == "ba2000":
        g = graphs.barabasi_albert(2000, seed=5)
    elif which == "ba3000_w20":
        g = graphs.barabasi_albert(3000, seed=8, lat_max=20)
    else:
        g = graphs.random_geometric(3000, seed=3)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_SPARSE_SSSP)
    exp = oracle.table(oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss),
                       True, oracle.ORC_INT_NS, 8, raw=True)
    assert np.array_equal(lat, exp["lat_int"])
    assert np.array_equal(rel, exp["rel"])
    if which.startswith("ba"):
        assert st.dist_enc == 2, "the workgroup kernel should take power-law graphs with small distances"


@pytest.mark.parametrize("bcap", ["3", "64"])
def test_workgroup_kernel_overflow_fallback(gpu, monkeypatch, bcap):
    """Forced bucket overflows in the workgroup kernel: flagged sources go to the wave kernel and,
    when that overflows too, to the block kernel; the tables stay exact."""
    set_form(monkeypatch, kernel="wg")
    set_form(monkeypatch, bcap=bcap)
    g = graphs.barabasi_albert(1500, seed=6)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_SPARSE_SSSP)
    exp = oracle.table(oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss),
                       True, oracle.ORC_INT_NS, 8, raw=True)
    assert np.array_equal(lat, exp["lat_int"])
    assert np.array_equal(rel, exp["rel"])


@pytest.mark.parametrize("which", ["ba2000", "ba2500_many_losses", "ba2000_w130"])
def test_workgroup_kernel_forms(gpu, monkeypatch, which):
    """The workgroup kernel's forms give the same exact tables: compact 8-byte arcs with the table
    of distinct reliabilities (<= 256 of them, weights < 128 quanta), or 16-byte arcs (> 256
    distinct losses, or weights of 128 quanta and more); fw_block bit 2 names the form."""
    set_form(monkeypatch, kernel="wg")
    g = graphs.barabasi_albert(2500 if which == "ba2500_many_losses" else 2000, seed=7,
                               lat_max=130 if which == "ba2000_w130" else 100)
    if which == "ba2500_many_losses":  # continuous losses: one distinct reliability per edge
        rng = np.random.default_rng(3)
        g = graphs.Graph(g.n, g.directed, g.src, g.dst, g.lat_ns, rng.random(g.m) * 0.05)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_SPARSE_SSSP)
    exp = oracle.table(oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss),
                       True, oracle.ORC_INT_NS, 8, raw=True)
    assert st.dist_enc == 2
    assert st.fw_block & 7 == (7 if which == "ba2000" else 5), st.fw_block
    assert np.array_equal(lat, exp["lat_int"])
    assert np.array_equal(rel, exp["rel"])


@pytest.mark.parametrize("lat_max", [1, 2, 20, 127])
def test_workgroup_kernel_two_level_steps(gpu, monkeypatch, lat_max):
    """A Dial step of the workgroup kernel settles buckets d and d + 1 together. Weights of 1..2
    quanta push into d + 1 during nearly every step (the consumed-prefix counts); 127 quanta is
    the largest compact-arc weight, where the bucket ring must hold max_w + 2 buckets."""
    set_form(monkeypatch, kernel="wg")
    g = graphs.barabasi_albert(2000, seed=9, lat_max=lat_max)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_SPARSE_SSSP)
    exp = oracle.table(oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss),
                       True, oracle.ORC_INT_NS, 8, raw=True)
    assert st.dist_enc == 2
    assert np.array_equal(lat, exp["lat_int"])
    assert np.array_equal(rel, exp["rel"])


def test_workgroup_kernel_two_level_stress(gpu, monkeypatch):
    """Two-level Dial steps with weights of 1..2 quanta on many sources (the skipped
    buckets' reset raced the other waves' bucket search; it now follows the first chunk's scan
    barrier). A race shows up as wrong rows or a hang; the test runs under the suite timeout."""
    set_form(monkeypatch, kernel="wg")
    g = graphs.barabasi_albert(12000, seed=11, lat_max=2)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_SPARSE_SSSP)
    assert st.dist_enc == 2
    rows = np.r_[0:16, 6000:6016, 11984:12000]
    exp = oracle.sssp_list(oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss),
                           rows, nthreads=8)
    for i, s in enumerate(rows):
        off = np.arange(g.n) != s
        assert np.array_equal(lat[s][off], exp["lat_int"][i][off]), s
        assert np.array_equal(rel[s][off], exp["rel"][i][off]), s
