"""The metric dense regime (VERDICT r04 "measure the dense regime Tor-atlas graphs actually hit"):
points of the unit square, complete graph, latency max(1, round(300 * dist)) ms. Shortest paths are
mostly the direct arc or a detour shorter by a rounding, so distances run to hundreds of quanta: the
level budget is passed and the build takes the blocked Floyd-Warshall (u16 f16-compare rounds).

The device generator (srt_gen_metric_device) is pinned entry by entry against the oracle's
restatement (orc_dense_weight), and the built rows against the oracle's dense Dijkstra
(orc_metric_sample, topology.c:1578-1814 / :1286-1389 restated): latency bit-exact in integer ns,
reliability within 1e-12 relative."""
import ctypes

import numpy as np
import pytest

import oracle
from shadow_amd import _lib

pytestmark = pytest.mark.gpu
REL_TOL = 1e-12
SCALE, SELF_MAX, LOSS_MAX = 300, 10, 500


def _gen(L, n, ld, seed):
    import torch
    w = torch.empty((ld, ld), dtype=torch.int32, device="cuda")
    r = torch.empty((ld, ld), dtype=torch.float64, device="cuda")
    _lib.check(L.srt_gen_metric_device(n, ld, 0, ld, seed, SCALE, SELF_MAX, LOSS_MAX, w.data_ptr(),
                                       r.data_ptr(), None), "srt_gen_metric_device")
    return w, r


def test_metric_generator_matches_oracle(gpu):
    import torch
    L = _lib.lib()
    n = ld = 1024
    w, _ = _gen(L, n, ld, seed=44)
    torch.cuda.synchronize()
    wh = w.cpu().numpy().view(np.uint32)
    rng = np.random.default_rng(0)
    for i, j in list(zip(rng.integers(0, n, 300), rng.integers(0, n, 300))) + [(5, 5), (0, 1)]:
        assert wh[i, j] == oracle.dense_weight(44, 0, SCALE, SELF_MAX, int(i), int(j)), (i, j)
    assert np.array_equal(wh[:n, :n], wh[:n, :n].T)
    off = ~np.eye(n, dtype=bool)
    assert wh[:n, :n][off].min() >= 1 and wh[:n, :n][off].max() <= 425


@pytest.mark.parametrize("n", [4096])
def test_metric_build_takes_fw_and_matches_oracle(gpu, n):
    """default dispatch: the levels are tried (n >= 4,096) and refused on budget, the FW runs"""
    import torch
    L = _lib.lib()
    ld = n
    w, r = _gen(L, n, ld, seed=45)
    lat = torch.empty_like(w)
    rel = torch.empty_like(r)
    st = _lib.BuildStats()
    _lib.check(L.srt_dense_build_device(n, ld, 0, w.data_ptr(), r.data_ptr(), lat.data_ptr(),
                                        rel.data_ptr(), None, 0, ctypes.byref(st)), "build")
    torch.cuda.synchronize()
    assert st.dist_enc != 12 and st.levels == 0, (st.dist_enc, st.levels)
    rows = np.array([0, 1, 1000, 2047, 3000, n - 1], np.int32)
    idx = torch.from_numpy(rows.astype(np.int64)).cuda()
    glat = lat.index_select(0, idx).cpu().numpy().view(np.uint32).astype(np.uint64) \
        * np.uint64(1_000_000)
    grel = rel.index_select(0, idx).cpu().numpy()
    clat, crel, _, _ = oracle.complete_sample(n, 45, 0, SELF_MAX, LOSS_MAX, rows, 8, metric=SCALE)
    off = np.arange(n)[None, :] != rows[:, None]
    bad = np.argwhere(np.where(off, glat, 0) != np.where(off, clat, 0))
    assert bad.size == 0, f"{len(bad)} latency mismatches, first {bad[:5].tolist()}"
    err = np.abs(grel - crel) / np.maximum(crel, 1e-300)
    assert float(err[off].max()) <= REL_TOL
    assert clat.max() > 200 * 1_000_000  # the regime: distances of hundreds of ms


def test_metric_full_size_c4metric(gpu):
    """the C4metric workload itself (n = 32,768, seed 44, the bench's config)
    through the default dispatch: the level build settles too few pairs in its first batch and
    hands over to the u16 FW rounds and rel_deep_kernel; 24 rows spread over the matrix (the first,
    the last, row-block edges and random ones) against the oracle's dense Dijkstra."""
    import torch
    L = _lib.lib()
    n = ld = 32768
    w, r = _gen(L, n, ld, seed=44)
    lat = torch.empty_like(w)
    rel = torch.empty_like(r)
    st = _lib.BuildStats()
    _lib.check(L.srt_dense_build_device(n, ld, 0, w.data_ptr(), r.data_ptr(), lat.data_ptr(),
                                        rel.data_ptr(), None, 0, ctypes.byref(st)), "build")
    torch.cuda.synchronize()
    assert st.dist_enc != 12 and st.levels == 0, (st.dist_enc, st.levels)
    del w, r
    rng = np.random.default_rng(7)
    rows = np.unique(np.concatenate([[0, 1, 127, 128, 16383, 16384, 32640, n - 1],
                                     rng.integers(0, n, 16)])).astype(np.int32)
    assert len(rows) >= 16
    idx = torch.from_numpy(rows.astype(np.int64)).cuda()
    glat = lat.index_select(0, idx).cpu().numpy().view(np.uint32).astype(np.uint64) \
        * np.uint64(1_000_000)
    grel = rel.index_select(0, idx).cpu().numpy()
    del lat, rel
    torch.cuda.empty_cache()
    clat, crel, _, _ = oracle.complete_sample(n, 44, 0, SELF_MAX, LOSS_MAX, rows, 16, metric=SCALE)
    off = np.arange(n)[None, :] != rows[:, None]
    bad = np.argwhere(np.where(off, glat, 0) != np.where(off, clat, 0))
    assert bad.size == 0, f"{len(bad)} latency mismatches, first {bad[:5].tolist()}"
    err = np.abs(grel - crel) / np.maximum(crel, 1e-300)
    assert float(err[off].max()) <= REL_TOL
    assert clat.max() > 300 * 1_000_000
