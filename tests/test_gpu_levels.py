"""Dense distances by bit-parallel Dial levels (shadow_amd/csrc/levels.hip, dist_enc 12) against
the CPU oracle's Dijkstra (oracle.c, restating topology.c:1578-1814), bit for bit in latency and
reliability (the post pass forms predecessors and path-order products from the level distances).

SRT_FORM levels=1 forces the level search at any size (the default takes it from n >= 4,096 when
its budget beats the FW); when the graph's distances pass the level budget the build must fall back
to the FW and still match. Sharded: virtual ranks on one GPU (row shards, arcs broadcast per rank's
segment, one verdict for all ranks)."""
import ctypes

import numpy as np
import pytest
from conftest import set_form

import oracle
from shadow_amd import _lib, graphs
from shadow_amd._lib import ALGO_DENSE_FW
from shadow_amd.topology import build_tables

pytestmark = pytest.mark.gpu
REL_TOL = 1e-12
MS = 1_000_000
LEVELS = 12


def _oracle(g):
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    return oracle.table(el, True, oracle.ORC_INT_NS, 8, raw=True)


def _check(g, lat, rel, what):
    exp = _oracle(g)
    bad = np.argwhere(lat != np.asarray(exp["lat_int"], np.uint64))
    assert bad.size == 0, f"{what}: {len(bad)} latency mismatches, first {bad[:5].tolist()}"
    err = np.abs(rel - exp["rel"]) / np.maximum(np.abs(exp["rel"]), 1e-300)
    assert float(err.max()) <= REL_TOL, f"{what}: max rel error {err.max()}"


def _directed_dense(n, seed, wmax):
    rng = np.random.default_rng(seed)
    i, j = np.nonzero(rng.random((n, n)) < 0.35)
    keep = i != j
    i, j = i[keep], j[keep]
    ring = np.arange(n)  # strongly connected
    src = np.concatenate([i, ring]).astype(np.int32)
    dst = np.concatenate([j, (ring + 1) % n]).astype(np.int32)
    lat = (rng.integers(1, wmax + 1, len(src)) * MS).astype(np.int64)
    loss = rng.integers(0, 300, len(src)) / 10000.0
    return graphs.Graph(n, True, src, dst, lat, loss, f"directed{n}")


@pytest.mark.parametrize("kind", ["complete300", "complete1000", "ties", "directed", "c1like",
                                  "manyrel", "transposed", "ties_transposed"])
def test_levels_match_oracle(gpu, monkeypatch, kind):
    """The post pass carries r(pred, t) as an index into the build's table of distinct arc
    reliabilities: by default one target-major word per pair with the level beside it
    (lvl_pred_kernel), one transpose, then rel_pk_kernel, which writes the u32 rows too;
    "transposed" (SRT_FORM pkw=0) keeps the u8 level rows and rel_tree_kernel; "manyrel" (more
    distinct values than the table holds) takes the f64 rows. "c1like" has distances past 31 quanta: the packed
    words cannot hold its levels (the transposed form, then the sweeps past 64)."""
    set_form(monkeypatch, levels="1")
    if kind in ("transposed", "ties_transposed"):
        set_form(monkeypatch, levels="1", pkw="0")
    if kind in ("complete300", "transposed"):
        g = graphs.complete_graph(300, seed=7)
    elif kind == "complete1000":  # C2's distribution: distances up to 9 quanta
        g = graphs.complete_graph(1000, seed=2)
    elif kind in ("ties", "ties_transposed"):  # 1-3 ms arcs: equal-length paths
        g = graphs.complete_graph(640, seed=11, lat_max=3)
    elif kind == "directed":  # in-arcs from the columns of w
        g = _directed_dense(500, 5, 40)
    elif kind == "manyrel":  # 44,850 distinct loss values: past the table's 2,048
        g0 = graphs.complete_graph(300, seed=9)
        loss = np.random.default_rng(9).random(g0.m) * 0.05
        g = graphs.Graph(g0.n, False, g0.src, g0.dst, g0.lat_ns, loss, "manyrel")
    else:  # C1's distribution at 50 vertices: distances of tens of quanta
        g = graphs.complete_graph(50, seed=1)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_DENSE_FW)
    assert st.dist_enc == LEVELS and 1 <= st.levels <= 254, (st.dist_enc, st.levels)
    _check(g, lat, rel, kind)


def test_levels_over_budget_falls_back(gpu, monkeypatch):
    """A ring of 200-ms hops: distances pass the 254-level budget, so the FW builds it."""
    set_form(monkeypatch, levels="1")
    n = 300
    src = np.arange(n, dtype=np.int32)
    dst = ((src + 1) % n).astype(np.int32)
    lat = np.full(n, 200 * MS, np.int64) + (src % 3) * MS
    loss = (src % 7) / 1000.0
    g = graphs.Graph(n, False, src, dst, lat, loss, "ring200")
    lat_t, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                  algo=ALGO_DENSE_FW)
    assert st.dist_enc != LEVELS and st.levels == 0
    _check(g, lat_t, rel, "ring fallback")


def test_levels_default_at_4096(gpu):
    """n = 4,096: the default dispatch takes the levels (no environment), rows vs the oracle."""
    import torch
    L = _lib.lib()
    n = ld = 4096
    w = torch.empty((ld, ld), dtype=torch.int32, device="cuda")
    r = torch.empty((ld, ld), dtype=torch.float64, device="cuda")
    _lib.check(L.srt_gen_complete_device(n, ld, 0, ld, 6, 1000, 10, 500, w.data_ptr(),
                                         r.data_ptr(), None), "generate")
    lat = torch.empty_like(w)
    rel = torch.empty_like(r)
    st = _lib.BuildStats()
    st.time_kernels = 1
    _lib.check(L.srt_dense_build_device(n, ld, 0, w.data_ptr(), r.data_ptr(), lat.data_ptr(),
                                        rel.data_ptr(), None, 0, ctypes.byref(st)), "build")
    torch.cuda.synchronize()
    assert st.dist_enc == LEVELS, st.dist_enc
    assert st.n_update == st.levels and st.work_bytes > 0
    rows = np.array([0, 1, 777, 2048, 4000, 4095], np.int32)
    idx = torch.from_numpy(rows.astype(np.int64)).cuda()
    glat = lat.index_select(0, idx).cpu().numpy().view(np.uint32).astype(np.uint64) * np.uint64(MS)
    grel = rel.index_select(0, idx).cpu().numpy()
    clat, crel, _, _ = oracle.complete_sample(n, 6, 1000, 10, 500, rows, 8)
    off = np.arange(n)[None, :] != rows[:, None]
    assert np.array_equal(np.where(off, glat, 0), np.where(off, clat, 0))
    err = np.abs(grel - crel) / np.maximum(crel, 1e-300)
    assert float(err[off].max()) <= REL_TOL


@pytest.mark.parametrize("ranks", [2, 3])
@pytest.mark.parametrize("kind", ["complete", "ties"])
def test_levels_virtual_ranks(gpu, monkeypatch, ranks, kind):
    """Row-sharded level builds: every rank extracts the in-arcs of its rows, broadcasts its
    segment, settles its own sources, and all ranks agree on the verdict (ld = 1,024: at 3 ranks
    the row blocks are 384 | 256 | 384)."""
    set_form(monkeypatch, levels="1")
    monkeypatch.setenv("SRT_VIRTUAL_RANKS", str(ranks))
    g = graphs.complete_graph(1000, seed=2) if kind == "complete" else \
        graphs.complete_graph(900, seed=4, lat_max=4)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_DENSE_FW, ngpus=1)
    assert st.dist_enc == LEVELS, st.dist_enc
    _check(g, lat, rel, f"virtual x{ranks} {kind}")


def test_levels_sub_ms_path_order(gpu, monkeypatch):
    """A level build with 0.1-0.3 ms edges (quantum 100 us): the f64 ms table is summed in path
    order along the level pass's predecessors (int16 rows, widened for the ms pass), bit for bit
    the reference's (double)ns / 1e6 hop sums."""
    from shadow_amd.topology import build_tables_subset
    set_form(monkeypatch, levels="1")
    rng = np.random.default_rng(42)
    g0 = graphs.complete_graph(300, seed=3)
    lat = rng.integers(1, 4, g0.m).astype(np.int64) * 100_000
    g = graphs.Graph(g0.n, False, g0.src, g0.dst, lat, g0.loss)
    full = oracle.table(oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss), True,
                        oracle.ORC_INT_NS, 8, raw=True)
    lat_t, rel, ms, _, st = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                                algo=ALGO_DENSE_FW, want_ms=True)
    assert st.dist_enc == LEVELS, st.dist_enc
    assert np.array_equal(lat_t, full["lat_int"])
    assert np.array_equal(rel, full["rel"])
    assert np.array_equal(ms, full["lat_ms"]), np.argwhere(ms != full["lat_ms"])[:5]


def _virtual_dense(L, n, ld, ranks, seed, lat_max=1000):
    """srt_dense_build_sharded on `ranks` virtual ranks of device 0 (row blocks generated on the
    device); returns {row: (lat_ns, rel)} for every row and each rank's stats."""
    import threading
    import torch
    comms = (ctypes.c_void_p * ranks)()
    _lib.check(L.srt_comm_init_virtual(ranks, 0, comms), "srt_comm_init_virtual")
    shards, bufs, streams = [], [], []
    try:
        for r in range(ranks):
            b, e = ctypes.c_int32(), ctypes.c_int32()
            L.srt_shard_rows(ld, 128, ranks, r, ctypes.byref(b), ctypes.byref(e))
            b, e = b.value, e.value
            w = torch.empty((e - b, ld), dtype=torch.int32, device="cuda")
            rr = torch.empty((e - b, ld), dtype=torch.float64, device="cuda")
            st = torch.cuda.Stream()
            _lib.check(L.srt_gen_complete_device(n, ld, b, e - b, seed, lat_max, 10, 500,
                                                 w.data_ptr(), rr.data_ptr(),
                                                 ctypes.c_void_p(st.cuda_stream)), "generate")
            shards.append((b, e))
            bufs.append((w, rr, torch.empty_like(w), torch.empty_like(rr)))
            streams.append(st)
        torch.cuda.synchronize()
        rcs = [None] * ranks
        stats = [_lib.BuildStats() for _ in range(ranks)]

        def work(r):
            L.srt_virtual_rank_bind(r, 0)
            w, rr, lat, rel = bufs[r]
            rcs[r] = L.srt_dense_build_sharded(ctypes.c_void_p(comms[r]), n, ld, 0, w.data_ptr(),
                                               rr.data_ptr(), lat.data_ptr(), rel.data_ptr(),
                                               ctypes.c_void_p(streams[r].cuda_stream), 0,
                                               ctypes.byref(stats[r]))
            L.srt_virtual_rank_bind(-1, 0)

        th = [threading.Thread(target=work, args=(r,)) for r in range(ranks)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        for r in range(ranks):
            _lib.check(rcs[r], f"rank {r}")
        lat = np.concatenate([bufs[r][2].cpu().numpy() for r in range(ranks)])[:n, :n]
        rel = np.concatenate([bufs[r][3].cpu().numpy() for r in range(ranks)])[:n, :n]
    finally:
        for r in range(ranks):
            L.srt_comm_free(ctypes.c_void_p(comms[r]))
    return lat.view(np.uint32).astype(np.uint64) * np.uint64(MS), rel, stats, shards


def test_levels_uneven_shards_default_budget(gpu, monkeypatch):
    """three virtual ranks with uneven row blocks (ld 4,096 = 32 tiles: 1,280 |
    1,408 | 1,408 rows) and the default, unforced level budget. The budget is taken from global
    quantities and agreed by a min all-reduce, so every rank takes the same path (no rank leaves for
    Floyd-Warshall while its peers wait in a broadcast); every row against the oracle."""
    monkeypatch.delenv("SRT_FORM", raising=False)
    L = _lib.lib()
    n = ld = 4096
    glat, grel, stats, shards = _virtual_dense(L, n, ld, 3, seed=12)
    assert len({e - b for b, e in shards}) > 1, shards
    assert {int(s.dist_enc) for s in stats} == {LEVELS}, [int(s.dist_enc) for s in stats]
    # one verdict for all ranks; each rank's own sources settle at their own last level
    assert all(int(s.levels) >= 1 for s in stats), [int(s.levels) for s in stats]
    rows = np.array([0, 1, 1279, 1280, 2000, 2687, 2688, 4095], np.int32)
    clat, crel, _, _ = oracle.complete_sample(n, 12, 1000, 10, 500, rows, 8)
    off = np.arange(n)[None, :] != rows[:, None]
    assert np.array_equal(np.where(off, glat[rows], 0), np.where(off, clat, 0))
    err = np.abs(grel[rows] - crel) / np.maximum(crel, 1e-300)
    assert float(err[off].max()) <= REL_TOL


def test_levels_memory_cap_falls_back(gpu, monkeypatch):
    """the level planes are capped by the memory the device has left
    (srt_levels_build: half of free + the scratch pool's unused bytes). SRT_FORM memcap (MiB, a
    test hook) stands in for a nearly full device: the budget drops below two levels and the build
    falls back to Floyd-Warshall instead of failing an allocation; the tables stay exact."""
    set_form(monkeypatch, levels="1", memcap="0")
    g = graphs.complete_graph(1000, seed=2)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_DENSE_FW)
    assert st.dist_enc != LEVELS and st.levels == 0, (st.dist_enc, st.levels)
    _check(g, lat, rel, "memory-capped")
    set_form(monkeypatch, levels="1", memcap="1")  # 1 MiB: 0.5 MiB of 128-KiB planes -> 4 levels
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_DENSE_FW)
    assert st.levels <= 4, st.levels
    _check(g, lat, rel, "memory-capped 1 MiB")
