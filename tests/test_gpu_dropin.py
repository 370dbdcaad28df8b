"""The drop-in path end to end on an MI355X (-m gpu): the reference's entry points and build
order, against the CPU oracle.

* AUTO dispatch: large sparse graphs (C3 20k RGG, C5 100k BA) build through srt_build_tables /
  srt_build_tables_multi / srt_build_tables_subset with SRT_ALGO_AUTO on the SSSP kernels
  (the reference computes any size lazily, topology.c:1578-1814); dense requests beyond the dense
  limit fail before any work.
* Tables over the attached vertices only (topology.c:1604-1656): sub-tables equal the oracle's
  full table restricted to the subset, for dense / sparse / directed graphs and virtual ranks.
* f64 path-order milliseconds (topology.c:1308, :1364): sub-millisecond edges give the
  reference's latency and worker.c:551's ceil(ms * 1e6) delay exactly.
* Runahead export (topology.c:1253-1264): worker_updateMinTimeJump receives each smaller path
  latency as the lookups' source runs store paths (the eager build stores none), in both build
  orders and after later attaches.
* The reference-signature entry points (topology_attach / getLatency / getReliability /
  isRoutable / incrementPathPacketCounter / detach) with Address and Random laid out as
  address.c:23-25 and random.c:15-18.
"""
import ctypes

import numpy as np
import pytest

import oracle
from shadow_amd import graphs
from shadow_amd._lib import ALGO_AUTO, ALGO_DENSE_FW, ALGO_SPARSE_SSSP, lib
from shadow_amd.topology import (Topology, build_tables, build_tables_subset, ip_to_net,
                                 set_min_time_jump_hook)

pytestmark = pytest.mark.gpu
REL_TOL = 1e-12
MS = 1_000_000


def _el(g):
    return oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)


def _check_sampled_rows(lat, rel, g, rows, what):
    """Full-table rows vs the oracle's raw rows off the diagonal (every row is its own
    source's)."""
    exp = oracle.sssp_list(_el(g), rows, nthreads=16)
    for i, s in enumerate(rows):
        off = np.arange(g.n) != s
        assert np.array_equal(lat[s][off], exp["lat_int"][i][off]), (what, s)
        err = np.abs(rel[s][off] - exp["rel"][i][off]) / np.maximum(exp["rel"][i][off], 1e-300)
        assert float(err.max() if err.size else 0.0) <= REL_TOL, (what, s)


def _expected_sub(g, verts, nthreads=16):
    """The oracle's raw rows of the subset's sources restricted to the subset:
    [i][j] = row(verts[i])[verts[j]]. The diagonal is left out (0)."""
    rows = oracle.sssp_list(_el(g), verts, nthreads=nthreads)
    lat = rows["lat_int"][:, verts].copy()
    rel = rows["rel"][:, verts].copy()
    np.fill_diagonal(lat, 0)
    np.fill_diagonal(rel, 0.0)
    return lat, rel


def test_auto_dispatch_c3_rgg_20000_full_table(gpu):
    """C3 through srt_build_tables (AUTO) and srt_build_tables_multi(ngpus=1): the multi-source
    SSSP (msssp.hip)."""
    g = graphs.random_geometric(20000, seed=3)
    rows = np.r_[0:8, 9_996:10_004, 19_992:20_000, np.linspace(8, 19_990, 24).astype(int)]
    lat, rel, st = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss, algo=ALGO_AUTO)
    assert st.algo == ALGO_SPARSE_SSSP and st.dist_enc == 3
    _check_sampled_rows(lat, rel, g, rows, "C3 AUTO")
    assert np.array_equal(lat, lat.T)
    off = ~np.eye(g.n, dtype=bool)
    print(f"C3 pairs whose rel(s->t) != rel(t->s) bitwise: {int((rel != rel.T)[off].sum()) // 2}")
    lat2, rel2, st2 = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss, algo=ALGO_AUTO,
                                   ngpus=1)
    assert st2.algo == ALGO_SPARSE_SSSP
    assert np.array_equal(lat, lat2) and np.array_equal(rel, rel2)


def test_auto_dispatch_c5_ba_100000_attached_subset(gpu):
    """C5 (n = 100,000 > the old 20,132 cut-off) through srt_build_tables_subset with AUTO:
    the workgroup SSSP over the attached vertices' rows, gathered to the sub-table."""
    g = graphs.barabasi_albert(100_000, seed=5)
    rng = np.random.default_rng(55)
    verts = np.unique(np.concatenate([rng.choice(g.n, 300, replace=False), [0, 1, 99_999]]))
    verts = verts.astype(np.int32)
    lat, rel, ms, mn, st = build_tables_subset(g.n, False, g.src, g.dst, g.lat_ns, g.loss,
                                               verts=verts, algo=ALGO_AUTO)
    assert st.algo == ALGO_SPARSE_SSSP and st.dist_enc == 2, "C5 takes the workgroup kernel"
    assert ms is None
    elat, erel = _expected_sub(g, verts)
    off = ~np.eye(len(verts), dtype=bool)
    assert np.array_equal(lat[off], elat[off])
    err = np.abs(rel[off] - erel[off]) / np.maximum(erel[off], 1e-300)
    assert float(err.max()) <= REL_TOL
    assert mn == int(lat.min())
    # the same subset on two virtual ranks (source shards + all-gather of the sub-table)
    import os
    os.environ["SRT_VIRTUAL_RANKS"] = "2"
    try:
        lat2, rel2, _, mn2, _ = build_tables_subset(g.n, False, g.src, g.dst, g.lat_ns, g.loss,
                                                    verts=verts, algo=ALGO_AUTO, ngpus=2)
    finally:
        del os.environ["SRT_VIRTUAL_RANKS"]
    assert np.array_equal(lat, lat2) and np.array_equal(rel, rel2) and mn == mn2


def test_dense_request_beyond_limit_fails_before_work(gpu):
    n = lib().srt_dense_max_n() + 1
    assert lib().srt_dense_max_n() >= 32768
    # a path graph: the request is refused on size alone, before any allocation of n^2 matrices
    src = np.arange(n - 1, dtype=np.int32)
    dst = src + 1
    lat = np.full(n - 1, MS, np.int64)
    loss = np.zeros(n - 1)
    with pytest.raises(RuntimeError, match="SRT_E_RANGE"):
        build_tables_subset(n, False, src, dst, lat, loss, verts=np.array([0, 1], np.int32),
                            algo=ALGO_DENSE_FW)
    # AUTO on the same graph takes the SSSP
    l2, r2, _, _, st = build_tables_subset(n, False, src, dst, lat, loss,
                                           verts=np.array([0, 5, n - 1], np.int32), algo=ALGO_AUTO)
    assert st.algo == ALGO_SPARSE_SSSP
    assert int(l2[0, 2]) == (n - 1) * MS and int(l2[1, 2]) == (n - 6) * MS


def _directed_graph(seed=12, n=400, m=3000, sub_ms=False):
    rng = np.random.default_rng(seed)
    ring = np.arange(n)
    src = np.concatenate([rng.integers(0, n, m), ring, ring]).astype(np.int32)
    dst = np.concatenate([rng.integers(0, n, m), (ring + 1) % n, ring]).astype(np.int32)
    unit = 1_000 if sub_ms else MS
    lat = (rng.integers(1, 20, len(src)) * unit).astype(np.int64)
    loss = rng.integers(0, 300, len(src)) / 10000.0
    return graphs.Graph(n, True, src, dst, lat, loss)


@pytest.mark.parametrize("which,algo", [("complete300", ALGO_DENSE_FW),
                                        ("complete300", ALGO_SPARSE_SSSP),
                                        ("rgg2000", ALGO_SPARSE_SSSP),
                                        ("rgg2000", ALGO_DENSE_FW),
                                        ("directed", ALGO_DENSE_FW),
                                        ("directed", ALGO_SPARSE_SSSP)])
def test_subset_tables_equal_restricted_full_table(gpu, which, algo):
    g = {"complete300": lambda: graphs.complete_graph(300, seed=21),
         "rgg2000": lambda: graphs.random_geometric(2000, seed=3),
         "directed": _directed_graph}[which]()
    full = oracle.table(_el(g), True, oracle.ORC_INT_NS, 8, raw=True)
    rng = np.random.default_rng(3)
    verts = np.sort(rng.choice(g.n, min(g.n, 77), replace=False)).astype(np.int32)
    lat, rel, ms, mn, st = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                               verts=verts, algo=algo)
    ix = np.ix_(verts, verts)
    assert np.array_equal(lat, full["lat_int"][ix]), which
    assert np.array_equal(rel, full["rel"][ix]), which
    assert mn == int(full["lat_int"][ix].min())
    for ngpus in (2, 3):
        import os
        os.environ["SRT_VIRTUAL_RANKS"] = str(ngpus)
        try:
            l2, r2, _, m2, _ = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                                   verts=verts, algo=algo, ngpus=ngpus)
        finally:
            del os.environ["SRT_VIRTUAL_RANKS"]
        assert np.array_equal(l2, lat) and np.array_equal(r2, rel) and m2 == mn, (which, ngpus)


def _sub_ms_graph(kind):
    """Edge latencies in whole microseconds (quantum 1 us): f64 ms sums in path order differ from
    the exact integer sums (0.1 + 0.2 ms)."""
    if kind == "directed":
        return _directed_graph(seed=31, sub_ms=True)
    rng = np.random.default_rng(77)
    if kind == "complete":
        g = graphs.complete_graph(120, seed=8)
        lat = rng.integers(1, 900, g.m).astype(np.int64) * 1_000  # 1..899 us
        return graphs.Graph(g.n, False, g.src, g.dst, lat, g.loss)
    g = graphs.random_geometric(1500, seed=4)
    lat = rng.integers(50, 3000, g.m).astype(np.int64) * 1_000 + 100  # sub-ms parts, q = 100 ns
    return graphs.Graph(g.n, False, g.src, g.dst, lat, g.loss)


@pytest.mark.parametrize("kind,algo", [("complete", ALGO_DENSE_FW), ("complete", ALGO_SPARSE_SSSP),
                                       ("rgg", ALGO_SPARSE_SSSP), ("rgg", ALGO_DENSE_FW),
                                       ("directed", ALGO_DENSE_FW),
                                       ("directed", ALGO_SPARSE_SSSP)])
def test_f64_ms_path_order_latency(gpu, kind, algo):
    g = _sub_ms_graph(kind)
    full = oracle.table(_el(g), True, oracle.ORC_INT_NS, 8, raw=True)
    lat, rel, ms, _, st = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                              algo=algo, want_ms=True)
    assert np.array_equal(lat, full["lat_int"])
    assert np.array_equal(rel, full["rel"])
    # bit-exact f64: the same hops added in the same order from 0.0
    assert np.array_equal(ms, full["lat_ms"]), np.argwhere(ms != full["lat_ms"])[:5]
    delay = np.ceil(ms * 1e6).astype(np.uint64)
    assert np.array_equal(delay, full["lat_ref"])
    assert (full["lat_ref"] != full["lat_int"]).any(), "the graph should exercise the f64 rounding"
    # subset + virtual ranks carry the ms table too
    verts = np.arange(0, g.n, 7, dtype=np.int32)
    import os
    os.environ["SRT_VIRTUAL_RANKS"] = "2"
    try:
        _, _, ms2, _, _ = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                              verts=verts, algo=algo, ngpus=2, want_ms=True)
    finally:
        del os.environ["SRT_VIRTUAL_RANKS"]
    assert np.array_equal(ms2, full["lat_ms"][np.ix_(verts, verts)])


def test_sub_ms_latency_through_topology_and_packet_path(gpu):
    """GML with microsecond latencies -> getLatency == the reference's f64 ms sum along the serving
    source's path, and the packet delay == ceil(ms * 1e6) (worker.c:551), on every looked-up pair
    (lazy-cache order, oracle/lazy_cache.py)."""
    from oracle.lazy_cache import LazyPathCache
    g = _sub_ms_graph("complete")
    top = Topology.from_gml(graphs.to_gml(g))
    full = oracle.table(_el(g), True, oracle.ORC_INT_NS, 8, raw=True)
    sim = LazyPathCache(full, directed=False)
    ips = [f"100.1.{v}.1" for v in range(g.n)]
    hosts = list(range(0, g.n, 3))
    for v in hosts:
        vert, _, _, _ = top.attach(ips[v], 1, ip_hint=f"11.0.0.{v + 1}")
        assert vert == v
        sim.attach(ips[v], v)
    top.compute_shortest_paths()
    verts, ms = top.table_vertices()
    assert np.array_equal(verts, np.array(hosts)) and ms is not None
    for s in hosts[::4]:
        for d in hosts[::3][::-1]:
            assert top.get_latency(ips[s], ips[d]) == sim.get_latency(ips[s], ips[d])
            ok, delay = top.send_packet(ips[s], ips[d], 0.0)
            assert (ok, delay) == sim.send_packet(ips[s], ips[d], 0.0)


def test_runahead_export_documented_order(gpu):
    """Attach first, then build (controller.c:367 before the eager build): the build stores no
    path, so nothing is exported; each lookup that runs a source hands over the smallest latency
    it stored when that is below the minimum so far (topology.c:1253-1264), as the reference's
    lazy cache does (oracle/lazy_cache.py). A later attach of a new vertex changes nothing until
    a run stores its pairs."""
    from oracle.lazy_cache import LazyPathCache
    calls = []
    cb = set_min_time_jump_hook(lambda ms: calls.append(ms))
    try:
        g = graphs.complete_graph(60, seed=13)
        top = Topology.from_gml(graphs.to_gml(g))
        full = oracle.table(_el(g), True, oracle.ORC_INT_NS, 8, raw=True)
        sim = LazyPathCache(full, directed=False)
        ips = [f"100.2.{v}.1" for v in range(g.n)]
        first = [3, 7, 11, 20, 41]
        for v in first:
            top.attach(ips[v], 1, ip_hint=f"11.0.0.{v + 1}")
            sim.attach(ips[v], v)
        top.compute_shortest_paths()
        verts, _ = top.table_vertices()
        assert list(verts) == first  # tables over the attached vertices only
        assert calls == []
        assert top.get_latency(ips[3], ips[41]) == sim.get_latency(ips[3], ips[41])
        m1 = min(full["lat_ms"][3, t] for t in first if t != 3)
        assert calls == [m1] and sim.minimum_path_latency == m1
        top.compute_shortest_paths()
        assert calls == [m1]  # nothing new stored
        for s, d in ((41, 3), (7, 7), (20, 11), (11, 7)):
            top.get_reliability(ips[s], ips[d])
            sim.get_reliability(ips[s], ips[d])
            assert calls[-1] == sim.minimum_path_latency
        # a host on a new vertex: the next lookup rebuilds over the grown set
        v_new = int(np.argmin(np.diag(full["lat_int"])))
        if v_new in first:
            v_new = 0
        top.attach(ips[v_new], 1, ip_hint=f"11.0.0.{v_new + 1}")
        sim.attach(ips[v_new], v_new)
        before = list(calls)
        assert top.get_latency(ips[v_new], ips[3]) == sim.get_latency(ips[v_new], ips[3])
        verts, _ = top.table_vertices()
        assert list(verts) == sorted(first + [v_new])
        assert (calls[-1] if calls else 0.0) == sim.minimum_path_latency
        assert calls[:len(before)] == before and all(x > y for x, y in zip(calls, calls[1:]))
        top.free()
    finally:
        set_min_time_jump_hook(None)
        del cb


def test_runahead_export_build_before_attach(gpu):
    """Eager build before any attach (tables over every vertex): nothing exported until a lookup
    runs a source; then the minimum over the paths it stored (the self path on its own lookup)."""
    calls = []
    cb = set_min_time_jump_hook(lambda ms: calls.append(ms))
    try:
        g = graphs.complete_graph(50, seed=14)
        top = Topology.from_gml(graphs.to_gml(g))
        full = oracle.table(_el(g), True, oracle.ORC_INT_NS, 8, raw=True)
        top.compute_shortest_paths()
        assert calls == []
        ips = [f"100.3.{v}.1" for v in range(g.n)]
        att = [2, 9, 30]
        for v in att:
            top.attach(ips[v], 1, ip_hint=f"11.0.0.{v + 1}")
        top.get_reliability(ips[2], ips[30])
        assert calls == [min(full["lat_ms"][2, 9], full["lat_ms"][2, 30])]
        top.get_latency(ips[9], ips[9])  # the self path of 9 is stored on its own lookup
        if full["lat_ms"][9, 9] < calls[0]:
            assert calls[-1] == full["lat_ms"][9, 9]
        verts, _ = top.table_vertices()
        assert len(verts) == g.n  # the full table covers the attached set: no rebuild
        top.free()
    finally:
        set_min_time_jump_hook(None)
        del cb


class Address(ctypes.Structure):
    """struct _Address (address.c:23-47): the network-order IP first."""
    _fields_ = [("ip", ctypes.c_uint32), ("mac", ctypes.c_uint32), ("ipString", ctypes.c_char_p),
                ("name", ctypes.c_char_p), ("idString", ctypes.c_char_p),
                ("referenceCount", ctypes.c_int), ("isLocal", ctypes.c_int),
                ("hostID", ctypes.c_uint32), ("magic", ctypes.c_uint32)]


class Random(ctypes.Structure):
    """struct _Random (random.c:15-18), advanced by rand_r(&seedState)."""
    _fields_ = [("seedState", ctypes.c_uint), ("initialSeed", ctypes.c_uint)]


def test_reference_signature_entry_points(gpu):
    """topology_attach/getLatency/getReliability/isRoutable/incrementPathPacketCounter/detach with
    the reference's struct layouts give what the _ip variants give on a twin topology."""
    g = graphs.random_geometric(300, seed=9)
    gml = graphs.to_gml(g, ip_base=None)  # no vertex IPs: every attach is a random pick
    a = Topology.from_gml(gml)
    b = Topology.from_gml(gml)
    L = lib()
    rnd = Random(12345, 12345)
    state = 12345
    addrs = []
    for h in range(40):
        ip = f"100.4.{h}.1"
        ad = Address(ip_to_net(ip), h, ip.encode(), b"h", b"h", 1, 0, h, 0)
        addrs.append(ad)
        down, up = ctypes.c_uint64(), ctypes.c_uint64()
        L.topology_attach(a._h, ctypes.byref(ad), ctypes.byref(rnd), None, None, None,
                          ctypes.byref(down), ctypes.byref(up))
        vb, db, ub, state = b.attach(ip, state)
        assert a.vertex_of(ip) == vb and (down.value, up.value) == (db, ub)
        assert rnd.seedState == state  # rand_r advanced the same stream
    for i in range(0, 40, 3):
        for j in range(0, 40, 7):
            pa, pb = ctypes.byref(addrs[i]), ctypes.byref(addrs[j])
            ia, ib = f"100.4.{i}.1", f"100.4.{j}.1"
            assert L.topology_getLatency(a._h, pa, pb) == b.get_latency(ia, ib)
            assert L.topology_getReliability(a._h, pa, pb) == b.get_reliability(ia, ib)
            assert L.topology_isRoutable(a._h, pa, pb) == 1
            L.topology_incrementPathPacketCounter(a._h, pa, pb)
            b.increment_path_packet_counter(ia, ib)
            assert a.packet_count(ia, ib) == b.packet_count(ia, ib)
    L.topology_detach(a._h, ctypes.byref(addrs[5]))
    assert L.topology_getLatency(a._h, ctypes.byref(addrs[5]), ctypes.byref(addrs[6])) == -1.0
    assert L.topology_isRoutable(a._h, ctypes.byref(addrs[5]), ctypes.byref(addrs[6])) == 0
    a.free()
    b.free()


def _both_orientations(g, seed):
    """Directed variant: each undirected edge becomes two directed edges with independent
    latencies (1..100,000 us) and losses; self-loops kept."""
    rng = np.random.default_rng(seed)
    off = g.src != g.dst
    src = np.concatenate([g.src[off], g.dst[off], g.src[~off]]).astype(np.int32)
    dst = np.concatenate([g.dst[off], g.src[off], g.dst[~off]]).astype(np.int32)
    lat = np.concatenate([rng.integers(1, 100_001, 2 * int(off.sum())) * 1_000,
                          g.lat_ns[~off]]).astype(np.int64)
    loss = np.concatenate([rng.integers(0, 101, 2 * int(off.sum())) / 10000.0, g.loss[~off]])
    return graphs.Graph(g.n, True, src, dst, lat, loss)


@pytest.mark.parametrize("directed", [False, True])
def test_fine_quantum_range_lifted(gpu, directed):
    """a 100k power-law graph with 1..100,000 us latencies (quantum 1 us, so the
    MST / (n - 1) * max_w bounds reach ~1e9-1e10 quanta) builds through AUTO: the hop bound
    through the hub (graph.c) keeps every distance provably inside the u32 tables. Rows of 64
    attached sources against the oracle."""
    g = graphs.barabasi_albert(100_000, seed=15)
    rng = np.random.default_rng(16)
    if directed:
        g = _both_orientations(g, 17)
    else:
        off = g.src != g.dst
        lat = g.lat_ns.copy()
        lat[off] = rng.integers(1, 100_001, int(off.sum())) * 1_000
        g = graphs.Graph(g.n, False, g.src, g.dst, lat, g.loss)
    q = ctypes.c_uint64()
    mw = ctypes.c_uint32()
    e = _lib_edges(g)
    assert lib().srt_latency_quantum(ctypes.byref(e[0]), ctypes.byref(q), ctypes.byref(mw)) == 0
    assert q.value == 1_000 and mw.value >= 99_000
    verts = np.unique(np.concatenate([rng.choice(g.n, 62, replace=False), [0, g.n - 1]]))
    verts = verts.astype(np.int32)
    lat, rel, ms, mn, st = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                               verts=verts, algo=ALGO_AUTO, want_ms=True)
    assert st.algo == ALGO_SPARSE_SSSP and ms is not None
    rows = oracle.sssp_list(_el(g), verts, nthreads=16)
    ix = np.ix_(np.arange(len(verts)), verts)
    off = ~np.eye(len(verts), dtype=bool)
    assert np.array_equal(lat[off], rows["lat_int"][ix][off])
    assert np.array_equal(rel[off], rows["rel"][ix][off])
    assert np.array_equal(ms[off], rows["lat_ms"][ix][off])  # f64 path-order ms (q = 1 us)
    # the undirected MST bound here is ~2.15e9 quanta and the directed (n - 1) * max_w ~1e10,
    # both past the u32 range; real distances reach ~2e5 quanta
    assert int(lat[off].max()) // 1_000 > 100_000


def _lib_edges(g):
    from shadow_amd._lib import Edges
    arrs = (np.ascontiguousarray(g.src, np.int32), np.ascontiguousarray(g.dst, np.int32),
            np.ascontiguousarray(g.lat_ns, np.int64), np.ascontiguousarray(g.loss, np.float64))
    e = Edges(g.n, int(g.directed), len(g.src), *(a.ctypes.data for a in arrs))
    return e, arrs


@pytest.mark.parametrize("kind", ["complete", "directed", "sub_ms"])
def test_dense_rows_few_attached(gpu, kind):
    """a dense graph with few attached vertices (<= n / 12) builds their rows by
    Bellman-Ford passes (srt_dense_rows_build_device, encoding 10) instead of the all-pairs FW;
    the sub-table equals the oracle's raw rows, the f64 ms table included."""
    if kind == "complete":
        g = graphs.complete_graph(600, seed=31)
    elif kind == "directed":
        g = graphs.complete_directed(480, seed=32)
    else:
        g = graphs.complete_graph(360, seed=33)
        rng = np.random.default_rng(34)
        g = graphs.Graph(g.n, False, g.src, g.dst, rng.integers(1, 900, g.m).astype(np.int64) * 1_000,
                         g.loss)
    rng = np.random.default_rng(35)
    verts = np.sort(rng.choice(g.n, g.n // 12, replace=False)).astype(np.int32)
    lat, rel, ms, mn, st = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                               verts=verts, algo=ALGO_AUTO, want_ms=kind == "sub_ms")
    assert st.dist_enc == 10, st.dist_enc
    rows = oracle.sssp_list(_el(g), verts, nthreads=16)
    ix = np.ix_(np.arange(len(verts)), verts)
    off = ~np.eye(len(verts), dtype=bool)
    assert np.array_equal(lat[off], rows["lat_int"][ix][off])
    assert np.array_equal(rel[off], rows["rel"][ix][off])
    full = oracle.table(_el(g), True, oracle.ORC_INT_NS, 8, raw=True)
    sub = np.ix_(verts, verts)
    assert np.array_equal(lat, full["lat_int"][sub]) and np.array_equal(rel, full["rel"][sub])
    if kind == "sub_ms":
        assert np.array_equal(ms, full["lat_ms"][sub])
    # the all-pairs build of the same graph (every vertex attached: no rows path) agrees on the
    # attached vertices' sub-table
    lat2, rel2, _, _, st2 = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                                verts=None, algo=ALGO_AUTO)
    assert st2.dist_enc != 10
    assert np.array_equal(lat, lat2[sub]) and np.array_equal(rel, rel2[sub])


def test_dense_rows_c4_50_attached(gpu):
    """C4 (n = 32,768 complete graph) with 50 attached vertices: their rows without the FW
    (<= 20 ms against the 322-ms all-pairs build), checked against the oracle's
    dense Dijkstra on every row."""
    import torch
    from shadow_amd._lib import BuildStats, check
    n = ld = 32768
    L = lib()
    w = torch.empty((ld, ld), dtype=torch.int32, device="cuda")
    r = torch.empty((ld, ld), dtype=torch.float64, device="cuda")
    check(L.srt_gen_complete_device(n, ld, 0, ld, 4, 1000, 10, 500, w.data_ptr(), r.data_ptr(),
                                    None), "generate")
    rng = np.random.default_rng(50)
    verts = np.sort(rng.choice(n, 50, replace=False)).astype(np.int32)
    dv = torch.from_numpy(verts).cuda()
    lat = torch.empty((50, ld), dtype=torch.int32, device="cuda")
    rel = torch.empty((50, ld), dtype=torch.float64, device="cuda")
    times = []
    for _ in range(3):
        st = BuildStats()
        st.count_ties = 0
        torch.cuda.synchronize()
        check(L.srt_dense_rows_build(n, ld, 50, dv.data_ptr(), w.data_ptr(), r.data_ptr(),
                                     lat.data_ptr(), rel.data_ptr(), None, ctypes.byref(st)),
              "rows build")
        torch.cuda.synchronize()
        times.append(st.ms_total)
    print(f"C4 rows of 50 attached vertices: {min(times):.2f} ms (distances {st.ms_fw:.2f} ms in "
          f"{st.n_update} passes, post {st.ms_post:.2f} ms)")
    glat = lat.cpu().numpy().view(np.uint32).astype(np.uint64) * np.uint64(1_000_000)
    grel = rel.cpu().numpy()
    del w, r
    clat, crel, _, _ = oracle.complete_sample(n, 4, 1000, 10, 500, verts, 16)
    offd = np.arange(n)[None, :] != verts[:, None]
    assert np.array_equal(np.where(offd, glat, 0), np.where(offd, clat, 0))
    assert np.array_equal(grel[offd], crel[offd])
