"""The lookup layer end to end on an MI355X (-m gpu): random lookup and packet traces through the
topology API give, per call and bit for bit, what the reference's lazy path cache gives
(oracle/lazy_cache.py, a restatement of topology.c:1166-1265, :1900-2022 and worker.c:541-555
over the oracle's raw per-source rows).

What the trace exercises (VERDICT r02 "what's missing" #1):
* the first source run for a pair serves it in both directions, with that source's own latency
  and reliability -- on an undirected graph the two directions' reliabilities differ bitwise on
  ~29% of C1's pairs (reversed products and ties), on a directed graph the latency itself differs;
* directed lookups still run their own source (topology.c:1919) and fall back to the reverse
  path (:1963-1967);
* packet counters per cached Path (:1983-1993), read back per pair at the end;
* the runahead minimum handed to worker_updateMinTimeJump as runs store paths (:1253-1264);
* attaches between lookups (the new vertex's pairs go to whichever end runs next), hosts sharing
  a vertex, unattached addresses (-1), direct mode (use_shortest_path = false), sub-ms latencies
  (the f64 path-order ms table) and the sparse build forced on a small graph.
"""
import numpy as np
import pytest

import oracle
from conftest import GOLDEN
from oracle.lazy_cache import LazyPathCache
from shadow_amd import graphs
from shadow_amd._lib import ALGO_AUTO, ALGO_DENSE_FW, ALGO_SPARSE_SSSP
from shadow_amd.topology import Topology, set_min_time_jump_hook

pytestmark = pytest.mark.gpu


def _ip_of_vertex(v):
    ip = 0x0B000001 + v  # graphs.to_gml's default ip_base
    return f"{ip >> 24 & 255}.{ip >> 16 & 255}.{ip >> 8 & 255}.{ip & 255}"


def _replay(g, gml, use_sp=True, algo=ALGO_AUTO, ops=2500, hosts=None, late=0, seed=0,
            ms_exact=True):
    """Run the same random trace through the product and the restatement; returns stats."""
    calls = []
    cb = set_min_time_jump_hook(lambda ms: calls.append(ms))
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    raw = oracle.table(el, use_sp, oracle.ORC_INT_NS, nthreads=8, raw=True)
    sim = LazyPathCache(raw, g.directed, use_sp)
    top = Topology.from_gml(gml, use_shortest_path=use_sp)
    top.set_build_opts(algo=algo)
    rng = np.random.default_rng(seed)
    try:
        nh = hosts or min(3 * g.n // 2, 400)
        host_v = [int(v) for v in rng.integers(0, g.n, nh)]
        host_ip = [f"100.{h // 200}.{h % 200}.9" for h in range(nh)]
        attached = []

        def attach(h):
            v, _, _, _ = top.attach(host_ip[h], 1, ip_hint=_ip_of_vertex(host_v[h]))
            assert v == host_v[h]
            sim.attach(host_ip[h], v)
            attached.append(h)

        for h in range(nh - late):
            attach(h)
        stats = {"runs": 0, "reverse_served": 0, "differs": 0}
        for k in range(ops):
            if len(attached) < nh and rng.random() < late / ops * 2:
                attach(len(attached))
                continue
            a = host_ip[attached[int(rng.integers(len(attached)))]]
            b = host_ip[attached[int(rng.integers(len(attached)))]]
            if rng.random() < 0.01:
                b = "9.9.9.9"  # never attached: -1 from both
            op = int(rng.integers(5))
            if op == 0:
                got, want = top.get_latency(a, b), sim.get_latency(a, b)
                if ms_exact:
                    assert got == want, (k, a, b, got, want)
                else:
                    assert got == want or np.isclose(got, want, rtol=1e-15, atol=0), (k, got, want)
            elif op == 1:
                got, want = top.get_reliability(a, b), sim.get_reliability(a, b)
                assert got == want, (k, a, b, got, want)
            elif op == 2:
                assert top.is_routable(a, b) == sim.is_routable(a, b)
            elif op == 3 and b != "9.9.9.9":
                top.increment_path_packet_counter(a, b)
                sim.increment(a, b)
            elif b != "9.9.9.9":
                chance = float(rng.random())
                boot = bool(rng.random() < 0.05)
                payload = 0 if rng.random() < 0.1 else 1400
                got = top.send_packet(a, b, chance, boot, payload)
                want = sim.send_packet(a, b, chance, boot, payload)
                assert got[0] == want[0], (k, got, want)
                if got[0]:
                    assert got[1] == want[1], (k, got, want)
            # the controller's minimum after every call (one offer per run vs one per path)
            assert (calls[-1] if calls else 0.0) == sim.minimum_path_latency, k
        # every pair of attached hosts: the serving path's source and its packet count
        vs = sorted({host_v[h] for h in attached})
        ip_of = {host_v[h]: host_ip[h] for h in attached}
        for x in vs:
            for y in vs:
                p = sim._get(x, y) or sim._get(y, x)
                assert top.path_source(ip_of[x], ip_of[y]) == (-1 if p is None else p.src), (x, y)
                assert top.packet_count(ip_of[x], ip_of[y]) == (0 if p is None else p.packets)
                if p is not None and x != y:
                    stats["reverse_served"] += int(p.src == y)
                    stats["differs"] += int(raw["rel"][x, y] != raw["rel"][y, x] or
                                            raw["lat_ms"][x, y] != raw["lat_ms"][y, x])
        stats["runs"] = sim.source_runs
        # the reference's diagnostics (topology.c:78-79): Dijkstra runs and self paths
        pc = top.path_counts()
        want = (sim.source_runs, sim.self_runs) if use_sp else (0, 0)
        assert (pc["shortest_paths"], pc["self_paths"]) == want, (pc, want)
        assert pc["builds"] >= 1 and pc["build_seconds"] >= 0  # (direct mode: a gather, untimed)
        return stats
    finally:
        top.free()
        set_min_time_jump_hook(None)
        del cb


def test_trace_c1_golden_gml(gpu):
    """C1 (50-node tor-style complete graph, the committed GML) with 75 hosts."""
    text = open(f"{GOLDEN}/c1.gml").read()
    g = graphs.complete_graph(50, seed=1, lat_max=300, self_max=10, loss_max=500)
    st = _replay(g, text, ops=3000, hosts=75, seed=1)
    assert st["reverse_served"] > 0 and st["differs"] > 0, st


@pytest.mark.parametrize("algo", [ALGO_DENSE_FW, ALGO_SPARSE_SSSP])
def test_trace_directed_rgg(gpu, algo):
    """Directed RGG (both orientations, independent latencies): lookup (s, t) after t's run is
    served t -> s's latency."""
    g = graphs.directed_rgg(400, seed=12)
    st = _replay(g, graphs.to_gml(g), algo=algo, ops=3000, seed=2)
    assert st["reverse_served"] > 0 and st["differs"] > 0, st


def test_trace_undirected_sub_ms_complete(gpu):
    """Undirected complete graph with microsecond latencies: the served ms is the serving source's
    own f64 path-order sum (the f64 ms table, raw rows)."""
    g = graphs.complete_graph(120, seed=8)
    rng = np.random.default_rng(77)
    lat = rng.integers(1, 900, g.m).astype(np.int64) * 1_000
    g = graphs.Graph(g.n, False, g.src, g.dst, lat, g.loss)
    st = _replay(g, graphs.to_gml(g), ops=3000, seed=3)
    assert st["reverse_served"] > 0, st


def test_trace_late_attaches(gpu):
    """Hosts attach between lookups: each new vertex starts a table generation and its pairs are
    stored by whichever end runs first afterwards (attach epochs, pairorder.c)."""
    g = graphs.random_geometric(300, seed=5)
    _replay(g, graphs.to_gml(g), ops=3000, hosts=150, late=60, seed=4)
    gd = graphs.directed_rgg(200, seed=6)
    _replay(gd, graphs.to_gml(gd), ops=3000, hosts=120, late=50, seed=5)


@pytest.mark.parametrize("directed", [False, True])
def test_trace_direct_mode(gpu, directed):
    """use_shortest_path = false: a miss stores only the pair's direct edge (topology.c:1816-1858);
    the first direction looked up serves the pair."""
    g = graphs.complete_directed(60, seed=9) if directed else graphs.complete_graph(60, seed=9)
    st = _replay(g, graphs.to_gml(g), use_sp=False, ops=2500, hosts=80, seed=6)
    if directed:
        assert st["reverse_served"] > 0 and st["differs"] > 0, st
