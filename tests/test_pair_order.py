"""The product's pair-order layer (shadow_amd/csrc/pairorder.c) against the lazy-cache restatement
(oracle/lazy_cache.py) on CPU: which cached path serves each lookup, and what each miss stores.

The reference serves a vertex pair, in both directions, from the first source run that stored it
(topology.c:1189-1215, :1900-1981); directed lookups still run their own source (:1919) and then
fall back to the reverse path (:1963-1967). The C layer decides this from per-vertex run stamps
per attach epoch; the restatement replays the reference's cache literally. Both see the same
random traces -- directed and undirected, shortest-path and direct mode, attaches before and
between lookups, several hosts per vertex -- and must agree on every lookup's serving vertex, on
the paths each miss stores (through the runahead minimum they feed), and on a final peek of every
pair. No GPU: the tables here are random stand-ins (the pair order never reads them).
"""
import ctypes

import numpy as np
import pytest

from oracle.lazy_cache import LazyPathCache
from shadow_amd._lib import PAIR_REACH_FN, PAIR_STORE_FN, lib


class _Runahead:
    """topology.c's offer rule over the paths a lookup stored (minimumPathLatency, :1253-1264)."""

    def __init__(self, lat):
        self.lat, self.minimum = lat, 0.0

    def __call__(self, _ctx, src, targets, count):
        best = min(float(self.lat[src, targets[i]]) for i in range(count))
        if self.minimum == 0 or best < self.minimum:
            self.minimum = best


def _replay(n, directed, use_sp, seed, ops, late_attach, oneway=False):
    rng = np.random.default_rng(seed)
    lat = rng.integers(1, 50, (n, n)).astype(np.float64)  # ms; ties on purpose
    rel = rng.random((n, n))
    if oneway:
        # two strongly connected halves A = [0, n/2), B = [n/2, n) joined by one-way arcs A -> B:
        # no vertex of B reaches A (the oracle's rows hold INFINITY there)
        lat[n // 2:, :n // 2] = np.inf
    sim = LazyPathCache({"lat_ms": lat, "rel": rel}, directed, use_sp)
    L = lib()
    po = L.srt_pair_order_new(n, int(directed), int(use_sp))
    assert po
    reach_cb = PAIR_REACH_FN(lambda _c, s, t: int(np.isfinite(lat[s, t])))
    if oneway:
        L.srt_pair_order_set_reach(po, reach_cb, None)
    ra = _Runahead(lat)
    cb = PAIR_STORE_FN(ra)
    hosts = {}
    try:
        nh = 3 * n // 2
        host_vertex = rng.integers(0, n, nh)
        first = nh if not late_attach else nh // 3
        for h in range(first):
            hosts[h] = int(host_vertex[h])
            sim.attach(h, hosts[h])
            assert L.srt_pair_order_attach(po, hosts[h]) == 0
        for k in range(ops):
            if late_attach and len(hosts) < nh and rng.random() < 0.05:
                h = len(hosts)
                hosts[h] = int(host_vertex[h])
                sim.attach(h, hosts[h])
                L.srt_pair_order_attach(po, hosts[h])
                continue
            a, b = (int(x) for x in rng.choice(list(hosts), 2))
            try:
                p = sim.path_entry(a, b)
            except RuntimeError:  # the reference's panic: no stored path joins them
                p = None
            f = L.srt_pair_order_lookup(po, hosts[a], hosts[b], cb, None)
            if p is None:
                assert f == -8, (k, hosts[a], hosts[b], f)  # SRT_E_NOPATH
                assert ra.minimum == sim.minimum_path_latency, k
                continue
            assert f == p.src, (k, hosts[a], hosts[b], f, p.src)
            assert (hosts[b] if f == hosts[a] else hosts[a]) == p.dst
            assert ra.minimum == sim.minimum_path_latency, k
        # every pair of attached vertices: the stored direction, without recording anything
        att = sorted(set(hosts.values()))
        for x in att:
            for y in att:
                p = sim._get(x, y) or sim._get(y, x)
                if x == y:
                    p = sim._get(x, x)
                want = -1 if p is None else p.src
                assert L.srt_pair_order_peek(po, x, y) == want, (x, y)
        # the reference's diagnostics (topology.c:78-79): Dijkstra runs and self paths
        runs, selfs = ctypes.c_uint32(), ctypes.c_uint32()
        L.srt_pair_order_counts(po, ctypes.byref(runs), ctypes.byref(selfs))
        assert (runs.value, selfs.value) == ((sim.source_runs, sim.self_runs) if use_sp else (0, 0))
        if use_sp:
            # one recorded run per source per attach epoch it ran in (directed sources re-run on
            # every miss in the reference; those re-runs store nothing new)
            for v in att:
                assert L.srt_pair_order_runs(po, v) <= 1 + len(hosts)
        return sim
    finally:
        L.srt_pair_order_free(po)


@pytest.mark.parametrize("directed", [False, True])
@pytest.mark.parametrize("use_sp", [True, False])
@pytest.mark.parametrize("late_attach", [False, True])
def test_pair_order_matches_lazy_cache(directed, use_sp, late_attach):
    for seed in range(3):
        sim = _replay(40, directed, use_sp, 100 * seed + 7, 1500, late_attach)
        if use_sp:
            assert sim.source_runs > 0


@pytest.mark.parametrize("late_attach", [False, True])
def test_pair_order_unreachable_targets(late_attach):
    """a source run stores only the targets it reaches (topology.c:1744-1753). On a
    directed graph with one-way reachability, the pair {s, t} (t unreachable from s) is stored by
    t's run even when s ran first, and a lookup whose ends do not reach each other either way
    finds no path."""
    for seed in range(4):
        _replay(40, True, True, 31 * seed + 5, 1500, late_attach, oneway=True)


def test_pair_order_unreachable_small():
    L = lib()
    po = L.srt_pair_order_new(3, 1, 1)
    reach = PAIR_REACH_FN(lambda _c, s, t: int(not (s == 1 and t == 0)))  # 1 does not reach 0
    L.srt_pair_order_set_reach(po, reach, None)
    try:
        for v in range(3):
            L.srt_pair_order_attach(po, v)
        assert L.srt_pair_order_lookup(po, 1, 2, None, None) == 1  # source 1 runs first
        assert L.srt_pair_order_peek(po, 1, 0) == -1               # ... but cannot store {0, 1}
        assert L.srt_pair_order_lookup(po, 0, 2, None, None) == 0  # source 0 runs
        assert L.srt_pair_order_peek(po, 1, 0) == 0                # {0, 1} is 0's path
        assert L.srt_pair_order_lookup(po, 1, 0, None, None) == 0  # served 0 -> 1
    finally:
        L.srt_pair_order_free(po)


def test_pair_order_directed_reverse_serving():
    """The case the verdict names: on a directed graph, once t's source ran, getLatency(s, t)
    is served t's path t -> s, and s still runs (its other pairs are stored from s)."""
    L = lib()
    po = L.srt_pair_order_new(5, 1, 1)
    try:
        for v in range(5):
            L.srt_pair_order_attach(po, v)
        assert L.srt_pair_order_lookup(po, 3, 1, None, None) == 3  # source 3 runs
        assert L.srt_pair_order_runs(po, 3) == 1 and L.srt_pair_order_runs(po, 1) == 0
        assert L.srt_pair_order_lookup(po, 1, 3, None, None) == 3  # served 3 -> 1
        assert L.srt_pair_order_runs(po, 1) == 1                   # and source 1 ran
        assert L.srt_pair_order_peek(po, 1, 4) == 1                # storing (1, 4)
        assert L.srt_pair_order_lookup(po, 1, 3, None, None) == 3  # no further run recorded
        assert L.srt_pair_order_runs(po, 1) == 1
        assert L.srt_pair_order_peek(po, 2, 2) == -1
        assert L.srt_pair_order_lookup(po, 2, 2, None, None) == 2  # self path
        assert L.srt_pair_order_peek(po, 2, 2) == 2
    finally:
        L.srt_pair_order_free(po)


def test_pair_order_unattached_and_bad_arguments():
    L = lib()
    po = L.srt_pair_order_new(4, 0, 1)
    try:
        L.srt_pair_order_attach(po, 0)
        assert L.srt_pair_order_lookup(po, 0, 1, None, None) == -9  # SRT_E_UNATTACHED
        assert L.srt_pair_order_lookup(po, 0, 7, None, None) == -1  # SRT_E_ARG
        assert L.srt_pair_order_attach(po, 4) == -1
    finally:
        L.srt_pair_order_free(po)
    assert not L.srt_pair_order_new(0, 0, 1)


def test_pair_order_concurrent_lookups_agree():
    """Lookups from several threads (Shadow's worker threads) decide every pair once: each
    lookup's serving vertex equals the final stored direction of its pair."""
    import threading
    n = 64
    L = lib()
    po = L.srt_pair_order_new(n, 0, 1)
    try:
        for v in range(n):
            L.srt_pair_order_attach(po, v)
        results = [[] for _ in range(8)]

        def work(i):
            rng = np.random.default_rng(i)
            for _ in range(4000):
                a, b = (int(x) for x in rng.integers(0, n, 2))
                results[i].append((a, b, L.srt_pair_order_lookup(po, a, b, None, None)))

        th = [threading.Thread(target=work, args=(i,)) for i in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for res in results:
            for a, b, f in res:
                assert f == L.srt_pair_order_peek(po, a, b) and f in (a, b)
    finally:
        L.srt_pair_order_free(po)
