"""The packet path from many worker threads at once (Shadow's --parallelism workers
call getLatency / getReliability / incrementPathPacketCounter concurrently, worker.c:541-555).

The lookups take no lock once their pair is stored: the IP map is read lock-free and the packet
counters are atomic (topology.c's per-source counter pages). The first lookup of a pair decides
its serving path (the lazy cache's run order, topology.c:1189-1215), so the trace first runs every
source once, in a fixed order, on one thread; then 8 or 32 threads replay disjoint packet traces
through srt_topology_send_packets_ip at the same time. Every packet's fate and delay, and every
pair's final counter, must equal the lazy-cache restatement's (oracle/lazy_cache.py) replay of
the same packets."""
import threading
import time

import numpy as np
import pytest

import oracle
from oracle.lazy_cache import LazyPathCache
from shadow_amd import graphs
from shadow_amd.topology import Topology, ip_to_net

pytestmark = pytest.mark.gpu


def _ip(v):
    ip = 0x0B000001 + v  # graphs.to_gml's default ip_base
    return f"{ip >> 24 & 255}.{ip >> 16 & 255}.{ip >> 8 & 255}.{ip & 255}"


@pytest.mark.parametrize("threads", [8, 32])
@pytest.mark.parametrize("kind", ["undirected", "directed"])
def test_concurrent_packet_trace(gpu, threads, kind):
    g = graphs.complete_graph(160, seed=3) if kind == "undirected" else \
        graphs.directed_rgg(300, seed=14)
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    raw = oracle.table(el, True, oracle.ORC_INT_NS, nthreads=8, raw=True)
    sim = LazyPathCache(raw, g.directed, True)
    top = Topology.from_gml(graphs.to_gml(g))
    rng = np.random.default_rng(threads)
    try:
        ips = [_ip(v) for v in range(g.n)]
        for v in range(g.n):
            got, _, _, _ = top.attach(f"100.{v // 200}.{v % 200}.7", 1, ip_hint=ips[v])
            assert got == v
            sim.attach(f"100.{v // 200}.{v % 200}.7", v)
        host = [f"100.{v // 200}.{v % 200}.7" for v in range(g.n)]
        # every source runs once, in one fixed order: every pair is stored before the threads
        order = rng.permutation(g.n)
        for i, v in enumerate(order):
            u = int(order[(i + 1) % g.n])
            assert top.get_latency(host[v], host[u]) == sim.get_latency(host[v], host[u])
        per = 20000
        k = threads * per
        a = rng.integers(0, g.n, k)
        b = rng.integers(0, g.n, k)
        chance = rng.random(k)
        boot = (rng.random(k) < 0.02).astype(np.uint8)
        pay = np.where(rng.random(k) < 0.05, 0, 1400).astype(np.uint64)
        src = np.array([ip_to_net(host[v]) for v in a], np.uint32)
        dst = np.array([ip_to_net(host[v]) for v in b], np.uint32)
        out = [None] * threads

        def work(i):
            s = slice(i * per, (i + 1) * per)
            out[i] = top.send_packets(src[s], dst[s], chance[s], boot[s], pay[s])

        th = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        print(f"{kind}: {k} packets on {threads} threads in {dt * 1e3:.1f} ms "
              f"({k / dt:.3g} packets/s)")
        for i in range(threads):
            for j in range(i * per, (i + 1) * per, 97):  # a spread sample of the fates
                want = sim.send_packet(host[a[j]], host[b[j]], chance[j], bool(boot[j]), int(pay[j]))
                got = (bool(out[i][0][j - i * per]), int(out[i][1][j - i * per]))
                assert got[0] == want[0] and (not got[0] or got[1] == want[1]), (j, got, want)
        # every packet through the restatement (the sampled ones above already counted)
        sampled = np.zeros(k, bool)
        for i in range(threads):
            sampled[np.arange(i * per, (i + 1) * per, 97)] = True
        for j in np.nonzero(~sampled)[0]:
            sim.send_packet(host[a[j]], host[b[j]], chance[j], bool(boot[j]), int(pay[j]))
        for x in range(0, g.n, 3):
            for y in range(g.n):
                p = sim._get(x, y) or sim._get(y, x)
                assert top.packet_count(host[x], host[y]) == (0 if p is None else p.packets), (x, y)
    finally:
        top.free()
