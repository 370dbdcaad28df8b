#!/usr/bin/env python3
"""Packet-path throughput (worker.c:541-555) at 1 / 8 / 32 host threads.

The C3 graph (20,000-vertex RGG) with one host per vertex; every source runs once (so every pair
is stored and lookups take no lock), then T threads replay disjoint random packet traces through
srt_topology_send_packets_ip (one C call per 250k-packet batch; ctypes releases the GIL), first
once untimed (warm-up: counter pages allocated), then timed. Prints one JSON line: packets/s per
thread count, with the table build time. Test infrastructure."""
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from shadow_amd import graphs  # noqa: E402
from shadow_amd.topology import Topology, ip_to_net  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    g = graphs.random_geometric(n, seed=3)
    t0 = time.perf_counter()
    top = Topology.from_gml(graphs.to_gml(g))
    host = [f"{10 + v // 65536}.{v // 256 % 256}.{v % 256}.7" for v in range(n)]
    ips = [0x0B000001 + v for v in range(n)]
    hints = [f"{ip >> 24 & 255}.{ip >> 16 & 255}.{ip >> 8 & 255}.{ip & 255}" for ip in ips]
    top.attach_batch(host, [1] * n, ip_hints=hints)
    top.compute_shortest_paths()
    build_s = time.perf_counter() - t0
    rng = np.random.default_rng(1)
    net = np.array([ip_to_net(h) for h in host], np.uint32)
    t1 = time.perf_counter()
    order = rng.permutation(n)
    first = np.roll(order, 1)
    top.send_packets(net[order], net[first], np.zeros(n), np.ones(n, np.uint8))  # every source runs
    runs_s = time.perf_counter() - t1
    res = {"graph": f"C3 RGG n={n}, {g.m} edges, one host per vertex",
           "setup_s": round(build_s, 2), "first_runs_s": round(runs_s, 2), "threads": {}}
    batch = 250_000
    for threads in (1, 8, 32):
        nb = 4 if threads == 1 else 2
        k = threads * nb * batch
        a = net[rng.integers(0, n, k)]
        b = net[rng.integers(0, n, k)]
        ch = rng.random(k)

        def work(i):
            for q in range(nb):
                o = (i * nb + q) * batch
                top.send_packets(a[o:o + batch], b[o:o + batch], ch[o:o + batch])

        # warm-up: the same trace once untimed, so the lazily allocated per-path counter pages
        # (topology.c cnt_slot) exist before the timed pass, at every thread count alike
        th = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        th = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
        t2 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t2
        res["threads"][str(threads)] = {"packets": k, "seconds": round(dt, 3),
                                        "packets_per_s": round(k / dt, 1)}
        print(f"[packet_rate] {threads} threads: {k / dt:.3g} packets/s", file=sys.stderr,
              flush=True)
    res["cpus_visible"] = len(os.sched_getaffinity(0))
    print(json.dumps(res), flush=True)
    top.free()


if __name__ == "__main__":
    main()
