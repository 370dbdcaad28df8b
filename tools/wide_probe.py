"""Time the u64 rows (wide.hip) on VERDICT r02's directed 100k BA graph with 1..100,000 us
latencies (q = 1 us; the graph is not strongly connected, so its bound passes SRT_INF): build
time for K attached sources, and the same sources' rows of the undirected variant (u32 kernels)
for scale. Test infrastructure: prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from shadow_amd import graphs  # noqa: E402
from shadow_amd._lib import ALGO_AUTO  # noqa: E402
from shadow_amd.topology import build_tables_subset  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    b = graphs.barabasi_albert(100_000, m=3, seed=5)
    rng = np.random.default_rng(7)
    lat = rng.integers(1, 100_001, b.m).astype(np.int64) * 1000
    verts = np.sort(rng.choice(b.n, k, replace=False)).astype(np.int32)
    out = {"sources": k}
    for directed in (True, False):
        g = graphs.Graph(b.n, directed, b.src, b.dst, lat, b.loss, "ba100k_us")
        build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss, verts=verts,
                            algo=ALGO_AUTO, want_ms=True)  # warm
        t0 = time.perf_counter()
        _, _, _, _, st = build_tables_subset(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                             verts=verts, algo=ALGO_AUTO, want_ms=True)
        wall = (time.perf_counter() - t0) * 1e3
        key = "directed" if directed else "undirected"
        out[key] = {"dist_enc": st.dist_enc, "ms_rows": round(st.ms_total, 2),
                    "ms_wall": round(wall, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
