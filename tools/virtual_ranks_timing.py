#!/usr/bin/env python3
"""Schedule cost of the row-sharded dense paths on ONE GPU (virtual ranks, SRT_VIRTUAL_RANKS):
the ranks share the device, so the build time is total work + schedule overhead. Compares the
single-GPU build, the sharded all-tile rounds (SRT_FORM sym=0) and the sharded symmetric rounds.
usage: python tools/virtual_ranks_timing.py [n]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from shadow_amd import graphs  # noqa: E402
from shadow_amd._lib import ALGO_DENSE_FW  # noqa: E402
from shadow_amd.topology import build_tables  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
g = graphs.complete_graph(n, seed=4, lat_max=1000)
ref = None
for label, env, ngpus in [("single", {}, None), ("virtual2 all-tile", {"SRT_VIRTUAL_RANKS": "2", "SRT_FORM": "sym=0"}, 1),
                          ("virtual2 symmetric", {"SRT_VIRTUAL_RANKS": "2"}, 1),
                          ("virtual4 symmetric", {"SRT_VIRTUAL_RANKS": "4"}, 1)]:
    for k in ("SRT_VIRTUAL_RANKS", "SRT_FORM"):
        os.environ.pop(k, None)
    os.environ.update(env)
    best = None
    for rep in range(2):
        t0 = time.perf_counter()
        lat, rel, st = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss, algo=ALGO_DENSE_FW,
                                    ngpus=ngpus)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    if ref is None:
        ref = (lat, rel)
    same = bool(np.array_equal(lat, ref[0]) and np.array_equal(rel, ref[1]))
    print(f"{label:22s} wall {best * 1e3:8.1f} ms  fw {st.ms_fw:8.1f} ms  post {st.ms_post:7.1f} ms  "
          f"enc {st.dist_enc}  same_as_single {same}", flush=True)
