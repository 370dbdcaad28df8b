"""Time the multi-source sparse kernel (msssp.hip) on a bench graph (the per-batch phase
profile of round 2 was retired from the product; rocprofv3 gives the kernel time).
python tools/msssp_probe.py c3 [--reps 2]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from shadow_amd import graphs  # noqa: E402
from shadow_amd._lib import BuildStats  # noqa: E402
from shadow_amd.topology import SparseGraph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("graph")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--nsrc", type=int, default=0)
a = ap.parse_args()
g = graphs.random_geometric(20000, seed=3) if a.graph == "c3" else \
    graphs.barabasi_albert(100_000, seed=5)
sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
ns = a.nsrc or g.n
lat = torch.empty((ns, g.n), dtype=torch.int32, device="cuda")
rel = torch.empty((ns, g.n), dtype=torch.float64, device="cuda")
for r in range(a.reps):
    st = BuildStats()
    torch.cuda.synchronize()
    t = time.perf_counter()
    sg.rows(0, ns, lat.data_ptr(), rel.data_ptr(), None, st)
    torch.cuda.synchronize()
    print(f"{a.graph} rows 0..{ns}: {1e3 * (time.perf_counter() - t):.1f} ms wall, kernel "
          f"{st.ms_update:.1f} ms, dist_enc {st.dist_enc} "
          f"SRT_FORM={os.environ.get('SRT_FORM')}", flush=True)
sg.free()
