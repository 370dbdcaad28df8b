#!/usr/bin/env python3
"""Per-build timing of the C5 derived build (wgsssp_kernel core rows + derive_chain_kernel), one
JSON line per build, so the run-to-run spread of the core kernel is visible build by build (the
bench line only carries the average of its timed builds). Timing only: the rows go to device
buffers and nothing is checked (bench.py and tests/test_gpu_derive.py check them).

usage: python tools/c5_launches.py [--builds 8] [--n 100000]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from shadow_amd import _lib, graphs  # noqa: E402
from shadow_amd.topology import SparseGraph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--builds", type=int, default=8)
    ap.add_argument("--n", type=int, default=100000)
    a = ap.parse_args()
    g = graphs.barabasi_albert(a.n, seed=5)
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss, device=0)
    lat = torch.empty((g.n, g.n), dtype=torch.int32, device="cuda")
    rel = torch.empty((g.n, g.n), dtype=torch.float64, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    lib = os.path.basename(_lib.LIB_PATH)
    for b in range(a.builds):
        s = _lib.BuildStats()
        s.time_kernels = 1
        t0 = time.perf_counter()
        sg.rows(0, g.n, lat.data_ptr(), rel.data_ptr(), st.cuda_stream, s)
        st.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"lib": lib, "build": b, "wall_ms": round(wall, 1),
                          "ms_core": round(s.ms_core, 1), "ms_derive": round(s.ms_derive, 1),
                          "n_derived": int(s.n_derived)}), flush=True)


if __name__ == "__main__":
    main()
