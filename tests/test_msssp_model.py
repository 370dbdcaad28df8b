"""CPU model of the multi-source kernel's algorithm (tools/msssp_sim.c): 64 sources pulled to a
fixed point with delta-stepping over the lane minimum reach the oracle's canonical table bit for
bit (latency and path-order reliability), in place (Gauss-Seidel) and from the previous pass's
states (Jacobi, the GPU's worst case), on undirected and directed graphs. The kernel itself is
checked against the oracle in tests/test_gpu_msssp.py."""
import ctypes
import os
import sys

import numpy as np
import pytest

import oracle
from shadow_amd import graphs

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import msssp_sim  # noqa: E402


@pytest.fixture(scope="module")
def simlib():
    return msssp_sim.load()


@pytest.mark.parametrize("which,jacobi,delta", [("rgg", 0, 16), ("rgg", 1, 1), ("drgg", 1, 8),
                                                ("ba", 0, 4)])
def test_model_matches_oracle(simlib, which, jacobi, delta):
    if which == "rgg":
        g = graphs.random_geometric(1500, seed=8)
    elif which == "drgg":
        g = graphs.directed_rgg(1200, seed=9)
    else:
        g = graphs.barabasi_albert(1500, seed=10)
    n, irp, icol, iw, ir, orp, ocol = msssp_sim.csr(g)
    cl = msssp_sim.clusters(n, orp, ocol)
    srcs = cl[len(cl) // 2]
    D = np.empty((64, n), np.uint32)
    R = np.empty((64, n), np.float64)
    c = msssp_sim.Counts()
    P = ctypes.c_void_p
    assert simlib.msssp_sim_batch(n, P(irp.ctypes.data), P(icol.ctypes.data), P(iw.ctypes.data),
                                  P(ir.ctypes.data), P(orp.ctypes.data), P(ocol.ctypes.data),
                                  len(srcs), P(srcs.ctypes.data), ctypes.c_uint32(delta), jacobi,
                                  P(D.ctypes.data), P(R.ctypes.data), ctypes.byref(c)) == 0
    k = len(srcs)
    ref = oracle.sssp_list(oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss), srcs)
    q = int(np.gcd.reduce(g.lat_ns[g.lat_ns > 0]))
    off = np.ones((k, n), bool)
    off[np.arange(k), srcs] = False
    reach = ref["lat_int"] != np.uint64(0xFFFFFFFFFFFFFFFF)
    assert np.array_equal(D[:k][off & reach].astype(np.uint64), (ref["lat_int"] // q)[off & reach])
    assert np.array_equal(R[:k][off].view(np.uint64), ref["rel"][off].view(np.uint64))
    assert c.passes > 0 and c.pulls > 0
