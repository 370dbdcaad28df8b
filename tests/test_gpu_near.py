"""lvl_near_kernel (levels.hip; levels 2 and 3 from the in-arc runs, taken for shares of at least
16,384 sources) where C4 does not reach it: weight-1 runs longer than 64 arcs (the kernel's tail
loop). A 16,384-node complete graph with latencies U{1..200} ms has ~82 one-ms in-arcs per vertex;
the default one-GPU schedule (encoding 12) is checked against the CPU oracle's dense Dijkstra on
rows spread over the graph: latency bit-exact, reliability within 1e-12 relative (north_star).
The canonical predecessor rule is the reference's Dijkstra (topology.c:1679-1701) up to igraph's
tie order."""
import ctypes

import numpy as np
import pytest

import oracle
from shadow_amd import _lib

pytestmark = pytest.mark.gpu
REL_TOL = 1e-12


@pytest.mark.parametrize("n,lat_max,seed", [(16384, 200, 41), (16384 + 96, 150, 42)])
def test_levels_near_kernel_long_weight1_runs(gpu, n, lat_max, seed):
    import torch
    L = _lib.lib()
    ld = (n + 255) // 256 * 256
    w = torch.empty((ld, ld), dtype=torch.int32, device="cuda")
    r = torch.empty((ld, ld), dtype=torch.float64, device="cuda")
    _lib.check(L.srt_gen_complete_device(n, ld, 0, ld, seed, lat_max, 10, 500, w.data_ptr(),
                                         r.data_ptr(), None), "generate")
    lat = torch.empty_like(w)
    rel = torch.empty_like(r)
    st = _lib.BuildStats()
    _lib.check(L.srt_dense_build_device(n, ld, 0, w.data_ptr(), r.data_ptr(), lat.data_ptr(),
                                        rel.data_ptr(), None, 0, ctypes.byref(st)), "build")
    torch.cuda.synchronize()
    del w, r
    assert st.dist_enc == 12, st.dist_enc
    rows = np.array(sorted({0, 1, 63, 64, 4095, 8191, 8192, n // 2 + 7, n - 97, n - 33, n - 1}),
                    np.int32)
    idx = torch.from_numpy(rows.astype(np.int64)).cuda()
    glat = lat.index_select(0, idx)[:, :n].cpu().numpy().view(np.uint32).astype(np.uint64) \
        * np.uint64(1_000_000)
    grel = rel.index_select(0, idx)[:, :n].cpu().numpy()
    del lat, rel
    clat, crel, _, _ = oracle.complete_sample(n, seed, lat_max, 10, 500, rows, 16)
    off = np.arange(n)[None, :] != rows[:, None]
    bad = np.argwhere(np.where(off, glat, 0) != np.where(off, clat, 0))
    assert bad.size == 0, f"{len(bad)} latency mismatches, first {bad[:5].tolist()}"
    err = np.abs(grel - crel) / np.maximum(crel, 1e-300)
    assert float(err[off].max()) <= REL_TOL
