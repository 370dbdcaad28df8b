#!/usr/bin/env python3
"""End-to-end drop-in time: the reference's entry points timed from host inputs to
host tables, beside the device-resident build that bench.py reports.

  C3  topology API: GML text -> srt_topology_new_from_string (topology.c:326-1122 restated) ->
      topology_computeShortestPaths (topology.c:1604-1656): the canonical graph, the sparse rows,
      the tables staged into the generation's host buffers.
  C4  srt_build_tables on the host edge list of the 32768-node complete graph (537M edges, the
      graph bench.py's generator fills on the device): the edge scan (quantum, validation), the
      edges staged to the device through a two-slot pinned ring and scattered into the dense
      matrices there, the level build, the tables staged back. The result is compared entry by entry with the device-resident build of
      the same graph (srt_gen_complete_device + srt_dense_build_device, the bench path).

Each build runs twice (the second sees the pinned slot cache warm); the line carries the wall time
and the library's own phase clocks (srt_build_stats ms_canon, ms_upload, ms_total, ms_download).
C4 then runs once more into page-locked tables the caller allocated (hipHostMalloc, timed), which
the library moves with one DMA per table instead of the staging ring.

usage: python tools/dropin_time.py [--only c3|c4] [--out profiles/r05_dropin.json]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from shadow_amd import _lib, graphs  # noqa: E402
from shadow_amd.topology import Topology  # noqa: E402

MS = 1_000_000


def log(*a):
    print("[dropin]", *a, file=sys.stderr, flush=True)


def phases(st):
    return {k: round(getattr(st, k), 1) for k in ("ms_canon", "ms_upload", "ms_total", "ms_download")}


def c3():
    g = graphs.random_geometric(20_000, seed=3)
    text = graphs.to_gml(g)
    out = {"graph": "C3", "n": g.n, "edges": int(g.m), "runs": []}
    for rep in range(2):
        t0 = time.perf_counter()
        top = Topology.from_gml(text)
        t1 = time.perf_counter()
        top.compute_shortest_paths(1)
        t2 = time.perf_counter()
        st = top.stats()
        out["runs"].append({"parse_ms": round((t1 - t0) * 1e3, 1),
                            "compute_shortest_paths_ms": round((t2 - t1) * 1e3, 1),
                            **phases(st), "algo": st.algo, "dist_enc": st.dist_enc})
        log("C3", out["runs"][-1])
        top.free()
    return out


def complete_edges(n, seed, lat_max, self_max, loss_max):
    """complete_graph(n, seed, ...) written row block by row block (no n^2/2 int64 temporaries)"""
    m = n * (n + 1) // 2
    src = np.empty(m, np.int32)
    dst = np.empty(m, np.int32)
    lat = np.empty(m, np.int64)
    loss = np.empty(m, np.float64)
    pos = 0
    for i in range(n):
        j = np.arange(i, n, dtype=np.uint64)
        ii = np.full(j.shape, i, np.uint64)
        k = len(j)
        src[pos:pos + k] = i
        dst[pos:pos + k] = j
        h0 = np.uint64(1) + graphs.hash_u64(seed, 0, ii, j) % np.uint64(lat_max)
        h1 = graphs.hash_u64(seed, 1, ii, j) % np.uint64(loss_max + 1)
        h0[0] = 1 + int(graphs.hash_u64(seed, 2, ii[:1], j[:1])[0] % np.uint64(self_max))
        h1[0] = int(graphs.hash_u64(seed, 3, ii[:1], j[:1])[0] % np.uint64(loss_max + 1))
        lat[pos:pos + k] = h0.astype(np.int64) * MS
        loss[pos:pos + k] = h1.astype(np.float64) / 10000.0
        pos += k
        if i % 4096 == 0:
            log(f"C4 edges: row {i}/{n}")
    return src, dst, lat, loss


def c4(n=32768, seed=4):
    import torch
    L = _lib.lib()
    t0 = time.perf_counter()
    src, dst, lat_ns, loss = complete_edges(n, seed, 1000, 10, 500)
    gen_s = time.perf_counter() - t0
    log(f"C4 edge list: {len(src)} edges in {gen_s:.1f} s")
    e = _lib.Edges(n, 0, len(src), src.ctypes.data, dst.ctypes.data, lat_ns.ctypes.data,
                   loss.ctypes.data)
    o = _lib.BuildOpts(0, _lib.ALGO_AUTO, 1, 0)
    lat = np.empty((n, n), np.uint32)
    rel = np.empty((n, n), np.float64)
    q = ctypes.c_uint64()
    out = {"graph": "C4", "n": n, "edges": int(len(src)), "edge_list_gen_s": round(gen_s, 1),
           "runs": []}
    for rep in range(2):
        st = _lib.BuildStats()
        t1 = time.perf_counter()
        _lib.check(L.srt_build_tables(ctypes.byref(e), ctypes.byref(o), lat.ctypes.data,
                                      ctypes.byref(q), rel.ctypes.data, ctypes.byref(st)),
                   "srt_build_tables")
        t2 = time.perf_counter()
        out["runs"].append({"srt_build_tables_ms": round((t2 - t1) * 1e3, 1), **phases(st),
                            "dist_enc": st.dist_enc, "levels": st.levels})
        log("C4", out["runs"][-1])
    # the same call into page-locked tables (hipHostMalloc by the caller): one DMA per table
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    pl, pr = ctypes.c_void_p(), ctypes.c_void_p()
    t1 = time.perf_counter()
    assert hip.hipHostMalloc(ctypes.byref(pl), n * n * 4, 0) == 0
    assert hip.hipHostMalloc(ctypes.byref(pr), n * n * 8, 0) == 0
    pin_ms = (time.perf_counter() - t1) * 1e3
    st = _lib.BuildStats()
    t1 = time.perf_counter()
    _lib.check(L.srt_build_tables(ctypes.byref(e), ctypes.byref(o), pl.value, ctypes.byref(q),
                                  pr.value, ctypes.byref(st)), "srt_build_tables")
    t2 = time.perf_counter()
    plat = np.ctypeslib.as_array(ctypes.cast(pl, ctypes.POINTER(ctypes.c_uint32)), (n, n))
    prel = np.ctypeslib.as_array(ctypes.cast(pr, ctypes.POINTER(ctypes.c_double)), (n, n))
    same = bool(np.array_equal(plat, lat)) and bool(np.array_equal(prel, rel))
    out["pinned_tables"] = {"host_malloc_ms": round(pin_ms, 1),
                            "srt_build_tables_ms": round((t2 - t1) * 1e3, 1), **phases(st),
                            "same_tables": same}
    log("C4 pinned tables", out["pinned_tables"])
    del plat, prel
    hip.hipHostFree(pl)
    hip.hipHostFree(pr)
    del src, dst, lat_ns, loss
    # the bench path on the same graph, compared entry by entry
    ld = n
    w = torch.empty((ld, ld), dtype=torch.int32, device="cuda")
    r = torch.empty((ld, ld), dtype=torch.float64, device="cuda")
    _lib.check(L.srt_gen_complete_device(n, ld, 0, ld, seed, 1000, 10, 500, w.data_ptr(),
                                         r.data_ptr(), None), "generate")
    dl = torch.empty_like(w)
    dr = torch.empty_like(r)
    st = _lib.BuildStats()
    _lib.check(L.srt_dense_build_device(n, ld, 0, w.data_ptr(), r.data_ptr(), dl.data_ptr(),
                                        dr.data_ptr(), None, 0, ctypes.byref(st)), "build")
    torch.cuda.synchronize()
    del w, r
    q_ms = q.value // MS
    same_lat = same_rel = True
    for b in range(0, n, 4096):
        hl = dl[b:b + 4096].cpu().numpy().view(np.uint32)
        hr = dr[b:b + 4096].cpu().numpy()
        same_lat &= bool(np.array_equal(lat[b:b + 4096].astype(np.uint64) * np.uint64(q_ms),
                                        hl.astype(np.uint64)))
        same_rel &= bool(np.array_equal(rel[b:b + 4096], hr))
    out["quantum_ns"] = int(q.value)
    out["matches_device_resident_build"] = {"lat": same_lat, "rel": same_rel}
    out["device_resident_ms_total"] = round(st.ms_total, 1)
    log("C4 parity vs device-resident build:", out["matches_device_resident_build"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["c3", "c4"], default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch  # one HIP runtime for torch and the library: torch initialises it first
    assert torch.cuda.is_available()
    res = {"host_cpus": os.cpu_count(), "staging_threads": min(16, os.cpu_count() or 1)}
    if a.only in (None, "c3"):
        res["c3"] = c3()
    if a.only in (None, "c4"):
        res["c4"] = c4()
    s = json.dumps(res)
    print(s, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
