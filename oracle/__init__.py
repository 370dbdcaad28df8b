"""TEST INFRASTRUCTURE ONLY -- CPU oracle for Shadow's routing precomputation.

Python binding of oracle/oracle.c, the plain-C restatement of
/root/reference/src/main/routing/topology.c (see oracle.h for the file:line map). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package; the product
(shadow_amd/) never does.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

ORC_INT_NS = 0
ORC_F64_MS = 1
U64_MAX = np.iinfo(np.uint64).max


class _Graph(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int32),
        ("directed", ctypes.c_int32),
        ("m", ctypes.c_int64),
        ("src", ctypes.c_void_p),
        ("dst", ctypes.c_void_p),
        ("lat_ns", ctypes.c_void_p),
        ("loss", ctypes.c_void_p),
    ]


_lib = None


def build() -> None:
    """Compile liboracle.so in place (gcc)."""
    import subprocess

    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_sssp_rows.restype = ctypes.c_int
        L.orc_sssp_rows.argtypes = [ctypes.POINTER(_Graph), ctypes.c_int, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_int] + [ctypes.c_void_p] * 5
        L.orc_sssp_list.restype = ctypes.c_int
        L.orc_sssp_list.argtypes = [ctypes.POINTER(_Graph), ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_int32, ctypes.c_int] + [ctypes.c_void_p] * 5
        for fn in (L.orc_table, L.orc_table_raw):
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.POINTER(_Graph), ctypes.c_int, ctypes.c_int,
                           ctypes.c_int] + [ctypes.c_void_p] * 4
        _lib = L
    return _lib


class EdgeList:
    """Edges in GML order: src/dst vertex indices, latency in ns, packet_loss."""

    def __init__(self, n, directed, src, dst, lat_ns, loss):
        self.n = int(n)
        self.directed = int(bool(directed))
        self.src = np.ascontiguousarray(src, dtype=np.int32)
        self.dst = np.ascontiguousarray(dst, dtype=np.int32)
        self.lat_ns = np.ascontiguousarray(lat_ns, dtype=np.int64)
        self.loss = np.ascontiguousarray(loss, dtype=np.float64)
        self.m = len(self.src)

    def _c(self) -> _Graph:
        return _Graph(self.n, self.directed, self.m, self.src.ctypes.data, self.dst.ctypes.data,
                      self.lat_ns.ctypes.data, self.loss.ctypes.data)


def _ptr(a):
    return None if a is None else a.ctypes.data


def sssp_rows(g: EdgeList, s0: int = 0, s1: int | None = None, mode: int = ORC_INT_NS,
              nthreads: int = 1, want_pred: bool = False):
    """Raw per-source rows [s0, s1): dict of lat_int, lat_ref, rel, lat_ms (, pred)."""
    s1 = g.n if s1 is None else s1
    rows = s1 - s0
    out = {
        "lat_int": np.empty((rows, g.n), np.uint64),
        "lat_ref": np.empty((rows, g.n), np.uint64),
        "rel": np.empty((rows, g.n), np.float64),
        "lat_ms": np.empty((rows, g.n), np.float64),
    }
    pred = np.empty((rows, g.n), np.int32) if want_pred else None
    cg = g._c()
    rc = lib().orc_sssp_rows(ctypes.byref(cg), mode, s0, s1, nthreads, _ptr(out["lat_int"]),
                             _ptr(out["lat_ref"]), _ptr(out["rel"]), _ptr(out["lat_ms"]),
                             _ptr(pred))
    if rc:
        raise RuntimeError("orc_sssp_rows failed")
    if want_pred:
        out["pred"] = pred
    return out


def sssp_list(g: EdgeList, sources, mode: int = ORC_INT_NS, nthreads: int = 1):
    """Raw rows of an arbitrary source list: row i belongs to sources[i]."""
    src = np.ascontiguousarray(sources, dtype=np.int32)
    k = len(src)
    out = {
        "lat_int": np.empty((k, g.n), np.uint64),
        "lat_ref": np.empty((k, g.n), np.uint64),
        "rel": np.empty((k, g.n), np.float64),
        "lat_ms": np.empty((k, g.n), np.float64),
    }
    cg = g._c()
    rc = lib().orc_sssp_list(ctypes.byref(cg), mode, src.ctypes.data, k, nthreads,
                             _ptr(out["lat_int"]), _ptr(out["lat_ref"]), _ptr(out["rel"]),
                             _ptr(out["lat_ms"]), None)
    if rc:
        raise RuntimeError("orc_sssp_list failed")
    return out


def table(g: EdgeList, use_shortest_path: bool = True, mode: int = ORC_INT_NS,
          nthreads: int = 1, raw: bool = False):
    """Full n x n table. raw=False: as the reference's lookup API returns every pair when sources
    run in increasing vertex order (undirected: the row of min(s, t)). raw=True: entry (s, t) is
    source s's own row (what the product's tables hold; lazy_cache.py picks the serving row)."""
    n = g.n
    out = {
        "lat_int": np.empty((n, n), np.uint64),
        "lat_ref": np.empty((n, n), np.uint64),
        "rel": np.empty((n, n), np.float64),
        "lat_ms": np.empty((n, n), np.float64),
    }
    cg = g._c()
    fn = lib().orc_table_raw if raw else lib().orc_table
    rc = fn(ctypes.byref(cg), int(bool(use_shortest_path)), mode, nthreads,
                         _ptr(out["lat_int"]), _ptr(out["lat_ref"]), _ptr(out["rel"]),
                         _ptr(out["lat_ms"]))
    if rc:
        raise RuntimeError("orc_table failed (direct mode needs a complete graph)")
    return out


def complete_sample(n: int, seed: int, lat_max: int, self_max: int, loss_max: int, sources,
                    nthreads: int = 1, metric: int = 0):
    """Dense Dijkstra rows of the synthetic complete graph for the given sources (metric > 0: the
    metric graph of scale `metric` ms instead of U{1..lat_max}).
    Returns (lat_ns [k,n] u64, rel [k,n] f64, matrix_gen_seconds, sssp_seconds)."""
    L = lib()
    if not hasattr(L, "_cs_set"):
        for f in (L.orc_complete_sample, L.orc_metric_sample):
            f.restype = ctypes.c_int
            f.argtypes = [ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint32,
                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                          ctypes.c_int32, ctypes.c_int, ctypes.c_void_p,
                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_dense_weight.restype = ctypes.c_uint32
        L.orc_dense_weight.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        L._cs_set = True
    src = np.ascontiguousarray(sources, dtype=np.int32)
    k = len(src)
    lat = np.empty((k, n), np.uint64)
    rel = np.empty((k, n), np.float64)
    gs, ss = ctypes.c_double(), ctypes.c_double()
    fn, p = (L.orc_metric_sample, metric) if metric else (L.orc_complete_sample, lat_max)
    rc = fn(n, seed, p, self_max, loss_max, src.ctypes.data, k, nthreads,
            lat.ctypes.data, rel.ctypes.data, ctypes.byref(gs), ctypes.byref(ss))
    if rc:
        raise RuntimeError("orc_complete_sample failed")
    return lat, rel, gs.value, ss.value


def dense_weight(seed: int, lat_max: int, metric: int, self_max: int, i: int, j: int) -> int:
    """one weight (ms) of the synthetic dense generators (metric > 0: the metric graph)"""
    complete_sample(1, 0, 1, 1, 0, [0])  # binds the signatures
    return int(lib().orc_dense_weight(seed, lat_max, metric, self_max, i, j))
