"""The canonical arc form (shadow_amd/csrc/graph.c srt_canon_build) on the CPU: one arc per
ordered vertex pair, the (minimum latency, lowest edge index) edge of that pair (topology.c:377-381
re-finds "an" edge with igraph_get_eid; the lowest index is the canonical choice), both
directions of an undirected edge, self-loops kept apart for the diagonal rule, columns ascending,
and for directed graphs the in-arc CSR as the transpose. Checked against a dictionary
restatement on random multigraphs (parallel edges with equal and unequal latencies, self-loops),
sparse rows (sorted path) and dense rows (the per-thread scratch path, n >= 4,096)."""
import ctypes

import numpy as np
import pytest

from shadow_amd import _lib


class Canon(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("directed", ctypes.c_int32),
                ("quantum_ns", ctypes.c_uint64), ("max_w_q", ctypes.c_uint32),
                ("dist_bound", ctypes.c_uint64), ("wide", ctypes.c_int32),
                ("arcs", ctypes.c_int64),
                ("rowptr", ctypes.POINTER(ctypes.c_int32)), ("col", ctypes.POINTER(ctypes.c_int32)),
                ("w", ctypes.POINTER(ctypes.c_uint32)), ("r", ctypes.POINTER(ctypes.c_double)),
                ("in_rowptr", ctypes.POINTER(ctypes.c_int32)),
                ("in_col", ctypes.POINTER(ctypes.c_int32)),
                ("in_w", ctypes.POINTER(ctypes.c_uint32)), ("in_r", ctypes.POINTER(ctypes.c_double)),
                ("self_w", ctypes.POINTER(ctypes.c_uint32)),
                ("self_r", ctypes.POINTER(ctypes.c_double)),
                ("edges", ctypes.c_void_p), ("verify_dense", ctypes.c_int32)]


def _canon(native, n, directed, src, dst, lat, loss):
    src = np.ascontiguousarray(src, np.int32)
    dst = np.ascontiguousarray(dst, np.int32)
    lat = np.ascontiguousarray(lat, np.int64)
    loss = np.ascontiguousarray(loss, np.float64)
    e = _lib.Edges(n, int(directed), len(src), src.ctypes.data, dst.ctypes.data, lat.ctypes.data,
                   loss.ctypes.data)
    c = Canon()
    native.srt_canon_build.restype = ctypes.c_int
    native.srt_canon_build.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert native.srt_canon_build(ctypes.byref(e), ctypes.byref(c)) == 0
    rp = np.ctypeslib.as_array(c.rowptr, (n + 1,)).copy()
    m = int(rp[-1])
    out = {"q": c.quantum_ns, "rp": rp,
           "col": np.ctypeslib.as_array(c.col, (max(m, 1),))[:m].copy(),
           "w": np.ctypeslib.as_array(c.w, (max(m, 1),))[:m].copy(),
           "r": np.ctypeslib.as_array(c.r, (max(m, 1),))[:m].copy(),
           "self_w": np.ctypeslib.as_array(c.self_w, (n,)).copy(),
           "self_r": np.ctypeslib.as_array(c.self_r, (n,)).copy(),
           "dist_bound": c.dist_bound, "wide": c.wide}
    if directed:
        irp = np.ctypeslib.as_array(c.in_rowptr, (n + 1,)).copy()
        out["irp"] = irp
        out["icol"] = np.ctypeslib.as_array(c.in_col, (max(m, 1),))[:m].copy()
        out["iw"] = np.ctypeslib.as_array(c.in_w, (max(m, 1),))[:m].copy()
    native.srt_canon_free.argtypes = [ctypes.c_void_p]
    native.srt_canon_free(ctypes.byref(c))
    return out


def _expect(n, directed, src, dst, lat, loss, q):
    best, selfb = {}, {}
    for e in range(len(src)):
        u, v, x = int(src[e]), int(dst[e]), int(lat[e])
        if u == v:
            if u not in selfb or x < selfb[u][0]:
                selfb[u] = (x, e)
            continue
        for a, b in ((u, v),) + (() if directed else ((v, u),)):
            if (a, b) not in best or x < best[(a, b)][0]:
                best[(a, b)] = (x, e)
    return best, selfb


@pytest.mark.parametrize("n,m,directed,dense", [(60, 400, False, False), (60, 400, True, False),
                                                 (4100, 0, False, True), (4100, 0, True, True)])
def test_canonical_arcs_match_restatement(native, n, m, directed, dense):
    rng = np.random.default_rng(n + m + directed)
    if dense:  # complete-ish rows (the scratch path) plus parallel edges and self-loops
        i = np.repeat(np.arange(40), n)
        j = np.tile(np.arange(n), 40)
        extra = rng.integers(0, 40, 3000), rng.integers(0, n, 3000)
        src = np.concatenate([i, extra[0], np.arange(n)])
        dst = np.concatenate([j, extra[1], np.arange(n)])
    else:
        src = rng.integers(0, n, m)
        dst = rng.integers(0, n, m)
    lat = rng.integers(1, 6, len(src)) * 1_000_000
    loss = rng.integers(0, 100, len(src)) / 10000.0
    got = _canon(native, n, directed, src, dst, lat, loss)
    best, selfb = _expect(n, directed, src, dst, lat, loss, got["q"])
    assert got["q"] == 1_000_000
    rows = {}
    for (a, b), (x, e) in best.items():
        rows.setdefault(a, []).append((b, x // 1_000_000, 1.0 - loss[e]))
    for u in range(n):
        want = sorted(rows.get(u, []))
        s, t = got["rp"][u], got["rp"][u + 1]
        have = list(zip(got["col"][s:t].tolist(), got["w"][s:t].tolist(), got["r"][s:t].tolist()))
        assert have == want, u
        if u in selfb:
            assert got["self_w"][u] == selfb[u][0] // 1_000_000
            assert got["self_r"][u] == 1.0 - loss[selfb[u][1]]
        else:
            assert got["self_w"][u] == 0x7FFFFFFF
    if directed:  # the in-arc CSR is the transpose, sources ascending
        for v in range(0, n, max(1, n // 50)):
            s, t = got["irp"][v], got["irp"][v + 1]
            want = sorted((a, x // 1_000_000) for (a, b), (x, e) in best.items() if b == v)
            assert list(zip(got["icol"][s:t].tolist(), got["iw"][s:t].tolist())) == want
