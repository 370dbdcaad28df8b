"""Drive tools/msssp_sim.c: pulls per vertex and passes per 64-source batch of the multi-source
SSSP on the bench graphs, and a check of its tables against oracle/ (test infrastructure).

python tools/msssp_sim.py c3 --delta 16 --batches 4 [--jacobi] [--check]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from shadow_amd import graphs  # noqa: E402

SO = "/tmp/libmsssp_sim.so"


class Counts(ctypes.Structure):
    _fields_ = [("pulls", ctypes.c_int64), ("passes", ctypes.c_int64),
                ("buckets", ctypes.c_int64), ("arcs", ctypes.c_int64),
                ("hub_arcs", ctypes.c_int64), ("hub_pulls", ctypes.c_int64)]


def load():
    src = os.path.join(os.path.dirname(__file__), "msssp_sim.c")
    subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", src, "-o", SO])
    return ctypes.CDLL(SO)


def csr(g):
    off = g.src != g.dst
    s = np.concatenate([g.src[off], g.dst[off]]) if not g.directed else g.src[off]
    d = np.concatenate([g.dst[off], g.src[off]]) if not g.directed else g.dst[off]
    lat = np.concatenate([g.lat_ns[off], g.lat_ns[off]]) if not g.directed else g.lat_ns[off]
    loss = np.concatenate([g.loss[off], g.loss[off]]) if not g.directed else g.loss[off]
    # canonical arc per ordered pair: (min latency, lowest edge index); r = 1.0 - loss, a full
    # double (no spare mantissa bits to carry other data)
    eidx = np.concatenate([np.nonzero(off)[0]] * (1 if g.directed else 2))
    o = np.lexsort((eidx, lat, d, s))
    s, d, lat, loss = s[o], d[o], lat[o], loss[o]
    keep = np.ones(len(s), bool)
    keep[1:] = (s[1:] != s[:-1]) | (d[1:] != d[:-1])
    s, d, lat, loss = s[keep], d[keep], lat[keep], loss[keep]
    q = np.gcd.reduce(lat)
    w = (lat // q).astype(np.uint32)
    r = 1.0 - loss
    n = g.n
    oi = np.lexsort((s, d))  # in-arcs grouped by head, sorted by tail
    irp = np.searchsorted(d[oi], np.arange(n + 1)).astype(np.int32)
    oo = np.lexsort((d, s))
    orp = np.searchsorted(s[oo], np.arange(n + 1)).astype(np.int32)
    return (n, irp, s[oi].astype(np.int32), w[oi], r[oi], orp, d[oo].astype(np.int32))


def clusters(n, orp, ocol, size=64):
    import scipy.sparse as sp
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    rows = np.repeat(np.arange(n), np.diff(orp))
    A = sp.csr_matrix((np.ones(len(ocol)), (rows, ocol)), shape=(n, n))
    perm = reverse_cuthill_mckee(A, symmetric_mode=True)
    done = np.zeros(n, bool)
    out = []
    for seed in perm:
        if done[seed]:
            continue
        cl, q, h = [seed], [seed], 0
        done[seed] = True
        while len(cl) < size and h < len(q):
            u = q[h]
            h += 1
            for v in ocol[orp[u]:orp[u + 1]]:
                if not done[v] and len(cl) < size:
                    done[v] = True
                    cl.append(v)
                    q.append(v)
        out.append(np.array(cl, np.int32))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("graph")
    ap.add_argument("--delta", type=int, default=16)
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--jacobi", action="store_true")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--n", type=int, default=0)
    a = ap.parse_args()
    if a.graph == "c3":
        g = graphs.random_geometric(a.n or 20000, seed=3)
    elif a.graph == "c5":
        g = graphs.barabasi_albert(a.n or 100000, m=3, seed=5)
    elif a.graph == "drgg":
        g = graphs.directed_rgg(a.n or 3000, seed=7)
    else:
        raise SystemExit("graph: c3 | c5 | drgg")
    L = load()
    n, irp, icol, iw, ir, orp, ocol = csr(g)
    cl = clusters(n, orp, ocol)
    rng = np.random.default_rng(0)
    pick = rng.choice(len(cl), min(a.batches, len(cl)), replace=False)
    tp = tq = 0
    for ci in pick:
        srcs = cl[ci]
        D = np.empty((64, n), np.uint32)
        R = np.empty((64, n), np.float64)
        c = Counts()
        P = ctypes.c_void_p
        rc = L.msssp_sim_batch(n, P(irp.ctypes.data), P(icol.ctypes.data), P(iw.ctypes.data),
                               P(ir.ctypes.data), P(orp.ctypes.data), P(ocol.ctypes.data),
                               len(srcs), P(srcs.ctypes.data), ctypes.c_uint32(a.delta),
                               int(a.jacobi), P(D.ctypes.data), P(R.ctypes.data), ctypes.byref(c))
        assert rc == 0
        tp += c.pulls
        tq += c.passes
        line = (f"batch {ci}: pulls/n {c.pulls / n:.2f} passes {c.passes} buckets {c.buckets} "
                f"arcs/arcs {c.arcs / len(icol):.2f} (in-degree > 64: {c.hub_pulls} pulls, "
                f"{c.hub_arcs / len(icol):.2f} arcs/arcs)")
        if a.check:
            import oracle
            e = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
            ref = oracle.sssp_list(e, srcs)
            k = len(srcs)
            q = int(np.gcd.reduce(g.lat_ns[g.lat_ns > 0]))
            lat = ref["lat_int"] // q
            mask = np.ones((k, n), bool)
            mask[np.arange(k), srcs] = False  # the diagonal follows its own rule
            dd = D[:k].astype(np.uint64)
            dd[D[:k] == 0xFFFFFFFF] = np.uint64(0xFFFFFFFFFFFFFFFF)
            reach = ref["lat_int"] != np.uint64(0xFFFFFFFFFFFFFFFF)
            okd = np.array_equal(dd[mask & reach], lat[mask & reach])
            okr = np.array_equal(R[:k][mask].view(np.uint64), ref["rel"][mask].view(np.uint64))
            line += f" | lat exact {okd} rel bit-exact {okr}"
        print(line, flush=True)
    print(f"{a.graph} delta {a.delta} jacobi {int(a.jacobi)}: mean pulls/n {tp / len(pick) / n:.2f} "
          f"passes {tq / len(pick):.1f}")


if __name__ == "__main__":
    main()
