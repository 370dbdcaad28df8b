"""Seeded synthetic network graphs for the benchmark configurations and GML I/O.

All latencies are whole milliseconds (the constraint of the reference's own converter,
src/tools/convert_legacy_topology.py:23-27) and every vertex carries a self-loop so the diagonal
rule (topology.c:1431-1576) is exercised. packet_loss is k / 10000 so it round-trips through a
GML text exactly. The hash is shared bit-for-bit with the device generator in csrc/dense.hip.

  C1  complete, n=50,     latency U{1..300} ms, self U{1..10}, loss U{0..500}e-4, seed 1
  C2  complete, n=1000,   same distributions, seed 2
  C3  random geometric,   n=20000, radius sqrt(8/(pi n)), latency max(1, round(1000 d)) ms
  C4  complete, n=32768,  latency U{1..1000} ms, loss U{0..500}e-4, seed 4 (device generator)
  C5  Barabasi-Albert m=3, n=100000, latency U{1..100} ms, loss U{0..100}e-4, seed 5
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

MS = 1_000_000
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def hash_u64(seed: int, stream: int, i, j) -> np.ndarray:
    """srt_hash(seed, stream, i, j) of csrc/srt_device.h."""
    with np.errstate(over="ignore"):
        k = _splitmix64(np.uint64(seed) * np.uint64(4) + np.uint64(stream))
        ij = (np.asarray(i, dtype=np.uint64) << np.uint64(32)) | np.asarray(j, dtype=np.uint64)
        return _splitmix64(k ^ ij)


@dataclass
class Graph:
    n: int
    directed: bool
    src: np.ndarray     # int32, GML edge order
    dst: np.ndarray     # int32
    lat_ns: np.ndarray  # int64
    loss: np.ndarray    # float64
    name: str = ""

    @property
    def m(self) -> int:
        return len(self.src)


def complete_graph(n: int, seed: int, lat_max: int = 300, self_max: int = 10,
                   loss_max: int = 500, name: str = "") -> Graph:
    """Complete undirected graph with self-loops; edge (i, j), i <= j, in row order."""
    iu, ju = np.triu_indices(n)
    iu = iu.astype(np.uint64)
    ju = ju.astype(np.uint64)
    self_loop = iu == ju
    lat = np.where(self_loop,
                   np.uint64(1) + hash_u64(seed, 2, iu, ju) % np.uint64(self_max),
                   np.uint64(1) + hash_u64(seed, 0, iu, ju) % np.uint64(lat_max))
    k = np.where(self_loop, hash_u64(seed, 3, iu, ju), hash_u64(seed, 1, iu, ju)) % np.uint64(loss_max + 1)
    loss = k.astype(np.float64) / 10000.0
    return Graph(n, False, iu.astype(np.int32), ju.astype(np.int32),
                 lat.astype(np.int64) * MS, loss, name or f"complete{n}")


def complete_dense(n: int, seed: int, lat_max: int = 300, self_max: int = 10,
                   loss_max: int = 500):
    """Dense (w_ms u32, r f64) matrices of complete_graph, as srt_gen_complete_device fills them."""
    i = np.arange(n, dtype=np.uint64)[:, None]
    j = np.arange(n, dtype=np.uint64)[None, :]
    a = np.minimum(i, j)
    b = np.maximum(i, j)
    diag = a == b
    lat = np.where(diag, np.uint64(1) + hash_u64(seed, 2, a, b) % np.uint64(self_max),
                   np.uint64(1) + hash_u64(seed, 0, a, b) % np.uint64(lat_max))
    k = np.where(diag, hash_u64(seed, 3, a, b), hash_u64(seed, 1, a, b)) % np.uint64(loss_max + 1)
    return lat.astype(np.uint32), 1.0 - k.astype(np.float64) / 10000.0


def hub_leaf(n: int, hubs: int, seed: int, hub_max: int = 3, spoke: int = 5,
             loss_max: int = 500) -> Graph:
    """Hubs 0..hubs-1 joined to each other (U{1..hub_max} ms) and to every leaf (`spoke` ms); no
    leaf-leaf edges; every vertex with a self-loop. A hub reaches everything within `spoke` quanta,
    a leaf needs 2 * spoke for another leaf: row shards of hubs and of leaves settle their sources
    at different levels (tests/levels_protocol.py: on either side of the level build's batch)."""
    iu, ju = np.triu_indices(n)
    keep = (iu == ju) | (iu < hubs)
    iu, ju = iu[keep].astype(np.uint64), ju[keep].astype(np.uint64)
    self_loop = iu == ju
    lat = np.where(self_loop, np.uint64(1) + hash_u64(seed, 2, iu, ju) % np.uint64(10),
                   np.where(ju < np.uint64(hubs),
                            np.uint64(1) + hash_u64(seed, 0, iu, ju) % np.uint64(hub_max),
                            np.uint64(spoke)))
    k = hash_u64(seed, 1, iu, ju) % np.uint64(loss_max + 1)
    return Graph(n, False, iu.astype(np.int32), ju.astype(np.int32), lat.astype(np.int64) * MS,
                 k.astype(np.float64) / 10000.0, f"hubleaf{n}_{hubs}")


def dense_of(g: Graph):
    """(w_ms u32, r f64) matrices of a simple undirected whole-millisecond graph, the dense build's
    input form: SRT_INF (0x7FFFFFFF) and 0.0 where there is no edge, self-loops on the diagonal,
    r = 1.0 - loss (topology.c:396)."""
    assert not g.directed
    w = np.full((g.n, g.n), 0x7FFFFFFF, np.uint32)
    r = np.zeros((g.n, g.n))
    q = (g.lat_ns // MS).astype(np.uint32)
    assert np.all(q.astype(np.int64) * MS == g.lat_ns)
    w[g.src, g.dst] = q
    w[g.dst, g.src] = q
    r[g.src, g.dst] = 1.0 - g.loss
    r[g.dst, g.src] = 1.0 - g.loss
    return w, r


def _rand01(seed: int, stream: int, i) -> np.ndarray:
    return (hash_u64(seed, stream, i, 0) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def random_geometric(n: int, seed: int = 3, avg_degree: float = 8.0, loss_max: int = 100,
                     self_max: int = 10, name: str = "") -> Graph:
    """Random geometric graph in the unit square, components joined by their nearest pairs."""
    idx = np.arange(n, dtype=np.uint64)
    x = _rand01(seed, 4, idx)
    y = _rand01(seed, 5, idx)
    r = math.sqrt(avg_degree / (math.pi * n))
    cell = np.floor(x / r).astype(np.int64), np.floor(y / r).astype(np.int64)
    ncell = int(math.ceil(1.0 / r)) + 1
    key = cell[0] * ncell + cell[1]
    order = np.argsort(key, kind="stable")
    skey = key[order]
    starts = np.searchsorted(skey, np.arange(ncell * ncell), side="left")
    ends = np.searchsorted(skey, np.arange(ncell * ncell), side="right")
    src, dst = [], []
    for cx in range(ncell):
        for cy in range(ncell):
            c = cx * ncell + cy
            a = order[starts[c]:ends[c]]
            if len(a) == 0:
                continue
            for dx, dy in ((0, 0), (1, -1), (1, 0), (1, 1), (0, 1)):
                nx, ny = cx + dx, cy + dy
                if not (0 <= nx < ncell and 0 <= ny < ncell):
                    continue
                b = order[starts[nx * ncell + ny]:ends[nx * ncell + ny]]
                if len(b) == 0:
                    continue
                d2 = (x[a][:, None] - x[b][None, :]) ** 2 + (y[a][:, None] - y[b][None, :]) ** 2
                ii, jj = np.nonzero(d2 <= r * r)
                u, v = a[ii], b[jj]
                keep = u < v if (dx, dy) == (0, 0) else np.ones(len(u), bool)
                src.append(np.minimum(u, v)[keep])
                dst.append(np.maximum(u, v)[keep])
    src = np.concatenate(src) if src else np.zeros(0, np.int64)
    dst = np.concatenate(dst) if dst else np.zeros(0, np.int64)
    # join components: each non-giant component links its nearest vertex pair to the giant one
    parent = np.arange(n)

    def find(a):
        while parent[a] != a:
            parent[a] = parent[parent[a]]
            a = parent[a]
        return a

    for u, v in zip(src.tolist(), dst.tolist()):
        ru, rv = find(u), find(v)
        if ru != rv:
            parent[ru] = rv
    roots = np.array([find(v) for v in range(n)])
    labels, counts = np.unique(roots, return_counts=True)
    giant = labels[np.argmax(counts)]
    gmask = roots == giant
    gidx = np.nonzero(gmask)[0]
    extra_s, extra_d = [], []
    for lab in labels:
        if lab == giant:
            continue
        comp = np.nonzero(roots == lab)[0]
        d2 = (x[comp][:, None] - x[gidx][None, :]) ** 2 + (y[comp][:, None] - y[gidx][None, :]) ** 2
        ci, gi = np.unravel_index(np.argmin(d2), d2.shape)
        u, v = int(comp[ci]), int(gidx[gi])
        extra_s.append(min(u, v))
        extra_d.append(max(u, v))
    if extra_s:
        src = np.concatenate([src, np.array(extra_s)])
        dst = np.concatenate([dst, np.array(extra_d)])
    o = np.lexsort((dst, src))
    src, dst = src[o].astype(np.int64), dst[o].astype(np.int64)
    dist = np.sqrt((x[src] - x[dst]) ** 2 + (y[src] - y[dst]) ** 2)
    lat_ms = np.maximum(1, np.round(1000.0 * dist)).astype(np.int64)
    k = hash_u64(seed, 1, src.astype(np.uint64), dst.astype(np.uint64)) % np.uint64(loss_max + 1)
    loss = k.astype(np.float64) / 10000.0
    # self-loops first in each vertex's block is irrelevant to the semantics; append them
    sidx = np.arange(n, dtype=np.uint64)
    slat = (np.uint64(1) + hash_u64(seed, 2, sidx, sidx) % np.uint64(self_max)).astype(np.int64)
    sloss = (hash_u64(seed, 3, sidx, sidx) % np.uint64(loss_max + 1)).astype(np.float64) / 10000.0
    src = np.concatenate([src, np.arange(n)]).astype(np.int32)
    dst = np.concatenate([dst, np.arange(n)]).astype(np.int32)
    lat = np.concatenate([lat_ms, slat]) * MS
    loss = np.concatenate([loss, sloss])
    return Graph(n, False, src, dst, lat.astype(np.int64), loss, name or f"rgg{n}")


def directed_rgg(n: int, seed: int = 3, avg_degree: float = 8.0, loss_max: int = 100,
                 lat_max: int = 300, name: str = "") -> Graph:
    """random_geometric's structure with both orientations of every edge as separate directed
    edges of independent latency and loss (strongly connected), self-loops kept."""
    g = random_geometric(n, seed=seed, avg_degree=avg_degree, loss_max=loss_max)
    off = g.src != g.dst
    a, b = g.src[off].astype(np.uint64), g.dst[off].astype(np.uint64)
    src = np.concatenate([a, b, g.src[~off].astype(np.uint64)])
    dst = np.concatenate([b, a, g.dst[~off].astype(np.uint64)])
    lat = np.concatenate([(np.uint64(1) + hash_u64(seed, 7, src[:2 * len(a)], dst[:2 * len(a)])
                           % np.uint64(lat_max)).astype(np.int64) * MS, g.lat_ns[~off]])
    k = hash_u64(seed, 8, src[:2 * len(a)], dst[:2 * len(a)]) % np.uint64(loss_max + 1)
    loss = np.concatenate([k.astype(np.float64) / 10000.0, g.loss[~off]])
    return Graph(n, True, src.astype(np.int32), dst.astype(np.int32), lat, loss,
                 name or f"drgg{n}")


def complete_directed(n: int, seed: int, lat_max: int = 300, self_max: int = 10,
                      loss_max: int = 500, name: str = "") -> Graph:
    """Complete directed graph with self-loops: edge (i, j) for every ordered pair, i -> j and
    j -> i drawn independently (topology.c:409-511 calls it complete)."""
    i, j = np.meshgrid(np.arange(n, dtype=np.uint64), np.arange(n, dtype=np.uint64), indexing="ij")
    i, j = i.ravel(), j.ravel()
    self_loop = i == j
    lat = np.where(self_loop, np.uint64(1) + hash_u64(seed, 2, i, j) % np.uint64(self_max),
                   np.uint64(1) + hash_u64(seed, 9, i, j) % np.uint64(lat_max))
    k = hash_u64(seed, 10, i, j) % np.uint64(loss_max + 1)
    return Graph(n, True, i.astype(np.int32), j.astype(np.int32), lat.astype(np.int64) * MS,
                 k.astype(np.float64) / 10000.0, name or f"dcomplete{n}")


def barabasi_albert(n: int, m: int = 3, seed: int = 5, lat_max: int = 100, loss_max: int = 100,
                    self_max: int = 10, name: str = "") -> Graph:
    """Preferential attachment: clique on m+1 vertices, each new vertex links to m distinct
    existing vertices drawn proportionally to degree (hash-seeded)."""
    src, dst = [], []
    rep = []
    for a in range(m + 1):
        for b in range(a + 1, m + 1):
            src.append(a)
            dst.append(b)
            rep += [a, b]
    rep = list(rep)
    for v in range(m + 1, n):
        chosen = []
        k = 0
        while len(chosen) < m:
            h = int(hash_u64(seed, 6, v, k))
            k += 1
            t = rep[h % len(rep)]
            if t not in chosen:
                chosen.append(t)
        for t in chosen:
            src.append(t)
            dst.append(v)
            rep += [t, v]
    src = np.array(src, np.int64)
    dst = np.array(dst, np.int64)
    lat_ms = (1 + hash_u64(seed, 0, src.astype(np.uint64), dst.astype(np.uint64)) % np.uint64(lat_max)).astype(np.int64)
    k = hash_u64(seed, 1, src.astype(np.uint64), dst.astype(np.uint64)) % np.uint64(loss_max + 1)
    loss = k.astype(np.float64) / 10000.0
    sidx = np.arange(n, dtype=np.uint64)
    slat = (np.uint64(1) + hash_u64(seed, 2, sidx, sidx) % np.uint64(self_max)).astype(np.int64)
    sloss = (hash_u64(seed, 3, sidx, sidx) % np.uint64(loss_max + 1)).astype(np.float64) / 10000.0
    return Graph(n, False, np.concatenate([src, np.arange(n)]).astype(np.int32),
                 np.concatenate([dst, np.arange(n)]).astype(np.int32),
                 (np.concatenate([lat_ms, slat]) * MS).astype(np.int64),
                 np.concatenate([loss, sloss]), name or f"ba{n}")


def to_gml(g: Graph, ip_base: int | None = 0x0B000001, country: str | None = "US",
           bandwidth: str = "1 Gbit") -> str:
    """GML text in the format of /root/reference/docs/network_graph_spec.md:16-37."""
    out = ["graph [", f"  directed {1 if g.directed else 0}"]
    for v in range(g.n):
        out.append("  node [")
        out.append(f"    id {v}")
        if ip_base is not None:
            ip = ip_base + v
            out.append(f'    ip_address "{ip >> 24 & 255}.{ip >> 16 & 255}.{ip >> 8 & 255}.{ip & 255}"')
        if country is not None:
            out.append(f'    country_code "{country}"')
        out.append(f'    bandwidth_down "{bandwidth}"')
        out.append(f'    bandwidth_up "{bandwidth}"')
        out.append("  ]")
    lat_ms = g.lat_ns // MS
    whole = (g.lat_ns % MS) == 0
    for e in range(g.m):
        lat = f"{int(lat_ms[e])} ms" if whole[e] else f"{int(g.lat_ns[e])} ns"
        out.append("  edge [")
        out.append(f"    source {int(g.src[e])}")
        out.append(f"    target {int(g.dst[e])}")
        out.append(f'    latency "{lat}"')
        out.append(f"    packet_loss {repr(float(g.loss[e]))}")
        out.append("  ]")
    out.append("]")
    return "\n".join(out) + "\n"
