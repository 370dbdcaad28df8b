"""TEST INFRASTRUCTURE ONLY -- the reference's lazy path cache, replayed in Python.

A literal restatement of /root/reference/src/main/routing/topology.c's lookup side over the
oracle's raw per-source rows (oracle.table(..., raw=True): entry (s, t) = what source s computes
for t, the diagonal rule on the diagonal, the direct edge in direct mode):

  _topology_getPathFromCache      topology.c:1166-1187
  _topology_shouldStorePath       topology.c:1189-1215
  _topology_storePathInCache      topology.c:1217-1265 (minimumPathLatency, :1253-1264)
  _topology_computeShortestPathToSelf  (store only)  topology.c:1573
  _topology_computeSourcePaths    (store loop)       topology.c:1604-1656, :1737-1798
  _topology_lookupDirectPath      (store only)       topology.c:1855
  _topology_getPathEntry          topology.c:1900-1981
  topology_incrementPathPacketCounter / getLatency / getReliability / isRoutable  :1983-2022
  topology_attach / topology_detach (the IP map and verticesWithAttachedHosts)     :2218-2281
  worker_sendPacket               worker.c:541-555

It is the checker for the product's pair-order layer (shadow_amd/csrc/pairorder.c), which decides
the same thing from per-vertex run stamps; nothing here is imported by the product.

One thing the restatement cannot reproduce: the order in which a source run visits its targets is
a GHashTable iteration order (:1401-1404). It changes only the sequence of intermediate
worker_updateMinTimeJump calls inside one run, not the minimum after the run, so `min_after`
(the topology's minimumPathLatency after each call) is what tests compare.
"""
from __future__ import annotations

import math


class Path:
    """path.c:13-38: latency (ms), reliability, packet count."""

    __slots__ = ("src", "dst", "latency", "reliability", "packets")

    def __init__(self, src, dst, latency, reliability):
        self.src, self.dst = src, dst
        self.latency, self.reliability, self.packets = latency, reliability, 0


class LazyPathCache:
    def __init__(self, raw: dict, directed: bool, use_shortest_path: bool = True):
        self.lat_ms = raw["lat_ms"]
        self.rel = raw["rel"]
        self.directed = bool(directed)
        self.use_shortest_path = bool(use_shortest_path)
        self.ip_to_vertex = {}           # virtualIP (:2225-2230)
        self.attached = []               # verticesWithAttachedHosts, insertion order
        self._attached_set = set()
        self.cache = {}                  # pathCache: src -> {dst: Path}
        self.minimum_path_latency = 0.0  # :1254
        self.exports = []                # worker_updateMinTimeJump arguments, in order
        self.source_runs = 0             # shortestPathCount (:1719)
        self.self_runs = 0               # selfPathCount (:1536)

    # -- attach / detach ------------------------------------------------------------------
    def attach(self, ip, vertex: int) -> None:
        self.ip_to_vertex[ip] = int(vertex)
        if vertex not in self._attached_set:  # g_hash_table_replace: one entry per vertex (:2231)
            self._attached_set.add(vertex)
            self.attached.append(int(vertex))

    def detach(self, ip) -> None:
        self.ip_to_vertex.pop(ip, None)  # verticesWithAttachedHosts keeps the vertex (:2274-2281)

    # -- cache ------------------------------------------------------------------------------
    def _get(self, s, d):
        src_cache = self.cache.get(s)
        return src_cache.get(d) if src_cache is not None else None

    def _should_store(self, is_direct, s, d) -> bool:
        if self._get(s, d) is not None or self._get(d, s) is not None:
            return False
        # :1204-1211 (a non-direct path while direct paths are wanted) needs
        # computeSourcePaths with use_shortest_path = false, which getPathEntry never calls
        assert is_direct or self.use_shortest_path
        return True

    def _store(self, is_direct, s, d, latency, reliability) -> None:
        if not self._should_store(is_direct, s, d):
            return
        self.cache.setdefault(s, {})[d] = Path(s, d, float(latency), float(reliability))
        if self.minimum_path_latency == 0 or latency < self.minimum_path_latency:
            self.minimum_path_latency = float(latency)
            self.exports.append(self.minimum_path_latency)

    def _compute_source(self, s, d) -> bool:
        if s == d:  # _topology_computeShortestPathToSelf
            self.self_runs += 1
            self._store(True, s, s, self.lat_ms[s, s], self.rel[s, s])
            return True
        self.source_runs += 1
        for t in list(self.attached):
            if t == s:  # a one-vertex result path: skipped (:1744-1753)
                continue
            latency = self.lat_ms[s, t]
            if math.isinf(latency):  # unreachable: igraph's empty path is skipped (:1744-1753)
                continue
            if latency == 0:  # :1787-1791
                latency = 1.0
            self._store(False, s, t, latency, self.rel[s, t])
        return True

    def _lookup_direct(self, s, d) -> bool:
        self._store(True, s, d, self.lat_ms[s, d], self.rel[s, d])
        return True

    def path_entry(self, src_ip, dst_ip):
        s = self.ip_to_vertex.get(src_ip, -1)
        if s < 0:
            return None
        d = self.ip_to_vertex.get(dst_ip, -1)
        if d < 0:
            return None
        path = self._get(s, d)
        if path is None and not self.directed:
            path = self._get(d, s)
        if path is None:
            if not self.use_shortest_path:
                ok = self._lookup_direct(s, d)
            else:
                ok = self._compute_source(s, d)
            if ok:
                path = self._get(s, d)
                if path is None:
                    path = self._get(d, s)
            if path is None:
                raise RuntimeError(f"unable to find path between vertex {s} and vertex {d}")
        return path

    # -- the lookup API ---------------------------------------------------------------------
    def get_latency(self, src_ip, dst_ip) -> float:
        p = self.path_entry(src_ip, dst_ip)
        return p.latency if p is not None else -1.0

    def get_reliability(self, src_ip, dst_ip) -> float:
        p = self.path_entry(src_ip, dst_ip)
        return p.reliability if p is not None else -1.0

    def is_routable(self, src_ip, dst_ip) -> bool:
        return self.get_latency(src_ip, dst_ip) > -1

    def increment(self, src_ip, dst_ip) -> None:
        p = self.path_entry(src_ip, dst_ip)
        if p is None:
            raise RuntimeError("unable to find path")
        p.packets += 1

    def packet_count(self, src_ip, dst_ip) -> int:
        """Count on the path a lookup would be served from, without computing anything."""
        s, d = self.ip_to_vertex.get(src_ip, -1), self.ip_to_vertex.get(dst_ip, -1)
        p = self._get(s, d)
        if p is None:  # directed too: a lookup that misses (s, d) is served (d, s) (:1963-1967)
            p = self._get(d, s)
        return p.packets if p is not None else 0

    def send_packet(self, src_ip, dst_ip, chance, bootstrapping=False, payload_length=1):
        """worker.c:541-555: (delivered, delay_ns)."""
        reliability = self.get_reliability(src_ip, dst_ip)
        if bootstrapping or chance <= reliability or payload_length == 0:
            latency = self.get_latency(src_ip, dst_ip)
            delay = int(math.ceil(latency * 1000000.0))
            self.increment(src_ip, dst_ip)
            return True, delay
        return False, None
