"""Python mirror of Shadow's routing interface (include/topology.h), over the C-ABI.

Method names follow /root/reference/src/main/routing/topology.h:17-28 so the parity tests read
like the reference's call sites (controller.c:173, host.c:172, worker.c:542-554):

    top = Topology.new(path, use_shortest_path=True)        # topology_new
    top.attach(ip, rand_state, ip_hint, city, country)      # topology_attach
    top.get_latency(src_ip, dst_ip)                         # topology_getLatency (ms, -1)
    top.get_reliability(src_ip, dst_ip)                     # topology_getReliability
    top.is_routable(src_ip, dst_ip)                         # topology_isRoutable
    top.increment_path_packet_counter(src_ip, dst_ip)       # topology_incrementPathPacketCounter
    top.compute_shortest_paths()                            # eager GPU build (addition)
    top.table()                                             # zero-copy (lat_ns, rel) view

IPs are dotted strings or network-order u32, as Address.ip is (address.c:23-25).
"""
from __future__ import annotations

import ctypes
import socket
import struct

import numpy as np

from . import _lib
from ._lib import BuildOpts, BuildStats, Edges, check, lib


def ip_to_net(ip) -> int:
    """dotted string -> network-order u32 as stored in Address (inet_pton semantics)."""
    if isinstance(ip, (int, np.integer)):
        return int(ip)
    return struct.unpack("=I", socket.inet_aton(ip))[0]


class Topology:
    def __init__(self, handle: int):
        if not handle:
            raise ValueError("topology_new failed (see the [shadow-routing] log)")
        self._h = ctypes.c_void_p(handle)
        self._keep = []

    # -- construction ------------------------------------------------------------------------
    @classmethod
    def new(cls, graph_path: str, use_shortest_path: bool = True) -> "Topology":
        return cls(lib().topology_new(graph_path.encode(), int(bool(use_shortest_path))))

    @classmethod
    def from_gml(cls, text: str, use_shortest_path: bool = True) -> "Topology":
        return cls(lib().srt_topology_new_from_string(text.encode(), int(bool(use_shortest_path))))

    @staticmethod
    def try_from_gml(text: str, use_shortest_path: bool = True):
        h = lib().srt_topology_new_from_string(text.encode(), int(bool(use_shortest_path)))
        return Topology(h) if h else None

    def free(self) -> None:
        if self._h:
            lib().topology_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    # -- graph facts ---------------------------------------------------------------------------
    @property
    def n(self) -> int:
        return lib().srt_topology_vertex_count(self._h)

    @property
    def m(self) -> int:
        return lib().srt_topology_edge_count(self._h)

    @property
    def directed(self) -> bool:
        return bool(lib().srt_topology_is_directed(self._h))

    @property
    def complete(self) -> bool:
        return bool(lib().srt_topology_is_complete(self._h))

    def edges(self):
        e = Edges()
        check(lib().srt_topology_edges(self._h, ctypes.byref(e)), "srt_topology_edges")
        m = e.m
        def arr(ptr, ct, dt):
            if m == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), (m,)).astype(dt)
        return (e.n, bool(e.directed), arr(e.src, ctypes.c_int32, np.int32),
                arr(e.dst, ctypes.c_int32, np.int32), arr(e.lat_ns, ctypes.c_int64, np.int64),
                arr(e.loss, ctypes.c_double, np.float64))

    # -- attach --------------------------------------------------------------------------------
    def attach(self, ip, rand_state: int = 1, ip_hint=None, city_hint=None, country_hint=None):
        """Returns (vertex, bw_down_KiB, bw_up_KiB, new_rand_state)."""
        st = ctypes.c_uint32(rand_state)
        down, up = ctypes.c_uint64(0), ctypes.c_uint64(0)
        enc = lambda s: None if s is None else s.encode()
        v = lib().srt_topology_attach_ip(self._h, ip_to_net(ip), ctypes.byref(st), enc(ip_hint),
                                         enc(city_hint), enc(country_hint), ctypes.byref(down),
                                         ctypes.byref(up))
        if v < 0:
            check(v, "attach")
        return v, down.value, up.value, st.value

    def attach_batch(self, ips, rand_states, ip_hints=None, city_hints=None, country_hints=None):
        """Attach many hosts in order (srt_topology_attach_batch_ip). Returns (vertices, bw_down,
        bw_up, new_rand_states) as numpy arrays."""
        h = len(ips)
        ipn = np.array([ip_to_net(x) for x in ips], dtype=np.uint32)
        st = np.ascontiguousarray(np.asarray(rand_states, dtype=np.uint32).copy())
        out = np.zeros(h, dtype=np.int32)
        down = np.zeros(h, dtype=np.uint64)
        up = np.zeros(h, dtype=np.uint64)

        def strs(a):
            if a is None:
                return None
            arr = (ctypes.c_char_p * h)()
            for i, x in enumerate(a):
                arr[i] = None if x is None else x.encode()
            return arr

        hints = [strs(ip_hints), strs(city_hints), strs(country_hints)]
        ptr = lambda x: x.ctypes.data_as(ctypes.c_void_p)
        r = lib().srt_topology_attach_batch_ip(self._h, h, ptr(ipn), ptr(st), *hints, ptr(out),
                                               ptr(down), ptr(up))
        if r < 0:
            check(r, "attach_batch")
        return out, down, up, st

    def detach(self, ip) -> None:
        lib().srt_topology_detach_ip(self._h, ip_to_net(ip))

    def vertex_of(self, ip) -> int:
        return lib().srt_topology_vertex_of_ip(self._h, ip_to_net(ip))

    # -- build + lookups -----------------------------------------------------------------------
    def set_build_opts(self, device=0, algo=_lib.ALGO_AUTO, fw_block=0) -> None:
        o = BuildOpts(device, algo, 1, fw_block)
        lib().srt_topology_set_build_opts(self._h, ctypes.byref(o))

    def compute_shortest_paths(self, n_gpus: int = 1) -> None:
        check(lib().topology_computeShortestPaths(self._h, n_gpus), "topology_computeShortestPaths")

    def stats(self) -> BuildStats:
        s = BuildStats()
        check(lib().srt_topology_last_stats(self._h, ctypes.byref(s)), "stats")
        return s

    def table(self):
        """(lat_ns u64 [k,k], rel f64 [k,k]) copies of the current tables over their k vertices
        (table_vertices(); every vertex while nothing is attached)."""
        latp = ctypes.c_void_p()
        relp = ctypes.c_void_p()
        q = ctypes.c_uint64()
        n = ctypes.c_int()
        check(lib().topology_getTable(self._h, ctypes.byref(latp), ctypes.byref(q),
                                      ctypes.byref(relp), ctypes.byref(n)), "topology_getTable")
        nn = n.value
        lat = np.ctypeslib.as_array(ctypes.cast(latp, ctypes.POINTER(ctypes.c_uint32)), (nn, nn))
        rel = np.ctypeslib.as_array(ctypes.cast(relp, ctypes.POINTER(ctypes.c_double)), (nn, nn))
        return lat.astype(np.uint64) * np.uint64(q.value), rel.copy()

    def table_vertices(self):
        """(vertices int32 [k], lat_ms f64 [k,k] or None) of the current tables."""
        vp, mp = ctypes.c_void_p(), ctypes.c_void_p()
        k = ctypes.c_int32()
        check(lib().srt_topology_table_info(self._h, ctypes.byref(vp), ctypes.byref(k),
                                            ctypes.byref(mp)), "srt_topology_table_info")
        kk = k.value
        verts = np.ctypeslib.as_array(ctypes.cast(vp, ctypes.POINTER(ctypes.c_int32)), (kk,)).copy()
        ms = None
        if mp.value:
            ms = np.ctypeslib.as_array(ctypes.cast(mp, ctypes.POINTER(ctypes.c_double)),
                                       (kk, kk)).copy()
        return verts, ms

    def get_latency(self, src, dst) -> float:
        return lib().srt_topology_latency_ip(self._h, ip_to_net(src), ip_to_net(dst))

    def get_reliability(self, src, dst) -> float:
        return lib().srt_topology_reliability_ip(self._h, ip_to_net(src), ip_to_net(dst))

    def is_routable(self, src, dst) -> bool:
        return self.get_latency(src, dst) > -1

    def increment_path_packet_counter(self, src, dst) -> None:
        check(lib().srt_topology_increment_ip(self._h, ip_to_net(src), ip_to_net(dst)),
              "topology_incrementPathPacketCounter")

    def packet_count(self, src, dst) -> int:
        return lib().srt_topology_packet_count_ip(self._h, ip_to_net(src), ip_to_net(dst))

    def path_source(self, src, dst) -> int:
        """Vertex whose source run stored the path a lookup (src, dst) is served from (-1: none
        yet); the lazy-cache order of topology.c:1189-1215, :1900-1981."""
        return lib().srt_topology_path_source_ip(self._h, ip_to_net(src), ip_to_net(dst))

    def path_counts(self) -> dict:
        """The reference's diagnostics (topology.c:78-79, logged at :1142-1164): lookups that
        would have run a source's Dijkstra, self paths computed, and the table builds run here
        with their device seconds."""
        sp, sf, nb, sec = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int32(), ctypes.c_double()
        check(lib().srt_topology_path_counts(self._h, ctypes.byref(sp), ctypes.byref(sf),
                                             ctypes.byref(nb), ctypes.byref(sec)),
              "srt_topology_path_counts")
        return {"shortest_paths": sp.value, "self_paths": sf.value, "builds": nb.value,
                "build_seconds": sec.value}

    def send_packet(self, src, dst, chance: float, bootstrapping: bool = False,
                    payload_length: int = 1):
        """worker_sendPacket's decision (worker.c:541-555): (delivered, delay_ns or None)."""
        d = ctypes.c_uint64(0)
        r = lib().srt_topology_send_packet_ip(self._h, ip_to_net(src), ip_to_net(dst),
                                              float(chance), int(bool(bootstrapping)),
                                              int(payload_length), ctypes.byref(d))
        if r < 0:
            check(r, "send_packet")
        return (True, d.value) if r == 1 else (False, None)

    def send_packets(self, src_net, dst_net, chance, bootstrapping=None, payload_length=None):
        """Trace replay: network-order u32 IP arrays -> (delivered bool[k], delay_ns u64[k])."""
        src = np.ascontiguousarray(src_net, np.uint32)
        dst = np.ascontiguousarray(dst_net, np.uint32)
        ch = np.ascontiguousarray(chance, np.float64)
        k = len(src)
        boot = None if bootstrapping is None else np.ascontiguousarray(bootstrapping, np.uint8)
        pay = None if payload_length is None else np.ascontiguousarray(payload_length, np.uint64)
        out = np.zeros(k, np.uint8)
        delay = np.zeros(k, np.uint64)
        ptr = lambda a: None if a is None else a.ctypes.data
        check(lib().srt_topology_send_packets_ip(self._h, k, ptr(src), ptr(dst), ptr(ch),
                                                 ptr(boot), ptr(pay), ptr(out), ptr(delay)),
              "send_packets")
        return out.astype(bool), delay

    def min_latency_ms(self) -> float:
        return lib().srt_topology_min_latency_ms(self._h)


MIN_HOOK = ctypes.CFUNCTYPE(None, ctypes.c_double)


def set_min_time_jump_hook(fn):
    """Route the runahead export (worker_updateMinTimeJump) to fn(ms); None restores it. Returns
    the ctypes callback, which the caller must keep alive while it is installed."""
    cb = MIN_HOOK(fn) if fn is not None else None
    lib().srt_set_min_time_jump_hook(ctypes.cast(cb, ctypes.c_void_p) if cb else None)
    return cb


def parse_time_nanosec(s: str) -> int:
    return lib().srt_parse_time_nanosec(s.encode())


def parse_bandwidth(s: str) -> int:
    return lib().srt_parse_bandwidth(s.encode())


def build_tables_subset(n, directed, src, dst, lat_ns, loss, verts=None, use_shortest_path=True,
                        device=0, algo=_lib.ALGO_AUTO, ngpus=1, want_ms=False):
    """srt_build_tables_subset -> (lat_ns u64 [k,k], rel f64 [k,k], lat_ms f64 [k,k] or None,
    min_lat_ns, stats) over the vertices `verts` (increasing; None = all)."""
    src = np.ascontiguousarray(src, np.int32)
    dst = np.ascontiguousarray(dst, np.int32)
    lat_ns = np.ascontiguousarray(lat_ns, np.int64)
    loss = np.ascontiguousarray(loss, np.float64)
    e = Edges(n, int(bool(directed)), len(src), src.ctypes.data, dst.ctypes.data,
              lat_ns.ctypes.data, loss.ctypes.data)
    o = BuildOpts(device, algo, int(bool(use_shortest_path)), 0)
    vv = None if verts is None else np.ascontiguousarray(verts, np.int32)
    k = n if vv is None else len(vv)
    lat = np.empty((k, k), np.uint32)
    rel = np.empty((k, k), np.float64)
    ms = np.empty((k, k), np.float64) if want_ms else None
    q = ctypes.c_uint64()
    mn = ctypes.c_uint32()
    st = BuildStats()
    check(lib().srt_build_tables_subset(ctypes.byref(e), ctypes.byref(o), int(ngpus), k,
                                        None if vv is None else vv.ctypes.data, lat.ctypes.data,
                                        ctypes.byref(q), rel.ctypes.data,
                                        None if ms is None else ms.ctypes.data, ctypes.byref(mn),
                                        ctypes.byref(st)), "srt_build_tables_subset")
    return lat.astype(np.uint64) * np.uint64(q.value), rel, ms, int(mn.value) * q.value, st


def build_tables(n, directed, src, dst, lat_ns, loss, use_shortest_path=True, device=0,
                 algo=_lib.ALGO_AUTO, ngpus=None):
    """srt_build_tables on host arrays -> (lat_ns u64 [n,n], rel f64 [n,n], stats).
    ngpus: run srt_build_tables_multi (one host thread per GPU of this process, RCCL)."""
    src = np.ascontiguousarray(src, np.int32)
    dst = np.ascontiguousarray(dst, np.int32)
    lat_ns = np.ascontiguousarray(lat_ns, np.int64)
    loss = np.ascontiguousarray(loss, np.float64)
    e = Edges(n, int(bool(directed)), len(src), src.ctypes.data, dst.ctypes.data,
              lat_ns.ctypes.data, loss.ctypes.data)
    o = BuildOpts(device, algo, int(bool(use_shortest_path)), 0)
    lat = np.empty((n, n), np.uint32)
    rel = np.empty((n, n), np.float64)
    q = ctypes.c_uint64()
    st = BuildStats()
    if ngpus is None:
        check(lib().srt_build_tables(ctypes.byref(e), ctypes.byref(o), lat.ctypes.data,
                                     ctypes.byref(q), rel.ctypes.data, ctypes.byref(st)),
              "srt_build_tables")
    else:
        check(lib().srt_build_tables_multi(ctypes.byref(e), ctypes.byref(o), int(ngpus),
                                           lat.ctypes.data, ctypes.byref(q), rel.ctypes.data,
                                           ctypes.byref(st)), "srt_build_tables_multi")
    return lat.astype(np.uint64) * np.uint64(q.value), rel, st


class SparseGraph:
    """Device-resident canonical CSR (srt_sparse_graph_*): rows of any source range are computed
    on the device into caller-provided device buffers (torch tensors or raw pointers)."""

    def __init__(self, n, directed, src, dst, lat_ns, loss, device=0):
        self._keep = [np.ascontiguousarray(src, np.int32), np.ascontiguousarray(dst, np.int32),
                      np.ascontiguousarray(lat_ns, np.int64), np.ascontiguousarray(loss, np.float64)]
        s, d, l, p = self._keep
        e = Edges(n, int(bool(directed)), len(s), s.ctypes.data, d.ctypes.data, l.ctypes.data,
                  p.ctypes.data)
        h = ctypes.c_void_p()
        check(lib().srt_sparse_graph_new(ctypes.byref(e), device, ctypes.byref(h)),
              "srt_sparse_graph_new")
        self._h = h
        self._keep = None
        nn, dd, aa, qq = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_uint64()
        check(lib().srt_sparse_graph_info(h, ctypes.byref(nn), ctypes.byref(dd), ctypes.byref(aa),
                                          ctypes.byref(qq)), "srt_sparse_graph_info")
        self.n, self.directed, self.arcs, self.quantum_ns = nn.value, bool(dd.value), aa.value, qq.value

    def rows(self, src_begin, src_end, lat_ptr, rel_ptr, stream=None, stats=None):
        """srt_sparse_graph_rows into device pointers (row stride n)."""
        st = ctypes.byref(stats) if stats is not None else None
        check(lib().srt_sparse_graph_rows(self._h, src_begin, src_end, ctypes.c_void_p(lat_ptr),
                                          ctypes.c_void_p(rel_ptr), ctypes.c_void_p(stream), st),
              "srt_sparse_graph_rows")

    def rows_list(self, srcs_ptr, nsrc, lat_ptr, rel_ptr, stream=None, stats=None):
        """srt_sparse_graph_rows_list: row i of the device buffers is source srcs[i] (a device
        int32 array of nsrc vertices)."""
        st = ctypes.byref(stats) if stats is not None else None
        check(lib().srt_sparse_graph_rows_list(self._h, int(nsrc), ctypes.c_void_p(srcs_ptr),
                                               ctypes.c_void_p(lat_ptr), ctypes.c_void_p(rel_ptr),
                                               None, ctypes.c_void_p(stream), st),
              "srt_sparse_graph_rows_list")

    def free(self):
        if getattr(self, "_h", None):
            lib().srt_sparse_graph_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
