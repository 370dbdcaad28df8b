"""ctypes binding of libshadow_routing.so (the C-ABI in include/shadow_routing.h, topology.h).

The library is built in-tree (shadow_amd/libshadow_routing.so) by `make -C shadow_amd/csrc`
or __graft_entry__.build(). Loading fails loudly when it is missing: there is no Python or CPU
fallback for any routing computation.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# SRT_LIB_PATH: a side-by-side build of the same sources (tools: A/B of build-time variants)
LIB_PATH = os.environ.get("SRT_LIB_PATH") or os.path.join(_HERE, "libshadow_routing.so")
CSRC = os.path.join(_HERE, "csrc")

SRT_OK = 0
SRT_INF = 0x7FFFFFFF
ALGO_AUTO, ALGO_DENSE_FW, ALGO_SPARSE_SSSP = 0, 1, 2

ERRORS = {
    -1: "SRT_E_ARG", -2: "SRT_E_PARSE", -3: "SRT_E_INVALID", -4: "SRT_E_NOMEM",
    -5: "SRT_E_DEVICE", -6: "SRT_E_RANGE", -7: "SRT_E_COMM", -8: "SRT_E_NOPATH",
    -9: "SRT_E_UNATTACHED",
}


class Edges(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int32),
        ("directed", ctypes.c_int32),
        ("m", ctypes.c_int64),
        ("src", ctypes.c_void_p),
        ("dst", ctypes.c_void_p),
        ("lat_ns", ctypes.c_void_p),
        ("loss", ctypes.c_void_p),
    ]


class BuildOpts(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("algo", ctypes.c_int32),
        ("use_shortest_path", ctypes.c_int32),
        ("fw_block", ctypes.c_int32),
    ]


class BuildStats(ctypes.Structure):
    _fields_ = [
        ("time_kernels", ctypes.c_int32),
        ("algo", ctypes.c_int32),
        ("fw_block", ctypes.c_int32),
        ("ess_arcs", ctypes.c_int64),
        ("ms_total", ctypes.c_double),
        ("ms_fw", ctypes.c_double),
        ("ms_post", ctypes.c_double),
        ("max_depth", ctypes.c_int32),
        ("n_update", ctypes.c_int32),
        ("ms_update", ctypes.c_double),
        ("ms_comm", ctypes.c_double),
        ("dist_enc", ctypes.c_int32),
        ("count_ties", ctypes.c_int32),
        ("tied_pairs", ctypes.c_int64),
        ("levels", ctypes.c_int32),
        ("work_bytes", ctypes.c_int64),
        ("ms_pred", ctypes.c_double),
        ("ms_rel", ctypes.c_double),
        ("n_derived", ctypes.c_int32),
        ("ms_core", ctypes.c_double),
        ("ms_derive", ctypes.c_double),
        ("rel_table", ctypes.c_int32),
        ("ms_canon", ctypes.c_double),
        ("ms_upload", ctypes.c_double),
        ("ms_download", ctypes.c_double),
    ]


# (name, restype, argtypes) for every exported symbol of the C-ABI
_VP, _I32, _I64, _U32, _U64, _D, _CP = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                         ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double,
                                         ctypes.c_char_p)
SIGNATURES = {
    # shadow_routing.h
    "srt_parse_time_nanosec": (_I64, [_CP]),
    "srt_parse_bandwidth": (_I64, [_CP]),
    "srt_build_tables": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP]),
    "srt_build_tables_multi": (ctypes.c_int, [_VP, _VP, _I32, _VP, _VP, _VP, _VP]),
    "srt_build_tables_subset": (ctypes.c_int, [_VP, _VP, _I32, _I32, _VP, _VP, _VP, _VP, _VP, _VP,
                                               _VP]),
    "srt_dense_max_n": (ctypes.c_int, []),
    "srt_latency_quantum": (ctypes.c_int, [_VP, _VP, _VP]),
    "srt_dense_build_device": (ctypes.c_int, [_I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP, _I32, _VP]),
    "srt_dense_rows_build": (ctypes.c_int, [_I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    "srt_gen_complete_device": (ctypes.c_int, [_I32, _I32, _I32, _I32, _U64, _U32, _U32, _U32,
                                                _VP, _VP, _VP]),
    "srt_gen_metric_device": (ctypes.c_int, [_I32, _I32, _I32, _I32, _U64, _U32, _U32, _U32,
                                              _VP, _VP, _VP]),
    "srt_sparse_max_n": (ctypes.c_int, []),
    "srt_sparse_build_device": (ctypes.c_int, [_I32, _I32, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP,
                                               _VP, _VP, _I32, _I32, _U32, _VP, _VP, _VP, _VP]),
    "srt_sparse_graph_new": (ctypes.c_int, [_VP, _I32, _VP]),
    "srt_sparse_graph_info": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
    "srt_sparse_graph_rows": (ctypes.c_int, [_VP, _I32, _I32, _VP, _VP, _VP, _VP]),
    "srt_sparse_graph_rows_list": (ctypes.c_int, [_VP, _I32, _VP, _VP, _VP, _VP, _VP, _VP]),
    "srt_sparse_graph_free": (None, [_VP]),
    "srt_comm_unique_id": (ctypes.c_int, [_VP]),
    "srt_comm_init": (ctypes.c_int, [_VP, _I32, _I32, _I32, _VP]),
    "srt_comm_init_all": (ctypes.c_int, [_I32, _VP, _VP]),
    "srt_comm_init_virtual": (ctypes.c_int, [_I32, _I32, _VP]),
    "srt_comm_init_solo": (ctypes.c_int, [_I32, _I32, _I32, _VP]),
    "srt_comm_init_solo_wire": (ctypes.c_int, [_I32, _I32, _I32, _D, _D, _VP]),
    "srt_comm_wire_ms": (_D, [_VP]),
    "srt_comm_log_enable": (ctypes.c_int, [_VP, _I32]),
    "srt_comm_log_read": (_I64, [_VP, _VP, _I64]),
    "srt_comm_count": (ctypes.c_int, [_VP, _VP]),
    "srt_virtual_rank_bind": (ctypes.c_int, [_I32, _I32]),
    "srt_comm_free": (None, [_VP]),
    "srt_shard_rows": (None, [_I32, _I32, _I32, _I32, _VP, _VP]),
    "srt_dense_build_sharded": (ctypes.c_int, [_VP, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP,
                                               _I32, _VP]),
    "srt_sparse_allgather": (ctypes.c_int, [_VP, _I32, _I32, _VP, _VP, _VP]),
    "srt_version": (_CP, []),
    "srt_last_error": (_CP, []),
    "srt_pair_order_new": (_VP, [_I32, _I32, _I32]),
    "srt_pair_order_free": (None, [_VP]),
    "srt_pair_order_attach": (ctypes.c_int, [_VP, _I32]),
    "srt_pair_order_lookup": (_I32, [_VP, _I32, _I32, _VP, _VP]),
    "srt_pair_order_peek": (_I32, [_VP, _I32, _I32]),
    "srt_pair_order_runs": (_I32, [_VP, _I32]),
    "srt_pair_order_counts": (None, [_VP, _VP, _VP]),
    "srt_pair_order_add_source_runs": (None, [_VP, _U32]),
    "srt_pair_order_set_reach": (None, [_VP, _VP, _VP]),
    "srt_device_count": (ctypes.c_int, []),
    "srt_device_sync": (ctypes.c_int, [_I32]),
    # topology.h (reference signatures)
    "topology_new": (_VP, [_CP, ctypes.c_int]),
    "topology_free": (None, [_VP]),
    "topology_attach": (None, [_VP, _VP, _VP, _CP, _CP, _CP, _VP, _VP]),
    "topology_detach": (None, [_VP, _VP]),
    "topology_isRoutable": (ctypes.c_int, [_VP, _VP, _VP]),
    "topology_getLatency": (_D, [_VP, _VP, _VP]),
    "topology_getReliability": (_D, [_VP, _VP, _VP]),
    "topology_incrementPathPacketCounter": (None, [_VP, _VP, _VP]),
    "topology_computeShortestPaths": (ctypes.c_int, [_VP, ctypes.c_int]),
    "topology_getTable": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
    # topology.h (IP-level additions)
    "srt_topology_new_from_string": (_VP, [_CP, ctypes.c_int]),
    "srt_topology_attach_ip": (_I32, [_VP, _U32, _VP, _CP, _CP, _CP, _VP, _VP]),
    "srt_topology_attach_batch_ip": (_I32, [_VP, _I32, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    "srt_topology_detach_ip": (None, [_VP, _U32]),
    "srt_topology_ipmap_tables": (ctypes.c_int64, [_VP]),
    "srt_topology_vertex_of_ip": (_I32, [_VP, _U32]),
    "srt_topology_latency_ip": (_D, [_VP, _U32, _U32]),
    "srt_topology_reliability_ip": (_D, [_VP, _U32, _U32]),
    "srt_topology_increment_ip": (ctypes.c_int, [_VP, _U32, _U32]),
    "srt_topology_packet_count_ip": (_U64, [_VP, _U32, _U32]),
    "srt_topology_path_source_ip": (_I32, [_VP, _U32, _U32]),
    "srt_topology_send_packet_ip": (ctypes.c_int, [_VP, _U32, _U32, ctypes.c_double, ctypes.c_int,
                                                   _U64, _VP]),
    "srt_topology_send_packets_ip": (ctypes.c_int, [_VP, ctypes.c_int64, _VP, _VP, _VP, _VP, _VP,
                                                    _VP, _VP]),
    "srt_topology_vertex_count": (_I32, [_VP]),
    "srt_topology_edge_count": (_I64, [_VP]),
    "srt_topology_is_directed": (ctypes.c_int, [_VP]),
    "srt_topology_is_complete": (ctypes.c_int, [_VP]),
    "srt_topology_edges": (ctypes.c_int, [_VP, _VP]),
    "srt_topology_min_latency_ms": (_D, [_VP]),
    "srt_topology_table_info": (ctypes.c_int, [_VP, _VP, _VP, _VP]),
    "srt_topology_path_counts": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
    "srt_set_min_time_jump_hook": (None, [_VP]),
    "srt_topology_set_build_opts": (None, [_VP, _VP]),
    "srt_topology_last_stats": (ctypes.c_int, [_VP, _VP]),
}

# srt_pair_reach_fn: (ctx, s, t) -> 1 if s reaches t
PAIR_REACH_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32)
# srt_pair_store_fn: (ctx, src, targets, count)
PAIR_STORE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int32,
                                 ctypes.POINTER(ctypes.c_int32), ctypes.c_int32)

_lib = None


def build(verbose: bool = False) -> str:
    """Compile libshadow_routing.so in-tree (hipcc --offload-arch=gfx950 + gcc)."""
    cmd = ["make", "-C", CSRC, "-j8"]
    if not verbose:
        cmd.append("-s")
    subprocess.run(cmd, check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    """Load the native library (torch, if used, must be imported first so that one HIP runtime
    serves both)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `make -C {CSRC}` or "
                "__graft_entry__.build(); there is no fallback implementation")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != SRT_OK:
        msg = lib().srt_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed: {ERRORS.get(rc, rc)}: {msg}")
