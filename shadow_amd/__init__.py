"""shadow_amd -- MI355X-native routing-table build for Shadow's network graph.

The product is the C-ABI library libshadow_routing.so (csrc/: C host layer + gfx950 HIP kernels +
RCCL); this package holds its ctypes binding (_lib), the Python mirror of the routing interface
(topology), and the synthetic graph generators used by tests and bench.py (graphs).
"""
__all__ = ["_lib", "graphs", "topology"]
