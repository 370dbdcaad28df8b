"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of Shadow's IP -> vertex attachment.

Follows /root/reference/src/main/routing/topology.c:
  _topology_findAttachmentVertexHelperHook  :2024-2100  (candidate queues, exact-IP clearing)
  _topology_getLongestPrefixMatch           :2102-2130  (~(vertexIP ^ ip) on network-order u32)
  _topology_findAttachmentVertex            :2132-2216  (city > country > all; LPM or rand_r pick)
  address_stringToIP                        address.c:145-152 (inet_pton, INADDR_NONE)
  random_nextDouble                         random.c:32-43 (glibc rand_r / RAND_MAX)
"""
from __future__ import annotations

import ctypes
import ctypes.util
import socket
import struct

INADDR_NONE = 0xFFFFFFFF
INADDR_ANY = 0
INADDR_LOOPBACK = 0x7F000001  # host-order constant compared with network-order values (:2051)
RAND_MAX = 2147483647

_libc = ctypes.CDLL(ctypes.util.find_library("c"))
_libc.rand_r.argtypes = [ctypes.POINTER(ctypes.c_uint)]
_libc.rand_r.restype = ctypes.c_int
_libm = ctypes.CDLL(ctypes.util.find_library("m"))
_libm.round.argtypes = [ctypes.c_double]
_libm.round.restype = ctypes.c_double


def string_to_ip(s):
    if s is None:
        return INADDR_NONE
    try:
        return struct.unpack("=I", socket.inet_pton(socket.AF_INET, s))[0]
    except OSError:
        return INADDR_NONE


def next_double(state: list) -> float:
    st = ctypes.c_uint(state[0])
    v = _libc.rand_r(ctypes.byref(st))
    state[0] = st.value
    return float(v) / float(RAND_MAX)


def _usable(ip):
    return ip != INADDR_NONE and ip != INADDR_ANY and ip != INADDR_LOOPBACK


def find_attachment_vertex(vertices, rand_state: list, ip_hint=None, city_hint=None,
                           country_hint=None) -> int:
    """vertices: list of dicts with optional 'ip', 'city', 'country' (in vertex-index order)."""
    requested_usable = False
    requested_ip = 0
    if ip_hint is not None:
        ip = string_to_ip(ip_hint)
        if _usable(ip):
            requested_usable, requested_ip = True, ip
    city, country, allq = [], [], []
    n_city = n_country = n_all = 0
    found_exact = False
    for v, a in enumerate(vertices):
        ip_str = a.get("ip") or ""
        cty = a.get("city") or None
        ctr = a.get("country") or None
        city_match = cty is not None and city_hint is not None and cty.lower() == city_hint.lower()
        country_match = (ctr is not None and country_hint is not None
                         and ctr.lower() == country_hint.lower())
        usable, vip = False, INADDR_NONE
        if ip_str:
            ip = string_to_ip(ip_str)
            if _usable(ip):
                usable, vip = True, ip
        if requested_usable and usable and vip == requested_ip:
            if not found_exact:
                city.clear()
                country.clear()
                allq.clear()
            found_exact = True
            allq.append(v)
            n_all += 1
        if found_exact:
            continue
        allq.append(v)
        n_all += usable
        if city_match:
            city.append(v)
            n_city += usable
        if country_match:
            country.append(v)
            n_country += usable
    if city:
        cand, use_lpm = city, requested_usable and n_city > 0
    elif country:
        cand, use_lpm = country, requested_usable and n_country > 0
    else:
        cand, use_lpm = allq, ip_hint is not None and n_all > 0
    assert cand, "numCandidates > 0 (topology.c:2182)"
    if use_lpm and not found_exact:
        best_match, best = 0, -1
        for v in cand:
            vip = string_to_ip(vertices[v].get("ip") or "")
            match = (~(vip ^ requested_ip)) & 0xFFFFFFFF
            if match > best_match or best_match == 0:
                best_match, best = match, v
        return best
    u = next_double(rand_state)
    idx = int(_libm.round(float(len(cand) - 1) * u))  # C round(): half away from zero
    return cand[idx]
