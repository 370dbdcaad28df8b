#!/usr/bin/env python3
"""Host-side rows of SURVEY.md §8f at scale (CPU only, no GPU):

  f-2  GML ingestion: the single-pass reader + validation (topology.c:326-1122) on the C3 and C5
       graphs written as GML (ip_address and country_code on every vertex).
  f-3  batched attach (srt_topology_attach_batch_ip) of 100,000 hosts on the C5 graph: one third
       exact-IP hints, one third other IP hints (longest prefix match), one third without hints
       (random pick), against the per-host vertex scan of the reference (topology.c:2024-2216)
       restated in oracle/attach.py (test infrastructure; timed on a sample and checked for
       parity on that sample).

usage: python tools/bench_host.py [--out profiles/r01_host_paths.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from shadow_amd import graphs  # noqa: E402
from shadow_amd.topology import Topology  # noqa: E402


def ip_str(x):
    return f"{x >> 24 & 255}.{x >> 16 & 255}.{x >> 8 & 255}.{x & 255}"


def gml_row(name, g):
    text = graphs.to_gml(g)
    t0 = time.perf_counter()
    top = Topology.from_gml(text)
    dt = time.perf_counter() - t0
    mb = len(text) / 1e6
    return top, text, {"graph": name, "n": g.n, "edges": int(g.m), "gml_mb": round(mb, 1),
                       "parse_validate_ms": round(dt * 1e3, 1),
                       "mb_per_s": round(mb / dt, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--hosts", type=int, default=100_000)
    ap.add_argument("--sample", type=int, default=20)
    a = ap.parse_args()
    res = {"gml": [], "attach": None}
    _, _, r3 = gml_row("C3", graphs.random_geometric(20_000, seed=3))
    res["gml"].append(r3)
    g5 = graphs.barabasi_albert(100_000, m=3, seed=5)
    top, text, r5 = gml_row("C5", g5)
    res["gml"].append(r5)
    print(json.dumps(res["gml"]), flush=True)

    rng = np.random.default_rng(11)
    h = a.hosts
    kind = rng.integers(0, 3, size=h)
    vert_ip = 0x0B000001 + rng.integers(0, g5.n, size=h)  # the vertices' own addresses
    other_ip = rng.integers(0x0C000000, 0xDF000000, size=h)
    ip_hints = [ip_str(int(vert_ip[i])) if kind[i] == 0 else
                ip_str(int(other_ip[i])) if kind[i] == 1 else None for i in range(h)]
    country = [None if kind[i] == 2 else "us" for i in range(h)]
    addrs = [ip_str(0x64000000 + i) for i in range(h)]
    seeds = rng.integers(1, 2**31, size=h).astype(np.uint32)
    t0 = time.perf_counter()
    vs, _, _, states = top.attach_batch(addrs, seeds, ip_hints, None, country)
    dt = time.perf_counter() - t0

    from oracle import attach as oa  # test infrastructure: the per-host scan, timed on a sample
    verts = [{"ip": ip_str(0x0B000001 + v), "country": "US"} for v in range(g5.n)]
    idx = rng.choice(h, size=a.sample, replace=False)
    t1 = time.perf_counter()
    ok = True
    for i in idx:
        st = [int(seeds[i])]
        w = oa.find_attachment_vertex(verts, st, ip_hints[i], None, country[i])
        ok &= (w == int(vs[i])) and (st[0] == int(states[i]))
    ds = (time.perf_counter() - t1) / a.sample
    res["attach"] = {
        "graph": "C5", "vertices": g5.n, "hosts": h,
        "hints": "1/3 exact ip, 1/3 other ip (LPM over the country queue), 1/3 none (random)",
        "batch_ms": round(dt * 1e3, 1), "us_per_host": round(dt / h * 1e6, 2),
        "scan_restatement_ms_per_host": round(ds * 1e3, 1),
        "scan_sample_hosts": a.sample, "sample_parity": bool(ok),
        "note": "the scan is oracle/attach.py (Python) restating the reference's per-host "
                "O(V) vertex scan; the batch is the indexed O(log V) C path"}
    print(json.dumps(res["attach"]), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
