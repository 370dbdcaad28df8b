"""Generate the committed golden fixtures under tests/golden/ (run from the repo root).

Sources of truth, in order of strength:
  1. known answers from the reference's own inline graphs (single vertex + self-loop):
     src/test/phold/phold.yaml:7-21, src/test/tcp/tcp-blocking-lossy.yaml:7-21,
     src/main/core/support/configuration.rs:733-746 (1_gbit_switch),
     docs/network_graph_spec.md:16-37, src/test/config/convert/topology.expected.gml (directed)
     -- the GML texts are data fixtures copied from those files;
  2. the units-grammar known answers of src/main/core/support/units.rs:583-722;
  3. C1 (50-node tor-style complete graph): the C oracle's raw per-source table, with the latency
     matrix cross-checked against networkx (third-party Dijkstra) and, for pairs whose shortest
     path is unique, the reliability of both directions cross-checked against the products along
     networkx's path (forward for s -> t, reversed for t -> s); rel_served_ascending is the table
     the reference serves when sources run in increasing vertex order;
  4. hand-built tie graphs whose expected values are derived by hand below (the canonical tie
     rule of SURVEY.md §8a-4);
  5. attach cases from oracle/attach.py (restatement of topology.c:2024-2216).
The reference itself cannot run here (igraph, glib and the Rust units parser are absent).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from oracle import attach as attach_ref  # noqa: E402
from shadow_amd import graphs  # noqa: E402

MS = 1_000_000

KNOWN = [
    ("phold", "src/test/phold/phold.yaml:7-21", """graph [
  directed 0
  node [
    id 0
    country_code "US"
    bandwidth_down "81920 Kibit"
    bandwidth_up "81920 Kibit"
  ]
  edge [
    source 0
    target 0
    latency "50 ms"
    packet_loss 0.0
  ]
]""", 50 * MS, 1.0),
    ("tcp_blocking_lossy", "src/test/tcp/tcp-blocking-lossy.yaml:7-21", """graph [
  directed 0
  node [
    id 0
    country_code "US"
    bandwidth_down "81920 Kibit"
    bandwidth_up "81920 Kibit"
  ]
  edge [
    source 0
    target 0
    latency "50 ms"
    packet_loss 0.25
  ]
]""", 50 * MS, 0.75),
    ("one_gbit_switch", "src/main/core/support/configuration.rs:733-746", """graph [
  directed 0
  node [
    id 0
    ip_address "0.0.0.0"
    bandwidth_up "1 Gbit"
    bandwidth_down "1 Gbit"
  ]
  edge [
    source 0
    target 0
    latency "1 ms"
    packet_loss 0.0
  ]
]""", 1 * MS, 1.0),
    ("spec_example", "docs/network_graph_spec.md:16-37", """graph [
  directed 0
  node [
    id 0
    label "node at 1.2.3.4"
    country_code "US"
    city_code "Portland"
    ip_address "1.2.3.4"
    bandwidth_down "100 Mbit"
    bandwidth_up "100 Mbit"
  ]
  edge [
    source 0
    target 0
    label "path from 1.2.3.4 to 1.2.3.4"
    latency "10 ms"
    jitter "0 ms"
    packet_loss 0.0
  ]
]""", 10 * MS, 1.0),
    ("convert_expected_directed", "src/test/config/convert/topology.expected.gml", """graph [
  directed 1
  node [
    id 0
    label "poi-1"
    country_code "US"
    bandwidth_down "81920 Kibit"
    bandwidth_up "81920 Kibit"
  ]
  edge [
    source 0
    target 0
    latency "50 ms"
    packet_loss 0.0
  ]
]""", 50 * MS, 1.0),
]

# units.rs:583-722 (Time<TimePrefix> and BitsPerSec<SiPrefixUpper> cases), as the C exports see
# them: parse_time_nanosec -> ns, parse_bandwidth -> bit/s, -1 on error.
UNITS_TIME = [
    ("10", 10_000_000_000), ("10 s", 10_000_000_000), ("10s", 10_000_000_000),
    ("10   s", 10_000_000_000), ("10sec", 10_000_000_000), ("10  m", 600_000_000_000),
    ("10  min", 600_000_000_000), ("10 ms", 10_000_000), ("10 μs", 10_000),
    ("10 millisecond", 10_000_000), ("10 milliseconds", 10_000_000),
    ("-10 ms", -1), ("abc 10 ms", -1), ("10.5 ms", -1), ("10 abc", -1),
    ("4200 sec", 4_200_000_000_000), ("1 hour", 3_600_000_000_000), ("70 min", 4_200_000_000_000),
    ("1000000123 ns", 1_000_000_123), ("0 ms", 0), ("+10 ms", 10_000_000), ("", -1), (".", -1),
    ("10 us", 10_000), ("50 ms", 50_000_000), ("  10 ms  ", -1), ("10 ms ", 10_000_000),
    ("10 MS", -1), ("10 hrs", 36_000_000_000_000), ("9223372036854775807 ns", 9223372036854775807),
    ("9223372036854775808 ns", -1), ("18446744073709551615 ns", -1),
    ("18446744073709551616 ns", -1), ("18446744073709551615 ms", -2),
]
UNITS_BW = [
    ("10", 10), ("10 bit", 10), ("10bit", 10), ("10   bit", 10), ("10  Kbit", 10_000),
    ("10 Kibit", 10_240), ("10 Mbit", 10_000_000), ("10 megabit", 10_000_000),
    ("10 megabits", 10_000_000), ("-10 Kbit", -1), ("abc 10 Kbit", -1), ("10.5 Kbit", -1),
    ("10 abc", -1), ("10 mbit", -1), ("1024 Kbit", 1_024_000), ("1000 Kibit", 1_024_000),
    ("81920 Kibit", 83_886_080), ("1 Gbit", 1_000_000_000), ("100 Mbit", 100_000_000),
    ("1 Tibit", 1_099_511_627_776), ("10 K", 10_000), ("10 bits", 10),
]


def known_answers():
    out = []
    for name, src, gml, lat_ns, rel in KNOWN:
        out.append({"name": name, "source": src, "gml": gml, "use_shortest_path": True,
                    "pairs": [[0, 0, lat_ns, rel]]})
    return out


def tie_graphs():
    """Hand-derived expectations for the canonical tie rule. Every pair (s, t)
    is source s's own path (the raw row; which row serves a lookup is the lazy-cache order)."""
    def gml(n, edges, directed=False):
        edge_store.append({"n": n, "directed": directed, "edges": edges})
        g = ["graph [", f"  directed {1 if directed else 0}"]
        for v in range(n):
            g += ["  node [", f"    id {v}", '    bandwidth_down "1 Gbit"',
                  '    bandwidth_up "1 Gbit"', "  ]"]
        for (a, b, lat, loss) in edges:
            g += ["  edge [", f"    source {a}", f"    target {b}", f'    latency "{lat} ms"',
                  f"    packet_loss {loss}", "  ]"]
        return "\n".join(g + ["]"])

    cases = []
    edge_store = []
    # T1 triangle: 0-2 direct 10 ties 0-1-2 (5+5); pred(0,2) = 0 (key (0,0) < (5,1)) -> direct
    e = [(0, 1, 5, 0.1), (1, 2, 5, 0.2), (0, 2, 10, 0.3), (0, 0, 100, 0.0), (1, 1, 100, 0.0),
         (2, 2, 100, 0.0)]
    cases.append({"name": "triangle_direct_vs_two_hop", "gml": gml(3, e), "pairs": [
        [0, 2, 10 * MS, 0.7], [2, 0, 10 * MS, 0.7], [0, 1, 5 * MS, 0.9], [1, 2, 5 * MS, 0.8],
        # diagonal: v0 min(100, 2*5 via nb1, 2*10) = 10, rel 0.9^2
        [0, 0, 10 * MS, 0.9 * 0.9],
        # v1: 2*5 via nb0 (loss .1) ties 2*5 via nb2 (loss .2): first in neighbor order -> nb0
        [1, 1, 10 * MS, 0.9 * 0.9],
        [2, 2, 10 * MS, 0.8 * 0.8]]})
    # T2 square, equal lengths 2+3 / 3+2: pred(0,3) = 1 (D=2 < D=3)
    e = [(0, 1, 2, 0.1), (1, 3, 3, 0.2), (0, 2, 3, 0.3), (2, 3, 2, 0.4)] + \
        [(v, v, 50, 0.0) for v in range(4)]
    cases.append({"name": "square_pred_by_distance", "gml": gml(4, e), "pairs": [
        [0, 3, 5 * MS, (1.0 * 0.9) * 0.8],
        # (3,0) from source 3: 3-1-0 (3+2) ties 3-2-0 (2+3); pred(3,0)=2 (D[3][2]=2 < D[3][1]=3)
        [3, 0, 5 * MS, (1.0 * 0.6) * 0.7],
        # (1,2) from source 1: 1-0-2 (2+3) ties 1-3-2 (3+2); pred(1,2)=0 (D[1][0]=2 < D[1][3]=3)
        [1, 2, 5 * MS, (1.0 * 0.9) * 0.7],
        # (2,1) from source 2: 2-0-1 (3+2) ties 2-3-1 (2+3); pred(2,1)=3 (D[2][3]=2 < D[2][0]=3)
        [2, 1, 5 * MS, (1.0 * 0.6) * 0.8]]})
    # T3 diamond with equal D[u]: pred(0,3) among u=1,2 (both D=1) -> lower index 1
    e = [(0, 1, 1, 0.1), (0, 2, 1, 0.2), (1, 3, 1, 0.3), (2, 3, 1, 0.4)] + \
        [(v, v, 50, 0.0) for v in range(4)]
    cases.append({"name": "diamond_pred_by_index", "gml": gml(4, e), "pairs": [
        [0, 3, 2 * MS, (1.0 * 0.9) * 0.7],
        # (3,0) from source 3: D[3][1] = D[3][2] = 1 -> lower index 1: 3-1-0
        [3, 0, 2 * MS, (1.0 * 0.7) * 0.9],
        [1, 2, 2 * MS, (1.0 * 0.9) * 0.8],
        # (2,1) from source 2: D[2][0] = D[2][3] = 1 -> lower index 0: 2-0-1
        [2, 1, 2 * MS, (1.0 * 0.8) * 0.9],
        [0, 0, 2 * MS, 0.9 * 0.9], [3, 3, 2 * MS, 0.7 * 0.7]]})
    # T4 directed: the true directed table (no reference symmetry quirk)
    e = [(0, 1, 1, 0.1), (1, 0, 5, 0.2), (1, 2, 1, 0.3), (2, 0, 1, 0.4), (0, 2, 10, 0.5),
         (0, 0, 50, 0.0), (1, 1, 50, 0.0), (2, 2, 50, 0.0)]
    cases.append({"name": "directed_cycle", "gml": gml(3, e, directed=True), "pairs": [
        [0, 2, 2 * MS, (1.0 * 0.9) * 0.7], [2, 0, 1 * MS, 0.6], [1, 0, 2 * MS, (1.0 * 0.7) * 0.6],
        [0, 1, 1 * MS, 0.9], [2, 1, 2 * MS, (1.0 * 0.6) * 0.9], [1, 2, 1 * MS, 0.7],
        # directed diagonal: out-edges only, doubled: v0 2*1 via nb1, v2 2*1 via nb0
        [0, 0, 2 * MS, 0.9 * 0.9], [1, 1, 2 * MS, 0.7 * 0.7], [2, 2, 2 * MS, 0.6 * 0.6]]})
    # T5 no self-loops: diagonal from the cheapest incident edge, doubled
    e = [(0, 1, 7, 0.1), (1, 2, 3, 0.2)]
    cases.append({"name": "path_no_selfloops", "gml": gml(3, e), "pairs": [
        [0, 2, 10 * MS, (1.0 * 0.9) * 0.8], [2, 0, 10 * MS, (1.0 * 0.8) * 0.9],
        [0, 0, 14 * MS, 0.9 * 0.9], [1, 1, 6 * MS, 0.8 * 0.8], [2, 2, 6 * MS, 0.8 * 0.8]]})
    # T6 parallel edges collapse to the (min latency, lowest index) edge
    e = [(0, 1, 9, 0.5), (0, 1, 4, 0.3), (0, 1, 4, 0.1), (1, 2, 1, 0.0), (0, 0, 50, 0.0),
         (1, 1, 50, 0.0), (2, 2, 50, 0.0)]
    cases.append({"name": "parallel_edges", "gml": gml(3, e), "pairs": [
        [0, 1, 4 * MS, 0.7], [0, 2, 5 * MS, (1.0 * 0.7) * 1.0]]})
    for case, es in zip(cases, edge_store):
        case.update(es)
    return cases


def attach_cases():
    verts = [
        {"ip": "11.0.0.1", "city": "Portland", "country": "US"},
        {"ip": "11.0.0.2", "city": "Seattle", "country": "US"},
        {"ip": "12.0.0.1", "city": "Berlin", "country": "DE"},
        {"ip": "", "city": "Paris", "country": "FR"},
        {"ip": "11.0.1.9", "city": "", "country": "US"},
        {"ip": "127.0.0.1", "city": "Berlin", "country": "DE"},
        {"ip": "1.0.0.127", "city": "", "country": "CA"},
    ]
    lines = ["graph [", "  directed 0"]
    for v, a in enumerate(verts):
        lines += ["  node [", f"    id {v}"]
        if a["ip"]:
            lines.append(f'    ip_address "{a["ip"]}"')
        if a["city"]:
            lines.append(f'    city_code "{a["city"]}"')
        lines.append(f'    country_code "{a["country"]}"')
        lines += ['    bandwidth_down "1 Gbit"', '    bandwidth_up "81920 Kibit"', "  ]"]
    for v in range(len(verts)):
        for u in range(v, len(verts)):
            lines += ["  edge [", f"    source {v}", f"    target {u}",
                      f'    latency "{1 + (v * 7 + u * 3) % 20} ms"', "    packet_loss 0.0", "  ]"]
    lines.append("]")
    hints = [
        (None, None, None), ("11.0.0.2", None, None), ("11.0.0.200", None, None),
        ("11.0.1.1", None, "US"), (None, "berlin", None), (None, None, "us"),
        ("12.0.0.9", "Seattle", None), ("99.1.2.3", None, "FR"), (None, "Nowhere", "Nowhere"),
        ("not-an-ip", None, None), ("0.0.0.0", None, None), ("1.0.0.127", None, None),
        ("127.0.0.1", None, None), (None, None, "CA"),
    ]
    out = []
    for seed in (1, 7, 12345):
        state = [seed]
        for (ip, city, country) in hints:
            before = state[0]
            v = attach_ref.find_attachment_vertex(verts, state, ip, city, country)
            out.append({"seed_before": before, "ip_hint": ip, "city_hint": city,
                        "country_hint": country, "vertex": v, "seed_after": state[0]})
    return {"gml": "\n".join(lines), "cases": out,
            "bw_down_kib": 1_000_000_000 // 8192, "bw_up_kib": 83_886_080 // 8192}


def c1():
    g = graphs.complete_graph(50, seed=1, lat_max=300, self_max=10, loss_max=500, name="C1")
    gml = graphs.to_gml(g)
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    t = oracle.table(el, True, oracle.ORC_INT_NS, raw=True)
    tf = oracle.table(el, True, oracle.ORC_F64_MS, raw=True)
    served = oracle.table(el, True, oracle.ORC_INT_NS)  # sources in increasing vertex order
    assert np.array_equal(t["lat_int"], tf["lat_int"]) and np.array_equal(t["rel"], tf["rel"])
    assert np.array_equal(t["lat_int"], t["lat_ref"]), "whole-ms graph: integer ns == ceil(ms*1e6)"
    import networkx as nx
    G = nx.Graph()
    for e in range(g.m):
        a, b = int(g.src[e]), int(g.dst[e])
        if a != b:
            G.add_edge(a, b, weight=int(g.lat_ns[e]), r=1.0 - float(g.loss[e]))
    nx_unique = 0
    unique_dir_differ = 0  # unique shortest path, yet rel(s->t) != rel(t->s) bitwise
    for s in range(g.n):
        dist = nx.single_source_dijkstra_path_length(G, s, weight="weight")
        for t_, d in dist.items():
            if t_ != s:
                assert int(t["lat_int"][s, t_]) == d, (s, t_)
        for t_ in range(s + 1, g.n):
            paths = list(nx.all_shortest_paths(G, s, t_, weight="weight"))
            if len(paths) == 1:
                p = paths[0]
                rel = 1.0
                for a, b in zip(p[:-1], p[1:]):
                    rel *= G[a][b]["r"]
                back = 1.0  # source t_'s own row multiplies the same hops in reverse order
                for a, b in zip(p[::-1][:-1], p[::-1][1:]):
                    back *= G[a][b]["r"]
                assert t["rel"][s, t_] == rel and t["rel"][t_, s] == back
                nx_unique += 1
                unique_dir_differ += int(rel != back)
    off = ~np.eye(g.n, dtype=bool)
    dir_differ = int((t["rel"][off] != t["rel"].T[off]).sum()) // 2
    np.savez_compressed(os.path.join(HERE, "c1_expected.npz"), lat_ns=t["lat_int"],
                        rel=t["rel"], lat_ms=t["lat_ms"], rel_served_ascending=served["rel"])
    with open(os.path.join(HERE, "c1.gml"), "w") as f:
        f.write(gml)
    return {"n": g.n, "edges": g.m, "networkx_version": nx.__version__,
            "pairs_with_unique_path_checked": nx_unique,
            "unique_path_pairs_rel_direction_differs": unique_dir_differ,
            "pairs_rel_direction_differs": dir_differ}


def main():
    meta = {"c1": c1()}
    with open(os.path.join(HERE, "known_answers.json"), "w") as f:
        json.dump(known_answers(), f, indent=1)
    with open(os.path.join(HERE, "units_cases.json"), "w") as f:
        json.dump({"time_ns": UNITS_TIME, "bandwidth_bps": UNITS_BW}, f, indent=1, ensure_ascii=False)
    ties = tie_graphs()
    for case in ties:  # the oracle must agree with the hand derivation before it is committed
        e = np.array(case["edges"], dtype=np.float64)
        el = oracle.EdgeList(case["n"], case["directed"], e[:, 0].astype(np.int32),
                             e[:, 1].astype(np.int32), (e[:, 2] * MS).astype(np.int64), e[:, 3])
        t = oracle.table(el, True, raw=True)
        for s_, t_, lat, rel in case["pairs"]:
            assert int(t["lat_int"][s_, t_]) == lat and t["rel"][s_, t_] == rel, (case["name"], s_, t_)
    with open(os.path.join(HERE, "ties.json"), "w") as f:
        json.dump(ties, f, indent=1)
    with open(os.path.join(HERE, "attach_cases.json"), "w") as f:
        json.dump(attach_cases(), f, indent=1)
    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
