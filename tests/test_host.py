"""Host-side C layer (no GPU): units grammar, GML reader + validation rules, attach, ABI."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from shadow_amd import graphs
from shadow_amd.topology import Topology, parse_bandwidth, parse_time_nanosec

MS = 1_000_000


# ---- units.rs grammar (units.rs:404-437, :583-722, :776-837) -----------------------------------
def test_units_known_answers(native):
    cases = json.load(open(os.path.join(GOLDEN, "units_cases.json")))
    for s, want in cases["time_ns"]:
        assert parse_time_nanosec(s) == want, repr(s)
    for s, want in cases["bandwidth_bps"]:
        assert parse_bandwidth(s) == want, repr(s)


def test_units_whitespace_and_newline(native):
    assert parse_time_nanosec("10\tms") == 10 * MS
    assert parse_time_nanosec("10 ms") == 10 * MS  # Unicode \s (NBSP) between value and unit
    assert parse_time_nanosec("10 m\ns") == -1           # '.' does not match '\n' in (.*)$


# ---- GML reader + validation (topology.c:525-1038) --------------------------------------------
BASE_NODE = 'node [ id {id} bandwidth_down "1 Gbit" bandwidth_up "1 Gbit" {extra} ]'
BASE_EDGE = 'edge [ source {a} target {b} latency "{lat}" packet_loss {loss} {extra} ]'


def gml(nodes, edges, directed=0, header=""):
    body = "\n".join([BASE_NODE.format(id=i, extra=x) for i, x in nodes] +
                     [BASE_EDGE.format(a=a, b=b, lat=l, loss=p, extra=x) for a, b, l, p, x in edges])
    return f"graph [ directed {directed} {header}\n{body}\n]"


def tri(**kw):
    nodes = [(0, ""), (1, ""), (2, "")]
    edges = [(0, 1, "5 ms", 0.1, ""), (1, 2, "5 ms", 0.2, ""), (0, 2, "10 ms", 0.3, "")]
    return gml(nodes, edges, **kw)


def test_parse_accepts_reference_fixtures(native):
    for c in json.load(open(os.path.join(GOLDEN, "known_answers.json"))):
        t = Topology.from_gml(c["gml"])
        assert t.n == 1 and t.m == 1
    t = Topology.from_gml(open(os.path.join(GOLDEN, "c1.gml")).read())
    n, directed, src, dst, lat, loss = t.edges()
    g = graphs.complete_graph(50, seed=1)
    assert n == 50 and not directed
    assert np.array_equal(src, g.src) and np.array_equal(dst, g.dst)
    assert np.array_equal(lat, g.lat_ns) and np.array_equal(loss, g.loss)
    assert t.complete


@pytest.mark.parametrize("text,ok,why", [
    (tri(), True, "plain triangle"),
    (gml([(0, ""), (1, "")], [(0, 1, "1 ms", 0.0, "")]), True, "two nodes"),
    (gml([(0, ""), (1, "")], []), False, "disconnected (topology.c:707-713)"),
    (gml([(0, ""), (1, "")], [(0, 1, "1 ms", 0.0, "")], directed=1), False,
     "directed edge only one way: not strongly connected"),
    (gml([(0, ""), (1, "")], [(0, 1, "0 ms", 0.0, "")]), False, "latency must be > 0 (:922)"),
    (gml([(0, ""), (1, "")], [(0, 1, "1.5 ms", 0.0, "")]), False, "fractional value (units.rs)"),
    (gml([(0, ""), (1, "")], [(0, 1, "1 ms", 1.5, "")]), False, "loss > 1 (:942)"),
    (gml([(0, ""), (1, "")], [(0, 1, "1 ms", -0.1, "")]), False, "loss < 0"),
    (gml([(0, ""), (1, "")], [(0, 1, "1 ms", 1.0, "")]), True, "loss == 1 allowed"),
    (gml([(0, 'foo 1'), (1, "")], [(0, 1, "1 ms", 0.0, "")]), False, "unsupported vertex attr"),
    (gml([(0, 'identifier 1'), (1, "")], [(0, 1, "1 ms", 0.0, "")]), True,
     "prefix match of 'id' (topology.c:184-188)"),
    (gml([(0, 'Label "x"'), (1, "")], [(0, 1, "1 ms", 0.0, "")]), True, "case-insensitive prefix"),
    (gml([(0, 'ip_address 5'), (1, "")], [(0, 1, "1 ms", 0.0, "")]), False, "ip_address must be a string"),
    (gml([(0, ""), (1, "")], [(0, 1, "1 ms", 0.0, 'jitter "2 ms"')]), True, "jitter ok"),
    (gml([(0, ""), (1, "")], [(0, 1, "1 ms", 0.0, 'color "red"')]), False, "unsupported edge attr"),
    (gml([(0, ""), (1, "")], [(0, 1, "1 ms", 0.0, 'graphics [ x 1 ]')]), True, "nested list skipped"),
    ('graph [ node [ id 0 bandwidth_down "1 Gbit" bandwidth_up "1 Gbit" ] '
     'edge [ source 0 target 0 latency 10 packet_loss 0.0 ] ]', False, "numeric latency"),
    ('graph [ node [ id 0 bandwidth_down "1 Gbit" ] edge [ source 0 target 0 latency "1 ms" '
     'packet_loss 0.0 ] ]', False, "missing bandwidth_up"),
    ('graph [ node [ id 0 bandwidth_down "4 Kbit" bandwidth_up "1 Gbit" ] edge [ source 0 target 0 '
     'latency "1 ms" packet_loss 0.0 ] ]', False, "bandwidth < 8 Kibit rounds to 0 KiB/s"),
    ('graph [ node [ id 0 bandwidth_down "1 Gbit" bandwidth_up "1 Gbit" ] edge [ source 0 target 0 '
     'latency "1 ms" ] ]', False, "missing packet_loss"),
    ('graph [ node [ id 0 bandwidth_down "1 Gbit" bandwidth_up "1 Gbit" ] edge [ source 0 target 7 '
     'latency "1 ms" packet_loss 0.0 ] ]', False, "unknown node id"),
    ('# comment\nCreator "x"\ngraph [ node [ id 3 bandwidth_down "1 Gbit" bandwidth_up "1 Gbit" ] '
     'edge [ source 3 target 3 latency "1 ms" packet_loss 0.0 ] ]', True, "comments, top-level keys"),
])
def test_validation_rules(native, text, ok, why):
    t = Topology.try_from_gml(text)
    assert (t is not None) == ok, why


def test_complete_detection_and_direct_mode(native):
    """_topology_isComplete (:409-511): self-loops required; !complete && !use_shortest_path
    fails (:696-699)."""
    g = graphs.complete_graph(6, seed=3)
    assert Topology.from_gml(graphs.to_gml(g), use_shortest_path=False).complete
    nose = graphs.Graph(g.n, False, g.src[g.src != g.dst], g.dst[g.src != g.dst],
                        g.lat_ns[g.src != g.dst], g.loss[g.src != g.dst])
    assert not Topology.from_gml(graphs.to_gml(nose)).complete
    assert Topology.try_from_gml(graphs.to_gml(nose), use_shortest_path=False) is None


def test_topology_new_from_file(native, tmp_path):
    p = tmp_path / "g.gml"
    p.write_text(tri())
    t = Topology.new(str(p))
    assert t.n == 3 and t.m == 3 and not t.directed
    with pytest.raises(ValueError):
        Topology.new(str(tmp_path / "missing.gml"))


# ---- attach (topology.c:2024-2281) ---------------------------------------------------------
def test_attach_matches_restatement(native):
    fx = json.load(open(os.path.join(GOLDEN, "attach_cases.json")))
    top = Topology.from_gml(fx["gml"])
    for i, c in enumerate(fx["cases"]):
        v, down, up, after = top.attach(f"100.64.{i // 250}.{i % 250 + 1}", c["seed_before"],
                                        c["ip_hint"], c["city_hint"], c["country_hint"])
        assert v == c["vertex"], c
        assert after == c["seed_after"], c
        assert down == fx["bw_down_kib"] and up == fx["bw_up_kib"]


def test_attach_detach_lookup(native):
    top = Topology.from_gml(tri())
    v, _, _, _ = top.attach("11.0.0.9", 1, None, None, None)
    assert top.vertex_of("11.0.0.9") == v
    top.detach("11.0.0.9")
    assert top.vertex_of("11.0.0.9") == -1
    # unattached endpoints: -1, not routable (topology.c:1905-1915, :2019-2022); no build needed
    assert top.get_latency("11.0.0.9", "11.0.0.10") == -1
    assert not top.is_routable("11.0.0.9", "11.0.0.10")


def test_ipmap_bounded_under_attach_detach_cycles(native):
    """20,000 attach / detach cycles of fresh addresses leave the IP map at a
    bounded number of tables (a rehash of a mostly-tombstone table keeps its capacity, and replaced
    tables are reclaimed once no reader holds them), and lookups stay right throughout."""
    from shadow_amd.topology import ip_to_net
    top = Topology.from_gml(tri())
    keep = [f"12.0.0.{i}" for i in range(1, 9)]
    for ip in keep:
        top.attach(ip, 1, None, None, None)
    for i in range(20000):
        ip = f"13.{(i >> 16) & 255}.{(i >> 8) & 255}.{i & 255}"
        top.attach(ip, 1, None, None, None)
        assert top.vertex_of(ip) >= 0
        top.detach(ip)
        assert top.vertex_of(ip) == -1
    assert all(top.vertex_of(ip) >= 0 for ip in keep)
    k = native.srt_topology_ipmap_tables(top._h)
    assert 1 <= k <= 2, k
    assert ip_to_net("12.0.0.1") != 0


def _attach_world(rng, n):
    """Vertex attributes with duplicates, gaps and the special addresses the reference treats as
    unusable (0.0.0.0, 255.255.255.255, an unparsable string, and 1.0.0.127, whose network-order
    value equals the host-order INADDR_LOOPBACK constant, topology.c:2051)."""
    pool = [f"10.{a}.{b}.{c}" for a, b, c in rng.integers(0, 4, size=(24, 3))]
    special = ["0.0.0.0", "255.255.255.255", "bogus", "1.0.0.127", "127.0.0.1", "10.20.30.40"]
    cities = ["Portland", "portland", "PORTLAND", "Berlin", "berlin", "Lima", "zz"]
    countries = ["US", "us", "DE", "Pe", "pe"]
    verts = []
    for v in range(n):
        a = {}
        r = rng.random()
        if r < 0.7:
            a["ip"] = pool[rng.integers(len(pool))]
        elif r < 0.85:
            a["ip"] = special[rng.integers(len(special))]
        if rng.random() < 0.6:
            a["city"] = cities[rng.integers(len(cities) - 1)]
        if rng.random() < 0.7:
            a["country"] = countries[rng.integers(len(countries))]
        verts.append(a)
    for v in (n - 7, n - 3):  # the all-zero-match queue: city "zz", both at 10.20.30.40
        verts[v] = {"ip": "10.20.30.40", "city": "zz", "country": "US"}
    nodes = []
    for v, a in enumerate(verts):
        extra = " ".join(f'{k} "{a[x]}"' for x, k in (("ip", "ip_address"), ("city", "city_code"),
                                                   ("country", "country_code")) if x in a)
        nodes.append((v, extra))
    edges = [(v, v, "1 ms", 0.0, "") for v in range(n)]
    edges += [(v, v + 1, "2 ms", 0.0, "") for v in range(n - 1)]
    return verts, gml(nodes, edges), pool


def _attach_hosts(rng, h, pool):
    ipish = pool + ["0.0.0.0", "127.0.0.1", "1.0.0.127", "bogus", "245.235.225.215", "10.9.9.9",
                    "11.3.2.1", "200.1.2.3"]
    out = []
    for i in range(h):
        ip = None if rng.random() < 0.25 else ipish[rng.integers(len(ipish))]
        city = None if rng.random() < 0.5 else ["portland", "Berlin", "LIMA", "zz", "Oslo",
                                                 "ZZ"][rng.integers(6)]
        ctry = None if rng.random() < 0.5 else ["us", "De", "PE", "FR"][rng.integers(4)]
        out.append((ip, city, ctry, int(rng.integers(1, 2**31))))
    # 245.235.225.215 is ~10.20.30.40: every match in city "zz" is 0 -> the queue's last vertex
    out.append(("245.235.225.215", "zz", None, 7))
    return out


@pytest.mark.parametrize("seed", [0, 1, 2, 3, 4, 5])
def test_attach_indexed_matches_restatement(native, seed):
    """The O(log n) indexed attach (single and batched) against the pure-Python restatement of
    the reference's per-host vertex scan (oracle/attach.py), hints and seeds randomized."""
    from oracle import attach as oa
    rng = np.random.default_rng(seed)
    verts, text, pool = _attach_world(rng, 257)
    hosts = _attach_hosts(rng, 600, pool)
    want, want_state = [], []
    for ip, city, ctry, sd in hosts:
        st = [sd]
        want.append(oa.find_attachment_vertex(verts, st, ip, city, ctry))
        want_state.append(st[0])
    top = Topology.from_gml(text)
    for i, (ip, city, ctry, sd) in enumerate(hosts):
        v, _, _, after = top.attach(f"100.65.{i // 250}.{i % 250 + 1}", sd, ip, city, ctry)
        assert (v, after) == (want[i], want_state[i]), hosts[i]
    top2 = Topology.from_gml(text)
    addrs = [f"100.66.{i // 250}.{i % 250 + 1}" for i in range(len(hosts))]
    vs, down, up, states = top2.attach_batch(addrs, [h[3] for h in hosts], [h[0] for h in hosts],
                                             [h[1] for h in hosts], [h[2] for h in hosts])
    assert vs.tolist() == want and states.tolist() == want_state
    assert top2.vertex_of(addrs[5]) == want[5]
    assert hosts[-1][0] == "245.235.225.215" and want[-1] == 257 - 3


# ---- C-ABI exports ---------------------------------------------------------------------------
def _declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b([a-z_][a-zA-Z0-9_]*)\s*\(", text)) - {"if", "sizeof"}


def test_library_exports_every_declared_symbol(native):
    from shadow_amd import _lib
    names = {n for n in _declared("shadow_routing.h") | _declared("topology.h")
             if n.startswith(("srt_", "topology_"))}
    assert len(names) > 40
    for n in sorted(names):
        assert hasattr(native, n), f"{n} declared in include/ but not exported"
        assert n in _lib.SIGNATURES, f"{n} missing from the ctypes signature table"


def test_version_and_device_count_without_gpu(native):
    assert b"gfx950" in native.srt_version()
    assert native.srt_device_count() >= 0


def test_shard_rows_partition(native):
    for n, align, R in [(32768, 128, 8), (1024, 128, 3), (1000, 64, 7), (130, 128, 4)]:
        got = []
        for r in range(R):
            b, e = ctypes.c_int32(), ctypes.c_int32()
            native.srt_shard_rows(n, align, R, r, ctypes.byref(b), ctypes.byref(e))
            got.append((b.value, e.value))
            assert b.value % align == 0 and e.value % align == 0
        assert got[0][0] == 0 and got[-1][1] >= n and got[-1][1] < n + align
        for (b0, e0), (b1, e1) in zip(got, got[1:]):
            assert e0 == b1


def test_range_check(native):
    """Latencies beyond the u32 quantum range fail loudly (SRT_E_RANGE), never silently."""
    from shadow_amd._lib import Edges
    src = np.array([0], np.int32)
    dst = np.array([1], np.int32)
    lat = np.array([2**40], np.int64)
    loss = np.array([0.0])
    e = Edges(2, 0, 1, src.ctypes.data, dst.ctypes.data, lat.ctypes.data, loss.ctypes.data)
    q, mw = ctypes.c_uint64(), ctypes.c_uint32()
    assert native.srt_latency_quantum(ctypes.byref(e), ctypes.byref(q), ctypes.byref(mw)) == 0
    lat2 = np.array([3, 2**40], np.int64)
    src2, dst2 = np.array([0, 0], np.int32), np.array([1, 1], np.int32)
    e2 = Edges(2, 0, 2, src2.ctypes.data, dst2.ctypes.data, lat2.ctypes.data, np.zeros(2).ctypes.data)
    assert native.srt_latency_quantum(ctypes.byref(e2), ctypes.byref(q), ctypes.byref(mw)) == -6


# ---- bench.py parity helpers (the N > 1 check of the driver's scaling run) ------------------------
def test_bench_parity_rows_cover_first_and_last_rank(native):
    """At N ranks the bench checks rows of rank 0 and of the last rank (including each one's
    last row), gathered to rank 0; the kernel-free helpers are plain host code."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    class FakeCtx:
        world, rank = 8, 0
    n = 32768
    blocks = [(q * 4096, (q + 1) * 4096) for q in range(8)]
    rows = bench.parity_rows(FakeCtx(), lambda q: blocks[q], n, 4)
    assert rows[0] == 0 and 4095 in rows and 28672 in rows and n - 1 in rows
    assert all(r < 4096 or r >= 28672 for r in rows)
    # compare_rows: the diagonal is ignored, every other entry of a row is its source's own
    sample = np.array([0, 3], np.int32)
    lat = np.arange(2 * 6, dtype=np.uint64).reshape(2, 6)
    rel = np.linspace(0.5, 1.0, 12).reshape(2, 6)
    lat2, rel2 = lat.copy(), rel.copy()
    lat2[0, 0] += 7          # diagonal: own rule, not compared
    rel2[1, 3] = 0.0
    r = bench.compare_rows(sample, 6, lat2, rel2, lat, rel)
    assert r["lat_bit_exact"] and r["rel_max_rel_err"] == 0.0 and r["rel_exact_frac"] == 1.0
    rel2[1, 1] *= 1.0 + 1e-9  # t < s: compared too (no mirror)
    r = bench.compare_rows(sample, 6, lat2, rel2, lat, rel)
    assert r["lat_bit_exact"] and r["rel_max_rel_err"] > 0.0
    lat2[1, 5] += 1
    r = bench.compare_rows(sample, 6, lat2, rel2, lat, rel)
    assert not r["lat_bit_exact"]


def test_form_keys_documented_and_few():
    """SRT_FORM: the library reads at most ten keys, every one of them listed
    in the §5 table, and the table lists no key the library does not read."""
    import glob
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    used = set()
    for f in glob.glob(os.path.join(root, "shadow_amd", "csrc", "*.*")):
        used |= set(re.findall(r'srt_form_(?:int|is)\("([a-z0-9_]+)"', open(f).read()))
    doc = open(os.path.join(root, "INTEGRATION.md")).read()
    sec = doc[doc.index("## 5."):]
    sec = sec[:sec.index("\n## ", 4)] if "\n## " in sec[4:] else sec
    listed = set(re.findall(r"^\| `([a-z0-9_]+)` \|", sec, re.M)) - {"SRT_LOG_LEVEL",
                                                                    "SRT_VIRTUAL_RANKS", "SRT_FORM"}
    assert len(used) <= 10, sorted(used)
    assert used == listed, (sorted(used - listed), sorted(listed - used))
