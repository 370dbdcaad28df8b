"""HIP path vs the CPU oracle, through the C-ABI (run on an MI355X with -m gpu).

Latency tables must be bit-exact in integer ns; reliability must be within 1e-12 relative
(north_star). Because the GPU forms the product in the same path order as the oracle
(topology.c:1364-1365) the match is in fact exact; the tolerance is the contract.
"""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, set_form
from shadow_amd import graphs
from shadow_amd._lib import ALGO_DENSE_FW, ALGO_SPARSE_SSSP
from shadow_amd.topology import Topology, build_tables

pytestmark = pytest.mark.gpu
REL_TOL = 1e-12
MS = 1_000_000


def assert_tables(lat_ns, rel, exp_lat, exp_rel, what=""):
    exp_lat = np.asarray(exp_lat, dtype=np.uint64)
    bad = np.argwhere(lat_ns != exp_lat)
    assert bad.size == 0, f"{what}: {len(bad)} latency mismatches, first {bad[:5].tolist()}"
    err = np.abs(rel - exp_rel) / np.maximum(np.abs(exp_rel), 1e-300)
    assert float(err.max()) <= REL_TOL, f"{what}: max rel error {err.max()}"


def _oracle(g, use_sp=True, nthreads=8):
    """The oracle's raw per-source table: the product's tables hold every source's own row."""
    el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
    return oracle.table(el, use_sp, oracle.ORC_INT_NS, nthreads, raw=True)


def test_known_answers(gpu):
    for c in json.load(open(os.path.join(GOLDEN, "known_answers.json"))):
        top = Topology.from_gml(c["gml"])
        lat, rel = top.table()
        for s, d, lat_ns, r in c["pairs"]:
            assert int(lat[s, d]) == lat_ns and rel[s, d] == r, c["name"]


@pytest.mark.parametrize("algo", [ALGO_DENSE_FW, ALGO_SPARSE_SSSP])
def test_tie_graphs(gpu, algo):
    for c in json.load(open(os.path.join(GOLDEN, "ties.json"))):
        e = np.array(c["edges"], dtype=np.float64)
        lat, rel, _ = build_tables(c["n"], c["directed"], e[:, 0], e[:, 1],
                                   (e[:, 2] * MS).astype(np.int64), e[:, 3], algo=algo)
        for s, d, lat_ns, r in c["pairs"]:
            assert int(lat[s, d]) == lat_ns, (c["name"], s, d)
            assert rel[s, d] == r, (c["name"], s, d)


def test_c1_golden_through_gml(gpu):
    """C1: GML text -> topology_new path -> GPU tables == committed oracle/networkx tables."""
    text = open(os.path.join(GOLDEN, "c1.gml")).read()
    top = Topology.from_gml(text)
    assert top.n == 50 and top.complete and not top.directed
    lat, rel = top.table()
    exp = np.load(os.path.join(GOLDEN, "c1_expected.npz"))
    assert_tables(lat, rel, exp["lat_ns"], exp["rel"], "C1")
    assert np.array_equal(rel, exp["rel"])  # same path, same multiplication order


@pytest.mark.parametrize("algo,square", [(ALGO_DENSE_FW, "1"), (ALGO_DENSE_FW, "0"),
                                          (ALGO_SPARSE_SSSP, "1")])
def test_c2_complete_1000(gpu, monkeypatch, algo, square):
    """C2's full table; the dense build by min-plus squaring (its default at ld <= 2048, encoding
    11) and by the 256-pivot FW rounds (SRT_FORM square=0)."""
    set_form(monkeypatch, square=square)
    g = graphs.complete_graph(1000, seed=2)
    lat, rel, st = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss, algo=algo)
    exp = _oracle(g)
    assert_tables(lat, rel, exp["lat_int"], exp["rel"], f"C2 algo={algo}")
    if algo == ALGO_DENSE_FW:
        assert (st.dist_enc == 11) == (square == "1"), st.dist_enc


@pytest.mark.parametrize("n", [257, 3000])
def test_sparse_rgg(gpu, n):
    g = graphs.random_geometric(n, seed=3)
    lat, rel, st = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss, algo=ALGO_SPARSE_SSSP)
    exp = _oracle(g)
    assert_tables(lat, rel, exp["lat_int"], exp["rel"], f"RGG{n} sparse")
    lat2, rel2, _ = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss, algo=ALGO_DENSE_FW)
    assert_tables(lat2, rel2, exp["lat_int"], exp["rel"], f"RGG{n} dense")


def test_barabasi_albert_small(gpu):
    g = graphs.barabasi_albert(2000, seed=5)
    exp = _oracle(g)
    for algo in (ALGO_SPARSE_SSSP, ALGO_DENSE_FW):
        lat, rel, _ = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss, algo=algo)
        assert_tables(lat, rel, exp["lat_int"], exp["rel"], f"BA2000 algo={algo}")


@pytest.mark.parametrize("algo", [ALGO_DENSE_FW, ALGO_SPARSE_SSSP])
def test_directed_random(gpu, algo):
    rng = np.random.default_rng(11)
    n, m = 300, 2400
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    ring = np.arange(n)  # strongly connected backbone
    src = np.concatenate([src, ring, ring]).astype(np.int32)
    dst = np.concatenate([dst, (ring + 1) % n, ring]).astype(np.int32)
    lat = (rng.integers(1, 20, len(src)) * MS).astype(np.int64)
    loss = rng.integers(0, 300, len(src)) / 10000.0
    g = graphs.Graph(n, True, src, dst, lat, loss)
    lat_ns, rel, _ = build_tables(n, True, src, dst, lat, loss, algo=algo)
    exp = _oracle(g)
    assert_tables(lat_ns, rel, exp["lat_int"], exp["rel"], "directed")


def test_direct_mode(gpu):
    g = graphs.complete_graph(70, seed=4)
    lat, rel, _ = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss, use_shortest_path=False)
    exp = _oracle(g, use_sp=False)
    assert_tables(lat, rel, exp["lat_int"], exp["rel"], "direct")


def test_lookup_api_end_to_end(gpu):
    """attach -> getLatency/getReliability/isRoutable/incrementPathPacketCounter (worker.c:542-554),
    served in the reference's lazy-cache order (oracle/lazy_cache.py)."""
    from oracle.lazy_cache import LazyPathCache
    g = graphs.complete_graph(40, seed=7)
    top = Topology.from_gml(graphs.to_gml(g))
    exp = _oracle(g)
    sim = LazyPathCache(exp, directed=False)
    ips = []
    for v in range(40):
        ip = f"11.0.0.{v + 1}"
        vert, down, up, _ = top.attach(f"100.0.{v}.1", 1, ip_hint=ip)
        assert vert == v and down == up == 1_000_000_000 // 8192
        ips.append(f"100.0.{v}.1")
        sim.attach(ips[-1], v)
    for s in range(0, 40, 3):
        for d in range(0, 40, 5)[::-1]:
            assert top.get_latency(ips[s], ips[d]) == sim.get_latency(ips[s], ips[d])
            assert top.get_latency(ips[s], ips[d]) == int(exp["lat_int"][s, d]) / 1e6
            assert top.get_reliability(ips[s], ips[d]) == sim.get_reliability(ips[s], ips[d])
            assert top.is_routable(ips[s], ips[d])
    assert top.get_latency(ips[0], "9.9.9.9") == -1
    assert not top.is_routable("9.9.9.9", ips[0])
    top.increment_path_packet_counter(ips[1], ips[2])
    top.increment_path_packet_counter(ips[2], ips[1])  # undirected: one counter per pair
    assert top.packet_count(ips[1], ips[2]) == 2
    # runahead export: min over attached pairs incl. the diagonal
    assert top.min_latency_ms() == int(exp["lat_int"].min()) / 1e6


def test_device_generator_matches_host(gpu):
    import torch
    from shadow_amd._lib import lib
    n, ld = 300, 320
    w = torch.empty((ld, ld), dtype=torch.int32, device="cuda")
    r = torch.empty((ld, ld), dtype=torch.float64, device="cuda")
    rc = lib().srt_gen_complete_device(n, ld, 0, ld, 4, 1000, 10, 500, w.data_ptr(), r.data_ptr(),
                                       None)
    assert rc == 0
    torch.cuda.synchronize()
    hw, hr = graphs.complete_dense(n, 4, lat_max=1000, self_max=10, loss_max=500)
    assert np.array_equal(w[:n, :n].cpu().numpy().view(np.uint32), hw)
    assert np.array_equal(r[:n, :n].cpu().numpy(), hr)


def test_dense_device_api_and_sharded_single_rank(gpu):
    """srt_dense_build_device and srt_dense_build_sharded (1-rank RCCL comm) on device data."""
    import torch
    from shadow_amd._lib import BuildStats, lib
    n, ld = 700, 768
    w = torch.empty((ld, ld), dtype=torch.int32, device="cuda")
    r = torch.empty((ld, ld), dtype=torch.float64, device="cuda")
    L = lib()
    assert L.srt_gen_complete_device(n, ld, 0, ld, 8, 300, 10, 500, w.data_ptr(), r.data_ptr(),
                                     None) == 0
    lat = torch.empty_like(w)
    rel = torch.empty_like(r)
    st = BuildStats()
    assert L.srt_dense_build_device(n, ld, 0, w.data_ptr(), r.data_ptr(), lat.data_ptr(),
                                    rel.data_ptr(), None, 0, ctypes.byref(st)) == 0
    torch.cuda.synchronize()
    g = graphs.complete_graph(n, seed=8)
    exp = _oracle(g)
    lat_ns = lat[:n, :n].cpu().numpy().view(np.uint32).astype(np.uint64) * np.uint64(MS)
    assert_tables(lat_ns, rel[:n, :n].cpu().numpy(), exp["lat_int"], exp["rel"], "device api")
    uid = (ctypes.c_uint8 * 128)()
    assert L.srt_comm_unique_id(uid) == 0
    comm = ctypes.c_void_p()
    assert L.srt_comm_init(uid, 1, 0, torch.cuda.current_device(), ctypes.byref(comm)) == 0
    lat2 = torch.empty_like(w)
    rel2 = torch.empty_like(r)
    assert L.srt_dense_build_sharded(comm, n, ld, 0, w.data_ptr(), r.data_ptr(), lat2.data_ptr(),
                                     rel2.data_ptr(), None, 0, None) == 0
    torch.cuda.synchronize()
    L.srt_comm_free(comm)
    assert torch.equal(lat2[:n, :n], lat[:n, :n]) and torch.equal(rel2[:n, :n], rel[:n, :n])


@pytest.mark.parametrize("hop_ms,enc,sym,env", [
    (1, 4, "1", {}), (1, 3, "0", {}), (160, 2, "1", {}), (400, 1, "1", {}),
    (1, 11, "1", {"square": "1"}), (1, 11, "0", {"square": "1"}), (160, 2, "1", {"square": "1"})])
def test_dense_distance_encoding_tiers(gpu, monkeypatch, hop_ms, enc, sym, env):
    """Each distance encoding of the dense build (fw16.hip) is exact where it is chosen.

    A 256-vertex ring with hop latencies hop_ms / hop_ms+1 (gcd 1 ms) plus a few chords: the
    largest distance is ~128 * hop_ms quanta, so hop_ms = 1 fits the f16-compare path (cap
    0x3DFF), 160 saturates it and falls back to the u16 pk_min path (cap 0x7FFF), and 400
    saturates both and ends on the u32 kernels. Every tier must match the oracle bit for bit.
    The graph is undirected, so the f16-compare tier runs its upper-triangle form (encoding 4)
    unless SRT_FORM sym=0 forces every tile (encoding 3); the two-stream forms (encodings 6 and 7)
    start at n = 8,192 (test_dense_round_sizes_multi_round). The round
    schedules are forced with square=0: by default a matrix of ld <= 2048 takes min-plus squaring to a fixed
    point (encoding 11) -- on this ring, ~128-arc paths, so seven or more passes; at hop 160 the
    squaring saturates the f16-compare cap and the build falls back to the u16 rounds (2).
    """
    set_form(monkeypatch, sym=sym, square="0")
    set_form(monkeypatch, **env)
    n = 256
    rng = np.random.default_rng(hop_ms)
    src = list(range(n))
    dst = [(i + 1) % n for i in range(n)]
    lat = [(hop_ms + (i % 2)) * MS for i in range(n)]
    for _ in range(12):  # long chords keep the diameter large but break the ring's ties
        a, b = (int(x) for x in rng.choice(n, 2, replace=False))
        src.append(a)
        dst.append(b)
        lat.append(int(hop_ms * n // 3) * MS)
    loss = rng.integers(0, 100, len(src)) * 1e-4
    g = graphs.Graph(n, 0, np.array(src, np.int32), np.array(dst, np.int32),
                     np.array(lat, np.int64), loss)
    got_lat, got_rel, st = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss,
                                        algo=ALGO_DENSE_FW)
    exp = _oracle(g)
    assert_tables(got_lat, got_rel, exp["lat_int"], exp["rel"], f"hop {hop_ms} ms")
    assert st.dist_enc == enc, f"expected encoding {enc}, build used {st.dist_enc}"


@pytest.mark.parametrize("n,enc", [(8192, 7), (8200, 6)])
def test_dense_round_sizes_multi_round(gpu, monkeypatch, n, enc):
    """The two-stream schedules of the one-GPU FW (from ld = 8,192): 256-pivot rounds where ld is
    a multiple of 256 (encoding 7), 128-pivot rounds otherwise (n = 8,200: ld = 8,320, encoding
    6). A ring with chords, distances of a few thousand quanta (past the level budget, so the FW
    runs), sampled rows against the oracle bit for bit: the chain stream's cross updates between
    a round's panels and the rest launches that start past them."""
    set_form(monkeypatch, levels="0")
    rng = np.random.default_rng(n)
    src = list(range(n))
    dst = [(i + 1) % n for i in range(n)]
    lat = [(1 + (i % 3)) * MS for i in range(n)]
    for _ in range(40):
        a, b = (int(x) for x in rng.choice(n, 2, replace=False))
        src.append(a)
        dst.append(b)
        lat.append(int(rng.integers(5, 60)) * MS)
    loss = rng.integers(0, 100, len(src)) * 1e-4
    g = graphs.Graph(n, 0, np.array(src, np.int32), np.array(dst, np.int32),
                     np.array(lat, np.int64), loss)
    got_lat, got_rel, st = build_tables(g.n, False, g.src, g.dst, g.lat_ns, g.loss,
                                        algo=ALGO_DENSE_FW)
    assert st.dist_enc == enc, st.dist_enc
    rows = np.r_[0:8, n // 2:n // 2 + 8, n - 8:n].astype(np.int32)
    exp = oracle.sssp_list(oracle.EdgeList(g.n, False, g.src, g.dst, g.lat_ns, g.loss), rows,
                           nthreads=8)
    off = np.arange(n)[None, :] != rows[:, None]
    assert np.array_equal(np.where(off, got_lat[rows], 0), np.where(off, exp["lat_int"], 0))
    err = np.abs(got_rel[rows] - exp["rel"]) / np.maximum(np.abs(exp["rel"]), 1e-300)
    assert float(err[off].max()) <= REL_TOL


@pytest.mark.parametrize("n,seed", [(700, 8), (1000, 2)])
def test_dense_lookahead_schedule_one_gpu(gpu, monkeypatch, n, seed):
    """The single-GPU entry (upper-triangle rounds on one stream) and the 1-rank sharded entry
    (the sharded FW's lookahead schedule: split update, pivot panel k+1 on the high-priority
    stream, double-buffered receive panels) give the oracle's tables, and the same ones."""
    import torch
    from shadow_amd._lib import lib
    set_form(monkeypatch, square="0")
    ld = (n + 127) // 128 * 128
    L = lib()
    w = torch.empty((ld, ld), dtype=torch.int32, device="cuda")
    r = torch.empty((ld, ld), dtype=torch.float64, device="cuda")
    assert L.srt_gen_complete_device(n, ld, 0, ld, seed, 300, 10, 500, w.data_ptr(), r.data_ptr(),
                                     None) == 0
    exp = _oracle(graphs.complete_graph(n, seed=seed))
    lat = torch.empty_like(w)
    rel = torch.empty_like(r)
    assert L.srt_dense_build_device(n, ld, 0, w.data_ptr(), r.data_ptr(), lat.data_ptr(),
                                    rel.data_ptr(), None, 0, None) == 0
    torch.cuda.synchronize()
    lat_ns = lat[:n, :n].cpu().numpy().view(np.uint32).astype(np.uint64) * np.uint64(MS)
    assert_tables(lat_ns, rel[:n, :n].cpu().numpy(), exp["lat_int"], exp["rel"], "lookahead")
    uid = (ctypes.c_uint8 * 128)()
    assert L.srt_comm_unique_id(uid) == 0
    comm = ctypes.c_void_p()
    assert L.srt_comm_init(uid, 1, 0, torch.cuda.current_device(), ctypes.byref(comm)) == 0
    lat2 = torch.empty_like(w)
    rel2 = torch.empty_like(r)
    assert L.srt_dense_build_sharded(comm, n, ld, 0, w.data_ptr(), r.data_ptr(), lat2.data_ptr(),
                                     rel2.data_ptr(), None, 0, None) == 0
    torch.cuda.synchronize()
    L.srt_comm_free(comm)
    assert torch.equal(lat2[:n, :n], lat[:n, :n]) and torch.equal(rel2[:n, :n], rel[:n, :n])


@pytest.mark.parametrize("kind", ["dense", "sparse", "directed"])
@pytest.mark.parametrize("ngpus", [1, 8])
def test_in_process_multi_gpu_build(gpu, kind, ngpus):
    """srt_build_tables_multi (Shadow's one-process form: a host thread per GPU, communicators from
    ncclCommInitAll, sharded kernels + RCCL) equals the oracle; ngpus is clamped to the devices
    present, so on a one-GPU box both requests exercise the threaded path with one rank."""
    if kind == "dense":
        g = graphs.complete_graph(700, seed=9)
        algo = ALGO_DENSE_FW
    elif kind == "sparse":
        g = graphs.random_geometric(1500, seed=3)
        algo = ALGO_SPARSE_SSSP
    else:
        rng = np.random.default_rng(21)
        n, m = 300, 2500
        ring = np.arange(n)
        src = np.concatenate([rng.integers(0, n, m), ring]).astype(np.int32)
        dst = np.concatenate([rng.integers(0, n, m), (ring + 1) % n]).astype(np.int32)
        lat = (rng.integers(1, 30, len(src)) * MS).astype(np.int64)
        loss = rng.integers(0, 200, len(src)) / 10000.0
        g = graphs.Graph(n, True, src, dst, lat, loss)
        algo = ALGO_DENSE_FW
    lat, rel, _ = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss, algo=algo,
                               ngpus=ngpus)
    exp = _oracle(g)
    assert_tables(lat, rel, exp["lat_int"], exp["rel"], f"multi {kind} x{ngpus}")


def _ring_graph(n, hop_ms, seed):
    """Ring with hop latencies hop_ms / hop_ms+1 plus long chords (test_dense_distance_encoding_tiers)."""
    rng = np.random.default_rng(seed)
    src, dst = list(range(n)), [(i + 1) % n for i in range(n)]
    lat = [(hop_ms + (i % 2)) * MS for i in range(n)]
    for _ in range(12):
        a, b = (int(x) for x in rng.choice(n, 2, replace=False))
        src.append(a)
        dst.append(b)
        lat.append(int(hop_ms * n // 3) * MS)
    loss = rng.integers(0, 100, len(src)) * 1e-4
    return graphs.Graph(n, 0, np.array(src, np.int32), np.array(dst, np.int32),
                        np.array(lat, np.int64), loss)


@pytest.mark.parametrize("kind", ["dense", "dense2000", "ring_f16", "sparse", "directed",
                                  "ring_u16", "ring_u32"])
@pytest.mark.parametrize("ranks", [2, 3, 4])
def test_virtual_ranks_sharded_build(gpu, monkeypatch, kind, ranks):
    """The multi-rank sharded builds on ONE GPU: SRT_VIRTUAL_RANKS=R runs R ranks of
    srt_build_tables_multi on device 0, each with its own host thread, stream and workspaces, and
    the collectives (pivot-panel broadcasts under the lookahead schedule, the exact-flag
    all-reduce, the essential-arc count all-reduce and segment broadcasts, the symmetry
    exchange, the sparse all-gather) as device-to-device copies. The C host logic of the
    N-rank paths -- shard partition, owners, lookahead order, offsets of every exchange -- is
    the code the RCCL runs use; the tables must equal the oracle's. Undirected graphs on the
    f16-compare tier take the row-sharded symmetric rounds (kept-tile checkerboard, pivot-row
    gather, final transpose fill) in 128-pivot rounds (encoding 8: the band of tile row K staged
    as two half-panels, P_a closed and applied to the b rows, then P_b closed)."""
    monkeypatch.setenv("SRT_VIRTUAL_RANKS", str(ranks))
    algo = ALGO_DENSE_FW
    if kind == "dense":
        g = graphs.complete_graph(700, seed=9)
    elif kind == "dense2000":
        g = graphs.complete_graph(2000, seed=13)
    elif kind == "ring_f16":
        g = _ring_graph(1000, 1, 1)
    elif kind == "sparse":
        g = graphs.random_geometric(1500, seed=3)
        algo = ALGO_SPARSE_SSSP
    elif kind == "directed":
        rng = np.random.default_rng(21)
        n, m = 300, 2500
        ring = np.arange(n)
        src = np.concatenate([rng.integers(0, n, m), ring]).astype(np.int32)
        dst = np.concatenate([rng.integers(0, n, m), (ring + 1) % n]).astype(np.int32)
        lat = (rng.integers(1, 30, len(src)) * MS).astype(np.int64)
        loss = rng.integers(0, 200, len(src)) / 10000.0
        g = graphs.Graph(n, True, src, dst, lat, loss)
    elif kind == "ring_u16":  # saturates the f16-compare cap: u16 pk_min tier on every rank
        g = _ring_graph(384, 160, 160)  # max distance ~30.8k quanta < 0x7FFF; 3 row blocks
    else:  # saturates both u16 caps: the u32 rounds with their own panel broadcasts
        g = _ring_graph(640, 400, 400)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss, algo=algo,
                                ngpus=1)
    exp = _oracle(g)
    assert_tables(lat, rel, exp["lat_int"], exp["rel"], f"virtual x{ranks} {kind}")
    want_enc = {"dense": 8, "dense2000": 8, "ring_f16": 8, "directed": 3, "ring_u16": 2,
                "ring_u32": 1}
    if kind in want_enc:
        assert st.dist_enc == want_enc[kind], f"encoding {st.dist_enc}"


def test_packet_path_trace_replay(gpu):
    """the packet-path consumer (worker.c:541-555) on a recorded trace gives the
    reference's drop decisions, delivery delays and per-path packet counts. Expected values come
    from the committed C1 oracle tables (raw per-source rows) replayed through the reference's
    lazy cache (oracle/lazy_cache.py): delivered iff bootstrapping, chance <= rel or an empty
    payload; delay = ceil(lat_ms * 1e6) ns (worker.c:550-551)."""
    from oracle.lazy_cache import LazyPathCache
    from shadow_amd.topology import ip_to_net
    text = open(os.path.join(GOLDEN, "c1.gml")).read()
    top = Topology.from_gml(text)
    exp = np.load(os.path.join(GOLDEN, "c1_expected.npz"))
    sim = LazyPathCache({"lat_ms": exp["lat_ms"], "rel": exp["rel"]}, directed=False)
    rng = np.random.default_rng(2024)
    hosts = []
    for h in range(120):  # hosts spread over the vertices; some share a vertex
        ip = f"12.{h // 250}.{h % 250}.7"
        v, _, _, _ = top.attach(ip, rand_state=h + 1)
        hosts.append((ip_to_net(ip), v))
        sim.attach(ip_to_net(ip), v)
    k = 20000
    si = rng.integers(0, len(hosts), k)
    di = rng.integers(0, len(hosts), k)
    src = np.array([hosts[i][0] for i in si], np.uint32)
    dst = np.array([hosts[i][0] for i in di], np.uint32)
    vs = np.array([hosts[i][1] for i in si])
    vd = np.array([hosts[i][1] for i in di])
    chance = rng.random(k)
    boot = (rng.random(k) < 0.05).astype(np.uint8)
    payload = np.where(rng.random(k) < 0.1, 0, 1400).astype(np.uint64)
    delivered, delay = top.send_packets(src, dst, chance, boot, payload)
    want = np.zeros(k, bool)
    want_delay = np.zeros(k, np.uint64)
    for i in range(k):
        ok, d = sim.send_packet(int(src[i]), int(dst[i]), float(chance[i]), bool(boot[i]),
                                int(payload[i]))
        want[i] = ok
        want_delay[i] = d if ok else 0
    assert np.array_equal(delivered, want)
    assert np.array_equal(delay[want], want_delay[want])
    # the serving row matters: some delivered pair is served from its destination's row
    assert any(sim._get(int(a), int(b)) is None for a, b in zip(vs[want], vd[want]) if a != b)
    # per-path counters (topology.c:1983-1993): one Path per stored pair, both directions
    for x in sorted(set(vs) | set(vd)):
        for y in sorted(set(vs) | set(vd)):
            p = sim._get(x, y) or sim._get(y, x)
            hx = next(h for h in hosts if h[1] == x)[0]
            hy = next(h for h in hosts if h[1] == y)[0]
            assert top.packet_count(hx, hy) == (0 if p is None else p.packets), (x, y)
    # single-packet form agrees with the trace form
    ok, d = top.send_packet(src[0], dst[0], chance[0], bool(boot[0]), int(payload[0]))
    assert ok == bool(want[0]) and (not ok or d == want_delay[0])


@pytest.mark.parametrize("reltree", ["1", "0"])
def test_reliability_parent_slots_overflow(gpu, monkeypatch, reltree):
    """rel_tree_kernel keeps the values of a row's parents (targets that are some target's
    predecessor) in 7,168 LDS slots for n > 4,096. A comb -- 120 chains of 60 one-ms hops from
    vertex 0, each ending in a leaf -- gives row 0 7,200 parents (distances <= 61): that row must
    hand over to the sweeps untouched, the others (distances past 64) take the sweeps anyway.
    SRT_FORM reltree=0 runs the per-level kernel instead; both exact."""
    set_form(monkeypatch, reltree=reltree, levels="0")
    chains, depth = 120, 60
    src, dst = [], []
    v = 1
    for _ in range(chains):
        prev = 0
        for _ in range(depth + 1):
            src.append(prev)
            dst.append(v)
            prev = v
            v += 1
    n = v
    rng = np.random.default_rng(21)
    g = graphs.Graph(n, False, np.array(src, np.int32), np.array(dst, np.int32),
                     np.full(len(src), MS, np.int64), rng.integers(0, 200, len(src)) * 1e-4)
    lat, rel, st = build_tables(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss,
                                algo=ALGO_DENSE_FW)
    exp = _oracle(g)
    assert_tables(lat, rel, exp["lat_int"], exp["rel"], f"comb reltree={reltree}")
