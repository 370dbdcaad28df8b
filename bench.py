#!/usr/bin/env python3
"""Routing-table build benchmark (BASELINE.json metric: build time & node-pairs/s, GB/s vs HBM).

A "step" is one complete routing-table build on device-resident synthetic input -- the eager
replacement of the reference's per-source lazy Dijkstra (topology.c:1578-1814): distances,
canonical predecessors, path-order reliabilities, the undirected symmetry rule and the diagonal
rule. value = whole-job node-pairs/s = n^2 * steps / (max over ranks of the timed region).

Workloads:
  c4 (default)  32,768-node complete graph (configs[3]). The north-star config; it fits one
                MI355X (w 4 GiB + r 8 GiB + lat 4 GiB + rel 8 GiB), so the same graph runs at
                1/2/4/8 GPUs (strong scaling: rows sharded). Its distances end at 5 quanta, so the
                build takes the bit-parallel Dial levels (dist_enc 12); graphs whose distances pass
                the level budget take the blocked Floyd-Warshall (e.g. c4metric).
  c4metric      32,768 points in the unit square, complete graph, latency max(1, round(300 *
                dist)) ms (Tor-atlas-like metric latencies, distances of hundreds of ms): the
                blocked Floyd-Warshall regime of the same n.
  c2            1,000-node complete graph (configs[1]), min-plus squaring / blocked FW.
  c3            20,000-node random geometric graph (deg ~8), multi-source SSSP (configs[2]).
  c5            100,000-node Barabasi-Albert graph (m=3), source-sharded SSSP + ncclAllGather
                (configs[4]); 120 GB of tables per GPU.

Launch: python bench.py [--gpus N]  (N > 1 without torchrun: bench.py starts the N rank processes
itself, as child processes, before anything touches a GPU)  or  torchrun --nproc-per-node N
bench.py --gpus N.  --dry-run prints each rank's environment and exits before importing torch.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

# torch, torch.distributed and the native library are imported by _runtime() -- after the
# launcher has decided whether this process is a rank (the launcher itself never imports them)
torch = dist = _lib = None


def _runtime():
    global torch, dist, _lib
    import torch as _torch  # before the library: one HIP runtime
    import torch.distributed as _dist
    from shadow_amd import _lib as _l
    torch, dist, _lib = _torch, _dist, _l

WORKLOADS = {
    "c4": dict(kind="dense", n=32768, seed=4, lat_max=1000, self_max=10, loss_max=500,
               desc="C4: 32768-node complete graph, latency U{1..1000} ms, loss U{0..500}e-4"),
    "c4metric": dict(kind="dense", n=32768, seed=44, lat_max=0, metric=300, self_max=10,
                     loss_max=500,
                     desc="C4metric: 32768 points in the unit square, complete graph, latency "
                          "max(1, round(300*dist)) ms, loss U{0..500}e-4 (Tor-atlas-like metric "
                          "latencies)"),
    "c2": dict(kind="dense", n=1000, seed=2, lat_max=300, self_max=10, loss_max=500,
               desc="C2: 1000-node complete graph, latency U{1..300} ms, loss U{0..500}e-4"),
    "c3": dict(kind="sparse", n=20000, seed=3, gen="rgg",
               desc="C3: 20000-node random geometric graph, avg degree 8, latency "
                    "max(1, round(1000*dist)) ms, loss U{0..100}e-4"),
    "c5": dict(kind="sparse", n=100000, seed=5, gen="ba",
               desc="C5: 100000-node Barabasi-Albert graph (m=3), latency U{1..100} ms, "
                    "loss U{0..100}e-4"),
}
METRIC = "routing-table build time & node-pairs/sec (GB/s vs HBM peak), 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md, HBM3E spec peak
L2_PEAK_GBS = 34500.0            # MI355X_MICROARCH.md §L2: 4 MiB per XCD, ~34.5 TB/s aggregate
LDS_PEAK_TBS = 256 * 256 * 2.4e9 / 1e12  # 256 B/clk/CU x 256 CUs x 2.4 GHz = 157.3 TB/s
# VALU: 256 CU x 4 SIMD x 64 lanes x 2.4 GHz = 157.3 T lane-cycles/s; a wave64 relaxation costs
# `cyc_per_relax` SIMD cycles under the issue model below, so the relaxation roof is
# 157.3 T / cyc_per_relax.
VALU_LANE_CYCLES_T = 256 * 4 * 64 * 2.4e9 / 1e12
# full-rate VALU issue: one wave64 instruction per SIMD every 2 cycles (T instructions/s)
VALU_ISSUE_T = 256 * 4 * 2.4e9 / 2 / 1e12
FW_B = 64
SHARD_ALIGN = 128  # row-shard / update-tile alignment (srt_device.h SRT_SHARD_ALIGN)


def cpu_threads() -> int:
    """Host threads of the all-cores CPU leg: this process's CPU share (OMP_NUM_THREADS on the
    GPU box, 16 there; os.cpu_count() reports the whole machine), capped by the affinity set."""
    avail = len(os.sched_getaffinity(0))
    want = int(os.environ.get("OMP_NUM_THREADS") or avail)
    return max(1, min(want, avail, 64))


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


class Ctx:
    def __init__(self, args):
        self.args = args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={self.world}")
        assert torch.cuda.is_available(), "bench.py needs MI355X GPUs"
        torch.cuda.set_device(self.local_rank)
        self.dev = torch.device("cuda", self.local_rank)
        if self.world > 1:
            dist.init_process_group("nccl", device_id=self.dev)
        self.L = _lib.lib()
        self.stream = torch.cuda.Stream(device=self.dev)
        self.sp = ctypes.c_void_p(self.stream.cuda_stream)
        self.comm = ctypes.c_void_p()
        if self.world > 1:
            uid = torch.zeros(128, dtype=torch.uint8, device=self.dev)
            if self.rank == 0:
                h = (ctypes.c_uint8 * 128)()
                _lib.check(self.L.srt_comm_unique_id(h), "srt_comm_unique_id")
                uid.copy_(torch.tensor(list(bytes(h)), dtype=torch.uint8))
            dist.broadcast(uid, 0)
            hid = (ctypes.c_uint8 * 128)(*uid.cpu().tolist())
            _lib.check(self.L.srt_comm_init(hid, self.world, self.rank, self.local_rank,
                                            ctypes.byref(self.comm)), "srt_comm_init")

    def timed(self, step):
        """W warmup steps, then exactly K steps between barrier + synchronize; max over ranks."""
        a = self.args
        for i in range(a.warmup):
            step(None)
            log(self.rank, f"[bench] warmup {i + 1}/{a.warmup} done")
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        stats = []
        t0 = time.perf_counter()
        for i in range(a.steps):
            st = _lib.BuildStats()
            st.time_kernels = 1
            step(st)
            stats.append(st)
            log(self.rank, f"[bench] step {i + 1}/{a.steps}: {st.ms_total:.1f} ms "
                           f"(distances {st.ms_fw:.1f}, post {st.ms_post:.1f})")
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if self.world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, stats

    def rccl_ranks(self) -> int:
        """ranks of the RCCL communicator (ncclCommCount); 0 at N = 1 (no communicator)"""
        if self.world == 1:
            return 0
        k = ctypes.c_int32()
        _lib.check(self.L.srt_comm_count(self.comm, ctypes.byref(k)), "srt_comm_count")
        return int(k.value)

    def per_rank(self, vals):
        """every rank's list of floats, on every rank (one all_gather)"""
        t = torch.tensor(vals, dtype=torch.float64, device=self.dev)
        if self.world == 1:
            return [vals]
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t)
        return [o.cpu().tolist() for o in out]

    def close(self):
        if self.world > 1:
            self.L.srt_comm_free(self.comm)
            dist.destroy_process_group()


# ------------------------------------------------------------------------------------------
# parity helpers (outside the timed region)
# ------------------------------------------------------------------------------------------
def all_sum(c: Ctx, v: int) -> int:
    if c.world == 1:
        return v
    t = torch.tensor([v], dtype=torch.int64, device=c.dev)
    dist.all_reduce(t)
    return int(t.item())


def parity_rows(c: Ctx, rank_range, n: int, k_per_rank: int) -> np.ndarray:
    """Sample sources: k_per_rank spread over rank 0's rows and over the last rank's
    (rank_range(q) -> [a, z)), always including the last row of each."""
    out = set()
    for q in sorted({0, c.world - 1}):
        a, z = rank_range(q)
        z = min(z, n)
        if z > a:
            out.update(np.linspace(a, z - 1, k_per_rank).astype(int).tolist())
    return np.array(sorted(out), np.int32)


def dense_range(c: Ctx, n: int):
    def f(q):
        bq, eq = ctypes.c_int32(), ctypes.c_int32()
        c.L.srt_shard_rows(ld_of(n), SHARD_ALIGN, c.world, q, ctypes.byref(bq), ctypes.byref(eq))
        return bq.value, eq.value
    return f


def gather_rows(c: Ctx, sample, get_lat, get_rel, n, quantum_ns):
    """Rows of `sample` from the ranks that own them, on rank 0 (numpy): lat in ns, rel f64.
    Dense shards hold rows [b, e) locally; the last rank sends its sampled rows over the
    process group."""
    rng = dense_range(c, n)
    ld_rows = []
    owner = []
    for s in sample:
        for q in range(c.world):
            bq, eq = rng(q)
            if bq <= s < eq:
                owner.append(q)
                ld_rows.append(int(s) - bq)
                break
    owner = np.array(owner)
    glat = np.zeros((len(sample), n), np.uint64)
    grel = np.zeros((len(sample), n), np.float64)
    for q in sorted(set(owner.tolist())):
        sel = np.nonzero(owner == q)[0]
        loc = torch.tensor([ld_rows[i] for i in sel], dtype=torch.int64, device=c.dev)
        if c.rank == q:
            tl = get_lat(loc)[:, :n].contiguous()
            tr = get_rel(loc)[:, :n].contiguous()
        else:
            tl = torch.empty((len(sel), n), dtype=torch.int32, device=c.dev)
            tr = torch.empty((len(sel), n), dtype=torch.float64, device=c.dev)
        if q != 0 and c.world > 1:
            dist.broadcast(tl, src=q)
            dist.broadcast(tr, src=q)
        if c.rank == 0:
            glat[sel] = tl.cpu().numpy().view(np.uint32).astype(np.uint64) * np.uint64(quantum_ns)
            grel[sel] = tr.cpu().numpy()
    return glat, grel


def ld_of(n: int) -> int:
    return (n + SHARD_ALIGN - 1) // SHARD_ALIGN * SHARD_ALIGN


def compare_rows(sample, n, glat, grel, clat, crel) -> dict:
    """Latency bit-exact and reliability off the diagonal: every table row is its own source's
    row (the lookup layer picks which row serves a pair, pairorder.c)."""
    off = np.arange(n)[None, :] != sample[:, None]
    lat_ok = bool(np.array_equal(np.where(off, glat, 0), np.where(off, clat, 0)))
    rerr = np.abs(grel - crel) / np.maximum(crel, 1e-300)
    return {"rows_checked": int(len(sample)), "rows": [int(x) for x in sample],
            "lat_bit_exact": lat_ok,
            "rel_max_rel_err": float(rerr[off].max()) if off.any() else 0.0,
            "rel_exact_frac": float((grel[off] == crel[off]).mean()) if off.any() else 1.0}


# ------------------------------------------------------------------------------------------
# dense: Dial levels or blocked Floyd-Warshall (C2, C4, C4metric)
# ------------------------------------------------------------------------------------------
def run_dense(c: Ctx, wl):
    L, world, rank = c.L, c.world, c.rank
    n = wl["n"]
    ld = (n + SHARD_ALIGN - 1) // SHARD_ALIGN * SHARD_ALIGN
    b, e = ctypes.c_int32(), ctypes.c_int32()
    L.srt_shard_rows(ld, SHARD_ALIGN, world, rank, ctypes.byref(b), ctypes.byref(e))
    b, e = b.value, e.value
    nr = e - b
    # device-resident synthetic input (outside the timed region)
    w = torch.empty((max(nr, 1), ld), dtype=torch.int32, device=c.dev)
    r = torch.empty((max(nr, 1), ld), dtype=torch.float64, device=c.dev)
    lat = torch.empty_like(w)
    rel = torch.empty_like(r)
    gen = L.srt_gen_metric_device if wl.get("metric") else L.srt_gen_complete_device
    _lib.check(gen(n, ld, b, nr, wl["seed"], wl.get("metric") or wl["lat_max"], wl["self_max"],
                   wl["loss_max"], w.data_ptr(), r.data_ptr(), c.sp), "generate")
    torch.cuda.synchronize()

    def step(stats):
        sptr = ctypes.byref(stats) if stats is not None else None
        if world == 1:
            rc = L.srt_dense_build_device(n, ld, 0, w.data_ptr(), r.data_ptr(), lat.data_ptr(),
                                          rel.data_ptr(), c.sp, 0, sptr)
        else:
            rc = L.srt_dense_build_sharded(c.comm, n, ld, 0, w.data_ptr(), r.data_ptr(),
                                           lat.data_ptr(), rel.data_ptr(), c.sp, 0, sptr)
        _lib.check(rc, "build")

    elapsed, stats = c.timed(step)
    c.last = stats[-1]
    c.ms_comm = [float(st.ms_comm) for st in stats]
    # dominant kernel: the FW update (phase 3) of every round, timed with HIP events on the
    # stream it is launched on (per round: one launch, or two on the owner of the next block
    # under the lookahead schedule)
    n_upd = sum(s.n_update for s in stats)
    ms_upd = sum(s.ms_update for s in stats)
    avg_upd_ms = ms_upd / max(n_upd, 1)
    # 4: u16 + f16-compare mins on upper-triangle tiles (undirected), 3: the same on every tile,
    # 2: u16 pk_min, 1: u32
    enc = int(stats[-1].dist_enc)
    if enc == 12:
        return dense_levels_tail(c, wl, step, elapsed, stats, lat, rel, nr, ld)
    s_d = 4 if enc == 1 else 2
    # VALU issue model per wave64 relaxation (cycles per SIMD): full-rate ops (v_add_u32) issue in
    # 2 cycles, packed / 3-input ops (v_pk_minimum3_f16, v_pk_min_u16, v_min3_u32) in 4
    # (profiles/r01_valu_issue_rates*.txt):
    #   enc 3: 2 x v_add_u32 + 1 x v_pk_minimum3_f16 per 4 relaxations -> 8/4 = 2.0 cycles
    #   enc 2: 1 x v_add_u32 + 1 x v_pk_min_u16 per 2 relaxations      -> 6/2 = 3.0 cycles
    #   enc 1: 2 x v_add_u32 + 1 x v_min3_u32 per 2 relaxations         -> 8/2 = 4.0 cycles
    cyc_per_relax = {11: 2.0, 9: 2.0, 8: 2.0, 7: 2.0, 6: 2.0, 5: 2.0, 4: 2.0, 3: 2.0, 2: 3.0,
                     1: 4.0}[enc]
    instr_per_relax = {11: 0.75, 9: 0.75, 8: 0.75, 7: 0.75, 6: 0.75, 5: 0.75, 4: 0.75, 3: 0.75,
                       2: 1.0, 1: 1.5}[enc]
    # the 8-wave update kernel (fwq_update_kernel; third template argument: 32-pivot stages/tile)
    uk, st2 = "fwq_update_kernel", ", 2"
    kname = {11: "fwq_update_kernel<false, 20, 8>", 9: "fwq_update_kernel<true, 4, 8>", 8: "fwq_update_kernel<true, 4, 4>", 7: "fwq_update_kernel<true, 4, 8>", 6: "fwq_update_kernel<true, 4, 4>", 5: f"{uk}<true, 4{st2}>",
             4: f"{uk}<true, 0{st2}>" if world == 1 else f"{uk}<true, 4{st2}>",
             3: f"{uk}<false, 0{st2}>",
             2: "fw16_update_kernel<false>", 1: "fw_update_kernel"}[enc]
    # LDS bytes per relaxation: operand reads (fwq: 4 ds_read_b128 per 64 relaxations per lane =
    # 1 B; fwh: 6 per 128 = 0.75 B) + the staged A/B slices (sA 16 KB + sB 8 KB per 32 pivots per
    # 128x128 tile = 0.047 B)
    lds_b_per_relax = 1.0 + 24576.0 / (32 * 128 * 128)
    # elements a timed launch updates: every local row; (enc 4, one GPU) the upper-triangle 128x128
    # tiles; (enc 4, sharded) this rank's kept tiles (fw16.hip sym_kept: one orientation of each
    # tile pair) less the next pivot block's tile row and column, which run in their own launch
    tiles = ld // 128
    pivots = FW_B  # pivots applied per element per timed unit
    if enc == 11:  # ld <= 2048, one GPU: min-plus squaring D <- min(D, D (x) D); a timed unit
        # is one squaring (ld / 256 launches over every tile, ld pivots per element)
        elems = float(ld) * ld
        pivots = ld
    elif enc == 7:  # one GPU, 256-pivot rounds on two update streams: a timed unit is the pair of
        # rest launches of a round j, every upper-triangle tile but the crosses of tile rows
        # 2j + 2 and 2j + 3; of the crosses of 2j and 2j + 1 (which the chain stream updated),
        # the tiles of 2j + 1's take the last 64-pivot panel, the others of 2j's the last three
        cross2 = 2 * tiles - 1  # tiles in the crosses of two adjacent tile rows (upper)
        rest = tiles * (tiles + 1) // 2 - cross2
        c1 = tiles - 2   # cross of 2j + 1 less the next round's two tiles in it
        c0 = tiles - 3   # cross of 2j less (2j, 2j + 1) and the next round's two tiles in it
        elems = float(rest) * 128 * 128
        pivots = (float(rest - c1 - c0) * 256 + float(c1) * 64 + float(c0) * 192) / rest
    elif enc == 6:  # one GPU, 128-pivot rounds on two update streams: a timed unit is the pair of
        # rest launches of a round j, every upper-triangle tile but the cross of j + 1; the cross
        # of j (T - 1 tiles of it) takes only the second 64-pivot panel
        rest = tiles * (tiles + 1) // 2 - tiles
        elems = float(rest) * 128 * 128
        pivots = (float(rest - (tiles - 1)) * 128 + float(tiles - 1) * 64) / rest
    elif enc == 5:  # one GPU, two update streams: a timed unit is the pair of rest-of-round
        # launches (first start to last end), all upper-triangle tiles but the next pivot
        # block's tile row and column (T tiles, their own launches)
        elems = float(tiles * (tiles + 1) // 2 - tiles) * 128 * 128
    elif enc == 4 and world == 1:
        elems = float(tiles * (tiles + 1) // 2) * 128 * 128
    elif enc in (4, 8, 9):  # row-sharded symmetric rounds (8: 128, 9: 256 pivots per round)
        if enc in (8, 9):
            pivots = 128 if enc == 8 else 256
        kept = lambda i, j: i == j or ((i < j) == ((i + j) % 2 == 0))
        tb, te = b // 128, e // 128
        nkept = sum(1 for i in range(tb, te) for j in range(tiles) if kept(i, j))
        cross = (tiles // 2 / max(world, 1) + (te - tb) / 2) * (2 if enc == 9 else 1)  # row/col K1 (and K1 + 1)
        elems = float(max(nkept - cross, 1)) * 128 * 128
    else:
        elems = float(nr) * ld
    bytes_per_round = 2.0 * elems * s_d  # round-streaming model: read + write what is updated
    relax_per_round = elems * pivots
    achieved_gbs = bytes_per_round / (avg_upd_ms * 1e-3) / 1e9
    relax_t = relax_per_round / (avg_upd_ms * 1e-3) / 1e12
    relax_peak_t = VALU_LANE_CYCLES_T / cyc_per_relax
    traffic = None
    pmc = {}
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_traffic_{c.args.workload}_n{world}.json")
    if os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path))
        if pmc.get("kernel") == kname:
            traffic = pmc.get("hbm_bytes_per_launch")
            if enc in (5, 6, 7) and traffic is not None:  # the timed unit is two launches
                traffic = 2.0 * traffic
    lds = None
    if enc >= 3:
        lds_tbs = relax_per_round * lds_b_per_relax / (avg_upd_ms * 1e-3) / 1e12
        lds = {"achieved": round(lds_tbs, 2), "peak": LDS_PEAK_TBS, "unit": "TB/s",
               "frac": round(lds_tbs / LDS_PEAK_TBS, 4), "bytes_per_relax": lds_b_per_relax,
               "peak_basis": "256 B/clk/CU (ds_read_b128) x 256 CUs x 2.4 GHz "
                             "(MI355X_MICROARCH.md §LDS)"}
        if traffic is not None and pmc.get("lds_array_busy_frac") is not None:
            lds["pmc_lds_array_busy_frac"] = round(pmc["lds_array_busy_frac"], 4)
            lds["pmc_clock_ghz"] = round(pmc.get("clock_ghz", 0.0), 3)
    roofline = {
        # the north-star metric is GB/s vs HBM peak; the kernel itself is VALU-issue bound (min-plus
        # has no MFMA form), so the binding roof is reported beside it under "valu"
        "bound": "hbm", "binding": "valu-issue", "kernel": kname,
        "achieved": round(achieved_gbs, 1),
        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
        "traffic": traffic, "bytes_per_launch": bytes_per_round,
        "avg_launch_ms": round(avg_upd_ms, 4), "launches_timed": n_upd,
        "model": f"2*elements*{s_d} B per timed unit (SURVEY §8d round-streaming, "
                 f"{ {7: 'B=256 (four 64-pivot panels per C-tile residency)', 6: 'B=128 (two 64-pivot panels per C-tile residency)', 8: 'B=128 (two 64-pivot panels per C-tile residency)', 9: 'B=256 (four 64-pivot panels per C-tile residency)', 11: f'B=256 (one 256-pivot block per C-tile residency; a squaring applies all {ld} pivots)'}.get(enc, 'B=64')}, "
                 f"{ {9: 'u16 f16-compare, row-sharded kept tiles, 256-pivot rounds (unit: one round, first start to last end)', 8: 'u16 f16-compare, row-sharded kept tiles, 128-pivot rounds (unit: one round, first start to last end)', 7: 'u16 f16-compare, upper triangle on two streams, 256-pivot rounds (unit: both rest launches)', 6: 'u16 f16-compare, upper triangle on two streams, 128-pivot rounds (unit: both rest launches)', 5: 'u16 f16-compare, upper triangle on two streams (unit: both rest launches)', 4: 'u16 f16-compare, upper triangle', 3: 'u16 f16-compare', 2: 'u16 pk_min', 1: 'u32', 11: 'u16 f16-compare, min-plus squaring split over 256-pivot blocks (unit: one squaring, all its launches)'}[enc]}"
                 f" distances; elements updated per unit = {int(elems)}, "
                 f"pivots per element = {pivots:.2f})",
        "algorithmic_min_bytes": float(nr) * ld * (4 + 8),
        "lds": lds,
        "valu": {"achieved": round(relax_t, 2), "peak": round(relax_peak_t, 1),
                 "unit": "Trelax/s", "frac": round(relax_t / relax_peak_t, 4),
                 "instr_per_relax": instr_per_relax, "cycles_per_relax": cyc_per_relax,
                 "relax_per_launch": relax_per_round,
                 "peak_basis": "256 CU x 4 SIMD x 64 lanes x 2.4 GHz / cycles_per_relax "
                               "(v_add_u32 2 cycles, packed/3-input ops 4 cycles per wave64)"},
    }
    # untimed check build: the tied-pair count (srt_build_stats.tied_pairs), summed over ranks
    chk = _lib.BuildStats()
    chk.count_ties = 1
    step(chk)
    tied = all_sum(c, int(chk.tied_pairs))
    # parity rows: rank 0's first / middle / last rows and the last rank's (gathered to rank 0)
    sample = parity_rows(c, dense_range(c, n), n, k_per_rank=8)
    glat, grel = gather_rows(c, sample, lambda rr: lat[rr], lambda rr: rel[rr], n, 1_000_000)
    cpu = parity = None
    if rank == 0 and not c.args.no_cpu_baseline:
        import oracle  # cpu_baseline leg and the parity check only
        if world == 1:
            one = np.array([17 % n], np.int32)
            _, _, _, t1 = oracle.complete_sample(n, wl["seed"], wl["lat_max"], wl["self_max"],
                                                 wl["loss_max"], one, 1, metric=wl.get("metric", 0))
            k = int(max(2, min(64, c.args.cpu_seconds / max(t1, 1e-3))))
            srcs = np.unique(np.linspace(0, n - 1, k).astype(np.int32))
            _, _, gen_s, sssp_s = oracle.complete_sample(n, wl["seed"], wl["lat_max"],
                                                         wl["self_max"], wl["loss_max"], srcs, 1,
                                                         metric=wl.get("metric", 0))
            cpu = {"value": round(len(srcs) * n / sssp_s, 1), "unit": "node-pairs/s", "cores": 1,
                   "kind": "port",
                   "sample": f"{len(srcs)} of {n} sources, dense O(n^2) Dijkstra per source "
                             f"(oracle/oracle.c orc_complete_sample), {sssp_s:.1f} s, 1 thread "
                             f"(the reference serializes Dijkstra on graphLock, topology.c:130-148); "
                             f"matrix generation ({gen_s:.1f} s) excluded"}
            # all-cores leg (SURVEY §8d ii): the same per-source Dijkstra sharded over host threads
            nt = cpu_threads()
            kk = int(max(nt, min(32 * nt, nt * c.args.cpu_seconds / 2 / max(t1, 1e-3))))
            msrcs = np.unique(np.linspace(0, n - 1, kk).astype(np.int32))
            _, _, _, mt_s = oracle.complete_sample(n, wl["seed"], wl["lat_max"], wl["self_max"],
                                                   wl["loss_max"], msrcs, nt,
                                                   metric=wl.get("metric", 0))
            cpu["all_cores"] = {"value": round(len(msrcs) * n / mt_s, 1), "cores": nt,
                                "sample": f"{len(msrcs)} of {n} sources over {nt} threads, "
                                          f"{mt_s:.1f} s (no graphLock: the reference cannot do "
                                          f"this)"}
        # full-size parity of the last build's rows against the oracle
        clat, crel, _, _ = oracle.complete_sample(n, wl["seed"], wl["lat_max"], wl["self_max"],
                                                  wl["loss_max"], sample, cpu_threads(),
                                                  metric=wl.get("metric", 0))
        parity = compare_rows(sample, n, glat, grel, clat, crel)
    if parity is not None:
        parity.update({"tied_pairs": tied, "tied_frac": tied / float(n * (n - 1))})
    s0 = stats[-1]
    # pivots per round (one C-tile residency): 256 (enc 7, 9), 128 (enc 6, 8), else the 64-pivot
    # diagonal block FW_B
    round_pivots = {7: 256, 9: 256, 6: 128, 8: 128, 11: ld}.get(enc, FW_B)
    config = {"workload": wl["desc"], "n": n, "ld": ld, "pivots_per_round": round_pivots,
              "diag_block": FW_B,
              "parallelism": f"row-shard x{world}" + (" + RCCL pivot-panel broadcast"
                                                      if world > 1 else ""),
              "rows_per_rank": nr, "ess_arcs": int(s0.ess_arcs),
              "max_tree_depth": int(s0.max_depth),
              "ms_fw": round(s0.ms_fw, 3), "ms_post": round(s0.ms_post, 3)}
    return elapsed, "u32" if enc == 1 else "u16", "strong", config, roofline, cpu, parity


def dense_cpu_and_parity(c: Ctx, wl, step, lat, rel):
    """untimed: the tied-pair count (check build), the CPU baseline legs and the sampled parity"""
    n, world, rank = wl["n"], c.world, c.rank
    chk = _lib.BuildStats()
    chk.count_ties = 1
    step(chk)
    tied = all_sum(c, int(chk.tied_pairs))
    sample = parity_rows(c, dense_range(c, n), n, k_per_rank=8)
    glat, grel = gather_rows(c, sample, lambda rr: lat[rr], lambda rr: rel[rr], n, 1_000_000)
    cpu = parity = None
    if rank == 0 and not c.args.no_cpu_baseline:
        import oracle  # cpu_baseline leg and the parity check only
        if world == 1:
            one = np.array([17 % n], np.int32)
            _, _, _, t1 = oracle.complete_sample(n, wl["seed"], wl["lat_max"], wl["self_max"],
                                                 wl["loss_max"], one, 1, metric=wl.get("metric", 0))
            k = int(max(2, min(64, c.args.cpu_seconds / max(t1, 1e-3))))
            srcs = np.unique(np.linspace(0, n - 1, k).astype(np.int32))
            _, _, gen_s, sssp_s = oracle.complete_sample(n, wl["seed"], wl["lat_max"],
                                                         wl["self_max"], wl["loss_max"], srcs, 1,
                                                         metric=wl.get("metric", 0))
            cpu = {"value": round(len(srcs) * n / sssp_s, 1), "unit": "node-pairs/s", "cores": 1,
                   "kind": "port",
                   "sample": f"{len(srcs)} of {n} sources, dense O(n^2) Dijkstra per source "
                             f"(oracle/oracle.c orc_complete_sample), {sssp_s:.1f} s, 1 thread "
                             f"(the reference serializes Dijkstra on graphLock, topology.c:130-148); "
                             f"matrix generation ({gen_s:.1f} s) excluded"}
            nt = cpu_threads()
            kk = int(max(nt, min(32 * nt, nt * c.args.cpu_seconds / 2 / max(t1, 1e-3))))
            msrcs = np.unique(np.linspace(0, n - 1, kk).astype(np.int32))
            _, _, _, mt_s = oracle.complete_sample(n, wl["seed"], wl["lat_max"], wl["self_max"],
                                                   wl["loss_max"], msrcs, nt,
                                                   metric=wl.get("metric", 0))
            cpu["all_cores"] = {"value": round(len(msrcs) * n / mt_s, 1), "cores": nt,
                                "sample": f"{len(msrcs)} of {n} sources over {nt} threads, "
                                          f"{mt_s:.1f} s (no graphLock: the reference cannot do "
                                          f"this)"}
        clat, crel, _, _ = oracle.complete_sample(n, wl["seed"], wl["lat_max"], wl["self_max"],
                                                  wl["loss_max"], sample, cpu_threads(),
                                                  metric=wl.get("metric", 0))
        parity = compare_rows(sample, n, glat, grel, clat, crel)
    if parity is not None:
        parity.update({"tied_pairs": tied, "tied_frac": tied / float(n * (n - 1))})
    return cpu, parity


def dense_levels_tail(c: Ctx, wl, step, elapsed, stats, lat, rel, nr, ld):
    """Dense builds whose distances came from the bit-parallel Dial levels (levels.hip, dist_enc
    12). Three kernels carry the build, each timed by the library with HIP events on the build's
    stream (srt_build_stats: ms_update over the lvl_step launches, ms_pred, ms_rel); the roofline
    object names the one with the most time, the others are listed beside it, each against the
    roof that bounds it:
      lvl_step_kernel (per level d): its gathers are one 4-B Delta_{d-w}[k] word per (in-arc k->j
        of weight w < d, target j, 32-source word) the unit walked before its early exit --
        srt_build_stats.work_bytes, counted on the device -- served from the
        L2 / MALL (the planes are re-read by every in-arc), so they are priced against the L2 peak
        (34.5 TB/s, MI355X_MICROARCH.md); its compulsory HBM bytes (the level plane written, R read
        and written, the earlier planes read once) are reported beside them;
      lvl_pred_kernel: every level plane read once (levels x n x nsrc / 8 B) and one packed 4-B
        word per pair written (predecessor | reliability index | level);
      rel_pk_kernel: per pair the packed word read, the u32 distance and the f64 reliability
        written (4 + 4 + 8 B).
    main() adds "build": the whole step against HBM, the tables' compulsory bytes (n^2 x 12)
    over ms_per_step."""
    n, world = wl["n"], c.world
    n_upd = sum(s.n_update for s in stats)
    ms_upd = sum(s.ms_update for s in stats)
    wbytes = sum(float(s.work_bytes) for s in stats)
    s0 = stats[-1]
    k = len(stats)
    levels = int(s0.levels)
    pairs = float(nr) * n
    ntab = int(s0.rel_table)
    plane = float(n) * nr / 8.0  # one level plane: n targets x nsrc bits
    # lvl_step compulsory HBM per launch, averaged over the levels: the plane written, R read and
    # written, and each earlier plane read once
    step_hbm = sum(3.0 * plane + (d - 1) * plane for d in range(1, levels + 1)) / max(levels, 1)
    kern = {
        "lvl_step_kernel": (ms_upd / max(n_upd, 1), wbytes / max(n_upd, 1), n_upd, "l2",
                            "per level d: one 4-B Delta_{d-w}[k] word gathered per (in-arc k->j "
                            "of weight w < d, target j, 32-source word) that the unit walked -- "
                            "counted on the device, since a unit stops once its sources are all "
                            "settled or found -- served by the L2 / MALL; "
                            f"averaged over the {levels} levels of a build"),
        "lvl_pred_kernel": (sum(s.ms_pred for s in stats) / k,
                            levels * plane + pairs * 4.0, k, "hbm",
                            "every level plane read once (levels x n x nsrc / 8 B) + per pair one "
                            f"packed word (u16 predecessor | index into the {ntab} distinct arc "
                            "reliabilities | 5-bit level, 4 B)"),
        "rel_pk_kernel": (sum(s.ms_rel for s in stats) / k, pairs * 16.0, k, "hbm",
                          "per pair: the packed word read, the u32 distance and the f64 "
                          "reliability written (16 B)"),
    }
    peaks = {"hbm": HBM_PEAK_GBS, "l2": L2_PEAK_GBS}
    total = {name: v[0] * v[2] / k for name, v in kern.items()}  # ms per build
    dom = max(total, key=total.get)
    avg_ms, per_launch, launches, bound, model = kern[dom]
    achieved = per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    pmc_k = {}  # per-kernel PMC HBM bytes per launch (profiles/pmc_traffic_<wl>_n<N>.json)
    pmc_tcc = {}  # per-kernel L2 (TCC) hits and misses per launch, same file
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_traffic_{c.args.workload}_n{world}.json")
    if os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path))
        pmc_k = {kk: v.get("hbm_bytes_per_launch") for kk, v in pmc.get("kernels", {}).items()}
        pmc_tcc = {kk: (v["TCC_HIT_sum"], v["TCC_MISS_sum"]) for kk, v in pmc.get("kernels", {}).items()
                   if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v}
    others = {}
    for name, (ms, b, nl, bd, _) in kern.items():
        gbs = b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        o = {"ms_per_build": round(total[name], 3), "avg_launch_ms": round(ms, 4),
             "bound": bd, "bytes_per_launch": b, "achieved": round(gbs, 1), "peak": peaks[bd],
             "frac": round(gbs / peaks[bd], 4), "traffic": pmc_k.get(name)}
        if name == "lvl_step_kernel":
            hb = step_hbm / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
            o["hbm_compulsory"] = {"bytes_per_launch": step_hbm, "achieved": round(hb, 1),
                                   "peak": HBM_PEAK_GBS, "frac": round(hb / HBM_PEAK_GBS, 4)}
        if name in pmc_tcc and ms > 0:
            # the L2's side of the kernel: its TCC requests (hits + misses, PMC,
            # per launch) at 64 B each, over the live launch time, against the L2 peak
            hit, miss = pmc_tcc[name]
            req_b = (hit + miss) * 64.0
            l2 = req_b / (ms * 1e-3) / 1e9
            o["l2_requests"] = {"bytes_per_launch": req_b, "bytes_per_request": 64,
                                "achieved": round(l2, 1), "peak": L2_PEAK_GBS,
                                "frac": round(l2 / L2_PEAK_GBS, 4),
                                "hit_rate": round(hit / max(hit + miss, 1), 3), "source": "pmc"}
        if name == "lvl_pred_kernel":
            # neither roof binds it: its plane-slice gathers come from the L2 / MALL at a small
            # fraction of either peak, each batch waiting on the previous one
            o["limiter"] = "gather latency (L2 / MALL), below both the HBM and the L2 peak"
        others[name] = o
    amin = float(nr) * ld * (4 + 8)
    roofline = {
        "bound": bound, "kernel": dom,
        "achieved": round(achieved, 1), "peak": peaks[bound], "unit": "GB/s",
        "frac": round(achieved / peaks[bound], 4), "traffic": pmc_k.get(dom),
        "bytes_per_launch": per_launch, "avg_launch_ms": round(avg_ms, 4),
        "launches_timed": launches, "model": model, "kernels": others,
        "algorithmic_min_bytes": amin,
    }
    cpu, parity = dense_cpu_and_parity(c, wl, step, lat, rel)
    config = {"workload": wl["desc"], "n": n, "ld": ld, "distances": "bit-parallel Dial levels",
              "levels": int(s0.levels),
              # distinct arc reliabilities of the packed post pass (0: f64 rows)
              "rel_table": int(s0.rel_table),
              "parallelism": f"row-shard x{world}" + (" (one exchange and one agreement, "
                                                      "the counts all-gathered, the first "
                                                      "batch's arcs streamed weight by weight "
                                                      "under the levels, one vote per batch)"
                                                      if world > 1 else ""),
              "rows_per_rank": nr, "ess_arcs": int(s0.ess_arcs),
              "max_level": int(s0.max_depth),
              "ms_fw": round(s0.ms_fw, 3), "ms_post": round(s0.ms_post, 3)}
    return elapsed, "u32", "strong", config, roofline, cpu, parity


# ------------------------------------------------------------------------------------------
# sparse: multi-source SSSP over CSR (C3, C5)
# ------------------------------------------------------------------------------------------
def run_sparse(c: Ctx, wl):
    from shadow_amd import graphs
    from shadow_amd.topology import SparseGraph
    L, world, rank = c.L, c.world, c.rank
    n = wl["n"]
    t0 = time.perf_counter()
    g = graphs.random_geometric(n, seed=wl["seed"]) if wl["gen"] == "rgg" else \
        graphs.barabasi_albert(n, seed=wl["seed"])
    log(rank, f"[bench] generated {g.name}: {g.m} edges in {time.perf_counter() - t0:.1f} s")
    sg = SparseGraph(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss, device=c.local_rank)
    per = (n + world - 1) // world  # source block of each rank (ncclAllGather slices)
    s0, s1 = rank * per, min(n, (rank + 1) * per)
    rows_all = per * world
    lat = torch.empty((rows_all, n), dtype=torch.int32, device=c.dev)
    rel = torch.empty((rows_all, n), dtype=torch.float64, device=c.dev)
    torch.cuda.synchronize()

    comm_ms = []

    def step(stats):
        lp = lat.data_ptr() + s0 * n * 4
        rp = rel.data_ptr() + s0 * n * 8
        if s1 > s0:
            sg.rows(s0, s1, lp, rp, c.stream.cuda_stream, stats)
        if world > 1:
            ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ea.record(c.stream)
            _lib.check(L.srt_sparse_allgather(c.comm, n, per, ctypes.c_void_p(lat.data_ptr()),
                                              ctypes.c_void_p(rel.data_ptr()), c.sp),
                       "srt_sparse_allgather")
            eb.record(c.stream)
        c.stream.synchronize()
        if world > 1 and stats is not None:
            comm_ms.append(ea.elapsed_time(eb))

    elapsed, stats = c.timed(step)
    c.last = stats[-1]
    c.ms_comm = list(comm_ms) if comm_ms else [0.0] * len(stats)
    arcs = sg.arcs
    # algorithmic bytes per source: row pointers, every arc once (col 4 + w 4 +
    # reliability 8), the output row (lat 4 + rel 8)
    bytes_per_src = (n + 1) * 4 + arcs * 16 + n * 12
    nsrc = s1 - s0
    k_ms = sum(s.ms_update for s in stats) / max(sum(s.n_update for s in stats), 1)
    achieved_gbs = nsrc * bytes_per_src / (k_ms * 1e-3) / 1e9
    # the kernel the build used (srt_build_stats.dist_enc for sparse builds): 2 = workgroup per
    # source with the LDS-packed distance row, 1 = wave per source, 0 = the block kernel
    enc = int(stats[-1].dist_enc)
    # the kernel's form from the build (srt_build_stats.fw_block of sparse builds)
    form = int(stats[-1].fw_block)
    tf = lambda b: "true" if b else "false"
    kname = {3: f"msssp_kernel<{tf(g.directed)}, {'unsigned short' if form & 16 else 'unsigned int'}>",
             2: f"wgsssp_kernel<1024, true, {tf(form & 2)}>",
             1: f"wsssp_kernel<{tf(g.directed)}, {tf(form & 1)}, {tf(form & 2)}>"
             }.get(enc, "sssp_kernel")
    model = "per source: (n+1)*4 + arcs*16 + n*12 B (SURVEY §8d work-efficient gather model)"
    bytes_launch = float(nsrc * bytes_per_src)
    if enc == 3:
        # multi-source kernel: the graph and each vertex's 64-lane working state are shared by
        # the 64 sources of a batch
        nb = (nsrc + 63) // 64
        sd = 2 if form & 16 else 4  # 16-bit working distances (form bit 16)
        bytes_launch = float(nsrc * n * 12 + nb * (2 * n * 64 * (sd + 8) + (n + 1) * 8 + arcs * 16))
        model = (f"per 64-source batch: each vertex's 64-lane state (u{8 * sd} D + f64 R) written "
                 "and read once, the graph once ((n+1)*8 + arcs*16 B); per source its output row "
                 "(n*12 B)")
        achieved_gbs = bytes_launch / (k_ms * 1e-3) / 1e9
    others = None
    nder = int(stats[-1].n_derived)
    if nder:
        # derived build (fw_block bit 64): the core rows' kernel over n - nder sources (each also
        # stores its canonical arcs, 4 B per target), then derive_chain_kernel over nder rows
        # (srt_build_stats.work_bytes: the neighbours' distance rows, one neighbour's arcs, the
        # output rows). The roofline names the core kernel, the derivation is listed beside it
        ncore = nsrc - nder
        core_ms = sum(s.ms_core for s in stats) / len(stats)
        der_ms = sum(s.ms_derive for s in stats) / len(stats)
        bytes_launch = float(ncore * (bytes_per_src + n * 4))
        achieved_gbs = bytes_launch / (core_ms * 1e-3) / 1e9
        k_ms = core_ms
        model = (f"core rows ({ncore} sources): per source (n+1)*4 + arcs*16 + n*12 B (SURVEY §8d) "
                 f"+ n*4 B of canonical arcs; the other {nder} rows derived (derive_chain_kernel)")
        dbytes = float(stats[-1].work_bytes)
        others = [{"kernel": "derive_chain_kernel<1024, 16384>", "rows": nder,
                   "bytes_per_launch": dbytes, "avg_launch_ms": round(der_ms, 3),
                   "achieved": round(dbytes / (der_ms * 1e-3) / 1e9, 1),
                   "model": "per derived row: deg * n*4 B (neighbour distance rows) + n*4 B (one "
                            "optimal neighbour's canonical arcs) + n*12 B (lat + rel rows out)"}]
    traffic = None
    valu = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_traffic_{c.args.workload}_n{world}.json")
    if os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path))
        if pmc.get("kernel") == kname:
            traffic = pmc.get("hbm_bytes_per_launch")
            vi = pmc.get("SQ_INSTS_VALU_per_launch")
            if vi and k_ms > 0:
                # the VALU side: wave64 VALU instructions per launch (PMC) over
                # the live launch time, against the full-rate issue peak (256 CU x 4 SIMD, one
                # wave64 instruction per 2 cycles at 2.4 GHz)
                t = vi / (k_ms * 1e-3) / 1e12
                valu = {"instructions_per_launch": vi, "achieved": round(t, 4),
                        "peak": round(VALU_ISSUE_T, 4), "unit": "T wave-instr/s",
                        "frac": round(t / VALU_ISSUE_T, 4), "source": "pmc SQ_INSTS_VALU"}
                if pmc.get("SQ_INSTS_VALU_per_pull"):
                    valu["per_pull"] = pmc["SQ_INSTS_VALU_per_pull"]
    roofline = {"bound": "hbm", "kernel": kname,
        "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
        "bytes_per_launch": bytes_launch, "avg_launch_ms": round(k_ms, 3),
        "launches_timed": len(stats),
        "model": model,
        "relax_per_launch": float(nsrc - nder) * arcs}
    if valu:
        roofline["valu"] = valu
    if others:
        roofline["kernels"] = others
    # untimed check build: the tied-pair count over this rank's rows, summed over ranks
    chk = _lib.BuildStats()
    chk.count_ties = 1
    step(chk)
    tied = all_sum(c, int(chk.tied_pairs))
    # after the all-gather every rank holds every row: rank 0 checks its own block's and the
    # last rank's block's rows
    sample = parity_rows(c, lambda q: (q * per, (q + 1) * per), n, k_per_rank=8)
    glat = rel_rows = None
    if rank == 0:
        idx = torch.from_numpy(sample.astype(np.int64)).to(c.dev)
        glat = lat.index_select(0, idx).cpu().numpy().view(np.uint32).astype(np.uint64) \
            * np.uint64(sg.quantum_ns)
        rel_rows = rel.index_select(0, idx).cpu().numpy()
    cpu = parity = None
    if rank == 0 and not c.args.no_cpu_baseline:
        import oracle  # cpu_baseline leg and the parity check only
        el = oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss)
        if world == 1:
            t1 = time.perf_counter()
            oracle.sssp_rows(el, 0, 1)
            one = max(time.perf_counter() - t1, 1e-4)
            k = int(max(2, min(2000, c.args.cpu_seconds / one)))
            srcs = np.linspace(0, n - k, 3).astype(np.int64)  # three contiguous sample blocks
            kk = max(1, k // 3)
            t1 = time.perf_counter()
            for a in srcs:
                oracle.sssp_rows(el, int(a), int(a) + kk)
            cs = time.perf_counter() - t1
            cpu = {"value": round(3 * kk * n / cs, 1), "unit": "node-pairs/s", "cores": 1,
                   "kind": "port",
                   "sample": f"{3 * kk} of {n} sources (3 blocks of {kk}), binary-heap Dijkstra "
                             f"per source (oracle/oracle.c orc_sssp_rows), {cs:.1f} s, 1 thread "
                             f"(the reference serializes Dijkstra on graphLock, "
                             f"topology.c:130-148)"}
            nt = cpu_threads()
            mk = int(max(nt, min(256 * nt, nt * c.args.cpu_seconds / 2 / one)))
            mk = min(mk, max(nt, int(2e9 / (n * 32))))  # the oracle's output rows: <= ~2 GB
            a0 = max(0, n // 2 - mk // 2)
            t1 = time.perf_counter()
            oracle.sssp_rows(el, a0, min(n, a0 + mk), nthreads=nt)
            mt_s = time.perf_counter() - t1
            cpu["all_cores"] = {"value": round(min(mk, n - a0) * n / mt_s, 1), "cores": nt,
                                "sample": f"{min(mk, n - a0)} of {n} sources over {nt} threads, "
                                          f"{mt_s:.1f} s (no graphLock: the reference cannot do "
                                          f"this)"}
        ex = oracle.sssp_list(el, sample, nthreads=cpu_threads())
        parity = compare_rows(sample, n, glat, rel_rows, ex["lat_int"], ex["rel"])
    if parity is not None:
        parity.update({"tied_pairs": tied, "tied_frac": tied / float(n * (n - 1))})
    sg.free()
    s0st = stats[-1]
    config = {"workload": wl["desc"], "n": n, "edges": int(g.m), "arcs": int(arcs),
              "parallelism": f"source-shard x{world}" + (" + RCCL allgather" if world > 1 else ""),
              "sources_per_rank": nsrc,
              "sources_recomputed_after_bucket_overflow": int(s0st.ess_arcs),
              "kernel_form": int(s0st.fw_block),
              # srt_build_stats.fw_block bit 64: the independent set's rows derived from their
              # neighbours' (derive.hip) instead of run by the kernel
              "derived_rows": bool(int(s0st.fw_block) & 64),
              "ms_sssp": round(s0st.ms_fw, 3)}
    return elapsed, "u32", "strong", config, roofline, cpu, parity


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch(n: int) -> int:
    """`bench.py --gpus N` from a plain shell: start N rank processes of this same command line
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1), one per GPU, as
    children -- nothing here touches the GPU. Rank 0 prints the JSON line. If a rank fails, the
    others are stopped (by PID) so a peer waiting in a collective cannot hang the job. Returns the
    first non-zero exit status, else 0."""
    import signal
    import subprocess
    port = int(os.environ.get("MASTER_PORT") or free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                    "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0",
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)]
                                      + sys.argv[1:], env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print(f"[bench] rank {procs.index(p)} exited with {rc}; stopping the others",
                      file=sys.stderr, flush=True)
                stop()
        time.sleep(0.05)
    return status


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="budget of the CPU-baseline sample (rank 0, N=1 only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="print this rank's launch environment and exit before importing torch")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args.gpus))
    if args.dry_run:  # one write per line: the ranks share the launcher's stdout
        sys.stdout.write(json.dumps({"rank": int(os.environ.get("RANK", "0")),
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                          "world_size": int(os.environ.get("WORLD_SIZE", "1")),
                          "master_addr": os.environ.get("MASTER_ADDR"),
                          "master_port": os.environ.get("MASTER_PORT"),
                          "torch_imported": "torch" in sys.modules, "pid": os.getpid()}) + "\n")
        sys.stdout.flush()
        return
    _runtime()
    c = Ctx(args)
    wl = WORKLOADS[args.workload]
    runner = run_dense if wl["kind"] == "dense" else run_sparse
    elapsed, dtype, scaling, config, roofline, cpu, parity = runner(c, wl)
    n = wl["n"]
    if roofline is not None and "build" not in roofline:
        # the whole step against HBM: the tables' compulsory bytes (n^2 x (4 + 8), whole job)
        amin = float(n) * n * 12.0
        bgbs = amin / (elapsed / args.steps) / 1e9
        roofline["build"] = {"bytes": amin, "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
                             "achieved": round(bgbs, 1), "peak": HBM_PEAK_GBS,
                             "frac": round(bgbs / HBM_PEAK_GBS, 4),
                             "model": "the tables' compulsory bytes (u32 lat + f64 rel per pair, "
                                      "all ranks) over the whole timed step"}
    # per-rank split of the last timed step and the collectives' device time (all ranks)
    ms_comm = sum(c.ms_comm) / max(len(c.ms_comm), 1)
    pr = c.per_rank([float(c.last.ms_total), float(c.last.ms_fw), float(c.last.ms_post), ms_comm])
    rccl = c.rccl_ranks()
    value = float(n) * float(n) * args.steps / elapsed
    if cpu is not None:
        cpu["speedup"] = round(value / cpu["value"], 1)
    if c.rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "node-pairs/s",
            "n_gpus": c.world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None,
            "dtype": dtype,  # integer latency quanta
            "data": "synthetic", "config": config, "roofline": roofline,
            "cpu_baseline": cpu, "parity": parity,
            "rccl_ranks": rccl,
            # device time the streams spent inside collectives per step (waits for peers
            # included; the band broadcasts overlap the update, so this is not on the critical
            # path by itself), mean over the timed steps, max over ranks
            "ms_comm": round(max(p[3] for p in pr), 3),
            "per_rank": [{"rank": q, "ms_total": round(p[0], 3), "ms_fw": round(p[1], 3),
                          "ms_post": round(p[2], 3), "ms_comm": round(p[3], 3)}
                         for q, p in enumerate(pr)],
        }
        print(json.dumps(line), flush=True)
    c.close()


if __name__ == "__main__":
    main()
