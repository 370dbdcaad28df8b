#!/usr/bin/env python3
"""Routing-table build benchmark (BASELINE.json metric: build time & node-pairs/s, GB/s vs HBM).

A "step" is one complete routing-table build on device-resident synthetic input: distances
(blocked Floyd-Warshall, pivot-row panels broadcast over RCCL when sharded), canonical
predecessors, path-order reliabilities, the undirected symmetry mirror and the diagonal rule.
value = whole-job node-pairs/s = n^2 * steps / (max over ranks of the timed region).

Default workload C4: the 32,768-node complete graph the north-star target is
quoted on; it fits one MI355X (w 4 GiB + r 8 GiB + lat 4 GiB + rel 8 GiB), so the same graph runs
at 1/2/4/8 GPUs (strong scaling, rows sharded across ranks). `--workload c2` runs the 1,000-node
complete graph of configs[1].

Launch: python bench.py [--gpus 1]  or  torchrun --nproc-per-node N bench.py --gpus N
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
import torch  # noqa: E402  (before the library: one HIP runtime)
import torch.distributed as dist  # noqa: E402

from shadow_amd import _lib  # noqa: E402

WORKLOADS = {
    "c4": dict(n=32768, seed=4, lat_max=1000, self_max=10, loss_max=500,
               desc="C4: 32768-node complete graph, latency U{1..1000} ms, loss U{0..500}e-4"),
    "c2": dict(n=1000, seed=2, lat_max=300, self_max=10, loss_max=500,
               desc="C2: 1000-node complete graph, latency U{1..300} ms, loss U{0..500}e-4"),
}
METRIC = "routing-table build time & node-pairs/sec (GB/s vs HBM peak), 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md, HBM3E spec peak
# VALU: 256 CU x 4 SIMD x 64 lanes x 2.4 GHz = 157.3 T lane-cycles/s; a wave64 relaxation costs
# `cyc_per_relax` SIMD cycles under the issue model below, so the relaxation roof is
# 157.3 T / cyc_per_relax.
VALU_LANE_CYCLES_T = 256 * 4 * 64 * 2.4e9 / 1e12
FW_B = 64
SHARD_ALIGN = 128  # row-shard / update-tile alignment (srt_device.h SRT_SHARD_ALIGN)


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="budget of the CPU-baseline sample (rank 0, N=1 only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    assert torch.cuda.is_available(), "bench.py needs MI355X GPUs"
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    L = _lib.lib()
    wl = WORKLOADS[args.workload]
    n = wl["n"]
    ld = (n + SHARD_ALIGN - 1) // SHARD_ALIGN * SHARD_ALIGN
    b, e = ctypes.c_int32(), ctypes.c_int32()
    L.srt_shard_rows(ld, SHARD_ALIGN, world, rank, ctypes.byref(b), ctypes.byref(e))
    b, e = b.value, e.value
    nr = e - b
    stream = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(stream.cuda_stream)

    # device-resident synthetic input (outside the timed region)
    w = torch.empty((max(nr, 1), ld), dtype=torch.int32, device=dev)
    r = torch.empty((max(nr, 1), ld), dtype=torch.float64, device=dev)
    lat = torch.empty_like(w)
    rel = torch.empty_like(r)
    _lib.check(L.srt_gen_complete_device(n, ld, b, nr, wl["seed"], wl["lat_max"], wl["self_max"],
                                         wl["loss_max"], w.data_ptr(), r.data_ptr(), sp),
               "srt_gen_complete_device")
    comm = ctypes.c_void_p()
    if world > 1:
        uid = torch.zeros(128, dtype=torch.uint8, device=dev)
        if rank == 0:
            h = (ctypes.c_uint8 * 128)()
            _lib.check(L.srt_comm_unique_id(h), "srt_comm_unique_id")
            uid.copy_(torch.tensor(list(bytes(h)), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        hid = (ctypes.c_uint8 * 128)(*uid.cpu().tolist())
        _lib.check(L.srt_comm_init(hid, world, rank, local_rank, ctypes.byref(comm)), "srt_comm_init")
    torch.cuda.synchronize()

    def step(stats=None):
        sptr = ctypes.byref(stats) if stats is not None else None
        if world == 1:
            rc = L.srt_dense_build_device(n, ld, 0, w.data_ptr(), r.data_ptr(), lat.data_ptr(),
                                          rel.data_ptr(), sp, 0, sptr)
        else:
            rc = L.srt_dense_build_sharded(comm, n, ld, 0, w.data_ptr(), r.data_ptr(),
                                           lat.data_ptr(), rel.data_ptr(), sp, 0, sptr)
        _lib.check(rc, "build")

    for i in range(args.warmup):
        step()
        log(rank, f"[bench] warmup {i + 1}/{args.warmup} done")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stats = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        st = _lib.BuildStats()
        st.time_kernels = 1
        step(st)
        stats.append(st)
        log(rank, f"[bench] step {i + 1}/{args.steps}: {st.ms_total:.1f} ms "
                  f"(fw {st.ms_fw:.1f}, post {st.ms_post:.1f})")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = elapsed * 1e3 / args.steps
    pairs = float(n) * float(n)
    value = pairs * args.steps / elapsed

    # dominant kernel: the FW update (phase 3) launches, timed with HIP events on `stream`
    n_upd = sum(s.n_update for s in stats)
    ms_upd = sum(s.ms_update for s in stats)
    avg_upd_ms = ms_upd / max(n_upd, 1)
    enc = int(stats[-1].dist_enc)  # 3: u16 + f16-compare mins, 2: u16 pk_min, 1: u32
    s_d = 4 if enc == 1 else 2
    # VALU issue model per wave64 relaxation (cycles per SIMD): full-rate ops (v_add_u32) issue in
    # 2 cycles, packed / 3-input ops (v_pk_minimum3_f16, v_pk_min_u16, v_min3_u32) in 4
    # (profiles/r01_valu_issue_rates*.txt):
    #   enc 3: 2 x v_add_u32 + 1 x v_pk_minimum3_f16 per 4 relaxations -> 8/4 = 2.0 cycles
    #   enc 2: 1 x v_add_u32 + 1 x v_pk_min_u16 per 2 relaxations      -> 6/2 = 3.0 cycles
    #   enc 1: 2 x v_add_u32 + 1 x v_min3_u32 per 2 relaxations         -> 8/2 = 4.0 cycles
    cyc_per_relax = {3: 2.0, 2: 3.0, 1: 4.0}[enc]
    instr_per_relax = {3: 0.75, 2: 1.0, 1: 1.5}[enc]
    kname = {3: "fwh_update_kernel", 2: "fw16_update_kernel<false>", 1: "fw_update_kernel"}[enc]
    bytes_per_launch = 2.0 * nr * ld * s_d  # round-streaming model: read + write the local rows
    relax_per_launch = float(nr) * ld * FW_B
    achieved_gbs = bytes_per_launch / (avg_upd_ms * 1e-3) / 1e9
    relax_t = relax_per_launch / (avg_upd_ms * 1e-3) / 1e12
    relax_peak_t = VALU_LANE_CYCLES_T / cyc_per_relax
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.workload}_n{world}.json")
    if os.path.exists(pmc_path):
        traffic = json.load(open(pmc_path)).get("hbm_bytes_per_launch")
    roofline = {
        # the north-star metric is GB/s vs HBM peak; the kernel itself is VALU-issue bound (min-plus
        # has no MFMA form), so the binding roof is reported beside it under "valu"
        "bound": "hbm", "binding": "valu-issue",
        "kernel": kname,
        "achieved": round(achieved_gbs, 1),
        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
        "traffic": traffic, "bytes_per_launch": bytes_per_launch,
        "avg_launch_ms": round(avg_upd_ms, 4), "launches_timed": n_upd,
        "model": f"2*rows*ld*{s_d} B per round (SURVEY §8d round-streaming, B=64, "
                 f"{ {3: 'u16 f16-compare', 2: 'u16 pk_min', 1: 'u32'}[enc]} distances)",
        "algorithmic_min_bytes": float(nr) * ld * (4 + 8),
        "valu": {"achieved": round(relax_t, 2), "peak": round(relax_peak_t, 1),
                 "unit": "Trelax/s", "frac": round(relax_t / relax_peak_t, 4),
                 "instr_per_relax": instr_per_relax, "cycles_per_relax": cyc_per_relax,
                 "relax_per_launch": relax_per_launch,
                 "peak_basis": "256 CU x 4 SIMD x 64 lanes x 2.4 GHz / cycles_per_relax "
                               "(v_add_u32 2 cycles, packed/3-input ops 4 cycles per wave64)"},
    }

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle  # cpu_baseline leg only
        one = np.array([17 % n], np.int32)
        _, _, _, t1 = oracle.complete_sample(n, wl["seed"], wl["lat_max"], wl["self_max"],
                                             wl["loss_max"], one, 1)
        k = int(max(2, min(64, args.cpu_seconds / max(t1, 1e-3))))
        srcs = np.unique(np.linspace(0, n - 1, k).astype(np.int32))
        clat, crel, gen_s, sssp_s = oracle.complete_sample(n, wl["seed"], wl["lat_max"],
                                                           wl["self_max"], wl["loss_max"], srcs, 1)
        cpu = {"value": round(len(srcs) * n / sssp_s, 1), "unit": "node-pairs/s", "cores": 1,
               "kind": "port",
               "sample": f"{len(srcs)} of {n} sources, dense O(n^2) Dijkstra per source "
                         f"(oracle/oracle.c orc_complete_sample), {sssp_s:.1f} s, 1 thread "
                         f"(the reference serializes Dijkstra on graphLock, topology.c:130-148); "
                         f"matrix generation ({gen_s:.1f} s) excluded",
               "speedup": round(value / (len(srcs) * n / sssp_s), 1)}
        # full-size parity spot check of the last step's rows against the oracle
        glat = lat[srcs.astype(np.int64)].cpu().numpy().view(np.uint32)[:, :n].astype(np.uint64) \
            * np.uint64(1_000_000)
        grel = rel[srcs.astype(np.int64)].cpu().numpy()[:, :n]
        upper = np.arange(n)[None, :] > srcs[:, None]
        diag = np.arange(n)[None, :] == srcs[:, None]
        lat_ok = bool(np.array_equal(np.where(diag, 0, glat), np.where(diag, 0, clat)))
        rerr = np.abs(grel - crel) / np.maximum(crel, 1e-300)
        parity = {"rows_checked": int(len(srcs)), "lat_bit_exact": lat_ok,
                  "rel_max_rel_err_upper": float(rerr[upper].max()) if upper.any() else 0.0,
                  "rel_exact_frac_upper": float((grel[upper] == crel[upper]).mean())
                  if upper.any() else 1.0}

    if rank == 0:
        s0 = stats[-1]
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "node-pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "u32" if enc == 1 else "u16",  # integer latency quanta
            "data": "synthetic",
            "config": {"workload": wl["desc"], "n": n, "ld": ld, "fw_block": FW_B,
                       "parallelism": f"row-shard x{world}" + (" + RCCL pivot-panel broadcast"
                                                               if world > 1 else ""),
                       "rows_per_rank": nr, "ess_arcs": int(s0.ess_arcs),
                       "max_tree_depth": int(s0.max_depth),
                       "ms_fw": round(s0.ms_fw, 3), "ms_post": round(s0.ms_post, 3)},
            "roofline": roofline, "cpu_baseline": cpu, "parity": parity,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        L.srt_comm_free(comm)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
