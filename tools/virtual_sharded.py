#!/usr/bin/env python3
"""Full-size rehearsal of the N-rank sharded dense build on ONE GPU (virtual ranks).

Each of R host threads binds to a virtual rank on device 0 (own workspaces and streams), generates
its row block of the synthetic complete graph on the device, and runs srt_dense_build_sharded with
a virtual communicator (collectives as device-to-device copies ordered by events and host
barriers). This exercises the multi-rank host logic -- partition, owners, lookahead, pivot-row
gather, panel broadcast, final transpose fill, the post pass's all-reduce / segment broadcasts and
the symmetry exchange -- at the bench workload's full size, where offsets and buffer sizes are
largest. The ranks share the GPU, so the time is total work plus schedule overhead, not a scaling
number (the N-GPU runs are the driver's). Sampled rows are checked against the C oracle.

usage: python tools/virtual_sharded.py [--workload c4] [--ranks 2] [--rows 3]
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from shadow_amd import _lib  # noqa: E402

WORKLOADS = {
    "c4": dict(n=32768, seed=4, lat_max=1000, self_max=10, loss_max=500),
    "c2": dict(n=1000, seed=2, lat_max=300, self_max=10, loss_max=500),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--rows", type=int, default=3, help="sampled rows checked against the oracle")
    ap.add_argument("--sym", default=None, help="SRT_FORM sym override (0: all-tile rounds)")
    a = ap.parse_args()
    if a.sym is not None:
        os.environ["SRT_FORM"] = f"sym={a.sym}"
    wl = WORKLOADS[a.workload]
    n, R = wl["n"], a.ranks
    L = _lib.lib()
    ld = (n + 127) // 128 * 128
    comms = (ctypes.c_void_p * R)()
    _lib.check(L.srt_comm_init_virtual(R, 0, comms), "srt_comm_init_virtual")
    shards, bufs, streams = [], [], []
    for r in range(R):
        b, e = ctypes.c_int32(), ctypes.c_int32()
        L.srt_shard_rows(ld, 128, R, r, ctypes.byref(b), ctypes.byref(e))
        b, e = b.value, e.value
        nr = max(e - b, 1)
        w = torch.empty((nr, ld), dtype=torch.int32, device="cuda")
        rr = torch.empty((nr, ld), dtype=torch.float64, device="cuda")
        lat = torch.empty_like(w)
        rel = torch.empty_like(rr)
        st = torch.cuda.Stream()
        if e > b:
            _lib.check(L.srt_gen_complete_device(n, ld, b, e - b, wl["seed"], wl["lat_max"],
                                                 wl["self_max"], wl["loss_max"], w.data_ptr(),
                                                 rr.data_ptr(), ctypes.c_void_p(st.cuda_stream)),
                       "gen")
        shards.append((b, e))
        bufs.append((w, rr, lat, rel))
        streams.append(st)
    torch.cuda.synchronize()
    rcs = [None] * R
    stats = [_lib.BuildStats() for _ in range(R)]

    def work(r):
        L.srt_virtual_rank_bind(r, 0)
        w, rr, lat, rel = bufs[r]
        stats[r].time_kernels = 0
        rcs[r] = L.srt_dense_build_sharded(ctypes.c_void_p(comms[r]), n, ld, 0, w.data_ptr(),
                                           rr.data_ptr(), lat.data_ptr(), rel.data_ptr(),
                                           ctypes.c_void_p(streams[r].cuda_stream), 0,
                                           ctypes.byref(stats[r]))
        L.srt_virtual_rank_bind(-1, 0)

    times = []
    for rep in range(2):
        th = [threading.Thread(target=work, args=(r,)) for r in range(R)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        for r in range(R):
            _lib.check(rcs[r], f"rank {r}")
    import oracle  # test infrastructure: the checker only
    srcs = np.unique(np.linspace(0, n - 1, a.rows).astype(np.int32))
    clat, crel, _, _ = oracle.complete_sample(n, wl["seed"], wl["lat_max"], wl["self_max"],
                                              wl["loss_max"], srcs, 1)
    ok, worst = True, 0.0
    for i, s in enumerate(srcs):
        r = [q for q, (b, e) in enumerate(shards) if b <= s < e][0]
        b = shards[r][0]
        glat = bufs[r][2][s - b, :n].cpu().numpy().view(np.uint32).astype(np.uint64) * \
            np.uint64(1_000_000)
        grel = bufs[r][3][s - b, :n].cpu().numpy()
        off = np.arange(n) != s
        ok &= bool(np.array_equal(glat[off], clat[i][off]))
        worst = max(worst, float((np.abs(grel - crel[i]) / np.maximum(crel[i], 1e-300))[off].max()))
    print(json.dumps({"workload": a.workload, "n": n, "virtual_ranks": R,
                      "dist_enc": int(stats[0].dist_enc), "ms_per_build": round(min(times) * 1e3, 1),
                      "rows_checked": int(len(srcs)), "lat_bit_exact": ok,
                      "rel_max_rel_err": worst}), flush=True)
    for r in range(R):
        L.srt_comm_free(ctypes.c_void_p(comms[r]))
    if not ok or worst > 1e-12:
        sys.exit(1)


if __name__ == "__main__":
    main()
