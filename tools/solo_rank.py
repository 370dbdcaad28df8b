#!/usr/bin/env python3
"""One rank of the N-rank sharded dense build, alone on one GPU, without the wire (timing only).

srt_comm_init_solo gives rank r of R a communicator whose collectives return at once: the rank
runs exactly its own schedule of the sharded build -- its row block, its kept tiles, the
next-row tiles first, panel assembly + closure on the high-priority stream, the final fill and
its share of the post pass -- on an otherwise idle GPU. The rank holds only its own rows, as a
real rank does. The level build (C4's default, dist_enc 12) counts and extracts its own rows'
in-arcs and synthesises what its peers would send from them (the counts and the in-arc segments
of peer target j are those of own row row0 + j % rows, levels.hip lvl_solo_*; C4's in-arcs are
uniformly random, so each target's level and predecessor work matches a real rank's). Blocks
other ranks would send are synthetic or a small constant, so the tables are NOT correct and
nothing is checked; what it measures is one rank's compute plus its critical chain at N ranks,
i.e. the N-GPU build time minus the collectives' own cost. The N-GPU runs themselves are the
driver's.

--wire-gbps 0,50,64,100,150 adds a wire model (srt_comm_init_solo_wire): each collective holds
its stream for --wire-lat-us + the bytes this rank would receive / GB/s, so the schedule feels
where a wire of that speed would sit on its critical chain.

usage: python tools/solo_rank.py [--ranks 8] [--which 0,3,7] [--workload c4] [--wire-gbps 0,64]
"""
import argparse
import ctypes
import json
import os
import sys

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
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--which", default=None, help="comma-separated ranks (default: 0, R/2, R-1)")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--time-kernels", type=int, default=1,
                    help="1: HIP events around the update launches, as bench.py times them")
    ap.add_argument("--wire-gbps", default="0", help="comma-separated effective GB/s (0: no wire)")
    ap.add_argument("--wire-lat-us", type=float, default=10.0, help="per-collective latency")
    a = ap.parse_args()
    wl = WORKLOADS[a.workload]
    n, R = wl["n"], a.ranks
    which = sorted({0, R // 2, R - 1}) if a.which is None else [int(x) for x in a.which.split(",")]
    L = _lib.lib()
    ld = (n + 127) // 128 * 128
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    wires = [float(x) for x in a.wire_gbps.split(",")]
    for r, gbps in [(r, g) for r in which for g in wires]:
        b, e = ctypes.c_int32(), ctypes.c_int32()
        L.srt_shard_rows(ld, 128, R, r, ctypes.byref(b), ctypes.byref(e))
        b, e = b.value, e.value
        nr = e - b
        comm = ctypes.c_void_p()
        _lib.check(L.srt_comm_init_solo_wire(R, r, 0, gbps, a.wire_lat_us if gbps > 0 else 0.0,
                                             ctypes.byref(comm)), "srt_comm_init_solo_wire")
        # the rank's own rows only (a real rank's footprint)
        w = torch.empty((nr, ld), dtype=torch.int32, device="cuda")
        rr = torch.empty((nr, ld), dtype=torch.float64, device="cuda")
        _lib.check(L.srt_gen_complete_device(n, ld, b, nr, wl["seed"], wl["lat_max"],
                                             wl["self_max"], wl["loss_max"], w.data_ptr(),
                                             rr.data_ptr(), sp), "gen")
        lat = torch.empty((nr, ld), dtype=torch.int32, device="cuda")
        rel = torch.empty((nr, ld), dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        best = None
        wire0 = L.srt_comm_wire_ms(comm)
        for _ in range(a.reps):
            s = _lib.BuildStats()
            s.time_kernels = a.time_kernels
            _lib.check(L.srt_dense_build_sharded(comm, n, ld, 0, w.data_ptr(), rr.data_ptr(),
                                                 lat.data_ptr(), rel.data_ptr(), sp, 0,
                                                 ctypes.byref(s)), f"rank {r}")
            torch.cuda.synchronize()
            if best is None or s.ms_total < best.ms_total:
                best = s
        rounds = ld // 64
        print(json.dumps({
            "workload": a.workload, "n": n, "ranks": R, "rank": r, "rows": nr,
            "wire_gbps": gbps, "wire_lat_us": a.wire_lat_us if gbps > 0 else 0.0,
            "wire_ms_per_build": round((L.srt_comm_wire_ms(comm) - wire0) / a.reps, 2),
            "time_kernels": a.time_kernels,
            "dist_enc": int(best.dist_enc), "levels": int(best.levels),
            "ms_total": round(best.ms_total, 2),
            "ms_fw": round(best.ms_fw, 2), "ms_post": round(best.ms_post, 2),
            "us_per_round": round(best.ms_fw * 1e3 / rounds, 1),
            "update_unit_us": round(best.ms_update * 1e3 / max(best.n_update, 1), 1),
            # level build (dist_enc 12): the lvl_step launches, the predecessor pass and rel_pk
            "ms_levels": round(best.ms_update, 3), "n_levels_timed": int(best.n_update),
            "ms_pred": round(best.ms_pred, 3), "ms_rel": round(best.ms_rel, 3),
            "ms_comm": round(best.ms_comm, 3)}), flush=True)
        L.srt_comm_free(comm)
        del w, rr, lat, rel
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
