"""The C library's N-rank protocol of the row-sharded level build against its gloo rehearsal
(ADVICE r05 high).

srt_dense_build_sharded runs on R virtual ranks of device 0 (one host thread each; the virtual
communicator's collectives are device copies lined up by host barriers, so a rank that called a
different collective than its peers would pair with the wrong one). Every rank's collective log
(srt_comm_log_*: op, size, root / reduction) must be identical, and equal to the sequence the
numpy + gloo restatement of srt_levels_build makes for the same graph, shards and level caps
(tests/levels_protocol.py; the committed fixture tests/golden/levels_protocol.json, which
tests/test_dist_gloo.py re-derives over gloo). The cases cover the first-batch build, capped
budgets on some ranks, ranks whose own sources settle on either side of the first batch of levels
(the batch decision from the summed vote, the heavier arcs fetched by every rank), and a budget
divergence that sends every rank to Floyd-Warshall together. The tables are checked against the
oracle."""
import ctypes
import json
import os
import sys
import threading

import numpy as np
import pytest
from conftest import set_form

import oracle
from shadow_amd import _lib

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import levels_protocol as lp  # noqa: E402

pytestmark = pytest.mark.gpu
LEVELS = 12
MS = 1_000_000
_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "levels_protocol.json")


def _sharded_logged(L, w, r, n, R):
    """srt_dense_build_sharded on R virtual ranks with the collective log on; returns the tables
    (n x n), each rank's log and stats."""
    import torch
    ld = (n + lp.ALIGN - 1) // lp.ALIGN * lp.ALIGN
    W = np.full((ld, ld), lp.INF, np.uint32)
    Rr = np.zeros((ld, ld))
    W[:n, :n] = w
    Rr[:n, :n] = r
    comms = (ctypes.c_void_p * R)()
    _lib.check(L.srt_comm_init_virtual(R, 0, comms), "srt_comm_init_virtual")
    try:
        bufs, streams = [], []
        for q in range(R):
            b, e = lp.shard(ld, R, q)
            wt = torch.from_numpy(np.ascontiguousarray(W[b:e]).view(np.int32)).cuda()
            rt = torch.from_numpy(np.ascontiguousarray(Rr[b:e])).cuda()
            bufs.append((wt, rt, torch.empty_like(wt), torch.empty_like(rt)))
            streams.append(torch.cuda.Stream())
            _lib.check(L.srt_comm_log_enable(ctypes.c_void_p(comms[q]), 1), "srt_comm_log_enable")
        torch.cuda.synchronize()
        rcs = [None] * R
        stats = [_lib.BuildStats() for _ in range(R)]

        def work(q):
            L.srt_virtual_rank_bind(q, 0)
            wt, rt, lat, rel = bufs[q]
            rcs[q] = L.srt_dense_build_sharded(ctypes.c_void_p(comms[q]), n, ld, 0, wt.data_ptr(),
                                               rt.data_ptr(), lat.data_ptr(), rel.data_ptr(),
                                               ctypes.c_void_p(streams[q].cuda_stream), 0,
                                               ctypes.byref(stats[q]))
            L.srt_virtual_rank_bind(-1, 0)

        th = [threading.Thread(target=work, args=(q,)) for q in range(R)]
        for t in th:
            t.start()
        for t in th:
            t.join(300)
            assert not t.is_alive(), "a virtual rank did not return (collectives paired wrongly?)"
        torch.cuda.synchronize()
        for q in range(R):
            _lib.check(rcs[q], f"rank {q}")
        logs = []
        for q in range(R):
            k = L.srt_comm_log_read(ctypes.c_void_p(comms[q]), None, 0)
            buf = np.zeros(3 * max(k, 1), np.int64)
            L.srt_comm_log_read(ctypes.c_void_p(comms[q]), buf.ctypes.data, k)
            logs.append(buf[:3 * k].reshape(k, 3).tolist())
        lat = np.concatenate([bufs[q][2].cpu().numpy() for q in range(R)])
        rel = np.concatenate([bufs[q][3].cpu().numpy() for q in range(R)])
    finally:
        for q in range(R):
            L.srt_comm_free(ctypes.c_void_p(comms[q]))
    return lat, rel, logs, stats


@pytest.mark.parametrize("name", list(lp.CASES))
def test_level_protocol_logs_match_rehearsal(gpu, monkeypatch, name):
    spec, R, lcaps, outcome = lp.CASES[name]
    with open(_GOLDEN) as f:
        gold = json.load(f)[name]
    form = {"levels": "1"}
    form.update({f"lcap_r{q}": str(c) for q, c in lcaps.items()})
    set_form(monkeypatch, **form)
    g, w, r = lp.case_graph(spec)
    n = g.n
    lat, rel, logs, stats = _sharded_logged(gpu, w, r, n, R)
    assert all(lg == logs[0] for lg in logs), logs  # SPMD: one sequence on every rank
    if outcome == "levels":
        assert logs[0] == gold["calls"], (logs[0], gold["calls"])
        assert {int(s.dist_enc) for s in stats} == {LEVELS}
        assert [int(s.levels) for s in stats] == gold["own_levels"]
    else:  # the level build's part of the log, then the FW's collectives
        assert logs[0][:len(gold["calls"])] == gold["calls"], (logs[0], gold["calls"])
        assert LEVELS not in {int(s.dist_enc) for s in stats}
    exp = oracle.table(oracle.EdgeList(g.n, g.directed, g.src, g.dst, g.lat_ns, g.loss), raw=True)
    glat = lat[:n, :n].view(np.uint32).astype(np.uint64) * np.uint64(MS)
    assert np.array_equal(glat, exp["lat_int"]), np.argwhere(glat != exp["lat_int"])[:5]
    err = np.abs(rel[:n, :n] - exp["rel"]) / np.maximum(np.abs(exp["rel"]), 1e-300)
    assert float(err.max()) <= 1e-12
    if n < lat.shape[0]:  # the padding rows of the last shard: no path
        assert np.all(lat[n:, :n].view(np.uint32) == lp.INF)
