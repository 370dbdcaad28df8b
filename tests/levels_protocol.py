"""The N-rank protocol of the row-sharded Dial level build (shadow_amd/csrc/levels.hip,
srt_levels_build), restated in numpy over torch.distributed (gloo) -- test infrastructure.

Each rank does what srt_levels_build does with its row shard and logs every collective as the C
library's collective log does (srt_comm_log_read: (op, a, b) -- 1 broadcast (bytes, root),
2 all-reduce (count, op_min), 3 all-gather (bytes per rank, 0), 5/6 group begin/end):

  1. count pass over its rows; one sum all-reduce of the exchange: the weight histogram in 20-bit
     limbs + the allocation-failure count, every rank's arcs per weight <= 8, every rank's
     distinct reliabilities of its arcs of weight <= 8 (the union table, from the exchange);
  2. its level budget (forced: the whole 254-level budget, or this rank's lcap); one min
     all-reduce of (budget, allocations, wire allocated);
  3. (4 below) every target's counts of the weights <= lx (one all-gather of u16 blocks);
  5. the first extraction (w <= lx = min(lmax, 8)), streamed when the union fits the table: per
     weight w one all-gather of every rank's arcs of weight w, one u32 each (source | table
     index), each rank's block padded to the largest -- sent one weight ahead of the levels but
     never past the current batch; else extract() below;
  6. per batch (levels 1-5, then 6, 7, 8 one at a time, then 8 at a time): the vote (sum
     all-reduce of 4 int32: not-done, settled-pair limbs);
     all ranks done -> the levels stand; after the batch ending at lx < lmax, extract(lmax): the
     all-gather (when lw <= 31 and the arcs came out of the stash), then one broadcast group of
     every rank's segment as the arcs' 4-B words and either u16 table indices or the f64s.

The distances, canonical predecessors (largest weight, then smallest tail) and path-order
reliabilities of the rank's rows are computed too, so the caller can check them against the
oracle. tests/golden/levels_protocol.json holds the sequences for the cases below
(tests/golden/make_levels_protocol.py); tests/test_dist_gloo.py re-derives them over gloo and
tests/test_gpu_protocol.py compares every virtual rank's log of the C build with them.
"""
import os

import numpy as np
import torch
import torch.distributed as dist

from shadow_amd import graphs

ALIGN, LVL_STRIDE, LVL_WMAX, RT_CAP, STASH_W, STASH_SEG, BATCH, B1 = 128, 256, 254, 2048, 32, 512, 8, 5
X_LIMBS, X_CNT = 2 * 256 + 2, 2 * 8  # levels.hip LVL_X_LIMBS, LVL_X_CNT
INF = 0x7FFFFFFF
BCAST, ALLREDUCE, ALLGATHER, GBEGIN, GEND = 1, 2, 3, 5, 6

# name -> (graph, R, per-rank level caps (SRT_FORM lcap_r<rank>), expected outcome)
CASES = {
    # the budget is capped on ranks 1.. (12 levels): first-batch extraction only (C4's shape)
    "complete300_r2": (("complete", 300, 5, 4), 2, {1: 12}, "levels"),
    "complete600_r3": (("complete", 600, 5, 4), 3, {1: 12, 2: 12}, "levels"),
    # hubs on rank 0 settle at level 5, leaves at level 10: ranks finish on either side of the
    # first batch; every rank fetches the heavier arcs and runs batch 2
    "hubleaf384_r3": (("hubleaf", 384, 128, 7), 3, {}, "levels"),
    "hubleaf640_r2": (("hubleaf", 640, 256, 9), 2, {}, "levels"),
    # one rank's budget of 1 level: every rank leaves for Floyd-Warshall after the agreement
    "capfall300_r2": (("complete", 300, 5, 4), 2, {1: 1}, "fw"),
}


def case_graph(spec):
    kind = spec[0]
    if kind == "complete":
        _, n, seed, lat_max = spec
        g = graphs.complete_graph(n, seed=seed, lat_max=lat_max)
    else:
        _, n, hubs, seed = spec
        g = graphs.hub_leaf(n, hubs, seed)
    w, r = graphs.dense_of(g)
    return g, w, r


def shard(ld, R, rank):
    nb = (ld + ALIGN - 1) // ALIGN
    return nb * rank // R * ALIGN, nb * (rank + 1) // R * ALIGN


def _lvl_estimate(hist, L, ntgt, nw):
    t, below = 0.0, 0.0
    for d in range(1, L + 1):
        if d >= 2:
            below += float(hist[d - 1])
        t += (below * nw * 4.0 + ntgt * nw * 4.0 * 3.0) / 4.0e9 + 0.03
    return t


def _limbs(v, bits, k):
    v = np.asarray(v, np.uint64)
    return [((v >> np.uint64(bits * i)) & np.uint64((1 << bits) - 1)).astype(np.int64) for i in range(k)]


def rank_protocol(rank, R, g, w, r, lcaps, fw_ms=1e30):
    """One rank of srt_levels_build over an initialised gloo group. Returns (outcome, calls,
    row0, D rows or None, rel rows or None, own level D)."""
    n = g.n
    ld = (n + ALIGN - 1) // ALIGN * ALIGN
    b, e = shard(ld, R, rank)
    max_rows = max(shard(ld, R, q)[1] - shard(ld, R, q)[0] for q in range(R))
    calls = []

    def allreduce(vec, op_min=0):
        t = torch.from_numpy(np.ascontiguousarray(vec, np.int32).copy())
        dist.all_reduce(t, op=dist.ReduceOp.MIN if op_min else dist.ReduceOp.SUM)
        calls.append((ALLREDUCE, int(t.numel()), op_min))
        return t.numpy().astype(np.int64)

    off_diag = ~np.eye(n, dtype=bool)
    arcw = np.where(off_diag & (w >= 1) & (w <= LVL_WMAX), w, 0).astype(np.int64)  # row j: j's in-arcs
    rows = np.arange(b, min(e, n))
    # 1. counts of this rank's rows, the stash overflow (a quarter-row segment past 512 light arcs)
    hist = np.zeros(LVL_STRIDE, np.int64)
    if rows.size:
        hist += np.bincount(arcw[rows].ravel(), minlength=LVL_STRIDE)[:LVL_STRIDE]
        hist[0] = 0
        Q = ((n + 1023) >> 10) << 8
        light = (arcw[rows] >= 1) & (arcw[rows] <= STASH_W)
        for wv in range(4):
            lo, hi = wv * Q, min(n, wv * Q + Q)
            if lo < hi:
                hist[0] += int((light[:, lo:hi].sum(axis=1) > STASH_SEG).sum())
    # the one sum exchange: limbs + failure count (+ pad), each rank's arcs per weight <= 8 (its
    # own slot, 16-bit halves), each rank's distinct light reliabilities (w <= 8) as int32 pairs
    xcnt = np.zeros((R, X_CNT), np.int64)
    for x in range(1, BATCH + 1):
        c = int((arcw[rows] == x).sum()) if rows.size else 0
        xcnt[rank, 2 * (x - 1)], xcnt[rank, 2 * (x - 1) + 1] = c & 0xFFFF, c >> 16
    xblk = np.zeros((R, (RT_CAP + 1) * 2), np.int64)
    if rows.size:
        vals = np.unique(r[rows][(arcw[rows] >= 1) & (arcw[rows] <= BATCH)].view(np.uint64))
        k = min(vals.size, RT_CAP)
        xblk[rank, 1] = vals.size
        xblk[rank, 2:2 + 2 * k] = vals[:k].view(np.int32).astype(np.int64)
    lo20, hi20 = _limbs(hist, 20, 2)
    red = allreduce(np.concatenate([lo20, hi20, [0, 0], xcnt.ravel(), xblk.ravel()]))
    hist = red[:LVL_STRIDE] + (red[LVL_STRIDE:2 * LVL_STRIDE] << 20)
    assert red[2 * LVL_STRIDE] == 0
    xc = red[X_LIMBS:X_LIMBS + R * X_CNT].reshape(R, X_CNT)
    pcnt = xc[:, 0::2] | (xc[:, 1::2] << 16)  # [rank][weight - 1]
    xb = red[X_LIMBS + R * X_CNT:].reshape(R, (RT_CAP + 1) * 2)
    union, fit = [], True
    for q in range(R):
        if xb[q, 0] or xb[q, 1] > RT_CAP:
            fit = False
        else:
            union.append(xb[q, 2:2 + 2 * xb[q, 1]].astype(np.int32).view(np.uint64))
    if fit:
        u = np.unique(np.concatenate(union))
        fit = 0 < u.size <= RT_CAP
    # 2. the budget (this rank's), then one min agreement of (budget, allocations, wire)
    lmax = 0
    for x in range(1, LVL_WMAX + 1):
        if _lvl_estimate(hist, x, n, max_rows / 32.0) > 0.5 * fw_ms:
            break
        lmax = x
    if rank in lcaps:
        lmax = min(lmax, lcaps[rank])
    lx_own = min(lmax, BATCH)
    wire_words = sum(R * int(pcnt[:, x - 1].max()) for x in range(1, lx_own + 1))
    stream_ok = int(R > 1 and hist[0] == 0 and fit and n <= 32768 and lx_own >= 1
                    and wire_words * 4.0 < 2e9)
    ag = allreduce([lmax, 1, stream_ok], 1)
    lmax, stream_ok = int(ag[0]), int(ag[2])
    nz = np.nonzero(hist[1:])[0]
    wmin = int(nz[0]) + 1 if nz.size else 0
    if lmax < 2 or not wmin or wmin > lmax:
        return "fw", calls, b, None, None, 0
    # 3. every target's counts of the first extraction's weights from its owner: one all-gather
    # of u16 blocks ([weight][row], padded to the largest shard); the heavier weights' counts
    # travel the same way before extract(lmax)
    cnt = np.zeros((ld, lmax + 2), np.int64)
    lx = min(lmax, BATCH)

    def share_counts(w0, w1):
        if w1 < w0:
            return
        blk = np.zeros((w1 - w0 + 1, max_rows), np.int32)  # (u16 on the C wire; gloo has no int16)
        for x in range(w0, w1 + 1):
            blk[x - w0, :rows.size] = (arcw[rows] == x).sum(axis=1) if rows.size else 0
        parts = [torch.zeros(blk.size, dtype=torch.int32) for _ in range(R)]
        dist.all_gather(parts, torch.from_numpy(blk.ravel()))
        calls.append((ALLGATHER, blk.size * 2, 0))
        for q in range(R):
            qb, qe = shard(ld, R, q)
            pb = parts[q].numpy().reshape(w1 - w0 + 1, max_rows)
            cnt[qb:qe, w0:w1 + 1] = pb[:, :qe - qb].T

    share_counts(1, lx)

    def extract(lw):
        sorted_w = lw <= STASH_W and hist[0] == 0
        numbered = False
        if sorted_w and lw <= 31:  # numbered segments (the reliability blocks)
            vals = r[rows][(arcw[rows] >= 1) & (arcw[rows] <= lw)] if rows.size else np.zeros(0)
            mine = np.unique(vals.view(np.uint64))
            blk = np.zeros(RT_CAP + 1, np.uint64)
            head = np.zeros(2, np.int32)
            head[1] = min(mine.size, 0x7FFFFFFF)
            blk[0] = head.view(np.uint64)[0]
            k = min(mine.size, RT_CAP)
            blk[1:1 + k] = mine[:k]
            parts = [torch.zeros(RT_CAP + 1, dtype=torch.int64) for _ in range(R)]
            dist.all_gather(parts, torch.from_numpy(blk.view(np.int64)))
            calls.append((ALLGATHER, (RT_CAP + 1) * 8, 0))
            union, fit = [], True
            for t_ in parts:
                v = t_.numpy().view(np.uint64)
                hd = v[:1].view(np.int32)
                if hd[0] or hd[1] > RT_CAP:
                    fit = False
                else:
                    union.append(v[1:1 + hd[1]])
            if fit:
                u = np.unique(np.concatenate(union)) if union else np.zeros(0, np.uint64)
                numbered = 0 < u.size <= RT_CAP
        calls.append((GBEGIN, 0, 0))
        for q in range(R):
            qb, qe = shard(ld, R, q)
            c = int(cnt[qb:min(qe, n), 1:lw + 1].sum())
            if c:
                calls.append((BCAST, c * 4, q))
                calls.append((BCAST, c * (2 if numbered else 8), q))
        calls.append((GEND, 0, 0))

    # 4. the first extraction: streamed (per weight, every rank's block padded to the largest:
    # one all-gather of one u32 per arc, all of them sent before the first vote), or extract()
    if not stream_ok:
        extract(lx)
    lw = lx
    wq = 0  # streamed weights sent: one ahead of the levels, never past the current batch
    # the levels of the local sources (bit-parallel Dial levels restated as boolean matmuls)
    src = np.arange(b, min(e, n))
    ns = src.size
    D = np.full((ns, n), INF, np.int64)
    D[np.arange(ns), src] = 0
    M = {x: (arcw.T == x).astype(np.float32) for x in range(1, lmax + 1) if hist[x]}  # M[k, j]
    Dl, all_done, settled = 0, False, 0
    d0 = 1
    while d0 <= lmax:  # batches: levels 1-5, then 6, 7, 8 one at a time, then 8 at a time
        d1 = min(lmax, B1) if d0 == 1 else d0 if d0 <= BATCH else min(lmax, d0 + BATCH - 1)
        for d in range(d0, d1 + 1):
            while stream_ok and wq < min(lx, d + 1, d1):
                wq += 1
                calls.append((ALLGATHER, int(pcnt[:, wq - 1].max()) * 4, 0))
            hit = np.zeros((ns, n), bool)
            for x, Mx in M.items():
                if x <= min(d, lw):
                    hit |= ((D == d - x).astype(np.float32) @ Mx) > 0
            new = hit & (D == INF)
            D[new] = d
            if d >= 2:
                settled += int(new.sum())
            if not Dl and d >= 2 and (D < INF).all():
                Dl = d
        vote = allreduce([0 if Dl else 1] + [int(x) for x in _limbs(settled, 21, 3)])
        all_done = vote[0] == 0
        if all_done:
            break
        sg = int(vote[1]) + (int(vote[2]) << 21) + (int(vote[3]) << 42)
        frac = (sg + n + int(hist[1])) / float(n * n)
        if d1 == lx and d1 < lmax and frac < 0.25 and fw_ms < 1e29:
            break
        if d1 == lx and lx < lmax:
            share_counts(lx + 1, lmax)
            extract(lmax)
            lw = lmax
        d0 = d1 + 1
    if not all_done:
        return "fw", calls, b, None, None, Dl
    # canonical predecessors and path-order reliabilities, level by level
    rel = np.zeros((ns, n))
    Wl = np.where(arcw.T <= lmax, arcw.T, 0)  # Wl[k, j]
    for i, s in enumerate(src):
        Ds = D[i]
        tight = (Wl > 0) & (Ds[:, None] + Wl == Ds[None, :])
        score = np.where(tight, Wl * (n + 1) + (n - np.arange(n))[:, None], -1)
        pred = score.argmax(axis=0)
        rel[i, s] = 1.0
        for d in np.unique(Ds[Ds > 0]):
            js = np.nonzero(Ds == d)[0]
            u = pred[js]
            rel[i, js] = np.where(u == s, 1.0, rel[i, u]) * r[u, js]
    return "levels", calls, b, D, rel, Dl


def gloo_worker(rank, R, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=R)
    spec, _, lcaps, _ = CASES[name]
    g, w, r = case_graph(spec)
    out = rank_protocol(rank, R, g, w, r, lcaps)
    q.put((rank,) + out)
    dist.barrier()
    dist.destroy_process_group()
