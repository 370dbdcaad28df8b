/*
 * levels.hip -- exact all-pairs shortest distances on dense graphs by bit-parallel Dial levels.
 *
 * Replaces, when it is cheaper, the blocked Floyd-Warshall of fw16.hip for the distance phase of
 * _topology_computeSourcePaths (/root/reference/src/main/routing/topology.c:1578-1814, the igraph
 * Dijkstra of :1679-1701) on complete / dense graphs. Edge weights are integer quanta >= 1, so
 * Dijkstra's settle order is Dial's bucket order, and one bucket (distance level d) of EVERY source
 * can be settled at once with bit operations:
 *
 *   Delta_d[j] = ( OR over in-arcs (k -> j, w <= d) of Delta_{d-w}[k] )  AND NOT  R_{d-1}[j]
 *   R_d[j]     = R_{d-1}[j] OR Delta_d[j]
 *
 * where Delta_d[j] is the bit set of sources s with D[s][j] == d, R_d[j] those with D[s][j] <= d,
 * and Delta_0[k] = R_0[k] = {k}. This is the last-hop decomposition D[s][j] = min_k D[s][k] +
 * w(k, j) (every weight >= 1, so Delta_{d-w} is final when level d is formed), i.e. the same
 * distances Dijkstra settles; the canonical predecessors and path-order reliabilities are formed
 * afterwards from the distances by the dense post pass exactly as after Floyd-Warshall.
 *
 * Only arcs with w <= lmax take part. If every pair is settled by level D <= lmax, every arc with
 * w > lmax >= D is longer than the distance it joins, so it lies on no shortest path and the
 * result is exact. Otherwise the build falls back to Floyd-Warshall (the caller's).
 *
 * Layout (HBM). Bit sets run over this rank's sources (nsrc, a multiple of 128): nw = nsrc / 32
 * words per vertex. lev[d - 1][j][word] for d = 1..lmax, R[j][word]; one wave owns a (target j,
 * 64-word source chunk) unit, so every arc costs one coalesced 256-B gather of Delta_{d-w}[k].
 * In-arcs come from the rows of w (undirected: row j holds j's in-arcs, and a row-sharded rank has
 * them for its rows) or its columns (directed, one GPU), grouped by (target, weight).
 */
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cstring>
#include <vector>

#include "srt_device.h"

#define LVL_STRIDE 256 /* per-target offsets: weight 0..255 */
/* levels enqueued per host round trip: a batch's levels past the one that settles every pair
 * return at once (lvl_step_kernel's prev test); the first batch is LVL_B1 levels (C4's distances
 * end at 4-5: one vote), then one level per batch up to LVL_BATCH, then LVL_BATCH per batch */
#define LVL_BATCH 8
#define LVL_B1 5
#define LVL_WMAX 254   /* largest level budget (distances stay u8: the post pass's small path) */
#define LVL_PB 12 /* lvl_pred_kernel: gathers per pipelined batch */
#define LVL_NEAR_NW 2048 /* lvl_near_kernel: a target's plane row in LDS, four per workgroup */
#define LVL_NEAR_MIN_NW 512 /* ... and only for shares of at least 16,384 sources */

/* ---- in-arc extraction ------------------------------------------------------------------- */
/* COUNT: per (target, weight) histogram of arcs with 1 <= w <= LVL_WMAX; FILL: the arcs (k | w << 16)
 * at cursor positions from off (weights above lmax were masked out of off). Rows form: local row
 * jj of w is target row0 + jj's in-arc row (undirected). */
/* The count pass also keeps each row's light arcs (w <= LVL_STASH_W; C4: ~1,050 per row) in a
 * stash, so the fill reads them instead of the whole w row again (when lmax <= LVL_STASH_W and
 * the row's arcs fit). Wave q of the row's workgroup scans the row's q-th quarter and appends
 * its light arcs in vertex order (a ballot prefix per step) to its own LVL_STASH_SEG-entry
 * segment, so the stash holds the row's light arcs in vertex order. The fill then places them by
 * weight in that order (per-wave counts, then a ballot rank per weight): every target's in-arcs
 * come out sorted by (weight, source) with no sort pass. A segment that overflows marks the
 * row (-1) and counts in *sovf: that build takes the full-row fill and the segmented sort. */
#define LVL_STASH_W 32
#define LVL_STASH_SEG 512
#define LVL_STASH_CAP (4 * LVL_STASH_SEG)
template <bool FILL>
__global__ __launch_bounds__(256) void lvl_arcs_rows_kernel(int n, int ld, int row0,
                                                            const uint32_t* __restrict__ w,
                                                            int32_t* __restrict__ cnt, int lmax,
                                                            const int32_t* __restrict__ off,
                                                            uint32_t* __restrict__ arcs,
                                                            const double* __restrict__ r = nullptr,
                                                            double* __restrict__ ar = nullptr,
                                                            unsigned long long* __restrict__ dkey = nullptr,
                                                            uint32_t* __restrict__ stash = nullptr,
                                                            int32_t* __restrict__ scnt = nullptr,
                                                            unsigned long long* __restrict__ sovf = nullptr) {
    __shared__ int h[LVL_STRIDE];
    __shared__ unsigned long long s_key[4];
    __shared__ int wc[4][LVL_STASH_W + 1];
    const int jj = blockIdx.x, j = row0 + jj;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (FILL && stash && j < n && lmax <= LVL_STASH_W &&
        min(min(scnt[(size_t)jj * 4], scnt[(size_t)jj * 4 + 1]),
            min(scnt[(size_t)jj * 4 + 2], scnt[(size_t)jj * 4 + 3])) >= 0) {
        for (int i = tid; i <= lmax; i += 256) h[i] = off[(size_t)j * LVL_STRIDE + i];
        for (int i = tid; i < 4 * (LVL_STASH_W + 1); i += 256) wc[i / (LVL_STASH_W + 1)][i % (LVL_STASH_W + 1)] = 0;
        __syncthreads();
        const uint32_t* sr = stash + (size_t)jj * LVL_STASH_CAP + wv * LVL_STASH_SEG;
        const int m = scnt[(size_t)jj * 4 + wv];
        for (int q = lane; q < m; q += 64) {
            const uint32_t x = sr[q] >> 16;
            if (x <= (uint32_t)lmax) atomicAdd(&wc[wv][x], 1);
        }
        __syncthreads();
        /* lane x (x <= lmax <= 32) keeps this wave's next position for weight x: the weight's
         * start plus the earlier waves' arcs of that weight */
        int run = 0;
        if (lane <= lmax) {
            run = h[lane];
            for (int v = 0; v < wv; ++v) run += wc[v][lane];
        }
        for (int q0 = 0; q0 < m; q0 += 64) {
            const int q = q0 + lane;
            const uint32_t e = q < m ? sr[q] : 0u, x = e >> 16;
            const bool valid = q < m && x >= 1u && x <= (uint32_t)lmax;
            unsigned long long pend = __ballot(valid);
            int pos = 0;
            while (pend) {
                const int x0 = __builtin_amdgcn_readlane((int)x, __builtin_ctzll(pend));
                const unsigned long long mm = __ballot(valid && (int)x == x0);
                const int base = __builtin_amdgcn_readlane(run, x0);
                if (valid && (int)x == x0) pos = base + __popcll(mm & lt);
                if (lane == x0) run += __popcll(mm);
                pend &= ~mm;
            }
            if (valid) {
                arcs[pos] = e;
                ar[pos] = r[(size_t)jj * ld + (e & 0xFFFFu)]; /* undirected: r(k -> j) = r(j -> k) */
            }
        }
        return;
    }
    /* COUNT also takes the diagonal rule's key from the same row reads (topology.c:1431-1576, as
     * dense_diag_kernel): min over the row's out-edges of (self-loop L, other 2L) << 32 | u */
    unsigned long long best = ~0ull;
    for (int i = tid; i < LVL_STRIDE; i += 256)
        h[i] = FILL ? (j < n ? off[(size_t)j * LVL_STRIDE + i] : 0) : 0;
    __syncthreads();
    const int wmax = FILL ? lmax : LVL_WMAX;
    if (FILL) {
        if (j < n) {
            const uint32_t* row = w + (size_t)jj * ld;
            for (int k4 = tid * 4; k4 < n; k4 += 1024) {
                const uint4 v = *reinterpret_cast<const uint4*>(row + k4);
                const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int k = k4 + q;
                    if (k < n && k != j && x[q] >= 1u && x[q] <= (uint32_t)wmax) {
                        const int p = atomicAdd(&h[x[q]], 1);
                        arcs[p] = (uint32_t)k | (x[q] << 16);
                        ar[p] = r[(size_t)jj * ld + k]; /* undirected: r(k -> j) = r(j -> k) */
                    }
                }
            }
        }
        return;
    }
    int run = 0;
    if (j < n) {
        const uint32_t* row = w + (size_t)jj * ld;
        const int Q = ((n + 1023) >> 10) << 8; /* a wave's quarter of the row, 256-aligned */
        const int lo = wv * Q, hi = min(n, lo + Q);
        uint32_t* seg = stash ? stash + (size_t)jj * LVL_STASH_CAP + wv * LVL_STASH_SEG : nullptr;
        for (int b0 = lo; b0 < hi; b0 += 256) {
            const int k4 = b0 + lane * 4;
            uint4 v = make_uint4(SRT_INF, SRT_INF, SRT_INF, SRT_INF);
            if (k4 < hi) v = *reinterpret_cast<const uint4*>(row + k4);
            const uint32_t x[4] = {v.x, v.y, v.z, v.w};
            int c = 0;
            bool cand[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = k4 + q;
                if (k < n && x[q] < SRT_INF) {
                    const unsigned long long lat = k == j ? x[q] : 2ull * x[q];
                    best = min(best, (lat << 32) | (uint32_t)k);
                }
                const bool arc = k < n && k != j && x[q] >= 1u && x[q] <= (uint32_t)wmax;
                if (arc) atomicAdd(&h[x[q]], 1);
                cand[q] = arc && x[q] <= LVL_STASH_W;
                c += cand[q];
            }
            if (seg) { /* vertex order: the lane's exclusive prefix of the counts (0..4) */
                const unsigned long long b1 = __ballot(c & 1), b2 = __ballot(c & 2), b4 = __ballot(c & 4);
                int p = run + __popcll(b1 & lt) + 2 * __popcll(b2 & lt) + 4 * __popcll(b4 & lt);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (cand[q]) {
                        if (p < LVL_STASH_SEG) seg[p] = (uint32_t)(k4 + q) | (x[q] << 16);
                        ++p;
                    }
                run += __popcll(b1) + 2 * __popcll(b2) + 4 * __popcll(b4);
            }
        }
    }
    if (stash && lane == 0) {
        const bool over = run > LVL_STASH_SEG;
        scnt[(size_t)jj * 4 + wv] = over ? -1 : run;
        if (over) atomicAdd(sovf, 1ull);
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(best, o);
        best = y < best ? y : best;
    }
    if (lane == 0) s_key[wv] = best;
    __syncthreads();
    for (int i = tid; i < LVL_STRIDE; i += 256) cnt[(size_t)j * LVL_STRIDE + i] = h[i];
    if (tid == 0 && dkey)
        dkey[jj] = min(min(s_key[0], s_key[1]), min(s_key[2], s_key[3]));
}

/* The diagonal rule of the held rows from the keys the count pass took: D[s][s] = the key's
 * latency (0 with no out-edge), rel = r or r^2 (0.0), as dense_diag_kernel */
__global__ void lvl_diag_kernel(int n, int ld, int row0, int lrows,
                                const unsigned long long* __restrict__ dkey,
                                const double* __restrict__ r, uint32_t* __restrict__ d,
                                double* __restrict__ rel) {
    const int jj = blockIdx.x * blockDim.x + threadIdx.x;
    if (jj >= lrows) return;
    const int v = row0 + jj;
    const unsigned long long best = dkey[jj];
    const size_t ix = (size_t)jj * ld + v;
    if (best == ~0ull) {
        d[ix] = 0;
        rel[ix] = 0.0;
    } else {
        const int u = (int)(best & 0xFFFFFFFFu);
        const double x = r[(size_t)jj * ld + u];
        d[ix] = (uint32_t)(best >> 32);
        rel[ix] = u == v ? x : x * x;
    }
}

/* Columns form (directed graph on one GPU): workgroup of 64 target columns j0.., lane = column,
 * the four waves sweep the rows k (one coalesced 256-B segment of a row per wave and step). */
template <bool FILL>
__global__ __launch_bounds__(256) void lvl_arcs_cols_kernel(int n, int ld,
                                                            const uint32_t* __restrict__ w,
                                                            int32_t* __restrict__ cnt, int lmax,
                                                            const int32_t* __restrict__ off,
                                                            uint32_t* __restrict__ arcs,
                                                            const double* __restrict__ r = nullptr,
                                                            double* __restrict__ ar = nullptr) {
    __shared__ int h[64 * LVL_STRIDE];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int j0 = blockIdx.x * 64, j = j0 + lane;
    for (int i = threadIdx.x; i < 64 * LVL_STRIDE; i += 256) {
        const int c = i / LVL_STRIDE, ww = i % LVL_STRIDE;
        h[i] = FILL ? (j0 + c < n ? off[(size_t)(j0 + c) * LVL_STRIDE + ww] : 0) : 0;
    }
    __syncthreads();
    const int wmax = FILL ? lmax : LVL_WMAX;
    if (j < n) {
        for (int k = wv; k < n; k += 4) {
            const uint32_t x = w[(size_t)k * ld + j];
            if (k != j && x >= 1u && x <= (uint32_t)wmax) {
                if (FILL) {
                    const int p = atomicAdd(&h[lane * LVL_STRIDE + x], 1);
                    arcs[p] = (uint32_t)k | (x << 16);
                    ar[p] = r[(size_t)k * ld + j];
                } else
                    atomicAdd(&h[lane * LVL_STRIDE + x], 1);
            }
        }
    }
    if (FILL) return;
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * LVL_STRIDE; i += 256) {
        const int c = i / LVL_STRIDE, ww = i % LVL_STRIDE;
        if (j0 + c < ld) cnt[(size_t)(j0 + c) * LVL_STRIDE + ww] = h[i];
    }
}

/* weight histogram over the count rows (for the level budget) */
__global__ void lvl_hist_kernel(size_t count, const int32_t* __restrict__ cnt,
                                unsigned long long* __restrict__ hist, unsigned mult = 1) {
    __shared__ unsigned long long s[LVL_STRIDE];
    for (int i = threadIdx.x; i < LVL_STRIDE; i += blockDim.x) s[i] = 0;
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
         i += (size_t)gridDim.x * blockDim.x)
        if (cnt[i]) atomicAdd(&s[i % LVL_STRIDE], (unsigned long long)cnt[i]);
    __syncthreads();
    for (int i = threadIdx.x; i < LVL_STRIDE; i += blockDim.x)
        if (s[i]) atomicAdd(&hist[i], s[i] * mult);
}

/* N > 1: the histogram all-reduced in 20-bit limbs (int32 sums of R ranks cannot overflow), then
 * only the (target, weight <= lmax) counts -- the in-arc offsets need no heavier weight: 2.9 MB
 * on C4 instead of the 33.5-MB (target x 256 weights) block */
__global__ void lvl_hist_limbs_kernel(int to, unsigned long long* __restrict__ hist,
                                      int32_t* __restrict__ limbs) {
    const int i = threadIdx.x;
    if (i >= LVL_STRIDE) return;
    if (to) {
        limbs[i] = (int32_t)(hist[i] & 0xFFFFFull);
        limbs[LVL_STRIDE + i] = (int32_t)(hist[i] >> 20);
    } else {
        hist[i] = (unsigned long long)(uint32_t)limbs[i] +
                  ((unsigned long long)(uint32_t)limbs[LVL_STRIDE + i] << 20);
    }
}
/* N > 1: every target's counts of weights w0..w1 from its owner: each rank's block holds its own
 * targets' counts as u16 ([weight][row], padded to the largest shard), all-gathered (2 B per
 * (target, weight) instead of the int32 sum all-reduce of every column up to lmax + 1) */
__global__ void lvl_cnt_gpack_kernel(int row0, int nrows, int max_rows, int w0, int w1, int me,
                                     const int32_t* __restrict__ cnt, uint16_t* __restrict__ cg) {
    const int jj = blockIdx.x * blockDim.x + threadIdx.x;
    if (jj >= nrows) return;
    uint16_t* blk = cg + (size_t)me * max_rows * (w1 - w0 + 1);
    for (int w = w0; w <= w1; ++w)
        blk[(size_t)(w - w0) * max_rows + jj] = (uint16_t)cnt[(size_t)(row0 + jj) * LVL_STRIDE + w];
}
__global__ void lvl_cnt_gunpack_kernel(int ld, int R, int max_rows, int w0, int w1,
                                       const uint16_t* __restrict__ cg, int32_t* __restrict__ cnt) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ld) return;
    const long long nb = ld / SRT_SHARD_ALIGN; /* the owner of row j (srt_shard_rows) */
    int q = 0;
    while (q + 1 < R && (int)(nb * (q + 1) / R) * SRT_SHARD_ALIGN <= j) ++q;
    const int jj = j - (int)(nb * q / R) * SRT_SHARD_ALIGN;
    const uint16_t* blk = cg + (size_t)q * max_rows * (w1 - w0 + 1);
    for (int w = w0; w <= w1; ++w) cnt[(size_t)j * LVL_STRIDE + w] = blk[(size_t)(w - w0) * max_rows + jj];
}

/* ---- the arcs' distinct reliabilities (packed post pass) ------------------------------------ *
 * The post pass carries r(pred, t) per pair as a 16-bit index into a table of the distinct arc
 * reliabilities instead of the f64 itself (C4: 501 values): the predecessor and the index share one
 * 4-B word (10 B per pair before, plus their two transposes). The table is exact -- each entry is
 * an arc's double, bit for bit. An open-addressing hash over the value bits (LVL_RT_SLOTS slots,
 * linear probing) gives each arc a slot, one workgroup numbers the occupied slots in slot order,
 * and the arcs' slots become dense indices. More than LVL_RT_CAP distinct values (or a probe run
 * past LVL_RT_PROBE) keeps the f64 form. */
#define LVL_RT_SLOTS 8192 /* global slots: <= 2048 values at a load of 1/4 */
#define LVL_RT_PROBE 256
#define LVL_RT_CAP 2048
#define LVL_RT_LDS 2048 /* a workgroup's private table */
static __device__ __forceinline__ unsigned lvl_rt_hash(unsigned long long b) {
    b ^= b >> 33;
    b *= 0xff51afd7ed558ccdull;
    b ^= b >> 33;
    return (unsigned)b & (LVL_RT_SLOTS - 1u);
}
static __device__ __forceinline__ int lvl_rt_global_slot(unsigned long long v, unsigned long long* H) {
    unsigned h = lvl_rt_hash(v);
    for (int p = 0; p < LVL_RT_PROBE; ++p, h = (h + 1u) & (LVL_RT_SLOTS - 1u)) {
        unsigned long long x = __hip_atomic_load(&H[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (x == ~0ull) x = atomicCAS(&H[h], ~0ull, v); /* ~0: empty (a NaN, never a reliability) */
        if (x == ~0ull || x == v) return (int)h;
    }
    return -1;
}
/* Each arc of [lo, hi) (device-held bounds when lo_p / hi_p are given) gets its value's global
 * slot. A workgroup takes a contiguous run of arcs and dedupes it in a private LDS table first, so
 * the global table sees each distinct value once per workgroup instead of once per arc: every arc
 * probing the global table hammered its ~500 hot lines (C4: 87 us for 1.07 M arcs). Values past
 * the LDS table's probe go to the global table directly (marked 0x8000 in the first pass). */
__global__ __launch_bounds__(256) void lvl_rt_hash_kernel(const int32_t* __restrict__ lo_p,
                                                          const int32_t* __restrict__ hi_p, int lo, int hi,
                                                          const double* __restrict__ ar,
                                                          unsigned long long* __restrict__ H,
                                                          uint16_t* __restrict__ rix, int* __restrict__ ovf) {
    __shared__ unsigned long long key[LVL_RT_LDS];
    __shared__ uint16_t gs[LVL_RT_LDS];
    const int a = lo_p ? *lo_p : lo, b = hi_p ? *hi_p : hi, tid = threadIdx.x;
    const int per = max(0, (b - a + (int)gridDim.x - 1) / (int)gridDim.x);
    const int c0 = a + (int)blockIdx.x * per, c1 = min(b, c0 + per);
    for (int s = tid; s < LVL_RT_LDS; s += 256) key[s] = ~0ull;
    __syncthreads();
    bool bad = false;
    for (int i = c0 + tid; i < c1; i += 256) {
        const unsigned long long v = (unsigned long long)__double_as_longlong(ar[i]);
        unsigned h = lvl_rt_hash(v) & (LVL_RT_LDS - 1u);
        int p = 0;
        for (; p < 64; ++p, h = (h + 1u) & (LVL_RT_LDS - 1u)) {
            unsigned long long x = __hip_atomic_load(&key[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (x == ~0ull) x = atomicCAS(&key[h], ~0ull, v);
            if (x == ~0ull || x == v) break;
        }
        uint16_t out = (uint16_t)h;
        if (p == 64) {
            const int g = lvl_rt_global_slot(v, H);
            bad |= g < 0;
            out = (uint16_t)(0x8000u | (unsigned)max(g, 0));
        }
        rix[i] = out;
    }
    __syncthreads();
    for (int s = tid; s < LVL_RT_LDS; s += 256) {
        const unsigned long long v = key[s];
        if (v == ~0ull) continue;
        const int g = lvl_rt_global_slot(v, H);
        bad |= g < 0;
        gs[s] = (uint16_t)max(g, 0);
    }
    if (bad) *ovf = 1;
    __syncthreads();
    for (int i = c0 + tid; i < c1; i += 256) { /* (this thread's own first-pass entries) */
        const uint16_t x = rix[i];
        rix[i] = (x & 0x8000u) ? (uint16_t)(x & 0x7FFFu) : gs[x];
    }
}
static unsigned lvl_rt_grid(int64_t count) {
    const int64_t g = (count + 4095) / 4096;
    return (unsigned)(g < 1 ? 1 : g > 512 ? 512 : g);
}
/* one workgroup: dense index of every occupied slot (slot order), the table, its size */
__global__ __launch_bounds__(1024) void lvl_rt_compact_kernel(const unsigned long long* __restrict__ H,
                                                              uint16_t* __restrict__ map,
                                                              double* __restrict__ rtab,
                                                              int* __restrict__ ntab) {
    constexpr int PER = LVL_RT_SLOTS / 1024;
    __shared__ int wsum[16];
    const int tid = threadIdx.x, lane = tid & 63;
    int c = 0;
    for (int k = 0; k < PER; ++k) c += H[tid * PER + k] != ~0ull;
    int inc = c;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[tid >> 6] = inc;
    __syncthreads();
    int base = inc - c, total = 0;
    for (int w = 0; w < 16; ++w) {
        base += w < (tid >> 6) ? wsum[w] : 0;
        total += wsum[w];
    }
    for (int k = 0; k < PER; ++k) {
        const unsigned long long v = H[tid * PER + k];
        if (v == ~0ull) continue;
        map[tid * PER + k] = (uint16_t)base;
        if (base < LVL_RT_CAP) rtab[base] = __longlong_as_double((long long)v);
        ++base;
    }
    if (tid == 0) *ntab = total;
}
__global__ void lvl_rt_remap_kernel(int total, const uint16_t* __restrict__ map,
                                    uint16_t* __restrict__ rix) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < total) rix[i] = map[rix[i]];
}

/* N > 1 (numbered segments): each arc's index into the union table, sorted by value bits, of
 * every rank's distinct reliabilities -- the same numbering on every rank */
__global__ void lvl_rt_index_kernel(int total, const double* __restrict__ ar,
                                    const unsigned long long* __restrict__ tab, int ntab,
                                    uint16_t* __restrict__ rix) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const unsigned long long b = (unsigned long long)__double_as_longlong(ar[i]);
    int lo = 0, hi = ntab - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (tab[mid] < b) lo = mid + 1;
        else hi = mid;
    }
    rix[i] = (uint16_t)lo;
}

/* ---- timing-only solo rank (srt_comm_init_solo*, tools/solo_rank.py) ------------------------ *
 * A solo rank runs exactly one real rank's work on its own rows; what a real rank would receive
 * from its peers it synthesises from its own rows instead (the collectives only charge the wire
 * model). Peer target j = js + shift (js one of the rank's own rows) takes js's counts, then js's
 * in-arc segment with every source moved by the same shift (mod n; each weight's run rotated so
 * it stays sorted by source). The graph is then a union of shifted copies of the rank's rows:
 * every vertex keeps distinct random in-neighbours, and on C4 its distances match the real
 * graph's (sampled: max 4, mean 3.292 against 3.290); plain copies (no shift) collapsed the
 * vertices onto the rank's rows and stretched the distances to 6. */
__global__ void lvl_solo_counts_kernel(int n, int row0, int nrows, int lrows, int32_t* __restrict__ cnt) {
    const int j = blockIdx.x;
    if (j >= n || (j >= row0 && j < row0 + nrows)) return;
    const int js = row0 + ((j - row0) % lrows + lrows) % lrows;
    for (int x = threadIdx.x; x < LVL_STRIDE; x += blockDim.x)
        cnt[(size_t)j * LVL_STRIDE + x] = cnt[(size_t)js * LVL_STRIDE + x];
}
__global__ void lvl_solo_arcs_kernel(int n, int row0, int nrows, int lrows, int w0, int w1, int nw,
                                     const int32_t* __restrict__ off, uint32_t* __restrict__ arcs,
                                     uint16_t* __restrict__ rix, double* __restrict__ ar,
                                     uint32_t* __restrict__ aoff) {
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (j >= n || (j >= row0 && j < row0 + nrows)) return;
    const int js = row0 + ((j - row0) % lrows + lrows) % lrows;
    const int shift = ((j - js) % n + n) % n;
    for (int x = w0; x <= w1; ++x) {
        const int g0 = off[(size_t)j * LVL_STRIDE + x], c = off[(size_t)j * LVL_STRIDE + x + 1] - g0;
        if (c <= 0) continue;
        const int s0 = off[(size_t)js * LVL_STRIDE + x];
        int nwr = 0; /* sources that wrap past n: the run's tail, which goes first */
        for (int i0 = 0; i0 < c; i0 += 64) {
            const int i = i0 + lane;
            nwr += __popcll(__ballot(i < c && (int)(arcs[s0 + i] & 0xFFFFu) + shift >= n));
        }
        for (int i = lane; i < c; i += 64) {
            const uint32_t e = arcs[s0 + i];
            int k = (int)(e & 0xFFFFu) + shift;
            const bool wr = k >= n;
            if (wr) k -= n;
            const int d = g0 + (wr ? i - (c - nwr) : nwr + i);
            arcs[d] = (uint32_t)k | (e & 0xFFFF0000u);
            if (rix) rix[d] = rix[s0 + i];
            if (ar) ar[d] = ar[s0 + i];
            if (aoff) aoff[d] = (uint32_t)k * (uint32_t)nw * 4u;
        }
    }
}

/* N > 1, streamed: the arcs of weight d from this rank's own sources (Delta_0) set as bits of
 * plane d - 1 before the levels, so level d needs none of its peers' weight-d arcs. The targets
 * j0..j1 are this rank's rows and the graph is undirected, so an in-arc (k, w) of own target j is
 * the arc j -> k: bit j of row k. Weight 1 also goes into R (level 1 is these bits alone). */
__global__ void lvl_direct_kernel(int j0, int j1, int nw, int lw, size_t plane, const int32_t* __restrict__ off,
                                  const uint32_t* __restrict__ arcs, uint32_t* __restrict__ lev,
                                  uint32_t* __restrict__ R) {
    const int j = j0 + blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (j >= j1) return;
    const int a0 = off[(size_t)j * LVL_STRIDE + 1], a1 = off[(size_t)j * LVL_STRIDE + lw + 1];
    const int s = j - j0;
    const uint32_t bit = 1u << (s & 31);
    for (int i = a0 + lane; i < a1; i += 64) {
        const uint32_t e = arcs[i];
        const int k = (int)(e & 0xFFFFu), w = (int)(e >> 16);
        const size_t o = (size_t)k * nw + (s >> 5);
        atomicOr(lev + (size_t)(w - 1) * plane + o, bit);
        if (w == 1) atomicOr(R + o, bit);
    }
}

/* The solo rank's Delta_0 bits without synthesising its peers' segments first: peer target j's
 * runs are own row js's, every source moved by shift (lvl_solo_arcs_kernel), so its own-source
 * arcs are row js's arcs whose moved source falls in [row0, row0 + nrows). A wave per target, a
 * lane per arc of weight <= lw (as lvl_direct_kernel; a binary search per (target, weight) ran
 * 63 us on one rank of N = 8). */
__global__ void lvl_solo_direct_kernel(int n, int row0, int nrows, int lrows, int nw, int lw, size_t plane,
                                       const int32_t* __restrict__ off, const uint32_t* __restrict__ arcs,
                                       uint32_t* __restrict__ lev, uint32_t* __restrict__ R) {
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (j >= n) return;
    const bool own = j >= row0 && j < row0 + nrows;
    const int js = own ? j : row0 + ((j - row0) % lrows + lrows) % lrows;
    const int shift = own ? 0 : ((j - js) % n + n) % n;
    const int a0 = off[(size_t)js * LVL_STRIDE + 1], a1 = off[(size_t)js * LVL_STRIDE + lw + 1];
    for (int i = a0 + lane; i < a1; i += 64) {
        const uint32_t e = arcs[i];
        int k = (int)(e & 0xFFFFu) + shift;
        if (k >= n) k -= n;
        const int s = k - row0, w = (int)(e >> 16);
        if (s < 0 || s >= nrows) continue;
        const size_t o = (size_t)j * nw + (s >> 5);
        const uint32_t bit = 1u << (s & 31);
        atomicOr(lev + (size_t)(w - 1) * plane + o, bit);
        if (w == 1) atomicOr(R + o, bit);
    }
}

/* ---- N > 1: the first batch's in-arcs streamed weight by weight ----------------------------- *
 * Level d reads its peers' arcs of weight < d only (an arc of weight d matters to its own source
 * alone), so the segments travel one weight at a time on a second stream and level d waits for
 * weight d - 1 alone: the wire of weight d runs under level d's gathers. On the wire the arcs of
 * one weight are rank-major, target-major within (offw: the exclusive scan of the counts in
 * [weight][target] order, lvl_offsets_kernel), one u32 per arc -- its source and its
 * index into the union table of distinct reliabilities (or the source alone, with the f64 beside
 * it when the union passes the table) -- and each receiver places them into its (target,
 * weight)-major arcs (4 B per arc on the wire instead of 6). */
/* The wire of weight w: one block of maxc[w] u32 per rank (rank q's arcs of weight w, its targets
 * in order, then padding), all-gathered; wtab[2 (w - 1)] = the weight's base in the wire,
 * wtab[2 (w - 1) + 1] = maxc[w]; zw[(w - 1) (R + 1) + q] = offw at rank q's first target */
__global__ void lvl_wire_pack_kernel(int ld, int row0, int lrows, int lw, int R, int me,
                                     const int32_t* __restrict__ off, const int32_t* __restrict__ offw,
                                     const int32_t* __restrict__ zw, const int32_t* __restrict__ wtab,
                                     const uint32_t* __restrict__ arcs, const uint16_t* __restrict__ rix,
                                     const double* __restrict__ ar, uint32_t* __restrict__ wire,
                                     double* __restrict__ wire64) {
    const int jj = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (jj >= lrows) return;
    const int j = row0 + jj;
    for (int w = 1; w <= lw; ++w) {
        const int a0 = off[(size_t)j * LVL_STRIDE + w], c = off[(size_t)j * LVL_STRIDE + w + 1] - a0;
        const size_t o = (size_t)wtab[2 * (w - 1)] + (size_t)me * wtab[2 * (w - 1) + 1] +
                         (offw[(size_t)(w - 1) * ld + j] - zw[(w - 1) * (R + 1) + me]);
        for (int i = lane; i < c; i += 64) {
            wire[o + i] = (arcs[a0 + i] & 0xFFFFu) | (rix ? (uint32_t)rix[a0 + i] << 16 : 0u);
            if (wire64) wire64[o + i] = ar[a0 + i];
        }
    }
}
__global__ void lvl_wire_unpack_kernel(int n, int ld, int row0, int nrows, int w, int nw, int R,
                                       const int32_t* __restrict__ off, const int32_t* __restrict__ offw,
                                       const int32_t* __restrict__ zw, const int32_t* __restrict__ wtab,
                                       const uint32_t* __restrict__ wire, const double* __restrict__ wire64,
                                       uint32_t* __restrict__ arcs, uint16_t* __restrict__ rix,
                                       double* __restrict__ ar, uint32_t* __restrict__ aoff) {
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (j >= n || (j >= row0 && j < row0 + nrows)) return;
    const long long nb = ld / SRT_SHARD_ALIGN; /* the owner of row j (srt_shard_rows) */
    int q = 0;
    while (q + 1 < R && (int)(nb * (q + 1) / R) * SRT_SHARD_ALIGN <= j) ++q;
    const int a0 = off[(size_t)j * LVL_STRIDE + w], c = off[(size_t)j * LVL_STRIDE + w + 1] - a0;
    const size_t o = (size_t)wtab[2 * (w - 1)] + (size_t)q * wtab[2 * (w - 1) + 1] +
                     (offw[(size_t)(w - 1) * ld + j] - zw[(w - 1) * (R + 1) + q]);
    for (int i = lane; i < c; i += 64) {
        const uint32_t e = wire[o + i], k = e & 0xFFFFu;
        arcs[a0 + i] = k | ((uint32_t)w << 16);
        if (rix) rix[a0 + i] = (uint16_t)(e >> 16);
        if (wire64) ar[a0 + i] = wire64[o + i];
        aoff[a0 + i] = k * (uint32_t)nw * 4u;
    }
}
/* Offsets of the (target, weight <= lw) in-arcs without masking the counts or scanning all 256
 * weight columns: per target its arcs up to lw (lvl_tot_kernel), one scan over the targets, then
 * the target's weight prefixes (lvl_off_kernel writes off[j][0 .. lw + 1]; columns past lw + 1
 * are never read: every reader stops at lw + 1). The counts stay whole for a later, heavier
 * extraction. */
__global__ void lvl_tot_kernel(int ld, int lw, const int32_t* __restrict__ cnt, int32_t* __restrict__ tot) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > ld) return;
    int t = 0;
    if (j < ld)
        for (int w = 1; w <= lw; ++w) t += cnt[(size_t)j * LVL_STRIDE + w];
    tot[j] = t;
}
__global__ void lvl_off_kernel(int ld, int lw, const int32_t* __restrict__ cnt, const int32_t* __restrict__ base,
                               int32_t* __restrict__ off) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > ld) return;
    int run = base[j];
    off[(size_t)j * LVL_STRIDE] = run;
    if (j == ld) return;
    for (int w = 1; w <= lw; ++w) {
        off[(size_t)j * LVL_STRIDE + w] = run;
        run += cnt[(size_t)j * LVL_STRIDE + w];
    }
    off[(size_t)j * LVL_STRIDE + lw + 1] = run;
}

/* The offsets of a first extraction (lw <= LVL_BATCH) in two launches: per target the (target,
 * weight)-major starts off[j][0..lw + 1] and (offw != NULL, the streamed wire) the
 * [weight][target] scan offw with its values at the shard starts (dsz). A workgroup takes 256
 * targets, a thread one target. The first kernel sums each workgroup's columns (the target
 * totals and the lw weights); the second adds the earlier workgroups' sums, scans its targets and
 * writes. They replace seven launches (totals, two scans, offsets, columns, two scans, sizes).
 * (One workgroup doing it all ran ~0.4 ms: one CU's latency on a rank's critical path.) */
static __device__ __forceinline__ void lvl_off_cols(int ld, int lw, int j, const int32_t* __restrict__ cnt,
                                                    int (&x)[LVL_BATCH + 1]) {
    x[0] = 0;
#pragma unroll
    for (int w = 1; w <= LVL_BATCH; ++w) {
        x[w] = j < ld && w <= lw ? cnt[(size_t)j * LVL_STRIDE + w] : 0;
        x[0] += x[w];
    }
}
__global__ __launch_bounds__(256) void lvl_off_part_kernel(int ld, int lw, const int32_t* __restrict__ cnt,
                                                           int32_t* __restrict__ part) {
    __shared__ int ws[4][LVL_BATCH + 1];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int x[LVL_BATCH + 1];
    lvl_off_cols(ld, lw, blockIdx.x * 256 + tid, cnt, x);
#pragma unroll
    for (int c = 0; c <= LVL_BATCH; ++c) {
        int v = x[c];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) ws[wv][c] = v;
    }
    __syncthreads();
    if (tid <= LVL_BATCH) part[blockIdx.x * (LVL_BATCH + 1) + tid] = ws[0][tid] + ws[1][tid] + ws[2][tid] + ws[3][tid];
}
__global__ __launch_bounds__(256) void lvl_offsets_kernel(int ld, int lw, int R, const int32_t* __restrict__ cnt,
                                                          const int32_t* __restrict__ part, int32_t* __restrict__ off,
                                                          int32_t* __restrict__ offw, int32_t* __restrict__ dsz) {
    __shared__ int pre[LVL_BATCH + 1], tot[LVL_BATCH + 1], colB[LVL_BATCH + 2], ws[4][LVL_BATCH + 1];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, b = blockIdx.x, nb = gridDim.x;
    if (tid < 4 * (LVL_BATCH + 1)) { /* four threads per column: the earlier blocks' sums, all sums */
        const int c = tid >> 2, k = tid & 3;
        int p = 0, t = 0;
        for (int q = k; q < nb; q += 4) {
            const int v = part[q * (LVL_BATCH + 1) + c];
            t += v;
            if (q < b) p += v;
        }
        p += __shfl_xor(p, 1);
        p += __shfl_xor(p, 2);
        t += __shfl_xor(t, 1);
        t += __shfl_xor(t, 2);
        if (k == 0) {
            pre[c] = p;
            tot[c] = t;
        }
    }
    __syncthreads();
    if (tid == 0) { /* offw's base of each weight */
        int r = 0;
        for (int w = 1; w <= lw; ++w) {
            colB[w] = r;
            r += tot[w];
        }
        colB[lw + 1] = r;
    }
    const int j = b * 256 + tid;
    int x[LVL_BATCH + 1], ex[LVL_BATCH + 1];
    lvl_off_cols(ld, lw, j, cnt, x);
#pragma unroll
    for (int c = 0; c <= LVL_BATCH; ++c) {
        int v = x[c];
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(v, o);
            if (lane >= o) v += y;
        }
        ex[c] = v - x[c];
        if (lane == 63) ws[wv][c] = v;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c <= LVL_BATCH; ++c) {
        int add = pre[c];
        for (int v = 0; v < wv; ++v) add += ws[v][c];
        ex[c] += add;
    }
    if (j < ld) {
        int32_t* oj = off + (size_t)j * LVL_STRIDE;
        int r = ex[0];
        oj[0] = r;
#pragma unroll
        for (int w = 1; w <= LVL_BATCH; ++w)
            if (w <= lw) {
                oj[w] = r;
                r += x[w];
            }
        oj[lw + 1] = r;
        if (offw) {
#pragma unroll
            for (int w = 1; w <= LVL_BATCH; ++w)
                if (w <= lw) offw[(size_t)(w - 1) * ld + j] = colB[w] + ex[w];
            if (dsz && j % SRT_SHARD_ALIGN == 0) { /* a shard start (srt_shard_rows) */
                const long long nbs = ld / SRT_SHARD_ALIGN;
                for (int q = 0; q < R; ++q)
                    if ((int)(nbs * q / R) * SRT_SHARD_ALIGN == j)
                        for (int w = 1; w <= lw; ++w) dsz[(w - 1) * (R + 1) + q] = colB[w] + ex[w];
            }
        }
    } else if (j == ld) {
        off[(size_t)ld * LVL_STRIDE] = tot[0];
        if (offw) {
            offw[(size_t)lw * ld] = colB[lw + 1];
            if (dsz) /* q == R: the weight's end, the next weight's start */
                for (int w = 1; w <= lw; ++w) dsz[(w - 1) * (R + 1) + R] = colB[w + 1];
        }
    }
}

/* N > 1, the one exchange ahead of every decision (a sum all-reduce of int32; each rank fills
 * its own slots, the others stay zero): the weight histogram's 20-bit limbs (512) and the
 * allocation-failure count (+1 pad), every rank's own arcs per weight w <= LVL_BATCH as 16-bit
 * halves (R x 16), and every rank's distinct light reliabilities -- a header (probe overflow,
 * count) then up to LVL_RT_CAP values, as int32 pairs (R x (LVL_RT_CAP + 1) x 2). */
#define LVL_X_LIMBS (2 * LVL_STRIDE + 2)
#define LVL_X_CNT (2 * LVL_BATCH)
static size_t lvl_x_words(int R) { return LVL_X_LIMBS + (size_t)R * LVL_X_CNT + (size_t)R * (LVL_RT_CAP + 1) * 2; }
/* per rank q in [q0, q1) and weight w <= LVL_BATCH: its shard's arcs of weight w, into the
 * exchange as 16-bit halves (a rank counts its own shard; a solo rank every shard of its
 * synthesised counts) */
__global__ void lvl_rank_counts_kernel(int n, int ld, int R, int q0, const int32_t* __restrict__ cnt,
                                       int32_t* __restrict__ xcnt) {
    const int q = q0 + (int)blockIdx.y, w = 1 + (int)blockIdx.x;
    const long long nb = ld / SRT_SHARD_ALIGN;
    const int b = (int)(nb * q / R) * SRT_SHARD_ALIGN, e = min(n, (int)(nb * (q + 1) / R) * SRT_SHARD_ALIGN);
    unsigned s = 0;
    for (int j = b + threadIdx.x; j < e; j += blockDim.x) s += (unsigned)cnt[(size_t)j * LVL_STRIDE + w];
    for (int o = 32; o > 0; o >>= 1) s += (unsigned)__shfl_xor((int)s, o);
    __shared__ unsigned ws[4];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = ws[0] + ws[1] + ws[2] + ws[3];
        xcnt[(size_t)q * LVL_X_CNT + (w - 1) * 2] = (int32_t)(t & 0xFFFFu);
        xcnt[(size_t)q * LVL_X_CNT + (w - 1) * 2 + 1] = (int32_t)(t >> 16);
    }
}
/* the distinct reliabilities of this rank's light arcs (1 <= w <= wl) straight from the count
 * pass's stash: each workgroup dedupes a run of rows in its LDS table and writes the table out
 * whole (tabs[block], coalesced); lvl_rt_merge_kernel folds the tables into the global table H.
 * Inserting each workgroup's values straight into H (agent-scope atomics on ~500 hot lines, from
 * every workgroup) took 72 us on a rank of C4 at N = 8. */
__global__ __launch_bounds__(256) void lvl_rt_hash_stash_kernel(int nrows, int ld, int wl,
                                                                const uint32_t* __restrict__ stash,
                                                                const int32_t* __restrict__ scnt,
                                                                const double* __restrict__ r,
                                                                unsigned long long* __restrict__ H,
                                                                unsigned long long* __restrict__ tabs,
                                                                int* __restrict__ ovf) {
    __shared__ unsigned long long key[LVL_RT_LDS];
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int per = (nrows + (int)gridDim.x - 1) / (int)gridDim.x;
    const int r0 = (int)blockIdx.x * per, r1 = min(nrows, r0 + per);
    for (int k = tid; k < LVL_RT_LDS; k += 256) key[k] = ~0ull;
    __syncthreads();
    bool bad = false;
    constexpr int PL = LVL_STASH_SEG / 64; /* a segment's entries per lane, loaded together */
    for (int jj = r0; jj < r1; ++jj) { /* wave wv: the row's segment wv */
        const int m = scnt[(size_t)jj * 4 + wv];
        const uint32_t* sg = stash + (size_t)jj * LVL_STASH_CAP + wv * LVL_STASH_SEG;
        uint32_t e[PL];
#pragma unroll
        for (int q = 0; q < PL; ++q) e[q] = q * 64 + lane < m ? sg[q * 64 + lane] : 0u;
        unsigned long long v[PL];
#pragma unroll
        for (int q = 0; q < PL; ++q) {
            const uint32_t x = e[q] >> 16;
            v[q] = x >= 1u && x <= (uint32_t)wl
                       ? (unsigned long long)__double_as_longlong(r[(size_t)jj * ld + (e[q] & 0xFFFFu)])
                       : ~0ull;
        }
#pragma unroll
        for (int q = 0; q < PL; ++q) {
            if (v[q] == ~0ull) continue;
            unsigned h = lvl_rt_hash(v[q]) & (LVL_RT_LDS - 1u);
            int p = 0;
            for (; p < 64; ++p, h = (h + 1u) & (LVL_RT_LDS - 1u)) {
                unsigned long long y = __hip_atomic_load(&key[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (y == ~0ull) y = atomicCAS(&key[h], ~0ull, v[q]);
                if (y == ~0ull || y == v[q]) break;
            }
            if (p == 64) bad |= lvl_rt_global_slot(v[q], H) < 0;
        }
    }
    __syncthreads();
    for (int k = tid; k < LVL_RT_LDS; k += 256) tabs[(size_t)blockIdx.x * LVL_RT_LDS + k] = key[k];
    if (bad) *ovf = 1;
}
/* slot k of every workgroup table mostly holds the same value (the same hash, the same probe):
 * thread (k, chunk) walks LVL_RT_MC tables' slot k (independent loads) and inserts each value it
 * has not just inserted into H -- a few inserts per slot and chunk instead of one per table */
#define LVL_RT_MC 16
__global__ __launch_bounds__(256) void lvl_rt_merge_kernel(int ntab, const unsigned long long* __restrict__ tabs,
                                                           unsigned long long* __restrict__ H,
                                                           int* __restrict__ ovf) {
    const int k = (blockIdx.x * 256 + threadIdx.x) % LVL_RT_LDS;
    const int t0 = (blockIdx.x * 256 + threadIdx.x) / LVL_RT_LDS * LVL_RT_MC;
    if (t0 >= ntab) return;
    unsigned long long v[LVL_RT_MC];
#pragma unroll
    for (int t = 0; t < LVL_RT_MC; ++t) v[t] = t0 + t < ntab ? tabs[(size_t)(t0 + t) * LVL_RT_LDS + k] : ~0ull;
    unsigned long long seen[4] = {~0ull, ~0ull, ~0ull, ~0ull};
    bool bad = false;
#pragma unroll
    for (int t = 0; t < LVL_RT_MC; ++t) {
        if (v[t] == ~0ull || v[t] == seen[0] || v[t] == seen[1] || v[t] == seen[2] || v[t] == seen[3]) continue;
        bad |= lvl_rt_global_slot(v[t], H) < 0;
        seen[3] = seen[2];
        seen[2] = seen[1];
        seen[1] = seen[0];
        seen[0] = v[t];
    }
    if (bad) *ovf = 1;
}

/* the own arcs in [*lo, *hi): each one's byte offset of its source row (aoff) and its index into
 * the sorted table of distinct reliabilities (by value bits, binary search) -- one pass */
__global__ void lvl_own_index_kernel(const int32_t* __restrict__ lo, const int32_t* __restrict__ hi, int nw,
                                     const uint32_t* __restrict__ arcs, const double* __restrict__ ar,
                                     const unsigned long long* __restrict__ tab, int ntab,
                                     uint32_t* __restrict__ aoff, uint16_t* __restrict__ rix) {
    const int a = *lo, b = *hi;
    for (int i = a + blockIdx.x * blockDim.x + threadIdx.x; i < b; i += gridDim.x * blockDim.x) {
        aoff[i] = (arcs[i] & 0xFFFFu) * (uint32_t)nw * 4u;
        const unsigned long long v = (unsigned long long)__double_as_longlong(ar[i]);
        int l = 0, h = ntab - 1;
        while (l < h) {
            const int mid = (l + h) >> 1;
            if (tab[mid] < v) l = mid + 1;
            else h = mid;
        }
        rix[i] = (uint16_t)l;
    }
}

/* the second stream and the per-weight events of the streamed extraction, per state slot (made
 * once, kept: a stream's creation costs more than a build's host work) */
static hipStream_t g_lvl_cs[SRT_STATE_SLOTS];
static hipEvent_t g_lvl_ev[SRT_STATE_SLOTS][LVL_BATCH + 2];
static int lvl_side_stream(hipStream_t* cs, hipEvent_t** ev) {
    const int k = srt_state_slot();
    if (!g_lvl_cs[k]) {
        SRT_HIPCHK(hipStreamCreateWithFlags(&g_lvl_cs[k], hipStreamNonBlocking));
        for (int i = 0; i < LVL_BATCH + 2; i++)
            SRT_HIPCHK(hipEventCreateWithFlags(&g_lvl_ev[k][i], hipEventDisableTiming));
    }
    *cs = g_lvl_cs[k];
    *ev = g_lvl_ev[k];
    return SRT_OK;
}
/* the host-side set that deduplicates the exchanged reliability blocks, per slot */
static std::vector<unsigned long long> g_lvl_uset[SRT_STATE_SLOTS];
/* The build's host round trips (the exchange, the agreement, one vote per batch) go through
 * pinned staging, per slot, made once and grown when a larger exchange needs it: a copy to or
 * from pageable memory is staged by the runtime and blocks the calling thread. Layout (u64
 * words): the one-GPU histogram, the agreement and failure flag, the vote's read-back, then the
 * exchange, the union table and the wire's per-weight bases. */
#define LVL_PIN_HIST 0
#define LVL_PIN_AG LVL_STRIDE
#define LVL_PIN_HW (LVL_PIN_AG + 4)
#define LVL_PIN_X (LVL_PIN_HW + LVL_H_WORDS - LVL_H_INC)
static unsigned long long* g_lvl_pin[SRT_STATE_SLOTS];
static size_t g_lvl_pin_words[SRT_STATE_SLOTS];
static hipEvent_t g_lvl_wev[SRT_STATE_SLOTS];
static int lvl_pinned(size_t words, unsigned long long** p) {
    const int k = srt_state_slot();
    if (g_lvl_pin_words[k] < words) {
        if (g_lvl_pin[k]) SRT_HIPCHK(hipHostFree(g_lvl_pin[k]));
        g_lvl_pin[k] = NULL;
        g_lvl_pin_words[k] = 0;
        SRT_HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&g_lvl_pin[k]), words * sizeof(unsigned long long),
                                 hipHostMallocDefault));
        g_lvl_pin_words[k] = words;
    }
    *p = g_lvl_pin[k];
    return SRT_OK;
}
/* Wait for the stream with the calling thread spinning on an event. hipStreamSynchronize sleeps
 * on the completion interrupt past a short active window, and the wake-up cost 30-60 us per round
 * trip in the traces of one rank of N = 8 (three or four per build). */
static int lvl_wait(hipStream_t st) {
    hipEvent_t& e = g_lvl_wev[srt_state_slot()];
    if (!e) SRT_HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    SRT_HIPCHK(hipEventRecord(e, st));
    hipError_t r;
    while ((r = hipEventQuery(e)) == hipErrorNotReady) {
    }
    SRT_HIPCHK(r);
    return SRT_OK;
}

/* byte offset of each arc's source row inside a level plane (k * nw * 4; nw is this rank's) */
__global__ void lvl_aoff_kernel(int total, int nw, const uint32_t* __restrict__ arcs,
                                uint32_t* __restrict__ aoff) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < total) aoff[i] = (arcs[i] & 0xFFFFu) * (uint32_t)nw * 4u;
}

/* ---- the levels ---------------------------------------------------------------------------- */
/* R = {j} for the local sources j (distance 0), everything else empty */
__global__ void lvl_init_kernel(int n, int src0, int nsrc, int nw, uint32_t* __restrict__ R) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nsrc) return;
    const int j = src0 + i;
    if (j < n) R[(size_t)j * nw + (i >> 5)] = 1u << (i & 31);
}

/* Level 1 without the unit walk: Delta_1[j] = {s : w(s, j) = 1} (every arc is >= 1 quantum), so
 * the level is j's weight-1 in-arcs set as bits (~33 per C4 target) in a zeroed plane and in R.
 * A wave owns target j (its row of both), a lane an arc; the arcs are sorted by source, so lanes
 * of one word are adjacent: a segmented OR (shuffle-up scan) leaves each word's bits in its last
 * lane, which stores them. No atomics: a same-address counter atomic per wave alone cost 0.40 ms
 * on C4 (serialised at the memory side), so the host counts the level's pairs from the weight
 * histogram instead. */
__global__ __launch_bounds__(256) void lvl_first_kernel(int n, int nw, int src0, int nsrc,
                                                        const int32_t* __restrict__ off,
                                                        const uint32_t* __restrict__ arcs,
                                                        uint32_t* __restrict__ lev0,
                                                        uint32_t* __restrict__ R) {
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (j < n) {
        const int a0 = off[(size_t)j * LVL_STRIDE + 1], a1 = off[(size_t)j * LVL_STRIDE + 2];
        for (int i0 = a0; i0 < a1; i0 += 64) {
            const int i = i0 + lane;
            const int ks = i < a1 ? (int)(arcs[i] & 0xFFFFu) - src0 : -1;
            const bool in = ks >= 0 && ks < nsrc;
            const int wd = in ? ks >> 5 : -1 - lane; /* out-of-range lanes: words of their own */
            uint32_t bits = in ? 1u << (ks & 31) : 0u;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t yb = (uint32_t)__shfl_up((int)bits, o);
                const int yw = __shfl_up(wd, o);
                if (lane >= o && yw == wd) bits |= yb;
            }
            const int nwd = __shfl_down(wd, 1);
            if (in && (lane == 63 || nwd != wd)) {
                const size_t o = (size_t)j * nw + wd;
                lev0[o] |= bits;
                R[o] |= bits;
            }
        }
    }
}

/* Levels 2 and 3, the near part: the bits that arcs of weight d (Delta_0: the own source itself)
 * and of weight d - 1 (Delta_1) contribute to Delta_d[t], set into plane d - 1 before
 * lvl_step_kernel, which then skips that weight group (its gathers read a plane that is nearly
 * empty: Delta_1[u] is u's ~33 weight-1 in-arcs among n sources). Delta_1[u] is exactly u's
 * weight-1 run of in-arcs, so a wave per target t reads, for each in-arc (u, d - 1), u's run
 * (~130 B, coalesced) instead of one 256-B plane slice per source chunk, and ORs the sources
 * into an LDS copy of t's plane row, which it then writes whole. add: the row already holds the
 * own-arc bits (streamed N > 1, lvl_direct_kernel), so it is read first and the weight-d run is
 * not scanned. */
__global__ __launch_bounds__(256) void lvl_near_kernel(int d, int n, int nw, int src0, int nsrc, int add,
                                                       const int32_t* __restrict__ off,
                                                       const uint32_t* __restrict__ arcs,
                                                       uint32_t* __restrict__ lev) {
    extern __shared__ uint32_t near_row[]; /* per wave: nw words */
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + wv;
    uint32_t* row = near_row + (size_t)wv * nw;
    const size_t plane = (size_t)n * nw;
    uint32_t* prow = lev + (size_t)(d - 1) * plane + (size_t)(t < n ? t : 0) * nw;
    for (int i = lane; i < nw; i += 64) row[i] = t < n && add ? prow[i] : 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (t < n) {
        const int32_t* ot = off + (size_t)t * LVL_STRIDE;
        if (!add) /* the own sources' arcs of weight d into t */
            for (int i = ot[d] + lane; i < ot[d + 1]; i += 64) {
                const int ks = (int)(arcs[i] & 0xFFFFu) - src0;
                if (ks >= 0 && ks < nsrc) atomicOr(&row[ks >> 5], 1u << (ks & 31));
            }
        /* each in-arc (u, d - 1): u's weight-1 run. The runs' bounds of 64 arcs come in one
         * vector load per lane, then four runs are read at a time (their first 64 entries in
         * flight together; a longer run's tail after) */
        const int a1 = ot[d];
        for (int c0 = ot[d - 1]; c0 < a1; c0 += 64) {
            int ub0 = 0, ub1 = 0;
            if (c0 + lane < a1) {
                const int u = (int)(arcs[c0 + lane] & 0xFFFFu);
                ub0 = off[(size_t)u * LVL_STRIDE + 1];
                ub1 = off[(size_t)u * LVL_STRIDE + 2];
            }
            const int na = min(64, a1 - c0);
            for (int k = 0; k < na; k += 4) {
                uint32_t e[4];
                int b0[4], b1[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    b0[q] = k + q < na ? __builtin_amdgcn_readlane(ub0, k + q) : 0;
                    b1[q] = k + q < na ? __builtin_amdgcn_readlane(ub1, k + q) : 0;
                    e[q] = b0[q] + lane < b1[q] ? arcs[b0[q] + lane] : 0xFFFFFFFFu;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int ks = (int)(e[q] & 0xFFFFu) - src0;
                    if (e[q] != 0xFFFFFFFFu && ks >= 0 && ks < nsrc) atomicOr(&row[ks >> 5], 1u << (ks & 31));
                    for (int i = b0[q] + 64 + lane; i < b1[q]; i += 64) { /* (runs past 64) */
                        const int kt = (int)(arcs[i] & 0xFFFFu) - src0;
                        if (kt >= 0 && kt < nsrc) atomicOr(&row[kt >> 5], 1u << (kt & 31));
                    }
                }
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (t < n)
        for (int i = lane; i < nw; i += 64) prow[i] = row[i];
}

/* Level d: one wave per (target j, 64-word source chunk c). Units are handed out XCD-major (each
 * XCD takes a contiguous run of chunk-major units), so an XCD works on one source chunk at a time
 * and the Delta rows of that chunk are the only gathered data in its L2. */
static __device__ __forceinline__ uint32_t lvl_step_unit(unsigned g, int d, int direct, int n, int nw,
                                                       int nchunk, int src0, int nsrc, uint32_t& gath,
                                                       const int32_t* __restrict__ off,
                                                       const uint32_t* __restrict__ arcs,
                                                       const uint32_t* __restrict__ aoff,
                                                       uint32_t* __restrict__ lev,
                                                       uint32_t* __restrict__ R,
                                                       uint8_t* __restrict__ done,
                                                       int* __restrict__ incomplete) {
    const int tgrp = (n + 3) >> 2;
    const int c = (int)(g / (unsigned)tgrp);
    /* the wave index through readfirstlane: j is then wave-uniform to the compiler, so the offsets
     * and the arcs come through scalar loads and every gather's row address is an SGPR */
    const int j = (int)(g % (unsigned)tgrp) * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (c >= nchunk || j >= n) return 0u;
    const int lane = threadIdx.x & 63, word = c * 64 + lane;
    const bool valid = word < nw;
    const size_t plane = (size_t)n * nw; /* words per level */
    uint32_t* out = lev + (size_t)(d - 1) * plane + (size_t)j * nw + word;
    const size_t u = (size_t)j * nchunk + c;
    if (done[u]) {
        if (valid) *out = 0u;
        return 0u;
    }
    uint32_t acc = 0;
    const int32_t* oj = off + (size_t)j * LVL_STRIDE;
    /* arcs of weight d: the path (k, j) itself, Delta_0[k] = {k}; 64 arcs per step, one per lane,
     * and the few whose source lies in this unit's chunk go to the lane owning its word (direct:
     * lvl_direct_kernel left them in the plane) */
    if (direct) {
        if (valid) acc = *out;
    } else {
        const int a0 = oj[d], a1 = oj[d + 1], cw0 = c * 64 * 32;
        for (int i0 = a0; i0 < a1; i0 += 64) {
            const int i = i0 + lane;
            const int ks = i < a1 ? (int)(arcs[i] & 0xFFFFu) - src0 : -1;
            unsigned long long m = __ballot(ks >= 0 && ks < nsrc && (unsigned)(ks - cw0) < 64u * 32u);
            while (m) {
                const int j = __builtin_ctzll(m);
                m &= m - 1ull;
                const int kj = __builtin_amdgcn_readlane(ks, j);
                if ((kj >> 5) == word) acc |= 1u << (kj & 31);
            }
        }
    }
    /* arcs of weight w < d: Delta_{d-w}[k], one weight group at a time so the group's plane base is
     * one scalar pointer and an arc costs one VALU add (its row's byte offset k * nw * 4, aoff, plus
     * the lane's) and one gather; sixteen gathers in flight. Lanes past nw read word 0 of the row
     * (a valid address) and drop it, so the loop has no per-lane branch. */
    const uint32_t lane4 = (uint32_t)(valid ? word : 0) * 4u;
    /* The unit's settled sources, read before the gathers: once every source of the unit is
     * settled or found, the later gathers cannot change the level's new bits (acc & ~r), so the
     * walk stops. On C4 a source at distance 4 is nearly always found through a weight-1 arc from
     * a vertex at distance 3, so level 4 needs the first weight group alone wherever the unit
     * holds no source at distance 5. Sources past n (padding of the last shard) never appear:
     * they count as settled. */
    uint32_t* rp = R + (size_t)j * nw + word;
    const uint32_t r = valid ? *rp : 0u;
    const int s0 = src0 + word * 32;
    const uint32_t full = !valid ? 0u : s0 + 32 <= n ? 0xFFFFFFFFu : s0 >= n ? 0u : (1u << (n - s0)) - 1u;
    constexpr int LVL_SB = 16; /* (8 measured the same, 32/48 slower; pipelined batches did not help) */
    for (int w = 1; w < d; ++w) {
        if (direct == 2 && w == d - 1) continue; /* lvl_near_kernel set this group's bits */
        if (!__any(((acc | r) & full) != full)) break;
        const int g1 = oj[w + 1];
        const char* base = reinterpret_cast<const char*>(lev + (size_t)(d - w - 1) * plane);
        for (int i = oj[w]; i < g1; i += LVL_SB) { /* LVL_SB in flight, the tail predicated */
            uint32_t a[LVL_SB], v[LVL_SB];
#pragma unroll
            for (int q = 0; q < LVL_SB; ++q) a[q] = aoff[i + q]; /* padded: one scalar burst */
#pragma unroll
            for (int q = 0; q < LVL_SB; ++q)
                v[q] = i + q < g1 ? *reinterpret_cast<const uint32_t*>(base + (a[q] + lane4)) : 0u;
#pragma unroll
            for (int q = 0; q < LVL_SB; ++q) acc |= v[q];
            if (valid) gath += (uint32_t)min(LVL_SB, g1 - i); /* the lane's 4-B gathers */
            if (i + LVL_SB < g1 && !__any(((acc | r) & full) != full)) break;
        }
    }
    if (!valid) acc = 0;
    bool inc = false;
    uint32_t settled = 0;
    if (valid) {
        const uint32_t nb = acc & ~r;
        settled = (uint32_t)__builtin_popcount(nb);
        *out = nb;
        if (nb) *rp = r | nb;
        inc = ((r | nb) & full) != full;
    }
    /* completion: a flag, not a count -- one same-address atomic per wave serialised at the memory
     * side (~6 ms per level at C4's 524k units); the flag is read first (an L2 hit once set), so
     * only the first few waves of a level store it */
    const unsigned long long m = __ballot(inc);
    if (lane == 0) {
        if (!m)
            done[u] = 1;
        else if (!__hip_atomic_load(incomplete, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            __hip_atomic_store(incomplete, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return settled;
}

/* Persistent grid (a few workgroups per CU, each looping over unit blocks): the units live only a
 * few microseconds, so a one-shot grid of 131k workgroups was bound by workgroup dispatch. Block p
 * of XCD p % 8 takes that XCD's contiguous run of unit blocks (chunk-major): 0.69 ms per C4 level
 * against 0.80 when all XCDs walk the same chunk together (lvl_pred_kernel's order). */
__global__ __launch_bounds__(256) void lvl_step_kernel(int d, int direct, int n, int nw, int nchunk, int src0,
                                                       int nsrc, unsigned nblk,
                                                       const int32_t* __restrict__ off,
                                                       const uint32_t* __restrict__ arcs,
                                                       const uint32_t* __restrict__ aoff,
                                                       uint32_t* __restrict__ lev,
                                                       uint32_t* __restrict__ R,
                                                       uint8_t* __restrict__ done,
                                                       int* __restrict__ incomplete,
                                                       const int* __restrict__ prev,
                                                       unsigned long long* __restrict__ nset,
                                                       unsigned long long* __restrict__ ngath) {
    /* the levels are enqueued in batches without a host round trip per level: a level whose
     * predecessor settled every pair (prev == 0) has nothing to do */
    if (prev && !__hip_atomic_load(prev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    const unsigned x = blockIdx.x & 7u, per = nblk >> 3, L = gridDim.x >> 3;
    uint32_t settled = 0; /* pairs this lane settled (one add per block at the end) */
    uint32_t gath = 0;    /* 4-B words this lane gathered (the early exit makes it data-dependent) */
    for (unsigned u = blockIdx.x >> 3; u < per; u += L)
        settled += lvl_step_unit(x * per + u, d, direct, n, nw, nchunk, src0, nsrc, gath, off, arcs, aoff, lev, R,
                                 done, incomplete);
    unsigned long long c = settled, gb = gath;
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor(c, o);
        gb += __shfl_xor(gb, o);
    }
    __shared__ unsigned long long s_c[4], s_g[4];
    if ((threadIdx.x & 63) == 0) {
        s_c[threadIdx.x >> 6] = c;
        s_g[threadIdx.x >> 6] = gb;
    }
    __syncthreads();
    if (threadIdx.x == 0 && (s_c[0] | s_c[1] | s_c[2] | s_c[3]))
        atomicAdd(nset, s_c[0] + s_c[1] + s_c[2] + s_c[3]);
    if (threadIdx.x == 0 && (s_g[0] | s_g[1] | s_g[2] | s_g[3]))
        atomicAdd(ngath, 4ull * (s_g[0] + s_g[1] + s_g[2] + s_g[3]));
}

/* Distance rows of the local sources from the levels: the u32 table rows (SRT_INF on padding) and
 * the u8 level rows the reliability pass reads (0 on the diagonal and padding) -- the FW finish
 * pass folded in: every settled distance is <= the level budget (<= 254), so the rows are exact
 * and small by construction. Thread = four consecutive targets t0..t0 + 3 (256 threads = 1,024
 * targets per workgroup), looping over 16 source words: per word it reads the four targets' word
 * of every level (the same lines for the 16 words of a workgroup row), keeps the 32 sources' four
 * distances as bytes (0xFF: none; 32 VGPRs, 8 waves per SIMD) and writes 16 B of u32 and 4 B of u8
 * per source row. */
__global__ __launch_bounds__(256) void lvl_out_kernel(int n, int ld, int nw, int src0, int nlev,
                                                      const uint32_t* __restrict__ lev,
                                                      uint32_t* __restrict__ lat,
                                                      uint8_t* __restrict__ l8) {
    const int t0 = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (t0 >= ld) return;
    const size_t plane = (size_t)n * nw;
    const int sw1 = min(nw, (int)(blockIdx.y + 1) * 16);
    for (int sw = blockIdx.y * 16; sw < sw1; ++sw) {
        uint32_t v[32]; /* per source: the distances to t0..t0 + 3, one byte each */
        const int sg0 = src0 + sw * 32;
#pragma unroll
        for (int s = 0; s < 32; ++s) {
            const int sg = sg0 + s;
            uint32_t x = 0xFFFFFFFFu;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (sg == t0 + q) x &= ~(0xFFu << (8 * q));
            v[s] = x;
        }
        for (int d = 1; d <= nlev; ++d) {
            uint32_t m[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                m[q] = t0 + q < n ? lev[(size_t)(d - 1) * plane + (size_t)(t0 + q) * nw + sw] : 0u;
            if (!(m[0] | m[1] | m[2] | m[3])) continue;
#pragma unroll
            for (int s = 0; s < 32; ++s) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if ((m[q] >> s) & 1u)
                        v[s] = (v[s] & ~(0xFFu << (8 * q))) | ((uint32_t)d << (8 * q));
            }
        }
#pragma unroll
        for (int s = 0; s < 32; ++s) {
            const size_t o = (size_t)(sw * 32 + s) * ld + t0;
            uint32_t x[4], b = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t y = (v[s] >> (8 * q)) & 0xFFu;
                x[q] = y == 0xFFu ? SRT_INF : y;
                b |= (y == 0xFFu ? 0u : y) << (8 * q);
            }
            *reinterpret_cast<uint4*>(lat + o) = make_uint4(x[0], x[1], x[2], x[3]);
            *reinterpret_cast<uint32_t*>(l8 + o) = b;
        }
    }
}

/* The same rows for builds of at most LVL_OUT_L levels, without lvl_out_kernel's re-fetches (its
 * 4-B plane reads come back 16 times per 64-B sector: C4 fetched 8.9 GB for 0.65 GB of planes).
 * Workgroup = 256 targets x 8 source words: every level's 8 words of every target are staged in
 * LDS with one 32-B read per (target, level), then thread = one target runs over the 8 words (256
 * sources) from LDS, keeping a word's 32 distances as bytes, and writes 4 B of u32 and 1 B of u8
 * per source row (a wave's 64 consecutive targets: 256 B / 64 B runs). */
#define LVL_OUT_L 16
__global__ __launch_bounds__(256) void lvl_out8_kernel(int n, int ld, int nw, int src0, int nlev,
                                                       const uint32_t* __restrict__ lev,
                                                       uint32_t* __restrict__ lat,
                                                       uint8_t* __restrict__ l8) {
    extern __shared__ uint4 smo[]; /* [level][half][target]: words w0..w0+3 | +4..+7 (8 KB per level) */
    auto sm = reinterpret_cast<uint4(*)[2][256]>(smo);
    const int tid = threadIdx.x, t = blockIdx.x * 256 + tid;
    const int w0 = blockIdx.y * 8;
    const size_t plane = (size_t)n * nw;
    const bool tv = t < n;
    for (int d = 0; d < nlev; ++d) {
        uint4 a = make_uint4(0u, 0u, 0u, 0u), b = a;
        if (tv) { /* nw is a multiple of 4 (nsrc % 128 == 0): 16-B aligned words */
            const uint4* p = reinterpret_cast<const uint4*>(lev + (size_t)d * plane + (size_t)t * nw + w0);
            a = p[0];
            b = w0 + 4 < nw ? p[1] : make_uint4(0u, 0u, 0u, 0u);
        }
        sm[d][0][tid] = a;
        sm[d][1][tid] = b;
    }
    /* (thread tid reads back only its own entries: no barrier needed) */
    if (t >= ld) return;
    const int k1 = min(8, nw - w0);
    for (int k = 0; k < k1; ++k) {
        uint32_t v[8]; /* sources 4i..4i+3 of the word, one byte each (0xFF: none) */
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = 0xFFFFFFFFu;
        const int sg0 = src0 + (w0 + k) * 32;
        if (t >= sg0 && t < sg0 + 32) { /* the diagonal */
            const int sd = t - sg0;
            v[sd >> 2] &= ~(0xFFu << (8 * (sd & 3)));
        }
        for (int d = 0; d < nlev; ++d) {
            const uint4 q = sm[d][k >> 2][tid];
            const uint32_t m = (k & 3) == 0 ? q.x : (k & 3) == 1 ? q.y : (k & 3) == 2 ? q.z : q.w;
            if (!m) continue;
#pragma unroll
            for (int sidx = 0; sidx < 32; ++sidx)
                if ((m >> sidx) & 1u)
                    v[sidx >> 2] = (v[sidx >> 2] & ~(0xFFu << (8 * (sidx & 3)))) |
                                   ((uint32_t)(d + 1) << (8 * (sidx & 3)));
        }
#pragma unroll
        for (int sidx = 0; sidx < 32; ++sidx) {
            const size_t o = (size_t)((w0 + k) * 32 + sidx) * ld + t;
            const uint32_t y = (v[sidx >> 2] >> (8 * (sidx & 3))) & 0xFFu;
            lat[o] = y == 0xFFu ? SRT_INF : y;
            l8[o] = (uint8_t)(y == 0xFFu ? 0u : y);
        }
    }
}

/* per-target segment starts of the (target, weight) offsets, for the segmented sort */
__global__ void lvl_segs_kernel(int ld, const int32_t* __restrict__ off, int32_t* __restrict__ seg) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j <= ld) seg[j] = off[(size_t)j * LVL_STRIDE];
}

/* PT = uint32_t: the packed form -- one word per pair, (u16) predecessor | reliability index << 16
 * (the arc's reliability is rtab[index], lvl_rtab_*), written into predT; rT and ar unused */
/* Canonical predecessors from the levels (the rule of every build kernel: among the tight in-arcs
 * u -> t, D[s][u] + w = D[s][t], the smallest (D[s][u], u) -- so the largest w, then the smallest u;
 * Dijkstra with a (dist, vertex) heap, topology.c:1679-1701 up to igraph's tie order).
 * One wave per (target t, 64-word source chunk), the same units as lvl_step_kernel. For the
 * sources at level d (Delta_d[t]) the arcs are taken by weight w = d, d - 1, ..., 1 and, inside a
 * weight, by ascending u (the in-arcs are sorted so): the arc (u, w) is tight for exactly the
 * sources in Delta_{d-w}[u] (u itself when w = d), and a source takes its first tight arc. A source
 * hit by two arcs of its winning weight is a tied pair (srt_build_stats.tied_pairs). A level stops
 * as soon as every source of the wave has its arc. Outputs, target-major as pred_cols*_kernel's
 * (stride ldp): predT[t][sl] = u (-1 on the diagonal), rT[t][sl] = r(u, t). */
template <typename PT>
static __device__ __forceinline__ void lvl_pred_unit(unsigned g, uint16_t (*sidx)[64 * 40], int n,
                                                     int nw, int nchunk, int src0, int nsrc, int nlev,
                                                       const int32_t* __restrict__ off,
                                                       const uint32_t* __restrict__ arcs,
                                                       const uint32_t* __restrict__ aoff,
                                                       const double* __restrict__ ar,
                                                       const uint16_t* __restrict__ rix,
                                                       const uint32_t* __restrict__ lev,
                                                       PT* __restrict__ predT,
                                                       double* __restrict__ rT, size_t ldp,
                                                       unsigned long long* __restrict__ ties) {
    constexpr bool PK = std::is_same_v<PT, uint32_t>;
    const int tgrp = (n + 3) >> 2;
    const int c = (int)(g / (unsigned)tgrp);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int t = (int)(g % (unsigned)tgrp) * 4 + wv;
    if (c >= nchunk || t >= n) return;
    const int lane = threadIdx.x & 63, word = c * 64 + lane;
    const bool valid = word < nw;
    const size_t plane = (size_t)n * nw;
    uint16_t* my = &sidx[wv][lane * 40];
#pragma unroll
    for (int q = 0; q < 32; q += 8)
        *reinterpret_cast<uint4*>(my + q) = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    const int32_t* ot = off + (size_t)t * LVL_STRIDE;
    const int a_t = ot[0];
    const uint32_t lane4 = (uint32_t)(valid ? word : 0) * 4u;
    unsigned tied = 0;
    /* one arc's candidates: x = its tight sources among the pending ones */
    auto take = [&](uint32_t x, uint32_t& H, uint32_t& T, int i) {
        uint32_t nb = x & ~H;
        T |= x & H;
        H |= x;
        while (nb) {
            my[__builtin_ctz(nb)] = (uint16_t)(i - a_t);
            nb &= nb - 1u;
        }
    };
    /* PK: the level of each of the lane's 32 sources as five bit planes (level <= 31), so the
     * packed word carries it (pred | rix << 16 | level << 27) for rel_pk_kernel */
    uint32_t lvb[5] = {0u, 0u, 0u, 0u, 0u};
    for (int d = 1; d <= nlev; ++d) {
        uint32_t pend = valid ? lev[(size_t)(d - 1) * plane + (size_t)t * nw + word] : 0u;
        if constexpr (PK) {
#pragma unroll
            for (int k = 0; k < 5; ++k)
                if ((d >> k) & 1) lvb[k] |= pend;
        }
        if (!__any(pend != 0u)) continue;
        for (int w = d; w >= 1; --w) {
            const int g0 = ot[w], g1 = ot[w + 1];
            if (g0 == g1) continue;
            uint32_t H = 0, T = 0;
            if (w == d) {
                /* the direct arc (u, t): tight for the source u itself. 64 arcs per step, one per
                 * lane; the few whose source lies in this unit's chunk (~2 of C4's ~33 per
                 * weight) go to the lane owning the source's word. Distinct arcs have distinct
                 * sources, so there are no ties here and the order does not matter. */
                const int cw0 = c * 64 * 32; /* the chunk's first source (local index) */
                for (int i0 = g0; i0 < g1; i0 += 64) {
                    const int i = i0 + lane;
                    const int us = i < g1 ? (int)(arcs[i] & 0xFFFFu) - src0 : -1;
                    unsigned long long m =
                        __ballot(us >= 0 && us < nsrc && (unsigned)(us - cw0) < 64u * 32u);
                    while (m) {
                        const int j = __builtin_ctzll(m);
                        m &= m - 1ull;
                        const int uj = __builtin_amdgcn_readlane(us, j);
                        if ((uj >> 5) == word) take(pend & (1u << (uj & 31)), H, T, i0 + j);
                    }
                }
            }
            else { /* sixteen gathers in flight (a predicated tail), then their candidates in
                      * arc order */
                const char* base = reinterpret_cast<const char*>(lev + (size_t)(d - w - 1) * plane);
                /* LVL_PB gathers per batch, software-pipelined: the next batch's gathers are in
                 * flight while this batch's candidates are taken (C4: 7.2 -> 5.1 ms against 16
                 * unpipelined; 12 keeps 7 waves per SIMD -- 16 pipelined, 84 VGPRs and 5 waves,
                 * measured 6.2) */
                uint32_t v[LVL_PB], vn[LVL_PB];
                {
                    uint32_t a[LVL_PB];
#pragma unroll
                    for (int q = 0; q < LVL_PB; ++q) a[q] = aoff[g0 + q];
#pragma unroll
                    for (int q = 0; q < LVL_PB; ++q)
                        v[q] = g0 + q < g1 ? *reinterpret_cast<const uint32_t*>(base + (a[q] + lane4)) : 0u;
                }
                for (int i = g0; i < g1; i += LVL_PB) {
                    const int i2 = i + LVL_PB;
                    if (i2 < g1) {
                        uint32_t a[LVL_PB];
#pragma unroll
                        for (int q = 0; q < LVL_PB; ++q) a[q] = aoff[i2 + q];
#pragma unroll
                        for (int q = 0; q < LVL_PB; ++q)
                            vn[q] = i2 + q < g1 ? *reinterpret_cast<const uint32_t*>(base + (a[q] + lane4)) : 0u;
                    }
#pragma unroll
                    for (int q = 0; q < LVL_PB; ++q) take(v[q] & pend, H, T, i + q);
#pragma unroll
                    for (int q = 0; q < LVL_PB; ++q) v[q] = vn[q];
                    /* without the tie count the first tight arc is all a source needs: the walk
                     * of the weight ends once every pending source has one */
                    if (!ties && !__any((pend & ~H) != 0u)) break;
                }

            }
            tied += __builtin_popcount(T);
            pend &= ~H;
            if (!__any(pend != 0u)) break;
        }
    }
    if (ties) {
        for (int m = 32; m > 0; m >>= 1) tied += __shfl_xor(tied, m);
        if (lane == 0 && tied) atomicAdd(&ties[blockIdx.x & 1023u], (unsigned long long)tied);
    }
    /* Output, coalesced: the wave writes its 2,048 sources in four quarters of 512, lane l taking
     * 8 consecutive sources (another lane's entries, back from LDS), so every store instruction
     * covers one contiguous run (1 KB of int16 predecessors, 4 KB of reliabilities per quarter)
     * instead of 64 strided 16-B pieces. The walk's LDS writes are the wave's own. */
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int cs0 = c * 64 * 32; /* the chunk's first local source */
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int sl0 = cs0 + q * 512 + lane * 8;
        /* the levels of sources sl0 .. sl0 + 7: bits (lane & 3) * 8.. of word q * 16 + lane / 4,
         * which lane q * 16 + lane / 4 holds (every lane takes part in the shuffles) */
        uint32_t lq[5];
#pragma unroll
        for (int k = 0; k < 5; ++k)
            lq[k] = PK ? ((uint32_t)__shfl((int)lvb[k], q * 16 + (lane >> 2)) >> ((lane & 3) * 8)) : 0u;
        if (sl0 >= nsrc) continue; /* nsrc is a multiple of 128: whole groups of 8 */
        const uint4 raw =
            *reinterpret_cast<const uint4*>(&sidx[wv][(q * 16 + (lane >> 2)) * 40 + (lane & 3) * 8]);
        const uint32_t ix[4] = {raw.x, raw.y, raw.z, raw.w};
        int32_t pv[8];
        double rv[8];
        uint32_t kv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const uint32_t x = (ix[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
            const int sg = src0 + sl0 + e;
            const bool h = sg < n && sg != t && x != 0xFFFFu;
            const int k = a_t + (h ? (int)x : 0);
            pv[e] = h ? (int)(arcs[k] & 0xFFFFu) : -1;
            if constexpr (PK) {
                uint32_t l = 0;
#pragma unroll
                for (int kk = 0; kk < 5; ++kk) l |= ((lq[kk] >> e) & 1u) << kk;
                kv[e] = ((uint32_t)pv[e] & 0xFFFFu) | (h ? (uint32_t)rix[k] << 16 : 0u) |
                        (h ? l << 27 : 0u);
            }
            else
                rv[e] = h ? ar[k] : 0.0;
        }
        PT* pp = predT + (size_t)t * ldp + sl0;
        if constexpr (PK) { /* 32 B per lane: a wave's quarter is one 2-KB run */
            /* non-temporal: the words do not displace the gathered plane slices from the MALL
             * (5.16 against 5.31-5.36 ms with plain stores, r05pn) */
            typedef unsigned u32x4n __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store((u32x4n){kv[0], kv[1], kv[2], kv[3]}, reinterpret_cast<u32x4n*>(pp));
            __builtin_nontemporal_store((u32x4n){kv[4], kv[5], kv[6], kv[7]}, reinterpret_cast<u32x4n*>(pp + 4));
            continue;
        }
        double* rp = rT + (size_t)t * ldp + sl0;
        if constexpr (sizeof(PT) == 2) { /* -1 -> 0xFFFF, read back as int16 -1 */
            uint32_t w2[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
                w2[e] = ((uint32_t)pv[2 * e] & 0xFFFFu) | ((uint32_t)pv[2 * e + 1] << 16);
            *reinterpret_cast<uint4*>(pp) = make_uint4(w2[0], w2[1], w2[2], w2[3]);
        } else {
            *reinterpret_cast<int4*>(pp) = make_int4(pv[0], pv[1], pv[2], pv[3]);
            *reinterpret_cast<int4*>(pp + 4) = make_int4(pv[4], pv[5], pv[6], pv[7]);
        }
#pragma unroll
        for (int e = 0; e < 8; e += 2)
            *reinterpret_cast<double2*>(rp + e) = make_double2(rv[e], rv[e + 1]);
    }
}

template <typename PT>
/* The units walked chunk-major by all eight XCDs together (block u * 8 + XCD): the planes'
 * gathered slices are one source chunk's at a time for the whole GPU (8 MB per plane, in the
 * MALL), where XCD-private runs of chunks had 16 chunks' slices in flight (~384 MB on C4): 8.16
 * against 8.40 ms on C4. */
__global__ __launch_bounds__(256) void lvl_pred_kernel(int n, int nw, int nchunk, int src0, int nsrc,
                                                       int nlev, unsigned nblk,
                                                       const int32_t* __restrict__ off,
                                                       const uint32_t* __restrict__ arcs,
                                                       const uint32_t* __restrict__ aoff,
                                                       const double* __restrict__ ar,
                                                       const uint16_t* __restrict__ rix,
                                                       const uint32_t* __restrict__ lev,
                                                       PT* __restrict__ predT,
                                                       double* __restrict__ rT, size_t ldp,
                                                       unsigned long long* __restrict__ ties) {
    /* per wave and lane: the winning arc of each of its 32 sources (index into t's arcs), 40 u16
     * per lane so the read-back is four 16-B loads */
    __shared__ __attribute__((aligned(16))) uint16_t sidx[4][64 * 40];
    const unsigned x = blockIdx.x & 7u, per = nblk >> 3, L = gridDim.x >> 3;
    for (unsigned u = blockIdx.x >> 3; u < per; u += L)
        lvl_pred_unit<PT>(u * 8u + x, sidx, n, nw, nchunk, src0, nsrc, nlev, off, arcs, aoff, ar,
                          rix, lev, predT, rT, ldp, ties);
}

__global__ void lvl_sum_kernel(const unsigned long long* __restrict__ v, int k,
                               unsigned long long* __restrict__ out) {
    unsigned long long s = 0;
    for (int i = threadIdx.x; i < k; i += blockDim.x) s += v[i];
    for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m);
    __shared__ unsigned long long w[16];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long x = 0;
        for (int i = 0; i < (int)(blockDim.x >> 6); i++) x += w[i];
        *out += x;
    }
}

/* ---- host ----------------------------------------------------------------------------------- */
/* Streaming-gather rate assumed by the level budget (bytes per ms) and the cost of one level's
 * launch + completion read-back. */
#define LVL_BYTES_PER_MS 4.0e9
#define LVL_LEVEL_MS 0.03

/* Estimated time of levels 1..L (ms): every level gathers one 4-B word per (arc of weight < d,
 * source word) and reads/writes R and Delta once. */
/* the largest level budget L whose predicted time stays within limit_ms: level d gathers a row of
 * nw words per arc of weight < d and touches three planes (one running sum, not a sum per L: the
 * budget of a graph like C4 passes 200 levels, and the quadratic form cost ~30 us of host time
 * on every build's critical path) */
static int lvl_budget(const unsigned long long* hist, double ntgt, double nw, double limit_ms) {
    double t = 0, below = 0; /* arcs with weight < d */
    int L = 0;
    for (int d = 1; d <= LVL_WMAX; ++d) {
        if (d >= 2) below += (double)hist[d - 1];
        t += (below * nw * 4.0 + ntgt * nw * 4.0 * 3.0) / LVL_BYTES_PER_MS + LVL_LEVEL_MS;
        if (t > limit_ms) break;
        L = d;
    }
    return L;
}

/* persistent grid of a 256-thread unit kernel: its resident workgroups per CU x the CUs, a multiple
 * of 8 (one share per XCD), at most the unit blocks */
static unsigned lvl_grid(const void* fn, unsigned nblk, int reserve_cus = 0) {
    int dev = 0, cus = 256, per = 4;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    cus = max(8, cus - reserve_cus);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 256, 0) != hipSuccess || per < 1) per = 4;
    (void)hipGetLastError();
    unsigned g = (unsigned)(cus * per) & ~7u;
    if (g < 8) g = 8;
    return g < nblk ? g : nblk;
}

/* The state a successful level build keeps for its post pass (srt_levels_pred), per state slot:
 * the sorted in-arcs with their reliabilities and the level planes. Freed by srt_levels_release
 * (stream-ordered). */
typedef struct {
    int held;
    int n, nw, nchunk, row0, nrows, D;
    unsigned nblk;
    int32_t* off;
    uint32_t* arcs;
    uint32_t* aoff;
    double* ar;
    uint16_t* rix; /* packed form: each arc's index into rtab (NULL: more than LVL_RT_CAP values) */
    double* rtab;
    int ntab;
    uint32_t* lev;
    uint8_t* l8; /* u8 distance rows (nrows x ld) for the reliability pass */
    int pkw;     /* the post pass is the packed words with levels + rel_pk (no lat / l8 rows) */
    int total;   /* in-arcs held (w <= lmax) */
    unsigned long long* dkey; /* the diagonal rule's key per local row (undirected rows form) */
    const double* r_rows;
    void* p[40]; /* every allocation of the build (LVL_ALLOC), freed together */
    int k;
    hipStream_t st;
    hipEvent_t wlast; /* the streamed extraction's last weight (side stream), or NULL */
} lvl_state;
static lvl_state g_lvl[SRT_STATE_SLOTS];

static void lvl_free(lvl_state* L, hipStream_t st) {
    if (L->wlast) (void)hipStreamWaitEvent(st, L->wlast, 0); /* the side stream is done with them */
    for (int i = 0; i < L->k; i++)
        if (L->p[i]) (void)hipFreeAsync(L->p[i], st);
    memset(L, 0, sizeof(*L));
}

void srt_levels_release(hipStream_t st) { lvl_free(&g_lvl[srt_state_slot()], st); }

/* the diagonal rule of the held build's rows into d / rel (row stride ld); 0 = applied, 1 = the
 * build kept no keys (directed: the caller's dense_diag_kernel) */
int srt_levels_diag(int n, int ld, uint32_t* d, double* rel, hipStream_t st, int* applied) {
    const lvl_state* L = &g_lvl[srt_state_slot()];
    *applied = 0;
    if (!L->held || !L->dkey) return SRT_OK;
    const int lrows = max(0, min(L->nrows, n - L->row0));
    if (lrows > 0)
        lvl_diag_kernel<<<srt_ceil_div(lrows, 256), 256, 0, st>>>(n, ld, L->row0, lrows, L->dkey,
                                                                  L->r_rows, d, rel);
    SRT_HIPCHK(hipGetLastError());
    *applied = 1;
    return SRT_OK;
}

/* the held build's table of distinct arc reliabilities (packed form), NULL when it has none */
const double* srt_levels_rtab(int* ntab) {
    const lvl_state* L = &g_lvl[srt_state_slot()];
    *ntab = L->held && L->rix ? L->ntab : 0;
    return L->held && L->rix ? L->rtab : NULL;
}

const uint8_t* srt_levels_l8(void) {
    const lvl_state* L = &g_lvl[srt_state_slot()];
    return L->held ? L->l8 : NULL;
}

#define LVL_ALLOC(ptr, bytes)                                      \
    do {                                                           \
        if (L->k >= (int)(sizeof(L->p) / sizeof(L->p[0]))) {       \
            srt_set_error("levels: allocation table full");        \
            return SRT_E_NOMEM;                                    \
        }                                                          \
        SRT_HIPCHK(srt_malloc_async(&(ptr), (bytes), st));         \
        L->p[L->k++] = (void*)(ptr);                               \
    } while (0)
/* the same, but a failed allocation only clears *ok (the caller agrees on a verdict first) */
#define LVL_TRY_ALLOC(ptr, bytes, ok)                                                   \
    do {                                                                                \
        (ptr) = NULL;                                                                   \
        if (*(ok) && L->k < (int)(sizeof(L->p) / sizeof(L->p[0])) &&                    \
            srt_malloc_async(&(ptr), (bytes), st) == hipSuccess) {                      \
            L->p[L->k++] = (void*)(ptr);                                                \
        } else {                                                                        \
            (void)hipGetLastError();                                                    \
            (ptr) = NULL;                                                               \
            *(ok) = 0;                                                                  \
        }                                                                               \
    } while (0)

/* One stream-ordered allocation for a group of buffers (each 256-B aligned): a build's ~20
 * scratch buffers cost one pool call instead of twenty on the host's critical path */
struct lvl_arena {
    void** p[24];
    size_t b[24];
    int k = 0;
    template <typename T>
    void add(T** ptr, size_t bytes) {
        p[k] = reinterpret_cast<void**>(ptr);
        b[k++] = bytes;
    }
    size_t total() const {
        size_t t = 0;
        for (int i = 0; i < k; i++) t += (b[i] + 255) & ~(size_t)255;
        return t;
    }
    void carve(char* base) const {
        for (int i = 0; i < k; i++) {
            *p[i] = base;
            base += (b[i] + 255) & ~(size_t)255;
        }
    }
};

/* bytes the build can still take from the device: free memory plus what the library's scratch
 * pool holds unused (its release threshold keeps freed blocks mapped) */
static size_t lvl_avail_bytes(void) {
    const int cap_mb = srt_form_int("memcap", -1); /* test hook: a nearly full device */
    if (cap_mb >= 0) return (size_t)cap_mb << 20;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    uint64_t res = 0, used = 0;
    hipMemPool_t pool = srt_scratch_pool();
    if (hipMemPoolGetAttribute(pool, hipMemPoolAttrReservedMemCurrent, &res) == hipSuccess &&
        hipMemPoolGetAttribute(pool, hipMemPoolAttrUsedMemCurrent, &used) == hipSuccess && res > used)
        fr += (size_t)(res - used);
    (void)hipGetLastError();
    return fr;
}

/* settled fraction of all pairs the first batch must reach for the build to go on */
#define LVL_MIN_SETTLED 0.25

/* The host-side words of a build (one allocation, zeroed): the weight histogram, the completion
 * flags, the agreement words and the settled-pair counter, and the batch vote. Offsets in u64. */
#define LVL_H_INC 256                            /* int dinc[LVL_WMAX + 1], then dflag[2] */
#define LVL_H_AGREE 512                          /* int32 agreement words [3]; u64 nset at +2 */
#define LVL_H_VOTE 520                           /* int32 [4] */
#define LVL_H_WORDS (LVL_H_VOTE + 2)

/* N > 1, the end of a batch of levels: this rank's vote -- not done (its last level left a pair
 * unsettled) and its settled-pair count in 21-bit limbs -- for one sum all-reduce, so every rank
 * takes the batch's decision (stop, continue, extract heavier arcs, or Floyd-Warshall) from the
 * same numbers */
__global__ void lvl_vote_kernel(const int* __restrict__ inc_last,
                                const unsigned long long* __restrict__ nset,
                                int32_t* __restrict__ vote) {
    if (threadIdx.x) return;
    const unsigned long long s = *nset;
    vote[0] = *inc_last != 0;
    vote[1] = (int32_t)(s & 0x1FFFFFull);
    vote[2] = (int32_t)((s >> 21) & 0x1FFFFFull);
    vote[3] = (int32_t)(s >> 42);
}

/* One build of the local rows' distances (nrows x ld). comm (NULL on one GPU): undirected row
 * shards, every rank sees every target's in-arcs after the segment broadcasts. fw_ms: the
 * predicted Floyd-Warshall time (of the largest shard); the level budget keeps the predicted level
 * time under half of it. *levels = the level that settled every pair (0: not applicable / over
 * budget / out of memory -- the caller runs Floyd-Warshall). *gather_bytes: the Delta words
 * gathered (the kernel's algorithmic bytes). On success the slot keeps the arcs and the planes for
 * the post pass until srt_levels_release; lat_rows hold the u32 rows, unless the post pass writes
 * them itself (srt_levels_pkw_ready).
 *
 * The N > 1 protocol. Every branch after the first collective is taken on values every rank holds
 * alike -- the exchanged histogram and blocks, the agreed budget, allocation outcome and wire, and
 * each batch's summed vote -- so every rank makes the same collective calls in the same order and
 * no rank leaves while its peers wait in one. In order:
 *   1. one sum all-reduce of the exchange (lvl_x_words): the histogram limbs, the allocation-
 *      failure count, every rank's arcs per weight w <= LVL_BATCH, every rank's distinct light
 *      reliabilities (so the union table and the wire's block sizes need no later round trip);
 *   2. one min all-reduce of (budget, allocation outcome, wire allocated) -- each rank allocated
 *      for its own budget, which is at least the agreed one;
 *   3. the (target, weight <= lmax) counts (sum);
 *   4. the first batch's arcs: streamed, one all-gather per weight w <= lx (every rank's block
 *      padded to the largest), sent one weight ahead of the levels on the side stream; or, where
 *      that form does not apply, extract(): the reliability blocks' all-gather and one broadcast
 *      group of the segments;
 *   5. per batch of levels (1-5, then 6, 7, 8 one at a time, then 8 at a time) the vote
 *      (sum); after the batch ending at lx < lmax, extract(lmax) as in 4's second form.
 * The vote's "all done" is the verdict. tests/test_dist_gloo.py rehearses this sequence over gloo
 * and tests/test_gpu_protocol.py checks every rank's collective log (srt_comm_log_*) against it. */
int srt_levels_build(const srt_comm* comm, int n, int ld, int row0, int nrows, int directed,
                     const uint32_t* w_rows, const double* r_rows, uint32_t* lat_rows, double fw_ms,
                     hipStream_t st, evpool_t* evp, int* levels, int64_t* gather_bytes) {
    *levels = 0;
    *gather_bytes = 0;
    lvl_state* L = &g_lvl[srt_state_slot()];
    if (L->held) lvl_free(L, st);
    const int R = comm ? srt_comm_size(comm) : 1;
    /* rank-independent applicability: the shards are SRT_SHARD_ALIGN (128) aligned, so nrows %
     * 128 == 0 on every rank once ld % 128 == 0; the 32-bit plane offsets are checked against the
     * largest shard */
    if (n > 65535 || ld % 128 || nrows % 128 || row0 % 128 || R > 64) return SRT_OK;
    if (R > 1 && directed) return SRT_OK; /* in-arcs of a directed graph span every rank's rows */
    int max_rows = nrows;
    for (int q = 0; q < R && R > 1; q++) {
        int32_t b = 0, e = 0;
        srt_shard_rows(ld, SRT_SHARD_ALIGN, R, q, &b, &e);
        max_rows = max(max_rows, e - b);
    }
    if ((size_t)n * (size_t)(max_rows / 32) * 4 > 0xFFFFFFFFull) return SRT_OK; /* 32-bit offsets */
    const int nw = nrows / 32, nchunk = (nw + 63) / 64;
    /* a timing-only communicator (srt_comm_init_solo*, tools/solo_rank.py): the rank does a real
     * rank's work on its own rows and synthesises what its peers would send (lvl_solo_*) */
    const bool solo = R > 1 && srt_comm_is_solo(comm);
    const int lrows = min(nrows, max(0, n - row0));
    L->st = st;
    /* on any early return below the allocations go back (lvl_free), unless the build is held */
    struct guard {
        lvl_state* L;
        hipStream_t st;
        ~guard() {
            if (!L->held) lvl_free(L, st);
        }
    } gd{L, st};
    const size_t ncnt = (size_t)ld * LVL_STRIDE;
    unsigned long long* dhist = NULL; /* the host-side words (LVL_H_*), a few KB */
    LVL_ALLOC(dhist, LVL_H_WORDS * sizeof(unsigned long long));
    SRT_HIPCHK(hipMemsetAsync(dhist, 0, LVL_H_WORDS * sizeof(unsigned long long), st));
    int* dinc = reinterpret_cast<int*>(dhist + LVL_H_INC);
    int32_t* dagree = reinterpret_cast<int32_t*>(dhist + LVL_H_AGREE);
    int32_t* dvote = reinterpret_cast<int32_t*>(dhist + LVL_H_VOTE);
    int* dflag = dinc + LVL_WMAX + 1; /* [0] probe overflow, [1] distinct values */
    const int me = R > 1 ? srt_comm_rank(comm) : 0;
    /* the count pass's buffers, softly: a rank short of memory sends every rank to the FW through
     * the failure count it adds to the exchange (its slots stay zero) */
    int ok = 1;
    int32_t *cnt = NULL, *off = NULL, *tb = NULL, *xbuf = NULL;
    unsigned long long* dkey = NULL;
    uint32_t* stash = NULL;
    int32_t* scnt = NULL;
    unsigned long long* H = NULL;
    uint16_t* map = NULL;
    /* a group of buffers in one allocation (soft: a failure clears *okp) */
    auto commit = [&](const lvl_arena& a, int* okp) {
        char* base = NULL;
        if (a.k) LVL_TRY_ALLOC(base, a.total(), okp);
        if (base) a.carve(base);
    };
    lvl_arena a1;
    a1.add(&cnt, (ncnt + 1) * sizeof(int32_t));
    a1.add(&off, (ncnt + 1) * sizeof(int32_t));
    a1.add(&tb, 2 * ((size_t)ld + 1) * sizeof(int32_t)); /* per-target totals, their scan */
    a1.add(&H, LVL_RT_SLOTS * sizeof(unsigned long long));
    a1.add(&map, LVL_RT_SLOTS * sizeof(uint16_t));
    if (!directed) {
        a1.add(&dkey, (size_t)nrows * sizeof(unsigned long long));
        a1.add(&stash, (size_t)nrows * LVL_STASH_CAP * sizeof(uint32_t));
        a1.add(&scnt, (size_t)nrows * 4 * sizeof(int32_t));
    }
    const size_t xn = R > 1 ? lvl_x_words(R) : 0;
    if (R > 1) a1.add(&xbuf, xn * sizeof(int32_t));
    commit(a1, &ok);
    constexpr size_t LVL_GB = LVL_RT_CAP + 1;
    int32_t* const xlimbs = xbuf;
    int32_t* const xcnt = xbuf ? xbuf + LVL_X_LIMBS : NULL;
    int32_t* const xblk = xbuf ? xcnt + (size_t)R * LVL_X_CNT : NULL; /* R blocks of LVL_GB u64 */
    if (ok) {
        SRT_HIPCHK(hipMemsetAsync(cnt, 0, (ncnt + 1) * sizeof(int32_t), st));
        if (directed)
            lvl_arcs_cols_kernel<false><<<ld / 64, 256, 0, st>>>(n, ld, w_rows, cnt, 0, NULL, NULL);
        else
            lvl_arcs_rows_kernel<false><<<nrows, 256, 0, st>>>(n, ld, row0, w_rows, cnt, 0, NULL, NULL,
                                                               NULL, NULL, dkey, stash, scnt, dhist);
        if (solo && lrows > 0) lvl_solo_counts_kernel<<<n, 256, 0, st>>>(n, row0, nrows, lrows, cnt);
        SRT_HIPCHK(hipGetLastError());
        /* this rank's rows (a solo rank: every row of its synthesised counts, which are its own
         * rows' n / lrows times over when that divides) */
        const bool rep = solo && lrows > 0 && lrows == nrows && n % lrows == 0;
        const bool own = R > 1 && (!solo || rep);
        lvl_hist_kernel<<<own ? 256 : 1024, 256, 0, st>>>(own ? (size_t)(rep ? lrows : nrows) * LVL_STRIDE : ncnt,
                                                         own ? cnt + (size_t)row0 * LVL_STRIDE : cnt, dhist,
                                                         rep ? (unsigned)(n / lrows) : 1u);
        SRT_HIPCHK(hipGetLastError());
        if (R > 1) {
            SRT_HIPCHK(hipMemsetAsync(xbuf, 0, xn * sizeof(int32_t), st));
            lvl_hist_limbs_kernel<<<1, LVL_STRIDE, 0, st>>>(1, dhist, xlimbs);
            lvl_rank_counts_kernel<<<dim3(LVL_BATCH, solo ? R : 1), 256, 0, st>>>(n, ld, R, solo ? 0 : me, cnt, xcnt);
            if (!directed && lrows > 0) { /* this rank's distinct light reliabilities, its block */
                int32_t* hd = xblk + (size_t)me * LVL_GB * 2;
                SRT_HIPCHK(hipMemsetAsync(H, 0xFF, LVL_RT_SLOTS * sizeof(unsigned long long), st));
                /* the workgroup tables in the offsets' buffer (free until the offsets) */
                size_t ntb = (ncnt + 1) * sizeof(int32_t) / (LVL_RT_LDS * sizeof(unsigned long long));
                ntb = ntb < 512 ? ntb : 512;
                ntb = ntb < (size_t)lrows ? ntb : (size_t)lrows;
                const int nt = (int)(ntb > 0 ? ntb : 1);
                unsigned long long* tabs = reinterpret_cast<unsigned long long*>(off);
                lvl_rt_hash_stash_kernel<<<nt, 256, 0, st>>>(lrows, ld, LVL_BATCH, stash, scnt, r_rows, H,
                                                             tabs, hd);
                lvl_rt_merge_kernel<<<LVL_RT_LDS / 256 * srt_ceil_div(nt, LVL_RT_MC), 256, 0, st>>>(nt, tabs, H, hd);
                lvl_rt_compact_kernel<<<1, 1024, 0, st>>>(H, map, reinterpret_cast<double*>(hd + 2), hd + 1);
            }
            SRT_HIPCHK(hipGetLastError());
        }
    }
    int rc;
    unsigned long long* pin;
    if ((rc = lvl_pinned(LVL_PIN_X + (R > 1 ? (xn + 1) / 2 + LVL_RT_CAP + 2 * LVL_BATCH + 4 : 4), &pin)))
        return rc;
    int32_t* hx = reinterpret_cast<int32_t*>(pin + LVL_PIN_X); /* the exchange, back on the host */
    unsigned long long* ht = pin + LVL_PIN_X + (xn + 1) / 2;    /* the union table, then its flags */
    int32_t* hwt = reinterpret_cast<int32_t*>(ht + LVL_RT_CAP + 2); /* the wire's per-weight base, block */
    int32_t* hag = reinterpret_cast<int32_t*>(pin + LVL_PIN_AG);    /* the agreement, the failure flag */
    int failed = !ok;
    if (R > 1) {
        hag[3] = failed;
        SRT_HIPCHK(hipMemcpyAsync(xlimbs + 2 * LVL_STRIDE, &hag[3], sizeof(int32_t), hipMemcpyHostToDevice, st));
        if ((rc = srt_coll_allreduce_i32(comm, xbuf, xn, 0, st))) return rc;
        SRT_HIPCHK(hipMemcpyAsync(hx, xbuf, xn * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    }
    unsigned long long hist[LVL_STRIDE];
    if (R == 1)
        SRT_HIPCHK(hipMemcpyAsync(pin + LVL_PIN_HIST, dhist, sizeof(hist), hipMemcpyDeviceToHost, st));
    if ((rc = lvl_wait(st))) return rc;
    if (R == 1) memcpy(hist, pin + LVL_PIN_HIST, sizeof(hist));
    if (R > 1) { /* the summed histogram from its limbs, on the host (one read-back) */
        failed = hx[2 * LVL_STRIDE];
        for (int i = 0; i < LVL_STRIDE; i++)
            hist[i] = (unsigned long long)(uint32_t)hx[i] + ((unsigned long long)(uint32_t)hx[LVL_STRIDE + i] << 20);
    }
    if (failed) return SRT_OK; /* out of device memory somewhere: Floyd-Warshall on every rank */
    /* the union of every rank's distinct light reliabilities (sorted by bits: the same table on
     * every rank) and, per weight <= LVL_BATCH, the largest rank's arcs (the streamed wire's
     * block): both from the exchange, so the streamed extraction needs no further round trip */
    /* The blocks come in hash-slot order and mostly repeat each other (C4: ~500 values per rank,
     * the same ones), so they are deduplicated through an open-addressing set first and only the
     * distinct values sorted: sorting the concatenation (4,000 values at N = 8) cost ~0.1-0.2 ms of
     * host time on the critical path. A solo rank's peers hold its own values (their rows are
     * shifted copies of its rows), so it pays the same. */
    std::vector<unsigned long long> u;
    bool fit = R > 1;
    if (fit) {
        size_t all = 0;
        for (int q = 0; q < R && fit; q++) {
            const int32_t* hd = hx + LVL_X_LIMBS + (size_t)R * LVL_X_CNT + (size_t)(solo ? me : q) * LVL_GB * 2;
            if (hd[0] || hd[1] > LVL_RT_CAP) fit = false;
            all += (size_t)max(hd[1], 0);
        }
        size_t cap = 64;
        while (cap < 2 * all) cap <<= 1;
        std::vector<unsigned long long>& set = g_lvl_uset[srt_state_slot()];
        set.assign(cap, ~0ull); /* (a NaN pattern: never a reliability's bits) */
        int shift = 64;
        for (size_t c = cap; c > 1; c >>= 1) --shift;
        for (int q = 0; q < R && fit; q++) {
            const int32_t* hd = hx + LVL_X_LIMBS + (size_t)R * LVL_X_CNT + (size_t)(solo ? me : q) * LVL_GB * 2;
            const unsigned long long* v = reinterpret_cast<const unsigned long long*>(hd + 2);
            for (int k = 0; k < hd[1]; ++k) {
                size_t h = (size_t)((v[k] * 0x9E3779B97F4A7C15ull) >> shift);
                while (set[h] != ~0ull && set[h] != v[k]) h = (h + 1) & (cap - 1);
                if (set[h] == ~0ull) {
                    set[h] = v[k];
                    u.push_back(v[k]);
                }
            }
        }
        if (fit) {
            std::sort(u.begin(), u.end());
            fit = !u.empty() && u.size() <= (size_t)LVL_RT_CAP;
        }
    }
    /* level budget from global quantities (the summed histogram, the largest shard's words): the
     * largest L whose predicted time stays under half the FW time */
    const double nw_all = (double)max_rows / 32.0;
    int lmax = lvl_budget(hist, (double)n, nw_all, 0.5 * fw_ms);
    /* and by memory: the planes (lmax x n x nw words) within half of what the device has left */
    const size_t plane = (size_t)n * nw;
    if (plane > 0) {
        const size_t cap = lvl_avail_bytes() / 2 / (plane * sizeof(uint32_t));
        if ((size_t)lmax > cap) lmax = (int)cap;
    }
    if (R > 1) { /* test hook: this rank's memory stands in for a smaller budget (lcap_r<rank>) */
        char key[32];
        snprintf(key, sizeof(key), "lcap_r%d", me);
        const int lc = srt_form_int(key, -1);
        if (lc >= 0 && lc < lmax) lmax = lc;
    }
    /* Every allocation of the build up front, softly, sized by THIS rank's budget: the agreed
     * budget is the ranks' minimum, so the buffers fit it. Then one min all-reduce agrees the
     * budget, the allocation outcome and whether the wire could be allocated. */
    const int lmax_own = max(lmax, 0);
    int64_t total64 = 0;
    for (int x = 1; x <= lmax_own; ++x) total64 += (int64_t)hist[x];
    const int32_t total_own = (int32_t)(total64 < 0x7FFFFFF0ll ? total64 : 0x7FFFFFF0ll);
    uint32_t *arcs = NULL, *arcs2 = NULL, *aoff = NULL, *lev = NULL, *Rb = NULL;
    double *ar = NULL, *ar2 = NULL;
    int32_t* seg = NULL;
    void *tmp = NULL, *stmp = NULL;
    uint8_t* done = NULL;
    size_t tmp_bytes = 0, sb = 0;
    SRT_HIPCHK(hipcub::DeviceScan::ExclusiveSum(NULL, tmp_bytes, cnt, off, (int)(ncnt + 1), st));
    const bool need_sort_own = total_own > 0 && !(!directed && lmax_own <= LVL_STASH_W && hist[0] == 0);
    if (need_sort_own)
        SRT_HIPCHK(hipcub::DeviceSegmentedRadixSort::SortPairs(NULL, sb, arcs, arcs2, ar, ar2, total_own,
                                                               ld, seg, seg + 1, 0, 24, st));
    lvl_arena a2;
    if (total64 <= 0x7FFFFFF0ll && lmax_own >= 2) {
        a2.add(&tmp, tmp_bytes);
        a2.add(&arcs, ((size_t)total_own + 8) * sizeof(uint32_t));
        a2.add(&ar, ((size_t)total_own + 8) * sizeof(double));
        if (need_sort_own) {
            a2.add(&arcs2, ((size_t)total_own + 8) * sizeof(uint32_t));
            a2.add(&ar2, ((size_t)total_own + 8) * sizeof(double));
            a2.add(&seg, ((size_t)ld + 1) * sizeof(int32_t));
            a2.add(&stmp, sb);
        }
        a2.add(&aoff, ((size_t)total_own + 64) * sizeof(uint32_t)); /* + a gather batch's tail */
        a2.add(&lev, (size_t)lmax_own * plane * sizeof(uint32_t) + 16);
        a2.add(&Rb, plane * sizeof(uint32_t) + 16);
        a2.add(&done, (size_t)n * nchunk + 16);
    }
    /* the distinct arc reliabilities (packed post pass, n <= 32768) */
    uint16_t* rix = NULL;
    double* rtab = NULL;
    if (total_own > 0 && n <= 32768) {
        a2.add(&rix, ((size_t)total_own + 8) * sizeof(uint16_t));
        a2.add(&rtab, LVL_RT_CAP * sizeof(double));
    }
    /* N > 1: the segments' reliability blocks (extract()), the counts' all-gather blocks (u16,
     * every weight up to the budget), and the streamed wire's offsets at the shard starts */
    double* gat = NULL;
    if (total_own > 0 && n <= 32768 && R > 1) a2.add(&gat, (size_t)R * LVL_GB * sizeof(double));
    uint16_t* cg = NULL;
    int32_t* packed = NULL;
    if (R > 1) {
        a2.add(&cg, ((size_t)R * max_rows * max(lmax_own, 1) + 8) * sizeof(uint16_t));
        a2.add(&packed, (size_t)4 * LVL_BATCH * 65 * sizeof(int32_t));
    }
    commit(a2, &ok);
    /* the streamed first extraction's wire (extract_streamed): every rank's block of a weight
     * padded to the largest; needs the union table (fit) and at most 2 GB */
    const int lx_own = min(lmax_own, LVL_BATCH);
    size_t wire_words = 0;
    for (int x = 1; x <= lx_own && R > 1; ++x) {
        int mx = 0;
        for (int q = 0; q < R; q++) {
            const int32_t* c = hx + LVL_X_LIMBS + (size_t)q * LVL_X_CNT + (x - 1) * 2;
            mx = max(mx, (int)((uint32_t)c[0] | ((uint32_t)c[1] << 16)));
        }
        wire_words += (size_t)R * mx;
    }
    int32_t* offw = NULL;
    uint32_t* wire = NULL;
    int stream_ok = R > 1 && !directed && hist[0] == 0 && fit && n <= 32768 && lx_own >= 1 &&
                    srt_form_int("pkw", 1) != 0 && (double)wire_words * 4.0 < 2e9;
    if (stream_ok && ok) {
        int sok = 1;
        lvl_arena a3;
        a3.add(&offw, ((size_t)lx_own * ld + 1) * sizeof(int32_t));
        /* (also the [weight][target] counts before their scan) */
        a3.add(&wire, max(wire_words + 8, (size_t)lx_own * ld + 1) * sizeof(uint32_t));
        commit(a3, &sok);
        stream_ok = sok;
    }
    /* N > 1: what needs no agreed value is done on the side stream while the main stream
     * carries the agreement and the count all-gather (on the main stream it delayed them): the
     * level state's zeroing and, for the streamed extraction, the union table and the wire's
     * per-weight bases, sized by this rank's budget (lx_own >= the agreed lx; the entries of the
     * weights up to lx are the same either way). The main stream waits for it (wev[prep]) before
     * the extraction; wasted when a rank falls back. */
    hipEvent_t* wev = NULL; /* wev[w]: the arcs of weight w are in place on this rank */
    hipStream_t wcs = NULL; /* the side stream */
    const int prep = LVL_BATCH + 1;
    bool prepped = false;
    if (R > 1 && ok && Rb && done) { /* (not allocated under a budget below 2) */
        if ((rc = lvl_side_stream(&wcs, &wev))) return rc;
        SRT_HIPCHK(hipEventRecord(wev[prep], st)); /* the allocations are ordered on st */
        SRT_HIPCHK(hipStreamWaitEvent(wcs, wev[prep], 0));
        prepped = true;
    }
    if (R > 1) { /* the agreement goes out first; the side stream's calls are made under it */
        hag[0] = lmax;
        hag[1] = ok;
        hag[2] = stream_ok;
        SRT_HIPCHK(hipMemcpyAsync(dagree, hag, 3 * sizeof(int32_t), hipMemcpyHostToDevice, st));
        if ((rc = srt_coll_allreduce_i32(comm, dagree, 3, 1, st))) return rc;
        SRT_HIPCHK(hipMemcpyAsync(hag, dagree, 3 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    }
    if (prepped) {
        SRT_HIPCHK(hipMemsetAsync(Rb, 0, plane * sizeof(uint32_t), wcs));
        SRT_HIPCHK(hipMemsetAsync(done, 0, (size_t)n * nchunk, wcs));
        lvl_init_kernel<<<srt_ceil_div(nrows, 256), 256, 0, wcs>>>(n, row0, nrows, nw, Rb);
        SRT_HIPCHK(hipGetLastError());
    }
    if (prepped && stream_ok && lev && rtab) {
        SRT_HIPCHK(hipMemsetAsync(lev, 0, (size_t)lx_own * plane * sizeof(uint32_t), wcs));
        const int nu = (int)u.size();
        memcpy(ht, u.data(), u.size() * sizeof(unsigned long long));
        const int hf[2] = {0, nu};
        memcpy(ht + LVL_RT_CAP, hf, sizeof(hf));
        SRT_HIPCHK(hipMemcpyAsync(rtab, ht, (size_t)nu * sizeof(double), hipMemcpyHostToDevice, wcs));
        SRT_HIPCHK(hipMemcpyAsync(dflag, ht + LVL_RT_CAP, 2 * sizeof(int), hipMemcpyHostToDevice, wcs));
        /* the wire: per weight every rank's block padded to the largest rank's arcs (from the
         * exchange's per-rank counts): the weight's base and that block size */
        size_t base = 0;
        for (int w = 1; w <= lx_own; ++w) {
            int mx = 0;
            for (int q = 0; q < R; q++) {
                const int32_t* c = hx + LVL_X_LIMBS + (size_t)q * LVL_X_CNT + (w - 1) * 2;
                mx = max(mx, (int)((uint32_t)c[0] | ((uint32_t)c[1] << 16)));
            }
            hwt[2 * (w - 1)] = (int32_t)base;
            hwt[2 * (w - 1) + 1] = mx;
            base += (size_t)R * mx;
        }
        SRT_HIPCHK(hipMemcpyAsync(packed + LVL_BATCH * 65, hwt, 2 * (size_t)lx_own * sizeof(int32_t),
                                  hipMemcpyHostToDevice, wcs));
    }
    if (prepped) SRT_HIPCHK(hipEventRecord(wev[prep], wcs));
    if (R > 1) {
        if ((rc = lvl_wait(st))) return rc;
        lmax = hag[0];
        ok = hag[1];
        stream_ok = hag[2];
    }
    /* From here every branch reads agreed or global values only: hist is summed over the ranks
     * (hist[0] is the stash-overflow count), the budget, the allocation outcome and the wire are
     * agreed. In-arcs come out of the ordered stash already in (weight, source) order, on every
     * rank, when no row overflowed its stash: no sort. */
    int wmin = 0;
    for (int x = 1; x <= LVL_WMAX && !wmin; ++x)
        if (hist[x]) wmin = x;
    if (lmax < 2 || !wmin || wmin > lmax) return SRT_OK;
    total64 = 0;
    for (int x = 1; x <= lmax; ++x) total64 += (int64_t)hist[x];
    if (total64 > 0x7FFFFFF0ll) return SRT_OK; /* int32 arc offsets (global) */
    if (!ok) return SRT_OK; /* out of device memory somewhere: Floyd-Warshall on every rank */
    const int32_t total = (int32_t)total64;
    const bool want_rt = total > 0 && n <= 32768;
    /* The in-arcs are extracted for the first batch of levels only (w <= lx = min(lmax, LVL_BATCH):
     * levels d <= lx use no heavier arc) and again up to lmax if the levels run past it: C4 ends
     * at level 5, and its ~20-quantum budget would extract, number and (N > 1) send 2.5x the arcs
     * it uses. The counts stay whole (narrow offsets) for the second extraction. */
    const int lx = min(lmax, LVL_BATCH);
    /* every target's counts of weights w0..w1 on every rank (a solo rank has them: synthesised) */
    auto share_counts = [&](int w0, int w1) -> int {
        if (R == 1 || w1 < w0) return SRT_OK;
        const size_t blk = (size_t)max_rows * (w1 - w0 + 1);
        if (nrows > 0)
            lvl_cnt_gpack_kernel<<<srt_ceil_div(nrows, 256), 256, 0, st>>>(row0, nrows, max_rows, w0, w1, me,
                                                                           cnt, cg);
        SRT_HIPCHK(hipGetLastError());
        int rc_ = srt_coll_allgather(comm, cg, blk * sizeof(uint16_t), st);
        if (rc_) return rc_;
        if (!solo) lvl_cnt_gunpack_kernel<<<srt_ceil_div(ld, 256), 256, 0, st>>>(ld, R, max_rows, w0, w1, cg, cnt);
        SRT_HIPCHK(hipGetLastError());
        return SRT_OK;
    };
    if ((rc = share_counts(1, lx))) return rc; /* the first extraction's weights */
    /* offsets of the (target, weight <= lw) in-arcs: narrow scan, counts untouched */
    auto offsets = [&](int lw, int32_t* ow = NULL, int32_t* osz = NULL) -> int {
        if (lw <= LVL_BATCH) { /* a first extraction: two launches (with the wire's offsets) */
            const int nb = (ld + 1 + 255) / 256; /* (the thread of target ld writes the totals) */
            lvl_off_part_kernel<<<nb, 256, 0, st>>>(ld, lw, cnt, tb);
            lvl_offsets_kernel<<<nb, 256, 0, st>>>(ld, lw, R, cnt, tb, off, ow, osz);
            SRT_HIPCHK(hipGetLastError());
            return SRT_OK;
        }
        lvl_tot_kernel<<<srt_ceil_div(ld + 1, 256), 256, 0, st>>>(ld, lw, cnt, tb);
        SRT_HIPCHK(hipGetLastError());
        SRT_HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, tb, tb + ld + 1, ld + 1, st));
        lvl_off_kernel<<<srt_ceil_div(ld + 1, 256), 256, 0, st>>>(ld, lw, cnt, tb + ld + 1, off);
        SRT_HIPCHK(hipGetLastError());
        return SRT_OK;
    };
    uint32_t* const arcsA = arcs;
    double* const arA = ar;
    int32_t total_x = 0;          /* the arcs of the current extraction */
    auto extract = [&](int lw) -> int {
        int numbered = 0; /* the segments travelled as arcs + table indices */
        int64_t t64 = 0;
        for (int x = 1; x <= lw; ++x) t64 += (int64_t)hist[x];
        total_x = (int32_t)t64;
        const int sorted_w = !directed && lw <= LVL_STASH_W && hist[0] == 0; /* global values */
        int rc_ = offsets(lw); /* (target, weight <= lw)-major */
        if (rc_) return rc_;
        if (directed)
            lvl_arcs_cols_kernel<true><<<ld / 64, 256, 0, st>>>(n, ld, w_rows, NULL, lw, off, arcsA,
                                                                r_rows, arA);
        else
            lvl_arcs_rows_kernel<true><<<nrows, 256, 0, st>>>(n, ld, row0, w_rows, NULL, lw, off, arcsA,
                                                              r_rows, arA, NULL, stash, scnt);
        SRT_HIPCHK(hipGetLastError());
        if (R > 1) { /* every rank filled its rows' segment: broadcast the segments */
            int32_t hoff[65];
            for (int q = 0; q <= R; q++) {
                int32_t b = ld, e = ld;
                if (q < R) srt_shard_rows(ld, SRT_SHARD_ALIGN, R, q, &b, &e);
                SRT_HIPCHK(hipMemcpyAsync(&hoff[q], off + (size_t)b * LVL_STRIDE, sizeof(int32_t),
                                          hipMemcpyDeviceToHost, st));
            }
            if ((rc_ = lvl_wait(st))) return rc_;
            /* Numbered segments: the packed post pass needs each arc's index into the table of
             * distinct reliabilities, not its f64. Each rank numbers its own segment's values
             * (hash + compact), the blocks are all-gathered (16 KB per rank), every rank takes
             * the union sorted by value bits -- the same table everywhere -- and the segments
             * travel as arcs + u16 indices: 6 B per arc instead of 12. Taken when the post pass
             * will be the packed one (levels <= lw <= 31, pkw) and the fill needs no sort (the
             * sort carries the f64s); more than LVL_RT_CAP values in the union (or a probe
             * overflow) keeps the f64 segments, on every rank alike. */
            const int me = srt_comm_rank(comm);
            /* the arcs this process numbers: its own segment, or (solo) every segment at once,
             * in block 0 */
            const int nb0 = hoff[me], nb1 = hoff[me + 1], qb = me;
            if (gat && sorted_w && lw <= 31 && srt_form_int("pkw", 1) != 0) {
                SRT_HIPCHK(hipMemsetAsync(gat, 0, (size_t)R * LVL_GB * sizeof(double), st));
                if (nb1 > nb0) {
                    SRT_HIPCHK(hipMemsetAsync(dflag, 0, 2 * sizeof(int), st));
                    SRT_HIPCHK(hipMemsetAsync(H, 0xFF, LVL_RT_SLOTS * sizeof(unsigned long long), st));
                    lvl_rt_hash_kernel<<<lvl_rt_grid(nb1 - nb0), 256, 0, st>>>(NULL, NULL, nb0, nb1, arA, H,
                                                                              rix, dflag);
                    lvl_rt_compact_kernel<<<1, 1024, 0, st>>>(H, map, gat + qb * LVL_GB + 1, dflag + 1);
                    SRT_HIPCHK(hipGetLastError());
                    SRT_HIPCHK(hipMemcpyAsync(gat + qb * LVL_GB, dflag, 2 * sizeof(int),
                                              hipMemcpyDeviceToDevice, st));
                }
                if ((rc_ = srt_coll_allgather(comm, gat, LVL_GB * sizeof(double), st))) return rc_;
                std::vector<unsigned long long> hg((size_t)R * LVL_GB);
                SRT_HIPCHK(hipMemcpyAsync(hg.data(), gat, hg.size() * sizeof(unsigned long long),
                                          hipMemcpyDeviceToHost, st));
                if ((rc_ = lvl_wait(st))) return rc_;
                std::vector<unsigned long long> u;
                bool fit = true;
                for (int q = 0; q < R && fit; q++) {
                    int hd[2];
                    memcpy(hd, &hg[(size_t)q * LVL_GB], sizeof(hd));
                    if (hd[0] || hd[1] > LVL_RT_CAP) fit = false;
                    else u.insert(u.end(), hg.begin() + (size_t)q * LVL_GB + 1,
                                  hg.begin() + (size_t)q * LVL_GB + 1 + hd[1]);
                }
                if (fit) {
                    std::sort(u.begin(), u.end());
                    u.erase(std::unique(u.begin(), u.end()), u.end());
                    fit = !u.empty() && u.size() <= (size_t)LVL_RT_CAP;
                }
                if (fit) {
                    const int nu = (int)u.size(), hf[2] = {0, nu};
                    SRT_HIPCHK(hipMemcpyAsync(rtab, u.data(), u.size() * sizeof(double),
                                              hipMemcpyHostToDevice, st));
                    SRT_HIPCHK(hipMemcpyAsync(dflag, hf, sizeof(hf), hipMemcpyHostToDevice, st));
                    if (nb1 > nb0)
                        lvl_rt_index_kernel<<<srt_ceil_div(nb1 - nb0, 256), 256, 0, st>>>(
                            nb1 - nb0, arA + nb0, reinterpret_cast<const unsigned long long*>(rtab), nu,
                            rix + nb0);
                    SRT_HIPCHK(hipGetLastError());
                    if ((rc_ = lvl_wait(st))) return rc_; /* hf and u leave scope */
                    numbered = 1;
                }
            }
            rc_ = srt_coll_group_begin(comm);
            for (int q = 0; q < R && !rc_; q++)
                if (hoff[q + 1] > hoff[q]) {
                    const size_t c = (size_t)(hoff[q + 1] - hoff[q]);
                    rc_ = srt_coll_bcast(comm, arcsA + hoff[q], c * sizeof(uint32_t), q, st);
                    if (!rc_)
                        rc_ = numbered ? srt_coll_bcast(comm, rix + hoff[q], c * sizeof(uint16_t), q, st)
                                       : srt_coll_bcast(comm, arA + hoff[q], c * sizeof(double), q, st);
                }
            const int rc2 = srt_coll_group_end(comm);
            if (rc_ || rc2) return rc_ ? rc_ : rc2;
            if (solo && lrows > 0) {
                lvl_solo_arcs_kernel<<<srt_ceil_div(n, 4), 256, 0, st>>>(n, row0, nrows, lrows, 1, lw, nw, off,
                                                                         arcsA, numbered ? rix : NULL,
                                                                         numbered ? NULL : arA, NULL);
                SRT_HIPCHK(hipGetLastError());
            }
        }
        /* in-arcs of each target sorted by (weight, source vertex): the order the predecessor
         * search walks them in (the full-row fill's atomics leave the order inside a weight
         * arbitrary; the ordered stash fill needs no sort) */
        arcs = arcsA;
        ar = arA;
        if (total_x > 0 && !sorted_w) {
            lvl_segs_kernel<<<srt_ceil_div(ld + 1, 256), 256, 0, st>>>(ld, off, seg);
            SRT_HIPCHK(hipGetLastError());
            SRT_HIPCHK(hipcub::DeviceSegmentedRadixSort::SortPairs(stmp, sb, arcsA, arcs2, arA, ar2,
                                                                   total_x, ld, seg, seg + 1, 0, 24,
                                                                   st));
            arcs = arcs2;
            ar = ar2;
        }
        if (total_x > 0) {
            lvl_aoff_kernel<<<srt_ceil_div(total_x, 256), 256, 0, st>>>(total_x, nw, arcs, aoff);
            SRT_HIPCHK(hipGetLastError());
        }
        /* the reliability table: its flags are read with the levels' completion (no round trip) */
        if (want_rt && total_x > 0 && !numbered) {
            SRT_HIPCHK(hipMemsetAsync(dflag, 0, 2 * sizeof(int), st));
            SRT_HIPCHK(hipMemsetAsync(H, 0xFF, LVL_RT_SLOTS * sizeof(unsigned long long), st));
            lvl_rt_hash_kernel<<<lvl_rt_grid(total_x), 256, 0, st>>>(NULL, NULL, 0, total_x, ar, H, rix, dflag);
            lvl_rt_compact_kernel<<<1, 1024, 0, st>>>(H, map, rtab, dflag + 1);
            lvl_rt_remap_kernel<<<srt_ceil_div(total_x, 256), 256, 0, st>>>(total_x, map, rix);
            SRT_HIPCHK(hipGetLastError());
        }
        return 0;
    };
    int streamed = 0;       /* the weights the streamed extraction delivers on the side stream */
    int wnum = 0;           /* its arcs carry table indices (else their f64s travel beside) */
    /* N > 1, the first extraction: the arcs of weight <= lw streamed weight by weight on the side
     * stream (the kernels above); level d then waits for ev[d - 1] only. Taken when the fill is the
     * ordered stash (sorted_w) and the reliabilities can be numbered; otherwise extract(). One
     * host round trip: the gathered reliability blocks and the wire offsets come back together. */
    auto extract_streamed = [&](int lw) -> int {
        int64_t t64 = 0;
        for (int x = 1; x <= lw; ++x) t64 += (int64_t)hist[x];
        total_x = (int32_t)t64;
        int rc_;
        /* offsets over the arcs with w <= lw, (target, weight)-major, and the wire's: offw, the
         * [weight][target] scan of every target's counts (gathered), dsz its values at the shard
         * starts; the wire's per-weight bases are on the device since the agreement */
        int32_t* const dsz = packed;
        const int32_t* dwt = packed + LVL_BATCH * 65;
        if ((rc_ = offsets(lw, offw, dsz))) return rc_;
        lvl_arcs_rows_kernel<true><<<nrows, 256, 0, st>>>(n, ld, row0, w_rows, NULL, lw, off, arcsA,
                                                          r_rows, arA, NULL, stash, scnt);
        const int32_t* lo = off + (size_t)row0 * LVL_STRIDE;
        const int32_t* hi = off + (size_t)(row0 + nrows) * LVL_STRIDE;
        /* each own arc's row offset and its index into the union table (on the device since the
         * agreement) */
        lvl_own_index_kernel<<<512, 256, 0, st>>>(lo, hi, nw, arcsA, arA,
                                                  reinterpret_cast<const unsigned long long*>(rtab), (int)u.size(),
                                                  aoff, rix);
        if (lrows > 0)
            lvl_wire_pack_kernel<<<srt_ceil_div(lrows, 4), 256, 0, st>>>(ld, row0, lrows, lw, R, me, off, offw, dsz,
                                                                        dwt, arcsA, rix, arA, wire, NULL);
        SRT_HIPCHK(hipGetLastError());
        SRT_HIPCHK(hipEventRecord(wev[0], st));
        SRT_HIPCHK(hipStreamWaitEvent(wcs, wev[0], 0));
        /* while weight 1 travels: the own sources' arcs into their planes (zeroed since the
         * agreement) */
        if (solo && lrows > 0)
            lvl_solo_direct_kernel<<<srt_ceil_div(n, 4), 256, 0, st>>>(n, row0, nrows, lrows, nw, lw, plane, off,
                                                                       arcsA, lev, Rb);
        else if (!solo && lrows > 0)
            lvl_direct_kernel<<<srt_ceil_div(lrows, 4), 256, 0, st>>>(row0, row0 + lrows, nw, lw, plane, off,
                                                                     arcsA, lev, Rb);
        SRT_HIPCHK(hipGetLastError());
        wnum = 1;
        arcs = arcsA;
        ar = arA;
        streamed = lw;
        return 0;
    };
    /* weight w of the streamed extraction on the side stream: the all-gather of the blocks, their
     * placement (the solo rank synthesises its peers' arcs instead), and, after the last weight of
     * a build whose reliabilities were not numbered, the local table over every arc. Enqueued just
     * before level w, so the host's calls for weight w + 1 overlap the levels on the GPU. */
    auto stream_weight = [&](int w) -> int {
        const size_t base = (size_t)hwt[2 * (w - 1)], mx = (size_t)hwt[2 * (w - 1) + 1];
        int rc_ = srt_coll_allgather(comm, wire + base, mx * sizeof(uint32_t), wcs);
        if (rc_) return rc_;
        SRT_HIPCHK(hipEventRecord(wev[w], wcs));
        return SRT_OK;
    };
    /* Weight w's placement, on the main stream between two levels: the all-gather finished under
     * the previous level, and the whole GPU places the arcs in ~12 us. On the side stream the
     * placement got only the CUs the persistent level grid left free and ended with the level
     * it ran beside (72-135 us per weight on one rank of N = 8), and the last weight's all-gather
     * queued behind it. */
    int wp = 0; /* the streamed weights placed so far */
    auto place_weight = [&](int w) -> int {
        const int32_t* dsz = packed;
        const int32_t* dwt = packed + LVL_BATCH * 65;
        SRT_HIPCHK(hipStreamWaitEvent(st, wev[w], 0));
        if (solo && lrows > 0)
            lvl_solo_arcs_kernel<<<srt_ceil_div(n, 4), 256, 0, st>>>(n, row0, nrows, lrows, w, w, nw, off, arcs,
                                                                     wnum ? rix : NULL, wnum ? NULL : ar, aoff);
        else if (!solo)
            lvl_wire_unpack_kernel<<<srt_ceil_div(n, 4), 256, 0, st>>>(n, ld, row0, nrows, w, nw, R, off, offw,
                                                                       dsz, dwt, wire, NULL, arcs, rix, ar, aoff);
        SRT_HIPCHK(hipGetLastError());
        return SRT_OK;
    };
    if (R == 1) {
        SRT_HIPCHK(hipMemsetAsync(Rb, 0, plane * sizeof(uint32_t), st));
        SRT_HIPCHK(hipMemsetAsync(done, 0, (size_t)n * nchunk, st));
        lvl_init_kernel<<<srt_ceil_div(nrows, 256), 256, 0, st>>>(n, row0, nrows, nw, Rb);
        SRT_HIPCHK(hipGetLastError());
    }
    if (prepped) SRT_HIPCHK(hipStreamWaitEvent(st, wev[prep], 0));
    if ((rc = stream_ok ? extract_streamed(lx) : extract(lx))) return rc;
    unsigned nblk = (unsigned)(((n + 3) / 4) * nchunk);
    nblk = (nblk + 7u) & ~7u;
    /* while the streamed arcs are still arriving, one CU per XCD stays free for the broadcast
     * (RCCL's kernels, the unpack) beside the persistent level grid */
    const unsigned pgrid = lvl_grid((const void*)lvl_step_kernel, nblk, streamed ? 8 : 0);
    /* the levels in batches of LVL_BATCH, one host round trip per batch. After the first batch
     * the settled fraction decides whether the rest is worth it: a graph with far-apart vertices
     * (metric latencies, C4metric: 0.2% settled after 8 levels, distances of hundreds of quanta)
     * goes to the FW at once instead of spending its whole budget first (77 ms there). At N > 1
     * the decision is taken from the summed vote (lvl_vote_kernel): the fraction of all n^2 pairs,
     * the same number on every rank and the one a single GPU would see. A rank whose own sources
     * settled early runs the later levels as no-ops (lvl_step_kernel's prev test) and keeps its D. */
    int D = 0, all_done = 0, hflag[2] = {0, 0};
    unsigned long long* nset = reinterpret_cast<unsigned long long*>(dagree + 4);
    unsigned long long* ngath = nset + 1; /* the level kernels' gathered bytes (dhist word 515) */
    const int ev0 = evp ? evp->used : 0;
    if (evp && (rc = evpool_reserve(evp, ev0 + 2 * lmax))) return rc;
    int wq = 0; /* the streamed weights enqueued so far */
    for (int d0 = 1, d1 = 0; d0 <= lmax; d0 = d1 + 1) {
        /* batches: levels 1-5 (C4's distances end at 4-5), then one level at a time up to
         * LVL_BATCH (a level nobody needs is never launched, nor its weight waited for), then
         * LVL_BATCH at a time */
        d1 = d0 == 1 ? min(lmax, LVL_B1) : d0 <= LVL_BATCH ? d0 : min(lmax, d0 + LVL_BATCH - 1);
        for (int d = d0; d <= d1; ++d) {
            /* weights go out one ahead of the levels (every rank alike: a settled rank still sends
             * its arcs), but not past the batch they are for: a weight nobody's level needs is
             * never sent (C4 ends at level 5) */
            while (wq < min(streamed, min(d + 1, d1)))
                if ((rc = stream_weight(++wq))) return rc;
            if (D && d > D) continue; /* this rank's sources are settled: nothing to run */
            /* Level d reads the arcs of weight < d only: an arc of weight d counts for its own
             * source alone (Delta_0), and lvl_direct_kernel put those into the planes from this
             * rank's rows. So level d waits for weight d - 1, and level 1 for nothing. */
            while (wp < min(d - 1, wq))
                if ((rc = place_weight(++wp))) return rc;
            if (evp) SRT_HIPCHK(hipEventRecord(evp->ev[evp->used++], st));
            if (d == 1) { /* the weight-1 arcs as bits; level 2 takes up the completion flags
                           * (dinc[1] stays set: a graph settled at level 1 reports 2 levels).
                           * Streamed: lvl_direct_kernel has set them. */
                SRT_HIPCHK(hipMemsetAsync(dinc + 1, 0xFF, sizeof(int), st));
                if (!streamed) {
                    SRT_HIPCHK(hipMemsetAsync(lev, 0, plane * sizeof(uint32_t), st));
                    lvl_first_kernel<<<srt_ceil_div(n, 4), 256, 0, st>>>(n, nw, row0, nrows, off, arcs,
                                                                          lev, Rb);
                }
            } else {
                /* levels 2 and 3: the weight-d and weight-(d - 1) groups from the in-arc runs
                 * (lvl_near_kernel); later levels stop after their first group almost
                 * everywhere (the early exit), so they keep the gathers. The runs are read whole
                 * for every target whatever a rank's share of the sources, so they pay only for
                 * a wide share (C4: 14.5 -> 14.1 ms on one GPU; a rank of N = 8, 128 words,
                 * went 2.55 -> 2.86 ms) */
                const bool near = d <= 3 && d <= lx && nw >= LVL_NEAR_MIN_NW && nw <= LVL_NEAR_NW;
                if (near)
                    lvl_near_kernel<<<srt_ceil_div(n, 4), 256, 4 * (size_t)nw * sizeof(uint32_t), st>>>(
                        d, n, nw, row0, nrows, d <= streamed, off, arcs, lev);
                lvl_step_kernel<<<pgrid, 256, 0, st>>>(d, near ? 2 : d <= streamed, n, nw, nchunk, row0, nrows, nblk,
                                                      off, arcs, aoff, lev, Rb, done, dinc + d,
                                                      dinc + d - 1, nset, ngath);
            }
            if (evp) SRT_HIPCHK(hipEventRecord(evp->ev[evp->used++], st));
        }
        SRT_HIPCHK(hipGetLastError());
        /* the batch's weights in place before anything after its levels (the post pass reads
         * every arc up to the last level) */
        while (wp < wq)
            if ((rc = place_weight(++wp))) return rc;
        if (R > 1) {
            lvl_vote_kernel<<<1, 64, 0, st>>>(dinc + d1, nset, dvote);
            SRT_HIPCHK(hipGetLastError());
            if ((rc = srt_coll_allreduce_i32(comm, dvote, 4, 0, st))) return rc;
        }
        /* one read-back: the completion flags, the table flags, the settled pairs and the vote
         * are neighbours in the host-side words (four copies cost ~20 us each of round trip) */
        unsigned long long* const hw = pin + LVL_PIN_HW;
        SRT_HIPCHK(hipMemcpyAsync(hw, dhist + LVL_H_INC, (LVL_H_WORDS - LVL_H_INC) * sizeof(unsigned long long),
                                  hipMemcpyDeviceToHost, st));
        if ((rc = lvl_wait(st))) return rc;
        const int* hinc = reinterpret_cast<const int*>(hw);
        const int32_t* vote = reinterpret_cast<const int32_t*>(hw + (LVL_H_VOTE - LVL_H_INC));
        unsigned long long settled = hw[LVL_H_AGREE + 2 - LVL_H_INC];
        hflag[0] = hinc[LVL_WMAX + 1];
        hflag[1] = hinc[LVL_WMAX + 2];
        int inc[LVL_BATCH];
        for (int d = d0; d <= d1; ++d) inc[d - d0] = hinc[d];
        for (int d = d0; d <= d1 && !D; ++d)
            if (inc[d - d0] == 0) D = d;
        if (R > 1) {
            all_done = vote[0] == 0;
            settled = (unsigned long long)(uint32_t)vote[1] + ((unsigned long long)(uint32_t)vote[2] << 21) +
                      ((unsigned long long)(uint32_t)vote[3] << 42);
        } else {
            all_done = D != 0;
        }
        if (all_done) break;
        /* settled pairs of all sources: the levels >= 2 counted by lvl_step_kernel, every source's
         * own vertex (level 0) and the weight-1 arcs (level 1, lvl_first_kernel counts none) */
        const double frac = ((double)settled + (double)n + (double)hist[1]) / ((double)n * (double)n);
        /* at the end of the first LVL_BATCH levels (a forced level build, fw_ms = 1e30 from
         * SRT_FORM levels=1, runs its whole budget) */
        if (d1 == lx && d1 < lmax && frac < LVL_MIN_SETTLED && fw_ms < 1e29)
            break; /* -> Floyd-Warshall, every rank */
        if (d1 == lx && lx < lmax) { /* the heavier arcs: their counts, then every arc up to lmax */
            while (wq < streamed) /* (the first extraction's last weights, for the collectives) */
                if ((rc = stream_weight(++wq))) return rc;
            while (wp < wq) /* its writes come first */
                if ((rc = place_weight(++wp))) return rc;
            if ((rc = share_counts(lx + 1, lmax)) || (rc = extract(lmax))) return rc;
        }
    }
    /* the side stream's last weight before anything frees the wire (lvl_free waits for it too) */
    if (wq) L->wlast = wev[wq];
    if (evp && D) evp->used = ev0 + 2 * D; /* the levels that did work */
    /* the bytes the level kernels gathered, counted on the device (the early exit skips the
     * later weight groups of a unit, so the model -- every arc of weight < d for every level --
     * would overstate them) */
    const unsigned long long* hw_last = pin + LVL_PIN_HW; /* the last batch's read-back */
    const int64_t gathered = (int64_t)hw_last[LVL_H_AGREE + 3 - LVL_H_INC];
    if (!all_done) return SRT_OK; /* the verdict, alike on every rank (the summed vote) */
    int ntab = 0;
    if (want_rt && !hflag[0] && hflag[1] <= LVL_RT_CAP)
        ntab = hflag[1];
    else
        rix = NULL, rtab = NULL; /* (freed with the state) */
    /* the packed post pass writes the u32 rows itself (rel_pk_kernel): the table of distinct arc
     * reliabilities, 5-bit levels and u16 vertices (n <= 32768) */
    /* 1: lvl_pred_kernel's target-major packed words with the level, one transpose, then
     * rel_pk_kernel, which writes the u32 rows too; 0 (past the packed form, or SRT_FORM pkw=0):
     * lvl_out8 rows + the predecessor rows + rel_tree_kernel */
    const int pkw = rix && D <= 31 && n <= 32768 ? (srt_form_int("pkw", 1) != 0) : 0;
    uint8_t* l8 = NULL;
    if (!pkw) {
        LVL_ALLOC(l8, (size_t)nrows * ld);
        if (D <= LVL_OUT_L) {
            const int lds = D * 2 * 256 * (int)sizeof(uint4);
            SRT_HIPCHK(hipFuncSetAttribute((const void*)lvl_out8_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds));
            lvl_out8_kernel<<<dim3(srt_ceil_div(ld, 256), srt_ceil_div(nw, 8)), 256, lds, st>>>(
                n, ld, nw, row0, D, lev, lat_rows, l8);
        } else {
            lvl_out_kernel<<<dim3(srt_ceil_div(ld, 1024), srt_ceil_div(nw, 16)), 256, 0, st>>>(
                n, ld, nw, row0, D, lev, lat_rows, l8);
        }
        SRT_HIPCHK(hipGetLastError());
    }
    *levels = D;
    *gather_bytes = gathered;
    L->held = 1;
    L->n = n;
    L->nw = nw;
    L->nchunk = nchunk;
    L->row0 = row0;
    L->nrows = nrows;
    L->D = D;
    L->nblk = nblk;
    L->off = off;
    L->arcs = arcs;
    L->aoff = aoff;
    L->ar = ar;
    L->rix = rix;
    L->rtab = rtab;
    L->ntab = ntab;
    L->lev = lev;
    L->l8 = l8;
    L->pkw = pkw;
    L->total = total_x;
    L->dkey = dkey; /* the diagonal keys of this rank's rows */
    L->r_rows = r_rows;
    return SRT_OK;
}

/* the held build's post pass: 1 srt_levels_pred's packed words with levels + a transpose +
 * rel_pk_kernel, 0 the u8 level rows + rel_tree_kernel */
int srt_levels_pkw_ready(void) {
    const lvl_state* L = &g_lvl[srt_state_slot()];
    return L->held ? L->pkw : 0;
}

/* Canonical predecessors and their arc reliabilities of the held level build, target-major
 * (predT[t][sl], rT[t][sl], row stride ldp), as pred_cols*_kernel leave them for the transposes
 * and the reliability passes; ties != NULL adds the tied pairs. pred16: predT holds int16 (n <=
 * 32768: half the bytes of the predecessor slab and its transpose), else int32. */
int srt_levels_pred(void* predT, int pred16, double* rT, size_t ldp, unsigned long long* ties,
                    hipStream_t st) {
    /* pred16 == 2: the packed form (srt_levels_rtab) */
    lvl_state* L = &g_lvl[srt_state_slot()];
    if (!L->held) {
        srt_set_error("levels: no held level build for the predecessor pass");
        return SRT_E_ARG;
    }
    unsigned long long* part = NULL;
    if (ties) {
        SRT_HIPCHK(srt_malloc_async(&part, 1024 * sizeof(unsigned long long), st));
        SRT_HIPCHK(hipMemsetAsync(part, 0, 1024 * sizeof(unsigned long long), st));
    }
    if (pred16 && L->n > 32768) {
        srt_set_error("levels: int16 predecessors need n <= 32768 (n = %d)", L->n);
        return SRT_E_ARG;
    }
    if (pred16 == 2 && !L->rix) {
        srt_set_error("levels: the packed form needs the reliability table");
        return SRT_E_ARG;
    }
    if (pred16 == 2)
        lvl_pred_kernel<uint32_t><<<lvl_grid((const void*)lvl_pred_kernel<uint32_t>, L->nblk), 256, 0, st>>>(
            L->n, L->nw, L->nchunk, L->row0, L->nrows, L->D, L->nblk, L->off, L->arcs, L->aoff, L->ar,
            L->rix, L->lev, (uint32_t*)predT, rT, ldp, part);
    else if (pred16)
        lvl_pred_kernel<int16_t><<<lvl_grid((const void*)lvl_pred_kernel<int16_t>, L->nblk), 256, 0, st>>>(
            L->n, L->nw, L->nchunk, L->row0, L->nrows, L->D, L->nblk, L->off, L->arcs, L->aoff, L->ar,
            L->rix, L->lev, (int16_t*)predT, rT, ldp, part);
    else
        lvl_pred_kernel<int32_t><<<lvl_grid((const void*)lvl_pred_kernel<int32_t>, L->nblk), 256, 0, st>>>(
            L->n, L->nw, L->nchunk, L->row0, L->nrows, L->D, L->nblk, L->off, L->arcs, L->aoff, L->ar,
            L->rix, L->lev, (int32_t*)predT, rT, ldp, part);
    SRT_HIPCHK(hipGetLastError());
    if (ties) {
        lvl_sum_kernel<<<1, 1024, 0, st>>>(part, 1024, ties);
        SRT_HIPCHK(hipGetLastError());
        SRT_HIPCHK(hipFreeAsync(part, st));
    }
    return SRT_OK;
}
