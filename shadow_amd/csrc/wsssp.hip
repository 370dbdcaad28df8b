/*
 * wsssp.hip -- wave-per-source exact bucket SSSP (Dial's algorithm) for sparse graphs, gfx950.
 *
 * Replaces, for the eager all-pairs build, the per-source igraph Dijkstra of
 * /root/reference/src/main/routing/topology.c:1578-1814 and the per-hop path walk of :1286-1389.
 *
 * One wavefront owns one source at a time (persistent grid, 64-thread workgroups, no
 * workgroup-wide barriers). Distances are integer quanta >= 1 per arc, so a circular array of C
 * buckets (C = power of two > max arc weight) holds every pending vertex: the bucket of value d
 * only ever holds entries pushed for exactly d, each vertex at most once (a push happens only on a
 * strict decrease). Buckets are popped in increasing d, so every vertex is settled exactly once,
 * in nondecreasing distance order -- which is what lets the predecessor and the path-order
 * reliability be formed at settle time:
 *   pred(s,t) = argmin (D[s][u], u) over tight in-arcs (the canonical tie rule);
 *   every tight u has D[s][u] <= D[s][t] - 1, so it is already settled with its final rel;
 *   rel(s,t) = rel(s,pred) * r(pred,t) -- the left-to-right product of topology.c:1364-1365.
 * For undirected graphs the out-arcs scanned to relax t's neighbours are also t's in-arcs, so one
 * pass over them does both; directed graphs scan the in-arc CSR separately.
 *
 * Memory: the distance row is the output lat row (u32 quanta, L2-coherent loads and atomics),
 * the rel row is the output rel row; buckets live in a per-wave global slot (C x bcap vertex ids);
 * bucket counts and the non-empty mask live in LDS. A bucket overflow flags the source and the
 * caller recomputes it with the workgroup-per-source kernel (sparse.hip) -- never approximate.
 *
 * Arc work inside one step is balanced across lanes merge-path style: the settled vertices of a
 * 64-entry chunk are laid end to end by an exclusive scan of their degrees, and each lane finds
 * the vertex owning its arc position with one LDS write + a wave max-scan.
 */
#include "srt_device.h"

#define WL 64

static __device__ __forceinline__ uint32_t ld_coherent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
static __device__ __forceinline__ double ld_coherent(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static __device__ __forceinline__ int wave_scan_excl(int v, int lane, int* total) {
    int x = v;
#pragma unroll
    for (int off = 1; off < WL; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    *total = __shfl(x, WL - 1);
    return x - v;
}

static __device__ __forceinline__ int wave_scan_max(int v, int lane) {
#pragma unroll
    for (int off = 1; off < WL; off <<= 1) {
        const int y = __shfl_up(v, off);
        if (lane >= off) v = max(v, y);
    }
    return v;
}

template <bool DIRECTED>
__global__ __launch_bounds__(WL) void wsssp_kernel(
    int n, int src_begin, int nsrc, const int32_t* __restrict__ rowptr,
    const uint2* __restrict__ cw, const double* __restrict__ r,
    const int32_t* __restrict__ in_rowptr, const uint2* __restrict__ in_cw,
    const double* __restrict__ in_r, uint32_t* __restrict__ lat, double* __restrict__ rel,
    size_t ldo, uint32_t* __restrict__ ws, int nb, int bcap, int* __restrict__ overflow) {
    __shared__ uint32_t bcnt[256];
    __shared__ unsigned long long bmask[4];
    __shared__ int s_beg[WL], s_excl[WL], s_own[WL];
    __shared__ unsigned long long s_best[WL];
    __shared__ int s_ovf;
    const int lane = threadIdx.x;
    uint32_t* buckets = ws + (size_t)blockIdx.x * nb * bcap;
    const uint32_t bmaskm = (uint32_t)nb - 1u;

    for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int s = src_begin + si;
        uint32_t* dist = lat + (size_t)si * ldo;
        double* rr = rel + (size_t)si * ldo;
        for (int v = lane; v < n; v += WL) {
            dist[v] = (v == s) ? 0u : SRT_INF;
            rr[v] = 0.0;
        }
        for (int b = lane; b < nb; b += WL) bcnt[b] = 0;
        if (lane < 4) bmask[lane] = 0ull;
        if (lane == 0) {
            s_ovf = 0;
            buckets[0] = (uint32_t)s;
            bcnt[0] = 1;
            bmask[0] = 1ull;
        }
        __threadfence_block();
        __syncthreads();
        uint32_t d = 0; /* value of the bucket being processed */
        for (;;) {
            /* next non-empty bucket at or after position d (circular); all pending values lie
             * in [d, d + max_w] and C > max_w, so the offset is the value step */
            const uint32_t p0 = d & bmaskm;
            int found = -1;
            for (int q = 0; q < nb && found < 0; q += 64) {
                /* bits of positions p0+q .. p0+q+63 (mod nb), assembled from the mask words */
                const int pos = (int)((p0 + (uint32_t)q + (uint32_t)lane) & bmaskm);
                const bool set = (bmask[pos >> 6] >> (pos & 63)) & 1ull;
                const unsigned long long bal = __ballot(set && q + lane < nb);
                if (bal) found = q + __ffsll((long long)bal) - 1;
            }
            if (found < 0) break;
            d += (uint32_t)found;
            const int b = (int)(d & bmaskm);
            const int cnt = min((int)bcnt[b], bcap);
            __syncthreads();
            if (lane == 0) {
                bcnt[b] = 0;
                bmask[b >> 6] &= ~(1ull << (b & 63));
            }
            __syncthreads();
            const uint32_t* bk = buckets + (size_t)b * bcap;
            for (int c0 = 0; c0 < cnt; c0 += WL) {
                const int i = c0 + lane;
                int v = -1, beg = 0, deg = 0;
                if (i < cnt) {
                    v = (int)ld_coherent(bk + i);
                    if (ld_coherent(dist + v) == d) {
                        beg = rowptr[v];
                        deg = rowptr[v + 1] - beg;
                    } else {
                        v = -1; /* stale: improved after it was pushed */
                    }
                }
                int total;
                const int excl = wave_scan_excl(deg, lane, &total);
                s_beg[lane] = beg;
                s_excl[lane] = excl;
                s_best[lane] = ~0ull;
                __syncthreads();
                for (int a0 = 0; a0 < total; a0 += WL) {
                    /* owner of arc position a0 + lane: heads scattered, then a max-scan */
                    s_own[lane] = -1;
                    __syncthreads();
                    if (deg > 0 && excl >= a0 && excl < a0 + WL) s_own[excl - a0] = lane;
                    const unsigned long long cover = __ballot(deg > 0 && excl <= a0);
                    __syncthreads();
                    int own = s_own[lane];
                    if (lane == 0 && own < 0 && cover) own = 63 - __clzll((long long)cover);
                    own = wave_scan_max(own, lane);
                    const int a = a0 + lane;
                    if (a < total && own >= 0) {
                        const int k = s_beg[own] + (a - s_excl[own]);
                        const uint2 e = cw[k];
                        const uint32_t u = e.x, wk = e.y;
                        const uint32_t du = ld_coherent(dist + u);
                        const uint32_t nd = d + wk;
                        if (nd < du) {
                            const uint32_t old = atomicMin(dist + u, nd);
                            if (nd < old) {
                                const int b2 = (int)(nd & bmaskm);
                                const int slot = (int)atomicAdd(&bcnt[b2], 1u);
                                if (slot < bcap) {
                                    buckets[(size_t)b2 * bcap + slot] = u;
                                    atomicOr(&bmask[b2 >> 6], 1ull << (b2 & 63));
                                } else {
                                    s_ovf = 1;
                                }
                            }
                        }
                        if (!DIRECTED && du + wk == d)
                            atomicMin(&s_best[own], ((unsigned long long)du << 32) | (uint32_t)k);
                    }
                    __syncthreads();
                }
                if (DIRECTED) {
                    /* tight in-arcs (u -> v): the same merge-path walk over the in-CSR */
                    int ibeg = 0, ideg = 0;
                    if (v >= 0) {
                        ibeg = in_rowptr[v];
                        ideg = in_rowptr[v + 1] - ibeg;
                    }
                    int itotal;
                    const int iexcl = wave_scan_excl(ideg, lane, &itotal);
                    __syncthreads();
                    s_beg[lane] = ibeg;
                    s_excl[lane] = iexcl;
                    __syncthreads();
                    for (int a0 = 0; a0 < itotal; a0 += WL) {
                        s_own[lane] = -1;
                        __syncthreads();
                        if (ideg > 0 && iexcl >= a0 && iexcl < a0 + WL) s_own[iexcl - a0] = lane;
                        const unsigned long long cover = __ballot(ideg > 0 && iexcl <= a0);
                        __syncthreads();
                        int own = s_own[lane];
                        if (lane == 0 && own < 0 && cover) own = 63 - __clzll((long long)cover);
                        own = wave_scan_max(own, lane);
                        const int a = a0 + lane;
                        if (a < itotal && own >= 0) {
                            const int k = s_beg[own] + (a - s_excl[own]);
                            const uint2 e = in_cw[k];
                            const uint32_t du = ld_coherent(dist + e.x);
                            if (du < SRT_INF && du + e.y == d)
                                atomicMin(&s_best[own], ((unsigned long long)du << 32) | (uint32_t)k);
                        }
                        __syncthreads();
                    }
                }
                __syncthreads();
                /* settle: path-order reliability from the canonical predecessor */
                if (v >= 0) {
                    double x = 1.0;
                    if (v != s) {
                        /* a settled vertex always has the tight arc it was pushed over; the
                         * guard only keeps a broken invariant from reading out of bounds */
                        const unsigned long long key = s_best[lane];
                        x = 0.0;
                        if (key != ~0ull) {
                            const int k = (int)(uint32_t)key;
                            const uint32_t u = DIRECTED ? in_cw[k].x : cw[k].x;
                            x = ld_coherent(rr + u) * (DIRECTED ? in_r[k] : r[k]);
                        }
                    }
                    rr[v] = x;
                }
                __threadfence_block(); /* settled rel visible to the later steps of this wave */
                __syncthreads();
            }
            if (s_ovf) break;
        }
        if (s_ovf && lane == 0) overflow[si] = 1;
        __syncthreads();
    }
}

int srt_sparse_diag(int n, int src_begin, int src_end, const int32_t* rowptr, const int32_t* col,
                    const uint32_t* w, const double* r, const uint32_t* self_w,
                    const double* self_r, uint32_t* lat, double* rel, size_t ldo, hipStream_t st);

/* Rows [src_begin, src_end) by the wave-per-source kernel. *overflowed receives the number of
 * sources whose buckets overflowed; their indices (relative to src_begin) are flagged in ovf
 * (device, nsrc ints, zeroed here) for the caller to recompute. */
int srt_wsssp_rows(int n, int directed, const int32_t* rowptr, const uint2* cw, const double* r,
                   const int32_t* in_rowptr, const uint2* in_cw, const double* in_r,
                   uint32_t max_w, int src_begin, int src_end, uint32_t* lat, double* rel,
                   int* ovf, hipStream_t st) {
    int nb = 1;
    while ((uint32_t)nb <= max_w) nb <<= 1;
    if (nb > 256) {
        srt_set_error("wsssp: max arc weight %u quanta needs more than 256 buckets", max_w);
        return SRT_E_ARG;
    }
    const int nsrc = src_end - src_begin;
    int bcap = n < 8192 ? n : 8192;
    const char* env = getenv("SRT_WSSSP_BCAP"); /* tests: force bucket overflows */
    if (env && atoi(env) > 0) bcap = atoi(env);
    int cus = 256;
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        cus = prop.multiProcessorCount;
    /* 16 waves per CU, bounded by an 8 GiB bucket workspace */
    const size_t per_slot = (size_t)nb * bcap * sizeof(uint32_t);
    size_t slots = (size_t)16 * cus;
    const size_t budget = (size_t)8 << 30;
    if (slots * per_slot > budget) slots = budget / per_slot;
    if (slots > (size_t)nsrc) slots = nsrc;
    if (slots < 1) slots = 1;
    uint32_t* ws = NULL;
    if (hipMallocAsync((void**)&ws, slots * per_slot, st) != hipSuccess) {
        (void)hipGetLastError();
        srt_set_error("wsssp: bucket workspace of %zu MiB failed", (slots * per_slot) >> 20);
        return SRT_E_NOMEM;
    }
    SRT_HIPCHK(hipMemsetAsync(ovf, 0, (size_t)nsrc * sizeof(int), st));
    if (directed)
        wsssp_kernel<true><<<(unsigned)slots, WL, 0, st>>>(n, src_begin, nsrc, rowptr, cw, r, in_rowptr,
                                                           in_cw, in_r, lat, rel, (size_t)n, ws, nb,
                                                           bcap, ovf);
    else
        wsssp_kernel<false><<<(unsigned)slots, WL, 0, st>>>(n, src_begin, nsrc, rowptr, cw, r, in_rowptr,
                                                            in_cw, in_r, lat, rel, (size_t)n, ws, nb,
                                                            bcap, ovf);
    SRT_HIPCHK(hipGetLastError());
    SRT_HIPCHK(hipFreeAsync(ws, st));
    return SRT_OK;
}
