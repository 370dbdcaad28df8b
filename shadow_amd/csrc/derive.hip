/*
 * derive.hip -- neighbour-row derivation of sparse all-pairs rows, gfx950.
 *
 * The rows of _topology_computeSourcePaths (/root/reference/src/main/routing/topology.c:1578-1814:
 * one Dijkstra per source, the path-order reliability product of :1364-1365) for the sources of an
 * independent set I of low-degree vertices, from the rows of their neighbours ("core" rows, built
 * by the workgroup SSSP kernel with their canonical arcs, wsssp.hip `codes`). On a BA graph with
 * m = 3 every degree-3 vertex is in I (preferential attachment never links two of them): C5 builds
 * 54k rows by SSSP and derives the other 46k.
 *
 * For s in I and t != s every path leaves s through a neighbour k, all outside I:
 *   D[s][t] = min_k w(s,k) + D[k][t]                              (exact: weights >= 1 quantum)
 * The canonical predecessor (every kernel's rule: argmin (D[s][u], u) over the tight in-arcs
 * u -> t, i.e. the largest w, then the smallest u) is the best, by that row-independent key, of the
 * canonical arcs into t of the optimal neighbours (those with w(s,k) + D[k][t] = D[s][t]), and of
 * the direct arc when t is a neighbour: an arc is tight for s exactly when it is tight for some
 * optimal k (tools/c5_derive_model.py checks both claims against the oracle). The reliability is
 * then the path-order product from s, re-formed here in sweeps over the derived predecessors (a
 * target resolves once its predecessor has) -- never taken from k's row, whose product associates
 * from k.
 */
#include "srt_device.h"

#define DV_THREADS 1024
#define DV_MAXDEG 8 /* largest degree the host puts in I */
#define DV_J 4      /* targets per thread per phase-A step: their loads overlap */

static __device__ __forceinline__ double dv_ld(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
static __device__ __forceinline__ void dv_st(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
/* order of canonical arcs u | w << 17 | ridx << 24: the largest w, then the smallest u */
static __device__ __forceinline__ uint32_t dv_key(uint32_t code) {
    return ((127u - ((code >> 17) & 0x7Fu)) << 17) | (code & 0x1FFFFu);
}

/* One workgroup per derived source (persistent grid over I). Rows are placed by source: row of
 * vertex v = v - src_begin, in lat / rel (stride ldo); core vertex k's codes are row crow[k] of
 * codes (stride n). scratch: n words per workgroup (its row of derived codes). */
__global__ __launch_bounds__(DV_THREADS) void derive_rows_kernel(
    int n, int nI, const int32_t* __restrict__ I, int src_begin, const int2* __restrict__ rowptr,
    const uint2* __restrict__ cw, const uint8_t* __restrict__ ridx, const double* __restrict__ rtab,
    int ntab, const int32_t* __restrict__ crow, const uint32_t* __restrict__ codes,
    uint32_t* __restrict__ lat, double* __restrict__ rel, size_t ldo, uint32_t* __restrict__ scratch,
    int32_t* __restrict__ max_depth) {
    extern __shared__ uint32_t dbm[]; /* done[nw], fresh[nw] */
    __shared__ double s_tab[256];
    __shared__ int s_nb[DV_MAXDEG], s_w[DV_MAXDEG], s_rx[DV_MAXDEG], s_cr[DV_MAXDEG];
    __shared__ int s_any;
    const int tid = threadIdx.x, nw = (n + 31) >> 5;
    uint32_t* done = dbm;
    uint32_t* fresh = dbm + nw;
    for (int i = tid; i < ntab; i += DV_THREADS) s_tab[i] = rtab[i];
    uint32_t* cs = scratch + (size_t)blockIdx.x * (size_t)((n + 3) & ~3); /* 16-B aligned rows */
    int depth_max = 0;
    for (int si = blockIdx.x; si < nI; si += gridDim.x) {
        const int s = I[si];
        uint32_t* ol = lat + (size_t)(s - src_begin) * ldo;
        double* orr = rel + (size_t)(s - src_begin) * ldo;
        const int2 be = rowptr[s];
        const int deg = min(be.y - be.x, DV_MAXDEG);
        __syncthreads(); /* the previous source is done with s_nb and the bitmaps */
        if (tid < deg) {
            const uint2 e = cw[be.x + tid];
            s_nb[tid] = (int)e.x;
            s_w[tid] = (int)e.y;
            s_rx[tid] = ridx[be.x + tid];
            s_cr[tid] = crow[e.x];
        }
        for (int q = tid; q < 2 * nw; q += DV_THREADS) dbm[q] = 0u;
        __syncthreads();
        /* phase A: distances and derived codes, DV_J targets per thread at a time (the deg row
         * loads of all of them in flight together, then the codes of the tight neighbours) */
        for (int t0 = 0; t0 < n; t0 += DV_J * DV_THREADS) {
            uint32_t dk[DV_J][DV_MAXDEG];
#pragma unroll
            for (int j = 0; j < DV_J; ++j) {
                const int t = t0 + j * DV_THREADS + tid;
#pragma unroll
                for (int i = 0; i < DV_MAXDEG; ++i)
                    dk[j][i] = (i < deg && t < n)
                                   ? lat[(size_t)(s_nb[i] - src_begin) * ldo + t]
                                   : SRT_INF;
            }
            uint32_t D[DV_J];
#pragma unroll
            for (int j = 0; j < DV_J; ++j) {
                D[j] = SRT_INF;
#pragma unroll
                for (int i = 0; i < DV_MAXDEG; ++i)
                    if (dk[j][i] < SRT_INF) D[j] = min(D[j], (uint32_t)s_w[i] + dk[j][i]);
            }
            uint32_t cd[DV_J][DV_MAXDEG];
#pragma unroll
            for (int j = 0; j < DV_J; ++j) {
                const int t = t0 + j * DV_THREADS + tid;
#pragma unroll
                for (int i = 0; i < DV_MAXDEG; ++i) {
                    cd[j][i] = ~0u;
                    if (dk[j][i] < SRT_INF && (uint32_t)s_w[i] + dk[j][i] == D[j])
                        cd[j][i] = t == s_nb[i]
                                       ? ((uint32_t)s | ((uint32_t)s_w[i] << 17) |
                                          ((uint32_t)s_rx[i] << 24))
                                       : codes[(size_t)s_cr[i] * n + t];
                }
            }
#pragma unroll
            for (int j = 0; j < DV_J; ++j) {
                const int t = t0 + j * DV_THREADS + tid;
                if (t >= n) continue;
                uint32_t best = ~0u, bk = ~0u;
#pragma unroll
                for (int i = 0; i < DV_MAXDEG; ++i)
                    if (cd[j][i] != ~0u && dv_key(cd[j][i]) < bk) {
                        bk = dv_key(cd[j][i]);
                        best = cd[j][i];
                    }
                if (t == s) {
                    D[j] = 0;
                    best = ~0u;
                }
                ol[t] = D[j];
                cs[t] = best;
                if (t == s || D[j] >= SRT_INF) { /* resolved: the source, or unreachable */
                    atomicOr(&done[t >> 5], 1u << (t & 31));
                    dv_st(orr + t, t == s ? 1.0 : 0.0);
                }
            }
        }
        __threadfence_block();
        __syncthreads();
        /* phase B: rel(s,t) = rel(s,u) * r(u,t) once u has resolved (path order from s), in
         * sweeps; a thread owns whole bitmap words and reads its 32 targets' codes at once */
        int depth = 0;
        for (;;) {
            if (tid == 0) s_any = 0;
            __syncthreads();
            int any = 0;
            for (int w = tid; w < nw; w += DV_THREADS) {
                uint32_t pend = ~done[w];
                if (w == nw - 1 && (n & 31)) pend &= (1u << (n & 31)) - 1u;
                if (!pend) continue;
                uint32_t c[32];
                const uint4* cp = reinterpret_cast<const uint4*>(cs + (size_t)w * 32);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint4 x = (w * 32 + q * 4 + 3 < n) ? cp[q]
                                    : make_uint4(~0u, ~0u, ~0u, ~0u);
                    c[4 * q] = x.x;
                    c[4 * q + 1] = x.y;
                    c[4 * q + 2] = x.z;
                    c[4 * q + 3] = x.w;
                }
                if (w * 32 + 32 > n) /* the ragged last word: no 16-byte tail reads */
                    for (int b = 0; b < 32; ++b) c[b] = w * 32 + b < n ? cs[w * 32 + b] : ~0u;
                uint32_t ready = 0u;
#pragma unroll
                for (int b = 0; b < 32; ++b) {
                    const uint32_t u = c[b] & 0x1FFFFu;
                    if (((pend >> b) & 1u) && c[b] != ~0u && ((done[u >> 5] >> (u & 31)) & 1u))
                        ready |= 1u << b;
                }
                if (!ready) continue;
#pragma unroll
                for (int b0 = 0; b0 < 32; b0 += 8) { /* eight predecessor loads in flight */
                    if (!((ready >> b0) & 0xFFu)) continue;
                    double ru[8];
#pragma unroll
                    for (int b = 0; b < 8; ++b)
                        ru[b] = ((ready >> (b0 + b)) & 1u) ? dv_ld(orr + (c[b0 + b] & 0x1FFFFu))
                                                           : 0.0;
#pragma unroll
                    for (int b = 0; b < 8; ++b)
                        if ((ready >> (b0 + b)) & 1u)
                            dv_st(orr + w * 32 + b0 + b, ru[b] * s_tab[c[b0 + b] >> 24]);
                }
                fresh[w] = ready; /* word w belongs to this thread alone */
                any = 1;
            }
            if (any) s_any = 1;
            __threadfence_block();
            __syncthreads();
            if (!s_any) break;
            ++depth;
            for (int w = tid; w < nw; w += DV_THREADS) {
                done[w] |= fresh[w];
                fresh[w] = 0u;
            }
            __syncthreads();
        }
        depth_max = depth > depth_max ? depth : depth_max;
    }
    if (max_depth && tid == 0) atomicMax(max_depth, depth_max);
}

/* The rows of the nI sources I (device list) by derivation, into lat / rel rows placed by source
 * (row v - src_begin, stride ldo), from the core rows already there and their codes (row crow[k]
 * of codes, stride n). rowptr / cw / ridx: the original-order CSR with each arc's index into
 * rtab (ntab <= 256 distinct reliabilities). Every source of I has degree <= DV_MAXDEG and every
 * neighbour is a core vertex (the caller's independent set). */
int srt_derive_rows(int n, int nI, const int32_t* I, int src_begin, const int2* rowptr,
                    const uint2* cw, const uint8_t* ridx, const double* rtab, int ntab,
                    const int32_t* crow, const uint32_t* codes, uint32_t* lat, double* rel,
                    size_t ldo, hipStream_t st) {
    if (nI <= 0) return SRT_OK;
    if (ntab > 256 || n > srt_path_sweeps_max_n()) {
        srt_set_error("derive: %d reliabilities or n = %d outside the kernel's range", ntab, n);
        return SRT_E_ARG;
    }
    int cus = 256, dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        cus = prop.multiProcessorCount;
    const int grid = nI < 2 * cus ? nI : 2 * cus;
    uint32_t* scratch = NULL;
    SRT_HIPCHK(srt_malloc_async(&scratch, (size_t)grid * ((n + 3) & ~3) * sizeof(uint32_t), st));
    const size_t lds = 2 * (size_t)((n + 31) / 32) * sizeof(uint32_t);
    SRT_HIPCHK(hipFuncSetAttribute((const void*)derive_rows_kernel,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    derive_rows_kernel<<<grid, DV_THREADS, lds, st>>>(n, nI, I, src_begin, rowptr, cw, ridx, rtab,
                                                      ntab, crow, codes, lat, rel, ldo, scratch,
                                                      NULL);
    SRT_HIPCHK(hipGetLastError());
    SRT_HIPCHK(hipFreeAsync(scratch, st));
    return SRT_OK;
}
