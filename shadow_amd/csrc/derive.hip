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

#define DV_MAXDEG SRT_DERIVE_MAXDEG /* largest degree the host puts in I (build.hip) */
#define DV_J 2  /* targets per thread per phase-A step: their loads overlap */
#define DV_JB 1 /* targets per thread per phase-B step (4: 138 vs 125 ms on C5) */
/* (round-5 A/B forms -- phase A without the speculative code loads, per-phase wall-clock
 * profiles, the phase-A-only probe -- were measured and left the library: DESIGN §5.9) */

/* order of canonical arcs u | w << 17 | ridx << 24: the largest w, then the smallest u */
static __device__ __forceinline__ uint32_t dv_key(uint32_t code) {
    return ((127u - ((code >> 17) & 0x7Fu)) << 17) | (code & 0x1FFFFu);
}

/* One workgroup per derived source (persistent grid over I, one per CU). Rows are placed
 * by source: row of vertex v = v - src_begin, in lat / rel (stride ldo); core vertex k's codes are
 * row crow[k] of codes (stride n); cs: n codes of scratch per workgroup. Phase A forms the
 * distances and the derived codes; phase B the reliability on demand: a thread takes
 * its targets in index order (coalesced code reads and rel writes) and forms rel(s,t) once its
 * predecessor's is done; if not, it climbs the predecessor chain to the first vertex whose
 * predecessor is done, forms that one, and repeats. A done bit (LDS) is set after the value is
 * stored (workgroup release/acquire), so a value is read only once final; two threads that form
 * the same vertex store the same product. The ancestors near s are shared by most chains and
 * stay in cache; no list, no per-level barrier (a distance-ordered form -- a per-row list by
 * distance, one barrier per level -- measured 250 vs 125 ms on C5: ~200 levels per row). */
template <int NT, int CACHE>
__global__ __launch_bounds__(NT) void derive_chain_kernel(
    int n, int nI, const int32_t* __restrict__ I, int src_begin, const int2* __restrict__ rowptr,
    const uint2* __restrict__ cw, const uint8_t* __restrict__ ridx, const double* __restrict__ rtab,
    int ntab, const int32_t* __restrict__ crow, const uint32_t* __restrict__ codes,
    uint32_t* __restrict__ lat, double* __restrict__ rel, size_t ldo, uint32_t* __restrict__ cs_all,
    size_t lds_n, unsigned* __restrict__ queue) {
    /* dynamic LDS: one done bit per target, then (CACHE) the reliability of vertices < CACHE --
     * the oldest vertices of a BA graph are its hubs, the parents of most targets */
    extern __shared__ __attribute__((aligned(16))) uint32_t cdone[];
    double* cache = reinterpret_cast<double*>(cdone + (((n + 31) / 32 + 3) & ~3));
    __shared__ double s_tab[256];
    __shared__ int s_nb[DV_MAXDEG], s_w[DV_MAXDEG], s_rx[DV_MAXDEG], s_cr[DV_MAXDEG];
    const int tid = threadIdx.x, nw = (n + 31) >> 5;
    for (int i = tid; i < ntab; i += NT) s_tab[i] = rtab[i];
    uint32_t* cs = cs_all + (size_t)blockIdx.x * lds_n;
    auto rel_of = [&](uint32_t u, const double* orr) -> double {
        if (CACHE && u < (uint32_t)CACHE) return cache[u];
        return __hip_atomic_load(orr + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto put = [&](uint32_t y, double v, double* orr) {
        __hip_atomic_store(orr + y, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (CACHE && y < (uint32_t)CACHE) cache[y] = v;
    };
    auto is_done = [&](uint32_t v) {
        return (__hip_atomic_load(&cdone[v >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >>
                (v & 31)) & 1u;
    };
    __shared__ int s_next; /* rows from a work queue (a late workgroup does not hold the end back) */
    for (;;) {
        if (tid == 0) s_next = (int)atomicAdd(queue, 1u);
        __syncthreads();
        const int si = s_next;
        if (si >= nI) break;
        const int s = I[si];
        uint32_t* ol = lat + (size_t)(s - src_begin) * ldo;
        double* orr = rel + (size_t)(s - src_begin) * ldo;
        const int2 be = rowptr[s];
        const int deg = min(be.y - be.x, DV_MAXDEG);
        __syncthreads(); /* the previous source is done with the shared state */
        if (tid < deg) {
            const uint2 e = cw[be.x + tid];
            s_nb[tid] = (int)e.x;
            s_w[tid] = (int)e.y;
            s_rx[tid] = ridx[be.x + tid];
            s_cr[tid] = crow[e.x];
        }
        for (int q = tid; q < nw; q += NT) cdone[q] = 0u;
        __threadfence_block();
        __syncthreads();
        /* phase A (as derive_rows_kernel): distances, derived codes; s and the unreachable
         * targets are done at once */
        for (int t0 = 0; t0 < n; t0 += DV_J * NT) {
            uint32_t dk[DV_J][DV_MAXDEG];
#pragma unroll
            for (int j = 0; j < DV_J; ++j) {
                const int t = t0 + j * NT + tid;
#pragma unroll
                for (int i = 0; i < DV_MAXDEG; ++i)
                    dk[j][i] = (i < deg && t < n)
                                   ? lat[(size_t)(s_nb[i] - src_begin) * ldo + t]
                                   : SRT_INF;
            }
            /* every neighbour's code with its distance: no second round trip */
            uint32_t cv[DV_J][DV_MAXDEG];
#pragma unroll
            for (int j = 0; j < DV_J; ++j) {
                const int t = t0 + j * NT + tid;
#pragma unroll
                for (int i = 0; i < DV_MAXDEG; ++i)
                    cv[j][i] = (i < deg && t < n) ? codes[(size_t)s_cr[i] * n + t] : ~0u;
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
                const int t = t0 + j * NT + tid;
#pragma unroll
                for (int i = 0; i < DV_MAXDEG; ++i) {
                    cd[j][i] = ~0u;
                    if (dk[j][i] < SRT_INF && (uint32_t)s_w[i] + dk[j][i] == D[j])
                        cd[j][i] = t == s_nb[i]
                                       ? ((uint32_t)s | ((uint32_t)s_w[i] << 17) |
                                          ((uint32_t)s_rx[i] << 24))
                                       : cv[j][i];
                }
            }
#pragma unroll
            for (int j = 0; j < DV_J; ++j) {
                const int t = t0 + j * NT + tid;
                if (t >= n) continue;
                uint32_t best = ~0u, bk = ~0u;
#pragma unroll
                for (int i = 0; i < DV_MAXDEG; ++i)
                    if (cd[j][i] != ~0u && dv_key(cd[j][i]) < bk) {
                        bk = dv_key(cd[j][i]);
                        best = cd[j][i];
                    }
                if (t == s) D[j] = 0;
                ol[t] = D[j];
                cs[t] = best;
                if (t == s || D[j] >= SRT_INF) {
                    put((uint32_t)t, t == s ? 1.0 : 0.0, orr);
                    __hip_atomic_fetch_or(&cdone[t >> 5], 1u << (t & 31), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        }
        __threadfence_block();
        __syncthreads();
        /* target t (its code ct) once its predecessor is not formed: climb to the first ancestor
         * whose predecessor is, form it, and repeat until t is formed */
        auto climb = [&](int t, uint32_t ct) {
            for (;;) {
                uint32_t y = (uint32_t)t, cy = ct;
                while (!is_done(cy & 0x1FFFFu)) {
                    y = cy & 0x1FFFFu;
                    cy = cs[y];
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const double rp = rel_of(cy & 0x1FFFFu, orr);
                put(y, rp * s_tab[cy >> 24], orr);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __hip_atomic_fetch_or(&cdone[y >> 5], 1u << (y & 31), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                if (y == (uint32_t)t) break;
            }
        };
        /* phase B: on-demand path-order products. DV_JB targets per thread per step: their
         * codes, then the predecessors' values of the ready ones, in flight together; a target
         * whose predecessor is not formed yet climbs alone */
        for (int t0 = 0; t0 < n; t0 += DV_JB * NT) {
            uint32_t cj[DV_JB];
            bool rdy[DV_JB];
#pragma unroll
            for (int j = 0; j < DV_JB; ++j) {
                const int t = t0 + j * NT + tid;
                cj[j] = (t < n && !is_done((uint32_t)t)) ? cs[t] : ~0u;
            }
#pragma unroll
            for (int j = 0; j < DV_JB; ++j) rdy[j] = cj[j] != ~0u && is_done(cj[j] & 0x1FFFFu);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            double rp[DV_JB];
#pragma unroll
            for (int j = 0; j < DV_JB; ++j) rp[j] = rdy[j] ? rel_of(cj[j] & 0x1FFFFu, orr) : 0.0;
#pragma unroll
            for (int j = 0; j < DV_JB; ++j)
                if (rdy[j]) put((uint32_t)(t0 + j * NT + tid), rp[j] * s_tab[cj[j] >> 24], orr);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#pragma unroll
            for (int j = 0; j < DV_JB; ++j)
                if (rdy[j]) {
                    const int t = t0 + j * NT + tid;
                    __hip_atomic_fetch_or(&cdone[t >> 5], 1u << (t & 31), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                }
#pragma unroll
            for (int j = 0; j < DV_JB; ++j) {
                const int t = t0 + j * NT + tid;
                if (cj[j] == ~0u || rdy[j] || is_done((uint32_t)t)) continue;
                climb(t, cj[j]);
            }
        }
    }
}


/* The rows of the nI sources I (device list) by derivation, into lat / rel rows placed by source
 * (row v - src_begin, stride ldo), from the core rows already there and their codes (row crow[k]
 * of codes, stride n). rowptr / cw / ridx: the original-order CSR with each arc's index into
 * rtab (ntab <= 256 distinct reliabilities). Every source of I has degree <= DV_MAXDEG and every
 * neighbour is a core vertex (the caller's independent set). Stream-ordered, no wait. */
int srt_derive_rows_async(int n, int nI, const int32_t* I, int src_begin, const int2* rowptr,
                          const uint2* cw, const uint8_t* ridx, const double* rtab, int ntab,
                          const int32_t* crow, const uint32_t* codes, uint32_t* lat, double* rel,
                          size_t ldo, hipStream_t st) {
    if (nI <= 0) return SRT_OK;
    if (ntab > 256 || n > (1 << 17)) {
        srt_set_error("derive: %d distinct reliabilities (at most 256) or n = %d past 2^17", ntab, n);
        return SRT_E_ARG;
    }
    int cus = 256, dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        cus = prop.multiProcessorCount;
    /* 1,024 threads, one workgroup per CU, 16,384 cached parents: 118 ms on C5 against 125 (512
     * threads x 2, 8,192 cached) and 133 (256 x 4, no cache). Deriving the codes from the row's
     * own distances in LDS instead of the core kernel's stores: core 391 -> 338 ms but derive
     * 116 -> 202 ms (the in-arc scans), dropped */
    constexpr int NTD = 1024, CACHED = 16384;
    const int grid = nI < cus ? nI : cus;
    const size_t np = ((size_t)n + 3) & ~(size_t)3;
    uint32_t* cs = NULL;
    SRT_HIPCHK(srt_malloc_async(&cs, ((size_t)grid * np + 4) * sizeof(uint32_t), st));
    unsigned* queue = cs + (size_t)grid * np;
    SRT_HIPCHK(hipMemsetAsync(queue, 0, sizeof(unsigned), st));
    const size_t lds = (size_t)((((n + 31) / 32) + 3) & ~3) * sizeof(uint32_t) + (size_t)CACHED * 8;
    SRT_HIPCHK(hipFuncSetAttribute((const void*)derive_chain_kernel<NTD, CACHED>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    derive_chain_kernel<NTD, CACHED><<<grid, NTD, lds, st>>>(n, nI, I, src_begin, rowptr, cw, ridx,
                                                             rtab, ntab, crow, codes, lat, rel, ldo,
                                                             cs, np, queue);
    SRT_HIPCHK(hipGetLastError());
    SRT_HIPCHK(hipFreeAsync(cs, st));
    return SRT_OK;
}
