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
 * Vertex order: the kernel runs on a Cuthill-McKee relabelling of the graph (build.hip), so a
 * frontier's neighbours sit in nearby words of the working distance row and each random access
 * shares cache lines with the next ones (the C3 profile without it: 28% L2 hits, 245 GB fetched
 * for 44 GB of algorithmic bytes). Arcs of a relabelled row stay sorted by ORIGINAL neighbour
 * index, so the (D[u], arc index) key still breaks ties by original vertex index.
 * Memory: per wave a working distance row (u32 quanta) and a reliability row (f64), both in
 * relabelled order, and a bucket ring (C x bcap vertex ids) in global memory; bucket counts and
 * the non-empty mask in LDS. The predecessor's reliability is read from the relabelled row, where
 * graph neighbours sit close together; when the source is done, one pass gathers both rows into
 * the output rows in original order with whole-line writes (settle-time scattered 4- and 8-byte
 * writes into the output rows were partial-line HBM writes). A bucket overflow flags the source
 * and the caller recomputes it with the workgroup-per-source kernel (sparse.hip) -- never
 * approximate.
 *
 * Arc work inside one step is balanced across lanes merge-path style: the settled vertices of a
 * 64-entry chunk are laid end to end by an exclusive scan of their degrees, and each lane finds
 * the vertex owning its arc position with one LDS write + a wave max-scan.
 */
#include "srt_device.h"

#define WL 64

/* Every row a wave touches is private to its workgroup (one wave), so workgroup-scope relaxed
 * atomic loads are coherent with the wave's own stores and atomics and may be served by the
 * CU's L1 / the XCD's L2 (agent scope would send every load past the per-XCD L2). */
static __device__ __forceinline__ uint32_t ld_coherent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
static __device__ __forceinline__ double ld_coherent(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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

template <bool DIRECTED, bool LDSD, bool RELP>
__global__ __launch_bounds__(WL) void wsssp_kernel(
    int n, int src_begin, const int32_t* __restrict__ srcs, int nsrc,
    const int2* __restrict__ rowptr, const uint2* __restrict__ cw, const double* __restrict__ r,
    const int2* __restrict__ in_rowptr, const uint2* __restrict__ in_cw,
    const double* __restrict__ in_r, const int32_t* __restrict__ perm,
    const int32_t* __restrict__ inv, uint32_t* __restrict__ lat, double* __restrict__ rel,
    size_t ldo, uint32_t* __restrict__ ws, int nb, int bcap, int* __restrict__ overflow) {
    __shared__ uint32_t bcnt[256];
    __shared__ unsigned long long bmask[4];
    __shared__ int s_beg[WL], s_excl[WL], s_own[WL];
    __shared__ unsigned long long s_best[WL];
    __shared__ int s_ovf;
    const int lane = threadIdx.x;
    extern __shared__ uint32_t sdist[]; /* LDSD: the working row lives in LDS */
    /* per slot: the path-order reliability row (f64, relabelled order), the bucket ring, then
     * (global form) the distance row (relabelled order) */
    const size_t relw = RELP ? 2 * (size_t)n : 0;
    const size_t slot_words = (relw + (size_t)nb * bcap + (LDSD ? 0 : n) + 1) & ~(size_t)1;
    double* relp = reinterpret_cast<double*>(ws + (size_t)blockIdx.x * slot_words);
    uint32_t* buckets = ws + (size_t)blockIdx.x * slot_words + relw;
    uint32_t* dist = LDSD ? sdist : buckets + (size_t)nb * bcap; /* working row, relabelled */
    auto dload = [&](uint32_t i) -> uint32_t {
        if constexpr (LDSD) return sdist[i];
        else return ld_coherent(dist + i);
    };
    const uint32_t bmaskm = (uint32_t)nb - 1u;

    for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int s = inv[srcs ? srcs[si] : src_begin + si];
        uint32_t* ol = lat + (size_t)si * ldo; /* output rows, original order */
        double* rr = rel + (size_t)si * ldo;
        for (int v = lane; v < n; v += WL) {
            dist[v] = (v == s) ? 0u : SRT_INF;
            if (RELP) {
                relp[v] = 0.0;
            } else {
                ol[v] = SRT_INF;
                rr[v] = 0.0;
            }
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
                    if (dload((uint32_t)v) == d) {
                        const int2 be = rowptr[v];
                        beg = be.x;
                        deg = be.y - be.x;
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
                        const uint32_t du = dload(u);
                        const uint32_t nd = d + wk;
                        if (nd < du) {
                            const uint32_t old =
                                LDSD ? atomicMin(sdist + u, nd)
                                     : __hip_atomic_fetch_min(dist + u, nd, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_WORKGROUP);
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
                        const int2 be = in_rowptr[v];
                        ibeg = be.x;
                        ideg = be.y - be.x;
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
                            const uint32_t du = dload(e.x);
                            if (du < SRT_INF && du + e.y == d)
                                atomicMin(&s_best[own], ((unsigned long long)du << 32) | (uint32_t)k);
                        }
                        __syncthreads();
                    }
                }
                __syncthreads();
                /* settle: path-order reliability from the canonical predecessor, kept in the
                 * relabelled row (the predecessor is a graph neighbour, so its entry is usually
                 * near v's); the distance is already final in dist[v] */
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
                            x = ld_coherent(RELP ? relp + u : rr + perm[u]) *
                                (DIRECTED ? in_r[k] : r[k]);
                        }
                    }
                    if (RELP) {
                        relp[v] = x;
                    } else {
                        const int vo = perm[v];
                        ol[vo] = d;
                        rr[vo] = x;
                    }
                }
                __threadfence_block(); /* settled rel visible to the later steps of this wave */
                __syncthreads();
            }
            if (s_ovf) break;
        }
        /* output rows in original order: whole-line writes, the relabelled rows gathered
         * (unreached vertices keep INF / 0) */
        __threadfence_block();
        __syncthreads();
        if (RELP) {
            for (int i = lane; i < n; i += WL) {
                const int v = inv[i];
                ol[i] = dload((uint32_t)v);
                rr[i] = ld_coherent(relp + v);
            }
        }
        if (s_ovf && lane == 0) overflow[si] = 1;
        __syncthreads();
    }
}


/* Rows [src_begin, src_end) by the wave-per-source kernel. *overflowed receives the number of
 * sources whose buckets overflowed; their indices (relative to src_begin) are flagged in ovf
 * (device, nsrc ints, zeroed here) for the caller to recompute. */
/* the form of the last sparse launch on this thread (srt_build_stats.fw_block of sparse builds):
 * wave kernel: 1 = working row in LDS, 2 = private relabelled reliability row; workgroup kernel:
 * 4 | 1 = original vertex order, 4 | 2 = compact arcs */
static thread_local int g_sparse_form = 0;
int srt_sparse_last_form(void) { return g_sparse_form; }

int srt_wsssp_rows(int n, int directed, const int2* rowptr, const uint2* cw, const double* r,
                   const int2* in_rowptr, const uint2* in_cw, const double* in_r,
                   const int32_t* perm, const int32_t* inv, uint32_t max_w, int local,
                   int src_begin, int src_end, const int32_t* srcs, uint32_t* lat, double* rel,
                   int* ovf, hipStream_t st) {
    int nb = 1;
    while ((uint32_t)nb <= max_w) nb <<= 1;
    if (nb > 256) {
        srt_set_error("wsssp: max arc weight %u quanta needs more than 256 buckets", max_w);
        return SRT_E_ARG;
    }
    const int nsrc = src_end - src_begin;
    int bcap = n < 8192 ? n : 8192;
    const int fb = srt_form_int("bcap", 0); /* tests: force bucket overflows */
    if (fb > 0) bcap = fb;
    int cus = 256;
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        cus = prop.multiProcessorCount;
    /* working distance row in LDS when it fits (LDS atomics and gathers instead of divergent
     * global ones -- the global form is bound by the texture path at one line per lane), else a
     * global row with up to SRT_WSSSP_WAVES (default 16) waves per CU */
    const size_t lds_row = (size_t)n * sizeof(uint32_t), lds_static = 4096;
    /* the LDS form holds few waves per CU and each wave's bucket steps are a latency chain
     * (C3, n = 20000: 2 waves/CU, 354 ms vs 70 ms for the global form at 16), so it is the
     * default only while it still fits 8 waves per CU */
    const bool ldsd = 8 * (lds_row + lds_static) <= 160 * 1024;
    /* the kernel's slot layout: f64 reliability row, bucket ring, u32 distance row (global form),
     * padded to 8 bytes */
    const bool relp = local != 0;
    g_sparse_form = (ldsd ? 1 : 0) | (relp ? 2 : 0);
    const size_t per_slot =
        (((relp ? 2 * (size_t)n : 0) + (size_t)nb * bcap + (ldsd ? 0 : n) + 1) & ~(size_t)1) *
        sizeof(uint32_t);
    /* 16 waves per CU (24 / 32 / 40 measured slower on C3: 65.1 / 66.6 / 65.4 vs 62.0 ms) */
    size_t slots = ldsd ? (size_t)cus * ((160 * 1024) / (lds_row + lds_static)) : (size_t)16 * cus;
    /* the random gathers into the working rows are served by L2 / Infinity Cache / HBM; past
     * about 1.4 GB of rows in flight more waves only thrash (C5, n = 100,000: 16 waves/CU
     * 2.90 s, 3,500 waves 2.6 s, 8/CU 2.66 s; C3, n = 20,000: 16/CU 73 ms, 8/CU 98 ms) */
    if (!ldsd) {
        const size_t cap = ((size_t)1400 << 20) / ((size_t)n * sizeof(uint32_t));
        if (slots > cap) slots = cap > (size_t)cus ? cap : (size_t)cus;
    }
    /* workspace budget: what the tables and the graph leave free, up to 64 GiB (C5 at 32
     * waves/CU: 8192 slots x 4.6 MB) */
    size_t budget = (size_t)16 << 30, free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > ((size_t)8 << 30)) {
        budget = free_b - ((size_t)8 << 30);
        if (budget > ((size_t)64 << 30)) budget = (size_t)64 << 30;
    }
    if (slots * per_slot > budget) slots = budget / per_slot;
    if (slots > (size_t)nsrc) slots = nsrc;
    if (slots < 1) slots = 1;
    uint32_t* ws = NULL;
    if (srt_malloc_async((void**)&ws, slots * per_slot, st) != hipSuccess) {
        (void)hipGetLastError();
        srt_set_error("wsssp: bucket workspace of %zu MiB failed", (slots * per_slot) >> 20);
        return SRT_E_NOMEM;
    }
    SRT_HIPCHK(hipMemsetAsync(ovf, 0, (size_t)nsrc * sizeof(int), st));
    const size_t dyn = ldsd ? lds_row : 0;
#define SRT_WSSSP_LAUNCH(D, L, R)                                                                \
    do {                                                                                         \
        if (dyn) SRT_HIPCHK(hipFuncSetAttribute((const void*)wsssp_kernel<D, L, R>,               \
                                                hipFuncAttributeMaxDynamicSharedMemorySize,       \
                                                (int)dyn));                                       \
        wsssp_kernel<D, L, R><<<(unsigned)slots, WL, dyn, st>>>(                                  \
            n, src_begin, srcs, nsrc, rowptr, cw, r, in_rowptr, in_cw, in_r, perm, inv, lat, rel, \
            (size_t)n, ws, nb, bcap, ovf);                                                        \
    } while (0)
#define SRT_WSSSP_LAUNCH2(D, L)                                                                  \
    do {                                                                                         \
        if (relp) SRT_WSSSP_LAUNCH(D, L, true);                                                   \
        else SRT_WSSSP_LAUNCH(D, L, false);                                                       \
    } while (0)
    if (directed && ldsd) SRT_WSSSP_LAUNCH2(true, true);
    else if (directed) SRT_WSSSP_LAUNCH2(true, false);
    else if (ldsd) SRT_WSSSP_LAUNCH2(false, true);
    else SRT_WSSSP_LAUNCH2(false, false);
#undef SRT_WSSSP_LAUNCH2
#undef SRT_WSSSP_LAUNCH
    SRT_HIPCHK(hipGetLastError());
    SRT_HIPCHK(hipFreeAsync(ws, st));
    return SRT_OK;
}

/* ------------------------------------------------------------------------------------------ *
 * Workgroup-per-source form for large power-law graphs (C5: n = 100,000, Barabasi-Albert).
 * The wave kernel above keeps its working distance row in HBM; on such graphs the frontier has
 * no locality, so nearly every relaxation is a random line fetch beyond L2 and the kernel is bound
 * by that traffic (C5 profile: ~7 TB of lines for 2.7 s). Here one 1024-thread workgroup owns a
 * source and keeps the whole distance row in LDS, packed three 10-bit values per word (133 KB at
 * n = 100,000; code 1023 = unreached), so relaxations, staleness checks and the canonical
 * predecessor search touch only LDS; one bucket step spreads its arcs over 1024 lanes instead of
 * 64 (C5: 1.07 s with 1024 threads, 1.43 s with 512, 2.7 s for the wave kernel). Reliability
 * lives in a private relabelled f64 row (L2 / Infinity Cache), the output rows are written once
 * at the end with whole lines. Same Dial bucket order, settle-time canonical
 * predecessor argmin (D[u], arc rank) and path-order reliability as wsssp_kernel, so the tables
 * are identical. A distance above 1022 quanta or a full bucket flags the source, which the caller
 * recomputes with the wave kernel; the caller only picks this form when a probe source shows every
 * distance fits (d(a, b) <= 2 ecc(s0)). Undirected graphs only.
 * ------------------------------------------------------------------------------------------ */
#define WG_INF 1023u
/* arc windows in flight per lane. Same-box C5 A/Bs: 3 beat 4 by 1.1%, 2 beat 3 by 0.3%, and 1 and
 * 6 lost 1.9% and 4.5% (profiles/r02g/ab_ak_*) */
#define WG_AK 2
#define WG_NBLK 256 /* 64-arc blocks indexed per chunk (arcs beyond: whole-chunk search) */

static __device__ __forceinline__ uint32_t wg_get(const uint32_t* sd, uint32_t v) {
    return (sd[v / 3] >> (10 * (v % 3))) & 1023u;
}

/* lower the 10-bit field of v to nd if that is smaller; true when this call lowered it. old: the
 * word as the caller last read it (a stale value only costs one failed CAS) */
static __device__ __forceinline__ bool wg_lower(uint32_t* sd, uint32_t v, uint32_t nd, uint32_t old) {
    uint32_t* p = sd + v / 3;
    const uint32_t sh = 10 * (v % 3);
    for (;;) {
        const uint32_t cur = (old >> sh) & 1023u;
        if (nd >= cur) return false;
        const uint32_t nw = (old & ~(1023u << sh)) | (nd << sh);
        const uint32_t prev = atomicCAS(p, old, nw);
        if (prev == old) return true;
        old = prev;
    }
}

/* bucket entry: x = v | min(deg, WG_DEGC) << 17 (v < 2^17: srt_wgsssp_max_n), y = row begin, so a
 * popped entry needs no row-pointer load; a degree at the clamp reloads rowptr[v] */
#define WG_DEGC 32767u
/* workgroup barrier ordering LDS only (no wait for outstanding global stores); the barriers that
 * must publish global stores to the other waves stay __syncthreads() */
#define WG_LDS_BARRIER()                                                \
    do {                                                                \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); \
        __builtin_amdgcn_s_barrier();                                   \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); \
    } while (0)
/* the canonical in-arc of a vertex settled at distance dl from its compact-arc key (D[u] << 40 |
 * u << 8 | ridx): u | w << 17 | ridx << 24, w = dl - D[u] < 128; ~0 for the source */
static __device__ __forceinline__ uint32_t wg_code(unsigned long long key, bool src, uint32_t dl) {
    if (src || key == ~0ull) return ~0u;
    const uint32_t du = (uint32_t)(key >> 40), u = (uint32_t)(key >> 8) & 0x1FFFFu;
    return u | ((dl - du) << 17) | ((uint32_t)(key & 0xFFu) << 24);
}
static __device__ __forceinline__ uint2 wg_entry(uint32_t v, uint32_t beg, uint32_t deg) {
    return make_uint2(v | (min(deg, WG_DEGC) << 17), beg);
}
static __device__ __forceinline__ uint2 ld_coherent2(const uint2* p) {
    const unsigned long long x = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return make_uint2((uint32_t)x, (uint32_t)(x >> 32));
}

/* arcs for the workgroup kernel: (neighbour u, weight, begin of u's row, degree of u), relabelled */
__global__ void wg_arcs_kernel(int n, const int2* __restrict__ rowptr, const uint2* __restrict__ cw,
                               uint4* __restrict__ ca) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const int2 be = rowptr[v];
    for (int k = be.x; k < be.y; ++k) {
        const uint2 e = cw[k];
        const int2 bu = rowptr[e.x];
        ca[k] = make_uint4(e.x, e.y, (uint32_t)bu.x, (uint32_t)(bu.y - bu.x));
    }
}

/* compact arcs (CMP form of the workgroup kernel, original vertex order): 8 bytes per arc,
 * x = u | w << 17 | ridx << 24 (u < 2^17, w < 128, ridx = index of the arc's reliability in the
 * graph's table of distinct values, <= 256 of them), y = begin of u's row | min(deg u, 4095) << 20
 * (arcs < 2^20). Half the bytes of the uint4 arcs, and the settle step reads its reliability from
 * the 2-KB table instead of a random line of r[] */
__global__ void wg_arcs_cmp_kernel(int n, const int2* __restrict__ rowptr, const uint2* __restrict__ cw,
                                   const uint8_t* __restrict__ ridx, uint2* __restrict__ ca) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const int2 be = rowptr[v];
    for (int k = be.x; k < be.y; ++k) {
        const uint2 e = cw[k];
        const int2 bu = rowptr[e.x];
        const uint32_t deg = (uint32_t)min(bu.y - bu.x, 4095);
        ca[k] = make_uint2(e.x | (e.y << 17) | ((uint32_t)ridx[k] << 24), (uint32_t)bu.x | (deg << 20));
    }
}

/* ORIG: the graph in its original vertex order (inv == NULL): the reliability row is the output
 * row itself (settle-time stores and predecessor loads go to rr), so no end-of-source gather of a
 * private relabelled row (one random line per vertex: ~40% of the kernel's memory traffic on C5,
 * profiles/r02_c5) */
template <int WG, bool ORIG = false, bool CMP = false>
__global__ __launch_bounds__(WG) void wgsssp_kernel(
    int n, int src_begin, const int32_t* __restrict__ srcs, int nsrc,
    const int2* __restrict__ rowptr, const void* __restrict__ cav,
    const double* __restrict__ r, const int32_t* __restrict__ inv, uint32_t* __restrict__ lat,
    double* __restrict__ rel, size_t ldo, uint32_t* __restrict__ ws, int nb, int bcap,
    int* __restrict__ overflow, int two = 0,
    int place = 0, uint32_t* __restrict__ codes = nullptr, unsigned* __restrict__ queue = nullptr) {
    /* place: source s0 = srcs[si] writes output row (and overflow flag) s0 - src_begin instead of
     * si. codes (CMP only): the canonical in-arc of every settled vertex v, row si (stride n):
     * u | w << 17 | ridx << 24 (~0 for the source) -- the neighbour-row derivation's input
     * (derive.hip) */
    /* CMP: cav holds the compact arcs and r the table of distinct reliabilities */
    /* two (SRT_FORM wg_two): a step settles the entries of buckets d and d + 1 present at its start.
     * An entry at d + 1 is final then (every unsettled vertex is at >= d and arcs are >= 1
     * quantum), and its tight predecessors are at <= d: settled, or level 0 of this step. The
     * level-0 entries come first in the step's index order; a chunk holding both levels stores its
     * level-0 reliabilities before a full barrier and only then loads the level-1 ones. Pushes
     * during the step may append to bucket d + 1: bst[] keeps each bucket's consumed prefix. */
    static_assert(!CMP || ORIG, "compact arcs key ties on u: original vertex order only");
    const uint4* __restrict__ ca = reinterpret_cast<const uint4*>(cav);
    const uint2* __restrict__ cc = reinterpret_cast<const uint2*>(cav);
    extern __shared__ uint32_t sd[]; /* packed distances, relabelled order */
    __shared__ uint32_t bcnt[256]; /* entries per bucket; the search ballots on bcnt > bst */
    __shared__ uint32_t bst[256];  /* consumed prefix of each bucket (two-level steps) */
    /* s_off[i] = row begin - exclusive arc offset of chunk entry i (arc a of owner i is at
     * a + s_off[i]); s_blk[B] = the owner of chunk arc 64 B, so a wave's owner search runs over
     * [s_blk[B], s_blk[B + 1]] (a few entries) instead of the whole chunk */
    __shared__ int s_off[WG], s_excl[WG], s_wtot[WG / WL];
    __shared__ uint16_t s_blk[WG_NBLK];
    __shared__ unsigned long long s_best[WG];
    __shared__ int s_ovf;
    const int tid = threadIdx.x, lane = tid & (WL - 1), wv = tid >> 6;
    const int words = (n + 2) / 3;
    const size_t slot_words = ((size_t)nb * bcap * 2 + (ORIG ? 0 : 2 * (size_t)n) + 1) & ~(size_t)1;
    uint2* buckets = reinterpret_cast<uint2*>(ws + (size_t)blockIdx.x * slot_words);
    double* relp = ORIG ? nullptr : reinterpret_cast<double*>(buckets + (size_t)nb * bcap);
    const uint32_t bm = (uint32_t)nb - 1u;
    /* sources from a work queue, not a fixed stride: with one workgroup per CU, a workgroup that
     * started late (its CU still busy at launch) or ran slowly left its whole stride to the end:
     * single C5 launches took 620-1,008 ms against ~390 */
    __shared__ int s_next;
    for (;;) {
        if (tid == 0) s_next = queue ? (int)atomicAdd(queue, 1u) : -1;
        __syncthreads();
        const int si = s_next;
        if (si >= nsrc || si < 0) break;
        const int s0 = srcs ? srcs[si] : src_begin + si;
        const int s = ORIG ? s0 : inv[s0];
        const int orow = place ? s0 - src_begin : si;
        uint32_t* ol = lat + (size_t)orow * ldo;
        double* rr = rel + (size_t)orow * ldo;
        uint32_t* cd = CMP && codes ? codes + (size_t)si * n : nullptr;
        if (ORIG) relp = rr;
        for (int q = tid; q < words; q += WG) sd[q] = 0x3FFFFFFFu; /* three unreached fields */
        /* ORIG: the output row is written at settle time; unreached entries get their 0 at the
         * end (no full-row initialisation pass) */
        if (!ORIG)
            for (int v = tid; v < n; v += WG) relp[v] = 0.0;
        for (int b = tid; b < nb; b += WG) {
            bcnt[b] = 0;
            bst[b] = 0;
        }
        __syncthreads();
        if (tid == 0) {
            s_ovf = 0;
            sd[s / 3] &= ~(1023u << (10 * (s % 3))); /* D[s] = 0 */
            const int2 be = rowptr[s];
            buckets[0] = wg_entry((uint32_t)s, (uint32_t)be.x, (uint32_t)(be.y - be.x));
            bcnt[0] = 1;
        }
        __threadfence_block();
        __syncthreads();
        /* deferred settle: the reliability of the lane's last settled vertex pv is stored after
         * the next chunk's arcs (or after the last step), so its two loads overlap the bucket
         * search, the next entry load and the arcs; nothing reads rel(s, pv) before a larger
         * distance value is settled -- a later step, whose first chunk's post-arcs barrier is a
         * full one that orders the store before that chunk's settle loads */
        int pv = -1;
        double pa = 0.0, pb = 0.0;
        uint32_t d = 0;
        for (;;) {
            /* next non-empty bucket at or after d (circular), found by every wave itself: bcnt
             * and bst are final since the step's last post-arc barrier, a full one (the pushed
             * entries are visible), and nothing writes either before every wave has passed the
             * first chunk's scan barrier (the popped and the skipped buckets are reset there), so
             * every wave finds the same bucket -- no workgroup barrier and broadcast here */
            int found = -1;
            const uint32_t p0 = d & bm;
            for (int q = 0; q < nb && found < 0; q += WL) {
                const int pos = (int)((p0 + (uint32_t)q + (uint32_t)lane) & bm);
                const bool set = q + lane < nb && bcnt[pos] > bst[pos];
                const unsigned long long bal = __ballot(set);
                if (bal) found = q + __ffsll((long long)bal) - 1;
            }
            if (found < 0) break;
            d += (uint32_t)found;
            const int b = (int)(d & bm), b1 = (int)((d + 1u) & bm);
            const int st0 = (int)bst[b], st1 = two ? (int)bst[b1] : 0;
            const int n0 = max(0, min((int)bcnt[b], bcap) - st0);
            const int n1 = two ? max(0, min((int)bcnt[b1], bcap) - st1) : 0;
            const int cnt = n0 + n1;
            /* bucket b is reset after the first chunk's scan barrier (every thread has read its
             * counts by then): no push of this step targets b (nd >= d + 1, and the ring is longer
             * than the largest weight), and the next search follows this step's last barrier;
             * bucket d + 1 keeps its count and records the consumed prefix */
            const uint2* bk = buckets + (size_t)b * bcap + st0;
            const uint2* bk1 = buckets + (size_t)b1 * bcap + st1;
            for (int c0 = 0; c0 < cnt; c0 += WG) {
                const int i = c0 + tid;
                const int lvl = i >= n0; /* 1: an entry of bucket d + 1 */
                const uint32_t dl = d + (uint32_t)lvl;
                int v = -1, beg = 0, deg = 0;
                uint2 en = make_uint2(0u, 0u);
                if (i < cnt) en = ld_coherent2(lvl ? bk1 + (i - n0) : bk + i);
                if (i < cnt) {
                    v = (int)(en.x & 0x1FFFFu);
                    if (wg_get(sd, (uint32_t)v) == dl) {
                        beg = (int)en.y;
                        deg = (int)(en.x >> 17);
                        if ((uint32_t)deg == WG_DEGC) {
                            const int2 be = rowptr[v];
                            deg = be.y - be.x;
                        }
                    } else {
                        v = -1; /* stale: improved after it was pushed */
                    }
                }
                /* workgroup exclusive scan of the degrees */
                int wtot;
                const int wex = wave_scan_excl(deg, lane, &wtot);
                if (lane == 0) s_wtot[wv] = wtot;
                WG_LDS_BARRIER();
                if (c0 == 0 && tid == 0) {
                    bcnt[b] = 0;
                    bst[b] = 0;
                    if (two) bst[b1] = (uint32_t)(st1 + n1);
                }
                /* the buckets the search skipped over (bcnt == bst: consumed, or empty) restart
                 * at 0/0 for their next wrap; reset only here, after every wave's search, so no
                 * wave can read an old bcnt beside a zeroed bst. No push targets them before the
                 * arcs below, which follow the next barrier. */
                if (c0 == 0 && two && tid < found) {
                    bcnt[(p0 + (uint32_t)tid) & bm] = 0;
                    bst[(p0 + (uint32_t)tid) & bm] = 0;
                }
                int base = 0, total = 0;
                for (int q = 0; q < WG / WL; ++q) {
                    base += q < wv ? s_wtot[q] : 0;
                    total += s_wtot[q];
                }
                const int x = base + wex;
                s_off[tid] = beg - x;
                s_excl[tid] = x;
                s_best[tid] = ~0ull;
                {
                    int B = (x + 63) >> 6; /* first block start in [x, x + deg): usually 0 or 1 */
                    const int Be = min((x + deg - 1) >> 6, WG_NBLK - 1);
                    if (deg > 0 && B <= Be) {
                        s_blk[B] = (uint16_t)tid;
                        for (++B; B <= Be; ++B) s_blk[B] = (uint16_t)tid; /* hubs */
                    }
                }
                /* the owner of the last arc closes the last block's range */
                if (deg > 0 && x + deg == total && (total - 1) / WL + 1 < WG_NBLK)
                    s_blk[(total - 1) / WL + 1] = (uint16_t)tid;
                WG_LDS_BARRIER();
                /* WG_AK arc windows per pass: the owner searches (fixed-step, unrolled) and the
                 * arc loads of every window are issued before any of them is used, so their
                 * latencies overlap instead of adding up */
                for (int a0 = 0; a0 < total; a0 += WG * WG_AK) {
                    int own[WG_AK];
                    uint4 e[WG_AK];
                    uint2 ec[WG_AK];
                    /* owner: the last entry whose exclusive offset is <= a, searched between the
                     * owners of the wave's block start and of the next block start (wave-uniform
                     * bounds, one step count for all windows) */
                    int hi[WG_AK], len = 0;
                    const int totu = __builtin_amdgcn_readfirstlane(total);
#pragma unroll
                    for (int j = 0; j < WG_AK; ++j) { /* all the bound reads issued together */
                        const int B = min((a0 + j * WG) / WL + __builtin_amdgcn_readfirstlane(wv),
                                          WG_NBLK - 2);
                        own[j] = s_blk[B];
                        hi[j] = s_blk[B + 1];
                    }
#pragma unroll
                    for (int j = 0; j < WG_AK; ++j) {
                        const int B = (a0 + j * WG) / WL + __builtin_amdgcn_readfirstlane(wv);
                        if (B * WL >= totu) { /* no arcs for this wave in the window */
                            own[j] = 0;
                            hi[j] = 0;
                        } else if (B + 1 < WG_NBLK) {
                            own[j] = __builtin_amdgcn_readfirstlane(own[j]);
                            hi[j] = __builtin_amdgcn_readfirstlane(hi[j]);
                        } else {
                            own[j] = 0;
                            hi[j] = WG - 1;
                        }
                        len = max(len, hi[j] - own[j]);
                    }
                    len = __builtin_amdgcn_readfirstlane(len);
                    for (int step = len > 0 ? 1 << (31 - __builtin_clz(len)) : 0; step >= 1;
                         step >>= 1) {
                        /* clamped at hi: taking hi when s_excl[hi] <= a is the answer (the owner
                         * is at most hi), so the lifting stays exact */
                        int q[WG_AK];
#pragma unroll
                        for (int j = 0; j < WG_AK; ++j) {
                            q[j] = min(own[j] + step, hi[j]);
                            q[j] = s_excl[q[j]] <= a0 + j * WG + tid ? q[j] : own[j];
                        }
#pragma unroll
                        for (int j = 0; j < WG_AK; ++j) own[j] = q[j];
                    }
#pragma unroll
                    for (int j = 0; j < WG_AK; ++j)
                        if (a0 + j * WG + tid < total) {
                            const int arc = a0 + j * WG + tid + s_off[own[j]];
                            if constexpr (CMP)
                                ec[j] = cc[arc];
                            else
                                e[j] = ca[arc];
                        }
#pragma unroll
                    for (int j = 0; j < WG_AK; ++j) {
                        if (a0 + j * WG + tid >= total) continue;
                        uint32_t u, wk, ridx = 0, begu, degu;
                        if constexpr (CMP) {
                            u = ec[j].x & 0x1FFFFu;
                            wk = (ec[j].x >> 17) & 0x7Fu;
                            ridx = ec[j].x >> 24;
                            begu = ec[j].y & 0xFFFFFu;
                            degu = ec[j].y >> 20;
                            if (degu == 4095u) degu = WG_DEGC; /* clamped: reloaded at pop */
                        } else {
                            u = e[j].x;
                            wk = e[j].y;
                            begu = e[j].z;
                            degu = e[j].w;
                        }
                        const uint32_t wu = sd[u / 3];
                        const uint32_t du = (wu >> (10 * (u % 3))) & 1023u;
                        const uint32_t dow = d + (uint32_t)(c0 + own[j] >= n0); /* owner's D */
                        const uint32_t nd = dow + wk;
                        if (nd < du) {
                            if (nd >= WG_INF) {
                                s_ovf = 1; /* not representable in 10 bits */
                            } else if (wg_lower(sd, u, nd, wu)) {
                                const int b2 = (int)(nd & bm);
                                const int slot = (int)atomicAdd(&bcnt[b2], 1u);
                                if (slot < bcap) {
                                    buckets[(size_t)b2 * bcap + slot] = wg_entry(u, begu, degu);
                                } else {
                                    s_ovf = 1;
                                }
                            }
                        }
                        /* canonical predecessor key (D[u], rank of the arc in the row), with u
                         * carried along so the settle step needs no second arc load */
                        if (du != WG_INF && du + wk == dow) {
                            if constexpr (CMP) /* (D[u], u) with the arc's reliability index */
                                atomicMin(&s_best[own[j]], ((unsigned long long)du << 40) |
                                                               ((unsigned long long)u << 8) | ridx);
                            else
                                atomicMin(&s_best[own[j]],
                                          ((unsigned long long)du << 40) |
                                              ((unsigned long long)(a0 + j * WG + tid - s_excl[own[j]]) << 20) |
                                              u);
                        }
                    }
                }
                /* the lane's vertex of the previous chunk: its two loads (issued at that chunk's
                 * settle) have had this chunk's head and arcs to arrive */
                if (pv >= 0) {
                    relp[pv] = pa * pb;
                    pv = -1;
                }
                /* full barrier after a step's first chunk (it may settle children of the previous
                 * chunk's vertices: their reliability stores visible) and after its last (the
                 * next step's search and entry loads follow with no other barrier: this pass's
                 * bucket stores visible); an LDS barrier in between */
                const bool mixed = two && n1 > 0 && c0 + WG > n0; /* level-1 lanes in this chunk */
                if (c0 == 0 || c0 + WG >= cnt || mixed)
                    __syncthreads();
                else
                    WG_LDS_BARRIER();
                /* a chunk with level-1 lanes: its level-0 lanes store their reliability now, and
                 * the level-1 lanes (children of any level-0 vertex of the step) load theirs after
                 * a full barrier */
                if (mixed) {
                    if (v >= 0 && !lvl) {
                        double xa = 1.0, xb = 1.0;
                        if (cd) cd[v] = wg_code(s_best[tid], v == s, dl);
                        if (v != s) {
                            const unsigned long long key = s_best[tid];
                            xa = 0.0;
                            if (key != ~0ull) {
                                if constexpr (CMP) {
                                    xa = ld_coherent(relp + (uint32_t)((key >> 8) & 0x1FFFFu));
                                    xb = r[key & 0xFFu];
                                } else {
                                    xa = ld_coherent(relp + (uint32_t)(key & 0xFFFFFu));
                                    xb = r[beg + (int)((key >> 20) & 0xFFFFFu)];
                                }
                            }
                        }
                        relp[v] = xa * xb;
                        v = -1; /* settled: no deferred store */
                    }
                    __threadfence_block();
                    __syncthreads();
                }
                /* settle: path-order reliability from the canonical predecessor, issued now and
                 * stored one chunk later */
                if (v >= 0) {
                    if (cd) cd[v] = wg_code(s_best[tid], v == s, dl);
                    pv = v;
                    pa = 1.0;
                    pb = 1.0;
                    if (v != s) {
                        const unsigned long long key = s_best[tid];
                        pa = 0.0;
                        if (key != ~0ull) {
                            if constexpr (CMP) {
                                pa = ld_coherent(relp + (uint32_t)((key >> 8) & 0x1FFFFu));
                                pb = r[key & 0xFFu];
                            } else {
                                pa = ld_coherent(relp + (uint32_t)(key & 0xFFFFFu));
                                pb = r[beg + (int)((key >> 20) & 0xFFFFFu)];
                            }
                        }
                    }
                }
            }
            if (s_ovf) break;
        }
        if (pv >= 0) relp[pv] = pa * pb;
        __threadfence_block();
        __syncthreads();
        /* output rows in original order, whole lines */
        for (int i = tid; i < n; i += WG) {
            const int v = ORIG ? i : inv[i];
            const uint32_t dv = wg_get(sd, (uint32_t)v);
            ol[i] = dv == WG_INF ? SRT_INF : dv;
            if (!ORIG)
                rr[i] = ld_coherent(relp + v);
            else if (dv == WG_INF)
                rr[i] = 0.0; /* unreached */
        }
        if (s_ovf && tid == 0) overflow[orow] = 1;
        __syncthreads();
    }
}

/* largest n the packed LDS row holds beside the kernel's static LDS (1024 threads: ~18 KB) */
int srt_wgsssp_max_n(void) { return 3 * ((137 * 1024) / 4); }

/* Rows [src_begin, src_end) by the workgroup kernel (undirected graphs, n <= srt_wgsssp_max_n,
 * max arc weight < 256 quanta). ovf[i] = 1 marks a source to recompute (distance above 1022 or a
 * full bucket). */
int srt_wgsssp_rows(int n, const int2* rowptr, const uint2* cw, const double* r, const int32_t* inv,
                    uint32_t max_w, int src_begin, int src_end, const int32_t* srcs, uint32_t* lat,
                    double* rel, int* ovf, hipStream_t st, const uint8_t* ridx,
                    const double* rtab, int place, uint32_t* codes) {
    /* two-level steps push up to d + 1 + max_w: the ring then needs max_w + 2 buckets */
    const int two = max_w + 2u <= 256u;
    int nb = 1;
    while ((uint32_t)nb <= max_w + (uint32_t)two) nb <<= 1;
    if (inv) { /* the relabelled form was retired (measured slower than the original order) */
        srt_set_error("wgsssp: the kernel runs on the original vertex order (inv must be NULL)");
        return SRT_E_ARG;
    }
    if (nb > 256 || n > srt_wgsssp_max_n()) {
        srt_set_error("wgsssp: n = %d or max arc weight %u outside the kernel's range", n, max_w);
        return SRT_E_ARG;
    }
    const int nsrc = src_end - src_begin;
    int bcap = n < 32768 ? n : 32768; /* entries per bucket (uint2) */
    const int fb = srt_form_int("bcap", 0); /* tests: force bucket overflows */
    if (fb > 0) bcap = fb;
    int cus = 256, dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        cus = prop.multiProcessorCount;
    /* arcs carrying their head's row bounds (built per call: a few MB, microseconds) */
    int2 last;
    SRT_HIPCHK(hipMemcpyAsync(&last, rowptr + (n - 1), sizeof(int2), hipMemcpyDeviceToHost, st));
    SRT_HIPCHK(hipStreamSynchronize(st));
    /* compact 8-byte arcs: original order, a reliability table, w < 128, arcs < 2^20 */
    const bool cmp = !inv && ridx && rtab && max_w < 128 && last.y < (1 << 20);
    g_sparse_form = 4 | (inv ? 0 : 1) | (cmp ? 2 : 0);
    if (codes && !cmp) {
        srt_set_error("wgsssp: arc codes need the compact-arc form");
        return SRT_E_ARG;
    }
    void* ca = NULL;
    const size_t arc_bytes = cmp ? sizeof(uint2) : sizeof(uint4);
    if (srt_malloc_async(&ca, ((size_t)last.y + 1) * arc_bytes, st) != hipSuccess) {
        (void)hipGetLastError();
        srt_set_error("wgsssp: arc array of %d arcs failed", last.y);
        return SRT_E_NOMEM;
    }
    if (cmp)
        wg_arcs_cmp_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, rowptr, cw, ridx,
                                                                        (uint2*)ca);
    else
        wg_arcs_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, rowptr, cw, (uint4*)ca);
    SRT_HIPCHK(hipGetLastError());
    const size_t slot_words = ((size_t)nb * bcap * 2 + (inv ? 2 * (size_t)n : 0) + 1) & ~(size_t)1;
    size_t slots = (size_t)cus; /* one workgroup per CU: the packed row takes most of the LDS */
    if (slots > (size_t)nsrc) slots = nsrc;
    uint32_t* ws = NULL;
    /* + the work queue's counter, past the slots */
    if (srt_malloc_async((void**)&ws, (slots * (slot_words + 2) + 2) * sizeof(uint32_t), st) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFreeAsync(ca, st);
        srt_set_error("wgsssp: workspace of %zu MiB failed", (slots * slot_words * 4) >> 20);
        return SRT_E_NOMEM;
    }
    /* placed rows flag overflows at their row: the caller clears the flags */
    if (!place) SRT_HIPCHK(hipMemsetAsync(ovf, 0, (size_t)nsrc * sizeof(int), st));
    unsigned* queue = ws + slots * (slot_words + 2);
    SRT_HIPCHK(hipMemsetAsync(queue, 0, sizeof(unsigned), st));
    const size_t dyn = (size_t)((n + 2) / 3) * sizeof(uint32_t);
    if (cmp) { /* original order, compact arcs, reliabilities from the table */
        SRT_HIPCHK(hipFuncSetAttribute((const void*)wgsssp_kernel<1024, true, true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
        wgsssp_kernel<1024, true, true><<<(unsigned)slots, 1024, dyn, st>>>(
            n, src_begin, srcs, nsrc, rowptr, ca, rtab, inv, lat, rel, (size_t)n, ws, nb, bcap, ovf,
            two, place, codes, queue);
    } else { /* the graph in original order: reliability straight into the output rows */
        SRT_HIPCHK(hipFuncSetAttribute((const void*)wgsssp_kernel<1024, true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
        wgsssp_kernel<1024, true><<<(unsigned)slots, 1024, dyn, st>>>(
            n, src_begin, srcs, nsrc, rowptr, ca, r, inv, lat, rel, (size_t)n, ws, nb, bcap, ovf,
            two, place, codes, queue);
    }
    SRT_HIPCHK(hipGetLastError());
    SRT_HIPCHK(hipFreeAsync(ws, st));
    SRT_HIPCHK(hipFreeAsync(ca, st));
    return SRT_OK;
}
