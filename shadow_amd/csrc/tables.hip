/*
 * tables.hip -- passes shared by every build form, gfx950:
 *   - path-order latency in f64 milliseconds (the reference's `totalLatency`),
 *   - path-order reliability by sweeps over rows held in HBM (rows too long for LDS),
 *   - sub-table gathers for tables over the attached vertices only,
 *   - the minimum table entry (runahead export).
 *
 * Reference: /root/reference/src/main/routing/topology.c:1308 (`totalLatency = 0.0`), :1364
 * (`totalLatency += edgeLatency` hop by hop, s -> t), :294 (edge latency = (double)ns / 1e6 ms),
 * :1604-1656 (paths are computed towards the vertices with attached hosts only), :1253-1264 (the
 * minimum path latency handed to worker_updateMinTimeJump).
 *
 * Every build keeps latencies as exact integer quanta (quantum = gcd of the edge latencies), so a
 * hop (u -> t) on a shortest path has weight D[s][t] - D[s][u] quanta and (double)(w_q * q) / 1e6
 * is bit-for-bit the reference's (double)ns / 1e6. When every edge is a whole number of ms these
 * sums are exact integers and equal lat_q * q / 1e6, so the f64 table is only built when some edge
 * latency has a sub-millisecond part (topology.c / build.hip decide).
 */
#include "srt_device.h"

#define PS_THREADS 1024

static __device__ __forceinline__ double ld_wg(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
static __device__ __forceinline__ void st_wg(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

/* One workgroup per row (persistent grid). Row r belongs to source s = srcs[r] (or src_begin + r).
 * P: the canonical predecessor row (dense post pass, HAS_PRED), else recomputed here from the
 * final distance row over the in-arc CSR: argmin (D[s][u], u) among tight in-arcs u -> t, the rule
 * every build kernel applies, into the block's scratch row.
 * MS: out[t] = out[pred] + ms(pred -> t), from 0.0 at the source (topology.c:1308, :1364).
 * REL: rel[t] = rel[pred] * rel[t] in place, the rel row arriving with r(pred, t) (the product of
 * topology.c:1365; rows flagged in `only`, as rel_sweeps_kernel in dense.hip for n beyond its LDS).
 * Targets resolve in sweeps once their predecessor has: done / fresh bitmaps in LDS; a sweep
 * reads out[pred] only for predecessors resolved in an earlier sweep (barrier-ordered), so each
 * entry is formed once, in path order. The diagonal is the "path to self" rule: MS writes
 * out[s] = D[s][s] q / 1e6 (self-loop L or 2L, exact doubling) at the end, so the pass runs after
 * the diagonal rule has written D[s][s]. */
template <bool HAS_PRED, bool MS, bool REL, typename DT = uint32_t>
__global__ __launch_bounds__(PS_THREADS) void path_sweeps_kernel(
    int n, int nrows, const int32_t* __restrict__ srcs, int src_begin,
    const DT* __restrict__ D, size_t ldd, const int32_t* __restrict__ pred, size_t ldp,
    const int32_t* __restrict__ irp, const int32_t* __restrict__ icol,
    const uint32_t* __restrict__ iw, uint64_t q, double* __restrict__ out, size_t ldo,
    const int32_t* __restrict__ only, int32_t* __restrict__ pws, int32_t* __restrict__ max_depth) {
    extern __shared__ uint32_t bm[];
    __shared__ int s_any;
    const int nw = (n + 31) >> 5;
    uint32_t* done = bm;
    uint32_t* fresh = bm + nw;
    const int tid = threadIdx.x;
    int depth_max = 0;
    for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
        if (only && !only[r]) continue;
        const int s = srcs ? srcs[r] : src_begin + r;
        const DT* Dr = D + (size_t)r * ldd;
        double* o = out + (size_t)r * ldo;
        /* SRT_INF for u32 rows; the u64 rows of wide.hip mark unreachable with ~0 */
        constexpr DT INF = sizeof(DT) == 4 ? (DT)SRT_INF : (DT)~(DT)0;
        const int32_t* P;
        if constexpr (HAS_PRED) {
            P = pred + (size_t)r * ldp;
        } else {
            static_assert(HAS_PRED || sizeof(DT) == 4, "u64 rows come with their predecessors");
            int32_t* pw = pws + (size_t)blockIdx.x * n;
            for (int t = tid; t < n; t += PS_THREADS) {
                int bu = -1;
                const uint32_t dt = Dr[t];
                if (t != s && dt < SRT_INF) {
                    uint64_t best = ~0ull;
                    const int ke = irp[t + 1];
                    for (int k = irp[t]; k < ke; ++k) {
                        const int u = icol[k];
                        const uint32_t du = u == s ? 0u : Dr[u];
                        if (du < SRT_INF && du + iw[k] == dt) {
                            const uint64_t key = ((uint64_t)du << 32) | (uint32_t)u;
                            if (key < best) {
                                best = key;
                                bu = u;
                            }
                        }
                    }
                }
                pw[t] = bu;
            }
            P = pw;
        }
        for (int w = tid; w < 2 * nw; w += PS_THREADS) bm[w] = 0u;
        if (MS)
            for (int t = tid; t < n; t += PS_THREADS) st_wg(o + t, 0.0);
        __threadfence_block();
        __syncthreads();
        if (tid == 0) {
            done[s >> 5] = 1u << (s & 31);
            if (REL) st_wg(o + s, 1.0);
        }
        __threadfence_block();
        __syncthreads();
        int depth = 0;
        for (;;) {
            if (tid == 0) s_any = 0;
            __syncthreads();
            int any = 0;
            for (int w = tid; w < nw; w += PS_THREADS) {
                uint32_t pend = ~done[w];
                if (w == nw - 1 && (n & 31)) pend &= (1u << (n & 31)) - 1u;
                uint32_t got = 0u;
                while (pend) {
                    const int b = __ffs(pend) - 1;
                    pend &= pend - 1u;
                    const int t = (w << 5) + b;
                    const int p = P[t];
                    if (p < 0 || !((done[p >> 5] >> (p & 31)) & 1u)) continue;
                    if constexpr (MS) {
                        const DT dp = p == s ? (DT)0 : Dr[p];
                        const double hop = (double)((uint64_t)(Dr[t] - dp) * q) / 1e6;
                        st_wg(o + t, ld_wg(o + p) + hop);
                    } else {
                        st_wg(o + t, ld_wg(o + p) * ld_wg(o + t));
                    }
                    got |= 1u << b;
                }
                if (got) {
                    fresh[w] = got; /* word w belongs to this thread alone */
                    any = 1;
                }
            }
            if (any) s_any = 1;
            __threadfence_block();
            __syncthreads();
            if (!s_any) break;
            ++depth;
            for (int w = tid; w < nw; w += PS_THREADS) {
                done[w] |= fresh[w];
                fresh[w] = 0u;
            }
            __syncthreads();
        }
        if (MS && tid == 0) o[s] = Dr[s] < INF ? (double)((uint64_t)Dr[s] * q) / 1e6 : 0.0;
        depth_max = depth > depth_max ? depth : depth_max;
        __syncthreads();
    }
    if (max_depth && tid == 0) srt_max_once(max_depth, depth_max);
}

/* largest n whose two row bitmaps fit the LDS */
int srt_path_sweeps_max_n(void) { return (150 * 1024 / 8) * 32; }

static int path_grid(int nrows) {
    int cus = 256, dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        cus = prop.multiProcessorCount;
    return nrows < 2 * cus ? nrows : 2 * cus;
}

int srt_path_ms_rows(int n, int nrows, const int32_t* srcs, int src_begin, const uint32_t* D,
                     size_t ldd, const int32_t* pred, size_t ldp, const int32_t* irp,
                     const int32_t* icol, const uint32_t* iw, uint64_t quantum_ns, double* out,
                     size_t ldo, hipStream_t st) {
    if (nrows <= 0) return SRT_OK;
    if (n > srt_path_sweeps_max_n() || (!pred && (!irp || !icol || !iw))) {
        srt_set_error("path-order ms pass: n = %d beyond its range or no predecessor source", n);
        return SRT_E_RANGE;
    }
    const int grid = path_grid(nrows);
    const size_t lds = 2 * (size_t)((n + 31) / 32) * sizeof(uint32_t);
    int32_t* pws = NULL;
    if (!pred && srt_malloc_async((void**)&pws, (size_t)grid * n * sizeof(int32_t), st) != hipSuccess) {
        (void)hipGetLastError();
        srt_set_error("path-order ms pass: scratch of %zu MiB failed",
                      ((size_t)grid * n * sizeof(int32_t)) >> 20);
        return SRT_E_NOMEM;
    }
    if (pred) {
        SRT_HIPCHK(hipFuncSetAttribute((const void*)path_sweeps_kernel<true, true, false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        path_sweeps_kernel<true, true, false><<<grid, PS_THREADS, lds, st>>>(
            n, nrows, srcs, src_begin, D, ldd, pred, ldp, NULL, NULL, NULL, quantum_ns, out, ldo,
            NULL, NULL, NULL);
    } else {
        SRT_HIPCHK(hipFuncSetAttribute((const void*)path_sweeps_kernel<false, true, false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        path_sweeps_kernel<false, true, false><<<grid, PS_THREADS, lds, st>>>(
            n, nrows, srcs, src_begin, D, ldd, NULL, 0, irp, icol, iw, quantum_ns, out, ldo, NULL,
            pws, NULL);
    }
    SRT_HIPCHK(hipGetLastError());
    if (pws) SRT_HIPCHK(hipFreeAsync(pws, st));
    return SRT_OK;
}

/* u64 distance rows with their predecessor rows (wide.hip): the reliability product in place
 * over rel rows holding r(pred, t) (rel != NULL), and/or the f64-ms sums into ms (ms != NULL) */
int srt_path_rows_u64(int n, int nrows, const int32_t* srcs, int src_begin, const uint64_t* D,
                      size_t ldd, const int32_t* pred, size_t ldp, uint64_t quantum_ns, double* rel,
                      size_t ldr, double* ms, size_t ldm, hipStream_t st) {
    if (nrows <= 0) return SRT_OK;
    if (n > srt_path_sweeps_max_n() || !pred) {
        srt_set_error("path-order pass (u64 rows): n = %d beyond its range or no predecessors", n);
        return SRT_E_RANGE;
    }
    const int grid = path_grid(nrows);
    const size_t lds = 2 * (size_t)((n + 31) / 32) * sizeof(uint32_t);
    if (rel) {
        SRT_HIPCHK(hipFuncSetAttribute((const void*)path_sweeps_kernel<true, false, true, uint64_t>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        path_sweeps_kernel<true, false, true, uint64_t><<<grid, PS_THREADS, lds, st>>>(
            n, nrows, srcs, src_begin, D, ldd, pred, ldp, NULL, NULL, NULL, quantum_ns, rel, ldr,
            NULL, NULL, NULL);
        SRT_HIPCHK(hipGetLastError());
    }
    if (ms) {
        SRT_HIPCHK(hipFuncSetAttribute((const void*)path_sweeps_kernel<true, true, false, uint64_t>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        path_sweeps_kernel<true, true, false, uint64_t><<<grid, PS_THREADS, lds, st>>>(
            n, nrows, srcs, src_begin, D, ldd, pred, ldp, NULL, NULL, NULL, quantum_ns, ms, ldm,
            NULL, NULL, NULL);
        SRT_HIPCHK(hipGetLastError());
    }
    return SRT_OK;
}

/* path-order reliability by sweeps with the predecessor rows in HBM (dense rows beyond the LDS
 * form of rel_sweeps_kernel): rel rows arrive holding r(pred, t); rows with only[r] == 0 skip */
int srt_rel_sweeps_rows(int n, int nrows, int row0, const int32_t* pred, size_t ldp, double* rel,
                        size_t ldr, const int32_t* only, int32_t* max_depth, hipStream_t st) {
    if (nrows <= 0) return SRT_OK;
    if (n > srt_path_sweeps_max_n()) {
        srt_set_error("reliability sweeps: n = %d beyond the bitmap range", n);
        return SRT_E_RANGE;
    }
    const int grid = path_grid(nrows);
    const size_t lds = 2 * (size_t)((n + 31) / 32) * sizeof(uint32_t);
    SRT_HIPCHK(hipFuncSetAttribute((const void*)path_sweeps_kernel<true, false, true>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    path_sweeps_kernel<true, false, true><<<grid, PS_THREADS, lds, st>>>(
        n, nrows, NULL, row0, (const uint32_t*)NULL, 0, pred, ldp, NULL, NULL, NULL, 0, rel, ldr, only, NULL,
        max_depth);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

/* out[i][j] = in[rows[i] (or i)][cols[j]]: the sub-table of the attached vertices */
template <typename T>
__global__ __launch_bounds__(256) void gather_sub_kernel(int nr, int nc,
                                                         const int32_t* __restrict__ rows,
                                                         const int32_t* __restrict__ cols,
                                                         const T* __restrict__ in, size_t ldi,
                                                         T* __restrict__ out, size_t ldo) {
    const int i = blockIdx.y;
    if (i >= nr) return;
    const T* src = in + (size_t)(rows ? rows[i] : i) * ldi;
    T* dst = out + (size_t)i * ldo;
    for (int j = blockIdx.x * 256 + threadIdx.x; j < nc; j += gridDim.x * 256) dst[j] = src[cols[j]];
}

template <typename T>
static int gather_sub(int nr, int nc, const int32_t* rows, const int32_t* cols, const T* in,
                      size_t ldi, T* out, size_t ldo, hipStream_t st) {
    if (nr <= 0 || nc <= 0) return SRT_OK;
    for (int r0 = 0; r0 < nr; r0 += 65535) { /* grid.y limit */
        const int rr = nr - r0 < 65535 ? nr - r0 : 65535;
        dim3 g((unsigned)(srt_ceil_div(nc, 256) < 64 ? srt_ceil_div(nc, 256) : 64), (unsigned)rr);
        gather_sub_kernel<T><<<g, 256, 0, st>>>(rr, nc, rows ? rows + r0 : NULL, cols,
                                                rows ? in : in + (size_t)r0 * ldi, ldi,
                                                out + (size_t)r0 * ldo, ldo);
    }
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

int srt_gather_sub_u32(int nr, int nc, const int32_t* rows, const int32_t* cols, const uint32_t* in,
                       size_t ldi, uint32_t* out, size_t ldo, hipStream_t st) {
    return gather_sub<uint32_t>(nr, nc, rows, cols, in, ldi, out, ldo, st);
}
int srt_gather_sub_f64(int nr, int nc, const int32_t* rows, const int32_t* cols, const double* in,
                       size_t ldi, double* out, size_t ldo, hipStream_t st) {
    return gather_sub<double>(nr, nc, rows, cols, in, ldi, out, ldo, st);
}

/* minimum of a rows x cols u32 table (row stride ld) into *dmin (device, preset by the caller) */
__global__ __launch_bounds__(256) void table_min_kernel(int rows, int cols, const uint32_t* __restrict__ t,
                                                        size_t ld, uint32_t* __restrict__ dmin) {
    uint32_t m = 0xFFFFFFFFu;
    for (int i = blockIdx.y; i < rows; i += gridDim.y)
        for (int j = blockIdx.x * 256 + threadIdx.x; j < cols; j += gridDim.x * 256)
            m = min(m, t[(size_t)i * ld + j]);
    for (int off = 32; off > 0; off >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, off));
    if ((threadIdx.x & 63) == 0 && m != 0xFFFFFFFFu) atomicMin(dmin, m);
}

int srt_table_min(int rows, int cols, const uint32_t* t, size_t ld, uint32_t* dmin, hipStream_t st) {
    if (rows <= 0 || cols <= 0) return SRT_OK;
    dim3 g((unsigned)(srt_ceil_div(cols, 256) < 16 ? srt_ceil_div(cols, 256) : 16),
           (unsigned)(rows < 4096 ? rows : 4096));
    table_min_kernel<<<g, 256, 0, st>>>(rows, cols, t, ld, dmin);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

/* one-hop tables (use_shortest_path = false, topology.c:1816-1858): ms = (double)(w q) / 1e6 */
__global__ __launch_bounds__(256) void quanta_to_ms_kernel(int rows, int cols, const uint32_t* __restrict__ w,
                                                           size_t ldw, uint64_t q, double* __restrict__ out,
                                                           size_t ldo) {
    const int i = blockIdx.y;
    for (int j = blockIdx.x * 256 + threadIdx.x; j < cols; j += gridDim.x * 256) {
        const uint32_t x = w[(size_t)i * ldw + j];
        out[(size_t)i * ldo + j] = x < SRT_INF ? (double)((uint64_t)x * q) / 1e6 : 0.0;
    }
}

int srt_quanta_to_ms(int rows, int cols, const uint32_t* w, size_t ldw, uint64_t q, double* out,
                     size_t ldo, hipStream_t st) {
    for (int r0 = 0; r0 < rows; r0 += 65535) {
        const int rr = rows - r0 < 65535 ? rows - r0 : 65535;
        dim3 g((unsigned)(srt_ceil_div(cols, 256) < 64 ? srt_ceil_div(cols, 256) : 64), (unsigned)rr);
        quanta_to_ms_kernel<<<g, 256, 0, st>>>(rr, cols, w + (size_t)r0 * ldw, ldw, q,
                                               out + (size_t)r0 * ldo, ldo);
    }
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

/* Tied pairs of rows built by the SSSP kernels (srt_build_stats.tied_pairs): targets t != s whose
 * smallest D[s][u] over tight in-arcs u -> t is reached by two or more u (with D[s][s] = 0) --
 * the class where igraph's heap order, not the canonical rule, picks the reference's predecessor. */
__global__ __launch_bounds__(256) void tie_count_kernel(int n, int nrows, const int32_t* __restrict__ srcs,
                                                        int src_begin, const uint32_t* __restrict__ D,
                                                        size_t ldd, const int32_t* __restrict__ irp,
                                                        const int32_t* __restrict__ icol,
                                                        const uint32_t* __restrict__ iw,
                                                        unsigned long long* __restrict__ out) {
    unsigned long long c = 0;
    for (int r = blockIdx.y; r < nrows; r += gridDim.y) {
        const int s = srcs ? srcs[r] : src_begin + r;
        const uint32_t* Dr = D + (size_t)r * ldd;
        for (int t = blockIdx.x * 256 + threadIdx.x; t < n; t += gridDim.x * 256) {
            const uint32_t dt = Dr[t];
            if (t == s || dt >= SRT_INF) continue;
            uint32_t best = SRT_INF, cnt = 0;
            const int ke = irp[t + 1];
            for (int k = irp[t]; k < ke; ++k) {
                const int u = icol[k];
                const uint32_t du = u == s ? 0u : Dr[u];
                if (du < SRT_INF && du + iw[k] == dt) {
                    cnt = du < best ? 1u : cnt + (du == best);
                    best = min(best, du);
                }
            }
            c += cnt >= 2;
        }
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

int srt_tie_count_rows(int n, int nrows, const int32_t* srcs, int src_begin, const uint32_t* D,
                       size_t ldd, const int32_t* irp, const int32_t* icol, const uint32_t* iw,
                       int64_t* tied, hipStream_t st) {
    if (nrows <= 0) return SRT_OK;
    unsigned long long* d = NULL;
    SRT_HIPCHK(srt_malloc_async((void**)&d, sizeof(*d), st));
    SRT_HIPCHK(hipMemsetAsync(d, 0, sizeof(*d), st));
    dim3 g((unsigned)(srt_ceil_div(n, 256) < 8 ? srt_ceil_div(n, 256) : 8),
           (unsigned)(nrows < 8192 ? nrows : 8192));
    tie_count_kernel<<<g, 256, 0, st>>>(n, nrows, srcs, src_begin, D, ldd, irp, icol, iw, d);
    SRT_HIPCHK(hipGetLastError());
    unsigned long long h = 0;
    SRT_HIPCHK(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, st));
    SRT_HIPCHK(hipFreeAsync(d, st));
    SRT_HIPCHK(hipStreamSynchronize(st));
    *tied += (int64_t)h;
    return SRT_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* Dense matrices straight from the edge list (the canonical arc rule of graph.c on the device: */
/* per ordered pair the minimum-latency edge, the lowest edge index among equal latencies, both */
/* directions of an undirected edge, self-loops on the diagonal). Rows [row0, row0 + nrows) of  */
/* an ld-wide matrix; the f64 matrix holds the u64 minimum latency and the u32 matrix the edge  */
/* index until srt_scatter_final turns them into quanta and reliabilities in place.            */
/* ------------------------------------------------------------------------------------------ */
__global__ __launch_bounds__(256) void scatter_min_kernel(int64_t m, const int32_t* __restrict__ src,
                                                          const int32_t* __restrict__ dst,
                                                          const int64_t* __restrict__ lat, int directed,
                                                          int32_t row0, uint32_t nrows, int ld,
                                                          unsigned long long* __restrict__ minlat) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (int64_t)gridDim.x * 256) {
        const int32_t u = src[e], v = dst[e];
        const unsigned long long l = (unsigned long long)lat[e];
        if ((uint32_t)(u - row0) < nrows) atomicMin(minlat + (size_t)(u - row0) * ld + v, l);
        if (!directed && u != v && (uint32_t)(v - row0) < nrows)
            atomicMin(minlat + (size_t)(v - row0) * ld + u, l);
    }
}

__global__ __launch_bounds__(256) void scatter_idx_kernel(int64_t m, const int32_t* __restrict__ src,
                                                          const int32_t* __restrict__ dst,
                                                          const int64_t* __restrict__ lat, int directed,
                                                          int32_t row0, uint32_t nrows, int ld,
                                                          const unsigned long long* __restrict__ minlat,
                                                          uint32_t* __restrict__ eidx) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (int64_t)gridDim.x * 256) {
        const int32_t u = src[e], v = dst[e];
        const unsigned long long l = (unsigned long long)lat[e];
        if ((uint32_t)(u - row0) < nrows) {
            const size_t o = (size_t)(u - row0) * ld + v;
            if (minlat[o] == l) atomicMin(eidx + o, (uint32_t)e);
        }
        if (!directed && u != v && (uint32_t)(v - row0) < nrows) {
            const size_t o = (size_t)(v - row0) * ld + u;
            if (minlat[o] == l) atomicMin(eidx + o, (uint32_t)e);
        }
    }
}

__global__ __launch_bounds__(256) void scatter_final_kernel(int32_t row0, int nrows, int ld, uint64_t q,
                                                            const double* __restrict__ loss,
                                                            uint32_t* __restrict__ w, double* __restrict__ r,
                                                            unsigned long long* __restrict__ arcs) {
    const size_t total = (size_t)nrows * ld;
    unsigned long long cnt = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
        const unsigned long long k = __builtin_bit_cast(unsigned long long, r[i]);
        const uint32_t e = w[i];
        if (k == ~0ull) {
            w[i] = SRT_INF;
            r[i] = 0.0;
        } else {
            w[i] = (uint32_t)(k / q);
            r[i] = 1.0f - loss[e]; /* topology.c:396, as graph.c's canonical arcs */
            cnt += (size_t)row0 + i / ld != i % ld;
        }
    }
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(arcs, cnt);
}

int srt_scatter_prepare(int nrows, int ld, uint32_t* w, double* r, hipStream_t st) {
    SRT_HIPCHK(hipMemsetAsync(w, 0xFF, (size_t)nrows * ld * sizeof(uint32_t), st));
    SRT_HIPCHK(hipMemsetAsync(r, 0xFF, (size_t)nrows * ld * sizeof(double), st));
    return SRT_OK;
}

static unsigned scatter_grid(int64_t m) {
    const int64_t b = (m + 255) / 256;
    return (unsigned)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

int srt_scatter_min(int64_t m, const int32_t* src, const int32_t* dst, const int64_t* lat, int directed,
                    int32_t row0, int nrows, int ld, double* r, hipStream_t st) {
    if (m <= 0 || nrows <= 0) return SRT_OK;
    scatter_min_kernel<<<scatter_grid(m), 256, 0, st>>>(m, src, dst, lat, directed, row0, (uint32_t)nrows,
                                                        ld, (unsigned long long*)r);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

int srt_scatter_idx(int64_t m, const int32_t* src, const int32_t* dst, const int64_t* lat, int directed,
                    int32_t row0, int nrows, int ld, const double* r, uint32_t* w, hipStream_t st) {
    if (m <= 0 || nrows <= 0) return SRT_OK;
    scatter_idx_kernel<<<scatter_grid(m), 256, 0, st>>>(m, src, dst, lat, directed, row0, (uint32_t)nrows,
                                                        ld, (const unsigned long long*)r, w);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

int srt_scatter_final(int32_t row0, int nrows, int ld, uint64_t q, const double* loss, uint32_t* w,
                      double* r, unsigned long long* arcs, hipStream_t st) {
    if (nrows <= 0) return SRT_OK;
    const size_t total = (size_t)nrows * ld;
    const size_t b = (total + 255) / 256;
    scatter_final_kernel<<<(unsigned)(b < 8192 ? b : 8192), 256, 0, st>>>(row0, nrows, ld, q, loss, w, r, arcs);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}
