/*
 * sparse.hip -- multi-source shortest paths for sparse graphs on gfx950.
 *
 * One workgroup (1024 threads) per source; the whole distance row lives in LDS, so every
 * relaxation is an LDS atomic min (ds_min_u32) and the CSR (shared by all sources) streams from
 * L2. The label-correcting loop is a bucketed frontier Bellman-Ford (delta-stepping style): a
 * bitmap marks improved vertices, each round compacts the "near" ones (dist < threshold) into a
 * queue with wavefront ballots + one LDS atomic per wave, relaxes their arcs, and the threshold
 * advances by delta when the near set drains.
 *
 * After the distances settle, the same workgroup computes the canonical predecessor of every
 * target (argmin (D[s][u], u) over tight in-arcs) and the path-order reliability
 * rel(s,t) = rel(s,pred) * r(pred,t) by a breadth-first walk down the predecessor tree
 * (children of v are found among v's out-arcs), i.e. the product is formed in exactly the order
 * /root/reference/src/main/routing/topology.c:1342-1366 forms it.
 *
 * Working-set layout (bytes): [A: 4n] dist during SSSP/pred, two frontier bitmaps during the tree
 * walk; [Bq: 4n] near queue during SSSP, predecessor arc index afterwards; [C: n/8] improved
 * bitmap. For n <= srt_sparse_max_n() (~20k) it is LDS (one workgroup per CU); beyond that the
 * same layout lives in a per-workgroup slot of an HBM workspace and the grid is persistent
 * (2 workgroups per CU, each looping over sources), with every relaxation an L2 atomic. All
 * threads of a workgroup share one CU and its L1, so workgroup barriers order the slot's
 * global-memory traffic exactly as they order LDS.
 */
#include "srt_device.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#define SP_THREADS 1024
#define SP_WAVES (SP_THREADS / 64)

static __device__ __forceinline__ int wave_excl_scan(int v, int lane, int* total) {
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    *total = __shfl(x, 63);
    return x - v;
}

template <bool G>
__global__ __launch_bounds__(SP_THREADS) void sssp_kernel(
    int n, int src_begin, const int32_t* __restrict__ srcs, int nsrc, uint32_t delta,
    const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, const uint32_t* __restrict__ w,
    const int32_t* __restrict__ in_rowptr, const int32_t* __restrict__ in_col,
    const uint32_t* __restrict__ in_w, const double* __restrict__ in_r, uint32_t* __restrict__ lat,
    double* __restrict__ rel, size_t ldo, int32_t* __restrict__ max_depth, uint32_t* ws,
    size_t slot_words) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int nwords = (n + 31) >> 5;
    const int a_words = n > 2 * nwords ? n : 2 * nwords;
    uint32_t* base = G ? ws + (size_t)blockIdx.x * slot_words : smem;
    uint32_t* dist = base;                                     /* region A */
    uint32_t* queue = base + a_words;                          /* region B */
    int32_t* arc = reinterpret_cast<int32_t*>(base + a_words); /* region B after SSSP */
    uint32_t* bits = base + a_words + n;                       /* region C */
    __shared__ int s_qlen;
    __shared__ uint32_t s_minfar;
    __shared__ int s_any;
    const int tid = threadIdx.x, lane = tid & 63;
    int depth = 0;
  for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
    const int s = srcs ? srcs[si] : src_begin + si;
    __syncthreads(); /* the previous source's walk is done with the working set */
    for (int v = tid; v < n; v += SP_THREADS) dist[v] = SRT_INF;
    for (int q = tid; q < nwords; q += SP_THREADS) bits[q] = 0;
    __syncthreads();
    if (tid == 0) {
        dist[s] = 0;
        bits[s >> 5] = 1u << (s & 31);
    }
    uint32_t thr = delta;
    for (;;) {
        if (tid == 0) {
            s_qlen = 0;
            s_minfar = SRT_INF;
        }
        __syncthreads();
        /* compact the near set (dist < thr) of improved vertices into the queue */
        uint32_t myfar = SRT_INF;
        for (int q0 = 0; q0 < nwords; q0 += SP_THREADS) {
            const int q = q0 + tid;
            uint32_t word = q < nwords ? bits[q] : 0u, near = 0u;
            uint32_t x = word;
            while (x) {
                const int b = __ffs(x) - 1;
                x &= x - 1;
                const uint32_t dv = dist[(q << 5) + b];
                if (dv < thr)
                    near |= 1u << b;
                else
                    myfar = min(myfar, dv);
            }
            if (near) bits[q] = word & ~near;
            const int c = __popc(near);
            int tot;
            const int pre = wave_excl_scan(c, lane, &tot);
            int base = 0;
            if (lane == 0 && tot) base = atomicAdd(&s_qlen, tot);
            base = __shfl(base, 0);
            int o = base + pre;
            while (near) {
                const int b = __ffs(near) - 1;
                near &= near - 1;
                queue[o++] = (uint32_t)((q << 5) + b);
            }
        }
        /* wave min of the far distances, one LDS atomic per wave */
        for (int off = 32; off > 0; off >>= 1) myfar = min(myfar, (uint32_t)__shfl_xor((int)myfar, off));
        if (lane == 0 && myfar < SRT_INF) atomicMin(&s_minfar, myfar);
        __syncthreads();
        const int qlen = s_qlen;
        if (qlen == 0) {
            const uint32_t mf = s_minfar;
            if (mf >= SRT_INF) break;
            thr = mf + delta;
            __syncthreads();
            continue;
        }
        /* relax the out-arcs of the near set */
        for (int i = tid; i < qlen; i += SP_THREADS) {
            const int v = (int)queue[i];
            const uint32_t dv = dist[v];
            const int kb = rowptr[v], ke = rowptr[v + 1];
            for (int k = kb; k < ke; ++k) {
                const int u = col[k];
                const uint32_t nd = dv + w[k];
                if (nd < dist[u]) {
                    const uint32_t old = atomicMin(&dist[u], nd);
                    if (nd < old) atomicOr(&bits[u >> 5], 1u << (u & 31));
                }
            }
        }
        __syncthreads();
    }
    __syncthreads();
    /* latency row + canonical predecessor arc of every target */
    uint32_t* latrow = lat + (size_t)si * ldo;
    for (int t = tid; t < n; t += SP_THREADS) {
        const uint32_t dt = dist[t];
        latrow[t] = (t == s) ? 0u : dt;
        int bk = -1;
        if (t != s && dt < SRT_INF) {
            uint64_t best = ~0ull;
            const int kb = in_rowptr[t], ke = in_rowptr[t + 1];
            for (int k = kb; k < ke; ++k) {
                const int u = in_col[k];
                const uint32_t du = dist[u];
                if (du < SRT_INF && du + in_w[k] == dt) {
                    const uint64_t key = ((uint64_t)du << 32) | (uint32_t)u;
                    if (key < best) {
                        best = key;
                        bk = k;
                    }
                }
            }
        }
        arc[t] = bk;
    }
    __syncthreads();
    /* breadth-first walk down the predecessor tree; frontier bitmaps reuse region A */
    uint32_t* cur = base;
    uint32_t* nxt = base + nwords;
    double* relrow = rel + (size_t)si * ldo;
    for (int t = tid; t < n; t += SP_THREADS) relrow[t] = (t == s) ? 1.0 : 0.0;
    for (int q = tid; q < 2 * nwords; q += SP_THREADS) base[q] = 0u;
    __syncthreads();
    if (tid == 0) cur[s >> 5] = 1u << (s & 31);
    __syncthreads();
    int sdepth = 0;
    for (;;) {
        if (tid == 0) s_any = 0;
        __syncthreads();
        int any = 0;
        for (int q = tid; q < nwords; q += SP_THREADS) {
            uint32_t x = cur[q];
            if (!x) continue;
            cur[q] = 0u;
            while (x) {
                const int b = __ffs(x) - 1;
                x &= x - 1;
                const int v = (q << 5) + b;
                const double rv = __hip_atomic_load(relrow + v, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP);
                const int kb = rowptr[v], ke = rowptr[v + 1];
                for (int k = kb; k < ke; ++k) {
                    const int u = col[k];
                    const int a = arc[u];
                    if (a >= 0 && in_col[a] == v) {
                        __hip_atomic_store(relrow + u, rv * in_r[a], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                        atomicOr(&nxt[u >> 5], 1u << (u & 31));
                        any = 1;
                    }
                }
            }
        }
        if (any) s_any = 1;
        __syncthreads();
        if (!s_any) break;
        ++sdepth;
        uint32_t* t = cur;
        cur = nxt;
        nxt = t;
        __syncthreads();
    }
    depth = max(depth, sdepth);
  }
    if (tid == 0) srt_max_once(max_depth, depth);
}

/* Diagonal rule (topology.c:1431-1576) from the canonical CSR: min over (self-loop L, v) and
 * (2L, u) for out-arcs (v,u), first strict minimum in neighbor order. */
__global__ void sparse_diag_kernel(int n, int src_begin, int src_end, const int32_t* __restrict__ srcs,
                                   const int32_t* __restrict__ rowptr,
                                   const int32_t* __restrict__ col, const uint32_t* __restrict__ w,
                                   const double* __restrict__ r, const uint32_t* __restrict__ self_w,
                                   const double* __restrict__ self_r, uint32_t* __restrict__ lat,
                                   double* __restrict__ rel, size_t ldo) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= src_end - src_begin) return;
    const int v = srcs ? srcs[i] : src_begin + i;
    uint64_t best = ~0ull;
    int bk = -2;
    if (self_w[v] < SRT_INF) {
        best = ((uint64_t)self_w[v] << 32) | (uint32_t)v;
        bk = -1;
    }
    for (int k = rowptr[v]; k < rowptr[v + 1]; ++k) {
        const uint64_t key = ((2ull * w[k]) << 32) | (uint32_t)col[k];
        if (key < best) {
            best = key;
            bk = k;
        }
    }
    const size_t ix = (size_t)i * ldo + v;
    if (bk == -2) {
        lat[ix] = 0;
        rel[ix] = 0.0;
    } else if (bk == -1) {
        lat[ix] = self_w[v];
        rel[ix] = self_r[v];
    } else {
        lat[ix] = 2u * w[bk];
        rel[ix] = r[bk] * r[bk];
    }
}

/* host wrapper so the wave-per-source kernel (wsssp.hip) shares the diagonal rule */
int srt_sparse_diag(int n, int src_begin, int src_end, const int32_t* srcs, const int32_t* rowptr,
                    const int32_t* col, const uint32_t* w, const double* r, const uint32_t* self_w,
                    const double* self_r, uint32_t* lat, double* rel, size_t ldo, hipStream_t st) {
    sparse_diag_kernel<<<srt_ceil_div(src_end - src_begin, 256), 256, 0, st>>>(
        n, src_begin, src_end, srcs, rowptr, col, w, r, self_w, self_r, lat, rel, ldo);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

size_t srt_sparse_lds_bytes(int n) {
    const int nwords = (n + 31) / 32;
    const int a_words = n > 2 * nwords ? n : 2 * nwords;
    return (size_t)4 * ((size_t)a_words + n + nwords);
}

int srt_sparse_max_n(void) {
    /* 8n + n/8 bytes (+ the static LDS of the kernel) must fit the 160 KiB LDS */
    return (160 * 1024 - 256) * 8 / 65;
}

/* rows of sources srcs[0 .. src_end - src_begin) (device list), or of [src_begin, src_end) when
 * srcs is NULL */
int srt_sparse_block_rows(int32_t n, const int32_t* rowptr, const int32_t* col, const uint32_t* w,
                          const double* r, const int32_t* in_rowptr, const int32_t* in_col,
                          const uint32_t* in_w, const double* in_r, const uint32_t* self_w,
                          const double* self_r, int32_t src_begin, int32_t src_end,
                          const int32_t* srcs, uint32_t delta, uint32_t* lat_rows,
                          double* rel_rows, void* stream, srt_build_stats* stats) {
    if (n <= 0 || src_begin < 0 || (!srcs && src_end > n) || src_begin >= src_end || !rowptr || !col || !w ||
        !r || !in_rowptr || !in_col || !in_w || !in_r || !self_w || !self_r || !lat_rows ||
        !rel_rows) {
        srt_set_error("srt_sparse_build_device: bad arguments");
        return SRT_E_ARG;
    }
    hipStream_t st = (hipStream_t)stream;
    /* the depth counter and events, released on every return path */
    struct guard_t {
        int32_t* depth = nullptr;
        hipEvent_t e[3] = {nullptr, nullptr, nullptr};
        ~guard_t() {
            if (depth) (void)hipFree(depth);
            for (hipEvent_t x : e)
                if (x) (void)hipEventDestroy(x);
        }
    } g;
    SRT_HIPCHK(hipMalloc(&g.depth, sizeof(int32_t)));
    int32_t* depth = g.depth;
    SRT_HIPCHK(hipMemsetAsync(depth, 0, sizeof(int32_t), st));
    for (hipEvent_t& x : g.e) SRT_HIPCHK(hipEventCreate(&x));
    hipEvent_t e0 = g.e[0], e1 = g.e[1], ek = g.e[2];
    SRT_HIPCHK(hipEventRecord(e0, st));
    if (delta == 0) delta = 8; /* bucket width of the label-correcting loop, in quanta */
    const size_t ldo = (size_t)n;
    const int nsrc = src_end - src_begin;
    if (n <= srt_sparse_max_n()) {
        const size_t lds = srt_sparse_lds_bytes(n);
        SRT_HIPCHK(hipFuncSetAttribute((const void*)sssp_kernel<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        sssp_kernel<false><<<nsrc, SP_THREADS, lds, st>>>(n, src_begin, srcs, nsrc, delta, rowptr, col, w,
                                                          in_rowptr, in_col, in_w, in_r, lat_rows,
                                                          rel_rows, ldo, depth, NULL, 0);
    } else {
        int cus = 256;
        hipDeviceProp_t prop;
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
            cus = prop.multiProcessorCount;
        const int slots = std::min(nsrc, 2 * cus);
        const size_t slot_words = srt_sparse_lds_bytes(n) / 4 + 64; /* 256-B separated slots */
        uint32_t* ws = NULL;
        if (srt_malloc_async((void**)&ws, (size_t)slots * slot_words * 4, st) != hipSuccess) {
            (void)hipGetLastError();
            srt_set_error("srt_sparse_build_device: workspace of %zu MiB failed",
                          (size_t)slots * slot_words * 4 >> 20);
            return SRT_E_NOMEM;
        }
        sssp_kernel<true><<<slots, SP_THREADS, 0, st>>>(n, src_begin, srcs, nsrc, delta, rowptr, col, w,
                                                        in_rowptr, in_col, in_w, in_r, lat_rows,
                                                        rel_rows, ldo, depth, ws, slot_words);
        SRT_HIPCHK(hipFreeAsync(ws, st));
    }
    SRT_HIPCHK(hipGetLastError());
    SRT_HIPCHK(hipEventRecord(ek, st)); /* end of the SSSP kernel (the dominant launch) */
    sparse_diag_kernel<<<srt_ceil_div(src_end - src_begin, 256), 256, 0, st>>>(
        n, src_begin, src_end, srcs, rowptr, col, w, r, self_w, self_r, lat_rows, rel_rows, ldo);
    SRT_HIPCHK(hipGetLastError());
    SRT_HIPCHK(hipEventRecord(e1, st));
    SRT_HIPCHK(hipEventSynchronize(e1));
    float ms = 0, msk = 0;
    SRT_HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    SRT_HIPCHK(hipEventElapsedTime(&msk, e0, ek));
    int32_t dmax = 0;
    SRT_HIPCHK(hipMemcpy(&dmax, depth, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (stats) {
        stats->algo = SRT_ALGO_SPARSE_SSSP;
        stats->ms_fw = ms;
        stats->ms_total = ms;
        stats->max_depth = dmax;
        stats->n_update = 1;
        stats->ms_update = msk;
    }
    return SRT_OK;
}

extern "C" int srt_sparse_build_device(int32_t n, int32_t directed, const int32_t* rowptr,
                                       const int32_t* col, const uint32_t* w, const double* r,
                                       const int32_t* in_rowptr, const int32_t* in_col,
                                       const uint32_t* in_w, const double* in_r,
                                       const uint32_t* self_w, const double* self_r,
                                       int32_t src_begin, int32_t src_end, uint32_t delta,
                                       uint32_t* lat_rows, double* rel_rows, void* stream,
                                       srt_build_stats* stats) {
    (void)directed;
    return srt_sparse_block_rows(n, rowptr, col, w, r, in_rowptr, in_col, in_w, in_r, self_w, self_r,
                                 src_begin, src_end, NULL, delta, lat_rows, rel_rows, stream, stats);
}
