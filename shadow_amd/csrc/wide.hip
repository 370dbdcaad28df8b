/*
 * wide.hip -- shortest-path rows whose distances may pass the u32 tables' range (SRT_INF = 2^31 - 1 quanta), gfx950.
 *
 * The reference keeps path latencies as i64 nanoseconds (units.rs:807-837) and f64 milliseconds
 * (topology.c:294, :1308, :1364), so a graph whose quanta range passes u32 -- a 100k-vertex
 * graph with 1 us quanta and 100 ms edges -- still builds there. Every other kernel here keeps
 * u32 quanta (graph.c proves the bound first); graphs beyond it come here (srt_canon.wide):
 *   1. wide_sssp_kernel: one workgroup of 1,024 threads per source row, u64 distances in HBM,
 *      Bellman-Ford over a frontier bitmap in LDS (a vertex re-enters when its distance drops),
 *      each frontier vertex's arcs spread over one wave's lanes, u64 atomicMin per arc;
 *   2. wide_pred_kernel: the canonical predecessor of every target, argmin (D[s][u], u) over
 *      the tight in-arcs (the rule of every build kernel), and r(pred, t);
 *   3. the path-order passes of tables.hip over those predecessor rows (u64 distances): the
 *      reliability product (topology.c:1365) and the f64-ms latency sum (topology.c:1364);
 *   4. the diagonal rule (sparse.hip, topology.c:1431-1576).
 * The u32 `lat` rows saturate at SRT_INF - 1 = 0x7FFFFFFE quanta for reachable pairs (SRT_INF:
 * unreachable);
 * the f64 ms rows carry the reference's value, so wide tables need them (build.hip refuses a
 * wide graph without them).
 * A fallback for correctness at any range: measured on C5-sized graphs in DESIGN §5.6.
 */
#include "srt_device.h"

#define WD_THREADS 1024
#define WD_INF (~0ull)

int srt_path_rows_u64(int n, int nrows, const int32_t* srcs, int src_begin, const uint64_t* D,
                      size_t ldd, const int32_t* pred, size_t ldp, uint64_t quantum_ns, double* rel,
                      size_t ldr, double* ms, size_t ldm, hipStream_t st);
int srt_sparse_diag(int n, int src_begin, int src_end, const int32_t* srcs, const int32_t* rowptr,
                    const int32_t* col, const uint32_t* w, const double* r, const uint32_t* self_w,
                    const double* self_r, uint32_t* lat, double* rel, size_t ldo, hipStream_t st);

static __device__ __forceinline__ uint64_t ld_dev(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* rows r of [0, nrows): source srcs[r] (or src_begin + r); D row r at D + r * ldd; qws: one
 * n-entry frontier queue per workgroup */
__global__ __launch_bounds__(WD_THREADS) void wide_sssp_kernel(
    int n, const int32_t* __restrict__ rp, const int32_t* __restrict__ col,
    const uint32_t* __restrict__ w, int nrows, const int32_t* __restrict__ srcs, int src_begin,
    uint64_t* __restrict__ D, size_t ldd, int32_t* __restrict__ qws) {
    extern __shared__ uint32_t bm[];
    __shared__ int s_qlen;
    const int nw = (n + 31) >> 5;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int32_t* q = qws + (size_t)blockIdx.x * n;
    for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
        const int s = srcs ? srcs[r] : src_begin + r;
        uint64_t* Dr = D + (size_t)r * ldd;
        uint32_t* cur = bm;
        uint32_t* nxt = bm + nw;
        for (int t = tid; t < n; t += WD_THREADS) Dr[t] = WD_INF;
        for (int i = tid; i < 2 * nw; i += WD_THREADS) bm[i] = 0u;
        __threadfence();
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_store(Dr + s, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            cur[s >> 5] = 1u << (s & 31);
        }
        __threadfence();
        __syncthreads();
        for (;;) {
            /* the frontier as a queue (ballot-free: one LDS atomic per non-empty word) */
            if (tid == 0) s_qlen = 0;
            __syncthreads();
            for (int i = tid; i < nw; i += WD_THREADS) {
                uint32_t bits = cur[i];
                if (!bits) continue;
                cur[i] = 0u;
                int o = atomicAdd(&s_qlen, __popc(bits));
                while (bits) {
                    const int b = __ffs(bits) - 1;
                    bits &= bits - 1u;
                    q[o++] = (i << 5) + b;
                }
            }
            __threadfence_block();
            __syncthreads();
            const int qlen = s_qlen;
            if (qlen == 0) break;
            /* relax: a wave per frontier vertex, its arcs over the lanes */
            for (int i = wv; i < qlen; i += WD_THREADS / 64) {
                const int u = q[i];
                const uint64_t du = ld_dev(Dr + u);
                const int ke = rp[u + 1];
                for (int k = rp[u] + lane; k < ke; k += 64) {
                    const int v = col[k];
                    const uint64_t nd = du + w[k];
                    if (nd < ld_dev(Dr + v)) {
                        const uint64_t old = atomicMin((unsigned long long*)(Dr + v), (unsigned long long)nd);
                        if (nd < old) atomicOr(&nxt[v >> 5], 1u << (v & 31));
                    }
                }
            }
            __threadfence();
            __syncthreads();
            uint32_t* t = cur;
            cur = nxt;
            nxt = t;
        }
        __syncthreads();
    }
}

/* predecessor, r(pred, t) and the saturated u32 row; the diagonal is the caller's */
__global__ __launch_bounds__(256) void wide_pred_kernel(
    int n, int nrows, const int32_t* __restrict__ srcs, int src_begin,
    const uint64_t* __restrict__ D, size_t ldd, const int32_t* __restrict__ irp,
    const int32_t* __restrict__ icol, const uint32_t* __restrict__ iw, const double* __restrict__ ir,
    int32_t* __restrict__ pred, size_t ldp, uint32_t* __restrict__ lat, double* __restrict__ rel,
    size_t ldo) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int r = blockIdx.y;
    if (t >= n || r >= nrows) return;
    const int s = srcs ? srcs[r] : src_begin + r;
    const uint64_t* Dr = D + (size_t)r * ldd;
    const uint64_t dt = Dr[t];
    int bu = -1;
    double br = 0.0;
    if (t != s && dt != WD_INF) {
        uint64_t bd = WD_INF;
        const int ke = irp[t + 1];
        for (int k = irp[t]; k < ke; ++k) {
            const int u = icol[k];
            const uint64_t du = u == s ? 0ull : Dr[u];
            if (du == WD_INF || du + iw[k] != dt) continue;
            if (du < bd || (du == bd && u < bu)) {
                bd = du;
                bu = u;
                br = ir[k];
            }
        }
    }
    pred[(size_t)r * ldp + t] = bu;
    lat[(size_t)r * ldo + t] = dt == WD_INF ? SRT_INF : (dt >= SRT_INF ? SRT_INF - 1u : (uint32_t)dt);
    rel[(size_t)r * ldo + t] = bu >= 0 ? br : 0.0;
}

/* D[r][s] = the diagonal rule's latency (lat[r][s], from srt_sparse_diag), for the ms pass */
__global__ void wide_diag_copy_kernel(int nrows, const int32_t* __restrict__ srcs, int src_begin,
                                      const uint32_t* __restrict__ lat, size_t ldo,
                                      uint64_t* __restrict__ D, size_t ldd) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    const int s = srcs ? srcs[r] : src_begin + r;
    D[(size_t)r * ldd + s] = lat[(size_t)r * ldo + s];
}

int srt_wide_max_n(void) { return (150 * 1024 / 8) * 32; }

/* rows [src_begin, src_end) (or srcs[0 .. src_end - src_begin)) into lat / rel / lms (row
 * stride ldo; lms may be NULL). out-CSR (rp, col, w, r), in-CSR (irp, icol, iw, ir), self arcs. */
int srt_wide_rows(int n, const int32_t* rp, const int32_t* col, const uint32_t* w, const double* r,
                  const int32_t* irp, const int32_t* icol, const uint32_t* iw, const double* ir,
                  const uint32_t* sw, const double* sr, uint64_t quantum_ns, int src_begin,
                  int src_end, const int32_t* srcs, uint32_t* lat, double* rel, double* lms,
                  size_t ldo, hipStream_t st) {
    const int nrows = src_end - src_begin;
    if (nrows <= 0) return SRT_OK;
    if (n > srt_wide_max_n()) {
        srt_set_error("wide-distance rows: n = %d beyond the frontier bitmap range", n);
        return SRT_E_RANGE;
    }
    int cus = 256, dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        cus = prop.multiProcessorCount;
    /* rows per chunk: u64 distances + i32 predecessors, <= 4 GiB of scratch */
    const size_t per_row = (size_t)n * (sizeof(uint64_t) + sizeof(int32_t));
    int chunk = (int)std::min<size_t>((size_t)nrows, std::max<size_t>(1, (4ull << 30) / per_row));
    const int grid = std::min(chunk, 2 * cus);
    uint64_t* D = nullptr;
    int32_t *P = nullptr, *Q = nullptr;
    SRT_HIPCHK(srt_malloc_async((void**)&D, (size_t)chunk * n * sizeof(uint64_t), st));
    SRT_HIPCHK(srt_malloc_async((void**)&P, (size_t)chunk * n * sizeof(int32_t), st));
    SRT_HIPCHK(srt_malloc_async((void**)&Q, (size_t)grid * n * sizeof(int32_t), st));
    const size_t lds = 2 * (size_t)((n + 31) / 32) * sizeof(uint32_t);
    SRT_HIPCHK(hipFuncSetAttribute((const void*)wide_sssp_kernel,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int rc = SRT_OK;
    for (int r0 = 0; r0 < nrows && !rc; r0 += chunk) {
        const int nr = std::min(chunk, nrows - r0);
        const int32_t* cs = srcs ? srcs + r0 : nullptr;
        const int cb = srcs ? 0 : src_begin + r0;
        uint32_t* lo = lat + (size_t)r0 * ldo;
        double* ro = rel + (size_t)r0 * ldo;
        wide_sssp_kernel<<<std::min(nr, grid), WD_THREADS, lds, st>>>(n, rp, col, w, nr, cs, cb, D,
                                                                     (size_t)n, Q);
        SRT_HIPCHK(hipGetLastError());
        wide_pred_kernel<<<dim3(srt_ceil_div(n, 256), nr), 256, 0, st>>>(
            n, nr, cs, cb, D, (size_t)n, irp, icol, iw, ir, P, (size_t)n, lo, ro, ldo);
        SRT_HIPCHK(hipGetLastError());
        /* path-order reliability first (it starts from 1.0 at the source), then the diagonal
         * rule over it, then the ms sums with the diagonal's latency at the source */
        rc = srt_path_rows_u64(n, nr, cs, cb, D, (size_t)n, P, (size_t)n, quantum_ns, ro, ldo,
                               nullptr, 0, st);
        if (!rc)
            rc = srt_sparse_diag(n, cb, cb + nr, cs, rp, col, w, r, sw, sr, lo, ro, ldo, st);
        if (!rc && lms) {
            wide_diag_copy_kernel<<<srt_ceil_div(nr, 256), 256, 0, st>>>(nr, cs, cb, lo, ldo, D,
                                                                        (size_t)n);
            SRT_HIPCHK(hipGetLastError());
            rc = srt_path_rows_u64(n, nr, cs, cb, D, (size_t)n, P, (size_t)n, quantum_ns, nullptr, 0,
                                   lms + (size_t)r0 * ldo, ldo, st);
        }
    }
    (void)hipFreeAsync(Q, st);
    (void)hipFreeAsync(P, st);
    (void)hipFreeAsync(D, st);
    return rc;
}
