/*
 * dense.hip -- dense all-pairs build for gfx950: blocked min-plus Floyd-Warshall with LDS tiles,
 * then the canonical-predecessor / path-order reliability pass and the diagonal rule. Every
 * source row is its own (the lookup layer picks which row serves a pair, pairorder.c).
 *
 * Reference semantics (/root/reference/src/main/routing/topology.c):
 *   distances      Dijkstra per source (:1682) -> here FW over integer latency quanta
 *   predecessor    first-settled tight in-edge -> canonical argmin (D[s][u], u) over tight (u,t)
 *   reliability    product of (1 - loss) in path order from the source (:1308-1309, :1365)
 *   pair cache     the first source run serves a pair (:1194-1199) -> raw rows + pairorder.c
 *   diagonal       shortest path to self (:1431-1576)
 *
 * Layout: every matrix is ld x ld row-major (ld % 64 == 0, rows/cols >= n are padding),
 * distances u32 quanta with SRT_INF = 0x7FFFFFFF (a + b never wraps: both operands <= INF),
 * reliabilities f64. No MFMA: min-plus is not an FMA contraction; the hot loop is
 * v_add_u32 + v_min3_u32 over 4x4 register blocks fed by ds_read_b128 from LDS.
 */
#include "srt_device.h"

evpool_t* srt_evpool(int slot) {
    static evpool_t pools[SRT_STATE_SLOTS];
    return &pools[slot % SRT_STATE_SLOTS];
}

#define B SRT_FW_B
#define LDT SRT_FW_LDT

/* ------------------------------------------------------------------------------------------ */
/* synthetic complete graph (SURVEY.md §8d C1/C2/C4 generators)                               */
/* ------------------------------------------------------------------------------------------ */
__global__ void gen_complete_kernel(int n, int ld, int row0, uint64_t seed, uint32_t lat_max,
                                    uint32_t self_max, uint32_t loss_max, uint32_t* __restrict__ w,
                                    double* __restrict__ r) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = row0 + blockIdx.y;
    if (j >= ld) return;
    size_t ix = (size_t)blockIdx.y * ld + j;
    if (i >= n || j >= n) {
        w[ix] = SRT_INF;
        r[ix] = 0.0;
        return;
    }
    uint32_t a = i < j ? i : j, b = i < j ? j : i;
    uint32_t lat, k;
    if (a == b) {
        lat = 1u + (uint32_t)(srt_hash(seed, 2, a, a) % self_max);
        k = (uint32_t)(srt_hash(seed, 3, a, a) % (loss_max + 1u));
    } else {
        lat = 1u + (uint32_t)(srt_hash(seed, 0, a, b) % lat_max);
        k = (uint32_t)(srt_hash(seed, 1, a, b) % (loss_max + 1u));
    }
    w[ix] = lat;
    double loss = (double)k / 10000.0;
    r[ix] = 1.0 - loss;
}

extern "C" int srt_gen_complete_device(int32_t n, int32_t ld, int32_t row0, int32_t nrows,
                                       uint64_t seed, uint32_t lat_max_ms, uint32_t self_max_ms,
                                       uint32_t loss_max_e4, uint32_t* w, double* r, void* stream) {
    if (n <= 0 || ld < n || ld % B || !w || !r || lat_max_ms == 0 || self_max_ms == 0 ||
        row0 < 0 || nrows < 0 || row0 + nrows > ld) {
        srt_set_error("srt_gen_complete_device: bad arguments");
        return SRT_E_ARG;
    }
    if (nrows == 0) return SRT_OK;
    dim3 grid(srt_ceil_div(ld, 256), nrows);
    gen_complete_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(n, ld, row0, seed, lat_max_ms,
                                                               self_max_ms, loss_max_e4, w, r);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

/* The metric complete graph (bench workload c4metric; oracle/oracle.c metric_lat restates it):
 * point i at 16-bit grid coordinates of the unit square from the counter hash, latency
 * max(1, round(scale * dist)) ms with the rounding settled in exact integers (a double estimate,
 * corrected against ((2L - 1) 2^15)^2 <= scale^2 d2), loss and self-loops as gen_complete_kernel.
 * Distances reach hundreds of quanta: past the level budget, the FW builds it (Tor-atlas regime). */
static __device__ __forceinline__ uint32_t metric_coord(uint64_t seed, uint32_t i, int axis) {
    return (uint32_t)(srt_hash(seed, 0, i, 0xFFFFFFFFu - (uint32_t)axis) & 0xFFFFu);
}
__global__ void gen_metric_kernel(int n, int ld, int row0, uint64_t seed, uint32_t scale,
                                  uint32_t self_max, uint32_t loss_max, uint32_t* __restrict__ w,
                                  double* __restrict__ r) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = row0 + blockIdx.y;
    if (j >= ld) return;
    const size_t ix = (size_t)blockIdx.y * ld + j;
    if (i >= n || j >= n) {
        w[ix] = SRT_INF;
        r[ix] = 0.0;
        return;
    }
    const uint32_t a = i < j ? i : j, b = i < j ? j : i;
    uint32_t lat, k;
    if (a == b) {
        lat = 1u + (uint32_t)(srt_hash(seed, 2, a, a) % self_max);
        k = (uint32_t)(srt_hash(seed, 3, a, a) % (loss_max + 1u));
    } else {
        const int64_t dx = (int64_t)metric_coord(seed, a, 0) - metric_coord(seed, b, 0);
        const int64_t dy = (int64_t)metric_coord(seed, a, 1) - metric_coord(seed, b, 1);
        const uint64_t d2 = (uint64_t)(dx * dx + dy * dy);
        const uint64_t A = (uint64_t)scale * scale * d2;
        uint64_t L = (uint64_t)((double)scale * sqrt((double)d2) / 65536.0 + 0.5);
        auto f = [](uint64_t x) { return ((2ull * x - 1ull) << 15) * ((2ull * x - 1ull) << 15); };
        while (L > 0 && f(L) > A) L--;
        while (f(L + 1) <= A) L++;
        lat = L > 0 ? (uint32_t)L : 1u;
        k = (uint32_t)(srt_hash(seed, 1, a, b) % (loss_max + 1u));
    }
    w[ix] = lat;
    r[ix] = 1.0 - (double)k / 10000.0;
}

extern "C" int srt_gen_metric_device(int32_t n, int32_t ld, int32_t row0, int32_t nrows,
                                     uint64_t seed, uint32_t scale_ms, uint32_t self_max_ms,
                                     uint32_t loss_max_e4, uint32_t* w, double* r, void* stream) {
    if (n <= 0 || n > 65535 || ld < n || ld % B || !w || !r || scale_ms == 0 || scale_ms > 1024 ||
        self_max_ms == 0 || row0 < 0 || nrows < 0 || row0 + nrows > ld) {
        srt_set_error("srt_gen_metric_device: bad arguments");
        return SRT_E_ARG;
    }
    if (nrows == 0) return SRT_OK;
    dim3 grid(srt_ceil_div(ld, 256), nrows);
    gen_metric_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(n, ld, row0, seed, scale_ms,
                                                             self_max_ms, loss_max_e4, w, r);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* D <- W with a zero diagonal and INF padding                                                */
/* ------------------------------------------------------------------------------------------ */
__global__ void init_dist_kernel(int n, int ld, int row0, const uint32_t* __restrict__ w,
                                 uint32_t* __restrict__ d) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = row0 + blockIdx.y; /* global row */
    if (j >= ld) return;
    size_t ix = (size_t)blockIdx.y * ld + j;
    uint32_t v = (i < n && j < n) ? w[ix] : SRT_INF;
    if (v > SRT_INF) v = SRT_INF;
    d[ix] = (i == j) ? 0u : v;
}

/* ------------------------------------------------------------------------------------------ */
/* 64x64x64 min-plus tile product: C = min(C, A (x) Bm), 256 threads, 4x4 outputs per thread. */
/* A is staged transposed (At[m][row]) so a thread's 4 rows are one ds_read_b128, Bm row-major. */
/* ------------------------------------------------------------------------------------------ */
__device__ __forceinline__ void stage_tile(uint32_t* __restrict__ s, const uint32_t* __restrict__ g,
                                           int ldg, int tid) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        int idx = tid + it * 256; /* 1024 uint4 = 64 rows x 16 */
        int row = idx >> 4, c4 = (idx & 15) << 2;
        uint4 v = *reinterpret_cast<const uint4*>(g + (size_t)row * ldg + c4);
        *reinterpret_cast<uint4*>(s + row * LDT + c4) = v;
    }
}

__device__ __forceinline__ void stage_tile_T(uint32_t* __restrict__ s, const uint32_t* __restrict__ g,
                                             int ldg, int tid) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        int idx = tid + it * 256;
        int row = idx >> 4, c4 = (idx & 15) << 2;
        uint4 v = *reinterpret_cast<const uint4*>(g + (size_t)row * ldg + c4);
        s[(c4 + 0) * LDT + row] = v.x;
        s[(c4 + 1) * LDT + row] = v.y;
        s[(c4 + 2) * LDT + row] = v.z;
        s[(c4 + 3) * LDT + row] = v.w;
    }
}

__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) {
    return min(a, min(b, c));
}

/* acc (4x4 in registers) <- min(acc, sAt (x) sB); LDS already staged and synchronized. */
__device__ __forceinline__ void minplus_acc(uint32_t (&acc)[4][4], const uint32_t* __restrict__ sAt,
                                            const uint32_t* __restrict__ sB, int tx, int ty) {
#pragma unroll 8
    for (int m = 0; m < B; m += 2) {
        uint4 a0 = *reinterpret_cast<const uint4*>(sAt + m * LDT + 4 * ty);
        uint4 b0 = *reinterpret_cast<const uint4*>(sB + m * LDT + 4 * tx);
        uint4 a1 = *reinterpret_cast<const uint4*>(sAt + (m + 1) * LDT + 4 * ty);
        uint4 b1 = *reinterpret_cast<const uint4*>(sB + (m + 1) * LDT + 4 * tx);
        const uint32_t av0[4] = {a0.x, a0.y, a0.z, a0.w};
        const uint32_t bv0[4] = {b0.x, b0.y, b0.z, b0.w};
        const uint32_t av1[4] = {a1.x, a1.y, a1.z, a1.w};
        const uint32_t bv1[4] = {b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
                acc[a][b] = umin3(acc[a][b], av0[a] + bv0[b], av1[a] + bv1[b]);
    }
}

__device__ __forceinline__ void load_acc(uint32_t (&acc)[4][4], const uint32_t* __restrict__ C,
                                         int ldc, int tx, int ty) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        uint4 v = *reinterpret_cast<const uint4*>(C + (size_t)(4 * ty + a) * ldc + 4 * tx);
        acc[a][0] = v.x;
        acc[a][1] = v.y;
        acc[a][2] = v.z;
        acc[a][3] = v.w;
    }
}

/* store only the 16-byte rows that changed: unchanged tiles cost no HBM write */
__device__ __forceinline__ void store_acc(const uint32_t (&acc)[4][4], const uint32_t (&old)[4][4],
                                          uint32_t* __restrict__ C, int ldc, int tx, int ty) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        uint4* p = reinterpret_cast<uint4*>(C + (size_t)(4 * ty + a) * ldc + 4 * tx);
        if (old[a][0] != acc[a][0] || old[a][1] != acc[a][1] || old[a][2] != acc[a][2] ||
            old[a][3] != acc[a][3])
            *p = make_uint4(acc[a][0], acc[a][1], acc[a][2], acc[a][3]);
    }
}

/* Phase 1: closure of the diagonal tile (pivots kB..kB+63), in LDS, one workgroup. */
__global__ __launch_bounds__(256) void fw_diag_kernel(uint32_t* __restrict__ P, int ld, int k0) {
    __shared__ __attribute__((aligned(16))) uint32_t s[B * LDT];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    uint32_t* T = P + k0;
    stage_tile(s, T, ld, tid);
    __syncthreads();
    for (int m = 0; m < B; ++m) {
        uint4 bm = *reinterpret_cast<const uint4*>(s + m * LDT + 4 * tx);
        uint32_t am[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) am[a] = s[(4 * ty + a) * LDT + m];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            uint4* row = reinterpret_cast<uint4*>(s + (4 * ty + a) * LDT + 4 * tx);
            uint4 v = *row;
            v.x = min(v.x, am[a] + bm.x);
            v.y = min(v.y, am[a] + bm.y);
            v.z = min(v.z, am[a] + bm.z);
            v.w = min(v.w, am[a] + bm.w);
            *row = v;
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        uint4 v = *reinterpret_cast<const uint4*>(s + (4 * ty + a) * LDT + 4 * tx);
        *reinterpret_cast<uint4*>(T + (size_t)(4 * ty + a) * ld + 4 * tx) = v;
    }
}

/* Phase 2: pivot-row panel tiles (k, j): X <- Dkk* (x) X, and pivot-column tiles (i, k):
 * X <- X (x) Dkk*. P = the B x ld pivot-row panel (closed diagonal tile at column k0).
 * D holds `nrow_tiles` local row tiles whose first global row is row0. */
__global__ __launch_bounds__(256) void fw_panel_kernel(uint32_t* __restrict__ D, int ld, int row0,
                                                       int nrow_tiles, uint32_t* __restrict__ P,
                                                       int k0, int ncol_tiles, int do_row,
                                                       int do_col) {
    __shared__ __attribute__((aligned(16))) uint32_t sA[B * LDT];
    __shared__ __attribute__((aligned(16))) uint32_t sB[B * LDT];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    int bid = blockIdx.x;
    uint32_t* C;
    if (bid < ncol_tiles) {
        if (!do_row || bid * B == k0) return;
        C = P + bid * B;
        stage_tile_T(sA, P + k0, ld, tid); /* Dkk* */
        stage_tile(sB, C, ld, tid);
    } else {
        bid -= ncol_tiles;
        if (!do_col || bid >= nrow_tiles || row0 + bid * B == k0) return;
        C = D + (size_t)bid * B * ld + k0;
        stage_tile_T(sA, C, ld, tid);
        stage_tile(sB, P + k0, ld, tid);
    }
    __syncthreads();
    uint32_t acc[4][4], old[4][4];
    load_acc(old, C, ld, tx, ty);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = old[a][b];
    minplus_acc(acc, sA, sB, tx, ty);
    store_acc(acc, old, C, ld, tx, ty);
}

/* Phase 3: every other tile (i, j): D_ij <- min(D_ij, D_ik (x) P_kj). */
__global__ __launch_bounds__(256) void fw_update_kernel(uint32_t* __restrict__ D, int ld, int row0,
                                                        const uint32_t* __restrict__ P, int k0) {
    __shared__ __attribute__((aligned(16))) uint32_t sA[B * LDT];
    __shared__ __attribute__((aligned(16))) uint32_t sB[B * LDT];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int J = blockIdx.x, I = blockIdx.y;
    if (J * B == k0 || row0 + I * B == k0) return;
    uint32_t* C = D + (size_t)I * B * ld + J * B;
    stage_tile_T(sA, D + (size_t)I * B * ld + k0, ld, tid);
    stage_tile(sB, P + J * B, ld, tid);
    __syncthreads();
    uint32_t acc[4][4], old[4][4];
    load_acc(old, C, ld, tx, ty);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = old[a][b];
    minplus_acc(acc, sA, sB, tx, ty);
    store_acc(acc, old, C, ld, tx, ty);
}

/* One FW round on a row shard. P is the B x ld pivot-row panel: in place (D + (k0-row0)*ld) on
 * the rank that owns rows [k0, k0+B), a received copy elsewhere. The owner part (diagonal closure
 * + row panel) must finish before the panel is broadcast; the rest runs on every rank. */
static int fw_owner_part(uint32_t* D, int ld, int row0, int nrows, uint32_t* P, int k0,
                         hipStream_t st) {
    const int nb = ld / B, nrb = nrows / B;
    fw_diag_kernel<<<1, 256, 0, st>>>(P, ld, k0);
    fw_panel_kernel<<<nb, 256, 0, st>>>(D, ld, row0, nrb, P, k0, nb, 1, 0);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

static int fw_shard_part(uint32_t* D, int ld, int row0, int nrows, const uint32_t* P, int k0,
                         hipStream_t st, evpool_t* evp) {
    const int nb = ld / B, nrb = nrows / B;
    if (nrb == 0) return SRT_OK;
    fw_panel_kernel<<<nb + nrb, 256, 0, st>>>(D, ld, row0, nrb, (uint32_t*)P, k0, nb, 0, 1);
    if (evp) SRT_HIPCHK(hipEventRecord(evp->ev[evp->used++], st));
    fw_update_kernel<<<dim3(nb, nrb), 256, 0, st>>>(D, ld, row0, P, k0);
    if (evp) SRT_HIPCHK(hipEventRecord(evp->ev[evp->used++], st));
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

int srt_dense_fw_device(int32_t n, int32_t ld, uint32_t* d, hipStream_t st, evpool_t* evp) {
    (void)n;
    for (int k0 = 0; k0 < ld; k0 += B) {
        uint32_t* P = d + (size_t)k0 * ld;
        int rc = fw_owner_part(d, ld, 0, ld, P, k0, st);
        if (!rc) rc = fw_shard_part(d, ld, 0, ld, P, k0, st, evp);
        if (rc) return rc;
    }
    return SRT_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* Essential arcs: (u,t) with W[u][t] == D[u][t] (u != t). Every tight predecessor of any      */
/* (s,t) is essential: D[s][u] + W[u][t] = D[s][t] <= D[s][u] + D[u][t] forces D[u][t] = W.    */
/* Rows are local (global row = row0 + blockIdx.x); counts go to cnt[global row].            */
/* ------------------------------------------------------------------------------------------ */
/* four consecutive distances (u32 table, or the exact u16 FW matrix: half the bytes) */
static __device__ __forceinline__ uint4 ld_d4(const uint32_t* p) {
    return *reinterpret_cast<const uint4*>(p);
}
static __device__ __forceinline__ uint4 ld_d4(const uint16_t* p) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    return make_uint4(v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16);
}

template <typename DT>
__global__ __launch_bounds__(256) void ess_count_kernel(int n, int ld, int row0,
                                                        const uint32_t* __restrict__ w,
                                                        const DT* __restrict__ d,
                                                        int32_t* __restrict__ cnt) {
    const int u = row0 + blockIdx.x;
    if (u >= n) return;
    const uint32_t* wr = w + (size_t)blockIdx.x * ld;
    const DT* dr = d + (size_t)blockIdx.x * ld;
    int c = 0;
    const int n4 = n & ~3; /* rows are 16-B aligned (ld % 64 == 0): 4 columns per load */
    for (int t = threadIdx.x * 4; t < n4; t += blockDim.x * 4) {
        const uint4 x = *reinterpret_cast<const uint4*>(wr + t);
        const uint4 y = ld_d4(dr + t);
        c += (t != u && x.x < SRT_INF && x.x == y.x) + (t + 1 != u && x.y < SRT_INF && x.y == y.y) +
             (t + 2 != u && x.z < SRT_INF && x.z == y.z) + (t + 3 != u && x.w < SRT_INF && x.w == y.w);
    }
    for (int t = n4 + threadIdx.x; t < n; t += blockDim.x) {
        uint32_t x = wr[t];
        c += (t != u && x < SRT_INF && x == (uint32_t)dr[t]) ? 1 : 0;
    }
    __shared__ int red[256];
    red[threadIdx.x] = c;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) cnt[u] = red[0];
}

/* exclusive scan of cnt[0..n) into ptr[0..n], one workgroup of 1024 threads */
__global__ __launch_bounds__(1024) void scan_kernel(int n, const int32_t* __restrict__ cnt,
                                                    int32_t* __restrict__ ptr) {
    __shared__ int64_t part[1024];
    const int tid = threadIdx.x;
    const int chunk = (n + 1023) / 1024;
    const int b = tid * chunk, e = min(n, b + chunk);
    int64_t s = 0;
    for (int i = b; i < e; ++i) s += cnt[i];
    part[tid] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        int64_t v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int64_t run = part[tid] - s;
    for (int i = b; i < e; ++i) {
        ptr[i] = (int32_t)run;
        run += cnt[i];
    }
    if (tid == 1023) ptr[n] = (int32_t)part[1023];
}

/* fill essential out-arcs of local row u at ptr[u], ascending t (wave ballot compaction) */
template <typename DT>
__global__ __launch_bounds__(256) void ess_fill_kernel(int n, int ld, int row0,
                                                       const uint32_t* __restrict__ w,
                                                       const double* __restrict__ r,
                                                       const DT* __restrict__ d,
                                                       const int32_t* __restrict__ ptr,
                                                       int32_t* __restrict__ col,
                                                       uint32_t* __restrict__ aw,
                                                       double* __restrict__ ar) {
    const int u = row0 + blockIdx.x;
    if (u >= n) return;
    const uint32_t* wr = w + (size_t)blockIdx.x * ld;
    const DT* dr = d + (size_t)blockIdx.x * ld;
    const double* rr = r + (size_t)blockIdx.x * ld;
    __shared__ int wave_cnt[4];
    __shared__ int base;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) base = ptr[u];
    __syncthreads();
    /* 4 consecutive columns per lane (one 16-B load of w and of d), 1024 per pass; arcs stay in
     * ascending t: lane-major, then the lane's 4. A lane's count (0..4) is spread over three
     * ballots, so its exclusive prefix in the wave is three masked popcounts. */
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int t0 = 0; t0 < n; t0 += 1024) {
        const int t = t0 + threadIdx.x * 4;
        uint32_t x[4] = {0, 0, 0, 0}, y[4] = {1, 1, 1, 1};
        if (t + 4 <= n) {
            const uint4 a = *reinterpret_cast<const uint4*>(wr + t);
            const uint4 b = ld_d4(dr + t);
            x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
            y[0] = b.x; y[1] = b.y; y[2] = b.z; y[3] = b.w;
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (t + q < n) {
                    x[q] = wr[t + q];
                    y[q] = (uint32_t)dr[t + q];
                }
        }
        bool ok[4];
        int c = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ok[q] = t + q < n && t + q != u && x[q] < SRT_INF && x[q] == y[q];
            c += ok[q];
        }
        const uint64_t b0 = __ballot(c & 1), b1 = __ballot(c & 2), b2 = __ballot(c & 4);
        const int before = __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
        if (lane == 0) wave_cnt[wv] = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
        __syncthreads();
        int o = base + before;
        for (int q = 0; q < wv; ++q) o += wave_cnt[q];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (ok[q]) {
                col[o] = t + q;
                aw[o] = x[q];
                ar[o] = rr[t + q];
                ++o;
            }
        __syncthreads();
        if (threadIdx.x == 0) base += wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3];
        __syncthreads();
    }
}

/* transpose an arc list (directed graphs: In*(t) from Out*(u)) */
/* (dtotal: the arc count read on the device, when the host did not wait for it) */
__global__ void arc_count_by_col(int64_t arcs, const int32_t* __restrict__ col,
                                 int32_t* __restrict__ cnt, const int32_t* __restrict__ dtotal) {
    if (dtotal) arcs = *dtotal;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < arcs;
         i += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&cnt[col[i]], 1);
}

__global__ void arc_transpose_fill(int n, const int32_t* __restrict__ ptr,
                                   const int32_t* __restrict__ col, const uint32_t* __restrict__ aw,
                                   const double* __restrict__ ar, int32_t* __restrict__ cursor,
                                   int32_t* __restrict__ tcol, uint32_t* __restrict__ tw,
                                   double* __restrict__ tr) {
    int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n) return;
    for (int k = ptr[u]; k < ptr[u + 1]; ++k) {
        int t = col[k];
        int o = atomicAdd(&cursor[t], 1);
        tcol[o] = u;
        tw[o] = aw[k];
        tr[o] = ar[k];
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Canonical predecessor, sources across lanes.                                               */
/* pred(s,t) = argmin over essential in-arcs (u,t) with D[s][u] + w == D[s][t] of (D[s][u], u) */
/* A wave takes 64 consecutive local sources; t and the arc list of t are wave-uniform (scalar */
/* loads), and D[s][u] for the 64 sources is one coalesced 256-byte read of row u of DT, the   */
/* transpose of the local row block. Blocks are mapped so that each XCD works on its own      */
/* source block at a time (its 8 MB column slab stays in that XCD's L2 / the Infinity Cache). */
/* ------------------------------------------------------------------------------------------ */
/* out[c][r] = in[r][c]; BM (block-major, 64 or 128): out[r / BM][c][r % BM], ldo = the stride of
 * a BM-row block, so each block's transpose is one contiguous slab */
template <typename T, typename TO = T, int BM = 0, bool NTS = false>
__global__ __launch_bounds__(256) void transpose_kernel(int rows, int cols, const T* __restrict__ in,
                                                        size_t ldi, TO* __restrict__ out, size_t ldo) {
    __shared__ T tile[64][65];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
    T v[16]; /* all 16 loads in flight before the LDS stores */
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int r = r0 + ty + 4 * q, c = c0 + tx;
        v[q] = (r < rows && c < cols) ? in[(size_t)r * ldi + c] : (T)0;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) tile[ty + 4 * q][tx] = v[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int a = ty + 4 * q, c = c0 + a, r = r0 + tx;
        if (r < rows && c < cols) {
            if constexpr (BM != 0)
                out[(size_t)(r / BM) * ldo + (size_t)c * BM + (r % BM)] = (TO)tile[tx][a];
            else if constexpr (NTS) /* streaming: rows read once, by a later pass */
                __builtin_nontemporal_store((TO)tile[tx][a], out + (size_t)c * ldo + r);
            else
                out[(size_t)c * ldo + r] = (TO)tile[tx][a];
        }
    }
}

/* Running minimum of canonical keys (high part D[s][u], low part u or its rank); with TIES, *tie
 * records whether the minimum D is reached by two different candidates -- the pairs whose
 * predecessor igraph's heap order decides (equal tentative distances settle in an
 * order the build cannot reproduce), reported as srt_build_stats.tied_pairs. */
template <bool TIES, int SH, typename K>
__device__ __forceinline__ void key_min(K& best, uint32_t& tie, K key) {
    if constexpr (TIES) {
        const bool same = key != ~(K)0 && (key >> SH) == (best >> SH);
        tie = key < best ? (uint32_t)same : (tie | (uint32_t)same);
    }
    best = min(best, key);
}

/* one atomic per wave: the wave's tie count */
static __device__ __forceinline__ void add_ties(unsigned long long* out, uint32_t c) {
    unsigned long long v = c;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(out, v);
}

template <typename T, bool UR, bool TIES>
__global__ __launch_bounds__(256) void pred_cols_kernel(int n, int row0, int nloc, int ldT,
                                                        size_t bsD, const T* __restrict__ DT,
                                                        const int32_t* __restrict__ iptr,
                                                        const uint2* __restrict__ uw,
                                                        const double* __restrict__ ar,
                                                        int32_t* __restrict__ predT,
                                                        double* __restrict__ rT, int nsb,
                                                        int tch, int tper, int sorted,
                                                        unsigned long long* __restrict__ ties) {
    /* UR: write the predecessor vertex and the reliability of its arc (predT, rT) for the
     * level-order pass; otherwise the arc index.
     * sorted: t's in-arc list is in ascending u (undirected: the out-lists of the ballot-compacted
     * essential arcs); the transposed lists of a directed graph are not, and key on u itself.
     * Narrow distances (u8/u16: D < 2^16) and in-degrees < 2^16 pack the key (D[s][u], arc rank
     * in t's list) into 32 bits; the lists are sorted by u, so the rank orders like u. A check is
     * then add, compare, pack, select, min; the winner's vertex and reliability are read once. */
    constexpr bool NARROW = sizeof(T) <= 2;
    const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
    const int sb = (j / tch) * 8 + xcd, tc = j % tch;
    if (sb >= nsb) return;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sl = sb * 64 + lane;
    const int s = row0 + sl;
    const bool valid = sl < nloc && s < n;
    const int t1 = min(n, (tc + 1) * tper);
    /* this source block's contiguous slab of the block-major transpose: DB[u * 64] = D[s][u] */
    const T* __restrict__ DB = DT + (size_t)sb * bsD + lane;
    uint32_t nties = 0;
    for (int t = tc * tper + wv; t < t1; t += 4) {
        const uint32_t dst = DB[(size_t)t * 64];
        uint32_t tie = 0;
        const int kb = __builtin_amdgcn_readfirstlane(iptr[t]);
        const int ke = __builtin_amdgcn_readfirstlane(iptr[t + 1]);
        int bk = -1;
        if (NARROW && ke - kb <= 0xFFFF) {
            uint32_t best = 0xFFFFFFFFu;
            int k = kb;
#define SRT_PRED_TRY32(dd, aa, kk)                                                              \
    key_min<TIES, 16>(best, tie,                                                               \
                      ((dd) + (aa).y == dst)                                                   \
                          ? (((dd) << 16) | (sorted ? (uint32_t)((kk) - kb) : (aa).x))         \
                          : 0xFFFFFFFFu);
            /* 16 (then 4, 1) candidate arcs per step: one batch of scalar loads, then the gathers
             * in flight together. The loop is latency bound: with 4 per step, u8 and u16 distances
             * measured the same (47 ms on C4); 16 per step 37 ms; 32 per step no better. */
            for (; k + 16 <= ke; k += 16) {
                uint2 a[16];
                uint32_t dd[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) a[q] = uw[k + q];
#pragma unroll
                for (int q = 0; q < 16; ++q) dd[q] = DB[(size_t)a[q].x * 64];
#pragma unroll
                for (int q = 0; q < 16; ++q) SRT_PRED_TRY32(dd[q], a[q], k + q)
            }
            for (; k + 4 <= ke; k += 4) {
                const uint2 a0 = uw[k], a1 = uw[k + 1], a2 = uw[k + 2], a3 = uw[k + 3];
                const uint32_t d0 = DB[(size_t)a0.x * 64], d1 = DB[(size_t)a1.x * 64];
                const uint32_t d2 = DB[(size_t)a2.x * 64], d3 = DB[(size_t)a3.x * 64];
                SRT_PRED_TRY32(d0, a0, k)
                SRT_PRED_TRY32(d1, a1, k + 1)
                SRT_PRED_TRY32(d2, a2, k + 2)
                SRT_PRED_TRY32(d3, a3, k + 3)
            }
            for (; k < ke; ++k) {
                const uint2 a0 = uw[k];
                const uint32_t d0 = DB[(size_t)a0.x * 64];
                SRT_PRED_TRY32(d0, a0, k)
            }
#undef SRT_PRED_TRY32
            if (best != 0xFFFFFFFFu) {
                if (sorted) {
                    bk = kb + (int)(best & 0xFFFFu);
                } else { /* find the winning vertex's arc in the (unsorted) list */
                    const uint32_t u = best & 0xFFFFu;
                    for (int q = kb; q < ke; ++q) bk = (uw[q].x == u) ? q : bk;
                }
            }
        } else {
            uint64_t best = ~0ull;
            int k = kb;
            for (; k < ke; ++k) {
                const uint2 a0 = uw[k];
                const uint32_t d0 = DB[(size_t)a0.x * 64];
                if (d0 + a0.y == dst) {
                    const uint64_t key = ((uint64_t)d0 << 32) | a0.x;
                    if (key < best) bk = k;
                    key_min<TIES, 32>(best, tie, key);
                }
            }
        }
        if (TIES && valid && s != t) nties += tie;
        if (valid) {
            const size_t o = (size_t)t * ldT + sl;
            if (UR) {
                const bool has = s != t && bk >= 0;
                predT[o] = has ? (int32_t)uw[bk].x : -1;
                rT[o] = has ? ar[bk] : 0.0;
            } else {
                predT[o] = (s == t) ? -1 : bk;
            }
        }
    }
    if (TIES) add_ties(ties, nties);
}

/* Byte distances, two sources per lane: a wave covers a 128-source block, one 128-B line of its
 * block-major slab (DT[s / 128][u][s % 128], 4 MB at n = 32,768) per candidate arc. Same keys and
 * outputs as pred_cols_kernel<uint8_t, true> for each of the lane's two sources. */
template <int U, bool TIES>
__global__ __launch_bounds__(256) void pred_cols2_kernel(int n, int row0, int nloc, int ldT,
                                                         size_t bsD, const uint8_t* __restrict__ DT,
                                                         const int32_t* __restrict__ iptr,
                                                         const uint2* __restrict__ uw,
                                                         const double* __restrict__ ar,
                                                         int32_t* __restrict__ predT,
                                                         double* __restrict__ rT, int nsb, int tch,
                                                         int tper, int sorted,
                                                         unsigned long long* __restrict__ ties) {
    const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
    const int sb = (j / tch) * 8 + xcd, tc = j % tch;
    if (sb >= nsb) return;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sl = sb * 128 + 2 * lane;
    const int s = row0 + sl;
    const bool v0 = sl < nloc && s < n, v1 = sl + 1 < nloc && s + 1 < n;
    const int t1 = min(n, (tc + 1) * tper);
    /* the slab through a buffer descriptor: row u is the scalar offset u * 128, the lane's two
     * bytes the constant vector offset, so no per-arc 64-bit address lives in VGPRs */
    const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(DT) + (size_t)sb * bsD, 0, (int)bsD, 0x00020000);
    const int voff = 2 * lane;
#define SRT_DB(u) ((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(slab, voff, (int)(u) * 128, 0))
    uint32_t nties = 0;
    for (int t = tc * tper + wv; t < t1; t += 4) {
        uint32_t tie0 = 0, tie1 = 0;
        const uint32_t dst = SRT_DB(t);
        const uint32_t dst0 = dst & 0xFFu, dst1 = dst >> 8;
        const int kb = __builtin_amdgcn_readfirstlane(iptr[t]);
        const int ke = __builtin_amdgcn_readfirstlane(iptr[t + 1]);
        uint32_t best0 = 0xFFFFFFFFu, best1 = 0xFFFFFFFFu;
        int k = kb;
#define SRT_PRED_TRY2(dd, aa, kk)                                                               \
    {                                                                                           \
        const uint32_t lo = (dd) & 0xFFu, hi = (dd) >> 8;                                       \
        const uint32_t id = sorted ? (uint32_t)((kk) - kb) : (aa).x;                            \
        key_min<TIES, 16>(best0, tie0, (lo + (aa).y == dst0) ? ((lo << 16) | id) : 0xFFFFFFFFu); \
        key_min<TIES, 16>(best1, tie1, (hi + (aa).y == dst1) ? ((hi << 16) | id) : 0xFFFFFFFFu); \
    }
        for (; k + U <= ke; k += U) {
            uint2 a[U];
            uint32_t dd[U];
#pragma unroll
            for (int q = 0; q < U; ++q) a[q] = uw[k + q];
#pragma unroll
            for (int q = 0; q < U; ++q) dd[q] = SRT_DB(a[q].x);
#pragma unroll
            for (int q = 0; q < U; ++q) SRT_PRED_TRY2(dd[q], a[q], k + q)
        }
        for (; k + 4 <= ke; k += 4) {
            uint2 a[4];
            uint32_t dd[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) a[q] = uw[k + q];
#pragma unroll
            for (int q = 0; q < 4; ++q) dd[q] = SRT_DB(a[q].x);
#pragma unroll
            for (int q = 0; q < 4; ++q) SRT_PRED_TRY2(dd[q], a[q], k + q)
        }
        for (; k < ke; ++k) {
            const uint2 a0 = uw[k];
            const uint32_t d0 = SRT_DB(a0.x);
            SRT_PRED_TRY2(d0, a0, k)
        }
#undef SRT_PRED_TRY2
        int bk0 = -1, bk1 = -1;
        if (sorted) {
            if (best0 != 0xFFFFFFFFu) bk0 = kb + (int)(best0 & 0xFFFFu);
            if (best1 != 0xFFFFFFFFu) bk1 = kb + (int)(best1 & 0xFFFFu);
        } else { /* find the winning vertices' arcs in the (unsorted) list */
            const uint32_t u0 = best0 != 0xFFFFFFFFu ? (best0 & 0xFFFFu) : 0xFFFFFFFFu;
            const uint32_t u1 = best1 != 0xFFFFFFFFu ? (best1 & 0xFFFFu) : 0xFFFFFFFFu;
            for (int q = kb; q < ke; ++q) {
                const uint32_t u = uw[q].x;
                bk0 = (u == u0) ? q : bk0;
                bk1 = (u == u1) ? q : bk1;
            }
        }
        const size_t o = (size_t)t * ldT + sl;
        const bool h0 = s != t && bk0 >= 0, h1 = s + 1 != t && bk1 >= 0;
        if (TIES) nties += (v0 && h0 ? tie0 : 0u) + (v1 && h1 ? tie1 : 0u);
        if (v0 && v1 && (o & 1) == 0) {
            *reinterpret_cast<int2*>(predT + o) =
                make_int2(h0 ? (int32_t)uw[bk0].x : -1, h1 ? (int32_t)uw[bk1].x : -1);
            rT[o] = h0 ? ar[bk0] : 0.0;
            rT[o + 1] = h1 ? ar[bk1] : 0.0;
        } else {
            if (v0) {
                predT[o] = h0 ? (int32_t)uw[bk0].x : -1;
                rT[o] = h0 ? ar[bk0] : 0.0;
            }
            if (v1) {
                predT[o + 1] = h1 ? (int32_t)uw[bk1].x : -1;
                rT[o + 1] = h1 ? ar[bk1] : 0.0;
            }
        }
    }
#undef SRT_DB
    if (TIES) add_ties(ties, nties);
}

/* Byte distances without the tie count: the canonical predecessor as ONE 32-bit minimum per arc
 * and source. Every distance fits a byte (<= 254) and the arcs come with A = (w' << 23) | id,
 * w' = min(w, 257), id = the arc's rank in t's list (sorted lists) or its tail (n <= 32,768, so
 * both fit 15 bits), and the row offset u * 128 (pack_uk_kernel). The key
 *   key = ((D[s][u] + w') << 23) | (D[s][u] << 15) | id = D[s][u] * (2^23 + 2^15) + A
 * is one v_mad_u32_u24, and its minimum over t's in-arcs orders first by D[s][u] + w -- the
 * smallest is D[s][t] exactly when some arc lies on a shortest path, which the winner is checked
 * for -- then by (D[s][u], id): pred_cols2_kernel's (D[s][u], rank) rule among the arcs with
 * D[s][u] + w = D[s][t], without its per-arc compare and select (12 -> 5 VALU per arc and wave). */
__global__ void pack_uk_kernel(int n, const int32_t* __restrict__ iptr, const int32_t* __restrict__ col,
                               const uint32_t* __restrict__ w, int sorted, uint2* __restrict__ uk) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= n) return;
    const int kb = iptr[t], ke = iptr[t + 1];
    for (int k = kb + (threadIdx.x & 63); k < ke; k += 64) {
        const uint32_t u = (uint32_t)col[k];
        const uint32_t id = sorted ? (uint32_t)(k - kb) : u;
        uk[k] = make_uint2(u << 7, (min(w[k], 257u) << 23) | id);
    }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void pred_cols3_kernel(int n, int row0, int nloc, int ldT,
                                                         size_t bsD, const uint8_t* __restrict__ DT,
                                                         const int32_t* __restrict__ iptr,
                                                         const uint2* __restrict__ uk,
                                                         const double* __restrict__ ar,
                                                         int32_t* __restrict__ predT,
                                                         double* __restrict__ rT, int nsb, int tch,
                                                         int tper, int sorted) {
    const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
    const int sb = (j / tch) * 8 + xcd, tc = j % tch;
    if (sb >= nsb) return;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sl = sb * 128 + 2 * lane;
    const int s = row0 + sl;
    const bool v0 = sl < nloc && s < n, v1 = sl + 1 < nloc && s + 1 < n;
    const int t1 = min(n, (tc + 1) * tper);
    const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(DT) + (size_t)sb * bsD, 0, (int)bsD, 0x00020000);
    const int voff = 2 * lane;
    /* the multiplier in a VGPR: v_mad_u32_u24 then reads one scalar operand (the arc's A), not
     * a literal and an SGPR, which would cost a v_mov per arc */
    uint32_t KM;
    asm volatile("v_mov_b32 %0, %1" : "=v"(KM) : "i"((1u << 23) + (1u << 15)));
#define SRT_DB3(off) ((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(slab, voff, (int)(off), 0))
    for (int t = tc * tper + wv; t < t1; t += 4) {
        const uint32_t dst = SRT_DB3(t * 128);
        const uint32_t dst0 = dst & 0xFFu, dst1 = dst >> 8;
        const int kb = __builtin_amdgcn_readfirstlane(iptr[t]);
        const int ke = __builtin_amdgcn_readfirstlane(iptr[t + 1]);
        uint32_t best0 = 0xFFFFFFFFu, best1 = 0xFFFFFFFFu;
        int k = kb;
        for (; k + U <= ke; k += U) {
            uint2 a[U];
            uint32_t dd[U];
#pragma unroll
            for (int q = 0; q < U; ++q) a[q] = uk[k + q];
#pragma unroll
            for (int q = 0; q < U; ++q) dd[q] = SRT_DB3(a[q].x);
#pragma unroll
            for (int q = 0; q < U; q += 2) {
                best0 = min(best0, min(__umul24(dd[q] & 0xFFu, KM) + a[q].y,
                                       __umul24(dd[q + 1] & 0xFFu, KM) + a[q + 1].y));
                best1 = min(best1, min(__umul24(dd[q] >> 8, KM) + a[q].y,
                                       __umul24(dd[q + 1] >> 8, KM) + a[q + 1].y));
            }
        }
        for (; k < ke; ++k) {
            const uint2 a0 = uk[k];
            const uint32_t d0 = SRT_DB3(a0.x);
            best0 = min(best0, __umul24(d0 & 0xFFu, KM) + a0.y);
            best1 = min(best1, __umul24(d0 >> 8, KM) + a0.y);
        }
        /* the winner lies on a shortest path iff its D[s][u] + w is D[s][t] */
        int bk0 = -1, bk1 = -1;
        const bool w0 = best0 != 0xFFFFFFFFu && (best0 >> 23) == dst0;
        const bool w1 = best1 != 0xFFFFFFFFu && (best1 >> 23) == dst1;
        if (sorted) {
            if (w0) bk0 = kb + (int)(best0 & 0x7FFFu);
            if (w1) bk1 = kb + (int)(best1 & 0x7FFFu);
        } else {
            const uint32_t u0 = w0 ? ((best0 & 0x7FFFu) << 7) : 0xFFFFFFFFu;
            const uint32_t u1 = w1 ? ((best1 & 0x7FFFu) << 7) : 0xFFFFFFFFu;
            for (int q = kb; q < ke; ++q) {
                const uint32_t u = uk[q].x;
                bk0 = (u == u0) ? q : bk0;
                bk1 = (u == u1) ? q : bk1;
            }
        }
        const size_t o = (size_t)t * ldT + sl;
        const bool h0 = s != t && bk0 >= 0, h1 = s + 1 != t && bk1 >= 0;
        if (v0 && v1 && (o & 1) == 0) {
            const int32_t p0 = h0 ? (int32_t)(uk[bk0].x >> 7) : -1;
            const int32_t p1 = h1 ? (int32_t)(uk[bk1].x >> 7) : -1;
            const double r0 = h0 ? ar[bk0] : 0.0, r1 = h1 ? ar[bk1] : 0.0;
            if constexpr (NT) {
                /* streaming stores: the 50 MB of outputs per source block do not allocate in
                 * L2, which holds the block's 4-MB slab */
                __builtin_nontemporal_store(p0, predT + o);
                __builtin_nontemporal_store(p1, predT + o + 1);
                __builtin_nontemporal_store(r0, rT + o);
                __builtin_nontemporal_store(r1, rT + o + 1);
            } else {
                *reinterpret_cast<int2*>(predT + o) = make_int2(p0, p1);
                rT[o] = r0;
                rT[o + 1] = r1;
            }
        } else {
            if (v0) {
                predT[o] = h0 ? (int32_t)(uk[bk0].x >> 7) : -1;
                rT[o] = h0 ? ar[bk0] : 0.0;
            }
            if (v1) {
                predT[o + 1] = h1 ? (int32_t)(uk[bk1].x >> 7) : -1;
                rT[o + 1] = h1 ? ar[bk1] : 0.0;
            }
        }
    }
#undef SRT_DB3
}

/* Path-order reliability by sweeps for rows with a large distance range (rel_levels_kernel
 * flagged them), one workgroup per row, same in-place (u, r) input. A target resolves once its
 * predecessor resolved in an earlier sweep (double-buffered LDS bitmaps; the sweeps = the depth
 * of the row's predecessor tree). */
template <typename PT = int32_t>
__global__ __launch_bounds__(512) void rel_sweeps_kernel(int n, int ld, int row0,
                                                         const PT* __restrict__ pred,
                                                         double* __restrict__ rel,
                                                         int32_t* __restrict__ max_depth,
                                                         const int32_t* __restrict__ only,
                                                         const int32_t* __restrict__ srcs = nullptr) {
    extern __shared__ __attribute__((aligned(16))) int32_t smem[];
    const int s = srcs ? srcs[blockIdx.x] : row0 + blockIdx.x; /* srcs: row i is source srcs[i] */
    if (s >= n || !only[blockIdx.x]) return;
    const int nw = (n + 31) >> 5;
    int32_t* pu = smem;                                   /* n predecessor vertices */
    uint32_t* done = reinterpret_cast<uint32_t*>(smem + n); /* resolved before this sweep */
    uint32_t* fresh = done + nw;                           /* resolved during this sweep */
    const PT* pg = pred + (size_t)blockIdx.x * ld;
    double* rr = rel + (size_t)blockIdx.x * ld;
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
        if constexpr (std::is_same_v<PT, uint32_t>) /* packed rows: the low half, int16 */
            pu[t] = (int32_t)(int16_t)(pg[t] & 0xFFFFu);
        else
            pu[t] = pg[t];
    }
    for (int q = threadIdx.x; q < nw; q += blockDim.x) {
        done[q] = 0u;
        fresh[q] = 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        done[s >> 5] = 1u << (s & 31);
        __hip_atomic_store(rr + s, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    /* each thread owns t = tid + i*blockDim (i < 64 for n <= 32768) */
    uint64_t pending = 0;
    int nt = 0;
    for (int t = threadIdx.x; t < n; t += blockDim.x, ++nt)
        if (t != s && pu[t] >= 0) pending |= 1ull << nt;
    __threadfence_block();
    __syncthreads();
    int depth = 0;
    for (;;) {
        int any = 0;
        int i = 0;
        for (int t = threadIdx.x; t < n; t += blockDim.x, ++i) {
            if (!((pending >> i) & 1ull)) continue;
            const int u = pu[t];
            if (!((done[u >> 5] >> (u & 31)) & 1u)) {
                any = 1;
                continue;
            }
            const double ru = __hip_atomic_load(rr + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const double rt = __hip_atomic_load(rr + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(rr + t, ru * rt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            atomicOr(&fresh[t >> 5], 1u << (t & 31));
            pending &= ~(1ull << i);
        }
        ++depth;
        __threadfence_block();
        if (!__syncthreads_or(any)) break;
        for (int q = threadIdx.x; q < nw; q += blockDim.x) {
            done[q] |= fresh[q];
            fresh[q] = 0u;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) srt_max_once(max_depth, depth);
}

/* Reliability in increasing-distance order, one workgroup per local source row, in place: the
 * rel row arrives holding r(pred(s,t), t) and the pred row the predecessor vertex (pred_cols
 * UR form). Every arc is >= 1 quantum, so D[s][pred] < D[s][t] and pass L (targets with
 * D[s][t] == L) only reads values final since an earlier pass: each entry is formed once,
 * rel(s,t) = rel(s,pred) * r(pred,t), the left-to-right product of topology.c:1364-1365.
 * Rows whose largest distance exceeds maxl passes are flagged for rel_sweeps_kernel. */
template <int NT, int MAXN>
__global__ __launch_bounds__(NT) void rel_levels_kernel(int n, int ld, int row0,
                                                         const uint32_t* __restrict__ lat,
                                                         int32_t* __restrict__ pred,
                                                         double* __restrict__ rel, int maxl,
                                                         int32_t* __restrict__ max_depth,
                                                         int32_t* __restrict__ sweep,
                                                         const int32_t* __restrict__ srcs = nullptr) {
    /* each thread owns t = tid + i * NT (i < PER, n <= MAXN); the row's distances are read once
     * and kept as bytes in registers (levels <= maxl <= 254 once the row qualifies), so a pass
     * only compares registers and touches memory for its own targets. The row reads go through
     * buffer descriptors (constant scalar offset per i, one vector offset), which keeps the 64
     * unrolled loads from holding 64-bit addresses. */
    constexpr int PER = MAXN / NT;
    const int s = srcs ? srcs[blockIdx.x] : row0 + blockIdx.x; /* srcs: row i is source srcs[i] */
    if (s >= n) return;
    const int tid = threadIdx.x;
    const uint32_t* dl = lat + (size_t)blockIdx.x * ld;
    int32_t* pg = pred + (size_t)blockIdx.x * ld;
    double* rr = rel + (size_t)blockIdx.x * ld;
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(dl), 0, n * 4, 0x00020000);
    __shared__ uint32_t red[NT / 64];
    extern __shared__ uint16_t s_wlist[]; /* NT / 64 waves x 64 x PER target indices */
    uint32_t lv[PER / 4];
    uint32_t mx = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        /* out of range reads 0 (the descriptor's bound): not a target of any pass, like the
         * source itself and unreachable vertices */
        /* read once: non-temporal (aux 2), so the row's distances do not displace the rel
         * rows that the level passes re-read from L2 */
        const uint32_t d = __builtin_amdgcn_raw_buffer_load_b32(rd, tid * 4, i * NT * 4, 2);
        const uint32_t x = (tid + i * NT != s && d < SRT_INF) ? d : 0u;
        mx = max(mx, x);
        const uint32_t b = min(x, 255u) << (8 * (i & 3));
        lv[i >> 2] = (i & 3) ? (lv[i >> 2] | b) : b;
    }
    for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
    if ((tid & 63) == 0) red[tid >> 6] = mx;
    if (tid == 0) rr[s] = 1.0;
    __threadfence_block();
    __syncthreads();
    mx = 0;
    for (int i = 0; i < NT / 64; ++i) mx = max(mx, red[i]);
    if (tid == 0) sweep[blockIdx.x] = (int)mx > maxl;
    if ((int)mx > maxl) return; /* long distance range: rel_sweeps_kernel takes the row */
    /* per pass, each wave compacts its targets of level L into its own LDS list (ballot +
     * prefix popcount), then walks the list with its lanes: the loads of different targets are
     * independent and stay in flight together */
    const int lane = tid & 63;
    uint16_t* wl = s_wlist + (size_t)(tid >> 6) * (64 * PER);
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint32_t L = 1; L <= mx; ++L) {
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const bool hit = ((lv[i >> 2] >> (8 * (i & 3))) & 0xFFu) == L;
            const uint64_t m = __ballot(hit);
            if (hit) wl[cnt + __popcll(m & lt)] = (uint16_t)(tid + i * NT);
            cnt += __popcll(m);
        }
        /* the list is written and read by this wave only */
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        /* QB targets per lane in flight: a pass costs about two dependent global latencies
         * (pred, then rel of the predecessor) per 64 * QB targets of the wave */
        constexpr int QB = 8;
        for (int j = lane; j < cnt; j += 64 * QB) {
            int t[QB], u[QB];
            double rt[QB], ru[QB];
#pragma unroll
            for (int q = 0; q < QB; ++q) t[q] = j + 64 * q < cnt ? (int)wl[j + 64 * q] : -1;
#pragma unroll
            for (int q = 0; q < QB; ++q) u[q] = t[q] >= 0 ? __builtin_nontemporal_load(pg + t[q]) : -1;
#pragma unroll
            for (int q = 0; q < QB; ++q) rt[q] = t[q] >= 0 ? rr[t[q]] : 0.0;
            /* u < 0: unreachable, cannot happen on a validated graph; the entry is kept */
#pragma unroll
            for (int q = 0; q < QB; ++q) ru[q] = u[q] >= 0 ? rr[u[q]] : 1.0;
#pragma unroll
            for (int q = 0; q < QB; ++q)
                if (t[q] >= 0) rr[t[q]] = ru[q] * rt[q];
        }
        __threadfence_block();
        __syncthreads();
    }
    if (tid == 0) srt_max_once(max_depth, (int)mx);
}

/* The same level-order product with the row held on chip: rel_levels_kernel's passes touch the
 * row's pred and rel lines once per level in scattered 4-8 B pieces (C4: ~2.4x the row bytes,
 * 12.1 ms). Here every thread loads its PER targets (t = tid + i * NT) once, coalesced: the level
 * byte and the arc reliability stay in registers, the predecessor goes to LDS as u16. Only the
 * targets that are some target's predecessor ("parents": C4 rows have ~1-3k of 32k, the vertices
 * at distance <= 2-3 quanta) get a value slot in LDS, found by a bitmap rank (word prefix +
 * popcount). Pass L forms rel(s,t) = rel(s,u) * r(u,t) for the targets at distance L from the
 * parents' slots and files the parents among them; the row is written once at the end. Rows with
 * more parents than the cap slots (or a distance range beyond maxl) return untouched and flagged
 * for rel_sweeps_kernel. Dynamic LDS: rel_tree_lds(NT, PER, cap). */
static constexpr size_t rel_tree_lds(int nt, int per, int cap, int ntab = 0) {
    return (size_t)8 * nt + (size_t)2 * nt * per + (size_t)8 * cap + (size_t)8 * ntab;
}

/* PT = uint32_t: the packed rows of the level build (predecessor | reliability index << 16,
 * srt_levels_rtab): the arc reliability comes from the table (in LDS) instead of the rel row, which
 * is then written, not read -- every entry, 0.0 for the unreachable ones. */
template <int NT, int PER, typename LT, typename PT = int32_t>
__global__ __launch_bounds__(NT) void rel_tree_kernel(int n, int ld, int row0,
                                                      const LT* __restrict__ lat,
                                                      const PT* __restrict__ pred,
                                                      double* __restrict__ rel, int maxl, int cap,
                                                      int32_t* __restrict__ max_depth,
                                                      int32_t* __restrict__ sweep,
                                                      const int32_t* __restrict__ srcs = nullptr,
                                                      const double* __restrict__ rtab = nullptr,
                                                      int ntab = 0) {
    constexpr bool PK = std::is_same_v<PT, uint32_t>;
    /* the rows' loads: non-temporal (aux 2) on the FW path; cached for the packed rows, measured
     * 5.27-5.38 against 5.48-5.57 ms on C4 (`profiles/r04/exp/`) */
    constexpr int AUX = PK ? 0 : 2;
    const int s = srcs ? srcs[blockIdx.x] : row0 + blockIdx.x; /* srcs: row i is source srcs[i] */
    if (s >= n) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int nw = (n + 31) >> 5; /* <= NT (n <= 32 NT) */
    extern __shared__ __attribute__((aligned(16))) uint32_t tsm[];
    uint32_t* par = tsm;                                          /* parent bitmap, nw words */
    uint32_t* pre = tsm + NT;                                     /* parents before each word */
    uint16_t* spu = reinterpret_cast<uint16_t*>(tsm + 2 * NT);    /* predecessor per target */
    double* slot = reinterpret_cast<double*>(spu + NT * PER);     /* cap parent values */
    double* srt = slot + cap;                                     /* PK: the ntab reliabilities */
    __shared__ uint32_t red[NT / 64], wsum[NT / 64];
    for (int q = tid; q < nw; q += NT) par[q] = 0u;
    /* PK: each target's table index is stashed in the slot area until x is formed (the slots
     * take parent values only after that; cap * 8 >= 2 * NT * PER) */
    uint16_t* stash = reinterpret_cast<uint16_t*>(slot);
    if constexpr (PK) /* the table, and 0.0 at ntab: the index of s and of unreachable targets */
        for (int q = tid; q <= ntab; q += NT) srt[q] = q < ntab ? rtab[q] : 0.0;
    const LT* dl = lat + (size_t)blockIdx.x * ld;
    const PT* pg = pred + (size_t)blockIdx.x * ld;
    double* rr = rel + (size_t)blockIdx.x * ld;
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<LT*>(dl), 0, n * (int)sizeof(LT), 0x00020000);
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<PT*>(pg), 0, n * (int)sizeof(PT), 0x00020000);
    const __amdgpu_buffer_rsrc_t rv =
        __builtin_amdgcn_make_buffer_rsrc(rr, 0, n * 8, 0x00020000);
    uint32_t lv[PER / 4];
    double x[PER];
    uint32_t mx = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        /* out of range reads 0 (the descriptors' bound): no level, like s and unreachable targets */
        /* u32 table rows (SRT_INF: unreachable) or a level build's u8 rows (0: s itself) */
        uint32_t d;
        if constexpr (sizeof(LT) == 1)
            d = __builtin_amdgcn_raw_buffer_load_b8(rd, tid, i * NT, AUX);
        else
            d = __builtin_amdgcn_raw_buffer_load_b32(rd, tid * 4, i * NT * 4, 2);
        uint32_t p; /* int32 rows, or int16 (-1 -> 0xFFFF either way below) */
        if constexpr (sizeof(PT) == 2)
            p = __builtin_amdgcn_raw_buffer_load_b16(rp, tid * 2, i * NT * 2, 2);
        else
            p = __builtin_amdgcn_raw_buffer_load_b32(rp, tid * 4, i * NT * 4, AUX);
        if constexpr (PK) {
            const uint32_t t = (uint32_t)(tid + i * NT);
            const uint32_t hi = ((p & 0xFFFFu) == 0xFFFFu || t == (uint32_t)s || t >= (uint32_t)n)
                                    ? (uint32_t)ntab : (p >> 16) & 0x7FFu; /* (level above) */
            stash[t] = (uint16_t)hi;
            p &= 0xFFFFu;
        }
        const uint32_t l = (tid + i * NT != s && d < SRT_INF) ? d : 0u;
        mx = max(mx, l);
        const uint32_t b = min(l, 255u) << (8 * (i & 3));
        lv[i >> 2] = (i & 3) ? (lv[i >> 2] | b) : b;
        spu[tid + i * NT] = (uint16_t)p; /* -1 -> 0xFFFF (n <= 32768) */
    }
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    if (lane == 0) red[tid >> 6] = mx;
    __syncthreads(); /* par zeroed, red */
    mx = 0;
    for (int i = 0; i < NT / 64; ++i) mx = max(mx, red[i]);
#pragma unroll
    for (int i = 0; i < PER; ++i) { /* mark the parents */
        const uint32_t l = (lv[i >> 2] >> (8 * (i & 3))) & 0xFFu;
        const uint32_t u = spu[tid + i * NT];
        const uint32_t bit = 1u << (u & 31); /* tested first: ~one atomic per parent */
        if (l && u != 0xFFFFu && (int)u != s && !(par[u >> 5] & bit)) atomicOr(&par[u >> 5], bit);
    }
    __syncthreads();
    /* exclusive prefix of the parent counts over the bitmap words (one word per thread) */
    const uint32_t c = tid < nw ? (uint32_t)__popc(par[tid]) : 0u;
    uint32_t inc = c;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[tid >> 6] = inc;
    __syncthreads();
    uint32_t base = 0, total = 0;
    for (int i = 0; i < NT / 64; ++i) {
        base += i < (tid >> 6) ? wsum[i] : 0u;
        total += wsum[i];
    }
    if (tid < nw) pre[tid] = base + inc - c;
    const bool bail = (int)mx > maxl || total > (uint32_t)cap;
    if (tid == 0) sweep[blockIdx.x] = bail;
    if constexpr (PK) { /* the arc reliabilities from the table (0.0: s, unreachable) */
        /* the levels packed before the 64 registers of x are loaded (else the compiler keeps the
         * 32 unpacked level bytes beside them and spills) */
#pragma unroll
        for (int k = 0; k < PER / 4; ++k) asm volatile("" : "+v"(lv[k]));
        int tx = tid; /* opaque: no stash addresses kept from the load loop */
        asm volatile("" : "+v"(tx));
        if (bail || mx == 0) { /* rel_sweeps_kernel's input: r(pred, t) in the rel row (mx = 0:
                                * every entry 0.0, and rel(s, s) = 1) */
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int t = tx + i * NT;
                if (t < n) rr[t] = !bail && t == s ? 1.0 : srt[stash[t]];
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < PER; ++i) x[i] = srt[stash[tx + i * NT]];
    } else {
        if (bail) return; /* uniform: rel_sweeps_kernel takes the row from its untouched input */
        if (mx == 0) { /* no reachable target: only rel(s, s) */
            if (tid == 0) rr[s] = 1.0;
            return;
        }
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const uint32_t v0 = __builtin_amdgcn_raw_buffer_load_b32(rv, tid * 8, i * NT * 8, 0);
            const uint32_t v1 = __builtin_amdgcn_raw_buffer_load_b32(rv, tid * 8 + 4, i * NT * 8, 0);
            x[i] = __hiloint2double((int)v1, (int)v0);
        }
    }
    __syncthreads();
    auto rank = [&](uint32_t u) {
        return pre[u >> 5] + (uint32_t)__popc(par[u >> 5] & ((1u << (u & 31)) - 1u));
    };
    uint32_t L = 1;
    do { /* passes 1..mx (mx >= 1: one pass at least, so x needs no second copy for a skip) */
        /* opaque per pass: keeps the compiler from hoisting the PER unpacked levels and target
         * indices out of the loop (they would not fit beside x) */
#pragma unroll
        for (int k = 0; k < PER / 4; ++k) asm volatile("" : "+v"(lv[k]));
        int tl = tid;
        asm volatile("" : "+v"(tl));
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            if (((lv[i >> 2] >> (8 * (i & 3))) & 0xFFu) != L) continue;
            const uint32_t t = (uint32_t)(tl + i * NT);
            const uint32_t u = spu[t];
            /* u == s: the direct arc (rel(s,s) = 1); u < 0 cannot happen on a validated graph
             * and keeps the entry, as in rel_levels_kernel */
            const double ru = (u == 0xFFFFu || (int)u == s) ? 1.0 : slot[rank(u)];
            x[i] = ru * x[i];
            if ((par[t >> 5] >> (t & 31)) & 1u) slot[rank(t)] = x[i];
        }
        __syncthreads();
    } while (++L <= mx);
    int tw = tid;
    asm volatile("" : "+v"(tw));
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int t = tw + i * NT;
        /* PK: every entry (the row was not pre-filled); rel(s, s) = 1 */
        if (t < n && (PK || ((lv[i >> 2] >> (8 * (i & 3))) & 0xFFu)))
            __builtin_nontemporal_store(PK && t == s ? 1.0 : x[i], rr + t);
    }
    if (tid == 0) {
        rr[s] = 1.0;
        srt_max_once(max_depth, (int)mx);
    }
}

/* rel_tree_kernel at the row's size class (n <= 32768) */
template <typename LT, typename PT>
static void rel_tree_launch(int n, int ld, int row0, int lrows, const LT* d, const PT* pred,
                            double* rel, int32_t* depth, int32_t* sweep, const int32_t* srcs,
                            hipStream_t st, const double* rtab = nullptr, int ntab = 0) {
    if (n <= 1024) {
        const int lds = (int)rel_tree_lds(256, 4, 1024, ntab + 1);
        (void)hipFuncSetAttribute((const void*)rel_tree_kernel<256, 4, LT, PT>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        rel_tree_kernel<256, 4, LT, PT><<<lrows, 256, lds, st>>>(
            n, ld, row0, d, pred, rel, 64, 1024, depth, sweep, srcs, rtab, ntab);
    } else if (n <= 4096) {
        const int lds = (int)rel_tree_lds(512, 8, 4096, ntab + 1);
        (void)hipFuncSetAttribute((const void*)rel_tree_kernel<512, 8, LT, PT>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        rel_tree_kernel<512, 8, LT, PT><<<lrows, 512, lds, st>>>(n, ld, row0, d, pred, rel, 64, 4096,
                                                                 depth, sweep, srcs, rtab, ntab);
    } else {
        /* 64 KB of predecessors and 7,168 parent slots (C4 rows have ~1-3k parents): 128 KB; the
         * packed form: 8,192 slots (its index stash) and the table (<= 2,049 values): 152 KB */
        const int cap = rtab ? 8192 : 7168, lds = (int)rel_tree_lds(1024, 32, cap, ntab + 1);
        (void)hipFuncSetAttribute((const void*)rel_tree_kernel<1024, 32, LT, PT>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        rel_tree_kernel<1024, 32, LT, PT><<<lrows, 1024, lds, st>>>(n, ld, row0, d, pred, rel, 64,
                                                                    cap, depth, sweep, srcs, rtab,
                                                                    ntab);
    }
}

/* Round 5: the reliability pass of the source-major packed words (srt_levels_pred's, transposed: pred | rix << 16
 * | level << 27 per pair). rel(s,t) = rel(s,pred) * r(pred,t) needs, besides the pair's own word,
 * only rel(s,pred) -- and the predecessors of a row are few (its "parents": C4 rows have ~1-3k of
 * 32k targets, the vertices at distance <= 2-3 quanta). So a row's pass computes the parents alone,
 * in level order (a parent's own predecessor is a parent one level down, topology.c:1364-1365's
 * left-to-right product), then streams every pair once: 4 B read, the u32 distance and the f64
 * reliability written (16 B per pair, nothing else). rel_tree_kernel kept every target's
 * predecessor and value on chip (152 KB of LDS, one 1,024-thread row per CU); here only the
 * parents' words and values are in LDS (~72 KB: two rows per CU, one row's stores under the other's
 * loads), the row's words in registers (thread = 4 consecutive targets per 16-B piece, K pieces).
 * A row with more parents than the cap slots takes rel_sweeps_kernel from the r(pred, t) it
 * leaves in the rel row (sweep[row] = 1). */
#define REL_PK_NT 512
/* (plain row stores: non-temporal ones measured 4.47-4.53 against 3.83 ms, r05nt; the per-phase
 * wall-clock profile of round 5 is in DESIGN §5.8b) */
template <int K>
__global__ __launch_bounds__(REL_PK_NT) void rel_pk_kernel(int n, int ld, int row0,
                                                           const uint32_t* __restrict__ pk,
                                                           uint32_t* __restrict__ lat,
                                                           double* __restrict__ rel,
                                                           const double* __restrict__ rtab, int ntab,
                                                           int cap, int32_t* __restrict__ max_depth,
                                                           int32_t* __restrict__ sweep) {
    constexpr int NT = REL_PK_NT;
    const int s = row0 + (int)blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int nwb = ld >> 5; /* parent bitmap words (ld % 128 == 0) */
    extern __shared__ __attribute__((aligned(16))) uint32_t psm[];
    uint32_t* par = psm;                                         /* parent bitmap */
    uint32_t* pre = psm + nwb;                                   /* parents before each word */
    double* srt = reinterpret_cast<double*>(psm + 2 * nwb);      /* the ntab reliabilities, 0.0 */
    double* pval = srt + ((ntab + 2) & ~1);                      /* cap parent values */
    uint32_t* pinfo = reinterpret_cast<uint32_t*>(pval + cap);   /* cap parent words */
    __shared__ uint32_t wsum[NT / 64], red[NT / 64];
    for (int q = tid; q < nwb; q += NT) par[q] = 0u;
    for (int q = tid; q <= ntab; q += NT) srt[q] = q < ntab ? rtab[q] : 0.0;
    /* the row through a buffer descriptor: one 32-bit offset per piece, and pieces past the row
     * read 0 (level 0: written as "no path", and never stored: t0 >= ld) */
    const __amdgpu_buffer_rsrc_t rrow = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(pk + (size_t)blockIdx.x * ld), 0, ld * 4, 0x00020000);
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    uint4 wd[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rrow, tid * 16, k * NT * 16, 0);
        wd[k] = make_uint4(v.x, v.y, v.z, v.w);
        /* targets past n (the row's padding) carry no word: a transpose leaves them as they were */
        const int t4 = 4 * (tid + k * NT);
        if (t4 + 3 >= n) {
            if (t4 + 0 >= n) wd[k].x = 0xFFFFu;
            if (t4 + 1 >= n) wd[k].y = 0xFFFFu;
            if (t4 + 2 >= n) wd[k].z = 0xFFFFu;
            if (t4 + 3 >= n) wd[k].w = 0xFFFFu;
        }
    }
    __syncthreads(); /* par zeroed */
    uint32_t mx = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t e4[4] = {wd[k].x, wd[k].y, wd[k].z, wd[k].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t w = e4[e], l = w >> 27, u = w & 0xFFFFu;
            mx = max(mx, l);
            /* a row's 32k targets name only its ~1-3k parents: test before the atomic, so the
             * LDS atomics are ~one per parent instead of one per target (hub parents' words
             * would otherwise serialise thousands of them) */
            const uint32_t bit = 1u << (u & 31);
            if (l && (int)u != s && !(par[u >> 5] & bit)) atomicOr(&par[u >> 5], bit);
        }
    }
    /* opaque words from here on: else the compiler keeps every word's decoded fields live
     * across the phases (3 registers per target, one row per CU) */
#pragma unroll
    for (int k = 0; k < K; ++k)
        asm volatile("" : "+v"(wd[k].x), "+v"(wd[k].y), "+v"(wd[k].z), "+v"(wd[k].w));
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    if (lane == 0) red[tid >> 6] = mx;
    __syncthreads(); /* par, red */
    mx = 0;
    for (int i = 0; i < NT / 64; ++i) mx = max(mx, red[i]);
    /* exclusive prefix of the parent counts; thread tid owns bitmap words tid * wpt.. */
    const int wpt = (nwb + NT - 1) / NT;
    uint32_t c = 0;
    for (int i = 0; i < wpt; ++i) {
        const int q = tid * wpt + i;
        if (q < nwb) c += (uint32_t)__popc(par[q]);
    }
    uint32_t inc = c;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[tid >> 6] = inc;
    __syncthreads();
    uint32_t base = 0, total = 0;
    for (int i = 0; i < NT / 64; ++i) {
        base += i < (tid >> 6) ? wsum[i] : 0u;
        total += wsum[i];
    }
    uint32_t run = base + inc - c;
    for (int i = 0; i < wpt; ++i) {
        const int q = tid * wpt + i;
        if (q < nwb) {
            pre[q] = run;
            run += (uint32_t)__popc(par[q]);
        }
    }
    const bool bail = total > (uint32_t)cap;
    if (tid == 0) sweep[blockIdx.x] = bail;
    __syncthreads(); /* pre */
    auto rank = [&](uint32_t u) {
        return pre[u >> 5] + (uint32_t)__popc(par[u >> 5] & ((1u << (u & 31)) - 1u));
    };
    if (!bail) {
        /* the parents' own words into their slots */
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t e4[4] = {wd[k].x, wd[k].y, wd[k].z, wd[k].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t t = 4u * (uint32_t)(tid + k * NT) + e;
                if ((int)t < n && ((par[t >> 5] >> (t & 31)) & 1u)) pinfo[rank(t)] = e4[e];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
        /* the parents' values by level: a level-L parent's predecessor is s or a parent of level
         * L - 1 (every arc >= 1 quantum); parents sit below the row's largest level */
        for (uint32_t lv = 1; lv < mx; ++lv) {
            for (int q = tid; q < (int)total; q += NT) {
                const uint32_t w = pinfo[q];
                if ((w >> 27) != lv) continue;
                const uint32_t u = w & 0xFFFFu;
                const double ru = (int)u == s ? 1.0 : pval[rank(u)];
                pval[q] = ru * srt[(w >> 16) & 0x7FFu];
            }
            __syncthreads();
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
        asm volatile("" : "+v"(wd[k].x), "+v"(wd[k].y), "+v"(wd[k].z), "+v"(wd[k].w));
    uint32_t* lr = lat + (size_t)blockIdx.x * ld;
    double* rr = rel + (size_t)blockIdx.x * ld;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int t0 = 4 * (tid + k * NT);
        if (t0 >= ld) continue;
        const uint32_t e4[4] = {wd[k].x, wd[k].y, wd[k].z, wd[k].w};
        uint32_t lv[4];
        double x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t w = e4[e], l = w >> 27, u = w & 0xFFFFu;
            const int t = t0 + e;
            if (!l) { /* s itself (the diagonal rule follows), or no path / padding */
                lv[e] = t == s ? 0u : SRT_INF;
                x[e] = t == s ? 1.0 : 0.0;
            } else {
                lv[e] = l;
                const double r = srt[(w >> 16) & 0x7FFu];
                /* bail: r(pred, t) for rel_sweeps_kernel */
                x[e] = bail ? r : ((int)u == s ? 1.0 : pval[rank(u)]) * r;
            }
        }
        /* whole 16-B pieces: one coalesced 1-KB run per wave for the u32 row, two for the f64 */
        typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
        typedef double f64x2v __attribute__((ext_vector_type(2)));
        *reinterpret_cast<u32x4v*>(lr + t0) = (u32x4v){lv[0], lv[1], lv[2], lv[3]};
        *reinterpret_cast<f64x2v*>(rr + t0) = (f64x2v){x[0], x[1]};
        *reinterpret_cast<f64x2v*>(rr + t0 + 2) = (f64x2v){x[2], x[3]};
        /* one piece at a time: hoisting every piece's LDS reads costs the second row per CU */
        __builtin_amdgcn_sched_barrier(0);
    }
    if (tid == 0) srt_max_once(max_depth, (int)mx);
}

/* rel_pk_kernel at the row's width, then the sweeps for the rows over the parent cap */
static int rel_pk_launch(int n, int ld, int row0, int lrows, const uint32_t* pk, uint32_t* lat,
                         double* rel, const double* rtab, int ntab, int32_t* depth, int32_t* sweep,
                         hipStream_t st) {
    if (lrows <= 0) return SRT_OK;
    if (ld > 32768 || ntab > 2048) {
        srt_set_error("rel_pk_launch: ld %d / %d reliabilities beyond the packed form", ld, ntab);
        return SRT_E_ARG;
    }
    /* two rows per CU: ~80 KB of LDS per workgroup, the rest of it parent slots (12 B each) */
    const int fixed = 8 * (ld >> 5) + 8 * ((ntab + 2) & ~1);
    const int cap = min(n, (80 * 1024 - fixed) / 12) & ~63;
    const int lds = fixed + 12 * cap;
    const void* fn;
    const int K = (ld + 4 * REL_PK_NT - 1) / (4 * REL_PK_NT) <= 1 ? 1
                  : (ld + 4 * REL_PK_NT - 1) / (4 * REL_PK_NT) <= 2 ? 2
                  : (ld + 4 * REL_PK_NT - 1) / (4 * REL_PK_NT) <= 4 ? 4
                  : (ld + 4 * REL_PK_NT - 1) / (4 * REL_PK_NT) <= 8 ? 8 : 16;
    switch (K) {
    case 1: fn = (const void*)rel_pk_kernel<1>; break;
    case 2: fn = (const void*)rel_pk_kernel<2>; break;
    case 4: fn = (const void*)rel_pk_kernel<4>; break;
    case 8: fn = (const void*)rel_pk_kernel<8>; break;
    default: fn = (const void*)rel_pk_kernel<16>; break;
    }
    SRT_HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
#define REL_PK_GO(KK)                                                                          \
    rel_pk_kernel<KK><<<lrows, REL_PK_NT, lds, st>>>(n, ld, row0, pk, lat, rel, rtab, ntab, cap, \
                                                     depth, sweep)
    switch (K) {
    case 1: REL_PK_GO(1); break;
    case 2: REL_PK_GO(2); break;
    case 4: REL_PK_GO(4); break;
    case 8: REL_PK_GO(8); break;
    default: REL_PK_GO(16); break;
    }
#undef REL_PK_GO
    SRT_HIPCHK(hipGetLastError());
    const size_t slds = (size_t)n * sizeof(int32_t) + 2 * (size_t)((n + 31) / 32) * 4;
    SRT_HIPCHK(hipFuncSetAttribute((const void*)rel_sweeps_kernel<uint32_t>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)slds));
    rel_sweeps_kernel<uint32_t><<<lrows, 512, slds, st>>>(n, ld, row0, pk, rel, depth, sweep, nullptr);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

/* Rows with deep predecessor trees (metric / Tor-atlas-like graphs: ~100 hops, hundreds of distinct
 * distances, ~8k parents of 32k targets -- too deep for rel_tree_kernel's level passes, too many
 * parents for its slots). rel_sweeps_kernel rescans the whole row once per tree level (C4metric:
 * 221 ms). Here one wave owns a row: a counting sort of its targets by distance (every arc >= 1
 * quantum, so a predecessor is strictly nearer: distance order is a topological order of the tree),
 * then the targets in that order, 64 at a time, rel(s,t) = rel(s,pred) * r(pred,t) -- the
 * left-to-right product of topology.c:1364-1365 -- with one dependent round trip per distance
 * value present in a 64-entry chunk. The rel row arrives holding r(pred, t) (in place); the
 * sorted list goes to `ord` (ld u32 per row: dist << 16 | t). Rows with a distance past
 * ORD_NB - 1 stay flagged for the sweeps. */
#define ORD_NB 1024
#define ORD_WAVES 4
template <typename PT>
__global__ __launch_bounds__(64 * ORD_WAVES) void rel_order_kernel(int n, int ld, int row0, int lrows,
                                                                   const uint32_t* __restrict__ d,
                                                                   const PT* __restrict__ pred,
                                                                   double* __restrict__ rel,
                                                                   uint32_t* __restrict__ ord,
                                                                   int32_t* __restrict__ only,
                                                                   int32_t* __restrict__ max_depth) {
    __shared__ uint32_t cnt_all[ORD_WAVES][ORD_NB];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    uint32_t* cnt = cnt_all[wv];
    const int waves = (int)gridDim.x * ORD_WAVES;
    for (int row = (int)blockIdx.x * ORD_WAVES + wv; row < lrows; row += waves) {
        if (!only[row]) continue;
        const int s = row0 + row;
        const uint32_t* dr = d + (size_t)row * ld;
        const PT* pr = pred + (size_t)row * ld;
        double* rr = rel + (size_t)row * ld;
        uint32_t* od = ord + (size_t)row * ld;
        for (int i = lane; i < ORD_NB; i += 64) cnt[i] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        /* histogram of the reachable targets' distances (s itself and no-path entries left out) */
        uint32_t mx = 0;
        for (int t = lane; t < n; t += 64) {
            const uint32_t x = dr[t];
            if (t == s || x >= SRT_INF) continue;
            mx = max(mx, x);
            if (x < ORD_NB) atomicAdd(&cnt[x], 1u);
        }
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
        if (mx >= ORD_NB) continue; /* stays flagged: rel_sweeps_kernel */
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        /* exclusive prefix in place: lane l owns buckets [16 l, 16 l + 16) */
        constexpr int PER = ORD_NB / 64;
        uint32_t loc = 0;
        for (int k = 0; k < PER; ++k) loc += cnt[lane * PER + k];
        uint32_t inc = loc;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
            if (lane >= o) inc += y;
        }
        uint32_t run = inc - loc;
        for (int k = 0; k < PER; ++k) {
            const uint32_t c = cnt[lane * PER + k];
            cnt[lane * PER + k] = run;
            run += c;
        }
        const int total = (int)__shfl(inc, 63);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int t = lane; t < n; t += 64) {
            const uint32_t x = dr[t];
            if (t == s || x >= SRT_INF) continue;
            const uint32_t pos = atomicAdd(&cnt[x], 1u);
            od[pos] = (x << 16) | (uint32_t)t;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); /* the list, then read back */
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        /* the targets in distance order; inside a chunk, one step per distance value */
        for (int base = 0; base < total; base += 64) {
            const int i = base + lane;
            const bool act = i < total;
            const uint32_t e = act ? __hip_atomic_load(od + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                                   : 0xFFFFFFFFu;
            const int t = (int)(e & 0xFFFFu);
            const uint32_t dist = e >> 16;
            int p = act ? (int)pr[t] : -1;
            const double r = act ? rr[t] : 0.0;
            uint32_t cur = act ? dist : 0xFFFFu;
            for (int o = 32; o > 0; o >>= 1) cur = min(cur, (uint32_t)__shfl_xor((int)cur, o));
            bool pend = act;
            while (__any(pend)) {
                if (pend && dist == cur) {
                    /* p < 0 cannot happen on a reachable target of a validated graph: kept */
                    const double ru = p == s ? 1.0
                                    : p < 0  ? 1.0
                                             : __hip_atomic_load(rr + p, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_store(rr + t, ru * r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    pend = false;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                uint32_t nx = pend ? dist : 0xFFFFu;
                for (int o = 32; o > 0; o >>= 1) nx = min(nx, (uint32_t)__shfl_xor((int)nx, o));
                cur = nx;
            }
        }
        if (lane == 0) {
            __hip_atomic_store(rr + s, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            only[row] = 0;
            srt_max_once(max_depth, (int)mx);
        }
    }
}

/* Path-order reliability of lrows rows whose rel rows hold r(pred, t) (pred rows beside them):
 * rel_tree_kernel for n <= 32768 (rel_levels_kernel past it, or under SRT_FORM reltree=0), then
 * the sweeps for the rows it flagged. depth, sweep: device scratch (max depth, per-row flags). */
/* Deep rows, parents only (rel_pk_kernel's idea on the FW path's int32 predecessor rows): only the
 * parents' values must be readable by other targets, and a metric row has ~8k of them among 32k
 * targets. One workgroup per row:
 *   A. the row's predecessors, coalesced: the parent bitmap (LDS atomics), its prefix ranks;
 *   B. the parents' own (distance, predecessor, r(pred, t)) into rank slots, a histogram of their
 *      distances, and a counting sort of the slots by distance;
 *   C. the parents' values in distance order (every arc >= 1 quantum: a parent's predecessor is a
 *      nearer parent), one barrier per distance present, LDS only;
 *   D. every target once, coalesced: rel(s,t) = rel(s,pred) * r(pred,t) from the slots -- the
 *      left-to-right product of topology.c:1364-1365.
 * 24 B of HBM per pair (d and pred twice, r in, rel out) and no scattered global access. Rows with
 * more parents than the cap (or distances past DEEP_NB - 1) stay flagged for rel_order_kernel. */
#define DEEP_NT 512
#define DEEP_NB 1024
__global__ __launch_bounds__(DEEP_NT) void rel_deep_kernel(int n, int ld, int row0, int lrows,
                                                           const uint32_t* __restrict__ d,
                                                           const int32_t* __restrict__ pred,
                                                           double* __restrict__ rel, int cap,
                                                           int32_t* __restrict__ only,
                                                           int32_t* __restrict__ max_depth) {
    const int row = blockIdx.x;
    if (row >= lrows || !only[row]) return;
    const int s = row0 + row, tid = threadIdx.x, lane = tid & 63;
    const int nwb = ld >> 5;
    extern __shared__ __attribute__((aligned(16))) uint32_t dsm[];
    uint32_t* par = dsm;                                       /* parent bitmap (nwb words) */
    uint32_t* pre = dsm + nwb;                                 /* parents before each word */
    uint32_t* hist = dsm + 2 * nwb;                            /* DEEP_NB bucket offsets */
    double* pval = reinterpret_cast<double*>(hist + DEEP_NB);  /* cap values (r(pred,t) first) */
    uint16_t* pp = reinterpret_cast<uint16_t*>(pval + cap);    /* the slot's predecessor */
    uint16_t* pd = pp + cap;                                   /* the slot's distance */
    uint16_t* ord = pd + cap;                                  /* slots in distance order */
    __shared__ uint32_t wsum[DEEP_NT / 64], red[DEEP_NT / 64];
    const uint32_t* dr = d + (size_t)row * ld;
    const int32_t* pr = pred + (size_t)row * ld;
    double* rr = rel + (size_t)row * ld;
    for (int q = tid; q < nwb; q += DEEP_NT) par[q] = 0u;
    for (int q = tid; q < DEEP_NB; q += DEEP_NT) hist[q] = 0u;
    __syncthreads();
    /* A */
    uint32_t mx = 0;
    for (int t = tid; t < n; t += DEEP_NT) {
        const uint32_t x = dr[t];
        const int p = pr[t];
        if (t == s || x >= SRT_INF || p < 0) continue;
        mx = max(mx, x);
        const uint32_t bit = 1u << (p & 31); /* tested first: ~one atomic per parent */
        if (p != s && !(par[p >> 5] & bit)) atomicOr(&par[p >> 5], bit);
    }
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    if (lane == 0) red[tid >> 6] = mx;
    __syncthreads();
    mx = 0;
    for (int i = 0; i < DEEP_NT / 64; ++i) mx = max(mx, red[i]);
    const int wpt = (nwb + DEEP_NT - 1) / DEEP_NT;
    uint32_t c = 0;
    for (int i = 0; i < wpt; ++i) {
        const int q = tid * wpt + i;
        if (q < nwb) c += (uint32_t)__popc(par[q]);
    }
    uint32_t inc = c;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[tid >> 6] = inc;
    __syncthreads();
    uint32_t base = 0, total = 0;
    for (int i = 0; i < DEEP_NT / 64; ++i) {
        base += i < (tid >> 6) ? wsum[i] : 0u;
        total += wsum[i];
    }
    uint32_t run = base + inc - c;
    for (int i = 0; i < wpt; ++i) {
        const int q = tid * wpt + i;
        if (q < nwb) {
            pre[q] = run;
            run += (uint32_t)__popc(par[q]);
        }
    }
    if (total > (uint32_t)cap || mx >= DEEP_NB) return; /* uniform: stays flagged */
    __syncthreads();
    auto rank = [&](uint32_t u) {
        return pre[u >> 5] + (uint32_t)__popc(par[u >> 5] & ((1u << (u & 31)) - 1u));
    };
    /* B: the parents' own entries (every parent is a reachable target: its own predecessor is
     * s or another parent) */
    for (int t = tid; t < n; t += DEEP_NT) {
        if (!((par[t >> 5] >> (t & 31)) & 1u)) continue;
        const uint32_t k = rank((uint32_t)t);
        const uint32_t x = dr[t];
        pd[k] = (uint16_t)x;
        pp[k] = (uint16_t)pr[t];
        pval[k] = rr[t];
        atomicAdd(&hist[x], 1u);
    }
    __syncthreads();
    /* exclusive prefix of the distance histogram (DEEP_NB / DEEP_NT buckets per thread) */
    {
        constexpr int PB = DEEP_NB / DEEP_NT;
        uint32_t loc = 0, v[PB];
#pragma unroll
        for (int k = 0; k < PB; ++k) loc += (v[k] = hist[tid * PB + k]);
        uint32_t in2 = loc;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)in2, o);
            if (lane >= o) in2 += y;
        }
        __syncthreads(); /* wsum reuse */
        if (lane == 63) wsum[tid >> 6] = in2;
        __syncthreads();
        uint32_t b2 = 0;
        for (int i = 0; i < (tid >> 6); ++i) b2 += wsum[i];
        uint32_t r2 = b2 + in2 - loc;
#pragma unroll
        for (int k = 0; k < PB; ++k) {
            hist[tid * PB + k] = r2;
            r2 += v[k];
        }
    }
    __syncthreads();
    for (int k = tid; k < (int)total; k += DEEP_NT) ord[atomicAdd(&hist[pd[k]], 1u)] = (uint16_t)k;
    __syncthreads();
    /* C: hist[x] is now the end of bucket x; bucket 1's start is 0 (no parent at distance 0) */
    uint32_t b0 = 0;
    for (uint32_t x = 1; x < mx && b0 < total; ++x) {
        const uint32_t b1 = hist[x];
        if (b1 == b0) continue; /* uniform: hist is shared */
        for (uint32_t i = b0 + tid; i < b1; i += DEEP_NT) {
            const uint32_t k = ord[i];
            const uint32_t p = pp[k];
            const double ru = (int)p == s ? 1.0 : pval[rank(p)];
            pval[k] = ru * pval[k];
        }
        b0 = b1;
        __syncthreads();
    }
    /* D: every target, in index order */
    for (int t = tid; t < n; t += DEEP_NT) {
        const uint32_t x = dr[t];
        const int p = pr[t];
        if (t == s) {
            rr[t] = 1.0;
            continue;
        }
        if (x >= SRT_INF || p < 0) continue; /* kept, as rel_sweeps_kernel keeps it */
        const double r = rr[t];
        rr[t] = (p == s ? 1.0 : pval[rank((uint32_t)p)]) * r;
    }
    if (tid == 0) {
        only[row] = 0;
        srt_max_once(max_depth, (int)mx);
    }
}

/* the rows rel_tree_kernel handed over (sweep[row] != 0) through rel_order_kernel first: the
 * sweeps then see only rows with distances past ORD_NB - 1 */
template <typename PT>
static int rel_order_launch(int n, int ld, int row0, int lrows, const uint32_t* d, const PT* pred,
                            double* rel, uint32_t* ord, int32_t* sweep, int32_t* depth,
                            hipStream_t st) {
    if (!ord || !d || lrows <= 0 || n > 65535) return SRT_OK;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipGetLastError();
    const int grid = min(srt_ceil_div(lrows, ORD_WAVES), cus * 8);
    rel_order_kernel<PT><<<grid, 64 * ORD_WAVES, 0, st>>>(n, ld, row0, lrows, d, pred, rel, ord,
                                                          sweep, depth);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

static int rel_rows_launch(int n, int ld, int row0, int lrows, const uint32_t* d, int32_t* pred,
                           double* rel, int32_t* depth, int32_t* sweep, const int32_t* srcs,
                           hipStream_t st, const uint8_t* l8 = nullptr,
                           const int16_t* pred16 = nullptr, const uint32_t* pk = nullptr,
                           const double* rtab = nullptr, int ntab = 0, uint32_t* ord = nullptr) {
    if (lrows <= 0) return SRT_OK;
    int rc;
    const bool tree = n <= 32768 && srt_form_int("reltree", 1) != 0;
    if (pk) { /* a level build's u8 rows and packed (predecessor | reliability index) rows */
        rel_tree_launch(n, ld, row0, lrows, l8, pk, rel, depth, sweep, srcs, st, rtab, ntab);
        SRT_HIPCHK(hipGetLastError());
        const size_t lds = (size_t)n * sizeof(int32_t) + 2 * (size_t)((n + 31) / 32) * 4;
        SRT_HIPCHK(hipFuncSetAttribute((const void*)rel_sweeps_kernel<uint32_t>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        rel_sweeps_kernel<uint32_t><<<lrows, 512, lds, st>>>(n, ld, row0, pk, rel, depth, sweep,
                                                             srcs);
        SRT_HIPCHK(hipGetLastError());
        return SRT_OK;
    }
    if (pred16) { /* a level build's u8 distance rows and int16 predecessor rows (n <= 32768) */
        rel_tree_launch(n, ld, row0, lrows, l8, pred16, rel, depth, sweep, srcs, st);
        SRT_HIPCHK(hipGetLastError());
        const size_t lds = (size_t)n * sizeof(int32_t) + 2 * (size_t)((n + 31) / 32) * 4;
        SRT_HIPCHK(hipFuncSetAttribute((const void*)rel_sweeps_kernel<int16_t>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        rel_sweeps_kernel<int16_t><<<lrows, 512, lds, st>>>(n, ld, row0, pred16, rel, depth, sweep,
                                                            srcs);
        SRT_HIPCHK(hipGetLastError());
        return SRT_OK;
    }
    if (tree && l8)
        rel_tree_launch(n, ld, row0, lrows, l8, (const int32_t*)pred, rel, depth, sweep, srcs, st);
    else if (tree)
        rel_tree_launch(n, ld, row0, lrows, d, (const int32_t*)pred, rel, depth, sweep, srcs, st);
    else if (n <= 1024) {
        rel_levels_kernel<256, 1024><<<lrows, 256, 2048, st>>>(n, ld, row0, d, pred, rel, 64, depth,
                                                              sweep, srcs);
    } else if (n <= 4096) {
        rel_levels_kernel<512, 4096><<<lrows, 512, 8192, st>>>(n, ld, row0, d, pred, rel, 64, depth,
                                                              sweep, srcs);
    } else if (n <= 32768) {
        SRT_HIPCHK(hipFuncSetAttribute((const void*)rel_levels_kernel<1024, 32768>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
        rel_levels_kernel<1024, 32768><<<lrows, 1024, 65536, st>>>(n, ld, row0, d, pred, rel, 64,
                                                                  depth, sweep, srcs);
    } else {
        SRT_HIPCHK(hipFuncSetAttribute((const void*)rel_levels_kernel<1024, 65536>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
        rel_levels_kernel<1024, 65536><<<lrows, 1024, 131072, st>>>(n, ld, row0, d, pred, rel, 64,
                                                                  depth, sweep, srcs);
    }
    SRT_HIPCHK(hipGetLastError());
    /* deep rows (distance range past the level passes' 64): parents only in distance order
     * (rel_deep_kernel), then what it left (more parents than its slots) one wave per row */
    if (tree && !srcs && !l8 && n <= 65535) {
        const int fixed = 8 * (ld >> 5) + 4 * DEEP_NB;
        const int cap = min(n, (160 * 1024 - 1024 - fixed) / 14) & ~63;
        const int lds = fixed + 14 * cap;
        SRT_HIPCHK(hipFuncSetAttribute((const void*)rel_deep_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        rel_deep_kernel<<<lrows, DEEP_NT, lds, st>>>(n, ld, row0, lrows, d, pred, rel, cap, sweep,
                                                     depth);
        SRT_HIPCHK(hipGetLastError());
    }
    if (tree && !srcs && !l8 &&
        (rc = rel_order_launch<int32_t>(n, ld, row0, lrows, d, pred, rel, ord, sweep, depth, st)))
        return rc;
    if (n <= 32768) {
        const size_t lds = (size_t)n * sizeof(int32_t) + 2 * (size_t)((n + 31) / 32) * 4;
        SRT_HIPCHK(hipFuncSetAttribute((const void*)rel_sweeps_kernel<int32_t>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        rel_sweeps_kernel<int32_t><<<lrows, 512, lds, st>>>(n, ld, row0, pred, rel, depth, sweep,
                                                            srcs);
        SRT_HIPCHK(hipGetLastError());
        return SRT_OK;
    }
    return srt_rel_sweeps_rows(n, lrows, row0, pred, (size_t)ld, rel, (size_t)ld, sweep, depth, st);
}

__global__ void pack_uw_kernel(int64_t arcs, const int32_t* __restrict__ col,
                               const uint32_t* __restrict__ w, uint2* __restrict__ uw,
                               const int32_t* __restrict__ dtotal) {
    if (dtotal) arcs = *dtotal;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < arcs;
         i += (int64_t)gridDim.x * blockDim.x)
        uw[i] = make_uint2((uint32_t)col[i], w[i]);
}

/* Diagonal rule (topology.c:1431-1576): min over incident OUT edges of (self-loop: L,
 * other: 2L) with the first strict minimum in (neighbor, edge) order; rel r or r^2. */
__global__ __launch_bounds__(256) void dense_diag_kernel(int n, int ld, int row0, int nrows,
                                                         const uint32_t* __restrict__ w,
                                                         const double* __restrict__ r,
                                                         uint32_t* __restrict__ d,
                                                         double* __restrict__ rel,
                                                         const int32_t* __restrict__ srcs = nullptr) {
    /* srcs: output row lr is source srcs[lr], whose edges are row srcs[lr] of the full w / r */
    const int lr = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (lr >= nrows) return;
    const int v = srcs ? srcs[lr] : row0 + lr;
    const int lane = threadIdx.x & 63;
    if (v >= n) return;
    const size_t wrow = (size_t)(srcs ? v : lr) * ld;
    const uint32_t* wr = w + wrow;
    uint64_t best = ~0ull;
    auto take = [&](uint32_t x, int u) {
        if (x >= SRT_INF) return;
        const uint64_t lat = (u == v) ? x : 2ull * x;
        const uint64_t key = (lat << 32) | (uint32_t)u;
        best = key < best ? key : best;
    };
    const int n4 = n & ~3; /* rows are 16-B aligned (ld % 64 == 0): 4 columns per load */
    for (int u = lane * 4; u < n4; u += 256) {
        const uint4 x = *reinterpret_cast<const uint4*>(wr + u);
        take(x.x, u);
        take(x.y, u + 1);
        take(x.z, u + 2);
        take(x.w, u + 3);
    }
    for (int u = n4 + lane; u < n; u += 64) take(wr[u], u);
    for (int off = 32; off > 0; off >>= 1) {
        uint64_t o = __shfl_xor(best, off);
        best = o < best ? o : best;
    }
    if (lane == 0) {
        size_t ix = (size_t)lr * ld + v;
        if (best == ~0ull) {
            d[ix] = 0;
            rel[ix] = 0.0;
        } else {
            int u = (int)(best & 0xffffffffu);
            double x = r[wrow + u];
            d[ix] = (uint32_t)(best >> 32);
            rel[ix] = (u == v) ? x : x * x;
        }
    }
}


/* ------------------------------------------------------------------------------------------ */
/* host orchestration of the dense post pass (single GPU or one row shard)                    */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    size_t n_cap, arc_cap, tarc_cap;
    int32_t *cnt, *ptr, *tptr, *cursor, *col, *tcol, *depth;
    unsigned long long* ties; /* tied-pair count of the predecessor pass */
    uint32_t *aw, *tw;
    double *ar, *tr;
    uint32_t* panel;
    size_t panel_cap;
    uint2* uw;
    size_t uw_cap;
    uint32_t* dt;   /* transpose of the local row block, then the predecessor rows */
    int32_t* predt; /* predecessors, sources across columns */
    size_t dt_cap, predt_cap;
    double* rt; /* reliability of each predecessor arc, sources across columns */
    size_t rt_cap;
    int32_t* h_total; /* pinned: the essential-arc total of a post pass that did not wait for it */
    int total_pending;
    /* time_kernels: events around the level post pass's predecessor and reliability kernels,
     * read after the build's final wait (dense_finish_rows) */
    hipEvent_t kev[4];
    int kev_on;
    int diag_done; /* the level post pass applied the diagonal rule itself */
    int pred16;    /* dt holds int16 predecessor rows (level post pass, n <= 32768; 2: packed
                    * predecessor | reliability index words) */
} dense_ws;

static dense_ws g_ws[SRT_STATE_SLOTS];

static int ws_grow(void** p, size_t* cap, size_t need, size_t elem) {
    if (*cap >= need && *p) return SRT_OK;
    if (*p) SRT_HIPCHK(hipFree(*p));
    *p = NULL;
    size_t c = need + need / 4 + 1024;
    SRT_HIPCHK(hipMalloc(p, c * elem));
    *cap = c;
    return SRT_OK;
}

static int ws_get(dense_ws** out, int n) {
    dense_ws* ws = &g_ws[srt_state_slot()];
    if (ws->n_cap < (size_t)n + 1 || !ws->cnt) {
        if (ws->cnt) {
            SRT_HIPCHK(hipFree(ws->cnt));
            SRT_HIPCHK(hipFree(ws->ptr));
            SRT_HIPCHK(hipFree(ws->tptr));
            SRT_HIPCHK(hipFree(ws->cursor));
            SRT_HIPCHK(hipFree(ws->depth));
            SRT_HIPCHK(hipFree(ws->ties));
        }
        size_t c = (size_t)n + 1;
        SRT_HIPCHK(hipMalloc(&ws->cnt, c * sizeof(int32_t)));
        SRT_HIPCHK(hipMalloc(&ws->ptr, c * sizeof(int32_t)));
        SRT_HIPCHK(hipMalloc(&ws->tptr, c * sizeof(int32_t)));
        SRT_HIPCHK(hipMalloc(&ws->cursor, c * sizeof(int32_t)));
        SRT_HIPCHK(hipMalloc(&ws->depth, sizeof(int32_t)));
        SRT_HIPCHK(hipMalloc(&ws->ties, sizeof(unsigned long long)));
        ws->n_cap = c;
    }
    *out = ws;
    return SRT_OK;
}

static int grow_arcs(dense_ws* ws, size_t need) {
    int rc;
    size_t c1 = ws->arc_cap, c2 = ws->arc_cap, c3 = ws->arc_cap;
    if ((rc = ws_grow((void**)&ws->col, &c1, need, sizeof(int32_t)))) return rc;
    if ((rc = ws_grow((void**)&ws->aw, &c2, need, sizeof(uint32_t)))) return rc;
    if ((rc = ws_grow((void**)&ws->ar, &c3, need, sizeof(double)))) return rc;
    ws->arc_cap = c1;
    return SRT_OK;
}

/* gather hook for sharded builds: makes the essential-arc counts / arcs global */
typedef int (*ess_gather_fn)(void* ctx, dense_ws* ws, int n, int phase, int32_t total,
                             hipStream_t st);

/* The post pass of a level build (levels.hip): the canonical predecessors and their arc
 * reliabilities come straight from the level planes and the sorted in-arcs (lvl_pred_kernel,
 * target-major like pred_cols*_kernel's output), so no essential-arc lists, slab transpose or
 * predecessor search over the distances; then the same row transposes and path-order reliability
 * passes as below. */
static int dense_post_levels(int32_t n, int32_t ld, int32_t row0, int32_t nrows, uint32_t* d,
                             double* rel, hipStream_t st, srt_build_stats* stats, dense_ws* ws,
                             int lrows);

static int dense_post(int32_t n, int32_t ld, int32_t row0, int32_t nrows, int32_t directed,
                      const uint32_t* w, const double* r, uint32_t* d, const uint16_t* d16,
                      double* rel, hipStream_t st, srt_build_stats* stats, ess_gather_fn gather,
                      void* gctx, int lvl = 0) {
    dense_ws* ws;
    int rc = ws_get(&ws, n);
    if (rc) return rc;
    const int lrows = max(0, min(nrows, n - row0)); /* real (non-padding) local rows */
    ws->pred16 = 0;
    if (lvl) /* the distances came from the Dial levels: predecessors from the level planes */
        return dense_post_levels(n, ld, row0, nrows, d, rel, st, stats, ws, lrows);
    SRT_HIPCHK(hipMemsetAsync(ws->cnt, 0, (size_t)(n + 1) * sizeof(int32_t), st));
    /* the exact u16 FW matrix when the build kept one: the same values in half the bytes
     * (C4: count 1.37 -> 1.08 ms, fill 1.52 -> 1.50 ms against the u32 table) */
    const bool ess16 = d16 != nullptr;
    if (lrows > 0 && ess16)
        ess_count_kernel<uint16_t><<<lrows, 256, 0, st>>>(n, ld, row0, w, d16, ws->cnt);
    else if (lrows > 0)
        ess_count_kernel<uint32_t><<<lrows, 256, 0, st>>>(n, ld, row0, w, d, ws->cnt);
    if (gather && (rc = gather(gctx, ws, n, 0, 0, st))) return rc; /* all-reduce counts */
    scan_kernel<<<1, 1024, 0, st>>>(n, ws->cnt, ws->ptr);
    SRT_HIPCHK(hipGetLastError());
    /* small graphs (n <= 2,048, one GPU) size the arc arrays for n (n - 1) arcs and let the
     * kernels read the total on the device: no host round trip in the middle of the pass */
    const bool nowait = !gather && n <= 2048;
    const int32_t* dtotal = nowait ? ws->ptr + n : nullptr;
    int32_t total = 0;
    if (nowait) {
        total = n * (n - 1);
    } else {
        SRT_HIPCHK(hipMemcpyAsync(&total, ws->ptr + n, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        SRT_HIPCHK(hipStreamSynchronize(st));
    }
    if (total < 0) {
        srt_set_error("essential-arc count overflow");
        return SRT_E_RANGE;
    }
    if ((rc = grow_arcs(ws, (size_t)total + 1))) return rc;
    if (lrows > 0) {
        if (ess16)
            ess_fill_kernel<uint16_t><<<lrows, 256, 0, st>>>(n, ld, row0, w, r, d16, ws->ptr,
                                                             ws->col, ws->aw, ws->ar);
        else
            ess_fill_kernel<uint32_t><<<lrows, 256, 0, st>>>(n, ld, row0, w, r, d, ws->ptr,
                                                             ws->col, ws->aw, ws->ar);
    }
    SRT_HIPCHK(hipGetLastError());
    if (gather && (rc = gather(gctx, ws, n, 1, total, st))) return rc; /* share the arcs */
    const int32_t *iptr = ws->ptr, *icol = ws->col;
    const uint32_t* iw = ws->aw;
    const double* ir = ws->ar;
    if (directed) {
        size_t t1 = ws->tarc_cap, t2 = ws->tarc_cap, t3 = ws->tarc_cap;
        if ((rc = ws_grow((void**)&ws->tcol, &t1, (size_t)total + 1, sizeof(int32_t)))) return rc;
        if ((rc = ws_grow((void**)&ws->tw, &t2, (size_t)total + 1, sizeof(uint32_t)))) return rc;
        if ((rc = ws_grow((void**)&ws->tr, &t3, (size_t)total + 1, sizeof(double)))) return rc;
        ws->tarc_cap = t1;
        SRT_HIPCHK(hipMemsetAsync(ws->cnt, 0, (size_t)n * sizeof(int32_t), st));
        if (total > 0)
            arc_count_by_col<<<min(srt_ceil_div(total, 256), 2048), 256, 0, st>>>(total, ws->col,
                                                                                  ws->cnt, dtotal);
        scan_kernel<<<1, 1024, 0, st>>>(n, ws->cnt, ws->tptr);
        SRT_HIPCHK(hipMemcpyAsync(ws->cursor, ws->tptr, (size_t)n * sizeof(int32_t),
                                  hipMemcpyDeviceToDevice, st));
        arc_transpose_fill<<<srt_ceil_div(n, 256), 256, 0, st>>>(n, ws->ptr, ws->col, ws->aw, ws->ar,
                                                                ws->cursor, ws->tcol, ws->tw, ws->tr);
        SRT_HIPCHK(hipGetLastError());
        iptr = ws->tptr;
        icol = ws->tcol;
        iw = ws->tw;
        ir = ws->tr;
    }
    SRT_HIPCHK(hipMemsetAsync(ws->depth, 0, sizeof(int32_t), st));
    const bool ties = stats && stats->count_ties;
    if (ties) SRT_HIPCHK(hipMemsetAsync(ws->ties, 0, sizeof(unsigned long long), st));
    if (n > srt_dense_max_n()) { /* the entry points refuse such n before FW */
        srt_set_error("dense predecessor pass supports n <= %d (n = %d)", srt_dense_max_n(), n);
        return SRT_E_RANGE;
    }
    if (lrows > 0) {
        const size_t slab = (size_t)ld * nrows;
        /* the transpose is block-major (DT[s / 64][u][s % 64]): a 64-source block's slab is
         * contiguous, so it spreads over every L2 set and fills whole lines (a row-major transpose
         * with its power-of-two stride put the slab in a few sets: 37.6 vs 30.0 ms with one line
         * of padding on C4) */
        const size_t bsD = (size_t)ld * 64;
        size_t c1 = ws->dt_cap, c2 = ws->predt_cap, c3 = ws->uw_cap;
        if ((rc = ws_grow((void**)&ws->dt, &c1, slab, sizeof(uint32_t)))) return rc;
        ws->dt_cap = c1;
        if ((rc = ws_grow((void**)&ws->predt, &c2, slab, sizeof(int32_t)))) return rc;
        ws->predt_cap = c2;
        if ((rc = ws_grow((void**)&ws->uw, &c3, (size_t)total + 1, sizeof(uint2)))) return rc;
        ws->uw_cap = c3;
        /* byte distances without the tie count take the one-minimum form (pred_cols3_kernel;
         * C4 post pass 38.1 -> 36.3 ms against pred_cols2_kernel, which the tie count keeps) */
        const bool key3 = d16 && srt_fw16_small() && !ties && n <= 32768;
        if (total > 0 && key3)
            pack_uk_kernel<<<srt_ceil_div(n, 4), 256, 0, st>>>(n, iptr, icol, iw, !directed, ws->uw);
        else if (total > 0)
            pack_uw_kernel<<<min(srt_ceil_div(total, 256), 2048), 256, 0, st>>>(total, icol, iw,
                                                                                ws->uw, dtotal);
        /* DT[u][sl] = D[row0 + sl][u], from the u16 working matrix when the build kept one
         * (half the bytes per candidate arc: the predecessor search is bound by these reads).
         * With small distances (every local one <= 64 quanta) the search also emits the arc
         * reliability and the reliability pass runs in level order in place; otherwise it emits
         * arc indices for the sweep pass. */
        const int nsb = nrows / 64;
        const int tch = max(1, min(n, 256));
        const int tper = srt_ceil_div(n, tch);
        const int grid = srt_ceil_div(nsb, 8) * 8 * tch;
        size_t c4 = ws->rt_cap;
        if ((rc = ws_grow((void**)&ws->rt, &c4, slab, sizeof(double)))) return rc;
        ws->rt_cap = c4;
        if (d16 && srt_fw16_small()) {
            /* every distance fits a byte: the transposed slab of a 64-source block is 2 MB and
             * stays in its XCD's L2 */
            uint8_t* dt8 = reinterpret_cast<uint8_t*>(ws->dt);
            const int nsb2 = srt_ceil_div(nrows, 128);
            transpose_kernel<uint16_t, uint8_t, 128><<<dim3(srt_ceil_div(ld, 64), srt_ceil_div(nrows, 64)),
                                                     256, 0, st>>>(nrows, ld, d16, (size_t)ld, dt8,
                                                                   (size_t)ld * 128);
            /* 16 candidate arcs in flight per step: 17.3 ms on C4 against 18.7 (8) and 20.0 (32);
             * streaming (non-temporal) output stores: 13.9 against 14.5 ms on C4, post pass 35.4
             * against 36.3 ms, same box */
            if (key3)
                pred_cols3_kernel<16, true><<<srt_ceil_div(nsb2, 8) * 8 * tch, 256, 0, st>>>(
                    n, row0, lrows, nrows, (size_t)ld * 128, dt8, iptr, ws->uw, ir, ws->predt, ws->rt,
                    nsb2, tch, tper, !directed);
            else if (ties)
                pred_cols2_kernel<16, true><<<srt_ceil_div(nsb2, 8) * 8 * tch, 256, 0, st>>>(
                    n, row0, lrows, nrows, (size_t)ld * 128, dt8, iptr, ws->uw, ir, ws->predt, ws->rt,
                    nsb2, tch, tper, !directed, ws->ties);
            else
                pred_cols2_kernel<16, false><<<srt_ceil_div(nsb2, 8) * 8 * tch, 256, 0, st>>>(
                    n, row0, lrows, nrows, (size_t)ld * 128, dt8, iptr, ws->uw, ir, ws->predt, ws->rt,
                    nsb2, tch, tper, !directed, ws->ties);
        } else if (d16) {
            uint16_t* dt16 = reinterpret_cast<uint16_t*>(ws->dt);
            transpose_kernel<uint16_t, uint16_t, 64><<<dim3(srt_ceil_div(ld, 64), srt_ceil_div(nrows, 64)),
                                                         256, 0, st>>>(nrows, ld, d16, (size_t)ld, dt16, bsD);
            if (ties)
                pred_cols_kernel<uint16_t, true, true><<<grid, 256, 0, st>>>(
                    n, row0, lrows, nrows, bsD, dt16, iptr, ws->uw, ir, ws->predt, ws->rt, nsb, tch,
                    tper, !directed, ws->ties);
            else
                pred_cols_kernel<uint16_t, true, false><<<grid, 256, 0, st>>>(
                    n, row0, lrows, nrows, bsD, dt16, iptr, ws->uw, ir, ws->predt, ws->rt, nsb, tch,
                    tper, !directed, ws->ties);
        } else {
            transpose_kernel<uint32_t, uint32_t, 64><<<dim3(srt_ceil_div(ld, 64), srt_ceil_div(nrows, 64)),
                                                         256, 0, st>>>(nrows, ld, d, (size_t)ld, ws->dt, bsD);
            if (ties)
                pred_cols_kernel<uint32_t, true, true><<<grid, 256, 0, st>>>(
                    n, row0, lrows, nrows, bsD, ws->dt, iptr, ws->uw, ir, ws->predt, ws->rt, nsb, tch,
                    tper, !directed, ws->ties);
            else
                pred_cols_kernel<uint32_t, true, false><<<grid, 256, 0, st>>>(
                    n, row0, lrows, nrows, bsD, ws->dt, iptr, ws->uw, ir, ws->predt, ws->rt, nsb, tch,
                    tper, !directed, ws->ties);
        }
        /* predecessor rows pred[sl][t] = predT[t][sl] (reuses the DT buffer) and the arc
         * reliabilities straight into the rel rows, where the passes below finish them in place */
        int32_t* pred = reinterpret_cast<int32_t*>(ws->dt);
        /* (streaming stores measured neutral here: these transposes already run at ~5.3 TB/s) */
        transpose_kernel<uint32_t><<<dim3(srt_ceil_div(nrows, 64), srt_ceil_div(n, 64)), 256, 0, st>>>(
            n, nrows, reinterpret_cast<const uint32_t*>(ws->predt), (size_t)nrows,
            reinterpret_cast<uint32_t*>(pred), (size_t)ld);
        transpose_kernel<double><<<dim3(srt_ceil_div(nrows, 64), srt_ceil_div(n, 64)), 256, 0, st>>>(
            n, nrows, ws->rt, (size_t)nrows, rel, (size_t)ld);
        /* level order for rows whose distances span <= 64 quanta, sweeps for the rest
         * (ws->cursor is free here and carries the per-row hand-over flags) */
        /* the target-major predecessors (predt) are free after the transpose: the order kernel's
         * per-row lists */
        if ((rc = rel_rows_launch(n, ld, row0, lrows, d, pred, rel, ws->depth, ws->cursor, nullptr,
                                  st, nullptr, nullptr, nullptr, nullptr, 0,
                                  reinterpret_cast<uint32_t*>(ws->predt))))
            return rc;
    }
    if (stats && nowait) { /* read after the build's final wait (dense_collect_total) */
        if (!ws->h_total) SRT_HIPCHK(hipHostMalloc((void**)&ws->h_total, sizeof(int32_t)));
        SRT_HIPCHK(hipMemcpyAsync(ws->h_total, ws->ptr + n, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        ws->total_pending = 1;
    } else if (stats) {
        stats->ess_arcs = total;
    }
    return SRT_OK;
}

static int dense_post_levels(int32_t n, int32_t ld, int32_t row0, int32_t nrows, uint32_t* d,
                             double* rel, hipStream_t st, srt_build_stats* stats, dense_ws* ws,
                             int lrows) {
    int rc;
    if (lrows < nrows && srt_levels_pkw_ready()) { /* the padding rows of the last shard (or a
        * shard past n): rel_pk_kernel writes the real rows only, so these take SRT_INF / 0 here,
        * as lvl_out8_kernel's rows do on the other form */
        SRT_HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d + (size_t)lrows * ld), (int)SRT_INF,
                                     (size_t)(nrows - lrows) * ld, st));
        SRT_HIPCHK(hipMemsetAsync(rel + (size_t)lrows * ld, 0, (size_t)(nrows - lrows) * ld * sizeof(double), st));
    }
    if (lrows > 0 && srt_levels_pkw_ready()) {
        /* source-major packed words (lvl_pkw_kernel) + rel_pk_kernel, which writes the u32 rows
         * too: 4 B per pair written and read between them, no transposes, no u8 rows */
        const size_t slab = (size_t)ld * nrows;
        size_t c1 = ws->dt_cap;
        if ((rc = ws_grow((void**)&ws->dt, &c1, slab, sizeof(uint32_t)))) return rc;
        ws->dt_cap = c1;
        const bool ties = stats && stats->count_ties;
        if (ties) SRT_HIPCHK(hipMemsetAsync(ws->ties, 0, sizeof(unsigned long long), st));
        const bool kt = stats && stats->time_kernels;
        if (kt && !ws->kev[0])
            for (int i = 0; i < 4; i++) SRT_HIPCHK(hipEventCreate(&ws->kev[i]));
        int ntab = 0;
        const double* rtab = srt_levels_rtab(&ntab);
        if (stats) stats->rel_table = ntab;
        uint32_t* pk = reinterpret_cast<uint32_t*>(ws->dt);
        if (kt) SRT_HIPCHK(hipEventRecord(ws->kev[0], st));
        {   /* target-major packed words (with the level), then one u32 transpose */
            size_t c2 = ws->predt_cap;
            if ((rc = ws_grow((void**)&ws->predt, &c2, slab, sizeof(int32_t)))) return rc;
            ws->predt_cap = c2;
            if ((rc = srt_levels_pred(ws->predt, 2, nullptr, (size_t)nrows, ties ? ws->ties : NULL,
                                      st)))
                return rc;
        }
        if (kt) SRT_HIPCHK(hipEventRecord(ws->kev[1], st));
        transpose_kernel<uint32_t><<<dim3(srt_ceil_div(nrows, 64), srt_ceil_div(n, 64)), 256, 0, st>>>(
                n, nrows, reinterpret_cast<const uint32_t*>(ws->predt), (size_t)nrows, pk, (size_t)ld);
        ws->pred16 = 2; /* dense_path_ms reads the packed words' low half */
        SRT_HIPCHK(hipMemsetAsync(ws->depth, 0, sizeof(int32_t), st));
        if (kt) SRT_HIPCHK(hipEventRecord(ws->kev[2], st));
        if ((rc = rel_pk_launch(n, ld, row0, lrows, pk, d, rel, rtab, ntab, ws->depth, ws->cursor,
                                st)))
            return rc;
        if (kt) {
            SRT_HIPCHK(hipEventRecord(ws->kev[3], st));
            ws->kev_on = 1;
        }
        if ((rc = srt_levels_diag(n, ld, d, rel, st, &ws->diag_done))) return rc;
    } else if (lrows > 0) {
        const size_t slab = (size_t)ld * nrows;
        size_t c1 = ws->dt_cap, c2 = ws->predt_cap, c4 = ws->rt_cap;
        if ((rc = ws_grow((void**)&ws->dt, &c1, slab, sizeof(uint32_t)))) return rc;
        ws->dt_cap = c1;
        if ((rc = ws_grow((void**)&ws->predt, &c2, slab, sizeof(int32_t)))) return rc;
        ws->predt_cap = c2;
        if ((rc = ws_grow((void**)&ws->rt, &c4, slab, sizeof(double)))) return rc;
        ws->rt_cap = c4;
        const bool ties = stats && stats->count_ties;
        if (ties) SRT_HIPCHK(hipMemsetAsync(ws->ties, 0, sizeof(unsigned long long), st));
        const bool kt = stats && stats->time_kernels;
        if (kt && !ws->kev[0])
            for (int i = 0; i < 4; i++) SRT_HIPCHK(hipEventCreate(&ws->kev[i]));
        if (kt) SRT_HIPCHK(hipEventRecord(ws->kev[0], st));
        /* int16 predecessors while every vertex fits (half the slab's bytes), widened by the
         * transpose into the int32 rows the reliability passes read; with the build's table of
         * distinct arc reliabilities, one packed word per pair (predecessor | index << 16): 4 B
         * written, transposed and read instead of 2 + 8 */
        int ntab = 0;
        const double* rtab = n <= 32768 ? srt_levels_rtab(&ntab) : nullptr;
        const int p16 = rtab ? 2 : n <= 32768;
        if (stats) stats->rel_table = rtab ? ntab : 0;
        if ((rc = srt_levels_pred(ws->predt, p16, ws->rt, (size_t)nrows, ties ? ws->ties : NULL, st)))
            return rc;
        if (kt) SRT_HIPCHK(hipEventRecord(ws->kev[1], st));
        int32_t* pred = reinterpret_cast<int32_t*>(ws->dt);
        int16_t* pred16 = p16 == 1 ? reinterpret_cast<int16_t*>(ws->dt) : nullptr;
        uint32_t* pk = p16 == 2 ? reinterpret_cast<uint32_t*>(ws->dt) : nullptr;
        ws->pred16 = p16;
        if (pk)
            transpose_kernel<uint32_t><<<dim3(srt_ceil_div(nrows, 64), srt_ceil_div(n, 64)), 256, 0, st>>>(
                n, nrows, reinterpret_cast<const uint32_t*>(ws->predt), (size_t)nrows, pk, (size_t)ld);
        else if (p16) /* int16 rows: the reliability passes read them as they are */
            transpose_kernel<int16_t><<<dim3(srt_ceil_div(nrows, 64), srt_ceil_div(n, 64)), 256, 0, st>>>(
                n, nrows, reinterpret_cast<const int16_t*>(ws->predt), (size_t)nrows, pred16, (size_t)ld);
        else
            transpose_kernel<uint32_t><<<dim3(srt_ceil_div(nrows, 64), srt_ceil_div(n, 64)), 256, 0, st>>>(
                n, nrows, reinterpret_cast<const uint32_t*>(ws->predt), (size_t)nrows,
                reinterpret_cast<uint32_t*>(pred), (size_t)ld);
        if (!pk)
            transpose_kernel<double><<<dim3(srt_ceil_div(nrows, 64), srt_ceil_div(n, 64)), 256, 0, st>>>(
                n, nrows, ws->rt, (size_t)nrows, rel, (size_t)ld);
        SRT_HIPCHK(hipMemsetAsync(ws->depth, 0, sizeof(int32_t), st));
        /* every level-built distance is <= 254 quanta: level order in place for every row that
         * spans <= 64 quanta, sweeps for the rest (as dense_post); the level rows as u8 */
        if (kt) SRT_HIPCHK(hipEventRecord(ws->kev[2], st));
        if ((rc = rel_rows_launch(n, ld, row0, lrows, d, pred, rel, ws->depth, ws->cursor, nullptr,
                                  st, srt_levels_l8(), pred16, pk, rtab, ntab)))
            return rc;
        if (kt) {
            SRT_HIPCHK(hipEventRecord(ws->kev[3], st));
            ws->kev_on = 1;
        }
        /* the diagonal rule from the keys the level build's count pass took (no second read
         * of the w rows); directed builds keep dense_diag_kernel */
        if ((rc = srt_levels_diag(n, ld, d, rel, st, &ws->diag_done))) return rc;
    }
    srt_levels_release(st);
    if (stats) stats->ess_arcs = 0; /* no essential-arc lists in this form */
    return SRT_OK;
}

/* the essential-arc total of a post pass that did not wait for it (after the stream's work) */
static void dense_collect_total(int32_t n, srt_build_stats* stats) {
    dense_ws* ws;
    if (!stats || ws_get(&ws, n) || !ws->total_pending) return;
    stats->ess_arcs = *ws->h_total;
    ws->total_pending = 0;
}

static int dense_finish_rows(int32_t n, int32_t ld, int32_t row0, int32_t nrows, const uint32_t* w,
                             const double* r, uint32_t* d, double* rel, hipStream_t st,
                             srt_build_stats* stats) {
    const int lrows = max(0, min(nrows, n - row0));
    dense_ws* wsd;
    int rcw = ws_get(&wsd, n);
    if (rcw) return rcw;
    if (lrows > 0 && !wsd->diag_done)
        dense_diag_kernel<<<srt_ceil_div(lrows, 4), 256, 0, st>>>(n, ld, row0, lrows, w, r, d, rel);
    wsd->diag_done = 0;
    SRT_HIPCHK(hipGetLastError());
    if (stats) {
        dense_ws* ws;
        int rc = ws_get(&ws, n);
        if (rc) return rc;
        int32_t depth = 0;
        unsigned long long nt = 0;
        SRT_HIPCHK(hipMemcpyAsync(&depth, ws->depth, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        if (stats->count_ties)
            SRT_HIPCHK(hipMemcpyAsync(&nt, ws->ties, sizeof(nt), hipMemcpyDeviceToHost, st));
        SRT_HIPCHK(hipStreamSynchronize(st));
        stats->max_depth = depth;
        stats->tied_pairs = (int64_t)nt;
        dense_collect_total(n, stats);
        if (ws->kev_on) {
            float a = 0, b = 0;
            SRT_HIPCHK(hipEventElapsedTime(&a, ws->kev[0], ws->kev[1]));
            SRT_HIPCHK(hipEventElapsedTime(&b, ws->kev[2], ws->kev[3]));
            stats->ms_pred = a;
            stats->ms_rel = b;
            ws->kev_on = 0;
        }
    }
    return SRT_OK;
}

/* ---- a few source rows on a dense graph (srt_dense_rows_build_device) ---------------------- */
/* The canonical predecessor of (source row i, target t) is argmin over u with
 * D[i][u] + W[u][t] == D[i][t] of (D[i][u], u) -- pred_cols_kernel's rule. Without every row of D
 * the essential-arc filter is not available; an arc can only be tight for some row if
 * W[u][t] <= max_i D[i][t], which keeps a few percent of a complete graph's arcs (distances are a
 * few hops of the shortest arcs). Those candidates are listed per target (CSR over t, u
 * ascending), the rows are transposed 64 sources to a 128-byte line, and one wave per (t, source
 * block) walks t's candidates with the sources across its lanes, as pred_cols2_kernel does. */
#define ROWS_CAP 0x3DFFu
__global__ void rows_maxd_kernel(int nsub, int ld, const uint16_t* __restrict__ ds,
                                 uint32_t* __restrict__ maxd) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ld) return;
    uint32_t m = 0;
    for (int i = 0; i < nsub; ++i) {
        const uint32_t d = ds[(size_t)i * ld + t];
        if (d < ROWS_CAP && d > m) m = d;
    }
    maxd[t] = m;
}

/* one wave per target t: wt row t is column t of W (the u16 matrix itself when W is symmetric);
 * FILL = 0 counts the candidates u != t with W[u][t] <= maxd[t], FILL = 1 writes them in order */
template <bool FILL>
__global__ __launch_bounds__(256) void rows_cand_kernel(int n, int ld, const uint16_t* __restrict__ wt,
                                                       const uint32_t* __restrict__ maxd,
                                                       int32_t* __restrict__ cnt,
                                                       const int32_t* __restrict__ ptr,
                                                       uint32_t* __restrict__ cand) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (t >= n) return;
    const uint32_t lim = maxd[t];
    const uint16_t* row = wt + (size_t)t * ld;
    int base = FILL ? ptr[t] : 0;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int u0 = 0; u0 < n; u0 += 512) {
        const int u = u0 + lane * 8;
        uint4 v = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (u < ld) v = *reinterpret_cast<const uint4*>(row + u);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
        uint32_t m = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t w = (w4[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
            if (u + q < n && u + q != t && w <= lim) m |= 1u << q;
        }
        const int c = __popc(m);
        /* a lane's count (0..8) in four ballots: its exclusive prefix is four masked popcounts */
        int pre = 0, tot = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint64_t bal = __ballot((c >> b) & 1);
            pre += __popcll(bal & lt) << b;
            tot += __popcll(bal) << b;
        }
        if (FILL) {
            int o = base + pre;
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if ((m >> q) & 1u) {
                    const uint32_t w = (w4[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
                    cand[o++] = (uint32_t)(u + q) | (w << 16);
                }
        }
        base += tot;
    }
    if (!FILL && lane == 0) cnt[t] = base;
}

/* DT[b][u][l] = ds[b * 64 + l][u] (rows past nsub: the cap) */
__global__ void rows_dt_kernel(int nsub, int ld, const uint16_t* __restrict__ ds,
                               uint16_t* __restrict__ dt) {
    const int l = threadIdx.x & 63, b = blockIdx.y;
    const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (u >= ld) return;
    const int i = b * 64 + l;
    dt[((size_t)b * ld + u) * 64 + l] = i < nsub ? ds[(size_t)i * ld + u] : (uint16_t)ROWS_CAP;
}

template <bool TIES>
__global__ __launch_bounds__(256) void rows_pred_kernel(int n, int ld, int nsub,
                                                        const int32_t* __restrict__ verts,
                                                        const uint16_t* __restrict__ dt,
                                                        const int32_t* __restrict__ ptr,
                                                        const uint32_t* __restrict__ cand,
                                                        const double* __restrict__ r,
                                                        int32_t* __restrict__ pred,
                                                        double* __restrict__ rel,
                                                        unsigned long long* __restrict__ ties) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63, b = blockIdx.y;
    if (t >= n) return;
    const int i = b * 64 + lane;
    const uint16_t* db = dt + (size_t)b * ld * 64 + lane;
    const uint32_t tgt = db[(size_t)t * 64];
    uint32_t best = 0xFFFFFFFFu, tie = 0;
    const int e = ptr[t + 1];
    for (int j0 = ptr[t]; j0 < e; j0 += 8) {
        uint32_t cu[8], d[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) cu[q] = j0 + q < e ? cand[j0 + q] : 0xFFFFFFFFu;
#pragma unroll
        for (int q = 0; q < 8; ++q) d[q] = cu[q] != 0xFFFFFFFFu ? db[(size_t)(cu[q] & 0xFFFFu) * 64] : 0xFFFFu;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (cu[q] == 0xFFFFFFFFu || d[q] + (cu[q] >> 16) != tgt) continue;
            const uint32_t key = (d[q] << 16) | (cu[q] & 0xFFFFu);
            if (TIES && ((key ^ best) >> 16) == 0) tie = 1;
            if (key < best) {
                if (TIES && (key >> 16) < (best >> 16)) tie = 0;
                best = key;
            }
        }
    }
    if (i >= nsub) return;
    const int s = verts[i];
    const bool has = best != 0xFFFFFFFFu && t != s;
    const int u = has ? (int)(best & 0xFFFFu) : -1;
    pred[(size_t)i * ld + t] = u;
    rel[(size_t)i * ld + t] = has ? r[(size_t)u * ld + t] : 0.0;
    if (TIES) {
        const uint64_t tb = __ballot(has && tie);
        if (lane == 0 && tb) atomicAdd(ties, (unsigned long long)__popcll(tb));
    }
}

/* Tables of nsub sources (device list dverts, host copy hverts) on a dense graph without the
 * all-pairs FW: distance rows by Bellman-Ford passes (srt_fw16_rows), canonical predecessors
 * (rows_pred_kernel), path-order reliability (rel_levels_kernel / rel_sweeps_kernel), the diagonal
 * rule and, with lat_ms, the f64 path-order ms rows. Rows are full width (ld); *used = 0 (and
 * nothing written) when a distance reaches the u16 cap or n is beyond the LDS forms -- the caller
 * then runs the FW. w, r: ld x ld device matrices. */
int srt_dense_rows_build_device(int32_t n, int32_t ld, int32_t nsub, const int32_t* dverts,
                                const uint32_t* w, const double* r, uint32_t* lat_rows,
                                double* rel_rows, double* lms_rows, uint64_t quantum_ns,
                                int32_t directed, hipStream_t st, srt_build_stats* stats, int* used) {
    *used = 0;
    if (n > 32768 || ld % 128 || nsub < 1 || nsub > n) return SRT_OK;
    const int nsp = srt_ceil_div(nsub, 128) * 128, nb64 = srt_ceil_div(nsub, 64);
    struct scratch {
        void* p[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
        hipStream_t s;
        ~scratch() {
            for (void* x : p)
                if (x) (void)hipFreeAsync(x, s);
        }
        int get(int k, size_t bytes) {
            if (srt_malloc_async(&p[k], bytes ? bytes : 16, s) != hipSuccess) {
                (void)hipGetLastError();
                srt_set_error("dense rows build: scratch of %zu MiB failed", bytes >> 20);
                return SRT_E_NOMEM;
            }
            return SRT_OK;
        }
    } sc;
    sc.s = st;
    int rc;
    if ((rc = sc.get(0, (size_t)ld * ld * sizeof(uint16_t))) ||
        (rc = sc.get(1, (size_t)nsp * ld * sizeof(uint16_t))) ||
        (rc = sc.get(2, ((size_t)ld * nsub + 2 * (size_t)nsub + 2) * sizeof(int32_t))) ||
        (rc = sc.get(3, sizeof(unsigned long long))) ||
        (rc = sc.get(4, (size_t)nb64 * ld * 64 * sizeof(uint16_t))) ||
        (rc = sc.get(5, (size_t)(3 * ld + 3) * sizeof(int32_t))))
        return rc;
    uint16_t* w16 = (uint16_t*)sc.p[0];
    uint16_t* ds = (uint16_t*)sc.p[1];
    int32_t* pred = (int32_t*)sc.p[2];
    int32_t* sweep = pred + (size_t)ld * nsub;
    int32_t* depth = sweep + nsub;
    unsigned long long* ties = (unsigned long long*)sc.p[3];
    uint16_t* dt = (uint16_t*)sc.p[4];
    uint32_t* maxd = (uint32_t*)sc.p[5];
    int32_t* ccnt = (int32_t*)sc.p[5] + ld;
    int32_t* ptr = ccnt + ld + 1; /* n + 1 candidate offsets */
    hipEvent_t e0, e1, e2;
    SRT_HIPCHK(hipEventCreate(&e0));
    SRT_HIPCHK(hipEventCreate(&e1));
    SRT_HIPCHK(hipEventCreate(&e2));
    struct evs {
        hipEvent_t* e[3];
        ~evs() {
            for (hipEvent_t* x : e) (void)hipEventDestroy(*x);
        }
    } ev{{&e0, &e1, &e2}};
    SRT_HIPCHK(hipEventRecord(e0, st));
    int exact = 0, small = 0, passes = 0;
    rc = srt_fw16_rows(n, ld, nsub, dverts, w, w16, ds, lat_rows, st, &exact, &small, &passes);
    if (rc) return rc;
    if (!exact) return SRT_OK; /* a distance at the u16 cap: the FW's wider tiers take it */
    SRT_HIPCHK(hipEventRecord(e1, st));
    const bool ct = stats && stats->count_ties;
    SRT_HIPCHK(hipMemsetAsync(ties, 0, sizeof(unsigned long long), st));
    SRT_HIPCHK(hipMemsetAsync(depth, 0, sizeof(int32_t), st));
    /* candidate arcs per target: column t of W is row t of W (symmetric) or of its transpose */
    const uint16_t* wt = w16;
    if (directed) {
        if ((rc = sc.get(6, (size_t)ld * ld * sizeof(uint16_t)))) return rc;
        transpose_kernel<uint16_t><<<dim3(ld / 64, ld / 64), 256, 0, st>>>(ld, ld, w16, (size_t)ld,
                                                                           (uint16_t*)sc.p[6],
                                                                           (size_t)ld);
        wt = (const uint16_t*)sc.p[6];
    }
    rows_maxd_kernel<<<srt_ceil_div(ld, 256), 256, 0, st>>>(nsub, ld, ds, maxd);
    rows_cand_kernel<false><<<srt_ceil_div(n, 4), 256, 0, st>>>(n, ld, wt, maxd, ccnt, NULL, NULL);
    scan_kernel<<<1, 1024, 0, st>>>(n, ccnt, ptr);
    SRT_HIPCHK(hipGetLastError());
    int32_t total = 0;
    SRT_HIPCHK(hipMemcpyAsync(&total, ptr + n, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    SRT_HIPCHK(hipStreamSynchronize(st));
    if ((rc = sc.get(7, ((size_t)total + 1) * sizeof(uint32_t)))) return rc;
    uint32_t* cand = (uint32_t*)sc.p[7];
    rows_cand_kernel<true><<<srt_ceil_div(n, 4), 256, 0, st>>>(n, ld, wt, maxd, NULL, ptr, cand);
    rows_dt_kernel<<<dim3(ld / 4, nb64), 256, 0, st>>>(nsub, ld, ds, dt);
    dim3 pg(srt_ceil_div(n, 4), nb64);
    if (ct)
        rows_pred_kernel<true><<<pg, 256, 0, st>>>(n, ld, nsub, dverts, dt, ptr, cand, r, pred,
                                                    rel_rows, ties);
    else
        rows_pred_kernel<false><<<pg, 256, 0, st>>>(n, ld, nsub, dverts, dt, ptr, cand, r, pred,
                                                     rel_rows, ties);
    SRT_HIPCHK(hipGetLastError());
    if ((rc = rel_rows_launch(n, ld, 0, nsub, lat_rows, pred, rel_rows, depth, sweep, dverts, st)))
        return rc;
    dense_diag_kernel<<<srt_ceil_div(nsub, 4), 256, 0, st>>>(n, ld, 0, nsub, w, r, lat_rows, rel_rows,
                                                             dverts);
    SRT_HIPCHK(hipGetLastError());
    if (lms_rows &&
        (rc = srt_path_ms_rows(n, nsub, dverts, 0, lat_rows, (size_t)ld, pred, (size_t)ld, NULL, NULL,
                               NULL, quantum_ns, lms_rows, (size_t)ld, st)))
        return rc;
    SRT_HIPCHK(hipEventRecord(e2, st));
    SRT_HIPCHK(hipEventSynchronize(e2));
    if (stats) {
        float a = 0, b = 0;
        SRT_HIPCHK(hipEventElapsedTime(&a, e0, e1));
        SRT_HIPCHK(hipEventElapsedTime(&b, e1, e2));
        unsigned long long nt = 0;
        int32_t dep = 0;
        SRT_HIPCHK(hipMemcpy(&nt, ties, sizeof(nt), hipMemcpyDeviceToHost));
        SRT_HIPCHK(hipMemcpy(&dep, depth, sizeof(dep), hipMemcpyDeviceToHost));
        stats->algo = SRT_ALGO_DENSE_FW;
        stats->dist_enc = SRT_DENC_ROWS;
        stats->fw_block = passes; /* dense rows builds: the Bellman-Ford passes */
        stats->ms_fw = a;
        stats->ms_post = b;
        stats->ms_total = a + b;
        stats->n_update = passes;
        stats->ms_update = a;
        stats->max_depth = dep;
        stats->tied_pairs = ct ? (int64_t)nt : 0;
        stats->ess_arcs = total; /* dense rows builds: the candidate arcs */
    }
    *used = 1;
    return SRT_OK;
}

extern "C" int srt_dense_rows_build(int32_t n, int32_t ld, int32_t nsub, const int32_t* dverts,
                                    const uint32_t* w, const double* r, uint32_t* lat_rows,
                                    double* rel_rows, void* stream, srt_build_stats* stats) {
    if (n <= 0 || ld < n || ld % 128 || nsub < 1 || !dverts || !w || !r || !lat_rows || !rel_rows) {
        srt_set_error("srt_dense_rows_build: bad arguments");
        return SRT_E_ARG;
    }
    int used = 0;
    /* symmetric w assumed unknown here: the candidate lists come from the transpose */
    const int rc = srt_dense_rows_build_device(n, ld, nsub, dverts, w, r, lat_rows, rel_rows, NULL, 0,
                                               1, (hipStream_t)stream, stats, &used);
    if (rc) return rc;
    if (!used) {
        srt_set_error("srt_dense_rows_build: n = %d beyond 32768 or a distance at the u16 cap", n);
        return SRT_E_RANGE;
    }
    return SRT_OK;
}

int srt_dense_post_device(int32_t n, int32_t ld, int32_t directed, const uint32_t* w, const double* r,
                          uint32_t* d, const uint16_t* d16, double* rel, hipStream_t st,
                          srt_build_stats* stats, int lvl) {
    int rc = dense_post(n, ld, 0, ld, directed, w, r, d, d16, rel, st, stats, NULL, NULL, lvl);
    if (rc) return rc;
    return dense_finish_rows(n, ld, 0, ld, w, r, d, rel, st, stats);
}

/* ------------------------------------------------------------------------------------------ */
/* public device-resident dense build                                                         */
/* ------------------------------------------------------------------------------------------ */
extern "C" int srt_dense_max_n(void) { return SRT_DENSE_MAX_N; }

/* HIP events of one build, released on every return path */
struct build_events {
    hipEvent_t e[3] = {nullptr, nullptr, nullptr};
    ~build_events() {
        for (hipEvent_t x : e)
            if (x) (void)hipEventDestroy(x);
    }
    int create() {
        for (hipEvent_t& x : e) SRT_HIPCHK(hipEventCreate(&x));
        return SRT_OK;
    }
};

/* f64 path-order ms rows [row0, row0 + lrows) from the predecessor rows the post pass left in the
 * workspace (tables.hip); runs after the diagonal rule */
template <typename T>
__global__ void widen16_kernel(size_t cnt, const T* __restrict__ in, int32_t* __restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt;
         i += (size_t)gridDim.x * blockDim.x)
        out[i] = (int16_t)(in[i] & 0xFFFF); /* int16 rows, or the packed words' low half */
}

static int dense_path_ms(int32_t n, int32_t ld, int32_t row0, int32_t nrows, const uint32_t* d,
                         uint64_t q, double* lms, hipStream_t st) {
    const int lrows = max(0, min(nrows, n - row0));
    if (lrows == 0) return SRT_OK;
    dense_ws* ws;
    int rc = ws_get(&ws, n);
    if (rc) return rc;
    const int32_t* pred = reinterpret_cast<const int32_t*>(ws->dt);
    if (ws->pred16) { /* the level post pass left int16 rows: widened into the free slab */
        const size_t cnt = (size_t)lrows * ld;
        const int64_t nb = srt_ceil_div((int64_t)cnt, 256);
        const unsigned g = (unsigned)(nb < 65536 ? nb : 65536);
        if (ws->pred16 == 2)
            widen16_kernel<uint32_t><<<g, 256, 0, st>>>(cnt, reinterpret_cast<const uint32_t*>(ws->dt),
                                                        ws->predt);
        else
            widen16_kernel<int16_t><<<g, 256, 0, st>>>(cnt, reinterpret_cast<const int16_t*>(ws->dt),
                                                       ws->predt);
        SRT_HIPCHK(hipGetLastError());
        pred = ws->predt;
    }
    return srt_path_ms_rows(n, lrows, NULL, row0, d, (size_t)ld, pred, (size_t)ld, NULL, NULL, NULL, q,
                            lms, (size_t)ld, st);
}

/* Dial levels (levels.hip) instead of the FW when the graph's distances are small enough for the
 * level budget to beat the FW's predicted time (61 T relaxations/s, the measured update rate;
 * symmetric rounds do half the relaxations, plus the rounds' chain). n >= 4,096: below that the
 * FW's squaring or rounds
 * cost less than the levels' launches. SRT_FORM levels=0 keeps the FW, =1 tries the levels at any
 * size. *exact = 1 when the levels settled every pair (the u16 matrix and lat rows are final). */
static int dense_try_levels(const srt_comm* comm, int n, int ld, int row0, int nrows, int directed,
                            const uint32_t* w_rows, const double* r_rows, uint32_t* lat_rows,
                            hipStream_t st,
                            evpool_t* evp, srt_build_stats* stats, int* exact) {
    *exact = 0;
    const int mode = srt_form_int("levels", -1);
    if (mode == 0 || (mode < 0 && n < 4096) || ld % 128) return SRT_OK;
    /* relaxations at the update's rate + ~50 us of round chain per 128 pivots, for the largest
     * shard (the same on every rank; srt_levels_build also agrees the budget by a min all-reduce) */
    int max_rows = nrows;
    const int R = comm ? srt_comm_size(comm) : 1;
    for (int q = 0; q < R && R > 1; q++) {
        int32_t qb = 0, qe = 0;
        srt_shard_rows(ld, SRT_SHARD_ALIGN, R, q, &qb, &qe);
        max_rows = max(max_rows, qe - qb);
    }
    const double fw_ms = (double)max_rows * ld * ld / (directed ? 1.0 : 2.0) / 6.1e10 + ld / 128 * 0.05;
    if (evp) {
        evp->used = 0;
        evp->group = 2;
    }
    int nlev = 0;
    int64_t bytes = 0;
    const int rc = srt_fw16_levels(comm, n, ld, row0, nrows, directed, w_rows, r_rows, lat_rows, st, evp,
                                   mode > 0 ? 1e30 : fw_ms, &nlev, &bytes);
    if (rc) return rc;
    if (stats) {
        stats->levels = nlev;
        stats->work_bytes = nlev ? bytes : 0;
    }
    *exact = nlev > 0;
    return SRT_OK;
}

int srt_dense_build_device_ms(int32_t n, int32_t ld, int32_t directed, const uint32_t* w,
                              const double* r, uint32_t* lat, double* rel, double* lat_ms,
                              uint64_t quantum_ns, hipStream_t st, int32_t fw_block,
                              srt_build_stats* stats) {
    if (n <= 0 || ld < n || ld % B || !w || !r || !lat || !rel) {
        srt_set_error("srt_dense_build_device: bad arguments (n=%d ld=%d)", n, ld);
        return SRT_E_ARG;
    }
    if (n > srt_dense_max_n()) { /* refused before any FW round runs */
        srt_set_error("dense build supports n <= %d (n = %d); use the sparse SSSP", srt_dense_max_n(), n);
        return SRT_E_RANGE;
    }
    if (fw_block != 0 && fw_block != B) {
        srt_set_error("srt_dense_build_device: fw_block must be 0 or %d", B);
        return SRT_E_ARG;
    }
    build_events ev;
    int rc = ev.create();
    if (rc) return rc;
    hipEvent_t e0 = ev.e[0], e1 = ev.e[1], e2 = ev.e[2];
    SRT_HIPCHK(hipEventRecord(e0, st));
    evpool_t* evp = NULL;
    if (stats && stats->time_kernels && (rc = evpool_begin(&evp, ld / B))) return rc;
    /* narrowest exact encoding first: Dial levels (small distances) -> f16-compare u16 -> pk_min
     * u16 -> u32 */
    int exact = 0, enc = SRT_DENC_U32;
    if ((rc = dense_try_levels(NULL, n, ld, 0, ld, directed, w, r, lat, st, evp, stats, &exact)))
        return rc;
    if (exact) enc = SRT_DENC_LEVELS;
    for (int fm = 1; fm >= 0 && !exact && ld % 128 == 0; --fm) {
        if (evp) {
            evp->used = 0;
            evp->group = 2;
        }
        int sym = !directed;
        rc = srt_fw16_build(n, ld, 0, ld, w, lat, st, evp, NULL, NULL, NULL, 0, fm, &sym, &exact);
        if (rc) return rc;
        if (exact)
            enc = !fm ? SRT_DENC_U16
                      : sym == 5 ? SRT_DENC_SQUARE
                      : sym == 4 ? SRT_DENC_F16CMP_SYM256
                      : sym == 3 ? SRT_DENC_F16CMP_SYM128
                      : sym == 2 ? SRT_DENC_F16CMP_SYM2
                                 : sym ? SRT_DENC_F16CMP_SYM : SRT_DENC_F16CMP;
    }
    if (!exact) { /* u32 path: ld not a multiple of 128, or a distance reached 0x7FFF quanta */
        if (evp) {
            evp->used = 0;
            evp->group = 2;
        }
        dim3 g(srt_ceil_div(ld, 256), ld);
        init_dist_kernel<<<g, 256, 0, st>>>(n, ld, 0, w, lat);
        SRT_HIPCHK(hipGetLastError());
        rc = srt_dense_fw_device(n, ld, lat, st, evp);
        if (rc) return rc;
    }
    SRT_HIPCHK(hipEventRecord(e1, st));
    rc = srt_dense_post_device(n, ld, directed, w, r, lat, exact ? srt_fw16_matrix() : NULL, rel,
                               st, stats, enc == SRT_DENC_LEVELS);
    if (rc) return rc;
    if (lat_ms) {
        if ((rc = dense_path_ms(n, ld, 0, ld, lat, quantum_ns, lat_ms, st))) return rc;
    }
    SRT_HIPCHK(hipEventRecord(e2, st));
    if (stats) {
        SRT_HIPCHK(hipEventSynchronize(e2));
        float a = 0, b = 0;
        SRT_HIPCHK(hipEventElapsedTime(&a, e0, e1));
        SRT_HIPCHK(hipEventElapsedTime(&b, e1, e2));
        stats->algo = SRT_ALGO_DENSE_FW;
        stats->fw_block = B;
        stats->dist_enc = enc;
        stats->ms_fw = a;
        stats->ms_post = b;
        stats->ms_total = a + b;
        if (evp && (rc = evpool_sum(evp, e2, stats))) return rc;
    }
    return SRT_OK;
}

extern "C" int srt_dense_build_device(int32_t n, int32_t ld, int32_t directed, const uint32_t* w,
                                      const double* r, uint32_t* lat, double* rel, void* stream,
                                      int32_t fw_block, srt_build_stats* stats) {
    return srt_dense_build_device_ms(n, ld, directed, w, r, lat, rel, NULL, 0, (hipStream_t)stream,
                                     fw_block, stats);
}

/* ------------------------------------------------------------------------------------------ */
/* row-sharded dense build over RCCL (one process per GPU)                                    */
/* ------------------------------------------------------------------------------------------ */
/* collectives: srt_coll_* (comm.hip) -- RCCL, or virtual ranks sharing one device */

typedef struct {
    const srt_comm* comm;
    int ld;
} shard_ctx;

static int shard_owner(void* vctx, int k0) {
    const shard_ctx* ctx = (const shard_ctx*)vctx;
    const int R = srt_comm_size(ctx->comm);
    for (int q = 0; q < R; q++) {
        int32_t qb, qe;
        srt_shard_rows(ctx->ld, SRT_SHARD_ALIGN, R, q, &qb, &qe);
        if (k0 >= qb && k0 < qe) return q;
    }
    return 0;
}

static int shard_bcast(void* vctx, void* panel, size_t bytes, int owner, hipStream_t st) {
    const shard_ctx* ctx = (const shard_ctx*)vctx;
    return srt_coll_bcast(ctx->comm, panel, bytes, owner, st);
}

static int shard_gather(void* vctx, dense_ws* ws, int n, int phase, int32_t total, hipStream_t st) {
    (void)total;
    shard_ctx* ctx = (shard_ctx*)vctx;
    const int R = srt_comm_size(ctx->comm);
    if (phase == 0) /* counts are zero outside each rank's rows: a sum all-reduce assembles them */
        return srt_coll_allreduce_i32(ctx->comm, ws->cnt, (size_t)n, 0, st);
    /* every rank filled its own rows' contiguous arc segment: broadcast each segment */
    int32_t* hptr = (int32_t*)malloc((size_t)(n + 1) * sizeof(int32_t));
    if (!hptr) return SRT_E_NOMEM;
    if (hipMemcpyAsync(hptr, ws->ptr, (size_t)(n + 1) * sizeof(int32_t), hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
        free(hptr);
        srt_set_error("hipMemcpy of the essential-arc offsets failed");
        return SRT_E_DEVICE;
    }
    int rc = srt_coll_group_begin(ctx->comm);
    for (int q = 0; q < R && !rc; q++) {
        int32_t b, e;
        srt_shard_rows(ctx->ld, SRT_SHARD_ALIGN, R, q, &b, &e);
        b = min(b, n);
        e = min(e, n);
        const size_t o = (size_t)hptr[b], c = (size_t)(hptr[e] - hptr[b]);
        if (c == 0) continue;
        rc = srt_coll_bcast(ctx->comm, ws->col + o, c * sizeof(int32_t), q, st);
        if (!rc) rc = srt_coll_bcast(ctx->comm, ws->aw + o, c * sizeof(uint32_t), q, st);
        if (!rc) rc = srt_coll_bcast(ctx->comm, ws->ar + o, c * sizeof(double), q, st);
    }
    const int rc2 = srt_coll_group_end(ctx->comm);
    free(hptr);
    return rc ? rc : rc2;
}

int srt_dense_build_sharded_ms(srt_comm* comm, int32_t n, int32_t ld, int32_t directed,
                               const uint32_t* w_rows, const double* r_rows, uint32_t* lat_rows,
                               double* rel_rows, double* lms_rows, uint64_t quantum_ns,
                               hipStream_t st, int32_t fw_block, srt_build_stats* stats) {
    if (!comm || n <= 0 || ld < n || ld % SRT_SHARD_ALIGN || !w_rows || !r_rows || !lat_rows || !rel_rows) {
        srt_set_error("srt_dense_build_sharded: bad arguments");
        return SRT_E_ARG;
    }
    if (n > srt_dense_max_n()) { /* refused before any FW round runs */
        srt_set_error("dense build supports n <= %d (n = %d); use the sparse SSSP", srt_dense_max_n(), n);
        return SRT_E_RANGE;
    }
    if (fw_block != 0 && fw_block != B) {
        srt_set_error("srt_dense_build_sharded: fw_block must be 0 or %d", B);
        return SRT_E_ARG;
    }
    const int R = srt_comm_size(comm), me = srt_comm_rank(comm);
    int32_t b, e;
    srt_shard_rows(ld, SRT_SHARD_ALIGN, R, me, &b, &e);
    const int nr = e - b;
    dense_ws* ws;
    int rc = ws_get(&ws, n);
    if (rc) return rc;
    size_t pc = ws->panel_cap;
    if ((rc = ws_grow((void**)&ws->panel, &pc, (size_t)B * ld, sizeof(uint32_t)))) return rc;
    ws->panel_cap = pc;
    build_events ev;
    if ((rc = ev.create())) return rc;
    hipEvent_t e0 = ev.e[0], e1 = ev.e[1], e2 = ev.e[2];
    SRT_HIPCHK(hipEventRecord(e0, st));
    evpool_t* evp = NULL;
    if (stats && stats->time_kernels && (rc = evpool_begin(&evp, ld / B))) return rc;
    shard_ctx ctx = {comm, ld};
    srt_comm_timing(comm, stats && stats->time_kernels);
    int exact = 0, enc = SRT_DENC_U32;
    /* symmetric rounds up to 1,024 tile columns (fw16.hip SYM_TMAX, the panel-position table) */
    const bool sym = !directed && R > 1 && ld <= 1024 * 128 && srt_form_int("sym", 1) != 0;
    if ((rc = dense_try_levels(comm, n, ld, b, nr, directed, w_rows, r_rows, lat_rows, st, evp, stats,
                               &exact)))
        return rc;
    if (exact) enc = SRT_DENC_LEVELS;
    for (int fm = 1; fm >= 0 && !exact; --fm) {
        if (evp) {
            evp->used = 0;
            evp->group = 2;
        }
        if (fm && sym) /* undirected: each rank updates half of its row block (fw16.hip) */
            rc = srt_fw16_build_sym_sharded(comm, n, ld, b, nr, w_rows, lat_rows, st, evp, &exact);
        else
            rc = srt_fw16_build(n, ld, b, nr, w_rows, lat_rows, st, evp, shard_owner,
                                R > 1 ? shard_bcast : NULL, &ctx, me, fm, NULL, &exact);
        if (rc) return rc;
        if (R > 1) { /* every rank must agree before falling back to a wider encoding */
            int32_t* flag = ws->cnt;
            SRT_HIPCHK(hipMemcpyAsync(flag, &exact, sizeof(int32_t), hipMemcpyHostToDevice, st));
            if ((rc = srt_coll_allreduce_i32(comm, flag, 1, 1, st))) return rc;
            SRT_HIPCHK(hipMemcpyAsync(&exact, flag, sizeof(int32_t), hipMemcpyDeviceToHost, st));
            SRT_HIPCHK(hipStreamSynchronize(st));
        }
        if (exact)
            enc = fm ? (sym ? (srt_fw16_sharded_round_pivots() == 256   ? SRT_DENC_F16CMP_SYMSH256
                               : srt_fw16_sharded_round_pivots() == 128 ? SRT_DENC_F16CMP_SYMSH128
                                                                        : SRT_DENC_F16CMP_SYM)
                            : SRT_DENC_F16CMP)
                     : SRT_DENC_U16;
    }
    if (!exact) {
        if (evp) {
            evp->used = 0;
            evp->group = 2;
        }
        if (nr > 0) {
            dim3 g(srt_ceil_div(ld, 256), nr);
            init_dist_kernel<<<g, 256, 0, st>>>(n, ld, b, w_rows, lat_rows);
            SRT_HIPCHK(hipGetLastError());
        }
        for (int k0 = 0; k0 < ld; k0 += B) {
            const int owner = shard_owner(&ctx, k0);
            uint32_t* P;
            if (owner == me) {
                P = lat_rows + (size_t)(k0 - b) * ld;
                if ((rc = fw_owner_part(lat_rows, ld, b, nr, P, k0, st))) return rc;
            } else {
                P = ws->panel;
            }
            if (R > 1 && (rc = srt_coll_bcast(comm, P, (size_t)B * ld * sizeof(uint32_t), owner, st)))
                return rc;
            if ((rc = fw_shard_part(lat_rows, ld, b, nr, P, k0, st, evp))) return rc;
        }
    }
    SRT_HIPCHK(hipEventRecord(e1, st));
    rc = dense_post(n, ld, b, nr, directed, w_rows, r_rows, lat_rows,
                    exact ? srt_fw16_matrix() : NULL, rel_rows, st, stats,
                    R > 1 ? shard_gather : NULL, &ctx, enc == SRT_DENC_LEVELS);
    if (rc) return rc;
    if ((rc = dense_finish_rows(n, ld, b, nr, w_rows, r_rows, lat_rows, rel_rows, st, stats))) return rc;
    if (lms_rows) {
        if ((rc = dense_path_ms(n, ld, b, nr, lat_rows, quantum_ns, lms_rows, st))) return rc;
    }
    SRT_HIPCHK(hipEventRecord(e2, st));
    if (stats) {
        SRT_HIPCHK(hipEventSynchronize(e2));
        float a = 0, c = 0;
        SRT_HIPCHK(hipEventElapsedTime(&a, e0, e1));
        SRT_HIPCHK(hipEventElapsedTime(&c, e1, e2));
        stats->algo = SRT_ALGO_DENSE_FW;
        stats->fw_block = B;
        stats->dist_enc = enc;
        stats->ms_fw = a;
        stats->ms_post = c;
        stats->ms_total = a + c;
        if (evp && (rc = evpool_sum(evp, e2, stats))) return rc;
        stats->ms_comm = srt_comm_timing_ms(comm);
    }
    srt_comm_timing(comm, 0);
    return SRT_OK;
}

extern "C" int srt_dense_build_sharded(srt_comm* comm, int32_t n, int32_t ld, int32_t directed,
                                       const uint32_t* w_rows, const double* r_rows,
                                       uint32_t* lat_rows, double* rel_rows, void* stream,
                                       int32_t fw_block, srt_build_stats* stats) {
    return srt_dense_build_sharded_ms(comm, n, ld, directed, w_rows, r_rows, lat_rows, rel_rows,
                                      NULL, 0, (hipStream_t)stream, fw_block, stats);
}
