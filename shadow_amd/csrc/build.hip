/*
 * build.hip -- host orchestration of one routing-table build on one GPU.
 *
 * Replaces the lazy per-source Dijkstra of /root/reference/src/main/routing/topology.c:1578-1814
 * (run on a cache miss from _topology_getPathEntry, :1923-1961) with one eager all-pairs build:
 *   use_shortest_path == false : direct edge gather (topology.c:1816-1858)
 *   dense graphs               : blocked Floyd-Warshall + predecessor/reliability pass (dense.hip)
 *   sparse graphs              : multi-source LDS SSSP + tree walk (sparse.hip)
 * Every path runs on the GPU; a device failure is returned as SRT_E_DEVICE, never replaced by a
 * host computation.
 */
#include <stdlib.h>
#include <string.h>

#include "srt_device.h"

int srt_sparse_max_n(void);

extern "C" int srt_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

extern "C" int srt_device_sync(int32_t device) {
    SRT_HIPCHK(hipSetDevice(device));
    SRT_HIPCHK(hipDeviceSynchronize());
    return SRT_OK;
}

__global__ void mirror_lower_tiles(int n, int ld, double* __restrict__ rel) {
    __shared__ double tile[64][65];
    const int I = blockIdx.y, J = blockIdx.x;
    if (J > I) return;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int a = ty; a < 64; a += 4) {
        int t = J * 64 + a, s = I * 64 + tx;
        tile[a][tx] = (t < n && s < n) ? rel[(size_t)t * ld + s] : 0.0;
    }
    __syncthreads();
    for (int a = ty; a < 64; a += 4) {
        int s = I * 64 + a, t = J * 64 + tx;
        if (s < n && t < n && s > t) rel[(size_t)s * ld + t] = tile[tx][a];
    }
}

extern "C" int srt_mirror_lower_device(int32_t n, int32_t ld, double* rel, void* stream) {
    if (n <= 0 || ld < n || !rel) {
        srt_set_error("srt_mirror_lower_device: bad arguments");
        return SRT_E_ARG;
    }
    dim3 g(srt_ceil_div(n, 64), srt_ceil_div(n, 64));
    mirror_lower_tiles<<<g, 256, 0, (hipStream_t)stream>>>(n, ld, rel);
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

/* RAII-free device buffer list: everything allocated here is released on every exit path */
typedef struct {
    void* p[24];
    int k;
} dbufs;

static int dalloc(dbufs* b, void** out, size_t bytes) {
    if (b->k >= 24) return SRT_E_NOMEM;
    void* p = NULL;
    if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) {
        srt_set_error("hipMalloc(%zu) failed", bytes);
        return SRT_E_NOMEM;
    }
    b->p[b->k++] = p;
    *out = p;
    return SRT_OK;
}

static void dfree(dbufs* b) {
    for (int i = 0; i < b->k; i++) (void)hipFree(b->p[i]);
    b->k = 0;
}

#define TRY(x)                  \
    do {                        \
        rc = (x);               \
        if (rc) goto out;       \
    } while (0)
#define TRYHIP(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            srt_set_error("HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, __LINE__); \
            rc = SRT_E_DEVICE;                                                             \
            goto out;                                                                      \
        }                                                                                  \
    } while (0)

static int choose_algo(const srt_canon* c, const srt_build_opts* o) {
    if (o && o->algo == SRT_ALGO_DENSE_FW) return SRT_ALGO_DENSE_FW;
    if (o && o->algo == SRT_ALGO_SPARSE_SSSP) return SRT_ALGO_SPARSE_SSSP;
    const double n = c->n;
    /* FW costs n^3 cheap LDS relaxations; the SSSP costs ~n * arcs * (re-relaxation factor)
     * gathers. Dense wins once arcs are within ~1/16 of n^2, or the graph is tiny. */
    if (c->n <= 2048 || (double)c->arcs * 16.0 >= n * n) return SRT_ALGO_DENSE_FW;
    if (c->n > srt_sparse_max_n()) return SRT_ALGO_DENSE_FW;
    return SRT_ALGO_SPARSE_SSSP;
}

extern "C" int srt_build_tables(const srt_edges* g, const srt_build_opts* opts, uint32_t* lat_q,
                                uint64_t* quantum_ns, double* rel, srt_build_stats* stats) {
    if (!g || !lat_q || !quantum_ns || !rel) {
        srt_set_error("srt_build_tables: null argument");
        return SRT_E_ARG;
    }
    srt_canon c;
    int rc = srt_canon_build(g, &c);
    if (rc) return rc;
    *quantum_ns = c.quantum_ns;
    const int n = c.n;
    const int use_sp = opts ? opts->use_shortest_path : 1;
    int algo = use_sp ? choose_algo(&c, opts) : SRT_ALGO_DENSE_FW;
    srt_build_stats local;
    memset(&local, 0, sizeof(local));
    dbufs B;
    B.k = 0;
    hipStream_t st = NULL;
    uint32_t* hw = NULL;
    double* hr = NULL;
    TRYHIP(hipSetDevice(opts ? opts->device : 0));
    TRYHIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    if (algo == SRT_ALGO_DENSE_FW) {
        const int ld = srt_ceil_div(n, 64) * 64;
        const size_t ll = (size_t)ld * ld;
        hw = (uint32_t*)malloc(ll * sizeof(uint32_t));
        hr = (double*)malloc(ll * sizeof(double));
        if (!hw || !hr) {
            rc = SRT_E_NOMEM;
            goto out;
        }
        for (size_t i = 0; i < ll; i++) {
            hw[i] = SRT_INF;
            hr[i] = 0.0;
        }
        for (int u = 0; u < n; u++) {
            for (int k = c.rowptr[u]; k < c.rowptr[u + 1]; k++) {
                hw[(size_t)u * ld + c.col[k]] = c.w[k];
                hr[(size_t)u * ld + c.col[k]] = c.r[k];
            }
            hw[(size_t)u * ld + u] = c.self_w[u];
            hr[(size_t)u * ld + u] = c.self_r[u];
        }
        uint32_t *dw, *dlat;
        double *dr, *drel;
        TRY(dalloc(&B, (void**)&dw, ll * sizeof(uint32_t)));
        TRY(dalloc(&B, (void**)&dr, ll * sizeof(double)));
        TRY(dalloc(&B, (void**)&dlat, ll * sizeof(uint32_t)));
        TRY(dalloc(&B, (void**)&drel, ll * sizeof(double)));
        TRYHIP(hipMemcpyAsync(dw, hw, ll * sizeof(uint32_t), hipMemcpyHostToDevice, st));
        TRYHIP(hipMemcpyAsync(dr, hr, ll * sizeof(double), hipMemcpyHostToDevice, st));
        if (use_sp) {
            TRY(srt_dense_build_device(n, ld, c.directed, dw, dr, dlat, drel, st,
                                       opts ? opts->fw_block : 0, &local));
        } else {
            /* direct mode: the (complete) graph's own edges, self-loop on the diagonal */
            TRYHIP(hipMemcpyAsync(dlat, dw, ll * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
            TRYHIP(hipMemcpyAsync(drel, dr, ll * sizeof(double), hipMemcpyDeviceToDevice, st));
            local.algo = SRT_ALGO_DENSE_FW;
        }
        TRYHIP(hipMemcpy2DAsync(lat_q, (size_t)n * sizeof(uint32_t), dlat, (size_t)ld * sizeof(uint32_t),
                                (size_t)n * sizeof(uint32_t), n, hipMemcpyDeviceToHost, st));
        TRYHIP(hipMemcpy2DAsync(rel, (size_t)n * sizeof(double), drel, (size_t)ld * sizeof(double),
                                (size_t)n * sizeof(double), n, hipMemcpyDeviceToHost, st));
        TRYHIP(hipStreamSynchronize(st));
        if (!use_sp) {
            for (size_t i = 0; i < (size_t)n * n; i++)
                if (lat_q[i] >= SRT_INF) {
                    srt_set_error("use_shortest_path=false requires a complete graph");
                    rc = SRT_E_INVALID;
                    goto out;
                }
        }
    } else {
        const size_t nn = (size_t)n * n;
        const int64_t arcs = c.arcs;
        int32_t *d_rp, *d_col, *d_irp, *d_icol;
        uint32_t *d_w, *d_iw, *d_sw, *d_lat;
        double *d_r, *d_ir, *d_sr, *d_rel;
        TRY(dalloc(&B, (void**)&d_rp, (size_t)(n + 1) * sizeof(int32_t)));
        TRY(dalloc(&B, (void**)&d_col, (size_t)arcs * sizeof(int32_t)));
        TRY(dalloc(&B, (void**)&d_w, (size_t)arcs * sizeof(uint32_t)));
        TRY(dalloc(&B, (void**)&d_r, (size_t)arcs * sizeof(double)));
        TRY(dalloc(&B, (void**)&d_sw, (size_t)n * sizeof(uint32_t)));
        TRY(dalloc(&B, (void**)&d_sr, (size_t)n * sizeof(double)));
        TRY(dalloc(&B, (void**)&d_lat, nn * sizeof(uint32_t)));
        TRY(dalloc(&B, (void**)&d_rel, nn * sizeof(double)));
        TRYHIP(hipMemcpyAsync(d_rp, c.rowptr, (size_t)(n + 1) * sizeof(int32_t), hipMemcpyHostToDevice, st));
        TRYHIP(hipMemcpyAsync(d_col, c.col, (size_t)arcs * sizeof(int32_t), hipMemcpyHostToDevice, st));
        TRYHIP(hipMemcpyAsync(d_w, c.w, (size_t)arcs * sizeof(uint32_t), hipMemcpyHostToDevice, st));
        TRYHIP(hipMemcpyAsync(d_r, c.r, (size_t)arcs * sizeof(double), hipMemcpyHostToDevice, st));
        TRYHIP(hipMemcpyAsync(d_sw, c.self_w, (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice, st));
        TRYHIP(hipMemcpyAsync(d_sr, c.self_r, (size_t)n * sizeof(double), hipMemcpyHostToDevice, st));
        if (c.directed) {
            TRY(dalloc(&B, (void**)&d_irp, (size_t)(n + 1) * sizeof(int32_t)));
            TRY(dalloc(&B, (void**)&d_icol, (size_t)arcs * sizeof(int32_t)));
            TRY(dalloc(&B, (void**)&d_iw, (size_t)arcs * sizeof(uint32_t)));
            TRY(dalloc(&B, (void**)&d_ir, (size_t)arcs * sizeof(double)));
            TRYHIP(hipMemcpyAsync(d_irp, c.in_rowptr, (size_t)(n + 1) * sizeof(int32_t), hipMemcpyHostToDevice, st));
            TRYHIP(hipMemcpyAsync(d_icol, c.in_col, (size_t)arcs * sizeof(int32_t), hipMemcpyHostToDevice, st));
            TRYHIP(hipMemcpyAsync(d_iw, c.in_w, (size_t)arcs * sizeof(uint32_t), hipMemcpyHostToDevice, st));
            TRYHIP(hipMemcpyAsync(d_ir, c.in_r, (size_t)arcs * sizeof(double), hipMemcpyHostToDevice, st));
        } else {
            d_irp = d_rp;
            d_icol = d_col;
            d_iw = d_w;
            d_ir = d_r;
        }
        /* bucket width: the mean arc weight */
        double sumw = 0;
        for (int64_t k = 0; k < arcs; k++) sumw += c.w[k];
        uint32_t delta = arcs > 0 ? (uint32_t)(sumw / (double)arcs + 0.5) : 1u;
        if (delta < 1) delta = 1;
        TRY(srt_sparse_build_device(n, c.directed, d_rp, d_col, d_w, d_r, d_irp, d_icol, d_iw, d_ir,
                                    d_sw, d_sr, 0, n, delta, d_lat, d_rel, st, &local));
        if (!c.directed) TRY(srt_mirror_lower_device(n, n, d_rel, st));
        TRYHIP(hipMemcpyAsync(lat_q, d_lat, nn * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        TRYHIP(hipMemcpyAsync(rel, d_rel, nn * sizeof(double), hipMemcpyDeviceToHost, st));
        TRYHIP(hipStreamSynchronize(st));
    }
    if (stats) *stats = local;
out:
    if (st) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
    }
    dfree(&B);
    free(hw);
    free(hr);
    srt_canon_free(&c);
    return rc;
}
