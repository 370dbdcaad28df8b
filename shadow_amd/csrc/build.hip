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

#include <algorithm>

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

/* ---- device-resident sparse graph (canonical CSR uploaded once, rows computed per shard) ---- */
struct srt_sparse_graph {
    int device;
    int32_t n, directed;
    int64_t arcs;
    uint64_t quantum_ns;
    uint32_t delta, max_w;
    int local; /* relabelled arcs span <= 4096 vertices on average (graph.c CM order) */
    int32_t *rp, *col, *irp, *icol;
    uint32_t *w, *iw, *sw;
    double *r, *ir, *sr;
    uint2 *cw, *icw; /* packed (col, w) arcs for the wave-per-source kernel */
    /* the same graph relabelled in Cuthill-McKee order for the wave-per-source kernel: perm[new] =
     * old, inv[old] = new; rows keep their arcs sorted by ORIGINAL neighbour index */
    int32_t *perm, *inv;
    int2 *rp2, *irp2; /* (begin, end) of each relabelled row */
    uint2 *cw2, *icw2;
    double *r2, *ir2;
};

int srt_wgsssp_max_n(void);
int srt_wgsssp_rows(int n, const int2* rowptr, const uint2* cw, const double* r, const int32_t* inv,
                    uint32_t max_w, int src_begin, int src_end, uint32_t* lat, double* rel,
                    int* ovf, hipStream_t st);
int srt_wsssp_rows(int n, int directed, const int2* rowptr, const uint2* cw, const double* r,
                   const int2* in_rowptr, const uint2* in_cw, const double* in_r,
                   const int32_t* perm, const int32_t* inv, uint32_t max_w, int local,
                   int src_begin,
                   int src_end, uint32_t* lat, double* rel, int* ovf, hipStream_t st);
int srt_sparse_diag(int n, int src_begin, int src_end, const int32_t* rowptr, const int32_t* col,
                    const uint32_t* w, const double* r, const uint32_t* self_w,
                    const double* self_r, uint32_t* lat, double* rel, size_t ldo, hipStream_t st);

static int up(void** d, const void* h, size_t bytes) {
    *d = NULL;
    if (hipMalloc(d, bytes ? bytes : 4) != hipSuccess) {
        (void)hipGetLastError();
        srt_set_error("hipMalloc of %zu bytes failed", bytes);
        return SRT_E_NOMEM;
    }
    if (bytes && hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice) != hipSuccess) {
        srt_set_error("hipMemcpy of %zu bytes failed", bytes);
        return SRT_E_DEVICE;
    }
    return SRT_OK;
}

extern "C" void srt_sparse_graph_free(srt_sparse_graph* g) {
    if (!g) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(g->device);
    void* ps[] = {g->rp, g->col, g->w, g->r, g->sw, g->sr, g->cw, g->perm, g->inv, g->rp2, g->cw2, g->r2};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    if (g->directed) {
        void* qs[] = {g->irp, g->icol, g->iw, g->ir, g->icw, g->irp2, g->icw2, g->ir2};
        for (void* p : qs)
            if (p) (void)hipFree(p);
    }
    (void)hipSetDevice(prev);
    free(g);
}

/* Cuthill-McKee order of the undirected structure (out-arcs, plus in-arcs when directed):
 * breadth-first from the lowest-degree unvisited vertex, neighbours in increasing degree. */
static int cuthill_mckee(const srt_canon* c, int32_t* perm, int32_t* inv) {
    const int n = c->n;
    int32_t* deg = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    int32_t* byd = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    int32_t* nb = (int32_t*)malloc((size_t)(c->arcs * (c->directed ? 2 : 1) + 1) * sizeof(int32_t));
    if (!deg || !byd || !nb) {
        free(deg);
        free(byd);
        free(nb);
        return SRT_E_NOMEM;
    }
    for (int v = 0; v < n; v++) {
        deg[v] = c->rowptr[v + 1] - c->rowptr[v];
        if (c->directed) deg[v] += c->in_rowptr[v + 1] - c->in_rowptr[v];
        byd[v] = v;
        inv[v] = -1;
    }
    std::stable_sort(byd, byd + n, [&](int32_t a, int32_t b) { return deg[a] < deg[b]; });
    int head = 0, tail = 0, next_start = 0;
    while (tail < n) {
        while (inv[byd[next_start]] >= 0) next_start++;
        const int st = byd[next_start];
        inv[st] = tail;
        perm[tail++] = st;
        while (head < tail) {
            const int v = perm[head++];
            int m = 0;
            for (int k = c->rowptr[v]; k < c->rowptr[v + 1]; k++)
                if (inv[c->col[k]] < 0) nb[m++] = c->col[k];
            if (c->directed)
                for (int k = c->in_rowptr[v]; k < c->in_rowptr[v + 1]; k++)
                    if (inv[c->in_col[k]] < 0) nb[m++] = c->in_col[k];
            std::stable_sort(nb, nb + m, [&](int32_t a, int32_t b) {
                return deg[a] != deg[b] ? deg[a] < deg[b] : a < b;
            });
            for (int i = 0; i < m; i++) {
                if (inv[nb[i]] >= 0) continue; /* duplicate (out- and in-neighbour) */
                inv[nb[i]] = tail;
                perm[tail++] = nb[i];
            }
        }
    }
    free(deg);
    free(byd);
    free(nb);
    return SRT_OK;
}

/* CSR rows in relabelled order; each row keeps its arcs in original-neighbour order */
static void relabel_csr(int n, const int32_t* rp, const int32_t* col, const uint32_t* w,
                        const double* r, const int32_t* perm, const int32_t* inv, int2* rp2,
                        uint2* cw2, double* r2) {
    int o = 0;
    for (int i = 0; i < n; i++) {
        const int v = perm[i];
        const int b = o;
        for (int k = rp[v]; k < rp[v + 1]; k++, o++) {
            cw2[o] = make_uint2((uint32_t)inv[col[k]], w[k]);
            r2[o] = r[k];
        }
        rp2[i] = make_int2(b, o);
    }
}

static int sparse_graph_from_canon(const srt_canon* c, int device, srt_sparse_graph** out) {
    *out = NULL;
    srt_sparse_graph* g = (srt_sparse_graph*)calloc(1, sizeof(srt_sparse_graph));
    if (!g) return SRT_E_NOMEM;
    g->device = device;
    g->n = c->n;
    g->directed = c->directed;
    g->arcs = c->arcs;
    g->quantum_ns = c->quantum_ns;
    g->max_w = 0;
    for (int64_t k = 0; k < c->arcs; k++) g->max_w = c->w[k] > g->max_w ? c->w[k] : g->max_w;
    /* bucket width of the label-correcting loop: the mean arc weight */
    double sumw = 0;
    for (int64_t k = 0; k < c->arcs; k++) sumw += c->w[k];
    g->delta = c->arcs > 0 ? (uint32_t)(sumw / (double)c->arcs + 0.5) : 1u;
    if (g->delta < 1) g->delta = 1;
    int rc = hipSetDevice(device) == hipSuccess ? SRT_OK : SRT_E_DEVICE;
    const size_t n1 = (size_t)(c->n + 1), na = (size_t)c->arcs, nv = (size_t)c->n;
    if (!rc) rc = up((void**)&g->rp, c->rowptr, n1 * 4);
    if (!rc) rc = up((void**)&g->col, c->col, na * 4);
    if (!rc) rc = up((void**)&g->w, c->w, na * 4);
    if (!rc) rc = up((void**)&g->r, c->r, na * 8);
    if (!rc) rc = up((void**)&g->sw, c->self_w, nv * 4);
    if (!rc) rc = up((void**)&g->sr, c->self_r, nv * 8);
    uint2* hcw = (uint2*)malloc((na ? na : 1) * sizeof(uint2));
    if (!hcw && !rc) rc = SRT_E_NOMEM;
    if (!rc) {
        for (size_t k = 0; k < na; k++) hcw[k] = make_uint2((uint32_t)c->col[k], c->w[k]);
        rc = up((void**)&g->cw, hcw, na * sizeof(uint2));
    }
    if (c->directed) {
        if (!rc) rc = up((void**)&g->irp, c->in_rowptr, n1 * 4);
        if (!rc) rc = up((void**)&g->icol, c->in_col, na * 4);
        if (!rc) rc = up((void**)&g->iw, c->in_w, na * 4);
        if (!rc) rc = up((void**)&g->ir, c->in_r, na * 8);
        if (!rc) {
            for (size_t k = 0; k < na; k++) hcw[k] = make_uint2((uint32_t)c->in_col[k], c->in_w[k]);
            rc = up((void**)&g->icw, hcw, na * sizeof(uint2));
        }
    } else {
        g->irp = g->rp;
        g->icol = g->col;
        g->iw = g->w;
        g->ir = g->r;
        g->icw = g->cw;
    }
    /* relabelled copy for the wave-per-source kernel */
    int32_t* hperm = (int32_t*)malloc(nv * sizeof(int32_t));
    int32_t* hinv = (int32_t*)malloc(nv * sizeof(int32_t));
    int2* hrp = (int2*)malloc(nv * sizeof(int2));
    double* hr = (double*)malloc((na ? na : 1) * sizeof(double));
    if (!rc && (!hperm || !hinv || !hrp || !hr || !hcw)) rc = SRT_E_NOMEM;
    if (!rc) rc = cuthill_mckee(c, hperm, hinv);
    if (!rc) {
        relabel_csr(c->n, c->rowptr, c->col, c->w, c->r, hperm, hinv, hrp, hcw, hr);
        /* locality of the relabelled graph: the wave kernel keeps its reliability row in
         * relabelled order when an arc's ends are close there (RGG-like graphs: the
         * predecessor's entry is near), else writes the output rows at settle time */
        double span = 0.0;
        for (int32_t v = 0; v < c->n; v++)
            for (int32_t k = hrp[v].x; k < hrp[v].y; k++) span += fabs((double)v - (double)hcw[k].x);
        g->local = na == 0 || span / (double)na <= 4096.0;
        rc = up((void**)&g->perm, hperm, nv * 4);
        if (!rc) rc = up((void**)&g->inv, hinv, nv * 4);
        if (!rc) rc = up((void**)&g->rp2, hrp, nv * sizeof(int2));
        if (!rc) rc = up((void**)&g->cw2, hcw, na * sizeof(uint2));
        if (!rc) rc = up((void**)&g->r2, hr, na * 8);
    }
    if (!rc && c->directed) {
        relabel_csr(c->n, c->in_rowptr, c->in_col, c->in_w, c->in_r, hperm, hinv, hrp, hcw, hr);
        rc = up((void**)&g->irp2, hrp, nv * sizeof(int2));
        if (!rc) rc = up((void**)&g->icw2, hcw, na * sizeof(uint2));
        if (!rc) rc = up((void**)&g->ir2, hr, na * 8);
    } else if (!rc) {
        g->irp2 = g->rp2;
        g->icw2 = g->cw2;
        g->ir2 = g->r2;
    }
    free(hperm);
    free(hinv);
    free(hrp);
    free(hr);
    free(hcw);
    if (rc) {
        srt_sparse_graph_free(g);
        return rc;
    }
    *out = g;
    return SRT_OK;
}

extern "C" int srt_sparse_graph_new(const srt_edges* e, int32_t device, srt_sparse_graph** out) {
    if (!e || !out) {
        srt_set_error("srt_sparse_graph_new: null argument");
        return SRT_E_ARG;
    }
    srt_canon c;
    int rc = srt_canon_build(e, &c);
    if (rc) return rc;
    rc = sparse_graph_from_canon(&c, device, out);
    srt_canon_free(&c);
    return rc;
}

extern "C" int srt_sparse_graph_info(const srt_sparse_graph* g, int32_t* n, int32_t* directed,
                                     int64_t* arcs, uint64_t* quantum_ns) {
    if (!g) {
        srt_set_error("srt_sparse_graph_info: null graph");
        return SRT_E_ARG;
    }
    if (n) *n = g->n;
    if (directed) *directed = g->directed;
    if (arcs) *arcs = g->arcs;
    if (quantum_ns) *quantum_ns = g->quantum_ns;
    return SRT_OK;
}

/* Rows of a source range: the wave-per-source bucket kernel (wsssp.hip) when the arc weights fit
 * its bucket ring, with any source whose buckets overflowed recomputed by the
 * workgroup-per-source kernel (sparse.hip); SRT_SPARSE_KERNEL=block (or SRT_SPARSE_WORKSET=hbm)
 * selects the workgroup kernel for every source. */
extern "C" int srt_sparse_graph_rows(const srt_sparse_graph* g, int32_t src_begin, int32_t src_end,
                                     uint32_t* lat_rows, double* rel_rows, void* stream,
                                     srt_build_stats* stats) {
    if (!g) {
        srt_set_error("srt_sparse_graph_rows: null graph");
        return SRT_E_ARG;
    }
    const char* kenv = getenv("SRT_SPARSE_KERNEL");
    const char* wenv = getenv("SRT_SPARSE_WORKSET");
    const bool block = (kenv && !strcmp(kenv, "block")) || (wenv && !strcmp(wenv, "hbm"));
    if (block || g->max_w >= 256 || src_begin < 0 || src_end > g->n || src_begin >= src_end)
        return srt_sparse_build_device(g->n, g->directed, g->rp, g->col, g->w, g->r, g->irp,
                                       g->icol, g->iw, g->ir, g->sw, g->sr, src_begin, src_end,
                                       g->delta, lat_rows, rel_rows, stream, stats);
    hipStream_t st = (hipStream_t)stream;
    const int nsrc = src_end - src_begin;
    /* events, the overflow flags and host buffers are released on every return path */
    struct rows_scratch {
        hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
        int* ovf = nullptr;
        int* ovf1 = nullptr;
        uint32_t* row = nullptr;
        int* hov = nullptr;
        hipStream_t st = nullptr;
        ~rows_scratch() {
            for (hipEvent_t e : ev)
                if (e) (void)hipEventDestroy(e);
            if (ovf) (void)hipFreeAsync(ovf, st);
            if (ovf1) (void)hipFree(ovf1);
            free(row);
            free(hov);
        }
    } sc;
    sc.st = st;
    SRT_HIPCHK(hipMallocAsync((void**)&sc.ovf, (size_t)nsrc * sizeof(int), st));
    int* const ovf = sc.ovf;
    SRT_HIPCHK(hipEventCreate(&sc.ev[0]));
    SRT_HIPCHK(hipEventCreate(&sc.ev[1]));
    SRT_HIPCHK(hipEventCreate(&sc.ev[2]));
    hipEvent_t e0 = sc.ev[0], e1 = sc.ev[1], e2 = sc.ev[2];
    SRT_HIPCHK(hipEventRecord(e0, st));
    /* large power-law graphs (relabelled arcs far apart): the workgroup kernel with the distance
     * row packed in LDS, once a probe source shows every distance fits its 10-bit fields
     * (d(a, b) <= 2 ecc(s0)); SRT_SPARSE_WG=0/1 disables / allows it at any size */
    const char* genv = getenv("SRT_SPARSE_WG");
    bool wg = !g->directed && g->n <= srt_wgsssp_max_n() &&
              (genv ? atoi(genv) != 0 : (g->n > 32768 && !g->local));
    int rc = SRT_OK;
    if (wg) {
        rc = srt_wgsssp_rows(g->n, g->rp2, g->cw2, g->r2, g->inv, g->max_w, src_begin,
                             src_begin + 1, lat_rows, rel_rows, ovf, st);
        if (rc) return rc;
        uint32_t* row = sc.row = (uint32_t*)malloc((size_t)g->n * sizeof(uint32_t));
        int pov = 1;
        if (!row) return SRT_E_NOMEM;
        SRT_HIPCHK(hipMemcpyAsync(row, lat_rows, (size_t)g->n * sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, st));
        SRT_HIPCHK(hipMemcpyAsync(&pov, ovf, sizeof(int), hipMemcpyDeviceToHost, st));
        SRT_HIPCHK(hipStreamSynchronize(st));
        uint32_t ecc = 0;
        for (int32_t i = 0; i < g->n; i++)
            if (row[i] != SRT_INF && row[i] > ecc) ecc = row[i];
        wg = !pov && 2ull * ecc <= 1022ull;
        if (wg && nsrc > 1)
            rc = srt_wgsssp_rows(g->n, g->rp2, g->cw2, g->r2, g->inv, g->max_w, src_begin + 1,
                                 src_end, lat_rows + (size_t)g->n, rel_rows + (size_t)g->n, ovf + 1,
                                 st);
        if (rc) return rc;
    }
    if (!wg)
        rc = srt_wsssp_rows(g->n, g->directed, g->rp2, g->cw2, g->r2, g->irp2, g->icw2, g->ir2,
                            g->perm, g->inv, g->max_w, g->local, src_begin, src_end, lat_rows,
                            rel_rows, ovf, st);
    if (rc) return rc;
    SRT_HIPCHK(hipEventRecord(e1, st));
    rc = srt_sparse_diag(g->n, src_begin, src_end, g->rp, g->col, g->w, g->r, g->sw, g->sr,
                         lat_rows, rel_rows, (size_t)g->n, st);
    if (rc) return rc;
    int* hov = sc.hov = (int*)malloc((size_t)nsrc * sizeof(int));
    if (!hov) return SRT_E_NOMEM;
    SRT_HIPCHK(hipMemcpyAsync(hov, ovf, (size_t)nsrc * sizeof(int), hipMemcpyDeviceToHost, st));
    sc.ovf = nullptr;
    SRT_HIPCHK(hipFreeAsync(ovf, st));
    SRT_HIPCHK(hipStreamSynchronize(st));
    int nov = 0;
    int*& ovf1 = sc.ovf1;
    for (int i = 0; i < nsrc && !rc; i++) {
        if (!hov[i]) continue;
        ++nov;
        int again = 1;
        if (wg) { /* the workgroup kernel's overflow: the wave kernel first */
            if (!ovf1) SRT_HIPCHK(hipMalloc((void**)&ovf1, sizeof(int)));
            rc = srt_wsssp_rows(g->n, g->directed, g->rp2, g->cw2, g->r2, g->irp2, g->icw2, g->ir2,
                                g->perm, g->inv, g->max_w, g->local, src_begin + i,
                                src_begin + i + 1, lat_rows + (size_t)i * g->n,
                                rel_rows + (size_t)i * g->n, ovf1, st);
            if (!rc && hipMemcpyAsync(&again, ovf1, sizeof(int), hipMemcpyDeviceToHost, st) ==
                           hipSuccess &&
                hipStreamSynchronize(st) != hipSuccess)
                rc = SRT_E_DEVICE;
            if (!rc && !again) /* the wave kernel wrote the row; the diagonal rule again */
                rc = srt_sparse_diag(g->n, src_begin + i, src_begin + i + 1, g->rp, g->col, g->w,
                                     g->r, g->sw, g->sr, lat_rows + (size_t)i * g->n,
                                     rel_rows + (size_t)i * g->n, (size_t)g->n, st);
        }
        if (!rc && again)
            rc = srt_sparse_build_device(g->n, g->directed, g->rp, g->col, g->w, g->r, g->irp,
                                         g->icol, g->iw, g->ir, g->sw, g->sr, src_begin + i,
                                         src_begin + i + 1, g->delta,
                                         lat_rows + (size_t)i * g->n, rel_rows + (size_t)i * g->n,
                                         stream, NULL);
    }
    if (rc) return rc;
    SRT_HIPCHK(hipEventRecord(e2, st));
    SRT_HIPCHK(hipEventSynchronize(e2));
    float a = 0, b = 0;
    SRT_HIPCHK(hipEventElapsedTime(&a, e0, e1));
    SRT_HIPCHK(hipEventElapsedTime(&b, e0, e2));
    if (nov) srt_log(SRT_LOG_INFO, "wsssp: %d of %d sources overflowed their buckets and were "
                     "recomputed by the workgroup kernel", nov, nsrc);
    if (stats) {
        stats->algo = SRT_ALGO_SPARSE_SSSP;
        stats->ms_fw = b;
        stats->ms_total = b;
        stats->n_update = 1;
        stats->ms_update = a;
        stats->ess_arcs = nov; /* sparse builds: sources recomputed after a bucket overflow */
        stats->dist_enc = wg ? 2 : 1; /* sparse builds: 2 = workgroup kernel, 1 = wave kernel */
    }
    return SRT_OK;
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
        const int ld = srt_ceil_div(n, 128) * 128; /* the u16 FW tiles need ld % 128 == 0 */
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
        srt_sparse_graph* sg = NULL;
        uint32_t* d_lat;
        double* d_rel;
        TRY(sparse_graph_from_canon(&c, opts ? opts->device : 0, &sg));
        rc = dalloc(&B, (void**)&d_lat, nn * sizeof(uint32_t));
        if (!rc) rc = dalloc(&B, (void**)&d_rel, nn * sizeof(double));
        if (!rc) rc = srt_sparse_graph_rows(sg, 0, n, d_lat, d_rel, st, &local);
        if (!rc && !c.directed) rc = srt_mirror_lower_device(n, n, d_rel, st);
        srt_sparse_graph_free(sg);
        if (rc) goto out;
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

/* ------------------------------------------------------------------------------------------ */
/* In-process multi-GPU build (Shadow is one process): one host thread per GPU, RCCL           */
/* communicators from ncclCommInitAll, the same sharded kernels as the one-process-per-GPU     */
/* path (dense: row shards + pivot-panel broadcast; sparse: source shards + allgather).        */
/* ------------------------------------------------------------------------------------------ */
#include <pthread.h>

typedef struct {
    int rank, R, dev, directed, algo, n, ld;
    int virt; /* virtual ranks on one device: per-rank state slots */
    srt_comm* comm;
    const srt_canon* c;
    const uint32_t* hw; /* dense: host w/r matrices, ld x ld */
    const double* hr;
    uint32_t* lat_q; /* host outputs, n x n */
    double* rel;
    int rc;
    char err[256];
    srt_build_stats st;
} mjob;

static void mjob_fail(mjob* j, int rc) {
    j->rc = rc;
    snprintf(j->err, sizeof(j->err), "%s", srt_last_error());
}

static void* mjob_dense(void* p) {
    mjob* j = (mjob*)p;
    int rc = SRT_OK;
    dbufs B;
    B.k = 0;
    hipStream_t st = NULL;
    int32_t b, e;
    srt_shard_rows(j->ld, SRT_SHARD_ALIGN, j->R, j->rank, &b, &e);
    const int nr = e - b;
    const size_t rows = (size_t)(nr > 0 ? nr : 1) * j->ld;
    uint32_t *dw, *dlat;
    double *dr, *drel;
    srt_set_virtual_slot(j->virt ? j->rank : -1);
    TRYHIP(hipSetDevice(j->dev));
    TRYHIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    TRY(dalloc(&B, (void**)&dw, rows * sizeof(uint32_t)));
    TRY(dalloc(&B, (void**)&dr, rows * sizeof(double)));
    TRY(dalloc(&B, (void**)&dlat, rows * sizeof(uint32_t)));
    TRY(dalloc(&B, (void**)&drel, rows * sizeof(double)));
    if (nr > 0) {
        TRYHIP(hipMemcpyAsync(dw, j->hw + (size_t)b * j->ld, (size_t)nr * j->ld * sizeof(uint32_t),
                              hipMemcpyHostToDevice, st));
        TRYHIP(hipMemcpyAsync(dr, j->hr + (size_t)b * j->ld, (size_t)nr * j->ld * sizeof(double),
                              hipMemcpyHostToDevice, st));
    }
    TRY(srt_dense_build_sharded(j->comm, j->n, j->ld, j->directed, dw, dr, dlat, drel, st, 0, &j->st));
    {
        const int r1 = e < j->n ? e : j->n;
        if (r1 > b) {
            TRYHIP(hipMemcpy2DAsync(j->lat_q + (size_t)b * j->n, (size_t)j->n * sizeof(uint32_t), dlat,
                                    (size_t)j->ld * sizeof(uint32_t), (size_t)j->n * sizeof(uint32_t),
                                    r1 - b, hipMemcpyDeviceToHost, st));
            TRYHIP(hipMemcpy2DAsync(j->rel + (size_t)b * j->n, (size_t)j->n * sizeof(double), drel,
                                    (size_t)j->ld * sizeof(double), (size_t)j->n * sizeof(double),
                                    r1 - b, hipMemcpyDeviceToHost, st));
        }
        TRYHIP(hipStreamSynchronize(st));
    }
out:
    if (rc) mjob_fail(j, rc);
    if (st) (void)hipStreamDestroy(st);
    dfree(&B);
    return NULL;
}

static void* mjob_sparse(void* p) {
    mjob* j = (mjob*)p;
    int rc = SRT_OK;
    dbufs B;
    B.k = 0;
    hipStream_t st = NULL;
    srt_sparse_graph* sg = NULL;
    const int n = j->n, per = srt_ceil_div(n, j->R);
    const int s0 = j->rank * per, s1 = (s0 + per < n) ? s0 + per : n;
    const size_t all = (size_t)per * j->R * n;
    uint32_t* dlat;
    double* drel;
    srt_set_virtual_slot(j->virt ? j->rank : -1);
    TRYHIP(hipSetDevice(j->dev));
    TRYHIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    TRY(sparse_graph_from_canon(j->c, j->dev, &sg));
    TRY(dalloc(&B, (void**)&dlat, all * sizeof(uint32_t)));
    TRY(dalloc(&B, (void**)&drel, all * sizeof(double)));
    if (s1 > s0)
        TRY(srt_sparse_graph_rows(sg, s0, s1, dlat + (size_t)s0 * n, drel + (size_t)s0 * n, st, &j->st));
    /* the symmetry rule needs the other shards' rows: gather, mirror, keep our block */
    TRY(srt_sparse_allgather(j->comm, n, per, dlat, drel, st));
    if (!j->directed) TRY(srt_mirror_lower_device(n, n, drel, st));
    if (s1 > s0) {
        TRYHIP(hipMemcpyAsync(j->lat_q + (size_t)s0 * n, dlat + (size_t)s0 * n,
                              (size_t)(s1 - s0) * n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        TRYHIP(hipMemcpyAsync(j->rel + (size_t)s0 * n, drel + (size_t)s0 * n,
                              (size_t)(s1 - s0) * n * sizeof(double), hipMemcpyDeviceToHost, st));
    }
    TRYHIP(hipStreamSynchronize(st));
out:
    if (rc) mjob_fail(j, rc);
    if (sg) srt_sparse_graph_free(sg);
    if (st) (void)hipStreamDestroy(st);
    dfree(&B);
    return NULL;
}

extern "C" int srt_build_tables_multi(const srt_edges* g, const srt_build_opts* opts, int32_t ngpus,
                                      uint32_t* lat_q, uint64_t* quantum_ns, double* rel,
                                      srt_build_stats* stats) {
    if (!g || !lat_q || !quantum_ns || !rel || ngpus < 1) {
        srt_set_error("srt_build_tables_multi: bad argument");
        return SRT_E_ARG;
    }
    const int avail = srt_device_count();
    if (avail < 1) {
        srt_set_error("srt_build_tables_multi: no HIP device");
        return SRT_E_DEVICE;
    }
    /* SRT_VIRTUAL_RANKS=R (tests): R ranks on device 0, collectives as device copies */
    const char* venv = getenv("SRT_VIRTUAL_RANKS");
    const int virt = venv && atoi(venv) > 0 ? (atoi(venv) < 64 ? atoi(venv) : 64) : 0;
    const int R = virt ? virt : (ngpus < avail ? ngpus : avail);
    const int use_sp = opts ? opts->use_shortest_path : 1;
    if (!use_sp) return srt_build_tables(g, opts, lat_q, quantum_ns, rel, stats);
    srt_canon c;
    int rc = srt_canon_build(g, &c);
    if (rc) return rc;
    *quantum_ns = c.quantum_ns;
    const int n = c.n;
    const int algo = choose_algo(&c, opts);
    const int ld = srt_ceil_div(n, SRT_SHARD_ALIGN) * SRT_SHARD_ALIGN;
    uint32_t* hw = NULL;
    double* hr = NULL;
    srt_comm** comms = (srt_comm**)calloc((size_t)R, sizeof(srt_comm*));
    mjob* jobs = (mjob*)calloc((size_t)R, sizeof(mjob));
    pthread_t* th = (pthread_t*)calloc((size_t)R, sizeof(pthread_t));
    int* devs = (int*)calloc((size_t)R, sizeof(int));
    if (!comms || !jobs || !th || !devs) {
        rc = SRT_E_NOMEM;
        goto done;
    }
    if (algo == SRT_ALGO_DENSE_FW) {
        const size_t ll = (size_t)ld * ld;
        hw = (uint32_t*)malloc(ll * sizeof(uint32_t));
        hr = (double*)malloc(ll * sizeof(double));
        if (!hw || !hr) {
            rc = SRT_E_NOMEM;
            goto done;
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
    }
    for (int i = 0; i < R; i++) devs[i] = virt ? 0 : i;
    if ((rc = virt ? srt_comm_init_virtual(R, 0, comms) : srt_comm_init_all(R, devs, comms)))
        goto done;
    for (int i = 0; i < R; i++) {
        mjob* j = &jobs[i];
        j->rank = i;
        j->R = R;
        j->virt = virt;
        j->dev = devs[i];
        j->directed = c.directed;
        j->algo = algo;
        j->n = n;
        j->ld = ld;
        j->comm = comms[i];
        j->c = &c;
        j->hw = hw;
        j->hr = hr;
        j->lat_q = lat_q;
        j->rel = rel;
        if (pthread_create(&th[i], NULL, algo == SRT_ALGO_DENSE_FW ? mjob_dense : mjob_sparse, j)) {
            /* a collective would wait forever for the missing rank: refuse before any started */
            for (int k = 0; k < i; k++) pthread_join(th[k], NULL);
            rc = SRT_E_NOMEM;
            srt_set_error("srt_build_tables_multi: pthread_create failed");
            goto done;
        }
    }
    for (int i = 0; i < R; i++) pthread_join(th[i], NULL);
    for (int i = 0; i < R && !rc; i++)
        if (jobs[i].rc) {
            rc = jobs[i].rc;
            srt_set_error("rank %d: %s", i, jobs[i].err);
        }
    if (!rc && stats) *stats = jobs[0].st;
done:
    if (comms)
        for (int i = 0; i < R; i++)
            if (comms[i]) srt_comm_free(comms[i]);
    free(comms);
    free(jobs);
    free(th);
    free(devs);
    free(hw);
    free(hr);
    srt_canon_free(&c);
    return rc;
}
