/*
 * build.hip -- host orchestration of one routing-table build on one GPU.
 *
 * Replaces the lazy per-source Dijkstra of /root/reference/src/main/routing/topology.c:1578-1814
 * (run on a cache miss from _topology_getPathEntry, :1923-1961) with one eager all-pairs build:
 *   use_shortest_path == false : direct edge gather (topology.c:1816-1858)
 *   dense graphs               : blocked Floyd-Warshall (fw16.hip) + predecessor/reliability pass
 *                                (dense.hip)
 *   sparse graphs              : multi-source shared-frontier SSSP, 64 sources per workgroup,
 *                                on local graphs (msssp.hip); otherwise per-source bucket SSSP
 *                                with settle-time predecessor and reliability (wsssp.hip, one
 *                                wave or one workgroup per source; sparse.hip for overflowing
 *                                sources)
 * Every table row is its own source's row; pairorder.c decides which row serves a pair.
 * Every path runs on the GPU; a device failure is returned as SRT_E_DEVICE, never replaced by a
 * host computation.
 */
#include <stdlib.h>
#include <string.h>

#include <pthread.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <vector>

#include "srt_device.h"

int srt_sparse_block_rows(int32_t n, const int32_t* rowptr, const int32_t* col, const uint32_t* w,
                          const double* r, const int32_t* in_rowptr, const int32_t* in_col,
                          const uint32_t* in_w, const double* in_r, const uint32_t* self_w,
                          const double* self_r, int32_t src_begin, int32_t src_end,
                          const int32_t* srcs, uint32_t delta, uint32_t* lat_rows,
                          double* rel_rows, void* stream, srt_build_stats* stats);

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

/* AUTO: FW costs n^3 cheap register/LDS relaxations, the SSSP ~ n * arcs gathers, so dense wins
 * once arcs are within ~1/16 of n^2 (or the graph is tiny) -- up to the dense form's size limit
 * (srt_dense_max_n: 16-bit predecessor keys, int32 arc offsets). Everything else, of any size,
 * takes the sparse SSSP, like the reference's per-source Dijkstra (topology.c:1578-1814). An
 * explicit DENSE_FW request beyond the limit is refused before any work (SRT_E_RANGE). */
static int choose_algo(const srt_canon* c, const srt_build_opts* o) {
    if (o && o->algo == SRT_ALGO_DENSE_FW) return SRT_ALGO_DENSE_FW;
    if (o && o->algo == SRT_ALGO_SPARSE_SSSP) return SRT_ALGO_SPARSE_SSSP;
    const double n = c->n;
    const bool dense_shape = c->n <= 2048 || (double)c->arcs * 16.0 >= n * n;
    return dense_shape && c->n <= SRT_DENSE_MAX_N ? SRT_ALGO_DENSE_FW : SRT_ALGO_SPARSE_SSSP;
}

/* ---- device-resident sparse graph (canonical CSR uploaded once, rows computed per shard) ---- */
struct srt_sparse_graph {
    int device;
    int32_t n, directed;
    int64_t arcs;
    uint64_t quantum_ns;
    uint32_t delta, max_w;
    uint64_t dist_bound; /* srt_canon.dist_bound */
    int wide;            /* srt_canon.wide: u64 rows (wide.hip) */
    int local; /* relabelled arcs span <= 4096 vertices on average (graph.c CM order) */
    int32_t *rp, *col, *irp, *icol;
    uint32_t *w, *iw, *sw;
    double *r, *ir, *sr;
    uint2 *cw, *icw; /* packed (col, w) arcs for the wave-per-source kernel */
    /* the same graph relabelled in Cuthill-McKee order for the wave-per-source kernel: perm[new] =
     * old, inv[old] = new; rows keep their arcs sorted by ORIGINAL neighbour index */
    int32_t *perm, *inv;
    int2 *rp2, *irp2; /* (begin, end) of each relabelled row */
    int2* rpo;        /* (begin, end) of each original row (the workgroup kernel's order) */
    /* the distinct arc reliabilities (<= 256 of them, else NULL) and each arc's index into them */
    double* rtab;
    uint8_t* ridx;
    uint2 *cw2, *icw2;
    double *r2, *ir2;
    /* host copy of the relabelled out-rows, for the multi-source kernel's source clusters */
    int2* h_rp2;
    uint2* h_cw2;
    int32_t* h_inv;
    /* the clusters of the last source set (the same rows are usually asked for again): the
     * sources (original ids, or the range [ck_b0, ck_b0 + ck_n) when ck_list is 0), the radius,
     * then nbatch x 64 sources and rows and the rows left to the single-source kernels */
    int32_t ck_n, ck_b0, ck_list, ck_rmax, ck_maxb, ck_nb, ck_nrest;
    int32_t *ck_srcs, *ck_bsrc, *ck_brow, *ck_rest;
    pthread_mutex_t ck_mu; /* all-zero (calloc) is the default mutex */
    /* neighbour-row derivation (derive.hip, undirected): an independent set I of vertices of
     * degree <= DERIVE_MAXDEG and the rest ("core"), both ascending; crow[v] = v's index in the
     * core list (-1 for I) */
    int32_t nI, ncore;
    int64_t degI; /* summed degree of I (the derivation's neighbour-row reads) */
    int32_t *dI, *dcore, *crow;
    int32_t ntab; /* entries of rtab */
    /* the derived build's canonical-arc codes of the core rows (ncore x n u32; C5: 21.6 GB), kept
     * across builds: from the scratch pool they were re-mapped by every build (past the pool's
     * release threshold), and builds whose fresh mapping came out fragmented ran wgsssp_kernel at
     * 620-765 ms instead of ~396 */
    uint32_t* codes;
    size_t codes_cap;
    pthread_mutex_t codes_mu;
};

#define DERIVE_MAXDEG SRT_DERIVE_MAXDEG /* derive.hip's DV_MAXDEG */

int srt_wgsssp_max_n(void);
int srt_wide_rows(int n, const int32_t* rp, const int32_t* col, const uint32_t* w, const double* r,
                  const int32_t* irp, const int32_t* icol, const uint32_t* iw, const double* ir,
                  const uint32_t* sw, const double* sr, uint64_t quantum_ns, int src_begin,
                  int src_end, const int32_t* srcs, uint32_t* lat, double* rel, double* lms,
                  size_t ldo, hipStream_t st);
int srt_wgsssp_rows(int n, const int2* rowptr, const uint2* cw, const double* r, const int32_t* inv,
                    uint32_t max_w, int src_begin, int src_end, const int32_t* srcs, uint32_t* lat,
                    double* rel, int* ovf, hipStream_t st, const uint8_t* ridx,
                    const double* rtab, int place = 0, uint32_t* codes = nullptr);
int srt_derive_rows_async(int n, int nI, const int32_t* I, int src_begin, const int2* rowptr,
                          const uint2* cw, const uint8_t* ridx, const double* rtab, int ntab,
                          const int32_t* crow, const uint32_t* codes, uint32_t* lat, double* rel,
                          size_t ldo, hipStream_t st);
int srt_wsssp_rows(int n, int directed, const int2* rowptr, const uint2* cw, const double* r,
                   const int2* in_rowptr, const uint2* in_cw, const double* in_r,
                   const int32_t* perm, const int32_t* inv, uint32_t max_w, int local,
                   int src_begin, int src_end, const int32_t* srcs, uint32_t* lat, double* rel,
                   int* ovf, hipStream_t st);
int srt_sparse_last_form(void);
int srt_sparse_diag(int n, int src_begin, int src_end, const int32_t* srcs, const int32_t* rowptr,
                    const int32_t* col, const uint32_t* w, const double* r, const uint32_t* self_w,
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
    void* ps[] = {g->rp, g->col, g->w, g->r, g->sw, g->sr, g->cw, g->perm, g->inv, g->rp2, g->cw2, g->r2,
                  g->rpo, g->rtab, g->ridx, g->dI, g->dcore, g->crow, g->codes};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    if (g->directed) {
        void* qs[] = {g->irp, g->icol, g->iw, g->ir, g->icw, g->irp2, g->icw2, g->ir2};
        for (void* p : qs)
            if (p) (void)hipFree(p);
    }
    (void)hipSetDevice(prev);
    free(g->h_rp2);
    free(g->h_cw2);
    free(g->h_inv);
    free(g->ck_srcs);
    free(g->ck_bsrc);
    free(g->ck_brow);
    free(g->ck_rest);
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

/* The independent set of the neighbour-row derivation: vertices of degree 1..DERIVE_MAXDEG taken
 * greedily in (degree, index) order, each blocking its neighbours (on a BA graph with m = 3 every
 * degree-3 vertex: they are never adjacent). Undirected graphs only. */
static int derive_sets(const srt_canon* c, srt_sparse_graph* g) {
    const int n = c->n;
    std::vector<int32_t> order((size_t)n), I, core;
    std::vector<uint8_t> blocked((size_t)n, 0), inI((size_t)n, 0);
    for (int v = 0; v < n; v++) order[v] = v;
    auto deg = [&](int v) { return c->rowptr[v + 1] - c->rowptr[v]; };
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return deg(a) < deg(b); });
    for (int v : order) {
        const int d = deg(v);
        if (d > DERIVE_MAXDEG) break;
        if (d < 1 || blocked[v]) continue;
        inI[v] = 1;
        blocked[v] = 1;
        for (int k = c->rowptr[v]; k < c->rowptr[v + 1]; k++) blocked[c->col[k]] = 1;
    }
    std::vector<int32_t> crow((size_t)n, -1);
    for (int v = 0; v < n; v++) {
        if (inI[v]) {
            I.push_back(v);
        } else {
            crow[v] = (int32_t)core.size();
            core.push_back(v);
        }
    }
    g->nI = (int32_t)I.size();
    g->ncore = (int32_t)core.size();
    g->degI = 0;
    for (int v : I) g->degI += deg(v);

    int rc = up((void**)&g->dI, I.data(), I.size() * 4);
    if (!rc) rc = up((void**)&g->dcore, core.data(), core.size() * 4);
    if (!rc) rc = up((void**)&g->crow, crow.data(), (size_t)n * 4);
    return rc;
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
    g->dist_bound = c->dist_bound;
    g->wide = c->wide;
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
        for (int32_t v = 0; v < c->n; v++) hrp[v] = make_int2(c->rowptr[v], c->rowptr[v + 1]);
        rc = up((void**)&g->rpo, hrp, nv * sizeof(int2));
        /* table of the distinct arc reliabilities when there are few (generators draw loss from a
         * grid of 1e-4 steps; the workgroup kernel then carries an 8-bit index per arc) */
        if (!rc && na > 0) {
            double* tab = (double*)malloc(na * sizeof(double));
            uint8_t* idx = (uint8_t*)malloc(na);
            if (!tab || !idx) {
                rc = SRT_E_NOMEM;
            } else {
                memcpy(tab, c->r, na * sizeof(double));
                std::sort(tab, tab + na);
                /* bitwise-distinct values (every r is a finite value in [0, 1]) */
                const size_t nt = (size_t)(std::unique(tab, tab + na) - tab);
                if (nt <= 256) {
                    for (size_t k = 0; k < na; k++)
                        idx[k] = (uint8_t)(std::lower_bound(tab, tab + nt, c->r[k]) - tab);
                    rc = up((void**)&g->rtab, tab, nt * sizeof(double));
                    if (!rc) rc = up((void**)&g->ridx, idx, na);
                    g->ntab = (int32_t)nt;
                }
            }
            free(tab);
            free(idx);
        }
        if (!rc) relabel_csr(c->n, c->rowptr, c->col, c->w, c->r, hperm, hinv, hrp, hcw, hr);
        if (!rc) {
            g->h_rp2 = (int2*)malloc(nv * sizeof(int2));
            g->h_cw2 = (uint2*)malloc((na ? na : 1) * sizeof(uint2));
            g->h_inv = (int32_t*)malloc(nv * sizeof(int32_t));
            if (!g->h_rp2 || !g->h_cw2 || !g->h_inv) {
                rc = SRT_E_NOMEM;
            } else {
                memcpy(g->h_rp2, hrp, nv * sizeof(int2));
                memcpy(g->h_cw2, hcw, na * sizeof(uint2));
                memcpy(g->h_inv, hinv, nv * sizeof(int32_t));
            }
        }
        if (!rc) rc = up((void**)&g->perm, hperm, nv * 4);
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
    }
    if (!rc && !c->directed) {
        g->irp2 = g->rp2;
        g->icw2 = g->cw2;
        g->ir2 = g->r2;
        rc = derive_sets(c, g);
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

int srt_msssp_max_n(void);
int srt_ms_scatter_rows(int nr, int n, const int32_t* rows, const uint32_t* tl, const double* tr,
                        uint32_t* lat, double* rel, size_t ldo, hipStream_t st);
int srt_msssp_rows(int n, int directed, const int2* orp, const uint2* ocw, const int2* irp,
                   const uint2* icw, const double* ir, const int32_t* inv, uint32_t delta,
                   int nbatch, const int32_t* bsrc, const int32_t* brow, uint32_t* lat,
                   double* rel, size_t ldo, int d16, hipStream_t st);

/* Sweep order for the source clusters: breadth-first from a pseudo-peripheral vertex of each
 * component (the far end of a breadth-first search from the component's first vertex), so clusters
 * are cut off a front that moves across the graph and leave no scattered remainders behind it. */
static void ms_sweep_order(const srt_sparse_graph* g, std::vector<int32_t>& order) {
    const int n = g->n;
    std::vector<int32_t> seen((size_t)n, -1), q;
    q.reserve((size_t)n);
    order.clear();
    order.reserve((size_t)n);
    int tag = 0;
    auto bfs = [&](int s, std::vector<int32_t>& out) {
        out.clear();
        out.push_back(s);
        seen[s] = tag;
        for (size_t h = 0; h < out.size(); h++)
            for (int a = g->h_rp2[out[h]].x; a < g->h_rp2[out[h]].y; a++) {
                const int v = (int)g->h_cw2[a].x;
                if (seen[v] != tag) {
                    seen[v] = tag;
                    out.push_back(v);
                }
            }
    };
    std::vector<char> placed((size_t)n, 0);
    for (int v0 = 0; v0 < n; v0++) {
        if (placed[v0]) continue;
        ++tag;
        bfs(v0, q); /* the component of v0; its last vertex is far from v0 */
        const int far = q.back();
        ++tag;
        bfs(far, q);
        for (int v : q) placed[v] = 1;
        order.insert(order.end(), q.begin(), q.end());
    }
}

/* Batches of the multi-source kernel (msssp.hip): the sources in groups of 64, each a compact
 * cluster, grown breadth-first (hop radius <= rmax) from the first unassigned source in the sweep
 * order, so the 64 distance fields of a batch stay close everywhere and their frontiers overlap. A
 * group that cannot fill 48 of its 64 lanes within that radius (scattered sources, e.g. a few
 * attached hosts on a large graph; or 8,192 vertices visited first) becomes a batch of its own
 * while all batches fit max_batches (the kernel's concurrent slots), else goes to `rest`, for the
 * single-source kernels: the shared
 * frontier only pays when the sources are close. rowof[v] (relabelled v): the output row of source
 * v, -1 when v is not a source; rest receives output rows. */
static void ms_clusters(const srt_sparse_graph* g, const int32_t* rowof, int nsrc, int rmax,
                        int max_batches, std::vector<int32_t>& bsrc, std::vector<int32_t>& brow,
                        std::vector<int32_t>& rest) {
    std::vector<int32_t> small_src, small_cnt; /* clusters under 48 sources, in order */
    const int n = g->n;
    std::vector<int32_t> order, stamp((size_t)n, -1), queue, depth((size_t)n, 0), found;
    std::vector<char> done((size_t)n, 0);
    ms_sweep_order(g, order);
    int assigned = 0, cl = 0;
    for (int p = 0; p < n && assigned < nsrc; p++) {
        const int seed = order[p];
        if (rowof[seed] < 0 || done[seed]) continue;
        found.clear();
        queue.clear();
        queue.push_back(seed);
        stamp[seed] = cl;
        depth[seed] = 0;
        for (size_t h = 0; h < queue.size() && found.size() < 64; h++) {
            const int u = queue[h];
            if (rowof[u] >= 0 && !done[u]) found.push_back(u);
            /* hop radius, and a visit budget that bounds the host work on small-world graphs */
            if (depth[u] >= rmax || queue.size() >= 8192) continue;
            for (int a = g->h_rp2[u].x; a < g->h_rp2[u].y; a++) {
                const int v = (int)g->h_cw2[a].x;
                if (stamp[v] != cl) {
                    stamp[v] = cl;
                    depth[v] = depth[u] + 1;
                    queue.push_back(v);
                }
            }
        }
        for (int v : found) done[v] = 1;
        assigned += (int)found.size();
        if (found.size() >= 48) {
            const size_t base = bsrc.size();
            bsrc.resize(base + 64, -1);
            brow.resize(base + 64, -1);
            for (size_t k = 0; k < found.size(); k++) {
                bsrc[base + k] = found[k];
                brow[base + k] = rowof[found[k]];
            }
        } else {
            small_cnt.push_back((int32_t)found.size());
            small_src.insert(small_src.end(), found.begin(), found.end());
        }
        cl++;
    }
    /* the small clusters (the sweep's remainders, or sources scattered over the graph) still ride
     * the multi-source kernel while every batch fits the kernel's concurrent slots: a batch costs
     * about the same wall time whatever its lane count, and the single-source kernels would run
     * after it */
    const bool fit = (int)(bsrc.size() / 64 + small_cnt.size()) <= max_batches;
    size_t o = 0;
    for (int32_t c : small_cnt) {
        if (fit) {
            const size_t base = bsrc.size();
            bsrc.resize(base + 64, -1);
            brow.resize(base + 64, -1);
            for (int32_t k = 0; k < c; k++) {
                bsrc[base + k] = small_src[o + k];
                brow[base + k] = rowof[small_src[o + k]];
            }
        } else {
            for (int32_t k = 0; k < c; k++) rest.push_back(rowof[small_src[o + k]]);
        }
        o += (size_t)c;
    }
}

/* Rows of nsrc sources (the device list srcs, or [src_begin, src_end) when srcs is NULL): the
 * wave-per-source bucket kernel (wsssp.hip) when the arc weights fit its bucket ring, or the
 * workgroup kernel with the row packed in LDS on large power-law graphs; any source whose buckets
 * overflowed is recomputed (wave kernel, then the workgroup-per-source kernel of sparse.hip).
 * SRT_FORM kernel=block (or SRT_FORM hbm=1) selects the sparse.hip kernel for every
 * source. lms (optional): the f64 path-order ms rows (tables.hip), q the quantum in ns. */
/* Every row of an undirected graph, placed by source (row v = v): the core rows by the workgroup
 * kernel, with their canonical arcs, then the independent set's rows by derivation (derive.hip).
 * A core source whose buckets overflowed has no codes: then the set's rows take the kernel too.
 * (Deriving each chunk's ready set on a second stream beside the kernel's next chunk measured
 * slower: 829 vs 529 ms on C5.) */
struct derived_times {
    float core = 0, derive = 0; /* HIP-event ms of the core rows' kernel and of the derivation */
    bool fallback = false;      /* a core row overflowed: the set's rows took the kernel */
};

static int sparse_rows_derived(const srt_sparse_graph* g, uint32_t* lat_rows, double* rel_rows,
                               int* ovf, hipStream_t st, derived_times* tm) {
    const int n = g->n;
    struct evs {
        hipEvent_t e[3] = {nullptr, nullptr, nullptr};
        ~evs() {
            for (hipEvent_t x : e)
                if (x) (void)hipEventDestroy(x);
        }
    } ev;
    for (hipEvent_t& x : ev.e) SRT_HIPCHK(hipEventCreate(&x));
    /* the codes: the graph's own buffer (one allocation, same placement every build) when no other
     * build of this graph holds it, else stream-ordered scratch */
    srt_sparse_graph* gm = const_cast<srt_sparse_graph*>(g);
    const size_t cbytes = (size_t)g->ncore * n * sizeof(uint32_t);
    uint32_t* codes = NULL;
    const bool own = pthread_mutex_trylock(&gm->codes_mu) == 0;
    struct unlock {
        pthread_mutex_t* m;
        ~unlock() {
            if (m) pthread_mutex_unlock(m);
        }
    } ul{own ? &gm->codes_mu : nullptr};
    if (own) {
        if (gm->codes_cap < cbytes) {
            SRT_HIPCHK(hipStreamSynchronize(st)); /* earlier builds on st are done with the old one */
            if (gm->codes) (void)hipFree(gm->codes);
            gm->codes = NULL;
            gm->codes_cap = 0;
            if (hipMalloc((void**)&gm->codes, cbytes) != hipSuccess) {
                (void)hipGetLastError();
                gm->codes = NULL;
            } else {
                gm->codes_cap = cbytes;
            }
        }
        codes = gm->codes;
    }
    const bool scratch = codes == NULL;
    if (scratch) SRT_HIPCHK(srt_malloc_async(&codes, cbytes, st));
    SRT_HIPCHK(hipMemsetAsync(ovf, 0, (size_t)n * sizeof(int), st));
    SRT_HIPCHK(hipEventRecord(ev.e[0], st));
    int rc = srt_wgsssp_rows(n, g->rpo, g->cw, g->r, NULL, g->max_w, 0, g->ncore, g->dcore, lat_rows,
                             rel_rows, ovf, st, g->ridx, g->rtab, 1, codes);
    if (!rc && hipEventRecord(ev.e[1], st) != hipSuccess) rc = SRT_E_DEVICE;
    std::vector<int> hov((size_t)n);
    if (!rc && hipMemcpyAsync(hov.data(), ovf, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, st) !=
                   hipSuccess)
        rc = SRT_E_DEVICE;
    if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = SRT_E_DEVICE;
    bool core_ovf = false;
    for (int v = 0; v < n && !rc; v++) core_ovf |= hov[v] != 0;
    if (!rc && core_ovf) /* (the set's flags are still 0: every flag is a core row's) */
        rc = srt_wgsssp_rows(n, g->rpo, g->cw, g->r, NULL, g->max_w, 0, g->nI, g->dI, lat_rows,
                             rel_rows, ovf, st, g->ridx, g->rtab, 1, NULL);
    else if (!rc)
        rc = srt_derive_rows_async(n, g->nI, g->dI, 0, g->rpo, g->cw, g->ridx, g->rtab, g->ntab,
                                   g->crow, codes, lat_rows, rel_rows, (size_t)n, st);
    if (!rc && hipEventRecord(ev.e[2], st) != hipSuccess) rc = SRT_E_DEVICE;
    if (scratch) (void)hipFreeAsync(codes, st);
    if (!rc && hipEventSynchronize(ev.e[2]) == hipSuccess) {
        (void)hipEventElapsedTime(&tm->core, ev.e[0], ev.e[1]);
        (void)hipEventElapsedTime(&tm->derive, ev.e[1], ev.e[2]);
        tm->fallback = core_ovf;
    }
    if (own && rc) (void)hipStreamSynchronize(st); /* the buffer is free before it is unlocked */
    return rc;
}

static int sparse_rows(const srt_sparse_graph* g, int32_t src_begin, int32_t src_end,
                       const int32_t* srcs, uint32_t* lat_rows, double* rel_rows, double* lms,
                       hipStream_t st, srt_build_stats* stats, int allow_ms = 1) {
    if (!g || src_begin < 0 || src_begin >= src_end || (!srcs && src_end > g->n)) {
        srt_set_error("sparse rows: bad source range [%d, %d)", src_begin, src_end);
        return SRT_E_ARG;
    }
    const int nsrc = src_end - src_begin;
    if (g->wide) { /* distances may pass u32 quanta: the u64 rows (wide.hip) */
        struct evs {
            hipEvent_t e[2] = {nullptr, nullptr};
            ~evs() {
                for (hipEvent_t x : e)
                    if (x) (void)hipEventDestroy(x);
            }
        } wev;
        SRT_HIPCHK(hipEventCreate(&wev.e[0]));
        SRT_HIPCHK(hipEventCreate(&wev.e[1]));
        SRT_HIPCHK(hipEventRecord(wev.e[0], st));
        int wrc;
        wrc = srt_wide_rows(g->n, g->rp, g->col, g->w, g->r, g->irp, g->icol, g->iw, g->ir, g->sw,
                            g->sr, g->quantum_ns, src_begin, src_end, srcs, lat_rows, rel_rows, lms,
                            (size_t)g->n, st);
        if (wrc) return wrc;
        SRT_HIPCHK(hipEventRecord(wev.e[1], st));
        SRT_HIPCHK(hipEventSynchronize(wev.e[1]));
        float a = 0;
        SRT_HIPCHK(hipEventElapsedTime(&a, wev.e[0], wev.e[1]));
        if (stats) {
            stats->algo = SRT_ALGO_SPARSE_SSSP;
            stats->ms_fw = a;
            stats->ms_total = a;
            stats->dist_enc = 4;
        }
        return SRT_OK;
    }
    /* source i of this call: srcs + i, or the range */
    auto one = [&](int i) { return srcs ? srcs + i : (const int32_t*)NULL; };
    const int b0 = srcs ? 0 : src_begin;
    /* SRT_FORM kernel=block|ms|wg|wave forces one sparse kernel for every source (tests) */
    const bool block = srt_form_is("kernel", "block");
    int rc = SRT_OK;
    /* the multi-source kernel (msssp.hip) where the relabelled graph is local (RGG-like, where
     * the 64 frontiers of a source cluster overlap). Sources are clustered here, on the host,
     * before the timed span */
    const bool k_ms = srt_form_is("kernel", "ms"), k_wg = srt_form_is("kernel", "wg"),
               k_wave = srt_form_is("kernel", "wave");
    bool ms = allow_ms && !block && g->n <= srt_msssp_max_n() && g->h_rp2 &&
              (k_ms || (!k_wg && !k_wave && g->local != 0));
    std::vector<int32_t> ms_bsrc, ms_brow, ms_rest, hs;
    if (ms) {
        std::vector<int32_t> rowof((size_t)g->n, -1);
        hs.resize((size_t)nsrc);
        if (srcs) SRT_HIPCHK(hipMemcpy(hs.data(), srcs, (size_t)nsrc * 4, hipMemcpyDeviceToHost));
        for (int i = 0; i < nsrc && ms; i++) {
            const int s = srcs ? hs[i] : b0 + i;
            if (s < 0 || s >= g->n || rowof[g->h_inv[s]] >= 0) ms = false; /* duplicates */
            else rowof[g->h_inv[s]] = i;
        }
        /* the hop radius of a cluster */
        const int rmax = 24;
        int cus = 256, dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
            cus = prop.multiProcessorCount;
        const int maxb = 2 * cus; /* the batch budget: two per CU, the rest single-source */
        srt_sparse_graph* gm = const_cast<srt_sparse_graph*>(g); /* the cluster cache */
        pthread_mutex_lock(&gm->ck_mu);
        const bool hit = ms && gm->ck_bsrc && gm->ck_n == nsrc && gm->ck_rmax == rmax &&
                         gm->ck_maxb == maxb &&
                         gm->ck_list == (srcs != NULL) &&
                         (srcs ? !memcmp(gm->ck_srcs, hs.data(), (size_t)nsrc * 4)
                               : gm->ck_b0 == b0);
        if (hit) {
            ms_bsrc.assign(gm->ck_bsrc, gm->ck_bsrc + (size_t)gm->ck_nb * 64);
            ms_brow.assign(gm->ck_brow, gm->ck_brow + (size_t)gm->ck_nb * 64);
            ms_rest.assign(gm->ck_rest, gm->ck_rest + gm->ck_nrest);
        } else if (ms) {
            ms_clusters(g, rowof.data(), nsrc, rmax, maxb, ms_bsrc, ms_brow, ms_rest);
            free(gm->ck_srcs);
            free(gm->ck_bsrc);
            free(gm->ck_brow);
            free(gm->ck_rest);
            gm->ck_n = nsrc;
            gm->ck_b0 = b0;
            gm->ck_list = srcs != NULL;
            gm->ck_rmax = rmax;
            gm->ck_maxb = maxb;
            gm->ck_nb = (int32_t)(ms_bsrc.size() / 64);
            gm->ck_nrest = (int32_t)ms_rest.size();
            gm->ck_srcs = (int32_t*)malloc((size_t)(srcs ? nsrc : 1) * 4);
            gm->ck_bsrc = (int32_t*)malloc((ms_bsrc.size() + 1) * 4);
            gm->ck_brow = (int32_t*)malloc((ms_brow.size() + 1) * 4);
            gm->ck_rest = (int32_t*)malloc((ms_rest.size() + 1) * 4);
            if (gm->ck_srcs && gm->ck_bsrc && gm->ck_brow && gm->ck_rest) {
                if (srcs) memcpy(gm->ck_srcs, hs.data(), (size_t)nsrc * 4);
                memcpy(gm->ck_bsrc, ms_bsrc.data(), ms_bsrc.size() * 4);
                memcpy(gm->ck_brow, ms_brow.data(), ms_brow.size() * 4);
                memcpy(gm->ck_rest, ms_rest.data(), ms_rest.size() * 4);
            } else { /* no cache, no harm */
                free(gm->ck_bsrc);
                gm->ck_bsrc = NULL;
            }
        }
        pthread_mutex_unlock(&gm->ck_mu);
        if (ms_bsrc.empty()) ms = false; /* every source scattered: the single-source kernels */
    }
    if (block || (g->max_w >= 256 && !ms)) {
        const int ct = stats && stats->count_ties;
        rc = srt_sparse_block_rows(g->n, g->rp, g->col, g->w, g->r, g->irp, g->icol, g->iw, g->ir,
                                   g->sw, g->sr, b0, b0 + nsrc, srcs, g->delta, lat_rows, rel_rows,
                                   st, stats);
        if (!rc && ct) {
            stats->count_ties = 1;
            stats->tied_pairs = 0;
            rc = srt_tie_count_rows(g->n, nsrc, srcs, b0, lat_rows, (size_t)g->n, g->irp, g->icol,
                                    g->iw, &stats->tied_pairs, st);
        }
        if (!rc && lms)
            rc = srt_path_ms_rows(g->n, nsrc, srcs, b0, lat_rows, (size_t)g->n, NULL, 0, g->irp,
                                  g->icol, g->iw, g->quantum_ns, lms, (size_t)g->n, st);
        return rc;
    }
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
    SRT_HIPCHK(srt_malloc_async((void**)&sc.ovf, (size_t)nsrc * sizeof(int), st));
    int* const ovf = sc.ovf;
    SRT_HIPCHK(hipEventCreate(&sc.ev[0]));
    SRT_HIPCHK(hipEventCreate(&sc.ev[1]));
    SRT_HIPCHK(hipEventCreate(&sc.ev[2]));
    hipEvent_t e0 = sc.ev[0], e1 = sc.ev[1], e2 = sc.ev[2];
    SRT_HIPCHK(hipEventRecord(e0, st));
    /* large power-law graphs (relabelled arcs far apart): the workgroup kernel with the distance
     * row packed in LDS, once a probe source shows every distance fits its 10-bit fields
     * (d(a, b) <= 2 ecc(s0)); SRT_FORM kernel=wg allows it at any size */
    int32_t* ms_dev = NULL; /* bsrc then brow, freed on the stream after the launch */
    int ms_d16 = 0;
    if (ms) {
        const int nb = (int)(ms_bsrc.size() / 64);
        const size_t bb = ms_bsrc.size() * sizeof(int32_t);
        SRT_HIPCHK(srt_malloc_async((void**)&ms_dev, 2 * bb, st));
        SRT_HIPCHK(hipMemcpyAsync(ms_dev, ms_bsrc.data(), bb, hipMemcpyHostToDevice, st));
        SRT_HIPCHK(hipMemcpyAsync(ms_dev + ms_bsrc.size(), ms_brow.data(), bb,
                                  hipMemcpyHostToDevice, st));
        /* bucket width: 8 mean arc weights (C3: 64 quanta; same-box sweep in DESIGN §5.4) */
        const uint32_t delta = 8u * g->delta;
        /* 16-bit working distances when every finite distance provably fits (half the bytes of
         * every row access) */
        const int d16 = g->dist_bound < 0xFFFFull;
        ms_d16 = d16;
        rc = srt_msssp_rows(g->n, g->directed, g->rp2, g->cw2, g->irp2, g->icw2, g->ir2,
                            g->inv, delta, nb, ms_dev, ms_dev + ms_bsrc.size(), lat_rows, rel_rows,
                            (size_t)g->n, d16, st);
        if (rc) return rc;
        SRT_HIPCHK(hipFreeAsync(ms_dev, st));
        SRT_HIPCHK(hipMemsetAsync(ovf, 0, (size_t)nsrc * sizeof(int), st));
        if (!ms_rest.empty()) {
            /* scattered sources: the single-source kernels into scratch rows, scattered after */
            const int nr = (int)ms_rest.size();
            std::vector<int32_t> rs((size_t)nr);
            for (int i = 0; i < nr; i++) rs[i] = srcs ? hs[ms_rest[i]] : b0 + ms_rest[i];
            int32_t* dr = NULL;
            uint32_t* tl = NULL;
            double* tr = NULL;
            SRT_HIPCHK(srt_malloc_async((void**)&dr, 2 * (size_t)nr * 4, st));
            SRT_HIPCHK(srt_malloc_async((void**)&tl, (size_t)nr * g->n * 4, st));
            SRT_HIPCHK(srt_malloc_async((void**)&tr, (size_t)nr * g->n * 8, st));
            SRT_HIPCHK(hipMemcpyAsync(dr, rs.data(), (size_t)nr * 4, hipMemcpyHostToDevice, st));
            SRT_HIPCHK(hipMemcpyAsync(dr + nr, ms_rest.data(), (size_t)nr * 4,
                                      hipMemcpyHostToDevice, st));
            rc = sparse_rows(g, 0, nr, dr, tl, tr, NULL, st, NULL, 0);
            if (!rc)
                rc = srt_ms_scatter_rows(nr, g->n, dr + nr, tl, tr, lat_rows, rel_rows,
                                         (size_t)g->n, st);
            (void)hipFreeAsync(tr, st);
            (void)hipFreeAsync(tl, st);
            (void)hipFreeAsync(dr, st);
            if (rc) return rc;
        }
    }
    bool derived = false;
    derived_times dtm;
    bool wg = !ms && !g->directed && g->n <= srt_wgsssp_max_n() &&
              (k_wg || (!k_wave && g->n > 32768 && !g->local));
    /* the workgroup kernel keeps its row in LDS (any order serves), so it runs on the original
     * vertex order and writes reliability straight into the output rows */
    const int2* wrp = g->rpo;
    const uint2* wcw = g->cw;
    const double* wr = g->r;
    const int32_t* winv = NULL;
    if (wg) {
        rc = srt_wgsssp_rows(g->n, wrp, wcw, wr, winv, g->max_w, b0, b0 + 1, one(0),
                             lat_rows, rel_rows, ovf, st, g->ridx, g->rtab);
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
        /* every row of the graph in one call (the full table): the core rows by the kernel with
         * their canonical arcs, the independent set's rows derived from them (derive.hip;
         * SRT_FORM derive=0 keeps the kernel for every row) */
        derived = wg && !srcs && b0 == 0 && nsrc == g->n && g->nI > 0 && g->ridx && g->rtab &&
                  g->max_w < 128 && g->arcs < (1 << 20) && srt_form_int("derive", 1) != 0;
        if (derived)
            rc = sparse_rows_derived(g, lat_rows, rel_rows, ovf, st, &dtm);
        else if (wg && nsrc > 1)
            rc = srt_wgsssp_rows(g->n, wrp, wcw, wr, winv, g->max_w, b0 + 1, b0 + nsrc,
                                 one(1), lat_rows + (size_t)g->n, rel_rows + (size_t)g->n, ovf + 1,
                                 st, g->ridx, g->rtab);
        if (rc) return rc;
    }
    if (!wg && !ms)
        rc = srt_wsssp_rows(g->n, g->directed, g->rp2, g->cw2, g->r2, g->irp2, g->icw2, g->ir2,
                            g->perm, g->inv, g->max_w, g->local, b0, b0 + nsrc, srcs, lat_rows,
                            rel_rows, ovf, st);
    if (rc) return rc;
    /* the multi-source kernel's form: 8, | 16 with 16-bit working distances */
    const int form = ms ? 8 | (ms_d16 ? 16 : 0) : srt_sparse_last_form() | (derived ? 64 : 0);
    SRT_HIPCHK(hipEventRecord(e1, st));
    rc = srt_sparse_diag(g->n, b0, b0 + nsrc, srcs, g->rp, g->col, g->w, g->r, g->sw, g->sr,
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
        uint32_t* lr = lat_rows + (size_t)i * g->n;
        double* rr = rel_rows + (size_t)i * g->n;
        int again = 1;
        if (wg) { /* the workgroup kernel's overflow: the wave kernel first */
            if (!ovf1) SRT_HIPCHK(hipMalloc((void**)&ovf1, sizeof(int)));
            rc = srt_wsssp_rows(g->n, g->directed, g->rp2, g->cw2, g->r2, g->irp2, g->icw2, g->ir2,
                                g->perm, g->inv, g->max_w, g->local, b0 + i, b0 + i + 1, one(i), lr,
                                rr, ovf1, st);
            if (!rc && hipMemcpyAsync(&again, ovf1, sizeof(int), hipMemcpyDeviceToHost, st) ==
                           hipSuccess &&
                hipStreamSynchronize(st) != hipSuccess)
                rc = SRT_E_DEVICE;
            if (!rc && !again) /* the wave kernel wrote the row; the diagonal rule again */
                rc = srt_sparse_diag(g->n, b0 + i, b0 + i + 1, one(i), g->rp, g->col, g->w, g->r,
                                     g->sw, g->sr, lr, rr, (size_t)g->n, st);
        }
        if (!rc && again)
            rc = srt_sparse_block_rows(g->n, g->rp, g->col, g->w, g->r, g->irp, g->icol, g->iw,
                                       g->ir, g->sw, g->sr, b0 + i, b0 + i + 1, one(i), g->delta,
                                       lr, rr, st, NULL);
    }
    if (rc) return rc;
    if (lms &&
        (rc = srt_path_ms_rows(g->n, nsrc, srcs, b0, lat_rows, (size_t)g->n, NULL, 0, g->irp,
                               g->icol, g->iw, g->quantum_ns, lms, (size_t)g->n, st)))
        return rc;
    SRT_HIPCHK(hipEventRecord(e2, st));
    SRT_HIPCHK(hipEventSynchronize(e2));
    float a = 0, b = 0;
    SRT_HIPCHK(hipEventElapsedTime(&a, e0, e1));
    SRT_HIPCHK(hipEventElapsedTime(&b, e0, e2));
    int64_t tied = 0; /* outside the timed span: a check pass, not part of the build */
    if (stats && stats->count_ties &&
        (rc = srt_tie_count_rows(g->n, nsrc, srcs, b0, lat_rows, (size_t)g->n, g->irp, g->icol,
                                 g->iw, &tied, st)))
        return rc;
    if (nov) srt_log(SRT_LOG_INFO, "wsssp: %d of %d sources overflowed their buckets and were "
                     "recomputed", nov, nsrc);
    if (stats) {
        stats->algo = SRT_ALGO_SPARSE_SSSP;
        stats->ms_fw = b;
        stats->ms_total = b;
        stats->n_update = 1;
        stats->ms_update = a;
        stats->ess_arcs = nov; /* sparse builds: sources recomputed after a bucket overflow */
        /* sparse builds: 3 = multi-source kernel, 2 = workgroup kernel, 1 = wave kernel */
        stats->dist_enc = ms ? 3 : wg ? 2 : 1;
        stats->fw_block = form;       /* sparse builds: the kernel's form (srt_sparse_last_form) */
        stats->tied_pairs = tied;
        /* derived builds: the split of the timed span, and the derivation's algorithmic bytes per
         * row -- the neighbours' distance rows (4 B per target each), one optimal neighbour's
         * canonical arcs (4 B) and the output rows (4 + 8 B) */
        stats->n_derived = derived && !dtm.fallback ? g->nI : 0;
        stats->ms_core = derived ? dtm.core : 0.0;
        stats->ms_derive = derived ? dtm.derive : 0.0;
        stats->work_bytes = stats->n_derived ? (g->degI + 4 * (int64_t)g->nI) * 4 * (int64_t)g->n : 0;
    }
    return SRT_OK;
}

extern "C" int srt_sparse_graph_rows(const srt_sparse_graph* g, int32_t src_begin, int32_t src_end,
                                     uint32_t* lat_rows, double* rel_rows, void* stream,
                                     srt_build_stats* stats) {
    if (!g) {
        srt_set_error("srt_sparse_graph_rows: null graph");
        return SRT_E_ARG;
    }
    if (g->wide) { /* the u32 rows would saturate: only the f64 ms rows carry these latencies */
        srt_set_error("srt_sparse_graph_rows: shortest-path latencies may pass the u32 range; use "
                      "srt_sparse_graph_rows_list with lat_ms_rows");
        return SRT_E_RANGE;
    }
    return sparse_rows(g, src_begin, src_end, NULL, lat_rows, rel_rows, NULL, (hipStream_t)stream,
                       stats);
}

extern "C" int srt_sparse_graph_rows_list(const srt_sparse_graph* g, int32_t nsrc,
                                          const int32_t* srcs, uint32_t* lat_rows, double* rel_rows,
                                          double* lat_ms_rows, void* stream,
                                          srt_build_stats* stats) {
    if (!g || nsrc <= 0 || !srcs || !lat_rows || !rel_rows) {
        srt_set_error("srt_sparse_graph_rows_list: bad arguments");
        return SRT_E_ARG;
    }
    if (g->wide && !lat_ms_rows) { /* the u32 rows would saturate (SRT_INF - 1) */
        srt_set_error("srt_sparse_graph_rows_list: shortest-path latencies may pass the u32 range; "
                      "the f64 lat_ms_rows output is required");
        return SRT_E_RANGE;
    }
    return sparse_rows(g, 0, nsrc, srcs, lat_rows, rel_rows, lat_ms_rows, (hipStream_t)stream, stats);
}

/* ------------------------------------------------------------------------------------------ */
/* Table build over a vertex subset (the attached vertices, topology.c:1604-1656): entry [i][j]  */
/* is the pair (verts[i], verts[j]); verts strictly increasing, so the subset keeps vertex       */
/* order and the undirected rule "pair computed from min(s, t)" is the sub-table's upper         */
/* triangle. verts == NULL: every vertex (nsub = n).                                             */
/* ------------------------------------------------------------------------------------------ */
static void merge_stats(srt_build_stats* acc, const srt_build_stats* s, int first) {
    if (first) {
        *acc = *s;
        return;
    }
    acc->ms_total += s->ms_total;
    acc->ms_fw += s->ms_fw;
    acc->ms_post += s->ms_post;
    acc->ms_update += s->ms_update;
    acc->n_update += s->n_update;
    acc->ess_arcs += s->ess_arcs;
    acc->tied_pairs += s->tied_pairs;
    acc->max_depth = s->max_depth > acc->max_depth ? s->max_depth : acc->max_depth;
    if (s->dist_enc < acc->dist_enc) acc->dist_enc = s->dist_enc;
}

static int check_verts(int n, int nsub, const int32_t* verts) {
    if (!verts) return nsub == n ? SRT_OK : SRT_E_ARG;
    if (nsub < 1 || nsub > n) return SRT_E_ARG;
    for (int i = 0; i < nsub; i++)
        if (verts[i] < 0 || verts[i] >= n || (i && verts[i] <= verts[i - 1])) return SRT_E_ARG;
    return SRT_OK;
}

/* device memory for row chunks after `reserved` bytes: what is free beyond a 12 GiB reserve,
 * capped at 48 GiB; when less than that reserve is free, half of what is free. `sharers` ranks
 * (virtual ranks on one device) read the same free figure at once, so each takes its share. */
static size_t chunk_budget(size_t reserved, int sharers) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        return (size_t)1 << 30;
    }
    size_t budget;
    if (free_b > reserved + ((size_t)12 << 30)) {
        budget = free_b - reserved - ((size_t)12 << 30);
        if (budget > ((size_t)48 << 30)) budget = (size_t)48 << 30;
    } else {
        budget = free_b > reserved ? (free_b - reserved) / 2 : 0;
    }
    return budget / (size_t)(sharers > 1 ? sharers : 1);
}

/* ------------------------------------------------------------------------------------------ */
/* Host <-> device staging of the dense matrices and the tables. No n x n host matrix is built:  */
/* host threads fill (or drain) one pinned slot of a two-slot ring while the DMA engine moves    */
/* the other, so the 12 B/pair cross PCIe once at the link's rate and the first touch of the     */
/* caller's pageable table pages is spread over the threads. Slots are cached for the process.   */
/* ------------------------------------------------------------------------------------------ */
#define STG_SLOT ((size_t)64 << 20)
#define STG_CACHE 16

static pthread_mutex_t stg_mu = PTHREAD_MUTEX_INITIALIZER;
static void* stg_free_slots[STG_CACHE];
static int stg_nfree = 0;

static void* stg_get(void) {
    void* p = NULL;
    pthread_mutex_lock(&stg_mu);
    if (stg_nfree > 0) p = stg_free_slots[--stg_nfree];
    pthread_mutex_unlock(&stg_mu);
    if (!p && hipHostMalloc(&p, STG_SLOT, hipHostMallocPortable) != hipSuccess) p = NULL;
    return p;
}

static void stg_put(void* p) {
    if (!p) return;
    pthread_mutex_lock(&stg_mu);
    if (stg_nfree < STG_CACHE) {
        stg_free_slots[stg_nfree++] = p;
        p = NULL;
    }
    pthread_mutex_unlock(&stg_mu);
    if (p) (void)hipHostFree(p);
}

static double host_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* host threads for one rank's staging: the CPUs (at most 16) shared by `sharers` ranks */
static int stg_threads(int sharers) {
    long c = sysconf(_SC_NPROCESSORS_ONLN);
    c = c < 1 ? 1 : c > 16 ? 16 : c;
    c /= sharers > 1 ? sharers : 1;
    return c < 1 ? 1 : (int)c;
}

typedef struct {
    void (*fn)(void* ctx, int part, int nparts);
    void* ctx;
    int part, nparts;
} par_arg;

static void* par_main(void* p) {
    par_arg* a = (par_arg*)p;
    a->fn(a->ctx, a->part, a->nparts);
    return NULL;
}

/* fn(ctx, i, nt) for i < nt, part 0 on the calling thread */
static void par_run(int nt, void (*fn)(void*, int, int), void* ctx) {
    pthread_t th[16];
    par_arg arg[16];
    int started[16] = {0};
    nt = nt < 1 ? 1 : nt > 16 ? 16 : nt;
    for (int i = 1; i < nt; i++) {
        arg[i] = {fn, ctx, i, nt};
        started[i] = pthread_create(&th[i], NULL, par_main, &arg[i]) == 0;
        if (!started[i]) fn(ctx, i, nt); /* no thread: do the part here */
    }
    fn(ctx, 0, nt);
    for (int i = 1; i < nt; i++)
        if (started[i]) pthread_join(th[i], NULL);
}

typedef struct {
    const srt_canon* c;
    int ld, r0, rows;
    uint32_t* w;
    double* r;
} fill_ctx;

/* rows [r0, r0 + rows) of the dense matrices: SRT_INF / 0 off the arcs, the arcs' quanta and
 * reliabilities, the self-loop on the diagonal (rows >= n stay SRT_INF / 0) */
static void fill_part(void* p, int part, int nparts) {
    const fill_ctx* f = (const fill_ctx*)p;
    const srt_canon* c = f->c;
    const int a = (int)((int64_t)f->rows * part / nparts), b = (int)((int64_t)f->rows * (part + 1) / nparts);
    for (int i = a; i < b; i++) {
        uint32_t* wr = f->w + (size_t)i * f->ld;
        double* rr = f->r + (size_t)i * f->ld;
        for (int t = 0; t < f->ld; t++) {
            wr[t] = SRT_INF;
            rr[t] = 0.0;
        }
        const int u = f->r0 + i;
        if (u >= c->n) continue;
        for (int k = c->rowptr[u]; k < c->rowptr[u + 1]; k++) {
            wr[c->col[k]] = c->w[k];
            rr[c->col[k]] = c->r[k];
        }
        wr[u] = c->self_w[u];
        rr[u] = c->self_r[u];
    }
}

typedef struct {
    char* dst;
    size_t dpitch, width;
    const char* src;
    int rows;
} drain_ctx;

static void drain_part(void* p, int part, int nparts) {
    const drain_ctx* d = (const drain_ctx*)p;
    const int a = (int)((int64_t)d->rows * part / nparts), b = (int)((int64_t)d->rows * (part + 1) / nparts);
    if (d->dpitch == d->width)
        memcpy(d->dst + (size_t)a * d->width, d->src + (size_t)a * d->width, (size_t)(b - a) * d->width);
    else
        for (int i = a; i < b; i++) memcpy(d->dst + (size_t)i * d->dpitch, d->src + (size_t)i * d->width, d->width);
}

/* ---- the edge-list form: the edges themselves go to the device and are scattered there ---- */
#define SRT_FALLBACK_CANON (-1000) /* internal: redo the build from the host canonical form */

typedef struct {
    const srt_edges* g;
    uint64_t q[16], mx[16];
    int64_t selfl[16];
    int bad[16];
} scan_ctx;

static uint64_t gcd_u64(uint64_t a, uint64_t b) {
    while (b) {
        const uint64_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}

/* the gcd, the maximum and the self-loops of a slice of the edges; bad = a non-positive latency
 * or an endpoint out of range (the host canonical form then reports it) */
static void scan_part(void* p, int part, int nparts) {
    scan_ctx* s = (scan_ctx*)p;
    const srt_edges* g = s->g;
    const int64_t a = g->m * part / nparts, b = g->m * (part + 1) / nparts;
    uint64_t q = 0, mx = 0;
    int64_t sl = 0;
    int bad = 0;
    /* divisibility by the running gcd q = 2^t d (d odd) without a division: l % q == 0 iff
     * ctz(l) >= t and (l >> t) * d^-1 (mod 2^64) <= (2^64 - 1) / d */
    int t = 0;
    uint64_t dinv = 1, lim = ~0ull;
    for (int64_t e = a; e < b; e++) {
        const int64_t l = g->lat_ns[e];
        const int32_t u = g->src[e], v = g->dst[e];
        bad |= (l <= 0) | ((uint32_t)u >= (uint32_t)g->n) | ((uint32_t)v >= (uint32_t)g->n);
        sl += u == v;
        const uint64_t x = (uint64_t)l;
        mx = x > mx ? x : mx;
        if (q == 0 || __builtin_ctzll(x | (1ull << 63)) < t || (x >> t) * dinv > lim) {
            if (l <= 0) continue;
            q = gcd_u64(q, x);
            t = __builtin_ctzll(q);
            const uint64_t d = q >> t;
            dinv = d; /* Newton: d * dinv == 1 (mod 2^64) after five steps from d */
            for (int i = 0; i < 5; i++) dinv *= 2 - d * dinv;
            lim = ~0ull / d;
        }
    }
    s->q[part] = q;
    s->mx[part] = mx;
    s->selfl[part] = sl;
    s->bad[part] = bad;
}

/* the edge-list form of a graph whose dense build can start from its edges: 0 = built, 1 = take
 * the host canonical form (invalid edges, a distance bound that may pass u32 quanta, too many
 * edges for the device copy, edge indices past u32) */
static int canon_from_edges(const srt_edges* g, srt_canon* c) {
    memset(c, 0, sizeof(*c));
    if (!g || g->n <= 0 || g->m <= 0 || g->m >= 0xFFFFFFFFll ||
        (size_t)g->m * 24 > ((size_t)96 << 30))
        return 1;
    scan_ctx s;
    memset(&s, 0, sizeof(s));
    s.g = g;
    const int nt = g->m >= (1 << 20) ? stg_threads(1) : 1;
    par_run(nt, scan_part, &s);
    uint64_t q = 0, mx = 0;
    int64_t sl = 0;
    for (int i = 0; i < nt; i++) {
        if (s.bad[i]) return 1;
        q = gcd_u64(q, s.q[i]);
        mx = s.mx[i] > mx ? s.mx[i] : mx;
        sl += s.selfl[i];
    }
    const uint64_t mq = mx / q;
    if (mq >= SRT_INF / 2 || (uint64_t)(g->n - 1) * mq >= SRT_INF) return 1;
    c->n = g->n;
    c->directed = g->directed;
    c->quantum_ns = q;
    c->max_w_q = (uint32_t)mq;
    c->dist_bound = (uint64_t)(g->n - 1) * mq;
    c->arcs = (g->m - sl) * (g->directed ? 1 : 2); /* upper bound until the scatter counts them */
    c->edges = g;
    return 0;
}

/* rows [row0, row0 + nrows) of the dense matrices from the edge list: the edges staged to the
 * device through the pinned ring (each chunk's minima scattered as it lands), the lowest-index
 * pass, then quanta / reliabilities in place */
static int dense_scatter(const srt_canon* c, int ld, int row0, int nrows, uint32_t* dw, double* dr,
                         hipStream_t st, int sharers, unsigned long long* arcs_out) {
    const srt_edges* g = c->edges;
    const int64_t m = g->m;
    const int64_t per = (int64_t)(STG_SLOT / 24);
    dbufs B;
    B.k = 0;
    int rc = SRT_OK;
    int32_t *es = NULL, *ed = NULL;
    int64_t* el = NULL;
    double* eloss = NULL;
    unsigned long long* darcs = NULL;
    void* slot[2] = {stg_get(), stg_get()};
    hipEvent_t ev[2] = {NULL, NULL};
    const int nt = stg_threads(sharers);
    unsigned long long arcs = 0;
    if (!slot[0] || !slot[1]) {
        srt_set_error("dense staging: pinned slots unavailable");
        rc = SRT_E_DEVICE;
        goto out;
    }
    TRY(dalloc(&B, (void**)&es, (size_t)m * sizeof(int32_t)));
    TRY(dalloc(&B, (void**)&ed, (size_t)m * sizeof(int32_t)));
    TRY(dalloc(&B, (void**)&el, (size_t)m * sizeof(int64_t)));
    TRY(dalloc(&B, (void**)&eloss, (size_t)m * sizeof(double)));
    TRY(dalloc(&B, (void**)&darcs, sizeof(unsigned long long)));
    TRYHIP(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
    TRYHIP(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
    TRYHIP(hipMemsetAsync(darcs, 0, sizeof(unsigned long long), st));
    TRY(srt_scatter_prepare(nrows, ld, dw, dr, st));
    for (int64_t k = 0, e0 = 0; e0 < m; k++, e0 += per) {
        const int s = (int)(k & 1);
        const int64_t cnt = m - e0 < per ? m - e0 : per;
        if (k >= 2) TRYHIP(hipEventSynchronize(ev[s]));
        char* b = (char*)slot[s];
        drain_ctx parts[4] = {
            {b, (size_t)cnt * 4, (size_t)cnt * 4, (const char*)(g->src + e0), 1},
            {b + (size_t)per * 4, (size_t)cnt * 4, (size_t)cnt * 4, (const char*)(g->dst + e0), 1},
            {b + (size_t)per * 8, (size_t)cnt * 8, (size_t)cnt * 8, (const char*)(g->lat_ns + e0), 1},
            {b + (size_t)per * 16, (size_t)cnt * 8, (size_t)cnt * 8, (const char*)(g->loss + e0), 1}};
        for (int a = 0; a < 4; a++) { /* each array as rows of 64 KiB, split over the threads */
            drain_ctx d = parts[a];
            const size_t row = (size_t)64 << 10;
            const size_t full = d.width / row;
            if (full > 0) {
                drain_ctx dd = {d.dst, row, row, d.src, (int)full};
                par_run(nt, drain_part, &dd);
            }
            const size_t done = full * row;
            if (done < d.width) memcpy(d.dst + done, d.src + done, d.width - done);
        }
        TRYHIP(hipMemcpyAsync(es + e0, b, (size_t)cnt * 4, hipMemcpyHostToDevice, st));
        TRYHIP(hipMemcpyAsync(ed + e0, b + (size_t)per * 4, (size_t)cnt * 4, hipMemcpyHostToDevice, st));
        TRYHIP(hipMemcpyAsync(el + e0, b + (size_t)per * 8, (size_t)cnt * 8, hipMemcpyHostToDevice, st));
        TRYHIP(hipMemcpyAsync(eloss + e0, b + (size_t)per * 16, (size_t)cnt * 8, hipMemcpyHostToDevice, st));
        TRYHIP(hipEventRecord(ev[s], st));
        TRY(srt_scatter_min(cnt, es + e0, ed + e0, el + e0, c->directed, row0, nrows, ld, dr, st));
    }
    TRY(srt_scatter_idx(m, es, ed, el, c->directed, row0, nrows, ld, dr, dw, st));
    TRY(srt_scatter_final(row0, nrows, ld, c->quantum_ns, eloss, dw, dr, darcs, st));
    TRYHIP(hipMemcpyAsync(&arcs, darcs, sizeof(arcs), hipMemcpyDeviceToHost, st));
    TRYHIP(hipStreamSynchronize(st));
    if (arcs_out) *arcs_out = arcs;
    /* the auto choice took the dense build on an upper bound of the arcs: confirm it (one rank's
     * rows suffice for the whole graph only when they are all of them; N ranks sum their counts,
     * build_rank) */
    if (c->verify_dense && row0 == 0 && nrows >= c->n) {
        const double n = c->n;
        if (!(c->n <= 2048 || (double)arcs * 16.0 >= n * n)) rc = SRT_FALLBACK_CANON;
    }
out:
    if (st) (void)hipStreamSynchronize(st);
    for (int s = 0; s < 2; s++) {
        if (ev[s]) (void)hipEventDestroy(ev[s]);
        stg_put(slot[s]);
    }
    dfree(&B);
    return rc;
}

/* rows [row0, row0 + nrows) of the ld x ld matrices into dw / dr (row row0 at dw[0]) */
static int dense_upload(const srt_canon* c, int ld, int row0, int nrows, uint32_t* dw, double* dr,
                        hipStream_t st, int sharers, unsigned long long* arcs_out = NULL) {
    if (nrows <= 0) return SRT_OK;
    if (!c->rowptr) return dense_scatter(c, ld, row0, nrows, dw, dr, st, sharers, arcs_out);
    const size_t row_b = (size_t)ld * (sizeof(uint32_t) + sizeof(double));
    const int per = (int)(STG_SLOT / row_b);
    if (per < 1) {
        srt_set_error("dense staging: a row of %d entries passes the %zu-byte slot", ld, STG_SLOT);
        return SRT_E_RANGE;
    }
    void* slot[2] = {stg_get(), stg_get()};
    hipEvent_t ev[2] = {NULL, NULL};
    int rc = SRT_OK;
    const int nt = stg_threads(sharers);
    if (!slot[0] || !slot[1] || hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) != hipSuccess) {
        srt_set_error("dense staging: pinned slots or events unavailable");
        rc = SRT_E_DEVICE;
    }
    for (int k = 0, r = 0; !rc && r < nrows; k++, r += per) {
        const int s = k & 1, rows = nrows - r < per ? nrows - r : per;
        if (k >= 2 && hipEventSynchronize(ev[s]) != hipSuccess) rc = SRT_E_DEVICE;
        if (rc) break;
        fill_ctx f = {c, ld, row0 + r, rows, (uint32_t*)slot[s],
                      (double*)((char*)slot[s] + (size_t)per * ld * sizeof(uint32_t))};
        par_run(nt, fill_part, &f);
        if (hipMemcpyAsync(dw + (size_t)r * ld, f.w, (size_t)rows * ld * sizeof(uint32_t),
                           hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(dr + (size_t)r * ld, f.r, (size_t)rows * ld * sizeof(double),
                           hipMemcpyHostToDevice, st) != hipSuccess ||
            hipEventRecord(ev[s], st) != hipSuccess)
            rc = SRT_E_DEVICE;
    }
    /* the slots go back to the cache only once their copies are done */
    if (hipStreamSynchronize(st) != hipSuccess && !rc) rc = SRT_E_DEVICE;
    if (rc == SRT_E_DEVICE) srt_set_error("dense staging upload failed");
    for (int s = 0; s < 2; s++) {
        if (ev[s]) (void)hipEventDestroy(ev[s]);
        stg_put(slot[s]);
    }
    return rc;
}

/* rows x width bytes from device src (pitch spitch) into host dst (pitch dpitch), after the work
 * already on `st`; returns when dst holds them */
static int table_download(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                          int rows, hipStream_t st, int sharers) {
    if (rows <= 0 || width == 0) return SRT_OK;
    {   /* a page-locked destination (hipHostMalloc / hipHostRegister by the caller): one DMA */
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, dst) == hipSuccess && at.type == hipMemoryTypeHost) {
            if (hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, hipMemcpyDeviceToHost, st) !=
                    hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                srt_set_error("table download to pinned memory failed");
                return SRT_E_DEVICE;
            }
            return SRT_OK;
        }
        (void)hipGetLastError(); /* a pageable pointer is "invalid value" to the query */
    }
    /* a contiguous table is moved as rows of up to 1 MiB */
    int64_t R = rows;
    if (dpitch == width && spitch == width && (size_t)rows * width > STG_SLOT) {
        size_t w = width;
        while (w * 2 <= ((size_t)1 << 20) && (R & 1) == 0) {
            w *= 2;
            R /= 2;
        }
        width = dpitch = spitch = w;
    }
    const int per = (int)(STG_SLOT / width);
    if (per < 1) {
        srt_set_error("table staging: a row of %zu bytes passes the slot", width);
        return SRT_E_RANGE;
    }
    void* slot[2] = {stg_get(), stg_get()};
    hipEvent_t ev[2] = {NULL, NULL};
    int rc = SRT_OK;
    const int nt = stg_threads(sharers);
    if (!slot[0] || !slot[1] || hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) != hipSuccess) {
        srt_set_error("table staging: pinned slots or events unavailable");
        rc = SRT_E_DEVICE;
    }
    int64_t prev_r = -1;
    int prev_rows = 0;
    for (int64_t k = 0, r = 0; !rc; k++) {
        const int s = (int)(k & 1);
        const int rows_k = r < R ? (int)(R - r < per ? R - r : per) : 0;
        if (rows_k > 0 &&
            (hipMemcpy2DAsync(slot[s], width, (const char*)src + (size_t)r * spitch, spitch, width,
                              rows_k, hipMemcpyDeviceToHost, st) != hipSuccess ||
             hipEventRecord(ev[s], st) != hipSuccess)) {
            rc = SRT_E_DEVICE;
            break;
        }
        if (prev_r >= 0) { /* drain the previous chunk while this one moves */
            if (hipEventSynchronize(ev[s ^ 1]) != hipSuccess) {
                rc = SRT_E_DEVICE;
                break;
            }
            drain_ctx d = {(char*)dst + (size_t)prev_r * dpitch, dpitch, width,
                           (const char*)slot[s ^ 1], prev_rows};
            par_run(nt, drain_part, &d);
        }
        prev_r = rows_k > 0 ? r : -1;
        prev_rows = rows_k;
        if (rows_k == 0) break;
        r += rows_k;
    }
    if (hipStreamSynchronize(st) != hipSuccess && !rc) rc = SRT_E_DEVICE;
    if (rc == SRT_E_DEVICE) srt_set_error("table staging download failed");
    for (int s = 0; s < 2; s++) {
        if (ev[s]) (void)hipEventDestroy(ev[s]);
        stg_put(slot[s]);
    }
    return rc;
}

/* the nsub x nsub sub-tables (contiguous on the device) into the caller's buffers */
static int download_sub(int nsub, const uint32_t* slat, const double* srel, const double* sms,
                        uint32_t* lat_q, double* rel, double* lat_ms, hipStream_t st,
                        srt_build_stats* local) {
    SRT_HIPCHK(hipStreamSynchronize(st)); /* the transfer alone is timed */
    const double t0 = host_ms();
    const size_t w4 = (size_t)nsub * sizeof(uint32_t), w8 = (size_t)nsub * sizeof(double);
    int rc = table_download(lat_q, w4, slat, w4, w4, nsub, st, 1);
    if (!rc) rc = table_download(rel, w8, srel, w8, w8, nsub, st, 1);
    if (!rc && sms) rc = table_download(lat_ms, w8, sms, w8, w8, nsub, st, 1);
    local->ms_download = host_ms() - t0;
    return rc;
}

/* one GPU */
static int build_one(const srt_canon* c, const srt_build_opts* opts, int algo, int nsub,
                     const int32_t* verts, uint32_t* lat_q, double* rel, double* lat_ms,
                     uint32_t* min_q, srt_build_stats* stats) {
    const int n = c->n;
    const int use_sp = opts ? opts->use_shortest_path : 1;
    const uint64_t q = c->quantum_ns;
    srt_build_stats local;
    memset(&local, 0, sizeof(local));
    if (stats) {
        local.time_kernels = stats->time_kernels;
        local.count_ties = stats->count_ties;
    }
    dbufs B;
    B.k = 0;
    hipStream_t st = NULL;
    int32_t* dverts = NULL;
    uint32_t* dmin = NULL;
    uint32_t *slat = NULL, *dlat = NULL;
    double *srel = NULL, *sms = NULL, *drel = NULL, *dms = NULL;
    const size_t ns2 = (size_t)nsub * nsub;
    int rc = SRT_OK;
    TRYHIP(hipSetDevice(opts ? opts->device : 0));
    TRYHIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    TRY(dalloc(&B, (void**)&dmin, sizeof(uint32_t)));
    TRYHIP(hipMemsetAsync(dmin, 0xFF, sizeof(uint32_t), st));
    if (verts) {
        TRY(dalloc(&B, (void**)&dverts, (size_t)nsub * sizeof(int32_t)));
        TRYHIP(hipMemcpyAsync(dverts, verts, (size_t)nsub * sizeof(int32_t), hipMemcpyHostToDevice, st));
    }
    if (!use_sp || algo == SRT_ALGO_DENSE_FW) {
        if (n > SRT_DENSE_MAX_N) {
            srt_set_error("dense build supports n <= %d (n = %d); use the sparse SSSP",
                          SRT_DENSE_MAX_N, n);
            rc = SRT_E_RANGE;
            goto out;
        }
        const int ld = srt_ceil_div(n, 128) * 128; /* the u16 FW tiles need ld % 128 == 0 */
        const size_t ll = (size_t)ld * ld;
        uint32_t* dw;
        double* dr;
        TRY(dalloc(&B, (void**)&dw, ll * sizeof(uint32_t)));
        TRY(dalloc(&B, (void**)&dr, ll * sizeof(double)));
        {
            const double t0 = host_ms();
            TRY(dense_upload(c, ld, 0, ld, dw, dr, st, 1));
            local.ms_upload = host_ms() - t0;
        }
        /* a few attached vertices: their rows alone (Bellman-Ford passes, ~6 nsub n^2 work)
         * instead of the all-pairs FW (n^3 / 2), as the reference computes paths from attached
         * sources only (topology.c:1604-1656) */
        int rows_used = 0;
        if (use_sp && verts && (size_t)nsub * 12 <= (size_t)n) {
            uint32_t* rl;
            double *rr, *rm = NULL;
            TRY(dalloc(&B, (void**)&rl, (size_t)nsub * ld * sizeof(uint32_t)));
            TRY(dalloc(&B, (void**)&rr, (size_t)nsub * ld * sizeof(double)));
            if (lat_ms) TRY(dalloc(&B, (void**)&rm, (size_t)nsub * ld * sizeof(double)));
            TRY(srt_dense_rows_build_device(n, ld, nsub, dverts, dw, dr, rl, rr, rm, q, c->directed,
                                            st, &local, &rows_used));
            if (rows_used) {
                TRY(dalloc(&B, (void**)&slat, ns2 * sizeof(uint32_t)));
                TRY(dalloc(&B, (void**)&srel, ns2 * sizeof(double)));
                TRY(srt_gather_sub_u32(nsub, nsub, NULL, dverts, rl, ld, slat, nsub, st));
                TRY(srt_gather_sub_f64(nsub, nsub, NULL, dverts, rr, ld, srel, nsub, st));
                if (rm) {
                    TRY(dalloc(&B, (void**)&sms, ns2 * sizeof(double)));
                    TRY(srt_gather_sub_f64(nsub, nsub, NULL, dverts, rm, ld, sms, nsub, st));
                }
                TRY(srt_table_min(nsub, nsub, slat, nsub, dmin, st));
                TRY(download_sub(nsub, slat, srel, sms, lat_q, rel, lat_ms, st, &local));
                TRYHIP(hipMemcpyAsync(min_q, dmin, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
                TRYHIP(hipStreamSynchronize(st));
            }
        }
        if (!rows_used) {
            TRY(dalloc(&B, (void**)&dlat, ll * sizeof(uint32_t)));
            TRY(dalloc(&B, (void**)&drel, ll * sizeof(double)));
            if (lat_ms) TRY(dalloc(&B, (void**)&dms, ll * sizeof(double)));
        }
        if (rows_used) {
            /* done: the attached rows */
        } else if (use_sp) {
            TRY(srt_dense_build_device_ms(n, ld, c->directed, dw, dr, dlat, drel, dms, q, st,
                                          opts ? opts->fw_block : 0, &local));
        } else {
            /* direct mode (topology.c:1816-1858): the (complete) graph's own edges, the self-loop
             * on the diagonal */
            TRYHIP(hipMemcpyAsync(dlat, dw, ll * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
            TRYHIP(hipMemcpyAsync(drel, dr, ll * sizeof(double), hipMemcpyDeviceToDevice, st));
            if (dms) TRY(srt_quanta_to_ms(n, n, dw, ld, q, dms, ld, st));
            local.algo = SRT_ALGO_DENSE_FW;
        }
        if (rows_used) {
        } else if (verts) {
            TRY(dalloc(&B, (void**)&slat, ns2 * sizeof(uint32_t)));
            TRY(dalloc(&B, (void**)&srel, ns2 * sizeof(double)));
            TRY(srt_gather_sub_u32(nsub, nsub, dverts, dverts, dlat, ld, slat, nsub, st));
            TRY(srt_gather_sub_f64(nsub, nsub, dverts, dverts, drel, ld, srel, nsub, st));
            if (dms) {
                TRY(dalloc(&B, (void**)&sms, ns2 * sizeof(double)));
                TRY(srt_gather_sub_f64(nsub, nsub, dverts, dverts, dms, ld, sms, nsub, st));
            }
            TRY(srt_table_min(nsub, nsub, slat, nsub, dmin, st));
            TRY(download_sub(nsub, slat, srel, sms, lat_q, rel, lat_ms, st, &local));
        } else {
            TRY(srt_table_min(n, n, dlat, ld, dmin, st));
            TRYHIP(hipStreamSynchronize(st)); /* the transfer alone is timed */
            const double t0 = host_ms();
            TRY(table_download(lat_q, (size_t)n * sizeof(uint32_t), dlat, (size_t)ld * sizeof(uint32_t),
                               (size_t)n * sizeof(uint32_t), n, st, 1));
            TRY(table_download(rel, (size_t)n * sizeof(double), drel, (size_t)ld * sizeof(double),
                               (size_t)n * sizeof(double), n, st, 1));
            if (dms)
                TRY(table_download(lat_ms, (size_t)n * sizeof(double), dms, (size_t)ld * sizeof(double),
                                   (size_t)n * sizeof(double), n, st, 1));
            local.ms_download = host_ms() - t0;
        }
        if (!rows_used) {
            TRYHIP(hipMemcpyAsync(min_q, dmin, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
            TRYHIP(hipStreamSynchronize(st));
        }
        if (!use_sp) {
            for (size_t i = 0; i < ns2; i++)
                if (lat_q[i] >= SRT_INF) {
                    srt_set_error("use_shortest_path=false requires a complete graph");
                    rc = SRT_E_INVALID;
                    goto out;
                }
        }
    } else {
        srt_sparse_graph* sg = NULL;
        TRY(sparse_graph_from_canon(c, opts ? opts->device : 0, &sg));
        /* the sub-table (every source row of the subset, its columns) on the device; the
         * full-width rows of a chunk of sources are gathered into it */
        const size_t per_row = (size_t)n * (sizeof(uint32_t) + sizeof(double) + (lat_ms ? sizeof(double) : 0));
        rc = dalloc(&B, (void**)&slat, ns2 * sizeof(uint32_t));
        if (!rc) rc = dalloc(&B, (void**)&srel, ns2 * sizeof(double));
        if (!rc && lat_ms) rc = dalloc(&B, (void**)&sms, ns2 * sizeof(double));
        int chunk = nsub;
        if (!rc && verts) {
            const size_t cb = chunk_budget(0, 1) / per_row;
            chunk = (int)(cb < (size_t)nsub ? (cb > 0 ? cb : 1) : (size_t)nsub);
            rc = dalloc(&B, (void**)&dlat, (size_t)chunk * n * sizeof(uint32_t));
            if (!rc) rc = dalloc(&B, (void**)&drel, (size_t)chunk * n * sizeof(double));
            if (!rc && lat_ms) rc = dalloc(&B, (void**)&dms, (size_t)chunk * n * sizeof(double));
        }
        for (int r0 = 0; r0 < nsub && !rc; r0 += chunk) {
            const int r1 = r0 + chunk < nsub ? r0 + chunk : nsub;
            srt_build_stats cs;
            memset(&cs, 0, sizeof(cs));
            cs.count_ties = local.count_ties;
            if (verts) {
                rc = sparse_rows(sg, 0, r1 - r0, dverts + r0, dlat, drel, dms, st, &cs);
                if (!rc) rc = srt_gather_sub_u32(r1 - r0, nsub, NULL, dverts, dlat, n, slat + (size_t)r0 * nsub, nsub, st);
                if (!rc) rc = srt_gather_sub_f64(r1 - r0, nsub, NULL, dverts, drel, n, srel + (size_t)r0 * nsub, nsub, st);
                if (!rc && dms) rc = srt_gather_sub_f64(r1 - r0, nsub, NULL, dverts, dms, n, sms + (size_t)r0 * nsub, nsub, st);
            } else {
                rc = sparse_rows(sg, r0, r1, NULL, slat + (size_t)r0 * n, srel + (size_t)r0 * n,
                                 sms ? sms + (size_t)r0 * n : NULL, st, &cs);
            }
            merge_stats(&local, &cs, r0 == 0);
        }
        if (!rc) rc = srt_table_min(nsub, nsub, slat, nsub, dmin, st);
        srt_sparse_graph_free(sg);
        if (rc) goto out;
        TRY(download_sub(nsub, slat, srel, sms, lat_q, rel, lat_ms, st, &local));
        TRYHIP(hipMemcpyAsync(min_q, dmin, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        TRYHIP(hipStreamSynchronize(st));
    }
    if (stats) *stats = local;
out:
    if (st) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
    }
    dfree(&B);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* In-process multi-GPU build (Shadow is one process): one host thread per GPU, RCCL           */
/* communicators from ncclCommInitAll, the same sharded kernels as the one-process-per-GPU     */
/* path (dense: row shards + pivot-panel broadcast; sparse: source shards + all-gather).       */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int state; /* 0 wait, 1 go, -1 abort */
} start_gate;

typedef struct {
    int rank, R, dev, directed, algo, n, ld;
    int virt; /* virtual ranks on one device: per-rank state slots */
    start_gate* gate;
    srt_comm* comm;
    const srt_canon* c;
    int nsub;
    const int32_t* verts; /* host subset (NULL: all vertices) */
    uint32_t* lat_q;      /* host outputs, nsub x nsub */
    double* rel;
    double* lat_ms;
    uint32_t min_q;
    int rc;
    char err[256];
    srt_build_stats st;
} mjob;

static void mjob_fail(mjob* j, int rc) {
    j->rc = rc;
    snprintf(j->err, sizeof(j->err), "%s", srt_last_error());
}

/* every rank thread starts only once all R exist: a rank that never started cannot leave the
 * others waiting in a collective */
static int gate_wait(start_gate* g) {
    pthread_mutex_lock(&g->mu);
    while (g->state == 0) pthread_cond_wait(&g->cv, &g->mu);
    const int s = g->state;
    pthread_mutex_unlock(&g->mu);
    return s;
}

static void* mjob_dense(void* p) {
    mjob* j = (mjob*)p;
    if (gate_wait(j->gate) < 0) return NULL;
    int rc = SRT_OK;
    dbufs B;
    B.k = 0;
    hipStream_t st = NULL;
    int32_t b, e;
    srt_shard_rows(j->ld, SRT_SHARD_ALIGN, j->R, j->rank, &b, &e);
    const int nr = e - b, n = j->n, nsub = j->nsub;
    const size_t rows = (size_t)(nr > 0 ? nr : 1) * j->ld;
    uint32_t *dw, *dlat, *dmin;
    double *dr, *drel, *dms = NULL;
    srt_set_virtual_slot(j->virt ? j->rank : -1);
    TRYHIP(hipSetDevice(j->dev));
    TRYHIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    TRY(dalloc(&B, (void**)&dw, rows * sizeof(uint32_t)));
    TRY(dalloc(&B, (void**)&dr, rows * sizeof(double)));
    TRY(dalloc(&B, (void**)&dlat, rows * sizeof(uint32_t)));
    TRY(dalloc(&B, (void**)&drel, rows * sizeof(double)));
    TRY(dalloc(&B, (void**)&dmin, sizeof(uint32_t)));
    if (j->lat_ms) TRY(dalloc(&B, (void**)&dms, rows * sizeof(double)));
    TRYHIP(hipMemsetAsync(dmin, 0xFF, sizeof(uint32_t), st));
    {
        const double t0 = host_ms();
        unsigned long long arcs = 0;
        TRY(dense_upload(j->c, j->ld, b, nr, dw, dr, st, j->R, &arcs));
        j->st.ms_upload = host_ms() - t0;
        /* the edge form's dense choice rests on an upper bound of the arcs (parallel edges count
         * once per edge): the ranks sum their exact counts (three 24-bit limbs: an int32 sum of up
         * to 64 ranks cannot overflow) and every rank takes the same verdict, falling back to the
         * host canonical form together when the graph is not dense-shaped after all */
        if (j->R > 1 && j->c->verify_dense && !j->c->rowptr) {
            int32_t h[3] = {(int32_t)(arcs & 0xFFFFFF), (int32_t)((arcs >> 24) & 0xFFFFFF), (int32_t)(arcs >> 48)};
            int32_t* dcount;
            TRY(dalloc(&B, (void**)&dcount, sizeof(h)));
            TRYHIP(hipMemcpyAsync(dcount, h, sizeof(h), hipMemcpyHostToDevice, st));
            TRY(srt_coll_allreduce_i32(j->comm, dcount, 3, 0, st));
            TRYHIP(hipMemcpyAsync(h, dcount, sizeof(h), hipMemcpyDeviceToHost, st));
            TRYHIP(hipStreamSynchronize(st));
            const double total = (double)h[0] + (double)h[1] * 16777216.0 + (double)h[2] * 281474976710656.0;
            const double nn = (double)n * (double)n;
            if (!(n <= 2048 || total * 16.0 >= nn)) {
                rc = SRT_FALLBACK_CANON;
                goto out;
            }
        }
    }
    TRY(srt_dense_build_sharded_ms(j->comm, n, j->ld, j->directed, dw, dr, dlat, drel, dms,
                                   j->c->quantum_ns, st, 0, &j->st));
    {
        /* this rank's rows of the (sub-)table: slots whose vertex lies in [b, min(e, n)) */
        const int r1 = e < n ? e : n;
        int i0 = 0, i1 = 0;
        if (j->verts) {
            while (i0 < nsub && j->verts[i0] < b) i0++;
            i1 = i0;
            while (i1 < nsub && j->verts[i1] < r1) i1++;
        } else {
            i0 = b < n ? b : n;
            i1 = r1 > i0 ? r1 : i0;
        }
        const int cnt = i1 - i0;
        if (cnt > 0 && j->verts) {
            int32_t* hrows = (int32_t*)malloc((size_t)cnt * sizeof(int32_t));
            if (!hrows) {
                rc = SRT_E_NOMEM;
                goto out;
            }
            for (int i = 0; i < cnt; i++) hrows[i] = j->verts[i0 + i] - b;
            int32_t *drows, *dcols;
            uint32_t* sl;
            double *sr, *sm = NULL;
            rc = dalloc(&B, (void**)&drows, (size_t)cnt * sizeof(int32_t));
            if (!rc) rc = dalloc(&B, (void**)&dcols, (size_t)nsub * sizeof(int32_t));
            if (!rc && hipMemcpyAsync(drows, hrows, (size_t)cnt * sizeof(int32_t), hipMemcpyHostToDevice, st) != hipSuccess)
                rc = SRT_E_DEVICE;
            if (!rc && hipMemcpyAsync(dcols, j->verts, (size_t)nsub * sizeof(int32_t), hipMemcpyHostToDevice, st) != hipSuccess)
                rc = SRT_E_DEVICE;
            if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = SRT_E_DEVICE;
            free(hrows);
            if (rc) goto out;
            TRY(dalloc(&B, (void**)&sl, (size_t)cnt * nsub * sizeof(uint32_t)));
            TRY(dalloc(&B, (void**)&sr, (size_t)cnt * nsub * sizeof(double)));
            TRY(srt_gather_sub_u32(cnt, nsub, drows, dcols, dlat, j->ld, sl, nsub, st));
            TRY(srt_gather_sub_f64(cnt, nsub, drows, dcols, drel, j->ld, sr, nsub, st));
            if (dms) {
                TRY(dalloc(&B, (void**)&sm, (size_t)cnt * nsub * sizeof(double)));
                TRY(srt_gather_sub_f64(cnt, nsub, drows, dcols, dms, j->ld, sm, nsub, st));
            }
            TRY(srt_table_min(cnt, nsub, sl, nsub, dmin, st));
            const double t0 = host_ms();
            const size_t w4 = (size_t)nsub * sizeof(uint32_t), w8 = (size_t)nsub * sizeof(double);
            TRY(table_download(j->lat_q + (size_t)i0 * nsub, w4, sl, w4, w4, cnt, st, j->R));
            TRY(table_download(j->rel + (size_t)i0 * nsub, w8, sr, w8, w8, cnt, st, j->R));
            if (sm) TRY(table_download(j->lat_ms + (size_t)i0 * nsub, w8, sm, w8, w8, cnt, st, j->R));
            j->st.ms_download = host_ms() - t0;
        } else if (cnt > 0) {
            TRY(srt_table_min(cnt, n, dlat, j->ld, dmin, st));
            const double t0 = host_ms();
            const size_t w4 = (size_t)n * sizeof(uint32_t), w8 = (size_t)n * sizeof(double);
            TRY(table_download(j->lat_q + (size_t)i0 * n, w4, dlat, (size_t)j->ld * sizeof(uint32_t), w4,
                               cnt, st, j->R));
            TRY(table_download(j->rel + (size_t)i0 * n, w8, drel, (size_t)j->ld * sizeof(double), w8, cnt,
                               st, j->R));
            if (dms)
                TRY(table_download(j->lat_ms + (size_t)i0 * n, w8, dms, (size_t)j->ld * sizeof(double), w8,
                                   cnt, st, j->R));
            j->st.ms_download = host_ms() - t0;
        }
        TRYHIP(hipMemcpyAsync(&j->min_q, dmin, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
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
    if (gate_wait(j->gate) < 0) return NULL;
    int rc = SRT_OK;
    dbufs B;
    B.k = 0;
    hipStream_t st = NULL;
    srt_sparse_graph* sg = NULL;
    const int n = j->n, nsub = j->nsub, per = srt_ceil_div(nsub, j->R);
    const int s0 = j->rank * per < nsub ? j->rank * per : nsub;
    const int s1 = (s0 + per < nsub) ? s0 + per : nsub;
    /* this rank's source rows only: every row is its own source's (no mirror), and the host
     * table the ranks of this process share receives each shard directly */
    const size_t all = (size_t)(s1 > s0 ? s1 - s0 : 1) * nsub;
    uint32_t *slat, *dlat = NULL, *dmin;
    double *srel, *sms = NULL, *drel = NULL, *dms = NULL;
    int32_t* dverts = NULL;
    int chunk = s1 - s0;
    srt_set_virtual_slot(j->virt ? j->rank : -1);
    TRYHIP(hipSetDevice(j->dev));
    TRYHIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    TRY(sparse_graph_from_canon(j->c, j->dev, &sg));
    TRY(dalloc(&B, (void**)&slat, all * sizeof(uint32_t)));
    TRY(dalloc(&B, (void**)&srel, all * sizeof(double)));
    TRY(dalloc(&B, (void**)&dmin, sizeof(uint32_t)));
    if (j->lat_ms) TRY(dalloc(&B, (void**)&sms, all * sizeof(double)));
    TRYHIP(hipMemsetAsync(dmin, 0xFF, sizeof(uint32_t), st));
    if (j->verts && s1 > s0) {
        const size_t per_row = (size_t)n * (sizeof(uint32_t) + sizeof(double) + (sms ? sizeof(double) : 0));
        const size_t cb = chunk_budget(0, j->virt ? j->R : 1) / per_row;
        chunk = (int)(cb < (size_t)(s1 - s0) ? (cb > 0 ? cb : 1) : (size_t)(s1 - s0));
        TRY(dalloc(&B, (void**)&dverts, (size_t)nsub * sizeof(int32_t)));
        TRYHIP(hipMemcpyAsync(dverts, j->verts, (size_t)nsub * sizeof(int32_t), hipMemcpyHostToDevice, st));
        TRY(dalloc(&B, (void**)&dlat, (size_t)chunk * n * sizeof(uint32_t)));
        TRY(dalloc(&B, (void**)&drel, (size_t)chunk * n * sizeof(double)));
        if (sms) TRY(dalloc(&B, (void**)&dms, (size_t)chunk * n * sizeof(double)));
    }
    for (int r0 = s0; r0 < s1; r0 += chunk) {
        const int r1 = r0 + chunk < s1 ? r0 + chunk : s1;
        srt_build_stats cs;
        memset(&cs, 0, sizeof(cs));
        cs.count_ties = j->st.count_ties;
        if (j->verts) {
            const size_t o = (size_t)(r0 - s0) * nsub;
            TRY(sparse_rows(sg, 0, r1 - r0, dverts + r0, dlat, drel, dms, st, &cs));
            TRY(srt_gather_sub_u32(r1 - r0, nsub, NULL, dverts, dlat, n, slat + o, nsub, st));
            TRY(srt_gather_sub_f64(r1 - r0, nsub, NULL, dverts, drel, n, srel + o, nsub, st));
            if (dms) TRY(srt_gather_sub_f64(r1 - r0, nsub, NULL, dverts, dms, n, sms + o, nsub, st));
        } else {
            const size_t o = (size_t)(r0 - s0) * n;
            TRY(sparse_rows(sg, r0, r1, NULL, slat + o, srel + o, sms ? sms + o : NULL, st, &cs));
        }
        merge_stats(&j->st, &cs, r0 == s0);
    }
    if (s1 > s0) {
        TRY(srt_table_min(s1 - s0, nsub, slat, nsub, dmin, st));
        TRYHIP(hipMemcpyAsync(j->lat_q + (size_t)s0 * nsub, slat,
                              (size_t)(s1 - s0) * nsub * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        TRYHIP(hipMemcpyAsync(j->rel + (size_t)s0 * nsub, srel,
                              (size_t)(s1 - s0) * nsub * sizeof(double), hipMemcpyDeviceToHost, st));
        if (sms)
            TRYHIP(hipMemcpyAsync(j->lat_ms + (size_t)s0 * nsub, sms,
                                  (size_t)(s1 - s0) * nsub * sizeof(double), hipMemcpyDeviceToHost, st));
    }
    TRYHIP(hipMemcpyAsync(&j->min_q, dmin, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    TRYHIP(hipStreamSynchronize(st));
out:
    if (rc) mjob_fail(j, rc);
    if (sg) srt_sparse_graph_free(sg);
    if (st) (void)hipStreamDestroy(st);
    dfree(&B);
    return NULL;
}

static int build_multi(const srt_canon* c, const srt_build_opts* opts, int algo, int R, int virt,
                       int nsub, const int32_t* verts, uint32_t* lat_q, double* rel,
                       double* lat_ms, uint32_t* min_q, srt_build_stats* stats) {
    const int n = c->n;
    const int ld = srt_ceil_div(n, SRT_SHARD_ALIGN) * SRT_SHARD_ALIGN;
    int rc = SRT_OK;
    start_gate gate;
    pthread_mutex_init(&gate.mu, NULL);
    pthread_cond_init(&gate.cv, NULL);
    gate.state = 0;
    int started = 0;
    srt_comm** comms = (srt_comm**)calloc((size_t)R, sizeof(srt_comm*));
    mjob* jobs = (mjob*)calloc((size_t)R, sizeof(mjob));
    pthread_t* th = (pthread_t*)calloc((size_t)R, sizeof(pthread_t));
    int* devs = (int*)calloc((size_t)R, sizeof(int));
    if (!comms || !jobs || !th || !devs) {
        rc = SRT_E_NOMEM;
        goto done;
    }
    if (algo == SRT_ALGO_DENSE_FW) {
        if (n > SRT_DENSE_MAX_N) {
            srt_set_error("dense build supports n <= %d (n = %d); use the sparse SSSP",
                          SRT_DENSE_MAX_N, n);
            rc = SRT_E_RANGE;
            goto done;
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
        j->directed = c->directed;
        j->algo = algo;
        j->n = n;
        j->ld = ld;
        j->gate = &gate;
        j->comm = comms[i];
        j->c = c;
        j->nsub = nsub;
        j->verts = verts;
        j->lat_q = lat_q;
        j->rel = rel;
        j->lat_ms = lat_ms;
        j->min_q = 0xFFFFFFFFu;
        if (stats) {
            j->st.count_ties = stats->count_ties;
            j->st.time_kernels = stats->time_kernels;
        }
        if (pthread_create(&th[i], NULL, algo == SRT_ALGO_DENSE_FW ? mjob_dense : mjob_sparse, j)) {
            rc = SRT_E_NOMEM;
            srt_set_error("srt_build_tables_multi: pthread_create failed for rank %d", i);
            break;
        }
        started++;
    }
    /* open the gate only when every rank exists; otherwise the started ones leave at once */
    pthread_mutex_lock(&gate.mu);
    gate.state = rc ? -1 : 1;
    pthread_cond_broadcast(&gate.cv);
    pthread_mutex_unlock(&gate.mu);
    for (int i = 0; i < started; i++) pthread_join(th[i], NULL);
    if (rc) goto done;
    for (int i = 0; i < R && !rc; i++)
        if (jobs[i].rc) {
            rc = jobs[i].rc;
            srt_set_error("rank %d: %s", i, jobs[i].err);
        }
    if (!rc) {
        uint32_t m = 0xFFFFFFFFu;
        for (int i = 0; i < R; i++) m = jobs[i].min_q < m ? jobs[i].min_q : m;
        *min_q = m;
        if (stats) {
            *stats = jobs[0].st;
            for (int i = 1; i < R; i++) {
                stats->tied_pairs += jobs[i].st.tied_pairs;
                if (jobs[i].st.ms_upload > stats->ms_upload) stats->ms_upload = jobs[i].st.ms_upload;
                if (jobs[i].st.ms_download > stats->ms_download)
                    stats->ms_download = jobs[i].st.ms_download;
            }
        }
    }
done:
    if (comms)
        for (int i = 0; i < R; i++)
            if (comms[i]) srt_comm_free(comms[i]);
    pthread_mutex_destroy(&gate.mu);
    pthread_cond_destroy(&gate.cv);
    free(comms);
    free(jobs);
    free(th);
    free(devs);
    return rc;
}

/* SRT_VIRTUAL_RANKS=R (tests): R ranks on device 0, collectives as device copies */
static int virtual_ranks_env(void) {
    const char* venv = getenv("SRT_VIRTUAL_RANKS");
    const int v = venv ? atoi(venv) : 0;
    return v > 0 ? (v < 64 ? v : 64) : 0;
}

static int build_tables_subset_impl(const srt_edges* g, const srt_build_opts* opts, int32_t ngpus,
                                    int virt, int32_t nsub, const int32_t* verts, uint32_t* lat_q,
                                    uint64_t* quantum_ns, double* rel, double* lat_ms,
                                    uint32_t* min_lat_q, srt_build_stats* stats) {
    if (!g || !lat_q || !quantum_ns || !rel || ngpus < 1) {
        srt_set_error("srt_build_tables_subset: null argument");
        return SRT_E_ARG;
    }
    if (check_verts(g->n, nsub, verts)) {
        srt_set_error("srt_build_tables_subset: the subset must be 1..n strictly increasing vertex "
                      "indices (or NULL with nsub = n)");
        return SRT_E_ARG;
    }
    const int avail = srt_device_count();
    if (avail < 1) {
        srt_set_error("srt_build_tables: no HIP device");
        return SRT_E_DEVICE;
    }
    const int use_sp = opts ? opts->use_shortest_path : 1;
    const int forced = opts ? opts->algo : SRT_ALGO_AUTO;
    /* a dense-shaped graph (by its edge count, an upper bound on its arcs) goes to the device as
     * its edge list; every other graph, and one the edge form refuses, through the host canonical
     * CSR (graph.c). The dense auto choice is confirmed on the exact arcs by a one-rank scatter. */
    int edge_form = 0;
    if (forced != SRT_ALGO_SPARSE_SSSP && g->n <= SRT_DENSE_MAX_N && g->m > 0) {
        const double n = g->n, ub = (double)g->m * (g->directed ? 1 : 2);
        edge_form = g->n <= 2048 || ub * 16.0 >= n * n || forced == SRT_ALGO_DENSE_FW || !use_sp;
    }
    int rc = SRT_OK;
    for (int attempt = 0; attempt < 2; attempt++) {
        srt_canon c;
        const double t0 = host_ms();
        if (edge_form && attempt == 0 && canon_from_edges(g, &c) == 0) {
            c.verify_dense = use_sp && forced != SRT_ALGO_DENSE_FW;
        } else {
            if (attempt == 0) edge_form = 0;
            rc = srt_canon_build(g, &c);
            if (rc) return rc;
        }
        const double ms_canon = host_ms() - t0;
        *quantum_ns = c.quantum_ns;
        const int algo = use_sp ? (c.wide && forced != SRT_ALGO_DENSE_FW ? SRT_ALGO_SPARSE_SSSP
                                                                          : choose_algo(&c, opts))
                                : SRT_ALGO_DENSE_FW;
        if (use_sp && c.wide && (algo == SRT_ALGO_DENSE_FW || !lat_ms)) {
            srt_set_error("shortest-path latencies may pass the u32 range (bound %llu quanta of %llu "
                          "ns): only the sparse u64 rows build this graph, and its latencies are "
                          "served from the f64 ms table (%s)",
                          (unsigned long long)c.dist_bound, (unsigned long long)c.quantum_ns,
                          algo == SRT_ALGO_DENSE_FW ? "dense requested" : "no lat_ms output");
            srt_canon_free(&c);
            return SRT_E_RANGE;
        }
        const int R = virt ? virt : (ngpus < avail ? ngpus : avail);
        uint32_t mq = 0xFFFFFFFFu;
        if (R > 1 && use_sp)
            rc = build_multi(&c, opts, algo, R, virt, nsub, verts, lat_q, rel, lat_ms, &mq, stats);
        else
            rc = build_one(&c, opts, algo, nsub, verts, lat_q, rel, lat_ms, &mq, stats);
        if (!rc && min_lat_q) *min_lat_q = mq;
        if (!rc && stats) stats->ms_canon = ms_canon;
        srt_canon_free(&c);
        if (rc != SRT_FALLBACK_CANON) break;
        srt_log(SRT_LOG_INFO, "edge-list dense build: too few distinct arcs, the host canonical form decides");
    }
    return rc;
}

/* SRT_VIRTUAL_RANKS applies only to a multi-GPU request (ngpus > 1): a variable left set must not
 * turn the one-GPU builds (every lazy topology build) into the virtual multi-rank path */
extern "C" int srt_build_tables_subset(const srt_edges* g, const srt_build_opts* opts, int32_t ngpus,
                                       int32_t nsub, const int32_t* verts, uint32_t* lat_q,
                                       uint64_t* quantum_ns, double* rel, double* lat_ms,
                                       uint32_t* min_lat_q, srt_build_stats* stats) {
    return build_tables_subset_impl(g, opts, ngpus, ngpus > 1 ? virtual_ranks_env() : 0, nsub,
                                    verts, lat_q, quantum_ns, rel, lat_ms, min_lat_q, stats);
}

extern "C" int srt_build_tables(const srt_edges* g, const srt_build_opts* opts, uint32_t* lat_q,
                                uint64_t* quantum_ns, double* rel, srt_build_stats* stats) {
    if (!g) {
        srt_set_error("srt_build_tables: null argument");
        return SRT_E_ARG;
    }
    return srt_build_tables_subset(g, opts, 1, g->n, NULL, lat_q, quantum_ns, rel, NULL, NULL, stats);
}

extern "C" int srt_build_tables_multi(const srt_edges* g, const srt_build_opts* opts, int32_t ngpus,
                                      uint32_t* lat_q, uint64_t* quantum_ns, double* rel,
                                      srt_build_stats* stats) {
    if (!g || ngpus < 1) {
        srt_set_error("srt_build_tables_multi: bad argument");
        return SRT_E_ARG;
    }
    /* ngpus == 1 still runs the threaded, communicator-driven form (tests of that path);
     * SRT_VIRTUAL_RANKS (tests) runs that many virtual ranks on device 0 */
    const int avail = srt_device_count();
    const int virt = virtual_ranks_env();
    if (ngpus == 1 && !virt && avail >= 1) {
        srt_canon c;
        int rc = srt_canon_build(g, &c);
        if (rc) return rc;
        *quantum_ns = c.quantum_ns;
        const int use_sp = opts ? opts->use_shortest_path : 1;
        uint32_t mq;
        if (!use_sp)
            rc = build_one(&c, opts, SRT_ALGO_DENSE_FW, g->n, NULL, lat_q, rel, NULL, &mq, stats);
        else
            rc = build_multi(&c, opts, choose_algo(&c, opts), 1, 0, g->n, NULL, lat_q, rel, NULL,
                             &mq, stats);
        srt_canon_free(&c);
        return rc;
    }
    return build_tables_subset_impl(g, opts, ngpus, virt, g->n, NULL, lat_q, quantum_ns, rel, NULL,
                                    NULL, stats);
}
