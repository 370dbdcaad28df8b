/*
 * oracle.c -- TEST INFRASTRUCTURE ONLY. CPU restatement of Shadow's routing precomputation
 * (/root/reference/src/main/routing/topology.c); see oracle.h for the line map and rules.
 * This file is the parity checker and the CPU baseline; it is never part of the product path.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---------------------------------------------------------------------------------------------
 * Canonical arcs: one per ordered vertex pair (u != v), the (min latency, lowest index) edge.
 * Undirected edges give both directions (igraph IGRAPH_OUT on an undirected graph = ALL).
 * ------------------------------------------------------------------------------------------- */
typedef struct {
    int32_t n;
    int32_t* rowptr; /* n+1 */
    int32_t* col;    /* arcs */
    int64_t* eidx;   /* canonical edge index of the arc */
} orc_csr;

typedef struct {
    int32_t u, v;
    int64_t lat, e;
} arc_t;

static int arc_cmp(const void* a, const void* b) {
    const arc_t* x = (const arc_t*)a;
    const arc_t* y = (const arc_t*)b;
    if (x->u != y->u) return x->u < y->u ? -1 : 1;
    if (x->v != y->v) return x->v < y->v ? -1 : 1;
    if (x->lat != y->lat) return x->lat < y->lat ? -1 : 1;
    if (x->e != y->e) return x->e < y->e ? -1 : 1;
    return 0;
}

static int build_csr(const orc_graph* g, orc_csr* c) {
    int64_t cap = g->directed ? g->m : 2 * g->m;
    arc_t* a = (arc_t*)malloc((size_t)(cap > 0 ? cap : 1) * sizeof(arc_t));
    if (!a) return -1;
    int64_t k = 0;
    for (int64_t e = 0; e < g->m; e++) {
        int32_t u = g->src[e], v = g->dst[e];
        if (u == v) continue; /* self-loops never shorten a path; used only by the self rule */
        a[k++] = (arc_t){u, v, g->lat_ns[e], e};
        if (!g->directed) a[k++] = (arc_t){v, u, g->lat_ns[e], e};
    }
    qsort(a, (size_t)k, sizeof(arc_t), arc_cmp);
    c->n = g->n;
    c->rowptr = (int32_t*)calloc((size_t)g->n + 1, sizeof(int32_t));
    c->col = (int32_t*)malloc((size_t)(k > 0 ? k : 1) * sizeof(int32_t));
    c->eidx = (int64_t*)malloc((size_t)(k > 0 ? k : 1) * sizeof(int64_t));
    if (!c->rowptr || !c->col || !c->eidx) {
        free(a);
        return -1;
    }
    int64_t w = 0;
    for (int64_t i = 0; i < k; i++) {
        if (i > 0 && a[i].u == a[i - 1].u && a[i].v == a[i - 1].v) continue; /* parallel edge */
        c->col[w] = a[i].v;
        c->eidx[w] = a[i].e;
        c->rowptr[a[i].u + 1]++;
        w++;
    }
    for (int32_t i = 0; i < g->n; i++) c->rowptr[i + 1] += c->rowptr[i];
    free(a);
    return 0;
}

static void free_csr(orc_csr* c) {
    free(c->rowptr);
    free(c->col);
    free(c->eidx);
}

/* ---------------------------------------------------------------------------------------------
 * Binary heap keyed by (distance, vertex index): pop order of Dijkstra with the canonical tie
 * rule. Lazy deletion (stale entries skipped on pop).
 * ------------------------------------------------------------------------------------------- */
typedef struct {
    double kd;   /* f64 key (mode F64) */
    uint64_t ki; /* integer key (mode INT) */
    int32_t v;
} hent;

typedef struct {
    hent* h;
    int64_t size, cap;
    int mode;
} heap_t;

static inline int hless(const heap_t* H, const hent* a, const hent* b) {
    if (H->mode == ORC_F64_MS) {
        if (a->kd != b->kd) return a->kd < b->kd;
    } else {
        if (a->ki != b->ki) return a->ki < b->ki;
    }
    return a->v < b->v;
}

static int hpush(heap_t* H, hent x) {
    if (H->size == H->cap) {
        int64_t nc = H->cap ? 2 * H->cap : 1024;
        hent* nh = (hent*)realloc(H->h, (size_t)nc * sizeof(hent));
        if (!nh) return -1;
        H->h = nh;
        H->cap = nc;
    }
    int64_t i = H->size++;
    H->h[i] = x;
    while (i > 0) {
        int64_t p = (i - 1) / 2;
        if (!hless(H, &H->h[i], &H->h[p])) break;
        hent t = H->h[i];
        H->h[i] = H->h[p];
        H->h[p] = t;
        i = p;
    }
    return 0;
}

static hent hpop(heap_t* H) {
    hent top = H->h[0];
    H->h[0] = H->h[--H->size];
    int64_t i = 0;
    for (;;) {
        int64_t l = 2 * i + 1, r = l + 1, b = i;
        if (l < H->size && hless(H, &H->h[l], &H->h[b])) b = l;
        if (r < H->size && hless(H, &H->h[r], &H->h[b])) b = r;
        if (b == i) break;
        hent t = H->h[i];
        H->h[i] = H->h[b];
        H->h[b] = t;
        i = b;
    }
    return top;
}

/* ceil(ms * SIMTIME_ONE_MILLISECOND) as worker.c:551 */
static inline uint64_t ms_to_ns_ref(double ms) { return (uint64_t)ceil(ms * 1000000.0); }
/* (gdouble)timeNanoSec / 1000000.0 as topology.c:294 */
static inline double ns_to_ms(int64_t ns) { return (double)ns / 1000000.0; }

/* One source. Settles vertices in (dist, index) order; when v is settled its predecessor is
 * final, so the path-order accumulations (topology.c:1342-1374) are done by DP over settle order. */
static int sssp_one(const orc_graph* g, const orc_csr* c, int mode, int32_t s, heap_t* H,
                    uint64_t* di, double* dd, char* settled, uint64_t* lat_int, double* rel,
                    double* lms, int32_t* pred) {
    const int32_t n = g->n;
    for (int32_t v = 0; v < n; v++) {
        di[v] = UINT64_MAX;
        dd[v] = INFINITY;
        settled[v] = 0;
        pred[v] = -1;
    }
    di[s] = 0;
    dd[s] = 0.0;
    H->size = 0;
    H->mode = mode;
    if (hpush(H, (hent){0.0, 0, s})) return -1;
    lat_int[s] = 0;
    lms[s] = 0.0;
    rel[s] = 1.0;
    while (H->size > 0) {
        hent x = hpop(H);
        int32_t u = x.v;
        if (settled[u]) continue;
        if (mode == ORC_F64_MS ? (x.kd != dd[u]) : (x.ki != di[u])) continue;
        settled[u] = 1;
        if (u != s) {
            int32_t p = pred[u];
            int64_t e = -1;
            for (int32_t k = c->rowptr[p]; k < c->rowptr[p + 1]; k++)
                if (c->col[k] == u) {
                    e = c->eidx[k];
                    break;
                }
            /* topology.c:1364-1365: totalLatency += edgeLatency; totalReliability *= edgeRel */
            lat_int[u] = lat_int[p] + (uint64_t)g->lat_ns[e];
            lms[u] = lms[p] + ns_to_ms(g->lat_ns[e]);
            rel[u] = rel[p] * (1.0 - g->loss[e]);
        }
        for (int32_t k = c->rowptr[u]; k < c->rowptr[u + 1]; k++) {
            int32_t v = c->col[k];
            if (settled[v]) continue;
            int64_t e = c->eidx[k];
            if (mode == ORC_F64_MS) {
                double nd = dd[u] + ns_to_ms(g->lat_ns[e]);
                if (nd < dd[v]) { /* strict: first settled tight predecessor wins */
                    dd[v] = nd;
                    pred[v] = u;
                    if (hpush(H, (hent){nd, 0, v})) return -1;
                }
            } else {
                uint64_t nd = di[u] + (uint64_t)g->lat_ns[e];
                if (nd < di[v]) {
                    di[v] = nd;
                    pred[v] = u;
                    if (hpush(H, (hent){0.0, nd, v})) return -1;
                }
            }
        }
    }
    for (int32_t v = 0; v < n; v++) {
        if (!settled[v]) {
            lat_int[v] = UINT64_MAX;
            lms[v] = INFINITY;
            rel[v] = 0.0;
            pred[v] = -1;
        }
    }
    pred[s] = -1;
    return 0;
}

typedef struct {
    const orc_graph* g;
    const orc_csr* c;
    int mode;
    int32_t s0, s1, stride, first;
    const int32_t* list; /* sources list[i - s0] instead of i, when set */
    uint64_t* lat_int;
    uint64_t* lat_ref;
    double* rel;
    double* lat_ms;
    int32_t* pred;
    int rc;
} job_t;

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    const int32_t n = j->g->n;
    heap_t H = {0};
    uint64_t* di = (uint64_t*)malloc((size_t)n * sizeof(uint64_t));
    double* dd = (double*)malloc((size_t)n * sizeof(double));
    char* st = (char*)malloc((size_t)n);
    uint64_t* li = (uint64_t*)malloc((size_t)n * sizeof(uint64_t));
    double* lm = (double*)malloc((size_t)n * sizeof(double));
    double* rl = (double*)malloc((size_t)n * sizeof(double));
    int32_t* pr = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    j->rc = (!di || !dd || !st || !li || !lm || !rl || !pr) ? -1 : 0;
    for (int32_t i = j->s0 + j->first; i < j->s1 && j->rc == 0; i += j->stride) {
        const int32_t s = j->list ? j->list[i - j->s0] : i;
        if (sssp_one(j->g, j->c, j->mode, s, &H, di, dd, st, li, rl, lm, pr)) {
            j->rc = -1;
            break;
        }
        size_t off = (size_t)(i - j->s0) * (size_t)n;
        for (int32_t t = 0; t < n; t++) {
            if (j->lat_int) j->lat_int[off + t] = li[t];
            if (j->lat_ref) j->lat_ref[off + t] = (li[t] == UINT64_MAX) ? UINT64_MAX : ms_to_ns_ref(lm[t]);
            if (j->rel) j->rel[off + t] = rl[t];
            if (j->lat_ms) j->lat_ms[off + t] = lm[t];
            if (j->pred) j->pred[off + t] = pr[t];
        }
    }
    free(H.h);
    free(di);
    free(dd);
    free(st);
    free(li);
    free(lm);
    free(rl);
    free(pr);
    return NULL;
}

int orc_sssp_rows(const orc_graph* g, int mode, int32_t s0, int32_t s1, int nthreads,
                  uint64_t* lat_int, uint64_t* lat_ref, double* rel, double* lat_ms, int32_t* pred) {
    if (!g || g->n <= 0 || s0 < 0 || s1 > g->n || s0 > s1) return -1;
    orc_csr c;
    if (build_csr(g, &c)) return -1;
    if (nthreads < 1) nthreads = 1;
    job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    int rc = 0;
    for (int i = 0; i < nthreads; i++) {
        jobs[i] = (job_t){g, &c, mode, s0, s1, nthreads, i, NULL, lat_int, lat_ref, rel, lat_ms, pred, 0};
        if (nthreads == 1)
            worker(&jobs[i]);
        else
            pthread_create(&th[i], NULL, worker, &jobs[i]);
    }
    for (int i = 0; i < nthreads; i++) {
        if (nthreads > 1) pthread_join(th[i], NULL);
        if (jobs[i].rc) rc = -1;
    }
    free(jobs);
    free(th);
    free_csr(&c);
    return rc;
}

/* orc_sssp_rows for an arbitrary source list: row i is source srcs[i] (sources in [0, n)) */
int orc_sssp_list(const orc_graph* g, int mode, const int32_t* srcs, int32_t k, int nthreads,
                  uint64_t* lat_int, uint64_t* lat_ref, double* rel, double* lat_ms, int32_t* pred) {
    if (!g || g->n <= 0 || !srcs || k < 0) return -1;
    for (int32_t i = 0; i < k; i++)
        if (srcs[i] < 0 || srcs[i] >= g->n) return -1;
    orc_csr c;
    if (build_csr(g, &c)) return -1;
    if (nthreads < 1) nthreads = 1;
    job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    int rc = 0;
    for (int i = 0; i < nthreads; i++) {
        jobs[i] = (job_t){g, &c, mode, 0, k, nthreads, i, srcs, lat_int, lat_ref, rel, lat_ms, pred, 0};
        if (nthreads == 1)
            worker(&jobs[i]);
        else
            pthread_create(&th[i], NULL, worker, &jobs[i]);
    }
    for (int i = 0; i < nthreads; i++) {
        if (nthreads > 1) pthread_join(th[i], NULL);
        if (jobs[i].rc) rc = -1;
    }
    free(jobs);
    free(th);
    free_csr(&c);
    return rc;
}

/* topology.c:1431-1576. Candidates are the incident OUT edges of v (undirected: all incident
 * edges); self-loop -> L, other edge -> 2L (:1491-1497); first strict minimum wins (:1499) in the
 * canonical incidence order (neighbor index, edge index). No edges -> latency 0 (:1516-1519),
 * reliability stays at its initial 0.0 (:1435). */
void orc_self_path(const orc_graph* g, int32_t v, uint64_t* lat_int, uint64_t* lat_ref, double* rel,
                   double* lat_ms) {
    int64_t best = -1;
    int32_t best_nb = 0;
    double best_ms = -1.0;
    for (int64_t e = 0; e < g->m; e++) {
        int32_t a = g->src[e], b = g->dst[e], nb;
        if (a == v)
            nb = b;
        else if (!g->directed && b == v)
            nb = a;
        else
            continue;
        double ms = ns_to_ms(g->lat_ns[e]);
        if (nb != v) ms *= 2.0f;
        /* visit order: (neighbor index, edge index); keep the first strict minimum */
        int better;
        if (best < 0 || ms < best_ms)
            better = 1;
        else if (ms == best_ms)
            better = (nb < best_nb) || (nb == best_nb && e < best);
        else
            better = 0;
        if (better) {
            best = e;
            best_nb = nb;
            best_ms = ms;
        }
    }
    if (best < 0) {
        *lat_int = 0;
        *lat_ref = 0;
        *rel = 0.0;
        if (lat_ms) *lat_ms = 0.0;
        return;
    }
    int direct = (best_nb == v);
    double r = 1.0f - g->loss[best];
    *lat_int = direct ? (uint64_t)g->lat_ns[best] : 2 * (uint64_t)g->lat_ns[best];
    *lat_ref = ms_to_ns_ref(best_ms);
    *rel = direct ? r : r * r;
    if (lat_ms) *lat_ms = best_ms;
}

static int table_impl(const orc_graph* g, int use_shortest_path, int mode, int nthreads, int raw,
                      uint64_t* lat_int, uint64_t* lat_ref, double* rel, double* lat_ms) {
    const int32_t n = g->n;
    const size_t nn = (size_t)n * (size_t)n;
    if (!use_shortest_path) {
        /* topology.c:1816-1858: the (canonical) direct edge s->t, self-loop on the diagonal */
        for (size_t i = 0; i < nn; i++) {
            lat_int[i] = UINT64_MAX;
            lat_ref[i] = UINT64_MAX;
            rel[i] = 0.0;
            if (lat_ms) lat_ms[i] = INFINITY;
        }
        int64_t* best = (int64_t*)malloc(nn * sizeof(int64_t));
        if (!best) return -1;
        for (size_t i = 0; i < nn; i++) best[i] = -1;
        for (int64_t e = 0; e < g->m; e++) {
            int32_t a = g->src[e], b = g->dst[e];
            for (int dir = 0; dir < (g->directed ? 1 : 2); dir++) {
                size_t ix = dir ? (size_t)b * n + a : (size_t)a * n + b;
                int64_t cur = best[ix];
                if (cur < 0 || g->lat_ns[e] < g->lat_ns[cur]) best[ix] = e;
            }
        }
        int rc = 0;
        for (size_t i = 0; i < nn; i++) {
            int64_t e = best[i];
            if (e < 0) {
                rc = -1;
                continue;
            }
            double ms = 0.0 + ns_to_ms(g->lat_ns[e]);
            lat_int[i] = (uint64_t)g->lat_ns[e];
            lat_ref[i] = ms_to_ns_ref(ms);
            rel[i] = 1.0 * (1.0f - g->loss[e]);
            if (lat_ms) lat_ms[i] = ms;
        }
        free(best);
        return rc;
    }
    if (orc_sssp_rows(g, mode, 0, n, nthreads, lat_int, lat_ref, rel, lat_ms, NULL)) return -1;
    if (!g->directed && !raw) {
        /* one cache entry per unordered pair, computed from min(s,t) (topology.c:1194-1199) */
        for (int32_t s = 0; s < n; s++)
            for (int32_t t = 0; t < s; t++) {
                size_t lo = (size_t)t * n + s, hi = (size_t)s * n + t;
                lat_int[hi] = lat_int[lo];
                lat_ref[hi] = lat_ref[lo];
                rel[hi] = rel[lo];
                if (lat_ms) lat_ms[hi] = lat_ms[lo];
            }
    }
    for (int32_t v = 0; v < n; v++) {
        size_t d = (size_t)v * n + v;
        orc_self_path(g, v, &lat_int[d], &lat_ref[d], &rel[d], lat_ms ? &lat_ms[d] : NULL);
    }
    return 0;
}

int orc_table(const orc_graph* g, int use_shortest_path, int mode, int nthreads, uint64_t* lat_int,
              uint64_t* lat_ref, double* rel, double* lat_ms) {
    return table_impl(g, use_shortest_path, mode, nthreads, 0, lat_int, lat_ref, rel, lat_ms);
}

int orc_table_raw(const orc_graph* g, int use_shortest_path, int mode, int nthreads,
                  uint64_t* lat_int, uint64_t* lat_ref, double* rel, double* lat_ms) {
    return table_impl(g, use_shortest_path, mode, nthreads, 1, lat_int, lat_ref, rel, lat_ms);
}

/* ---------------------------------------------------------------------------------------------
 * CPU baseline on the dense synthetic complete graphs (C2 / C4 of SURVEY.md §8d): the weight
 * matrix is generated from the same counter hash as shadow_amd/graphs.py and the device
 * generator, then a dense O(n^2) Dijkstra (linear (dist, index) selection -- the canonical order,
 * strict-< relaxation) runs per sampled source with path-order reliability.
 * ------------------------------------------------------------------------------------------- */
static inline uint64_t smix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint64_t ghash(uint64_t seed, uint64_t stream, uint32_t i, uint32_t j) {
    return smix(smix(seed * 4ull + stream) ^ (((uint64_t)i << 32) | j));
}

typedef struct {
    int32_t n, r0, r1;
    uint64_t seed;
    uint32_t lat_max, self_max;
    uint32_t* W;
    uint32_t metric; /* 0: U{1..lat_max}; else the metric graph with scale `metric` ms */
} genjob_t;

/* The metric graph (bench workload c4metric; shadow_amd/csrc/dense.hip gen_metric_kernel restates
 * it on the device): point i at 16-bit grid coordinates of the unit square, latency
 * max(1, round(scale * dist)) ms with the rounding decided in exact integer arithmetic, so the two
 * generators agree bit for bit: L = the largest L with ((2L - 1) 2^15)^2 <= scale^2 d2, where d2 is
 * the squared grid distance (scale * sqrt(d2) / 2^16 >= L - 1/2). */
static inline uint32_t metric_coord(uint64_t seed, uint32_t i, int axis) {
    return (uint32_t)(ghash(seed, 0, i, 0xFFFFFFFFu - (uint32_t)axis) & 0xFFFFu);
}
static inline uint32_t metric_lat(uint64_t seed, uint32_t scale, uint32_t a, uint32_t b) {
    const int64_t dx = (int64_t)metric_coord(seed, a, 0) - metric_coord(seed, b, 0);
    const int64_t dy = (int64_t)metric_coord(seed, a, 1) - metric_coord(seed, b, 1);
    const uint64_t d2 = (uint64_t)(dx * dx + dy * dy);
    const uint64_t A = (uint64_t)scale * scale * d2;
    uint64_t L = (uint64_t)((double)scale * sqrt((double)d2) / 65536.0 + 0.5);
#define METRIC_F(L) (((2ull * (L) - 1ull) << 15) * ((2ull * (L) - 1ull) << 15))
    while (L > 0 && METRIC_F(L) > A) L--;
    while (METRIC_F(L + 1) <= A) L++;
#undef METRIC_F
    return L > 0 ? (uint32_t)L : 1u;
}

static void* gen_worker(void* a) {
    genjob_t* j = (genjob_t*)a;
    for (int32_t i = j->r0; i < j->r1; i++)
        for (int32_t k = 0; k < j->n; k++) {
            uint32_t x = i < k ? i : k, y = i < k ? k : i;
            j->W[(size_t)i * j->n + k] =
                (x == y)    ? 1u + (uint32_t)(ghash(j->seed, 2, x, x) % j->self_max)
                : j->metric ? metric_lat(j->seed, j->metric, x, y)
                            : 1u + (uint32_t)(ghash(j->seed, 0, x, y) % j->lat_max);
        }
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

typedef struct {
    int32_t n;
    uint64_t seed;
    uint32_t loss_max;
    const uint32_t* W;
    const int32_t* sources;
    int32_t k0, k1;
    uint64_t* lat_out;
    double* rel_out;
} djob_t;

static void* dense_worker(void* a) {
    djob_t* j = (djob_t*)a;
    const int32_t n = j->n;
    uint32_t* dist = (uint32_t*)malloc((size_t)n * sizeof(uint32_t));
    int32_t* pred = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    uint8_t* done = (uint8_t*)malloc((size_t)n);
    double* rel = (double*)malloc((size_t)n * sizeof(double));
    for (int32_t q = j->k0; q < j->k1; q++) {
        const int32_t s = j->sources[q];
        for (int32_t v = 0; v < n; v++) {
            dist[v] = 0xFFFFFFFFu;
            pred[v] = -1;
            done[v] = 0;
        }
        dist[s] = 0;
        rel[s] = 1.0;
        for (int32_t it = 0; it < n; it++) {
            uint32_t best = 0xFFFFFFFFu;
            int32_t u = -1;
            for (int32_t v = 0; v < n; v++)
                if (!done[v] && dist[v] < best) {
                    best = dist[v];
                    u = v;
                }
            if (u < 0) break;
            done[u] = 1;
            if (u != s) {
                const int32_t p = pred[u];
                const uint32_t x = p < u ? p : u, y = p < u ? u : p;
                const double loss = (double)(ghash(j->seed, 1, x, y) % (j->loss_max + 1u)) / 10000.0;
                rel[u] = rel[p] * (1.0 - loss);
            }
            const uint32_t* row = j->W + (size_t)u * n;
            const uint32_t du = dist[u];
            for (int32_t v = 0; v < n; v++) {
                if (v == u || done[v]) continue;
                const uint32_t nd = du + row[v];
                if (nd < dist[v]) {
                    dist[v] = nd;
                    pred[v] = u;
                }
            }
        }
        for (int32_t v = 0; v < n; v++) {
            j->lat_out[(size_t)q * n + v] = (uint64_t)dist[v] * 1000000ull;
            j->rel_out[(size_t)q * n + v] = rel[v];
        }
    }
    free(dist);
    free(pred);
    free(done);
    free(rel);
    return NULL;
}

static int dense_sample(int32_t n, uint64_t seed, uint32_t lat_max, uint32_t metric,
                        uint32_t self_max, uint32_t loss_max, const int32_t* sources, int32_t k,
                        int nthreads, uint64_t* lat_out, double* rel_out, double* gen_seconds,
                        double* sssp_seconds);

int orc_complete_sample(int32_t n, uint64_t seed, uint32_t lat_max, uint32_t self_max,
                        uint32_t loss_max, const int32_t* sources, int32_t k, int nthreads,
                        uint64_t* lat_out, double* rel_out, double* gen_seconds,
                        double* sssp_seconds) {
    return dense_sample(n, seed, lat_max, 0, self_max, loss_max, sources, k, nthreads, lat_out,
                        rel_out, gen_seconds, sssp_seconds);
}

int orc_metric_sample(int32_t n, uint64_t seed, uint32_t scale_ms, uint32_t self_max,
                      uint32_t loss_max, const int32_t* sources, int32_t k, int nthreads,
                      uint64_t* lat_out, double* rel_out, double* gen_seconds,
                      double* sssp_seconds) {
    if (scale_ms == 0 || scale_ms > 1024) return -1;
    return dense_sample(n, seed, 0, scale_ms, self_max, loss_max, sources, k, nthreads, lat_out,
                        rel_out, gen_seconds, sssp_seconds);
}

/* the weight of one pair of the generators (tests pin the device generator against it) */
uint32_t orc_dense_weight(uint64_t seed, uint32_t lat_max, uint32_t metric, uint32_t self_max,
                          uint32_t i, uint32_t j) {
    const uint32_t x = i < j ? i : j, y = i < j ? j : i;
    if (x == y) return 1u + (uint32_t)(ghash(seed, 2, x, x) % self_max);
    return metric ? metric_lat(seed, metric, x, y) : 1u + (uint32_t)(ghash(seed, 0, x, y) % lat_max);
}

static int dense_sample(int32_t n, uint64_t seed, uint32_t lat_max, uint32_t metric,
                        uint32_t self_max, uint32_t loss_max, const int32_t* sources, int32_t k,
                        int nthreads, uint64_t* lat_out, double* rel_out, double* gen_seconds,
                        double* sssp_seconds) {
    if (n <= 0 || k <= 0 || !sources || !lat_out || !rel_out) return -1;
    uint32_t* W = (uint32_t*)malloc((size_t)n * (size_t)n * sizeof(uint32_t));
    if (!W) return -1;
    int gt = 16;
    double t0 = now_s();
    pthread_t th[64];
    genjob_t gj[64];
    for (int i = 0; i < gt; i++) {
        gj[i] = (genjob_t){n, (int32_t)((int64_t)n * i / gt), (int32_t)((int64_t)n * (i + 1) / gt),
                           seed, lat_max, self_max, W, metric};
        pthread_create(&th[i], NULL, gen_worker, &gj[i]);
    }
    for (int i = 0; i < gt; i++) pthread_join(th[i], NULL);
    double t1 = now_s();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    djob_t dj[64];
    for (int i = 0; i < nthreads; i++) {
        dj[i] = (djob_t){n, seed, loss_max, W, sources, (int32_t)((int64_t)k * i / nthreads),
                         (int32_t)((int64_t)k * (i + 1) / nthreads), lat_out, rel_out};
        if (nthreads == 1)
            dense_worker(&dj[i]);
        else
            pthread_create(&th[i], NULL, dense_worker, &dj[i]);
    }
    if (nthreads > 1)
        for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    double t2 = now_s();
    free(W);
    if (gen_seconds) *gen_seconds = t1 - t0;
    if (sssp_seconds) *sssp_seconds = t2 - t1;
    return 0;
}
