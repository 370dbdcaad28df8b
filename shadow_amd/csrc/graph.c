/*
 * graph.c -- canonical arc form of a validated edge list + latency quantum, and logging.
 *
 * Canonical arcs: one per ordered vertex pair (u != v), the (min latency, lowest edge index) edge
 * of that pair (igraph Dijkstra relaxes every parallel edge, so the minimum wins the distance;
 * the reference then re-finds "an" edge with igraph_get_eid, topology.c:377-381, whose choice
 * among parallel edges igraph leaves unspecified -- the lowest index is our canonical choice).
 * Undirected edges give both directions (IGRAPH_OUT on an undirected graph = ALL).
 * Self-loops never shorten a path; they only feed the diagonal rule (topology.c:1431-1576).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "srt_internal.h"

static int g_log_level = -1;

static int log_level(void) {
    if (g_log_level < 0) {
        const char* e = getenv("SRT_LOG_LEVEL");
        g_log_level = e ? atoi(e) : SRT_LOG_WARNING;
    }
    return g_log_level;
}

/* SRT_FORM: forcing of internal forms for tests and A/B runs, a comma-separated
 * list of key=value pairs, re-read at every call (tests change it between builds). Production
 * builds never set it: every form is chosen from the graph and the device. */
static const char* form_find(const char* key) {
    const char* e = getenv("SRT_FORM");
    if (!e) return NULL;
    const size_t kl = strlen(key);
    for (const char* p = e; *p;) {
        while (*p == ',' || *p == ' ') p++;
        if (!strncmp(p, key, kl) && p[kl] == '=') return p + kl + 1;
        while (*p && *p != ',') p++;
    }
    return NULL;
}

int srt_form_int(const char* key, int dflt) {
    const char* v = form_find(key);
    return v && *v && *v != ',' ? atoi(v) : dflt;
}

int srt_form_is(const char* key, const char* value) {
    const char* v = form_find(key);
    if (!v) return 0;
    const size_t l = strlen(value);
    return !strncmp(v, value, l) && (v[l] == '\0' || v[l] == ',');
}

void srt_log(int level, const char* fmt, ...) {
    if (level > log_level()) return;
    static const char* names[] = {"error", "warning", "info", "debug"};
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    fprintf(stderr, "[shadow-routing] %s: %s\n", names[level < 0 ? 0 : (level > 3 ? 3 : level)],
            buf);
}

static __thread char g_err[1024];

void srt_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    srt_log(SRT_LOG_ERROR, "%s", g_err);
}

const char* srt_last_error(void) { return g_err; }

const char* srt_version(void) { return "shadow-routing-mi355x 0.1.0 (gfx950)"; }

static uint64_t gcd64(uint64_t a, uint64_t b) {
    while (b) {
        uint64_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}

/* ---- canonical arcs ------------------------------------------------------------------------
 * Rows by a counting sort of the edge list (each row's entries land in ascending edge index), then
 * every row on its own: a dense row (degree >= n / 8: complete graphs) through a per-thread scratch
 * indexed by head vertex, a sparse row by a sort; the first entry of the smallest latency of each
 * head is its canonical arc (ties to the lowest edge index: the entries are in index order).
 * Rows are canonicalised by up to 16 threads. O(m) for dense graphs, where a global sort of the
 * 2m arcs (C4: 1.07e9) took minutes. */
typedef struct {
    int32_t v;
    int32_t pad;
    int64_t lat;
    int64_t e;
} rent;

static int rent_cmp(const void* x, const void* y) {
    const rent* a = (const rent*)x;
    const rent* b = (const rent*)y;
    if (a->v != b->v) return a->v < b->v ? -1 : 1;
    if (a->lat != b->lat) return a->lat < b->lat ? -1 : 1;
    if (a->e != b->e) return a->e < b->e ? -1 : 1;
    return 0;
}

/* union-find for the MST bound */
static int32_t uf_find(int32_t* p, int32_t x) {
    while (p[x] != x) {
        p[x] = p[p[x]];
        x = p[x];
    }
    return x;
}

/* Largest hop count of a breadth-first search from `root` over a CSR; -1 if some vertex is
 * unreachable, -2 out of memory. */
static int64_t hop_ecc_csr(int32_t n, const int32_t* ptr, const int32_t* adj, int32_t root) {
    int32_t* q = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    int32_t* dep = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    int64_t ecc = -2;
    if (q && dep) {
        for (int32_t v = 0; v < n; v++) dep[v] = -1;
        int32_t head = 0, tail = 0;
        dep[root] = 0;
        q[tail++] = root;
        ecc = 0;
        while (head < tail) {
            const int32_t u = q[head++];
            if (dep[u] > ecc) ecc = dep[u];
            for (int32_t j = ptr[u]; j < ptr[u + 1]; j++)
                if (dep[adj[j]] < 0) {
                    dep[adj[j]] = dep[u] + 1;
                    q[tail++] = adj[j];
                }
        }
        if (tail < n) ecc = -1;
    }
    free(q);
    free(dep);
    return ecc;
}

typedef struct {
    int32_t u, v;
    int64_t lat;
} marc;

static int marc_cmp(const void* x, const void* y) {
    const marc* a = (const marc*)x;
    const marc* b = (const marc*)y;
    if (a->lat != b->lat) return a->lat < b->lat ? -1 : 1;
    return 0;
}

int srt_latency_quantum(const srt_edges* g, uint64_t* quantum_ns, uint32_t* max_w_q) {
    uint64_t q = 0;
    uint64_t mx = 0;
    for (int64_t e = 0; e < g->m; e++) {
        if (g->lat_ns[e] <= 0) {
            srt_set_error("edge %lld has non-positive latency", (long long)e);
            return SRT_E_INVALID;
        }
        q = gcd64(q, (uint64_t)g->lat_ns[e]);
        if ((uint64_t)g->lat_ns[e] > mx) mx = (uint64_t)g->lat_ns[e];
    }
    if (q == 0) q = 1000000; /* no edges: any quantum, tables hold zeros / INF */
    *quantum_ns = q;
    uint64_t mq = mx / q;
    if (mq >= SRT_INF / 2) {
        srt_set_error("edge latency %llu ns exceeds the u32 quantum range (quantum %llu ns)",
                      (unsigned long long)mx, (unsigned long long)q);
        return SRT_E_RANGE;
    }
    *max_w_q = (uint32_t)mq;
    return SRT_OK;
}

void srt_canon_free(srt_canon* c) {
    if (!c) return;
    if (c->in_rowptr != c->rowptr) {
        free(c->in_rowptr);
        free(c->in_col);
        free(c->in_w);
        free(c->in_r);
    }
    free(c->rowptr);
    free(c->col);
    free(c->w);
    free(c->r);
    free(c->self_w);
    free(c->self_r);
    memset(c, 0, sizeof(*c));
}

typedef struct {
    int32_t n;
    const int64_t* rp; /* row starts into a */
    rent* a;
    int32_t* ucnt;     /* canonical arcs per row (compacted at the row's start) */
    int32_t next;      /* next row to take (atomic) */
    int failed;
} canon_job;

static void* canon_rows(void* arg) {
    canon_job* j = (canon_job*)arg;
    const int32_t n = j->n;
    int32_t* stamp = NULL;
    int64_t* best = NULL;
    for (;;) {
        const int32_t u0 = __atomic_fetch_add(&j->next, 64, __ATOMIC_RELAXED);
        if (u0 >= n) break;
        const int32_t u1 = u0 + 64 < n ? u0 + 64 : n;
        for (int32_t u = u0; u < u1; u++) {
            rent* r = j->a + j->rp[u];
            const int64_t deg = j->rp[u + 1] - j->rp[u];
            int32_t k = 0;
            if (deg * 8 >= n && deg > 64) { /* dense row: scratch by head vertex */
                if (!stamp) {
                    stamp = (int32_t*)malloc((size_t)n * sizeof(int32_t));
                    best = (int64_t*)malloc((size_t)n * sizeof(int64_t));
                    if (!stamp || !best) {
                        __atomic_store_n(&j->failed, 1, __ATOMIC_RELAXED);
                        break;
                    }
                    for (int32_t v = 0; v < n; v++) stamp[v] = -1;
                }
                for (int64_t i = 0; i < deg; i++) {
                    const int32_t v = r[i].v;
                    if (stamp[v] != u) {
                        stamp[v] = u;
                        best[v] = i;
                    } else if (r[i].lat < r[best[v]].lat) {
                        best[v] = i; /* strict: the lowest edge index keeps equal latencies */
                    }
                }
                /* heads in ascending order; every kept entry sits at or after its slot */
                int64_t* pick = best; /* (reused below as the ordered list of picks) */
                int32_t cnt = 0;
                for (int32_t v = 0; v < n; v++)
                    if (stamp[v] == u) pick[cnt++] = best[v];
                /* picks ascend in v but not in position: copy out through a small buffer */
                rent* tmp = (rent*)malloc((size_t)cnt * sizeof(rent));
                if (!tmp) {
                    __atomic_store_n(&j->failed, 1, __ATOMIC_RELAXED);
                    break;
                }
                for (int32_t i = 0; i < cnt; i++) tmp[i] = r[pick[i]];
                memcpy(r, tmp, (size_t)cnt * sizeof(rent));
                free(tmp);
                k = cnt;
                /* restore the scratch's contract for the next row (stamp by row id) */
            } else if (deg > 0) {
                qsort(r, (size_t)deg, sizeof(rent), rent_cmp);
                for (int64_t i = 0; i < deg; i++)
                    if (i == 0 || r[i].v != r[i - 1].v) r[k++] = r[i];
            }
            j->ucnt[u] = k;
        }
    }
    free(stamp);
    free(best);
    return NULL;
}

static int canon_threads(void) {
    long c = sysconf(_SC_NPROCESSORS_ONLN);
    return c < 1 ? 1 : c > 16 ? 16 : (int)c;
}

int srt_canon_build(const srt_edges* g, srt_canon* c) {
    memset(c, 0, sizeof(*c));
    if (!g || g->n <= 0 || g->m < 0) {
        srt_set_error("empty graph");
        return SRT_E_ARG;
    }
    int rc = srt_latency_quantum(g, &c->quantum_ns, &c->max_w_q);
    if (rc) return rc;
    const int32_t n = g->n;
    c->n = n;
    c->directed = g->directed;
    const uint64_t q = c->quantum_ns;
    c->self_w = (uint32_t*)malloc((size_t)n * sizeof(uint32_t));
    c->self_r = (double*)malloc((size_t)n * sizeof(double));
    int64_t* self_e = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    int64_t* rp = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    int64_t* cur = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    int32_t* ucnt = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    rent* a = NULL;
    if (!c->self_w || !c->self_r || !self_e || !rp || !cur || !ucnt) goto nomem;
    for (int32_t v = 0; v < n; v++) self_e[v] = -1;
    /* rows: counts, then the entries in edge order */
    for (int64_t e = 0; e < g->m; e++) {
        const int32_t u = g->src[e], v = g->dst[e];
        if (u < 0 || u >= n || v < 0 || v >= n) {
            free(self_e);
            free(rp);
            free(cur);
            free(ucnt);
            srt_canon_free(c);
            srt_set_error("edge %lld has an endpoint out of range", (long long)e);
            return SRT_E_ARG;
        }
        if (u == v) {
            if (self_e[u] < 0 || g->lat_ns[e] < g->lat_ns[self_e[u]]) self_e[u] = e;
            continue;
        }
        rp[u + 1]++;
        if (!g->directed) rp[v + 1]++;
    }
    for (int32_t v = 0; v < n; v++) {
        c->self_w[v] = self_e[v] < 0 ? SRT_INF : (uint32_t)((uint64_t)g->lat_ns[self_e[v]] / q);
        c->self_r[v] = self_e[v] < 0 ? 0.0 : 1.0f - g->loss[self_e[v]];
    }
    free(self_e);
    self_e = NULL;
    for (int32_t v = 0; v < n; v++) rp[v + 1] += rp[v];
    const int64_t k = rp[n];
    a = (rent*)malloc((size_t)(k > 0 ? k : 1) * sizeof(rent));
    if (!a) goto nomem;
    memcpy(cur, rp, (size_t)n * sizeof(int64_t));
    for (int64_t e = 0; e < g->m; e++) {
        const int32_t u = g->src[e], v = g->dst[e];
        if (u == v) continue;
        a[cur[u]++] = (rent){v, 0, g->lat_ns[e], e};
        if (!g->directed) a[cur[v]++] = (rent){u, 0, g->lat_ns[e], e};
    }
    free(cur);
    cur = NULL;
    {
        canon_job job = {n, rp, a, ucnt, 0, 0};
        const int nt = n >= 4096 ? canon_threads() : 1;
        pthread_t th[16];
        int started = 0;
        for (int i = 1; i < nt; i++)
            if (pthread_create(&th[started], NULL, canon_rows, &job) == 0) started++;
        canon_rows(&job);
        for (int i = 0; i < started; i++) pthread_join(th[i], NULL);
        if (job.failed) goto nomem;
    }
    /* the CSR of canonical arcs */
    int64_t arcs = 0;
    for (int32_t u = 0; u < n; u++) arcs += ucnt[u];
    if (arcs >= 0x7FFFFFFFll) {
        free(a);
        free(rp);
        free(ucnt);
        srt_canon_free(c);
        srt_set_error("%lld canonical arcs pass the int32 CSR", (long long)arcs);
        return SRT_E_RANGE;
    }
    c->rowptr = (int32_t*)malloc(((size_t)n + 1) * sizeof(int32_t));
    c->col = (int32_t*)malloc((size_t)(arcs > 0 ? arcs : 1) * sizeof(int32_t));
    c->w = (uint32_t*)malloc((size_t)(arcs > 0 ? arcs : 1) * sizeof(uint32_t));
    c->r = (double*)malloc((size_t)(arcs > 0 ? arcs : 1) * sizeof(double));
    if (!c->rowptr || !c->col || !c->w || !c->r) goto nomem;
    c->rowptr[0] = 0;
    for (int32_t u = 0; u < n; u++) c->rowptr[u + 1] = c->rowptr[u] + ucnt[u];
    for (int32_t u = 0; u < n; u++) {
        const rent* r = a + rp[u];
        int32_t o = c->rowptr[u];
        for (int32_t i = 0; i < ucnt[u]; i++, o++) {
            c->col[o] = r[i].v;
            c->w[o] = (uint32_t)((uint64_t)r[i].lat / q);
            c->r[o] = 1.0f - g->loss[r[i].e]; /* topology.c:396 */
        }
    }
    c->arcs = arcs;
    free(a);
    a = NULL;
    free(rp);
    rp = NULL;
    free(ucnt);
    ucnt = NULL;
    /* in-arcs (directed): the transpose, sources ascending per target */
    if (g->directed) {
        c->in_rowptr = (int32_t*)calloc((size_t)n + 1, sizeof(int32_t));
        c->in_col = (int32_t*)malloc((size_t)(arcs > 0 ? arcs : 1) * sizeof(int32_t));
        c->in_w = (uint32_t*)malloc((size_t)(arcs > 0 ? arcs : 1) * sizeof(uint32_t));
        c->in_r = (double*)malloc((size_t)(arcs > 0 ? arcs : 1) * sizeof(double));
        int32_t* pos = (int32_t*)malloc((size_t)n * sizeof(int32_t));
        if (!c->in_rowptr || !c->in_col || !c->in_w || !c->in_r || !pos) {
            free(pos);
            goto nomem;
        }
        for (int64_t i = 0; i < arcs; i++) c->in_rowptr[c->col[i] + 1]++;
        for (int32_t v = 0; v < n; v++) c->in_rowptr[v + 1] += c->in_rowptr[v];
        memcpy(pos, c->in_rowptr, (size_t)n * sizeof(int32_t));
        for (int32_t u = 0; u < n; u++)
            for (int32_t i = c->rowptr[u]; i < c->rowptr[u + 1]; i++) {
                const int32_t o = pos[c->col[i]]++;
                c->in_col[o] = u;
                c->in_w[o] = c->w[i];
                c->in_r[o] = c->r[i];
            }
        free(pos);
    } else {
        c->in_rowptr = c->rowptr;
        c->in_col = c->col;
        c->in_w = c->w;
        c->in_r = c->r;
    }
    /* Range bound on any shortest distance: the hop bound through the highest-degree vertex p,
     * D(a, b) <= D(a, p) + D(p, b) <= (ecc_in(p) + ecc_out(p)) * max_w, and -- where that bound
     * does not already keep the distances below 16 bits (the multi-source kernel's u16 rows) --
     * the smaller of it and (undirected) the MST weight or (directed) (n - 1) * max_w. */
    uint64_t bound = UINT64_MAX;
    {
        int32_t p = 0;
        for (int32_t v = 1; v < n; v++)
            if (c->rowptr[v + 1] - c->rowptr[v] > c->rowptr[p + 1] - c->rowptr[p]) p = v;
        const int64_t eo = hop_ecc_csr(n, c->rowptr, c->col, p);
        const int64_t ei = g->directed ? hop_ecc_csr(n, c->in_rowptr, c->in_col, p) : eo;
        if (eo >= 0 && ei >= 0) bound = (uint64_t)(eo + ei) * (uint64_t)c->max_w_q;
    }
    if (bound >= 0xFFFFull) {
        uint64_t b2;
        if (!g->directed) { /* Kruskal over the u < v arcs */
            int64_t h = 0;
            for (int32_t u = 0; u < n; u++)
                for (int32_t i = c->rowptr[u]; i < c->rowptr[u + 1]; i++) h += c->col[i] > u;
            marc* m = (marc*)malloc((size_t)(h > 0 ? h : 1) * sizeof(marc));
            int32_t* par = (int32_t*)malloc((size_t)n * sizeof(int32_t));
            if (!m || !par) {
                free(m);
                free(par);
                goto nomem;
            }
            h = 0;
            for (int32_t u = 0; u < n; u++)
                for (int32_t i = c->rowptr[u]; i < c->rowptr[u + 1]; i++)
                    if (c->col[i] > u) m[h++] = (marc){u, c->col[i], (int64_t)c->w[i]};
            qsort(m, (size_t)h, sizeof(marc), marc_cmp);
            for (int32_t i = 0; i < n; i++) par[i] = i;
            b2 = 0;
            for (int64_t i = 0; i < h; i++) {
                const int32_t x = uf_find(par, m[i].u), y = uf_find(par, m[i].v);
                if (x != y) {
                    par[x] = y;
                    b2 += (uint64_t)m[i].lat;
                }
            }
            free(m);
            free(par);
        } else {
            b2 = (uint64_t)(n - 1) * (uint64_t)c->max_w_q;
        }
        if (b2 < bound) bound = b2;
    }
    if (2ull * c->max_w_q >= SRT_INF) {
        srt_canon_free(c);
        srt_set_error("an edge latency of %llu quanta of %llu ns passes the u32 arc range",
                      (unsigned long long)c->max_w_q, (unsigned long long)q);
        return SRT_E_RANGE;
    }
    /* distances that may pass u32 quanta: the u64 rows (wide.hip) build the graph */
    c->wide = bound >= SRT_INF;
    c->dist_bound = bound;
    return SRT_OK;
nomem:
    free(self_e);
    free(rp);
    free(cur);
    free(ucnt);
    free(a);
    srt_canon_free(c);
    srt_set_error("out of host memory in the canonical arc build");
    return SRT_E_NOMEM;
}
