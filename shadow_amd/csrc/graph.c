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

typedef struct {
    int32_t u, v;
    int64_t lat;
    int64_t e;
} carc;

static int carc_cmp(const void* a, const void* b) {
    const carc* x = (const carc*)a;
    const carc* y = (const carc*)b;
    if (x->u != y->u) return x->u < y->u ? -1 : 1;
    if (x->v != y->v) return x->v < y->v ? -1 : 1;
    if (x->lat != y->lat) return x->lat < y->lat ? -1 : 1;
    if (x->e != y->e) return x->e < y->e ? -1 : 1;
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

/* Largest hop count of a breadth-first search from `root` over the k arcs (u -> v, or v -> u when
 * backward); -1 if some vertex is unreachable. */
static int64_t hop_ecc(int32_t n, const carc* a, int64_t k, int32_t root, int backward) {
    int32_t* ptr = (int32_t*)calloc((size_t)n + 1, sizeof(int32_t));
    int32_t* adj = (int32_t*)malloc((size_t)(k > 0 ? k : 1) * sizeof(int32_t));
    int32_t* q = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    int32_t* dep = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    int64_t ecc = -2;
    if (ptr && adj && q && dep) {
        for (int64_t i = 0; i < k; i++) ptr[(backward ? a[i].v : a[i].u) + 1]++;
        for (int32_t v = 0; v < n; v++) ptr[v + 1] += ptr[v];
        for (int64_t i = 0; i < k; i++) {
            const int32_t x = backward ? a[i].v : a[i].u;
            adj[ptr[x]++] = backward ? a[i].u : a[i].v;
        }
        for (int32_t v = n; v > 0; v--) ptr[v] = ptr[v - 1];
        ptr[0] = 0;
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
    free(ptr);
    free(adj);
    free(q);
    free(dep);
    return ecc;
}

static int lat_cmp(const void* a, const void* b) {
    const carc* x = (const carc*)a;
    const carc* y = (const carc*)b;
    if (x->lat != y->lat) return x->lat < y->lat ? -1 : 1;
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

static int fill_csr(const srt_edges* g, carc* a, int64_t k, uint64_t q, int32_t** rowptr,
                    int32_t** col, uint32_t** w, double** r, int64_t* arcs_out) {
    qsort(a, (size_t)k, sizeof(carc), carc_cmp);
    int64_t uniq = 0;
    for (int64_t i = 0; i < k; i++)
        if (!(i > 0 && a[i].u == a[i - 1].u && a[i].v == a[i - 1].v)) uniq++;
    *rowptr = (int32_t*)calloc((size_t)g->n + 1, sizeof(int32_t));
    *col = (int32_t*)malloc((size_t)(uniq > 0 ? uniq : 1) * sizeof(int32_t));
    *w = (uint32_t*)malloc((size_t)(uniq > 0 ? uniq : 1) * sizeof(uint32_t));
    *r = (double*)malloc((size_t)(uniq > 0 ? uniq : 1) * sizeof(double));
    if (!*rowptr || !*col || !*w || !*r) return SRT_E_NOMEM;
    int64_t o = 0;
    for (int64_t i = 0; i < k; i++) {
        if (i > 0 && a[i].u == a[i - 1].u && a[i].v == a[i - 1].v) continue;
        (*col)[o] = a[i].v;
        (*w)[o] = (uint32_t)((uint64_t)a[i].lat / q);
        (*r)[o] = 1.0f - g->loss[a[i].e]; /* topology.c:396 */
        (*rowptr)[a[i].u + 1]++;
        o++;
    }
    for (int32_t i = 0; i < g->n; i++) (*rowptr)[i + 1] += (*rowptr)[i];
    *arcs_out = uniq;
    return SRT_OK;
}

int srt_canon_build(const srt_edges* g, srt_canon* c) {
    memset(c, 0, sizeof(*c));
    if (!g || g->n <= 0 || g->m < 0) {
        srt_set_error("empty graph");
        return SRT_E_ARG;
    }
    int rc = srt_latency_quantum(g, &c->quantum_ns, &c->max_w_q);
    if (rc) return rc;
    c->n = g->n;
    c->directed = g->directed;
    const uint64_t q = c->quantum_ns;
    int64_t cap = g->directed ? g->m : 2 * g->m;
    carc* a = (carc*)malloc((size_t)(cap > 0 ? cap : 1) * sizeof(carc));
    c->self_w = (uint32_t*)malloc((size_t)g->n * sizeof(uint32_t));
    c->self_r = (double*)malloc((size_t)g->n * sizeof(double));
    if (!a || !c->self_w || !c->self_r) {
        free(a);
        srt_canon_free(c);
        return SRT_E_NOMEM;
    }
    int64_t* self_e = (int64_t*)malloc((size_t)g->n * sizeof(int64_t));
    if (!self_e) {
        free(a);
        srt_canon_free(c);
        return SRT_E_NOMEM;
    }
    for (int32_t v = 0; v < g->n; v++) self_e[v] = -1;
    int64_t k = 0;
    for (int64_t e = 0; e < g->m; e++) {
        int32_t u = g->src[e], v = g->dst[e];
        if (u < 0 || u >= g->n || v < 0 || v >= g->n) {
            free(a);
            free(self_e);
            srt_canon_free(c);
            srt_set_error("edge %lld has an endpoint out of range", (long long)e);
            return SRT_E_ARG;
        }
        if (u == v) {
            if (self_e[u] < 0 || g->lat_ns[e] < g->lat_ns[self_e[u]]) self_e[u] = e;
            continue;
        }
        a[k++] = (carc){u, v, g->lat_ns[e], e};
        if (!g->directed) a[k++] = (carc){v, u, g->lat_ns[e], e};
    }
    for (int32_t v = 0; v < g->n; v++) {
        c->self_w[v] = self_e[v] < 0 ? SRT_INF : (uint32_t)((uint64_t)g->lat_ns[self_e[v]] / q);
        c->self_r[v] = self_e[v] < 0 ? 0.0 : 1.0f - g->loss[self_e[v]];
    }
    free(self_e);
    /* Range bound on any shortest distance: the smaller of (undirected) the MST weight or
     * (directed) (n - 1) * max_w, and the hop bound through the highest-degree vertex p:
     * D(a, b) <= D(a, p) + D(p, b) <= (ecc_in(p) + ecc_out(p)) * max_w in hops, which keeps
     * small-world graphs with fine quanta (a 100k power-law graph at 1 us) in the u32 tables. */
    uint64_t bound;
    if (!g->directed) {
        carc* b = (carc*)malloc((size_t)(k > 0 ? k : 1) * sizeof(carc));
        int32_t* par = (int32_t*)malloc((size_t)g->n * sizeof(int32_t));
        if (!b || !par) {
            free(a);
            free(b);
            free(par);
            srt_canon_free(c);
            return SRT_E_NOMEM;
        }
        memcpy(b, a, (size_t)k * sizeof(carc));
        qsort(b, (size_t)k, sizeof(carc), lat_cmp);
        for (int32_t i = 0; i < g->n; i++) par[i] = i;
        bound = 0;
        for (int64_t i = 0; i < k; i++) {
            int32_t x = uf_find(par, b[i].u), y = uf_find(par, b[i].v);
            if (x != y) {
                par[x] = y;
                bound += (uint64_t)b[i].lat / q;
            }
        }
        free(b);
        free(par);
    } else {
        bound = (uint64_t)(g->n - 1) * (uint64_t)c->max_w_q;
    }
    {
        int32_t* deg = (int32_t*)calloc((size_t)g->n, sizeof(int32_t));
        if (deg) {
            for (int64_t i = 0; i < k; i++) deg[a[i].u]++;
            int32_t p = 0;
            for (int32_t v = 1; v < g->n; v++)
                if (deg[v] > deg[p]) p = v;
            free(deg);
            const int64_t eo = hop_ecc(g->n, a, k, p, 0);
            const int64_t ei = g->directed ? hop_ecc(g->n, a, k, p, 1) : eo;
            if (eo >= 0 && ei >= 0) {
                const uint64_t hb = (uint64_t)(eo + ei) * (uint64_t)c->max_w_q;
                if (hb < bound) bound = hb;
            }
        }
    }
    if (2ull * c->max_w_q >= SRT_INF) {
        free(a);
        srt_canon_free(c);
        srt_set_error("an edge latency of %llu quanta of %llu ns passes the u32 arc range",
                      (unsigned long long)c->max_w_q, (unsigned long long)q);
        return SRT_E_RANGE;
    }
    /* distances that may pass u32 quanta: the u64 rows (wide.hip) build the graph */
    c->wide = bound >= SRT_INF;
    c->dist_bound = bound;
    rc = fill_csr(g, a, k, q, &c->rowptr, &c->col, &c->w, &c->r, &c->arcs);
    if (rc == SRT_OK && g->directed) {
        for (int64_t i = 0; i < k; i++) {
            int32_t t = a[i].u;
            a[i].u = a[i].v;
            a[i].v = t;
        }
        int64_t in_arcs = 0;
        rc = fill_csr(g, a, k, q, &c->in_rowptr, &c->in_col, &c->in_w, &c->in_r, &in_arcs);
    } else if (rc == SRT_OK) {
        c->in_rowptr = c->rowptr;
        c->in_col = c->col;
        c->in_w = c->w;
        c->in_r = c->r;
    }
    free(a);
    if (rc) srt_canon_free(c);
    return rc;
}
