/*
 * topology.c -- Shadow's routing module (drop-in for /root/reference/src/main/routing/topology.c)
 * with the all-pairs tables built eagerly on MI355X.
 *
 * Load + validation restate topology.c:326-1122; attach restates :2024-2281; the lookup API keeps
 * the semantics of :1900-2022 but reads row-major tables holding every source's own row instead of
 * running lazy Dijkstra under a global lock. Which row serves a pair -- the first source run that
 * stored it, as in the reference's lazy cache (:1189-1215, :1917-1967) -- is decided by
 * pairorder.c. Tables are immutable once built, so lookups are lock-free once their pair is
 * stored: the IP -> vertex map is read without a lock (writers -- attach, detach -- serialise among
 * themselves), the packet counters are atomic, and only a pair's first lookup (a source run)
 * takes the pair order's lock.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <ctype.h>
#include <math.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <sys/mman.h>

#include "gml.h"
#include "srt_internal.h"
#include "topology.h"

/* ---- Shadow entry points used by the reference-signature wrappers -----------------------
 * Provided by Shadow when linked into it; weak fallbacks in shadow_compat.c otherwise. */
extern uint32_t address_toNetworkIP(Address* address);
extern double random_nextDouble(Random* random);
extern void worker_updateMinTimeJump(double minPathLatency);

#define TOPOLOGY_MAGIC 0x70b0109au

/* ---- u32 -> i32 map (IP in network order -> vertex), lock-free reads ----------------------
 * Open addressing over 64-bit slot words (key << 32 | (u32)value; value -1 = empty, -2 =
 * tombstone), so a reader sees a key and its value in one atomic load. Writers (attach, detach)
 * serialise on ip_lock; a rehash builds a new table and publishes it. Readers take no lock: each
 * one counts itself in a per-thread stripe around its probe, so a writer that finds every stripe
 * at zero right after publishing a new table knows no reader still holds an older one, and frees
 * the retired tables then (otherwise they wait for a later rehash, or topology_free). A rehash of
 * a table that is mostly tombstones keeps its capacity, so attach/detach cycles do not grow it. */
typedef struct ipmap_tab {
    size_t cap, used; /* used: live + tombstones (probe-chain length bound) */
    struct ipmap_tab* retired;
    _Atomic uint64_t slot[];
} ipmap_tab;

#define IPM_STRIPES 64
/* one reader count per 128 B (two cache lines: no false sharing through the adjacent-line
 * prefetch either); the array is allocated 128-B aligned on first use (ipm_stripes) */
typedef struct {
    _Atomic long n;
    char pad[128 - sizeof(long)];
} ipm_stripe;

typedef struct {
    _Atomic(ipmap_tab*) cur;
    ipmap_tab* retired; /* replaced tables not yet known to be unread */
    ipm_stripe* rd;     /* IPM_STRIPES reader counts (set before the first table is published) */
} ipmap_t;

#define IPM_EMPTY 0xFFFFFFFFull /* value -1 */

static _Thread_local int ipm_tid = -1;
static _Atomic int ipm_next_tid;
static int ipm_stripe_of_thread(void) {
    if (ipm_tid < 0) ipm_tid = atomic_fetch_add(&ipm_next_tid, 1) & (IPM_STRIPES - 1);
    return ipm_tid;
}

static size_t h32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

static uint64_t ipm_word(uint32_t k, int32_t v) { return ((uint64_t)k << 32) | (uint32_t)v; }
static int32_t ipm_val(uint64_t w) { return (int32_t)(uint32_t)w; }
static uint32_t ipm_key(uint64_t w) { return (uint32_t)(w >> 32); }

static ipmap_tab* ipm_alloc(size_t cap) {
    ipmap_tab* t = (ipmap_tab*)malloc(sizeof(ipmap_tab) + cap * sizeof(uint64_t));
    if (!t) return NULL;
    t->cap = cap;
    t->used = 0;
    t->retired = NULL;
    for (size_t i = 0; i < cap; i++) atomic_init(&t->slot[i], IPM_EMPTY);
    return t;
}

static void ipm_free_list(ipmap_tab* t) {
    while (t) {
        ipmap_tab* nx = t->retired;
        free(t);
        t = nx;
    }
}

/* caller holds ip_lock (writer) */
static int ipmap_put(ipmap_t* m, uint32_t k, int32_t v) {
    if (!m->rd) { /* before any table exists: no reader can be counting yet */
        m->rd = (ipm_stripe*)aligned_alloc(128, sizeof(ipm_stripe) * IPM_STRIPES);
        if (!m->rd) return -1;
        for (int i = 0; i < IPM_STRIPES; i++) atomic_init(&m->rd[i].n, 0);
    }
    ipmap_tab* t = atomic_load_explicit(&m->cur, memory_order_relaxed);
    if (!t || (t->used + 1) * 2 > t->cap) { /* grow, or drop the tombstones: a new table */
        size_t live = 0;
        for (size_t i = 0; t && i < t->cap; i++)
            live += ipm_val(atomic_load_explicit(&t->slot[i], memory_order_relaxed)) >= 0;
        size_t nc = t ? t->cap : 64; /* mostly tombstones: the same capacity */
        while ((live + 1) * 4 > nc) nc *= 2;
        ipmap_tab* nt = ipm_alloc(nc);
        if (!nt) return -1;
        for (size_t i = 0; t && i < t->cap; i++) {
            const uint64_t w = atomic_load_explicit(&t->slot[i], memory_order_relaxed);
            if (ipm_val(w) < 0) continue;
            size_t h = h32(ipm_key(w)) & (nc - 1);
            while (ipm_val(atomic_load_explicit(&nt->slot[h], memory_order_relaxed)) != -1)
                h = (h + 1) & (nc - 1);
            atomic_store_explicit(&nt->slot[h], w, memory_order_relaxed);
            nt->used++;
        }
        atomic_store_explicit(&m->cur, nt, memory_order_seq_cst); /* publish */
        if (t) {
            t->retired = m->retired;
            m->retired = t;
        }
        /* a reader counted in no stripe now will load nt: every retired table is unread */
        long busy = 0;
        for (int i = 0; i < IPM_STRIPES && !busy; i++)
            busy = atomic_load_explicit(&m->rd[i].n, memory_order_seq_cst);
        if (!busy) {
            ipm_free_list(m->retired);
            m->retired = NULL;
        }
        t = nt;
    }
    size_t h = h32(k) & (t->cap - 1), tomb = (size_t)-1;
    for (;;) {
        const uint64_t w = atomic_load_explicit(&t->slot[h], memory_order_relaxed);
        const int32_t x = ipm_val(w);
        if (x == -1) break;
        if (x >= 0 && ipm_key(w) == k) {
            atomic_store_explicit(&t->slot[h], ipm_word(k, v), memory_order_release);
            return 0;
        }
        if (x == -2 && tomb == (size_t)-1) tomb = h;
        h = (h + 1) & (t->cap - 1);
    }
    if (tomb != (size_t)-1)
        h = tomb;
    else
        t->used++;
    atomic_store_explicit(&t->slot[h], ipm_word(k, v), memory_order_release);
    return 0;
}

/* no lock: count this reader in its stripe, one load of the table, then of each probed slot */
static int32_t ipmap_get(const ipmap_t* cm, uint32_t k) {
    ipmap_t* m = (ipmap_t*)cm;
    if (!atomic_load_explicit(&m->cur, memory_order_acquire)) return -1; /* (rd set before cur) */
    _Atomic long* rd = &m->rd[ipm_stripe_of_thread()].n;
    atomic_fetch_add_explicit(rd, 1, memory_order_seq_cst);
    const ipmap_tab* t = atomic_load_explicit(&m->cur, memory_order_seq_cst);
    int32_t r = -1;
    if (t) {
        size_t h = h32(k) & (t->cap - 1);
        for (size_t probes = 0; probes < t->cap; probes++) {
            const uint64_t w = atomic_load_explicit(&((ipmap_tab*)t)->slot[h], memory_order_acquire);
            const int32_t x = ipm_val(w);
            if (x == -1) break;
            if (x >= 0 && ipm_key(w) == k) {
                r = x;
                break;
            }
            h = (h + 1) & (t->cap - 1);
        }
    }
    atomic_fetch_sub_explicit(rd, 1, memory_order_release);
    return r;
}

/* caller holds ip_lock (writer) */
static void ipmap_del(ipmap_t* m, uint32_t k) {
    ipmap_tab* t = atomic_load_explicit(&m->cur, memory_order_relaxed);
    if (!t) return;
    size_t h = h32(k) & (t->cap - 1);
    for (;;) {
        const uint64_t w = atomic_load_explicit(&t->slot[h], memory_order_relaxed);
        const int32_t x = ipm_val(w);
        if (x == -1) return;
        if (x >= 0 && ipm_key(w) == k) {
            atomic_store_explicit(&t->slot[h], ipm_word(k, -2), memory_order_release);
            return;
        }
        h = (h + 1) & (t->cap - 1);
    }
}

static void ipmap_free(ipmap_t* m) {
    free(atomic_load(&m->cur));
    ipm_free_list(m->retired);
    m->retired = NULL;
    free(m->rd);
    m->rd = NULL;
}

/* the tables an ipmap holds (live + retired), for the growth test */
static size_t ipmap_tables(const ipmap_t* m) {
    size_t k = atomic_load(&((ipmap_t*)m)->cur) ? 1 : 0;
    for (const ipmap_tab* t = m->retired; t; t = t->retired) k++;
    return k;
}

/* ---- packet counters, one per cached Path (the served pair's source, target) ------------
 * Lock-free: per source vertex a directory of 1,024-counter pages over the targets, both
 * allocated on first use and installed by compare-and-swap (a loser frees its copy); an increment
 * is one relaxed fetch-add (topology.c:1983-1993: path_incrementPacketCount on the cached Path). */
#define CNT_PAGE 1024
typedef struct {
    int32_t n, npages;
    _Atomic(_Atomic(_Atomic uint64_t*)*)* dir; /* n directories of npages page pointers */
} cntmap_t;

static int cnt_init(cntmap_t* m, int32_t n) {
    m->n = n;
    m->npages = (n + CNT_PAGE - 1) / CNT_PAGE;
    m->dir = calloc((size_t)n, sizeof(*m->dir));
    return m->dir ? 0 : -1;
}

static _Atomic uint64_t* cnt_slot(cntmap_t* m, int32_t from, int32_t to, int create) {
    _Atomic(_Atomic uint64_t*)* d = atomic_load_explicit(&m->dir[from], memory_order_acquire);
    if (!d) {
        if (!create) return NULL;
        _Atomic(_Atomic uint64_t*)* nd = calloc((size_t)m->npages, sizeof(*nd));
        if (!nd) return NULL;
        _Atomic(_Atomic uint64_t*)* exp = NULL;
        if (atomic_compare_exchange_strong_explicit(&m->dir[from], &exp, nd, memory_order_acq_rel,
                                                    memory_order_acquire))
            d = nd;
        else {
            free(nd);
            d = exp;
        }
    }
    _Atomic uint64_t* pg = atomic_load_explicit(&d[to / CNT_PAGE], memory_order_acquire);
    if (!pg) {
        if (!create) return NULL;
        _Atomic uint64_t* np = calloc(CNT_PAGE, sizeof(*np));
        if (!np) return NULL;
        _Atomic uint64_t* exp = NULL;
        if (atomic_compare_exchange_strong_explicit(&d[to / CNT_PAGE], &exp, np,
                                                    memory_order_acq_rel, memory_order_acquire))
            pg = np;
        else {
            free(np);
            pg = exp;
        }
    }
    return &pg[to % CNT_PAGE];
}

static void cnt_free(cntmap_t* m) {
    if (!m->dir) return;
    for (int32_t v = 0; v < m->n; v++) {
        _Atomic(_Atomic uint64_t*)* d = atomic_load(&m->dir[v]);
        if (!d) continue;
        for (int32_t p = 0; p < m->npages; p++) free((void*)atomic_load(&d[p]));
        free((void*)d);
    }
    free((void*)m->dir);
    m->dir = NULL;
}

/* ---- the topology object -------------------------------------------------------------- */
struct _Topology {
    uint32_t magic;
    int use_shortest_path;
    int directed;
    int complete;
    int32_t n;
    int64_t m;
    /* validated attributes */
    double* vid;
    const char** vip;      /* "" if absent */
    const char** vcity;    /* NULL if absent */
    const char** vcountry; /* NULL if absent */
    uint64_t* bw_down_kib;
    uint64_t* bw_up_kib;
    int has_ip_attr;
    int32_t* esrc;
    int32_t* edst;
    int64_t* elat_ns;
    double* eloss;
    gml_graph gml; /* owns the attribute strings */
    /* attach state (topology.c:37-42) */
    pthread_rwlock_t ip_lock;
    ipmap_t ipmap;
    uint8_t* attached; /* verticesWithAttachedHosts */
    atomic_int attach_gen; /* bumped whenever a vertex joins the attached set */
    /* tables: one immutable generation per build, published through `tb` (acquire/release);
     * replaced generations stay allocated until topology_free, so a lookup that loaded the
     * previous pointer keeps reading valid memory */
    pthread_mutex_t build_lock;
    _Atomic(struct tables*) tb;
    int build_failed;
    int ngpus;
    uint64_t quantum_ns;
    /* which cached path serves a pair (pairorder.c) */
    srt_pair_order* po;
    /* runahead (topology.c:1253-1264): minimumPathLatency over the stored paths, 0 = none yet */
    pthread_mutex_t min_lock;
    double min_path_ms;
    srt_build_opts opts;
    srt_build_stats stats;
    int32_t builds;       /* table generations built */
    double build_seconds; /* their device time (srt_build_stats.ms_total) */
    /* counters (lock-free) */
    cntmap_t counters;
    /* attach index (built on the first attach) */
    pthread_mutex_t ax_lock;
    void* ax;
};

static int magic_ok(const Topology* t) { return t && t->magic == TOPOLOGY_MAGIC; }

/* One generation of routing tables over a vertex subset: the vertices with attached hosts (the
 * reference computes paths towards those only, topology.c:1604-1656), or every vertex when the
 * build ran before any attach. Entry [i][j] is the pair (verts[i], verts[j]). */
typedef struct tables {
    int32_t nslot;
    int all;            /* every vertex, slot == vertex */
    int32_t* slot_of;   /* n entries: slot of a vertex, -1 when not in the table */
    int32_t* verts;     /* nslot vertices, increasing */
    uint32_t* lat_q;    /* nslot x nslot quanta */
    double* rel;        /* nslot x nslot */
    double* lat_ms;     /* f64 path-order ms (sub-ms edge latencies), else NULL */
    uint32_t min_q;     /* smallest entry (diagonal included) */
    atomic_int checked_gen; /* attach generation this table was last found to cover */
    struct tables* prev;
} tables_t;

/* the n^2 tables: anonymous mappings advised onto huge pages, so the library's threaded download
 * (build.hip table_download) first-touches 2-MB pages instead of faulting 4-KB ones (C3: 13 GB/s
 * into malloc'd tables against 38 GB/s into numpy's huge-page-advised arrays) */
static void* tab_alloc(size_t bytes) {
    void* p = mmap(NULL, bytes ? bytes : 1, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return NULL;
    (void)madvise(p, bytes ? bytes : 1, MADV_HUGEPAGE);
    return p;
}
static void tab_free(void* p, size_t bytes) {
    if (p) munmap(p, bytes ? bytes : 1);
}

static void tables_free_all(tables_t* tb) {
    while (tb) {
        tables_t* p = tb->prev;
        const size_t nn = (size_t)tb->nslot * (size_t)tb->nslot;
        free(tb->slot_of);
        free(tb->verts);
        tab_free(tb->lat_q, nn * sizeof(uint32_t));
        tab_free(tb->rel, nn * sizeof(double));
        tab_free(tb->lat_ms, nn * sizeof(double));
        free(tb);
        tb = p;
    }
}
static void attach_index_free(Topology* t);

/* address_stringToIP (address.c:145-152): network order, INADDR_NONE on failure */
static uint32_t string_to_ip(const char* s) {
    struct in_addr a;
    if (s && inet_pton(AF_INET, s, &a) == 1) return a.s_addr;
    return INADDR_NONE;
}

/* ---- validation (topology.c:525-1038) -------------------------------------------------- */
static int prefix_ci(const char* name, const char* expected) {
    return strncasecmp(name, expected, strlen(expected)) == 0; /* topology.c:184-188 */
}

static int check_type(const gml_attr* a, int want_string) {
    if (a->is_string == want_string) return 1;
    srt_log(SRT_LOG_WARNING, "graph attribute '%s' with type '%s' is supported, but we found "
            "unsupported type '%s'", a->name, want_string ? "STRING" : "NUMERIC",
            a->is_string ? "STRING" : "NUMERIC");
    return 0;
}

static int check_attributes(const gml_graph* g) {
    int ok = 1;
    for (int i = 0; i < g->nva; i++) {
        const gml_attr* a = &g->va[i];
        const char* nm = a->name;
        if (prefix_ci(nm, "id"))
            ok = ok && check_type(a, 0);
        else if (prefix_ci(nm, "ip_address") || prefix_ci(nm, "city_code") ||
                 prefix_ci(nm, "country_code") || prefix_ci(nm, "bandwidth_down") ||
                 prefix_ci(nm, "bandwidth_up") || prefix_ci(nm, "label"))
            ok = ok && check_type(a, 1);
        else {
            srt_log(SRT_LOG_ERROR, "vertex attribute '%s' is unsupported", nm);
            ok = 0;
        }
    }
    static const char* vreq[] = {"id", "bandwidth_down", "bandwidth_up"};
    for (int i = 0; i < 3; i++)
        if (!gml_vattr(g, vreq[i])) {
            srt_log(SRT_LOG_WARNING, "the vertex attribute '%s' is required but not provided",
                    vreq[i]);
            ok = 0;
        }
    for (int i = 0; i < g->nea; i++) {
        const gml_attr* a = &g->ea[i];
        const char* nm = a->name;
        if (prefix_ci(nm, "latency") || prefix_ci(nm, "jitter") || prefix_ci(nm, "label"))
            ok = ok && check_type(a, 1);
        else if (prefix_ci(nm, "packet_loss"))
            ok = ok && check_type(a, 0);
        else {
            srt_log(SRT_LOG_ERROR, "edge attribute '%s' is unsupported", nm);
            ok = 0;
        }
    }
    static const char* ereq[] = {"latency", "packet_loss"};
    for (int i = 0; i < 2; i++)
        if (!gml_eattr(g, ereq[i])) {
            srt_log(SRT_LOG_WARNING, "the edge attribute '%s' is required but not provided",
                    ereq[i]);
            ok = 0;
        }
    return ok;
}

/* BFS reachability over out-arcs (forward) or in-arcs (backward). */
static int32_t reach_count(int32_t n, int64_t m, const int32_t* es, const int32_t* ed, int directed,
                           int backward) {
    int32_t* deg = (int32_t*)calloc((size_t)n + 1, sizeof(int32_t));
    int32_t* adj = (int32_t*)malloc((size_t)(2 * m + 1) * sizeof(int32_t));
    int32_t* q = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    uint8_t* seen = (uint8_t*)calloc((size_t)n, 1);
    if (!deg || !adj || !q || !seen) {
        free(deg);
        free(adj);
        free(q);
        free(seen);
        return -1;
    }
    for (int64_t e = 0; e < m; e++) {
        int32_t a = backward ? ed[e] : es[e], b = backward ? es[e] : ed[e];
        deg[a + 1]++;
        if (!directed) deg[b + 1]++;
    }
    for (int32_t i = 0; i < n; i++) deg[i + 1] += deg[i];
    int32_t* pos = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    if (!pos) {
        free(deg);
        free(adj);
        free(q);
        free(seen);
        return -1;
    }
    memcpy(pos, deg, (size_t)n * sizeof(int32_t));
    for (int64_t e = 0; e < m; e++) {
        int32_t a = backward ? ed[e] : es[e], b = backward ? es[e] : ed[e];
        adj[pos[a]++] = b;
        if (!directed) adj[pos[b]++] = a;
    }
    int32_t head = 0, tail = 0, cnt = 0;
    q[tail++] = 0;
    seen[0] = 1;
    while (head < tail) {
        int32_t u = q[head++];
        cnt++;
        for (int32_t k = deg[u]; k < deg[u + 1]; k++)
            if (!seen[adj[k]]) {
                seen[adj[k]] = 1;
                q[tail++] = adj[k];
            }
    }
    free(deg);
    free(adj);
    free(q);
    free(seen);
    free(pos);
    return cnt;
}

/* _topology_isComplete (topology.c:409-511): every vertex needs >= n incident OUT edges; an
 * undirected self-loop is listed twice by igraph and corrected once (:464-480). */
static int is_complete(const gml_graph* g) {
    int32_t n = g->n;
    int64_t* cnt = (int64_t*)calloc((size_t)n, sizeof(int64_t));
    uint8_t* loop = (uint8_t*)calloc((size_t)n, 1);
    if (!cnt || !loop) {
        free(cnt);
        free(loop);
        return 0;
    }
    for (int64_t e = 0; e < g->m; e++) {
        int32_t a = g->esrc[e], b = g->edst[e];
        cnt[a]++;
        if (!g->directed) cnt[b]++;
        if (a == b) loop[a] = 1;
    }
    int complete = 1;
    for (int32_t v = 0; v < n && complete; v++) {
        int64_t c = cnt[v] - ((!g->directed && loop[v]) ? 1 : 0);
        if (c < n) complete = 0;
    }
    free(cnt);
    free(loop);
    return complete;
}

static int bandwidth_kib(const gml_attr* a, int32_t v, uint64_t* out) {
    /* _topology_findVertexAttributeStringBandwidth (topology.c:210-233) */
    if (!a || !a->is_string) return 0;
    const char* s = a->str[v];
    if (!s || !s[0]) return 0;
    int64_t bw = srt_parse_bandwidth(s);
    if (bw == -2) {
        srt_log(SRT_LOG_ERROR, "bandwidth '%s' overflows (the reference panics here)", s);
        return 0;
    }
    if (bw < 0) return 0;
    *out = (uint64_t)(bw / (8 * 1024));
    return 1;
}

static int edge_time_ns(const gml_attr* a, int64_t e, int64_t* out) {
    /* _topology_findEdgeAttributeStringTimeMs (topology.c:280-302) */
    if (!a || !a->is_string) return 0;
    const char* s = a->str[e];
    if (!s || !s[0]) return 0;
    int64_t ns = srt_parse_time_nanosec(s);
    if (ns == -2) {
        srt_log(SRT_LOG_ERROR, "time '%s' overflows (the reference panics here)", s);
        return 0;
    }
    if (ns < 0) return 0;
    *out = ns;
    return 1;
}

static int validate_and_extract(Topology* t) {
    const gml_graph* g = &t->gml;
    srt_log(SRT_LOG_INFO, "checking graph attributes...");
    if (!check_attributes(g)) {
        srt_log(SRT_LOG_ERROR, "topology validation failed because of problem with graph, vertex, "
                "or edge attributes");
        return 0;
    }
    t->n = g->n;
    t->m = g->m;
    t->directed = g->directed;
    /* strongly connected, one cluster (topology.c:671-713) */
    int connected = g->n > 0;
    if (connected) {
        int32_t f = reach_count(g->n, g->m, g->esrc, g->edst, g->directed, 0);
        connected = (f == g->n);
        if (connected && g->directed) connected = reach_count(g->n, g->m, g->esrc, g->edst, 1, 1) == g->n;
    }
    t->complete = g->n > 0 && is_complete(g);
    if (!t->complete && !t->use_shortest_path) {
        srt_log(SRT_LOG_ERROR, "The 'use_shortest_path' feature is disabled/false, but the graph is "
                "not complete");
        return 0;
    }
    if (!connected) {
        srt_log(SRT_LOG_ERROR, "topology must be strongly connected with a single cluster");
        return 0;
    }
    /* vertices (topology.c:718-890) */
    const gml_attr* aid = gml_vattr(g, "id");
    const gml_attr* adown = gml_vattr(g, "bandwidth_down");
    const gml_attr* aup = gml_vattr(g, "bandwidth_up");
    const gml_attr* aip = gml_vattr(g, "ip_address");
    const gml_attr* acity = gml_vattr(g, "city_code");
    const gml_attr* acountry = gml_vattr(g, "country_code");
    int32_t n = g->n;
    t->vid = (double*)malloc((size_t)n * sizeof(double));
    t->vip = (const char**)malloc((size_t)n * sizeof(char*));
    t->vcity = (const char**)malloc((size_t)n * sizeof(char*));
    t->vcountry = (const char**)malloc((size_t)n * sizeof(char*));
    t->bw_down_kib = (uint64_t*)malloc((size_t)n * sizeof(uint64_t));
    t->bw_up_kib = (uint64_t*)malloc((size_t)n * sizeof(uint64_t));
    t->attached = (uint8_t*)calloc((size_t)n, 1);
    if (!t->vid || !t->vip || !t->vcity || !t->vcountry || !t->bw_down_kib || !t->bw_up_kib ||
        !t->attached)
        return 0;
    t->has_ip_attr = aip && aip->is_string;
    int ok = 1;
    for (int32_t v = 0; v < n; v++) {
        double id = aid->num[v];
        if (isnan(id)) {
            srt_log(SRT_LOG_WARNING, "required attribute 'id' on vertex %d is NULL", v);
            ok = 0;
        }
        t->vid[v] = id;
        if (!(bandwidth_kib(adown, v, &t->bw_down_kib[v]) && t->bw_down_kib[v] > 0)) {
            srt_log(SRT_LOG_WARNING, "required attribute 'bandwidth_down' on vertex %d is NAN or "
                    "negative", v);
            ok = 0;
        }
        if (!(bandwidth_kib(aup, v, &t->bw_up_kib[v]) && t->bw_up_kib[v] > 0)) {
            srt_log(SRT_LOG_WARNING, "required attribute 'bandwidth_up' on vertex %d is NAN or "
                    "negative", v);
            ok = 0;
        }
        t->vip[v] = (aip && aip->is_string) ? aip->str[v] : "";
        t->vcity[v] = (acity && acity->is_string && acity->str[v][0]) ? acity->str[v] : NULL;
        t->vcountry[v] =
            (acountry && acountry->is_string && acountry->str[v][0]) ? acountry->str[v] : NULL;
    }
    if (!ok) {
        srt_log(SRT_LOG_WARNING, "unable to validate graph vertices");
        return 0;
    }
    /* edges (topology.c:892-1038) + weight extraction (:1065-1122) */
    const gml_attr* alat = gml_eattr(g, "latency");
    const gml_attr* aloss = gml_eattr(g, "packet_loss");
    const gml_attr* ajit = gml_eattr(g, "jitter");
    int64_t m = g->m;
    t->esrc = g->esrc;
    t->edst = g->edst;
    t->elat_ns = (int64_t*)malloc((size_t)(m > 0 ? m : 1) * sizeof(int64_t));
    t->eloss = (double*)malloc((size_t)(m > 0 ? m : 1) * sizeof(double));
    if (!t->elat_ns || !t->eloss) return 0;
    for (int64_t e = 0; e < m; e++) {
        int64_t ns = 0;
        if (!(edge_time_ns(alat, e, &ns) && (double)ns / 1000000.0 > 0.0)) {
            srt_log(SRT_LOG_WARNING, "required attribute 'latency' on edge %lld is missing, NAN or "
                    "non-positive", (long long)e);
            ok = 0;
        }
        t->elat_ns[e] = ns;
        double loss = aloss->num ? aloss->num[e] : NAN;
        if (isnan(loss) || !(loss >= 0.0f && loss <= 1.0f)) {
            srt_log(SRT_LOG_WARNING, "required attribute 'packet_loss' on edge %lld is missing, NAN "
                    "or out of range [0.0,1.0]", (long long)e);
            ok = 0;
        }
        t->eloss[e] = loss;
        int64_t jns;
        (void)ajit;
        (void)jns; /* jitter parses to ns >= 0 whenever present, so it can never fail (:956-970) */
    }
    if (!ok) {
        srt_log(SRT_LOG_WARNING, "unable to validate graph edges");
        return 0;
    }
    srt_log(SRT_LOG_INFO, "successfully parsed gml and validated topology: %d vertices, %lld edges, "
            "%s, %s", n, (long long)m, t->directed ? "directed" : "undirected",
            t->complete ? "complete" : "incomplete");
    return 1;
}

static Topology* topology_from_text(const char* text, size_t len, int useShortestPath) {
    Topology* t = (Topology*)calloc(1, sizeof(Topology));
    if (!t) return NULL;
    t->magic = TOPOLOGY_MAGIC;
    t->use_shortest_path = useShortestPath ? 1 : 0;
    pthread_rwlock_init(&t->ip_lock, NULL);
    pthread_mutex_init(&t->build_lock, NULL);
    pthread_mutex_init(&t->ax_lock, NULL);
    pthread_mutex_init(&t->min_lock, NULL);
    atomic_store(&t->tb, NULL);
    atomic_store(&t->attach_gen, 0);
    t->min_path_ms = 0.0;
    t->ngpus = 1;
    t->opts.device = 0;
    t->opts.algo = SRT_ALGO_AUTO;
    char err[512];
    if (gml_parse(text, len, &t->gml, err, sizeof(err))) {
        srt_log(SRT_LOG_ERROR, "GML read failed: %s", err);
        topology_free(t);
        return NULL;
    }
    if (!validate_and_extract(t)) {
        srt_log(SRT_LOG_ERROR, "we failed to create the simulation topology because we were unable "
                "to validate the topology gml file");
        topology_free(t);
        return NULL;
    }
    t->po = srt_pair_order_new(t->n, t->directed, t->use_shortest_path);
    if (!t->po || cnt_init(&t->counters, t->n)) {
        srt_log(SRT_LOG_ERROR, "out of memory for the path order of %d vertices", t->n);
        topology_free(t);
        return NULL;
    }
    return t;
}

Topology* srt_topology_new_from_string(const char* gmlText, int useShortestPath) {
    if (!gmlText) return NULL;
    return topology_from_text(gmlText, strlen(gmlText), useShortestPath);
}

Topology* topology_new(const char* graphPath, int useShortestPath) {
    if (!graphPath) return NULL;
    FILE* f = fopen(graphPath, "rb");
    if (!f) {
        srt_log(SRT_LOG_ERROR, "fopen returned NULL while attempting to open graph file path '%s'",
                graphPath);
        return NULL;
    }
    fseek(f, 0, SEEK_END);
    long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* buf = (char*)malloc((size_t)(len > 0 ? len : 0) + 1);
    if (!buf) {
        fclose(f);
        return NULL;
    }
    size_t got = fread(buf, 1, (size_t)(len > 0 ? len : 0), f);
    fclose(f);
    buf[got] = 0;
    /* the path is not retained: the controller unlinks the temp file (controller.c:173-174) */
    Topology* t = topology_from_text(buf, got, useShortestPath);
    free(buf);
    return t;
}

int srt_topology_path_counts(Topology* t, uint32_t* shortestPathCount, uint32_t* selfPathCount,
                             int32_t* builds, double* buildSeconds) {
    if (!magic_ok(t)) return SRT_E_ARG;
    srt_pair_order_counts(t->po, shortestPathCount, selfPathCount);
    pthread_mutex_lock(&t->build_lock);
    if (builds) *builds = t->builds;
    if (buildSeconds) *buildSeconds = t->build_seconds;
    pthread_mutex_unlock(&t->build_lock);
    return SRT_OK;
}

void topology_free(Topology* t) {
    if (!t) return;
    if (t->po) { /* _topology_clearCache's summary (topology.c:1142-1164) */
        uint32_t sp = 0, self = 0;
        srt_pair_order_counts(t->po, &sp, &self);
        srt_log(SRT_LOG_INFO, "path cache cleared, computed %u shortest paths with dijkstra, and %u "
                "shortest self paths", sp, self);
        srt_log(SRT_LOG_INFO, "routing tables: %d builds, %f seconds of device time", t->builds,
                t->build_seconds);
    }
    free(t->vid);
    free(t->vip);
    free(t->vcity);
    free(t->vcountry);
    free(t->bw_down_kib);
    free(t->bw_up_kib);
    free(t->attached);
    free(t->elat_ns);
    free(t->eloss);
    ipmap_free(&t->ipmap);
    tables_free_all(atomic_load(&t->tb));
    cnt_free(&t->counters);
    gml_free(&t->gml);
    pthread_rwlock_destroy(&t->ip_lock);
    pthread_mutex_destroy(&t->build_lock);
    attach_index_free(t);
    srt_pair_order_free(t->po);
    pthread_mutex_destroy(&t->ax_lock);
    pthread_mutex_destroy(&t->min_lock);
    t->magic = 0;
    free(t);
}

/* ---- attach (topology.c:2024-2272) ----------------------------------------------------- *
 * The reference scans every vertex per host (hook :2024-2100), re-parsing its IP string and
 * comparing hint strings, and then takes the longest prefix match (:2102-2130) or a random
 * candidate (:2188-2196). The outcome depends only on the vertex attributes and the hints, so the
 * attributes are indexed once (lazily, on the first attach) and every attach is O(log n):
 *  - raw vertex IPs (string_to_ip of the attribute, INADDR_NONE when absent), all vertices
 *    sorted by (ip, vertex);
 *  - city and country codes interned case-insensitively (g_ascii_strcasecmp); per code the
 *    vertices in index order (the candidate queue), the count with a usable IP, and the same
 *    vertices sorted by (ip, vertex).
 * Candidate queues are the reference's: an exact usable-IP match keeps only the exact matches
 * (in index order); otherwise city, then country, then all vertices.
 * LPM: match = ~(ip ^ key) is largest where ip ^ key is smallest; XOR with a fixed key is a
 * bijection, so one IP value wins, found by a 32-step bit descent over the sorted queue (see
 * lpm_pick; the nearest neighbours of key in sorted order are not enough: {0x0, 0x7} with key
 * 0x8 is won by 0x0). The reference's update rule (match > best || best == 0) keeps the first
 * candidate with the largest match when that match is > 0, which is the first vertex of the
 * winning IP's (ip, vertex)-sorted run; when every match is 0 it ends on the last candidate of
 * the queue. */
typedef struct {
    uint32_t ip;
    int32_t v;
} ipv_t;

typedef struct {
    char** names;    /* sorted, lowercase, unique */
    int32_t count;
    int32_t* ptr;    /* count + 1 */
    int32_t* list;   /* vertices of each code, index order */
    ipv_t* sorted;   /* the same segments sorted by (ip, vertex) */
    int32_t* usable; /* per code: vertices with a usable IP */
} code_index;

typedef struct {
    uint32_t* vip; /* raw IP per vertex */
    ipv_t* all_sorted;
    int32_t all_usable;
    code_index city, country;
} attach_index;

static int ip_usable(uint32_t ip) {
    /* INADDR_LOOPBACK is host order compared to a network-order value (topology.c:2051) */
    return ip != INADDR_NONE && ip != INADDR_ANY && ip != INADDR_LOOPBACK;
}

static int ipv_cmp(const void* a, const void* b) {
    const ipv_t* x = (const ipv_t*)a;
    const ipv_t* y = (const ipv_t*)b;
    if (x->ip != y->ip) return x->ip < y->ip ? -1 : 1;
    return (x->v > y->v) - (x->v < y->v);
}

static char* lower_dup(const char* s) {
    size_t n = strlen(s);
    char* d = (char*)malloc(n + 1);
    if (!d) return NULL;
    for (size_t i = 0; i <= n; i++) d[i] = (char)tolower((unsigned char)s[i]);
    return d;
}

typedef struct {
    char* key;
    int32_t v;
} keyv_t;

static int keyv_cmp(const void* a, const void* b) {
    const keyv_t* x = (const keyv_t*)a;
    const keyv_t* y = (const keyv_t*)b;
    int c = strcmp(x->key, y->key);
    if (c) return c;
    return (x->v > y->v) - (x->v < y->v);
}

static int code_index_build(code_index* ci, const char** codes, int32_t n, const uint32_t* vip) {
    memset(ci, 0, sizeof(*ci));
    keyv_t* kv = (keyv_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(keyv_t));
    if (!kv) return SRT_E_NOMEM;
    int32_t m = 0;
    for (int32_t v = 0; v < n; v++) {
        if (!codes[v]) continue;
        kv[m].key = lower_dup(codes[v]);
        if (!kv[m].key) {
            for (int32_t q = 0; q < m; q++) free(kv[q].key);
            free(kv);
            return SRT_E_NOMEM;
        }
        kv[m++].v = v;
    }
    qsort(kv, (size_t)m, sizeof(keyv_t), keyv_cmp); /* by code, then vertex index */
    int32_t nc = 0;
    for (int32_t q = 0; q < m; q++)
        if (q == 0 || strcmp(kv[q].key, kv[q - 1].key)) nc++;
    ci->names = (char**)calloc((size_t)(nc > 0 ? nc : 1), sizeof(char*));
    ci->ptr = (int32_t*)calloc((size_t)nc + 1, sizeof(int32_t));
    ci->list = (int32_t*)malloc((size_t)(m > 0 ? m : 1) * sizeof(int32_t));
    ci->sorted = (ipv_t*)malloc((size_t)(m > 0 ? m : 1) * sizeof(ipv_t));
    ci->usable = (int32_t*)calloc((size_t)(nc > 0 ? nc : 1), sizeof(int32_t));
    if (!ci->names || !ci->ptr || !ci->list || !ci->sorted || !ci->usable) {
        for (int32_t q = 0; q < m; q++) free(kv[q].key);
        free(kv);
        return SRT_E_NOMEM;
    }
    int32_t c = -1;
    for (int32_t q = 0; q < m; q++) {
        if (c < 0 || strcmp(kv[q].key, ci->names[c])) { /* duplicates are freed below */
            ci->names[++c] = kv[q].key;
            ci->ptr[c] = q;
        } else {
            free(kv[q].key);
        }
        ci->list[q] = kv[q].v;
        ci->sorted[q].ip = vip[kv[q].v];
        ci->sorted[q].v = kv[q].v;
        ci->usable[c] += ip_usable(vip[kv[q].v]);
    }
    ci->count = nc;
    ci->ptr[nc] = m;
    for (int32_t k = 0; k < nc; k++)
        qsort(ci->sorted + ci->ptr[k], (size_t)(ci->ptr[k + 1] - ci->ptr[k]), sizeof(ipv_t), ipv_cmp);
    free(kv);
    return SRT_OK;
}

static void code_index_free(code_index* ci) {
    for (int32_t k = 0; k < ci->count; k++) free(ci->names[k]);
    free(ci->names);
    free(ci->ptr);
    free(ci->list);
    free(ci->sorted);
    free(ci->usable);
    memset(ci, 0, sizeof(*ci));
}

/* interned id of a hint (case-insensitive), -1 when no vertex carries it */
static int32_t code_lookup(const code_index* ci, const char* hint) {
    if (!hint || ci->count == 0) return -1;
    char* key = lower_dup(hint);
    if (!key) return -1;
    int32_t lo = 0, hi = ci->count - 1, found = -1;
    while (lo <= hi) {
        int32_t mid = lo + (hi - lo) / 2;
        int c = strcmp(ci->names[mid], key);
        if (c == 0) {
            found = mid;
            break;
        }
        if (c < 0) lo = mid + 1;
        else hi = mid - 1;
    }
    free(key);
    return found;
}

/* first position in s[0, len) whose ip is >= key */
static int32_t ipv_lower(const ipv_t* s, int32_t len, uint32_t key) {
    int32_t lo = 0, hi = len;
    while (lo < hi) {
        int32_t mid = lo + (hi - lo) / 2;
        if (s[mid].ip < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/* first position in [lo, hi) whose ip is >= key */
static int32_t ipv_lower_in(const ipv_t* s, int32_t lo, int32_t hi, uint32_t key) {
    while (lo < hi) {
        int32_t mid = lo + (hi - lo) / 2;
        if (s[mid].ip < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/* _topology_getLongestPrefixMatch over one candidate queue: `sorted` is the queue sorted by
 * (ip, vertex), `last` the queue's last vertex in queue order. The smallest ip ^ key is found by
 * descending the bits from the top, as in a binary trie: [lo, hi) holds the IPs that agree with
 * the best choice so far above bit b, ordered so that bit b = 0 comes first; keep the half whose
 * bit b equals key's when it is non-empty. The range ends on one IP value. */
static int32_t lpm_pick(const ipv_t* sorted, int32_t len, int32_t last, uint32_t key) {
    int32_t lo = 0, hi = len;
    for (int b = 31; b >= 0; --b) {
        const uint32_t bit = 1u << b;
        const uint32_t high = b == 31 ? 0u : sorted[lo].ip & ~((bit << 1) - 1u);
        const int32_t split = ipv_lower_in(sorted, lo, hi, high | bit);
        if (key & bit) {
            if (split < hi) lo = split;
        } else {
            if (split > lo) hi = split;
        }
    }
    if (~(sorted[lo].ip ^ key) == 0u) return last; /* every match is 0: the update rule ends on the last */
    return sorted[lo].v; /* the first vertex holding the best IP */
}

static void attach_index_free(Topology* t) {
    attach_index* ax = (attach_index*)t->ax;
    if (!ax) return;
    free(ax->vip);
    free(ax->all_sorted);
    code_index_free(&ax->city);
    code_index_free(&ax->country);
    free(ax);
    t->ax = NULL;
}

static attach_index* attach_index_of(Topology* t) {
    pthread_mutex_lock(&t->ax_lock);
    if (!t->ax) {
        const int32_t n = t->n;
        attach_index* ax = (attach_index*)calloc(1, sizeof(attach_index));
        int ok = ax != NULL;
        if (ok) {
            ax->vip = (uint32_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(uint32_t));
            ax->all_sorted = (ipv_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(ipv_t));
            ok = ax->vip && ax->all_sorted;
        }
        if (ok) {
            for (int32_t v = 0; v < n; v++) {
                const char* ipStr = t->vip[v];
                ax->vip[v] = (ipStr && ipStr[0]) ? string_to_ip(ipStr) : INADDR_NONE;
                ax->all_sorted[v].ip = ax->vip[v];
                ax->all_sorted[v].v = v;
                ax->all_usable += ip_usable(ax->vip[v]);
            }
            qsort(ax->all_sorted, (size_t)n, sizeof(ipv_t), ipv_cmp);
            ok = code_index_build(&ax->city, t->vcity, n, ax->vip) == SRT_OK &&
                 code_index_build(&ax->country, t->vcountry, n, ax->vip) == SRT_OK;
        }
        t->ax = ax;
        if (!ok) attach_index_free(t);
    }
    attach_index* r = (attach_index*)t->ax;
    pthread_mutex_unlock(&t->ax_lock);
    return r;
}

static int32_t find_attachment_vertex(Topology* t, uint32_t* rand_state, Random* rnd,
                                      const char* ipHint, const char* cityHint,
                                      const char* countryHint) {
    attach_index* ax = attach_index_of(t);
    if (!ax) return -1;
    const int32_t n = t->n;
    int requestedIPIsUsable = 0;
    uint32_t requestedIP = 0;
    if (ipHint) {
        uint32_t ip = string_to_ip(ipHint);
        if (ip_usable(ip)) {
            requestedIPIsUsable = 1;
            requestedIP = ip;
        }
    }
    /* candidate queue: `seg` in queue order (NULL: all vertices), `sorted` by (ip, vertex) */
    const int32_t* seg = NULL;
    const ipv_t* sorted = ax->all_sorted;
    int32_t len = n, useLPM = 0, exact = 0;
    if (requestedIPIsUsable) {
        const int32_t a = ipv_lower(ax->all_sorted, n, requestedIP);
        const int32_t b = ipv_lower(ax->all_sorted, n, requestedIP + 1u);
        if (b > a && ax->all_sorted[a].ip == requestedIP) { /* exact matches, index order */
            exact = 1;
            sorted = ax->all_sorted + a;
            len = (requestedIP == 0xFFFFFFFFu ? n : b) - a;
        }
    }
    if (!exact) {
        const int32_t c = code_lookup(&ax->city, cityHint);
        const int32_t k = c < 0 ? code_lookup(&ax->country, countryHint) : -1;
        if (c >= 0) {
            seg = ax->city.list + ax->city.ptr[c];
            sorted = ax->city.sorted + ax->city.ptr[c];
            len = ax->city.ptr[c + 1] - ax->city.ptr[c];
            useLPM = requestedIPIsUsable && ax->city.usable[c] > 0;
        } else if (k >= 0) {
            seg = ax->country.list + ax->country.ptr[k];
            sorted = ax->country.sorted + ax->country.ptr[k];
            len = ax->country.ptr[k + 1] - ax->country.ptr[k];
            useLPM = requestedIPIsUsable && ax->country.usable[k] > 0;
        } else {
            useLPM = ipHint && ax->all_usable > 0; /* the hint's presence, not its usability (:2178) */
        }
    }
    if (len <= 0) return -1;
    if (useLPM) return lpm_pick(sorted, len, seg ? seg[len - 1] : n - 1, requestedIP);
    /* :2188-2196 */
    double u;
    if (rnd)
        u = random_nextDouble(rnd);
    else
        u = (double)rand_r(rand_state) / (double)RAND_MAX; /* random.c:32-43 */
    const int indexRange = len - 1;
    int chosenIndex = (int)round((double)(indexRange * u));
    if (chosenIndex >= len) chosenIndex = len - 1;
    if (exact) return sorted[chosenIndex].v; /* the run is in vertex order */
    return seg ? seg[chosenIndex] : chosenIndex;
}

static int32_t attach_common(Topology* t, uint32_t ipNet, uint32_t* rand_state, Random* rnd,
                             const char* ipHint, const char* cityHint, const char* countryHint,
                             uint64_t* bwDownOut, uint64_t* bwUpOut) {
    if (!magic_ok(t)) return SRT_E_ARG;
    int32_t v = find_attachment_vertex(t, rand_state, rnd, ipHint, cityHint, countryHint);
    if (v < 0) {
        srt_log(SRT_LOG_ERROR, "no attachment vertex found");
        abort(); /* utility_assert(numCandidates > 0), topology.c:2182 */
    }
    pthread_rwlock_wrlock(&t->ip_lock);
    ipmap_put(&t->ipmap, ipNet, v);
    if (!t->attached[v]) {
        t->attached[v] = 1;
        srt_pair_order_attach(t->po, v);
        atomic_fetch_add(&t->attach_gen, 1);
    }
    pthread_rwlock_unlock(&t->ip_lock);
    if (bwUpOut) *bwUpOut = t->bw_up_kib[v];
    if (bwDownOut) *bwDownOut = t->bw_down_kib[v];
    srt_log(SRT_LOG_INFO, "attached address to vertex %d ('%ld') using hints (ip=%s, citycode=%s, "
            "countrycode=%s)", v, (long)t->vid[v], ipHint ? ipHint : "(null)",
            cityHint ? cityHint : "(null)", countryHint ? countryHint : "(null)");
    return v;
}

int32_t srt_topology_attach_ip(Topology* t, uint32_t ipNet, uint32_t* randState, const char* ipHint,
                               const char* citycodeHint, const char* countrycodeHint,
                               uint64_t* bwDownOut, uint64_t* bwUpOut) {
    if (!randState) return SRT_E_ARG;
    return attach_common(t, ipNet, randState, NULL, ipHint, citycodeHint, countrycodeHint,
                         bwDownOut, bwUpOut);
}

/* Batched attach: hosts in order, each exactly as srt_topology_attach_ip
 * would attach it (host h draws from randStates[h] only when its pick is random), with one
 * write-lock for the IP map. Hint arrays may be NULL or hold NULL entries; output arrays may
 * be NULL. Returns the number of hosts attached, or a negative error code for a host without a
 * candidate (the reference asserts, topology.c:2182) -- the hosts before it stay attached. */
int32_t srt_topology_attach_batch_ip(Topology* t, int32_t nhosts, const uint32_t* ipNet,
                                     uint32_t* randStates, const char* const* ipHints,
                                     const char* const* citycodeHints,
                                     const char* const* countrycodeHints, int32_t* outVertex,
                                     uint64_t* bwDownOut, uint64_t* bwUpOut) {
    if (!magic_ok(t) || nhosts < 0 || (nhosts > 0 && (!ipNet || !randStates))) return SRT_E_ARG;
    if (!attach_index_of(t)) return SRT_E_NOMEM;
    int32_t* vs = (int32_t*)malloc((size_t)(nhosts > 0 ? nhosts : 1) * sizeof(int32_t));
    if (!vs) return SRT_E_NOMEM;
    int32_t done = 0, rc = 0;
    for (; done < nhosts; done++) {
        const int32_t v = find_attachment_vertex(
            t, randStates + done, NULL, ipHints ? ipHints[done] : NULL,
            citycodeHints ? citycodeHints[done] : NULL,
            countrycodeHints ? countrycodeHints[done] : NULL);
        if (v < 0) {
            srt_set_error("attach batch: no attachment vertex for host %d", done);
            rc = SRT_E_ARG;
            break;
        }
        vs[done] = v;
    }
    pthread_rwlock_wrlock(&t->ip_lock);
    for (int32_t h = 0; h < done; h++) {
        ipmap_put(&t->ipmap, ipNet[h], vs[h]);
        if (!t->attached[vs[h]]) {
            t->attached[vs[h]] = 1;
            srt_pair_order_attach(t->po, vs[h]);
            atomic_fetch_add(&t->attach_gen, 1);
        }
    }
    pthread_rwlock_unlock(&t->ip_lock);
    for (int32_t h = 0; h < done; h++) {
        if (outVertex) outVertex[h] = vs[h];
        if (bwDownOut) bwDownOut[h] = t->bw_down_kib[vs[h]];
        if (bwUpOut) bwUpOut[h] = t->bw_up_kib[vs[h]];
    }
    free(vs);
    srt_log(SRT_LOG_INFO, "attached %d addresses in one batch", done);
    return rc ? rc : done;
}

void topology_attach(Topology* t, Address* address, Random* randomSourcePool, char* ipHint,
                     char* citycodeHint, char* countrycodeHint, uint64_t* bwDownOut,
                     uint64_t* bwUpOut) {
    attach_common(t, address_toNetworkIP(address), NULL, randomSourcePool, ipHint, citycodeHint,
                  countrycodeHint, bwDownOut, bwUpOut);
}

void srt_topology_detach_ip(Topology* t, uint32_t ipNet) {
    if (!magic_ok(t)) return;
    pthread_rwlock_wrlock(&t->ip_lock);
    ipmap_del(&t->ipmap, ipNet); /* verticesWithAttachedHosts is left as is (:2274-2281) */
    pthread_rwlock_unlock(&t->ip_lock);
}

void topology_detach(Topology* t, Address* address) {
    srt_topology_detach_ip(t, address_toNetworkIP(address));
}

/* tables the IP map holds (current + retired): bounded under attach / detach cycles */
int64_t srt_topology_ipmap_tables(Topology* t) {
    if (!magic_ok(t)) return -1;
    pthread_rwlock_rdlock(&t->ip_lock);
    const int64_t k = (int64_t)ipmap_tables(&t->ipmap);
    pthread_rwlock_unlock(&t->ip_lock);
    return k;
}

/* lock-free (the packet path's two lookups per call, topology.c:1905-1915) */
int32_t srt_topology_vertex_of_ip(Topology* t, uint32_t ipNet) {
    if (!magic_ok(t)) return -1;
    return ipmap_get(&t->ipmap, ipNet);
}

/* ---- build + lookups ------------------------------------------------------------------ */
int srt_topology_edges(Topology* t, srt_edges* out) {
    if (!magic_ok(t) || !out) return SRT_E_ARG;
    out->n = t->n;
    out->directed = t->directed;
    out->m = t->m;
    out->src = t->esrc;
    out->dst = t->edst;
    out->lat_ns = t->elat_ns;
    out->loss = t->eloss;
    return SRT_OK;
}

void srt_topology_set_build_opts(Topology* t, const srt_build_opts* opts) {
    if (magic_ok(t) && opts) t->opts = *opts;
}

int srt_topology_last_stats(Topology* t, srt_build_stats* stats) {
    if (!magic_ok(t) || !stats) return SRT_E_ARG;
    *stats = t->stats;
    return SRT_OK;
}

/* runahead hook: tests (and embedders without Shadow's worker) receive the exported minimum
 * here instead of worker_updateMinTimeJump */
static void (*g_min_hook)(double) = NULL;

void srt_set_min_time_jump_hook(void (*fn)(double)) { g_min_hook = fn; }

static double tables_latency_ms(const Topology* t, const tables_t* tb, size_t i) {
    return tb->lat_ms ? tb->lat_ms[i] : (double)((uint64_t)tb->lat_q[i] * t->quantum_ns) / 1000000.0;
}

/* minimum path latency (ms) over pairs of attached vertices, diagonal included; < 0 if none */
static double attached_min_ms(Topology* t, const tables_t* tb) {
    const int32_t n = t->n;
    int32_t na = 0;
    for (int32_t v = 0; v < n; v++) na += t->attached[v] != 0;
    if (na == 0) return -1.0;
    if (na == tb->nslot && !tb->lat_ms) /* the table is the attached set: the device minimum */
        return (double)((uint64_t)tb->min_q * t->quantum_ns) / 1000000.0;
    double best = -1.0;
    for (int32_t a = 0; a < tb->nslot; a++) {
        if (!t->attached[tb->verts[a]]) continue;
        const size_t row = (size_t)a * tb->nslot;
        for (int32_t b = 0; b < tb->nslot; b++) {
            if (!t->attached[tb->verts[b]]) continue;
            const double ms = tables_latency_ms(t, tb, row + b);
            if (best < 0 || ms < best) best = ms;
        }
    }
    return best;
}

double srt_topology_min_latency_ms(Topology* t) {
    if (!magic_ok(t)) return 0.0;
    const tables_t* tb = atomic_load_explicit(&t->tb, memory_order_acquire);
    if (!tb) return 0.0;
    pthread_rwlock_rdlock(&t->ip_lock);
    const double m = attached_min_ms(t, tb);
    pthread_rwlock_unlock(&t->ip_lock);
    return m < 0 ? 0.0 : m;
}

/* _topology_storePathInCache's minimum (topology.c:1253-1264): a stored path below the minimum so
 * far (or the first one: 0 means none) becomes the minimum and goes to worker_updateMinTimeJump.
 * The reference hands it over once per stored path; here one source run offers the smallest of
 * the paths it stored, which leaves the controller's minimum (controller.c:141-153) the same after
 * every run. A 0-ms path (a vertex without edges) would trip controller.c:144's assertion in the
 * reference; it is logged and not handed over. */
static void offer_min(Topology* t, double ms) {
    pthread_mutex_lock(&t->min_lock);
    if (t->min_path_ms == 0.0 || ms < t->min_path_ms) {
        t->min_path_ms = ms;
        if (ms > 0.0) {
            if (g_min_hook)
                g_min_hook(ms);
            else
                worker_updateMinTimeJump(ms);
        } else {
            srt_log(SRT_LOG_WARNING, "a stored path has latency %g ms: not handed to "
                    "worker_updateMinTimeJump (it requires > 0, controller.c:144)", ms);
        }
    }
    pthread_mutex_unlock(&t->min_lock);
}

typedef struct {
    Topology* t;
    const tables_t* tb;
} store_ctx;

/* srt_pair_store_fn: the paths src -> targets[] a lookup just stored (under the pair order's
 * lock, so runs offer their minima in run order) */
static void on_paths_stored(void* vctx, int32_t src, const int32_t* targets, int32_t count) {
    const store_ctx* c = (const store_ctx*)vctx;
    const int32_t a = c->tb->slot_of[src];
    if (a < 0) return;
    double best = -1.0;
    for (int32_t i = 0; i < count; i++) {
        const int32_t b = c->tb->slot_of[targets[i]];
        if (b < 0) continue; /* attached after this table was built (a concurrent attach) */
        const double ms = tables_latency_ms(c->t, c->tb, (size_t)a * c->tb->nslot + b);
        if (best < 0.0 || ms < best) best = ms;
    }
    if (best >= 0.0) offer_min(c->t, best);
}

static int tables_cover_attached(const Topology* t, const tables_t* tb) {
    if (!tb) return 0;
    if (tb->all) return 1;
    for (int32_t v = 0; v < t->n; v++)
        if (t->attached[v] && tb->slot_of[v] < 0) return 0;
    return 1;
}

/* Build a new generation over the attached vertices (every vertex when none is attached yet).
 * Caller holds build_lock. */
static int build_generation(Topology* t, int nGPUs) {
    const int32_t n = t->n;
    tables_t* tb = (tables_t*)calloc(1, sizeof(tables_t));
    if (!tb) return SRT_E_NOMEM;
    tb->slot_of = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    tb->verts = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    if (!tb->slot_of || !tb->verts) {
        tables_free_all(tb);
        return SRT_E_NOMEM;
    }
    pthread_rwlock_rdlock(&t->ip_lock);
    int32_t k = 0;
    for (int32_t v = 0; v < n; v++) {
        tb->slot_of[v] = t->attached[v] ? k : -1;
        if (t->attached[v]) tb->verts[k++] = v;
    }
    atomic_store(&tb->checked_gen, atomic_load(&t->attach_gen));
    pthread_rwlock_unlock(&t->ip_lock);
    if (k == 0 || k == n) { /* nothing attached yet, or everything: the full table */
        tb->all = 1;
        for (int32_t v = 0; v < n; v++) {
            tb->slot_of[v] = v;
            tb->verts[v] = v;
        }
        k = n;
    }
    tb->nslot = k;
    srt_edges e;
    srt_topology_edges(t, &e);
    uint64_t q = 0;
    uint32_t mx = 0;
    int rc = srt_latency_quantum(&e, &q, &mx);
    if (rc) {
        tables_free_all(tb);
        return rc;
    }
    const size_t nn = (size_t)k * (size_t)k;
    tb->lat_q = (uint32_t*)tab_alloc(nn * sizeof(uint32_t));
    tb->rel = (double*)tab_alloc(nn * sizeof(double));
    /* whole-ms edges: f64 ms sums are exact integers, lat_q * q / 1e6 is the reference's value */
    if (q % 1000000u) tb->lat_ms = (double*)tab_alloc(nn * sizeof(double));
    if (!tb->lat_q || !tb->rel || ((q % 1000000u) && !tb->lat_ms)) {
        tables_free_all(tb);
        return SRT_E_NOMEM;
    }
    srt_build_opts o = t->opts;
    o.use_shortest_path = t->use_shortest_path;
    /* nGPUs > 1: one host thread per GPU of this process, RCCL between them */
    rc = srt_build_tables_subset(&e, &o, nGPUs > 1 ? nGPUs : 1, k, tb->all ? NULL : tb->verts,
                                 tb->lat_q, &t->quantum_ns, tb->rel, tb->lat_ms, &tb->min_q,
                                 &t->stats);
    if (rc) {
        tables_free_all(tb);
        return rc;
    }
    tb->prev = atomic_load(&t->tb);
    atomic_store_explicit(&t->tb, tb, memory_order_release);
    t->builds++;
    t->build_seconds += t->stats.ms_total * 1e-3;
    srt_log(SRT_LOG_INFO, "routing tables built over %d of %d vertices (%s)", k, n,
            tb->all ? "all" : "attached");
    return SRT_OK;
}

/* tables covering every attached vertex; builds (lazily, like _topology_getPathEntry's cache miss
 * at topology.c:1923-1961) when there are none or an attach added a vertex since */
static const tables_t* ensure_tables(Topology* t, int nGPUs) {
    const tables_t* tb = atomic_load_explicit(&t->tb, memory_order_acquire);
    pthread_mutex_lock(&t->build_lock);
    tb = atomic_load_explicit(&t->tb, memory_order_acquire);
    pthread_rwlock_rdlock(&t->ip_lock);
    const int ok = tables_cover_attached(t, tb);
    if (ok) atomic_store(&((tables_t*)tb)->checked_gen, atomic_load(&t->attach_gen));
    pthread_rwlock_unlock(&t->ip_lock);
    if (!ok && !t->build_failed) {
        const int rc = build_generation(t, nGPUs);
        if (rc) {
            t->build_failed = 1;
            srt_log(SRT_LOG_ERROR, "routing table build failed (%d): %s", rc, srt_last_error());
        }
        tb = atomic_load_explicit(&t->tb, memory_order_acquire);
    }
    pthread_mutex_unlock(&t->build_lock);
    return t->build_failed ? NULL : tb;
}

int topology_computeShortestPaths(Topology* t, int nGPUs) {
    if (!magic_ok(t)) return SRT_E_ARG;
    t->ngpus = nGPUs > 1 ? nGPUs : 1;
    if (!ensure_tables(t, t->ngpus)) return t->build_failed ? SRT_E_DEVICE : SRT_E_NOMEM;
    return SRT_OK;
}

int topology_getTable(Topology* t, const uint32_t** latQ, uint64_t* quantumNs, const double** rel,
                      int* n) {
    if (!magic_ok(t)) return SRT_E_ARG;
    int rc = topology_computeShortestPaths(t, t->ngpus);
    if (rc) return rc;
    const tables_t* tb = atomic_load_explicit(&t->tb, memory_order_acquire);
    if (latQ) *latQ = tb->lat_q;
    if (quantumNs) *quantumNs = t->quantum_ns;
    if (rel) *rel = tb->rel;
    if (n) *n = tb->nslot;
    return SRT_OK;
}

int srt_topology_table_info(Topology* t, const int32_t** verts, int32_t* nslot, const double** latMs) {
    if (!magic_ok(t)) return SRT_E_ARG;
    const tables_t* tb = atomic_load_explicit(&t->tb, memory_order_acquire);
    if (!tb) return SRT_E_ARG;
    if (verts) *verts = tb->verts;
    if (nslot) *nslot = tb->nslot;
    if (latMs) *latMs = tb->lat_ms;
    return SRT_OK;
}

/* _topology_getPathEntry (topology.c:1900-1981): the tables holding the pair, the index of the
 * path it is served from (row of the path's source) and that path's ends (*sv = its source, *dv =
 * the other end), or NULL with *err set. */
static const tables_t* path_entry(Topology* t, uint32_t srcIp, uint32_t dstIp, size_t* idx,
                                  int32_t* sv, int32_t* dv, int* err) {
    int32_t s = srt_topology_vertex_of_ip(t, srcIp);
    if (s < 0) {
        srt_log(SRT_LOG_ERROR, "source address is not connected to topology");
        *err = SRT_E_UNATTACHED;
        return NULL;
    }
    int32_t d = srt_topology_vertex_of_ip(t, dstIp);
    if (d < 0) {
        srt_log(SRT_LOG_ERROR, "destination address is not connected to topology");
        *err = SRT_E_UNATTACHED;
        return NULL;
    }
    /* a miss stores paths to every attached vertex (topology.c:1604), so the tables must cover
     * every vertex attached so far, not only s and d */
    const tables_t* tb = atomic_load_explicit(&t->tb, memory_order_acquire);
    if (!tb || atomic_load_explicit(&tb->checked_gen, memory_order_relaxed) !=
                   atomic_load_explicit(&t->attach_gen, memory_order_relaxed)) {
        tb = ensure_tables(t, t->ngpus);
        if (!tb || tb->slot_of[s] < 0 || tb->slot_of[d] < 0) {
            srt_log(SRT_LOG_ERROR, "unable to find path between vertex %d and vertex %d", s, d);
            abort(); /* utility_panic (topology.c:1970-1976) */
        }
    }
    store_ctx ctx = {t, tb};
    const int32_t from = srt_pair_order_lookup(t->po, s, d, on_paths_stored, &ctx);
    if (from < 0) {
        srt_log(SRT_LOG_ERROR, "unable to find path between vertex %d and vertex %d (%d)", s, d, from);
        abort(); /* utility_panic (topology.c:1970-1976) */
    }
    const int32_t to = from == s ? d : s;
    *idx = (size_t)tb->slot_of[from] * tb->nslot + tb->slot_of[to];
    if (sv) *sv = from;
    if (dv) *dv = to;
    return tb;
}

double srt_topology_latency_ip(Topology* t, uint32_t srcIp, uint32_t dstIp) {
    if (!magic_ok(t)) return -1.0;
    size_t i;
    int err;
    const tables_t* tb = path_entry(t, srcIp, dstIp, &i, NULL, NULL, &err);
    if (!tb) return -1.0;
    return tables_latency_ms(t, tb, i);
}

double srt_topology_reliability_ip(Topology* t, uint32_t srcIp, uint32_t dstIp) {
    if (!magic_ok(t)) return -1.0;
    size_t i;
    int err;
    const tables_t* tb = path_entry(t, srcIp, dstIp, &i, NULL, NULL, &err);
    if (!tb) return -1.0;
    return tb->rel[i];
}

/* the served Path (source, target) -- path_incrementPacketCount on the cached object (:1983-1993);
 * a pair has one Path whichever direction is looked up */
static int increment_pair(Topology* t, int32_t from, int32_t to) {
    _Atomic uint64_t* c = cnt_slot(&t->counters, from, to, 1);
    if (!c) return SRT_E_NOMEM;
    atomic_fetch_add_explicit(c, 1, memory_order_relaxed);
    return SRT_OK;
}

int srt_topology_increment_ip(Topology* t, uint32_t srcIp, uint32_t dstIp) {
    if (!magic_ok(t)) return SRT_E_ARG;
    size_t i;
    int32_t s, d;
    int err;
    if (!path_entry(t, srcIp, dstIp, &i, &s, &d, &err)) return err;
    return increment_pair(t, s, d);
}

int32_t srt_topology_path_source_ip(Topology* t, uint32_t srcIp, uint32_t dstIp) {
    if (!magic_ok(t)) return -1;
    const int32_t s = srt_topology_vertex_of_ip(t, srcIp), d = srt_topology_vertex_of_ip(t, dstIp);
    if (s < 0 || d < 0) return -1;
    const int32_t from = srt_pair_order_peek(t->po, s, d);
    return from < 0 ? -1 : from;
}

uint64_t srt_topology_packet_count_ip(Topology* t, uint32_t srcIp, uint32_t dstIp) {
    if (!magic_ok(t)) return 0;
    const int32_t s = srt_topology_vertex_of_ip(t, srcIp), d = srt_topology_vertex_of_ip(t, dstIp);
    if (s < 0 || d < 0) return 0;
    const int32_t from = srt_pair_order_peek(t->po, s, d);
    if (from < 0) return 0;
    _Atomic uint64_t* c = cnt_slot(&t->counters, from, from == s ? d : s, 0);
    return c ? atomic_load_explicit(c, memory_order_relaxed) : 0;
}

/* worker_sendPacket (/root/reference/src/main/core/worker.c:541-555): the fate of one packet on
 * the path src -> dst. Delivered when bootstrapping, when chance <= reliability (:548) or when
 * the payload is empty; then *delayNs = (u64)ceil(latency_ms * SIMTIME_ONE_MILLISECOND) (:550-551)
 * and the pair's packet counter is incremented (:554). Returns 1 delivered, 0 dropped, or a
 * negative SRT_E_* code. `chance` is the caller's random_nextDouble(host random) draw (:543). */
int srt_topology_send_packet_ip(Topology* t, uint32_t srcIp, uint32_t dstIp, double chance,
                                int bootstrapping, uint64_t payloadLength, uint64_t* delayNs) {
    if (!magic_ok(t)) return SRT_E_ARG;
    size_t i;
    int32_t s, d;
    int err;
    const tables_t* tb = path_entry(t, srcIp, dstIp, &i, &s, &d, &err);
    if (!tb) return err;
    const double reliability = tb->rel[i];
    if (bootstrapping || chance <= reliability || payloadLength == 0) {
        /* the reference's getLatency and incrementPathPacketCounter probe the cache again: on a
         * directed graph served d's path, each runs source s once more (its diagnostics count) */
        if (t->directed && s != d && s != srt_topology_vertex_of_ip(t, srcIp)) /* (s: the path's) */
            srt_pair_order_add_source_runs(t->po, 2u);
        const double latency = tables_latency_ms(t, tb, i);
        if (delayNs) *delayNs = (uint64_t)ceil(latency * 1000000.0);
        const int rc = increment_pair(t, s, d);
        return rc ? rc : 1;
    }
    return 0;
}

/* srt_topology_send_packet_ip over a trace of `count` packets (one lookup per packet, no locks
 * but the counter's). delivered[k] = 1/0; delay[k] is written for delivered packets. Returns
 * SRT_OK or the first negative code (stopping there). */
int srt_topology_send_packets_ip(Topology* t, int64_t count, const uint32_t* srcIp,
                                 const uint32_t* dstIp, const double* chance,
                                 const uint8_t* bootstrapping, const uint64_t* payloadLength,
                                 uint8_t* delivered, uint64_t* delayNs) {
    if (!magic_ok(t) || count < 0 || (count && (!srcIp || !dstIp || !chance || !delivered)))
        return SRT_E_ARG;
    for (int64_t k = 0; k < count; k++) {
        const int r = srt_topology_send_packet_ip(t, srcIp[k], dstIp[k], chance[k],
                                                  bootstrapping ? bootstrapping[k] : 0,
                                                  payloadLength ? payloadLength[k] : 1,
                                                  delayNs ? delayNs + k : NULL);
        if (r < 0) return r;
        delivered[k] = (uint8_t)r;
    }
    return SRT_OK;
}

double topology_getLatency(Topology* t, Address* src, Address* dst) {
    return srt_topology_latency_ip(t, address_toNetworkIP(src), address_toNetworkIP(dst));
}

double topology_getReliability(Topology* t, Address* src, Address* dst) {
    return srt_topology_reliability_ip(t, address_toNetworkIP(src), address_toNetworkIP(dst));
}

int topology_isRoutable(Topology* t, Address* src, Address* dst) {
    return topology_getLatency(t, src, dst) > -1 ? 1 : 0; /* topology.c:2019-2022 */
}

void topology_incrementPathPacketCounter(Topology* t, Address* src, Address* dst) {
    if (srt_topology_increment_ip(t, address_toNetworkIP(src), address_toNetworkIP(dst))) {
        srt_log(SRT_LOG_ERROR, "unable to find path between nodes");
        abort(); /* utility_panic (topology.c:1990) */
    }
}

int32_t srt_topology_vertex_count(Topology* t) { return magic_ok(t) ? t->n : -1; }
int64_t srt_topology_edge_count(Topology* t) { return magic_ok(t) ? t->m : -1; }
int srt_topology_is_directed(Topology* t) { return magic_ok(t) ? t->directed : -1; }
int srt_topology_is_complete(Topology* t) { return magic_ok(t) ? t->complete : -1; }
