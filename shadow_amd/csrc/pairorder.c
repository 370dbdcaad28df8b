/*
 * pairorder.c -- which cached path the reference serves for a vertex pair.
 *
 * Restates the lazy path cache of /root/reference/src/main/routing/topology.c over tables that
 * hold every source's raw row:
 *   - a lookup (s, t) checks the cache for (s, t), and for (t, s) unless the graph is directed
 *     (_topology_getPathEntry, :1917-1921);
 *   - a miss computes source s for every attached target (_topology_computeSourcePaths,
 *     :1578-1814; targets = verticesWithAttachedHosts at that moment, :1604) or, with
 *     use_shortest_path = false, the one direct edge s -> t (_topology_lookupDirectPath,
 *     :1816-1858); the self pair takes _topology_computeShortestPathToSelf (:1597-1599);
 *   - a path (x, y) is stored only if neither (x, y) nor (y, x) is cached
 *     (_topology_shouldStorePath, :1194-1199), and the lookup after the miss falls back to
 *     (t, s) for any graph (:1963-1967).
 * So the first source computed for a pair (with the other end attached) serves it for good, in
 * both directions, with its own row's latency and reliability: a directed lookup (s, t) whose
 * pair t computed first returns the t -> s path (and still runs source s, :1919).
 *
 * Model: per vertex, the sequence numbers of its source runs, one per attach epoch (the attached
 * set only grows: topology_detach leaves verticesWithAttachedHosts alone, :2274-2281; a second
 * run in the same epoch stores nothing new). The pair {x, y} is stored by the earliest run of x
 * or y made while both were attached. Reads are lock-free (a seqlock over the per-vertex run
 * lists); runs are recorded under a mutex. Direct mode keeps two bits per unordered pair (stored,
 * and which end stored it), set by compare-and-swap.
 *
 * Unreachable targets: a source run stores only the targets it reaches -- igraph returns an empty
 * path for the others and the store loop skips it (:1744-1753). With a reachability predicate
 * (srt_pair_order_set_reach), a run of x decides {x, y} only when x reaches y, so on a directed
 * graph that is not strongly connected the pair is stored by the first run from an end that
 * reaches the other; a pair neither end reaches is never stored (SRT_E_NOPATH, the reference's
 * panic at :1970-1976). Without a predicate every pair is reachable, which topology_new guarantees
 * (it refuses graphs that are not strongly connected, :674).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "srt_internal.h"

typedef struct {
    int32_t epoch; /* attach epoch of the run */
    int32_t pad;
    int64_t seq;   /* global order of runs */
} po_run;

/* A vertex's runs, appended in place: an entry is written before the count that publishes it, and
 * never changes after. A full list is copied into one of twice the capacity and the old one
 * retired, so a vertex's lists total O(runs) memory. */
typedef struct {
    _Atomic int32_t count;
    int32_t cap;
    po_run r[];
} po_list;

struct srt_pair_order {
    int32_t n, directed, per_source;
    pthread_mutex_t mu;
    atomic_uint_fast64_t version; /* seqlock: odd while a run list is being replaced */
    int64_t next_seq;
    atomic_int epoch;           /* bumped when the attached set grows */
    _Atomic int32_t* att_epoch; /* epoch from which v is attached; INT32_MAX = never */
    int32_t* att_list;          /* attached vertices, in attach order */
    int32_t natt;
    _Atomic(po_list*)* runs; /* per-source mode */
    po_list** retired;       /* replaced lists: lock-free readers may still hold them */
    size_t nretired, cap_retired;
    int32_t* scratch;            /* targets stored by one run */
    atomic_uchar* self_done;     /* (v, v) stored */
    _Atomic uint64_t* pairbits;  /* direct mode: 2 bits per unordered pair {a < b} */
    srt_pair_reach_fn reach;     /* NULL: every pair reachable */
    void* reach_ctx;
    /* the reference's diagnostics (topology.c:78-79): lookups that miss its cache and run a
     * source (shortestPathCount, :1719) or the self path (selfPathCount, :1536) */
    atomic_uint source_runs, self_runs;
};

void srt_pair_order_set_reach(srt_pair_order* po, srt_pair_reach_fn fn, void* ctx) {
    if (!po) return;
    po->reach = fn;
    po->reach_ctx = ctx;
}

static int reaches(const srt_pair_order* po, int32_t s, int32_t t) {
    return !po->reach || po->reach(po->reach_ctx, s, t);
}

srt_pair_order* srt_pair_order_new(int32_t n, int32_t directed, int32_t per_source) {
    if (n <= 0) return NULL;
    srt_pair_order* po = (srt_pair_order*)calloc(1, sizeof(*po));
    if (!po) return NULL;
    po->n = n;
    po->directed = directed ? 1 : 0;
    po->per_source = per_source ? 1 : 0;
    pthread_mutex_init(&po->mu, NULL);
    atomic_init(&po->version, 0);
    atomic_init(&po->epoch, 0);
    po->att_epoch = (_Atomic int32_t*)malloc((size_t)n * sizeof(*po->att_epoch));
    po->att_list = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    po->self_done = (atomic_uchar*)calloc((size_t)n, sizeof(atomic_uchar));
    int ok = po->att_epoch && po->att_list && po->self_done;
    if (ok && po->per_source) {
        po->runs = (_Atomic(po_list*)*)calloc((size_t)n, sizeof(*po->runs));
        po->scratch = (int32_t*)malloc((size_t)n * sizeof(int32_t));
        ok = po->runs && po->scratch;
    } else if (ok) {
        /* n (n - 1) / 2 pairs, 32 per word; calloc'd pages stay untouched until used */
        const uint64_t pairs = (uint64_t)n * (uint64_t)(n - 1) / 2;
        po->pairbits = (_Atomic uint64_t*)calloc((size_t)(pairs / 32 + 1), sizeof(uint64_t));
        ok = po->pairbits != NULL;
    }
    if (!ok) {
        srt_pair_order_free(po);
        return NULL;
    }
    for (int32_t v = 0; v < n; v++) atomic_init(&po->att_epoch[v], INT32_MAX);
    return po;
}

void srt_pair_order_free(srt_pair_order* po) {
    if (!po) return;
    if (po->runs)
        for (int32_t v = 0; v < po->n; v++) free(atomic_load(&po->runs[v]));
    for (size_t i = 0; i < po->nretired; i++) free(po->retired[i]);
    free(po->retired);
    free(po->runs);
    free(po->scratch);
    free((void*)po->att_epoch);
    free(po->att_list);
    free((void*)po->self_done);
    free((void*)po->pairbits);
    pthread_mutex_destroy(&po->mu);
    free(po);
}

int srt_pair_order_attach(srt_pair_order* po, int32_t v) {
    if (!po || v < 0 || v >= po->n) return SRT_E_ARG;
    pthread_mutex_lock(&po->mu);
    if (atomic_load_explicit(&po->att_epoch[v], memory_order_relaxed) == INT32_MAX) {
        const int e = atomic_load_explicit(&po->epoch, memory_order_relaxed) + 1;
        atomic_store_explicit(&po->epoch, e, memory_order_release);
        atomic_store_explicit(&po->att_epoch[v], e, memory_order_release);
        po->att_list[po->natt++] = v;
    }
    pthread_mutex_unlock(&po->mu);
    return SRT_OK;
}

/* seq of the first run in L made while both ends were attached (epoch >= a), or INT64_MAX */
static int64_t valid_run(const po_list* L, int32_t a) {
    if (!L) return INT64_MAX;
    const int32_t cnt = atomic_load_explicit(&((po_list*)L)->count, memory_order_acquire);
    for (int32_t i = 0; i < cnt; i++)
        if (L->r[i].epoch >= a) return L->r[i].seq;
    return INT64_MAX;
}

static int32_t att_of(const srt_pair_order* po, int32_t v) {
    return atomic_load_explicit(&po->att_epoch[v], memory_order_acquire);
}

/* per-source mode: the end whose run stored {x, y} (-1: not stored yet); a run stores the pair
 * only if its source reaches the other end */
static int32_t stored_from_raw(const srt_pair_order* po, int32_t x, int32_t y) {
    const int32_t ax = att_of(po, x), ay = att_of(po, y);
    const int32_t a = ax > ay ? ax : ay;
    const int64_t sx = reaches(po, x, y)
                           ? valid_run(atomic_load_explicit(&po->runs[x], memory_order_acquire), a)
                           : INT64_MAX;
    const int64_t sy = reaches(po, y, x)
                           ? valid_run(atomic_load_explicit(&po->runs[y], memory_order_acquire), a)
                           : INT64_MAX;
    if (sx == INT64_MAX && sy == INT64_MAX) return -1;
    return sx < sy ? x : y;
}

/* the same, as one consistent snapshot of both run lists */
static int32_t stored_from(srt_pair_order* po, int32_t x, int32_t y) {
    for (;;) {
        const uint64_t v1 = atomic_load_explicit(&po->version, memory_order_acquire);
        if (v1 & 1u) {
            sched_yield();
            continue;
        }
        const int32_t f = stored_from_raw(po, x, y);
        atomic_thread_fence(memory_order_acquire);
        if (atomic_load_explicit(&po->version, memory_order_relaxed) == v1) return f;
    }
}

static int32_t last_epoch(const srt_pair_order* po, int32_t v) {
    po_list* L = atomic_load_explicit(&po->runs[v], memory_order_acquire);
    const int32_t cnt = L ? atomic_load_explicit(&L->count, memory_order_acquire) : 0;
    return cnt ? L->r[cnt - 1].epoch : -1;
}

/* Record a source run of x in the current epoch and list the targets it stores (caller holds
 * mu). Returns the number of stored targets (in po->scratch), or a negative error. */
static int32_t record_run(srt_pair_order* po, int32_t x) {
    const int32_t e = atomic_load_explicit(&po->epoch, memory_order_acquire);
    po_list* old = atomic_load_explicit(&po->runs[x], memory_order_relaxed);
    const int32_t cnt = old ? atomic_load_explicit(&old->count, memory_order_relaxed) : 0;
    po_list* L = old;
    if (!old || cnt == old->cap) { /* grow: a copy with twice the capacity */
        const int32_t cap = cnt ? 2 * cnt : 4;
        L = (po_list*)malloc(sizeof(po_list) + (size_t)cap * sizeof(po_run));
        if (!L) return SRT_E_NOMEM;
        if (old && po->nretired == po->cap_retired) {
            const size_t nc = po->cap_retired ? 2 * po->cap_retired : 64;
            po_list** nr = (po_list**)realloc(po->retired, nc * sizeof(po_list*));
            if (!nr) {
                free(L);
                return SRT_E_NOMEM;
            }
            po->retired = nr;
            po->cap_retired = nc;
        }
        L->cap = cap;
        if (cnt) memcpy(L->r, old->r, (size_t)cnt * sizeof(po_run));
        atomic_init(&L->count, cnt);
    }
    const int64_t seq = ++po->next_seq;
    L->r[cnt].epoch = e;
    L->r[cnt].pad = 0;
    L->r[cnt].seq = seq;
    /* seqlock write: readers retry across the publication */
    atomic_fetch_add_explicit(&po->version, 1, memory_order_relaxed);
    atomic_thread_fence(memory_order_release);
    if (L != old) atomic_store_explicit(&po->runs[x], L, memory_order_release);
    atomic_store_explicit(&L->count, cnt + 1, memory_order_release);
    atomic_fetch_add_explicit(&po->version, 1, memory_order_release);
    if (old && L != old) po->retired[po->nretired++] = old;
    /* targets stored by this run: attached y != x, reached from x, whose pair this run decides */
    int32_t k = 0;
    for (int32_t i = 0; i < po->natt; i++) {
        const int32_t y = po->att_list[i];
        if (y == x || !reaches(po, x, y)) continue;
        const int32_t ay = att_of(po, y), ax = att_of(po, x);
        const int32_t a = ax > ay ? ax : ay;
        if (valid_run(L, a) != seq) continue; /* stored by an earlier run of x, or y not attached */
        if (reaches(po, y, x) &&
            valid_run(atomic_load_explicit(&po->runs[y], memory_order_relaxed), a) < seq)
            continue;
        po->scratch[k++] = y;
    }
    return k;
}

static void pair_index(int32_t s, int32_t t, size_t* word, unsigned* shift, int32_t* lo, int32_t* hi) {
    const int32_t a = s < t ? s : t, b = s < t ? t : s;
    const uint64_t idx = (uint64_t)b * (uint64_t)(b - 1) / 2 + (uint64_t)a;
    *word = (size_t)(idx / 32);
    *shift = (unsigned)(2 * (idx % 32));
    *lo = a;
    *hi = b;
}

int32_t srt_pair_order_lookup(srt_pair_order* po, int32_t s, int32_t t, srt_pair_store_fn on_store,
                              void* ctx) {
    if (!po || s < 0 || t < 0 || s >= po->n || t >= po->n) return SRT_E_ARG;
    if (att_of(po, s) == INT32_MAX || att_of(po, t) == INT32_MAX) return SRT_E_UNATTACHED;
    if (s == t) { /* (s, s): the self path, stored on its first lookup (:1597-1599, :1573) */
        if (!atomic_exchange_explicit(&po->self_done[s], 1, memory_order_acq_rel)) {
            if (po->per_source) /* direct mode takes the self-loop edge, uncounted (:1816) */
                atomic_fetch_add_explicit(&po->self_runs, 1u, memory_order_relaxed);
            if (on_store) on_store(ctx, s, &s, 1);
        }
        return s;
    }
    if (!po->per_source) { /* direct mode: the pair itself (:1816-1858) */
        size_t w;
        unsigned sh;
        int32_t lo, hi;
        pair_index(s, t, &w, &sh, &lo, &hi);
        uint64_t old = atomic_load_explicit(&po->pairbits[w], memory_order_acquire);
        for (;;) {
            const uint64_t bits = (old >> sh) & 3u;
            if (bits & 1u) return (bits & 2u) ? hi : lo;
            const uint64_t want = 1u | (s == hi ? 2u : 0u);
            if (atomic_compare_exchange_weak_explicit(&po->pairbits[w], &old, old | (want << sh),
                                                      memory_order_acq_rel, memory_order_acquire)) {
                if (on_store) on_store(ctx, s, &t, 1);
                return s;
            }
        }
    }
    int32_t f = stored_from(po, s, t);
    if (f == s) return s;
    /* directed: the reference's cache probe is (s, t) only (:1917-1921), so every lookup not
     * served s's own path runs source s again (:1923-1961), storing nothing new after the first
     * run of an attach epoch */
    if (po->directed) atomic_fetch_add_explicit(&po->source_runs, 1u, memory_order_relaxed);
    if (f == t && (!po->directed || last_epoch(po, s) == atomic_load(&po->epoch))) return t;
    /* a miss: source s runs (undirected: the pair is not stored; directed: (s, t) is not, and s
     * has not run since the attached set last grew) */
    pthread_mutex_lock(&po->mu);
    f = stored_from_raw(po, s, t);
    const int run = po->directed ? (f != s && last_epoch(po, s) != atomic_load(&po->epoch)) : f < 0;
    if (run && !po->directed) atomic_fetch_add_explicit(&po->source_runs, 1u, memory_order_relaxed);
    if (run) {
        const int32_t k = record_run(po, s);
        if (k < 0) {
            pthread_mutex_unlock(&po->mu);
            return k;
        }
        if (on_store && k > 0) on_store(ctx, s, po->scratch, k);
        f = stored_from_raw(po, s, t);
    }
    pthread_mutex_unlock(&po->mu);
    return f < 0 ? SRT_E_NOPATH : f; /* neither end reaches the other (:1970-1976) */
}

int32_t srt_pair_order_peek(srt_pair_order* po, int32_t s, int32_t t) {
    if (!po || s < 0 || t < 0 || s >= po->n || t >= po->n) return SRT_E_ARG;
    if (s == t) return atomic_load(&po->self_done[s]) ? s : -1;
    if (!po->per_source) {
        size_t w;
        unsigned sh;
        int32_t lo, hi;
        pair_index(s, t, &w, &sh, &lo, &hi);
        const uint64_t bits = (atomic_load(&po->pairbits[w]) >> sh) & 3u;
        return (bits & 1u) ? ((bits & 2u) ? hi : lo) : -1;
    }
    return stored_from(po, s, t);
}

void srt_pair_order_add_source_runs(srt_pair_order* po, uint32_t k) {
    if (po && po->per_source) atomic_fetch_add_explicit(&po->source_runs, k, memory_order_relaxed);
}

void srt_pair_order_counts(srt_pair_order* po, uint32_t* source_runs, uint32_t* self_paths) {
    if (source_runs) *source_runs = po ? atomic_load(&po->source_runs) : 0u;
    if (self_paths) *self_paths = po ? atomic_load(&po->self_runs) : 0u;
}

int32_t srt_pair_order_runs(srt_pair_order* po, int32_t v) {
    if (!po || v < 0 || v >= po->n || !po->per_source) return 0;
    po_list* L = atomic_load(&po->runs[v]);
    return L ? atomic_load(&L->count) : 0;
}
