/*
 * gml.c -- single-pass GML subset reader (see gml.h for the igraph semantics it restates).
 */
#define _GNU_SOURCE
#include "gml.h"

#include <math.h>
#include <pthread.h>
#include <unistd.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int attr;
    int is_str;
    double num;
    size_t str; /* offset into pool */
} kv_t;

typedef struct {
    char** names;
    int* is_string;
    int count, cap;
} attr_tab;

typedef struct {
    const char* p;
    const char* end;
    int line;
    char* err;
    size_t errlen;
    /* string pool */
    char* pool;
    size_t pool_len, pool_cap;
    /* attribute tables */
    attr_tab vt, et;
    /* records */
    kv_t* vkv;
    int64_t vkv_len, vkv_cap;
    int64_t* vstart; /* per node start into vkv (n+1) */
    int64_t n, n_cap;
    double* node_id;
    kv_t* ekv;
    int64_t ekv_len, ekv_cap;
    int64_t* estart;
    int64_t m, m_cap;
    double* esrc_id;
    double* edst_id;
    int directed;
} ps_t;

static int fail(ps_t* s, const char* fmt, ...) {
    if (s->err && s->errlen) {
        int k = snprintf(s->err, s->errlen, "GML line %d: ", s->line);
        if (k < 0) k = 0;
        if ((size_t)k < s->errlen) {
            va_list ap;
            va_start(ap, fmt);
            vsnprintf(s->err + k, s->errlen - (size_t)k, fmt, ap);
            va_end(ap);
        }
    }
    return -1;
}

#define GROW(ptr, len, cap, type)                                                       \
    do {                                                                                \
        if ((len) >= (cap)) {                                                           \
            size_t nc_ = (cap) ? (size_t)(cap) * 2 : 64;                                \
            type* np_ = (type*)realloc((ptr), nc_ * sizeof(type));                      \
            if (!np_) return fail(s, "out of memory");                                  \
            (ptr) = np_;                                                                \
            (cap) = nc_;                                                                \
        }                                                                               \
    } while (0)

static void skip_ws(ps_t* s) {
    while (s->p < s->end) {
        char c = *s->p;
        if (c == '\n') {
            s->line++;
            s->p++;
        } else if (c == ' ' || c == '\t' || c == '\r' || c == '\f' || c == '\v') {
            s->p++;
        } else if (c == '#') {
            while (s->p < s->end && *s->p != '\n') s->p++;
        } else {
            break;
        }
    }
}

enum { T_EOF, T_KEY, T_NUM, T_STR, T_OPEN, T_CLOSE, T_BAD };

typedef struct {
    int kind;
    const char* b;
    size_t len;
    double num;
} tok_t;

static int is_key0(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_'; }
static int is_key1(char c) { return is_key0(c) || (c >= '0' && c <= '9'); }

static tok_t next_tok(ps_t* s) {
    tok_t t = {T_EOF, NULL, 0, 0.0};
    skip_ws(s);
    if (s->p >= s->end) return t;
    char c = *s->p;
    if (c == '[') {
        s->p++;
        t.kind = T_OPEN;
        return t;
    }
    if (c == ']') {
        s->p++;
        t.kind = T_CLOSE;
        return t;
    }
    if (c == '"') {
        const char* b = ++s->p;
        while (s->p < s->end && *s->p != '"') {
            if (*s->p == '\n') s->line++;
            s->p++;
        }
        if (s->p >= s->end) {
            t.kind = T_BAD;
            return t;
        }
        t.kind = T_STR;
        t.b = b;
        t.len = (size_t)(s->p - b);
        s->p++;
        return t;
    }
    if (is_key0(c)) {
        const char* b = s->p;
        while (s->p < s->end && is_key1(*s->p)) s->p++;
        t.kind = T_KEY;
        t.b = b;
        t.len = (size_t)(s->p - b);
        return t;
    }
    if ((c >= '0' && c <= '9') || c == '-' || c == '+' || c == '.') {
        char buf[128];
        const char* b = s->p;
        while (s->p < s->end && ((*s->p >= '0' && *s->p <= '9') || *s->p == '-' || *s->p == '+' ||
                                 *s->p == '.' || *s->p == 'e' || *s->p == 'E'))
            s->p++;
        size_t len = (size_t)(s->p - b);
        if (len == 0 || len >= sizeof(buf)) {
            t.kind = T_BAD;
            return t;
        }
        memcpy(buf, b, len);
        buf[len] = 0;
        char* e = NULL;
        t.num = strtod(buf, &e);
        if (!e || *e != 0) {
            t.kind = T_BAD;
            return t;
        }
        t.kind = T_NUM;
        return t;
    }
    t.kind = T_BAD;
    return t;
}

/* Decode the XML entities igraph's GML reader decodes. Returns pool offset. */
static int pool_add(ps_t* s, const char* b, size_t len, size_t* off) {
    if (s->pool_len + len + 1 > s->pool_cap) {
        size_t nc = s->pool_cap ? s->pool_cap : 4096;
        while (nc < s->pool_len + len + 1) nc *= 2;
        char* np = (char*)realloc(s->pool, nc);
        if (!np) return fail(s, "out of memory");
        s->pool = np;
        s->pool_cap = nc;
    }
    *off = s->pool_len;
    char* d = s->pool + s->pool_len;
    size_t k = 0;
    for (size_t i = 0; i < len; i++) {
        static const struct {
            const char* ent;
            char c;
        } ents[] = {{"&quot;", '"'}, {"&amp;", '&'}, {"&lt;", '<'}, {"&gt;", '>'}, {"&apos;", '\''}};
        int hit = 0;
        if (b[i] == '&') {
            for (size_t e = 0; e < sizeof(ents) / sizeof(ents[0]); e++) {
                size_t el = strlen(ents[e].ent);
                if (i + el <= len && memcmp(b + i, ents[e].ent, el) == 0) {
                    d[k++] = ents[e].c;
                    i += el - 1;
                    hit = 1;
                    break;
                }
            }
        }
        if (!hit) d[k++] = b[i];
    }
    d[k] = 0;
    s->pool_len += k + 1;
    return 0;
}

static int attr_index(ps_t* s, attr_tab* tab, const char* b, size_t len, int is_str) {
    for (int i = 0; i < tab->count; i++)
        if (strlen(tab->names[i]) == len && memcmp(tab->names[i], b, len) == 0) {
            if (is_str) tab->is_string[i] = 1;
            return i;
        }
    if (tab->count == tab->cap) {
        int nc = tab->cap ? tab->cap * 2 : 16;
        char** nn = (char**)realloc(tab->names, (size_t)nc * sizeof(char*));
        int* ns = (int*)realloc(tab->is_string, (size_t)nc * sizeof(int));
        if (!nn || !ns) return fail(s, "out of memory");
        tab->names = nn;
        tab->is_string = ns;
        tab->cap = nc;
    }
    char* name = (char*)malloc(len + 1);
    if (!name) return fail(s, "out of memory");
    memcpy(name, b, len);
    name[len] = 0;
    tab->names[tab->count] = name;
    tab->is_string[tab->count] = is_str;
    return tab->count++;
}

/* Skip a nested list body (after its '['). */
static int skip_list(ps_t* s) {
    int depth = 1;
    while (depth > 0) {
        tok_t t = next_tok(s);
        if (t.kind == T_EOF || t.kind == T_BAD) return fail(s, "unterminated list");
        if (t.kind == T_OPEN) depth++;
        if (t.kind == T_CLOSE) depth--;
    }
    return 0;
}

static int keyeq(const tok_t* t, const char* lit) {
    return t->len == strlen(lit) && memcmp(t->b, lit, t->len) == 0;
}

/* node [ ... ] or edge [ ... ] body */
static int parse_element(ps_t* s, int is_node) {
    int have_id = 0, have_src = 0, have_dst = 0;
    double id = NAN, sid = NAN, did = NAN;
    attr_tab* tab = is_node ? &s->vt : &s->et;
    for (;;) {
        tok_t k = next_tok(s);
        if (k.kind == T_CLOSE) break;
        if (k.kind != T_KEY) return fail(s, "expected key in %s", is_node ? "node" : "edge");
        tok_t v = next_tok(s);
        if (v.kind == T_OPEN) {
            if (skip_list(s)) return -1;
            continue;
        }
        if (v.kind != T_NUM && v.kind != T_STR) return fail(s, "bad value for key");
        if (is_node && keyeq(&k, "id")) {
            if (v.kind != T_NUM) return fail(s, "node id must be numeric");
            id = v.num;
            have_id = 1;
        }
        if (!is_node && keyeq(&k, "source")) {
            if (v.kind != T_NUM) return fail(s, "edge source must be numeric");
            sid = v.num;
            have_src = 1;
            continue;
        }
        if (!is_node && keyeq(&k, "target")) {
            if (v.kind != T_NUM) return fail(s, "edge target must be numeric");
            did = v.num;
            have_dst = 1;
            continue;
        }
        int a = attr_index(s, tab, k.b, k.len, v.kind == T_STR);
        if (a < 0) return -1;
        kv_t kv = {a, v.kind == T_STR, v.num, 0};
        if (v.kind == T_STR && pool_add(s, v.b, v.len, &kv.str)) return -1;
        if (is_node) {
            GROW(s->vkv, s->vkv_len, s->vkv_cap, kv_t);
            s->vkv[s->vkv_len++] = kv;
        } else {
            GROW(s->ekv, s->ekv_len, s->ekv_cap, kv_t);
            s->ekv[s->ekv_len++] = kv;
        }
    }
    if (is_node) {
        if (!have_id) return fail(s, "node without id");
        GROW(s->node_id, s->n, s->n_cap, double);
        size_t cap2 = s->n_cap;
        int64_t* ns = (int64_t*)realloc(s->vstart, (cap2 + 1) * sizeof(int64_t));
        if (!ns) return fail(s, "out of memory");
        s->vstart = ns;
        s->node_id[s->n] = id;
        s->n++;
        s->vstart[s->n] = s->vkv_len;
    } else {
        if (!have_src || !have_dst) return fail(s, "edge without source/target");
        GROW(s->esrc_id, s->m, s->m_cap, double);
        size_t cap2 = s->m_cap;
        double* nd = (double*)realloc(s->edst_id, cap2 * sizeof(double));
        int64_t* ne = (int64_t*)realloc(s->estart, (cap2 + 1) * sizeof(int64_t));
        if (!nd || !ne) return fail(s, "out of memory");
        s->edst_id = nd;
        s->estart = ne;
        s->esrc_id[s->m] = sid;
        s->edst_id[s->m] = did;
        s->m++;
        s->estart[s->m] = s->ekv_len;
    }
    return 0;
}

/* The graph list's items from s->p: node and edge lists, other lists skipped, key-value pairs
 * (only `directed` is kept; the last one wins). Stops at the graph's closing ']' (*closed = 1) or,
 * with stop != NULL, at the first item that starts at or after stop (a parallel chunk's end). */
static int parse_items(ps_t* s, const char* stop, int* closed, int* have_dir, int* dir) {
    *closed = 0;
    for (;;) {
        skip_ws(s);
        if (stop && s->p >= stop) return 0;
        tok_t k = next_tok(s);
        if (k.kind == T_CLOSE) {
            *closed = 1;
            return 0;
        }
        if (k.kind != T_KEY) return fail(s, "expected key in graph");
        tok_t v = next_tok(s);
        if (v.kind == T_OPEN) {
            if (keyeq(&k, "node")) {
                if (parse_element(s, 1)) return -1;
            } else if (keyeq(&k, "edge")) {
                if (parse_element(s, 0)) return -1;
            } else if (skip_list(s)) {
                return -1;
            }
            continue;
        }
        if (v.kind != T_NUM && v.kind != T_STR) return fail(s, "bad value in graph");
        if (keyeq(&k, "directed") && v.kind == T_NUM) {
            *have_dir = 1;
            *dir = v.num != 0.0;
        }
    }
}

static int parse_graph(ps_t* s) {
    int closed = 0, have_dir = 0, dir = 0;
    if (parse_items(s, NULL, &closed, &have_dir, &dir)) return -1;
    if (have_dir) s->directed = dir;
    return 0;
}

/* ---- the graph list in parallel (large files) ------------------------------------------------ *
 * Shadow's own GML and Tor-atlas-derived topologies are one `graph [` list of millions of `node
 * [...]` / `edge [...]` items; one core tokenises ~140 MB/s. Above GML_PAR_MIN bytes the list is
 * cut at candidate item starts (a line that begins, after blanks, with `node [` or `edge [`),
 * each piece is parsed by its own thread into its own records, string pool and attribute tables,
 * and the pieces are concatenated in file order (attributes keep their first-seen order and are
 * strings if any piece saw a string). A candidate inside a quoted string or a nested list is
 * caught because the previous piece, parsing from a true item start, does not stop exactly on
 * it; then, or on any error, the list is parsed again by one thread, which also writes the error
 * message with its line. */
#define GML_PAR_MIN ((size_t)64 << 20)
#define GML_PAR_MAXT 16

typedef struct {
    ps_t s;
    const char* stop;
    int rc, closed, have_dir, dir;
} gml_piece;

static void* piece_run(void* arg) {
    gml_piece* c = (gml_piece*)arg;
    c->rc = pool_add(&c->s, "", 0, &(size_t){0}) ? -1 : 0;
    c->s.vstart = (int64_t*)calloc(1, sizeof(int64_t));
    c->s.estart = (int64_t*)calloc(1, sizeof(int64_t));
    if (!c->s.vstart || !c->s.estart) c->rc = -1;
    if (!c->rc) c->rc = parse_items(&c->s, c->stop, &c->closed, &c->have_dir, &c->dir);
    return NULL;
}

static void ps_free(ps_t* s) {
    for (int i = 0; i < s->vt.count; i++) free(s->vt.names[i]);
    for (int i = 0; i < s->et.count; i++) free(s->et.names[i]);
    free(s->vt.names);
    free(s->vt.is_string);
    free(s->et.names);
    free(s->et.is_string);
    free(s->vkv);
    free(s->ekv);
    free(s->vstart);
    free(s->estart);
    free(s->node_id);
    free(s->esrc_id);
    free(s->edst_id);
    free(s->pool);
}

/* a candidate item start at or after q: the first line from q that begins with node/edge and '[' */
static const char* next_item_start(const char* q, const char* end) {
    while (q < end) {
        const char* nl = (const char*)memchr(q, '\n', (size_t)(end - q));
        if (!nl) return NULL;
        const char* b = nl + 1;
        while (b < end && (*b == ' ' || *b == '\t' || *b == '\r')) b++;
        if (end - b > 5 && (memcmp(b, "node", 4) == 0 || memcmp(b, "edge", 4) == 0)) {
            const char* x = b + 4;
            while (x < end && (*x == ' ' || *x == '\t' || *x == '\r' || *x == '\n')) x++;
            if (x < end && *x == '[') return b;
        }
        q = b;
    }
    return NULL;
}

/* Merging the pieces: the attribute maps and every piece's offsets into the merged arrays are
 * planned on one thread (cheap), then each piece copies its records, remapped, on its own thread
 * (on one thread the merge took ~170 ms of a 200-MB file's ~540). */
typedef struct {
    ps_t* s;
    ps_t* c;
    int vmap[1024], emap[1024];
    size_t pbase;
    int64_t vk0, ek0, n0, m0;
} piece_copy_t;

static void* piece_copy(void* arg) {
    piece_copy_t* q = (piece_copy_t*)arg;
    ps_t* s = q->s;
    const ps_t* c = q->c;
    memcpy(s->pool + q->pbase, c->pool, c->pool_len);
    for (int64_t k = 0; k < c->vkv_len; k++) {
        kv_t kv = c->vkv[k];
        kv.attr = q->vmap[kv.attr];
        if (kv.is_str) kv.str += q->pbase;
        s->vkv[q->vk0 + k] = kv;
    }
    for (int64_t k = 0; k < c->ekv_len; k++) {
        kv_t kv = c->ekv[k];
        kv.attr = q->emap[kv.attr];
        if (kv.is_str) kv.str += q->pbase;
        s->ekv[q->ek0 + k] = kv;
    }
    memcpy(s->node_id + q->n0, c->node_id, (size_t)c->n * sizeof(double));
    for (int64_t i = 1; i <= c->n; i++) s->vstart[q->n0 + i] = q->vk0 + c->vstart[i];
    memcpy(s->esrc_id + q->m0, c->esrc_id, (size_t)c->m * sizeof(double));
    memcpy(s->edst_id + q->m0, c->edst_id, (size_t)c->m * sizeof(double));
    for (int64_t i = 1; i <= c->m; i++) s->estart[q->m0 + i] = q->ek0 + c->estart[i];
    return NULL;
}

/* append the k pieces' records to s in order; -1 when out of memory */
static int pieces_merge(ps_t* s, gml_piece* pc, int k) {
    piece_copy_t* q = (piece_copy_t*)calloc((size_t)k, sizeof(piece_copy_t));
    if (!q) return -1;
    size_t pool = s->pool_len;
    int64_t vk = s->vkv_len, ek = s->ekv_len, n = s->n, m = s->m;
    int rc = 0;
    for (int i = 0; i < k && !rc; i++) {
        ps_t* c = &pc[i].s;
        q[i].s = s;
        q[i].c = c;
        for (int a = 0; a < c->vt.count && !rc; a++)
            if ((q[i].vmap[a] = attr_index(s, &s->vt, c->vt.names[a], strlen(c->vt.names[a]), c->vt.is_string[a])) < 0)
                rc = -1;
        for (int a = 0; a < c->et.count && !rc; a++)
            if ((q[i].emap[a] = attr_index(s, &s->et, c->et.names[a], strlen(c->et.names[a]), c->et.is_string[a])) < 0)
                rc = -1;
        q[i].pbase = pool;
        q[i].vk0 = vk;
        q[i].ek0 = ek;
        q[i].n0 = n;
        q[i].m0 = m;
        pool += c->pool_len;
        vk += c->vkv_len;
        ek += c->ekv_len;
        n += c->n;
        m += c->m;
    }
    /* the merged arrays at their final sizes (the starts one longer) */
    if (!rc) {
        char* np = (char*)realloc(s->pool, pool > 0 ? pool : 1);
        if (np) { s->pool = np; s->pool_cap = pool; }
        kv_t* nv = (kv_t*)realloc(s->vkv, (size_t)(vk > 0 ? vk : 1) * sizeof(kv_t));
        if (nv) { s->vkv = nv; s->vkv_cap = vk; }
        kv_t* ne = (kv_t*)realloc(s->ekv, (size_t)(ek > 0 ? ek : 1) * sizeof(kv_t));
        if (ne) { s->ekv = ne; s->ekv_cap = ek; }
        double* ni = (double*)realloc(s->node_id, (size_t)(n > 0 ? n : 1) * sizeof(double));
        if (ni) { s->node_id = ni; s->n_cap = n; }
        int64_t* vs = (int64_t*)realloc(s->vstart, (size_t)(n + 1) * sizeof(int64_t));
        if (vs) s->vstart = vs;
        double* es = (double*)realloc(s->esrc_id, (size_t)(m > 0 ? m : 1) * sizeof(double));
        if (es) { s->esrc_id = es; s->m_cap = m; }
        double* ed = (double*)realloc(s->edst_id, (size_t)(m > 0 ? m : 1) * sizeof(double));
        if (ed) s->edst_id = ed;
        int64_t* est = (int64_t*)realloc(s->estart, (size_t)(m + 1) * sizeof(int64_t));
        if (est) s->estart = est;
        if (!np || !nv || !ne || !ni || !vs || !es || !ed || !est) rc = -1;
    }
    if (!rc) {
        pthread_t th[GML_PAR_MAXT];
        int started[GML_PAR_MAXT];
        for (int i = 0; i < k; i++) {
            started[i] = pthread_create(&th[i], NULL, piece_copy, &q[i]) == 0;
            if (!started[i]) piece_copy(&q[i]);
        }
        for (int i = 0; i < k; i++)
            if (started[i]) pthread_join(th[i], NULL);
        s->pool_len = pool;
        s->vkv_len = vk;
        s->ekv_len = ek;
        s->n = n;
        s->m = m;
    }
    free(q);
    return rc;
}

/* The graph list from s->p (just past its '['), in nt pieces. Returns the number of pieces when it
 * was parsed (s->p past the closing ']'), 0 when the caller should parse it with one thread
 * (nothing changed), -1 when merging the pieces ran out of memory. */
static int parse_graph_parallel(ps_t* s, int nt) {
    const char* b[GML_PAR_MAXT + 1];
    int k = 0;
    b[k++] = s->p;
    const size_t body = (size_t)(s->end - s->p);
    for (int i = 1; i < nt; i++) {
        const char* q = next_item_start(s->p + body / (size_t)nt * (size_t)i, s->end);
        if (!q) break;
        if (q > b[k - 1]) b[k++] = q;
    }
    if (k < 2) return 0;
    gml_piece pc[GML_PAR_MAXT];
    pthread_t th[GML_PAR_MAXT];
    int started[GML_PAR_MAXT];
    memset(pc, 0, sizeof(pc));
    for (int i = 0; i < k; i++) {
        pc[i].s.p = b[i];
        pc[i].s.end = s->end;
        pc[i].s.line = 1;
        pc[i].stop = i + 1 < k ? b[i + 1] : NULL;
        started[i] = pthread_create(&th[i], NULL, piece_run, &pc[i]) == 0;
        if (!started[i]) piece_run(&pc[i]);
    }
    for (int i = 0; i < k; i++)
        if (started[i]) pthread_join(th[i], NULL);
    int ok = 1;
    for (int i = 0; i < k && ok; i++) { /* every piece ends exactly where the next begins */
        if (pc[i].rc || pc[i].s.vt.count > 1024 || pc[i].s.et.count > 1024) ok = 0;
        else if (i + 1 < k) ok = !pc[i].closed && pc[i].s.p == b[i + 1];
        else ok = pc[i].closed;
    }
    int dir = -1, rc = ok;
    for (int i = 0; i < k; i++)
        if (pc[i].have_dir) dir = pc[i].dir;
    if (rc == 1 && pieces_merge(s, pc, k)) rc = fail(s, "out of memory");
    if (rc == 1) {
        if (dir >= 0) s->directed = dir;
        s->p = pc[k - 1].s.p;
        rc = k;
    }
    for (int i = 0; i < k; i++) ps_free(&pc[i].s);
    return rc;
}

/* open-addressing id -> index map */
typedef struct {
    int64_t* keys;
    int32_t* vals;
    size_t cap;
} idmap;

static size_t hash64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    return (size_t)x;
}

static int build_columns(ps_t* s, attr_tab* tab, kv_t* kv, int64_t* start, int64_t count,
                         gml_attr** out, int* nout) {
    gml_attr* cols = (gml_attr*)calloc((size_t)(tab->count > 0 ? tab->count : 1), sizeof(gml_attr));
    if (!cols) return fail(s, "out of memory");
    *out = cols;
    *nout = tab->count;
    for (int a = 0; a < tab->count; a++) {
        cols[a].name = tab->names[a];
        tab->names[a] = NULL;
        cols[a].is_string = tab->is_string[a];
        if (cols[a].is_string) {
            cols[a].str = (char**)malloc((size_t)(count > 0 ? count : 1) * sizeof(char*));
            if (!cols[a].str) return fail(s, "out of memory");
        } else {
            cols[a].num = (double*)malloc((size_t)(count > 0 ? count : 1) * sizeof(double));
            if (!cols[a].num) return fail(s, "out of memory");
        }
    }
    /* "" for missing strings lives at pool offset 0 (see gml_parse) */
    for (int64_t i = 0; i < count; i++) {
        for (int a = 0; a < tab->count; a++) {
            if (cols[a].is_string)
                cols[a].str[i] = NULL; /* fixed up below */
            else
                cols[a].num[i] = NAN;
        }
        for (int64_t k = start[i]; k < start[i + 1]; k++) {
            gml_attr* c = &cols[kv[k].attr];
            if (c->is_string) {
                if (kv[k].is_str) {
                    c->str[i] = (char*)(uintptr_t)(kv[k].str + 1);
                } else {
                    char buf[64];
                    snprintf(buf, sizeof(buf), "%.17g", kv[k].num);
                    size_t off;
                    if (pool_add(s, buf, strlen(buf), &off)) return -1;
                    c->str[i] = (char*)(uintptr_t)(off + 1);
                }
            } else {
                c->num[i] = kv[k].num;
            }
        }
    }
    return 0;
}

static void fix_strings(gml_attr* cols, int na, int64_t count, char* pool) {
    for (int a = 0; a < na; a++) {
        if (!cols[a].is_string) continue;
        for (int64_t i = 0; i < count; i++) {
            uintptr_t o = (uintptr_t)cols[a].str[i];
            cols[a].str[i] = o ? pool + (o - 1) : pool; /* pool[0] == '\0' */
        }
    }
}

int gml_parse(const char* text, size_t len, gml_graph* out, char* err, size_t errlen) {
    long nc = sysconf(_SC_NPROCESSORS_ONLN);
    int nt = nc > GML_PAR_MAXT ? GML_PAR_MAXT : nc > 1 ? (int)nc : 1;
    const size_t per = (size_t)16 << 20; /* at least 16 MB per piece */
    if ((size_t)nt > len / per) nt = (int)(len / per) > 1 ? (int)(len / per) : 1;
    return gml_parse_ex(text, len, out, err, errlen, nt, GML_PAR_MIN);
}

int gml_parse_ex(const char* text, size_t len, gml_graph* out, char* err, size_t errlen, int nthreads,
                 size_t par_min) {
    int used_par = 0; /* the graph list was parsed in pieces */
    memset(out, 0, sizeof(*out));
    ps_t st;
    memset(&st, 0, sizeof(st));
    ps_t* s = &st;
    s->p = text;
    s->end = text + len;
    s->line = 1;
    s->err = err;
    s->errlen = errlen;
    if (err && errlen) err[0] = 0;
    size_t empty;
    int rc = -1;
    if (pool_add(s, "", 0, &empty)) goto done;
    s->vstart = (int64_t*)calloc(1, sizeof(int64_t));
    s->estart = (int64_t*)calloc(1, sizeof(int64_t));
    if (!s->vstart || !s->estart) {
        fail(s, "out of memory");
        goto done;
    }
    int found = 0;
    for (;;) {
        tok_t k = next_tok(s);
        if (k.kind == T_EOF) break;
        if (k.kind != T_KEY) {
            fail(s, "expected key at top level");
            goto done;
        }
        tok_t v = next_tok(s);
        if (v.kind == T_OPEN) {
            if (keyeq(&k, "graph") && !found) {
                int par = 0;
                if (nthreads > 1 && (size_t)(s->end - s->p) >= par_min)
                    par = parse_graph_parallel(s, nthreads < GML_PAR_MAXT ? nthreads : GML_PAR_MAXT);
                used_par = par > 0 ? par : 0;
                if (par < 0 || (!par && parse_graph(s))) goto done;
                found = 1;
            } else if (skip_list(s)) {
                goto done;
            }
        } else if (v.kind != T_NUM && v.kind != T_STR) {
            fail(s, "bad top-level value");
            goto done;
        }
    }
    if (!found) {
        fail(s, "no graph found");
        goto done;
    }
    if (s->n > INT32_MAX) {
        fail(s, "too many nodes");
        goto done;
    }
    /* resolve edge endpoints through node ids */
    idmap map = {0};
    map.cap = 16;
    while (map.cap < (size_t)s->n * 2 + 16) map.cap *= 2;
    map.keys = (int64_t*)malloc(map.cap * sizeof(int64_t));
    map.vals = (int32_t*)malloc(map.cap * sizeof(int32_t));
    if (!map.keys || !map.vals) {
        free(map.keys);
        free(map.vals);
        fail(s, "out of memory");
        goto done;
    }
    for (size_t i = 0; i < map.cap; i++) map.vals[i] = -1;
    for (int64_t i = 0; i < s->n; i++) {
        int64_t key = (int64_t)s->node_id[i];
        size_t h = hash64((uint64_t)key) & (map.cap - 1);
        while (map.vals[h] >= 0 && map.keys[h] != key) h = (h + 1) & (map.cap - 1);
        if (map.vals[h] >= 0) {
            free(map.keys);
            free(map.vals);
            fail(s, "duplicate node id %lld", (long long)key);
            goto done;
        }
        map.keys[h] = key;
        map.vals[h] = (int32_t)i;
    }
    out->esrc = (int32_t*)malloc((size_t)(s->m > 0 ? s->m : 1) * sizeof(int32_t));
    out->edst = (int32_t*)malloc((size_t)(s->m > 0 ? s->m : 1) * sizeof(int32_t));
    if (!out->esrc || !out->edst) {
        free(map.keys);
        free(map.vals);
        fail(s, "out of memory");
        goto done;
    }
    for (int64_t e = 0; e < s->m; e++) {
        for (int end = 0; end < 2; end++) {
            int64_t key = (int64_t)(end ? s->edst_id[e] : s->esrc_id[e]);
            size_t h = hash64((uint64_t)key) & (map.cap - 1);
            while (map.vals[h] >= 0 && map.keys[h] != key) h = (h + 1) & (map.cap - 1);
            if (map.vals[h] < 0) {
                free(map.keys);
                free(map.vals);
                fail(s, "edge %lld references unknown node id %lld", (long long)e, (long long)key);
                goto done;
            }
            if (end)
                out->edst[e] = map.vals[h];
            else
                out->esrc[e] = map.vals[h];
        }
    }
    free(map.keys);
    free(map.vals);
    if (build_columns(s, &s->vt, s->vkv, s->vstart, s->n, &out->va, &out->nva)) goto done;
    if (build_columns(s, &s->et, s->ekv, s->estart, s->m, &out->ea, &out->nea)) goto done;
    fix_strings(out->va, out->nva, s->n, s->pool);
    fix_strings(out->ea, out->nea, s->m, s->pool);
    out->directed = s->directed;
    out->n = (int32_t)s->n;
    out->m = s->m;
    out->pool = s->pool;
    out->pieces = used_par > 1 ? used_par : 1;
    s->pool = NULL;
    rc = 0;
done:
    for (int i = 0; i < s->vt.count; i++) free(s->vt.names[i]);
    for (int i = 0; i < s->et.count; i++) free(s->et.names[i]);
    free(s->vt.names);
    free(s->vt.is_string);
    free(s->et.names);
    free(s->et.is_string);
    free(s->vkv);
    free(s->ekv);
    free(s->vstart);
    free(s->estart);
    free(s->node_id);
    free(s->esrc_id);
    free(s->edst_id);
    free(s->pool);
    if (rc) gml_free(out);
    /* an error after a parallel graph list: one thread again, for the message and its line */
    if (rc && used_par) return gml_parse_ex(text, len, out, err, errlen, 1, par_min);
    return rc;
}

void gml_free(gml_graph* g) {
    if (!g) return;
    for (int i = 0; i < g->nva; i++) {
        free(g->va[i].name);
        free(g->va[i].num);
        free(g->va[i].str);
    }
    for (int i = 0; i < g->nea; i++) {
        free(g->ea[i].name);
        free(g->ea[i].num);
        free(g->ea[i].str);
    }
    free(g->va);
    free(g->ea);
    free(g->esrc);
    free(g->edst);
    free(g->pool);
    memset(g, 0, sizeof(*g));
}

const gml_attr* gml_vattr(const gml_graph* g, const char* name) {
    for (int i = 0; i < g->nva; i++)
        if (strcmp(g->va[i].name, name) == 0) return &g->va[i];
    return NULL;
}

const gml_attr* gml_eattr(const gml_graph* g, const char* name) {
    for (int i = 0; i < g->nea; i++)
        if (strcmp(g->ea[i].name, name) == 0) return &g->ea[i];
    return NULL;
}
