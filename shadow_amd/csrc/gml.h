/*
 * gml.h -- GML subset reader producing the attribute model Shadow's topology code validates.
 *
 * Replaces igraph_read_graph_gml (called at /root/reference/src/main/routing/topology.c:347) for
 * the attributes topology.c reads: vertex order = order of `node` lists, edge order = order of
 * `edge` lists, edge endpoints resolved through node `id`, an attribute is STRING if any element
 * gives it a quoted string and NUMERIC otherwise, missing numeric = NaN, missing string = "".
 * Nested lists inside node/edge (e.g. `graphics [...]`) are skipped like igraph does.
 */
#ifndef SRT_GML_H
#define SRT_GML_H

#include <stddef.h>
#include <stdint.h>

typedef struct gml_attr {
    char* name;
    int is_string;  /* IGRAPH_ATTRIBUTE_STRING vs NUMERIC */
    double* num;    /* per element (NaN if missing) when !is_string */
    char** str;     /* per element ("" if missing) when is_string */
} gml_attr;

typedef struct gml_graph {
    int directed;
    int32_t n;
    int64_t m;
    int32_t* esrc;
    int32_t* edst;
    int nva, nea;
    gml_attr* va;
    gml_attr* ea;
    char* pool; /* string storage */
    int pieces; /* the graph list was parsed in this many pieces (1: one thread) */
} gml_graph;

/* Returns 0 on success; on error returns -1 and writes a message into err (if non-NULL). */
int gml_parse(const char* text, size_t len, gml_graph* out, char* err, size_t errlen);
/* gml_parse with the graph list cut into up to nthreads pieces parsed in parallel when it holds
 * at least par_min bytes (gml_parse: the online CPUs up to 16, one per 16 MB, from 64 MB on).
 * The result, and any error message, is the one-thread parse's. */
int gml_parse_ex(const char* text, size_t len, gml_graph* out, char* err, size_t errlen, int nthreads,
                 size_t par_min);
void gml_free(gml_graph* g);
/* Exact-name attribute lookup (igraph_cattribute_has_attr semantics). */
const gml_attr* gml_vattr(const gml_graph* g, const char* name);
const gml_attr* gml_eattr(const gml_graph* g, const char* name);

#endif
