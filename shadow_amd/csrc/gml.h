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
} gml_graph;

/* Returns 0 on success; on error returns -1 and writes a message into err (if non-NULL). */
int gml_parse(const char* text, size_t len, gml_graph* out, char* err, size_t errlen);
void gml_free(gml_graph* g);
/* Exact-name attribute lookup (igraph_cattribute_has_attr semantics). */
const gml_attr* gml_vattr(const gml_graph* g, const char* name);
const gml_attr* gml_eattr(const gml_graph* g, const char* name);

#endif
