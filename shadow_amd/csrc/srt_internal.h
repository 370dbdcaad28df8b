/*
 * srt_internal.h -- private helpers shared by the host C layer and the HIP translation units.
 */
#ifndef SRT_INTERNAL_H
#define SRT_INTERNAL_H

#include <stdint.h>

#include "shadow_routing.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { SRT_LOG_ERROR = 0, SRT_LOG_WARNING = 1, SRT_LOG_INFO = 2, SRT_LOG_DEBUG = 3 };
void srt_log(int level, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void srt_set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
/* SRT_FORM=key=value,... (tests / A/B only): srt_form_int -> the value of key, or dflt when unset;
 * srt_form_is -> 1 when key is set to exactly value (graph.c) */
int srt_form_int(const char* key, int dflt);
int srt_form_is(const char* key, const char* value);

/* Canonical dense / CSR forms of an edge list (host side, see graph.c). */
typedef struct srt_canon {
    int32_t n;
    int32_t directed;
    uint64_t quantum_ns;
    uint32_t max_w_q;
    /* upper bound on every finite shortest distance, in quanta (graph.c: MST, (n - 1) max_w or
     * the hop bound through the highest-degree vertex); < SRT_INF unless wide */
    uint64_t dist_bound;
    /* 1: the bound reaches SRT_INF (2^31 - 1) quanta -- only the u64 rows of wide.hip build this graph */
    int32_t wide;
    /* CSR of canonical out-arcs (self-loops excluded), columns ascending */
    int64_t arcs;
    int32_t* rowptr;
    int32_t* col;
    uint32_t* w;
    double* r;
    /* CSR of canonical in-arcs (directed graphs only; aliases the out-CSR when undirected) */
    int32_t* in_rowptr;
    int32_t* in_col;
    uint32_t* in_w;
    double* in_r;
    /* canonical self-loop per vertex (SRT_INF if none) */
    uint32_t* self_w;
    double* self_r;
    /* edge-list form (build.hip, dense builds): no CSR (rowptr NULL); the dense matrices are
     * scattered from these edges on the device, arcs holds an upper bound until then and
     * verify_dense asks the scatter to confirm the auto choice of the dense build */
    const srt_edges* edges;
    int32_t verify_dense;
} srt_canon;

int srt_canon_build(const srt_edges* g, srt_canon* c);
void srt_canon_free(srt_canon* c);

#ifdef __cplusplus
}
#endif

#endif
