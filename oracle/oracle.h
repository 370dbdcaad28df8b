/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY (never linked into the product library).
 *
 * A plain-C CPU restatement of Shadow's routing precomputation path, used as the parity checker
 * for the HIP implementation in shadow_amd/ and as the CPU baseline ("kind": "port") in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Follows /root/reference/src/main/routing/topology.c:
 *   - per-source Dijkstra, mode IGRAPH_OUT            topology.c:1578-1814 (call at :1682)
 *   - path-order latency sum / reliability product     topology.c:1286-1389 (:1308-1309, :1364-1365)
 *   - edge weight = (double)ns / 1e6 ms                topology.c:280-302 (:294)
 *   - edge reliability = 1.0 - packet_loss             topology.c:363-403 (:396)
 *   - diagonal ("shortest path to self") rule          topology.c:1431-1576
 *   - direct mode (use_shortest_path = false)          topology.c:1816-1858, :1948-1958
 *   - one cached entry per unordered pair (symmetry)   topology.c:1189-1215, :1918-1921, :1964-1967
 *     (orc_table: the pairs as served when sources run in increasing vertex order; the lazy-cache
 *     order itself is restated in oracle/lazy_cache.py over orc_table_raw's per-source rows)
 *   - delay = ceil(latency_ms * 1e6) ns                worker.c:550-551
 *
 * Tie rule: igraph's Dijkstra keeps the first-settled tight predecessor; igraph
 * is absent from this container, so the canonical rule is Dijkstra with a (distance, vertex index)
 * heap and strict-< relaxation, i.e. pred(s,t) = argmin over tight in-edges (u,t) of (D[s][u], u).
 * Which row serves a pair: the reference serves {s,t} from whichever end's source ran first (with
 * the other end attached), for directed graphs too (topology.c:1194-1199, :1964-1967). orc_table
 * fixes that order to increasing vertex index (undirected: the row of min(s,t), mirrored);
 * orc_table_raw keeps every source's own row, and oracle/lazy_cache.py replays a lookup trace in
 * the reference's order over it.
 * Parallel edges collapse to the (min latency, lowest edge index) edge for a vertex pair.
 *
 * Parity status: multi-vertex routing is "parity unpinned" by the reference's own tests (every
 * graph in the reference's test suite has one vertex and one self-loop); the oracle
 * is pinned by those single-vertex known answers, by networkx for the latency matrix, and by
 * hand-built tie graphs (tests/golden/).
 */
#ifndef SRT_ORACLE_H
#define SRT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_graph {
    int32_t n;             /* vertices, GML order */
    int32_t directed;      /* GML graph.directed */
    int64_t m;             /* edges, GML order */
    const int32_t* src;    /* edge source vertex index */
    const int32_t* dst;    /* edge target vertex index */
    const int64_t* lat_ns; /* parse_time_nanosec(latency) */
    const double* loss;    /* packet_loss */
} orc_graph;

/* Distance arithmetic of the per-source Dijkstra.
 * ORC_INT_NS: exact integer nanoseconds (the canonical parity target, "integer ns").
 * ORC_F64_MS: f64 milliseconds exactly as igraph sees the weights (topology.c:1108, :1682).
 * On graphs whose latencies are whole milliseconds both modes select identical paths. */
enum { ORC_INT_NS = 0, ORC_F64_MS = 1 };

/* Per-source rows [s0, s1): for every target t the canonical shortest path from s.
 *   lat_int[r*n+t]  integer ns sum along the path          (UINT64_MAX if unreachable)
 *   lat_ref[r*n+t]  ceil(f64 ms path-order sum * 1e6)      (worker.c:551)
 *   rel[r*n+t]      f64 product of (1-loss) in path order  (topology.c:1365)
 *   lat_ms[r*n+t]   f64 ms path-order sum (the value topology_getLatency() returns)
 *   pred[r*n+t]     canonical predecessor of t (-1 for t == s or unreachable)
 * Diagonal entries hold the empty path (0, 0, 1.0). Any output pointer may be NULL.
 * nthreads > 1 shards sources over pthreads. Returns 0 on success. */
int orc_sssp_rows(const orc_graph* g, int mode, int32_t s0, int32_t s1, int nthreads,
                  uint64_t* lat_int, uint64_t* lat_ref, double* rel, double* lat_ms, int32_t* pred);
/* orc_sssp_rows for the sources srcs[0..k): row i belongs to srcs[i] */
int orc_sssp_list(const orc_graph* g, int mode, const int32_t* srcs, int32_t k, int nthreads,
                  uint64_t* lat_int, uint64_t* lat_ref, double* rel, double* lat_ms, int32_t* pred);

/* Full n*n table as the reference's lookup API would return it for every vertex pair:
 * shortest-path or direct mode, diagonal rule, symmetry rule. lat_ms (optional) is the f64
 * value topology_getLatency() returns. Returns 0 on success, -1 if direct mode lacks an edge. */
int orc_table(const orc_graph* g, int use_shortest_path, int mode, int nthreads,
              uint64_t* lat_int, uint64_t* lat_ref, double* rel, double* lat_ms);

/* orc_table without the pair rule: entry (s, t) is what source s computes for t (its raw row),
 * the diagonal rule on the diagonal; direct mode: the direct edge s -> t. */
int orc_table_raw(const orc_graph* g, int use_shortest_path, int mode, int nthreads,
                  uint64_t* lat_int, uint64_t* lat_ref, double* rel, double* lat_ms);

/* Diagonal rule only (topology.c:1431-1576) for vertex v. */
void orc_self_path(const orc_graph* g, int32_t v, uint64_t* lat_int, uint64_t* lat_ref,
                   double* rel, double* lat_ms);

/* CPU baseline on the synthetic complete graph (graphs.complete_graph / srt_gen_complete_device
 * with the same seed and distributions): dense O(n^2) Dijkstra from k sampled sources.
 * lat_out/rel_out are k x n raw per-source rows (lat in ns). Times exclude nothing but the
 * matrix generation, reported separately. */
int orc_complete_sample(int32_t n, uint64_t seed, uint32_t lat_max, uint32_t self_max,
                        uint32_t loss_max, const int32_t* sources, int32_t k, int nthreads,
                        uint64_t* lat_out, double* rel_out, double* gen_seconds,
                        double* sssp_seconds);
/* the same on the metric complete graph (points in the unit square, latency
 * max(1, round(scale_ms * dist)) ms; bench workload c4metric) */
int orc_metric_sample(int32_t n, uint64_t seed, uint32_t scale_ms, uint32_t self_max,
                      uint32_t loss_max, const int32_t* sources, int32_t k, int nthreads,
                      uint64_t* lat_out, double* rel_out, double* gen_seconds,
                      double* sssp_seconds);
uint32_t orc_dense_weight(uint64_t seed, uint32_t lat_max, uint32_t metric, uint32_t self_max,
                          uint32_t i, uint32_t j);

#ifdef __cplusplus
}
#endif

#endif
