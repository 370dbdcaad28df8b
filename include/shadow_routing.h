/*
 * shadow_routing.h -- C-ABI of the MI355X-native routing-table build for Shadow.
 *
 * Drop-in boundary: Shadow's routing module, /root/reference/src/main/routing/topology.h:17-28.
 * The reference-signature entry points (topology_new, topology_attach, topology_getLatency, ...)
 * are declared in include/topology.h and implemented on top of the srt_* functions below.
 * Everything here uses plain C types (no glib, no torch): pointers, sizes, status codes.
 *
 * Table layout: row-major lat[n][n] in u32 quanta of `quantum_ns` nanoseconds
 * and rel[n][n] f64, indexed by graph vertex index (GML order). The diagonal holds the
 * "shortest path to self" rule (topology.c:1431-1576); undirected graphs are symmetric.
 */
#ifndef SHADOW_ROUTING_H
#define SHADOW_ROUTING_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ----------------------------------------------------------------------- */
enum {
    SRT_OK = 0,
    SRT_E_ARG = -1,       /* bad argument / shape */
    SRT_E_PARSE = -2,     /* GML or unit parse error */
    SRT_E_INVALID = -3,   /* graph failed validation (topology.c:659-1038) */
    SRT_E_NOMEM = -4,     /* host or device allocation failed */
    SRT_E_DEVICE = -5,    /* HIP error (never a silent CPU fallback) */
    SRT_E_RANGE = -6,     /* path latencies exceed the u32-quantum table range */
    SRT_E_COMM = -7,      /* RCCL error */
    SRT_E_NOPATH = -8,    /* pair has no path (reference: utility_panic, topology.c:1970-1976) */
    SRT_E_UNATTACHED = -9 /* address not attached (reference: returns -1, topology.c:1905-1915) */
};

/* ---- units grammar (restates src/main/core/support/units.rs:404-437, :776-837) ----------- */
/* Nanoseconds, or -1 on a parse error / value > i64::MAX, or -2 where the reference's
 * `.unwrap()` on the unit conversion would panic (u64 overflow, units.rs:821). */
int64_t srt_parse_time_nanosec(const char* s);
/* Bits per second, or -1 / -2 with the same meaning (units.rs:776-805). */
int64_t srt_parse_bandwidth(const char* s);

/* ---- device build ------------------------------------------------------------------------ */
enum { SRT_ALGO_AUTO = 0, SRT_ALGO_DENSE_FW = 1, SRT_ALGO_SPARSE_SSSP = 2 };

/* Graph handed over as canonical arrays (one arc per ordered vertex pair, see srt_canon_*). */
typedef struct srt_edges {
    int32_t n;
    int32_t directed;
    int64_t m;
    const int32_t* src;    /* edge source vertex index (GML order) */
    const int32_t* dst;    /* edge target vertex index */
    const int64_t* lat_ns; /* parse_time_nanosec(latency) */
    const double* loss;    /* packet_loss */
} srt_edges;

typedef struct srt_build_opts {
    int32_t device;            /* HIP device ordinal */
    int32_t algo;              /* SRT_ALGO_* */
    int32_t use_shortest_path; /* network.use_shortest_path (configuration.rs:204-209) */
    int32_t fw_block;          /* 0 = default pivot-block edge */
} srt_build_opts;

typedef struct srt_build_stats {
    int32_t time_kernels; /* input: 1 = bracket every FW update launch with HIP events */
    int32_t algo;        /* algorithm actually used */
    int32_t fw_block;    /* dense: pivot-block edge used by FW; sparse: the kernel's form --
                          * wave kernel 1 = working row in LDS | 2 = private relabelled
                          * reliability row; workgroup kernel 4 | 1 = original vertex order
                          * | 2 = compact 8-byte arcs; multi-source kernel 8 | 16 = 16-bit
                          * working distances */
    int64_t ess_arcs;    /* essential arcs found by the predecessor pass (dense) */
    double ms_total;     /* wall time of the device build (HIP events), excl. host copies */
    double ms_fw;        /* shortest-distance kernels */
    double ms_post;      /* predecessor / reliability / diagonal / symmetry kernels */
    int32_t max_depth;   /* deepest shortest-path tree seen by the reliability pass */
    int32_t n_update;    /* FW update-kernel launches timed (time_kernels = 1) */
    double ms_update;    /* summed HIP-event duration of those launches */
    double ms_comm;      /* sharded builds (time_kernels = 1): device time the streams spent inside
                          * collectives, an event pair around each collective or group, waits for
                          * the peers included (they overlap the update on their own stream) */
    int32_t dist_enc;    /* sparse builds: 4 = u64 distances (wide.hip; the graph's range passes
                          * SRT_INF quanta), 3 = multi-source kernel (64 sources per workgroup),
                          * 2 = workgroup-per-source kernel (LDS-packed rows),
                          * 1 = wave-per-source kernel, 0 = workgroup kernel for every source.
                          * Dense: the distance encoding the build finished with: 12 = bit-parallel
                          * Dial levels (no FW rounds; levels.hip), (9: retired 256-pivot
                          * sharded rounds), 8 = u16
                          * f16-compare row-sharded symmetric rounds of 128 pivots (N > 1;
                          * 4 with SRT_FORM shkb=64), 7 = 5 with
                          * 256-pivot rounds (four panels per C-tile residency), 6 = 5 with
                          * 128-pivot rounds (two panels per C-tile residency), 5 = 4 on two
                          * update streams (one GPU, n >= 8192), 4 = u16 with
                          * f16-compare mins, upper-triangle rounds (undirected; one GPU, or
                          * row-sharded kept tiles in 64-pivot rounds),
                          * 3 = u16 f16-compare (cap 0x3DFF), 2 = u16 pk_min (cap 0x7FFF), 1 = u32 */
    int32_t count_ties;  /* input: 1 = count tied pairs (below) */
    int64_t tied_pairs;  /* pairs (s, t), s != t, whose smallest D[s][u] over the tight
                          * predecessors u of t is reached by two or more u: igraph's heap order
                          * picks the reference's predecessor there (topology.c:1679-1701), the
                          * build takes the smallest u -- the class where reliability can differ */
    int32_t levels;      /* dense level builds (dist_enc 12): the Dial level that settled every pair */
    int64_t work_bytes;  /* algorithmic bytes of the timed launches (level builds: the Delta words
                          * gathered over all levels, counted on the device -- a unit stops early
                          * once its sources are settled), 0 where the bench models them itself */
    double ms_pred;      /* level builds (time_kernels = 1): HIP-event time of the predecessor pass
                          * (lvl_pred_kernel) */
    double ms_rel;       /* ... and of the path-order reliability pass (rel_tree_kernel and the
                          * sweeps of the rows it hands over) */
    int32_t n_derived;   /* sparse full-table builds with derived rows (fw_block bit 64): the rows
                          * formed from their neighbours' (derive.hip), the rest by the kernel;
                          * work_bytes = the derivation's algorithmic bytes */
    double ms_core;      /* ... HIP-event time of the core rows' kernel (with their canonical arcs) */
    double ms_derive;    /* ... and of the derivation (or of the kernel for the set's rows, when a
                          * core row overflowed its buckets: n_derived = 0) */
    int32_t rel_table;   /* dense level builds: the distinct arc reliabilities of the packed post
                          * pass (predecessor | reliability index words); 0 = f64 rows */
    double ms_canon;     /* host clock: the canonical graph (srt_canon_build) */
    double ms_upload;    /* ... the dense matrices filled from it and moved to the device (pinned
                          * two-slot staging; the slowest rank of a sharded build) */
    double ms_download;  /* ... the tables moved into the caller's buffers (same staging) */
} srt_build_stats;

/* Build the full tables for an edge list on one GPU; outputs are host buffers of n*n entries.
 * quantum_ns: the latency quantum (gcd of all edge latencies). Thread-safe per call. */
int srt_build_tables(const srt_edges* g, const srt_build_opts* opts, uint32_t* lat_q,
                     uint64_t* quantum_ns, double* rel, srt_build_stats* stats);

/* srt_build_tables over `ngpus` GPUs of this process (one host thread per GPU, RCCL over xGMI):
 * dense graphs shard rows with the pivot-panel broadcast, sparse graphs shard sources and
 * all-gather. The in-process form Shadow (one process) uses; bench.py runs the same kernels one
 * process per GPU. */
int srt_build_tables_multi(const srt_edges* g, const srt_build_opts* opts, int32_t ngpus,
                           uint32_t* lat_q, uint64_t* quantum_ns, double* rel,
                           srt_build_stats* stats);

/* Tables over a vertex subset -- the vertices with attached hosts, which are the only targets the
 * reference ever computes paths to (topology.c:1604-1656): outputs are nsub x nsub host tables
 * whose entry [i][j] is the pair (verts[i], verts[j]); verts strictly increasing (NULL with
 * nsub = n: every vertex). ngpus > 1 shards the build like srt_build_tables_multi.
 * lat_ms (optional, may be NULL): the path latency as the reference's f64 millisecond sum in path
 * order (topology.c:1308, :1364) -- differs from lat_q * quantum / 1e6 only when some edge latency
 * has a sub-millisecond part. min_lat_q (optional): the smallest table entry, diagonal included
 * (the runahead minimum, topology.c:1253-1264). */
int srt_build_tables_subset(const srt_edges* g, const srt_build_opts* opts, int32_t ngpus,
                            int32_t nsub, const int32_t* verts, uint32_t* lat_q,
                            uint64_t* quantum_ns, double* rel, double* lat_ms, uint32_t* min_lat_q,
                            srt_build_stats* stats);

/* Largest n of the dense (Floyd-Warshall) form; SRT_ALGO_AUTO sends larger graphs, and sparse
 * ones of any size, to the SSSP; an explicit SRT_ALGO_DENSE_FW beyond it fails with SRT_E_RANGE
 * before any work. */
int srt_dense_max_n(void);

/* Quantum and u32-range check used by srt_build_tables. Returns SRT_OK or SRT_E_RANGE. */
int srt_latency_quantum(const srt_edges* g, uint64_t* quantum_ns, uint32_t* max_w_q);

/* ---- device-resident dense build (benchmark / zero-copy path) ----------------------------
 * All pointers are HIP device pointers on the current device; `stream` is a hipStream_t (NULL =
 * default stream). Every matrix is ld x ld row-major with ld % 64 == 0 and ld >= n (rows and
 * columns >= n are padding). w: u32 quanta, diagonal = self-loop (SRT_INF = no edge);
 * r: f64 edge reliability (1 - loss). Outputs lat (u32 quanta) and rel (f64).
 * The predecessor-pass workspace is allocated on first use and cached per device. */
#define SRT_INF 0x7FFFFFFFu
int srt_dense_build_device(int32_t n, int32_t ld, int32_t directed, const uint32_t* w,
                           const double* r, uint32_t* lat, double* rel, void* stream,
                           int32_t fw_block, srt_build_stats* stats);

/* Synthetic graph generators on the device (seeded counter-based hash; identical to
 * shadow_amd/graphs.py so tests can rebuild the same graph on the host). */
/* Rows of nsub sources (device vertex list dverts) on a dense device graph (w, r: ld x ld, as for
 * srt_dense_build_device) without the all-pairs FW: Bellman-Ford passes on u16 quanta, canonical
 * predecessors, path-order reliability, the diagonal rule. lat_rows / rel_rows: nsub x ld (row i =
 * source dverts[i]). SRT_E_RANGE when n > 32768 or a distance reaches the u16 cap. The table
 * builds take this path by themselves when at most n / 12 vertices are attached. */
int srt_dense_rows_build(int32_t n, int32_t ld, int32_t nsub, const int32_t* dverts,
                         const uint32_t* w, const double* r, uint32_t* lat_rows, double* rel_rows,
                         void* stream, srt_build_stats* stats);
int srt_gen_complete_device(int32_t n, int32_t ld, int32_t row0, int32_t nrows, uint64_t seed,
                            uint32_t lat_max_ms, uint32_t self_max_ms, uint32_t loss_max_e4,
                            uint32_t* w, double* r, void* stream);
/* the metric complete graph (Tor-atlas-like): n points of the unit square, latency
 * max(1, round(scale_ms * dist)) ms (scale_ms <= 1024), loss and self-loops as above;
 * oracle/oracle.c orc_metric_sample generates the same weights */
int srt_gen_metric_device(int32_t n, int32_t ld, int32_t row0, int32_t nrows, uint64_t seed,
                          uint32_t scale_ms, uint32_t self_max_ms, uint32_t loss_max_e4,
                          uint32_t* w, double* r, void* stream);

/* ---- device-resident sparse build (CSR of canonical arcs, self-loops excluded) ----------
 * Computes rows [src_begin, src_end) (row r of lat_rows/rel_rows = source src_begin + r, row
 * stride n) with one workgroup per source. The per-source working set (distance row, frontier
 * queue, bitmaps: ~8n + n/8 bytes) is LDS-resident for n <= srt_sparse_max_n() and lives in a
 * per-workgroup HBM slot beyond (persistent grid of 2 workgroups per CU; environment variable
 * SRT_FORM hbm=1 forces the HBM form for testing). delta = bucket width in quanta
 * (0 = default). Each row is its own source's (no symmetry rule is applied: see
 * srt_pair_order). */
int srt_sparse_max_n(void);
int srt_sparse_build_device(int32_t n, int32_t directed, const int32_t* rowptr,
                            const int32_t* col, const uint32_t* w, const double* r,
                            const int32_t* in_rowptr, const int32_t* in_col,
                            const uint32_t* in_w, const double* in_r, const uint32_t* self_w,
                            const double* self_r, int32_t src_begin, int32_t src_end,
                            uint32_t delta, uint32_t* lat_rows, double* rel_rows, void* stream,
                            srt_build_stats* stats);
/* Canonical CSR built on the host from an edge list and uploaded once to `device`; rows of any
 * source range can then be computed on that device (one shard per rank in a sharded build).
 * Replaces the per-source igraph Dijkstra of topology.c:1578-1814 (_topology_computeSourcePaths). */
typedef struct srt_sparse_graph srt_sparse_graph;
int srt_sparse_graph_new(const srt_edges* g, int32_t device, srt_sparse_graph** out);
int srt_sparse_graph_info(const srt_sparse_graph* g, int32_t* n, int32_t* directed, int64_t* arcs,
                          uint64_t* quantum_ns);
int srt_sparse_graph_rows(const srt_sparse_graph* g, int32_t src_begin, int32_t src_end,
                          uint32_t* lat_rows, double* rel_rows, void* stream,
                          srt_build_stats* stats);
/* Rows of an arbitrary source list (srcs: nsrc device ints; row r = source srcs[r], stride n),
 * e.g. the attached vertices. lat_ms_rows (optional): the f64 path-order ms rows -- required when
 * the graph's distances may pass the u32 range (SRT_E_RANGE without it; srt_sparse_graph_rows
 * refuses such a graph the same way). */
int srt_sparse_graph_rows_list(const srt_sparse_graph* g, int32_t nsrc, const int32_t* srcs,
                               uint32_t* lat_rows, double* rel_rows, double* lat_ms_rows,
                               void* stream, srt_build_stats* stats);
void srt_sparse_graph_free(srt_sparse_graph* g);

/* ---- multi-GPU (one process per GPU; RCCL over xGMI) ----------------------------------- */
typedef struct srt_comm srt_comm;
/* 128-byte RCCL unique id, created on rank 0 and shared by the caller (e.g. torch.distributed). */
int srt_comm_unique_id(uint8_t out[128]);
int srt_comm_init(const uint8_t id[128], int32_t nranks, int32_t rank, int32_t device,
                  srt_comm** comm);
void srt_comm_free(srt_comm* comm);
/* In-process communicators for `ndev` devices (ncclCommInitAll): comms[i] drives devices[i]. */
int srt_comm_init_all(int32_t ndev, const int32_t* devices, srt_comm** comms);
/* `nranks` virtual ranks of one process on one device (tests of the sharded schedules on one
 * GPU): each comms[i] is driven by its own host thread; collectives become device-to-device
 * copies ordered by events and host barriers. srt_build_tables_multi uses them when the
 * environment sets SRT_VIRTUAL_RANKS. */
/* Timing only (tools/solo_rank.py): rank `rank` of `nranks` alone on `device`, every collective a
 * no-op, so one rank's compute and critical chain at N ranks is measured without the wire. The
 * tables it produces are NOT correct. */
int srt_comm_init_solo(int32_t nranks, int32_t rank, int32_t device, srt_comm** comm);
/* srt_comm_init_solo with a wire model: each collective holds its stream for lat_us + the bytes
 * this rank receives / gbps (GB/s), spun on the device wall clock; a group pays once, at its end.
 * srt_comm_wire_ms: the modelled wire time issued so far. Timing only, like srt_comm_init_solo. */
int srt_comm_init_solo_wire(int32_t nranks, int32_t rank, int32_t device, double gbps,
                            double lat_us, srt_comm** comm);
double srt_comm_wire_ms(const srt_comm* comm);
/* Collective log: with on != 0 every srt_coll_* call of the communicator appends (op, a, b) --
 * 1 broadcast (bytes, root), 2 all-reduce (count, op_min), 3 all-gather (bytes per rank, 0),
 * 4 exchange (0, 0), 5 group begin, 6 group end, 7 sparse all-gather (rows per rank, n).
 * Enabling clears the log. srt_comm_log_read copies up to cap entries (3 int64 each) into out
 * and returns the number logged. The ranks' logs of one build must be identical (SPMD). */
int srt_comm_log_enable(srt_comm* comm, int32_t on);
int64_t srt_comm_log_read(const srt_comm* comm, int64_t* out, int64_t cap);
/* ranks of the communicator: ncclCommCount for RCCL, nranks for virtual / timing-only ranks */
int srt_comm_count(const srt_comm* comm, int32_t* count);
int srt_comm_init_virtual(int32_t nranks, int32_t device, srt_comm** comms);
/* Bind the calling host thread to virtual rank `rank` on `device` (its own workspaces and
 * streams) before it drives that rank's srt_dense_build_sharded / srt_sparse_graph_rows;
 * rank < 0 returns the thread to the per-device state. */
int srt_virtual_rank_bind(int32_t rank, int32_t device);
/* Row-block partition used by every sharded build: rank r owns rows [begin, end). */
void srt_shard_rows(int32_t n, int32_t align, int32_t nranks, int32_t rank, int32_t* begin,
                    int32_t* end);
/* Dense FW over row shards: each rank passes its rows [begin,end) of w/r (ld columns) and gets
 * the same rows of lat/rel. Pivot-row panels are broadcast with RCCL once per round. */
int srt_dense_build_sharded(srt_comm* comm, int32_t n, int32_t ld, int32_t directed,
                            const uint32_t* w_rows, const double* r_rows, uint32_t* lat_rows,
                            double* rel_rows, void* stream, int32_t fw_block,
                            srt_build_stats* stats);
/* Sparse: each rank computes its source rows, then ncclAllGather assembles the full tables
 * (lat_all: n x n u32, rel_all: n x n f64, each rank's slice written in place). */
int srt_sparse_allgather(srt_comm* comm, int32_t n, int32_t rows_per_rank, uint32_t* lat_all,
                         double* rel_all, void* stream);

/* ---- misc ------------------------------------------------------------------------------ */
const char* srt_version(void);
const char* srt_last_error(void); /* thread-local message for the last failing call */
/* ---- pair order: which cached path the reference serves (pairorder.c) -------------------
 * Restates the lazy cache of topology.c:1166-1265 + :1900-1981 over tables holding every
 * source's raw row: a pair is served, in both directions, from the first source run (or, with
 * use_shortest_path = false, the first direct-edge lookup) that stored it. per_source = 1 for
 * shortest-path mode (a miss runs source s for every attached target, :1578-1814), 0 for direct
 * mode (a miss stores the pair s -> t, :1816-1858). Thread-safe; lookups are lock-free once
 * their pair is stored. */
typedef struct srt_pair_order srt_pair_order;
/* called (under the object's lock) with the paths a lookup stored: src -> targets[i] */
typedef void (*srt_pair_store_fn)(void* ctx, int32_t src, const int32_t* targets, int32_t count);
srt_pair_order* srt_pair_order_new(int32_t n, int32_t directed, int32_t per_source);
void srt_pair_order_free(srt_pair_order* po);
/* v joins the attached set (verticesWithAttachedHosts, topology.c:2231); idempotent */
int srt_pair_order_attach(srt_pair_order* po, int32_t v);
/* lookup (s, t): the source vertex of the path served (s or t), after recording the run or store
 * a miss causes; SRT_E_UNATTACHED if an end is not attached, SRT_E_NOPATH if no stored path
 * joins them (neither end reaches the other) */
int32_t srt_pair_order_lookup(srt_pair_order* po, int32_t s, int32_t t, srt_pair_store_fn on_store,
                              void* ctx);
/* the same without recording anything: -1 while the pair is not stored */
int32_t srt_pair_order_peek(srt_pair_order* po, int32_t s, int32_t t);
/* optional reachability predicate (1: s reaches t); a source run stores only the targets it reaches
 * (topology.c:1744-1753), so on a directed graph that is not strongly connected a pair is decided
 * by the first run from an end that reaches the other. NULL (the default): every pair reachable.
 * Set before the first lookup. */
typedef int (*srt_pair_reach_fn)(void* ctx, int32_t s, int32_t t);
void srt_pair_order_set_reach(srt_pair_order* po, srt_pair_reach_fn fn, void* ctx);
/* recorded source runs of v (one per attach epoch it ran in) */
int32_t srt_pair_order_runs(srt_pair_order* po, int32_t v);
/* the reference's path counters (topology.c:78-79): lookups that would have run a source's
 * Dijkstra (shortestPathCount, :1719; on a directed graph every lookup not served s's own path) and
 * the self paths computed (selfPathCount, :1536); shortest-path mode only */
void srt_pair_order_counts(srt_pair_order* po, uint32_t* source_runs, uint32_t* self_paths);
/* k more source runs (shortest-path mode): a caller that answers with one lookup what the
 * reference does with several -- worker_sendPacket's getReliability, getLatency and
 * incrementPathPacketCounter (worker.c:541-555), each a cache probe that, on a directed graph,
 * runs the source again while the pair is served the other end's path */
void srt_pair_order_add_source_runs(srt_pair_order* po, uint32_t k);

int srt_device_count(void);
int srt_device_sync(int32_t device);

#ifdef __cplusplus
}
#endif

#endif
