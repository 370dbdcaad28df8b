/*
 * topology.h -- drop-in replacement for Shadow's routing header.
 *
 * Reference interface: /root/reference/src/main/routing/topology.h:17-28 (same names, same
 * argument meaning, same error behaviour). glib typedefs are restated with their ABI types
 * (gchar = char, gboolean = int, gdouble = double, guint64 = uint64_t) so the header builds
 * without glib; inside Shadow the glib definitions are ABI-identical.
 *
 * Address / Random stay opaque Shadow types: the implementation calls Shadow's own
 * address_toNetworkIP() (address.h:78), address_toString(), random_nextDouble() (random.c:39)
 * and worker_updateMinTimeJump() (worker.c:627). Weak fallbacks for standalone use live in
 * shadow_amd/csrc/shadow_compat.c and are overridden by Shadow's strong symbols at link time.
 */
#ifndef SRT_TOPOLOGY_H
#define SRT_TOPOLOGY_H

#include <stdint.h>

#include "shadow_routing.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct _Topology Topology;
typedef struct _Address Address;
typedef struct _Random Random;

/* ---- reference signatures (topology.h:17-28) -------------------------------------------- */
/* topology.c:2328-2354: load + validate the GML file, extract edge weights; NULL on failure. */
Topology* topology_new(const char* graphPath, int useShortestPath);
/* topology.c:2283-2326 */
void topology_free(Topology* top);
/* topology.c:2218-2272: choose a vertex for the address from the hints (exact IP > city >
 * country > all; LPM or rand_r pick) and report the vertex bandwidths in KiB/s. */
void topology_attach(Topology* top, Address* address, Random* randomSourcePool, char* ipHint,
                     char* citycodeHint, char* countrycodeHint, uint64_t* bwDownOut,
                     uint64_t* bwUpOut);
/* topology.c:2274-2281 */
void topology_detach(Topology* top, Address* address);
/* topology.c:2019-2022 */
int topology_isRoutable(Topology* top, Address* srcAddress, Address* dstAddress);
/* topology.c:1995-2005: path latency in ms, -1 if an endpoint is not attached */
double topology_getLatency(Topology* top, Address* srcAddress, Address* dstAddress);
/* topology.c:2007-2017: path reliability in [0,1], -1 if an endpoint is not attached */
double topology_getReliability(Topology* top, Address* srcAddress, Address* dstAddress);
/* topology.c:1983-1993: panics (abort) if the path cannot be found */
void topology_incrementPathPacketCounter(Topology* top, Address* srcAddress, Address* dstAddress);

/* ---- additions behind the same ABI -------------------------------------- */
/* Eager build on the GPU(s) of the tables over the vertices with attached hosts -- the only
 * targets the reference computes paths to (topology.c:1604-1656) -- or over every vertex while
 * nothing is attached. Call it after the hosts are attached (controller.c:367); it is idempotent,
 * and the lookups call it lazily: a lookup whose vertex joined the attached set after the last
 * build rebuilds. The tables hold every source's own row; which row serves a pair follows the
 * reference's lazy cache (the first source run that stored the pair, topology.c:1189-1215,
 * :1900-1981; see srt_pair_order in shadow_routing.h). Runahead: the lookups hand
 * worker_updateMinTimeJump() each smaller path latency as their runs store paths, as
 * _topology_storePathInCache does (topology.c:1253-1264); the eager build itself stores none. */
int topology_computeShortestPaths(Topology* top, int nGPUs);
/* Zero-copy view of the current tables (valid until topology_free): n x n over the table's
 * vertices (srt_topology_table_info gives them; every vertex when the table is full). Entry
 * [i][j] is source verts[i]'s own path to verts[j]; a lookup may be served the [j][i] entry. */
int topology_getTable(Topology* top, const uint32_t** latQ, uint64_t* quantumNs,
                      const double** rel, int* n);
/* The current table's vertices (increasing), their count, and the f64 path-order ms table (NULL
 * when every edge latency is whole ms: lat_q * quantum / 1e6 is then the reference's value). */
int srt_topology_table_info(Topology* top, const int32_t** verts, int32_t* nslot,
                            const double** latMs);
/* The reference's diagnostics (topology.c:78-79, logged by _topology_clearCache at :1142-1164,
 * which topology_free also logs): lookups that would have run a source's Dijkstra
 * (shortestPathCount) and self paths computed (selfPathCount); and the table builds this
 * topology ran with their device time (HIP events, the analogue of USE_PERF_TIMERS'
 * shortestPathTotalTime). Any pointer may be NULL. */
int srt_topology_path_counts(Topology* top, uint32_t* shortestPathCount, uint32_t* selfPathCount,
                             int32_t* builds, double* buildSeconds);
/* Receive the runahead minimum instead of worker_updateMinTimeJump (tests, embedders); NULL
 * restores the Shadow call. Process-wide. */
void srt_set_min_time_jump_hook(void (*fn)(double minPathLatencyMs));

/* ---- network-order IP variants (no Shadow types; used by the Python mirror and tests) --- */
Topology* srt_topology_new_from_string(const char* gmlText, int useShortestPath);
int32_t srt_topology_attach_ip(Topology* top, uint32_t ipNet, uint32_t* randState,
                               const char* ipHint, const char* citycodeHint,
                               const char* countrycodeHint, uint64_t* bwDownOut,
                               uint64_t* bwUpOut);
/* Batched attach of nhosts addresses, each exactly as srt_topology_attach_ip
 * in order; per-host rand_r states; hint arrays and output arrays may be NULL. Returns the
 * number attached or a negative SRT_E_* code. Replaces topology.c:2132-2272 per host. */
int32_t srt_topology_attach_batch_ip(Topology* top, int32_t nhosts, const uint32_t* ipNet,
                                     uint32_t* randStates, const char* const* ipHints,
                                     const char* const* citycodeHints,
                                     const char* const* countrycodeHints, int32_t* outVertex,
                                     uint64_t* bwDownOut, uint64_t* bwUpOut);
void srt_topology_detach_ip(Topology* top, uint32_t ipNet);
/* tables the IP -> vertex map holds (the current one + replaced ones not yet reclaimed); stays
 * bounded under attach / detach cycles (diagnostic) */
int64_t srt_topology_ipmap_tables(Topology* top);
int32_t srt_topology_vertex_of_ip(Topology* top, uint32_t ipNet);
double srt_topology_latency_ip(Topology* top, uint32_t srcIpNet, uint32_t dstIpNet);
double srt_topology_reliability_ip(Topology* top, uint32_t srcIpNet, uint32_t dstIpNet);
int srt_topology_increment_ip(Topology* top, uint32_t srcIpNet, uint32_t dstIpNet);
/* packets counted on the path a lookup (src, dst) is served from; 0 while it is not stored
 * (computes nothing) */
uint64_t srt_topology_packet_count_ip(Topology* top, uint32_t srcIpNet, uint32_t dstIpNet);
/* source vertex of the path a lookup (src, dst) is served from, -1 while not stored (peek) */
int32_t srt_topology_path_source_ip(Topology* top, uint32_t srcIpNet, uint32_t dstIpNet);
/* Packet-path consumer (worker.c:541-555): deliver/drop decision, delay in ns and the packet
 * counter for one packet (1 delivered, 0 dropped, < 0 error) or a trace of them. */
int srt_topology_send_packet_ip(Topology* top, uint32_t srcIpNet, uint32_t dstIpNet, double chance,
                                int bootstrapping, uint64_t payloadLength, uint64_t* delayNs);
int srt_topology_send_packets_ip(Topology* top, int64_t count, const uint32_t* srcIpNet,
                                 const uint32_t* dstIpNet, const double* chance,
                                 const uint8_t* bootstrapping, const uint64_t* payloadLength,
                                 uint8_t* delivered, uint64_t* delayNs);
/* Graph facts established by validation (topology.c:659-716). */
int32_t srt_topology_vertex_count(Topology* top);
int64_t srt_topology_edge_count(Topology* top);
int srt_topology_is_directed(Topology* top);
int srt_topology_is_complete(Topology* top);
/* Validated canonical edge arrays (GML order) -- the input of the device build. */
int srt_topology_edges(Topology* top, srt_edges* out);
/* Minimum latency (ms) over pairs of attached vertices incl. the diagonal (runahead export,
 * controller.c:141-153); 0 if nothing is attached. */
double srt_topology_min_latency_ms(Topology* top);
/* Select the algorithm / device for topology_computeShortestPaths. */
void srt_topology_set_build_opts(Topology* top, const srt_build_opts* opts);
int srt_topology_last_stats(Topology* top, srt_build_stats* stats);

#ifdef __cplusplus
}
#endif

#endif
