/*
 * srt_device.h -- shared device-side definitions for the gfx950 kernels.
 */
#ifndef SRT_DEVICE_H
#define SRT_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "srt_internal.h"

/* a running maximum many workgroups raise once each (per-row depth counters): read it first, so
 * the same-address atomic -- serialised at the memory side, ~12 ns each -- runs only to raise it */
static __device__ __forceinline__ void srt_max_once(int32_t* p, int v) {
    if (v > __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(p, v);
}

#define SRT_HIPCHK(expr)                                                                   \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            srt_set_error("HIP error %s at %s:%d (%s)", hipGetErrorString(e_), __FILE__,   \
                          __LINE__, #expr);                                                \
            return SRT_E_DEVICE;                                                           \
        }                                                                                  \
    } while (0)

/* Per-thread slot of the static per-device state (workspaces, event pools, FW buffers and
 * streams): the current device (0..63), or 64 + r for virtual rank r when several ranks share
 * one device inside one process (srt_build_tables_multi with SRT_VIRTUAL_RANKS, comm.hip). */
#define SRT_STATE_SLOTS 128
/* the neighbour-row derivation's largest source degree (build.hip picks I, derive.hip sizes its
 * per-thread neighbour arrays by it) */
#define SRT_DERIVE_MAXDEG 4
int srt_state_slot(void);
/* stream-ordered scratch from the library's private pool of the current device (comm.hip) */
hipMemPool_t srt_scratch_pool(void);
#define srt_malloc_async(ptr, bytes, st) \
    hipMallocFromPoolAsync((void**)(ptr), (bytes), srt_scratch_pool(), (st))
void srt_set_virtual_slot(int rank); /* -1: back to the device slot */

/* Collectives over an srt_comm: RCCL, or (virtual ranks on one device) device-to-device copies
 * ordered by events and host barriers. Every rank calls the same sequence. */
int srt_coll_bcast(const srt_comm* c, void* buf, size_t bytes, int root, hipStream_t st);
int srt_coll_allreduce_i32(const srt_comm* c, int32_t* buf, size_t count, int op_min,
                           hipStream_t st);
int srt_coll_group_begin(const srt_comm* c);
int srt_coll_group_end(const srt_comm* c);
/* point-to-point exchange: to each peer q send send_bytes[q] from send[q], receive
 * recv_bytes[q] into recv[q] (arrays of comm size; zero bytes skip the pair) */
int srt_coll_exchange(const srt_comm* c, void* const* send, const size_t* send_bytes,
                      void* const* recv, const size_t* recv_bytes, hipStream_t st);
int srt_comm_rank(const srt_comm* c);
int srt_comm_is_solo(const srt_comm* c); /* timing-only communicator (srt_comm_init_solo) */
int srt_comm_size(const srt_comm* c);
/* ms_comm: on = 1 starts timing every collective (or group) of c with an event pair;
 * srt_comm_timing_ms waits for the last one and returns the summed spans (ms) */
void srt_comm_timing(const srt_comm* c, int on);
double srt_comm_timing_ms(const srt_comm* c);

/* pivot-block edge of the blocked Floyd-Warshall and the output-tile edge of its kernels */
#define SRT_FW_B 64
/* row-shard alignment of every sharded dense build (the u16 update tile is 128 rows) */
#define SRT_SHARD_ALIGN 128
/* LDS row stride (u32) of a 64-wide tile: +4 keeps 16-byte alignment for ds_read_b128 */
#define SRT_FW_LDT (SRT_FW_B + 4)

/* counter-based generator hash (shadow_amd/graphs.py restates it bit for bit) */
__host__ __device__ static inline uint64_t srt_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__host__ __device__ static inline uint64_t srt_hash(uint64_t seed, uint64_t stream, uint32_t i,
                                                    uint32_t j) {
    return srt_splitmix64(srt_splitmix64(seed * 4ull + stream) ^ (((uint64_t)i << 32) | j));
}

static inline int srt_ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

/* internal (C++ linkage) entry points shared between translation units */
/* HIP events bracketing every FW update launch (stats->time_kernels): the per-launch duration
 * of the dominant kernel that bench.py reports against the roofline. */
typedef struct {
    hipEvent_t* ev;
    int cap, used;
    /* 2: (start, end) per timed launch; 4: (start A, start B, end A, end B) per round for the
     * launch pairs of two update streams, which drift apart and overlap across rounds: the unit's
     * time is their period, (last end - first start) / pairs */
    int group;
} evpool_t;

evpool_t* srt_evpool(int dev);


static inline int evpool_begin(evpool_t** out, int rounds) {
    evpool_t* p = srt_evpool(srt_state_slot());
    if (p->cap < 4 * rounds) {
        hipEvent_t* ne = (hipEvent_t*)realloc(p->ev, sizeof(hipEvent_t) * 4 * rounds);
        if (!ne) return SRT_E_NOMEM;
        p->ev = ne;
        for (int i = p->cap; i < 4 * rounds; i++) SRT_HIPCHK(hipEventCreate(&p->ev[i]));
        p->cap = 4 * rounds;
    }
    p->used = 0;
    p->group = 2;
    *out = p;
    return SRT_OK;
}

/* grow the pool to at least n events without resetting what it holds */
static inline int evpool_reserve(evpool_t* p, int n) {
    if (p->cap >= n) return SRT_OK;
    hipEvent_t* ne = (hipEvent_t*)realloc(p->ev, sizeof(hipEvent_t) * n);
    if (!ne) return SRT_E_NOMEM;
    p->ev = ne;
    for (int i = p->cap; i < n; i++) SRT_HIPCHK(hipEventCreate(&p->ev[i]));
    p->cap = n;
    return SRT_OK;
}

static inline int evpool_sum(evpool_t* p, hipEvent_t last, srt_build_stats* stats) {
    SRT_HIPCHK(hipEventSynchronize(last));
    double tot = 0;
    const int g = p->group == 4 ? 4 : 2;
    if (g == 2) {
        for (int i = 0; i + 1 < p->used; i += 2) {
            float ms = 0;
            SRT_HIPCHK(hipEventElapsedTime(&ms, p->ev[i], p->ev[i + 1]));
            tot += ms;
        }
    } else if (p->used >= 4) { /* relative to the first start A */
        const int l = p->used - 4;
        float sb = 0, ea = 0, eb = 0;
        SRT_HIPCHK(hipEventElapsedTime(&sb, p->ev[0], p->ev[1]));
        SRT_HIPCHK(hipEventElapsedTime(&ea, p->ev[0], p->ev[l + 2]));
        SRT_HIPCHK(hipEventElapsedTime(&eb, p->ev[0], p->ev[l + 3]));
        tot = (ea > eb ? ea : eb) - (sb < 0 ? sb : 0);
    }
    stats->ms_update = tot;
    stats->n_update = p->used / g;
    return SRT_OK;
}


typedef int (*srt_panel_bcast_fn)(void* ctx, void* panel, size_t bytes, int owner, hipStream_t st);
typedef int (*srt_owner_fn)(void* ctx, int k0);
/* packed-u16 Floyd-Warshall over a row shard (fw16.hip). d16: nrows x ld u16. *sym = 1 on input
 * (undirected, symmetric w) lets a single-shard f16-compare build update only upper-triangle tiles;
 * on output it says whether that form ran (sym may be NULL). fm = 1 selects the
 * f16-compare instruction mix (cap 0x3DFF), fm = 0 the v_pk_min_u16 mix (cap 0x7FFF). Returns
 * SRT_OK and *exact = 1 when every distance is below the cap (else the caller reruns with the
 * next wider path). lat_rows receives the distances widened to u32 quanta. */
/* row-sharded symmetric rounds (undirected, f16-compare path, >= 2 ranks; fw16.hip) */
int srt_fw16_build_sym_sharded(const srt_comm* comm, int n, int ld, int row0, int nrows,
                               const uint32_t* w_rows, uint32_t* lat_rows, hipStream_t st,
                               evpool_t* evp, int* exact);
int srt_fw16_build(int n, int ld, int row0, int nrows, const uint32_t* w_rows, uint32_t* lat_rows,
                   hipStream_t st, evpool_t* evp, srt_owner_fn owner_of, srt_panel_bcast_fn bcast,
                   void* ctx, int rank, int fm, int* sym, int* exact);
/* levels.hip: distance rows of the local sources by bit-parallel Dial levels (see there) */
int srt_levels_build(const srt_comm* comm, int n, int ld, int row0, int nrows, int directed,
                     const uint32_t* w_rows, const double* r_rows, uint32_t* lat_rows, double fw_ms,
                     hipStream_t st, evpool_t* evp, int* levels, int64_t* gather_bytes);
/* predecessors (int16 when pred16, else int32) + arc reliabilities of the held level build
 * (target-major, row stride ldp) */
int srt_levels_pred(void* predT, int pred16, double* rT, size_t ldp, unsigned long long* ties,
                    hipStream_t st);
/* 1 when the held level build's post pass is the packed-word form (srt_levels_pred with pred16 = 2:
 * pred | reliability index << 16 | level << 27 per pair, one transpose, then rel_pk_kernel writes
 * the u32 rows too); 0: the u8 level rows + srt_levels_pred + rel_tree_kernel */
int srt_levels_pkw_ready(void);
/* frees the held level build (stream-ordered) */
void srt_levels_release(hipStream_t st);
/* the held build's u8 distance rows (nrows x ld, 0 on the diagonal), NULL if none */
const uint8_t* srt_levels_l8(void);
/* the held level build's distinct arc reliabilities (the packed post pass: predecessor | index << 16
 * words, srt_levels_pred with pred16 = 2); NULL (ntab 0) when the build keeps the f64 form */
const double* srt_levels_rtab(int* ntab);
/* the diagonal rule of the held build's rows (keys from its row reads); *applied = 0 when it kept
 * none (directed builds: dense_diag_kernel) */
int srt_levels_diag(int n, int ld, uint32_t* d, double* rel, hipStream_t st, int* applied);
/* the same into this slot's FW matrix + the finish pass (fw16.hip); *nlev = 0: FW instead */
int srt_fw16_levels(const srt_comm* comm, int n, int ld, int row0, int nrows, int directed,
                    const uint32_t* w_rows, const double* r_rows, uint32_t* lat_rows,
                    hipStream_t st, evpool_t* evp, double fw_ms, int* nlev, int64_t* bytes);
/* the u16 working matrix of the last srt_fw16_build on the current device (row shard x ld) */
const uint16_t* srt_fw16_matrix(void);
/* 1 when every real distance of that build is <= 254 quanta (the post pass then reads u8) */
int srt_fw16_small(void);
/* distance encodings of the dense build, reported (negated) in srt_build_stats.fw_block */
enum {
    SRT_DENC_U32 = 1,
    SRT_DENC_U16 = 2,
    SRT_DENC_F16CMP = 3,
    SRT_DENC_F16CMP_SYM = 4,
    SRT_DENC_F16CMP_SYM2 = 5, /* one GPU, upper triangle on two update streams */
    SRT_DENC_F16CMP_SYM128 = 6, /* 5 with 128-pivot rounds (8-wave update, 4 stages per tile) */
    SRT_DENC_F16CMP_SYM256 = 7, /* 5 with 256-pivot rounds (8 stages per tile) */
    SRT_DENC_F16CMP_SYMSH128 = 8, /* 4 (row-sharded, >= 2 ranks) with 128-pivot rounds */
    SRT_DENC_F16CMP_SYMSH256 = 9, /* 4 (row-sharded) with 256-pivot rounds */
    SRT_DENC_ROWS = 10,           /* a few source rows by Bellman-Ford passes, no FW */
    SRT_DENC_SQUARE = 11,         /* ld <= 2048 on one GPU: min-plus squaring to a fixed point */
    SRT_DENC_LEVELS = 12          /* bit-parallel Dial levels (levels.hip), no FW rounds */
};
int srt_dense_rows_build_device(int32_t n, int32_t ld, int32_t nsub, const int32_t* dverts,
                                const uint32_t* w, const double* r, uint32_t* lat_rows,
                                double* rel_rows, double* lms_rows, uint64_t quantum_ns,
                                int32_t directed, hipStream_t st, srt_build_stats* stats, int* used);
/* pivots per round of this thread's last srt_fw16_build_sym_sharded (64 or 128) */
int srt_fw16_sharded_round_pivots(void);
/* distance rows of nsub sources on a dense graph by Bellman-Ford passes on u16 quanta (fw16.hip);
 * w16: ld x ld scratch, ds: (nsub rounded up to 128) x ld scratch, lat_rows: nsub x ld u32 */
int srt_fw16_rows(int n, int ld, int nsub, const int32_t* dverts, const uint32_t* w, uint16_t* w16,
                  uint16_t* ds, uint32_t* lat_rows, hipStream_t st, int* exact, int* small,
                  int* passes);

int srt_dense_post_device(int32_t n, int32_t ld, int32_t directed, const uint32_t* w,
                          const double* r, uint32_t* d, const uint16_t* d16, double* rel,
                          hipStream_t st, srt_build_stats* stats, int lvl);

/* Largest dense n: the predecessor keys pack a 16-bit rank and the essential-arc offsets are
 * int32 (n^2 < 2^31), rounded down to the 128 tile. */
#define SRT_DENSE_MAX_N 46336
/* Dense builds with the optional f64 path-order ms table (lat_ms / lms_rows may be NULL). */
int srt_dense_build_device_ms(int32_t n, int32_t ld, int32_t directed, const uint32_t* w,
                              const double* r, uint32_t* lat, double* rel, double* lat_ms,
                              uint64_t quantum_ns, hipStream_t st, int32_t fw_block,
                              srt_build_stats* stats);
int srt_dense_build_sharded_ms(srt_comm* comm, int32_t n, int32_t ld, int32_t directed,
                               const uint32_t* w_rows, const double* r_rows, uint32_t* lat_rows,
                               double* rel_rows, double* lms_rows, uint64_t quantum_ns,
                               hipStream_t st, int32_t fw_block, srt_build_stats* stats);

/* tables.hip: path-order passes, sub-table gathers, table minimum */
int srt_path_sweeps_max_n(void);
/* out rows (f64 ms, path order) of nrows sources (srcs[r], or src_begin + r) from their distance
 * rows D (diagonal rule applied) and either predecessor rows or the in-arc CSR */
int srt_path_ms_rows(int n, int nrows, const int32_t* srcs, int src_begin, const uint32_t* D,
                     size_t ldd, const int32_t* pred, size_t ldp, const int32_t* irp,
                     const int32_t* icol, const uint32_t* iw, uint64_t quantum_ns, double* out,
                     size_t ldo, hipStream_t st);
int srt_rel_sweeps_rows(int n, int nrows, int row0, const int32_t* pred, size_t ldp, double* rel,
                        size_t ldr, const int32_t* only, int32_t* max_depth, hipStream_t st);
int srt_gather_sub_u32(int nr, int nc, const int32_t* rows, const int32_t* cols, const uint32_t* in,
                       size_t ldi, uint32_t* out, size_t ldo, hipStream_t st);
int srt_gather_sub_f64(int nr, int nc, const int32_t* rows, const int32_t* cols, const double* in,
                       size_t ldi, double* out, size_t ldo, hipStream_t st);
int srt_table_min(int rows, int cols, const uint32_t* t, size_t ld, uint32_t* dmin, hipStream_t st);
/* dense matrices from the edge list on the device (tables.hip): prepare (all-ones), the minimum
 * latency per pair into r's bits, the lowest index among the minima into w, then in place the
 * quanta / reliabilities (SRT_INF / 0 where no edge) with the off-diagonal arcs counted */
int srt_scatter_prepare(int nrows, int ld, uint32_t* w, double* r, hipStream_t st);
int srt_scatter_min(int64_t m, const int32_t* src, const int32_t* dst, const int64_t* lat, int directed,
                    int32_t row0, int nrows, int ld, double* r, hipStream_t st);
int srt_scatter_idx(int64_t m, const int32_t* src, const int32_t* dst, const int64_t* lat, int directed,
                    int32_t row0, int nrows, int ld, const double* r, uint32_t* w, hipStream_t st);
int srt_scatter_final(int32_t row0, int nrows, int ld, uint64_t q, const double* loss, uint32_t* w,
                      double* r, unsigned long long* arcs, hipStream_t st);
/* adds the tied pairs of nrows distance rows (diagonal rule applied) to *tied */
int srt_tie_count_rows(int n, int nrows, const int32_t* srcs, int src_begin, const uint32_t* D,
                       size_t ldd, const int32_t* irp, const int32_t* icol, const uint32_t* iw,
                       int64_t* tied, hipStream_t st);
int srt_quanta_to_ms(int rows, int cols, const uint32_t* w, size_t ldw, uint64_t q, double* out,
                     size_t ldo, hipStream_t st);
/* collectives: all-gather of equal byte blocks, rank q's block at buf + q * bytes */
int srt_coll_allgather(const srt_comm* c, void* buf, size_t bytes, hipStream_t st);

#endif
