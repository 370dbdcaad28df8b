/*
 * comm.hip -- multi-GPU plumbing: RCCL communicator (one process per GPU, xGMI inside the node)
 * and the row-block partition shared by every sharded build.
 *
 * The reference has no multi-device code at all: these collectives are new.
 * Dense builds broadcast one pivot-row panel per Floyd-Warshall round; sparse builds shard the
 * sources and assemble the tables with one ncclAllGather.
 */
#include <pthread.h>
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include "srt_device.h"

/* Virtual ranks: several ranks of one process on one device (tests of the sharded schedules on
 * a one-GPU box; RCCL refuses two ranks on one device). Collectives become device-to-device
 * copies on the callers' streams, ordered by events; host barriers line the ranks up at each
 * call, which every rank makes in the same order (SPMD), as with RCCL. */
typedef struct srt_loop {
    int nranks, refs;
    pthread_barrier_t bar;
    pthread_mutex_t mu;
    void** ptr;           /* per rank: its buffer of the current call */
    void** sendp;         /* [from * R + to] */
    size_t* sendb;        /* [from * R + to] */
    hipEvent_t* ready;    /* per rank: its inputs are written */
    hipEvent_t* done;     /* per rank: it has read what it needs */
} srt_loop;

struct srt_comm {
    ncclComm_t nc;
    int nranks, rank, device;
    srt_loop* loop; /* non-NULL: virtual ranks */
    int solo;       /* timing only: one rank alone, every collective a no-op (srt_comm_init_solo) */
    /* solo wire model (srt_comm_init_solo_wire): each collective occupies its stream for
     * wire_lat_us + bytes received / wire_gbps; a group's bytes are summed and paid at its end */
    double wire_gbps, wire_lat_us, wire_ticks_per_us;
    int in_group;
    size_t group_bytes;
    double wire_us_total; /* modelled wire time issued on the streams (ms_comm of a solo build) */
    /* srt_build_stats.ms_comm: an event pair around every collective (or group) while timing is
     * on -- the device time the streams spend inside collectives, waits for the peers included */
    int timing, t_open;
    hipEvent_t* tev;
    int tcap, tused;
    hipStream_t t_stream; /* the stream the open group's first collective named */
    /* collective log (srt_comm_log_enable): (op, a, b) per call, in call order -- what the ranks'
     * sequences are compared by (tests/test_gpu_protocol.py against the gloo rehearsal) */
    int log_on;
    int64_t* logv;
    size_t log_n, log_cap;
};

enum { SRT_LOG_BCAST = 1, SRT_LOG_ALLREDUCE, SRT_LOG_ALLGATHER, SRT_LOG_EXCHANGE, SRT_LOG_GROUP_BEGIN,
       SRT_LOG_GROUP_END, SRT_LOG_SPARSE_ALLGATHER };

static void c_log(const srt_comm* cc, int op, int64_t a, int64_t b) {
    srt_comm* c = const_cast<srt_comm*>(cc);
    if (!c->log_on) return;
    if (c->log_n == c->log_cap) {
        const size_t nc = c->log_cap ? 2 * c->log_cap : 256;
        int64_t* nv = (int64_t*)realloc(c->logv, nc * 3 * sizeof(int64_t));
        if (!nv) return; /* the log stops growing; the comparison then fails on its length */
        c->logv = nv;
        c->log_cap = nc;
    }
    int64_t* e = c->logv + 3 * c->log_n++;
    e[0] = op;
    e[1] = a;
    e[2] = b;
}

extern "C" int srt_comm_log_enable(srt_comm* c, int32_t on) {
    if (!c) {
        srt_set_error("srt_comm_log_enable: bad arguments");
        return SRT_E_ARG;
    }
    c->log_on = on != 0;
    c->log_n = 0;
    return SRT_OK;
}

extern "C" int64_t srt_comm_log_read(const srt_comm* c, int64_t* out, int64_t cap) {
    if (!c) return -1;
    const int64_t k = (int64_t)c->log_n;
    if (out)
        for (int64_t i = 0; i < k && i < cap; i++)
            for (int f = 0; f < 3; f++) out[3 * i + f] = c->logv[3 * i + f];
    return k;
}

static thread_local int t_vslot = -1;
void srt_set_virtual_slot(int rank) { t_vslot = rank; }
/* The builds' stream-ordered scratch (srt_malloc_async / hipFreeAsync) comes from a private
 * pool per device, not the device's default pool: its release threshold (SRT_POOL_KEEP) keeps
 * up to that much freed scratch mapped across synchronisations, so a small build does not re-map
 * its scratch each time (~0.2 ms of a 0.9-ms C2 build), while the caller's own stream-ordered
 * frees (the default pool) keep the default release behaviour, and anything above the threshold
 * goes back to the driver at the next synchronisation. */
#define SRT_POOL_KEEP (4ull << 30)
static hipMemPool_t g_pool[64];
static pthread_mutex_t g_pool_mu = PTHREAD_MUTEX_INITIALIZER;

hipMemPool_t srt_scratch_pool(void) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    hipMemPool_t p = __atomic_load_n(&g_pool[dev & 63], __ATOMIC_ACQUIRE);
    if (p) return p;
    pthread_mutex_lock(&g_pool_mu);
    p = g_pool[dev & 63];
    if (!p) {
        hipMemPoolProps props;
        memset(&props, 0, sizeof(props));
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        if (hipMemPoolCreate(&p, &props) == hipSuccess) {
            uint64_t keep = SRT_POOL_KEEP;
            (void)hipMemPoolSetAttribute(p, hipMemPoolAttrReleaseThreshold, &keep);
        } else {
            (void)hipGetLastError();
            (void)hipDeviceGetDefaultMemPool(&p, dev); /* still correct, only without the cap */
        }
        __atomic_store_n(&g_pool[dev & 63], p, __ATOMIC_RELEASE);
    }
    pthread_mutex_unlock(&g_pool_mu);
    return p;
}

int srt_state_slot(void) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (t_vslot >= 0) return 64 + (t_vslot & 63);
    return dev & 63;
}

#define SRT_NCCLCHK(expr)                                                                  \
    do {                                                                                   \
        ncclResult_t r_ = (expr);                                                          \
        if (r_ != ncclSuccess) {                                                           \
            srt_set_error("RCCL error %s at %s:%d (%s)", ncclGetErrorString(r_), __FILE__, \
                          __LINE__, #expr);                                                \
            return SRT_E_COMM;                                                             \
        }                                                                                  \
    } while (0)

extern "C" int srt_comm_unique_id(uint8_t out[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    SRT_NCCLCHK(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof(id));
    return SRT_OK;
}

extern "C" int srt_comm_init(const uint8_t id[128], int32_t nranks, int32_t rank, int32_t device,
                             srt_comm** comm) {
    if (!id || !comm || nranks < 1 || rank < 0 || rank >= nranks) {
        srt_set_error("srt_comm_init: bad arguments");
        return SRT_E_ARG;
    }
    SRT_HIPCHK(hipSetDevice(device));
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    srt_comm* c = (srt_comm*)calloc(1, sizeof(srt_comm));
    if (!c) return SRT_E_NOMEM;
    ncclResult_t r = ncclCommInitRank(&c->nc, nranks, uid, rank);
    if (r != ncclSuccess) {
        srt_set_error("ncclCommInitRank: %s", ncclGetErrorString(r));
        free(c);
        return SRT_E_COMM;
    }
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    *comm = c;
    return SRT_OK;
}

extern "C" int srt_comm_init_all(int32_t ndev, const int32_t* devices, srt_comm** comms) {
    if (ndev < 1 || !devices || !comms) {
        srt_set_error("srt_comm_init_all: bad arguments");
        return SRT_E_ARG;
    }
    ncclComm_t* nc = (ncclComm_t*)calloc((size_t)ndev, sizeof(ncclComm_t));
    if (!nc) return SRT_E_NOMEM;
    ncclResult_t r = ncclCommInitAll(nc, ndev, devices);
    if (r != ncclSuccess) {
        free(nc);
        srt_set_error("ncclCommInitAll: %s", ncclGetErrorString(r));
        return SRT_E_COMM;
    }
    for (int i = 0; i < ndev; i++) {
        comms[i] = (srt_comm*)calloc(1, sizeof(srt_comm));
        if (!comms[i]) {
            for (int k = 0; k < ndev; k++) {
                (void)ncclCommDestroy(nc[k]);
                free(comms[k]);
                comms[k] = NULL;
            }
            free(nc);
            return SRT_E_NOMEM;
        }
        comms[i]->nc = nc[i];
        comms[i]->nranks = ndev;
        comms[i]->rank = i;
        comms[i]->device = devices[i];
    }
    free(nc);
    return SRT_OK;
}

extern "C" int srt_comm_init_virtual(int32_t nranks, int32_t device, srt_comm** comms) {
    if (nranks < 1 || nranks > 64 || !comms) {
        srt_set_error("srt_comm_init_virtual: bad arguments");
        return SRT_E_ARG;
    }
    SRT_HIPCHK(hipSetDevice(device));
    srt_loop* L = (srt_loop*)calloc(1, sizeof(srt_loop));
    if (!L) return SRT_E_NOMEM;
    const int R = nranks;
    L->nranks = R;
    L->refs = R;
    L->ptr = (void**)calloc((size_t)R, sizeof(void*));
    L->sendp = (void**)calloc((size_t)R * R, sizeof(void*));
    L->sendb = (size_t*)calloc((size_t)R * R, sizeof(size_t));
    L->ready = (hipEvent_t*)calloc((size_t)R, sizeof(hipEvent_t));
    L->done = (hipEvent_t*)calloc((size_t)R, sizeof(hipEvent_t));
    if (!L->ptr || !L->sendp || !L->sendb || !L->ready || !L->done) return SRT_E_NOMEM;
    pthread_barrier_init(&L->bar, NULL, (unsigned)R);
    pthread_mutex_init(&L->mu, NULL);
    for (int i = 0; i < R; i++) {
        SRT_HIPCHK(hipEventCreateWithFlags(&L->ready[i], hipEventDisableTiming));
        SRT_HIPCHK(hipEventCreateWithFlags(&L->done[i], hipEventDisableTiming));
        comms[i] = (srt_comm*)calloc(1, sizeof(srt_comm));
        if (!comms[i]) return SRT_E_NOMEM;
        comms[i]->nranks = R;
        comms[i]->rank = i;
        comms[i]->device = device;
        comms[i]->loop = L;
    }
    return SRT_OK;
}

/* Timing-only communicator: rank `rank` of `nranks` runs its own schedule alone on `device` and
 * every collective returns at once without moving data, so the tables are NOT correct. It
 * measures one rank's compute and critical chain at N ranks without the wire
 * (tools/solo_rank.py); never used by a build that returns tables. */
extern "C" int srt_comm_init_solo(int32_t nranks, int32_t rank, int32_t device, srt_comm** comm) {
    if (nranks < 1 || rank < 0 || rank >= nranks || !comm) {
        srt_set_error("srt_comm_init_solo: bad arguments");
        return SRT_E_ARG;
    }
    SRT_HIPCHK(hipSetDevice(device));
    srt_comm* c = (srt_comm*)calloc(1, sizeof(srt_comm));
    if (!c) return SRT_E_NOMEM;
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    c->solo = 1;
    *comm = c;
    return SRT_OK;
}

/* srt_comm_init_solo plus a wire model: every collective holds its stream for
 * lat_us + (bytes this rank receives) / gbps, as a spin on the device's constant-rate wall clock,
 * so one rank's schedule feels a wire of that speed without the peers (the other ranks' sends
 * are what it waits for on a real node). gbps <= 0: no wire (srt_comm_init_solo). */
extern "C" int srt_comm_init_solo_wire(int32_t nranks, int32_t rank, int32_t device, double gbps,
                                       double lat_us, srt_comm** comm) {
    int rc = srt_comm_init_solo(nranks, rank, device, comm);
    if (rc) return rc;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess ||
        khz <= 0) {
        srt_comm_free(*comm);
        *comm = NULL;
        srt_set_error("srt_comm_init_solo_wire: no wall-clock rate on device %d", device);
        return SRT_E_DEVICE;
    }
    (*comm)->wire_gbps = gbps;
    (*comm)->wire_lat_us = lat_us > 0 ? lat_us : 0.0;
    (*comm)->wire_ticks_per_us = (double)khz / 1000.0;
    return SRT_OK;
}

/* one wave spins until `ticks` of the constant-rate wall clock have passed (s_memrealtime) */
__global__ __launch_bounds__(64) void wire_spin_kernel(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

/* the stream a solo group's wire time is paid on: the one its first collective names */
static thread_local hipStream_t t_group_stream = nullptr;

static int solo_wire(const srt_comm* cc, size_t bytes, hipStream_t st) {
    srt_comm* c = const_cast<srt_comm*>(cc);
    if (c->wire_gbps <= 0.0) return SRT_OK;
    if (c->in_group) {
        c->group_bytes += bytes;
        if (!t_group_stream) t_group_stream = st;
        return SRT_OK;
    }
    const double us = c->wire_lat_us + (double)bytes / (c->wire_gbps * 1e3);
    c->wire_us_total += us;
    wire_spin_kernel<<<1, 64, 0, st>>>((uint64_t)(us * c->wire_ticks_per_us + 0.5));
    SRT_HIPCHK(hipGetLastError());
    return SRT_OK;
}

extern "C" double srt_comm_wire_ms(const srt_comm* c) { return c ? c->wire_us_total * 1e-3 : 0.0; }

/* ---- collective timing (srt_build_stats.ms_comm) ----------------------------------------- */
void srt_comm_timing(const srt_comm* cc, int on) {
    srt_comm* c = const_cast<srt_comm*>(cc);
    if (!c) return;
    c->timing = on;
    c->tused = 0;
    c->t_open = 0;
}

static int t_record(srt_comm* c, hipStream_t st) {
    if (c->tused == c->tcap) {
        const int nc = c->tcap ? 2 * c->tcap : 512;
        hipEvent_t* ne = (hipEvent_t*)realloc(c->tev, sizeof(hipEvent_t) * (size_t)nc);
        if (!ne) return SRT_E_NOMEM;
        c->tev = ne;
        for (int i = c->tcap; i < nc; i++) SRT_HIPCHK(hipEventCreate(&c->tev[i]));
        c->tcap = nc;
    }
    SRT_HIPCHK(hipEventRecord(c->tev[c->tused++], st));
    return SRT_OK;
}

/* before a collective on st: opens its span (inside a group, only the group's first one does) */
static int t_begin(const srt_comm* cc, hipStream_t st) {
    srt_comm* c = const_cast<srt_comm*>(cc);
    if (!c->timing) return SRT_OK;
    if (c->in_group) {
        if (c->t_open) return SRT_OK;
        c->t_open = 1;
        c->t_stream = st;
    }
    return t_record(c, st);
}

/* after a collective on st (outside a group), or at the group's end */
static int t_end(const srt_comm* cc, hipStream_t st) {
    srt_comm* c = const_cast<srt_comm*>(cc);
    if (!c->timing || c->in_group) return SRT_OK;
    return t_record(c, st);
}

double srt_comm_timing_ms(const srt_comm* cc) {
    srt_comm* c = const_cast<srt_comm*>(cc);
    if (!c || !c->timing || c->tused < 2) return 0.0;
    if (hipEventSynchronize(c->tev[c->tused - 1]) != hipSuccess) return -1.0;
    double tot = 0.0;
    for (int i = 0; i + 1 < c->tused; i += 2) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, c->tev[i], c->tev[i + 1]) == hipSuccess) tot += ms;
    }
    return tot;
}

/* RCCL ranks of the communicator (ncclCommCount); virtual and timing-only ranks report theirs */
extern "C" int srt_comm_count(const srt_comm* c, int32_t* count) {
    if (!c || !count) {
        srt_set_error("srt_comm_count: bad arguments");
        return SRT_E_ARG;
    }
    if (c->loop || c->solo) {
        *count = c->nranks;
        return SRT_OK;
    }
    int k = 0;
    SRT_NCCLCHK(ncclCommCount(c->nc, &k));
    *count = k;
    return SRT_OK;
}

extern "C" int srt_virtual_rank_bind(int32_t rank, int32_t device) {
    srt_set_virtual_slot(rank);
    SRT_HIPCHK(hipSetDevice(device));
    return SRT_OK;
}

extern "C" void srt_comm_free(srt_comm* comm) {
    if (!comm) return;
    if (comm->loop) {
        srt_loop* L = comm->loop;
        pthread_mutex_lock(&L->mu);
        const int last = --L->refs == 0;
        pthread_mutex_unlock(&L->mu);
        if (last) {
            for (int i = 0; i < L->nranks; i++) {
                (void)hipEventDestroy(L->ready[i]);
                (void)hipEventDestroy(L->done[i]);
            }
            pthread_barrier_destroy(&L->bar);
            pthread_mutex_destroy(&L->mu);
            free(L->ptr);
            free(L->sendp);
            free(L->sendb);
            free(L->ready);
            free(L->done);
            free(L);
        }
    } else if (!comm->solo) {
        (void)ncclCommDestroy(comm->nc);
    }
    for (int i = 0; i < comm->tcap; i++) (void)hipEventDestroy(comm->tev[i]);
    free(comm->tev);
    free(comm->logv);
    free(comm);
}

/* ---- collectives ------------------------------------------------------------------------ */
static void loop_wait(srt_loop* L) { pthread_barrier_wait(&L->bar); }

__global__ void allreduce_i32_kernel(int32_t* __restrict__ dst, const int32_t* __restrict__ src,
                                     size_t count, int op_min) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) dst[i] = op_min ? min(dst[i], src[i]) : dst[i] + src[i];
}

static int bcast_impl(const srt_comm* c, void* buf, size_t bytes, int root, hipStream_t st) {
    if (c->solo) return root == c->rank ? solo_wire(c, 0, st) : solo_wire(c, bytes, st);
    if (!c->loop) {
        SRT_NCCLCHK(ncclBroadcast(buf, buf, bytes, ncclUint8, root, c->nc, st));
        return SRT_OK;
    }
    srt_loop* L = c->loop;
    const int me = c->rank, R = c->nranks;
    L->ptr[me] = buf;
    SRT_HIPCHK(hipEventRecord(L->ready[me], st));
    loop_wait(L);
    if (me != root) {
        SRT_HIPCHK(hipStreamWaitEvent(st, L->ready[root], 0));
        if (bytes) SRT_HIPCHK(hipMemcpyAsync(buf, L->ptr[root], bytes, hipMemcpyDeviceToDevice, st));
        SRT_HIPCHK(hipEventRecord(L->done[me], st));
    }
    loop_wait(L);
    if (me == root)
        for (int q = 0; q < R; q++)
            if (q != root) SRT_HIPCHK(hipStreamWaitEvent(st, L->done[q], 0));
    loop_wait(L);
    return SRT_OK;
}

static int allreduce_impl(const srt_comm* c, int32_t* buf, size_t count, int op_min,
                          hipStream_t st) {
    /* ring all-reduce: 2 (R - 1) / R of the buffer in */
    if (c->solo)
        return solo_wire(c, 2 * (size_t)(c->nranks - 1) * count * sizeof(int32_t) / c->nranks, st);
    if (!c->loop) {
        SRT_NCCLCHK(ncclAllReduce(buf, buf, count, ncclInt32, op_min ? ncclMin : ncclSum, c->nc, st));
        return SRT_OK;
    }
    srt_loop* L = c->loop;
    const int me = c->rank, R = c->nranks;
    L->ptr[me] = buf;
    SRT_HIPCHK(hipEventRecord(L->ready[me], st));
    loop_wait(L);
    if (me == 0) { /* rank 0 reduces every rank's buffer into its own */
        for (int q = 1; q < R; q++) {
            SRT_HIPCHK(hipStreamWaitEvent(st, L->ready[q], 0));
            if (count)
                allreduce_i32_kernel<<<(unsigned)((count + 255) / 256), 256, 0, st>>>(
                    buf, (const int32_t*)L->ptr[q], count, op_min);
        }
        SRT_HIPCHK(hipGetLastError());
        SRT_HIPCHK(hipEventRecord(L->done[0], st));
    }
    loop_wait(L);
    if (me != 0) {
        SRT_HIPCHK(hipStreamWaitEvent(st, L->done[0], 0));
        if (count)
            SRT_HIPCHK(hipMemcpyAsync(buf, L->ptr[0], count * sizeof(int32_t),
                                      hipMemcpyDeviceToDevice, st));
        SRT_HIPCHK(hipEventRecord(L->ready[me], st));
    }
    loop_wait(L);
    if (me == 0) /* rank 0's buffer stays untouched until every rank has its copy */
        for (int q = 1; q < R; q++) SRT_HIPCHK(hipStreamWaitEvent(st, L->ready[q], 0));
    loop_wait(L);
    return SRT_OK;
}

int srt_coll_group_begin(const srt_comm* c) {
    c_log(c, SRT_LOG_GROUP_BEGIN, 0, 0);
    if (!c->loop && !c->solo) SRT_NCCLCHK(ncclGroupStart());
    srt_comm* m = const_cast<srt_comm*>(c);
    m->in_group = 1;
    m->t_open = 0;
    if (c->solo) {
        m->group_bytes = 0;
        t_group_stream = nullptr;
    }
    return SRT_OK;
}

int srt_coll_group_end(const srt_comm* c) {
    c_log(c, SRT_LOG_GROUP_END, 0, 0);
    if (!c->loop && !c->solo) SRT_NCCLCHK(ncclGroupEnd());
    srt_comm* m = const_cast<srt_comm*>(c);
    const int was = m->in_group;
    m->in_group = 0;
    int rc = SRT_OK;
    if (c->solo && was && t_group_stream) rc = solo_wire(c, m->group_bytes, t_group_stream);
    if (was && m->t_open) { /* close the group's span on its first collective's stream, also
                             * after a failed wire span */
        m->t_open = 0;
        const int e = t_end(c, m->t_stream);
        if (!rc) rc = e;
    }
    return rc;
}

static int exchange_impl(const srt_comm* c, void* const* send, const size_t* send_bytes,
                         void* const* recv, const size_t* recv_bytes, hipStream_t st) {
    const int me = c->rank, R = c->nranks;
    if (c->solo) {
        size_t in = 0;
        for (int q = 0; q < R; q++)
            if (q != me) in += recv_bytes[q];
        return solo_wire(c, in, st);
    }
    if (!c->loop) {
        SRT_NCCLCHK(ncclGroupStart());
        for (int q = 0; q < R; q++)
            if (q != me && send_bytes[q])
                SRT_NCCLCHK(ncclSend(send[q], send_bytes[q], ncclUint8, q, c->nc, st));
        for (int q = 0; q < R; q++)
            if (q != me && recv_bytes[q])
                SRT_NCCLCHK(ncclRecv(recv[q], recv_bytes[q], ncclUint8, q, c->nc, st));
        SRT_NCCLCHK(ncclGroupEnd());
        return SRT_OK;
    }
    srt_loop* L = c->loop;
    for (int q = 0; q < R; q++) {
        L->sendp[me * R + q] = send[q];
        L->sendb[me * R + q] = q == me ? 0 : send_bytes[q];
    }
    SRT_HIPCHK(hipEventRecord(L->ready[me], st));
    loop_wait(L);
    for (int q = 0; q < R; q++) {
        if (q == me || !recv_bytes[q]) continue;
        if (L->sendb[q * R + me] != recv_bytes[q]) {
            srt_set_error("virtual exchange: rank %d sends %zu bytes to %d, which expects %zu", q,
                          L->sendb[q * R + me], me, recv_bytes[q]);
            loop_wait(L);
            loop_wait(L);
            return SRT_E_COMM;
        }
        SRT_HIPCHK(hipStreamWaitEvent(st, L->ready[q], 0));
        SRT_HIPCHK(hipMemcpyAsync(recv[q], L->sendp[q * R + me], recv_bytes[q],
                                  hipMemcpyDeviceToDevice, st));
    }
    SRT_HIPCHK(hipEventRecord(L->done[me], st));
    loop_wait(L);
    for (int q = 0; q < R; q++) /* the send buffers stay untouched until the peers have read */
        if (q != me && L->sendb[me * R + q]) SRT_HIPCHK(hipStreamWaitEvent(st, L->done[q], 0));
    loop_wait(L);
    return SRT_OK;
}

extern "C" void srt_shard_rows(int32_t n, int32_t align, int32_t nranks, int32_t rank,
                               int32_t* begin, int32_t* end) {
    if (align < 1) align = 1;
    if (nranks < 1) nranks = 1;
    const int64_t nb = (n + align - 1) / align;
    const int64_t b = nb * rank / nranks, e = nb * (rank + 1) / nranks;
    *begin = (int32_t)(b * align);
    *end = (int32_t)(e * align);
}

int srt_comm_rank(const srt_comm* c) { return c ? c->rank : -1; }
int srt_comm_is_solo(const srt_comm* c) { return c ? c->solo : 0; }
int srt_comm_size(const srt_comm* c) { return c ? c->nranks : 0; }

static int allgather_impl(const srt_comm* c, void* buf, size_t bytes, hipStream_t st) {
    if (c->solo) return solo_wire(c, (size_t)(c->nranks - 1) * bytes, st);
    if (bytes == 0) return SRT_OK;
    if (c->loop) { /* every rank broadcasts its block in turn */
        for (int q = 0; q < c->nranks; q++) {
            const int rc = bcast_impl(c, (uint8_t*)buf + bytes * q, bytes, q, st);
            if (rc) return rc;
        }
        return SRT_OK;
    }
    SRT_NCCLCHK(ncclAllGather((uint8_t*)buf + bytes * c->rank, buf, bytes, ncclUint8, c->nc, st));
    return SRT_OK;
}

static int sparse_allgather_impl(srt_comm* comm, int32_t n, int32_t rows_per_rank,
                                 uint32_t* lat_all, double* rel_all, void* stream) {
    if (!comm || n <= 0 || rows_per_rank <= 0 || !lat_all || !rel_all) {
        srt_set_error("srt_sparse_allgather: bad arguments");
        return SRT_E_ARG;
    }
    hipStream_t st = (hipStream_t)stream;
    const size_t cnt = (size_t)rows_per_rank * n;
    if (comm->solo) return solo_wire(comm, (size_t)(comm->nranks - 1) * cnt * 12, st);
    if (comm->loop) { /* every rank broadcasts its block in turn */
        for (int q = 0; q < comm->nranks; q++) {
            int rc = bcast_impl(comm, lat_all + cnt * q, cnt * sizeof(uint32_t), q, st);
            if (!rc) rc = bcast_impl(comm, rel_all + cnt * q, cnt * sizeof(double), q, st);
            if (rc) return rc;
        }
        return SRT_OK;
    }
    SRT_NCCLCHK(ncclGroupStart());
    SRT_NCCLCHK(ncclAllGather(lat_all + cnt * comm->rank, lat_all, cnt, ncclUint32, comm->nc, st));
    SRT_NCCLCHK(ncclAllGather(rel_all + cnt * comm->rank, rel_all, cnt, ncclFloat64, comm->nc, st));
    SRT_NCCLCHK(ncclGroupEnd());
    return SRT_OK;
}

/* ---- timed entry points: each collective (or its group) is one span of ms_comm ----------- */
/* the closing event is recorded whatever the call returns, so a failed collective cannot leave
 * the begin/end events of later spans paired across collectives */
#define SRT_TIMED(st, call)                       \
    do {                                          \
        int r_ = t_begin(c, st);                  \
        if (r_) return r_;                        \
        r_ = (call);                              \
        const int e_ = t_end(c, st);              \
        return r_ ? r_ : e_;                      \
    } while (0)

int srt_coll_bcast(const srt_comm* c, void* buf, size_t bytes, int root, hipStream_t st) {
    c_log(c, SRT_LOG_BCAST, (int64_t)bytes, root);
    SRT_TIMED(st, bcast_impl(c, buf, bytes, root, st));
}

int srt_coll_allreduce_i32(const srt_comm* c, int32_t* buf, size_t count, int op_min,
                           hipStream_t st) {
    c_log(c, SRT_LOG_ALLREDUCE, (int64_t)count, op_min);
    SRT_TIMED(st, allreduce_impl(c, buf, count, op_min, st));
}

int srt_coll_exchange(const srt_comm* c, void* const* send, const size_t* send_bytes,
                      void* const* recv, const size_t* recv_bytes, hipStream_t st) {
    c_log(c, SRT_LOG_EXCHANGE, 0, 0); /* (the byte counts differ per rank) */
    SRT_TIMED(st, exchange_impl(c, send, send_bytes, recv, recv_bytes, st));
}

int srt_coll_allgather(const srt_comm* c, void* buf, size_t bytes, hipStream_t st) {
    c_log(c, SRT_LOG_ALLGATHER, (int64_t)bytes, 0);
    SRT_TIMED(st, allgather_impl(c, buf, bytes, st));
}

extern "C" int srt_sparse_allgather(srt_comm* c, int32_t n, int32_t rows_per_rank,
                                    uint32_t* lat_all, double* rel_all, void* stream) {
    if (!c) {
        srt_set_error("srt_sparse_allgather: bad arguments");
        return SRT_E_ARG;
    }
    c_log(c, SRT_LOG_SPARSE_ALLGATHER, rows_per_rank, n);
    SRT_TIMED((hipStream_t)stream, sparse_allgather_impl(c, n, rows_per_rank, lat_all, rel_all, stream));
}
