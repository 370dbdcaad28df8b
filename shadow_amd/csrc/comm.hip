/*
 * comm.hip -- multi-GPU plumbing: RCCL communicator (one process per GPU, xGMI inside the node)
 * and the row-block partition shared by every sharded build.
 *
 * The reference has no multi-device code at all: these collectives are new.
 * Dense builds broadcast one pivot-row panel per Floyd-Warshall round; sparse builds shard the
 * sources and assemble the tables with one ncclAllGather.
 */
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include "srt_device.h"

struct srt_comm {
    ncclComm_t nc;
    int nranks, rank, device;
};

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

extern "C" void srt_comm_free(srt_comm* comm) {
    if (!comm) return;
    (void)ncclCommDestroy(comm->nc);
    free(comm);
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
int srt_comm_size(const srt_comm* c) { return c ? c->nranks : 0; }
ncclComm_t srt_comm_nccl(const srt_comm* c) { return c->nc; }

extern "C" int srt_sparse_allgather(srt_comm* comm, int32_t n, int32_t rows_per_rank,
                                    uint32_t* lat_all, double* rel_all, void* stream) {
    if (!comm || n <= 0 || rows_per_rank <= 0 || !lat_all || !rel_all) {
        srt_set_error("srt_sparse_allgather: bad arguments");
        return SRT_E_ARG;
    }
    hipStream_t st = (hipStream_t)stream;
    const size_t cnt = (size_t)rows_per_rank * n;
    SRT_NCCLCHK(ncclGroupStart());
    SRT_NCCLCHK(ncclAllGather(lat_all + cnt * comm->rank, lat_all, cnt, ncclUint32, comm->nc, st));
    SRT_NCCLCHK(ncclAllGather(rel_all + cnt * comm->rank, rel_all, cnt, ncclFloat64, comm->nc, st));
    SRT_NCCLCHK(ncclGroupEnd());
    return SRT_OK;
}
