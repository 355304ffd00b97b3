// snk_comm.hip — data-parallel DQN across GPUs with RCCL over xGMI.
//
// New relative to the reference (single-process Julia): one
// process per GPU, envs sharded by rank (weak scaling, no env exchange), and
// ONE collective per DQN update: the in-place average of the P fp32 gradient
// (1.12 MB at bs = 12, latency-bound on xGMI) between the backward and
// RMSProp, so every replica applies the same update. Replicas start from
// rank 0's parameters (broadcast at attach).
#include <rccl/rccl.h>

#include <cstring>

#include "snk_internal.hpp"

using namespace snk;

struct snk_comm_s {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
};

#define SNK_NCCL(call)                                                                   \
    do {                                                                                 \
        ncclResult_t r_ = (call);                                                        \
        if (r_ != ncclSuccess) {                                                         \
            ::snk::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call,               \
                             ncclGetErrorString(r_));                                    \
            throw ::snk::Error{SNK_ERR_HIP};                                             \
        }                                                                                \
    } while (0)

static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");

extern "C" int snk_comm_unique_id(uint8_t *id128) {
    return guard([&] {
        SNK_CHECK(id128, SNK_ERR_INVALID, "NULL argument");
        ncclUniqueId id;
        SNK_NCCL(ncclGetUniqueId(&id));
        memcpy(id128, id.internal, 128);
    });
}

extern "C" int snk_comm_create(snk_comm *out, int32_t nranks, int32_t rank, const uint8_t *id128) {
    return guard([&] {
        SNK_CHECK(out && id128 && nranks >= 1 && rank >= 0 && rank < nranks, SNK_ERR_INVALID,
                  "bad comm arguments");
        ncclUniqueId id;
        memcpy(id.internal, id128, 128);
        auto *h = new snk_comm_s();
        h->nranks = nranks;
        h->rank = rank;
        ncclResult_t r = ncclCommInitRank(&h->comm, nranks, id, rank);
        if (r != ncclSuccess) {
            delete h;
            set_error("ncclCommInitRank: %s", ncclGetErrorString(r));
            throw Error{SNK_ERR_HIP};
        }
        *out = h;
    });
}

extern "C" int snk_comm_destroy(snk_comm h) {
    return guard([&] {
        if (!h) return;
        (void)hipStreamSynchronize(stream());
        if (h->comm) (void)ncclCommDestroy(h->comm);
        delete h;
    });
}

namespace snk {
void comm_allreduce_mean(snk_comm h, float *buf, int64_t n, hipStream_t s) {
    SNK_NCCL(ncclAllReduce(buf, buf, (size_t)n, ncclFloat32, ncclAvg, h->comm, s));
}
void comm_broadcast(snk_comm h, float *buf, int64_t n, int root, hipStream_t s) {
    SNK_NCCL(ncclBroadcast(buf, buf, (size_t)n, ncclFloat32, root, h->comm, s));
}
int comm_size(snk_comm h) { return h->nranks; }
int comm_rank(snk_comm h) { return h->rank; }
// point-to-point gather: every rank but root sends its n_send floats, root
// receives rank r's n_recv[r] into recv[r]. On xGMI each sender has its own
// link to root, so the transfers run side by side (one group).
void comm_gather_to_root(snk_comm h, const float *send, int64_t n_send, float *const *recv, const int64_t *n_recv,
                         int root, hipStream_t s) {
    SNK_NCCL(ncclGroupStart());
    if (h->rank == root) {
        for (int r = 0; r < h->nranks; ++r)
            if (r != root && n_recv[r] > 0) SNK_NCCL(ncclRecv(recv[r], (size_t)n_recv[r], ncclFloat32, r, h->comm, s));
    } else if (n_send > 0) {
        SNK_NCCL(ncclSend(send, (size_t)n_send, ncclFloat32, root, h->comm, s));
    }
    SNK_NCCL(ncclGroupEnd());
}
}  // namespace snk

extern "C" int snk_comm_allreduce_mean(snk_comm h, float *buf_dev, int64_t n) {
    return guard([&] {
        SNK_CHECK(h && buf_dev && n >= 0, SNK_ERR_INVALID, "bad allreduce arguments");
        comm_allreduce_mean(h, buf_dev, n, stream());
    });
}

extern "C" int snk_comm_info(snk_comm h, int32_t *nranks_out, int32_t *rank_out) {
    return guard([&] {
        SNK_CHECK(h && h->comm && nranks_out && rank_out, SNK_ERR_INVALID, "bad comm_info arguments");
        int n = 0, r = 0;
        SNK_NCCL(ncclCommCount(h->comm, &n));
        SNK_NCCL(ncclCommUserRank(h->comm, &r));
        *nranks_out = n;
        *rank_out = r;
    });
}

extern "C" int snk_comm_broadcast(snk_comm h, float *buf_dev, int64_t n, int32_t root) {
    return guard([&] {
        SNK_CHECK(h && buf_dev && n >= 0, SNK_ERR_INVALID, "bad broadcast arguments");
        comm_broadcast(h, buf_dev, n, root, stream());
    });
}
