// Multi-GPU plumbing: RCCL over xGMI.
//
// One process per GPU (launched by torchrun); the 128-byte ncclUniqueId is
// created by rank 0 and handed to the other ranks by the Python driver over
// the host control plane (torch.distributed gloo). The only device-data
// collective of the path is the plane-coefficient broadcast (24 B); an int64
// all-reduce of the per-rank counts is provided for reporting. Frames are
// sharded by contiguous global-id ranges, so no point data ever moves.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/svx.h"

static_assert(sizeof(ncclUniqueId) == SV_UNIQUE_ID_BYTES, "unique id size");

struct sv_comm {
    ncclComm_t comm = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    void* buf = nullptr;  // 4 KB device scratch
};

extern "C" int sv_comm_set_error(const char* msg);  // runtime.hip

#define NCCL_TRY(expr)                                                              \
    do {                                                                            \
        ncclResult_t r_ = (expr);                                                   \
        if (r_ != ncclSuccess) {                                                    \
            char m_[256];                                                           \
            snprintf(m_, sizeof m_, "%s: %s", #expr, ncclGetErrorString(r_));       \
            sv_comm_set_error(m_);                                                  \
            return SV_E_COMM;                                                       \
        }                                                                           \
    } while (0)

#define HIPC_TRY(expr)                                                              \
    do {                                                                            \
        hipError_t e_ = (expr);                                                     \
        if (e_ != hipSuccess) {                                                     \
            char m_[256];                                                           \
            snprintf(m_, sizeof m_, "%s: %s", #expr, hipGetErrorString(e_));        \
            sv_comm_set_error(m_);                                                  \
            return SV_E_HIP;                                                        \
        }                                                                           \
    } while (0)

extern "C" {

int sv_comm_unique_id(uint8_t* out_id) {
    if (!out_id) return sv_comm_set_error("null id"), SV_E_ARG;
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(out_id, &id, sizeof id);
    return SV_OK;
}

int sv_comm_init(int nranks, int rank, const uint8_t* id, int device, sv_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return sv_comm_set_error("sv_comm_init: bad arguments"), SV_E_ARG;
    *out = nullptr;
    HIPC_TRY(hipSetDevice(device));
    sv_comm* c = new sv_comm;
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&c->buf, 4096);
    if (e != hipSuccess) {
        sv_comm_destroy(c);
        HIPC_TRY(e);
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        c->comm = nullptr;
        sv_comm_destroy(c);
        NCCL_TRY(r);
    }
    *out = c;
    return SV_OK;
}

int sv_comm_destroy(sv_comm* c) {
    if (!c) return SV_OK;
    (void)hipSetDevice(c->device);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->buf) (void)hipFree(c->buf);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return SV_OK;
}

int sv_comm_broadcast_plane(sv_comm* c, sv_plane* inout, int root) {
    if (!c || !inout) return sv_comm_set_error("null"), SV_E_ARG;
    HIPC_TRY(hipSetDevice(c->device));
    double h[3] = {inout->a, inout->b, inout->c};
    HIPC_TRY(hipMemcpyAsync(c->buf, h, sizeof h, hipMemcpyHostToDevice, c->stream));
    NCCL_TRY(ncclBroadcast(c->buf, c->buf, 3, ncclDouble, root, c->comm, c->stream));
    HIPC_TRY(hipMemcpyAsync(h, c->buf, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIPC_TRY(hipStreamSynchronize(c->stream));
    inout->a = h[0];
    inout->b = h[1];
    inout->c = h[2];
    return SV_OK;
}

int sv_comm_allreduce_i64(sv_comm* c, int64_t* inout, int n) {
    if (!c || !inout || n < 0 || n > 512) return sv_comm_set_error("bad args"), SV_E_ARG;
    if (n == 0) return SV_OK;
    HIPC_TRY(hipSetDevice(c->device));
    HIPC_TRY(hipMemcpyAsync(c->buf, inout, 8 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    NCCL_TRY(ncclAllReduce(c->buf, c->buf, n, ncclInt64, ncclSum, c->comm, c->stream));
    HIPC_TRY(hipMemcpyAsync(inout, c->buf, 8 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIPC_TRY(hipStreamSynchronize(c->stream));
    return SV_OK;
}

}  // extern "C"
