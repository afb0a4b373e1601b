// Multi-GPU plumbing: RCCL over xGMI.
//
// Two ways to drive the GPUs of a node, both over the same sv_comm handles:
//   * one process per GPU (torchrun): rank 0 creates the 128-byte ncclUniqueId
//     and the Python driver hands it to the other ranks over its host control
//     plane (svx/control.py, plain TCP); sv_comm_init per rank;
//   * one process driving every GPU: sv_comm_init_all
//     (ncclCommInitAll), collectives of all devices inside one
//     sv_comm_group_start / sv_comm_group_end.
// The only device-data collective of the path is the broadcast of the plane
// (3 doubles) from the root, written straight into device memory on the
// batch's stream (sv_comm_broadcast_plane_dev), where the pipeline reads it
// (sv_batch_pipeline_dev): no host copy on the receivers and no host sync per
// step. An int64 all-reduce of the per-rank counts is provided for reporting.
// Frames are sharded by contiguous global-id ranges, so no point data moves.
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
    void* buf = nullptr;  // 4 KB device scratch of the synchronous host-plane / count calls (on c->stream)
};

extern "C" int sv_comm_set_error(const char* msg);                                  // runtime.hip
extern "C" int sv_batch_stream_internal(sv_batch* b, int* device, hipStream_t* stream,
                                        double** abc_slot);   // runtime.hip

namespace {
// The root's host plane into the comm's device buffer, on the batch stream.
__global__ void store_abc_kernel(double a, double b, double c, double* __restrict__ dst) {
    if (threadIdx.x == 0) {
        dst[0] = a;
        dst[1] = b;
        dst[2] = c;
    }
}
}  // namespace

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

int sv_comm_init_all(int n, const int* devices, sv_comm** out) {
    if (n < 1 || n > 64 || !devices || !out) return sv_comm_set_error("sv_comm_init_all: bad arguments"), SV_E_ARG;
    ncclComm_t comms[64];
    for (int i = 0; i < n; ++i) out[i] = nullptr;
    NCCL_TRY(ncclCommInitAll(comms, n, devices));
    for (int i = 0; i < n; ++i) {
        sv_comm* c = new sv_comm;
        c->comm = comms[i];
        c->device = devices[i];
        out[i] = c;
        hipError_t e = hipSetDevice(devices[i]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipMalloc(&c->buf, 4096);
        if (e != hipSuccess) {
            for (int j = 0; j <= i; ++j) {
                sv_comm_destroy(out[j]);
                out[j] = nullptr;
            }
            for (int j = i + 1; j < n; ++j) ncclCommDestroy(comms[j]);
            HIPC_TRY(e);
        }
    }
    return SV_OK;
}

int sv_comm_group_start(void) {
    NCCL_TRY(ncclGroupStart());
    return SV_OK;
}

int sv_comm_group_end(void) {
    NCCL_TRY(ncclGroupEnd());
    return SV_OK;
}

int sv_comm_broadcast_plane_dev(sv_comm* c, sv_batch* b, const sv_plane* plane, int root, const double** out_dplane) {
    if (!c || !b || !out_dplane) return sv_comm_set_error("sv_comm_broadcast_plane_dev: null"), SV_E_ARG;
    int dev = -1;
    hipStream_t s = nullptr;
    if (sv_batch_stream_internal(b, &dev, &s, nullptr) != SV_OK || dev != c->device)
        return sv_comm_set_error("sv_comm_broadcast_plane_dev: batch and comm are on different devices"), SV_E_ARG;
    int rank = -1;
    NCCL_TRY(ncclCommUserRank(c->comm, &rank));
    if (rank == root && !plane) return sv_comm_set_error("sv_comm_broadcast_plane_dev: the root needs the plane"), SV_E_ARG;
    HIPC_TRY(hipSetDevice(c->device));
    // the plane lands in the batch's own slot, written and read on the batch's stream only
    double* buf = nullptr;
    if (sv_batch_stream_internal(b, &dev, &s, &buf) != SV_OK)
        return sv_comm_set_error("sv_comm_broadcast_plane_dev: no device memory for the plane slot"), SV_E_HIP;
    if (rank == root) {
        hipLaunchKernelGGL(store_abc_kernel, dim3(1), dim3(64), 0, s, plane->a, plane->b, plane->c, buf);
        HIPC_TRY(hipGetLastError());
    }
    NCCL_TRY(ncclBroadcast(buf, buf, 3, ncclDouble, root, c->comm, s));
    *out_dplane = buf;
    return SV_OK;
}

int sv_multi_pipeline(int n, sv_comm* const* comms, sv_batch* const* batches, const sv_camera* cam,
                      const sv_plane* plane, int root, double point_thr, int hist_thr, int sync) {
    if (n < 1 || !comms || !batches || !cam || !plane || root < 0 || root >= n)
        return sv_comm_set_error("sv_multi_pipeline: bad arguments"), SV_E_ARG;
    const double* dplane[64];
    if (n > 64) return sv_comm_set_error("sv_multi_pipeline: at most 64 devices"), SV_E_ARG;
    NCCL_TRY(ncclGroupStart());
    for (int i = 0; i < n; ++i) {
        const int rc = sv_comm_broadcast_plane_dev(comms[i], batches[i], i == root ? plane : nullptr, root, &dplane[i]);
        if (rc != SV_OK) {
            (void)ncclGroupEnd();
            return rc;
        }
    }
    NCCL_TRY(ncclGroupEnd());
    for (int i = 0; i < n; ++i)
        if (int rc = sv_batch_pipeline_dev(batches[i], cam, dplane[i], point_thr, hist_thr, 0, 0)) return rc;
    if (sync)
        for (int i = 0; i < n; ++i)
            if (int rc = sv_batch_sync(batches[i])) return rc;
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
