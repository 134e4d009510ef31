// comm.hip -- the frame-end gather of the multi-GPU split over RCCL.
//
// The reference has no multi-GPU path: CUDARayTracer::Process (RayTracing/RayTracing.cpp:205-234)
// renders the whole frame into one surface.  Split over N GPUs, each rank renders its tiles
// into a compact shard ([entry][256] float4, rt_render_params.out_shard) and ONE gather per frame
// brings the shards to the root over xGMI, where rt_unshard / rt_unshard_tiles scatter them into
// the pitched surface.  That gather is the path's only exchange, so it is the only collective.
//
// Communicators come from an id made by one rank (rt_comm_unique_id) and passed to every rank
// by the host's own channel (one process per GPU), or from rt_comm_init_all (one process driving
// N devices, as a single-threaded C++ host does).  The gather is a group of point-to-point
// transfers: every non-root rank sends its shard (its own byte count, so cost-aware plans with
// uneven shards move no padding) and the root receives shard r at gathered + r * stride; the
// root's own shard is a device-to-device copy on the same stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <new>
#include <string>

#include "rt_abi.h"

void rt_internal_set_error(const char* msg);

struct rt_comm {
    ncclComm_t nccl;
    int rank, nranks, device;
};

static int nccl_fail(const char* what, ncclResult_t r) {
    const std::string m = std::string(what) + ": " + ncclGetErrorString(r);
    rt_internal_set_error(m.c_str());
    return 1;
}

static int hip_fail(const char* what, hipError_t e) {
    const std::string m = std::string(what) + ": " + hipGetErrorString(e);
    rt_internal_set_error(m.c_str());
    return 1;
}

static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "rt_comm id size");

extern "C" int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]) {
    if (!id) return nccl_fail("rt_comm_unique_id", ncclInvalidArgument);
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return nccl_fail("ncclGetUniqueId", r);
    std::memcpy(id, u.internal, RT_COMM_ID_BYTES);
    return 0;
}

extern "C" int rt_comm_init_rank(rt_comm** comm, int nranks, int rank, const uint8_t id[RT_COMM_ID_BYTES]) {
    if (!comm || !id || nranks <= 0 || rank < 0 || rank >= nranks) return nccl_fail("rt_comm_init_rank", ncclInvalidArgument);
    *comm = nullptr;
    int dev = 0;
    const hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail("rt_comm_init_rank: hipGetDevice", e);
    ncclUniqueId u;
    std::memcpy(u.internal, id, RT_COMM_ID_BYTES);
    rt_comm* c = new (std::nothrow) rt_comm{nullptr, rank, nranks, dev};
    if (!c) return nccl_fail("rt_comm_init_rank", ncclSystemError);
    const ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return nccl_fail("ncclCommInitRank", r);
    }
    *comm = c;
    return 0;
}

extern "C" int rt_comm_init_all(rt_comm** comms, int ndev, const int* devices) {
    if (!comms || !devices || ndev <= 0) return nccl_fail("rt_comm_init_all", ncclInvalidArgument);
    ncclComm_t* raw = new (std::nothrow) ncclComm_t[ndev];
    if (!raw) return nccl_fail("rt_comm_init_all", ncclSystemError);
    const ncclResult_t r = ncclCommInitAll(raw, ndev, devices);
    if (r != ncclSuccess) {
        delete[] raw;
        return nccl_fail("ncclCommInitAll", r);
    }
    for (int i = 0; i < ndev; i++) comms[i] = new rt_comm{raw[i], i, ndev, devices[i]};
    delete[] raw;
    return 0;
}

extern "C" int rt_comm_destroy(rt_comm* comm) {
    if (!comm) return 0;
    const ncclResult_t r = ncclCommDestroy(comm->nccl);
    delete comm;
    return r == ncclSuccess ? 0 : nccl_fail("ncclCommDestroy", r);
}

extern "C" int rt_comm_rank(const rt_comm* comm) { return comm ? comm->rank : -1; }
extern "C" int rt_comm_size(const rt_comm* comm) { return comm ? comm->nranks : -1; }

extern "C" int rt_comm_group_start(void) {
    const ncclResult_t r = ncclGroupStart();
    return r == ncclSuccess ? 0 : nccl_fail("ncclGroupStart", r);
}

extern "C" int rt_comm_group_end(void) {
    const ncclResult_t r = ncclGroupEnd();
    return r == ncclSuccess ? 0 : nccl_fail("ncclGroupEnd", r);
}

extern "C" int rt_gather_shards(rt_comm* comm, const void* shard, size_t shard_bytes, void* gathered, size_t stride,
                                const size_t* recv_bytes, int root, void* stream) {
    if (!comm || root < 0 || root >= comm->nranks || (shard_bytes && !shard))
        return nccl_fail("rt_gather_shards", ncclInvalidArgument);
    hipStream_t st = (hipStream_t)stream;
    const bool is_root = comm->rank == root;
    if (is_root) {
        if (!gathered) return nccl_fail("rt_gather_shards: root needs the gathered buffer", ncclInvalidArgument);
        for (int r = 0; r < comm->nranks; r++) {
            const size_t n = recv_bytes ? recv_bytes[r] : shard_bytes;
            if (n > stride) return nccl_fail("rt_gather_shards: a shard exceeds the stride", ncclInvalidArgument);
        }
        // the root copies its own recv_bytes[root] bytes out of `shard`: never more than it holds
        if (recv_bytes && recv_bytes[root] > shard_bytes)
            return nccl_fail("rt_gather_shards: recv_bytes[root] exceeds the root's shard_bytes", ncclInvalidArgument);
    }
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return nccl_fail("ncclGroupStart", r);
    if (is_root) {
        for (int q = 0; q < comm->nranks && r == ncclSuccess; q++) {
            const size_t n = recv_bytes ? recv_bytes[q] : shard_bytes;
            char* dst = (char*)gathered + (size_t)q * stride;
            if (q == root) {
                if (n) {
                    const hipError_t e = hipMemcpyAsync(dst, shard, n, hipMemcpyDeviceToDevice, st);
                    if (e != hipSuccess) {
                        ncclGroupEnd();
                        return hip_fail("rt_gather_shards: local copy", e);
                    }
                }
            } else if (n) {
                r = ncclRecv(dst, n, ncclUint8, q, comm->nccl, st);
            }
        }
    } else if (shard_bytes) {
        r = ncclSend(shard, shard_bytes, ncclUint8, root, comm->nccl, st);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail("rt_gather_shards: send/recv", r);
    if (r2 != ncclSuccess) return nccl_fail("ncclGroupEnd", r2);
    return 0;
}
