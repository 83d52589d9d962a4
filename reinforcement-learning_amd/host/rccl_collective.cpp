// rccl_collective.cpp -- the Learner's rlgpu_collective over a native RCCL communicator (include/
// rlgpu_learner.h rlgpu_rccl_*): one rank per GPU, RCCL over xGMI, no Python in the loop.
//
// The reference trains in one process (PPOLearner.cpp:360-371 batch-advantage moments, :521-526 the
// gradient before clip_grad_norm_, Learner.cpp:959-967 return samples); with arenas sharded over the
// GPUs of a node these become the three exchanges below.  The gradient all-reduce runs on the
// learner's stream (enqueued, no host wait: the optimizer step that follows on the same stream is
// ordered after it); the fp64 moments and the return samples are host values, staged through a small
// device buffer.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "../../include/rlgpu_learner.h"
#include "../csrc/common.hpp"

namespace {

struct RcclState {
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    int world = 1;
    void* stage = nullptr;  // device staging for the host-buffer collectives
    size_t stage_bytes = 0;
};

void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess)
        throw rlgpu::Error(RLGPU_ERR_STATE, std::string(what) + ": " + ncclGetErrorString(r));
}

void* stage(RcclState* st, size_t bytes) {
    if (bytes > st->stage_bytes) {
        if (st->stage) {
            RLGPU_CHECK_HIP(hipStreamSynchronize(st->stream));
            (void)hipFree(st->stage);
        }
        RLGPU_CHECK_HIP(hipMalloc(&st->stage, bytes));
        st->stage_bytes = bytes;
    }
    return st->stage;
}

// the callbacks never let an exception reach the C caller: a failure is a nonzero status
int allreduce_f32(void* user, float* d_buf, int64_t n) {
    return rlgpu::guarded([&] {
        auto* st = (RcclState*)user;
        nccl_check(ncclAllReduce(d_buf, d_buf, (size_t)n, ncclFloat32, ncclSum, st->comm, st->stream), "ncclAllReduce");
    });
}

int allreduce_f64(void* user, double* h_buf, int64_t n) {
    return rlgpu::guarded([&] {
        auto* st = (RcclState*)user;
        auto* d = (double*)stage(st, (size_t)n * sizeof(double));
        RLGPU_CHECK_HIP(hipMemcpyAsync(d, h_buf, (size_t)n * sizeof(double), hipMemcpyHostToDevice, st->stream));
        nccl_check(ncclAllReduce(d, d, (size_t)n, ncclFloat64, ncclSum, st->comm, st->stream), "ncclAllReduce");
        RLGPU_CHECK_HIP(hipMemcpyAsync(h_buf, d, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, st->stream));
        RLGPU_CHECK_HIP(hipStreamSynchronize(st->stream));
    });
}

int allgather_f32(void* user, const float* h_in, int64_t n, float* h_out) {
    return rlgpu::guarded([&] {
        auto* st = (RcclState*)user;
        const size_t in_bytes = (size_t)n * sizeof(float);
        auto* d = (float*)stage(st, in_bytes * (size_t)(st->world + 1));
        float* din = d + (size_t)n * st->world;
        RLGPU_CHECK_HIP(hipMemcpyAsync(din, h_in, in_bytes, hipMemcpyHostToDevice, st->stream));
        nccl_check(ncclAllGather(din, d, (size_t)n, ncclFloat32, st->comm, st->stream), "ncclAllGather");
        RLGPU_CHECK_HIP(hipMemcpyAsync(h_out, d, in_bytes * (size_t)st->world, hipMemcpyDeviceToHost, st->stream));
        RLGPU_CHECK_HIP(hipStreamSynchronize(st->stream));
    });
}

}  // namespace

extern "C" int rlgpu_rccl_unique_id(uint8_t* out, int32_t out_bytes) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(out && out_bytes >= RLGPU_RCCL_ID_BYTES, "rlgpu_rccl_unique_id: needs a 128-byte buffer");
        ncclUniqueId id;
        nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
        std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    });
}

extern "C" int rlgpu_rccl_collective_create(const uint8_t* id, int32_t rank, int32_t world, void* stream,
                                            rlgpu_collective* out) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(id && out, "rlgpu_rccl_collective_create: null argument");
        RLGPU_REQUIRE(world >= 1 && rank >= 0 && rank < world, "rlgpu_rccl_collective_create: bad rank / world");
        auto* st = new RcclState();
        st->stream = rlgpu::as_stream(stream);
        st->world = world;
        ncclUniqueId uid;
        std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
        const ncclResult_t r = ncclCommInitRank(&st->comm, world, uid, rank);
        if (r != ncclSuccess) {
            delete st;
            nccl_check(r, "ncclCommInitRank");
        }
        out->user = st;
        out->allreduce_sum_f32 = allreduce_f32;
        out->allreduce_sum_f64 = allreduce_f64;
        out->allgather_f32 = allgather_f32;
    });
}

extern "C" int rlgpu_rccl_collective_destroy(rlgpu_collective* c) {
    return rlgpu::guarded([&] {
        if (!c || !c->user) return;
        auto* st = (RcclState*)c->user;
        if (st->stream) (void)hipStreamSynchronize(st->stream);
        if (st->comm) (void)ncclCommDestroy(st->comm);
        if (st->stage) (void)hipFree(st->stage);
        delete st;
        std::memset(c, 0, sizeof(*c));
    });
}
