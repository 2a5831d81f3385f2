// comm_internal.hpp — communicator internals shared by communicator.cpp and comm_ops.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>

struct BaguaSingleCommunicatorC {
    ncclComm_t comm = nullptr;
    size_t rank = 0;
    size_t nranks = 1;
    int device_id = 0;
    hipStream_t stream = nullptr;
    std::atomic<bool> aborted{false};
};

namespace bagua {
ncclDataType_t nccl_dtype(int d);
int nccl_status(ncclResult_t r);
}  // namespace bagua
