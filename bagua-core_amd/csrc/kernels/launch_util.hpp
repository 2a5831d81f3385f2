// launch_util.hpp — host-side launch helpers shared by the kernel TUs.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "bagua_kernels.h"

namespace bagua {

// 256 CUs x 8 resident 256-thread workgroups: enough waves in flight to
// cover HBM latency on a streaming kernel; larger problems grid-stride.
constexpr int kTargetBlocks = 2048;

// last hipError_t seen by a launcher on this thread (bagua_last_hip_error)
extern thread_local int g_last_hip_error;

// Bench instrumentation (bagua_time_next_kernel): when armed, the next kernel
// this library launches on this thread records `start`/`stop` at its own start
// and end (hipExtLaunchKernel), so its duration excludes dispatch overhead.
// bagua_time_next_kernels arms up to kMaxTimed launches the same way (one event
// pair each, in launch order) and remembers which kernel each one was.
struct KernelTiming {
    hipEvent_t start = nullptr, stop = nullptr;
};
constexpr int kMaxTimed = 32;
struct KernelTimingQueue {
    KernelTiming pairs[kMaxTimed];
    const void* fn[kMaxTimed] = {};
    int armed = 0, used = 0;
};
extern thread_local KernelTimingQueue g_kernel_timing;

inline KernelTiming take_timing(const void* fn) {
    KernelTimingQueue& q = g_kernel_timing;
    if (q.used >= q.armed) return KernelTiming{};
    q.fn[q.used] = fn;
    return q.pairs[q.used++];
}

// every kernel of the library is launched through here
template <typename F, typename... Args>
inline void launch(F kernel, const dim3& grid, const dim3& block, uint32_t shmem, hipStream_t s, Args... args) {
    const KernelTiming t = take_timing(reinterpret_cast<const void*>(kernel));
    // one launch path for timed and untimed launches: hipLaunchKernel instead of the
    // Ext call when nothing is timed costs the host the same (4.6-5.2 us per launch
    // either way, profiles/r03_host_overhead_ab.jsonl)
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, t.start, t.stop, 0u, args...);
}

// launch-shape knob read per call (measurement sweeps, tools/grid_sweep.py);
// `dflt` when unset
inline int tune_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return (e && *e) ? atoi(e) : dflt;
}

inline int check_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_last_hip_error = (int)e;
        return BAGUA_ERR_HIP;
    }
    return BAGUA_OK;
}

// v1 convention: CUDACHECK prints and exits (bagua-core-internal/cpp/include/bagua_utils.h:5)
inline void v1_check(int status, const char* file, int line) {
    if (status != BAGUA_OK) {
        printf("Failed: bagua kernel error %s:%d '%s'\n", file, line, bagua_status_string(status));
        exit(EXIT_FAILURE);
    }
}

}  // namespace bagua
