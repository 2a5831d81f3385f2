// status.cpp — status strings and the last-HIP-error slot of the C ABI.
#include "bagua_kernels.h"
#include "launch_util.hpp"

namespace bagua {
thread_local int g_last_hip_error = 0;
thread_local KernelTiming g_kernel_timing;
}

extern "C" {

const char* bagua_status_string(int status) {
    switch (status) {
        case BAGUA_OK: return "ok";
        case BAGUA_ERR_INVALID_ARG: return "invalid argument (sizes, chunking or target chunk)";
        case BAGUA_ERR_WORKSPACE: return "workspace too small";
        case BAGUA_ERR_HIP: return "HIP kernel launch failed";
        case BAGUA_ERR_UNSUPPORTED: return "unsupported dtype or layout for this entry point";
    }
    return "unknown bagua status";
}

int bagua_last_hip_error(void) { return bagua::g_last_hip_error; }

int bagua_time_next_kernel(void* start_event, void* stop_event) {
    if ((start_event == nullptr) != (stop_event == nullptr)) return BAGUA_ERR_INVALID_ARG;
    bagua::g_kernel_timing.start = static_cast<hipEvent_t>(start_event);
    bagua::g_kernel_timing.stop = static_cast<hipEvent_t>(stop_event);
    return BAGUA_OK;
}

}  // extern "C"
