// status.cpp — status strings and the last-HIP-error slot of the C ABI.
#include "bagua_kernels.h"
#include "launch_util.hpp"

#include <cxxabi.h>

#include <cstdlib>
#include <cstring>
#include <string>

namespace bagua {
thread_local int g_last_hip_error = 0;
thread_local KernelTimingQueue g_kernel_timing;
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
    if (!start_event) return bagua_time_next_kernels(nullptr, nullptr, 0);
    return bagua_time_next_kernels(&start_event, &stop_event, 1);
}

int bagua_time_next_kernels(void* const* start_events, void* const* stop_events, int n) {
    if (n < 0 || n > bagua::kMaxTimed || (n > 0 && (!start_events || !stop_events))) return BAGUA_ERR_INVALID_ARG;
    for (int i = 0; i < n; ++i)
        if (!start_events[i] || !stop_events[i]) return BAGUA_ERR_INVALID_ARG;
    bagua::KernelTimingQueue& q = bagua::g_kernel_timing;
    q = bagua::KernelTimingQueue{};
    for (int i = 0; i < n; ++i)
        q.pairs[i] = bagua::KernelTiming{static_cast<hipEvent_t>(start_events[i]), static_cast<hipEvent_t>(stop_events[i])};
    q.armed = n;
    return BAGUA_OK;
}

int bagua_timed_kernels(void) { return bagua::g_kernel_timing.used; }

int bagua_timed_kernel_name(int i, char* buf, size_t len) {
    const bagua::KernelTimingQueue& q = bagua::g_kernel_timing;
    if (i < 0 || i >= q.used || !buf || !len) return BAGUA_ERR_INVALID_ARG;
    const char* mangled = hipKernelNameRefByPtr(q.fn[i], nullptr);
    std::string name = mangled ? mangled : "?";
    int st = 0;
    char* dem = abi::__cxa_demangle(name.c_str(), nullptr, nullptr, &st);
    if (st == 0 && dem) {
        // "void bagua::minmax_quantize_kernel<bagua::F32, true>(...)" -> "minmax_quantize_kernel"
        std::string d = dem;
        const size_t paren = d.find_first_of("<(");
        std::string base = d.substr(0, paren);
        const size_t sp = base.find_last_of(": ");
        name = sp == std::string::npos ? base : base.substr(sp + 1);
    }
    free(dem);
    strncpy(buf, name.c_str(), len - 1);
    buf[len - 1] = 0;
    return BAGUA_OK;
}

}  // extern "C"
