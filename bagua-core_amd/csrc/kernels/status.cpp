// status.cpp — status strings and the last-HIP-error slot of the C ABI.
#include "bagua_kernels.h"
#include "launch_util.hpp"

namespace bagua {
thread_local int g_last_hip_error = 0;
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

}  // extern "C"
