// tensor_ops.cpp — codec dispatch on raw tensors.
//
// Mirrors RawBaguaTensor::{compress, decompress_from, reduce_mean_inplace,
// reduce_sum_inplace, add_inplace, addmul_inplace, clone_from}
// (bagua-core-internal/src/datatypes/mod.rs:129-522) including its
// argument checks: `num_elements_allocated % n_chunks == 0`
// (datatypes/mod.rs:322-326), chunk_size = allocated / n_chunks, output from
// the device pool.  The reference's per-call cub temp-size query and temp
// pool pull (:337-345) become a per-stream workspace reused in stream order.
#include <hip/hip_runtime.h>

#include <cstring>
#include <atomic>
#include <map>
#include <mutex>
#include <thread>

#include "bagua_core.h"
#include "runtime_util.hpp"

namespace bagua {

int log_level() {
    static int lvl = [] {
        const char* s = std::getenv("LOG_LEVEL");
        if (!s) return 1;
        if (!strcasecmp(s, "error")) return 0;
        if (!strcasecmp(s, "info")) return 2;
        if (!strcasecmp(s, "debug") || !strcasecmp(s, "trace")) return 3;
        return 1;
    }();
    return lvl;
}

// Workspace key: (device, stream handle, host thread when the handle is the
// hipStreamPerThread sentinel, which names a different stream on every thread
// and must not share one workspace between them).
struct WorkspaceKey {
    int device;
    uint64_t stream;
    std::thread::id tid;
    bool operator<(const WorkspaceKey& o) const {
        if (device != o.device) return device < o.device;
        if (stream != o.stream) return stream < o.stream;
        return tid < o.tid;
    }
};

static WorkspaceKey workspace_key(int device_id, uint64_t stream) {
    WorkspaceKey k{device_id, stream, std::thread::id()};
    if ((hipStream_t)(uintptr_t)stream == hipStreamPerThread) k.tid = std::this_thread::get_id();
    return k;
}

static std::mutex g_ws_mu;
static std::map<WorkspaceKey, std::pair<uint64_t, size_t>>& workspaces() {
    static auto* cache = new std::map<WorkspaceKey, std::pair<uint64_t, size_t>>();  // outlives static teardown
    return *cache;
}

int stream_workspace(int device_id, uint64_t stream, size_t bytes, uint64_t* out) {
    *out = 0;
    std::lock_guard<std::mutex> g(g_ws_mu);
    auto& slot = workspaces()[workspace_key(device_id, stream)];
    if (slot.second >= bytes && slot.first) {
        *out = slot.first;
        return BAGUA_OK;
    }
    if (slot.first) {
        // growing: queued work on this stream may still read the old block
        if (hipStreamSynchronize((hipStream_t)(uintptr_t)stream) != hipSuccess) return BAGUA_ERR_HIP;
        pool_free(slot.first);
        slot = {0, 0};
    }
    uint64_t p = 0;
    const size_t want = bytes < 65536 ? 65536 : bytes;
    // a stream's workspace outlives any op, so it never belongs to a capture arena
    const int rc = pool_alloc_block(device_id, want, &p);
    if (rc != BAGUA_OK) return rc;
    slot = {p, want};
    *out = p;
    return BAGUA_OK;
}

int release_stream_workspace(int device_id, uint64_t stream) {
    std::lock_guard<std::mutex> g(g_ws_mu);
    auto it = workspaces().find(workspace_key(device_id, stream));
    if (it == workspaces().end()) return BAGUA_OK;
    // queued work on the stream may still read the block
    if (hipStreamSynchronize((hipStream_t)(uintptr_t)stream) != hipSuccess) return BAGUA_ERR_HIP;
    if (it->second.first) pool_free(it->second.first);
    workspaces().erase(it);
    return BAGUA_OK;
}

size_t stream_workspace_count() {
    std::lock_guard<std::mutex> g(g_ws_mu);
    return workspaces().size();
}

static bool codec_dtype(int d) { return is_float_dtype(d); }

static int check_chunks(const bagua_tensor_t* t, int n_chunks, size_t* chunk_size) {
    if (!t || n_chunks <= 0) return BAGUA_ERR_INVALID_ARG;
    // datatypes/mod.rs:322-326 "compression tensor size % n_chunks must be 0"
    if (t->num_elem_allocated % (uint64_t)n_chunks != 0) return BAGUA_ERR_INVALID_ARG;
    const uint64_t cs = t->num_elem_allocated / (uint64_t)n_chunks;
    if (cs > 0x7fffffffULL || t->num_elem > 0x7fffffffULL) return BAGUA_ERR_INVALID_ARG;  // i32 kernel ABI
    *chunk_size = (size_t)cs;
    return BAGUA_OK;
}

static int compress_into(const bagua_tensor_t* t, int method, int n_chunks, uint64_t stream, int target,
                         uint64_t out_ptr, size_t out_bytes) {
    size_t cs = 0;
    int rc = check_chunks(t, n_chunks, &cs);
    if (rc) return rc;
    if (!codec_dtype(t->dtype)) return BAGUA_ERR_UNSUPPORTED;  // datatypes/mod.rs:376-384 unimplemented!()
    void* s = (void*)(uintptr_t)stream;
    if (method == BAGUA_COMPRESSION_MINMAX_UINT8) {
        const size_t ws_bytes = bagua_minmax_u8_workspace_bytes((int)cs, n_chunks);
        uint64_t ws = 0;
        if ((rc = stream_workspace(t->device_id, stream, ws_bytes, &ws)) != BAGUA_OK) return rc;
        return bagua_minmax_u8_compress(t->dtype, (const void*)(uintptr_t)t->ptr, (int)t->num_elem, (int)cs, n_chunks,
                                        (uint8_t*)(uintptr_t)out_ptr, out_bytes, (void*)(uintptr_t)ws, ws_bytes, target,
                                        s);
    }
    if (method == BAGUA_COMPRESSION_ONEBIT) {
        const size_t ws_bytes = bagua_onebit_workspace_bytes((int)cs, n_chunks);
        uint64_t ws = 0;
        if ((rc = stream_workspace(t->device_id, stream, ws_bytes, &ws)) != BAGUA_OK) return rc;
        return bagua_onebit_compress(t->dtype, (const void*)(uintptr_t)t->ptr, (int)t->num_elem, (int)cs, n_chunks,
                                     (uint8_t*)(uintptr_t)out_ptr, out_bytes, (void*)(uintptr_t)ws, ws_bytes, target, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

}  // namespace bagua

using namespace bagua;

extern "C" {

size_t bagua_dtype_bytes(int dtype) {
    switch (dtype) {
        case BAGUA_DTYPE_F32: return 4;
        case BAGUA_DTYPE_F16:
        case BAGUA_DTYPE_BF16: return 2;
        case BAGUA_DTYPE_U8: return 1;
        case BAGUA_DTYPE_I64:
        case BAGUA_DTYPE_U64: return 8;
    }
    return 0;
}

size_t bagua_compressed_size(int method, int dtype, size_t n_chunks, size_t chunk_size) {
    if (method == BAGUA_COMPRESSION_MINMAX_UINT8)
        return bagua_minmax_u8_compressed_bytes(dtype, (int)chunk_size, (int)n_chunks);
    if (method == BAGUA_COMPRESSION_ONEBIT) return bagua_onebit_compressed_bytes((int)chunk_size, (int)n_chunks);
    return 0;
}

int bagua_tensor_compress(const bagua_tensor_t* t, int method, int n_chunks, uint64_t stream, int target_chunk,
                          bagua_tensor_t* out) {
    size_t cs = 0;
    int rc = check_chunks(t, n_chunks, &cs);
    if (rc) return rc;
    if (!out) return BAGUA_ERR_INVALID_ARG;
    const size_t bytes = bagua_compressed_size(method, t->dtype, n_chunks, cs);
    if (!bytes) return BAGUA_ERR_UNSUPPORTED;
    uint64_t p = 0;
    rc = pool_alloc(t->device_id, bytes, &p);
    if (rc) return rc;
    rc = compress_into(t, method, n_chunks, stream, target_chunk, p, bytes);
    if (rc) {
        pool_free(p);
        return rc;
    }
    // datatypes/mod.rs:386-393: BaguaTensorRaw{U8, num_elem = num_elem_allocated = S}
    out->ptr = p;
    out->num_elem = bytes;
    out->num_elem_allocated = bytes;
    out->dtype = BAGUA_DTYPE_U8;
    out->device_id = t->device_id;
    return BAGUA_OK;
}

int bagua_tensor_compress_into(const bagua_tensor_t* t, int method, int n_chunks, uint64_t stream, int target_chunk,
                               const bagua_tensor_t* out) {
    size_t cs = 0;
    int rc = check_chunks(t, n_chunks, &cs);
    if (rc) return rc;
    if (!out || out->dtype != BAGUA_DTYPE_U8) return BAGUA_ERR_INVALID_ARG;
    const size_t bytes = bagua_compressed_size(method, t->dtype, n_chunks, cs);
    if (out->num_elem_allocated < bytes) return BAGUA_ERR_INVALID_ARG;
    return compress_into(t, method, n_chunks, stream, target_chunk, out->ptr, bytes);
}

int bagua_tensor_decompress_from(const bagua_tensor_t* t, int method, int n_chunks, const bagua_tensor_t* compressed,
                                 uint64_t stream) {
    size_t cs = 0;
    int rc = check_chunks(t, n_chunks, &cs);
    if (rc) return rc;
    if (!compressed || !codec_dtype(t->dtype)) return BAGUA_ERR_UNSUPPORTED;
    // datatypes/mod.rs:415-418: input bytes = compressed.num_elements_allocated * dtype bytes
    const size_t in_bytes = compressed->num_elem_allocated * bagua_dtype_bytes(compressed->dtype);
    void* s = (void*)(uintptr_t)stream;
    if (method == BAGUA_COMPRESSION_MINMAX_UINT8)
        return bagua_minmax_u8_decompress(t->dtype, (const uint8_t*)(uintptr_t)compressed->ptr, in_bytes, (int)cs,
                                          n_chunks, (void*)(uintptr_t)t->ptr, s);
    if (method == BAGUA_COMPRESSION_ONEBIT)
        return bagua_onebit_decompress(t->dtype, (const uint8_t*)(uintptr_t)compressed->ptr, in_bytes, (int)cs, n_chunks,
                                       (void*)(uintptr_t)t->ptr, s);
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_tensor_reduce_inplace(const bagua_tensor_t* t, int n_chunks, int target_chunk, int average,
                                uint64_t stream) {
    size_t cs = 0;
    int rc = check_chunks(t, n_chunks, &cs);
    if (rc) return rc;
    if (!codec_dtype(t->dtype)) return BAGUA_ERR_UNSUPPORTED;
    return bagua_reduce_chunks(t->dtype, (void*)(uintptr_t)t->ptr, (int)cs, n_chunks, target_chunk, average,
                               (void*)(uintptr_t)stream);
}

int bagua_tensor_add_inplace(const bagua_tensor_t* t, const bagua_tensor_t* o, uint64_t stream) {
    if (!t || !o || t->dtype != o->dtype || t->num_elem != o->num_elem) return BAGUA_ERR_INVALID_ARG;
    return bagua_add_inplace(t->dtype, (void*)(uintptr_t)t->ptr, (const void*)(uintptr_t)o->ptr, (int)t->num_elem,
                             (void*)(uintptr_t)stream);
}

int bagua_tensor_addmul_inplace(const bagua_tensor_t* t, const bagua_tensor_t* o, float factor, uint64_t stream) {
    if (!t || !o || t->dtype != o->dtype || t->num_elem != o->num_elem) return BAGUA_ERR_INVALID_ARG;
    return bagua_addmul_inplace(t->dtype, (void*)(uintptr_t)t->ptr, (const void*)(uintptr_t)o->ptr, (int)t->num_elem,
                                factor, (void*)(uintptr_t)stream);
}

int bagua_tensor_clone_from(const bagua_tensor_t* t, const bagua_tensor_t* o, uint64_t stream) {
    // datatypes/mod.rs:129-141
    if (!t || !o || t->dtype != o->dtype || t->num_elem != o->num_elem) return BAGUA_ERR_INVALID_ARG;
    const size_t bytes = t->num_elem * bagua_dtype_bytes(t->dtype);
    hipError_t e = hipMemcpyAsync((void*)(uintptr_t)t->ptr, (const void*)(uintptr_t)o->ptr, bytes,
                                  hipMemcpyDeviceToDevice, (hipStream_t)(uintptr_t)stream);
    return e == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP;
}

}  // extern "C"

extern "C" {
int bagua_release_stream_resources(int device_id, uint64_t stream) {
    DeviceGuard guard(device_id);
    const int rc = release_stream_workspace(device_id, stream);
    const int rk = bagua_minmax_u8_release_stream((void*)(uintptr_t)stream);
    return rc != BAGUA_OK ? rc : rk;
}

size_t bagua_stream_workspace_count(void) { return stream_workspace_count(); }

// datatypes/mod.rs:969-980: the comm stream waits for a tensor's ready event
int bagua_stream_wait_event(uint64_t stream, uint64_t event) {
    if (!event) return BAGUA_OK;
    return hipStreamWaitEvent((hipStream_t)(uintptr_t)stream, (hipEvent_t)(uintptr_t)event, 0) == hipSuccess
               ? BAGUA_OK
               : BAGUA_ERR_HIP;
}

// cuda_utils.rs:1-6 cuda_memcpy_device_to_host_sync (to_numpy_* read-back)
int bagua_memcpy_device_to_host_sync(void* host, uint64_t device_ptr, size_t bytes) {
    if (!bytes) return BAGUA_OK;
    return hipMemcpy(host, (const void*)(uintptr_t)device_ptr, bytes, hipMemcpyDeviceToHost) == hipSuccess
               ? BAGUA_OK
               : BAGUA_ERR_HIP;
}
}  // extern "C"
