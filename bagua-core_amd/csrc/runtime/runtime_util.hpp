// runtime_util.hpp — internal helpers of the host runtime.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>

#include "bagua_core.h"

namespace bagua {

int pool_alloc(int device_id, size_t bytes, uint64_t* out);
int pool_free(uint64_t ptr);
int pool_free_after(uint64_t ptr, const uint64_t* streams, int n);
int pool_trim(int device_id);
int pool_alloc_block(int device_id, size_t bytes, uint64_t* out);  // no capture-arena bookkeeping
int pool_free_block(uint64_t ptr);
void* pool_capture_begin();
int pool_capture_end(void* arena);
int pool_capture_release(void* arena);
size_t pool_bytes(int device_id, bool cached);
size_t pool_bytes_pending(int device_id);

// Per-(device, stream) scratch reused by every launch on that stream; stream
// order makes reuse safe without host synchronisation.  *out = the block;
// BAGUA_ERR_HIP when growing it could not wait for the stream (a fault or
// sticky error on it), BAGUA_ERR_OOM when the pool has no block.
int stream_workspace(int device_id, uint64_t stream, size_t bytes, uint64_t* out);
// Frees the stream's workspace after the stream has drained (communicator teardown).
int release_stream_workspace(int device_id, uint64_t stream);
size_t stream_workspace_count();

// RAII current-device switch (communicators/mod.rs:32-35 does cudaSetDevice)
class DeviceGuard {
   public:
    explicit DeviceGuard(int device) {
        (void)hipGetDevice(&prev_);
        if (device >= 0 && device != prev_) {
            (void)hipSetDevice(device);
            switched_ = true;
        }
    }
    ~DeviceGuard() {
        if (switched_) (void)hipSetDevice(prev_);
    }

   private:
    int prev_ = 0;
    bool switched_ = false;
};

// RAII pool allocation
class PoolBuffer {
   public:
    PoolBuffer() = default;
    PoolBuffer(const PoolBuffer&) = delete;
    PoolBuffer& operator=(const PoolBuffer&) = delete;
    ~PoolBuffer() { reset(); }
    int allocate(int device, size_t bytes) {
        reset();
        bytes_ = bytes;
        return pool_alloc(device, bytes, &ptr_);
    }
    void reset() {
        if (ptr_) pool_free(ptr_);
        ptr_ = 0;
    }
    uint64_t ptr() const { return ptr_; }
    size_t bytes() const { return bytes_; }
    // the caller takes over the block (e.g. to free it behind a stream)
    void release_to_caller() { ptr_ = 0; }
    template <typename P>
    P* as() const { return reinterpret_cast<P*>((uintptr_t)ptr_); }

   private:
    uint64_t ptr_ = 0;
    size_t bytes_ = 0;
};

// level-filtered stderr logging (the reference's LOG_LEVEL env, py/lib.rs:489-496)
int log_level();  // 0=error 1=warn 2=info 3=debug
#define BAGUA_LOG(level, ...)                                   \
    do {                                                        \
        if (::bagua::log_level() >= (level)) {                  \
            std::fprintf(stderr, "[bagua-core] " __VA_ARGS__);  \
            std::fputc('\n', stderr);                           \
        }                                                       \
    } while (0)

inline bool is_float_dtype(int d) {
    return d == BAGUA_DTYPE_F32 || d == BAGUA_DTYPE_F16 || d == BAGUA_DTYPE_BF16;
}

}  // namespace bagua
