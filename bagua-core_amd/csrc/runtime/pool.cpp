// pool.cpp — device memory pool (replaces CUDA_DEVICE_MEMORY_POOL,
// bagua-core-internal/src/resource_pool/mod.rs:11-60: a sized object pool of
// cudaMalloc'd blocks per device).
//
// Size classes are 4 per power of two (<= 25 % slack), so a 1 GiB gradient
// bucket and its ~256 MiB compressed buffer do not double in size the way a
// power-of-two pool would on a 288 GB HBM device.  Blocks are reused per
// class; bagua_pool_trim() returns cached blocks to HIP.  A block freed with
// bagua_pool_free_after() waits in a pending list until events recorded on
// the given streams have completed (the pool itself is not stream-ordered).
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "bagua_core.h"
#include "runtime_util.hpp"

namespace bagua {
namespace {

size_t size_class(size_t bytes) {
    if (bytes <= 256) return 256;
    size_t p = 1;
    while (p < bytes) p <<= 1;  // p/2 < bytes <= p
    const size_t q = p / 8;     // quarter steps between p/2 and p
    size_t c = p / 2;
    while (c < bytes) c += q;
    return c;
}

// a block freed behind queued work: reusable once every event has completed
struct PendingBlock {
    uint64_t ptr;
    size_t cls;
    std::vector<hipEvent_t> events;
};

struct DevicePool {
    std::map<size_t, std::vector<uint64_t>> free_blocks;  // class -> blocks
    std::vector<PendingBlock> pending;
    std::vector<hipEvent_t> spare_events;
    size_t in_use = 0, cached = 0, pending_bytes = 0;
};

struct Pool {
    std::mutex mu;
    std::unordered_map<int, DevicePool> dev;
    std::unordered_map<uint64_t, std::pair<int, size_t>> live;  // ptr -> (device, class)
};

Pool& pool() {
    static Pool* p = new Pool();  // never destroyed: blocks may outlive static teardown
    return *p;
}

// Moves pending blocks whose streams have drained to the free lists (P.mu held).
void reap_pending(DevicePool& d, bool wait) {
    size_t keep = 0;
    for (size_t i = 0; i < d.pending.size(); ++i) {
        PendingBlock& b = d.pending[i];
        bool done = true;
        for (hipEvent_t e : b.events) {
            const hipError_t q = wait ? hipEventSynchronize(e) : hipEventQuery(e);
            if (q == hipErrorNotReady) {
                done = false;
                break;
            }
            if (q != hipSuccess) (void)hipGetLastError();  // a faulted stream: the block is not read any more
        }
        if (!done) {
            if (keep != i) d.pending[keep] = std::move(b);
            ++keep;
            continue;
        }
        for (hipEvent_t e : b.events) d.spare_events.push_back(e);
        d.pending_bytes -= b.cls;
        d.cached += b.cls;
        d.free_blocks[b.cls].push_back(b.ptr);
    }
    d.pending.resize(keep);
}

// Capture arena: while the calling thread captures a HIP graph, every block its
// ops take from the pool belongs to the graph (the graph's kernels address it on
// every replay), so frees inside the capture are deferred to the arena's release
// and no pool call queries events (a query during capture invalidates it).
struct CaptureArena {
    std::vector<uint64_t> held;
};
thread_local CaptureArena* t_arena = nullptr;

bool arena_holds(uint64_t ptr) {
    if (!t_arena) return false;
    for (uint64_t p : t_arena->held)
        if (p == ptr) return true;
    return false;
}

}  // namespace

int pool_alloc(int device_id, size_t bytes, uint64_t* out) {
    if (!out) return BAGUA_ERR_INVALID_ARG;
    const int rc = pool_alloc_block(device_id, bytes, out);
    if (rc == BAGUA_OK && t_arena) t_arena->held.push_back(*out);
    return rc;
}

int pool_alloc_block(int device_id, size_t bytes, uint64_t* out) {
    const size_t cls = size_class(bytes ? bytes : 1);
    Pool& P = pool();
    {
        std::lock_guard<std::mutex> g(P.mu);
        DevicePool& d = P.dev[device_id];
        if (!d.pending.empty() && !t_arena) reap_pending(d, false);
        auto it = d.free_blocks.find(cls);
        if (it != d.free_blocks.end() && !it->second.empty()) {
            *out = it->second.back();
            it->second.pop_back();
            d.cached -= cls;
            d.in_use += cls;
            P.live[*out] = {device_id, cls};
            return BAGUA_OK;
        }
    }
    DeviceGuard guard(device_id);
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, cls);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        // free cached blocks of this device and retry once
        pool_trim(device_id);
        e = hipMalloc(&p, cls);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return BAGUA_ERR_OOM;
        }
    }
    std::lock_guard<std::mutex> g(P.mu);
    *out = (uint64_t)(uintptr_t)p;
    P.dev[device_id].in_use += cls;
    P.live[*out] = {device_id, cls};
    return BAGUA_OK;
}

int pool_free(uint64_t ptr) {
    if (!ptr) return BAGUA_OK;
    if (arena_holds(ptr)) return BAGUA_OK;  // the graph keeps it (capture_release frees it)
    return pool_free_block(ptr);
}

int pool_free_block(uint64_t ptr) {
    Pool& P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.live.find(ptr);
    if (it == P.live.end()) return BAGUA_ERR_INVALID_ARG;
    const int dev = it->second.first;
    const size_t cls = it->second.second;
    P.live.erase(it);
    DevicePool& d = P.dev[dev];
    d.in_use -= cls;
    d.cached += cls;
    d.free_blocks[cls].push_back(ptr);
    return BAGUA_OK;
}

int pool_free_after(uint64_t ptr, const uint64_t* streams, int n) {
    if (!ptr) return BAGUA_OK;
    if (arena_holds(ptr)) return BAGUA_OK;
    if (n <= 0) return pool_free(ptr);
    if (!streams) return BAGUA_ERR_INVALID_ARG;
    Pool& P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.live.find(ptr);
    if (it == P.live.end()) return BAGUA_ERR_INVALID_ARG;
    const int dev = it->second.first;
    const size_t cls = it->second.second;
    DevicePool& d = P.dev[dev];
    DeviceGuard guard(dev);
    PendingBlock b{ptr, cls, {}};
    for (int i = 0; i < n; ++i) {
        hipEvent_t e = nullptr;
        if (!d.spare_events.empty()) {
            e = d.spare_events.back();
            d.spare_events.pop_back();
        } else if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) {
            // completion only (the block is reused on this device): no system-scope fence
            (void)hipGetLastError();
            e = nullptr;
        }
        if (!e || hipEventRecord(e, (hipStream_t)(uintptr_t)streams[i]) != hipSuccess) {
            (void)hipGetLastError();
            // cannot order the reuse behind the stream: wait for it here instead
            if (e) d.spare_events.push_back(e);
            (void)hipStreamSynchronize((hipStream_t)(uintptr_t)streams[i]);
            continue;
        }
        b.events.push_back(e);
    }
    P.live.erase(it);
    d.in_use -= cls;
    d.pending_bytes += cls;
    d.pending.push_back(std::move(b));
    return BAGUA_OK;
}

int pool_trim(int device_id) {
    Pool& P = pool();
    std::vector<uint64_t> release;
    {
        std::lock_guard<std::mutex> g(P.mu);
        DevicePool& d = P.dev[device_id];
        if (!d.pending.empty()) {
            DeviceGuard guard(device_id);
            reap_pending(d, true);
        }
        for (auto& kv : d.free_blocks) {
            for (uint64_t p : kv.second) release.push_back(p);
            kv.second.clear();
        }
        d.cached = 0;
    }
    if (release.empty()) return BAGUA_OK;
    DeviceGuard guard(device_id);
    (void)hipDeviceSynchronize();  // a cached block may still be read by queued work
    for (uint64_t p : release) (void)hipFree((void*)(uintptr_t)p);
    return BAGUA_OK;
}

void* pool_capture_begin() {
    if (t_arena) return nullptr;  // no nesting
    t_arena = new CaptureArena();
    return t_arena;
}

int pool_capture_end(void* arena) {
    if (!arena || arena != t_arena) return BAGUA_ERR_INVALID_ARG;
    t_arena = nullptr;
    return BAGUA_OK;
}

int pool_capture_release(void* arena) {
    if (!arena || arena == t_arena) return BAGUA_ERR_INVALID_ARG;
    CaptureArena* a = static_cast<CaptureArena*>(arena);
    int rc = BAGUA_OK;
    for (uint64_t p : a->held) {
        const int r = pool_free_block(p);
        if (r && !rc) rc = r;
    }
    delete a;
    return rc;
}

size_t pool_bytes_pending(int device_id) {
    Pool& P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.dev.find(device_id);
    return it == P.dev.end() ? 0 : it->second.pending_bytes;
}

size_t pool_bytes(int device_id, bool cached) {
    Pool& P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.dev.find(device_id);
    if (it == P.dev.end()) return 0;
    return cached ? it->second.cached : it->second.in_use;
}

}  // namespace bagua

extern "C" {
int bagua_pool_alloc(int device_id, size_t bytes, uint64_t* ptr) { return bagua::pool_alloc(device_id, bytes, ptr); }
int bagua_pool_free(uint64_t ptr) { return bagua::pool_free(ptr); }
int bagua_pool_free_after(uint64_t ptr, const uint64_t* streams, int n) {
    return bagua::pool_free_after(ptr, streams, n);
}
int bagua_pool_trim(int device_id) { return bagua::pool_trim(device_id); }
size_t bagua_pool_bytes_pending(int device_id) { return bagua::pool_bytes_pending(device_id); }
void* bagua_pool_capture_begin(void) { return bagua::pool_capture_begin(); }
int bagua_pool_capture_end(void* arena) { return bagua::pool_capture_end(arena); }
int bagua_pool_capture_release(void* arena) { return bagua::pool_capture_release(arena); }
size_t bagua_pool_bytes_in_use(int device_id) { return bagua::pool_bytes(device_id, false); }
size_t bagua_pool_bytes_cached(int device_id) { return bagua::pool_bytes(device_id, true); }
}
