// loopback.cpp — in-process transport: p virtual ranks, one host thread each,
// all on ONE device.  Collectives are device-to-device copies between the
// ranks' buffers, bracketed by host barriers:
//
//   rank r: sync own stream (its send data is final) -> publish pointers ->
//   barrier -> copy what it receives on its own stream -> sync -> barrier
//   (nobody reuses a buffer another rank may still be reading).
//
// Semantics follow NCCL's (alltoall block j <-> rank j; allgather rank j's
// block at j*count; grouped send/recv matched per (sender, receiver) pair in
// posting order).  It exists so the comm ops (comm_ops.cpp) — the same code
// that runs over RCCL on an 8-GPU node — are parity-tested at p > 1 on a
// one-GPU box.  Barriers time out (60 s) instead of hanging.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "bagua_core.h"
#include "comm_internal.hpp"
#include "runtime_util.hpp"

namespace bagua {
namespace {

struct Post {
    int peer;
    void* ptr;
    size_t bytes;
};

struct LoopbackGroup {
    explicit LoopbackGroup(int n, int dev) : p(n), device(dev), ptr(n), sends(n), recvs(n) {}
    int p, device;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;
    std::vector<const void*> ptr;            // per-rank published pointer
    std::vector<std::vector<Post>> sends, recvs;

    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const uint64_t my = gen;
        if (++arrived == p) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(60), [&] { return gen != my || broken; }) || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};

class LoopbackTransport final : public Transport {
   public:
    LoopbackTransport(LoopbackGroup* g, int rank) : g_(g), r_(rank) {}

    int alltoall(const void* s, void* rcv, size_t n, int d, hipStream_t st) override {
        const size_t b = n * bagua_dtype_bytes(d);
        if (!enter(st, s)) return BAGUA_ERR_COMM;
        for (int j = 0; j < g_->p; ++j)
            if (copy((uint8_t*)rcv + j * b, (const uint8_t*)g_->ptr[j] + r_ * b, b, st)) return BAGUA_ERR_HIP;
        return leave(st);
    }
    int allgather(const void* s, void* rcv, size_t n, int d, hipStream_t st) override {
        const size_t b = n * bagua_dtype_bytes(d);
        if (!enter(st, s)) return BAGUA_ERR_COMM;
        for (int j = 0; j < g_->p; ++j) {
            uint8_t* dst = (uint8_t*)rcv + j * b;
            if (dst == g_->ptr[j]) continue;  // in place
            if (copy(dst, g_->ptr[j], b, st)) return BAGUA_ERR_HIP;
        }
        return leave(st);
    }
    int broadcast(void* buf, size_t n, int d, int root, hipStream_t st) override {
        const size_t b = n * bagua_dtype_bytes(d);
        if (!enter(st, buf)) return BAGUA_ERR_COMM;
        if (r_ != root && copy(buf, g_->ptr[root], b, st)) return BAGUA_ERR_HIP;
        return leave(st);
    }
    int allreduce(const void* s, void* rcv, size_t n, int d, int op, hipStream_t st) override {
        // SUM / AVG over ranks in rank order (test transport; not bit-matched to RCCL)
        if (op != BAGUA_OP_SUM && op != BAGUA_OP_AVG) return BAGUA_ERR_UNSUPPORTED;
        const size_t b = n * bagua_dtype_bytes(d);
        PoolBuffer acc;
        if (acc.allocate(g_->device, b ? b : 1)) return BAGUA_ERR_OOM;
        if (!enter(st, s)) return BAGUA_ERR_COMM;
        if (copy(acc.as<void>(), g_->ptr[0], b, st)) return BAGUA_ERR_HIP;
        for (int j = 1; j < g_->p; ++j)
            if (bagua_add_inplace(d, acc.as<void>(), g_->ptr[j], (int)n, st)) return BAGUA_ERR_HIP;
        if (op == BAGUA_OP_AVG && bagua_divide_inplace(d, acc.as<void>(), (float)g_->p, (int)n, st)) return BAGUA_ERR_HIP;
        if (hipStreamSynchronize(st) != hipSuccess || !g_->barrier()) return BAGUA_ERR_COMM;  // all reads of s done
        if (copy(rcv, acc.as<void>(), b, st)) return BAGUA_ERR_HIP;
        return hipStreamSynchronize(st) == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP;
    }
    int reduce(const void* s, void* rcv, size_t n, int d, int op, int root, hipStream_t st) override {
        // SUM / AVG over ranks in rank order on the root; the others only contribute
        if (op != BAGUA_OP_SUM && op != BAGUA_OP_AVG) return BAGUA_ERR_UNSUPPORTED;
        const size_t b = n * bagua_dtype_bytes(d);
        PoolBuffer acc;
        if (r_ == root && acc.allocate(g_->device, b ? b : 1)) return BAGUA_ERR_OOM;
        if (!enter(st, s)) return BAGUA_ERR_COMM;
        if (r_ == root) {
            if (copy(acc.as<void>(), g_->ptr[0], b, st)) return BAGUA_ERR_HIP;
            for (int j = 1; j < g_->p; ++j)
                if (bagua_add_inplace(d, acc.as<void>(), g_->ptr[j], (int)n, st)) return BAGUA_ERR_HIP;
            if (op == BAGUA_OP_AVG && bagua_divide_inplace(d, acc.as<void>(), (float)g_->p, (int)n, st))
                return BAGUA_ERR_HIP;
        }
        if (hipStreamSynchronize(st) != hipSuccess || !g_->barrier()) return BAGUA_ERR_COMM;  // all reads of s done
        if (r_ == root && copy(rcv, acc.as<void>(), b, st)) return BAGUA_ERR_HIP;
        return hipStreamSynchronize(st) == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP;
    }
    int send(const void* buf, size_t n, int d, int peer, hipStream_t st) override {
        my_sends_.push_back({peer, const_cast<void*>(buf), n * bagua_dtype_bytes(d)});
        return in_group_ ? BAGUA_OK : flush(st);
    }
    int recv(void* buf, size_t n, int d, int peer, hipStream_t st) override {
        my_recvs_.push_back({peer, buf, n * bagua_dtype_bytes(d)});
        stream_ = st;
        return in_group_ ? BAGUA_OK : flush(st);
    }
    int group_start() override {
        in_group_ = true;
        return BAGUA_OK;
    }
    int group_end() override {
        in_group_ = false;
        return flush(stream_);
    }
    int abort() override { return BAGUA_OK; }

    void set_stream(hipStream_t s) { stream_ = s; }

   private:
    bool enter(hipStream_t st, const void* publish) {
        if (hipStreamSynchronize(st) != hipSuccess) return false;
        g_->ptr[r_] = publish;
        return g_->barrier();
    }
    int leave(hipStream_t st) {
        if (hipStreamSynchronize(st) != hipSuccess) return BAGUA_ERR_HIP;
        return g_->barrier() ? BAGUA_OK : BAGUA_ERR_COMM;
    }
    int copy(void* dst, const void* src, size_t b, hipStream_t st) {
        if (!b) return BAGUA_OK;
        return hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToDevice, st) == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP;
    }
    // every rank calls flush() at its group end (NCCL grouped p2p: all ranks take part)
    int flush(hipStream_t st) {
        if (hipStreamSynchronize(st) != hipSuccess) return BAGUA_ERR_HIP;
        g_->sends[r_] = my_sends_;
        g_->recvs[r_] = my_recvs_;
        if (!g_->barrier()) return BAGUA_ERR_COMM;
        std::vector<int> taken(g_->p, 0);  // k-th receive from q matches q's k-th send to me
        for (const Post& rv : my_recvs_) {
            int seen = 0;
            const Post* match = nullptr;
            for (const Post& sd : g_->sends[rv.peer]) {
                if (sd.peer != r_) continue;
                if (seen++ == taken[rv.peer]) { match = &sd; break; }
            }
            if (!match || match->bytes != rv.bytes) return BAGUA_ERR_COMM;
            ++taken[rv.peer];
            if (copy(rv.ptr, match->ptr, rv.bytes, st)) return BAGUA_ERR_HIP;
        }
        my_sends_.clear();
        my_recvs_.clear();
        return leave(st);
    }

    LoopbackGroup* g_;
    int r_;
    bool in_group_ = false;
    hipStream_t stream_ = nullptr;
    std::vector<Post> my_sends_, my_recvs_;
};

}  // namespace
}  // namespace bagua

using namespace bagua;

extern "C" {

void* bagua_loopback_group_create(int nranks, int device_id) {
    if (nranks <= 0) return nullptr;
    return new LoopbackGroup(nranks, device_id);
}

void bagua_loopback_group_destroy(void* group) { delete static_cast<LoopbackGroup*>(group); }

BaguaSingleCommunicatorC* bagua_loopback_communicator_create(void* group, size_t rank, uint64_t stream_ptr) {
    auto* g = static_cast<LoopbackGroup*>(group);
    if (!g || rank >= (size_t)g->p) return nullptr;
    auto* tr = new LoopbackTransport(g, (int)rank);
    tr->set_stream((hipStream_t)(uintptr_t)stream_ptr);
    auto* c = new BaguaSingleCommunicatorC();
    c->t = tr;
    c->rank = rank;
    c->nranks = (size_t)g->p;
    c->device_id = g->device;
    c->stream = (hipStream_t)(uintptr_t)stream_ptr;
    return c;
}

}  // extern "C"
