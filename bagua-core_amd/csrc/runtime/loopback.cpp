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
//
// Every collective also publishes what it is (kind, bytes, root, op, this rank's
// collective sequence number) beside its pointer; after the barrier every rank
// compares all of them, and grouped send/recv compares every (sender, receiver)
// pair's posted sizes.  Ranks that posted different collectives -- different piece
// schedules, one rank in the ring op and another in the centralized one -- all
// return BAGUA_ERR_COMM (after one more barrier, so nobody republishes while a peer
// still reads) instead of copying past a buffer's end.  abort() breaks the group:
// a rank waiting for a peer that never comes returns at once.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
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

enum CollKind { kAllToAll = 1, kAllGather, kBroadcast, kAllReduce, kReduce, kP2P };

// what a rank's current collective is; every rank's must be equal
struct CollDesc {
    int kind = 0, root = 0, op = 0;
    size_t bytes = 0;
    uint64_t seq = 0;
    bool operator==(const CollDesc& o) const {
        return kind == o.kind && root == o.root && op == o.op && bytes == o.bytes && seq == o.seq;
    }
};

const char* kind_name(int k) {
    static const char* n[] = {"?", "alltoall", "allgather", "broadcast", "allreduce", "reduce", "send/recv"};
    return k >= 0 && k <= kP2P ? n[k] : "?";
}

struct LoopbackGroup {
    explicit LoopbackGroup(int n, int dev)
        : p(n), device(dev), cfg(read_schedule_config()), ptr(n), desc(n), sends(n), recvs(n) {
        // test hook: BAGUA_LOOPBACK_ABORT_HOLD_S=<s> makes abort() leave a waiting rank
        // waiting for <s> seconds instead of releasing it, as a transport whose blocked
        // call never returns (the scheduler must then leave the call behind, not hang)
        const char* h = std::getenv("BAGUA_LOOPBACK_ABORT_HOLD_S");
        hold_s = h && *h ? std::atoi(h) : 0;
    }
    int p, device;
    int hold_s = 0;
    ScheduleConfig cfg;  // one process: every virtual rank reads the same environment, once
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;
    std::vector<const void*> ptr;            // per-rank published pointer
    std::vector<CollDesc> desc;              // per-rank published collective
    std::vector<std::vector<Post>> sends, recvs;

    void break_all() {
        if (hold_s > 0) return;  // the test hook: a waiting rank stays inside its call
        std::lock_guard<std::mutex> lk(mu);
        broken = true;
        cv.notify_all();
    }

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
        const auto limit = std::chrono::seconds(hold_s > 0 ? hold_s : 60);
        if (!cv.wait_for(lk, limit, [&] { return gen != my || broken; }) || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};

class LoopbackTransport final : public Transport {
    // a call in progress (the owner may not free the transport under it)
    struct Busy {
        explicit Busy(LoopbackTransport* t) : t_(t) { t_->inflight_.fetch_add(1); }
        ~Busy() { t_->inflight_.fetch_sub(1); }
        LoopbackTransport* t_;
    };
    std::atomic<int> inflight_{0};

   public:
    LoopbackTransport(LoopbackGroup* g, int rank) : g_(g), r_(rank) {}
    bool in_use() const override { return inflight_.load() > 0 || in_group_; }

    int alltoall(const void* s, void* rcv, size_t n, int d, hipStream_t st) override {
        Busy busy(this);
        const size_t b = n * bagua_dtype_bytes(d);
        if (int rc = enter(st, s, kAllToAll, b)) return rc;
        for (int j = 0; j < g_->p; ++j)
            if (copy((uint8_t*)rcv + j * b, (const uint8_t*)g_->ptr[j] + r_ * b, b, st)) return BAGUA_ERR_HIP;
        return leave(st);
    }
    int allgather(const void* s, void* rcv, size_t n, int d, hipStream_t st) override {
        Busy busy(this);
        const size_t b = n * bagua_dtype_bytes(d);
        if (int rc = enter(st, s, kAllGather, b)) return rc;
        for (int j = 0; j < g_->p; ++j) {
            uint8_t* dst = (uint8_t*)rcv + j * b;
            if (dst == g_->ptr[j]) continue;  // in place
            if (copy(dst, g_->ptr[j], b, st)) return BAGUA_ERR_HIP;
        }
        return leave(st);
    }
    int broadcast(void* buf, size_t n, int d, int root, hipStream_t st) override {
        Busy busy(this);
        const size_t b = n * bagua_dtype_bytes(d);
        if (int rc = enter(st, buf, kBroadcast, b, root)) return rc;
        if (r_ != root && copy(buf, g_->ptr[root], b, st)) return BAGUA_ERR_HIP;
        return leave(st);
    }
    int allreduce(const void* s, void* rcv, size_t n, int d, int op, hipStream_t st) override {
        Busy busy(this);
        // SUM / AVG over ranks in rank order (test transport; not bit-matched to RCCL)
        if (op != BAGUA_OP_SUM && op != BAGUA_OP_AVG) return BAGUA_ERR_UNSUPPORTED;
        const size_t b = n * bagua_dtype_bytes(d);
        PoolBuffer acc;
        if (acc.allocate(g_->device, b ? b : 1)) return BAGUA_ERR_OOM;
        if (int rc = enter(st, s, kAllReduce, b, 0, op)) return rc;
        if (copy(acc.as<void>(), g_->ptr[0], b, st)) return BAGUA_ERR_HIP;
        for (int j = 1; j < g_->p; ++j)
            if (bagua_add_inplace(d, acc.as<void>(), g_->ptr[j], (int)n, st)) return BAGUA_ERR_HIP;
        if (op == BAGUA_OP_AVG && bagua_divide_inplace(d, acc.as<void>(), (float)g_->p, (int)n, st)) return BAGUA_ERR_HIP;
        if (hipStreamSynchronize(st) != hipSuccess || !g_->barrier()) return BAGUA_ERR_COMM;  // all reads of s done
        if (copy(rcv, acc.as<void>(), b, st)) return BAGUA_ERR_HIP;
        return hipStreamSynchronize(st) == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP;
    }
    int reduce(const void* s, void* rcv, size_t n, int d, int op, int root, hipStream_t st) override {
        Busy busy(this);
        // SUM / AVG over ranks in rank order on the root; the others only contribute
        if (op != BAGUA_OP_SUM && op != BAGUA_OP_AVG) return BAGUA_ERR_UNSUPPORTED;
        const size_t b = n * bagua_dtype_bytes(d);
        PoolBuffer acc;
        if (r_ == root && acc.allocate(g_->device, b ? b : 1)) return BAGUA_ERR_OOM;
        if (int rc = enter(st, s, kReduce, b, root, op)) return rc;
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
        Busy busy(this);
        my_sends_.push_back({peer, const_cast<void*>(buf), n * bagua_dtype_bytes(d)});
        return in_group_ ? BAGUA_OK : flush(st);
    }
    int recv(void* buf, size_t n, int d, int peer, hipStream_t st) override {
        Busy busy(this);
        my_recvs_.push_back({peer, buf, n * bagua_dtype_bytes(d)});
        stream_ = st;
        return in_group_ ? BAGUA_OK : flush(st);
    }
    int group_start() override {
        in_group_ = true;
        return BAGUA_OK;
    }
    int group_end() override {
        Busy busy(this);
        in_group_ = false;
        return flush(stream_);
    }
    int abort() override {
        g_->break_all();
        return BAGUA_OK;
    }

    void set_stream(hipStream_t s) { stream_ = s; }

   private:
    // publish this rank's pointer and collective, wait for every rank, compare
    int enter(hipStream_t st, const void* publish, int kind, size_t bytes, int root = 0, int op = 0) {
        if (hipStreamSynchronize(st) != hipSuccess) return BAGUA_ERR_HIP;
        g_->ptr[r_] = publish;
        CollDesc me;
        me.kind = kind;
        me.bytes = bytes;
        me.root = root;
        me.op = op;
        me.seq = seq_++;
        g_->desc[r_] = me;
        if (!g_->barrier()) return BAGUA_ERR_COMM;
        for (int j = 0; j < g_->p; ++j)
            if (!(g_->desc[j] == g_->desc[0])) {
                if (r_ == 0)
                    BAGUA_LOG(0, "loopback: collective mismatch, rank 0 posted %s of %zu bytes (#%llu), rank %d "
                                 "%s of %zu bytes (#%llu)", kind_name(g_->desc[0].kind), g_->desc[0].bytes,
                              (unsigned long long)g_->desc[0].seq, j, kind_name(g_->desc[j].kind), g_->desc[j].bytes,
                              (unsigned long long)g_->desc[j].seq);
                return mismatch();
            }
        return BAGUA_OK;
    }
    // every rank saw the same mismatch: one more barrier (nobody republishes while a
    // peer is still comparing), then all fail alike
    int mismatch() {
        (void)g_->barrier();
        return BAGUA_ERR_COMM;
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
        my_sends_.clear();
        my_recvs_.clear();
        if (int rc = enter(st, nullptr, kP2P, 0)) return rc;
        // every pair's posted sizes must agree: the k-th receive rank r posts from q has
        // the size of the k-th send q posts to r, and nothing is left unmatched (every
        // rank checks every pair, so all reach the same verdict)
        const int p = g_->p;
        for (int r = 0; r < p; ++r)
            for (int q = 0; q < p; ++q) {
                std::vector<size_t> sent, got;
                for (const Post& sd : g_->sends[q])
                    if (sd.peer == r) sent.push_back(sd.bytes);
                for (const Post& rv : g_->recvs[r])
                    if (rv.peer == q) got.push_back(rv.bytes);
                if (sent != got) {
                    if (r_ == 0)
                        BAGUA_LOG(0, "loopback: send/recv mismatch, rank %d posts %zu sends to rank %d, which posts "
                                     "%zu receives from it (or their sizes differ)", q, sent.size(), r, got.size());
                    return mismatch();
                }
            }
        std::vector<int> taken(p, 0);  // k-th receive from q matches q's k-th send to me
        for (const Post& rv : g_->recvs[r_]) {
            int seen = 0;
            const Post* match = nullptr;
            for (const Post& sd : g_->sends[rv.peer]) {
                if (sd.peer != r_) continue;
                if (seen++ == taken[rv.peer]) { match = &sd; break; }
            }
            ++taken[rv.peer];
            if (copy(rv.ptr, match->ptr, rv.bytes, st)) return BAGUA_ERR_HIP;
        }
        return leave(st);
    }

    LoopbackGroup* g_;
    int r_;
    std::atomic<bool> in_group_{false};
    uint64_t seq_ = 0;  // collectives this rank posted
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
    c->cfg = g->cfg;
    return c;
}

}  // extern "C"
