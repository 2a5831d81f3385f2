// communicator.cpp — RCCL communicator (replaces the Aluminum NCCLBackend
// wrappers of bagua-core-internal/src/communicators/mod.rs and the C shim
// bagua-core-c/src/lib.rs:9-69, whose symbols were Rust-mangled: exported
// unmangled here).
//
// One communicator = one transport (an ncclComm_t for the product) + the
// stream every collective and codec kernel of the comm ops is enqueued on
// (the reference binds an Al::NCCLCommunicator to a stream the same way,
// communicators/mod.rs:44).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <string>
#include <vector>

#include "bagua_core.h"
#include "comm_internal.hpp"
#include "runtime_util.hpp"

namespace bagua {

static const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string base64_encode(const uint8_t* p, size_t n) {
    std::string o;
    for (size_t i = 0; i < n; i += 3) {
        uint32_t v = (uint32_t)p[i] << 16;
        if (i + 1 < n) v |= (uint32_t)p[i + 1] << 8;
        if (i + 2 < n) v |= p[i + 2];
        o += kB64[(v >> 18) & 63];
        o += kB64[(v >> 12) & 63];
        o += i + 1 < n ? kB64[(v >> 6) & 63] : '=';
        o += i + 2 < n ? kB64[v & 63] : '=';
    }
    return o;
}

bool base64_decode(const char* s, std::vector<uint8_t>* out) {
    out->clear();
    uint32_t v = 0;
    int bits = 0;
    for (; *s && *s != '='; ++s) {
        const char* f = std::strchr(kB64, *s);
        if (!f) return false;
        v = (v << 6) | (uint32_t)(f - kB64);
        bits += 6;
        if (bits >= 8) {
            bits -= 8;
            out->push_back((uint8_t)((v >> bits) & 0xff));
        }
    }
    return true;
}

ncclDataType_t nccl_dtype(int d) {
    switch (d) {
        case BAGUA_DTYPE_F32: return ncclFloat32;
        case BAGUA_DTYPE_F16: return ncclFloat16;
        case BAGUA_DTYPE_BF16: return ncclBfloat16;
        case BAGUA_DTYPE_U8: return ncclUint8;
        case BAGUA_DTYPE_I64: return ncclInt64;
        case BAGUA_DTYPE_U64: return ncclUint64;
    }
    return ncclUint8;
}

static ncclRedOp_t nccl_op(int op) {
    switch (op) {
        case BAGUA_OP_PROD: return ncclProd;
        case BAGUA_OP_MIN: return ncclMin;
        case BAGUA_OP_MAX: return ncclMax;
        case BAGUA_OP_AVG: return ncclAvg;
    }
    return ncclSum;
}

int nccl_status(ncclResult_t r) {
    if (r == ncclSuccess) return BAGUA_OK;
    BAGUA_LOG(0, "RCCL error: %s", ncclGetErrorString(r));
    return BAGUA_ERR_COMM;
}

// ------------------------------------------------------------ RCCL transport --
class RcclTransport final : public Transport {
   public:
    explicit RcclTransport(ncclComm_t c) : comm_(c) {}
    ~RcclTransport() override {
        if (!comm_) return;
        if (!aborted_.load())
            (void)ncclCommDestroy(comm_);
        else
            (void)release_if_idle();  // an abort deferred until now (the owner checked in_use())
    }
    int allreduce(const void* s, void* r, size_t n, int d, int op, hipStream_t st) override {
        Call g(this);
        return g.ok ? nccl_status(ncclAllReduce(s, r, n, nccl_dtype(d), nccl_op(op), comm_, st)) : BAGUA_ERR_ABORTED;
    }
    int broadcast(void* b, size_t n, int d, int root, hipStream_t st) override {
        Call g(this);
        return g.ok ? nccl_status(ncclBroadcast(b, b, n, nccl_dtype(d), root, comm_, st)) : BAGUA_ERR_ABORTED;
    }
    int reduce(const void* s, void* r, size_t n, int d, int op, int root, hipStream_t st) override {
        Call g(this);
        return g.ok ? nccl_status(ncclReduce(s, r, n, nccl_dtype(d), nccl_op(op), root, comm_, st))
                    : BAGUA_ERR_ABORTED;
    }
    int alltoall(const void* s, void* r, size_t n, int d, hipStream_t st) override {
        Call g(this);
        return g.ok ? nccl_status(ncclAllToAll(s, r, n, nccl_dtype(d), comm_, st)) : BAGUA_ERR_ABORTED;
    }
    int allgather(const void* s, void* r, size_t n, int d, hipStream_t st) override {
        Call g(this);
        return g.ok ? nccl_status(ncclAllGather(s, r, n, nccl_dtype(d), comm_, st)) : BAGUA_ERR_ABORTED;
    }
    int send(const void* b, size_t n, int d, int peer, hipStream_t st) override {
        Call g(this);
        return g.ok ? nccl_status(ncclSend(b, n, nccl_dtype(d), peer, comm_, st)) : BAGUA_ERR_ABORTED;
    }
    int recv(void* b, size_t n, int d, int peer, hipStream_t st) override {
        Call g(this);
        return g.ok ? nccl_status(ncclRecv(b, n, nccl_dtype(d), peer, comm_, st)) : BAGUA_ERR_ABORTED;
    }
    // Group brackets stay balanced after an abort (the calls between them fail).  An
    // open bracket counts as use: ncclGroupEnd runs the grouped sends/recvs against the
    // communicator, so it may not be freed between a grouped call and its group end.
    int group_start() override {
        depth_.fetch_add(1);
        return nccl_status(ncclGroupStart());
    }
    int group_end() override {
        int rc;
        {
            Call g(this);  // inside RCCL while the group's tasks are issued
            rc = nccl_status(ncclGroupEnd());
            depth_.fetch_sub(1);
        }
        return rc;
    }
    // From any thread (the scheduler's monitor aborts a stuck op's communicator while
    // the worker may be enqueueing).  Later calls fail with BAGUA_ERR_ABORTED at once.
    // ncclCommAbort, which frees the communicator, runs only when no call is inside RCCL
    // and no group bracket is open: right away, after up to 2 s for a call that is about
    // to return, or else deferred to the moment the last such call returns (a call
    // blocked on a peer returns when that peer's process ends or the peer posts) or to
    // the transport's destruction.  The communicator is never freed under a call.
    int abort() override {
        if (aborted_.exchange(true)) return BAGUA_OK;
        const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(2);
        while (in_use() && std::chrono::steady_clock::now() < until)
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        const int rc = release_if_idle();
        if (!released_.load())
            BAGUA_LOG(1, "communicator abort deferred: a call is still inside RCCL; the communicator is "
                         "released when it returns");
        return rc;
    }
    bool in_use() const override { return inflight_.load() > 0 || depth_.load() > 0; }

   private:
    // ncclCommAbort once, by whichever thread finds the transport aborted and idle
    int release_if_idle() {
        std::lock_guard<std::mutex> g(release_mu_);
        if (released_.load() || !comm_ || in_use()) return BAGUA_OK;
        released_.store(true);
        return nccl_status(ncclCommAbort(comm_));
    }
    // A call enters (inflight_ first, then the flag) while abort() sets the flag first,
    // then reads inflight_: with sequentially consistent atomics either the call sees
    // the abort and stays out of RCCL, or the abort sees the call and defers.
    struct Call {
        explicit Call(RcclTransport* t) : t_(t) {
            t_->inflight_.fetch_add(1);
            ok = !t_->aborted_.load() && t_->comm_;
        }
        ~Call() {
            t_->inflight_.fetch_sub(1);
            if (t_->aborted_.load()) (void)t_->release_if_idle();
        }
        RcclTransport* t_;
        bool ok = false;
    };
    ncclComm_t comm_;
    std::atomic<bool> aborted_{false};
    std::atomic<bool> released_{false};
    std::atomic<int> inflight_{0};
    std::atomic<int> depth_{0};
    std::mutex release_mu_;
};

Transport* make_rccl_transport(ncclComm_t comm) { return new RcclTransport(comm); }

static int32_t env_i32(const char* name, int32_t dflt) {
    const char* v = std::getenv(name);
    return v && *v ? (int32_t)std::strtol(v, nullptr, 10) : dflt;
}

ScheduleConfig read_schedule_config() {
    ScheduleConfig c;
    c.pieces_cap = env_i32("BAGUA_PIPELINE_PIECES", c.pieces_cap);
    c.min_piece = env_i32("BAGUA_PIPELINE_MIN_PIECE", c.min_piece);
    {  // tri-state: unset -1 (the op's automatic schedules taper), 0 never, 1 every plain count
        const int32_t t = env_i32("BAGUA_PIPELINE_TAPER", -1);
        c.taper = t < 0 ? -1 : (t == 1 ? 1 : 0);
    }
    c.multipath = env_i32("BAGUA_RING_MULTIPATH", 0) != 0;
    c.check = env_i32("BAGUA_CHECK_SCHEDULE", 0) != 0;
    return c;
}

// Every rank adopts rank 0's schedule switches: an allgather of each rank's
// ScheduleConfig on `stream` (the communicator's first collective, posted by every
// rank inside creation), a warning naming the ranks whose environment differed.
static int agree_schedule_config(Transport* t, size_t rank, size_t nranks, int device, hipStream_t stream,
                                 ScheduleConfig* cfg) {
    if (nranks <= 1) return BAGUA_OK;
    const size_t one = sizeof(ScheduleConfig);
    PoolBuffer buf;
    int rc = buf.allocate(device, one * nranks);
    if (rc) return rc;
    std::vector<ScheduleConfig> all(nranks);
    uint8_t* base = buf.as<uint8_t>();
    if (hipMemcpyAsync(base + rank * one, cfg, one, hipMemcpyHostToDevice, stream) != hipSuccess) return BAGUA_ERR_HIP;
    if ((rc = t->allgather(base + rank * one, base, one, BAGUA_DTYPE_U8, stream)) != BAGUA_OK) return rc;
    if (hipMemcpyAsync(all.data(), base, one * nranks, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        return BAGUA_ERR_HIP;
    for (size_t r = 1; r < nranks; ++r)
        if (!(all[r] == all[0]) && rank == 0)
            BAGUA_LOG(1, "rank %zu's schedule environment (BAGUA_PIPELINE_*, BAGUA_RING_MULTIPATH, "
                         "BAGUA_CHECK_SCHEDULE) differs from rank 0's; every rank uses rank 0's", r);
    *cfg = all[0];
    return BAGUA_OK;
}

}  // namespace bagua

using namespace bagua;

BaguaSingleCommunicatorC* BaguaSingleCommunicatorC::lane(int i) {
    if (i <= 0) return this;
    std::lock_guard<std::mutex> g(lanes_mu);
    while ((int)lanes.size() < i) {
        DeviceGuard guard(device_id);
        hipStream_t s = nullptr;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
        auto* v = new BaguaSingleCommunicatorC();
        v->t = t;
        v->rank = rank;
        v->nranks = nranks;
        v->device_id = device_id;
        v->stream = s;
        v->own_stream = true;
        v->parent = this;
        v->async = async;
        v->cfg = cfg;
        v->aborted.store(aborted.load());
        // lanes run codec work beside each other: no one-launch encode (it needs every CU)
        (void)bagua_minmax_u8_set_stream_resident(s, 0);
        lanes.push_back(v);
    }
    return lanes[(size_t)i - 1];
}

#define COMM_CHECK(c)                                        \
    do {                                                     \
        if (!(c) || !(c)->t) return BAGUA_ERR_INVALID_ARG;   \
        if ((c)->aborted.load()) return BAGUA_ERR_ABORTED;   \
    } while (0)

extern "C" {

int bagua_generate_nccl_unique_id_str(char* buf, size_t buf_len) {
    // communicators/mod.rs:226-240: base64 of the 128-byte ncclUniqueId
    ncclUniqueId id;
    int rc = nccl_status(ncclGetUniqueId(&id));
    if (rc) return rc;
    const std::string s = base64_encode(reinterpret_cast<const uint8_t*>(id.internal), NCCL_UNIQUE_ID_BYTES);
    if (!buf || buf_len < s.size() + 1) return BAGUA_ERR_INVALID_ARG;
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return BAGUA_OK;
}

BaguaSingleCommunicatorC* bagua_single_communicator_c_create(size_t rank, size_t nranks, size_t device_id,
                                                             uint64_t stream_ptr, const char* nccl_unique_id_str) {
    // communicators/mod.rs:25-60
    if (!nccl_unique_id_str || rank >= nranks) return nullptr;
    if (hipSetDevice((int)device_id) != hipSuccess) return nullptr;
    std::vector<uint8_t> bytes;
    if (!base64_decode(nccl_unique_id_str, &bytes) || bytes.size() < NCCL_UNIQUE_ID_BYTES) return nullptr;
    ncclUniqueId id;
    std::memcpy(id.internal, bytes.data(), NCCL_UNIQUE_ID_BYTES);
    ncclComm_t comm = nullptr;
    if (ncclCommInitRank(&comm, (int)nranks, id, (int)rank) != ncclSuccess) return nullptr;
    auto* c = new BaguaSingleCommunicatorC();
    c->t = make_rccl_transport(comm);
    c->rank = rank;
    c->nranks = nranks;
    c->device_id = (int)device_id;
    c->stream = (hipStream_t)(uintptr_t)stream_ptr;
    c->cfg = read_schedule_config();
    if (agree_schedule_config(c->t, rank, nranks, c->device_id, c->stream, &c->cfg) != BAGUA_OK) {
        BAGUA_LOG(0, "communicator rank %zu/%zu: could not agree on the schedule switches", rank, nranks);
        c->t->abort();
        delete c->t;
        delete c;
        return nullptr;
    }
    BAGUA_LOG(3, "communicator rank %zu/%zu on device %zu ready", rank, nranks, device_id);
    return c;
}

void bagua_single_communicator_c_destroy(BaguaSingleCommunicatorC** ptr) {
    // bagua-core-c/src/lib.rs:32-53: null-safe, nulls the caller's pointer
    if (!ptr || !*ptr) return;
    BaguaSingleCommunicatorC* c = *ptr;
    if (c->t && c->aborted.load()) c->t->abort();
    *ptr = nullptr;
    if (c->t && c->t->in_use()) {
        // a thread is still inside an (aborted) call on this communicator: freeing it, or
        // its transport, would pull them from under that call -- both are kept
        BAGUA_LOG(0, "communicator rank %zu/%zu destroyed while a call is still inside it: kept", c->rank,
                  c->nranks);
        return;
    }
    delete c->t;
    delete c;
}

int32_t bagua_single_communicator_c_nranks(BaguaSingleCommunicatorC** ptr, size_t* nranks) {
    // bagua-core-c/src/lib.rs:55-69: 0 success, -1 null pointer
    if (!ptr || !*ptr || !nranks) return -1;
    *nranks = (*ptr)->nranks;
    return 0;
}

int32_t bagua_single_communicator_c_rank(BaguaSingleCommunicatorC** ptr, size_t* rank) {
    if (!ptr || !*ptr || !rank) return -1;
    *rank = (*ptr)->rank;
    return 0;
}

uint64_t bagua_single_communicator_c_stream(BaguaSingleCommunicatorC* c) {
    return c ? (uint64_t)(uintptr_t)c->stream : 0;
}

int bagua_comm_abort(BaguaSingleCommunicatorC* c) {
    // communicators/mod.rs:456-466
    if (!c) return BAGUA_ERR_INVALID_ARG;
    if (c->parent) c = c->parent;  // a lane view aborts the communicator it shares
    c->aborted.store(true);
    {
        std::lock_guard<std::mutex> g(c->lanes_mu);
        for (BaguaSingleCommunicatorC* v : c->lanes) v->aborted.store(true);
    }
    return c->t ? c->t->abort() : BAGUA_OK;
}

int bagua_comm_check_abort(BaguaSingleCommunicatorC* c) { return c && c->aborted.load() ? 1 : 0; }

int bagua_comm_schedule_config(BaguaSingleCommunicatorC* c, int32_t* out, int n) {
    if (!c || !out || n < 5) return BAGUA_ERR_INVALID_ARG;
    out[0] = c->cfg.pieces_cap;
    out[1] = c->cfg.min_piece;
    out[2] = c->cfg.taper;
    out[3] = c->cfg.multipath;
    out[4] = c->cfg.check;
    return BAGUA_OK;
}

int bagua_comm_allreduce_inplace(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int op) {
    // communicators/mod.rs:1020-1043 (count = num_elements_allocated)
    COMM_CHECK(c);
    if (!t) return BAGUA_ERR_INVALID_ARG;
    void* p = (void*)(uintptr_t)t->ptr;
    return c->t->allreduce(p, p, t->num_elem_allocated, t->dtype, op, c->stream);
}

int bagua_comm_allreduce(BaguaSingleCommunicatorC* c, const bagua_tensor_t* s, const bagua_tensor_t* r, int op) {
    COMM_CHECK(c);
    if (!s || !r || s->dtype != r->dtype || s->num_elem_allocated != r->num_elem_allocated) return BAGUA_ERR_INVALID_ARG;
    return c->t->allreduce((const void*)(uintptr_t)s->ptr, (void*)(uintptr_t)r->ptr, s->num_elem_allocated, s->dtype,
                           op, c->stream);
}

int bagua_comm_broadcast(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int root) {
    COMM_CHECK(c);
    if (!t) return BAGUA_ERR_INVALID_ARG;
    return c->t->broadcast((void*)(uintptr_t)t->ptr, t->num_elem_allocated, t->dtype, root, c->stream);
}

int bagua_comm_reduce_inplace(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int root, int op) {
    // communicators/mod.rs reduce_inplace (count = num_elements_allocated)
    COMM_CHECK(c);
    if (!t || root < 0 || (size_t)root >= c->nranks) return BAGUA_ERR_INVALID_ARG;
    void* p = (void*)(uintptr_t)t->ptr;
    return c->t->reduce(p, p, t->num_elem_allocated, t->dtype, op, root, c->stream);
}

int bagua_comm_reduce(BaguaSingleCommunicatorC* c, const bagua_tensor_t* s, const bagua_tensor_t* r, int root,
                      int op) {
    COMM_CHECK(c);
    if (!s || !r || s->dtype != r->dtype || s->num_elem_allocated != r->num_elem_allocated || root < 0 ||
        (size_t)root >= c->nranks)
        return BAGUA_ERR_INVALID_ARG;
    return c->t->reduce((const void*)(uintptr_t)s->ptr, (void*)(uintptr_t)r->ptr, s->num_elem_allocated, s->dtype, op,
                        root, c->stream);
}

int bagua_comm_alltoall(BaguaSingleCommunicatorC* c, const bagua_tensor_t* s, const bagua_tensor_t* r) {
    COMM_CHECK(c);
    if (!s || !r || s->dtype != r->dtype || s->num_elem_allocated % c->nranks ||
        r->num_elem_allocated < s->num_elem_allocated)
        return BAGUA_ERR_INVALID_ARG;
    return c->t->alltoall((const void*)(uintptr_t)s->ptr, (void*)(uintptr_t)r->ptr, s->num_elem_allocated / c->nranks,
                          s->dtype, c->stream);
}

int bagua_comm_alltoall_inplace(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t) {
    // communicators/mod.rs:602-630: count = allocated / nranks; rank r's slot r*count
    COMM_CHECK(c);
    if (!t || t->num_elem_allocated % c->nranks) return BAGUA_ERR_INVALID_ARG;  // "tensors must be aligned"
    const size_t bytes = t->num_elem_allocated * bagua_dtype_bytes(t->dtype);
    PoolBuffer tmp;
    int rc = tmp.allocate(c->device_id, bytes);
    if (rc) return rc;
    bagua_tensor_t r = *t;
    r.ptr = tmp.ptr();
    rc = bagua_comm_alltoall(c, t, &r);
    if (rc) return rc;
    if (hipMemcpyAsync((void*)(uintptr_t)t->ptr, tmp.as<void>(), bytes, hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
        return BAGUA_ERR_HIP;
    // the temp block goes back to the pool only after the copy has drained
    return hipStreamSynchronize(c->stream) == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP;
}

int bagua_comm_allgather_inplace(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t) {
    // communicators/mod.rs:760-787: in-place allgather, own slot at rank*count
    COMM_CHECK(c);
    if (!t || t->num_elem_allocated % c->nranks) return BAGUA_ERR_INVALID_ARG;
    const size_t count = t->num_elem_allocated / c->nranks;
    uint8_t* base = (uint8_t*)(uintptr_t)t->ptr;
    const size_t esz = bagua_dtype_bytes(t->dtype);
    return c->t->allgather(base + c->rank * count * esz, base, count, t->dtype, c->stream);
}

int bagua_comm_allgather(BaguaSingleCommunicatorC* c, const bagua_tensor_t* s, const bagua_tensor_t* r) {
    COMM_CHECK(c);
    if (!s || !r || r->num_elem_allocated != s->num_elem_allocated * c->nranks) return BAGUA_ERR_INVALID_ARG;
    return c->t->allgather((const void*)(uintptr_t)s->ptr, (void*)(uintptr_t)r->ptr, s->num_elem_allocated, s->dtype,
                           c->stream);
}

int bagua_comm_send(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int peer) {
    COMM_CHECK(c);
    if (!t) return BAGUA_ERR_INVALID_ARG;
    return c->t->send((const void*)(uintptr_t)t->ptr, t->num_elem_allocated, t->dtype, peer, c->stream);
}

int bagua_comm_recv(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int peer) {
    COMM_CHECK(c);
    if (!t) return BAGUA_ERR_INVALID_ARG;
    return c->t->recv((void*)(uintptr_t)t->ptr, t->num_elem_allocated, t->dtype, peer, c->stream);
}

int bagua_comm_group_start(void) { return nccl_status(ncclGroupStart()); }
int bagua_comm_group_end(void) { return nccl_status(ncclGroupEnd()); }

int bagua_comm_synchronize(BaguaSingleCommunicatorC* c) {
    if (!c) return BAGUA_ERR_INVALID_ARG;
    return hipStreamSynchronize(c->stream) == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP;
}

int bagua_comm_barrier(BaguaSingleCommunicatorC* c) {
    // communicators/mod.rs:973-: a tiny allreduce, then wait for it
    COMM_CHECK(c);
    PoolBuffer b;
    int rc = b.allocate(c->device_id, 4);
    if (rc) return rc;
    if (hipMemsetAsync(b.as<void>(), 0, 4, c->stream) != hipSuccess) return BAGUA_ERR_HIP;
    rc = c->t->allreduce(b.as<void>(), b.as<void>(), 1, BAGUA_DTYPE_F32, BAGUA_OP_SUM, c->stream);
    if (rc) return rc;
    return bagua_comm_synchronize(c);
}

}  // extern "C"
