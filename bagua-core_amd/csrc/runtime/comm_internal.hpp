// comm_internal.hpp — the transport behind a communicator.
//
// The comm ops (comm_ops.cpp) are written against this interface.  Product
// communicators use RcclTransport (RCCL over xGMI).  LoopbackTransport runs p
// virtual ranks as p host threads on ONE device, with collectives as
// device-to-device copies: it executes the very same op code at p > 1 on a
// one-GPU box, which is how the multi-rank path is parity-tested there.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "bagua_core.h"

#include <atomic>
#include <cstddef>
#include <cstdlib>
#include <mutex>
#include <vector>

namespace bagua {

struct Transport {
    virtual ~Transport() = default;
    // count is in elements of `dtype` (bagua dtype codes)
    virtual int allreduce(const void* send, void* recv, size_t count, int dtype, int op, hipStream_t s) = 0;
    virtual int broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s) = 0;
    // the reduction of every rank's `send` lands in `recv` on `root` (recv is unused elsewhere)
    virtual int reduce(const void* send, void* recv, size_t count, int dtype, int op, int root, hipStream_t s) = 0;
    // block j of `send` (count elements at j*count) goes to rank j; block j of `recv` comes from rank j
    virtual int alltoall(const void* send, void* recv, size_t count, int dtype, hipStream_t s) = 0;
    // rank j's `count` elements land at recv + j*count (in place when send == recv + rank*count)
    virtual int allgather(const void* send, void* recv, size_t count, int dtype, hipStream_t s) = 0;
    virtual int send(const void* buf, size_t count, int dtype, int peer, hipStream_t s) = 0;
    virtual int recv(void* buf, size_t count, int dtype, int peer, hipStream_t s) = 0;
    virtual int group_start() = 0;
    virtual int group_end() = 0;
    virtual int abort() = 0;
    // a call of some thread is still inside the transport (or a group bracket is open):
    // the transport may not be freed (bagua_single_communicator_c_destroy keeps it)
    virtual bool in_use() const { return false; }
};

Transport* make_rccl_transport(ncclComm_t comm);
ncclDataType_t nccl_dtype(int d);
int nccl_status(ncclResult_t r);

// The environment switches that change WHICH collectives an op posts (its piece
// schedule, its exchange pattern, the descriptor check).  Ranks that disagreed on
// them would post different collectives: a crash on the loopback transport, a hang
// over RCCL.  So they are read once, when a communicator is created, and over RCCL
// every rank adopts rank 0's values (agree_schedule_config, communicator.cpp); an op
// never reads them from its own rank's environment.
struct ScheduleConfig {
    int32_t pieces_cap = 4;        // BAGUA_PIPELINE_PIECES: most pieces per chunk (1 disables)
    int32_t min_piece = 1 << 20;   // BAGUA_PIPELINE_MIN_PIECE: payload bytes per chunk piece
    // BAGUA_PIPELINE_TAPER: first and last piece half size (from 3 pieces).  -1 (unset):
    // the schedules an op chooses itself (the caller asked for 0 pieces) are tapered;
    // 0: none unless the caller asks (BAGUA_PIECES_TAPERED); 1: every plain count too
    int32_t taper = -1;
    int32_t multipath = 0;         // BAGUA_RING_MULTIPATH=1: relayed ring exchange from 6 ranks
    int32_t check = 0;             // BAGUA_CHECK_SCHEDULE=1: ranks compare op descriptors first
    int32_t reserved[3] = {0, 0, 0};
    bool operator==(const ScheduleConfig& o) const {
        return pieces_cap == o.pieces_cap && min_piece == o.min_piece && taper == o.taper &&
               multipath == o.multipath && check == o.check;
    }
};
ScheduleConfig read_schedule_config();

// set by the native scheduler's worker thread: comm ops it runs are async
extern thread_local bool g_async_ops;

}  // namespace bagua

struct BaguaSingleCommunicatorC {
    bagua::Transport* t = nullptr;
    size_t rank = 0;
    size_t nranks = 1;
    int device_id = 0;
    hipStream_t stream = nullptr;
    std::atomic<bool> aborted{false};
    bagua::ScheduleConfig cfg;  // fixed at creation, equal on every rank (see ScheduleConfig)
    std::atomic<uint64_t> op_seq{0};  // ops checked so far (BAGUA_CHECK_SCHEDULE; a lane view counts on its parent)
    // pipelined ops: a second stream for the exchange of piece k while `stream`
    // runs the codec on piece k+1, and the events that order the two (lazy)
    hipStream_t side = nullptr;
    std::vector<hipEvent_t> events;
    hipEvent_t join = nullptr;  // async ops: the side stream's end, waited for by `stream`
    // async ops (bagua_comm_set_async, or the native scheduler's worker): an op returns
    // once its work is enqueued; buffers go back to the pool behind the stream
    bool async = false;
    // Lane views (the scheduler's cross-bucket pipelining, backend.cpp): communicators
    // that share this one's transport, rank and device but own their streams, side
    // streams and events, so consecutive buckets' ops run on different streams and
    // bucket b+1's codec prefix overlaps bucket b's exchange and tail.  The claim this
    // rests on: RCCL (2.26.6, the librccl that PyTorch 2.10+rocm7.0 loads first and this
    // library binds to; /opt/rocm's 2.27.7 otherwise) runs one
    // communicator's operations in the order they are issued whatever the user stream
    // -- every launch of a communicator is chained behind the previous one on the
    // communicator's internal device stream before the user stream joins it -- and the
    // scheduler's one worker thread issues every lane's ops, so the collective order
    // stays identical on every rank.  Pinned by test_native_scheduler_lanes_over_rccl
    // (7 buckets x 2 steps on 3 lanes of one RCCL communicator, bit-exact against the
    // oracle).  A view never owns the transport.
    BaguaSingleCommunicatorC* parent = nullptr;
    bool own_stream = false;
    std::mutex lanes_mu;
    std::vector<BaguaSingleCommunicatorC*> lanes;  // lanes[i] = view i + 1 (lane 0 is this one)

    // lane `i` (0: this communicator itself); nullptr when its stream cannot be created
    BaguaSingleCommunicatorC* lane(int i);

    int ensure_side(size_t n_events) {
        if (!side && hipStreamCreateWithFlags(&side, hipStreamNonBlocking) != hipSuccess) {
            side = nullptr;
            return -1;
        }
        // cross-stream ordering on one device needs no system-scope fence (the
        // producer kernel's own end-of-kernel release covers the device);
        // BAGUA_EVENT_SYSTEM_FENCE=1 restores it (A/B)
        static const unsigned flags = [] {
            const char* v = std::getenv("BAGUA_EVENT_SYSTEM_FENCE");
            return (v && *v && std::atoi(v) != 0) ? (unsigned)hipEventDisableTiming
                                                   : (unsigned)(hipEventDisableTiming | hipEventDisableSystemFence);
        }();
        while (events.size() < n_events) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, flags) != hipSuccess) return -1;
            events.push_back(e);
        }
        if (!join && hipEventCreateWithFlags(&join, flags) != hipSuccess) {
            join = nullptr;
            return -1;
        }
        return 0;
    }
    ~BaguaSingleCommunicatorC() {
        for (BaguaSingleCommunicatorC* v : lanes) delete v;
        // per-stream workspaces and one-launch encode slots of the streams this
        // communicator ran ops on (the side stream is destroyed right after);
        // release waits for the streams, so an aborted communicator, whose
        // streams may hold collectives that never complete, keeps them
        if (!aborted.load()) {
            (void)bagua_release_stream_resources(device_id, (uint64_t)(uintptr_t)stream);
            if (side) (void)bagua_release_stream_resources(device_id, (uint64_t)(uintptr_t)side);
        }
        // a lane view's stream leaves the one-launch encode's opt-out set even when the
        // stream itself is kept (aborted): a later stream reusing the handle value must
        // not inherit the opt-out
        if (own_stream && stream) (void)bagua_minmax_u8_set_stream_resident(stream, 1);
        for (hipEvent_t e : events) (void)hipEventDestroy(e);
        if (join) (void)hipEventDestroy(join);
        if (side) (void)hipStreamDestroy(side);
        if (own_stream && stream && !aborted.load()) (void)hipStreamDestroy(stream);
    }
};

namespace bagua {
inline bool async_ops(const BaguaSingleCommunicatorC* c) { return c->async || g_async_ops; }
}  // namespace bagua
