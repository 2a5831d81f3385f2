// backend.cpp — native bucket + ordered-bucket scheduler.
//
// Replaces the reference's Rust scheduler (bagua-core-internal/src/lib.rs:
// 125-338, BaguaCommBackend) and bucket (datatypes/mod.rs:1072-1267,
// BaguaBucket):
//   * register_ordered_buckets fixes the order (duplicate tensor names or
//     pointers are refused, lib.rs:270-298);
//   * mark_communication_ready(tensor, ready event) marks a tensor, and while
//     the FRONT bucket is fully ready it is rotated to the back and scheduled on
//     a bounded channel to one worker thread (lib.rs:300-319);
//   * the worker makes the bucket's stream wait for every tensor's ready event,
//     builds the communication tensor (in place when the tensors are back to
//     back, else a pool buffer packed on the stream and copied back after the
//     ops, datatypes/mod.rs:963-1070), runs the bucket's comm ops through the
//     C ABI (comm_ops.cpp) and marks the item done (lib.rs:209-254);
//   * wait_pending_comm_ops waits for every scheduled item (lib.rs:321-337);
//   * a monitor fails an op that runs longer than 300 s (lib.rs:255-265,
//     BAGUA_COMM_OP_TIMEOUT_S or bagua_comm_backend_set_op_timeout_ms): the
//     reference panics and its hook exits the process (py/lib.rs:498-504); here the
//     monitor logs the op, keeps the message (bagua_comm_backend_failure_message),
//     aborts the op's communicators -- ncclCommAbort releases RCCL kernels waiting
//     for a peer that never comes, the loopback transport breaks its barrier -- and
//     wait_pending_comm_ops returns BAGUA_ERR_ABORTED instead of waiting forever.
//   * cross-bucket pipelining (async mode, BAGUA_SCHED_LANES, default 3): bucket
//     i of the registration order runs its ops on lane 1 + i % lanes of its
//     communicator -- a view with its own streams (comm_internal.hpp) -- so the
//     next bucket's compress prefix and enqueue overlap this bucket's exchange and
//     tail instead of queueing behind them on one stream.  A bucket always uses
//     the same lane (its executions stay in stream order), the worker issues every
//     lane's ops in schedule order (the collective order every rank sees), and
//     buckets with hierarchical ops or several communicators stay on lane 0.
// No Python on this path: the worker never takes the GIL unless a bucket
// carries a Python callback op (python_ffi_op.rs), which ctypes runs with it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "bagua_core.h"
#include "comm_internal.hpp"
#include "runtime_util.hpp"

namespace {

struct BucketTensor {
    bagua_tensor_t t;
    std::string name;
};

}  // namespace

struct BaguaBucketC {
    std::string name;
    int sched_index = 0;  // position in the scheduler's registration order (its lane)
    std::vector<BucketTensor> tensors;
    std::vector<bagua_bucket_op_t> ops;
    // readiness per tensor (guarded by `mu`): a mark is one hash lookup and a flag, and
    // the readiness test a compare -- the reference's name set (datatypes/mod.rs:1256-1266)
    // costs a walk over the bucket per mark
    std::unordered_map<std::string, std::vector<int>> index;  // name -> tensor indices
    std::vector<uint8_t> ready;       // tensor i marked since the last reset
    std::vector<uint64_t> events;     // tensor i's ready event of the next execution (0: none)
    std::vector<uint8_t> padding;     // "bagua_padding_tensor*": always counts as ready
    int marked = 0, needed = 0;       // marked non-padding tensors / non-padding tensors
    std::mutex mu;

    void init_index() {
        const size_t n = tensors.size();
        ready.assign(n, 0);
        events.assign(n, 0);
        padding.assign(n, 0);
        marked = needed = 0;
        for (size_t i = 0; i < n; ++i) {
            index[tensors[i].name].push_back((int)i);
            padding[i] = tensors[i].name.rfind("bagua_padding_tensor", 0) == 0;
            needed += !padding[i];
        }
    }
    void mark_locked(int i, uint64_t ev) {
        if (!ready[i]) {
            ready[i] = 1;
            marked += !padding[i];
        }
        if (ev) events[i] = ev;
    }
    void reset_locked() {
        std::fill(ready.begin(), ready.end(), 0);
        marked = 0;
    }
    bool ready_for_comm() {  // datatypes/mod.rs:1256-1266 (padding tensors count as ready)
        std::lock_guard<std::mutex> g(mu);
        return marked == needed;
    }
};

namespace {

using namespace bagua;

hipStream_t ops_stream(const std::vector<bagua_bucket_op_t>& ops) {
    for (const bagua_bucket_op_t& op : ops) {
        if (op.intranode) return op.intranode->stream;  // hierarchical: the node's stream (communicators/mod.rs:385-392)
        if (op.comm) return op.comm->stream;
    }
    return nullptr;
}

// the ops return once enqueued: run by the scheduler's worker, or on a communicator
// set async (bagua_comm_set_async)
bool ops_async(const std::vector<bagua_bucket_op_t>& ops) {
    if (g_async_ops) return true;
    for (const bagua_bucket_op_t& op : ops)
        if ((op.comm && op.comm->async) || (op.intranode && op.intranode->async)) return true;
    return false;
}

int run_op(const bagua_bucket_op_t& op, const bagua_tensor_t* flat, const char* bucket_name, hipStream_t s,
           bool async) {
    if (op.intranode) {  // hierarchical mode (communicators/mod.rs:390-427)
        switch (op.kind) {
            case BAGUA_BUCKET_OP_CENTRALIZED_LOW_PRECISION:
                return bagua_centralized_low_precision_hierarchical(op.intranode, op.comm, flat, op.average,
                                                                    op.compression);
            case BAGUA_BUCKET_OP_CENTRALIZED_FULL_PRECISION:
                return bagua_centralized_full_precision_hierarchical(op.intranode, op.comm, flat, op.average);
            case BAGUA_BUCKET_OP_DECENTRALIZED_LOW_PRECISION:
                return bagua_decentralized_low_precision_hierarchical(op.intranode, op.comm, flat, &op.weight,
                                                                      &op.left_peer_weight, &op.right_peer_weight,
                                                                      op.compression);
            default:
                break;
        }
    }
    switch (op.kind) {
        case BAGUA_BUCKET_OP_CENTRALIZED_LOW_PRECISION:
            return op.fused ? bagua_centralized_low_precision_synchronous(op.comm, flat, op.average, op.compression)
                            : bagua_centralized_low_precision_synchronous_unfused(op.comm, flat, op.average,
                                                                                  op.compression);
        case BAGUA_BUCKET_OP_CENTRALIZED_FULL_PRECISION:
            return bagua_centralized_full_precision_synchronous(op.comm, flat, op.average);
        case BAGUA_BUCKET_OP_DECENTRALIZED_LOW_PRECISION:
            return bagua_decentralized_low_precision_synchronous(op.comm, flat, &op.weight, &op.left_peer_weight,
                                                                 &op.right_peer_weight, op.compression);
        case BAGUA_BUCKET_OP_CALLBACK:
            // the callback sees the previous ops' results, as in the reference (their
            // Drop synced), also when the worker runs the ops async
            if (async && s && hipStreamSynchronize(s) != hipSuccess) return BAGUA_ERR_HIP;
            if (op.callback) op.callback(op.user, bucket_name);  // python_ffi_op.rs: call with the bucket name
            return BAGUA_OK;
    }
    return BAGUA_ERR_UNSUPPORTED;
}

// the ready events a bucket collected, consumed once (datatypes/mod.rs:969-980 zeroes them)
std::vector<uint64_t> take_events(BaguaBucketC* b) {
    std::lock_guard<std::mutex> g(b->mu);
    std::vector<uint64_t> ev;
    for (uint64_t& e : b->events) {  // one stream wait per distinct event (tensors often share one)
        if (e && std::find(ev.begin(), ev.end(), e) == ev.end()) ev.push_back(e);
        e = 0;
    }
    return ev;
}

std::vector<bagua_bucket_op_t> copy_ops(BaguaBucketC* b) {
    std::lock_guard<std::mutex> g(b->mu);
    return b->ops;
}

std::vector<BucketTensor> copy_tensors(BaguaBucketC* b) {
    std::lock_guard<std::mutex> g(b->mu);
    return b->tensors;
}

// `to` waits for the work queued on `from` so far (nothing when they are the same stream)
int order_after(hipStream_t to, hipStream_t from) {
    if (to == from) return BAGUA_OK;
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return BAGUA_ERR_HIP;
    const bool ok = hipEventRecord(e, from) == hipSuccess && hipStreamWaitEvent(to, e, 0) == hipSuccess;
    (void)hipEventDestroy(e);  // released once the recorded work completes
    return ok ? BAGUA_OK : BAGUA_ERR_HIP;
}

// get_communication_tensor + ops + Drop (datatypes/mod.rs:963-1070) with the
// tensors, events and ops the bucket had when it was scheduled (lib.rs:143-146
// clones the ops; the reference reads each tensor's data_ptr at run time, here
// the descriptors refreshed by mark-ready / execute).  `s` carries the ready
// waits, the pack and the copy-back; the ops run on their communicator's stream
// `os`, ordered after the pack and before the copy-back.
int execute_bucket(BaguaBucketC* b, const std::vector<BucketTensor>& tensors, const std::vector<uint64_t>& events,
                   const std::vector<bagua_bucket_op_t>& ops, hipStream_t s) {
    if (tensors.empty()) return BAGUA_ERR_INVALID_ARG;
    const bagua_tensor_t& first = tensors[0].t;
    DeviceGuard guard(first.device_id);
    // :969-980 the stream waits for every tensor's ready event -- unless it has already
    // completed: a stream wait costs the queue a barrier packet (a few us between two
    // buckets' kernels) even when there is nothing left to wait for
    for (uint64_t ev : events) {
        const hipError_t q = hipEventQuery((hipEvent_t)(uintptr_t)ev);
        if (q == hipSuccess) continue;
        if (q != hipErrorNotReady) (void)hipGetLastError();
        if (hipStreamWaitEvent(s, (hipEvent_t)(uintptr_t)ev, 0) != hipSuccess) return BAGUA_ERR_HIP;
    }
    if (ops.empty()) return BAGUA_OK;
    hipStream_t os = ops_stream(ops);
    if (!os) os = s;
    const bool async = ops_async(ops);
    const size_t esz = bagua_dtype_bytes(first.dtype);
    uint64_t total_alloc = 0, total = 0;
    bool contig = true;
    uint64_t cur = 0;
    for (size_t i = 0; i < tensors.size(); ++i) {
        const bagua_tensor_t& t = tensors[i].t;
        total_alloc += t.num_elem_allocated;
        total += t.num_elem;
        if (i > 0 && t.ptr != cur) contig = false;
        cur = t.ptr + t.num_elem_allocated * esz;
    }
    int rc = BAGUA_OK;
    if (contig) {
        if ((rc = order_after(os, s)) != BAGUA_OK) return rc;
        const bagua_tensor_t flat{first.ptr, total_alloc, total_alloc, first.dtype, first.device_id};
        for (const bagua_bucket_op_t& op : ops)
            if ((rc = run_op(op, &flat, b->name.c_str(), os, async)) != BAGUA_OK) break;
        const int rc2 = order_after(s, os);  // the caller's stream sees the results
        return rc != BAGUA_OK ? rc : rc2;
    }
    // :999-1038 pack num_elements() of every tensor into a pool buffer on the stream
    PoolBuffer buf;
    if ((rc = buf.allocate(first.device_id, total_alloc * esz)) != BAGUA_OK) return rc;
    uint8_t* dst = buf.as<uint8_t>();
    for (const BucketTensor& t : tensors) {
        const size_t bytes = t.t.num_elem * esz;
        if (bytes && hipMemcpyAsync(dst, (const void*)(uintptr_t)t.t.ptr, bytes, hipMemcpyDeviceToDevice, s) !=
                         hipSuccess)
            return BAGUA_ERR_HIP;
        dst += bytes;
    }
    if ((rc = order_after(os, s)) != BAGUA_OK) return rc;  // the ops read the packed buffer
    const bagua_tensor_t flat{buf.ptr(), total, total_alloc, first.dtype, first.device_id};
    for (const bagua_bucket_op_t& op : ops)
        if ((rc = run_op(op, &flat, b->name.c_str(), os, async)) != BAGUA_OK) break;
    // :1043-1070 copy back, then wait for the stream (the buffer returns to the pool);
    // async: the buffer returns to the pool behind the stream instead.  Queued work
    // of a failed op still writes the buffer: the copy-back is skipped, the buffer's
    // release stays ordered behind both streams.
    const int ord = order_after(s, os);
    if (rc == BAGUA_OK) rc = ord;
    const uint8_t* src = buf.as<uint8_t>();
    for (const BucketTensor& t : tensors) {
        const size_t bytes = t.t.num_elem * esz;
        if (rc == BAGUA_OK && bytes &&
            hipMemcpyAsync((void*)(uintptr_t)t.t.ptr, src, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
            rc = BAGUA_ERR_HIP;
        src += bytes;
    }
    if (async) {
        const uint64_t sv[2] = {(uint64_t)(uintptr_t)s, (uint64_t)(uintptr_t)os};
        const uint64_t p = buf.ptr();
        buf.release_to_caller();
        (void)pool_free_after(p, sv, os == s ? 1 : 2);
        return rc;
    }
    const hipError_t e = hipStreamSynchronize(s);
    const hipError_t e2 = os == s ? hipSuccess : hipStreamSynchronize(os);
    return rc != BAGUA_OK ? rc : (e == hipSuccess && e2 == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP);
}

// the bucket's ops moved onto lane `lane` of their communicator: every op on one
// (non-hierarchical) communicator, else nothing changes (false)
bool ops_on_lane(std::vector<bagua_bucket_op_t>* ops, int lane) {
    BaguaSingleCommunicatorC* comm = nullptr;
    for (const bagua_bucket_op_t& op : *ops) {
        if (op.intranode) return false;
        if (!op.comm) continue;
        if (comm && op.comm != comm) return false;
        comm = op.comm;
    }
    if (!comm || comm->parent) return false;
    BaguaSingleCommunicatorC* view = comm->lane(lane);
    if (!view) return false;
    for (bagua_bucket_op_t& op : *ops)
        if (op.comm) op.comm = view;
    return true;
}

struct Scheduled {
    BaguaBucketC* bucket = nullptr;
    int lane_hint = 0;                     // the bucket's registration index
    std::vector<BucketTensor> tensors;     // tensor descriptors at scheduling time
    std::vector<uint64_t> events;          // ready events at scheduling time
    std::vector<bagua_bucket_op_t> ops;    // the bucket's ops at scheduling time
    bool done = false;                     // executed (sync) / enqueued (async)
    int status = BAGUA_OK;
    std::chrono::steady_clock::time_point started;  // the worker picked it up (monitor clock)
    std::atomic<bool> timed_out{false};    // the monitor aborted its communicators
    std::atomic<int64_t> abort_ns{0};      // when (steady clock)
    bool waited = false;                   // wait_pending_comm_ops is done with it (guarded by mu)
    // async: an event recorded on the bucket's stream behind its work, shared by every
    // bucket the worker enqueued on that stream since the previous record (back to the
    // backend's pool with the last of them)
    std::shared_ptr<void> finished;
};

}  // namespace

struct BaguaCommBackendC {
    int device = 0;
    size_t cap = 1;
    std::mutex mu;
    std::condition_variable cv_work, cv_space, cv_done;
    std::deque<BaguaBucketC*> ordered;
    std::unordered_map<std::string, BaguaBucketC*> mapping;  // tensor name -> bucket
    std::deque<std::shared_ptr<Scheduled>> channel;          // bounded by `cap`
    std::deque<std::shared_ptr<Scheduled>> pending;          // scheduled, not yet waited for
    std::shared_ptr<Scheduled> current;
    std::chrono::steady_clock::time_point current_start;
    std::vector<std::string> failures;
    // items the worker picked up and the monitor watches until their work completed
    std::deque<std::shared_ptr<Scheduled>> inflight;
    std::vector<std::shared_ptr<Scheduled>> stuck;  // abandoned items (their worker call never returned)
    std::chrono::milliseconds op_timeout{300000};  // lib.rs:255-265 (BAGUA_COMM_OP_TIMEOUT_S)
    bool stop = false;
    bool worker_done = false;   // work() returned (destroy waits for it, or leaves a stuck worker)
    bool stop_monitor = false;  // the monitor outlives `stop` until the worker is done or left
    bool async = true;                  // BAGUA_BACKEND_SYNC=1: every op waits for its stream
    // BAGUA_SCHED_LANES (async only; 1 = every bucket on the comm's stream).  3: 32 x 25 MiB at
    // one rank 1,521-1,582 GiB/s vs 1,373-1,475 with 2 and 1,380-1,419 with 4
    // (profiles/r04_sched_lanes_sweep.jsonl)
    int lanes = 3;
    std::thread worker, monitor;
    // async, worker thread only: buckets enqueued whose completion is not recorded yet,
    // with their stream
    std::vector<std::pair<std::shared_ptr<Scheduled>, hipStream_t>> uncovered;
    // completion events for reuse: an event returns here when the last bucket sharing it
    // is released by wait_pending_comm_ops (after its synchronisation); own mutex, never
    // held while taking `mu`
    std::mutex spare_mu;
    std::vector<hipEvent_t> spare;

    std::shared_ptr<void> completion_event(hipStream_t s) {
        hipEvent_t e = nullptr;
        {
            std::lock_guard<std::mutex> lk(spare_mu);
            if (!spare.empty()) {
                e = spare.back();
                spare.pop_back();
            }
        }
        // completion only: no system-scope fence (profiles/r02_slot_event_ab.jsonl)
        if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess)
            e = nullptr;
        if (e && hipEventRecord(e, s) != hipSuccess) {
            (void)hipEventDestroy(e);
            e = nullptr;
        }
        if (!e) return nullptr;
        return std::shared_ptr<void>(e, [this](void* x) {
            std::lock_guard<std::mutex> lk(spare_mu);
            spare.push_back((hipEvent_t)x);
        });
    }

    // Completion of the enqueued buckets: ONE event per stream behind all of them,
    // recorded when the worker runs out of queued buckets.  A lane's stream runs its
    // buckets in order, so the last record covers every earlier one, and a burst of
    // buckets costs one record per lane instead of one per bucket (a record is ~3 us of
    // worker time; the buckets are marked done -- wait_pending_comm_ops may look at them
    // only once covered).
    void cover_uncovered() {
        if (uncovered.empty()) return;
        std::vector<std::pair<hipStream_t, std::shared_ptr<void>>> recs;
        for (const auto& u : uncovered) {
            bool seen = false;
            for (const auto& r : recs) seen = seen || r.first == u.second;
            if (seen) continue;
            std::shared_ptr<void> e = completion_event(u.second);
            if (!e) (void)hipStreamSynchronize(u.second);  // nothing to wait on later: drain now
            recs.emplace_back(u.second, std::move(e));
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            for (const auto& u : uncovered) {
                for (const auto& r : recs)
                    if (r.first == u.second) u.first->finished = r.second;
                // also after a failed op: its bucket's earlier work may still be queued,
                // and wait_pending_comm_ops must not return before it drained
                if (!u.first->finished && u.first->status == BAGUA_OK) u.first->status = BAGUA_ERR_HIP;
                u.first->done = true;
            }
        }
        uncovered.clear();
        cv_done.notify_all();
    }

    // BAGUA_SCHED_PROFILE=1: host time per bucket (waiting for work / execute_bucket /
    // completion event), printed when the backend is destroyed (measurement hook)
    bool profile = false;
    std::vector<std::array<double, 3>> prof;
    size_t prof_n = 0;
    double prof_quantile(int k, double q) const {  // over the second half of the buckets (warm)
        std::vector<double> v;
        for (size_t i = prof.size() / 2; i < prof.size(); ++i) v.push_back(prof[i][k]);
        if (v.empty()) return 0;
        std::sort(v.begin(), v.end());
        return v[(size_t)(q * (double)(v.size() - 1))];
    }
    double prof_median(int k) const { return prof_quantile(k, 0.5); }

    void work() {
        (void)hipSetDevice(device);  // lib.rs:210-213
        using clk = std::chrono::steady_clock;
        auto us = [](clk::time_point a, clk::time_point b) {
            return std::chrono::duration<double, std::micro>(b - a).count();
        };
        // async: ops return once enqueued; buckets run back to back on their lane's
        // stream and wait_pending_comm_ops waits for the completion events covering them
        // (cover_uncovered)
        g_async_ops = async;
        for (;;) {
            std::shared_ptr<Scheduled> item;
            const clk::time_point t_wait = clk::now();
            {
                std::unique_lock<std::mutex> lk(mu);
                if (channel.empty() && !uncovered.empty()) {  // out of work: record completions
                    lk.unlock();
                    cover_uncovered();
                    lk.lock();
                }
                cv_work.wait(lk, [&] { return stop || !channel.empty(); });
                if (channel.empty()) {  // stopping with nothing queued
                    lk.unlock();
                    cover_uncovered();
                    lk.lock();
                    worker_done = true;
                    cv_done.notify_all();
                    return;
                }
                item = channel.front();
                channel.pop_front();
                cv_space.notify_all();
                current = item;
                current_start = std::chrono::steady_clock::now();
                item->started = current_start;
                while (!inflight.empty() && inflight.front()->waited) inflight.pop_front();
                inflight.push_back(item);
            }
            const clk::time_point t_exec = clk::now();
            int nl;
            {
                std::lock_guard<std::mutex> lk(mu);
                nl = lanes;
            }
            std::vector<bagua_bucket_op_t> ops = item->ops;
            if (async && nl > 1 && !ops_on_lane(&ops, 1 + item->lane_hint % nl)) ops = item->ops;
            hipStream_t s = ops_stream(ops);
            const int rc = execute_bucket(item->bucket, item->tensors, item->events, ops, s);
            const clk::time_point t_fin = clk::now();
            bool idle = false;
            {
                std::lock_guard<std::mutex> lk(mu);
                if (item->status == BAGUA_OK) item->status = rc;  // the monitor's ABORTED stays
                if (!async) item->done = true;
                current.reset();
                idle = channel.empty();
            }
            if (async) {
                uncovered.emplace_back(item, s);
                if (idle) cover_uncovered();
            } else {
                cv_done.notify_all();
            }
            if (profile && prof.size() < (1u << 20)) {  // bounded: a measurement hook, not a log
                prof.push_back({us(t_wait, t_exec), us(t_exec, t_fin), us(t_fin, clk::now())});
                ++prof_n;
            }
        }
    }

    // A watched item's work is over: executed (sync) or its completion event reached
    // (async; a bucket without one failed or was waited for already).  Caller holds mu.
    static bool settled_locked(const Scheduled& it, std::shared_ptr<void>* ev) {
        if (!it.done) return false;
        *ev = it.finished;
        return !it.finished;
    }

    std::condition_variable cv_watch;

    void watch() {
        std::unique_lock<std::mutex> lk(mu);
        while (!stop_monitor) {
            // tick: a quarter of the limit, between 10 ms and 5 s
            const auto tick = std::max(std::chrono::milliseconds(10),
                                       std::min(std::chrono::milliseconds(5000), op_timeout / 4));
            cv_watch.wait_for(lk, tick);
            if (stop_monitor) break;
            const auto now = std::chrono::steady_clock::now();
            std::vector<std::shared_ptr<Scheduled>> expired;
            for (auto it = inflight.begin(); it != inflight.end();) {
                std::shared_ptr<void> ev;
                bool over = (*it)->waited || settled_locked(**it, &ev);
                if (!over && ev) {
                    const hipError_t q = hipEventQuery((hipEvent_t)ev.get());
                    over = q != hipErrorNotReady;
                    if (q != hipSuccess && q != hipErrorNotReady) (void)hipGetLastError();
                }
                if ((*it)->waited || over || (*it)->timed_out.load()) {
                    it = inflight.erase(it);
                    continue;
                }
                if (now - (*it)->started > op_timeout) {
                    expired.push_back(*it);
                    it = inflight.erase(it);
                    continue;
                }
                ++it;
            }
            if (expired.empty()) continue;
            for (const auto& item : expired) {
                const long long s_lim = (long long)(op_timeout.count() / 1000);
                const std::string msg = "comm op on bucket " + item->bucket->name + " has not finished for " +
                                        (s_lim ? std::to_string(s_lim) + " s"
                                               : std::to_string((long long)op_timeout.count()) + " ms") +
                                        "; its communicators are aborted";
                failures.push_back(msg);
                BAGUA_LOG(0, "%s", msg.c_str());
                if (item->status == BAGUA_OK) item->status = BAGUA_ERR_ABORTED;
            }
            lk.unlock();  // an abort may wait for calls inside RCCL
            for (const auto& item : expired) {
                for (const bagua_bucket_op_t& op : item->ops) {
                    if (op.comm) (void)bagua_comm_abort(op.comm);
                    if (op.intranode) (void)bagua_comm_abort(op.intranode);
                }
                item->abort_ns.store(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                         std::chrono::steady_clock::now().time_since_epoch())
                                         .count());
                item->timed_out.store(true);
            }
            lk.lock();
            cv_done.notify_all();
        }
    }

    // How long wait_pending_comm_ops still waits for an aborted op's work to drain
    // (RCCL kernels leave once their communicator is aborted; a transport that does not
    // release them must not turn the failure into a hang)
    static bool abandoned(const Scheduled& it) {
        if (!it.timed_out.load()) return false;
        const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                std::chrono::steady_clock::now().time_since_epoch())
                                .count();
        return now - it.abort_ns.load() > 10'000'000'000LL;
    }

    // the event completed (true), failed, or belongs to an abandoned op (false); polls,
    // so the monitor's abort can end the wait
    static bool wait_event(hipEvent_t e, const Scheduled& it) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t q = hipEventQuery(e);
            if (q == hipSuccess) return true;
            if (q != hipErrorNotReady) {
                (void)hipGetLastError();
                return false;
            }
            if (abandoned(it)) return false;
            if (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(20))
                std::this_thread::yield();
            else
                std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
    }
};

extern "C" {

BaguaBucketC* bagua_bucket_create(const char* name, const bagua_tensor_t* tensors, const char* const* tensor_names,
                                  int n, int* status) {
    // datatypes/mod.rs:1079-1118 (same dtype and device; allocated >= num_elem)
    int st = BAGUA_OK;
    if (!name || !tensors || !tensor_names || n <= 0) st = BAGUA_ERR_INVALID_ARG;
    for (int i = 0; st == BAGUA_OK && i < n; ++i) {
        if (!tensor_names[i] || tensors[i].dtype != tensors[0].dtype || tensors[i].device_id != tensors[0].device_id ||
            tensors[i].num_elem_allocated < tensors[i].num_elem || !bagua_dtype_bytes(tensors[i].dtype))
            st = BAGUA_ERR_INVALID_ARG;
    }
    if (status) *status = st;
    if (st != BAGUA_OK) return nullptr;
    auto* b = new BaguaBucketC();
    b->name = name;
    for (int i = 0; i < n; ++i) b->tensors.push_back(BucketTensor{tensors[i], tensor_names[i]});
    b->init_index();
    return b;
}

void bagua_bucket_destroy(BaguaBucketC* b) { delete b; }

int bagua_bucket_append_op(BaguaBucketC* b, const bagua_bucket_op_t* op) {
    if (!b || !op) return BAGUA_ERR_INVALID_ARG;
    // a node worker in hierarchical mode has no internode communicator
    if (op->kind != BAGUA_BUCKET_OP_CALLBACK && !op->comm && !op->intranode) return BAGUA_ERR_INVALID_ARG;
    if (op->intranode && op->intranode->rank == 0 && !op->comm) return BAGUA_ERR_INVALID_ARG;
    if (op->kind < BAGUA_BUCKET_OP_CENTRALIZED_LOW_PRECISION || op->kind > BAGUA_BUCKET_OP_CALLBACK)
        return BAGUA_ERR_UNSUPPORTED;
    std::lock_guard<std::mutex> g(b->mu);
    b->ops.push_back(*op);
    return BAGUA_OK;
}

int bagua_bucket_clear_ops(BaguaBucketC* b) {
    if (!b) return BAGUA_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(b->mu);
    b->ops.clear();
    return BAGUA_OK;
}

int bagua_bucket_num_ops(BaguaBucketC* b) {
    if (!b) return -1;
    std::lock_guard<std::mutex> g(b->mu);
    return (int)b->ops.size();
}

int bagua_bucket_mark_tensor_ready(BaguaBucketC* b, const char* tensor_name, uint64_t ready_event) {
    return bagua_bucket_mark_tensor_ready_desc(b, tensor_name, ready_event, nullptr);
}

namespace {
// a tensor's current descriptor replaces the recorded one (the reference reads
// data_ptr/numel from the torch tensor at run time, datatypes/mod.rs:775-791);
// dtype and device may not change (datatypes/mod.rs:1079-1118).  Caller holds mu.
int refresh_locked(BucketTensor& t, const bagua_tensor_t* cur) {
    if (!cur) return BAGUA_OK;
    if (cur->dtype != t.t.dtype || cur->device_id != t.t.device_id || cur->num_elem_allocated < cur->num_elem)
        return BAGUA_ERR_INVALID_ARG;
    t.t = *cur;
    return BAGUA_OK;
}
}  // namespace

int bagua_bucket_mark_tensor_ready_desc(BaguaBucketC* b, const char* tensor_name, uint64_t ready_event,
                                        const bagua_tensor_t* current) {
    if (!b || !tensor_name) return BAGUA_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(b->mu);
    const auto it = b->index.find(tensor_name);
    if (it == b->index.end()) return BAGUA_ERR_INVALID_ARG;
    for (const int i : it->second) {
        const int rc = refresh_locked(b->tensors[i], current);
        if (rc != BAGUA_OK) return rc;
        b->mark_locked(i, ready_event);
    }
    return BAGUA_OK;
}

int bagua_bucket_refresh_tensor(BaguaBucketC* b, const char* tensor_name, const bagua_tensor_t* current) {
    if (!b || !tensor_name || !current) return BAGUA_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(b->mu);
    const auto it = b->index.find(tensor_name);
    if (it == b->index.end()) return BAGUA_ERR_INVALID_ARG;
    for (const int i : it->second) {
        const int rc = refresh_locked(b->tensors[i], current);
        if (rc != BAGUA_OK) return rc;
    }
    return BAGUA_OK;
}

int bagua_bucket_ready_for_comm(BaguaBucketC* b) { return b && b->ready_for_comm() ? 1 : 0; }

int bagua_bucket_reset_comm_ready(BaguaBucketC* b) {
    if (!b) return BAGUA_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(b->mu);
    b->reset_locked();
    return BAGUA_OK;
}

int bagua_bucket_execute(BaguaBucketC* b, uint64_t stream) {
    if (!b) return BAGUA_ERR_INVALID_ARG;
    const std::vector<bagua_bucket_op_t> ops = copy_ops(b);
    hipStream_t s = stream ? (hipStream_t)(uintptr_t)stream : ops_stream(ops);
    return execute_bucket(b, copy_tensors(b), take_events(b), ops, s);
}

BaguaCommBackendC* bagua_comm_backend_create(size_t schedule_channel_cap, int device_id) {
    if (hipSetDevice(device_id) != hipSuccess) return nullptr;  // lib.rs:177-181
    auto* be = new BaguaCommBackendC();
    be->device = device_id;
    const char* sync = std::getenv("BAGUA_BACKEND_SYNC");
    be->async = !(sync && *sync && std::atoi(sync) != 0);
    be->cap = schedule_channel_cap ? schedule_channel_cap : 1;
    const char* ln = std::getenv("BAGUA_SCHED_LANES");
    if (ln && *ln) be->lanes = std::max(1, std::min(8, std::atoi(ln)));
    const char* to = std::getenv("BAGUA_COMM_OP_TIMEOUT_S");
    if (to && *to && std::atof(to) > 0)  // at least 1 ms, as bagua_comm_backend_set_op_timeout_ms
        be->op_timeout = std::chrono::milliseconds(std::max(1LL, (long long)(std::atof(to) * 1000)));
    const char* prof = std::getenv("BAGUA_SCHED_PROFILE");
    be->profile = prof && *prof && std::atoi(prof) != 0;
    be->worker = std::thread([be] { be->work(); });
    be->monitor = std::thread([be] { be->watch(); });
    return be;
}

void bagua_comm_backend_destroy(BaguaCommBackendC* be) {
    if (!be) return;
    {
        std::lock_guard<std::mutex> lk(be->mu);
        be->stop = true;
    }
    be->cv_work.notify_all();
    be->cv_space.notify_all();
    // The worker drains what is queued, then exits; the monitor keeps watching until
    // then, so an op stuck during the drain is still failed and aborted.  A worker whose
    // call never returns from an aborted op (abandoned, as wait_pending_comm_ops has it)
    // is left behind: joining it would hang, and it still uses the backend, so the
    // backend is left allocated with it.
    bool left = false;
    {
        std::unique_lock<std::mutex> lk(be->mu);
        while (!be->worker_done) {
            if (be->current && be->abandoned(*be->current)) {
                left = true;
                break;
            }
            be->cv_done.wait_for(lk, std::chrono::milliseconds(100));
        }
        be->stop_monitor = true;
    }
    be->cv_watch.notify_all();
    if (be->monitor.joinable()) be->monitor.join();
    if (left) {
        BAGUA_LOG(0, "comm backend destroyed while its worker is stuck in an aborted op: the worker and the "
                     "backend are left behind");
        if (be->worker.joinable()) be->worker.detach();
        return;
    }
    if (be->worker.joinable()) be->worker.join();
    int n = 0;
    (void)bagua_comm_backend_wait_pending_comm_ops(be, &n);
    for (hipEvent_t e : be->spare) (void)hipEventDestroy(e);
    if (be->profile && be->prof_n)
        fprintf(stderr, "[bagua-core] scheduler: %zu buckets, host us per bucket (p50 / p90 / max of the second "
                        "half): waiting for work %.2f / %.2f / %.2f, execute_bucket %.2f / %.2f / %.2f, completion "
                        "event %.2f / %.2f / %.2f\n", be->prof_n, be->prof_median(0), be->prof_quantile(0, 0.9),
                be->prof_quantile(0, 1.0), be->prof_median(1), be->prof_quantile(1, 0.9), be->prof_quantile(1, 1.0),
                be->prof_median(2), be->prof_quantile(2, 0.9), be->prof_quantile(2, 1.0));
    delete be;
}

int bagua_comm_backend_wait_pending_comm_ops(BaguaCommBackendC* be, int* completed) {
    // lib.rs:321-337: wait for every scheduled op; the first failure is returned
    if (!be) return BAGUA_ERR_INVALID_ARG;
    // first every scheduled bucket enqueued (the worker launches undisturbed: a
    // hipEventSynchronize beside its launches slowed them), then every bucket's work
    // completed (async: its completion event)
    int n = 0, rc = BAGUA_OK;
    std::unique_lock<std::mutex> lk(be->mu);
    while (!be->pending.empty()) {
        std::vector<std::shared_ptr<Scheduled>> items(be->pending.begin(), be->pending.end());
        be->pending.clear();
        for (const auto& item : items)
            while (!item->done && !be->abandoned(*item)) be->cv_done.wait_for(lk, std::chrono::milliseconds(100));
        lk.unlock();
        // one wait per distinct completion event (buckets share them)
        std::vector<std::pair<void*, bool>> synced;
        for (const auto& item : items) {
            void* e = item->finished.get();
            if (!e) continue;
            bool seen = false;
            for (const auto& x : synced) seen = seen || x.first == e;
            if (!seen) synced.emplace_back(e, be->wait_event((hipEvent_t)e, *item));
        }
        lk.lock();
        for (const auto& item : items) {
            if (!item->done) {  // abandoned: its worker never returned from the aborted op
                if (item->status == BAGUA_OK) item->status = BAGUA_ERR_ABORTED;
                be->stuck.push_back(item);  // kept, never reused
            }
            for (const auto& x : synced)
                if (x.first == item->finished.get() && !x.second && item->status == BAGUA_OK)
                    item->status = item->timed_out.load() ? BAGUA_ERR_ABORTED : BAGUA_ERR_HIP;
            item->finished.reset();
            item->waited = true;
            ++n;
            if (rc == BAGUA_OK && item->status != BAGUA_OK) rc = item->status;
        }
    }
    if (completed) *completed = n;
    return rc;
}

int bagua_comm_backend_register_ordered_buckets(BaguaCommBackendC* be, BaguaBucketC* const* buckets, int n) {
    // lib.rs:270-298: calling again replaces the previous buckets
    if (!be || (n > 0 && !buckets)) return BAGUA_ERR_INVALID_ARG;
    int done = 0;
    const int rc = bagua_comm_backend_wait_pending_comm_ops(be, &done);
    if (rc != BAGUA_OK) return rc;
    std::unordered_map<std::string, BaguaBucketC*> mapping;
    std::unordered_set<uint64_t> ptrs;
    for (int i = 0; i < n; ++i) {
        if (!buckets[i]) return BAGUA_ERR_INVALID_ARG;
        for (const BucketTensor& t : buckets[i]->tensors) {
            if (mapping.count(t.name) || ptrs.count(t.t.ptr)) {
                BAGUA_LOG(0, "TensorError: duplicated tensor detected, name %s, ptr %llu", t.name.c_str(),
                          (unsigned long long)t.t.ptr);
                return BAGUA_ERR_INVALID_ARG;
            }
            mapping[t.name] = buckets[i];
            ptrs.insert(t.t.ptr);
        }
    }
    std::lock_guard<std::mutex> lk(be->mu);
    be->mapping.swap(mapping);
    be->ordered.assign(buckets, buckets + n);
    for (int i = 0; i < n; ++i) buckets[i]->sched_index = i;
    return BAGUA_OK;
}

int bagua_comm_backend_mark_communication_ready(BaguaCommBackendC* be, const char* tensor_name, uint64_t ready_event) {
    return bagua_comm_backend_mark_communication_ready_desc(be, tensor_name, ready_event, nullptr);
}

int bagua_comm_backend_mark_communication_ready_desc(BaguaCommBackendC* be, const char* tensor_name,
                                                     uint64_t ready_event, const bagua_tensor_t* current) {
    // lib.rs:300-319
    if (!be || !tensor_name) return BAGUA_ERR_INVALID_ARG;
    std::unique_lock<std::mutex> lk(be->mu);
    if (be->ordered.empty()) return BAGUA_ERR_INVALID_ARG;  // "ordered buckets not yet set in comm backend"
    auto it = be->mapping.find(tensor_name);
    if (it == be->mapping.end()) return BAGUA_ERR_INVALID_ARG;
    int rc = bagua_bucket_mark_tensor_ready_desc(it->second, tensor_name, ready_event, current);
    if (rc != BAGUA_OK) return rc;
    while (be->ordered.front()->ready_for_comm()) {
        BaguaBucketC* b = be->ordered.front();
        be->ordered.pop_front();
        bagua_bucket_reset_comm_ready(b);
        be->ordered.push_back(b);
        // bounded channel (flume::bounded(schedule_channel_cap)): wait for space
        be->cv_space.wait(lk, [&] { return be->stop || be->channel.size() < be->cap; });
        if (be->stop) return BAGUA_ERR_INVALID_ARG;
        auto item = std::make_shared<Scheduled>();
        item->bucket = b;
        item->lane_hint = b->sched_index;
        item->tensors = copy_tensors(b);
        item->events = take_events(b);
        item->ops = copy_ops(b);
        be->channel.push_back(item);
        be->pending.push_back(item);
        be->cv_work.notify_all();
    }
    return BAGUA_OK;
}

int bagua_comm_backend_set_lanes(BaguaCommBackendC* be, int lanes) {
    // waits for everything scheduled, so no bucket changes lane while in flight
    if (!be || lanes < 1 || lanes > 8) return BAGUA_ERR_INVALID_ARG;
    int done = 0;
    const int rc = bagua_comm_backend_wait_pending_comm_ops(be, &done);
    std::lock_guard<std::mutex> lk(be->mu);
    be->lanes = lanes;
    return rc;
}

int bagua_comm_backend_lanes(BaguaCommBackendC* be) {
    if (!be) return -1;
    std::lock_guard<std::mutex> lk(be->mu);
    return be->async ? be->lanes : 1;
}

int bagua_comm_backend_stuck(BaguaCommBackendC* be) {
    if (!be) return -1;
    std::lock_guard<std::mutex> lk(be->mu);
    return (int)be->stuck.size();
}

int bagua_comm_backend_failures(BaguaCommBackendC* be) {
    if (!be) return -1;
    std::lock_guard<std::mutex> lk(be->mu);
    return (int)be->failures.size();
}

int bagua_comm_backend_failure_message(BaguaCommBackendC* be, int i, char* buf, size_t len) {
    if (!be || i < 0) return -1;
    std::lock_guard<std::mutex> lk(be->mu);
    if ((size_t)i >= be->failures.size()) return -1;
    const std::string& m = be->failures[(size_t)i];
    if (buf && len) {
        const size_t n = std::min(len - 1, m.size());
        std::memcpy(buf, m.data(), n);
        buf[n] = 0;
    }
    return (int)m.size();
}

int bagua_comm_backend_set_op_timeout_ms(BaguaCommBackendC* be, int64_t ms) {
    if (!be || ms <= 0) return BAGUA_ERR_INVALID_ARG;
    {
        std::lock_guard<std::mutex> lk(be->mu);
        be->op_timeout = std::chrono::milliseconds(ms);
    }
    be->cv_watch.notify_all();
    return BAGUA_OK;
}

}  // extern "C"
