// comm_ops.cpp — the compressed-gradient comm ops on one flat communication
// tensor, enqueued on the communicator's stream.
//
//   centralized (centralized_low_precision_synchronous.rs:30-71):
//     compress(p, all) -> alltoall -> decompress -> reduce_{mean,sum}(rank)
//     -> compress(p, rank) -> allgather -> decompress
//   here:  compress(p, all) -> ncclAllToAll (out of place)
//          -> [fused] dequantise p versions + reduce + min/max partials
//          -> requantise own chunk -> in-place ncclAllGather -> decompress
//   The fused middle reads the p received segments once (p*cs bytes) instead
//   of decompressing them to fp32 and re-reading that (SURVEY.md §7 "hard
//   parts"); every arithmetic step is unchanged, so the result is bitwise
//   that of the reference sequence.  `_unfused` keeps the reference order.
//
//   decentralized (decentralized_low_precision_synchronous.rs:42-152): ring
//   exchange of whole-bucket (n_chunks = 1) compressed diffs.
//
// All buffers come from the device pool; the op waits for its stream before
// returning them (the reference syncs in BaguaCommunicationTensor::drop,
// datatypes/mod.rs:1062-1066).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "bagua_core.h"
#include "comm_internal.hpp"
#include "runtime_util.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <cstdlib>
#include <vector>

using namespace bagua;

namespace bagua {
thread_local bool g_async_ops = false;
}

namespace {

// BAGUA_OP_PROFILE=1: host us per centralized op, by phase, printed at exit (measurement hook)
struct OpProfile {
    bool on = false;
    std::vector<double> us[5];
    size_t n = 0;
    std::mutex mu;
    OpProfile() {
        const char* e = std::getenv("BAGUA_OP_PROFILE");
        on = e && *e == '1';
    }
    static double median(std::vector<double> v) {
        if (v.empty()) return 0;
        std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
        return v[v.size() / 2];
    }
    ~OpProfile() {
        if (on && n)
            fprintf(stderr, "[bagua-core] centralized op host us, medians (n=%zu): plan+alloc %.2f, compress %.2f, "
                            "middle %.2f, tail %.2f, finish %.2f\n", n, median(us[0]), median(us[1]), median(us[2]),
                    median(us[3]), median(us[4]));
    }
};
OpProfile g_op_prof;
struct OpTimer {
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    double lap() {
        const auto now = std::chrono::steady_clock::now();
        const double d = std::chrono::duration<double, std::micro>(now - t).count();
        t = now;
        return d;
    }
};

struct Chunking {
    int p = 1, rank = 0;
    size_t cs = 0, S = 0;
};

int plan(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int method, Chunking* k) {
    if (!c || !c->t || !t) return BAGUA_ERR_INVALID_ARG;
    if (c->aborted.load()) return BAGUA_ERR_ABORTED;
    k->p = (int)c->nranks;
    k->rank = (int)c->rank;
    if (t->num_elem_allocated % (uint64_t)k->p) return BAGUA_ERR_INVALID_ARG;
    k->cs = t->num_elem_allocated / (uint64_t)k->p;
    k->S = bagua_compressed_size(method, t->dtype, (size_t)k->p, k->cs);
    if (!k->S) return BAGUA_ERR_UNSUPPORTED;
    if (k->S % (size_t)k->p) return BAGUA_ERR_INVALID_ARG;  // communicators/mod.rs:603-607 alltoall alignment
    return BAGUA_OK;
}

bagua_tensor_t u8_view(uint64_t ptr, size_t bytes, int device) {
    bagua_tensor_t v;
    v.ptr = ptr;
    v.num_elem = bytes;
    v.num_elem_allocated = bytes;
    v.dtype = BAGUA_DTYPE_U8;
    v.device_id = device;
    return v;
}

// end of an op: wait for its stream (the reference syncs in
// BaguaCommunicationTensor::drop, datatypes/mod.rs:1062-1066), or, async, return
// with the work enqueued (OpBuffers then go back to the pool behind the stream)
int finish(BaguaSingleCommunicatorC* c, int rc) {
    if (async_ops(c)) return rc;
    const hipError_t e = hipStreamSynchronize(c->stream);
    if (rc) return rc;
    return e == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP;
}

// a pool buffer of one op: freed after the op's stream sync, or (async) behind the
// op's stream, which the side stream has joined by then (finish_both)
class OpBuffer {
   public:
    explicit OpBuffer(BaguaSingleCommunicatorC* c) : c_(c) {}
    OpBuffer(const OpBuffer&) = delete;
    OpBuffer& operator=(const OpBuffer&) = delete;
    ~OpBuffer() { release(); }
    int allocate(int device, size_t bytes) {
        release();
        return pool_alloc(device, bytes, &ptr_);
    }
    void release() {
        if (!ptr_) return;
        if (async_ops(c_)) {
            const uint64_t s = (uint64_t)(uintptr_t)c_->stream;
            (void)pool_free_after(ptr_, &s, 1);
        } else {
            (void)pool_free(ptr_);
        }
        ptr_ = 0;
    }
    uint64_t ptr() const { return ptr_; }
    template <typename P>
    P* as() const { return reinterpret_cast<P*>((uintptr_t)ptr_); }

   private:
    BaguaSingleCommunicatorC* c_;
    uint64_t ptr_ = 0;
};

#define TRY(x)                 \
    do {                       \
        rc = (x);              \
        if (rc) return finish(c, rc); \
    } while (0)

int env_int(const char* name, long dflt);
int check_schedule(BaguaSingleCommunicatorC* c, int op, int method, const bagua_tensor_t* t, uint64_t chunk,
                   int sched, int average);
enum { kOpCentralized = 1, kOpCentralizedUnfused, kOpCentralizedPipelined, kOpOneBitPipelined, kOpRing,
       kOpRingUnfused, kOpRingPipelined };

int centralized(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int average, int method, bool fused) {
    OpTimer tm;
    double ph[5] = {0, 0, 0, 0, 0};
    struct Commit {
        double* ph;
        ~Commit() {
            if (!g_op_prof.on) return;
            std::lock_guard<std::mutex> g(g_op_prof.mu);
            if (g_op_prof.n >= (1u << 20)) return;  // bounded: a measurement hook, not a log
            for (int i = 0; i < 5; ++i) g_op_prof.us[i].push_back(ph[i]);
            ++g_op_prof.n;
        }
    } commit{ph};
    Chunking k;
    int rc = plan(c, t, method, &k);
    if (rc) return rc;
    DeviceGuard guard(c->device_id);
    if ((rc = check_schedule(c, fused ? kOpCentralized : kOpCentralizedUnfused, method, t, k.cs, 1, average)))
        return rc;
    const uint64_t s = (uint64_t)(uintptr_t)c->stream;
    if (k.p == 1 && fused && method == BAGUA_COMPRESSION_MINMAX_UINT8 && t->num_elem == t->num_elem_allocated &&
        k.cs <= 0x7fffffffULL && env_int("BAGUA_ONE_RANK_FUSED", 1) != 0) {
        // one rank: the whole sequence as the min/max pass + one table-driven pass over the
        // tensor (bagua_minmax_u8_centralized_one_rank: the second header follows from the
        // first), no compressed buffer at all; BAGUA_ONE_RANK_FUSED=0: the steps below (A/B)
        const size_t ws_bytes = bagua_minmax_u8_workspace_bytes((int)k.cs, 1);
        uint64_t ws = 0;
        if ((rc = stream_workspace(c->device_id, s, ws_bytes, &ws)) != BAGUA_OK) return finish(c, rc);
        ph[0] = tm.lap();
        rc = bagua_minmax_u8_centralized_one_rank(t->dtype, (void*)(uintptr_t)t->ptr, (int)k.cs, average,
                                                  (void*)(uintptr_t)ws, ws_bytes, (void*)(uintptr_t)s);
        ph[2] = tm.lap();
        return finish(c, rc);
    }
    if (k.p == 1 && fused && method == BAGUA_COMPRESSION_ONEBIT && t->num_elem == t->num_elem_allocated &&
        k.cs <= 0x7fffffffULL && env_int("BAGUA_ONE_RANK_FUSED", 1) != 0) {
        // the same for the 1-bit codec: encode pass, one workgroup for both scales, one
        // pass writing +-scale2 from the bits (bagua_onebit_centralized_one_rank)
        const size_t ws_bytes = bagua_onebit_one_rank_workspace_bytes((int)k.cs);
        uint64_t ws = 0;
        if ((rc = stream_workspace(c->device_id, s, ws_bytes, &ws)) != BAGUA_OK) return finish(c, rc);
        ph[0] = tm.lap();
        rc = bagua_onebit_centralized_one_rank(t->dtype, (void*)(uintptr_t)t->ptr, (int)k.cs, average,
                                               (void*)(uintptr_t)ws, ws_bytes, (void*)(uintptr_t)s);
        ph[2] = tm.lap();
        return finish(c, rc);
    }
    // 2. (below) alltoall: slot j of recv <- rank j's segment `rank`.  One rank receives
    // its own bytes: the MinMax steps below read them from `send` itself (their reads and
    // the requantise's writes are separate kernels in stream order; no recv buffer), the
    // 1-bit middle step -- one kernel that reads every segment's header while rewriting
    // its own -- from a device copy (RCCL's single-rank copy kernel was slower: 1 GiB op
    // 1.257 -> 1.222 ms)
    const bool self_alias = k.p == 1 && method == BAGUA_COMPRESSION_MINMAX_UINT8;
    OpBuffer send(c), recv(c);
    TRY(send.allocate(c->device_id, k.S));
    if (!self_alias) TRY(recv.allocate(c->device_id, k.S));
    const bagua_tensor_t sv = u8_view(send.ptr(), k.S, c->device_id);
    const bagua_tensor_t rv = u8_view(recv.ptr(), k.S, c->device_id);
    ph[0] = tm.lap();
    // 1. compress every chunk (target -1)
    TRY(bagua_tensor_compress_into(t, method, k.p, s, -1, &sv));
    ph[1] = tm.lap();
    if (k.p == 1 && !self_alias)
        TRY(hipMemcpyAsync(recv.as<void>(), send.as<void>(), k.S, hipMemcpyDeviceToDevice, c->stream) == hipSuccess
                ? BAGUA_OK
                : BAGUA_ERR_HIP);
    else if (k.p > 1)
        TRY(c->t->alltoall(send.as<void>(), recv.as<void>(), k.S / k.p, BAGUA_DTYPE_U8, c->stream));
    uint8_t* const rbuf = self_alias ? send.as<uint8_t>() : recv.as<uint8_t>();
    const bagua_tensor_t* const rview = self_alias ? &sv : &rv;
    // 3. reduce the p received versions of the own chunk and requantise it into send[rank]
    bool done = false;
    // the fused kernels treat every allocated element as valid (the reference
    // compresses num_elements(), datatypes/mod.rs:339): other tensors run unfused
    if (fused && method == BAGUA_COMPRESSION_MINMAX_UINT8 && t->num_elem == t->num_elem_allocated) {
        const size_t ws_bytes = bagua_minmax_u8_workspace_bytes((int)k.cs, k.p);
        uint64_t ws = 0;
        if ((rc = stream_workspace(c->device_id, s, ws_bytes, &ws)) != BAGUA_OK) return finish(c, rc);
        // the reduced chunk is dead (step 5's decompress rewrites every element): below
        // p = 2*sizeof(T) recomputing it from the p received segments moves fewer bytes
        // than storing it and reading it back (p*cs vs 2*cs*sizeof(T); p = 1: 10 -> 3 bytes
        // per element); BAGUA_REDUCE_RECOMPUTE=0/1 forces either way (A/B)
        const int rcm = env_int("BAGUA_REDUCE_RECOMPUTE", -1);
        const bool recompute = rcm >= 0 ? rcm != 0 : (size_t)k.p < 2 * bagua_dtype_bytes(t->dtype);
        if (recompute && k.p == 1) {
            // one rank: the own chunk is the whole tensor and nothing is gathered, so the
            // requantise writes the final decompressed values (no step-5 launch) and not the
            // requantised segment, which nothing would read
            rc = bagua_minmax_u8_reduce_requantize_final(t->dtype, rbuf, k.S, (int)k.cs, k.p, (void*)(uintptr_t)t->ptr,
                                                         average, nullptr, 0, k.rank,
                                                         (void*)(uintptr_t)ws, ws_bytes, (void*)(uintptr_t)s);
            ph[2] = tm.lap();
            if (rc == BAGUA_OK) {
                const int r = finish(c, BAGUA_OK);
                ph[4] = tm.lap();
                return r;
            }
        } else {
            rc = bagua_minmax_u8_reduce_requantize(t->dtype, rbuf, k.S, (int)k.cs, k.p,
                                                   recompute ? nullptr : (void*)(uintptr_t)t->ptr, average,
                                                   send.as<uint8_t>(), k.S, k.rank, (void*)(uintptr_t)ws, ws_bytes,
                                                   (void*)(uintptr_t)s);
        }
        if (rc == BAGUA_OK) done = true;
        else if (rc != BAGUA_ERR_UNSUPPORTED) return finish(c, rc);
    } else if (fused && method == BAGUA_COMPRESSION_ONEBIT && t->num_elem == t->num_elem_allocated) {
        const size_t ws_bytes = bagua_onebit_workspace_bytes((int)k.cs, 1);
        uint64_t ws = 0;
        if ((rc = stream_workspace(c->device_id, s, ws_bytes, &ws)) != BAGUA_OK) return finish(c, rc);
        // the reduced chunk is not stored: step 5's decompress rewrites every element
        rc = bagua_onebit_reduce_requantize(t->dtype, recv.as<uint8_t>(), k.S, (int)k.cs, k.p,
                                            nullptr, average, send.as<uint8_t>(), k.S, k.rank,
                                            (void*)(uintptr_t)ws, ws_bytes, (void*)(uintptr_t)s);
        if (rc == BAGUA_OK) done = true;
        else if (rc != BAGUA_ERR_UNSUPPORTED) return finish(c, rc);
    }
    if (!done) {
        TRY(bagua_tensor_decompress_from(t, method, k.p, rview, s));
        TRY(bagua_tensor_reduce_inplace(t, k.p, k.rank, average, s));
        TRY(bagua_tensor_compress_into(t, method, k.p, s, k.rank, &sv));
    }
    // 4. allgather the requantised chunks in place (one rank: nothing to move), 5. decompress everything
    if (k.p > 1) TRY(bagua_comm_allgather_inplace(c, &sv));
    TRY(bagua_tensor_decompress_from(t, method, k.p, &sv, s));
    return finish(c, BAGUA_OK);
}

// ---- pipelined centralized op ---------------------------------------------
// The same op as above with each chunk cut into `pieces` element ranges and
// two streams: the codec runs on the communicator's stream, the exchange of
// piece k on a side stream while the codec works on piece k+1:
//
//   stream: partials | Q0 Q1 .. Qk | R0 R1 .. Rk RQ | D0 D1 .. Dk
//   side  :             A0 A1 .. Ak            G0 G1 .. Gk
//   (Q quantise, A alltoall as grouped send/recv, R fused dequantise+reduce,
//    RQ requantise own chunk, G allgather, D dequantise; each arrow an event)
//
// A segment keeps one header per chunk and the pieces are disjoint byte ranges
// of it, so every buffer holds exactly the bytes of the unpieced op and the
// result is bit-identical to it (and to the reference sequence).
int env_int(const char* name, long dflt) {
    const char* v = std::getenv(name);
    return v && *v ? (int)std::strtol(v, nullptr, 10) : (int)dflt;
}

int auto_pieces(const BaguaSingleCommunicatorC* c, size_t payload_bytes) {
    // BAGUA_PIPELINE_PIECES caps the count (1 disables), pieces keep at least
    // BAGUA_PIPELINE_MIN_PIECE payload bytes per chunk (= elements for MinMax
    // u8; the exchange of a piece is p times that); both read once, at the
    // communicator's creation (ScheduleConfig)
    const int kmax = c->cfg.pieces_cap;
    const int min_piece = c->cfg.min_piece;
    size_t k = payload_bytes / (size_t)(min_piece > 0 ? min_piece : 1);
    if (k > (size_t)kmax) k = (size_t)kmax;
    return k < 1 ? 1 : (int)k;
}

// The op's piece schedule (bagua_kernels.h: a count, optionally OR-ed with
// BAGUA_PIECES_TAPERED): the caller's, tapered from 3 pieces when the communicator's
// ScheduleConfig (equal on every rank) says so -- by default the schedules the op
// chose itself (the caller passed 0 pieces), since round 6: at the same count the
// first piece (quantised before any byte is on the wire) and the last one (reduced and
// dequantised after the wire) are half size, so the unhidden codec shrinks with the same
// number of exchange groups (1 GiB fp32, 4 pieces, one GPU's kernels: prefix 208 -> 183,
// suffix 56 -> 38 us, profiles/r06_pipe_probe_t4.json).  BAGUA_PIPELINE_TAPER=0 keeps
// every automatic schedule uniform, =1 tapers explicit counts too.  Fixed once per op
// and passed to every building block, so all of one op's ranges agree.
int op_schedule(const BaguaSingleCommunicatorC* c, int count, int caller) {
    int sched = count | (caller & BAGUA_PIECES_TAPERED);
    const bool automatic = (caller & BAGUA_PIECES_COUNT_MASK) == 0;
    const bool taper = c->cfg.taper > 0 || (c->cfg.taper < 0 && automatic);
    if (count >= 3 && !(sched & BAGUA_PIECES_TAPERED) && taper) sched |= BAGUA_PIECES_TAPERED;
    return sched;
}

// ---- BAGUA_CHECK_SCHEDULE: ranks compare what they are about to post ---------
// Opt-in (ScheduleConfig::check, equal on every rank): before an op's first
// collective the ranks allgather a small descriptor of the op -- which op, codec,
// dtype, p, chunk size, tensor sizes, piece schedule, average, op number -- on the
// op's own communicator and stream, and every rank returns BAGUA_ERR_INVALID_ARG
// when any two differ, before any of them posts a collective the others do not
// match (which over RCCL hangs; centralized_low_precision_synchronous.rs:30-71 is
// the sequence every rank must post alike).  Costs one small allgather and a host
// round trip per op.
//
// The op number assumes ONE issuing thread per communicator (its lane views count on
// the parent): ops issued concurrently from several threads could number differently
// on different ranks and report a false mismatch.  A stream being captured into a HIP
// graph cannot be synchronised, so the check is refused there (BAGUA_ERR_UNSUPPORTED)
// rather than breaking the capture.
constexpr int kDescFields = 10;
const char* const kDescName[kDescFields] = {"op",       "method",         "dtype",   "nranks",  "chunk elements",
                                            "num_elem", "num_elem_alloc", "schedule", "average", "op number"};

int check_schedule(BaguaSingleCommunicatorC* c, int op, int method, const bagua_tensor_t* t, uint64_t chunk,
                   int sched, int average) {
    if (!c->cfg.check || c->nranks <= 1) return BAGUA_OK;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(c->stream, &cap) != hipSuccess) return BAGUA_ERR_HIP;
    if (cap != hipStreamCaptureStatusNone) {
        BAGUA_LOG(0, "BAGUA_CHECK_SCHEDULE: the op's stream is being captured; the check needs a host round trip");
        return BAGUA_ERR_UNSUPPORTED;
    }
    BaguaSingleCommunicatorC* root = c->parent ? c->parent : c;
    const int64_t mine[kDescFields] = {op, method, t->dtype, (int64_t)c->nranks, (int64_t)chunk, (int64_t)t->num_elem,
                                       (int64_t)t->num_elem_allocated, sched, average != 0,
                                       (int64_t)root->op_seq.fetch_add(1)};
    const size_t one = sizeof(mine), p = c->nranks;
    PoolBuffer buf;
    int rc = buf.allocate(c->device_id, one * p);
    if (rc) return rc;
    std::vector<int64_t> all(kDescFields * p);
    uint8_t* base = buf.as<uint8_t>();
    if (hipMemcpyAsync(base + c->rank * one, mine, one, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return BAGUA_ERR_HIP;
    if ((rc = c->t->allgather(base + c->rank * one, base, one, BAGUA_DTYPE_U8, c->stream)) != BAGUA_OK) return rc;
    if (hipMemcpyAsync(all.data(), base, one * p, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return BAGUA_ERR_HIP;
    for (size_t j = 0; j < p; ++j)
        for (int f = 0; f < kDescFields; ++f)
            if (all[j * kDescFields + f] != mine[f]) {
                BAGUA_LOG(0, "rank %zu: op schedule mismatch with rank %zu: %s %lld here, %lld there", c->rank, j,
                          kDescName[f], (long long)mine[f], (long long)all[j * kDescFields + f]);
                return BAGUA_ERR_INVALID_ARG;
            }
    return BAGUA_OK;
}

bool valid_schedule(int pieces) {
    return (pieces & ~(BAGUA_PIECES_COUNT_MASK | BAGUA_PIECES_TAPERED | BAGUA_PIECES_MULTIPATH)) == 0;
}

// Whether the op runs pipelined: every rank must decide alike (they would otherwise
// post different collectives), so only values equal on every rank enter -- sizes,
// dtype, p -- never this rank's pointer.  A rank whose tensor is not 16-B aligned
// runs the same schedule on an aligned staging copy (with_aligned_copy).
bool pipeline_fits(const BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, const Chunking& k) {
    const size_t esz = bagua_dtype_bytes(t->dtype);
    const size_t vec = t->dtype == BAGUA_DTYPE_F32 ? 4 : 8;  // payload bytes per 16-B vector
    return k.p <= 16 && t->num_elem == t->num_elem_allocated && (k.S / k.p) % vec == 0 && (k.cs * esz) % 16 == 0 &&
           c->t != nullptr;
}

// Runs op(descriptors) on 16-B aligned copies of the tensors that are not aligned:
// copied into one pool block on the op's stream first and back after the op (whose
// work, side stream included, the stream has joined by then).  The aligned tensors
// are passed as they are.
template <typename F>
int with_aligned_copy(BaguaSingleCommunicatorC* c, std::vector<const bagua_tensor_t*> ts, F&& op) {
    size_t total = 0;
    std::vector<size_t> off(ts.size(), 0);
    for (size_t i = 0; i < ts.size(); ++i)
        if (ts[i]->ptr % 16) {
            off[i] = total;
            total += (ts[i]->num_elem_allocated * bagua_dtype_bytes(ts[i]->dtype) + 255) / 256 * 256;
        }
    if (!total) return op(ts);
    OpBuffer stage(c);
    int rc = stage.allocate(c->device_id, total);
    if (rc) return finish(c, rc);
    std::vector<bagua_tensor_t> copies(ts.size());
    std::vector<const bagua_tensor_t*> use(ts.size());
    for (size_t i = 0; i < ts.size(); ++i) {
        use[i] = ts[i];
        if (!(ts[i]->ptr % 16)) continue;
        copies[i] = *ts[i];
        copies[i].ptr = stage.ptr() + off[i];
        use[i] = &copies[i];
        if (hipMemcpyAsync((void*)(uintptr_t)copies[i].ptr, (const void*)(uintptr_t)ts[i]->ptr,
                           ts[i]->num_elem_allocated * bagua_dtype_bytes(ts[i]->dtype), hipMemcpyDeviceToDevice,
                           c->stream) != hipSuccess)
            return finish(c, BAGUA_ERR_HIP);
    }
    rc = op(use);
    if (rc) return rc;  // the op finished (or enqueued) its own failure handling
    for (size_t i = 0; i < ts.size(); ++i)
        if (ts[i]->ptr % 16 &&
            hipMemcpyAsync((void*)(uintptr_t)ts[i]->ptr, (const void*)(uintptr_t)use[i]->ptr,
                           ts[i]->num_elem_allocated * bagua_dtype_bytes(ts[i]->dtype), hipMemcpyDeviceToDevice,
                           c->stream) != hipSuccess)
            return finish(c, BAGUA_ERR_HIP);
    return finish(c, BAGUA_OK);
}

// bytes [lo, hi) of every segment that piece q of schedule `sched` covers: the header
// travels with piece 0, the slack with the last non-empty piece; empty pieces move nothing
void piece_bytes(const Chunking& k, int sched, int q, size_t* lo, size_t* hi) {
    int b = 0, e = 0;
    bagua_minmax_u8_piece_range((int)k.cs, sched, q, &b, &e);
    const size_t co = k.S / k.p;
    if (q > 0 && b == e) {
        *lo = *hi = 0;
        return;
    }
    *lo = q == 0 ? 0 : 32 + (size_t)b;
    *hi = (size_t)e == k.cs ? co : 32 + (size_t)e;
}

// 1-bit segment bytes of tile range [tb, te): header with piece 0 when `header`, the rest
// of the segment (slack) with the last tile
void onebit_piece_bytes(const Chunking& k, int tb, int te, bool header, size_t* lo, size_t* hi) {
    const size_t co = k.S / k.p;
    const int tiles = (int)((k.cs + 1023) / 1024);
    *lo = header ? 0 : 32 + (size_t)tb * 128;
    *hi = te >= tiles ? co : 32 + (size_t)te * 128;
    if (!header && tb >= te) *lo = *hi = 0;
}

// one piece of the alltoall (send -> recv) or of the in-place allgather (send)
int exchange_piece(BaguaSingleCommunicatorC* c, const Chunking& k, uint8_t* send, uint8_t* recv, size_t lo,
                   size_t hi, bool alltoall) {
    if (hi <= lo) return BAGUA_OK;
    const size_t co = k.S / k.p, len = hi - lo;
    hipStream_t s1 = c->side;
    if (alltoall &&
        hipMemcpyAsync(recv + k.rank * co + lo, send + k.rank * co + lo, len, hipMemcpyDeviceToDevice, s1) != hipSuccess)
        return BAGUA_ERR_HIP;
    if (k.p == 1) return BAGUA_OK;
    int rc = c->t->group_start();
    for (int j = 0; j < k.p && !rc; ++j) {
        if (j == k.rank) continue;
        if (alltoall) {
            rc = c->t->send(send + j * co + lo, len, BAGUA_DTYPE_U8, j, s1);
            if (!rc) rc = c->t->recv(recv + j * co + lo, len, BAGUA_DTYPE_U8, j, s1);
        } else {
            rc = c->t->send(send + k.rank * co + lo, len, BAGUA_DTYPE_U8, j, s1);
            if (!rc) rc = c->t->recv(send + j * co + lo, len, BAGUA_DTYPE_U8, j, s1);
        }
    }
    const int rc_end = c->t->group_end();
    return rc ? rc : rc_end;
}

int finish_both(BaguaSingleCommunicatorC* c, int rc) {
    if (async_ops(c)) {
        // the op's stream takes over the side stream's tail: its completion is the op's
        if (hipEventRecord(c->join, c->side) != hipSuccess || hipStreamWaitEvent(c->stream, c->join, 0) != hipSuccess)
            return rc ? rc : BAGUA_ERR_HIP;
        return rc;
    }
    const hipError_t e1 = hipStreamSynchronize(c->side);
    const int r0 = finish(c, rc);
    if (r0) return r0;
    return e1 == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP;
}

#define TRY2(x)                          \
    do {                                 \
        rc = (x);                        \
        if (rc) return finish_both(c, rc); \
    } while (0)
#define HIP2(x) TRY2((x) == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP)

int centralized_pipelined(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int average, int pieces) {
    Chunking k;
    if (!valid_schedule(pieces)) return BAGUA_ERR_INVALID_ARG;
    int rc = plan(c, t, BAGUA_COMPRESSION_MINMAX_UINT8, &k);
    if (rc) return rc;
    const int caller = pieces;
    pieces &= BAGUA_PIECES_COUNT_MASK;
    if (pieces < 1) pieces = k.p == 1 ? 1 : auto_pieces(c, k.cs);  // one rank: no exchange to hide
    if (pieces == 1 || !pipeline_fits(c, t, k)) return centralized(c, t, average, BAGUA_COMPRESSION_MINMAX_UINT8, true);
    if (t->ptr % 16)
        return with_aligned_copy(c, {t}, [&](const std::vector<const bagua_tensor_t*>& u) {
            return centralized_pipelined(c, u[0], average, pieces | (caller & BAGUA_PIECES_TAPERED));
        });
    const int sched = op_schedule(c, pieces, caller);
    DeviceGuard guard(c->device_id);
    if ((rc = check_schedule(c, kOpCentralizedPipelined, BAGUA_COMPRESSION_MINMAX_UINT8, t, k.cs, sched, average)))
        return rc;
    if (c->ensure_side(4 * (size_t)pieces + 1)) return BAGUA_ERR_HIP;
    hipStream_t s0 = c->stream, s1 = c->side;
    hipEvent_t* quantised = c->events.data();
    hipEvent_t* exchanged = quantised + pieces;
    hipEvent_t* gathered = exchanged + pieces;
    hipEvent_t* requantised_piece = gathered + pieces;
    hipEvent_t requantised = requantised_piece[pieces];
    const int dt = t->dtype, cs = (int)k.cs, p = k.p;
    void* x = (void*)(uintptr_t)t->ptr;
    OpBuffer send(c), recv(c);
    TRY(send.allocate(c->device_id, k.S));
    TRY(recv.allocate(c->device_id, k.S));
    uint8_t* sb = send.as<uint8_t>();
    uint8_t* rb = recv.as<uint8_t>();
    size_t ws_bytes = bagua_minmax_u8_workspace_bytes(cs, p);
    const size_t pws = bagua_minmax_u8_pipeline_workspace_bytes(cs, sched);
    if (pws > ws_bytes) ws_bytes = pws;
    uint64_t wsp = 0;
    if ((rc = stream_workspace(c->device_id, (uint64_t)(uintptr_t)s0, ws_bytes, &wsp)) != BAGUA_OK)
        return finish(c, rc);
    void* ws = (void*)(uintptr_t)wsp;
    // the side stream starts after everything already queued on the op's stream
    HIP2(hipEventRecord(requantised, s0));
    HIP2(hipStreamWaitEvent(s1, requantised, 0));
    // 1. min/max of every chunk, then quantise + exchange piece by piece
    // (backwards: the chunks' first pieces, quantised next, stay in the Infinity Cache)
    TRY2(bagua_minmax_u8_compress_stage(env_int("BAGUA_PARTIALS_FORWARD", 0) ? 1 : 5, dt, x, (int)t->num_elem, cs, p,
                                        sb, k.S, ws, ws_bytes, -1, s0));
    for (int q = 0; q < pieces; ++q) {
        int b, e;
        bagua_minmax_u8_piece_range(cs, sched, q, &b, &e);
        if (q == 0 || b < e)
            TRY2(bagua_minmax_u8_quantize_range(dt, x, (int)t->num_elem, cs, p, sb, k.S, ws, ws_bytes, -1, b, e, s0));
        HIP2(hipEventRecord(quantised[q], s0));
    }
    for (int q = 0; q < pieces; ++q) {
        size_t lo, hi;
        piece_bytes(k, sched, q, &lo, &hi);
        HIP2(hipStreamWaitEvent(s1, quantised[q], 0));
        TRY2(exchange_piece(c, k, sb, rb, lo, hi, true));
        HIP2(hipEventRecord(exchanged[q], s1));
    }
    // 2. reduce the p received versions of the own chunk piece by piece, requantise it.
    // The reduced chunk need not be stored (the final dequantise rewrites the own chunk
    // of x): with `recompute` each reduce piece emits its min/max partials only and the
    // requantise recomputes the piece from the received segments, (2p + 1) L bytes per
    // piece of L elements instead of (p + 2 sizeof(T) + 1) L, at twice the table
    // lookups.  Measured on 1 GiB fp32 (tools/pipeline_kernels_probe.py,
    // profiles/r06_pipe_probe_p{4,8}.json) it pays at p = 2 only -- the middle step 71.0
    // -> 58.0 us with 4 pieces, 42.6 -> 35.4 with 8 -- and loses from p = 4 on (the
    // lookups, not the bytes, bound these kernels), so it runs where 2p <= sizeof(T).
    // BAGUA_PIPE_RECOMPUTE=0 / 1 forces either (A/B).
    const int rc_env = env_int("BAGUA_PIPE_RECOMPUTE", -1);
    const bool recompute = rc_env >= 0 ? rc_env != 0 : 2 * (size_t)p <= bagua_dtype_bytes(dt);
    // every piece dequantises the same p segment headers: reduce piece 0 leaves its tables
    // in the workspace and the later pieces (and the recompute requantise) copy them
    // (BAGUA_PIECES_TABLES; BAGUA_PIPE_TABLES=0: every launch builds its own, A/B)
    const int tsched = sched | (env_int("BAGUA_PIPE_TABLES", 1) != 0 ? BAGUA_PIECES_TABLES : 0);
    for (int q = 0; q < pieces; ++q) {
        HIP2(hipStreamWaitEvent(s0, exchanged[q], 0));
        TRY2(bagua_minmax_u8_reduce_piece(dt, rb, k.S, cs, p, recompute ? nullptr : x, average, k.rank, tsched, q, ws,
                                          ws_bytes, s0));
    }
    // requantise piece by piece, so the allgather of piece q starts while piece q+1 is
    // requantised.  Every requantise needs the whole chunk's min/max, and each of its
    // workgroups folds all pieces' partials itself.  BAGUA_PIPE_PREFOLD=1 folds them once
    // in one workgroup first (BAGUA_PIECES_FOLDED): measured no faster -- the middle step
    // 58.7 vs 58.9 us at p = 2, 43.4 vs 44.3 at p = 8 (profiles/r06_pipe_probe_p4_prefold.json)
    // -- the fold is not what bounds the requantise, so it is off (A/B switch)
    const bool prefold = env_int("BAGUA_PIPE_PREFOLD", 0) != 0;
    if (prefold) TRY2(bagua_minmax_u8_fold_piece_partials(dt, cs, sched, ws, ws_bytes, s0));
    const int rq_sched = tsched | (prefold ? BAGUA_PIECES_FOLDED : 0);
    for (int q = 0; q < pieces; ++q) {
        if (recompute)
            TRY2(bagua_minmax_u8_reduce_requantize_piece(dt, rb, k.S, cs, p, average, sb, k.S, k.rank, rq_sched, q, ws,
                                                         ws_bytes, s0));
        else
            TRY2(bagua_minmax_u8_requantize_piece(dt, x, cs, p, sb, k.S, k.rank, rq_sched, q, ws, ws_bytes, s0));
        HIP2(hipEventRecord(requantised_piece[q], s0));
    }
    // 3. allgather + dequantise piece by piece
    for (int q = 0; q < pieces; ++q) {
        size_t lo, hi;
        piece_bytes(k, sched, q, &lo, &hi);
        HIP2(hipStreamWaitEvent(s1, requantised_piece[q], 0));
        TRY2(exchange_piece(c, k, sb, rb, lo, hi, false));
        HIP2(hipEventRecord(gathered[q], s1));
    }
    for (int q = 0; q < pieces; ++q) {
        int b, e;
        bagua_minmax_u8_piece_range(cs, sched, q, &b, &e);
        HIP2(hipStreamWaitEvent(s0, gathered[q], 0));
        if (b < e) TRY2(bagua_minmax_u8_decompress_range(dt, sb, k.S, cs, p, x, b, e, s0));
    }
    return finish_both(c, BAGUA_OK);
}

// The 1-bit op, pipelined the same way.  A 1-bit header (scale) needs the whole
// chunk's |x| partials, so the alltoall sends the sign bits of piece q as soon
// as they are encoded and the headers with the last piece; the fused middle
// step (which needs every received scale) runs once, after the last piece.
// The allgather sends the headers with piece 0 and the decode of piece q
// follows its arrival.
//
//   stream: E0 E1 .. Ek F | R+F | D0 D1 .. Dk
//   side  :    A0 A1 .. Ak+hdr   G0+hdr G1 .. Gk
int centralized_pipelined_onebit(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int average, int pieces) {
    Chunking k;
    if (!valid_schedule(pieces)) return BAGUA_ERR_INVALID_ARG;
    int rc = plan(c, t, BAGUA_COMPRESSION_ONEBIT, &k);
    if (rc) return rc;
    pieces &= BAGUA_PIECES_COUNT_MASK;  // 1-bit pieces are tile ranges: no tapered schedule
    if (pieces < 1) pieces = k.p == 1 ? 1 : auto_pieces(c, k.cs / 8);  // sign bits per chunk
    if (pieces == 1 || k.p > 16 || t->num_elem != t->num_elem_allocated || k.cs > 0x7fffffffULL)
        return centralized(c, t, average, BAGUA_COMPRESSION_ONEBIT, true);
    DeviceGuard guard(c->device_id);
    if ((rc = check_schedule(c, kOpOneBitPipelined, BAGUA_COMPRESSION_ONEBIT, t, k.cs, pieces, average))) return rc;
    if (c->ensure_side(2 * (size_t)pieces + 2)) return BAGUA_ERR_HIP;
    hipStream_t s0 = c->stream, s1 = c->side;
    hipEvent_t* encoded = c->events.data();
    hipEvent_t* gathered = encoded + pieces;
    hipEvent_t exchanged = gathered[pieces], requantised = gathered[pieces + 1];
    const int dt = t->dtype, cs = (int)k.cs, p = k.p;
    void* x = (void*)(uintptr_t)t->ptr;
    OpBuffer send(c), recv(c);
    TRY(send.allocate(c->device_id, k.S));
    TRY(recv.allocate(c->device_id, k.S));
    uint8_t* sb = send.as<uint8_t>();
    uint8_t* rb = recv.as<uint8_t>();
    const size_t ws_bytes = bagua_onebit_workspace_bytes(cs, p);
    uint64_t wsp = 0;
    if ((rc = stream_workspace(c->device_id, (uint64_t)(uintptr_t)s0, ws_bytes, &wsp)) != BAGUA_OK)
        return finish(c, rc);
    void* ws = (void*)(uintptr_t)wsp;
    HIP2(hipEventRecord(requantised, s0));
    HIP2(hipStreamWaitEvent(s1, requantised, 0));
    // 1. encode piece by piece (bits + partials of every chunk), headers last
    for (int q = 0; q < pieces; ++q) {
        int tb, te;
        bagua_onebit_piece_range(cs, pieces, q, &tb, &te);
        if (te > tb) TRY2(bagua_onebit_encode_range(dt, x, (int)t->num_elem, cs, p, sb, k.S, ws, ws_bytes, tb, te, s0));
        if (q == pieces - 1) TRY2(bagua_onebit_finalize(ws, ws_bytes, (int)t->num_elem, cs, p, sb, k.S, s0));
        HIP2(hipEventRecord(encoded[q], s0));
    }
    for (int q = 0; q < pieces; ++q) {
        int tb, te;
        bagua_onebit_piece_range(cs, pieces, q, &tb, &te);
        size_t lo, hi;
        onebit_piece_bytes(k, tb, te, false, &lo, &hi);
        HIP2(hipStreamWaitEvent(s1, encoded[q], 0));
        TRY2(exchange_piece(c, k, sb, rb, lo, hi, true));
        if (q == pieces - 1) TRY2(exchange_piece(c, k, sb, rb, 0, 32, true));  // the headers
    }
    HIP2(hipEventRecord(exchanged, s1));
    // 2. decode the p received segments of the own chunk, reduce, re-encode it (not stored)
    HIP2(hipStreamWaitEvent(s0, exchanged, 0));
    TRY2(bagua_onebit_reduce_requantize(dt, rb, k.S, cs, p, nullptr, average, sb, k.S, k.rank, ws, ws_bytes, s0));
    HIP2(hipEventRecord(requantised, s0));
    // 3. allgather (headers with piece 0) + decode piece by piece
    HIP2(hipStreamWaitEvent(s1, requantised, 0));
    for (int q = 0; q < pieces; ++q) {
        int tb, te;
        bagua_onebit_piece_range(cs, pieces, q, &tb, &te);
        size_t lo, hi;
        onebit_piece_bytes(k, tb, te, q == 0, &lo, &hi);
        TRY2(exchange_piece(c, k, sb, rb, lo, hi, false));
        HIP2(hipEventRecord(gathered[q], s1));
    }
    for (int q = 0; q < pieces; ++q) {
        int tb, te;
        bagua_onebit_piece_range(cs, pieces, q, &tb, &te);
        HIP2(hipStreamWaitEvent(s0, gathered[q], 0));
        if (te > tb) TRY2(bagua_onebit_decompress_range(dt, sb, k.S, cs, p, x, tb, te, s0));
    }
    return finish_both(c, BAGUA_OK);
}

// ---- ring exchange schedule ------------------------------------------------
// The reference sends the whole compressed bucket straight to both ring peers
// (decentralized_low_precision_synchronous.rs:98-115).  On a fully connected
// xGMI node that loads 2 of each GPU's 7 links and leaves 5 idle.  From 6
// ranks on, each piece's bytes are cut into p slices: slices 0..2 go straight
// to the peer, slice k >= 3 is sent to relay rank r + (k-1) (for the right
// peer; r - (k-1) for the left one), which forwards it in the next group.
// Per directed link offset o the load is then (a = 3/p direct, b = 1/p per
// relay): o = +-1: a + b; o = +-2: 3b; others 4b, i.e. at most 4/p of the
// payload per link (8 ranks: 1/2) instead of all of it.  The schedule is
// deterministic and symmetric, and every transfer carries a key (hop, flow,
// slice) so that both ends post the transfers between two ranks in the same
// order (NCCL matches grouped p2p in posting order per pair).
constexpr int kRingMinMultipath = 6;

struct RingPlan {
    int p = 1, r = 0, pieces = 1, groups = 1;
    int sched = 1;  // piece schedule (count + BAGUA_PIECES_TAPERED)
    bool mp = false;
    Chunking k;
    size_t slot = 0;  // relay scratch bytes per slice
};

enum { kBufMine = 0, kBufLeft = 1, kBufRight = 2, kBufRelay = 3 };

// p + 1 slice boundaries of bytes [lo, hi), inner ones on 64-B lines
void ring_slices(size_t lo, size_t hi, int p, size_t* b) {
    const size_t len = hi - lo;
    b[0] = lo;
    b[p] = hi;
    for (int i = 1; i < p; ++i) {
        size_t x = (lo + len * (size_t)i / (size_t)p) & ~(size_t)63;
        if (x < b[i - 1]) x = b[i - 1];
        b[i] = x < hi ? x : hi;
    }
}

int ring_plan(int nranks, int rank, int chunk_size, int pieces, bool multipath, RingPlan* P) {
    if (nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks || chunk_size < 0 || !valid_schedule(pieces) ||
        (pieces & BAGUA_PIECES_COUNT_MASK) < 1)
        return BAGUA_ERR_INVALID_ARG;
    P->p = nranks;
    P->r = rank;
    P->sched = pieces;
    pieces &= BAGUA_PIECES_COUNT_MASK;
    P->pieces = pieces;
    P->mp = multipath && nranks >= kRingMinMultipath;
    P->groups = pieces + (P->mp ? 1 : 0);
    P->k.p = 1;
    P->k.cs = (size_t)chunk_size;
    P->k.S = bagua_minmax_u8_compressed_bytes(BAGUA_DTYPE_F32, chunk_size, 1);  // align32(n) + 32 for every dtype
    P->slot = 0;
    if (P->mp) {
        size_t b[65];
        for (int q = 0; q < pieces; ++q) {
            size_t lo, hi;
            piece_bytes(P->k, P->sched, q, &lo, &hi);
            if (hi <= lo) continue;
            ring_slices(lo, hi, nranks, b);
            for (int i = 3; i < nranks; ++i)
                if (b[i + 1] - b[i] > P->slot) P->slot = b[i + 1] - b[i];
        }
        P->slot = (P->slot + 63) & ~(size_t)63;
    }
    return BAGUA_OK;
}

size_t ring_relay_bytes(const RingPlan& P) { return P.mp ? 4 * (size_t)(P.p - 3) * P.slot : 0; }

// transfers of group g: the direct slices and first hops of piece g (g < pieces),
// the relays' second hops of piece g - 1 (multipath, g > 0)
std::vector<bagua_p2p_op_t> ring_ops(const RingPlan& P, int g) {
    std::vector<bagua_p2p_op_t> v;
    const int p = P.p, r = P.r;
    auto rk = [&](int x) { return ((x % p) + p) % p; };
    auto key = [](int hop, int flow, int slice) { return hop * 4096 + flow * 2048 + slice; };
    auto add = [&](int peer, int send, int buf, int k, size_t off, size_t len) {
        if (len) v.push_back(bagua_p2p_op_t{peer, send, buf, k, (uint64_t)off, (uint64_t)len});
    };
    auto relay_off = [&](int q, int flow, int slice) {
        return ((size_t)((q & 1) * 2 + flow) * (size_t)(p - 3) + (size_t)(slice - 3)) * P.slot;
    };
    const int left = rk(r - 1), right = rk(r + 1);
    size_t b[65];
    if (g < P.pieces) {
        size_t lo, hi;
        piece_bytes(P.k, P.sched, g, &lo, &hi);
        if (hi > lo) {
            const size_t dhi = P.mp ? (ring_slices(lo, hi, p, b), b[3]) : hi;
            // flow 0: towards the right peer (lands in its left buffer); flow 1: towards the left peer
            add(right, 1, kBufMine, key(0, 0, 0), lo, dhi - lo);
            add(left, 1, kBufMine, key(0, 1, 0), lo, dhi - lo);
            add(left, 0, kBufLeft, key(0, 0, 0), lo, dhi - lo);
            add(right, 0, kBufRight, key(0, 1, 0), lo, dhi - lo);
            if (P.mp)
                for (int i = 3; i < p; ++i) {
                    const int d = i - 1;
                    const size_t len = b[i + 1] - b[i];
                    add(rk(r + d), 1, kBufMine, key(1, 0, i), b[i], len);
                    add(rk(r - d), 1, kBufMine, key(1, 1, i), b[i], len);
                    add(rk(r - d), 0, kBufRelay, key(1, 0, i), relay_off(g, 0, i), len);  // source r-d's slice
                    add(rk(r + d), 0, kBufRelay, key(1, 1, i), relay_off(g, 1, i), len);  // source r+d's slice
                }
        }
    }
    if (P.mp && g > 0) {
        const int q = g - 1;
        size_t lo, hi;
        piece_bytes(P.k, P.sched, q, &lo, &hi);
        if (hi > lo) {
            ring_slices(lo, hi, p, b);
            for (int i = 3; i < p; ++i) {
                const int d = i - 1;
                const size_t len = b[i + 1] - b[i];
                add(rk(r - d + 1), 1, kBufRelay, key(2, 0, i), relay_off(q, 0, i), len);  // source r-d -> its right
                add(rk(r + d - 1), 1, kBufRelay, key(2, 1, i), relay_off(q, 1, i), len);  // source r+d -> its left
                add(rk(r + d - 1), 0, kBufLeft, key(2, 0, i), b[i], len);    // left peer's slice via (r-1)+d
                add(rk(r - d + 1), 0, kBufRight, key(2, 1, i), b[i], len);   // right peer's slice via (r+1)-d
            }
        }
    }
    std::stable_sort(v.begin(), v.end(), [](const bagua_p2p_op_t& a, const bagua_p2p_op_t& c) {
        if (a.peer != c.peer) return a.peer < c.peer;
        if (a.is_send != c.is_send) return a.is_send > c.is_send;
        return a.key < c.key;
    });
    return v;
}

// one group of the ring exchange on the side stream
int ring_exchange_group(BaguaSingleCommunicatorC* c, const RingPlan& P, int g, uint8_t* const bufs[4]) {
    const std::vector<bagua_p2p_op_t> ops = ring_ops(P, g);
    if (ops.empty()) return BAGUA_OK;
    hipStream_t s1 = c->side;
    if (P.p == 1) {
        // one rank is its own left and right peer: every receive is a device copy of the
        // send with the same key (no RCCL self send/recv)
        for (const bagua_p2p_op_t& o : ops) {
            if (o.is_send) continue;
            for (const bagua_p2p_op_t& src : ops)
                if (src.is_send && src.key == o.key && src.bytes == o.bytes) {
                    if (hipMemcpyAsync(bufs[o.buffer] + o.offset, bufs[src.buffer] + src.offset, o.bytes,
                                       hipMemcpyDeviceToDevice, s1) != hipSuccess)
                        return BAGUA_ERR_HIP;
                    break;
                }
        }
        return BAGUA_OK;
    }
    int rc = c->t->group_start();
    for (const bagua_p2p_op_t& o : ops) {
        if (rc) break;
        uint8_t* ptr = bufs[o.buffer] + o.offset;
        rc = o.is_send ? c->t->send(ptr, o.bytes, BAGUA_DTYPE_U8, o.peer, s1)
                       : c->t->recv(ptr, o.bytes, BAGUA_DTYPE_U8, o.peer, s1);
    }
    const int rc_end = c->t->group_end();
    return rc ? rc : rc_end;
}

// Opt-in (BAGUA_PIECES_MULTIPATH in the op's `pieces`, or BAGUA_RING_MULTIPATH=1 read
// once at the communicator's creation): the only timing so far is RCCL's socket
// transport between processes on one GPU, where multipath was 5.3x slower than
// the direct exchange (profiles/r02_b_ar8_shared_gpu_rccl_socket.json); until an
// xGMI node shows it faster, the default is the reference's direct exchange
// (decentralized_low_precision_synchronous.rs:98-115).
bool ring_multipath_enabled(const BaguaSingleCommunicatorC* c) {
    return (int)c->nranks >= kRingMinMultipath && c->cfg.multipath;
}

}  // namespace

extern "C" {

int bagua_centralized_low_precision_pipelined(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int average,
                                              int method, int pieces) {
    if (method == BAGUA_COMPRESSION_ONEBIT) return centralized_pipelined_onebit(c, t, average, pieces);
    if (method != BAGUA_COMPRESSION_MINMAX_UINT8) return centralized(c, t, average, method, true);
    return centralized_pipelined(c, t, average, pieces);
}

int bagua_centralized_low_precision_synchronous(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int average,
                                                int method) {
    return bagua_centralized_low_precision_pipelined(c, t, average, method, 0);
}

int bagua_centralized_low_precision_synchronous_unfused(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t,
                                                        int average, int method) {
    return centralized(c, t, average, method, false);
}

int bagua_centralized_full_precision_synchronous(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int average) {
    // centralized_full_precision_synchronous.rs:44-50 (non-scattergather branch)
    if (!c) return BAGUA_ERR_INVALID_ARG;
    int rc = bagua_comm_allreduce_inplace(c, t, average ? BAGUA_OP_AVG : BAGUA_OP_SUM);
    return finish(c, rc);
}


static int decentralized(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, const bagua_tensor_t* weight,
                         const bagua_tensor_t* left, const bagua_tensor_t* right, int method, bool allow_fused,
                         int pieces = 1) {
    if (!c || !c->t || !t || !weight || !left || !right || !valid_schedule(pieces)) return BAGUA_ERR_INVALID_ARG;
    if (c->aborted.load()) return BAGUA_ERR_ABORTED;
    DeviceGuard guard(c->device_id);
    const uint64_t s = (uint64_t)(uintptr_t)c->stream;
    void* sp = (void*)(uintptr_t)s;
    int rc;
    if (t->num_elem_allocated > 0x7fffffffULL) return BAGUA_ERR_INVALID_ARG;
    const int n = (int)t->num_elem_allocated;
    const size_t S = bagua_compressed_size(method, t->dtype, 1, t->num_elem_allocated);
    if (!S) return BAGUA_ERR_UNSUPPORTED;
    // fused kernels (csrc/kernels/decentralized.hip) for fully valid, same-shape
    // MinMax buckets; anything else runs the reference's op sequence.  The choice (and
    // with it the pipelined exchange schedule) depends only on values equal on every
    // rank; a rank whose tensors are not 16-B aligned runs on aligned copies
    bool fused = allow_fused && method == BAGUA_COMPRESSION_MINMAX_UINT8 && t->num_elem == t->num_elem_allocated;
    for (const bagua_tensor_t* o : {weight, left, right})
        fused = fused && o->dtype == t->dtype && o->num_elem == t->num_elem;
    if (fused && (t->ptr % 16 || weight->ptr % 16 || left->ptr % 16 || right->ptr % 16))
        return with_aligned_copy(c, {t, weight, left, right}, [&](const std::vector<const bagua_tensor_t*>& u) {
            return decentralized(c, u[0], u[1], u[2], u[3], method, allow_fused, pieces);
        });
    // the exchange schedule, from values equal on every rank (ScheduleConfig included)
    const int caller = pieces;
    pieces &= BAGUA_PIECES_COUNT_MASK;
    if (pieces < 1) pieces = c->nranks == 1 ? 1 : auto_pieces(c, (size_t)n);
    const int sched = op_schedule(c, pieces, caller);
    const bool multipath =
        (caller & BAGUA_PIECES_MULTIPATH) ? (int)c->nranks >= kRingMinMultipath : ring_multipath_enabled(c);
    const bool pipelined = fused && (pieces > 1 || multipath);
    if ((rc = check_schedule(c, pipelined ? kOpRingPipelined : (allow_fused ? kOpRing : kOpRingUnfused), method, t,
                             (uint64_t)n, pipelined ? sched | (multipath ? BAGUA_PIECES_MULTIPATH : 0) : 1, 1)))
        return rc;
    if (fused && !pipelined && c->nranks == 1 && env_int("BAGUA_ONE_RANK_FUSED", 1) != 0) {
        // one rank: both peers' payloads are its own bytes, so the op is the mix pass and
        // one pass applying d = dq(q(mixed)) to all four tensors, no payload written
        // (bagua_ring_one_rank_minmax); BAGUA_ONE_RANK_FUSED=0: the steps below (A/B)
        const size_t wsb = bagua_minmax_u8_workspace_bytes(n, 1);
        uint64_t wsp = 0;
        if ((rc = stream_workspace(c->device_id, s, wsb, &wsp)) != BAGUA_OK) return finish(c, rc);
        rc = bagua_ring_one_rank_minmax(t->dtype, (void*)(uintptr_t)t->ptr, (void*)(uintptr_t)weight->ptr,
                                        (void*)(uintptr_t)left->ptr, (void*)(uintptr_t)right->ptr, n,
                                        (void*)(uintptr_t)wsp, wsb, sp);
        if (rc != BAGUA_ERR_UNSUPPORTED) return finish(c, rc);
    }
    OpBuffer mine(c), lbuf(c), rbuf(c);
    TRY(mine.allocate(c->device_id, S));
    TRY(lbuf.allocate(c->device_id, S));
    TRY(rbuf.allocate(c->device_id, S));
    const bagua_tensor_t mv = u8_view(mine.ptr(), S, c->device_id);
    const bagua_tensor_t lv = u8_view(lbuf.ptr(), S, c->device_id);
    const bagua_tensor_t rv = u8_view(rbuf.ptr(), S, c->device_id);
    void* tp = (void*)(uintptr_t)t->ptr;
    void* wp = (void*)(uintptr_t)weight->ptr;
    void* lp = (void*)(uintptr_t)left->ptr;
    void* rp = (void*)(uintptr_t)right->ptr;
    bool mixed = false;
    if (fused) {
        // :45-64 t += L/3 + R/3 - 5W/3 (three rounded steps) with the min/max partials, then quantise
        const size_t wsb = bagua_minmax_u8_workspace_bytes(n, 1);
        uint64_t wsp = 0;
        if ((rc = stream_workspace(c->device_id, s, wsb, &wsp)) != BAGUA_OK) return finish(c, rc);
        void* ws = (void*)(uintptr_t)wsp;
        rc = bagua_ring_mix_minmax(t->dtype, tp, lp, rp, wp, n, ws, wsb, sp);
        if (rc == BAGUA_OK) {
            if (pipelined) {
                // pipelined: quantise piece q -> exchange piece q (side stream) -> apply piece q;
                // one header for the whole bucket, travelling with piece 0.  Multipath: the
                // relayed slices of piece q arrive with group q + 1.
                RingPlan plan;
                TRY(ring_plan((int)c->nranks, (int)c->rank, n, sched, multipath, &plan));
                if (plan.k.S != S) return finish(c, BAGUA_ERR_INVALID_ARG);
                OpBuffer relay(c);
                if (ring_relay_bytes(plan)) TRY(relay.allocate(c->device_id, ring_relay_bytes(plan)));
                if (c->ensure_side(2 * (size_t)pieces + 1)) return finish(c, BAGUA_ERR_HIP);
                hipStream_t s1 = c->side;
                hipEvent_t* quantised = c->events.data();
                hipEvent_t* exchanged = quantised + pieces;
                hipEvent_t start = exchanged[pieces];
                uint8_t* mb = mine.as<uint8_t>();
                uint8_t* lb = lbuf.as<uint8_t>();
                uint8_t* rb = rbuf.as<uint8_t>();
                uint8_t* const bufs[4] = {mb, lb, rb, relay.as<uint8_t>()};
                HIP2(hipEventRecord(start, c->stream));
                HIP2(hipStreamWaitEvent(s1, start, 0));
                for (int q = 0; q < pieces; ++q) {
                    int b, e;
                    bagua_minmax_u8_piece_range(n, sched, q, &b, &e);
                    if (q == 0 || b < e)
                        TRY2(bagua_minmax_u8_quantize_range(t->dtype, tp, n, n, 1, mb, S, ws, wsb, -1, b, e, sp));
                    HIP2(hipEventRecord(quantised[q], c->stream));
                }
                for (int g = 0; g < plan.groups; ++g) {
                    if (g < pieces) HIP2(hipStreamWaitEvent(s1, quantised[g], 0));
                    TRY2(ring_exchange_group(c, plan, g, bufs));
                    const int done = plan.mp ? g - 1 : g;  // the piece this group completes
                    if (done >= 0) HIP2(hipEventRecord(exchanged[done], s1));
                }
                for (int q = 0; q < pieces; ++q) {
                    int b, e;
                    bagua_minmax_u8_piece_range(n, sched, q, &b, &e);
                    HIP2(hipStreamWaitEvent(c->stream, exchanged[q], 0));
                    if (b < e)
                        TRY2(bagua_ring_apply_minmax_range(t->dtype, mb, lb, rb, S, n, b, e, tp, wp, lp, rp, sp));
                }
                return finish_both(c, BAGUA_OK);
            }
            TRY(bagua_minmax_u8_compress_stage(2, t->dtype, tp, n, n, 1, mine.as<uint8_t>(), S, ws, wsb, -1, sp));
            mixed = true;
        } else if (rc != BAGUA_ERR_UNSUPPORTED) {
            return finish(c, rc);
        }
    }
    if (!mixed) {
        // :45-60: t += L/3; t += R/3; t += W*(-5/3)  (f64 literals cast to f32)
        TRY(bagua_tensor_addmul_inplace(t, left, (float)(1.0 / 3.0), s));
        TRY(bagua_tensor_addmul_inplace(t, right, (float)(1.0 / 3.0), s));
        TRY(bagua_tensor_addmul_inplace(t, weight, (float)(-5.0 / 3.0), s));
        // :61-64 whole-bucket compress (n_chunks = 1)
        TRY(bagua_tensor_compress_into(t, method, 1, s, -1, &mv));
    }
    // :98-115 ring exchange inside one group.  One rank is its own left and right
    // peer: what it would receive are its own bytes, so the op reads `mine` in their
    // place (RCCL's self send/recv of 2 x S bytes took 206 us for 2^27 bf16).
    const int p = (int)c->nranks, r = (int)c->rank;
    const int lpeer = (r + p - 1) % p, rpeer = (r + 1) % p;
    if (p > 1) {
        TRY(c->t->group_start());
        rc = bagua_comm_send(c, &mv, lpeer);
        if (!rc) rc = bagua_comm_send(c, &mv, rpeer);
        if (!rc) rc = bagua_comm_recv(c, &lv, lpeer);
        if (!rc) rc = bagua_comm_recv(c, &rv, rpeer);
        const int rc_end = c->t->group_end();
        if (rc || rc_end) return finish(c, rc ? rc : rc_end);
    }
    const bagua_tensor_t* from_l = p > 1 ? &lv : &mv;
    const bagua_tensor_t* from_r = p > 1 ? &rv : &mv;
    // :126-151
    if (fused) {
        rc = bagua_ring_apply_minmax(t->dtype, mine.as<uint8_t>(), (const uint8_t*)(uintptr_t)from_l->ptr,
                                     (const uint8_t*)(uintptr_t)from_r->ptr, S, n, tp, wp, lp, rp, sp);
        if (rc == BAGUA_OK) return finish(c, BAGUA_OK);
        if (rc != BAGUA_ERR_UNSUPPORTED) return finish(c, rc);
    }
    TRY(bagua_tensor_decompress_from(t, method, 1, from_l, s));
    TRY(bagua_tensor_add_inplace(left, t, s));
    TRY(bagua_tensor_decompress_from(t, method, 1, from_r, s));
    TRY(bagua_tensor_add_inplace(right, t, s));
    TRY(bagua_tensor_decompress_from(t, method, 1, &mv, s));
    TRY(bagua_tensor_add_inplace(t, weight, s));
    TRY(bagua_tensor_clone_from(weight, t, s));
    return finish(c, BAGUA_OK);
}

int bagua_comm_set_async(BaguaSingleCommunicatorC* c, int on) {
    if (!c) return BAGUA_ERR_INVALID_ARG;
    c->async = on != 0;
    return BAGUA_OK;
}

int bagua_ring_exchange_plan(int nranks, int rank, int chunk_size, int pieces, int multipath, int* groups,
                             size_t* relay_bytes) {
    RingPlan P;
    const int rc = ring_plan(nranks, rank, chunk_size, pieces, multipath != 0, &P);
    if (rc) return rc;
    if (groups) *groups = P.groups;
    if (relay_bytes) *relay_bytes = ring_relay_bytes(P);
    return BAGUA_OK;
}

int bagua_ring_exchange_ops(int nranks, int rank, int chunk_size, int pieces, int multipath, int group,
                            bagua_p2p_op_t* ops, int max_ops) {
    RingPlan P;
    const int rc = ring_plan(nranks, rank, chunk_size, pieces, multipath != 0, &P);
    if (rc) return -rc;
    if (group < 0 || group >= P.groups) return -BAGUA_ERR_INVALID_ARG;
    const std::vector<bagua_p2p_op_t> v = ring_ops(P, group);
    if (!ops || (int)v.size() > max_ops) return -BAGUA_ERR_INVALID_ARG;
    std::copy(v.begin(), v.end(), ops);
    return (int)v.size();
}

int bagua_decentralized_low_precision_synchronous(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t,
                                                  const bagua_tensor_t* weight, const bagua_tensor_t* left,
                                                  const bagua_tensor_t* right, int method) {
    return decentralized(c, t, weight, left, right, method, true, 0);
}

}  // extern "C"

// communicators/mod.rs:390-427, execute_communication with a hierarchical
// communicator (:243-336): every rank of the node reduces (AVG or SUM) into the
// node leader (intranode rank 0, :264-283 / :312-325), the leader runs the op among
// the leaders on the internode communicator, and the leader broadcasts the result
// over the node (:286-294 / :327-330).  The leader's two communicators share one
// stream and device (:250-256, :356-360).
template <typename F>
static int hierarchical(BaguaSingleCommunicatorC* intra, BaguaSingleCommunicatorC* inter, const bagua_tensor_t* t,
                        bool intranode_average, F&& op) {
    if (!intra || !intra->t || !t) return BAGUA_ERR_INVALID_ARG;
    if (intra->aborted.load()) return BAGUA_ERR_ABORTED;
    const bool leader = intra->rank == 0;
    if (leader && (!inter || inter->stream != intra->stream || inter->device_id != intra->device_id))
        return BAGUA_ERR_INVALID_ARG;
    DeviceGuard guard(intra->device_id);
    int rc = bagua_comm_reduce_inplace(intra, t, 0, intranode_average ? BAGUA_OP_AVG : BAGUA_OP_SUM);
    if (!rc && leader) rc = op(inter);
    if (!rc) rc = bagua_comm_broadcast(intra, t, 0);
    return finish(intra, rc);
}

extern "C" {

int bagua_centralized_low_precision_hierarchical(BaguaSingleCommunicatorC* intranode,
                                                 BaguaSingleCommunicatorC* internode, const bagua_tensor_t* t,
                                                 int average, int method) {
    // centralized_low_precision_synchronous.rs:25-30: intranode average = the op's average
    return hierarchical(intranode, internode, t, average != 0, [&](BaguaSingleCommunicatorC* c) {
        return bagua_centralized_low_precision_synchronous(c, t, average, method);
    });
}

int bagua_centralized_full_precision_hierarchical(BaguaSingleCommunicatorC* intranode,
                                                  BaguaSingleCommunicatorC* internode, const bagua_tensor_t* t,
                                                  int average) {
    return hierarchical(intranode, internode, t, average != 0, [&](BaguaSingleCommunicatorC* c) {
        return bagua_centralized_full_precision_synchronous(c, t, average);
    });
}

int bagua_decentralized_low_precision_hierarchical(BaguaSingleCommunicatorC* intranode,
                                                   BaguaSingleCommunicatorC* internode, const bagua_tensor_t* t,
                                                   const bagua_tensor_t* weight, const bagua_tensor_t* left,
                                                   const bagua_tensor_t* right, int method) {
    // decentralized_low_precision_synchronous.rs:37-41: the node always averages
    return hierarchical(intranode, internode, t, true, [&](BaguaSingleCommunicatorC* c) {
        return bagua_decentralized_low_precision_synchronous(c, t, weight, left, right, method);
    });
}

int bagua_decentralized_low_precision_pipelined(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t,
                                                const bagua_tensor_t* weight, const bagua_tensor_t* left,
                                                const bagua_tensor_t* right, int method, int pieces) {
    return decentralized(c, t, weight, left, right, method, true, pieces);
}

int bagua_decentralized_low_precision_synchronous_unfused(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t,
                                                          const bagua_tensor_t* weight, const bagua_tensor_t* left,
                                                          const bagua_tensor_t* right, int method) {
    return decentralized(c, t, weight, left, right, method, false);
}

}  // extern "C"
