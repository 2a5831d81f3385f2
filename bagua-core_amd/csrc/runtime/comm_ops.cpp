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

using namespace bagua;

namespace {

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

int finish(BaguaSingleCommunicatorC* c, int rc) {
    const hipError_t e = hipStreamSynchronize(c->stream);
    if (rc) return rc;
    return e == hipSuccess ? BAGUA_OK : BAGUA_ERR_HIP;
}

#define TRY(x)                 \
    do {                       \
        rc = (x);              \
        if (rc) return finish(c, rc); \
    } while (0)

int centralized(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int average, int method, bool fused) {
    Chunking k;
    int rc = plan(c, t, method, &k);
    if (rc) return rc;
    DeviceGuard guard(c->device_id);
    const uint64_t s = (uint64_t)(uintptr_t)c->stream;
    PoolBuffer send, recv;
    TRY(send.allocate(c->device_id, k.S));
    TRY(recv.allocate(c->device_id, k.S));
    const bagua_tensor_t sv = u8_view(send.ptr(), k.S, c->device_id);
    const bagua_tensor_t rv = u8_view(recv.ptr(), k.S, c->device_id);
    // 1. compress every chunk (target -1)
    TRY(bagua_tensor_compress_into(t, method, k.p, s, -1, &sv));
    // 2. alltoall: slot j of recv <- rank j's segment `rank`
    TRY(c->t->alltoall(send.as<void>(), recv.as<void>(), k.S / k.p, BAGUA_DTYPE_U8, c->stream));
    // 3. reduce the p received versions of the own chunk and requantise it into send[rank]
    bool done = false;
    if (fused && method == BAGUA_COMPRESSION_MINMAX_UINT8) {
        const size_t ws_bytes = bagua_minmax_u8_workspace_bytes((int)k.cs, k.p);
        const uint64_t ws = stream_workspace(c->device_id, s, ws_bytes);
        if (!ws) return finish(c, BAGUA_ERR_OOM);
        rc = bagua_minmax_u8_reduce_requantize(t->dtype, recv.as<uint8_t>(), k.S, (int)k.cs, k.p,
                                               (void*)(uintptr_t)t->ptr, average, send.as<uint8_t>(), k.S, k.rank,
                                               (void*)(uintptr_t)ws, ws_bytes, (void*)(uintptr_t)s);
        if (rc == BAGUA_OK) done = true;
        else if (rc != BAGUA_ERR_UNSUPPORTED) return finish(c, rc);
    }
    if (!done) {
        TRY(bagua_tensor_decompress_from(t, method, k.p, &rv, s));
        TRY(bagua_tensor_reduce_inplace(t, k.p, k.rank, average, s));
        TRY(bagua_tensor_compress_into(t, method, k.p, s, k.rank, &sv));
    }
    // 4. allgather the requantised chunks in place, 5. decompress everything
    TRY(bagua_comm_allgather_inplace(c, &sv));
    TRY(bagua_tensor_decompress_from(t, method, k.p, &sv, s));
    return finish(c, BAGUA_OK);
}

}  // namespace

extern "C" {

int bagua_centralized_low_precision_synchronous(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t, int average,
                                                int method) {
    return centralized(c, t, average, method, true);
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

int bagua_decentralized_low_precision_synchronous(BaguaSingleCommunicatorC* c, const bagua_tensor_t* t,
                                                  const bagua_tensor_t* weight, const bagua_tensor_t* left,
                                                  const bagua_tensor_t* right, int method) {
    if (!c || !c->t || !t || !weight || !left || !right) return BAGUA_ERR_INVALID_ARG;
    if (c->aborted.load()) return BAGUA_ERR_ABORTED;
    DeviceGuard guard(c->device_id);
    const uint64_t s = (uint64_t)(uintptr_t)c->stream;
    int rc;
    // :45-60: t += L/3; t += R/3; t += W*(-5/3)  (f64 literals cast to f32)
    TRY(bagua_tensor_addmul_inplace(t, left, (float)(1.0 / 3.0), s));
    TRY(bagua_tensor_addmul_inplace(t, right, (float)(1.0 / 3.0), s));
    TRY(bagua_tensor_addmul_inplace(t, weight, (float)(-5.0 / 3.0), s));
    // :61-64 whole-bucket compress (n_chunks = 1)
    if (t->num_elem_allocated > 0x7fffffffULL) return BAGUA_ERR_INVALID_ARG;
    const size_t S = bagua_compressed_size(method, t->dtype, 1, t->num_elem_allocated);
    if (!S) return BAGUA_ERR_UNSUPPORTED;
    PoolBuffer mine, lbuf, rbuf;
    TRY(mine.allocate(c->device_id, S));
    TRY(lbuf.allocate(c->device_id, S));
    TRY(rbuf.allocate(c->device_id, S));
    const bagua_tensor_t mv = u8_view(mine.ptr(), S, c->device_id);
    const bagua_tensor_t lv = u8_view(lbuf.ptr(), S, c->device_id);
    const bagua_tensor_t rv = u8_view(rbuf.ptr(), S, c->device_id);
    TRY(bagua_tensor_compress_into(t, method, 1, s, -1, &mv));
    // :98-115 ring exchange inside one group
    const int p = (int)c->nranks, r = (int)c->rank;
    const int lpeer = (r + p - 1) % p, rpeer = (r + 1) % p;
    TRY(c->t->group_start());
    rc = bagua_comm_send(c, &mv, lpeer);
    if (!rc) rc = bagua_comm_send(c, &mv, rpeer);
    if (!rc) rc = bagua_comm_recv(c, &lv, lpeer);
    if (!rc) rc = bagua_comm_recv(c, &rv, rpeer);
    const int rc_end = c->t->group_end();
    if (rc || rc_end) return finish(c, rc ? rc : rc_end);
    // :126-151
    TRY(bagua_tensor_decompress_from(t, method, 1, &lv, s));
    TRY(bagua_tensor_add_inplace(left, t, s));
    TRY(bagua_tensor_decompress_from(t, method, 1, &rv, s));
    TRY(bagua_tensor_add_inplace(right, t, s));
    TRY(bagua_tensor_decompress_from(t, method, 1, &mv, s));
    TRY(bagua_tensor_add_inplace(t, weight, s));
    TRY(bagua_tensor_clone_from(weight, t, s));
    return finish(c, BAGUA_OK);
}

}  // extern "C"
