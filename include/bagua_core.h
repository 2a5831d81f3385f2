/*
 * bagua_core.h — C ABI of the MI355X host runtime (libbagua_core.so).
 *
 * Replaces, behind plain pointers and sizes, the parts of the reference's
 * Rust host that sit on the compressed-gradient path:
 *   - device memory pool      bagua-core-internal/src/resource_pool/mod.rs:11-60
 *   - tensor codec dispatch   bagua-core-internal/src/datatypes/mod.rs:313-484,665-742
 *   - communicator            bagua-core-internal/src/communicators/mod.rs:25-60,430-1043
 *                             bagua-core-c/src/lib.rs:9-69 (C shim, exported UNMANGLED here)
 *   - comm ops                src/comm_ops/centralized_low_precision_synchronous.rs:16-73
 *                             src/comm_ops/decentralized_low_precision_synchronous.rs:23-154
 * Collectives are RCCL (librccl) over xGMI; no Aluminum, no MPI.
 *
 * Every function returns a bagua_status_t-compatible int (0 = ok) unless it
 * returns a size or handle; nothing here calls exit().
 */
#ifndef BAGUA_CORE_H
#define BAGUA_CORE_H

#include <stddef.h>
#include <stdint.h>

#include "bagua_kernels.h"

#ifdef __cplusplus
extern "C" {
#endif

/* tensor dtypes: kernels' F32/F16/BF16 plus the reference's U8/I64/U64 (datatypes/mod.rs:40-47) */
enum { BAGUA_DTYPE_U8 = 3, BAGUA_DTYPE_I64 = 4, BAGUA_DTYPE_U64 = 5 };

/* compression methods: "MinMaxUInt8" (datatypes/mod.rs:744-747) and the 1-bit extension */
enum { BAGUA_COMPRESSION_NONE = 0, BAGUA_COMPRESSION_MINMAX_UINT8 = 1, BAGUA_COMPRESSION_ONEBIT = 2 };

/* reduction ops, Aluminum/BaguaReductionOp numbering (datatypes/mod.rs:24-38) */
enum { BAGUA_OP_SUM = 0, BAGUA_OP_PROD = 1, BAGUA_OP_MIN = 2, BAGUA_OP_MAX = 3, BAGUA_OP_AVG = 10 };

enum { BAGUA_ERR_COMM = 16, BAGUA_ERR_OOM = 17, BAGUA_ERR_ABORTED = 18 };

/* BaguaTensorRaw (datatypes/mod.rs:79-86) without the Rust ownership vector */
typedef struct bagua_tensor {
    uint64_t ptr;
    uint64_t num_elem;
    uint64_t num_elem_allocated;
    int32_t dtype;
    int32_t device_id;
} bagua_tensor_t;

size_t bagua_dtype_bytes(int dtype);
/* cuda_utils.rs:1-6: synchronous device-to-host copy (to_numpy_* read-back) */
int bagua_memcpy_device_to_host_sync(void* host, uint64_t device_ptr, size_t bytes);
/* datatypes/mod.rs:969-980: make `stream` wait for a tensor's ready event (0 = no event) */
int bagua_stream_wait_event(uint64_t stream, uint64_t event);

/* ---------------------------------------------------------------- pool -- */
/* CUDA_DEVICE_MEMORY_POOL (resource_pool/mod.rs:53-60): size-classed reuse of hipMalloc'd blocks */
int bagua_pool_alloc(int device_id, size_t bytes, uint64_t* ptr);
int bagua_pool_free(uint64_t ptr);
/* Stream-ordered free: the block is reused only after everything queued so far on
 * each of `streams` (n of them; 0 = the null stream) has completed (an event per
 * stream, queried at the next allocation).  For buffers that queued work may still
 * read, e.g. a compressed tensor dropped right after a decompress_from. */
int bagua_pool_free_after(uint64_t ptr, const uint64_t* streams, int n);
int bagua_pool_trim(int device_id);
/* Blocks freed with bagua_pool_free_after whose streams have not drained yet. */
size_t bagua_pool_bytes_pending(int device_id);
/* HIP-graph capture of comm ops on the calling thread: between begin and end, the
 * blocks the ops take from the pool belong to the graph (frees are deferred) and the
 * pool queries no events.  Release the arena once the graph is destroyed and no
 * replay is in flight.  Returns NULL when an arena is already open on this thread. */
void* bagua_pool_capture_begin(void);
int bagua_pool_capture_end(void* arena);
int bagua_pool_capture_release(void* arena);
/* Drops `stream`'s per-stream workspace and its one-launch encode slot after the
 * stream has drained.  Communicator teardown calls it for its streams; call it
 * before destroying any other stream that ran codec calls. */
int bagua_release_stream_resources(int device_id, uint64_t stream);
/* Number of live per-stream workspaces (diagnostics). */
size_t bagua_stream_workspace_count(void);
size_t bagua_pool_bytes_in_use(int device_id);
size_t bagua_pool_bytes_cached(int device_id);

/* --------------------------------------------------------- tensor codec -- */
/* MinMaxUInt8CompressionParameters::get_compressed_buffer_size (datatypes/mod.rs:669-704) */
size_t bagua_compressed_size(int method, int dtype, size_t n_chunks, size_t chunk_size);
/* RawBaguaTensor::compress (datatypes/mod.rs:313-396): `out` receives a pool-owned U8
 * tensor of bagua_compressed_size() bytes (release it with bagua_pool_free). */
int bagua_tensor_compress(const bagua_tensor_t* t, int method, int n_chunks, uint64_t stream,
                          int target_chunk, bagua_tensor_t* out);
/* the same into a caller-provided U8 buffer of exactly bagua_compressed_size() bytes */
int bagua_tensor_compress_into(const bagua_tensor_t* t, int method, int n_chunks, uint64_t stream,
                               int target_chunk, const bagua_tensor_t* out);
/* RawBaguaTensor::decompress_from (datatypes/mod.rs:398-446) */
int bagua_tensor_decompress_from(const bagua_tensor_t* t, int method, int n_chunks,
                                 const bagua_tensor_t* compressed, uint64_t stream);
/* reduce_mean_inplace / reduce_sum_inplace (datatypes/mod.rs:448-522) */
int bagua_tensor_reduce_inplace(const bagua_tensor_t* t, int n_chunks, int target_chunk, int average,
                                uint64_t stream);
/* add / addmul / clone_from (datatypes/mod.rs:129-274) */
int bagua_tensor_add_inplace(const bagua_tensor_t* t, const bagua_tensor_t* other, uint64_t stream);
int bagua_tensor_addmul_inplace(const bagua_tensor_t* t, const bagua_tensor_t* other, float factor,
                                uint64_t stream);
int bagua_tensor_clone_from(const bagua_tensor_t* t, const bagua_tensor_t* other, uint64_t stream);

/* --------------------------------------------------------- communicator -- */
typedef struct BaguaSingleCommunicatorC BaguaSingleCommunicatorC;

/* bagua-core-c/src/lib.rs:9-69, unmangled; nccl_unique_id_str is base64 of ncclUniqueId */
BaguaSingleCommunicatorC* bagua_single_communicator_c_create(size_t rank, size_t nranks, size_t device_id,
                                                             uint64_t stream_ptr,
                                                             const char* nccl_unique_id_str);
void bagua_single_communicator_c_destroy(BaguaSingleCommunicatorC** ptr);
int32_t bagua_single_communicator_c_nranks(BaguaSingleCommunicatorC** ptr, size_t* nranks);
/* additional accessors / collectives (communicators/mod.rs) */
int32_t bagua_single_communicator_c_rank(BaguaSingleCommunicatorC** ptr, size_t* rank);
uint64_t bagua_single_communicator_c_stream(BaguaSingleCommunicatorC* comm);
int bagua_generate_nccl_unique_id_str(char* buf, size_t buf_len);
int bagua_comm_abort(BaguaSingleCommunicatorC* comm);
int bagua_comm_check_abort(BaguaSingleCommunicatorC* comm);
/* The switches that shape an op's collectives, fixed when the communicator is created
 * and equal on every rank (rank 0's environment wins; an op never reads them again):
 * out[0..4] = BAGUA_PIPELINE_PIECES (piece cap), BAGUA_PIPELINE_MIN_PIECE,
 * BAGUA_PIPELINE_TAPER, BAGUA_RING_MULTIPATH, BAGUA_CHECK_SCHEDULE.  With the last on,
 * every op first allgathers a descriptor of itself (op, codec, dtype, p, chunk size,
 * tensor sizes, piece schedule, average, op number) and all ranks return
 * BAGUA_ERR_INVALID_ARG, before posting anything, when any two differ. */
int bagua_comm_schedule_config(BaguaSingleCommunicatorC* comm, int32_t* out, int n);
int bagua_comm_allreduce_inplace(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t, int op);
int bagua_comm_allreduce(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* send, const bagua_tensor_t* recv,
                         int op);
int bagua_comm_broadcast(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t, int root);
/* reduce (communicators/mod.rs reduce / reduce_inplace): the SUM / AVG / ... of every
 * rank's tensor lands on `root` */
int bagua_comm_reduce_inplace(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t, int root, int op);
int bagua_comm_reduce(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* send, const bagua_tensor_t* recv, int root,
                      int op);
int bagua_comm_alltoall(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* send, const bagua_tensor_t* recv);
int bagua_comm_alltoall_inplace(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t);
int bagua_comm_allgather_inplace(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t);
int bagua_comm_allgather(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* send, const bagua_tensor_t* recv);
int bagua_comm_send(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t, int peer);
int bagua_comm_recv(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t, int peer);
int bagua_comm_group_start(void);
int bagua_comm_group_end(void);
int bagua_comm_barrier(BaguaSingleCommunicatorC* comm);
int bagua_comm_synchronize(BaguaSingleCommunicatorC* comm);

/* In-process loopback transport (test harness): nranks virtual ranks, one host
 * thread each, on one device; collectives are device-to-device copies.  Runs
 * the comm ops below at nranks > 1 on a single GPU.  Destroy communicators
 * with bagua_single_communicator_c_destroy, then the group. */
void* bagua_loopback_group_create(int nranks, int device_id);
void bagua_loopback_group_destroy(void* group);
BaguaSingleCommunicatorC* bagua_loopback_communicator_create(void* group, size_t rank, uint64_t stream_ptr);

/* ------------------------------------------------------------- comm ops -- */
/* Async mode (off by default): the comm ops below return as soon as their work is
 * enqueued on the communicator's stream instead of waiting for it (the reference's
 * datatypes/mod.rs:1062-1066 sync); their temporary buffers go back to the pool
 * behind the stream.  Synchronise the stream (bagua_comm_synchronize) before
 * reading a result on the host.  The native scheduler runs its ops this way and
 * waits for each bucket in bagua_comm_backend_wait_pending_comm_ops. */
int bagua_comm_set_async(BaguaSingleCommunicatorC* comm, int on);
/* CentralizedLowPrecisionSynchronous::execute_background_communication on one
 * flat communication tensor (centralized_low_precision_synchronous.rs:16-73). */
int bagua_centralized_low_precision_synchronous(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t,
                                                int average, int method);
/* The same op with each chunk cut into `pieces` element ranges, the exchange of
 * one piece (side stream, grouped send/recv) overlapping the codec kernels of
 * the next; bit-identical to the unpieced op.  pieces = 0 picks automatically
 * (BAGUA_PIPELINE_PIECES cap, default 4; BAGUA_PIPELINE_MIN_PIECE payload bytes
 * per chunk piece, default 1 MiB; one rank: unpieced), 1 disables; the op above
 * runs this with pieces = 0.  MinMaxUInt8 and the 1-bit codec; shapes the fused
 * kernels cannot take run unpieced. */
int bagua_centralized_low_precision_pipelined(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t, int average,
                                              int method, int pieces);
/* the reference's unfused sequence, kept for A/B measurement and parity */
int bagua_centralized_low_precision_synchronous_unfused(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t,
                                                        int average, int method);
/* CentralizedFullPrecisionSynchronous (allreduce SUM/AVG), the baseline denominator */
int bagua_centralized_full_precision_synchronous(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t,
                                                 int average);
/* DecentralizedLowPrecisionSynchronous, ring peers (decentralized_low_precision_synchronous.rs:23-154) */
int bagua_decentralized_low_precision_synchronous(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t,
                                                  const bagua_tensor_t* weight,
                                                  const bagua_tensor_t* left_peer_weight,
                                                  const bagua_tensor_t* right_peer_weight, int method);
/* The same with the bucket cut into `pieces` element ranges: after the mix pass
 * (whole-bucket min/max), piece q is quantised, sent to both peers on a side
 * stream and applied as it arrives, so quantise, exchange and apply overlap;
 * bit-identical to the unpieced op.  pieces = 0 picks automatically (as above),
 * 1 disables; the op above runs this with pieces = 0. */
int bagua_decentralized_low_precision_pipelined(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t,
                                                const bagua_tensor_t* weight, const bagua_tensor_t* left_peer_weight,
                                                const bagua_tensor_t* right_peer_weight, int method, int pieces);
/* Ring exchange schedule of the fused decentralized op (host-only, no device work).
 * The reference sends the whole compressed bucket straight to both ring peers
 * (decentralized_low_precision_synchronous.rs:98-115), which loads 2 of a
 * GPU's 7 xGMI links.  Opt-in (BAGUA_RING_MULTIPATH=1, from nranks >= 6), each
 * piece's bytes are cut into nranks slices: 3 go straight to the peer, slice k
 * (3 <= k < nranks) is relayed through rank +-(k-1), so every link carries at
 * most 4/nranks of the payload (8 ranks: half) instead of all of it; the relay
 * forwards in the next group, so there are pieces + 1 groups.  Bytes arrive
 * unchanged: the op stays bit-identical.
 * Fills `ops` (capacity max_ops) with group `group`'s transfers for a bucket of
 * `chunk_size` elements (n_chunks = 1 MinMax segments) cut into `pieces`, sorted
 * so the k-th transfer between two ranks is the same message on both sides
 * (NCCL's in-order p2p matching); returns the count (< 0: error).  *relay_bytes
 * receives the relay scratch size (bytes). */
typedef struct bagua_p2p_op {
    int32_t peer;
    int32_t is_send;
    int32_t buffer; /* 0 own payload, 1 left peer's payload, 2 right peer's payload, 3 relay scratch */
    int32_t key;    /* (hop, flow, slice) order key */
    uint64_t offset;
    uint64_t bytes;
} bagua_p2p_op_t;
int bagua_ring_exchange_plan(int nranks, int rank, int chunk_size, int pieces, int multipath, int* groups,
                             size_t* relay_bytes);
int bagua_ring_exchange_ops(int nranks, int rank, int chunk_size, int pieces, int multipath, int group,
                            bagua_p2p_op_t* ops, int max_ops);
/* Hierarchical mode (communicators/mod.rs:243-427): intranode reduce (AVG when the op
 * averages; always AVG for the decentralized op) into intranode rank 0, the op among
 * the node leaders on `internode` (needed on the leader only, same stream and device as
 * `intranode`), intranode broadcast from rank 0.  Workers pass internode = NULL. */
int bagua_centralized_low_precision_hierarchical(BaguaSingleCommunicatorC* intranode,
                                                 BaguaSingleCommunicatorC* internode, const bagua_tensor_t* t,
                                                 int average, int method);
int bagua_centralized_full_precision_hierarchical(BaguaSingleCommunicatorC* intranode,
                                                  BaguaSingleCommunicatorC* internode, const bagua_tensor_t* t,
                                                  int average);
int bagua_decentralized_low_precision_hierarchical(BaguaSingleCommunicatorC* intranode,
                                                   BaguaSingleCommunicatorC* internode, const bagua_tensor_t* t,
                                                   const bagua_tensor_t* weight, const bagua_tensor_t* left,
                                                   const bagua_tensor_t* right, int method);
/* the reference's unfused op sequence (3 addmul, compress, 3 x decompress + add, clone), for A/B */
int bagua_decentralized_low_precision_synchronous_unfused(BaguaSingleCommunicatorC* comm, const bagua_tensor_t* t,
                                                          const bagua_tensor_t* weight,
                                                          const bagua_tensor_t* left_peer_weight,
                                                          const bagua_tensor_t* right_peer_weight, int method);

/* ------------------------------------------------------ bucket + scheduler -- */
/* BaguaBucket (datatypes/mod.rs:1072-1267) and BaguaCommBackend (src/lib.rs:125-338)
 * in C++: a bucket is a named list of tensors (same dtype and device) plus comm
 * ops; the backend schedules buckets in registration order as their tensors are
 * marked ready and runs their ops on one native worker thread. */
typedef struct BaguaBucketC BaguaBucketC;
typedef struct BaguaCommBackendC BaguaCommBackendC;

enum {
    BAGUA_BUCKET_OP_CENTRALIZED_LOW_PRECISION = 1,   /* centralized_low_precision_synchronous.rs */
    BAGUA_BUCKET_OP_CENTRALIZED_FULL_PRECISION = 2,  /* centralized_full_precision_synchronous.rs */
    BAGUA_BUCKET_OP_DECENTRALIZED_LOW_PRECISION = 3, /* decentralized_low_precision_synchronous.rs */
    BAGUA_BUCKET_OP_CALLBACK = 4                     /* python_ffi_op.rs: callback(user, bucket name) */
};

typedef struct bagua_bucket_op {
    int32_t kind;
    int32_t average;     /* centralized ops */
    int32_t compression; /* BAGUA_COMPRESSION_* (low-precision ops) */
    int32_t fused;       /* centralized low precision: 1 = fused / pipelined, 0 = the reference's sequence */
    BaguaSingleCommunicatorC* comm;
    bagua_tensor_t weight, left_peer_weight, right_peer_weight; /* decentralized op */
    void (*callback)(void* user, const char* bucket_name);     /* BAGUA_BUCKET_OP_CALLBACK */
    void* user;
    /* hierarchical mode when set: the node's communicator (comm = the internode one,
     * NULL on the node's workers), see bagua_*_hierarchical */
    BaguaSingleCommunicatorC* intranode;
} bagua_bucket_op_t;

/* NULL on error (*status says why): empty list, mixed dtype / device, allocated < num_elem */
BaguaBucketC* bagua_bucket_create(const char* name, const bagua_tensor_t* tensors, const char* const* tensor_names,
                                  int n, int* status);
void bagua_bucket_destroy(BaguaBucketC* bucket);
int bagua_bucket_append_op(BaguaBucketC* bucket, const bagua_bucket_op_t* op);
int bagua_bucket_clear_ops(BaguaBucketC* bucket);
int bagua_bucket_num_ops(BaguaBucketC* bucket);
/* readiness by tensor name (datatypes/mod.rs:793-813, 1256-1266); the event (0 = none)
 * is waited for by the stream of the bucket's next execution */
int bagua_bucket_mark_tensor_ready(BaguaBucketC* bucket, const char* tensor_name, uint64_t ready_event);
/* the same, and `current` (non-NULL) replaces the tensor's recorded descriptor: the
 * reference reads data_ptr / numel from the torch tensor at run time
 * (datatypes/mod.rs:775-791), so a storage swapped after the bucket was created is
 * followed.  dtype and device must not change (BAGUA_ERR_INVALID_ARG). */
int bagua_bucket_mark_tensor_ready_desc(BaguaBucketC* bucket, const char* tensor_name, uint64_t ready_event,
                                        const bagua_tensor_t* current);
int bagua_bucket_refresh_tensor(BaguaBucketC* bucket, const char* tensor_name, const bagua_tensor_t* current);
int bagua_bucket_ready_for_comm(BaguaBucketC* bucket);
int bagua_bucket_reset_comm_ready(BaguaBucketC* bucket);
/* run the bucket's ops now on its communication tensor (in place when the tensors are
 * back to back, else packed into a pool buffer and copied back, datatypes/mod.rs:963-1070).
 * `stream` (0 = the first op's communicator stream) carries the ready-event waits, the pack
 * and the copy-back; the ops run on their communicator's stream, ordered after the pack
 * and before the copy-back by events.  Synchronous (returns after both streams drained)
 * unless an op's communicator is async (bagua_comm_set_async): then it returns once the
 * work is queued. */
int bagua_bucket_execute(BaguaBucketC* bucket, uint64_t stream);

BaguaCommBackendC* bagua_comm_backend_create(size_t schedule_channel_cap, int device_id);
/* drains what is already scheduled, then stops the worker */
void bagua_comm_backend_destroy(BaguaCommBackendC* backend);
/* lib.rs:270-298: replaces the previous buckets; duplicate tensor names or pointers are
 * refused.  The buckets must outlive their registration. */
int bagua_comm_backend_register_ordered_buckets(BaguaCommBackendC* backend, BaguaBucketC* const* buckets, int n);
/* lib.rs:300-319 (the tensor by name) */
int bagua_comm_backend_mark_communication_ready(BaguaCommBackendC* backend, const char* tensor_name,
                                               uint64_t ready_event);
/* the same with the tensor's current descriptor (see bagua_bucket_mark_tensor_ready_desc);
 * a scheduled bucket runs with the descriptors it had when it was scheduled */
int bagua_comm_backend_mark_communication_ready_desc(BaguaCommBackendC* backend, const char* tensor_name,
                                                    uint64_t ready_event, const bagua_tensor_t* current);
/* lib.rs:321-337: *completed = ops waited for; returns the first failure's status */
int bagua_comm_backend_wait_pending_comm_ops(BaguaCommBackendC* backend, int* completed);
/* The monitor (lib.rs:255-265): an op whose work has not completed 300 s after the
 * worker picked it up (BAGUA_COMM_OP_TIMEOUT_S, or set_op_timeout_ms) is failed: its
 * message is kept, its communicators are aborted (bagua_comm_abort: ncclCommAbort
 * releases RCCL kernels waiting for an absent peer) and wait_pending_comm_ops
 * returns BAGUA_ERR_ABORTED instead of blocking.  The reference panics the process
 * instead (py/lib.rs:498-504).  failures = how many ops failed this way;
 * failure_message copies message i into buf (NUL-terminated, truncated to len) and
 * returns its full length, -1 when there is no message i. */
int bagua_comm_backend_failures(BaguaCommBackendC* backend);
/* Ops abandoned by wait_pending_comm_ops: aborted, and their worker call never
 * returned.  While any exists, the buffers those ops were given must stay alive (the
 * call may still touch them); destroy then leaves the worker and the backend behind
 * instead of joining a thread that never returns. */
int bagua_comm_backend_stuck(BaguaCommBackendC* backend);
int bagua_comm_backend_failure_message(BaguaCommBackendC* backend, int i, char* buf, size_t len);
int bagua_comm_backend_set_op_timeout_ms(BaguaCommBackendC* backend, int64_t ms);
/* Cross-bucket pipelining (no reference counterpart): bucket i of the registration
 * order runs on lane 1 + i % lanes of its communicator -- a view with its own
 * streams -- so consecutive buckets overlap on the GPU; 1 = every bucket on the
 * communicator's stream (the reference's one stream).  Default 3 (BAGUA_SCHED_LANES),
 * async schedulers only.  set_lanes first waits for everything scheduled;
 * bagua_comm_backend_lanes returns the lanes in effect. */
int bagua_comm_backend_set_lanes(BaguaCommBackendC* backend, int lanes);
int bagua_comm_backend_lanes(BaguaCommBackendC* backend);

#ifdef __cplusplus
}
#endif
#endif /* BAGUA_CORE_H */
