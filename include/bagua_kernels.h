/*
 * bagua_kernels.h — C ABI of the MI355X (gfx950) gradient-codec kernels.
 *
 * Drop-in replacement for the `extern "C"` block of the reference
 * (bagua-core-internal/kernels/bagua_kernels.cu:573-691), which the Rust host
 * binds in bagua-core-internal/src/kernels/mod.rs:3-137 with
 * `#[link(name = "bagua_kernels", kind = "static")]`.  Built as
 * libbagua_kernels.so / libbagua_kernels.a from bagua-core_amd/csrc/kernels.
 *
 * Streams are opaque pointers (`hipStream_t`, ABI-identical to the
 * reference's `cudaStream_t`; 0 = the null stream).  All calls are
 * asynchronous on that stream, never allocate, never synchronise.
 *
 * Two API levels:
 *  - v1: the reference's exact symbol names and signatures (void return).
 *    Errors print "Failed: ..." and exit(EXIT_FAILURE), the reference's
 *    CUDACHECK convention (bagua-core-internal/cpp/include/bagua_utils.h:5).
 *  - v2: `bagua_*` entry points returning a bagua_status_t, dtype-generic,
 *    plus the bf16 and 1-bit sign+scale extensions and fused kernels.
 *    v1 functions are thin wrappers over v2.
 */
#ifndef BAGUA_KERNELS_H
#define BAGUA_KERNELS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* bagua_stream_t; /* hipStream_t */
typedef uint16_t bagua_half_t; /* IEEE binary16 bits (reference `half`) */
typedef uint16_t bagua_bf16_t; /* bfloat16 bits (extension) */

/* dtype codes: reference BaguaTensorDtype F32/F16 (datatypes/mod.rs:40-47) + BF16 */
enum { BAGUA_DTYPE_F32 = 0, BAGUA_DTYPE_F16 = 1, BAGUA_DTYPE_BF16 = 2 };

typedef enum {
    BAGUA_OK = 0,
    BAGUA_ERR_INVALID_ARG = 1,  /* sizes / chunking / target out of range */
    BAGUA_ERR_WORKSPACE = 2,    /* temp buffer too small */
    BAGUA_ERR_HIP = 3,          /* kernel launch failed (see bagua_last_hip_error) */
    BAGUA_ERR_UNSUPPORTED = 4   /* dtype not supported by this entry point */
} bagua_status_t;

const char* bagua_status_string(int status);
int bagua_last_hip_error(void);
/* Measurement hook: the next kernel this library launches on the calling thread
 * records the two hipEvent_t (created with timing) at its own start and end
 * (hipExtLaunchKernel), so hipEventElapsedTime gives the kernel's duration
 * without dispatch overhead.  Both NULL disarms.  One-shot. */
int bagua_time_next_kernel(void* start_event, void* stop_event);
/* The same for the next n (<= 32) kernels this library launches on the calling
 * thread, one event pair each in launch order (e.g. every kernel of one comm op);
 * n = 0 disarms.  bagua_timed_kernels: how many of the armed pairs were used;
 * bagua_timed_kernel_name: the i-th timed kernel's name ("minmax_quantize_kernel"). */
int bagua_time_next_kernels(void* const* start_events, void* const* stop_events, int n);
int bagua_timed_kernels(void);
int bagua_timed_kernel_name(int i, char* buf, size_t len);

/* ======================================================================== */
/* v2 — MinMax-UInt8 codec (format: datatypes/mod.rs:669-704, K:455-500)     */
/* ======================================================================== */
/* Compressed bytes S = align32(chunk_size*num_chunks) + align32(2*sizeof T)*num_chunks
 * (replaces MinMaxUInt8CompressionParameters::get_compressed_buffer_size, datatypes/mod.rs:669). */
size_t bagua_minmax_u8_compressed_bytes(int dtype, int chunk_size, int num_chunks);
/* Workspace for bagua_minmax_u8_compress (replaces the cub temp-size query, K:268-310). */
size_t bagua_minmax_u8_workspace_bytes(int chunk_size, int num_chunks);
/* compress_{f32,f16}_to_uint8_host (K:661-676): per-chunk min/max header + uint8 payload.
 * target_chunk = -1 compresses all chunks, otherwise only chunk `target_chunk`.
 * `input` must hold num_chunks*chunk_size elements: as in the reference
 * (K:468-472, K:538-545), elements at or past input_num_element are left out of
 * the chunk's min/max but still quantised with its parameters. */
int bagua_minmax_u8_compress(int dtype, const void* input, int input_num_element, int chunk_size,
                             int num_chunks, uint8_t* output, size_t output_bytes, void* workspace,
                             size_t workspace_bytes, int target_chunk, bagua_stream_t stream);
/* The two passes of bagua_minmax_u8_compress launched separately (stage 1:
 * per-workgroup min/max partials into `workspace`; stage 2: fold partials,
 * header, quantise).  Same arguments in both calls; used for per-kernel
 * timing and for overlapping the passes with other work.  Stage 5 is stage 1
 * sweeping each chunk from its end to its start (same partials), so that the
 * chunks' beginnings are what the Infinity Cache holds afterwards. */
int bagua_minmax_u8_compress_stage(int stage, int dtype, const void* input, int input_num_element,
                                   int chunk_size, int num_chunks, uint8_t* output, size_t output_bytes,
                                   void* workspace, size_t workspace_bytes, int target_chunk,
                                   bagua_stream_t stream);
/* 1 when bagua_minmax_u8_compress would take the one-launch encode for these
 * arguments on this stream (whole, fully valid chunks of >= 4 Mi elements in
 * total, vector-alignable payloads), 0 when it runs the
 * two-pass encode.  Measurement and tests only; no launch. */
int bagua_minmax_u8_resident_path(int dtype, const void* input, int input_num_element, int chunk_size,
                                  int num_chunks, uint8_t* output, size_t output_bytes, int target_chunk,
                                  bagua_stream_t stream);
/* Measurement hook: while set, every one-launch encode writes wall_clock64
 * stamps into `device_buffer` (>= 8 * CU count u64), 8 slots per workgroup:
 * start, end of pass 1, exchange done, end of pass 2, end of the streamed
 * part of pass 2, end of its LDS part.  NULL disarms. */
int bagua_minmax_u8_resident_trace(void* device_buffer);
/* The one-launch encode keeps a small device slot per stream (its ticket
 * counter and min/max exchange granules; 64 per device).  hipStreamPerThread
 * gets one slot per calling host thread.  Release drops the stream's slot once
 * every workgroup launched on it has passed the min/max exchange (a device
 * counter read on a private stream: no other stream is synchronised); when all
 * slots are owned, the least recently used one is reclaimed the same way. */
int bagua_minmax_u8_release_stream(bagua_stream_t stream);
/* allowed = 0: compress calls on `stream` always take the two-pass encode (a stream
 * that runs codec work beside another codec stream, e.g. the scheduler's lanes);
 * 1 (the default) restores the one-launch encode.  Releasing the stream resets it. */
int bagua_minmax_u8_set_stream_resident(bagua_stream_t stream, int allowed);
/* Streams currently holding a slot on `device_id` (tests and diagnostics). */
int bagua_minmax_u8_resident_slots_in_use(int device_id);
/* measurement: how many workgroups of `stream`'s one-launch encodes timed out waiting
 * for their chunk's partials (contention with other streams' kernels) and re-read the
 * missing slices instead.  Synchronises `stream`. */
int bagua_minmax_u8_resident_give_ups(bagua_stream_t stream, uint64_t* count);
/* decompress_uint8_to_{f32,f16}_host (K:667-681) */
int bagua_minmax_u8_decompress(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                               int num_chunks, void* output, bagua_stream_t stream);

/* ======================================================================== */
/* v2 — 1-bit sign + scale codec (extension; format in DESIGN.md §4)         */
/* ======================================================================== */
size_t bagua_onebit_compressed_bytes(int chunk_size, int num_chunks);
size_t bagua_onebit_workspace_bytes(int chunk_size, int num_chunks);
int bagua_onebit_compress(int dtype, const void* input, int input_num_element, int chunk_size,
                          int num_chunks, uint8_t* output, size_t output_bytes, void* workspace,
                          size_t workspace_bytes, int target_chunk, bagua_stream_t stream);
int bagua_onebit_decompress(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                            int num_chunks, void* output, bagua_stream_t stream);
/* Pieced 1-bit codec (the pipelined centralized op): a chunk's 1024-element
 * tiles split into `pieces` tile ranges (bagua_onebit_piece_range; trailing
 * ranges may be empty).  bagua_onebit_encode_range writes the sign bits and
 * |x| tile partials (workspace) of tiles [tile_begin, tile_end) of EVERY chunk
 * and no header; once every range is encoded, bagua_onebit_finalize writes the
 * headers (scale, count) and slack from the partials: together exactly the
 * bytes of bagua_onebit_compress (target -1).  bagua_onebit_decompress_range
 * decodes tiles [tile_begin, tile_end) of every chunk (headers present). */
int bagua_onebit_piece_range(int chunk_size, int pieces, int piece, int* tile_begin, int* tile_end);
int bagua_onebit_encode_range(int dtype, const void* input, int input_num_element, int chunk_size, int num_chunks,
                              uint8_t* output, size_t output_bytes, void* workspace, size_t workspace_bytes,
                              int tile_begin, int tile_end, bagua_stream_t stream);
int bagua_onebit_finalize(const void* workspace, size_t workspace_bytes, int input_num_element, int chunk_size,
                          int num_chunks, uint8_t* output, size_t output_bytes, bagua_stream_t stream);
int bagua_onebit_decompress_range(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                  int num_chunks, void* output, int tile_begin, int tile_end, bagua_stream_t stream);
/* Middle step of the centralized op with the 1-bit codec, fused: decode the
 * num_chunks received segments of `input`, reduce them into chunk
 * `target_chunk` of `tensor` in the reference's summation order (mean if
 * `average`), and encode that chunk into segment `target_chunk` of `output`.
 * Equal to bagua_onebit_decompress + bagua_reduce_chunks + bagua_onebit_compress
 * (target) on a fully valid tensor.  BAGUA_ERR_UNSUPPORTED for num_chunks > 16.
 * `tensor` may be NULL: the reduced chunk is then only encoded, not stored
 * (the centralized op overwrites it with its final decompress anyway). */
int bagua_onebit_reduce_requantize(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                   int num_chunks, void* tensor, int average, uint8_t* output, size_t output_bytes,
                                   int target_chunk, void* workspace, size_t workspace_bytes, bagua_stream_t stream);

/* ======================================================================== */
/* v2 — chunk reduction and elementwise ops                                  */
/* ======================================================================== */
/* reduce_{mean,sum}_{f32,f16}_inplace_host (K:646-660): chunk target_chunk =
 * sum (or mean) of the num_chunks chunks, in the reference's summation order. */
int bagua_reduce_chunks(int dtype, void* input, int chunk_size, int num_chunks, int target_chunk,
                        int average, bagua_stream_t stream);
/* Fused dequantise(num_chunks MinMax-UInt8 segments) + reduce into `output`
 * (chunk_size elements), bit-identical to decompress + reduce_{mean,sum}. */
int bagua_minmax_u8_decompress_reduce(int dtype, const uint8_t* input, size_t input_bytes,
                                      int chunk_size, int num_chunks, void* output, int average,
                                      bagua_stream_t stream);

/* Middle step of the compressed centralized all-reduce
 * (centralized_low_precision_synchronous.rs:40-60: decompress_from ->
 * reduce_{mean,sum}_inplace(target) -> compress(target)) as two kernels:
 * dequantise the num_chunks received segments of `input` and reduce them into
 * chunk `target_chunk` of `tensor` (num_chunks*chunk_size elements), then
 * requantise that chunk into segment `target_chunk` of `output` (a
 * num_chunks-segment MinMax-UInt8 buffer of output_bytes).  Bit-identical to
 * the unfused sequence.  Returns BAGUA_ERR_UNSUPPORTED when the shape has no
 * vector path (num_chunks > 16 or misaligned); callers then run the unfused ops.
 * `tensor` may be NULL: the reduced chunk is then not stored (the centralized
 * op overwrites it with its final decompress anyway); a partials-only pass is
 * followed by a requantise that recomputes the reduced values from `input`
 * (same bytes; 2*num_chunks*chunk_size payload bytes read instead of
 * num_chunks*chunk_size + 2*chunk_size*sizeof(T) moved, so it pays for
 * num_chunks < 2*sizeof(T)). */
int bagua_minmax_u8_reduce_requantize(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                      int num_chunks, void* tensor, int average, uint8_t* output,
                                      size_t output_bytes, int target_chunk, void* workspace,
                                      size_t workspace_bytes, bagua_stream_t stream);
/* The same middle step (reduced chunk recomputed, never stored) with the op's
 * final decompress of the own chunk fused in: chunk `target_chunk` of `tensor`
 * receives the decompressed requantised values -- exactly what
 * bagua_minmax_u8_decompress of `output` writes there.  For one rank
 * (num_chunks = 1) this is the op's whole tail: the final decompress launch is
 * saved.  `tensor` must be 16-B aligned at the chunk (else UNSUPPORTED).
 * `output` may be NULL (output_bytes is then ignored): the requantised segment
 * is not stored -- one rank gathers nothing, so nothing would read it. */
int bagua_minmax_u8_reduce_requantize_final(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                            int num_chunks, void* tensor, int average, uint8_t* output,
                                            size_t output_bytes, int target_chunk, void* workspace,
                                            size_t workspace_bytes, bagua_stream_t stream);

/* The whole compressed centralized op at ONE rank
 * (centralized_low_precision_synchronous.rs:30-71 with num_chunks = 1), in place:
 * tensor <- decompress(compress(reduce(decompress(compress(tensor))))), two kernels
 * (the min/max pass, then one pass whose output is a 256-entry table of the first
 * quantised byte; the second header follows from the first).
 * Bit-identical to the op's sequence; every element valid (num_elem elements). */
int bagua_minmax_u8_centralized_one_rank(int dtype, void* tensor, int num_elem, int average, void* workspace,
                                         size_t workspace_bytes, bagua_stream_t stream);

/* The same for the 1-bit codec (this repository's extension): at one
 * rank the fused middle step's table has two entries (the reduced value of a 0 and
 * of a 1 sign bit, equal in magnitude), so the op is the encode pass (sign bits +
 * |x| tile partials), one workgroup deriving the first scale, the two reduced values
 * and the second scale through the encoder's fixed tree, and one pass writing
 * +-scale2 from the bits.  Bit-identical to the op's sequence; every element valid.
 * Workspace: bagua_onebit_one_rank_workspace_bytes(num_elem), 16-B aligned. */
size_t bagua_onebit_one_rank_workspace_bytes(int num_elem);
int bagua_onebit_centralized_one_rank(int dtype, void* tensor, int num_elem, int average, void* workspace,
                                      size_t workspace_bytes, bagua_stream_t stream);

/* Pipelined all-reduce building blocks (no reference counterpart: the same
 * kernels restricted to part of every chunk, so communication of one piece
 * overlaps the codec work of the next).  A chunk splits into `pieces` element
 * ranges (bagua_minmax_u8_piece_range; trailing ranges may be empty).  Each
 * segment keeps ONE header for the whole chunk, so the pieced sequence writes
 * exactly the bytes of the unpieced one:
 *   stage 1 of bagua_minmax_u8_compress_stage (all chunks), then
 *   bagua_minmax_u8_quantize_range per piece (the range at 0 writes headers);
 *   bagua_minmax_u8_reduce_piece per piece (fused dequantise + reduce of the
 *   target chunk; min/max partials to the piece's workspace slot), then
 *   bagua_minmax_u8_requantize_pieces (folds every slot), or
 *   bagua_minmax_u8_requantize_piece per piece (each folds every slot; the
 *   allgather of piece q can start once piece q is requantised);
 *   bagua_minmax_u8_decompress_range per piece (needs the headers present).
 * `pieces` is a piece schedule: the count (1..0xFFFF), optionally OR-ed with
 * BAGUA_PIECES_TAPERED -- from 3 pieces on the first and the last piece are then
 * half the size of the others.  Every call of one op must pass the same schedule. */
#define BAGUA_PIECES_COUNT_MASK 0xFFFF
#define BAGUA_PIECES_TAPERED 0x10000
/* decentralized ring op only: the relayed (multipath) exchange from 6 ranks on
 * (the reference's direct exchange otherwise); ignored by the piece functions */
#define BAGUA_PIECES_MULTIPATH 0x20000
/* requantise calls only: every piece's min/max partials were already folded into one
 * (bagua_minmax_u8_fold_piece_partials), so each requantise workgroup reads one value */
#define BAGUA_PIECES_FOLDED 0x40000
/* reduce / requantise piece calls of one op: bagua_minmax_u8_reduce_piece(piece 0) leaves
 * the p x 256 dequantisation tables in the workspace; with this bit the later pieces and
 * bagua_minmax_u8_reduce_requantize_piece copy them instead of recomputing them (piece 0
 * must have run first on the same workspace and received segments) */
#define BAGUA_PIECES_TABLES 0x80000
int bagua_minmax_u8_piece_range(int chunk_size, int pieces, int piece, int* begin, int* end);
size_t bagua_minmax_u8_pipeline_workspace_bytes(int chunk_size, int pieces);
int bagua_minmax_u8_quantize_range(int dtype, const void* input, int input_num_element, int chunk_size,
                                   int num_chunks, uint8_t* output, size_t output_bytes, void* workspace,
                                   size_t workspace_bytes, int target_chunk, int elem_begin, int elem_end,
                                   bagua_stream_t stream);
int bagua_minmax_u8_decompress_range(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                     int num_chunks, void* output, int elem_begin, int elem_end,
                                     bagua_stream_t stream);
int bagua_minmax_u8_reduce_piece(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size, int num_chunks,
                                 void* tensor, int average, int target_chunk, int pieces, int piece, void* workspace,
                                 size_t workspace_bytes, bagua_stream_t stream);
int bagua_minmax_u8_requantize_pieces(int dtype, const void* tensor, int chunk_size, int num_chunks, uint8_t* output,
                                      size_t output_bytes, int target_chunk, int pieces, const void* workspace,
                                      size_t workspace_bytes, bagua_stream_t stream);
int bagua_minmax_u8_requantize_piece(int dtype, const void* tensor, int chunk_size, int num_chunks, uint8_t* output,
                                     size_t output_bytes, int target_chunk, int pieces, int piece,
                                     const void* workspace, size_t workspace_bytes, bagua_stream_t stream);
/* The same pipeline without storing the reduced chunk: bagua_minmax_u8_reduce_piece
 * with tensor == NULL emits each piece's min/max partials only, and
 * bagua_minmax_u8_reduce_requantize_piece recomputes piece `piece` of the reduced
 * target chunk from the p received segments (`input`, as reduce_piece read them:
 * same tables, same summation tree, so the same values bit for bit), folds every
 * piece's partials and quantises it into segment target_chunk of `output` (the
 * range at 0 writes the header, the one ending at chunk_size the slack).  The
 * tensor is left untouched.  BAGUA_ERR_UNSUPPORTED for num_chunks > 16 or
 * misaligned segments (use the storing pair). */
int bagua_minmax_u8_reduce_requantize_piece(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                            int num_chunks, int average, uint8_t* output, size_t output_bytes,
                                            int target_chunk, int pieces, int piece, const void* workspace,
                                            size_t workspace_bytes, bagua_stream_t stream);
/* Fold every piece's min/max partials (written by bagua_minmax_u8_reduce_piece) into one
 * value in the workspace, after the last reduce piece; the requantise calls that follow
 * pass `pieces | BAGUA_PIECES_FOLDED` and read that one value instead of folding
 * pieces x workgroups partials in every workgroup. */
int bagua_minmax_u8_fold_piece_partials(int dtype, int chunk_size, int pieces, void* workspace, size_t workspace_bytes,
                                        bagua_stream_t stream);

/* Decentralized ring op (decentralized_low_precision_synchronous.rs:45-64,126-151)
 * as two fused passes around the MinMax quantise pass, bit-identical to the
 * reference's elementwise sequence (every intermediate rounded to T where the
 * reference stores it):
 *   bagua_ring_mix_minmax: tensor = ((tensor + L/3) + R/3) + W*(-5/3), each an
 *     addmul as bagua_addmul_inplace computes it, and the min/max partials of the
 *     result into `workspace` exactly as stage 1 of bagua_minmax_u8_compress_stage
 *     (n_chunks = 1, same workspace_bytes) would; follow with stage 2.
 *   bagua_ring_apply_minmax: L += dq(from_left); R += dq(from_right);
 *     tensor = dq(mine) + W; W = tensor (n_chunks = 1 MinMax buffers).
 * Both return BAGUA_ERR_UNSUPPORTED for tensors not 16-B aligned (callers run the
 * elementwise sequence). */
int bagua_ring_mix_minmax(int dtype, void* tensor, const void* left, const void* right, const void* weight,
                          int num_elem, void* workspace, size_t workspace_bytes, bagua_stream_t stream);
int bagua_ring_apply_minmax(int dtype, const uint8_t* mine, const uint8_t* from_left, const uint8_t* from_right,
                            size_t compressed_bytes, int num_elem, void* tensor, void* weight, void* left,
                            void* right, bagua_stream_t stream);
/* The same on elements [elem_begin, elem_end) only (the pipelined op applies each
 * piece as it arrives; elem_begin and elem_end multiples of 16 / sizeof(T), or
 * elem_end = num_elem; the headers of all three buffers must be present). */
int bagua_ring_apply_minmax_range(int dtype, const uint8_t* mine, const uint8_t* from_left, const uint8_t* from_right,
                                  size_t compressed_bytes, int num_elem, int elem_begin, int elem_end, void* tensor,
                                  void* weight, void* left, void* right, bagua_stream_t stream);
/* The whole ring op at one rank (its own left and right peer, so both peers' payloads
 * are its own bytes): the mix pass, then one pass that folds the mix's min/max
 * partials into the header and applies L += d, R += d, tensor = d + W, W = tensor with
 * d = dq(q(mixed)) per element, writing no payload.  Bit-identical to mix + stage 2 +
 * bagua_ring_apply_minmax(mine, mine, mine); the same workspace as
 * bagua_ring_mix_minmax; BAGUA_ERR_UNSUPPORTED for tensors not 16-B aligned. */
int bagua_ring_one_rank_minmax(int dtype, void* tensor, void* weight, void* left, void* right, int num_elem,
                               void* workspace, size_t workspace_bytes, bagua_stream_t stream);

/* K:196-266 elementwise kernels, dtype-generic (f32, f16, bf16) */
int bagua_add_inplace(int dtype, void* x, const void* y, int n, bagua_stream_t stream);
int bagua_addmul_inplace(int dtype, void* x, const void* y, int n, float factor, bagua_stream_t stream);
int bagua_substract_inplace(int dtype, void* x, const void* y, int n, bagua_stream_t stream);
int bagua_average_inplace(int dtype, void* x, const void* y, int n, bagua_stream_t stream);
int bagua_divide_inplace(int dtype, void* x, float d, int n, bagua_stream_t stream);

/* ======================================================================== */
/* v1 — the reference's extern "C" surface (K:573-691), same names/ABI       */
/* ======================================================================== */
void divide_inplace_f32_host(float* x, float D_, int N, bagua_stream_t stream);
void divide_inplace_f16_host(bagua_half_t* x, float D_, int N, bagua_stream_t stream);
void add_inplace_f32_host(float* x, float* y, int N, bagua_stream_t stream);
void add_inplace_f16_host(bagua_half_t* x, bagua_half_t* y, int N, bagua_stream_t stream);
void addmul_inplace_f32_host(float* x, float* y, int N, const float factor, bagua_stream_t stream);
void addmul_inplace_f16_host(bagua_half_t* x, bagua_half_t* y, int N, const float factor,
                             bagua_stream_t stream);
void substract_inplace_f32_host(float* x, float* y, int N, bagua_stream_t stream);
void substract_inplace_f16_host(bagua_half_t* x, bagua_half_t* y, int N, bagua_stream_t stream);
void average_inplace_f32_host(float* x, float* y, int N, bagua_stream_t stream);
void average_inplace_f16_host(bagua_half_t* x, bagua_half_t* y, int N, bagua_stream_t stream);
void async_model_average_host(float* tensor, const float* reduced_tensor_copy,
                              const float* tensor_copy, const float nranks, const int N,
                              bagua_stream_t stream);
void reduce_mean_f32_inplace_host(float* input, int chunk_size, int num_chunks, int target_chunk,
                                  bagua_stream_t stream);
void reduce_mean_f16_inplace_host(bagua_half_t* input, int chunk_size, int num_chunks,
                                  int target_chunk, bagua_stream_t stream);
void reduce_sum_f32_inplace_host(float* input, int chunk_size, int num_chunks, int target_chunk,
                                 bagua_stream_t stream);
void reduce_sum_f16_inplace_host(bagua_half_t* input, int chunk_size, int num_chunks,
                                 int target_chunk, bagua_stream_t stream);
void compress_f32_to_uint8_host(float* input, int input_num_element, int chunk_size,
                                int num_chunks, uint8_t* output, size_t output_size,
                                void* dev_buffer, size_t dev_size, int target_chunk,
                                bagua_stream_t stream);
void decompress_uint8_to_f32_host(uint8_t* input, size_t input_size, int chunk_size,
                                  int num_chunks, float* output, bagua_stream_t stream);
void compress_f16_to_uint8_host(bagua_half_t* input, int input_num_element, int chunk_size,
                                int num_chunks, uint8_t* output, size_t output_size,
                                void* dev_buffer, size_t dev_size, int target_chunk,
                                bagua_stream_t stream);
void decompress_uint8_to_f16_host(uint8_t* input, size_t input_size, int chunk_size,
                                  int num_chunks, bagua_half_t* output, bagua_stream_t stream);
size_t array_min_max_size_f32_host(float* input, int input_num_element, float* output,
                                   bagua_stream_t stream);
size_t array_min_max_size_f16_host(bagua_half_t* input, int input_num_element,
                                   bagua_half_t* output, bagua_stream_t stream);

/* v1-style extensions (same conventions as the v1 block) */
void compress_bf16_to_uint8_host(bagua_bf16_t* input, int input_num_element, int chunk_size,
                                 int num_chunks, uint8_t* output, size_t output_size,
                                 void* dev_buffer, size_t dev_size, int target_chunk,
                                 bagua_stream_t stream);
void decompress_uint8_to_bf16_host(uint8_t* input, size_t input_size, int chunk_size,
                                   int num_chunks, bagua_bf16_t* output, bagua_stream_t stream);
size_t array_min_max_size_bf16_host(bagua_bf16_t* input, int input_num_element,
                                    bagua_bf16_t* output, bagua_stream_t stream);
void reduce_mean_bf16_inplace_host(bagua_bf16_t* input, int chunk_size, int num_chunks,
                                   int target_chunk, bagua_stream_t stream);
void reduce_sum_bf16_inplace_host(bagua_bf16_t* input, int chunk_size, int num_chunks,
                                  int target_chunk, bagua_stream_t stream);
void add_inplace_bf16_host(bagua_bf16_t* x, bagua_bf16_t* y, int N, bagua_stream_t stream);
void addmul_inplace_bf16_host(bagua_bf16_t* x, bagua_bf16_t* y, int N, const float factor,
                              bagua_stream_t stream);
void compress_f32_to_onebit_host(float* input, int input_num_element, int chunk_size,
                                 int num_chunks, uint8_t* output, size_t output_size,
                                 void* dev_buffer, size_t dev_size, int target_chunk,
                                 bagua_stream_t stream);
void decompress_onebit_to_f32_host(uint8_t* input, size_t input_size, int chunk_size,
                                   int num_chunks, float* output, bagua_stream_t stream);
void compress_bf16_to_onebit_host(bagua_bf16_t* input, int input_num_element, int chunk_size,
                                  int num_chunks, uint8_t* output, size_t output_size,
                                  void* dev_buffer, size_t dev_size, int target_chunk,
                                  bagua_stream_t stream);
void decompress_onebit_to_bf16_host(uint8_t* input, size_t input_size, int chunk_size,
                                    int num_chunks, bagua_bf16_t* output, bagua_stream_t stream);
size_t onebit_temp_size_host(int chunk_size, int num_chunks);

#ifdef __cplusplus
}
#endif
#endif /* BAGUA_KERNELS_H */
