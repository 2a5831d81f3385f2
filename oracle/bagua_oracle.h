/*
 * bagua_oracle.h — CPU restatement of the bagua-core gradient-codec hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product path (bagua-core_amd/csrc).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product never links it.
 *
 * Every function cites the reference file:line it restates; paths are
 * relative to the reference repository root (BaguaSys/bagua-core):
 *   K   = bagua-core-internal/kernels/bagua_kernels.cu
 *   DT  = bagua-core-internal/src/datatypes/mod.rs
 *   CUB = bagua-core-internal/third_party/cub-1.8.0/cub
 *
 * PARITY UNPINNED: the reference ships no golden vectors, KATs or tests for
 * this path and cannot be built or imported here (F5), so no
 * reference output pins this restatement.  It rests on (1) source reading
 * with line citations, and (2) an independently written numpy restatement
 * (oracle/oracle_np.py) that must agree with it bit-for-bit on every
 * committed fixture (tests/golden/).
 * bf16 (F2) and the 1-bit sign+scale codec (F1) have no reference
 * counterpart: their formats are defined by this repository and
 * are "parity unpinned" with respect to the reference.
 */
#ifndef BAGUA_ORACLE_H
#define BAGUA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* dtype codes (DT:40-47 BaguaTensorDtype F32/F16; BF16 is an extension) */
enum { ORC_F32 = 0, ORC_F16 = 1, ORC_BF16 = 2 };

/* scalar conversions (exposed so tests can pin them against numpy) */
float orc_half_to_float(uint16_t h);
uint16_t orc_float_to_half(float f);
float orc_bf16_to_float(uint16_t b);
uint16_t orc_float_to_bf16(float f);

/* DT:669-704 MinMaxUInt8CompressionParameters::get_compressed_buffer_size */
size_t orc_minmax_compressed_size(int n_chunks, size_t chunk_size, int dtype);

/* K:312-371 array_min_max via cub::DeviceReduce::Min/Max (init = +-T_MAX). */
void orc_minmax(const void* in, int dtype, int64_t n, float* out_min, float* out_max);

/* K:533-560 compress_float_to_uint8_host + K:455-479 kernel. Returns 0 / <0 error. */
int orc_compress_minmax_u8(const void* in, int dtype, int in_num_elem, int chunk_size,
                           int num_chunks, uint8_t* out, size_t out_bytes, int target_chunk);

/* K:562-571 decompress_uint8_to_float_host + K:481-500 kernel. */
int orc_decompress_minmax_u8(const uint8_t* in, size_t in_bytes, int chunk_size,
                             int num_chunks, void* out, int dtype);

/* K:373-400 reduce_chunk_inplace, K:171-194 block_y_reduce, K:502-531 launch table. */
int orc_reduce_chunks(void* inout, int dtype, int chunk_size, int num_chunks,
                      int target_chunk, int average);

/* K:220-242 add_inplace / addmul_inplace (x += y, x += y*factor). */
void orc_add_inplace(void* x, const void* y, int dtype, int64_t n);
void orc_addmul_inplace(void* x, const void* y, int dtype, int64_t n, float factor);

/* 1-bit sign+scale codec — format defined by this repository. */
size_t orc_onebit_compressed_size(int n_chunks, size_t chunk_size);
float orc_onebit_tree_sum(const float* v, int64_t n);
int orc_compress_onebit(const void* in, int dtype, int in_num_elem, int chunk_size,
                        int num_chunks, uint8_t* out, size_t out_bytes, int target_chunk);
int orc_decompress_onebit(const uint8_t* in, size_t in_bytes, int chunk_size,
                          int num_chunks, void* out, int dtype);

/* number of OpenMP threads the oracle runs with (1 when built without OpenMP) */
int orc_num_threads(void);
int orc_set_num_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
