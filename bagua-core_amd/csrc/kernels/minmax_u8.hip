// minmax_u8.hip — MinMax-UInt8 gradient codec for gfx950 (MI355X).
//
// Replaces the reference's per-chunk cub::DeviceReduce::Min + ::Max passes
// (bagua_kernels.cu:312-371, 2p serial launches) and the scalar
// compress/decompress kernels (bagua_kernels.cu:455-500, 4-byte loads /
// 1-byte stores, 1024-thread blocks) with three streaming kernels:
//
//   minmax_partials  : one read of the chunk, 16-B loads, fused min AND max,
//                      wave64 shuffles + LDS, one partial per workgroup
//   minmax_quantize  : folds the partials (L2-resident, tiny), writes the
//                      header, quantises with 16-B loads / 4-B or 8-B stores;
//                      sweeps the chunk in REVERSE so the tail the previous
//                      kernel just streamed is re-read from the 256 MiB
//                      Infinity Cache first
//   minmax_dequantize: 4/8-B loads, 16-B stores
//
// Payload bytes and header values are bit-identical to the reference
// expressions (see codec_common.hpp); NaN / signed-zero handling of the
// min/max is pinned order-independently.
#include <stdio.h>
#include <stdlib.h>

#include "codec_common.hpp"
#include "launch_util.hpp"

#include <type_traits>

namespace bagua {

constexpr int kVecPerBlockTile = kBlock * kSubtiles;  // 1024 x 16-B vectors = 16 KiB in flight per block
// Launch shapes picked on MI355X with tools/stream_probe.hip:
// the read-only min/max pass wants 8 vectors in flight per lane on 4 blocks
// per CU; quantise and dequantise 4 per lane.  Round 3 (tools/grid_sweep.py,
// profiles/r03_grid_sweep.jsonl): more, shorter workgroups let the dispatcher
// balance the tail -- dequantise one tile per workgroup (16384 for 256 MiB f32:
// 48.25 -> 47.75 us), quantise 32 per CU (51.0 -> 50.1 us).  Round 4 keeps the
// dequantise at one tile per workgroup up to 1 GiB (65536: 214 -> 189.5 us per 1 GiB
// decode, 256 MiB unchanged; 8192 stays best for the quantise;
// profiles/r04_minmax_grid_sweep.jsonl).
constexpr int kPartialsSub = 8;
constexpr int kPartialsBlocks = 1024;
constexpr int kQuantBlocks = 8192;
constexpr int kDequantBlocks = 65536;
// the one-rank op's table pass (read + write, like the dequantise)
constexpr int kOneRankBlocks = 16384;  // 1 GiB op 0.524 -> 0.521 ms (profiles/r04_one_rank_grid_sweep.jsonl)
// the Infinity Cache: min/max passes over larger buckets read non-temporally except
// for the part the next kernel re-reads first (partials_nt, one_rank_impl)
constexpr int kPartialsNtAboveMiB = 256;

__device__ __forceinline__ int64_t chunk_valid(int64_t in_num_elem, int64_t cs, int c) {
    // K:538-545: remaining elements, clamped to [0, chunk_size]
    int64_t r = in_num_elem - (int64_t)c * cs;
    return r < 0 ? 0 : (r < cs ? r : cs);
}

template <typename T>
__device__ __forceinline__ void fold(float f, uint32_t& lo, uint32_t& hi) {
    const int32_t k = f2key(f);
    lo = min(lo, min_space_key(k));
    hi = min(hi, max_space_key(k));
}

// ------------------------------------------------------------------------
// pass 1: per-workgroup partial min/max of each active chunk
// ------------------------------------------------------------------------
// REV: the grid sweeps each chunk from its end to its start (min/max is
// order-free), so what the Infinity Cache holds afterwards is the chunk's
// beginning -- the piece the pipelined op quantises first
// NTL: non-temporal loads (no Infinity-Cache allocation; faster for a bucket larger
// than the cache, tools/stream_probe.hip at 1 GiB: 6.7-6.8 vs 6.1-6.2 TB/s) for the
// first `nt_until` vectors of each chunk's sweep; the tiles swept after them load with
// the default policy, so the Infinity Cache keeps them for a pass that re-reads them
// first (the sweep's end: a chunk's tail going forward, its beginning with REV)
template <typename T, bool REV = false, bool NTL = false>
__global__ __launch_bounds__(kBlock) void minmax_partials_kernel(
    const typename T::storage* __restrict__ in, int64_t in_num_elem, int64_t cs, int target,
    uint2* __restrict__ partials, int64_t nt_until) {
    using S = typename T::storage;
    constexpr int N = Vec<T>::N;
    const int c = target < 0 ? (int)blockIdx.y : target;
    const int64_t n = chunk_valid(in_num_elem, cs, c);
    const S* src = in + (int64_t)c * cs;

    // body starts on a 128-B line (head elements go to the scalar path)
    int64_t j0 = (int64_t)(((128u - ((uintptr_t)src & 127u)) & 127u) / sizeof(S));
    if (((uintptr_t)src % sizeof(S)) != 0) j0 = n;  // misaligned element pointer: all scalar
    if (j0 > n) j0 = n;
    const int64_t nvec = (n - j0) / N;
    const uint4* __restrict__ vsrc = reinterpret_cast<const uint4*>(src + j0);

    uint32_t lo = min_space(T::init_max());
    uint32_t hi = max_space(-T::init_max());
    constexpr int SUB = kPartialsSub;
    const int64_t stride = (int64_t)gridDim.x * kBlock * SUB;
    const int64_t ntile = (nvec + kBlock * SUB - 1) / (kBlock * SUB);
    for (int64_t fwd = (int64_t)blockIdx.x * kBlock * SUB; fwd < nvec; fwd += stride) {
        const int64_t base = REV ? (ntile - 1) * kBlock * SUB - fwd : fwd;
        if (base + kBlock * SUB <= nvec) {  // full tile: SUB loads in flight per lane
            uint4 r[SUB];
            if (NTL && fwd + kBlock * SUB <= nt_until) {
#pragma unroll
                for (int k = 0; k < SUB; ++k) r[k] = nt_load16(&vsrc[base + k * kBlock + threadIdx.x]);
            } else {
#pragma unroll
                for (int k = 0; k < SUB; ++k) r[k] = vsrc[base + k * kBlock + threadIdx.x];  // default policy
            }
#pragma unroll
            for (int k = 0; k < SUB; ++k) {
                float f[N];
                unpack16<T>(r[k], f);
#pragma unroll
                for (int i = 0; i < N; ++i) fold<T>(f[i], lo, hi);
            }
            continue;
        }
        for (int k = 0; k < SUB; ++k) {
            const int64_t v = base + k * kBlock + threadIdx.x;
            if (v >= nvec) continue;
            float f[N];
            unpack16<T>(vsrc[v], f);
#pragma unroll
            for (int i = 0; i < N; ++i) fold<T>(f[i], lo, hi);
        }
    }
    if (blockIdx.x == 0) {  // head before the first line and the ragged tail, scalar
        for (int64_t j = threadIdx.x; j < j0; j += kBlock) fold<T>(T::to_f(src[j]), lo, hi);
        for (int64_t j = j0 + nvec * N + threadIdx.x; j < n; j += kBlock) fold<T>(T::to_f(src[j]), lo, hi);
    }

    lo = wave_umin(lo);
    hi = wave_umin(hi);
    __shared__ uint32_t red[2][kWavesPerBlock];
    const int w = threadIdx.x / kWave;
    if (lane_id() == 0) { red[0][w] = lo; red[1][w] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 1; i < kWavesPerBlock; ++i) { lo = min(lo, red[0][i]); hi = min(hi, red[1][i]); }
        partials[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = make_uint2(lo, hi);
    }
}

// ------------------------------------------------------------------------
// pass 2: fold partials, write header, quantise
// ------------------------------------------------------------------------
template <typename T, bool kReverse>
__global__ __launch_bounds__(kBlock) void minmax_quantize_kernel(
    const typename T::storage* __restrict__ in, int64_t in_num_elem, int64_t cs, int64_t e0, int64_t e1,
    int target, const uint2* __restrict__ partials, int npartials, uint8_t* __restrict__ out,
    int64_t chunk_offset, int64_t out_bytes, int num_chunks) {
    // quantises elements [e0, e1) of each chunk (the whole chunk: [0, cs));
    // the range starting at 0 writes the header, the one ending at cs the slack
    using S = typename T::storage;
    constexpr int N = Vec<T>::N;
    const int cidx = kReverse ? (int)(gridDim.y - 1 - blockIdx.y) : (int)blockIdx.y;
    const int c = target < 0 ? cidx : target;
    // K:468-472: every element of the range is quantised with the chunk's
    // parameters, also those at or past in_num_elem (only the min/max of pass 1
    // is limited to the valid prefix, K:538-545); the input holds p*cs elements
    (void)in_num_elem;
    const int64_t len = e1 - e0;
    const S* src = in + (int64_t)c * cs + e0;
    uint8_t* seg = out + (int64_t)c * chunk_offset;
    uint8_t* payload = seg + 32 + e0;
    const int a = common_alignment<T>((uintptr_t)src, (uintptr_t)payload);
    const int64_t j0 = a < 0 ? len : (a < len ? a : len);
    const int64_t nvec = a < 0 ? 0 : (len - j0) / N;
    const uint4* __restrict__ vsrc = reinterpret_cast<const uint4*>(src + j0);
    uint8_t* vdst = payload + j0;
    const int64_t ntiles = (nvec + kVecPerBlockTile - 1) / kVecPerBlockTile;
    // the first tile's loads go out before the partials fold below (they do not need
    // the chunk's parameters): a workgroup otherwise starts with an L2 round trip and a
    // barrier and no HBM request in flight -- with ~4 workgroups per CU slot per launch
    // that idle start recurred four times per slot
    uint4 pre[kSubtiles];
    const int64_t t_first = blockIdx.x;
    const int64_t base_first = (kReverse ? (ntiles - 1 - t_first) : t_first) * kVecPerBlockTile;
    const bool have_pre = t_first < ntiles && base_first + kVecPerBlockTile <= nvec;
    if (have_pre) {
#pragma unroll
        for (int k = 0; k < kSubtiles; ++k) pre[k] = nt_load16(&vsrc[base_first + k * kBlock + threadIdx.x]);
    }

    // fold the chunk's partials (written by pass 1; L2/MALL-resident)
    uint32_t lo = 0xffffffffu, hi = 0xffffffffu;
    for (int i = threadIdx.x; i < npartials; i += kBlock) {
        const uint2 p = partials[(int64_t)cidx * npartials + i];
        lo = min(lo, p.x);
        hi = min(hi, p.y);
    }
    lo = wave_umin(lo);
    hi = wave_umin(hi);
    __shared__ uint32_t red[2][kWavesPerBlock];
    const int w = threadIdx.x / kWave;
    if (lane_id() == 0) { red[0][w] = lo; red[1][w] = hi; }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kWavesPerBlock; ++i) { lo = min(lo, red[0][i]); hi = min(hi, red[1][i]); }
    // the header holds T values (K:462-463); min/max of T data are exact in T
    const float mn = from_min_space(lo), mx = from_max_space(hi);
    const QParams q = make_qparams(mn, mx);

    if (blockIdx.x == 0 && e0 == 0) {
        // header {T min, T max, zero gap} (reference leaves the gap uninitialised)
        if (threadIdx.x < 32) {
            uint32_t hb = 0;
            const uint32_t bmn = sizeof(S) == 4 ? __float_as_uint(mn) : (uint32_t)T::from_f(mn);
            const uint32_t bmx = sizeof(S) == 4 ? __float_as_uint(mx) : (uint32_t)T::from_f(mx);
            const int t = threadIdx.x;
            if (t < (int)sizeof(S)) hb = (bmn >> (8 * t)) & 0xff;
            else if (t < 2 * (int)sizeof(S)) hb = (bmx >> (8 * (t - (int)sizeof(S)))) & 0xff;
            seg[t] = (uint8_t)hb;
        }
    }
    if (blockIdx.x == 0 && e1 == cs) {
        // slack after the payload, and the buffer tail after the last segment
        for (int64_t j = 32 + cs + threadIdx.x; j < chunk_offset; j += kBlock) seg[j] = 0;
        if (target < 0 && c == num_chunks - 1)
            for (int64_t j = (int64_t)num_chunks * chunk_offset + threadIdx.x; j < out_bytes; j += kBlock)
                out[j] = 0;
    }

    if (a < 0) {  // no common vector alignment: scalar path over the whole chunk
        for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < len; j += (int64_t)gridDim.x * kBlock)
            payload[j] = (uint8_t)quant(T::to_f(src[j]), q);
        return;
    }
    if (have_pre) {
#pragma unroll
        for (int k = 0; k < kSubtiles; ++k) {
            const int64_t v = base_first + k * kBlock + threadIdx.x;
            float f[N];
            unpack16<T>(pre[k], f);
            quant_store_vec<T>(f, q, vdst + v * N);
        }
    }
    for (int64_t t = blockIdx.x + (have_pre ? gridDim.x : 0); t < ntiles; t += gridDim.x) {
        const int64_t base = (kReverse ? (ntiles - 1 - t) : t) * kVecPerBlockTile;
        if (base + kVecPerBlockTile <= nvec) {
            // full tile: all loads issued before any is consumed
            uint4 r[kSubtiles];
#pragma unroll
            for (int k = 0; k < kSubtiles; ++k) r[k] = nt_load16(&vsrc[base + k * kBlock + threadIdx.x]);
#pragma unroll
            for (int k = 0; k < kSubtiles; ++k) {
                const int64_t v = base + k * kBlock + threadIdx.x;
                float f[N];
                unpack16<T>(r[k], f);
                quant_store_vec<T>(f, q, vdst + v * N);
            }
            continue;
        }
        for (int k = 0; k < kSubtiles; ++k) {  // ragged last tile
            const int64_t v = base + k * kBlock + threadIdx.x;
            if (v >= nvec) continue;
            float f[N];
            unpack16<T>(nt_load16(&vsrc[v]), f);
            quant_store_vec<T>(f, q, vdst + v * N);
        }
    }
    if (blockIdx.x == 0) {
        for (int64_t j = threadIdx.x; j < j0; j += kBlock) payload[j] = (uint8_t)quant(T::to_f(src[j]), q);
        for (int64_t j = j0 + nvec * N + threadIdx.x; j < len; j += kBlock)
            payload[j] = (uint8_t)quant(T::to_f(src[j]), q);
    }
}

// ------------------------------------------------------------------------
// dequantise
// ------------------------------------------------------------------------
template <typename T, bool NTS = true>
__global__ __launch_bounds__(kBlock) void minmax_dequantize_kernel(
    const uint8_t* __restrict__ in, int64_t chunk_offset, int64_t cs, int64_t e0, int64_t e1,
    typename T::storage* __restrict__ out) {
    // dequantises elements [e0, e1) of each chunk
    using S = typename T::storage;
    constexpr int N = Vec<T>::N;
    const int c = blockIdx.y;
    const uint8_t* seg = in + (int64_t)c * chunk_offset;
    const uint8_t* payload = seg + 32 + e0;
    S* dst = out + (int64_t)c * cs + e0;
    const int64_t len = e1 - e0;
    const int a = common_alignment<T>((uintptr_t)dst, (uintptr_t)payload);
    const int64_t j0 = a < 0 ? len : (a < len ? a : len);
    const int64_t nvec = a < 0 ? 0 : (len - j0) / N;
    uint4* __restrict__ vdst = reinterpret_cast<uint4*>(dst + j0);
    const uint8_t* vsrc = payload + j0;
    const int64_t stride = (int64_t)gridDim.x * kVecPerBlockTile;
    using W = typename Vec<T>::out_bytes;  // the N payload bytes of one vector
    // the first tile's payload loads go out before the header read and the table build
    // (one tile per workgroup up to 1 GiB: that prologue was the workgroup's whole
    // latency, with no HBM request in flight)
    W pre[kSubtiles];
    const int64_t base_first = (int64_t)blockIdx.x * kVecPerBlockTile;
    const bool have_pre = base_first + kVecPerBlockTile <= nvec;
    if (have_pre) {
#pragma unroll
        for (int k = 0; k < kSubtiles; ++k) pre[k] = load_word<T>(vsrc + (base_first + k * kBlock + threadIdx.x) * N);
    }
    const QParams q = read_header<T>(seg);
    static_assert(kBlock == 256, "one table entry per thread");
    __shared__ uint32_t lut[256];  // stored T bits of every byte value (codec_common.hpp)
    lut[threadIdx.x] = stored_bits<T>(dequant(threadIdx.x, q));
    __syncthreads();

    if (a < 0) {
        for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < len; j += (int64_t)gridDim.x * kBlock)
            dst[j] = storage_from_bits<T>(lut[payload[j]]);
        return;
    }
    for (int64_t base = base_first; base < nvec; base += stride) {
        if (base + kVecPerBlockTile <= nvec) {
            // full tile: raw loads first (no unpacking inside the load block, or
            // each load gets its own vmcnt(0) wait), then dequantise and store
            W raw[kSubtiles];
            if (base == base_first) {
#pragma unroll
                for (int k = 0; k < kSubtiles; ++k) raw[k] = pre[k];
            } else {
#pragma unroll
                for (int k = 0; k < kSubtiles; ++k)
                    raw[k] = load_word<T>(vsrc + (base + k * kBlock + threadIdx.x) * N);
            }
#pragma unroll
            for (int k = 0; k < kSubtiles; ++k) {
                uint32_t b[N];
                split_bytes<T>(raw[k], b);
#pragma unroll
                for (int i = 0; i < N; ++i) b[i] = lut[b[i]];
                if constexpr (NTS) nt_store16(pack_stored<T>(b), &vdst[base + k * kBlock + threadIdx.x]);
                else vdst[base + k * kBlock + threadIdx.x] = pack_stored<T>(b);
            }
            continue;
        }
        for (int k = 0; k < kSubtiles; ++k) {
            const int64_t v = base + k * kBlock + threadIdx.x;
            if (v >= nvec) continue;
            uint32_t b[N];
            split_bytes<T>(load_word<T>(vsrc + v * N), b);
#pragma unroll
            for (int i = 0; i < N; ++i) b[i] = lut[b[i]];
            if constexpr (NTS) nt_store16(pack_stored<T>(b), &vdst[v]);
            else vdst[v] = pack_stored<T>(b);
        }
    }
    if (blockIdx.x == 0) {
        for (int64_t j = threadIdx.x; j < j0; j += kBlock) dst[j] = storage_from_bits<T>(lut[payload[j]]);
        for (int64_t j = j0 + nvec * N + threadIdx.x; j < len; j += kBlock)
            dst[j] = storage_from_bits<T>(lut[payload[j]]);
    }
}

// ------------------------------------------------------------------------
// the centralized op at ONE rank, after the min/max pass (p = 1)
// ------------------------------------------------------------------------
// centralized_low_precision_synchronous.rs:30-71 with one rank is, per element,
//   b1 = Q1(x)                 compress, header1 = min/max of x
//   y  = T(T(dq1(b1)) + 0 + 0) decompress, then reduce over one chunk (K:373-400:
//                              s = 0.0f + c0, the BY = 2 tree adds 0.0f; mean: x 1)
//   b2 = Q2(y)                 compress, header2 = min/max of y (as stored in T)
//   out = T(dq2(b2))           decompress
// so `out` is a function of b1 alone: a 256-entry table per launch.  header2
// needs no pass over y:
//  * header1 finite and scale1 finite > 0: Q1 (x*scale, rint, fminf(ub), - lb,
//    saturate) and dq1 ((b + lb) / scale, then T rounding, + 0.0f) are monotone
//    non-decreasing, and Q1(NaN) = Q1(max) (fminf(NaN, ub) = ub), so
//    min y = y(Q1(min x)) and max y = y(Q1(max x)), both finite or +-inf, never
//    NaN (dq1 of a finite lb over a positive scale);
//  * every element NaN (header = the init values, min > max): every b1 is Q1(NaN),
//    so y takes one value, header2 = (y, y) -- or the init values if y is NaN;
//  * otherwise (a +-inf in the header, or max - min overflowing: scale1 is +0 or
//    NaN) every b1 decodes to NaN -- scale1 = +0 comes with every byte 255 (mx
//    finite: (255 + lb)/0 = 0/0) or every byte 0 with lb NaN -- so header2 is the
//    min/max over no value: the init values (T::init_max, -T::init_max).
// Bit-identical to the four-kernel sequence (tests/test_gpu_codec.py
// test_one_rank_op_matches_sequence, incl. NaN, +-inf and all-NaN buckets); reads
// 4N and writes 4N bytes after the 4N of the min/max pass (12N) instead of 18N.
template <typename T, int AV>
__device__ __forceinline__ float one_rank_reduce(float c0) {
    float s = 0.0f + c0;  // s[0] of the BY = 2 tree
    s = s + 0.0f;         // + s[1] (no second chunk)
    if constexpr (AV == 0) return s;
    else return s * 1.0f;  // mean over p = 1: the exact reciprocal (reduce.hip avg_finish)
}

// The op's parameters from the folded min/max keys: Q1 (the first quantisation) and the
// table entry for byte b (the T bits of the op's final value for b1 = b).
template <typename T, int AV>
__device__ __forceinline__ uint32_t one_rank_entry(uint32_t lo, uint32_t hi, uint32_t b, QParams* q1_out) {
    const float mn1 = from_min_space(lo), mx1 = from_max_space(hi);
    const QParams q1 = make_qparams(mn1, mx1);
    const bool regular = __builtin_isfinite(mn1) && __builtin_isfinite(mx1) && __builtin_isfinite(q1.scale) &&
                         q1.scale > 0.0f;
    auto y_of = [&](uint32_t c) { return as_stored<T>(one_rank_reduce<T, AV>(as_stored<T>(dequant(c, q1)))); };
    float mn2 = T::init_max(), mx2 = -T::init_max();
    if (regular) {
        mn2 = y_of(quant(mn1, q1));
        mx2 = y_of(quant(mx1, q1));
    } else if (!(mn1 <= mx1)) {
        // every element NaN (the header holds the init values): one byte value for all of
        // them, so one y value -- the min and max of y unless it is NaN itself (the f16
        // init header has a finite, negative scale: y = -inf there)
        const float ys = y_of(quant(__int_as_float(0x7fc00000), q1));
        if (!__builtin_isnan(ys)) mn2 = mx2 = ys;
    }
    const QParams q2 = make_qparams(mn2, mx2);
    *q1_out = q1;
    return stored_bits<T>(dequant(quant(y_of(b), q2), q2));
}

template <typename T, int AV>
__global__ __launch_bounds__(kBlock) void minmax_one_rank_kernel(typename T::storage* __restrict__ x, int64_t n,
                                                                 const uint2* __restrict__ partials, int npartials) {
    using S = typename T::storage;
    constexpr int N = Vec<T>::N;
    // the body on 16-B vectors (head elements before the first aligned one go scalar)
    int64_t j0 = (int64_t)(((16u - ((uintptr_t)x & 15u)) & 15u) / sizeof(S));
    if (((uintptr_t)x % sizeof(S)) != 0) j0 = n;
    if (j0 > n) j0 = n;
    const int64_t nvec = (n - j0) / N;
    uint4* __restrict__ v = reinterpret_cast<uint4*>(x + j0);
    const int64_t ntiles = (nvec + kVecPerBlockTile - 1) / kVecPerBlockTile;
    // the first tile's loads go out before the partials fold and the table build (the
    // workgroup's prologue otherwise runs with no HBM request in flight)
    uint4 pre[kSubtiles];
    const int64_t base_first = (ntiles - 1 - (int64_t)blockIdx.x) * kVecPerBlockTile;
    const bool have_pre = (int64_t)blockIdx.x < ntiles && base_first + kVecPerBlockTile <= nvec;
    if (have_pre) {
#pragma unroll
        for (int k = 0; k < kSubtiles; ++k) pre[k] = nt_load16(&v[base_first + k * kBlock + threadIdx.x]);
    }
    __shared__ uint32_t lut[256];  // b1 -> the T bits of the op's final value
    uint32_t lo = 0xffffffffu, hi = 0xffffffffu;
    for (int i = threadIdx.x; i < npartials; i += kBlock) {
        const uint2 p = partials[i];
        lo = min(lo, p.x);
        hi = min(hi, p.y);
    }
    lo = wave_umin(lo);
    hi = wave_umin(hi);
    __shared__ uint32_t red[2][kWavesPerBlock];
    const int w = threadIdx.x / kWave;
    if (lane_id() == 0) { red[0][w] = lo; red[1][w] = hi; }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kWavesPerBlock; ++i) { lo = min(lo, red[0][i]); hi = min(hi, red[1][i]); }
    QParams q1;
    static_assert(kBlock == 256, "one table entry per thread");
    lut[threadIdx.x] = one_rank_entry<T, AV>(lo, hi, threadIdx.x, &q1);
    __syncthreads();

    // reverse sweep: the min/max pass read the tail last, so it is re-read from the
    // Infinity Cache first.  (Software-pipelining the next tile's loads ahead of this
    // tile's stores measured no gain at 25 MiB or 1 GiB: profiles/r05_small_sweep2.json.)
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t base = (ntiles - 1 - t) * kVecPerBlockTile;
        if (base + kVecPerBlockTile <= nvec) {
            uint4 r[kSubtiles];
            if (t == (int64_t)blockIdx.x) {
#pragma unroll
                for (int k = 0; k < kSubtiles; ++k) r[k] = pre[k];
            } else {
#pragma unroll
                for (int k = 0; k < kSubtiles; ++k) r[k] = nt_load16(&v[base + k * kBlock + threadIdx.x]);
            }
#pragma unroll
            for (int k = 0; k < kSubtiles; ++k) {
                float f[N];
                unpack16<T>(r[k], f);
                uint32_t b[N];
#pragma unroll
                for (int i = 0; i < N; i += 4) {
                    const uint32_t q = quant_pack4(f[i], f[i + 1], f[i + 2], f[i + 3], q1);
#pragma unroll
                    for (int e = 0; e < 4; ++e) b[i + e] = lut[(q >> (8 * e)) & 0xff];
                }
                nt_store16(pack_stored<T>(b), &v[base + k * kBlock + threadIdx.x]);
            }
            continue;
        }
        for (int k = 0; k < kSubtiles; ++k) {
            const int64_t vi = base + k * kBlock + threadIdx.x;
            if (vi >= nvec) continue;
            float f[N];
            unpack16<T>(nt_load16(&v[vi]), f);
            uint32_t b[N];
#pragma unroll
            for (int i = 0; i < N; ++i) b[i] = lut[quant(f[i], q1)];
            nt_store16(pack_stored<T>(b), &v[vi]);
        }
    }
    if (blockIdx.x == 0) {
        for (int64_t j = threadIdx.x; j < j0; j += kBlock) x[j] = storage_from_bits<T>(lut[quant(T::to_f(x[j]), q1)]);
        for (int64_t j = j0 + nvec * N + threadIdx.x; j < n; j += kBlock)
            x[j] = storage_from_bits<T>(lut[quant(T::to_f(x[j]), q1)]);
    }
}

// ------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------
// workgroups per chunk: one per tile of (kBlock * sub) vectors, capped so the
// whole launch has about `target` workgroups (the rest grid-strides)
static int blocks_for(int64_t elems, int per_vec, int nact, int sub = kSubtiles, int target = kQuantBlocks) {
    const int64_t nvec = elems / per_vec + 1;
    const int64_t tile = (int64_t)kBlock * sub;
    int64_t tiles = (nvec + tile - 1) / tile;
    const int64_t per_chunk = (target + nact - 1) / nact;
    if (tiles > per_chunk) tiles = per_chunk;
    return (int)(tiles < 1 ? 1 : tiles);
}

// workgroups of the min/max pass = partials each chunk's quantise pass folds;
// shared with producers of the same partials (decentralized.hip)
int minmax_partials_blocks(int64_t cs, int per_vec, int nact, size_t ws_bytes) {
    const int nblk = blocks_for(cs, per_vec, nact, kPartialsSub, kPartialsBlocks);
    const int64_t cap = (int64_t)(ws_bytes / sizeof(uint2)) / (nact > 0 ? nact : 1);
    if (cap < 1) return 0;
    return nblk > cap ? (int)cap : nblk;
}

// Load policy of the min/max pass: BAGUA_PARTIALS_NT=1 / 0 forces non-temporal /
// default loads (A/B).  Unset: non-temporal for the pipelined op's backward pass (stage
// 5) over more than the 256 MiB Infinity Cache -- a 1 GiB pass takes 154.8 instead of
// 172.5 us (0.87 of 8 TB/s), the first quantise piece then misses the chunks' cached
// beginnings (51 -> 57 us), a net 14 us off the op's unhidden prefix -- since kept
// by loading the sweep's last 256 MiB with the default policy (compress_impl); elsewhere
// the next kernel's cache hits are worth more (256 MiB buckets 2,001 vs 1,860 GiB/s;
// profiles/r04_partials_nt_ab.jsonl); the one-rank op splits its pass the same way
// (one_rank_impl).
template <typename T>
static bool partials_nt(int64_t elems, bool rev) {
    const int env = tune_int("BAGUA_PARTIALS_NT", -1);
    if (env >= 0) return env != 0;
    return rev && elems * (int64_t)sizeof(typename T::storage) > ((int64_t)kPartialsNtAboveMiB << 20);
}

// defined in minmax_resident.hip; BAGUA_ERR_UNSUPPORTED when the shape is not eligible
template <typename T>
int resident_compress_impl(const void* input, int64_t in_num_elem, int64_t cs, int p, uint8_t* out,
                           int64_t out_bytes, int target, hipStream_t s);

// stage bit 1: min/max partials pass; bit 2: quantise pass (3 = whole compress);
// bit 4: the partials pass sweeps each chunk backwards (with bit 1 only).
// Both stages derive the same partials count from the same arguments.
template <typename T>
static int compress_impl(const void* input, int in_num_elem, int cs, int p, uint8_t* out,
                         size_t out_bytes, void* ws, size_t ws_bytes, int target, hipStream_t s,
                         int stages = 3, int e0 = 0, int e1 = -1) {
    using S = typename T::storage;
    if (e1 < 0) e1 = cs;
    if (p <= 0 || p > 65535 || cs < 0 || target < -1 || target >= p || !input || !out || e0 < 0 || e1 < e0 ||
        e1 > cs)
        return BAGUA_ERR_INVALID_ARG;
    const int64_t chunk_offset = (int64_t)(out_bytes / (size_t)p);  // K:537
    if (chunk_offset < (int64_t)cs + 32) return BAGUA_ERR_INVALID_ARG;
    const int nact = target < 0 ? p : 1;
    const int nblk = ws ? minmax_partials_blocks(cs, Vec<T>::N, nact, ws_bytes) : 0;
    if (nblk < 1) return BAGUA_ERR_WORKSPACE;
    uint2* partials = static_cast<uint2*>(ws);
    if (stages == 3 && e0 == 0 && e1 == cs) {  // one-launch encode when eligible (minmax_resident.hip)
        const int rc = resident_compress_impl<T>(input, in_num_elem, cs, p, out, (int64_t)out_bytes, target, s);
        if (rc != BAGUA_ERR_UNSUPPORTED) return rc;
    }
    if (stages & 1) {
        const bool rev = (stages & 4) != 0;
        const bool nt = partials_nt<T>((int64_t)cs * nact, rev);
        const dim3 grid(nblk, nact);
        const S* src = static_cast<const S*>(input);
        // the last 256 MiB of the backward sweep, over all chunks, load with the default
        // policy, so the chunks' beginnings -- the first quantise piece -- stay in the
        // Infinity Cache (1 GiB, p = 1, 4 pieces: pass + piece 0 217 -> 208 us, piece 0
        // 55 -> 49.5 us; profiles/r04_partials_keep_ab.jsonl); BAGUA_PARTIALS_KEEP_MIB
        // overrides (0: every load non-temporal)
        const int keep_mib = tune_int("BAGUA_PARTIALS_KEEP_MIB", kPartialsNtAboveMiB);
        const int64_t chunk_bytes = (int64_t)cs * (int64_t)sizeof(S);
        const int64_t keep = ((int64_t)keep_mib << 20) / nact;
        const int64_t nt_until = keep > 0 ? (chunk_bytes > keep ? (chunk_bytes - keep) / 16 : 0) : INT64_MAX;
        if (rev && nt)
            launch(minmax_partials_kernel<T, true, true>, grid, dim3(kBlock), 0, s, src, (int64_t)in_num_elem,
                   (int64_t)cs, target, partials, nt_until);
        else if (rev)
            launch(minmax_partials_kernel<T, true, false>, grid, dim3(kBlock), 0, s, src, (int64_t)in_num_elem,
                   (int64_t)cs, target, partials, INT64_MAX);
        else if (nt)
            launch(minmax_partials_kernel<T, false, true>, grid, dim3(kBlock), 0, s, src, (int64_t)in_num_elem,
                   (int64_t)cs, target, partials, INT64_MAX);
        else
            launch(minmax_partials_kernel<T, false, false>, grid, dim3(kBlock), 0, s, src, (int64_t)in_num_elem,
                   (int64_t)cs, target, partials, INT64_MAX);
    }
    // (Folding the partials once per chunk in a separate launch, so each quantise
    // workgroup reads one partial instead of up to 1024, measured no faster in the ring
    // op: 658.7 vs 664.1 us, profiles/r05_quant_prefold_ab.json.)
    if (stages & 2)
        launch((minmax_quantize_kernel<T, true>),
               dim3(blocks_for(e1 - e0, Vec<T>::N, nact, kSubtiles, tune_int("BAGUA_TUNE_QUANT_BLOCKS", kQuantBlocks)),
                    nact),
               dim3(kBlock), 0, s, static_cast<const S*>(input), (int64_t)in_num_elem, (int64_t)cs, (int64_t)e0,
               (int64_t)e1, target, partials, nblk, out, chunk_offset, (int64_t)out_bytes, p);
    return check_launch();
}

// Grid of a requantise whose every workgroup folds `npartials` min/max partials
// first (the fused reduce's 2048 per piece): the fold traffic is workgroups x
// npartials x 8 B, so the grid is capped at ~8 MB of it (never below 512, which
// still streams at full rate).  A 1 GiB bucket's requantise pieces at p = 2 / 4 /
// 8 (4 pieces, npartials 8192): 53.7 / 27.6 / 14.4 us per piece with the codec's
// 8192 workgroups, 32.8 / 16.8 / 9.5 with 512 (tools/pipeline_kernels_probe.py,
// profiles/r03_requantise_grid_ab.jsonl).  BAGUA_TUNE_RQ_BLOCKS overrides (A/B).
static int fold_grid_target(int npartials) {
    const int env = tune_int("BAGUA_TUNE_RQ_BLOCKS", 0);
    if (env > 0) return env;
    int64_t g = ((int64_t)8 << 20) / ((int64_t)(npartials > 0 ? npartials : 1) * 8);
    if (g < 512) g = 512;
    if (g > kQuantBlocks) g = kQuantBlocks;
    return (int)g;
}

// defined in reduce.hip
int fused_blocks(int64_t cs, int per_vec);
template <typename T>
int dequant_reduce_impl(const uint8_t* in, size_t in_bytes, int cs, int p, void* out, int average, uint2* partials,
                        int blocks, hipStream_t s, int e0, int e1, FusedTables tb = FusedTables{});
template <typename T>
int dequant_reduce_quantize_impl(const uint8_t* in, size_t in_bytes, int cs, int p, int average,
                                 const uint2* partials, int npartials, uint8_t* seg, int64_t seg_bytes, int blocks,
                                 hipStream_t s, void* final_chunk, int e0 = 0, int e1 = -1,
                                 const float* tab_in = nullptr);

template <typename T>
static int reduce_requantize_impl(const uint8_t* recv, size_t recv_bytes, int cs, int p, void* tensor, int average,
                                  uint8_t* out, size_t out_bytes, int target, void* ws, size_t ws_bytes,
                                  hipStream_t s, void* final_tensor = nullptr) {
    using S = typename T::storage;
    if (final_tensor) tensor = nullptr;  // the final decompress of the own chunk replaces the store
    if (p <= 0 || p > kMaxFusedChunks || cs < 0 || target < 0 || target >= p || (!out && !final_tensor))
        return BAGUA_ERR_UNSUPPORTED;
    const int64_t chunk_offset = (int64_t)(out_bytes / (size_t)p);
    if (out && chunk_offset < (int64_t)cs + 32) return BAGUA_ERR_INVALID_ARG;
    const int blocks = fused_blocks(cs, Vec<T>::N);
    if (!ws || ws_bytes < (size_t)blocks * sizeof(uint2)) return BAGUA_ERR_WORKSPACE;
    if (!tensor) {
        // the reduced chunk is not stored: a partials-only pass, then the requantise
        // recomputes it from the p received segments (p*cs bytes read twice instead of
        // cs*sizeof(T) written and read back)
        uint2* partials = static_cast<uint2*>(ws);
        int rc = dequant_reduce_impl<T>(recv, recv_bytes, cs, p, nullptr, average, partials, blocks, s, 0, cs);
        if (rc) return rc;
        return dequant_reduce_quantize_impl<T>(
            recv, recv_bytes, cs, p, average, partials, blocks, out ? out + (int64_t)target * chunk_offset : nullptr,
            chunk_offset,
            blocks, s, final_tensor ? static_cast<void*>(static_cast<S*>(final_tensor) + (int64_t)target * cs) : nullptr);
    }
    S* chunk = static_cast<S*>(tensor) + (int64_t)target * cs;
    uint2* partials = static_cast<uint2*>(ws);
    int rc = dequant_reduce_impl<T>(recv, recv_bytes, cs, p, chunk, average, partials, blocks, s, 0, cs);
    if (rc) return rc;
    launch((minmax_quantize_kernel<T, true>),
           dim3(blocks_for(cs, Vec<T>::N, 1, kSubtiles, fold_grid_target(blocks)), 1), dim3(kBlock), 0, s,
           static_cast<const S*>(tensor), (int64_t)p * cs, (int64_t)cs, (int64_t)0, (int64_t)cs, target, partials,
           blocks, out, chunk_offset, (int64_t)out_bytes, p);
    return check_launch();
}

// ---- pipelined all-reduce building blocks ---------------------------------
// A chunk is cut into `pieces` element ranges of L = align(ceil(cs/pieces), 512)
// elements (trailing ones may be empty).  Piece k's fused reduce writes its
// `fused_blocks(longest piece)` min/max partials to slot k of the workspace;
// the requantise folds all of them, which is the same min/max as one pass.
//
// A piece schedule `pieces` is a count, optionally OR-ed with
// BAGUA_PIECES_TAPERED: from 3 pieces on, the first and the last piece are then
// half the size of the others (weights 1, 2, ..., 2, 1; edges 512-aligned).  The
// pipelined op's codec work before the first exchange (quantise piece 0) and
// after the last one (dequantise the last piece) is then that of 2(pieces-1)
// pieces with only `pieces` exchange groups.  The schedule is an argument of
// every piece function (the op reads its configuration once and passes it on),
// so every rank and every building block of one op sees the same ranges.
static bool piece_schedule_ok(int pieces) {
    const int n = pieces & BAGUA_PIECES_COUNT_MASK;
    return n >= 1 && (pieces & ~(BAGUA_PIECES_COUNT_MASK | BAGUA_PIECES_TAPERED | BAGUA_PIECES_MULTIPATH |
                                 BAGUA_PIECES_FOLDED | BAGUA_PIECES_TABLES)) == 0;
}
static int piece_count(int pieces) { return pieces & BAGUA_PIECES_COUNT_MASK; }

static void piece_range(int cs, int schedule, int k, int* b, int* e) {
    const int pieces = piece_count(schedule);
    if (pieces >= 3 && (schedule & BAGUA_PIECES_TAPERED)) {
        const int64_t W = 2 * (int64_t)(pieces - 1);
        auto edge = [&](int j) -> int {
            const int64_t w = j == 0 ? 0 : (j >= pieces ? W : 2 * (int64_t)j - 1);
            const int64_t x = ((int64_t)cs * w / W + 511) / 512 * 512;
            return (int)(x < cs ? x : cs);
        };
        *b = edge(k);
        *e = edge(k + 1);
        return;
    }
    const int64_t L = (((int64_t)cs + pieces - 1) / pieces + 511) / 512 * 512;
    const int64_t lo = (int64_t)k * L, hi = lo + L;
    *b = (int)(lo < cs ? lo : cs);
    *e = (int)(hi < cs ? hi : cs);
}

static int piece_blocks(int cs, int schedule, int per_vec) {
    int longest = 0;
    for (int k = 0; k < piece_count(schedule); ++k) {
        int b, e;
        piece_range(cs, schedule, k, &b, &e);
        if (e - b > longest) longest = e - b;
    }
    return fused_blocks(longest, per_vec);
}

// tensor == nullptr: the piece's min/max partials only, nothing stored (the
// requantise then recomputes the piece from the received segments:
// reduce_requantize_piece_impl)
// the one folded partial (bagua_minmax_u8_fold_piece_partials) sits after the largest
// partials region any dtype writes (f32's, 4 elements per vector) -- inside the
// workspace's 256-byte tail
static uint2* folded_slot(void* ws, int cs, int pieces) {
    return static_cast<uint2*>(ws) + (size_t)piece_count(pieces) * piece_blocks(cs, pieces, 4);
}

// the p x 256 dequantisation tables reduce piece 0 leaves for the op's later pieces and
// requantise (BAGUA_PIECES_TABLES), after the folded slot's 256-byte tail
constexpr size_t kPieceTablesBytes = (size_t)kMaxFusedChunks * 256 * sizeof(float);
static float* piece_tables(void* ws, int cs, int pieces) {
    return reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(ws) +
                                    (size_t)piece_count(pieces) * piece_blocks(cs, pieces, 4) * sizeof(uint2) + 256);
}
static bool tables_fit(const void* ws, size_t ws_bytes, int cs, int pieces) {
    return ws && (const uint8_t*)piece_tables(const_cast<void*>(ws), cs, pieces) + kPieceTablesBytes <=
                     (const uint8_t*)ws + ws_bytes;
}

// one workgroup folds n {min, max} key partials into out[0]
__global__ __launch_bounds__(kBlock) void fold_partials_kernel(const uint2* __restrict__ in, int64_t n,
                                                               uint2* __restrict__ out) {
    uint32_t lo = 0xffffffffu, hi = 0xffffffffu;
    for (int64_t i = threadIdx.x; i < n; i += kBlock) {
        const uint2 v = in[i];
        lo = min(lo, v.x);
        hi = min(hi, v.y);
    }
    lo = wave_umin(lo);
    hi = wave_umin(hi);
    __shared__ uint32_t red[2][kWavesPerBlock];
    const int w = threadIdx.x / kWave;
    if (lane_id() == 0) { red[0][w] = lo; red[1][w] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 1; i < kWavesPerBlock; ++i) { lo = min(lo, red[0][i]); hi = min(hi, red[1][i]); }
        out[0] = make_uint2(lo, hi);
    }
}

template <typename T>
static int fold_piece_partials_impl(int cs, int pieces, void* ws, size_t ws_bytes, hipStream_t s) {
    if (cs < 0 || !piece_schedule_ok(pieces)) return BAGUA_ERR_INVALID_ARG;
    const int blocks = piece_blocks(cs, pieces, Vec<T>::N);
    const int n = piece_count(pieces) * blocks;
    uint2* slot = ws ? folded_slot(ws, cs, pieces) : nullptr;
    if (!ws || (uint8_t*)(slot + 1) > (uint8_t*)ws + ws_bytes) return BAGUA_ERR_WORKSPACE;
    launch(fold_partials_kernel, dim3(1), dim3(kBlock), 0, s, static_cast<const uint2*>(ws), (int64_t)n, slot);
    return check_launch();
}

template <typename T>
static int reduce_piece_impl(const uint8_t* recv, size_t recv_bytes, int cs, int p, void* tensor, int average,
                             int target, int pieces, int piece, void* ws, size_t ws_bytes, hipStream_t s) {
    using S = typename T::storage;
    if (p <= 0 || cs < 0 || target < 0 || target >= p || !piece_schedule_ok(pieces) || piece < 0 ||
        piece >= piece_count(pieces))
        return BAGUA_ERR_INVALID_ARG;
    const int blocks = piece_blocks(cs, pieces, Vec<T>::N);
    if (!ws || ws_bytes < (size_t)piece_count(pieces) * blocks * sizeof(uint2)) return BAGUA_ERR_WORKSPACE;
    int b, e;
    piece_range(cs, pieces, piece, &b, &e);
    S* chunk = tensor ? static_cast<S*>(tensor) + (int64_t)target * cs : nullptr;
    // piece 0 leaves its tables in the workspace (when it has room); with
    // BAGUA_PIECES_TABLES the later pieces copy them instead of building their own
    FusedTables tb;
    if (tables_fit(ws, ws_bytes, cs, pieces)) {
        if (piece == 0) tb.out = piece_tables(ws, cs, pieces);
        else if (pieces & BAGUA_PIECES_TABLES) tb.in = piece_tables(ws, cs, pieces);
    } else if (pieces & BAGUA_PIECES_TABLES) {
        return BAGUA_ERR_WORKSPACE;
    }
    return dequant_reduce_impl<T>(recv, recv_bytes, cs, p, chunk, average,
                                  static_cast<uint2*>(ws) + (size_t)piece * blocks, blocks, s, b, e, tb);
}

// Requantise piece `piece` of the own chunk straight from the p received segments:
// fold every piece's partials (bagua_minmax_u8_reduce_piece with tensor == nullptr),
// recompute the reduced values (the same tables and summation tree, so the same T
// values bit for bit) and quantise them into segment `target` of `out` -- the bytes
// reduce_piece (storing) + requantize_piece write, without storing the reduced chunk
// and reading it back: (2p + 1) L bytes per piece of L elements instead of (p + 9) L
// at fp32.
template <typename T>
static int reduce_requantize_piece_impl(const uint8_t* recv, size_t recv_bytes, int cs, int p, int average,
                                        uint8_t* out, size_t out_bytes, int target, int pieces, int piece,
                                        const void* ws, size_t ws_bytes, hipStream_t s) {
    if (p <= 0 || cs < 0 || target < 0 || target >= p || !out || !piece_schedule_ok(pieces) || piece < 0 ||
        piece >= piece_count(pieces))
        return BAGUA_ERR_INVALID_ARG;
    if (p > kMaxFusedChunks) return BAGUA_ERR_UNSUPPORTED;
    const int64_t chunk_offset = (int64_t)(out_bytes / (size_t)p);
    if (chunk_offset < (int64_t)cs + 32) return BAGUA_ERR_INVALID_ARG;
    const int blocks = piece_blocks(cs, pieces, Vec<T>::N);
    const bool folded = (pieces & BAGUA_PIECES_FOLDED) != 0;
    const int partials = folded ? 1 : piece_count(pieces) * blocks;
    const uint2* part = folded ? folded_slot(const_cast<void*>(ws), cs, pieces) : static_cast<const uint2*>(ws);
    if (!ws || ws_bytes < (size_t)((const uint8_t*)(part + partials) - (const uint8_t*)ws)) return BAGUA_ERR_WORKSPACE;
    int b, e;
    piece_range(cs, pieces, piece, &b, &e);
    if (b == e && piece > 0) return BAGUA_OK;  // empty trailing piece: its bytes were written by the others
    const int grid = (int)std::min<int64_t>(fused_blocks(e - b, Vec<T>::N),
                                            tune_int("BAGUA_TUNE_RRQ_BLOCKS", fold_grid_target(partials)));
    const float* tab = nullptr;  // BAGUA_PIECES_TABLES: the tables reduce piece 0 left
    if (pieces & BAGUA_PIECES_TABLES) {
        if (!tables_fit(ws, ws_bytes, cs, pieces)) return BAGUA_ERR_WORKSPACE;
        tab = piece_tables(const_cast<void*>(ws), cs, pieces);
    }
    return dequant_reduce_quantize_impl<T>(recv, recv_bytes, cs, p, average, part, partials,
                                           out + (int64_t)target * chunk_offset, chunk_offset, grid, s, nullptr, b,
                                           e, tab);
}

// requantise elements [e0, e1) of the own chunk from every piece's partials (the
// whole chunk: [0, cs)); the range at 0 writes the header, the one ending at cs
// the slack
template <typename T>
static int requantize_pieces_impl(const void* tensor, int cs, int p, uint8_t* out, size_t out_bytes, int target,
                                  int pieces, const void* ws, size_t ws_bytes, hipStream_t s, int e0 = 0,
                                  int e1 = -1) {
    using S = typename T::storage;
    if (e1 < 0) e1 = cs;
    if (p <= 0 || cs < 0 || target < 0 || target >= p || !tensor || !out || !piece_schedule_ok(pieces) || e0 < 0 ||
        e1 < e0 || e1 > cs)
        return BAGUA_ERR_INVALID_ARG;
    const int64_t chunk_offset = (int64_t)(out_bytes / (size_t)p);
    if (chunk_offset < (int64_t)cs + 32) return BAGUA_ERR_INVALID_ARG;
    const int blocks = piece_blocks(cs, pieces, Vec<T>::N);
    const bool folded = (pieces & BAGUA_PIECES_FOLDED) != 0;
    const int partials = folded ? 1 : piece_count(pieces) * blocks;
    const uint2* part = folded ? folded_slot(const_cast<void*>(ws), cs, pieces) : static_cast<const uint2*>(ws);
    if (!ws || ws_bytes < (size_t)((const uint8_t*)(part + partials) - (const uint8_t*)ws)) return BAGUA_ERR_WORKSPACE;
    launch((minmax_quantize_kernel<T, true>),
           dim3(blocks_for(e1 - e0, Vec<T>::N, 1, kSubtiles, fold_grid_target(partials)), 1), dim3(kBlock), 0,
           s, static_cast<const S*>(tensor), (int64_t)p * cs, (int64_t)cs, (int64_t)e0, (int64_t)e1, target,
           part, partials, out, chunk_offset, (int64_t)out_bytes, p);
    return check_launch();
}

template <typename T>
static int one_rank_impl(void* tensor, int num_elem, int average, void* ws, size_t ws_bytes, hipStream_t s) {
    using S = typename T::storage;
    if (!tensor || num_elem < 0) return BAGUA_ERR_INVALID_ARG;
    const int nblk = ws ? minmax_partials_blocks(num_elem, Vec<T>::N, 1, ws_bytes) : 0;
    if (nblk < 1) return BAGUA_ERR_WORKSPACE;
    uint2* partials = static_cast<uint2*>(ws);
    // the table pass sweeps backwards: the tail the min/max pass reads last is re-read
    // first, from the Infinity Cache.  Above the cache size only the last 256 MiB load
    // with the default policy, the rest non-temporally: 1 GiB op 0.503 -> 0.474 ms
    // (sweep of the kept size 0..512 MiB: profiles/r04_one_rank_keep_probe*.jsonl);
    // BAGUA_ONE_RANK_KEEP_MIB overrides (-1: every load with the default policy)
    const int64_t bytes = (int64_t)num_elem * (int64_t)sizeof(S);
    const int keep_mib = tune_int("BAGUA_ONE_RANK_KEEP_MIB", kPartialsNtAboveMiB);
    const int64_t keep = keep_mib < 0 ? bytes : ((int64_t)keep_mib << 20);
    if (keep < bytes)
        launch(minmax_partials_kernel<T, false, true>, dim3(nblk, 1), dim3(kBlock), 0, s,
               static_cast<const S*>(tensor), (int64_t)num_elem, (int64_t)num_elem, -1, partials,
               (int64_t)((bytes - keep) / 16));
    else
        launch(minmax_partials_kernel<T, false, false>, dim3(nblk, 1), dim3(kBlock), 0, s,
               static_cast<const S*>(tensor), (int64_t)num_elem, (int64_t)num_elem, -1, partials, INT64_MAX);
    const dim3 grid(
        blocks_for(num_elem, Vec<T>::N, 1, kSubtiles, tune_int("BAGUA_TUNE_ONE_RANK_BLOCKS", kOneRankBlocks)), 1);
    // (folding the partials and building the table once in a one-workgroup kernel, the
    // table pass loading them, measured no faster: 25 MiB 14.9 vs 14.7 us, 1 GiB 326 vs
    // 321 us, profiles/r05_one_rank_header_ab.json -- the per-workgroup prologue is hidden
    // behind the first tile's loads)
    // (default-policy stores of the result instead of non-temporal ones: 25 MiB op 23.7 ->
    // 24.9 us, 1 GiB 512 -> 528 us, the 32 x 25 MiB scheduler line 1,496 / 1,554 -> 1,417 /
    // 1,436 GiB/s, profiles/r05_one_rank_nts_ab.json)
    auto go = [&](auto av) {
        constexpr int AV = decltype(av)::value;
        launch(minmax_one_rank_kernel<T, AV>, grid, dim3(kBlock), 0, s, static_cast<S*>(tensor), (int64_t)num_elem,
               static_cast<const uint2*>(partials), nblk);
    };
    if (average) go(std::integral_constant<int, 1>{});
    else go(std::integral_constant<int, 0>{});
    return check_launch();
}

template <typename T>
static int decompress_impl(const uint8_t* in, size_t in_bytes, int cs, int p, void* out, hipStream_t s,
                           int e0 = 0, int e1 = -1) {
    using S = typename T::storage;
    if (e1 < 0) e1 = cs;
    if (p <= 0 || p > 65535 || cs < 0 || !in || !out || e0 < 0 || e1 < e0 || e1 > cs) return BAGUA_ERR_INVALID_ARG;
    const int64_t chunk_offset = (int64_t)(in_bytes / (size_t)p);  // K:566
    if (chunk_offset < (int64_t)cs + 32) return BAGUA_ERR_INVALID_ARG;
    // nt stores: with default-policy stores the decoded bucket's dirty lines sit in the
    // Infinity Cache and the next encode's pass 2 pays for them (85 -> 119 us per
    // 256 MiB encode)
    launch(minmax_dequantize_kernel<T, true>,
           dim3(blocks_for(e1 - e0, Vec<T>::N, p, kSubtiles, tune_int("BAGUA_TUNE_DEQUANT_BLOCKS", kDequantBlocks)), p),
           dim3(kBlock), 0, s, in, chunk_offset, (int64_t)cs, (int64_t)e0, (int64_t)e1, static_cast<S*>(out));
    return check_launch();
}

}  // namespace bagua

using namespace bagua;

extern "C" {

size_t bagua_minmax_u8_compressed_bytes(int dtype, int chunk_size, int num_chunks) {
    // datatypes/mod.rs:669-704
    const size_t esz = dtype == BAGUA_DTYPE_F32 ? 4 : 2;
    auto al = [](size_t x, size_t a) { return (x + a - 1) / a * a; };
    return al((size_t)chunk_size * (size_t)num_chunks, 32) + al(2 * esz, 32) * (size_t)num_chunks;
}

size_t bagua_minmax_u8_workspace_bytes(int /*chunk_size*/, int num_chunks) {
    // one uint2 partial per workgroup; at most kTargetBlocks + num_chunks workgroups
    return sizeof(uint2) * ((size_t)kTargetBlocks + (size_t)(num_chunks > 0 ? num_chunks : 1)) + 256;
}

int bagua_minmax_u8_compress(int dtype, const void* input, int input_num_element, int chunk_size,
                             int num_chunks, uint8_t* output, size_t output_bytes, void* workspace,
                             size_t workspace_bytes, int target_chunk, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return compress_impl<F32>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                      workspace, workspace_bytes, target_chunk, s);
        case BAGUA_DTYPE_F16:
            return compress_impl<F16>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                      workspace, workspace_bytes, target_chunk, s);
        case BAGUA_DTYPE_BF16:
            return compress_impl<BF16>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                       workspace, workspace_bytes, target_chunk, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_minmax_u8_decompress(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                               int num_chunks, void* output, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32: return decompress_impl<F32>(input, input_bytes, chunk_size, num_chunks, output, s);
        case BAGUA_DTYPE_F16: return decompress_impl<F16>(input, input_bytes, chunk_size, num_chunks, output, s);
        case BAGUA_DTYPE_BF16: return decompress_impl<BF16>(input, input_bytes, chunk_size, num_chunks, output, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_minmax_u8_compress_stage(int stage, int dtype, const void* input, int input_num_element, int chunk_size,
                                   int num_chunks, uint8_t* output, size_t output_bytes, void* workspace,
                                   size_t workspace_bytes, int target_chunk, bagua_stream_t stream) {
    if (stage != 1 && stage != 2 && stage != 5) return BAGUA_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return compress_impl<F32>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                      workspace, workspace_bytes, target_chunk, s, stage);
        case BAGUA_DTYPE_F16:
            return compress_impl<F16>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                      workspace, workspace_bytes, target_chunk, s, stage);
        case BAGUA_DTYPE_BF16:
            return compress_impl<BF16>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                       workspace, workspace_bytes, target_chunk, s, stage);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_minmax_u8_reduce_requantize(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                      int num_chunks, void* tensor, int average, uint8_t* output, size_t output_bytes,
                                      int target_chunk, void* workspace, size_t workspace_bytes,
                                      bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return reduce_requantize_impl<F32>(input, input_bytes, chunk_size, num_chunks, tensor, average, output,
                                               output_bytes, target_chunk, workspace, workspace_bytes, s);
        case BAGUA_DTYPE_F16:
            return reduce_requantize_impl<F16>(input, input_bytes, chunk_size, num_chunks, tensor, average, output,
                                               output_bytes, target_chunk, workspace, workspace_bytes, s);
        case BAGUA_DTYPE_BF16:
            return reduce_requantize_impl<BF16>(input, input_bytes, chunk_size, num_chunks, tensor, average, output,
                                                output_bytes, target_chunk, workspace, workspace_bytes, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_minmax_u8_reduce_requantize_final(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                            int num_chunks, void* tensor, int average, uint8_t* output,
                                            size_t output_bytes, int target_chunk, void* workspace,
                                            size_t workspace_bytes, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (!tensor) return BAGUA_ERR_INVALID_ARG;
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return reduce_requantize_impl<F32>(input, input_bytes, chunk_size, num_chunks, nullptr, average, output,
                                               output_bytes, target_chunk, workspace, workspace_bytes, s, tensor);
        case BAGUA_DTYPE_F16:
            return reduce_requantize_impl<F16>(input, input_bytes, chunk_size, num_chunks, nullptr, average, output,
                                               output_bytes, target_chunk, workspace, workspace_bytes, s, tensor);
        case BAGUA_DTYPE_BF16:
            return reduce_requantize_impl<BF16>(input, input_bytes, chunk_size, num_chunks, nullptr, average, output,
                                                output_bytes, target_chunk, workspace, workspace_bytes, s, tensor);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_minmax_u8_centralized_one_rank(int dtype, void* tensor, int num_elem, int average, void* workspace,
                                         size_t workspace_bytes, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32: return one_rank_impl<F32>(tensor, num_elem, average, workspace, workspace_bytes, s);
        case BAGUA_DTYPE_F16: return one_rank_impl<F16>(tensor, num_elem, average, workspace, workspace_bytes, s);
        case BAGUA_DTYPE_BF16: return one_rank_impl<BF16>(tensor, num_elem, average, workspace, workspace_bytes, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

// ---- pipelined all-reduce building blocks ---------------------------------
#define BAGUA_DTYPE_DISPATCH(dtype, call)                   \
    switch (dtype) {                                        \
        case BAGUA_DTYPE_F32: { using T = F32; return call; } \
        case BAGUA_DTYPE_F16: { using T = F16; return call; } \
        case BAGUA_DTYPE_BF16: { using T = BF16; return call; } \
    }                                                       \
    return BAGUA_ERR_UNSUPPORTED

int bagua_minmax_u8_piece_range(int chunk_size, int pieces, int piece, int* begin, int* end) {
    if (chunk_size < 0 || !piece_schedule_ok(pieces) || piece < 0 || piece >= piece_count(pieces) || !begin || !end)
        return BAGUA_ERR_INVALID_ARG;
    piece_range(chunk_size, pieces, piece, begin, end);
    return BAGUA_OK;
}

size_t bagua_minmax_u8_pipeline_workspace_bytes(int chunk_size, int pieces) {
    if (chunk_size < 0 || !piece_schedule_ok(pieces)) return 0;
    return (size_t)piece_count(pieces) * (size_t)piece_blocks(chunk_size, pieces, 4) * sizeof(uint2) + 256 +
           kPieceTablesBytes;
}

int bagua_minmax_u8_quantize_range(int dtype, const void* input, int input_num_element, int chunk_size,
                                   int num_chunks, uint8_t* output, size_t output_bytes, void* workspace,
                                   size_t workspace_bytes, int target_chunk, int elem_begin, int elem_end,
                                   bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    BAGUA_DTYPE_DISPATCH(dtype, compress_impl<T>(input, input_num_element, chunk_size, num_chunks, output,
                                                 output_bytes, workspace, workspace_bytes, target_chunk, s, 2,
                                                 elem_begin, elem_end));
}

int bagua_minmax_u8_decompress_range(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                     int num_chunks, void* output, int elem_begin, int elem_end,
                                     bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    BAGUA_DTYPE_DISPATCH(dtype, decompress_impl<T>(input, input_bytes, chunk_size, num_chunks, output, s, elem_begin,
                                                   elem_end));
}

int bagua_minmax_u8_reduce_piece(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size, int num_chunks,
                                 void* tensor, int average, int target_chunk, int pieces, int piece, void* workspace,
                                 size_t workspace_bytes, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    BAGUA_DTYPE_DISPATCH(dtype, reduce_piece_impl<T>(input, input_bytes, chunk_size, num_chunks, tensor, average,
                                                     target_chunk, pieces, piece, workspace, workspace_bytes, s));
}

int bagua_minmax_u8_reduce_requantize_piece(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                            int num_chunks, int average, uint8_t* output, size_t output_bytes,
                                            int target_chunk, int pieces, int piece, const void* workspace,
                                            size_t workspace_bytes, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    BAGUA_DTYPE_DISPATCH(dtype, reduce_requantize_piece_impl<T>(input, input_bytes, chunk_size, num_chunks, average,
                                                                output, output_bytes, target_chunk, pieces, piece,
                                                                workspace, workspace_bytes, s));
}

int bagua_minmax_u8_fold_piece_partials(int dtype, int chunk_size, int pieces, void* workspace, size_t workspace_bytes,
                                        bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    BAGUA_DTYPE_DISPATCH(dtype, fold_piece_partials_impl<T>(chunk_size, pieces, workspace, workspace_bytes, s));
}

int bagua_minmax_u8_requantize_pieces(int dtype, const void* tensor, int chunk_size, int num_chunks, uint8_t* output,
                                      size_t output_bytes, int target_chunk, int pieces, const void* workspace,
                                      size_t workspace_bytes, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    BAGUA_DTYPE_DISPATCH(dtype, requantize_pieces_impl<T>(tensor, chunk_size, num_chunks, output, output_bytes,
                                                          target_chunk, pieces, workspace, workspace_bytes, s));
}
int bagua_minmax_u8_requantize_piece(int dtype, const void* tensor, int chunk_size, int num_chunks, uint8_t* output,
                                     size_t output_bytes, int target_chunk, int pieces, int piece,
                                     const void* workspace, size_t workspace_bytes, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (chunk_size < 0 || !piece_schedule_ok(pieces) || piece < 0 || piece >= piece_count(pieces))
        return BAGUA_ERR_INVALID_ARG;
    int b, e;
    piece_range(chunk_size, pieces, piece, &b, &e);
    if (b == e && piece > 0) return BAGUA_OK;  // empty trailing piece: its bytes were written by the others
    BAGUA_DTYPE_DISPATCH(dtype, requantize_pieces_impl<T>(tensor, chunk_size, num_chunks, output, output_bytes,
                                                          target_chunk, pieces, workspace, workspace_bytes, s, b, e));
}
#undef BAGUA_DTYPE_DISPATCH

// ---- v1 surface (bagua_kernels.cu:661-689) --------------------------------
void compress_f32_to_uint8_host(float* input, int input_num_element, int chunk_size, int num_chunks,
                                uint8_t* output, size_t output_size, void* dev_buffer, size_t dev_size,
                                int target_chunk, bagua_stream_t stream) {
    v1_check(bagua_minmax_u8_compress(BAGUA_DTYPE_F32, input, input_num_element, chunk_size, num_chunks,
                                      output, output_size, dev_buffer, dev_size, target_chunk, stream),
             __FILE__, __LINE__);
}
void compress_f16_to_uint8_host(bagua_half_t* input, int input_num_element, int chunk_size, int num_chunks,
                                uint8_t* output, size_t output_size, void* dev_buffer, size_t dev_size,
                                int target_chunk, bagua_stream_t stream) {
    v1_check(bagua_minmax_u8_compress(BAGUA_DTYPE_F16, input, input_num_element, chunk_size, num_chunks,
                                      output, output_size, dev_buffer, dev_size, target_chunk, stream),
             __FILE__, __LINE__);
}
void compress_bf16_to_uint8_host(bagua_bf16_t* input, int input_num_element, int chunk_size, int num_chunks,
                                 uint8_t* output, size_t output_size, void* dev_buffer, size_t dev_size,
                                 int target_chunk, bagua_stream_t stream) {
    v1_check(bagua_minmax_u8_compress(BAGUA_DTYPE_BF16, input, input_num_element, chunk_size, num_chunks,
                                      output, output_size, dev_buffer, dev_size, target_chunk, stream),
             __FILE__, __LINE__);
}
void decompress_uint8_to_f32_host(uint8_t* input, size_t input_size, int chunk_size, int num_chunks,
                                  float* output, bagua_stream_t stream) {
    v1_check(bagua_minmax_u8_decompress(BAGUA_DTYPE_F32, input, input_size, chunk_size, num_chunks, output,
                                        stream),
             __FILE__, __LINE__);
}
void decompress_uint8_to_f16_host(uint8_t* input, size_t input_size, int chunk_size, int num_chunks,
                                  bagua_half_t* output, bagua_stream_t stream) {
    v1_check(bagua_minmax_u8_decompress(BAGUA_DTYPE_F16, input, input_size, chunk_size, num_chunks, output,
                                        stream),
             __FILE__, __LINE__);
}
void decompress_uint8_to_bf16_host(uint8_t* input, size_t input_size, int chunk_size, int num_chunks,
                                   bagua_bf16_t* output, bagua_stream_t stream) {
    v1_check(bagua_minmax_u8_decompress(BAGUA_DTYPE_BF16, input, input_size, chunk_size, num_chunks, output,
                                        stream),
             __FILE__, __LINE__);
}
// K:683-689: the reference returns cub's temp bytes; here: our partials workspace
size_t array_min_max_size_f32_host(float*, int, float*, bagua_stream_t) {
    return bagua_minmax_u8_workspace_bytes(0, kTargetBlocks);
}
size_t array_min_max_size_f16_host(bagua_half_t*, int, bagua_half_t*, bagua_stream_t) {
    return bagua_minmax_u8_workspace_bytes(0, kTargetBlocks);
}
size_t array_min_max_size_bf16_host(bagua_bf16_t*, int, bagua_bf16_t*, bagua_stream_t) {
    return bagua_minmax_u8_workspace_bytes(0, kTargetBlocks);
}

}  // extern "C"
