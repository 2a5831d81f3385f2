// reduce.hip — chunk reduction (the scatter-reduce step of the compressed
// all-reduce) for gfx950.
//
// Reference: reduce_chunk_inplace<bx,by,T,avg> (bagua_kernels.cu:373-400)
// with block_y_reduce (:171-194) and the block_dim_y table (:502-531).  The
// reference spreads the p chunk reads over `by` threads and sums them through
// shared memory; here ONE lane owns a 16-byte column of all p chunks and
// reproduces exactly the same float summation tree in registers:
//   s[y] = 0.0f + c[y] + c[y+by] + ...   (y < by, by = f(p))
//   s[y] += s[y+h] for h = by/2 .. 1
// so results are bit-identical while every load is a coalesced 16-B vector
// and no LDS or barrier is needed.
//
// The fused variant dequantises p MinMax-UInt8 segments on the fly (the
// alltoall receive buffer) and reduces them in the same order —
// bit-identical to decompress_from + reduce_{mean,sum}_inplace — writing
// only the reduced chunk (reads p*cs bytes instead of 5*p*cs*4/4 ...).  It
// optionally emits min/max partials of the result so requantising the own
// chunk needs no extra pass over it.
#include "codec_common.hpp"
#include "launch_util.hpp"

namespace bagua {

// K:152-169 __from_float: the mean is a / n.  For n = 2^k the reciprocal is exact,
// so a * 2^-k is the same correctly rounded value as a / 2^k (also for NaN, +-inf,
// +-0 and denormal results): one multiply instead of a correctly rounded division
// (~10 VALU ops per element).  AV: 0 = sum, 1 = / p, 2 = * (1/p) for p = 2^k.
template <int AV>
__device__ __forceinline__ float avg_finish(float s, float pf, float inv) {
    if constexpr (AV == 0) return s;
    else if constexpr (AV == 1) return s / pf;
    else return s * inv;
}
inline int avg_mode(int average, int p) { return !average ? 0 : (p > 0 && (p & (p - 1)) == 0) ? 2 : 1; }



// ---------------------------------------------------------------- plain ----
template <typename T, int BY, int AV, bool VEC>
__global__ __launch_bounds__(kBlock) void reduce_chunks_kernel(typename T::storage* __restrict__ x,
                                                                int64_t cs, int p, int target) {
    using S = typename T::storage;
    constexpr int N = VEC ? Vec<T>::N : 1;
    const int64_t nitems = VEC ? cs / N : cs;
    const float pf = (float)p;
    const float inv = 1.0f / pf;  // exact when AV == 2
    S* dst = x + (int64_t)target * cs;
    for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < nitems; v += (int64_t)gridDim.x * kBlock) {
        float s[N][BY];
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
            for (int y = 0; y < BY; ++y) s[i][y] = 0.0f;
        for (int r = 0; r * BY < p; ++r) {
#pragma unroll
            for (int y = 0; y < BY; ++y) {
                const int c = r * BY + y;
                if (c >= p) break;
                if constexpr (VEC) {
                    const uint4 raw = *reinterpret_cast<const uint4*>(x + (int64_t)c * cs + v * N);
                    float f[Vec<T>::N];
                    unpack16<T>(raw, f);
#pragma unroll
                    for (int i = 0; i < N; ++i) s[i][y] = s[i][y] + f[i];
                } else {
                    s[0][y] = s[0][y] + T::to_f(x[(int64_t)c * cs + v]);
                }
            }
        }
        float o[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            tree_finish<BY>(s[i]);
            o[i] = avg_finish<AV>(s[i][0], pf, inv);  // K:152-169 __from_float: a / n
        }
        if constexpr (VEC) {
            float f[Vec<T>::N];
#pragma unroll
            for (int i = 0; i < N; ++i) f[i] = o[i];
            *reinterpret_cast<uint4*>(dst + v * N) = pack16<T>(f);
        } else {
            dst[v] = T::from_f(o[0]);
        }
    }
    if constexpr (VEC) {  // ragged tail (< N elements), scalar
        if (blockIdx.x == 0 && threadIdx.x < cs - nitems * N) {
            const int64_t j = nitems * N + threadIdx.x;
            float s[BY];
#pragma unroll
            for (int y = 0; y < BY; ++y) s[y] = 0.0f;
            for (int c = 0; c < p; ++c) {
                const int y = c % BY;
                s[y] = s[y] + T::to_f(x[(int64_t)c * cs + j]);
            }
            tree_finish<BY>(s);
            dst[j] = T::from_f(avg_finish<AV>(s[0], pf, inv));
        }
    }
}


template <typename T, int BY, int AV>
static void launch_reduce(typename T::storage* x, int64_t cs, int p, int target, hipStream_t s) {
    // one lane keeps N x BY partial sums in registers: vectorise only while that stays small
    constexpr bool kVecFits = Vec<T>::N * BY <= 64;
    const bool vec = kVecFits && ((uintptr_t)x % 16 == 0) &&
                     ((cs * (int64_t)sizeof(typename T::storage)) % 16 == 0);
    const int64_t items = vec ? cs / Vec<T>::N : cs;
    int64_t blocks = (items + kBlock - 1) / kBlock;
    if (blocks > kTargetBlocks) blocks = kTargetBlocks;
    if (blocks < 1) blocks = 1;
    if constexpr (kVecFits) {
        if (vec) {
            launch((reduce_chunks_kernel<T, BY, AV, true>), dim3(blocks), dim3(kBlock), 0, s, x, cs, p,
                               target);
            return;
        }
    }
        launch((reduce_chunks_kernel<T, BY, AV, false>), dim3(blocks), dim3(kBlock), 0, s, x, cs, p, target);
}

template <typename T, int AV>
static void dispatch_reduce(typename T::storage* x, int64_t cs, int p, int target, hipStream_t s) {
    switch (reduce_by(p)) {
        case 2: launch_reduce<T, 2, AV>(x, cs, p, target, s); break;
        case 4: launch_reduce<T, 4, AV>(x, cs, p, target, s); break;
        case 8: launch_reduce<T, 8, AV>(x, cs, p, target, s); break;
        case 16: launch_reduce<T, 16, AV>(x, cs, p, target, s); break;
        default: launch_reduce<T, 32, AV>(x, cs, p, target, s); break;
    }
}

template <typename T>
static int reduce_impl(void* x, int cs, int p, int target, int average, hipStream_t s) {
    if (!x || cs < 0 || p <= 0 || target < 0 || target >= p) return BAGUA_ERR_INVALID_ARG;
    using S = typename T::storage;
    switch (avg_mode(average, p)) {
        case 0: dispatch_reduce<T, 0>(static_cast<S*>(x), cs, p, target, s); break;
        case 1: dispatch_reduce<T, 1>(static_cast<S*>(x), cs, p, target, s); break;
        default: dispatch_reduce<T, 2>(static_cast<S*>(x), cs, p, target, s); break;
    }
    return check_launch();
}

// ---------------------------------------------- fused dequantise + reduce --
// Each lane reduces Q output vectors per step, taken at block stride so every
// load (N payload bytes of one segment) and every 16-B store of a wave is
// contiguous; Q = 64 / (N * BY) keeps BY x Q x N = 64 payload bytes in flight
// per lane (and 64 accumulators) for every p.  Summation follows the
// reference's tree order (block_y_reduce, K:171-194).
template <typename T, int BY>
constexpr int fused_q() {
    return (64 / (Vec<T>::N * BY)) < 1 ? 1 : 64 / (Vec<T>::N * BY);
}

// dequantisation tables of the p segments in LDS: lut[c][b] = byte b of segment
// c dequantised and rounded to T, as the reference stores it before reducing
// (codec_common.hpp "dequantisation tables")
template <typename T>
__device__ __forceinline__ void build_luts(const uint8_t* in, int64_t chunk_offset, int p, QParams* qp,
                                           float (*lut)[256]) {
    using S = typename T::storage;
    for (int c = threadIdx.x; c < p; c += kBlock) {
        const uint8_t* seg = in + (int64_t)c * chunk_offset;
        S hmn, hmx;
        __builtin_memcpy(&hmn, seg, sizeof(S));
        __builtin_memcpy(&hmx, seg + sizeof(S), sizeof(S));
        qp[c] = make_qparams(T::to_f(hmn), T::to_f(hmx));
    }
    __syncthreads();
    for (int i = threadIdx.x; i < p * 256; i += kBlock) lut[i >> 8][i & 255] = as_stored<T>(dequant(i & 255, qp[i >> 8]));
    __syncthreads();
}

// the p dequantisation tables of an earlier launch of the same op (every piece of one op
// dequantises the same p segment headers): copied from `tab` into LDS instead of p x 256
// correctly rounded divisions per workgroup
__device__ __forceinline__ void load_luts(const float* __restrict__ tab, int p, float (*lut)[256]) {
    for (int i = threadIdx.x; i < p * 256; i += kBlock) lut[i >> 8][i & 255] = tab[i];
    __syncthreads();
}

// The reduced chunk, tile by tile: every full 16-B vector v of the result goes
// to vec(v, packed T vector), each element j of the ragged tail (< N elements,
// workgroup 0) to tail(j, value rounded to T).  `base` = payload byte e0 of
// segment 0.  Summation follows the reference's tree order (block_y_reduce,
// K:171-194), then / p for the mean (K:152-169 __from_float).
// PF > 0: p is known at compile time (PF = 1: no second, duplicate load per vector
// for the BY = 2 tree of a single segment)
template <typename T, int BY, int AV, int PF, typename VecF, typename TailF>
__device__ __forceinline__ void reduce_tiles(const uint8_t* base, int64_t chunk_offset, int64_t cs, int p_rt,
                                             const float (*lut)[256], VecF&& vec, TailF&& tail) {
    const int p = PF > 0 ? PF : p_rt;
    constexpr int N = Vec<T>::N;
    constexpr int Q = fused_q<T, BY>();
    const float pf = (float)p;
    const float inv = 1.0f / pf;  // exact when AV == 2
    // fast path: every segment's payload N-byte aligned (checked on host)
    const int64_t nvec = cs / N;
    // a 32-bit block-tile counter from blockIdx: wave-uniform to the compiler, so the loop and
    // the full-tile test are scalar (an int64 tile index ended up in VGPRs, with exec-mask
    // loop control)
    const int ntiles = (int)((nvec + (int64_t)kBlock * Q - 1) / ((int64_t)kBlock * Q));
    for (int bt = blockIdx.x; bt < ntiles; bt += gridDim.x) {
        const int64_t tile = (int64_t)bt * kBlock * Q;
        const bool full = tile + (int64_t)kBlock * Q <= nvec;
        float s[Q][N][BY];
#pragma unroll
        for (int q = 0; q < Q; ++q)
#pragma unroll
            for (int i = 0; i < N; ++i)
#pragma unroll
                for (int y = 0; y < BY; ++y) s[q][i][y] = 0.0f;
        for (int r = 0; r * BY < p; ++r) {
            typename Vec<T>::out_bytes w[BY][Q];
            if (full) {  // unconditional loads: all BY x Q in flight before the first use
#pragma unroll
                for (int y = 0; y < BY; ++y)
#pragma unroll
                    for (int q = 0; q < Q; ++q) {
                        const int c = r * BY + y < p ? r * BY + y : p - 1;
                        w[y][q] = load_word<T>(base + (int64_t)c * chunk_offset +
                                               (tile + q * kBlock + threadIdx.x) * N);
                    }
            } else {
#pragma unroll
                for (int y = 0; y < BY; ++y)
#pragma unroll
                    for (int q = 0; q < Q; ++q) {
                        const int64_t v = tile + q * kBlock + threadIdx.x;
                        const int c = r * BY + y;
                        if (c < p && v < nvec) w[y][q] = load_word<T>(base + (int64_t)c * chunk_offset + v * N);
                    }
            }
#pragma unroll
            for (int y = 0; y < BY; ++y) {
                const int c = r * BY + y;
                if (c >= p) break;
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    uint32_t b[N];
                    split_bytes<T>(w[y][q], b);
#pragma unroll
                    for (int i = 0; i < N; ++i) s[q][i][y] = s[q][i][y] + lut[c][b[i]];
                }
            }
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int64_t v = tile + q * kBlock + threadIdx.x;
            if (!full && v >= nvec) continue;
            float o[N];
#pragma unroll
            for (int i = 0; i < N; ++i) {
                tree_finish<BY>(s[q][i]);
                o[i] = avg_finish<AV>(s[q][i][0], pf, inv);
            }
            vec(v, pack16<T>(o));
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < cs - nvec * N) {  // ragged tail (< N elements)
        const int64_t j = nvec * N + threadIdx.x;
        float s[BY];
#pragma unroll
        for (int y = 0; y < BY; ++y) s[y] = 0.0f;
        for (int c = 0; c < p; ++c) {
            const int y = c % BY;
            s[y] = s[y] + lut[c][base[(int64_t)c * chunk_offset + j]];
        }
        tree_finish<BY>(s);
        tail(j, T::from_f(avg_finish<AV>(s[0], pf, inv)));
    }
}

// the workgroup's {min, max} keys -> partials[blockIdx.x]
__device__ __forceinline__ void store_block_partial(uint32_t lo, uint32_t hi, uint2* partials) {
    lo = wave_umin(lo);
    hi = wave_umin(hi);
    __shared__ uint32_t red[2][kWavesPerBlock];
    const int w = threadIdx.x / kWave;
    if (lane_id() == 0) { red[0][w] = lo; red[1][w] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 1; i < kWavesPerBlock; ++i) { lo = min(lo, red[0][i]); hi = min(hi, red[1][i]); }
        partials[blockIdx.x] = make_uint2(lo, hi);
    }
}

// STORE: write the reduced chunk to `out`; PARTIALS: emit the min/max partials of
// its values as stored in T (what the requantiser reads back).  !STORE needs
// PARTIALS: the requantise then recomputes the values (dequant_reduce_quantize_kernel).
// tab_in: tables of an earlier launch of the op (nullptr: build them); tab_out: workgroup 0
// leaves its tables there for the later launches (nullptr: nothing written)
template <typename T, int BY, int AV, bool PARTIALS, bool STORE = true, int PF = 0>
__global__ __launch_bounds__(kBlock) void dequant_reduce_kernel(
    const uint8_t* __restrict__ in, int64_t chunk_offset, int64_t e0, int64_t cs, int p,
    typename T::storage* __restrict__ out, uint2* __restrict__ partials, const float* __restrict__ tab_in,
    float* __restrict__ tab_out) {
    // reduces elements [e0, e0 + cs) of the chunk (`out` points at element e0)
    using S = typename T::storage;
    constexpr int N = Vec<T>::N;
    static_assert(STORE || PARTIALS, "a pass that neither stores nor reduces does nothing");
    // reduce_by(p) = BY keeps p <= 2 BY: tables for 2 BY segments (4 KiB at p <= 4)
    __shared__ QParams qp[2 * BY];
    __shared__ float lut[2 * BY][256];
    if (tab_in) {
        load_luts(tab_in, p, lut);
    } else {
        build_luts<T>(in, chunk_offset, p, qp, lut);
        if (tab_out && blockIdx.x == 0)
            for (int i = threadIdx.x; i < p * 256; i += kBlock) tab_out[i] = lut[i >> 8][i & 255];
    }
    uint32_t lo = min_space(T::init_max()), hi = max_space(-T::init_max());
    reduce_tiles<T, BY, AV, PF>(
        in + 32 + e0, chunk_offset, cs, p, lut,
        [&](int64_t v, const uint4& packed) {
            if constexpr (STORE) *reinterpret_cast<uint4*>(out + v * N) = packed;
            if constexpr (PARTIALS) {
                float st[N];
                unpack16<T>(packed, st);
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    const int32_t k = f2key(st[i]);  // NaN wraps to a huge key in both spaces
                    lo = min(lo, min_space_key(k));
                    hi = min(hi, max_space_key(k));
                }
            }
        },
        [&](int64_t j, S o) {
            if constexpr (STORE) out[j] = o;
            if constexpr (PARTIALS) {
                const int32_t k = f2key(T::to_f(o));
                lo = min(lo, min_space_key(k));
                hi = min(hi, max_space_key(k));
            }
        });
    if constexpr (PARTIALS) store_block_partial(lo, hi, partials);
}

// Requantise the own chunk without reading a stored copy of it: fold the min/max
// partials the partials-only pass emitted, then recompute every reduced value from
// the p received segments (the same LDS tables and summation tree, so the same T
// values bit for bit) and quantise it into the payload of segment `seg` (header and
// slack included) -- the bytes minmax_quantize_kernel writes from the stored chunk.
// Reads p*cs payload bytes instead of the stored chunk's cs*sizeof(T) (and saves its
// write), so it pays for p < 2*sizeof(T).
//
// FINAL: also write the decompressed requantised chunk (what the op's final
// decompress writes there, minmax_dequantize_kernel's table and nt stores) to
// `final_out` -- one rank's op then needs no final decompress launch -- and, with
// seg == nullptr, skip the segment (nothing reads it: one rank gathers nothing;
// plain stores of it left 268 MB dirty in the Infinity Cache in front of the next
// 1 GiB encode, +40 us, nt stores cost the kernel +76 us).
//
// A range [e0, e0 + cs) of the chunk (cs_total elements; the pipelined op's pieces):
// the range at element 0 writes the header, the one ending at cs_total the slack.
template <typename T, int BY, int AV, int PF = 0, bool FINAL = false>
__global__ __launch_bounds__(kBlock) void dequant_reduce_quantize_kernel(
    const uint8_t* __restrict__ in, int64_t chunk_offset, int64_t cs, int p, const uint2* __restrict__ partials,
    int npartials, uint8_t* __restrict__ seg, int64_t seg_bytes, typename T::storage* __restrict__ final_out,
    int64_t e0, int64_t cs_total, const float* __restrict__ tab_in) {
    using S = typename T::storage;
    constexpr int N = Vec<T>::N;
    __shared__ QParams qp[2 * BY];  // p <= 2 BY, as in dequant_reduce_kernel
    __shared__ float lut[2 * BY][256];
    uint32_t lo = 0xffffffffu, hi = 0xffffffffu;
    for (int i = threadIdx.x; i < npartials; i += kBlock) {
        const uint2 pr = partials[i];
        lo = min(lo, pr.x);
        hi = min(hi, pr.y);
    }
    lo = wave_umin(lo);
    hi = wave_umin(hi);
    __shared__ uint32_t red[2][kWavesPerBlock];
    const int w = threadIdx.x / kWave;
    if (lane_id() == 0) { red[0][w] = lo; red[1][w] = hi; }
    if (tab_in) load_luts(tab_in, p, lut);  // their barriers publish red[][] too
    else build_luts<T>(in, chunk_offset, p, qp, lut);
#pragma unroll
    for (int i = 0; i < kWavesPerBlock; ++i) { lo = min(lo, red[0][i]); hi = min(hi, red[1][i]); }
    const float mn = from_min_space(lo), mx = from_max_space(hi);  // exact in T (header, K:462-463)
    const QParams q = make_qparams(mn, mx);
    __shared__ uint32_t lut2[FINAL ? 256 : 1];  // stored T bits of every byte value (the final decompress)
    if constexpr (FINAL) {
        static_assert(kBlock == 256, "one table entry per thread");
        lut2[threadIdx.x] = stored_bits<T>(dequant(threadIdx.x, q));
        __syncthreads();
    }
    if (blockIdx.x == 0 && (!FINAL || seg)) {
        const int t = threadIdx.x;
        if (t < 32 && e0 == 0) {  // header {T min, T max, zero gap}
            const uint32_t bmn = sizeof(S) == 4 ? __float_as_uint(mn) : (uint32_t)T::from_f(mn);
            const uint32_t bmx = sizeof(S) == 4 ? __float_as_uint(mx) : (uint32_t)T::from_f(mx);
            uint32_t hb = 0;
            if (t < (int)sizeof(S)) hb = (bmn >> (8 * t)) & 0xff;
            else if (t < 2 * (int)sizeof(S)) hb = (bmx >> (8 * (t - (int)sizeof(S)))) & 0xff;
            seg[t] = (uint8_t)hb;
        }
        if (e0 + cs == cs_total)
            for (int64_t j = 32 + cs_total + t; j < seg_bytes; j += kBlock) seg[j] = 0;  // slack
    }
    uint8_t* payload = seg ? seg + 32 + e0 : nullptr;  // FINAL without a segment writes no payload
    reduce_tiles<T, BY, AV, PF>(
        in + 32 + e0, chunk_offset, cs, p, lut,
        [&](int64_t v, const uint4& packed) {
            float st[N];
            unpack16<T>(packed, st);
            if constexpr (!FINAL) {
                quant_store_vec<T>(st, q, payload + v * N);
            } else {
                typename Vec<T>::out_bytes w;
                if constexpr (N == 4) w = quant_pack4(st[0], st[1], st[2], st[3], q);
                else w = make_uint2(quant_pack4(st[0], st[1], st[2], st[3], q), quant_pack4(st[4], st[5], st[6], st[7], q));
                if (seg) *reinterpret_cast<typename Vec<T>::out_bytes*>(payload + v * N) = w;  // plain (store_bytes)
                uint32_t b[N];
                split_bytes<T>(w, b);
#pragma unroll
                for (int i = 0; i < N; ++i) b[i] = lut2[b[i]];
                nt_store16(pack_stored<T>(b), final_out + v * N);
            }
        },
        [&](int64_t j, S o) {
            const uint32_t b = quant(T::to_f(o), q);
            if (!FINAL || seg) payload[j] = (uint8_t)b;
            if constexpr (FINAL) final_out[j] = storage_from_bits<T>(lut2[b]);
        });
}

// p = 2 known at compile time (the reduce_tiles PF parameter) for the op's recompute pair
// (partials-only reduce + requantise, its default at p = 2 in f32): the segment loop unrolls
// and every table row is an immediate LDS offset -- reduce 23.1 -> 18.3 us, requantise 31.6
// -> 28.4 us per 1 GiB piece (profiles/r06_reduce_pf/).  At p = 4 / 8 the same gained
// the recompute requantise 2 us and the storing reduce nothing, leaving the storing pair
// the faster there, so only p = 2 is built.  BAGUA_REDUCE_PF=0: the runtime-p kernels (A/B)
static bool pf_on() {
    static const bool on = tune_int("BAGUA_REDUCE_PF", 1) != 0;
    return on;
}

template <typename T, int BY, int AV>
static void launch_fused(const uint8_t* in, int64_t co, int64_t e0, int64_t cs, int p, typename T::storage* out,
                         uint2* partials, int blocks, hipStream_t s, FusedTables tb) {
    // out == nullptr: partials only (the requantise recomputes the chunk)
    if (p == 1 && BY == 2) {
        if (!out)
            launch((dequant_reduce_kernel<T, 2, AV, true, false, 1>), dim3(blocks), dim3(kBlock), 0, s, in, co, e0,
                   cs, p, out, partials, tb.in, tb.out);
        else if (partials)
            launch((dequant_reduce_kernel<T, 2, AV, true, true, 1>), dim3(blocks), dim3(kBlock), 0, s, in, co, e0,
                   cs, p, out, partials, tb.in, tb.out);
        else
            launch((dequant_reduce_kernel<T, 2, AV, false, true, 1>), dim3(blocks), dim3(kBlock), 0, s, in, co, e0,
                   cs, p, out, partials, tb.in, tb.out);
    } else if (!out) {
        if (BY == 2 && p == 2 && pf_on())  // the op's recompute reduce
            launch((dequant_reduce_kernel<T, 2, AV, true, false, 2>), dim3(blocks), dim3(kBlock), 0, s, in, co, e0,
                   cs, p, out, partials, tb.in, tb.out);
        else
            launch((dequant_reduce_kernel<T, BY, AV, true, false>), dim3(blocks), dim3(kBlock), 0, s, in, co, e0,
                   cs, p, out, partials, tb.in, tb.out);
    } else if (partials)
        launch((dequant_reduce_kernel<T, BY, AV, true>), dim3(blocks), dim3(kBlock), 0, s, in, co, e0,
                           cs, p, out, partials, tb.in, tb.out);
    else
        launch((dequant_reduce_kernel<T, BY, AV, false>), dim3(blocks), dim3(kBlock), 0, s, in, co,
                           e0, cs, p, out, partials, tb.in, tb.out);
}

template <typename T, int AV>
static void dispatch_fused(const uint8_t* in, int64_t co, int64_t e0, int64_t cs, int p, typename T::storage* out,
                           uint2* partials, int blocks, hipStream_t s, FusedTables tb) {
    switch (reduce_by(p)) {  // p <= kMaxFusedChunks (16) keeps BY <= 8
        case 2: launch_fused<T, 2, AV>(in, co, e0, cs, p, out, partials, blocks, s, tb); break;
        case 4: launch_fused<T, 4, AV>(in, co, e0, cs, p, out, partials, blocks, s, tb); break;
        default: launch_fused<T, 8, AV>(in, co, e0, cs, p, out, partials, blocks, s, tb); break;
    }
}

// range [e0, e0 + len) of a chunk of cs elements
struct RqRange {
    int64_t e0, len, cs;
};

template <typename T, int AV, int PF, bool FINAL>
static void launch_reduce_quantize(int by, const uint8_t* in, int64_t co, RqRange r, int p, const uint2* partials,
                                   int npartials, uint8_t* seg, int64_t seg_bytes, typename T::storage* final_out,
                                   int blocks, hipStream_t s, const float* tab_in) {
    if constexpr (PF > 0) {  // p known: only its own tree width (reduce_by(PF)) is built
        constexpr int BYP = PF <= 4 ? 2 : PF <= 8 ? 4 : 8;
        (void)by;
        launch((dequant_reduce_quantize_kernel<T, BYP, AV, PF, FINAL>), dim3(blocks), dim3(kBlock), 0, s, in, co,
               r.len, p, partials, npartials, seg, seg_bytes, final_out, r.e0, r.cs, tab_in);
    } else {
        switch (by) {
            case 2:
                launch((dequant_reduce_quantize_kernel<T, 2, AV, PF, FINAL>), dim3(blocks), dim3(kBlock), 0, s, in, co,
                       r.len, p, partials, npartials, seg, seg_bytes, final_out, r.e0, r.cs, tab_in);
                break;
            case 4:
                launch((dequant_reduce_quantize_kernel<T, 4, AV, PF, FINAL>), dim3(blocks), dim3(kBlock), 0, s, in, co,
                       r.len, p, partials, npartials, seg, seg_bytes, final_out, r.e0, r.cs, tab_in);
                break;
            default:
                launch((dequant_reduce_quantize_kernel<T, 8, AV, PF, FINAL>), dim3(blocks), dim3(kBlock), 0, s, in, co,
                       r.len, p, partials, npartials, seg, seg_bytes, final_out, r.e0, r.cs, tab_in);
                break;
        }
    }
}

template <typename T, int AV>
static void dispatch_reduce_quantize(const uint8_t* in, int64_t co, RqRange r, int p, const uint2* partials,
                                     int npartials, uint8_t* seg, int64_t seg_bytes, typename T::storage* final_out,
                                     int blocks, hipStream_t s, const float* tab_in) {
    if (p == 1) {  // one segment: the BY = 2 tree with p known (no duplicate loads)
        if (final_out)
            launch_reduce_quantize<T, AV, 1, true>(2, in, co, r, p, partials, npartials, seg, seg_bytes, final_out,
                                                   blocks, s, tab_in);
        else
            launch_reduce_quantize<T, AV, 1, false>(2, in, co, r, p, partials, npartials, seg, seg_bytes, nullptr,
                                                    blocks, s, tab_in);
        return;
    }
    if (final_out)
        launch_reduce_quantize<T, AV, 0, true>(reduce_by(p), in, co, r, p, partials, npartials, seg, seg_bytes,
                                               final_out, blocks, s, tab_in);
    else if (p == 2 && pf_on())  // the op's recompute requantise
        launch_reduce_quantize<T, AV, 2, false>(2, in, co, r, p, partials, npartials, seg, seg_bytes, nullptr,
                                                blocks, s, tab_in);
    else
        launch_reduce_quantize<T, AV, 0, false>(reduce_by(p), in, co, r, p, partials, npartials, seg, seg_bytes,
                                                nullptr, blocks, s, tab_in);
}

int fused_blocks(int64_t cs, int per_vec) {
    int64_t b = (cs / per_vec + kBlock - 1) / kBlock;
    if (b > kTargetBlocks) b = kTargetBlocks;
    return (int)(b < 1 ? 1 : b);
}

template <typename T>
int dequant_reduce_impl(const uint8_t* in, size_t in_bytes, int cs, int p, void* out, int average,
                        uint2* partials, int blocks, hipStream_t s, int e0, int e1, FusedTables tb) {
    // reduces elements [e0, e1) of the chunk whose element 0 is at `out`;
    // out == nullptr: partials only (nothing stored)
    using S = typename T::storage;
    if (!in || (!out && !partials) || cs < 0 || p <= 0 || e0 < 0 || e1 < e0 || e1 > cs) return BAGUA_ERR_INVALID_ARG;
    if (p > kMaxFusedChunks) return BAGUA_ERR_UNSUPPORTED;  // caller falls back to decompress + reduce
    const int64_t co = (int64_t)(in_bytes / (size_t)p);
    if (co < (int64_t)cs + 32) return BAGUA_ERR_INVALID_ARG;
    constexpr int N = Vec<T>::N;
    // vector path: out 16-B aligned and every segment payload N-byte aligned
    S* o = out ? static_cast<S*>(out) + e0 : nullptr;
    const bool aligned = ((uintptr_t)o % 16 == 0) && (((uintptr_t)in + 32 + e0) % N == 0) && (co % N == 0);
    if (!aligned) return BAGUA_ERR_UNSUPPORTED;  // caller falls back to decompress + reduce
    switch (avg_mode(average, p)) {
        case 0: dispatch_fused<T, 0>(in, co, e0, e1 - e0, p, o, partials, blocks, s, tb); break;
        case 1: dispatch_fused<T, 1>(in, co, e0, e1 - e0, p, o, partials, blocks, s, tb); break;
        default: dispatch_fused<T, 2>(in, co, e0, e1 - e0, p, o, partials, blocks, s, tb); break;
    }
    return check_launch();
}

// quantise the reduced chunk, recomputed from the p received segments, into `seg`
// (seg_bytes: the segment incl. header and slack), after dequant_reduce_impl with
// out == nullptr emitted `npartials` partials; `blocks` is this launch's grid.
// Elements [e0, e1) only (default: the whole chunk); final_chunk needs the whole chunk.
template <typename T>
int dequant_reduce_quantize_impl(const uint8_t* in, size_t in_bytes, int cs, int p, int average,
                                 const uint2* partials, int npartials, uint8_t* seg, int64_t seg_bytes, int blocks,
                                 hipStream_t s, void* final_chunk, int e0, int e1, const float* tab_in) {
    using S = typename T::storage;
    if (e1 < 0) e1 = cs;
    if (!in || !partials || (!seg && !final_chunk) || cs < 0 || p <= 0 || npartials < 1 || e0 < 0 || e1 < e0 ||
        e1 > cs || (final_chunk && (e0 != 0 || e1 != cs)))
        return BAGUA_ERR_INVALID_ARG;
    if (p > kMaxFusedChunks) return BAGUA_ERR_UNSUPPORTED;
    const int64_t co = (int64_t)(in_bytes / (size_t)p);
    if (co < (int64_t)cs + 32 || (seg && seg_bytes < (int64_t)cs + 32)) return BAGUA_ERR_INVALID_ARG;
    constexpr int N = Vec<T>::N;
    const bool aligned = (((uintptr_t)in + 32 + e0) % N == 0) && (co % N == 0) &&
                         (((uintptr_t)seg + 32 + e0) % N == 0) && ((uintptr_t)final_chunk % 16 == 0);
    if (!aligned) return BAGUA_ERR_UNSUPPORTED;
    S* const fo = static_cast<S*>(final_chunk);
    const RqRange r{e0, (int64_t)e1 - e0, cs};
    switch (avg_mode(average, p)) {
        case 0: dispatch_reduce_quantize<T, 0>(in, co, r, p, partials, npartials, seg, seg_bytes, fo, blocks, s, tab_in); break;
        case 1: dispatch_reduce_quantize<T, 1>(in, co, r, p, partials, npartials, seg, seg_bytes, fo, blocks, s, tab_in); break;
        default: dispatch_reduce_quantize<T, 2>(in, co, r, p, partials, npartials, seg, seg_bytes, fo, blocks, s, tab_in); break;
    }
    return check_launch();
}

template int dequant_reduce_impl<F32>(const uint8_t*, size_t, int, int, void*, int, uint2*, int, hipStream_t, int, int,
                                      FusedTables);
template int dequant_reduce_impl<F16>(const uint8_t*, size_t, int, int, void*, int, uint2*, int, hipStream_t, int, int,
                                      FusedTables);
template int dequant_reduce_impl<BF16>(const uint8_t*, size_t, int, int, void*, int, uint2*, int, hipStream_t, int,
                                       int, FusedTables);
template int dequant_reduce_quantize_impl<F32>(const uint8_t*, size_t, int, int, int, const uint2*, int, uint8_t*,
                                               int64_t, int, hipStream_t, void*, int, int, const float*);
template int dequant_reduce_quantize_impl<F16>(const uint8_t*, size_t, int, int, int, const uint2*, int, uint8_t*,
                                               int64_t, int, hipStream_t, void*, int, int, const float*);
template int dequant_reduce_quantize_impl<BF16>(const uint8_t*, size_t, int, int, int, const uint2*, int, uint8_t*,
                                                int64_t, int, hipStream_t, void*, int, int, const float*);

}  // namespace bagua

using namespace bagua;

extern "C" {

int bagua_reduce_chunks(int dtype, void* input, int chunk_size, int num_chunks, int target_chunk, int average,
                        bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32: return reduce_impl<F32>(input, chunk_size, num_chunks, target_chunk, average, s);
        case BAGUA_DTYPE_F16: return reduce_impl<F16>(input, chunk_size, num_chunks, target_chunk, average, s);
        case BAGUA_DTYPE_BF16: return reduce_impl<BF16>(input, chunk_size, num_chunks, target_chunk, average, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_minmax_u8_decompress_reduce(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                      int num_chunks, void* output, int average, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return dequant_reduce_impl<F32>(input, input_bytes, chunk_size, num_chunks, output, average, nullptr,
                                            fused_blocks(chunk_size, 4), s, 0, chunk_size, FusedTables{});
        case BAGUA_DTYPE_F16:
            return dequant_reduce_impl<F16>(input, input_bytes, chunk_size, num_chunks, output, average, nullptr,
                                            fused_blocks(chunk_size, 8), s, 0, chunk_size, FusedTables{});
        case BAGUA_DTYPE_BF16:
            return dequant_reduce_impl<BF16>(input, input_bytes, chunk_size, num_chunks, output, average, nullptr,
                                             fused_blocks(chunk_size, 8), s, 0, chunk_size, FusedTables{});
    }
    return BAGUA_ERR_UNSUPPORTED;
}

// ---- v1 surface (bagua_kernels.cu:646-660) --------------------------------
void reduce_mean_f32_inplace_host(float* input, int chunk_size, int num_chunks, int target_chunk,
                                  bagua_stream_t stream) {
    v1_check(bagua_reduce_chunks(BAGUA_DTYPE_F32, input, chunk_size, num_chunks, target_chunk, 1, stream),
             __FILE__, __LINE__);
}
void reduce_mean_f16_inplace_host(bagua_half_t* input, int chunk_size, int num_chunks, int target_chunk,
                                  bagua_stream_t stream) {
    v1_check(bagua_reduce_chunks(BAGUA_DTYPE_F16, input, chunk_size, num_chunks, target_chunk, 1, stream),
             __FILE__, __LINE__);
}
void reduce_sum_f32_inplace_host(float* input, int chunk_size, int num_chunks, int target_chunk,
                                 bagua_stream_t stream) {
    v1_check(bagua_reduce_chunks(BAGUA_DTYPE_F32, input, chunk_size, num_chunks, target_chunk, 0, stream),
             __FILE__, __LINE__);
}
void reduce_sum_f16_inplace_host(bagua_half_t* input, int chunk_size, int num_chunks, int target_chunk,
                                 bagua_stream_t stream) {
    v1_check(bagua_reduce_chunks(BAGUA_DTYPE_F16, input, chunk_size, num_chunks, target_chunk, 0, stream),
             __FILE__, __LINE__);
}
void reduce_mean_bf16_inplace_host(bagua_bf16_t* input, int chunk_size, int num_chunks, int target_chunk,
                                   bagua_stream_t stream) {
    v1_check(bagua_reduce_chunks(BAGUA_DTYPE_BF16, input, chunk_size, num_chunks, target_chunk, 1, stream),
             __FILE__, __LINE__);
}
void reduce_sum_bf16_inplace_host(bagua_bf16_t* input, int chunk_size, int num_chunks, int target_chunk,
                                  bagua_stream_t stream) {
    v1_check(bagua_reduce_chunks(BAGUA_DTYPE_BF16, input, chunk_size, num_chunks, target_chunk, 0, stream),
             __FILE__, __LINE__);
}

}  // extern "C"
