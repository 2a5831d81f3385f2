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



// ---------------------------------------------------------------- plain ----
template <typename T, int BY, bool AVG, bool VEC>
__global__ __launch_bounds__(kBlock) void reduce_chunks_kernel(typename T::storage* __restrict__ x,
                                                                int64_t cs, int p, int target) {
    using S = typename T::storage;
    constexpr int N = VEC ? Vec<T>::N : 1;
    const int64_t nitems = VEC ? cs / N : cs;
    const float pf = (float)p;
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
            o[i] = AVG ? s[i][0] / pf : s[i][0];  // K:152-169 __from_float: a / n
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
            dst[j] = T::from_f(AVG ? s[0] / pf : s[0]);
        }
    }
}


template <typename T, int BY, bool AVG>
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
            launch((reduce_chunks_kernel<T, BY, AVG, true>), dim3(blocks), dim3(kBlock), 0, s, x, cs, p,
                               target);
            return;
        }
    }
        launch((reduce_chunks_kernel<T, BY, AVG, false>), dim3(blocks), dim3(kBlock), 0, s, x, cs, p, target);
}

template <typename T, bool AVG>
static void dispatch_reduce(typename T::storage* x, int64_t cs, int p, int target, hipStream_t s) {
    switch (reduce_by(p)) {
        case 2: launch_reduce<T, 2, AVG>(x, cs, p, target, s); break;
        case 4: launch_reduce<T, 4, AVG>(x, cs, p, target, s); break;
        case 8: launch_reduce<T, 8, AVG>(x, cs, p, target, s); break;
        case 16: launch_reduce<T, 16, AVG>(x, cs, p, target, s); break;
        default: launch_reduce<T, 32, AVG>(x, cs, p, target, s); break;
    }
}

template <typename T>
static int reduce_impl(void* x, int cs, int p, int target, int average, hipStream_t s) {
    if (!x || cs < 0 || p <= 0 || target < 0 || target >= p) return BAGUA_ERR_INVALID_ARG;
    using S = typename T::storage;
    if (average) dispatch_reduce<T, true>(static_cast<S*>(x), cs, p, target, s);
    else dispatch_reduce<T, false>(static_cast<S*>(x), cs, p, target, s);
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

template <typename T, int BY, bool AVG, bool PARTIALS>
__global__ __launch_bounds__(kBlock) void dequant_reduce_kernel(
    const uint8_t* __restrict__ in, int64_t chunk_offset, int64_t e0, int64_t cs, int p,
    typename T::storage* __restrict__ out, uint2* __restrict__ partials) {
    // reduces elements [e0, e0 + cs) of the chunk (`out` points at element e0)
    using S = typename T::storage;
    constexpr int N = Vec<T>::N;
    constexpr int Q = fused_q<T, BY>();
    __shared__ QParams qp[kMaxFusedChunks];
    for (int c = threadIdx.x; c < p; c += kBlock) {
        const uint8_t* seg = in + (int64_t)c * chunk_offset;
        S hmn, hmx;
        __builtin_memcpy(&hmn, seg, sizeof(S));
        __builtin_memcpy(&hmx, seg + sizeof(S), sizeof(S));
        qp[c] = make_qparams(T::to_f(hmn), T::to_f(hmx));
    }
    __syncthreads();
    // dequantised value of every byte of every segment, as the reference stores
    // it in T before reducing (codec_common.hpp "dequantisation tables")
    __shared__ float lut[kMaxFusedChunks][256];
    for (int i = threadIdx.x; i < p * 256; i += kBlock) lut[i >> 8][i & 255] = as_stored<T>(dequant(i & 255, qp[i >> 8]));
    __syncthreads();
    const float pf = (float)p;
    uint32_t lo = min_space(T::init_max()), hi = max_space(-T::init_max());
    // fast path: every segment's payload N-byte aligned and out 16-B aligned (checked on host)
    const int64_t nvec = cs / N;
    const uint8_t* base = in + 32 + e0;
    for (int64_t tile = (int64_t)blockIdx.x * kBlock * Q; tile < nvec; tile += (int64_t)gridDim.x * kBlock * Q) {
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
                o[i] = AVG ? s[q][i][0] / pf : s[q][i][0];
            }
            const uint4 packed = pack16<T>(o);
            *reinterpret_cast<uint4*>(out + v * N) = packed;
            if constexpr (PARTIALS) {
                // min/max of the values as stored in T (what the requantiser reads back)
                float st[N];
                unpack16<T>(packed, st);
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    const int32_t k = f2key(st[i]);  // NaN wraps to a huge key in both spaces
                    lo = min(lo, min_space_key(k));
                    hi = min(hi, max_space_key(k));
                }
            }
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
        const S o = T::from_f(AVG ? s[0] / pf : s[0]);
        out[j] = o;
        if constexpr (PARTIALS) {
            const int32_t k = f2key(T::to_f(o));
            lo = min(lo, min_space_key(k));
            hi = min(hi, max_space_key(k));
        }
    }
    if constexpr (PARTIALS) {
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
}

template <typename T, int BY, bool AVG>
static void launch_fused(const uint8_t* in, int64_t co, int64_t e0, int64_t cs, int p, typename T::storage* out,
                         uint2* partials, int blocks, hipStream_t s) {
    if (partials)
        launch((dequant_reduce_kernel<T, BY, AVG, true>), dim3(blocks), dim3(kBlock), 0, s, in, co, e0,
                           cs, p, out, partials);
    else
        launch((dequant_reduce_kernel<T, BY, AVG, false>), dim3(blocks), dim3(kBlock), 0, s, in, co,
                           e0, cs, p, out, partials);
}

template <typename T, bool AVG>
static void dispatch_fused(const uint8_t* in, int64_t co, int64_t e0, int64_t cs, int p, typename T::storage* out,
                           uint2* partials, int blocks, hipStream_t s) {
    switch (reduce_by(p)) {  // p <= kMaxFusedChunks (16) keeps BY <= 8
        case 2: launch_fused<T, 2, AVG>(in, co, e0, cs, p, out, partials, blocks, s); break;
        case 4: launch_fused<T, 4, AVG>(in, co, e0, cs, p, out, partials, blocks, s); break;
        default: launch_fused<T, 8, AVG>(in, co, e0, cs, p, out, partials, blocks, s); break;
    }
}

int fused_blocks(int64_t cs, int per_vec) {
    int64_t b = (cs / per_vec + kBlock - 1) / kBlock;
    if (b > kTargetBlocks) b = kTargetBlocks;
    return (int)(b < 1 ? 1 : b);
}

template <typename T>
int dequant_reduce_impl(const uint8_t* in, size_t in_bytes, int cs, int p, void* out, int average,
                        uint2* partials, int blocks, hipStream_t s, int e0, int e1) {
    // reduces elements [e0, e1) of the chunk whose element 0 is at `out`
    using S = typename T::storage;
    if (!in || !out || cs < 0 || p <= 0 || e0 < 0 || e1 < e0 || e1 > cs) return BAGUA_ERR_INVALID_ARG;
    if (p > kMaxFusedChunks) return BAGUA_ERR_UNSUPPORTED;  // caller falls back to decompress + reduce
    const int64_t co = (int64_t)(in_bytes / (size_t)p);
    if (co < (int64_t)cs + 32) return BAGUA_ERR_INVALID_ARG;
    constexpr int N = Vec<T>::N;
    // vector path: out 16-B aligned and every segment payload N-byte aligned
    S* o = static_cast<S*>(out) + e0;
    const bool aligned = ((uintptr_t)o % 16 == 0) && (((uintptr_t)in + 32 + e0) % N == 0) && (co % N == 0);
    if (!aligned) return BAGUA_ERR_UNSUPPORTED;  // caller falls back to decompress + reduce
    if (average) dispatch_fused<T, true>(in, co, e0, e1 - e0, p, o, partials, blocks, s);
    else dispatch_fused<T, false>(in, co, e0, e1 - e0, p, o, partials, blocks, s);
    return check_launch();
}

template int dequant_reduce_impl<F32>(const uint8_t*, size_t, int, int, void*, int, uint2*, int, hipStream_t, int, int);
template int dequant_reduce_impl<F16>(const uint8_t*, size_t, int, int, void*, int, uint2*, int, hipStream_t, int, int);
template int dequant_reduce_impl<BF16>(const uint8_t*, size_t, int, int, void*, int, uint2*, int, hipStream_t, int, int);

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
                                            fused_blocks(chunk_size, 4), s, 0, chunk_size);
        case BAGUA_DTYPE_F16:
            return dequant_reduce_impl<F16>(input, input_bytes, chunk_size, num_chunks, output, average, nullptr,
                                            fused_blocks(chunk_size, 8), s, 0, chunk_size);
        case BAGUA_DTYPE_BF16:
            return dequant_reduce_impl<BF16>(input, input_bytes, chunk_size, num_chunks, output, average, nullptr,
                                             fused_blocks(chunk_size, 8), s, 0, chunk_size);
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
