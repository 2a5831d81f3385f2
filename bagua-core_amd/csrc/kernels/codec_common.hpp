// codec_common.hpp — dtype traits and wave64 helpers shared by the gfx950
// codec kernels.  Numerics follow the reference kernels exactly
// (bagua-core-internal/kernels/bagua_kernels.cu, cited as K:line):
// every float expression is one IEEE binary32 op, round-to-nearest-even,
// denormals preserved; the library is compiled with -ffp-contract=off and
// correctly rounded f32 division (see Makefile).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bagua_kernels.h"

namespace bagua {

constexpr int kWave = 64;          // CDNA wavefront
constexpr int kBlock = 256;        // 4 waves per workgroup for the streaming kernels
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kSubtiles = 4;       // vectors in flight per lane per tile
constexpr int kMaxFusedChunks = 16;  // fused dequantise+reduce handles p <= 16

// The fused reduce kernels' dequantisation tables in global memory (reduce.hip): `in`,
// the p x 256 floats an earlier launch of the same op left (nullptr: build them);
// `out`, where workgroup 0 of this launch leaves its own (nullptr: nothing written)
struct FusedTables {
    const float* in = nullptr;
    float* out = nullptr;
};

// ----------------------------------------------------------------- dtypes --
struct F32 {
    using storage = float;
    static constexpr int kDtype = BAGUA_DTYPE_F32;
    __device__ static __forceinline__ float load(const storage* p, int64_t i) { return p[i]; }
    __device__ static __forceinline__ float to_f(storage v) { return v; }
    __device__ static __forceinline__ storage from_f(float v) { return v; }
    // K:306/359/369 (f16) and cub Traits<float>::Max (f32): reduction init
    __device__ static __forceinline__ float init_max() { return __int_as_float(0x7f7fffff); }
};

struct F16 {
    using storage = uint16_t;
    static constexpr int kDtype = BAGUA_DTYPE_F16;
    __device__ static __forceinline__ float to_f(storage v) {
        return (float)__builtin_bit_cast(_Float16, v);
    }
    __device__ static __forceinline__ float load(const storage* p, int64_t i) { return to_f(p[i]); }
    __device__ static __forceinline__ storage from_f(float v) {  // __float2half: RNE
        return __builtin_bit_cast(uint16_t, (_Float16)v);
    }
    __device__ static __forceinline__ float init_max() { return 65504.0f; }
};

struct BF16 {
    using storage = uint16_t;
    static constexpr int kDtype = BAGUA_DTYPE_BF16;
    __device__ static __forceinline__ float to_f(storage v) {
        return __uint_as_float((uint32_t)v << 16);
    }
    __device__ static __forceinline__ float load(const storage* p, int64_t i) { return to_f(p[i]); }
    __device__ static __forceinline__ storage from_f(float v) {  // RNE (v_cvt_pk_bf16_f32)
        return __builtin_bit_cast(uint16_t, (__bf16)v);
    }
    __device__ static __forceinline__ float init_max() { return __uint_as_float(0x7f7f0000u); }
};

// a float value as it reads back after a store to T (identity for f32): the
// reference materialises every decompressed value in a T tensor first
template <typename T>
__device__ __forceinline__ float as_stored(float f) {
    if constexpr (sizeof(typename T::storage) == 4) return f;
    else return T::to_f(T::from_f(f));
}

// ------------------------------------------------------ order-free min/max --
// Total-order key (-0 < +0).  Min runs in the space u = key - key(-inf) and
// max in u = key(+inf) - key, both as unsigned: any NaN wraps to a huge
// value and never wins, so the result is independent of reduction order.
__device__ __forceinline__ int32_t f2key(float f) {
    int32_t i = __float_as_int(f);
    return i ^ ((i >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float key2f(int32_t k) {
    return __int_as_float(k ^ ((k >> 31) & 0x7fffffff));
}
// All offset arithmetic is done in uint32 (wrapping, well defined): a signed
// int32 subtraction here overflows for half the float range.
constexpr uint32_t kKeyNegInf = 0x807fffffu;  // f2key(-inf) as bits
constexpr uint32_t kKeyPosInf = 0x7f800000u;  // f2key(+inf)

__device__ __forceinline__ uint32_t min_space_key(int32_t k) { return (uint32_t)k - kKeyNegInf; }
__device__ __forceinline__ uint32_t max_space_key(int32_t k) { return kKeyPosInf - (uint32_t)k; }
__device__ __forceinline__ uint32_t min_space(float f) { return min_space_key(f2key(f)); }
__device__ __forceinline__ uint32_t max_space(float f) { return max_space_key(f2key(f)); }
__device__ __forceinline__ float from_min_space(uint32_t u) { return key2f((int32_t)(u + kKeyNegInf)); }
__device__ __forceinline__ float from_max_space(uint32_t u) { return key2f((int32_t)(kKeyPosInf - u)); }

__device__ __forceinline__ uint32_t wave_umin(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, kWave));
    return v;
}

// --------------------------------------------------- MinMax quantisation --
// K:465-467 / K:491-493 with the reference's exact types.
struct QParams {
    float scale, lower_bound, upper_bound;
};

__device__ __forceinline__ QParams make_qparams(float mn, float mx) {
    const float eps = (float)1e-7;            // K:10
    float d = (mx - mn) + eps;
    QParams q;
    q.scale = (float)(255.0 / (double)d);     // `255.0 / (...)` is a double division
    q.upper_bound = __builtin_rintf(mx * q.scale);
    q.lower_bound = (float)((double)q.upper_bound - 255.0);
    return q;
}

// K:410-422; the float->uint8 conversion saturates (NaN -> 0), see DESIGN.md §3.
__device__ __forceinline__ uint32_t quant(float x, const QParams& q) {
    float level = __builtin_rintf(x * q.scale);
    level = __builtin_fminf(level, q.upper_bound);
    float v = level - q.lower_bound;
    v = __builtin_fminf(__builtin_fmaxf(v, 0.0f), 255.0f);
    return (uint32_t)v;
}

// The level quant() converts, before the conversion: always an integer, NaN or
// +-inf (rint results and lower_bound = ub - 255 are integers, so is their
// difference after rounding).
__device__ __forceinline__ float quant_level(float x, const QParams& q) {
    const float level = __builtin_fminf(__builtin_rintf(x * q.scale), q.upper_bound);
    return level - q.lower_bound;
}

// 4 quantised bytes packed LSB-first by v_cvt_pk_u8_f32, which converts AND places
// a byte in one instruction.  On integers, NaN and +-inf -- every value
// quant_level() produces -- it equals quant()'s saturating conversion
// (tools/cvt_probe.hip checks all such f32 bit patterns: 0 mismatches; on
// non-integers it rounds where the cast truncates, which cannot occur here).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t quant_pack4(float a, float b, float c, float d, const QParams& q) {
    // the products as two packed multiplies (v_pk_mul_f32: two IEEE products per lane)
    const f32x2 s2 = {q.scale, q.scale};
    const f32x2 p01 = f32x2{a, b} * s2, p23 = f32x2{c, d} * s2;
    const float ub = q.upper_bound, lb = q.lower_bound;
    uint32_t w = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_fminf(__builtin_rintf(p01.x), ub) - lb, 0, 0u);
    w = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_fminf(__builtin_rintf(p01.y), ub) - lb, 1, w);
    w = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_fminf(__builtin_rintf(p23.x), ub) - lb, 2, w);
    return __builtin_amdgcn_cvt_pk_u8_f32(__builtin_fminf(__builtin_rintf(p23.y), ub) - lb, 3, w);
}

// K:424-432
__device__ __forceinline__ float dequant(uint32_t b, const QParams& q) {
    return ((float)b + q.lower_bound) / q.scale;
}

// ---------------------------------------------- chunk summation order --
// block_y_reduce (K:171-194): partial sums s[y] = 0.0f + c[y] + c[y+BY] + ...
// are folded s[y] += s[y+h] for h = BY/2 .. 1; BY from the launch table K:504-529.
template <int BY>
__device__ __forceinline__ void tree_finish(float (&s)[BY]) {
#pragma unroll
    for (int h = BY / 2; h >= 1; h /= 2)
#pragma unroll
        for (int y = 0; y < h; ++y) s[y] = s[y] + s[y + h];
}
inline int reduce_by(int p) { return p <= 4 ? 2 : p <= 8 ? 4 : p <= 16 ? 8 : p <= 32 ? 16 : 32; }

// ------------------------------------------------------------ vectors ------
// One 16-byte vector of T: 4 x f32 or 8 x 16-bit.
template <typename T> struct Vec;
template <> struct Vec<F32> {
    static constexpr int N = 4;
    using out_bytes = uint32_t;  // N quantised bytes
};
template <> struct Vec<F16> {
    static constexpr int N = 8;
    using out_bytes = uint2;
};
template <> struct Vec<BF16> {
    static constexpr int N = 8;
    using out_bytes = uint2;
};

template <typename T>
__device__ __forceinline__ void unpack16(const uint4& r, float (&f)[Vec<T>::N]) {
    if constexpr (Vec<T>::N == 4) {
        f[0] = __uint_as_float(r.x); f[1] = __uint_as_float(r.y);
        f[2] = __uint_as_float(r.z); f[3] = __uint_as_float(r.w);
    } else {
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f[2 * i] = T::to_f((uint16_t)(w[i] & 0xffff));
            f[2 * i + 1] = T::to_f((uint16_t)(w[i] >> 16));
        }
    }
}

template <typename T>
__device__ __forceinline__ uint4 pack16(const float (&f)[Vec<T>::N]) {
    if constexpr (Vec<T>::N == 4) {
        return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]),
                          __float_as_uint(f[2]), __float_as_uint(f[3]));
    } else {
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            w[i] = (uint32_t)T::from_f(f[2 * i]) | ((uint32_t)T::from_f(f[2 * i + 1]) << 16);
        return make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// Start element j0 of the vectorised body of a (T-stream, byte-stream) pair:
// the T-stream at t_addr + j0*sizeof(T) must be 16-B aligned and the byte
// stream at byte_addr + j0 N-B aligned.  Among those, prefer the j0 that puts
// the byte stream on a 128-B line: the MinMax payload starts 32 B into its
// segment, and a 256-B wave access that straddles three lines instead of two
// cost ~20 % on both quantise and dequantise (measured).
// The j0 head elements run on the scalar path.  -1: no common alignment.
template <typename T>
__host__ __device__ __forceinline__ int common_alignment(uintptr_t t_addr, uintptr_t byte_addr) {
    constexpr int N = Vec<T>::N;
    constexpr int esz = (int)sizeof(typename T::storage);
    const int j1 = (int)((128 - byte_addr % 128) % 128);  // the only line-aligned start below 128
    if ((t_addr + (uintptr_t)j1 * esz) % 16 == 0) return j1;
    for (int j = 0; j < N; ++j)
        if (((t_addr + (uintptr_t)j * esz) % 16 == 0) && ((byte_addr + j) % N == 0)) return j;
    return -1;
}

// ------------------------------------------------ non-temporal accesses ----
// (the builtins need native vector types, not HIP_vector_type)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 nt_load16(const void* p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_store16(const uint4& v, void* p) {
    u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}
__device__ __forceinline__ uint2 nt_load8(const void* p) {
    const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ void nt_store8(const uint2& v, void* p) {
    u32x2 w = {v.x, v.y};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x2*>(p));
}

// N quantised bytes -> one 4-B (f32) or 8-B (16-bit) access.  PLAIN stores on
// purpose: the compressed payload (1/4 of the input) then stays in L2 / the
// 256 MiB Infinity Cache for whoever reads it next (the decode, RCCL).  The
// whole-step cache-policy sweep (tools/policy_probe.hip) put
// this at 142 us vs 152 us with nt stores, although nt is faster in isolation.
template <typename T>
__device__ __forceinline__ void store_bytes(uint8_t* p, uint32_t (&b)[Vec<T>::N]) {
    if constexpr (Vec<T>::N == 4) {
        *reinterpret_cast<uint32_t*>(p) = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
    } else {
        uint2 v;
        v.x = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
        v.y = b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24);
        *reinterpret_cast<uint2*>(p) = v;
    }
}

// the N quantised bytes of one unpacked vector, as one 4-B (f32) / 8-B (16-bit)
// plain store (see store_bytes for the cache policy)
template <typename T>
__device__ __forceinline__ void quant_store_vec(const float (&f)[Vec<T>::N], const QParams& q, uint8_t* p) {
    if constexpr (Vec<T>::N == 4) {
        *reinterpret_cast<uint32_t*>(p) = quant_pack4(f[0], f[1], f[2], f[3], q);
    } else {
        uint2 v;
        v.x = quant_pack4(f[0], f[1], f[2], f[3], q);
        v.y = quant_pack4(f[4], f[5], f[6], f[7], q);
        *reinterpret_cast<uint2*>(p) = v;
    }
}

// raw payload word of one vector (nt load) and its split into N bytes
template <typename T>
__device__ __forceinline__ typename Vec<T>::out_bytes load_word(const uint8_t* p) {
    if constexpr (Vec<T>::N == 4) return __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p));
    else return nt_load8(p);
}
template <typename T>
__device__ __forceinline__ void split_bytes(const typename Vec<T>::out_bytes& x, uint32_t (&b)[Vec<T>::N]) {
    if constexpr (Vec<T>::N == 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) b[i] = (x >> (8 * i)) & 0xff;
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) { b[i] = (x.x >> (8 * i)) & 0xff; b[4 + i] = (x.y >> (8 * i)) & 0xff; }
    }
}

template <typename T>
__device__ __forceinline__ void load_bytes(const uint8_t* p, uint32_t (&b)[Vec<T>::N]) {
    if constexpr (Vec<T>::N == 4) {
        const uint32_t x = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p));
#pragma unroll
        for (int i = 0; i < 4; ++i) b[i] = (x >> (8 * i)) & 0xff;
    } else {
        const uint2 x = nt_load8(p);
#pragma unroll
        for (int i = 0; i < 4; ++i) { b[i] = (x.x >> (8 * i)) & 0xff; b[4 + i] = (x.y >> (8 * i)) & 0xff; }
    }
}

// --------------------------------------------------- dequantisation tables --
// A segment's payload byte has 256 possible values, so a workgroup evaluates
// dequant() once per value into LDS and each element becomes one table read
// instead of a correctly rounded f32 division (~10 VALU ops).  Entries are
// computed by the very same expression, so results are bit-identical.
// Stored form: the T bits the reference's decompress writes (f32 bits, or the
// 16-bit pattern zero-extended).
template <typename T>
__device__ __forceinline__ uint32_t stored_bits(float f) {
    if constexpr (sizeof(typename T::storage) == 4) return __float_as_uint(f);
    else return (uint32_t)T::from_f(f);
}
template <typename T>
__device__ __forceinline__ float from_stored_bits(uint32_t u) {
    if constexpr (sizeof(typename T::storage) == 4) return __uint_as_float(u);
    else return T::to_f((typename T::storage)u);
}
template <typename T>
__device__ __forceinline__ typename T::storage storage_from_bits(uint32_t u) {
    if constexpr (sizeof(typename T::storage) == 4) return __uint_as_float(u);
    else return (typename T::storage)u;
}
// one 16-B vector of T from N table entries (bits as stored)
template <typename T>
__device__ __forceinline__ uint4 pack_stored(const uint32_t (&u)[Vec<T>::N]) {
    if constexpr (Vec<T>::N == 4) return make_uint4(u[0], u[1], u[2], u[3]);
    else return make_uint4(u[0] | (u[1] << 16), u[2] | (u[3] << 16), u[4] | (u[5] << 16), u[6] | (u[7] << 16));
}

template <typename T>
__device__ __forceinline__ QParams read_header(const uint8_t* seg) {
    using S = typename T::storage;
    S hmn, hmx;
    __builtin_memcpy(&hmn, seg, sizeof(S));               // K:488-489 (header as T)
    __builtin_memcpy(&hmx, seg + sizeof(S), sizeof(S));
    return make_qparams(T::to_f(hmn), T::to_f(hmx));
}

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & (kWave - 1)); }

}  // namespace bagua
