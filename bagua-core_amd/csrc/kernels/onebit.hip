// onebit.hip — 1-bit sign + scale gradient codec for gfx950 (extension; the
// reference has only MinMaxUInt8).  Format: DESIGN.md §4.
//
// The bit layout is lane-native: one wave owns a 1024-element tile; element
// r = sub*256 + lane*4 + e of the tile is bit (sub*4+e) of the 16-bit field at
// byte 2*lane, i.e. each lane's 16 elements are one field it builds and reads
// alone (encode: compares + shifts, one shuffle to pair fields into dwords;
// decode: one 2-byte load and a sign-bit flip per element).  An earlier
// ballot layout (bit `lane` of word sub*4+e) cost 32 v_readlane per tile to
// decode.  Element loads/stores are 16 B (f32) / 8 B (16-bit) per lane, and a
// tile's 128 bit bytes are one coalesced wave access.
//
// scale = mean(|x|) with a FIXED summation tree (lane-local pairs, then a
// 64-lane xor butterfly per tile, then the same 1024-tree over the tile
// partials), so the encoder is single-pass over the input and its result is
// independent of grid size and bit-reproducible against the oracle.
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "codec_common.hpp"
#include "launch_util.hpp"

namespace bagua {

constexpr int kObTile = 1024;
constexpr int kObTileBytes = 128;
constexpr int kObFinalizeThreads = 1024;
// encode / decode grid caps: 64 B of loads in flight per lane (one tile per
// iteration for 32-bit types, two for 16-bit ones).  Round 1 picked 1024 encode
// workgroups over 2048 (profiles/r01_onebit_shape_sweep.jsonl); round 3 found
// one tile per wave better still (16384 workgroups for 2^26 f32 elements):
// encode 45.8 -> 43.8 us, decode 42.7 -> 42.0 us per 256 MiB
// (tools/grid_sweep.py, profiles/r03_grid_sweep.jsonl); round 4 kept one tile per
// wave up to 1 GiB buckets (65536 workgroups): 1 GiB encode 186 -> 176 us, decode
// 193 -> 190 us, 256 MiB unchanged (profiles/r04_onebit_shape_sweep.jsonl)
constexpr int kObEncodeBlocks = 65536;
constexpr int kObDecodeBlocks = 65536;

__device__ __forceinline__ int64_t ob_valid(int64_t in_num_elem, int64_t cs, int c) {
    int64_t r = in_num_elem - (int64_t)c * cs;
    return r < 0 ? 0 : (r < cs ? r : cs);
}

// 4 consecutive elements of T starting at p (vector load when 4*sizeof(T)-aligned)
template <typename T>
__device__ __forceinline__ void load4(const typename T::storage* p, int64_t j, int64_t n, bool vec, float (&f)[4]) {
    using S = typename T::storage;
    if (vec && j + 4 <= n) {
        if constexpr (sizeof(S) == 4) {
            const uint4 v = nt_load16(p + j);
            f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y);
            f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
        } else {
            const uint2 v = nt_load8(p + j);
            f[0] = T::to_f((uint16_t)(v.x & 0xffff)); f[1] = T::to_f((uint16_t)(v.x >> 16));
            f[2] = T::to_f((uint16_t)(v.y & 0xffff)); f[3] = T::to_f((uint16_t)(v.y >> 16));
        }
        return;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = (j + e < n) ? T::load(p, j + e) : 0.0f;
}

// 4 elements from one 16-B (f32) / 8-B (16-bit) load
template <typename T>
__device__ __forceinline__ void unpack4(const uint4& v, float (&f)[4]) {
    f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y);
    f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
}
template <typename T>
__device__ __forceinline__ void unpack4(const uint2& v, float (&f)[4]) {
    f[0] = T::to_f((uint16_t)(v.x & 0xffff)); f[1] = T::to_f((uint16_t)(v.x >> 16));
    f[2] = T::to_f((uint16_t)(v.y & 0xffff)); f[3] = T::to_f((uint16_t)(v.y >> 16));
}

template <typename T, bool NTS = true>
__device__ __forceinline__ void store4(typename T::storage* p, int64_t j, int64_t n, bool vec, const float (&f)[4]) {
    using S = typename T::storage;
    if (vec && j + 4 <= n) {
        if constexpr (sizeof(S) == 4) {
            const uint4 v = make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
            if constexpr (NTS) nt_store16(v, p + j);
            else *reinterpret_cast<uint4*>(p + j) = v;
        } else {
            uint2 v;
            v.x = (uint32_t)T::from_f(f[0]) | ((uint32_t)T::from_f(f[1]) << 16);
            v.y = (uint32_t)T::from_f(f[2]) | ((uint32_t)T::from_f(f[3]) << 16);
            if constexpr (NTS) nt_store8(v, p + j);
            else *reinterpret_cast<uint2*>(p + j) = v;
        }
        return;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (j + e < n) p[j + e] = T::from_f(f[e]);
}

// this wave's index in the grid, through readfirstlane so the compiler knows it (and every
// tile index and bound derived from it) is wave-uniform: scalar loop control and SGPR-based
// addresses instead of 64-bit VALU arithmetic and exec-mask branches per tile
__device__ __forceinline__ int64_t grid_wave() {
    return (int64_t)blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
}

// the 64-lane tree of the tile sum: s[l] += s[l^h], h = 32..1 (== s[l] + s[l+h])
__device__ __forceinline__ float wave_tree_sum(float s) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s = s + __shfl_xor(s, o, kWave);
    return s;
}

// The same tree with its result in lane 0 only (the streaming kernels store lane 0's):
// s[l] += s[l+h] for h = 32, 16 by swapping halves across lanes (gfx950's permlane swaps),
// h = 8..1 by DPP row shifts -- no LDS round trip per level, and 8 instructions where the
// shuffles above take ~36 plus six ds_bpermute waits.  Every lane of the wave must be active
__device__ __forceinline__ float wave_tree_sum_lane0(float s) {
    s = s + __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false)[1]);
    s = s + __uint_as_float(__builtin_amdgcn_permlane16_swap(__float_as_uint(s), __float_as_uint(s), false, false)[1]);
    s = s + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x108, 0xf, 0xf, false));  // row_shl:8
    s = s + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x104, 0xf, 0xf, false));  // row_shl:4
    s = s + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x102, 0xf, 0xf, false));  // row_shl:2
    s = s + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x101, 0xf, 0xf, false));  // row_shl:1
    return s;
}

// lane l + 1's value in even lanes l (an even lane and its odd neighbour share a DPP row)
__device__ __forceinline__ uint32_t odd_neighbour(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xf, 0xf, false);  // row_shl:1
}

// lane-local part of the tile tree for values a[sub][e]
__device__ __forceinline__ float lane_tree(const float (&a)[4][4]) {
    float q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = (a[k][0] + a[k][1]) + (a[k][2] + a[k][3]);
    return (q[0] + q[1]) + (q[2] + q[3]);
}

// ------------------------------------------------------------------------
// encode: bits + per-tile |x| partials, one wave per tile
// ------------------------------------------------------------------------
template <typename T, int TPI, bool NTL = true>
__global__ __launch_bounds__(kBlock) void onebit_encode_kernel(
    const typename T::storage* __restrict__ in, int64_t in_num_elem, int64_t cs, int target,
    uint8_t* __restrict__ out, int64_t chunk_offset, float* __restrict__ partials, int64_t tiles_per_chunk,
    int64_t t_begin, int64_t t_end) {
    using S = typename T::storage;
    const int c = target < 0 ? (int)blockIdx.y : target;
    const int64_t n = ob_valid(in_num_elem, cs, c);
    const S* src = in + (int64_t)c * cs;
    const bool vec = ((uintptr_t)src % (4 * sizeof(S))) == 0;
    uint8_t* bits = out + (int64_t)c * chunk_offset + 32;
    float* part = partials + (int64_t)blockIdx.y * tiles_per_chunk;
    const int lane = lane_id();
    const int64_t wave = grid_wave();
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    // a lane reads 4 consecutive elements per sub-tile: 16 B for f32 but only 8 B
    // for 16-bit types, so those take TPI = 2 tiles per iteration (64 B in flight
    // per lane either way)
    for (int64_t t0 = t_begin + wave * TPI; t0 < t_end; t0 += nwaves * TPI) {
        float a[TPI][4][4];
        if (vec && (t0 + TPI) * kObTile <= n) {
            // full tiles: every load issued unconditionally before any is used (a
            // guarded load gets its own s_waitcnt vmcnt(0) and the wave serialises)
            using L = std::conditional_t<sizeof(S) == 4, uint4, uint2>;  // 4 elements: 16 B (f32) / 8 B
            L raw[TPI][4];
#pragma unroll
            for (int u = 0; u < TPI; ++u)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const S* p = src + (t0 + u) * kObTile + k * 256 + lane * 4;
                    if constexpr (sizeof(S) == 4) raw[u][k] = NTL ? nt_load16(p) : *reinterpret_cast<const uint4*>(p);
                    else raw[u][k] = NTL ? nt_load8(p) : *reinterpret_cast<const uint2*>(p);
                }
#pragma unroll
            for (int u = 0; u < TPI; ++u)
#pragma unroll
                for (int k = 0; k < 4; ++k) unpack4<T>(raw[u][k], a[u][k]);
        } else {
#pragma unroll
            for (int u = 0; u < TPI; ++u)
#pragma unroll
                for (int k = 0; k < 4; ++k) load4<T>(src, (t0 + u) * kObTile + k * 256 + lane * 4, n, vec, a[u][k]);
        }
#pragma unroll
        for (int u = 0; u < TPI; ++u) {
            const int64_t t = t0 + u;
            if (t >= t_end) break;
            // the lane's 16 sign bits form its own 16-bit field (bit sub*4+e)
            uint32_t field = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int e = 0; e < 4; ++e) field |= (a[u][k][e] < 0.0f ? 1u : 0u) << (k * 4 + e);
            // even lanes store their field and the odd neighbour's as one dword
            const uint32_t next = odd_neighbour(field);
            if ((lane & 1) == 0) reinterpret_cast<uint32_t*>(bits + t * kObTileBytes)[lane >> 1] = field | (next << 16);
            float ab[4][4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int e = 0; e < 4; ++e) ab[k][e] = __builtin_fabsf(a[u][k][e]);
            const float s = wave_tree_sum_lane0(lane_tree(ab));
            if (lane == 0) part[t] = s;
        }
    }
}

// ------------------------------------------------------------------------
// finalize: scale = F(partials) / n, header, slack (one workgroup per chunk)
// ------------------------------------------------------------------------
__device__ __forceinline__ float tile_from(const float* v, int64_t base, int64_t count, int lane) {
    float a[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t r = base + k * 256 + lane * 4 + e;
            const float x = v[r < count ? r : count - 1];  // clamped: no load waits behind a branch
            a[k][e] = r < count ? x : 0.0f;
        }
    return wave_tree_sum(lane_tree(a));
}

// Levels >= 2 of the chunk tree: lvl[0][0, ceil(m1 / 1024)) holds the level-1 group
// sums (published by a barrier); returns the root to every thread.
__device__ __forceinline__ float upper_tree(int64_t m1, float (&lvl)[2][2048]) {
    const int lane = lane_id(), wave = threadIdx.x / kWave, nw = kObFinalizeThreads / kWave;
    int cur = 0;
    bool done = m1 <= kObTile;
    int64_t m = (m1 + kObTile - 1) / kObTile;
    while (!done) {
        const int64_t g = (m + kObTile - 1) / kObTile;
        for (int64_t i = wave; i < g; i += nw) {
            const float s = tile_from(lvl[cur], i * kObTile, m, lane);
            if (lane == 0) lvl[cur ^ 1][i] = s;
        }
        __syncthreads();
        done = m <= kObTile;
        cur ^= 1;
        m = g;
    }
    return lvl[cur][0];
}

// The fixed 1024-tree over a chunk's m1 tile partials get(r), by one
// kObFinalizeThreads workgroup: level 1 -> 2 straight from `get` (each wave takes
// kFinBatch groups at once and issues all their loads before any tree, so the pass
// costs one memory latency instead of one per group),
// the higher levels in LDS.  Every thread returns the total (0 when m1 = 0).
template <typename Get>
__device__ __forceinline__ float chunk_tree(const Get& get, int64_t m1, float (&lvl)[2][2048]) {
    // the wave index through readfirstlane: the compiler then knows the group branches below
    // are wave-uniform (scalar branches, not exec masks)
    const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
    const int nw = kObFinalizeThreads / kWave;
    if (m1 <= 0) return 0.0f;
    int64_t m = m1;
    const int64_t g1 = (m + kObTile - 1) / kObTile;
    constexpr int kFinBatch = 4;
    for (int64_t g0 = wave; g0 < g1; g0 += (int64_t)nw * kFinBatch) {
        float a[kFinBatch][4][4];
        if ((g0 + (int64_t)(kFinBatch - 1) * nw + 1) * kObTile <= m) {
            // every group of the batch is full: one base per group, immediate offsets
#pragma unroll
            for (int j = 0; j < kFinBatch; ++j) {
                const int64_t bj = (g0 + (int64_t)j * nw) * kObTile + lane * 4;
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int e = 0; e < 4; ++e) a[j][k][e] = get(bj + k * 256 + e);
            }
        } else {
        // otherwise per group, a wave-uniform branch: a full group's loads unconditional,
        // only the chunk's last, ragged group read element by element (guarded).  Guarded
        // loads for the whole batch are serialised by the compiler under this workgroup's
        // 128-VGPR budget: the finalize of 32 groups (one ragged batch) took 10.7 us, this
        // way 4.6; of 64 (one full batch) 5.3
#pragma unroll
        for (int j = 0; j < kFinBatch; ++j) {
            const int64_t g = g0 + (int64_t)j * nw;
            const int64_t bj = g * kObTile + lane * 4;
            if ((g + 1) * kObTile <= m) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int e = 0; e < 4; ++e) a[j][k][e] = get(bj + k * 256 + e);
            } else if (g * kObTile < m) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int64_t r = bj + k * 256 + e;
                        a[j][k][e] = r < m ? get(r) : 0.0f;
                    }
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int e = 0; e < 4; ++e) a[j][k][e] = 0.0f;
            }
        }
        }
#pragma unroll
        for (int j = 0; j < kFinBatch; ++j) {
            const int64_t g = g0 + (int64_t)j * nw;
            const float s = wave_tree_sum(lane_tree(a[j]));
            if (lane == 0 && g < g1) lvl[0][g] = s;
        }
    }
    __syncthreads();
    return upper_tree(m1, lvl);
}

__global__ __launch_bounds__(kObFinalizeThreads) void onebit_finalize_kernel(
    const float* __restrict__ partials, int64_t tiles_per_chunk, int64_t in_num_elem, int64_t cs, int target,
    uint8_t* __restrict__ out, int64_t chunk_offset, int64_t out_bytes, int num_chunks) {
    __shared__ float lvl[2][2048];  // level >= 2 values: <= ceil(2^21 / 1024)
    const int c = target < 0 ? (int)blockIdx.x : target;
    const int64_t n = ob_valid(in_num_elem, cs, c);
    const float* part = partials + (int64_t)blockIdx.x * tiles_per_chunk;
    const int64_t m1 = (n + kObTile - 1) / kObTile;  // tiles holding valid elements
    const float total = chunk_tree([part](int64_t r) { return part[r]; }, m1, lvl);
    uint8_t* seg = out + (int64_t)c * chunk_offset;
    if (threadIdx.x < 32) {
        const float scale = n > 0 ? total / (float)n : 0.0f;
        const uint32_t sb = __float_as_uint(scale), nb = (uint32_t)n;
        const int t = threadIdx.x;
        uint32_t b = 0;
        if (t < 4) b = (sb >> (8 * t)) & 0xff;
        else if (t < 8) b = (nb >> (8 * (t - 4))) & 0xff;
        seg[t] = (uint8_t)b;
    }
    const int64_t tiles = (cs + kObTile - 1) / kObTile;
    for (int64_t j = 32 + tiles * kObTileBytes + threadIdx.x; j < chunk_offset; j += kObFinalizeThreads) seg[j] = 0;
    if (target < 0 && c == num_chunks - 1)
        for (int64_t j = (int64_t)num_chunks * chunk_offset + threadIdx.x; j < out_bytes; j += kObFinalizeThreads)
            out[j] = 0;
}

// ------------------------------------------------------------------------
// decode
// ------------------------------------------------------------------------
template <typename T, bool NTS>
__global__ __launch_bounds__(kBlock) void onebit_decode_kernel(const uint8_t* __restrict__ in, int64_t chunk_offset,
                                                              int64_t cs, typename T::storage* __restrict__ out,
                                                              int64_t t_begin, int64_t t_end) {
    using S = typename T::storage;
    const int c = blockIdx.y;
    const uint8_t* seg = in + (int64_t)c * chunk_offset;
    float scale;
    __builtin_memcpy(&scale, seg, 4);
    const uint8_t* bits = seg + 32;
    S* dst = out + (int64_t)c * cs;
    const bool vec = ((uintptr_t)dst % (4 * sizeof(S))) == 0;
    const int lane = lane_id();
    const int64_t wave = grid_wave();
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    const uint32_t sbits = __float_as_uint(scale);
    for (int64_t t = t_begin + wave; t < t_end; t += nwaves) {
        // the lane's own 16-bit field: no cross-lane traffic
        const uint32_t field = reinterpret_cast<const uint16_t*>(bits + t * kObTileBytes)[lane];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float f[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)  // bit ? -scale : +scale, as a sign-bit flip
                f[e] = __uint_as_float(sbits ^ ((field << (31 - (k * 4 + e))) & 0x80000000u));
            store4<T, NTS>(dst, t * kObTile + k * 256 + lane * 4, cs, vec, f);
        }
    }
}

// ------------------------------------------------------------------------
// fused middle step of the centralized op (1-bit): decode the p received
// segments of the own chunk, reduce them in the reference's tree order
// (decompress_from -> reduce_{mean,sum}_inplace, centralized_low_precision_
// synchronous.rs:40-52) and re-encode the result (compress(target)) in one
// pass: the reduced chunk is written once (or not at all when the caller
// overwrites it anyway, STORE = false: the centralized op's final decompress
// rewrites every element), its bits and |x| tile partials come from registers;
// onebit_finalize_kernel then writes the header.
// ------------------------------------------------------------------------
template <typename T, int BY, bool AVG, bool STORE>
__global__ __launch_bounds__(kBlock) void onebit_reduce_encode_kernel(
    const uint8_t* __restrict__ in, int64_t chunk_offset, int64_t cs, int p, typename T::storage* __restrict__ chunk,
    uint8_t* __restrict__ out_seg, float* __restrict__ part) {
    __shared__ float pos[kMaxFusedChunks], neg[kMaxFusedChunks];
    if (threadIdx.x < (unsigned)p) {  // segment c decodes to +-scale_c as stored in T
        float sc;
        __builtin_memcpy(&sc, in + (int64_t)threadIdx.x * chunk_offset, 4);
        pos[threadIdx.x] = as_stored<T>(sc);
        neg[threadIdx.x] = as_stored<T>(-sc);
    }
    __syncthreads();
    using S = typename T::storage;
    const int lane = lane_id();
    const int64_t tiles = (cs + kObTile - 1) / kObTile;
    const int64_t wave = grid_wave();
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    const bool vec = ((uintptr_t)chunk % (4 * sizeof(S))) == 0;
    const float pf = (float)p;
    uint8_t* bits = out_seg + 32;
    for (int64_t t = wave; t < tiles; t += nwaves) {
        float s[16][BY];
#pragma unroll
        for (int b = 0; b < 16; ++b)
#pragma unroll
            for (int y = 0; y < BY; ++y) s[b][y] = 0.0f;
        for (int r = 0; r * BY < p; ++r) {
            uint32_t f[BY];
#pragma unroll
            for (int y = 0; y < BY; ++y) {  // each lane's 16-bit field of every segment
                const int c = r * BY + y < p ? r * BY + y : p - 1;
                f[y] = reinterpret_cast<const uint16_t*>(in + (int64_t)c * chunk_offset + 32 + t * kObTileBytes)[lane];
            }
#pragma unroll
            for (int y = 0; y < BY; ++y) {
                const int c = r * BY + y;
                if (c >= p) break;
#pragma unroll
                for (int b = 0; b < 16; ++b) s[b][y] = s[b][y] + (((f[y] >> b) & 1u) ? neg[c] : pos[c]);
            }
        }
        float x[4][4];
        uint32_t field = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int b = k * 4 + e;
                tree_finish<BY>(s[b]);
                const int64_t j = t * kObTile + k * 256 + lane * 4 + e;
                // the reduced value as stored in T; padding past cs stays 0 (as the encoder sees it)
                const float v = j < cs ? as_stored<T>(AVG ? s[b][0] / pf : s[b][0]) : 0.0f;
                x[k][e] = v;
                field |= (v < 0.0f ? 1u : 0u) << b;
            }
        if constexpr (STORE) {
#pragma unroll
            for (int k = 0; k < 4; ++k) store4<T>(chunk, t * kObTile + k * 256 + lane * 4, cs, vec, x[k]);
        }
        const uint32_t next = odd_neighbour(field);
        if ((lane & 1) == 0) reinterpret_cast<uint32_t*>(bits + t * kObTileBytes)[lane >> 1] = field | (next << 16);
        float ab[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) ab[k][e] = __builtin_fabsf(x[k][e]);
        const float sum = wave_tree_sum_lane0(lane_tree(ab));
        if (lane == 0) part[t] = sum;
    }
}

// ------------------------------------------------------------------------
// The same fused middle step, table-driven.  A reduced element depends only on
// its p sign bits (segment c decodes to +-scale_c), so every value the
// reference tree can produce is tabulated once per workgroup in LDS:
//   p <= 8 : lut[bits] = as_stored(avg ? tree(bits) / p : tree(bits)), 2^p entries;
//   p <= 16: the tree (BY = 8) is ((s0+s4)+(s2+s6)) + ((s1+s5)+(s3+s7)) with
//            s_y = (0 + v_y) + v_{y+8}: the even-y half depends on the 8 even
//            segments' bits, the odd-y half on the 8 odd ones, so two 256-entry
//            tables and one add (then the average and the rounding to T).
// The per-element bit indexes come from an 8x8 bit-matrix transpose of the
// lane's 16-bit fields (row = segment, column = element).  Same expressions,
// same order, so the same bits as onebit_reduce_encode_kernel.
// ------------------------------------------------------------------------
// bit (row r, column c) at position 8r + c  ->  position 8c + r
__device__ __forceinline__ uint64_t transpose8x8(uint64_t x) {
    uint64_t t;
    t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
    x = x ^ t ^ (t << 7);
    t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
    x = x ^ t ^ (t << 14);
    t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
    x = x ^ t ^ (t << 28);
    return x;
}

// idx[b] (b < 16) = sum over rows k < 8 of bit b of rows[k], << k
__device__ __forceinline__ void bit_columns(const uint32_t (&rows)[8], uint32_t (&idx)[16]) {
    uint64_t lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        lo |= (uint64_t)(rows[k] & 0xffu) << (8 * k);
        hi |= (uint64_t)((rows[k] >> 8) & 0xffu) << (8 * k);
    }
    lo = transpose8x8(lo);
    hi = transpose8x8(hi);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        idx[b] = (uint32_t)(lo >> (8 * b)) & 0xffu;
        idx[b + 8] = (uint32_t)(hi >> (8 * b)) & 0xffu;
    }
}

// the reference tree over p <= 8 segments for the sign pattern `bits`
template <int BY>
__device__ __forceinline__ float lut_tree(int bits, int p, const float* pos, const float* neg) {
    float s[BY];
#pragma unroll
    for (int y = 0; y < BY; ++y) s[y] = 0.0f;
    for (int r = 0; r * BY < p; ++r)
#pragma unroll
        for (int y = 0; y < BY; ++y) {
            const int c = r * BY + y;
            if (c < p) s[y] = s[y] + (((bits >> c) & 1) ? neg[c] : pos[c]);
        }
    tree_finish<BY>(s);
    return s[0];
}

// one half (parity 0: y even, 1: y odd) of the BY = 8 tree; bit k of `bits` is
// segment 2k + parity
__device__ __forceinline__ float lut_half(int bits, int parity, int p, const float* pos, const float* neg) {
    float s[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int y = parity + 2 * m;
        s[m] = 0.0f;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int c = y + 8 * r;
            const int k = (c - parity) / 2;
            if (c < p) s[m] = s[m] + (((bits >> k) & 1) ? neg[c] : pos[c]);
        }
    }
    // h = 4: s_y += s_{y+4}; h = 2: s_y += s_{y+2}  ->  (s[0] + s[2]) + (s[1] + s[3])
    return (s[0] + s[2]) + (s[1] + s[3]);
}

// PMAX = 2: p <= 2, the index is read bit by bit; 4 and 8: the 8x8 transpose (4, re-encode
// only: the pair table); 16: two tables
template <typename T, int PMAX, bool STORE, int UT = (PMAX == 2 ? 2 : 1)>
__global__ __launch_bounds__(kBlock) void onebit_reduce_encode_lut_kernel(
    const uint8_t* __restrict__ in, int64_t chunk_offset, int64_t cs, int p, int average,
    typename T::storage* __restrict__ chunk, uint8_t* __restrict__ out_seg, float* __restrict__ part) {
    constexpr bool WIDE = PMAX > 8;
    __shared__ float pos[kMaxFusedChunks], neg[kMaxFusedChunks];
    __shared__ float lut[WIDE ? 2 : 1][256];
    if (threadIdx.x < (unsigned)p) {  // segment c decodes to +-scale_c as stored in T
        float sc;
        __builtin_memcpy(&sc, in + (int64_t)threadIdx.x * chunk_offset, 4);
        pos[threadIdx.x] = as_stored<T>(sc);
        neg[threadIdx.x] = as_stored<T>(-sc);
    }
    __syncthreads();
    const float pf = (float)p;
    for (int i = threadIdx.x; i < 256; i += kBlock) {
        if constexpr (WIDE) {
            lut[0][i] = lut_half(i, 0, p, pos, neg);
            lut[1][i] = lut_half(i, 1, p, pos, neg);
        } else if (i < (1 << p)) {
            const float v = p <= 4 ? lut_tree<2>(i, p, pos, neg) : lut_tree<4>(i, p, pos, neg);
            lut[0][i] = as_stored<T>(average ? v / pf : v);
        } else if (PMAX <= 4 && i < (1 << PMAX)) {
            lut[0][i] = 0.0f;  // entries of segments >= p, never indexed (read by the tables below)
        }
    }
    __syncthreads();
    // p <= 2, the re-encode only (no reduced chunk stored): a lane's four elements of sub-tile
    // k have values lut[idx_e], idx_e = bit e of the nibble k of segment 0's field | bit e of
    // segment 1's << 1, so their part of the |x| tree, (|a0| + |a1|) + (|a2| + |a3|), is one of
    // 256 values -- tabulated here in that order, looked up by the two nibbles -- and the sign
    // bits of all 16 elements follow from the two fields with bitwise operations
    __shared__ float gtab[PMAX == 2 && !STORE ? 256 : 1];
    uint32_t negm[4] = {0, 0, 0, 0};  // all-ones where lut[idx] < 0 (the re-encoded bit of idx)
    if constexpr (PMAX == 2 && !STORE) {
        const int i = threadIdx.x;  // kBlock == 256: one entry per thread
        float a[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] = __builtin_fabsf(lut[0][((i >> e) & 1) | (((i >> (4 + e)) & 1) << 1)]);
        gtab[i] = (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
        for (int k = 0; k < 4; ++k) negm[k] = lut[0][k] < 0.0f ? 0xffffffffu : 0u;
        __syncthreads();
    }
    // 2 < p <= 4, the re-encode only: the two elements of a pair (2j, 2j + 1) take 8 bits of
    // the four fields, so the pair's part of the |x| tree, |a0| + |a1|, and its two sign bits
    // are one of 256 entries, looked up by an index gathered with word-wide masks (process
    // below: bit 0 / 1 segment 0's bit of element 0 / 1, bits 2-3 segment 2's, 4-5 segment
    // 1's, 6-7 segment 3's).  Per tile and lane that is 8 lookups and ~30 bitwise operations
    // in place of the 8x8 transpose, 16 lookups and the per-element sign and |x| work
    constexpr bool PAIRS = PMAX == 4 && !STORE;
    __shared__ uint2 ptab[PAIRS ? 256 : 1];
    if constexpr (PAIRS) {
        const int i = threadIdx.x;  // kBlock == 256: one entry per thread
        const int i0 = (i & 1) | ((i >> 3) & 2) | (i & 4) | ((i >> 3) & 8);
        const int i1 = ((i >> 1) & 1) | ((i >> 4) & 2) | ((i >> 1) & 4) | ((i >> 4) & 8);
        const float v0 = lut[0][i0], v1 = lut[0][i1];
        ptab[i] = make_uint2(__float_as_uint(__builtin_fabsf(v0) + __builtin_fabsf(v1)),
                             (v0 < 0.0f ? 1u : 0u) | (v1 < 0.0f ? 2u : 0u));
        __syncthreads();
    }
    using S = typename T::storage;
    const int lane = lane_id();
    const int64_t tiles = (cs + kObTile - 1) / kObTile;
    const int64_t wave = grid_wave();
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    const bool vec = ((uintptr_t)chunk % (4 * sizeof(S))) == 0;
    uint8_t* bits = out_seg + 32;
    // every segment's 16-bit field of this lane for tile t, loaded unconditionally
    // (segments >= p read the last one and are masked to 0 after the loads)
    auto load_fields = [&](int64_t t, uint32_t (&f)[PMAX]) {
#pragma unroll
        for (int c = 0; c < PMAX; ++c) {
            const int cc = c < p ? c : p - 1;
            f[c] = reinterpret_cast<const uint16_t*>(in + (int64_t)cc * chunk_offset + 32 + t * kObTileBytes)[lane];
        }
    };
    auto process = [&](int64_t t, uint32_t (&f)[PMAX]) {
#pragma unroll
        for (int c = 0; c < PMAX; ++c) f[c] = c < p ? f[c] : 0u;
        if constexpr (PMAX == 2 && !STORE) {
            if ((t + 1) * kObTile <= cs) {  // a full tile: the group table and bitwise signs
                const uint32_t f0 = f[0], f1 = f[1];
                const uint32_t field = ((negm[0] & ~f0 & ~f1) | (negm[1] & f0 & ~f1) | (negm[2] & ~f0 & f1) |
                                        (negm[3] & f0 & f1)) & 0xffffu;
                float q[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) q[k] = gtab[((f0 >> (4 * k)) & 15u) | (((f1 >> (4 * k)) & 15u) << 4)];
                const uint32_t next = odd_neighbour(field);
                if ((lane & 1) == 0)
                    reinterpret_cast<uint32_t*>(bits + t * kObTileBytes)[lane >> 1] = field | (next << 16);
                const float sum = wave_tree_sum_lane0((q[0] + q[1]) + (q[2] + q[3]));
                if (lane == 0) part[t] = sum;
                return;
            }
        }
        if constexpr (PAIRS) {
            if ((t + 1) * kObTile <= cs) {
                // 2-bit group g of A is segment 0's pair g (g < 8) or segment 1's (g - 8); B the same
                // for segments 2 and 3.  Nibble m of E holds A's and B's group 2m, of O group 2m + 1;
                // nibbles m and m + 4 together are the index of pair 2m (E) or 2m + 1 (O), m < 4
                const uint32_t A = f[0] | (f[1] << 16), B = f[2] | (f[3] << 16);
                const uint32_t E = (A & 0x33333333u) | ((B & 0x33333333u) << 2);
                const uint32_t O = ((A >> 2) & 0x33333333u) | (B & 0xccccccccu);
                // bytes 0 / 1: pairs 0 / 4 (ie), 2 / 6 (je), 1 / 5 (io), 3 / 7 (jo)
                const uint32_t ie = (E & 0x0f0fu) | ((E >> 12) & 0xf0f0u), je = ((E >> 4) & 0x0f0fu) | ((E >> 16) & 0xf0f0u);
                const uint32_t io = (O & 0x0f0fu) | ((O >> 12) & 0xf0f0u), jo = ((O >> 4) & 0x0f0fu) | ((O >> 16) & 0xf0f0u);
                const uint32_t idx[8] = {ie & 255u, io & 255u, je & 255u, jo & 255u, ie >> 8, io >> 8, je >> 8, jo >> 8};
                uint32_t field = 0;
                float q[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {  // sub-tile k: pairs 2k and 2k + 1
                    const uint2 a = ptab[idx[2 * k]], b = ptab[idx[2 * k + 1]];
                    q[k] = __uint_as_float(a.x) + __uint_as_float(b.x);
                    field |= (a.y | (b.y << 2)) << (4 * k);
                }
                const uint32_t next = odd_neighbour(field);
                if ((lane & 1) == 0)
                    reinterpret_cast<uint32_t*>(bits + t * kObTileBytes)[lane >> 1] = field | (next << 16);
                const float sum = wave_tree_sum_lane0((q[0] + q[1]) + (q[2] + q[3]));
                if (lane == 0) part[t] = sum;
                return;
            }
        }
        float x[4][4];
        if constexpr (WIDE) {
            uint32_t re[8], ro[8], ia[16], ib[16];
#pragma unroll
            for (int k = 0; k < 8; ++k) { re[k] = f[2 * k]; ro[k] = f[2 * k + 1]; }
            bit_columns(re, ia);
            bit_columns(ro, ib);
#pragma unroll
            for (int b = 0; b < 16; ++b) {
                const float v = lut[0][ia[b]] + lut[1][ib[b]];
                x[b / 4][b % 4] = as_stored<T>(average ? v / pf : v);
            }
        } else if constexpr (PMAX == 2) {
            const uint32_t g = f[0] | (f[1] << 16);  // bit b: segment 0 at b, segment 1 at b + 16
#pragma unroll
            for (int b = 0; b < 16; ++b) x[b / 4][b % 4] = lut[0][((g >> b) & 1u) | ((g >> (b + 15)) & 2u)];
        } else {
            uint32_t rows[8], ix[16];
#pragma unroll
            for (int k = 0; k < 8; ++k) rows[k] = k < PMAX ? f[k < PMAX ? k : 0] : 0u;
            bit_columns(rows, ix);
#pragma unroll
            for (int b = 0; b < 16; ++b) x[b / 4][b % 4] = lut[0][ix[b]];
        }
        if ((t + 1) * kObTile > cs) {  // the ragged last tile: padding past cs stays 0 (as the encoder sees it)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (t * kObTile + k * 256 + lane * 4 + e >= cs) x[k][e] = 0.0f;
        }
        uint32_t field = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) field |= (x[k][e] < 0.0f ? 1u : 0u) << (k * 4 + e);
        if constexpr (STORE) {
#pragma unroll
            for (int k = 0; k < 4; ++k) store4<T>(chunk, t * kObTile + k * 256 + lane * 4, cs, vec, x[k]);
        }
        const uint32_t next = odd_neighbour(field);
        if ((lane & 1) == 0) reinterpret_cast<uint32_t*>(bits + t * kObTileBytes)[lane >> 1] = field | (next << 16);
        float ab[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) ab[k][e] = __builtin_fabsf(x[k][e]);
        const float sum = wave_tree_sum_lane0(lane_tree(ab));
        if (lane == 0) part[t] = sum;
    };
    // U tiles per wave iteration, all their loads issued before the first is used: at
    // p <= 2 a tile's input is 4 B per lane, and one tile at a time kept a wave waiting a
    // whole memory latency per 1,024 elements (1 GiB, p = 2: 46.5 us; U = 2 / 4 / 8 with
    // 4,096 workgroups 35.1 / 38.7 / 48.8 us, profiles/r06_sweeps/ob_middle_*.json).
    // The transposing paths keep one tile (U = 4 there: p = 4 30.7 -> 33.0, p = 8
    // 18.9 -> 22.7 us; profiles/r06_onebit_middle_unroll.json)
    constexpr int U = UT;
    for (int64_t t0 = wave; t0 < tiles; t0 += U * nwaves) {
        uint32_t f[U][PMAX];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t0 + u * nwaves < tiles) load_fields(t0 + u * nwaves, f[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t0 + u * nwaves < tiles) process(t0 + u * nwaves, f[u]);
    }
}

// ------------------------------------------------------------------------
// The centralized op at one rank (centralized_low_precision_synchronous.rs:30-71
// with p = 1: encode -> alltoall of the own bytes -> decode + reduce + re-encode
// -> allgather of nothing -> decode) in two streaming passes.  At p = 1 the fused
// middle step's table (onebit_reduce_encode_lut_kernel) has two entries: every
// reduced element is v0 (its sign bit 0) or v1 (bit 1), and |v0| == |v1| (the
// rounding to T and the tree's additions of 0 are sign-symmetric), so
//   re-encoded bit  = bit ? (v1 < 0) : (v0 < 0)
//   re-encoded scale = F(|v0| at every valid position, 0 past n) / n
// with F the encoder's fixed tree: every full tile has one partial, the ragged
// last tile another, and chunk_tree folds them exactly as the finalize would
// fold stored partials.  onebit_one_rank_kernel (one workgroup) derives scale1
// from the encode's tile partials, then v0, v1 and scale2; the decode writes
// bit2 ? -scale2 : +scale2 from the encode's bits.  The reduced chunk, the second
// bit plane and the table kernel (VALU-bound, 0.11 of HBM peak at 1 GiB) are gone;
// the bytes are the 1-bit op's (bit-identical to the multi-kernel sequence).
// ------------------------------------------------------------------------
struct OneRankOut {
    float scale2;
    uint32_t mpos, mneg;  // all-ones when v0 < 0 / v1 < 0 (re-encoded bit of a 0 / 1 bit)
    uint32_t pad;
};

// Level 1 of the first scale's tree across the whole GPU: group g (1024 tile partials)
// -> level1[g], one wave per group -- the same fold chunk_tree's level 1 does in one
// workgroup, where 2^18 partials (1 GiB) took that workgroup 16 us
__global__ __launch_bounds__(kBlock) void onebit_tree_level1_kernel(const float* __restrict__ partials, int64_t m1,
                                                                   float* __restrict__ level1) {
    const int64_t g = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    const int64_t g1 = (m1 + kObTile - 1) / kObTile;
    if (g >= g1) return;
    const float s = tile_from(partials, g * kObTile, m1, lane_id());
    if (lane_id() == 0) level1[g] = s;
}

template <typename T>
__global__ __launch_bounds__(kObFinalizeThreads) void onebit_one_rank_kernel(const float* __restrict__ level1,
                                                                            int64_t n, int average, float pf,
                                                                            OneRankOut* __restrict__ out) {
    __shared__ float lvl[2][2048];
    const int64_t m1 = (n + kObTile - 1) / kObTile;
    float total1 = 0.0f;
    if (m1 > 0) {  // the first tree from its level-1 sums (onebit_tree_level1_kernel)
        const int64_t g1 = (m1 + kObTile - 1) / kObTile;
        for (int64_t i = threadIdx.x; i < g1; i += kObFinalizeThreads) lvl[0][i] = level1[i];
        __syncthreads();
        total1 = upper_tree(m1, lvl);
    }
    __syncthreads();  // every thread has read the first tree's root before lvl is reused
    const float scale1 = n > 0 ? total1 / (float)n : 0.0f;
    // the table kernel's p = 1 entries: segment 0 decodes to +-scale1 as stored in T
    const float pos[1] = {as_stored<T>(scale1)}, neg[1] = {as_stored<T>(-scale1)};
    const float t0 = lut_tree<2>(0, 1, pos, neg), t1 = lut_tree<2>(1, 1, pos, neg);
    const float v0 = as_stored<T>(average ? t0 / pf : t0);
    const float v1 = as_stored<T>(average ? t1 / pf : t1);
    // the re-encode's tile partials: a full tile of |v|, and the ragged last tile
    const int lane = lane_id();
    const float a = __builtin_fabsf(v0);
    float full[4][4], last[4][4];
    const int64_t rem = n % kObTile;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            full[k][e] = a;
            last[k][e] = (k * 256 + lane * 4 + e) < rem ? a : 0.0f;
        }
    const float pfull = wave_tree_sum(lane_tree(full));
    const float plast = rem ? wave_tree_sum(lane_tree(last)) : pfull;
    // level 1 of the second tree without its 2^18 inputs: every group of 1024 full tiles
    // folds to the same value; only the group holding the ragged tile (or the ragged end
    // of the tile list) differs
    const int64_t nfull = n / kObTile;  // full tiles; the ragged one (if any) is tile nfull
    const int64_t g1 = (m1 + kObTile - 1) / kObTile;
    float grp[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) grp[k][e] = pfull;
    const float gfull = wave_tree_sum(lane_tree(grp));
    const int64_t lastg = g1 - 1, lb = lastg * kObTile;  // the last group: tiles [lb, m1)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t r = lb + k * 256 + lane * 4 + e;
            grp[k][e] = r < nfull ? pfull : (r < m1 ? plast : 0.0f);
        }
    const float glast = wave_tree_sum(lane_tree(grp));
    float total2 = 0.0f;
    if (m1 > 0) {
        for (int64_t i = threadIdx.x; i < g1; i += kObFinalizeThreads) lvl[0][i] = i == lastg ? glast : gfull;
        __syncthreads();
        total2 = upper_tree(m1, lvl);
    }
    if (threadIdx.x == 0) {
        OneRankOut o;
        o.scale2 = n > 0 ? total2 / (float)n : 0.0f;
        o.mpos = v0 < 0.0f ? 0xffffffffu : 0u;
        o.mneg = v1 < 0.0f ? 0xffffffffu : 0u;
        o.pad = 0;
        *out = o;
    }
}

template <typename T, bool NTS>
__global__ __launch_bounds__(kBlock) void onebit_one_rank_decode_kernel(const uint8_t* __restrict__ bits,
                                                                       const OneRankOut* __restrict__ o,
                                                                       int64_t cs, typename T::storage* __restrict__ out,
                                                                       int64_t tiles) {
    using S = typename T::storage;
    const bool vec = ((uintptr_t)out % (4 * sizeof(S))) == 0;
    const int lane = lane_id();
    const int64_t wave = grid_wave();
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    const uint32_t sbits = __float_as_uint(o->scale2), mpos = o->mpos, mneg = o->mneg;
    for (int64_t t = wave; t < tiles; t += nwaves) {
        const uint32_t f1 = reinterpret_cast<const uint16_t*>(bits + t * kObTileBytes)[lane];
        const uint32_t field = (f1 & mneg) | (~f1 & mpos);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float f[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)  // bit ? -scale2 : +scale2, as a sign-bit flip
                f[e] = __uint_as_float(sbits ^ ((field << (31 - (k * 4 + e))) & 0x80000000u));
            store4<T, NTS>(out, t * kObTile + k * 256 + lane * 4, cs, vec, f);
        }
    }
}

// ------------------------------------------------------------------------
// host
// ------------------------------------------------------------------------
static int64_t ob_tiles(int64_t cs) { return (cs + kObTile - 1) / kObTile; }

static int ob_blocks(int64_t tiles, int nact, int target_blocks = kTargetBlocks) {
    int64_t b = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    const int64_t cap = (target_blocks + nact - 1) / nact;
    if (b > cap) b = cap;
    return (int)(b < 1 ? 1 : b);
}

// stage 0: encode every tile + finalize; 1: encode tiles [t_begin, t_end) only
// (bits + |x| partials, no header); 2: finalize only (header + slack from the
// partials every stage-1 range left in the workspace)
template <typename T>
static int ob_compress_impl(const void* input, int in_num_elem, int cs, int p, uint8_t* out, size_t out_bytes,
                            void* ws, size_t ws_bytes, int target, hipStream_t s, int stage = 0,
                            int64_t t_begin = 0, int64_t t_end = INT64_MAX) {
    using S = typename T::storage;
    if (p <= 0 || p > 65535 || cs < 0 || target < -1 || target >= p || !out || (!input && stage != 2) ||
        t_begin < 0 || t_end < t_begin)
        return BAGUA_ERR_INVALID_ARG;
    const int64_t co = (int64_t)(out_bytes / (size_t)p);
    const int64_t tiles = ob_tiles(cs);
    if (co < 32 + tiles * kObTileBytes) return BAGUA_ERR_INVALID_ARG;
    const int nact = target < 0 ? p : 1;
    if (!ws || ws_bytes < (size_t)nact * (size_t)(tiles > 0 ? tiles : 1) * sizeof(float)) return BAGUA_ERR_WORKSPACE;
    if (((uintptr_t)out + 32) % 4 || co % 4) return BAGUA_ERR_INVALID_ARG;  // bit tiles are written as dwords
    float* partials = static_cast<float*>(ws);
    const int64_t tb = stage == 2 ? 0 : t_begin, te = stage == 2 ? tiles : (t_end < tiles ? t_end : tiles);
    // nt loads: default-policy loads behind the decode's default-policy stores take
    // 77 us instead of 47 (profiles/r01_decode_store_ab.jsonl)
    if (stage != 2 && te > tb) {
        const dim3 grid(ob_blocks(te - tb, nact, tune_int("BAGUA_TUNE_OB_ENCODE_BLOCKS", kObEncodeBlocks)), nact);
        // BAGUA_TUNE_OB_ENCODE_TPI=2: f32 tiles two per wave iteration (A/B; 16-bit types always take two)
        if (sizeof(S) == 4 && tune_int("BAGUA_TUNE_OB_ENCODE_TPI", 1) == 2)
            launch(onebit_encode_kernel<T, 2, true>, grid, dim3(kBlock), 0, s, static_cast<const S*>(input),
                   (int64_t)in_num_elem, (int64_t)cs, target, out, co, partials, tiles, tb, te);
        else
            launch(onebit_encode_kernel<T, sizeof(S) == 4 ? 1 : 2, true>, grid, dim3(kBlock), 0, s,
                   static_cast<const S*>(input), (int64_t)in_num_elem, (int64_t)cs, target, out, co, partials, tiles,
                   tb, te);
    }
    if (stage != 1)
        launch(onebit_finalize_kernel, dim3(nact), dim3(kObFinalizeThreads), 0, s, partials, tiles,
               (int64_t)in_num_elem, (int64_t)cs, target, out, co, (int64_t)out_bytes, p);
    return check_launch();
}

template <typename T>
static int ob_decompress_impl(const uint8_t* in, size_t in_bytes, int cs, int p, void* out, hipStream_t s,
                              int64_t t_begin = 0, int64_t t_end = INT64_MAX) {
    using S = typename T::storage;
    if (p <= 0 || p > 65535 || cs < 0 || !in || !out || t_begin < 0 || t_end < t_begin) return BAGUA_ERR_INVALID_ARG;
    const int64_t co = (int64_t)(in_bytes / (size_t)p);
    const int64_t tiles = ob_tiles(cs);
    if (co < 32 + tiles * kObTileBytes) return BAGUA_ERR_INVALID_ARG;
    if (((uintptr_t)in + 32) % 4 || co % 4) return BAGUA_ERR_INVALID_ARG;
    const int64_t te = t_end < tiles ? t_end : tiles;
    if (te <= t_begin) return BAGUA_OK;
    // Store policy by the bucket's size (all p chunks, not this launch's tile range):
    // up to the 256 MiB Infinity Cache, default-policy stores (256 MiB f32: decode 42.6
    // vs 47.8 us with nt stores, and the next encode unaffected,
    // profiles/r04_onebit_decode_store_ab.jsonl); past it the cache cannot keep the
    // dirty lines, which the next encode then writes back (1 GiB: encode 196 -> 186 us,
    // decode 201 -> 194 us with nt stores, same file).  BAGUA_OB_DECODE_NT=1 / 0
    // forces either (A/B).
    const int env = tune_int("BAGUA_OB_DECODE_NT", -1);
    const int nt = env >= 0 ? env : ((int64_t)cs * p * (int64_t)sizeof(S) > ((int64_t)256 << 20) ? 1 : 0);
    const dim3 grid(ob_blocks(te - t_begin, p, tune_int("BAGUA_TUNE_OB_DECODE_BLOCKS", kObDecodeBlocks)), p);
    if (nt == 1)
        launch(onebit_decode_kernel<T, true>, grid, dim3(kBlock), 0, s, in, co, (int64_t)cs, static_cast<S*>(out),
               t_begin, te);
    else
        launch(onebit_decode_kernel<T, false>, grid, dim3(kBlock), 0, s, in, co, (int64_t)cs, static_cast<S*>(out),
               t_begin, te);
    return check_launch();
}

template <typename T, int BY, bool AVG>
static void launch_ob_reduce(const uint8_t* in, int64_t co, int64_t cs, int p, typename T::storage* chunk,
                             uint8_t* seg, float* part, int blocks, hipStream_t s) {
    if (chunk)
        launch(onebit_reduce_encode_kernel<T, BY, AVG, true>, dim3(blocks), dim3(kBlock), 0, s, in, co, cs, p, chunk,
               seg, part);
    else
        launch(onebit_reduce_encode_kernel<T, BY, AVG, false>, dim3(blocks), dim3(kBlock), 0, s, in, co, cs, p,
               chunk, seg, part);
}

template <typename T, int PMAX>
static void launch_ob_reduce_lut(const uint8_t* in, int64_t co, int64_t cs, int p, int average,
                                 typename T::storage* chunk, uint8_t* seg, float* part, int blocks, hipStream_t s) {
    if constexpr (PMAX <= 4) {  // tiles per wave iteration of the re-encode: BAGUA_OB_MIDDLE_U (A/B)
        const int u = tune_int("BAGUA_OB_MIDDLE_U", PMAX == 2 ? 2 : 1);
        if (!chunk && u == 1) {
            launch(onebit_reduce_encode_lut_kernel<T, PMAX, false, 1>, dim3(blocks), dim3(kBlock), 0, s, in, co, cs,
                   p, average, chunk, seg, part);
            return;
        }
        if (!chunk && u == 2) {
            launch(onebit_reduce_encode_lut_kernel<T, PMAX, false, 2>, dim3(blocks), dim3(kBlock), 0, s, in, co, cs,
                   p, average, chunk, seg, part);
            return;
        }
        if (!chunk && u == 4) {
            launch(onebit_reduce_encode_lut_kernel<T, PMAX, false, 4>, dim3(blocks), dim3(kBlock), 0, s, in, co, cs,
                   p, average, chunk, seg, part);
            return;
        }
        if (!chunk && u == 8) {
            launch(onebit_reduce_encode_lut_kernel<T, PMAX, false, 8>, dim3(blocks), dim3(kBlock), 0, s, in, co, cs,
                   p, average, chunk, seg, part);
            return;
        }
    }
    if (chunk)
        launch(onebit_reduce_encode_lut_kernel<T, PMAX, true>, dim3(blocks), dim3(kBlock), 0, s, in, co, cs, p,
               average, chunk, seg, part);
    else
        launch(onebit_reduce_encode_lut_kernel<T, PMAX, false>, dim3(blocks), dim3(kBlock), 0, s, in, co, cs, p,
               average, chunk, seg, part);
}

template <typename T>
static int ob_reduce_requantize_impl(const uint8_t* recv, size_t recv_bytes, int cs, int p, void* tensor,
                                     int average, uint8_t* out, size_t out_bytes, int target, void* ws,
                                     size_t ws_bytes, hipStream_t s) {
    using S = typename T::storage;
    if (p <= 0 || p > kMaxFusedChunks || cs < 0 || target < 0 || target >= p || !recv || !out)
        return BAGUA_ERR_UNSUPPORTED;  // caller runs decompress + reduce + compress
    const int64_t co_in = (int64_t)(recv_bytes / (size_t)p), co = (int64_t)(out_bytes / (size_t)p);
    const int64_t tiles = ob_tiles(cs);
    if (co_in < 32 + tiles * kObTileBytes || co < 32 + tiles * kObTileBytes) return BAGUA_ERR_INVALID_ARG;
    if (((uintptr_t)recv + 32) % 4 || co_in % 4 || ((uintptr_t)out + 32) % 4 || co % 4) return BAGUA_ERR_INVALID_ARG;
    if (!ws || ws_bytes < (size_t)(tiles > 0 ? tiles : 1) * sizeof(float)) return BAGUA_ERR_WORKSPACE;
    S* chunk = tensor ? static_cast<S*>(tensor) + (int64_t)target * cs : nullptr;  // nullptr: not stored
    float* part = static_cast<float*>(ws);
    uint8_t* seg = out + (int64_t)target * co;
    static const bool lut_on = [] {  // BAGUA_ONEBIT_LUT=0: the per-element tree kernel (A/B)
        const char* v = std::getenv("BAGUA_ONEBIT_LUT");
        return !(v && v[0] == '0');
    }();
    if (tiles > 0 && lut_on) {
        // p <= 2: 4,096 workgroups (two tiles per wave iteration, above); the transposing
        // paths are fastest at 2,048 (profiles/r06_sweeps/ob_middle_*.json)
        const int blocks = ob_blocks(tiles, 1, tune_int("BAGUA_TUNE_OB_MIDDLE_BLOCKS", p <= 2 ? 4096 : kTargetBlocks));
        if (p <= 2)
            launch_ob_reduce_lut<T, 2>(recv, co_in, cs, p, average, chunk, seg, part, blocks, s);
        else if (p <= 4)
            launch_ob_reduce_lut<T, 4>(recv, co_in, cs, p, average, chunk, seg, part, blocks, s);
        else if (p <= 8)
            launch_ob_reduce_lut<T, 8>(recv, co_in, cs, p, average, chunk, seg, part, blocks, s);
        else
            launch_ob_reduce_lut<T, 16>(recv, co_in, cs, p, average, chunk, seg, part, blocks, s);
    } else if (tiles > 0) {
        const int blocks = ob_blocks(tiles, 1);
        switch (reduce_by(p)) {
            case 2:
                if (average) launch_ob_reduce<T, 2, true>(recv, co_in, cs, p, chunk, seg, part, blocks, s);
                else launch_ob_reduce<T, 2, false>(recv, co_in, cs, p, chunk, seg, part, blocks, s);
                break;
            case 4:
                if (average) launch_ob_reduce<T, 4, true>(recv, co_in, cs, p, chunk, seg, part, blocks, s);
                else launch_ob_reduce<T, 4, false>(recv, co_in, cs, p, chunk, seg, part, blocks, s);
                break;
            default:
                if (average) launch_ob_reduce<T, 8, true>(recv, co_in, cs, p, chunk, seg, part, blocks, s);
                else launch_ob_reduce<T, 8, false>(recv, co_in, cs, p, chunk, seg, part, blocks, s);
                break;
        }
    }
    // header + slack of the own segment (the tensor is fully valid: num_elem = p * cs)
    launch(onebit_finalize_kernel, dim3(1), dim3(kObFinalizeThreads), 0, s, part, tiles, (int64_t)p * cs,
           (int64_t)cs, target, out, co, (int64_t)out_bytes, p);
    return check_launch();
}

// workspace of the one-rank op: [0, 32) OneRankOut, the encode's bit tiles at 32,
// its tile partials after them (256-B aligned)
static int64_t onerank_partials_offset(int64_t tiles) { return (32 + tiles * kObTileBytes + 255) / 256 * 256; }

template <typename T>
static int ob_one_rank_impl(void* tensor, int n, int average, void* ws, size_t ws_bytes, hipStream_t s) {
    using S = typename T::storage;
    if (n < 0 || (!tensor && n > 0) || !ws || (uintptr_t)ws % 16) return BAGUA_ERR_INVALID_ARG;
    const int64_t tiles = ob_tiles(n);
    const int64_t off = onerank_partials_offset(tiles);
    const int64_t g1 = (tiles + kObTile - 1) / kObTile;
    if (ws_bytes < (size_t)(off + ((tiles > 0 ? tiles : 1) + g1) * (int64_t)sizeof(float))) return BAGUA_ERR_WORKSPACE;
    uint8_t* seg = static_cast<uint8_t*>(ws);
    float* partials = reinterpret_cast<float*>(seg + off);
    float* level1 = partials + (tiles > 0 ? tiles : 1);
    // 1. sign bits + |x| tile partials of the whole tensor (one chunk)
    if (tiles > 0) {
        const int rc = ob_compress_impl<T>(tensor, n, n, 1, seg, (size_t)(32 + tiles * kObTileBytes), partials,
                                           (size_t)tiles * sizeof(float), -1, s, 1, 0, tiles);
        if (rc) return rc;
    }
    // 2. scale1 (level 1 of its tree across the GPU, the rest in one workgroup), the two
    // reduced values, scale2
    if (g1 > 0)
        launch(onebit_tree_level1_kernel, dim3((unsigned)((g1 + kWavesPerBlock - 1) / kWavesPerBlock)), dim3(kBlock), 0,
               s, partials, tiles, level1);
    launch(onebit_one_rank_kernel<T>, dim3(1), dim3(kObFinalizeThreads), 0, s, level1, (int64_t)n, average, 1.0f,
           reinterpret_cast<OneRankOut*>(seg));
    // 3. the result, from the bits (store policy as the decode's, by size)
    if (tiles > 0) {
        const int env = tune_int("BAGUA_OB_DECODE_NT", -1);
        const int nt = env >= 0 ? env : ((int64_t)n * (int64_t)sizeof(S) > ((int64_t)256 << 20) ? 1 : 0);
        const dim3 grid(ob_blocks(tiles, 1, tune_int("BAGUA_TUNE_OB_DECODE_BLOCKS", kObDecodeBlocks)));
        if (nt == 1)
            launch(onebit_one_rank_decode_kernel<T, true>, grid, dim3(kBlock), 0, s, seg + 32,
                   reinterpret_cast<const OneRankOut*>(seg), (int64_t)n, static_cast<S*>(tensor), tiles);
        else
            launch(onebit_one_rank_decode_kernel<T, false>, grid, dim3(kBlock), 0, s, seg + 32,
                   reinterpret_cast<const OneRankOut*>(seg), (int64_t)n, static_cast<S*>(tensor), tiles);
    }
    return check_launch();
}

}  // namespace bagua

using namespace bagua;

extern "C" {

size_t bagua_onebit_one_rank_workspace_bytes(int num_elem) {
    const int64_t tiles = ob_tiles(num_elem < 0 ? 0 : num_elem);
    const int64_t g1 = (tiles + kObTile - 1) / kObTile;
    return (size_t)(onerank_partials_offset(tiles) + ((tiles > 0 ? tiles : 1) + g1) * (int64_t)sizeof(float));
}

int bagua_onebit_centralized_one_rank(int dtype, void* tensor, int num_elem, int average, void* workspace,
                                      size_t workspace_bytes, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32: return ob_one_rank_impl<F32>(tensor, num_elem, average, workspace, workspace_bytes, s);
        case BAGUA_DTYPE_F16: return ob_one_rank_impl<F16>(tensor, num_elem, average, workspace, workspace_bytes, s);
        case BAGUA_DTYPE_BF16: return ob_one_rank_impl<BF16>(tensor, num_elem, average, workspace, workspace_bytes, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

size_t bagua_onebit_compressed_bytes(int chunk_size, int num_chunks) {
    return (size_t)num_chunks * (32 + (size_t)ob_tiles(chunk_size) * kObTileBytes);
}

size_t bagua_onebit_workspace_bytes(int chunk_size, int num_chunks) {
    const int64_t t = ob_tiles(chunk_size);
    return (size_t)(num_chunks > 0 ? num_chunks : 1) * (size_t)(t > 0 ? t : 1) * sizeof(float) + 256;
}

int bagua_onebit_compress(int dtype, const void* input, int input_num_element, int chunk_size, int num_chunks,
                          uint8_t* output, size_t output_bytes, void* workspace, size_t workspace_bytes,
                          int target_chunk, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return ob_compress_impl<F32>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                         workspace, workspace_bytes, target_chunk, s);
        case BAGUA_DTYPE_F16:
            return ob_compress_impl<F16>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                         workspace, workspace_bytes, target_chunk, s);
        case BAGUA_DTYPE_BF16:
            return ob_compress_impl<BF16>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                          workspace, workspace_bytes, target_chunk, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_onebit_decompress(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size, int num_chunks,
                            void* output, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32: return ob_decompress_impl<F32>(input, input_bytes, chunk_size, num_chunks, output, s);
        case BAGUA_DTYPE_F16: return ob_decompress_impl<F16>(input, input_bytes, chunk_size, num_chunks, output, s);
        case BAGUA_DTYPE_BF16: return ob_decompress_impl<BF16>(input, input_bytes, chunk_size, num_chunks, output, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_onebit_piece_range(int chunk_size, int pieces, int piece, int* tile_begin, int* tile_end) {
    if (chunk_size < 0 || pieces < 1 || piece < 0 || piece >= pieces || !tile_begin || !tile_end)
        return BAGUA_ERR_INVALID_ARG;
    const int64_t tiles = ob_tiles(chunk_size), per = (tiles + pieces - 1) / pieces;
    const int64_t b = (int64_t)piece * per < tiles ? (int64_t)piece * per : tiles;
    *tile_begin = (int)b;
    *tile_end = (int)(b + per < tiles ? b + per : tiles);
    return BAGUA_OK;
}

int bagua_onebit_encode_range(int dtype, const void* input, int input_num_element, int chunk_size, int num_chunks,
                              uint8_t* output, size_t output_bytes, void* workspace, size_t workspace_bytes,
                              int tile_begin, int tile_end, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return ob_compress_impl<F32>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                         workspace, workspace_bytes, -1, s, 1, tile_begin, tile_end);
        case BAGUA_DTYPE_F16:
            return ob_compress_impl<F16>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                         workspace, workspace_bytes, -1, s, 1, tile_begin, tile_end);
        case BAGUA_DTYPE_BF16:
            return ob_compress_impl<BF16>(input, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                          workspace, workspace_bytes, -1, s, 1, tile_begin, tile_end);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_onebit_finalize(const void* workspace, size_t workspace_bytes, int input_num_element, int chunk_size,
                          int num_chunks, uint8_t* output, size_t output_bytes, bagua_stream_t stream) {
    // the header math is dtype-independent (partials are f32)
    return ob_compress_impl<F32>(nullptr, input_num_element, chunk_size, num_chunks, output, output_bytes,
                                 const_cast<void*>(workspace), workspace_bytes, -1, static_cast<hipStream_t>(stream), 2);
}

int bagua_onebit_decompress_range(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                  int num_chunks, void* output, int tile_begin, int tile_end, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return ob_decompress_impl<F32>(input, input_bytes, chunk_size, num_chunks, output, s, tile_begin, tile_end);
        case BAGUA_DTYPE_F16:
            return ob_decompress_impl<F16>(input, input_bytes, chunk_size, num_chunks, output, s, tile_begin, tile_end);
        case BAGUA_DTYPE_BF16:
            return ob_decompress_impl<BF16>(input, input_bytes, chunk_size, num_chunks, output, s, tile_begin,
                                            tile_end);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_onebit_reduce_requantize(int dtype, const uint8_t* input, size_t input_bytes, int chunk_size,
                                   int num_chunks, void* tensor, int average, uint8_t* output, size_t output_bytes,
                                   int target_chunk, void* workspace, size_t workspace_bytes, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return ob_reduce_requantize_impl<F32>(input, input_bytes, chunk_size, num_chunks, tensor, average, output,
                                                  output_bytes, target_chunk, workspace, workspace_bytes, s);
        case BAGUA_DTYPE_F16:
            return ob_reduce_requantize_impl<F16>(input, input_bytes, chunk_size, num_chunks, tensor, average, output,
                                                  output_bytes, target_chunk, workspace, workspace_bytes, s);
        case BAGUA_DTYPE_BF16:
            return ob_reduce_requantize_impl<BF16>(input, input_bytes, chunk_size, num_chunks, tensor, average,
                                                   output, output_bytes, target_chunk, workspace, workspace_bytes, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

size_t onebit_temp_size_host(int chunk_size, int num_chunks) {
    return bagua_onebit_workspace_bytes(chunk_size, num_chunks);
}

#define V1(call) v1_check((call), __FILE__, __LINE__)
void compress_f32_to_onebit_host(float* input, int input_num_element, int chunk_size, int num_chunks, uint8_t* output,
                                 size_t output_size, void* dev_buffer, size_t dev_size, int target_chunk,
                                 bagua_stream_t stream) {
    V1(bagua_onebit_compress(BAGUA_DTYPE_F32, input, input_num_element, chunk_size, num_chunks, output, output_size,
                             dev_buffer, dev_size, target_chunk, stream));
}
void compress_bf16_to_onebit_host(bagua_bf16_t* input, int input_num_element, int chunk_size, int num_chunks,
                                  uint8_t* output, size_t output_size, void* dev_buffer, size_t dev_size,
                                  int target_chunk, bagua_stream_t stream) {
    V1(bagua_onebit_compress(BAGUA_DTYPE_BF16, input, input_num_element, chunk_size, num_chunks, output,
                             output_size, dev_buffer, dev_size, target_chunk, stream));
}
void decompress_onebit_to_f32_host(uint8_t* input, size_t input_size, int chunk_size, int num_chunks, float* output,
                                   bagua_stream_t stream) {
    V1(bagua_onebit_decompress(BAGUA_DTYPE_F32, input, input_size, chunk_size, num_chunks, output, stream));
}
void decompress_onebit_to_bf16_host(uint8_t* input, size_t input_size, int chunk_size, int num_chunks,
                                    bagua_bf16_t* output, bagua_stream_t stream) {
    V1(bagua_onebit_decompress(BAGUA_DTYPE_BF16, input, input_size, chunk_size, num_chunks, output, stream));
}
#undef V1

}  // extern "C"
