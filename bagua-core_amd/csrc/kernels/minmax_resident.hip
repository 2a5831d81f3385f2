// minmax_resident.hip — one-launch MinMax-UInt8 encode that keeps part of
// every chunk on chip across the chunk-wide min/max exchange.
//
// The reference encode (bagua_kernels.cu:533-571) reads each chunk three
// times (cub Min, cub Max, compress_float_to_uint8, K:268-371 + K:455-479);
// the two-kernel path in minmax_u8.hip reads it twice.  No payload byte can
// be emitted before the chunk's min/max is known, so the second read is
// intrinsic to any encoder that streams the chunk from HBM twice — but not to
// one that keeps what it read.  This kernel runs ONE workgroup per CU (the
// grid is the CU count), each owning one contiguous slice of a chunk:
//
//   pass 1: stream the slice once (default-policy loads): the first
//           R vectors per lane stay in VGPRs, the next H per lane are parked
//           in LDS (up to ~156 KiB per CU), the rest are only folded into the
//           min/max; publish the workgroup's {min, max} as two 8-byte
//           {tag, value} granules (the data is the flag: one atomic store
//           each, no fence, MI355X guide Guideline 16 R2)
//   exchange: one wave re-reads the chunk's granules until every tag is this
//           launch's, folds them (order-free keys, codec_common.hpp)
//   pass 2: quantise the streamed part first, in reverse (the lines pass 1
//           read last are the ones the 256 MiB Infinity Cache still holds),
//           then the LDS part, then the VGPR part, and write header / slack.
//
// Per-launch state lives in a library-owned slot (one per stream; the
// hipStreamPerThread sentinel gets one per host thread) that is never reset:
// launch k on a slot draws tickets [kG, (k+1)G) from monotonic counters, so
// its tag is k+1 (no memset node, graph-replay safe).  The tickets (and the
// drain count below) are spread over kResLanes counters on separate 128-B lines,
// workgroup g on counter g % kResLanes (its XCD under round-robin placement):
// 256 returning atomics on ONE word serialise at the memory side (≈ 88 per µs,
// MI355X guide "dequeue"), which held the last workgroup's start ~3 µs back.  Every workgroup bumps a
// second counter once it is done with the slot (after the exchange), so the
// host can tell when every launch it issued on a slot has let go of it; a
// slot changes owner (release, or LRU reclaim when all 64 are taken) only then.
// (An event recorded behind every launch cost 3-5 us per step, even without a
// system-scope fence: profiles/r02_slot_event_ab.jsonl.)
//
// Residency: the exchange needs every workgroup of a chunk resident at once.
// The grid equals the CU count and the kernel admits one workgroup per CU,
// but another stream's kernels can occupy CUs, so the wait is BOUNDED: a
// workgroup that times out folds every slice whose partials are still
// missing straight from memory (min/max is order-free and idempotent, so any
// mix of published partials and re-read slices is the chunk's exact min/max)
// and quantises its own slice.  The late workgroup, once it runs, finds the
// partials of all the others published and finishes normally.  No second
// kernel, no spin without a deadline; the bytes are the same either way.
//
// Bit-identity: the same per-element expressions as minmax_quantize_kernel;
// the min/max is order-free, so slicing cannot change it.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <map>
#include <mutex>
#include <set>
#include <thread>
#include <utility>

#include "codec_common.hpp"
#include "launch_util.hpp"

namespace bagua {

constexpr int kResMaxGrid = 1024;
constexpr int kResSlots = 64;
constexpr int kResLanes = 8;  // ticket / drain counters per slot (one per XCD)

struct ResidentSlot {
    uint64_t ticket[kResLanes][16];   // monotonic ticket counters, one 128-B line each (workgroup g: lane g % 8)
    uint64_t drained[kResLanes][16];  // workgroups done with the slot, per lane (once each, at its end)
    uint64_t gave_up;                 // workgroups that timed out in the exchange (bagua_minmax_u8_resident_give_ups)
    uint64_t pad0[15];
    uint64_t gran[2 * kResMaxGrid];   // {tag << 32 | min key}, {tag << 32 | max key} per workgroup
};
static_assert(sizeof(ResidentSlot) % 64 == 0, "slot alignment");

struct ResidentArgs {
    const void* in;
    int64_t cs;            // chunk size (elements)
    int target;            // -1: all chunks
    int nact;              // active chunks
    int bpc;               // workgroups per active chunk
    int grid;              // launched workgroups (the CU count; idle ones >= nact * bpc)
    uint8_t* out;
    int64_t chunk_offset;  // bytes per segment
    int64_t out_bytes;
    int num_chunks;
    ResidentSlot* slot;
    uint64_t timeout_ticks;  // wall_clock64 ticks a workgroup waits for its chunk's partials
    uint64_t* trace;         // measurement hook: 8 wall_clock64 slots per workgroup, or nullptr
};

__device__ __forceinline__ void trace_stamp(const ResidentArgs& a, int g, int k) {
    if (a.trace != nullptr && threadIdx.x == 0) a.trace[8 * g + k] = wall_clock64();
}

// every launch on a slot has the same grid, so counter c receives the same number
// of tickets per launch: the workgroups g < grid with g % kResLanes == c
__device__ __forceinline__ uint32_t tag_of_ticket(uint64_t ticket, int grid, int lane) {
    const uint64_t per_launch = (uint64_t)((grid - lane + kResLanes - 1) / kResLanes);
    return (uint32_t)((ticket / per_launch) % 0xffffffffull) + 1u;  // never 0 (the zeroed state)
}

template <typename T, int BLOCK>
struct SliceGeom {
    using S = typename T::storage;
    int c;               // chunk index in the tensor
    int cl;              // active-chunk index
    int b;               // slice index within the chunk
    const S* src;        // chunk start
    uint8_t* seg;        // chunk's segment
    uint8_t* payload;    // seg + 32
    int64_t j0;          // elements before the vector body (scalar head)
    int64_t nvec;        // body vectors
    int64_t v0, v1;      // this slice's vectors [v0, v1)
    bool last;           // last slice of the chunk: owns head, tail and slack

    __device__ __forceinline__ SliceGeom(const ResidentArgs& a, int g) {
        constexpr int N = Vec<T>::N;
        cl = g / a.bpc;
        b = g - cl * a.bpc;
        c = a.target < 0 ? cl : a.target;
        src = static_cast<const S*>(a.in) + (int64_t)c * a.cs;
        seg = a.out + (int64_t)c * a.chunk_offset;
        payload = seg + 32;
        const int al = common_alignment<T>((uintptr_t)src, (uintptr_t)payload);  // host checked >= 0
        j0 = al < a.cs ? al : a.cs;
        nvec = (a.cs - j0) / N;
        const int64_t per = ((nvec + a.bpc - 1) / a.bpc + BLOCK - 1) / BLOCK * BLOCK;
        v0 = (int64_t)b * per;
        v0 = v0 < nvec ? v0 : nvec;
        v1 = v0 + per < nvec ? v0 + per : nvec;
        last = (b == a.bpc - 1);
    }
};

template <typename T>
__device__ __forceinline__ void fold_vec(const uint4& r, uint32_t& lo, uint32_t& hi) {
    float f[Vec<T>::N];
    unpack16<T>(r, f);
#pragma unroll
    for (int i = 0; i < Vec<T>::N; ++i) {
        const int32_t k = f2key(f[i]);
        lo = min(lo, min_space_key(k));
        hi = min(hi, max_space_key(k));
    }
}

// the scalar head and tail elements of a chunk (owned by its last slice)
template <typename T, int BLOCK>
__device__ __forceinline__ void fold_scalars(const ResidentArgs& a, const SliceGeom<T, BLOCK>& s, uint32_t& lo,
                                             uint32_t& hi) {
    constexpr int N = Vec<T>::N;
    const int t = (int)threadIdx.x;
    for (int64_t j = t; j < s.j0; j += BLOCK) {
        const int32_t k = f2key(T::to_f(s.src[j]));
        lo = min(lo, min_space_key(k));
        hi = min(hi, max_space_key(k));
    }
    for (int64_t j = s.j0 + s.nvec * N + t; j < a.cs; j += BLOCK) {
        const int32_t k = f2key(T::to_f(s.src[j]));
        lo = min(lo, min_space_key(k));
        hi = min(hi, max_space_key(k));
    }
}

template <int SB, int BLOCK, bool NT = false>
__device__ __forceinline__ void load_tile(const uint4* __restrict__ v, int64_t base, int t, uint4 (&r)[SB]) {
#pragma unroll
    for (int j = 0; j < SB; ++j) r[j] = NT ? nt_load16(&v[base + j * BLOCK + t]) : v[base + j * BLOCK + t];
}

template <typename T>
__device__ __forceinline__ void quant_store(const uint4& r, const QParams& q, uint8_t* dst) {
    float f[Vec<T>::N];
    unpack16<T>(r, f);
    quant_store_vec<T>(f, q, dst);
}

// header of chunk c (slice 0), slack after the payload and the buffer tail
// (last slice), scalar head and tail elements (last slice) -- the same bytes
// minmax_quantize_kernel writes
template <typename T, int BLOCK>
__device__ void write_extras(const ResidentArgs& a, const SliceGeom<T, BLOCK>& s, float mn, float mx,
                             const QParams& q) {
    using S = typename T::storage;
    constexpr int N = Vec<T>::N;
    const int t = (int)threadIdx.x;
    if (s.b == 0 && t < 32) {
        const uint32_t bmn = sizeof(S) == 4 ? __float_as_uint(mn) : (uint32_t)T::from_f(mn);
        const uint32_t bmx = sizeof(S) == 4 ? __float_as_uint(mx) : (uint32_t)T::from_f(mx);
        uint32_t hb = 0;
        if (t < (int)sizeof(S)) hb = (bmn >> (8 * t)) & 0xff;
        else if (t < 2 * (int)sizeof(S)) hb = (bmx >> (8 * (t - (int)sizeof(S)))) & 0xff;
        s.seg[t] = (uint8_t)hb;
    }
    if (!s.last) return;
    for (int64_t j = 32 + a.cs + t; j < a.chunk_offset; j += BLOCK) s.seg[j] = 0;
    if (a.target < 0 && s.c == a.num_chunks - 1)
        for (int64_t j = (int64_t)a.num_chunks * a.chunk_offset + t; j < a.out_bytes; j += BLOCK) a.out[j] = 0;
    for (int64_t j = t; j < s.j0; j += BLOCK) s.payload[j] = (uint8_t)quant(T::to_f(s.src[j]), q);
    for (int64_t j = s.j0 + s.nvec * N + t; j < a.cs; j += BLOCK)
        s.payload[j] = (uint8_t)quant(T::to_f(s.src[j]), q);
}

// one wave folds the granules of active chunk `cl`; false once `deadline` passes
__device__ __forceinline__ bool sweep_chunk(const ResidentArgs& a, int cl, uint32_t tag, uint64_t deadline,
                                            uint32_t& lo, uint32_t& hi, bool bounded) {
    const int lane = lane_id();
    const uint64_t* g = a.slot->gran + 2 * (int64_t)cl * a.bpc;
    const int n = 2 * a.bpc;
    for (;;) {
        bool ok = true;
        uint32_t l = 0xffffffffu, h = 0xffffffffu;
        for (int i = lane; i < n; i += kWave) {
            const uint64_t x = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok &= (uint32_t)(x >> 32) == tag;
            if (i & 1) h = min(h, (uint32_t)x);
            else l = min(l, (uint32_t)x);
        }
        if (__all(ok)) {
            lo = wave_umin(l);
            hi = wave_umin(h);
            return true;
        }
        if (bounded && (uint64_t)wall_clock64() > deadline) return false;
        __builtin_amdgcn_s_sleep(2);
    }
}

// after a give-up: the calling thread's share of the chunk's min/max, taking a
// slice's published partials when both carry this launch's tag and re-reading
// the slice otherwise.  Threads may disagree about a granule that lands
// meanwhile; every slice is then still covered whole (by the granule some
// thread took, or by all threads' strided re-reads), so the union is exact.
template <typename T, int BLOCK>
__device__ void fold_missing_slices(const ResidentArgs& a, int cl, uint32_t tag, uint32_t& lo, uint32_t& hi) {
    const int t = (int)threadIdx.x;
    for (int b = 0; b < a.bpc; ++b) {
        const int gg = cl * a.bpc + b;
        const uint64_t* gr = a.slot->gran + 2 * (int64_t)gg;
        const uint64_t x0 = __hip_atomic_load(gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t x1 = __hip_atomic_load(gr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(x0 >> 32) == tag && (uint32_t)(x1 >> 32) == tag) {
            lo = min(lo, (uint32_t)x0);
            hi = min(hi, (uint32_t)x1);
            continue;
        }
        const SliceGeom<T, BLOCK> sg(a, gg);
        const uint4* __restrict__ v = reinterpret_cast<const uint4*>(sg.src + sg.j0);
        for (int64_t i = sg.v0 + t; i < sg.v1; i += BLOCK) fold_vec<T>(v[i], lo, hi);
        if (sg.last) fold_scalars<T, BLOCK>(a, sg, lo, hi);
    }
}

// NTM: non-temporal load mask -- bit 0: pass 2's re-reads of the streamed part;
// bit 1: pass 1's loads of the part kept on chip (held in VGPRs / parked in LDS), which
// nothing re-reads, so they need not take Infinity-Cache lines from the streamed part
template <typename T, int BLOCK, int R, int H, int SB, int NTM>
__global__ __launch_bounds__(BLOCK, 1) void minmax_resident_encode_kernel(ResidentArgs a) {
    constexpr int N = Vec<T>::N;
    constexpr bool NT = (NTM & 1) != 0;
    constexpr bool NT1 = (NTM & 2) != 0;
    constexpr int W = BLOCK / kWave;
    // dynamic LDS only (guide Guideline 17): [H * BLOCK parked vectors][scratch]
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    uint4* park = smem;
    uint32_t* scratch = reinterpret_cast<uint32_t*>(smem + H * BLOCK);  // 2*W + 4 words
    const int t = (int)threadIdx.x;
    const int g = (int)blockIdx.x;

    const int lane_c = g % kResLanes;
    if (t == 0) {
        const uint64_t ticket = __hip_atomic_fetch_add(&a.slot->ticket[lane_c][0], (uint64_t)1, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        scratch[2 * W] = tag_of_ticket(ticket, a.grid, lane_c);
    }
    __syncthreads();
    const uint32_t tag = scratch[2 * W];
    trace_stamp(a, g, 0);
    if (g >= a.nact * a.bpc) {  // idle: the grid is the CU count on every launch of the slot
        if (t == 0)
            __hip_atomic_fetch_add(&a.slot->drained[lane_c][0], (uint64_t)1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        return;
    }

    const SliceGeom<T, BLOCK> s(a, g);
    const uint4* __restrict__ v = reinterpret_cast<const uint4*>(s.src + s.j0);
    const int64_t v0 = s.v0, v1 = s.v1;
    const int64_t stream0 = v0 + (int64_t)(R + H) * BLOCK;  // first streamed vector

    // ---- pass 1 ------------------------------------------------------------
    uint32_t lo = min_space(T::init_max());
    uint32_t hi = max_space(-T::init_max());
    uint4 held[R > 0 ? R : 1];
    if (v1 > v0) {
        const int64_t vl = v1 - 1;  // clamp: a duplicate of a slice element never changes the min/max
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t i = v0 + (int64_t)k * BLOCK + t;
            held[k] = NT1 ? nt_load16(&v[i < vl ? i : vl]) : v[i < vl ? i : vl];
        }
        // software-pipelined: the next batch of parked vectors is in flight while the
        // current one (first: the held vectors) is folded, so memory never waits on VALU
        uint4 cur[SB], nxt[SB];
#pragma unroll
        for (int j = 0; j < SB; ++j) {
            if (j < H) {
                const int64_t i = v0 + (int64_t)(R + j) * BLOCK + t;
                cur[j] = NT1 ? nt_load16(&v[i < vl ? i : vl]) : v[i < vl ? i : vl];
            }
        }
#pragma unroll
        for (int k = 0; k < R; ++k) fold_vec<T>(held[k], lo, hi);
#pragma unroll
        for (int kb = 0; kb < H; kb += SB) {
#pragma unroll
            for (int j = 0; j < SB; ++j) {
                if (kb + SB + j < H) {
                    const int64_t i = v0 + (int64_t)(R + kb + SB + j) * BLOCK + t;
                    nxt[j] = NT1 ? nt_load16(&v[i < vl ? i : vl]) : v[i < vl ? i : vl];
                }
            }
#pragma unroll
            for (int j = 0; j < SB; ++j) {
                if (kb + j < H) {
                    fold_vec<T>(cur[j], lo, hi);
                    park[(kb + j) * BLOCK + t] = cur[j];
                }
            }
#pragma unroll
            for (int j = 0; j < SB; ++j) cur[j] = nxt[j];
        }
        // streamed part: full tiles double-buffered (2 x SB loads in flight per
        // lane: with one wave per SIMD nothing else hides the latency), then the
        // ragged tail tile
        const int64_t tile = (int64_t)SB * BLOCK;
        const int64_t nfull = v1 > stream0 ? (v1 - stream0) / tile : 0;
        if (nfull > 0) {
            uint4 ra[SB], rb[SB];
            load_tile<SB, BLOCK>(v, stream0, t, ra);
            for (int64_t i = 0; i < nfull; i += 2) {
                // unconditional (clamped) prefetches keep the wait counts static
                load_tile<SB, BLOCK>(v, stream0 + (i + 1 < nfull ? i + 1 : nfull - 1) * tile, t, rb);
#pragma unroll
                for (int j = 0; j < SB; ++j) fold_vec<T>(ra[j], lo, hi);
                load_tile<SB, BLOCK>(v, stream0 + (i + 2 < nfull ? i + 2 : nfull - 1) * tile, t, ra);
                if (i + 1 < nfull) {
#pragma unroll
                    for (int j = 0; j < SB; ++j) fold_vec<T>(rb[j], lo, hi);
                }
            }
        }
        for (int j = 0; j < SB; ++j) {
            const int64_t i = stream0 + nfull * tile + j * BLOCK + t;
            if (i < v1) fold_vec<T>(v[i], lo, hi);
        }
    }
    if (s.last) fold_scalars<T, BLOCK>(a, s, lo, hi);
    lo = wave_umin(lo);
    hi = wave_umin(hi);
    const int w = t / kWave;
    if (lane_id() == 0) { scratch[w] = lo; scratch[W + w] = hi; }
    __syncthreads();
    if (t == 0) {
#pragma unroll
        for (int i = 1; i < W; ++i) { lo = min(lo, scratch[i]); hi = min(hi, scratch[W + i]); }
        uint64_t* mine = a.slot->gran + 2 * (int64_t)g;
        __hip_atomic_store(mine, ((uint64_t)tag << 32) | lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(mine + 1, ((uint64_t)tag << 32) | hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // the first tile pass 2 re-reads (the top full tile: reverse order) is loaded
    // now, so its latency overlaps the exchange wait instead of following it
    const int64_t tile2 = (int64_t)SB * BLOCK;
    const int64_t nfull2 = v1 > stream0 ? (v1 - stream0) / tile2 : 0;
    uint4 pre[SB], pre2[SB];
    if (nfull2 > 0) load_tile<SB, BLOCK, NT>(v, stream0 + (nfull2 - 1) * tile2, t, pre);
    if (nfull2 > 1) load_tile<SB, BLOCK, NT>(v, stream0 + (nfull2 - 2) * tile2, t, pre2);

    trace_stamp(a, g, 1);
    // ---- exchange ------------------------------------------------------------
    if (w == 0) {
        const uint64_t deadline = wall_clock64() + a.timeout_ticks;
        uint32_t l = 0, h = 0;
        const bool ok = sweep_chunk(a, s.cl, tag, deadline, l, h, true);
        if (lane_id() == 0) {
            scratch[2 * W + 1] = ok ? 1u : 0u;
            scratch[2 * W + 2] = l;
            scratch[2 * W + 3] = h;
        }
    }
    __syncthreads();
    if (scratch[2 * W + 1] == 0u) {
        // gave up waiting: the whole workgroup folds the missing slices itself
        if (t == 0) __hip_atomic_fetch_add(&a.slot->gave_up, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t l = 0xffffffffu, h = 0xffffffffu;
        fold_missing_slices<T, BLOCK>(a, s.cl, tag, l, h);
        l = wave_umin(l);
        h = wave_umin(h);
        if (lane_id() == 0) { scratch[w] = l; scratch[W + w] = h; }
        __syncthreads();
        if (t == 0) {
#pragma unroll
            for (int i = 1; i < W; ++i) { l = min(l, scratch[i]); h = min(h, scratch[W + i]); }
            scratch[2 * W + 2] = l;
            scratch[2 * W + 3] = h;
        }
        __syncthreads();
    }
    const float mn = from_min_space(scratch[2 * W + 2]), mx = from_max_space(scratch[2 * W + 3]);
    const QParams q = make_qparams(mn, mx);
    trace_stamp(a, g, 2);

    // ---- pass 2 ------------------------------------------------------------
    write_extras<T, BLOCK>(a, s, mn, mx, q);
    uint8_t* vdst = s.payload + s.j0;
    if (v1 > stream0) {
        // reverse order (what pass 1 read last is re-read first): the ragged
        // top tile, then the full tiles double-buffered from the top down
        const int64_t tile = (int64_t)SB * BLOCK;
        const int64_t nfull = (v1 - stream0) / tile;
        for (int j = 0; j < SB; ++j) {
            const int64_t i = stream0 + nfull * tile + j * BLOCK + t;
            if (i < v1) quant_store<T>(v[i], q, vdst + i * N);
        }
        if (nfull > 0) {
            uint4 ra[SB], rb[SB];
#pragma unroll
            for (int j = 0; j < SB; ++j) { ra[j] = pre[j]; rb[j] = pre2[j]; }  // loaded before the exchange
            for (int64_t i = nfull - 1; i >= 0; i -= 2) {
                if (i != nfull - 1 || nfull < 2) load_tile<SB, BLOCK, NT>(v, stream0 + (i >= 1 ? i - 1 : 0) * tile, t, rb);
                const int64_t ba = stream0 + i * tile;
#pragma unroll
                for (int j = 0; j < SB; ++j) quant_store<T>(ra[j], q, vdst + (ba + j * BLOCK + t) * N);
                load_tile<SB, BLOCK, NT>(v, stream0 + (i >= 2 ? i - 2 : 0) * tile, t, ra);
                if (i >= 1) {
                    const int64_t bb = ba - tile;
#pragma unroll
                    for (int j = 0; j < SB; ++j) quant_store<T>(rb[j], q, vdst + (bb + j * BLOCK + t) * N);
                }
            }
        }
    }
    trace_stamp(a, g, 4);
    if (v0 + (int64_t)(R + H) * BLOCK <= v1) {
        // the whole on-chip part is inside the slice (every slice of a bucket this path
        // takes): no per-vector guards, so the LDS reads of a batch issue back to back
        // and the quantise+stores pipeline (a guarded vector was its own exec-masked
        // block that waited on its own ds_read: 11 us for 36 % of the payload)
        uint8_t* vd = vdst + (v0 + t) * N;
#pragma unroll
        for (int kb = 0; kb < H; kb += SB) {
            uint4 r[SB];
#pragma unroll
            for (int j = 0; j < SB; ++j)
                if (kb + j < H) r[j] = park[(kb + j) * BLOCK + t];
#pragma unroll
            for (int j = 0; j < SB; ++j)
                if (kb + j < H) quant_store<T>(r[j], q, vd + (int64_t)(R + kb + j) * BLOCK * N);
        }
        trace_stamp(a, g, 5);
#pragma unroll
        for (int k = 0; k < R; ++k) quant_store<T>(held[k], q, vd + (int64_t)k * BLOCK * N);
    } else {
#pragma unroll
        for (int k = 0; k < H; ++k) {
            const int64_t i = v0 + (int64_t)(R + k) * BLOCK + t;
            if (i < v1) quant_store<T>(park[k * BLOCK + t], q, vdst + i * N);
        }
        trace_stamp(a, g, 5);
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t i = v0 + (int64_t)k * BLOCK + t;
            if (i < v1) quant_store<T>(held[k], q, vdst + i * N);
        }
    }
    if (a.trace != nullptr) {
        __syncthreads();
        trace_stamp(a, g, 3);
    }
    // the workgroup let go of the slot (its granule reads ended at the exchange's
    // barriers); counted last, so no later load waits behind this atomic (on gfx9
    // a non-returning atomic still holds vmcnt: mid-kernel it cost ~1.3 us,
    // profiles/r03_resident_versions_ab.jsonl)
    if (t == 0)
        __hip_atomic_fetch_add(&a.slot->drained[lane_c][0], (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------
// Slot keys.  hipStreamPerThread is a sentinel that names a DIFFERENT real
// stream on every host thread, so two threads launching on it must not share a
// slot (their tickets and granules would interleave): the sentinel is keyed
// together with the calling thread.  Every other handle is one stream.
struct StreamKey {
    hipStream_t s = nullptr;
    std::thread::id tid{};
    bool operator<(const StreamKey& o) const { return s != o.s ? s < o.s : tid < o.tid; }
    bool operator==(const StreamKey& o) const { return s == o.s && tid == o.tid; }
};
static StreamKey stream_key(hipStream_t s) {
    StreamKey k;
    k.s = s;
    if (s == hipStreamPerThread) k.tid = std::this_thread::get_id();
    return k;
}

struct SlotState {
    bool used = false;
    bool captured = false;  // a graph holds a launch on this slot: never reused (see below)
    StreamKey owner;
    uint64_t last_use = 0;  // LRU clock
    uint64_t launched = 0;  // workgroups launched on the slot since it was zeroed
};

struct ResidentDevice {
    bool init = false, ok = false;
    int grid = 0;
    int clock_khz = 0;
    ResidentSlot* slots = nullptr;
    uint64_t* probe_host = nullptr;  // pinned landing buffer for reading `drained` (kResLanes lines)
    SlotState state[kResSlots];
    std::map<StreamKey, int> stream_slot;
    uint64_t clock = 0;
    bool warned_full = false;
};
static std::mutex g_res_mu;
// streams whose compress calls never take the one-launch encode: streams that run
// codec work concurrently with another codec stream (the scheduler's lanes), where two
// encodes each needing every CU resident would wait on each other (bounded, but slow);
// guarded by g_res_mu
static std::set<hipStream_t>& resident_off_streams() {
    static auto* s = new std::set<hipStream_t>();
    return *s;
}
static uint64_t* g_res_trace = nullptr;  // bagua_minmax_u8_resident_trace
static ResidentDevice g_res_dev[64];

// kernel configurations: {BLOCK, R vectors per lane in VGPRs, H per lane in LDS, SB stream batch}
struct ResidentCfg {
    int block, r, h, sb;
    int ntm;  // non-temporal loads: bit 0 pass-2 re-reads, bit 1 pass-1 loads of the on-chip part
};
static constexpr ResidentCfg kResCfg[] = {
    {256, 32, 39, 8, 0},   // 0
    {256, 48, 39, 8, 0},   // 1
    {512, 24, 19, 8, 0},   // 2
    {256, 0, 0, 8, 0},     // 3: no retention (Infinity Cache only)
    {256, 32, 0, 8, 0},    // 4: VGPRs only
    {256, 16, 39, 16, 0},  // 5
    {256, 64, 39, 8, 0},   // 6
    {256, 80, 39, 8, 0},   // 7
    {256, 72, 39, 8, 0},   // 8
    {512, 28, 19, 8, 0},   // 9
    {256, 80, 39, 8, 1},    // 10
    {512, 28, 19, 8, 1},       // 11
    {512, 28, 19, 8, 3},       // 12: 11 + the on-chip part loaded non-temporally
    {512, 28, 19, 8, 2},       // 13: only the on-chip part non-temporal
};
constexpr int kResNumCfg = (int)(sizeof(kResCfg) / sizeof(kResCfg[0]));
// 12: config 11 with the on-chip part of pass 1 also loaded non-temporally.  The
// one-bucket loop is unchanged (1,894-1,898 vs 1,892-1,916 GiB/s), and alternating
// buckets -- a bucket last touched a whole other bucket ago, as in training -- gain
// 1,900-1,928 vs 1,849-1,886 GiB/s (profiles/r04_resident_ntm_ab.jsonl; 13, the
// on-chip part non-temporal with default re-reads, shortens the encode to 78-80 us
// but slows the decode after it by as much)
constexpr int kResDefaultCfg = 12;

static size_t resident_lds_bytes(const ResidentCfg& c) {
    return (size_t)c.h * c.block * 16 + 16 * ((2 * (c.block / kWave) + 4 + 3) / 4);
}

template <typename T, int CFG>
static void* resident_kernel_ptr() {
    constexpr ResidentCfg c = kResCfg[CFG];
    return reinterpret_cast<void*>(&minmax_resident_encode_kernel<T, c.block, c.r, c.h, c.sb, c.ntm>);
}

template <typename T>
static void* resident_kernel_for(int cfg) {
    switch (cfg) {
        case 0: return resident_kernel_ptr<T, 0>();
        case 1: return resident_kernel_ptr<T, 1>();
        case 2: return resident_kernel_ptr<T, 2>();
        case 3: return resident_kernel_ptr<T, 3>();
        case 4: return resident_kernel_ptr<T, 4>();
        case 5: return resident_kernel_ptr<T, 5>();
        case 6: return resident_kernel_ptr<T, 6>();
        case 7: return resident_kernel_ptr<T, 7>();
        case 8: return resident_kernel_ptr<T, 8>();
        case 9: return resident_kernel_ptr<T, 9>();
        case 10: return resident_kernel_ptr<T, 10>();
        case 11: return resident_kernel_ptr<T, 11>();
        case 12: return resident_kernel_ptr<T, 12>();
        case 13: return resident_kernel_ptr<T, 13>();
    }
    return nullptr;
}

static int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return (e && *e) ? atoi(e) : dflt;
}

// Per-device state (slot array zeroed once); false when the resident path is
// unavailable on `dev`.  Caller holds g_res_mu.
static bool device_ready(int dev) {
    if (dev < 0 || dev >= 64) return false;
    ResidentDevice& d = g_res_dev[dev];
    if (!d.init) {
        d.init = true;
        int cus = 0, khz = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return false;
        if (cus < 1 || cus > kResMaxGrid || khz < 1) return false;
        void* p = nullptr;
        const size_t bytes = sizeof(ResidentSlot) * kResSlots;
        if (hipMalloc(&p, bytes) != hipSuccess) return false;
        if (hipMemset(p, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            (void)hipFree(p);
            return false;
        }
        // no private stream: with GPU_MAX_HW_QUEUES = 4 one more stream shares a
        // hardware queue with the caller's streams and serialised, e.g., the
        // host-resident bench's H2D and D2H copies (43 -> 27 GiB/s)
        void* h = nullptr;
        if (hipHostMalloc(&h, sizeof(ResidentSlot::drained), hipHostMallocDefault) != hipSuccess) {
            (void)hipFree(p);
            return false;
        }
        d.probe_host = static_cast<uint64_t*>(h);
        d.slots = static_cast<ResidentSlot*>(p);
        d.grid = cus;
        d.clock_khz = khz;
        d.ok = true;
    }
    return d.ok;
}

// Waits until every workgroup launched on slot `idx` has let go of it (its
// `drained` count reaches the launched count).  The counter is read with a copy
// on `via` (a stream the caller knows to be alive: the stream being released,
// or the stream about to take the slot over), which is drained first; the old
// owner's launches may run on another stream, hence the loop.  Caller holds
// g_res_mu.  Rare: release, or more than kResSlots streams.
static int wait_slot_drained(int dev, int idx, hipStream_t via) {
    ResidentDevice& d = g_res_dev[dev];
    const uint64_t want = d.state[idx].launched;
    for (;;) {
        if (hipMemcpyAsync(d.probe_host, &d.slots[idx].drained[0][0], sizeof(ResidentSlot::drained),
                           hipMemcpyDeviceToHost, via) != hipSuccess ||
            hipStreamSynchronize(via) != hipSuccess) {
            g_last_hip_error = (int)hipGetLastError();
            return BAGUA_ERR_HIP;
        }
        uint64_t got = 0;
        for (int c = 0; c < kResLanes; ++c) got += d.probe_host[16 * c];
        if (got >= want) return BAGUA_OK;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// Slot of stream `s` on `dev` (caller holds g_res_mu; device_ready(dev) is
// true), or -1.  A new stream takes a free slot; when all kResSlots are owned
// the least recently used one is reclaimed once every launch issued on it has
// let go of it (wait_slot_drained), so no two launches ever run on one slot at
// once.  The ticket counter stays monotonic across owners.
static int acquire_slot_locked(int dev, hipStream_t s) {
    ResidentDevice& d = g_res_dev[dev];
    const StreamKey key = stream_key(s);
    int idx = -1;
    auto it = d.stream_slot.find(key);
    if (it != d.stream_slot.end()) {
        idx = it->second;
    } else {
        for (int i = 0; i < kResSlots && idx < 0; ++i)
            if (!d.state[i].used && !d.state[i].captured) idx = i;
        if (idx < 0) {
            for (int i = 0; i < kResSlots; ++i)
                if (!d.state[i].captured && (idx < 0 || d.state[i].last_use < d.state[idx].last_use)) idx = i;
            if (idx < 0) return -1;  // every slot is held by a captured graph
            SlotState& old = d.state[idx];
            if (wait_slot_drained(dev, idx, s) != BAGUA_OK) return -1;
            d.stream_slot.erase(old.owner);
            if (!d.warned_full) {
                d.warned_full = true;
                fprintf(stderr,
                        "[bagua-core] one-launch encode: %d streams in use on device %d; reclaiming the least "
                        "recently used slot (release streams with bagua_minmax_u8_release_stream)\n",
                        kResSlots, dev);
            }
        }
        SlotState& st = d.state[idx];
        st.used = true;
        st.owner = key;
        d.stream_slot.emplace(key, idx);
    }
    d.state[idx].last_use = ++d.clock;
    return idx;
}

// Launch plan of the one-launch encode; ok == false: not eligible (the caller
// runs the two-kernel encode)
struct ResidentPlan {
    bool ok = false;
    int cfg = 0;
    int dev = 0;
    size_t lds = 0;
    ResidentArgs a{};
};

template <typename T>
static ResidentPlan resident_plan(const void* input, int64_t in_num_elem, int64_t cs, int p, uint8_t* out,
                                  int64_t out_bytes, int target, hipStream_t s) {
    using S = typename T::storage;
    ResidentPlan pl;
    const int cfg = env_int("BAGUA_RESIDENT_CFG", kResDefaultCfg);
    if (env_int("BAGUA_RESIDENT", 1) == 0 || cfg < 0 || cfg >= kResNumCfg || p <= 0) return pl;
    {
        std::lock_guard<std::mutex> lk(g_res_mu);
        if (resident_off_streams().count(s)) return pl;
    }
    const int nact = target < 0 ? p : 1;
    const int64_t chunk_offset = out_bytes / p;
    // whole chunks only, every active chunk fully valid, large enough to pay for the exchange
    if (in_num_elem < (target < 0 ? (int64_t)p * cs : ((int64_t)target + 1) * cs)) return pl;
    // below ~12 Mi elements the fixed cost of the exchange (~4 us: publish + sweep across
    // XCDs) and of starting one 512-thread workgroup per CU (~3 us) loses to the
    // two-kernel encode (crossover between 8 Mi and 16 Mi)
    if (cs * nact < env_int("BAGUA_RESIDENT_MIN_ELEMS", 12 << 20)) return pl;
    for (int i = 0; i < nact; ++i) {
        const int c = target < 0 ? i : target;
        const uintptr_t src = (uintptr_t)(static_cast<const S*>(input) + (int64_t)c * cs);
        const uintptr_t pay = (uintptr_t)(out + (int64_t)c * chunk_offset + 32);
        if (src % sizeof(S) != 0 || common_alignment<T>(src, pay) < 0) return pl;
    }
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return pl;
    int grid = 0, khz = 0;
    {
        std::lock_guard<std::mutex> lk(g_res_mu);
        if (!device_ready(dev)) return pl;
        grid = g_res_dev[dev].grid;
        khz = g_res_dev[dev].clock_khz;
    }
    if (nact > grid) return pl;
    const ResidentCfg& c = kResCfg[cfg];
    void* kern = resident_kernel_for<T>(cfg);
    const size_t lds = resident_lds_bytes(c);
    {
        // once per (device, dtype, configuration): dynamic LDS above the default, and
        // one workgroup per CU must be admissible (the exchange needs the grid resident)
        static int admitted[64][kResNumCfg];  // 0 unknown, 1 yes, -1 no
        std::lock_guard<std::mutex> lk(g_res_mu);
        int& st = admitted[dev][cfg];
        if (st == 0) {
            int per_cu = 0;
            st = (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess &&
                  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, c.block, lds) == hipSuccess &&
                  per_cu >= 1)
                     ? 1
                     : -1;
            (void)hipGetLastError();
        }
        if (st < 0) return pl;
    }
    ResidentArgs& a = pl.a;
    a.in = input;
    a.cs = cs;
    a.target = target;
    a.nact = nact;
    a.bpc = grid / nact;
    a.grid = grid;
    a.out = out;
    a.chunk_offset = chunk_offset;
    a.out_bytes = out_bytes;
    a.num_chunks = p;
    a.slot = nullptr;  // taken at launch (resident_compress_impl)
    // bounded wait: the exchange normally completes a few us after the slowest
    // workgroup's pass 1, which reads the active chunks; allow that pass to run
    // at as little as 0.5 TB/s before giving up (then the waiting workgroups
    // re-read the missing slices themselves)
    const int64_t active_bytes = cs * nact * (int64_t)sizeof(S);
    const int64_t us = env_int("BAGUA_RESIDENT_TIMEOUT_US", (int)(200 + active_bytes / 500000));
    a.timeout_ticks = (uint64_t)(us < 0 ? 0 : us) * (uint64_t)khz / 1000u;
    a.trace = g_res_trace;
    pl.cfg = cfg;
    pl.lds = lds;
    pl.dev = dev;
    pl.ok = true;
    return pl;
}

// BAGUA_ERR_UNSUPPORTED: not eligible (the caller runs the two-kernel encode)
template <typename T>
int resident_compress_impl(const void* input, int64_t in_num_elem, int64_t cs, int p, uint8_t* out,
                           int64_t out_bytes, int target, hipStream_t s) {
    ResidentPlan pl = resident_plan<T>(input, in_num_elem, cs, p, out, out_bytes, target, s);
    if (!pl.ok) return BAGUA_ERR_UNSUPPORTED;
    // slot choice, launch and the slot's launched count happen under one lock, so a
    // reclaim (acquire_slot_locked) always waits for the slot's latest launch
    std::lock_guard<std::mutex> lk(g_res_mu);
    ResidentDevice& d = g_res_dev[pl.dev];
    const int idx = acquire_slot_locked(pl.dev, s);
    if (idx < 0) return BAGUA_ERR_UNSUPPORTED;
    // A launch captured into a graph keeps this slot's address: every replay draws
    // tickets and bumps `drained` without the host knowing, so the slot can never
    // be handed to another stream again (16 KiB stays with the graph).
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess) (void)hipGetLastError();
    if (cap != hipStreamCaptureStatusNone) d.state[idx].captured = true;
    pl.a.slot = d.slots + idx;
    const ResidentArgs& a = pl.a;
    switch (pl.cfg) {
#define BAGUA_RES_LAUNCH(I)                                                                                 \
    case I: {                                                                                               \
        constexpr ResidentCfg k = kResCfg[I];                                                               \
        launch(minmax_resident_encode_kernel<T, k.block, k.r, k.h, k.sb, k.ntm>, dim3(a.grid), dim3(k.block),     \
               (uint32_t)pl.lds, s, a);                                                                     \
        break;                                                                                              \
    }
        BAGUA_RES_LAUNCH(0)
        BAGUA_RES_LAUNCH(1)
        BAGUA_RES_LAUNCH(2)
        BAGUA_RES_LAUNCH(3)
        BAGUA_RES_LAUNCH(4)
        BAGUA_RES_LAUNCH(5)
        BAGUA_RES_LAUNCH(6)
        BAGUA_RES_LAUNCH(7)
        BAGUA_RES_LAUNCH(8)
        BAGUA_RES_LAUNCH(9)
        BAGUA_RES_LAUNCH(10)
        BAGUA_RES_LAUNCH(11)
        BAGUA_RES_LAUNCH(12)
        BAGUA_RES_LAUNCH(13)
#undef BAGUA_RES_LAUNCH
        default:
            return BAGUA_ERR_UNSUPPORTED;  // a configuration without a launch: never silently skip the encode
    }
    const int rc = check_launch();
    if (rc == BAGUA_OK) d.state[idx].launched += (uint64_t)a.grid;  // each workgroup drains once
    return rc;
}

// Drops the slot of stream `s` on every device once the stream's one-launch
// encodes have let go of it (wait_slot_drained).  Safe to call for streams that never ran
// one; the next launch on `s` takes a slot again.
int release_stream_slot(hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_res_mu);
    const StreamKey key = stream_key(s);
    int rc = BAGUA_OK;
    for (int dev = 0; dev < 64; ++dev) {
        ResidentDevice& d = g_res_dev[dev];
        if (!d.ok) continue;
        auto it = d.stream_slot.find(key);
        if (it == d.stream_slot.end()) continue;
        SlotState& st = d.state[it->second];
        if (st.captured) {  // a graph still holds it: unmap the stream, never reuse the slot
            d.stream_slot.erase(it);
            continue;
        }
        if (wait_slot_drained(dev, it->second, s) != BAGUA_OK) {
            rc = BAGUA_ERR_HIP;
            continue;  // faulted: keep the slot owned
        }
        st.used = false;
        st.last_use = 0;
        d.stream_slot.erase(it);
    }
    return rc;
}

// workgroups of stream `s`'s one-launch encodes that gave up waiting for their
// chunk's partials (measurement: contention with other streams' kernels).
// Synchronises `s`; *count = 0 when the stream never ran the one-launch encode.
int resident_give_ups(hipStream_t s, uint64_t* count) {
    std::lock_guard<std::mutex> lk(g_res_mu);
    *count = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || !g_res_dev[dev].ok) return BAGUA_OK;
    ResidentDevice& d = g_res_dev[dev];
    auto it = d.stream_slot.find(stream_key(s));
    if (it == d.stream_slot.end()) return BAGUA_OK;
    if (hipMemcpyAsync(d.probe_host, &d.slots[it->second].gave_up, sizeof(uint64_t), hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        g_last_hip_error = (int)hipGetLastError();
        return BAGUA_ERR_HIP;
    }
    *count = *d.probe_host;
    return BAGUA_OK;
}

int resident_slots_in_use(int dev) {
    std::lock_guard<std::mutex> lk(g_res_mu);
    if (dev < 0 || dev >= 64 || !g_res_dev[dev].ok) return 0;
    return (int)g_res_dev[dev].stream_slot.size();
}

template <typename T>
int resident_eligible(const void* input, int64_t in_num_elem, int64_t cs, int p, uint8_t* out, int64_t out_bytes,
                      int target, hipStream_t s) {
    return resident_plan<T>(input, in_num_elem, cs, p, out, out_bytes, target, s).ok ? 1 : 0;
}

template int resident_compress_impl<F32>(const void*, int64_t, int64_t, int, uint8_t*, int64_t, int, hipStream_t);
template int resident_compress_impl<F16>(const void*, int64_t, int64_t, int, uint8_t*, int64_t, int, hipStream_t);
template int resident_compress_impl<BF16>(const void*, int64_t, int64_t, int, uint8_t*, int64_t, int, hipStream_t);

}  // namespace bagua

extern "C" int bagua_minmax_u8_release_stream(bagua_stream_t stream) {
    {
        std::lock_guard<std::mutex> lk(bagua::g_res_mu);
        bagua::resident_off_streams().erase(static_cast<hipStream_t>(stream));
    }
    return bagua::release_stream_slot(static_cast<hipStream_t>(stream));
}

extern "C" int bagua_minmax_u8_set_stream_resident(bagua_stream_t stream, int allowed) {
    std::lock_guard<std::mutex> lk(bagua::g_res_mu);
    if (allowed) bagua::resident_off_streams().erase(static_cast<hipStream_t>(stream));
    else bagua::resident_off_streams().insert(static_cast<hipStream_t>(stream));
    return BAGUA_OK;
}

extern "C" int bagua_minmax_u8_resident_slots_in_use(int device_id) { return bagua::resident_slots_in_use(device_id); }

extern "C" int bagua_minmax_u8_resident_give_ups(bagua_stream_t stream, uint64_t* count) {
    if (!count) return BAGUA_ERR_INVALID_ARG;
    return bagua::resident_give_ups(static_cast<hipStream_t>(stream), count);
}

extern "C" int bagua_minmax_u8_resident_trace(void* device_buffer) {
    std::lock_guard<std::mutex> lk(bagua::g_res_mu);
    bagua::g_res_trace = static_cast<uint64_t*>(device_buffer);
    return BAGUA_OK;
}

extern "C" int bagua_minmax_u8_resident_path(int dtype, const void* input, int input_num_element, int chunk_size,
                                             int num_chunks, uint8_t* output, size_t output_bytes, int target_chunk,
                                             bagua_stream_t stream) {
    using namespace bagua;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (num_chunks <= 0 || chunk_size < 0 || target_chunk < -1 || target_chunk >= num_chunks || !input || !output)
        return 0;
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return resident_eligible<F32>(input, input_num_element, chunk_size, num_chunks, output,
                                          (int64_t)output_bytes, target_chunk, s);
        case BAGUA_DTYPE_F16:
            return resident_eligible<F16>(input, input_num_element, chunk_size, num_chunks, output,
                                          (int64_t)output_bytes, target_chunk, s);
        case BAGUA_DTYPE_BF16:
            return resident_eligible<BF16>(input, input_num_element, chunk_size, num_chunks, output,
                                           (int64_t)output_bytes, target_chunk, s);
    }
    return 0;
}

namespace bagua {

}  // namespace bagua
