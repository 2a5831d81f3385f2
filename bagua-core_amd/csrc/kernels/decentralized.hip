// decentralized.hip — the elementwise steps of the decentralized low-precision
// ring op (decentralized_low_precision_synchronous.rs:42-152) fused into two
// streaming kernels around the (unchanged) MinMax quantise pass.
//
// Reference sequence on one bucket (n elements of T), each step a full pass:
//   t += L*(1/3); t += R*(1/3); t += W*(-5/3)          :45-60  3 x addmul
//   compress(t, n_chunks = 1)                           :61-64  min/max + quantise
//   ... ring exchange of the compressed bytes ...
//   t = dq(from_left);  L += t                          :126-133
//   t = dq(from_right); R += t                          :134-141
//   t = dq(mine);       t += W;  W = t                  :142-151
// Bytes moved (bf16, N elements of 2 B): 18N + 5N + 31N = 54N.  Fused:
//   ring_mix   : the three addmuls in registers + the min/max partials of the
//                result (the quantise pass folds them as its own)        10N
//   quantise   : minmax_quantize_kernel, unchanged                        3N
//   ring_apply : the three dequantise+adds and the clone in one pass     17N
// Every intermediate is rounded to T exactly where the reference stores it
// (as_stored<T>), so all four tensors end bit-identical to the reference op.
// One rank (its own left and right peer) runs two passes instead, 24N: the mix's
// min/max only (8N read, nothing stored), then the mix recomputed, quantised and
// dequantised in registers and applied to all four tensors (8N + 8N), no payload
// (ring_one_rank_kernel, bagua_ring_one_rank_minmax).
#include "codec_common.hpp"
#include "launch_util.hpp"

#include <type_traits>

namespace bagua {

int minmax_partials_blocks(int64_t cs, int per_vec, int nact, size_t ws_bytes);  // minmax_u8.hip

// vectors per tensor per iteration, all loads issued before any is consumed
// (profiles/r01_ring_unroll_ab.jsonl, 2^27 bf16, interleaved runs on one box:
// apply 455-487 -> 406-436 us and the op 1.02-1.05 -> 0.97-1.01 ms from U = 1 to
// U = 4; the mix moves within noise)
constexpr int kMixUnroll = 4;

// ring_apply variants (tools/ring_apply_sweep.py; BAGUA_RING_APPLY_CFG selects one,
// read per call): vectors per tensor per batch, nt-store mask (bit 0 l, 1 r, 2 t,
// 3 w), nt loads of l / r / w, contiguous ranges per workgroup, grid cap
struct ApplyCfg {
    int u, sp;
    bool ntl, contig;
    int max_blocks;
};
constexpr ApplyCfg kApplyCfg[] = {
    {4, 0xF, false, false, 4096},  // 0: round 2 (nt stores, grid-strided)
    {4, 0x0, false, false, 4096},  // 1: default-policy stores
    {4, 0xC, false, false, 4096},  // 2: nt t / w, default l / r
    {4, 0x3, false, false, 4096},  // 3: default t / w, nt l / r
    {4, 0xF, true, false, 4096},   // 4: + nt loads
    {2, 0xF, false, false, 4096},  // 5: U = 2
    {4, 0xF, false, true, 4096},   // 6: contiguous ranges
    {4, 0x0, true, false, 4096},   // 7: nt loads, default stores
    {4, 0xF, false, true, 1024},   // 8: contiguous, 4 workgroups per CU
    {4, 0xF, false, false, 1024},  // 9: grid-strided, 1024 workgroups
    {4, 0xF, true, true, 4096},    // 10: contiguous + nt loads
    {2, 0xF, false, true, 4096},   // 11: contiguous, U = 2
    {4, 0xF, false, true, 2048},   // 12: contiguous, 2048 workgroups
    {4, 0xF, false, true, 8192},   // 13: contiguous, 8192 workgroups
    {2, 0xF, true, true, 8192},    // 14: contiguous, U = 2, nt loads, 8192 workgroups
    {8, 0xF, false, true, 4096},   // 15: contiguous, U = 8
    {2, 0xF, true, true, 16384},   // 16
    {2, 0xF, true, true, 32768},   // 17: one tile per workgroup
    {4, 0xF, true, true, 8192},    // 18
    {1, 0xF, true, true, 16384},   // 19
    {1, 0xF, true, true, 65536},   // 20: one tile per workgroup
    {2, 0xF, true, false, 8192},   // 21: grid-strided, U = 2, nt loads
    {2, 0xC, true, true, 8192},    // 22: as 14 with default-policy l / r stores
};
constexpr int kApplyNumCfg = (int)(sizeof(kApplyCfg) / sizeof(kApplyCfg[0]));
constexpr int kApplyDefaultCfg = 20;  // one 256-vector tile per workgroup, nt loads (profiles/r03_ring_apply_sweep3.jsonl)
static int apply_cfg() {
    const char* e = getenv("BAGUA_RING_APPLY_CFG");
    const int c = (e && *e) ? atoi(e) : kApplyDefaultCfg;
    return c >= 0 && c < kApplyNumCfg ? c : kApplyDefaultCfg;
}

// K:236-244 addmul as the elementwise kernels compute it (elementwise.hip)
template <typename T>
__device__ __forceinline__ float addmul(float x, float y, float f) {
    if constexpr (sizeof(typename T::storage) == 4) return __builtin_fmaf(y, f, x);
    else return as_stored<T>(x + as_stored<T>(y * f));
}

// addmul<T> already returns a value rounded to T (the 16-bit path ends in
// as_stored; f32 is stored as computed), and rounding is idempotent, so no
// further rounding is applied between the steps
template <typename T>
__device__ __forceinline__ float mix(float t, float l, float r, float w, float f13, float f53) {
    t = addmul<T>(t, l, f13);
    t = addmul<T>(t, r, f13);
    return addmul<T>(t, w, f53);
}

// STORE = false: the min/max partials of the mixed values only, t untouched (the
// one-rank op's first pass; its second pass recomputes the mix, ring_one_rank_kernel).
// TILES (without CONTIG): workgroups stride over whole U-vector tiles instead of
// single vectors (the U loads of a stream 4 KiB apart instead of a grid apart).
template <typename T, int U, bool CONTIG = false, bool NTS = false, bool STORE = true, bool TILES = false>
__global__ __launch_bounds__(kBlock) void ring_mix_kernel(typename T::storage* __restrict__ t,
                                                          const typename T::storage* __restrict__ l,
                                                          const typename T::storage* __restrict__ r,
                                                          const typename T::storage* __restrict__ w, int64_t n,
                                                          float f13, float f53, uint2* __restrict__ partials,
                                                          int64_t keep_from = INT64_MAX) {
    // vectors from keep_from on load with the default policy (they stay in the Infinity
    // Cache for the pass that re-reads them first; the rest non-temporally)
    constexpr int N = Vec<T>::N;
    uint32_t lo = min_space(T::init_max()), hi = max_space(-T::init_max());
    const int64_t nvec = n / N;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    // one vector of each of the four tensors
    auto body = [&](int64_t v, const uint4& rt, const uint4& rl, const uint4& rr, const uint4& rw) {
        float ft[N], fl[N], fr[N], fw[N];
        unpack16<T>(rt, ft);
        unpack16<T>(rl, fl);
        unpack16<T>(rr, fr);
        unpack16<T>(rw, fw);
#pragma unroll
        for (int i = 0; i < N; ++i) {
            ft[i] = mix<T>(ft[i], fl[i], fr[i], fw[i], f13, f53);
            const int32_t k = f2key(ft[i]);  // NaN wraps to a huge key in both spaces
            lo = min(lo, min_space_key(k));
            hi = min(hi, max_space_key(k));
        }
        // plain store: the quantise pass re-reads t next (NTS: non-temporal, A/B)
        if constexpr (!STORE) (void)v;
        else if constexpr (NTS) nt_store16(pack16<T>(ft), reinterpret_cast<uint4*>(t) + v);
        else reinterpret_cast<uint4*>(t)[v] = pack16<T>(ft);
    };
    const uint4* t4 = reinterpret_cast<const uint4*>(t);
    const uint4* l4 = reinterpret_cast<const uint4*>(l);
    const uint4* r4 = reinterpret_cast<const uint4*>(r);
    const uint4* w4 = reinterpret_cast<const uint4*>(w);
    auto ld = [&](const uint4* p, int64_t u) { return u >= keep_from ? p[u] : nt_load16(p + u); };
    // U vectors per tensor per iteration (4U x 16 B in flight per lane), all loads
    // issued before any is consumed; the last partial iteration goes one by one.
    // All four streams load non-temporally: default-policy t/w loads (or l/r) were
    // slower (profiles/r01_ring_mix_policy_ab.jsonl)
    auto batch = [&](int64_t v, int64_t kstep) {
        uint4 rt[U], rl[U], rr[U], rw[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            rt[k] = ld(t4, v + k * kstep);
            rl[k] = ld(l4, v + k * kstep);
            rr[k] = ld(r4, v + k * kstep);
            rw[k] = ld(w4, v + k * kstep);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) body(v + k * kstep, rt[k], rl[k], rr[k], rw[k]);
    };
    if constexpr (CONTIG) {  // one contiguous range per workgroup
        const int64_t tile = (int64_t)U * kBlock;
        const int64_t per = ((nvec + gridDim.x - 1) / gridDim.x + tile - 1) / tile * tile;
        const int64_t v0 = (int64_t)blockIdx.x * per;  // (not lo / hi: those are the min/max keys)
        const int64_t v1 = v0 + per < nvec ? v0 + per : nvec;
        int64_t base = v0;
        for (; base + tile <= v1; base += tile) batch(base + threadIdx.x, kBlock);
        for (int64_t u = base + threadIdx.x; u < v1; u += kBlock)
            body(u, ld(t4, u), ld(l4, u), ld(r4, u), ld(w4, u));
    } else if constexpr (TILES) {
        const int64_t tile = (int64_t)U * kBlock;
        for (int64_t base = (int64_t)blockIdx.x * tile; base < nvec; base += (int64_t)gridDim.x * tile) {
            if (base + tile <= nvec) {
                batch(base + threadIdx.x, kBlock);
            } else {
                for (int64_t u = base + threadIdx.x; u < nvec; u += kBlock)
                    body(u, ld(t4, u), ld(l4, u), ld(r4, u), ld(w4, u));
            }
        }
    } else {
        for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < nvec; v += stride * U) {
            if (v + (U - 1) * stride < nvec) {
                batch(v, stride);
            } else {
                for (int64_t u = v; u < nvec; u += stride)
                    body(u, ld(t4, u), ld(l4, u), ld(r4, u), ld(w4, u));
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < n - nvec * N) {  // ragged tail
        const int64_t j = nvec * N + threadIdx.x;
        const float x = mix<T>(T::to_f(t[j]), T::to_f(l[j]), T::to_f(r[j]), T::to_f(w[j]), f13, f53);
        if constexpr (STORE) t[j] = T::from_f(x);
        const int32_t k = f2key(x);
        lo = min(lo, min_space_key(k));
        hi = min(hi, max_space_key(k));
    }
    lo = wave_umin(lo);
    hi = wave_umin(hi);
    __shared__ uint32_t red[2][kWavesPerBlock];
    const int wv = threadIdx.x / kWave;
    if (lane_id() == 0) { red[0][wv] = lo; red[1][wv] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 1; i < kWavesPerBlock; ++i) { lo = min(lo, red[0][i]); hi = min(hi, red[1][i]); }
        partials[blockIdx.x] = make_uint2(lo, hi);
    }
}

// 16-B stores of the apply pass, per output: non-temporal or default policy
template <bool NT>
__device__ __forceinline__ void store16(const uint4& v, uint4* p) {
    if constexpr (NT) nt_store16(v, p);
    else *p = v;
}
template <bool NT>
__device__ __forceinline__ uint4 load16(const uint4* p) {
    if constexpr (NT) return nt_load16(p);
    else return *p;
}

// SP: non-temporal store mask (bit 0 l, 1 r, 2 t, 3 w); NTL: non-temporal loads of
// l / r / w; CONTIG: each workgroup sweeps one contiguous range instead of the
// grid-strided loop (ring_apply variants, BAGUA_RING_APPLY_CFG, tools/ring_apply_sweep.py)
template <typename T, int U, int SP, bool NTL, bool CONTIG>
__global__ __launch_bounds__(kBlock) void ring_apply_kernel(const uint8_t* __restrict__ mine,
                                                            const uint8_t* __restrict__ from_left,
                                                            const uint8_t* __restrict__ from_right,
                                                            typename T::storage* __restrict__ t,
                                                            typename T::storage* __restrict__ w,
                                                            typename T::storage* __restrict__ l,
                                                            typename T::storage* __restrict__ r, int64_t n,
                                                            int64_t e0, int64_t e1) {
    // elements [e0, e1) (e0 a multiple of N; e1 too unless it is n)
    constexpr int N = Vec<T>::N;
    __shared__ float tm[256], tl[256], tr[256];
    const uint8_t* pm = mine + 32;
    const uint8_t* pl = from_left + 32;
    const uint8_t* pr = from_right + 32;
    const int64_t nvec = n / N, v1 = e1 / N;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    auto body = [&](int64_t v, const uint32_t (&bm)[N], const uint32_t (&bl)[N], const uint32_t (&br)[N],
                    const uint4& rl, const uint4& rr, const uint4& rw) {
        float fl[N], fr[N], fw[N], ft[N];
        unpack16<T>(rl, fl);
        unpack16<T>(rr, fr);
        unpack16<T>(rw, fw);
#pragma unroll
        for (int i = 0; i < N; ++i) {
            fl[i] = fl[i] + tl[bl[i]];   // L += dq(from_left)
            fr[i] = fr[i] + tr[br[i]];   // R += dq(from_right)
            ft[i] = tm[bm[i]] + fw[i];   // t = dq(mine) + W
        }
        const uint4 ot = pack16<T>(ft);
        store16<(SP & 1) != 0>(pack16<T>(fl), reinterpret_cast<uint4*>(l) + v);
        store16<(SP & 2) != 0>(pack16<T>(fr), reinterpret_cast<uint4*>(r) + v);
        store16<(SP & 4) != 0>(ot, reinterpret_cast<uint4*>(t) + v);
        store16<(SP & 8) != 0>(ot, reinterpret_cast<uint4*>(w) + v);  // W = t (clone)
    };
    const uint4* l4 = reinterpret_cast<const uint4*>(l);
    const uint4* r4 = reinterpret_cast<const uint4*>(r);
    const uint4* w4 = reinterpret_cast<const uint4*>(w);
    auto one = [&](int64_t v) {
        uint32_t bm[N], bl[N], br[N];
        load_bytes<T>(pm + v * N, bm);
        load_bytes<T>(pl + v * N, bl);
        load_bytes<T>(pr + v * N, br);
        body(v, bm, bl, br, load16<NTL>(l4 + v), load16<NTL>(r4 + v), load16<NTL>(w4 + v));
    };
    // U vectors per tensor per iteration (k-th at offset k * kstep), all loads
    // issued before any is consumed
    struct Regs {
        uint32_t bm[U][N], bl[U][N], br[U][N];
        uint4 rl[U], rr[U], rw[U];
    };
    auto load_batch = [&](int64_t v, int64_t kstep, Regs& g) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int64_t u = v + k * kstep;
            load_bytes<T>(pm + u * N, g.bm[k]);
            load_bytes<T>(pl + u * N, g.bl[k]);
            load_bytes<T>(pr + u * N, g.br[k]);
            g.rl[k] = load16<NTL>(l4 + u);
            g.rr[k] = load16<NTL>(r4 + u);
            g.rw[k] = load16<NTL>(w4 + u);
        }
    };
    auto use_batch = [&](int64_t v, int64_t kstep, const Regs& g) {
#pragma unroll
        for (int k = 0; k < U; ++k) body(v + k * kstep, g.bm[k], g.bl[k], g.br[k], g.rl[k], g.rr[k], g.rw[k]);
    };
    auto batch = [&](int64_t v, int64_t kstep) {
        Regs g;
        load_batch(v, kstep, g);
        use_batch(v, kstep, g);
    };
    // per-byte dequantised values of the three buffers (codec_common.hpp "dequantisation
    // tables"), built after the first batch's loads are out: with one tile per workgroup
    // (the default shape) the header reads and the barrier were otherwise the whole
    // prologue of every workgroup, with no HBM request in flight
    auto tables = [&]() {
        const QParams qm = read_header<T>(mine), ql = read_header<T>(from_left), qr = read_header<T>(from_right);
        static_assert(kBlock == 256, "one table entry per thread");
        tm[threadIdx.x] = as_stored<T>(dequant(threadIdx.x, qm));
        tl[threadIdx.x] = as_stored<T>(dequant(threadIdx.x, ql));
        tr[threadIdx.x] = as_stored<T>(dequant(threadIdx.x, qr));
        __syncthreads();
    };
    if constexpr (CONTIG) {
        const int64_t tile = (int64_t)U * kBlock;
        const int64_t vb = e0 / N, nv = v1 - vb;
        const int64_t per = ((nv + gridDim.x - 1) / gridDim.x + tile - 1) / tile * tile;
        const int64_t lo = vb + (int64_t)blockIdx.x * per;
        const int64_t hi = lo + per < v1 ? lo + per : v1;
        int64_t base = lo;
        if (base + tile <= hi) {
            Regs g;
            load_batch(base + threadIdx.x, kBlock, g);
            tables();
            use_batch(base + threadIdx.x, kBlock, g);
            base += tile;
        } else {
            tables();
        }
        for (; base + tile <= hi; base += tile) batch(base + threadIdx.x, kBlock);
        for (int64_t u = base + threadIdx.x; u < hi; u += kBlock) one(u);
    } else {
        tables();
        for (int64_t v = e0 / N + (int64_t)blockIdx.x * kBlock + threadIdx.x; v < v1; v += stride * U) {
            if (v + (U - 1) * stride < v1) {
                batch(v, stride);
            } else {
                for (int64_t u = v; u < v1; u += stride) one(u);
            }
        }
    }
    if (e1 == n && blockIdx.x == 0 && threadIdx.x < n - nvec * N) {
        const int64_t j = nvec * N + threadIdx.x;
        l[j] = T::from_f(T::to_f(l[j]) + tl[pl[j]]);
        r[j] = T::from_f(T::to_f(r[j]) + tr[pr[j]]);
        const typename T::storage o = T::from_f(tm[pm[j]] + T::to_f(w[j]));
        t[j] = o;
        w[j] = o;
    }
}

// One rank (p = 1) is its own left and right peer: what it receives from both is its
// own compressed bytes, so :126-151 become, per element, with d = dq(q(t_mixed)) under
// the bucket's one header (n_chunks = 1),
//   L += d;  R += d;  t = d + W;  W = t.
// This pass folds the mix pass's min/max partials into that header (as the quantise
// pass does), quantises and dequantises each mixed element in registers, and writes the
// four tensors: the payload is neither written nor read back (16N bytes for bf16
// instead of the quantise pass's 3N and the apply pass's 17N).  Every expression is the
// one those two passes evaluate (the quantise pass's quant_pack4 / quant, the apply
// pass's as_stored dequantisation table under the header as stored in T), so the four
// tensors are bit-identical to the two-pass sequence (test_ring_one_rank_matches_sequence).
// CONTIG: contiguous ranges of U-vector batches per workgroup (otherwise grid-strided).
// MIX: t, l, r, w are the op's inputs (the first pass only folded the mixed values'
// min/max, ring_mix_kernel<STORE = false>) and the mix is recomputed here, the same
// three rounded addmuls, instead of being stored by the first pass and read back (2N
// + 2N bytes); otherwise t holds the mixed values.
template <typename T, int U, bool CONTIG, bool MIX>
__global__ __launch_bounds__(kBlock) void ring_one_rank_kernel(typename T::storage* __restrict__ t,
                                                               typename T::storage* __restrict__ w,
                                                               typename T::storage* __restrict__ l,
                                                               typename T::storage* __restrict__ r, int64_t n,
                                                               const uint2* __restrict__ partials, int npartials,
                                                               float f13, float f53) {
    constexpr int N = Vec<T>::N;
    static_assert(N % 4 == 0, "quant_pack4 packs four elements");
    __shared__ float tab[256];
    __shared__ uint32_t red[2][kWavesPerBlock];
    const int64_t nvec = n / N;
    uint4* t4 = reinterpret_cast<uint4*>(t);
    uint4* w4 = reinterpret_cast<uint4*>(w);
    uint4* l4 = reinterpret_cast<uint4*>(l);
    uint4* r4 = reinterpret_cast<uint4*>(r);
    QParams q;
    auto body = [&](int64_t v, const uint4& rt, const uint4& rw, const uint4& rl, const uint4& rr) {
        float ft[N], fw[N], fl[N], fr[N];
        unpack16<T>(rt, ft);
        unpack16<T>(rw, fw);
        unpack16<T>(rl, fl);
        unpack16<T>(rr, fr);
        if constexpr (MIX) {
#pragma unroll
            for (int i = 0; i < N; ++i) ft[i] = mix<T>(ft[i], fl[i], fr[i], fw[i], f13, f53);
        }
#pragma unroll
        for (int i = 0; i < N; i += 4) {
            const uint32_t b = quant_pack4(ft[i], ft[i + 1], ft[i + 2], ft[i + 3], q);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float d = tab[(b >> (8 * e)) & 0xff];
                fl[i + e] = fl[i + e] + d;   // L += dq(from_left)
                fr[i + e] = fr[i + e] + d;   // R += dq(from_right)
                ft[i + e] = d + fw[i + e];   // t = dq(mine) + W
            }
        }
        const uint4 ot = pack16<T>(ft);
        nt_store16(pack16<T>(fl), l4 + v);
        nt_store16(pack16<T>(fr), r4 + v);
        nt_store16(ot, t4 + v);
        nt_store16(ot, w4 + v);  // W = t (clone)
    };
    struct Regs {
        uint4 rt[U], rw[U], rl[U], rr[U];
    };
    auto load_batch = [&](int64_t v, int64_t kstep, Regs& g) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int64_t u = v + k * kstep;
            g.rt[k] = nt_load16(t4 + u);
            g.rw[k] = nt_load16(w4 + u);
            g.rl[k] = nt_load16(l4 + u);
            g.rr[k] = nt_load16(r4 + u);
        }
    };
    auto use_batch = [&](int64_t v, int64_t kstep, const Regs& g) {
#pragma unroll
        for (int k = 0; k < U; ++k) body(v + k * kstep, g.rt[k], g.rw[k], g.rl[k], g.rr[k]);
    };
    auto one = [&](int64_t u) { body(u, nt_load16(t4 + u), nt_load16(w4 + u), nt_load16(l4 + u), nt_load16(r4 + u)); };
    // the header from the mix pass's partials (minmax_quantize_kernel's fold) and the
    // dequantisation table of the header as the apply pass reads it back (T values);
    // run after the first batch's loads are out
    auto prologue = [&]() {
        uint32_t lo = 0xffffffffu, hi = 0xffffffffu;
        for (int i = threadIdx.x; i < npartials; i += kBlock) {
            const uint2 p = partials[i];
            lo = min(lo, p.x);
            hi = min(hi, p.y);
        }
        lo = wave_umin(lo);
        hi = wave_umin(hi);
        const int wv = threadIdx.x / kWave;
        if (lane_id() == 0) { red[0][wv] = lo; red[1][wv] = hi; }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kWavesPerBlock; ++i) { lo = min(lo, red[0][i]); hi = min(hi, red[1][i]); }
        const float mn = from_min_space(lo), mx = from_max_space(hi);
        q = make_qparams(mn, mx);
        const QParams qh = make_qparams(T::to_f(T::from_f(mn)), T::to_f(T::from_f(mx)));
        static_assert(kBlock == 256, "one table entry per thread");
        tab[threadIdx.x] = as_stored<T>(dequant(threadIdx.x, qh));
        __syncthreads();
    };
    const int64_t tile = (int64_t)U * kBlock;
    if constexpr (CONTIG) {
        // MIX: backwards (the first pass read the tail last; it is in the Infinity Cache)
        const int64_t bidx = MIX ? (int64_t)gridDim.x - 1 - blockIdx.x : (int64_t)blockIdx.x;
        const int64_t per = ((nvec + gridDim.x - 1) / gridDim.x + tile - 1) / tile * tile;
        const int64_t lo = bidx * per;
        const int64_t hi = lo + per < nvec ? lo + per : nvec;
        int64_t base = lo;
        if (base + tile <= hi) {
            Regs g;
            load_batch(base + threadIdx.x, kBlock, g);
            prologue();
            use_batch(base + threadIdx.x, kBlock, g);
            base += tile;
        } else {
            prologue();
        }
        for (; base + tile <= hi; base += tile) {
            Regs g;
            load_batch(base + threadIdx.x, kBlock, g);
            use_batch(base + threadIdx.x, kBlock, g);
        }
        for (int64_t u = base + threadIdx.x; u < hi; u += kBlock) one(u);
    } else {
        // (whether a lane's first batch is whole differs between lanes here, so the
        // prologue and its barriers come first, uniformly)
        prologue();
        const int64_t stride = (int64_t)gridDim.x * kBlock;
        for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < nvec; v += stride * U) {
            if (v + (U - 1) * stride < nvec) {
                Regs g;
                load_batch(v, stride, g);
                use_batch(v, stride, g);
            } else {
                for (int64_t u = v; u < nvec; u += stride) one(u);
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < n - nvec * N) {  // ragged tail
        const int64_t j = nvec * N + threadIdx.x;
        const float x = MIX ? mix<T>(T::to_f(t[j]), T::to_f(l[j]), T::to_f(r[j]), T::to_f(w[j]), f13, f53)
                            : T::to_f(t[j]);
        const float d = tab[quant(x, q)];
        l[j] = T::from_f(T::to_f(l[j]) + d);
        r[j] = T::from_f(T::to_f(r[j]) + d);
        const typename T::storage o = T::from_f(d + T::to_f(w[j]));
        t[j] = o;
        w[j] = o;
    }
}

static float round_to_t(int dtype, float f) {
    if (dtype == BAGUA_DTYPE_F16) return (float)(_Float16)f;
    if (dtype == BAGUA_DTYPE_BF16) {
        uint32_t u = __builtin_bit_cast(uint32_t, f);
        if ((u & 0x7fffffffu) > 0x7f800000u) return f;
        u += 0x7fffu + ((u >> 16) & 1u);
        return __builtin_bit_cast(float, u & 0xffff0000u);
    }
    return f;
}

static bool aligned16(const void* p) { return (uintptr_t)p % 16 == 0; }

template <typename T>
static int mix_impl(void* t, const void* l, const void* r, const void* w, int n, void* ws, size_t ws_bytes,
                    float f13, float f53, hipStream_t s) {
    using S = typename T::storage;
    if (!t || !l || !r || !w || n < 0) return BAGUA_ERR_INVALID_ARG;
    if (!aligned16(t) || !aligned16(l) || !aligned16(r) || !aligned16(w)) return BAGUA_ERR_UNSUPPORTED;
    const int nblk = ws ? minmax_partials_blocks(n, Vec<T>::N, 1, ws_bytes) : 0;
    if (nblk < 1) return BAGUA_ERR_WORKSPACE;
    // A/B knobs (tools/kernel_ab.py --variants): contiguous ranges per workgroup, a
    // non-temporal store of the mixed t.  (The grid stays nblk: the quantise pass folds
    // exactly that many partials.)
    const bool contig = tune_int("BAGUA_RING_MIX_CONTIG", 0) == 1;
    const bool nts = tune_int("BAGUA_RING_MIX_NTS", 0) == 1;
    // workgroups stride over whole U-vector tiles (BAGUA_RING_MIX_TILES=0: over single
    // vectors, the round-1..4 shape): 2^27 bf16, one box, 244 -> 219 us, the p = 1 op
    // sequence 658 -> 631 us (profiles/r05_one_rank_ring_mix_tiles_trace.csv)
    const bool tiles = tune_int("BAGUA_RING_MIX_TILES", 1) == 1;
    const int grid = nblk;
    auto go = [&](auto kern) {
        launch(kern, dim3(grid), dim3(kBlock), 0, s, static_cast<S*>(t), static_cast<const S*>(l),
               static_cast<const S*>(r), static_cast<const S*>(w), (int64_t)n, f13, f53, static_cast<uint2*>(ws),
               (int64_t)INT64_MAX);
    };
    // (U = 2 and 8 vectors per tensor per batch measured slower than 4: mix 233 / 238 vs
    // 228 us, profiles/r05_ring_mix_unroll_ab.json; tile-strided 228 / 222 vs 221 us,
    // r05_ring_mix_tile_u_trace.csv)
    if (tiles && !contig && nts) go(ring_mix_kernel<T, kMixUnroll, false, true, true, true>);
    else if (tiles && !contig) go(ring_mix_kernel<T, kMixUnroll, false, false, true, true>);
    else if (contig && nts) go(ring_mix_kernel<T, kMixUnroll, true, true>);
    else if (contig) go(ring_mix_kernel<T, kMixUnroll, true, false>);
    else if (nts) go(ring_mix_kernel<T, kMixUnroll, false, true>);
    else go(ring_mix_kernel<T, kMixUnroll, false, false>);
    return check_launch();
}

// ring_one_rank_kernel shapes (BAGUA_RING_ONE_RANK_CFG, A/B): vectors per tensor per
// batch, contiguous ranges, workgroups (cap)
struct OneRankCfg {
    int u;
    bool contig;
    int max_blocks;
};
constexpr OneRankCfg kOneRankCfg[] = {
    {1, true, 65536},  // 0: one 256-vector tile per workgroup (the apply pass's shape)
    {2, true, 8192},   // 1
    {1, true, 16384},  // 2
    {4, false, 4096},  // 3: grid-strided
    {2, true, 32768},  // 4
    {2, true, 16384},  // 5
    {4, true, 16384},  // 6
    {4, true, 8192},   // 7
    {8, true, 8192},   // 8
};
constexpr int kOneRankNumCfg = (int)(sizeof(kOneRankCfg) / sizeof(kOneRankCfg[0]));

template <typename T>
static int one_rank_impl(void* t, void* w, void* l, void* r, int n, void* ws, size_t ws_bytes, float f13, float f53,
                         hipStream_t s) {
    using S = typename T::storage;
    if (!t || !w || !l || !r || n < 0) return BAGUA_ERR_INVALID_ARG;
    if (!aligned16(t) || !aligned16(w) || !aligned16(l) || !aligned16(r)) return BAGUA_ERR_UNSUPPORTED;
    // the mix pass (its partials count is what the fold below reads)
    int nblk = ws ? minmax_partials_blocks(n, Vec<T>::N, 1, ws_bytes) : 0;
    if (nblk < 1) return BAGUA_ERR_WORKSPACE;
    // BAGUA_RING_ONE_RANK_RECOMPUTE=0: the first pass stores the mixed t (A/B)
    const bool recompute = tune_int("BAGUA_RING_ONE_RANK_RECOMPUTE", 1) != 0;
    // first-pass grid (A/B; both passes are here, so any count the workspace holds): 512 /
    // 768 / 2048 workgroups measured against the default 1024, within noise except 2048,
    // whose 2048 partials every second-pass workgroup folds (pass 2 352 -> 382 us)
    if (recompute) {
        const int64_t want = tune_int("BAGUA_RING_ONE_RANK_MIX_BLOCKS", 0);
        const int64_t cap = (int64_t)(ws_bytes / sizeof(uint2));
        if (want > 0) nblk = (int)(want < cap ? want : cap);
    }
    if (recompute) {
        // BAGUA_RING_ONE_RANK_KEEP_MIB (A/B, default 0): the last MiB of the four inputs,
        // read last here, load with the default policy to stay in the 256 MiB Infinity
        // Cache for the second pass, which sweeps backwards and reads them first
        const int64_t keep = (int64_t)tune_int("BAGUA_RING_ONE_RANK_KEEP_MIB", 0) << 20;
        const int64_t nvec = (int64_t)n / Vec<T>::N;
        int64_t keep_from = nvec - (keep > 0 ? keep / 4 / 16 : 0);
        if (keep <= 0) keep_from = INT64_MAX;
        else if (keep_from < 0) keep_from = 0;
        auto go1 = [&](auto kern) {
            launch(kern, dim3(nblk), dim3(kBlock), 0, s, static_cast<S*>(t), static_cast<const S*>(l),
                   static_cast<const S*>(r), static_cast<const S*>(w), (int64_t)n, f13, f53, static_cast<uint2*>(ws),
                   keep_from);
        };
        // first-pass shapes (BAGUA_RING_ONE_RANK_MIX_CFG, A/B; 2^27 bf16, one box, rocprof
        // kernel trace, profiles/r05_one_rank_ring_shapes_trace.csv): 0 vector-strided U = 4, 208 us;
        // 1 tile-strided U = 4, 184 us (default); 2 tile-strided U = 8, 190 us; 3
        // contiguous ranges, 206 us; 4 tile-strided U = 2, 188 us
        switch (tune_int("BAGUA_RING_ONE_RANK_MIX_CFG", 1)) {
            case 0: go1(ring_mix_kernel<T, kMixUnroll, false, false, false>); break;
            case 2: go1(ring_mix_kernel<T, 8, false, false, false, true>); break;
            case 3: go1(ring_mix_kernel<T, 4, true, false, false>); break;
            case 4: go1(ring_mix_kernel<T, 2, false, false, false, true>); break;
            default: go1(ring_mix_kernel<T, 4, false, false, false, true>); break;
        }
        const int rc = check_launch();
        if (rc != BAGUA_OK) return rc;
    } else {
        const int rc = mix_impl<T>(t, l, r, w, n, ws, ws_bytes, f13, f53, s);
        if (rc != BAGUA_OK) return rc;
    }
    int ci = tune_int("BAGUA_RING_ONE_RANK_CFG", 0);
    if (ci < 0 || ci >= kOneRankNumCfg) ci = 0;
    const OneRankCfg& c = kOneRankCfg[ci];
    int64_t blocks = ((int64_t)n / Vec<T>::N + (int64_t)c.u * kBlock - 1) / ((int64_t)c.u * kBlock);
    if (blocks > c.max_blocks) blocks = c.max_blocks;
    if (blocks < 1) blocks = 1;
    auto go = [&](auto kern) {
        launch(kern, dim3((unsigned)blocks), dim3(kBlock), 0, s, static_cast<S*>(t), static_cast<S*>(w),
               static_cast<S*>(l), static_cast<S*>(r), (int64_t)n, static_cast<const uint2*>(ws), nblk, f13, f53);
    };
    auto pick = [&](auto mixc) {
        constexpr bool M = decltype(mixc)::value;
        if (!c.contig) go(ring_one_rank_kernel<T, 4, false, M>);
        else if (c.u == 2) go(ring_one_rank_kernel<T, 2, true, M>);
        else if (c.u == 4) go(ring_one_rank_kernel<T, 4, true, M>);
        else if (c.u == 8) go(ring_one_rank_kernel<T, 8, true, M>);
        else go(ring_one_rank_kernel<T, 1, true, M>);
    };
    if (recompute) pick(std::true_type{});
    else pick(std::false_type{});
    return check_launch();
}

template <typename T>
static int apply_impl(const uint8_t* mine, const uint8_t* from_left, const uint8_t* from_right, size_t comp_bytes,
                      int n, void* t, void* w, void* l, void* r, hipStream_t s, int e0 = 0, int e1 = -1) {
    using S = typename T::storage;
    constexpr int N = Vec<T>::N;
    if (e1 < 0) e1 = n;
    if (!mine || !from_left || !from_right || !t || !w || !l || !r || n < 0) return BAGUA_ERR_INVALID_ARG;
    if (e0 < 0 || e1 < e0 || e1 > n || e0 % N || (e1 != n && e1 % N)) return BAGUA_ERR_INVALID_ARG;
    if (e1 == e0) return BAGUA_OK;
    if (comp_bytes < (size_t)n + 32) return BAGUA_ERR_INVALID_ARG;
    if (!aligned16(t) || !aligned16(w) || !aligned16(l) || !aligned16(r)) return BAGUA_ERR_UNSUPPORTED;
    for (const uint8_t* p : {mine, from_left, from_right})
        if ((uintptr_t)(p + 32) % N) return BAGUA_ERR_UNSUPPORTED;
    int64_t blocks = ((int64_t)(e1 - e0) / N + kBlock - 1) / kBlock;
    const ApplyCfg& c = kApplyCfg[apply_cfg()];
    if (blocks > c.max_blocks) blocks = c.max_blocks;
    if (blocks < 1) blocks = 1;
    switch (apply_cfg()) {
#define BAGUA_APPLY_LAUNCH(I)                                                                                      \
    case I:                                                                                                        \
        launch(ring_apply_kernel<T, kApplyCfg[I].u, kApplyCfg[I].sp, kApplyCfg[I].ntl, kApplyCfg[I].contig>,       \
               dim3(blocks), dim3(kBlock), 0, s, mine, from_left, from_right, static_cast<S*>(t), static_cast<S*>(w), \
               static_cast<S*>(l), static_cast<S*>(r), (int64_t)n, (int64_t)e0, (int64_t)e1);                      \
        break;
        BAGUA_APPLY_LAUNCH(0)
        BAGUA_APPLY_LAUNCH(1)
        BAGUA_APPLY_LAUNCH(2)
        BAGUA_APPLY_LAUNCH(3)
        BAGUA_APPLY_LAUNCH(4)
        BAGUA_APPLY_LAUNCH(5)
        BAGUA_APPLY_LAUNCH(6)
        BAGUA_APPLY_LAUNCH(7)
        BAGUA_APPLY_LAUNCH(8)
        BAGUA_APPLY_LAUNCH(9)
        BAGUA_APPLY_LAUNCH(10)
        BAGUA_APPLY_LAUNCH(11)
        BAGUA_APPLY_LAUNCH(12)
        BAGUA_APPLY_LAUNCH(13)
        BAGUA_APPLY_LAUNCH(14)
        BAGUA_APPLY_LAUNCH(15)
        BAGUA_APPLY_LAUNCH(16)
        BAGUA_APPLY_LAUNCH(17)
        BAGUA_APPLY_LAUNCH(18)
        BAGUA_APPLY_LAUNCH(19)
        BAGUA_APPLY_LAUNCH(20)
        BAGUA_APPLY_LAUNCH(21)
        BAGUA_APPLY_LAUNCH(22)
#undef BAGUA_APPLY_LAUNCH
        default:
            return BAGUA_ERR_UNSUPPORTED;
    }
    return check_launch();
}

}  // namespace bagua

using namespace bagua;

extern "C" {

int bagua_ring_mix_minmax(int dtype, void* tensor, const void* left, const void* right, const void* weight,
                          int num_elem, void* workspace, size_t workspace_bytes, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    // :45-60 factors are f64 literals cast to f32, then to T by the 16-bit kernels (K:600)
    const float f13 = round_to_t(dtype, (float)(1.0 / 3.0)), f53 = round_to_t(dtype, (float)(-5.0 / 3.0));
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return mix_impl<F32>(tensor, left, right, weight, num_elem, workspace, workspace_bytes, f13, f53, s);
        case BAGUA_DTYPE_F16:
            return mix_impl<F16>(tensor, left, right, weight, num_elem, workspace, workspace_bytes, f13, f53, s);
        case BAGUA_DTYPE_BF16:
            return mix_impl<BF16>(tensor, left, right, weight, num_elem, workspace, workspace_bytes, f13, f53, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_ring_one_rank_minmax(int dtype, void* tensor, void* weight, void* left, void* right, int num_elem,
                               void* workspace, size_t workspace_bytes, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const float f13 = round_to_t(dtype, (float)(1.0 / 3.0)), f53 = round_to_t(dtype, (float)(-5.0 / 3.0));
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return one_rank_impl<F32>(tensor, weight, left, right, num_elem, workspace, workspace_bytes, f13, f53, s);
        case BAGUA_DTYPE_F16:
            return one_rank_impl<F16>(tensor, weight, left, right, num_elem, workspace, workspace_bytes, f13, f53, s);
        case BAGUA_DTYPE_BF16:
            return one_rank_impl<BF16>(tensor, weight, left, right, num_elem, workspace, workspace_bytes, f13, f53,
                                       s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_ring_apply_minmax(int dtype, const uint8_t* mine, const uint8_t* from_left, const uint8_t* from_right,
                            size_t compressed_bytes, int num_elem, void* tensor, void* weight, void* left,
                            void* right, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return apply_impl<F32>(mine, from_left, from_right, compressed_bytes, num_elem, tensor, weight, left,
                                   right, s);
        case BAGUA_DTYPE_F16:
            return apply_impl<F16>(mine, from_left, from_right, compressed_bytes, num_elem, tensor, weight, left,
                                   right, s);
        case BAGUA_DTYPE_BF16:
            return apply_impl<BF16>(mine, from_left, from_right, compressed_bytes, num_elem, tensor, weight, left,
                                    right, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

int bagua_ring_apply_minmax_range(int dtype, const uint8_t* mine, const uint8_t* from_left, const uint8_t* from_right,
                                  size_t compressed_bytes, int num_elem, int elem_begin, int elem_end, void* tensor,
                                  void* weight, void* left, void* right, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
        case BAGUA_DTYPE_F32:
            return apply_impl<F32>(mine, from_left, from_right, compressed_bytes, num_elem, tensor, weight, left,
                                   right, s, elem_begin, elem_end);
        case BAGUA_DTYPE_F16:
            return apply_impl<F16>(mine, from_left, from_right, compressed_bytes, num_elem, tensor, weight, left,
                                   right, s, elem_begin, elem_end);
        case BAGUA_DTYPE_BF16:
            return apply_impl<BF16>(mine, from_left, from_right, compressed_bytes, num_elem, tensor, weight, left,
                                    right, s, elem_begin, elem_end);
    }
    return BAGUA_ERR_UNSUPPORTED;
}

}  // extern "C"
