/*
 * bagua_oracle.c — CPU restatement of the bagua-core gradient-codec hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see bagua_oracle.h).  Built with
 * -ffp-contract=off and no fast-math so every float operation below is one
 * IEEE-754 binary32 operation with round-to-nearest-even, exactly as the
 * reference CUDA kernels evaluate them (nvcc defaults: -ftz=false,
 * -prec-div=true; no contraction site exists in the codec expressions).
 *
 * Citations: K = bagua-core-internal/kernels/bagua_kernels.cu,
 * DT = bagua-core-internal/src/datatypes/mod.rs, CUB = .../third_party/cub-1.8.0/cub.
 */
#include "bagua_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

int orc_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* the OpenMP team size of later calls (the CPU baseline: the host cores it may use) */
int orc_set_num_threads(int n) {
#ifdef _OPENMP
    if (n >= 1) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

/* ------------------------------------------------------------------------ */
/* scalar helpers                                                           */
/* ------------------------------------------------------------------------ */
static inline float u32f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t fu32(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

float orc_half_to_float(uint16_t h) {
    uint32_t sign = (uint32_t)(h >> 15) << 31;
    uint32_t exp = (h >> 10) & 0x1f, man = h & 0x3ff;
    if (exp == 0) {
        float f = ldexpf((float)man, -24); /* exact: man < 2^10 */
        return sign ? -f : f;
    }
    if (exp == 31) return u32f(sign | 0x7f800000u | (man << 13));
    return u32f(sign | ((exp + 112u) << 23) | (man << 13));
}

/* round-to-nearest-even float -> IEEE half (what __float2half does) */
uint16_t orc_float_to_half(float f) {
    uint32_t u = fu32(f);
    uint16_t sign = (uint16_t)((u >> 16) & 0x8000);
    uint32_t a = u & 0x7fffffffu;
    if (a > 0x7f800000u) return (uint16_t)(sign | 0x7e00 | ((a >> 13) & 0x3ff)); /* NaN */
    if (a >= 0x47800000u) return (uint16_t)(sign | 0x7c00);                         /* >= 2^16 */
    if (a < 0x38800000u) {                                                            /* < 2^-14 */
        float m = rintf(u32f(a) * 16777216.0f); /* exact scaling by 2^24, then RNE */
        return (uint16_t)(sign | (uint16_t)m);  /* m == 1024 is the smallest normal */
    }
    uint32_t h = (((a >> 23) - 112u) << 10) | ((a & 0x7fffffu) >> 13);
    uint32_t rem = a & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++; /* carry may reach inf: correct */
    return (uint16_t)(sign | h);
}

float orc_bf16_to_float(uint16_t b) { return u32f((uint32_t)b << 16); }

uint16_t orc_float_to_bf16(float f) {
    uint32_t u = fu32(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x0040); /* quiet NaN */
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

static inline size_t dtype_size(int dtype) { return dtype == ORC_F32 ? 4 : 2; }

static inline float load_f(const void* p, int dtype, int64_t i) {
    switch (dtype) {
        case ORC_F32: return ((const float*)p)[i];
        case ORC_F16: return orc_half_to_float(((const uint16_t*)p)[i]);
        default: return orc_bf16_to_float(((const uint16_t*)p)[i]);
    }
}

static inline void store_f(void* p, int dtype, int64_t i, float v) {
    switch (dtype) {
        case ORC_F32: ((float*)p)[i] = v; break;
        case ORC_F16: ((uint16_t*)p)[i] = orc_float_to_half(v); break;
        default: ((uint16_t*)p)[i] = orc_float_to_bf16(v); break;
    }
}

/* raw T bytes of a float already representable in T (header values) */
static inline void store_raw(uint8_t* dst, int dtype, float v) {
    if (dtype == ORC_F32) { memcpy(dst, &v, 4); return; }
    uint16_t h = dtype == ORC_F16 ? orc_float_to_half(v) : orc_float_to_bf16(v);
    memcpy(dst, &h, 2);
}

static inline float load_raw(const uint8_t* src, int dtype) {
    if (dtype == ORC_F32) { float v; memcpy(&v, src, 4); return v; }
    uint16_t h; memcpy(&h, src, 2);
    return dtype == ORC_F16 ? orc_half_to_float(h) : orc_bf16_to_float(h);
}

/* Reduction init (K:306,359,369 for f16 = +-65504; cub Traits<float>::Max =
 * FLT_MAX, CUB util_type.cuh:1044-1049).  bf16: largest finite bf16 (ext). */
static inline float dtype_max(int dtype) {
    switch (dtype) {
        case ORC_F32: return u32f(0x7f7fffffu);
        case ORC_F16: return 65504.0f;
        default: return u32f(0x7f7f0000u);
    }
}

/* ------------------------------------------------------------------------ */
/* sizes                                                                    */
/* ------------------------------------------------------------------------ */
static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

size_t orc_minmax_compressed_size(int n_chunks, size_t chunk_size, int dtype) {
    /* DT:679-693: align32(chunk_size*n_chunks) + align32(2*sizeof(T))*n_chunks */
    return align_up(chunk_size * (size_t)n_chunks, 32) +
           align_up(2 * dtype_size(dtype), 32) * (size_t)n_chunks;
}

/* ------------------------------------------------------------------------ */
/* per-chunk min/max                                                        */
/* ------------------------------------------------------------------------ */
/* Total-order key: monotone in the float order with -0 < +0. */
static inline int32_t key_of(float f) {
    int32_t i = (int32_t)fu32(f);
    return i ^ ((i >> 31) & 0x7fffffff);
}
static inline float f_of_key(int32_t k) {
    return u32f((uint32_t)(k ^ ((k >> 31) & 0x7fffffff)));
}

/*
 * K:312-341 (f32: cub::DeviceReduce::Min then ::Max) and K:343-371 (f16:
 * cub::DeviceReduce::Reduce with Min()/Max() at init +-65504).  cub returns
 * op(init, aggregate) (CUB device/dispatch/dispatch_reduce.cuh:133-147) with
 * CUB_MIN(a,b) = (b<a)?b:a, CUB_MAX(a,b) = (b>a)?b:a (util_macro.cuh:61-66);
 * an empty range writes init.  For NaN-free input without a +0/-0 tie this
 * is min/max over {init} U values, which is what is computed here.  The two
 * order-dependent corners of the reference are pinned to an
 * order-independent rule: NaN elements are skipped, and -0 < +0.
 */
void orc_minmax(const void* in, int dtype, int64_t n, float* out_min, float* out_max) {
    const float init = dtype_max(dtype);
    int32_t kmin = key_of(init), kmax = key_of(-init);
#ifdef _OPENMP
#pragma omp parallel
    {
        int32_t lmin = key_of(init), lmax = key_of(-init);
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            float x = load_f(in, dtype, i);
            if (x != x) continue;
            int32_t k = key_of(x);
            if (k < lmin) lmin = k;
            if (k > lmax) lmax = k;
        }
#pragma omp critical
        {
            if (lmin < kmin) kmin = lmin;
            if (lmax > kmax) kmax = lmax;
        }
    }
#else
    for (int64_t i = 0; i < n; ++i) {
        float x = load_f(in, dtype, i);
        if (x != x) continue;
        int32_t k = key_of(x);
        if (k < kmin) kmin = k;
        if (k > kmax) kmax = k;
    }
#endif
    *out_min = f_of_key(kmin);
    *out_max = f_of_key(kmax);
}

/* ------------------------------------------------------------------------ */
/* MinMax-UInt8 quantise / dequantise                                       */
/* ------------------------------------------------------------------------ */
/* K:10: `const float eps = 1e-7;` (double literal converted to float) */
static const double kEpsLiteral = 1e-7;

typedef struct { float scale, lower_bound, upper_bound; } qparams;

/* K:465-467 / K:491-493, evaluated with the reference's exact types:
 *   float scale = 255.0 / (max_ - min_ + eps);   // double division, then float
 *   float upper_bound = rintf(max_ * scale);
 *   float lower_bound = upper_bound - 255.0;      // double subtraction, then float */
static inline qparams make_qparams(float mn, float mx) {
    const float eps = (float)kEpsLiteral;
    float d = (mx - mn) + eps;
    qparams q;
    q.scale = (float)(255.0 / (double)d);
    q.upper_bound = rintf(mx * q.scale);
    q.lower_bound = (float)((double)q.upper_bound - 255.0);
    return q;
}

/* K:410-422 __minmax_uint8_compress: level = rintf(x*scale);
 * level = min(level, upper_bound) (CUDA min(float,float) == fminf);
 * return level - lower_bound, converted to uint8_t.  The conversion is
 * pinned as saturating truncation (nvcc's cvt.rzi clamps; NaN -> 0); in the
 * normal regime the value is already an integer in [0, 255]. */
static inline uint8_t quant(float x, qparams q) {
    float level = rintf(x * q.scale);
    level = fminf(level, q.upper_bound);
    float v = level - q.lower_bound;
    v = fminf(fmaxf(v, 0.0f), 255.0f);
    return (uint8_t)v;
}

/* K:424-432 __minmax_uint8_decompress: (i + lower_bound) / scale */
static inline float dequant(uint8_t b, qparams q) {
    return ((float)b + q.lower_bound) / q.scale;
}

int orc_compress_minmax_u8(const void* in, int dtype, int in_num_elem, int chunk_size,
                           int num_chunks, uint8_t* out, size_t out_bytes, int target_chunk) {
    if (num_chunks <= 0 || chunk_size < 0 || target_chunk < -1 || target_chunk >= num_chunks)
        return -1;
    const size_t esz = dtype_size(dtype);
    const size_t chunk_offset = out_bytes / (size_t)num_chunks; /* K:537 */
    if (chunk_offset < (size_t)chunk_size + 32) return -2;
    int remaining = in_num_elem; /* K:538 */
    for (int c = 0; c < num_chunks; ++c) {
        int n_c = remaining < chunk_size ? remaining : chunk_size;
        if (n_c < 0) n_c = 0;
        remaining -= chunk_size;
        if (target_chunk != -1 && c != target_chunk) continue; /* K:540 */
        const void* src = (const uint8_t*)in + (size_t)c * chunk_size * esz;
        uint8_t* seg = out + (size_t)c * chunk_offset;
        float mn, mx;
        orc_minmax(src, dtype, n_c, &mn, &mx); /* K:541-542, header as T */
        /* K:462-467: kernel re-reads header as T and widens to float */
        memset(seg, 0, 32); /* header gap defined as zero (reference: uninitialised, F7) */
        store_raw(seg, dtype, mn);
        store_raw(seg + esz, dtype, mx);
        qparams q = make_qparams(load_raw(seg, dtype), load_raw(seg + esz, dtype));
        uint8_t* payload = seg + 32; /* K:470 */
        /* K:468-472: EVERY element i < chunk_size of the chunk is quantised
         * with the chunk's parameters -- including elements at or past
         * in_num_elem, which only the min/max (K:541, min(remaining, cs))
         * leaves out.  The input must hold num_chunks*chunk_size elements
         * (DT:327: chunk_size = num_elements_allocated / n_chunks). */
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
        for (int64_t j = 0; j < chunk_size; ++j)
            payload[j] = quant(load_f(src, dtype, j), q);
        /* slack after the payload: zero (reference: uninitialised) */
        memset(seg + 32 + chunk_size, 0, chunk_offset - 32 - (size_t)chunk_size);
    }
    if (target_chunk == -1) /* buffer tail beyond the last segment: zero */
        memset(out + (size_t)num_chunks * chunk_offset, 0,
               out_bytes - (size_t)num_chunks * chunk_offset);
    return 0;
}

int orc_decompress_minmax_u8(const uint8_t* in, size_t in_bytes, int chunk_size,
                             int num_chunks, void* out, int dtype) {
    if (num_chunks <= 0 || chunk_size < 0) return -1;
    const size_t esz = dtype_size(dtype);
    const size_t chunk_offset = in_bytes / (size_t)num_chunks; /* K:566 */
    if (chunk_offset < (size_t)chunk_size + 32) return -2;
    for (int c = 0; c < num_chunks; ++c) {
        const uint8_t* seg = in + (size_t)c * chunk_offset;
        qparams q = make_qparams(load_raw(seg, dtype), load_raw(seg + esz, dtype)); /* K:488-493 */
        void* dst = (uint8_t*)out + (size_t)c * chunk_size * esz;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
        for (int64_t j = 0; j < chunk_size; ++j)
            store_f(dst, dtype, j, dequant(seg[32 + j], q)); /* K:495-499 */
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* chunk reduction (scatter-reduce step)                                    */
/* ------------------------------------------------------------------------ */
/* K:504-529: block_dim_y by num_chunks */
static inline int reduce_block_y(int p) {
    return p <= 4 ? 2 : p <= 8 ? 4 : p <= 16 ? 8 : p <= 32 ? 16 : 32;
}

int orc_reduce_chunks(void* inout, int dtype, int chunk_size, int num_chunks,
                      int target_chunk, int average) {
    if (num_chunks <= 0 || chunk_size < 0 || target_chunk < 0 || target_chunk >= num_chunks)
        return -1;
    const int by = reduce_block_y(num_chunks);
    const size_t esz = dtype_size(dtype);
    void* dst = (uint8_t*)inout + (size_t)target_chunk * chunk_size * esz;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t j = 0; j < chunk_size; ++j) {
        float s[32];
        /* K:385-388: thread y accumulates 0.0f + in[y] + in[y+by] + ... */
        for (int y = 0; y < by; ++y) {
            float acc = 0.0f;
            for (int i = y; i < num_chunks; i += by)
                acc = acc + load_f(inout, dtype, (int64_t)i * chunk_size + j);
            s[y] = acc;
        }
        /* K:171-194: shared-memory tree halving over y */
        for (int h = by / 2; h >= 1; h /= 2)
            for (int y = 0; y < h; ++y) s[y] = s[y] + s[y + h];
        /* K:152-169 __from_float: a / n (float / int -> float division) */
        float r = average ? s[0] / (float)num_chunks : s[0];
        store_f(dst, dtype, j, r);
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* elementwise ops used by the decentralized low-precision op               */
/* ------------------------------------------------------------------------ */
/* K:220-230: f32 x += y; f16 __hadd (correctly rounded half add; computing
 * in float and rounding once is exact here since 24 >= 2*11+2). bf16: same
 * rule (extension). */
void orc_add_inplace(void* x, const void* y, int dtype, int64_t n) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 0; i < n; ++i)
        store_f(x, dtype, i, load_f(x, dtype, i) + load_f(y, dtype, i));
}

/* K:232-242 + K:83-91: f32 `x[i] += y[i] * factor` as nvcc contracts it by
 * default (-fmad=true): fmaf(y, factor, x).  f16: __hadd(a, __hmul(b,
 * half(factor))) — two half roundings.  bf16: the f16 rule in bf16. */
void orc_addmul_inplace(void* x, const void* y, int dtype, int64_t n, float factor) {
    if (dtype == ORC_F32) {
        float* xf = (float*)x;
        const float* yf = (const float*)y;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
        for (int64_t i = 0; i < n; ++i) xf[i] = fmaf(yf[i], factor, xf[i]);
        return;
    }
    uint16_t fh = dtype == ORC_F16 ? orc_float_to_half(factor) : orc_float_to_bf16(factor);
    float f16 = dtype == ORC_F16 ? orc_half_to_float(fh) : orc_bf16_to_float(fh);
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 0; i < n; ++i) {
        float prod = load_f(y, dtype, i) * f16; /* exact in float (<= 2*11 bits) */
        uint16_t pr = dtype == ORC_F16 ? orc_float_to_half(prod) : orc_float_to_bf16(prod);
        float p = dtype == ORC_F16 ? orc_half_to_float(pr) : orc_bf16_to_float(pr);
        store_f(x, dtype, i, load_f(x, dtype, i) + p);
    }
}

/* ------------------------------------------------------------------------ */
/* 1-bit sign + scale codec (this repository's format)        */
/* ------------------------------------------------------------------------ */
/*
 * Segment per chunk: 32-byte header {f32 scale, u32 n_valid, 24 zero bytes}
 * followed by ceil(chunk_size/1024) bit tiles of 128 bytes.  Element j of a
 * chunk lives in tile t = j/1024 at r = j%1024 = sub*256 + lane*4 + e; its
 * bit is bit (sub*4 + e) of the little-endian u16 at byte 2*lane of the tile
 * (each lane's 16 elements form one 16-bit field).
 * bit = (x < 0).  scale = tree_sum(|x|) / n_valid (0 when n_valid == 0).
 * Decode: bit ? -scale : +scale, rounded to T.
 */
#define OB_TILE 1024
#define OB_TILE_BYTES 128

size_t orc_onebit_compressed_size(int n_chunks, size_t chunk_size) {
    size_t tiles = (chunk_size + OB_TILE - 1) / OB_TILE;
    return (size_t)n_chunks * (32 + tiles * OB_TILE_BYTES);
}

/* sum of 1024 values (missing ones are 0): lane-local pairs, then a 64-lane tree */
static float tile_tree(const float* v, int64_t count) {
    float s[64];
    for (int lane = 0; lane < 64; ++lane) {
        float q[4];
        for (int sub = 0; sub < 4; ++sub) {
            float a[4];
            for (int e = 0; e < 4; ++e) {
                int64_t r = (int64_t)sub * 256 + lane * 4 + e;
                a[e] = r < count ? v[r] : 0.0f;
            }
            q[sub] = (a[0] + a[1]) + (a[2] + a[3]);
        }
        s[lane] = (q[0] + q[1]) + (q[2] + q[3]);
    }
    for (int h = 32; h >= 1; h /= 2)
        for (int l = 0; l < h; ++l) s[l] = s[l] + s[l + h];
    return s[0];
}

/* F over tile partials already in part[0..n), level by level in place: tile t of a
 * level reads part[1024t, 1024t + 1024) and writes part[t], and every tile that reads
 * part[t] (tile t / 1024) has run before it, so one ascending pass per level is exact */
static float tree_sum_levels(float* part, int64_t n) {
    while (n > OB_TILE) {
        const int64_t nt = (n + OB_TILE - 1) / OB_TILE;
        for (int64_t t = 0; t < nt; ++t) {
            const int64_t cnt = n - t * OB_TILE;
            part[t] = tile_tree(part + t * OB_TILE, cnt < OB_TILE ? cnt : OB_TILE);
        }
        n = nt;
    }
    return tile_tree(part, n);
}

/* F(v): one tile -> tile_tree; more -> F(tile partials).  F(empty) = 0. */
float orc_onebit_tree_sum(const float* v, int64_t n) {
    if (n <= 0) return 0.0f;
    if (n <= OB_TILE) return tile_tree(v, n);
    int64_t nt = (n + OB_TILE - 1) / OB_TILE;
    float* part = (float*)malloc(sizeof(float) * (size_t)nt);
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t t = 0; t < nt; ++t) {
        int64_t cnt = n - t * OB_TILE;
        part[t] = tile_tree(v + t * OB_TILE, cnt < OB_TILE ? cnt : OB_TILE);
    }
    float r = tree_sum_levels(part, nt);
    free(part);
    return r;
}

/* one tile of a chunk in one pass: its sign bits (bit = x < 0, little-endian u16
 * field per lane) and tile_tree of its |x| (the first level of F) */
static float onebit_tile(const void* src, int dtype, int64_t base, int64_t count, uint8_t* tile_bits) {
    uint16_t w[64];
    float s[64];
    for (int lane = 0; lane < 64; ++lane) {
        float q[4];
        w[lane] = 0;
        for (int sub = 0; sub < 4; ++sub) {
            float a[4];
            for (int e = 0; e < 4; ++e) {
                const int64_t r = (int64_t)sub * 256 + lane * 4 + e;
                a[e] = 0.0f;
                if (r < count) {
                    const float x = load_f(src, dtype, base + r);
                    a[e] = fabsf(x);
                    if (x < 0.0f) w[lane] |= (uint16_t)(1u << (sub * 4 + e));
                }
            }
            q[sub] = (a[0] + a[1]) + (a[2] + a[3]);
        }
        s[lane] = (q[0] + q[1]) + (q[2] + q[3]);
    }
    for (int lane = 0; lane < 64; ++lane) {
        tile_bits[2 * lane] = (uint8_t)(w[lane] & 0xff);
        tile_bits[2 * lane + 1] = (uint8_t)(w[lane] >> 8);
    }
    for (int h = 32; h >= 1; h /= 2)
        for (int l = 0; l < h; ++l) s[l] = s[l] + s[l + h];
    return s[0];
}

int orc_compress_onebit(const void* in, int dtype, int in_num_elem, int chunk_size,
                        int num_chunks, uint8_t* out, size_t out_bytes, int target_chunk) {
    if (num_chunks <= 0 || chunk_size < 0 || target_chunk < -1 || target_chunk >= num_chunks)
        return -1;
    const size_t esz = dtype_size(dtype);
    const size_t chunk_offset = out_bytes / (size_t)num_chunks;
    const int64_t tiles = ((int64_t)chunk_size + OB_TILE - 1) / OB_TILE;
    if (chunk_offset < 32 + (size_t)tiles * OB_TILE_BYTES) return -2;
    /* tile partials of one chunk: one small block per call (no per-chunk copy of |x|) */
    float* part = (float*)malloc(sizeof(float) * (size_t)(tiles > 0 ? tiles : 1));
    if (!part) return -3;
    int remaining = in_num_elem;
    for (int c = 0; c < num_chunks; ++c) {
        int n_c = remaining < chunk_size ? remaining : chunk_size;
        if (n_c < 0) n_c = 0;
        remaining -= chunk_size;
        if (target_chunk != -1 && c != target_chunk) continue;
        const void* src = (const uint8_t*)in + (size_t)c * chunk_size * esz;
        uint8_t* seg = out + (size_t)c * chunk_offset;
        uint8_t* bits = seg + 32;
        /* elements past n_c (a partially valid chunk) are neither summed nor signed */
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
        for (int64_t t = 0; t < tiles; ++t) {
            const int64_t cnt = (int64_t)n_c - t * OB_TILE;
            part[t] = onebit_tile(src, dtype, t * OB_TILE, cnt < 0 ? 0 : (cnt < OB_TILE ? cnt : OB_TILE),
                                  bits + t * OB_TILE_BYTES);
        }
        const int64_t valid_tiles = ((int64_t)n_c + OB_TILE - 1) / OB_TILE;
        float total = n_c > 0 ? tree_sum_levels(part, valid_tiles) : 0.0f;
        float scale = n_c > 0 ? total / (float)n_c : 0.0f;
        uint32_t nv = (uint32_t)n_c;
        memset(seg, 0, 32);
        memcpy(seg, &scale, 4);
        memcpy(seg + 4, &nv, 4);
        memset(seg + 32 + (size_t)tiles * OB_TILE_BYTES, 0,
               chunk_offset - 32 - (size_t)tiles * OB_TILE_BYTES);
    }
    free(part);
    if (target_chunk == -1)
        memset(out + (size_t)num_chunks * chunk_offset, 0,
               out_bytes - (size_t)num_chunks * chunk_offset);
    return 0;
}

int orc_decompress_onebit(const uint8_t* in, size_t in_bytes, int chunk_size, int num_chunks,
                          void* out, int dtype) {
    if (num_chunks <= 0 || chunk_size < 0) return -1;
    const size_t esz = dtype_size(dtype);
    const size_t chunk_offset = in_bytes / (size_t)num_chunks;
    const int64_t tiles = ((int64_t)chunk_size + OB_TILE - 1) / OB_TILE;
    if (chunk_offset < 32 + (size_t)tiles * OB_TILE_BYTES) return -2;
    for (int c = 0; c < num_chunks; ++c) {
        const uint8_t* seg = in + (size_t)c * chunk_offset;
        float scale;
        memcpy(&scale, seg, 4);
        const uint8_t* bits = seg + 32;
        void* dst = (uint8_t*)out + (size_t)c * chunk_size * esz;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
        for (int64_t j = 0; j < chunk_size; ++j) {
            int64_t t = j / OB_TILE;
            int r = (int)(j % OB_TILE);
            int sub = r / 256, lane = (r / 4) % 64, e = r % 4;
            int k = sub * 4 + e;
            int bit = (bits[t * OB_TILE_BYTES + 2 * lane + k / 8] >> (k % 8)) & 1;
            store_f(dst, dtype, j, bit ? -scale : scale);
        }
    }
    return 0;
}
