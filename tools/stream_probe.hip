// stream_probe.hip — dev tool: HBM streaming ceilings and codec-loop variants
// on gfx950, timed with hipEvents, interleaved rounds in one process
// (cdna_hip_programming.md §5.4 rule 24).  f32, 256 MiB, aligned.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -ffp-contract=off \
//         -fhip-fp32-correctly-rounded-divide-sqrt -o stream_probe stream_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st16(u32x4 v, u32x4* p) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <bool NT>
__device__ __forceinline__ void st4(uint32_t v, uint32_t* p) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

struct Q { float scale, lb, ub; };
__device__ __forceinline__ uint32_t quant(float x, Q q) {
    float l = __builtin_rintf(x * q.scale);
    l = __builtin_fminf(l, q.ub);
    float v = l - q.lb;
    v = __builtin_fminf(__builtin_fmaxf(v, 0.f), 255.f);
    return (uint32_t)v;
}
__device__ __forceinline__ float dequant(uint32_t b, Q q) { return ((float)b + q.lb) / q.scale; }

// ---- ceilings --------------------------------------------------------------
template <int SUB, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ in, u32x4* __restrict__ out, int64_t nvec) {
    for (int64_t base = (int64_t)blockIdx.x * 256 * SUB; base < nvec; base += (int64_t)gridDim.x * 256 * SUB) {
        u32x4 r[SUB];
#pragma unroll
        for (int k = 0; k < SUB; ++k) { int64_t v = base + k * 256 + threadIdx.x; if (v < nvec) r[k] = ld16<NTL>(in + v); }
#pragma unroll
        for (int k = 0; k < SUB; ++k) { int64_t v = base + k * 256 + threadIdx.x; if (v < nvec) st16<NTS>(r[k], out + v); }
    }
}

template <int SUB, bool NTL>
__global__ __launch_bounds__(256) void read_k(const u32x4* __restrict__ in, uint32_t* __restrict__ sink, int64_t nvec) {
    uint32_t acc = 0;
    for (int64_t base = (int64_t)blockIdx.x * 256 * SUB; base < nvec; base += (int64_t)gridDim.x * 256 * SUB) {
        u32x4 r[SUB];
#pragma unroll
        for (int k = 0; k < SUB; ++k) { int64_t v = base + k * 256 + threadIdx.x; if (v < nvec) r[k] = ld16<NTL>(in + v); else r[k] = 0; }
#pragma unroll
        for (int k = 0; k < SUB; ++k) acc ^= r[k].x ^ r[k].y ^ r[k].z ^ r[k].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int SUB, bool NTS>
__global__ __launch_bounds__(256) void write_k(u32x4* __restrict__ out, int64_t nvec) {
    for (int64_t base = (int64_t)blockIdx.x * 256 * SUB; base < nvec; base += (int64_t)gridDim.x * 256 * SUB) {
#pragma unroll
        for (int k = 0; k < SUB; ++k) { int64_t v = base + k * 256 + threadIdx.x; if (v < nvec) st16<NTS>(u32x4{(uint32_t)v, 1u, 2u, 3u}, out + v); }
    }
}

// ---- quantise variants -------------------------------------------------------
// (a) lane = 4 consecutive floats per vector, 4-B store per vector (current product layout)
template <int SUB, bool NTL, bool NTS, bool REV>
__global__ __launch_bounds__(256) void quant4_k(const u32x4* __restrict__ in, uint32_t* __restrict__ out, int64_t nvec, Q q) {
    const int64_t ntiles = (nvec + 256 * SUB - 1) / (256 * SUB);
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t base = (REV ? ntiles - 1 - t : t) * 256 * SUB;
        u32x4 r[SUB];
#pragma unroll
        for (int k = 0; k < SUB; ++k) { int64_t v = base + k * 256 + threadIdx.x; if (v < nvec) r[k] = ld16<NTL>(in + v); }
#pragma unroll
        for (int k = 0; k < SUB; ++k) {
            int64_t v = base + k * 256 + threadIdx.x;
            if (v >= nvec) continue;
            uint32_t b = quant(__uint_as_float(r[k].x), q) | (quant(__uint_as_float(r[k].y), q) << 8) |
                         (quant(__uint_as_float(r[k].z), q) << 16) | (quant(__uint_as_float(r[k].w), q) << 24);
            st4<NTS>(b, out + v);
        }
    }
}

// (b) lane = 16 consecutive floats (4 vectors), one 16-B store
template <int SUB, bool NTL, bool NTS, bool REV>
__global__ __launch_bounds__(256) void quant16_k(const u32x4* __restrict__ in, u32x4* __restrict__ out, int64_t nvec, Q q) {
    // nvec counts 16-B input vectors; lane handles 4 consecutive input vectors per sub-step
    const int64_t nout = nvec / 4;
    const int64_t ntiles = (nout + 256 * SUB - 1) / (256 * SUB);
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t base = (REV ? ntiles - 1 - t : t) * 256 * SUB;
        u32x4 r[SUB][4];
#pragma unroll
        for (int k = 0; k < SUB; ++k) {
            int64_t o = base + k * 256 + threadIdx.x;
            if (o < nout)
#pragma unroll
                for (int j = 0; j < 4; ++j) r[k][j] = ld16<NTL>(in + 4 * o + j);
        }
#pragma unroll
        for (int k = 0; k < SUB; ++k) {
            int64_t o = base + k * 256 + threadIdx.x;
            if (o >= nout) continue;
            uint32_t w[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                w[j] = quant(__uint_as_float(r[k][j].x), q) | (quant(__uint_as_float(r[k][j].y), q) << 8) |
                       (quant(__uint_as_float(r[k][j].z), q) << 16) | (quant(__uint_as_float(r[k][j].w), q) << 24);
            st16<NTS>(u32x4{w[0], w[1], w[2], w[3]}, out + o);
        }
    }
}

// ---- dequantise variants -------------------------------------------------------
template <int SUB, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void deq4_k(const uint32_t* __restrict__ in, u32x4* __restrict__ out, int64_t nvec, Q q) {
    for (int64_t base = (int64_t)blockIdx.x * 256 * SUB; base < nvec; base += (int64_t)gridDim.x * 256 * SUB) {
        uint32_t b[SUB];
#pragma unroll
        for (int k = 0; k < SUB; ++k) {
            int64_t v = base + k * 256 + threadIdx.x;
            if (v < nvec) { if constexpr (NTL) b[k] = __builtin_nontemporal_load(in + v); else b[k] = in[v]; }
        }
#pragma unroll
        for (int k = 0; k < SUB; ++k) {
            int64_t v = base + k * 256 + threadIdx.x;
            if (v >= nvec) continue;
            u32x4 o = {__float_as_uint(dequant(b[k] & 0xff, q)), __float_as_uint(dequant((b[k] >> 8) & 0xff, q)),
                       __float_as_uint(dequant((b[k] >> 16) & 0xff, q)), __float_as_uint(dequant(b[k] >> 24, q))};
            st16<NTS>(o, out + v);
        }
    }
}

// 16 B of bytes per lane -> 4 x 16-B stores at the lane's 64 contiguous bytes
template <int SUB, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void deq16_k(const u32x4* __restrict__ in, u32x4* __restrict__ out, int64_t nin, Q q) {
    for (int64_t base = (int64_t)blockIdx.x * 256 * SUB; base < nin; base += (int64_t)gridDim.x * 256 * SUB) {
        u32x4 b[SUB];
#pragma unroll
        for (int k = 0; k < SUB; ++k) { int64_t v = base + k * 256 + threadIdx.x; if (v < nin) b[k] = ld16<NTL>(in + v); }
#pragma unroll
        for (int k = 0; k < SUB; ++k) {
            int64_t v = base + k * 256 + threadIdx.x;
            if (v >= nin) continue;
            const uint32_t w[4] = {b[k].x, b[k].y, b[k].z, b[k].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                u32x4 o = {__float_as_uint(dequant(w[j] & 0xff, q)), __float_as_uint(dequant((w[j] >> 8) & 0xff, q)),
                           __float_as_uint(dequant((w[j] >> 16) & 0xff, q)), __float_as_uint(dequant(w[j] >> 24, q))};
                st16<NTS>(o, out + 4 * v + j);
            }
        }
    }
}

// q read from a device header per block (like the product), optionally forced uniform
template <bool UNIFORM>
__global__ __launch_bounds__(256) void deq4_hdr_k(const uint32_t* __restrict__ in, u32x4* __restrict__ out, int64_t nvec,
                                                  const float* hdr) {
    Q q{hdr[0], hdr[1], hdr[2]};
    if constexpr (UNIFORM) {
        q.scale = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, q.scale)));
        q.lb = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, q.lb)));
    }
    for (int64_t base = (int64_t)blockIdx.x * 1024; base < nvec; base += (int64_t)gridDim.x * 1024) {
        uint32_t b[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) b[k] = __builtin_nontemporal_load(in + base + k * 256 + threadIdx.x);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            u32x4 o = {__float_as_uint(dequant(b[k] & 0xff, q)), __float_as_uint(dequant((b[k] >> 8) & 0xff, q)),
                       __float_as_uint(dequant((b[k] >> 16) & 0xff, q)), __float_as_uint(dequant(b[k] >> 24, q))};
            __builtin_nontemporal_store(o, out + base + k * 256 + threadIdx.x);
        }
    }
}

// 256-entry table of the exactly-divided values in LDS: no division per element
__global__ __launch_bounds__(256) void deq4_lut_k(const uint32_t* __restrict__ in, u32x4* __restrict__ out, int64_t nvec,
                                                  Q q) {
    __shared__ float lut[256];
    lut[threadIdx.x] = dequant(threadIdx.x, q);
    __syncthreads();
    for (int64_t base = (int64_t)blockIdx.x * 1024; base < nvec; base += (int64_t)gridDim.x * 1024) {
        uint32_t b[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) b[k] = __builtin_nontemporal_load(in + base + k * 256 + threadIdx.x);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            u32x4 o = {__float_as_uint(lut[b[k] & 0xff]), __float_as_uint(lut[(b[k] >> 8) & 0xff]),
                       __float_as_uint(lut[(b[k] >> 16) & 0xff]), __float_as_uint(lut[b[k] >> 24])};
            __builtin_nontemporal_store(o, out + base + k * 256 + threadIdx.x);
        }
    }
}

// ---- min/max read pass ---------------------------------------------------------
__device__ __forceinline__ int32_t key(float f) { int32_t i = __float_as_int(f); return i ^ ((i >> 31) & 0x7fffffff); }
template <int SUB, bool NTL>
__global__ __launch_bounds__(256) void minmax_k(const u32x4* __restrict__ in, uint2* __restrict__ part, int64_t nvec) {
    uint32_t lo = ~0u, hi = ~0u;
    for (int64_t base = (int64_t)blockIdx.x * 256 * SUB; base < nvec; base += (int64_t)gridDim.x * 256 * SUB) {
        u32x4 r[SUB];
        bool ok[SUB];
#pragma unroll
        for (int k = 0; k < SUB; ++k) { int64_t v = base + k * 256 + threadIdx.x; ok[k] = v < nvec; if (ok[k]) r[k] = ld16<NTL>(in + v); }
#pragma unroll
        for (int k = 0; k < SUB; ++k) {
            if (!ok[k]) continue;
            const uint32_t w[4] = {r[k].x, r[k].y, r[k].z, r[k].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                int32_t kk = key(__uint_as_float(w[j]));
                lo = min(lo, (uint32_t)kk - 0x807fffffu);
                hi = min(hi, 0x7f800000u - (uint32_t)kk);
            }
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) { lo = min(lo, (uint32_t)__shfl_xor((int)lo, o)); hi = min(hi, (uint32_t)__shfl_xor((int)hi, o)); }
    __shared__ uint32_t s[2][4];
    if ((threadIdx.x & 63) == 0) { s[0][threadIdx.x / 64] = lo; s[1][threadIdx.x / 64] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 4; ++i) { lo = min(lo, s[0][i]); hi = min(hi, s[1][i]); }
        part[blockIdx.x] = make_uint2(lo, hi);
    }
}

// the product kernels, compiled into this TU for side-by-side timing
#include "../csrc/kernels/minmax_u8.hip"
#include "../csrc/kernels/minmax_resident.hip"
#include "../csrc/kernels/reduce.hip"
#include "../csrc/kernels/status.cpp"

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : (1ll << 26);  // floats
    const int rounds = argc > 2 ? atoi(argv[2]) : 15;
    const int64_t nvec = n / 4;
    u32x4 *x, *y, *bytes;
    uint32_t* sink;
    uint2* part;
    CK(hipMalloc(&x, n * 4));
    CK(hipMalloc(&y, n * 4));
    CK(hipMalloc(&bytes, n));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&part, 8 * 65536));
    {
        std::vector<float> h(n);
        uint64_t s = 0x5EED;
        for (int64_t i = 0; i < n; ++i) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            h[i] = ((int32_t)(s >> 33) - (1 << 30)) * 1e-12f;
        }
        CK(hipMemcpy(x, h.data(), n * 4, hipMemcpyHostToDevice));
    }
    Q q{255.0f / 2.2e-3f, 0, 0};
    q.ub = rintf(1.1e-3f * q.scale);
    q.lb = q.ub - 255.0f;
    struct V { std::string name; double bytes; std::function<void(int)> run; std::vector<float> t; };
    std::vector<V> vs;
    auto add = [&](std::string nm, double b, std::function<void(int)> f) { vs.push_back({nm, b, f, {}}); };
    const double R = n * 4.0, W = n * 4.0, B = n;
    for (int g : {1024, 2048, 4096}) {
        add("copy    SUB4 plain/plain g" + std::to_string(g), R + W, [=](int) { copy_k<4, false, false><<<g, 256>>>(x, y, nvec); });
        add("copy    SUB4 nt/nt       g" + std::to_string(g), R + W, [=](int) { copy_k<4, true, true><<<g, 256>>>(x, y, nvec); });
        add("read    SUB4 plain       g" + std::to_string(g), R, [=](int) { read_k<4, false><<<g, 256>>>(x, sink, nvec); });
        add("read    SUB8 plain       g" + std::to_string(g), R, [=](int) { read_k<8, false><<<g, 256>>>(x, sink, nvec); });
        add("read    SUB4 nt          g" + std::to_string(g), R, [=](int) { read_k<4, true><<<g, 256>>>(x, sink, nvec); });
        add("write   SUB4 plain       g" + std::to_string(g), W, [=](int) { write_k<4, false><<<g, 256>>>(y, nvec); });
        add("write   SUB4 nt          g" + std::to_string(g), W, [=](int) { write_k<4, true><<<g, 256>>>(y, nvec); });
        add("minmax  SUB4 plain       g" + std::to_string(g), R, [=](int) { minmax_k<4, false><<<g, 256>>>(x, part, nvec); });
        add("minmax  SUB8 plain       g" + std::to_string(g), R, [=](int) { minmax_k<8, false><<<g, 256>>>(x, part, nvec); });
    }
    for (int g : {2048, 4096}) {
        add("quant4  SUB4 nt/plain fwd g" + std::to_string(g), R + B, [=](int) { quant4_k<4, true, false, false><<<g, 256>>>(x, (uint32_t*)bytes, nvec, q); });
        add("quant4  SUB4 nt/plain rev g" + std::to_string(g), R + B, [=](int) { quant4_k<4, true, false, true><<<g, 256>>>(x, (uint32_t*)bytes, nvec, q); });
        add("quant4  SUB4 pl/plain rev g" + std::to_string(g), R + B, [=](int) { quant4_k<4, false, false, true><<<g, 256>>>(x, (uint32_t*)bytes, nvec, q); });
        add("quant4  SUB4 nt/nt    rev g" + std::to_string(g), R + B, [=](int) { quant4_k<4, true, true, true><<<g, 256>>>(x, (uint32_t*)bytes, nvec, q); });
        add("quant4  SUB8 nt/plain rev g" + std::to_string(g), R + B, [=](int) { quant4_k<8, true, false, true><<<g, 256>>>(x, (uint32_t*)bytes, nvec, q); });
        add("quant16 SUB1 nt/plain rev g" + std::to_string(g), R + B, [=](int) { quant16_k<1, true, false, true><<<g, 256>>>(x, bytes, nvec, q); });
        add("quant16 SUB2 nt/plain rev g" + std::to_string(g), R + B, [=](int) { quant16_k<2, true, false, true><<<g, 256>>>(x, bytes, nvec, q); });
        add("deq4    SUB4 nt/nt       g" + std::to_string(g), B + W, [=](int) { deq4_k<4, true, true><<<g, 256>>>((uint32_t*)bytes, y, nvec, q); });
        add("deq4    SUB4 pl/plain    g" + std::to_string(g), B + W, [=](int) { deq4_k<4, false, false><<<g, 256>>>((uint32_t*)bytes, y, nvec, q); });
        add("deq4    SUB8 pl/plain    g" + std::to_string(g), B + W, [=](int) { deq4_k<8, false, false><<<g, 256>>>((uint32_t*)bytes, y, nvec, q); });
        add("deq4    SUB8 nt/nt       g" + std::to_string(g), B + W, [=](int) { deq4_k<8, true, true><<<g, 256>>>((uint32_t*)bytes, y, nvec, q); });
        add("deq16   SUB1 pl/plain    g" + std::to_string(g), B + W, [=](int) { deq16_k<1, false, false><<<g, 256>>>(bytes, y, nvec / 4, q); });
        add("deq16   SUB2 pl/plain    g" + std::to_string(g), B + W, [=](int) { deq16_k<2, false, false><<<g, 256>>>(bytes, y, nvec / 4, q); });
        add("deq16   SUB2 nt/nt       g" + std::to_string(g), B + W, [=](int) { deq16_k<2, true, true><<<g, 256>>>(bytes, y, nvec / 4, q); });
    }
    // encode pair: minmax then quantise reverse (the product's sequence), timed as one unit
    add("pair minmax(g2048)+quant4 rev nt", 2 * R + B, [=](int) {
        minmax_k<4, false><<<2048, 256>>>(x, part, nvec);
        quant4_k<4, true, false, true><<<2048, 256>>>(x, (uint32_t*)bytes, nvec, q);
    });
    add("pair minmax(g2048)+quant4 fwd nt", 2 * R + B, [=](int) {
        minmax_k<4, false><<<2048, 256>>>(x, part, nvec);
        quant4_k<4, true, false, false><<<2048, 256>>>(x, (uint32_t*)bytes, nvec, q);
    });
    add("pair minmax(g2048)+quant4 rev plain", 2 * R + B, [=](int) {
        minmax_k<4, false><<<2048, 256>>>(x, part, nvec);
        quant4_k<4, false, false, true><<<2048, 256>>>(x, (uint32_t*)bytes, nvec, q);
    });
    // product path: 256 MiB, p = 1, through the real kernels
    uint8_t* comp;
    const size_t S = bagua_minmax_u8_compressed_bytes(0, (int)n, 1);
    CK(hipMalloc(&comp, S));
    uint8_t* ws;
    const size_t wsb = bagua_minmax_u8_workspace_bytes((int)n, 1);
    CK(hipMalloc(&ws, wsb));
    add("PRODUCT partials", R, [=](int) {
        bagua_minmax_u8_compress_stage(1, 0, x, (int)n, (int)n, 1, comp, S, ws, wsb, -1, nullptr); });
    add("PRODUCT quantize", R + B, [=](int) {
        bagua_minmax_u8_compress_stage(2, 0, x, (int)n, (int)n, 1, comp, S, ws, wsb, -1, nullptr); });
    add("PRODUCT dequantize", B + W, [=](int) {
        bagua_minmax_u8_decompress(0, comp, S, (int)n, 1, y, nullptr); });
    add("PRODUCT dequantize raw-launch g2048", B + W, [=](int) {
        hipLaunchKernelGGL(bagua::minmax_dequantize_kernel<bagua::F32>, dim3(2048, 1), dim3(256), 0, nullptr,
                           comp, (int64_t)S, (int64_t)n, (int64_t)0, (int64_t)n, (float*)y); });
    float* hdr;
    CK(hipMalloc(&hdr, 16));
    {
        float h[4] = {q.scale, q.lb, q.ub, 0};
        CK(hipMemcpy(hdr, h, 16, hipMemcpyHostToDevice));
    }
    for (int g : {2048, 4096}) {
        add("deq4 hdr(vgpr q)        g" + std::to_string(g), B + W, [=](int) { deq4_hdr_k<false><<<g, 256>>>((uint32_t*)bytes, y, nvec, hdr); });
        add("deq4 hdr(readfirstlane) g" + std::to_string(g), B + W, [=](int) { deq4_hdr_k<true><<<g, 256>>>((uint32_t*)bytes, y, nvec, hdr); });
        add("deq4 lut                g" + std::to_string(g), B + W, [=](int) { deq4_lut_k<<<g, 256>>>((uint32_t*)bytes, y, nvec, q); });
    }
    // order effects: what ran just before changes the cache state the next kernel sees
    add("ORDER pre: write y", W, [=](int) { write_k<4, false><<<4096, 256>>>(y, nvec); });
    add("ORDER deq4 nt/nt after write y", B + W, [=](int) { deq4_k<4, true, true><<<4096, 256>>>((uint32_t*)bytes, y, nvec, q); });
    add("ORDER deq4 nt/nt again", B + W, [=](int) { deq4_k<4, true, true><<<4096, 256>>>((uint32_t*)bytes, y, nvec, q); });
    add("ORDER deq4 lut after deq4", B + W, [=](int) { deq4_lut_k<<<4096, 256>>>((uint32_t*)bytes, y, nvec, q); });
    add("ORDER pre: read x", R, [=](int) { read_k<4, false><<<4096, 256>>>(x, sink, nvec); });
    add("ORDER deq4 lut after read x", B + W, [=](int) { deq4_lut_k<<<4096, 256>>>((uint32_t*)bytes, y, nvec, q); });
    add("ORDER pre: quant4 (writes bytes)", R + B, [=](int) { quant4_k<4, true, true, true><<<2048, 256>>>(x, (uint32_t*)bytes, nvec, q); });
    add("ORDER deq4 nt/nt after quant", B + W, [=](int) { deq4_k<4, true, true><<<4096, 256>>>((uint32_t*)bytes, y, nvec, q); });
    add("ORDER pre: quant4 again", R + B, [=](int) { quant4_k<4, true, true, true><<<2048, 256>>>(x, (uint32_t*)bytes, nvec, q); });
    add("ORDER PRODUCT dequantize after quant", B + W, [=](int) { bagua_minmax_u8_decompress(0, comp, S, (int)n, 1, y, nullptr); });
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& v : vs) v.run(0);  // warm
    CK(hipDeviceSynchronize());
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            CK(hipEventRecord(e0));
            v.run(r);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.t.push_back(ms);
        }
    std::printf("%-40s %10s %10s %9s\n", "variant", "median_us", "min_us", "GB/s(med)");
    for (auto& v : vs) {
        std::sort(v.t.begin(), v.t.end());
        const double med = v.t[v.t.size() / 2];
        std::printf("%-40s %10.2f %10.2f %9.1f\n", v.name.c_str(), med * 1e3, v.t[0] * 1e3, v.bytes / (med * 1e-3) / 1e9);
    }
    return 0;
}
