// policy_probe.hip — dev tool: cache-policy sweep of the whole MinMax-UInt8
// encode+decode step (partials -> quantise -> dequantise) run back to back,
// because the 256 MiB Infinity Cache couples the three kernels: which stream
// is left cache-resident by one kernel decides what the next one reads from
// HBM.  f32, 2^26 elements, p = 1.  Bit k of the policy mask selects the
// non-temporal form of: 0 partials load, 1 quantise load, 2 quantise store,
// 3 dequantise load, 4 dequantise store.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -fhip-fp32-correctly-rounded-divide-sqrt -o policy_probe policy_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);  \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct Q { float scale, lb, ub; };

template <bool NT, typename V> __device__ __forceinline__ V ld(const V* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}
template <bool NT, typename V> __device__ __forceinline__ void st(V v, V* p) {
    if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}
__device__ __forceinline__ uint32_t quant(float x, Q q) {
    float l = __builtin_rintf(x * q.scale);
    l = __builtin_fminf(l, q.ub);
    float v = __builtin_fminf(__builtin_fmaxf(l - q.lb, 0.f), 255.f);
    return (uint32_t)v;
}
__device__ __forceinline__ float dequant(uint32_t b, Q q) { return ((float)b + q.lb) / q.scale; }
__device__ __forceinline__ int32_t key(float f) { int32_t i = __float_as_int(f); return i ^ ((i >> 31) & 0x7fffffff); }

template <bool NTL>
__global__ __launch_bounds__(256) void partials_k(const u32x4* __restrict__ in, uint2* __restrict__ part, int64_t nvec) {
    uint32_t lo = ~0u, hi = ~0u;
    for (int64_t base = (int64_t)blockIdx.x * 2048; base < nvec; base += (int64_t)gridDim.x * 2048) {
        u32x4 r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = ld<NTL>(in + base + k * 256 + threadIdx.x);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t w[4] = {r[k].x, r[k].y, r[k].z, r[k].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int32_t kk = key(__uint_as_float(w[j]));
                lo = min(lo, (uint32_t)kk - 0x807fffffu);
                hi = min(hi, 0x7f800000u - (uint32_t)kk);
            }
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
        hi = min(hi, (uint32_t)__shfl_xor((int)hi, o));
    }
    __shared__ uint32_t s[2][4];
    if ((threadIdx.x & 63) == 0) { s[0][threadIdx.x / 64] = lo; s[1][threadIdx.x / 64] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 4; ++i) { lo = min(lo, s[0][i]); hi = min(hi, s[1][i]); }
        part[blockIdx.x] = make_uint2(lo, hi);
    }
}

template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void quant_k(const u32x4* __restrict__ in, uint32_t* __restrict__ out, int64_t nvec, Q q) {
    const int64_t ntiles = nvec / 1024;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t base = (ntiles - 1 - t) * 1024;
        u32x4 r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = ld<NTL>(in + base + k * 256 + threadIdx.x);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t b = quant(__uint_as_float(r[k].x), q) | (quant(__uint_as_float(r[k].y), q) << 8) |
                         (quant(__uint_as_float(r[k].z), q) << 16) | (quant(__uint_as_float(r[k].w), q) << 24);
            st<NTS>(b, out + base + k * 256 + threadIdx.x);
        }
    }
}

template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void deq_k(const uint32_t* __restrict__ in, u32x4* __restrict__ out, int64_t nvec, Q q) {
    for (int64_t base = (int64_t)blockIdx.x * 1024; base < nvec; base += (int64_t)gridDim.x * 1024) {
        uint32_t b[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) b[k] = ld<NTL>(in + base + k * 256 + threadIdx.x);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            u32x4 o = {__float_as_uint(dequant(b[k] & 0xff, q)), __float_as_uint(dequant((b[k] >> 8) & 0xff, q)),
                       __float_as_uint(dequant((b[k] >> 16) & 0xff, q)), __float_as_uint(dequant(b[k] >> 24, q))};
            st<NTS>(o, out + base + k * 256 + threadIdx.x);
        }
    }
}

struct Bufs { u32x4* x; uint32_t* bytes; u32x4* y; uint2* part; int64_t nvec; Q q; };
using StepFn = void (*)(const Bufs&, hipEvent_t*);

template <int M>
void step(const Bufs& b, hipEvent_t* ev) {
    constexpr bool PL = M & 1, QL = M & 2, QS = M & 4, DL = M & 8, DS = M & 16;
    if (ev) (void)hipEventRecord(ev[0]);
    partials_k<PL><<<1024, 256>>>(b.x, b.part, b.nvec);
    if (ev) (void)hipEventRecord(ev[1]);
    quant_k<QL, QS><<<2048, 256>>>(b.x, b.bytes, b.nvec, b.q);
    if (ev) (void)hipEventRecord(ev[2]);
    deq_k<DL, DS><<<4096, 256>>>(b.bytes, b.y, b.nvec, b.q);
    if (ev) (void)hipEventRecord(ev[3]);
}

template <size_t... I>
constexpr std::array<StepFn, sizeof...(I)> make_steps(std::index_sequence<I...>) { return {&step<(int)I>...}; }

int main(int argc, char** argv) {
    const int64_t n = 1ll << 26, nvec = n / 4;
    const int rounds = argc > 1 ? atoi(argv[1]) : 5, steps = 10;
    Bufs b;
    CK(hipMalloc(&b.x, n * 4));
    CK(hipMalloc(&b.y, n * 4));
    CK(hipMalloc(&b.bytes, n));
    CK(hipMalloc(&b.part, 8 * 4096));
    CK(hipMemset(b.x, 0x3a, n * 4));
    b.nvec = nvec;
    b.q = Q{255.0f / 2.2e-3f, 0, 0};
    b.q.ub = rintf(1.1e-3f * b.q.scale);
    b.q.lb = b.q.ub - 255.0f;
    auto fns = make_steps(std::make_index_sequence<32>{});
    std::vector<std::vector<float>> tot(32), per(32 * 3);
    hipEvent_t ev[4], s0, s1;
    for (auto& evi : ev) CK(hipEventCreate(&evi));
    CK(hipEventCreate(&s0));
    CK(hipEventCreate(&s1));
    for (int m = 0; m < 32; ++m) fns[m](b, nullptr);
    CK(hipDeviceSynchronize());
    for (int r = 0; r < rounds; ++r)
        for (int m = 0; m < 32; ++m) {
            for (int w = 0; w < 2; ++w) fns[m](b, nullptr);  // bring caches to the steady state of this policy
            CK(hipEventRecord(s0));
            for (int s = 0; s < steps; ++s) fns[m](b, nullptr);
            CK(hipEventRecord(s1));
            fns[m](b, ev);
            CK(hipEventSynchronize(ev[3]));
            float ms;
            CK(hipEventElapsedTime(&ms, s0, s1));
            tot[m].push_back(ms * 1e3f / steps);
            for (int k = 0; k < 3; ++k) {
                CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
                per[m * 3 + k].push_back(ms * 1e3f);
            }
        }
    auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    std::vector<int> order(32);
    for (int m = 0; m < 32; ++m) order[m] = m;
    std::sort(order.begin(), order.end(), [&](int a, int c) { return med(tot[a]) < med(tot[c]); });
    std::printf("mask  pL qL qS dL dS   step_us  partials quantise dequant  (nt = 1)\n");
    for (int m : order)
        std::printf("%4d   %d  %d  %d  %d  %d  %8.2f  %8.2f %8.2f %8.2f\n", m, m & 1, (m >> 1) & 1, (m >> 2) & 1,
                    (m >> 3) & 1, (m >> 4) & 1, med(tot[m]), med(per[m * 3]), med(per[m * 3 + 1]), med(per[m * 3 + 2]));
    return 0;
}
