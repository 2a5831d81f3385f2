// elementwise.hip — in-place vector ops (bagua_kernels.cu:196-266, exports :574-628).
//
// On the hot path only add / addmul matter (the decentralized low-precision
// op, decentralized_low_precision_synchronous.rs:45-60,126-151); the rest
// are kept so libbagua_kernels exports every symbol the reference's Rust FFI
// binds (src/kernels/mod.rs:3-137).  16-byte vectorised grid-stride loops.
//
// Numerics:
//  f32 addmul: nvcc contracts `x += y*factor` (-fmad=true) -> fmaf(y, factor, x)
//  f16: __hadd/__hmul/__hsub are correctly rounded half ops == one float op +
//       RNE to half (24 >= 2*11+2); bf16 follows the same rule (extension).
//  f16 average: __hadd(a,b) / half(2) (K:53-61) -> half(half(a+b) / 2).
//  f16 divide: the reference's __hdiv uses an approximate reciprocal; here it
//       is the correctly rounded quotient (parity unpinned, off the hot path).
#include "codec_common.hpp"
#include "launch_util.hpp"

namespace bagua {

enum class Op { Add, AddMul, Sub, Avg, Div };

template <typename T, Op OP>
__device__ __forceinline__ float apply(float x, float y, float f) {
    if constexpr (OP == Op::Add) return x + y;
    if constexpr (OP == Op::Sub) return x - y;
    if constexpr (OP == Op::Div) return x / f;
    if constexpr (OP == Op::Avg) {
        if constexpr (sizeof(typename T::storage) == 4) return (x + y) / 2.0f;  // K:198 (exact halving)
        return T::to_f(T::from_f(x + y)) / 2.0f;
    }
    if constexpr (OP == Op::AddMul) {
        if constexpr (sizeof(typename T::storage) == 4) return __builtin_fmaf(y, f, x);
        return x + T::to_f(T::from_f(y * f));  // f is already rounded to T by the launcher
    }
    return x;
}

template <typename T, Op OP, bool VEC>
__global__ __launch_bounds__(kBlock) void binary_kernel(typename T::storage* __restrict__ x,
                                                        const typename T::storage* __restrict__ y,
                                                        int64_t n, float f) {
    constexpr int N = Vec<T>::N;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    int64_t done = 0;
    if constexpr (VEC) {
        const int64_t nvec = n / N;
        for (int64_t v = tid; v < nvec; v += stride) {
            float a[N], b[N];
            unpack16<T>(reinterpret_cast<const uint4*>(x)[v], a);
            if constexpr (OP != Op::Div) unpack16<T>(reinterpret_cast<const uint4*>(y)[v], b);
#pragma unroll
            for (int i = 0; i < N; ++i) a[i] = apply<T, OP>(a[i], OP == Op::Div ? 0.0f : b[i], f);
            reinterpret_cast<uint4*>(x)[v] = pack16<T>(a);
        }
        done = nvec * N;
    }
    for (int64_t i = done + tid; i < n; i += stride)
        x[i] = T::from_f(apply<T, OP>(T::to_f(x[i]), OP == Op::Div ? 0.0f : T::to_f(y[i]), f));
}

template <typename T, Op OP>
static int launch_binary(void* x, const void* y, int n, float f, hipStream_t s) {
    using S = typename T::storage;
    if (!x || (OP != Op::Div && !y) || n < 0) return BAGUA_ERR_INVALID_ARG;
    if (n == 0) return BAGUA_OK;
    const bool vec = ((uintptr_t)x % 16 == 0) && (OP == Op::Div || (uintptr_t)y % 16 == 0);
    int64_t blocks = ((int64_t)n / (vec ? Vec<T>::N : 1) + kBlock - 1) / kBlock;
    if (blocks > kTargetBlocks) blocks = kTargetBlocks;
    if (blocks < 1) blocks = 1;
    if (vec)
        launch((binary_kernel<T, OP, true>), dim3(blocks), dim3(kBlock), 0, s, static_cast<S*>(x),
                           static_cast<const S*>(y), (int64_t)n, f);
    else
        launch((binary_kernel<T, OP, false>), dim3(blocks), dim3(kBlock), 0, s, static_cast<S*>(x),
                           static_cast<const S*>(y), (int64_t)n, f);
    return check_launch();
}

__global__ __launch_bounds__(kBlock) void async_model_average_kernel(float* tensor, const float* reduced,
                                                                     const float* copy, float nranks, int n) {
    // K:257-266
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
        atomicAdd(&tensor[i], reduced[i] / nranks - copy[i]);
}

}  // namespace bagua

using namespace bagua;

namespace {
// round a host float to T and back: the 16-bit kernels take factor / divisor
// as a T value (K:600 `__float2half(factor)`, K:251 `__float2half(D_)`)
float round_to(int dtype, float f) {
    if (dtype == BAGUA_DTYPE_F16) return (float)(_Float16)f;
    if (dtype == BAGUA_DTYPE_BF16) {
        uint32_t u = __builtin_bit_cast(uint32_t, f);
        if ((u & 0x7fffffffu) > 0x7f800000u) return f;
        u += 0x7fffu + ((u >> 16) & 1u);
        return __builtin_bit_cast(float, u & 0xffff0000u);
    }
    return f;
}

template <Op OP>
int dispatch_binary(int dtype, void* x, const void* y, int n, float f, bagua_stream_t stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    f = round_to(dtype, f);
    switch (dtype) {
        case BAGUA_DTYPE_F32: return launch_binary<F32, OP>(x, y, n, f, s);
        case BAGUA_DTYPE_F16: return launch_binary<F16, OP>(x, y, n, f, s);
        case BAGUA_DTYPE_BF16: return launch_binary<BF16, OP>(x, y, n, f, s);
    }
    return BAGUA_ERR_UNSUPPORTED;
}
}  // namespace

extern "C" {

int bagua_add_inplace(int dtype, void* x, const void* y, int n, bagua_stream_t s) {
    return dispatch_binary<Op::Add>(dtype, x, y, n, 0.0f, s);
}
int bagua_addmul_inplace(int dtype, void* x, const void* y, int n, float factor, bagua_stream_t s) {
    return dispatch_binary<Op::AddMul>(dtype, x, y, n, factor, s);
}
int bagua_substract_inplace(int dtype, void* x, const void* y, int n, bagua_stream_t s) {
    return dispatch_binary<Op::Sub>(dtype, x, y, n, 0.0f, s);
}
int bagua_average_inplace(int dtype, void* x, const void* y, int n, bagua_stream_t s) {
    return dispatch_binary<Op::Avg>(dtype, x, y, n, 0.0f, s);
}
int bagua_divide_inplace(int dtype, void* x, float d, int n, bagua_stream_t s) {
    return dispatch_binary<Op::Div>(dtype, x, nullptr, n, d, s);
}

// ---- v1 surface (bagua_kernels.cu:574-628) --------------------------------
#define V1(call) v1_check((call), __FILE__, __LINE__)
void divide_inplace_f32_host(float* x, float D_, int N, bagua_stream_t s) { V1(bagua_divide_inplace(BAGUA_DTYPE_F32, x, D_, N, s)); }
void divide_inplace_f16_host(bagua_half_t* x, float D_, int N, bagua_stream_t s) { V1(bagua_divide_inplace(BAGUA_DTYPE_F16, x, D_, N, s)); }
void add_inplace_f32_host(float* x, float* y, int N, bagua_stream_t s) { V1(bagua_add_inplace(BAGUA_DTYPE_F32, x, y, N, s)); }
void add_inplace_f16_host(bagua_half_t* x, bagua_half_t* y, int N, bagua_stream_t s) { V1(bagua_add_inplace(BAGUA_DTYPE_F16, x, y, N, s)); }
void add_inplace_bf16_host(bagua_bf16_t* x, bagua_bf16_t* y, int N, bagua_stream_t s) { V1(bagua_add_inplace(BAGUA_DTYPE_BF16, x, y, N, s)); }
void addmul_inplace_f32_host(float* x, float* y, int N, const float factor, bagua_stream_t s) { V1(bagua_addmul_inplace(BAGUA_DTYPE_F32, x, y, N, factor, s)); }
void addmul_inplace_f16_host(bagua_half_t* x, bagua_half_t* y, int N, const float factor, bagua_stream_t s) { V1(bagua_addmul_inplace(BAGUA_DTYPE_F16, x, y, N, factor, s)); }
void addmul_inplace_bf16_host(bagua_bf16_t* x, bagua_bf16_t* y, int N, const float factor, bagua_stream_t s) { V1(bagua_addmul_inplace(BAGUA_DTYPE_BF16, x, y, N, factor, s)); }
void substract_inplace_f32_host(float* x, float* y, int N, bagua_stream_t s) { V1(bagua_substract_inplace(BAGUA_DTYPE_F32, x, y, N, s)); }
void substract_inplace_f16_host(bagua_half_t* x, bagua_half_t* y, int N, bagua_stream_t s) { V1(bagua_substract_inplace(BAGUA_DTYPE_F16, x, y, N, s)); }
void average_inplace_f32_host(float* x, float* y, int N, bagua_stream_t s) { V1(bagua_average_inplace(BAGUA_DTYPE_F32, x, y, N, s)); }
void average_inplace_f16_host(bagua_half_t* x, bagua_half_t* y, int N, bagua_stream_t s) { V1(bagua_average_inplace(BAGUA_DTYPE_F16, x, y, N, s)); }
void async_model_average_host(float* tensor, const float* reduced_tensor_copy, const float* tensor_copy,
                              const float nranks, const int N, bagua_stream_t stream) {
    if (N <= 0) return;
    int blocks = (N + kBlock - 1) / kBlock;
    if (blocks > kTargetBlocks) blocks = kTargetBlocks;
    launch(async_model_average_kernel, dim3(blocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                       tensor, reduced_tensor_copy, tensor_copy, nranks, N);
    V1(check_launch());
}
#undef V1

}  // extern "C"
