// cvt_probe.hip — exhaustive check (all 2^32 f32 bit patterns) that
// v_cvt_pk_u8_f32 equals the codec's saturating conversion
// (uint32)fminf(fmaxf(v, 0), 255) (codec_common.hpp quant()) on every f32 bit
// pattern the codec can feed it: integers, NaN, +-inf, +-0 (-DINTEGRAL_ONLY=0
// also counts non-integers, where the instruction rounds and the cast truncates).  Prints the mismatch count and the
// first few mismatching inputs.
//   hipcc --offload-arch=gfx950 -O3 tools/cvt_probe.hip -o tools/cvt_probe && ./tools/cvt_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#ifndef INTEGRAL_ONLY
#define INTEGRAL_ONLY 1
#endif

__global__ void probe(unsigned long long* bad, uint32_t* first) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < (1ull << 32); u += stride) {
        const float v = __uint_as_float((uint32_t)u);
        // the codec only converts level - lower_bound: an integer (or NaN / inf);
        // non-integral inputs differ by design (v_cvt_pk_u8_f32 rounds, the cast truncates)
        if (INTEGRAL_ONLY && __builtin_isfinite(v) && __builtin_rintf(v) != v) continue;
        const uint32_t ref = (uint32_t)__builtin_fminf(__builtin_fmaxf(v, 0.0f), 255.0f);
        const uint32_t got = __builtin_amdgcn_cvt_pk_u8_f32(v, 0, 0) & 0xffu;
        if (ref != got) {
            const unsigned long long k = atomicAdd(bad, 1ull);
            if (k < 8) first[k] = (uint32_t)u;
        }
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 32) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(first, 0, 32);
    probe<<<4096, 256>>>(bad, first);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    unsigned long long nb = 0;
    uint32_t f[8];
    (void)hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
    printf("{\"mismatches\": %llu, \"first\": [", nb);
    for (int i = 0; i < 8 && (unsigned long long)i < nb; ++i) printf("%s\"0x%08x\"", i ? ", " : "", f[i]);
    printf("]}\n");
    return 0;
}
