// store_policy_probe.hip -- which store cache policy should a decode use whose
// 4N output is followed by a kernel streaming ANOTHER 256 MiB buffer (the
// config-2 step: decode -> next encode)?  Every variant writes the same bytes;
// timed: the write kernel W alone, the read kernel R alone, and W then R.
// Policies (gfx950 buffer-store cache-policy bits: sc0 = 1, nt = 2, sc1 = 16).
//   hipcc --offload-arch=gfx950 -O3 -o store_policy_probe store_policy_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int AUX>
__global__ __launch_bounds__(256) void write_kernel(const uint32_t* __restrict__ in, uint32_t* out, int64_t nvec) {
    // like the decode: 4 payload bytes in -> 4 f32 out (16 B) per lane and vector
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
    for (int64_t v = (int64_t)blockIdx.x * 256 * 4 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256 * 4) {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = (v + k * 256 < nvec) ? __builtin_nontemporal_load(in + v + k * 256) : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t i = v + k * 256;
            if (i >= nvec) break;
            u32x4 o = {w[k] & 0xff, (w[k] >> 8) & 0xff, (w[k] >> 16) & 0xff, w[k] >> 24};
            if (AUX < 0) {
                *reinterpret_cast<u32x4*>(out + 4 * i) = o;  // plain global store
            } else if (AUX == 1000) {
                __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(out + 4 * i));
            } else {
                // byte offset within a 2 GiB window: the buffer stays below that
                __builtin_amdgcn_raw_buffer_store_b128(o, rs, (int)(16 * i), 0, AUX);
            }
        }
    }
}

__global__ __launch_bounds__(256) void read_kernel(const u32x4* __restrict__ a, int64_t nvec, uint32_t* sink) {
    uint32_t acc = 0;
    for (int64_t v = (int64_t)blockIdx.x * 256 * 8 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256 * 8) {
        u32x4 r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = (v + k * 256 < nvec) ? a[v + k * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= r[k].x ^ r[k].y ^ r[k].z ^ r[k].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int AUX>
static int run(const char* name, uint32_t* pay, uint32_t* y, u32x4* a, uint32_t* sink, int64_t nvec) {
    hipEvent_t e0, e1, e2;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1)); CHECK(hipEventCreate(&e2));
    const int wgrid = 16384, rgrid = 1024;
    float tw = 0, tr = 0, tboth = 0;
    const int reps = 20;
    for (int r = 0; r < reps + 2; ++r) {
        hipLaunchKernelGGL(read_kernel, dim3(rgrid), dim3(256), 0, 0, a, nvec, sink);  // flush-ish
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(write_kernel<AUX>, dim3(wgrid), dim3(256), 0, 0, pay, y, nvec);
        CHECK(hipEventRecord(e1, 0));
        hipLaunchKernelGGL(read_kernel, dim3(rgrid), dim3(256), 0, 0, a, nvec, sink);
        CHECK(hipEventRecord(e2, 0));
        CHECK(hipEventSynchronize(e2));
        float a1, a2;
        CHECK(hipEventElapsedTime(&a1, e0, e1));
        CHECK(hipEventElapsedTime(&a2, e1, e2));
        if (r >= 2) { tw += a1; tr += a2; tboth += a1 + a2; }
    }
    const double bytes_w = 16.0 * nvec + 4.0 * nvec, bytes_r = 16.0 * nvec;
    printf("{\"policy\": \"%s\", \"write_us\": %.2f, \"write_TBps\": %.3f, \"next_read_us\": %.2f, \"sum_us\": %.2f}\n",
           name, 1e3 * tw / reps, bytes_w / (1e-3 * tw / reps) / 1e12, 1e3 * tr / reps, 1e3 * tboth / reps);
    return 0;
}

int main() {
    const int64_t nvec = (int64_t)1 << 24;  // 16 Mi vectors: 256 MiB out, 64 MiB payload, 256 MiB other buffer
    uint32_t *pay, *y, *sink;
    u32x4* a;
    CHECK(hipMalloc(&pay, 4 * nvec));
    CHECK(hipMalloc(&y, 16 * nvec));
    CHECK(hipMalloc(&a, 16 * nvec));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(pay, 0x5a, 4 * nvec));
    CHECK(hipMemset(a, 0x33, 16 * nvec));
    CHECK(hipDeviceSynchronize());
    for (int round = 0; round < 2; ++round) {
        run<-1>("plain global", pay, y, a, sink, nvec);
        run<1000>("nt global (decode today)", pay, y, a, sink, nvec);
        run<0>("buffer 0", pay, y, a, sink, nvec);
        run<2>("buffer nt", pay, y, a, sink, nvec);
        run<1>("buffer sc0", pay, y, a, sink, nvec);
        run<16>("buffer sc1", pay, y, a, sink, nvec);
        run<17>("buffer sc0 sc1", pay, y, a, sink, nvec);
        run<3>("buffer sc0 nt", pay, y, a, sink, nvec);
        run<18>("buffer sc1 nt", pay, y, a, sink, nvec);
        run<19>("buffer sc0 sc1 nt", pay, y, a, sink, nvec);
    }
    return 0;
}
