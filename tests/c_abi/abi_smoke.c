/*
 * abi_smoke.c — a plain C caller of the drop-in boundary (what the reference's
 * Rust FFI, bagua-core-internal/src/kernels/mod.rs:3-137, and its C shim,
 * bagua-core-c/src/lib.rs:9-69, bind), checked against the C oracle.
 *
 * TEST ONLY (links oracle/build/libbagua_oracle.so as the checker).  Runs on a
 * GPU box: tests/test_gpu_c_abi.py.  Exercises, through C declarations only:
 *   v1 names   array_min_max_size_f32_host, compress_f32_to_uint8_host,
 *              decompress_uint8_to_f32_host, reduce_mean_f32_inplace_host,
 *              addmul_inplace_f32_host
 *   v2 names   bagua_minmax_u8_compress / _decompress (status codes, bad args)
 *   C shim     bagua_generate_nccl_unique_id_str, bagua_single_communicator_c_create /
 *              _nranks / _destroy (null-safe), bagua_centralized_low_precision_synchronous
 * Every byte of the compressed buffers and every decoded float is compared
 * with the oracle; exits non-zero on the first difference.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "bagua_core.h"
#include "bagua_kernels.h"
#include "bagua_oracle.h"

#define CHECK(cond, ...)                                 \
    do {                                                 \
        if (!(cond)) {                                   \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                \
            fputc('\n', stderr);                         \
            exit(1);                                     \
        }                                                \
    } while (0)
#define HIPCHECK(x) CHECK((x) == hipSuccess, "%s", #x)

/* deterministic N(0, 1e-3^2)-ish inputs: splitmix64 -> Box-Muller */
static uint64_t sm_state = 0x5EEDull;
static uint64_t splitmix64(void) {
    uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static float gauss(void) {
    const double u1 = ((splitmix64() >> 11) + 1.0) / 9007199254740993.0;
    const double u2 = (splitmix64() >> 11) / 9007199254740992.0;
    return (float)(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
}

static void* dev_upload(const void* h, size_t bytes) {
    void* d = NULL;
    HIPCHECK(hipMalloc(&d, bytes ? bytes : 1));
    if (bytes) HIPCHECK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
    return d;
}

static void download(void* h, const void* d, size_t bytes) {
    HIPCHECK(hipDeviceSynchronize());
    HIPCHECK(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
}

int main(void) {
    const int p = 4, cs = (1 << 18) + 77; /* ragged chunks: scalar heads / tails, slack bytes */
    const int n = p * cs;
    float* x = (float*)malloc(sizeof(float) * (size_t)n);
    for (int i = 0; i < n; ++i) x[i] = gauss() * 1e-3f + (float)(i / cs) * 0.01f;
    hipStream_t s;
    HIPCHECK(hipStreamCreate(&s));

    /* ---- v1: the reference's exact entry points (K:573-691) ---------------- */
    const size_t S = orc_minmax_compressed_size(p, (size_t)cs, ORC_F32);
    CHECK(S == bagua_minmax_u8_compressed_bytes(BAGUA_DTYPE_F32, cs, p), "compressed size");
    float* dx = (float*)dev_upload(x, sizeof(float) * (size_t)n);
    uint8_t* dc = NULL;
    HIPCHECK(hipMalloc((void**)&dc, S));
    HIPCHECK(hipMemset(dc, 0xA5, S)); /* poison: every defined byte must be written */
    /* datatypes/mod.rs:337-345: temp size query per compress call */
    const size_t tmp_bytes = array_min_max_size_f32_host(dx, cs, (float*)dc, s);
    CHECK(tmp_bytes >= bagua_minmax_u8_workspace_bytes(cs, p), "temp size %zu", tmp_bytes);
    void* dtmp = NULL;
    HIPCHECK(hipMalloc(&dtmp, tmp_bytes));  /* the reference pulls exactly this much (DT:343-345) */
    compress_f32_to_uint8_host(dx, n, cs, p, dc, S, dtmp, tmp_bytes, -1, s);
    uint8_t* want = (uint8_t*)malloc(S);
    CHECK(orc_compress_minmax_u8(x, ORC_F32, n, cs, p, want, S, -1) == 0, "oracle compress");
    uint8_t* got = (uint8_t*)malloc(S);
    download(got, dc, S);
    for (size_t i = 0; i < S; ++i) CHECK(got[i] == want[i], "compressed byte %zu: %u vs %u", i, got[i], want[i]);

    float* dy = NULL;
    HIPCHECK(hipMalloc((void**)&dy, sizeof(float) * (size_t)n));
    decompress_uint8_to_f32_host(dc, S, cs, p, dy, s);
    float* y = (float*)malloc(sizeof(float) * (size_t)n);
    float* yw = (float*)malloc(sizeof(float) * (size_t)n);
    CHECK(orc_decompress_minmax_u8(want, S, cs, p, yw, ORC_F32) == 0, "oracle decompress");
    download(y, dy, sizeof(float) * (size_t)n);
    CHECK(memcmp(y, yw, sizeof(float) * (size_t)n) == 0, "decoded floats differ from the oracle");

    /* reduce_mean of the decoded chunks into chunk 2 (K:373-400), addmul (K:220-242) */
    reduce_mean_f32_inplace_host(dy, cs, p, 2, s);
    CHECK(orc_reduce_chunks(yw, ORC_F32, cs, p, 2, 1) == 0, "oracle reduce");
    addmul_inplace_f32_host(dy, dx, n, (float)(1.0 / 3.0), s);
    orc_addmul_inplace(yw, x, ORC_F32, n, (float)(1.0 / 3.0));
    download(y, dy, sizeof(float) * (size_t)n);
    CHECK(memcmp(y, yw, sizeof(float) * (size_t)n) == 0, "reduce_mean + addmul differ from the oracle");

    /* ---- v2: status codes instead of exit() ------------------------------- */
    CHECK(bagua_minmax_u8_compress(BAGUA_DTYPE_F32, dx, n, cs, p, dc, S, dtmp, 0, -1, s) == BAGUA_ERR_WORKSPACE,
          "too-small workspace must be refused");
    CHECK(bagua_minmax_u8_compress(BAGUA_DTYPE_F32, dx, n, cs, p, dc, S, dtmp, tmp_bytes, p, s) ==
              BAGUA_ERR_INVALID_ARG,
          "target chunk out of range must be refused");
    CHECK(strcmp(bagua_status_string(BAGUA_ERR_WORKSPACE), "workspace too small") == 0, "status string");

    /* ---- C shim + comm op (bagua-core-c/src/lib.rs:9-69, p = 1 over RCCL) --- */
    char id[512];
    CHECK(bagua_generate_nccl_unique_id_str(id, sizeof id) == 0, "unique id");
    BaguaSingleCommunicatorC* c = bagua_single_communicator_c_create(0, 1, 0, (uint64_t)(uintptr_t)s, id);
    CHECK(c != NULL, "communicator create");
    size_t nranks = 0;
    CHECK(bagua_single_communicator_c_nranks(&c, &nranks) == 0 && nranks == 1, "nranks");
    HIPCHECK(hipMemcpy(dx, x, sizeof(float) * (size_t)n, hipMemcpyHostToDevice));
    bagua_tensor_t t = {(uint64_t)(uintptr_t)dx, (uint64_t)n, (uint64_t)n, BAGUA_DTYPE_F32, 0};
    /* centralized_low_precision_synchronous.rs:30-71 at one rank: compress(1 chunk) ->
     * exchange (identity) -> decompress -> reduce_mean -> compress(own) -> decompress */
    CHECK(bagua_centralized_low_precision_synchronous(c, &t, 1, BAGUA_COMPRESSION_MINMAX_UINT8) == 0, "op");
    const size_t S1 = orc_minmax_compressed_size(1, (size_t)n, ORC_F32);
    uint8_t* w1 = (uint8_t*)malloc(S1);
    memcpy(yw, x, sizeof(float) * (size_t)n);
    CHECK(orc_compress_minmax_u8(yw, ORC_F32, n, n, 1, w1, S1, -1) == 0, "sim compress");
    CHECK(orc_decompress_minmax_u8(w1, S1, n, 1, yw, ORC_F32) == 0, "sim decompress");
    CHECK(orc_reduce_chunks(yw, ORC_F32, n, 1, 0, 1) == 0, "sim reduce");
    CHECK(orc_compress_minmax_u8(yw, ORC_F32, n, n, 1, w1, S1, 0) == 0, "sim compress own");
    CHECK(orc_decompress_minmax_u8(w1, S1, n, 1, yw, ORC_F32) == 0, "sim decompress");
    download(y, dx, sizeof(float) * (size_t)n);
    CHECK(memcmp(y, yw, sizeof(float) * (size_t)n) == 0, "centralized op differs from the oracle simulation");
    bagua_single_communicator_c_destroy(&c);
    CHECK(c == NULL, "destroy nulls the caller's pointer");
    bagua_single_communicator_c_destroy(&c); /* lib.rs:32-38: null is a no-op */
    CHECK(bagua_single_communicator_c_nranks(&c, &nranks) == -1, "nranks on null");

    HIPCHECK(hipFree(dx));
    HIPCHECK(hipFree(dy));
    HIPCHECK(hipFree(dc));
    HIPCHECK(hipFree(dtmp));
    HIPCHECK(hipStreamDestroy(s));
    free(x); free(want); free(got); free(y); free(yw); free(w1);
    printf("c abi smoke ok: %d elements, %d chunks, %zu compressed bytes\n", n, p, S);
    return 0;
}
