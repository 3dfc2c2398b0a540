// Standalone timing harness for the int8-MFMA Q4 GEMMs (development tool, not
// part of libbert.so): random Q8 activations and int8 weights at the MiniLM
// shapes, each kernel timed with hipEvents over `iters` launches.
//   build: make build/i8_bench      run: build/i8_bench [iters] [filter]
#include "../embedding.cpp_amd/csrc/gemm_i8.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace bertamd;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static void *dev_bytes(size_t bytes, uint32_t seed, int kind) {
    std::vector<uint8_t> h(bytes);
    uint32_t x = seed * 2654435761u + 1;
    for (size_t i = 0; i < bytes; i++) {
        x = x * 1664525u + 1013904223u;
        h[i] = (uint8_t)(x >> 24);
    }
    if (kind == 1) {  // f32 in [0.5, 1)
        float *p = (float *)h.data();
        for (size_t i = 0; i < bytes / 4; i++) p[i] = 0.5f + (float)(((uint32_t *)h.data())[i] >> 9) * 0x1p-24f;
    } else if (kind == 2) {  // fp16 in [2^-8, 2^-7)
        uint16_t *p = (uint16_t *)h.data();
        for (size_t i = 0; i < bytes / 2; i++) p[i] = (uint16_t)(0x1c00 | (p[i] & 0x3ff));
    } else if (kind == 3) {  // int8 weights in [-8, 7]
        for (size_t i = 0; i < bytes; i++) h[i] = (uint8_t)((int)(h[i] & 15) - 8);
    }
    void *d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
    return d;
}

template <typename F>
static void timeit(const char *name, double flops, int iters, F launch) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; i++) launch();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; i++) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1000.0 / iters;
    printf("%-28s %9.1f us  %7.1f TF/s\n", name, us, flops / us * 1e-6);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const int M = 131072, E = 384, I = 1536, iters = argc > 1 ? atoi(argv[1]) : 20;
    const char *filter = argc > 2 ? argv[2] : "";
    GemmArgs g{};
    g.A.q = dev_bytes((size_t)M * I, 1, 0);
    g.A.d = dev_bytes((size_t)M * (I / 32) * 4, 2, 2);
    g.Wi.q = (const int8_t *)dev_bytes((size_t)I * I, 3, 3);
    g.Wi.d = (const float *)dev_bytes((size_t)I * (I / 32) * 4, 4, 1);
    g.Wi.m = (const float *)dev_bytes((size_t)I * (I / 32) * 4, 5, 1);
    g.Wi.dh = (const uint16_t *)dev_bytes((size_t)I * (I / 32) * 2, 13, 2);
    g.bias = (const float *)dev_bytes((size_t)I * 4, 6, 1);
    g.ln_w = (const float *)dev_bytes((size_t)I * 4, 7, 1);
    g.ln_b = (const float *)dev_bytes((size_t)I * 4, 8, 1);
    g.eps = 1e-12f;
    g.X = (float *)dev_bytes((size_t)M * E * 4, 9, 1);
    g.out_act.q = dev_bytes((size_t)M * I, 10, 0);
    g.out_act.d = dev_bytes((size_t)M * (I / 32) * 4, 11, 0);
    // fp16 GELU table: any 64K table works for timing (the kernel reads [0, 0x8000 + neg_n])
    g.gelu.full = (const uint16_t *)dev_bytes(65536 * 2, 12, 2);
    g.gelu.neg_n = 17706;
    auto want = [&](const char *n) { return !*filter || strstr(n, filter); };
    if (want("up")) {
        GemmArgs a = g;
        a.K = E;
        a.N = I;
        timeit("up_gelu q4_0", 2.0 * M * I * E, iters, [&] { CK(launch_gemm_i8(W_Q4_0, EPI_GELU_ACT, a, M, 0)); });
        timeit("up_gelu q4_1", 2.0 * M * I * E, iters, [&] { CK(launch_gemm_i8(W_Q4_1, EPI_GELU_ACT, a, M, 0)); });
    }
    if (want("o_ln")) {
        GemmArgs a = g;
        a.K = E;
        a.N = E;
        timeit("o_ln q4_0", 2.0 * M * E * E, iters, [&] { CK(launch_gemm_i8(W_Q4_0, EPI_LN, a, M, 0)); });
    }
    if (want("down")) {
        GemmArgs a = g;
        a.K = I;
        a.N = E;
        timeit("down_ln q4_0", 2.0 * M * E * I, iters, [&] { CK(launch_gemm_i8(W_Q4_0, EPI_LN, a, M, 0)); });
        a.N = 256;  // resid kernel: N % 256
        timeit("down_resid(N=256) q4_0", 2.0 * M * 256 * I, iters, [&] { CK(launch_gemm_i8(W_Q4_0, EPI_RESID, a, M, 0)); });
    }
    return 0;
}
