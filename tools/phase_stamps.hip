// Per-phase timing of the persistent int8 GEMMs (development tool, not part
// of libbert.so): gemm_i8.hip compiled with -DPHASE_STAMPS, so lane 0 of the
// first and last wave of every workgroup stamps s_memtime at the phase
// boundaries of each tile (gemm_i8.hip STAMP slots).  Inputs as tools/i8_bench
// (random Q8 activations / int8 weights at the MiniLM shapes, M = 131072).
//   build: make build/phase_stamps     run: build/phase_stamps [up|down|o]
#define PHASE_STAMPS 1
#include "../embedding.cpp_amd/csrc/gemm_i8.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "stamps.h"

using namespace bertamd;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static void *dev_bytes(size_t bytes, uint32_t seed, int kind) {
    std::vector<uint8_t> h(bytes);
    uint32_t x = seed * 2654435761u + 1;
    for (size_t i = 0; i < bytes; i++) {
        x = x * 1664525u + 1013904223u;
        h[i] = (uint8_t)(x >> 24);
    }
    if (kind == 1) {
        float *p = (float *)h.data();
        for (size_t i = 0; i < bytes / 4; i++) p[i] = 0.5f + (float)(((uint32_t *)h.data())[i] >> 9) * 0x1p-24f;
    } else if (kind == 2) {
        uint16_t *p = (uint16_t *)h.data();
        for (size_t i = 0; i < bytes / 2; i++) p[i] = (uint16_t)(0x1c00 | (p[i] & 0x3ff));
    } else if (kind == 3) {
        for (size_t i = 0; i < bytes; i++) h[i] = (uint8_t)((int)(h[i] & 15) - 8);
    }
    void *d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
    return d;
}

template <typename F>
static void run(const char *name, int nslots, const char **slot_names, F launch) {
    const int NWG = 256;
    const size_t n = (size_t)NWG * STAMP_TILES * 2 * 16;
    unsigned long long *d;
    CK(hipMalloc(&d, n * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_buf), &d, sizeof(d)));
    { const int nb = NWG; CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_nblk), &nb, sizeof(nb))); }
    for (int i = 0; i < 5; i++) launch();  // warm (clock up)
    CK(hipMemset(d, 0, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(n);
    CK(hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost));
    printf("%s:\n", name);
    stamp_report(h, NWG, STAMP_TILES, nslots, slot_names, ms * 1000.0);
    CK(hipFree(d));
}

int main(int argc, char **argv) {
    const int M = 131072, E = 384, I = 1536;
    const char *filter = argc > 1 ? argv[1] : "";
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
    g.gelu.full = (const uint16_t *)dev_bytes(65536 * 2, 12, 2);
    g.gelu.neg_n = 17706;
    auto want = [&](const char *n) { return !*filter || strstr(n, filter); };
    if (want("up")) {
        GemmArgs a = g;
        a.K = E;
        a.N = I;
        const char *sl[] = {"main", "epi", "->next"};
        run("up_gelu q4_0", 3, sl, [&] { CK(launch_gemm_i8(W_Q4_0, EPI_GELU_ACT, a, M, 0)); });
    }
    const char *sl[] = {"main", "dma+bar", "sum+bar", "var+bar", "ln+q8", "bar", "xstore", "->next"};
    if (want("down")) {
        GemmArgs a = g;
        a.K = I;
        a.N = E;
        run("down_ln q4_0", 8, sl, [&] { CK(launch_gemm_i8(W_Q4_0, EPI_LN, a, M, 0)); });
    }
    if (want("o")) {
        GemmArgs a = g;
        a.K = E;
        a.N = E;
        run("o_ln q4_0 (int8)", 8, sl, [&] { CK(launch_gemm_i8(W_Q4_0, EPI_LN, a, M, 0)); });
    }
    return 0;
}
