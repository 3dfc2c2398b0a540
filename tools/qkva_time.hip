// Development timing of the fused QKV + attention kernel's phases (not part of
// libbert.so): qkv_attention_kernel<Q4_0, 2> at the C3 shape (1024 sentences x
// 128 tokens, MiniLM), random operands, timed with hipEvents as shipped (K =
// 384) and with the GEMM main loop emptied (K = 0: the attention phase, the
// tile epilogues and the fixed per-workgroup costs only).
//   build: make build/qkva_time      run: build/qkva_time [iters]
// With -DPHASE_STAMPS (make build/qkva_stamps) it also prints the per-phase
// cycle medians of one launch (kernels.hip STAMP slots: main loop, hi/lo split
// into the attention tiles + barrier, attention + barrier, per head pair).
#include "../embedding.cpp_amd/csrc/kernels.hip"
#ifdef PHASE_STAMPS
#include "stamps.h"
#endif

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace bertamd;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static uint16_t h16(float f) { _Float16 h = (_Float16)f; uint16_t u; std::memcpy(&u, &h, 2); return u; }
static float f16(uint16_t u) { _Float16 h; std::memcpy(&h, &u, 2); return (float)h; }

static void *dev_random(size_t bytes, uint32_t seed, int kind) {
    std::vector<uint8_t> h(bytes);
    uint32_t x = seed * 2654435761u + 1;
    for (size_t i = 0; i < bytes; i++) {
        x = x * 1664525u + 1013904223u;
        h[i] = (uint8_t)(x >> 24);
    }
    if (kind == 1) {  // fp16 in a modest range
        uint16_t *p = (uint16_t *)h.data();
        for (size_t i = 0; i < bytes / 2; i++) p[i] = (uint16_t)((p[i] & 0x83ff) | 0x2000);
    }
    void *d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char **argv) {
    const int S = 1024, L = 128, E = 384, H = 12, D = 32, iters = argc > 1 ? atoi(argv[1]) : 20;
    const int M = S * L, Mpad = M + 128;
    std::vector<int32_t> offs(S + 1);
    for (int s = 0; s <= S; s++) offs[s] = s * L;
    int32_t *d_off;
    CK(hipMalloc(&d_off, offs.size() * 4));
    CK(hipMemcpy(d_off, offs.data(), offs.size() * 4, hipMemcpyHostToDevice));
    std::vector<uint16_t> full(65536);
    for (int i = 0; i < 65536; i++) full[i] = h16(expf(f16((uint16_t)i)));
    const uint16_t nc = full[0xfbff];
    int neg_n = 0x7c00;
    while (neg_n > 0 && full[0x8000 | (neg_n - 1)] == nc) neg_n--;
    std::vector<uint16_t> comp((size_t)(1 + neg_n + 1 + 7) / 8 * 8, 0);
    comp[0] = full[0];
    for (int m = 0; m < neg_n; m++) comp[1 + m] = full[0x8000 | m];
    comp[1 + neg_n] = nc;
    uint16_t *d_comp;
    CK(hipMalloc(&d_comp, comp.size() * 2));
    CK(hipMemcpy(d_comp, comp.data(), comp.size() * 2, hipMemcpyHostToDevice));

    GemmArgs g{};
    // Q8 activations: random codes in [-127, 127], fp16 block scales near 0.02
    // (a realistic score spread for the softmax; constant inputs make every
    // exp-table read one address)
    {
        std::vector<int8_t> q((size_t)Mpad * E);
        uint32_t x = 12345;
        for (auto &v : q) {
            x = x * 1664525u + 1013904223u;
            v = (int8_t)((int)((x >> 24) % 255) - 127);
        }
        void *aq;
        CK(hipMalloc(&aq, q.size()));
        CK(hipMemcpy(aq, q.data(), q.size(), hipMemcpyHostToDevice));
        g.A.q = aq;
        std::vector<uint16_t> d((size_t)Mpad * (E / 32));
        for (auto &v : d) {
            x = x * 1664525u + 1013904223u;
            v = h16(0.01f + 0.02f * (float)(x >> 8) * 0x1p-24f);
        }
        void *ad;
        CK(hipMalloc(&ad, d.size() * 2));
        CK(hipMemcpy(ad, d.data(), d.size() * 2, hipMemcpyHostToDevice));
        g.A.d = ad;
    }
    g.W.q = dev_random((size_t)3 * E * E * 4, 3, 1);
    g.W.unscale = 1.0f / 16384;
    g.bias = (const float *)dev_random((size_t)3 * E * 4, 4, 0);
    CK(hipMemset((void *)g.bias, 0, (size_t)3 * E * 4));
    g.K = E;
    g.N = 3 * E;
    g.head_dim = D;
    // the producer / consumer kernel's int8 QKV weights (codes in [-8, 7], fp16 block scales)
    {
        std::vector<int8_t> wq((size_t)3 * E * E);
        uint32_t x = 77;
        for (auto &v : wq) {
            x = x * 1664525u + 1013904223u;
            v = (int8_t)((int)((x >> 24) & 15) - 8);
        }
        void *dq;
        CK(hipMalloc(&dq, wq.size()));
        CK(hipMemcpy(dq, wq.data(), wq.size(), hipMemcpyHostToDevice));
        g.Wi.q = (const int8_t *)dq;
        std::vector<uint16_t> dh((size_t)3 * E * (E / 32));
        for (auto &v : dh) {
            x = x * 1664525u + 1013904223u;
            v = h16(0.005f + 0.01f * (float)(x >> 8) * 0x1p-24f);
        }
        void *dd;
        CK(hipMalloc(&dd, dh.size() * 2));
        CK(hipMemcpy(dd, dh.data(), dh.size() * 2, hipMemcpyHostToDevice));
        g.Wi.dh = (const uint16_t *)dd;
    }
    AttnArgs a{};
    a.offsets = d_off;
    a.E = E;
    a.H = H;
    a.scale = 1.0f / sqrtf((float)D);
    a.expt.compact = d_comp;
    a.expt.pos_n = 1;
    a.expt.neg_n = neg_n;
    a.expt.n_pad = (int)comp.size();
    void *cq, *cd;
    CK(hipMalloc(&cq, (size_t)Mpad * E));
    CK(hipMalloc(&cd, (size_t)Mpad * (E / 32) * 4));
    a.ctx.q = cq;
    a.ctx.d = cd;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
#ifdef PHASE_STAMPS
    // every launch of a stamped kernel writes the buffer: set it before the first one
    const size_t n_st = (size_t)S * STAMP_TILES * 2 * 16;
    unsigned long long *d_st;
    CK(hipMalloc(&d_st, n_st * 8));
    CK(hipMemset(d_st, 0, n_st * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_buf), &d_st, sizeof(d_st)));
    { const int nb = S; CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_nblk), &nb, sizeof(nb))); }
#endif
    const bool pc = argc > 2 && !strcmp(argv[2], "pc");  // the producer / consumer kernel
    for (int K : {E, 0}) {
        if (pc && K == 0) break;
        g.K = K;
        auto launch = [&] {
            if (pc)
                hipLaunchKernelGGL((qkv_attention_pc_kernel<false>), dim3(S), dim3(QKPC_NW * 64), 0, 0, g, a);
            else
                hipLaunchKernelGGL((qkv_attention_kernel<W_Q4_0, 32, 2, false>), dim3(S), dim3(QKVA_NW * 64), 0, 0, g, a);
        };
        for (int i = 0; i < 3; i++) launch();
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; i++) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("qkv_attention%s q4_0 K=%d: %8.1f us\n", pc ? "_pc" : "", K, ms * 1000.0 / iters);
        fflush(stdout);
#ifdef PHASE_STAMPS
        if (K == E) {
            CK(hipMemset(d_st, 0, n_st * 8));
            launch();
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> h(n_st);
            CK(hipMemcpy(h.data(), d_st, n_st * 8, hipMemcpyDeviceToHost));
            if (pc) {
                const char *names[] = {"main|attn", "split|store", "->period"};
                stamp_report(h, S, STAMP_TILES, 3, names, ms * 1000.0 / iters);
            } else {
                const char *names[] = {"main", "split0", "attn0", "split1", "attn1", "->quad"};
                stamp_report(h, S, STAMP_TILES, 6, names, ms * 1000.0 / iters);
            }
        }
#endif
    }
    return 0;
}
