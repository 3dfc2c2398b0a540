// Development timing of the long-sentence attention kernel (not part of
// libbert.so): attention_long_kernel at the C4 / C5 shapes with random
// operands, hipEvent-timed; with -DPHASE_STAMPS (make build/attn_long_stamps)
// also the per-stage cycle medians of one launch (kernels.hip STAMPB slots:
// barrier + commit of the staged chunk, the chunk's key tiles, -> next stage;
// stages 0 .. nch - 1 are pass 1, nch .. 2 nch - 1 pass 2).
//   run: build/attn_long_time [c4|c5] [iters]
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

static void *dev_half(size_t n, uint32_t seed, float amp) {
    std::vector<uint16_t> h(n);
    uint32_t x = seed * 2654435761u + 1;
    for (size_t i = 0; i < n; i++) {
        x = x * 1664525u + 1013904223u;
        h[i] = h16(amp * ((float)(x >> 8) * 0x1p-24f - 0.5f));
    }
    void *d;
    CK(hipMalloc(&d, n * 2));
    CK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
    return d;
}

template <int WT>
static void run(int S, int L, int E, int H, int iters) {
    constexpr int D = 64;
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
    AttnArgs a{};
    a.qk_hi = (const uint16_t *)dev_half((size_t)Mpad * 2 * E, 1, 4.0f);
    a.qk_lo = (const uint16_t *)dev_half((size_t)Mpad * 2 * E, 2, 1e-3f);
    a.ldv = Mpad;
    a.vt_hi = (const uint16_t *)dev_half((size_t)E * Mpad, 3, 2.0f);
    a.vt_lo = (const uint16_t *)dev_half((size_t)E * Mpad, 4, 1e-3f);
    a.offsets = d_off;
    a.E = E;
    a.H = H;
    a.scale = 1.0f / sqrtf((float)D);
    a.expt.compact = d_comp;
    a.expt.pos_n = 1;
    a.expt.neg_n = neg_n;
    a.expt.n_pad = (int)comp.size();
    const size_t act_bytes = WT == W_F16 ? (size_t)Mpad * E * 2 : (size_t)Mpad * E + (size_t)Mpad * (E / 32) * 4;
    void *cq;
    CK(hipMalloc(&cq, act_bytes));
    a.ctx.q = cq;
    a.ctx.d = (char *)cq + (size_t)Mpad * E;
    const dim3 grid((L + ATTN_LONG_QB - 1) / ATTN_LONG_QB, H, S);
    const int nblk = grid.x * grid.y * grid.z;
#ifdef PHASE_STAMPS
    const size_t n_st = (size_t)nblk * STAMP_TILES * 2 * 16;
    unsigned long long *d_st;
    CK(hipMalloc(&d_st, n_st * 8));
    CK(hipMemset(d_st, 0, n_st * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_buf), &d_st, sizeof(d_st)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_nblk), &nblk, sizeof(nblk)));
#endif
    auto launch = [&] {
        hipLaunchKernelGGL((attention_long_kernel<WT, D>), grid, dim3(ATTN_LONG_NW * 64), 0, 0, a);
    };
    for (int i = 0; i < 3; i++) launch();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; i++) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1000.0 / iters, fl = 4.0 * S * (double)L * L * E;
    printf("attention_long S=%d n=%d E=%d H=%d: %8.1f us  %.1f TF/s useful (%.3f of 2516.6)\n", S, L, E, H, us,
           fl / us * 1e-6, fl / us * 1e-6 / 2516.6);
    fflush(stdout);
#ifdef PHASE_STAMPS
    CK(hipMemset(d_st, 0, n_st * 8));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(n_st);
    CK(hipMemcpy(h.data(), d_st, n_st * 8, hipMemcpyDeviceToHost));
    const int nch = (L + ATTN_LONG_NK(64) - 1) / ATTN_LONG_NK(64);
    // per stage: medians over workgroups
    for (int w = 0; w < 2; w++) {
        printf("  wave %s:", w ? "last" : "0   ");
        for (int st = 0; st < 2 * nch; st++) {
            std::vector<double> g0, g1, g2;
            for (int b = 0; b < nblk; b++) {
                const unsigned long long *s = &h[((size_t)(b * STAMP_TILES + st) * 2 + w) * 16];
                const unsigned long long *sn = &h[((size_t)(b * STAMP_TILES + st + 1) * 2 + w) * 16];
                if (s[0] && s[1] > s[0]) g0.push_back((double)(s[1] - s[0]));
                if (s[1] && s[2] > s[1]) g1.push_back((double)(s[2] - s[1]));
                if (st + 1 < 2 * nch && s[2] && sn[0] > s[2]) g2.push_back((double)(sn[0] - s[2]));
            }
            auto med = [](std::vector<double> &v) { std::sort(v.begin(), v.end()); return v.empty() ? 0.0 : v[v.size() / 2]; };
            printf("  [%d] bar %.0f tiles %.0f", st, med(g0), med(g1));
        }
        printf("\n");
    }
    // whole workgroup lifetime (first stamp to last) median
    std::vector<double> life;
    for (int b = 0; b < nblk; b++) {
        const unsigned long long a0 = h[((size_t)(b * STAMP_TILES) * 2) * 16], a1 = h[((size_t)(b * STAMP_TILES + 2 * nch - 1) * 2) * 16 + 2];
        if (a0 && a1 > a0) life.push_back((double)(a1 - a0));
    }
    std::sort(life.begin(), life.end());
    if (!life.empty()) printf("  workgroup lifetime median %.0f cyc\n", life[life.size() / 2]);
#endif
}

int main(int argc, char **argv) {
    const char *cfg = argc > 1 ? argv[1] : "c5";
    const int iters = argc > 2 ? atoi(argv[2]) : 10;
    if (!strcmp(cfg, "c4")) run<W_F16>(512, 256, 768, 12, iters);
    else run<W_Q4_1>(256, 512, 1024, 16, iters);
    return 0;
}
