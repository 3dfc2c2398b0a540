// Development check of the fused QKV + attention kernel's head-pair grouping
// (not part of libbert.so): the same F16 sentence batch through
// qkv_attention_kernel<W_F16, 1> (one head pair per main loop, plain tile
// order) and <W_F16, 2> (two pairs per main loop, grouped tile order, as
// runtime.cpp packs it), context outputs compared element by element, and
// the differences located by (head, row, dim).
//   build: make build/qkva_check      run: build/qkva_check
#include "../embedding.cpp_amd/csrc/kernels.hip"

#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace bertamd;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static uint16_t h16(float f) { _Float16 h = (_Float16)f; uint16_t u; std::memcpy(&u, &h, 2); return u; }
static float f16(uint16_t u) { _Float16 h; std::memcpy(&h, &u, 2); return (float)h; }

template <typename T>
static T *up(const std::vector<T> &v) {
    T *d;
    CK(hipMalloc(&d, v.size() * sizeof(T) + 16));
    CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

// fragment order of kernels.h WPtr (F16): tile j, block kb, lane: 8 halves of
// feature 16 j + (lane & 15), k = 32 kb + 8 (lane >> 4) ..; tile T of the
// packed copy holds source tile src(T) (runtime.cpp grouped order)
static std::vector<uint16_t> pack(const std::vector<float> &W, int N, int K, int G) {
    const int tpp = 12, nkb = K / 32;
    std::vector<uint16_t> out((size_t)N * K);
    for (int T = 0; T < N / 16; T++) {
        const int src = tpp * (G * (T / (G * tpp)) + T % G) + (T % (G * tpp)) / G;
        for (int kb = 0; kb < nkb; kb++)
            for (int lane = 0; lane < 64; lane++)
                for (int j = 0; j < 8; j++)
                    out[(((size_t)T * nkb + kb) * 64 + lane) * 8 + j] =
                        h16(W[(size_t)(16 * src + (lane & 15)) * K + 32 * kb + 8 * (lane >> 4) + j]);
    }
    return out;
}

int main() {
    const int E = 384, H = 12, D = 32, S = 8;
    std::vector<int32_t> offs(S + 1, 0);
    const int lens[S] = {128, 128, 77, 128, 1, 100, 128, 33};
    for (int s = 0; s < S; s++) offs[s + 1] = offs[s] + lens[s];
    const int M = offs[S], Mpad = (M + 127) / 128 * 128 + 128;
    uint32_t x = 12345;
    auto rnd = [&]() {  // ~N(0,1) via sum of uniforms
        float a = 0;
        for (int i = 0; i < 4; i++) { x = x * 1664525u + 1013904223u; a += (x >> 8) * (1.0f / 16777216.0f); }
        return (a - 2.0f) * 1.7320508f;
    };
    std::vector<uint16_t> xa((size_t)Mpad * E, 0);
    for (int i = 0; i < M * E; i++) xa[i] = h16(rnd());
    std::vector<float> W((size_t)3 * E * E), bias(3 * E);
    for (auto &w : W) w = 0.05f * rnd();
    for (auto &b : bias) b = 0.01f * rnd();
    // ggml's exp table, compact LDS view (runtime.cpp compact_table with pos_n = 1)
    std::vector<uint16_t> full(65536);
    for (int i = 0; i < 65536; i++) full[i] = h16(expf(f16((uint16_t)i)));
    const uint16_t nc = full[0xfbff];
    int neg_n = 0x7c00;
    while (neg_n > 0 && full[0x8000 | (neg_n - 1)] == nc) neg_n--;
    std::vector<uint16_t> comp((size_t)(1 + neg_n + 1 + 7) / 8 * 8, 0);
    comp[0] = full[0];
    for (int m = 0; m < neg_n; m++) comp[1 + m] = full[0x8000 | m];
    comp[1 + neg_n] = nc;

    GemmArgs g{};
    g.A.q = up(xa);
    g.K = E;
    g.N = 3 * E;
    g.bias = up(bias);
    g.head_dim = D;
    AttnArgs a{};
    a.offsets = up(offs);
    a.E = E;
    a.H = H;
    a.scale = 1.0f / sqrtf((float)D);
    a.expt.compact = up(comp);
    a.expt.pos_n = 1;
    a.expt.neg_n = neg_n;
    a.expt.n_pad = (int)comp.size();
    std::vector<std::vector<uint16_t>> out(2);
    for (int G = 1; G <= 2; G++) {
        g.W.q = up(pack(W, 3 * E, E, G));
        uint16_t *ctx;
        CK(hipMalloc(&ctx, (size_t)Mpad * E * 2));
        CK(hipMemset(ctx, 0xff, (size_t)Mpad * E * 2));
        a.ctx.q = ctx;
        if (G == 1)
            hipLaunchKernelGGL((qkv_attention_kernel<W_F16, 32, 1, false>), dim3(S), dim3(QKVA_NW * 64), 0, 0, g, a);
        else
            hipLaunchKernelGGL((qkv_attention_kernel<W_F16, 32, 2, false>), dim3(S), dim3(QKVA_NW * 64), 0, 0, g, a);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        out[G - 1].resize((size_t)M * E);
        CK(hipMemcpy(out[G - 1].data(), ctx, (size_t)M * E * 2, hipMemcpyDeviceToHost));
    }
    // locate the differences
    long nd = 0;
    double maxd = 0;
    std::vector<long> by_head(H, 0), by_dim(D, 0), by_row16(8, 0), by_sent(S, 0);
    for (int s = 0; s < S; s++)
        for (int r = offs[s]; r < offs[s + 1]; r++)
            for (int c = 0; c < E; c++) {
                const float u = f16(out[0][(size_t)r * E + c]), v = f16(out[1][(size_t)r * E + c]);
                if (u != v) {
                    nd++;
                    maxd = std::max(maxd, (double)fabsf(u - v) / (fabsf(u) + 1e-3));
                    by_head[c / D]++;
                    by_dim[c % D]++;
                    by_row16[((r - offs[s]) / 16) % 8]++;
                    by_sent[s]++;
                }
            }
    printf("elements differing: %ld of %ld (max rel %.3g)\n", nd, (long)M * E, maxd);
    printf("by head:");
    for (int h = 0; h < H; h++) printf(" %ld", by_head[h]);
    printf("\nby dim:");
    for (int d = 0; d < D; d++) printf(" %ld", by_dim[d]);
    printf("\nby 16-row group:");
    for (int i = 0; i < 8; i++) printf(" %ld", by_row16[i]);
    printf("\nby sentence:");
    for (int s = 0; s < S; s++) printf(" %ld", by_sent[s]);
    printf("\nsample ctx[0][0..7] G1 vs G2:");
    for (int c = 0; c < 8; c++) printf(" %.5f/%.5f", f16(out[0][c]), f16(out[1][c]));
    printf("\n");
    return 0;
}
