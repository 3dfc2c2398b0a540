// Development harness (not shipped): the fp6-MFMA Q4_0 GEMMs (gemm_f6.hip)
// against the int8-MFMA ones (gemm_i8.hip) on the same random MiniLM-shape
// inputs: outputs compared (the f6 Q8D output converted back to int8 by the
// library's converter; the FFN-up path is bitwise equal by construction, the
// LayerNorm epilogues sum in a different lane order), then each kernel timed
// with hipEvents over `iters` launches.
//   build: make build/f6_bench      run: build/f6_bench [iters] [filter]
#include "../embedding.cpp_amd/csrc/gemm_i8.hip"
#include "../embedding.cpp_amd/csrc/gemm_f6.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace bertamd;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static uint32_t rng_state = 12345;
static uint32_t rnd() {
    rng_state = rng_state * 1664525u + 1013904223u;
    return rng_state >> 8;
}
static uint16_t f16_in(int lo_exp) { return (uint16_t)(((lo_exp + 15) << 10) | (rnd() & 0x3ff)); }  // [2^e, 2^(e+1))

template <typename T>
static T *up(const std::vector<T> &h) {
    T *d;
    CK(hipMalloc(&d, h.size() * sizeof(T)));
    CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

struct Q4 {  // a random Q4_0 matrix [N][K]: nibbles 0..15 and fp16 d per block
    int N, K;
    std::vector<uint8_t> q;
    std::vector<uint16_t> d;
};

static Q4 rand_q4(int N, int K) {
    Q4 w{N, K, std::vector<uint8_t>((size_t)N * K), std::vector<uint16_t>((size_t)N * (K / 32))};
    for (auto &x : w.q) x = rnd() & 15;
    for (auto &x : w.d) x = f16_in(-8);
    return w;
}

static float h2f_host(uint16_t h) {
    const uint32_t e = (h >> 10) & 31, m = h & 1023;
    float v = e ? std::ldexp(1.0f + m / 1024.0f, (int)e - 15) : std::ldexp((float)m, -24);
    return (h & 0x8000) ? -v : v;
}

static I8W make_i8(const Q4 &w) {  // runtime.cpp upload_i8 layout (Q4_0)
    const int nkb = w.K / 32, nft = w.N / 32;
    auto perm = [](int m) { return 16 * ((m >> 2) & 1) + 4 * (m >> 3) + (m & 3); };
    std::vector<int8_t> q((size_t)w.N * w.K);
    std::vector<float> d((size_t)w.N * nkb);
    std::vector<uint16_t> dh((size_t)w.N * nkb);
    for (int ft = 0; ft < nft; ft++)
        for (int b = 0; b < nkb; b++)
            for (int lane = 0; lane < 64; lane++) {
                const int row = 32 * ft + perm(lane & 31), h = lane >> 5;
                for (int j = 0; j < 16; j++)
                    q[(((size_t)ft * nkb + b) * 64 + lane) * 16 + j] = (int8_t)(w.q[(size_t)row * w.K + 32 * b + 16 * h + j] - 8);
            }
    for (int ft = 0; ft < nft; ft++)
        for (int g = 0; g < nkb / 4; g++)
            for (int m = 0; m < 32; m++)
                for (int jj = 0; jj < 4; jj++) {
                    const int row = 32 * ft + perm(m);
                    const size_t at = (((size_t)ft * (nkb / 4) + g) * 32 + m) * 4 + jj;
                    dh[at] = w.d[(size_t)row * nkb + 4 * g + jj];
                    d[at] = h2f_host(dh[at]);
                }
    I8W r;
    r.q = up(q);
    r.d = up(d);
    r.dh = up(dh);
    return r;
}

static F6W make_f6(const Q4 &w) {  // runtime.cpp upload_f6 layout
    const int nkb = w.K / 32, nft = w.N / 32;
    std::vector<uint32_t> q16((size_t)w.N * nkb * 4), q8((size_t)w.N * nkb * 2), dw((size_t)w.N * nkb);
    for (int ft = 0; ft < nft; ft++)
        for (int b = 0; b < nkb; b++)
            for (int m = 0; m < 32; m++) {
                const int row = 32 * ft + m;
                uint32_t c6[6] = {0, 0, 0, 0, 0, 0};
                for (int e = 0; e < 32; e++) {
                    const int v = (int)w.q[(size_t)row * w.K + 32 * b + e] - 8;
                    const uint32_t code = (v < 0 ? 32u : 0u) | (uint32_t)(v < 0 ? -v : v);
                    const int bit = 6 * q8d_pos(e), wd = bit >> 5, o = bit & 31;
                    c6[wd] |= code << o;
                    if (o > 26) c6[wd + 1] |= code >> (32 - o);
                }
                const size_t i = ((size_t)ft * nkb + b) * 32 + m;
                for (int k = 0; k < 4; k++) q16[i * 4 + k] = c6[k];
                q8[i * 2] = c6[4];
                q8[i * 2 + 1] = c6[5];
            }
    for (int ft = 0; ft < nft; ft++)
        for (int g = 0; g < nkb / 4; g++)
            for (int m = 0; m < 32; m++)
                for (int v = 0; v < 4; v++)
                    dw[(((size_t)ft * (nkb / 4) + g) * 32 + m) * 4 + v] = w.d[(size_t)(32 * ft + m) * nkb + 4 * g + v];
    F6W r;
    r.q16 = (const uint4 *)up(q16);
    r.q8 = (const uint2 *)up(q8);
    r.dw = (const uint4 *)up(dw);
    return r;
}

template <typename F>
static double timeit(int iters, F launch) {
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
    return ms * 1000.0 / iters;
}

// compare the int8 output of the i8 kernel with the f6 kernel's Q8D output
static void compare_act(const char *name, const int8_t *q8, const uint16_t *d8, const void *qd, const uint16_t *dd,
                        int64_t nblk) {
    int8_t *conv;
    CK(hipMalloc(&conv, nblk * 32));
    CK(launch_q8_convert(false, qd, conv, nblk, 0));
    CK(hipDeviceSynchronize());
    std::vector<int8_t> a(nblk * 32), b(nblk * 32);
    std::vector<uint16_t> da(nblk), db(nblk);
    CK(hipMemcpy(a.data(), q8, nblk * 32, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), conv, nblk * 32, hipMemcpyDeviceToHost));
    CK(hipMemcpy(da.data(), d8, nblk * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(db.data(), dd, nblk * 2, hipMemcpyDeviceToHost));
    int64_t nq = 0, nd = 0, maxq = 0;
    for (int64_t i = 0; i < nblk * 32; i++)
        if (a[i] != b[i]) {
            nq++;
            maxq = std::max<int64_t>(maxq, std::abs((int)a[i] - (int)b[i]));
        }
    for (int64_t i = 0; i < nblk; i++) nd += da[i] != db[i];
    printf("%-22s codes differing %lld of %lld (max |dq| %lld), scales differing %lld of %lld\n", name, (long long)nq,
           (long long)(nblk * 32), (long long)maxq, (long long)nd, (long long)nblk);
    CK(hipFree(conv));
}

int main(int argc, char **argv) {
    const int M = 131072, E = 384, I = 1536, iters = argc > 1 ? atoi(argv[1]) : 20;
    const char *filter = argc > 2 ? argv[2] : "";
    auto want = [&](const char *n) { return !*filter || strstr(n, filter); };
    // activations: Q8 [M][I] (the FFN-down input) and [M][E] views of the same codes
    std::vector<int8_t> hq((size_t)M * I);
    std::vector<uint16_t> hd((size_t)M * (I / 32));
    for (auto &x : hq) x = (int8_t)((int)(rnd() % 255) - 127);
    for (auto &x : hd) x = f16_in(-6);
    int8_t *q8 = up(hq);
    uint16_t *d16 = up(hd);
    uint8_t *qd;
    CK(hipMalloc(&qd, (size_t)M * (I / 32) * Q8D_BLK));
    CK(launch_q8_convert(true, q8, qd, (int64_t)M * (I / 32), 0));
    // round trip of the converters
    {
        int8_t *back;
        CK(hipMalloc(&back, (size_t)M * I));
        CK(launch_q8_convert(false, qd, back, (int64_t)M * (I / 32), 0));
        std::vector<int8_t> hb((size_t)M * I);
        CK(hipMemcpy(hb.data(), back, hb.size(), hipMemcpyDeviceToHost));
        printf("q8 -> q8d -> q8 round trip: %s\n", memcmp(hb.data(), hq.data(), hb.size()) ? "MISMATCH" : "exact");
        CK(hipFree(back));
    }
    std::vector<uint16_t> tab(65536);
    for (int i = 0; i < 65536; i++) tab[i] = f16_in(-3);  // any finite table serves for equality and timing
    const uint16_t *gtab = up(tab);
    std::vector<float> bias(I), lw(E), lb(E);
    for (auto &x : bias) x = h2f_host(f16_in(-4)) * ((rnd() & 1) ? 1 : -1);
    for (auto &x : lw) x = 1.0f + h2f_host(f16_in(-5));
    for (auto &x : lb) x = h2f_host(f16_in(-6));
    const float *dbias = up(bias), *dlw = up(lw), *dlb = up(lb);
    std::vector<float> hx((size_t)M * E);
    for (auto &x : hx) x = h2f_host(f16_in(-1)) * ((rnd() & 1) ? 1 : -1);

    if (want("up")) {
        const Q4 w = rand_q4(I, E);
        GemmArgs a{};
        a.K = E;
        a.N = I;
        a.Wi = make_i8(w);
        a.Wf = make_f6(w);
        a.bias = dbias;
        a.gelu.full = gtab;
        a.gelu.neg_n = 17706;
        int8_t *u8;
        uint16_t *ud8, *udd;
        uint8_t *ud;
        CK(hipMalloc(&u8, (size_t)M * I));
        CK(hipMalloc(&ud8, (size_t)M * (I / 32) * 2));
        CK(hipMalloc(&ud, (size_t)M * (I / 32) * Q8D_BLK));
        CK(hipMalloc(&udd, (size_t)M * (I / 32) * 2));
        GemmArgs a8 = a, af = a;
        // A: the first E columns' worth of blocks of each row -> use [M][E] tensors
        int8_t *q8e;
        uint16_t *d16e;
        uint8_t *qde;
        CK(hipMalloc(&q8e, (size_t)M * E));
        CK(hipMalloc(&d16e, (size_t)M * (E / 32) * 2));
        CK(hipMalloc(&qde, (size_t)M * (E / 32) * Q8D_BLK));
        CK(hipMemcpy2D(q8e, E, q8, I, E, M, hipMemcpyDeviceToDevice));
        CK(hipMemcpy2D(d16e, E / 16, d16, I / 16, E / 16, M, hipMemcpyDeviceToDevice));
        CK(launch_q8_convert(true, q8e, qde, (int64_t)M * (E / 32), 0));
        a8.A.q = q8e;
        a8.A.d = d16e;
        a8.out_act.q = u8;
        a8.out_act.d = ud8;
        af.A.q = qde;
        af.A.d = d16e;
        af.out_act.q = ud;
        af.out_act.d = udd;
        CK(launch_gemm_i8(W_Q4_0, EPI_GELU_ACT, a8, M, 0));
        CK(launch_gemm_f6(EPI_GELU_ACT, af, M, 0));
        CK(hipDeviceSynchronize());
        compare_act("up_gelu (i8 vs f6)", u8, ud8, ud, udd, (int64_t)M * (I / 32));
        const double fl = 2.0 * M * I * E;
        const double t8 = timeit(iters, [&] { CK(launch_gemm_i8(W_Q4_0, EPI_GELU_ACT, a8, M, 0)); });
        const double tf = timeit(iters, [&] { CK(launch_gemm_f6(EPI_GELU_ACT, af, M, 0)); });
        printf("up_gelu  i8 %8.1f us %6.1f TOPS | f6 %8.1f us %6.1f TOPS\n", t8, fl / t8 * 1e-6, tf, fl / tf * 1e-6);
        fflush(stdout);
    }
    for (int pass = 0; pass < 2; pass++) {
        const char *nm = pass ? "o_ln" : "down_ln";
        if (!want(nm)) continue;
        const int K = pass ? E : I;
        const Q4 w = rand_q4(E, K);
        GemmArgs a{};
        a.K = K;
        a.N = E;
        a.Wi = make_i8(w);
        a.Wf = make_f6(w);
        a.bias = dbias;
        a.ln_w = dlw;
        a.ln_b = dlb;
        a.eps = 1e-12f;
        float *x8 = up(hx), *xf = up(hx);
        int8_t *o8;
        uint16_t *od8, *odd;
        uint8_t *od;
        CK(hipMalloc(&o8, (size_t)M * E));
        CK(hipMalloc(&od8, (size_t)M * (E / 32) * 2));
        CK(hipMalloc(&od, (size_t)M * (E / 32) * Q8D_BLK));
        CK(hipMalloc(&odd, (size_t)M * (E / 32) * 2));
        int8_t *qk8 = q8;
        uint16_t *dk = d16;
        uint8_t *qkd = qd;
        if (pass) {  // [M][E] activations
            CK(hipMalloc(&qk8, (size_t)M * E));
            CK(hipMalloc(&dk, (size_t)M * (E / 32) * 2));
            CK(hipMalloc(&qkd, (size_t)M * (E / 32) * Q8D_BLK));
            CK(hipMemcpy2D(qk8, E, q8, I, E, M, hipMemcpyDeviceToDevice));
            CK(hipMemcpy2D(dk, E / 16, d16, I / 16, E / 16, M, hipMemcpyDeviceToDevice));
            CK(launch_q8_convert(true, qk8, qkd, (int64_t)M * (E / 32), 0));
        }
        GemmArgs a8 = a, af = a;
        a8.A.q = qk8;
        a8.A.d = dk;
        a8.X = x8;
        a8.out_act.q = o8;
        a8.out_act.d = od8;
        af.A.q = qkd;
        af.A.d = dk;
        af.X = xf;
        af.out_act.q = od;
        af.out_act.d = odd;
        CK(launch_gemm_i8(W_Q4_0, EPI_LN, a8, M, 0));
        CK(launch_gemm_f6(EPI_LN, af, M, 0));
        CK(hipDeviceSynchronize());
        compare_act(pass ? "o_ln (i8 vs f6)" : "down_ln (i8 vs f6)", o8, od8, od, odd, (int64_t)M * (E / 32));
        {
            std::vector<float> ha((size_t)M * E), hb((size_t)M * E);
            CK(hipMemcpy(ha.data(), x8, ha.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hb.data(), xf, hb.size() * 4, hipMemcpyDeviceToHost));
            int64_t n = 0;
            double mx = 0;
            for (size_t i = 0; i < ha.size(); i++)
                if (ha[i] != hb[i]) {
                    n++;
                    mx = std::max(mx, (double)std::fabs(ha[i] - hb[i]));
                }
            printf("%-22s X differing %lld of %zu (max |dx| %.3g)\n", nm, (long long)n, ha.size(), mx);
        }
        const double fl = 2.0 * M * E * K;
        const double t8 = timeit(iters, [&] { CK(launch_gemm_i8(W_Q4_0, EPI_LN, a8, M, 0)); });
        const double tf = timeit(iters, [&] { CK(launch_gemm_f6(EPI_LN, af, M, 0)); });
        printf("%-8s i8 %8.1f us %6.1f TOPS | f6 %8.1f us %6.1f TOPS\n", nm, t8, fl / t8 * 1e-6, tf, fl / tf * 1e-6);
        fflush(stdout);
    }
    return 0;
}
