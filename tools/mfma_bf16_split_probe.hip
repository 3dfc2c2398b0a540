// Probe (development): does one v_mfma_f32_32x32x16_bf16 return the correctly
// rounded product of an fp16 d_w and an f32 d_a when they are fed as bf16
// parts (d_w = w0 + w1, d_a = a0 + a1 + a2: six exact partial products in one
// MFMA), i.e. RN(d_w * d_a) — and RN(c + d_w * d_a) with an accumulator c?
// If so, Q4_1's per-block d_w * d_a and m_w * s_a (f32 x f32 today, on the
// 64-cycle f32 MFMA) can run on the 32-cycle bf16 MFMA bit for bit.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_bf16_split_probe.hip -o build/mfma_bf16_split_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ __bf16 tobf(float x) { return __builtin_bit_cast(__bf16, (uint16_t)(__float_as_uint(x) >> 16)); }

// bf16 parts by truncation: x = p0 + p1 + p2 exactly when x has <= 24 significant bits
__device__ __forceinline__ void split3(float x, float &p0, float &p1, float &p2) {
    p0 = __uint_as_float(__float_as_uint(x) & 0xffff0000u);
    const float r = x - p0;  // exact
    p1 = __uint_as_float(__float_as_uint(r) & 0xffff0000u);
    p2 = r - p1;             // exact, <= 8 significant bits
}

// one wave per 32 x 32 tile: row i of A = d_w[i] parts, column j of B = d_a[j] parts
__global__ void probe(const float *dw, const float *da, const float *c, float *out, int tiles) {
    const int t = blockIdx.x;
    if (t >= tiles) return;
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    float w0, w1, w2, a0, a1, a2;
    split3(dw[t * 32 + r], w0, w1, w2);  // fp16 values: w2 == 0
    split3(da[t * 32 + r], a0, a1, a2);
    bf16x8 A, B;
    for (int k = 0; k < 8; k++) { A[k] = tobf(0.f); B[k] = tobf(0.f); }
    if (h == 0) {  // k = 0..7 from lanes 0-31; k = 8..15 (lanes 32-63) stay zero
        const float av[6] = {w0, w0, w0, w1, w1, w1}, bv[6] = {a0, a1, a2, a0, a1, a2};
        for (int k = 0; k < 6; k++) { A[k] = tobf(av[k]); B[k] = tobf(bv[k]); }
    }
    f32x16 acc;
    for (int i = 0; i < 16; i++) acc[i] = c ? c[(t * 64 + l) * 16 + i] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, acc, 0, 0, 0);
    for (int i = 0; i < 16; i++) out[(t * 64 + l) * 16 + i] = acc[i];
}

static uint32_t rng(uint64_t &s) { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 32); }

int main(int argc, char **argv) {
    const int tiles = argc > 1 ? atoi(argv[1]) : 65536;
    std::vector<float> dw(tiles * 32), da(tiles * 32), c(tiles * 64 * 16), out(tiles * 64 * 16);
    uint64_t s = 12345;
    for (size_t i = 0; i < dw.size(); i++) {
        // d_w: a positive normal fp16 value (ggml block scale), d_a: any positive f32 (amax / 127)
        const uint16_t hb = (uint16_t)(0x0400 + rng(s) % (0x7800 - 0x0400));
        _Float16 hv; std::memcpy(&hv, &hb, 2);
        dw[i] = (float)hv;
        da[i] = std::ldexp(1.0f + (rng(s) & 0x7fffff) * 0x1p-23f, -(int)(rng(s) % 30));
    }
    for (size_t i = 0; i < c.size(); i++) c[i] = std::ldexp((float)(int32_t)rng(s) * 0x1p-31f, -(int)(rng(s) % 24));
    float *d_dw, *d_da, *d_c, *d_out;
    CK(hipMalloc(&d_dw, dw.size() * 4)); CK(hipMalloc(&d_da, da.size() * 4));
    CK(hipMalloc(&d_c, c.size() * 4)); CK(hipMalloc(&d_out, out.size() * 4));
    CK(hipMemcpy(d_dw, dw.data(), dw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_da, da.data(), da.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_c, c.data(), c.size() * 4, hipMemcpyHostToDevice));
    for (int withc = 0; withc < 2; withc++) {
        hipLaunchKernelGGL(probe, dim3(tiles), dim3(64), 0, 0, d_dw, d_da, withc ? d_c : nullptr, d_out, tiles);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(out.data(), d_out, out.size() * 4, hipMemcpyDeviceToHost));
        size_t bad = 0, n = 0;
        for (int t = 0; t < tiles; t++)
            for (int l = 0; l < 64; l++)
                for (int i = 0; i < 16; i++) {
                    const int row = 8 * (i / 4) + 4 * (l >> 5) + (i % 4), col = l & 31;
                    const float cv = withc ? c[(t * 64 + l) * 16 + i] : 0.f;
                    // reference: RN(c + d_w * d_a); the product is exact in double, fma rounds once
                    const float ref = std::fmaf(dw[t * 32 + row], da[t * 32 + col], cv);
                    const float got = out[(t * 64 + l) * 16 + i];
                    n++;
                    if (std::memcmp(&ref, &got, 4)) {
                        if (bad < 5) printf("  mismatch: dw %a da %a c %a -> mfma %a ref %a\n", dw[t * 32 + row], da[t * 32 + col], cv, got, ref);
                        bad++;
                    }
                }
        printf("%s: %zu of %zu outputs differ from RN(%sd_w * d_a)\n", withc ? "with accumulator" : "product alone", bad, n,
               withc ? "c + " : "");
    }
    return 0;
}
