// Probe (development tool): semantics of gfx950's v_cvt_scalef32_2xpk16_fp6_f32
// as the Q8D producers use it (kernels_common.h q8d_codes16): two vectors of
// 16 f32 integer digits in [-16, 16] and a scale, one instruction, 6 dwords
// of e2m3 codes.  Checks, against the sign-magnitude codes the fp6 GEMMs
// expect (code = sign << 5 | |v| under the MFMA's 2^3 scale):
//   (1) which scale gives code(v) = sign << 5 | |v| (dst = src / scale or src * scale),
//   (2) the packing order (a[i] at bits 6i, b[i] at bits 96 + 6i),
//   (3) every digit value -16..16 in every slot.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float float16v __attribute__((ext_vector_type(16)));
typedef int int6v __attribute__((ext_vector_type(6)));

__global__ void probe(const float *in, float scale, int *out) {
    const int l = threadIdx.x;
    float16v a, b;
    for (int i = 0; i < 16; i++) {
        a[i] = in[(l * 32 + i) % 33];
        b[i] = in[(l * 32 + 16 + i) % 33];
    }
    const int6v r = __builtin_amdgcn_cvt_scalef32_2xpk16_fp6_f32(a, b, scale);
    for (int k = 0; k < 6; k++) out[l * 6 + k] = r[k];
}

int main() {
    float h_in[33];
    for (int i = 0; i < 33; i++) h_in[i] = (float)(i - 16);
    h_in[16] = -0.0f;  // negative zero in one slot
    float *d_in;
    int *d_out;
    hipMalloc(&d_in, sizeof h_in);
    hipMalloc(&d_out, 64 * 6 * 4);
    hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice);
    int bad_all = 0;
    for (float scale : {8.0f, 0.125f, 1.0f}) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_in, scale, d_out);
        int h_out[64 * 6];
        hipMemcpy(h_out, d_out, sizeof h_out, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; l++)
            for (int j = 0; j < 32; j++) {
                const float v = h_in[(l * 32 + j) % 33];
                const int iv = (int)v, m = iv < 0 ? -iv : iv;
                const unsigned want = ((v < 0 || (v == 0 && 1.0f / v < 0)) ? 32u : 0u) | (unsigned)m;
                const int bit = 6 * j, w = bit >> 5, o = bit & 31;
                unsigned long long two = (unsigned)h_out[l * 6 + w];
                if (w + 1 < 6) two |= (unsigned long long)(unsigned)h_out[l * 6 + w + 1] << 32;
                const unsigned got = (unsigned)(two >> o) & 63u;
                if (got != want) {
                    if (bad < 6) printf("scale %g lane %d slot %d value %g: got %u want %u\n", scale, l, j, v, got, want);
                    bad++;
                }
            }
        printf("scale %g: %d mismatches of %d\n", scale, bad, 64 * 32);
        if (scale == 8.0f || scale == 0.125f) bad_all += bad == 0 ? 0 : 1;
    }
    printf(bad_all < 2 ? "OK (one scale convention matches)\n" : "FAIL\n");
    return 0;
}
