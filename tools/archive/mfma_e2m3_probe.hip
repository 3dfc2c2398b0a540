// Probe (development tool): the block-scaled f8f6f4 MFMA with fp6 e2m3
// operands as an exact integer dot product, in the encoding the Q4_0 GEMMs
// use (gemm_q4.hip):
//   e2m3 under an E8M0 scale of 2^3 holds every integer v in [-16, 16] with the
//   code sign << 5 | |v| (|v| < 8: subnormals m/8; 8..15: exponent 1; 16:
//   exponent 2), so
//   - a Q4_0 weight q - 8 in [-8, 7] is its sign-magnitude code, scale 2^3;
//   - a Q8 activation q in [-127, 127] splits by magnitude, |q| = 16 H + L,
//     into two digits sharing q's sign: H (lanes 0-31, scale 2^7 = 16 * 2^3)
//     and L (lanes 32-63, scale 2^3), against the same weights in both lane
//     halves;
//   one v_mfma_scale_f32_32x32x64_f8f6f4 then returns the block's exact isum
//   sum_j q_j (q_w,j - 8) in f32.
// Checks the exact result on random and extreme codes, and the element order
// (element j at bits 6j .. 6j + 5 of the lane's 6 dwords, LSB first).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int int8v __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));

__device__ inline unsigned sm_code(int v) { return (v < 0 ? 32u : 0u) | (unsigned)(v < 0 ? -v : v); }

__device__ inline int8v pack6(const unsigned *c) {  // 32 codes -> 6 dwords, LSB first
    int8v r = {};
    for (int j = 0; j < 32; j++) {
        const int bit = 6 * j, w = bit >> 5, o = bit & 31;
        r[w] |= (int)(c[j] << o);
        if (o > 26) r[w + 1] |= (int)(c[j] >> (32 - o));
    }
    return r;
}

// A: q8 activations [32 tokens][32]; W: q4 codes [32 features][32] in [0, 15]
__global__ void probe(const signed char *A, const unsigned char *W, float *C) {
    const int l = threadIdx.x, r = l & 31, hh = l >> 5;
    unsigned ca[32], cw[32];
    for (int j = 0; j < 32; j++) {
        const int q = A[r * 32 + j], m = q < 0 ? -q : q;
        const int dig = hh ? (m & 15) : (m >> 4);
        ca[j] = (q < 0 ? 32u : 0u) | (unsigned)dig;
        cw[j] = sm_code((int)W[r * 32 + j] - 8);
    }
    const int8v a = pack6(ca), w = pack6(cw);
    float16v c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(w, a, float16v{}, 2, 2, 0, 130, 0, hh ? 130 : 134);
    for (int i = 0; i < 16; i++) {
        const int row = 8 * (i / 4) + 4 * hh + (i % 4);
        C[row * 32 + r] = c[i];
    }
}

int main() {
    signed char hA[1024];
    unsigned char hW[1024];
    float hC[1024];
    signed char *dA;
    unsigned char *dW;
    float *dC;
    hipMalloc(&dA, 1024);
    hipMalloc(&dW, 1024);
    hipMalloc(&dC, 4096);
    int bad = 0;
    for (int pass = 0; pass < 4; pass++) {
        srand(100 + pass);
        for (int i = 0; i < 1024; i++) {
            hA[i] = (signed char)(rand() % 255 - 127);
            hW[i] = (unsigned char)(rand() % 16);
        }
        if (pass == 1)  // extremes: every activation +-127, every weight -8 / 7
            for (int i = 0; i < 1024; i++) {
                hA[i] = (i & 1) ? 127 : -127;
                hW[i] = (i & 2) ? 0 : 15;
            }
        if (pass == 2)  // small magnitudes (subnormal codes on both sides)
            for (int i = 0; i < 1024; i++) {
                hA[i] = (signed char)(rand() % 15 - 7);
                hW[i] = (unsigned char)(rand() % 15 + 1);
            }
        hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
        hipMemcpy(dW, hW, 1024, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dW, dC);
        hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
        int nb = 0;
        for (int f = 0; f < 32; f++)
            for (int t = 0; t < 32; t++) {
                long want = 0;
                for (int j = 0; j < 32; j++) want += (long)hA[t * 32 + j] * ((int)hW[f * 32 + j] - 8);
                if (hC[f * 32 + t] != (float)want) {
                    if (nb < 4) printf("pass %d f %d t %d: got %.1f want %ld\n", pass, f, t, hC[f * 32 + t], want);
                    nb++;
                }
            }
        printf("e2m3 pass %d: %d mismatches of 1024\n", pass, nb);
        bad += nb;
    }
    printf(bad ? "FAIL\n" : "OK\n");
    return bad != 0;
}
