// Probe (development tool): the block-scaled f8f6f4 MFMA as an exact
// integer dot product.  v_mfma_scale_f32_32x32x64_f8f6f4 with bf6 (e3m2)
// operands: integers -8..8 are exact in e3m2, so a Q8 activation q in
// [-127, 127] splits into two digits q = 16 h + l (h in [-8, 8], l in [-8, 7])
// and ONE MFMA over K = 64 computes the exact block sum
//     isum = sum_j (16 h_j + l_j) w_j
// when lanes 0-31 carry the h digits of the 32-element block with E8M0 scale
// 2^4 and lanes 32-63 the l digits with scale 2^0, against the same 32
// weights w in both lane halves.  Checks: (1) the 6-bit packing (element j at
// bits 6j .. 6j + 5 of the lane's 6 dwords), (2) per-lane scales apply to the
// lane's own 32 elements, (3) the result equals the int32 dot exactly.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef int int8v __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));

// e3m2 code of an integer in [-8, 8]
__host__ __device__ inline unsigned e3m2(int v) {
    const unsigned s = v < 0 ? 32u : 0u;
    int a = v < 0 ? -v : v;
    if (a == 0) return s;
    int e = 0;
    while ((a >> (e + 1)) != 0) e++;              // a in [2^e, 2^(e+1))
    const unsigned m = (unsigned)((a << 2 >> e) & 3);  // 2 mantissa bits
    return s | ((unsigned)(e + 3) << 2) | m;
}

__device__ inline int8v pack6(const signed char *v) {  // 32 values -> 6 dwords, LSB first
    int8v r = {};
    for (int j = 0; j < 32; j++) {
        const unsigned c = e3m2(v[j]);
        const int bit = 6 * j, w = bit >> 5, o = bit & 31;
        r[w] |= (int)(c << o);
        if (o > 26) r[w + 1] |= (int)(c >> (32 - o));
    }
    return r;
}

// A: q8 activations [32 tokens][32], W: weights [32 features][32] (-8..7)
__global__ void probe(const signed char *A, const signed char *W, float *C, int scale_h, int scale_l) {
    const int l = threadIdx.x, r = l & 31, hh = l >> 5;
    signed char va[32], vw[32];
    for (int j = 0; j < 32; j++) {
        const int q = A[r * 32 + j];
        const int h = (q + (q >= 0 ? 8 : 7)) >> 4;  // round q / 16 (any split with |l| <= 8 works)
        const int lo = q - 16 * h;
        va[j] = (signed char)(hh ? lo : h);
        vw[j] = W[r * 32 + j];
    }
    const int8v a = pack6(va), b = pack6(vw);
    // A = weights (rows = features), B = activations (cols = tokens)
    float16v c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, a, float16v{}, 3, 3, 0, 127, 0,
                                                                  hh ? scale_l : scale_h);
    for (int i = 0; i < 16; i++) {
        const int row = 8 * (i / 4) + 4 * hh + (i % 4);
        C[row * 32 + r] = c[i];
    }
}

int main() {
    signed char hA[1024], hW[1024];
    srand(11);
    for (int i = 0; i < 1024; i++) {
        hA[i] = (signed char)(rand() % 255 - 127);
        hW[i] = (signed char)(rand() % 16 - 8);
    }
    hA[0] = 127; hA[1] = -127; hA[2] = 8; hA[3] = -8; hA[4] = 120; hA[5] = -121;
    signed char *dA, *dW;
    float *dC;
    hipMalloc(&dA, 1024); hipMalloc(&dW, 1024); hipMalloc(&dC, 4096);
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dW, hW, 1024, hipMemcpyHostToDevice);
    float hC[1024];
    int bad = 0;
    for (int pass = 0; pass < 2; pass++) {
        // pass 0: scales 2^4 / 2^0 (exact isum); pass 1: both 2^0 (h + l, a different sum)
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dW, dC, pass ? 127 : 131, 127);
        hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
        int nb = 0;
        for (int f = 0; f < 32; f++)
            for (int t = 0; t < 32; t++) {
                long want = 0;
                for (int j = 0; j < 32; j++) {
                    const int q = hA[t * 32 + j];
                    const int h = (q + (q >= 0 ? 8 : 7)) >> 4, lo = q - 16 * h;
                    want += (long)(pass ? h + lo : q) * hW[f * 32 + j];
                }
                if (hC[f * 32 + t] != (float)want) {
                    if (nb < 4) printf("pass %d f %d t %d: got %.1f want %ld\n", pass, f, t, hC[f * 32 + t], want);
                    nb++;
                }
            }
        printf("pass %d (%s): %d mismatches of 1024\n", pass, pass ? "scales 1/1" : "scales 16/1, exact isum", nb);
        bad += nb;
    }
    printf(bad ? "FAIL\n" : "OK\n");
    return bad != 0;
}
