// Probe (development tool): checks on the device the lane maps the Q4 x Q8
// int8-MFMA GEMM relies on (kernels.hip q4 main loop):
//  1. v_mfma_i32_32x32x32_i8 with lane (r, h) holding bytes j = 0..15 of
//     row / column r at k = 16h + j on BOTH operands returns
//     C[row][col] at lane col + 32h', register i with row = 8(i/4) + 4h' + i%4.
//  2. v_mfma_f32_32x32x16_f16 with only element 0 (and 1) of lanes 0-31 set
//     returns the exact outer product of two fp16 scale vectors (the per-block
//     d_w * d_a factors) in the same output layout.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef int int4v __attribute__((ext_vector_type(4)));
typedef int int16v __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));

__global__ void probe(const int8_t *A, const int8_t *B, const _Float16 *sa, const _Float16 *sb, int *C, float *D) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    int4v a, b;
    __builtin_memcpy(&a, A + r * 32 + 16 * h, 16);  // A[row r][k 16h..]
    __builtin_memcpy(&b, B + r * 32 + 16 * h, 16);  // B^T[col r][k 16h..]
    int16v c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, int16v{}, 0, 0, 0);
    half8 x = {}, y = {};
    if (h == 0) {
        x[0] = sa[r];
        y[0] = sb[r];
    }
    float16v d = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, y, float16v{}, 0, 0, 0);
    for (int i = 0; i < 16; i++) {
        const int row = 8 * (i / 4) + 4 * h + (i % 4);
        C[row * 32 + r] = c[i];
        D[row * 32 + r] = d[i];
    }
}

int main() {
    int8_t hA[1024], hB[1024];
    _Float16 hsa[32], hsb[32];
    srand(7);
    for (int i = 0; i < 1024; i++) {
        hA[i] = (int8_t)(rand() % 255 - 127);
        hB[i] = (int8_t)(rand() % 16 - 8);
    }
    for (int i = 0; i < 32; i++) {
        hsa[i] = (_Float16)((rand() % 2047 + 1) * 0x1p-14f);
        hsb[i] = (_Float16)((rand() % 2047 + 1) * 0x1p-9f);
    }
    int8_t *dA, *dB;
    _Float16 *dsa, *dsb;
    int *dC;
    float *dD;
    hipMalloc(&dA, 1024);
    hipMalloc(&dB, 1024);
    hipMalloc(&dsa, 64);
    hipMalloc(&dsb, 64);
    hipMalloc(&dC, 4096);
    hipMalloc(&dD, 4096);
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dsa, hsa, 64, hipMemcpyHostToDevice);
    hipMemcpy(dsb, hsb, 64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC, dD);
    int hC[1024];
    float hD[1024];
    hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
    hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
    int bad = 0, badd = 0;
    for (int m = 0; m < 32; m++)
        for (int n = 0; n < 32; n++) {
            int s = 0;
            for (int k = 0; k < 32; k++) s += hA[m * 32 + k] * hB[n * 32 + k];
            bad += hC[m * 32 + n] != s;
            const float want = (float)hsa[m] * (float)hsb[n];
            badd += hD[m * 32 + n] != want;
        }
    printf("i8 32x32x32 layout mismatches: %d / 1024; f16 outer-product mismatches: %d / 1024\n", bad, badd);
    return (bad || badd) ? 1 : 0;
}
