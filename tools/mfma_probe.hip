// Development probe: throughput of the Q4 GEMM inner-loop structure with
// register-only operands (no memory), per variant and waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));
typedef float float4v __attribute__((ext_vector_type(4)));

template <int VAR, int TILES>
__global__ __launch_bounds__(256) void probe(float *out, int iters) {
    const int lane = threadIdx.x & 63;
    half8 a0, a1, b0, b1;
    for (int j = 0; j < 8; j++) {
        a0[j] = (_Float16)(lane + j);
        a1[j] = (_Float16)(lane - j);
        b0[j] = (_Float16)(j * 0.5f);
        b1[j] = (_Float16)(j * 0.25f);
    }
    float16v acc[TILES];
    for (int t = 0; t < TILES; t++) acc[t] = float16v{};
    float da = 1.0f + lane * 1e-3f;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int t = 0; t < TILES; t++) {
            asm volatile("" : "+v"(a0), "+v"(a1));  // distinct operands per tile: no CSE across tiles
            if constexpr (VAR == 0) {  // 4 dependent MFMAs + 16 fma fold
                float16v b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, float16v{}, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, b, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, b, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, b, 0, 0, 0);
#pragma unroll
                for (int j = 0; j < 16; j++) acc[t][j] = __builtin_fmaf(da, b[j], acc[t][j]);
            } else if constexpr (VAR == 1) {  // 4 MFMAs accumulating (no fold)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc[t], 0, 0, 0);
            } else if constexpr (VAR == 2) {  // 16x16x32: 2 MFMAs + 4 fma per tile, x4 tiles to match work
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    asm volatile("" : "+v"(a0));
                    float4v b = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0, float4v{}, 0, 0, 0);
                    b = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, b, 0, 0, 0);
#pragma unroll
                    for (int j = 0; j < 4; j++) acc[t][4 * u + j] = __builtin_fmaf(da, b[j], acc[t][4 * u + j]);
                }
            }
        }
        if constexpr (VAR == 3) {  // pipelined: tile t+1's MFMAs issued before tile t's fold
            float16v bb[2];
            auto iss = [&](int t) {
                asm volatile("" : "+v"(a0), "+v"(a1));
                float16v b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, float16v{}, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, b, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, b, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, b, 0, 0, 0);
                bb[t & 1] = b;
            };
            iss(0);
#pragma unroll
            for (int t = 0; t < TILES; t++) {
                if (t + 1 < TILES) iss(t + 1);
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    float v = acc[t][j];
                    v = __builtin_fmaf(da, bb[t & 1][j], v);
                    asm volatile("" : "+v"(v));
                    acc[t][j] = v;
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if constexpr (VAR == 4) {  // pipelined, no sched_barrier / pinning: compiler schedule
            float16v bb[TILES];
#pragma unroll
            for (int t = 0; t < TILES; t++) {
                asm volatile("" : "+v"(a0), "+v"(a1));
                float16v b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, float16v{}, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, b, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, b, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, b, 0, 0, 0);
                bb[t] = b;
            }
#pragma unroll
            for (int t = 0; t < TILES; t++)
#pragma unroll
                for (int j = 0; j < 16; j++) acc[t][j] = __builtin_fmaf(da, bb[t][j], acc[t][j]);
        }
        da += 1e-7f;
        asm volatile("" : "+v"(a0), "+v"(b0));
    }
    float s = 0.f;
    for (int t = 0; t < TILES; t++)
        for (int j = 0; j < 16; j++) s += acc[t][j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int VAR, int TILES>
void run(const char *name, int wgs_per_cu, float *out) {
    const int iters = 2000, grid = 256 * wgs_per_cu;
    hipLaunchKernelGGL((probe<VAR, TILES>), dim3(grid), dim3(256), 0, 0, out, 10);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((probe<VAR, TILES>), dim3(grid), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // useful MFMA cycles: VAR0/1: 4 x 32x32x16 per tile; VAR2: 8 x 16x16x32 per tile (same flops)
    const double flops = (double)grid * 4 * iters * TILES * 4.0 * 32768;  // waves * tiles * 4 mfma * flops
    printf("%-28s waves/SIMD %d: %8.3f ms  %7.1f TF/s  (%.0f%% of 2516)\n", name, wgs_per_cu, ms, flops / ms * 1e-9,
           flops / ms * 1e-9 / 2516 * 100);
}

int main() {
    float *out;
    hipMalloc(&out, 256 * 8 * 256 * 4);
    for (int w = 1; w <= 3; w++) {
        run<0, 4>("32x32 chain4 + fold16", w, out);
        run<1, 4>("32x32 acc4 (no fold)", w, out);
        run<2, 4>("16x16 pair + fold4 (x4)", w, out);
        run<3, 4>("32x32 pipelined sched", w, out);
        run<4, 4>("32x32 batch4 then fold", w, out);
    }
    return 0;
}
