// Development probe: throughput of the Q4 GEMM inner-loop structure with
// register-only operands (no memory), per variant and waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));
typedef float float4v __attribute__((ext_vector_type(4)));

template <int VAR, int TILES>
__global__ __launch_bounds__(256) void probe(float *out, int iters, const half8 *wsrc) {
    const int lane = threadIdx.x & 63;
    __shared__ __attribute__((aligned(16))) _Float16 lds[128 * 80 + 64];
    __shared__ __attribute__((aligned(16))) float ldsf[256];
    for (int i = threadIdx.x; i < 128 * 80; i += 256) lds[i] = (_Float16)(i & 7);
    for (int i = threadIdx.x; i < 256; i += 256) ldsf[i] = 1.0f;
    __syncthreads();
    half8 wh[2][2], wl[2][2];
    for (int k = 0; k < 2; k++)
        for (int n = 0; n < 2; n++) {
            wh[k][n] = half8{} + (_Float16)(k + n);
            wl[k][n] = half8{} + (_Float16)(k - n);
        }
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
        if constexpr (VAR == 5 || VAR == 6) {  // 16x16 pipelined: pair for tile-part u+1 issued before fold of u (VAR6: packed fold)
            float4v bb[2];
            auto iss = [&](int u) {
                asm volatile("" : "+v"(a0));
                float4v b = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0, float4v{}, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, b, 0, 0, 0);
                bb[u & 1] = b;
            };
            iss(0);
#pragma unroll
            for (int u = 0; u < 4 * TILES; u++) {
                if (u + 1 < 4 * TILES) iss(u + 1);
                const int t = u / 4, o = 4 * (u % 4);
                if constexpr (VAR == 5) {
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        float v = acc[t][o + j];
                        v = __builtin_fmaf(da, bb[u & 1][j], v);
                        asm volatile("" : "+v"(v));
                        acc[t][o + j] = v;
                    }
                } else {
                    typedef float float2v __attribute__((ext_vector_type(2)));
#pragma unroll
                    for (int j = 0; j < 4; j += 2) {
                        float2v v = {acc[t][o + j], acc[t][o + j + 1]};
                        v = __builtin_elementwise_fma(float2v{da, da}, float2v{bb[u & 1][j], bb[u & 1][j + 1]}, v);
                        asm volatile("" : "+v"(v));
                        acc[t][o + j] = v[0];
                        acc[t][o + j + 1] = v[1];
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if constexpr (VAR == 7) {  // 32x32 pipelined with packed fold
            typedef float float2v __attribute__((ext_vector_type(2)));
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
                for (int j = 0; j < 16; j += 2) {
                    float2v v = {acc[t][j], acc[t][j + 1]};
                    v = __builtin_elementwise_fma(float2v{da, da}, float2v{bb[t & 1][j], bb[t & 1][j + 1]}, v);
                    asm volatile("" : "+v"(v));
                    acc[t][j] = v[0];
                    acc[t][j + 1] = v[1];
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if constexpr (VAR == 8 || VAR == 9) {
            // one "block" of the real Q4 loop: RT = 8 row tiles x NTW = 2 n-tiles,
            // A fragments + d_a read from LDS per row tile; VAR9 also streams W
            // fragments (hi, lo per n-tile) from global memory two blocks ahead
            constexpr int RT = 8, NTW = 2, T = RT * NTW;
            half8 a[RT];
            float4v dav[RT];
            const int c16 = lane & 15, g = lane >> 4;
            auto lds_a = [&](int rt) {
                a[rt] = *(const half8 *)(lds + (rt * 16 + c16) * 80 + 8 * g + (it & 1) * 32);
                dav[rt] = *(const float4v *)(ldsf + rt * 16 + 4 * g);
            };
            if constexpr (VAR == 9) {
                const int kb = it & 1;
#pragma unroll
                for (int nt = 0; nt < NTW; nt++) {
                    wh[kb][nt] = wsrc[((int64_t)(((blockIdx.x & 15) * 2 + nt) * 64 + (it & 63))) * 128 + lane];
                    wl[kb][nt] = wsrc[((int64_t)(((blockIdx.x & 15) * 2 + nt) * 64 + (it & 63))) * 128 + 64 + lane];
                }
            }
            const int kb = (it + 1) & 1;
            float4v bb[2];
            auto iss = [&](int t) {
                const int rt = t / NTW, nt = t % NTW;
                float4v b = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rt], wh[kb][nt], float4v{}, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rt], wl[kb][nt], b, 0, 0, 0);
                bb[t & 1] = b;
            };
            lds_a(0);
            if (NTW == 1) lds_a(1);
            iss(0);
#pragma unroll
            for (int t = 0; t < T; t++) {
#pragma unroll
                for (int rt = 0; rt < RT; rt++)
                    if (rt * NTW == t + 2) lds_a(rt);
                if (t + 1 < T) iss(t + 1);
                const int rt = t / NTW, nt = t % NTW;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float v = acc[(rt * NTW + nt) / 4][4 * ((rt * NTW + nt) % 4) + j];
                    v = __builtin_fmaf(dav[rt][j], bb[t & 1][j], v);
                    asm volatile("" : "+v"(v));
                    acc[(rt * NTW + nt) / 4][4 * ((rt * NTW + nt) % 4) + j] = v;
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
        asm volatile("" : "+v"(wh[0][0]), "+v"(wl[1][1]));
        asm volatile("" : "+v"(a0), "+v"(b0));
    }
    float s = 0.f;
    for (int t = 0; t < TILES; t++)
        for (int j = 0; j < 16; j++) s += acc[t][j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int VAR, int TILES>
void run(const char *name, int wgs_per_cu, float *out, const half8 *w) {
    const int iters = 2000, grid = 256 * wgs_per_cu;
    hipLaunchKernelGGL((probe<VAR, TILES>), dim3(grid), dim3(256), 0, 0, out, 10, w);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((probe<VAR, TILES>), dim3(grid), dim3(256), 0, 0, out, iters, w);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // useful MFMA cycles: VAR0/1: 4 x 32x32x16 per tile; VAR2: 8 x 16x16x32 per tile (same flops)
    // VAR 8/9: 16 tiles x 2 MFMA 16x16x32 (16384 flops) per iteration = 32 x 16384
    const double flops = (VAR >= 8) ? (double)grid * 4 * iters * 32.0 * 16384 : (double)grid * 4 * iters * TILES * 4.0 * 32768;
    printf("%-28s waves/SIMD %d: %8.3f ms  %7.1f TF/s  (%.0f%% of 2516)\n", name, wgs_per_cu, ms, flops / ms * 1e-9,
           flops / ms * 1e-9 / 2516 * 100);
}

int main() {
    float *out;
    hipMalloc(&out, 256 * 8 * 256 * 4);
    half8 *w;
    const size_t wn = (size_t)32 * 64 * 128;
    hipMalloc(&w, wn * 16);
    hipMemset(w, 0, wn * 16);
    for (int wv = 1; wv <= 3; wv++) {
        run<1, 4>("32x32 no fold (reg only)", wv, out, w);
        run<3, 4>("32x32 pipelined (reg only)", wv, out, w);
        run<7, 4>("32x32 pipelined pk fold", wv, out, w);
        run<5, 4>("16x16 pipelined (reg only)", wv, out, w);
        run<8, 4>("16x16 + LDS A/d_a reads", wv, out, w);
        run<9, 4>("16x16 + LDS + W global", wv, out, w);
    }
    return 0;
}
