// Calibration probe (development tool, not shipped): issue cost of the
// instructions the Q4 GEMM fold is built from, per SIMD, with 1..4 waves per
// SIMD.  Each kernel runs a fixed count of independent instructions per wave
// and stamps s_memtime around the loop; cycles per wave-instruction per SIMD =
// (loop cycles) / (instructions issued by all waves of that SIMD).
//   build: hipcc -O3 --offload-arch=gfx950 tools/calib_probe.hip -o build/calib_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float float16v __attribute__((ext_vector_type(16)));
typedef float float4v __attribute__((ext_vector_type(4)));
typedef int int16v __attribute__((ext_vector_type(16)));
typedef int int4v __attribute__((ext_vector_type(4)));
typedef int int8v __attribute__((ext_vector_type(8)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int ITER = 4096;

// op 0: v_fma_f32 x16 per iter; 1: v_cvt_f32_i32 + v_fma x16; 2: i8 mfma 32x32x32;
// 3: f16 mfma 32x32x16; 4: scaled fp6 mfma 32x32x64; 5: i8 mfma + 16 cvt + 16 fma (fold);
// 6: fp6 mfma + f16 dd mfma + 16 fma; 7: i8 mfma + dd mfma + 16 cvt + 16 fma;
// 8: two f16 mfma (int operands) + dd mfma + 16 fma
template <int OP>
__global__ void probe(float *out, long long *cyc, float seed) {
    extern __shared__ char lds_pad[];  // 96 KiB dynamic: one workgroup per CU
    const int lane = threadIdx.x & 63;
    if (seed < 0) lds_pad[threadIdx.x] = 0;
    float16v a0, a1, a2, a3;
    int16v i0, i1;
    for (int i = 0; i < 16; i++) {
        a0[i] = seed * (i + 1);
        a1[i] = seed * (i + 2);
        a2[i] = seed * (i + 3);
        a3[i] = seed * (i + 4);
        i0[i] = lane + i;
        i1[i] = lane - i;
    }
    int4v wq = {lane, lane * 3, lane * 5, lane * 7};
    int4v xq = {lane * 11, lane * 13, lane * 17, lane * 19};
    int8v w6 = {lane, lane * 3, lane * 5, lane * 7, lane * 9, lane * 11, 0, 0};
    int8v x6 = {lane * 13, lane * 15, lane * 17, lane * 19, lane * 21, lane * 23, 0, 0};
    half8 h0, h1;
    for (int j = 0; j < 8; j++) {
        h0[j] = (_Float16)(lane + j);
        h1[j] = (_Float16)(lane - j);
    }
    float16v dd = a3;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITER; it++) {
        if constexpr (OP == 0) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                a0[i] = __builtin_fmaf(a1[i], a2[i], a0[i]);
                asm volatile("" : "+v"(a0[i]));
            }
        } else if constexpr (OP == 1) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                asm volatile("" : "+v"(i0[i]));  // opaque: the cvt stays in the loop
                float v = __builtin_fmaf((float)i0[i], a2[i], a0[i]);
                asm volatile("" : "+v"(v));
                a0[i] = v;
            }
        } else if constexpr (OP == 2) {
            i0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(wq, xq, i0, 0, 0, 0);
            i1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(xq, wq, i1, 0, 0, 0);
        } else if constexpr (OP == 3) {
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(h0, h1, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(h1, h0, a1, 0, 0, 0);
        } else if constexpr (OP == 4) {
            a0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(w6, x6, a0, 3, 3, 0, 127, 0, 131);
            a1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(x6, w6, a1, 3, 3, 0, 127, 0, 131);
        } else if constexpr (OP == 5 || OP == 7) {
            // int8 fold: is = mfma(); (dd = mfma()); acc += (float) is * dd
            const float16v zf = {};
            int16v is = __builtin_amdgcn_mfma_i32_32x32x32_i8(wq, xq, __builtin_bit_cast(int16v, zf), 0, 0, 0);
            if constexpr (OP == 7) dd = __builtin_amdgcn_mfma_f32_32x32x16_f16(h0, h1, zf, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; i++) {
                float v = __builtin_fmaf((float)is[i], dd[i], a0[i]);
                asm volatile("" : "+v"(v));
                a0[i] = v;
            }
            wq[0] += 1;
        } else if constexpr (OP == 6) {
            const float16v zf = {};
            float16v is = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(w6, x6, zf, 3, 3, 0, 127, 0, 131);
            dd = __builtin_amdgcn_mfma_f32_32x32x16_f16(h0, h1, zf, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; i++) {
                float v = __builtin_fmaf(is[i], dd[i], a0[i]);
                asm volatile("" : "+v"(v));
                a0[i] = v;
            }
            w6[0] += 1;
        } else if constexpr (OP == 8) {
            const float16v zf = {};
            float16v is = __builtin_amdgcn_mfma_f32_32x32x16_f16(h0, h1, zf, 0, 0, 0);
            is = __builtin_amdgcn_mfma_f32_32x32x16_f16(h1, h0, is, 0, 0, 0);
            dd = __builtin_amdgcn_mfma_f32_32x32x16_f16(h0, h0, zf, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; i++) {
                float v = __builtin_fmaf(is[i], dd[i], a0[i]);
                asm volatile("" : "+v"(v));
                a0[i] = v;
            }
            h0[0] += (_Float16)1;
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0;
    for (int i = 0; i < 16; i++) s += a0[i] + a1[i] + (float)i0[i] + (float)i1[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        cyc[2 * blockIdx.x] = t1 - t0;
        cyc[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// VALU / MFMA instructions per iteration per wave, for the per-SIMD rate
struct OpInfo {
    const char *name;
    int valu, mfma;
};
static const OpInfo INFO[] = {{"v_fma_f32 x16", 16, 0},
                              {"cvt + fma x16", 32, 0},
                              {"i8 mfma 32x32x32 x2", 0, 2},
                              {"f16 mfma 32x32x16 x2", 0, 2},
                              {"fp6 scaled mfma 32x32x64 x2", 0, 2},
                              {"i8 mfma + 16 (cvt+fma)", 32, 1},
                              {"fp6 mfma + dd mfma + 16 fma", 16, 2},
                              {"i8 mfma + dd mfma + 16 (cvt+fma)", 32, 2},
                              {"2 f16 mfma + dd mfma + 16 fma", 16, 3}};

template <int OP>
static void run(int waves_per_simd, float *d_out, long long *d_cyc) {
    const int threads = 256 * waves_per_simd, blocks = 256;
    const size_t lds = 96 * 1024;
    CK(hipFuncSetAttribute((const void *)probe<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(threads), lds, 0, d_out, d_cyc, 1e-3f);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(threads), lds, 0, d_out, d_cyc, 1e-3f);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> c(2 * blocks);
    CK(hipMemcpy(c.data(), d_cyc, blocks * 16, hipMemcpyDeviceToHost));
    double avg = 0, rt = 0;
    for (int b = 0; b < blocks; b++) {
        avg += (double)c[2 * b];
        rt += (double)c[2 * b + 1];
    }
    avg /= blocks;
    rt /= blocks;  // 100 MHz ticks
    const double ghz = avg / (rt * 10.0);  // memtime ticks per ns
    const OpInfo &I = INFO[OP];
    const double per_iter = avg / ITER;  // cycles per iteration of every wave on the SIMD
    const double per_wave_iter = per_iter / waves_per_simd;
    const double ns_iter = rt * 10.0 / ITER / waves_per_simd;  // SIMD ns per wave-iteration
    printf("%-36s w/SIMD %d: %6.2f ticks  %6.2f ns (= %5.1f cyc @2.4GHz) per wave-iter (valu %d mfma %d); tick %.2f GHz; wall %.3f ms\n",
           I.name, waves_per_simd, per_wave_iter, ns_iter, ns_iter * 2.4, I.valu, I.mfma, ghz, ms);
    fflush(stdout);
}

int main() {
    float *d_out;
    long long *d_cyc;
    CK(hipMalloc(&d_out, 256 * 1024 * 4));
    CK(hipMalloc(&d_cyc, 256 * 16));
    for (int w = 1; w <= 4; w *= 2) {
        run<0>(w, d_out, d_cyc);
        run<1>(w, d_out, d_cyc);
        run<2>(w, d_out, d_cyc);
        run<3>(w, d_out, d_cyc);
        run<4>(w, d_out, d_cyc);
        run<5>(w, d_out, d_cyc);
        run<6>(w, d_out, d_cyc);
        run<7>(w, d_out, d_cyc);
        run<8>(w, d_out, d_cyc);
    }
    return 0;
}
