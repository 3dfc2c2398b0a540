// Exhaustive device check of the short Q8 scale divisions used by the
// activation quantisers (kernels.hip q8_scales) against IEEE division, over
// every positive finite f32 (development tool; run on the GPU box).
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

__device__ __forceinline__ float div127(float x) {  // RN(x / 127)
    const float r = 1.0f / 127.0f;
    const float q = x * r;
    const float e = __builtin_fmaf(-q, 127.0f, x);
    return __builtin_fmaf(e, r, q);
}
__device__ __forceinline__ float div127r(float x) {  // RN(127 / x)
    const float y = __builtin_amdgcn_rcpf(x);
    const float q = 127.0f * y;
    const float e = __builtin_fmaf(-x, q, 127.0f);
    return __builtin_fmaf(e, y, q);
}

__global__ void check(unsigned long long *bad, unsigned *first) {
    const uint64_t n = 0x7f800000ull;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const float x = __uint_as_float((uint32_t)i);
        volatile float c127 = 127.0f;
        const float d0 = x / c127, d1 = div127(x);
        const float i0 = c127 / x, i1 = div127r(x);
        if (__float_as_uint(d0) != __float_as_uint(d1)) {
            atomicAdd(&bad[0], 1ull);
        }
        if (i >= 0x0d000000u && i < 0x72000000u && __float_as_uint(i0) != __float_as_uint(i1)) {
            atomicAdd(&bad[1], 1ull);
            atomicMin(&first[0], (uint32_t)i);
            atomicMax(&first[1], (uint32_t)i);
        }
    }
}

int main() {
    unsigned long long *bad;
    unsigned *first;
    hipMalloc(&bad, 32);
    hipMalloc(&first, 32);
    hipMemset(bad, 0, 32);
    hipMemset(first, 0, 32);
    hipMemset(first, 0xff, 4);
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, bad, first);
    unsigned long long h[4];
    unsigned f[8];
    hipMemcpy(h, bad, 32, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
    printf("x/127 mismatches %llu; 127/x mismatches (x in [2^-101, 2^101)) %llu, x bits in [0x%08x, 0x%08x]\n", h[0], h[1], f[0], f[1]);
    return 0;
}
