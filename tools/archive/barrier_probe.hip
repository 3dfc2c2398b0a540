// Compile-only probe (hipcc -S): which waits does the compiler put in front of
// a workgroup barrier after a global store and a global load in flight?
// __syncthreads() vs a raw s_barrier preceded by an LDS-only wait (development tool).
#include <hip/hip_runtime.h>

__global__ void raw_barrier(float *p, float *q, float *r) {
    __shared__ float s[256];
    p[threadIdx.x] = 1.f;
    const float pre = r[threadIdx.x];
    s[threadIdx.x] = q[threadIdx.x];
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) only
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    q[threadIdx.x] = s[255 - threadIdx.x] + pre;
}

__global__ void sync_barrier(float *p, float *q, float *r) {
    __shared__ float s[256];
    p[threadIdx.x] = 1.f;
    const float pre = r[threadIdx.x];
    s[threadIdx.x] = q[threadIdx.x];
    __syncthreads();
    q[threadIdx.x] = s[255 - threadIdx.x] + pre;
}

__global__ void local_fence_barrier(float *p, float *q, float *r) {
    __shared__ float s[256];
    p[threadIdx.x] = 1.f;
    const float pre = r[threadIdx.x];
    s[threadIdx.x] = q[threadIdx.x];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    q[threadIdx.x] = s[255 - threadIdx.x] + pre;
}
