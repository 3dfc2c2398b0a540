// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths and patterns the library's kernels use (development tool; the
// MI355X guide calibrates only 16-byte-per-lane streaming accesses).  Each
// kernel moves a known number of bytes exactly once; tools/pmc_calib.sh runs
// one counter pass per counter and tools/pmc_calib.py prints counted / moved.
//   st16 / st8 / st4 / st2   fully coalesced stores of that many bytes per lane
//   ld16 / ld8 / ld4         fully coalesced loads (one 4-byte word per block stored)
//   st4_rows                 the fused kernel's context store pattern: a wave
//                            writes 4 bytes per lane into 32 rows 384 B apart,
//                            four passes complete 32 contiguous bytes per row
//   st8_ln                   the LN epilogues' f32 pattern: a lane writes two
//                            adjacent floats, 16 lanes cover 128 B of one row
//   scratch                  per-lane private stores through a dynamically
//                            indexed local array (register spills' path)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x)                                                                 \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));

template <typename T>
__global__ __launch_bounds__(256) void st_kernel(T *p, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = T(i);
}
__global__ __launch_bounds__(256) void st16_kernel(u32x4v *p, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = u32x4v{(unsigned)i, 1u, 2u, 3u};
}
__global__ __launch_bounds__(256) void st8_kernel(u32x2v *p, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = u32x2v{(unsigned)i, 1u};
}
__global__ __launch_bounds__(256) void ld16_kernel(const u32x4v *p, size_t n, unsigned *out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const u32x4v v = i < n ? p[i] : u32x4v{0u, 0u, 0u, 0u};
    unsigned s = v.x ^ v.y ^ v.z ^ v.w;
    for (int o = 32; o; o >>= 1) s ^= __shfl_xor(s, o);
    if (threadIdx.x == 0) out[blockIdx.x] = s;
}
__global__ __launch_bounds__(256) void ld8_kernel(const u32x2v *p, size_t n, unsigned *out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const u32x2v v = i < n ? p[i] : u32x2v{0u, 0u};
    unsigned s = v.x ^ v.y;
    for (int o = 32; o; o >>= 1) s ^= __shfl_xor(s, o);
    if (threadIdx.x == 0) out[blockIdx.x] = s;
}
__global__ __launch_bounds__(256) void ld4_kernel(const unsigned *p, size_t n, unsigned *out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    unsigned s = i < n ? p[i] : 0u;
    for (int o = 32; o; o >>= 1) s ^= __shfl_xor(s, o);
    if (threadIdx.x == 0) out[blockIdx.x] = s;
}
// rows of 384 bytes (E = 384 int8 codes); wave w of a block owns 32 rows and
// one 32-byte column block; lane (r, hh) writes bytes 8 m + 4 hh, m = 0..3
__global__ __launch_bounds__(256) void st4_rows_kernel(int8_t *p, size_t rows) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, r = lane & 31, hh = lane >> 5;
    const size_t blk = (size_t)blockIdx.x * 4 + wv;  // (32-row group, column block) pairs
    const size_t rg = blk / 12, cb = blk % 12;
    const size_t row = rg * 32 + r;
    if (row >= rows) return;
    for (int m = 0; m < 4; m++) *(uint32_t *)(p + row * 384 + cb * 32 + 8 * m + 4 * hh) = 0x01010101u * (m + 1);
}
// f32 rows of 384: lane (g, c16) of wave w writes columns 2 c16, 2 c16 + 1 of
// 4 rows 4 g .. 4 g + 3 in the wave's 32-column slice (the LN epilogue's
// two-column-per-lane layout)
__global__ __launch_bounds__(256) void st8_ln_kernel(float *p, size_t rows) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
    const size_t rt = blockIdx.x;  // 16-row tile
    for (int cs = wv; cs < 12; cs += 4)
        for (int i = 0; i < 4; i++) {
            const size_t row = rt * 16 + 4 * g + i;
            if (row < rows) *(u32x2v *)(p + row * 384 + cs * 32 + 2 * c16) = u32x2v{1u, 2u};
        }
}
__global__ __launch_bounds__(256) void scratch_kernel(unsigned *out, int sel, int reps) {
    volatile unsigned loc[64];
    for (int i = 0; i < 64; i++) loc[i] = threadIdx.x + i;
    unsigned s = 0;
    for (int k = 0; k < reps; k++) s += loc[(sel + k) & 63];
    if (s == 0xdeadbeefu) out[blockIdx.x] = s;
}

int main(int argc, char **argv) {
    const size_t BYTES = (size_t)256 << 20;
    void *buf;
    unsigned *sink;
    CHECK(hipMalloc(&buf, BYTES));
    CHECK(hipMalloc(&sink, BYTES / 16));
    CHECK(hipMemset(buf, 1, BYTES));
    const auto grid = [](size_t n) { return dim3((unsigned)((n + 255) / 256)); };
    // one launch of each; rocprofv3 separates them by kernel name
    hipLaunchKernelGGL(st16_kernel, grid(BYTES / 16), dim3(256), 0, 0, (u32x4v *)buf, BYTES / 16);
    hipLaunchKernelGGL(st8_kernel, grid(BYTES / 8), dim3(256), 0, 0, (u32x2v *)buf, BYTES / 8);
    hipLaunchKernelGGL(st_kernel<unsigned>, grid(BYTES / 4), dim3(256), 0, 0, (unsigned *)buf, BYTES / 4);
    hipLaunchKernelGGL(st_kernel<uint16_t>, grid(BYTES / 2), dim3(256), 0, 0, (uint16_t *)buf, BYTES / 2);
    hipLaunchKernelGGL(ld16_kernel, grid(BYTES / 16), dim3(256), 0, 0, (const u32x4v *)buf, BYTES / 16, sink);
    hipLaunchKernelGGL(ld8_kernel, grid(BYTES / 8), dim3(256), 0, 0, (const u32x2v *)buf, BYTES / 8, sink);
    hipLaunchKernelGGL(ld4_kernel, grid(BYTES / 4), dim3(256), 0, 0, (const unsigned *)buf, BYTES / 4, sink);
    const size_t rows = BYTES / 384 / 32 * 32;  // 384-byte rows
    hipLaunchKernelGGL(st4_rows_kernel, dim3((unsigned)(rows / 32 * 12 / 4)), dim3(256), 0, 0, (int8_t *)buf, rows);
    const size_t frows = BYTES / (384 * 4) / 16 * 16;  // f32 rows of 384
    hipLaunchKernelGGL(st8_ln_kernel, dim3((unsigned)(frows / 16)), dim3(256), 0, 0, (float *)buf, frows);
    const int sblocks = 8192;  // 8192 x 256 lanes x 64 words x 4 B = 512 MiB of private stores
    hipLaunchKernelGGL(scratch_kernel, dim3(sblocks), dim3(256), 0, 0, sink, argc, 4);
    CHECK(hipDeviceSynchronize());
    printf("bytes st16 st8 st4 st2 ld16 ld8 ld4 %zu\n", BYTES);
    printf("bytes st4_rows %zu\n", rows * 384);
    printf("bytes st8_ln %zu\n", frows * 384 * 4);
    printf("bytes scratch %zu\n", (size_t)sblocks * 256 * 64 * 4);
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
