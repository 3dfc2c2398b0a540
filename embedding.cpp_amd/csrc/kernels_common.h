// kernels_common.h — device helpers shared by the kernel translation units
// (kernels.hip: F16/F32 GEMMs, attention, embeddings, pooling; gemm_i8.hip:
// the Q4 x Q8 int8-MFMA GEMMs).  ggml numerics restated in SURVEY.md
// Appendix A.
#pragma once
#include "kernels.h"

namespace bertamd {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float float4v __attribute__((ext_vector_type(4)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef float float16v __attribute__((ext_vector_type(16)));
typedef _Float16 half4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));  // 16 raw bytes as a register vector
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));

// Development phase stamps (tools/phase_stamps.hip): compiled out of the
// library; with -DPHASE_STAMPS lane 0 of waves 0 and NW - 1 of each
// workgroup records s_memtime (shader cycles) per persistent-tile iteration
// and slot into g_stamp_buf[((blockIdx.x * STAMP_TILES + it) * 2 + w) * 16 + slot].
#ifdef PHASE_STAMPS
constexpr int STAMP_TILES = 32;
static __device__ unsigned long long *g_stamp_buf;  // set by the tool before any launch
static __device__ int g_stamp_nblk;                 // workgroups the buffer holds
#define STAMPB(bid, it, slot, nw)                                                                               \
    do {                                                                                                        \
        const int w_ = threadIdx.x >> 6;                                                                        \
        if ((threadIdx.x & 63) == 0 && (w_ == 0 || w_ == (nw) - 1) && (it) < STAMP_TILES && g_stamp_buf &&      \
            (int)(bid) < g_stamp_nblk)                                                                          \
            g_stamp_buf[(((bid) * STAMP_TILES + (it)) * 2 + (w_ != 0)) * 16 + (slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define STAMP(it, slot, nw) STAMPB(blockIdx.x, it, slot, nw)
#else
#define STAMPB(bid, it, slot, nw) ((void)0)
#define STAMP(it, slot, nw) ((void)0)
#endif

__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

// Four Q8 codes rint(x_j * id) packed little-endian: y + 1.5*2^23 rounds the
// already-rounded product y = x*id to an integer (round-to-nearest-even, as
// rintf) and leaves it, two's complement, in the low mantissa byte; two byte
// permutes gather the four low bytes.  Exact for |y| < 2^22 (here |y| <= 127).
__device__ __forceinline__ uint32_t q8_pack4(float x0, float x1, float x2, float x3, float id) {
    const float M = 12582912.0f;
    const uint32_t b0 = __float_as_uint(x0 * id + M), b1 = __float_as_uint(x1 * id + M);
    const uint32_t b2 = __float_as_uint(x2 * id + M), b3 = __float_as_uint(x3 * id + M);
    const uint32_t lo = __builtin_amdgcn_perm(b1, b0, 0x0c0c0400u);  // bytes: b0.0, b1.0, 0, 0
    const uint32_t hi = __builtin_amdgcn_perm(b3, b2, 0x04000c0cu);  // bytes: 0, 0, b2.0, b3.0
    return lo | hi;
}

// Q8 block scales of ggml's quantize_row_q8_0/q8_1 (AVX2 form): d = amax / 127
// and id = 127 / amax (0 when amax == 0), correctly rounded like the IEEE
// divisions they replace: x / 127 by one Newton step on RN(1/127), and 127 / x
// by one step on v_rcp_f32 inside [2^-101, 2^101) (outside it, the division).
// tools/div_check.hip verifies both on the device for every positive finite
// f32 (tests/test_gpu_parity.py::test_q8_scale_division_exhaustive).
__device__ __forceinline__ float div127(float x) {
    const float r = 1.0f / 127.0f;
    const float q = x * r;
    return __builtin_fmaf(__builtin_fmaf(-q, 127.0f, x), r, q);
}
__device__ __forceinline__ float div127r(float x) {
    const float y = __builtin_amdgcn_rcpf(x);
    const float q = 127.0f * y;
    return __builtin_fmaf(__builtin_fmaf(-x, q, 127.0f), y, q);
}
__device__ __forceinline__ void q8_scales(float amax, float &d, float &id) {
    d = div127(amax);
    if (__builtin_expect(amax >= 0x1p-101f && amax < 0x1p101f, 1))
        id = div127r(amax);
    else
        id = amax != 0.f ? 127.f / amax : 0.f;
}

// ---------------------------------------------------------------------------
// Activation block store: one 32-element block of one row, in the format the
// next matmul consumes (ggml quantize_row_q8_0 / q8_1 AVX2 semantics:
// d = amax/127, q = rint(x * (127/amax)); fp16 RNE; or f32).
template <int WT>
__device__ __forceinline__ void store_act_block(const ActPtr &A, int64_t ld, int64_t row, int blk, const float *v) {
    if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 32; j++) amax = fmaxf(amax, fabsf(v[j]));
        float d, id;
        q8_scales(amax, d, id);
        uint32_t pk[8];
#pragma unroll
        for (int w = 0; w < 8; w++) pk[w] = q8_pack4(v[4 * w], v[4 * w + 1], v[4 * w + 2], v[4 * w + 3], id);
        uint4 *dst = (uint4 *)((int8_t *)A.q + row * ld + blk * 32);
        dst[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        dst[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
        if constexpr (WT == W_Q4_0) {
            ((uint16_t *)A.d)[row * (ld / 32) + blk] = f2h(d);
        } else {
            ((float *)A.d)[row * (ld / 32) + blk] = d;  // Q8_1's s = d*sum(q) is not needed: m_w is in the split W
        }
    } else if constexpr (WT == W_F16) {
        half8 *dst = (half8 *)((_Float16 *)A.q + row * ld + blk * 32);
#pragma unroll
        for (int w = 0; w < 4; w++) {
            half8 h;
#pragma unroll
            for (int j = 0; j < 8; j++) h[j] = (_Float16)v[8 * w + j];
            dst[w] = h;
        }
    } else {
        float4v *dst = (float4v *)((float *)A.q + row * ld + blk * 32);
#pragma unroll
        for (int w = 0; w < 8; w++) dst[w] = float4v{v[4 * w], v[4 * w + 1], v[4 * w + 2], v[4 * w + 3]};
    }
}

// The same for one quarter (8 elements) of a block: the four quarters of a
// block are four adjacent lanes (t & 3), all active; the block's amax is
// combined with two xor-shuffles, so each lane needs only its own 8 values.
template <int WT>
__device__ __forceinline__ void store_act_quarter(const ActPtr &A, int64_t ld, int64_t row, int blk, int qq,
                                                  const float *v) {
    if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 8; j++) amax = fmaxf(amax, fabsf(v[j]));
        amax = fmaxf(amax, __shfl_xor(amax, 1));
        amax = fmaxf(amax, __shfl_xor(amax, 2));
        float d, id;
        q8_scales(amax, d, id);
        uint32_t pk[2];
#pragma unroll
        for (int w = 0; w < 2; w++) pk[w] = q8_pack4(v[4 * w], v[4 * w + 1], v[4 * w + 2], v[4 * w + 3], id);
        *(uint2 *)((int8_t *)A.q + row * ld + blk * 32 + 8 * qq) = make_uint2(pk[0], pk[1]);
        if (qq == 0) {
            if constexpr (WT == W_Q4_0)
                ((uint16_t *)A.d)[row * (ld / 32) + blk] = f2h(d);
            else
                ((float *)A.d)[row * (ld / 32) + blk] = d;
        }
    } else if constexpr (WT == W_F16) {
        half8 h;
#pragma unroll
        for (int j = 0; j < 8; j++) h[j] = (_Float16)v[j];
        *(half8 *)((_Float16 *)A.q + row * ld + blk * 32 + 8 * qq) = h;
    } else {
        float4v *dst = (float4v *)((float *)A.q + row * ld + blk * 32 + 8 * qq);
        dst[0] = float4v{v[0], v[1], v[2], v[3]};
        dst[1] = float4v{v[4], v[5], v[6], v[7]};
    }
}

// The same for a quarter held in the transposed MFMA layout: the four
// quarters of a block are lanes c16, c16 + 16, c16 + 32, c16 + 48 (qq = lane
// >> 4), so the amax is combined with the two row-swapping permutes (VALU, no
// LDS round trip).
template <int WT>
__device__ __forceinline__ void store_act_quarter_t(const ActPtr &A, int64_t ld, int64_t row, int blk, int qq,
                                                    const float *v) {
    static_assert(WT == W_Q4_0 || WT == W_Q4_1, "Q8 activation formats only");
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 8; j++) amax = fmaxf(amax, fabsf(v[j]));
    {
        const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
        amax = fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
    }
    {
        const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
        amax = fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
    }
    float d, id;
    q8_scales(amax, d, id);
    const uint32_t p0 = q8_pack4(v[0], v[1], v[2], v[3], id), p1 = q8_pack4(v[4], v[5], v[6], v[7], id);
    *(uint2 *)((int8_t *)A.q + row * ld + blk * 32 + 8 * qq) = make_uint2(p0, p1);
    if (qq == 0) {
        if constexpr (WT == W_Q4_0)
            ((uint16_t *)A.d)[row * (ld / 32) + blk] = f2h(d);
        else
            ((float *)A.d)[row * (ld / 32) + blk] = d;
    }
}

// ggml's fp16 GELU table through its LDS-resident pair view (kernels.h
// HalfTable): entry m < cap + 1 holds table[m] (low half) and table[0x8000 | m]
// (high half); the host verified every finite pattern: negative magnitudes
// beyond cap read entry cap (ggml's constant run), positive ones beyond cap are
// h itself (identity run).  Branch-free: and, min, read, shift, select.
// Non-finite inputs (which b + W.x with finite weights cannot produce) follow
// their sign's rule instead of ggml's NaN.
__device__ __forceinline__ uint32_t gelu_lookup(const uint32_t *pair, uint32_t cap, uint32_t h) {
    const uint32_t v = pair[min(h & 0x7fffu, cap)] >> ((h >> 11) & 16u);
    return (h - (cap + 1u) < 0x8000u - (cap + 1u)) ? h : v;  // low 16 bits are the result
}

}  // namespace bertamd
