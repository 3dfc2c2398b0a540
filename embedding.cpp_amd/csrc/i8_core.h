// i8_core.h — the int8-MFMA building blocks of the Q4 x Q8 GEMMs (gemm_i8.hip)
// shared with the fused QKV + attention kernel (kernels.hip): the A-chunk LDS
// layout and staging, the weight ring, the per-block isum / d_w d_a / fold
// step and the chunk-staged main loop.  See gemm_i8.hip for the arithmetic
// (ggml_vec_dot_q4_x_q8_x restated per block).
#pragma once
#include "kernels_common.h"

namespace bertamd {

// Q4_1 per-block fold order: 1 = ggml's plain-C vec_dot_q4_1_q8_1 exactly
// (sumf += fmaf(d_w d_a, isum, m_w s_a), in block order), 0 = the m_w s_a
// terms accumulated two blocks at a time on the f32 MFMA (one fma per output
// per block).  See DESIGN.md §4 (which ggml build the GPU lands on).
#ifndef I8_Q41_GENERIC
#define I8_Q41_GENERIC 0
#endif
// W_Q4_1B (kernels.h): Q4_1's scale products on the bf16 MFMA — d_w * d_a and
// m_w * s_a (fp16 x f32) as sums of exact bf16 x bf16 partial products (d_w =
// w0 + w1, d_a = a0 + a1 + a2 in bf16 parts) in one v_mfma_f32_32x32x16_bf16
// (32 cycles) instead of the f32 MFMA (64 cycles per 32 x 32 tile); the d_a /
// s_a parts are made once per chunk when the A chunk is staged (I8Chunk holds
// them as packed 16-byte MFMA operands).  tools/mfma_bf16_split_probe.hip
// checks the rounding on the device.

typedef int int4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef int int16v __attribute__((ext_vector_type(16)));


// FFN-up kernel shape: waves per workgroup, f-tiles and t-tiles per wave
// (tools/i8_bench sweeps them; 8 x 2 x 2 measured best)
constexpr int I8_KC = 128;          // K per LDS chunk: 4 quant blocks (one scale vector)
constexpr int I8_LDQ = I8_KC + 16;  // token row stride of the LDS chunk, bytes: ds_read_b128 conflict-free

template <int BM, bool Q1, bool BF = false>
struct I8Chunk {
    static constexpr bool BFS = Q1 && BF;  // Q8_1 scales as packed bf16-part operands (W_Q4_1B)
    static constexpr int QB = BM * I8_LDQ;          // int8 q [BM][LDQ]
    // d_a [4][BM]: fp16 (Q8_0) | f32 (Q8_1) | 16-byte bf16-part operand (BFS)
    static constexpr int DB = 4 * BM * (BFS ? 16 : Q1 ? 4 : 2);
    // s_a [4][BM] (Q8_1: s = d * sum q, ggml quantize_row_q8_1): f32 | 16-byte operand (BFS)
    static constexpr int SB = Q1 ? 4 * BM * (BFS ? 16 : 4) : 0;
    static constexpr int BYTES = QB + DB + SB;
};

// x = p0 + p1 + p2 exactly as bf16 values (x has <= 24 significant bits), as
// the packed MFMA operand {p0, p1, p2, p0, p1, p2, 0, 0}; the weight side is
// {w0, w0, w0, w1, w1, w1, 0, 0} (i8_wparts), so k = 0..5 hold the six cross
// products of the two splits
__device__ __forceinline__ int4v i8_aparts(float x) {
    const uint32_t b = __float_as_uint(x), h0 = b >> 16;
    const float r = x - __uint_as_float(b & 0xffff0000u);  // exact
    const uint32_t br = __float_as_uint(r), h1 = br >> 16;
    const uint32_t h2 = __float_as_uint(r - __uint_as_float(br & 0xffff0000u)) >> 16;  // exact, <= 8 bits
    return int4v{(int)(h0 | (h1 << 16)), (int)(h2 | (h0 << 16)), (int)(h1 | (h2 << 16)), 0};
}
// an fp16-valued weight scale (<= 11 significant bits) as {w0, w0, w0, w1, w1, w1, 0, 0}
__device__ __forceinline__ int4v i8_wparts(float w) {
    const uint32_t b = __float_as_uint(w), h0 = b >> 16;
    const uint32_t h1 = __float_as_uint(w - __uint_as_float(b & 0xffff0000u)) >> 16;  // exact
    return int4v{(int)(h0 | (h0 << 16)), (int)(h0 | (h1 << 16)), (int)(h1 | (h1 << 16)), 0};
}

// The (token, block) items of an A chunk in flight: 32 q bytes + d each
// (separate arrays: an array of structs carried across the chunk loop was
// left in scratch by the compiler).
template <int IT>
struct I8Items {
    int4v q0[IT], q1[IT];
    float d[IT];         // Q8_1
    uint16_t d16[IT];    // Q8_0
};

template <int WT, int BM, int NT>
__device__ __forceinline__ void i8_stage_load(I8Items<(4 * BM + NT - 1) / NT> &st, const ActPtr &A, int K, int64_t m0,
                                              int k0) {
    constexpr int IT = (4 * BM + NT - 1) / NT;
#pragma unroll
    for (int it = 0; it < IT; it++) {
        // unconditional (surplus threads re-load item % (4 BM)): exact wait counts
        int item = (threadIdx.x + it * NT) % (4 * BM);
        asm volatile("" : "+v"(item));  // addresses built here, not hoisted out of the loop (spills)
        {
            const int r = item >> 2, bb = item & 3;
            const int64_t row = m0 + r;
            const int4v *p = (const int4v *)((const int8_t *)A.q + row * K + k0 + 32 * bb);
            st.q0[it] = p[0];
            st.q1[it] = p[1];
            const int64_t bi = row * (K >> 5) + (k0 >> 5) + bb;
            if constexpr (WT == W_Q4_0)
                st.d16[it] = ((const uint16_t *)A.d)[bi];
            else
                st.d[it] = ((const float *)A.d)[bi];
        }
    }
}

template <int WT, int BM, int NT>
__device__ __forceinline__ void i8_stage_store(const I8Items<(4 * BM + NT - 1) / NT> &st, char *buf) {
    constexpr int IT = (4 * BM + NT - 1) / NT;
    using C = I8Chunk<BM, wt_q41(WT), WT == W_Q4_1B>;
#pragma unroll
    for (int it = 0; it < IT; it++) {
        int item = threadIdx.x + it * NT;
        asm volatile("" : "+v"(item));
        if (4 * BM % NT == 0 || item < 4 * BM) {
            const int r = item >> 2, bb = item & 3;
            int4v *q = (int4v *)(buf + r * I8_LDQ + 32 * bb);
            q[0] = st.q0[it];
            q[1] = st.q1[it];
            if constexpr (WT == W_Q4_0)
                ((uint16_t *)(buf + C::QB))[bb * BM + r] = st.d16[it];
            else if constexpr (!C::BFS)
                ((float *)(buf + C::QB))[bb * BM + r] = st.d[it];
            if constexpr (wt_q41(WT)) {
                // ggml quantize_row_q8_1: s = d * (float) sum_j q_j (int sum, f32 product)
                const int4v a = st.q0[it], b = st.q1[it];
                int s = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) s = __builtin_amdgcn_sdot4(a[j], 0x01010101, s, false);
#pragma unroll
                for (int j = 0; j < 4; j++) s = __builtin_amdgcn_sdot4(b[j], 0x01010101, s, false);
                const float sv = st.d[it] * (float)s;
                if constexpr (C::BFS) {
                    ((int4v *)(buf + C::QB))[bb * BM + r] = i8_aparts(st.d[it]);
                    ((int4v *)(buf + C::QB + C::DB))[bb * BM + r] = i8_aparts(sv);
                } else {
                    ((float *)(buf + C::QB + C::DB))[bb * BM + r] = sv;
                }
            }
        }
    }
}

// Weight fragment of f-tile ft, block b: 16 bytes per lane.
__device__ __forceinline__ int4v i8_wq(const I8W &W, int nkb, int ft, int b) {
    return ((const int4v *)W.q)[((int64_t)ft * nkb + b) * 64 + (threadIdx.x & 63)];
}
// f32 scale vector (4 blocks) of weight row (lane & 31) of f-tile ft, group g.
__device__ __forceinline__ float4v i8_wvec(const float *v, int nkb, int ft, int g) {
    return ((const float4v *)v)[((int64_t)ft * (nkb >> 2) + g) * 32 + (threadIdx.x & 31)];
}

// Per-block operands of the activation side, read from the LDS chunk one
// block ahead of their MFMAs: the Q8 fragment and the block scale — Q4_0: the
// one-hot fp16 operand of the d_w * d_a MFMA (d_a at k = BB, lanes 32-63
// zero); Q4_1: d_a as f32 for the f32 MFMA.
template <int T>
struct I8AOps {
    int4v xa[T];
    uint32_t d16[T];  // Q4_0: fp16 d_a (the one-hot operand is built where it is used)
    float da[T];      // Q4_1
    int4v dp[T];      // W_Q4_1B: d_a as its bf16-part operand
};

template <int WT, int BM, int T, int BB>
__device__ __forceinline__ void i8_aops(I8AOps<T> &o, const char *buf, int tt0) {
    using C = I8Chunk<BM, wt_q41(WT), WT == W_Q4_1B>;
    const int lane = threadIdx.x & 63, l32 = lane & 31, hh = lane >> 5;
#pragma unroll
    for (int t = 0; t < T; t++) {
        const int r = 32 * (tt0 + t) + l32;
        o.xa[t] = *(const int4v *)(buf + r * I8_LDQ + 32 * BB + 16 * hh);
        if constexpr (WT == W_Q4_0) {
            o.d16[t] = ((const uint16_t *)(buf + C::QB))[BB * BM + r];
        } else if constexpr (C::BFS) {
            o.dp[t] = ((const int4v *)(buf + C::QB))[BB * BM + r];
        } else {
            o.da[t] = ((const float *)(buf + C::QB))[BB * BM + r];
        }
    }
}

// Pipeline state carried from block to block and across the tiles of a
// persistent workgroup.  Weight fragments stream through a 4-slot register
// ring (slot = block & 3), two blocks ahead; the A chunk (and the chunk's
// weight scales) are loaded in the middle of the previous chunk.  Every load
// is unconditional and issued in the order it is consumed, so each wait is
// an exact vmcnt (an older slow A load never blocks a younger weight wait).
// The last blocks of a tile load the first blocks / chunk of the workgroup's
// next tile.
// AH: weight blocks in flight ahead of the block being computed (2: a slot is
// refilled two blocks after it is consumed; 3: one block after — the lead of a
// 6-slot ring with the registers of 4, where the kernel's register budget has
// room for the longer live ranges).
template <int WT, int NT, int BM, int F, int AH = 2>
struct I8Pipe {
    static_assert(AH == 2 || AH == 3, "2 or 3 weight blocks ahead");
    static constexpr int IT = (4 * BM + NT - 1) / NT;
    I8Items<IT> st;
    int4v wf[4][F];
    uint2 wr[F];             // Q4_0: fp16 d_w of the chunk's 4 blocks
    float4v wdr[F], wmr[F];  // Q4_1: f32 d_w, m_w

    // weight fragments of block b (of the tile at ft0 when b < nkb, else
    // block b - nkb of the next tile at ft0n) into ring slot S
    template <int S>
    __device__ __forceinline__ void wload(const GemmArgs &g, int nkb, int ft0, int ft0n, int b) {
        const bool nx = b >= nkb;
        const int ft = nx ? ft0n : ft0, bb = nx ? b - nkb : b;
#pragma unroll
        for (int f = 0; f < F; f++) wf[S][f] = i8_wq(g.Wi, nkb, ft + f, bb);
    }
    // A chunk c of the tile at m0 and the weight scales of that chunk
    __device__ __forceinline__ void cload(const GemmArgs &g, int64_t m0, int ft0, int c) {
        const int lane = threadIdx.x & 63, nkb = g.K >> 5;
        i8_stage_load<WT, BM, NT>(st, g.A, g.K, m0, c * I8_KC);
#pragma unroll
        for (int f = 0; f < F; f++) {
            if constexpr (wt_q41(WT)) {
                wdr[f] = i8_wvec(g.Wi.d, nkb, ft0 + f, c);
                wmr[f] = i8_wvec(g.Wi.m, nkb, ft0 + f, c);
            } else {
                wr[f] = ((const uint2 *)g.Wi.dh)[((int64_t)(ft0 + f) * (nkb >> 2) + c) * 32 + (lane & 31)];
            }
        }
    }
    // first loads of a tile (before its main loop, in consumption order)
    __device__ __forceinline__ void prime(const GemmArgs &g, int64_t m0, int ft0) {
        const int nkb = g.K >> 5;
        wload<0>(g, nkb, ft0, ft0, 0);
        wload<1>(g, nkb, ft0, ft0, 1);
        if constexpr (AH == 3) wload<2>(g, nkb, ft0, ft0, 2);
        cload(g, m0, ft0, 0);
    }
};

// One quant block (BB = its index inside the chunk) of the main loop, with
// its activation operands `cur` (the next block's are read into `nxt`).
template <int WT, int BM, int F, int T, int BB, bool PIPE>
__device__ __forceinline__ void i8_block(const char *buf, int tt0, const int4v (&wfc)[F], const int4v (&ws)[F],
                                         const float4v (&wd)[F], const float4v (&wm)[F], const I8AOps<T> &cur,
                                         I8AOps<T> &nxt, float16v (&acc)[F][T]) {
    using C = I8Chunk<BM, wt_q41(WT), WT == W_Q4_1B>;
    const int lane = threadIdx.x & 63, l32 = lane & 31, hh = lane >> 5;
    const float16v zf = {};
    if constexpr (BB < 3) i8_aops<WT, BM, T, BB + 1>(nxt, buf, tt0);
#if I8_Q41_GENERIC
    // ggml's plain-C ggml_vec_dot_q4_1_q8_1 per block: sumf += fmaf(d_w d_a,
    // (float) isum, m_w * s_a) — m_w * s_a rounded on its own (the f32 MFMA with
    // one nonzero product per output), then one fma and one add per output
    float16v ms[F][T];
    if constexpr (wt_q41(WT)) {
        const float *sbuf = (const float *)(buf + C::QB + C::DB);
#pragma unroll
        for (int t = 0; t < T; t++) {
            const float sa = sbuf[BB * BM + 32 * (tt0 + t) + l32];
#pragma unroll
            for (int f = 0; f < F; f++)
                ms[f][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(hh ? 0.f : wm[f][BB], sa, zf, 0, 0, 0);
        }
    }
#else
    if constexpr (wt_q41(WT) && (BB & 1)) {
        if constexpr (C::BFS) {
            // m_w * s_a of blocks b - 1 (k = 0..5, lanes 0-31) and b (k = 8..13, lanes
            // 32-63) as bf16 partial products, one bf16 MFMA
            const int4v *sbuf = (const int4v *)(buf + C::QB + C::DB);
            int4v mp[F];
#pragma unroll
            for (int f = 0; f < F; f++) mp[f] = i8_wparts(hh ? wm[f][BB] : wm[f][BB - 1]);
#pragma unroll
            for (int t = 0; t < T; t++) {
                const int4v sp = sbuf[(BB - 1 + hh) * BM + 32 * (tt0 + t) + l32];
#pragma unroll
                for (int f = 0; f < F; f++)
                    acc[f][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, mp[f]),
                                                                        __builtin_bit_cast(bf16x8, sp), acc[f][t], 0, 0, 0);
            }
        } else {
            // m_w * s_a of blocks b - 1 (k = 0, lanes 0-31) and b (k = 1, lanes 32-63)
            const float *sbuf = (const float *)(buf + C::QB + C::DB);
#pragma unroll
            for (int t = 0; t < T; t++) {
                const float sa = sbuf[(BB - 1 + hh) * BM + 32 * (tt0 + t) + l32];
#pragma unroll
                for (int f = 0; f < F; f++)
                    acc[f][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(hh ? wm[f][BB] : wm[f][BB - 1], sa, acc[f][t], 0, 0, 0);
            }
        }
    }
#endif
    // dd = d_w * d_a, exact: Q4_0 fp16 x fp16 on the f16 MFMA (ws: the f-tile's
    // four block scales at k = 0..3, oh: d_a one-hot at k = BB); Q4_1 f32 x f32
    // on the f32 MFMA
    int4v oh[T];
    if constexpr (WT == W_Q4_0) {
#pragma unroll
        for (int t = 0; t < T; t++) {
            const uint32_t v = hh ? 0u : ((BB & 1) ? cur.d16[t] << 16 : cur.d16[t]);
            oh[t] = int4v{0, 0, 0, 0};
            oh[t][BB >> 1] = (int)v;
        }
    }
    int4v wp[F];  // W_Q4_1B: d_w of block BB as its bf16-part operand (zero in lanes 32-63, as wd)
    if constexpr (C::BFS) {
#pragma unroll
        for (int f = 0; f < F; f++) wp[f] = i8_wparts(wd[f][BB]);
    }
    auto ddmfma = [&](int f, int t) {
        if constexpr (WT == W_Q4_0) {
            return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, ws[f]),
                                                          __builtin_bit_cast(half8, oh[t]), zf, 0, 0, 0);
        } else if constexpr (C::BFS) {
            return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wp[f]),
                                                           __builtin_bit_cast(bf16x8, cur.dp[t]), zf, 0, 0, 0);
        } else {
            return __builtin_amdgcn_mfma_f32_32x32x2f32(wd[f][BB], cur.da[t], zf, 0, 0, 0);
        }
    };
    // software pipeline over the F x T tiles: tile p + 1's two MFMAs are in
    // flight while tile p is folded
    // (PIPE false: issue and fold tile by tile; latency left to other waves)
    int16v is[2];
    float16v dd[2];
    is[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wfc[0], cur.xa[0], __builtin_bit_cast(int16v, zf), 0, 0, 0);
    dd[0] = ddmfma(0, 0);
#pragma unroll
    for (int p = 0; p < F * T; p++) {
        if (!PIPE && p > 0) {
            is[p & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wfc[p / T], cur.xa[p % T], __builtin_bit_cast(int16v, zf),
                                                              0, 0, 0);
            dd[p & 1] = ddmfma(p / T, p % T);
        }
        if (PIPE && p + 1 < F * T) {
            is[(p + 1) & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wfc[(p + 1) / T], cur.xa[(p + 1) % T],
                                                                     __builtin_bit_cast(int16v, zf), 0, 0, 0);
            dd[(p + 1) & 1] = ddmfma((p + 1) / T, (p + 1) % T);
        }
        // tile p + 1's MFMAs are issued before tile p's fold reads tile p's
        // results (left to itself the scheduler folds right behind the MFMA
        // that produces the operands and waits out its latency)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 16; i++) {
            // (one v_fma_f32 per output: the packed v_pk_fma_f32 fold measured slower
            // in every kernel, round 5 — DESIGN.md §3 "What bounds the GEMMs")
#if I8_Q41_GENERIC
            float v;
            if constexpr (wt_q41(WT))
                v = acc[p / T][p % T][i] + __builtin_fmaf((float)is[p & 1][i], dd[p & 1][i], ms[p / T][p % T][i]);
            else
                v = __builtin_fmaf((float)is[p & 1][i], dd[p & 1][i], acc[p / T][p % T][i]);
#else
            float v = __builtin_fmaf((float)is[p & 1][i], dd[p & 1][i], acc[p / T][p % T][i]);
#endif
            asm volatile("" : "+v"(v));  // keep the fold here: sunk past the MFMAs it would keep every tile live
            acc[p / T][p % T][i] = v;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

struct I8NoHook {
    __device__ __forceinline__ void operator()(int, int) const {}
};

// acc[f][t] = A[m0 + 32 (tt0 + t) ..][:] . W[32 (ft0 + f) ..][:]^T over the
// whole K for this wave's F f-tiles x T t-tiles (tokens of the workgroup's
// BM-row tile, staged through `smem`, 2 * I8Chunk::BYTES).  `pp` holds this
// tile's first loads on entry (I8Pipe::prime) and the next tile's (m0n,
// ft0n) on return.  Returns after a final barrier (the LDS may be reused).
// hook(c, nch) runs at the start of every chunk c, after that chunk's barrier
// (memory traffic of the caller's epilogue interleaved with the main loop).
template <int WT, int NT, int BM, int F, int T, bool PIPE = true, typename Hook = I8NoHook, int AH = 2>
__device__ __forceinline__ void i8_mainloop(const GemmArgs &g, int64_t m0, int ft0, int tt0, int64_t m0n, int ft0n,
                                            char *smem, I8Pipe<WT, NT, BM, F, AH> &pp, float16v (&acc)[F][T],
                                            const Hook &hook = Hook()) {
    constexpr bool Q1 = wt_q41(WT);
    using C = I8Chunk<BM, Q1, WT == W_Q4_1B>;
    const int lane = threadIdx.x & 63, hh = lane >> 5;
    const int nkb = g.K >> 5, nch = g.K / I8_KC;
    const float4v z4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int f = 0; f < F; f++)
#pragma unroll
        for (int t = 0; t < T; t++) acc[f][t] = float16v{};
    int4v ws[F];
    float4v wd[F], wm[F];
    auto wscale_use = [&]() {
#pragma unroll
        for (int f = 0; f < F; f++) {
            if constexpr (Q1) {
                wd[f] = hh ? z4 : pp.wdr[f];  // d_w: rows at k = 0 (lanes 0-31), zero at k = 1 (lanes 32-63)
                wm[f] = pp.wmr[f];            // m_w: both lane halves (two blocks per MFMA)
            } else {
                // the four fp16 d_w of the chunk's blocks at k = 0..3 (k = 4..7: a finite copy)
                ws[f] = int4v{(int)pp.wr[f].x, (int)pp.wr[f].y, (int)pp.wr[f].x, (int)pp.wr[f].y};
            }
        }
    };
    i8_stage_store<WT, BM, NT>(pp.st, smem);
    wscale_use();
    __syncthreads();

    for (int c = 0; c < nch; c++) {
        const bool more = c + 1 < nch;
        const int b0 = 4 * c;
        const char *buf = smem + (c & 1) * C::BYTES;
        hook(c, nch);
        I8AOps<T> a0, a1;
        i8_aops<WT, BM, T, 0>(a0, buf, tt0);
        constexpr int A = AH;
        i8_block<WT, BM, F, T, 0, PIPE>(buf, tt0, pp.wf[0], ws, wd, wm, a0, a1, acc);
        pp.template wload<(0 + A) & 3>(g, nkb, ft0, ft0n, b0 + 0 + A);
        i8_block<WT, BM, F, T, 1, PIPE>(buf, tt0, pp.wf[1], ws, wd, wm, a1, a0, acc);
        pp.template wload<(1 + A) & 3>(g, nkb, ft0, ft0n, b0 + 1 + A);
        pp.cload(g, more ? m0 : m0n, more ? ft0 : ft0n, more ? c + 1 : 0);
        i8_block<WT, BM, F, T, 2, PIPE>(buf, tt0, pp.wf[2], ws, wd, wm, a0, a1, acc);
        pp.template wload<(2 + A) & 3>(g, nkb, ft0, ft0n, b0 + 2 + A);
        i8_block<WT, BM, F, T, 3, PIPE>(buf, tt0, pp.wf[3], ws, wd, wm, a1, a0, acc);
        pp.template wload<(3 + A) & 3>(g, nkb, ft0, ft0n, b0 + 3 + A);
        if (more) {
            i8_stage_store<WT, BM, NT>(pp.st, smem + ((c + 1) & 1) * C::BYTES);
            wscale_use();
        }
        __syncthreads();
    }
}

// Q8 block of 32 consecutive outputs held as 16 per lane by lanes l and
// l ^ 32 (same token): ggml quantize_row_q8_0 / q8_1 (d = amax/127,
// q = rint(x * 127/amax)); lane half hh stores bytes 16 hh .. 16 hh + 15.
template <int WT>
__device__ __forceinline__ void i8_store_q8_half(const ActPtr &out, int64_t ld, int64_t row, int blk, int hh,
                                                 const float (&y)[16]) {
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 16; i++) amax = fmaxf(amax, fabsf(y[i]));
    {
        const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
        amax = fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
    }
    float d, id;
    q8_scales(amax, d, id);
    uint4 pk;
    pk.x = q8_pack4(y[0], y[1], y[2], y[3], id);
    pk.y = q8_pack4(y[4], y[5], y[6], y[7], id);
    pk.z = q8_pack4(y[8], y[9], y[10], y[11], id);
    pk.w = q8_pack4(y[12], y[13], y[14], y[15], id);
    *(uint4 *)((int8_t *)out.q + row * ld + 32 * blk + 16 * hh) = pk;
    if (hh == 0) {
        if constexpr (WT == W_Q4_0)
            ((uint16_t *)out.d)[row * (ld >> 5) + blk] = f2h(d);
        else
            ((float *)out.d)[row * (ld >> 5) + blk] = d;
    }
}

// XCD-aware tile order (as gemm_kernel): linear ids are dealt round-robin over
// the 8 XCDs; each XCD walks a contiguous range, n fastest.
__device__ __forceinline__ int xcd_linear(int orig, int nwg) {
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
}

}  // namespace bertamd

namespace bertamd {

// Main loop over an A panel resident in LDS: K / I8_KC chunks in the I8Chunk
// layout, back to back from `apanel` (BM rows each).  No staging and no
// barriers, so a subset of a workgroup's waves can run it while the others do
// something else (qkv_attention_pc_kernel).  Weight fragments stream through
// the same 4-slot register ring as i8_mainloop, two blocks ahead, the weight
// scales one chunk ahead; the block step is i8_block, so the sums are the
// chunk-staged main loop's, bit for bit.  The ring lives in the caller
// (I8ResRing) and runs across calls: ring.start(g, ft) loads f-tile ft's first
// two blocks and scales; each call consumes the ring for ft0 and, when ftn >= 0,
// refills it with f-tile ftn's first blocks and scales at its end, so their
// L2 latency passes during whatever the caller does between two calls.
template <int WT, int F, int AH = 2>
struct I8ResRing {
    int4v wf[4][F];
    uint2 wr[F];
    float4v wdr[F], wmr[F];
    // Every load is unconditional (a block / chunk past the end reloads the
    // last one, and the caller drops it), so the compiler's waits stay exact
    // vmcnt counts: behind a conditional load the control-flow merge made it
    // wait for vmcnt(0) — for the refill just issued — before the next block.
    __device__ __forceinline__ void wload(const GemmArgs &g, int slot, int ft0, int b) {
        const int nkb = g.K >> 5, bb = b < nkb ? b : nkb - 1;
#pragma unroll
        for (int f = 0; f < F; f++) wf[slot][f] = i8_wq(g.Wi, nkb, ft0 + f, bb);
    }
    __device__ __forceinline__ void sload(const GemmArgs &g, int ft0, int c) {  // weight scales of chunk c (4 blocks)
        const int nkb = g.K >> 5, nch = g.K / I8_KC, lane = threadIdx.x & 63, cc = c < nch ? c : nch - 1;
#pragma unroll
        for (int f = 0; f < F; f++) {
            if constexpr (wt_q41(WT)) {
                wdr[f] = i8_wvec(g.Wi.d, nkb, ft0 + f, cc);
                wmr[f] = i8_wvec(g.Wi.m, nkb, ft0 + f, cc);
            } else {
                wr[f] = ((const uint2 *)g.Wi.dh)[((int64_t)(ft0 + f) * (nkb >> 2) + cc) * 32 + (lane & 31)];
            }
        }
    }
    __device__ __forceinline__ void start(const GemmArgs &g, int ft0) {
        wload(g, 0, ft0, 0);
        wload(g, 1, ft0, 1);
        if constexpr (AH == 3) wload(g, 2, ft0, 2);
        sload(g, ft0, 0);
    }
};

template <int WT, int BM, int F, int T, int AH>
__device__ __forceinline__ void i8_resident_mainloop(const GemmArgs &g, const char *apanel, int ft0, int tt0,
                                                     float16v (&acc)[F][T], I8ResRing<WT, F, AH> &ring, int ftn) {
    constexpr bool Q1 = wt_q41(WT);
    using C = I8Chunk<BM, Q1, WT == W_Q4_1B>;
    const int lane = threadIdx.x & 63, hh = lane >> 5;
    const int nch = g.K / I8_KC;
    const float4v z4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int f = 0; f < F; f++)
#pragma unroll
        for (int t = 0; t < T; t++) acc[f][t] = float16v{};
    int4v ws[F];
    float4v wd[F], wm[F];
    auto wscale_use = [&]() {
#pragma unroll
        for (int f = 0; f < F; f++) {
            if constexpr (Q1) {
                wd[f] = hh ? z4 : ring.wdr[f];
                wm[f] = ring.wmr[f];
            } else {
                ws[f] = int4v{(int)ring.wr[f].x, (int)ring.wr[f].y, (int)ring.wr[f].x, (int)ring.wr[f].y};
            }
        }
    };
#pragma unroll 1
    for (int c = 0; c < nch; c++) {
        const int b0 = 4 * c;
        const bool last = c + 1 == nch;
        const char *buf = apanel + c * C::BYTES;
        wscale_use();
        // the next chunk's scales, or the next f-tile's first (none: f-tile ft0's again, dropped)
        ring.sload(g, last && ftn >= 0 ? ftn : ft0, last ? 0 : c + 1);
        I8AOps<T> a0, a1;
        i8_aops<WT, BM, T, 0>(a0, buf, tt0);
        // block b0 + j + A into slot (j + A) & 3; past the f-tile's last block,
        // the first blocks of f-tile ftn
        constexpr int A = AH;
        auto refill = [&](int j) {
            const int b = b0 + j + A;
            const bool nx = b >= 4 * nch;
            ring.wload(g, (j + A) & 3, nx && ftn >= 0 ? ftn : ft0, nx ? b - 4 * nch : b);
        };
        i8_block<WT, BM, F, T, 0, true>(buf, tt0, ring.wf[0], ws, wd, wm, a0, a1, acc);
        refill(0);
        i8_block<WT, BM, F, T, 1, true>(buf, tt0, ring.wf[1], ws, wd, wm, a1, a0, acc);
        refill(1);
        i8_block<WT, BM, F, T, 2, true>(buf, tt0, ring.wf[2], ws, wd, wm, a0, a1, acc);
        refill(2);
        i8_block<WT, BM, F, T, 3, true>(buf, tt0, ring.wf[3], ws, wd, wm, a1, a0, acc);
        refill(3);
    }
}

}  // namespace bertamd
