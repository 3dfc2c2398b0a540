// gemm_i8.hip — the Q4_0 / Q4_1 weight GEMMs on the gfx950 int8 MFMA.
//
// Replaces ggml_mul_mat over Q4 weights (reference bert.cpp:910-974: the
// QKV, O, FFN-up and FFN-down projections), whose CPU kernel is
// ggml_vec_dot_q4_x_q8_x: the activation row is
// quantised to Q8 blocks of 32 (d_a, q_a) and per block
//     sumf += (d_w * d_a) * (float) isum,   isum = sum_j q_w[j] * q_a[j]  (exact int32)
// (+ m_w * s_a for Q4_1).  Here, per 32 x 32 output tile and block:
//   isum = v_mfma_i32_32x32x32_i8(W_q, X_q)          exact, ggml's isum
//   dd   = v_mfma_f32_32x32x2_f32(d_w, d_a)          exact f32 product, ggml's d
//   acc  = fma((float) isum, dd, acc)                 ggml's fold (VALU)
// and for Q4_1 every two blocks acc += m_w * s_a through the same f32 MFMA.
// The weight nibbles are expanded to int8 once at load (runtime.cpp
// repack_i8: 1 B/weight + the f32 scale vectors); the scales are applied
// in-kernel per block, as ggml does.  Lane maps (checked on the device by
// tools/mfma_i8_probe.hip): lane (r = l & 31, h = l >> 5) holds bytes
// k = 16h .. 16h + 15 of weight row / token r; the 32 x 32 result holds
// C[row 8(i/4) + 4h + i%4][col r] in register i.  Weight row m of a 32-row
// tile is feature 16((m>>2)&1) + 4(m>>3) + (m&3) (repack_i8), so a lane holds
// 16 CONSECUTIVE output features 16h .. 16h+15 of one token: half of one
// output Q8 block, and the epilogues quantise in registers.
//
// Compiled with -ffp-contract=off: every fused multiply-add below is explicit.
#include "kernels_common.h"

#include <algorithm>
#include <cstdlib>

namespace bertamd {

typedef int int4v __attribute__((ext_vector_type(4)));
typedef int int16v __attribute__((ext_vector_type(16)));


// FFN-up kernel shape: waves per workgroup, f-tiles and t-tiles per wave
// (tools/i8_bench sweeps them; 8 x 2 x 2 measured best)
#ifndef I8_UP_WAVES
#define I8_UP_WAVES 8
#endif
#ifndef I8_UP_F
#define I8_UP_F 2
#endif
#ifndef I8_UP_T
#define I8_UP_T 2
#endif

constexpr int I8_KC = 128;          // K per LDS chunk: 4 quant blocks (one scale vector)
constexpr int I8_LDQ = I8_KC + 16;  // token row stride of the LDS chunk, bytes: ds_read_b128 conflict-free

template <int BM, bool Q1>
struct I8Chunk {
    static constexpr int QB = BM * I8_LDQ;          // int8 q [BM][LDQ]
    static constexpr int DB = 4 * BM * (Q1 ? 4 : 2);  // d_a [4][BM]: fp16 (Q8_0) | f32 (Q8_1)
    static constexpr int SB = Q1 ? 4 * BM * 4 : 0;  // f32 s_a [4][BM] (Q8_1: s = d * sum q, ggml quantize_row_q8_1)
    static constexpr int BYTES = QB + DB + SB;
};

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
    using C = I8Chunk<BM, WT == W_Q4_1>;
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
            else
                ((float *)(buf + C::QB))[bb * BM + r] = st.d[it];
            if constexpr (WT == W_Q4_1) {
                // ggml quantize_row_q8_1: s = d * (float) sum_j q_j (int sum, f32 product)
                const int4v a = st.q0[it], b = st.q1[it];
                int s = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) s = __builtin_amdgcn_sdot4(a[j], 0x01010101, s, false);
#pragma unroll
                for (int j = 0; j < 4; j++) s = __builtin_amdgcn_sdot4(b[j], 0x01010101, s, false);
                ((float *)(buf + C::QB + C::DB))[bb * BM + r] = st.d[it] * (float)s;
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
};

template <int WT, int BM, int T, int BB>
__device__ __forceinline__ void i8_aops(I8AOps<T> &o, const char *buf, int tt0) {
    using C = I8Chunk<BM, WT == W_Q4_1>;
    const int lane = threadIdx.x & 63, l32 = lane & 31, hh = lane >> 5;
#pragma unroll
    for (int t = 0; t < T; t++) {
        const int r = 32 * (tt0 + t) + l32;
        o.xa[t] = *(const int4v *)(buf + r * I8_LDQ + 32 * BB + 16 * hh);
        if constexpr (WT == W_Q4_0) {
            o.d16[t] = ((const uint16_t *)(buf + C::QB))[BB * BM + r];
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
template <int WT, int NT, int BM, int F>
struct I8Pipe {
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
            if constexpr (WT == W_Q4_1) {
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
        cload(g, m0, ft0, 0);
    }
};

// One quant block (BB = its index inside the chunk) of the main loop, with
// its activation operands `cur` (the next block's are read into `nxt`).
template <int WT, int BM, int F, int T, int BB, bool PIPE>
__device__ __forceinline__ void i8_block(const char *buf, int tt0, const int4v (&wfc)[F], const int4v (&ws)[F],
                                         const float4v (&wd)[F], const float4v (&wm)[F], const I8AOps<T> &cur,
                                         I8AOps<T> &nxt, float16v (&acc)[F][T]) {
    using C = I8Chunk<BM, WT == W_Q4_1>;
    const int lane = threadIdx.x & 63, l32 = lane & 31, hh = lane >> 5;
    const float16v zf = {};
    if constexpr (BB < 3) i8_aops<WT, BM, T, BB + 1>(nxt, buf, tt0);
    if constexpr (WT == W_Q4_1 && (BB & 1)) {
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
    auto ddmfma = [&](int f, int t) {
        if constexpr (WT == W_Q4_0)
            return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, ws[f]),
                                                          __builtin_bit_cast(half8, oh[t]), zf, 0, 0, 0);
        else
            return __builtin_amdgcn_mfma_f32_32x32x2f32(wd[f][BB], cur.da[t], zf, 0, 0, 0);
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
            float v = __builtin_fmaf((float)is[p & 1][i], dd[p & 1][i], acc[p / T][p % T][i]);
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
template <int WT, int NT, int BM, int F, int T, bool PIPE = true, typename Hook = I8NoHook>
__device__ __forceinline__ void i8_mainloop(const GemmArgs &g, int64_t m0, int ft0, int tt0, int64_t m0n, int ft0n,
                                            char *smem, I8Pipe<WT, NT, BM, F> &pp, float16v (&acc)[F][T],
                                            const Hook &hook = Hook()) {
    constexpr bool Q1 = WT == W_Q4_1;
    using C = I8Chunk<BM, Q1>;
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
        i8_block<WT, BM, F, T, 0, PIPE>(buf, tt0, pp.wf[0], ws, wd, wm, a0, a1, acc);
        pp.template wload<2>(g, nkb, ft0, ft0n, b0 + 2);
        i8_block<WT, BM, F, T, 1, PIPE>(buf, tt0, pp.wf[1], ws, wd, wm, a1, a0, acc);
        pp.template wload<3>(g, nkb, ft0, ft0n, b0 + 3);
        pp.cload(g, more ? m0 : m0n, more ? ft0 : ft0n, more ? c + 1 : 0);
        i8_block<WT, BM, F, T, 2, PIPE>(buf, tt0, pp.wf[2], ws, wd, wm, a0, a1, acc);
        pp.template wload<0>(g, nkb, ft0, ft0n, b0 + 4);
        i8_block<WT, BM, F, T, 3, PIPE>(buf, tt0, pp.wf[3], ws, wd, wm, a1, a0, acc);
        pp.template wload<1>(g, nkb, ft0, ft0n, b0 + 5);
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

// ---------------------------------------------------------------------------
// FFN up + GELU (bert.cpp:965-971): U = gelu(b + W.h) in the down GEMM's Q8
// format.  Persistent: one 12-wave workgroup per CU (3 waves per SIMD) walks
// 64 x 384 tiles; ggml's fp16 GELU table (entries [0, 0x8000 + neg_n],
// kernels.h GELU_FLAT_LDS) is read into LDS once.  Wave w: f-tile w of the
// tile (32 features), both 32-token t-tiles.
template <int WT, int NWV, int F, int T>
__global__ __launch_bounds__(NWV * 64) void i8_up_gelu_kernel(GemmArgs g, int n_mtiles, int n_ntiles) {
    constexpr int NT = NWV * 64, BM = 32 * T, BN = 32 * NWV * F;
    constexpr bool PIPE = NWV <= 12;
    using C = I8Chunk<BM, WT == W_Q4_1>;
    __shared__ __attribute__((aligned(16))) char smem[2 * C::BYTES];
    __shared__ __attribute__((aligned(16))) uint16_t gtab[GELU_FLAT_LDS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hh = lane >> 5;
    const int nflat8 = (0x8000 + g.gelu.neg_n + 1 + 7) / 8;
    for (int i = tid; i < nflat8; i += NT) ((uint4 *)gtab)[i] = ((const uint4 *)g.gelu.full)[i];
    const float xlo = h2f((uint16_t)(0x8000 | g.gelu.neg_n));
    const int nwg = n_mtiles * n_ntiles;
    const int fw = F * wv, tw = 0;
    auto coords = [&](int tile, int64_t &m0_, int &ft0_) {
        const int lin = xcd_linear(tile, nwg);
        const int mt = lin / n_ntiles, nt = lin - mt * n_ntiles;
        m0_ = (int64_t)mt * BM;
        ft0_ = nt * (BN / 32) + fw;
    };
    if ((int)blockIdx.x >= nwg) return;
    int64_t m0;
    int ft0;
    coords(blockIdx.x, m0, ft0);
    I8Pipe<WT, NT, BM, F> pp;
    pp.prime(g, m0, ft0);
    for (int tile = blockIdx.x, it = 0; tile < nwg; tile += gridDim.x, it++) {
        int64_t m0n = m0;
        int ft0n = ft0;
        if (tile + (int)gridDim.x < nwg) coords(tile + gridDim.x, m0n, ft0n);
        float16v acc[F][T];
        STAMP(it, 0, NWV);
        i8_mainloop<WT, NT, BM, F, T, PIPE>(g, m0, ft0, tw, m0n, ft0n, smem, pp, acc);
        STAMP(it, 1, NWV);
        const int64_t mc = m0;
        const int fc = ft0;
        m0 = m0n;
        ft0 = ft0n;
#pragma unroll
        for (int f = 0; f < F; f++) {
            const int col = 32 * (fc + f) + 16 * hh;
            float bias[16];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4v b4 = *(const float4v *)(g.bias + col + 4 * q);
#pragma unroll
                for (int j = 0; j < 4; j++) bias[4 * q + j] = b4[j];
            }
#pragma unroll
            for (int t = 0; t < T; t++) {
                float y[16];
#pragma unroll
                for (int i = 0; i < 16; i++) y[i] = h2f(gtab[f2h(fmaxf(bias[i] + acc[f][t][i], xlo))]);
                i8_store_q8_half<WT>(g.out_act, g.N, mc + 32 * (tw + t) + l32, fc + f, hh, y);
            }
        }
        STAMP(it, 2, NWV);
    }
}

// ---------------------------------------------------------------------------
// Projection + residual + LayerNorm for n_embd = 384 (bert.cpp:944-962 and
// :973-992): X = LN((b + W.x) + X), stored f32 and in the next GEMM's Q8
// format.  One 12-wave workgroup owns BM = 64 whole rows: wave w holds f-tile
// w (32 features) of both 32-token t-tiles, so a row's 384 values are spread
// over 12 waves x 2 lane halves x 16.  ggml_norm's double sums go lane ->
// lane pair -> the twelve waves (LDS partials, fixed order).
// The residual tile (64 rows x 384 f32, 96 KiB, contiguous in X) moves between
// HBM and the workgroup through LDS in whole 1 KiB pieces: in by LDS-DMA
// (global_load_lds_dwordx4, 8 per wave), out by 16-byte stores of consecutive
// threads — instead of each lane gathering and scattering its own row (32
// cache lines per wave instruction).  16-byte chunk c of row r sits at LDS
// chunk c ^ (r & 15), so the epilogue's row-per-lane reads are conflict-free.
// With OV (I8_LN_OV, default) that traffic overlaps the main loops: the tile's
// residual comes in piece by piece during its own main loop (LDS-DMA issued at
// the chunk starts), and the previous tile's LN output leaves xs during the same
// chunks, each wave draining one 1 KiB piece of xs to X just before refilling
// that piece with the new residual; the last tile's output leaves after the loop.
__device__ __forceinline__ int i8_xs_chunk(int r, int c) { return r * 96 + (c ^ (r & 15)); }

#ifndef I8_LN_OV
#define I8_LN_OV 1
#endif

template <int WT, bool OV = I8_LN_OV>
__global__ __launch_bounds__(768) void i8_ln384_kernel(GemmArgs g, int n_mtiles) {
    constexpr int NT = 768, BM = 64, F = 1, T = 2, NCOL = 384, NWV = 12;
    constexpr int XCH = BM * NCOL / 4;  // 16-byte chunks of the residual tile
    using C = I8Chunk<BM, WT == W_Q4_1>;
    __shared__ __attribute__((aligned(16))) char smem[2 * C::BYTES];
    __shared__ double red[2][NWV][BM];
    __shared__ __attribute__((aligned(16))) float xs[BM * NCOL];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hh = lane >> 5;
    const int ft0 = wv;
    const int col = 32 * ft0 + 16 * hh;
    if ((int)blockIdx.x >= n_mtiles) return;
    int64_t m0n = (int64_t)xcd_linear(blockIdx.x, n_mtiles) * BM;
    I8Pipe<WT, NT, BM, F> pp;
    pp.prime(g, m0n, ft0);
    // wave w's piece k: LDS chunks 64 (8 w + k) .. + 63 of xs, i.e. lane l holds
    // chunk j = 64 (8 w + k) + l = (row r, column chunk cs ^ (r & 15)) of the tile
    constexpr int PIECES = XCH / NT;  // 1 KiB pieces per wave
    auto piece_off = [&](int k, int &j0) {
        j0 = 64 * (8 * wv + k);
        const int j = j0 + lane, r = j / 96, cs = j - 96 * r;
        return r * NCOL + 4 * (cs ^ (r & 15));
    };
    auto dma_in = [&](const float *xt, int k) {
        int j0;
        const int off = piece_off(k, j0);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(xt + off),
                                         (__attribute__((address_space(3))) void *)(xs + 4 * j0), 16, 0, 0);
    };
    auto store_out = [&](float *xt, int k) {
        int j0;
        const int off = piece_off(k, j0);
        *(float4v *)(xt + off) = *(const float4v *)(xs + 4 * (j0 + lane));
    };
    int64_t mprev = -1;
    for (int tile = blockIdx.x, it = 0; tile < n_mtiles; tile += gridDim.x, it++) {
        const int64_t m0 = m0n;
        if (tile + (int)gridDim.x < n_mtiles) m0n = (int64_t)xcd_linear(tile + gridDim.x, n_mtiles) * BM;
        float16v acc[F][T];
        STAMP(it, 0, NWV);
        if constexpr (OV) {
            // chunk c drains and refills pieces c ppc .. (previous output out, this residual in)
            const float *xin = g.X + m0 * NCOL;
            float *xout = g.X + mprev * NCOL;
            const bool prev = mprev >= 0;
            auto hook = [&](int c, int nch) {
                const int ppc = (PIECES + nch - 1) / nch, k1 = min(PIECES, (c + 1) * ppc);
#pragma unroll 1
                for (int k = c * ppc; k < k1; k++) {
                    if (prev) store_out(xout, k);
                    dma_in(xin, k);
                }
            };
            i8_mainloop<WT, NT, BM, F, T>(g, m0, ft0, 0, m0n, ft0, smem, pp, acc, hook);
        } else {
            i8_mainloop<WT, NT, BM, F, T>(g, m0, ft0, 0, m0n, ft0, smem, pp, acc);
        }
        STAMP(it, 1, NWV);
        if constexpr (!OV) {  // residual tile -> xs
#pragma unroll 1
            for (int k = 0; k < PIECES; k++) dma_in(g.X + m0 * NCOL, k);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA pieces have landed
        __syncthreads();                                   // ... and every other wave's
        STAMP(it, 2, NWV);
        // v = (b + W.x) + x  (ggml: add(repeat(b), mul_mat) then add(cur, inpL))
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int r = 32 * t + l32;
            double s = 0.0;
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                const float4v x4 = *(const float4v *)(xs + 4 * i8_xs_chunk(r, (col >> 2) + qq));
                const float4v b4 = *(const float4v *)(g.bias + col + 4 * qq);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float v = (b4[j] + acc[0][t][4 * qq + j]) + x4[j];
                    acc[0][t][4 * qq + j] = v;
                    s += (double)v;
                }
            }
            s += __shfl_xor(s, 32);
            if (hh == 0) red[0][wv][r] = s;
        }
        __syncthreads();
        STAMP(it, 3, NWV);
        float mean[T];
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int r = 32 * t + l32;
            double tot = 0.0;
#pragma unroll
            for (int w = 0; w < NWV; w++) tot += red[0][w][r];
            mean[t] = (float)(tot / NCOL);
            double s2 = 0.0;
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const float v = acc[0][t][i] - mean[t];
                acc[0][t][i] = v;
                s2 += (double)(v * v);
            }
            s2 += __shfl_xor(s2, 32);
            if (hh == 0) red[1][wv][r] = s2;
        }
        __syncthreads();
        STAMP(it, 4, NWV);
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int r = 32 * t + l32;
            const int64_t row = m0 + r;
            double tot = 0.0;
#pragma unroll
            for (int w = 0; w < NWV; w++) tot += red[1][w][r];
            const float var = (float)(tot / NCOL);
            const float scale = 1.0f / sqrtf(var + g.eps);
            float y[16];
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                const float4v w4 = *(const float4v *)(g.ln_w + col + 4 * qq);
                const float4v b4 = *(const float4v *)(g.ln_b + col + 4 * qq);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float z = acc[0][t][4 * qq + j] * scale;
                    z = w4[j] * z;
                    y[4 * qq + j] = z + b4[j];
                }
                // in place: each (row, chunk) is this lane's alone
                *(float4v *)(xs + 4 * i8_xs_chunk(r, (col >> 2) + qq)) =
                    float4v{y[4 * qq], y[4 * qq + 1], y[4 * qq + 2], y[4 * qq + 3]};
            }
            i8_store_q8_half<WT>(g.out_act, NCOL, row, ft0, hh, y);
        }
        STAMP(it, 5, NWV);
        mprev = m0;
        if constexpr (!OV) {
            __syncthreads();
            STAMP(it, 6, NWV);
#pragma unroll 1
            for (int k = 0; k < PIECES; k++) store_out(g.X + m0 * NCOL, k);  // xs -> X
            STAMP(it, 7, NWV);
        }
        // the next tile's main loop reuses `red` and rewrites xs (pieces) only
        // after the main loop's first barrier
    }
    if constexpr (OV) {  // the last tile's LN output
        __syncthreads();
        if (mprev >= 0) {
#pragma unroll 1
            for (int k = 0; k < PIECES; k++) store_out(g.X + mprev * NCOL, k);
        }
    }
}

// ---------------------------------------------------------------------------
// Projection + residual for rows too wide for one workgroup (n_embd 768 /
// 1024): X = (b + W.x) + X; LayerNorm then runs in launch_ln.
template <int WT>
__global__ __launch_bounds__(512) void i8_resid_kernel(GemmArgs g, int n_mtiles, int n_ntiles) {
    constexpr int NT = 512, BM = 64, BN = 256, F = 1, T = 2;
    using C = I8Chunk<BM, WT == W_Q4_1>;
    __shared__ __attribute__((aligned(16))) char smem[2 * C::BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hh = lane >> 5;
    const int nwg = n_mtiles * n_ntiles;
    const int fw = wv, tw = 0;
    auto coords = [&](int tile, int64_t &m0_, int &ft0_) {
        const int lin = xcd_linear(tile, nwg);
        const int mt = lin / n_ntiles, nt = lin - mt * n_ntiles;
        m0_ = (int64_t)mt * BM;
        ft0_ = nt * (BN / 32) + fw;
    };
    if ((int)blockIdx.x >= nwg) return;
    int64_t m0n;
    int ft0n;
    coords(blockIdx.x, m0n, ft0n);
    I8Pipe<WT, NT, BM, F> pp;
    pp.prime(g, m0n, ft0n);
    for (int tile = blockIdx.x; tile < nwg; tile += gridDim.x) {
        const int64_t m0 = m0n;
        const int ft0 = ft0n;
        if (tile + (int)gridDim.x < nwg) coords(tile + gridDim.x, m0n, ft0n);
        float16v acc[F][T];
        i8_mainloop<WT, NT, BM, F, T>(g, m0, ft0, tw, m0n, ft0n, smem, pp, acc);
#pragma unroll
        for (int f = 0; f < F; f++) {
            const int col = 32 * (ft0 + f) + 16 * hh;
#pragma unroll
            for (int t = 0; t < T; t++) {
                const int64_t row = m0 + 32 * (tw + t) + l32;
                float4v *xp = (float4v *)(g.X + row * g.N + col);
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    const float4v x4 = xp[qq];
                    const float4v b4 = *(const float4v *)(g.bias + col + 4 * qq);
                    float4v o;
#pragma unroll
                    for (int j = 0; j < 4; j++) o[j] = (b4[j] + acc[f][t][4 * qq + j]) + x4[j];
                    xp[qq] = o;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
static int n_cus_i8() {
    static int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            c = 256;
        return c;
    }();
    return n;
}

static int persistent_grid(int tiles) { return std::max(1, std::min(tiles, std::max(8, n_cus_i8() / 8 * 8))); }

bool i8_gemm_supported(int epi, int N, int K) {
    if (K % I8_KC) return false;
    if (epi == EPI_GELU_ACT) return N % (32 * I8_UP_WAVES * I8_UP_F) == 0;
    if (epi == EPI_RESID) return N % 256 == 0;
    if (epi == EPI_LN) return N == 384;
    return false;
}

template <int WT>
static hipError_t i8_gemm_t(int epi, const GemmArgs &a, int Mpad, hipStream_t s) {
    if (epi == EPI_GELU_ACT) {
        if (0x8000 + a.gelu.neg_n + 1 > GELU_FLAT_LDS) return hipErrorInvalidValue;
        constexpr int NWV = I8_UP_WAVES, F = I8_UP_F, T = I8_UP_T;
        if (a.N % (32 * NWV * F) || Mpad % (32 * T)) return hipErrorInvalidValue;
        const int mt = Mpad / (32 * T), nt = a.N / (32 * NWV * F);
        hipLaunchKernelGGL((i8_up_gelu_kernel<WT, NWV, F, T>), dim3(persistent_grid(mt * nt)), dim3(NWV * 64), 0, s, a, mt, nt);
    } else if (epi == EPI_LN) {
        const int mt = Mpad / 64;
        hipLaunchKernelGGL((i8_ln384_kernel<WT>), dim3(persistent_grid(mt)), dim3(768), 0, s, a, mt);
    } else if (epi == EPI_RESID) {
        const int mt = Mpad / 64, nt = a.N / 256;
        hipLaunchKernelGGL((i8_resid_kernel<WT>), dim3(persistent_grid(mt * nt)), dim3(512), 0, s, a, mt, nt);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_gemm_i8(int wtype, int epi, const GemmArgs &a, int Mpad, hipStream_t s) {
    if (!i8_gemm_supported(epi, a.N, a.K) || Mpad % 128) return hipErrorInvalidValue;
    switch (wtype) {
        case W_Q4_0: return i8_gemm_t<W_Q4_0>(epi, a, Mpad, s);
        case W_Q4_1: return i8_gemm_t<W_Q4_1>(epi, a, Mpad, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace bertamd
