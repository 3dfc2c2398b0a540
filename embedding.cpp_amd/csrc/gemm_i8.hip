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
#include "i8_core.h"

#include <algorithm>
#include <cstdlib>

namespace bertamd {

#ifndef I8_UP_WAVES
#define I8_UP_WAVES 8
#endif
#ifndef I8_UP_F
#define I8_UP_F 2
#endif
#ifndef I8_UP_T
#define I8_UP_T 2
#endif
#ifndef I8_PRIO
#define I8_PRIO 0  // A/B: static issue priority 1 for the later-dispatched half of the waves (FFN-up / FFN-down)
#endif
#ifndef I8_UP_AHEAD
#define I8_UP_AHEAD 3  // weight blocks in flight (i8_core.h I8Pipe)
#endif
constexpr int I8_UP_MAX_N = 4096;  // FFN-up features staged in LDS (n_intermediate: 1536 / 3072 / 4096)


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
    using C = I8Chunk<BM, wt_q41(WT), WT == W_Q4_1B>;
    __shared__ __attribute__((aligned(16))) char smem[2 * C::BYTES];
    __shared__ __attribute__((aligned(16))) uint16_t gtab[GELU_FLAT_LDS];
    // the bias, read by every tile's epilogue: from LDS there (from global memory
    // each epilogue waited out an L2 round trip after the main loop)
    __shared__ __attribute__((aligned(16))) float bias_s[I8_UP_MAX_N];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hh = lane >> 5;
    if (I8_PRIO && wv >= NWV / 2) __builtin_amdgcn_s_setprio(1);
    const int nflat8 = (0x8000 + g.gelu.neg_n + 1 + 7) / 8;
    for (int i = tid; i < nflat8; i += NT) ((uint4 *)gtab)[i] = ((const uint4 *)g.gelu.full)[i];
    for (int i = tid; i < g.N / 4; i += NT) ((float4v *)bias_s)[i] = ((const float4v *)g.bias)[i];
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
    I8Pipe<WT, NT, BM, F, I8_UP_AHEAD> pp;
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
                const float4v b4 = *(const float4v *)(bias_s + col + 4 * q);
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
#ifndef I8_LN_AHEAD
#define I8_LN_AHEAD 3  // weight blocks in flight (i8_core.h I8Pipe): 3 spills 64 B/lane at this kernel's
                       // register budget and is still faster (FFN-down 299 -> 285 us, A/B)
#endif

#ifndef I8_LN_PIPE
#define I8_LN_PIPE 1  // i8_block's two-tile software pipeline in this kernel's main loop
#endif

template <int WT, bool NTX, bool OV = I8_LN_OV>
__global__ __launch_bounds__(768) void i8_ln384_kernel(GemmArgs g, int n_mtiles) {
    constexpr int NT = 768, BM = 64, F = 1, T = 2, NCOL = 384, NWV = 12;
    constexpr int XCH = BM * NCOL / 4;  // 16-byte chunks of the residual tile
    using C = I8Chunk<BM, wt_q41(WT), WT == W_Q4_1B>;
    __shared__ __attribute__((aligned(16))) char smem[2 * C::BYTES];
    __shared__ double red[2][NWV][BM];
    __shared__ __attribute__((aligned(16))) float xs[BM * NCOL];
    // b, LN weight and LN bias, read by every tile's epilogue: from LDS there
    // (from global memory each epilogue phase waited out an L2 round trip)
    __shared__ __attribute__((aligned(16))) float lnp[3][NCOL];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hh = lane >> 5;
    const int ft0 = wv;
    const int col = 32 * ft0 + 16 * hh;
    if ((int)blockIdx.x >= n_mtiles) return;
    if (tid < 3 * NCOL / 4) {
        const int v = tid / (NCOL / 4), i = tid - v * (NCOL / 4);
        ((float4v *)lnp[v])[i] = ((const float4v *)(v == 0 ? g.bias : v == 1 ? g.ln_w : g.ln_b))[i];
    }
    if (I8_PRIO && wv >= 2 * NWV / 3) __builtin_amdgcn_s_setprio(1);  // (3 waves per SIMD: the youngest)
    int64_t m0n = (int64_t)xcd_linear(blockIdx.x, n_mtiles) * BM;
    I8Pipe<WT, NT, BM, F, I8_LN_AHEAD> pp;
    pp.prime(g, m0n, ft0);
    // wave w's piece k: LDS chunks 64 (P w + k) .. + 63 of xs (P = PIECES), i.e.
    // lane l holds chunk j = 64 (P w + k) + l = (row r, column chunk cs ^ (r & 15))
    constexpr int PIECES = XCH / NT;  // 1 KiB pieces per wave
    static_assert(PIECES * NT == XCH, "whole pieces per wave");
    auto piece_off = [&](int k, int &j0) {
        j0 = 64 * (PIECES * wv + k);
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
        const float4v v = *(const float4v *)(xs + 4 * (j0 + lane));
        if constexpr (NTX) __builtin_nontemporal_store(v, (float4v *)(xt + off));
        else *(float4v *)(xt + off) = v;
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
            i8_mainloop<WT, NT, BM, F, T, I8_LN_PIPE, decltype(hook), I8_LN_AHEAD>(g, m0, ft0, 0, m0n, ft0, smem, pp, acc,
                                                                                   hook);
        } else {
            i8_mainloop<WT, NT, BM, F, T, I8_LN_PIPE, I8NoHook, I8_LN_AHEAD>(g, m0, ft0, 0, m0n, ft0, smem, pp, acc);
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
                const float4v b4 = *(const float4v *)(lnp[0] + col + 4 * qq);
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
                const float4v w4 = *(const float4v *)(lnp[1] + col + 4 * qq);
                const float4v b4 = *(const float4v *)(lnp[2] + col + 4 * qq);
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
    using C = I8Chunk<BM, wt_q41(WT), WT == W_Q4_1B>;
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
// The QKV projection (bert.cpp:905-926) on the int8 MFMA, for the batches that
// do not take the fused kernel: y = b + W.x over the head-major features,
// split hi / lo into Q | K [Mpad][2E] and V^T [E][ldv] as gemm_kernel's
// EPI_QKV.  Same main loop and fold as qkv_attention_pc_kernel's producers
// (i8_block over the blocks in order), so a sentence's Q, K and V are bitwise
// the same whichever path it takes.  Persistent 64-row x 384-feature tiles;
// lane (r, hh) of f-tile ft holds token 32 t + r, features 32 ft + 16 hh ..
template <int WT>
__global__ __launch_bounds__(768) void i8_qkv_kernel(GemmArgs g, int n_mtiles, int n_ntiles) {
    constexpr int NT = 768, BM = 64, BN = 384, F = 1, T = 2;
    using C = I8Chunk<BM, wt_q41(WT), WT == W_Q4_1B>;
    __shared__ __attribute__((aligned(16))) char smem[2 * C::BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hh = lane >> 5;
    const int nwg = n_mtiles * n_ntiles, E = g.N / 3, D = g.head_dim;
    auto coords = [&](int tile, int64_t &m0_, int &ft0_) {
        const int lin = xcd_linear(tile, nwg);
        const int mt = lin / n_ntiles, nt = lin - mt * n_ntiles;
        m0_ = (int64_t)mt * BM;
        ft0_ = nt * (BN / 32) + wv;
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
        i8_mainloop<WT, NT, BM, F, T>(g, m0, ft0, 0, m0n, ft0n, smem, pp, acc);
        const int f0 = 32 * ft0 + 16 * hh;  // head-major feature h 3D + part D + dd of acc[0][t][0]
        const int hd = f0 / (3 * D), part = (f0 - hd * 3 * D) / D, dd = f0 - hd * 3 * D - part * D;
        float bias[16];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const float4v b4 = *(const float4v *)(g.bias + f0 + 4 * q);
#pragma unroll
            for (int j = 0; j < 4; j++) bias[4 * q + j] = b4[j];
        }
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int64_t row = m0 + 32 * t + l32;
            half8 hv[2], lv[2];
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const float y = bias[i] + acc[0][t][i];
                const _Float16 yh = (_Float16)y;
                hv[i >> 3][i & 7] = yh;
                lv[i >> 3][i & 7] = (_Float16)(y - (float)yh);
            }
            if (part < 2) {
                const int64_t o = row * (2 * E) + part * E + hd * D + dd;
                *(half8 *)(g.qk_hi + o) = hv[0];
                *(half8 *)(g.qk_hi + o + 8) = hv[1];
                *(half8 *)(g.qk_lo + o) = lv[0];
                *(half8 *)(g.qk_lo + o + 8) = lv[1];
            } else {
                const int64_t c0 = hd * D + dd;
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    ((_Float16 *)g.vt_hi)[(c0 + i) * g.ldv + row] = hv[i >> 3][i & 7];
                    ((_Float16 *)g.vt_lo)[(c0 + i) * g.ldv + row] = lv[i >> 3][i & 7];
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Small batches (one server sentence: 128 padded rows).  The batch kernels
// give a workgroup whole 64-row x 384-column tiles over the full K, so a
// 128-row batch runs on 2-6 CUs and each kernel lasts one tile's walk of K
// (FFN-down: ~36 us).  Here a workgroup owns 32 rows x 32 NW columns, one
// f-tile per wave (4 N / (32 NW) workgroups at 128 rows), and each wave's
// walk of K is latency-bound, not issue-bound: so the operands are fetched a
// whole segment (SEG chunks = 4 SEG quant blocks) ahead — the A chunks of the
// next segment into registers while this one is computed (one barrier per
// segment), the weight fragments through a 4 SEG-slot register ring refilled
// 4 SEG blocks ahead.  The block step is i8_block, in block order: every sum
// is the batch kernels' bit for bit, so a sentence's embedding does not depend
// on the batch it came in.  Epilogues: EPI_QKV and EPI_GELU_ACT as the batch
// kernels (the GELU table read from L2 instead of LDS: the same entries);
// EPI_RESID X = (b + W.x) + X, for EPI_LN followed by i8_ln384_rows_kernel.
// (A 12-wave form with the LayerNorm in its epilogue — whole rows per
// workgroup, 4 workgroups for one sentence — measured 24 us against 20 us for
// the two kernels: at 4 CUs the block steps are issue-bound.)
// Epilogue of a 32 x 32 small tile in the MFMA output layout: token `row`,
// this lane's 16 outputs (f-tile ft0, lane half hh).
// Its global operands (bias; EPI_RESID: the residual x) are loaded by
// i8_small_epi_pre, which a kernel may issue before its main loop.
struct I8EpiPre {
    float4v b[4], x[4];
};
template <int EPI>
__device__ __forceinline__ void i8_small_epi_pre(const GemmArgs &g, int64_t row, int ft0, int hh, I8EpiPre &pre) {
    const int f0 = 32 * ft0 + 16 * hh;
#pragma unroll
    for (int q = 0; q < 4; q++) pre.b[q] = *(const float4v *)(g.bias + f0 + 4 * q);
    if constexpr (EPI == EPI_RESID) {
#pragma unroll
        for (int q = 0; q < 4; q++) pre.x[q] = *(const float4v *)(g.X + row * g.N + f0 + 4 * q);
    }
}
template <int WT, int EPI>
__device__ __forceinline__ void i8_small_epi(const GemmArgs &g, const float16v &acc, int64_t row, int ft0, int hh,
                                             const I8EpiPre &pre) {
    const int f0 = 32 * ft0 + 16 * hh;
    float bias[16];
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
        for (int j = 0; j < 4; j++) bias[4 * q + j] = pre.b[q][j];
    if constexpr (EPI == EPI_QKV) {  // i8_qkv_kernel's epilogue
        const int E = g.N / 3, D = g.head_dim;
        const int hd = f0 / (3 * D), part = (f0 - hd * 3 * D) / D, dd = f0 - hd * 3 * D - part * D;
        half8 hv[2], lv[2];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const float y = bias[i] + acc[i];
            const _Float16 yh = (_Float16)y;
            hv[i >> 3][i & 7] = yh;
            lv[i >> 3][i & 7] = (_Float16)(y - (float)yh);
        }
        if (part < 2) {
            const int64_t o = row * (2 * E) + part * E + hd * D + dd;
            *(half8 *)(g.qk_hi + o) = hv[0];
            *(half8 *)(g.qk_hi + o + 8) = hv[1];
            *(half8 *)(g.qk_lo + o) = lv[0];
            *(half8 *)(g.qk_lo + o + 8) = lv[1];
        } else {
            const int64_t c0 = hd * D + dd;
#pragma unroll
            for (int i = 0; i < 16; i++) {
                ((_Float16 *)g.vt_hi)[(c0 + i) * g.ldv + row] = hv[i >> 3][i & 7];
                ((_Float16 *)g.vt_lo)[(c0 + i) * g.ldv + row] = lv[i >> 3][i & 7];
            }
        }
    } else if constexpr (EPI == EPI_GELU_ACT) {  // i8_up_gelu_kernel's epilogue
        const uint16_t *gt = g.gelu.full;
        const float xlo = h2f((uint16_t)(0x8000 | g.gelu.neg_n));
        float y[16];
#pragma unroll
        for (int i = 0; i < 16; i++) y[i] = h2f(gt[f2h(fmaxf(bias[i] + acc[i], xlo))]);
        i8_store_q8_half<WT>(g.out_act, g.N, row, ft0, hh, y);
    } else {  // EPI_RESID: i8_resid_kernel's / i8_ln384_kernel's v = (b + W.x) + x
        float4v *xp = (float4v *)(g.X + row * g.N + f0);
#pragma unroll
        for (int qq = 0; qq < 4; qq++) {
            const float4v x4 = pre.x[qq];
            float4v o;
#pragma unroll
            for (int j = 0; j < 4; j++) o[j] = (bias[4 * qq + j] + acc[4 * qq + j]) + x4[j];
            xp[qq] = o;
        }
    }
}

#ifndef I8_SK_WAVES
#define I8_SK_WAVES 2
#endif
#ifndef I8_SK_SEG
#define I8_SK_SEG 4
#endif

template <int WT, int EPI, int NW, int SEG>
__global__ __launch_bounds__(NW * 64) void i8_small_kernel(GemmArgs g, int n_mtiles, int n_ntiles) {
    constexpr int NT = NW * 64, BM = 32, F = 1, T = 1, NS = 4 * SEG;  // NS: blocks per segment
    constexpr bool Q1 = wt_q41(WT);
    using C = I8Chunk<BM, Q1, WT == W_Q4_1B>;
    constexpr int IT = (4 * BM + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) char smem[2 * SEG * C::BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hh = lane >> 5;
    const int nwg = n_mtiles * n_ntiles;
    if ((int)blockIdx.x >= nwg) return;
    const int lin = xcd_linear(blockIdx.x, nwg);
    const int mt = lin / n_ntiles, nt = lin - mt * n_ntiles;
    const int64_t m0 = (int64_t)mt * BM;
    const int ft0 = nt * NW + wv;
    const int K = g.K, nkb = K >> 5, nch = K / I8_KC, nseg = (nch + SEG - 1) / SEG;

    int4v wf[NS][F];                                    // weight ring: block b in slot b % NS
    uint2 wr[2][SEG][F];                                // Q4_0 d_w (this / next segment)
    float4v wdr[2][SEG][F], wmr[2][SEG][F];             // Q4_1 d_w, m_w
    I8Items<IT> st[SEG];                                // the next segment's A chunks
    auto load_scales = [&](int set, int sg) {
#pragma unroll
        for (int cc = 0; cc < SEG; cc++) {
            const int c = sg * SEG + cc;
            if (c < nch) {
                if constexpr (Q1) {
                    wdr[set][cc][0] = i8_wvec(g.Wi.d, nkb, ft0, c);
                    wmr[set][cc][0] = i8_wvec(g.Wi.m, nkb, ft0, c);
                } else {
                    wr[set][cc][0] = ((const uint2 *)g.Wi.dh)[((int64_t)ft0 * (nkb >> 2) + c) * 32 + (lane & 31)];
                }
            }
        }
    };
    auto load_a = [&](int sg) {
#pragma unroll
        for (int cc = 0; cc < SEG; cc++)
            if (sg * SEG + cc < nch) i8_stage_load<WT, BM, NT>(st[cc], g.A, K, m0, (sg * SEG + cc) * I8_KC);
    };
    auto store_a = [&](int sg) {
#pragma unroll
        for (int cc = 0; cc < SEG; cc++)
            if (sg * SEG + cc < nch) i8_stage_store<WT, BM, NT>(st[cc], smem + ((sg & 1) * SEG + cc) * C::BYTES);
    };
#pragma unroll
    for (int j = 0; j < NS; j++)
        if (j < nkb) wf[j][0] = i8_wq(g.Wi, nkb, ft0, j);
    load_scales(0, 0);
    load_a(0);
    store_a(0);
    __syncthreads();

    float16v acc[F][T];
    acc[0][0] = float16v{};
    const float4v z4 = {0.f, 0.f, 0.f, 0.f};
    for (int sg = 0; sg < nseg; sg++) {
        const bool more = sg + 1 < nseg;
        if (more) {
            load_scales(1, sg + 1);
            load_a(sg + 1);
        }
#pragma unroll
        for (int cc = 0; cc < SEG; cc++) {
            const int c = sg * SEG + cc;
            if (c < nch) {
                const char *buf = smem + ((sg & 1) * SEG + cc) * C::BYTES;
                int4v ws[F];
                float4v wd[F], wm[F];
                if constexpr (Q1) {
                    wd[0] = hh ? z4 : wdr[0][cc][0];  // i8_mainloop's wscale_use
                    wm[0] = wmr[0][cc][0];
                } else {
                    ws[0] = int4v{(int)wr[0][cc][0].x, (int)wr[0][cc][0].y, (int)wr[0][cc][0].x, (int)wr[0][cc][0].y};
                }
                auto refill = [&](int j) {  // slot 4 cc + j: block 4 c + j done, block 4 c + j + NS next
                    const int b = 4 * c + j + NS;
                    if (b < nkb) wf[4 * cc + j][0] = i8_wq(g.Wi, nkb, ft0, b);
                };
                I8AOps<T> a0, a1;
                i8_aops<WT, BM, T, 0>(a0, buf, 0);
                i8_block<WT, BM, F, T, 0, true>(buf, 0, wf[4 * cc + 0], ws, wd, wm, a0, a1, acc);
                refill(0);
                i8_block<WT, BM, F, T, 1, true>(buf, 0, wf[4 * cc + 1], ws, wd, wm, a1, a0, acc);
                refill(1);
                i8_block<WT, BM, F, T, 2, true>(buf, 0, wf[4 * cc + 2], ws, wd, wm, a0, a1, acc);
                refill(2);
                i8_block<WT, BM, F, T, 3, true>(buf, 0, wf[4 * cc + 3], ws, wd, wm, a1, a0, acc);
                refill(3);
            }
        }
        if (more) {
            store_a(sg + 1);
#pragma unroll
            for (int cc = 0; cc < SEG; cc++) {
                wr[0][cc][0] = wr[1][cc][0];
                wdr[0][cc][0] = wdr[1][cc][0];
                wmr[0][cc][0] = wmr[1][cc][0];
            }
        }
        __syncthreads();
    }
    I8EpiPre pre;
    i8_small_epi_pre<EPI>(g, m0 + l32, ft0, hh, pre);
    i8_small_epi<WT, EPI>(g, acc[0][0], m0 + l32, ft0, hh, pre);
}

// Small batches, Q4_0: the K loop split over the waves of a workgroup.  One
// 32-token x 32-feature tile per workgroup; wave w computes blocks
// b = NW r + w (r < R rounds; every operand of its blocks loaded up front) —
// isum on the int8 MFMA and d_w * d_a on the fp16 MFMA exactly as i8_block —
// and leaves float(isum) and d_w d_a in LDS; then each thread folds its
// outputs over the round's blocks in block order, acc = fma(float(isum),
// d_w d_a, acc), the batch kernels' chain bit for bit.  The per-block products
// are independent, only the fold is sequential, so the chain (NW fmas a round
// per output) is all that is serial.  Epilogue: i8_small_epi in wave 0.
#ifndef I8_KS
#define I8_KS 1
#endif
#ifndef I8_KS_ROWS  // at most this many padded rows (one workgroup per 32 x 32 tile: at 1024 rows
#define I8_KS_ROWS 512  // i8_small_kernel's two-wave tiles win, tools/small_rows_probe.py)
#endif
#ifndef I8_KS_NW48  // waves for K <= 1536 (48 / I8_KS_NW48 rounds)
#define I8_KS_NW48 16
#endif

template <int EPI, int NW, int R>
__global__ __launch_bounds__(NW * 64) void i8_small_ks_kernel(GemmArgs g, int n_mtiles, int n_ntiles) {
    constexpr int NT = NW * 64, PER = (1024 + NT - 1) / NT;
    __shared__ float fis[NW][1024], fdd[NW][1024];  // [wave][i 64 + lane]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hh = lane >> 5;
    const int nwg = n_mtiles * n_ntiles;
    if ((int)blockIdx.x >= nwg) return;
    const int lin = xcd_linear(blockIdx.x, nwg);
    const int mt = lin / n_ntiles, ft0 = lin - mt * n_ntiles;
    const int64_t row = (int64_t)mt * 32 + l32;
    const int K = g.K, nkb = K >> 5, nr = (nkb + NW - 1) / NW;

    int4v wq[R], xa[R];
    uint32_t dw[R], da[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int b = min(NW * r + wv, nkb - 1);  // clamped: a wave past the last block loads and drops it
        wq[r] = i8_wq(g.Wi, nkb, ft0, b);
        xa[r] = *(const int4v *)((const int8_t *)g.A.q + row * K + 32 * b + 16 * hh);
        dw[r] = ((const uint16_t *)g.Wi.dh)[(((int64_t)ft0 * (nkb >> 2) + (b >> 2)) * 32 + l32) * 4 + (b & 3)];
        da[r] = ((const uint16_t *)g.A.d)[row * nkb + b];
    }
    I8EpiPre pre;  // the epilogue's global operands, issued with the block operands (wave 0's)
    if (wv == 0) i8_small_epi_pre<EPI>(g, row, ft0, hh, pre);
    const float16v zf = {};
    float acc[PER];
#pragma unroll
    for (int p = 0; p < PER; p++) acc[p] = 0.f;
#pragma unroll
    for (int r = 0; r < R; r++) {
        if (r >= nr) break;
        if (NW * r + wv < nkb) {
            const int16v is = __builtin_amdgcn_mfma_i32_32x32x32_i8(wq[r], xa[r], __builtin_bit_cast(int16v, zf), 0, 0, 0);
            const int4v ws = int4v{(int)dw[r], 0, 0, 0}, oh = int4v{hh ? 0 : (int)da[r], 0, 0, 0};
            const float16v dd = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, ws),
                                                                        __builtin_bit_cast(half8, oh), zf, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; i++) {
                fis[wv][i * 64 + lane] = (float)is[i];
                fdd[wv][i * 64 + lane] = dd[i];
            }
        }
        __syncthreads();
        const int nb = min(NW, nkb - NW * r);
#pragma unroll
        for (int p = 0; p < PER; p++) {
            const int e = tid + p * NT;
            if (1024 % NT == 0 || e < 1024) {
                if (nb == NW) {  // a whole round: every LDS read issued before the chain
                    float fi[NW], fd[NW];
#pragma unroll
                    for (int w = 0; w < NW; w++) {
                        fi[w] = fis[w][e];
                        fd[w] = fdd[w][e];
                    }
#pragma unroll
                    for (int w = 0; w < NW; w++) acc[p] = __builtin_fmaf(fi[w], fd[w], acc[p]);
                } else {
                    for (int w = 0; w < nb; w++) acc[p] = __builtin_fmaf(fis[w][e], fdd[w][e], acc[p]);
                }
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int p = 0; p < PER; p++) {
        const int e = tid + p * NT;
        if (1024 % NT == 0 || e < 1024) fis[0][e] = acc[p];
    }
    __syncthreads();
    if (wv) return;
    float16v a;
#pragma unroll
    for (int i = 0; i < 16; i++) a[i] = fis[0][i * 64 + lane];
    i8_small_epi<W_Q4_0, EPI>(g, a, row, ft0, hh, pre);
}

// LayerNorm of 384-wide rows after i8_small_kernel's residual: i8_ln384_kernel's
// epilogue with its reduction order — lane (w = l & 31 < 12, hh = l >> 5) holds
// columns 32 w + 16 hh .. + 15 (its wave w / lane half hh there); double sums
// over the 16 in order, the lane-half pair, then the twelve in order.  One wave
// per row.
template <int WT>
__global__ __launch_bounds__(256) void i8_ln384_rows_kernel(GemmArgs g, int Mpad) {
    const int lane = threadIdx.x & 63, w = lane & 31, hh = lane >> 5;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= Mpad) return;
    const bool on = w < 12;
    const int col = 32 * (on ? w : 0) + 16 * hh;
    float *xr = g.X + row * 384 + col;
    float4v lw[4], lb[4];  // issued with the row's loads, not after the reductions' barriers
#pragma unroll
    for (int qq = 0; qq < 4; qq++) {
        lw[qq] = *(const float4v *)(g.ln_w + col + 4 * qq);
        lb[qq] = *(const float4v *)(g.ln_b + col + 4 * qq);
    }
    float v[16];
#pragma unroll
    for (int qq = 0; qq < 4; qq++) {
        const float4v x4 = *(const float4v *)(xr + 4 * qq);
#pragma unroll
        for (int j = 0; j < 4; j++) v[4 * qq + j] = x4[j];
    }
    // the twelve lane sums pass through LDS (twelve independent reads; a chain
    // of twelve shuffles measured 2 us of this kernel's 4.5), summed in order
    __shared__ double part[2][4][12];
    const int wv = threadIdx.x >> 6;
    auto row_sum = [&](double s, int j) {  // s: this lane's 16-term sum; the row total in every lane
        s += __shfl_xor(s, 32);
        if (lane < 12) part[j][wv][lane] = s;
        __syncthreads();
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < 12; k++) tot += part[j][wv][k];
        return tot;
    };
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 16; i++) s += (double)v[i];
    const float mean = (float)(row_sum(s, 0) / 384);
    double s2 = 0.0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        v[i] = v[i] - mean;
        s2 += (double)(v[i] * v[i]);
    }
    const float var = (float)(row_sum(s2, 1) / 384);
    const float scale = 1.0f / sqrtf(var + g.eps);
    if (!on) return;  // both lane halves of a column block leave together (i8_store_q8_half pairs them)
    float y[16];
#pragma unroll
    for (int qq = 0; qq < 4; qq++) {
        const float4v w4 = lw[qq], b4 = lb[qq];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            float z = v[4 * qq + j] * scale;
            z = w4[j] * z;
            y[4 * qq + j] = z + b4[j];
        }
        *(float4v *)(xr + 4 * qq) = float4v{y[4 * qq], y[4 * qq + 1], y[4 * qq + 2], y[4 * qq + 3]};
    }
    i8_store_q8_half<WT>(g.out_act, 384, row, w, hh, y);
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
    if (epi == EPI_QKV) return N % 384 == 0;
    return false;
}

template <int WT>
static hipError_t i8_gemm_t(int epi, const GemmArgs &a, int Mpad, hipStream_t s) {
    if (epi == EPI_GELU_ACT) {
        if (0x8000 + a.gelu.neg_n + 1 > GELU_FLAT_LDS || a.N > I8_UP_MAX_N) return hipErrorInvalidValue;
        constexpr int NWV = I8_UP_WAVES, F = I8_UP_F, T = I8_UP_T;
        if (a.N % (32 * NWV * F) || Mpad % (32 * T)) return hipErrorInvalidValue;
        const int mt = Mpad / (32 * T), nt = a.N / (32 * NWV * F);
        hipLaunchKernelGGL((i8_up_gelu_kernel<WT, NWV, F, T>), dim3(persistent_grid(mt * nt)), dim3(NWV * 64), 0, s, a, mt, nt);
    } else if (epi == EPI_LN) {
        const int mt = Mpad / 64;
        if (a.nt_x)
            hipLaunchKernelGGL((i8_ln384_kernel<WT, true>), dim3(persistent_grid(mt)), dim3(768), 0, s, a, mt);
        else
            hipLaunchKernelGGL((i8_ln384_kernel<WT, false>), dim3(persistent_grid(mt)), dim3(768), 0, s, a, mt);
    } else if (epi == EPI_RESID) {
        const int mt = Mpad / 64, nt = a.N / 256;
        hipLaunchKernelGGL((i8_resid_kernel<WT>), dim3(persistent_grid(mt * nt)), dim3(512), 0, s, a, mt, nt);
    } else if (epi == EPI_QKV) {
        if (a.head_dim <= 0 || a.head_dim % 16 || (a.N / 3) % a.head_dim) return hipErrorInvalidValue;
        const int mt = Mpad / 64, nt = a.N / 384;
        hipLaunchKernelGGL((i8_qkv_kernel<WT>), dim3(persistent_grid(mt * nt)), dim3(768), 0, s, a, mt, nt);
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
        case W_Q4_1B: return i8_gemm_t<W_Q4_1B>(epi, a, Mpad, s);
    }
    return hipErrorInvalidValue;
}

template <int WT>
static hipError_t i8_small_t(int epi, const GemmArgs &a, int Mpad, hipStream_t s) {
    constexpr int NW = I8_SK_WAVES, SEG = I8_SK_SEG;
    if (Mpad % 32) return hipErrorInvalidValue;
    const int mt = Mpad / 32;
    if (a.N % (32 * NW) || (epi == EPI_LN && a.N != 384)) return hipErrorInvalidValue;
    const int nt = a.N / (32 * NW);
    const dim3 grid(mt * nt), block(NW * 64);
    if constexpr (WT == W_Q4_0) {
        const int nkb = a.K >> 5;
        if (I8_KS && Mpad <= I8_KS_ROWS && nkb <= 96 && (epi != EPI_QKV || (a.head_dim > 0 && a.head_dim % 16 == 0 && (a.N / 3) % a.head_dim == 0))) {
            const dim3 gk(mt * (a.N / 32));
            const int ntk = a.N / 32;
            auto go = [&](auto kern, int nw) { hipLaunchKernelGGL(kern, gk, dim3(nw * 64), 0, s, a, mt, ntk); };
            const int e2 = epi == EPI_LN ? EPI_RESID : epi;
#define I8_KS_GO(E)                                                                       \
    (nkb <= 12 ? go(i8_small_ks_kernel<E, 12, 1>, 12)                                  \
               : nkb <= 48 ? go(i8_small_ks_kernel<E, I8_KS_NW48, 48 / I8_KS_NW48>, I8_KS_NW48)             \
                           : go(i8_small_ks_kernel<E, 16, 6>, 16))
            switch (e2) {
                case EPI_QKV: I8_KS_GO(EPI_QKV); break;
                case EPI_GELU_ACT: I8_KS_GO(EPI_GELU_ACT); break;
                case EPI_RESID: I8_KS_GO(EPI_RESID); break;
                default: return hipErrorInvalidValue;
            }
#undef I8_KS_GO
            if (epi == EPI_LN && !a.defer_ln) {  // (defer_ln: the caller launches the LayerNorm pass)
                const hipError_t e = hipGetLastError();
                if (e != hipSuccess) return e;
                hipLaunchKernelGGL((i8_ln384_rows_kernel<WT>), dim3(Mpad / 4), dim3(256), 0, s, a, Mpad);
            }
            return hipGetLastError();
        }
    }
    switch (epi) {
        case EPI_QKV:
            if (a.head_dim <= 0 || a.head_dim % 16 || (a.N / 3) % a.head_dim) return hipErrorInvalidValue;
            hipLaunchKernelGGL((i8_small_kernel<WT, EPI_QKV, NW, SEG>), grid, block, 0, s, a, mt, nt);
            break;
        case EPI_GELU_ACT: hipLaunchKernelGGL((i8_small_kernel<WT, EPI_GELU_ACT, NW, SEG>), grid, block, 0, s, a, mt, nt); break;
        case EPI_RESID: hipLaunchKernelGGL((i8_small_kernel<WT, EPI_RESID, NW, SEG>), grid, block, 0, s, a, mt, nt); break;
        case EPI_LN: {
            hipLaunchKernelGGL((i8_small_kernel<WT, EPI_RESID, NW, SEG>), grid, block, 0, s, a, mt, nt);
            if (a.defer_ln) break;  // the caller launches the LayerNorm pass (launch_ln384_rows_i8)
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((i8_ln384_rows_kernel<WT>), dim3(Mpad / 4), dim3(256), 0, s, a, Mpad);
            break;
        }
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_ln384_rows_i8(int wtype, const GemmArgs &a, int Mpad, hipStream_t s) {
    if (a.N != 384 || Mpad % 4) return hipErrorInvalidValue;
    switch (wtype) {
        case W_Q4_0: hipLaunchKernelGGL((i8_ln384_rows_kernel<W_Q4_0>), dim3(Mpad / 4), dim3(256), 0, s, a, Mpad); break;
        case W_Q4_1:
        case W_Q4_1B: hipLaunchKernelGGL((i8_ln384_rows_kernel<W_Q4_1>), dim3(Mpad / 4), dim3(256), 0, s, a, Mpad); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_gemm_i8_small(int wtype, int epi, const GemmArgs &a, int Mpad, hipStream_t s) {
    if (!i8_gemm_supported(epi, a.N, a.K) || Mpad % 128) return hipErrorInvalidValue;
    switch (wtype) {
        case W_Q4_0: return i8_small_t<W_Q4_0>(epi, a, Mpad, s);
        case W_Q4_1: return i8_small_t<W_Q4_1>(epi, a, Mpad, s);
        case W_Q4_1B: return i8_small_t<W_Q4_1B>(epi, a, Mpad, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace bertamd
