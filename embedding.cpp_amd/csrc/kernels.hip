// kernels.hip — the CDNA4 (gfx950) kernel pipeline behind bert_eval_batch.
//
// Replaces the ggml CPU ops emitted by the reference's bert_build
// (reference bert.cpp:845-1012; op inventory SURVEY.md §2a).  Numerics follow
// the ggml semantics restated in SURVEY.md Appendix A wherever they are cheap
// to reproduce exactly (Q8 activation quantisation, fp16 GELU/exp tables,
// double-accumulated LayerNorm and softmax sums, fp16 activation rounding);
// the weight GEMMs here run on fp16 MFMA; Q4 weights for them are expanded
// once at load into exact fp16 hi/lo pairs of d_w * q (runtime.cpp repack), so
// the kernels apply only the activation scale d_a per block.
// The Q4 FFN GEMMs that run on the int8 MFMA instead live in gemm_i8.hip.
//
// Compiled with -ffp-contract=off: every fused multiply-add below is explicit.
#include "kernels_common.h"
#include "i8_core.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace bertamd {

constexpr int BM_MAX = GEMM_BM;  // M padding unit; GEMM tiles use BM = 128, 64 or 32
#ifndef GEMM_KB
#define GEMM_KB 2
#endif
constexpr int KB = GEMM_KB;           // 32-element quant blocks per main-loop chunk
constexpr int KC = 32 * KB;           // K per main-loop chunk
constexpr int LDA_H = KC + (KB == 2 ? 16 : 8);  // fp16 A-tile row stride (halves): 160 / 272 B, ds_read_b128 conflict-free
constexpr int LDA_F = KC + 8;         // f32 A-tile row stride (floats)


// ---------------------------------------------------------------------------
// LayerNorm row phase for GEMM slices, four lanes per (row, 32-column block):
// task t -> quarter qq = t & 3, block b, row r.  v = (bias + acc) + x; two-pass
// statistics in double (ggml_norm), combined quarter -> block (two shuffles)
// -> row (fixed block order); then y = w * (v * scale) + b, stored to X and in
// the next matmul's activation format.  The caller keeps each task's bias in
// registers across slices and loads the residual x one slice ahead, so the
// row phases do not wait on HBM latency.
struct LnTask {
    int r, b, qq, c;
    float4v bias[2];
};

template <int NBLK, int NT>
__device__ __forceinline__ void ln_tasks(LnTask (&tk)[64 * NBLK / NT], int tid, const float *__restrict__ bias) {
#pragma unroll
    for (int k = 0; k < 64 * NBLK / NT; k++) {
        const int t = tid + k * NT;
        tk[k].qq = t & 3;
        tk[k].b = (t >> 2) % NBLK;
        tk[k].r = (t >> 2) / NBLK;
        tk[k].c = 32 * tk[k].b + 8 * tk[k].qq;
#pragma unroll
        for (int h = 0; h < 2; h++) tk[k].bias[h] = *(const float4v *)(bias + tk[k].c + 4 * h);
    }
}

template <int NBLK, int NT>
__device__ __forceinline__ void ln_xload(float4v (&xv)[64 * NBLK / NT][2], const LnTask (&tk)[64 * NBLK / NT],
                                         const float *X, int64_t row0) {
#pragma unroll
    for (int k = 0; k < 64 * NBLK / NT; k++) {
        const float4v *xp = (const float4v *)(X + (row0 + tk[k].r) * (int64_t)(NBLK * 32) + tk[k].c);
        xv[k][0] = xp[0];
        xv[k][1] = xp[1];
    }
}

template <int WT, int NBLK, int NT>
__device__ __forceinline__ void ln_row_phase_q(float *stage, int ld, double *red, int64_t row0,
                                               const LnTask (&tk)[64 * NBLK / NT],
                                               const float4v (&xv)[64 * NBLK / NT][2], float *X,
                                               const float *__restrict__ lnw, const float *__restrict__ lnb,
                                               float eps, const ActPtr &out) {
    constexpr int ncols = NBLK * 32, TPT = 64 * NBLK / NT;
    double *red1 = red, *red2 = red + 16 * NBLK;
    float4v vv[TPT][2];  // the task's values between the passes (registers, not the stage)
#pragma unroll
    for (int k = 0; k < TPT; k++) {
        const float *sp = stage + tk[k].r * ld + tk[k].c;
        double s = 0.0;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            float4v v = *(const float4v *)(sp + 4 * h);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                v[j] = (tk[k].bias[h][j] + v[j]) + xv[k][h][j];
                s += (double)v[j];
            }
            vv[k][h] = v;
        }
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        if (tk[k].qq == 0) red1[tk[k].r * NBLK + tk[k].b] = s;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < TPT; k++) {
        double tot = 0.0;
#pragma unroll
        for (int q = 0; q < NBLK; q++) tot += red1[tk[k].r * NBLK + q];
        const float mean = (float)(tot / ncols);
        double s2 = 0.0;
#pragma unroll
        for (int h = 0; h < 2; h++) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float v = vv[k][h][j] - mean;
                vv[k][h][j] = v;
                s2 += (double)(v * v);
            }
        }
        s2 += __shfl_xor(s2, 1);
        s2 += __shfl_xor(s2, 2);
        if (tk[k].qq == 0) red2[tk[k].r * NBLK + tk[k].b] = s2;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < TPT; k++) {
        double tot = 0.0;
#pragma unroll
        for (int q = 0; q < NBLK; q++) tot += red2[tk[k].r * NBLK + q];
        const float var = (float)(tot / ncols);
        const float scale = 1.0f / sqrtf(var + eps);
        float y[8];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const float4v v = vv[k][h];
            const float4v w = *(const float4v *)(lnw + tk[k].c + 4 * h);
            const float4v lb = *(const float4v *)(lnb + tk[k].c + 4 * h);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float z = v[j] * scale;
                z = w[j] * z;
                y[4 * h + j] = z + lb[j];
            }
        }
        float4v *xo = (float4v *)(X + (row0 + tk[k].r) * (int64_t)ncols + tk[k].c);
        xo[0] = float4v{y[0], y[1], y[2], y[3]};
        xo[1] = float4v{y[4], y[5], y[6], y[7]};
        store_act_quarter<WT>(out, ncols, row0 + tk[k].r, tk[k].b, tk[k].qq, y);
    }
}

// ---------------------------------------------------------------------------
// Embeddings: x = pos[i] + (type[0] + word[id]) then LayerNorm (bert.cpp:880-898).
// Eight consecutive elements e0..e0+7 (e0 % 8 == 0) of row `row` of a ggml
// table (get_rows dequantisation: Q4_0 (q-8)*d, Q4_1 fmaf(q, d, m) as gcc
// contracts ggml's x*d + m).
__device__ __forceinline__ void table8(const void *tab, int type, int64_t row, int E, int e0, float *v) {
    if (type == W_F32) {
        const float4v *p = (const float4v *)((const float *)tab + row * E + e0);
        const float4v x0 = p[0], x1 = p[1];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            v[j] = x0[j];
            v[4 + j] = x1[j];
        }
    } else if (type == W_F16) {
        const half8 h = *(const half8 *)((const _Float16 *)tab + row * E + e0);
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = (float)h[j];
    } else {
        const bool q1 = type == W_Q4_1;
        const int bs = q1 ? 20 : 18, i0 = e0 & 31;
        const uint8_t *blk = (const uint8_t *)tab + (row * (E >> 5) + (e0 >> 5)) * bs;
        const float d = h2f(*(const uint16_t *)blk);
        const float m = q1 ? h2f(*(const uint16_t *)(blk + 2)) : 0.f;
        const uint16_t *qp = (const uint16_t *)(blk + (q1 ? 4 : 2) + (i0 & 15));  // byte i: elements i, i + 16
        const int sh = i0 >= 16 ? 4 : 0;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const uint32_t two = qp[w];
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const int q = (int)((two >> (8 * k + sh)) & 15u);
                v[2 * w + k] = q1 ? fmaf((float)q, d, m) : (float)(q - 8) * d;
            }
        }
    }
}

// 16 rows per workgroup, four lanes per (row, 32-element block) like the GEMM
// LayerNorm epilogue (ln_row_phase_q): values stay in registers, statistics
// in double combined quarter -> block (shuffles) -> row (fixed block order).
// Position of every packed row inside its sentence (positions 0..n-1,
// bert.cpp:874-878), one workgroup per sentence: embed_ln_kernel then reads
// it instead of searching the offsets per row (small batches: no rowpos, the
// embed kernel searches the offsets itself — one kernel launch less).
__global__ __launch_bounds__(128) void row_pos_kernel(const int32_t *__restrict__ offsets, int32_t *__restrict__ rowpos) {
    const int s = blockIdx.x, beg = offsets[s], end = offsets[s + 1];
    for (int r = beg + (int)threadIdx.x; r < end; r += 128) rowpos[r] = r - beg;
}

template <int WT, int NBLK>
__global__ __launch_bounds__(256) void embed_ln_kernel(EmbedArgs a) {
    constexpr int E = NBLK * 32, TPT = 64 * NBLK / 256;  // tasks per thread
    __shared__ double red1[16 * NBLK], red2[16 * NBLK];
    __shared__ int rinfo[32];  // [16][2]: token, position (-1 = padding row)
    const int tid = threadIdx.x;
    const int64_t row0 = (int64_t)blockIdx.x * 16;
    if (tid < 16) {
        const int64_t row = row0 + tid;
        int tok = -1, pos = 0;
        if (row < a.M) {
            tok = min(max(a.tokens[row], 0), a.n_vocab - 1);  // ids are validated on the host path;
            int p;
            if (a.rowpos) {
                p = a.rowpos[row];
            } else {  // last sentence s with offsets[s] <= row
                int lo = 0, hi = a.n_seqs - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (a.offsets[mid] <= row) lo = mid;
                    else hi = mid - 1;
                }
                p = (int)(row - a.offsets[lo]);
            }
            pos = min(p, a.n_pos - 1);  // clamp keeps device-fed ids in bounds
        }
        rinfo[2 * tid] = tok;
        rinfo[2 * tid + 1] = pos;
    }
    __syncthreads();
    float v[TPT][8];
#pragma unroll
    for (int it = 0; it < TPT; it++) {
        const int t = tid + 256 * it, qq = t & 3, b = (t >> 2) % NBLK, r = (t >> 2) / NBLK, e0 = 32 * b + 8 * qq;
        const int tok = rinfo[2 * r], pos = rinfo[2 * r + 1];
        double s = 0.0;
        if (tok >= 0) {
            float w[8], ty[8], p[8];
            table8(a.word, a.word_t, tok, E, e0, w);
            table8(a.type, a.type_t, 0, E, e0, ty);
            table8(a.pos, a.pos_t, pos, E, e0, p);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                v[it][j] = p[j] + (ty[j] + w[j]);
                s += (double)v[it][j];
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) v[it][j] = 0.f;
        }
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        if (qq == 0) red1[r * NBLK + b] = s;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < TPT; it++) {
        const int t = tid + 256 * it, qq = t & 3, b = (t >> 2) % NBLK, r = (t >> 2) / NBLK;
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < NBLK; k++) tot += red1[r * NBLK + k];
        const float mean = (float)(tot / E);
        double s2 = 0.0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            v[it][j] = v[it][j] - mean;
            s2 += (double)(v[it][j] * v[it][j]);
        }
        s2 += __shfl_xor(s2, 1);
        s2 += __shfl_xor(s2, 2);
        if (qq == 0) red2[r * NBLK + b] = s2;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < TPT; it++) {
        const int t = tid + 256 * it, qq = t & 3, b = (t >> 2) % NBLK, r = (t >> 2) / NBLK, c = 32 * b + 8 * qq;
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < NBLK; k++) tot += red2[r * NBLK + k];
        const float var = (float)(tot / E);
        const float scale = 1.0f / sqrtf(var + a.eps);
        const float4v w0 = *(const float4v *)(a.ln_w + c), w1 = *(const float4v *)(a.ln_w + c + 4);
        const float4v b0 = *(const float4v *)(a.ln_b + c), b1 = *(const float4v *)(a.ln_b + c + 4);
        float y[8];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            y[j] = w0[j] * (v[it][j] * scale) + b0[j];
            y[4 + j] = w1[j] * (v[it][4 + j] * scale) + b1[j];
        }
        float4v *xo = (float4v *)(a.X + (row0 + r) * (int64_t)E + c);
        xo[0] = float4v{y[0], y[1], y[2], y[3]};
        xo[1] = float4v{y[4], y[5], y[6], y[7]};
        store_act_quarter<WT>(a.Xa, E, row0 + r, b, qq, y);
    }
}

// LayerNorm of 16 X rows from row0 in place (+ activation store), NT threads,
// four lanes per (row, 32-element block), TPT tasks per thread; red: 16 * NBLK
// doubles, stat: 16 floats of LDS (barriers inside; the caller orders the
// slices).  Statistics as ggml_norm: mean = double sum / E, then the double
// sum of the f32 squares of (x - mean).  A row's 32-wide block partials are
// summed in block order by one thread per row (not by every lane of the row),
// which then writes the row's mean / scale.
template <int WT, int NBLK, int NT>
__device__ __forceinline__ void ln_rows16(float *X, const float *__restrict__ lnw, const float *__restrict__ lnb,
                                          float eps, const ActPtr &out, int64_t row0, double *red, float *stat) {
    constexpr int E = NBLK * 32, TPT = 64 * NBLK / NT;
    static_assert(TPT * NT == 64 * NBLK, "whole tasks per thread");
    const int tid = threadIdx.x;
    float v[TPT][8];
#pragma unroll
    for (int it = 0; it < TPT; it++) {
        const int t = tid + NT * it, qq = t & 3, b = (t >> 2) % NBLK, r = (t >> 2) / NBLK, c = 32 * b + 8 * qq;
        const float4v *xp = (const float4v *)(X + (row0 + r) * (int64_t)E + c);
        const float4v x0 = xp[0], x1 = xp[1];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            v[it][j] = x0[j];
            v[it][4 + j] = x1[j];
        }
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < 8; j++) s += (double)v[it][j];
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        if (qq == 0) red[r * NBLK + b] = s;
    }
    __syncthreads();
    if (tid < 16) {
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < NBLK; k++) tot += red[tid * NBLK + k];
        stat[tid] = (float)(tot / E);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < TPT; it++) {
        const int t = tid + NT * it, qq = t & 3, b = (t >> 2) % NBLK, r = (t >> 2) / NBLK;
        const float mean = stat[r];
        double s2 = 0.0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            v[it][j] = v[it][j] - mean;
            s2 += (double)(v[it][j] * v[it][j]);
        }
        s2 += __shfl_xor(s2, 1);
        s2 += __shfl_xor(s2, 2);
        if (qq == 0) red[r * NBLK + b] = s2;  // the row sums were read before the last barrier
    }
    __syncthreads();
    if (tid < 16) {
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < NBLK; k++) tot += red[tid * NBLK + k];
        const float var = (float)(tot / E);
        stat[tid] = 1.0f / sqrtf(var + eps);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < TPT; it++) {
        const int t = tid + NT * it, qq = t & 3, b = (t >> 2) % NBLK, r = (t >> 2) / NBLK, c = 32 * b + 8 * qq;
        const float scale = stat[r];
        const float4v w0 = *(const float4v *)(lnw + c), w1 = *(const float4v *)(lnw + c + 4);
        const float4v b0 = *(const float4v *)(lnb + c), b1 = *(const float4v *)(lnb + c + 4);
        float y[8];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            y[j] = w0[j] * (v[it][j] * scale) + b0[j];
            y[4 + j] = w1[j] * (v[it][4 + j] * scale) + b1[j];
        }
        float4v *xo = (float4v *)(X + (row0 + r) * (int64_t)E + c);
        xo[0] = float4v{y[0], y[1], y[2], y[3]};
        xo[1] = float4v{y[4], y[5], y[6], y[7]};
        store_act_quarter<WT>(out, E, row0 + r, b, qq, y);
    }
    __syncthreads();  // stat / red are reused by the next slice
}

// LayerNorm of X rows in place (+ activation store) after a separate residual
// GEMM (EPI_RESID): 16 rows per workgroup.
template <int WT, int NBLK>
__global__ __launch_bounds__(256) void ln_rows_kernel(float *X, const float *__restrict__ lnw,
                                                      const float *__restrict__ lnb, float eps, ActPtr out) {
    __shared__ double red[16 * NBLK];
    __shared__ float stat[16];
    ln_rows16<WT, NBLK, 256>(X, lnw, lnb, eps, out, (int64_t)blockIdx.x * 16, red, stat);
}

// ---------------------------------------------------------------------------
// GEMM: C[M][N] = A[M][K] . W[N][K]^T on MFMA, fused epilogues.
//
// Workgroup tile BM x BN, NW waves side by side along N (each wave owns all
// BM rows x WN columns).  K is walked in chunks of 64 (two 32-element quant
// blocks); the A chunk is converted once into an LDS tile (double-buffered,
// register-prefetched one chunk ahead) and the W fragments come straight from
// the repacked, L2-resident weight stream into registers, also one chunk ahead.
//
// Q4_0 / Q4_1 (ggml's vec_dot_q4_x_q8_x arithmetic):
// both MFMA operands are the raw integers (q8 in [-127,127], q4-8 in [-8,7] or
// q4 in [0,15]) held exactly in fp16, so v_mfma_f32_16x16x32_f16 returns the
// exact integer block sum; each 32-block is then folded in with ONE f32 fma,
// acc = fma(d_a * d_w, sum, acc)  (+ m_w * s_a for Q4_1), the very operation
// ggml performs.  F16: activations rounded to fp16 (ggml's F16 vec_dot_type),
// plain fp16 MFMA with f32 accumulation.  F32: v_mfma_f32_16x16x4_f32 (exact
// f32 products, k-ordered fma chain).
//
// Output columns are interleaved per pair of n-tiles (kernels.h WPtr), so each
// lane owns two adjacent columns of 4 rows per pair: bias / GELU / Q8 / LN
// epilogues run in registers and store 8-byte (f32) or 2-byte (int8) pieces
// that coalesce into whole rows.
// One thread's 16-element A piece in flight: 16 bytes (Q8 codes + the block's
// d), 32 (fp16) or 64 (f32), as register vectors.  (Round 1 held them in a
// 64-byte array of HIP uint4 structs: the struct copies global -> AReg -> LDS
// became memcpys that kept the array in scratch, 176 B/lane in every F16 GEMM.)
template <int WT>
struct AReg {
    u32x4v r[WT == W_F32 ? 4 : WT == W_F16 ? 2 : 1];
    float d;
};

template <int WT, int KBT = KB>
__device__ __forceinline__ void a_load(AReg<WT> &ar, const ActPtr &A, int K, int64_t m0, int k0, int item) {
    const int r = item / (2 * KBT), s = item % (2 * KBT);  // 2 KBT 16-element pieces per chunk row
    const int64_t row = m0 + r;
    const int k = k0 + s * 16;
    if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
        ar.r[0] = *(const u32x4v *)((const int8_t *)A.q + row * K + k);
        const int64_t bi = row * (K >> 5) + (k >> 5);
        if constexpr (WT == W_Q4_0) {
            ar.d = h2f(((const uint16_t *)A.d)[bi]);
        } else {
            ar.d = ((const float *)A.d)[bi];
        }
    } else if constexpr (WT == W_F16) {
        const u32x4v *p = (const u32x4v *)((const uint16_t *)A.q + row * K + k);
        ar.r[0] = p[0];
        ar.r[1] = p[1];
    } else {
        const u32x4v *p = (const u32x4v *)((const float *)A.q + row * K + k);
        ar.r[0] = p[0];
        ar.r[1] = p[1];
        ar.r[2] = p[2];
        ar.r[3] = p[3];
    }
}

// 4 signed bytes -> 4 exact fp16 integers: 0x6400 | (b ^ 0x80) is 1152 + b.
__device__ __forceinline__ void i8x4_to_f16(uint32_t x, half2v &lo, half2v &hi) {
    x ^= 0x80808080u;
    const uint32_t l = (x & 0xffu) | ((x & 0xff00u) << 8) | 0x64006400u;
    const uint32_t h = ((x >> 16) & 0xffu) | ((x >> 8) & 0xff0000u) | 0x64006400u;
    const half2v off = {(_Float16)1152.f, (_Float16)1152.f};
    lo = __builtin_bit_cast(half2v, l) - off;
    hi = __builtin_bit_cast(half2v, h) - off;
}

template <int WT, int BM, int LDA = LDA_H, int KBT = KB>
__device__ __forceinline__ void a_store(const AReg<WT> &ar, char *buf, int item, float unscale) {
    const int r = item / (2 * KBT), s = item % (2 * KBT);
    constexpr int A_BYTES = (WT == W_F32) ? BM * LDA_F * 4 : BM * LDA * 2;
    if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
        const u32x4v w = ar.r[0];
        half8 h0, h1;
        half2v a, b;
        i8x4_to_f16(w.x, a, b);
        h0[0] = a[0]; h0[1] = a[1]; h0[2] = b[0]; h0[3] = b[1];
        i8x4_to_f16(w.y, a, b);
        h0[4] = a[0]; h0[5] = a[1]; h0[6] = b[0]; h0[7] = b[1];
        i8x4_to_f16(w.z, a, b);
        h1[0] = a[0]; h1[1] = a[1]; h1[2] = b[0]; h1[3] = b[1];
        i8x4_to_f16(w.w, a, b);
        h1[4] = a[0]; h1[5] = a[1]; h1[6] = b[0]; h1[7] = b[1];
        half8 *dst = (half8 *)((_Float16 *)buf + r * LDA + s * 16);
        dst[0] = h0;
        dst[1] = h1;
        if ((s & 1) == 0) {
            float *sc = (float *)(buf + A_BYTES);  // [block of the chunk][BM]: d_a * 2^-S (exact)
            sc[(s >> 1) * BM + r] = ar.d * unscale;
        }
    } else if constexpr (WT == W_F16) {
        u32x4v *dst = (u32x4v *)((uint16_t *)buf + r * LDA + s * 16);
        dst[0] = ar.r[0];
        dst[1] = ar.r[1];
    } else {
        u32x4v *dst = (u32x4v *)((float *)buf + r * LDA_F + s * 16);
        dst[0] = ar.r[0];
        dst[1] = ar.r[1];
        dst[2] = ar.r[2];
        dst[3] = ar.r[3];
    }
}

template <int WT> struct WFrag;
template <> struct WFrag<W_Q4_0> { half8 hi, lo; };
template <> struct WFrag<W_Q4_1> { half8 hi, lo; };
template <> struct WFrag<W_F16> { half8 h; };
template <> struct WFrag<W_F32> { float4v f[2]; };

template <int WT>
__device__ __forceinline__ WFrag<WT> w_load(const WPtr &W, int64_t tile) {
    const int lane = threadIdx.x & 63;
    WFrag<WT> f;
    if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
        f.hi = ((const half8 *)W.q)[(tile * 2) * 64 + lane];
        f.lo = ((const half8 *)W.q)[(tile * 2 + 1) * 64 + lane];
    } else if constexpr (WT == W_F16) {
        f.h = ((const half8 *)W.q)[tile * 64 + lane];
    } else {
        f.f[0] = ((const float4v *)W.q)[(tile * 64 + lane) * 2];
        f.f[1] = ((const float4v *)W.q)[(tile * 64 + lane) * 2 + 1];
    }
    return f;
}

// GEMM main loop, shared by gemm_kernel and qkv_attention_kernel:
// acc[rt][nt] += A[m0 + 16 rt .. ][:] . W[16 (ntile0 + nt) .. ][:]^T for this
// wave's NTW n-tiles over the whole K (rows m0 .. m0 + BM of A; the A chunks
// go through `smem`, 2 * A_BUF bytes; returns after a final barrier).
// Lane (g, c16) holds acc[rt][nt][i] = C[row 16 rt + 4 g + i][col c16 of the
// n-tile]; with TRANS (Q4 / F16 only) the MFMA operands are swapped and it
// holds C[row 16 rt + c16][col 4 g + i] (four adjacent columns of one row).
// The loop's first loads (A chunk 0 into registers, W blocks 0 and 1) come
// from a MainloopPre the caller filled with mainloop_preload, early enough
// for their latency to hide behind other work where it can.
// W blocks in flight in the main loop's register ring: 2 (split planes, F16)
constexpr int w_ring(int wt) { return wt == W_F32 ? 1 : 2; }

template <int WT, int NW, int BM, int NTW, int KBT = KB>
struct MainloopPre {
    static constexpr int IT = (BM * (2 * KBT) + NW * 64 - 1) / (NW * 64);
    AReg<WT> ar[IT];
    WFrag<WT> wf[w_ring(WT)][NTW];
};

template <int WT, int NW, int BM, int NTW, int KBT = KB>
__device__ __forceinline__ void mainloop_preload(MainloopPre<WT, NW, BM, NTW, KBT> &pre, const GemmArgs &args,
                                                 int64_t m0, int64_t ntile0) {
    constexpr int NT = NW * 64, ITEMS = BM * (2 * KBT), IT = MainloopPre<WT, NW, BM, NTW, KBT>::IT;
    const int tid = threadIdx.x, nkb = args.K >> 5;
#pragma unroll
    for (int it = 0; it < IT; it++) {
        // every A address in the main loop is rebuilt from an opaque piece index
        // where it is used: hoisted, the per-lane 64-bit pointers stayed live
        // across the fused kernel's attention phase and were spilled (its
        // scratch 64 -> 20 bytes per lane)
        int item = tid + it * NT;
        asm volatile("" : "+v"(item));
        if (item < ITEMS) a_load<WT, KBT>(pre.ar[it], args.A, args.K, m0, 0, item);
    }
    if constexpr (WT != W_F32) {
#pragma unroll
        for (int kb = 0; kb < w_ring(WT); kb++)  // K >= 32 * w_ring(WT): launch_gemm / launch_qkv_attention
#pragma unroll
            for (int nt = 0; nt < NTW; nt++) pre.wf[kb][nt] = w_load<WT>(args.W, (ntile0 + nt) * nkb + kb);
    }
}

template <int WT, int NW, int BM, int NTW, bool TRANS = false, int KBT = KB>
__device__ __forceinline__ void gemm_mainloop(const GemmArgs &args, int64_t m0, int64_t ntile0, char *smem,
                                              float4v (&acc)[BM / 16][NTW],
                                              const MainloopPre<WT, NW, BM, NTW, KBT> &pre) {
    static_assert(!TRANS || WT != W_F32, "transposed main loop: fp16 MFMA formats only");
    static_assert(KBT == KB || WT != W_F32, "f32 main loop: the global chunk only");
    // KBT 32-wide blocks per chunk (one barrier per chunk)
    constexpr int KB = KBT, KC = 32 * KBT, LDA_H = KC + (KBT == 2 ? 16 : 8);
    constexpr int NT = NW * 64;
    constexpr int RT = BM / 16;
    constexpr bool QP = (WT == W_Q4_0 || WT == W_Q4_1);
    constexpr int AT = WT;
    constexpr bool F32P = (WT == W_F32);
    constexpr int A_BYTES = F32P ? BM * LDA_F * 4 : BM * LDA_H * 2;
    constexpr int A_BUF = A_BYTES + (QP ? KB * BM * 4 : 0);
    constexpr int ITEMS = BM * (KC / 16);            // 16-element A pieces per chunk
    constexpr int IT = (ITEMS + NT - 1) / NT;        // pieces per thread
    const int tid = threadIdx.x, lane = tid & 63;
    const int g = lane >> 4, c16 = lane & 15;
    const int K = args.K, nkc = K / KC, nkb = K >> 5;
    const float unscale = args.W.unscale;
#pragma unroll
    for (int i = 0; i < RT; i++)
#pragma unroll
        for (int j = 0; j < NTW; j++) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

    AReg<AT> ar[IT];
#pragma unroll
    for (int it = 0; it < IT; it++) {
        int item = tid + it * NT;
        asm volatile("" : "+v"(item));
        if (item < ITEMS) a_store<AT, BM, LDA_H, KBT>(pre.ar[it], smem, item, unscale);
    }
    // W fragments of the WR blocks in flight: block b lives in wf[b % WR] and
    // is replaced by block b + WR as soon as its MFMAs are issued; the chunk
    // loop runs CPR chunks per ring turn so that every slot index is static
    constexpr int WR = w_ring(WT), CPR = WR > KB ? WR / KB : 1;
    static_assert(F32P || (WR % KB == 0 || KB % WR == 0), "ring vs chunk");
    WFrag<WT> wf[WR][NTW];
    if constexpr (!F32P) {
#pragma unroll
        for (int kb = 0; kb < WR; kb++)
#pragma unroll
            for (int nt = 0; nt < NTW; nt++) wf[kb][nt] = pre.wf[kb][nt];
    }
    __syncthreads();

    const float4v zero4 = {0.f, 0.f, 0.f, 0.f};
    auto chunk = [&](const int kc, auto P) {
        constexpr int PC = decltype(P)::value;  // chunk index inside the ring turn
        const bool more = kc + 1 < nkc;
        if (more) {
#pragma unroll
            for (int it = 0; it < IT; it++) {
                int item = tid + it * NT;
                asm volatile("" : "+v"(item));
                if (item < ITEMS) a_load<AT, KBT>(ar[it], args.A, K, m0, (kc + 1) * KC, item);
            }
        }
        const char *abuf = smem + (kc & 1) * A_BUF;
#pragma unroll
        for (int kb = 0; kb < KB; kb++) {
            const int SL = (PC * KB + kb) % WR;  // this block's ring slot (static: kb is unrolled)
            if constexpr (QP) {
                // Per (row tile, n-tile): blk = A.hi + A.lo  (two MFMAs: the exact
                // d_w-scaled block dot product, f32-accumulated), then ONE fma
                // folds it in with the row's d_a:  acc = fma(d_a * 2^-S, blk, acc).
                // Software-pipelined: tile t+1's MFMA pair is in flight while
                // tile t is folded; A fragments are read from LDS two tiles ahead.
                constexpr int T = RT * NTW;
                const float *sc = (const float *)(abuf + A_BYTES) + kb * BM;
                half8 a[RT];
                float4v da[RT];  // TRANS: da[rt][0] = d_a of row 16 rt + c16
                auto lds_a = [&](int rt) {
                    a[rt] = *(const half8 *)((const _Float16 *)abuf + (rt * 16 + c16) * LDA_H + kb * 32 + 8 * g);
                    if constexpr (TRANS)
                        da[rt][0] = sc[rt * 16 + c16];
                    else
                        da[rt] = *(const float4v *)(sc + rt * 16 + g * 4);
                };
                auto mfma = [&](const half8 &x, const half8 &w, const float4v &c) {
                    return TRANS ? __builtin_amdgcn_mfma_f32_16x16x32_f16(w, x, c, 0, 0, 0)
                                 : __builtin_amdgcn_mfma_f32_16x16x32_f16(x, w, c, 0, 0, 0);
                };
                auto blk_of = [&](int rt_, int nt_) {
                    const float4v b = mfma(a[rt_], wf[SL][nt_].hi, zero4);
                    return mfma(a[rt_], wf[SL][nt_].lo, b);
                };
#pragma unroll
                for (int rt = 0; rt < RT; rt++)
                    if (rt * NTW <= 1) lds_a(rt);
                float4v blk[2];
                blk[0] = blk_of(0, 0);
#pragma unroll
                for (int t = 0; t < T; t++) {
#pragma unroll
                    for (int rt = 0; rt < RT; rt++)
                        if (rt * NTW == t + 2) lds_a(rt);
                    if (t + 1 < T) blk[(t + 1) & 1] = blk_of((t + 1) / NTW, (t + 1) % NTW);
                    const int rt = t / NTW, nt = t % NTW;
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        float v = acc[rt][nt][i];
                        v = __builtin_fmaf(TRANS ? da[rt][0] : da[rt][i], blk[t & 1][i], v);
                        asm volatile("" : "+v"(v));  // keep the fold here (no sinking past MFMAs)
                        acc[rt][nt][i] = v;
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (kc * KB + kb + WR < nkb) {
#pragma unroll
                    for (int nt = 0; nt < NTW; nt++)
                        wf[SL][nt] = w_load<WT>(args.W, (ntile0 + nt) * nkb + kc * KB + kb + WR);
                }
            } else if constexpr (WT == W_F16) {
                half8 a[RT];
#pragma unroll
                for (int rt = 0; rt < RT; rt++)
                    a[rt] = *(const half8 *)((const _Float16 *)abuf + (rt * 16 + c16) * LDA_H + kb * 32 + 8 * g);
#pragma unroll
                for (int nt = 0; nt < NTW; nt++)
#pragma unroll
                    for (int rt = 0; rt < RT; rt++)
                        acc[rt][nt] = TRANS ? __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[SL][nt].h, a[rt], acc[rt][nt], 0, 0, 0)
                                            : __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rt], wf[SL][nt].h, acc[rt][nt], 0, 0, 0);
                if (kc * KB + kb + WR < nkb) {
#pragma unroll
                    for (int nt = 0; nt < NTW; nt++) wf[SL][nt] = w_load<WT>(args.W, (ntile0 + nt) * nkb + kc * KB + kb + WR);
                }
            } else {
#pragma unroll
                for (int nt = 0; nt < NTW; nt++) wf[0][nt] = w_load<WT>(args.W, (ntile0 + nt) * nkb + kc * KB + kb);
#pragma unroll
                for (int cc = 0; cc < 2; cc++) {
                    float4v a[RT];
#pragma unroll
                    for (int rt = 0; rt < RT; rt++)
                        a[rt] = *(const float4v *)((const float *)abuf + (rt * 16 + c16) * LDA_F + kb * 32 + cc * 16 + 4 * g);
#pragma unroll
                    for (int nt = 0; nt < NTW; nt++) {
                        const float4v b = wf[0][nt].f[cc];
#pragma unroll
                        for (int j = 0; j < 4; j++)
#pragma unroll
                            for (int rt = 0; rt < RT; rt++)
                                acc[rt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rt][j], b[j], acc[rt][nt], 0, 0, 0);
                    }
                }
            }
        }
        if (more) {
#pragma unroll
            for (int it = 0; it < IT; it++) {
                int item = tid + it * NT;
                asm volatile("" : "+v"(item));
                if (item < ITEMS) a_store<AT, BM, LDA_H, KBT>(ar[it], smem + ((kc + 1) & 1) * A_BUF, item, unscale);
            }
        }
        __syncthreads();
    };
    for (int kc = 0; kc < nkc; kc += CPR) {
        chunk(kc, std::integral_constant<int, 0>{});
        if constexpr (CPR > 1) {
            static_assert(CPR == 2, "two chunks per ring turn");
            if (kc + 1 < nkc) chunk(kc + 1, std::integral_constant<int, 1>{});
        }
    }
}

// X = (b + W.x) + X for the wave's column pairs (EPI_RESID): lane
// (g, c16), pair p, row tile rt, i: row m0 + 16 rt + 4 g + i, columns
// colw + 32 p + {0, 1}
template <int RT, int NP, int NTW>
__device__ __forceinline__ void resid_epilogue(const GemmArgs &args, int64_t m0, int colw,
                                               const float4v (&acc)[RT][NTW]) {
    const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
    for (int p = 0; p < NP; p++) {
        const int col = colw + 32 * p;
        const float2v b = *(const float2v *)(args.bias + col);
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                float2v *xp = (float2v *)(args.X + (m0 + rt * 16 + 4 * g + i) * args.N + col);
                const float2v x = *xp;
                *xp = float2v{(b[0] + acc[rt][2 * p][i]) + x[0], (b[1] + acc[rt][2 * p + 1][i]) + x[1]};
            }
    }
}

template <int WT, int EPI, int BN, int NW, int BM>
__global__ __launch_bounds__(NW * 64) void gemm_kernel(GemmArgs args, int n_mtiles, int n_ntiles) {
    constexpr int NT = NW * 64;
    constexpr int WN = BN / NW;
    constexpr int NTW = WN / 16;
    constexpr int NP = NTW / 2;  // column pairs per wave
    constexpr int RT = BM / 16;
    constexpr bool QP = (WT == W_Q4_0 || WT == W_Q4_1);
    constexpr int AT = WT;
    constexpr bool F32P = (WT == W_F32);
    constexpr int A_BYTES = F32P ? BM * LDA_F * 4 : BM * LDA_H * 2;
    constexpr int A_BUF = A_BYTES + (QP ? KB * BM * 4 : 0);
    constexpr int ITEMS = BM * (KC / 16);            // 16-element A pieces per chunk
    constexpr int IT = (ITEMS + NT - 1) / NT;        // pieces per thread
    // Q4 / F16 GELU: transposed accumulators (Q4: in block-8 column order,
    // gemm_gelu_blk8), epilogue in registers; otherwise 16-row LDS slices
    constexpr bool GELU_T = (QP || WT == W_F16) && EPI == EPI_GELU_ACT;
    // LN: two 16-row slice buffers (stage + row partials) for BN <= 768
    constexpr int EPI_LDS = (EPI == EPI_QKV || EPI == EPI_NONE || EPI == EPI_RESID || GELU_T) ? 0 : (EPI == EPI_LN && BN <= 768 ? 2 : 1) * (16 * (BN + 4) * 4 + ((EPI == EPI_LN) ? 2 * 16 * (BN / 32) * 8 : 0));
    constexpr int SMEM = (2 * A_BUF > EPI_LDS) ? 2 * A_BUF : EPI_LDS;
    static_assert(NTW % 2 == 0, "wave tile must hold whole column pairs");
    static_assert(EPI == EPI_QKV || EPI == EPI_NONE || EPI == EPI_RESID || (BN / 32) % NW == 0,
                  "epilogue: whole quarter-tasks per thread");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];
    constexpr bool GT_LDS = EPI == EPI_GELU_ACT;
    __shared__ __attribute__((aligned(16))) uint16_t gtab[GT_LDS ? (GELU_T ? GELU_FLAT_LDS : HALF_TABLE_LDS) : 8];

    // XCD-aware tile order: linear block ids are dealt round-robin over the 8
    // XCDs; remap so that each XCD walks a contiguous range, n fastest, so the
    // N-tiles that share an A panel run on one XCD (bijective for any count).
    // A persistent launch (GELU_T: gridDim.x a multiple of 8, each workgroup
    // walking ids blockIdx.x + k * gridDim.x) keeps every id on its XCD.
    const int nwg = n_mtiles * n_ntiles;
    auto tile_of = [&](int orig, int64_t &m0_, int &n0_) {
        const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
        const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
        const int mt = lin / n_ntiles;
        m0_ = (int64_t)mt * BM;
        n0_ = (lin - mt * n_ntiles) * BN;
    };

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int g = lane >> 4, c16 = lane & 15;
    if constexpr (GELU_T) {
        // ggml's GELU table, entries [0, 0x8000 + neg_n] (every positive pattern,
        // negatives up to the first of the constant run) -> LDS once per
        // workgroup; inputs below -|h(neg_n)| are clamped onto that entry.
        const int nflat8 = (0x8000 + args.gelu.neg_n + 1 + 7) / 8;
        for (int i = tid; i < nflat8; i += NT) ((uint4 *)gtab)[i] = ((const uint4 *)args.gelu.full)[i];
        const float xlo = h2f((uint16_t)(0x8000 | args.gelu.neg_n));
        int64_t m0;
        int n0;
        tile_of(blockIdx.x, m0, n0);
        MainloopPre<WT, NW, BM, NTW> pre;
        mainloop_preload(pre, args, m0, (n0 + wv * WN) >> 4);
        for (int t = blockIdx.x; t < nwg; t += gridDim.x) {
            float4v acc[RT][NTW];
            gemm_mainloop<WT, NW, BM, NTW, true>(args, m0, (n0 + wv * WN) >> 4, smem, acc, pre);
            const int64_t mc = m0;
            const int nc = n0;
#pragma unroll
            for (int p = 0; p < NP; p++) {
                const int col = nc + wv * WN + 32 * p + 8 * g;
                const float4v b0 = *(const float4v *)(args.bias + col), b1 = *(const float4v *)(args.bias + col + 4);
                if constexpr (QP) {
                    // Transposed accumulators over W repacked in block-8 order
                    // (gemm_gelu_blk8): lane (g, c16) holds acc[rt][2p + t][i] =
                    // C[mc + 16 rt + c16][32 pb + 8 g + 4 t + i] (pb = the pair's
                    // 32-column block), i.e. one quarter of one row's Q8 block.
#pragma unroll
                    for (int rt = 0; rt < RT; rt++) {
                        float y[8];
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            y[i] = h2f(gtab[f2h(fmaxf(b0[i] + acc[rt][2 * p][i], xlo))]);
                            y[4 + i] = h2f(gtab[f2h(fmaxf(b1[i] + acc[rt][2 * p + 1][i], xlo))]);
                        }
                        store_act_quarter_t<AT>(args.out_act, args.N, mc + rt * 16 + c16, col >> 5, g, y);
                    }
                } else {
                    // F16 (plain pair-interleaved tile order, kernels.h WPtr): lane
                    // (g, c16) holds acc[rt][2p + t][i] = C[mc + 16 rt + c16][32 pb +
                    // 8 g + 2 i + t]: eight adjacent fp16 outputs, one 16-byte store.
                    // ggml's gelu output is the table's fp16 value, stored as is.
                    const float bb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
                    for (int rt = 0; rt < RT; rt++) {
                        uint4 pk;
                        uint32_t *pw = (uint32_t *)&pk;
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const uint32_t h0 = gtab[f2h(fmaxf(bb[2 * i] + acc[rt][2 * p][i], xlo))];
                            const uint32_t h1 = gtab[f2h(fmaxf(bb[2 * i + 1] + acc[rt][2 * p + 1][i], xlo))];
                            pw[i] = h0 | (h1 << 16);
                        }
                        *(uint4 *)((uint16_t *)args.out_act.q + (mc + rt * 16 + c16) * args.N + col) = pk;
                    }
                }
            }
            if (t + (int)gridDim.x < nwg) {
                tile_of(t + gridDim.x, m0, n0);
                mainloop_preload(pre, args, m0, (n0 + wv * WN) >> 4);
            }
        }
        return;
    }

    int64_t m0;
    int n0;
    tile_of(blockIdx.x, m0, n0);
    const int64_t ntile0 = (n0 + wv * WN) >> 4;
    if constexpr (GT_LDS) {  // GELU table -> LDS (read after the main loop's barriers)
        for (int i = tid; i < args.gelu.n_pad / 8; i += NT) ((uint4 *)gtab)[i] = ((const uint4 *)args.gelu.compact)[i];
    }

    // LN (384 wide): the residual rows of the first 16-row slice are loaded
    // before the main loop (their latency hides behind it; the later slices'
    // loads overlap the previous slice's row phase).  Wider rows would spill.
    constexpr int LN_TPT = EPI == EPI_LN ? 64 * (BN / 32) / NT : 1;
    constexpr bool XPRE = EPI == EPI_LN && BN == 384;
    [[maybe_unused]] float4v xv[2][LN_TPT][2];
    if constexpr (XPRE) {
        LnTask t0[LN_TPT];  // (row, column) of ln_tasks; its bias loads come after the main loop
#pragma unroll
        for (int k = 0; k < LN_TPT; k++) {
            const int t = tid + k * NT;
            t0[k].r = (t >> 2) / (BN / 32);
            t0[k].c = 32 * ((t >> 2) % (BN / 32)) + 8 * (t & 3);
        }
        ln_xload<BN / 32, NT>(xv[0], t0, args.X, m0);
    }
    float4v acc[RT][NTW];
    {
        MainloopPre<WT, NW, BM, NTW> pre;
        mainloop_preload(pre, args, m0, ntile0);
        gemm_mainloop<WT, NW, BM, NTW, false>(args, m0, ntile0, smem, acc, pre);
    }

    // ---- epilogue, in registers.  Lane (g, c16), pair p, row-tile rt, i:
    //      row = m0 + rt*16 + 4g + i, columns col0 + {0, 1} with
    //      col0 = n0 + wv*WN + 32p + 2*c16; values acc[rt][2p][i], acc[rt][2p+1][i].
    const int colw = n0 + wv * WN + 2 * c16;
    if constexpr (EPI == EPI_NONE) {  // keep the accumulators observable, store nothing
        float t = 0.f;
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int j = 0; j < NTW; j++) t += acc[rt][j][0] + acc[rt][j][3];
        if (t == 1234.5678f) args.X[tid] = t;
    } else if constexpr (EPI == EPI_RESID) {  // X = (b + W.x) + X, in registers
        resid_epilogue<RT, NP>(args, m0, colw, acc);
    } else if constexpr (EPI == EPI_QKV) {
        // y = b + W.x in f32 (ggml), split hi = fp16(y), lo = fp16(y - hi) for the
        // attention MFMAs.  A column pair lies wholly in Q|K or in V (E % 32 == 0).
        const int E = args.N / 3, D = args.head_dim;
#pragma unroll
        for (int p = 0; p < NP; p++) {
            const int fcol = colw + 32 * p;  // head-major feature: h*3D + part*D + d (D % 32 == 0)
            const float2v b = *(const float2v *)(args.bias + fcol);
            const int hd = fcol / (3 * D), part = (fcol - hd * 3 * D) / D, dd = fcol - hd * 3 * D - part * D;
            const int col = part * E + hd * D + dd;  // Q | K | V column of the classic layout
            if (part < 2) {
#pragma unroll
                for (int rt = 0; rt < RT; rt++)
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int64_t row = m0 + rt * 16 + 4 * g + i;
                        const float y0 = b[0] + acc[rt][2 * p][i], y1 = b[1] + acc[rt][2 * p + 1][i];
                        const _Float16 h0 = (_Float16)y0, h1 = (_Float16)y1;
                        *(half2v *)((_Float16 *)args.qk_hi + row * (2 * E) + col) = half2v{h0, h1};
                        *(half2v *)((_Float16 *)args.qk_lo + row * (2 * E) + col) =
                            half2v{(_Float16)(y0 - (float)h0), (_Float16)(y1 - (float)h1)};
                    }
            } else {
#pragma unroll
                for (int rt = 0; rt < RT; rt++) {
                    const int64_t row0 = m0 + rt * 16 + 4 * g;
#pragma unroll
                    for (int t = 0; t < 2; t++) {
                        half4v hv, lv;
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const float y = b[t] + acc[rt][2 * p + t][i];
                            hv[i] = (_Float16)y;
                            lv[i] = (_Float16)(y - (float)hv[i]);
                        }
                        const int64_t c = col + t - 2 * E;
                        *(half4v *)((_Float16 *)args.vt_hi + c * args.ldv + row0) = hv;
                        *(half4v *)((_Float16 *)args.vt_lo + c * args.ldv + row0) = lv;
                    }
                }
            }
        }
    } else {
        // GELU / LayerNorm epilogues through a 16-row LDS slice: one thread per
        // (32-column block quarter, row) task, TPT tasks per thread whose column
        // operands stay in registers across the slices.  Row stride BN + 4 floats
        // is odd in 16-byte slots, so the 16 lanes reading one block of 16 rows
        // hit 16 slots.
        constexpr int LD = BN + 4, NBLK = BN / 32, TPT = 64 * NBLK / NT;
        constexpr int SLICE_BYTES = 16 * LD * 4 + ((EPI == EPI_LN) ? 2 * 16 * NBLK * 8 : 0);
        constexpr int NSB = (EPI == EPI_LN && 2 * SLICE_BYTES <= SMEM) ? 2 : 1;  // LN: stage + red double-buffered
        constexpr bool LN = EPI == EPI_LN;
        [[maybe_unused]] LnTask tk[LN ? TPT : 1];
        [[maybe_unused]] float4v gb[LN ? 1 : TPT][2];
        if constexpr (LN) {
            ln_tasks<NBLK, NT>(tk, tid, args.bias);
            if constexpr (!XPRE) ln_xload<NBLK, NT>(xv[0], tk, args.X, m0);
        } else {
#pragma unroll
            for (int k = 0; k < TPT; k++) {
                const int t = tid + k * NT, c = 32 * ((t >> 2) % NBLK) + 8 * (t & 3);
                gb[k][0] = *(const float4v *)(args.bias + n0 + c);
                gb[k][1] = *(const float4v *)(args.bias + n0 + c + 4);
            }
        }
#pragma unroll
        for (int rt = 0; rt < RT; rt++) {
            // with two slice buffers the previous slice's readers never share a buffer with this
            // slice's writers, except across one full slice (whose own barriers separate them)
            float *stage = (float *)(smem + (rt % NSB) * SLICE_BYTES);
            double *red = (double *)(smem + (rt % NSB) * SLICE_BYTES + 16 * LD * 4);  // [2][16][NBLK]
            if (NSB == 1 || rt == 0) __syncthreads();
#pragma unroll
            for (int p = 0; p < NP; p++)
#pragma unroll
                for (int i = 0; i < 4; i++)
                    *(float2v *)(stage + (4 * g + i) * LD + wv * WN + 32 * p + 2 * c16) =
                        float2v{acc[rt][2 * p][i], acc[rt][2 * p + 1][i]};
            __syncthreads();
            const int64_t row0 = m0 + rt * 16;
            if constexpr (EPI == EPI_GELU_ACT) {
                // gelu(b + W.x) through ggml's fp16 table, four lanes per block
                const uint32_t *tab = (const uint32_t *)(GT_LDS ? gtab : args.gelu.compact);
                const uint32_t cap = (uint32_t)args.gelu.cap;
#pragma unroll
                for (int k = 0; k < TPT; k++) {
                    const int t = tid + k * NT;
                    const int qq = t & 3, b = (t >> 2) % NBLK, r = (t >> 2) / NBLK, c = 32 * b + 8 * qq;
                    const float *sp = stage + r * LD + c;
                    float y[8];
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const float4v v = *(const float4v *)(sp + 4 * h);
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            y[4 * h + j] = h2f((uint16_t)gelu_lookup(tab, cap, f2h(gb[k][h][j] + v[j])));
                    }
                    store_act_quarter<AT>(args.out_act, args.N, row0 + r, (n0 >> 5) + b, qq, y);
                }
            } else {
                if (rt + 1 < RT) ln_xload<NBLK, NT>(xv[(rt + 1) & 1], tk, args.X, row0 + 16);
                ln_row_phase_q<AT, NBLK, NT>(stage, LD, red, row0, tk, xv[rt & 1], args.X, args.ln_w, args.ln_b, args.eps,
                                             args.out_act);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Attention for sentences of n <= 128 tokens (reference bert.cpp:928-942):
// one workgroup per (sentence, group of heads), wave w owns queries
// 32w..32w+31; heads of the group are processed in turn, so ggml's exp table
// is copied into LDS once per workgroup.
//
// f32 accuracy on fp16 MFMA: the QKV GEMM stored every value x split exactly
// into hi = fp16(x), lo = fp16(x - hi); K.Q^T is hi*hi + hi*lo + lo*hi (three
// v_mfma_f32_32x32x16_f16; the dropped lo*lo term is 2^-22 relative), so S
// carries f32-level error like ggml's f32 mul_mat.  Swapped QK^T: S^T = K . Q^T
// puts one query per lane column, so ggml's soft_max (max, p =
// exp_tab[fp16(s - max)], double sum, scale by (float)(1/sum)) runs in
// registers with one cross-half shuffle.  The probabilities are fp16 table
// values, exact as MFMA operands: ctx^T = (V^T_hi + V^T_lo) . P^T in two MFMAs
// with exact products and f32 accumulation, then the 1/sum scale is applied to
// the 32 outputs of each query (ggml scales P first: the two orders differ by
// f32 rounding only).  The context is quantised to the O-projection's
// activation format in registers.

// Shared pieces of the two attention kernels (32 queries per wave, lane
// (r, hh) = query r, key / dimension half hh of the 32x32 MFMA layout).
// S^T tile (32 keys from LDS row k0 x this wave's 32 queries), split-fp16.
template <int D>
__device__ __forceinline__ float16v attn_qk(const _Float16 *Kh, const _Float16 *Kl, int kst, int k0, int r, int hh,
                                            const half8 *qh, const half8 *ql) {
    float16v S = {};
#pragma unroll
    for (int ks = 0; ks < D / 16; ks++) {
        const int off = (k0 + r) * kst + 16 * ks + 8 * hh;
        const half8 kh = *(const half8 *)&Kh[off], kl = *(const half8 *)&Kl[off];
        S = __builtin_amdgcn_mfma_f32_32x32x16_f16(kl, qh[ks], S, 0, 0, 0);
        S = __builtin_amdgcn_mfma_f32_32x32x16_f16(kh, ql[ks], S, 0, 0, 0);
        S = __builtin_amdgcn_mfma_f32_32x32x16_f16(kh, qh[ks], S, 0, 0, 0);
    }
    return S;
}

// o += V^T . P^T for 32 keys from LDS column k0 (P = the tile's fp16 table
// values, exact): k-step ks, B element j of lane half hh is key
// k0 + 16 ks + 8 (j >> 2) + 4 hh + (j & 3) = register 8 ks + j of the S tile.
template <int D>
__device__ __forceinline__ void attn_pv(float16v *o, const _Float16 *Vh, const _Float16 *Vl, int vst, int k0, int r,
                                        int hh, const float16v &P) {
#pragma unroll
    for (int ks = 0; ks < 2; ks++) {
        half8 ph;
#pragma unroll
        for (int j = 0; j < 8; j++) ph[j] = (_Float16)P[8 * ks + j];
        const int key = k0 + 16 * ks + 4 * hh;
#pragma unroll
        for (int dt = 0; dt < D / 32; dt++) {
            const int off = (dt * 32 + r) * vst + key;
            const half4v h0 = *(const half4v *)&Vh[off], h1 = *(const half4v *)&Vh[off + 8];
            const half4v l0 = *(const half4v *)&Vl[off], l1 = *(const half4v *)&Vl[off + 8];
            const half8 vh = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
            const half8 vl = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vl, ph, o[dt], 0, 0, 0);
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, ph, o[dt], 0, 0, 0);
        }
    }
}

// The same with P given as the table's fp16 values (two 8-key halves), for
// NDT 32-dim blocks starting at block dt0.
template <int D, int NDT = D / 32>
__device__ __forceinline__ void attn_pv_h(float16v *o, const _Float16 *Vh, const _Float16 *Vl, int vst, int k0, int r,
                                          int hh, const half8 (&ph)[2], int dt0 = 0) {
#pragma unroll
    for (int ks = 0; ks < 2; ks++) {
        const int key = k0 + 16 * ks + 4 * hh;
#pragma unroll
        for (int dt = 0; dt < NDT; dt++) {
            const int off = ((dt0 + dt) * 32 + r) * vst + key;
            const half4v h0 = *(const half4v *)&Vh[off], h1 = *(const half4v *)&Vh[off + 8];
            const half4v l0 = *(const half4v *)&Vl[off], l1 = *(const half4v *)&Vl[off + 8];
            const half8 vh = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
            const half8 vl = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vl, ph[ks], o[dt], 0, 0, 0);
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, ph[ks], o[dt], 0, 0, 0);
        }
    }
}

// ctx = o * (float)(1/sum), stored in the O-projection's activation format:
// lane (r, hh) holds ctx[row][h D + 32 dt + (j & 3) + 8 (j >> 2) + 4 hh], one
// 32-value quant block per (query, dt) split over the lane pair (r, hh); NDT
// blocks from block dt0.
template <int WT, int D, int NDT = D / 32>
__device__ __forceinline__ void attn_store_ctx(const AttnArgs &a, float16v *o, float rs, int64_t row, bool valid,
                                               int h, int hh, int dt0 = 0) {
    const int E = a.E;
    asm volatile("" : "+v"(row));  // context addresses built here, not hoisted (spills)
#pragma unroll
    for (int dt = 0; dt < NDT; dt++) {
#pragma unroll
        for (int j = 0; j < 16; j++) o[dt][j] *= rs;
        const int col0 = h * D + (dt0 + dt) * 32;
        if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
            float amax = 0.f;
#pragma unroll
            for (int j = 0; j < 16; j++) amax = fmaxf(amax, fabsf(o[dt][j]));
            amax = fmaxf(amax, __shfl_xor(amax, 32));
            float d, id;
            q8_scales(amax, d, id);
            uint32_t pk[4];
#pragma unroll
            for (int m = 0; m < 4; m++)
                pk[m] = q8_pack4(o[dt][4 * m], o[dt][4 * m + 1], o[dt][4 * m + 2], o[dt][4 * m + 3], id);
            if (valid) {
#pragma unroll
                for (int m = 0; m < 4; m++) *(uint32_t *)((int8_t *)a.ctx.q + row * E + col0 + 8 * m + 4 * hh) = pk[m];
                if (hh == 0) {
                    const int64_t bi = row * (E >> 5) + (col0 >> 5);
                    if constexpr (WT == W_Q4_0)
                        ((uint16_t *)a.ctx.d)[bi] = f2h(d);
                    else
                        ((float *)a.ctx.d)[bi] = d;
                }
            }
        } else if (valid) {
#pragma unroll
            for (int m = 0; m < 4; m++) {
                const int col = col0 + 8 * m + 4 * hh;
                if constexpr (WT == W_F16) {
                    *(half4v *)((_Float16 *)a.ctx.q + row * E + col) =
                        half4v{(_Float16)o[dt][4 * m], (_Float16)o[dt][4 * m + 1], (_Float16)o[dt][4 * m + 2],
                               (_Float16)o[dt][4 * m + 3]};
                } else {
                    *(float4v *)((float *)a.ctx.q + row * E + col) =
                        float4v{o[dt][4 * m], o[dt][4 * m + 1], o[dt][4 * m + 2], o[dt][4 * m + 3]};
                }
            }
        }
    }
}

template <int WT, int D>
__global__ __launch_bounds__(256) void attention_short_kernel(AttnArgs a, int heads_per_wg) {
    constexpr int NK = 128;      // keys staged (n <= 128)
    constexpr int KST = D + 8;   // K row stride, halves: conflict-free ds_read_b128 (80 / 144 B)
    constexpr int VST = NK + 4;  // V^T row stride, halves: 66 dwords, conflict-free ds_read_b64
    __shared__ __attribute__((aligned(16))) _Float16 Kh[NK * KST], Kl[NK * KST], Vh[D * VST], Vl[D * VST];
    __shared__ __attribute__((aligned(16))) uint16_t etab[EXP_TABLE_LDS];
    const int s = blockIdx.y;
    const int beg = a.offsets[s], n = a.offsets[s + 1] - beg;
    if (n > NK) return;  // attention_long_kernel handles these sentences
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
    const int E = a.E, E2 = 2 * E;
    const bool v_aligned = (beg & 7) == 0;
    const int epos = a.expt.pos_n, eneg = a.expt.neg_n;
    for (int i = tid; i < a.expt.n_pad / 8; i += 256) ((uint4 *)etab)[i] = ((const uint4 *)a.expt.compact)[i];

    const int h_beg = blockIdx.x * heads_per_wg, h_end = min(h_beg + heads_per_wg, a.H);
    // K and V^T tiles of the next head are prefetched into registers while the
    // current head computes (KIT / VIT 16-byte pieces per thread and plane)
    constexpr int KIT = NK * (D / 8) / 256, VIT = D * (NK / 8) / 256;
    uint4 pkh[KIT], pkl[KIT];
    half8 pvh[VIT], pvl[VIT];
    auto fetch = [&](int h) {
#pragma unroll
        for (int i = 0; i < KIT; i++) {
            const int idx = tid + 256 * i, key = idx / (D / 8), c = (idx - key * (D / 8)) * 8;
            pkh[i] = pkl[i] = uint4{0u, 0u, 0u, 0u};
            if (key < n) {
                const int64_t off = (int64_t)(beg + key) * E2 + E + h * D + c;
                pkh[i] = *(const uint4 *)(a.qk_hi + off);
                pkl[i] = *(const uint4 *)(a.qk_lo + off);
            }
        }
#pragma unroll
        for (int i = 0; i < VIT; i++) {
            const int idx = tid + 256 * i, d = idx / (NK / 8), k8 = (idx - d * (NK / 8)) * 8;
            const int64_t off = (int64_t)(h * D + d) * a.ldv + beg + k8;
            pvh[i] = pvl[i] = half8{};
            if (k8 + 8 <= n && v_aligned) {
                pvh[i] = *(const half8 *)(a.vt_hi + off);
                pvl[i] = *(const half8 *)(a.vt_lo + off);
            } else {
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (k8 + j < n) {
                        pvh[i][j] = ((const _Float16 *)a.vt_hi)[off + j];
                        pvl[i][j] = ((const _Float16 *)a.vt_lo)[off + j];
                    }
            }
        }
    };
    auto commit = [&]() {
#pragma unroll
        for (int i = 0; i < KIT; i++) {
            const int idx = tid + 256 * i, key = idx / (D / 8), c = (idx - key * (D / 8)) * 8;
            *(uint4 *)&Kh[key * KST + c] = pkh[i];
            *(uint4 *)&Kl[key * KST + c] = pkl[i];
        }
#pragma unroll
        for (int i = 0; i < VIT; i++) {
            const int idx = tid + 256 * i, d = idx / (NK / 8), k8 = (idx - d * (NK / 8)) * 8;
            const half8 vh = pvh[i], vl = pvl[i];
            *(half4v *)&Vh[d * VST + k8] = half4v{vh[0], vh[1], vh[2], vh[3]};
            *(half4v *)&Vh[d * VST + k8 + 4] = half4v{vh[4], vh[5], vh[6], vh[7]};
            *(half4v *)&Vl[d * VST + k8] = half4v{vl[0], vl[1], vl[2], vl[3]};
            *(half4v *)&Vl[d * VST + k8 + 4] = half4v{vl[4], vl[5], vl[6], vl[7]};
        }
    };
    if (h_beg < h_end) fetch(h_beg);
    for (int h = h_beg; h < h_end; h++) {
        __syncthreads();  // previous head's LDS reads are done
        commit();
        __syncthreads();
        if (h + 1 < h_end) fetch(h + 1);
        const int q0 = wv * 32;
        if (q0 >= n) continue;

        // Q^T fragments (B operand): lane (r, hh) holds Q[q0 + r][16 ks + 8 hh + j]
        half8 qh[D / 16], ql[D / 16];
        {
            const int qr = min(q0 + r, n - 1);
            const int64_t off = (int64_t)(beg + qr) * E2 + h * D + 8 * hh;
#pragma unroll
            for (int ks = 0; ks < D / 16; ks++) {
                qh[ks] = *(const half8 *)(a.qk_hi + off + 16 * ks);
                ql[ks] = *(const half8 *)(a.qk_lo + off + 16 * ks);
            }
        }
        const int nkt = (n + 31) >> 5;
        float16v S[4];
        const float16v zero16 = {};
#pragma unroll
        for (int kt = 0; kt < 4; kt++) S[kt] = kt < nkt ? attn_qk<D>(Kh, Kl, KST, 32 * kt, r, hh, qh, ql) : zero16;
        // soft_max over keys for query q0 + r: this lane holds keys
        // 32 kt + (j & 3) + 8 (j >> 2) + 4 hh, the partner lane (r, 1 - hh) the rest
        // keys >= n are masked to -inf in the one partial tile; `lim` is made
        // opaque per head so the per-element lane masks are not hoisted out of
        // the head loop into (spilled) scalar registers
        int lim = n - 4 * hh;
        asm volatile("" : "+v"(lim));
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; kt++) {
            if (kt < nkt) {
#pragma unroll
                for (int j = 0; j < 16; j++) S[kt][j] = S[kt][j] * a.scale;  // ggml_scale after K.Q
                if (32 * kt + 32 > n) {
#pragma unroll
                    for (int j = 0; j < 16; j++)
                        if (32 * kt + (j & 3) + 8 * (j >> 2) >= lim) S[kt][j] = -INFINITY;
                }
#pragma unroll
                for (int j = 0; j < 16; j++) mx = fmaxf(mx, S[kt][j]);
            }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        // ggml's double sum of the fp16 probabilities, exactly: p * 2^24 is an
        // integer for every fp16 p in [0, 1], and n <= 128 of them fit a uint32
        uint32_t sum = 0;
#pragma unroll
        for (int kt = 0; kt < 4; kt++) {
            if (kt < nkt) {
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    // s - max <= 0: exp_tab[fp16(s - max)] from LDS, indexed by the
                    // magnitude fp16(max - s); -inf (masked) -> +inf -> the 0 entry
                    const uint32_t hm = f2h(mx - S[kt][j]);
                    const float p = h2f(etab[epos + min(hm, (uint32_t)eneg)]);
                    S[kt][j] = p;
                    sum += (uint32_t)(p * 16777216.0f);
                }
            }
        }
        sum += __shfl_xor(sum, 32);
        const float rs = (float)(1.0 / ((double)sum * 0x1p-24));
        float16v o[D / 32];
#pragma unroll
        for (int dt = 0; dt < D / 32; dt++) o[dt] = zero16;
#pragma unroll
        for (int kt = 0; kt < 4; kt++)
            if (kt < nkt) attn_pv<D>(o, Vh, Vl, VST, 32 * kt, r, hh, S[kt]);
        attn_store_ctx<WT, D>(a, o, rs, beg + q0 + r, q0 + r < n, h, hh);
    }
}

// Small batches (the server's one sentence), Q4_0, head dim 32, n_embd 384:
// the int8 QKV projection of one head fused with its attention — one 12-wave
// workgroup per (head, sentence).  Wave t < 3 nt (nt = the sentence's 32-row
// tiles) computes tile (row tile t / 3, part t % 3 of the head's Q | K | V) over
// the 12 quant blocks in block order with every operand loaded up front (the
// i8 fold of i8_block: acc = fma(float(isum), d_w d_a, acc)), splits b + W.x
// hi / lo (i8_small_epi's EPI_QKV arithmetic) into the head's LDS tiles (keys
// past the sentence zero, as attention_short_kernel stages them); then waves
// 0 .. nt - 1 run attention_short_kernel's per-head body on those tiles.  Every
// value is the unfused pair's bit for bit; Q, K and V never leave the CU and
// one launch per layer goes away.
#ifndef QKVA_SMALL
#define QKVA_SMALL 1
#endif

__global__ __launch_bounds__(768) void qkv_attention_small_kernel(GemmArgs g, AttnArgs a) {
    constexpr int D = 32, E = 384, NKB = E / 32, NK = 128, KST = D + 8, VST = NK + 4;
    __shared__ __attribute__((aligned(16))) _Float16 Qh[NK * KST], Ql[NK * KST], Kh[NK * KST], Kl[NK * KST];
    __shared__ __attribute__((aligned(16))) _Float16 Vh[D * VST], Vl[D * VST];
    __shared__ __attribute__((aligned(16))) uint16_t etab[EXP_TABLE_LDS];
    const int h = blockIdx.x, s = blockIdx.y;
    const int beg = a.offsets[s], n = a.offsets[s + 1] - beg;
    if (n > NK || n <= 0 || g.K != E || a.E != E) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
    const int nt = (n + 31) >> 5;
    const int epos = a.expt.pos_n, eneg = a.expt.neg_n;
    for (int i = tid; i < a.expt.n_pad / 8; i += 768) ((uint4 *)etab)[i] = ((const uint4 *)a.expt.compact)[i];

    if (wv < 3 * nt) {
        const int rt = wv / 3, part = wv - 3 * rt, ft0 = 3 * h + part;  // head-major f-tile of Q | K | V
        const int64_t row = beg + 32 * rt + r;                          // (rows past the batch: spare rows)
        // operands of blocks b .. b + 5 in flight (a six-slot ring, slot b % 6)
        constexpr int RING = 6;
        int4v wq[RING], xa[RING];
        uint32_t dw[RING], da[RING];
        auto load = [&](int b) {
            const int sl = b % RING;
            wq[sl] = i8_wq(g.Wi, NKB, ft0, b);
            xa[sl] = *(const int4v *)((const int8_t *)g.A.q + row * E + 32 * b + 16 * hh);
            dw[sl] = ((const uint16_t *)g.Wi.dh)[(((int64_t)ft0 * (NKB >> 2) + (b >> 2)) * 32 + r) * 4 + (b & 3)];
            da[sl] = ((const uint16_t *)g.A.d)[row * NKB + b];
        };
#pragma unroll
        for (int b = 0; b < RING; b++) load(b);
        const int f0 = 32 * ft0 + 16 * hh;
        float4v b4[4];
#pragma unroll
        for (int q = 0; q < 4; q++) b4[q] = *(const float4v *)(g.bias + f0 + 4 * q);
        const float16v zf = {};
        float16v acc = {};
#pragma unroll
        for (int b = 0; b < NKB; b++) {
            const int sl = b % RING;
            const int16v is = __builtin_amdgcn_mfma_i32_32x32x32_i8(wq[sl], xa[sl], __builtin_bit_cast(int16v, zf), 0, 0, 0);
            const int4v ws = int4v{(int)dw[sl], 0, 0, 0}, oh = int4v{hh ? 0 : (int)da[sl], 0, 0, 0};
            const float16v dd = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, ws),
                                                                        __builtin_bit_cast(half8, oh), zf, 0, 0, 0);
            if (b + RING < NKB) load(b + RING);
#pragma unroll
            for (int i = 0; i < 16; i++) acc[i] = __builtin_fmaf((float)is[i], dd[i], acc[i]);
        }
        const int key = 32 * rt + r;
        const bool live = key < n;
        half8 hv[2], lv[2];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const float y = b4[i >> 2][i & 3] + acc[i];
            const _Float16 yh = (_Float16)y;
            hv[i >> 3][i & 7] = live ? yh : (_Float16)0.f;
            lv[i >> 3][i & 7] = live ? (_Float16)(y - (float)yh) : (_Float16)0.f;
        }
        if (part < 2) {
            _Float16 *th = part ? Kh : Qh, *tl = part ? Kl : Ql;
            *(half8 *)&th[key * KST + 16 * hh] = hv[0];
            *(half8 *)&th[key * KST + 16 * hh + 8] = hv[1];
            *(half8 *)&tl[key * KST + 16 * hh] = lv[0];
            *(half8 *)&tl[key * KST + 16 * hh + 8] = lv[1];
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                Vh[(16 * hh + i) * VST + key] = hv[i >> 3][i & 7];
                Vl[(16 * hh + i) * VST + key] = lv[i >> 3][i & 7];
            }
        }
    }
    __syncthreads();
    const int q0 = wv * 32;
    if (q0 >= n) return;
    // attention_short_kernel's per-head body, Q from the LDS tiles
    half8 qh[D / 16], ql[D / 16];
    {
        const int qr = min(q0 + r, n - 1);
#pragma unroll
        for (int ks = 0; ks < D / 16; ks++) {
            qh[ks] = *(const half8 *)&Qh[qr * KST + 16 * ks + 8 * hh];
            ql[ks] = *(const half8 *)&Ql[qr * KST + 16 * ks + 8 * hh];
        }
    }
    const int nkt = (n + 31) >> 5;
    float16v S[4];
    const float16v zero16 = {};
#pragma unroll
    for (int kt = 0; kt < 4; kt++) S[kt] = kt < nkt ? attn_qk<D>(Kh, Kl, KST, 32 * kt, r, hh, qh, ql) : zero16;
    int lim = n - 4 * hh;
    asm volatile("" : "+v"(lim));
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; kt++) {
        if (kt < nkt) {
#pragma unroll
            for (int j = 0; j < 16; j++) S[kt][j] = S[kt][j] * a.scale;
            if (32 * kt + 32 > n) {
#pragma unroll
                for (int j = 0; j < 16; j++)
                    if (32 * kt + (j & 3) + 8 * (j >> 2) >= lim) S[kt][j] = -INFINITY;
            }
#pragma unroll
            for (int j = 0; j < 16; j++) mx = fmaxf(mx, S[kt][j]);
        }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    uint32_t sum = 0;
#pragma unroll
    for (int kt = 0; kt < 4; kt++) {
        if (kt < nkt) {
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const uint32_t hm = f2h(mx - S[kt][j]);
                const float p = h2f(etab[epos + min(hm, (uint32_t)eneg)]);
                S[kt][j] = p;
                sum += (uint32_t)(p * 16777216.0f);
            }
        }
    }
    sum += __shfl_xor(sum, 32);
    const float rs = (float)(1.0 / ((double)sum * 0x1p-24));
    float16v o[D / 32];
#pragma unroll
    for (int dt = 0; dt < D / 32; dt++) o[dt] = zero16;
#pragma unroll
    for (int kt = 0; kt < 4; kt++)
        if (kt < nkt) attn_pv<D>(o, Vh, Vl, VST, 32 * kt, r, hh, S[kt]);
    attn_store_ctx<W_Q4_0, D>(a, o, rs, beg + q0 + r, q0 + r < n, h, hh);
}

hipError_t launch_qkv_attention_small(const GemmArgs &g, const AttnArgs &a, int n_seqs, hipStream_t s) {
    if (!QKVA_SMALL || g.K != 384 || a.E != 384 || a.H * 32 != a.E || n_seqs <= 0) return hipErrorNotSupported;
    hipLaunchKernelGGL(qkv_attention_small_kernel, dim3(a.H, n_seqs), dim3(768), 0, s, g, a);
    return hipGetLastError();
}

// QKV projection fused with attention, for batches whose sentences all have
// n <= 128 tokens, heads of D = 32 (MiniLM) or 64 (e5-base, bge-large): one
// 12-wave workgroup per sentence, so Q, K and V (hi/lo, 4 bytes a value)
// never leave the CU — the unfused pair writes and re-reads 12 bytes per
// token and feature.  The QKV features go through the GEMM main loop in
// 192-feature units (a head pair at D = 32, one head at D = 64), NTW units per
// main loop (ntw, chosen per context at load) and one unit at a time through the attention
// tiles: the main loop (gemm_mainloop, the 128 rows from the sentence's first
// token) computes the unit's head-major QKV features (kernels.h GemmArgs), one
// 16-feature n-tile per wave; b + W.x is split hi/lo into the unit's attention
// tiles in LDS, and 8 attention tasks of 32 queries run as in
// attention_short_kernel: (head, query block) at D = 32, (query block, 32-dim
// half of the context) at D = 64 (the two halves share the scores, computed
// by both waves).
constexpr int QKVA_NW = 12;  // waves
#ifndef QKVA_KB
#define QKVA_KB 2  // 32-wide blocks per main-loop chunk in the fused kernel
#endif
// (Keeping the <= 4 score tiles in registers between the max pass and the
// probability pass instead of recomputing them measured 360 -> 463 us with two
// units per main loop (spills) and 410 -> 413 us with one: the attention
// phase is not MFMA-bound)
// (Software-pipelined score tiles in the attention phase — tile kt + 1's K.Q
// MFMAs in flight during tile kt's softmax — measured 368 -> 392-399 us with
// 28 B/lane of spills: not kept.)

// D: head dim; NTW: 192-feature units per main loop (ntw); PK:
// sentence tiles (a.tiles)
template <int WT, int D, int NTW, bool PK>
__global__ __launch_bounds__(QKVA_NW * 64) void qkv_attention_kernel(GemmArgs g, AttnArgs a) {
    constexpr bool QP = (WT == W_Q4_0 || WT == W_Q4_1);
    constexpr int NW = QKVA_NW, BM = 128, RT = BM / 16;
    constexpr int HU = 192 / (3 * D);  // heads per unit
    constexpr int NK = 128, KST = D + 8, VST = NK + 4;
    constexpr int QKB = QKVA_KB, QLDA = 32 * QKB + (QKB == 2 ? 16 : 8);
    constexpr int A_BUF = BM * QLDA * 2 + (QP ? QKB * BM * 4 : 0);
    constexpr int SLOT = (4 * NK * KST + 2 * D * VST) * 2;  // Qh Ql Kh Kl, Vh Vl of one head, bytes
    constexpr int SMEM = (2 * A_BUF > HU * SLOT) ? 2 * A_BUF : HU * SLOT;
    static_assert(NW * 16 == HU * 3 * D, "one 16-feature n-tile per wave covers a unit");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];
    __shared__ __attribute__((aligned(16))) uint16_t etab[EXP_TABLE_LDS];
    // PK: a workgroup owns a tile of ns <= 4 consecutive sentences (AttnArgs.tiles:
    // runtime.cpp packs them so that their lengths rounded up to 32 sum to
    // <= 128); otherwise one sentence each (the single-sentence code is
    // compiled without any of the packing logic).  The GEMM runs over the
    // tile's n contiguous rows; in the attention tiles sentence j keeps its
    // rows for Q and K but its V^T keys start at a 32-aligned slot vs_j, and
    // its 32-query blocks get waves of their own, so every score, sum and P.V
    // step of a sentence is the one it gets alone in a workgroup (results do
    // not depend on the batch's other sentences, bit for bit).
    __shared__ int qtab[PK ? 4 : 1][4];     // query block -> {first tile row of its sentence, length, first query, vs}
    __shared__ uint8_t vslot[PK ? NK : 1];  // tile row -> V^T key slot
    const int s0 = PK ? a.tiles[2 * blockIdx.x] : (int)blockIdx.x;
    const int ns = PK ? a.tiles[2 * blockIdx.x + 1] : 1;
    const int beg = a.offsets[s0], n = a.offsets[s0 + ns] - beg;
    if (n > NK || n <= 0 || ns > 4) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int gq = lane >> 4, c16 = lane & 15, r = lane & 31, hh = lane >> 5;
    const int epos = a.expt.pos_n, eneg = a.expt.neg_n;
    for (int i = tid; i < a.expt.n_pad / 8; i += NW * 64) ((uint4 *)etab)[i] = ((const uint4 *)a.expt.compact)[i];
    if (PK && tid < NK) {  // read after the main loop's barriers
        int b = 0, vs = 0, qb_b = 0, qb_len = 0, qb_q = 0, qb_vs = 0, slot = 0;
        for (int j = 0; j < ns; j++) {
            const int e = a.offsets[s0 + j + 1] - beg, len = e - b, span = (len + 31) & ~31;
            if (tid >= b && tid < e) slot = vs + tid - b;
            if (32 * tid >= vs && 32 * tid < vs + span) {
                qb_b = b;
                qb_len = len;
                qb_q = 32 * tid - vs;
                qb_vs = vs;
            }
            b = e;
            vs += span;
        }
        vslot[PK ? tid : 0] = (uint8_t)slot;
        if (tid < 4) {
            qtab[PK ? tid : 0][0] = qb_b;
            qtab[PK ? tid : 0][1] = qb_len;
            qtab[PK ? tid : 0][2] = qb_q;
            qtab[PK ? tid : 0][3] = qb_vs;
        }
    }
    auto slot = [&](int hs, int plane) -> _Float16 * {  // plane: 0 Qh 1 Ql 2 Kh 3 Kl 4 Vh 5 Vl
        char *base = smem + hs * SLOT;
        return (_Float16 *)(plane < 4 ? base + plane * NK * KST * 2 : base + 4 * NK * KST * 2 + (plane - 4) * D * VST * 2);
    };
    int lim = n - 4 * hh;  // key mask limit for lane half hh (opaque: not hoisted into SGPRs)
    asm volatile("" : "+v"(lim));
    // wave w: n-tile w of the unit = features 16 w .. 16 w + 15 of the unit's
    // range (g.W is this kernel's own copy of the head-major QKV weights, in
    // plain tile order), i.e. head slot w / (3 D / 16), part (Q, K, V), head
    // dims d0 .. d0 + 15.  Q and K waves run the transposed main loop (a lane
    // holds one row x four adjacent dims: 8-byte stores into the row-major Q / K
    // tiles), V waves the plain one (one dim x four adjacent rows: 8-byte
    // stores into V^T).
    constexpr int WPH = 3 * D / 16;  // waves per head
    const int hs_w = wv / WPH, part_w = (wv % WPH) / (D / 16), d0 = 16 * (wv & (D / 16 - 1));

    for (int qd = 0; qd < a.H / (HU * NTW); qd++) {
        // units NTW qd ..: one main loop (one pass over the sentence's A panel)
        // serves NTW units.  g.W is in grouped tile order (runtime.cpp): wave
        // w's n-tiles nt0 + t are n-tile w of unit NTW qd + t, so acc[..][half]
        // plays the one-unit role of the split below.
        const int64_t nt0 = (int64_t)qd * NTW * NW + NTW * wv;
        float4v acc[RT][NTW];
        STAMP(qd, 0, NW);
        MainloopPre<WT, NW, BM, NTW, QKB> pre;
        mainloop_preload(pre, g, beg, nt0);
        if (part_w == 2)  // ends with a barrier
            gemm_mainloop<WT, NW, BM, NTW, false, QKB>(g, beg, nt0, smem, acc, pre);
        else
            gemm_mainloop<WT, NW, BM, NTW, true, QKB>(g, beg, nt0, smem, acc, pre);
        STAMP(qd, 1, NW);
#pragma unroll
        for (int half = 0; half < NTW; half++) {
            const int pr = NTW * qd + half;
            const int fpair = pr * (HU * 3 * D);  // first head-major feature of the unit
            {   // y = b + W.x -> hi / lo attention tiles (rows >= n: zero keys and values).
                // LDS byte offsets and row limits are rebuilt per pair behind opaque
                // moves, so the compiler does not hoist addresses / row masks out of
                // the pair loop (register pressure: they were spilled to scratch).
                if (part_w == 2) {
                    const float b = g.bias[fpair + 16 * wv + c16];
                    int rl = n - 4 * gq;  // row 16 rt + 4 gq + i is valid while 16 rt + i < rl
                    asm volatile("" : "+v"(rl));
                    uint32_t off = (uint32_t)((char *)slot(hs_w, 4) - smem) + (uint32_t)((d0 + c16) * VST + 4 * gq) * 2;
                    asm volatile("" : "+v"(off));
                    constexpr bool packed = PK;
#pragma unroll
                    for (int rt = 0; rt < RT; rt++) {
                        half4v hv, lv;
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const float y = rt * 16 + i < rl ? b + acc[rt][half][i] : 0.f;
                            hv[i] = (_Float16)y;
                            lv[i] = (_Float16)(y - (float)hv[i]);
                        }
                        if constexpr (packed) {
                            hv = half4v{};
                            lv = half4v{};
                        }
                        *(half4v *)(smem + off + rt * 32) = hv;
                        *(half4v *)(smem + off + D * VST * 2 + rt * 32) = lv;
                    }
                    if constexpr (packed) {
                        // zeros first (key slots between sentences), then each row at its
                        // sentence's slot: one wave's LDS writes land in program order
                        const uint32_t voff = (uint32_t)((char *)slot(hs_w, 4) - smem) + (uint32_t)((d0 + c16) * VST) * 2;
#pragma unroll
                        for (int rt = 0; rt < RT; rt++)
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                const int row = 16 * rt + 4 * gq + i;
                                if (row < n) {
                                    const float y = b + acc[rt][half][i];
                                    const _Float16 yh = (_Float16)y;
                                    const uint32_t o2 = voff + 2u * vslot[row];
                                    *(_Float16 *)(smem + o2) = yh;
                                    *(_Float16 *)(smem + o2 + D * VST * 2) = (_Float16)(y - (float)yh);
                                }
                            }
                    }
                } else {
                    const float4v b4 = *(const float4v *)(g.bias + fpair + 16 * wv + 4 * gq);
                    int rl = n - c16;  // row 16 rt + c16 is valid while 16 rt < rl
                    asm volatile("" : "+v"(rl));
                    uint32_t off = (uint32_t)((char *)slot(hs_w, 2 * part_w) - smem) + (uint32_t)(c16 * KST + d0 + 4 * gq) * 2;
                    asm volatile("" : "+v"(off));
#pragma unroll
                    for (int rt = 0; rt < RT; rt++) {
                        half4v hv, lv;
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const float y = rt * 16 < rl ? b4[i] + acc[rt][half][i] : 0.f;
                            hv[i] = (_Float16)y;
                            lv[i] = (_Float16)(y - (float)hv[i]);
                        }
                        *(half4v *)(smem + off + rt * 16 * KST * 2) = hv;
                        *(half4v *)(smem + off + NK * KST * 2 + rt * 16 * KST * 2) = lv;
                    }
                }
            }
            __syncthreads();
            STAMP(qd, 2 + 2 * half, NW);

            if (wv < 8) {  // attention task (head slot or dim half, query block: 32 queries of one sentence)
                const int hs = HU == 2 ? wv >> 2 : 0, qb = wv & 3, head = HU * pr + hs;
                const int dh = HU == 2 ? 0 : wv >> 2;  // D = 64: the 32-dim half of the context
                int kb = 0, len = n, qrel = 32 * qb, vs = 0;
                if constexpr (PK) {
                    kb = qtab[qb][0];
                    len = qtab[qb][1];
                    qrel = qtab[qb][2];
                    vs = qtab[qb][3];
                }
                if (PK ? len > 0 : qrel < n) {
                    const _Float16 *Qh = slot(hs, 0), *Ql = slot(hs, 1), *Kh = slot(hs, 2), *Kl = slot(hs, 3);
                    const _Float16 *Vh = slot(hs, 4), *Vl = slot(hs, 5);
                    const int qrow = kb + qrel + r;  // tile row of this lane's query (rows past the
                                                     // sentence read finite LDS data; never stored)
                    half8 qh[D / 16], ql[D / 16];
#pragma unroll
                    for (int ks = 0; ks < D / 16; ks++) {
                        qh[ks] = *(const half8 *)(Qh + qrow * KST + 16 * ks + 8 * hh);
                        ql[ks] = *(const half8 *)(Ql + qrow * KST + 16 * ks + 8 * hh);
                    }
                    // two passes over the key tiles (the second recomputes the identical
                    // scores): only one 32-key score tile is live, which keeps this
                    // phase inside the 12-wave register budget next to the GEMM's.
                    // Pass 1 takes the max of the unscaled K.Q: x -> fl(x * scale) is
                    // monotonic for scale > 0, so fl(max * scale) is ggml's max of the
                    // scaled scores.  Keys: the sentence's rows kb .. kb + len (K) and
                    // slots vs .. vs + len (V^T); scores of keys >= len are masked.
                    const int nkt = (len + 31) >> 5;
                    int klim = lim;  // key 32 kt + (j & 3) + 8 (j >> 2) + 4 hh valid while < len
                    if constexpr (PK) {
                        klim = len - 4 * hh;
                        asm volatile("" : "+v"(klim));
                    }
                    auto scores = [&](int kt) {
                        float16v S = attn_qk<D>(Kh, Kl, KST, kb + 32 * kt, r, hh, qh, ql);
                        if (32 * kt + 32 > len) {
#pragma unroll
                            for (int j = 0; j < 16; j++)
                                if (32 * kt + (j & 3) + 8 * (j >> 2) >= klim) S[j] = -INFINITY;
                        }
                        return S;
                    };
                    float mx = -INFINITY;
                    for (int kt = 0; kt < nkt; kt++) {
                        const float16v S = scores(kt);
#pragma unroll
                        for (int j = 0; j < 16; j++) mx = fmaxf(mx, S[j]);
                    }
                    mx = fmaxf(mx, __shfl_xor(mx, 32)) * a.scale;
                    const float2v mx2 = {mx, mx}, sc2 = {a.scale, a.scale};
                    // ggml's double sum of the fp16 probabilities, exactly: every p is a
                    // multiple of 2^-24 in [0, 1], so p * 2^24 is an integer and the
                    // sum of n <= 128 of them fits a uint32
                    uint32_t sum = 0;
                    float16v o[1];
                    o[0] = float16v{};
                    for (int kt = 0; kt < nkt; kt++) {
                        const float16v S = scores(kt);
                        half8 ph[2];
#pragma unroll
                        for (int j = 0; j < 16; j += 2) {
                            // ggml_scale after K.Q, then p = exp_tab[fp16(s - max)]: s - max <= 0, and
                            // fp16(max - s) is its magnitude exactly (IEEE subtraction is sign-symmetric;
                            // masked keys: +inf -> the constant-0 entry).  Two scores per packed f32
                            // op (v_pk_mul / v_pk_add: the same IEEE roundings per element)
                            const float2v d2 = mx2 - float2v{S[j], S[j + 1]} * sc2;
                            uint16_t pb[2];
#pragma unroll
                            for (int e = 0; e < 2; e++) {
                                const float de = d2[e];
                                const uint32_t hm = f2h(de);
                                pb[e] = etab[epos + min(hm, (uint32_t)eneg)];
                                ph[(j + e) >> 3][(j + e) & 7] = __builtin_bit_cast(_Float16, pb[e]);
                            }
                            const float2v p2 = float2v{h2f(pb[0]), h2f(pb[1])} * float2v{16777216.0f, 16777216.0f};
                            sum += (uint32_t)p2[0] + (uint32_t)p2[1];
                        }
                        attn_pv_h<D, 1>(o, Vh, Vl, VST, vs + 32 * kt, r, hh, ph, dh);
                    }
                    sum += __shfl_xor(sum, 32);
                    int orow = qrow;
                    asm volatile("" : "+v"(orow));
                    attn_store_ctx<WT, D, 1>(a, o, (float)(1.0 / ((double)sum * 0x1p-24)), beg + orow, qrel + r < len, head,
                                             hh, dh);
                }
            }
            __syncthreads();  // the next pair's tiles / the next quad's A chunks overwrite the attention tiles
            STAMP(qd, 3 + 2 * half, NW);
        }
    }
}

// QKV projection + attention with producer and consumer waves (Q4_0, head
// dim 32, n_embd 384: MiniLM; reference bert.cpp:905-942).  One 10-wave
// workgroup per sentence (or packed tile, PK, as qkv_attention_kernel).  The
// sentence's 128-row Q8 panel is loaded into LDS once.  Waves 0-5 produce: for
// head h they run the QKV projection of the head's 96 features on the int8
// MFMA over the resident panel (i8_resident_mainloop: no barriers; wave w:
// part w / 2 of Q | K | V, tokens 64 (w & 1) ..), then split b + W.x hi / lo
// into the head's attention tiles.  Waves 6-9 consume: query block w - 6 of
// the head finished in the previous period — the attention task of
// qkv_attention_kernel.  Period p overlaps head p's projection with head
// p - 1's attention; two barriers per period (the consumers are done with the
// tiles; the tiles hold the next head).  LDS: the panel (58 KB), one head's
// tiles (57 KB), the exp table (40 KB).
constexpr int QKPC_NP = 6, QKPC_NW = 10;  // producer waves, all waves
#ifndef QKPC_CPRIO
#define QKPC_CPRIO 0  // A/B: static issue priority of the consumer waves (round 4: 0, 1 and 2 within noise)
#endif
#ifndef QKPC_AHEAD
#define QKPC_AHEAD 2  // the producers' weight blocks in flight (i8_core.h I8ResRing)
#endif

template <bool PK>
__global__ __launch_bounds__(QKPC_NW * 64) void qkv_attention_pc_kernel(GemmArgs g, AttnArgs a) {
    constexpr int WT = W_Q4_0, D = 32, NP = QKPC_NP, NW = QKPC_NW, BM = 128, NT = NW * 64;
    constexpr int NK = 128, KST = D + 8, VST = NK + 4, E = 384, NKB = E / 32;
    using C = I8Chunk<BM, false>;
    constexpr int SLOT = (4 * NK * KST + 2 * D * VST) * 2;  // Qh Ql Kh Kl, Vh Vl of one head, bytes
    __shared__ __attribute__((aligned(16))) char apanel[(E / I8_KC) * C::BYTES];
    __shared__ __attribute__((aligned(16))) char tiles[SLOT];
    __shared__ __attribute__((aligned(16))) uint16_t etab[EXP_TABLE_LDS];
    __shared__ int qtab[PK ? 4 : 1][4];     // query block -> {first tile row of its sentence, length, first query, vs}
    __shared__ uint8_t vslot[PK ? NK : 1];  // tile row -> V^T key slot
    const int s0 = PK ? a.tiles[2 * blockIdx.x] : (int)blockIdx.x;
    const int ns = PK ? a.tiles[2 * blockIdx.x + 1] : 1;
    const int beg = a.offsets[s0], n = a.offsets[s0 + ns] - beg;
    if (n > NK || n <= 0 || ns > 4 || g.K != E || a.E != E) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: the role branches are scalar
    const int r = lane & 31, hh = lane >> 5;
    const int epos = a.expt.pos_n, eneg = a.expt.neg_n;
    for (int i = tid; i < a.expt.n_pad / 8; i += NT) ((uint4 *)etab)[i] = ((const uint4 *)a.expt.compact)[i];
    // the sentence's A panel: rows beg .. beg + 127 (rows past the batch are the
    // workspace's zero spare rows), chunk c = blocks 4c .. 4c + 3 in I8Chunk layout
    for (int it = tid; it < BM * NKB; it += NT) {
        const int row = it / NKB, b = it - row * NKB, c = b >> 2, bb = b & 3;
        const int4v *src = (const int4v *)((const int8_t *)g.A.q + (int64_t)(beg + row) * E + 32 * b);
        char *buf = apanel + c * C::BYTES;
        int4v *dst = (int4v *)(buf + row * I8_LDQ + 32 * bb);
        dst[0] = src[0];
        dst[1] = src[1];
        ((uint16_t *)(buf + C::QB))[bb * BM + row] = ((const uint16_t *)g.A.d)[(int64_t)(beg + row) * NKB + b];
    }
    // the attention tiles start zero: rows / key slots no token writes stay zero for every head
    for (int i = tid; i < SLOT / 16; i += NT) ((uint4 *)tiles)[i] = uint4{0u, 0u, 0u, 0u};
    if (PK && tid < NK) {
        int b = 0, vs = 0, qb_b = 0, qb_len = 0, qb_q = 0, qb_vs = 0, slt = 0;
        for (int j = 0; j < ns; j++) {
            const int e = a.offsets[s0 + j + 1] - beg, len = e - b, span = (len + 31) & ~31;
            if (tid >= b && tid < e) slt = vs + tid - b;
            if (32 * tid >= vs && 32 * tid < vs + span) {
                qb_b = b;
                qb_len = len;
                qb_q = 32 * tid - vs;
                qb_vs = vs;
            }
            b = e;
            vs += span;
        }
        vslot[PK ? tid : 0] = (uint8_t)slt;
        if (tid < 4) {
            qtab[PK ? tid : 0][0] = qb_b;
            qtab[PK ? tid : 0][1] = qb_len;
            qtab[PK ? tid : 0][2] = qb_q;
            qtab[PK ? tid : 0][3] = qb_vs;
        }
    }
    __syncthreads();
    auto plane = [&](int pl) -> _Float16 * {  // 0 Qh 1 Ql 2 Kh 3 Kl 4 Vh 5 Vl
        return (_Float16 *)(pl < 4 ? tiles + pl * NK * KST * 2 : tiles + 4 * NK * KST * 2 + (pl - 4) * D * VST * 2);
    };
    const int H = a.H;
    if (wv < NP) {
        // ---- producer: f-tile 3 h + part (part = w / 2: Q, K, V of head h), tokens
        // 64 (w & 1) .. + 63 as two 32-token t-tiles; lane (r, hh) holds token
        // 32 t + r of its t-tile t, head dims 16 hh .. 16 hh + 15 (i8_core.h)
        const int part = wv >> 1, tt0 = 2 * (wv & 1);
        I8ResRing<WT, 1, QKPC_AHEAD> ring;  // head p + 1's first weight blocks load during head p's split and barriers
        ring.start(g, part);
        for (int p = 0; p <= H; p++) {
            float16v acc[1][2];
            // head p's bias is loaded before its main loop: loaded after it, its wait
            // would also wait for head p + 1's weight blocks the main loop's end issues
            const int f0 = p * 3 * D + part * D + 16 * hh;  // head-major feature of acc[..][0]
            float bias[16];
            if (p < H) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float4v b4 = *(const float4v *)(g.bias + f0 + 4 * q);
#pragma unroll
                    for (int j = 0; j < 4; j++) bias[4 * q + j] = b4[j];
                }
                i8_resident_mainloop<WT, BM, 1, 2>(g, apanel, 3 * p + part, tt0, acc, ring, p + 1 < H ? 3 * (p + 1) + part : -1);
            }
            STAMP(p, 1, NW);
            __syncthreads();  // X: the consumers are done with head p - 1's tiles
            if (p < H) {
#pragma unroll
                for (int t = 0; t < 2; t++) {
                    const int row = 32 * (tt0 + t) + r;  // tile row (token of the tile)
                    if (row < n) {                       // rows >= n stay zero
                        half8 hv[2], lv[2];
#pragma unroll
                        for (int i = 0; i < 16; i++) {
                            const float y = bias[i] + acc[0][t][i];
                            const _Float16 yh = (_Float16)y;
                            hv[i >> 3][i & 7] = yh;
                            lv[i >> 3][i & 7] = (_Float16)(y - (float)yh);
                        }
                        if (part < 2) {  // Q | K: row-major [token][dim]
                            _Float16 *ph = plane(2 * part) + row * KST + 16 * hh, *pl = plane(2 * part + 1) + row * KST + 16 * hh;
                            *(half8 *)ph = hv[0];
                            *(half8 *)(ph + 8) = hv[1];
                            *(half8 *)pl = lv[0];
                            *(half8 *)(pl + 8) = lv[1];
                        } else {  // V^T [dim][key slot]
                            const int slot = PK ? (int)vslot[row] : row;
                            _Float16 *ph = plane(4) + (16 * hh) * VST + slot, *pl = plane(5) + (16 * hh) * VST + slot;
#pragma unroll
                            for (int i = 0; i < 16; i++) {
                                ph[i * VST] = hv[i >> 3][i & 7];
                                pl[i * VST] = lv[i >> 3][i & 7];
                            }
                        }
                    }
                }
            }
            STAMP(p, 2, NW);
            __syncthreads();  // Y: head p's tiles are complete
            STAMP(p + 1, 0, NW);
        }
    } else {
        // ---- consumer: query block qb of head p - 1 (32 queries of one sentence)
        const int qb = wv - NP;
        int lim = n - 4 * hh;  // key mask limit for lane half hh (opaque: not hoisted into SGPRs)
        asm volatile("" : "+v"(lim));
        const _Float16 *Qh = plane(0), *Ql = plane(1), *Kh = plane(2), *Kl = plane(3), *Vh = plane(4), *Vl = plane(5);
        int kb = 0, len = n, qrel = 32 * qb, vs = 0;
        if constexpr (PK) {
            kb = qtab[qb][0];
            len = qtab[qb][1];
            qrel = qtab[qb][2];
            vs = qtab[qb][3];
        }
        const bool qact = PK ? len > 0 : qrel < n;
        const int qrow = kb + qrel + r;  // tile row of this lane's query (rows past the sentence
                                         // read finite LDS data; never stored)
        float16v o[1];
        uint32_t sum = 0;
        // the context of head h, o * (1 / sum) in the O-projection's format
        auto store_ctx = [&](int h) {
            sum += __shfl_xor(sum, 32);
            int orow = qrow;
            asm volatile("" : "+v"(orow));
            attn_store_ctx<WT, D, 1>(a, o, (float)(1.0 / ((double)sum * 0x1p-24)), beg + orow, qrel + r < len, h, hh, 0);
        };
        for (int p = 0; p <= H; p++) {
            const int head = p - 1;
            const bool act = head >= 0 && qact;
            sum = 0;
            if (act) {
                const int nkt = (len + 31) >> 5;
                // key 32 kt + (j & 3) + 8 (j >> 2) + 4 hh valid while < len.  Opaque per
                // head: loop-invariant, the 64 mask compares were hoisted out of the head
                // loop as 64-bit lane masks and spilled the SGPRs
                int klim = PK ? len - 4 * hh : lim;
                asm volatile("" : "+v"(klim));
                half8 qh[D / 16], ql[D / 16];
#pragma unroll
                for (int ks = 0; ks < D / 16; ks++) {
                    qh[ks] = *(const half8 *)(Qh + qrow * KST + 16 * ks + 8 * hh);
                    ql[ks] = *(const half8 *)(Ql + qrow * KST + 16 * ks + 8 * hh);
                }
                auto scores = [&](int kt) {
                    float16v S = attn_qk<D>(Kh, Kl, KST, kb + 32 * kt, r, hh, qh, ql);
                    if (32 * kt + 32 > len) {
#pragma unroll
                        for (int j = 0; j < 16; j++)
                            if (32 * kt + (j & 3) + 8 * (j >> 2) >= klim) S[j] = -INFINITY;
                    }
                    return S;
                };
                // pass 1: the score tiles (up to 4: n <= 128 keys), kept in registers for
                // pass 2, and their max — of the unscaled K.Q: x -> fl(x * scale) is
                // monotonic, so fl(max * scale) is ggml's max of the scaled scores.  The
                // tiles' MFMA chains are independent, so they cover each other's latency
                // (a consumer wave is the only one of its role on its SIMD)
                float16v Sk[4];
                float mx = -INFINITY;
#pragma unroll
                for (int kt = 0; kt < 4; kt++) {
                    if (kt < nkt) {
                        Sk[kt] = scores(kt);
#pragma unroll
                        for (int j = 0; j < 16; j++) mx = fmaxf(mx, Sk[kt][j]);
                    }
                }
                mx = fmaxf(mx, __shfl_xor(mx, 32)) * a.scale;
                const float2v mx2 = {mx, mx}, sc2 = {a.scale, a.scale};
                // pass 2: p = exp_tab[fp16(s - max)], the exact integer sum of p * 2^24, and
                // V.P over the key tiles in order
                o[0] = float16v{};
#pragma unroll
                for (int kt = 0; kt < 4; kt++) {
                    if (kt >= nkt) continue;
                    half8 ph[2];
#pragma unroll
                    for (int j = 0; j < 16; j += 2) {
                        const float2v d2 = mx2 - float2v{Sk[kt][j], Sk[kt][j + 1]} * sc2;
                        uint16_t pb[2];
#pragma unroll
                        for (int e = 0; e < 2; e++) {
                            const uint32_t hm = f2h(d2[e]);
                            pb[e] = etab[epos + min(hm, (uint32_t)eneg)];
                            ph[(j + e) >> 3][(j + e) & 7] = __builtin_bit_cast(_Float16, pb[e]);
                        }
                        const float2v pp = float2v{h2f(pb[0]), h2f(pb[1])} * float2v{16777216.0f, 16777216.0f};
                        sum += (uint32_t)pp[0] + (uint32_t)pp[1];
                    }
                    attn_pv_h<D, 1>(o, Vh, Vl, VST, vs + 32 * kt, r, hh, ph, 0);
                }
            }
            STAMP(p, 1, NW);
            __syncthreads();  // X: this head's tiles may be overwritten
            if (act) store_ctx(head);
            STAMP(p, 2, NW);
            __syncthreads();  // Y
            STAMP(p + 1, 0, NW);
        }
    }
}

template <int WT, int D>
static hipError_t qkv_attn_t(const GemmArgs &g, const AttnArgs &a, int n_blocks, int ntw, hipStream_t s) {
    const bool pk = a.tiles != nullptr;
    if constexpr (D == 32 && WT == W_Q4_0) {
        if (ntw == 0) {  // producer / consumer waves (qkv_attention_pc_kernel; g.Wi: int8 QKV weights)
            if (pk)
                hipLaunchKernelGGL((qkv_attention_pc_kernel<true>), dim3(n_blocks), dim3(QKPC_NW * 64), 0, s, g, a);
            else
                hipLaunchKernelGGL((qkv_attention_pc_kernel<false>), dim3(n_blocks), dim3(QKPC_NW * 64), 0, s, g, a);
            return hipGetLastError();
        }
    }
    if (ntw == 2) {
        if (pk)
            hipLaunchKernelGGL((qkv_attention_kernel<WT, D, 2, true>), dim3(n_blocks), dim3(QKVA_NW * 64), 0, s, g, a);
        else
            hipLaunchKernelGGL((qkv_attention_kernel<WT, D, 2, false>), dim3(n_blocks), dim3(QKVA_NW * 64), 0, s, g, a);
    } else {
        if (pk)
            hipLaunchKernelGGL((qkv_attention_kernel<WT, D, 1, true>), dim3(n_blocks), dim3(QKVA_NW * 64), 0, s, g, a);
        else
            hipLaunchKernelGGL((qkv_attention_kernel<WT, D, 1, false>), dim3(n_blocks), dim3(QKVA_NW * 64), 0, s, g, a);
    }
    return hipGetLastError();
}

template <int WT>
static hipError_t qkv_attn_w(const GemmArgs &g, const AttnArgs &a, int n_blocks, int ntw, hipStream_t s) {
    switch (a.H > 0 ? a.E / a.H : 0) {
        case 32: return qkv_attn_t<WT, 32>(g, a, n_blocks, ntw, s);
        case 64: return qkv_attn_t<WT, 64>(g, a, n_blocks, ntw, s);
    }
    return hipErrorInvalidValue;
}

static int n_cus() {
    static int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            c = 256;
        return c;
    }();
    return n;
}

// The kernel holds one workgroup per CU (LDS) and its cost per workgroup is
// nearly independent of the rows used (the GEMM runs 128 rows), so it runs in
// rounds of n_cus tiles; the packed variant costs ~8 % more per workgroup
// (measured: 414 vs 382 us at 1024 single-sentence tiles), so packing is used
// only when it saves more than that in rounds.
#ifdef PHASE_STAMPS
// development builds only (tools/variant_lib.sh with -DPHASE_STAMPS=1): point
// this translation unit's stamp buffer at a device buffer (tools/pipe_stamps.py)
hipError_t stamps_set(unsigned long long *buf, int nblk) {
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_buf), &buf, sizeof(buf));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_nblk), &nblk, sizeof(nblk));
    return e;
}
}  // namespace bertamd
// (not declared in bert_amd.h: exists only in -DPHASE_STAMPS variant libraries)
extern "C" __attribute__((visibility("default"))) int bert_amd_dev_stamps(void *buf, int nblk) {
    return bertamd::stamps_set((unsigned long long *)buf, nblk) == hipSuccess ? 0 : -1;
}
namespace bertamd {
#endif

bool qkv_attention_pack_pays(int n_seqs, int n_tiles) {
    const int64_t c = n_cus(), plain = (n_seqs + c - 1) / c, packed = (n_tiles + c - 1) / c;
    return n_tiles < n_seqs && packed * 11 < plain * 10;
}

bool qkv_attention_supported(int wtype, int E, int H, int max_len, int ntw) {
    if (H <= 0 || E % H || ntw < 0 || ntw > 2) return false;
    const int D = E / H;
    if (ntw == 0) return max_len <= 128 && D == 32 && E == 384 && wtype == W_Q4_0;  // qkv_attention_pc_kernel
    return max_len <= 128 && (D == 32 || D == 64) && H % (192 / (3 * D) * ntw) == 0 && E % KC == 0 &&
           wtype != W_F32;
}

hipError_t launch_qkv_attention(int wtype, const GemmArgs &g, const AttnArgs &a, int n_blocks, int ntw, hipStream_t s) {
    if (!qkv_attention_supported(wtype, a.E, a.H, 0, ntw)) return hipErrorInvalidValue;
    switch (wtype) {
        case W_F16: return qkv_attn_w<W_F16>(g, a, n_blocks, ntw, s);
        case W_Q4_0: return qkv_attn_w<W_Q4_0>(g, a, n_blocks, ntw, s);
        case W_Q4_1: return qkv_attn_w<W_Q4_1>(g, a, n_blocks, ntw, s);
    }
    return hipErrorInvalidValue;
}

// Attention for 128 < n <= 512: one 8-wave workgroup per (256-query block,
// head, sentence), wave w owning queries 32w..32w+31 of the block.  Keys
// stream through LDS in 128-key chunks, twice: pass 1 finds every query's
// maximum score; pass 2 recomputes the identical scores (same MFMA sequence)
// for p = exp_tab[fp16(s - max)], the exact double sum and P.V.  So ggml's
// soft_max (global max first) holds without materialising the n x n scores.
// Eight waves share each staged chunk (two per SIMD, one workgroup per CU at
// head dim 64: 110 KiB of LDS), so one wave's MFMAs cover the other's
// softmax VALU and the chunk loads are amortised over 256 queries.
constexpr int ATTN_LONG_NW = 8, ATTN_LONG_QB = 32 * ATTN_LONG_NW;  // waves, queries per workgroup

#ifndef ATTN_LONG_KT_UNROLL
#define ATTN_LONG_KT_UNROLL(D) 1  // A/B: -D'ATTN_LONG_KT_UNROLL(D)=4' (the round-2 form)
#endif

// keys per staged chunk, waves per SIMD (the register budget: 4 -> 128 VGPRs).
// Head dim 64 stages 64-key chunks (77 KiB of LDS) so that two workgroups share
// a CU, four waves per SIMD (round 4: C5 attention 1531 -> 1383 us, C4 715 ->
// 674 us at 128 VGPRs, 24-28 B/lane of scratch outside the key-tile loop)
#ifndef ATTN_LONG_NK
#define ATTN_LONG_NK(D) ((D) == 64 ? 64 : 128)
#endif
#ifndef ATTN_LONG_OCC
#define ATTN_LONG_OCC(D) 4
#endif
#ifndef ATTN_LONG_PRIO
#define ATTN_LONG_PRIO 0  // A/B: issue priority 1 for waves NW/2 .. NW - 1
#endif

template <int WT, int D>
// D = 32: two workgroups per CU (78 KiB of LDS each; the register budget
// capped at 128 for four waves per SIMD) — 423 -> 333 us at MiniLM 512 x 256
__global__ __launch_bounds__(ATTN_LONG_NW * 64, ATTN_LONG_OCC(D)) void attention_long_kernel(AttnArgs a) {
    constexpr int NK = ATTN_LONG_NK(D), KST = D + 8, VST = NK + 4, NT = ATTN_LONG_NW * 64;
    __shared__ __attribute__((aligned(16))) _Float16 Kh[NK * KST], Kl[NK * KST], Vh[D * VST], Vl[D * VST];
    __shared__ __attribute__((aligned(16))) uint16_t etab[EXP_TABLE_LDS];
    const int qb = blockIdx.x, h = blockIdx.y, s = blockIdx.z;
    const int beg = a.offsets[s], n = a.offsets[s + 1] - beg;
    // n <= 128 belongs to attention_short_kernel, whatever the chunk size NK
    if (n <= 128 || qb * ATTN_LONG_QB >= n) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
    const int E = a.E, E2 = 2 * E;
    const bool v_aligned = (beg & 7) == 0;
    const int epos = a.expt.pos_n, eneg = a.expt.neg_n;
    for (int i = tid; i < a.expt.n_pad / 8; i += NT) ((uint4 *)etab)[i] = ((const uint4 *)a.expt.compact)[i];

    const int q0 = qb * ATTN_LONG_QB + wv * 32;
    const bool active = q0 < n;  // wave-uniform
    half8 qh[D / 16], ql[D / 16];
    {
        const int qr = min(q0 + r, n - 1);
        const int64_t off = (int64_t)(beg + qr) * E2 + h * D + 8 * hh;
#pragma unroll
        for (int ks = 0; ks < D / 16; ks++) {
            qh[ks] = *(const half8 *)(a.qk_hi + off + 16 * ks);
            ql[ks] = *(const half8 *)(a.qk_lo + off + 16 * ks);
        }
    }
    // The 2*nch stages (pass 1: K of chunk c; pass 2: K and V^T of chunk c)
    // are register-prefetched one stage ahead: KIT / VIT 16-byte pieces per
    // thread and plane.
    constexpr int KIT = NK * (D / 8) / NT, VIT = D * (NK / 8) / NT;
    static_assert(KIT * NT == NK * (D / 8) && VIT * NT == D * (NK / 8), "whole 16-byte pieces per thread");
    uint4 pkh[KIT], pkl[KIT];
    half8 pvh[VIT], pvl[VIT];
    auto fetch = [&](int c, bool with_v) {
        const int kbase = c * NK;
#pragma unroll
        for (int i = 0; i < KIT; i++) {
            const int idx = tid + NT * i, key = idx / (D / 8), col = (idx - key * (D / 8)) * 8;
            pkh[i] = pkl[i] = uint4{0u, 0u, 0u, 0u};
            if (kbase + key < n) {
                const int64_t off = (int64_t)(beg + kbase + key) * E2 + E + h * D + col;
                pkh[i] = *(const uint4 *)(a.qk_hi + off);
                pkl[i] = *(const uint4 *)(a.qk_lo + off);
            }
        }
        if (!with_v) return;
#pragma unroll
        for (int i = 0; i < VIT; i++) {
            const int idx = tid + NT * i, d = idx / (NK / 8), k8 = (idx - d * (NK / 8)) * 8;
            const int64_t off = (int64_t)(h * D + d) * a.ldv + beg + kbase + k8;
            pvh[i] = pvl[i] = half8{};
            if (kbase + k8 + 8 <= n && v_aligned) {
                pvh[i] = *(const half8 *)(a.vt_hi + off);
                pvl[i] = *(const half8 *)(a.vt_lo + off);
            } else {
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (kbase + k8 + j < n) {
                        pvh[i][j] = ((const _Float16 *)a.vt_hi)[off + j];
                        pvl[i][j] = ((const _Float16 *)a.vt_lo)[off + j];
                    }
            }
        }
    };
    auto commit = [&](bool with_v) {
#pragma unroll
        for (int i = 0; i < KIT; i++) {
            const int idx = tid + NT * i, key = idx / (D / 8), col = (idx - key * (D / 8)) * 8;
            *(uint4 *)&Kh[key * KST + col] = pkh[i];
            *(uint4 *)&Kl[key * KST + col] = pkl[i];
        }
        if (!with_v) return;
#pragma unroll
        for (int i = 0; i < VIT; i++) {
            const int idx = tid + NT * i, d = idx / (NK / 8), k8 = (idx - d * (NK / 8)) * 8;
            const half8 vh = pvh[i], vl = pvl[i];
            *(half4v *)&Vh[d * VST + k8] = half4v{vh[0], vh[1], vh[2], vh[3]};
            *(half4v *)&Vh[d * VST + k8 + 4] = half4v{vh[4], vh[5], vh[6], vh[7]};
            *(half4v *)&Vl[d * VST + k8] = half4v{vl[0], vl[1], vl[2], vl[3]};
            *(half4v *)&Vl[d * VST + k8 + 4] = half4v{vl[4], vl[5], vl[6], vl[7]};
        }
    };
    // scaled, masked scores of the 32-key tile starting at absolute key k0
    int lim = n - 4 * hh;
    asm volatile("" : "+v"(lim));
    // unscaled (ggml_scale after K.Q is applied where the scores are used: pass 1
    // takes the max of the unscaled scores, exact since x -> fl(x * scale) is
    // monotonic for scale > 0; pass 2 scales them)
    auto scores = [&](int k0, int kl0) {
        float16v S = attn_qk<D>(Kh, Kl, KST, kl0, r, hh, qh, ql);
        if (k0 + 32 > n) {
#pragma unroll
            for (int j = 0; j < 16; j++)
                if (k0 + (j & 3) + 8 * (j >> 2) >= lim) S[j] = -INFINITY;
        }
        return S;
    };
    const int nch = (n + NK - 1) / NK;
    float mx = -INFINITY;
    uint64_t sum = 0;  // the probabilities' exact sum in units of 2^-24 (as in attention_short_kernel)
    float16v o[D / 32];
    const int sbid = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);  // (phase stamps)
    (void)sbid;
#if ATTN_LONG_PRIO
    if (wv >= ATTN_LONG_NW / 2) __builtin_amdgcn_s_setprio(1);  // the later-dispatched half of each SIMD pair
#endif
    // stage st: the staged chunk (pass 1: K of chunk st; pass 2: K and V^T of
    // chunk st - nch) goes from registers to LDS, and the next stage's loads start
    auto stage = [&](int st) {
        STAMPB(sbid, st, 0, ATTN_LONG_NW);
        __syncthreads();  // the previous stage's LDS reads are done
        commit(st >= nch);
        __syncthreads();
        STAMPB(sbid, st, 1, ATTN_LONG_NW);
        if (st + 1 < 2 * nch) fetch(st + 1 < nch ? st + 1 : st + 1 - nch, st + 1 >= nch);
    };
    fetch(0, false);
    // pass 1: maxima.  Two key tiles at a time (independent MFMA chains; o is not live yet)
    for (int c = 0; c < nch; c++) {
        stage(c);
        if (active) {
#pragma unroll
            for (int kt = 0; kt < NK / 32; kt += 2) {
                const int k0 = c * NK + 32 * kt;
                if (k0 >= n) break;
                const float16v S0 = scores(k0, 32 * kt);
                if (k0 + 32 < n) {
                    const float16v S1 = scores(k0 + 32, 32 * kt + 32);
#pragma unroll
                    for (int j = 0; j < 16; j++) mx = fmaxf(mx, fmaxf(S0[j], S1[j]));
                } else {
#pragma unroll
                    for (int j = 0; j < 16; j++) mx = fmaxf(mx, S0[j]);
                }
            }
        }
        STAMPB(sbid, c, 2, ATTN_LONG_NW);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32)) * a.scale;
#pragma unroll
    for (int dt = 0; dt < D / 32; dt++) o[dt] = float16v{};
    // pass 2: p, sum, P.V.  The key-tile loop stays rolled — unrolled, the
    // compiler keeps more tiles' operands live: at D = 64 it spilled 80 B/lane
    // at 256 VGPRs (208 VGPRs, no scratch rolled); at D = 32 rolled is what fits
    // the 128-VGPR budget of two workgroups per CU.  (Software-pipelining the
    // score tiles — the next tile's K.Q MFMAs issued before this tile's softmax
    // — measured 1 - 3 % slower: not kept.)
    const float2v mx2 = {mx, mx}, sc2 = {a.scale, a.scale};
    for (int c = 0; c < nch; c++) {
        stage(nch + c);
        if (active) {
            constexpr int KTU = ATTN_LONG_KT_UNROLL(D);
#pragma unroll KTU
            for (int kt = 0; kt < NK / 32; kt++) {
                const int k0 = c * NK + 32 * kt;
                if (k0 >= n) break;
                float16v S = scores(k0, 32 * kt);
                uint32_t part = 0;  // 16 terms <= 2^24
#pragma unroll
                for (int j = 0; j < 16; j += 2) {
                    // |s - max| as fp16 (s scaled); masked -inf -> +inf -> 0.  Two scores
                    // per packed f32 op (the same IEEE roundings per element)
                    const float2v d2 = mx2 - float2v{S[j], S[j + 1]} * sc2;
#pragma unroll
                    for (int e = 0; e < 2; e++) {
                        const uint32_t hm = f2h(d2[e]);
                        S[j + e] = h2f(etab[epos + min(hm, (uint32_t)eneg)]);
                    }
                    const float2v p2 = float2v{S[j], S[j + 1]} * float2v{16777216.0f, 16777216.0f};
                    part += (uint32_t)p2[0] + (uint32_t)p2[1];
                }
                sum += part;
                attn_pv<D>(o, Vh, Vl, VST, 32 * kt, r, hh, S);
            }
        }
        STAMPB(sbid, nch + c, 2, ATTN_LONG_NW);
    }
    double tot = (double)sum * 0x1p-24;  // exact (< 2^34 units), and so is the pair sum
    tot += __shfl_xor(tot, 32);
    if (active) attn_store_ctx<WT, D>(a, o, (float)(1.0 / tot), beg + q0 + r, q0 + r < n, h, hh);
}

// ---------------------------------------------------------------------------
// Mean pool + L2 normalise for one sentence (bert.cpp:995-1006):
// m[e] = sum_t x[t][e] * (1.0f/N); s = sum m^2 (double); len = sqrtf(s);
// out = m * (1.0f/len).
// Mean pooling as ggml's mul_mat by a column of 1/N (bert.cpp:995-1001), then
// sum of squares in double, sqrtf, 1.0f/len, scale (:1002-1006).  One thread
// per 4 columns; the token loop is unrolled 8-deep so loads are in flight
// together (the fma chain per column stays in token order).
// out_row (optional): the output row of each sentence of the batch.
__global__ __launch_bounds__(256) void pool_l2_kernel(const float *X, const int32_t *offsets, int E, float *out,
                                                      const int32_t *out_row) {
    __shared__ double red[4];
    const int s = blockIdx.x, tid = threadIdx.x, c = 4 * tid;
    const int beg = offsets[s], n = offsets[s + 1] - beg;
    const float invN = 1.0f / n;
    float4v acc = {0.f, 0.f, 0.f, 0.f};
    if (c < E) {
        const float *p = X + (int64_t)beg * E + c;
        int t = 0;
        for (; t + 8 <= n; t += 8) {
            float4v x[8];
#pragma unroll
            for (int u = 0; u < 8; u++) x[u] = *(const float4v *)(p + (int64_t)(t + u) * E);
#pragma unroll
            for (int u = 0; u < 8; u++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[j] = fmaf(x[u][j], invN, acc[j]);
        }
        for (; t < n; t++) {
            const float4v x = *(const float4v *)(p + (int64_t)t * E);
#pragma unroll
            for (int j = 0; j < 4; j++) acc[j] = fmaf(x[j], invN, acc[j]);
        }
    }
    double ss = 0.0;
#pragma unroll
    for (int j = 0; j < 4; j++) ss += (double)(acc[j] * acc[j]);
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    const double tot = red[0] + red[1] + red[2] + red[3];
    const float len = sqrtf((float)tot);
    const float r = 1.0f / len;
    const int64_t orow = out_row ? out_row[s] : s;
    if (c < E) *(float4v *)(out + orow * E + c) = float4v{acc[0] * r, acc[1] * r, acc[2] * r, acc[3] * r};
}

// Token ids of a batch in a new sentence order: sentence i of the new batch
// is sentence perm[i] of the caller's (one workgroup per sentence).
__global__ __launch_bounds__(128) void gather_tokens_kernel(const int32_t *__restrict__ src, const int32_t *__restrict__ src_off,
                                                            const int32_t *__restrict__ perm,
                                                            const int32_t *__restrict__ dst_off, int32_t *__restrict__ dst) {
    const int i = blockIdx.x, s = perm[i];
    const int b = src_off[s], n = src_off[s + 1] - b, d = dst_off[i];
    for (int t = threadIdx.x; t < n; t += 128) dst[d + t] = src[b + t];
}

// ---------------------------------------------------------------------------
// launchers
template <int WT>
static hipError_t embed_t(EmbedArgs a, int Mpad, hipStream_t s) {
    if (a.n_seqs > 64)
        hipLaunchKernelGGL(row_pos_kernel, dim3(a.n_seqs), dim3(128), 0, s, a.offsets, a.rowpos);
    else
        a.rowpos = nullptr;  // embed_ln_kernel searches the offsets
    switch (a.E) {
        case 384: hipLaunchKernelGGL((embed_ln_kernel<WT, 12>), dim3(Mpad / 16), dim3(256), 0, s, a); break;
        case 768: hipLaunchKernelGGL((embed_ln_kernel<WT, 24>), dim3(Mpad / 16), dim3(256), 0, s, a); break;
        case 1024: hipLaunchKernelGGL((embed_ln_kernel<WT, 32>), dim3(Mpad / 16), dim3(256), 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_embed(int wtype, const EmbedArgs &a, int Mpad, hipStream_t s) {
    switch (wtype) {
        case W_F32: return embed_t<W_F32>(a, Mpad, s);
        case W_F16: return embed_t<W_F16>(a, Mpad, s);
        case W_Q4_0: return embed_t<W_Q4_0>(a, Mpad, s);
        case W_Q4_1: return embed_t<W_Q4_1>(a, Mpad, s);
    }
    return hipErrorInvalidValue;
}

// 384-wide LN GEMMs (one 12-wave workgroup per CU): 64-row tiles cost half a
// 128-row one (tools/gemm_bench: 162 us either way at M = 131072), so they are
// used when they take fewer rounds of n_cus workgroups than twice the 128-row
// count — i.e. when 128-row tiles would leave the last round mostly empty.
// (and 32-row tiles for small batches, one server sentence = 128 rows: a row
// tile's latency, not the chip, bounds those; the per-row sums do not depend on
// the tile height)
#ifndef LN_SMALL_ROWS
#define LN_SMALL_ROWS 512
#endif
#ifndef LN_SMALL_BM
#define LN_SMALL_BM 16
#endif
static bool ln_half_rows(int Mpad) {
    const int c = n_cus(), r128 = (Mpad / 128 + c - 1) / c, r64 = (Mpad / 64 + c - 1) / c;
    return r64 < 2 * r128;
}

template <int WT, int EPI, int BN, int NW, int BM>
static hipError_t gemm_t(const GemmArgs &a, int Mpad, hipStream_t s) {
    const int mt = Mpad / BM, nt = a.N / BN;
    int grid = mt * nt;
    if constexpr ((WT == W_Q4_0 || WT == W_Q4_1 || WT == W_F16) && EPI == EPI_GELU_ACT) {
        // persistent: one workgroup per CU (the GELU table fills the LDS), a multiple of 8
        if (0x8000 + a.gelu.neg_n + 1 > GELU_FLAT_LDS) return hipErrorInvalidValue;
        grid = std::min(grid, std::max(8, n_cus() / 8 * 8));
    }
    hipLaunchKernelGGL((gemm_kernel<WT, EPI, BN, NW, BM>), dim3(grid), dim3(NW * 64), 0, s, a, mt, nt);
    return hipGetLastError();
}

// Q4 weights (split hi/lo planes, two MFMAs per block): waves own 32 columns x
// 128 rows, so each W fragment pair read from L2 feeds 8 row tiles and the
// L2 stream stays at (M/128) * N * K * 4 bytes.  F16/F32: waves own 64 columns x
// 64 rows.  LayerNorm GEMMs own whole rows (BN = E).
template <int WT>
static hipError_t gemm_w(int epi, const GemmArgs &a, int Mpad, hipStream_t s) {
    if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
        if (epi == EPI_QKV) return gemm_t<WT, EPI_QKV, 384, 12, 128>(a, Mpad, s);
        if (epi == EPI_GELU_ACT)  // 12 waves (3 per SIMD) where N allows; the GELU table fills the LDS
            return a.N % 384 == 0 ? gemm_t<WT, EPI_GELU_ACT, 384, 12, 128>(a, Mpad, s)
                                  : gemm_t<WT, EPI_GELU_ACT, 256, 8, 128>(a, Mpad, s);
        if (epi == EPI_LN && a.N == 384)
            return Mpad <= LN_SMALL_ROWS ? gemm_t<WT, EPI_LN, 384, 12, LN_SMALL_BM>(a, Mpad, s)
                   : ln_half_rows(Mpad)  ? gemm_t<WT, EPI_LN, 384, 12, 64>(a, Mpad, s)
                                         : gemm_t<WT, EPI_LN, 384, 12, 128>(a, Mpad, s);
        if (epi == EPI_RESID) return gemm_t<WT, EPI_RESID, 256, 8, 128>(a, Mpad, s);
    } else if constexpr (WT == W_F16) {
        // tools/gemm_bench (e5 shapes): 12-wave 384-column tiles win by 1.3-1.8x over
        // 4-6 waves and by 11-14 % over 768 x 64 tiles (qkv 343 us, up+GELU 368 us)
        if (epi == EPI_QKV) return gemm_t<WT, EPI_QKV, 384, 12, 128>(a, Mpad, s);
        if (epi == EPI_GELU_ACT)
            return a.N % 384 == 0 ? gemm_t<WT, EPI_GELU_ACT, 384, 12, 128>(a, Mpad, s)
                                  : gemm_t<WT, EPI_GELU_ACT, 256, 4, 64>(a, Mpad, s);
        switch (a.N) {
            case 384:
                return Mpad <= LN_SMALL_ROWS ? gemm_t<WT, EPI_LN, 384, 12, LN_SMALL_BM>(a, Mpad, s)
                       : ln_half_rows(Mpad)  ? gemm_t<WT, EPI_LN, 384, 12, 64>(a, Mpad, s)
                                             : gemm_t<WT, EPI_LN, 384, 12, 128>(a, Mpad, s);
            case 768: return gemm_t<WT, EPI_LN, 768, 12, 64>(a, Mpad, s);
            case 1024: return gemm_t<WT, EPI_LN, 1024, 8, 32>(a, Mpad, s);
        }
    } else {
        if (epi == EPI_QKV) return gemm_t<WT, EPI_QKV, 384, 6, 64>(a, Mpad, s);
        if (epi == EPI_GELU_ACT) return gemm_t<WT, EPI_GELU_ACT, 256, 4, 64>(a, Mpad, s);
        switch (a.N) {
            case 384: return gemm_t<WT, EPI_LN, 384, 6, 64>(a, Mpad, s);
            case 768: return gemm_t<WT, EPI_LN, 768, 12, 64>(a, Mpad, s);
            case 1024: return gemm_t<WT, EPI_LN, 1024, 8, 32>(a, Mpad, s);
        }
    }
    return hipErrorInvalidValue;
}

// Q4 weights: a 12-wave workgroup owns whole 384-wide rows; wider rows would
// spill (two W blocks in flight x hi/lo), so they add the residual in the GEMM
// and normalise in launch_ln.  F16 / F32 fuse LN up to 1024.
bool gemm_gelu_blk8(int wtype) { return wtype == W_Q4_0 || wtype == W_Q4_1; }

bool gemm_ln_fused(int wtype, int N) {
    if (wtype == W_Q4_0 || wtype == W_Q4_1) return N == 384;
    return N == 384 || N == 768 || N == 1024;
}

bool gemm_shape_supported(int epi, int N, int K) {
    if (K % KC) return false;
    if (epi == EPI_QKV) return N % 384 == 0;
    if (epi == EPI_GELU_ACT || epi == EPI_RESID) return N % 256 == 0;
    return N == 384 || N == 768 || N == 1024;
}

hipError_t launch_gemm(int wtype, int epi, int /*unused*/, const GemmArgs &a, int Mpad, hipStream_t s) {
    if (!gemm_shape_supported(epi, a.N, a.K) || Mpad % BM_MAX) return hipErrorInvalidValue;
    switch (wtype) {
        case W_F32: return gemm_w<W_F32>(epi, a, Mpad, s);
        case W_F16: return gemm_w<W_F16>(epi, a, Mpad, s);
        case W_Q4_0: return gemm_w<W_Q4_0>(epi, a, Mpad, s);
        case W_Q4_1: return gemm_w<W_Q4_1>(epi, a, Mpad, s);
    }
    return hipErrorInvalidValue;
}

template <int WT, int D>
static hipError_t attn_t(const AttnArgs &a, int n_seqs, int max_len, hipStream_t s) {
    // heads per workgroup: all of a sentence's heads when the batch alone fills
    // the GPU (the exp table is staged once), fewer for small batches
    const int hpw = std::max(1, std::min(a.H, n_seqs / 64));
    const int groups = (a.H + hpw - 1) / hpw;
    hipLaunchKernelGGL((attention_short_kernel<WT, D>), dim3(groups, n_seqs), dim3(256), 0, s, a, hpw);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || max_len <= 128) return e;
    hipLaunchKernelGGL((attention_long_kernel<WT, D>), dim3((max_len + ATTN_LONG_QB - 1) / ATTN_LONG_QB, a.H, n_seqs),
                       dim3(ATTN_LONG_NW * 64), 0, s, a);
    return hipGetLastError();
}

template <int WT>
static hipError_t attn_w(int d, const AttnArgs &a, int n_seqs, int max_len, hipStream_t s) {
    if (d == 32) return attn_t<WT, 32>(a, n_seqs, max_len, s);
    if (d == 64) return attn_t<WT, 64>(a, n_seqs, max_len, s);
    return hipErrorInvalidValue;
}

hipError_t launch_attention(int wtype, int d_head, const AttnArgs &a, int n_seqs, int max_len, hipStream_t s) {
    if (max_len > 512) return hipErrorInvalidValue;
    switch (wtype) {
        case W_F32: return attn_w<W_F32>(d_head, a, n_seqs, max_len, s);
        case W_F16: return attn_w<W_F16>(d_head, a, n_seqs, max_len, s);
        case W_Q4_0: return attn_w<W_Q4_0>(d_head, a, n_seqs, max_len, s);
        case W_Q4_1: return attn_w<W_Q4_1>(d_head, a, n_seqs, max_len, s);
    }
    return hipErrorInvalidValue;
}

template <int WT>
static hipError_t ln_w(float *X, int Mpad, int E, const float *w, const float *b, float eps, const ActPtr &out,
                       hipStream_t s) {
    switch (E) {
        case 384: hipLaunchKernelGGL((ln_rows_kernel<WT, 12>), dim3(Mpad / 16), dim3(256), 0, s, X, w, b, eps, out); break;
        case 768: hipLaunchKernelGGL((ln_rows_kernel<WT, 24>), dim3(Mpad / 16), dim3(256), 0, s, X, w, b, eps, out); break;
        case 1024: hipLaunchKernelGGL((ln_rows_kernel<WT, 32>), dim3(Mpad / 16), dim3(256), 0, s, X, w, b, eps, out); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_ln(int wtype, float *X, int Mpad, int E, const float *w, const float *b, float eps,
                     const ActPtr &out, hipStream_t s) {
    switch (wtype) {
        case W_F32: return ln_w<W_F32>(X, Mpad, E, w, b, eps, out, s);
        case W_F16: return ln_w<W_F16>(X, Mpad, E, w, b, eps, out, s);
        case W_Q4_0: return ln_w<W_Q4_0>(X, Mpad, E, w, b, eps, out, s);
        case W_Q4_1: return ln_w<W_Q4_1>(X, Mpad, E, w, b, eps, out, s);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_pool(const float *X, const int32_t *offsets, int n_seqs, int E, float *out, hipStream_t s,
                       const int32_t *out_row) {
    if (E > 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pool_l2_kernel, dim3(n_seqs), dim3(256), 0, s, X, offsets, E, out, out_row);
    return hipGetLastError();
}

hipError_t launch_gather_tokens(const int32_t *src, const int32_t *src_off, const int32_t *perm, const int32_t *dst_off,
                                int32_t *dst, int n_seqs, hipStream_t s) {
    hipLaunchKernelGGL(gather_tokens_kernel, dim3(n_seqs), dim3(128), 0, s, src, src_off, perm, dst_off, dst);
    return hipGetLastError();
}

}  // namespace bertamd
