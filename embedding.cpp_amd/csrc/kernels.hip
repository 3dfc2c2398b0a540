// kernels.hip — the CDNA4 (gfx950) kernel pipeline behind bert_eval_batch.
//
// Replaces the ggml CPU ops emitted by the reference's bert_build
// (reference bert.cpp:845-1012; op inventory SURVEY.md §2a).  Numerics follow
// the ggml semantics restated in SURVEY.md Appendix A wherever they are cheap
// to reproduce exactly (Q8 activation quantisation, fp16 GELU/exp tables,
// double-accumulated LayerNorm and softmax sums, fp16 activation rounding);
// the weight GEMMs run on fp16 MFMA with the Q4 weights dequantised in
// registers (DESIGN.md §3-4 for the precision argument).
//
// Compiled with -ffp-contract=off: every fused multiply-add below is explicit.
#include "kernels.h"

namespace bertamd {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float float4v __attribute__((ext_vector_type(4)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef float float16v __attribute__((ext_vector_type(16)));
typedef _Float16 half4v __attribute__((ext_vector_type(4)));

constexpr int BM_MAX = GEMM_BM;  // M padding unit; GEMM tiles use BM = 64 or 32
constexpr int KC = 64;       // K per main-loop chunk = two 32-element quant blocks
constexpr int LDA_H = 80;    // fp16 A-tile row stride (halves) = 160 B: ds_read_b128 conflict-free
constexpr int LDA_F = 72;    // f32  A-tile row stride (floats) = 288 B: ds_read_b128 conflict-free

__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

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
        const float d = amax / 127.f;
        const float id = amax != 0.f ? 127.f / amax : 0.f;
        uint32_t pk[8];
        int qsum = 0;
#pragma unroll
        for (int w = 0; w < 8; w++) {
            uint32_t x = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int q = (int)rintf(v[4 * w + j] * id);
                qsum += q;
                x |= ((uint32_t)(q & 0xff)) << (8 * j);
            }
            pk[w] = x;
        }
        uint4 *dst = (uint4 *)((int8_t *)A.q + row * ld + blk * 32);
        dst[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        dst[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
        if constexpr (WT == W_Q4_0) {
            ((uint16_t *)A.d)[row * (ld / 32) + blk] = f2h(d);
        } else {
            ((float *)A.d)[row * (ld / 32) + blk] = d;
            ((float *)A.s)[row * (ld / 32) + blk] = d * (float)qsum;  // quantize_row_q8_1: s = d * sum(q)
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

// ---------------------------------------------------------------------------
// LayerNorm over 16 staged rows (ggml_norm + mul(repeat(w)) + add(repeat(b)),
// reference bert.cpp:891-897/955-961/985-991): one thread per 32-column block,
// double partial sums combined in a fixed order, two-pass mean/variance.
// Optionally first adds bias and residual: v = (bias + acc) + resid.
template <int WT, bool HAS_BIAS, bool HAS_RESID>
__device__ void ln_row_phase(float *stage, int ld, int ncols, double *red, int64_t row0, const float *__restrict__ bias,
                             float *X, const float *__restrict__ lnw, const float *__restrict__ lnb, float eps,
                             const ActPtr &out, int tid, int nthreads) {
    const int nblk = ncols >> 5, ntask = 16 * nblk;
    double *red1 = red, *red2 = red + ntask;
    for (int t = tid; t < ntask; t += nthreads) {
        const int r = t / nblk, b = t - r * nblk;
        float *sp = stage + r * ld + b * 32;
        const float *xr = X + (row0 + r) * (int64_t)ncols + b * 32;
        double s = 0.0;
#pragma unroll 8
        for (int j = 0; j < 32; j++) {
            float v = sp[j];
            if constexpr (HAS_BIAS) v = bias[b * 32 + j] + v;
            if constexpr (HAS_RESID) v = v + xr[j];
            sp[j] = v;
            s += (double)v;
        }
        red1[t] = s;
    }
    __syncthreads();
    for (int t = tid; t < ntask; t += nthreads) {
        const int r = t / nblk, b = t - r * nblk;
        double tot = 0.0;
        for (int k = 0; k < nblk; k++) tot += red1[r * nblk + k];
        const float mean = (float)(tot / ncols);
        float *sp = stage + r * ld + b * 32;
        double s2 = 0.0;
#pragma unroll 8
        for (int j = 0; j < 32; j++) {
            const float v = sp[j] - mean;
            sp[j] = v;
            s2 += (double)(v * v);
        }
        red2[t] = s2;
    }
    __syncthreads();
    for (int t = tid; t < ntask; t += nthreads) {
        const int r = t / nblk, b = t - r * nblk;
        double tot = 0.0;
        for (int k = 0; k < nblk; k++) tot += red2[r * nblk + k];
        const float var = (float)(tot / ncols);
        const float scale = 1.0f / sqrtf(var + eps);
        const float *sp = stage + r * ld + b * 32;
        float y[32];
#pragma unroll
        for (int j = 0; j < 32; j++) {
            float v = sp[j] * scale;
            v = lnw[b * 32 + j] * v;
            y[j] = v + lnb[b * 32 + j];
        }
        float4v *xo = (float4v *)(X + (row0 + r) * (int64_t)ncols + b * 32);
#pragma unroll
        for (int w = 0; w < 8; w++) xo[w] = float4v{y[4 * w], y[4 * w + 1], y[4 * w + 2], y[4 * w + 3]};
        store_act_block<WT>(out, ncols, row0 + r, b, y);
    }
    __syncthreads();
}

// LayerNorm row phase for GEMM slices: task t -> (block b = t / 16, row r = t % 16),
// v = (bias + acc) + x, two-pass double statistics combined in a fixed block order.
template <int WT, int NBLK>
__device__ void ln_row_phase_t(float *stage, int ld, double *red, int64_t row0, const float *__restrict__ bias,
                               float *X, const float *__restrict__ lnw, const float *__restrict__ lnb, float eps,
                               const ActPtr &out, int tid, int nthreads) {
    constexpr int ncols = NBLK * 32, ntask = 16 * NBLK;
    double *red1 = red, *red2 = red + ntask;
    for (int t = tid; t < ntask; t += nthreads) {
        const int b = t >> 4, r = t & 15;
        float *sp = stage + r * ld + 32 * b;
        const float *xr = X + (row0 + r) * (int64_t)ncols + 32 * b;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            float4v v = *(float4v *)(sp + 4 * k);
            const float4v bb = *(const float4v *)(bias + 32 * b + 4 * k);
            const float4v x = *(const float4v *)(xr + 4 * k);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                v[j] = (bb[j] + v[j]) + x[j];
                s += (double)v[j];
            }
            *(float4v *)(sp + 4 * k) = v;
        }
        red1[r * NBLK + b] = s;
    }
    __syncthreads();
    for (int t = tid; t < ntask; t += nthreads) {
        const int b = t >> 4, r = t & 15;
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < NBLK; k++) tot += red1[r * NBLK + k];
        const float mean = (float)(tot / ncols);
        float *sp = stage + r * ld + 32 * b;
        double s2 = 0.0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            float4v v = *(float4v *)(sp + 4 * k);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                v[j] = v[j] - mean;
                s2 += (double)(v[j] * v[j]);
            }
            *(float4v *)(sp + 4 * k) = v;
        }
        red2[r * NBLK + b] = s2;
    }
    __syncthreads();
    for (int t = tid; t < ntask; t += nthreads) {
        const int b = t >> 4, r = t & 15;
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < NBLK; k++) tot += red2[r * NBLK + k];
        const float var = (float)(tot / ncols);
        const float scale = 1.0f / sqrtf(var + eps);
        const float *sp = stage + r * ld + 32 * b;
        float y[32];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const float4v v = *(const float4v *)(sp + 4 * k);
            const float4v w = *(const float4v *)(lnw + 32 * b + 4 * k);
            const float4v bb = *(const float4v *)(lnb + 32 * b + 4 * k);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float z = v[j] * scale;
                z = w[j] * z;
                y[4 * k + j] = z + bb[j];
            }
        }
        float4v *xo = (float4v *)(X + (row0 + r) * (int64_t)ncols + 32 * b);
#pragma unroll
        for (int k = 0; k < 8; k++) xo[k] = float4v{y[4 * k], y[4 * k + 1], y[4 * k + 2], y[4 * k + 3]};
        store_act_block<WT>(out, ncols, row0 + r, b, y);
    }
}

// ---------------------------------------------------------------------------
// Embeddings: x = pos[i] + (type[0] + word[id]) then LayerNorm (bert.cpp:880-898).
__device__ __forceinline__ float table_elem(const void *tab, int type, int64_t row, int E, int e) {
    switch (type) {
        case W_F32: return ((const float *)tab)[row * E + e];
        case W_F16: return h2f(((const uint16_t *)tab)[row * E + e]);
        case W_Q4_0: {
            const uint8_t *blk = (const uint8_t *)tab + (row * (E >> 5) + (e >> 5)) * 18;
            const uint16_t dh = (uint16_t)(blk[0] | (blk[1] << 8));
            const int i = e & 31;
            const uint8_t byte = blk[2 + (i & 15)];
            const int q = i < 16 ? (byte & 15) : (byte >> 4);
            return (float)(q - 8) * h2f(dh);
        }
        default: {
            const uint8_t *blk = (const uint8_t *)tab + (row * (E >> 5) + (e >> 5)) * 20;
            const uint16_t dh = (uint16_t)(blk[0] | (blk[1] << 8)), mh = (uint16_t)(blk[2] | (blk[3] << 8));
            const int i = e & 31;
            const uint8_t byte = blk[4 + (i & 15)];
            const int q = i < 16 ? (byte & 15) : (byte >> 4);
            return fmaf((float)q, h2f(dh), h2f(mh));  // ggml's x*d + m, contracted by gcc -mfma
        }
    }
}

template <int WT>
__global__ __launch_bounds__(256) void embed_ln_kernel(EmbedArgs a) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    const int E = a.E, ld = E + 4, nblk = E >> 5;
    float *stage = (float *)dsm;
    double *red = (double *)(dsm + (size_t)16 * ld * 4);
    int *rinfo = (int *)(red + 2 * 16 * nblk);  // [16][2]: token, position (-1 = padding row)
    const int tid = threadIdx.x;
    const int64_t row0 = (int64_t)blockIdx.x * 16;
    if (tid < 16) {
        const int64_t row = row0 + tid;
        int tok = -1, pos = 0;
        if (row < a.M) {
            int lo = 0, hi = a.n_seqs;  // largest s with offsets[s] <= row
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (a.offsets[mid] <= row) lo = mid; else hi = mid;
            }
            tok = min(max(a.tokens[row], 0), a.n_vocab - 1);  // ids are validated on the host path;
            pos = min((int)(row - a.offsets[lo]), a.n_pos - 1); // clamp keeps device-fed ids in bounds
        }
        rinfo[2 * tid] = tok;
        rinfo[2 * tid + 1] = pos;
    }
    __syncthreads();
    for (int idx = tid; idx < 16 * E; idx += 256) {
        const int r = idx / E, e = idx - r * E;
        const int tok = rinfo[2 * r], pos = rinfo[2 * r + 1];
        float v = 0.f;
        if (tok >= 0) {
            const float w = table_elem(a.word, a.word_t, tok, E, e);
            const float ty = table_elem(a.type, a.type_t, 0, E, e);
            const float p = table_elem(a.pos, a.pos_t, pos, E, e);
            v = p + (ty + w);
        }
        stage[r * ld + e] = v;
    }
    __syncthreads();
    ln_row_phase<WT, false, false>(stage, ld, E, red, row0, nullptr, a.X, a.ln_w, a.ln_b, a.eps, a.Xa, tid, 256);
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
struct AReg {
    uint4 r[4];
    float d, s;
};

template <int WT>
__device__ __forceinline__ void a_load(AReg &ar, const ActPtr &A, int K, int64_t m0, int k0, int item) {
    const int r = item >> 2, s = item & 3;
    const int64_t row = m0 + r;
    const int k = k0 + s * 16;
    if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
        ar.r[0] = *(const uint4 *)((const int8_t *)A.q + row * K + k);
        const int64_t bi = row * (K >> 5) + (k >> 5);
        if constexpr (WT == W_Q4_0) {
            ar.d = h2f(((const uint16_t *)A.d)[bi]);
        } else {
            ar.d = ((const float *)A.d)[bi];
            ar.s = ((const float *)A.s)[bi];
        }
    } else if constexpr (WT == W_F16) {
        const uint4 *p = (const uint4 *)((const uint16_t *)A.q + row * K + k);
        ar.r[0] = p[0];
        ar.r[1] = p[1];
    } else {
        const uint4 *p = (const uint4 *)((const float *)A.q + row * K + k);
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

template <int WT, int BM>
__device__ __forceinline__ void a_store(const AReg &ar, char *buf, int item) {
    const int r = item >> 2, s = item & 3;
    constexpr int A_BYTES = (WT == W_F32) ? BM * LDA_F * 4 : BM * LDA_H * 2;
    if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
        const uint32_t *w = (const uint32_t *)&ar.r[0];
        half8 h0, h1;
        half2v a, b;
        i8x4_to_f16(w[0], a, b);
        h0[0] = a[0]; h0[1] = a[1]; h0[2] = b[0]; h0[3] = b[1];
        i8x4_to_f16(w[1], a, b);
        h0[4] = a[0]; h0[5] = a[1]; h0[6] = b[0]; h0[7] = b[1];
        i8x4_to_f16(w[2], a, b);
        h1[0] = a[0]; h1[1] = a[1]; h1[2] = b[0]; h1[3] = b[1];
        i8x4_to_f16(w[3], a, b);
        h1[4] = a[0]; h1[5] = a[1]; h1[6] = b[0]; h1[7] = b[1];
        half8 *dst = (half8 *)((_Float16 *)buf + r * LDA_H + s * 16);
        dst[0] = h0;
        dst[1] = h1;
        if ((s & 1) == 0) {
            float *sc = (float *)(buf + A_BYTES);  // [dA: 2][BM] then [sA: 2][BM]
            sc[(s >> 1) * BM + r] = ar.d;
            if constexpr (WT == W_Q4_1) sc[2 * BM + (s >> 1) * BM + r] = ar.s;
        }
    } else if constexpr (WT == W_F16) {
        uint4 *dst = (uint4 *)((uint16_t *)buf + r * LDA_H + s * 16);
        dst[0] = ar.r[0];
        dst[1] = ar.r[1];
    } else {
        uint4 *dst = (uint4 *)((float *)buf + r * LDA_F + s * 16);
        dst[0] = ar.r[0];
        dst[1] = ar.r[1];
        dst[2] = ar.r[2];
        dst[3] = ar.r[3];
    }
}

template <int WT> struct WFrag;
template <> struct WFrag<W_Q4_0> { uint32_t q; _Float16 d; };
template <> struct WFrag<W_Q4_1> { uint32_t q; _Float16 d, m; };
template <> struct WFrag<W_F16> { half8 h; };
template <> struct WFrag<W_F32> { float4v f[2]; };

template <int WT>
__device__ __forceinline__ WFrag<WT> w_load(const WPtr &W, int64_t tile) {
    const int lane = threadIdx.x & 63;
    WFrag<WT> f;
    if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
        f.q = ((const uint32_t *)W.q)[tile * 64 + lane];
        f.d = ((const _Float16 *)W.d)[tile * 16 + (lane & 15)];
        if constexpr (WT == W_Q4_1) f.m = ((const _Float16 *)W.m)[tile * 16 + (lane & 15)];
    } else if constexpr (WT == W_F16) {
        f.h = ((const half8 *)W.q)[tile * 64 + lane];
    } else {
        f.f[0] = ((const float4v *)W.q)[(tile * 64 + lane) * 2];
        f.f[1] = ((const float4v *)W.q)[(tile * 64 + lane) * 2 + 1];
    }
    return f;
}

// 8 nibbles -> 8 exact fp16 integers (q-8 for Q4_0, q for Q4_1).  Nibble slot s
// holds fragment element 2s (s<4) or 2(s-4)+1 (s>=4), so (x >> 4j) & 0x000F000F
// yields elements (2j, 2j+1); 0x6400|q is the fp16 value 1024+q.
template <int WT>
__device__ __forceinline__ half8 w_int(uint32_t x) {
    half8 r;
    const _Float16 o = (WT == W_Q4_0) ? (_Float16)1032.f : (_Float16)1024.f;
    const half2v off = {o, o};
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t w = ((x >> (4 * j)) & 0x000F000Fu) | 0x64006400u;
        const half2v h = __builtin_bit_cast(half2v, w) - off;
        r[2 * j] = h[0];
        r[2 * j + 1] = h[1];
    }
    return r;
}

template <int WT, int EPI, int BN, int NW, int BM>
__global__ __launch_bounds__(NW * 64) void gemm_kernel(GemmArgs args, int n_mtiles, int n_ntiles) {
    constexpr int NT = NW * 64;
    constexpr int WN = BN / NW;
    constexpr int NTW = WN / 16;
    constexpr int NP = NTW / 2;  // column pairs per wave
    constexpr int RT = BM / 16;
    constexpr bool QP = (WT == W_Q4_0 || WT == W_Q4_1);
    constexpr bool F32P = (WT == W_F32);
    constexpr int A_BYTES = F32P ? BM * LDA_F * 4 : BM * LDA_H * 2;
    constexpr int A_BUF = A_BYTES + (QP ? 4 * BM * 4 : 0);
    constexpr int EPI_LDS = (EPI == EPI_BIAS_F32) ? 0 : 16 * (BN + 4) * 4 + ((EPI == EPI_LN) ? 2 * 16 * (BN / 32) * 8 : 0);
    constexpr int SMEM = (2 * A_BUF > EPI_LDS) ? 2 * A_BUF : EPI_LDS;
    static_assert(NTW % 2 == 0, "wave tile must hold whole column pairs");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

    // XCD-aware tile order: linear block ids are dealt round-robin over the 8
    // XCDs; remap so that each XCD walks a contiguous range, n fastest, so the
    // N-tiles that share an A panel run on one XCD (bijective for any count).
    const int nwg = n_mtiles * n_ntiles, orig = blockIdx.x;
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int mt = lin / n_ntiles, ntile = lin - mt * n_ntiles;

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int g = lane >> 4, c16 = lane & 15;
    const int64_t m0 = (int64_t)mt * BM;
    const int n0 = ntile * BN;
    const int K = args.K, nkc = K / KC, nkb = K >> 5;
    const int64_t ntile0 = (n0 + wv * WN) >> 4;

    float4v acc[RT][NTW];
#pragma unroll
    for (int i = 0; i < RT; i++)
#pragma unroll
        for (int j = 0; j < NTW; j++) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

    AReg ar;
    const bool stager = tid < BM * (KC / 16);
    if (stager) {
        a_load<WT>(ar, args.A, K, m0, 0, tid);
        a_store<WT, BM>(ar, smem, tid);
    }
    WFrag<WT> wf[F32P ? 1 : 2][NTW], wn[F32P ? 1 : 2][NTW];
    if constexpr (!F32P) {
#pragma unroll
        for (int kb = 0; kb < 2; kb++)
#pragma unroll
            for (int nt = 0; nt < NTW; nt++) wf[kb][nt] = w_load<WT>(args.W, (ntile0 + nt) * nkb + kb);
    }
    __syncthreads();

    const float4v zero4 = {0.f, 0.f, 0.f, 0.f};
    for (int kc = 0; kc < nkc; kc++) {
        const bool more = kc + 1 < nkc;
        if (stager && more) a_load<WT>(ar, args.A, K, m0, (kc + 1) * KC, tid);
        if constexpr (!F32P) {
            if (more) {
#pragma unroll
                for (int kb = 0; kb < 2; kb++)
#pragma unroll
                    for (int nt = 0; nt < NTW; nt++)
                        wn[kb][nt] = w_load<WT>(args.W, (ntile0 + nt) * nkb + (kc + 1) * 2 + kb);
            }
        }
        const char *abuf = smem + (kc & 1) * A_BUF;
#pragma unroll
        for (int kb = 0; kb < 2; kb++) {
            if constexpr (QP) {
                half8 a[RT];
                float4v da[RT], sa[RT];
                const float *sc = (const float *)(abuf + A_BYTES);
#pragma unroll
                for (int rt = 0; rt < RT; rt++) {
                    a[rt] = *(const half8 *)((const _Float16 *)abuf + (rt * 16 + c16) * LDA_H + kb * 32 + 8 * g);
                    da[rt] = *(const float4v *)(sc + kb * BM + rt * 16 + g * 4);
                    if constexpr (WT == W_Q4_1) sa[rt] = *(const float4v *)(sc + 2 * BM + kb * BM + rt * 16 + g * 4);
                }
                half8 b[NTW];
                float dw[NTW], mw[NTW];
#pragma unroll
                for (int nt = 0; nt < NTW; nt++) {
                    b[nt] = w_int<WT>(wf[kb][nt].q);
                    dw[nt] = (float)wf[kb][nt].d;
                    if constexpr (WT == W_Q4_1) mw[nt] = (float)wf[kb][nt].m;
                }
                // software pipeline: MFMA of tile t+1 in flight while tile t's
                // integer sum is folded in (keeps two block sums live, not RT*NTW)
                constexpr int T = RT * NTW;
                float4v blk[2];
                blk[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], zero4, 0, 0, 0);
#pragma unroll
                for (int t = 0; t < T; t++) {
                    if (t + 1 < T)
                        blk[(t + 1) & 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(t + 1) % RT], b[(t + 1) / RT],
                                                                                   zero4, 0, 0, 0);
                    const int rt = t % RT, nt = t / RT;
#pragma unroll
                    for (int i = 0; i < 4; i += 2) {  // packed f32: two rows per instruction
                        const float2v dw2 = {dw[nt], dw[nt]};
                        const float2v sc2 = float2v{da[rt][i], da[rt][i + 1]} * dw2;  // exact: fp16 x fp16
                        float2v a2 = {acc[rt][nt][i], acc[rt][nt][i + 1]};
                        a2 = __builtin_elementwise_fma(sc2, float2v{blk[t & 1][i], blk[t & 1][i + 1]}, a2);
                        if constexpr (WT == W_Q4_1) {
                            const float2v mw2 = {mw[nt], mw[nt]};
                            a2 = __builtin_elementwise_fma(mw2, float2v{sa[rt][i], sa[rt][i + 1]}, a2);
                        }
                        asm volatile("" : "+v"(a2));  // keep the fold here (no sinking past MFMAs)
                        acc[rt][nt][i] = a2[0];
                        acc[rt][nt][i + 1] = a2[1];
                    }
                    __builtin_amdgcn_sched_barrier(0);
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
                        acc[rt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rt], wf[kb][nt].h, acc[rt][nt], 0, 0, 0);
            } else {
#pragma unroll
                for (int nt = 0; nt < NTW; nt++) wf[0][nt] = w_load<WT>(args.W, (ntile0 + nt) * nkb + kc * 2 + kb);
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
            if (stager) a_store<WT, BM>(ar, smem + ((kc + 1) & 1) * A_BUF, tid);
            if constexpr (!F32P) {
#pragma unroll
                for (int kb = 0; kb < 2; kb++)
#pragma unroll
                    for (int nt = 0; nt < NTW; nt++) wf[kb][nt] = wn[kb][nt];
            }
        }
        __syncthreads();
    }

    // ---- epilogue, in registers.  Lane (g, c16), pair p, row-tile rt, i:
    //      row = m0 + rt*16 + 4g + i, columns col0 + {0, 1} with
    //      col0 = n0 + wv*WN + 32p + 2*c16; values acc[rt][2p][i], acc[rt][2p+1][i].
    const int colw = n0 + wv * WN + 2 * c16;
    if constexpr (EPI == EPI_BIAS_F32) {
#pragma unroll
        for (int p = 0; p < NP; p++) {
            const int col = colw + 32 * p;
            const float2v b = *(const float2v *)(args.bias + col);
#pragma unroll
            for (int rt = 0; rt < RT; rt++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int64_t row = m0 + rt * 16 + 4 * g + i;
                    *(float2v *)(args.out_f32 + row * args.N + col) =
                        float2v{b[0] + acc[rt][2 * p][i], b[1] + acc[rt][2 * p + 1][i]};  // b + W.x
                }
        }
    } else {
        // GELU / LayerNorm epilogues through a 16-row LDS slice: one thread per
        // (32-column block, row).  Row stride BN + 4 floats is odd in 16-byte
        // slots, so the 16 lanes reading one block of 16 rows hit 16 slots.
        constexpr int LD = BN + 4, NBLK = BN / 32;
        float *stage = (float *)smem;
        double *red = (double *)(smem + 16 * LD * 4);  // [2][16][NBLK]
#pragma unroll
        for (int rt = 0; rt < RT; rt++) {
            __syncthreads();
#pragma unroll
            for (int p = 0; p < NP; p++)
#pragma unroll
                for (int i = 0; i < 4; i++)
                    *(float2v *)(stage + (4 * g + i) * LD + wv * WN + 32 * p + 2 * c16) =
                        float2v{acc[rt][2 * p][i], acc[rt][2 * p + 1][i]};
            __syncthreads();
            const int64_t row0 = m0 + rt * 16;
            if constexpr (EPI == EPI_GELU_ACT) {
                for (int t = tid; t < 16 * NBLK; t += NT) {
                    const int b = t >> 4, r = t & 15, col0 = n0 + 32 * b;
                    const float *sp = stage + r * LD + 32 * b;
                    float y[32];
                    uint16_t hv[32];
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        const float4v v = *(const float4v *)(sp + 4 * k);
                        const float4v bb = *(const float4v *)(args.bias + col0 + 4 * k);
#pragma unroll
                        for (int j = 0; j < 4; j++) hv[4 * k + j] = args.gelu_tab[f2h(bb[j] + v[j])];  // gelu(b + W.x)
                    }
#pragma unroll
                    for (int j = 0; j < 32; j++) y[j] = h2f(hv[j]);
                    store_act_block<WT>(args.out_act, args.N, row0 + r, col0 >> 5, y);
                }
            } else {
                ln_row_phase_t<WT, NBLK>(stage, LD, red, row0, args.bias, args.X, args.ln_w, args.ln_b, args.eps,
                                         args.out_act, tid, NT);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Attention for sentences of n <= 128 tokens: one workgroup per (head,
// sentence), wave w owns queries 32w..32w+31 (reference bert.cpp:928-942).
//
// f32 accuracy on fp16 MFMA: every operand x is split exactly into
// hi = fp16(x), lo = fp16(x - hi) and a product is hi*hi + hi*lo + lo*hi
// (three v_mfma_f32_32x32x16_f16; the dropped lo*lo term is 2^-22 relative),
// so S and the context carry f32-level error like ggml's f32 mul_mat.
// Swapped QK^T: S^T = K . Q^T puts one query per lane column, so ggml's
// soft_max (max, p = exp_tab[fp16(s - max)], double sum, p *= (float)(1/sum))
// runs in registers (one cross-half shuffle), and the normalised P^T
// accumulator is directly the B operand of ctx^T = V^T . P^T (no LDS round trip
// for P).  K (row-major) and V^T are staged once per workgroup in LDS as hi/lo
// planes; the context is quantised to the O-projection's activation format in
// registers.
template <int WT, int D>
__global__ __launch_bounds__(256) void attention_short_kernel(AttnArgs a) {
    constexpr int NK = 128;      // keys staged (n <= 128)
    constexpr int KST = D + 8;   // K row stride, halves: conflict-free ds_read_b128 (80 / 144 B)
    constexpr int VST = NK + 4;  // V^T row stride, halves: 66 dwords, conflict-free ds_read_b64
    __shared__ __attribute__((aligned(16))) _Float16 Kh[NK * KST], Kl[NK * KST], Vh[D * VST], Vl[D * VST];
    const int h = blockIdx.x, s = blockIdx.y;
    const int beg = a.offsets[s], n = a.offsets[s + 1] - beg;
    if (n > NK) return;  // attention_long_kernel handles these sentences
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
    const int E = a.E, E3 = 3 * E;
    const float *base = a.qkv + (int64_t)beg * E3;

    for (int idx = tid; idx < NK * (D / 4); idx += 256) {
        const int key = idx / (D / 4), d0 = (idx - key * (D / 4)) * 4;
        float4v k = {0.f, 0.f, 0.f, 0.f}, v = {0.f, 0.f, 0.f, 0.f};
        if (key < n) {
            k = *(const float4v *)(base + (int64_t)key * E3 + E + h * D + d0);
            v = *(const float4v *)(base + (int64_t)key * E3 + 2 * E + h * D + d0);
        }
        half4v khi, klo;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            khi[j] = (_Float16)k[j];
            klo[j] = (_Float16)(k[j] - (float)khi[j]);
            const _Float16 vh = (_Float16)v[j];
            Vh[(d0 + j) * VST + key] = vh;
            Vl[(d0 + j) * VST + key] = (_Float16)(v[j] - (float)vh);
        }
        *(half4v *)&Kh[key * KST + d0] = khi;
        *(half4v *)&Kl[key * KST + d0] = klo;
    }
    __syncthreads();
    const int q0 = wv * 32;
    if (q0 >= n) return;

    // Q^T fragments (B operand): lane (r, hh) holds Q[q0 + r][16 ks + 8 hh + j]
    half8 qh[D / 16], ql[D / 16];
    {
        const int qr = min(q0 + r, n - 1);
        const float *qp = base + (int64_t)qr * E3 + h * D + 8 * hh;
#pragma unroll
        for (int ks = 0; ks < D / 16; ks++) {
            const float4v x0 = *(const float4v *)(qp + 16 * ks), x1 = *(const float4v *)(qp + 16 * ks + 4);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                qh[ks][j] = (_Float16)x0[j];
                ql[ks][j] = (_Float16)(x0[j] - (float)qh[ks][j]);
                qh[ks][4 + j] = (_Float16)x1[j];
                ql[ks][4 + j] = (_Float16)(x1[j] - (float)qh[ks][4 + j]);
            }
        }
    }
    const int nkt = (n + 31) >> 5;
    float16v S[4];
    const float16v zero16 = {};
#pragma unroll
    for (int kt = 0; kt < 4; kt++) {
        S[kt] = zero16;
        if (kt < nkt) {
#pragma unroll
            for (int ks = 0; ks < D / 16; ks++) {
                const int off = (kt * 32 + r) * KST + 16 * ks + 8 * hh;
                const half8 kh = *(const half8 *)&Kh[off], kl = *(const half8 *)&Kl[off];
                S[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kl, qh[ks], S[kt], 0, 0, 0);
                S[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kh, ql[ks], S[kt], 0, 0, 0);
                S[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kh, qh[ks], S[kt], 0, 0, 0);
            }
        }
    }
    // soft_max over keys for query q0 + r: this lane holds keys
    // 32 kt + (j & 3) + 8 (j >> 2) + 4 hh, the partner lane (r, 1 - hh) the rest
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; kt++)
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int key = kt * 32 + (j & 3) + 8 * (j >> 2) + 4 * hh;
            const float sv = key < n ? S[kt][j] * a.scale : -INFINITY;  // ggml_scale after K.Q
            S[kt][j] = sv;
            mx = fmaxf(mx, sv);
        }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    double sum = 0.0;
#pragma unroll
    for (int kt = 0; kt < 4; kt++)
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const float p = h2f(a.exp_tab[f2h(S[kt][j] - mx)]);  // -inf -> table -> 0
            S[kt][j] = p;
            sum += (double)p;
        }
    sum += __shfl_xor(sum, 32);
    const float rs = (float)(1.0 / sum);
    // ctx^T = V^T . P^T.  k-step ks of key tile kt: B element j of lane half hh
    // is key 32 kt + 16 ks + 8 (j >> 2) + 4 hh + (j & 3) = register 8 ks + j.
    float16v o[D / 32];
#pragma unroll
    for (int dt = 0; dt < D / 32; dt++) o[dt] = zero16;
#pragma unroll
    for (int kt = 0; kt < 4; kt++) {
        if (kt < nkt) {
#pragma unroll
            for (int ks = 0; ks < 2; ks++) {
                half8 ph, pl;
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const float p = S[kt][8 * ks + j] * rs;  // ggml: p *= (float)(1/sum) before V.P
                    ph[j] = (_Float16)p;
                    pl[j] = (_Float16)(p - (float)ph[j]);
                }
                const int key = kt * 32 + 16 * ks + 4 * hh;
#pragma unroll
                for (int dt = 0; dt < D / 32; dt++) {
                    const int off = (dt * 32 + r) * VST + key;
                    const half4v h0 = *(const half4v *)&Vh[off], h1 = *(const half4v *)&Vh[off + 8];
                    const half4v l0 = *(const half4v *)&Vl[off], l1 = *(const half4v *)&Vl[off + 8];
                    const half8 vh = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
                    const half8 vl = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vl, ph, o[dt], 0, 0, 0);
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, pl, o[dt], 0, 0, 0);
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, ph, o[dt], 0, 0, 0);
                }
            }
        }
    }
    // lane (r, hh) holds ctx[q0 + r][h D + 32 dt + (j & 3) + 8 (j >> 2) + 4 hh]:
    // one 32-value quant block per (query, dt), split over the lane pair (r, hh).
    const int q = q0 + r;
    const int64_t row = beg + q;
#pragma unroll
    for (int dt = 0; dt < D / 32; dt++) {
        const int col0 = h * D + dt * 32;
        if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
            float amax = 0.f;
#pragma unroll
            for (int j = 0; j < 16; j++) amax = fmaxf(amax, fabsf(o[dt][j]));
            amax = fmaxf(amax, __shfl_xor(amax, 32));
            const float d = amax / 127.f;
            const float id = amax != 0.f ? 127.f / amax : 0.f;
            int qs = 0;
            uint32_t pk[4];
#pragma unroll
            for (int m = 0; m < 4; m++) {
                uint32_t x = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int qv = (int)rintf(o[dt][4 * m + j] * id);
                    qs += qv;
                    x |= ((uint32_t)(qv & 0xff)) << (8 * j);
                }
                pk[m] = x;
            }
            qs += __shfl_xor(qs, 32);
            if (q < n) {
#pragma unroll
                for (int m = 0; m < 4; m++) *(uint32_t *)((int8_t *)a.ctx.q + row * E + col0 + 8 * m + 4 * hh) = pk[m];
                if (hh == 0) {
                    const int64_t bi = row * (E >> 5) + (col0 >> 5);
                    if constexpr (WT == W_Q4_0) {
                        ((uint16_t *)a.ctx.d)[bi] = f2h(d);
                    } else {
                        ((float *)a.ctx.d)[bi] = d;
                        ((float *)a.ctx.s)[bi] = d * (float)qs;
                    }
                }
            }
        } else if (q < n) {
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

// ---------------------------------------------------------------------------
// Attention for sentences of n > 128 tokens, one (sentence, head, 64-query block)
// per workgroup: 4 waves x 16 queries.
// S = (K.Q) * scale on f32 MFMA (exact f32 products, as ggml's f32 mul_mat),
// rows kept in LDS; ggml_soft_max: max, p = exp_tab[fp16(s - max)], double
// sum, p *= (float)(1/sum); ctx = V^T.P on f32 MFMA; quantised to the O-proj's
// activation format in the epilogue.
template <int WT, int D>
__global__ __launch_bounds__(256) void attention_long_kernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    const int s = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * ATT_QB;
    const int beg = a.offsets[s], n = a.offsets[s + 1] - beg;
    if (q0 >= n || n <= 128) return;  // n <= 128: attention_short_kernel
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane >> 4, c16 = lane & 15;
    const int E = a.E, E3 = 3 * E;
    const int nk16 = (n + 15) & ~15;
    const int LDS_S = ((nk16 + 55) / 64) * 64 + 8;  // == 8 (mod 64) dwords: conflict-free float4 row reads
    float *S = (float *)dsm + wv * 16 * LDS_S;
    const float *base = a.qkv + (int64_t)beg * E3;
    const int qw0 = q0 + wv * 16;  // this wave's first query

    float4v qf[D / 16];
    {
        const int qr = min(qw0 + c16, n - 1);
#pragma unroll
        for (int c = 0; c < D / 16; c++) qf[c] = *(const float4v *)(base + (int64_t)qr * E3 + h * D + 16 * c + 4 * g);
    }
    for (int key0 = 0; key0 < n; key0 += 16) {
        const int kr = min(key0 + c16, n - 1);
        float4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < D / 16; c++) {
            const float4v kf = *(const float4v *)(base + (int64_t)kr * E3 + E + h * D + 16 * c + 4 * g);
#pragma unroll
            for (int j = 0; j < 4; j++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[c][j], kf[j], acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) S[(g * 4 + i) * LDS_S + key0 + c16] = acc[i] * a.scale;
    }
    __syncthreads();
    {
        const int rr = lane >> 2, part = lane & 3;
        float *row = S + rr * LDS_S;
        float mx = -INFINITY;
        for (int k = part; k < n; k += 4) mx = fmaxf(mx, row[k]);
        mx = fmaxf(mx, __shfl_xor(mx, 1));
        mx = fmaxf(mx, __shfl_xor(mx, 2));
        double sum = 0.0;
        for (int k = part; k < n; k += 4) {
            const float p = h2f(a.exp_tab[f2h(row[k] - mx)]);
            row[k] = p;
            sum += (double)p;
        }
        sum += __shfl_xor(sum, 1);
        sum += __shfl_xor(sum, 2);
        const float r = (float)(1.0 / sum);
        for (int k = part; k < n; k += 4) row[k] = row[k] * r;
        for (int k = n + part; k < nk16; k += 4) row[k] = 0.f;
    }
    __syncthreads();
    float4v o[D / 16];
#pragma unroll
    for (int dt = 0; dt < D / 16; dt++) o[dt] = float4v{0.f, 0.f, 0.f, 0.f};
    const float *vbase = base + 2 * E + h * D;
    for (int kc = 0; kc < nk16; kc += 16) {
        const float4v pf = *(const float4v *)(S + c16 * LDS_S + kc + 4 * g);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int vr = min(kc + 4 * g + j, n - 1);
#pragma unroll
            for (int dt = 0; dt < D / 16; dt++) {
                const float vv = vbase[(int64_t)vr * E3 + dt * 16 + c16];
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pf[j], vv, o[dt], 0, 0, 0);
            }
        }
    }
    __syncthreads();
    float *T = S;  // reuse: [16][D + 4]
#pragma unroll
    for (int dt = 0; dt < D / 16; dt++)
#pragma unroll
        for (int i = 0; i < 4; i++) T[(g * 4 + i) * (D + 4) + dt * 16 + c16] = o[dt][i];
    __syncthreads();
    if (lane < 16 * (D / 32)) {
        const int rr = lane / (D / 32), blk = lane % (D / 32);
        const int q = qw0 + rr;
        if (q < n) {
            float v[32];
#pragma unroll
            for (int j = 0; j < 32; j++) v[j] = T[rr * (D + 4) + blk * 32 + j];
            store_act_block<WT>(a.ctx, E, beg + q, h * (D / 32) + blk, v);
        }
    }
}

// ---------------------------------------------------------------------------
// Mean pool + L2 normalise for one sentence (bert.cpp:995-1006):
// m[e] = sum_t x[t][e] * (1.0f/N); s = sum m^2 (double); len = sqrtf(s);
// out = m * (1.0f/len).
__global__ __launch_bounds__(256) void pool_l2_kernel(const float *X, const int32_t *offsets, int E, float *out) {
    __shared__ float m[1024];
    __shared__ double red[4];
    const int s = blockIdx.x, tid = threadIdx.x;
    const int beg = offsets[s], n = offsets[s + 1] - beg;
    const float invN = 1.0f / n;
    double ss = 0.0;
    for (int e = tid; e < E; e += 256) {
        float acc = 0.f;
        for (int t = 0; t < n; t++) acc = fmaf(X[(int64_t)(beg + t) * E + e], invN, acc);
        m[e] = acc;
        ss += (double)(acc * acc);
    }
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    const double tot = red[0] + red[1] + red[2] + red[3];
    const float len = sqrtf((float)tot);
    const float r = 1.0f / len;
    for (int e = tid; e < E; e += 256) out[(int64_t)s * E + e] = m[e] * r;
}

// ---------------------------------------------------------------------------
// launchers
template <int WT>
static hipError_t embed_t(const EmbedArgs &a, int Mpad, hipStream_t s) {
    const size_t smem = (size_t)16 * (a.E + 4) * 4 + (size_t)2 * 16 * (a.E / 32) * 8 + 16 * 2 * 4;
    static bool attr_set = false;
    if (!attr_set) {
        hipFuncSetAttribute((const void *)embed_ln_kernel<WT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(embed_ln_kernel<WT>, dim3(Mpad / 16), dim3(256), smem, s, a);
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

template <int WT, int EPI, int BN, int NW, int BM>
static hipError_t gemm_t(const GemmArgs &a, int Mpad, hipStream_t s) {
    const int mt = Mpad / BM, nt = a.N / BN;
    hipLaunchKernelGGL((gemm_kernel<WT, EPI, BN, NW, BM>), dim3(mt * nt), dim3(NW * 64), 0, s, a, mt, nt);
    return hipGetLastError();
}

// Wave tiles hold 4 n-tiles (64 columns) for QKV / FFN-up (64-row tiles); the
// LayerNorm GEMMs own whole rows (BN = E) and use 32-row tiles to keep the
// row-statistics epilogue inside the register budget.
template <int WT>
static hipError_t gemm_w(int epi, const GemmArgs &a, int Mpad, hipStream_t s) {
    if (epi == EPI_BIAS_F32) return gemm_t<WT, EPI_BIAS_F32, 384, 6, 64>(a, Mpad, s);
    if (epi == EPI_GELU_ACT) return gemm_t<WT, EPI_GELU_ACT, 256, 4, 64>(a, Mpad, s);
    switch (a.N) {
        case 384: return gemm_t<WT, EPI_LN, 384, 6, 64>(a, Mpad, s);
        case 768: return gemm_t<WT, EPI_LN, 768, 12, 64>(a, Mpad, s);
        case 1024: return gemm_t<WT, EPI_LN, 1024, 8, 32>(a, Mpad, s);
    }
    return hipErrorInvalidValue;
}

bool gemm_shape_supported(int epi, int N, int K) {
    if (K % KC) return false;
    if (epi == EPI_BIAS_F32) return N % 384 == 0;
    if (epi == EPI_GELU_ACT) return N % 256 == 0;
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
    hipLaunchKernelGGL((attention_short_kernel<WT, D>), dim3(a.H, n_seqs), dim3(256), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || max_len <= 128) return e;
    const int nk16 = (max_len + 15) & ~15;
    const int lds_s = ((nk16 + 55) / 64) * 64 + 8;
    const size_t smem = (size_t)4 * 16 * lds_s * 4;
    static bool attr_set = false;
    if (!attr_set) {
        hipFuncSetAttribute((const void *)attention_long_kernel<WT, D>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL((attention_long_kernel<WT, D>), dim3((max_len + ATT_QB - 1) / ATT_QB, a.H, n_seqs), dim3(256),
                       smem, s, a);
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

hipError_t launch_pool(const float *X, const int32_t *offsets, int n_seqs, int E, float *out, hipStream_t s) {
    if (E > 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pool_l2_kernel, dim3(n_seqs), dim3(256), 0, s, X, offsets, E, out);
    return hipGetLastError();
}

}  // namespace bertamd
