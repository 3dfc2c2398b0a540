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

constexpr int BM = GEMM_BM;  // 64 rows per GEMM workgroup
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
#pragma unroll
        for (int w = 0; w < 8; w++) {
            uint32_t x = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int q = (int)rintf(v[4 * w + j] * id);
                x |= ((uint32_t)(q & 0xff)) << (8 * j);
            }
            pk[w] = x;
        }
        uint4 *dst = (uint4 *)((int8_t *)A.q + row * ld + blk * 32);
        dst[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        dst[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
        if constexpr (WT == W_Q4_0)
            ((uint16_t *)A.d)[row * (ld / 32) + blk] = f2h(d);
        else
            ((float *)A.d)[row * (ld / 32) + blk] = d;
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
// BM rows x WN columns).  The A chunk (64 rows x 64 k) is dequantised once into
// an fp16 (f32 for F32 weights) LDS tile, double-buffered, register-prefetched.
// W fragments come straight from the repacked weight stream (L2-resident) into
// registers and are dequantised there (Q4: magic-number nibble -> fp16, packed
// f16 math).  MFMA: v_mfma_f32_16x16x32_f16, or v_mfma_f32_16x16x4_f32 (exact
// f32 products) for F32 weights.
struct AReg {
    uint4 r[4];
    float d;
};

template <int WT>
__device__ __forceinline__ void a_load(AReg &ar, const ActPtr &A, int K, int64_t m0, int k0, int item) {
    const int r = item >> 2, s = item & 3;
    const int64_t row = m0 + r;
    const int k = k0 + s * 16;
    if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
        ar.r[0] = *(const uint4 *)((const int8_t *)A.q + row * K + k);
        if constexpr (WT == W_Q4_0)
            ar.d = h2f(((const uint16_t *)A.d)[row * (K >> 5) + (k >> 5)]);
        else
            ar.d = ((const float *)A.d)[row * (K >> 5) + (k >> 5)];
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

template <int WT>
__device__ __forceinline__ void a_store(const AReg &ar, char *buf, int item) {
    const int r = item >> 2, s = item & 3;
    if constexpr (WT == W_Q4_0 || WT == W_Q4_1) {
        const int8_t *b = (const int8_t *)&ar.r[0];
        half8 h0, h1;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            h0[j] = (_Float16)((float)b[j] * ar.d);  // exact f32 product, one fp16 rounding
            h1[j] = (_Float16)((float)b[8 + j] * ar.d);
        }
        half8 *dst = (half8 *)((_Float16 *)buf + r * LDA_H + s * 16);
        dst[0] = h0;
        dst[1] = h1;
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

// 8 nibbles -> 8 fp16 weights.  Nibble slot s holds fragment element 2s (s<4)
// or 2(s-4)+1 (s>=4), so (x >> 4j) & 0x000F000F yields elements (2j, 2j+1).
// 0x6400|q is the fp16 value 1024+q; subtracting 1032 gives q-8 exactly.
template <int WT>
__device__ __forceinline__ half8 w_dequant(const WFrag<WT> &f) {
    if constexpr (WT == W_F16) {
        return f.h;
    } else {
        half8 r;
        const half2v dd = {f.d, f.d};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t w = ((f.q >> (4 * j)) & 0x000F000Fu) | 0x64006400u;
            half2v h = __builtin_bit_cast(half2v, w);
            if constexpr (WT == W_Q4_0) {
                const half2v off = {(_Float16)1032.f, (_Float16)1032.f};
                h = (h - off) * dd;  // fp16((q-8)*d): product of exact operands, one rounding
            } else {
                const half2v off = {(_Float16)1024.f, (_Float16)1024.f};
                const half2v mm = {f.m, f.m};
                h = __builtin_elementwise_fma(h - off, dd, mm);  // fp16(q*d + m), one rounding
            }
            r[2 * j] = h[0];
            r[2 * j + 1] = h[1];
        }
        return r;
    }
}

template <int WT, int EPI, int BN, int NW>
__global__ __launch_bounds__(NW * 64) void gemm_kernel(GemmArgs args) {
    constexpr int NT = NW * 64;
    constexpr int WN = BN / NW;
    constexpr int NTW = WN / 16;
    constexpr int RT = BM / 16;
    constexpr bool F32P = (WT == W_F32);
    constexpr int A_BUF = F32P ? BM * LDA_F * 4 : BM * LDA_H * 2;
    constexpr int LDS_ST = BN + 4;
    constexpr int STAGE = 16 * LDS_ST * 4;
    constexpr int RED = (EPI == EPI_LN) ? 2 * 16 * (BN / 32) * 8 : 0;
    constexpr int SMEM = (2 * A_BUF > STAGE + RED) ? 2 * A_BUF : STAGE + RED;
    static_assert(WN % 16 == 0, "wave tile");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int g = lane >> 4, c16 = lane & 15;
    const int64_t m0 = (int64_t)blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
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
        a_store<WT>(ar, smem, tid);
    }
    __syncthreads();

    for (int kc = 0; kc < nkc; kc++) {
        const bool more = kc + 1 < nkc;
        if (stager && more) a_load<WT>(ar, args.A, K, m0, (kc + 1) * KC, tid);
        // Q4/F16 fragments are small: fetch both k-blocks up front; F32 ones per k-block.
        WFrag<WT> wf[F32P ? 1 : 2][NTW];
        if constexpr (!F32P) {
#pragma unroll
            for (int kb = 0; kb < 2; kb++)
#pragma unroll
                for (int nt = 0; nt < NTW; nt++) wf[kb][nt] = w_load<WT>(args.W, (ntile0 + nt) * nkb + kc * 2 + kb);
        }
        const char *abuf = smem + (kc & 1) * A_BUF;
#pragma unroll
        for (int kb = 0; kb < 2; kb++) {
            if constexpr (F32P) {
#pragma unroll
                for (int nt = 0; nt < NTW; nt++) wf[0][nt] = w_load<WT>(args.W, (ntile0 + nt) * nkb + kc * 2 + kb);
            }
            if constexpr (!F32P) {
                half8 a[RT];
#pragma unroll
                for (int rt = 0; rt < RT; rt++)
                    a[rt] = *(const half8 *)((const _Float16 *)abuf + (rt * 16 + c16) * LDA_H + kb * 32 + 8 * g);
#pragma unroll
                for (int nt = 0; nt < NTW; nt++) {
                    const half8 b = w_dequant<WT>(wf[kb][nt]);
#pragma unroll
                    for (int rt = 0; rt < RT; rt++)
                        acc[rt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rt], b, acc[rt][nt], 0, 0, 0);
                }
            } else {
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
        if (stager && more) a_store<WT>(ar, smem + ((kc + 1) & 1) * A_BUF, tid);
        __syncthreads();
    }

    // ---- epilogue: one 16-row slice at a time through LDS ----
    float *stage = (float *)smem;
    double *red = (double *)(smem + STAGE);
    constexpr int NBLK = BN / 32;
#pragma unroll
    for (int rt = 0; rt < RT; rt++) {
#pragma unroll
        for (int nt = 0; nt < NTW; nt++)
#pragma unroll
            for (int i = 0; i < 4; i++) stage[(g * 4 + i) * LDS_ST + wv * WN + nt * 16 + c16] = acc[rt][nt][i];
        __syncthreads();
        const int64_t row0 = m0 + rt * 16;
        if constexpr (EPI == EPI_LN) {
            ln_row_phase<WT, true, true>(stage, LDS_ST, BN, red, row0, args.bias, args.X, args.ln_w, args.ln_b,
                                         args.eps, args.out_act, tid, NT);
        } else {
            for (int t = tid; t < 16 * NBLK; t += NT) {
                const int r = t / NBLK, b = t - r * NBLK;
                const float *sp = stage + r * LDS_ST + b * 32;
                const int col0 = n0 + b * 32;
                const int64_t row = row0 + r;
                if constexpr (EPI == EPI_BIAS_F32) {
                    float4v *op = (float4v *)(args.out_f32 + row * args.N + col0);
                    const float4v *bp = (const float4v *)(args.bias + col0);
#pragma unroll
                    for (int w = 0; w < 8; w++) op[w] = bp[w] + *(const float4v *)(sp + 4 * w);  // b + W.x
                } else {
                    float y[32];
#pragma unroll
                    for (int j = 0; j < 32; j++) {
                        const float v = args.bias[col0 + j] + sp[j];
                        y[j] = h2f(args.gelu_tab[f2h(v)]);  // ggml_vec_gelu_f32 via fp16 table
                    }
                    store_act_block<WT>(args.out_act, args.N, row, col0 >> 5, y);
                }
            }
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------
// Attention for one (sentence, head, 64-query block): 4 waves x 16 queries.
// S = (K.Q) * scale on f32 MFMA (exact f32 products, as ggml's f32 mul_mat),
// rows kept in LDS; ggml_soft_max: max, p = exp_tab[fp16(s - max)], double
// sum, p *= (float)(1/sum); ctx = V^T.P on f32 MFMA; quantised to the O-proj's
// activation format in the epilogue.
template <int WT, int D>
__global__ __launch_bounds__(256) void attention_kernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    const int s = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * ATT_QB;
    const int beg = a.offsets[s], n = a.offsets[s + 1] - beg;
    if (q0 >= n) return;
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

template <int WT, int EPI, int BN, int NW>
static hipError_t gemm_t(const GemmArgs &a, int Mpad, hipStream_t s) {
    hipLaunchKernelGGL((gemm_kernel<WT, EPI, BN, NW>), dim3(Mpad / BM, a.N / BN), dim3(NW * 64), 0, s, a);
    return hipGetLastError();
}

template <int WT>
static hipError_t gemm_w(int epi, const GemmArgs &a, int Mpad, hipStream_t s) {
    if (epi == EPI_BIAS_F32) return gemm_t<WT, EPI_BIAS_F32, 384, 4>(a, Mpad, s);
    if (epi == EPI_GELU_ACT) return gemm_t<WT, EPI_GELU_ACT, 256, 4>(a, Mpad, s);
    switch (a.N) {
        case 384: return gemm_t<WT, EPI_LN, 384, 4>(a, Mpad, s);
        case 768: return gemm_t<WT, EPI_LN, 768, 8>(a, Mpad, s);
        case 1024: return gemm_t<WT, EPI_LN, 1024, 8>(a, Mpad, s);
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
    if (!gemm_shape_supported(epi, a.N, a.K) || Mpad % BM) return hipErrorInvalidValue;
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
    const int nk16 = (max_len + 15) & ~15;
    const int lds_s = ((nk16 + 55) / 64) * 64 + 8;
    const size_t smem = (size_t)4 * 16 * lds_s * 4;
    static bool attr_set = false;
    if (!attr_set) {
        hipFuncSetAttribute((const void *)attention_kernel<WT, D>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL((attention_kernel<WT, D>), dim3((max_len + ATT_QB - 1) / ATT_QB, a.H, n_seqs), dim3(256), smem, s, a);
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
