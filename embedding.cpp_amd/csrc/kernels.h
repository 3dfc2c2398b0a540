// kernels.h — launch interface between the host runtime and the HIP kernels.
//
// One fixed pipeline replaces the reference's per-sentence ggml graph
// (reference bert.cpp:845-1012 built, :1080 computed, once per sentence):
//
//   embed_ln  : get_rows x3 + add + add + norm/mul/add   (bert.cpp:880-898)
//   per layer:
//     gemm<QKV>   : Q|K|V = b + W.x for all three heads-blocks  (:905-926)
//     attention   : K.Q, scale, soft_max, V^T.P, permute/cpy   (:928-942)
//     gemm<LN>    : LN(b_o + W_o.ctx + x)                       (:944-962)
//     gemm<GELU>  : gelu(b_i + W_i.h)                           (:965-971)
//     gemm<LN>    : LN(h + b_o2 + W_o2.u)                       (:973-992)
//   pool_l2   : mean pool as matvec, sum of squares, sqrt, 1/len, scale (:995-1006)
//
// Sentences of different lengths are packed row-wise ("ragged batch"): rows
// [offsets[s], offsets[s+1]) belong to sentence s; attention never mixes
// sentences, so per-sentence semantics equal the reference's one-at-a-time loop.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bertamd {

// weight type of the 2-D matrices; the activation format feeding a GEMM
// follows it exactly like ggml's vec_dot_type:
//   W_F32 -> f32, W_F16 -> fp16 (RNE), W_Q4_0 -> Q8_0 (int8 + fp16 d),
//   W_Q4_1 -> Q8_1 (int8 + f32 d)
enum WType : int { W_F32 = 0, W_F16 = 1, W_Q4_0 = 2, W_Q4_1 = 3 };
// gemm_i8.hip only: Q4_1 with its per-block scale products d_w * d_a and
// m_w * s_a on the bf16 MFMA as exact partial products (i8_core.h i8_aparts),
// instead of the f32 MFMA; the same weights and activations as W_Q4_1
constexpr int W_Q4_1B = 4;
__host__ __device__ constexpr bool wt_q41(int wt) { return wt == W_Q4_1 || wt == W_Q4_1B; }

struct ActPtr {
    void *q = nullptr;  // int8 [M][K] | fp16 [M][K] | f32 [M][K]
    void *d = nullptr;  // per-32-block scale [M][K/32]: fp16 (Q8_0) | f32 (Q8_1)
};

// Weights repacked at load time into MFMA fragment order:
//   per (16-row n-tile, 32-wide k-block) one 64-lane fragment; lane l holds
//   row (l & 15), k = 8(l >> 4) .. +7.  Output columns are interleaved in pairs
//   of n-tiles: repacked tile 2p+t, lane column c holds weight row 32p + 2c + t,
//   so after the MFMA each lane owns two ADJACENT output columns (vectorised
//   epilogue stores, in-register Q8 blocks).
//   Q4_x: q = fp16 [N/16][K/32][2][64][8]: the dequantised weight w = d*(q-8)
//         (Q4_0) or d*q + m (Q4_1), times 2^S, split as hi = fp16(w),
//         lo = fp16(w - hi).  For Q4_0 the split is exact (w has <= 15
//         significant bits), so an fp16 MFMA over integer Q8 activations
//         returns d_w * sum(q_a * q_w) exactly in each product; `unscale` = 2^-S.
//   F16 : q = fp16 [N/16][K/32][64][8]
//   F32 : q = f32  [N/16][K/32][64][8]
struct WPtr {
    const void *q = nullptr;
    float unscale = 1.f;
};

// Q4_0 / Q4_1 weights for the int8-MFMA GEMMs (gemm_i8.hip), repacked at load
// (runtime.cpp repack_i8) per 32-row f-tile ft and 32-wide k block b:
//   q: int8 [N/32][K/32][64][16]: lane (m = l & 31, h = l >> 5) byte j holds
//      q - 8 (Q4_0) or q (Q4_1) of weight row 32 ft + perm(m), k = 32 b + 16 h + j,
//      perm(m) = 16 ((m >> 2) & 1) + 4 (m >> 3) + (m & 3) (so that a lane of the
//      32x32 MFMA result holds 16 consecutive output features)
//   d: f32 [N/32][K/128][32][4]: d_w of row 32 ft + perm(m), blocks 4g .. 4g + 3
//   m: Q4_1's m_w, same layout (null for Q4_0)
//   dh: Q4_0: the fp16 d_w themselves, fp16 [N/32][K/128][32][4] (the f16-MFMA scale operand)
struct I8W {
    const int8_t *q = nullptr;
    const float *d = nullptr;
    const float *m = nullptr;
    const uint16_t *dh = nullptr;
};

enum Epi : int {
    EPI_QKV = 0,       // y = b + W.x split hi/lo for attention (Q|K row-major, V transposed)
    EPI_GELU_ACT = 1,  // gelu(b + W.x) in the next matmul's activation format
    EPI_LN = 2,        // LN((b + W.x) + X) -> X and activation format (the workgroup owns whole rows)
    EPI_RESID = 3,     // (b + W.x) + X -> X; LayerNorm then runs in launch_ln (rows too wide for one tile)
    EPI_NONE = 4       // main-loop probe (tools/gemm_bench): nothing stored
};

// Piecewise view of a 65536-entry fp16 -> fp16 table (ggml's GELU / exp
// tables, built on the host with glibc exactly as ggml_init builds them) whose
// non-trivial part fits LDS.  Entries for h in [0, pos_n) and
// [0x8000, 0x8000 + neg_n) are stored compactly: compact[h] and
// compact[pos_n + (h & 0x7fff)].  Beyond them the host has verified that the
// table is h itself (pos_identity) or the constant neg_const; every other
// pattern (inf / NaN, non-identity positives) reads `full` in global memory.
constexpr int HALF_TABLE_LDS = 36864;  // max compact GELU entries (72 KiB of LDS)
constexpr int EXP_TABLE_LDS = 20480;   // max compact exp entries (40 KiB of LDS)
constexpr int GELU_FLAT_LDS = 50480;  // Q4 FFN-up GEMM: GELU entries [0, 0x8000 + neg_n] (98.6 KiB of LDS)
struct HalfTable {
    const uint16_t *full = nullptr;
    const uint16_t *compact = nullptr;  // n_pad entries, n_pad % 8 == 0
    int pos_n = 0, neg_n = 0, n_pad = 0;
    int pos_identity = 0;
    uint32_t neg_const = 0;
    int cap = 0;  // GELU pair view: compact holds (cap + 1) x {table[m], table[0x8000 | m]}
};

struct GemmArgs {
    ActPtr A;              // [Mpad][K] in the activation format of wtype
    int K = 0;
    WPtr W;                // [N][K] repacked
    I8W Wi;                // the same weights for the int8 path (Q4 GEMMs in gemm_i8.hip)
    int N = 0;
    const float *bias = nullptr;   // [N]
    // EPI_QKV: y = b + W.x (f32, as ggml), stored split for the attention MFMAs:
    // Q | K as hi/lo fp16 planes [Mpad][2E], V transposed as hi/lo planes [E][ldv].
    // The QKV weight rows are head-major (runtime.cpp): feature h*3D + part*D + d
    // is row d of head h of Q, K or V (part 0, 1, 2), so a 3D-wide column range
    // holds one head's Q, K and V (qkv_attention_kernel).
    int head_dim = 0;
    uint16_t *qk_hi = nullptr, *qk_lo = nullptr, *vt_hi = nullptr, *vt_lo = nullptr;  // fp16 bits
    int64_t ldv = 0;
    ActPtr out_act;                // EPI_GELU_ACT: [Mpad][N]; EPI_LN: [Mpad][N]
    float *X = nullptr;            // EPI_LN: residual in / LN out, f32 [Mpad][N]
    const float *ln_w = nullptr, *ln_b = nullptr;
    float eps = 0.f;
    HalfTable gelu;                      // EPI_GELU_ACT: ggml's fp16 GELU table
    // EPI_LN in launch_gemm_i8_small: leave (b + W.x) + X in X; the caller runs
    // the LayerNorm pass (launch_ln384_rows_i8) as a launch of its own
    int defer_ln = 0;
    // EPI_LN (i8_ln384_kernel): store the f32 rows X with the nontemporal cache
    // policy (the next reader is another kernel, which reads them from HBM /
    // the fabric anyway; without them the weights stay in L2).  Off where the
    // next reader gains from them being cached (the last layer's X -> pooling)
    int nt_x = 0;
};

struct EmbedArgs {
    const int32_t *tokens = nullptr;   // [M] packed
    const int32_t *offsets = nullptr;  // [n_seqs+1]
    int32_t *rowpos = nullptr;         // [M] scratch: position of each packed row in its sentence
    int n_seqs = 0, M = 0, E = 0, n_vocab = 0, n_pos = 0;
    const void *word = nullptr, *pos = nullptr, *type = nullptr;  // ggml row format of `ttype`
    int word_t = 0, pos_t = 0, type_t = 0;
    const float *ln_w = nullptr, *ln_b = nullptr;
    float eps = 0.f;
    float *X = nullptr;
    ActPtr Xa;
};

struct AttnArgs {
    const uint16_t *qk_hi = nullptr, *qk_lo = nullptr;  // fp16 [Mpad][2E]: Q | K (GemmArgs EPI_QKV)
    const uint16_t *vt_hi = nullptr, *vt_lo = nullptr;  // fp16 [E][ldv]: V^T
    int64_t ldv = 0;
    const int32_t *offsets = nullptr;
    // qkv_attention_kernel only: tile t packs sentences tiles[2t] .. tiles[2t] +
    // tiles[2t + 1] - 1 (their lengths rounded up to 32 sum to <= 128) into one
    // workgroup; null: one sentence per workgroup
    const int32_t *tiles = nullptr;
    int E = 0, H = 0;
    float scale = 0.f;                 // 1.0f / sqrtf(d_head)
    HalfTable expt;                    // ggml's fp16 exp table
    ActPtr ctx;                        // [Mpad][E] activation format
};

constexpr int GEMM_BM = 128;  // M padding unit = the largest GEMM row tile
constexpr int ATT_QB = 64;    // queries per attention workgroup

// Launchers (kernels.hip).  Return hipSuccess or the launch error.
hipError_t launch_embed(int wtype, const EmbedArgs &a, int Mpad, hipStream_t s);
hipError_t launch_gemm(int wtype, int epi, int E_or_bn, const GemmArgs &a, int Mpad, hipStream_t s);
hipError_t launch_attention(int wtype, int d_head, const AttnArgs &a, int n_seqs, int max_len, hipStream_t s);
// whether packing n_seqs sentences into n_tiles workgroups is worth the packed variant
bool qkv_attention_pack_pays(int n_seqs, int n_tiles);
// QKV GEMM + attention in one kernel (sentences <= 128 tokens, head dim 32 or
// 64); g: the QKV GemmArgs (head-major weights in the kernel's grouped tile
// order), a: the AttnArgs (its Q/K/V pointers unused).  ntw: 192-feature
// units (head pairs at head dim 32) per GEMM main loop, 1 or 2 — the grouping
// of the kernel's QKV weight copy (runtime.cpp), chosen per context at load;
// 0: the producer / consumer kernel (head dim 32, n_embd 384; plain tile order).
bool qkv_attention_supported(int wtype, int E, int H, int max_len, int ntw);
// n_blocks: tiles (a.tiles) or sentences (a.tiles == null)
hipError_t launch_qkv_attention(int wtype, const GemmArgs &g, const AttnArgs &a, int n_blocks, int ntw, hipStream_t s);
// Small batches, Q4_0 at n_embd 384 / head dim 32, every sentence <= 128 tokens:
// the int8 QKV of one head and its attention in one workgroup per (head,
// sentence), bitwise the unfused pair (kernels.hip qkv_attention_small_kernel).
// hipErrorNotSupported when the shape does not fit.
hipError_t launch_qkv_attention_small(const GemmArgs &g, const AttnArgs &a, int n_seqs, hipStream_t s);
// out_row (optional): output row of each sentence (default: its batch index)
hipError_t launch_pool(const float *X, const int32_t *offsets, int n_seqs, int E, float *out, hipStream_t s,
                       const int32_t *out_row = nullptr);
// dst = the batch's token ids with sentence i taken from sentence perm[i]
hipError_t launch_gather_tokens(const int32_t *src, const int32_t *src_off, const int32_t *perm, const int32_t *dst_off,
                                int32_t *dst, int n_seqs, hipStream_t s);
hipError_t launch_ln(int wtype, float *X, int Mpad, int E, const float *w, const float *b, float eps,
                     const ActPtr &out, hipStream_t s);
bool gemm_shape_supported(int epi, int N, int K);
bool gemm_ln_fused(int wtype, int N);  // false: EPI_RESID + launch_ln
// true: the EPI_GELU_ACT weights are repacked in block-8 column order (repacked
// tile 2p + t, fragment row r <- weight row 32p + 8(r >> 2) + 4t + (r & 3)), so
// the transposed accumulators give each lane 8 adjacent columns of one row
bool gemm_gelu_blk8(int wtype);

// Q4 x Q8 GEMMs on the int8 MFMA (gemm_i8.hip): EPI_GELU_ACT (N % 256 == 0),
// EPI_LN (N == 384), EPI_RESID (N % 256 == 0), EPI_QKV (N % 384 == 0; the
// head-major QKV weights of qkv_attention_pc_kernel); K % 128 == 0; Mpad % 128 == 0.
bool i8_gemm_supported(int epi, int N, int K);
#ifdef PHASE_STAMPS
hipError_t stamps_set(unsigned long long *buf, int nblk);  // development stamp builds (kernels.hip)
#endif
hipError_t launch_gemm_i8(int wtype, int epi, const GemmArgs &a, int Mpad, hipStream_t s);
// the same GEMMs (bitwise) in 32-row tiles for small batches (EPI_LN: residual
// kernel + a LayerNorm kernel in i8_ln384_kernel's reduction order)
hipError_t launch_gemm_i8_small(int wtype, int epi, const GemmArgs &a, int Mpad, hipStream_t s);
// the LayerNorm pass after a small EPI_LN GEMM launched with defer_ln
// (i8_ln384_rows_kernel: X = LN(X) in i8_ln384_kernel's order, + its Q8 form)
hipError_t launch_ln384_rows_i8(int wtype, const GemmArgs &a, int Mpad, hipStream_t s);

}  // namespace bertamd
