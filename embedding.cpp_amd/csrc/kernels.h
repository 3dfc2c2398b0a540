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
// W_Q4_0D: Q4_0 weights whose GEMMs run on the block-scaled fp6 MFMA
// (gemm_f6.hip); the same ggml Q8_0 activations (d, q), stored as Q8D: per
// 32-block 48 bytes of fp6 digit codes (kernels_common.h q8d_*) + fp16 d.
enum WType : int { W_F32 = 0, W_F16 = 1, W_Q4_0 = 2, W_Q4_1 = 3, W_Q4_0D = 4, W_Q4_0N = 5, W_Q4_1N = 6 };
// W_Q4_0N / W_Q4_1N: Q4 weights kept as ggml's nibbles and dequantised inside
// the fp16 MFMA GEMM (WPtr below); their activations are Q4_0's / Q4_1's
// (ggml Q8_0 / Q8_1).
constexpr int act_of(int wt) { return wt == W_Q4_0N ? W_Q4_0 : wt == W_Q4_1N ? W_Q4_1 : wt; }
constexpr int Q8D_BLK = 48;  // code bytes per Q8D block

struct ActPtr {
    void *q = nullptr;  // int8 [M][K] | fp16 [M][K] | f32 [M][K] | Q8D codes [M][K/32][48 B]
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
//   Q4_0N: q = uint32 [N/16][K/32][64]: lane (c, g)'s 8 nibbles q (k = 8 g + j
//         at bits 4 (j >> 1) + 16 (j & 1), so one and-or per pair makes two
//         fp16 integers 1024 + q); d = fp16 [N/16][K/32][16] (d_w of column c).
//         The MFMA takes q - 8 as exact fp16 integers against the Q8 codes
//         (isum exact in f32) and the fold applies d_w * d_a per block, as
//         ggml_vec_dot_q4_0_q8_0; 0.56 B per weight.
//   Q4_1N: q = uint32 [N/16][K/32][64][2] (plain main loop only): the 8
//         nibbles q (same bit order as Q4_0N) and the fp16 d | m << 16 of
//         column c; the fold adds ggml's m_w * s_a term per block
//         (vec_dot_q4_1_q8_1: d_w d_a isum + m_w s_a, s_a = d_a sum(q_a)).
//   F16 : q = fp16 [N/16][K/32][64][8]
//   F32 : q = f32  [N/16][K/32][64][8]
struct WPtr {
    const void *q = nullptr;
    float unscale = 1.f;
    const uint16_t *d = nullptr;  // Q4_0N block scales
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

// Q4_0 weights for the fp6-MFMA GEMMs (gemm_f6.hip), repacked at load
// (runtime.cpp upload_f6) per 32-row f-tile ft (features 32 ft .. 32 ft + 31,
// natural order) and 32-wide k block b: the 32 codes of q - 8 (e2m3
// sign-magnitude, 6 bits each, element k at Q8D position q8d_pos(k)) as
//   q16: [N/32][K/32][32 rows] x 16 B (code dwords 0-3)
//   q8 : [N/32][K/32][32 rows] x 8 B  (code dwords 4-5)
//   dw : [N/32][K/128][32 rows] x 4 dwords: dword v = fp16 d_w of block 4 g + v
//        in the low half (the d_w operand of the d_w * d_a MFMA)
struct F6W {
    const uint4 *q16 = nullptr;
    const uint2 *q8 = nullptr;
    const uint4 *dw = nullptr;
};

enum Epi : int {
    EPI_QKV = 0,       // y = b + W.x split hi/lo for attention (Q|K row-major, V transposed)
    EPI_GELU_ACT = 1,  // gelu(b + W.x) in the next matmul's activation format
    EPI_LN = 2,        // LN((b + W.x) + X) -> X and activation format (the workgroup owns whole rows)
    EPI_RESID = 3,     // (b + W.x) + X -> X; LayerNorm then runs in launch_ln (rows too wide for one tile)
    EPI_NONE = 4,      // main-loop probe (tools/gemm_bench): nothing stored
    EPI_RESLN = 5      // EPI_RESID over all of a row tile's column tiles in one workgroup, then
                       // LayerNorm of its rows -> X and activation format (Q4 weights, N 768 / 1024)
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
    F6W Wf;                // the same weights for the fp6 path (Q4_0 GEMMs in gemm_f6.hip)
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
// QKV GEMM + attention in one kernel (sentences <= 128 tokens, head dim 32);
// g: the QKV GemmArgs (head-major weights), a: the AttnArgs (its Q/K/V pointers unused)
bool qkv_attention_supported(int wtype, int E, int H, int max_len);
// head pairs per GEMM main loop of that kernel (its QKV copy's tile grouping, runtime.cpp)
int qkv_attention_ntw(int wtype);
// n_blocks: tiles (a.tiles) or sentences (a.tiles == null); wtype W_Q4_0D: Q4_0
// weights, int8 Q8_0 input, context stored as Q8D
hipError_t launch_qkv_attention(int wtype, const GemmArgs &g, const AttnArgs &a, int n_blocks, hipStream_t s);
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
// EPI_LN (N == 384), EPI_RESID (N % 256 == 0); K % 128 == 0; Mpad % 128 == 0.
bool i8_gemm_supported(int epi, int N, int K);
hipError_t launch_gemm_i8(int wtype, int epi, const GemmArgs &a, int Mpad, hipStream_t s);
// The whole FFN of an n_embd 384 layer in one kernel (gemm_i8.hip
// i8_ffn384_kernel): u = the FFN-up GemmArgs (A = Xa, bias, gelu pair view, and
// in Wi the weight stream of both projections, runtime.cpp upload_ffn_i8),
// d = the FFN-down + LN GemmArgs (Wi, bias, X, ln_w / ln_b, eps, out_act);
// u.A and d.out_act may be the same buffer.  I % 384 == 0; Mpad % 64 == 0.
bool i8_ffn_supported(int E, int I);
hipError_t launch_ffn_i8(int wtype, const GemmArgs &u, const GemmArgs &d, int Mpad, hipStream_t s);

// Q4_0 x Q8D GEMMs on the fp6 MFMA (gemm_f6.hip): A in Q8D; EPI_GELU_ACT
// (N % 512 == 0, output Q8D), EPI_LN (N == 384, output `out_type` W_Q4_0D or
// ggml's Q8_0 W_Q4_0); K 384 or 1536; Mpad % 128 == 0.
bool f6_gemm_supported(int epi, int N, int K);
hipError_t launch_gemm_f6(int epi, const GemmArgs &a, int Mpad, hipStream_t s, int out_type = W_Q4_0D);
// Q8_0 (int8 q [nblk][32]) <-> Q8D codes [nblk][48 B]; the fp16 d are shared
hipError_t launch_q8_convert(bool to_q8d, const void *src, void *dst, int64_t nblk, hipStream_t s);

}  // namespace bertamd
