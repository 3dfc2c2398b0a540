// gemm_f6.hip — the Q4_0 weight GEMMs on the gfx950 block-scaled fp6 MFMA.
//
// Replaces ggml_mul_mat over Q4_0 weights (reference bert.cpp:945-992: the O,
// FFN-up and FFN-down projections), whose CPU kernel is ggml_vec_dot_q4_0_q8_0
// (SURVEY.md Appendix A): the activation row is quantised to Q8_0 blocks of
// 32 (d_a, q_a) and per block
//     sumf += (d_w * d_a) * (float) isum,   isum = sum_j (q_w[j] - 8) * q_a[j]  (exact)
// Here, per 32 x 32 output tile (rows: 32 features, columns: 32 tokens) and
// block:
//   isum = v_mfma_scale_f32_32x32x64_f8f6f4 (fp6 e2m3 operands)   exact, in f32
//   dd   = v_mfma_f32_32x32x16_f16 (d_w x one-hot d_a)             exact f32 product
//   acc  = fma(isum, dd, acc)                                        ggml's fold, one VALU op
// The MFMA's K = 64 holds the block twice: lanes 0-31 the activations' high
// digits H against the weights (E8M0 scale 2^7 = 16 * 2^3), lanes 32-63 the low
// digits L (scale 2^3), |q_a| = 16 H + L with q_a's sign on both digits
// (kernels_common.h Q8D, the producers' format).  The weights q_w - 8 are
// their own e2m3 codes under the 2^3 scale.  Against the int8 MFMA this
// drops the int -> float conversion of every isum (half the fold's VALU work,
// tools/calib_probe.hip: 94 vs 143 cycles per tile and block at two waves per
// SIMD), and the weights stream as 0.75 B each.  The fold order per output is
// the int8 path's (block by block), so results are bitwise those of
// gemm_i8.hip.  Probe of the exact isum: tools/mfma_e2m3_probe.hip.
//
// Compiled with -ffp-contract=off: every fused multiply-add below is explicit.
#include "kernels_common.h"

#include <algorithm>

namespace bertamd {

typedef int int8v __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
// (register vectors throughout: arrays of HIP's uint4 / uint2 structs carried
// across the loop were left in scratch memory by the compiler)

constexpr int F6_KC = 128;                                // K per LDS chunk: 4 quant blocks
constexpr int F6_UP_NMAX = 4096;                          // FFN-up width held in LDS (bias)
// weight-ring depth (4: two blocks ahead, 2: one) and MFMA/fold pipelining per
// kernel (tools/f6_bench.hip sweeps them)
#ifndef F6_UP_WR
#define F6_UP_WR 2
#endif
#ifndef F6_UP_PIPE
#define F6_UP_PIPE true
#endif
#ifndef F6_LN_WR
#define F6_LN_WR 4
#endif
#ifndef F6_LN_PIPE
#define F6_LN_PIPE false
#endif
// development ablations (tools/f6_bench.hip only; results wrong): bit 1 no
// fold, 2 no dd MFMA, 4 no fp6 MFMA, 8 no weight loads, 16 no A-operand LDS
// reads, 32 no epilogue (one checksum store per lane and tile)
// development: every other CU of an XCD starts F6_DESYNC_UP / _LN shader
// cycles late, so the workgroups' HBM-bound epilogues stop coinciding
#ifndef F6_DESYNC_UP
#define F6_DESYNC_UP 0
#endif
#ifndef F6_DESYNC_LN
#define F6_DESYNC_LN 0
#endif
__device__ __forceinline__ void f6_desync(int cycles) {
    if (cycles > 0 && ((blockIdx.x >> 3) & 1)) {
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        while (__builtin_amdgcn_s_memtime() - t0 < (uint64_t)cycles) __builtin_amdgcn_s_sleep(8);
    }
}

#ifndef F6_ABL
#define F6_ABL 0
#endif
constexpr int F6_SCALE_W = 130, F6_SCALE_H = 134, F6_SCALE_L = 130;  // E8M0: 2^3, 2^7, 2^3

// LDS chunk: codes [4 blocks][BM tokens][48 B] (a token's blocks 48 B apart:
// ds_read_b128 conflict-free), then d_a [4][BM] as 16-byte one-hot records:
// block bb's record holds (fp16 d_a, 0) in dword bb and zeros elsewhere, the
// dd MFMA's operand exactly as one ds_read_b128 returns it.
template <int BM>
struct F6Chunk {
    static constexpr int CB = 4 * BM * Q8D_BLK;
    static constexpr int BYTES = CB + 4 * BM * 16;
};

// One chunk's activations in flight (register staging): 16-byte pieces, 12
// per token row (4 blocks x 48 B, contiguous in the row), and the fp16 d_a.
template <int BM, int NT>
struct F6Stage {
    static constexpr int NP = 12 * BM, IT = (NP + NT - 1) / NT;
    static constexpr int ND = 4 * BM, ITD = (ND + NT - 1) / NT;
    i32x4 v[IT];
    uint32_t d[ITD];
};

// Per-lane constants of the staging copy, computed once per kernel: the byte
// offset of each piece inside a chunk's rows (global) and its LDS offset;
// the same for the d_a halves.  Surplus threads re-load piece % NP (every load
// unconditional: exact wait counts) and skip the store.
template <int BM, int NT>
struct F6StageMap {
    using S = F6Stage<BM, NT>;
    int g[S::IT], l[S::IT], gd[S::ITD], ld[S::ITD];
    __device__ __forceinline__ void init(int nkb) {
#pragma unroll
        for (int it = 0; it < S::IT; it++) {
            const int p = (int)(threadIdx.x + it * NT) % S::NP;
            const int r = p / 12, rem = p - 12 * r, bb = rem / 3;
            g[it] = r * nkb * Q8D_BLK + 16 * rem;
            const int pl = (int)threadIdx.x + it * NT;
            l[it] = (S::NP % NT == 0 || pl < S::NP) ? (bb * BM + r) * Q8D_BLK + 16 * (rem - 3 * bb) : -1;
        }
#pragma unroll
        for (int it = 0; it < S::ITD; it++) {
            const int p = (int)(threadIdx.x + it * NT) % S::ND;
            gd[it] = (p >> 2) * nkb + (p & 3);
            const int pl = (int)threadIdx.x + it * NT;
            ld[it] = (S::ND % NT == 0 || pl < S::ND) ? F6Chunk<BM>::CB + ((p & 3) * BM + (p >> 2)) * 16 : -1;
        }
    }
};

// chunk c of the rows from m0 (a row's 4 blocks of the chunk are 192
// contiguous bytes); the bases are wave-uniform
template <int BM, int NT>
__device__ __forceinline__ void f6_stage_load(F6Stage<BM, NT> &st, const F6StageMap<BM, NT> &mp, const ActPtr &A,
                                              int nkb, int64_t m0, int c) {
    using S = F6Stage<BM, NT>;
    const char *ab = (const char *)A.q + (m0 * nkb + 4 * c) * Q8D_BLK;
    const uint16_t *db = (const uint16_t *)A.d + m0 * nkb + 4 * c;
#pragma unroll
    for (int it = 0; it < S::IT; it++) st.v[it] = *(const i32x4 *)(ab + mp.g[it]);
#pragma unroll
    for (int it = 0; it < S::ITD; it++) st.d[it] = db[mp.gd[it]];
}

template <int BM, int NT>
__device__ __forceinline__ void f6_stage_store(const F6Stage<BM, NT> &st, const F6StageMap<BM, NT> &mp, char *buf) {
    using S = F6Stage<BM, NT>;
#pragma unroll
    for (int it = 0; it < S::IT; it++)
        if (S::NP % NT == 0 || mp.l[it] >= 0) *(i32x4 *)(buf + mp.l[it]) = st.v[it];
#pragma unroll
    for (int it = 0; it < S::ITD; it++)
        if (S::ND % NT == 0 || mp.ld[it] >= 0) {
            const int bb = (mp.ld[it] - F6Chunk<BM>::CB) / (16 * BM), v = (int)st.d[it];
            *(i32x4 *)(buf + mp.ld[it]) = i32x4{bb == 0 ? v : 0, bb == 1 ? v : 0, bb == 2 ? v : 0, bb == 3 ? v : 0};
        }
}

typedef int int16v_ __attribute__((ext_vector_type(16)));
__device__ __forceinline__ int16v_ int16v_of(const int8v &a, const int8v &b) {
    int16v_ r;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r[i] = a[i];
        r[8 + i] = b[i];
    }
    return r;
}

// Activation operands of block BB of the chunk for the wave's T t-tiles:
// the token's digit plane of this lane half (hi: lanes 0-31, lo: 32-63) and
// its d_a dword.  Lane constants: lb = l32 * 48 + 16 hh (the plane's first 16
// bytes), l8 = 32 - 8 hh (its last 8, from there), lt = 4 l32 (the d_a dword).
template <int T>
struct F6AOps {
    int8v xa[T];
    i32x4 oh[T];  // the dd MFMA's one-hot d_a operand
};

struct F6Lane {
    int lb, l8, lt;
};

template <int BM, int T, int BB>
__device__ __forceinline__ void f6_aops(F6AOps<T> &o, const char *buf, const F6Lane &ln) {
#pragma unroll
    for (int t = 0; t < T; t++) {
        if constexpr (F6_ABL & 16) {
            o.xa[t] = int8v{ln.lb, ln.l8, BB, t, 3, 4, 0, 0};
            o.oh[t] = i32x4{ln.lt, BB, t, 0};
            continue;
        }
        const char *p = buf + ln.lb + (BB * BM + 32 * t) * Q8D_BLK;
        const i32x4 x = *(const i32x4 *)p;
        const i32x2 y = *(const i32x2 *)(p + ln.l8);
        o.xa[t] = int8v{x[0], x[1], x[2], x[3], y[0], y[1], 0, 0};
        o.oh[t] = *(const i32x4 *)(buf + F6Chunk<BM>::CB + (BB * BM + 32 * t) * 16 + ln.lt);
    }
}

// Pipeline state carried from block to block and across the tiles of a
// persistent workgroup (the gemm_i8.hip I8Pipe structure): weight fragments
// stream through a WR-slot register ring WR - 2 blocks ahead (WR = 4: two
// ahead; WR = 2: the next block), the A chunk and the chunk's d_w operand are
// loaded in the middle of the previous chunk; every load is unconditional and
// issued in consumption order (exact vmcnt waits).  Weight addresses: a
// wave-uniform base (SGPR) + the lane's row.
template <int NT, int BM, int F, int WR>
struct F6Pipe {
    F6Stage<BM, NT> st;
    F6StageMap<BM, NT> mp;
    int8v wq[WR][F];  // the MFMA operand itself (dwords 6, 7 unused by fp6; a ring of two
                      // vectors read as one 8-dword load kept the ring in scratch)
    i32x4 wdr[F];     // d_w of the chunk's 4 blocks (dword v: fp16 of block 4c + v)

    template <int S>
    __device__ __forceinline__ void wload(const GemmArgs &g, int nkb, int ft0, int ft0n, int b) {
        const bool nx = b >= nkb;
        const int ft = nx ? ft0n : ft0, bb = nx ? b - nkb : b;
        const unsigned r = threadIdx.x & 31u;
#pragma unroll
        for (int f = 0; f < F; f++) {
            const int64_t i0 = ((int64_t)(ft + f) * nkb + bb) * 32;
            if constexpr (F6_ABL & 8) {
                wq[S][f] = int8v{(int)r, (int)i0, f, bb, 1, 2, 0, 0};
            } else {
                const i32x4 a = ((const i32x4 *)g.Wf.q16 + i0)[r];
                const i32x2 b = ((const i32x2 *)g.Wf.q8 + i0)[r];
                wq[S][f] = int8v{a[0], a[1], a[2], a[3], b[0], b[1], 0, 0};
            }
        }
    }
    __device__ __forceinline__ void cload(const GemmArgs &g, int64_t m0, int ft0, int c) {
        const int nkb = g.K >> 5;
        f6_stage_load<BM, NT>(st, mp, g.A, nkb, m0, c);
#pragma unroll
        for (int f = 0; f < F; f++)
            wdr[f] = ((const i32x4 *)g.Wf.dw + ((int64_t)(ft0 + f) * (nkb >> 2) + c) * 32)[threadIdx.x & 31u];
    }
    __device__ __forceinline__ void prime(const GemmArgs &g, int64_t m0, int ft0) {
        const int nkb = g.K >> 5;
        mp.init(nkb);
        wload<0>(g, nkb, ft0, ft0, 0);
        if constexpr (WR == 4) wload<1>(g, nkb, ft0, ft0, 1);
        static_assert(WR == 2 || WR == 4, "weight ring of 2 or 4 slots");
        cload(g, m0, ft0, 0);
    }
};

// One quant block (BB: its index inside the chunk) of the main loop, with its
// activation operands `cur` (the next block's are read into `nxt`).
template <int BM, int F, int T, int BB, bool PIPE>
__device__ __forceinline__ void f6_block(const char *buf, const F6Lane &ln, const int8v (&wq)[F],
                                         const i32x4 (&wd)[F], const F6AOps<T> &cur, F6AOps<T> &nxt,
                                         float16v (&acc)[F][T]) {
    const int hh = (threadIdx.x & 63) >> 5;
    const int sb = hh ? F6_SCALE_L : F6_SCALE_H;
    const float16v zf = {};
    if constexpr (BB < 3) f6_aops<BM, T, BB + 1>(nxt, buf, ln);
    // dd: the one-hot d_a operand holds (d_a, 0) in dword BB (k = 2 BB), the
    // d_w operand the chunk's four d_w at k = 0, 2, 4, 6 (lanes 32-63 zero)
    auto mm = [&](int f, int t, float16v &is, float16v &dd) {
        if constexpr (F6_ABL & 4)
            is = __builtin_bit_cast(float16v, int16v_of(cur.xa[t], wq[f]));
        else
            is = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wq[f], cur.xa[t], zf, 2, 2, 0, F6_SCALE_W, 0, sb);
        if constexpr (F6_ABL & 2)
            dd = is;
        else
            dd = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, wd[f]),
                                                        __builtin_bit_cast(half8, cur.oh[t]), zf, 0, 0, 0);
    };
    // software pipeline over the F x T tiles: tile p + 1's two MFMAs are in
    // flight while tile p is folded (PIPE false: tile by tile)
    float16v is[2], dd[2];
    mm(0, 0, is[0], dd[0]);
#pragma unroll
    for (int p = 0; p < F * T; p++) {
        if (!PIPE && p > 0) mm(p / T, p % T, is[p & 1], dd[p & 1]);
        if (PIPE && p + 1 < F * T) mm((p + 1) / T, (p + 1) % T, is[(p + 1) & 1], dd[(p + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (F6_ABL & 1) {
            acc[p / T][p % T][p] += is[p & 1][p] + dd[p & 1][p];
        } else {
            // v_pk_fma_f32: two of the lane's 16 sums per issue
            float16v v = __builtin_elementwise_fma(is[p & 1], dd[p & 1], acc[p / T][p % T]);
            asm volatile("" : "+v"(v));  // keep the fold here: sunk past the MFMAs it would keep every tile live
            acc[p / T][p % T] = v;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// acc[f][t] = A[m0 + 32 (tt0 + t) ..][:] . W[32 (ft0 + f) ..][:]^T over the
// whole K for the wave's F f-tiles x T t-tiles (tt0 = 0: the wave covers the
// BM rows); `pp` holds this tile's first loads on entry and the next tile's
// (m0n, ft0n) on return.  Returns after a final barrier (the LDS may be reused).
// NCH = K / 128 chunks (a compile-time trip count; the loop stays rolled:
// unrolled, the scheduler's hoisting spilled 36-604 B per lane).
template <int NT, int BM, int F, int T, int WR, bool PIPE, int NCH>
__device__ __forceinline__ void f6_mainloop(const GemmArgs &g, int64_t m0, int ft0, int64_t m0n, int ft0n, char *smem,
                                            F6Pipe<NT, BM, F, WR> &pp, float16v (&acc)[F][T]) {
    using C = F6Chunk<BM>;
    const int lane = threadIdx.x & 63, hh = lane >> 5;
    const int nkb = 4 * NCH, nch = NCH;
    // this lane's token rows in the chunk buffer (t-tile 0), its plane half
    F6Lane ln{(lane & 31) * Q8D_BLK + 16 * hh, 32 - 8 * hh, 16 * (lane & 31)};
    asm volatile("" : "+v"(ln.lb), "+v"(ln.l8), "+v"(ln.lt));
#pragma unroll
    for (int f = 0; f < F; f++)
#pragma unroll
        for (int t = 0; t < T; t++) acc[f][t] = float16v{};
    i32x4 wd[F];
    auto wscale_use = [&]() {
#pragma unroll
        for (int f = 0; f < F; f++) wd[f] = hh ? i32x4{0, 0, 0, 0} : pp.wdr[f];
    };
    f6_stage_store<BM, NT>(pp.st, pp.mp, smem);
    wscale_use();
    __syncthreads();
#pragma unroll 1
    for (int c = 0; c < nch; c++) {
        const bool more = c + 1 < nch;
        const int b0 = 4 * c;
        const char *buf = smem + (c & 1) * C::BYTES;
        F6AOps<T> a0, a1;
        f6_aops<BM, T, 0>(a0, buf, ln);
        if constexpr (WR == 4) {
            f6_block<BM, F, T, 0, PIPE>(buf, ln, pp.wq[0], wd, a0, a1, acc);
            pp.template wload<2>(g, nkb, ft0, ft0n, b0 + 2);
            f6_block<BM, F, T, 1, PIPE>(buf, ln, pp.wq[1], wd, a1, a0, acc);
            pp.template wload<3>(g, nkb, ft0, ft0n, b0 + 3);
            pp.cload(g, more ? m0 : m0n, more ? ft0 : ft0n, more ? c + 1 : 0);
            f6_block<BM, F, T, 2, PIPE>(buf, ln, pp.wq[2], wd, a0, a1, acc);
            pp.template wload<0>(g, nkb, ft0, ft0n, b0 + 4);
            f6_block<BM, F, T, 3, PIPE>(buf, ln, pp.wq[3], wd, a1, a0, acc);
            pp.template wload<1>(g, nkb, ft0, ft0n, b0 + 5);
        } else {
            pp.template wload<1>(g, nkb, ft0, ft0n, b0 + 1);
            f6_block<BM, F, T, 0, PIPE>(buf, ln, pp.wq[0], wd, a0, a1, acc);
            pp.template wload<0>(g, nkb, ft0, ft0n, b0 + 2);
            f6_block<BM, F, T, 1, PIPE>(buf, ln, pp.wq[1], wd, a1, a0, acc);
            pp.template wload<1>(g, nkb, ft0, ft0n, b0 + 3);
            pp.cload(g, more ? m0 : m0n, more ? ft0 : ft0n, more ? c + 1 : 0);
            f6_block<BM, F, T, 2, PIPE>(buf, ln, pp.wq[0], wd, a0, a1, acc);
            pp.template wload<0>(g, nkb, ft0, ft0n, b0 + 4);
            f6_block<BM, F, T, 3, PIPE>(buf, ln, pp.wq[1], wd, a1, a0, acc);
        }
        if (more) {
            f6_stage_store<BM, NT>(pp.st, pp.mp, smem + ((c + 1) & 1) * C::BYTES);
            wscale_use();
        }
        __syncthreads();
    }
}

// XCD-aware tile order: linear ids are dealt round-robin over the 8 XCDs;
// each XCD walks a contiguous range, n fastest.
__device__ __forceinline__ int f6_xcd_linear(int orig, int nwg) {
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
}

// Features held by lane half hh in register i of a 32 x 32 result: row
// 8 (i >> 2) + 4 hh + (i & 3) of the f-tile (weights in natural row order),
// which is Q8D position 16 hh + i of the output block.
__device__ __forceinline__ int f6_row(int i, int hh) { return 8 * (i >> 2) + 4 * hh + (i & 3); }

// ---------------------------------------------------------------------------
// FFN up + GELU (bert.cpp:965-971): U = gelu(b + W.h) in Q8D.  Persistent:
// one 8-wave workgroup per CU walks 64 x 512 tiles; ggml's fp16 GELU table
// (entries [0, 0x8000 + neg_n], kernels.h GELU_FLAT_LDS) is read into LDS once.
// Wave w: f-tiles 2w, 2w + 1 of the tile, both 32-token t-tiles.
template <int NWV, int F, int T, int NCH>
__global__ __launch_bounds__(NWV * 64) void f6_up_gelu_kernel(GemmArgs g, int n_mtiles, int n_ntiles) {
    constexpr int NT = NWV * 64, BM = 32 * T, BN = 32 * NWV * F;
    using C = F6Chunk<BM>;
    __shared__ __attribute__((aligned(16))) char smem[2 * C::BYTES];
    __shared__ __attribute__((aligned(16))) uint16_t gtab[(F6_ABL & 32) ? 8 : GELU_FLAT_LDS];
    __shared__ __attribute__((aligned(16))) float sbias[F6_UP_NMAX];  // the epilogue reads bias from LDS
    const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: tile coordinates in SGPRs
    const int nflat8 = (0x8000 + g.gelu.neg_n + 1 + 7) / 8;
    if constexpr ((F6_ABL & 32) == 0)
        for (int i = tid; i < nflat8; i += NT) ((uint4 *)gtab)[i] = ((const uint4 *)g.gelu.full)[i];
    for (int i = tid; i < g.N; i += NT) sbias[i] = g.bias[i];
    const float xlo = h2f((uint16_t)(0x8000 | g.gelu.neg_n));
    const int nwg = n_mtiles * n_ntiles, nbo = g.N >> 5;
    const int fw = F * wv;
    auto coords = [&](int tile, int64_t &m0_, int &ft0_) {
        const int lin = f6_xcd_linear(tile, nwg);
        const int mt = lin / n_ntiles, nt = lin - mt * n_ntiles;
        m0_ = (int64_t)mt * BM;
        ft0_ = nt * (BN / 32) + fw;
    };
    if ((int)blockIdx.x >= nwg) return;
    f6_desync(F6_DESYNC_UP);
    int64_t m0;
    int ft0;
    coords(blockIdx.x, m0, ft0);
    F6Pipe<NT, BM, F, F6_UP_WR> pp;
    pp.prime(g, m0, ft0);
    for (int tile = blockIdx.x; tile < nwg; tile += gridDim.x) {
        int64_t m0n = m0;
        int ft0n = ft0;
        if (tile + (int)gridDim.x < nwg) coords(tile + gridDim.x, m0n, ft0n);
        float16v acc[F][T];
        f6_mainloop<NT, BM, F, T, F6_UP_WR, F6_UP_PIPE, NCH>(g, m0, ft0, m0n, ft0n, smem, pp, acc);
        const int64_t mc = m0;
        const int fc = ft0;
        m0 = m0n;
        ft0 = ft0n;
        if constexpr ((F6_ABL & 32) != 0) {
            float cs = 0.f;
#pragma unroll
            for (int f = 0; f < F; f++)
#pragma unroll
                for (int t = 0; t < T; t++)
#pragma unroll
                    for (int i = 0; i < 16; i++) cs += acc[f][t][i];
            ((float *)g.out_act.q)[(int64_t)tile * NT + tid] = cs;
            continue;
        }
#pragma unroll
        for (int f = 0; f < F; f++) {
            float bias[16];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4v b4 = *(const float4v *)(sbias + 32 * (fc + f) + 8 * q + 4 * hh);
#pragma unroll
                for (int j = 0; j < 4; j++) bias[4 * q + j] = b4[j];
            }
#pragma unroll
            for (int t = 0; t < T; t++) {
                float y[16];
#pragma unroll
                for (int i = 0; i < 16; i++) y[i] = h2f(gtab[f2h(fmaxf(bias[i] + acc[f][t][i], xlo))]);
                const int64_t bi = (mc + 32 * t + l32) * nbo + fc + f;
                q8d_store_pair((char *)g.out_act.q + bi * Q8D_BLK, (uint16_t *)g.out_act.d + bi, hh, y,
                               (F6_ABL & 64) == 0 || g.eps == 12345.f);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Projection + residual + LayerNorm for n_embd = 384 (bert.cpp:944-962 and
// :973-992): X = LN((b + W.x) + X), stored f32 and in Q8D.  One 12-wave
// workgroup owns BM = 64 whole rows: wave w holds f-tile w (32 features) of
// both 32-token t-tiles, so a row's 384 values are spread over 12 waves x 2
// lane halves x 16.  ggml_norm's double sums go lane -> lane pair -> the
// twelve waves (LDS partials, fixed order).
// Q8 block of 32 outputs held as 16 per lane by lanes l and l ^ 32 in the
// natural-order accumulator layout (element 4q + j of lane half hh is column
// 8q + 4hh + j), stored as ggml's Q8_0 (int8 codes + fp16 d; the i8 path's
// i8_store_q8_half arithmetic): four dwords per lane.
__device__ __forceinline__ void f6_store_q8_0(const ActPtr &out, int64_t row, int blk, int hh, const float (&y)[16],
                                              bool valid = true) {
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 16; i++) amax = fmaxf(amax, fabsf(y[i]));
    {
        const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
        amax = fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
    }
    float d, id;
    q8_scales(amax, d, id);
    uint32_t *dst = (uint32_t *)((int8_t *)out.q + row * 384 + 32 * blk + 4 * hh);
    uint32_t pk[4];
#pragma unroll
    for (int q = 0; q < 4; q++) pk[q] = q8_pack4(y[4 * q], y[4 * q + 1], y[4 * q + 2], y[4 * q + 3], id);
    if (!valid) return;
#pragma unroll
    for (int q = 0; q < 4; q++) dst[2 * q] = pk[q];
    if (hh == 0) ((uint16_t *)out.d)[row * 12 + blk] = f2h(d);
}

template <int NCH, bool OUT_Q8D>
__global__ __launch_bounds__(768) void f6_ln384_kernel(GemmArgs g, int n_mtiles) {
    constexpr int NT = 768, BM = 64, F = 1, T = 2, NCOL = 384, NWV = 12, NBO = NCOL / 32;
    using C = F6Chunk<BM>;
    __shared__ __attribute__((aligned(16))) char smem[2 * C::BYTES];
    __shared__ double red[2][NWV][BM];
    __shared__ __attribute__((aligned(16))) float prm[3][NCOL];  // bias, ln_w, ln_b
    const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), ft0 = wv;
    for (int i = tid; i < 3 * NCOL; i += NT) {
        const int k = i / NCOL, c = i - k * NCOL;
        prm[k][c] = (k == 0 ? g.bias : k == 1 ? g.ln_w : g.ln_b)[c];
    }
    if ((int)blockIdx.x >= n_mtiles) return;
    f6_desync(F6_DESYNC_LN);
    int64_t m0n = (int64_t)f6_xcd_linear(blockIdx.x, n_mtiles) * BM;
    F6Pipe<NT, BM, F, F6_LN_WR> pp;
    pp.prime(g, m0n, ft0);
    for (int tile = blockIdx.x; tile < n_mtiles; tile += gridDim.x) {
        const int64_t m0 = m0n;
        if (tile + (int)gridDim.x < n_mtiles) m0n = (int64_t)f6_xcd_linear(tile + gridDim.x, n_mtiles) * BM;
        float16v acc[F][T];
        f6_mainloop<NT, BM, F, T, F6_LN_WR, F6_LN_PIPE, NCH>(g, m0, ft0, m0n, ft0, smem, pp, acc);
        if constexpr ((F6_ABL & 32) != 0) {
            float cs = 0.f;
#pragma unroll
            for (int t = 0; t < T; t++)
#pragma unroll
                for (int i = 0; i < 16; i++) cs += acc[0][t][i];
            g.X[(int64_t)tile * NT + tid] = cs;
            continue;
        }
        // v = (b + W.x) + x  (ggml: add(repeat(b), mul_mat) then add(cur, inpL));
        // the residual rows are loaded all at once, the parameters come from LDS
        float4v xv[T][4];
#pragma unroll
        for (int t = 0; t < T; t++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                xv[t][q] = *(const float4v *)(g.X + (m0 + 32 * t + l32) * NCOL + 32 * ft0 + 8 * q + 4 * hh);
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int r = 32 * t + l32;
            double s = 0.0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4v b4 = *(const float4v *)(prm[0] + 32 * ft0 + 8 * q + 4 * hh);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float v = (b4[j] + acc[0][t][4 * q + j]) + xv[t][q][j];
                    acc[0][t][4 * q + j] = v;
                    s += (double)v;
                }
            }
            s += __shfl_xor(s, 32);
            if (hh == 0) red[0][wv][r] = s;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int r = 32 * t + l32;
            double tot = 0.0;
#pragma unroll
            for (int w = 0; w < NWV; w++) tot += red[0][w][r];
            const float mean = (float)(tot / NCOL);
            double s2 = 0.0;
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const float v = acc[0][t][i] - mean;
                acc[0][t][i] = v;
                s2 += (double)(v * v);
            }
            s2 += __shfl_xor(s2, 32);
            if (hh == 0) red[1][wv][r] = s2;
        }
        __syncthreads();
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
            float *xr = g.X + row * NCOL + 32 * ft0 + 4 * hh;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4v w4 = *(const float4v *)(prm[1] + 32 * ft0 + 8 * q + 4 * hh);
                const float4v b4 = *(const float4v *)(prm[2] + 32 * ft0 + 8 * q + 4 * hh);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float z = acc[0][t][4 * q + j] * scale;
                    z = w4[j] * z;
                    y[4 * q + j] = z + b4[j];
                }
                if ((F6_ABL & 64) == 0 || g.eps == 12345.f)
                    *(float4v *)(xr + 8 * q) = float4v{y[4 * q], y[4 * q + 1], y[4 * q + 2], y[4 * q + 3]};
            }
            const int64_t bi = row * NBO + ft0;
            if constexpr (OUT_Q8D)
                q8d_store_pair((char *)g.out_act.q + bi * Q8D_BLK, (uint16_t *)g.out_act.d + bi, hh, y,
                               (F6_ABL & 64) == 0 || g.eps == 12345.f);
            else
                f6_store_q8_0(g.out_act, row, ft0, hh, y, (F6_ABL & 64) == 0 || g.eps == 12345.f);
        }
        // the next tile's main loop reuses `red` only after its own barriers
    }
}

// ---------------------------------------------------------------------------
// Format converters between ggml's Q8_0 (int8 q, fp16 d) and Q8D, one thread
// per 32-element block: exact re-encodings of the same (d, q).
__global__ __launch_bounds__(256) void q8_to_q8d_kernel(const int8_t *__restrict__ q, uint8_t *__restrict__ out,
                                                        int64_t nblk) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= nblk) return;
    uint32_t pl[2][6] = {{0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0}};
#pragma unroll
    for (int e = 0; e < 32; e++) {
        const int v = q[b * 32 + e], m = v < 0 ? -v : v;
        const uint32_t s = v < 0 ? 32u : 0u;
        const int bit = 6 * q8d_pos(e), w = bit >> 5, o = bit & 31;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const uint32_t code = (uint32_t)(k ? (m & 15) : (m >> 4)) | s;
            pl[k][w] |= code << o;
            if (o > 26) pl[k][w + 1] |= code >> (32 - o);
        }
    }
    char *blk = (char *)out + b * Q8D_BLK;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        *(uint4 *)(blk + 16 * k) = make_uint4(pl[k][0], pl[k][1], pl[k][2], pl[k][3]);
        *(uint2 *)(blk + 32 + 8 * k) = make_uint2(pl[k][4], pl[k][5]);
    }
}

__global__ __launch_bounds__(256) void q8d_to_q8_kernel(const uint8_t *__restrict__ in, int8_t *__restrict__ q,
                                                        int64_t nblk) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= nblk) return;
    const char *blk = (const char *)in + b * Q8D_BLK;
#pragma unroll
    for (int e = 0; e < 32; e++) {
        const int p = q8d_pos(e), bit = 6 * p;
        auto code = [&](int plane) {
            const int n = bit >> 3, o = bit & 7;
            const uint32_t two = (uint32_t)(uint8_t)*q8d_byte((char *)blk, plane, n) |
                                 (n + 1 < 24 ? (uint32_t)(uint8_t)*q8d_byte((char *)blk, plane, n + 1) << 8 : 0u);
            return (two >> o) & 63u;
        };
        const uint32_t h = code(0), l = code(1);
        const int m = (int)(16 * (h & 15u) + (l & 15u));
        q[b * 32 + e] = (int8_t)((h | l) & 32u ? -m : m);
    }
}

// ---------------------------------------------------------------------------
static int n_cus_f6() {
    static int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            c = 256;
        return c;
    }();
    return n;
}

static int f6_persistent_grid(int tiles) { return std::max(1, std::min(tiles, std::max(8, n_cus_f6() / 8 * 8))); }

#ifndef F6_UP_FT
#define F6_UP_FT 22  // f-tiles x t-tiles per wave (development: 14 = F 1, T 4)
#endif
constexpr int F6_UP_WAVES = 8, F6_UP_F = F6_UP_FT / 10, F6_UP_T = F6_UP_FT % 10;

bool f6_gemm_supported(int epi, int N, int K) {
    if (K != 384 && K != 1536) return false;  // the chunk loops are unrolled per K
    if (epi == EPI_GELU_ACT) return N % (32 * F6_UP_WAVES * F6_UP_F) == 0;
    if (epi == EPI_LN) return N == 384;
    return false;
}

hipError_t launch_gemm_f6(int epi, const GemmArgs &a, int Mpad, hipStream_t s, int out_type) {
    if (!f6_gemm_supported(epi, a.N, a.K) || Mpad % 128) return hipErrorInvalidValue;
    if (out_type != W_Q4_0D && (epi != EPI_LN || out_type != W_Q4_0)) return hipErrorInvalidValue;
    if (epi == EPI_GELU_ACT) {
        if (0x8000 + a.gelu.neg_n + 1 > GELU_FLAT_LDS) return hipErrorInvalidValue;
        constexpr int NWV = F6_UP_WAVES, F = F6_UP_F, T = F6_UP_T;
        const int mt = Mpad / (32 * T), nt = a.N / (32 * NWV * F);
        if (a.K == 384)
            hipLaunchKernelGGL((f6_up_gelu_kernel<NWV, F, T, 3>), dim3(f6_persistent_grid(mt * nt)), dim3(NWV * 64), 0,
                               s, a, mt, nt);
        else
            hipLaunchKernelGGL((f6_up_gelu_kernel<NWV, F, T, 12>), dim3(f6_persistent_grid(mt * nt)), dim3(NWV * 64), 0,
                               s, a, mt, nt);
    } else {
        const int mt = Mpad / 64;
        const dim3 grid(f6_persistent_grid(mt)), blk(768);
        const bool q8d = out_type == W_Q4_0D;
        auto kern = a.K == 384 ? (q8d ? f6_ln384_kernel<3, true> : f6_ln384_kernel<3, false>)
                               : (q8d ? f6_ln384_kernel<12, true> : f6_ln384_kernel<12, false>);
        hipLaunchKernelGGL(kern, grid, blk, 0, s, a, mt);
    }
    return hipGetLastError();
}

hipError_t launch_q8_convert(bool to_q8d, const void *src, void *dst, int64_t nblk, hipStream_t s) {
    if (nblk <= 0) return hipSuccess;
    const int grid = (int)((nblk + 255) / 256);
    if (to_q8d)
        hipLaunchKernelGGL(q8_to_q8d_kernel, dim3(grid), dim3(256), 0, s, (const int8_t *)src, (uint8_t *)dst, nblk);
    else
        hipLaunchKernelGGL(q8d_to_q8_kernel, dim3(grid), dim3(256), 0, s, (const uint8_t *)src, (int8_t *)dst, nblk);
    return hipGetLastError();
}

}  // namespace bertamd
