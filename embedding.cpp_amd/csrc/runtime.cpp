// runtime.cpp — host runtime behind the reference C ABI (include/bert.h).
//
// Replaces the reference's bert.cpp runtime (loader bert.cpp:143-659, context
// and arena bert.cpp:79-137/803-842, eval loop bert.cpp:1020-1108, encode
// drivers bert.cpp:1110-1198) with:
//   - a native GGUF reader (gguf_io.cpp) and the same hparam / tensor-shape
//     validation as the reference loader (bert.cpp:496-513, 623-652);
//   - per-device weight replicas, repacked once at load into MFMA fragment
//     order (no per-call graph, no arena, no mem-per-token probe);
//   - a fixed kernel pipeline over a ragged batch of sentences (kernels.hip);
//   - data-parallel sharding of a batch over the context's devices, one host
//     thread per device, no collectives.
// Nothing throws across the ABI: load returns NULL, eval logs and returns.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "bert.h"
#include "bert_amd.h"
#include "ggml_formats.h"
#include "gguf_io.h"
#include "kernels.h"
#include "tokenizer.h"

using namespace bertamd;

namespace {

thread_local std::string g_err;

void set_err(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

#define HIP_OK_RC(expr, rc)                                                           \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess) {                                                       \
            set_err("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
            return rc;                                                                \
        }                                                                             \
    } while (0)
#define HIP_OK(expr)                                                                  \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess) {                                                       \
            set_err("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
            return false;                                                             \
        }                                                                             \
    } while (0)

// ggml_init's fp16 tables (GELU tanh form and exp), built with this host's libm
// exactly like ggml builds them.
// Compact LDS view of a full table (kernels.h HalfTable): the shortest
// [0, pos_n) / [0x8000, 0x8000 + neg_n) ranges outside which every finite
// entry is h itself (positive side, if allowed) or one constant (negative side).
struct CompactTable {
    std::vector<uint16_t> compact;
    int pos_n = 0, neg_n = 0, pos_identity = 0;
    uint32_t neg_const = 0;
};
CompactTable compact_table(const std::vector<uint16_t> &full, bool identity_tail, int pos_n_fixed) {
    CompactTable c;
    if (identity_tail) {
        int p = 0x7c00;
        while (p > 0 && full[(size_t)(p - 1)] == (uint16_t)(p - 1)) p--;
        c.pos_n = p;
        c.pos_identity = 1;
    } else {
        c.pos_n = pos_n_fixed;  // positives beyond it read the global table
    }
    c.neg_const = full[0xfbff];
    int n = 0x7c00;
    while (n > 0 && full[(size_t)(0x8000 | (n - 1))] == c.neg_const) n--;
    c.neg_n = n;
    const int tot = c.pos_n + c.neg_n + 1, pad = (tot + 7) / 8 * 8;  // + neg_const at [pos_n + neg_n]
    c.compact.assign((size_t)pad, 0);
    c.compact[(size_t)(c.pos_n + c.neg_n)] = (uint16_t)c.neg_const;
    for (int h = 0; h < c.pos_n; h++) c.compact[(size_t)h] = full[(size_t)h];
    for (int m = 0; m < c.neg_n; m++) c.compact[(size_t)(c.pos_n + m)] = full[(size_t)(0x8000 | m)];
    // self-check of the device lookup rules on every finite pattern they serve
    // (kernels.hip gelu_lookup; soft_max's exp lookup only sees s - max <= 0)
    for (uint32_t h = 0; h < 65536; h++) {
        const uint32_t mag = h & 0x7fffu;
        const bool neg = (h & 0x8000u) != 0;
        if (mag >= 0x7c00u || (!neg && !identity_tail && mag > 0)) continue;
        uint32_t v;
        if (neg) v = c.compact[(size_t)(c.pos_n + std::min<uint32_t>(mag, (uint32_t)c.neg_n))];
        else v = mag >= (uint32_t)c.pos_n ? h : c.compact[mag];
        if (v != full[h]) c.pos_n = c.neg_n = 1 << 20;  // poison: load_impl reports it
    }
    return c;
}

// GELU pair view (kernels.hip gelu_lookup): entry m = {table[m], table[0x8000 | m]}
// for m <= cap = max(pos_n, neg_n); checked on every finite pattern.
std::vector<uint16_t> pair_table(const std::vector<uint16_t> &full, const CompactTable &c, int &cap) {
    cap = std::max(c.pos_n, c.neg_n);
    const int n = 2 * (cap + 1), pad = (n + 7) / 8 * 8;
    std::vector<uint16_t> t((size_t)pad, 0);
    for (int m = 0; m <= cap; m++) {
        t[(size_t)(2 * m)] = full[(size_t)m];
        t[(size_t)(2 * m + 1)] = full[(size_t)(0x8000 | m)];
    }
    for (uint32_t h = 0; h < 65536; h++) {
        if ((h & 0x7fffu) >= 0x7c00u) continue;
        const uint32_t m = std::min<uint32_t>(h & 0x7fffu, (uint32_t)cap);
        uint32_t v = t[2 * m + (h >> 15)];
        if (h < 0x8000u && h > (uint32_t)cap) v = h;
        if (v != full[h]) cap = 1 << 20;  // poison: load_impl reports it
    }
    return t;
}

struct HostTables {
    std::vector<uint16_t> gelu, expt, gelu_pair;
    int gelu_cap = 0;
    CompactTable gelu_c, exp_c;
    HostTables() : gelu(65536), expt(65536) {
        const float A = 0.044715f, S = 0.79788456080286535587989211986876f;
        for (int i = 0; i < 65536; i++) {
            const float f = f16_to_f32((uint16_t)i);
            const float g = 0.5f * f * (1.0f + tanhf(S * f * fmaf(A * f, f, 1.0f)));
            gelu[i] = f32_to_f16(g);
            expt[i] = f32_to_f16(expf(f));
        }
        gelu_c = compact_table(gelu, true, 0);
        gelu_pair = pair_table(gelu, gelu_c, gelu_cap);
        exp_c = compact_table(expt, false, 1);  // soft_max only feeds s - max <= 0
    }
};
const HostTables &tables() {
    static HostTables t;
    return t;
}
HalfTable half_table(const uint16_t *full, const uint16_t *compact, const CompactTable &c) {
    HalfTable t;
    t.full = full;
    t.compact = compact;
    t.pos_n = c.pos_n;
    t.neg_n = c.neg_n;
    t.n_pad = (int)c.compact.size();
    t.pos_identity = c.pos_identity;
    t.neg_const = c.neg_const;
    return t;
}

struct HParams {
    int32_t n_vocab = 0, n_max_tokens = 0, n_embd = 0, n_intermediate = 0, n_head = 0, n_layer = 0;
    float eps = 1e-12f;
};

struct DevMat {
    WPtr w;
};

struct DevLayer {
    WPtr qkv, o, up, down;
    I8W o8, up8, down8;  // Q4 weights for the int8-MFMA GEMMs (gemm_i8.hip)
    I8W qkv8;            // head-major QKV on the int8 MFMA (qkva_ntw 0: qkv_attention_pc_kernel + i8 EPI_QKV)
    WPtr qkv_plain;  // head-major QKV in grouped, plain tile order: qkv_attention_kernel's copy (when supported)
    float *b_qkv = nullptr, *b_o = nullptr, *b_up = nullptr, *b_down = nullptr;
    float *ln1_w = nullptr, *ln1_b = nullptr, *ln2_w = nullptr, *ln2_b = nullptr;
};

struct Workspace {
    int64_t cap_rows = 0;   // padded rows
    int64_t cap_seqs = 0;
    float *X = nullptr, *out = nullptr;
    uint16_t *qk_hi = nullptr, *qk_lo = nullptr, *vt_hi = nullptr, *vt_lo = nullptr;  // fp16: kernels.h GemmArgs EPI_QKV
    ActPtr Xa, Ca, Ua;
    int32_t *tok = nullptr, *off = nullptr, *rowpos = nullptr;
    int32_t *tiles = nullptr;  // qkv_attention_kernel's sentence tiles: [first, count] pairs
    int32_t *perm = nullptr;   // eval_device in tile order: caller's index of each sentence
    std::vector<int32_t> h_tiles;
    std::vector<void *> allocs;
    // pinned host staging for the host-pointer ABI
    int32_t *h_tok = nullptr, *h_off = nullptr;
    float *h_out = nullptr;
    int64_t h_cap_rows = 0, h_cap_seqs = 0;
    uint64_t gen = 0;  // bumped when the device buffers are reallocated (captured graphs hold their addresses)
};

struct ProfEntry {
    double ms = 0;
    int64_t n = 0;
};

// One evaluation lane of a replica: a workspace with its streams and events.
// Lane 0 serves bert_eval_batch, eval_device and debug_embed; bert_encode_batch
// adds lanes (encode_lanes) to run several of its slices at once on one
// device, each lane's slices in its own host thread and streams.
struct Lane {
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;               // second row group (run_pipeline)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // recorded on the stream of the last eval that used the workspace; every
    // eval makes its own stream wait on it first (ws_acquire), so a call on one
    // stream (the library's, a caller's, the null stream) never rewrites
    // buffers an earlier call on another stream is still reading
    hipEvent_t ev_free = nullptr;
    Workspace ws;
    // small host batches: the pipeline's launches captured once per batch shape
    // (the sentences' token offsets) and replayed as one graph launch
    // (run_host_pipeline); valid for one workspace generation and option state
    std::map<std::vector<int32_t>, hipGraphExec_t> graphs;
    uint64_t graphs_ws_gen = 0, graphs_opt_gen = 0;
};

struct Replica {
    int device = 0;
    std::vector<std::unique_ptr<Lane>> lanes;  // lanes[0] exists once built
    void *word = nullptr, *pos = nullptr, *type = nullptr;
    float *ln_e_w = nullptr, *ln_e_b = nullptr;
    std::vector<DevLayer> L;
    uint16_t *gelu_tab = nullptr, *exp_tab = nullptr, *gelu_compact = nullptr, *exp_compact = nullptr;
    std::vector<void *> weight_allocs;
    // profiling: events recorded around each launch when enabled
    bool prof = false;
    std::mutex prof_mu;  // lanes launch from several host threads
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
    std::map<std::string, ProfEntry> prof_acc;
};

int wtype_of(uint32_t ggml_type) {
    switch (ggml_type) {
        case GT_F32: return W_F32;
        case GT_F16: return W_F16;
        case GT_Q4_0: return W_Q4_0;
        case GT_Q4_1: return W_Q4_1;
    }
    return -1;
}

}  // namespace

struct bert_ctx {
    HParams hp;
    int wtype = 0;                      // kernels.h WType of the 2-D weights
    uint32_t word_t = 0, pos_t = 0, type_t = 0;
    std::vector<std::string> id_to_token;
    int32_t cls_id = 101, sep_id = 102, pad_id = 0;
    WordPieceTokenizer tokenizer;
    std::vector<std::unique_ptr<Replica>> reps;
    // which Q4 projections run on the int8-MFMA GEMMs (gemm_i8.hip; i8_select)
    bool i8_qkv = false, i8_o = false, i8_down = false, i8_up = false;
    // Q4_1 int8 GEMMs: scale products on the bf16 MFMA (kernels.h W_Q4_1B) or
    // the f32 MFMA (load option "q41bf"): 1 every int8
    // projection, 0 none, -1 (default) every one but the 384-wide FFN-down +
    // LN kernel (i8_ln384_kernel), where the bf16 part operands spill
    int q41bf = -1;
    // the fused QKV + attention kernel's form, fixed at load: 1 or 2 = the
    // head-pair kernel with that many 192-feature units per main loop (the tile
    // grouping of its QKV weight copy), 0 = the producer / consumer kernel on an
    // int8 head-major copy (Q4_0, head dim 32, n_embd 384); -1 (default) = 0
    // where it exists, else 2
    int qkva_ntw = -1;
    // run_pipeline knobs: defaults, then the load options (LoadOpts), then
    // bert_amd_set_option; nothing is read from the environment after load.
    // unfused: every batch on the QKV GEMM + attention pair (A/B checks);
    // two row groups on two streams (default on); fused-tile packing
    // -1 = when it pays (default), 0 = never, 1 = always; batches of fewer than
    // fuse_min sentences skip the fused QKV + attention kernel (one workgroup per
    // sentence: its latency, not the chip, bounds a small batch) for the unfused
    // pair, whose GEMM and attention spread a sentence over many workgroups
    int split = 1, pack = -1, fuse_min = 48;
    bool unfused = false;
    // batches of at most small_rows padded rows run the int8 GEMMs in their
    // 32-row-tile form (gemm_i8.hip i8_small_kernel: the same sums, spread over
    // many more workgroups; a one-sentence batch is 128 rows); 0 = never
    int small_rows = 2048;
    // host batches of at most graph_seqs sentences (and fewer than fuse_min, so
    // that the pipeline makes no host copy) replay a captured HIP graph of their
    // launches: one launch instead of ~33 per call; 0 = never (default: the
    // one-sentence call measured 327 us eager, 332 us replayed — the device's
    // ~4.5 us per dependent kernel bounds it, not the host's launches)
    int graph_seqs = 0;
    // the 384-wide LN kernel stores X with the nontemporal policy (GemmArgs
    // nt_x; not the last layer's, which pooling reads next): 1 (default) / 0
    int nt_x = 1;
    // small batches (<= 512 padded rows, every sentence <= 128 tokens; Q4_0 at
    // n_embd 384, head dim 32, int8 QKV): each head's QKV and attention in one
    // kernel (kernels.hip qkv_attention_small_kernel; bitwise the unfused pair)
    bool small_qkva = true;
    // load-time: the word-embedding table stays in its GGUF row format on the
    // device (Q4 rows dequantised in embed_ln_kernel as get_rows does, the same
    // f32 values as the load-time f32 copy; option emb_raw, default 1) instead
    // of f32 rows: MiniLM Q4_0's table 47 -> 6.6 MB, embed_ln 96-98 -> 90-92 us
    // on the headline batch (round 6, profiles/r06_embraw_ab.txt), bitwise equal
    bool emb_raw = true;
    uint64_t opt_gen = 0;  // bumped by every option change (captured graphs are dropped)
    // bert_encode_batch: slices evaluated at once per device (lanes), >= 1,
    // and consecutive slices a lane evaluates as one ragged batch (merge, >= 1),
    // merging only up to encode_merge_rows sentences (slices that large already
    // fill the chip alone): at most lanes x max(n_batch_size,
    // min(merge x n_batch_size, encode_merge_rows)) sentences in flight per
    // device.  Batch 16, 4096 texts of 8..128 tokens (bench consumer line):
    // lanes x merge 1 x 1 12 k emb/s, 4 x 1 35-56 k, 2 x 4 101 k, 4 x 4 109 k,
    // 8 x 4 92 k, 6 x 8 124 k, 4 x 8 173 k, 2 x 16 184 k (device-resident 265 k)
    int encode_lanes = 2, encode_merge = 16, encode_merge_rows = 256;
    std::mutex mu;  // one eval at a time per context (the reference ctx is not re-entrant either)
};

namespace {

template <typename T>
bool dmalloc(std::vector<void *> &track, T **p, size_t bytes) {
    void *q = nullptr;
    HIP_OK(hipMalloc(&q, bytes < 16 ? 16 : bytes));
    track.push_back(q);
    *p = (T *)q;
    return true;
}

// Weight staging for a load over one or more devices.  The host form of every
// device weight buffer (repack, repack_i8, table_f32: the costly part of a
// load) is made ONCE, by a recording pass over build_replica; then one host
// thread per device replays the same sequence of puts, allocating and copying
// on its own device, so N replicas cost one repack plus N concurrent uploads
// (reference bert.cpp:1065-1107: the replicas serve independent sentences).
struct StageBuf {
    std::vector<uint8_t> own;  // bytes made by the recording pass
    const void *ext = nullptr; // or host memory that outlives the load (GGUF data, tables())
    size_t n = 0;
    float unscale = 1.f;       // split-fp16 weights' 2^-S (kernels.h WPtr)
};
struct Stager {
    std::vector<StageBuf> *book = nullptr;  // shared; filled while recording, read-only on replay
    bool replay = false;
    size_t next = 0;                        // replay cursor (one Stager per replica)
    std::vector<void *> *track = nullptr;   // replay: the replica's allocations
    // record: make the bytes; replay: allocate on the current device and copy
    template <typename T, typename F>
    bool put(T **p, F make, float *unscale = nullptr) {
        if (!replay) {
            StageBuf b;
            make(b);
            b.n = b.ext ? b.n : b.own.size();
            book->push_back(std::move(b));
            return true;
        }
        if (next >= book->size()) {
            set_err("internal: weight staging replay out of step");
            return false;
        }
        const StageBuf &b = (*book)[next++];
        if (!dmalloc(*track, p, b.n)) return false;
        HIP_OK(hipMemcpy(*p, b.ext ? b.ext : b.own.data(), b.n, hipMemcpyHostToDevice));
        if (unscale) *unscale = b.unscale;
        return true;
    }
    // host memory that stays valid for the whole load: referenced, not copied
    template <typename T>
    bool put_ext(T **p, const void *src, size_t bytes) {
        return put(p, [&](StageBuf &b) {
            b.ext = src;
            b.n = bytes;
        });
    }
    // record: bytes of the vector get(*h) (h made once by the caller); replay: h is unused
    template <typename T, typename H, typename G>
    bool put_vec_or(T **p, const std::shared_ptr<H> &h, G get) {
        return put(p, [&](StageBuf &b) {
            const auto &v = get(*h);
            b.own.assign((const uint8_t *)v.data(), (const uint8_t *)(v.data() + v.size()));
        });
    }
    template <typename T, typename V>
    bool put_vec(T **p, const std::vector<V> &v) {  // record: a copy of v's bytes
        return put(p, [&](StageBuf &b) { b.own.assign((const uint8_t *)v.data(), (const uint8_t *)(v.data() + v.size())); });
    }
};

// Repack a [N][K] ggml-format matrix (given as row pointers) into MFMA
// fragment order (kernels.h WPtr).
struct Packed {
    std::vector<uint8_t> q;
    float unscale = 1.f;
};

Packed repack(uint32_t type, const std::vector<const uint8_t *> &rows_in, int64_t K) {
    const int64_t N = (int64_t)rows_in.size(), nkb = K / 32, ntl = N / 16;
    // column interleave (kernels.h WPtr): repacked tile 2p+t, lane column c
    // <- weight row 32p + 2c + t, i.e. repacked row 16*(2p+t) + c
    std::vector<const uint8_t *> rows((size_t)N);
    for (int64_t pr = 0; pr < N / 32; pr++)
        for (int t = 0; t < 2; t++)
            for (int c = 0; c < 16; c++) rows[(size_t)(32 * pr + 16 * t + c)] = rows_in[(size_t)(32 * pr + 2 * c + t)];
    Packed p;
    if (type == GT_Q4_0 || type == GT_Q4_1) {
        // w = d*(q-8) | d*q + m, exact in double; scaled by 2^S so that
        // max|w| lands in [2^13, 2^14): the fp16 hi part stays far from
        // overflow and the lo part stays normal for all but negligible weights
        const int bs = type == GT_Q4_0 ? 18 : 20, qoff = type == GT_Q4_0 ? 2 : 4;
        auto wval = [&](const uint8_t *row, int64_t k) -> double {
            const uint8_t *blk = row + (k >> 5) * bs;
            const int e = (int)(k & 31);
            const uint8_t byte = blk[qoff + (e & 15)];
            const int qv = e < 16 ? (byte & 15) : (byte >> 4);
            uint16_t dh, mh;
            std::memcpy(&dh, blk, 2);
            const double d = f16_to_f32(dh);
            if (type == GT_Q4_0) return d * (qv - 8);
            std::memcpy(&mh, blk + 2, 2);
            return d * qv + (double)f16_to_f32(mh);
        };
        double amax = 0.0;
        for (int64_t n = 0; n < N; n++)
            for (int64_t kb = 0; kb < nkb; kb++) {
                const uint8_t *blk = rows[(size_t)n] + kb * bs;
                uint16_t dh, mh = 0;
                std::memcpy(&dh, blk, 2);
                if (type == GT_Q4_1) std::memcpy(&mh, blk + 2, 2);
                const double d = std::fabs((double)f16_to_f32(dh)), m = (double)f16_to_f32(mh);
                amax = std::max(amax, type == GT_Q4_0 ? 8.0 * d : std::max(std::fabs(m), std::fabs(m + 15.0 * d)));
            }
        int S = 0;
        if (amax > 0.0) {
            int e2;
            std::frexp(amax, &e2);  // amax in [2^(e2-1), 2^e2)
            S = 14 - e2;
        }
        const double scale = std::ldexp(1.0, S);
        p.unscale = (float)std::ldexp(1.0, -S);
        p.q.resize((size_t)N * K * 4);
        uint16_t *q = (uint16_t *)p.q.data();
        for (int64_t nt = 0; nt < ntl; nt++)
            for (int64_t kb = 0; kb < nkb; kb++)
                for (int lane = 0; lane < 64; lane++) {
                    const int c = lane & 15, g = lane >> 4;
                    uint16_t *hi = &q[(((nt * nkb + kb) * 2 + 0) * 64 + lane) * 8];
                    uint16_t *lo = &q[(((nt * nkb + kb) * 2 + 1) * 64 + lane) * 8];
                    for (int j = 0; j < 8; j++) {
                        const double w = wval(rows[(size_t)(nt * 16 + c)], kb * 32 + 8 * g + j) * scale;
                        hi[j] = f32_to_f16((float)w);
                        lo[j] = f32_to_f16((float)(w - (double)f16_to_f32(hi[j])));
                    }
                }
    } else if (type == GT_F16) {
        p.q.resize((size_t)N * K * 2);
        uint16_t *q = (uint16_t *)p.q.data();
        for (int64_t nt = 0; nt < ntl; nt++)
            for (int64_t kb = 0; kb < nkb; kb++)
                for (int lane = 0; lane < 64; lane++) {
                    const int c = lane & 15, g = lane >> 4;
                    const uint16_t *src = (const uint16_t *)rows[nt * 16 + c] + kb * 32 + 8 * g;
                    std::memcpy(&q[((nt * nkb + kb) * 64 + lane) * 8], src, 16);
                }
    } else {
        p.q.resize((size_t)N * K * 4);
        float *q = (float *)p.q.data();
        for (int64_t nt = 0; nt < ntl; nt++)
            for (int64_t kb = 0; kb < nkb; kb++)
                for (int lane = 0; lane < 64; lane++) {
                    const int c = lane & 15, g = lane >> 4;
                    const float *src = (const float *)rows[nt * 16 + c] + kb * 32;
                    float *dst = &q[((nt * nkb + kb) * 64 + lane) * 8];
                    for (int cc = 0; cc < 2; cc++)
                        for (int j = 0; j < 4; j++) dst[cc * 4 + j] = src[16 * cc + 4 * g + j];
                }
    }
    return p;
}

struct I8Host {
    std::vector<int8_t> q;
    std::vector<float> d, m;
    std::vector<uint16_t> dh;
};

I8Host repack_i8(uint32_t type, const std::vector<const uint8_t *> &rows, int64_t K) {
    const int64_t N = (int64_t)rows.size(), nkb = K / 32, nft = N / 32;
    const bool q1 = type == GT_Q4_1;
    const int bs = q1 ? 20 : 18, qoff = q1 ? 4 : 2;
    auto perm = [](int m) { return 16 * ((m >> 2) & 1) + 4 * (m >> 3) + (m & 3); };
    I8Host h;
    h.q.resize((size_t)(N * K));
    h.d.resize((size_t)(N * nkb));
    h.m.resize(q1 ? (size_t)(N * nkb) : 0);
    h.dh.resize(q1 ? 0 : (size_t)(N * nkb));
    for (int64_t ft = 0; ft < nft; ft++)
        for (int64_t b = 0; b < nkb; b++)
            for (int lane = 0; lane < 64; lane++) {
                const int mrow = lane & 31, hf = lane >> 5;
                const uint8_t *blk = rows[(size_t)(32 * ft + perm(mrow))] + b * bs;
                int8_t *dst = &h.q[(size_t)(((ft * nkb + b) * 64 + lane) * 16)];
                for (int j = 0; j < 16; j++) {
                    const int e = 16 * hf + j;
                    const uint8_t byte = blk[qoff + (e & 15)];
                    const int v = e < 16 ? (byte & 15) : (byte >> 4);
                    dst[j] = (int8_t)(q1 ? v : v - 8);
                }
            }
    for (int64_t ft = 0; ft < nft; ft++)
        for (int64_t g = 0; g < nkb / 4; g++)
            for (int mrow = 0; mrow < 32; mrow++)
                for (int jj = 0; jj < 4; jj++) {
                    const uint8_t *blk = rows[(size_t)(32 * ft + perm(mrow))] + (4 * g + jj) * bs;
                    uint16_t dh, mh;
                    std::memcpy(&dh, blk, 2);
                    const size_t at = (size_t)(((ft * (nkb / 4) + g) * 32 + mrow) * 4 + jj);
                    h.d[at] = f16_to_f32(dh);
                    if (!q1) h.dh[at] = dh;
                    if (q1) {
                        std::memcpy(&mh, blk + 2, 2);
                        h.m[at] = f16_to_f32(mh);
                    }
                }
    return h;
}

// Repack a Q4_0 / Q4_1 [N][K] matrix for the int8-MFMA GEMMs (kernels.h
// I8W): nibbles expanded to int8 (q - 8 for Q4_0, q for Q4_1) in fragment
// order, the fp16 block scales (and Q4_1 minima) widened to f32 vectors.
// Weight row m of each 32-row tile holds feature perm(m), so that a lane of
// the 32x32 MFMA result holds 16 consecutive output features.  Staged as up
// to four buffers (q, d, m, dh); the repack runs once, while recording.
bool stage_i8(Stager &S, I8W &w, uint32_t type, const std::vector<const uint8_t *> &rows, int64_t K) {
    std::shared_ptr<I8Host> h;
    if (!S.replay) h = std::make_shared<I8Host>(repack_i8(type, rows, K));
    const bool q1 = type == GT_Q4_1;
    void *pq = nullptr, *pd = nullptr, *pm = nullptr, *ph = nullptr;
    if (!S.put_vec_or(&pq, h, [](const I8Host &x) -> const auto & { return x.q; }) ||
        !S.put_vec_or(&pd, h, [](const I8Host &x) -> const auto & { return x.d; }))
        return false;
    if (q1 && !S.put_vec_or(&pm, h, [](const I8Host &x) -> const auto & { return x.m; })) return false;
    if (!q1 && !S.put_vec_or(&ph, h, [](const I8Host &x) -> const auto & { return x.dh; })) return false;
    w.q = (const int8_t *)pq;
    w.d = (const float *)pd;
    w.m = (const float *)pm;
    w.dh = (const uint16_t *)ph;
    return true;
}

// A split-fp16 / f16 / f32 weight matrix in MFMA fragment order (repack, run
// once while recording).
template <typename F>
bool stage_packed(Stager &S, WPtr &w, F make_packed) {
    void *q = nullptr;
    float unscale = 1.f;
    if (!S.put(&q, [&](StageBuf &b) {
            Packed p = make_packed();
            b.own = std::move(p.q);
            b.unscale = p.unscale;
        }, &unscale))
        return false;
    w.q = q;
    w.unscale = unscale;
    return true;
}

std::vector<const uint8_t *> rows_of(const GGUFTensor *t) {
    const size_t rb = ggml_row_bytes(t->type, t->ne[0]);
    std::vector<const uint8_t *> r((size_t)t->ne[1]);
    for (int64_t i = 0; i < t->ne[1]; i++) r[(size_t)i] = t->data + (size_t)i * rb;
    return r;
}

// activation format (ggml's vec_dot_type of the weights, kernels.h WType) of
// a row of K values: element / block-scale bytes
size_t act_row_bytes(int at, int64_t K) { return (size_t)K * (at == W_F32 ? 4 : at == W_F16 ? 2 : 1); }
size_t act_scale_bytes(int at) { return at == W_Q4_0 ? 2 : at == W_Q4_1 ? 4 : 0; }

// Activation buffers carry GEMM_BM spare rows: qkv_attention_kernel reads the
// 128-row tile starting at each sentence's first token (rows past M are
// zero-filled and masked).
// The zero fill is enqueued on `st`, the stream whose kernels use the buffer
// (a plain hipMemset goes to the null stream, which does not order with the
// library's non-blocking streams: the first batch on a fresh workspace could
// race it).
bool alloc_act(std::vector<void *> &track, ActPtr &a, int wtype, int64_t rows, int64_t K, hipStream_t st) {
    rows += GEMM_BM;
    if (!dmalloc(track, &a.q, (size_t)rows * act_row_bytes(wtype, K))) return false;
    HIP_OK(hipMemsetAsync(a.q, 0, (size_t)rows * act_row_bytes(wtype, K), st));
    if (act_scale_bytes(wtype)) {
        if (!dmalloc(track, &a.d, (size_t)rows * (K / 32) * act_scale_bytes(wtype))) return false;
        HIP_OK(hipMemsetAsync(a.d, 0, (size_t)rows * (K / 32) * act_scale_bytes(wtype), st));
    }
    return true;
}

// Grows the workspace to Mpad rows / n_seqs sentences.  The old buffers may
// still be in use on any stream of the device (the library's or a caller's),
// so the device is drained before they are freed; the zero-fill of the new
// ones is issued on `st`, the stream the kernels that use them run on.
bool ensure_workspace(bert_ctx *ctx, Lane &ln, int64_t Mpad, int64_t n_seqs, hipStream_t st) {
    Workspace &w = ln.ws;
    if (Mpad <= w.cap_rows && n_seqs <= w.cap_seqs) return true;
    HIP_OK(hipDeviceSynchronize());
    const int64_t rows = std::max<int64_t>(Mpad, w.cap_rows), seqs = std::max<int64_t>(n_seqs, w.cap_seqs);
    for (void *p : w.allocs) hipFree(p);
    w.allocs.clear();
    // until every allocation below has succeeded the workspace is empty
    // (a failed grow must not leave capacities that point at freed memory)
    w.cap_rows = w.cap_seqs = 0;
    w.X = w.out = nullptr;
    w.qk_hi = w.qk_lo = w.vt_hi = w.vt_lo = nullptr;
    w.Xa = w.Ca = w.Ua = ActPtr{};
    w.tok = w.off = w.rowpos = w.tiles = w.perm = nullptr;
    const int64_t E = ctx->hp.n_embd, I = ctx->hp.n_intermediate;
    const int at = ctx->wtype;
    if (!dmalloc(w.allocs, &w.X, (size_t)rows * E * 4) || !dmalloc(w.allocs, &w.qk_hi, (size_t)rows * 2 * E * 2) ||
        !dmalloc(w.allocs, &w.qk_lo, (size_t)rows * 2 * E * 2) || !dmalloc(w.allocs, &w.vt_hi, (size_t)rows * E * 2) ||
        !dmalloc(w.allocs, &w.vt_lo, (size_t)rows * E * 2) ||
        !alloc_act(w.allocs, w.Xa, ctx->wtype, rows, E, st) || !alloc_act(w.allocs, w.Ca, at, rows, E, st) ||
        !alloc_act(w.allocs, w.Ua, at, rows, I, st) || !dmalloc(w.allocs, &w.out, (size_t)seqs * E * 4) ||
        !dmalloc(w.allocs, &w.tok, (size_t)rows * 4) || !dmalloc(w.allocs, &w.off, (size_t)(seqs + 1) * 4) ||
        !dmalloc(w.allocs, &w.rowpos, (size_t)rows * 4) || !dmalloc(w.allocs, &w.tiles, (size_t)seqs * 2 * 4) ||
        !dmalloc(w.allocs, &w.perm, (size_t)seqs * 4))
        return false;
    // padding rows must hold finite values: zero everything once
    HIP_OK(hipMemsetAsync(w.X, 0, (size_t)rows * E * 4, st));
    HIP_OK(hipMemsetAsync(w.qk_hi, 0, (size_t)rows * 2 * E * 2, st));
    HIP_OK(hipMemsetAsync(w.qk_lo, 0, (size_t)rows * 2 * E * 2, st));
    HIP_OK(hipMemsetAsync(w.vt_hi, 0, (size_t)rows * E * 2, st));
    HIP_OK(hipMemsetAsync(w.vt_lo, 0, (size_t)rows * E * 2, st));
    w.cap_rows = rows;
    w.cap_seqs = seqs;
    w.gen++;
    return true;
}

// ---- profiling helpers
struct Launch {
    Replica &R;
    hipStream_t s;
    const char *name;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    Launch(Replica &r, hipStream_t st, const char *n) : R(r), s(st), name(n) {
        if (R.prof) {
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0, s);
        }
    }
    ~Launch() {
        if (R.prof) {
            hipEventRecord(e1, s);
            std::lock_guard<std::mutex> lk(R.prof_mu);
            R.pending.push_back({name, {e0, e1}});
        }
    }
};

void drain_profile(Replica &R) {
    std::lock_guard<std::mutex> lk(R.prof_mu);
    for (auto &p : R.pending) {
        hipEventSynchronize(p.second.second);
        float ms = 0;
        hipEventElapsedTime(&ms, p.second.first, p.second.second);
        auto &e = R.prof_acc[p.first];
        e.ms += ms;
        e.n += 1;
        hipEventDestroy(p.second.first);
        hipEventDestroy(p.second.second);
    }
    R.pending.clear();
}

void clear_graphs(Lane &ln) {
    for (auto &g : ln.graphs) hipGraphExecDestroy(g.second);
    ln.graphs.clear();
}

// Workspace hand-over between evals (Replica::ev_free): an eval's first
// device operation waits for the previous eval's last one, whatever streams
// the two ran on; the eval records the event behind its own last operation.
bool ws_acquire(Lane &ln, hipStream_t st) {
    HIP_OK(hipStreamWaitEvent(st, ln.ev_free, 0));
    return true;
}
bool ws_release(Lane &ln, hipStream_t st) {
    HIP_OK(hipEventRecord(ln.ev_free, st));
    return true;
}

#define LAUNCH_OK(name, expr) LAUNCH_ON(name, st, expr)
#define LAUNCH_ON(name, stream, expr)                                                     \
    do {                                                                                  \
        Launch lp_(R, stream, name);                                                      \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) {                                                           \
            set_err("kernel %s launch failed: %s", name, hipGetErrorString(e_));          \
            return false;                                                                 \
        }                                                                                 \
    } while (0)

// Q4 models run selected projections on the int8-MFMA GEMMs (gemm_i8.hip:
// 1 B/weight, exact isum per block on the int8 MFMA, d_w * d_a applied in
// the kernel like ggml's vec_dot).  Default: FFN-up (faster than the
// split-fp16 GEMM) and FFN-down (as fast on full batches, faster on ragged
// ones) where its LayerNorm is fused (n_embd 384); the O projection too for
// Q4_0 at n_embd 384 (batch within noise of the split-fp16 GEMM, one sentence
// 15-20 us faster: its 32-row int8 tiles stream a quarter of the bytes; round
// 6), elsewhere it stays on the split-fp16 GEMM.  `v` (load option "i8", env
// BERT_AMD_I8): "0" none, "1" / "all" all three, or a list of up, o, down
// separated by '+' or ','; empty: the default.
void i8_select(bert_ctx *ctx, const std::string &spec) {
    // (the down GEMM only where its LayerNorm is fused, E = 384: wider rows use
    // the int8 residual kernel + launch_ln, 8 % slower than split-fp16 on C5)
    std::string v = spec.empty() ? (ctx->hp.n_embd == 384 ? (ctx->wtype == W_Q4_0 ? "up,down,o" : "up,down") : "up")
                                 : spec;
    std::replace(v.begin(), v.end(), '+', ',');
    const int E = ctx->hp.n_embd, I = ctx->hp.n_intermediate;
    const bool q4 = ctx->wtype == W_Q4_0 || ctx->wtype == W_Q4_1;
    const int ln = E == 384 ? EPI_LN : EPI_RESID;
    const bool all = v == "1" || v == "all";
    auto has = [&](const char *p) {
        const std::string t = std::string(",") + v + ",";
        return all || t.find(std::string(",") + p + ",") != std::string::npos;
    };
    // qkv: the unfused QKV GEMM on the int8 copy (as the producer / consumer
    // kernel's twin); the head-pair fused kernel has no int8 form, so a model
    // that would use it runs every batch on the unfused pair instead (the
    // results of a sentence must not depend on its batch)
    ctx->i8_qkv = q4 && (ctx->qkva_ntw == 0 || has("qkv")) && i8_gemm_supported(EPI_QKV, 3 * E, E);
    ctx->i8_up = q4 && has("up") && i8_gemm_supported(EPI_GELU_ACT, I, E);
    ctx->i8_o = q4 && has("o") && i8_gemm_supported(ln, E, E);
    ctx->i8_down = q4 && has("down") && i8_gemm_supported(ln, E, I);
}

// One encoder layer over the row group [row0, row0 + rows) (sentences
// d_off[0 .. nseq), absolute row offsets).  Xa / Ca / Ua / X point at the
// group's first row; the QKV + attention kernels index rows absolutely through
// the offsets, so they get the workspace bases (the unfused pair only runs
// with one group, row0 == 0).
// the fused small QKV + attention kernel computes a head's 3 x ceil(n / 32)
// QKV tiles on one workgroup: it wins for one sentence of 16 tokens (271 vs
// 286-314 us per call), not at 128 (311-314 vs 300-320): tools/opt_latency_ab.sh
#ifndef QKVA_SMALL_MAX_LEN
#define QKVA_SMALL_MAX_LEN 64
#endif
#ifndef QKVA_SMALL_ROWS  // (and the batch small: rows <= small_rows) — it wins at every
#define QKVA_SMALL_ROWS 2048  // small size, tools/qkva_batch_probe.py (16 x 48 tokens 450 vs 500 us)
#endif
// Q4_1's scale products on the bf16 MFMA for this int8 epilogue (option q41bf):
// by default everywhere but the 384-wide FFN-down + LN kernel (measured, round
// 6: C5 FFN-up 8.78 -> 7.62 ms, MiniLM Q4_1 FFN-up 366 -> 326 us, but its
// i8_ln384 FFN-down 366 -> 443 us)
static bool q41bf_for(int opt, int epi) { return opt > 0 || (opt < 0 && epi != EPI_LN); }

bool run_layer(bert_ctx *ctx, Replica &R, Lane &ln, int il, int64_t row0, int64_t rows, const int32_t *d_off, int nseq,
               const int32_t *d_tiles, int ntiles, int max_len, bool fused_qkv_attn, bool ln_fused, ActPtr Xa,
               ActPtr Ca, ActPtr Ua, float *X, hipStream_t st) {
    const HParams &hp = ctx->hp;
    Workspace &w = ln.ws;
    const int E = hp.n_embd, I = hp.n_intermediate, H = hp.n_head, D = E / H, wt = ctx->wtype;
    // the int8 GEMMs' weight form per epilogue (the same for the batch and the
    // small-batch kernels, so their results stay bitwise equal)
    auto wt8 = [&](int epi) { return wt == W_Q4_1 && q41bf_for(ctx->q41bf, epi) ? W_Q4_1B : wt; };
    // small batches: the int8 GEMMs in 32-row tiles (bitwise the same results)
    const bool small = rows <= ctx->small_rows;
    auto gemm_i8 = [&](int epi, const GemmArgs &a) {
        return small ? launch_gemm_i8_small(wt8(epi), epi, a, (int)rows, st)
                     : launch_gemm_i8(wt8(epi), epi, a, (int)rows, st);
    };
    if (!fused_qkv_attn && row0 != 0) {
        set_err("internal: unfused attention with a row split");
        return false;
    }
    {
        const DevLayer &L = R.L[il];
        GemmArgs q;
        q.A = w.Xa;
        q.K = E;
        q.W = L.qkv;
        q.N = 3 * E;
        q.bias = L.b_qkv;
        q.head_dim = D;
        q.qk_hi = w.qk_hi;
        q.qk_lo = w.qk_lo;
        q.vt_hi = w.vt_hi;
        q.vt_lo = w.vt_lo;
        q.ldv = w.cap_rows;
        AttnArgs aa;
        aa.qk_hi = w.qk_hi;
        aa.qk_lo = w.qk_lo;
        aa.vt_hi = w.vt_hi;
        aa.vt_lo = w.vt_lo;
        aa.ldv = w.cap_rows;
        aa.offsets = d_off;
        aa.E = E;
        aa.H = H;
        aa.scale = 1.0f / sqrtf((float)D);
        aa.expt = half_table(R.exp_tab, R.exp_compact, tables().exp_c);
        aa.ctx = w.Ca;
        if (fused_qkv_attn) {
            GemmArgs qf = q;
            qf.W = L.qkv_plain;
            aa.tiles = ntiles < nseq ? d_tiles : nullptr;  // no tile holds two sentences: plain kernel
            qf.Wi = L.qkv8;  // (qkva_ntw 0)
            LAUNCH_OK("qkv_attention", launch_qkv_attention(wt, qf, aa, ntiles, ctx->qkva_ntw, st));
        } else if (ctx->i8_qkv && ctx->small_qkva && !ctx->unfused && small && wt == W_Q4_0 && E == 384 && D == 32 &&
                   max_len <= QKVA_SMALL_MAX_LEN && rows <= QKVA_SMALL_ROWS) {
            // one sentence (the server's path): the head's QKV and attention in one kernel
            q.Wi = L.qkv8;
            LAUNCH_OK("qkv_attention", launch_qkv_attention_small(q, aa, nseq, st));
        } else if (ctx->i8_qkv) {  // the int8 QKV of the producer / consumer kernel, unfused
            q.Wi = L.qkv8;
            LAUNCH_OK("gemm_qkv", gemm_i8(EPI_QKV, q));
            LAUNCH_OK("attention", launch_attention(wt, D, aa, nseq, max_len, st));
        } else {
            LAUNCH_OK("gemm_qkv", launch_gemm(wt, EPI_QKV, 0, q, (int)rows, st));
            LAUNCH_OK("attention", launch_attention(wt, D, aa, nseq, max_len, st));
        }
        GemmArgs o;
        o.A = Ca;
        o.K = E;
        o.W = L.o;
        o.N = E;
        o.bias = L.b_o;
        o.X = X;
        o.out_act = Xa;
        o.ln_w = L.ln1_w;
        o.ln_b = L.ln1_b;
        o.eps = hp.eps;
        // small batches: the int8 O + LN is the 32-row residual GEMM, then the
        // LayerNorm pass as a launch of its own (counted as one in the profile)
        o.defer_ln = small;
        o.nt_x = ctx->nt_x;
        if (ctx->i8_o) {
            o.Wi = L.o8;
            if (E == 384) {
                LAUNCH_OK("gemm_o_ln", gemm_i8(EPI_LN, o));
                if (small) LAUNCH_OK("ln", launch_ln384_rows_i8(wt8(EPI_LN), o, (int)rows, st));
            } else {
                LAUNCH_OK("gemm_o_ln", gemm_i8(EPI_RESID, o));
                LAUNCH_OK("ln", launch_ln(wt, X, (int)rows, E, L.ln1_w, L.ln1_b, hp.eps, Xa, st));
            }
        } else if (ln_fused) {
            LAUNCH_OK("gemm_o_ln", launch_gemm(wt, EPI_LN, 0, o, (int)rows, st));
        } else {
            LAUNCH_OK("gemm_o_ln", launch_gemm(wt, EPI_RESID, 0, o, (int)rows, st));
            LAUNCH_OK("ln", launch_ln(wt, X, (int)rows, E, L.ln1_w, L.ln1_b, hp.eps, Xa, st));
        }

        GemmArgs u;
        u.A = Xa;
        u.K = E;
        u.W = L.up;
        u.N = I;
        u.bias = L.b_up;
        u.out_act = Ua;
        u.gelu = half_table(R.gelu_tab, R.gelu_compact, tables().gelu_c);
        u.gelu.n_pad = (int)tables().gelu_pair.size();  // the pair view (kernels.hip gelu_lookup)
        u.gelu.cap = tables().gelu_cap;
        GemmArgs dn;
        dn.A = Ua;
        dn.K = I;
        dn.W = L.down;
        dn.N = E;
        dn.bias = L.b_down;
        dn.X = X;
        dn.out_act = Xa;
        dn.ln_w = L.ln2_w;
        dn.ln_b = L.ln2_b;
        dn.eps = hp.eps;
        dn.defer_ln = small;  // (as O)
        dn.nt_x = ctx->nt_x && il + 1 < ctx->hp.n_layer;  // the last layer's X: pooling reads it next
        if (ctx->i8_up) {
            u.Wi = L.up8;
            LAUNCH_OK("gemm_up_gelu", gemm_i8(EPI_GELU_ACT, u));
        } else {
            LAUNCH_OK("gemm_up_gelu", launch_gemm(wt, EPI_GELU_ACT, 0, u, (int)rows, st));
        }

        if (ctx->i8_down) {
            dn.Wi = L.down8;
            if (E == 384) {
                LAUNCH_OK("gemm_down_ln", gemm_i8(EPI_LN, dn));
                if (small) LAUNCH_OK("ln", launch_ln384_rows_i8(wt8(EPI_LN), dn, (int)rows, st));
            } else {
                LAUNCH_OK("gemm_down_ln", gemm_i8(EPI_RESID, dn));
                LAUNCH_OK("ln", launch_ln(wt, X, (int)rows, E, L.ln2_w, L.ln2_b, hp.eps, Xa, st));
            }
        } else if (ln_fused) {
            LAUNCH_OK("gemm_down_ln", launch_gemm(wt, EPI_LN, 0, dn, (int)rows, st));
        } else {
            LAUNCH_OK("gemm_down_ln", launch_gemm(wt, EPI_RESID, 0, dn, (int)rows, st));
            LAUNCH_OK("ln", launch_ln(wt, X, (int)rows, E, L.ln2_w, L.ln2_b, hp.eps, Xa, st));
        }
    }
    return true;
}

// embed_ln's arguments for a batch resident in the replica's workspace
EmbedArgs embed_args(const bert_ctx *ctx, Replica &R, const Workspace &w, const int32_t *d_tok, const int32_t *d_off, int n_seqs,
                     int64_t M) {
    const HParams &hp = ctx->hp;
    EmbedArgs ea;
    ea.tokens = d_tok;
    ea.offsets = d_off;
    ea.rowpos = w.rowpos;
    ea.n_seqs = n_seqs;
    ea.M = (int)M;
    ea.E = hp.n_embd;
    ea.n_vocab = hp.n_vocab;
    ea.n_pos = hp.n_max_tokens;
    ea.word = R.word;
    ea.pos = R.pos;
    ea.type = R.type;
    ea.word_t = ea.pos_t = ea.type_t = W_F32;  // the replica holds f32 copies (table_f32)
    if (ctx->emb_raw) ea.word_t = (int)ctx->word_t;  // ... or the word table's own rows (emb_raw)
    ea.ln_w = R.ln_e_w;
    ea.ln_b = R.ln_e_b;
    ea.eps = hp.eps;
    ea.X = w.X;
    ea.Xa = w.Xa;
    return ea;
}

// Test tap (bert_amd_debug_layers): device buffers receiving the residual
// stream X and its Q8 / fp16 activation form Xa after every stage (stage 0 =
// embeddings + LN, stage l + 1 = encoder layer l), M rows each.
struct DebugTap {
    float *X = nullptr;
    char *q = nullptr, *d = nullptr;
};

// The fixed pipeline over a ragged batch already resident on the device.
// d_out_row (optional): output row of each sentence of the batch.
bool run_pipeline(bert_ctx *ctx, Replica &R, Lane &ln, const int32_t *d_tok, const int32_t *d_off, const int32_t *h_off,
                  int n_seqs, float *d_out, hipStream_t st, const int32_t *d_out_row = nullptr,
                  const DebugTap *tap = nullptr) {
    const HParams &hp = ctx->hp;
    const int64_t M = h_off[n_seqs];
    const int64_t Mpad = std::max<int64_t>(GEMM_BM, (M + GEMM_BM - 1) / GEMM_BM * GEMM_BM);
    int max_len = 0;
    for (int s = 0; s < n_seqs; s++) max_len = std::max(max_len, h_off[s + 1] - h_off[s]);
    if (!ensure_workspace(ctx, ln, Mpad, n_seqs, st)) return false;
    Workspace &w = ln.ws;
    const int E = hp.n_embd, I = hp.n_intermediate, H = hp.n_head, wt = ctx->wtype;
    const bool ln_fused = gemm_ln_fused(wt, E);
    // QKV + attention in one kernel when every sentence fits one 128-row tile
    // (option "unfused" forces the two-kernel path, for A/B checks)
    // (an int8 QKV copy without the producer / consumer kernel, i8 qkv: the
    // head-pair kernel has no int8 form, so every batch takes the unfused pair)
    // Small batches of short sentences take qkv_attention_small_kernel (run_layer)
    // whatever their count: one workgroup per (head, sentence) against the
    // producer / consumer kernel's one per 128-row tile (48 x 16 tokens: 575 vs
    // 856 us per call, tools/fuse_min_probe.py)
    const bool small_short = ctx->small_qkva && ctx->i8_qkv && !ctx->unfused && Mpad <= ctx->small_rows &&
                             Mpad <= QKVA_SMALL_ROWS && max_len <= QKVA_SMALL_MAX_LEN && wt == W_Q4_0 && E == 384 &&
                             E / H == 32 && !tap;
    const bool fused_qkv_attn = !ctx->unfused && n_seqs >= ctx->fuse_min && (!ctx->i8_qkv || ctx->qkva_ntw == 0) &&
                                qkv_attention_supported(wt, E, H, max_len, ctx->qkva_ntw) && !small_short;

    const EmbedArgs ea = embed_args(ctx, R, w, d_tok, d_off, n_seqs, M);
    LAUNCH_OK("embed_ln", launch_embed(ctx->wtype, ea, (int)Mpad, st));
    auto tap_stage = [&](int stage) {
        if (!tap) return true;
        const size_t xb = (size_t)M * E * 4, qb = (size_t)M * act_row_bytes(wt, E), db = (size_t)M * (E / 32) * act_scale_bytes(wt);
        HIP_OK(hipMemcpyAsync(tap->X + (size_t)stage * M * E, w.X, xb, hipMemcpyDeviceToDevice, st));
        HIP_OK(hipMemcpyAsync(tap->q + (size_t)stage * qb, w.Xa.q, qb, hipMemcpyDeviceToDevice, st));
        if (db) HIP_OK(hipMemcpyAsync(tap->d + (size_t)stage * db, w.Xa.d, db, hipMemcpyDeviceToDevice, st));
        return true;
    };
    if (!tap_stage(0)) return false;

    // Row groups (default; ctx->split = 0 turns them off):
    // with the fused QKV + attention path the batch is split at a 128-row-aligned
    // sentence boundary near M / 2 and the two halves run their layers on two
    // streams, so one half's LayerNorm GEMMs and VALU-bound FFN-up can overlap
    // the other half's MFMA-heavy fused kernel, and batches too small to fill
    // the GPU with one kernel at a time fill it with two.  Groups own disjoint
    // rows of every buffer; sentences never span groups, so results are
    // identical.  Measured (tools/ab_bench.sh, round 2): 1024 x 128 -0.6..+1.9 %,
    // 8..128-token batch +4.6 %, 8..40-token batch +20 %.  Per-kernel profiles
    // (bench.py's event pass, tools/profile_round.sh) run with the split off
    // (bert_amd_set_option "split" 0, or BERT_AMD_SPLIT=0 at load) so that
    // every launch is the whole batch.
    struct Group {
        int64_t row0, rows;  // rows: 128-multiple
        int seq0, nseq;
        hipStream_t s;
    };
    Group G[2] = {{0, Mpad, 0, n_seqs, st}, {0, 0, 0, 0, nullptr}};
    int ng = 1;
    if (ctx->split && !tap && fused_qkv_attn && ln_fused && n_seqs >= 512 && ln.stream2) {
        int best = -1;
        for (int s = 1; s < n_seqs; s++)
            if (h_off[s] % GEMM_BM == 0 &&
                (best < 0 || std::llabs(2LL * h_off[s] - M) < std::llabs(2LL * h_off[best] - M)))
                best = s;
        if (best > 0 && 4LL * h_off[best] >= M && 4LL * h_off[best] <= 3 * M) {
            G[0] = {0, h_off[best], 0, best, st};
            G[1] = {h_off[best], Mpad - h_off[best], best, n_seqs - best, ln.stream2};
            ng = 2;
            HIP_OK(hipEventRecord(ln.ev_fork, st));
            HIP_OK(hipStreamWaitEvent(ln.stream2, ln.ev_fork, 0));
        }
    }
    // Sentence tiles for the fused kernel: consecutive sentences packed greedily
    // into one workgroup while their lengths rounded up to 32 sum to <= 128
    // (kernels.hip qkv_attention_kernel: each keeps its own 32-query blocks and
    // 32-aligned keys, so short sentences share the GEMM rows and the
    // workgroup without changing a bit of their results).
    int ntl[2] = {0, 0};
    if (fused_qkv_attn) {
        std::vector<int32_t> &ht = w.h_tiles;
        ht.assign((size_t)2 * n_seqs, 0);
        auto span = [&](int s) { return (h_off[s + 1] - h_off[s] + 31) & ~31; };
        // ctx->pack (A/B and tests): 0 never packs, 1 always, -1 when it pays
        const bool no_pack = ctx->pack == 0, force_pack = ctx->pack == 1;
        for (int gi = 0; gi < ng; gi++) {
            int32_t *t = ht.data() + 2 * G[gi].seq0;
            for (int s = G[gi].seq0, e = G[gi].seq0 + G[gi].nseq; s < e;) {
                int k = s + 1, used = span(s);
                while (!no_pack && k < e && used + span(k) <= GEMM_BM) used += span(k++);
                // the packed kernel's contract (kernels.hip qkv_attention_kernel returns
                // without writing on a tile of more than 4 sentences or 128 rows)
                if (k - s > 4 || used > GEMM_BM) {
                    set_err("internal: sentence tile of %d sentences / %d rows", k - s, used);
                    return false;
                }
                t[2 * ntl[gi]] = s - G[gi].seq0;
                t[2 * ntl[gi] + 1] = k - s;
                ntl[gi]++;
                s = k;
            }
            if (!force_pack && !qkv_attention_pack_pays(G[gi].nseq, ntl[gi])) ntl[gi] = G[gi].nseq;  // plain kernel
        }
        // pageable source: the copy is staged before the call returns, so ht may be reused.
        // Only packed groups read the table (run_layer: tiles = nullptr when every
        // tile is one sentence), so a batch with none skips the upload
        bool packs = false;
        for (int gi = 0; gi < ng; gi++) packs |= ntl[gi] < G[gi].nseq;
        if (packs) HIP_OK(hipMemcpyAsync(w.tiles, ht.data(), (size_t)2 * n_seqs * 4, hipMemcpyHostToDevice, st));
        if (ng == 2) {
            HIP_OK(hipEventRecord(ln.ev_fork, st));
            HIP_OK(hipStreamWaitEvent(ln.stream2, ln.ev_fork, 0));
        }
    }
    auto act_rows = [&](ActPtr a, int at, int64_t row0, int64_t K) {
        if (!a.q) return a;
        a.q = (char *)a.q + row0 * (int64_t)act_row_bytes(at, K);
        if (a.d) a.d = (char *)a.d + row0 * (K / 32) * (int64_t)act_scale_bytes(at);
        return a;
    };
    for (int il = 0; il < hp.n_layer; il++) {
        for (int gi = 0; gi < ng; gi++) {
            const Group &gr = G[gi];
            if (!run_layer(ctx, R, ln, il, gr.row0, gr.rows, d_off + gr.seq0, gr.nseq, w.tiles + 2 * gr.seq0, ntl[gi],
                           max_len, fused_qkv_attn, ln_fused, act_rows(w.Xa, wt, gr.row0, E),
                           act_rows(w.Ca, wt, gr.row0, E), act_rows(w.Ua, wt, gr.row0, I), w.X + gr.row0 * E, gr.s))
                return false;
        }
        if (!tap_stage(il + 1)) return false;
    }
    if (ng == 2) {
        HIP_OK(hipEventRecord(ln.ev_join, ln.stream2));
        HIP_OK(hipStreamWaitEvent(st, ln.ev_join, 0));
    }
    LAUNCH_OK("pool_l2", launch_pool(w.X, d_off, n_seqs, E, d_out, st, d_out_row));
    return true;
}

// ---- loading
const GGUFTensor *need_tensor(const GGUFFile &f, const std::string &name, std::vector<int64_t> ne) {
    const GGUFTensor *t = f.tensor(name);
    if (!t) {
        set_err("tensor '%s' not found", name.c_str());
        return nullptr;
    }
    for (size_t i = 0; i < ne.size(); i++)
        if (i >= t->ne.size() || t->ne[i] != ne[i]) {
            set_err("tensor '%s' has wrong shape", name.c_str());
            return nullptr;
        }
    return t;
}

bool get_u32(const GGUFFile &f, const char *k, int32_t &out, bool req) {
    const GGUFValue *v = f.find(k);
    if (!v) {
        if (req) set_err("key not found in model: %s", k);
        return !req;
    }
    if (v->type != GV_U32) {
        set_err("key %s has wrong type", k);
        return false;
    }
    out = (int32_t)v->u;
    return true;
}

struct HostModel {
    const GGUFTensor *word, *pos, *type, *ln_e_w, *ln_e_b;
    struct L {
        const GGUFTensor *q_w, *q_b, *k_w, *k_b, *v_w, *v_b, *o_w, *o_b, *ln1_w, *ln1_b, *i_w, *i_b, *o2_w, *o2_b,
            *ln2_w, *ln2_b;
    };
    std::vector<L> layers;
};

// An embedding table as f32 rows, exactly as ggml_get_rows dequantises it
// (reference bert.cpp:880-887): F16 widened, Q4_0
// (q - 8) * d, Q4_1 q * d + m (one fused multiply-add, as ggml's compiled
// dequantize_row_q4_1).  The device keeps the f32 copy, so the gather is a
// plain row read (the quantised rows would cost five narrow loads per 8 values).
std::vector<float> table_f32(const GGUFTensor *t) {
    const int64_t E = t->ne[0], rows = t->nrows();
    std::vector<float> out((size_t)(E * rows));
    for (int64_t r = 0; r < rows; r++) {
        float *o = &out[(size_t)(r * E)];
        if (t->type == GT_F32) {
            std::memcpy(o, t->data + r * E * 4, (size_t)E * 4);
        } else if (t->type == GT_F16) {
            const uint16_t *h = (const uint16_t *)(t->data + r * E * 2);
            for (int64_t e = 0; e < E; e++) o[e] = f16_to_f32(h[e]);
        } else {
            const bool q1 = t->type == GT_Q4_1;
            const int bs = q1 ? 20 : 18;
            const uint8_t *row = t->data + r * (E / 32) * bs;
            for (int64_t b = 0; b < E / 32; b++) {
                const uint8_t *blk = row + b * bs;
                uint16_t dh, mh = 0;
                std::memcpy(&dh, blk, 2);
                if (q1) std::memcpy(&mh, blk + 2, 2);
                const float d = f16_to_f32(dh), m = f16_to_f32(mh);
                const uint8_t *qs = blk + (q1 ? 4 : 2);
                for (int j = 0; j < 32; j++) {
                    const int q = j < 16 ? (qs[j] & 15) : (qs[j - 16] >> 4);
                    o[b * 32 + j] = q1 ? std::fmaf((float)q, d, m) : (float)(q - 8) * d;
                }
            }
        }
    }
    return out;
}

// A new lane on R's device (the caller has set it current)
bool add_lane(Replica &R) {
    auto ln = std::make_unique<Lane>();
    HIP_OK(hipStreamCreateWithFlags(&ln->stream, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&ln->stream2, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&ln->ev_fork, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ln->ev_join, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ln->ev_free, hipEventDisableTiming));
    R.lanes.push_back(std::move(ln));
    return true;
}

// The device form of a model, as a sequence of staged buffers: with
// S.replay false it only makes the host bytes (no device call); with S.replay
// true it allocates and uploads them on R.device, in the same order.
bool build_replica(bert_ctx *ctx, const HostModel &hm, Stager &S, Replica &R) {
    if (S.replay) {
        HIP_OK(hipSetDevice(R.device));
        if (!add_lane(R)) return false;
        S.track = &R.weight_allocs;
    }
    auto table = [&](void **p, const GGUFTensor *t) {
        return S.put(p, [&](StageBuf &b) {
            const std::vector<float> v = table_f32(t);
            b.own.assign((const uint8_t *)v.data(), (const uint8_t *)(v.data() + v.size()));
        });
    };
    auto word_table = [&]() {
        if (!ctx->emb_raw) return table(&R.word, hm.word);
        return S.put_ext(&R.word, hm.word->data, hm.word->nbytes);
    };
    if (!word_table() || !table(&R.pos, hm.pos) || !table(&R.type, hm.type) ||
        !S.put_ext(&R.ln_e_w, hm.ln_e_w->data, hm.ln_e_w->nbytes) ||
        !S.put_ext(&R.ln_e_b, hm.ln_e_b->data, hm.ln_e_b->nbytes) ||
        !S.put_ext(&R.gelu_tab, tables().gelu.data(), 65536 * 2) ||
        !S.put_ext(&R.exp_tab, tables().expt.data(), 65536 * 2) ||
        !S.put_ext(&R.gelu_compact, tables().gelu_pair.data(), tables().gelu_pair.size() * 2) ||
        !S.put_ext(&R.exp_compact, tables().exp_c.compact.data(), tables().exp_c.compact.size() * 2))
        return false;
    const int64_t E = ctx->hp.n_embd, I = ctx->hp.n_intermediate;
    const uint32_t wt = hm.layers[0].q_w->type;
    for (const auto &l : hm.layers) {
        DevLayer dl;
        // QKV rows head-major (kernels.h GemmArgs EPI_QKV): feature h*3D + part*D + d
        // <- row d of head h of Q (part 0), K (1) or V (2)
        const int64_t Dh = E / ctx->hp.n_head;
        const std::vector<const uint8_t *> rq = rows_of(l.q_w), rk = rows_of(l.k_w), rv = rows_of(l.v_w);
        std::vector<const uint8_t *> rows((size_t)(3 * E));
        std::vector<float> bqkv((size_t)3 * E);
        for (int64_t hd = 0; hd < ctx->hp.n_head; hd++)
            for (int part = 0; part < 3; part++)
                for (int64_t d = 0; d < Dh; d++) {
                    const size_t dst = (size_t)(hd * 3 * Dh + part * Dh + d), src = (size_t)(hd * Dh + d);
                    rows[dst] = (part == 0 ? rq : part == 1 ? rk : rv)[src];
                    const GGUFTensor *bt = part == 0 ? l.q_b : part == 1 ? l.k_b : l.v_b;
                    bqkv[dst] = ((const float *)bt->data)[src];
                }
        if (ctx->i8_qkv) {
            // producer / consumer kernel and its unfused twin (or the unfused
            // int8 QKV GEMM alone, i8 qkv): int8 codes, head-major f-tiles
            if (!stage_i8(S, dl.qkv8, wt, rows, E)) return false;
        } else if (qkv_attention_supported(ctx->wtype, (int)E, (int)ctx->hp.n_head, 128, ctx->qkva_ntw)) {
            // undo repack's column interleave (row 32p + 2c + t <- 32p + 16t + c) so
            // that repacked tile j holds features 16j .. 16j + 15 in order
            // after the grouped tile order (kernels.hip qkv_attention_kernel): tile
            // G tpp q + G w + t <- n-tile w of 192-feature unit G q + t (tpp = 12
            // n-tiles per unit: a head pair at head dim 32, one head at 64; G =
            // units per main loop; G = 1 is the plain order)
            const size_t tpp = 12, G = (size_t)std::max(1, ctx->qkva_ntw);
            std::vector<const uint8_t *> quad(rows.size()), plain(rows.size());
            for (size_t T = 0; T < rows.size() / 16; T++) {
                const size_t src = tpp * (G * (T / (G * tpp)) + T % G) + (T % (G * tpp)) / G;
                for (int c = 0; c < 16; c++) quad[16 * T + c] = rows[16 * src + c];
            }
            for (size_t pr = 0; pr < rows.size() / 32; pr++)
                for (int t = 0; t < 2; t++)
                    for (int c = 0; c < 16; c++) plain[32 * pr + 2 * c + t] = quad[32 * pr + 16 * t + c];
            if (!stage_packed(S, dl.qkv_plain, [&] { return repack(wt, plain, E); })) return false;
        }
        std::vector<const uint8_t *> up_rows = rows_of(l.i_w);
        if (gemm_gelu_blk8(ctx->wtype)) {
            // block-8 column order (kernels.h gemm_gelu_blk8): repack's interleave
            // takes input row 32p + 2r + t to repacked row 16(2p + t) + r, which
            // must hold weight row 32p + 8(r >> 2) + 4t + (r & 3)
            const std::vector<const uint8_t *> src = up_rows;
            for (size_t pr = 0; pr < src.size() / 32; pr++)
                for (int t = 0; t < 2; t++)
                    for (int r = 0; r < 16; r++) up_rows[32 * pr + 2 * r + t] = src[32 * pr + 8 * (r >> 2) + 4 * t + (r & 3)];
        }
        if (!ctx->i8_qkv && !stage_packed(S, dl.qkv, [&] { return repack(wt, rows, E); })) return false;
        // each projection in the one format its GEMM reads (int8 or split fp16)
        if (!(ctx->i8_o ? stage_i8(S, dl.o8, wt, rows_of(l.o_w), E)
                        : stage_packed(S, dl.o, [&] { return repack(wt, rows_of(l.o_w), E); })) ||
            !(ctx->i8_up ? stage_i8(S, dl.up8, wt, rows_of(l.i_w), E)
                         : stage_packed(S, dl.up, [&] { return repack(wt, up_rows, E); })) ||
            !(ctx->i8_down ? stage_i8(S, dl.down8, wt, rows_of(l.o2_w), I)
                           : stage_packed(S, dl.down, [&] { return repack(wt, rows_of(l.o2_w), I); })))
            return false;
        if (!S.put_vec(&dl.b_qkv, bqkv) || !S.put_ext(&dl.b_o, l.o_b->data, E * 4) ||
            !S.put_ext(&dl.b_up, l.i_b->data, I * 4) || !S.put_ext(&dl.b_down, l.o2_b->data, E * 4) ||
            !S.put_ext(&dl.ln1_w, l.ln1_w->data, E * 4) || !S.put_ext(&dl.ln1_b, l.ln1_b->data, E * 4) ||
            !S.put_ext(&dl.ln2_w, l.ln2_w->data, E * 4) || !S.put_ext(&dl.ln2_b, l.ln2_b->data, E * 4))
            return false;
        R.L.push_back(dl);
    }
    if (S.replay) HIP_OK(hipDeviceSynchronize());
    return true;
}

void free_replica(Replica &R) {
    hipSetDevice(R.device);
    hipDeviceSynchronize();  // caller streams may still read the workspace
    drain_profile(R);
    for (auto &lp : R.lanes) {
        Lane &ln = *lp;
        clear_graphs(ln);
        for (void *p : ln.ws.allocs) hipFree(p);
        if (ln.ws.h_tok) hipHostFree(ln.ws.h_tok);
        if (ln.ws.h_off) hipHostFree(ln.ws.h_off);
        if (ln.ws.h_out) hipHostFree(ln.ws.h_out);
        if (ln.stream2) hipStreamDestroy(ln.stream2);
        if (ln.ev_fork) hipEventDestroy(ln.ev_fork);
        if (ln.ev_join) hipEventDestroy(ln.ev_join);
        if (ln.ev_free) hipEventDestroy(ln.ev_free);
        if (ln.stream) hipStreamDestroy(ln.stream);
    }
    R.lanes.clear();
    for (void *p : R.weight_allocs) hipFree(p);
}

std::vector<int> parse_device_env(int n_visible) {
    std::vector<int> devs;
    const char *env = std::getenv("BERT_AMD_DEVICES");
    if (env && *env) {
        std::string s(env);
        size_t p = 0;
        while (p < s.size()) {
            size_t q = s.find(',', p);
            if (q == std::string::npos) q = s.size();
            int d = std::atoi(s.substr(p, q - p).c_str());
            if (d >= 0 && d < n_visible) devs.push_back(d);
            p = q + 1;
        }
    }
    if (devs.empty())
        for (int d = 0; d < n_visible; d++) devs.push_back(d);
    return devs;
}

// Context options (bert_amd.h bert_amd_set_option), checked; the caller
// holds ctx->mu or owns the context.  Returns 0, or -2 with the error set.
int apply_option(bert_ctx *ctx, const std::string &k, int32_t value) {
    auto need = [&](bool ok, const char *what) {
        if (!ok) set_err("bert_amd option %s: %s", k.c_str(), what);
        return ok ? 0 : -2;
    };
    if (k == "split") {
        ctx->split = value != 0;
    } else if (k == "pack") {
        if (need(value >= -1 && value <= 1, "must be -1, 0 or 1")) return -2;
        ctx->pack = value;
    } else if (k == "fuse_min") {
        if (need(value >= 0, "must be >= 0")) return -2;
        ctx->fuse_min = value;
    } else if (k == "unfused") {
        ctx->unfused = value != 0;
    } else if (k == "small_qkva") {
        ctx->small_qkva = value != 0;
    } else if (k == "nt_x") {
        ctx->nt_x = value != 0;
    } else if (k == "small_rows" || k == "graph_seqs") {
        if (need(value >= 0, "must be >= 0")) return -2;
        (k == "small_rows" ? ctx->small_rows : ctx->graph_seqs) = value;
    } else if (k == "encode_lanes" || k == "encode_merge" || k == "encode_merge_rows") {
        if (need(value >= 1, "must be >= 1")) return -2;
        (k == "encode_lanes" ? ctx->encode_lanes : k == "encode_merge" ? ctx->encode_merge : ctx->encode_merge_rows) = value;
    } else {
        set_err("bert_amd option: unknown option '%s'", k.c_str());
        return -2;
    }
    ctx->opt_gen++;
    return 0;
}

// Load options (bert_amd.h bert_amd_load_opts): "key=value" items separated by
// ';'.  Defaults come from the environment (BERT_AMD_<KEY>, upper case), read
// here once per load and never again; the explicit string overrides them.
// Load-time keys: i8 (the int8-MFMA projections, i8_select) and qkva_ntw (the
// fused kernel's weight grouping); every bert_amd_set_option key is accepted
// too.  Returns false with the error set.
bool parse_load_options(bert_ctx *ctx, const char *opts, std::string &i8_spec) {
    static const char *keys[] = {"i8", "qkva_ntw", "q41bf", "split", "pack", "fuse_min", "unfused", "small_rows", "graph_seqs",
                                 "small_qkva", "encode_lanes", "encode_merge", "encode_merge_rows", "emb_raw", "nt_x"};
    std::vector<std::pair<std::string, std::string>> kv;
    for (const char *k : keys) {
        std::string env = "BERT_AMD_" + std::string(k);
        for (char &c : env) c = (char)std::toupper((unsigned char)c);
        if (const char *e = std::getenv(env.c_str()); e && *e) kv.push_back({k, e});
    }
    for (std::string o = opts ? opts : ""; !o.empty();) {
        const size_t semi = o.find(';');
        const std::string item = o.substr(0, semi);
        o = semi == std::string::npos ? "" : o.substr(semi + 1);
        if (item.empty()) continue;
        const size_t eq = item.find('=');
        if (eq == std::string::npos || eq == 0) {
            set_err("bert_amd_load_opts: malformed option '%s' (key=value expected)", item.c_str());
            return false;
        }
        kv.push_back({item.substr(0, eq), item.substr(eq + 1)});
    }
    for (const auto &p : kv) {
        if (p.first == "i8") {
            i8_spec = p.second;
            continue;
        }
        char *end = nullptr;
        const long v = std::strtol(p.second.c_str(), &end, 10);
        if (p.second.empty() || *end) {
            set_err("bert_amd option %s: '%s' is not an integer", p.first.c_str(), p.second.c_str());
            return false;
        }
        if (v < INT32_MIN || v > INT32_MAX) {  // no silent wrap when narrowing to int32
            set_err("bert_amd option %s: '%s' is out of the int32 range", p.first.c_str(), p.second.c_str());
            return false;
        }
        if (p.first == "qkva_ntw") {
            if (v < -1 || v > 2) {
                set_err("bert_amd option qkva_ntw: must be -1 (auto), 0, 1 or 2");
                return false;
            }
            ctx->qkva_ntw = (int)v;
        } else if (p.first == "emb_raw") {
            if (v < 0 || v > 1) {
                set_err("bert_amd option emb_raw: must be 0 or 1");
                return false;
            }
            ctx->emb_raw = v != 0;
        } else if (p.first == "q41bf") {
            if (v < -1 || v > 1) {
                set_err("bert_amd option q41bf: must be -1 (auto), 0 or 1");
                return false;
            }
            ctx->q41bf = (int)v;
        } else if (apply_option(ctx, p.first, (int32_t)v) != 0) {
            return false;
        }
    }
    return true;
}

bert_ctx *load_impl(const char *fname, const int32_t *devices, int32_t n_devices, const char *opts) {
    if (!fname) {
        set_err("null model path");
        return nullptr;
    }
    std::printf("%s: loading model from '%s' - please wait ...\n", "bert_load_from_file", fname);
    GGUFFile f;
    std::string err;
    if (!f.open(fname, err)) {
        set_err("%s", err.c_str());
        return nullptr;
    }
    auto ctx = std::make_unique<bert_ctx>();
    HParams &hp = ctx->hp;
    // reference bert.cpp:506-512
    const GGUFValue *toks = f.find("tokenizer.ggml.tokens");
    if (!toks || toks->type != GV_ARR || toks->arr_type != GV_STR) {
        set_err("cannot find tokenizer vocab in model file");
        return nullptr;
    }
    hp.n_vocab = (int32_t)toks->arr_n;
    if (!get_u32(f, "bert.context_length", hp.n_max_tokens, true) ||
        !get_u32(f, "bert.embedding_length", hp.n_embd, true) ||
        !get_u32(f, "bert.feed_forward_length", hp.n_intermediate, true) ||
        !get_u32(f, "bert.attention.head_count", hp.n_head, true) ||
        !get_u32(f, "bert.block_count", hp.n_layer, true))
        return nullptr;
    const GGUFValue *eps = f.find("bert.attention.layer_norm_epsilon");
    if (!eps || eps->type != GV_F32) {
        set_err("key not found in model: bert.attention.layer_norm_epsilon");
        return nullptr;
    }
    hp.eps = (float)eps->f;
    // header sanity before anything indexes layers or divides by the head count
    if (hp.n_layer <= 0 || hp.n_layer > 1024 || hp.n_head <= 0 || hp.n_embd <= 0 || hp.n_embd % hp.n_head ||
        hp.n_intermediate <= 0 || hp.n_max_tokens <= 0 || hp.n_vocab <= 0) {
        set_err("invalid hparams: n_vocab=%d n_max_tokens=%d n_embd=%d n_intermediate=%d n_head=%d n_layer=%d",
                hp.n_vocab, hp.n_max_tokens, hp.n_embd, hp.n_intermediate, hp.n_head, hp.n_layer);
        return nullptr;
    }
    // tokenizer (reference bert.cpp:515-578)
    if (!f.find("tokenizer.ggml.scores")) { set_err("cannot find tokenizer scores in model file"); return nullptr; }
    if (!f.find("tokenizer.ggml.token_type")) { set_err("cannot find token type list in GGUF file"); return nullptr; }
    ctx->id_to_token = toks->arr_str;
    get_u32(f, "tokenizer.ggml.cls_token_id", ctx->cls_id, false);
    get_u32(f, "tokenizer.ggml.seperator_token_id", ctx->sep_id, false);
    get_u32(f, "tokenizer.ggml.padding_token_id", ctx->pad_id, false);
    const GGUFValue *blob = f.find("blob.tokenizer.json");
    if (!blob || blob->type != GV_STR) {
        set_err("key not found in model: blob.tokenizer.json");
        return nullptr;
    }
    if (!ctx->tokenizer.load(blob->s, err)) {
        set_err("%s", err.c_str());
        return nullptr;
    }
    // tensors (reference bert.cpp:623-652)
    const int64_t E = hp.n_embd, I = hp.n_intermediate;
    HostModel hm;
    if (!(hm.word = need_tensor(f, "embeddings.word_embeddings.weight", {E, hp.n_vocab})) ||
        !(hm.type = need_tensor(f, "embeddings.token_type_embeddings.weight", {E, 2})) ||
        !(hm.pos = need_tensor(f, "embeddings.position_embeddings.weight", {E, hp.n_max_tokens})) ||
        !(hm.ln_e_w = need_tensor(f, "embeddings.LayerNorm.weight", {E})) ||
        !(hm.ln_e_b = need_tensor(f, "embeddings.LayerNorm.bias", {E})))
        return nullptr;
    for (int il = 0; il < hp.n_layer; il++) {
        const std::string p = "encoder.layer." + std::to_string(il) + ".";
        HostModel::L l;
        if (!(l.ln1_w = need_tensor(f, p + "attention.output.LayerNorm.weight", {E})) ||
            !(l.ln1_b = need_tensor(f, p + "attention.output.LayerNorm.bias", {E})) ||
            !(l.ln2_w = need_tensor(f, p + "output.LayerNorm.weight", {E})) ||
            !(l.ln2_b = need_tensor(f, p + "output.LayerNorm.bias", {E})) ||
            !(l.q_w = need_tensor(f, p + "attention.self.query.weight", {E, E})) ||
            !(l.q_b = need_tensor(f, p + "attention.self.query.bias", {E})) ||
            !(l.k_w = need_tensor(f, p + "attention.self.key.weight", {E, E})) ||
            !(l.k_b = need_tensor(f, p + "attention.self.key.bias", {E})) ||
            !(l.v_w = need_tensor(f, p + "attention.self.value.weight", {E, E})) ||
            !(l.v_b = need_tensor(f, p + "attention.self.value.bias", {E})) ||
            !(l.o_w = need_tensor(f, p + "attention.output.dense.weight", {E, E})) ||
            !(l.o_b = need_tensor(f, p + "attention.output.dense.bias", {E})) ||
            !(l.i_w = need_tensor(f, p + "intermediate.dense.weight", {E, I})) ||
            !(l.i_b = need_tensor(f, p + "intermediate.dense.bias", {I})) ||
            !(l.o2_w = need_tensor(f, p + "output.dense.weight", {I, E})) ||
            !(l.o2_b = need_tensor(f, p + "output.dense.bias", {E})))
            return nullptr;
        hm.layers.push_back(l);
    }
    // one weight type for the 2-D matrices; 1-D tensors must be f32
    const uint32_t wt = hm.layers[0].q_w->type;
    ctx->wtype = wtype_of(wt);
    if (ctx->wtype < 0) { set_err("unsupported weight type %u", wt); return nullptr; }
    for (auto &l : hm.layers) {
        for (const GGUFTensor *t : {l.q_w, l.k_w, l.v_w, l.o_w, l.i_w, l.o2_w})
            if (t->type != wt) { set_err("mixed weight types are not supported (%s)", t->name.c_str()); return nullptr; }
        for (const GGUFTensor *t : {l.q_b, l.k_b, l.v_b, l.o_b, l.i_b, l.o2_b, l.ln1_w, l.ln1_b, l.ln2_w, l.ln2_b})
            if (t->type != GT_F32) { set_err("1-D tensor %s is not f32", t->name.c_str()); return nullptr; }
    }
    for (const GGUFTensor *t : {hm.word, hm.pos, hm.type})
        if (wtype_of(t->type) < 0) { set_err("unsupported embedding table type for %s", t->name.c_str()); return nullptr; }
    if (hm.ln_e_w->type != GT_F32 || hm.ln_e_b->type != GT_F32) { set_err("embedding LayerNorm must be f32"); return nullptr; }
    ctx->word_t = hm.word->type;
    ctx->pos_t = hm.pos->type;
    ctx->type_t = hm.type->type;
    const int D = (int)(E / hp.n_head);
    if ((E != 384 && E != 768 && E != 1024) || (D != 32 && D != 64) || I % 256 || hp.n_max_tokens > 512 ||
        !gemm_shape_supported(EPI_QKV, (int)(3 * E), (int)E) || !gemm_shape_supported(gemm_ln_fused(ctx->wtype, (int)E) ? EPI_LN : EPI_RESID, (int)E, (int)I)) {
        set_err("unsupported shape: n_embd=%d n_head=%d n_intermediate=%d n_max_tokens=%d", hp.n_embd, hp.n_head,
                hp.n_intermediate, hp.n_max_tokens);
        return nullptr;
    }
    if (tables().gelu_cap >= (1 << 20) || tables().gelu_c.pos_n >= (1 << 20) || tables().exp_c.pos_n >= (1 << 20)) {
        set_err("fp16 GELU/exp table self-check failed: the device lookup rules do not reproduce this host's tables");
        return nullptr;
    }
    if ((int)tables().gelu_pair.size() > HALF_TABLE_LDS || (int)tables().exp_c.compact.size() > EXP_TABLE_LDS) {
        set_err("this host's libm gives fp16 GELU/exp tables whose compact part exceeds LDS (%zu, %zu entries)",
                tables().gelu_pair.size(), tables().exp_c.compact.size());
        return nullptr;
    }
    std::string i8_spec;
    if (!parse_load_options(ctx.get(), opts, i8_spec)) return nullptr;
    // the producer / consumer fused kernel exists for Q4_0 at head dim 32, n_embd
    // 384 (MiniLM; measured +1.2% batch-1024, +6% ragged over the head-pair
    // kernel): auto takes it there and the 2-unit head-pair kernel
    // elsewhere; an explicit 0 on another shape takes the head-pair kernel on
    // the same plain-order copy
    const bool pc_ok = qkv_attention_supported(ctx->wtype, (int)E, hp.n_head, 128, 0);
    if (ctx->qkva_ntw < 0) ctx->qkva_ntw = pc_ok ? 0 : 2;
    if (ctx->qkva_ntw == 0 && !pc_ok) ctx->qkva_ntw = 1;
    i8_select(ctx.get(), i8_spec);
    // devices
    int n_visible = 0;
    if (hipGetDeviceCount(&n_visible) != hipSuccess || n_visible <= 0) {
        set_err("no HIP device visible: this library runs the embedding path on MI355X GPUs only");
        return nullptr;
    }
    std::vector<int> devs;
    if (devices && n_devices > 0) {
        for (int i = 0; i < n_devices; i++)
            if (devices[i] >= 0 && devices[i] < n_visible) devs.push_back(devices[i]);
    } else {
        devs = parse_device_env(n_visible);
    }
    if (devs.empty()) { set_err("no usable device in the requested list"); return nullptr; }
    // the host forms of every weight buffer, made once (Stager), then one
    // upload thread per replica
    std::vector<StageBuf> book;
    {
        Stager rec;
        rec.book = &book;
        Replica scratch;
        if (!build_replica(ctx.get(), hm, rec, scratch)) return nullptr;
    }
    for (int d : devs) {
        ctx->reps.push_back(std::make_unique<Replica>());
        ctx->reps.back()->device = d;
    }
    std::vector<std::string> errs(devs.size());
    {
        std::vector<std::thread> th;
        for (size_t i = 0; i < devs.size(); i++)
            th.emplace_back([&, i] {
                try {
                    Stager up;
                    up.book = &book;
                    up.replay = true;
                    if (!build_replica(ctx.get(), hm, up, *ctx->reps[i]) ) errs[i] = g_err;
                    else if (up.next != book.size()) errs[i] = "internal: weight staging replay out of step";
                } catch (const std::exception &e) {
                    errs[i] = e.what();
                } catch (...) {
                    errs[i] = "unknown exception";
                }
            });
        for (auto &t : th) t.join();
    }
    for (size_t i = 0; i < devs.size(); i++)
        if (!errs[i].empty()) {
            set_err("device %d: %s", devs[i], errs[i].c_str());
            for (auto &r : ctx->reps) free_replica(*r);
            return nullptr;
        }
    std::printf("%s: n_vocab = %d, n_max_tokens = %d, n_embd = %d, n_intermediate = %d, n_head = %d, n_layer = %d, "
                "weights = %s, devices = %zu\n",
                "bert_load_from_file", hp.n_vocab, hp.n_max_tokens, hp.n_embd, hp.n_intermediate, hp.n_head,
                hp.n_layer, ggml_type_str(wt), devs.size());
    return ctx.release();
}

bool grow_pinned(Workspace &w, int64_t rows, int64_t seqs, int64_t E) {
    // callers hold ctx->mu and the replica's previous copies have completed
    // (eval_host_slice synchronises its stream), so the old buffers are idle
    if (rows > w.h_cap_rows) {
        if (w.h_tok) hipHostFree(w.h_tok);
        w.h_tok = nullptr;
        w.h_cap_rows = 0;
        HIP_OK(hipHostMalloc((void **)&w.h_tok, (size_t)rows * 4, hipHostMallocDefault));
        w.h_cap_rows = rows;
    }
    if (seqs > w.h_cap_seqs) {
        if (w.h_off) hipHostFree(w.h_off);
        if (w.h_out) hipHostFree(w.h_out);
        w.h_off = nullptr;
        w.h_out = nullptr;
        w.h_cap_seqs = 0;
        HIP_OK(hipHostMalloc((void **)&w.h_off, (size_t)(seqs + 1) * 4, hipHostMallocDefault));
        HIP_OK(hipHostMalloc((void **)&w.h_out, (size_t)seqs * E * 4, hipHostMallocDefault));
        w.h_cap_seqs = seqs;
    }
    return true;
}

// run_pipeline over the lane's workspace (tokens / offsets uploaded, h_off the
// host offsets).  Small batches (<= graph_seqs sentences, fewer than fuse_min:
// the unfused pair, so the pipeline makes no host copy; profiling off) replay a
// HIP graph captured on the first batch of the same token offsets: the
// launches' arguments depend only on the offsets, the workspace addresses
// (graphs are dropped when it is reallocated) and the options (dropped on any
// change).  At most 256 graphs per lane (then the cache starts over).
bool run_host_pipeline(bert_ctx *ctx, Replica &R, Lane &ln, int n, hipStream_t st, const int32_t *d_out_row) {
    Workspace &w = ln.ws;
    const int64_t M = w.h_off[n];
    const int64_t Mpad = std::max<int64_t>(GEMM_BM, (M + GEMM_BM - 1) / GEMM_BM * GEMM_BM);
    if (R.prof || d_out_row || n > ctx->graph_seqs || n >= ctx->fuse_min || Mpad > w.cap_rows || n > w.cap_seqs)
        return run_pipeline(ctx, R, ln, w.tok, w.off, w.h_off, n, w.out, st, d_out_row);
    if (ln.graphs_ws_gen != w.gen || ln.graphs_opt_gen != ctx->opt_gen || ln.graphs.size() >= 256) {
        clear_graphs(ln);
        ln.graphs_ws_gen = w.gen;
        ln.graphs_opt_gen = ctx->opt_gen;
    }
    std::vector<int32_t> key(w.h_off, w.h_off + n + 1);
    auto it = ln.graphs.find(key);
    if (it == ln.graphs.end()) {
        HIP_OK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        const bool ok = run_pipeline(ctx, R, ln, w.tok, w.off, w.h_off, n, w.out, st);
        const std::string err = ok ? std::string() : g_err;
        hipGraph_t g = nullptr;
        const hipError_t e = hipStreamEndCapture(st, &g);
        if (!ok || e != hipSuccess || !g) {
            if (g) hipGraphDestroy(g);
            set_err("graph capture: %s", ok ? hipGetErrorString(e) : err.c_str());
            return false;
        }
        hipGraphExec_t ex = nullptr;
        const hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
        hipGraphDestroy(g);
        if (ei != hipSuccess) {
            set_err("graph instantiate: %s", hipGetErrorString(ei));
            return false;
        }
        it = ln.graphs.emplace(std::move(key), ex).first;
    }
    HIP_OK(hipGraphLaunch(it->second, st));
    return true;
}

// Evaluate sentences [s0, s1) of a host batch on replica R; results go
// straight into the caller's embedding rows.
bool eval_host_slice(bert_ctx *ctx, Replica &R, Lane &ln, bert_vocab_id **toks, const int32_t *ntok, float **embs, int s0,
                     int s1) {
    const int n = s1 - s0;
    if (n <= 0) return true;
    HIP_OK(hipSetDevice(R.device));
    int64_t M = 0;
    for (int s = s0; s < s1; s++) M += ntok[s];
    if (!grow_pinned(ln.ws, M, n, ctx->hp.n_embd)) return false;
    Workspace &w = ln.ws;
    // token rows contiguous in the caller's memory (one [n][len] array): upload
    // them from there instead of gathering them into the pinned buffer first
    bool tok_direct = true;
    int64_t pos = 0;
    for (int s = s0; s < s1; s++) {
        w.h_off[s - s0] = (int32_t)pos;
        tok_direct = tok_direct && toks[s] == toks[s0] + pos;
        pos += ntok[s];
    }
    w.h_off[n] = (int32_t)pos;
    if (!tok_direct)
        for (int s = s0; s < s1; s++) std::memcpy(w.h_tok + w.h_off[s - s0], toks[s], (size_t)ntok[s] * 4);
    const int64_t Mpad = std::max<int64_t>(GEMM_BM, (M + GEMM_BM - 1) / GEMM_BM * GEMM_BM);
    const hipStream_t st = ln.stream;
    const int E = ctx->hp.n_embd;
    // caller rows contiguous (one [n][E] array, the usual case): the embeddings
    // go straight from the device into them, without the pinned bounce buffer
    // and the host copy (host-API batch 1024 x 128, tools/host_ab.sh: minimum 6.80-6.85 -> 6.71-6.78 ms).
    // Rows that are a permutation of one [n][E] block (bert_encode_batch's
    // length-sorted inputs, eval_grouped's tile order): the pool kernel writes
    // each sentence into its caller row of w.out (d_out_row) and one copy lands
    // them all in place.
    bool direct = true;
    for (int s = s0 + 1; direct && s < s1; s++) direct = embs[s] == embs[s0] + (size_t)(s - s0) * E;
    float *base = embs[s0];
    std::vector<int32_t> out_row;
    if (!direct) {
        for (int s = s0 + 1; s < s1; s++) base = std::min(base, embs[s]);
        out_row.resize(n);
        std::vector<char> seen(n, 0);
        bool perm = true;
        for (int s = s0; perm && s < s1; s++) {
            const size_t d = (size_t)(embs[s] - base);
            perm = d % E == 0 && d / E < (size_t)n && !seen[d / E];
            if (perm) {
                seen[d / E] = 1;
                out_row[s - s0] = (int32_t)(d / E);
            }
        }
        if (!perm) out_row.clear();
    }
    if (!ensure_workspace(ctx, ln, Mpad, n, st) || !ws_acquire(ln, st)) return false;
    HIP_OK(hipMemcpyAsync(w.tok, tok_direct ? toks[s0] : w.h_tok, (size_t)M * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(w.off, w.h_off, (size_t)(n + 1) * 4, hipMemcpyHostToDevice, st));
    // (pageable source: staged before the call returns)
    if (!out_row.empty()) HIP_OK(hipMemcpyAsync(w.perm, out_row.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    const bool ok = run_host_pipeline(ctx, R, ln, n, st, out_row.empty() ? nullptr : w.perm);
    if (!ws_release(ln, st) || !ok) return false;
    if (direct || !out_row.empty()) {
        HIP_OK(hipMemcpyAsync(direct ? embs[s0] : base, w.out, (size_t)n * E * 4, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        drain_profile(R);
        return true;
    }
    HIP_OK(hipMemcpyAsync(w.h_out, w.out, (size_t)n * E * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    drain_profile(R);
    for (int s = s0; s < s1; s++) std::memcpy(embs[s], w.h_out + (size_t)(s - s0) * E, (size_t)E * 4);
    return true;
}

void dispatch_batch(bert_ctx *ctx, int32_t n, bert_vocab_id **toks, int32_t *ntok, float **embs);

// Order for sentences of <= 128 tokens that lets the fused kernel's
// consecutive packing (run_pipeline) fill its 128-row tiles: first-fit
// decreasing on the lengths rounded up to 32 (classes 128, 96, 64, 32), each
// bin's sentences adjacent: 128 alone, 96 + 32, 64 + 64, 64 + 32 + 32, 4 x 32.
// Results do not depend on the order (packed sentences are bitwise equal to
// the sentence alone), and the caller's output rows are addressed per sentence.
std::vector<int> tile_order(const int32_t *ntok, const std::vector<int> &idx) {
    std::vector<int> cls[4];  // span 32, 64, 96, 128
    for (int s : idx) cls[std::min(3, (ntok[s] - 1) >> 5)].push_back(s);
    std::vector<int> out;
    out.reserve(idx.size());
    size_t i32 = 0;
    for (int s : cls[3]) out.push_back(s);
    for (int s : cls[2]) {
        out.push_back(s);
        if (i32 < cls[0].size()) out.push_back(cls[0][i32++]);
    }
    for (size_t k = 0; k < cls[1].size(); k += 2) {
        out.push_back(cls[1][k]);
        if (k + 1 < cls[1].size()) {
            out.push_back(cls[1][k + 1]);
        } else {
            for (int j = 0; j < 2 && i32 < cls[0].size(); j++) out.push_back(cls[0][i32++]);
        }
    }
    while (i32 < cls[0].size()) out.push_back(cls[0][i32++]);
    return out;
}

// Workgroups run_pipeline's consecutive packing makes of sentences in `order`.
int greedy_tiles(const int32_t *ntok, const std::vector<int> &order) {
    int tiles = 0;
    for (size_t i = 0; i < order.size();) {
        int used = (ntok[order[i]] + 31) & ~31;
        size_t k = i + 1;
        while (k < order.size() && used + ((ntok[order[k]] + 31) & ~31) <= GEMM_BM) used += (ntok[order[k++]] + 31) & ~31;
        tiles++;
        i = k;
    }
    return tiles;
}

// A batch whose sentences all fit one 128-row tile runs the fused QKV +
// attention kernel; a mixed batch is evaluated as two ragged batches (short
// sentences, then the rest), so one long sentence does not move every short
// one onto the unfused pair.  Sentences are independent, so the results do
// not depend on the grouping.  The short sentences are also put in tile order
// (tile_order) so that they share fused-kernel workgroups.  `run` evaluates
// one group.
template <typename F>
void eval_grouped(bert_ctx *ctx, int32_t n, bert_vocab_id **toks, int32_t *ntok, float **embs, F run) {
    const HParams &hp = ctx->hp;
    if (!qkv_attention_supported(ctx->wtype, hp.n_embd, hp.n_head, GEMM_BM, ctx->qkva_ntw)) {
        run(n, toks, ntok, embs);
        return;
    }
    std::vector<int> shrt, lng;
    for (int s = 0; s < n; s++) (ntok[s] <= GEMM_BM ? shrt : lng).push_back(s);
    shrt = tile_order(ntok, shrt);
    for (const std::vector<int> *grp : {&shrt, &lng}) {
        if (grp->empty()) continue;
        std::vector<bert_vocab_id *> t;
        std::vector<int32_t> c;
        std::vector<float *> e;
        for (int s : *grp) {
            t.push_back(toks[s]);
            c.push_back(ntok[s]);
            e.push_back(embs[s]);
        }
        run((int32_t)grp->size(), t.data(), c.data(), e.data());
    }
}

// bert_encode_batch's slices [k * chunk, ...) of the length-sorted inputs,
// several at once: every replica gets ctx->encode_lanes lanes (created on
// first use), each lane a host thread that takes the next encode_merge
// consecutive slices and evaluates them as one ragged batch on its own
// workspace and streams — small slices (the reference consumers pass 16) each
// fill only a few CUs, so merging and running them side by side is what fills
// the device.  Each group is evaluated exactly as bert_eval_batch would
// (sentences are independent: results identical, bitwise, to any slicing);
// the working set stays bounded by lanes x merge x n_batch_size sentences.
void encode_slices(bert_ctx *ctx, int32_t n, int32_t chunk, bert_vocab_id **toks, int32_t *ntok, float **embs) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (chunk < ctx->encode_merge_rows)
        chunk = (int32_t)std::min<int64_t>({(int64_t)n, (int64_t)chunk * ctx->encode_merge,
                                            std::max<int64_t>(chunk, ctx->encode_merge_rows)});
    const int nslice = (n + chunk - 1) / chunk, nr = (int)ctx->reps.size();
    const int nl = std::max(1, std::min(ctx->encode_lanes, (nslice + nr - 1) / nr));
    for (auto &r : ctx->reps) {
        if ((int)r->lanes.size() >= nl) continue;
        if (hipSetDevice(r->device) != hipSuccess) {
            set_err("bert_encode_batch: hipSetDevice(%d) failed", r->device);
            std::fprintf(stderr, "%s\n", g_err.c_str());
            return;
        }
        while ((int)r->lanes.size() < nl)
            if (!add_lane(*r)) {
                set_err("bert_encode_batch: lane creation failed: %s", g_err.c_str());
                std::fprintf(stderr, "%s\n", g_err.c_str());
                return;
            }
    }
    // every worker's failures are collected (g_err is per thread) and reported
    // on the calling thread; nothing escapes a worker (an exception leaving a
    // std::thread would terminate the process)
    std::atomic<int> next{0};
    std::vector<std::thread> th;
    std::vector<std::string> errs((size_t)nr * nl);
    for (int r = 0; r < nr; r++)
        for (int l = 0; l < nl; l++)
            th.emplace_back([&, r, l] {
                std::string &err = errs[(size_t)r * nl + l];
                try {
                    Replica &R = *ctx->reps[r];
                    Lane &ln = *R.lanes[l];
                    for (int k = next++; k < nslice; k = next++) {
                        const int32_t s0 = k * chunk, m = std::min(chunk, n - s0);
                        eval_grouped(ctx, m, toks + s0, ntok + s0, embs + s0,
                                     [&](int32_t mm, bert_vocab_id **t, int32_t *c, float **e) {
                                         if (!eval_host_slice(ctx, R, ln, t, c, e, 0, mm) && err.empty())
                                             err = "device " + std::to_string(R.device) + ": " + g_err;
                                     });
                    }
                } catch (const std::exception &e) {
                    if (err.empty()) err = e.what();
                } catch (...) {
                    if (err.empty()) err = "unknown exception";
                }
            });
    for (auto &t : th) t.join();
    for (const std::string &e : errs)
        if (!e.empty()) {
            std::fprintf(stderr, "bert_encode_batch: %s\n", e.c_str());
            set_err("bert_encode_batch: %s", e.c_str());
        }
}

// Host-pointer batch eval, sharded over the context's replicas by token count.
void eval_batch_impl(bert_ctx *ctx, int32_t n, bert_vocab_id **toks, int32_t *ntok, float **embs) {
    if (!ctx || n <= 0 || !toks || !ntok || !embs) return;
    for (int s = 0; s < n; s++) {
        if (ntok[s] > ctx->hp.n_max_tokens) {
            std::fprintf(stderr, "Too many tokens, maximum is %d\n", ctx->hp.n_max_tokens);
            return;
        }
        if (ntok[s] <= 0 || !toks[s] || !embs[s]) {
            std::fprintf(stderr, "%s: empty input %d\n", __func__, s);
            return;
        }
        for (int t = 0; t < ntok[s]; t++)
            if (toks[s][t] < 0 || toks[s][t] >= ctx->hp.n_vocab) {
                std::fprintf(stderr, "%s: token id %d out of range\n", __func__, toks[s][t]);
                return;
            }
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    eval_grouped(ctx, n, toks, ntok, embs, [&](int32_t m, bert_vocab_id **t, int32_t *c, float **e) {
        dispatch_batch(ctx, m, t, c, e);
    });
}

// Contiguous slices of a batch for nr replicas, balanced by token count:
// cut[0] = 0 <= cut[1] <= ... <= cut[nr] = n, slice r = [cut[r], cut[r+1]).
// Slice r ends at the first sentence where the running token count reaches
// r+1 nr-ths of the total, so every slice holds at most total/nr + one
// sentence's tokens (tests/test_abi.py::test_shard_cuts_balance_and_cover).
void shard_cuts(int32_t n, const int32_t *ntok, int nr, int32_t *cut) {
    for (int r = 0; r <= nr; r++) cut[r] = n;
    cut[0] = 0;
    int64_t total = 0;
    for (int s = 0; s < n; s++) total += ntok[s];
    int64_t acc = 0;
    int r = 1;
    for (int s = 0; s < n && r < nr; s++) {
        acc += ntok[s];
        while (r < nr && acc * nr >= total * r) cut[r++] = s + 1;
    }
}

// Shards one ragged batch over the context's replicas (caller holds ctx->mu).
void dispatch_batch(bert_ctx *ctx, int32_t n, bert_vocab_id **toks, int32_t *ntok, float **embs) {
    const int nr = (int)ctx->reps.size();
    std::vector<int> cut(nr + 1);
    shard_cuts(n, ntok, nr, cut.data());
    if (nr == 1) {
        if (!eval_host_slice(ctx, *ctx->reps[0], *ctx->reps[0]->lanes[0], toks, ntok, embs, 0, n))
            std::fprintf(stderr, "bert_eval_batch: %s\n", g_err.c_str());
        return;
    }
    std::vector<std::thread> th;
    std::vector<std::string> errs(nr);
    for (int r = 0; r < nr; r++)
        th.emplace_back([&, r] {
            try {
                if (!eval_host_slice(ctx, *ctx->reps[r], *ctx->reps[r]->lanes[0], toks, ntok, embs, cut[r], cut[r + 1]))
                    errs[r] = g_err;
            } catch (const std::exception &e) {
                errs[r] = e.what();
            } catch (...) {
                errs[r] = "unknown exception";
            }
        });
    for (auto &t : th) t.join();
    for (int r = 0; r < nr; r++)
        if (!errs[r].empty()) {
            std::fprintf(stderr, "bert_eval_batch: device %d: %s\n", ctx->reps[r]->device, errs[r].c_str());
            set_err("bert_eval_batch: device %d: %s", ctx->reps[r]->device, errs[r].c_str());
        }
}

}  // namespace

// ============================================================ C ABI (bert.h)

bool bert_params_parse(int argc, char **argv, bert_params &params) {
    // reference bert.cpp:681-733 (same flags; -s is advertised there but rejected too)
    auto usage = [&](FILE *o) {
        std::fprintf(o, "usage: %s [options]\n\noptions:\n", argv[0]);
        std::fprintf(o, "  -h, --help            show this help message and exit\n");
        std::fprintf(o, "  -t N, --threads N     number of threads to use during computation (default: %d)\n", params.n_threads);
        std::fprintf(o, "  -p PROMPT, --prompt PROMPT\n                        prompt to start generation with (default: random)\n");
        std::fprintf(o, "  --port p     port to bind in server mode (default: %d)\n", params.port);
        std::fprintf(o, "  -m FNAME, --model FNAME\n                        model path (default: %s)\n\n", params.model);
    };
    for (int i = 1; i < argc; i++) {
        const std::string arg = argv[i];
        const bool has_val = i + 1 < argc;
        if ((arg == "-t" || arg == "--threads") && has_val) params.n_threads = std::atoi(argv[++i]);
        else if ((arg == "-p" || arg == "--prompt") && has_val) params.prompt = argv[++i];
        else if (arg == "--port" && has_val) params.port = std::atoi(argv[++i]);
        else if ((arg == "-m" || arg == "--model") && has_val) params.model = argv[++i];
        else if (arg == "-h" || arg == "--help") { usage(stderr); std::exit(0); }
        else {
            std::fprintf(stderr, "error: unknown argument: %s\n", arg.c_str());
            usage(stderr);
            std::exit(0);
        }
    }
    return true;
}

bert_ctx *bert_load_from_file(const char *fname) {
    bert_ctx *c = nullptr;
    try {
        c = load_impl(fname, nullptr, 0, nullptr);
    } catch (const std::exception &e) {
        set_err("%s", e.what());
        c = nullptr;
    }
    if (!c) std::fprintf(stderr, "bert_load_from_file: %s\n", g_err.c_str());
    return c;
}

void bert_free(bert_ctx *ctx) {
    if (!ctx) return;
    for (auto &r : ctx->reps) free_replica(*r);
    delete ctx;
}

namespace {
// reference bert.cpp:738-781: [CLS] + Encode(text) up to the first pad id +
// [SEP], truncated so that the last slot is [SEP].
int32_t frame_tokens(const std::vector<int32_t> &ids, int32_t cls, int32_t sep, int32_t pad, bert_vocab_id *tokens,
                     int32_t n_max_tokens) {
    int32_t t = 0;
    tokens[t++] = cls;
    for (int32_t id : ids) {
        if (id == pad) break;
        if (t >= n_max_tokens) break;
        tokens[t++] = id;
        if (t >= n_max_tokens) break;
    }
    if (t >= n_max_tokens) tokens[n_max_tokens - 1] = sep;
    else tokens[t++] = sep;
    return t;
}
}  // namespace

void bert_tokenize(bert_ctx *ctx, const char *text, bert_vocab_id *tokens, int32_t *n_tokens, int32_t n_max_tokens) {
    if (!ctx || !text || !tokens || !n_tokens || n_max_tokens <= 0) return;
    std::vector<int32_t> ids;
    try {
        ids = ctx->tokenizer.encode(text);
    } catch (...) {
        ids.clear();
    }
    *n_tokens = frame_tokens(ids, ctx->cls_id, ctx->sep_id, ctx->pad_id, tokens, n_max_tokens);
}

void bert_eval(bert_ctx *ctx, int32_t n_threads, bert_vocab_id *tokens, int32_t n_tokens, float *embeddings) {
    // reference bert.cpp:1020-1028; embeddings == NULL was the reference's
    // arena-probe mode: nothing to probe here, so it is a no-op.
    (void)n_threads;
    if (!embeddings) return;
    bert_eval_batch(ctx, n_threads, 1, &tokens, &n_tokens, &embeddings);
}

void bert_eval_batch(bert_ctx *ctx, int32_t n_threads, int32_t n_batch_size, bert_vocab_id **batch_tokens,
                     int32_t *n_tokens, float **batch_embeddings) {
    (void)n_threads;
    if (!batch_embeddings) return;
    try {
        eval_batch_impl(ctx, n_batch_size, batch_tokens, n_tokens, batch_embeddings);
    } catch (const std::exception &e) {
        std::fprintf(stderr, "bert_eval_batch: %s\n", e.what());
    }
}

void bert_encode(bert_ctx *ctx, int32_t n_threads, const char *texts, float *embeddings) {
    bert_encode_batch(ctx, n_threads, 1, 1, &texts, &embeddings);
}

void bert_encode_batch(bert_ctx *ctx, int32_t n_threads, int32_t n_batch_size, int32_t n_inputs, const char **texts,
                       float **embeddings) {
    // reference bert.cpp:1119-1198: tokenise everything, sort by token count
    // (std::sort on the lengths, :1176-1177), evaluate in slices of
    // n_batch_size (the reference forces the slice to 1, :1128; here each
    // slice is one ragged GPU batch, and up to encode_lanes slices per device
    // run at once: encode_slices).  n_batch_size bounds each slice's working
    // set (a lane's device workspace and pinned staging grow to the largest
    // slice it ran); n_batch_size <= 0 means all inputs in one slice.  Sorting
    // makes each slice's lengths similar, so padding and tile waste stay small.
    if (!ctx || n_inputs <= 0 || !texts || !embeddings) return;
    const int32_t N = ctx->hp.n_max_tokens;
    std::vector<int32_t> ntok(n_inputs);
    std::vector<bert_vocab_id *> ptr(n_inputs);
    // tokenisation on n_threads host threads (the reference's thread count;
    // its CPU graph used them, bert.cpp:1128): contiguous ranges of inputs,
    // each thread appending its sentences' ids to its own array (the tokenizer
    // is stateless; no n_inputs x n_max_tokens buffer to zero and fault in)
    const int nt = std::max(1, std::min({(int)n_threads, n_inputs / 64 + 1,
                                         (int)std::max(1u, std::thread::hardware_concurrency())}));
    std::vector<std::vector<bert_vocab_id>> part(nt);
    std::vector<size_t> at(n_inputs);
    auto tok_range = [&](int t, int a, int b) {
        std::vector<bert_vocab_id> one((size_t)N);
        std::vector<bert_vocab_id> &v = part[t];
        v.reserve((size_t)(b - a) * 48);
        for (int i = a; i < b; i++) {
            bert_tokenize(ctx, texts[i], one.data(), &ntok[i], N);
            at[i] = v.size();
            v.insert(v.end(), one.begin(), one.begin() + std::max(0, ntok[i]));
        }
    };
    auto lo = [&](int t) { return (int)((int64_t)n_inputs * t / nt); };
    if (nt == 1) {
        tok_range(0, 0, n_inputs);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; t++) th.emplace_back(tok_range, t, lo(t), lo(t + 1));
        for (auto &t : th) t.join();
    }
    for (int t = 0; t < nt; t++)  // (the arrays no longer grow)
        for (int i = lo(t); i < lo(t + 1); i++) ptr[i] = part[t].data() + at[i];
    std::vector<int> idx(n_inputs);
    for (int i = 0; i < n_inputs; i++) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return ntok[a] < ntok[b]; });
    std::vector<bert_vocab_id *> sp(n_inputs);
    std::vector<int32_t> sn(n_inputs);
    std::vector<float *> se(n_inputs);
    for (int i = 0; i < n_inputs; i++) {
        sp[i] = ptr[idx[i]];
        sn[i] = ntok[idx[i]];
        se[i] = embeddings[idx[i]];
    }
    const int32_t chunk = n_batch_size > 0 ? std::min(n_batch_size, n_inputs) : n_inputs;
    if (chunk >= n_inputs) {
        bert_eval_batch(ctx, n_threads, n_inputs, sp.data(), sn.data(), se.data());
        return;
    }
    try {
        encode_slices(ctx, n_inputs, chunk, sp.data(), sn.data(), se.data());
    } catch (const std::exception &e) {
        std::fprintf(stderr, "bert_encode_batch: %s\n", e.what());
    }
}

int32_t bert_n_embd(bert_ctx *ctx) { return ctx ? ctx->hp.n_embd : 0; }
int32_t bert_n_max_tokens(bert_ctx *ctx) { return ctx ? ctx->hp.n_max_tokens : 0; }

const char *bert_vocab_id_to_token(bert_ctx *ctx, bert_vocab_id id) {
    if (!ctx || id < 0 || (size_t)id >= ctx->id_to_token.size()) return "";
    return ctx->id_to_token[(size_t)id].c_str();
}

// ============================================================ extensions (bert_amd.h)

bert_ctx *bert_amd_load(const char *fname, const int32_t *devices, int32_t n_devices) {
    return bert_amd_load_opts(fname, devices, n_devices, nullptr);
}

bert_ctx *bert_amd_load_opts(const char *fname, const int32_t *devices, int32_t n_devices, const char *options) {
    try {
        return load_impl(fname, devices, n_devices, options);
    } catch (const std::exception &e) {
        set_err("%s", e.what());
        return nullptr;
    }
}

int32_t bert_amd_n_devices(bert_ctx *ctx) { return ctx ? (int32_t)ctx->reps.size() : 0; }

int32_t bert_amd_hparams(bert_ctx *ctx, int32_t *o) {
    if (!ctx || !o) return -1;
    const HParams &h = ctx->hp;
    o[0] = h.n_vocab; o[1] = h.n_max_tokens; o[2] = h.n_embd; o[3] = h.n_intermediate;
    o[4] = h.n_head; o[5] = h.n_layer; o[6] = ctx->wtype;
    return 0;
}

int32_t bert_amd_eval_device(bert_ctx *ctx, int32_t slot, const int32_t *d_tokens, const int32_t *d_offsets,
                             const int32_t *h_offsets, int32_t n_seqs, float *d_out, void *hip_stream) {
    if (!ctx || slot < 0 || slot >= (int32_t)ctx->reps.size() || !d_tokens || !d_offsets || !h_offsets || n_seqs <= 0 ||
        !d_out) {
        set_err("bert_amd_eval_device: invalid arguments");
        return -1;
    }
    for (int s = 0; s < n_seqs; s++) {
        const int32_t n = h_offsets[s + 1] - h_offsets[s];
        if (n <= 0 || n > ctx->hp.n_max_tokens) {
            set_err("bert_amd_eval_device: sentence %d has %d tokens (max %d)", s, n, ctx->hp.n_max_tokens);
            return -2;
        }
    }
    Replica &R = *ctx->reps[slot];
    // one eval at a time per context: the workspace and the profiling state
    // are shared with bert_eval_batch and the profile_* calls
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(R.device) != hipSuccess) { set_err("hipSetDevice failed"); return -3; }
    // the caller's stream, as given: NULL is HIP's null (legacy default)
    // stream, which is ordered with the caller's other work on it
    const hipStream_t st = (hipStream_t)hip_stream;
    Lane &ln = *R.lanes[0];
    if (!ws_acquire(ln, st)) return -3;
    // every return below the acquire records the hand-over event first
    struct Release {
        Lane &ln;
        hipStream_t st;
        ~Release() { ws_release(ln, st); }
    } release{ln, st};
    try {
        // Short sentences in the caller's order may leave fused-kernel tiles
        // half empty: when the tile order (tile_order) needs fewer workgroups,
        // the batch is gathered into that order on the device and each
        // embedding is written back to its caller row (results unchanged).
        const HParams &hp = ctx->hp;
        std::vector<int32_t> ntok(n_seqs);
        int max_len = 0;
        for (int s = 0; s < n_seqs; s++) max_len = std::max(max_len, ntok[s] = h_offsets[s + 1] - h_offsets[s]);
        if (n_seqs > 1 && qkv_attention_supported(ctx->wtype, hp.n_embd, hp.n_head, max_len, ctx->qkva_ntw)) {
            std::vector<int> idx(n_seqs);
            for (int s = 0; s < n_seqs; s++) idx[s] = s;
            const std::vector<int> order = tile_order(ntok.data(), idx);
            const int t_order = greedy_tiles(ntok.data(), order);
            if (t_order < greedy_tiles(ntok.data(), idx) && qkv_attention_pack_pays(n_seqs, t_order)) {
                const int64_t M = h_offsets[n_seqs];
                const int64_t Mpad = std::max<int64_t>(GEMM_BM, (M + GEMM_BM - 1) / GEMM_BM * GEMM_BM);
                if (!ensure_workspace(ctx, ln, Mpad, n_seqs, st)) return -4;
                Workspace &w = ln.ws;
                std::vector<int32_t> off2(n_seqs + 1), perm(order.begin(), order.end());
                off2[0] = 0;
                for (int i = 0; i < n_seqs; i++) off2[i + 1] = off2[i] + ntok[order[i]];
                // pageable sources: staged before the calls return
                if (hipMemcpyAsync(w.off, off2.data(), (size_t)(n_seqs + 1) * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
                    hipMemcpyAsync(w.perm, perm.data(), (size_t)n_seqs * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
                    launch_gather_tokens(d_tokens, d_offsets, w.perm, w.off, w.tok, n_seqs, st) != hipSuccess) {
                    set_err("bert_amd_eval_device: reorder failed");
                    return -4;
                }
                if (!run_pipeline(ctx, R, ln, w.tok, w.off, off2.data(), n_seqs, d_out, st, w.perm)) return -4;
                return 0;
            }
        }
        if (!run_pipeline(ctx, R, ln, d_tokens, d_offsets, h_offsets, n_seqs, d_out, st)) return -4;
    } catch (const std::exception &e) {
        set_err("%s", e.what());
        return -5;
    }
    return 0;
}

int32_t bert_amd_profile_enable(bert_ctx *ctx, int32_t enable) {
    if (!ctx) return -1;
    std::lock_guard<std::mutex> lk(ctx->mu);
    for (auto &r : ctx->reps) {
        hipSetDevice(r->device);
        hipDeviceSynchronize();
        drain_profile(*r);
        r->prof = enable != 0;
        r->prof_acc.clear();
    }
    return 0;
}

int32_t bert_amd_profile_read(bert_ctx *ctx, char *names_buf, int32_t names_len, float *total_ms, int32_t *counts,
                              int32_t max_entries) {
    if (!ctx) return -1;
    std::lock_guard<std::mutex> lk(ctx->mu);
    std::map<std::string, ProfEntry> agg;
    for (auto &r : ctx->reps) {
        hipSetDevice(r->device);
        hipDeviceSynchronize();
        drain_profile(*r);
        for (auto &kv : r->prof_acc) {
            agg[kv.first].ms += kv.second.ms;
            agg[kv.first].n += kv.second.n;
        }
    }
    int i = 0, off = 0;
    for (auto &kv : agg) {
        if (i >= max_entries) break;
        const int need = (int)kv.first.size() + 1;
        if (names_buf && off + need <= names_len) {
            std::memcpy(names_buf + off, kv.first.c_str(), need);
            off += need;
        }
        if (total_ms) total_ms[i] = (float)kv.second.ms;
        if (counts) counts[i] = (int32_t)kv.second.n;
        i++;
    }
    return i;
}

int32_t bert_amd_debug_embed(bert_ctx *ctx, const int32_t *tokens, const int32_t *offsets, int32_t n_seqs,
                             float *X_out, void *q_out, void *d_out) {
    if (!ctx || !tokens || !offsets || n_seqs <= 0 || !X_out || !q_out) {
        set_err("bert_amd_debug_embed: invalid arguments");
        return -1;
    }
    const int64_t M = offsets[n_seqs];
    for (int s = 0; s < n_seqs; s++)
        if (offsets[s + 1] - offsets[s] <= 0 || offsets[s + 1] - offsets[s] > ctx->hp.n_max_tokens) {
            set_err("bert_amd_debug_embed: bad sentence length");
            return -2;
        }
    for (int64_t i = 0; i < M; i++)
        if (tokens[i] < 0 || tokens[i] >= ctx->hp.n_vocab) {
            set_err("bert_amd_debug_embed: token id out of range");
            return -2;
        }
    std::lock_guard<std::mutex> lk(ctx->mu);
    try {
        Replica &R = *ctx->reps[0];
        HIP_OK_RC(hipSetDevice(R.device), -3);
        Lane &ln = *R.lanes[0];
        const hipStream_t st = ln.stream;
        const int64_t Mpad = std::max<int64_t>(GEMM_BM, (M + GEMM_BM - 1) / GEMM_BM * GEMM_BM);
        if (!ensure_workspace(ctx, ln, Mpad, n_seqs, st) || !ws_acquire(ln, st)) return -3;
        Workspace &w = ln.ws;
        HIP_OK_RC(hipMemcpyAsync(w.tok, tokens, (size_t)M * 4, hipMemcpyHostToDevice, st), -3);
        HIP_OK_RC(hipMemcpyAsync(w.off, offsets, (size_t)(n_seqs + 1) * 4, hipMemcpyHostToDevice, st), -3);
        const EmbedArgs ea = embed_args(ctx, R, w, w.tok, w.off, n_seqs, M);
        HIP_OK_RC(launch_embed(ctx->wtype, ea, (int)Mpad, st), -4);
        const int64_t E = ctx->hp.n_embd;
        HIP_OK_RC(hipMemcpyAsync(X_out, w.X, (size_t)(M * E) * 4, hipMemcpyDeviceToHost, st), -3);
        HIP_OK_RC(hipMemcpyAsync(q_out, w.Xa.q, (size_t)M * act_row_bytes(ctx->wtype, E), hipMemcpyDeviceToHost, st), -3);
        if (d_out && act_scale_bytes(ctx->wtype))
            HIP_OK_RC(hipMemcpyAsync(d_out, w.Xa.d, (size_t)(M * (E / 32)) * act_scale_bytes(ctx->wtype),
                                     hipMemcpyDeviceToHost, st), -3);
        ws_release(ln, st);
        HIP_OK_RC(hipStreamSynchronize(st), -3);
    } catch (const std::exception &e) {
        set_err("%s", e.what());
        return -5;
    }
    return 0;
}

int32_t bert_amd_debug_layers(bert_ctx *ctx, const int32_t *tokens, const int32_t *offsets, int32_t n_seqs,
                              float *X_out, void *q_out, void *d_out) {
    if (!ctx || !tokens || !offsets || n_seqs <= 0 || !X_out || !q_out) {
        set_err("bert_amd_debug_layers: invalid arguments");
        return -1;
    }
    const int64_t M = offsets[n_seqs];
    for (int s = 0; s < n_seqs; s++)
        if (offsets[s + 1] - offsets[s] <= 0 || offsets[s + 1] - offsets[s] > ctx->hp.n_max_tokens) {
            set_err("bert_amd_debug_layers: bad sentence length");
            return -2;
        }
    for (int64_t i = 0; i < M; i++)
        if (tokens[i] < 0 || tokens[i] >= ctx->hp.n_vocab) {
            set_err("bert_amd_debug_layers: token id out of range");
            return -2;
        }
    std::lock_guard<std::mutex> lk(ctx->mu);
    Replica &R = *ctx->reps[0];
    std::vector<void *> bufs;
    struct Free {
        std::vector<void *> &b;
        ~Free() {
            for (void *p : b) hipFree(p);
        }
    } fr{bufs};
    try {
        HIP_OK_RC(hipSetDevice(R.device), -3);
        Lane &ln = *R.lanes[0];
        const hipStream_t st = ln.stream;
        const int64_t E = ctx->hp.n_embd, S = ctx->hp.n_layer + 1;
        const size_t xb = (size_t)(M * E) * 4, qb = (size_t)M * act_row_bytes(ctx->wtype, E),
                     db = (size_t)(M * (E / 32)) * act_scale_bytes(ctx->wtype);
        DebugTap tap;
        int32_t *d_tok = nullptr, *d_off = nullptr;
        float *d_emb = nullptr;
        if (!dmalloc(bufs, &tap.X, S * xb) || !dmalloc(bufs, &tap.q, S * qb) || !dmalloc(bufs, &tap.d, S * db + 16) ||
            !dmalloc(bufs, &d_tok, (size_t)M * 4) || !dmalloc(bufs, &d_off, (size_t)(n_seqs + 1) * 4) ||
            !dmalloc(bufs, &d_emb, (size_t)n_seqs * E * 4))
            return -3;
        HIP_OK_RC(hipMemcpy(d_tok, tokens, (size_t)M * 4, hipMemcpyHostToDevice), -3);
        HIP_OK_RC(hipMemcpy(d_off, offsets, (size_t)(n_seqs + 1) * 4, hipMemcpyHostToDevice), -3);
        if (!ws_acquire(ln, st)) return -3;
        const bool ok = run_pipeline(ctx, R, ln, d_tok, d_off, offsets, n_seqs, d_emb, st, nullptr, &tap);
        ws_release(ln, st);
        HIP_OK_RC(hipStreamSynchronize(st), -3);
        if (!ok) return -4;
        HIP_OK_RC(hipMemcpy(X_out, tap.X, S * xb, hipMemcpyDeviceToHost), -3);
        HIP_OK_RC(hipMemcpy(q_out, tap.q, S * qb, hipMemcpyDeviceToHost), -3);
        if (d_out && db) HIP_OK_RC(hipMemcpy(d_out, tap.d, S * db, hipMemcpyDeviceToHost), -3);
    } catch (const std::exception &e) {
        set_err("%s", e.what());
        return -5;
    }
    return 0;
}

int32_t bert_amd_set_option(bert_ctx *ctx, const char *key, int32_t value) {
    if (!ctx || !key) {
        set_err("bert_amd_set_option: invalid arguments");
        return -1;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    return apply_option(ctx, key, value);
}

int32_t bert_amd_get_option(bert_ctx *ctx, const char *key, int32_t *value) {
    if (!ctx || !key || !value) {
        set_err("bert_amd_get_option: invalid arguments");
        return -1;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    const std::string k = key;
    const std::pair<const char *, int32_t> opts[] = {
        {"split", ctx->split}, {"pack", ctx->pack}, {"fuse_min", ctx->fuse_min}, {"unfused", ctx->unfused},
        {"small_rows", ctx->small_rows}, {"graph_seqs", ctx->graph_seqs}, {"small_qkva", ctx->small_qkva},
        {"encode_lanes", ctx->encode_lanes}, {"encode_merge", ctx->encode_merge},
        {"encode_merge_rows", ctx->encode_merge_rows}, {"qkva_ntw", ctx->qkva_ntw},
        {"i8_qkv", ctx->i8_qkv}, {"i8_up", ctx->i8_up}, {"i8_o", ctx->i8_o}, {"i8_down", ctx->i8_down},
        {"q41bf", ctx->q41bf}, {"emb_raw", ctx->emb_raw}, {"nt_x", ctx->nt_x},
        // resolved: FFN-up / FFN-down on the bf16 scale products (Q4_1 on the int8 GEMMs)
        {"q41bf_qkv", ctx->wtype == W_Q4_1 && ctx->i8_qkv && q41bf_for(ctx->q41bf, EPI_QKV)},
        {"q41bf_o", ctx->wtype == W_Q4_1 && ctx->i8_o && q41bf_for(ctx->q41bf, ctx->hp.n_embd == 384 ? EPI_LN : EPI_RESID)},
        {"q41bf_up", ctx->wtype == W_Q4_1 && ctx->i8_up && q41bf_for(ctx->q41bf, EPI_GELU_ACT)},
        {"q41bf_down", ctx->wtype == W_Q4_1 && ctx->i8_down &&
                           q41bf_for(ctx->q41bf, ctx->hp.n_embd == 384 ? EPI_LN : EPI_RESID)}};
    for (const auto &o : opts)
        if (k == o.first) {
            *value = o.second;
            return 0;
        }
    set_err("bert_amd_get_option: unknown option '%s'", key);
    return -2;
}

int32_t bert_amd_shard_cuts(int32_t n_seqs, const int32_t *n_tokens, int32_t n_replicas, int32_t *cut) {
    if (n_seqs < 0 || (n_seqs > 0 && !n_tokens) || n_replicas <= 0 || !cut) {
        set_err("bert_amd_shard_cuts: invalid arguments");
        return -1;
    }
    shard_cuts(n_seqs, n_tokens, n_replicas, cut);
    return 0;
}

int64_t bert_amd_workspace_rows(bert_ctx *ctx, int32_t slot) {
    if (!ctx || slot < 0 || slot >= (int32_t)ctx->reps.size()) return -1;
    std::lock_guard<std::mutex> lk(ctx->mu);
    int64_t rows = 0;  // the largest lane (bert_encode_batch may have added lanes)
    for (auto &ln : ctx->reps[slot]->lanes) rows = std::max(rows, ln->ws.cap_rows);
    return rows;
}

const char *bert_amd_last_error(void) { return g_err.c_str(); }

int32_t bert_amd_tokenize_json(const char *tokenizer_json, const char *text, int32_t *tokens, int32_t n_max_tokens,
                               int32_t frame, int32_t cls_id, int32_t sep_id, int32_t pad_id) {
    if (!tokenizer_json || !text || !tokens || n_max_tokens <= 0) {
        set_err("bert_amd_tokenize_json: invalid arguments");
        return -1;
    }
    try {
        WordPieceTokenizer tk;
        std::string err;
        if (!tk.load(tokenizer_json, err)) {
            set_err("%s", err.c_str());
            return -2;
        }
        const std::vector<int32_t> ids = tk.encode(text);
        if (frame) return frame_tokens(ids, cls_id, sep_id, pad_id, tokens, n_max_tokens);
        const int32_t n = (int32_t)std::min<size_t>(ids.size(), (size_t)n_max_tokens);
        std::copy(ids.begin(), ids.begin() + n, tokens);
        return n;
    } catch (const std::exception &e) {
        set_err("%s", e.what());
        return -3;
    }
}
