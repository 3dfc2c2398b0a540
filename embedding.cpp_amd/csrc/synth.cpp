// synth.cpp — deterministic synthetic BERT GGUF generator (no network, no HF
// weights in this environment: SURVEY.md §8(d) "Synthetic inputs").
//
// Writes a GGUF with exactly the KV keys and tensor names/shapes the reference
// loader demands (reference bert.cpp:496-513, 515-578, 623-652; converter
// models/convert-to-gguf.py:145-340), with weights drawn from a splitmix64-seeded
// normal distribution, then converted to the requested ftype the way the
// reference tooling does it: f16 for 2-D *.weight tensors
// (convert-to-gguf.py:314-321), Q4_0/Q4_1 for every 2-D *.weight tensor
// (bert.cpp:1431-1436) through the ggml reference quantisers.
//
// Determinism: element i of tensor t comes from a stream seeded by
// (seed, t, i / CHUNK), so multithreaded generation is bit-reproducible on any
// host with this image's libm.
#include "bert_amd.h"
#include "ggml_formats.h"
#include "gguf_io.h"

#include <cmath>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

namespace bertamd {
namespace {

inline uint64_t splitmix64(uint64_t &s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

constexpr int64_t CHUNK = 1 << 16;

// N(mean, std) via Box-Muller on 53-bit uniforms.
void fill_normal(float *dst, int64_t n, uint64_t seed, uint64_t tensor_id, float mean, float std) {
    const int64_t nchunk = (n + CHUNK - 1) / CHUNK;
    auto work = [&](int64_t c0, int64_t c1) {
        for (int64_t c = c0; c < c1; c++) {
            uint64_t s = seed * 0x100000001b3ull ^ (tensor_id << 40) ^ (uint64_t)c;
            splitmix64(s);
            const int64_t i0 = c * CHUNK, i1 = std::min(n, i0 + CHUNK);
            for (int64_t i = i0; i < i1; i += 2) {
                double u1 = ((splitmix64(s) >> 11) + 1) * 0x1.0p-53;  // (0, 1]
                double u2 = (splitmix64(s) >> 11) * 0x1.0p-53;        // [0, 1)
                double r = std::sqrt(-2.0 * std::log(u1));
                double a = 6.283185307179586 * u2;
                dst[i] = (float)(mean + std * r * std::cos(a));
                if (i + 1 < i1) dst[i + 1] = (float)(mean + std * r * std::sin(a));
            }
        }
    };
    unsigned nt = std::thread::hardware_concurrency();
    if (nt > 16) nt = 16;
    if (nt <= 1 || nchunk < 4) { work(0, nchunk); return; }
    std::vector<std::thread> th;
    const int64_t per = (nchunk + nt - 1) / nt;
    for (unsigned t = 0; t < nt; t++) {
        int64_t c0 = t * per, c1 = std::min(nchunk, c0 + per);
        if (c0 < c1) th.emplace_back(work, c0, c1);
    }
    for (auto &t : th) t.join();
}

std::vector<uint8_t> convert(const std::vector<float> &x, int64_t ne0, uint32_t type) {
    const int64_t n = (int64_t)x.size();
    std::vector<uint8_t> out(ggml_row_bytes(type, ne0) * (size_t)(n / ne0));
    switch (type) {
        case GT_F32: std::memcpy(out.data(), x.data(), (size_t)n * 4); break;
        case GT_F16: {
            uint16_t *o = (uint16_t *)out.data();
            for (int64_t i = 0; i < n; i++) o[i] = f32_to_f16(x[i]);
        } break;
        case GT_Q4_0: quantize_row_q4_0(x.data(), (block_q4_0 *)out.data(), n); break;
        case GT_Q4_1: quantize_row_q4_1(x.data(), (block_q4_1 *)out.data(), n); break;
    }
    return out;
}

// A WordPiece vocabulary with BERT's special-token ids ([PAD]=0, [UNK]=100,
// [CLS]=101, [SEP]=102, [MASK]=103), single characters, their ##-continuations,
// then synthetic word pieces.
std::vector<std::string> make_vocab(int n_vocab) {
    std::vector<std::string> v;
    v.reserve(n_vocab);
    v.push_back("[PAD]");
    for (int i = 1; i < 100; i++) v.push_back("[unused" + std::to_string(i - 1) + "]");
    v.push_back("[UNK]");
    v.push_back("[CLS]");
    v.push_back("[SEP]");
    v.push_back("[MASK]");
    for (int c = 33; c < 127 && (int)v.size() < n_vocab; c++) {
        if (c >= 'A' && c <= 'Z') continue;  // the normaliser lowercases
        v.push_back(std::string(1, (char)c));
    }
    for (int c = 'a'; c <= 'z' && (int)v.size() < n_vocab; c++) v.push_back(std::string("##") + (char)c);
    for (int c = '0'; c <= '9' && (int)v.size() < n_vocab; c++) v.push_back(std::string("##") + (char)c);
    static const char *syl[] = {"ba", "ce", "di", "fo", "gu", "ha", "je", "ki", "lo", "mu", "na", "pe",
                                "qi", "ro", "su", "ta", "ve", "wi", "xo", "yu", "za", "an", "er", "in",
                                "on", "un", "st", "th", "ch", "sh", "ly", "ng"};
    const int ns = (int)(sizeof(syl) / sizeof(syl[0]));
    for (uint64_t k = 0; (int)v.size() < n_vocab; k++) {
        std::string w;
        uint64_t t = k;
        do { w += syl[t % ns]; t /= ns; } while (t);
        v.push_back((k % 3 == 2) ? "##" + w : w);
    }
    return v;
}

std::string json_escape(const std::string &s) {
    std::string o;
    for (char c : s) {
        if (c == '"' || c == '\\') { o += '\\'; o += c; }
        else o += c;
    }
    return o;
}

// HF tokenizer.json for a BERT WordPiece pipeline (the blob the reference keeps
// under "blob.tokenizer.json", bert.cpp:576-577).
std::string make_tokenizer_json(const std::vector<std::string> &vocab, int max_len) {
    std::string j;
    j.reserve(vocab.size() * 24 + 2048);
    j += "{\"version\":\"1.0\",\"truncation\":{\"direction\":\"Right\",\"max_length\":";
    j += std::to_string(max_len - 2);
    j += ",\"strategy\":\"LongestFirst\",\"stride\":0},\"padding\":null,\"added_tokens\":[";
    const int special[] = {0, 100, 101, 102, 103};
    for (int i = 0; i < 5; i++) {
        if (i) j += ",";
        j += "{\"id\":" + std::to_string(special[i]) + ",\"content\":\"" + vocab[special[i]] +
             "\",\"single_word\":false,\"lstrip\":false,\"rstrip\":false,\"normalized\":false,\"special\":true}";
    }
    j += "],\"normalizer\":{\"type\":\"BertNormalizer\",\"clean_text\":true,\"handle_chinese_chars\":true,"
         "\"strip_accents\":null,\"lowercase\":true},\"pre_tokenizer\":{\"type\":\"BertPreTokenizer\"},"
         "\"post_processor\":null,\"decoder\":{\"type\":\"WordPiece\",\"prefix\":\"##\",\"cleanup\":true},"
         "\"model\":{\"type\":\"WordPiece\",\"unk_token\":\"[UNK]\",\"continuing_subword_prefix\":\"##\","
         "\"max_input_chars_per_word\":100,\"vocab\":{";
    for (size_t i = 0; i < vocab.size(); i++) {
        if (i) j += ",";
        j += "\"" + json_escape(vocab[i]) + "\":" + std::to_string(i);
    }
    j += "}}}";
    return j;
}

}  // namespace
}  // namespace bertamd

using namespace bertamd;

extern "C" BERT_API int bert_amd_synth_model(const char *path, int32_t n_vocab, int32_t n_max_tokens,
                                             int32_t n_embd, int32_t n_intermediate, int32_t n_head,
                                             int32_t n_layer, int32_t ftype, uint64_t seed, float w_std) {
    if (!path || n_vocab < 200 || n_embd % 32 || n_intermediate % 32 || n_head <= 0 || n_embd % n_head ||
        n_layer <= 0 || n_max_tokens <= 0 || ftype < 0 || ftype > 3) {
        std::fprintf(stderr, "bert_amd_synth_model: invalid arguments\n");
        return -1;
    }
    const uint32_t wtype = ftype == 0 ? GT_F32 : ftype == 1 ? GT_F16 : ftype == 2 ? GT_Q4_0 : GT_Q4_1;
    GGUFWriter w;
    w.add_str("general.architecture", "bert");
    w.add_str("general.name", "synthetic-bert");
    w.add_u32("bert.context_length", (uint32_t)n_max_tokens);
    w.add_u32("bert.embedding_length", (uint32_t)n_embd);
    w.add_u32("bert.block_count", (uint32_t)n_layer);
    w.add_u32("bert.feed_forward_length", (uint32_t)n_intermediate);
    w.add_u32("bert.rope.dimension_count", (uint32_t)(n_embd / n_head));
    w.add_u32("bert.attention.head_count", (uint32_t)n_head);
    w.add_u32("bert.attention.head_count_kv", (uint32_t)n_head);
    w.add_f32("bert.attention.layer_norm_epsilon", 1e-12f);
    if (ftype >= 2) w.add_u32("general.file_type", (uint32_t)ftype);
    std::vector<std::string> vocab = make_vocab(n_vocab);
    w.add_str("blob.tokenizer.json", make_tokenizer_json(vocab, n_max_tokens));
    w.add_str("tokenizer.ggml.model", "bert");
    w.add_arr_str("tokenizer.ggml.tokens", vocab);
    w.add_arr_f32("tokenizer.ggml.scores", std::vector<float>(vocab.size(), 0.0f));
    w.add_arr_i32("tokenizer.ggml.token_type", std::vector<int32_t>(vocab.size(), 1));
    w.add_u32("tokenizer.ggml.unknown_token_id", 100);
    w.add_u32("tokenizer.ggml.seperator_token_id", 102);
    w.add_u32("tokenizer.ggml.padding_token_id", 0);
    w.add_u32("tokenizer.ggml.cls_token_id", 101);

    uint64_t tid = 0;
    auto add = [&](const std::string &name, std::vector<int64_t> ne, float mean, float std) {
        int64_t n = 1;
        for (auto d : ne) n *= d;
        std::vector<float> x((size_t)n);
        fill_normal(x.data(), n, seed, ++tid, mean, std);
        const bool is_w2d = ne.size() == 2 && name.size() > 6 && name.compare(name.size() - 6, 6, "weight") == 0;
        const uint32_t t = is_w2d ? wtype : GT_F32;
        w.add_tensor(name, ne, t, convert(x, ne[0], t));
    };
    const int64_t E = n_embd, I = n_intermediate;
    const float emb_std = 0.05f, b_std = 0.01f, lnw_std = 0.05f;
    add("embeddings.word_embeddings.weight", {E, n_vocab}, 0.0f, emb_std);
    add("embeddings.position_embeddings.weight", {E, n_max_tokens}, 0.0f, emb_std);
    add("embeddings.token_type_embeddings.weight", {E, 2}, 0.0f, emb_std);
    add("embeddings.LayerNorm.weight", {E}, 1.0f, lnw_std);
    add("embeddings.LayerNorm.bias", {E}, 0.0f, b_std);
    for (int il = 0; il < n_layer; il++) {
        const std::string p = "encoder.layer." + std::to_string(il) + ".";
        add(p + "attention.self.query.weight", {E, E}, 0.0f, w_std);
        add(p + "attention.self.query.bias", {E}, 0.0f, b_std);
        add(p + "attention.self.key.weight", {E, E}, 0.0f, w_std);
        add(p + "attention.self.key.bias", {E}, 0.0f, b_std);
        add(p + "attention.self.value.weight", {E, E}, 0.0f, w_std);
        add(p + "attention.self.value.bias", {E}, 0.0f, b_std);
        add(p + "attention.output.dense.weight", {E, E}, 0.0f, w_std);
        add(p + "attention.output.dense.bias", {E}, 0.0f, b_std);
        add(p + "attention.output.LayerNorm.weight", {E}, 1.0f, lnw_std);
        add(p + "attention.output.LayerNorm.bias", {E}, 0.0f, b_std);
        add(p + "intermediate.dense.weight", {E, I}, 0.0f, w_std);
        add(p + "intermediate.dense.bias", {I}, 0.0f, b_std);
        add(p + "output.dense.weight", {I, E}, 0.0f, w_std);
        add(p + "output.dense.bias", {E}, 0.0f, b_std);
        add(p + "output.LayerNorm.weight", {E}, 1.0f, lnw_std);
        add(p + "output.LayerNorm.bias", {E}, 0.0f, b_std);
    }
    std::string err;
    if (!w.write(path, err)) {
        std::fprintf(stderr, "bert_amd_synth_model: %s\n", err.c_str());
        return -2;
    }
    return 0;
}
