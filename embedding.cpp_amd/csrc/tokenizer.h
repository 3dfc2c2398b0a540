// tokenizer.h — native BERT WordPiece tokenizer driven by the HF tokenizer.json
// blob stored in the GGUF ("blob.tokenizer.json", reference bert.cpp:576-577).
//
// Replaces tokenizers-cpp@e47442f (Rust HF `tokenizers` behind a C++ shim,
// reference tokenizer.cpp:30-53; un-vendored, needs rustc) for the pipeline BERT
// checkpoints use: BertNormalizer (clean_text, handle_chinese_chars,
// strip_accents, lowercase) -> BertPreTokenizer (whitespace + punctuation
// split) -> WordPiece (greedy longest-match, "##" continuation,
// max_input_chars_per_word) -> truncation / padding from the JSON.
// Encode() returns content ids only (no [CLS]/[SEP]); bert_tokenize adds them,
// exactly like the reference (bert.cpp:738-781).
#pragma once
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace bertamd {

class WordPieceTokenizer {
public:
    bool load(const std::string &json, std::string &err);
    std::vector<int32_t> encode(const std::string &text) const;
    bool loaded() const { return !vocab_.empty(); }

    // exposed for tests
    std::string normalize(const std::string &text) const;
    std::vector<std::string> pre_tokenize(const std::string &normalized) const;

private:
    std::unordered_map<std::string, int32_t> vocab_;
    std::string prefix_ = "##";
    std::string unk_ = "[UNK]";
    int max_chars_ = 100;
    bool clean_text_ = true, chinese_ = true, lowercase_ = true;
    int strip_accents_ = -1;  // -1: follow lowercase (BERT default)
    int trunc_max_ = -1;      // content-token truncation (Encode without special tokens)
    int pad_len_ = -1;        // fixed padding length, -1 = none
    int32_t pad_id_ = 0;
    // added (special) tokens are matched verbatim before normalisation
    std::vector<std::pair<std::string, int32_t>> added_;
    bool added_first_[256] = {};  // first bytes of the added tokens
    int32_t unk_id_ = 0;
    // ASCII fast path (byte-for-byte the general path's decisions, tabulated
    // at load): 0 drop, 1 whitespace, 2 punctuation, 3 word character; and the
    // byte after normalisation
    uint8_t ascii_class_[128] = {}, ascii_norm_[128] = {};
    // the vocabulary again as an open-addressing table over one byte arena, so
    // that WordPiece looks candidate pieces up without building a string each
    struct VSlot {
        uint32_t hash = 0, off = 0, len = 0;
        int32_t id = -1;
    };
    std::string varena_;
    std::vector<VSlot> vslots_;
    uint32_t vmask_ = 0;
    // id of prefix_ + [p, p + n) (cont) or of [p, p + n), -1 if absent
    int32_t lookup(const char *p, size_t n, bool cont) const;
    void wordpiece(const std::string &w, size_t nchars, const size_t *off, std::vector<int32_t> &ids) const;
};

}  // namespace bertamd
