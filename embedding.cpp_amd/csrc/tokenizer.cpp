// tokenizer.cpp — see tokenizer.h.  Behaviour restated from the HF tokenizers
// BertNormalizer / BertPreTokenizer / WordPiece model (the engine that
// tokenizers-cpp wraps); verified against the python `tokenizers` package in
// tests/test_tokenizer.py.
#include "tokenizer.h"

#include <algorithm>
#include <cstring>
#include <memory>

namespace bertamd {
namespace {

#include "unicode_tables.inc"

// FNV-1a over bytes, continuing from h (the vocabulary table's hash)
inline uint32_t fnv1a(uint32_t h, const char *p, size_t n) {
    for (size_t i = 0; i < n; i++) h = (h ^ (uint8_t)p[i]) * 16777619u;
    return h;
}

template <size_t N>
bool in_ranges(const uint32_t (&r)[N][2], uint32_t cp) {
    size_t lo = 0, hi = N;
    while (lo < hi) {
        size_t mid = (lo + hi) / 2;
        if (cp < r[mid][0]) hi = mid;
        else if (cp > r[mid][1]) lo = mid + 1;
        else return true;
    }
    return false;
}

template <size_t N, size_t W>
const uint32_t *find_map(const uint32_t (&t)[N][W], uint32_t cp) {
    size_t lo = 0, hi = N;
    while (lo < hi) {
        size_t mid = (lo + hi) / 2;
        if (t[mid][0] < cp) lo = mid + 1;
        else hi = mid;
    }
    return (lo < N && t[lo][0] == cp) ? t[lo] : nullptr;
}

bool is_whitespace(uint32_t c) {
    if (c == '\t' || c == '\n' || c == '\r' || c == ' ') return true;
    // Unicode White_Space property (Rust char::is_whitespace)
    return (c >= 0x9 && c <= 0xD) || c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
           c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
bool is_control(uint32_t c) {
    if (c == '\t' || c == '\n' || c == '\r') return false;
    return in_ranges(kOther, c);
}
bool is_chinese(uint32_t c) {
    return (c >= 0x4E00 && c <= 0x9FFF) || (c >= 0x3400 && c <= 0x4DBF) || (c >= 0x20000 && c <= 0x2A6DF) ||
           (c >= 0x2A700 && c <= 0x2B73F) || (c >= 0x2B740 && c <= 0x2B81F) || (c >= 0x2B920 && c <= 0x2CEAF) ||
           (c >= 0xF900 && c <= 0xFAFF) || (c >= 0x2F800 && c <= 0x2FA1F);
}
bool is_punct(uint32_t c) {
    if ((c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126)) return true;
    return in_ranges(kPunct, c);
}

std::vector<uint32_t> utf8_decode(const std::string &s) {
    std::vector<uint32_t> out;
    out.reserve(s.size());
    size_t i = 0;
    while (i < s.size()) {
        const unsigned char c = (unsigned char)s[i];
        uint32_t cp;
        int n;
        if (c < 0x80) { cp = c; n = 1; }
        else if ((c >> 5) == 6) { cp = c & 0x1f; n = 2; }
        else if ((c >> 4) == 14) { cp = c & 0x0f; n = 3; }
        else if ((c >> 3) == 30) { cp = c & 0x07; n = 4; }
        else { out.push_back(0xFFFD); i++; continue; }
        if (i + n > s.size()) { out.push_back(0xFFFD); break; }
        bool ok = true;
        for (int k = 1; k < n; k++) {
            const unsigned char cc = (unsigned char)s[i + k];
            if ((cc >> 6) != 2) { ok = false; break; }
            cp = (cp << 6) | (cc & 0x3f);
        }
        if (!ok) { out.push_back(0xFFFD); i++; continue; }
        out.push_back(cp);
        i += n;
    }
    return out;
}

void utf8_append(std::string &o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3f)); }
    else if (cp < 0x10000) {
        o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3f)); o += (char)(0x80 | (cp & 0x3f));
    } else {
        o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3f));
        o += (char)(0x80 | ((cp >> 6) & 0x3f)); o += (char)(0x80 | (cp & 0x3f));
    }
}

void nfd_append(std::vector<uint32_t> &o, uint32_t cp) {
    if (cp >= 0xAC00 && cp <= 0xD7A3) {  // Hangul syllable, algorithmic
        const uint32_t s = cp - 0xAC00;
        o.push_back(0x1100 + s / 588);
        o.push_back(0x1161 + (s % 588) / 28);
        if (s % 28) o.push_back(0x11A7 + s % 28);
        return;
    }
    const uint32_t *m = find_map(kNFD, cp);
    if (!m) { o.push_back(cp); return; }
    for (int k = 1; k < 5 && m[k]; k++) o.push_back(m[k]);
}

// ------------------------------------------------------------- tiny JSON DOM
struct JVal {
    enum T { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
    bool b = false;
    double n = 0;
    std::string s;
    std::vector<JVal> a;
    std::vector<std::pair<std::string, JVal>> o;
    const JVal *get(const char *k) const {
        if (t != OBJ) return nullptr;
        for (auto &p : o)
            if (p.first == k) return &p.second;
        return nullptr;
    }
};

struct JParser {
    const char *p, *e;
    bool ok = true;
    void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) p++; }
    bool lit(const char *w) {
        size_t n = std::strlen(w);
        if ((size_t)(e - p) >= n && !std::memcmp(p, w, n)) { p += n; return true; }
        return false;
    }
    uint32_t hex4() {
        uint32_t v = 0;
        for (int i = 0; i < 4; i++) {
            if (p >= e) { ok = false; return 0; }
            char c = *p++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else ok = false;
        }
        return v;
    }
    std::string str() {
        std::string o;
        if (p >= e || *p != '"') { ok = false; return o; }
        p++;
        while (p < e && *p != '"') {
            char c = *p++;
            if (c != '\\') { o += c; continue; }
            if (p >= e) { ok = false; break; }
            char x = *p++;
            switch (x) {
                case '"': o += '"'; break;
                case '\\': o += '\\'; break;
                case '/': o += '/'; break;
                case 'b': o += '\b'; break;
                case 'f': o += '\f'; break;
                case 'n': o += '\n'; break;
                case 'r': o += '\r'; break;
                case 't': o += '\t'; break;
                case 'u': {
                    uint32_t cp = hex4();
                    if (cp >= 0xD800 && cp <= 0xDBFF && p + 1 < e && p[0] == '\\' && p[1] == 'u') {
                        p += 2;
                        uint32_t lo = hex4();
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    utf8_append(o, cp);
                } break;
                default: ok = false;
            }
        }
        if (p < e) p++; else ok = false;
        return o;
    }
    JVal val(int depth = 0) {
        JVal v;
        ws();
        if (p >= e || depth > 64) { ok = false; return v; }
        if (*p == '{') {
            v.t = JVal::OBJ; p++; ws();
            if (p < e && *p == '}') { p++; return v; }
            while (ok) {
                ws();
                std::string k = str();
                ws();
                if (p >= e || *p != ':') { ok = false; break; }
                p++;
                v.o.emplace_back(std::move(k), val(depth + 1));
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == '}') { p++; break; }
                ok = false;
            }
        } else if (*p == '[') {
            v.t = JVal::ARR; p++; ws();
            if (p < e && *p == ']') { p++; return v; }
            while (ok) {
                v.a.push_back(val(depth + 1));
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == ']') { p++; break; }
                ok = false;
            }
        } else if (*p == '"') {
            v.t = JVal::STR; v.s = str();
        } else if (lit("true")) { v.t = JVal::BOOL; v.b = true; }
        else if (lit("false")) { v.t = JVal::BOOL; v.b = false; }
        else if (lit("null")) { v.t = JVal::NUL; }
        else {
            char *end = nullptr;
            v.t = JVal::NUM;
            v.n = std::strtod(p, &end);
            if (end == p) ok = false;
            p = end;
        }
        return v;
    }
};

}  // namespace

bool WordPieceTokenizer::load(const std::string &json, std::string &err) {
    JParser jp{json.data(), json.data() + json.size()};
    JVal root = jp.val();
    if (!jp.ok || root.t != JVal::OBJ) { err = "tokenizer.json: parse error"; return false; }
    const JVal *model = root.get("model");
    if (!model || !model->get("vocab")) { err = "tokenizer.json: no model.vocab"; return false; }
    if (const JVal *t = model->get("type"); t && t->t == JVal::STR && t->s != "WordPiece") {
        err = "tokenizer.json: unsupported model type " + t->s;
        return false;
    }
    const JVal *voc = model->get("vocab");
    if (voc->t != JVal::OBJ) { err = "tokenizer.json: vocab is not an object"; return false; }
    vocab_.reserve(voc->o.size() * 2);
    for (auto &kv : voc->o) vocab_[kv.first] = (int32_t)kv.second.n;
    if (const JVal *v = model->get("unk_token"); v && v->t == JVal::STR) unk_ = v->s;
    if (const JVal *v = model->get("continuing_subword_prefix"); v && v->t == JVal::STR) prefix_ = v->s;
    if (const JVal *v = model->get("max_input_chars_per_word"); v && v->t == JVal::NUM) max_chars_ = (int)v->n;
    if (const JVal *nm = root.get("normalizer"); nm && nm->t == JVal::OBJ) {
        if (const JVal *v = nm->get("clean_text"); v && v->t == JVal::BOOL) clean_text_ = v->b;
        if (const JVal *v = nm->get("handle_chinese_chars"); v && v->t == JVal::BOOL) chinese_ = v->b;
        if (const JVal *v = nm->get("lowercase"); v && v->t == JVal::BOOL) lowercase_ = v->b;
        if (const JVal *v = nm->get("strip_accents"); v && v->t == JVal::BOOL) strip_accents_ = v->b ? 1 : 0;
    }
    if (const JVal *tr = root.get("truncation"); tr && tr->t == JVal::OBJ)
        if (const JVal *v = tr->get("max_length"); v && v->t == JVal::NUM) trunc_max_ = (int)v->n;
    if (const JVal *pd = root.get("padding"); pd && pd->t == JVal::OBJ) {
        if (const JVal *st = pd->get("strategy"); st && st->t == JVal::OBJ)
            if (const JVal *f = st->get("Fixed"); f && f->t == JVal::NUM) pad_len_ = (int)f->n;
        if (const JVal *v = pd->get("pad_id"); v && v->t == JVal::NUM) pad_id_ = (int32_t)v->n;
    }
    if (const JVal *at = root.get("added_tokens"); at && at->t == JVal::ARR)
        for (auto &t : at->a) {
            const JVal *c = t.get("content"), *id = t.get("id");
            if (c && id && c->t == JVal::STR && !c->s.empty()) added_.emplace_back(c->s, (int32_t)id->n);
        }
    std::sort(added_.begin(), added_.end(), [](auto &a, auto &b) { return a.first.size() > b.first.size(); });
    if (!vocab_.count(unk_)) { err = "tokenizer.json: unk token not in vocab"; return false; }
    unk_id_ = vocab_.at(unk_);
    {
        size_t cap = 16;
        while (cap < 2 * vocab_.size()) cap *= 2;
        vslots_.assign(cap, VSlot{});
        vmask_ = (uint32_t)(cap - 1);
        varena_.clear();
        for (auto &kv : vocab_) {
            VSlot e;
            e.hash = fnv1a(2166136261u, kv.first.data(), kv.first.size());
            e.off = (uint32_t)varena_.size();
            e.len = (uint32_t)kv.first.size();
            e.id = kv.second;
            varena_ += kv.first;
            uint32_t i = e.hash & vmask_;
            while (vslots_[i].id >= 0) i = (i + 1) & vmask_;
            vslots_[i] = e;
        }
    }
    for (auto &a : added_) added_first_[(unsigned char)a.first[0]] = true;
    // the ASCII fast path's tables, from the same predicates normalize() and
    // pre_tokenize() apply (NFD and accent stripping are the identity on ASCII)
    for (uint32_t c = 0; c < 128; c++) {
        uint32_t n = c;
        bool drop = false;
        if (clean_text_) {
            if (c == 0 || is_control(c)) drop = true;
            else if (is_whitespace(c)) n = ' ';
        }
        if (!drop && lowercase_)
            if (const uint32_t *m = find_map(kLower, n)) n = m[1];
        ascii_norm_[c] = (uint8_t)n;
        ascii_class_[c] = drop ? 0 : is_whitespace(n) ? 1 : is_punct(n) ? 2 : 3;
    }
    return true;
}

int32_t WordPieceTokenizer::lookup(const char *p, size_t n, bool cont) const {
    const size_t pl = cont ? prefix_.size() : 0;
    uint32_t h = 2166136261u;
    if (cont) h = fnv1a(h, prefix_.data(), pl);
    h = fnv1a(h, p, n);
    for (uint32_t i = h & vmask_;; i = (i + 1) & vmask_) {
        const VSlot &e = vslots_[i];
        if (e.id < 0) return -1;
        if (e.hash == h && e.len == pl + n && std::memcmp(varena_.data() + e.off, prefix_.data(), pl) == 0 &&
            std::memcmp(varena_.data() + e.off + pl, p, n) == 0)
            return e.id;
    }
}

// WordPiece on one pre-token w of nchars characters (byte offset of char k:
// off[k]): greedy longest match from the left, "##" continuations, [UNK] for
// the whole word if any piece is missing.
void WordPieceTokenizer::wordpiece(const std::string &w, size_t nchars, const size_t *off,
                                   std::vector<int32_t> &ids) const {
    if ((int)nchars > max_chars_) { ids.push_back(unk_id_); return; }
    const size_t base = ids.size();
    size_t start = 0;
    while (start < nchars) {
        size_t end = nchars;
        int32_t found = -1;
        while (start < end) {
            found = lookup(w.data() + off[start], off[end] - off[start], start > 0);
            if (found >= 0) break;
            end--;
        }
        if (found < 0) {
            ids.resize(base);
            ids.push_back(unk_id_);
            return;
        }
        ids.push_back(found);
        start = end;
    }
}

std::string WordPieceTokenizer::normalize(const std::string &text) const {
    std::vector<uint32_t> cps = utf8_decode(text), t;
    t.reserve(cps.size());
    for (uint32_t c : cps) {
        if (clean_text_) {
            if (c == 0 || c == 0xFFFD || is_control(c)) continue;
            if (is_whitespace(c)) c = ' ';
        }
        if (chinese_ && is_chinese(c)) {
            t.push_back(' '); t.push_back(c); t.push_back(' ');
        } else {
            t.push_back(c);
        }
    }
    const bool strip = strip_accents_ < 0 ? lowercase_ : strip_accents_ == 1;
    if (strip) {
        std::vector<uint32_t> d;
        d.reserve(t.size());
        for (uint32_t c : t) nfd_append(d, c);
        t.clear();
        for (uint32_t c : d)
            if (!in_ranges(kMn, c)) t.push_back(c);
    }
    std::string out;
    out.reserve(text.size());
    for (uint32_t c : t) {
        if (lowercase_) {
            if (const uint32_t *m = find_map(kLower, c)) {
                for (int k = 1; k < 4 && m[k]; k++) utf8_append(out, m[k]);
                continue;
            }
        }
        utf8_append(out, c);
    }
    return out;
}

std::vector<std::string> WordPieceTokenizer::pre_tokenize(const std::string &normalized) const {
    std::vector<std::string> words;
    std::string cur;
    for (uint32_t c : utf8_decode(normalized)) {
        if (is_whitespace(c)) {
            if (!cur.empty()) { words.push_back(cur); cur.clear(); }
        } else if (is_punct(c)) {
            if (!cur.empty()) { words.push_back(cur); cur.clear(); }
            std::string p;
            utf8_append(p, c);
            words.push_back(p);
        } else {
            utf8_append(cur, c);
        }
    }
    if (!cur.empty()) words.push_back(cur);
    return words;
}

std::vector<int32_t> WordPieceTokenizer::encode(const std::string &text) const {
    std::vector<int32_t> ids;
    const int32_t unk = unk_id_;
    // split out added (special) tokens first: they are never normalised
    std::vector<std::pair<std::string, int32_t>> pieces;  // id >= 0: special token
    {
        size_t i = 0, start = 0;
        while (i < text.size()) {
            bool hit = false;
            if (added_first_[(unsigned char)text[i]])
            for (auto &a : added_) {
                if (text.compare(i, a.first.size(), a.first) == 0) {
                    if (i > start) pieces.emplace_back(text.substr(start, i - start), -1);
                    pieces.emplace_back(a.first, a.second);
                    i += a.first.size();
                    start = i;
                    hit = true;
                    break;
                }
            }
            if (!hit) i++;
        }
        if (start < text.size()) pieces.emplace_back(text.substr(start), -1);
    }
    std::string word;
    std::vector<size_t> aoff;
    for (auto &pc : pieces) {
        if (pc.second >= 0) { ids.push_back(pc.second); continue; }
        const std::string &t = pc.first;
        if (std::all_of(t.begin(), t.end(), [](char ch) { return (unsigned char)ch < 0x80; })) {
            // ASCII: normalise, split and look up in one pass, one byte per char
            auto flush = [&]() {
                if (word.empty()) return;
                if (aoff.size() < word.size() + 1) {
                    aoff.resize(word.size() + 1);
                    for (size_t k = 0; k < aoff.size(); k++) aoff[k] = k;
                }
                wordpiece(word, word.size(), aoff.data(), ids);
                word.clear();
            };
            for (char ch : t) {
                const uint8_t c = (uint8_t)ch, cls = ascii_class_[c];
                if (cls == 0) continue;
                if (cls == 1) { flush(); continue; }
                if (cls == 2) {
                    flush();
                    word.assign(1, (char)ascii_norm_[c]);
                    flush();
                    continue;
                }
                word += (char)ascii_norm_[c];
            }
            flush();
            continue;
        }
        for (const std::string &w : pre_tokenize(normalize(pc.first))) {
            const std::vector<uint32_t> chars = utf8_decode(w);
            if ((int)chars.size() > max_chars_) { ids.push_back(unk); continue; }
            // byte offset of each char boundary
            std::vector<size_t> off(chars.size() + 1, 0);
            {
                size_t b = 0;
                for (size_t k = 0; k < chars.size(); k++) {
                    off[k] = b;
                    std::string tmp;
                    utf8_append(tmp, chars[k]);
                    b += tmp.size();
                }
                off[chars.size()] = b;
            }
            std::vector<int32_t> sub;
            size_t start = 0;
            bool bad = false;
            while (start < chars.size()) {
                size_t end = chars.size();
                int32_t found = -1;
                while (start < end) {
                    found = lookup(w.data() + off[start], off[end] - off[start], start > 0);
                    if (found >= 0) break;
                    end--;
                }
                if (found < 0) { bad = true; break; }
                sub.push_back(found);
                start = end;
            }
            if (bad) ids.push_back(unk);
            else ids.insert(ids.end(), sub.begin(), sub.end());
        }
    }
    if (trunc_max_ >= 0 && (int)ids.size() > trunc_max_) ids.resize(trunc_max_);
    if (pad_len_ > 0 && (int)ids.size() < pad_len_) ids.resize(pad_len_, pad_id_);
    return ids;
}

}  // namespace bertamd
