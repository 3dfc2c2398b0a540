// gguf_io.cpp — see gguf_io.h.
#include "gguf_io.h"

#include "ggml_formats.h"

#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace bertamd {

namespace {

struct Cursor {
    const uint8_t *p, *end;
    bool ok = true;
    bool need(size_t n) {
        if (!ok || (size_t)(end - p) < n) { ok = false; return false; }
        return true;
    }
    template <typename T> T get() {
        T v{};
        if (need(sizeof(T))) { std::memcpy(&v, p, sizeof(T)); p += sizeof(T); }
        return v;
    }
    std::string str() {
        const uint64_t n = get<uint64_t>();
        if (!need(n)) return {};
        std::string s((const char *)p, (size_t)n);
        p += n;
        return s;
    }
};

size_t scalar_size(uint32_t t) {
    switch (t) {
        case GV_U8: case GV_I8: case GV_BOOL: return 1;
        case GV_U16: case GV_I16: return 2;
        case GV_U32: case GV_I32: case GV_F32: return 4;
        case GV_U64: case GV_I64: case GV_F64: return 8;
        default: return 0;
    }
}

bool read_value(Cursor &c, uint32_t type, GGUFValue &v) {
    v.type = type;
    switch (type) {
        case GV_U8: v.u = c.get<uint8_t>(); break;
        case GV_I8: v.u = (uint64_t)(int64_t)c.get<int8_t>(); break;
        case GV_U16: v.u = c.get<uint16_t>(); break;
        case GV_I16: v.u = (uint64_t)(int64_t)c.get<int16_t>(); break;
        case GV_U32: v.u = c.get<uint32_t>(); break;
        case GV_I32: v.u = (uint64_t)(int64_t)c.get<int32_t>(); break;
        case GV_U64: v.u = c.get<uint64_t>(); break;
        case GV_I64: v.u = (uint64_t)c.get<int64_t>(); break;
        case GV_BOOL: v.u = c.get<uint8_t>(); break;
        case GV_F32: v.f = c.get<float>(); break;
        case GV_F64: v.f = c.get<double>(); break;
        case GV_STR: v.s = c.str(); break;
        case GV_ARR: {
            v.arr_type = c.get<uint32_t>();
            v.arr_n = c.get<uint64_t>();
            if (!c.ok) return false;
            const uint64_t left = (uint64_t)(c.end - c.p);
            if (v.arr_type == GV_STR) {
                if (v.arr_n > left / 8) return false;  // every string needs at least its 8-byte length
                v.arr_str.reserve((size_t)v.arr_n);
                for (uint64_t i = 0; i < v.arr_n && c.ok; i++) v.arr_str.push_back(c.str());
            } else {
                const size_t es = scalar_size(v.arr_type);
                if (es == 0) return false;  // nested arrays are not used by BERT GGUFs
                if (v.arr_n > left / es) return false;  // (also keeps arr_n * es from wrapping)
                const size_t nb = (size_t)v.arr_n * es;
                if (!c.need(nb)) return false;
                v.arr_raw.assign(c.p, c.p + nb);
                c.p += nb;
            }
        } break;
        default: return false;
    }
    return c.ok;
}

void put_bytes(std::vector<uint8_t> &o, const void *p, size_t n) {
    const uint8_t *b = (const uint8_t *)p;
    o.insert(o.end(), b, b + n);
}
template <typename T> void put(std::vector<uint8_t> &o, T v) { put_bytes(o, &v, sizeof(T)); }
void put_str(std::vector<uint8_t> &o, const std::string &s) {
    put<uint64_t>(o, s.size());
    put_bytes(o, s.data(), s.size());
}

void write_value(std::vector<uint8_t> &o, const GGUFValue &v) {
    switch (v.type) {
        case GV_U8: case GV_I8: case GV_BOOL: put<uint8_t>(o, (uint8_t)v.u); break;
        case GV_U16: case GV_I16: put<uint16_t>(o, (uint16_t)v.u); break;
        case GV_U32: case GV_I32: put<uint32_t>(o, (uint32_t)v.u); break;
        case GV_U64: case GV_I64: put<uint64_t>(o, v.u); break;
        case GV_F32: put<float>(o, (float)v.f); break;
        case GV_F64: put<double>(o, v.f); break;
        case GV_STR: put_str(o, v.s); break;
        case GV_ARR:
            put<uint32_t>(o, v.arr_type);
            put<uint64_t>(o, v.arr_n);
            if (v.arr_type == GV_STR) {
                for (auto &s : v.arr_str) put_str(o, s);
            } else {
                put_bytes(o, v.arr_raw.data(), v.arr_raw.size());
            }
            break;
        default: break;
    }
}

}  // namespace

GGUFFile::~GGUFFile() {
    if (map_) munmap(map_, map_size_);
    if (fd_ >= 0) close(fd_);
}

bool GGUFFile::open(const std::string &path, std::string &err) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) { err = "failed to open " + path + ": " + std::strerror(errno); return false; }
    struct stat st;
    if (fstat(fd_, &st) != 0 || st.st_size < 24) { err = "not a GGUF file: " + path; return false; }
    map_size_ = (size_t)st.st_size;
    map_ = mmap(nullptr, map_size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (map_ == MAP_FAILED) { map_ = nullptr; err = "mmap failed: " + path; return false; }
    Cursor c{(const uint8_t *)map_, (const uint8_t *)map_ + map_size_};
    const uint32_t magic = c.get<uint32_t>();
    if (magic != 0x46554747u) { err = "bad GGUF magic in " + path; return false; }
    version = c.get<uint32_t>();
    if (version != 2 && version != 3) { err = "unsupported GGUF version " + std::to_string(version); return false; }
    const uint64_t n_tensors = c.get<uint64_t>();
    const uint64_t n_kv = c.get<uint64_t>();
    for (uint64_t i = 0; i < n_kv && c.ok; i++) {
        std::string key = c.str();
        const uint32_t t = c.get<uint32_t>();
        GGUFValue v;
        if (!read_value(c, t, v)) { err = "bad KV '" + key + "'"; return false; }
        kv.emplace_back(std::move(key), std::move(v));
    }
    if (const GGUFValue *a = find("general.alignment")) {
        if (a->type != GV_U32) { err = "bad alignment"; return false; }
        alignment = (size_t)a->u;
    }
    if (alignment == 0 || alignment > (1u << 20) || (alignment & (alignment - 1))) { err = "bad alignment"; return false; }
    // every tensor info needs at least 8 (name) + 4 (rank) + 4 (type) + 8 (offset) bytes
    if (n_tensors > (uint64_t)(c.end - c.p) / 24) { err = "truncated GGUF header"; return false; }
    for (uint64_t i = 0; i < n_tensors && c.ok; i++) {
        GGUFTensor t;
        t.name = c.str();
        const uint32_t nd = c.get<uint32_t>();
        if (nd > 4) { err = "tensor rank > 4"; return false; }
        for (uint32_t d = 0; d < nd; d++) {
            const uint64_t ne = c.get<uint64_t>();
            // ne >= 1 and < 2^31 per dimension: the row product below cannot wrap
            if (c.ok && (ne == 0 || ne >= (1ull << 31))) { err = "bad tensor shape: " + t.name; return false; }
            t.ne.push_back((int64_t)ne);
        }
        t.type = c.get<uint32_t>();
        t.offset = c.get<uint64_t>();
        tensors.push_back(std::move(t));
    }
    if (!c.ok) { err = "truncated GGUF header"; return false; }
    size_t data_off = (size_t)(c.p - (const uint8_t *)map_);
    data_off = (data_off + alignment - 1) / alignment * alignment;
    if (data_off > map_size_) { err = "truncated GGUF file"; return false; }
    const size_t data_size = map_size_ - data_off;
    for (auto &t : tensors) {
        const int64_t ne0 = t.ne.empty() ? 1 : t.ne[0];
        const size_t rb = ggml_row_bytes(t.type, ne0);
        if (rb == 0) { err = "unsupported tensor type " + std::to_string(t.type) + " for " + t.name; return false; }
        if ((t.type == GT_Q4_0 || t.type == GT_Q4_1 || t.type == GT_Q8_0 || t.type == GT_Q8_1) && ne0 % QK) {
            err = "row length not a multiple of the block size: " + t.name;
            return false;
        }
        // nrows <= data_size / rb, checked dimension by dimension (no overflow)
        uint64_t rows = 1;
        const uint64_t max_rows = data_size / rb;
        for (size_t d = 1; d < t.ne.size(); d++) {
            if ((uint64_t)t.ne[d] > max_rows / rows) { err = "tensor data out of range: " + t.name; return false; }
            rows *= (uint64_t)t.ne[d];
        }
        t.nbytes = rb * (size_t)rows;
        if (t.offset > data_size || t.nbytes > data_size - t.offset) {
            err = "tensor data out of range: " + t.name;
            return false;
        }
        t.data = (const uint8_t *)map_ + data_off + t.offset;
    }
    return true;
}

const GGUFValue *GGUFFile::find(const std::string &key) const {
    for (auto &p : kv)
        if (p.first == key) return &p.second;
    return nullptr;
}

const GGUFTensor *GGUFFile::tensor(const std::string &name) const {
    for (auto &t : tensors)
        if (t.name == name) return &t;
    return nullptr;
}

void GGUFWriter::add_u32(const std::string &k, uint32_t v) { GGUFValue x; x.type = GV_U32; x.u = v; kv_.emplace_back(k, x); }
void GGUFWriter::add_f32(const std::string &k, float v) { GGUFValue x; x.type = GV_F32; x.f = v; kv_.emplace_back(k, x); }
void GGUFWriter::add_str(const std::string &k, const std::string &v) { GGUFValue x; x.type = GV_STR; x.s = v; kv_.emplace_back(k, x); }
void GGUFWriter::add_arr_str(const std::string &k, const std::vector<std::string> &v) {
    GGUFValue x; x.type = GV_ARR; x.arr_type = GV_STR; x.arr_n = v.size(); x.arr_str = v; kv_.emplace_back(k, x);
}
void GGUFWriter::add_arr_f32(const std::string &k, const std::vector<float> &v) {
    GGUFValue x; x.type = GV_ARR; x.arr_type = GV_F32; x.arr_n = v.size();
    x.arr_raw.resize(v.size() * 4); std::memcpy(x.arr_raw.data(), v.data(), v.size() * 4); kv_.emplace_back(k, x);
}
void GGUFWriter::add_arr_i32(const std::string &k, const std::vector<int32_t> &v) {
    GGUFValue x; x.type = GV_ARR; x.arr_type = GV_I32; x.arr_n = v.size();
    x.arr_raw.resize(v.size() * 4); std::memcpy(x.arr_raw.data(), v.data(), v.size() * 4); kv_.emplace_back(k, x);
}
void GGUFWriter::add_value(const std::string &k, const GGUFValue &v) {
    for (auto &p : kv_)
        if (p.first == k) { p.second = v; return; }
    kv_.emplace_back(k, v);
}
void GGUFWriter::add_tensor(const std::string &name, const std::vector<int64_t> &ne, uint32_t type,
                            std::vector<uint8_t> &&bytes) {
    t_.push_back(T{name, ne, type, std::move(bytes)});
}

bool GGUFWriter::write(const std::string &path, std::string &err) const {
    std::vector<uint8_t> h;
    put<uint32_t>(h, 0x46554747u);
    put<uint32_t>(h, 3);
    put<uint64_t>(h, t_.size());
    put<uint64_t>(h, kv_.size());
    for (auto &p : kv_) {
        put_str(h, p.first);
        put<uint32_t>(h, p.second.type);
        write_value(h, p.second);
    }
    uint64_t off = 0;
    for (auto &t : t_) {
        put_str(h, t.name);
        put<uint32_t>(h, (uint32_t)t.ne.size());
        for (int64_t d : t.ne) put<uint64_t>(h, (uint64_t)d);
        put<uint32_t>(h, t.type);
        put<uint64_t>(h, off);
        off += (t.bytes.size() + alignment - 1) / alignment * alignment;
    }
    while (h.size() % alignment) h.push_back(0);
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) { err = "cannot open " + path + " for writing"; return false; }
    bool ok = std::fwrite(h.data(), 1, h.size(), f) == h.size();
    static const uint8_t zeros[64] = {0};
    for (auto &t : t_) {
        ok = ok && std::fwrite(t.bytes.data(), 1, t.bytes.size(), f) == t.bytes.size();
        size_t pad = (alignment - t.bytes.size() % alignment) % alignment;
        while (ok && pad) {
            size_t n = pad < sizeof(zeros) ? pad : sizeof(zeros);
            ok = std::fwrite(zeros, 1, n, f) == n;
            pad -= n;
        }
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) err = "write error on " + path;
    return ok;
}

}  // namespace bertamd
