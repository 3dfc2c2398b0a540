// gguf_io.h — native GGUF v2/v3 reader and writer (host).
//
// Replaces the reference's use of ggml's gguf_* API (reference gguf.h:50-141,
// bert.cpp:173-204, 398-473) and the writer used by the quantiser
// (bert.cpp:1372-1573).  Container layout: SURVEY.md Appendix B.
// The reader mmaps the file; tensor data pointers stay valid while the
// GGUFFile lives.  Errors are reported by returning false + a message, never
// by throwing across the C ABI.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace bertamd {

enum gguf_vtype : uint32_t {
    GV_U8 = 0, GV_I8 = 1, GV_U16 = 2, GV_I16 = 3, GV_U32 = 4, GV_I32 = 5,
    GV_F32 = 6, GV_BOOL = 7, GV_STR = 8, GV_ARR = 9, GV_U64 = 10, GV_I64 = 11, GV_F64 = 12,
};

struct GGUFValue {
    uint32_t type = GV_U32;
    uint32_t arr_type = 0;            // element type when type == GV_ARR
    uint64_t u = 0;                   // integer / bool scalars (bit pattern)
    double f = 0;                     // float scalars
    std::string s;                    // string scalar
    std::vector<std::string> arr_str; // string arrays
    std::vector<uint8_t> arr_raw;     // numeric arrays, raw little-endian bytes
    uint64_t arr_n = 0;
};

struct GGUFTensor {
    std::string name;
    std::vector<int64_t> ne;  // ggml order: ne[0] is the contiguous dimension
    uint32_t type = 0;
    uint64_t offset = 0;      // relative to the data section
    const uint8_t *data = nullptr;
    size_t nbytes = 0;
    int64_t nrows() const { int64_t r = 1; for (size_t i = 1; i < ne.size(); i++) r *= ne[i]; return r; }
};

class GGUFFile {
public:
    ~GGUFFile();
    bool open(const std::string &path, std::string &err);
    uint32_t version = 0;
    size_t alignment = 32;
    std::vector<std::pair<std::string, GGUFValue>> kv;  // file order
    std::vector<GGUFTensor> tensors;                     // file order
    const GGUFValue *find(const std::string &key) const;
    const GGUFTensor *tensor(const std::string &name) const;

private:
    void *map_ = nullptr;
    size_t map_size_ = 0;
    int fd_ = -1;
};

// Writer: collects KVs and tensors, then writes header + aligned data.
class GGUFWriter {
public:
    void add_u32(const std::string &k, uint32_t v);
    void add_f32(const std::string &k, float v);
    void add_str(const std::string &k, const std::string &v);
    void add_arr_str(const std::string &k, const std::vector<std::string> &v);
    void add_arr_f32(const std::string &k, const std::vector<float> &v);
    void add_arr_i32(const std::string &k, const std::vector<int32_t> &v);
    void add_value(const std::string &k, const GGUFValue &v);  // copy from a reader
    void add_tensor(const std::string &name, const std::vector<int64_t> &ne, uint32_t type,
                    std::vector<uint8_t> &&bytes);
    bool write(const std::string &path, std::string &err) const;
    size_t alignment = 32;

private:
    std::vector<std::pair<std::string, GGUFValue>> kv_;
    struct T { std::string name; std::vector<int64_t> ne; uint32_t type; std::vector<uint8_t> bytes; };
    std::vector<T> t_;
};

}  // namespace bertamd
