// quantize_model.cpp — bert_model_quantize (reference bert.h:92,
// bert.cpp:1313-1599; models/quantize.cpp).
//
// Same contract as the reference: ftype 2 -> Q4_0, 3 -> Q4_1; every 2-D tensor
// whose name ends in "weight" (embedding tables included, bert.cpp:1431-1436)
// is quantised from F32/F16 with the ggml reference quantisers; everything else
// is copied; KV pairs are copied and general.quantization_version /
// general.file_type are set; tensor data is aligned to 32 bytes.
// Differences: errors return false instead of throwing across the ABI;
// quantisation is split over hardware threads by rows (bit-identical to a
// single-threaded run, as ggml's chunking is).
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "bert.h"
#include "ggml_formats.h"
#include "gguf_io.h"

using namespace bertamd;

bool bert_model_quantize(const char *fname_inp, const char *fname_out, int ftype) {
    uint32_t qtype;
    switch (ftype) {
        case 2: qtype = GT_Q4_0; break;
        case 3: qtype = GT_Q4_1; break;
        default: std::fprintf(stderr, "%s: invalid quantization type %d\n", __func__, ftype); return false;
    }
    if (!fname_inp || !fname_out) return false;
    GGUFFile in;
    std::string err;
    if (!in.open(fname_inp, err)) {
        std::fprintf(stderr, "%s: %s\n", __func__, err.c_str());
        return false;
    }
    GGUFWriter w;
    for (auto &kv : in.kv) w.add_value(kv.first, kv.second);
    w.add_u32("general.quantization_version", 2);
    w.add_u32("general.file_type", (uint32_t)ftype);
    unsigned nth = std::thread::hardware_concurrency();
    if (nth == 0) nth = 1;
    for (const GGUFTensor &t : in.tensors) {
        const bool is_weight = t.name.size() >= 6 && t.name.compare(t.name.size() - 6, 6, "weight") == 0;
        const bool quant = is_weight && t.ne.size() == 2 && t.type != qtype;
        if (!quant) {
            w.add_tensor(t.name, t.ne, t.type, std::vector<uint8_t>(t.data, t.data + t.nbytes));
            continue;
        }
        if (t.type != GT_F32 && t.type != GT_F16) {
            std::fprintf(stderr, "%s: requantizing from type %s is disabled\n", __func__, ggml_type_str(t.type));
            return false;
        }
        const int64_t ne0 = t.ne[0], nrows = t.ne[1];
        if (ne0 % QK) {
            std::fprintf(stderr, "%s: row size of %s is not a multiple of 32\n", __func__, t.name.c_str());
            return false;
        }
        const size_t orb = ggml_row_bytes(qtype, ne0), irb = ggml_row_bytes(t.type, ne0);
        std::vector<uint8_t> out((size_t)nrows * orb);
        auto work = [&](int64_t r0, int64_t r1) {
            std::vector<float> row((size_t)ne0);
            for (int64_t r = r0; r < r1; r++) {
                dequantize_row(t.type, t.data + (size_t)r * irb, row.data(), ne0);
                if (qtype == GT_Q4_0)
                    quantize_row_q4_0(row.data(), (block_q4_0 *)(out.data() + (size_t)r * orb), ne0);
                else
                    quantize_row_q4_1(row.data(), (block_q4_1 *)(out.data() + (size_t)r * orb), ne0);
            }
        };
        std::vector<std::thread> th;
        const int64_t per = (nrows + nth - 1) / nth;
        for (unsigned i = 0; i < nth; i++) {
            const int64_t r0 = i * per, r1 = std::min<int64_t>(nrows, r0 + per);
            if (r0 < r1) th.emplace_back(work, r0, r1);
        }
        for (auto &x : th) x.join();
        std::printf("%s: %36s %s -> %s\n", __func__, t.name.c_str(), ggml_type_str(t.type), ggml_type_str(qtype));
        w.add_tensor(t.name, t.ne, qtype, std::move(out));
    }
    if (!w.write(fname_out, err)) {
        std::fprintf(stderr, "%s: %s\n", __func__, err.c_str());
        return false;
    }
    return true;
}
