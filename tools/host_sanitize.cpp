// Host-code sanitizer driver (test infrastructure): the GGUF reader/writer,
// the WordPiece tokenizer and the Q4 quantiser of libbert.so, built as a CPU
// executable with -fsanitize=address,undefined (Makefile target
// build/host_sanitize, run by tests/test_sanitizers.py).  No GPU code.
//   host_sanitize synth <out.gguf>                   tiny synthetic model
//   host_sanitize parse <file.gguf>                  read + dequantise every tensor
//   host_sanitize tok <file.gguf> <text>...          tokenizer from the model's blob
//   host_sanitize quant <in.gguf> <out.gguf> <2|3>   bert_model_quantize
//   host_sanitize fuzz <file.gguf> <seed> <n>        n truncated / corrupted copies, parsed
//   host_sanitize tokfuzz <file.gguf> <seed> <n>     n random byte strings through the tokenizer
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "bert.h"
#include "bert_amd.h"
#include "ggml_formats.h"
#include "gguf_io.h"
#include "tokenizer.h"

using namespace bertamd;


static int parse(const char *path, bool quiet) {
    GGUFFile f;
    std::string err;
    if (!f.open(path, err)) {
        if (!quiet) std::printf("rejected: %s\n", err.c_str());
        return 1;
    }
    double sum = 0;
    for (const auto &t : f.tensors) {
        if (t.ne.empty() || t.ne[0] <= 0 || t.ne[0] > (1 << 20)) continue;
        const size_t rb = ggml_row_bytes(t.type, t.ne[0]);
        if (rb == 0 || rb * (size_t)t.nrows() > t.nbytes) continue;
        std::vector<float> row((size_t)t.ne[0]);
        for (int64_t r = 0; r < t.nrows(); r++) {
            const uint8_t *p = t.data + (size_t)r * rb;
            if (t.type == GT_F32) std::memcpy(row.data(), p, rb);
            else if (t.type == GT_F16) for (int64_t i = 0; i < t.ne[0]; i++) row[(size_t)i] = f16_to_f32(((const uint16_t *)p)[i]);
            else if (t.type == GT_Q4_0 || t.type == GT_Q4_1) dequantize_row(t.type, p, row.data(), t.ne[0]);
            else break;
            sum += row[0];
        }
    }
    for (const auto &kv : f.kv) sum += (double)kv.second.arr_str.size() + (double)kv.second.s.size();
    if (!quiet) std::printf("parsed: %zu kv, %zu tensors (checksum %g)\n", f.kv.size(), f.tensors.size(), sum);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const std::string cmd = argv[1];
    if (cmd == "synth")
        return bert_amd_synth_model(argv[2], 2000, 64, 64, 128, 2, 1, 1, 7, 0.05f) == 0 ? 0 : 1;
    if (cmd == "parse") return parse(argv[2], false) == 0 ? 0 : 3;
    if (cmd == "tok") {
        GGUFFile f;
        std::string err;
        if (!f.open(argv[2], err)) return 1;
        const GGUFValue *blob = f.find("blob.tokenizer.json");
        WordPieceTokenizer tk;
        if (!blob || !tk.load(blob->s, err)) return 1;
        for (int i = 3; i < argc; i++) {
            const std::vector<int32_t> ids = tk.encode(argv[i]);
            std::printf("%zu:", ids.size());
            for (int32_t id : ids) std::printf(" %d", id);
            std::printf("\n");
        }
        return 0;
    }
    if (cmd == "tokfuzz" && argc >= 5) {  // random byte strings (invalid UTF-8, controls, long words)
        GGUFFile f;
        std::string err;
        if (!f.open(argv[2], err)) return 1;
        const GGUFValue *blob = f.find("blob.tokenizer.json");
        WordPieceTokenizer tk;
        if (!blob || !tk.load(blob->s, err)) return 1;
        std::mt19937_64 rng((uint64_t)std::atoll(argv[3]));
        size_t total = 0;
        for (int i = 0, n = std::atoi(argv[4]); i < n; i++) {
            std::string s(rng() % 300, ' ');
            for (char &c : s) c = (char)((rng() & 1) ? rng() : "ab Q\xc3\xa9,.!\t\n"[rng() % 12]);
            total += tk.encode(s).size();
        }
        std::printf("tokfuzz: %zu ids\n", total);
        return 0;
    }
    if (cmd == "quant" && argc >= 5) return bert_model_quantize(argv[2], argv[3], std::atoi(argv[4])) ? 0 : 1;
    if (cmd == "fuzz" && argc >= 5) {
        std::ifstream in(argv[2], std::ios::binary);
        const std::vector<char> src((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
        std::mt19937_64 rng((uint64_t)std::atoll(argv[3]));
        const int n = std::atoi(argv[4]);
        const std::string tmp = std::string(argv[2]) + ".fuzz";
        int accepted = 0;
        for (int i = 0; i < n; i++) {
            std::vector<char> b = src;
            const int kind = i % 4;
            if (kind == 0) {
                b.resize(rng() % (b.size() + 1));  // truncation anywhere
            } else if (kind == 1) {                // random bytes in the header / KV / tensor-info region
                const size_t lim = std::min<size_t>(b.size(), 1 << 16);
                for (int j = 0; j < 8; j++) b[rng() % lim] = (char)rng();
            } else if (kind == 2) {                // 64-bit counts / sizes / offsets blown up
                const size_t lim = std::min<size_t>(b.size(), 1 << 16);
                const size_t at = 8 + (rng() % (lim > 16 ? lim - 16 : 1));
                const uint64_t v = (rng() & 1) ? ~0ull - (rng() & 0xffff) : (1ull << (rng() % 64));
                std::memcpy(&b[at], &v, 8);
            } else {                               // random 32-bit fields (types, dims, lengths)
                const size_t lim = std::min<size_t>(b.size(), 1 << 16);
                for (int j = 0; j < 4; j++) {
                    const size_t at = rng() % (lim > 4 ? lim - 4 : 1);
                    const uint32_t v = (uint32_t)rng();
                    std::memcpy(&b[at], &v, 4);
                }
            }
            std::ofstream(tmp, std::ios::binary).write(b.data(), (std::streamsize)b.size());
            accepted += parse(tmp.c_str(), true) == 0;
        }
        std::remove(tmp.c_str());
        std::printf("fuzz: %d variants, %d still parse\n", n, accepted);
        return 0;
    }
    return 2;
}
