// tok_bench.cpp — host-only timing of the WordPiece tokenizer as
// bert_encode_batch drives it (development; no GPU): the GGUF's tokenizer
// JSON, 4096 synthetic texts of vocabulary words (8..128 tokens framed, like
// bench.py's consumer line), encoded on 1, 2, 4, 8, 16 threads.
//   build/tok_bench <model.gguf> [n_texts]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "gguf_io.h"
#include "tokenizer.h"

using namespace bertamd;

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s model.gguf [n_texts]\n", argv[0]);
        return 2;
    }
    const int n = argc > 2 ? std::atoi(argv[2]) : 4096;
    GGUFFile f;
    std::string err;
    if (!f.open(argv[1], err)) {
        std::fprintf(stderr, "%s\n", err.c_str());
        return 1;
    }
    const GGUFValue *js = f.find("blob.tokenizer.json");
    const GGUFValue *toks = f.find("tokenizer.ggml.tokens");
    WordPieceTokenizer tk;
    if (!js || !toks || !tk.load(js->s, err)) {
        std::fprintf(stderr, "tokenizer: %s\n", err.c_str());
        return 1;
    }
    std::vector<std::string> words;
    for (size_t i = 1000; i < toks->arr_str.size(); i++) {
        const std::string &w = toks->arr_str[i];
        if (!w.empty() && std::all_of(w.begin(), w.end(), [](char c) { return c >= 'a' && c <= 'z'; })) words.push_back(w);
    }
    std::mt19937_64 rng(7);
    std::vector<std::string> texts(n);
    for (auto &t : texts) {
        const int k = 6 + (int)(rng() % 121);
        for (int j = 0; j < k; j++) {
            if (j) t += ' ';
            t += words[rng() % words.size()];
        }
    }
    for (int nt : {1, 2, 4, 8, 16}) {
        double best = 1e30;
        size_t total = 0;
        for (int rep = 0; rep < 5; rep++) {
            const auto t0 = std::chrono::steady_clock::now();
            std::vector<size_t> cnt(nt, 0);
            std::vector<std::thread> th;
            for (int t = 0; t < nt; t++)
                th.emplace_back([&, t] {
                    for (int i = (int)((int64_t)n * t / nt); i < (int)((int64_t)n * (t + 1) / nt); i++)
                        cnt[t] += tk.encode(texts[i]).size();
                });
            for (auto &x : th) x.join();
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            best = std::min(best, s);
            total = 0;
            for (size_t c : cnt) total += c;
        }
        std::printf("{\"threads\": %d, \"texts\": %d, \"tokens\": %zu, \"ms\": %.3f, \"us_per_text_thread\": %.2f}\n", nt, n,
                    total, best * 1e3, best * 1e6 * nt / n);
    }
    return 0;
}
