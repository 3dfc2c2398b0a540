/*
 * bert.h — drop-in C ABI for the MI355X-native BERT embedding path.
 *
 * Every declaration below is the one the reference exports from its own
 * bert.h (rinor/embedding.cpp, /root/reference/bert.h:14-96), so that the
 * reference's consumers (examples/server.cpp, examples/main.cpp,
 * examples/sample_dylib.py, benchmarks/run_mteb.py) link / dlopen this
 * library (build/libbert.so) unchanged.  The implementation behind it is a
 * fixed HIP kernel pipeline for gfx950 instead of the reference's ggml CPU
 * graph.
 *
 * Behavioural differences, all deliberate and documented in DESIGN.md:
 *   - errors never throw across the ABI: bert_load_from_file returns NULL,
 *     eval/encode log to stderr and leave the output untouched;
 *   - bert_eval_batch writes the L2-normalised mean-pooled vector
 *     (ggml graph node n-1), not the reference's over-read of node n-2
 *     (reference bert.cpp:1085,1098);
 *   - n_threads is accepted and ignored on the GPU path (host threads are
 *     one per visible GPU).
 * Extensions that the reference does not have live in bert_amd.h.
 */
#ifndef BERT_H
#define BERT_H

#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

#if defined(_WIN32)
#define BERT_API __declspec(dllexport)
#else
#define BERT_API __attribute__((visibility("default")))
#endif

#ifdef __cplusplus
extern "C"
{
#endif

    /* reference bert.h:19-24 (declared, unused by the reference itself) */
    enum llama_log_level
    {
        LLAMA_LOG_LEVEL_ERROR = 2,
        LLAMA_LOG_LEVEL_WARN = 3,
        LLAMA_LOG_LEVEL_INFO = 4
    };

    /* reference bert.h:26-33: CLI parameters (C++ default member initialisers,
       exactly as the reference declares them; consumers are C++). */
    struct bert_params
    {
        int32_t n_threads = 6;
        int32_t port = 8080; /* server mode port to bind */

        const char *model = "models/all-MiniLM-L6-v2/ggml-model-q4_0.bin"; /* model path */
        const char *prompt = "test prompt";
    };

    /* reference bert.h:35 / bert.cpp:697-733: -t -p --port -m -h */
    BERT_API bool bert_params_parse(int argc, char **argv, bert_params &params);

    struct bert_ctx;

    typedef int32_t bert_vocab_id;

    /* reference bert.h:41 / bert.cpp:783-819. Returns NULL on any error. */
    BERT_API struct bert_ctx *bert_load_from_file(const char *fname);
    /* reference bert.h:42 / bert.cpp:1014-1018 */
    BERT_API void bert_free(bert_ctx *ctx);

    /* Main api, does both tokenizing and evaluation.
       reference bert.h:46-50 / bert.cpp:1110-1117 */
    BERT_API void bert_encode(
        struct bert_ctx *ctx,
        int32_t n_threads,
        const char *texts,
        float *embeddings);

    /* n_batch_size - how many to process at a time
       n_inputs     - total size of texts and embeddings arrays
       reference bert.h:54-60 / bert.cpp:1119-1198 */
    BERT_API void bert_encode_batch(
        struct bert_ctx *ctx,
        int32_t n_threads,
        int32_t n_batch_size,
        int32_t n_inputs,
        const char **texts,
        float **embeddings);

    /* Api for separate tokenization & eval.
       reference bert.h:64-69 / bert.cpp:738-781 */
    BERT_API void bert_tokenize(
        struct bert_ctx *ctx,
        const char *text,
        bert_vocab_id *tokens,
        int32_t *n_tokens,
        int32_t n_max_tokens);

    /* reference bert.h:71-76 / bert.cpp:1020-1028 */
    BERT_API void bert_eval(
        struct bert_ctx *ctx,
        int32_t n_threads,
        bert_vocab_id *tokens,
        int32_t n_tokens,
        float *embeddings);

    /* reference bert.h:78-85 / bert.cpp:1030-1108.  (The reference's note
       "the longest input must be first" is vestigial: any order works.) */
    BERT_API void bert_eval_batch(
        struct bert_ctx *ctx,
        int32_t n_threads,
        int32_t n_batch_size,
        bert_vocab_id **batch_tokens,
        int32_t *n_tokens,
        float **batch_embeddings);

    /* reference bert.h:87-90 / bert.cpp:661-675 */
    BERT_API int32_t bert_n_embd(bert_ctx *ctx);
    BERT_API int32_t bert_n_max_tokens(bert_ctx *ctx);

    BERT_API const char *bert_vocab_id_to_token(bert_ctx *ctx, bert_vocab_id id);

    /* reference bert.h:92 / bert.cpp:1313-1599: ftype 2 = Q4_0, 3 = Q4_1 */
    BERT_API bool bert_model_quantize(const char *fname_inp, const char *fname_out, int ftype);

#ifdef __cplusplus
}
#endif

/* model quantization parameters (reference bert.h:98-106) */
typedef struct llama_model_quantize_params
{
    int nthread;                 /* number of threads to use for quantizing, <=0: hardware_concurrency */
    bool allow_requantize;       /* allow quantizing non-f32/f16 tensors */
    bool quantize_output_tensor; /* quantize output.weight */
    bool only_copy;              /* only copy tensors */
} llama_model_quantize_params;

#endif /* BERT_H */
