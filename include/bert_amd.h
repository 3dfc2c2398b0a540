/*
 * bert_amd.h — additive extensions of the drop-in library (not in the
 * reference ABI; the reference consumers never need them).
 *
 * They exist for three callers:
 *   - bench.py / tests: device-resident batch evaluation on a caller-chosen
 *     HIP stream (inputs already in HBM, nothing copied, no sync);
 *   - multi-GPU: choose the devices a context is replicated on (the
 *     reference ABI has no device argument; SURVEY.md §8(b) "No device
 *     argument");
 *   - tooling: the deterministic synthetic GGUF generator and per-kernel
 *     timing.
 * All functions are C-ABI, take plain pointers and sizes, never throw, and
 * return 0 on success / negative on error (message via bert_amd_last_error).
 */
#ifndef BERT_AMD_H
#define BERT_AMD_H

#include <stdint.h>

#include "bert.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Load a GGUF and replicate its weights on the given HIP devices (ordinals as
   seen by this process).  n_devices <= 0: all visible devices, or the list in
   env BERT_AMD_DEVICES="0,1,...".  Returns NULL on error. */
BERT_API struct bert_ctx *bert_amd_load(const char *fname, const int32_t *devices, int32_t n_devices);

/* bert_amd_load with options: "key=value" items separated by ';' (NULL or ""
   = none).  Every key's default may come from the environment
   (BERT_AMD_<KEY> in upper case), which is read once, inside this call; the
   string overrides it.  Load-time keys (they shape the device weights):
     "i8"       Q4 projections on the int8-MFMA GEMMs: "0" none, "all", or a
                list of up, o, down joined by '+' (default: up+o+down for Q4_0
                at n_embd 384, up+down for Q4_1 there, up otherwise)
     "qkva_ntw" the fused QKV + attention kernel: 0 producer / consumer
                waves on an int8 QKV copy (Q4_0, head dim 32, n_embd 384;
                elsewhere 1), 1 | 2 head-pair units per main loop of the
                head-pair kernel, -1 (default) 0 where it exists, else 2
     "q41bf"    Q4_1 on the int8 GEMMs: the per-block scale products d_w d_a
                and m_w s_a as exact bf16 partial products on the bf16 MFMA
                (kernels.h W_Q4_1B) instead of the f32 MFMA: 1 every int8
                projection, 0 none, -1 (default) all but the 384-wide FFN-down
                + LayerNorm kernel (where they cost more than they save)
     "emb_raw"  1 (default): the word-embedding table stays in its GGUF row
                format on the device (dequantised in the embedding kernel as
                ggml's get_rows does); 0: an f32 copy.  Same results
   and every bert_amd_set_option key below.  Returns NULL on error (an unknown
   key or a bad value included). */
BERT_API struct bert_ctx *bert_amd_load_opts(const char *fname, const int32_t *devices, int32_t n_devices,
                                             const char *options);

BERT_API int32_t bert_amd_n_devices(struct bert_ctx *ctx);

/* hparams: [n_vocab, n_max_tokens, n_embd, n_intermediate, n_head, n_layer, weight ggml type] */
BERT_API int32_t bert_amd_hparams(struct bert_ctx *ctx, int32_t *out7);

/* Device-resident evaluation on replica `slot` (index into the context's
   device list), enqueued on `hip_stream` (a hipStream_t; NULL = HIP's null
   stream, i.e. torch's default stream).  Asynchronous: returns after
   enqueueing; every kernel and workspace fill runs on `hip_stream`.  Takes
   the context's lock (one eval at a time per context, like bert_eval_batch).
     d_tokens   : int32, packed token ids of all sentences (device memory)
     d_offsets  : int32[n_seqs+1], prefix offsets into d_tokens (device memory)
     h_offsets  : the same offsets in host memory (used for grid sizing)
     d_out      : float[n_seqs * n_embd] (device memory), L2-normalised
   Workspace is grown on demand (allocation happens outside any capture when
   the caller warms up with the largest batch first). */
BERT_API int32_t bert_amd_eval_device(struct bert_ctx *ctx, int32_t slot, const int32_t *d_tokens,
                                      const int32_t *d_offsets, const int32_t *h_offsets, int32_t n_seqs,
                                      float *d_out, void *hip_stream);

/* Per-kernel-class timing with HIP events on the launch stream.
   enable != 0 turns it on for subsequent evals (adds event records between
   launches; never used inside bench.py's timed region). */
BERT_API int32_t bert_amd_profile_enable(struct bert_ctx *ctx, int32_t enable);
/* Copies up to max_entries: names (NUL-separated into names_buf), total ms
   and launch counts since enable.  Returns the number of entries. */
BERT_API int32_t bert_amd_profile_read(struct bert_ctx *ctx, char *names_buf, int32_t names_len, float *total_ms,
                                       int32_t *counts, int32_t max_entries);

/* Deterministic synthetic BERT GGUF (see csrc/synth.cpp).
   ftype: 0 = f32, 1 = f16, 2 = Q4_0, 3 = Q4_1 (2-D *.weight tensors). */
BERT_API int bert_amd_synth_model(const char *path, int32_t n_vocab, int32_t n_max_tokens, int32_t n_embd,
                                  int32_t n_intermediate, int32_t n_head, int32_t n_layer, int32_t ftype,
                                  uint64_t seed, float w_std);

/* Tokenizer without a model/GPU (tests, tooling): runs the native WordPiece
   tokenizer configured by an HF tokenizer.json string.  frame == 0: the content
   ids of Encode(text) (at most n_max_tokens); frame != 0: bert_tokenize's
   [CLS] ... [SEP] framing with the given special ids.  Returns the count. */
BERT_API int32_t bert_amd_tokenize_json(const char *tokenizer_json, const char *text, int32_t *tokens,
                                        int32_t n_max_tokens, int32_t frame, int32_t cls_id, int32_t sep_id,
                                        int32_t pad_id);

/* Test hook: the embeddings + LayerNorm stage alone (reference
   bert.cpp:865-898) on a host batch (packed ids + offsets[n_seqs+1]), on
   replica 0.  Copies back X (f32 [M][n_embd], the LayerNorm output) and the
   first GEMM's activation format of it: q [M][n_embd] (int8 for Q4 models,
   fp16 / f32 for F16 / F32) and d [M][n_embd/32] (fp16 for Q4_0, f32 for
   Q4_1; may be NULL).  Lets tests pin the integer stage bit-exactly against
   the oracle's quantiser. */
BERT_API int32_t bert_amd_debug_embed(struct bert_ctx *ctx, const int32_t *tokens, const int32_t *offsets,
                                      int32_t n_seqs, float *X_out, void *q_out, void *d_out);

/* Test hook: the whole pipeline on a host batch (replica 0, one row group,
   the kernels bert_eval_batch would pick for it under the context's options),
   copying back the residual stream after every stage: X_out f32
   [n_layer + 1][M][n_embd] (stage 0 = embeddings + LayerNorm, reference
   bert.cpp:865-898; stage l + 1 = the output of encoder layer l,
   bert.cpp:900-993) and its activation form as bert_amd_debug_embed's q / d,
   per stage.  Lets tests pin parity layer by layer against the oracle. */
BERT_API int32_t bert_amd_debug_layers(struct bert_ctx *ctx, const int32_t *tokens, const int32_t *offsets,
                                       int32_t n_seqs, float *X_out, void *q_out, void *d_out);

/* Rows (tokens, padded to the 128-row tile) the device workspace of replica
   `slot` currently holds; -1 on a bad argument.  Lets callers and tests see
   that bert_encode_batch's n_batch_size bounds the working set. */
BERT_API int64_t bert_amd_workspace_rows(struct bert_ctx *ctx, int32_t slot);

/* Per-context pipeline options (defaults, then bert_amd_load_opts /
   BERT_AMD_<KEY> at load; this call changes them afterwards):
     "split" 0 | 1     run large fused batches as two row groups on two streams
     "pack"  -1 | 0 | 1 pack short sentences into shared fused-kernel tiles
                        when it pays (-1, default) / never / always
     "fuse_min" n >= 0 batches of fewer than n sentences (default 48) run the
                        unfused QKV GEMM + attention pair instead of the fused
                        kernel (lower latency for small batches)
     "unfused" 0 | 1    1: every batch on the QKV GEMM + attention pair (A/B
                        checks; default 0)
     "small_rows" n >= 0 batches of at most n padded rows (default 2048; one
                        sentence is 128) run the int8 GEMMs in 32-row tiles
                        (Q4_0, K <= 3072, <= 512 rows: the K loop split
                        over 12-16 waves; latency of small batches; 0 = never)
     "small_qkva" 0 | 1  1 (default): small batches (<= small_rows, <= 2048 rows) whose
                        sentences all have <= 64 tokens (Q4_0, n_embd 384, head
                        dim 32) run each head's int8 QKV and its attention in one
                        kernel (same results; one launch less per layer)
     "nt_x" 0 | 1        1 (default): the 384-wide projection + LayerNorm kernel
                        stores X with the nontemporal cache policy (all but the
                        last layer's X, which the pooling reads next), so the
                        weights its tiles re-read stay in L2; 0 plain stores
     "graph_seqs" n >= 0 host batches of at most n sentences (and fewer than
                        fuse_min) replay a captured HIP graph of their launches
                        (default 0: measured no faster)
     "encode_lanes" n >= 1 bert_encode_batch: lanes per device, each a host
                        thread with its own workspace and streams (default 2;
                        BERT_AMD_ENCODE_LANES)
     "encode_merge" n >= 1 bert_encode_batch: consecutive n_batch_size slices a
                        lane evaluates as one ragged batch (default 16;
                        BERT_AMD_ENCODE_MERGE; 1 = one slice per GPU batch),
                        merged only up to "encode_merge_rows" sentences
                        (default 256; BERT_AMD_ENCODE_MERGE_ROWS).  At most
                        lanes x max(n_batch_size, min(merge x n_batch_size,
                        merge_rows)) sentences are in flight per device
   Results are identical under every setting. */
BERT_API int32_t bert_amd_set_option(struct bert_ctx *ctx, const char *key, int32_t value);

/* Reads an option back into *value: every bert_amd_set_option key, plus the
   load-time choices as resolved for this model — "qkva_ntw" (0, 1 or 2),
   "i8_qkv", "i8_up", "i8_o", "i8_down" (1 when that Q4 projection runs on
   the int8-MFMA GEMMs: for QKV, the producer / consumer kernel's int8 copy
   and its unfused int8 twin), "q41bf" (the load option: -1 auto, 0, 1) and
   "q41bf_qkv", "q41bf_o", "q41bf_up", "q41bf_down" (1 when that Q4_1
   projection's int8 GEMM takes its scale products on the bf16 MFMA,
   W_Q4_1B).  Lets bench.py price each kernel on the
   arithmetic it runs.  Returns 0, or -2 on an unknown key. */
BERT_API int32_t bert_amd_get_option(struct bert_ctx *ctx, const char *key, int32_t *value);

/* How bert_eval_batch splits a batch over n_replicas devices: contiguous
   sentence slices balanced by token count, slice r = [cut[r], cut[r+1]),
   cut[0] = 0, cut[n_replicas] = n_seqs (cut has n_replicas + 1 entries).
   Pure host function (no device needed); lets tests check balance and
   coverage.  Returns 0, or -1 on invalid arguments. */
BERT_API int32_t bert_amd_shard_cuts(int32_t n_seqs, const int32_t *n_tokens, int32_t n_replicas, int32_t *cut);

BERT_API const char *bert_amd_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* BERT_AMD_H */
