/*
 * ggml.h — minimal shim so the reference's consumers compile unchanged against
 * this library.  examples/main.cpp uses ggml_time_init / ggml_time_us
 * (reference examples/main.cpp:9-10,24-75); models/quantize.cpp calls
 * ggml_init / ggml_free only to initialise ggml's fp16 tables.  No tensor API
 * is provided: the embedding path does not go through ggml.
 */
#ifndef BERT_AMD_GGML_SHIM_H
#define BERT_AMD_GGML_SHIM_H

#include <stddef.h>
#include <stdint.h>
#include <time.h>

#ifdef __cplusplus
extern "C" {
#endif

static inline void ggml_time_init(void) {}

static inline int64_t ggml_time_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (int64_t)ts.tv_sec * 1000000 + (int64_t)ts.tv_nsec / 1000;
}

static inline int64_t ggml_time_ms(void) { return ggml_time_us() / 1000; }

struct ggml_init_params {
    size_t mem_size;
    void *mem_buffer;
    bool no_alloc;
};
struct ggml_context;
static inline struct ggml_context *ggml_init(struct ggml_init_params p) {
    (void)p;
    return (struct ggml_context *)0;
}
static inline void ggml_free(struct ggml_context *c) { (void)c; }

#ifdef __cplusplus
}
#endif

#endif
