/*
 * ggml/ggml.h — the same timing / init shim as include/ggml.h, at the path the
 * reference's models/quantize.cpp includes it from (reference
 * models/quantize.cpp:1: #include "ggml/ggml.h"), so that program compiles
 * unchanged against include/ and links build/libbert.so (its only call into
 * the library is bert_model_quantize, models/quantize.cpp:47).
 */
#include "../ggml.h"
