// quantize.cpp — ggml-exact reference quantisers and row dequantisers (host).
//
// Used by bert_model_quantize (reference bert.cpp:1313-1599, which calls
// ggml_quantize_chunk -> quantize_row_q4_{0,1}_reference of ggml@8ca2c19) and by
// the synthetic-model generator.  Restated from SURVEY.md Appendix A.
#include "ggml_formats.h"

#include <cfloat>
#include <cmath>

namespace bertamd {

// Q4_0: d = (signed value of largest magnitude) / -8, q = min(15, (int8)(x/d + 8.5))
void quantize_row_q4_0(const float *x, block_q4_0 *y, int64_t k) {
    const int64_t nb = k / QK;
    for (int64_t i = 0; i < nb; i++) {
        float amax = 0.0f, max = 0.0f;
        for (int j = 0; j < QK; j++) {
            const float v = x[i * QK + j];
            if (amax < std::fabs(v)) { amax = std::fabs(v); max = v; }
        }
        const float d = max / -8;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        y[i].d = f32_to_f16(d);
        for (int j = 0; j < QK / 2; ++j) {
            const float x0 = x[i * QK + j] * id;
            const float x1 = x[i * QK + QK / 2 + j] * id;
            int8_t t0 = (int8_t)(x0 + 8.5f), t1 = (int8_t)(x1 + 8.5f);
            const uint8_t xi0 = (uint8_t)(t0 < 15 ? t0 : 15);
            const uint8_t xi1 = (uint8_t)(t1 < 15 ? t1 : 15);
            y[i].qs[j] = (uint8_t)(xi0 | (xi1 << 4));
        }
    }
}

// Q4_1: d = (max-min)/15, m = min, q = min(15, (int8)((x-min)/d + 0.5))
void quantize_row_q4_1(const float *x, block_q4_1 *y, int64_t k) {
    const int64_t nb = k / QK;
    for (int64_t i = 0; i < nb; i++) {
        float min = FLT_MAX, max = -FLT_MAX;
        for (int j = 0; j < QK; j++) {
            const float v = x[i * QK + j];
            if (v < min) min = v;
            if (v > max) max = v;
        }
        const float d = (max - min) / ((1 << 4) - 1);
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        y[i].d = f32_to_f16(d);
        y[i].m = f32_to_f16(min);
        for (int j = 0; j < QK / 2; ++j) {
            const float x0 = (x[i * QK + j] - min) * id;
            const float x1 = (x[i * QK + QK / 2 + j] - min) * id;
            int8_t t0 = (int8_t)(x0 + 0.5f), t1 = (int8_t)(x1 + 0.5f);
            const uint8_t xi0 = (uint8_t)(t0 < 15 ? t0 : 15);
            const uint8_t xi1 = (uint8_t)(t1 < 15 ? t1 : 15);
            y[i].qs[j] = (uint8_t)(xi0 | (xi1 << 4));
        }
    }
}

void dequantize_row(uint32_t type, const void *src, float *dst, int64_t k) {
    switch (type) {
        case GT_F32: std::memcpy(dst, src, (size_t)k * 4); break;
        case GT_F16: {
            const uint16_t *s = (const uint16_t *)src;
            for (int64_t i = 0; i < k; i++) dst[i] = f16_to_f32(s[i]);
        } break;
        case GT_Q4_0: {
            const block_q4_0 *b = (const block_q4_0 *)src;
            for (int64_t i = 0; i < k / QK; i++) {
                const float d = f16_to_f32(b[i].d);
                for (int j = 0; j < QK / 2; j++) {
                    dst[i * QK + j] = (float)((b[i].qs[j] & 0x0f) - 8) * d;
                    dst[i * QK + j + QK / 2] = (float)((b[i].qs[j] >> 4) - 8) * d;
                }
            }
        } break;
        case GT_Q4_1: {
            const block_q4_1 *b = (const block_q4_1 *)src;
            for (int64_t i = 0; i < k / QK; i++) {
                const float d = f16_to_f32(b[i].d), m = f16_to_f32(b[i].m);
                for (int j = 0; j < QK / 2; j++) {
                    // gcc -O3 -mfma contracts ggml's `x*d + m` into one fma
                    dst[i * QK + j] = std::fma((float)(b[i].qs[j] & 0x0f), d, m);
                    dst[i * QK + j + QK / 2] = std::fma((float)(b[i].qs[j] >> 4), d, m);
                }
            }
        } break;
        default: break;
    }
}

}  // namespace bertamd
