// ggml_formats.h — on-disk tensor formats the drop-in must read, and the
// host-side IEEE binary16 conversion they are built on.
//
// The reference stores weights in ggml@8ca2c19 formats (reference .gitmodules:1-5;
// the submodule is not vendored).  The layouts below are restated from the
// published ggml block definitions of that era:
//   Q4_0 {fp16 d; u8 qs[16]}           value(j)    = (lo(qs[j])  - 8) * d,
//                                      value(j+16) = (hi(qs[j])  - 8) * d
//   Q4_1 {fp16 d; fp16 m; u8 qs[16]}   value       = q * d + m
//   Q8_0 {fp16 d; i8 qs[32]}, Q8_1 {f32 d; f32 s; i8 qs[32]}
// Host code only; device kernels use their own packed layouts.
#pragma once
#include <cstdint>
#include <cstring>

namespace bertamd {

enum ggml_type_id : uint32_t {
    GT_F32 = 0,
    GT_F16 = 1,
    GT_Q4_0 = 2,
    GT_Q4_1 = 3,
    GT_Q8_0 = 8,
    GT_Q8_1 = 9,
};

constexpr int QK = 32;  // elements per quant block (QK4_0 = QK4_1 = QK8_0 = 32)

#pragma pack(push, 1)
struct block_q4_0 { uint16_t d; uint8_t qs[QK / 2]; };
struct block_q4_1 { uint16_t d; uint16_t m; uint8_t qs[QK / 2]; };
#pragma pack(pop)
static_assert(sizeof(block_q4_0) == 18, "q4_0 block");
static_assert(sizeof(block_q4_1) == 20, "q4_1 block");

inline uint32_t f32_bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float bits_f32(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

// binary32 -> binary16, round-to-nearest-even (what F16C _cvtss_sh(x, 0) does;
// reference CMakeLists.txt:167 enables -mf16c).  Pure integer arithmetic so the
// result does not depend on the host FPU mode.
inline uint16_t f32_to_f16(float f) {
    const uint32_t x = f32_bits(f);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t exp = (x >> 23) & 0xffu;
    uint32_t man = x & 0x7fffffu;
    if (exp == 0xffu) return (uint16_t)(sign | 0x7c00u | (man ? (0x200u | (man >> 13)) : 0u));
    const int e = (int)exp - 127 + 15;
    if (e >= 31) return (uint16_t)(sign | 0x7c00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        man |= 0x800000u;
        const int shift = 14 - e;
        uint32_t h = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1u);
        const uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) h++;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)e << 10) | (man >> 13);
    const uint32_t rem = man & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;  // carry may roll into inf: correct
    return (uint16_t)(sign | h);
}

inline float f16_to_f32(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1fu;
    uint32_t man = h & 0x3ffu;
    uint32_t bits;
    if (exp == 0) {
        if (man == 0) {
            bits = sign;
        } else {
            int e = -1;
            do { man <<= 1; e++; } while (!(man & 0x400u));
            man &= 0x3ffu;
            bits = sign | ((uint32_t)(127 - 15 - e) << 23) | (man << 13);
        }
    } else if (exp == 31) {
        bits = sign | 0x7f800000u | (man << 13);
    } else {
        bits = sign | ((exp + 112u) << 23) | (man << 13);
    }
    return bits_f32(bits);
}

inline size_t ggml_row_bytes(uint32_t type, int64_t ne0) {
    switch (type) {
        case GT_F32: return (size_t)ne0 * 4;
        case GT_F16: return (size_t)ne0 * 2;
        case GT_Q4_0: return (size_t)(ne0 / QK) * sizeof(block_q4_0);
        case GT_Q4_1: return (size_t)(ne0 / QK) * sizeof(block_q4_1);
        case GT_Q8_0: return (size_t)(ne0 / QK) * 34;
        case GT_Q8_1: return (size_t)(ne0 / QK) * 40;
        default: return 0;
    }
}

inline const char *ggml_type_str(uint32_t type) {
    switch (type) {
        case GT_F32: return "f32";
        case GT_F16: return "f16";
        case GT_Q4_0: return "q4_0";
        case GT_Q4_1: return "q4_1";
        case GT_Q8_0: return "q8_0";
        case GT_Q8_1: return "q8_1";
        default: return "?";
    }
}

// Reference quantisers used by bert_model_quantize via ggml_quantize_chunk
// (reference bert.cpp:1487-1534; ggml quantize_row_q4_{0,1}_reference).
void quantize_row_q4_0(const float *x, block_q4_0 *y, int64_t k);
void quantize_row_q4_1(const float *x, block_q4_1 *y, int64_t k);
void dequantize_row(uint32_t type, const void *src, float *dst, int64_t k);

}  // namespace bertamd
