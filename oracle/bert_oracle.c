/*
 * bert_oracle.c — CPU restatement of the reference's embedding path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (build/libbert.so) links,
 * loads or calls this file; only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, as the checker.
 *
 * What it restates (one sentence at a time, exactly like the reference loop
 * at /root/reference/bert.cpp:1065-1107):
 *   - bert_build, reference bert.cpp:845-1012: op order and association;
 *   - the ggml@8ca2c19 CPU numerics of every op on that graph (ggml is an
 *     un-vendored submodule, reference .gitmodules:1-5; restated from the
 *     published ggml sources of that era):
 *       get_rows dequantisation, ggml_norm (double accumulators),
 *       mul_mat with vec_dot_type conversion of src1 (F16: fp16 RNE;
 *       Q4_0: Q8_0; Q4_1: Q8_1, AVX2 quantiser), the AVX/AVX2 dot kernels
 *       (8-lane accumulators, fma, hsum order), soft_max through the fp16
 *       exp table with a double sum, gelu through the fp16 tanh-GELU table,
 *       sum in double, sqrtf, 1/len, scale;
 *   - the output is graph node n-1 (the normalised vector); the reference
 *     copies node n-2 (bert.cpp:1085,1098), an over-read of the 1-element DIV
 *     node that this oracle deliberately does not replicate.
 *   - tensor names / shapes: bert.cpp:623-652; hparams: bert.cpp:496-513.
 *
 * PARITY STATUS: "parity unpinned" by the reference itself — the reference
 * holds no embedding golden vectors (examples/test_embedding.cpp prints only)
 * and cannot be built here (ggml and tokenizers-cpp absent).  The restatement
 * is cross-checked in tests/ against (i) an independent numpy restatement of
 * the same semantics and (ii) a locally constructed transformers.BertModel
 * (semantic check); see DESIGN.md §5.
 *
 * Threads: every row-parallel op is split over n_threads with OpenMP; the
 * result does not depend on the thread count (same as ggml).
 */
#include <fcntl.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <immintrin.h>

#define QK 32
enum { T_F32 = 0, T_F16 = 1, T_Q4_0 = 2, T_Q4_1 = 3 };

/* ------------------------------------------------------------------ fp16 */
static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* binary32 -> binary16 round-to-nearest-even (F16C _cvtss_sh(x, 0)) */
uint16_t oracle_f32_to_f16(float f) {
    uint32_t x = fbits(f), sign = (x >> 16) & 0x8000u, exp = (x >> 23) & 0xffu, man = x & 0x7fffffu;
    if (exp == 0xffu) return (uint16_t)(sign | 0x7c00u | (man ? (0x200u | (man >> 13)) : 0u));
    int e = (int)exp - 112;
    if (e >= 31) return (uint16_t)(sign | 0x7c00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        man |= 0x800000u;
        int sh = 14 - e;
        uint32_t h = man >> sh, rem = man & ((1u << sh) - 1u), half = 1u << (sh - 1);
        if (rem > half || (rem == half && (h & 1u))) h++;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)e << 10) | (man >> 13), rem = man & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
}

float oracle_f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16, exp = (h >> 10) & 0x1fu, man = h & 0x3ffu, b;
    if (exp == 0) {
        if (!man) b = sign;
        else {
            int e = -1;
            do { man <<= 1; e++; } while (!(man & 0x400u));
            b = sign | ((uint32_t)(112 - e) << 23) | ((man & 0x3ffu) << 13);
        }
    } else if (exp == 31) b = sign | 0x7f800000u | (man << 13);
    else b = sign | ((exp + 112u) << 23) | (man << 13);
    return bitsf(b);
}

static int g_simd = 0; /* the AVX2-intrinsics form of the checker (oracle_set_simd, below) */
/* fp16 <-> f32: the bit-exact software conversions, or F16C's vcvtps2ph (round
   to nearest even) / vcvtph2ps in the SIMD form — the same values for every
   non-NaN input (tests/test_oracle.py::test_fp16_conversion_bit_exact,
   ::test_simd_oracle_bitwise_scalar) */
static float F16(uint16_t h) { return g_simd ? _cvtsh_ss(h) : oracle_f16_to_f32(h); }
static uint16_t H16(float f) { return g_simd ? (uint16_t)_cvtss_sh(f, _MM_FROUND_TO_NEAREST_INT) : oracle_f32_to_f16(f); }

/* ggml_init builds these once (fp16 in, fp16 out). */
static uint16_t g_tab_gelu[65536], g_tab_exp[65536];
static int g_tabs_ready = 0;

static float gelu_f32(float x) {
    /* ggml_gelu_f32 (tanh form); gcc -O3 -mfma contracts 1+A*x*x into an fma */
    const float A = 0.044715f, S = 0.79788456080286535587989211986876f;
    return 0.5f * x * (1.0f + tanhf(S * x * fmaf(A * x, x, 1.0f)));
}

static void build_tables(void) {
    if (g_tabs_ready) return;
    for (int i = 0; i < 65536; i++) {
        float f = F16((uint16_t)i);
        g_tab_gelu[i] = H16(gelu_f32(f));
        g_tab_exp[i] = H16(expf(f));
    }
    g_tabs_ready = 1;
}

uint16_t oracle_tab_gelu(uint16_t h) { build_tables(); return g_tab_gelu[h]; }
uint16_t oracle_tab_exp(uint16_t h) { build_tables(); return g_tab_exp[h]; }

/* ------------------------------------------------------------ GGUF reader */
typedef struct { char name[96]; int nd; int64_t ne[4]; uint32_t type; uint64_t off; const uint8_t *data; } gtensor;

typedef struct {
    int n_vocab, n_max, n_embd, n_inter, n_head, n_layer;
    float eps;
    uint32_t wtype; /* type of the 2-D weights (vec_dot_type follows from it) */
    void *map; size_t map_size;
    int n_t; gtensor *t;
    /* per-tensor pointers */
    const gtensor *word, *pos, *type, *ln_e_w, *ln_e_b;
    struct olayer { const gtensor *q_w, *q_b, *k_w, *k_b, *v_w, *v_b, *o_w, *o_b, *ln1_w, *ln1_b,
                     *i_w, *i_b, *o2_w, *o2_b, *ln2_w, *ln2_b; } *L;
} omodel;

typedef struct { const uint8_t *p, *end; int ok; } cur_t;
static int need(cur_t *c, size_t n) { if (!c->ok || (size_t)(c->end - c->p) < n) { c->ok = 0; return 0; } return 1; }
static uint64_t rd(cur_t *c, int n) { uint64_t v = 0; if (need(c, n)) { memcpy(&v, c->p, n); c->p += n; } return v; }
static void rd_str(cur_t *c, const uint8_t **s, uint64_t *n) { *n = rd(c, 8); *s = c->p; if (need(c, *n)) c->p += *n; }
static int vsize(uint32_t t) {
    switch (t) { case 0: case 1: case 7: return 1; case 2: case 3: return 2; case 4: case 5: case 6: return 4;
                 case 10: case 11: case 12: return 8; default: return 0; }
}

static size_t row_bytes(uint32_t type, int64_t ne0) {
    switch (type) { case T_F32: return ne0 * 4; case T_F16: return ne0 * 2;
                    case T_Q4_0: return ne0 / QK * 18; case T_Q4_1: return ne0 / QK * 20; default: return 0; }
}

static const gtensor *find_t(omodel *m, const char *name) {
    for (int i = 0; i < m->n_t; i++) if (!strcmp(m->t[i].name, name)) return &m->t[i];
    return NULL;
}

static int key_is(const uint8_t *s, uint64_t n, const char *k) { return strlen(k) == n && !memcmp(s, k, n); }

void oracle_free(void *vm) {
    omodel *m = (omodel *)vm;
    if (!m) return;
    if (m->map) munmap(m->map, m->map_size);
    free(m->t); free(m->L); free(m);
}

void *oracle_load(const char *path) {
    build_tables();
    int fd = open(path, O_RDONLY);
    if (fd < 0) return NULL;
    struct stat st; fstat(fd, &st);
    omodel *m = (omodel *)calloc(1, sizeof(omodel));
    m->map_size = st.st_size;
    m->map = mmap(NULL, m->map_size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (m->map == MAP_FAILED) { free(m); return NULL; }
    cur_t c = {(const uint8_t *)m->map, (const uint8_t *)m->map + m->map_size, 1};
    if (rd(&c, 4) != 0x46554747u) { oracle_free(m); return NULL; }
    uint32_t ver = (uint32_t)rd(&c, 4);
    if (ver != 2 && ver != 3) { oracle_free(m); return NULL; }
    uint64_t n_t = rd(&c, 8), n_kv = rd(&c, 8);
    size_t align = 32;
    for (uint64_t i = 0; i < n_kv && c.ok; i++) {
        const uint8_t *k; uint64_t kn; rd_str(&c, &k, &kn);
        uint32_t t = (uint32_t)rd(&c, 4);
        if (t == 8) { const uint8_t *s; uint64_t sn; rd_str(&c, &s, &sn); continue; }
        if (t == 9) {
            uint32_t at = (uint32_t)rd(&c, 4); uint64_t an = rd(&c, 8);
            if (key_is(k, kn, "tokenizer.ggml.tokens")) m->n_vocab = (int)an;
            if (at == 8) { for (uint64_t j = 0; j < an && c.ok; j++) { const uint8_t *s; uint64_t sn; rd_str(&c, &s, &sn); } }
            else { size_t b = (size_t)an * vsize(at); if (need(&c, b)) c.p += b; }
            continue;
        }
        uint64_t raw = rd(&c, vsize(t));
        uint32_t u = (uint32_t)raw; float f; memcpy(&f, &u, 4);
        if (key_is(k, kn, "bert.context_length")) m->n_max = (int)u;
        else if (key_is(k, kn, "bert.embedding_length")) m->n_embd = (int)u;
        else if (key_is(k, kn, "bert.feed_forward_length")) m->n_inter = (int)u;
        else if (key_is(k, kn, "bert.attention.head_count")) m->n_head = (int)u;
        else if (key_is(k, kn, "bert.block_count")) m->n_layer = (int)u;
        else if (key_is(k, kn, "bert.attention.layer_norm_epsilon")) m->eps = f;
        else if (key_is(k, kn, "general.alignment")) align = (size_t)u;
    }
    m->n_t = (int)n_t;
    m->t = (gtensor *)calloc(n_t, sizeof(gtensor));
    for (uint64_t i = 0; i < n_t && c.ok; i++) {
        const uint8_t *s; uint64_t sn; rd_str(&c, &s, &sn);
        gtensor *t = &m->t[i];
        memcpy(t->name, s, sn < 95 ? sn : 95);
        t->nd = (int)rd(&c, 4);
        for (int d = 0; d < 4; d++) t->ne[d] = 1;
        for (int d = 0; d < t->nd; d++) t->ne[d] = (int64_t)rd(&c, 8);
        t->type = (uint32_t)rd(&c, 4);
        t->off = rd(&c, 8);
    }
    if (!c.ok) { oracle_free(m); return NULL; }
    size_t data = (size_t)(c.p - (const uint8_t *)m->map);
    data = (data + align - 1) / align * align;
    for (int i = 0; i < m->n_t; i++) m->t[i].data = (const uint8_t *)m->map + data + m->t[i].off;

    m->word = find_t(m, "embeddings.word_embeddings.weight");
    m->pos = find_t(m, "embeddings.position_embeddings.weight");
    m->type = find_t(m, "embeddings.token_type_embeddings.weight");
    m->ln_e_w = find_t(m, "embeddings.LayerNorm.weight");
    m->ln_e_b = find_t(m, "embeddings.LayerNorm.bias");
    if (!m->word || !m->pos || !m->type || !m->ln_e_w || !m->ln_e_b || m->n_layer <= 0) { oracle_free(m); return NULL; }
    m->L = (struct olayer *)calloc(m->n_layer, sizeof(struct olayer));
    char nm[160];
#define GET(field, suffix) do { snprintf(nm, sizeof nm, "encoder.layer.%d.%s", il, suffix); \
        m->L[il].field = find_t(m, nm); if (!m->L[il].field) { oracle_free(m); return NULL; } } while (0)
    for (int il = 0; il < m->n_layer; il++) {
        GET(q_w, "attention.self.query.weight"); GET(q_b, "attention.self.query.bias");
        GET(k_w, "attention.self.key.weight"); GET(k_b, "attention.self.key.bias");
        GET(v_w, "attention.self.value.weight"); GET(v_b, "attention.self.value.bias");
        GET(o_w, "attention.output.dense.weight"); GET(o_b, "attention.output.dense.bias");
        GET(ln1_w, "attention.output.LayerNorm.weight"); GET(ln1_b, "attention.output.LayerNorm.bias");
        GET(i_w, "intermediate.dense.weight"); GET(i_b, "intermediate.dense.bias");
        GET(o2_w, "output.dense.weight"); GET(o2_b, "output.dense.bias");
        GET(ln2_w, "output.LayerNorm.weight"); GET(ln2_b, "output.LayerNorm.bias");
    }
#undef GET
    m->wtype = m->L[0].q_w->type;
    return m;
}

int oracle_hparams(void *vm, int32_t *hp) {
    omodel *m = (omodel *)vm;
    hp[0] = m->n_vocab; hp[1] = m->n_max; hp[2] = m->n_embd; hp[3] = m->n_inter;
    hp[4] = m->n_head; hp[5] = m->n_layer; hp[6] = (int32_t)m->wtype;
    return 0;
}

/* --------------------------------------------------------- dequantisation */
static void dequant_row(uint32_t type, const uint8_t *src, float *dst, int64_t k) {
    if (type == T_F32) { memcpy(dst, src, k * 4); return; }
    if (type == T_F16) { const uint16_t *s = (const uint16_t *)src; for (int64_t i = 0; i < k; i++) dst[i] = F16(s[i]); return; }
    for (int64_t b = 0; b < k / QK; b++) {
        if (type == T_Q4_0) {
            const uint8_t *blk = src + b * 18; uint16_t dh; memcpy(&dh, blk, 2);
            float d = F16(dh);
            for (int j = 0; j < 16; j++) {
                dst[b * QK + j] = (float)((blk[2 + j] & 15) - 8) * d;
                dst[b * QK + j + 16] = (float)((blk[2 + j] >> 4) - 8) * d;
            }
        } else {
            const uint8_t *blk = src + b * 20; uint16_t dh, mh; memcpy(&dh, blk, 2); memcpy(&mh, blk + 2, 2);
            float d = F16(dh), mn = F16(mh);
            for (int j = 0; j < 16; j++) {
                dst[b * QK + j] = fmaf((float)(blk[4 + j] & 15), d, mn);
                dst[b * QK + j + 16] = fmaf((float)(blk[4 + j] >> 4), d, mn);
            }
        }
    }
}

/* ------------------------------------------------ vec_dot_type conversion */
/* quantize_row_q8_0 / q8_1, AVX2 variant: d = amax/127, q = rint(x * (127/amax)) */
typedef struct { float d; float s; int8_t q[QK]; } q8blk; /* d already fp16-rounded for Q8_0 */

void oracle_quantize_q8(const float *x, int64_t k, int is_q8_1, float *d_out, float *s_out, int8_t *q_out) {
    for (int64_t b = 0; b < k / QK; b++) {
        float amax = 0.0f;
        for (int j = 0; j < QK; j++) { float a = fabsf(x[b * QK + j]); amax = a > amax ? a : amax; }
        const float d = amax / 127.f;
        const float id = amax != 0.0f ? 127.f / amax : 0.0f;
        int isum = 0;
        for (int j = 0; j < QK; j++) {
            int q = (int)rintf(x[b * QK + j] * id);
            q_out[b * QK + j] = (int8_t)q;
            isum += q;
        }
        d_out[b] = is_q8_1 ? d : F16(H16(d));
        if (s_out) s_out[b] = d * (float)isum;
    }
}

/* Summation order of the dot kernels.  ggml computes the same products in a
   different f32 order per build; every order below is one a ggml@8ca2c19
   build of the reference runs (ggml.c: the AVX2 branch, the plain-C fallback
   after the SIMD #if chain, and the AVX-512 register width), so the spread
   between them measures how sensitive a model/input is to f32-level
   reassociation — the bound any non-ggml implementation can be held to
   (tests/golden/make_golden.py).
     0: AVX2 (the default checker)        1: plain C (generic fallback)
     2: 16-lane (AVX-512 register width) */
static int g_dot_variant = 0;
void oracle_set_dot_variant(int v) { g_dot_variant = v; }

static float dot_f32_generic(int n, const float *x, const float *y) {
    double sumf = 0.0; /* ggml_float */
    for (int i = 0; i < n; i++) sumf += (double)(x[i] * y[i]);
    return (float)sumf;
}
static float dot_f16_generic(int n, const uint16_t *x, const uint16_t *y) {
    double sumf = 0.0;
    for (int i = 0; i < n; i++) sumf += (double)(F16(x[i]) * F16(y[i]));
    return (float)sumf;
}
/* 16 lanes: one accumulator per lane, then 16 -> 8 -> the AVX2 hsum tail */
static float dot_f32_16(int n, const float *x, const float *y, int half) {
    float acc[16] = {0};
    int np = n & ~15;
    for (int i = 0; i < np; i += 16)
        for (int l = 0; l < 16; l++)
            acc[l] = fmaf(half ? F16(((const uint16_t *)x)[i + l]) : x[i + l],
                          half ? F16(((const uint16_t *)y)[i + l]) : y[i + l], acc[l]);
    for (int l = 0; l < 8; l++) acc[l] += acc[l + 8];
    float r4[4];
    for (int l = 0; l < 4; l++) r4[l] = acc[l + 4] + acc[l];
    float sumf = (r4[0] + r4[1]) + (r4[2] + r4[3]);
    for (int i = np; i < n; i++)
        sumf = fmaf(half ? F16(((const uint16_t *)x)[i]) : x[i], half ? F16(((const uint16_t *)y)[i]) : y[i], sumf);
    return sumf;
}

/* ggml_vec_dot_f32 (AVX: 4 accumulators x 8 lanes, fma, tree reduce, hadd) */
static float dot_f32(int n, const float *x, const float *y) {
    if (g_dot_variant == 1) return dot_f32_generic(n, x, y);
    if (g_dot_variant == 2) return dot_f32_16(n, x, y, 0);
    float acc[4][8] = {{0}};
    int np = n & ~31;
    for (int i = 0; i < np; i += 32)
        for (int j = 0; j < 4; j++)
            for (int l = 0; l < 8; l++) acc[j][l] = fmaf(x[i + 8 * j + l], y[i + 8 * j + l], acc[j][l]);
    for (int l = 0; l < 8; l++) { acc[0][l] += acc[2][l]; acc[1][l] += acc[3][l]; }
    for (int l = 0; l < 8; l++) acc[0][l] += acc[1][l];
    float r4[4];
    for (int l = 0; l < 4; l++) r4[l] = acc[0][l + 4] + acc[0][l];
    /* _mm_hadd_ps(t0,t0) twice */
    float h0 = r4[0] + r4[1], h1 = r4[2] + r4[3];
    float sumf = h0 + h1;
    for (int i = np; i < n; i++) sumf = fmaf(x[i], y[i], sumf); /* contracted by gcc -mfma */
    return sumf;
}

/* ggml_vec_dot_f16: fp16 inputs widened to f32, same SIMD structure, double leftovers */
static float dot_f16(int n, const uint16_t *x, const uint16_t *y) {
    if (g_dot_variant == 1) return dot_f16_generic(n, x, y);
    if (g_dot_variant == 2) return dot_f32_16(n, (const float *)x, (const float *)y, 1);
    float acc[4][8] = {{0}};
    int np = n & ~31;
    for (int i = 0; i < np; i += 32)
        for (int j = 0; j < 4; j++)
            for (int l = 0; l < 8; l++)
                acc[j][l] = fmaf(F16(x[i + 8 * j + l]), F16(y[i + 8 * j + l]), acc[j][l]);
    for (int l = 0; l < 8; l++) { acc[0][l] += acc[2][l]; acc[1][l] += acc[3][l]; }
    for (int l = 0; l < 8; l++) acc[0][l] += acc[1][l];
    float r4[4];
    for (int l = 0; l < 4; l++) r4[l] = acc[0][l + 4] + acc[0][l];
    double sumf = (double)((r4[0] + r4[1]) + (r4[2] + r4[3]));
    for (int i = np; i < n; i++) sumf += (double)(F16(x[i]) * F16(y[i]));
    return (float)sumf;
}

/* hsum_float_8 */
static float hsum8(const float *a) {
    float r[4];
    for (int l = 0; l < 4; l++) r[l] = a[l + 4] + a[l];
    r[0] += r[2]; r[1] += r[3];
    return r[0] + r[1];
}

/* ggml_vec_dot_q4_0_q8_0 (AVX2): per block 8 lanes of 4-product int sums,
   acc_l = fma(fp16(dw)*fp16(da), lane_l, acc_l) */
static float dot_q4_0_q8_0(int n, const uint8_t *w, const float *ad, const int8_t *aq) {
    float acc[16] = {0};
    float sumf = 0.0f;
    for (int b = 0; b < n / QK; b++) {
        const uint8_t *blk = w + b * 18; uint16_t dh; memcpy(&dh, blk, 2);
        const float d = F16(dh) * ad[b];
        int8_t wq[QK];
        for (int j = 0; j < 16; j++) { wq[j] = (int8_t)((blk[2 + j] & 15) - 8); wq[j + 16] = (int8_t)((blk[2 + j] >> 4) - 8); }
        if (g_dot_variant == 1) { /* sumf += sumi*d_x*d_y (gcc contracts the add into an fma) */
            int sumi = 0;
            for (int j = 0; j < QK; j++) sumi += wq[j] * aq[b * QK + j];
            sumf = fmaf((float)sumi * F16(dh), ad[b], sumf);
            continue;
        }
        if (g_dot_variant == 2) { /* 16 lanes of 2-product sums */
            for (int l = 0; l < 16; l++) {
                const int s2 = wq[2 * l] * aq[b * QK + 2 * l] + wq[2 * l + 1] * aq[b * QK + 2 * l + 1];
                acc[l] = fmaf(d, (float)s2, acc[l]);
            }
            continue;
        }
        for (int l = 0; l < 8; l++) {
            int s = 0;
            for (int j = 0; j < 4; j++) s += wq[4 * l + j] * aq[b * QK + 4 * l + j];
            acc[l] = fmaf(d, (float)s, acc[l]);
        }
    }
    if (g_dot_variant == 1) return sumf;
    if (g_dot_variant == 2) for (int l = 0; l < 8; l++) acc[l] += acc[l + 8];
    return hsum8(acc);
}

/* ggml_vec_dot_q4_1_q8_1 (AVX2): acc_l = fma(d0*d1, lane_l, acc_l); + sum m*s */
static float dot_q4_1_q8_1(int n, const uint8_t *w, const float *ad, const float *as, const int8_t *aq) {
    float acc[16] = {0};
    float summs = 0.0f, sumf = 0.0f;
    for (int b = 0; b < n / QK; b++) {
        const uint8_t *blk = w + b * 20; uint16_t dh, mh; memcpy(&dh, blk, 2); memcpy(&mh, blk + 2, 2);
        const float d0 = F16(dh), m0 = F16(mh);
        const float d = d0 * ad[b];
        int wq[QK];
        for (int j = 0; j < 16; j++) { wq[j] = blk[4 + j] & 15; wq[j + 16] = blk[4 + j] >> 4; }
        if (g_dot_variant == 1) { /* sumf += (d_x*d_y)*sumi + m_x*s_y */
            int sumi = 0;
            for (int j = 0; j < QK; j++) sumi += wq[j] * aq[b * QK + j];
            sumf += fmaf(d, (float)sumi, m0 * as[b]);
            continue;
        }
        summs += m0 * as[b];
        if (g_dot_variant == 2) {
            for (int l = 0; l < 16; l++) {
                const int s2 = wq[2 * l] * aq[b * QK + 2 * l] + wq[2 * l + 1] * aq[b * QK + 2 * l + 1];
                acc[l] = fmaf(d, (float)s2, acc[l]);
            }
            continue;
        }
        for (int l = 0; l < 8; l++) {
            int s = 0;
            for (int j = 0; j < 4; j++) s += wq[4 * l + j] * aq[b * QK + 4 * l + j];
            acc[l] = fmaf(d, (float)s, acc[l]);
        }
    }
    if (g_dot_variant == 1) return sumf;
    if (g_dot_variant == 2) for (int l = 0; l < 8; l++) acc[l] += acc[l + 8];
    return hsum8(acc) + summs;
}

/* ----------------------------------------------------------------- ops */
typedef struct {
    int K;              /* row length */
    uint32_t vtype;     /* vec_dot_type of the weight */
    float *f;           /* F32 rows      [N][K] (points at the source) */
    uint16_t *h;        /* F16 rows      [N][K] */
    float *d, *s;       /* Q8 scales     [N][K/32] */
    int8_t *q;          /* Q8 quants     [N][K] */
} act_t;

static void act_convert(act_t *a, const float *x, int N, int K, uint32_t wtype) {
    a->K = K; a->vtype = wtype; a->f = (float *)x;
    if (wtype == T_F16) {
        a->h = (uint16_t *)malloc((size_t)N * K * 2);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)N * K; i++) a->h[i] = H16(x[i]);
    } else if (wtype == T_Q4_0 || wtype == T_Q4_1) {
        a->d = (float *)malloc((size_t)N * (K / QK) * 4);
        a->s = (float *)malloc((size_t)N * (K / QK) * 4);
        a->q = (int8_t *)malloc((size_t)N * K);
#pragma omp parallel for schedule(static)
        for (int t = 0; t < N; t++)
            oracle_quantize_q8(x + (size_t)t * K, K, wtype == T_Q4_1, a->d + (size_t)t * (K / QK),
                               a->s + (size_t)t * (K / QK), a->q + (size_t)t * K);
    }
}
static void act_free(act_t *a) { free(a->h); free(a->d); free(a->s); free(a->q); memset(a, 0, sizeof *a); }

/* The AVX2 checker (variant 0) over one weight row unpacked once (below):
   identical operations to dot_f32 / dot_f16 / dot_q4_x_q8_x, without the
   per-call variant test and the per-(row, token) re-decoding of the weight
   blocks, so the compiler can vectorise the lane loops.  Variants 1 and 2
   (ggml's other build orders, only used to measure the spread) keep the
   per-call functions above. */
static float dot_f32_rows(int n, const float *x, const float *y) { /* = dot_f32 variant 0 */
    float acc[4][8] = {{0}};
    int np = n & ~31;
    for (int i = 0; i < np; i += 32)
        for (int j = 0; j < 4; j++)
            for (int l = 0; l < 8; l++) acc[j][l] = fmaf(x[i + 8 * j + l], y[i + 8 * j + l], acc[j][l]);
    for (int l = 0; l < 8; l++) { acc[0][l] += acc[2][l]; acc[1][l] += acc[3][l]; }
    for (int l = 0; l < 8; l++) acc[0][l] += acc[1][l];
    float r4[4];
    for (int l = 0; l < 4; l++) r4[l] = acc[0][l + 4] + acc[0][l];
    return (r4[0] + r4[1]) + (r4[2] + r4[3]);
}
static float dot_f16_rows(int n, const float *x, const float *y) { /* = dot_f16 variant 0, inputs pre-widened */
    int np = n & ~31;
    double sumf = (double)dot_f32_rows(np, x, y);
    for (int i = np; i < n; i++) sumf += (double)(x[i] * y[i]);
    return (float)sumf;
}
/* = dot_q4_0_q8_0 / dot_q4_1_q8_1 variant 0; wq: the row's codes (q - 8 for
   Q4_0, q for Q4_1), wd / wm: its fp16 d (and m) widened */
static float dot_q4_rows(int n, const int8_t *wq, const float *wd, const float *wm, const float *ad, const float *as,
                         const int8_t *aq) {
    float acc[8] = {0};
    float summs = 0.0f;
    for (int b = 0; b < n / QK; b++) {
        const float d = wd[b] * ad[b];
        if (wm) summs += wm[b] * as[b];
        const int8_t *w = wq + b * QK, *a = aq + b * QK;
        for (int l = 0; l < 8; l++) {
            const int s = w[4 * l] * a[4 * l] + w[4 * l + 1] * a[4 * l + 1] + w[4 * l + 2] * a[4 * l + 2] +
                          w[4 * l + 3] * a[4 * l + 3];
            acc[l] = fmaf(d, (float)s, acc[l]);
        }
    }
    return wm ? hsum8(acc) + summs : hsum8(acc);
}

/* ----------------------------------------------------- AVX2 intrinsics
   The same AVX2-order checker (variant 0) written with the instructions
   ggml's AVX2 build runs (reference CMakeLists.txt:164-177 builds ggml with
   -mavx2 -mfma -mf16c; ggml.c ggml_vec_dot_q4_0_q8_0 / _q4_1_q8_1 /
   ggml_vec_dot_f32 / _f16, AVX2 branches): per Q4 block
   sign/maddubs/madd give the 8 lanes of 4-product integer sums, cvt, one
   vfmadd per lane into 8-lane accumulators; f32 dots on 4 x 8-lane fma
   accumulators.  Every lane operation is the scalar variant-0 code's own
   (same fma, same adds in the same order), so results are bitwise the
   scalar checker's (tests/test_oracle.py::test_simd_oracle_bitwise_scalar);
   it exists to time the CPU baseline at ggml's SIMD speed (bench.py
   cpu_baseline).  Off by default (oracle_set_simd). */
void oracle_set_simd(int on) { g_simd = on; }
int oracle_simd_available(void) {
    return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma") && __builtin_cpu_supports("f16c");
}

static inline float hsum8_v(__m256 v) {
    float a[8];
    _mm256_storeu_ps(a, v);
    return hsum8(a);
}

/* = dot_f32_rows */
static float dot_f32_rows_avx2(int n, const float *x, const float *y) {
    __m256 a0 = _mm256_setzero_ps(), a1 = a0, a2 = a0, a3 = a0;
    const int np = n & ~31;
    for (int i = 0; i < np; i += 32) {
        a0 = _mm256_fmadd_ps(_mm256_loadu_ps(x + i), _mm256_loadu_ps(y + i), a0);
        a1 = _mm256_fmadd_ps(_mm256_loadu_ps(x + i + 8), _mm256_loadu_ps(y + i + 8), a1);
        a2 = _mm256_fmadd_ps(_mm256_loadu_ps(x + i + 16), _mm256_loadu_ps(y + i + 16), a2);
        a3 = _mm256_fmadd_ps(_mm256_loadu_ps(x + i + 24), _mm256_loadu_ps(y + i + 24), a3);
    }
    a0 = _mm256_add_ps(a0, a2);
    a1 = _mm256_add_ps(a1, a3);
    a0 = _mm256_add_ps(a0, a1);
    float t[8];
    _mm256_storeu_ps(t, a0);
    float r4[4];
    for (int l = 0; l < 4; l++) r4[l] = t[l + 4] + t[l];
    return (r4[0] + r4[1]) + (r4[2] + r4[3]);
}
/* = dot_f32 variant 0 (rows part, then the fma tail) */
static float dot_f32_avx2(int n, const float *x, const float *y) {
    float sumf = dot_f32_rows_avx2(n, x, y);
    for (int i = n & ~31; i < n; i++) sumf = fmaf(x[i], y[i], sumf);
    return sumf;
}
/* the attention / pool dots: the SIMD form when it is on (variant 0 only) */
static float dot_f32_any(int n, const float *x, const float *y) {
    return (g_simd && g_dot_variant == 0) ? dot_f32_avx2(n, x, y) : dot_f32(n, x, y);
}

/* = dot_q4_rows for NT consecutive tokens (their Q8 rows K apart, scales
   K / QK apart): one weight block load serves the tokens.  NT is a
   compile-time constant in the hot call (8 accumulators in registers). */
#define Q4_NT 8
static inline __attribute__((always_inline)) void q4_rows_avx2_n(const int NT, int K, const int8_t *wq,
                                                                 const float *wd, const float *wm, const float *ad,
                                                                 const float *as, const int8_t *aq, float *out) {
    const int nb = K / QK;
    __m256 acc[Q4_NT];
    float summs[Q4_NT];
    for (int j = 0; j < NT; j++) { acc[j] = _mm256_setzero_ps(); summs[j] = 0.0f; }
    const __m256i ones = _mm256_set1_epi16(1);
    for (int b = 0; b < nb; b++) {
        const __m256i w = _mm256_loadu_si256((const __m256i *)(wq + b * QK));
        const __m256i aw = _mm256_sign_epi8(w, w); /* |w| as unsigned bytes */
        const float wdb = wd[b];
        for (int j = 0; j < NT; j++) {
            const float d = wdb * ad[(size_t)j * nb + b];
            if (wm) summs[j] += wm[b] * as[(size_t)j * nb + b];
            const __m256i a = _mm256_loadu_si256((const __m256i *)(aq + (size_t)j * K + b * QK));
            const __m256i p16 = _mm256_maddubs_epi16(aw, _mm256_sign_epi8(a, w)); /* |w| * (a sign w), pairs */
            const __m256i p32 = _mm256_madd_epi16(p16, ones);                      /* lane l: bytes 4l .. 4l + 3 */
            acc[j] = _mm256_fmadd_ps(_mm256_set1_ps(d), _mm256_cvtepi32_ps(p32), acc[j]);
        }
    }
    for (int j = 0; j < NT; j++) out[j] = wm ? hsum8_v(acc[j]) + summs[j] : hsum8_v(acc[j]);
}
static void dot_q4_rows_avx2(int K, const int8_t *wq, const float *wd, const float *wm, const float *ad,
                             const float *as, const int8_t *aq, int nt, float *out) {
    if (nt == Q4_NT) {
        if (wm) q4_rows_avx2_n(Q4_NT, K, wq, wd, wm, ad, as, aq, out);
        else q4_rows_avx2_n(Q4_NT, K, wq, wd, NULL, ad, NULL, aq, out);
    } else {
        for (int j = 0; j < nt; j++)
            q4_rows_avx2_n(1, K, wq, wd, wm, ad + (size_t)j * (K / QK), wm ? as + (size_t)j * (K / QK) : NULL,
                           aq + (size_t)j * K, out + j);
    }
}

/* out[t][n] = bias[n] + (W . x_t)   — ggml_add(repeat(b), mul_mat(W, x)) */
static void mul_mat_bias(const gtensor *W, const gtensor *bias, const act_t *a, int N, float *out) {
    const int K = (int)W->ne[0], NO = (int)W->ne[1];
    const size_t rb = row_bytes(W->type, K);
    const float *b = (const float *)bias->data;
    const int fast = g_dot_variant == 0;
    float *hx = NULL; /* F16 activations widened once (exact) for the fast path */
    if (fast && W->type == T_F16) {
        hx = (float *)malloc((size_t)N * K * 4);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)N * K; i++) hx[i] = F16(a->h[i]);
    }
#pragma omp parallel
    {
        float *wf = (float *)malloc((size_t)K * 4), *wd = (float *)malloc((size_t)(K / QK + 1) * 4),
              *wm = (float *)malloc((size_t)(K / QK + 1) * 4);
        int8_t *wq = (int8_t *)malloc((size_t)K);
#pragma omp for schedule(static)
        for (int n = 0; n < NO; n++) {
            const uint8_t *wr = W->data + (size_t)n * rb;
            if (!fast) {
                for (int t = 0; t < N; t++) {
                    float v;
                    switch (W->type) {
                        case T_F32: v = dot_f32(K, (const float *)wr, a->f + (size_t)t * K); break;
                        case T_F16: v = dot_f16(K, (const uint16_t *)wr, a->h + (size_t)t * K); break;
                        case T_Q4_0: v = dot_q4_0_q8_0(K, wr, a->d + (size_t)t * (K / QK), a->q + (size_t)t * K); break;
                        default:
                            v = dot_q4_1_q8_1(K, wr, a->d + (size_t)t * (K / QK), a->s + (size_t)t * (K / QK),
                                              a->q + (size_t)t * K);
                            break;
                    }
                    out[(size_t)t * NO + n] = b[n] + v;
                }
                continue;
            }
            if (W->type == T_F16)
                for (int k = 0; k < K; k++) wf[k] = F16(((const uint16_t *)wr)[k]);
            if (W->type == T_Q4_0 || W->type == T_Q4_1) {
                const int q1 = W->type == T_Q4_1, bs = q1 ? 20 : 18, off = q1 ? 4 : 2;
                for (int bb = 0; bb < K / QK; bb++) {
                    const uint8_t *blk = wr + (size_t)bb * bs;
                    uint16_t dh, mh;
                    memcpy(&dh, blk, 2);
                    wd[bb] = F16(dh);
                    if (q1) { memcpy(&mh, blk + 2, 2); wm[bb] = F16(mh); }
                    for (int j = 0; j < 16; j++) {
                        wq[bb * QK + j] = (int8_t)((blk[off + j] & 15) - (q1 ? 0 : 8));
                        wq[bb * QK + j + 16] = (int8_t)((blk[off + j] >> 4) - (q1 ? 0 : 8));
                    }
                }
            }
            if (g_simd && (W->type == T_Q4_0 || W->type == T_Q4_1)) {
                const int q1 = W->type == T_Q4_1;
                for (int t = 0; t < N; t += Q4_NT) {
                    const int nt = N - t < Q4_NT ? N - t : Q4_NT;
                    float v[Q4_NT];
                    dot_q4_rows_avx2(K, wq, wd, q1 ? wm : NULL, a->d + (size_t)t * (K / QK),
                                     q1 ? a->s + (size_t)t * (K / QK) : NULL, a->q + (size_t)t * K, nt, v);
                    for (int j = 0; j < nt; j++) out[(size_t)(t + j) * NO + n] = b[n] + v[j];
                }
                continue;
            }
            if (g_simd) {
                for (int t = 0; t < N; t++) {
                    float v;
                    if (W->type == T_F32) {
                        v = dot_f32_avx2(K, (const float *)wr, a->f + (size_t)t * K);
                    } else { /* = dot_f16_rows */
                        const float *y = hx + (size_t)t * K;
                        const int np = K & ~31;
                        double sumf = (double)dot_f32_rows_avx2(np, wf, y);
                        for (int i = np; i < K; i++) sumf += (double)(wf[i] * y[i]);
                        v = (float)sumf;
                    }
                    out[(size_t)t * NO + n] = b[n] + v;
                }
                continue;
            }
            for (int t = 0; t < N; t++) {
                float v;
                switch (W->type) {
                    case T_F32: v = dot_f32(K, (const float *)wr, a->f + (size_t)t * K); break;
                    case T_F16: v = dot_f16_rows(K, wf, hx + (size_t)t * K); break;
                    case T_Q4_0:
                        v = dot_q4_rows(K, wq, wd, NULL, a->d + (size_t)t * (K / QK), NULL, a->q + (size_t)t * K);
                        break;
                    default:
                        v = dot_q4_rows(K, wq, wd, wm, a->d + (size_t)t * (K / QK), a->s + (size_t)t * (K / QK),
                                        a->q + (size_t)t * K);
                        break;
                }
                out[(size_t)t * NO + n] = b[n] + v;
            }
        }
        free(wf); free(wd); free(wm); free(wq);
    }
    free(hx);
}

/* ggml_norm then mul(repeat(w)) then add(repeat(b)), in place on x[N][E] */
static void layer_norm(float *x, int N, int E, const gtensor *w, const gtensor *b, float eps) {
    const float *wv = (const float *)w->data, *bv = (const float *)b->data;
#pragma omp parallel for schedule(static)
    for (int t = 0; t < N; t++) {
        float *r = x + (size_t)t * E;
        double sum = 0.0;
        for (int i = 0; i < E; i++) sum += (double)r[i];
        const float mean = (float)(sum / E);
        double sum2 = 0.0;
        for (int i = 0; i < E; i++) { float v = r[i] - mean; r[i] = v; sum2 += (double)(v * v); }
        const float var = (float)(sum2 / E);
        const float scale = 1.0f / sqrtf(var + eps);
        for (int i = 0; i < E; i++) r[i] *= scale;
        for (int i = 0; i < E; i++) r[i] = wv[i] * r[i];
        for (int i = 0; i < E; i++) r[i] = r[i] + bv[i];
    }
}

/* one sentence: reference bert_build (bert.cpp:845-1012) + compute */
/* embeddings: pos + (type[0] + word[id]) (bert.cpp:880-887), then the
   embedding LayerNorm (bert.cpp:889-898), into x[N][E] */
static void embed_ln(const omodel *m, const int32_t *tokens, int N, float *x) {
    const int E = m->n_embd;
    float *typ = (float *)malloc((size_t)E * 4);
    dequant_row(m->type->type, m->type->data, typ, E);
#pragma omp parallel for schedule(static)
    for (int t = 0; t < N; t++) {
        float *w = (float *)malloc((size_t)E * 4), *p = (float *)malloc((size_t)E * 4);
        dequant_row(m->word->type, m->word->data + (size_t)tokens[t] * row_bytes(m->word->type, E), w, E);
        dequant_row(m->pos->type, m->pos->data + (size_t)t * row_bytes(m->pos->type, E), p, E);
        for (int i = 0; i < E; i++) x[(size_t)t * E + i] = p[i] + (typ[i] + w[i]);
        free(w); free(p);
    }
    layer_norm(x, N, E, m->ln_e_w, m->ln_e_b, m->eps);
    free(typ);
}

/* the embedding stage alone (tests pin the GPU's embed_ln against it) */
int oracle_embed_ln(void *vm, const int32_t *tokens, int N, float *x_out) {
    omodel *m = (omodel *)vm;
    if (!m || N <= 0 || N > m->n_max) return -1;
    for (int i = 0; i < N; i++) if (tokens[i] < 0 || tokens[i] >= m->word->ne[1]) return -2;
    embed_ln(m, tokens, N, x_out);
    return 0;
}

/* Attention arithmetic (NOT a ggml build: a diagnostic).
     0: ggml's — K.Q and V.P as f32 dot products (in the dot variant's order),
        P scaled by 1/sum before V.P;
     1: the GPU kernels' operand form — K, Q and V carried as fp16 hi + lo
        pairs (hi = fp16(x), lo = fp16(x - hi): 22 significant bits instead of
        24), K.Q = sum(kh qh + kh ql + kl qh) (the lo.lo term dropped), V.P on
        the table's fp16 p with the 1/sum scale applied after; each dot summed
        exactly and rounded once (the MFMA's own f32 accumulation order is not
        restated).  Lets the tests measure how much of the GPU's distance to
        ggml comes from the attention operands rather than the GEMMs. */
static int g_attn_form = 0;
void oracle_set_attn_form(int f) { g_attn_form = f; }
static float split22(float x) {
    const float hi = F16(H16(x));
    return (float)((double)hi + (double)F16(H16(x - hi)));
}
static float dot_split(int n, const float *k, const float *q) {
    double s = 0.0;
    for (int i = 0; i < n; i++) {
        const double kh = F16(H16(k[i])), kl = (double)k[i] - kh, qh = F16(H16(q[i])), ql = (double)q[i] - qh;
        s += kh * qh + kh * ql + kl * qh;
    }
    return (float)s;
}

/* one encoder layer il on x[N][E] in place (bert.cpp:900-993) */
static void encoder_layer(const omodel *m, int il, float *x, int N) {
    const int E = m->n_embd, I = m->n_inter, H = m->n_head, D = E / H;
    float *tmp = (float *)malloc((size_t)N * E * 4);
    float *qkv = (float *)malloc((size_t)3 * N * E * 4), *ctx = (float *)malloc((size_t)N * E * 4);
    float *u = (float *)malloc((size_t)N * I * 4), *x1 = (float *)malloc((size_t)N * E * 4);
    const float kq_scale = 1.0f / sqrtf((float)D);
    const struct olayer *L = &m->L[il];
    act_t a = {0};
    act_convert(&a, x, N, E, L->q_w->type);
    float *Q = qkv, *K = qkv + (size_t)N * E, *V = qkv + (size_t)2 * N * E;
    mul_mat_bias(L->q_w, L->q_b, &a, N, Q);
    mul_mat_bias(L->k_w, L->k_b, &a, N, K);
    mul_mat_bias(L->v_w, L->v_b, &a, N, V);
    act_free(&a);
    /* attention per head (bert.cpp:930-942) */
#pragma omp parallel for schedule(static)
    for (int h = 0; h < H; h++) {
        float *kh = (float *)malloc((size_t)N * D * 4), *qh = (float *)malloc((size_t)N * D * 4);
        float *vt = (float *)malloc((size_t)D * N * 4), *P = (float *)malloc((size_t)N * 4);
        for (int t = 0; t < N; t++)
            for (int j = 0; j < D; j++) {
                kh[t * D + j] = K[(size_t)t * E + h * D + j];
                qh[t * D + j] = Q[(size_t)t * E + h * D + j];
                vt[(size_t)j * N + t] = V[(size_t)t * E + h * D + j]; /* ggml_cont(transpose(V)) */
            }
        if (g_attn_form == 1) { /* the GPU kernels' operand form (see oracle_set_attn_form) */
            for (int i = 0; i < N * D; i++) { kh[i] = split22(kh[i]); qh[i] = split22(qh[i]); vt[i] = split22(vt[i]); }
        }
        for (int q = 0; q < N; q++) {
            float mx = -INFINITY;
            for (int k = 0; k < N; k++) {
                const float s = g_attn_form == 1 ? dot_split(D, kh + k * D, qh + q * D) : dot_f32_any(D, kh + k * D, qh + q * D);
                P[k] = s * kq_scale;  /* mul_mat(K,Q), scale */
                mx = P[k] > mx ? P[k] : mx;
            }
            double sum = 0.0;
            for (int k = 0; k < N; k++) {
                if (P[k] == -INFINITY) { P[k] = 0.0f; continue; }
                const float val = F16(g_tab_exp[H16(P[k] - mx)]);
                sum += (double)val;
                P[k] = val;
            }
            const float r = (float)(1.0 / sum);
            if (g_attn_form == 1) { /* V.P on the table's fp16 values, then the 1/sum scale */
                for (int j = 0; j < D; j++) {
                    double acc = 0.0;
                    for (int k = 0; k < N; k++) acc += (double)P[k] * (double)vt[(size_t)j * N + k];
                    ctx[(size_t)q * E + h * D + j] = (float)acc * r;
                }
                continue;
            }
            for (int k = 0; k < N; k++) P[k] *= r;
            for (int j = 0; j < D; j++) ctx[(size_t)q * E + h * D + j] = dot_f32_any(N, vt + (size_t)j * N, P);
        }
        free(kh); free(qh); free(vt); free(P);
    }
    /* O-proj + residual + LN (bert.cpp:945-962) */
    act_convert(&a, ctx, N, E, L->o_w->type);
    mul_mat_bias(L->o_w, L->o_b, &a, N, x1);
    act_free(&a);
    for (int64_t i = 0; i < (int64_t)N * E; i++) x1[i] = x1[i] + x[i];
    layer_norm(x1, N, E, L->ln1_w, L->ln1_b, m->eps);
    /* FFN (bert.cpp:967-992) */
    act_convert(&a, x1, N, E, L->i_w->type);
    mul_mat_bias(L->i_w, L->i_b, &a, N, u);
    act_free(&a);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)N * I; i++) u[i] = F16(g_tab_gelu[H16(u[i])]);
    act_convert(&a, u, N, I, L->o2_w->type);
    mul_mat_bias(L->o2_w, L->o2_b, &a, N, tmp);
    act_free(&a);
    for (int64_t i = 0; i < (int64_t)N * E; i++) x[i] = x1[i] + tmp[i];
    layer_norm(x, N, E, L->ln2_w, L->ln2_b, m->eps);
    free(tmp); free(qkv); free(ctx); free(u); free(x1);
}

/* mean pool as mul_mat(cont(transpose(x)), 1/N) then L2 (bert.cpp:995-1006) */
static void pool_l2(const omodel *m, const float *x, int N, float *out) {
    const int E = m->n_embd;
    float *col = (float *)malloc((size_t)N * 4), *inv = (float *)malloc((size_t)N * 4);
    const float invN = 1.0f / N;
    for (int t = 0; t < N; t++) inv[t] = invN;
    for (int e = 0; e < E; e++) {
        for (int t = 0; t < N; t++) col[t] = x[(size_t)t * E + e];
        out[e] = dot_f32_any(N, col, inv);
    }
    double ss = 0.0;
    for (int e = 0; e < E; e++) ss += (double)(out[e] * out[e]);
    const float len = sqrtf((float)ss);
    const float r = 1.0f / len;
    for (int e = 0; e < E; e++) out[e] = out[e] * r;
    free(col); free(inv);
}

int oracle_eval(void *vm, const int32_t *tokens, int N, float *out) {
    omodel *m = (omodel *)vm;
    if (!m || N <= 0 || N > m->n_max) return -1;
    for (int i = 0; i < N; i++) if (tokens[i] < 0 || tokens[i] >= m->word->ne[1]) return -2;
    float *x = (float *)malloc((size_t)N * m->n_embd * 4);
    embed_ln(m, tokens, N, x);
    for (int il = 0; il < m->n_layer; il++) encoder_layer(m, il, x, N);
    pool_l2(m, x, N, out);
    free(x);
    return 0;
}

/* Per-stage residual stream of one sentence (tests pin the GPU layer by
   layer): xs_out[(n_layer + 1)][N][E], stage 0 the embedding LayerNorm
   output, stage l + 1 the output of encoder layer l (bert.cpp:900-993). */
int oracle_eval_layers(void *vm, const int32_t *tokens, int N, float *xs_out) {
    omodel *m = (omodel *)vm;
    if (!m || N <= 0 || N > m->n_max) return -1;
    for (int i = 0; i < N; i++) if (tokens[i] < 0 || tokens[i] >= m->word->ne[1]) return -2;
    const size_t st = (size_t)N * m->n_embd;
    embed_ln(m, tokens, N, xs_out);
    for (int il = 0; il < m->n_layer; il++) {
        memcpy(xs_out + (il + 1) * st, xs_out + il * st, st * 4);
        encoder_layer(m, il, xs_out + (il + 1) * st, N);
    }
    return 0;
}

/* One encoder layer il of one sentence from a given input x_in[N][E] (e.g.
   the GPU's own previous-stage output): separates a layer's own error from
   the error it inherits. */
int oracle_layer(void *vm, int il, const float *x_in, int N, float *x_out) {
    omodel *m = (omodel *)vm;
    if (!m || N <= 0 || N > m->n_max || il < 0 || il >= m->n_layer) return -1;
    memcpy(x_out, x_in, (size_t)N * m->n_embd * 4);
    encoder_layer(m, il, x_out, N);
    return 0;
}

/* reference bert_eval_batch loop: sentences one at a time */
int oracle_eval_batch(void *vm, const int32_t *tokens, const int32_t *offsets, int n_seq, float *out, int n_threads) {
    omodel *m = (omodel *)vm;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
    for (int s = 0; s < n_seq; s++) {
        int rc = oracle_eval(vm, tokens + offsets[s], offsets[s + 1] - offsets[s], out + (size_t)s * m->n_embd);
        if (rc) return rc;
    }
    return 0;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
