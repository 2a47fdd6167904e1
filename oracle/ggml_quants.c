/*
 * TEST INFRASTRUCTURE ONLY -- C restatement of ggml's K-quant dequantisers.
 *
 * Ollama's default tag llama3.2:3b is Q4_K_M, which stores most
 * matrices as Q4_K and some (attn_v / ffn_down of half the layers, output) as Q6_K.  The
 * dequantisers live in llama.cpp's ggml-quants.c (EXT: third-party, not vendored in the
 * reference, not present in this container, version unpinned -- SURVEY.md §8c).  This
 * file restates the published algorithms (dequantize_row_q4_K, dequantize_row_q6_K,
 * get_scale_min_k4, fp16 -> fp32) so the HIP dequant can be checked bit for bit.
 *
 * Floating-point contract: compiled with -ffp-contract=off (oracle/Makefile), i.e. the
 * non-fused forms  y = d1*q - m1  (Q4_K) and  y = (d*sc)*q  (Q6_K).  Whether a given
 * llama.cpp build contracts d1*q - m1 into an FMA depends on its compiler flags (EXT,
 * unpinned); the HIP kernels implement this same non-contracted form.
 *
 * Built by `make -C oracle` into oracle/_build/libggml_quants.so; used only by tests/.
 */
#include <stdint.h>
#include <string.h>

#define QK_K 256

typedef struct {
    uint16_t d;          /* fp16 super-block scale for the 6-bit scales */
    uint16_t dmin;       /* fp16 super-block scale for the 6-bit mins   */
    uint8_t scales[12];  /* 8 (scale, min) pairs, 6 bits each           */
    uint8_t qs[QK_K / 2];/* 4-bit quants                                */
} block_q4_K;           /* 144 bytes */

typedef struct {
    uint8_t ql[QK_K / 2];  /* low 4 bits  */
    uint8_t qh[QK_K / 4];  /* high 2 bits */
    int8_t scales[QK_K / 16];
    uint16_t d;            /* fp16 super-block scale */
} block_q6_K;             /* 210 bytes */

_Static_assert(sizeof(block_q4_K) == 144, "q4_K block size");
_Static_assert(sizeof(block_q6_K) == 210, "q6_K block size");

/* IEEE half -> float, exact (subnormals, inf, nan included) */
float ms_fp16_to_fp32(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1Fu;
    uint32_t man = h & 0x3FFu;
    uint32_t bits;
    if (exp == 0) {
        if (man == 0) {
            bits = sign;
        } else { /* subnormal: normalise */
            exp = 127 - 15 + 1;
            while ((man & 0x400u) == 0) { man <<= 1; exp -= 1; }
            man &= 0x3FFu;
            bits = sign | (exp << 23) | (man << 13);
        }
    } else if (exp == 0x1F) {
        bits = sign | 0x7F800000u | (man << 13);
    } else {
        bits = sign | ((exp + 127 - 15) << 23) | (man << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

static void get_scale_min_k4(int j, const uint8_t* q, uint8_t* d, uint8_t* m) {
    if (j < 4) {
        *d = q[j] & 63;
        *m = q[j + 4] & 63;
    } else {
        *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

/* k = number of weights (multiple of 256) */
void ms_dequantize_row_q4_K(const void* vx, float* y, int64_t k) {
    const block_q4_K* x = (const block_q4_K*)vx;
    const int64_t nb = k / QK_K;
    for (int64_t i = 0; i < nb; i++) {
        const uint8_t* q = x[i].qs;
        const float d = ms_fp16_to_fp32(x[i].d);
        const float min = ms_fp16_to_fp32(x[i].dmin);
        int is = 0;
        uint8_t sc, m;
        for (int j = 0; j < QK_K; j += 64) {
            get_scale_min_k4(is + 0, x[i].scales, &sc, &m);
            const float d1 = d * sc;
            const float m1 = min * m;
            get_scale_min_k4(is + 1, x[i].scales, &sc, &m);
            const float d2 = d * sc;
            const float m2 = min * m;
            for (int l = 0; l < 32; ++l) *y++ = d1 * (q[l] & 0xF) - m1;
            for (int l = 0; l < 32; ++l) *y++ = d2 * (q[l] >> 4) - m2;
            q += 32;
            is += 2;
        }
    }
}

void ms_dequantize_row_q6_K(const void* vx, float* y, int64_t k) {
    const block_q6_K* x = (const block_q6_K*)vx;
    const int64_t nb = k / QK_K;
    for (int64_t i = 0; i < nb; i++) {
        const float d = ms_fp16_to_fp32(x[i].d);
        const uint8_t* ql = x[i].ql;
        const uint8_t* qh = x[i].qh;
        const int8_t* sc = x[i].scales;
        for (int n = 0; n < QK_K; n += 128) {
            for (int l = 0; l < 32; ++l) {
                const int is = l / 16;
                const int8_t q1 = (int8_t)((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                const int8_t q2 = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                const int8_t q3 = (int8_t)((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                const int8_t q4 = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                y[l + 0] = d * sc[is + 0] * q1;
                y[l + 32] = d * sc[is + 2] * q2;
                y[l + 64] = d * sc[is + 4] * q3;
                y[l + 96] = d * sc[is + 6] * q4;
            }
            y += 128;
            ql += 64;
            qh += 32;
            sc += 8;
        }
    }
}
