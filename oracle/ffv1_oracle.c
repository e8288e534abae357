/*
 * ffv1_oracle.c -- CPU restatement of the reference FFV1 encoder + decoder.
 *
 * TEST INFRASTRUCTURE ONLY (see ffv1_oracle.h).  Written from the behaviour
 * of the reference (FFmpeg libavcodec 57.51.100); every block cites the
 * reference file:line whose semantics it restates.  Nothing here is linked
 * into, or called by, the MI355X product path.
 *
 * Parity pins: tests/golden/known_answers.json (SURVEY.md 8c MD5s of the
 * reference encoder's packets) and the FATE goldens tests/ref/vsynth/.
 */
#include "ffv1_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define AVERR_INVALIDDATA (-1094995529)
#define AVERR_EINVAL (-22)
#define AVERR_ENOSYS (-38)
#define AVERR_ENOMEM (-12)

/* ------------------------------------------------------------------------ */
/* small helpers                                                            */

static int ilog2u(unsigned v) /* av_log2 (libavutil/intmath.h:55-83) */
{
    int n = 0;
    while (v >> 1) { v >>= 1; n++; }
    return n;
}

static int median3(int a, int b, int c) /* mid_pred (mathops.h:95-120) */
{
    int lo = a < b ? a : b, hi = a < b ? b : a;
    return c < lo ? lo : (c > hi ? hi : c);
}

static int ceil_rshift(int a, int s) { return -((-a) >> s); }

/* fold() ffv1.h:148-159: wrap a residual into the signed range of `bits`. */
static int fold_residual(int d, int bits)
{
    if (bits == 8)
        return (int8_t)d;
    {
        unsigned half = 1u << (bits - 1);
        unsigned m = ((unsigned)d + half) & ((half << 1) - 1);
        return (int)m - (int)half;
    }
}

/* ------------------------------------------------------------------------ */
/* CRC-32/MPEG-2 style: MSB first, poly 0x04C11DB7, init 0, no xorout.      */
/* The reference keeps its table byte-swapped and stores the result with   */
/* AV_WL32 (crc.c:310-380, ffv1enc.c:1349-1350); net effect on the wire is  */
/* the plain MSB-first CRC written big-endian.                             */

static uint32_t crc_tab[256];
static int crc_ready;

static void crc_init(void)
{
    for (unsigned i = 0; i < 256; i++) {
        uint32_t r = i << 24;
        for (int k = 0; k < 8; k++)
            r = (r & 0x80000000u) ? (r << 1) ^ 0x04C11DB7u : (r << 1);
        crc_tab[i] = r;
    }
    crc_ready = 1;
}

uint32_t ffv1o_crc32(uint32_t crc, const uint8_t *buf, int64_t len)
{
    if (!crc_ready)
        crc_init();
    for (int64_t i = 0; i < len; i++)
        crc = (crc << 8) ^ crc_tab[(crc >> 24) ^ buf[i]];
    return crc;
}

static void put_be32(uint8_t *p, uint32_t v)
{
    p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = v;
}

/* ------------------------------------------------------------------------ */
/* Adaptive binary range coder (rangecoder.h:35-102, rangecoder.c:42-116)   */

typedef struct rc_tables {
    uint8_t to0[256];  /* state after coding a 0 ("zero_state") */
    uint8_t to1[256];  /* state after coding a 1 ("one_state")  */
} rc_tables;

typedef struct rc_enc {
    int low, range;
    int carry_run;      /* outstanding_count */
    int pending;        /* outstanding_byte, -1 = none yet */
    uint8_t *base, *ptr, *end;
    int overflow;
    const rc_tables *t;
} rc_enc;

/* ff_build_rac_states(c, 0.05*2^32, 256-8) (rangecoder.c:63-101). */
static void rc_default_tables(rc_tables *t)
{
    const int64_t ONE = (int64_t)1 << 32;
    const int factor = (int)(0.05 * (double)((int64_t)1 << 32));
    const int max_p = 256 - 8;
    int64_t p = ONE / 2;
    int prev = 0;

    memset(t, 0, sizeof(*t));
    for (int i = 0; i < 128; i++) {
        int p8 = (int)((256 * p + ONE / 2) >> 32);
        if (p8 <= prev)
            p8 = prev + 1;
        if (prev && prev < 256 && p8 <= max_p)
            t->to1[prev] = p8;
        p += ((ONE - p) * factor + ONE / 2) >> 32;
        prev = p8;
    }
    for (int i = 256 - max_p; i <= max_p; i++) {
        if (t->to1[i])
            continue;
        p = ((int64_t)i * ONE + 128) >> 8;
        p += ((ONE - p) * factor + ONE / 2) >> 32;
        int p8 = (int)((256 * p + ONE / 2) >> 32);
        if (p8 <= i)
            p8 = i + 1;
        if (p8 > max_p)
            p8 = max_p;
        t->to1[i] = p8;
    }
    for (int i = 1; i < 255; i++)
        t->to0[i] = 256 - t->to1[256 - i];
}

/* Custom transition install (ffv1.c:95-101, ffv1enc.c:1309-1315). */
static void rc_custom_tables(rc_tables *t, const rc_tables *dflt,
                             const uint8_t stt[256])
{
    *t = *dflt;
    for (int i = 1; i < 256; i++) {
        t->to1[i] = stt[i];
        t->to0[256 - i] = 256 - stt[i];
    }
}

static void rc_enc_init(rc_enc *c, uint8_t *buf, int64_t size,
                        const rc_tables *t)
{
    c->low = 0;
    c->range = 0xFF00;
    c->carry_run = 0;
    c->pending = -1;
    c->base = c->ptr = buf;
    c->end = buf + size;
    c->overflow = 0;
    c->t = t;
}

static void rc_emit(rc_enc *c, int byte)
{
    if (c->ptr < c->end)
        *c->ptr = (uint8_t)byte;
    else
        c->overflow = 1;
    c->ptr++;
}

/* renorm_encoder (rangecoder.h:52-75): shift out whole bytes while the
 * interval is narrower than 2^8; a byte can still be bumped by a carry, so
 * it is held back ("pending") together with a run of 0xFF bytes. */
static void rc_renorm(rc_enc *c)
{
    while (c->range < 0x100) {
        if (c->pending < 0) {
            c->pending = c->low >> 8;
        } else if (c->low <= 0xFF00) {
            rc_emit(c, c->pending);
            for (; c->carry_run; c->carry_run--)
                rc_emit(c, 0xFF);
            c->pending = c->low >> 8;
        } else if (c->low >= 0x10000) {
            rc_emit(c, c->pending + 1);
            for (; c->carry_run; c->carry_run--)
                rc_emit(c, 0x00);
            c->pending = (c->low >> 8) & 0xFF;
        } else {
            c->carry_run++;
        }
        c->low = (c->low & 0xFF) << 8;
        c->range <<= 8;
    }
}

/* put_rac (rangecoder.h:85-102) */
static void rc_put(rc_enc *c, uint8_t *st, int bit)
{
    int r1 = (c->range * *st) >> 8;
    if (bit) {
        c->low += c->range - r1;
        c->range = r1;
        *st = c->t->to1[*st];
    } else {
        c->range -= r1;
        *st = c->t->to0[*st];
    }
    rc_renorm(c);
}

/* ff_rac_terminate (rangecoder.c:104-116) */
static int64_t rc_finish(rc_enc *c)
{
    c->range = 0xFF;
    c->low += 0xFF;
    rc_renorm(c);
    c->range = 0xFF;
    rc_renorm(c);
    return c->ptr - c->base;
}

/* put_symbol_inline (ffv1enc.c:185-231): zero flag, unary exponent,
 * mantissa MSB->LSB, then sign, each in its own adaptive slot. */
static void rc_put_symbol(rc_enc *c, uint8_t st[32], int v, int is_signed)
{
    if (v == 0) {
        rc_put(c, &st[0], 1);
        return;
    }
    unsigned a = v < 0 ? -(unsigned)v : (unsigned)v;
    int e = ilog2u(a);
    rc_put(c, &st[0], 0);
    for (int i = 0; i < e; i++)
        rc_put(c, &st[1 + (i < 9 ? i : 9)], 1);
    rc_put(c, &st[1 + (e < 9 ? e : 9)], 0);
    for (int i = e - 1; i >= 0; i--)
        rc_put(c, &st[22 + (i < 9 ? i : 9)], (a >> i) & 1);
    if (is_signed)
        rc_put(c, &st[11 + (e < 10 ? e : 10)], v < 0);
}

/* ---- decoder side (rangecoder.h:104-147, ffv1dec.c:42-66) ---- */

typedef struct rc_dec {
    int low, range;
    const uint8_t *base, *ptr, *end;
    const rc_tables *t;
} rc_dec;

static void rc_dec_init(rc_dec *c, const uint8_t *buf, int64_t size,
                        const rc_tables *t)
{
    c->base = buf;
    c->end = buf + size;
    c->range = 0xFF00;
    c->low = (buf[0] << 8) | buf[1];
    c->ptr = buf + 2;
    c->t = t;
}

static int rc_get(rc_dec *c, uint8_t *st)
{
    int r1 = (c->range * *st) >> 8;
    int bit;
    c->range -= r1;
    if (c->low < c->range) {
        *st = c->t->to0[*st];
        bit = 0;
    } else {
        c->low -= c->range;
        c->range = r1;
        *st = c->t->to1[*st];
        bit = 1;
    }
    if (c->range < 0x100) {
        c->range <<= 8;
        c->low <<= 8;
        if (c->ptr < c->end)
            c->low += *c->ptr;
        c->ptr++;
    }
    return bit;
}

static int rc_get_symbol(rc_dec *c, uint8_t st[32], int is_signed)
{
    if (rc_get(c, &st[0]))
        return 0;
    int e = 0;
    while (rc_get(c, &st[1 + (e < 9 ? e : 9)])) {
        if (++e > 31)
            return FFV1O_AVERROR_INVALIDDATA; /* ffv1dec.c:53-54: the caller uses it as a value */
    }
    unsigned a = 1; /* wraps like the reference's int at e = 31 */
    for (int i = e - 1; i >= 0; i--)
        a = 2 * a + (unsigned)rc_get(c, &st[22 + (i < 9 ? i : 9)]);
    if (is_signed && rc_get(c, &st[11 + (e < 10 ? e : 10)]))
        return (int)(0u - a);
    return (int)a;
}

/* ------------------------------------------------------------------------ */
/* Golomb-Rice side (golomb.h:508-563, put_bits.h:35-190, ffv1.h:192-224)   */

typedef struct bitw {
    uint8_t *base, *end;
    int64_t nbits;
    int overflow;
} bitw;

static void bw_init(bitw *b, uint8_t *buf, int64_t size)
{
    b->base = buf;
    b->end = buf + (size > 0 ? size : 0);
    b->nbits = 0;
    b->overflow = 0;
}

/* MSB-first bit append; equivalent on the wire to put_bits + flush. */
static void bw_put(bitw *b, int n, uint32_t v)
{
    for (int i = n - 1; i >= 0; i--) {
        int64_t byte = b->nbits >> 3;
        int sh = 7 - (int)(b->nbits & 7);
        if (b->base + byte >= b->end) {
            b->overflow = 1;
        } else {
            if (sh == 7)
                b->base[byte] = 0;
            b->base[byte] |= ((v >> i) & 1) << sh;
        }
        b->nbits++;
    }
}

static int64_t bw_bytes(const bitw *b) { return (b->nbits + 7) >> 3; }

typedef struct bitr {
    const uint8_t *base;
    int64_t pos, nbits;
} bitr;

static int br_get(bitr *b, int n)
{
    int v = 0;
    for (int i = 0; i < n; i++) {
        int bit = 0;
        if (b->pos < b->nbits)
            bit = (b->base[b->pos >> 3] >> (7 - (b->pos & 7))) & 1;
        b->pos++;
        v = (v << 1) | bit;
    }
    return v;
}

typedef struct vlc_ctx {
    int drift, error_sum, bias, count;
} vlc_ctx;

static void vlc_reset(vlc_ctx *s)
{
    s->drift = 0;
    s->error_sum = 4;
    s->bias = 0;
    s->count = 1;
}

/* update_vlc_state (ffv1.h:192-224) */
static void vlc_adapt(vlc_ctx *s, int v)
{
    int drift = s->drift, count = s->count;
    s->error_sum = (uint16_t)(s->error_sum + (v < 0 ? -v : v));
    drift += v;
    if (count == 128) {
        count >>= 1;
        drift >>= 1;
        s->error_sum >>= 1;
    }
    count++;
    if (drift <= -count) {
        if (s->bias > -128)
            s->bias--;
        drift += count;
        if (drift <= -count)
            drift = -count + 1;
    } else if (drift > 0) {
        if (s->bias < 127)
            s->bias++;
        drift -= count;
        if (drift > 0)
            drift = 0;
    }
    s->drift = (int16_t)drift;
    s->count = count;
}

static int vlc_k(const vlc_ctx *s)
{
    int k = 0, i = s->count;
    while (i < s->error_sum) {
        k++;
        i += i;
    }
    return k;
}

/* put_vlc_symbol (ffv1enc.c:240-269) + set_sr_golomb/set_ur_golomb. */
static void vlc_put(bitw *b, vlc_ctx *s, int v, int bits)
{
    v = fold_residual(v - s->bias, bits);
    int k = vlc_k(s);
    int code = v ^ ((2 * s->drift + s->count) >> 31);
    unsigned u = code >= 0 ? 2u * (unsigned)code : (unsigned)(-2 * code - 1);
    unsigned q = u >> k;
    if (q < 12) {
        bw_put(b, (int)q + k + 1, (1u << k) + (u & ((1u << k) - 1)));
    } else {
        bw_put(b, 12 + bits, u - 12 + 1);
    }
    vlc_adapt(s, v);
}

static int vlc_get(bitr *b, vlc_ctx *s, int bits)
{
    int k = vlc_k(s);
    /* get_sr_golomb(gb, k, 12, bits) */
    int q = 0;
    while (q < 12 && br_get(b, 1) == 0)
        q++;
    unsigned u;
    if (q < 12) {
        u = ((unsigned)q << k) | (unsigned)br_get(b, k);
    } else {
        u = (unsigned)br_get(b, bits) + 11;
    }
    int v = (u & 1) ? -(int)((u + 1) >> 1) : (int)(u >> 1);
    v ^= ((2 * s->drift + s->count) >> 31);
    int ret = fold_residual(v + s->bias, bits);
    vlc_adapt(s, v);
    return ret;
}

static const uint8_t log2_run[41] = { /* ff_log2_run, bitstream.c:40-46 */
    0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3,
    4, 4, 5, 5, 6, 6, 7, 7, 8, 9, 10, 11, 12, 13, 14, 15,
    16, 17, 18, 19, 20, 21, 22, 23, 24,
};

/* ------------------------------------------------------------------------ */
/* Quantisation tables (ffv1enc.c:44-118, setup 846-879).                   */
/* Each table is given by the first index of every step on [0,127]; the     */
/* negative half mirrors it and index 128 copies -q[127] (the same rule     */
/* read_quant_table applies, ffv1dec.c:475-498).                           */

static void build_quant(int16_t q[256], const int *steps, int nsteps, int scale)
{
    int v = 0;
    for (int i = 0; i < 128; i++) {
        while (v < nsteps && i >= steps[v])
            v++;
        q[i] = (int16_t)(scale * v);
    }
    for (int i = 1; i < 128; i++)
        q[256 - i] = -q[i];
    q[128] = -q[127];
}

static const int Q11_STEPS[] = {1, 2, 5, 12, 35};        /* quant11      */
static const int Q5_STEPS[] = {1, 4};                    /* quant5       */
static const int Q9_10_STEPS[] = {5, 13, 27, 56};        /* quant9_10bit */
static const int Q5_10_STEPS[] = {11, 50};               /* quant5_10bit */

/* quant_tables[context_model] for the given depth */
static void build_quant_set(int16_t qt[5][256], int model, int bits)
{
    const int *qa, *qb;
    int na, nb;
    if (bits <= 8) {
        qa = Q11_STEPS; na = 5; qb = Q5_STEPS; nb = 2;
    } else {
        qa = Q9_10_STEPS; na = 4; qb = Q5_10_STEPS; nb = 2;
    }
    memset(qt, 0, 5 * 256 * sizeof(int16_t));
    build_quant(qt[0], qa, na, 1);
    build_quant(qt[1], qa, na, 11);
    if (model == 0) {
        build_quant(qt[2], qa, na, 121);
    } else {
        build_quant(qt[2], qb, nb, 121);
        build_quant(qt[3], qb, nb, 605);
        build_quant(qt[4], qb, nb, 3025);
    }
}

static int context_count_of(int model)
{
    return model ? (11 * 11 * 5 * 5 * 5 + 1) / 2 : (11 * 11 * 11 + 1) / 2;
}

/* ver2_state (ffv1enc.c:120-137): the custom state-transition table the
 * encoder installs for coder=1 ("range_tab"); format data of FFV1 v2+. */
static const uint8_t CUSTOM_STT[256] = {
    0, 10, 10, 10, 10, 16, 16, 16, 28, 16, 16, 29, 42, 49, 20, 49,
    59, 25, 26, 26, 27, 31, 33, 33, 33, 34, 34, 37, 67, 38, 39, 39,
    40, 40, 41, 79, 43, 44, 45, 45, 48, 48, 64, 50, 51, 52, 88, 52,
    53, 74, 55, 57, 58, 58, 74, 60, 101, 61, 62, 84, 66, 66, 68, 69,
    87, 82, 71, 97, 73, 73, 82, 75, 111, 77, 94, 78, 87, 81, 83, 97,
    85, 83, 94, 86, 99, 89, 90, 99, 111, 92, 93, 134, 95, 98, 105, 98,
    105, 110, 102, 108, 102, 118, 103, 106, 106, 113, 109, 112, 114, 112, 116, 125,
    115, 116, 117, 117, 126, 119, 125, 121, 121, 123, 145, 124, 126, 131, 127, 129,
    165, 130, 132, 138, 133, 135, 145, 136, 137, 139, 146, 141, 143, 142, 144, 148,
    147, 155, 151, 149, 151, 150, 152, 157, 153, 154, 156, 168, 158, 162, 161, 160,
    172, 163, 169, 164, 166, 184, 167, 170, 177, 174, 171, 173, 182, 176, 180, 178,
    175, 189, 179, 181, 186, 183, 192, 185, 200, 187, 191, 188, 190, 197, 193, 196,
    197, 194, 195, 196, 198, 202, 199, 201, 210, 203, 207, 204, 205, 206, 208, 214,
    209, 211, 221, 212, 213, 215, 224, 216, 217, 218, 219, 220, 222, 228, 223, 225,
    226, 224, 227, 229, 240, 230, 231, 232, 233, 234, 235, 236, 238, 239, 237, 242,
    241, 243, 242, 244, 245, 246, 247, 248, 249, 250, 251, 252, 252, 253, 254, 255,
};

/* ------------------------------------------------------------------------ */
/* encode_init parameter contract (ffv1enc.c:669-1029)                      */

typedef struct pixfmt_info {
    const char *name;
    int planes;        /* components: 1 gray, 2 gray + alpha (YA8), 3 yuv /
                          rgb, 4 yuva / rgb32 (desc->nb_components) */
    int hs, vs;
    int depth;         /* nominal depth of the storage format */
    int family;        /* 9, 10, 16 or 8: which switch group it enters;
                          32 packed RGB32 (ffv1enc.c:780-792), 100 + bits
                          planar GBR (:793-814) */
} pixfmt_info;

static const pixfmt_info PIXFMTS[] = {
    {"yuv420p", 3, 1, 1, 8, 8},   {"yuv422p", 3, 1, 0, 8, 8},
    {"yuv444p", 3, 0, 0, 8, 8},   {"yuv440p", 3, 0, 1, 8, 8},
    {"yuv411p", 3, 2, 0, 8, 8},   {"yuv410p", 3, 2, 2, 8, 8},
    {"gray", 1, 0, 0, 8, 8},
    {"yuv420p9", 3, 1, 1, 9, 9},  {"yuv422p9", 3, 1, 0, 9, 9},
    {"yuv444p9", 3, 0, 0, 9, 9},
    {"yuv420p10", 3, 1, 1, 10, 10}, {"yuv422p10", 3, 1, 0, 10, 10},
    {"yuv444p10", 3, 0, 0, 10, 10},
    {"yuv420p16", 3, 1, 1, 16, 16}, {"yuv422p16", 3, 1, 0, 16, 16},
    {"yuv444p16", 3, 0, 0, 16, 16}, {"gray16", 1, 0, 0, 16, 16},
    {"bgr0", 3, 0, 0, 8, 32},       {"0rgb32", 3, 0, 0, 8, 32},
    {"gbrp9", 3, 0, 0, 9, 109},     {"gbrp10", 3, 0, 0, 10, 110},
    {"gbrp12", 3, 0, 0, 12, 112},   {"gbrp14", 3, 0, 0, 14, 114},
    /* with alpha (ffv1enc.c:725-774, 780-786) */
    {"yuva420p", 4, 1, 1, 8, 8},    {"yuva422p", 4, 1, 0, 8, 8},
    {"yuva444p", 4, 0, 0, 8, 8},    {"ya8", 2, 0, 0, 8, 8},
    {"yuva420p9", 4, 1, 1, 9, 9},   {"yuva422p9", 4, 1, 0, 9, 9},
    {"yuva444p9", 4, 0, 0, 9, 9},
    {"yuva420p10", 4, 1, 1, 10, 10}, {"yuva422p10", 4, 1, 0, 10, 10},
    {"yuva444p10", 4, 0, 0, 10, 10},
    {"yuva420p16", 4, 1, 1, 16, 16}, {"yuva422p16", 4, 1, 0, 16, 16},
    {"yuva444p16", 4, 0, 0, 16, 16},
    {"bgra", 4, 0, 0, 8, 32},       {"rgb32", 4, 0, 0, 8, 32},
};

int ffv1o_configure(ffv1o_config *cfg, int width, int height,
                    const char *pix_fmt, int slices, int level, int coder,
                    int context, int gop_size, int bits_per_raw_sample,
                    int slicecrc)
{
    return ffv1o_configure2(cfg, width, height, pix_fmt, slices, level, coder, context, gop_size,
                            bits_per_raw_sample, slicecrc, 0);
}

int ffv1o_configure2(ffv1o_config *cfg, int width, int height,
                     const char *pix_fmt, int slices, int level, int coder,
                     int context, int gop_size, int bits_per_raw_sample,
                     int slicecrc, int pass)
{
    return ffv1o_configure3(cfg, width, height, pix_fmt, slices, level, coder, context, gop_size,
                            bits_per_raw_sample, slicecrc, pass, 0);
}

int ffv1o_configure3(ffv1o_config *cfg, int width, int height,
                     const char *pix_fmt, int slices, int level, int coder,
                     int context, int gop_size, int bits_per_raw_sample,
                     int slicecrc, int pass, int experimental)
{
    const pixfmt_info *pf = NULL;
    for (size_t i = 0; i < sizeof(PIXFMTS) / sizeof(PIXFMTS[0]); i++)
        if (!strcmp(PIXFMTS[i].name, pix_fmt))
            pf = &PIXFMTS[i];
    if (!pf || width <= 0 || height <= 0)
        return pf ? AVERR_INVALIDDATA : AVERR_ENOSYS;

    memset(cfg, 0, sizeof(*cfg));
    cfg->width = width;
    cfg->height = height;
    cfg->gop_size = gop_size;
    cfg->sar_num = 0;
    cfg->sar_den = 1;

    /* version selection, ffv1enc.c:678-697 */
    int version = 0;
    if (pass || slices > 1) /* AV_CODEC_FLAG_PASS1 | PASS2 (:680-682) */
        version = 2;
    if (slices == 0 && level < 0 && width * height > 720 * 576)
        version = 2;
    if (level <= 0 && version == 2)
        version = 3;
    if (level >= 0 && level <= 4) {
        if (level < version)
            return AVERR_EINVAL;
        version = level;
    }
    int ec = slicecrc;
    if (ec < 0)
        ec = version >= 3;
    /* versions 2 and 4 need -strict experimental (:703-706).  Version 2's
     * extradata has no ec field (write_extradata, ffv1enc.c:593-598), so
     * its packets with slice CRCs are unreadable by the reference decoder:
     * refused here */
    if ((version == 2 || version > 3) && !experimental)
        return AVERR_INVALIDDATA;
    if (version == 2 && ec)
        return AVERR_ENOSYS;

    /* coder, ffv1enc.c:708-718 (coder -1 keeps the private default 0) */
    int ac = 0;
    if (coder != -1)
        ac = coder > 0 ? 2 : 0;
    if (ac == 1)
        ac = 2;
    else if (ac == -2)
        ac = 1;
    if (coder == -2)
        ac = 1;

    /* pix_fmt switch, ffv1enc.c:720-820 */
    int bits = 0, packed = 0;
    if (pf->family == 32) { /* AV_PIX_FMT_0RGB32 (= bgr0 in memory), :787-792 */
        bits = bits_per_raw_sample ? bits_per_raw_sample : 8;
        if (bits != 8)
            return AVERR_ENOSYS;
    } else if (pf->family > 100) { /* GBRP9..14, :793-814 */
        bits = bits_per_raw_sample ? bits_per_raw_sample : pf->family - 100;
        packed = 1;
        if (version < 1)
            version = 1;
        if (ac == 0)
            ac = 2;
    }
    if (pf->family == 9 && !bits_per_raw_sample)
        bits = 9;
    if (pf->family == 32 || pf->family > 100)
        ; /* RGB: set above */
    else if (pf->family == 9 || pf->family == 10) {
        packed = 1;
        if (!bits_per_raw_sample && !bits)
            bits = 10;
    }
    if (pf->family >= 9 && pf->family <= 16) {
        if (!bits_per_raw_sample && !bits)
            bits = 16;
        else if (!bits)
            bits = bits_per_raw_sample;
        if (bits <= 8)
            return AVERR_INVALIDDATA;
        if (ac == 0)
            ac = 2;
        if (version < 1)
            version = 1;
    }
    if (!bits)
        bits = 8;
    if (context < 0 || context > 1)
        return AVERR_EINVAL;

    /* chroma_planes = nb_components >= 3, transparency = 4 or 2 components
     * (ffv1enc.c:772-774); RGB32 has alpha, 0RGB32 not (:780-792) */
    cfg->chroma_planes = pf->planes >= 3;
    cfg->chroma_h_shift = pf->planes >= 3 ? pf->hs : 0;
    cfg->chroma_v_shift = pf->planes >= 3 ? pf->vs : 0;
    cfg->transparency = pf->planes == 4 || pf->planes == 2;
    cfg->bits_per_raw_sample = bits;
    cfg->packed_at_lsb = packed;
    cfg->sample_bytes = pf->family == 32 ? 4 : pf->depth > 8 ? 2 : 1;
    cfg->colorspace = pf->family == 32 || pf->family > 100;
    cfg->version = version;
    cfg->ac = ac;
    cfg->ec = ec;
    cfg->context_model = context;
    cfg->num_h_slices = 1;
    cfg->num_v_slices = 1;
    /* v4 runs choose_rct_params on every slice (ffv1enc.c:1163-1164), which
     * reads plane 0 as 32-bit B, G, R words at 8 bit and planes 0-2 as u16
     * at the LUMA position otherwise: inside the frame only for the RGB
     * formats and 4:4:4 YCbCr above 8 bits (gray has no planes 1, 2;
     * subsampled chroma and 8-bit YCbCr are read past their end) */
    if (version > 3 && !cfg->colorspace &&
        !(cfg->chroma_planes && !cfg->chroma_h_shift && !cfg->chroma_v_shift && cfg->sample_bytes == 2))
        return AVERR_ENOSYS;
    if (version > 1) {
        int nv = (width > 352 || height > 288 || !slices) ? 2 : 1;
        for (; nv < 9; nv++)
            for (int nh = nv; nh < 2 * nv; nh++)
                if ((slices == nh * nv && slices <= 64) || !slices) {
                    cfg->num_h_slices = nh;
                    cfg->num_v_slices = nv;
                    return 0;
                }
        return AVERR_ENOSYS;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Encoder state                                                            */

typedef struct plane_state {
    uint8_t *rac;       /* [contexts][32]   */
    vlc_ctx *vlc;       /* [contexts]       */
} plane_state;

typedef struct slice_ctx {
    int x0, y0, w, h;   /* luma rectangle, ffv1.c:117-145 */
    plane_state ps[3];  /* plane_count: 2, 3 with alpha (ffv1enc.c:720, 890-891) */
    uint8_t *buf;
    int64_t cap;
    int64_t bytes;
    int error;
    int pcm;            /* the last frame coded this slice as PCM (v4) */
} slice_ctx;

struct ffv1o_enc {
    ffv1o_config cfg;
    int16_t qt[5][256];
    int contexts;
    int coded_bits;     /* "bits" argument of encode_line */
    rc_tables dflt, frame_tab;
    uint8_t stt[256];
    int nslices;
    slice_ctx *sl;
    int64_t picture_number;
    int plane_count;    /* 2 + transparency (ffv1enc.c:720, 890-891) */
    /* the slice being coded: encode_line's buffer check failed (ffv1enc.c:
     * 283-292), slice_coding_mode (1 = PCM, :294-304, 1207-1217) and the
     * RCT coefficients (v4: choose_rct_params, :1064-1144; else 1, 1) */
    int line_err, pcm, rct_by, rct_ry;
    int16_t *scratch;   /* one slice plane of samples */
    /* 2-pass (ffv1enc.c:898-986, 1236-1277) */
    int pass1;
    uint64_t rc_stat[256][2];    /* per state value, decisions 0 / 1 */
    uint64_t (*rc_stat2)[32][2]; /* per context and slot, of the quant set in use */
    int gob_count;
    uint8_t *init_states[2];     /* [context][32] per quant set, NULL = all 128 */
};

static void slice_rects(const ffv1o_config *cfg, int i, int *x0, int *y0,
                        int *w, int *h)
{
    int nh = cfg->num_h_slices, nv = cfg->num_v_slices;
    int sx = i % nh, sy = i / nh;
    int xs = (int)((int64_t)cfg->width * sx / nh);
    int xe = (int)((int64_t)cfg->width * (sx + 1) / nh);
    int ys = (int)((int64_t)cfg->height * sy / nv);
    int ye = (int)((int64_t)cfg->height * (sy + 1) / nv);
    *x0 = xs; *y0 = ys; *w = xe - xs; *h = ye - ys;
}

ffv1o_enc *ffv1o_enc_new(const ffv1o_config *cfg)
{
    if (cfg->num_h_slices * cfg->num_v_slices > 256)
        return NULL;
    ffv1o_enc *e = calloc(1, sizeof(*e));
    if (!e)
        return NULL;
    e->cfg = *cfg;
    e->plane_count = 2 + (cfg->transparency != 0);
    build_quant_set(e->qt, cfg->context_model, cfg->bits_per_raw_sample);
    e->contexts = context_count_of(cfg->context_model);
    /* encode_line's bits: RGB samples after the RCT carry one bit more
     * (encode_rgb_frame, ffv1enc.c:460-466: 9 for 8-bit) */
    if (cfg->colorspace)
        e->coded_bits = cfg->bits_per_raw_sample <= 8 ? 9 : cfg->bits_per_raw_sample + 1;
    else
        e->coded_bits = cfg->bits_per_raw_sample <= 8 ? 8 : cfg->bits_per_raw_sample;
    rc_default_tables(&e->dflt);
    if (cfg->ac == 2) {
        memcpy(e->stt, CUSTOM_STT, 256);
        rc_custom_tables(&e->frame_tab, &e->dflt, e->stt);
    } else {
        memcpy(e->stt, e->dflt.to1, 256);
        e->frame_tab = e->dflt;
    }
    e->nslices = cfg->num_h_slices * cfg->num_v_slices;
    e->sl = calloc(e->nslices, sizeof(slice_ctx));
    int64_t maxw = 0;
    for (int i = 0; i < e->nslices; i++) {
        slice_ctx *s = &e->sl[i];
        slice_rects(cfg, i, &s->x0, &s->y0, &s->w, &s->h);
        if ((int64_t)s->w * s->h > maxw)
            maxw = (int64_t)s->w * s->h;
        /* the reference's slice buffers in a packet of AV_INPUT_BUFFER_MIN_SIZE
         * + w*h*140 bytes (v4: w*h*12), ffv1enc.c:1232-1233, 1281-1282: slice
         * 0 codes on with the packet's coder (the whole packet), slice i in
         * pkt->size / slice_count bytes (:1317-1322); malloc'd pages are only
         * touched as far as used */
        const int64_t pkt = 16384 + (int64_t)cfg->width * cfg->height * (cfg->version > 3 ? 12 : 140);
        s->cap = i == 0 ? pkt : pkt / e->nslices;
        /* test hook: a smaller v4 buffer for slice 0 alone, so that it fails
         * the 35 * w check too (the HIP encoder's FFV1HIP_DEBUG=v4_cap0) */
        const char *hook = getenv("FFV1_ORACLE_V4_CAP0");
        if (hook && cfg->version > 3 && i == 0)
            s->cap = atoll(hook);
        s->buf = malloc(s->cap);
        for (int p = 0; p < e->plane_count; p++) {
            s->ps[p].rac = malloc((size_t)e->contexts * 32);
            s->ps[p].vlc = malloc((size_t)e->contexts * sizeof(vlc_ctx));
        }
    }
    e->scratch = malloc(4 * (size_t)maxw * sizeof(int16_t) + 16);
    return e;
}

/* find_best_state (ffv1enc.c:139-183): for a probability i/256 of a one and
 * k decisions seen, the starting state whose adaptation through one_state
 * codes the first k decisions in the fewest bits. */
static void find_best_state(uint8_t best[256][256], const uint8_t one_state[256])
{
    double l2[256];
    for (int i = 1; i < 256; i++)
        l2[i] = log2(i / 256.0);
    for (int i = 0; i < 256; i++) {
        double best_len[256];
        double p = i / 256.0;
        for (int j = 0; j < 256; j++)
            best_len[j] = 1 << 30;
        for (int j = i - 10 > 1 ? i - 10 : 1; j < (i + 11 < 256 ? i + 11 : 256); j++) {
            double occ[256] = {0};
            double len = 0;
            occ[j] = 1.0;
            if (!one_state[j])
                continue;
            for (int k = 0; k < 256; k++) {
                double nocc[256] = {0};
                for (int m = 1; m < 256; m++)
                    if (occ[m])
                        len -= occ[m] * (p * l2[m] + (1 - p) * l2[256 - m]);
                if (len < best_len[k]) {
                    best_len[k] = len;
                    best[i][k] = (uint8_t)j;
                }
                for (int m = 1; m < 256; m++)
                    if (occ[m]) {
                        nocc[one_state[m]] += occ[m] * p;
                        nocc[256 - one_state[256 - m]] += occ[m] * (1 - p);
                    }
                memcpy(occ, nocc, sizeof(occ));
            }
        }
    }
}

/* FFSWAP(int, a, b) on the 64-bit counters (ffv1enc.c:642-647):
 * { int tmp = b; b = a; a = tmp; } (libavutil/common.h:99), so b takes a
 * whole and a takes b truncated to 32 bits and sign-extended. */
static void swap_int(uint64_t *a, uint64_t *b)
{
    int t = (int)(uint32_t)*b;
    *b = *a;
    *a = (uint64_t)(int64_t)t;
}

/* sort_stt (ffv1enc.c:621-667): swap neighbouring states of the custom
 * transition table while that lowers the pass-1 cost. */
static void sort_stt(uint64_t rc_stat[256][2], uint8_t stt[256])
{
/* unparenthesised like the reference's macros: size0 / sizeX are one sum of
 * eight products evaluated left to right, and the 1e-14 test below sees the
 * rounding of that association */
#define COST(o, n) (double)rc_stat[o][0] * -log2((256 - (n)) / 256.0) + (double)rc_stat[o][1] * -log2((n) / 256.0)
#define COST2(o, n) COST(o, n) + COST(256 - (o), 256 - (n))
    int changed;
    do {
        changed = 0;
        for (int i = 12; i < 244; i++) {
            for (int i2 = i + 1; i2 < 245 && i2 < i + 4; i2++) {
                double size0 = COST2(i, i) + COST2(i2, i2);
                double sizeX = COST2(i, i2) + COST2(i2, i);
                if (size0 - sizeX > size0 * (1e-14) && i != 128 && i2 != 128) {
                    uint8_t t = stt[i];
                    stt[i] = stt[i2];
                    stt[i2] = t;
                    swap_int(&rc_stat[i][0], &rc_stat[i2][0]);
                    swap_int(&rc_stat[i][1], &rc_stat[i2][1]);
                    if (i != 256 - i2) {
                        t = stt[256 - i];
                        stt[256 - i] = stt[256 - i2];
                        stt[256 - i2] = t;
                        swap_int(&rc_stat[256 - i][0], &rc_stat[256 - i2][0]);
                        swap_int(&rc_stat[256 - i][1], &rc_stat[256 - i2][1]);
                    }
                    for (int j = 1; j < 256; j++) {
                        if (stt[j] == i)
                            stt[j] = (uint8_t)i2;
                        else if (stt[j] == i2)
                            stt[j] = (uint8_t)i;
                        if (i != 256 - i2) {
                            if (stt[256 - j] == 256 - i)
                                stt[256 - j] = (uint8_t)(256 - i2);
                            else if (stt[256 - j] == 256 - i2)
                                stt[256 - j] = (uint8_t)(256 - i);
                        }
                    }
                    changed = 1;
                }
            }
        }
    } while (changed);
#undef COST
#undef COST2
}

static int clip_int(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* Pass 2 (ffv1enc.c:906-986): parse stats_in (the last complete block
 * wins), sort the custom table, and derive every context's initial states
 * from the pass-1 decision counts. */
static int enc_pass2(ffv1o_enc *e, const char *stats)
{
    uint64_t rc_stat[256][2];
    uint64_t(*st2[2])[32][2];
    int counts[2] = {context_count_of(0), context_count_of(1)};
    int gob_count = 0, rc = 0;
    st2[0] = calloc((size_t)counts[0], sizeof(*st2[0]));
    st2[1] = calloc((size_t)counts[1], sizeof(*st2[1]));
    uint8_t(*best)[256] = malloc(256 * 256);
    const char *p = stats;
    char *next;
    for (;;) {
        for (int j = 0; j < 256; j++)
            for (int i = 0; i < 2; i++) {
                rc_stat[j][i] = (uint64_t)strtol(p, &next, 0);
                if (next == p) {
                    rc = AVERR_INVALIDDATA;
                    goto done;
                }
                p = next;
            }
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < counts[i]; j++)
                for (int k = 0; k < 32; k++)
                    for (int m = 0; m < 2; m++) {
                        st2[i][j][k][m] = (uint64_t)strtol(p, &next, 0);
                        if (next == p) {
                            rc = AVERR_INVALIDDATA;
                            goto done;
                        }
                        p = next;
                    }
        gob_count = (int)strtol(p, &next, 0);
        if (next == p || gob_count <= 0) {
            rc = AVERR_INVALIDDATA;
            goto done;
        }
        p = next;
        while (*p == '\n' || *p == ' ')
            p++;
        if (p[0] == 0)
            break;
    }
    if (e->cfg.ac == 2) {
        sort_stt(rc_stat, e->stt);
        rc_custom_tables(&e->frame_tab, &e->dflt, e->stt);
    }
    find_best_state(best, e->cfg.ac == 2 ? e->stt : e->dflt.to1);
    for (int i = 0; i < 2; i++) {
        uint8_t(*is)[32] = malloc((size_t)counts[i] * 32);
        for (int k = 0; k < 32; k++) {
            double a = 0, b = 0;
            int jp = 0;
            for (int j = 0; j < counts[i]; j++) {
                double pr = 128;
                if ((st2[i][j][k][0] + st2[i][j][k][1] > 200 && j) || a + b > 200) {
                    if (a + b)
                        pr = 256.0 * b / (a + b);
                    is[jp][k] = best[clip_int((int)round(pr), 1, 255)][clip_int((int)((a + b) / gob_count), 0, 255)];
                    for (jp++; jp < j; jp++)
                        is[jp][k] = is[jp - 1][k];
                    a = b = 0;
                }
                a += (double)st2[i][j][k][0];
                b += (double)st2[i][j][k][1];
                if (a + b)
                    pr = 256.0 * b / (a + b);
                is[j][k] = best[clip_int((int)round(pr), 1, 255)][clip_int((int)((a + b) / gob_count), 0, 255)];
            }
        }
        e->init_states[i] = (uint8_t *)is;
    }
done:
    free(best);
    free(st2[0]);
    free(st2[1]);
    return rc;
}

ffv1o_enc *ffv1o_enc_new2(const ffv1o_config *cfg, int pass, const char *stats_in)
{
    if (pass && cfg->version < 2)
        return NULL; /* av_assert0(s->version >= 2) */
    ffv1o_enc *e = ffv1o_enc_new(cfg);
    if (!e)
        return NULL;
    if (pass == 1) {
        e->pass1 = 1;
        e->rc_stat2 = calloc((size_t)e->contexts, sizeof(*e->rc_stat2));
    } else if (pass == 2 && stats_in) {
        if (enc_pass2(e, stats_in) < 0) {
            ffv1o_enc_free(e);
            return NULL;
        }
    }
    return e;
}

/* The pass-1 statistics as encode_frame writes them into stats_out at the
 * end of the stream (ffv1enc.c:1236-1277): 256 state pairs, a newline, the
 * (context, slot) pairs of both quant sets (the unused one all zero), the
 * keyframe count.  Returns the text length (without the NUL). */
int64_t ffv1o_enc_stats_out(const ffv1o_enc *e, char *buf, int64_t cap)
{
    if (!e->pass1)
        return AVERR_EINVAL;
    int64_t n = 0;
#define EMIT(...)                                                              \
    do {                                                                       \
        char tmp[64];                                                          \
        int l = snprintf(tmp, sizeof(tmp), __VA_ARGS__);                       \
        if (buf && n + l < cap)                                                \
            memcpy(buf + n, tmp, (size_t)l + 1);                               \
        n += l;                                                                \
    } while (0)
    for (int j = 0; j < 256; j++)
        EMIT("%llu %llu ", (unsigned long long)e->rc_stat[j][0], (unsigned long long)e->rc_stat[j][1]);
    EMIT("\n");
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < context_count_of(i); j++)
            for (int m = 0; m < 32; m++) {
                uint64_t a = 0, b = 0;
                if (i == e->cfg.context_model) {
                    a = e->rc_stat2[j][m][0];
                    b = e->rc_stat2[j][m][1];
                }
                EMIT("%llu %llu ", (unsigned long long)a, (unsigned long long)b);
            }
    EMIT("%d\n", e->gob_count);
#undef EMIT
    return n;
}

void ffv1o_enc_free(ffv1o_enc *e)
{
    if (!e)
        return;
    for (int i = 0; i < e->nslices; i++) {
        free(e->sl[i].buf);
        for (int p = 0; p < e->plane_count; p++) {
            free(e->sl[i].ps[p].rac);
            free(e->sl[i].ps[p].vlc);
        }
    }
    free(e->sl);
    free(e->scratch);
    free(e->rc_stat2);
    free(e->init_states[0]);
    free(e->init_states[1]);
    free(e);
}

/* write_quant_table(s) (ffv1enc.c:475-496): run lengths of each step. */
static void put_quant_tables(rc_enc *c, int16_t qt[5][256])
{
    for (int t = 0; t < 5; t++) {
        uint8_t st[32];
        memset(st, 128, 32);
        int last = 0, i;
        for (i = 1; i < 128; i++)
            if (qt[t][i] != qt[t][i - 1]) {
                rc_put_symbol(c, st, i - last - 1, 0);
                last = i;
            }
        rc_put_symbol(c, st, i - last - 1, 0);
    }
}

/* write_extradata (ffv1enc.c:545-619) */
int ffv1o_enc_extradata(ffv1o_enc *e, uint8_t *buf, int cap)
{
    const ffv1o_config *cfg = &e->cfg;
    if (cfg->version < 2)
        return 0;
    rc_enc c;
    uint8_t st[32];
    memset(st, 128, 32);
    rc_enc_init(&c, buf, cap - 4, &e->dflt);

    rc_put_symbol(&c, st, cfg->version, 0);
    if (cfg->version > 2)
        rc_put_symbol(&c, st, cfg->version == 3 ? 4 : 2, 0);
    rc_put_symbol(&c, st, cfg->ac, 0);
    if (cfg->ac == 2)
        for (int i = 1; i < 256; i++)
            rc_put_symbol(&c, st, e->stt[i] - e->dflt.to1[i], 1);
    rc_put_symbol(&c, st, cfg->colorspace, 0);
    rc_put_symbol(&c, st, cfg->bits_per_raw_sample, 0);
    rc_put(&c, &st[0], cfg->chroma_planes);
    rc_put_symbol(&c, st, cfg->chroma_h_shift, 0);
    rc_put_symbol(&c, st, cfg->chroma_v_shift, 0);
    rc_put(&c, &st[0], cfg->transparency);
    rc_put_symbol(&c, st, cfg->num_h_slices - 1, 0);
    rc_put_symbol(&c, st, cfg->num_v_slices - 1, 0);

    /* quant_table_count is always 2 (ffv1enc.c:847) */
    rc_put_symbol(&c, st, 2, 0);
    for (int set = 0; set < 2; set++) {
        int16_t qt[5][256];
        build_quant_set(qt, set, cfg->bits_per_raw_sample);
        put_quant_tables(&c, qt);
    }
    uint8_t st2[32][32];
    memset(st2, 128, sizeof(st2));
    for (int set = 0; set < 2; set++) { /* ffv1enc.c:591-607 */
        const uint8_t *is = e->init_states[set];
        int n = context_count_of(set) * 32, j = 0;
        while (is && j < n && is[j] == 128)
            j++;
        if (!is || j == n) {
            rc_put(&c, &st[0], 0);
            continue;
        }
        rc_put(&c, &st[0], 1);
        for (int i = 0; i < n; i++) {
            int pred = i >= 32 ? is[i - 32] : 128;
            rc_put_symbol(&c, st2[i & 31], (int8_t)(is[i] - pred), 1);
        }
    }
    if (cfg->version > 2) {
        rc_put_symbol(&c, st, cfg->ec, 0);
        rc_put_symbol(&c, st, cfg->gop_size < 2, 0);
    }
    int64_t n = rc_finish(&c);
    if (c.overflow)
        return AVERR_ENOMEM;
    put_be32(buf + n, ffv1o_crc32(0, buf, n));
    return (int)(n + 4);
}

/* write_header for v<2 keyframes (ffv1enc.c:498-522) */
static void put_v01_header(const ffv1o_enc *e, rc_enc *c)
{
    const ffv1o_config *cfg = &e->cfg;
    uint8_t st[32];
    memset(st, 128, 32);
    rc_put_symbol(c, st, cfg->version, 0);
    rc_put_symbol(c, st, cfg->ac, 0);
    if (cfg->ac == 2)
        for (int i = 1; i < 256; i++)
            rc_put_symbol(c, st, e->stt[i] - c->t->to1[i], 1);
    rc_put_symbol(c, st, cfg->colorspace, 0);
    if (cfg->version > 0)
        rc_put_symbol(c, st, cfg->bits_per_raw_sample, 0);
    rc_put(c, &st[0], cfg->chroma_planes);
    rc_put_symbol(c, st, cfg->chroma_h_shift, 0);
    rc_put_symbol(c, st, cfg->chroma_v_shift, 0);
    rc_put(c, &st[0], cfg->transparency);
    put_quant_tables(c, (int16_t(*)[256])e->qt);
}

/* write_header for v2 keyframes (ffv1enc.c:523-541): the slice layout
 * in-band, one state array for all of it; every plane's quant set index is
 * the context model (plane_count 2, 3 with alpha, ffv1enc.c:720, 890-891) */
static void put_v2_header(const ffv1o_enc *e, rc_enc *c)
{
    const ffv1o_config *cfg = &e->cfg;
    uint8_t st[32];
    memset(st, 128, 32);
    const int nh = cfg->num_h_slices, nv = cfg->num_v_slices, n = nh * nv;
    rc_put_symbol(c, st, n, 0);
    for (int i = 0; i < n; i++) {
        const slice_ctx *s = &e->sl[i];
        rc_put_symbol(c, st, (int)((int64_t)(s->x0 + 1) * nh / cfg->width), 0);
        rc_put_symbol(c, st, (int)((int64_t)(s->y0 + 1) * nv / cfg->height), 0);
        rc_put_symbol(c, st, (int)((int64_t)(s->w + 1) * nh / cfg->width) - 1, 0);
        rc_put_symbol(c, st, (int)((int64_t)(s->h + 1) * nv / cfg->height) - 1, 0);
        for (int j = 0; j < 2 + (cfg->transparency != 0); j++)
            rc_put_symbol(c, st, cfg->context_model, 0);
    }
}

/* encode_slice_header (ffv1enc.c:1031-1062) */
static void clear_slice_states(ffv1o_enc *e, slice_ctx *s);

static void put_slice_header(ffv1o_enc *e, slice_ctx *s, rc_enc *c)
{
    const ffv1o_config *cfg = &e->cfg;
    uint8_t st[32];
    memset(st, 128, 32);
    int nh = cfg->num_h_slices, nv = cfg->num_v_slices;
    rc_put_symbol(c, st, (int)((int64_t)(s->x0 + 1) * nh / cfg->width), 0);
    rc_put_symbol(c, st, (int)((int64_t)(s->y0 + 1) * nv / cfg->height), 0);
    rc_put_symbol(c, st, (int)((int64_t)(s->w + 1) * nh / cfg->width) - 1, 0);
    rc_put_symbol(c, st, (int)((int64_t)(s->h + 1) * nv / cfg->height) - 1, 0);
    for (int j = 0; j < e->plane_count; j++)
        rc_put_symbol(c, st, cfg->context_model, 0);
    rc_put_symbol(c, st, 3, 0); /* progressive picture structure */
    rc_put_symbol(c, st, cfg->sar_num, 0);
    rc_put_symbol(c, st, cfg->sar_den, 0);
    if (cfg->version > 3) { /* ffv1enc.c:1052-1061 */
        rc_put(c, &st[0], e->pcm);
        if (e->pcm)
            clear_slice_states(e, s);
        rc_put_symbol(c, st, e->pcm, 0);
        if (!e->pcm) {
            rc_put_symbol(c, st, e->rct_by, 0);
            rc_put_symbol(c, st, e->rct_ry, 0);
        }
    }
}

/* Load one slice plane into int16 storage, as encode_plane does
 * (ffv1enc.c:390-407): 8-bit, LSB-packed u16, or MSB-aligned u16 >> shift. */
static void load_plane(const ffv1o_config *cfg, const uint8_t *src,
                       int stride, int x0, int y0, int w, int h, int16_t *dst)
{
    /* YA8: Y and A bytes interleaved, encode_plane's pixel_stride 2
     * (ffv1enc.c:1199-1201); src points at the component's first byte */
    const int ps = cfg->transparency && !cfg->chroma_planes && !cfg->colorspace ? 2 : 1;
    for (int y = 0; y < h; y++) {
        const uint8_t *row = src + (int64_t)(y0 + y) * stride;
        for (int x = 0; x < w; x++) {
            int v;
            if (cfg->sample_bytes == 1) {
                v = row[ps * (x0 + x)];
            } else {
                v = row[2 * (x0 + x)] | (row[2 * (x0 + x) + 1] << 8);
                if (!cfg->packed_at_lsb)
                    v >>= 16 - cfg->bits_per_raw_sample;
            }
            dst[(int64_t)y * w + x] = (int16_t)v;
        }
    }
}

/* Neighbourhood of sample (x,y) inside one slice plane P (w x h), exactly as
 * the reference's zeroed ring buffer exposes it (ffv1enc.c:381-388):
 * rows above the slice are 0, L at x=0 is T, LT at x=0 is the sample two
 * rows up in column 0, RT past the right edge is T, LL at x=0 is 0 and at
 * x=1 is T(0). */
typedef struct taps {
    int X, L, T, LT, RT, LL, TT;
} taps;

static void get_taps(const int16_t *P, int w, int x, int y, taps *t)
{
    const int16_t *cur = P + (int64_t)y * w;
    const int16_t *up = y >= 1 ? cur - w : NULL;
    const int16_t *up2 = y >= 2 ? cur - 2 * w : NULL;
    t->X = cur[x];
    t->T = up ? up[x] : 0;
    int T0 = up ? up[0] : 0;
    t->L = x ? cur[x - 1] : T0;
    if (x)
        t->LT = up ? up[x - 1] : 0;
    else
        t->LT = up2 ? up2[0] : 0;
    t->RT = (x + 1 < w) ? (up ? up[x + 1] : 0) : t->T;
    t->LL = x >= 2 ? cur[x - 2] : (x == 1 ? T0 : 0);
    t->TT = up2 ? up2[x] : 0;
}

/* get_context + predict + sign normalisation + fold (ffv1.h:161-190,
 * ffv1enc.c:306-317). */
static void sample_symbol(const int16_t qt[5][256], int model1, int bits,
                          const taps *t, int *ctx_out, int *diff_out)
{
    int ctx = qt[0][(t->L - t->LT) & 0xFF] + qt[1][(t->LT - t->T) & 0xFF] +
              qt[2][(t->T - t->RT) & 0xFF];
    if (model1)
        ctx += qt[3][(t->LL - t->L) & 0xFF] + qt[4][(t->TT - t->T) & 0xFF];
    int pred = median3(t->L, t->L + t->T - t->LT, t->T);
    int diff = t->X - pred;
    if (ctx < 0) {
        ctx = -ctx;
        diff = -diff;
    }
    *ctx_out = ctx;
    *diff_out = fold_residual(diff, bits);
}

/* put_symbol_inline's statistics (ffv1enc.c:190-199): every decision of a
 * plane symbol counts into rc_stat[state before][bit] and rc_stat2[slot][bit],
 * counted here before the symbol is coded (the states then adapt the same
 * way in rc_put_symbol). */
static void count_symbol(ffv1o_enc *e, const uint8_t st[32], uint64_t stat2[32][2], int v)
{
    uint8_t s[32];
    memcpy(s, st, 32);
    const rc_tables *t = &e->frame_tab;
#define COUNT(slot, bit)                                  \
    do {                                                  \
        int b_ = (bit);                                   \
        e->rc_stat[s[slot]][b_]++;                        \
        stat2[slot][b_]++;                                \
        s[slot] = b_ ? t->to1[s[slot]] : t->to0[s[slot]]; \
    } while (0)
    if (v == 0) {
        COUNT(0, 1);
        return;
    }
    unsigned a = v < 0 ? -(unsigned)v : (unsigned)v;
    int ex = ilog2u(a);
    COUNT(0, 0);
    for (int i = 0; i < ex; i++)
        COUNT(1 + (i < 9 ? i : 9), 1);
    COUNT(1 + (ex < 9 ? ex : 9), 0);
    for (int i = ex - 1; i >= 0; i--)
        COUNT(22 + (i < 9 ? i : 9), (a >> i) & 1);
    COUNT(11 + (ex < 10 ? ex : 10), v < 0);
#undef COUNT
}

/* encode_line for the range coder: row y of slice plane P (w wide) */
static void code_row_rac(ffv1o_enc *e, rc_enc *c, plane_state *ps,
                         const int16_t *P, int w, int y)
{
    int model1 = e->cfg.context_model;
    if (c->end - c->ptr < (int64_t)w * 35) { /* ffv1enc.c:282-286 */
        e->line_err = 1;
        return;
    }
    if (e->pcm) { /* slice_coding_mode 1: every bit on a fresh state 128 (:294-304) */
        for (int x = 0; x < w; x++) {
            int v = P[(int64_t)y * w + x];
            for (int i = e->coded_bits - 1; i >= 0; i--) {
                uint8_t st = 128;
                rc_put(c, &st, (v >> i) & 1);
            }
        }
        return;
    }
    for (int x = 0; x < w; x++) {
        taps t;
        int ctx, diff;
        get_taps(P, w, x, y, &t);
        sample_symbol(e->qt, model1, e->coded_bits, &t, &ctx, &diff);
        if (e->pass1)
            count_symbol(e, ps->rac + (int64_t)ctx * 32, e->rc_stat2[ctx], diff);
        rc_put_symbol(c, ps->rac + (int64_t)ctx * 32, diff, 1);
    }
}

/* encode_line for Golomb-Rice incl. run mode (ffv1enc.c:306-370); the run
 * index persists across the lines of a plane (YCbCr: encode_plane resets it,
 * :379) or of the whole slice (RGB: encode_rgb_frame, :423) */
static void code_row_golomb(ffv1o_enc *e, bitw *b, plane_state *ps,
                            const int16_t *P, int w, int y, int *run_index_io)
{
    int model1 = e->cfg.context_model;
    int bits = e->coded_bits;
    int run_index = *run_index_io;
    int run_count = 0, run_mode = 0;
    if (b->end - b->base - (b->nbits >> 3) < (int64_t)w * 4) { /* ffv1enc.c:287-291 */
        e->line_err = 1;
        return;
    }
    for (int x = 0; x < w; x++) {
        taps t;
        int ctx, diff;
        get_taps(P, w, x, y, &t);
        sample_symbol(e->qt, model1, bits, &t, &ctx, &diff);
        if (ctx == 0)
            run_mode = 1;
        if (run_mode) {
            if (diff) {
                while (run_count >= 1 << log2_run[run_index]) {
                    run_count -= 1 << log2_run[run_index];
                    run_index++;
                    bw_put(b, 1, 1);
                }
                bw_put(b, 1 + log2_run[run_index], run_count);
                if (run_index)
                    run_index--;
                run_count = 0;
                run_mode = 0;
                if (diff > 0)
                    diff--;
            } else {
                run_count++;
            }
        }
        if (!run_mode)
            vlc_put(b, &ps->vlc[ctx], diff, bits);
    }
    if (run_mode) {
        while (run_count >= 1 << log2_run[run_index]) {
            run_count -= 1 << log2_run[run_index];
            run_index++;
            bw_put(b, 1, 1);
        }
        if (run_count)
            bw_put(b, 1, 1);
    }
    *run_index_io = run_index;
}

static void code_plane(ffv1o_enc *e, void *coder, int golomb, plane_state *ps,
                       const int16_t *P, int w, int h)
{
    int run_index = 0;
    for (int y = 0; y < h && !e->line_err; y++) {
        if (golomb)
            code_row_golomb(e, (bitw *)coder, ps, P, w, y, &run_index);
        else
            code_row_rac(e, (rc_enc *)coder, ps, P, w, y);
    }
}

/* The RCT of encode_rgb_frame (ffv1enc.c:430-458, v3: both coefficients 1):
 * pixel (x, y) of the slice as the three coded samples G', B', R'.  bgr0 is
 * one packed plane (B, G, R, X bytes); gbrp is three u16 planes whose first
 * is read as "b", second as "g", third as "r", as the reference does. */
static void rct_sample(const ffv1o_config *cfg, const uint8_t *const planes[4],
                       const int strides[4], int x, int y, int by, int ry, int pcm, int out[4])
{
    int b, g, r;
    int bits = cfg->bits_per_raw_sample;
    out[3] = 0;
    if (cfg->sample_bytes == 4) {
        const uint8_t *px = planes[0] + (int64_t)y * strides[0] + 4 * (int64_t)x;
        b = px[0];
        g = px[1];
        r = px[2];
        out[3] = px[3]; /* RGB32: a = v >> 24 (ffv1enc.c:440) */
    } else {
        const uint8_t *q0 = planes[0] + (int64_t)y * strides[0] + 2 * (int64_t)x;
        const uint8_t *q1 = planes[1] + (int64_t)y * strides[1] + 2 * (int64_t)x;
        const uint8_t *q2 = planes[2] + (int64_t)y * strides[2] + 2 * (int64_t)x;
        b = q0[0] | (q0[1] << 8);
        g = q1[0] | (q1[1] << 8);
        r = q2[0] | (q2[1] << 8);
    }
    if (pcm) { /* slice_coding_mode 1: no transform (ffv1enc.c:447) */
        out[0] = g;
        out[1] = b;
        out[2] = r;
        return;
    }
    b -= g;
    r -= g;
    g += (b * by + r * ry) >> 2;
    out[0] = g;
    out[1] = b + (1 << bits);
    out[2] = r + (1 << bits);
}

/* encode_line's "bits" (ffv1enc.c:393-405, 464-467): 8 or the raw depth
 * for YCbCr; RGB one more (9 at 8 bit) for the transformed samples, the raw
 * depth in PCM slices */
static int coded_bits_of(const ffv1o_config *cfg, int pcm)
{
    int bits = cfg->bits_per_raw_sample <= 8 ? 8 : cfg->bits_per_raw_sample;
    if (cfg->colorspace && !pcm)
        return bits + 1;
    return bits;
}

/* choose_rct_params (ffv1enc.c:1064-1144): the RCT luma coefficients whose
 * gradient-predicted G' residual is smallest over the slice.  Read as the
 * reference reads: 8-bit: one 32-bit B, G, R, X word per pixel of plane 0;
 * else three u16 planes as b, g, r at the slice's luma position.  The row's
 * differences are kept in int16 (sample_buffer) and the 15 sums in int,
 * both as the reference's arithmetic wraps. */
static void choose_rct(ffv1o_enc *e, const slice_ctx *s, const uint8_t *const planes[4],
                       const int strides[4])
{
    static const int coef[15][2] = {{0, 0}, {1, 1}, {2, 2}, {0, 2}, {2, 0}, {4, 0}, {0, 4}, {0, 3},
                                    {3, 0}, {3, 1}, {1, 3}, {1, 2}, {2, 1}, {0, 1}, {1, 0}};
    uint32_t stat[15] = {0};
    const int lbd = e->cfg.bits_per_raw_sample <= 8;
    int16_t *S = e->scratch; /* [3][w] */
    const int w = s->w;
    for (int y = 0; y < s->h; y++) {
        int lastr = 0, lastg = 0, lastb = 0;
        for (int x = 0; x < w; x++) {
            int b, g, r;
            const int X = s->x0 + x, Y = s->y0 + y;
            if (lbd) {
                const uint8_t *px = planes[0] + (int64_t)Y * strides[0] + 4 * (int64_t)X;
                b = px[0];
                g = px[1];
                r = px[2];
            } else {
                const uint8_t *q0 = planes[0] + (int64_t)Y * strides[0] + 2 * (int64_t)X;
                const uint8_t *q1 = planes[1] + (int64_t)Y * strides[1] + 2 * (int64_t)X;
                const uint8_t *q2 = planes[2] + (int64_t)Y * strides[2] + 2 * (int64_t)X;
                b = q0[0] | (q0[1] << 8);
                g = q1[0] | (q1[1] << 8);
                r = q2[0] | (q2[1] << 8);
            }
            int ar = r - lastr, ag = g - lastg, ab = b - lastb;
            if (x && y) {
                int bg = ag - S[x], bb = ab - S[w + x], br = ar - S[2 * w + x];
                br -= bg;
                bb -= bg;
                for (int i = 0; i < 15; i++) {
                    int v = bg + ((br * coef[i][0] + bb * coef[i][1]) >> 2);
                    stat[i] += (uint32_t)(v < 0 ? -v : v);
                }
            }
            S[x] = (int16_t)ag;
            S[w + x] = (int16_t)ab;
            S[2 * w + x] = (int16_t)ar;
            lastr = r;
            lastg = g;
            lastb = b;
        }
    }
    int best = 0;
    for (int i = 1; i < 15; i++)
        if ((int32_t)stat[i] < (int32_t)stat[best])
            best = i;
    e->rct_by = coef[best][1];
    e->rct_ry = coef[best][0];
}

/* encode_rgb_frame (ffv1enc.c:413-473): the lines of G', B', R' (and A
 * for RGB32) interleaved (row y of each plane in turn), plane contexts 0,
 * 1, 1, 2 ((p + 1) / 2); one run index for the whole slice; every plane
 * coded at 9 bits at 8-bit depth, alpha included (:464-465). */
static void code_rgb_slice(ffv1o_enc *e, slice_ctx *s, const uint8_t *const planes[4],
                           const int strides[4], void *coder, int golomb)
{
    int64_t n = (int64_t)s->w * s->h;
    int16_t *P[4] = {e->scratch, e->scratch + n, e->scratch + 2 * n, e->scratch + 3 * n};
    const int np = 3 + (e->cfg.transparency != 0);
    for (int y = 0; y < s->h; y++)
        for (int x = 0; x < s->w; x++) {
            int v[4];
            rct_sample(&e->cfg, planes, strides, s->x0 + x, s->y0 + y, e->rct_by, e->rct_ry, e->pcm, v);
            for (int p = 0; p < np; p++)
                P[p][(int64_t)y * s->w + x] = (int16_t)v[p];
        }
    int run_index = 0;
    for (int y = 0; y < s->h && !e->line_err; y++)
        for (int p = 0; p < np && !e->line_err; p++) {
            plane_state *ps = &s->ps[(p + 1) / 2];
            if (golomb)
                code_row_golomb(e, (bitw *)coder, ps, P[p], s->w, y, &run_index);
            else
                code_row_rac(e, (rc_enc *)coder, ps, P[p], s->w, y);
        }
}

static void clear_slice_states(ffv1o_enc *e, slice_ctx *s)
{
    const uint8_t *is = e->init_states[e->cfg.context_model];
    for (int p = 0; p < e->plane_count; p++) {
        if (is) /* ff_ffv1_clear_slice_state (ffv1.c:185-189) */
            memcpy(s->ps[p].rac, is, (size_t)e->contexts * 32);
        else
            memset(s->ps[p].rac, 128, (size_t)e->contexts * 32);
        for (int j = 0; j < e->contexts; j++)
            vlc_reset(&s->ps[p].vlc[j]);
    }
}

/* Planes of one slice in coding order: Y (plane context 0) then Cb, Cr
 * (both plane context 1), then A (plane context 2) at the luma size
 * (ffv1enc.c:1185-1198); YA8: Y and A of the one packed plane, A with plane
 * context 1 (:1199-1201).  planes[3] is the alpha plane of the YUVA
 * formats. */
typedef void (*plane_fn)(ffv1o_enc *, void *, plane_state *, const int16_t *,
                         int, int);

static void for_each_plane(ffv1o_enc *e, slice_ctx *s,
                           const uint8_t *const planes[4], const int strides[4],
                           void *coder, int golomb)
{
    const ffv1o_config *cfg = &e->cfg;
    if (cfg->transparency && !cfg->chroma_planes) { /* YA8 */
        for (int p = 0; p < 2; p++) {
            load_plane(cfg, planes[0] + p, strides[0], s->x0, s->y0, s->w, s->h, e->scratch);
            code_plane(e, coder, golomb, &s->ps[p], e->scratch, s->w, s->h);
        }
        return;
    }
    int np = cfg->chroma_planes ? 3 : 1;
    for (int p = 0; p < np; p++) {
        int x0 = s->x0, y0 = s->y0, w = s->w, h = s->h;
        if (p) {
            w = ceil_rshift(s->w, cfg->chroma_h_shift);
            h = ceil_rshift(s->h, cfg->chroma_v_shift);
            x0 = s->x0 >> cfg->chroma_h_shift;
            y0 = s->y0 >> cfg->chroma_v_shift;
        }
        load_plane(cfg, planes[p], strides[p], x0, y0, w, h, e->scratch);
        code_plane(e, coder, golomb, &s->ps[p ? 1 : 0], e->scratch, w, h);
    }
    if (cfg->transparency) {
        load_plane(cfg, planes[3], strides[3], s->x0, s->y0, s->w, s->h, e->scratch);
        code_plane(e, coder, golomb, &s->ps[2], e->scratch, s->w, s->h);
    }
}

static void code_slice_planes(ffv1o_enc *e, slice_ctx *s, const uint8_t *const planes[4],
                              const int strides[4], void *coder, int golomb)
{
    if (e->cfg.colorspace)
        code_rgb_slice(e, s, planes, strides, coder, golomb);
    else
        for_each_plane(e, s, planes, strides, coder, golomb);
}

/* encode_slice (ffv1enc.c:1146-1220) of slice i into its buffer.  Slices
 * are independent (their own coder, states and buffer), which is what the
 * reference's per-slice jobs rely on (avctx->execute, ffv1enc.c:1323); the
 * per-slice scratch fields of e (line_err, pcm, rct, scratch) belong to the
 * caller's thread. */
static int enc_slice(ffv1o_enc *e, int i, int key, const uint8_t *const planes[4],
                     const int strides[4])
{
    const ffv1o_config *cfg = &e->cfg;
    slice_ctx *s = &e->sl[i];
    rc_enc c;
    s->error = 0;
    /* slice 0 continues the packet-level coder that carries the key bit
     * (+ the v0/v1 header) coded with the default table, ffv1enc.c:1287-1315 */
    rc_enc_init(&c, s->buf, s->cap, &e->frame_tab);
    if (i == 0) {
        uint8_t ks = 128;
        c.t = &e->dflt;
        rc_put(&c, &ks, key);
        if (key && cfg->version < 2)
            put_v01_header(e, &c);
        else if (key && cfg->version == 2)
            put_v2_header(e, &c);
        c.t = &e->frame_tab;
    }
    /* v4 picks the slice's RCT coefficients; a range-coded v4 slice that
     * does not fit its buffer is coded again as PCM from the coder state it
     * started with */
    e->pcm = 0;
    e->rct_by = e->rct_ry = 1;
    if (cfg->version > 3)
        choose_rct(e, s, planes, strides);
    const rc_enc c_bak = c;
retry:
    e->line_err = 0;
    e->coded_bits = coded_bits_of(cfg, e->pcm);
    if (key)
        clear_slice_states(e, s);
    if (cfg->version > 2)
        put_slice_header(e, s, &c);

    if (cfg->ac == 0) {
        bitw b;
        int64_t ac_bytes = 0;
        if (cfg->version > 2) {
            uint8_t st = 129;
            rc_put(&c, &st, 0);
        }
        if (cfg->version > 2 || (s->x0 == 0 && s->y0 == 0))
            ac_bytes = rc_finish(&c);
        bw_init(&b, s->buf + ac_bytes, s->cap - ac_bytes);
        code_slice_planes(e, s, planes, strides, &b, 1);
        s->bytes = ac_bytes + bw_bytes(&b);
        s->error = b.overflow || c.overflow || e->line_err;
    } else {
        code_slice_planes(e, s, planes, strides, &c, 0);
        if (e->line_err && cfg->version > 3 && !e->pcm) {
            e->pcm = 1;
            c = c_bak;
            goto retry;
        }
        uint8_t st = 129;
        rc_put(&c, &st, 0);
        s->bytes = rc_finish(&c);
        s->error = c.overflow || e->line_err;
        s->pcm = e->pcm;
    }
    return s->error ? AVERR_INVALIDDATA : 0;
}

/* One worker of ffv1o_enc_frame_mt: slices t, t + n, ... with a private
 * copy of the encoder's per-slice scratch fields. */
typedef struct slice_job {
    ffv1o_enc w;
    int first, step, key, rc;
    const uint8_t *const *planes;
    const int *strides;
} slice_job;

static void *slice_worker(void *arg)
{
    slice_job *j = arg;
    for (int i = j->first; i < j->w.nslices && !j->rc; i += j->step)
        j->rc = enc_slice(&j->w, i, j->key, j->planes, j->strides);
    return NULL;
}

static int64_t assemble_packet(ffv1o_enc *e, uint8_t *out, int64_t cap);

int64_t ffv1o_enc_frame(ffv1o_enc *e, const uint8_t *const planes[4],
                        const int strides[4], uint8_t *out, int64_t cap,
                        int *key_out)
{
    return ffv1o_enc_frame_mt(e, planes, strides, out, cap, key_out, 1);
}

int64_t ffv1o_enc_frame_mt(ffv1o_enc *e, const uint8_t *const planes[4],
                           const int strides[4], uint8_t *out, int64_t cap,
                           int *key_out, int threads)
{
    const ffv1o_config *cfg = &e->cfg;
    int key = cfg->gop_size == 0 || e->picture_number % cfg->gop_size == 0;
    if (key)
        e->gob_count++; /* ffv1enc.c:1302 */
    if (threads > e->nslices)
        threads = e->nslices;
    if (threads <= 1 || e->pass1) {  /* pass 1 counts into one table: serial */
        for (int i = 0; i < e->nslices; i++) {
            int rc = enc_slice(e, i, key, planes, strides);
            if (rc)
                return rc;
        }
    } else {
        /* the reference's threading: one job per slice, threads =
         * min(cores, slices) (ffv1enc.c:1323, avctx->execute) */
        slice_job *jobs = calloc((size_t)threads, sizeof(slice_job));
        pthread_t *th = calloc((size_t)threads, sizeof(pthread_t));
        int64_t maxw = 0;
        for (int i = 0; i < e->nslices; i++)
            if ((int64_t)e->sl[i].w * e->sl[i].h > maxw)
                maxw = (int64_t)e->sl[i].w * e->sl[i].h;
        int rc = jobs && th ? 0 : AVERR_ENOMEM, started = 0;
        for (int t = 0; t < threads && !rc; t++) {
            jobs[t].w = *e;
            jobs[t].w.scratch = malloc(4 * (size_t)maxw * sizeof(int16_t) + 16);
            jobs[t].first = t;
            jobs[t].step = threads;
            jobs[t].key = key;
            jobs[t].planes = planes;
            jobs[t].strides = strides;
            if (!jobs[t].w.scratch || pthread_create(&th[t], NULL, slice_worker, &jobs[t])) {
                free(jobs[t].w.scratch);
                rc = AVERR_ENOMEM;
                break;
            }
            started++;
        }
        for (int t = 0; t < started; t++) {
            pthread_join(th[t], NULL);
            if (!rc)
                rc = jobs[t].rc;
            free(jobs[t].w.scratch);
        }
        free(jobs);
        free(th);
        if (rc)
            return rc;
    }
    int64_t pos = assemble_packet(e, out, cap);
    if (pos < 0)
        return pos;
    e->picture_number++;
    if (key_out)
        *key_out = key;
    return pos;
}

static int64_t assemble_packet(ffv1o_enc *e, uint8_t *out, int64_t cap)
{
    const ffv1o_config *cfg = &e->cfg;
    /* packet assembly, ffv1enc.c:1326-1354 */
    int64_t pos = 0;
    for (int i = 0; i < e->nslices; i++) {
        slice_ctx *s = &e->sl[i];
        int64_t n = s->bytes;
        int64_t need = n + 3 + 5;
        if (pos + need > cap)
            return AVERR_ENOMEM;
        memcpy(out + pos, s->buf, n);
        if (i > 0 || cfg->version > 2) {
            out[pos + n] = (uint8_t)(n >> 16);
            out[pos + n + 1] = (uint8_t)(n >> 8);
            out[pos + n + 2] = (uint8_t)n;
            n += 3;
        }
        if (cfg->ec) {
            out[pos + n++] = 0;
            put_be32(out + pos + n, ffv1o_crc32(0, out + pos, n));
            n += 4;
        }
        pos += n;
    }
    return pos;
}

/* The P-frame carry of every slice (PlaneContext.state, ffv1.h:72):
 * [slice][plane_ctx 0..1][context][32] bytes, range coder only; and the
 * picture number that places keyframes (ffv1enc.c:1299).  Used to resume a
 * stream mid-GOP in another encoder (the multi-rank exchange step). */
int64_t ffv1o_enc_get_states(const ffv1o_enc *e, uint8_t *buf, int64_t cap)
{
    const int pc = e->plane_count;
    int64_t per = (int64_t)e->contexts * 32, n = pc * per * e->nslices;
    if (!buf)
        return n;
    if (cap < n)
        return -1;
    for (int i = 0; i < e->nslices; i++)
        for (int p = 0; p < pc; p++)
            memcpy(buf + ((int64_t)pc * i + p) * per, e->sl[i].ps[p].rac, (size_t)per);
    return n;
}

int ffv1o_enc_set_states(ffv1o_enc *e, const uint8_t *buf, int64_t size,
                         int64_t picture_number)
{
    const int pc = e->plane_count;
    int64_t per = (int64_t)e->contexts * 32;
    if (size != pc * per * e->nslices)
        return -1;
    for (int i = 0; i < e->nslices; i++)
        for (int p = 0; p < pc; p++)
            memcpy(e->sl[i].ps[p].rac, buf + ((int64_t)pc * i + p) * per, (size_t)per);
    e->picture_number = picture_number;
    return 0;
}

int ffv1o_enc_last_slice_pcm(const ffv1o_enc *e, int *pcm, int n)
{
    for (int i = 0; i < n && i < e->nslices; i++)
        pcm[i] = e->sl[i].pcm;
    return e->nslices;
}

int ffv1o_enc_last_slice_bytes(const ffv1o_enc *e, int *bytes, int n)
{
    for (int i = 0; i < n && i < e->nslices; i++)
        bytes[i] = (int)e->sl[i].bytes;
    return e->nslices;
}

int64_t ffv1o_slice_symbols(const ffv1o_config *cfg,
                            const uint8_t *const planes[4],
                            const int strides[4], int slice, int32_t *out,
                            int64_t cap)
{
    int16_t qt[5][256];
    build_quant_set(qt, cfg->context_model, cfg->bits_per_raw_sample);
    int bits = cfg->bits_per_raw_sample <= 8 ? 8 : cfg->bits_per_raw_sample;
    int x0, y0, w, h;
    slice_rects(cfg, slice, &x0, &y0, &w, &h);
    int np = cfg->chroma_planes ? 3 : 1;
    int64_t n = 0;
    int16_t *P = malloc((size_t)w * h * sizeof(int16_t) + 16);
    for (int p = 0; p < np; p++) {
        int px = x0, py = y0, pw = w, ph = h;
        if (p) {
            pw = ceil_rshift(w, cfg->chroma_h_shift);
            ph = ceil_rshift(h, cfg->chroma_v_shift);
            px = x0 >> cfg->chroma_h_shift;
            py = y0 >> cfg->chroma_v_shift;
        }
        load_plane(cfg, planes[p], strides[p], px, py, pw, ph, P);
        for (int y = 0; y < ph; y++)
            for (int x = 0; x < pw; x++) {
                taps t;
                int ctx, diff;
                get_taps(P, pw, x, y, &t);
                sample_symbol((const int16_t(*)[256])qt, cfg->context_model,
                              bits, &t, &ctx, &diff);
                if (n < cap)
                    out[n] = (int32_t)(((uint32_t)ctx << 16) | (uint16_t)diff);
                n++;
            }
    }
    free(P);
    return n;
}

/* ------------------------------------------------------------------------ */
/* Decoder (ffv1dec.c) -- used only for lossless round-trip checks          */

typedef struct dslice {
    int x0, y0, w, h;
    int pcm, rct_by, rct_ry; /* v4 slice header (ffv1dec.c:344-356); else 0, 1, 1 */
    plane_state ps[3];
    int damaged; /* slice_damaged: set by a CRC / header / end mismatch, cleared by read_header */
    int qi;      /* v2: the slice's quant set from the keyframe header */
} dslice;

struct ffv1o_dec {
    ffv1o_config cfg;
    int version, micro_version, ac, ec, bits, chroma_planes, hs, vs, colorspace;
    int transparency, plane_count; /* ffv1dec.c:558-559, 693-695 */
    int cur_pcm;                   /* the slice being decoded is PCM */
    int num_h, num_v;
    int16_t qsets[2][5][256];
    int ctx_count[2];
    int16_t qt[5][256];     /* v0/v1 in-band tables */
    int contexts;
    rc_tables dflt, frame_tab;
    uint8_t stt[256];
    int nslices;
    dslice *sl;
    int key_ok;
    int16_t *scratch;
    /* last_picture for the concealment copy (ffv1dec.c:998-1021) */
    uint8_t *last[4];
    int last_row[4], last_rows[4];
    int have_last;
    uint8_t *init_states[2]; /* per quant set from the extradata, NULL = all 128 */
};

/* Planes of the output picture (the encoder's input layout): row bytes,
 * rows and bytes per pixel; YUVA's alpha is plane 3 at the luma size, YA8
 * one plane of Y and A bytes, bgr0 / RGB32 one plane of 4-byte pixels. */
static int out_planes(const ffv1o_dec *d, int row[4], int rows[4], int step[4])
{
    const ffv1o_config *c = &d->cfg;
    int sb = c->sample_bytes;
    int np = c->chroma_planes && sb != 4 ? 3 : 1;
    step[0] = np == 1 && c->transparency && !c->colorspace ? 2 : sb;
    row[0] = c->width * step[0];
    rows[0] = c->height;
    for (int k = 1; k < 3; k++) {
        step[k] = sb;
        row[k] = k < np ? ceil_rshift(c->width, c->chroma_h_shift) * sb : 0;
        rows[k] = k < np ? ceil_rshift(c->height, c->chroma_v_shift) : 0;
    }
    step[3] = sb;
    row[3] = rows[3] = 0;
    if (np == 3 && c->transparency) {
        row[3] = c->width * sb;
        rows[3] = c->height;
        np = 4;
    }
    return np;
}

/* read_quant_table(s), ffv1dec.c:475-515 */
static int get_quant_tables(rc_dec *c, int16_t qt[5][256])
{
    int count = 1;
    for (int t = 0; t < 5; t++) {
        uint8_t st[32];
        memset(st, 128, 32);
        int i = 0, v;
        for (v = 0; i < 128; v++) {
            unsigned len = (unsigned)rc_get_symbol(c, st, 0) + 1;
            if (len > (unsigned)(128 - i) || !len)
                return -1;
            while (len--)
                qt[t][i++] = (int16_t)(count * v);
        }
        for (i = 1; i < 128; i++)
            qt[t][256 - i] = -qt[t][i];
        qt[t][128] = -qt[t][127];
        count *= 2 * v - 1;
        if (count > 32768)
            return -1;
    }
    return (count + 1) / 2;
}

static void dec_alloc_slices(ffv1o_dec *d)
{
    d->nslices = d->num_h * d->num_v;
    d->sl = calloc(d->nslices, sizeof(dslice));
    int maxctx = 7563;
    for (int i = 0; i < d->nslices; i++) {
        slice_rects(&d->cfg, i, &d->sl[i].x0, &d->sl[i].y0, &d->sl[i].w,
                    &d->sl[i].h);
        for (int p = 0; p < 3; p++) {
            d->sl[i].ps[p].rac = malloc((size_t)maxctx * 32);
            d->sl[i].ps[p].vlc = malloc((size_t)maxctx * sizeof(vlc_ctx));
        }
    }
}

ffv1o_dec *ffv1o_dec_new(const ffv1o_config *cfg, const uint8_t *ex, int exn)
{
    ffv1o_dec *d = calloc(1, sizeof(*d));
    d->cfg = *cfg;
    rc_default_tables(&d->dflt);
    d->frame_tab = d->dflt;
    d->version = cfg->version;
    d->num_h = d->num_v = 1;
    d->scratch = malloc(4 * (size_t)cfg->width * cfg->height * sizeof(int16_t) + 16);
    d->transparency = cfg->transparency;
    d->plane_count = 2 + (cfg->transparency != 0);
    if (exn > 0) { /* read_extra_header, ffv1dec.c:517-636 */
        if (ffv1o_crc32(0, ex, exn) != 0)
            goto fail;
        rc_dec c;
        uint8_t st[32];
        memset(st, 128, 32);
        rc_dec_init(&c, ex, exn - 4, &d->dflt);
        d->version = rc_get_symbol(&c, st, 0);
        if (d->version > 2)
            d->micro_version = rc_get_symbol(&c, st, 0);
        d->ac = rc_get_symbol(&c, st, 0);
        if (d->ac == 2) {
            for (int i = 1; i < 256; i++)
                d->stt[i] = (uint8_t)(rc_get_symbol(&c, st, 1) + d->dflt.to1[i]);
            rc_custom_tables(&d->frame_tab, &d->dflt, d->stt);
        }
        d->colorspace = rc_get_symbol(&c, st, 0);
        if (d->colorspace > 1)
            goto fail;
        d->bits = rc_get_symbol(&c, st, 0);
        d->chroma_planes = rc_get(&c, &st[0]);
        d->hs = rc_get_symbol(&c, st, 0);
        d->vs = rc_get_symbol(&c, st, 0);
        d->transparency = rc_get(&c, &st[0]);
        d->plane_count = 1 + (d->chroma_planes || d->version < 4) + d->transparency;
        d->num_h = 1 + rc_get_symbol(&c, st, 0);
        d->num_v = 1 + rc_get_symbol(&c, st, 0);
        int nq = rc_get_symbol(&c, st, 0);
        if (nq < 1 || nq > 2)
            goto fail;
        for (int i = 0; i < nq; i++) {
            d->ctx_count[i] = get_quant_tables(&c, d->qsets[i]);
            if (d->ctx_count[i] < 0)
                goto fail;
        }
        uint8_t st2[32][32];
        memset(st2, 128, sizeof(st2));
        for (int i = 0; i < nq; i++) { /* read_extra_header, ffv1dec.c:592-601 */
            if (!rc_get(&c, &st[0]))
                continue;
            int n = d->ctx_count[i] * 32;
            uint8_t *is = malloc((size_t)n);
            for (int j = 0; j < n; j++) {
                int pred = j >= 32 ? is[j - 32] : 128;
                is[j] = (uint8_t)((pred + rc_get_symbol(&c, st2[j & 31], 1)) & 0xFF);
            }
            d->init_states[i] = is;
        }
        if (d->version > 2) {
            d->ec = rc_get_symbol(&c, st, 0);
            if (d->micro_version > 2)
                (void)rc_get_symbol(&c, st, 0);
        }
        d->cfg.num_h_slices = d->num_h;
        d->cfg.num_v_slices = d->num_v;
    }
    dec_alloc_slices(d);
    return d;
fail:
    free(d->scratch);
    free(d);
    return NULL;
}

void ffv1o_dec_free(ffv1o_dec *d)
{
    if (!d)
        return;
    for (int i = 0; i < d->nslices; i++)
        for (int p = 0; p < 3; p++) {
            free(d->sl[i].ps[p].rac);
            free(d->sl[i].ps[p].vlc);
        }
    for (int k = 0; k < 4; k++)
        free(d->last[k]);
    free(d->init_states[0]);
    free(d->init_states[1]);
    free(d->sl);
    free(d->scratch);
    free(d);
}

/* decode_line (ffv1dec.c:42-117): row y of slice plane P (w wide), samples
 * masked to `bits` (av_mod_uintp2); the run index persists as in
 * code_row_golomb. */
static void decode_row(void *coder, int golomb, plane_state *ps, const int16_t qt[5][256],
                       int model1, int16_t *P, int w, int y, int bits, int *run_index_io)
{
    int run_index = *run_index_io;
    int run_count = 0, run_mode = 0;
    for (int x = 0; x < w; x++) {
        taps t;
        P[(int64_t)y * w + x] = 0;
        get_taps(P, w, x, y, &t);
        int ctx = qt[0][(t.L - t.LT) & 0xFF] + qt[1][(t.LT - t.T) & 0xFF] +
                  qt[2][(t.T - t.RT) & 0xFF];
        if (model1)
            ctx += qt[3][(t.LL - t.L) & 0xFF] + qt[4][(t.TT - t.T) & 0xFF];
        int sign = ctx < 0, diff;
        if (sign)
            ctx = -ctx;
        if (!golomb) {
            diff = rc_get_symbol((rc_dec *)coder, ps->rac + (int64_t)ctx * 32, 1);
        } else {
            bitr *b = (bitr *)coder;
            if (ctx == 0 && run_mode == 0)
                run_mode = 1;
            if (run_mode) {
                if (run_count == 0 && run_mode == 1) {
                    if (br_get(b, 1)) {
                        run_count = 1 << log2_run[run_index];
                        if (x + run_count <= w)
                            run_index++;
                    } else {
                        run_count = log2_run[run_index]
                                        ? br_get(b, log2_run[run_index]) : 0;
                        if (run_index)
                            run_index--;
                        run_mode = 2;
                    }
                }
                run_count--;
                if (run_count < 0) {
                    run_mode = 0;
                    run_count = 0;
                    diff = vlc_get(b, &ps->vlc[ctx], bits);
                    if (diff >= 0)
                        diff++;
                } else {
                    diff = 0;
                }
            } else {
                diff = vlc_get(b, &ps->vlc[ctx], bits);
            }
        }
        /* a damaged stream can decode any int here (the reference's int
         * arithmetic wraps on it); unsigned keeps that defined */
        if (sign)
            diff = (int)(0u - (unsigned)diff);
        int pred = median3(t.L, t.L + t.T - t.LT, t.T);
        P[(int64_t)y * w + x] = (int16_t)(((unsigned)pred + (unsigned)diff) & ((1u << bits) - 1));
    }
    *run_index_io = run_index;
}

/* decode_line's PCM branch (ffv1dec.c:111-120): every bit on a fresh state 128 */
static void decode_row_pcm(rc_dec *c, int16_t *P, int w, int y, int bits)
{
    for (int x = 0; x < w; x++) {
        int v = 0;
        for (int i = 0; i < bits; i++) {
            uint8_t st = 128;
            v += v + rc_get(c, &st);
        }
        P[(int64_t)y * w + x] = (int16_t)v;
    }
}

/* decode_plane (ffv1dec.c:200-224): reconstruct into P, then store with
 * the pixel format's alignment. */
static void decode_plane_any(ffv1o_dec *d, void *coder, int golomb,
                             plane_state *ps, const int16_t qt[5][256],
                             int model1, int w, int h, uint8_t *dst,
                             int stride, int x0, int y0, int pixel_stride)
{
    int bits = d->bits <= 8 ? 8 : d->bits;
    int16_t *P = d->scratch;
    int run_index = 0;
    for (int y = 0; y < h; y++)
        if (d->cur_pcm)
            decode_row_pcm((rc_dec *)coder, P, w, y, bits);
        else
            decode_row(coder, golomb, ps, qt, model1, P, w, y, bits, &run_index);
    for (int y = 0; y < h; y++) {
        uint8_t *row = dst + (int64_t)(y0 + y) * stride;
        for (int x = 0; x < w; x++) {
            unsigned v = (uint16_t)P[(int64_t)y * w + x];
            if (d->cfg.sample_bytes == 1) {
                row[pixel_stride * (x0 + x)] = (uint8_t)v;
            } else {
                if (!d->cfg.packed_at_lsb)
                    v = (v << (16 - d->bits)) & 0xFFFF;
                row[2 * (x0 + x)] = (uint8_t)v;
                row[2 * (x0 + x) + 1] = (uint8_t)(v >> 8);
            }
        }
    }
}

/* decode_rgb_frame (ffv1dec.c:226-280): G', B', R' lines interleaved, then
 * the inverse RCT; bgr0 gets B, G, R and a zero fourth byte. */
static void decode_rgb_slice(ffv1o_dec *d, void *coder, int golomb, dslice *s,
                             const int16_t qt[5][256], int model1,
                             uint8_t *const planes[4], const int strides[4])
{
    int lbd = d->bits <= 8;
    int bits = (lbd ? 8 : d->bits) + !s->pcm; /* ffv1dec.c:252-255 */
    int offset = 1 << (lbd ? 8 : d->bits);
    int64_t n = (int64_t)s->w * s->h;
    int16_t *P[4] = {d->scratch, d->scratch + n, d->scratch + 2 * n, d->scratch + 3 * n};
    const int np = 3 + (d->transparency != 0);
    int run_index = 0;
    for (int y = 0; y < s->h; y++)
        for (int p = 0; p < np; p++)
            if (s->pcm)
                decode_row_pcm((rc_dec *)coder, P[p], s->w, y, bits);
            else
                decode_row(coder, golomb, &s->ps[(p + 1) / 2], qt, model1, P[p], s->w, y, bits,
                           &run_index);
    for (int y = 0; y < s->h; y++)
        for (int x = 0; x < s->w; x++) {
            int64_t i = (int64_t)y * s->w + x;
            int g = P[0][i], b = P[1][i], r = P[2][i];
            if (!s->pcm) { /* ffv1dec.c:263-269 */
                b -= offset;
                r -= offset;
                g -= (b * s->rct_by + r * s->rct_ry) >> 2;
                b += g;
                r += g;
            }
            int X = s->x0 + x, Y = s->y0 + y;
            if (lbd) { /* one 32-bit store of b + (g << 8) + (r << 16) + (a << 24): carries cross bytes */
                uint8_t *px = planes[0] + (int64_t)Y * strides[0] + 4 * (int64_t)X;
                const uint32_t a = np > 3 ? (uint32_t)P[3][i] : 0u;
                uint32_t v = (uint32_t)b + ((uint32_t)g << 8) + ((uint32_t)r << 16) + (a << 24);
                px[0] = (uint8_t)v;
                px[1] = (uint8_t)(v >> 8);
                px[2] = (uint8_t)(v >> 16);
                px[3] = (uint8_t)(v >> 24);
            } else {
                int v[3] = {b, g, r};
                for (int k = 0; k < 3; k++) {
                    uint8_t *q = planes[k] + (int64_t)Y * strides[k] + 2 * (int64_t)X;
                    q[0] = (uint8_t)v[k];
                    q[1] = (uint8_t)(v[k] >> 8);
                }
            }
        }
}

int ffv1o_dec_frame(ffv1o_dec *d, const uint8_t *pkt, int64_t size,
                    uint8_t *const planes[4], const int strides[4], int *key_out)
{
    rc_dec c0;
    uint8_t ks = 128;
    rc_dec_init(&c0, pkt, size, &d->dflt);
    int key = rc_get(&c0, &ks);
    if (key) {
        if (d->version < 2) { /* read_header v0/v1, ffv1dec.c:646-700 */
            uint8_t st[32];
            memset(st, 128, 32);
            d->version = rc_get_symbol(&c0, st, 0);
            d->ac = rc_get_symbol(&c0, st, 0);
            if (d->ac == 2) {
                for (int i = 1; i < 256; i++)
                    d->stt[i] = (uint8_t)(rc_get_symbol(&c0, st, 1) + d->dflt.to1[i]);
                rc_custom_tables(&d->frame_tab, &d->dflt, d->stt);
            } else {
                d->frame_tab = d->dflt;
            }
            d->colorspace = rc_get_symbol(&c0, st, 0);
            d->bits = d->version > 0 ? rc_get_symbol(&c0, st, 0) : 8;
            d->chroma_planes = rc_get(&c0, &st[0]);
            d->hs = rc_get_symbol(&c0, st, 0);
            d->vs = rc_get_symbol(&c0, st, 0);
            d->transparency = rc_get(&c0, &st[0]);
            d->plane_count = 2 + d->transparency; /* ffv1dec.c:695 */
            d->contexts = get_quant_tables(&c0, d->qt);
            if (d->contexts < 0)
                return -1;
        } else if (d->version == 2) { /* read_header v2, ffv1dec.c:801-868 */
            uint8_t st[32];
            memset(st, 128, 32);
            /* the reference takes any count up to the grid's; an encoder
             * writes the whole grid (ffv1enc.c:1008), and so must a packet
             * here */
            if (rc_get_symbol(&c0, st, 0) != d->nslices)
                return -1;
            const int64_t W = d->cfg.width, H = d->cfg.height;
            for (int j = 0; j < d->nslices; j++) {
                dslice *s = &d->sl[j];
                int64_t sx = rc_get_symbol(&c0, st, 0) * W, sy = rc_get_symbol(&c0, st, 0) * H;
                int64_t sw = (rc_get_symbol(&c0, st, 0) + 1) * W + sx;
                int64_t sh = (rc_get_symbol(&c0, st, 0) + 1) * H + sy;
                sx /= d->num_h;
                sy /= d->num_v;
                sw = sw / d->num_h - sx;
                sh = sh / d->num_v - sy;
                if ((uint32_t)sw > W || (uint32_t)sh > H || (uint32_t)sx + (uint64_t)(uint32_t)sw > (uint64_t)W ||
                    (uint32_t)sy + (uint64_t)(uint32_t)sh > (uint64_t)H)
                    return -1;
                s->x0 = (int)sx; s->y0 = (int)sy; s->w = (int)sw; s->h = (int)sh;
                /* each plane names its set; the slices here code every plane
                 * with one set, so they must agree (ours always do) */
                for (int k = 0; k < d->plane_count; k++) {
                    unsigned idx = (unsigned)rc_get_symbol(&c0, st, 0);
                    if (idx > 1 || !d->ctx_count[idx] || (k && (int)idx != s->qi))
                        return -1;
                    s->qi = (int)idx;
                }
            }
        }
        d->key_ok = 1;
    } else if (!d->key_ok) {
        return -3;
    }
    if (d->version == 0 && d->bits == 0)
        d->bits = 8;

    /* slice chain from the end of the packet, ffv1dec.c:948-989 */
    int trailer = 3 + (d->ec ? 5 : 0);
    int64_t starts[256], lens[256];
    int crc_bad[256];
    int n = d->nslices;
    const uint8_t *p = pkt + size;
    if (d->version > 2) { /* count slices (read_header :805-818) */
        int cnt = 0;
        const uint8_t *q = pkt + size;
        while (cnt < 256 && q - pkt > 3) {
            int64_t sz = (q[-trailer] << 16) | (q[-trailer + 1] << 8) | q[-trailer + 2];
            if (sz + trailer > q - pkt)
                break;
            q -= sz + trailer;
            cnt++;
        }
        if (cnt != n)
            return -1;
    }
    for (int i = n - 1; i >= 0; i--) {
        int64_t v;
        if (i || d->version > 2)
            v = ((p[-trailer] << 16) | (p[-trailer + 1] << 8) | p[-trailer + 2]) + trailer;
        else
            v = p - pkt;
        if (p - pkt < v)
            return -1;
        p -= v;
        crc_bad[i] = d->ec && ffv1o_crc32(0, p, v) != 0; /* ffv1dec.c:963-977 */
        starts[i] = p - pkt;
        lens[i] = v;
    }
    if (key) /* read_header clears slice_damaged (ffv1dec.c:820-825) */
        for (int i = 0; i < n; i++)
            d->sl[i].damaged = 0;

    for (int i = 0; i < n; i++) {
        dslice *s = &d->sl[i];
        rc_dec c;
        if (i == 0) {
            c = c0;
            c.end = pkt + starts[0] + lens[0];
        } else {
            rc_dec_init(&c, pkt + starts[i], lens[i], &d->frame_tab);
        }
        c.t = &d->frame_tab;
        int reset = 0;
        s->pcm = 0;
        s->rct_by = s->rct_ry = 1;
        const int16_t(*qt)[256] = (const int16_t(*)[256])d->qt;
        /* get_context takes the LL / TT terms when the table has them
         * (ffv1.h:161-176): context model 1's in-band v0/v1 tables */
        int model1 = d->qt[3][127] != 0;
        int contexts = d->contexts;
        if (d->version == 2) { /* the keyframe header's set (ffv1dec.c:845-858) */
            qt = (const int16_t(*)[256])d->qsets[s->qi];
            model1 = s->qi;
            contexts = d->ctx_count[s->qi];
        }
        d->sl[i].damaged |= crc_bad[i];
        if (d->version > 2) { /* decode_slice_header, ffv1dec.c:282-359 */
            uint8_t st[32];
            memset(st, 128, 32);
            int64_t W = d->cfg.width, H = d->cfg.height;
            int64_t sx = rc_get_symbol(&c, st, 0) * W, sy = rc_get_symbol(&c, st, 0) * H;
            int64_t sw = (rc_get_symbol(&c, st, 0) + 1) * W + sx;
            int64_t sh = (rc_get_symbol(&c, st, 0) + 1) * H + sy;
            sx /= d->num_h;
            sy /= d->num_v;
            sw = sw / d->num_h - sx;
            sh = sh / d->num_v - sy;
            int ok = (uint32_t)sw <= W && (uint32_t)sh <= H && (uint32_t)sx + (uint64_t)(uint32_t)sw <= (uint64_t)W &&
                     (uint32_t)sy + (uint64_t)(uint32_t)sh <= (uint64_t)H;
            int qi = 0;
            for (int j = 0; ok && j < d->plane_count; j++) {
                unsigned idx = (unsigned)rc_get_symbol(&c, st, 0);
                ok = idx < 2;
                qi = (int)idx; /* plane 0 and plane 1 read their own index; ours agree */
            }
            if (!ok) { /* ffv1dec.c:410-414: no decode, an empty rectangle */
                s->x0 = s->y0 = s->w = s->h = 0;
                s->damaged = 1;
                continue;
            }
            s->x0 = (int)sx; s->y0 = (int)sy; s->w = (int)sw; s->h = (int)sh;
            (void)rc_get_symbol(&c, st, 0); /* picture structure */
            (void)rc_get_symbol(&c, st, 0);
            (void)rc_get_symbol(&c, st, 0);
            s->pcm = 0;
            s->rct_by = s->rct_ry = 1;
            reset = 0;
            if (d->version > 3) { /* ffv1dec.c:344-356 */
                reset = rc_get(&c, &st[0]);
                s->pcm = rc_get_symbol(&c, st, 0);
                if (s->pcm != 1) {
                    s->rct_by = rc_get_symbol(&c, st, 0);
                    s->rct_ry = rc_get_symbol(&c, st, 0);
                    if ((uint64_t)(uint32_t)s->rct_by + (uint64_t)(uint32_t)s->rct_ry > 4) {
                        s->x0 = s->y0 = s->w = s->h = 0;
                        s->damaged = 1;
                        continue;
                    }
                }
            }
            qt = (const int16_t(*)[256])d->qsets[qi];
            model1 = qi;
            contexts = d->ctx_count[qi];
        }
        if (key || reset) /* ffv1dec.c:414-415 */
            for (int pp = 0; pp < d->plane_count; pp++) {
                if (d->version > 1 && d->init_states[model1]) /* ffv1.c:181-190 */
                    memcpy(s->ps[pp].rac, d->init_states[model1], (size_t)contexts * 32);
                else
                    memset(s->ps[pp].rac, 128, (size_t)contexts * 32);
                for (int j = 0; j < contexts; j++)
                    vlc_reset(&s->ps[pp].vlc[j]);
            }
        bitr b;
        void *coder = &c;
        int golomb = d->ac == 0;
        if (golomb) {
            int64_t acb = 0;
            if (d->version > 2) {
                uint8_t st = 129;
                (void)rc_get(&c, &st);
            }
            if (d->version > 2 || (s->x0 == 0 && s->y0 == 0))
                acb = (c.ptr - c.base) - 1;
            int64_t blen = (i == 0 ? lens[0] : lens[i]) - acb;
            b.base = c.base + acb;
            b.pos = 0;
            b.nbits = blen * 8;
            coder = &b;
        }
        d->cur_pcm = s->pcm;
        if (d->colorspace) {
            decode_rgb_slice(d, coder, golomb, s, qt, model1, planes, strides);
        } else if (d->chroma_planes || !d->transparency) { /* ffv1dec.c:437-449 */
            int np = d->chroma_planes ? 3 : 1;
            for (int pl = 0; pl < np; pl++) {
                int x0 = s->x0, y0 = s->y0, w = s->w, h = s->h;
                if (pl) {
                    w = ceil_rshift(s->w, d->hs);
                    h = ceil_rshift(s->h, d->vs);
                    x0 = s->x0 >> d->hs;
                    y0 = s->y0 >> d->vs;
                }
                decode_plane_any(d, coder, golomb, &s->ps[pl ? 1 : 0], qt, model1,
                                 w, h, planes[pl], strides[pl], x0, y0, 1);
            }
            if (d->transparency)
                decode_plane_any(d, coder, golomb, &s->ps[d->version >= 4 && !d->chroma_planes ? 1 : 2], qt,
                                 model1, s->w, s->h, planes[3], strides[3], s->x0, s->y0, 1);
        } else { /* YA8, ffv1dec.c:450-453 */
            for (int pl = 0; pl < 2; pl++)
                decode_plane_any(d, coder, golomb, &s->ps[pl], qt, model1, s->w, s->h, planes[0] + pl,
                                 strides[0], s->x0, s->y0, 2);
        }
        if (!golomb && d->version > 2) { /* ffv1dec.c:461-467 */
            uint8_t st = 129;
            (void)rc_get(&c, &st);
            if (c.end - c.ptr - 2 - 5 * d->ec)
                s->damaged = 1;
        }
    }

    /* concealment (ffv1dec.c:998-1021): a damaged slice's rectangle comes
     * from the previous picture; the x offset is in samples << (depth > 8),
     * which for packed bgr0 / RGB32 / YA8 is x bytes (not 4x / 2x) */
    int row[4], rows[4], step[4];
    int np = out_planes(d, row, rows, step);
    for (int i = n - 1; i >= 0 && d->have_last; i--) {
        dslice *s = &d->sl[i];
        if (!s->damaged || !s->w || !s->h)
            continue;
        for (int k = 0; k < np; k++) {
            int hs = k == 1 || k == 2 ? d->cfg.chroma_h_shift : 0, vs = k == 1 || k == 2 ? d->cfg.chroma_v_shift : 0;
            int pix = d->cfg.sample_bytes == 2;
            int bpp = step[k];
            int64_t xoff = (int64_t)(s->x0 >> hs) << pix;
            int64_t bytes = (int64_t)ceil_rshift(s->w, hs) * bpp;
            for (int y = 0; y < ceil_rshift(s->h, vs); y++) {
                int64_t yy = (s->y0 >> vs) + y;
                memcpy(planes[k] + yy * strides[k] + xoff,
                       d->last[k] + yy * d->last_row[k] + xoff, (size_t)bytes);
            }
        }
    }
    for (int k = 0; k < np; k++) {
        if (!d->last[k]) {
            d->last[k] = malloc((size_t)row[k] * rows[k] + 16);
            d->last_row[k] = row[k];
            d->last_rows[k] = rows[k];
        }
        for (int y = 0; y < rows[k]; y++)
            memcpy(d->last[k] + (int64_t)y * row[k], planes[k] + (int64_t)y * strides[k], (size_t)row[k]);
    }
    d->have_last = 1;
    if (key_out)
        *key_out = key;
    return 0;
}

/* sort_stt on caller-given counts and table (a host-only check of the
 * FFSWAP(int, ...) truncation, tests/test_twopass_host.py). */
void ffv1o_sort_stt(uint64_t rc_stat[512], uint8_t stt[256])
{
    sort_stt((uint64_t(*)[2])rc_stat, stt);
}
