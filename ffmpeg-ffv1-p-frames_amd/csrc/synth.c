/*
 * synth.c -- deterministic synthetic clips for the FFV1 encode path.
 *
 * "D1" is the reference's own FATE/benchmark source: the moving-gradient +
 * noise-block + moving-objects clip of tests/videogen.c:30-150 rendered in
 * RGB and converted with tests/utils.c:37-100 (rgb24 -> yuv420p).  The
 * generator below re-derives that clip from its description (integer only,
 * bit-exact), so the GPU box can build the same input without the
 * reference tree.  Frames are produced in order because the object
 * positions random-walk from frame to frame.
 *
 * Depth conversions match swscale's unscaled limited-range path used by the
 * reference benchmark commands (libswscale/swscale_unscaled.c:1421-1465:
 * "shiftonly" => v << (depth - 8)).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct vg_obj {
    int x, y, w, h;
    int r, g, b;
} vg_obj;

typedef struct ffv1syn_clip {
    int w, h;
    int frame;
    uint32_t seed;
    vg_obj obj[10];
    uint8_t *rgb;
} ffv1syn_clip;

/* LCG of tests/videogen.c:30-43 */
static unsigned vg_rand(uint32_t *s, int n)
{
    *s = *s * 314159u + 1u;
    return n == 256 ? (*s >> 24) : (*s % (unsigned)n);
}

/* 1 - x^2 cosine approximation, 8 fractional bits (videogen.c:52-66) */
static int vg_cos(int a)
{
    a &= 255;
    if (a >= 128)
        a = 256 - a;
    int flip = a > 64;
    if (flip)
        a = 128 - a;
    int v = 256 - ((a * a) >> 4);
    return flip ? -v : v;
}

static void vg_plot(ffv1syn_clip *c, int x, int y, int r, int g, int b)
{
    if (x < 0 || y < 0 || x >= c->w || y >= c->h)
        return;
    uint8_t *p = c->rgb + ((size_t)y * c->w + x) * 3;
    p[0] = (uint8_t)r;
    p[1] = (uint8_t)g;
    p[2] = (uint8_t)b;
}

ffv1syn_clip *ffv1syn_clip_new(int w, int h)
{
    if (w < 2 || h < 2 || (w & 1) || (h & 1))
        return NULL;
    ffv1syn_clip *c = calloc(1, sizeof(*c));
    if (!c)
        return NULL;
    c->w = w;
    c->h = h;
    c->seed = 1;
    c->rgb = malloc((size_t)w * h * 3);
    if (!c->rgb) {
        free(c);
        return NULL;
    }
    return c;
}

void ffv1syn_clip_free(ffv1syn_clip *c)
{
    if (c) {
        free(c->rgb);
        free(c);
    }
}

static void init_objects(ffv1syn_clip *c)
{
    const int w = c->w, h = c->h;
    for (int i = 0; i < 10; i++) {
            vg_obj *o = &c->obj[i];
            o->x = vg_rand(&c->seed, w);
            o->y = vg_rand(&c->seed, h);
            o->w = vg_rand(&c->seed, w / 4) + 10;
            o->h = vg_rand(&c->seed, h / 4) + 10;
            o->r = vg_rand(&c->seed, 256);
            o->g = vg_rand(&c->seed, 256);
            o->b = vg_rand(&c->seed, 256);
    }
}

/* the objects' random walk after frame c->frame is drawn */
static void move_objects(ffv1syn_clip *c)
{
    for (int i = 0; i < 10; i++) {
        c->obj[i].x += (int)vg_rand(&c->seed, 21) - 10;
        c->obj[i].y += (int)vg_rand(&c->seed, 21) - 10;
    }
}

static void render(ffv1syn_clip *c)
{
    const int num = c->frame, w = c->w, h = c->h;
    if (num == 0)
        init_objects(c);

    /* panning gradient background */
    const int dx = vg_cos(num * 256 / 50) * 35;
    const int dy = vg_cos(num * 256 / 50 + 256 / 10) * 30;
    for (int y = 0; y < h; y++) {
        const int yy = (y << 8) + dy;
        uint8_t *p = c->rgb + (size_t)y * w * 3;
        for (int x = 0; x < w; x++) {
            const int xx = (x << 8) + dx;
            p[3 * x + 0] = (uint8_t)((yy * 7) >> 8);
            p[3 * x + 1] = (uint8_t)(((xx + yy) * 9) >> 8);
            p[3 * x + 2] = (uint8_t)((xx * 5) >> 8);
        }
    }

    /* 26x26 full-range noise block at (10,30) */
    uint32_t s = (uint32_t)num;
    for (int y = 0; y < 26; y++)
        for (int x = 0; x < 26; x++) {
            int r = vg_rand(&s, 256), g = vg_rand(&s, 256), b = vg_rand(&s, 256);
            vg_plot(c, x + 10, y + 30, r, g, b);
        }

    /* ten noisy rectangles random-walking across the frame */
    for (int i = 0; i < 10; i++) {
        vg_obj *o = &c->obj[i];
        s = (uint32_t)i;
        for (int y = 0; y < o->h; y++)
            for (int x = 0; x < o->w; x++) {
                int r = o->r + vg_rand(&s, 50);
                int g = o->g + vg_rand(&s, 50);
                int b = o->b + vg_rand(&s, 50);
                vg_plot(c, x + o->x, y + o->y, r, g, b);
            }
    }
    move_objects(c);
}

/* BT.601 8-bit fixed point (FIX(x) = x * 256 rounded), 2x2 chroma average */
static void rgb_to_yuv420(const uint8_t *rgb, int w, int h, uint8_t *Y, uint8_t *U, uint8_t *V)
{
    for (int y = 0; y < h; y += 2)
        for (int x = 0; x < w; x += 2) {
            int rs = 0, gs = 0, bs = 0;
            for (int k = 0; k < 4; k++) {
                int px = x + (k & 1), py = y + (k >> 1);
                const uint8_t *p = rgb + ((size_t)py * w + px) * 3;
                int r = p[0], g = p[1], b = p[2];
                Y[(size_t)py * w + px] = (uint8_t)((77 * r + 150 * g + 29 * b + 128) >> 8);
                rs += r;
                gs += g;
                bs += b;
            }
            size_t ci = (size_t)(y / 2) * (w / 2) + x / 2;
            U[ci] = (uint8_t)(((-43 * rs - 85 * gs + 128 * bs + 511) >> 10) + 128);
            V[ci] = (uint8_t)(((128 * rs - 107 * gs - 21 * bs + 511) >> 10) + 128);
        }
}

/* Next frame as planar yuv420p (w*h*3/2 bytes). */
int ffv1syn_clip_next(ffv1syn_clip *c, uint8_t *out)
{
    render(c);
    const size_t n = (size_t)c->w * c->h;
    rgb_to_yuv420(c->rgb, c->w, c->h, out, out + n, out + n + n / 4);
    c->frame++;
    return c->frame - 1;
}

/*
 * "vsynth2": the reference's rotozoom clip (tests/rotozoom.c:28-195), a
 * 256x256 RGB picture (tests/reference.pnm, committed as a test fixture)
 * rotated and zoomed about the frame centre, bilinearly sampled with
 * wrap-around, in 16.16 fixed point.  The sine is a 7th-order Taylor series
 * on a folded angle; the interpolation products are taken mod 2^32 (the
 * reference computes them in int and keeps the low 8 bits of the result).
 */
#define RZ_ONE (1 << 16)
#define RZ_PI 205887 /* pi in 16.16 */

typedef struct ffv1syn_roto {
    int w, h;
    int frame;
    int hcos[360], hsin[360];
    uint8_t *rgb;
    uint8_t tab[3][256 * 256]; /* r, g, b planes of the source picture */
} ffv1syn_roto;

static int64_t rz_pow(int64_t a, int p)
{
    int64_t v = RZ_ONE;
    while (p-- > 0)
        v = v * a / RZ_ONE;
    return v;
}

static int64_t rz_sin(int64_t a)
{
    if (a < 0)
        a = RZ_PI - a;
    a %= 2 * RZ_PI;
    if (a >= RZ_PI * 3 / 2)
        a -= 2 * RZ_PI;
    if (a >= RZ_PI / 2)
        a = RZ_PI - a;
    return a - rz_pow(a, 3) / 6 + rz_pow(a, 5) / 120 - rz_pow(a, 7) / 5040;
}

/* src: the picture's 256x256 RGB24 samples (the PNM payload after its
 * 15-byte header). */
ffv1syn_roto *ffv1syn_roto_new(const uint8_t *src, int w, int h)
{
    if (w < 2 || h < 2 || (w & 1) || (h & 1))
        return NULL;
    ffv1syn_roto *r = calloc(1, sizeof(*r));
    if (!r)
        return NULL;
    r->rgb = malloc((size_t)w * h * 3);
    if (!r->rgb) {
        free(r);
        return NULL;
    }
    r->w = w;
    r->h = h;
    for (int i = 0; i < 256 * 256; i++)
        for (int k = 0; k < 3; k++)
            r->tab[k][i] = src[3 * i + k];
    for (int i = 0; i < 360; i++) {
        const int ang = 2 * i * RZ_PI / 360;
        const int amp = (int)(2 * RZ_ONE + rz_sin(ang));
        r->hcos[i] = (int)(amp * rz_sin(ang + RZ_PI / 2) / 2 / RZ_ONE);
        r->hsin[i] = (int)(amp * rz_sin(ang) / 2 / RZ_ONE);
    }
    return r;
}

void ffv1syn_roto_free(ffv1syn_roto *r)
{
    if (r) {
        free(r->rgb);
        free(r);
    }
}

static uint8_t rz_sample(const uint8_t *t, int x, int y)
{
    const int ix = x >> 16, iy = y >> 16;
    const uint32_t fx = x & 0xFFFF, fy = y & 0xFFFF;
    const uint32_t a = t[(ix & 255) + 256 * (iy & 255)];
    const uint32_t b = t[((ix + 1) & 255) + 256 * (iy & 255)];
    const uint32_t c = t[(ix & 255) + 256 * ((iy + 1) & 255)];
    const uint32_t d = t[((ix + 1) & 255) + 256 * ((iy + 1) & 255)];
    const uint32_t top = ((RZ_ONE - fx) * a + fx * b) >> 8;
    const uint32_t bot = ((RZ_ONE - fx) * c + fx * d) >> 8;
    return (uint8_t)(((RZ_ONE - fy) * top + fy * bot) >> 24);
}

int ffv1syn_roto_next(ffv1syn_roto *r, uint8_t *out)
{
    const int w = r->w, h = r->h, num = r->frame;
    const int c = r->hcos[num % 360], s = r->hsin[num % 360];
    /* the frame's top-left corner in source coordinates, rows stepped by
     * (s, c), columns by (c, -s) */
    int row_x = -(h / 2) * s - (w / 2) * c + RZ_ONE * w / 2;
    int row_y = -(h / 2) * c + (w / 2) * s + RZ_ONE * h / 2;
    for (int j = 0; j < h; j++) {
        int x = row_x, y = row_y;
        uint8_t *p = r->rgb + (size_t)j * w * 3;
        for (int i = 0; i < w; i++) {
            x += c;
            y -= s;
            for (int k = 0; k < 3; k++)
                p[3 * i + k] = rz_sample(r->tab[k], x, y);
        }
        row_x += s;
        row_y += c;
    }
    const size_t n = (size_t)w * h;
    rgb_to_yuv420(r->rgb, w, h, out, out + n, out + n + n / 4);
    r->frame++;
    return num;
}

/* Advance past the next frame without drawing it (the clip's only state
 * across frames is the objects' random walk). */
void ffv1syn_clip_skip(ffv1syn_clip *c)
{
    if (c->frame == 0)
        init_objects(c);
    move_objects(c);
    c->frame++;
}

/* u8 -> u16 little-endian, v << shift (shift = depth - 8). */
void ffv1syn_widen(const uint8_t *src, uint16_t *dst, int64_t n, int shift)
{
    for (int64_t i = 0; i < n; i++)
        dst[i] = (uint16_t)(src[i] << shift);
}
