/*
 * fake_lqr.c -- TEST DRIVER: the liblqr side of the energy callback contract.
 *
 * liblqr is not in this image, so this file restates the few pieces of it the
 * plug-in's callback touches [liblqr, unverified]: a reading window that
 * returns LQR_ER_LUMA values relative to the pixel being evaluated
 * (lqr_rwindow_get_radius / lqr_rwindow_read, as used at src/render.c:144,150)
 * and the energy build loop (rows outer, columns inner, one callback per
 * pixel).  The callback is the PATCHED dct_pixel_energy of INTEGRATION.md:
 * served from the GPU map (dcte_plugin.c) when the carver still has the
 * frame's size, else the reference's per-window code -- played here by the
 * oracle's window transform (test infrastructure).
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "dcte_plugin.h"
#include "dctenergy.h"

typedef struct {
    const double *luma; /* current carver image, w x h */
    int w, h, x, y, radius;
} LqrReadingWindow;

static int lqr_rwindow_get_radius(LqrReadingWindow *rw) { return rw->radius; }
static double lqr_rwindow_read(LqrReadingWindow *rw, int dx, int dy, int ch)
{
    (void)ch;
    return rw->luma[(size_t)(rw->y + dy) * rw->w + (rw->x + dx)];
}

/* the reference's EnergyParameters (src/render.h:9-16) + the patch's cache */
typedef struct {
    float edges, textures;
    int blocksize;
    double d[256];       /* params->data: the gathered window, data[dx][dy] */
    double *rows[16];    /* its row pointers (alloc_2d_double layout) */
    dcte_map_cache gpu;
} EnergyParameters;

static void params_init(EnergyParameters *p, float edges, float textures, int n)
{
    memset(p, 0, sizeof(*p));
    p->edges = edges;
    p->textures = textures;
    p->blocksize = n;
    for (int i = 0; i < n; i++) p->rows[i] = p->d + i * n;
}

float orc_window_energy(int n, const double *win, float edges, float textures); /* oracle */
int orc_seam_find(const float *E, long long stride, int w, int h, int *seam, float *M); /* oracle */

static long long g_fallback_calls, g_served_map, g_verified, g_bad;
static int g_verify;      /* re-run the original body on every hook-served callback */

static int clamp_offset_to_border(int base, int offset, int lo, int hi)
{
    if (base + offset - lo < 0) return offset - (base + offset - lo);
    if (base + offset - hi > 0) return offset - (base + offset - hi);
    return offset;
}

/* the reference callback body (src/render.c:134-157), first half: the gather */
static void gather_window(int x, int y, int w, int h, LqrReadingWindow *rw, EnergyParameters *p)
{
    int r = lqr_rwindow_get_radius(rw);
    for (int i = -r + 1; i <= r; i++)
        for (int j = -r + 1; j <= r; j++) {
            int ii = clamp_offset_to_border(x, i, 0, w - 1);
            int jj = clamp_offset_to_border(y, j, 0, h - 1);
            p->rows[i + r - 1][j + r - 1] = lqr_rwindow_read(rw, ii, jj, 0);
        }
}

/* second half: dctNxN + weighted_max_dct_correlation (the oracle plays them) */
static float window_energy(const EnergyParameters *p)
{
    return orc_window_energy(p->blocksize, p->d, p->edges, p->textures);
}

static float original_dct_pixel_energy(int x, int y, int w, int h, LqrReadingWindow *rw, void *extra)
{
    EnergyParameters *p = (EnergyParameters *)extra;
    gather_window(x, y, w, h, rw, p);
    g_fallback_calls++;
    return window_energy(p);
}

/* the patch's adapter: the hook reads liblqr's image
 * through the callback's reading window */
static double rwindow_read(void *rw, int dx, int dy)
{
    return lqr_rwindow_read((LqrReadingWindow *)rw, dx, dy, 0);
}

static int g_orientation; /* lqr_carver_get_orientation of the fake carver */
static int g_use_hook;    /* the plug-in was built with DCTE_PLUGIN_SEAM_HOOK */

/* the PATCHED callback */
static float dct_pixel_energy(int x, int y, int w, int h, LqrReadingWindow *rw, void *extra)
{
    EnergyParameters *p = (EnergyParameters *)extra;
    float v;
    if (dcte_plugin_lookup(&p->gpu, x, y, w, h, g_orientation, &v)) {
        g_served_map++;
        return v;
    }
    if (g_use_hook && dcte_plugin_lookup_hook(&p->gpu, x, y, w, h, g_orientation, rwindow_read, rw, &v)) {
        if (g_verify) {  /* test mode: what the original body returns for this window */
            gather_window(x, y, w, h, rw, p);
            const float ref = window_energy(p);
            g_verified++;
            if (!(fabsf(v - ref) <= 1e-5f * fabsf(ref) + 1e-9f)) g_bad++;
        }
        return v;
    }
    return original_dct_pixel_energy(x, y, w, h, rw, extra);
}

/* Carver built on px (w x h, bpp), energy function registered with radius
 * n/2; then `removed` columns are dropped from the right (as if seams had
 * been carved) and the energy is rebuilt on the narrower carver.  out holds
 * the (w - removed) x h energies of that last build.  transposed: the carver
 * is transposed first (vertical resize: liblqr evaluates the energy on the
 * transposed raw map, orientation 1); out is then h x (w - removed)... of the
 * transposed frame: (w - removed) rows of h. */
int fake_build_emap(const uint8_t *px, int w, int h, int bpp, int n, float edges, float textures,
                    int use_gpu, int removed, int transposed, float *out,
                    long long *fallback_calls, int *gpu_status)
{
    double *luma = (double *)malloc(sizeof(double) * (size_t)w * h);
    if (!luma) return -3;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const uint8_t *q = px + ((size_t)y * w + x) * bpp;
            luma[(size_t)y * w + x] = bpp == 1 ? (double)q[0] / 255
                : 0.2126 * ((double)q[0] / 255) + 0.7152 * ((double)q[1] / 255) + 0.0722 * ((double)q[2] / 255);
        }
    EnergyParameters p;
    params_init(&p, edges, textures, n);
    *gpu_status = use_gpu ? dcte_plugin_build(&p.gpu, px, w, h, bpp, (size_t)w * bpp, n, edges,
                                              textures, transposed)
                          : DCTE_ENODEV;
    /* the carver's current raw map: optionally transposed, then narrowed */
    int fw = transposed ? h : w, fh = transposed ? w : h;
    double *fr = luma;
    if (transposed) {
        fr = (double *)malloc(sizeof(double) * (size_t)w * h);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) fr[(size_t)x * h + y] = luma[(size_t)y * w + x];
    }
    int cw = fw - removed;
    double *cur = fr;
    if (removed) {
        cur = (double *)malloc(sizeof(double) * (size_t)cw * fh);
        for (int y = 0; y < fh; y++)
            for (int x = 0; x < cw; x++) cur[(size_t)y * cw + x] = fr[(size_t)y * fw + x];
    }
    g_fallback_calls = g_served_map = 0;
    g_orientation = transposed;
    LqrReadingWindow rw = {cur, cw, fh, 0, 0, n / 2};
    for (int y = 0; y < fh; y++)
        for (int x = 0; x < cw; x++) {
            rw.x = x;
            rw.y = y;
            out[(size_t)y * cw + x] = dct_pixel_energy(x, y, cw, fh, &rw, &p);
        }
    *fallback_calls = g_fallback_calls;
    dcte_plugin_release(&p.gpu);
    if (cur != fr) free(cur);
    if (fr != luma) free(fr);
    free(luma);
    return 0;
}

/* A DP that breaks ties the other way: the same recursion as orc_seam_find
 * (oracle/dcte_oracle.c), but the RIGHTMOST minimum wins among the parent
 * candidates and in the last row.  Stands in for a liblqr whose seam differs
 * from the mirror's on equal energies. */
static void seam_find_rightmost(const float *E, int w, int h, int *seam)
{
    float *prev = (float *)malloc(sizeof(float) * (size_t)w), *cur = (float *)malloc(sizeof(float) * (size_t)w);
    signed char *par = (signed char *)malloc((size_t)w * h);
    for (int x = 0; x < w; x++) prev[x] = E[x];
    for (int y = 1; y < h; y++) {
        for (int x = 0; x < w; x++) {
            int lo = x > 0 ? x - 1 : 0, hi = x < w - 1 ? x + 1 : w - 1, arg = lo;
            for (int c = lo + 1; c <= hi; c++)
                if (prev[c] <= prev[arg]) arg = c;
            cur[x] = E[(size_t)y * w + x] + prev[arg];
            par[(size_t)y * w + x] = (signed char)(arg - x);
        }
        float *t = prev;
        prev = cur;
        cur = t;
    }
    int x = 0;
    for (int c = 1; c < w; c++)
        if (prev[c] <= prev[x]) x = c;
    seam[h - 1] = x;
    for (int y = h - 1; y > 0; y--) {
        x += par[(size_t)y * w + x];
        seam[y - 1] = x;
    }
    free(prev);
    free(cur);
    free(par);
}

/* Shift the seam by one column in one row (the first row from the middle
 * down where the seam stays connected and inside the frame). */
static void seam_shift_one_row(int *s, int w, int h)
{
    for (int k = 0; k < h; k++) {
        const int y = (h / 2 + k) % h;
        for (int d = 1; d >= -1; d -= 2) {
            const int v = s[y] + d;
            if (v < 0 || v >= w) continue;
            if (y > 0 && abs(v - s[y - 1]) > 1) continue;
            if (y < h - 1 && abs(v - s[y + 1]) > 1) continue;
            s[y] = v;
            return;
        }
    }
}

/* Self-test of the hook's window check on the host (no device): a synthetic
 * cache over a random w x h luma frame with a band around a fixed seam, the
 * update pixels visited in liblqr's order (rows outer, columns inner).
 * Returns 0 when (1) every window matches, with fewer than 3 reads per
 * callback on average (each pixel read once); (2) with any one pixel of the
 * region moved by one 8-bit luma step, the first window holding it -- and no
 * earlier one -- is rejected (-1); (3) a window past the band misses (0);
 * else the failing case's code. */
typedef struct {
    int w, h, n, bpp, bw;
    int *x0, *a, *b;        /* band start per row; update columns [a, b] per row */
    unsigned char *bpx;
    double *luma;
} SelfTest;

static void selftest_reset(dcte_map_cache *c, const SelfTest *t, int *lo, int *hi)
{
    memset(c, 0, sizeof(*c));
    c->n = t->n;
    c->mw = t->w;
    c->mh = t->h;
    c->bpp = t->bpp;
    c->bw = t->bw;
    c->band_valid = 1;
    c->band_x0 = t->x0;
    c->band_px = t->bpx;
    for (int y = 0; y < t->h; y++) {
        lo[y] = 1;
        hi[y] = 0;
    }
    c->ver_lo = lo;
    c->ver_hi = hi;
}

int fake_window_check_selftest(int n, int bpp, unsigned seed)
{
    SelfTest t;
    t.w = 61;
    t.h = 23;
    t.n = n;
    t.bpp = bpp;
    const int w = t.w, h = t.h, r = n / 2, bw = t.bw = 8 * r + 4;
    unsigned char *px = (unsigned char *)malloc((size_t)w * h * bpp);
    t.luma = (double *)malloc(sizeof(double) * (size_t)w * h);
    t.x0 = (int *)malloc(sizeof(int) * h);
    t.a = (int *)malloc(sizeof(int) * h);
    t.b = (int *)malloc(sizeof(int) * h);
    t.bpx = (unsigned char *)malloc((size_t)h * bw * bpp);
    int *lo = (int *)malloc(sizeof(int) * h), *hi = (int *)malloc(sizeof(int) * h);
    int rc = 0;
    for (size_t i = 0; i < (size_t)w * h * bpp; i++) {
        seed = seed * 1664525u + 1013904223u;
        px[i] = (unsigned char)(seed >> 24);
    }
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const unsigned char *q = px + ((size_t)y * w + x) * bpp;
            t.luma[(size_t)y * w + x] = bpp == 1 ? (double)q[0] / 255
                : 0.2126 * ((double)q[0] / 255) + 0.7152 * ((double)q[1] / 255) + 0.0722 * ((double)q[2] / 255);
        }
    /* a seam wandering around column 30; band rows as dcte_band_gather builds
     * them, update columns as fake_resize's update_emap */
    int s[23];
    for (int y = 0; y < h; y++) s[y] = 30 + (y % 5 < 3 ? y % 5 : 5 - y % 5);
    for (int y = 0; y < h; y++) {
        int m = w;
        for (int j = -2 * r; j <= 2 * r; j++) {
            const int yy = y + j < 0 ? 0 : y + j >= h ? h - 1 : y + j;
            if (s[yy] < m) m = s[yy];
        }
        int a = m - 2 * r - 1, mx = w - bw > 0 ? w - bw : 0;
        t.x0[y] = a < 0 ? 0 : a > mx ? mx : a;
        for (int k = 0; k < bw; k++) {
            const int x = t.x0[y] + k < w - 1 ? t.x0[y] + k : w - 1;
            memcpy(t.bpx + ((size_t)y * bw + k) * bpp, px + ((size_t)y * w + x) * bpp, bpp);
        }
        t.a[y] = w;
        t.b[y] = -1;
        for (int y1 = y - r; y1 <= y + r; y1++) {
            if (y1 < 0 || y1 >= h) continue;
            if (s[y1] - r < t.a[y]) t.a[y] = s[y1] - r;
            if (s[y1] + r - 1 > t.b[y]) t.b[y] = s[y1] + r - 1;
        }
        if (t.a[y] < 0) t.a[y] = 0;
        if (t.b[y] > w - 1) t.b[y] = w - 1;
    }
    dcte_map_cache c;
    LqrReadingWindow rw = {t.luma, w, h, 0, 0, r};
    /* (1) */
    selftest_reset(&c, &t, lo, hi);
    long long calls = 0;
    for (int y = 0; y < h && !rc; y++)
        for (int x = t.a[y]; x <= t.b[y] && !rc; x++) {
            rw.x = x;
            rw.y = y;
            if (dcte_plugin_window_check(&c, x, y, w, h, rwindow_read, &rw) != 1) rc = 1;
            calls++;
        }
    if (!rc && (calls == 0 || c.reads > 3 * calls)) rc = 4;
    /* (2): every 5th pixel of the update windows' union */
    for (int py = 0; py < h && !rc; py++)
        for (int px0 = 0; px0 < w && !rc; px0 += 5) {
            int first_y = -1, first_x = -1;   /* the first callback whose window holds it */
            for (int y = 0; y < h && first_y < 0; y++)
                for (int x = t.a[y]; x <= t.b[y]; x++)
                    if (px0 >= x - r + 1 && px0 <= x + r && py >= y - r + 1 && py <= y + r) {
                        first_y = y;
                        first_x = x;
                        break;
                    }
            if (first_y < 0) continue;
            const double keep = t.luma[(size_t)py * w + px0];
            t.luma[(size_t)py * w + px0] = keep + (bpp == 1 ? 1.0 / 255 : 0.0722 / 255);
            selftest_reset(&c, &t, lo, hi);
            int got = 1, at_y = -1, at_x = -1;
            for (int y = 0; y < h && got == 1; y++)
                for (int x = t.a[y]; x <= t.b[y] && got == 1; x++) {
                    rw.x = x;
                    rw.y = y;
                    got = dcte_plugin_window_check(&c, x, y, w, h, rwindow_read, &rw);
                    at_y = y;
                    at_x = x;
                }
            if (got != -1 || at_y != first_y || at_x != first_x) rc = 2;
            t.luma[(size_t)py * w + px0] = keep;
        }
    /* (3) a pixel far left of the band: its window leaves it */
    if (!rc && t.x0[h / 2] > 0) {
        selftest_reset(&c, &t, lo, hi);
        rw.x = 0;
        rw.y = h / 2;
        if (dcte_plugin_window_check(&c, 0, h / 2, w, h, rwindow_read, &rw) != 0) rc = 3;
    }
    free(px);
    free(t.luma);
    free(t.x0);
    free(t.a);
    free(t.b);
    free(t.bpx);
    free(lo);
    free(hi);
    return rc;
}

/* liblqr's resize loop for the plug-in's carver (lqr_carver_resize,
 * src/render.c:377; carver set up with delta_x 1, rigidity 0 at
 * src/render.c:313) [liblqr, unverified]: the energy build (one callback per
 * pixel), then per seam
 *   - the cumulative-energy DP on the current energies (orc_seam_find: the
 *     restatement the device search is bit-identical to),
 *   - removal of the seam from the image and from the energy map,
 *   - update_emap: the callback re-evaluated around the seam -- for every
 *     row y1, columns [min s - r, max s + r - 1] over the seam rows y with
 *     |y - y1| <= r (r = the registered radius N/2), of the narrower image.
 * The plug-in is built on px as in init_carver_from_vals; `hook` selects the
 * patched callback with the seam hook (DCTE_PLUGIN_SEAM_HOOK).  Outputs: the
 * final energies (fh x cw), the final image bytes (fh x cw x bpp), the seams
 * (seams x fh) and counts[12] = {callbacks, fallback (original transform),
 * served from a map, served from a seam band, mirror steps, nanoseconds spent
 * in the update_emap callbacks (incl. the mirror's steps), hook-served values
 * re-checked against the original body (verify), of those off tolerance,
 * hook misses, hook still on at the end, window reads of the hook's check,
 * glue calls of the interleaved dialog that succeeded (fake_set_interleave)}.
 * transposed: vertical resize -- the carver works on the transposed frame.
 * diverge (tests of the hook's window check): 0 = liblqr follows the
 * mirror's rules; 1 = after the build liblqr's image differs slightly from
 * the frame the plug-in was given (+1e-3 luma); 2 = every seam liblqr carves
 * is shifted by one column in one row; 3 = liblqr's DP takes the rightmost
 * minimum on ties (seam_find_rightmost); 4 = after the first seam's update
 * liblqr's image changes (up to 1e-3 luma, varying along the row, so the AC
 * content changes) and it runs that update pass again at the SAME width (a
 * second callback pass over the same pixels, from row 0).
 * verify: re-run the original body on
 * every hook-served callback and count values off the parity tolerance. */
/* extra plug-in build flags for fake_resize (DCTE_PLUGIN_EXACT) */
static unsigned g_extra_flags;
void fake_set_plugin_flags(unsigned flags) { g_extra_flags = flags; }

/* The interactive dialog between the steps of a resize (src/interface.c:116,
 * 524, 662): the preview redraws and another carver is set up, each in the
 * DEFAULT (fast) mode, while the resize's own carver lives on.  With
 * fake_set_interleave(1), fake_resize does this after its build and after
 * every seam's update pass; the resize's energies must not change. */
static int g_interleave;
static long long g_interleaved;
void fake_set_interleave(int on) { g_interleave = on; }

static void dialog_interleave(const uint8_t *px, int w, int h, int bpp, int n, float edges,
                              float textures)
{
    dcte_map_cache other;
    if (dcte_plugin_build_ex(&other, px, w, h, bpp, (size_t)w * bpp, n, edges, textures, 1, 0u) ==
        DCTE_OK)
        g_interleaved++;
    dcte_plugin_release(&other);
    uint8_t *layer = (uint8_t *)malloc((size_t)w * h * bpp);
    if (layer && dcte_plugin_preview_u8(px, w, h, bpp, n, edges, textures, 0u, layer) == DCTE_OK)
        g_interleaved++;
    free(layer);
}

/* The PATCHED dct_energy_preview on a drawable of
 * dw x dh pixels with `channels` bytes each: the preview rectangle (x1, y1,
 * w, h) is read as gimp_pixel_rgn_get_rect hands it over (copied out of the
 * drawable, rows of w * channels bytes) and the glue draws the layer
 * (dcte_plugin_preview_u8); when the glue fails (no device) the original loop
 * runs -- dct_energy_preview_rows over the region (src/render.c:31-60, the
 * oracle plays it) and normalize_image (src/render.c:80-109, DOUBLE2GUCHAR
 * with GIMP's ROUND, src/render.h:6).  out: w * h * channels bytes.
 * *gpu_status = the glue's return code. */
int orc_preview_map_rows(const uint8_t *px, int w, int h, int bpp, size_t rowstride, int n,
                         float edges, float textures, int y0, int y1, int nthreads, float *out); /* oracle */

int fake_preview(const uint8_t *drawable, int dw, int dh, int channels, int x1, int y1, int w, int h,
                 int n, float edges, float textures, unsigned flags, uint8_t *out, int *gpu_status)
{
    if (x1 < 0 || y1 < 0 || w <= 0 || h <= 0 || x1 + w > dw || y1 + h > dh) return -1;
    uint8_t *region = (uint8_t *)malloc((size_t)w * h * channels);
    if (!region) return -3;
    for (int y = 0; y < h; y++)
        memcpy(region + (size_t)y * w * channels,
               drawable + ((size_t)(y1 + y) * dw + x1) * channels, (size_t)w * channels);
    *gpu_status = dcte_plugin_preview_u8(region, w, h, channels, n, edges, textures, flags, out);
    int rc = 0;
    if (*gpu_status != DCTE_OK) {
        float *E = (float *)malloc(sizeof(float) * (size_t)w * h);
        if (!E || orc_preview_map_rows(region, w, h, channels, (size_t)w * channels, n, edges,
                                       textures, 0, h, 1, E) != 0) {
            rc = -2;
        } else {
            double mn = E[0], mx = E[0];
            for (size_t i = 0; i < (size_t)w * h; i++) {
                if (E[i] > mx) mx = E[i];
                if (E[i] < mn) mn = E[i];
            }
            for (size_t i = 0; i < (size_t)w * h; i++) {
                /* (the reference divides by zero on a flat region; the guard
                 * draws 0 as the library does) */
                const uint8_t v = mx > mn ? (uint8_t)(int)(255 * (((double)E[i] - mn) / (mx - mn)) + 0.5) : 0;
                memset(out + i * channels, v, channels);
            }
        }
        free(E);
    }
    free(region);
    return rc;
}

int fake_resize(const uint8_t *px, int w, int h, int bpp, int n, float edges, float textures,
                int use_gpu, int hook, int seams, int transposed, int diverge, int verify,
                float *out_emap, uint8_t *out_px, int *out_seams, long long *counts, int *gpu_status)
{
    const int fw = transposed ? h : w, fh = transposed ? w : h;
    if (seams < 0 || seams >= fw) return -1;
    uint8_t *img = (uint8_t *)malloc((size_t)fw * fh * bpp);
    double *luma = (double *)malloc(sizeof(double) * (size_t)fw * fh);
    float *emap = (float *)malloc(sizeof(float) * (size_t)fw * fh);
    int *s = (int *)malloc(sizeof(int) * (size_t)fh);
    int *xmin = (int *)malloc(sizeof(int) * (size_t)fh), *xmax = (int *)malloc(sizeof(int) * (size_t)fh);
    if (!img || !luma || !emap || !s || !xmin || !xmax) return -3;
    for (int y = 0; y < fh; y++)
        for (int x = 0; x < fw; x++) {
            const uint8_t *q = transposed ? px + ((size_t)x * w + y) * bpp : px + ((size_t)y * w + x) * bpp;
            memcpy(img + ((size_t)y * fw + x) * bpp, q, bpp);
            luma[(size_t)y * fw + x] = bpp == 1 ? (double)q[0] / 255
                : 0.2126 * ((double)q[0] / 255) + 0.7152 * ((double)q[1] / 255) + 0.0722 * ((double)q[2] / 255);
        }
    EnergyParameters p;
    params_init(&p, edges, textures, n);
    *gpu_status = use_gpu ? dcte_plugin_build_ex(&p.gpu, px, w, h, bpp, (size_t)w * bpp, n, edges,
                                                 textures, transposed, (hook ? DCTE_PLUGIN_SEAM_HOOK : 0u) | g_extra_flags)
                          : DCTE_ENODEV;
    g_fallback_calls = g_served_map = g_verified = g_bad = g_interleaved = 0;
    g_orientation = transposed;
    g_use_hook = hook;
    g_verify = verify;
    if (g_interleave) dialog_interleave(px, w, h, bpp, n, edges, textures);
    long long calls = 0, update_ns = 0;
    int cw = fw;
    const int r = n / 2;
    LqrReadingWindow rw = {luma, cw, fh, 0, 0, r};
    for (int y = 0; y < fh; y++)
        for (int x = 0; x < cw; x++) {
            rw.x = x;
            rw.y = y;
            emap[(size_t)y * cw + x] = dct_pixel_energy(x, y, cw, fh, &rw, &p);
            calls++;
        }
    if (diverge == 1)
        for (size_t i = 0; i < (size_t)cw * fh; i++) luma[i] += 1e-3;
    for (int k = 0; k < seams; k++) {
        if (diverge == 3) seam_find_rightmost(emap, cw, fh, s);
        else orc_seam_find(emap, cw, cw, fh, s, NULL);
        if (diverge == 2) seam_shift_one_row(s, cw, fh);
        if (out_seams) memcpy(out_seams + (size_t)k * fh, s, sizeof(int) * (size_t)fh);
        /* carve: compact every row to cw - 1 (row stride follows the width) */
        for (int y = 0; y < fh; y++) {
            const size_t src = (size_t)y * cw, dst = (size_t)y * (cw - 1);
            for (int x = 0, o = 0; x < cw; x++) {
                if (x == s[y]) continue;
                luma[dst + o] = luma[src + x];
                emap[dst + o] = emap[src + x];
                memmove(img + (dst + o) * bpp, img + (src + x) * bpp, bpp);
                o++;
            }
        }
        cw--;
        /* update_emap */
        for (int y = 0; y < fh; y++) {
            xmin[y] = cw;
            xmax[y] = -1;
        }
        for (int y = 0; y < fh; y++)
            for (int y1 = y - r; y1 <= y + r; y1++) {
                if (y1 < 0 || y1 >= fh) continue;
                const int a = s[y] - r < 0 ? 0 : s[y] - r, b = s[y] + r - 1 > cw - 1 ? cw - 1 : s[y] + r - 1;
                if (a < xmin[y1]) xmin[y1] = a;
                if (b > xmax[y1]) xmax[y1] = b;
            }
        rw.w = cw;
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        for (int y = 0; y < fh; y++)
            for (int x = xmin[y]; x <= xmax[y]; x++) {
                rw.x = x;
                rw.y = y;
                emap[(size_t)y * cw + x] = dct_pixel_energy(x, y, cw, fh, &rw, &p);
                calls++;
            }
        clock_gettime(CLOCK_MONOTONIC, &t1);
        update_ns += (t1.tv_sec - t0.tv_sec) * 1000000000LL + (t1.tv_nsec - t0.tv_nsec);
        if (g_interleave) dialog_interleave(px, w, h, bpp, n, edges, textures);
        if (diverge == 4 && k == 0) {
            for (size_t i = 0; i < (size_t)cw * fh; i++) luma[i] += 1e-3 * (double)(i % 7) / 7.0;
            for (int y = 0; y < fh; y++)
                for (int x = xmin[y]; x <= xmax[y]; x++) {
                    rw.x = x;
                    rw.y = y;
                    emap[(size_t)y * cw + x] = dct_pixel_energy(x, y, cw, fh, &rw, &p);
                    calls++;
                }
        }
    }
    memcpy(out_emap, emap, sizeof(float) * (size_t)cw * fh);
    if (out_px) memcpy(out_px, img, (size_t)cw * fh * bpp);
    counts[0] = calls;
    counts[1] = g_fallback_calls;
    counts[2] = g_served_map;
    counts[3] = p.gpu.served_band;
    counts[4] = p.gpu.steps;
    counts[5] = update_ns;
    counts[6] = g_verified;
    counts[7] = g_bad;
    counts[8] = p.gpu.missed;
    counts[9] = p.gpu.hook_ok;
    counts[10] = p.gpu.reads;
    counts[11] = g_interleaved;
    dcte_plugin_release(&p.gpu);
    g_use_hook = g_verify = 0;
    free(img);
    free(luma);
    free(emap);
    free(s);
    free(xmin);
    free(xmax);
    return 0;
}
