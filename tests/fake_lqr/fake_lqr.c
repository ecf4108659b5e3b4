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
    dcte_map_cache gpu;
} EnergyParameters;

float orc_window_energy(int n, const double *win, float edges, float textures); /* oracle */
int orc_seam_find(const float *E, long long stride, int w, int h, int *seam, float *M); /* oracle */

static long long g_fallback_calls;

static int clamp_offset_to_border(int base, int offset, int lo, int hi)
{
    if (base + offset - lo < 0) return offset - (base + offset - lo);
    if (base + offset - hi > 0) return offset - (base + offset - hi);
    return offset;
}

/* the reference callback body (src/render.c:134-157) */
static float original_dct_pixel_energy(int x, int y, int w, int h, LqrReadingWindow *rw, void *extra)
{
    EnergyParameters *p = (EnergyParameters *)extra;
    int r = lqr_rwindow_get_radius(rw), n = p->blocksize;
    double d[256];
    for (int i = -r + 1; i <= r; i++)
        for (int j = -r + 1; j <= r; j++) {
            int ii = clamp_offset_to_border(x, i, 0, w - 1);
            int jj = clamp_offset_to_border(y, j, 0, h - 1);
            d[(i + r - 1) * n + (j + r - 1)] = lqr_rwindow_read(rw, ii, jj, 0);
        }
    g_fallback_calls++;
    return orc_window_energy(n, d, p->edges, p->textures);
}

static int g_orientation; /* lqr_carver_get_orientation of the fake carver */
static int g_use_hook;    /* the plug-in was built with DCTE_PLUGIN_SEAM_HOOK */

/* the PATCHED callback */
static float dct_pixel_energy(int x, int y, int w, int h, LqrReadingWindow *rw, void *extra)
{
    EnergyParameters *p = (EnergyParameters *)extra;
    float v;
    if (g_use_hook) {
        if (dcte_plugin_lookup_hook(&p->gpu, x, y, w, h, g_orientation, lqr_rwindow_read(rw, 0, 0, 0), &v))
            return v;
    } else if (dcte_plugin_lookup(&p->gpu, x, y, w, h, g_orientation, &v)) {
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
    EnergyParameters p = {edges, textures, n, {0}};
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
    g_fallback_calls = 0;
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
 * (seams x fh) and counts[6] = {callbacks, fallback (original code),
 * served from a map, served from a seam band, mirror steps, nanoseconds spent
 * in the update_emap callbacks (incl. the mirror's steps)}.
 * transposed: vertical resize -- the carver works on the transposed frame.
 * perturb (test of the hook's divergence check): after the build, liblqr's
 * image differs slightly from the frame the plug-in was given. */
int fake_resize(const uint8_t *px, int w, int h, int bpp, int n, float edges, float textures,
                int use_gpu, int hook, int seams, int transposed, int perturb, float *out_emap,
                uint8_t *out_px, int *out_seams, long long *counts, int *gpu_status)
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
    EnergyParameters p = {edges, textures, n, {0}};
    *gpu_status = use_gpu ? dcte_plugin_build_ex(&p.gpu, px, w, h, bpp, (size_t)w * bpp, n, edges,
                                                 textures, transposed, hook ? DCTE_PLUGIN_SEAM_HOOK : 0u)
                          : DCTE_ENODEV;
    g_fallback_calls = 0;
    g_orientation = transposed;
    g_use_hook = hook;
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
    if (perturb)
        for (size_t i = 0; i < (size_t)cw * fh; i++) luma[i] += 1e-3;
    for (int k = 0; k < seams; k++) {
        orc_seam_find(emap, cw, cw, fh, s, NULL);
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
    }
    memcpy(out_emap, emap, sizeof(float) * (size_t)cw * fh);
    if (out_px) memcpy(out_px, img, (size_t)cw * fh * bpp);
    counts[0] = calls;
    counts[1] = g_fallback_calls;
    counts[2] = p.gpu.served_map;
    counts[3] = p.gpu.served_band;
    counts[4] = p.gpu.steps;
    counts[5] = update_ns;
    dcte_plugin_release(&p.gpu);
    g_use_hook = 0;
    free(img);
    free(luma);
    free(emap);
    free(s);
    free(xmin);
    free(xmax);
    return 0;
}
