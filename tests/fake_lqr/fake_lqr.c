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
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

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

/* the PATCHED callback */
static float dct_pixel_energy(int x, int y, int w, int h, LqrReadingWindow *rw, void *extra)
{
    EnergyParameters *p = (EnergyParameters *)extra;
    float v;
    if (dcte_plugin_lookup(&p->gpu, x, y, w, h, g_orientation, &v)) return v;
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
