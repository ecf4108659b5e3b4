/* dcte_plugin.c -- see dcte_plugin.h.  One process-wide dcte_ctx, created on
 * first use over DCTE_NGPUS devices (unset = 1 device, 0 = all visible),
 * destroyed at exit.  One device by default: a GIMP frame fits one MI355X many
 * times over, and the single-device path is the one the GPU tests run. */
#include "dcte_plugin.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "dctenergy.h"

static dcte_ctx *g_ctx;
static int g_ctx_status = DCTE_ENODEV;
static pthread_once_t g_ctx_once = PTHREAD_ONCE_INIT;
/* the glue's calls on the shared context: an option set and the call it is
 * meant for must not interleave with another thread's */
static pthread_mutex_t g_ctx_lock = PTHREAD_MUTEX_INITIALIZER;

static void release_ctx(void)
{
    dcte_destroy(g_ctx);
    g_ctx = NULL;
}

static void create_ctx(void)
{
    const char *ng = getenv("DCTE_NGPUS");
    g_ctx_status = dcte_create(&g_ctx, ng && *ng ? atoi(ng) : 1, 0);
    if (g_ctx_status == DCTE_OK) atexit(release_ctx);
}

/* created once per process, whichever thread asks first */
static dcte_ctx *plugin_ctx(void)
{
    pthread_once(&g_ctx_once, create_ctx);
    return g_ctx_status == DCTE_OK ? g_ctx : NULL;
}

/* the arithmetic a glue call runs in (DCTE_PLUGIN_EXACT), set on the shared
 * context right before the call under g_ctx_lock; a carver mirror keeps the
 * mode it was created in (dcte_carver_create), so later calls of another
 * mode do not reach it */
static int set_mode(dcte_ctx *ctx, unsigned flags)
{
    return dcte_set_option(ctx, DCTE_OPT_EXACT, (flags & DCTE_PLUGIN_EXACT) ? 1.0 : 0.0);
}

static void release_hook(dcte_map_cache *c)
{
    dcte_carver_destroy(c->mirror);
    free(c->band_x0);
    free(c->band_e);
    free(c->band_px);
    free(c->ver_lo);
    free(c->ver_hi);
    c->mirror = NULL;
    c->band_x0 = NULL;
    c->band_e = NULL;
    c->band_px = NULL;
    c->ver_lo = c->ver_hi = NULL;
    c->band_valid = c->hook_ok = 0;
}

int dcte_plugin_build_ex(dcte_map_cache *c, const uint8_t *px, int w, int h, int bpp,
                         size_t rowstride, int blocksize, float edges, float textures,
                         int with_transposed, unsigned flags)
{
    if (!c) return DCTE_EINVAL;
    memset(c, 0, sizeof(*c));
    c->flags = flags;
    dcte_ctx *ctx = plugin_ctx();
    if (!ctx) return c->status = g_ctx_status;
    if (w <= 0 || h <= 0) return c->status = DCTE_EINVAL;
    pthread_mutex_lock(&g_ctx_lock);
    int st = set_mode(ctx, flags);
    const size_t npx = (size_t)w * (size_t)h;
    const int ho = with_transposed ? 1 : 0;
    if (st == DCTE_OK) {
        c->map = (float *)malloc(sizeof(float) * npx);
        if (ho) c->map_t = (float *)malloc(sizeof(float) * npx);
        if (!c->map || (ho && !c->map_t)) st = DCTE_ENOMEM;
    }
    if (st == DCTE_OK && (flags & DCTE_PLUGIN_SEAM_HOOK) && (bpp == 1 || bpp == 3)) {
        /* the mirror maps the frame of the resize orientation itself, and the
         * other orientation's map from the same upload */
        if (dcte_carver_create2(ctx, px, w, h, bpp, rowstride, blocksize, edges, textures, ho,
                                ho ? c->map_t : c->map, ho ? c->map : NULL, &c->mirror) == DCTE_OK) {
            c->hook_orientation = ho;
            c->n = blocksize;
            c->mw = dcte_carver_width(c->mirror);
            c->mh = dcte_carver_height(c->mirror);
            c->bw = dcte_carver_band_width(c->mirror);
            c->bpp = bpp;
            c->band_x0 = (int *)malloc(sizeof(int) * (size_t)c->mh);
            c->band_e = (float *)malloc(sizeof(float) * (size_t)c->mh * c->bw);
            c->band_px = (unsigned char *)malloc((size_t)c->mh * c->bw * bpp);
            c->ver_lo = (int *)malloc(sizeof(int) * (size_t)c->mh);
            c->ver_hi = (int *)malloc(sizeof(int) * (size_t)c->mh);
            c->last_x = -1;
            c->hook_ok = c->band_x0 && c->band_e && c->band_px && c->ver_lo && c->ver_hi;
            if (!c->hook_ok) release_hook(c);
        }
    }
    /* no mirror (no hook, or it could not be set up): both maps from one
     * upload, dcte_energy_map2 */
    if (st == DCTE_OK && !c->mirror)
        st = dcte_energy_map2(ctx, px, w, h, bpp, rowstride, blocksize, edges, textures, DCTE_LQR,
                              c->map, c->map_t);
    pthread_mutex_unlock(&g_ctx_lock);
    if (st != DCTE_OK) {
        release_hook(c);
        free(c->map);
        free(c->map_t);
        memset(c, 0, sizeof(*c));
        return c->status = st;
    }
    c->status = DCTE_OK;
    c->w = w;
    c->h = h;
    c->valid = 1;
    return DCTE_OK;
}

int dcte_plugin_preview_u8(const uint8_t *region, int w, int h, int channels, int blocksize,
                           float edges, float textures, unsigned flags, uint8_t *out)
{
    dcte_ctx *ctx = plugin_ctx();
    if (!ctx) return g_ctx_status;
    if (!region || !out || w <= 0 || h <= 0) return DCTE_EINVAL;
    pthread_mutex_lock(&g_ctx_lock);
    int st = set_mode(ctx, flags);
    if (st == DCTE_OK)
        st = dcte_energy_image_u8(ctx, region, w, h, channels, (size_t)w * (size_t)channels,
                                  blocksize, edges, textures, DCTE_PREVIEW, DCTE_NORM_PREVIEW,
                                  channels, out);
    pthread_mutex_unlock(&g_ctx_lock);
    return st;
}

int dcte_plugin_build(dcte_map_cache *c, const uint8_t *px, int w, int h, int bpp,
                      size_t rowstride, int blocksize, float edges, float textures,
                      int with_transposed)
{
    return dcte_plugin_build_ex(c, px, w, h, bpp, rowstride, blocksize, edges, textures,
                                with_transposed, 0u);
}

int dcte_plugin_lookup(const dcte_map_cache *c, int x, int y, int w, int h, int orientation,
                       float *out)
{
    if (!c || !c->valid || x < 0 || y < 0 || x >= w || y >= h) return 0;
    if (orientation == 0 && w == c->w && h == c->h) {
        *out = c->map[(size_t)y * (size_t)w + (size_t)x];
        return 1;
    }
    if (orientation == 1 && c->map_t && w == c->h && h == c->w) {
        *out = c->map_t[(size_t)y * (size_t)w + (size_t)x];
        return 1;
    }
    return 0;
}

/* liblqr's LQR_ER_LUMA of an 8-bit pixel [liblqr, unverified] (what the
 * reading window returns, src/render.c:315): per-channel tables of
 * 0.2126 * (R / 255) etc., added in the formula's order -- bit-identical to
 * evaluating it per pixel. */
static double g_luma_tab[4][256];
static pthread_once_t g_luma_once = PTHREAD_ONCE_INIT;

static void fill_luma_tables(void)
{
    for (int v = 0; v < 256; v++) {
        g_luma_tab[0][v] = (double)v / 255;
        g_luma_tab[1][v] = 0.2126 * ((double)v / 255);
        g_luma_tab[2][v] = 0.7152 * ((double)v / 255);
        g_luma_tab[3][v] = 0.0722 * ((double)v / 255);
    }
}

/* filled once per process, whichever thread's callback comes first */
static void luma_tables(void) { pthread_once(&g_luma_once, fill_luma_tables); }

static double lqr_luma(const unsigned char *q, int bpp)
{
    if (bpp == 1) return g_luma_tab[0][q[0]];
    return g_luma_tab[1][q[0]] + g_luma_tab[2][q[1]] + g_luma_tab[3][q[2]];
}

static int clamp_int(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* compare liblqr's luma at columns [a, b] of row yy with the band; 1 / 0 / -1 */
static int check_span(dcte_map_cache *c, int x, int y, int yy, int a, int b,
                      dcte_rwindow_read_fn rd, void *rw)
{
    const int k0 = a - c->band_x0[yy];
    if (k0 < 0 || b - c->band_x0[yy] >= c->bw) return 0;
    const unsigned char *q = c->band_px + ((size_t)yy * c->bw + (size_t)k0) * c->bpp;
    for (int xx = a; xx <= b; xx++, q += c->bpp) {
        c->reads++;
        if (!(fabs(lqr_luma(q, c->bpp) - rd(rw, xx - x, yy - y)) <= 1e-9)) return -1;
    }
    return 1;
}

int dcte_plugin_window_check(dcte_map_cache *c, int x, int y, int w, int h,
                             dcte_rwindow_read_fn rd, void *rw)
{
    if (!c || !c->band_valid || !rd || w != c->mw || h != c->mh) return 0;
    luma_tables();
    const int r = c->n / 2;
    /* the window's columns: the clamped offsets of render.c:146-152 cover
     * exactly [max(0, x - r + 1), min(w - 1, x + r)] (clamping repeats edge
     * columns, it adds none); rows likewise */
    const int a = clamp_int(x - r + 1, 0, w - 1), b = clamp_int(x + r, 0, w - 1);
    const int y0 = clamp_int(y - r + 1, 0, h - 1), y1 = clamp_int(y + r, 0, h - 1);
    for (int yy = y0; yy <= y1; yy++) {
        int lo = c->ver_lo[yy], hi = c->ver_hi[yy], rc = 1;
        if (a >= lo && b <= hi) continue;              /* checked by an earlier callback */
        if (lo <= hi && a <= hi + 1 && b >= lo - 1) {  /* extend the checked interval */
            if (a < lo) rc = check_span(c, x, y, yy, a, lo - 1, rd, rw);
            if (rc == 1 && b > hi) rc = check_span(c, x, y, yy, hi + 1, b, rd, rw);
            lo = a < lo ? a : lo;
            hi = b > hi ? b : hi;
        } else {                                       /* a new interval */
            rc = check_span(c, x, y, yy, a, b, rd, rw);
            lo = a;
            hi = b;
        }
        if (rc != 1) return rc;
        c->ver_lo[yy] = lo;
        c->ver_hi[yy] = hi;
    }
    return 1;
}

static void reset_checked(dcte_map_cache *c)
{
    for (int i = 0; i < c->mh; i++) {
        c->ver_lo[i] = 1;
        c->ver_hi[i] = 0;
    }
}

int dcte_plugin_lookup_hook(dcte_map_cache *c, int x, int y, int w, int h, int orientation,
                            dcte_rwindow_read_fn rd, void *rw, float *out)
{
    if (!c || !c->valid || !c->hook_ok || !rd || orientation != c->hook_orientation ||
        h != c->mh || x < 0 || y < 0 || x >= w || y >= h)
        return 0;
    /* liblqr carved since the mirror's last step: carve as many seams */
    while (w < c->mw) {
        pthread_mutex_lock(&g_ctx_lock);
        const int st = dcte_carver_step(c->mirror, NULL, c->band_x0, c->band_e, c->band_px);
        pthread_mutex_unlock(&g_ctx_lock);
        if (st != DCTE_OK) {
            release_hook(c);
            c->missed++;
            return 0;
        }
        c->mw--;
        c->steps++;
        c->band_valid = 1;
        reset_checked(c);                          /* nothing of the new band checked yet */
        c->last_y = 0;
        c->last_x = -1;
    }
    /* liblqr walks a pass (an update or a rebuild of its energy map) in
     * increasing rows, and along a row in increasing columns: a callback above
     * the previous one, or on its row but not to the right of it, starts
     * another pass, and liblqr's image may have changed since the columns
     * were checked */
    if (y < c->last_y || (y == c->last_y && x <= c->last_x)) reset_checked(c);
    c->last_y = y;
    c->last_x = x;
    const int chk = dcte_plugin_window_check(c, x, y, w, h, rd, rw);
    const int k = chk == 1 ? x - c->band_x0[y] : -1;
    if (chk <= 0 || k < 0 || k >= c->bw) {
        /* a window that differs from the mirror, or reaches past a band that
         * holds every window of liblqr's update region while the two carve the
         * same seams: the mirror no longer follows liblqr's image */
        if (chk >= 0) c->out_of_band++;
        release_hook(c);
        c->missed++;
        return 0;
    }
    *out = c->band_e[(size_t)y * c->bw + (size_t)k];
    c->served_band++;
    return 1;
}

void dcte_plugin_release(dcte_map_cache *c)
{
    if (!c) return;
    release_hook(c);
    free(c->map);
    free(c->map_t);
    memset(c, 0, sizeof(*c));
}
