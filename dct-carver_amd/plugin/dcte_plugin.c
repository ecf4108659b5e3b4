/* dcte_plugin.c -- see dcte_plugin.h.  One process-wide dcte_ctx, created on
 * first use over DCTE_NGPUS devices (unset = 1 device, 0 = all visible),
 * destroyed at exit.  One device by default: a GIMP frame fits one MI355X many
 * times over, and the single-device path is the one the GPU tests run. */
#include "dcte_plugin.h"

#include <stdlib.h>
#include <string.h>

#include "dctenergy.h"

static dcte_ctx *g_ctx;
static int g_ctx_status = 1; /* 1 = not tried yet */

static void release_ctx(void)
{
    dcte_destroy(g_ctx);
    g_ctx = NULL;
}

static dcte_ctx *plugin_ctx(void)
{
    if (g_ctx_status == 1) {
        const char *ng = getenv("DCTE_NGPUS");
        g_ctx_status = dcte_create(&g_ctx, ng && *ng ? atoi(ng) : 1, 0);
        if (g_ctx_status == DCTE_OK) atexit(release_ctx);
    }
    return g_ctx_status == DCTE_OK ? g_ctx : NULL;
}

int dcte_plugin_build(dcte_map_cache *c, const uint8_t *px, int w, int h, int bpp,
                      size_t rowstride, int blocksize, float edges, float textures,
                      int with_transposed)
{
    if (!c) return DCTE_EINVAL;
    memset(c, 0, sizeof(*c));
    dcte_ctx *ctx = plugin_ctx();
    if (!ctx) return c->status = g_ctx_status;
    if (w <= 0 || h <= 0) return c->status = DCTE_EINVAL;
    c->map = (float *)malloc(sizeof(float) * (size_t)w * (size_t)h);
    if (!c->map) return c->status = DCTE_ENOMEM;
    c->status = dcte_energy_map(ctx, px, w, h, bpp, rowstride, blocksize, edges, textures,
                                DCTE_LQR, 0, c->map);
    if (c->status == DCTE_OK && with_transposed) {
        c->map_t = (float *)malloc(sizeof(float) * (size_t)w * (size_t)h);
        c->status = c->map_t ? dcte_energy_map(ctx, px, w, h, bpp, rowstride, blocksize, edges,
                                               textures, DCTE_LQR, 1, c->map_t)
                             : DCTE_ENOMEM;
    }
    if (c->status != DCTE_OK) {
        int st = c->status;
        free(c->map);
        free(c->map_t);
        memset(c, 0, sizeof(*c));
        return c->status = st;
    }
    c->w = w;
    c->h = h;
    c->valid = 1;
    return DCTE_OK;
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

void dcte_plugin_release(dcte_map_cache *c)
{
    if (!c) return;
    free(c->map);
    free(c->map_t);
    memset(c, 0, sizeof(*c));
}
