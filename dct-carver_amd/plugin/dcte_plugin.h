/*
 * dcte_plugin.h -- plug-in side glue for libdctenergy_hip.so.
 *
 * Compiled INTO the dct-carver plug-in (plain C, no GIMP/liblqr types), next
 * to src/render.c.  The plug-in keeps one dcte_map_cache in its
 * EnergyParameters (src/render.h:9-16), fills it once per carver in
 * init_carver_from_vals (src/render.c:286-325) and lets dct_pixel_energy
 * (src/render.c:134-157) answer from it while liblqr asks for pixels of the
 * frame the map was built on (same width/height, horizontal orientation).
 * Every other call -- after a seam changed the carver size, in the
 * transposed (vertical) orientation, or when no GPU is present -- runs the
 * plug-in's original per-window code unchanged.  INTEGRATION.md has the patch.
 */
#ifndef DCTE_PLUGIN_H
#define DCTE_PLUGIN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct dcte_carver;

typedef struct {
    float *map;      /* w*h energies of the frame (orientation 0), owned */
    float *map_t;    /* h*w energies of the transposed frame (orientation 1), or NULL */
    int w, h;        /* frame size */
    int valid;
    int status;      /* DCTE_* code of the last build */
    unsigned flags;  /* the build's DCTE_PLUGIN_* flags: this carver's mode */
    /* opt-in seam hook (DCTE_PLUGIN_SEAM_HOOK): a device
     * mirror of the carver that replays each seam liblqr carves and hands
     * back the energies and pixels around it, so update_emap's callbacks are
     * served too -- each only after the callback's whole reading window
     * matched the mirror's pixels */
    struct dcte_carver *mirror;
    int hook_orientation;  /* the orientation liblqr resizes in */
    int hook_ok;           /* 0 once the mirror lost track of liblqr's image */
    int n;                 /* blocksize: the window is n x n, radius n / 2 */
    int mw, mh, bpp, bw;   /* mirror's current width, height; bytes per pixel; band width */
    int band_valid;
    int *band_x0;          /* mh: first band column per row */
    float *band_e;         /* mh x bw energies of the last step's band */
    unsigned char *band_px;/* mh x bw x bpp pixels of the carved frame (window check) */
    int *ver_lo, *ver_hi;  /* mh: columns of each row already checked against liblqr this pass */
    int last_y, last_x;    /* the previous hooked callback: one above it, or on its row and not
                              right of it, starts a new pass */
    long long served_band, missed, out_of_band, steps, reads;
} dcte_map_cache;

#define DCTE_PLUGIN_SEAM_HOOK 1u
/* every energy the plug-in serves is the reference's own double: the maps and
 * the hook's band updates in the exact mode (DCTE_OPT_EXACT), so liblqr carves
 * the reference's seams.  The mode belongs to the cache it was built with: a
 * later build or preview in the other mode (the dialog's preview, a second
 * carver, src/interface.c:116,524,662) does not change it. */
#define DCTE_PLUGIN_EXACT 2u

/* Build the map(s) for the frame handed to lqr_carver_new (src/render.c:312):
 * orientation 0 always, and the transposed frame's map too when
 * `with_transposed` (the plug-in passes vals->vertically, src/main.h:21:
 * liblqr transposes the carver for vertical resizes) -- both from one upload
 * of the frame (dcte_energy_map2, or dcte_carver_create2 with the seam hook).
 * Returns DCTE_OK, or an error code after which every lookup misses (the
 * plug-in then runs its original code).  The glue's calls on its process-wide
 * context are serialised by a mutex; the context is created once
 * (pthread_once) by whichever thread comes first. */
int dcte_plugin_build(dcte_map_cache *c, const uint8_t *px, int w, int h, int bpp,
                      size_t rowstride, int blocksize, float edges, float textures,
                      int with_transposed);

/* dcte_plugin_build with flags: DCTE_PLUGIN_SEAM_HOOK also sets up the
 * device mirror of the carver for the orientation liblqr will resize in
 * (with_transposed: vertical, 1; else 0).  Without a GPU, or when the mirror
 * cannot be set up, the build behaves as dcte_plugin_build.
 * DCTE_PLUGIN_EXACT: the maps and the mirror's band updates are computed in
 * the reference's fp64 arithmetic (bit-identical to the original callback);
 * without it they agree with it within 1e-5 relative. */
int dcte_plugin_build_ex(dcte_map_cache *c, const uint8_t *px, int w, int h, int bpp,
                         size_t rowstride, int blocksize, float edges, float textures,
                         int with_transposed, unsigned flags);

/* 1 and *out = energy when (x, y) of a w x h carver in `orientation` is
 * served from a map (orientation 0: the frame's size; 1: the transposed
 * frame's size, if that map was built); 0 otherwise. */
int dcte_plugin_lookup(const dcte_map_cache *c, int x, int y, int w, int h,
                       int orientation, float *out);

/* What the hook reads liblqr's image through: the callback's reading window,
 * rd(rw, dx, dy) = lqr_rwindow_read(rw, dx, dy, 0) (src/render.c:150), for
 * offsets of the window the callback would gather (dx, dy in -(r - 1) .. r,
 * r = n / 2, already clamped to the frame like clamp_offset_to_border,
 * src/render.c:122-132). */
typedef double (*dcte_rwindow_read_fn)(void *rw, int dx, int dy);

/* The seam hook, for the callbacks dcte_plugin_lookup misses: when the
 * carver has become narrower than the mirror (liblqr carved a seam), the
 * mirror carves its own seam on the GPU and pixels of its update band are
 * served.  A value is served only when EVERY element of the N x N window the
 * original body would gather (src/render.c:141-152: data[i][j] = read of the
 * clamped offsets (i, j), i, j in -(r - 1) .. r) equals liblqr's luma of the
 * mirror's pixel at the same position (|difference| <= 1e-9: distinct 8-bit
 * lumas differ by >= 7.8e-7), so the served energy is the energy of exactly
 * the window the original body would transform, whatever seam liblqr picked.
 * liblqr's image does not change between the callbacks of one update pass, so
 * each band pixel is read through `rd` and compared once per seam (per row, the
 * interval of columns already checked grows with the callbacks): about two
 * reads per callback instead of N^2.  A window that differs from the mirror,
 * or has a pixel outside the band (which holds every window of liblqr's update
 * region while the two carve the same seams), means the mirror no longer
 * follows liblqr's image: the hook misses and switches itself off for this
 * carver.  Misses return 0: the callback then runs its original body. */
int dcte_plugin_lookup_hook(dcte_map_cache *c, int x, int y, int w, int h, int orientation,
                            dcte_rwindow_read_fn rd, void *rw, float *out);

/* The window test of dcte_plugin_lookup_hook alone, on the current band (it
 * records what it checked): 1 = every element matches the mirror, 0 = a
 * window pixel lies outside the band (or no band), -1 = an element differs.
 * Exposed for tests. */
int dcte_plugin_window_check(dcte_map_cache *c, int x, int y, int w, int h,
                             dcte_rwindow_read_fn rd, void *rw);

/* The dialog preview (dct_energy_preview, src/render.c:421-501, called from
 * src/interface.c:524): region = the preview rectangle's pixels as
 * gimp_pixel_rgn_get_rect returns them (h rows of w * channels bytes,
 * channels 1, 3 or 4 -- alpha ignored, as convert_row_to_luminance does,
 * src/render.c:62-79); out = the drawn layer, w * h * channels bytes:
 * normalize_image's DOUBLE2GUCHAR grey of dct_energy_preview_rows' energies
 * (src/render.c:31-60, 80-109) in every channel.  flags: DCTE_PLUGIN_EXACT =
 * the reference's bytes exactly; else the energies within 1e-5 relative (the
 * bytes within +-1).  Returns DCTE_OK, or an error code (no device, channels
 * 2) after which the plug-in runs its original loop. */
int dcte_plugin_preview_u8(const uint8_t *region, int w, int h, int channels, int blocksize,
                           float edges, float textures, unsigned flags, uint8_t *out);

void dcte_plugin_release(dcte_map_cache *c);

#ifdef __cplusplus
}
#endif

#endif /* DCTE_PLUGIN_H */
