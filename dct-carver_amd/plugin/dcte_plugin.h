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

typedef struct {
    float *map;      /* w*h energies of the frame (orientation 0), owned */
    float *map_t;    /* h*w energies of the transposed frame (orientation 1), or NULL */
    int w, h;        /* frame size */
    int valid;
    int status;      /* DCTE_* code of the last build */
} dcte_map_cache;

/* Build the map(s) for the frame handed to lqr_carver_new (src/render.c:312):
 * orientation 0 always, and the transposed frame's map too when
 * `with_transposed` (the plug-in passes vals->vertically, src/main.h:21:
 * liblqr transposes the carver for vertical resizes).  Returns DCTE_OK, or
 * an error code after which every lookup misses (the plug-in then runs its
 * original code). */
int dcte_plugin_build(dcte_map_cache *c, const uint8_t *px, int w, int h, int bpp,
                      size_t rowstride, int blocksize, float edges, float textures,
                      int with_transposed);

/* 1 and *out = energy when (x, y) of a w x h carver in `orientation` is
 * served from a map (orientation 0: the frame's size; 1: the transposed
 * frame's size, if that map was built); 0 otherwise. */
int dcte_plugin_lookup(const dcte_map_cache *c, int x, int y, int w, int h,
                       int orientation, float *out);

void dcte_plugin_release(dcte_map_cache *c);

#ifdef __cplusplus
}
#endif

#endif /* DCTE_PLUGIN_H */
