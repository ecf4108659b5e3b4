/*
 * dctenergy.h -- C ABI of libdctenergy_hip.so, the MI355X (gfx950) backend
 * for the dct-carver energy map.
 *
 * Plain C types only (no HIP, GIMP, glib or liblqr types), so the existing C
 * plug-in links it without new build dependencies.
 *
 * What it replaces, in the reference (avivrosenberg/dct-carver):
 *   - the per-pixel liblqr energy callback dct_pixel_energy
 *     (src/render.c:134-157, registered at src/render.c:314-315 with radius
 *     N/2 and LQR_ER_LUMA), called W*H times by liblqr's energy build, and
 *     the arithmetic under it: dctNxN (src/dct.c:77-94) ->
 *     ddct8x8s / ddct16x16s / ddct2d (src/fft2d/shrtdct.c:55, :231;
 *     src/fft2d/fftsg2d.c:566) and weighted_max_dct_correlation
 *     (src/dct.c:96-110).  dcte_energy_map computes all W*H callback
 *     results of one carver build in one call; the plug-in then serves
 *     dct_pixel_energy(x, y, ...) from the returned map.
 *
 * Semantics (DCTE_LQR): out[y*w + x] = the value dct_pixel_energy(x, y, w, h,
 * rw, params) returns for a carver built on these pixels with blocksize N,
 * edges, textures -- liblqr luma 0.2126 R + 0.7152 G + 0.0722 B on channel/255
 * (grey: v/255) [liblqr, unverified], window offsets -(N/2-1)..N/2 with
 * replicate clamp, 2-D DCT-II (orthonormal N=8,16; unnormalised N=2,4),
 * weighted max with the last-maximum tie rule.  Results agree with the
 * reference CPU path to <= 1e-5 relative (measured ~3e-7), bit-exactly
 * wherever the edge/texture decision is within the fp32 error band.
 *
 * Errors: every entry point returns DCTE_OK (0) or a negative DCTE_E* code
 * and never exits the process (the reference exit(1)s on OOM,
 * src/fft2d/alloc.c:5-10, and silently leaves the data untransformed for a
 * bad N, src/dct.c:89-92; here a bad N is DCTE_EINVAL).
 *
 * Threading: one context serves one thread at a time (the reference callback
 * is not re-entrant either: it shares params->data, src/render.c:140).
 */
#ifndef DCTENERGY_H
#define DCTENERGY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history.  1: first release.  2 (r06): DCTE_OPT_FAIL_INJECT moved from
 * option id 8 to 9 (8 = the removed WIDE_BANDS, accepted as a no-op) -- a
 * caller built against version 1 that arms id 8 injects nothing; new entry
 * points dcte_energy_map2 and dcte_carver_create2; a dcte_carver keeps the
 * arithmetic mode (DCTE_OPT_EXACT, DCTE_OPT_TIE_TAU) it was created in. */
#define DCTE_ABI_VERSION 2

/* status codes */
#define DCTE_OK 0
#define DCTE_EINVAL (-1)   /* bad argument (N not in {2,4,8,16}, sizes, bpp) */
#define DCTE_ENODEV (-2)   /* no usable gfx950 device */
#define DCTE_ENOMEM (-3)   /* device or host allocation failed */
#define DCTE_EHIP (-4)     /* HIP runtime error (see dcte_last_error) */
#define DCTE_ERANGE (-5)   /* frame too large for one launch (> 4 GiB band) */
#define DCTE_ENOTSUP (-6)  /* recognised but not provided by this build */

/* energy semantics
 * DCTE_LQR     the liblqr energy callback dct_pixel_energy (src/render.c:134-157):
 *              liblqr luma [unverified] in [0,1], window -(N/2-1)..N/2,
 *              bpp 1 or 3 (alpha handling is liblqr's and unverifiable here)
 * DCTE_PREVIEW the dialog preview dct_energy_preview (src/render.c:31-79,
 *              421-479): u8 luma RGB2LUMINANCE (src/render.h:5; grey = the
 *              byte), window -(c-1)..N-c with c = (N-1)/2 (src/dct.h:8-9),
 *              clamp to the region passed in; bpp 1, 3 or 4 (alpha ignored,
 *              as convert_row_to_luminance does) */
#define DCTE_LQR 0
#define DCTE_PREVIEW 1

/* options for dcte_set_option */
#define DCTE_OPT_TIE_TAU 1 /* relative edge/texture margin refined in fp64
                              (default per N: 4e-6 for N = 2, 4; 2e-5 for
                              N = 8; 5e-5 for N = 16 -- at least twice the
                              derived worst-case fp32 error, DESIGN.md §5;
                              a negative value restores these defaults;
                              0 = never refine, >= 1 = refine every pixel) */
#define DCTE_OPT_PROFILE 2 /* 1 = time every map-kernel launch: HIP events
                              the launch itself records at the kernel's start
                              and end (dcte_profile_read) */
#define DCTE_OPT_PIN_HOST 3 /* host entry points: page-lock the caller's frame
                               and output (their whole pages) for the duration
                               of a call when they are at least this many MiB
                               (default 1; 0 = never), so the chunked H2D / D2H
                               copies overlap; the bytes no lock covers (partial
                               end pages, smaller buffers) are staged through a
                               page-locked buffer of the context -- no copy
                               takes the runtime's pageable path */
#define DCTE_OPT_TILE_H 4   /* output rows per map workgroup (0 = the kernel's
                               default, 128); results do not depend on it */
#define DCTE_OPT_DP_BANDWISE 5 /* 1 = run the seam search one launch per band of
                               rows even when every DP tile fits on the chip
                               (the mode frames wider than that use; no tile
                               then waits on another); same seams */
#define DCTE_OPT_DP_SPIN_LIMIT 6 /* polls after which a tile of the single-launch
                               seam search stops waiting for a neighbour (0 =
                               default, ~0.5 s; small values are for testing
                               the time-out path).  A timed-out search returns
                               seam = -1 from the device entry point; the host
                               entry points (dcte_seam_find, dcte_carve) run it
                               again band-wise and keep that stream band-wise.
                               Setting this option re-enables the single
                               launch. */
#define DCTE_OPT_TSTAMP_BUF 7 /* diagnostic, timing-probe builds (DCTE_TSTAMP=1)
                               only: device address of a buffer of 3 uint64
                               per map workgroup {start, end, HW_ID}; 0 = none.
                               Product builds ignore it. */
#define DCTE_OPT_LEGACY_8 8  /* DCTE_OPT_WIDE_BANDS of the first release
                               (removed): accepted and ignored, as its results
                               never depended on it */
#define DCTE_OPT_FAIL_INJECT 9 /* testing the error paths: 1 = the next map
                               launch is reported as failed (DCTE_EHIP) right
                               after it was queued; 2 = the next refinement
                               launch likewise (an exact-mode map call, which
                               has no refinement launch, disarms it).
                               One-shot; 0 = off.  (Id 8 in ABI version 1.) */
#define DCTE_OPT_EXACT 10   /* 1 = bit-identical to the reference for every
                               pixel: the map is computed in the reference's
                               own fp64 operation order (ddct8x8s / ddct16x16s /
                               ddct2d and the last-maximum scan) by a sliding-
                               window kernel, so liblqr's DP on it carves the
                               reference's seams -- every N, both semantics
                               (the preview's transposed window has kernels of
                               its own).  Seam-band updates and point energies are then
                               refined in fp64 too.  0 = the fp32 map with the
                               tie refinement (default; <= 1e-5 relative). */

#define DCTE_OPT_D2H_KERNEL 11 /* host entry points on one device: 1 (default)
                               = the maps go down through a copy kernel that
                               writes the page-locked output directly (the
                               GPU's own stores over PCIe, beside the SDMA
                               upload); 0 = the runtime's copy engine, which
                               on some runs serialised the two directions
                               (38 instead of 22 ms at 16384^2) */

typedef struct dcte_ctx dcte_ctx;

int dcte_abi_version(void);

/* Number of visible HIP devices (0 when none; never an error). */
int dcte_device_count(void);

/* Create a context on `ngpus` devices (0 = all visible).  Device memory,
 * streams and kernels are set up lazily on first use.  flags: 0, or
 * DCTE_CREATE_SAME_DEVICE: `ngpus` logical devices that are all physical
 * device 0 (each with its own streams and buffers), so the multi-device host
 * path -- band split, halo rows, per-device pipelines, the u8 min/max merge --
 * can be checked against the 1-device map on a 1-GPU machine. */
#define DCTE_CREATE_SAME_DEVICE 1u
int dcte_create(dcte_ctx **ctx, int ngpus, unsigned flags);
void dcte_destroy(dcte_ctx *ctx);

/* Number of devices the context uses. */
int dcte_ctx_devices(const dcte_ctx *ctx);

int dcte_set_option(dcte_ctx *ctx, int option, double value);

/* Host-buffer entry point: the full energy map of one frame.
 *   px        8-bit interleaved pixels, bpp channels (1 grey, 3 RGB), row y
 *             at px + y*rowstride (the buffer the plug-in hands to
 *             lqr_carver_new, src/render.c:159-173,312)
 *   n         blocksize N (2, 4, 8, 16)
 *   edges, textures   weights (PlugInVals, src/main.h:12-22)
 *   semantics DCTE_LQR or DCTE_PREVIEW
 *   transposed 1 = the map of the transposed frame (what the callback returns
 *             once liblqr has transposed the carver for a vertical resize);
 *             out then holds w rows of h floats
 *   out       caller-owned w*h floats, row-major
 * With several devices the frame is split into row bands; each device
 * receives its band plus the N/2-row halo straight from `px`. */
int dcte_energy_map(dcte_ctx *ctx, const uint8_t *px, int w, int h, int bpp,
                    size_t rowstride, int n, float edges, float textures,
                    int semantics, int transposed, float *out);

/* Both orientations of one frame from ONE upload (the plug-in's build for a
 * vertical resize, src/render.c:358-364 with vals->vertically, src/main.h:21:
 * liblqr transposes the carver, so its callbacks ask for the transposed
 * frame's map, and the plug-in keeps the untransposed map too).  out (w*h
 * floats, h rows of w) = dcte_energy_map(..., transposed = 0, out); out_t
 * (w rows of h) = dcte_energy_map(..., transposed = 1, out_t): the same bits
 * as the two calls.  Either may be NULL (not both).  One device: the frame is
 * uploaded in row chunks with each chunk mapped and its map downloaded as it
 * lands; the resident frame is then transposed in HBM and the transposed
 * map computed and downloaded chunk by chunk.  Several devices: the two
 * calls. */
int dcte_energy_map2(dcte_ctx *ctx, const uint8_t *px, int w, int h, int bpp,
                     size_t rowstride, int n, float edges, float textures,
                     int semantics, float *out, float *out_t);

/* Device-resident entry point (frames already in HBM; no copies, no sync).
 *   device    index into the context's devices
 *   d_px      device pointer to global row in_row0 of a w x h frame; rows
 *             [in_row0, in_row0 + in_rows) are readable and must include
 *             every row the clamp reaches for [y0, y1)
 *   d_out     device pointer; row y (y0 <= y < y1) at d_out + (y-y0)*out_stride
 *   stream    hipStream_t (NULL = default stream) the work is ordered on
 * Calls on different streams may run concurrently (separate scratch). */
int dcte_energy_map_device(dcte_ctx *ctx, int device, const void *d_px,
                           long long rowstride, int w, int h, int bpp,
                           int in_row0, int in_rows, int y0, int y1, int n,
                           float edges, float textures, int semantics, float *d_out,
                           long long out_stride, void *stream);

/* The same for TWO output row ranges in one map launch and one refinement
 * launch: [y0, y1) and [yb0, yb1) with y1 <= yb0 (yb0 == yb1: the second is
 * empty); row y of either at d_out + (y - y0) * out_stride.  For a row-band
 * shard: both halo-dependent edge ranges of a band after the
 * RCCL halo exchange.  The rows the clamp reaches for each range must be
 * readable; rows between the two ranges' needs are never read (they only
 * have to lie inside the [in_row0, in_row0 + in_rows) span). */
int dcte_energy_map_device2(dcte_ctx *ctx, int device, const void *d_px,
                            long long rowstride, int w, int h, int bpp,
                            int in_row0, int in_rows, int y0, int y1, int yb0, int yb1,
                            int n, float edges, float textures, int semantics,
                            float *d_out, long long out_stride, void *stream);

/* ---- seam carving support --------------------------------
 * After the initial map, liblqr carves one seam at a time and re-evaluates
 * the callback (src/render.c:134-157) only around the removed seam
 * (update_emap, during lqr_carver_resize at src/render.c:377) [liblqr,
 * unverified].  With the frame and its map resident in HBM this is one call
 * per seam:
 *
 * dcte_seam_carve_device: removes pixel d_seam[y] from every row y of the
 *   w x h frame (d_px) -> the (w-1) x h frame d_px_out, and writes the map of
 *   that frame to d_map_out: pixels whose window lies on one side of the
 *   seam are moved from d_map (the map of d_px), the <= N-1+drift pixels per
 *   row whose window straddles it are recomputed -- exactly the values
 *   dcte_energy_map gives for d_px_out (same fp32 passes, same refinement).
 *   d_seam: h device ints in [0, w) (values outside are clamped).
 *   In place: d_px_out == d_px with the same row stride AND d_map_out ==
 *   d_map with the same stride -- only the part right of the seam moves (the
 *   frame keeps its row stride, one pixel narrower).  Otherwise the output
 *   buffers must not overlap the inputs.  Stream-ordered. */
int dcte_seam_carve_device(dcte_ctx *ctx, int device, const void *d_px, long long rowstride,
                           int w, int h, int bpp, const int *d_seam, const float *d_map,
                           long long map_stride, void *d_px_out, long long out_rowstride,
                           float *d_map_out, long long map_out_stride, int n, float edges,
                           float textures, int semantics, void *stream);

/* Energies at listed pixels -- the batched form of the per-pixel callback
 * (one dct_pixel_energy per point, src/render.c:134-157), for a carver-side
 * hook that re-evaluates a set of pixels at once.  xy: count (x, y) pairs;
 * out[k] = energy of pixel (xy[2k], xy[2k+1]) of the w x h frame, equal to
 * that pixel of dcte_energy_map.  Host version: the frame and points are
 * copied to the first device; coordinates outside the frame are
 * DCTE_EINVAL.  Device version: whole frame resident, coordinates clamped,
 * stream-ordered. */
int dcte_energy_points(dcte_ctx *ctx, const uint8_t *px, int w, int h, int bpp,
                       size_t rowstride, const int *xy, int count, int n, float edges,
                       float textures, int semantics, float *out);
int dcte_energy_points_device(dcte_ctx *ctx, int device, const void *d_px, long long rowstride,
                              int w, int h, int bpp, const int *d_xy, int count, int n,
                              float edges, float textures, int semantics, float *d_out,
                              void *stream);

/* Energies of windows the caller filled (SURVEY §8b dcte_energy_window, in
 * batches): win = count windows of n*n doubles in the reference's data[i][j]
 * layout -- what dct_pixel_energy gathers (src/render.c:146-152: i = x
 * offset, j = y offset, luma in [0, 1]) -- and out[k] = the
 * weighted_max_dct_correlation of dctNxN of window k (src/dct.c:77-110),
 * computed in fp64 in the reference's operation order on the device:
 * bit-identical to the reference for any input.  For a liblqr-side hook that
 * keeps its own reading windows (seam updates after the carver shrank).
 * Host version: windows copied to the first device; device version:
 * stream-ordered. */
int dcte_energy_windows(dcte_ctx *ctx, const double *win, int count, int n, float edges,
                        float textures, float *out);
int dcte_energy_windows_device(dcte_ctx *ctx, int device, const double *d_win, int count, int n,
                               float edges, float textures, float *d_out, void *stream);

/* ---- minimum-energy seam ---------------------------------
 * liblqr's cumulative energy for the reference's carver configuration
 * (lqr_carver_init(carver, 1, 0), src/render.c:313: delta_x 1, rigidity 0)
 * [liblqr, unverified]: M[0] = E[0], M[y][x] = E[y][x] + min(M[y-1][x-1..x+1]),
 * float arithmetic, leftmost minimum on ties; the seam ends at the leftmost
 * minimum of the last row.  seam[y] = column to remove in row y (feed it to
 * dcte_seam_carve_device).  Vertical seams of a w x h map; for horizontal
 * seams pass the transposed map.
 * Device version: stream-ordered; if the search fails internally (a tile
 * waited ~1 s for a neighbour) d_seam is filled with -1.
 * Host version: map is w*h floats (row stride w); returns DCTE_EHIP on that
 * failure. */
int dcte_seam_find_device(dcte_ctx *ctx, int device, const float *d_map, long long map_stride,
                          int w, int h, int *d_seam, void *stream);
int dcte_seam_find(dcte_ctx *ctx, const float *map, int w, int h, int *seam);

/* ---- carving a whole frame (host buffers) --------------------------------
 * Removes `seams` minimum-energy seams one at a time -- the loop liblqr runs
 * in lqr_carver_resize (src/render.c:377) for the reference's carver set-up
 * (delta_x 1, rigidity 0, the DCT energy re-evaluated around every removed
 * seam) [liblqr, unverified]: energy map, then (dcte_seam_find_device ->
 * dcte_seam_carve_device) per seam, all in HBM on the first device; one
 * upload, one download.
 *   transposed 0: vertical seams, out is h rows of (w - seams) pixels;
 *              1: horizontal seams (the frame is carved transposed, as liblqr
 *              does for vertical resizes), out is (h - seams) rows of w pixels.
 *              Rows of out are dense (row stride = width * bpp).
 *   seam_cols  NULL, or seams * L ints (L = h, or w when transposed): entry
 *              k * L + i = the pixel removed from line i by step k, counted in
 *              that step's frame.
 * 0 <= seams < the carved dimension (w, or h when transposed). */
int dcte_carve(dcte_ctx *ctx, const uint8_t *px, int w, int h, int bpp, size_t rowstride,
               int n, float edges, float textures, int semantics, int seams, int transposed,
               uint8_t *out, int *seam_cols);

/* ---- device mirror of a liblqr carver -------------------
 * The update_emap hook of the plug-in: after the first
 * build, liblqr's resize loop (lqr_carver_resize, src/render.c:377) carves one
 * seam at a time and asks the energy callback again only around it
 * (update_emap) [liblqr, unverified].  A dcte_carver holds the carver's frame
 * and energy map in HBM and replays that loop: each step finds the seam
 * liblqr's DP picks on the same energies (dcte_seam_find_device: delta_x 1,
 * rigidity 0, src/render.c:313), carves it and updates the map
 * (dcte_seam_carve_device), then hands back the energies -- and the pixels,
 * so the caller can check that it follows liblqr's image -- of a band around
 * the seam: row y holds band_width columns from band_x0[y] on of the carved
 * frame, covering every pixel whose radius-N/2 window reaches the seam and
 * every pixel of those pixels' own N x N windows (the hook checks them).
 * Every value equals dcte_energy_map of the carved frame at that pixel.
 * liblqr semantics (DCTE_LQR), bpp 1 or 3.
 *
 * dcte_carver_create: uploads px (w x h; transposed = 1 mirrors a carver that
 *   liblqr transposed for a vertical resize: the frame is then h wide) and
 *   maps it; map_out (optional) receives that first map (width x height
 *   floats of the mirrored frame).
 * dcte_carver_step: one seam.  seam (height ints, columns in the frame before
 *   the step), band_x0 (height ints), band_e (height x band_width floats),
 *   band_px (height x band_width x bpp bytes): each optional.
 * Mode: a carver computes in the arithmetic the context was set to when the
 *   carver was created (DCTE_OPT_EXACT, DCTE_OPT_TIE_TAU) for its whole life:
 *   setting the context's options afterwards (another carver, a preview)
 *   changes nothing for it.  (The reference's callback is bit-identical per
 *   carver by construction, src/render.c:296-315.)
 * dcte_carver_create2: also map_other_out (optional, w*h floats): the map of
 *   the OTHER orientation of the same frame (transposed = 1: the frame as
 *   given, h rows of w; transposed = 0: the transposed frame, w rows of h)
 *   from the same upload -- the plug-in's vertical build needs both. */
typedef struct dcte_carver dcte_carver;
int dcte_carver_create(dcte_ctx *ctx, const uint8_t *px, int w, int h, int bpp, size_t rowstride,
                       int n, float edges, float textures, int transposed, float *map_out,
                       dcte_carver **out);
int dcte_carver_create2(dcte_ctx *ctx, const uint8_t *px, int w, int h, int bpp, size_t rowstride,
                        int n, float edges, float textures, int transposed, float *map_out,
                        float *map_other_out, dcte_carver **out);
int dcte_carver_step(dcte_carver *c, int *seam, int *band_x0, float *band_e, uint8_t *band_px);
int dcte_carver_width(const dcte_carver *c);       /* current width of the mirrored frame */
int dcte_carver_height(const dcte_carver *c);
int dcte_carver_band_width(const dcte_carver *c);  /* 4 N + 4 */
void dcte_carver_destroy(dcte_carver *c);

/* ---- energy image as 8-bit grey ----------------------
 * DCTE_NORM_PREVIEW: normalize_image (src/render.c:81-109, DOUBLE2GUCHAR of
 *   src/render.h:6): ROUND(255*(E-min)/(max-min)) in double, replicated to
 *   `channels` bytes per pixel; max == min -> 0 (the reference divides by
 *   zero there, src/render.c:101).
 * DCTE_NORM_LQR: the energy layer of display_carver_energy
 *   (src/render.c:175-202, lqr_carver_get_energy_image): (E-min)/(max-min)
 *   in float times 255, truncated [liblqr, unverified]. */
#define DCTE_NORM_LQR 0
#define DCTE_NORM_PREVIEW 1

/* host buffers: E (n floats) -> out (n*channels bytes), on the first device */
int dcte_normalize_u8(dcte_ctx *ctx, const float *E, size_t n, int mode, int channels,
                      uint8_t *out);

/* ---- context-free CPU entries -------------------------------
 * No context and no device: plain host code, for a caller that keeps its own
 * reading windows on the CPU (liblqr's per-pixel callback after seams shrank
 * the carver, src/render.c:134-157,377).  The GPU entry points never fall
 * back to these.
 *
 * dcte_energy_window: one window of n*n doubles in the reference's data[i][j]
 *   layout (src/render.c:146-152: i = x offset, j = y offset, luma in
 *   [0, 1]) -> *out = weighted_max_dct_correlation(dctNxN(window))
 *   (src/dct.c:77-110) in fp64 in the reference's operation order:
 *   bit-identical to the reference.  The window is not modified.
 * dcte_normalize_u8_host: dcte_normalize_u8 without a device (same bytes). */
int dcte_energy_window(int n, const double *win, float edges, float textures, float *out);
int dcte_normalize_u8_host(const float *E, size_t n, int mode, int channels, uint8_t *out);

/* energy map + normalisation without the f32 round trip to the host: out is
 * w*h*channels bytes.  Several devices: band maps, one global min/max. */
int dcte_energy_image_u8(dcte_ctx *ctx, const uint8_t *px, int w, int h, int bpp,
                         size_t rowstride, int n, float edges, float textures,
                         int semantics, int mode, int channels, uint8_t *out);

/* device pieces (stream-ordered, no sync): min/max of n floats into
 * d_minmax[0..1]; then normalise with a (possibly all-reduced) d_minmax */
int dcte_minmax_device(dcte_ctx *ctx, int device, const float *d_E, long long n,
                       float *d_minmax, void *stream);
int dcte_normalize_u8_device(dcte_ctx *ctx, int device, const float *d_E, long long n,
                             const float *d_minmax, int mode, int channels, uint8_t *d_out,
                             void *stream);

/* Pixels recomputed by the fp64 refinement in the last dcte_energy_map call
 * (diagnostic; device calls are not synchronised, so not counted). */
long long dcte_last_refined(const dcte_ctx *ctx);

/* Profiling (DCTE_OPT_PROFILE = 1): synchronises the recorded events and
 * returns the number of map-kernel launches and their summed device time
 * since the last read, then resets. */
int dcte_profile_read(dcte_ctx *ctx, long long *launches, double *kernel_ms);

const char *dcte_strerror(int code);

/* Text of the last HIP error seen by this context ("" if none). */
const char *dcte_last_error(const dcte_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif /* DCTENERGY_H */
