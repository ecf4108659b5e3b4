/*
 * ref_harness.c -- drives the REFERENCE's own compiled transforms.
 *
 * TEST INFRASTRUCTURE ONLY (see dcte_oracle.c).  Built by oracle/Makefile
 * into oracle/_ref/libdcte_ref.so together with the reference's unmodified
 * src/fft2d/{alloc,fftsg,fftsg2d,shrtdct}.c, compiled where they lie under
 * /root/reference with the reference's own flags (-DUSE_FFT2D_PTHREADS,
 * src/fft2d/Makefile.am:13-16).
 *
 * src/dct.c and src/render.c cannot be compiled here (they need the GIMP,
 * GTK and liblqr headers, which this image lacks), so the two thin pieces of
 * glue around the transforms are restated below, with the reference's own
 * scratch layout (row-pointer arrays from alloc_2d_double, ip[] / w[] sized
 * as in src/render.c:302-305, ip[0] = 0 once per carver):
 *   - dctNxN dispatch           src/dct.c:77-94
 *   - weighted max + edge LUT   src/dct.c:10-43, 56-73, 96-110
 *   - window gather + clamp     src/render.c:122-157
 *   - preview gather + luma     src/render.c:31-79 (row-streamed window over
 *                               u8 luma rows, RGB2LUMINANCE src/render.h:5)
 * Everything numeric (ddct8x8s, ddct16x16s, ddct2d) is the reference's code.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

/* prototypes as declared by the reference at src/dct.c:51-53 */
void ddct8x8s(int isgn, double **a);
void ddct16x16s(int isgn, double **a);
void ddct2d(int n1, int n2, int isgn, double **a, double *t, int *ip, double *w);
/* from src/fft2d/alloc.h */
int *alloc_1d_int(int n1);
void free_1d_int(int *i);
double *alloc_1d_double(int n1);
void free_1d_double(double *d);
double **alloc_2d_double(int n1, int n2);
void free_2d_double(double **dd);

typedef struct {
    int n;
    int *ip;
    double *w;
    double **data;
} ref_scratch;

static void scratch_init(ref_scratch *s, int n)
{
    s->n = n;
    s->ip = alloc_1d_int(2 + (int)sqrt(n / 2 + 0.5));
    s->w = alloc_1d_double(n * 3 / 2);
    s->data = alloc_2d_double(n, n);
    s->ip[0] = 0;
}

static void scratch_free(ref_scratch *s)
{
    free_1d_int(s->ip);
    free_1d_double(s->w);
    free_2d_double(s->data);
}

static void dispatch(ref_scratch *s)
{
    switch (s->n) {
    case 2:
    case 4: ddct2d(s->n, s->n, -1, s->data, NULL, s->ip, s->w); break;
    case 8: ddct8x8s(-1, s->data); break;
    case 16: ddct16x16s(-1, s->data); break;
    default: break;
    }
}

static float weighted_max(const ref_scratch *s, float edges, float textures)
{
    int k1, k2, b1 = 0, b2 = 0, n = s->n;
    double m = 0, v;
    for (k1 = 0; k1 < n; k1++)
        for (k2 = 0; k2 < n; k2++) {
            v = fabs(s->data[k1][k2]);
            if (m <= v && (k1 || k2)) {
                m = v;
                b1 = k1;
                b2 = k2;
            }
        }
    int edge = (b1 == 0 && b2 == 1) || (b1 == 1 && b2 == 0);
    return edge ? (float)(m * edges) : (float)(m * textures);
}

static int clamp_off(int base, int off, int lo, int hi)
{
    if (base + off - lo < 0) return off - (base + off - lo);
    if (base + off - hi > 0) return off - (base + off - hi);
    return off;
}

/* In-place reference transform of an n*n window given as a flat [dx][dy] array. */
int ref_dct(int n, double *win)
{
    ref_scratch s;
    if (n != 2 && n != 4 && n != 8 && n != 16) return -1;
    scratch_init(&s, n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) s.data[i][j] = win[i * n + j];
    dispatch(&s);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) win[i * n + j] = s.data[i][j];
    scratch_free(&s);
    return 0;
}

float ref_window_energy(int n, const double *win, float edges, float textures)
{
    ref_scratch s;
    scratch_init(&s, n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) s.data[i][j] = win[i * n + j];
    dispatch(&s);
    float e = weighted_max(&s, edges, textures);
    scratch_free(&s);
    return e;
}

/* Full map over a w*h luma plane (row-major doubles), serial, in liblqr's
 * build order (rows outer, columns inner), one scratch per "carver". */
int ref_energy_map_luma(const double *luma, int w, int h, int n, float edges,
                        float textures, float *out)
{
    if (n != 2 && n != 4 && n != 8 && n != 16) return -1;
    ref_scratch s;
    scratch_init(&s, n);
    int r = n / 2;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            for (int i = -r + 1; i <= r; i++)
                for (int j = -r + 1; j <= r; j++) {
                    int ii = clamp_off(x, i, 0, w - 1);
                    int jj = clamp_off(y, j, 0, h - 1);
                    s.data[i + r - 1][j + r - 1] = luma[(size_t)(y + jj) * w + (x + ii)];
                }
            dispatch(&s);
            out[(size_t)y * w + x] = weighted_max(&s, edges, textures);
        }
    scratch_free(&s);
    return 0;
}

/* Output rows [y0, y1) of the map of a w*h luma plane, OpenMP over rows with
 * one scratch per thread (the reference's per-carver scratch,
 * src/render.c:296-305, is what makes its callback non-re-entrant; each
 * thread owning one restores re-entrancy without touching the transforms).
 * The CPU baseline of bench.py: the reference path on the host cores. */
int ref_energy_map_luma_rows(const double *luma, int w, int h, int n, float edges,
                             float textures, int y0, int y1, int nthreads, float *out)
{
    if (n != 2 && n != 4 && n != 8 && n != 16) return -1;
    if (y0 < 0 || y1 > h || y0 > y1 || w <= 0) return -1;
    int r = n / 2;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
    {
        ref_scratch s;
        scratch_init(&s, n);
#pragma omp for schedule(dynamic, 4)
        for (int y = y0; y < y1; y++)
            for (int x = 0; x < w; x++) {
                for (int i = -r + 1; i <= r; i++)
                    for (int j = -r + 1; j <= r; j++) {
                        int ii = clamp_off(x, i, 0, w - 1);
                        int jj = clamp_off(y, j, 0, h - 1);
                        s.data[i + r - 1][j + r - 1] = luma[(size_t)(y + jj) * w + (x + ii)];
                    }
                dispatch(&s);
                out[(size_t)(y - y0) * w + x] = weighted_max(&s, edges, textures);
            }
        scratch_free(&s);
    }
    return 0;
}

/* Preview semantics (src/render.c:31-79, 421-479): the row-streamed window of
 * dct_energy_preview over u8 luma rows, one scratch per row as the reference
 * allocates it (src/render.c:37-41), reference transforms. */
int ref_preview_map(const uint8_t *px, int w, int h, int bpp, int n, float edges,
                    float textures, float *out)
{
    if (n != 2 && n != 4 && n != 8 && n != 16) return -1;
    if (bpp != 1 && bpp != 3 && bpp != 4) return -1;
    int c = (n - 1) / 2;
    unsigned char *L = (unsigned char *)malloc((size_t)w * h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const uint8_t *q = px + ((size_t)y * w + x) * bpp;
            L[(size_t)y * w + x] = bpp == 1 ? q[0]
                : (unsigned char)(16.0 + (q[0]) * 0.2568 + (q[1]) * 0.5041 + (q[2]) * 0.0979);
        }
    const unsigned char **rows = (const unsigned char **)malloc(sizeof(*rows) * n);
    for (int i = 0; i < n; i++) {                 /* initial fill, src/render.c:459-463 */
        int r0 = i - (c - 1);
        r0 = r0 < 0 ? 0 : (r0 > h - 1 ? h - 1 : r0);
        rows[i] = L + (size_t)r0 * w;
    }
    for (int y = 0; y < h; y++) {
        ref_scratch s;
        scratch_init(&s, n);
        for (int j = 0; j < w; j++) {             /* dct_energy_preview_rows */
            int left = j - (c - 1), right = j + n - c;
            for (int ii = 0; ii < n; ii++)
                for (int jj = left; jj <= right; jj++) {
                    int cj = jj < 0 ? 0 : (jj > w - 1 ? w - 1 : jj);
                    s.data[ii][jj - left] = rows[ii][cj];
                }
            dispatch(&s);
            out[(size_t)y * w + j] = weighted_max(&s, edges, textures);
        }
        scratch_free(&s);
        /* shuffle rows, append MIN(y + n - (c - 1), h - 1) (src/render.c:467-475) */
        for (int i = 1; i < n; i++) rows[i - 1] = rows[i];
        int nr = y + n - (c - 1);
        rows[n - 1] = L + (size_t)(nr < h - 1 ? nr : h - 1) * w;
    }
    free(rows);
    free(L);
    return 0;
}
