/*
 * dcte_oracle.c -- CPU ORACLE for the dct-carver energy map.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libdctenergy_hip.so,
 * the dctenergy Python package) links, loads or calls this file.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker / the timed CPU baseline.
 *
 * It is a plain-C restatement of the reference's hot path, written from the
 * reference's definitions, mirroring the reference's floating-point operation
 * ORDER so that results are bit-identical to the reference's own compiled
 * transforms (pinned by tests/test_oracle.py against oracle/_ref and the
 * golden fixtures in tests/golden/):
 *
 *   luma          liblqr LQR_ER_LUMA read for 8-bit RGB / grey
 *                 (requested at src/render.c:315; formula [liblqr, unverified],
 *                  SURVEY.md §8a-a2)
 *   window gather src/render.c:122-132 (clamp_offset_to_border) and
 *                 src/render.c:134-152 (dct_pixel_energy): data[dx][dy]
 *   dispatch      src/dct.c:77-94 (dctNxN): N=2,4 -> ddct2d, 8 -> ddct8x8s,
 *                 16 -> ddct16x16s
 *   ddct8x8s      src/fft2d/shrtdct.c:55-117 (forward branch, isgn<0)
 *   ddct16x16s    src/fft2d/shrtdct.c:231-386 (forward branch)
 *   ddct2d        src/fft2d/fftsg2d.c:566-627 -> ddct src/fft2d/fftsg.c:349-402,
 *                 cftx020 :3211, dctsub :3274, makect :724 (N=2,4 only)
 *   weighted max  src/dct.c:96-110 (weighted_max_dct_correlation) with the
 *                 edge-atom test src/dct.c:56-73 (edges = (0,1),(1,0))
 *   preview       the GTK preview's second energy semantics,
 *                 dct_energy_preview / dct_energy_preview_rows /
 *                 convert_row_to_luminance (src/render.c:31-79, :421-479):
 *                 u8 luma RGB2LUMINANCE (src/render.h:5), window rows and
 *                 columns -(c-1)..N-c with c = CENTER_ROW(N) = (N-1)/2
 *                 (src/dct.h:8-9), stored data[dy][dx]
 *
 *   seam DP       liblqr's cumulative energy for the carver configured at
 *                 src/render.c:313 (lqr_carver_init(carver, 1, 0): delta_x 1,
 *                 rigidity 0) and its seam backtrack [liblqr, unverified]
 *
 * Compile with -ffp-contract=off (the Makefile does): the reference is plain
 * C on x86-64 where gcc emits no fused multiply-adds.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* Twiddles.  Definitions (Ooura): Cn_kR = sqrt(2/n) cos(pi/2 k/n),          */
/* Cn_kI = sqrt(2/n) sin(pi/2 k/n), Wn_kR = cos(pi/2 k/n), Wn_kI = sin(...). */
/* Written as the exact binary64 values of the reference's decimal literals  */
/* (src/fft2d/shrtdct.c:45-52, 211-227); libm would differ in the last bit   */
/* for several of them.                                                       */
/* ------------------------------------------------------------------------ */
static const double k8c1 = 0x1.f6297cff75cb0p-2, k8s1 = 0x1.8f8b83c69a60bp-4;
static const double k8c2 = 0x1.d906bcf328d46p-2, k8s2 = 0x1.87de2a6aea963p-3;
static const double k8c3 = 0x1.a9b66290ea1a3p-2, k8s3 = 0x1.1c73b39ae68c8p-2;
static const double k8c4 = 0x1.6a09e667f3bcdp-2, k8w4 = 0x1.6a09e667f3bcdp-1;

static const double k16c[9] = {0.0,
    0x1.684b9c80f1a8bp-2, 0x1.63150b15e8536p-2, 0x1.5a730c6c21c67p-2,
    0x1.4e7ae9144f0fcp-2, 0x1.3f4a237187eafp-2, 0x1.2d062ef88e319p-2,
    0x1.17dc13dab2dd6p-2, 0x1.0000000000000p-2};
static const double k16s[8] = {0.0,
    0x1.1be35182fe5aap-5, 0x1.1a855dec071b5p-4, 0x1.a4608aafa8527p-4,
    0x1.1517a7bdb3895p-3, 0x1.5553e3f5b5e58p-3, 0x1.92469c0dcf32dp-3,
    0x1.cb598cc4beea0p-3};
static const double k16w4c = 0x1.d906bcf328d46p-1, k16w4s = 0x1.87de2a6aea963p-2;
static const double k16w8 = 0x1.6a09e667f3bcdp-1;

/* One 8-point forward pass over v[0], v[st], ..., v[7 st]; the operation
 * sequence is that of one loop iteration of shrtdct.c:62-89. */
static void fwd8(double *v, ptrdiff_t st)
{
    double p0 = v[0] + v[7 * st], m0 = v[0] - v[7 * st];
    double p2 = v[2 * st] + v[5 * st], m2 = v[2 * st] - v[5 * st];
    double p4 = v[4 * st] + v[3 * st], m4 = v[4 * st] - v[3 * st];
    double p6 = v[6 * st] + v[st], m6 = v[6 * st] - v[st];
    double u = p0 + p4, w = p2 + p6;
    v[0] = k8c4 * (u + w);
    v[4 * st] = k8c4 * (u - w);
    u = p0 - p4;
    w = p2 - p6;
    v[2 * st] = k8c2 * u - k8s2 * w;
    v[6 * st] = k8c2 * w + k8s2 * u;
    u = k8w4 * (m2 - m6);
    m2 = k8w4 * (m2 + m6);
    m6 = m2 - m4;
    m2 += m4;
    m4 = m0 - u;
    m0 += u;
    v[st] = k8c1 * m0 - k8s1 * m2;
    v[7 * st] = k8c1 * m2 + k8s1 * m0;
    v[3 * st] = k8c3 * m4 - k8s3 * m6;
    v[5 * st] = k8c3 * m6 + k8s3 * m4;
}

/* One 16-point forward pass; operation sequence of shrtdct.c:239-313. */
static void fwd16(double *v, ptrdiff_t st)
{
#define V(i) v[(i) * st]
    double e0, e1, f0, f1, g0, g1, h0, h1, q0, q1, q2, q3, q4, q5, q6, q7;
    double a, b;
    q0 = V(0) - V(15); a = V(0) + V(15);
    q1 = V(8) - V(7);  b = V(8) + V(7);
    e0 = a + b; e1 = a - b;
    q2 = V(2) - V(13); a = V(2) + V(13);
    q3 = V(10) - V(5); b = V(10) + V(5);
    f0 = a + b; f1 = a - b;
    q4 = V(4) - V(11); a = V(4) + V(11);
    q5 = V(12) - V(3); b = V(12) + V(3);
    g0 = a + b; g1 = a - b;
    q6 = V(6) - V(9);  a = V(6) + V(9);
    q7 = V(14) - V(1); b = V(14) + V(1);
    h0 = a + b; h1 = a - b;
    a = e0 + g0; b = f0 + h0;
    V(0) = k16c[8] * (a + b);
    V(8) = k16c[8] * (a - b);
    a = e0 - g0; b = f0 - h0;
    V(4) = k16c[4] * a - k16s[4] * b;
    V(12) = k16c[4] * b + k16s[4] * a;
    e0 = k16w8 * (f1 - h1);
    g0 = k16w8 * (f1 + h1);
    a = e1 + e0; b = g0 + g1;
    V(2) = k16c[2] * a - k16s[2] * b;
    V(14) = k16c[2] * b + k16s[2] * a;
    a = e1 - e0; b = g0 - g1;
    V(6) = k16c[6] * a - k16s[6] * b;
    V(10) = k16c[6] * b + k16s[6] * a;
    a = k16w8 * (q4 - q5);
    b = k16w8 * (q5 + q4);
    q4 = q0 - a; q5 = q1 - b;
    q0 += a; q1 += b;
    a = k16w4s * q6 - k16w4c * q7;
    b = k16w4s * q7 + k16w4c * q6;
    q6 = k16w4c * q2 - k16w4s * q3;
    q7 = k16w4c * q3 + k16w4s * q2;
    q2 = q6 + a; q3 = q7 + b;
    q6 -= a; q7 -= b;
    a = q0 + q2; b = q3 + q1;
    V(1) = k16c[1] * a - k16s[1] * b;
    V(15) = k16c[1] * b + k16s[1] * a;
    a = q0 - q2; b = q3 - q1;
    V(7) = k16c[7] * a - k16s[7] * b;
    V(9) = k16c[7] * b + k16s[7] * a;
    a = q4 - q7; b = q6 + q5;
    V(5) = k16c[5] * a - k16s[5] * b;
    V(11) = k16c[5] * b + k16s[5] * a;
    a = q4 + q7; b = q6 - q5;
    V(3) = k16c[3] * a - k16s[3] * b;
    V(13) = k16c[3] * b + k16s[3] * a;
#undef V
}

/* makect (fftsg.c:724-740) for nc = n, evaluated exactly as the reference
 * does it (libm cos/sin of atan(1)/nch multiples). */
static void small_ct(int n, double *c)
{
    int nch = n >> 1, j;
    double delta = atan(1.0) / nch;
    c[0] = cos(delta * nch);
    c[nch] = 0.5 * c[0];
    for (j = 1; j < nch; j++) {
        c[j] = 0.5 * cos(delta * j);
        c[n - j] = 0.5 * sin(delta * j);
    }
}

/* ddct(n, -1, ...) of fftsg.c:349-402 for n = 2 or 4 (prologue butterfly,
 * cftx020 for n = 4, dctsub), on a strided vector. */
static void fwd_small(int n, double *v, ptrdiff_t st, const double *c)
{
    if (n == 2) {
        double t = v[st];
        v[st] = v[0] - t;
        v[0] += t;
        v[st] *= c[0];                       /* dctsub: a[m] *= c[0], m = 1 */
        return;
    }
    /* n == 4 */
    double a0 = v[0], a1 = v[st], a2 = v[2 * st], a3 = v[3 * st], t;
    t = a3;
    a3 = a2 - a1;
    a2 += a1;
    a1 = a0 - t;
    a0 += t;
    /* cftx020 */
    {
        double r = a0 - a2, i = a1 - a3;
        a0 += a2;
        a1 += a3;
        a2 = r;
        a3 = i;
    }
    /* dctsub(4, a, nc = 4, c): j = 1, k = 3, kk = 1 */
    {
        double wr = c[1] - c[3], wi = c[1] + c[3];
        double x = wi * a1 - wr * a3;
        a1 = wr * a1 + wi * a3;
        a3 = x;
        a2 *= c[0];
    }
    v[0] = a0; v[st] = a1; v[2 * st] = a2; v[3 * st] = a3;
}

/* In-place 2-D forward transform of an n x n window d[i*n + j]
 * (i = first index = x offset, j = y offset), mirroring dctNxN. */
int orc_dct(int n, double *d)
{
    int i;
    if (n == 8) {
        for (i = 0; i < 8; i++) fwd8(d + i, 8);        /* along first index */
        for (i = 0; i < 8; i++) fwd8(d + 8 * i, 1);    /* along second index */
        return 0;
    }
    if (n == 16) {
        for (i = 0; i < 16; i++) fwd16(d + i, 16);
        for (i = 0; i < 16; i++) fwd16(d + 16 * i, 1);
        return 0;
    }
    if (n == 2 || n == 4) {
        double c[4];
        small_ct(n, c);
        /* ddct2d: rows (second index) first, then columns (ddxt2d_sub) */
        for (i = 0; i < n; i++) fwd_small(n, d + n * i, 1, c);
        for (i = 0; i < n; i++) fwd_small(n, d + i, n, c);
        return 0;
    }
    return -1; /* reference: error() and no transform (src/dct.c:89-92) */
}

/* weighted_max_dct_correlation, src/dct.c:96-110: last maximum wins
 * (max <= currval), DC excluded, class from the edge LUT ((0,1),(1,0)). */
float orc_weighted_max(int n, const double *d, float edges, float textures)
{
    int k1, k2, b1 = 0, b2 = 0;
    double m = 0, v;
    for (k1 = 0; k1 < n; k1++)
        for (k2 = 0; k2 < n; k2++) {
            v = fabs(d[k1 * n + k2]);
            if (m <= v && (k1 || k2)) {
                m = v;
                b1 = k1;
                b2 = k2;
            }
        }
    int edge = (b1 == 0 && b2 == 1) || (b1 == 1 && b2 == 0);
    return edge ? (float)(m * (double)edges) : (float)(m * (double)textures);
}

/* Energy of one window given in reference layout (n*n doubles, [dx][dy]);
 * the window is copied, not modified. */
float orc_window_energy(int n, const double *win, float edges, float textures)
{
    double d[256];
    memcpy(d, win, sizeof(double) * n * n);
    orc_dct(n, d);
    return orc_weighted_max(n, d, edges, textures);
}

/* liblqr LQR_ER_LUMA read of one 8-bit pixel [liblqr, unverified]. */
double orc_luma(const uint8_t *p, int bpp)
{
    if (bpp == 1) return (double)p[0] / 255;
    double r = (double)p[0] / 255, g = (double)p[1] / 255, b = (double)p[2] / 255;
    return 0.2126 * r + 0.7152 * g + 0.0722 * b;
}

/* clamp_offset_to_border (src/render.c:122-132) */
static int clamp_off(int base, int off, int lo, int hi)
{
    if (base + off - lo < 0) return off - (base + off - lo);
    if (base + off - hi > 0) return off - (base + off - hi);
    return off;
}

static int valid_n(int n) { return n == 2 || n == 4 || n == 8 || n == 16; }

/* Energy map over a luma plane.  `luma` holds rows [row0, row0 + nrows) of
 * the w x h image (row-major, w doubles per row); output rows [y0, y1) go to
 * out[(y - y0) * w + x].  dct_pixel_energy semantics (src/render.c:134-157)
 * with radius r = n/2; every clamped row must lie inside the rows held. */
int orc_energy_map_luma_rows(const double *luma, int row0, int nrows, int w, int h,
                             int n, float edges, float textures, int y0, int y1,
                             int nthreads, float *out)
{
    if (!valid_n(n) || w <= 0 || h <= 0 || y0 < 0 || y1 > h || y0 > y1) return -1;
    int r = n / 2;
    int need_lo = y0 - r + 1 < 0 ? 0 : y0 - r + 1;
    int need_hi = y1 - 1 + r > h - 1 ? h - 1 : y1 - 1 + r;
    if (y1 > y0 && (need_lo < row0 || need_hi >= row0 + nrows)) return -1;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int y = y0; y < y1; y++) {
        double d[256];
        for (int x = 0; x < w; x++) {
            for (int i = -r + 1; i <= r; i++) {
                int ii = clamp_off(x, i, 0, w - 1);
                for (int j = -r + 1; j <= r; j++) {
                    int jj = clamp_off(y, j, 0, h - 1);
                    d[(i + r - 1) * n + (j + r - 1)] =
                        luma[(size_t)(y + jj - row0) * w + (x + ii)];
                }
            }
            orc_dct(n, d);
            out[(size_t)(y - y0) * w + x] = orc_weighted_max(n, d, edges, textures);
        }
    }
    return 0;
}

/* Same, from 8-bit interleaved pixels (bpp 1 or 3, rowstride in bytes);
 * `px` points at row 0 of the full image. */
int orc_energy_map_rows(const uint8_t *px, int w, int h, int bpp, size_t rowstride,
                        int n, float edges, float textures, int y0, int y1,
                        int nthreads, float *out)
{
    if (bpp != 1 && bpp != 3) return -1;
    if (!valid_n(n) || w <= 0 || h <= 0 || y0 < 0 || y1 > h || y0 > y1) return -1;
    if (y1 == y0) return 0;
    int r = n / 2;
    int lo = y0 - r + 1 < 0 ? 0 : y0 - r + 1;
    int hi = y1 - 1 + r > h - 1 ? h - 1 : y1 - 1 + r;
    double *luma = (double *)malloc(sizeof(double) * (size_t)w * (hi - lo + 1));
    if (!luma) return -2;
    for (int y = lo; y <= hi; y++)
        for (int x = 0; x < w; x++)
            luma[(size_t)(y - lo) * w + x] =
                orc_luma(px + (size_t)y * rowstride + (size_t)x * bpp, bpp);
    int rc = orc_energy_map_luma_rows(luma, lo, hi - lo + 1, w, h, n, edges, textures,
                                      y0, y1, nthreads, out);
    free(luma);
    return rc;
}

int orc_energy_map(const uint8_t *px, int w, int h, int bpp, size_t rowstride, int n,
                   float edges, float textures, int nthreads, float *out)
{
    return orc_energy_map_rows(px, w, h, bpp, rowstride, n, edges, textures, 0, h,
                               nthreads, out);
}

/* ---- preview semantics (src/render.c:31-79, 421-479) ------------------- */

/* convert_row_to_luminance (src/render.c:62-79): grey copies the byte; 3 or
 * more channels use RGB2LUMINANCE (src/render.h:5), evaluated in double left
 * to right and truncated to guchar; 2 channels are rejected (the reference
 * reports an error and leaves the row unconverted). */
uint8_t orc_preview_luma(const uint8_t *p, int bpp)
{
    if (bpp == 1) return p[0];
    return (uint8_t)(16.0 + p[0] * 0.2568 + p[1] * 0.5041 + p[2] * 0.0979);
}

/* Preview energies (before normalize_image) of a w x h region, rows
 * [y0, y1) into out[(y - y0) * w + x]; px addresses the region's row 0. */
int orc_preview_map_rows(const uint8_t *px, int w, int h, int bpp, size_t rowstride, int n,
                         float edges, float textures, int y0, int y1, int nthreads, float *out)
{
    if (bpp != 1 && bpp != 3 && bpp != 4) return -1;
    if (!valid_n(n) || w <= 0 || h <= 0 || y0 < 0 || y1 > h || y0 > y1) return -1;
    const int c = (n - 1) / 2; /* CENTER_ROW / CENTER_COL */
    uint8_t *L = (uint8_t *)malloc((size_t)w * h);
    if (!L) return -2;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++)
            L[(size_t)y * w + x] = orc_preview_luma(px + (size_t)y * rowstride + (size_t)x * bpp, bpp);
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int y = y0; y < y1; y++) {
        double d[256];
        for (int x = 0; x < w; x++) {
            for (int ii = 0; ii < n; ii++) {            /* data[dy][dx] */
                int yy = y + ii - (c - 1);
                yy = yy < 0 ? 0 : (yy > h - 1 ? h - 1 : yy);
                for (int jj = 0; jj < n; jj++) {
                    int xx = x + jj - (c - 1);
                    xx = xx < 0 ? 0 : (xx > w - 1 ? w - 1 : xx);
                    d[ii * n + jj] = L[(size_t)yy * w + xx];
                }
            }
            orc_dct(n, d);
            out[(size_t)(y - y0) * w + x] = orc_weighted_max(n, d, edges, textures);
        }
    }
    free(L);
    return 0;
}

int orc_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ---- seam DP [liblqr, unverified] -------------------------
 * The carver is set up with delta_x = 1 and rigidity 0 (src/render.c:313),
 * so the cumulative energy is the classic 3-neighbour recursion, in float
 * (gfloat) arithmetic:
 *     M[0][x] = E[0][x]
 *     M[y][x] = E[y][x] + min(M[y-1][x-1], M[y-1][x], M[y-1][x+1])
 * with candidates scanned left to right and replaced only on a strictly
 * smaller value (the leftmost minimum wins; out-of-frame candidates do not
 * exist).  The seam ends at the leftmost minimum of the last row and follows
 * the recorded parents up.  seam[y] = column removed in row y.
 * M may be NULL; returns 0, or -1 on bad sizes. */
int orc_seam_find(const float *E, long long stride, int w, int h, int *seam, float *M)
{
    if (w <= 0 || h <= 0 || stride < w) return -1;
    float *m = (float *)malloc(sizeof(float) * (size_t)w * 2);
    signed char *par = (signed char *)malloc((size_t)w * (size_t)h);
    if (!m || !par) {
        free(m);
        free(par);
        return -1;
    }
    float *prev = m, *cur = m + w;
    for (int x = 0; x < w; x++) prev[x] = E[x];
    if (M) for (int x = 0; x < w; x++) M[x] = prev[x];
    for (int y = 1; y < h; y++) {
        const float *e = E + (size_t)y * stride;
        for (int x = 0; x < w; x++) {
            int lo = x > 0 ? x - 1 : 0, hi = x < w - 1 ? x + 1 : w - 1;
            float best = prev[lo];
            int arg = lo;
            for (int c = lo + 1; c <= hi; c++)
                if (prev[c] < best) {
                    best = prev[c];
                    arg = c;
                }
            cur[x] = e[x] + best;
            par[(size_t)y * w + x] = (signed char)(arg - x);
        }
        if (M) for (int x = 0; x < w; x++) M[(size_t)y * w + x] = cur[x];
        float *t = prev;
        prev = cur;
        cur = t;
    }
    int x = 0;
    for (int c = 1; c < w; c++)
        if (prev[c] < prev[x]) x = c;
    seam[h - 1] = x;
    for (int y = h - 1; y > 0; y--) {
        x += par[(size_t)y * w + x];
        seam[y - 1] = x;
    }
    free(m);
    free(par);
    return 0;
}
