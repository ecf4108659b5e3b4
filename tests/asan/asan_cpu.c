/*
 * asan_cpu.c -- CPU sanitizer driver: every host-side piece of
 * index-heavy C this repo ships or tests with, run under AddressSanitizer and
 * UBSan (tests/asan/Makefile, tests/test_asan.py).  TEST INFRASTRUCTURE ONLY.
 *
 *   1. the oracle's restatement (oracle/dcte_oracle.c): liblqr and preview
 *      maps over ragged frames (1 x 1 up, grey / RGB / RGBA, every N), window
 *      energies, the seam search -- and, where the reference's own fft2d
 *      transforms were built instrumented (DCTE_ASAN_REF), compared bit for
 *      bit with them through the restated glue (oracle/ref_harness.c: the
 *      window gather of src/render.c:122-157 and the shared scratch of
 *      src/render.c:140 / :296-305);
 *   2. the library's context-free host entries (dcte_host.cpp):
 *      dcte_energy_window on random and tie windows, dcte_normalize_u8_host
 *      on constant, one-element and random maps, every mode and channel count;
 *   3. the plug-in glue (dct-carver_amd/plugin/dcte_plugin.c) through the fake
 *      liblqr (tests/fake_lqr/fake_lqr.c): the hook's per-row checked
 *      intervals and window check (fake_window_check_selftest), an energy
 *      build and a resize loop (without a device: the no-device path).
 * Exit status 0 when every comparison holds; a sanitizer report aborts.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dctenergy.h"

#ifndef DCTE_ASAN_REF
#define DCTE_ASAN_REF 0
#endif

/* oracle/dcte_oracle.c */
float orc_window_energy(int n, const double *win, float edges, float textures);
double orc_luma(const uint8_t *p, int bpp);
int orc_energy_map(const uint8_t *px, int w, int h, int bpp, size_t rowstride, int n,
                   float edges, float textures, int nthreads, float *out);
int orc_preview_map_rows(const uint8_t *px, int w, int h, int bpp, size_t rowstride, int n,
                         float edges, float textures, int y0, int y1, int nthreads, float *out);
int orc_seam_find(const float *E, long long stride, int w, int h, int *seam, float *M);
#if DCTE_ASAN_REF
/* oracle/ref_harness.c over the reference's own transforms */
float ref_window_energy(int n, const double *win, float edges, float textures);
int ref_energy_map_luma(const double *luma, int w, int h, int n, float edges, float textures,
                        float *out);
int ref_preview_map(const uint8_t *px, int w, int h, int bpp, int n, float edges, float textures,
                    float *out);
#endif
/* tests/fake_lqr/fake_lqr.c */
int fake_build_emap(const uint8_t *px, int w, int h, int bpp, int n, float edges, float textures,
                    int use_gpu, int removed, int transposed, float *out,
                    long long *fallback_calls, int *gpu_status);
int fake_window_check_selftest(int n, int bpp, unsigned seed);
int fake_resize(const uint8_t *px, int w, int h, int bpp, int n, float edges, float textures,
                int use_gpu, int hook, int seams, int transposed, int diverge, int verify,
                float *out_emap, uint8_t *out_px, int *out_seams, long long *counts, int *gpu_status);

static unsigned g_rng = 12345u;
static unsigned rnd(void)
{
    g_rng = g_rng * 1664525u + 1013904223u;
    return g_rng >> 8;
}

static int g_fail;
#define CHECK(cond, ...)                                  \
    do {                                                  \
        if (!(cond)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                 \
            fprintf(stderr, "\n");                        \
            g_fail++;                                     \
        }                                                 \
    } while (0)

static const int kN[4] = {2, 4, 8, 16};

/* a frame of exactly w * h * bpp bytes (no slack: ASan sees any over-read) */
static uint8_t *frame(int w, int h, int bpp, int kind)
{
    uint8_t *px = (uint8_t *)malloc((size_t)w * h * bpp);
    for (size_t i = 0; i < (size_t)w * h * bpp; i++) {
        const size_t p = i / bpp, x = p % w, y = p / w;
        px[i] = kind == 0 ? (uint8_t)rnd()                              /* noise */
              : kind == 1 ? (uint8_t)((x % 31 == 0 || y % 23 == 0) ? 0 : 255) /* line art */
                          : (uint8_t)(16 + 3 * x + 5 * y);             /* ramp */
    }
    return px;
}

static void oracle_maps(void)
{
    static const int shapes[][2] = {{1, 1}, {1, 9}, {9, 1}, {2, 3}, {5, 7}, {16, 16}, {17, 33}, {40, 29}};
    for (size_t s = 0; s < sizeof(shapes) / sizeof(shapes[0]); s++)
        for (int bpp = 1; bpp <= 4; bpp++)
            for (int k = 0; k < 4; k++) {
                const int w = shapes[s][0], h = shapes[s][1], n = kN[k];
                uint8_t *px = frame(w, h, bpp, (int)(s % 3));
                float *a = (float *)malloc(sizeof(float) * w * h);
                float *b = (float *)malloc(sizeof(float) * w * h);
                if (bpp == 1 || bpp == 3) {
                    CHECK(orc_energy_map(px, w, h, bpp, (size_t)w * bpp, n, 0.3f, 0.7f, 1, a) == 0, "map");
#if DCTE_ASAN_REF
                    double *L = (double *)malloc(sizeof(double) * w * h);
                    for (int i = 0; i < w * h; i++) L[i] = orc_luma(px + (size_t)i * bpp, bpp);
                    CHECK(ref_energy_map_luma(L, w, h, n, 0.3f, 0.7f, b) == 0, "ref map");
                    CHECK(!memcmp(a, b, sizeof(float) * w * h), "liblqr map %dx%d bpp %d N %d", w, h, bpp, n);
                    free(L);
#endif
                }
                if (bpp != 2) {
                    CHECK(orc_preview_map_rows(px, w, h, bpp, (size_t)w * bpp, n, 0.3f, 0.7f, 0, h, 1, a) == 0,
                          "preview");
#if DCTE_ASAN_REF
                    CHECK(ref_preview_map(px, w, h, bpp, n, 0.3f, 0.7f, b) == 0, "ref preview");
                    CHECK(!memcmp(a, b, sizeof(float) * w * h), "preview map %dx%d bpp %d N %d", w, h, bpp, n);
#endif
                } else {
                    CHECK(orc_preview_map_rows(px, w, h, bpp, (size_t)w * bpp, n, 0.3f, 0.7f, 0, h, 1, a) != 0,
                          "bpp 2 accepted");
                }
                free(px);
                free(a);
                free(b);
            }
    /* the seam search on ragged maps, ties included */
    for (int w = 1; w <= 9; w += 4)
        for (int h = 1; h <= 7; h += 3) {
            float *E = (float *)malloc(sizeof(float) * w * h);
            int *seam = (int *)malloc(sizeof(int) * h);
            for (int i = 0; i < w * h; i++) E[i] = (float)(rnd() % 3);
            CHECK(orc_seam_find(E, w, w, h, seam, NULL) == 0, "seam");
            for (int y = 0; y < h; y++) CHECK(seam[y] >= 0 && seam[y] < w, "seam column");
            free(E);
            free(seam);
        }
}

static void host_entries(void)
{
    for (int k = 0; k < 4; k++) {
        const int n = kN[k];
        for (int rep = 0; rep < 200; rep++) {
            double *win = (double *)malloc(sizeof(double) * n * n);   /* exactly n * n */
            for (int i = 0; i < n * n; i++)
                win[i] = rep % 4 == 0 ? (double)(rnd() % 2) : (double)(rnd() % 256) / 255;
            float got = -1.0f;
            CHECK(dcte_energy_window(n, win, 0.3f, 0.7f, &got) == DCTE_OK, "window");
            CHECK(got == orc_window_energy(n, win, 0.3f, 0.7f), "window energy N %d rep %d", n, rep);
#if DCTE_ASAN_REF
            CHECK(got == ref_window_energy(n, win, 0.3f, 0.7f), "window energy vs ref N %d rep %d", n, rep);
#endif
            free(win);
        }
    }
    float dummy;
    CHECK(dcte_energy_window(3, NULL, 0.5f, 0.5f, &dummy) == DCTE_EINVAL, "bad n");
    for (int mode = 0; mode <= 1; mode++)
        for (int ch = 1; ch <= 4; ch++)
            for (int len = 1; len <= 129; len += 64) {
                float *E = (float *)malloc(sizeof(float) * len);
                uint8_t *o = (uint8_t *)malloc((size_t)len * ch);
                for (int i = 0; i < len; i++) E[i] = len == 65 ? 0.25f : (float)(rnd() % 1000) * 1e-3f;
                CHECK(dcte_normalize_u8_host(E, (size_t)len, mode, ch, o) == DCTE_OK, "normalize");
                for (int i = 0; i < len; i++)
                    for (int c = 1; c < ch; c++) CHECK(o[i * ch + c] == o[i * ch], "channels");
                if (len == 65) CHECK(o[0] == 0, "constant map -> 0");
                free(E);
                free(o);
            }
    uint8_t o1;
    float e1 = 1.0f;
    CHECK(dcte_normalize_u8_host(&e1, 1, 2, 1, &o1) == DCTE_EINVAL, "bad mode");
    CHECK(dcte_normalize_u8_host(&e1, 0, 0, 1, &o1) == DCTE_EINVAL, "empty");
}

static void plugin_glue(void)
{
    for (int k = 0; k < 4; k++)
        for (int bpp = 1; bpp <= 3; bpp += 2)
            for (unsigned seed = 1; seed <= 3; seed++)
                CHECK(fake_window_check_selftest(kN[k], bpp, seed) == 0, "window check N %d bpp %d", kN[k], bpp);
    /* energy builds and resize loops through the patched callback: without a
     * device the glue reports it and the original per-window body answers */
    const int w = 37, h = 21;
    for (int k = 0; k < 4; k++)
        for (int bpp = 1; bpp <= 3; bpp += 2) {
            const int n = kN[k];
            uint8_t *px = frame(w, h, bpp, k % 3);
            float *out = (float *)malloc(sizeof(float) * w * h);
            float *ref = (float *)malloc(sizeof(float) * w * h);
            long long calls = 0;
            int status = 0;
            CHECK(fake_build_emap(px, w, h, bpp, n, 0.3f, 0.7f, 1, 0, 0, out, &calls, &status) == 0, "build");
            orc_energy_map(px, w, h, bpp, (size_t)w * bpp, n, 0.3f, 0.7f, 1, ref);
            if (status != DCTE_OK) CHECK(!memcmp(out, ref, sizeof(float) * w * h), "fallback build N %d", n);
            const int seams = 5;
            float *em = (float *)malloc(sizeof(float) * w * h);
            uint8_t *op = (uint8_t *)malloc((size_t)w * h * bpp);
            int *os = (int *)malloc(sizeof(int) * seams * (w > h ? w : h));
            long long counts[16];
            for (int tr = 0; tr <= 1; tr++) {
                CHECK(fake_resize(px, w, h, bpp, n, 0.3f, 0.7f, 1, 1, seams, tr, 0, 1, em, op, os, counts,
                                  &status) == 0, "resize");
                CHECK(counts[7] == 0, "hook served a value off tolerance");
            }
            free(px);
            free(out);
            free(ref);
            free(em);
            free(op);
            free(os);
        }
}

int main(void)
{
    oracle_maps();
    host_entries();
    plugin_glue();
    printf("asan_cpu: %s (reference transforms %s)\n", g_fail ? "FAILED" : "ok",
           DCTE_ASAN_REF ? "compared" : "not built here");
    return g_fail ? 1 : 0;
}
