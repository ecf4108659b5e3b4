// dcte_pixel.h -- the energy of ONE pixel, fp32, by the map kernel's own passes.
//
// Host+device.  The sliding-window kernel (dcte_map) computes every row
// transform once per input row and reuses it across N output rows; a pixel's
// fast-path maxima nevertheless depend only on its N x N window and the fixed
// operation sequence of row_pass / Cols (dcte_passes.h), so evaluating the same
// passes on one window reproduces the map kernel's value bit for bit.  Used by
// the seam-update and point kernels (dcte_seam.hip) and by the host emulation
// (tests/emu).
//
// Window (a3/a4 of SURVEY §8): rows and columns  y - HL .. y - HL + N - 1,
// clamped to the frame, HL = N/2 - 1 (liblqr callback, src/render.c:146-150)
// or (N-1)/2 - 1 (preview, src/render.c:43-44).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "dcte_luma.h"
#include "dcte_passes.h"

namespace dcte {

DCTE_HD int clamp_px(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// the kernels' exact biased luma of one pixel (dcte_luma.h)
DCTE_HD float luma_biased(const uint8_t* p, int bpp, int sem)
{
    if (sem == kSemPreview)
        return (float)((int)preview_luma(p[0], bpp > 1 ? p[1] : 0u, bpp > 1 ? p[2] : 0u, bpp) -
                       kPreviewBias);
    const int L = bpp == 1 ? kLumaGrey * (int)p[0]
                           : kLumaR * (int)p[0] + kLumaG * (int)p[1] + kLumaB * (int)p[2];
    return (float)(L - kLumaBias);
}

constexpr DCTE_HD int halo_left(int n, int sem) { return sem == kSemLqr ? n / 2 - 1 : (n - 1) / 2 - 1; }

// (m_t, m_e) of pixel (x, y) of a w x h frame; `px` addresses global row
// `row0` (rows the window clamp reaches must be readable).
template <int N>
DCTE_HD void pixel_maxima(const uint8_t* px, long long rowstride, int row0, int w, int h,
                          int bpp, int sem, int x, int y, float& mt, float& me)
{
    const int HL = halo_left(N, sem);
    constexpr int CH = Lanes<N>::CH, S = Lanes<N>::S;
    float lrow[N];
    float ring[N][CH];
    mt = 0.0f;
    me = 0.0f;
    for (int lp = 0; lp < S; lp++) {
        for (int j = 0; j < N; j++) {   // input row y - HL + j -> ring slot j
            const int t = clamp_px(y - HL + j, 0, h - 1);
            const uint8_t* row = px + (long long)(t - row0) * rowstride;
            for (int i = 0; i < N; i++)
                lrow[i] = luma_biased(row + (long long)clamp_px(x - HL + i, 0, w - 1) * bpp, bpp, sem);
            row_pass<N>(lrow, 0, lp, ring[j]);
        }
        float t_, e_;
        Cols<N>::template run<0>(ring, lp, t_, e_);
        mt = fmaxf(mt, t_);
        me = fmaxf(me, e_);
    }
}

}  // namespace dcte
