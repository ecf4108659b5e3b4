// dcte_emu.cpp -- host emulation of the gfx950 kernel's fp32 arithmetic.
//
// TEST INFRASTRUCTURE.  Runs dcte_passes.h / dcte_math.h (the kernel's own
// code) on the CPU, pixel by pixel, so CPU-only tests can measure the fp32
// path's error against the oracle on large and adversarial inputs, and GPU
// tests can demand bit-equality between device and emulation.
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "dcte_luma.h"
#include "dcte_passes.h"

using namespace dcte;

namespace {

inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

inline float luma_biased(const uint8_t* p, int bpp, int sem)
{
    if (sem == kSemPreview)
        return (float)((int)preview_luma(p[0], bpp > 1 ? p[1] : 0u, bpp > 1 ? p[2] : 0u, bpp) - kPreviewBias);
    int L = bpp == 1 ? kLumaGrey * (int)p[0]
                     : kLumaR * (int)p[0] + kLumaG * (int)p[1] + kLumaB * (int)p[2];
    return (float)(L - kLumaBias);
}

template <int N>
void pixel(const uint8_t* px, int w, int h, int bpp, size_t rs, int x, int y, int sem,
           float& mt, float& me)
{
    const int HL = sem == kSemLqr ? N / 2 - 1 : (N - 1) / 2 - 1;
    constexpr int CH = Lanes<N>::CH, S = Lanes<N>::S;
    float lrow[N];
    float ring[N][CH];
    float mts[4] = {0, 0, 0, 0}, mes[4] = {0, 0, 0, 0};
    for (int lp = 0; lp < S; lp++) {
        for (int j = 0; j < N; j++) {   // input row y - HL + j -> slot j
            int t = clampi(y - HL + j, 0, h - 1);
            for (int i = 0; i < N; i++) {
                int xx = clampi(x - HL + i, 0, w - 1);
                lrow[i] = luma_biased(px + (size_t)t * rs + (size_t)xx * bpp, bpp, sem);
            }
            row_pass<N>(lrow, 0, lp, ring[j]);
        }
        Cols<N>::template run<0>(ring, lp, mts[lp], mes[lp]);
    }
    mt = fmaxf(fmaxf(mts[0], mts[1]), fmaxf(mts[2], mts[3]));
    me = fmaxf(fmaxf(mes[0], mes[1]), fmaxf(mes[2], mes[3]));
}

}  // namespace

extern "C" {

// Per-pixel emulation over rows [y0, y1).  we / wt are the kernel's scaled
// weights; outputs E (the kernel's fast-path value), and the raw m_e / m_t.
int emu_energy_map(const uint8_t* px, int w, int h, int bpp, size_t rowstride, int n,
                   float we, float wt, int sem, int y0, int y1, float* E, float* me_out,
                   float* mt_out)
{
    for (int y = y0; y < y1; y++)
        for (int x = 0; x < w; x++) {
            float mt, me;
            switch (n) {
            case 2: pixel<2>(px, w, h, bpp, rowstride, x, y, sem, mt, me); break;
            case 4: pixel<4>(px, w, h, bpp, rowstride, x, y, sem, mt, me); break;
            case 8: pixel<8>(px, w, h, bpp, rowstride, x, y, sem, mt, me); break;
            case 16: pixel<16>(px, w, h, bpp, rowstride, x, y, sem, mt, me); break;
            default: return -1;
            }
            size_t k = (size_t)(y - y0) * w + x;
            E[k] = me > mt ? me * we : mt * wt;
            if (me_out) me_out[k] = me;
            if (mt_out) mt_out[k] = mt;
        }
    return 0;
}
}
